"""Benchmark: HTM stream-steps/s of the batched MI355X engine (BASELINE.json).

Workload (BASELINE.json configs[1]): 1,024 Model-1
streams per GPU (2048-column SP, 12-cell BacktrackingTM), SP and TM learning
off, every stream starting from the Model-1 state trained on the GPU over
the reference's 2,184 training records (ML/Data/TrainingData.txt, replayed
from tests/golden/model1_traces.npz).  Inputs are synthetic, resident in HBM:
    cpu[s,t] = clip(trace[(t + 97 s) mod 2324] + d[s,t], 0, 100)
trace = TestingData.txt cpu column, d uniform integer in {-2..2} from
numpy PCG64(seed=724).  A step = one network.run(1) of every stream
(encoder -> SP -> TM -> raw anomaly).  N>1 GPUs: weak scaling, streams
sharded by rank, per-step RCCL gather of the anomaly scores to rank 0
(the SLO alerting path).

Run:  python bench.py [--gpus N] [--steps K] [--warmup W] [--streams S]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "HTM stream-steps/sec (2048-col SP+TM, learn on/off) at 1/2/4/8 GPUs; % HBM peak"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def make_inputs(n_total, s0, s1, t0, t1, trace):
    rng = np.random.Generator(np.random.PCG64(724))
    d = rng.integers(-2, 3, size=(t1, n_total))[t0:t1, s0:s1]
    t = np.arange(t0, t1)[:, None]
    s = np.arange(s0, s1)[None, :]
    return np.clip(trace[(t + 97 * s) % len(trace)] + d, 0, 100).astype(np.float64)


def trained_engine(rt, n_streams, seg_capacity, device, train_vals):
    """Train Model 1 on one stream (2184 records, learning on), then load that
    state into every stream of an n_streams engine."""
    import torch
    tr = rt.HTMEngine(1, device=device, seg_capacity=seg_capacity)
    v = torch.tensor(train_vals, dtype=torch.float64, device=f"cuda:{device}").reshape(-1, 1)
    t0 = time.time()
    tr.run(v)
    tr.status()
    train_s = time.time() - t0
    eng = rt.HTMEngine(n_streams, device=device, seg_capacity=seg_capacity)
    for region in rt._lib.ST:
        eng.import_state(region, tr.export_state(region, 0, 1), s0=0)
    eng.replicate(0)
    hdr = tr.tm_header(0)
    tr.close()
    return eng, train_s, hdr


def cpu_baseline(trace, train_vals, n_total, target_s=12.0):
    """The C oracle (OpenMP across streams) on a bounded sample of the same
    workload: trained Model-1 state cloned into C streams, inference only."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    oracle.build()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, len(os.sched_getaffinity(0)))
    m = oracle.OracleModel()
    for v in train_vals:
        m.step(v, True, True)
    n = 2 * threads
    models = [m.clone() for _ in range(n)]
    vals = make_inputs(n_total, 0, n, 0, 4096, trace)
    t0 = time.time()
    oracle.step_batch(models, vals[0], False, False, threads)
    one = time.time() - t0
    steps = max(4, int(target_s / max(one, 1e-3)))
    steps = min(steps, 4095)
    t0 = time.time()
    for k in range(1, steps + 1):
        oracle.step_batch(models, vals[k], False, False, threads)
    dt = time.time() - t0
    return dict(value=n * steps / dt, unit="stream-steps/s", cores=threads, kind="port",
                sample=f"{n} streams x {steps} steps of the config-2 workload (oracle/htm_oracle.c, "
                       f"OpenMP over streams, {threads} threads), {dt:.1f} s")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2324)
    ap.add_argument("--warmup", type=int, default=64)
    ap.add_argument("--streams", type=int, default=1024, help="streams per GPU")
    ap.add_argument("--seg-capacity", type=int, default=72 * 1024)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU oracle baseline")
    ap.add_argument("--no-profile", action="store_true", help="no per-kernel HIP events")
    ap.add_argument("--mode", choices=["step", "run"], default="step",
                    help="step: one htm_step (network.run(1) of every stream) per step, lockstep; "
                         "run: the K steps as htm_run replay chunks (each stream runs ahead independently)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl")
    import _pkg
    rt = _pkg.load()

    d = np.load(os.path.join(ROOT, "tests", "golden", "model1_traces.npz"))
    train_vals = [c for c, m in zip(d["train_cpu"], d["train_mem"]) if not (np.isnan(c) or np.isnan(m))][:2184]
    trace = d["test_cpu"].astype(np.float64)

    S = args.streams
    n_total = S * world
    s0, s1 = rt.fleet.shard_range(n_total, world, rank)
    eng, train_s, hdr = trained_engine(rt, S, args.seg_capacity, local, train_vals)
    eng.set_learning(False, False)
    T = args.warmup + args.steps
    vals = torch.tensor(make_inputs(n_total, s0, s1, 0, T, trace), device=f"cuda:{local}")
    scores = torch.empty((T, S), dtype=torch.float32, device=f"cuda:{local}")
    gather = rt.fleet.ScoreGather(n_total) if world > 1 else None
    gathered = None
    if world > 1 and rank == 0:
        gathered = torch.empty((args.steps, world, gather.width), dtype=torch.float32, device=f"cuda:{local}")

    for k in range(args.warmup):
        eng.step(vals[k], out=scores[k])
    torch.cuda.synchronize()
    c0 = eng.counters()
    if not args.no_profile:
        eng.profile(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    handles = []
    if args.mode == "run":
        eng.run(vals[args.warmup:], out=scores[args.warmup:])
        if world > 1:
            for k in range(args.steps):
                h, _ = gather.gather(scores[args.warmup + k], staging=gathered[k] if rank == 0 else None)
                handles.append(h)
    else:
        for k in range(args.steps):
            eng.step(vals[args.warmup + k], out=scores[args.warmup + k])
            if world > 1:
                h, _ = gather.gather(scores[args.warmup + k], staging=gathered[k] if rank == 0 else None)
                handles.append(h)
    for h in handles:
        h.wait()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    prof = eng.profile_read() if not args.no_profile else None
    eng.profile(False)
    c1 = eng.counters()
    if c1["error"]:
        raise RuntimeError(f"engine overflow flags {c1['error']}")
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    value = n_total * args.steps / dt
    roof = None
    if prof is not None and prof["tm_ms"] > 0:
        tm_bytes = c1["tm_bytes"] - c0["tm_bytes"]
        launches = prof["launches"]
        avg_ms = prof["tm_ms"] / launches
        achieved = tm_bytes / launches / (avg_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                "kernel": ("htm_run_kernel<false,true> (fused SP+TM)" if prof["sp_ms"] == 0
                           else "tm_step_kernel<false,true>"),
                "avg_launch_ms": round(avg_ms, 4), "steps_per_launch": prof["steps"] / launches,
                "bytes_per_launch": int(tm_bytes / launches),
                "sp_kernel_avg_ms": round(prof["sp_ms"] / launches, 4)}
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "stream-steps/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int32+f32",
        "data": "synthetic: TestingData cpu trace + PCG64(724) jitter, resident in HBM (SURVEY.md §8(d) config 2)",
        "config": {"workload": "config2: Model-1 streams (2048-col SP, 12-cell BacktrackingTM), SP+TM learn off, "
                               "from the GPU-trained Model-1 state",
                   "mode": args.mode,
                   "streams_per_gpu": S, "total_streams": n_total, "columns": 2048, "cells_per_column": 12,
                   "trained_segments": int(hdr.seg_live), "train_s": round(train_s, 2),
                   "parallelism": f"streams sharded over {world} GPU(s)" + (", RCCL gather of scores" if world > 1 else "")},
        "roofline": roof,
        "tm_counters": {k: c1[k] - c0[k] for k in ["inf_phase2", "inf_backtracks"]},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(trace, train_vals, n_total)
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
