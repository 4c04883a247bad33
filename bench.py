"""Benchmark: HTM stream-steps/s of the batched MI355X engine (BASELINE.json).

Workload (BASELINE.json configs[1]): 1,024 Model-1
streams per GPU (2048-column SP, 12-cell BacktrackingTM), SP and TM learning
off, every stream starting from the Model-1 state trained on the GPU over
the reference's 2,184 training records (ML/Data/TrainingData.txt, replayed
from tests/golden/model1_traces.npz).  Inputs are synthetic, resident in HBM:
    cpu[s,t] = clip(trace[(t + 97 s) mod 2324] + d[s,t], 0, 100)
trace = TestingData.txt cpu column, d uniform integer in {-2..2} from
numpy PCG64(seed=724).  A step = one network.run(1) of every stream
(encoder -> SP -> TM -> raw anomaly).  Before the W warm-up steps every
stream replays `--condition` records (default 64, config 2's warm-up in
SURVEY.md §8(d), untimed): the replicated state was trained
on another part of the trace, and a stream's first steps after meeting its
own trace position are a bursting transient, not the steady state a
continuously running stream is in (the conditioning and the warm-up run in
the measured mode: lockstep steps also bring the deferred-duty log, empty
after replay chunks, to its steady state).  `value` times the K steps in LOCKSTEP
(the headline, north_star's real-time stepping: one htm_step per step, every
stream advances one record and waits for the slowest); the same engine is
then timed in run mode (`run_mode`: the K steps as htm_run replay chunks,
each stream stepping through a chunk without waiting for the others -- the
reference's offline replay of recorded metrics, ModelTesting.py over
TestingData.txt, batched).  N>1 GPUs: weak scaling, streams sharded by
rank, RCCL gather of every step's anomaly scores to rank 0 (the SLO
alerting path).  roofline.traffic: at N=1, before the timed run, bench.py
runs the same workload under rocprofv3 once per counter pass (child
processes) and reads the HBM bytes per launch of the dominant kernel from
them (tools/pmc_summary.py; --no-pmc skips, --pmc-summary reuses passes).

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
L2_PEAK_GBS = 34500.0  # MI355X_MICROARCH.md, L2 (per XCD): ~34.5 TB/s aggregate


def make_inputs(n_total, s0, s1, t0, t1, trace):
    rng = np.random.Generator(np.random.PCG64(724))
    d = rng.integers(-2, 3, size=(t1, n_total))[t0:t1, s0:s1]
    t = np.arange(t0, t1)[:, None]
    s = np.arange(s0, s1)[None, :]
    return np.clip(trace[(t + 97 * s) % len(trace)] + d, 0, 100).astype(np.float64)


def trained_engine(rt, n_streams, seg_capacity, device, train_vals, world=1, **cfg):
    """Train Model 1 (or the config-5 cpu+mem model: cfg overrides) on one
    stream (2184 records, learning on), then load that state into every stream
    of an n_streams engine.  With N>1 ranks only rank 0 trains: the trained
    stream is broadcast to the other ranks in one collective (RCCL over xGMI,
    fleet.broadcast_state) instead of every rank re-training it."""
    import torch
    tr = rt.HTMEngine(1, device=device, seg_capacity=seg_capacity, **cfg)
    tv = np.asarray(train_vals, np.float64)
    v = torch.tensor(tv.reshape(tv.shape[0], -1), device=f"cuda:{device}")
    t0 = time.time()
    dist_info = "trained locally"
    if world > 1:
        import torch.distributed as dist
        if dist.get_rank() == 0:
            tr.run(v)
            tr.status()
        nb = rt.fleet.broadcast_state(tr, list(rt._lib.ST), src=0, device=f"cuda:{device}")
        dist_info = f"trained on rank 0, broadcast to {world - 1} rank(s): {nb} B in one collective"
    else:
        tr.run(v)
        tr.status()
    torch.cuda.synchronize()
    train_s = time.time() - t0
    eng = rt.HTMEngine(n_streams, device=device, seg_capacity=seg_capacity, **cfg)
    for region in rt._lib.ST:
        eng.import_state(region, tr.export_state(region, 0, 1), s0=0)
    eng.replicate(0)
    hdr = tr.tm_header(0)
    tr.close()
    return eng, train_s, hdr, dist_info


def cpu_baseline(trace, train_vals, n_total, target_s=12.0):
    """The C oracle (OpenMP across streams, every core this process may run
    on) on a bounded sample of the same workload: trained Model-1 state cloned
    into 2 x cores streams, inference only.  Beside it, the single-stream
    Python loop over the oracle -- one network.run(1) per call, the shape of
    ModelTesting.py:66-72's per-record loop -- and the reference's published
    per-prediction latency."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    oracle.build()
    # every CPU this process may use: the affinity set, capped by the box's CPU
    # allotment when it sets one (gpurun boxes export OMP_NUM_THREADS=16 per GPU
    # while the affinity mask lists the whole host)
    affinity = len(os.sched_getaffinity(0))
    threads = min(affinity, int(os.environ.get("OMP_NUM_THREADS", "0") or affinity))
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
    # single stream, Python loop (one call per step, like ModelTesting's loop)
    single = m.clone()
    t0 = time.time()
    k = 0
    while time.time() - t0 < 4.0 and k < 4095:
        single.step(float(vals[k + 1, 0]), False, False)
        k += 1
    ds = time.time() - t0
    return dict(value=n * steps / dt, unit="stream-steps/s", cores=threads, kind="port",
                sample=f"{n} streams x {steps} steps of the config-2 workload (oracle/htm_oracle.c, "
                       f"OpenMP over streams, {threads} threads: sched_getaffinity {affinity} capped by "
                       f"OMP_NUM_THREADS), {dt:.1f} s",
                single_stream_python_loop={"value": round(k / ds, 2), "unit": "stream-steps/s", "cores": 1,
                                           "ms_per_step": round(ds / k * 1e3, 3), "steps": k,
                                           "sample": "one stream, one oracle step per Python call "
                                                     "(ModelTesting.py:66-72 loop shape)"},
                reference_published={"ms_per_prediction": "20-50", "hardware": "AWS t2.large (2 vCPU), NuPIC 1.0.x",
                                     "source": "CSC 724 Final Project Report p.8 (SURVEY.md §6)"})


def learn_on_bytes(eng, S, seg_live):
    """Unique algorithmic bytes per stream-step of a learning step (SURVEY.md
    §8(d)'s learning terms, each byte counted once per step however often the
    kernel re-reads it -- a lower bound, write traffic of new segments and
    weak-column bumps excluded): SP -- the active input rows of the
    input-major connected map, the winners' potential permanences read and
    written and their potential-mask rows, both duty-cycle arrays read and
    written; TM -- every live segment's meta, synapse sources, connected mask
    and dutyCycle record read once, the winners' segment permanences read and
    written (one segment per active column), the seven cell bitmaps read and
    written, the pattern history."""
    c = eng.config
    nw, pw = c.sp_columns // 32, (c.n_fields * c.enc_n + 31) // 32
    n_pot = int(round(c.n_fields * c.enc_n * c.sp_potential_pct))
    sp = c.n_fields * c.enc_w * nw * 4 + c.sp_num_active * (n_pot * 4 * 2 + pw * 4) + 2 * c.sp_columns * 4 * 2
    cw = c.sp_columns * c.tm_cells_per_col // 32
    tm = seg_live / S * (4 + 64 + 4 + 12) + c.sp_num_active * 128 * 2 + 7 * cw * 4 * 2 + 2 * 16 * 64 * 2
    return sp + tm


def bench_learn_on(args, rt, trace, world, rank, local, pmc_summary=None, pmc_note=None):
    """The "learn on" half of BASELINE.json's metric (configs[2], SURVEY.md
    §8(d) config 3): 65,536 fresh Model-1 streams per GPU (seeds 2045 + the
    global stream index), SP+TM learning on, paged SP permanences (800 rows per
    stream), `learn_steps` lockstep htm_step calls timed after `learn_warmup`
    untimed ones, the barrier / max-over-ranks contract of the headline.  Its
    roofline counts unique bytes (learn_on_bytes)."""
    import torch
    S = args.learn_streams
    n_total = S * world
    import _pkg
    s0, s1 = _pkg.load().fleet.shard_range(n_total, world, rank)
    dev = f"cuda:{local}"
    cfg = rt.default_config(seg_capacity=10240, upd_capacity=512, seed_stride=1, sp_seed=2045 + s0, tm_seed=2045 + s0,
                            sp_perm_rows=800)
    t0 = time.time()
    eng = rt.HTMEngine(S, config=cfg, device=local)
    torch.cuda.synchronize()
    init_s = time.time() - t0
    eng.set_learning(True, True)
    eng.split_learning(args.split_learn == "on")
    W, K = args.learn_warmup, args.learn_steps
    vals = torch.tensor(make_inputs(n_total, s0, s1, 0, W + K, trace), device=dev)
    scores = torch.empty((W + K, S), dtype=torch.float32, device=dev)
    for k in range(W):
        eng.step(vals[k], out=scores[k])
    torch.cuda.synchronize()
    c0 = eng.counters()
    eng.profile(True)
    marks = []
    dt, _ = timed_replay(eng, vals, scores, W, K, "step", 1, None, None, rank, world, dev, marks=marks)
    # the step time per 64-step window of the region (segment pools grow, fewer
    # SP columns are new): HIP events on the step stream between the windows
    per64 = [{"steps": f"{W + k0}-{W + k1 - 1}", "ms_per_step": round(e0.elapsed_time(e1) / (k1 - k0), 4)}
             for (k0, e0), (k1, e1) in zip(marks, marks[1:])]
    prof = eng.profile_read()
    eng.profile(False)
    c1 = eng.counters()
    if c1["error"]:
        raise RuntimeError(f"learn-on engine overflow flags {c1['error']}")
    seg_live = (c0["seg_live"] + c1["seg_live"]) / 2
    per_ss = learn_on_bytes(eng, S, seg_live)
    launches = prof["launches"]
    split = args.split_learn == "on"
    tm_name = kernel_name(True, False, True, split)
    # a split step's kernels: the SP kernel (its learning) and the TM-only kernel, timed each
    avg_ms = (prof["tm_ms"] + prof["sp_ms"]) / launches
    per_launch = per_ss * S
    achieved = per_launch / (avg_ms * 1e-3) / 1e9
    traffic, tsrc, k = None, pmc_note, None
    if pmc_summary:
        traffic, k = split_traffic(pmc_summary, split, tm_name)
        if traffic:
            tsrc = (f"rocprofv3 --pmc passes of the learn-on leg ({pmc_summary}): {k.get('formula', '')}"
                    + (f", {tm_name} + {SP_LEARN_KERNEL}" if split else ""))
    rec = {"value": round(n_total * K / dt, 1), "unit": "stream-steps/s", "steps": K, "warmup": W,
           "ms_per_step": round(dt / K * 1e3, 4), "per_64_steps": per64,
           "config": {"workload": "config3: fresh Model-1 streams (seed 2045+s), SP+TM learning on, lockstep htm_step",
                      "streams_per_gpu": S, "total_streams": n_total, "sp_perm_rows": 800,
                      "sp_perm_rows_used_per_stream": round(eng.sp_perm_rows_used() / S, 1),
                      "live_segments_per_stream": round(c1["seg_live"] / S, 1), "init_s": round(init_s, 2),
                      "device_gb": round(eng.device_bytes() / 1e9, 1)},
           "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                        "traffic_over_algorithmic": round(traffic / per_launch, 3) if traffic else None,
                        "traffic_source": tsrc,
                        "kernel": f"{SP_LEARN_KERNEL} + {tm_name}" if split else tm_name,
                        "avg_launch_ms": round(avg_ms, 4), "sp_kernel_avg_ms": round(prof["sp_ms"] / launches, 4),
                        "tm_kernel_avg_ms": round(prof["tm_ms"] / launches, 4),
                        "bytes_per_launch": int(per_launch), "bytes_per_stream_step": int(per_ss),
                        "bytes_rule": "unique bytes (bench.learn_on_bytes, SURVEY.md 8(d) learning terms)",
                        "issue": issue_record(k)},
           "tm_counters": {k: c1[k] - c0[k] for k in ["inf_phase2", "inf_backtracks", "lrn_phase2", "lrn_backtracks"]}}
    eng.close()
    return rec


def sp_learn_bytes(eng):
    """Algorithmic bytes per stream-step of an SP learning step beyond its
    inference (SURVEY.md 8(d)'s SP learning terms, each byte once): the
    winners' potential permanences read and written and their potential-mask
    rows, both duty-cycle arrays read and written."""
    c = eng.config
    pw = (c.n_fields * c.enc_n + 31) // 32
    n_pot = int(round(c.n_fields * c.enc_n * c.sp_potential_pct))
    return c.sp_num_active * (n_pot * 4 * 2 + pw * 4) + 2 * c.sp_columns * 4 * 2


def bench_test_phase(args, eng, vals, scores, a, n_total, S, rank, world, dev):
    """The reference's test phase: ModelTesting.py:66 -> NetworkModel.py:40-44
    leave SP learning ON and switch TM learning OFF, so a test record runs the
    SP's adaptSynapses / duty cycles and the frozen TM.  The config-2 engine
    (1,024 replicas of the GPU-trained state, after the headline regions),
    `test_phase_warmup` untimed + `test_phase_steps` timed lockstep steps, the
    barrier / max-over-ranks contract.  A lockstep step of this mode runs the
    SP kernel (with learning) and then the TM-only frozen launch
    (htm_run_frozen_kernel, ordered); its roofline is the whole step's
    algorithmic bytes -- the TM kernel's own count plus the SP learning terms
    (sp_learn_bytes) -- over the wall-clock step time (both kernels and the sort
    inside it), a lower bound on the bandwidth the step achieves."""
    W, K = args.test_phase_warmup, args.test_phase_steps
    eng.set_learning(True, False)
    for k in range(a, a + W):
        eng.step(vals[k], out=scores[k])
    import torch
    torch.cuda.synchronize()
    c0 = eng.counters()
    dt, _ = timed_replay(eng, vals, scores, a + W, K, "step", 1, None, None, rank, world, dev)
    c1 = eng.counters()
    if c1["error"]:
        raise RuntimeError(f"test-phase engine overflow flags {c1['error']}")
    tm_per_ss = (c1["tm_bytes"] - c0["tm_bytes"]) / (K * S)
    per_ss = tm_per_ss + sp_learn_bytes(eng)
    achieved = per_ss * S / (dt / K) / 1e9
    eng.set_learning(False, False)
    return {"value": round(n_total * K / dt, 1), "unit": "stream-steps/s", "steps": K, "warmup": W,
            "ms_per_step": round(dt / K * 1e3, 4),
            "config": {"workload": "config2 streams (GPU-trained Model-1 replicas), SP learning ON, TM learning OFF: "
                                   "the reference's test phase (ModelTesting.py:66, NetworkModel.py:40-44), lockstep",
                       "mode": "lockstep: SP kernel with learning, cost-ordered stream list, TM-only frozen launch",
                       "streams_per_gpu": S, "total_streams": n_total},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "bytes_per_stream_step": int(per_ss),
                         "tm_bytes_per_stream_step": int(tm_per_ss), "sp_learn_bytes_per_stream_step": sp_learn_bytes(eng),
                         "time_basis": "wall-clock ms_per_step (SP kernel + sort + TM launch + flushes)",
                         "kernels": "sp_step_ord_kernel<true>, ord_sort_kernel, htm_run_frozen_kernel"},
            "tm_counters": {k: c1[k] - c0[k] for k in ["inf_phase2", "inf_backtracks"]}}


def launch_ranks(n):
    """bench.py --gpus N without a launcher: start N ranks of this same command
    (torch.distributed.run, one process per GPU, rendezvous on 127.0.0.1) and
    return their exit status.  Called before this process touches the GPU."""
    import socket
    import subprocess
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    print(f"bench: launching {n} ranks: {' '.join(cmd[1:])}", file=sys.stderr, flush=True)
    return subprocess.run(cmd).returncode


def bench_build_info(rt):
    """The optimisation level every unit of the loaded library built at
    (htm_build_info, csrc/cc.sh).  The bench kernel's unit must be -O3."""
    info = rt._lib.build_info()
    if info.get("tm_k_frozen.hip") != "-O3":
        raise SystemExit(f"bench.py: the bench kernel (tm_k_frozen.hip) was built at {info.get('tm_k_frozen.hip')}, "
                         "not -O3 (csrc/cc.sh fell back past a gfx950 verifier rejection): refusing to measure it")
    levels = {k: v for k, v in info.items() if k not in ("compiler", "arch")}
    return {"all_units_O3": all(v == "-O3" for v in levels.values()), "bench_kernel_unit": "tm_k_frozen.hip -O3",
            "below_O3": {k: v for k, v in levels.items() if v != "-O3"}, "compiler": info.get("compiler"),
            "arch": info.get("arch")}


def pmc_kernel(path, base):
    pm = json.load(open(path))
    ks = [v for n, v in pm.get("kernels", {}).items()
          if n.split("(")[0].replace("void ", "").strip() == base and ("hbm_bytes_per_dispatch" in v or "sq" in v)]
    return ks[0] if ks else None


# config 5's aggregate fields (StreamEngine/StreamAggregator.py:100-115: cpu %,
# mem %, mean and max response time in ms) in the MultiEncoder's sorted field
# order, each a ScalarEncoder (n 500, w 21, clipped) over its own range
FIELDS5 = (("cpu", 0.0, 100.0), ("max", 0.0, 5000.0), ("mean", 0.0, 2000.0), ("mem", 0.0, 100.0))
C5_KERNEL = "htm_run_frozen_spl_kernel"  # config 5's test phase: SP learning on, TM frozen, run chunks


def config5_inputs(d, n_total, s0, s1, n_rec):
    """Per-record aggregates [n_rec, S, 4] (FIELDS5 order): the reference's
    TestingData aggregate traces (cpu, max, mean, mem) shifted by 97 s per
    stream, cpu and mem with PCG64(724) jitter in {-2..2}, the response
    times scaled by a per-stream factor in [0.9, 1.1]; plus the record's mean
    response time and violation count (the SLO harness's labels)."""
    rng = np.random.Generator(np.random.PCG64(724))
    t_ = np.arange(n_rec)[:, None]
    g_ = np.arange(s0, s1)[None, :]
    idx = (t_ + 97 * g_) % len(d["test_cpu"])
    jit = rng.integers(-2, 3, size=(2, n_rec, n_total))[:, :, s0:s1]
    scale = rng.uniform(0.9, 1.1, size=n_total)[None, s0:s1]
    mean = np.round(d["test_mean"][idx] * scale)
    rec = np.stack([np.clip(d["test_cpu"][idx] + jit[0], 0, 100), np.round(d["test_max"][idx] * scale), mean,
                    np.clip(d["test_mem"][idx] + jit[1], 0, 100)], axis=2).astype(np.float64)
    return rec, mean.astype(np.int32), d["test_violations"][idx].astype(np.int32)


def config5_train_values(d):
    """The reference's training aggregates (FIELDS5 order), records with a
    null field skipped (ModelTraining.py:29-32), the first 2,184."""
    tr = np.stack([d["train_cpu"], d["train_max"].astype(np.float64), d["train_mean"].astype(np.float64),
                   d["train_mem"]], axis=1)
    return tr[~np.isnan(tr).any(axis=1)][:2184]


def run_config5(args, rt, d, world, rank, local, S, warm_rec, n_rec, pmc_summary=None, pmc_note=None):
    """Config 5 (BASELINE.json configs[4]): the Models 2/3 multi-field shape at
    its stated size -- the four aggregate fields (FIELDS5) into a 4096-column SP
    + 12-cell TM, trained on the GPU over the reference's training aggregates
    (one stream, SP+TM learning on), replicated to every stream; then the
    ModelTesting.py test phase (:66-72 -> NetworkModel.py:40-44: SP learning
    on, TM learning off, each record fed 1 + 7 times) and, per record,
    AnomalyLikelihood on the record's score (parity unpinned: NuPIC's
    likelihood, not in the reference) and the SLO harness on its 8-score
    window (ModelTesting.py:75-146, threshold 0.98, avg-response SLO 70 ms).
    N>1 GPUs: streams sharded, every record's likelihoods gathered to rank 0
    over RCCL.  `value` counts network stream-steps (8 per record)."""
    import torch
    import torch.distributed as dist
    W = 8
    dev = f"cuda:{local}"
    n_total = S * world
    s0, s1 = rt.fleet.shard_range(n_total, world, rank)
    mins = tuple(f[1] for f in FIELDS5)
    maxs = tuple(f[2] for f in FIELDS5)
    eng, train_s, hdr, _ = trained_engine(rt, S, args.c5_seg_capacity, local, config5_train_values(d), world=world,
                                          n_fields=4, sp_columns=4096, field_minval=mins, field_maxval=maxs)
    eng.set_learning(True, False)
    rec, means_np, viol_np = config5_inputs(d, n_total, s0, s1, warm_rec + n_rec)
    rec_t = torch.tensor(rec, device=dev)
    vals = rec_t.repeat_interleave(W, dim=0)  # [records * 8, S, 4]: 1 + 7 steps per record
    means = torch.tensor(means_np, device=dev)
    viol = torch.tensor(viol_np, device=dev)
    scores = torch.empty((vals.shape[0], S), dtype=torch.float32, device=dev)
    lik = rt.harness.AnomalyLikelihood(S, device=local)
    slo = rt.harness.SLOHarness(S, threshold=0.98, device=local)
    liks = torch.empty((warm_rec + n_rec, S), dtype=torch.float64, device=dev)
    gather = rt.fleet.ScoreGather(n_total) if world > 1 else None
    gathered = (torch.empty((warm_rec + n_rec, world, gather.width), dtype=torch.float64, device=dev)
                if world > 1 and rank == 0 else None)
    chunk_rec = max(1, args.c5_chunk // W)
    eng.set_run_chunk(chunk_rec * W)

    def replay(r0, r1, handles):
        for a in range(r0, r1, chunk_rec):
            b = min(r1, a + chunk_rec)
            eng.run(vals[a * W:b * W], out=scores[a * W:b * W])
            for r in range(a, b):
                lik.anomaly_probability(rec_t[r], scores[r * W], out=liks[r])
                slo.record(scores[r * W:(r + 1) * W], viol[r], means[r])
                if gather is not None:
                    h, _ = gather.gather(liks[r], staging=gathered[r] if rank == 0 else None)
                    handles.append(h)

    h0 = []
    replay(0, warm_rec, h0)
    for h in h0:
        h.wait()
    torch.cuda.synchronize()
    c0 = eng.counters()
    if not args.no_profile:
        eng.profile(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    handles = []
    replay(warm_rec, warm_rec + n_rec, handles)
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
        raise RuntimeError(f"config-5 engine overflow flags {c1['error']}")
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    steps = n_rec * W
    roof = None
    if prof is not None and prof["tm_ms"] > 0:
        # the fused kernel's own count of what it moves (frozen-index blocks,
        # records, state) plus the SP learning terms per
        # stream-step, over the HIP-event time of its launches
        launches = prof["launches"]
        per_launch = ((c1["tm_bytes"] - c0["tm_bytes"]) / launches
                      + sp_learn_bytes(eng) * S * prof["steps"] / launches)
        avg_ms = prof["tm_ms"] / launches
        achieved = per_launch / (avg_ms * 1e-3) / 1e9
        traffic, k = None, None
        if pmc_summary:
            k = pmc_kernel(pmc_summary, C5_KERNEL)
            traffic = int(k["hbm_bytes_per_dispatch"]) if k and "hbm_bytes_per_dispatch" in k else None
        roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                "traffic_over_algorithmic": round(traffic / per_launch, 3) if traffic else None,
                "traffic_source": (f"rocprofv3 --pmc passes of the config-5 workload ({pmc_summary}): "
                                   f"{k.get('formula', '')}" if traffic else pmc_note),
                "kernel": C5_KERNEL + " (fused SP+TM run chunks: 4096 columns, 4 fields, SP learning on)",
                "avg_launch_ms": round(avg_ms, 4), "steps_per_launch": prof["steps"] / launches,
                "bytes_per_launch": int(per_launch), "issue": issue_record(k)}
    st = slo.stats()
    out = {
        "value": round(n_total * steps / dt, 1), "unit": "stream-steps/s",
        "predictions_per_s": round(n_total * n_rec / dt, 1),
        "steps": steps, "warmup": warm_rec * W, "ms_per_step": round(dt / steps * 1e3, 4),
        "dtype": "int32+f32+f64",
        "data": "synthetic: the reference's TestingData aggregates (cpu, max, mean, mem) shifted per stream, "
                "PCG64(724) jitter, resident in HBM",
        "config": {"workload": "config5: cpu/max/mean/mem ScalarEncoders (2000 bits, per-field ranges) -> 4096-col SP "
                               "+ 12-cell TM from the GPU-trained state; the test phase (SP learn on, TM off), per "
                               "record 1+7 steps + AnomalyLikelihood + SLO harness (0.98)",
                   "fields": [f[0] for f in FIELDS5], "field_ranges": [[f[1], f[2]] for f in FIELDS5],
                   "mode": f"run chunks of {chunk_rec} records ({chunk_rec * W} steps), then per record the "
                           "likelihood and SLO kernels", "streams_per_gpu": S, "total_streams": n_total,
                   "columns": 4096, "cells_per_column": 12, "records": n_rec,
                   "trained_segments": int(hdr.seg_live), "train_s": round(train_s, 2),
                   "parallelism": f"streams sharded over {world} GPU(s)" +
                                  (", RCCL gather of likelihoods" if world > 1 else "")},
        "roofline": roof,
        "tm_counters": {k: c1[k] - c0[k] for k in ["inf_phase2", "inf_backtracks"]},
        "slo_totals": {k: int(v) for k, v in zip(["TP", "FP", "TN", "FN", "lead_sum"], st.sum(axis=0))},
    }
    lik.close()
    slo.close()
    eng.close()
    return out


def bench_config5(args, rt, d, world, rank, local):
    """bench.py --config 5: the config-5 workload (run_config5) as the line."""
    out = run_config5(args, rt, d, world, rank, local, args.streams, args.warmup // 8, args.steps // 8,
                      args.pmc_summary)
    line = {"metric": METRIC, "value": out.pop("value"), "unit": out.pop("unit"), "n_gpus": world,
            "steps": out.pop("steps"), "warmup": out.pop("warmup"), "ms_per_step": out.pop("ms_per_step"),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None}
    line.update(out)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def bench_single_stream(rt, src, trace, local, n_rec=256, warm_rec=16):
    """One Model-1 stream at the reference's own granularity: a prediction is
    one test record -- ModelTesting.py:66-72 feeds it 1 + 7 times
    (runNetwork, NetworkModel.py:35-44: SP learning on, TM learning off) and
    compares the eight scores on the host (:75-79).  The stream is the
    GPU-trained Model-1 state (`src` stream 0).  Timed per record, the scores
    copied to the host each record (the alarm decision): `lockstep_steps`
    (eight htm_step launches per record), `run_chunk` (the record's eight steps
    as one htm_run launch), and `facade` -- the reference's whole call pattern
    through the drop-in Network (tests/reference_model1.py: setData, run(1),
    getOutputData('anomalyScore')[0] eight times, the SDRClassifierRegion
    running beside it on the GPU).  Beside it the published 20-50 ms per
    prediction."""
    import torch
    dev = f"cuda:{local}"
    one = rt.HTMEngine(1, device=local, seg_capacity=72 * 1024)
    for region in rt._lib.ST:
        one.import_state(region, src.export_state(region, 0, 1), s0=0)
    one.set_learning(True, False)
    recs = trace[np.arange(warm_rec + n_rec) % len(trace)].astype(np.float64)
    v = torch.tensor(recs, device=dev)
    win = torch.empty((8, 1), dtype=torch.float32, device=dev)
    res = {}
    for name in ("lockstep_steps", "run_chunk"):
        for r in range(warm_rec + n_rec):
            if r == warm_rec:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            if name == "lockstep_steps":
                for j in range(8):
                    one.step(v[r:r + 1], out=win[j])
            else:
                one.run(v[r:r + 1].expand(8).reshape(8, 1), out=win)
            host = win.cpu().numpy()  # the host's alarm decision reads the window
        dt = time.perf_counter() - t0
        res[name] = {"ms_per_prediction": round(dt / n_rec * 1e3, 4), "records": n_rec,
                     "predictions_per_s": round(n_rec / dt, 1)}
    one.close()
    # the drop-in surface: Model 1 built and trained through the facade
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import reference_model1 as ref
    d = np.load(os.path.join(ROOT, "tests", "golden", "model1_traces.npz"))
    ds = rt.BatchRecordStream(["cpu"])
    net = ref.create_one_level_network(rt, ds, seg_capacity=72 * 1024, device=local)
    tmr = net.regions[ref.TMR]
    t0 = time.perf_counter()
    n_train = 0
    for cpu in d["train_cpu"]:
        if np.isnan(cpu):
            continue
        ds.setData(float(cpu))
        net.run(1)
        n_train += 1
        if n_train == 2184:
            break
    train_s = time.perf_counter() - t0
    f_rec = min(n_rec, 128)
    for r in range(warm_rec + f_rec):
        if r == warm_rec:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        w = []
        for j in range(8):
            ds.setData(float(recs[r]))
            if j == 0:
                tmr.setParameter("learningMode", False)  # NetworkModel.py:40-44
            net.run(1)
            w.append(tmr.getOutputData("anomalyScore")[0])
    dt = time.perf_counter() - t0
    res["facade"] = {"ms_per_prediction": round(dt / f_rec * 1e3, 4), "records": f_rec,
                     "predictions_per_s": round(f_rec / dt, 1), "train_records": n_train,
                     "train_ms_per_record": round(train_s / n_train * 1e3, 4),
                     "note": "Network facade + SDRClassifierRegion (steps 1..7) on the GPU, one stream"}
    del net
    res["workload"] = ("config 1 at its own granularity: one Model-1 stream (GPU-trained state), ModelTesting's "
                       "test phase, a prediction = one record = 1 + 7 network.run(1) steps (SP learn on, TM off) "
                       "and the eight scores read on the host")
    res["reference_published"] = {"ms_per_prediction": "20-50", "hardware": "AWS t2.large (2 vCPU), NuPIC 1.0.x",
                                  "source": "CSC 724 Final Project Report p.8 (SURVEY.md §6)"}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs of this node, one rank each (default 1).  Without WORLD_SIZE in the environment "
                         "and N > 1, bench.py launches the N ranks itself (torch.distributed.run, before any GPU "
                         "call) and exits with their status; under a launcher it must equal WORLD_SIZE")
    ap.add_argument("--cpu-standin", action="store_true",
                    help="launcher test only (tests/test_bench_launch.py): gloo on the CPU with a deterministic "
                         "stand-in engine in place of the HIP engine -- exercises the rank launch, sharding, "
                         "gathers and max-over-ranks timing; its line says so and measures nothing")
    ap.add_argument("--config", type=int, choices=[2, 3, 4, 5], default=2,
                    help="2 (default, the metric's config): trained Model-1 streams, learning off; "
                         "3: fresh streams (seed 2045 + s), SP+TM learning on, 256 steps; "
                         "4: fleet -- 131,072 streams per GPU sharing one frozen trained model; "
                         "5: cpu+mem encoders, 4096-column SP, AnomalyLikelihood + SLO harness per record")
    ap.add_argument("--steps", type=int, default=None, help="timed steps (config 2: 2324, config 3: 240)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (config 2: 64, config 3: 16)")
    ap.add_argument("--condition", type=int, default=None,
                    help="configs 2 and 4: records every stream steps through (untimed, in the measured mode) "
                         "before the warm-up, so the timed steps see streams in their steady state rather than "
                         "the transient of a state trained elsewhere meeting a new trace position (SURVEY.md 8(d) "
                         "config 2's 64-step warm-up; default 64, 0 = off)")
    ap.add_argument("--streams", type=int, default=None,
                    help="streams per GPU (config 2: 1024; config 3: 65536, BASELINE.json configs[2])")
    ap.add_argument("--sp-perm-rows", type=int, default=None,
                    help="paged SP permanences: pool rows per stream (config 3: 800 -- fresh streams touch "
                         "~25-30%% of their 2048 columns in 256 steps; 0 = dense)")
    ap.add_argument("--seg-capacity", type=int, default=None, help="segment slots per stream")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU oracle baseline")
    ap.add_argument("--no-profile", action="store_true", help="no per-kernel HIP events")
    ap.add_argument("--profile-every", type=int, default=5,
                    help="HIP events around every N-th launch of the timed region (HTM_OPT_PROFILE N; a timed "
                         "event record between dependent launches holds the queue ~12 us, so the roofline's "
                         "launch time is averaged over a sample: default every 5th -- prime to the deferred "
                         "flush's cadence (round 5: 8 steps, whose following launch ran beside the flush: every 4th "
                         "sampled that launch in half its samples, profiles/r05_ab/README.md; round 6: 6)")
    ap.add_argument("--mode", choices=["step", "run"], default="step",
                    help="step (default, the headline): lockstep -- one htm_step per step, every stream "
                         "advances one network.run(1) per step (north_star's real-time stepping); run: the K "
                         "steps as htm_run replay chunks, each stream steps through a chunk without waiting "
                         "for the others (the reference's offline replay of recorded metrics, batched)")
    ap.add_argument("--chunk", type=int, default=None,
                    help="steps per htm_run call (= per fused launch) in run mode (config 2: 2324, the "
                         "TestingData replay in one launch, whatever --steps is; 3, 5: 256; 4: 64)")
    ap.add_argument("--run-unit", type=int, default=None, help="engine: steps per work-queue unit (HTM_OPT_RUN_UNIT)")
    ap.add_argument("--other-steps", type=int, default=None,
                    help="after the timed region, also time this many steps in the other mode (run mode "
                         "beside the lockstep headline; config 2: 2324, config 4: 64, config 3: 0 = skip)")
    ap.add_argument("--pmc-summary", default=None,
                    help="JSON from tools/pmc_summary.py over rocprofv3 --pmc passes of this same command "
                         "(same gpurun call): fills roofline.traffic")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the counter passes bench.py runs itself (N=1) to fill roofline.traffic")
    ap.add_argument("--pmc-full", action="store_true",
                    help="every counter pass on every leg: FETCH_SIZE (a cross-check of the request-size formula, "
                         "calibrated in profiles/r02_final) and all three SQ passes on the learn_on and config5 legs "
                         "(default: the config-2 kernel gets all SQ passes, the other legs SQ pass 1 only)")
    ap.add_argument("--no-learn-on", action="store_true",
                    help="config 2: skip the learn_on sub-record (config 3's learning streams, BASELINE's 'learn on')")
    ap.add_argument("--learn-streams", type=int, default=65536, help="learn_on: streams per GPU")
    ap.add_argument("--learn-steps", type=int, default=240,
                    help="learn_on: timed lockstep steps (SURVEY.md 8(d) config 3: T = 256 = 16 untimed + 240)")
    ap.add_argument("--learn-warmup", type=int, default=16, help="learn_on: untimed steps")
    ap.add_argument("--pmc-summary-learn", default=None, help="counter summary of the learn_on leg (see --pmc-summary)")
    ap.add_argument("--no-test-phase", action="store_true",
                    help="config 2: skip the test_phase sub-record (SP learning on, TM learning off: the "
                         "reference's test phase, NetworkModel.py:40-44)")
    ap.add_argument("--test-phase-steps", type=int, default=256, help="test_phase: timed lockstep steps")
    ap.add_argument("--test-phase-warmup", type=int, default=16, help="test_phase: untimed steps")
    ap.add_argument("--no-config5", action="store_true",
                    help="config 2: skip the config5 sub-record (BASELINE configs[4] on this GPU's shard)")
    ap.add_argument("--c5-streams", type=int, default=1024, help="config5 sub-record: streams per GPU")
    ap.add_argument("--c5-records", type=int, default=64, help="config5 sub-record: timed test records (8 steps each)")
    ap.add_argument("--c5-warmup-records", type=int, default=8, help="config5 sub-record: untimed test records")
    ap.add_argument("--c5-chunk", type=int, default=256, help="config 5: steps per htm_run chunk")
    ap.add_argument("--c5-seg-capacity", type=int, default=128 * 1024, help="config 5: segment slots per stream")
    ap.add_argument("--pmc-summary-c5", default=None, help="counter summary of the config5 leg (see --pmc-summary)")
    ap.add_argument("--no-single-stream", action="store_true",
                    help="config 2: skip the single_stream sub-record (one Model-1 stream, ms per prediction)")
    ap.add_argument("--flush-mode", choices=["auto", "0", "1"], default="auto",
                    help="where the deferred-write flush runs (HTM_OPT_FLUSH_MODE): 0 beside the steps on the "
                         "engine's own HIP stream, 1 on the step stream; auto: the engine's default")
    ap.add_argument("--flush-every", type=int, default=0,
                    help="HTM_OPT_FLUSH_EVERY: lockstep steps between the periodic deferred-write flushes (0: the "
                         "engine default, 4)")
    ap.add_argument("--ordered", choices=["on", "off"], default="on",
                    help="HTM_OPT_ORDERED: frozen lockstep steps run their TM steps heaviest first (on, the engine "
                         "default) or one fused SP+TM workgroup per stream in stream order (off); results identical")
    ap.add_argument("--split-learn", choices=["on", "off"], default="on",
                    help="HTM_OPT_SPLIT_LEARN (config 3 and the learn_on leg): learning lockstep steps run the SP "
                         "kernel then the TM-only learning kernel (on, the engine default) or one fused kernel (off); "
                         "results identical")
    ap.add_argument("--shape", choices=["model1", "yaml"], default="model1",
                    help="model1 (default): the reference's Model-1 parameters (12 cells/column); yaml: the "
                         "reference's model.yaml set (RDSE, boostStrength 3, 32 cells/column; configs 2 and 4)")
    args = ap.parse_args()
    c3, c4, c5 = args.config == 3, args.config == 4, args.config == 5
    if c5:
        args.steps = 2048 if args.steps is None else args.steps
        args.warmup = 64 if args.warmup is None else args.warmup
        args.streams = args.c5_streams if args.streams is None else args.streams
        if args.seg_capacity is not None:
            args.c5_seg_capacity = args.seg_capacity
        if args.chunk is not None:
            args.c5_chunk = args.chunk
    if args.steps is None:
        args.steps = 240 if c3 else 256 if c4 else 2324
    if args.warmup is None:
        args.warmup = 16 if (c3 or c4) else 64
    if args.streams is None:
        args.streams = 65536 if c3 else 131072 if c4 else 1024
    if args.sp_perm_rows is None:
        args.sp_perm_rows = 800 if c3 else 0
    if args.seg_capacity is None:
        args.seg_capacity = 10240 if c3 else (1 << 17) if args.shape == "yaml" else 72 * 1024
    if args.chunk is None:
        args.chunk = 64 if c4 else 256 if (c3 or c5) else 2324
    if args.other_steps is None:
        args.other_steps = 0 if c3 else 64 if c4 else 2324
    if args.condition is None:
        args.condition = 0 if c3 else 64
    if c4:
        args.chunk = min(args.chunk, int(os.environ.get("HTM_C4_MAX_CHUNK", "64")))
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and (args.gpus or 1) > 1:
        # one process per GPU: launch the N ranks (before this process touches
        # the GPU) and report their status
        sys.exit(launch_ranks(args.gpus))
    if world_env is not None and args.gpus is not None and int(world_env) != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} disagrees with WORLD_SIZE={world_env}")
    standin = args.cpu_standin
    if standin:
        args.no_learn_on = args.no_cpu = args.no_pmc = args.no_profile = True
    learn_on = args.config == 2 and not args.no_learn_on and args.shape == "model1"
    config5 = args.config == 2 and not args.no_config5 and args.shape == "model1" and not standin
    pmc_note = pmc_note_learn = pmc_note_c5 = None
    if (int(world_env or "1") == 1 and not args.no_pmc
            and not os.environ.get("HTM_BENCH_PMC_CHILD")):
        # before this process touches the GPU: the HBM counter passes, each a
        # short run of this same command under rocprofv3 in a child process
        if not args.pmc_summary:
            args.pmc_summary, pmc_note = self_pmc_passes(args)
        if learn_on and not args.pmc_summary_learn:
            args.pmc_summary_learn, pmc_note_learn = self_pmc_passes(args, learn_leg=True)
        if config5 and not args.pmc_summary_c5:
            args.pmc_summary_c5, pmc_note_c5 = self_pmc_passes(args, c5_leg=True)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if standin:
        dev = "cpu"
        sync = lambda: None  # noqa: E731
    else:
        torch.cuda.set_device(local)
        dev = f"cuda:{local}"
        sync = torch.cuda.synchronize
    if world > 1:
        dist.init_process_group("gloo" if standin else "nccl")
    import _pkg
    rt = _pkg.load()
    build = None if standin else bench_build_info(rt)

    d = np.load(os.path.join(ROOT, "tests", "golden", "model1_traces.npz"))
    if c5:
        return bench_config5(args, rt, d, world, rank, local)
    train_vals = [c for c, m in zip(d["train_cpu"], d["train_mem"]) if not (np.isnan(c) or np.isnan(m))][:2184]
    trace = d["test_cpu"].astype(np.float64)

    S = args.streams
    n_total = S * world
    s0, s1 = rt.fleet.shard_range(n_total, world, rank)
    # the reference's model.yaml parameter set (RDSE, boosting, 32 cells/column) or Model 1
    shape = dict(rt._lib.MODEL_YAML) if args.shape == "yaml" else {}
    if standin:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import bench_standin
        eng = bench_standin.StandInEngine(S, s0)
        train_s, hdr, model_dist = 0.0, None, "cpu stand-in (launcher test: no HTM compute)"
    elif c3:
        # fresh per-stream init (seeds 2045 + global stream index), learning on
        cfg = rt.default_config(seg_capacity=args.seg_capacity, upd_capacity=512, seed_stride=1,
                                sp_seed=2045 + s0, tm_seed=2045 + s0, sp_perm_rows=args.sp_perm_rows)
        t0 = time.time()
        eng = rt.HTMEngine(S, config=cfg, device=local)
        sync()
        train_s, hdr, model_dist = time.time() - t0, None, "fresh per-stream init"
        eng.set_learning(True, True)
        eng.split_learning(args.split_learn == "on")
    elif c4:
        # one model trained on the GPU (2184 Model-1 records), shared by every stream
        model, train_s, hdr, model_dist = trained_engine(rt, 1, args.seg_capacity, local, train_vals, world=world,
                                                         **shape)
        eng = rt.HTMEngine.fleet(model, S, q_capacity=4096)
        model.close()
    else:
        eng, train_s, hdr, model_dist = trained_engine(rt, S, args.seg_capacity, local, train_vals, world=world,
                                                       **shape)
        eng.set_learning(False, False)
    single = (args.config == 2 and args.shape == "model1" and not args.no_single_stream and not standin
              and rank == 0)
    if single:
        # the GPU-trained Model-1 state, for the single-stream record after the headline
        single_src = rt.HTMEngine(1, device=local, seg_capacity=args.seg_capacity)
        for region in rt._lib.ST:
            single_src.import_state(region, eng.export_state(region, 0, 1), s0=0)
    if not c3:
        eng.set_run_chunk(args.chunk)  # one fused launch per htm_run call
    if args.flush_mode != "auto" and not standin:
        eng.flush_mode(int(args.flush_mode))
    if args.run_unit:
        eng.set_run_unit(args.run_unit)
    if args.ordered == "off" and not standin:
        eng.ordered_steps(False)
    if args.flush_every and not standin:
        eng.flush_every(args.flush_every)
    C = args.condition
    # the reference's test phase (SP learning on, TM learning off) on the same
    # engine after the headline and run-mode regions: config 2, Model-1 shape
    test_phase = (args.config == 2 and args.shape == "model1" and not args.no_test_phase and not standin
                  and args.test_phase_steps > 0)
    TP0 = C + args.warmup + args.steps + args.other_steps
    T = TP0 + ((args.test_phase_warmup + args.test_phase_steps) if test_phase else 0)
    if c4:
        # per-rank jitter stream (a 1M x T matrix per rank would not fit host memory)
        rng = np.random.Generator(np.random.PCG64([724, s0]))
        t_ = np.arange(T)[:, None]
        g_ = np.arange(s0, s1)[None, :]
        vals = torch.tensor(np.clip(trace[(t_ + 97 * g_) % len(trace)] + rng.integers(-2, 3, size=(T, S)), 0, 100)
                            .astype(np.float64), device=dev)
    else:
        vals = torch.tensor(make_inputs(n_total, s0, s1, 0, T, trace), device=dev)
    scores = torch.empty((T, S), dtype=torch.float32, device=dev)
    gather = rt.fleet.ScoreGather(n_total) if world > 1 else None
    gathered = None
    if world > 1 and rank == 0:
        gathered = (torch.empty((world, args.steps, gather.width), dtype=torch.float32, device=dev)
                    if args.mode == "run" else
                    torch.empty((args.steps, world, gather.width), dtype=torch.float32, device=dev))

    # conditioning and warm-up in the measured mode: lockstep steps also bring
    # the deferred-duty log to its steady state (its ring starts empty; the
    # first lockstep steps after replay chunks log every new active set)
    for a0, n_ in ((0, C), (C, args.warmup)):
        if not n_:
            continue
        if args.mode == "step":
            for k in range(a0, a0 + n_):
                eng.step(vals[k], out=scores[k])
        else:
            eng.run(vals[a0:a0 + n_], out=scores[a0:a0 + n_])
    sync()
    c0 = eng.counters()
    if not args.no_profile:
        eng.profile(True, every=args.profile_every if args.mode == "step" else 1)
    # the timed region: K steps bracketed by barrier + synchronize, max over ranks
    dt, _ = timed_replay(eng, vals, scores, C + args.warmup, args.steps, args.mode, args.chunk, gather, gathered,
                         rank, world, dev)
    prof = eng.profile_read() if not args.no_profile else None
    eng.profile(False)
    c1 = eng.counters()
    if c1["error"]:
        raise RuntimeError(f"engine overflow flags {c1['error']}")
    value = n_total * args.steps / dt
    other = None
    if args.other_steps > 0:
        # the other mode on the same engine: run mode (each stream steps through the
        # chunk without waiting for the others) beside the lockstep headline, or back
        omode = "run" if args.mode == "step" else "step"
        base = C + args.warmup + args.steps
        dl, _ = timed_replay(eng, vals, scores, base, args.other_steps, omode, args.other_steps, None, None,
                             rank, world, dev)
        other = {"mode": omode, "value": round(n_total * args.other_steps / dl, 1), "steps": args.other_steps,
                 "ms_per_step": round(dl / args.other_steps * 1e3, 4)}
    tp_rec = bench_test_phase(args, eng, vals, scores, TP0, n_total, S, rank, world, dev) if test_phase else None
    shape_name = ("model.yaml-shape (RDSE resolution 0.88, SP boostStrength 3.0, 2048 columns, 32-cell "
                  "BacktrackingTM; ML/HTM/params/model.yaml)" if args.shape == "yaml" else
                  "Model-1 (2048-col SP, 12-cell BacktrackingTM)")
    # the engine's ordered lockstep path (HTM_OPT_ORDERED): frozen, one step per
    # launch, dense SP permanences, at most 16,384 streams per GPU
    ordered = (args.ordered == "on" and args.mode == "step" and S <= 16384 and not c3 and not args.sp_perm_rows
               and not standin)
    roof = None
    split = c3 and args.split_learn == "on" and args.mode == "step" and not standin
    if prof is not None and prof["tm_ms"] > 0:
        launches = prof["launches"]
        avg_ms = (prof["tm_ms"] + (prof["sp_ms"] if split else 0.0)) / launches
        if c3:  # learning: unique bytes (the in-kernel count charges every pool re-scan)
            per_launch = learn_on_bytes(eng, S, (c0["seg_live"] + c1["seg_live"]) / 2) * S * prof["steps"] / launches
        else:   # frozen inference: the kernel's own count of the index blocks and state it moves,
            # over every launch of the timed region (the events sample some of them)
            all_launches = args.steps if args.mode == "step" else -(-args.steps // args.chunk)
            per_launch = (c1["tm_bytes"] - c0["tm_bytes"]) / all_launches
        achieved = per_launch / (avg_ms * 1e-3) / 1e9
        traffic, tsrc, k = None, pmc_note, None
        if args.pmc_summary:
            # HBM bytes per launch measured by rocprofv3 --pmc passes of THIS command
            # (tools/pmc_summary.py, run in the same gpurun call; corrections there)
            traffic, k = split_traffic(args.pmc_summary, split, kernel_name(c3, c4, eng.fused, split, ordered))
            if traffic:
                tsrc = (f"rocprofv3 --pmc passes of this command ({args.pmc_summary}): {k.get('formula', '')}; "
                        "calibrated on tools/fetch_calib (profiles/r02_final/pmc_summary.json)")
        roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                "traffic_over_algorithmic": round(traffic / per_launch, 3) if traffic else None,
                "traffic_source": tsrc,
                "kernel": (f"{SP_LEARN_KERNEL} + " if split else "") + kernel_name(c3, c4, eng.fused, split, ordered),
                "avg_launch_ms": round(avg_ms, 4), "steps_per_launch": prof["steps"] / launches,
                "profiled_launches": launches, "bytes_per_launch": int(per_launch), "issue": issue_record(k),
                "sp_kernel_avg_ms": round(prof["sp_ms"] / launches, 4) if not ordered else None}
        if ordered:
            roof["sp_kernel_note"] = ("ordered launches: the HIP events bracket the TM launch only; the SP kernel "
                                      "(sp_step_ord_kernel) and ord_sort_kernel before it are untimed here (their "
                                      "rocprofv3 kernel-trace averages are in profiles/<round>/kernel_stats.csv) "
                                      "but inside ms_per_step")
        if c4:
            # a fleet's streams share one model: its index and records are read
            # from the XCD L2s and the Infinity Cache, so the bytes the kernel
            # requests are not HBM bytes.  frac is the counter-measured HBM
            # traffic / time; the requested bytes are set against the L2 side
            # (aggregate L2 bandwidth, MI355X_MICROARCH.md, with the TCC hit rate)
            req_gbs = achieved
            hbm_gbs = traffic / (avg_ms * 1e-3) / 1e9 if traffic else None
            roof["achieved"] = round(hbm_gbs, 2) if hbm_gbs is not None else None
            roof["frac"] = round(hbm_gbs / HBM_PEAK_GBS, 5) if hbm_gbs is not None else None
            roof["frac_basis"] = ("counter HBM bytes per launch / HIP-event launch time" if hbm_gbs is not None else
                                  "no counters: HBM fraction not measured (requested bytes are L2-served)")
            l2 = (k or {}).get("l2") or {}
            roof["l2_side"] = {"requested_gbs": round(req_gbs, 2), "peak": L2_PEAK_GBS, "unit": "GB/s",
                               "frac": round(req_gbs / L2_PEAK_GBS, 5), "tcc_hit_rate": l2.get("hit_rate"),
                               "tcc_req_per_launch": l2.get("req"),
                               "basis": "bytes the kernel requests per launch (its own count: index blocks, "
                                        "records, state) / launch time, against the aggregate L2 bandwidth; "
                                        "hit rate TCC_HIT/(TCC_HIT+TCC_MISS) from the pmc_l2 pass"}
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "stream-steps/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int32+f32",
        "data": ("CPU STAND-IN ENGINE (launcher test; no HTM compute, not a measurement)" if standin else
                 "synthetic: TestingData cpu trace + PCG64(724) jitter, resident in HBM (SURVEY.md §8(d) config %d)"
                 % args.config),
        "config": {"workload": ("config3: fresh Model-1 streams (seed 2045+s), SP+TM learning on" if c3 else
                                "config4 fleet: streams sharing one frozen GPU-trained %s SP+TM, "
                                "per-stream TM state, learn off" % shape_name if c4 else
                                "config2: %s streams, SP+TM learn off, from the GPU-trained state" % shape_name),
                   "shape": args.shape,
                   "mode": ("lockstep: one htm_step per step, every stream advances one network.run(1) per step"
                            + (" (ordered: SP kernel, cost-ordered stream list, TM steps heaviest first)"
                               if ordered else "")
                            if args.mode == "step" else
                            "run: htm_run replay chunks, each stream steps through a chunk without waiting"),
                   "conditioning_steps": C, "flush_mode": args.flush_mode, "ordered": args.ordered,
                   "flush_every": args.flush_every,
                   "streams_per_gpu": S, "total_streams": n_total, "columns": eng.n_columns,
                   "cells_per_column": eng.cells_per_column,
                   "trained_segments": int(hdr.seg_live) if hdr is not None else None,
                   "segments_after": int(c1["seg_live"] // S) if c3 else None,
                   "sp_perm_rows": ({"per_stream": args.sp_perm_rows, "used_per_stream": round(eng.sp_perm_rows_used() / S, 1),
                                     "device_gb": round(eng.device_bytes() / 1e9, 1)} if c3 else None),
                   ("init_s" if c3 else "train_s"): round(train_s, 2),
                   "model_distribution": model_dist,
                   "parallelism": f"streams sharded over {world} GPU(s)" + (", RCCL gather of scores" if world > 1 else ""),
                   "build": build},
        "roofline": roof,
        "tm_counters": {k: c1[k] - c0[k] for k in ["inf_phase2", "inf_backtracks"]},
        ("run_mode" if args.mode == "step" else "lockstep"): other,
    }
    if tp_rec is not None:
        out["test_phase"] = tp_rec
    if rank == 0 and world == 1 and not args.no_cpu and not c3 and not c4 and args.shape == "model1":
        out["cpu_baseline"] = cpu_baseline(trace, train_vals, n_total)
    eng.close()
    if single:
        out["single_stream"] = bench_single_stream(rt, single_src, trace, local)
        single_src.close()
    if config5:
        out["config5"] = run_config5(args, rt, d, world, rank, local, args.c5_streams, args.c5_warmup_records,
                                     args.c5_records, args.pmc_summary_c5, pmc_note_c5)
    if learn_on:
        out["learn_on"] = bench_learn_on(args, rt, trace, world, rank, local, args.pmc_summary_learn, pmc_note_learn)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


# rocprofv3 --pmc passes (one run each; TCC block: 4 counters, FETCH_SIZE costs 3,
# WRITE_SIZE 2): L2 memory-side requests by size, FETCH_SIZE, writes
PMC_PASSES = {
    "pmc_rd": ["TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum"],
    "pmc_wr": ["WRITE_SIZE", "TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum"],
}
PMC_FETCH_PASS = {"pmc_fetch": ["FETCH_SIZE"]}  # (--pmc-full: traffic uses the request-size formula)
PMC_L2_PASS = {"pmc_l2": ["TCC_HIT_sum", "TCC_MISS_sum", "TCC_REQ_sum"]}
# where the waves' cycles go (SQ block: 8 counters per pass, SQ_WAVE_CYCLES in
# each so every pass normalises itself): issuing / parked on s_waitcnt or
# s_barrier / ready but not issued, per-unit issue, LDS bank conflicts
PMC_SQ_PASSES = {
    "pmc_sq1": ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"],
    "pmc_sq2": ["SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_FLAT",
                "SQ_WAIT_INST_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_INSTS_VALU"],
    "pmc_sq3": ["SQ_WAVE_CYCLES", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                "SQ_INST_LEVEL_VMEM", "SQ_INSTS_BRANCH", "SQ_ACTIVE_INST_MISC"],
}
SQ_LEARN_STEPS = 48  # the learn leg's SQ passes time this many steps (after its warm-up): fractions, not bytes


def issue_record(k):
    """roofline.issue: the SQ fractions of the dominant kernel's wave-cycles."""
    sq = (k or {}).get("sq")
    if not sq:
        return None
    keys = ("issue_active", "waiting", "issue_stalled", "valu", "salu", "lds", "vmem", "flat", "lds_issue_stalled",
            "lds_bank_conflict_over_lds_active", "cycles_per_wave", "waves")
    rec = {x: sq.get(x) for x in keys if sq.get(x) is not None}
    rec["basis"] = ("rocprofv3 SQ counter passes of this workload (median per dispatch): fractions of SQ_WAVE_CYCLES; "
                    "waiting = SQ_WAIT_ANY (parked on s_waitcnt for memory / LDS or on s_barrier), issue_stalled = "
                    "SQ_WAIT_INST_ANY, issue_active = SQ_ACTIVE_INST_ANY")
    return rec


def self_pmc_passes(args, steps=128, learn_leg=False, c5_leg=False):
    """Run this benchmark's workload (same config/streams, `steps` timed steps,
    the same launch shape as the timed region) under rocprofv3 once per
    counter pass and summarise them (tools/pmc_summary.py); learn_leg: the
    learn_on leg's workload (config 3 at --learn-streams, lockstep).  Returns
    (summary path, note); (None, reason) when the passes cannot run."""
    import shutil
    import subprocess
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    prof = shutil.which("rocprofv3")
    if not prof:
        return None, "rocprofv3 not found: traffic not measured"
    out = tempfile.mkdtemp(prefix="htm_pmc_", dir="/tmp")
    if learn_leg:
        child = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", "3", "--steps", str(args.learn_steps),
                 "--warmup", str(args.learn_warmup), "--other-steps", "0", "--no-cpu", "--no-profile", "--no-pmc", "--mode", "step",
                 "--streams", str(args.learn_streams), "--split-learn", args.split_learn]
    elif c5_leg or args.config == 5:
        recs, warm = (args.c5_records, args.c5_warmup_records) if c5_leg else (args.steps // 8, args.warmup // 8)
        child = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", "5", "--steps", str(8 * recs),
                 "--warmup", str(8 * warm), "--no-profile", "--no-pmc", "--streams",
                 str(args.c5_streams if c5_leg else args.streams), "--c5-chunk", str(args.c5_chunk),
                 "--c5-seg-capacity", str(args.c5_seg_capacity)]
    else:
        child = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", str(args.config), "--steps", str(steps),
                 "--warmup", "8", "--other-steps", "0", "--no-cpu", "--no-profile", "--no-pmc", "--mode", args.mode,
                 "--no-learn-on", "--no-test-phase", "--no-config5", "--no-single-stream", "--shape", args.shape]
        if args.flush_mode != "auto":
            child += ["--flush-mode", args.flush_mode]
        if args.ordered != "on":
            child += ["--ordered", args.ordered]
        if args.flush_every:
            child += ["--flush-every", str(args.flush_every)]
        for k in ("streams", "seg_capacity", "chunk", "run_unit", "sp_perm_rows", "condition"):
            v = getattr(args, k)
            if v is not None:
                child += ["--" + k.replace("_", "-"), str(v)]
    env = dict(os.environ, TMPDIR="/tmp", HTM_BENCH_PMC_CHILD="1")
    passes = dict(PMC_PASSES)
    full = getattr(args, "pmc_full", False)
    if full:
        passes.update(PMC_FETCH_PASS)
    if args.config == 4 and not learn_leg:
        passes.update(PMC_L2_PASS)  # the fleet's shared model is read from L2: its hit rate
    if (c5_leg or learn_leg) and not full:
        # the sub-record legs: one SQ pass (issue / wait fractions) -- keeps the
        # default run's 11 counter passes inside a few minutes
        passes.update({"pmc_sq1": PMC_SQ_PASSES["pmc_sq1"]})
    else:
        passes.update(PMC_SQ_PASSES)
    for name, counters in passes.items():
        t0 = time.time()
        cc = list(child)
        if learn_leg and name in PMC_SQ_PASSES:  # fractions: a shorter region of the same workload
            cc[cc.index("--steps") + 1] = str(min(args.learn_steps, SQ_LEARN_STEPS))
        cmd = [prof, "--pmc", *counters, "--output-format", "csv", "-d", os.path.join(out, "run", name), "-o", "run",
               "--", *cc]
        try:
            r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=420)
        except subprocess.TimeoutExpired:
            return None, "rocprofv3 pass %s timed out: traffic not measured" % name
        if r.returncode != 0:
            return None, "rocprofv3 pass %s failed (rc %d): traffic not measured" % (name, r.returncode)
        print(f"bench: counter pass {name} done in {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    import pmc_summary
    kernels = pmc_summary.summarise(os.path.join(out, "run"))
    path = os.path.join(out, "pmc_summary.json")
    json.dump({"source": out, "kernels": kernels}, open(path, "w"), indent=1)
    keep = os.environ.get("HTM_BENCH_PMC_KEEP")  # a directory to keep a copy of the summary in
    if keep:
        os.makedirs(keep, exist_ok=True)
        shutil.copy(path, os.path.join(keep, "pmc_summary_%s.json" % (
            "learn_on" if learn_leg else "config5" if c5_leg else "config%d" % args.config)))
    return path, None


SP_LEARN_KERNEL = "sp_step_ord_kernel<true, true>"  # the split learning step's SP kernel (paged permanences)


def kernel_name(c3, c4, fused, split=False, ordered=False):
    """The dominant kernel's name as rocprofv3 reports it (without the
    argument list): the fused SP+TM kernel, frozen-TM or learning variant
    (split learning steps: the TM-only learning kernel; ordered frozen steps:
    the TM-only frozen kernel)."""
    if not fused:
        return "tm_step_kernel<false, true>" if not c3 else "tm_step_kernel<true, false>"
    if c3:
        return "htm_run_tmlearn_kernel" if split else "htm_run_kernel<true>"
    return "htm_run_frozen_tm_kernel" if ordered else "htm_run_frozen_kernel"


def split_traffic(path, split, tm_kernel):
    """HBM bytes per learning step from the counter passes: the TM kernel's,
    plus the SP kernel's for a split step; (bytes, TM kernel record)."""
    k = pmc_kernel(path, tm_kernel)
    if not k and tm_kernel == "htm_run_frozen_tm_kernel":  # (A/B builds without the TM-only kernel)
        k = pmc_kernel(path, "htm_run_frozen_kernel")
    if not k or "hbm_bytes_per_dispatch" not in k:
        return None, k
    b = k["hbm_bytes_per_dispatch"]
    if split:
        ks = pmc_kernel(path, SP_LEARN_KERNEL)
        if not ks or "hbm_bytes_per_dispatch" not in ks:
            return None, k
        b += ks["hbm_bytes_per_dispatch"]
    return int(b), k


def timed_replay(eng, vals, scores, a, steps, mode, chunk, gather, gathered, rank, world, device, marks=None):
    """Steps [a, a + steps) of every stream, timed between barrier +
    synchronize on both sides, the max over ranks returned (the bench
    contract).  mode "step": one eng.step per step (lockstep) and, with N>1
    ranks, each step's scores gathered to rank 0 (SLO alerting input);
    "run": eng.run chunks of `chunk` steps, one gather_rows per chunk,
    overlapped with the next chunk.  marks (lockstep only): a list that gets a
    HIP event recorded on the step stream before step 0 and after every 64th
    step (and the last) -- the per-window breakdown of a long region.  Returns
    (seconds, gathered)."""
    import torch
    import torch.distributed as dist
    import _pkg
    max_over_ranks = _pkg.load().fleet.max_over_ranks
    cuda = torch.cuda.is_available() and str(device).startswith("cuda")
    sync = torch.cuda.synchronize if cuda else (lambda: None)
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    handles = []
    if mode == "run":
        for c0_ in range(0, steps, chunk):
            m = min(chunk, steps - c0_)
            eng.run(vals[a + c0_:a + c0_ + m], out=scores[a + c0_:a + c0_ + m])
            if gather is not None:
                h, _ = gather.gather_rows(scores[a + c0_:a + c0_ + m],
                                          staging=gathered[:, c0_:c0_ + m] if rank == 0 else None)
                handles.append(h)
    else:
        if marks is not None and cuda:
            marks.append((0, torch.cuda.Event(enable_timing=True)))
            marks[-1][1].record()
        for k in range(steps):
            eng.step(vals[a + k], out=scores[a + k])
            if marks is not None and cuda and ((k + 1) % 64 == 0 or k + 1 == steps):
                marks.append((k + 1, torch.cuda.Event(enable_timing=True)))
                marks[-1][1].record()
            if gather is not None:
                h, _ = gather.gather(scores[a + k], staging=gathered[k] if rank == 0 else None)
                handles.append(h)
        # the deferred dutyCycle() writes of these steps are part of the work
        # (HTM_OPT_DEFER_DUTY): completed inside the timed region
        if hasattr(eng, "flush"):
            eng.flush()
    for h in handles:
        h.wait()
    sync()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    return max_over_ranks(dt, device if cuda else None), gathered


if __name__ == "__main__":
    main()
