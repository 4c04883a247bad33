"""Diagnostic: where the TM kernel's cycles go, per stream-step, on the
config-2 workload (trained Model-1 state replicated into N streams, learning
off) or, STAMP_MODE=learn, config 3's (fresh streams, SP+TM learning on,
paged SP permanences: the bench's learn_on leg).  Needs the stamps build: make -C <pkg>/csrc stamps; run with
HTM_AMD_STAMPS=1."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["HTM_AMD_STAMPS"] = "1"
import _pkg  # noqa: E402
import bench  # noqa: E402

rt = _pkg.load()
MODE = os.environ.get("STAMP_MODE", "frozen")  # frozen: config 2; learn: config 3 (the bench's learn_on leg)
N = int(os.environ.get("STAMP_STREAMS", "65536" if MODE == "learn" else "1024"))
T = int(os.environ.get("STAMP_STEPS", "32" if MODE == "learn" else "200"))
W = int(os.environ.get("STAMP_WARMUP", "8" if MODE == "learn" else "16"))
d = np.load(os.path.join(ROOT, "tests", "golden", "model1_traces.npz"))
train = [c for c, m in zip(d["train_cpu"], d["train_mem"]) if not (np.isnan(c) or np.isnan(m))][:2184]
trace = d["test_cpu"].astype(np.float64)
if MODE == "learn":
    # config 3 / bench.bench_learn_on: fresh streams (seed 2045 + s), SP+TM learning on, paged SP
    cfg = rt.default_config(seg_capacity=10240, upd_capacity=512, seed_stride=1, sp_perm_rows=800)
    eng = rt.HTMEngine(N, config=cfg)
    eng.set_learning(True, True)
else:
    eng, _, hdr, _ = bench.trained_engine(rt, N, 72 * 1024, 0, train)
    eng.set_learning(False, False)
vals = torch.tensor(bench.make_inputs(N, 0, N, 0, T + W, trace), device="cuda")
for k in range(W):
    eng.step(vals[k])
torch.cuda.synchronize()
eng.debug_stamps()
eng.profile(True)
for k in range(W, W + T):
    eng.step(vals[k])
prof = eng.profile_read()
st = eng.debug_stamps()
steps = st["counts"]["steps"]
tot = sum(st["cycles"].values())
out = {"mode": MODE, "streams": N, "steps": T, "warmup": W, "tm_ms_per_launch": prof["tm_ms"] / prof["steps"],
       "sp_ms_per_launch": prof["sp_ms"] / prof["steps"],
       "cycles_per_stream_step": {k: round(v / steps, 1) for k, v in st["cycles"].items()},
       "total_cycles_per_stream_step": round(tot / steps, 1),
       "counts_per_stream_step": {k: round(v / steps, 3) for k, v in st["counts"].items()},
       "step_cycle_hist": st["step_cycle_hist"]}
tl = st["tail"]
ts = max(1, tl["counts"]["steps"])
out["tail"] = {"steps": tl["counts"]["steps"],
               "cycles_per_stream_step": {k: round(v / ts, 1) for k, v in tl["cycles"].items()},
               "total_cycles_per_stream_step": round(sum(tl["cycles"].values()) / ts, 1),
               "counts_per_stream_step": {k: round(v / ts, 3) for k, v in tl["counts"].items()}}
print(json.dumps(out, indent=1))
