"""Diagnostic: where a short timed region's excess over the long line goes.

The driver's bench command times 20 lockstep steps (--steps 20 --warmup 5)
and ends the region with htm_flush; the long line times 2,324.  This builds
bench.py's config-2 engine (1,024 replicas of the GPU-trained Model-1 state,
learning off), conditions and warms it up the bench's way, then times REGIONS
regions of STEPS steps each with a HIP event after every step and after the
final flush (events on the step stream), and prints per-step and flush times
(median over regions) beside the wall-clock region time.  Not a bench line."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkg  # noqa: E402
import bench  # noqa: E402

rt = _pkg.load()
STEPS = int(os.environ.get("SH_STEPS", "20"))
WARM = int(os.environ.get("SH_WARMUP", "5"))
COND = int(os.environ.get("SH_CONDITION", "64"))
REGIONS = int(os.environ.get("SH_REGIONS", "5"))
N = 1024
d = np.load(os.path.join(ROOT, "tests", "golden", "model1_traces.npz"))
train = [c for c, m in zip(d["train_cpu"], d["train_mem"]) if not (np.isnan(c) or np.isnan(m))][:2184]
trace = d["test_cpu"].astype(np.float64)
eng, _, _, _ = bench.trained_engine(rt, N, 72 * 1024, 0, train)
eng.set_learning(False, False)
if os.environ.get("SH_FLUSH_EVERY"):
    eng.flush_every(int(os.environ["SH_FLUSH_EVERY"]))
if os.environ.get("SH_FLUSH_MODE"):
    eng.flush_mode(int(os.environ["SH_FLUSH_MODE"]))
T = COND + WARM + REGIONS * STEPS
vals = torch.tensor(bench.make_inputs(N, 0, N, 0, T, trace), device="cuda")
scores = torch.empty((T, N), dtype=torch.float32, device="cuda")
for k in range(COND + WARM):
    eng.step(vals[k], out=scores[k])
torch.cuda.synchronize()
per_step, flush, wall = [], [], []
k0 = COND + WARM
for r in range(REGIONS):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(STEPS + 2)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev[0].record()
    for j in range(STEPS):
        eng.step(vals[k0 + j], out=scores[k0 + j])
        ev[j + 1].record()
    eng.flush()
    ev[STEPS + 1].record()
    torch.cuda.synchronize()
    wall.append((time.perf_counter() - t0) * 1e3)
    per_step.append([ev[j].elapsed_time(ev[j + 1]) for j in range(STEPS)])
    flush.append(ev[STEPS].elapsed_time(ev[STEPS + 1]))
    k0 += STEPS
ps = np.median(np.array(per_step), axis=0)
out = {"flush_mode": os.environ.get("SH_FLUSH_MODE", "default"), "flush_every": os.environ.get("SH_FLUSH_EVERY", "default"), "steps": STEPS, "warmup": WARM, "condition": COND, "regions": REGIONS,
       "wall_ms_per_step_median": round(float(np.median(wall)) / STEPS, 4),
       "wall_ms_per_step_each_region": [round(w / STEPS, 4) for w in wall],
       "step_ms_median_by_position": [round(float(x), 4) for x in ps],
       "final_flush_ms_median": round(float(np.median(flush)), 4),
       "steps_only_ms_per_step": round(float(ps.sum()) / STEPS, 4)}
print(json.dumps(out, indent=1))
