"""Diagnostic: config-2 lockstep launch times, fused (one SP+TM kernel) vs
unfused (SP kernel, then TM kernel), with HIP-event kernel times."""
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
N, K = 1024, 256
d = np.load(os.path.join(ROOT, "tests", "golden", "model1_traces.npz"))
train = [c for c, m in zip(d["train_cpu"], d["train_mem"]) if not (np.isnan(c) or np.isnan(m))][:2184]
trace = d["test_cpu"].astype(np.float64)
eng, _, _, _ = bench.trained_engine(rt, N, 72 * 1024, 0, train)
eng.set_learning(False, False)
vals = torch.tensor(bench.make_inputs(N, 0, N, 0, 64 + 4 * K, trace), device="cuda")
for k in range(64):
    eng.step(vals[k])
out = {}
for r, fused in enumerate((True, False, True, False)):
    eng.use_fused(fused)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        eng.step(vals[64 + r * K + k])
    eng.flush()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / K * 1e3
    eng.profile(True, 4)
    for k in range(32):
        eng.step(vals[64 + r * K + k])
    p = eng.profile_read()
    eng.profile(False)
    out.setdefault("fused" if fused else "unfused", []).append(
        {"wall_ms": round(wall, 4), "sp_ms": round(p["sp_ms"] / max(1, p["launches"]), 4),
         "tm_ms": round(p["tm_ms"] / max(1, p["launches"]), 4)})
print(json.dumps(out))
