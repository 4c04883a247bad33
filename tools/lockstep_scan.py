"""Lockstep launch time vs stream count on the config-2 workload: is a
lockstep step bound by the slowest stream's critical path (time flat in N
while all streams are resident) or by total work (time grows with N)?"""
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
NS = [int(x) for x in os.environ.get("SCAN_STREAMS", "64,256,512,768,1024,1536,2048,3072").split(",")]
K = int(os.environ.get("SCAN_STEPS", "64"))
d = np.load(os.path.join(ROOT, "tests", "golden", "model1_traces.npz"))
train = [c for c, m in zip(d["train_cpu"], d["train_mem"]) if not (np.isnan(c) or np.isnan(m))][:2184]
trace = d["test_cpu"].astype(np.float64)
base, _, _, _ = bench.trained_engine(rt, 1, 72 * 1024, 0, train)
out = {}
for n in NS:
    e = rt.HTMEngine(n, seg_capacity=72 * 1024)
    for region in rt._lib.ST:
        e.import_state(region, base.export_state(region, 0, 1), s0=0)
    e.replicate(0)
    e.set_learning(False, False)
    vals = torch.tensor(bench.make_inputs(n, 0, n, 0, 16 + 2 * K, trace), device="cuda")
    for k in range(16):
        e.step(vals[k])
    torch.cuda.synchronize()
    t = []
    for r in range(2):
        t0 = time.perf_counter()
        for k in range(K):
            e.step(vals[16 + r * K + k])
        torch.cuda.synchronize()
        t.append((time.perf_counter() - t0) / K * 1e3)
    out[n] = {"ms_per_step": round(min(t), 4), "stream_steps_per_s": round(n / min(t) * 1e3)}
    print(n, out[n], flush=True)
    del e, vals
    torch.cuda.empty_cache()
print(json.dumps(out))
