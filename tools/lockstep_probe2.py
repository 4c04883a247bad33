"""Diagnostic: bench.py's exact preparation order vs variants (which input
tensor is allocated first, counters read, scores written into one tensor)."""
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
N, K = 1024, 128
d = np.load(os.path.join(ROOT, "tests", "golden", "model1_traces.npz"))
train = [c for c, m in zip(d["train_cpu"], d["train_mem"]) if not (np.isnan(c) or np.isnan(m))][:2184]
trace = d["test_cpu"].astype(np.float64)
mode = sys.argv[1]
if mode == "vals_first":
    vals = torch.tensor(bench.make_inputs(N, 0, N, 0, 256, trace), device="cuda:0")
eng, _, _, _ = bench.trained_engine(rt, N, 72 * 1024, 0, train)
eng.set_learning(False, False)
eng.set_run_chunk(128)
if mode != "vals_first":
    vals = torch.tensor(bench.make_inputs(N, 0, N, 0, 256, trace), device="cuda:0")
scores = torch.empty((256, N), dtype=torch.float32, device="cuda:0")
eng.run(vals[:64], out=scores[:64])
eng.run(vals[64:128], out=scores[64:128])
torch.cuda.synchronize()
if mode != "no_counters":
    eng.counters()
for rep in range(2):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(64):
        eng.step(vals[128 + rep * 64 + k], out=scores[128 + rep * 64 + k])
    eng.flush()
    torch.cuda.synchronize()
    print(mode, rep, round((time.perf_counter() - t0) / 64 * 1e3, 4), flush=True)
