"""Diagnostic: lockstep ms/step of the config-2 engine after different
preparations (lockstep warm-up vs an htm_run chunk, profiling on/off,
counters read), to locate a slowdown seen between bench.py and ab_libs.py."""
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
vals = torch.tensor(bench.make_inputs(N, 0, N, 0, 4000, trace), device="cuda")


def timed(eng, a, label):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        eng.step(vals[a + k])
    eng.flush()
    torch.cuda.synchronize()
    print(label, round((time.perf_counter() - t0) / K * 1e3, 4), flush=True)


def fresh():
    eng, _, _, _ = bench.trained_engine(rt, N, 72 * 1024, 0, train)
    eng.set_learning(False, False)
    return eng


eng = fresh()
for k in range(16):
    eng.step(vals[k])
timed(eng, 16, "lockstep-warm t16")
timed(eng, 144, "lockstep-warm t144")
eng.close()
eng = fresh()
eng.run(vals[:128])
timed(eng, 128, "run-warm t128")
timed(eng, 256, "run-warm t256")
eng.set_run_chunk(128)
eng.run(vals[384:512])
timed(eng, 512, "run-warm again t512")
eng.close()
eng = fresh()
eng.set_run_chunk(128)
eng.run(vals[:128])
for k in range(16):
    eng.step(vals[128 + k])
timed(eng, 144, "run-warm + 16 lockstep t144")
