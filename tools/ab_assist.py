"""A/B of engine variants on the config-2 lockstep workload: one engine per
setting fed the same inputs, timed in interleaved rounds in one process
(cdna_hip_programming.md §5.4 rule 24).  A setting "a:t:f:g" = HTM_OPT_BT_ASSIST
a, HTM_OPT_BT_TAIL t, HTM_FX_MODE f, HTM_FX_GRAN g, HTM_FX_PID p (the last
three are read when the engine is created; g = 0 keeps the default, p = 0
drops the pid lists)."""
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
N = int(os.environ.get("AB_STREAMS", "1024"))
R, K = int(os.environ.get("AB_ROUNDS", "4")), int(os.environ.get("AB_STEPS", "64"))
modes = os.environ.get("AB_MODES", "0:0:0,0:0:1,0:0:2,0:0:3").split(",")
d = np.load(os.path.join(ROOT, "tests", "golden", "model1_traces.npz"))
train = [c for c, m in zip(d["train_cpu"], d["train_mem"]) if not (np.isnan(c) or np.isnan(m))][:2184]
trace = d["test_cpu"].astype(np.float64)
base, _, _, _ = bench.trained_engine(rt, 1, 72 * 1024, 0, train)
engs = {}
for m in modes:
    a_, t_, f_, g_, p_ = (int(x) for x in (m + ":0:0:0:1").split(":")[:5])
    os.environ["HTM_FX_PID"] = str(p_)
    os.environ["HTM_FX_MODE"] = str(f_)
    if g_:
        os.environ["HTM_FX_GRAN"] = str(g_)
    else:
        os.environ.pop("HTM_FX_GRAN", None)
    e = rt.HTMEngine(N, seg_capacity=72 * 1024)
    for region in rt._lib.ST:
        e.import_state(region, base.export_state(region, 0, 1), s0=0)
    e.replicate(0)
    e.set_learning(False, False)
    e.set_option(rt._lib.OPT_BT_ASSIST, a_)
    e.set_option(rt._lib.OPT_BT_TAIL, t_)
    engs[m] = e
vals = torch.tensor(bench.make_inputs(N, 0, N, 0, 16 + R * K, trace), device="cuda")
for m in modes:
    for k in range(16):
        engs[m].step(vals[k])
torch.cuda.synchronize()
times = {m: [] for m in modes}
outs = {m: [] for m in modes}
for r in range(R):
    for m in modes:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        o = [engs[m].step(vals[16 + r * K + k]) for k in range(K)]
        torch.cuda.synchronize()
        times[m].append((time.perf_counter() - t0) / K * 1e3)
        outs[m].append(torch.stack(o).cpu().numpy())
same = all(np.array_equal(np.concatenate(outs[m]), np.concatenate(outs[modes[0]])) for m in modes)
print(json.dumps({"streams": N, "steps_per_round": K, "rounds": R, "identical_scores": bool(same),
                  "ms_per_step": {m: [round(x, 4) for x in times[m]] for m in modes},
                  "median_ms": {m: round(float(np.median(times[m])), 4) for m in modes}}))
