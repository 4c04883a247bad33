"""Diagnostic (A/B build): the workgroup timeline of config-2 lockstep launches
-- when each stream's workgroup started and ended, its step bytes and final active cells
(s_memrealtime, 100 MHz), on which XCD.  usage:
HTM_AMD_LIB_VARIANT=ab HTM_WG_TRACE=1 python tools/wg_timeline.py  (make -C <pkg>/csrc ab)"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkg  # noqa: E402
import bench  # noqa: E402

rt = _pkg.load()
N = int(os.environ.get("AB_STREAMS", "1024"))
d = np.load(os.path.join(ROOT, "tests", "golden", "model1_traces.npz"))
train = [c for c, m in zip(d["train_cpu"], d["train_mem"]) if not (np.isnan(c) or np.isnan(m))][:2184]
trace = d["test_cpu"].astype(np.float64)
eng, _, _, _ = bench.trained_engine(rt, N, 72 * 1024, 0, train)
eng.set_learning(False, False)
vals = torch.tensor(bench.make_inputs(N, 0, N, 0, 80, trace), device="cuda")
for k in range(64):
    eng.step(vals[k])
torch.cuda.synchronize()
lib = eng._L
lib.htm_ab_wg_trace.restype = ctypes.c_int64
lib.htm_ab_wg_trace.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
cap = 2 * N + 4096
res = []
durs = []
for k in range(64, 80):
    eng.step(vals[k])
    buf = np.zeros((cap, 8), np.uint64)
    rows = lib.htm_ab_wg_trace(eng.h, buf.ctypes.data, cap)
    buf = buf[:rows]
    used = buf[:, 1] > 0
    b = buf[used].astype(np.int64)
    idx = np.nonzero(used)[0]
    t0 = b[:, 0].min()
    st, en = (b[:, 0] - t0) / 100.0, (b[:, 1] - t0) / 100.0  # us
    own = idx < N
    hel = ~own
    dd = np.full((3, N), np.nan)
    dd[0, idx[own]] = (en - st)[own]
    dd[1, idx[own]] = b[own, 4]
    dd[2, idx[own]] = b[own, 5]
    durs.append(dd)
    r = {"span_us": float(en.max()), "owners": int(own.sum()), "helpers": int(hel.sum()),
         "last_owner_start": float(st[own].max()), "last_owner_end": float(en[own].max()),
         "owner_dur_mean": float((en - st)[own].mean()), "owner_dur_p99": float(np.percentile((en - st)[own], 99))}
    if hel.any():
        r.update({"first_helper_start": float(st[hel].min()), "helper_end_max": float(en[hel].max()),
                  "helpers_started_before_last_owner": int((st[hel] < st[own].max()).sum())})
    # owners started in the second wave (after the first owner ended)
    first_end = en[own].min()
    r["second_wave_owners"] = int((st[own] > first_end).sum())
    r["second_wave_dur_mean"] = float((en - st)[own][st[own] > first_end].mean()) if r["second_wave_owners"] else 0.0
    r["ordered_sp_tm_jobs"] = [int((b[:, 6] >> 32).sum()), int((b[:, 6] & 0xFFFFFFFF).sum())]
    tt = b[:, 7]
    r["ordered_us_pick_sp_tm"] = [float(((tt >> 42) & 0x1FFFFF).sum() / 100.0), float(((tt >> 21) & 0x1FFFFF).sum() / 100.0),
                                  float((tt & 0x1FFFFF).sum() / 100.0)]
    xcc = b[:, 3] & 0xF
    r["owners_per_xcc"] = np.bincount(xcc[own], minlength=8).tolist()
    res.append(r)
keys = res[0].keys()
summ = {k: (float(np.median([x[k] for x in res])) if not isinstance(res[0][k], list) else res[-1][k]) for k in keys}
print(json.dumps({"median": summ, "launches": res[:4]}, indent=1))
if os.environ.get("WG_DUMP"):
    np.save(os.environ["WG_DUMP"], np.stack(durs))  # [launch][duration us, step bytes, active cells][stream]
