"""Diagnostic: a kernel-trace view of short timed regions (the driver's
`--steps 20 --warmup 5` shape).  Builds bench.py's config-2 engine, conditions
and warms it up, flushes the deferred writes as bench.py's counters() call
does, then times REGIONS regions of STEPS lockstep steps exactly as
bench.timed_replay does (profile every 5th launch, htm_flush at the end,
synchronize on both sides).  Before each region a one-element marker kernel
(torch add) is launched, so the region's kernels can be found in a
`rocprofv3 --kernel-trace` of this script.  Prints the host-timed regions as
JSON; `python tools/region_trace.py analyse <kernel_trace.csv> <json>` then
lays the last regions out on the GPU clock.  Not a bench line."""
import csv
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run():
    import torch
    import _pkg
    import bench
    rt = _pkg.load()
    steps, regions, n = int(os.environ.get("RT_STEPS", "20")), int(os.environ.get("RT_REGIONS", "6")), 1024
    d = np.load(os.path.join(ROOT, "tests", "golden", "model1_traces.npz"))
    train = [c for c, m in zip(d["train_cpu"], d["train_mem"]) if not (np.isnan(c) or np.isnan(m))][:2184]
    trace = d["test_cpu"].astype(np.float64)
    eng, _, _, _ = bench.trained_engine(rt, n, 72 * 1024, 0, train)
    eng.set_learning(False, False)
    T = 64 + 5 + regions * steps
    vals = torch.tensor(bench.make_inputs(n, 0, n, 0, T, trace), device="cuda")
    scores = torch.empty((T, n), dtype=torch.float32, device="cuda")
    for k in range(69):
        eng.step(vals[k], out=scores[k])
    torch.cuda.synchronize()
    eng.counters()
    marker = torch.zeros(1, device="cuda")
    out = []
    a = 69
    for r in range(regions):
        eng.profile(True, every=5)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        marker.add_(1.0)
        for k in range(steps):
            eng.step(vals[a + k], out=scores[a + k])
        eng.flush()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        eng.profile_read()
        eng.profile(False)
        out.append(round(dt * 1e3, 4))
        a += steps
    print(json.dumps({"steps": steps, "region_ms": out, "ms_per_step": [round(x / steps, 4) for x in out]}))


def analyse(path, js):
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    info = json.load(open(js)) if js else None
    marks = [i for i, k in enumerate(ks) if "elementwise" in k[2] or "vectorized" in k[2]]
    res = []
    for j, m in enumerate(marks):
        end = marks[j + 1] if j + 1 < len(marks) else len(ks)
        seg = ks[m:end]
        # the region's kernels: up to the last flush-done kernel before the next marker
        last = max(i for i, k in enumerate(seg) if "flush_done" in k[2]) if any("flush_done" in k[2] for k in seg) else len(seg) - 1
        seg = seg[:last + 1]
        t0 = seg[0][0]
        tm = [k for k in seg if "frozen_tm" in k[2] or "htm_run_frozen_kernel" in k[2]]
        busy = 0
        cur_s, cur_e = None, None
        for s, e, _ in seg:  # union of kernel intervals (the flush stream overlaps the steps)
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        first_step = next(k for k in seg if "sp_step" in k[2])
        fin = [k for k in seg if "fx_" in k[2] and k[0] >= tm[-1][1]]
        res.append({"gpu_span_us": round((seg[-1][1] - t0) / 1e3, 1), "gpu_busy_us": round(busy / 1e3, 1),
                    "marker_to_first_step_us": round((first_step[0] - seg[0][1]) / 1e3, 1),
                    "tm_launch_us_mean": round(float(np.mean([(e - s) / 1e3 for s, e, _ in tm])), 1),
                    "last_tm_end_to_region_end_us": round((seg[-1][1] - tm[-1][1]) / 1e3, 1),
                    "after_last_step": [(k[2].split("(")[0][:40], round((k[0] - tm[-1][1]) / 1e3, 1),
                                         round((k[1] - k[0]) / 1e3, 1)) for k in fin]})
    out = {"regions": res}
    if info:
        out["host_region_ms"] = info["region_ms"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "analyse":
        analyse(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
    else:
        run()
