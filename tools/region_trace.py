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
    """Per region (from a marker kernel to the last flush-done kernel before
    the next marker): the GPU span, when the first step's SP kernel starts
    after the marker, the TM launches, the flushes beside the steps and the
    final flush after the last TM launch."""
    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]) for r in rows)
    info = json.load(open(js)) if js else None
    marks = [i for i, k in enumerate(ks) if "elementwise" in k[2]]
    res = []
    for j, m in enumerate(marks):
        seg = ks[m:marks[j + 1] if j + 1 < len(marks) else len(ks)]
        done = [i for i, k in enumerate(seg) if "flush_done" in k[2]]
        if not done:
            continue
        seg = seg[:done[-1] + 1]
        t0 = seg[0][0]
        tm = [k for k in seg if "frozen_tm" in k[2] or k[2] == "htm_run_frozen_kernel"]
        sp = [k for k in seg if "sp_step" in k[2]]
        if not tm or not sp:
            continue
        fl = [k for k in seg if k[2] == "tm_fx_flush_kernel"]
        fin = [k for k in seg if k[2].startswith("tm_fx_") and k[0] >= tm[-1][1]]
        beside = [k for k in fl if k[0] < tm[-1][1]]
        tmd = [(e - s) / 1e3 for s, e, _ in tm]
        over = [(e - s) / 1e3 for s, e, _ in tm if any(f[0] < e and f[1] > s for f in beside)]
        res.append({"gpu_span_us": round((seg[-1][1] - t0) / 1e3, 1),
                    "marker_to_first_sp_us": round((sp[0][0] - seg[0][1]) / 1e3, 1),
                    "tm_launches": len(tm), "tm_us_median": round(float(np.median(tmd)), 1),
                    "tm_us_beside_a_flush": [round(x, 1) for x in over],
                    "flushes_beside": [round((e - s) / 1e3, 1) for s, e, _ in beside],
                    "final_flush_us": round((seg[-1][1] - tm[-1][1]) / 1e3, 1),
                    "final_flush_kernels": [(k[2], round((k[1] - k[0]) / 1e3, 1)) for k in fin]})
    out = {"regions": res}
    if info:
        out["host_region_ms"] = info["region_ms"]
        n = min(len(res), len(info["region_ms"]))
        out["host_minus_gpu_us"] = [round(h * 1e3 - r["gpu_span_us"], 1)
                                    for h, r in zip(info["region_ms"][-n:], res[-n:])]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "analyse":
        analyse(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
    else:
        run()
