"""Summarise a gpu_round.sh run into profiles/<tag>/: rocprof kernel stats,
PMC FETCH_SIZE / WRITE_SIZE per kernel, and the HBM traffic per stream-step
of the frozen inference kernel (the bench's dominant kernel).

FETCH_SIZE and WRITE_SIZE are in KB per dispatch.  Per MI355X_MICROARCH.md
(HBM section) gfx950's FETCH_SIZE reports half the bytes of 16-byte-per-lane
streaming reads, which is what the out-list block loads are, so it is
doubled ("fetch_corrected"); the kernel also issues 4/8-byte gathers, for
which the correction is uncalibrated -- the corrected figure is an upper
estimate, the raw one a lower."""
import csv
import json
import os
import shutil
import statistics
import sys

src, dst = sys.argv[1], sys.argv[2]
streams = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
# steps per dispatch of the frozen kernel: the PMC passes run one htm_run chunk
# of 256 steps (gpu_round.sh); 1 for per-step (--mode step) passes
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 256
os.makedirs(dst, exist_ok=True)
out = {"source": src, "streams": streams, "steps_per_dispatch": steps, "kernels": {}}
for name, cn in [("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")]:
    path = os.path.join(src, name, "run_counter_collection.csv")
    if not os.path.exists(path):
        continue
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == cn]
    per = {}
    for r in rows:
        per.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    for k, v in per.items():
        e = out["kernels"].setdefault(k, {})
        e[cn] = {"dispatches": len(v), "median_kb": statistics.median(v), "mean_kb": sum(v) / len(v)}
frozen = [k for k in out["kernels"] if "htm_run_frozen_kernel" in k or
          ("<false, true>" in k and ("htm_run_kernel" in k or "tm_step_kernel" in k))]
if frozen:
    e = out["kernels"][frozen[0]]
    f = e.get("FETCH_SIZE", {}).get("median_kb", 0.0) * 1024
    w = e.get("WRITE_SIZE", {}).get("median_kb", 0.0) * 1024
    out["frozen_kernel"] = frozen[0]
    u = streams * steps
    out["per_stream_step"] = {"fetch_raw": f / u, "fetch_corrected": 2 * f / u, "write": w / u,
                              "traffic": (2 * f + w) / u}
json.dump(out, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
ks = os.path.join(src, "prof", "run_kernel_stats.csv")
if os.path.exists(ks):
    shutil.copy(ks, os.path.join(dst, "kernel_stats.csv"))
for f in ["bench.json", "prof_bench.json", "stamps.json", "gpu_tests.log"]:
    if os.path.exists(os.path.join(src, f)):
        shutil.copy(os.path.join(src, f), os.path.join(dst, f))
print(json.dumps(out.get("per_stream_step"), indent=1))
