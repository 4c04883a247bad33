#!/bin/bash
# Round-end measurements on one GPU box: the default bench line (2,324-step
# region, its own counter passes), a rocprofv3 kernel trace + stats of the
# driver's command (20 steps, no counter passes inside the profiler), and the
# two fleet shapes (config 4) with their counter passes.  Each step has its own
# time limit; the first failure ends the call.
# usage: OUT=gpurun_out/r06_endB bash tools/gpu_round_end.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/round_end}
mkdir -p "$OUT"
HTM_BENCH_PMC_KEEP=$OUT timeout -k 10 420 python bench.py > "$OUT/driver.log" 2>&1 || exit 1
echo "driver.log done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-pmc --no-cpu > "$OUT/driver20_prof.log" 2>&1 || exit 1
echo "kernel trace done"
HTM_BENCH_PMC_KEEP=$OUT/c4 timeout -k 10 300 python bench.py --config 4 --no-cpu > "$OUT/c4.log" 2>&1 || exit 1
echo "c4 done"
HTM_BENCH_PMC_KEEP=$OUT/c4y timeout -k 10 300 python bench.py --config 4 --shape yaml --no-cpu > "$OUT/c4y.log" 2>&1 || exit 1
echo "c4y done"
