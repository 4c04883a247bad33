#!/bin/bash
# One GPU session: parity suite, bench, rocprof kernel stats, PMC HBM passes,
# and (STAMPS=1) the diagnostic per-phase stamps of the TM kernel.
# Usage (from the repo root on the GPU box): bash tools/gpu_round.sh TAG [STEPS]
set -o pipefail
TAG=${1:-r01}
STEPS=${2:-1024}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() { echo "== $1 ($(date +%T))"; }
step "parity tests" && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 && \
tail -3 $OUT/gpu_tests.log && \
{ [ "${STAMPS:-0}" != "1" ] || { step "stamps" && timeout -k 10 300 python -u tools/stamps.py > $OUT/stamps.json 2> $OUT/stamps.err && cat $OUT/stamps.json; }; } && \
step "bench" && \
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err && cat $OUT/bench.json && \
{ [ "${PROF:-1}" != "1" ] || { step "rocprof kernel stats" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps $STEPS --warmup 0 --lockstep-steps 0 --no-cpu > $OUT/prof_bench.json 2> $OUT/prof.err && \
step "pmc FETCH_SIZE" && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --mode run --steps 256 --chunk 256 --warmup 0 --lockstep-steps 0 --no-cpu --no-profile > $OUT/pmc_fetch.log 2>&1 && \
step "pmc WRITE_SIZE" && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --mode run --steps 256 --chunk 256 --warmup 0 --lockstep-steps 0 --no-cpu --no-profile > $OUT/pmc_write.log 2>&1; }; } && \
step "done"
