# round 2: full GPU suite + smoke + default bench at HEAD
set -o pipefail
OUT=gpurun_out/r02s
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
START=$(date +%s)
timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - START )) s"
cat $OUT/bench.json
