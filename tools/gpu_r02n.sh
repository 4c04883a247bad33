set -o pipefail
OUT=gpurun_out/r02n
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
AB_ROUNDS=3 timeout -k 10 900 python -u tools/ab_libs.py main prev > $OUT/ab_libs.txt 2> $OUT/ab_libs.err || { tail -20 $OUT/ab_libs.err; exit 1; }
tail -1 $OUT/ab_libs.txt
START=$(date +%s)
timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - START )) s"
cat $OUT/bench.json
