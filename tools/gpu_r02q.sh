# round 2: config tests (incl. config 3 at 65,536 paged streams) + config-3 bench with counter passes
set -o pipefail
OUT=gpurun_out/r02q
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_configs_gpu.py tests/test_sp_paged.py -x -v --timeout 600 --timeout-method thread > $OUT/config_tests.log 2>&1 || { tail -40 $OUT/config_tests.log; exit 1; }
tail -3 $OUT/config_tests.log
START=$(date +%s)
timeout -k 10 900 python -u bench.py --config 3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail -30 $OUT/bench_c3.err; exit 1; }
echo "bench wall $(( $(date +%s) - START )) s"
cat $OUT/bench_c3.json
