# round 2: paged SP permanences -- parity tests, then config 3 at 65,536 streams
set -o pipefail
OUT=gpurun_out/r02p
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_sp_paged.py tests/test_abi.py -x -v --timeout 300 --timeout-method thread > $OUT/paged_tests.log 2>&1 || { tail -40 $OUT/paged_tests.log; exit 1; }
tail -3 $OUT/paged_tests.log
START=$(date +%s)
timeout -k 10 600 python -u bench.py --config 3 --no-pmc > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail -30 $OUT/bench_c3.err; exit 1; }
echo "bench wall $(( $(date +%s) - START )) s"
cat $OUT/bench_c3.json
