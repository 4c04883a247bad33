# parity suite + config-2 bench (+ optional config 3) -- quick iteration loop
set -o pipefail
OUT=gpurun_out/${TAG:-quick}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
tail -3 $OUT/gpu_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
if [ "${C3:-0}" = "1" ]; then
  timeout -k 10 600 python -u bench.py --config 3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail $OUT/bench_c3.err; exit 1; }
  cat $OUT/bench_c3.json
fi
