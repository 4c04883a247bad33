# round 2: deferred dutyCycle writes -- parity tests, A/B on vs off, bench
set -o pipefail
OUT=gpurun_out/r02t
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_defer_duty.py -x -v --timeout 300 --timeout-method thread > $OUT/defer_tests.log 2>&1 || { tail -40 $OUT/defer_tests.log; exit 1; }
tail -3 $OUT/defer_tests.log
AB_ROUNDS=3 timeout -k 10 900 python -u tools/ab_libs.py main main@HTM_DEFER_DUTY=0 > $OUT/ab.txt 2> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
tail -1 $OUT/ab.txt
