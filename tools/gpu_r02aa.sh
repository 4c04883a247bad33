# A/B: one-round state load in lockstep steps
set -o pipefail
OUT=gpurun_out/r02aa
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_defer_duty.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
AB_ROUNDS=3 timeout -k 10 900 python -u tools/ab_libs.py main prev > $OUT/ab.txt 2> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
tail -1 $OUT/ab.txt
