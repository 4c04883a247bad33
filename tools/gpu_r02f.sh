set -o pipefail
OUT=gpurun_out/r02f
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_configs_gpu.py tests/test_network_facade.py -m gpu -x -v --timeout 400 --timeout-method thread --durations=0 > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed|s call" $OUT/tests.log | tail -20
AB_MODES=0:0:0:0:1,0:0:0:0:0 timeout -k 10 600 python -u tools/ab_assist.py > $OUT/ab_pid.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
cat $OUT/ab_pid.json
