set -o pipefail
OUT=gpurun_out/r02k
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_fleet_mode.py tests/test_configs_gpu.py tests/test_slo_harness.py -x -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
AB_ROUNDS=3 timeout -k 10 900 python -u tools/ab_libs.py main prev > $OUT/ab_libs.txt 2> $OUT/ab_libs.err || { tail -20 $OUT/ab_libs.err; exit 1; }
tail -1 $OUT/ab_libs.txt
