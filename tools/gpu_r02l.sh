set -o pipefail
OUT=gpurun_out/r02l
mkdir -p $OUT
for v in main; do
  if [ $v = main ]; then unset HTM_AMD_LIB_VARIANT; else export HTM_AMD_LIB_VARIANT=$v; fi
  timeout -k 10 300 python -u -m pytest tests/test_fleet_mode.py tests/test_gpu_parity.py tests/test_configs_gpu.py tests/test_slo_harness.py -x -q --timeout 200 --timeout-method thread > $OUT/fleet_$v.log 2>&1; echo "$v rc=$?"; tail -1 $OUT/fleet_$v.log
done
AB_ROUNDS=3 timeout -k 10 900 python -u tools/ab_libs.py main prev > $OUT/ab_libs.txt 2> $OUT/ab_libs.err || { tail -20 $OUT/ab_libs.err; exit 1; }
tail -1 $OUT/ab_libs.txt
