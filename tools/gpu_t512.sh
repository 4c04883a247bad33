# A/B of workgroup size / LDS budget variants (make variant VNAME=t128 VFLAGS=-DTM_NT=128)
set -o pipefail
V=${V:-t128}
mkdir -p gpurun_out/$V
HTM_AMD_LIB=libhtm_amd_$V.so HTM_TM_LDS_BUDGET=${BUDGET:-52000} timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fleet_mode.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$V/tests.log 2>&1; rc=$?; tail -3 gpurun_out/$V/tests.log; [ $rc = 0 ] || exit $rc
AB_TAG=$V AB_STAMPS=0 AB_STEPS=1200 AB_VARIANTS="$AB" bash tools/ab_fin.sh
