# A/B of engine variants on config 2 (parity of each variant first)
set -o pipefail
mkdir -p gpurun_out/ab2
for v in ${LIBS:-np}; do
  HTM_AMD_LIB=libhtm_amd_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab2/tests_$v.log 2>&1; rc=$?; echo "$v parity: $(tail -1 gpurun_out/ab2/tests_$v.log)"; [ $rc = 0 ] || exit $rc
done
AB_TAG=ab2 AB_STAMPS=0 AB_STEPS=1200 AB_VARIANTS="$AB" bash tools/ab_fin.sh
