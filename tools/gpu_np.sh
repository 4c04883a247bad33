# A/B of the qualification variants (push-on-threshold vs non-returning count + dense sweep)
set -o pipefail
T=${AB_TAG:-np4}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests_push.log 2>&1; rc=$?; echo "push parity: $(tail -1 gpurun_out/$T/tests_push.log)"; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/stamps.py > gpurun_out/$T/stamps_push.json 2>/dev/null || exit 1
HTM_AMD_LIB=libhtm_amd_stnp.so timeout -k 10 300 python -u tools/stamps.py > gpurun_out/$T/stamps_np.json 2>/dev/null || exit 1
AB_TAG=$T AB_STAMPS=0 AB_STEPS=1200 AB_VARIANTS="fused=1 fused=1,lib=np fused=1,fin=buckets" bash tools/ab_fin.sh
