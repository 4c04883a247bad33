# one optimisation iteration: parity of the default build, stamps (push + np), A/B bench
set -o pipefail
T=${AB_TAG:-it}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1; rc=$?; echo "parity: $(tail -1 gpurun_out/$T/tests.log)"; [ $rc = 0 ] || exit $rc
if [ -n "$IT_NP_PARITY" ]; then
HTM_AMD_LIB=libhtm_amd_np.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests_np.log 2>&1; rc=$?; echo "np parity: $(tail -1 gpurun_out/$T/tests_np.log)"; [ $rc = 0 ] || exit $rc
fi
timeout -k 10 300 python -u tools/stamps.py > gpurun_out/$T/stamps_push.json 2>gpurun_out/$T/stamps_push.err || exit 1
HTM_AMD_LIB=libhtm_amd_stnp.so timeout -k 10 300 python -u tools/stamps.py > gpurun_out/$T/stamps_np.json 2>/dev/null || exit 1
AB_TAG=$T AB_STAMPS=0 AB_STEPS=1200 AB_VARIANTS="${AB_VARIANTS:-fused=1 fused=1,lib=np}" bash tools/ab_fin.sh
