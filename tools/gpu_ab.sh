set -o pipefail
mkdir -p gpurun_out/r01g
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r01g/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r01g/gpu_tests.log; [ $rc = 0 ] || exit $rc
AB_TAG=r01g AB_VARIANTS="fused=1 fused=0" bash tools/ab_fin.sh || exit 1
AB_TAG=r01g_run AB_STAMPS=0 AB_VARIANTS="fused=1" AB_BENCH_ARGS="--mode run" bash tools/ab_fin.sh
