# work-queue + 3-workgroup occupancy: parity, then A/B of LDS budget / unit size
set -o pipefail
T=${AB_TAG:-q}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fleet_mode.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1; rc=$?; echo "parity: $(tail -1 gpurun_out/$T/tests.log)"; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u tools/stamps.py > gpurun_out/$T/stamps.json 2>gpurun_out/$T/stamps.err || exit 1
AB_TAG=$T AB_STAMPS=0 AB_STEPS=1200 AB_VARIANTS="${AB_VARIANTS:-fused=1 fused=1,budget=77824 fused=1,unit=256 fused=1,unit=64}" bash tools/ab_fin.sh
