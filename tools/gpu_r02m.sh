set -o pipefail
OUT=gpurun_out/r02m
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1; echo "rc=$?"
grep -E "PASSED|FAILED" $OUT/parity.log | head -30
grep -E "^E " $OUT/parity.log | head -20
