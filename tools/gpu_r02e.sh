set -o pipefail
OUT=gpurun_out/r02e
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_multilevel_gpu.py -x -v --timeout 300 --timeout-method thread > $OUT/ml_tests.log 2>&1 || { tail -40 $OUT/ml_tests.log; exit 1; }
tail -3 $OUT/ml_tests.log
AB_MODES=0:0:0:0,0:0:4:0,0:0:0:1024,0:0:4:1024 timeout -k 10 600 python -u tools/ab_assist.py > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
cat $OUT/ab.json
