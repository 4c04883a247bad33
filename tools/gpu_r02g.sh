set -o pipefail
OUT=gpurun_out/r02g
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_fleet_mode.py tests/test_configs_gpu.py -x -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
AB_MODES=0:0:0:0:1,0:0:0:0:0 timeout -k 10 600 python -u tools/ab_assist.py > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
cat $OUT/ab.json
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
