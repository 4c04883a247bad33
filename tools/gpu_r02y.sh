# round 2 final: calibrated profile of the lockstep bench, default bench, fleet (config 4) bench
set -o pipefail
OUT=gpurun_out/r02y
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_defer_duty.py tests/test_configs_gpu.py -x -q --timeout 600 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash tools/gpu_prof.sh $OUT/prof --steps 512 --warmup 16 --other-steps 0 --no-cpu --no-pmc > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
tail -1 $OUT/prof.log
timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 600 python -u bench.py --config 4 --no-pmc > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -20 $OUT/bench_c4.err; exit 1; }
cat $OUT/bench_c4.json
