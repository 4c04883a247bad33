# round 2 validation at HEAD: full GPU suite, smoke, default bench, calibrated profile
set -o pipefail
OUT=gpurun_out/r02w
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
bash tools/gpu_prof.sh $OUT/prof --steps 512 --warmup 16 --other-steps 0 --no-cpu --no-pmc > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
tail -1 $OUT/prof.log
