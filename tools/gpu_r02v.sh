# round 2: deferral ring log with dedup -- tests, A/B vs previous, kernel stats
set -o pipefail
OUT=gpurun_out/r02v
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_defer_duty.py -x -q --timeout 300 --timeout-method thread > $OUT/defer_tests.log 2>&1 || { tail -40 $OUT/defer_tests.log; exit 1; }
tail -2 $OUT/defer_tests.log
AB_ROUNDS=3 timeout -k 10 900 python -u tools/ab_libs.py main prev main@HTM_DEFER_CAP=64@HTM_DEFER_FLUSH_EVERY=32 > $OUT/ab.txt 2> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
tail -1 $OUT/ab.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 512 --warmup 16 --other-steps 0 --no-cpu --no-pmc > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { tail -5 $OUT/bench_prof.err; exit 1; }
grep -h "frozen_kernel\|flush" $OUT/prof/run_kernel_stats.csv | cut -c1-160
