# bench HIP-event launch time vs rocprof kernel stats with kernel-only flush completion
set -o pipefail
OUT=gpurun_out/r02x
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_defer_duty.py -x -q --timeout 300 --timeout-method thread > $OUT/defer_tests.log 2>&1 || { tail -40 $OUT/defer_tests.log; exit 1; }
tail -2 $OUT/defer_tests.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 512 --warmup 16 --other-steps 0 --no-cpu --no-pmc > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { tail -5 $OUT/bench_prof.err; exit 1; }
grep -h "frozen_kernel\|flush" $OUT/prof/run_kernel_stats.csv | cut -c1-170
python3 -c "import json; d=json.load(open('$OUT/bench_prof.json')); print(d['ms_per_step'], d['roofline']['avg_launch_ms'])"
