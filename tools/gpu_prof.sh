# Profile of the bench command: rocprofv3 kernel stats, PMC passes (L2
# memory-side requests by size, FETCH_SIZE, WRITE_SIZE) over the bench and
# over the counter-calibration microbench, the summary, then the bench line
# whose roofline.traffic comes from THIS run's passes.
# usage: bash tools/gpu_prof.sh <out dir> [bench args...]
set -o pipefail
OUT=${1:-gpurun_out/prof}
shift || true
BARGS=${@:-"--steps 512 --warmup 16 --other-steps 0 --no-cpu"}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
RD="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
WR="WRITE_SIZE TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
# calibration microbench (known bytes per dispatch)
timeout -k 10 120 ./tools/fetch_calib > $OUT/calib_bytes.json 2> $OUT/calib.err || { cat $OUT/calib.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $RD --output-format csv -d $OUT/calib/pmc_rd -o run -- ./tools/fetch_calib > /dev/null 2>> $OUT/calib.err || { tail -5 $OUT/calib.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/calib/pmc_fetch -o run -- ./tools/fetch_calib > /dev/null 2>> $OUT/calib.err || { tail -5 $OUT/calib.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $WR --output-format csv -d $OUT/calib/pmc_wr -o run -- ./tools/fetch_calib > /dev/null 2>> $OUT/calib.err || { tail -5 $OUT/calib.err; exit 1; }
# the bench: kernel stats, then the three counter passes (--no-profile: no HIP events;
# --no-pmc: the profiled runs do not start bench.py's own counter passes)
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/run/prof -o run -- python3 bench.py $BARGS --no-pmc > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { tail -5 $OUT/bench_prof.err; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc $RD --output-format csv -d $OUT/run/pmc_rd -o run -- python3 bench.py $BARGS --no-profile --no-pmc > /dev/null 2> $OUT/rd.err || { tail -5 $OUT/rd.err; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/run/pmc_fetch -o run -- python3 bench.py $BARGS --no-profile --no-pmc > /dev/null 2> $OUT/fetch.err || { tail -5 $OUT/fetch.err; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc $WR --output-format csv -d $OUT/run/pmc_wr -o run -- python3 bench.py $BARGS --no-profile --no-pmc > /dev/null 2> $OUT/wr.err || { tail -5 $OUT/wr.err; exit 1; }
python3 tools/pmc_summary.py $OUT/run $OUT --calib $OUT/calib $OUT/calib_bytes.json > $OUT/pmc_summary.txt 2>&1 || { cat $OUT/pmc_summary.txt; exit 1; }
cat $OUT/pmc_summary.txt
timeout -k 10 400 python3 bench.py $BARGS --pmc-summary $OUT/pmc_summary.json > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
