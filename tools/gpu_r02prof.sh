# lockstep profile: counter list, stamps, kernel stats, FETCH/WRITE passes
set -o pipefail
OUT=gpurun_out/r02prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --list-avail > $OUT/counters.txt 2>&1 || echo "list-avail rc=$?"
HTM_AMD_STAMPS=1 STAMP_STEPS=128 timeout -k 10 300 python -u tools/stamps.py > $OUT/stamps.json 2> $OUT/stamps.err || { tail -5 $OUT/stamps.err; exit 1; }
B="bench.py --steps 256 --warmup 16 --other-steps 0 --no-cpu"
BP="$B --no-profile"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $B > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { tail -5 $OUT/bench_prof.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $BP > $OUT/bench_fetch.json 2> $OUT/fetch.err || { tail -5 $OUT/fetch.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $BP > $OUT/bench_write.json 2> $OUT/write.err || { tail -5 $OUT/write.err; exit 1; }
ls -R $OUT | head -40
