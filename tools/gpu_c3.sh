set -o pipefail
OUT=gpurun_out/c3
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --config 3 --streams 4096 --steps 48 --warmup 16 > $OUT/bench_small.json 2> $OUT/bench_small.err || { tail -20 $OUT/bench_small.err; exit 1; }
cat $OUT/bench_small.json
timeout -k 10 600 python -u bench.py --config 3 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
