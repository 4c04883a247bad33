# A/B of the fused-launch chunk and work-queue unit (config 2), config 3 with the chosen unit
set -o pipefail
OUT=gpurun_out/abc
mkdir -p $OUT
run() { echo "== $1"; shift; timeout -k 10 240 "$@" > $OUT/cur.json 2> $OUT/cur.err || { tail -5 $OUT/cur.err; exit 1; }
        python -c "import json;d=json.load(open('$OUT/cur.json'));print(d['value'], d['roofline']['avg_launch_ms'], d['roofline']['steps_per_launch'])"; }
B="python -u bench.py --no-cpu --lockstep-steps 0"
run "chunk 2324 unit 64" $B --chunk 2324 --run-unit 64 && \
run "chunk 2324 unit 96" $B --chunk 2324 --run-unit 96 && \
run "chunk 2324 unit 48 rep" $B --chunk 2324 --run-unit 48 && \
run "c3 unit 16" python -u bench.py --config 3 --streams 8192 --steps 96 --warmup 8 && \
run "c3 unit 48" python -u bench.py --config 3 --streams 8192 --steps 96 --warmup 8 --run-unit 48
