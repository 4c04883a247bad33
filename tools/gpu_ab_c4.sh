# config 4 (fleet) launch chunk A/B with the auto work-queue unit, then config 5
set -o pipefail
OUT=gpurun_out/abc4
mkdir -p $OUT
run() { echo "== $1"; shift; timeout -k 10 400 "$@" > $OUT/cur.json 2> $OUT/cur.err || { tail -5 $OUT/cur.err; exit 1; }
        cp $OUT/cur.json $OUT/$(echo $1 | tr ' ' '_').json 2>/dev/null
        python -c "import json;d=json.load(open('$OUT/cur.json'));print(d['value'], d['roofline']['avg_launch_ms'], d['roofline']['steps_per_launch'], d.get('lockstep'))"; }
run "c4 chunk 64" python -u bench.py --config 4 --no-cpu && \
HTM_C4_MAX_CHUNK=256 run "c4 chunk 128" python -u bench.py --config 4 --no-cpu --chunk 128 --lockstep-steps 0 && \
run "c5" python -u bench.py --config 5 && cp $OUT/cur.json $OUT/bench_c5.json
