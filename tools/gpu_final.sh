# smoke() + config-3 bench with the current kernels
set -o pipefail
OUT=gpurun_out/final
mkdir -p $OUT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 700 python -u bench.py --config 3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail -5 $OUT/bench_c3.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_c3.json'));print('c3', d['value'], d['roofline']['avg_launch_ms'], d['config']['segments_after'])"
