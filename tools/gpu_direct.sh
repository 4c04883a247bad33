# parity suite + config 2 and config 4 benches (lockstep figures) after the direct-dispatch change
set -o pipefail
OUT=gpurun_out/direct
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
tail -3 $OUT/gpu_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('c2', d['value'], d['lockstep'])"
timeout -k 10 400 python -u bench.py --config 4 --no-cpu > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail $OUT/bench_c4.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_c4.json'));print('c4', d['value'], d['lockstep'])"
