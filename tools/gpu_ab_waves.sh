# frozen run kernel: 3 workgroups/CU (52 KiB LDS each, default) vs 2 (76 KiB: bigger counter window, fewer passes)
set -o pipefail
OUT=gpurun_out/abw
mkdir -p $OUT
run() { echo "== $1"; shift; timeout -k 10 240 "$@" > $OUT/cur.json 2> $OUT/cur.err || { tail -5 $OUT/cur.err; exit 1; }
        python -c "import json;d=json.load(open('$OUT/cur.json'));print(d['value'], d['roofline']['avg_launch_ms'], d['lockstep'])"; }
B="python -u bench.py --no-cpu --lockstep-steps 128"
run "w3 52K (default)" $B && \
HTM_AMD_LIB=libhtm_amd_w2.so HTM_TM_LDS_BUDGET=77824 run "w2 76K" $B && \
HTM_AMD_LIB=libhtm_amd_w2.so HTM_TM_LDS_BUDGET=77824 run "w2 76K unit 32" $B --run-unit 32
