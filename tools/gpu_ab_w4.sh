# frozen run kernel: 3 workgroups/CU (52 KiB LDS each, default) vs 4 (HTM_RUN_WAVES=4, ~38 KiB)
set -o pipefail
OUT=gpurun_out/abw4
mkdir -p $OUT
run() { echo "== $1"; shift; timeout -k 10 240 "$@" > $OUT/cur.json 2> $OUT/cur.err || { tail -5 $OUT/cur.err; exit 1; }
        python -c "import json;d=json.load(open('$OUT/cur.json'));print(d['value'], d['roofline']['avg_launch_ms'], d['lockstep'])" | tee -a $OUT/ab.txt; }
B="python -u bench.py --no-cpu --lockstep-steps 128"
run "w3 52K (default)" $B && \
HTM_AMD_LIB=libhtm_amd_w4.so HTM_TM_LDS_BUDGET=38912 run "w4 38K" $B && \
HTM_AMD_LIB=libhtm_amd_w4.so HTM_TM_LDS_BUDGET=36864 run "w4 36K" $B
