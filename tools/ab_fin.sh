# A/B of engine knobs on the config-2 workload (stamps + bench per variant)
set -o pipefail
OUT=gpurun_out/${AB_TAG:-ab}
mkdir -p $OUT
for v in ${AB_VARIANTS:-"fused=1"}; do
  export HTM_FUSED=$(echo $v | sed -n 's/.*fused=\([01]\).*/\1/p')
  export HTM_TM_FIN=$(echo $v | sed -n 's/.*fin=\([a-z]*\).*/\1/p')
  b=$(echo $v | sed -n 's/.*budget=\([0-9]*\).*/\1/p'); if [ -n "$b" ]; then export HTM_TM_LDS_BUDGET=$b; else unset HTM_TM_LDS_BUDGET; fi
  un=$(echo $v | sed -n 's/.*unit=\([0-9]*\).*/\1/p'); if [ -n "$un" ]; then export HTM_RUN_UNIT=$un; else unset HTM_RUN_UNIT; fi
  l=$(echo $v | sed -n 's/.*lib=\([a-z0-9]*\).*/\1/p'); if [ -n "$l" ]; then export HTM_AMD_LIB=libhtm_amd_$l.so; else unset HTM_AMD_LIB; fi
  tag=$(echo $v | tr ',=' '__')
  if [ "${AB_STAMPS:-1}" = "1" ]; then
    timeout -k 10 300 python -u tools/stamps.py > $OUT/stamps_$tag.json 2> $OUT/stamps_$tag.err || exit 1
  fi
  timeout -k 10 300 python -u bench.py --no-cpu --steps ${AB_STEPS:-600} ${AB_BENCH_ARGS} > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || exit 1
  echo "$v: $(cat $OUT/bench_$tag.json | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["roofline"]["avg_launch_ms"] if d["roofline"] else None)')"
done
