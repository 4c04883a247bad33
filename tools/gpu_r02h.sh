set -o pipefail
OUT=gpurun_out/r02h
mkdir -p $OUT
HTM_AMD_STAMPS=1 STAMP_STEPS=128 timeout -k 10 300 python -u tools/stamps.py > $OUT/stamps.json 2> $OUT/stamps.err || { tail -5 $OUT/stamps.err; exit 1; }
cat $OUT/stamps.json
