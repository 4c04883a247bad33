# where a deferred lockstep step goes: stamps + launch time vs streams
set -o pipefail
OUT=gpurun_out/r02z
mkdir -p $OUT
HTM_AMD_STAMPS=1 STAMP_STEPS=128 timeout -k 10 300 python -u tools/stamps.py > $OUT/stamps.json 2> $OUT/stamps.err || { tail -5 $OUT/stamps.err; exit 1; }
cat $OUT/stamps.json
SCAN_STREAMS=64,256,768,1024 SCAN_STEPS=64 timeout -k 10 300 python -u tools/lockstep_scan.py > $OUT/scan.json 2> $OUT/scan.err || { tail -5 $OUT/scan.err; exit 1; }
tail -1 $OUT/scan.json
