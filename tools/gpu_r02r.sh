# round 2: where the lockstep step goes (stamps, launch time vs streams), then the
# calibrated profile of the config-2 lockstep bench (profiles/r02_final)
set -o pipefail
OUT=gpurun_out/r02r
mkdir -p $OUT
HTM_AMD_STAMPS=1 STAMP_STEPS=128 timeout -k 10 300 python -u tools/stamps.py > $OUT/stamps.json 2> $OUT/stamps.err || { tail -5 $OUT/stamps.err; exit 1; }
cat $OUT/stamps.json
SCAN_STREAMS=64,256,512,768,1024 SCAN_STEPS=64 timeout -k 10 300 python -u tools/lockstep_scan.py > $OUT/scan.json 2> $OUT/scan.err || { tail -5 $OUT/scan.err; exit 1; }
cat $OUT/scan.json
bash tools/gpu_prof.sh $OUT/prof --steps 512 --warmup 16 --other-steps 0 --no-cpu --no-pmc
