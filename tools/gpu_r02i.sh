set -o pipefail
OUT=gpurun_out/r02i
mkdir -p $OUT
timeout -k 10 900 python -u tools/lockstep_scan.py > $OUT/scan.txt 2> $OUT/scan.err || { tail -5 $OUT/scan.err; exit 1; }
cat $OUT/scan.txt
