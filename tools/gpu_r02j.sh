set -o pipefail
OUT=gpurun_out/r02j
mkdir -p $OUT
AB_ROUNDS=3 timeout -k 10 1100 python -u tools/ab_libs.py main prev > $OUT/ab_libs.txt 2> $OUT/ab_libs.err || { tail -20 $OUT/ab_libs.err; exit 1; }
cat $OUT/ab_libs.txt
