# A/B: block -> list binary search (no owner map) vs main, lockstep config 2
set -o pipefail
OUT=gpurun_out/ab_bs
mkdir -p $OUT
AB_ROUNDS=3 timeout -k 10 900 python -u tools/ab_libs.py main bs bs8 > $OUT/ab.txt 2> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
cat $OUT/ab.txt
