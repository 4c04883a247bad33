#!/bin/bash
# learning-kernel stamps (config 3): early window (8 warm-up + 32 steps) and a
# late window (200 warm-up + 32 steps); needs make -C <pkg>/csrc stamps
set -o pipefail
T=${AB_TAG:-lst}
mkdir -p gpurun_out/$T
STAMP_MODE=learn timeout -k 10 300 python -u tools/stamps.py > gpurun_out/$T/stamps_early.json 2>gpurun_out/$T/early.err || exit 1
STAMP_MODE=learn STAMP_WARMUP=${LATE_WARMUP:-200} timeout -k 10 400 python -u tools/stamps.py > gpurun_out/$T/stamps_late.json 2>gpurun_out/$T/late.err || exit 1
