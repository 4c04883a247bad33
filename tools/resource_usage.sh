#!/bin/bash
# Kernel resource usage (VGPRs, SGPR spills, scratch, occupancy) of every
# kernel unit, as the compiler reports it (-Rpass-analysis=kernel-resource-usage),
# with the product library's flags.  usage: bash tools/resource_usage.sh [extra flags] > out.txt
cd "$(dirname "$0")/../real-time-anomaly-prediction-in-distributed-systems_amd/csrc" || exit 1
for u in tm_k_frozen.hip tm_k_frozen_paged.hip tm_k_learn.hip tm_k_learn_tm.hip tm_k_step.hip sp.hip tm.hip; do
    echo "== $u"
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math "$@" \
        -Rpass-analysis=kernel-resource-usage --offload-device-only -c -x hip "$u" -o /dev/null 2>&1 |
        grep -E "Function Name|TotalSGPRs|VGPRs:|AGPRs|ScratchSize|Occupancy|SGPRs Spill|VGPRs Spill|LDS Size" |
        sed -e 's/^.*remark: //' -e 's/^[^ ]*: //' -e 's/^\(Function Name\)/\1/' -e 's/^\([A-Z]\)/    \1/' -e 's/^    Function/Function/'
done
