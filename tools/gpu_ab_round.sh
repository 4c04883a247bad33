# parity suite + A/B of build variants + rocprof/PMC of the default build
set -o pipefail
T=${AB_TAG:-ab}
mkdir -p gpurun_out/$T
AB_TAG=$T AB_STAMPS=0 AB_STEPS=${AB_STEPS:-1200} AB_VARIANTS="${AB_VARIANTS:-fused=1}" bash tools/ab_fin.sh || exit $?
STAMPS=0 bash tools/gpu_round.sh $T ${PROF_STEPS:-600}
