// tm_k_learn.hip -- the fused SP+TM kernels that scan the segment pool: TM
// learning on (htm_run_kernel<true>), and TM learning off without the frozen
// index (HTM_OPT_FROZEN_INDEX 0).  Kernel bodies: tm_core.h.
#include "tm_core.h"

template <bool LEARN>
__global__ __launch_bounds__(TM_NT) void htm_run_kernel(HTM_RUN_ARGS) {
    htm_run_body<LEARN, false, true>(HTM_RUN_PASS);
}

TM_RUN_KERNEL_EXPORTS(run_learn, htm_run_kernel<true>)
TM_RUN_KERNEL_EXPORTS(run_infer, htm_run_kernel<false>)
