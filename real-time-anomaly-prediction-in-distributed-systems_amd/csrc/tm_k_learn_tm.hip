// tm_k_learn_tm.hip -- the TM learning kernel of a split lockstep step
// (HTM_OPT_SPLIT_LEARN): the SP kernel ran first, so the SP is compiled out
// (fewer registers live across the step), and the register budget it leaves
// takes 12 pool-scan batches in flight per thread instead of 8 (236 VGPRs; 16
// spill) -- the pool scans are the bulk of a learning step once the segment
// pools have grown.  Kernel body: tm_core.h.
#ifndef HTM_TMLEARN_SC_DEPTH
#define HTM_TMLEARN_SC_DEPTH 12
#endif
#define SC_DEPTH HTM_TMLEARN_SC_DEPTH
#include "tm_core.h"

#ifndef HTM_LEARN_WAVES
#define HTM_LEARN_WAVES 2
#endif

__global__ __launch_bounds__(TM_NT) __attribute__((amdgpu_waves_per_eu(HTM_LEARN_WAVES))) void htm_run_tmlearn_kernel(
    HTM_RUN_ARGS) {
    htm_run_body<true, false, false, false, true>(HTM_RUN_PASS);
}

TM_RUN_KERNEL_EXPORTS(run_learn_tm, htm_run_tmlearn_kernel)
