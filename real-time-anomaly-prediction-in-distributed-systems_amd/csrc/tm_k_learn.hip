// tm_k_learn.hip -- the fused SP+TM kernels that scan the segment pool: TM
// learning on (htm_run_kernel<true>), and TM learning off without the frozen
// index (HTM_OPT_FROZEN_INDEX 0).  Kernel bodies: tm_core.h.
#include "tm_core.h"

// waves per SIMD the kernels are compiled for (the LDS layout fits 3
// workgroups per CU; the register budget decides: 2 -> up to 256 VGPRs)
#ifndef HTM_LEARN_WAVES
#define HTM_LEARN_WAVES 2
#endif
// (A/B probes only: false compiles the paged SP permanences out)
#ifndef HTM_LEARN_PAGED
#define HTM_LEARN_PAGED true
#endif

template <bool LEARN>
__global__ __launch_bounds__(TM_NT) __attribute__((amdgpu_waves_per_eu(HTM_LEARN_WAVES))) void htm_run_kernel(
    HTM_RUN_ARGS) {
    htm_run_body<LEARN, false, HTM_LEARN_PAGED>(HTM_RUN_PASS);
}

TM_RUN_KERNEL_EXPORTS(run_learn, htm_run_kernel<true>)
TM_RUN_KERNEL_EXPORTS(run_infer, htm_run_kernel<false>)
