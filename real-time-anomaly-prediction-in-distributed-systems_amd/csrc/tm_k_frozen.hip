// tm_k_frozen.hip -- the frozen-inference kernels: fused encoder -> SP -> TM
// (frozen forward index) -> raw anomaly with TM learning off -- SP learning off
// too (the bench kernel) or on (the reference's test phase).
// Compiled for HTM_RUN_WAVES waves per SIMD (3: three 256-thread workgroups
// per CU, with the LDS budget sized to match).  Kernel bodies: tm_core.h.
#include "tm_core.h"

#ifndef HTM_RUN_WAVES
#define HTM_RUN_WAVES 3
#endif

// inference only (SP learning off too): the bench kernel
__global__ __launch_bounds__(TM_NT) __attribute__((amdgpu_waves_per_eu(HTM_RUN_WAVES))) void htm_run_frozen_kernel(
    HTM_RUN_ARGS) {
    htm_run_body<false, true, false, false>(HTM_RUN_PASS);
}
// the TM step alone (ordered lockstep steps: sp_step_ord_kernel ran every
// stream's SP first, with or without its learning), the SP compiled out
#ifndef HTM_TMONLY_WAVES
#define HTM_TMONLY_WAVES 3
#endif
__global__ __launch_bounds__(TM_NT) __attribute__((amdgpu_waves_per_eu(HTM_TMONLY_WAVES))) void htm_run_frozen_tm_kernel(
    HTM_RUN_ARGS) {
    htm_run_body<false, true, false, false, true>(HTM_RUN_PASS);
}
// TM frozen, SP learning on (ModelTesting's test phase, NetworkModel.py:40-44):
// the run-mode kernel (lockstep steps of this mode run the SP kernel and then
// the TM-only launch of htm_run_frozen_kernel).  Two waves per SIMD: at three
// the SP learning code spilled (168 VGPRs + 20-52 B/lane scratch); at two it
// takes 193 VGPRs and no scratch
#ifndef HTM_SPL_WAVES
#define HTM_SPL_WAVES 2
#endif
__global__ __launch_bounds__(TM_NT) __attribute__((amdgpu_waves_per_eu(HTM_SPL_WAVES))) void htm_run_frozen_spl_kernel(
    HTM_RUN_ARGS) {
    htm_run_body<false, true, false, true>(HTM_RUN_PASS);
}

TM_RUN_KERNEL_EXPORTS(run_frozen, htm_run_frozen_kernel)
TM_RUN_KERNEL_EXPORTS(run_frozen_tm, htm_run_frozen_tm_kernel)
TM_RUN_KERNEL_EXPORTS(run_frozen_spl, htm_run_frozen_spl_kernel)
