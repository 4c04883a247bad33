// tm_k_frozen.hip -- the frozen-inference kernel (the bench kernel): fused
// encoder -> SP -> TM (frozen forward index) -> raw anomaly, learning off.
// Compiled for HTM_RUN_WAVES waves per SIMD (3: three 256-thread workgroups
// per CU, with the LDS budget sized to match).  Kernel bodies: tm_core.h.
#include "tm_core.h"

#ifndef HTM_RUN_WAVES
#define HTM_RUN_WAVES 3
#endif

__global__ __launch_bounds__(TM_NT) __attribute__((amdgpu_waves_per_eu(HTM_RUN_WAVES))) void htm_run_frozen_kernel(
    HTM_RUN_ARGS) {
    htm_run_body<false, true, false>(HTM_RUN_PASS);
}

TM_RUN_KERNEL_EXPORTS(run_frozen, htm_run_frozen_kernel)
