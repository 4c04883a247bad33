// tm_k_step.hip -- unfused TM step kernels (one launch per step after the SP
// kernel): the SDR-input engines of Models 2/3 and HTM_OPT_FUSED 0.  Kernel
// bodies: tm_core.h.
#include "tm_core.h"

template <bool LEARN, bool FROZEN>
__global__ __launch_bounds__(TM_NT) void tm_step_kernel(DevCfg c, TmBufs b, SpBufs sp, float* scores, int keep_prev) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    tm_step_body<LEARN, FROZEN>(c, b, sp, scores, keep_prev, blockIdx.x, lds);
}

int tmk_launch_step(int learn, int frozen, int grid, size_t lds, hipStream_t st, DevCfg c, TmBufs b, SpBufs sp,
                    float* scores) {
    if (learn)
        hipLaunchKernelGGL((tm_step_kernel<true, false>), dim3(grid), dim3(TM_NT), lds, st, c, b, sp, scores, 0);
    else if (frozen)
        hipLaunchKernelGGL((tm_step_kernel<false, true>), dim3(grid), dim3(TM_NT), lds, st, c, b, sp, scores, 0);
    else
        hipLaunchKernelGGL((tm_step_kernel<false, false>), dim3(grid), dim3(TM_NT), lds, st, c, b, sp, scores, 0);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int tmk_attr_step(size_t lds_learn, size_t lds_frozen, size_t lds_scan) {
    const hipError_t e0 = hipFuncSetAttribute((const void*)tm_step_kernel<true, false>,
                                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_learn);
    const hipError_t e1 = hipFuncSetAttribute((const void*)tm_step_kernel<false, true>,
                                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_frozen);
    const hipError_t e2 = hipFuncSetAttribute((const void*)tm_step_kernel<false, false>,
                                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_scan);
    return e0 == hipSuccess && e1 == hipSuccess && e2 == hipSuccess ? 0 : -1;
}
