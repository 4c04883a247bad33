// tm_k_frozen_paged.hip -- the frozen-inference kernel for engines with paged
// SP permanences (SP learning may page in rows).  Kernel bodies: tm_core.h.
#include "tm_core.h"

__global__ __launch_bounds__(TM_NT) void htm_run_frozen_paged_kernel(HTM_RUN_ARGS) {
    htm_run_body<false, true, true>(HTM_RUN_PASS);
}

TM_RUN_KERNEL_EXPORTS(run_frozen_paged, htm_run_frozen_paged_kernel)
