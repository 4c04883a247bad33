// tm_k_wide.hip -- the heavy streams of an ordered frozen lockstep launch
// (HTM_OPT_WIDE): the same TM step as htm_run_frozen_kernel's TM-only launch,
// by HTM_WIDE_NT-thread workgroups (12 waves: 3 per SIMD at the narrow
// kernel's register budget).  The ordered launch's makespan is its heaviest
// step (a bursting stream's rank-window counting, profiles/r04_ab); three
// times the waves on that step's counting, listing and summation shorten it.
// tm_core.h is compiled here for TM_NT = HTM_WIDE_NT inside its own namespace
// (its layout and helpers depend on TM_NT: no symbol may be shared with the
// 256-thread units).
#ifndef HTM_WIDE_NT
#define HTM_WIDE_NT 768
#endif
#define TM_NT HTM_WIDE_NT
#include "sp_dev.h"
namespace htm_wide {
#include "tm_core.h"
}

__global__ __launch_bounds__(TM_NT) void htm_run_wide_kernel(HTM_RUN_ARGS) {
    htm_wide::htm_run_body<false, true, false, false, true, true>(HTM_RUN_PASS);
}

TM_RUN_KERNEL_EXPORTS(run_wide, htm_run_wide_kernel)

size_t tmk_wide_lds_bytes(const DevCfg& c) { return htm_wide::tm_layout(c, 0, 1).total; }

int launch_htm_run_wide(const DevCfg& c, const TmBufs& b, const SpBufs& sp, const double* values, float* scores,
                        int n, int grid, hipStream_t st) {
    if (n <= 0 || grid <= 0 || b.ord_role != 1 || !b.ord_est || b.wide_q < 0 || b.wide_q >= ORD_NB) return -1;
    size_t lds = tmk_wide_lds_bytes(c);
#ifdef HTM_WIDE_LDS_MIN
    // (experiment builds: a 256-thread heavy-step kernel kept alone on its CU
    // by its LDS request)
    if (lds < (size_t)HTM_WIDE_LDS_MIN) lds = (size_t)HTM_WIDE_LDS_MIN;
#endif
    return tmk_launch_run_wide(grid, lds, st, c, b, sp, values, scores, 1, 0, 0, 0, nullptr, 1, n);
}
