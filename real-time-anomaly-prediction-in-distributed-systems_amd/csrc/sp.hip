// sp.hip -- ScalarEncoder + SpatialPooler compute for N streams on gfx950.
//
// Reference path: RecordSensor -> SPRegion.compute -> nupic.core
// SpatialPooler::compute (spatialImp "cpp"), parameters
// ML/HTM/NetworkUtils.py:26-41,77-88,126-136; call site
// ML/HTM/NetworkModel.py:127 (network.run(1)).  Semantics: SURVEY.md
// Appendix A.1/A.2 (restated in oracle/htm_oracle.c).
//
// MI355X design:
//   * the connected matrix is stored input-major (connT[input][col/32]), so
//     the overlap of a 21-bit encoder SDR reads only 21 rows x 256 B instead
//     of the whole 2048 x 512-bit matrix;
//   * overlaps are accumulated as 7 bit-sliced planes per 32-column word
//     (one word per lane, one wave per stream), and global k-winner
//     inhibition is a radix select over the planes followed by a
//     highest-index tie break -- the nupic.core ">=" insertion order;
//   * learning touches only the active columns' potential permanences
//     (float32, potential order) and flips connected bits with atomicXor.
#include "sp_dev.h"

// ---------------------------------------------------------------------------
// SP initialisation: one lane per stream runs nupic::Random sequentially.
__global__ void sp_init_kernel(DevCfg c, SpBufs b, int n) {
    int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    uint32_t st[31];
    int32_t f, r;
    rng_seed(st, f, r, b.seeds[s]);
    // tieBreaker_[i] = 0.01 * getReal64()  (drawn, unused by global inhibition)
    for (int i = 0; i < c.ncol; i++) (void)rng_real64(st, f, r);
    const int nin = c.nin, pw = c.nin_pad >> 5;
    uint32_t* connT = b.connT + (size_t)s * c.nin_pad * c.nw;
    uint32_t* pot = b.potmask + (size_t)s * c.ncol * pw;
    float* perm = b.perm + (size_t)s * c.ncol * c.n_potential;
    const float span = 1.0f - c.sp_conn;  // synPermMax_ - synPermConnected_
    const float conn = c.sp_conn;
    for (int col = 0; col < c.ncol; col++) {
        float ratio = (float)nin / (float)c.ncol;
        float coord = (float)(((double)col + 0.5) * (double)ratio);
        int32_t center = (int32_t)floorf(coord);
        uint32_t* prow = pot + (size_t)col * pw;
        // WrappingNeighborhood(center, radius=nin) order + Knuth selection sampling
        uint32_t count = (uint32_t)nin;
        uint32_t k = (uint32_t)c.n_potential, chosen = 0;
        for (uint32_t i = 0; i < count && chosen < k; i++) {
            if (rng_u32(st, f, r, count - i) < k - chosen) {
                int32_t in = (center - nin + (int32_t)i) % nin;
                if (in < 0) in += nin;
                prow[in >> 5] |= 1u << (in & 31);
                chosen++;
            }
        }
        // initPermanence_ in input order; updatePermanencesForColumn_(raise)
        float* pr = perm + (size_t)col * c.n_potential;
        int rank = 0;
        for (int i = 0; i < nin; i++) {
            if (!((prow[i >> 5] >> (i & 31)) & 1u)) continue;
            float p;
            if (rng_real64(st, f, r) <= 0.5) {
                p = conn + (float)((double)span * rng_real64(st, f, r));
            } else {
                p = conn * (float)rng_real64(st, f, r);
            }
            p = (float)((double)(int32_t)(p * 100000.0f) / 100000.0);
            p = p < c.sp_trim ? 0.0f : p;
            // raisePermanencesToThreshold_: clip [0,1] (stimulus threshold 0 never loops)
            p = p > 1.0f ? 1.0f : p;
            p = p < 0.0f ? 0.0f : p;
            bool isconn = p >= c.sp_conn_thr;
            p = p > 1.0f ? 1.0f : p;
            p = p < c.sp_trim ? 0.0f : p;
            pr[rank++] = p;
            if (isconn) connT[(size_t)i * c.nw + (col >> 5)] |= 1u << (col & 31);
        }
    }
    uint32_t* sc = b.scalars + (size_t)s * 4;
    sc[0] = 0;
    sc[1] = 0;
    sc[2] = 0;  // min overlap duty cycle (float 0.0)
    sc[3] = 0;
}

int launch_sp_init(const DevCfg& c, const SpBufs& b, int n, hipStream_t st) {
    hipLaunchKernelGGL(sp_init_kernel, dim3((n + 63) / 64), dim3(64), 0, st, c, b, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---------------------------------------------------------------------------
template <bool LEARN>
__global__ __launch_bounds__(256) void sp_step_kernel(DevCfg c, SpBufs b, const double* values, int write_overlaps) {
    __shared__ SpShared sh;
    sp_step_body<LEARN>(c, b, values, blockIdx.x, sh, write_overlaps);
}

int launch_sp_step(const DevCfg& c, const SpBufs& b, const double* values, int learn, int n, int keep_overlaps,
                   hipStream_t st) {
    if (learn)
        hipLaunchKernelGGL(sp_step_kernel<true>, dim3(n), dim3(256), 0, st, c, b, values, keep_overlaps);
    else
        hipLaunchKernelGGL(sp_step_kernel<false>, dim3(n), dim3(64), 0, st, c, b, values, keep_overlaps);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
