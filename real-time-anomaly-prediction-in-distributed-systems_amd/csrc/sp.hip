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

#include <algorithm>

// ---------------------------------------------------------------------------
// SP initialisation: one lane per stream runs nupic::Random sequentially (the
// draw order is NuPIC's; draws depend on each other, so the parallelism is
// across streams).  The 31-word additive generator lives in registers: draw k
// updates word (3 + k) mod 31 from word k mod 31, so 31 consecutive draws have
// compile-time indices -- they are generated a block at a time into the lane's
// LDS buffer and consumed from there.  The column's potential and connected
// rows are built in the lane's LDS, stored column-major, and a second kernel
// transposes the connected rows into the input-major bitmap the overlap reads.

// (rng_block, the 31-draw generator step, is in sp_dev.h)
__device__ __forceinline__ void rng_seed_reg(uint32_t (&st)[31], uint64_t seed) {
    int32_t x = (int32_t)(seed % 2147483646ull + 1ull);
    st[0] = (uint32_t)x;
#pragma unroll
    for (int i = 1; i < 31; i++) {
        const int32_t hi = x / 127773, lo = x % 127773;
        x = 16807 * lo - 2836 * hi;
        if (x < 0) x += 2147483647;
        st[i] = (uint32_t)x;
    }
    // 310 burn-in draws = 10 blocks: the phase is 0 again afterwards
    for (int r = 0; r < 10; r++) {
#pragma unroll
        for (int j = 0; j < 31; j++) st[(3 + j) % 31] += st[j];
    }
}

struct RegRng {
    uint32_t st[31];
    uint32_t* buf;  // 31 words of LDS owned by the lane
    int idx;
    __device__ __forceinline__ uint32_t raw() {
        if (idx == 31) {
            rng_block(st, buf);
            idx = 0;
        }
        return buf[idx++];
    }
    // Random::getUInt32(max): raw draws are < 2^31 <= the rejection bound
    __device__ __forceinline__ uint32_t u32(uint32_t max) { return raw() % max; }
    // Random::getReal64(): getUInt64(2^48) (lo | hi << 32, never rejected) * 2^-48
    __device__ __forceinline__ double real64() {
        const uint64_t lo = raw();
        const uint64_t hi = raw();
        return (double)((lo | (hi << 32)) & ((1ull << 48) - 1ull)) * (1.0 / 281474976710656.0);
    }
};

__global__ void sp_init_kernel(DevCfg c, SpBufs b, uint32_t* connC, int s0, int n) {
    extern __shared__ uint32_t dyn[];
    const int pw = c.nin_pad >> 5;
    const int s = s0 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (s >= n) return;  // no barriers below: lanes are independent
    uint32_t* lane_lds = dyn + (size_t)threadIdx.x * (32 + 2 * (size_t)pw);
    RegRng g;
    rng_seed_reg(g.st, b.seeds[s]);
    g.buf = lane_lds;
    g.idx = 31;
    uint32_t* prow = lane_lds + 32;  // potential pool bits of the column
    uint32_t* crow = prow + pw;      // connected bits of the column
    // tieBreaker_[i] = 0.01 * getReal64()  (drawn, unused by global inhibition)
    for (int i = 0; i < c.ncol; i++) (void)g.real64();
    const int nin = c.nin;
    uint32_t* pot = b.potmask + (size_t)s * c.ncol * pw;
    uint32_t* cc = connC + (size_t)(s - s0) * c.ncol * pw;
    float* perm = c.sp_paged ? nullptr : b.perm + (size_t)s * c.ncol * c.n_potential;
    for (int col = 0; col < c.ncol; col++) {
        if (c.sp_paged && col % SP_CKPT_COLS == 0) {
            // paged permanences: the generator state at the group's first
            // column (state, hand-out index, the generated block)
            uint32_t* ck = b.ckpt + ((size_t)s * c.n_ckpt + (size_t)(col / SP_CKPT_COLS)) * SP_CKPT_WORDS;
#pragma unroll
            for (int j = 0; j < 31; j++) ck[j] = g.st[j];
            ck[31] = (uint32_t)g.idx;
            for (int j = 0; j < 31; j++) ck[32 + j] = g.buf[j];
        }
        for (int w = 0; w < pw; w++) prow[w] = crow[w] = 0u;
        const int32_t center = sp_column_center(c, col);
        // WrappingNeighborhood(center, radius = nin) order + Knuth selection sampling
        const uint32_t count = (uint32_t)nin;
        const uint32_t k = (uint32_t)c.n_potential;
        uint32_t chosen = 0;
        int32_t in = center % nin;  // (center - nin + i) mod nin at i = 0
        for (uint32_t i = 0; i < count && chosen < k; i++) {
            if (g.u32(count - i) < k - chosen) {
                prow[in >> 5] |= 1u << (in & 31);
                chosen++;
            }
            if (++in == nin) in = 0;
        }
        // initPermanence_ in input order; updatePermanencesForColumn_(raise)
        float* pr = perm + (size_t)col * c.n_potential;
        int rank = 0;
        for (int w = 0; w < pw; w++) {
            for (uint32_t x = prow[w]; x; x &= x - 1) {
                const int i = w * 32 + __ffs(x) - 1;
                const uint32_t r0 = g.raw(), r1 = g.raw(), r2 = g.raw(), r3 = g.raw();
                bool isconn;
                const float p = sp_init_value(c, r0, r1, r2, r3, isconn);
                if (!c.sp_paged) pr[rank] = p;
                rank++;
                if (isconn) crow[i >> 5] |= 1u << (i & 31);
            }
        }
        for (int w = 0; w < pw; w++) {
            pot[(size_t)col * pw + w] = prow[w];
            cc[(size_t)col * pw + w] = crow[w];
        }
    }
    uint32_t* sc = b.scalars + (size_t)s * 4;
    sc[0] = 0;
    sc[1] = 0;
    sc[2] = 0;  // min overlap duty cycle (float 0.0)
    sc[3] = 0;
    float* bf = b.boost + (size_t)s * c.ncol;  // boostFactors_ start at 1.0
    for (int col = 0; col < c.ncol; col++) bf[col] = 1.0f;
}

// connT[s][i][w] bit (col & 31) = connC[s][col][i / 32] bit (i & 31), w = col / 32:
// one thread per 32 x 32 bit tile (32 column-word loads, a register transpose,
// 32 input-row-word stores)
__global__ void sp_conn_transpose_kernel(DevCfg c, SpBufs b, const uint32_t* connC, int s0, int n) {
    const int pw = c.nin_pad >> 5, nw = c.nw;
    const size_t tiles = (size_t)nw * pw;
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int s = s0 + (int)(t / tiles);
    if (s >= n) return;
    const size_t r = t % tiles;
    const int w = (int)(r / pw), iw = (int)(r % pw);
    const uint32_t* src = connC + (size_t)(s - s0) * c.ncol * pw;
    uint32_t m[32];
#pragma unroll
    for (int j = 0; j < 32; j++) m[j] = src[(size_t)(w * 32 + j) * pw + iw];  // row j = column w*32+j
    // transpose: m[j] bit i (input iw*32+i of column w*32+j) -> o[i] bit j
#pragma unroll
    for (int sh = 16; sh > 0; sh >>= 1) {
        const uint32_t mask = sh == 16 ? 0x0000FFFFu : sh == 8 ? 0x00FF00FFu : sh == 4 ? 0x0F0F0F0Fu
                              : sh == 2 ? 0x33333333u : 0x55555555u;
#pragma unroll
        for (int j = 0; j < 32; j++) {
            if ((j & sh) == 0) {
                const uint32_t a = m[j], bb = m[j | sh];
                m[j] = (a & mask) | ((bb & mask) << sh);
                m[j | sh] = ((a >> sh) & mask) | (bb & ~mask);
            }
        }
    }
    uint32_t* dst = b.connT + (size_t)s * c.nin_pad * nw;
#pragma unroll
    for (int i = 0; i < 32; i++) dst[(size_t)(iw * 32 + i) * nw + w] = m[i];
}

int launch_sp_init(const DevCfg& c, const SpBufs& b, int n, hipStream_t st) {
    const int pw = c.nin_pad >> 5;
    // lanes per block: LDS for 32 rng words + two rows of pw words per lane
    const size_t per_lane = (32 + 2 * (size_t)pw) * 4;
    int lanes = (int)std::min<size_t>(64, std::max<size_t>(1, 32768 / per_lane));
    // column-major connected rows, a chunk of streams at a time (<= 1 GiB)
    const size_t per_stream = (size_t)c.ncol * pw * 4;
    const int chunk = (int)std::max<size_t>(1, std::min<size_t>((size_t)n, ((size_t)1 << 30) / per_stream));
    uint32_t* connC = nullptr;
    if (hipMalloc(&connC, per_stream * chunk) != hipSuccess) return -1;
    int rc = 0;
    for (int s0 = 0; s0 < n && !rc; s0 += chunk) {
        const int s1 = std::min(n, s0 + chunk);
        const int m = s1 - s0;
        hipLaunchKernelGGL(sp_init_kernel, dim3((m + lanes - 1) / lanes), dim3(lanes), per_lane * lanes, st, c, b,
                           connC, s0, s1);
        const size_t threads = (size_t)m * c.nw * pw;
        hipLaunchKernelGGL(sp_conn_transpose_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, c, b,
                           connC, s0, s1);
        if (hipGetLastError() != hipSuccess) rc = -1;
        if (!rc && hipStreamSynchronize(st) != hipSuccess) rc = -1;
    }
    (void)hipFree(connC);
    return rc;
}

// ---------------------------------------------------------------------------
// Paged SP permanences (DevCfg::sp_paged): the host-visible region
// HTM_ST_SP_PERM keeps its dense layout [ncol][n_potential]; these kernels
// convert between it and (pool rows + initial values replayed from the
// checkpoints).  Export: one lane per (stream, 8-column group) writes the
// initial values of the group's columns that have no row, then one wave per
// (stream, column) copies the pool rows.  Import: one lane per (stream,
// group) replays the initial values and gives a row to every column that
// differs from them (or already has one) -- so a stream imported from its own
// export holds no more rows than before.

__global__ void sp_perm_export_init_kernel(DevCfg c, SpBufs b, float* dst, int s0, int m) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (size_t)m * c.n_ckpt) return;
    const int sl = (int)(t / c.n_ckpt), g = (int)(t % c.n_ckpt), s = s0 + sl;
    const int lo = g * SP_CKPT_COLS, hi = min(lo + SP_CKPT_COLS, c.ncol) - 1;
    float* d = dst + (size_t)sl * c.ncol * c.n_potential;
    const uint32_t* map = b.prow + (size_t)s * c.ncol;
    sp_replay_init(sp_init_cfg(c, b), s, lo, hi, [&](int col, int k, float p) {
        if (map[col] == SP_ROW_NONE) d[(size_t)col * c.n_potential + k] = p;
    });
}

__global__ void sp_perm_export_rows_kernel(DevCfg c, SpBufs b, float* dst, int s0, int m) {
    const size_t w = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (w >= (size_t)m * c.ncol) return;
    const int sl = (int)(w / c.ncol), col = (int)(w % c.ncol);
    const uint32_t r = b.prow[(size_t)(s0 + sl) * c.ncol + col];
    if (r == SP_ROW_NONE) return;
    const float* src = b.pool + (size_t)r * c.pool_stride;
    float* d = dst + ((size_t)sl * c.ncol + col) * c.n_potential;
    for (int k = lane_id(); k < c.n_potential; k += 64) d[k] = src[k];
}

__global__ void sp_perm_import_kernel(DevCfg c, SpBufs b, const float* src, size_t src_stride, int s0, int m) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (size_t)m * c.n_ckpt) return;
    const int sl = (int)(t / c.n_ckpt), g = (int)(t % c.n_ckpt), s = s0 + sl;
    const int lo = g * SP_CKPT_COLS, hi = min(lo + SP_CKPT_COLS, c.ncol) - 1;
    const float* in = src + (size_t)sl * src_stride;
    uint32_t* map = b.prow + (size_t)s * c.ncol;
    uint32_t differ = 0;  // bit k: column lo + k differs from its initial values
    sp_replay_init(sp_init_cfg(c, b), s, lo, hi, [&](int col, int k, float p) {
        if (__float_as_uint(in[(size_t)col * c.n_potential + k]) != __float_as_uint(p)) differ |= 1u << (col - lo);
    });
    for (int col = lo; col <= hi; col++) {
        uint32_t r = map[col];
        if (r == SP_ROW_NONE && !((differ >> (col - lo)) & 1u)) continue;
        if (r == SP_ROW_NONE) {
            const unsigned long long x = atomicAdd(b.pool_next, 1ull);
            if (x >= c.pool_rows) {
                atomicOr(&b.err[s], SP_ERR_POOL);
                continue;
            }
            r = (uint32_t)x;
            map[col] = r;
        }
        float* row = b.pool + (size_t)r * c.pool_stride;
        const float* x = in + (size_t)col * c.n_potential;
        for (int k = 0; k < c.n_potential; k++) row[k] = x[k];
    }
}

int launch_sp_perm_export(const DevCfg& c, const SpBufs& b, float* dst, int s0, int m, hipStream_t st) {
    const size_t lanes = (size_t)m * c.n_ckpt;
    hipLaunchKernelGGL(sp_perm_export_init_kernel, dim3((unsigned)((lanes + 63) / 64)), dim3(64), 0, st, c, b, dst, s0, m);
    const size_t waves = (size_t)m * c.ncol;
    hipLaunchKernelGGL(sp_perm_export_rows_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, c, b, dst, s0, m);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_sp_perm_import(const DevCfg& c, const SpBufs& b, const float* src, size_t src_stride, int s0, int m,
                          hipStream_t st) {
    const size_t lanes = (size_t)m * c.n_ckpt;
    hipLaunchKernelGGL(sp_perm_import_kernel, dim3((unsigned)((lanes + 63) / 64)), dim3(64), 0, st, c, b, src,
                       src_stride, s0, m);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// The boosted inhibition's keys ((nw + 1) * 32 words) as dynamic LDS of the
// learning SP kernels, only when boostStrength != 0 (model.yaml): a static
// array sized for 4,096 columns (16.5 KiB) held every Model-1 learning SP
// workgroup to three per CU (41.5 KiB).
static size_t sp_bkey_lds(const DevCfg& c, int learn) {
    return learn && c.sp_boost != 0.0f ? (size_t)(c.nw + 1) * 32 * 4 : 0;
}

// ---------------------------------------------------------------------------
template <bool LEARN>
__global__ __launch_bounds__(256) void sp_step_kernel(DevCfg c, SpBufs b, const double* values, int write_overlaps,
                                                      const uint16_t* enc) {
    __shared__ SpShared sh;
    extern __shared__ __attribute__((aligned(16))) uint32_t sp_dyn[];  // boosted inhibition (sp_bkey_lds)
    sp_step_body<LEARN>(c, b, values, blockIdx.x, sh, write_overlaps, LEARN && c.sp_boost != 0.0f ? sp_dyn : nullptr,
                        enc);
}

// The SP of a split lockstep step, the fused kernel's four-wave SP (its
// learning staged through the overlap planes) as a kernel of its own:
//  * ordered frozen steps (HTM_OPT_ORDERED, dense SP): then the stream's TM
//    cost estimate -- the active cells TM phase 1 will list: a predicted
//    column's predicted cells in infPredictedState(t-1) (tm_bm), all K cells
//    of a bursting one -- to est[s] for ord_sort_kernel;
//  * learning steps (HTM_OPT_SPLIT_LEARN; PAGED: paged permanences): est is
//    null and the TM-only learning kernel follows.
template <bool LEARN, bool PAGED>
__global__ __launch_bounds__(256) void sp_step_ord_kernel(DevCfg c, SpBufs b, const double* values, int write_overlaps,
                                                          const uint16_t* enc, const uint32_t* tm_bm, uint16_t* est) {
    __shared__ SpShared sh;
    extern __shared__ __attribute__((aligned(16))) uint32_t sp_dyn[];  // boosted inhibition (sp_bkey_lds)
    __shared__ uint32_t planes[SP_PLANE_WORDS];
    const int s = blockIdx.x;
#ifdef HTM_SP_BKEY_STATIC  // (A/B builds: the round-5 static LDS footprint, 41.5 KiB)
    __shared__ uint32_t pad_[LEARN ? (HTM_MAXNW + 1) * 32 : 1];
    if (threadIdx.x == 0 && values == nullptr && enc == nullptr) pad_[s & 7] = 0u;
    if (threadIdx.x == 0 && values == nullptr && enc == nullptr) planes[0] = pad_[(s + 1) & 7];
#endif
    sp_step_body<LEARN, PAGED, true>(c, b, values, s, sh, write_overlaps,
                                     LEARN && c.sp_boost != 0.0f ? sp_dyn : nullptr, enc, planes);
    if (!est) return;
    __syncthreads();
    if (wave_id() == 0) {
        const int K = c.K, a = lane_id();
        const int nact = sh.nact < HTM_MAXACT ? sh.nact : HTM_MAXACT;
        const uint32_t* gp = tm_bm + (size_t)s * 4 * c.cw + c.cw;
        uint32_t v = 0;
        if (a < nact) {
            const uint32_t f = bm_field(gp, (uint32_t)sh.actlist[a] * (uint32_t)K, (uint32_t)K);
            v = f ? (uint32_t)__popc(f) : (uint32_t)K;
        }
        v = wave_sum_u32(v);
        if (a == 0) est[s] = (uint16_t)(v < 65535u ? v : 65535u);
    }
}

int launch_sp_step_ord(const DevCfg& c, const SpBufs& b, const double* values, int learn, int n, int keep_overlaps,
                       const uint32_t* tm_bm, uint16_t* est, hipStream_t st) {
    const uint16_t* enc = c.enc_type == HTM_ENC_RDSE ? b.enc_in : nullptr;  // (one step: row 0)
    if (learn && c.sp_paged)
        hipLaunchKernelGGL((sp_step_ord_kernel<true, true>), dim3(n), dim3(256), sp_bkey_lds(c, 1), st, c, b, values, keep_overlaps,
                           enc, tm_bm, est);
    else if (learn)
        hipLaunchKernelGGL((sp_step_ord_kernel<true, false>), dim3(n), dim3(256), sp_bkey_lds(c, 1), st, c, b, values, keep_overlaps,
                           enc, tm_bm, est);
    else
        hipLaunchKernelGGL((sp_step_ord_kernel<false, false>), dim3(n), dim3(256), 0, st, c, b, values, keep_overlaps,
                           enc, tm_bm, est);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Level-2 SP of Models 2/3 (SPRegion fed an SDR, MultiLevelNetworkModel.py:92-95):
// the input bitmap is staged in LDS; one workgroup per stream.
template <bool LEARN>
__global__ __launch_bounds__(256) void sp_step_sdr_kernel(DevCfg c, SpBufs b, const uint32_t* sdr, int write_overlaps) {
    __shared__ SpSharedSdr sh;
    extern __shared__ __attribute__((aligned(16))) uint32_t sp_dyn[];  // boosted inhibition (sp_bkey_lds)
    sp_step_body<LEARN>(c, b, sdr, blockIdx.x, sh, write_overlaps, LEARN && c.sp_boost != 0.0f ? sp_dyn : nullptr);
}

int launch_sp_step_sdr(const DevCfg& c, const SpBufs& b, const uint32_t* sdr, int learn, int n, int keep_overlaps,
                       hipStream_t st) {
    if (learn)
        hipLaunchKernelGGL(sp_step_sdr_kernel<true>, dim3(n), dim3(256), sp_bkey_lds(c, 1), st, c, b, sdr, keep_overlaps);
    else
        hipLaunchKernelGGL(sp_step_sdr_kernel<false>, dim3(n), dim3(256), 0, st, c, b, sdr, keep_overlaps);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_sp_step(const DevCfg& c, const SpBufs& b, const double* values, int learn, int n, int keep_overlaps,
                   hipStream_t st) {
    const uint16_t* enc = c.enc_type == HTM_ENC_RDSE ? b.enc_in : nullptr;  // (one step: row 0)
    if (learn)
        hipLaunchKernelGGL(sp_step_kernel<true>, dim3(n), dim3(256), sp_bkey_lds(c, 1), st, c, b, values, keep_overlaps, enc);
    else
        hipLaunchKernelGGL(sp_step_kernel<false>, dim3(n), dim3(64), 0, st, c, b, values, keep_overlaps, enc);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---------------------------------------------------------------------------
// RandomDistributedScalarEncoder (DevCfg::enc_type == HTM_ENC_RDSE): NuPIC
// 1.0.x nupic/encoders/random_distributed_scalar.py, the encoder of the
// reference's model.yaml parameter set (ML/HTM/params/model.yaml:15-21),
// restated as oracle/htm_oracle.c rdse_*.  Per stream and field the state is a
// header (bucket index range, offset, numTries, the encoder's nupic::Random)
// and the int16 bucket map [HTM_RDSE_BUCKETS][w].  The encoding of a record
// depends on every earlier record of its stream (the offset is the first value
// seen, buckets are created on demand with random draws), so one lane runs a
// stream through the steps of a launch in order; streams run in parallel.  The
// lists of active input bits go to SpBufs::enc_in for the SP kernels.
enum { RH_MIN = 0, RH_MAX = 1, RH_HAS_OFF = 2, RH_TRIES = 3, RH_OFF = 4, RH_RNG = 6, RH_F = 37, RH_R = 38 };

// nupic::Random on the header's state words (global memory, one lane)
__device__ __forceinline__ uint32_t rdse_raw(int32_t* h) {
    uint32_t* st = reinterpret_cast<uint32_t*>(h + RH_RNG);
    int32_t f = h[RH_F], r = h[RH_R];
    st[f] += st[r];
    const uint32_t i = (st[f] >> 1) & 0x7fffffffu;
    if (++f >= 31) { f = 0; ++r; }
    else if (++r >= 31) { r = 0; }
    h[RH_F] = f;
    h[RH_R] = r;
    return i;
}
// Random::getUInt32(max): raw draws are < 2^31 <= the rejection bound
__device__ __forceinline__ uint32_t rdse_u32(int32_t* h, uint32_t max) { return rdse_raw(h) % max; }

__device__ __forceinline__ double rdse_offset(const int32_t* h) {
    return __hiloint2double(h[RH_OFF + 1], h[RH_OFF]);
}

// _overlapOK(i, j, overlap) with _maxOverlap = 2
__device__ __forceinline__ bool rdse_overlap_ok(int w, int i, int j, int ov) {
    const int d = i > j ? i - j : j - i;
    return d < w ? ov == w - d : ov <= 2;
}

// _newRepresentation(from, new_idx) with _newRepresentationOK's running
// overlap against every existing bucket (adjacent buckets differ in one
// position: (i-1) % w below the middle bucket, i % w above)
__device__ void rdse_new_rep(const DevCfg& c, int32_t* h, int16_t* map, int from, int new_idx, uint32_t* bin) {
    const int n = c.enc_n, w = c.enc_w, mid = HTM_RDSE_BUCKETS / 2;
    int16_t* rep = map + (size_t)new_idx * w;
    const int16_t* nbr = map + (size_t)from * w;
    for (int k = 0; k < w; k++) rep[k] = nbr[k];
    const int ri = new_idx % w;
    const int lo = h[RH_MIN], hi = h[RH_MAX];
    for (;;) {
        const int bit = (int)rdse_u32(h, (uint32_t)n);
        rep[ri] = (int16_t)bit;
        bool ok = true;
        for (int k = 0; k < w && ok; k++) ok = nbr[k] != bit;
        if (ok) {
            for (int q = 0; q < (n + 31) / 32; q++) bin[q] = 0u;
            for (int k = 0; k < w; k++) bin[rep[k] >> 5] |= 1u << (rep[k] & 31);
            auto on = [&](int b) { return (int)((bin[b >> 5] >> (b & 31)) & 1u); };
            int run = 0;
            for (int k = 0; k < w; k++) run += on(map[(size_t)lo * w + k]);
            ok = rdse_overlap_ok(w, lo, new_idx, run);
            for (int i = lo + 1; ok && i <= mid; i++) {
                const int nb = (i - 1) % w;
                run += on(map[(size_t)i * w + nb]) - on(map[(size_t)(i - 1) * w + nb]);
                ok = rdse_overlap_ok(w, i, new_idx, run);
            }
            for (int i = mid + 1; ok && i <= hi; i++) {
                const int nb = i % w;
                run += on(map[(size_t)i * w + nb]) - on(map[(size_t)(i - 1) * w + nb]);
                ok = rdse_overlap_ok(w, i, new_idx, run);
            }
            if (ok) return;
        }
        h[RH_TRIES]++;
    }
}

// __init__: nupic::Random(seed), the middle bucket = the first w of
// numpy.arange(n) after Random.shuffle (swap(a[i], a[i + getUInt32(n - i)]));
// the shuffle runs in the map's own rows (n <= 500 w: below the middle row)
__global__ void rdse_init_kernel(DevCfg c, SpBufs b, int n_streams) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_streams * c.n_fields) return;
    const int s = t / c.n_fields;  // (field t % n_fields: the block is per (stream, field))
    uint8_t* blk = b.rdse + (size_t)t * c.rdse_block;
    int32_t* h = reinterpret_cast<int32_t*>(blk);
    int16_t* map = reinterpret_cast<int16_t*>(blk + RDSE_HDR_WORDS * 4);
    const int n = c.enc_n, w = c.enc_w, mid = HTM_RDSE_BUCKETS / 2;
    uint32_t st[31];
    int32_t rf, rr;
    rng_seed(st, rf, rr, b.rdse_seeds[s]);
    for (int i = 0; i < 31; i++) h[RH_RNG + i] = (int32_t)st[i];
    h[RH_F] = rf;
    h[RH_R] = rr;
    for (int i = 0; i < n; i++) map[i] = (int16_t)i;
    for (int i = 0; i < n; i++) {
        const int j = i + (int)rdse_u32(h, (uint32_t)(n - i));
        const int16_t x = map[i];
        map[i] = map[j];
        map[j] = x;
    }
    for (int k = 0; k < w; k++) map[(size_t)mid * w + k] = map[k];
    for (int i = 0; i < n && i < mid * w; i++) map[i] = 0;
    h[RH_MIN] = h[RH_MAX] = mid;
    h[RH_HAS_OFF] = 0;
    h[RH_TRIES] = 0;
    h[RH_OFF] = h[RH_OFF + 1] = 0;
}

int launch_rdse_init(const DevCfg& c, const SpBufs& b, int n, hipStream_t st) {
    const int lanes = n * c.n_fields;
    hipLaunchKernelGGL(rdse_init_kernel, dim3((lanes + 63) / 64), dim3(64), 0, st, c, b, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Python 2 round(): halves away from zero (v - trunc(v) is exact)
__device__ __forceinline__ double round_half_away(double v) {
    const double t = trunc(v);
    const double fr = __dadd_rn(v, -t);
    return fr >= 0.5 ? t + 1.0 : fr <= -0.5 ? t - 1.0 : t;
}

// encodeIntoArray for n_steps records of every stream: getBucketIndices (the
// first value sets the offset; NaN is missing: no bits, offset untouched),
// mapBucketIndexToNonZeroBits (the map grows one neighbour at a time towards
// the bucket, the recursion's order)
__global__ void rdse_encode_kernel(DevCfg c, SpBufs b, const double* values, int n_steps, int n_streams) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_streams) return;
    const int nf = c.n_fields, w = c.enc_w;
    uint32_t bin[64];  // newRep as a bitmap (n <= 2048 bits)
    for (int k = 0; k < n_steps; k++) {
        uint16_t* out = b.enc_in + ((size_t)k * n_streams + s) * c.enc_list;
        int cnt = 0;
        for (int f = 0; f < nf; f++) {
            const double x = values[((size_t)k * n_streams + s) * nf + f];
            uint8_t* blk = b.rdse + ((size_t)s * nf + f) * c.rdse_block;
            int32_t* h = reinterpret_cast<int32_t*>(blk);
            int16_t* map = reinterpret_cast<int16_t*>(blk + RDSE_HDR_WORDS * 4);
            int bkt = -1;
            if (!isnan(x)) {
                if (!h[RH_HAS_OFF]) {
                    const long long bits = __double_as_longlong(x);
                    h[RH_OFF] = (int32_t)(uint32_t)bits;
                    h[RH_OFF + 1] = (int32_t)(uint32_t)(bits >> 32);
                    h[RH_HAS_OFF] = 1;
                }
                double q = (double)(HTM_RDSE_BUCKETS / 2) +
                           round_half_away(__ddiv_rn(__dadd_rn(x, -rdse_offset(h)), c.rdse_res));
                q = q < 0.0 ? 0.0 : q > (double)(HTM_RDSE_BUCKETS - 1) ? (double)(HTM_RDSE_BUCKETS - 1) : q;
                bkt = (int)q;
                if (bkt < h[RH_MIN]) {
                    for (int i = h[RH_MIN] - 1; i >= bkt; i--) {
                        rdse_new_rep(c, h, map, h[RH_MIN], i, bin);
                        h[RH_MIN] = i;
                    }
                } else if (bkt > h[RH_MAX]) {
                    for (int i = h[RH_MAX] + 1; i <= bkt; i++) {
                        rdse_new_rep(c, h, map, h[RH_MAX], i, bin);
                        h[RH_MAX] = i;
                    }
                }
                const int16_t* row = map + (size_t)bkt * w;
                for (int j = 0; j < w; j++) out[1 + cnt++] = (uint16_t)(f * c.enc_n + row[j]);
            }
            if (k == n_steps - 1) b.enc_bucket[(size_t)s * 4 + f] = bkt;
        }
        out[0] = (uint16_t)cnt;
    }
}

int launch_rdse_encode(const DevCfg& c, const SpBufs& b, const double* values, int n_steps, int n, hipStream_t st) {
    hipLaunchKernelGGL(rdse_encode_kernel, dim3((n + 63) / 64), dim3(64), 0, st, c, b, values, n_steps, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
