// sp_dev.h -- ScalarEncoder + SpatialPooler step of one stream as device
// code, shared by the standalone SP kernel (sp.hip) and the fused SP+TM
// step/run kernels (tm.hip).  See sp.hip for the reference citations and
// the MI355X design notes.
#pragma once
#include <type_traits>

#include "htm_dev.h"

// ScalarEncoder._getFirstOnBit (double arithmetic, NaN -> missing)
__device__ __forceinline__ int enc_first_on_bit(const DevCfg& c, int f, double x) {
    if (isnan(x)) return -1;
    const double lo = c.enc_min[f], hi = c.enc_max[f], res = c.enc_resolution[f];
    if (x < lo) {
        if (!c.enc_clip) return -1;
        x = lo;
    }
    if (x > hi) {
        if (!c.enc_clip) return -1;
        x = hi;
    }
    double q = __ddiv_rn(__dadd_rn(__dadd_rn(x, -lo), __ddiv_rn(res, 2.0)), res);
    int centerbin = (int)q + c.enc_halfwidth;
    return centerbin - c.enc_halfwidth;
}

// ---------------------------------------------------------------------------
// Overlap + global inhibition by wave 0.  Lane l owns words l and l+64.
//
// Encoder input (SpShared): <= 2048 input bits, < 128 of them active, so the
// overlaps fit 7 bit-sliced planes and the active rows are listed.
struct SpShared {
    static constexpr int kPlanes = HTM_NPLANES;
    uint32_t in[64];           // input SDR bits (nin_pad <= 2048)
    uint32_t act[HTM_MAXNW];   // active columns bitmap
    uint32_t ovnz[HTM_MAXNW];  // overlap > 0
    int32_t act_inputs[256];   // active input rows
    uint16_t actlist[HTM_MAXACT];
    int32_t n_act_inputs;
    int32_t nact;
    uint32_t iter;
    int32_t nbump;
    uint16_t bump[HTM_MAXNW * 32 > 4096 ? 4096 : HTM_MAXNW * 32];
    float red[16];  // per-wave maxima (<= 16 waves)
#ifdef HTM_STAMPS
    uint64_t st_t_learn;  // shader clock when the learning part began (0: no learning)
#endif
    template <class F>
    __device__ __forceinline__ void each_active_input(const DevCfg&, F&& f) const {
        for (int a = 0; a < n_act_inputs; a++) f(act_inputs[a]);
    }
};

// External SDR input (the second level of Models 2/3: the L1 TM bottomUpOut,
// up to HTM_MAX_SDR bits, any number of them active): the whole input bitmap
// sits in LDS and the overlap walks its set bits; 15 planes hold overlaps up
// to 32767 >= any input width accepted.
struct SpSharedSdr {
    static constexpr int kPlanes = 15;
    uint32_t in[HTM_MAX_SDR / 32];
    uint32_t act[HTM_MAXNW];
    uint32_t ovnz[HTM_MAXNW];
    uint16_t actlist[HTM_MAXACT];
    int32_t nact;
    uint32_t iter;
    int32_t nbump;
    uint16_t bump[HTM_MAXNW * 32 > 4096 ? 4096 : HTM_MAXNW * 32];
    float red[16];
    template <class F>
    __device__ __forceinline__ void each_active_input(const DevCfg& c, F&& f) const {
        const int pw = c.nin_pad >> 5;
        for (int w = 0; w < pw; w++)
            for (uint32_t x = in[w]; x; x &= x - 1) f(w * 32 + __ffs(x) - 1);
    }
};

// Boosted inhibition (learning with boostStrength != 0, boostOverlaps_ then
// inhibitColumnsGlobal_ on the float32 products): bkey holds the stream's
// boost factors as float bits in a padded transposed layout, bkey[j * (nw + 1)
// + w] for column 32 w + j (lane-consecutive, so wave 0's accesses are
// conflict-free); it is overwritten with boost * overlap.
__device__ __forceinline__ uint32_t bkey_at(const DevCfg& c, int col) {
    return (uint32_t)((col & 31) * (c.nw + 1) + (col >> 5));
}

// Partial overlaps of the SpShared path by every wave of the workgroup:
// wave w adds the rows of listed inputs w, w + NW, ... (all of them loaded
// before any is added: one HBM round trip per wave) into its own bit-sliced
// planes and stores them to `planes` ([NW][HTM_NPLANES][128] words, LDS);
// sp_overlap_inhibit's wave 0 then sums the NW partials.  Call with every
// thread; a barrier must follow.
constexpr int SP_PLANE_WORDS = 4 * HTM_NPLANES * 128;  // (workgroups of <= 4 waves)
__device__ __forceinline__ void sp_overlap_partial(const DevCfg& c, const SpBufs& b, int s, const SpShared& sh,
                                                   uint32_t* planes) {
    constexpr int NPL = HTM_NPLANES;
    constexpr int RB = 8;
    const int l = lane_id(), w = wave_id(), nwv = blockDim.x >> 6;
    const int nw = c.nw;
    const uint32_t* connT = b.connT + (size_t)model_stream(c, s) * c.nin_pad * nw;
    uint32_t p0[NPL], p1[NPL];
#pragma unroll
    for (int k = 0; k < NPL; k++) { p0[k] = 0; p1[k] = 0; }
    const int na = sh.n_act_inputs;
    for (int a0 = w; a0 < na; a0 += RB * nwv) {
        uint32_t r0[RB], r1[RB];
#pragma unroll
        for (int u = 0; u < RB; u++) {
            const int a = a0 + u * nwv;
            const bool in = a < na;
            const uint32_t* row = connT + (size_t)(in ? sh.act_inputs[a] : 0) * nw;
            r0[u] = in && l < nw ? row[l] : 0u;
            r1[u] = in && (l + 64) < nw ? row[l + 64] : 0u;
        }
#pragma unroll
        for (int u = 0; u < RB; u++) {
            uint32_t x0 = r0[u], x1 = r1[u];
#pragma unroll
            for (int k = 0; k < NPL; k++) {
                uint32_t t0 = p0[k] & x0, t1 = p1[k] & x1;
                p0[k] ^= x0; p1[k] ^= x1;
                x0 = t0; x1 = t1;
            }
        }
    }
    uint32_t* mine = planes + w * NPL * 128;
#pragma unroll
    for (int k = 0; k < NPL; k++) {
        mine[k * 128 + l] = p0[k];
        mine[k * 128 + 64 + l] = p1[k];
    }
}

template <class SH>
__device__ __forceinline__ void sp_overlap_inhibit(const DevCfg& c, const SpBufs& b, int s, SH& sh, int write_overlaps,
                                                   uint32_t* bkey = nullptr, const uint32_t* planes = nullptr) {
    constexpr int NPL = SH::kPlanes;
    const int l = lane_id();
    const int nw = c.nw;
    uint32_t p0[NPL], p1[NPL];
#pragma unroll
    for (int k = 0; k < NPL; k++) { p0[k] = 0; p1[k] = 0; }
    const uint32_t* connT = b.connT + (size_t)model_stream(c, s) * c.nin_pad * nw;
    // bit-sliced add of each active input's connected-column row
    auto add_row = [&](uint32_t x0, uint32_t x1) {
#pragma unroll
        for (int k = 0; k < NPL; k++) {
            uint32_t t0 = p0[k] & x0, t1 = p1[k] & x1;
            p0[k] ^= x0; p1[k] ^= x1;
            x0 = t0; x1 = t1;
        }
    };
    if (planes) {
        // the waves' partial planes (sp_overlap_partial): wave 0's, then the
        // others added plane by plane (a partial's plane k carries in at bit k;
        // overlaps stay <= 127, so nothing carries past the top plane)
        const int nwv = blockDim.x >> 6;
#pragma unroll
        for (int k = 0; k < NPL; k++) {
            p0[k] = planes[k * 128 + l];
            p1[k] = planes[k * 128 + 64 + l];
        }
        for (int w = 1; w < nwv; w++) {
            const uint32_t* pw = planes + w * NPL * 128;
#pragma unroll
            for (int k = 0; k < NPL; k++) {
                uint32_t x0 = pw[k * 128 + l], x1 = pw[k * 128 + 64 + l];
#pragma unroll
                for (int j = k; j < NPL; j++) {
                    uint32_t t0 = p0[j] & x0, t1 = p1[j] & x1;
                    p0[j] ^= x0; p1[j] ^= x1;
                    x0 = t0; x1 = t1;
                }
            }
        }
    } else if constexpr (std::is_same<SH, SpShared>::value) {
        // the listed inputs' rows, eight loaded before any is added (one HBM
        // round trip per eight rows instead of one per row; a zero row adds
        // nothing)
        constexpr int RB = 8;
        const int na = sh.n_act_inputs;
        for (int a0 = 0; a0 < na; a0 += RB) {
            uint32_t r0[RB], r1[RB];
#pragma unroll
            for (int u = 0; u < RB; u++) {
                const bool in = a0 + u < na;
                const uint32_t* row = connT + (size_t)(in ? sh.act_inputs[a0 + u] : 0) * nw;
                r0[u] = in && l < nw ? row[l] : 0u;
                r1[u] = in && (l + 64) < nw ? row[l + 64] : 0u;
            }
#pragma unroll
            for (int u = 0; u < RB; u++) add_row(r0[u], r1[u]);
        }
    } else {
        sh.each_active_input(c, [&](int input) {
            const uint32_t* row = connT + (size_t)input * nw;
            add_row(l < nw ? row[l] : 0u, (l + 64) < nw ? row[l + 64] : 0u);
        });
    }
    // eligibility: overlap >= stimulusThreshold (bit-sliced compare)
    uint32_t gt0 = 0, gt1 = 0, eq0 = ~0u, eq1 = ~0u;
    for (int k = NPL - 1; k >= 0; k--) {
        if ((c.stim_thr >> k) & 1) { eq0 &= p0[k]; eq1 &= p1[k]; }
        else { gt0 |= eq0 & p0[k]; gt1 |= eq1 & p1[k]; eq0 &= ~p0[k]; eq1 &= ~p1[k]; }
    }
    uint32_t cand0 = (gt0 | eq0) & (l < nw ? ~0u : 0u);
    uint32_t cand1 = (gt1 | eq1) & ((l + 64) < nw ? ~0u : 0u);
    uint32_t win0 = 0, win1 = 0;
    uint32_t need = (uint32_t)c.num_desired;
    if (bkey) {
        // boosted overlaps boost * (Real)overlap as float bits (non-negative
        // floats order as their bits); eligible when >= stimulusThreshold
        const uint32_t ks = (uint32_t)nw + 1u;
        const float thr = (float)c.stim_thr;
        cand0 = cand1 = 0;
        for (int j = 0; j < 32; j++) {
            if (l < nw) {
                uint32_t ov = 0;
#pragma unroll
                for (int k = 0; k < NPL; k++) ov |= ((p0[k] >> j) & 1u) << k;
                const float f = __uint_as_float(bkey[j * ks + l]) * (float)ov;
                bkey[j * ks + l] = __float_as_uint(f);
                if (f >= thr) cand0 |= 1u << j;
            }
            if (l + 64 < nw) {
                uint32_t ov = 0;
#pragma unroll
                for (int k = 0; k < NPL; k++) ov |= ((p1[k] >> j) & 1u) << k;
                const float f = __uint_as_float(bkey[j * ks + l + 64]) * (float)ov;
                bkey[j * ks + l + 64] = __float_as_uint(f);
                if (f >= thr) cand1 |= 1u << j;
            }
        }
        // the num_desired-th largest eligible key: the largest T with at
        // least `need` eligible keys >= T, built bit by bit from the top
        uint32_t T = 0;
        for (int bit = 30; bit >= 0; bit--) {
            const uint32_t x = T | (1u << bit);
            uint32_t cnt = 0;
            for (int j = 0; j < 32; j++) {
                if (((cand0 >> j) & 1u) && bkey[j * ks + l] >= x) cnt++;
                if (((cand1 >> j) & 1u) && bkey[j * ks + l + 64] >= x) cnt++;
            }
            if (wave_sum_u32(cnt) >= need) T = x;
        }
        // above T: winners; equal to T: the ties the index order settles
        uint32_t t0 = 0, t1 = 0;
        for (int j = 0; j < 32; j++) {
            if ((cand0 >> j) & 1u) {
                const uint32_t kv = bkey[j * ks + l];
                if (kv > T) win0 |= 1u << j;
                else if (kv == T) t0 |= 1u << j;
            }
            if ((cand1 >> j) & 1u) {
                const uint32_t kv = bkey[j * ks + l + 64];
                if (kv > T) win1 |= 1u << j;
                else if (kv == T) t1 |= 1u << j;
            }
        }
        cand0 = t0;
        cand1 = t1;
        const uint32_t nwin = wave_sum_u32((uint32_t)(__popc(win0) + __popc(win1)));
        need = nwin < need ? need - nwin : 0u;
    } else {
        for (int k = NPL - 1; k >= 0; k--) {
            uint32_t h0 = cand0 & p0[k], h1 = cand1 & p1[k];
            uint32_t cnt = wave_sum_u32((uint32_t)(__popc(h0) + __popc(h1)));
            if (cnt >= need) {
                cand0 = h0; cand1 = h1;
            } else {
                win0 |= h0; win1 |= h1;
                need -= cnt;
                cand0 &= ~p0[k]; cand1 &= ~p1[k];
            }
        }
    }
    // ties at the threshold: the `need` highest column indices win.  Words
    // are ordered w = l (< 64) then l + 64; suffix counts over word index.
    uint32_t pc0 = __popc(cand0), pc1 = __popc(cand1);
    // suffix sum over words > w: total over all - inclusive prefix
    uint32_t incl1 = wave_incl_scan(pc1);
    uint32_t tot1 = lane63(incl1);
    uint32_t incl0 = wave_incl_scan(pc0);
    uint32_t tot0 = lane63(incl0);
    uint32_t above1 = tot1 - incl1;            // words l+65.. in the upper half
    uint32_t above0 = tot1 + (tot0 - incl0);   // whole upper half + words l+1..63
    // take = clamp(need - above, 0, popcount) in signed arithmetic
    int r1 = (int)need - (int)above1, r0 = (int)need - (int)above0;
    r1 = r1 < 0 ? 0 : (r1 > (int)pc1 ? (int)pc1 : r1);
    r0 = r0 < 0 ? 0 : (r0 > (int)pc0 ? (int)pc0 : r0);
    const uint32_t take1 = (uint32_t)r1, take0 = (uint32_t)r0;
    uint32_t keep0 = 0, keep1 = 0;
    for (uint32_t j = 0; j < take0; j++) { uint32_t pos = 31 - __clz(cand0); keep0 |= 1u << pos; cand0 &= ~(1u << pos); }
    for (uint32_t j = 0; j < take1; j++) { uint32_t pos = 31 - __clz(cand1); keep1 |= 1u << pos; cand1 &= ~(1u << pos); }
    uint32_t a0 = win0 | keep0, a1 = win1 | keep1;
    uint32_t nz0 = 0, nz1 = 0;
#pragma unroll
    for (int k = 0; k < NPL; k++) { nz0 |= p0[k]; nz1 |= p1[k]; }
    if (l < nw) { sh.act[l] = a0; sh.ovnz[l] = nz0; }
    if (l + 64 < nw) { sh.act[l + 64] = a1; sh.ovnz[l + 64] = nz1; }
    // ascending active list
    uint32_t q0 = __popc(a0), q1 = __popc(a1);
    uint32_t e0 = wave_incl_scan(q0) - q0;
    uint32_t t0 = lane63(e0 + q0);
    uint32_t e1 = t0 + wave_incl_scan(q1) - q1;
    uint32_t pos = e0;
    for (uint32_t x = a0; x; x &= x - 1) { if (pos < HTM_MAXACT) sh.actlist[pos] = (uint16_t)(l * 32 + __ffs(x) - 1); pos++; }
    pos = e1;
    for (uint32_t x = a1; x; x &= x - 1) { if (pos < HTM_MAXACT) sh.actlist[pos] = (uint16_t)((l + 64) * 32 + __ffs(x) - 1); pos++; }
    uint32_t total = lane63(e1 + q1);
    if (l == 0) sh.nact = (int32_t)total;
    if (write_overlaps) {
        int32_t* ov = b.overlaps + (size_t)s * c.ncol;
        for (int bit = 0; bit < 32; bit++) {
            if (l < nw) {
                int32_t v = 0;
#pragma unroll
                for (int k = 0; k < NPL; k++) v |= (int32_t)((p0[k] >> bit) & 1u) << k;
                ov[l * 32 + bit] = v;
            }
            if (l + 64 < nw) {
                int32_t v = 0;
#pragma unroll
                for (int k = 0; k < NPL; k++) v |= (int32_t)((p1[k] >> bit) & 1u) << k;
                ov[(l + 64) * 32 + bit] = v;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// SpatialPooler initialisation draws (nupic::Random, SURVEY.md Appendix A.2;
// oracle/htm_oracle.c sp_init).  Shared by sp_init_kernel (sp.hip) and the
// regeneration of a column's initial permanences for paged engines.

// 31 draws starting at phase 0 (draw index k = 0 mod 31): state and outputs
__device__ __forceinline__ void rng_block(uint32_t (&st)[31], uint32_t* out) {
#pragma unroll
    for (int j = 0; j < 31; j++) {
        const int f = (3 + j) % 31;
        st[f] += st[j];
        out[j] = (st[f] >> 1) & 0x7fffffffu;
    }
}

// What replaying the initialisation draws needs (a few scalars, so the cold
// out-of-line replay of a fused kernel receives them in registers)
struct SpInitCfg {
    int32_t nin, nin_pad, ncol, n_potential, n_ckpt;
    float sp_conn, sp_trim, sp_conn_thr;
    const uint32_t* potmask;
    const uint32_t* ckpt;
    const uint32_t* jump;  // SpBufs::jump (null: skip block by block)
};
__device__ __forceinline__ SpInitCfg sp_init_cfg(const DevCfg& c, const SpBufs& b) {
    return SpInitCfg{c.nin, c.nin_pad, c.ncol, c.n_potential, c.n_ckpt, c.sp_conn, c.sp_trim, c.sp_conn_thr,
                     b.potmask, b.ckpt, b.jump};
}

// Advance the generator (st: the 31-word state in sp_regen_row's form,
// wave-uniform) by nbk whole blocks of 31 draws at once.  The block map
// (st[(3 + j) % 31] += st[j], j = 0..30) is linear over Z/2^32, so nbk blocks
// are the product of the tabled powers B^(2^p) of nbk's set bits: lane j
// computes the new word j as row j of the matrix times the state (31
// multiply-adds, the state read from the lanes) -- a few matrix-vector
// products instead of nbk x 31 dependent scalar adds (the paged replays'
// skip was 63 % of their cycles, profiles/r05_learn).  Call with every lane.
__device__ __forceinline__ void sp_jump_blocks(uint32_t (&st)[31], uint32_t nbk, const uint32_t* jump) {
    const uint32_t l = (uint32_t)lane_id();
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < 31; j++) x = l == (uint32_t)j ? st[j] : x;
    for (uint32_t p = 0; nbk != 0u && p < SP_JUMP_POW; p++, nbk >>= 1) {
        if (!(nbk & 1u)) continue;
        const uint4* row = reinterpret_cast<const uint4*>(jump + ((size_t)p * 31u + (l < 31u ? l : 30u)) * 32u);
        uint4 r[8];
#pragma unroll
        for (int q = 0; q < 8; q++) r[q] = row[q];
        const uint32_t w[32] = {r[0].x, r[0].y, r[0].z, r[0].w, r[1].x, r[1].y, r[1].z, r[1].w,
                                r[2].x, r[2].y, r[2].z, r[2].w, r[3].x, r[3].y, r[3].z, r[3].w,
                                r[4].x, r[4].y, r[4].z, r[4].w, r[5].x, r[5].y, r[5].z, r[5].w,
                                r[6].x, r[6].y, r[6].z, r[6].w, r[7].x, r[7].y, r[7].z, r[7].w};
        uint32_t acc = 0;
#pragma unroll
        for (int i = 0; i < 31; i++) acc += w[i] * (uint32_t)__builtin_amdgcn_readlane((int)x, i);
        x = acc;
    }
#pragma unroll
    for (int j = 0; j < 31; j++) st[j] = (uint32_t)__builtin_amdgcn_readlane((int)x, j);
}

// mapColumn_: the centre input of column col (1-D, potentialRadius = nin)
template <class C>
__device__ __forceinline__ int32_t sp_column_center(const C& c, int col) {
    const float ratio = (float)c.nin / (float)c.ncol;
    const float coord = (float)(((double)col + 0.5) * (double)ratio);
    return (int32_t)floorf(coord);
}

// Random::getReal64() of two raw draws (getUInt64(2^48), never rejected)
__device__ __forceinline__ double sp_real64(uint32_t lo, uint32_t hi) {
    return (double)(((uint64_t)lo | ((uint64_t)hi << 32)) & ((1ull << 48) - 1ull)) * (1.0 / 281474976710656.0);
}

// initPermanence_ of one potential synapse from its four draws (connected
// with probability 0.5: synPermConnected + span * u, else synPermConnected *
// u; 5-digit truncation; trim), then updatePermanencesForColumn_(raise)'s
// clips (stimulusThreshold 0 never loops).  isconn: >= synPermConnected - eps.
template <class C>
__device__ __forceinline__ float sp_init_value(const C& c, uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3,
                                               bool& isconn) {
    const float span = 1.0f - c.sp_conn;  // synPermMax_ - synPermConnected_
    float p;
    if (sp_real64(r0, r1) <= 0.5) p = c.sp_conn + (float)((double)span * sp_real64(r2, r3));
    else p = c.sp_conn * (float)sp_real64(r2, r3);
    p = (float)((double)(int32_t)(p * 100000.0f) / 100000.0);
    p = p < c.sp_trim ? 0.0f : p;
    p = p > 1.0f ? 1.0f : p;
    p = p < 0.0f ? 0.0f : p;
    isconn = p >= c.sp_conn_thr;
    p = p > 1.0f ? 1.0f : p;
    p = p < c.sp_trim ? 0.0f : p;
    return p;
}

// Draws the potential-pool sampling of column col consumed: the selection
// walks inputs in WrappingNeighborhood order from the centre and stops once
// n_potential are chosen, so it made (wrap position of the last chosen input)
// + 1 draws -- read off the stored potential mask.
__device__ __forceinline__ uint32_t sp_sample_draws(const SpInitCfg& c, const uint32_t* prow, int col) {
    const int nin = c.nin;
    const int32_t c0 = sp_column_center(c, col) % nin;
    for (int d = nin - 1; d >= 0; d--) {
        int in = c0 + d;
        if (in >= nin) in -= nin;
        if ((prow[in >> 5] >> (in & 31)) & 1u) return (uint32_t)d + 1u;
    }
    return 0u;
}

// Paged engines: sp_init_kernel's draws for columns col_from..col_hi of
// stream s (one 8-column checkpoint group), replayed by ONE lane from the
// group's checkpoint: write(col, rank, p) receives every initial permanence in
// potential order.  Draws of the group's earlier columns and every column's
// sampling draws are skipped (whole 31-draw blocks advance the state without
// output); then every 4 draws give one permanence.  Registers only.
template <class W>
__device__ __forceinline__ void sp_replay_init(const SpInitCfg& c, int s, int col_from, int col_hi, W&& write) {
    const int pw = c.nin_pad >> 5;
    const int g0 = col_from - col_from % SP_CKPT_COLS;
    const uint32_t* pot = c.potmask + (size_t)s * c.ncol * pw;
    const uint32_t npd = 4u * (uint32_t)c.n_potential;  // permanence draws of a column
    // sampling draws of the group's columns, 16 bits each (<= nin <= 32768)
    uint64_t dlo = 0, dhi = 0;
    for (int k = 0; k < SP_CKPT_COLS && g0 + k <= col_hi; k++) {
        const uint64_t d = sp_sample_draws(c, pot + (size_t)(g0 + k) * pw, g0 + k);
        if (k < 4) dlo |= d << (16 * k);
        else dhi |= d << (16 * (k - 4));
    }
    auto draws = [&](int col) -> uint32_t {
        const int k = col - g0;
        return (uint32_t)((k < 4 ? dlo >> (16 * k) : dhi >> (16 * (k - 4))) & 0xFFFFull);
    };
    uint64_t sk = 0;  // draws to discard before the next permanence draw
    for (int k = g0; k < col_from; k++) sk += draws(k) + npd;
    sk += draws(col_from);
    int col = col_from;
    uint32_t i = 0, q0 = 0, q1 = 0, q2 = 0;
    auto take = [&](uint32_t raw) {
        if (col > col_hi) return;
        if (sk) {
            sk--;
            return;
        }
        const uint32_t ph = i & 3u;
        if (ph == 0) q0 = raw;
        else if (ph == 1) q1 = raw;
        else if (ph == 2) q2 = raw;
        else {
            bool isconn;
            write(col, (int)(i >> 2), sp_init_value(c, q0, q1, q2, raw, isconn));
        }
        if (++i == npd) {
            i = 0;
            col++;
            if (col <= col_hi) sk = draws(col);
        }
    };
    const uint32_t* ck = c.ckpt + ((size_t)s * c.n_ckpt + (size_t)(g0 / SP_CKPT_COLS)) * SP_CKPT_WORDS;
    uint32_t st[31];
#pragma unroll
    for (int j = 0; j < 31; j++) st[j] = ck[j];
    // draws the checkpoint's block had generated but not handed out yet
    for (uint32_t j = ck[31]; j < 31u; j++) take(ck[32 + j]);
    while (col <= col_hi) {
        if (sk >= 31) {
#pragma unroll
            for (int j = 0; j < 31; j++) st[(3 + j) % 31] += st[j];
            sk -= 31;
            continue;
        }
#pragma unroll
        for (int j = 0; j < 31; j++) {
            const int f = (3 + j) % 31;
            st[f] += st[j];
            take((st[f] >> 1) & 0x7fffffffu);
        }
    }
}

// The initial permanences of column col of stream s into a fresh pool row,
// replayed by the whole wave -- sp_replay_init's draws, in the same order.
// The draws the column skips (the group's earlier columns, its own sampling
// draws) advance the generator in whole 31-draw blocks, wave-uniformly in
// scalar registers.  The column's own draws, with an LDS scratch `buf` (512
// words, the wave's share of the SP's overlap planes, free while adapting):
// the generator moves into the lanes (lane j holds the window word j,
// x[n-31+j]) and each block of 31 draws is one stride-3 scan across the lanes
// (y[j] = v[j] + (j >= 3 ? y[j-3] : v[28+j])), written to buf in one store;
// every 256 draws the 64 lanes convert 64 permanences at once and store them
// coalesced (double-buffered: a block that crosses a round boundary writes
// the other half).  Without a scratch the draws go one by one (lane k % 64
// keeps rank k's four).  Inlined: as a call its arguments would arrive in
// VGPRs and the scalar control flow would stay per-lane (exec-masked).  Call
// with every lane of the wave.
template <bool LDSBUF>
static __device__ __forceinline__ void sp_regen_row(SpInitCfg c_, int s_, int col_, float* row_, uint32_t* buf,
                                                    unsigned long long* dbg = nullptr) {
    // wave-uniform for the compiler (pointers stay as passed: a readfirstlane'd
    // pointer trips LLVM's gfx950 verifier, a src_shared_base compare -- the
    // values loaded through them are made uniform where they are read)
    SpInitCfg c = c_;
    c.nin = __builtin_amdgcn_readfirstlane(c_.nin);
    c.nin_pad = __builtin_amdgcn_readfirstlane(c_.nin_pad);
    c.ncol = __builtin_amdgcn_readfirstlane(c_.ncol);
    c.n_potential = __builtin_amdgcn_readfirstlane(c_.n_potential);
    c.n_ckpt = __builtin_amdgcn_readfirstlane(c_.n_ckpt);
    c.sp_conn = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(c_.sp_conn)));
    c.sp_trim = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(c_.sp_trim)));
    c.sp_conn_thr = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(c_.sp_conn_thr)));
    const int s = __builtin_amdgcn_readfirstlane(s_), col = __builtin_amdgcn_readfirstlane(col_);
    float* const row = row_;  // (stores only: per-lane addresses are fine; a readfirstlane'd
                              // pointer trips LLVM's gfx950 verifier, src_shared_base compare)
    const uint32_t l = (uint32_t)lane_id();
    const int pw = c.nin_pad >> 5;
    const int g0 = col - col % SP_CKPT_COLS;
    const uint32_t* pot = c.potmask + (size_t)s * c.ncol * pw;
    const uint32_t npot = (uint32_t)c.n_potential;
    const uint32_t npd = 4u * npot;
    // sampling draws of the group's columns g0..col, one lane each
    uint32_t myd = 0;
#ifdef HTM_STAMPS
    const uint64_t ts0_ = __builtin_amdgcn_s_memtime();
#endif
    if (l < (uint32_t)SP_CKPT_COLS && g0 + (int)l <= col) myd = sp_sample_draws(c, pot + (size_t)(g0 + (int)l) * pw, g0 + (int)l);
    uint32_t sk = 0;  // draws to discard before the column's first permanence draw (< 2^31)
    for (int k = 0; k < col - g0; k++) sk += (uint32_t)__builtin_amdgcn_readlane((int)myd, k) + npd;
    sk += (uint32_t)__builtin_amdgcn_readlane((int)myd, col - g0);
    const uint32_t* ck = c.ckpt + ((size_t)s * c.n_ckpt + (size_t)(g0 / SP_CKPT_COLS)) * SP_CKPT_WORDS;
#ifdef HTM_STAMPS
    const uint64_t ts1_ = __builtin_amdgcn_s_memtime();
    auto stamp_gen = [&]() {  // sampling-draw count, then the whole-block skip
        if (dbg && l == 0) {
            const uint64_t ts2_ = __builtin_amdgcn_s_memtime();
            atomicAdd(&dbg[0], (unsigned long long)(ts1_ - ts0_));
            atomicAdd(&dbg[1], (unsigned long long)(ts2_ - ts1_));
        }
    };
#endif
    uint32_t i = 0;  // the column's draws taken so far
    const uint32_t pend = (uint32_t)__builtin_amdgcn_readfirstlane((int)ck[31]);
    if constexpr (LDSBUF) {
        // ---- LDS path (an explicit LDS pointer: generic accesses make LLVM
        // version the code on an is-shared test whose compare trips the gfx950
        // verifier).  Rounds converted so far; round r = draws [256 r, 256 r + 256)
        typedef __attribute__((address_space(3))) uint32_t lds_u32;
        lds_u32* const lb = (lds_u32*)buf;
        uint32_t rdone = 0;
        auto convert = [&](uint32_t r) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint32_t k = r * 64u + l;
            if (k < npot) {
                const lds_u32* q = lb + ((r & 1u) << 8) + 4u * l;
                bool isconn;
                row[k] = sp_init_value(c, q[0], q[1], q[2], q[3], isconn);
            }
            __builtin_amdgcn_wave_barrier();
        };
        auto rounds = [&]() {  // convert every complete round (and the last partial one)
            const uint32_t have = i < npd ? i : npd;
            while (rdone < (have >> 8)) convert(rdone++);
            if (have == npd && (npd & 255u) && rdone == (npd >> 8)) convert(rdone++);
        };
        // the checkpoint (state and the block's undelivered draws) in one load
        // per lane, read across the lanes afterwards (a load per word made 31
        // dependent round trips)
        const uint32_t ckst = l < 31u ? ck[l] : 0u, ckpd = l < 31u ? ck[32 + l] : 0u;
        // the checkpoint block's undelivered draws, one by one (lane 0 writes)
        for (uint32_t j = pend; j < 31u && i < npd; j++) {
            if (sk) {
                sk--;
                continue;
            }
            const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)ckpd, (int)j);
            if (l == 0) lb[i & 511u] = d;
            i++;
        }
        rounds();
        // whole blocks to skip: the scalar generator
        uint32_t st[31];
#pragma unroll
        for (int j = 0; j < 31; j++) st[j] = (uint32_t)__builtin_amdgcn_readlane((int)ckst, j);
        if (c.jump && sk >= 31u && i < npd) {
            // the tables cover skips below 2^SP_JUMP_POW blocks; the scalar
            // loop below takes any remainder
            const uint32_t nj = (sk / 31u) & ((1u << SP_JUMP_POW) - 1u);
            sp_jump_blocks(st, nj, c.jump);
            sk -= 31u * nj;
        }
        while (sk >= 31u && i < npd) {
#pragma unroll
            for (int j = 0; j < 31; j++) st[(3 + j) % 31] += st[j];
            sk -= 31u;
        }
#ifdef HTM_STAMPS
        stamp_gen();
#endif
        // the generator into the lanes: window word j = st[(3 + j) % 31]
        uint32_t v = 0;
#pragma unroll
        for (int j = 0; j < 31; j++) v = l == (uint32_t)j ? st[(3 + j) % 31] : v;
        while (i < npd) {
            v = rng_block_lanes(v);  // the next window = this block's values (DPP, htm_dev.h)
            // block draw j (lanes < 31): skipped while j < sk, else column draw i + j - sk
            if (l < 31u && l >= sk && i + (l - sk) < npd) lb[(i + (l - sk)) & 511u] = (v >> 1) & 0x7fffffffu;
            i += 31u - sk;
            sk = 0;
            rounds();
        }
        rounds();
        return;
    } else {
    // ---- one draw at a time (no scratch)
    uint32_t q0 = 0, q1 = 0, q2 = 0, q3 = 0;  // this lane's draws of its current rank
    // one draw: discarded, or the next of the column (true when the column is complete)
    auto take = [&](uint32_t raw) -> bool {
        if (sk) {
            sk--;
            return false;
        }
        const uint32_t k = i >> 2, ph = i & 3u;
        const bool mine = (k & 63u) == l;
        if (ph == 0u) q0 = mine ? raw : q0;
        else if (ph == 1u) q1 = mine ? raw : q1;
        else if (ph == 2u) q2 = mine ? raw : q2;
        else {
            q3 = mine ? raw : q3;
            // a round of 64 ranks complete (or the column's last): every lane
            // computes its rank's permanence, one coalesced store
            if ((k & 63u) == 63u || k + 1u == npot) {
                if (l <= (k & 63u)) {
                    bool isconn;
                    row[(k & ~63u) + l] = sp_init_value(c, q0, q1, q2, q3, isconn);
                }
            }
        }
        return ++i == npd;
    };
    // draws the checkpoint's block had generated but not handed out yet
    // (the checkpoint in one load per lane, read across the lanes)
    const uint32_t ckst = l < 31u ? ck[l] : 0u, ckpd = l < 31u ? ck[32 + l] : 0u;
    bool done = false;
    for (uint32_t j = pend; j < 31u && !done; j++) done = take((uint32_t)__builtin_amdgcn_readlane((int)ckpd, (int)j));
    uint32_t st[31];
#pragma unroll
    for (int j = 0; j < 31; j++) st[j] = (uint32_t)__builtin_amdgcn_readlane((int)ckst, j);
#ifdef HTM_STAMPS
    bool gen_ = false;
#endif
    if (c.jump && sk >= 31u && !done) {
        const uint32_t nj = (sk / 31u) & ((1u << SP_JUMP_POW) - 1u);  // (the loop takes any remainder)
        sp_jump_blocks(st, nj, c.jump);
        sk -= 31u * nj;
    }
    while (!done) {
        if (sk >= 31u) {
#pragma unroll
            for (int j = 0; j < 31; j++) st[(3 + j) % 31] += st[j];
            sk -= 31u;
            continue;
        }
#ifdef HTM_STAMPS
        if (!gen_) {
            gen_ = true;
            stamp_gen();
        }
#endif
#pragma unroll
        for (int j = 0; j < 31; j++) {
            const int f = (3 + j) % 31;
            st[f] += st[j];
            if (!done) done = take((st[f] >> 1) & 0x7fffffffu);
        }
    }
    }
}

// Permanence row of column col of stream s (wave-uniform; every lane of the
// wave calls it).  Paged engines hand a column a pool row on its first change
// (lane 0 regenerates the initial values into it); null when the pool is
// exhausted (flagged SP_ERR_POOL: the update is dropped, results invalid).
template <bool PAGED_OK, bool LDSBUF = false>
__device__ __forceinline__ float* sp_perm_row(const DevCfg& c, const SpBufs& b, int s, int col,
                                              uint32_t* scratch = nullptr) {
    const size_t ms = (size_t)model_stream(c, s);
    if (!PAGED_OK || !c.sp_paged) return b.perm + (ms * c.ncol + col) * c.n_potential;
    uint32_t r = 0, fresh = 0;
    uint32_t* slot = b.prow + ms * c.ncol + col;
    if (lane_id() == 0) {
        r = *slot;
        if (r == SP_ROW_NONE) {
            const unsigned long long x = atomicAdd(b.pool_next, 1ull);
            if (x < c.pool_rows) {
                r = (uint32_t)x;
                fresh = 1;
            } else {
                atomicOr(&b.err[s], SP_ERR_POOL);
            }
        }
    }
    r = (uint32_t)__shfl((int)r, 0, 64);
    if (__shfl((int)fresh, 0, 64)) {
        // the wave writes the initial values into the fresh row, then lane 0
        // publishes it; the wave's stores land before its loads of the row
        // (rows are 128-byte aligned and handed out once, so no cache line
        // holds an older copy)
#ifdef HTM_STAMPS
        const uint64_t t0_ = __builtin_amdgcn_s_memtime();
#endif
#ifdef HTM_STAMPS
        sp_regen_row<LDSBUF>(sp_init_cfg(c, b), (int)ms, col, b.pool + (size_t)r * c.pool_stride, scratch,
                             b.dbg ? reinterpret_cast<unsigned long long*>(&b.dbg[(size_t)s * 4 + 2]) : nullptr);
        if (b.dbg && lane_id() == 0) {
            atomicAdd(reinterpret_cast<unsigned long long*>(&b.dbg[(size_t)s * 4]), 1ull);
            atomicAdd(reinterpret_cast<unsigned long long*>(&b.dbg[(size_t)s * 4 + 1]),
                      (unsigned long long)(__builtin_amdgcn_s_memtime() - t0_));
        }
#else
        sp_regen_row<LDSBUF>(sp_init_cfg(c, b), (int)ms, col, b.pool + (size_t)r * c.pool_stride, scratch);
#endif
        if (lane_id() == 0) *slot = r;
        __threadfence();
    }
    if (r == SP_ROW_NONE) return nullptr;
    return b.pool + (size_t)r * c.pool_stride;
}

// updatePermanencesForColumn_ on one potential permanence: returns the new
// value and whether it is connected (>= synPermConnected - epsilon, tested
// after the raise-clip and before the trim-clip).
__device__ __forceinline__ float sp_update_perm(const DevCfg& c, float p, bool raise, bool& isconn) {
    if (raise) {
        p = p > 1.0f ? 1.0f : p;
        p = p < 0.0f ? 0.0f : p;
    }
    isconn = p >= c.sp_conn_thr;
    p = p > 1.0f ? 1.0f : p;
    p = p < c.sp_trim ? 0.0f : p;
    return p;
}

// One wave adapts one column: lane l owns inputs [8l, 8l+8) of each 512-bit
// chunk of the potential mask.  mode 0: adaptSynapses_ (+inc/-dec by input),
// mode 1: bumpUpWeakColumns_ (+synPermBelowStimulusInc, no raise).
template <bool PAGED_OK, bool LDSBUF = false>
__device__ __forceinline__ void sp_adapt_column(const DevCfg& c, const SpBufs& b, int s, int col, const uint32_t* in_bits, int mode,
                                                uint32_t* scratch = nullptr) {
    const int l = lane_id();
    const int pw = c.nin_pad >> 5;
    const size_t ms = (size_t)model_stream(c, s);
    const uint32_t* prow = b.potmask + (ms * c.ncol + col) * pw;
    // the first chunk's potential-mask word is loaded before the row lookup
    // (independent round trips in flight together)
    uint32_t pword = (l >> 2) < pw ? prow[l >> 2] : 0u;
    float* perm = sp_perm_row<PAGED_OK, LDSBUF>(c, b, s, col, scratch);
    if (!perm) return;
    uint32_t* connT = b.connT + ms * c.nin_pad * c.nw;
    const uint32_t cw = (uint32_t)col >> 5, cb = 1u << (col & 31);
    int rank_base = 0;
    for (int chunk = 0; chunk < pw; chunk += 16) {  // 16 words = 512 inputs per pass
        int wi = chunk + (l >> 2);
        uint32_t byte = 0, ibyte = 0;
        if (wi < pw) {
            if (chunk) pword = prow[wi];
            byte = (pword >> ((l & 3) * 8)) & 0xFFu;
            ibyte = (in_bits[wi] >> ((l & 3) * 8)) & 0xFFu;
        }
        const uint32_t pc = __popc(byte);
        const uint32_t incl = wave_incl_scan(pc);
        const uint32_t r0 = rank_base + incl - pc;
        // the lane's (<= 8, consecutive) permanences: every load issued before
        // any is used -- one HBM round trip per chunk, not one per synapse
        float pv[8];
#pragma unroll
        for (int k = 0; k < 8; k++) pv[k] = (uint32_t)k < pc ? perm[r0 + k] : 0.0f;
        uint32_t x = byte;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if ((uint32_t)k < pc) {
                const int j = __ffs(x) - 1;
                x &= x - 1;
                const int input = (chunk + (l >> 2)) * 32 + (l & 3) * 8 + j;
                float p = pv[k];
                const bool oldc = p >= c.sp_conn_thr;
                if (mode == 0) p = p + (((ibyte >> j) & 1u) ? c.sp_inc : -1 * c.sp_dec);
                else p = p + c.sp_below_inc;
                bool newc;
                p = sp_update_perm(c, p, mode == 0, newc);
                perm[r0 + k] = p;
                if (oldc != newc) atomicXor(&connT[(size_t)input * c.nw + cw], cb);
            }
        }
        rank_base += lane63(incl);
    }
}

// The same for the columns of one wave -- list[w], list[w + NW], ... (w =
// wave_id(), NW waves) -- with inputs of one 512-input chunk (nin_pad <= 512)
// and a 512-word LDS scratch for the wave (the fused kernels' overlap planes,
// free while adapting).  Software-pipelined: the pool rows of up to 64 of the
// wave's columns are looked up in one round trip (paged), and a column's
// potential-mask word and whole permanence row (coalesced 16-byte loads) are
// loaded while the previous column is updated; the row is staged through the
// scratch so each lane reads its (<= 8, consecutive) permanences by rank.  A
// column without a pool row (paged) regenerates its initial values first
// (sp_perm_row) and is loaded unpipelined.  Results equal sp_adapt_column's.
template <bool PAGED_OK>
__device__ __forceinline__ void sp_adapt_wave(const DevCfg& c, const SpBufs& b, int s, const uint16_t* list, int n,
                                              const uint32_t* in_bits, int mode, uint32_t* scratch) {
    const int l = lane_id(), w = wave_id(), nwv = blockDim.x >> 6;
    const int nk = n > w ? (n - w + nwv - 1) / nwv : 0;
    if (nk <= 0) return;
    const size_t ms = (size_t)model_stream(c, s);
    const int pw = c.nin_pad >> 5;
    const int npot = c.n_potential;
    const bool paged = PAGED_OK && c.sp_paged;
    uint32_t* connT = b.connT + ms * c.nin_pad * c.nw;
    // inputs of this lane: word l >> 2, byte l & 3
    const uint32_t ibyte = (l >> 2) < pw ? (in_bits[l >> 2] >> ((l & 3) * 8)) & 0xFFu : 0u;
    float4* const st4 = reinterpret_cast<float4*>(scratch);
    // 16-byte row loads: pool rows are 128-byte aligned, dense rows when npot % 4 == 0
    const bool vec = paged || (npot & 3) == 0;
    for (int k0 = 0; k0 < nk; k0 += 64) {
        const int kn = nk - k0 < 64 ? nk - k0 : 64;
        uint32_t mycol = 0u, myrow = SP_ROW_NONE;
        if (l < kn) {
            mycol = list[w + (k0 + l) * nwv];
            if (paged) myrow = b.prow[ms * c.ncol + mycol];
        }
        // stage of column j: its row pointer (null: a fresh paged column, loaded
        // after its regeneration), potential-mask word and row values
        auto rowp = [&](int j) -> const float* {
            const uint32_t col = (uint32_t)__builtin_amdgcn_readlane((int)mycol, j);
            if (!paged) return b.perm + (ms * c.ncol + col) * (size_t)npot;
            const uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)myrow, j);
            return r == SP_ROW_NONE ? nullptr : b.pool + (size_t)r * c.pool_stride;
        };
        auto load = [&](int j, const float* row, uint32_t& pword, float4& v0, float4& v1) {
            const uint32_t col = (uint32_t)__builtin_amdgcn_readlane((int)mycol, j);
            const uint32_t* prow = b.potmask + (ms * c.ncol + col) * pw;
            pword = (l >> 2) < pw ? prow[l >> 2] : 0u;
            const int i0 = 8 * l;
            v0 = v1 = make_float4(0.f, 0.f, 0.f, 0.f);
            if (i0 + 8 <= npot && vec) {
                v0 = *reinterpret_cast<const float4*>(row + i0);
                v1 = *reinterpret_cast<const float4*>(row + i0 + 4);
            } else if (i0 < npot) {
                float x[8];
#pragma unroll
                for (int q = 0; q < 8; q++) x[q] = i0 + q < npot ? row[i0 + q] : 0.f;
                v0 = make_float4(x[0], x[1], x[2], x[3]);
                v1 = make_float4(x[4], x[5], x[6], x[7]);
            }
        };
        uint32_t pw_c = 0u;
        float4 a0, a1;
        const float* row_c = rowp(0);
        if (row_c) load(0, row_c, pw_c, a0, a1);
        for (int j = 0; j < kn; j++) {
            const uint32_t col = (uint32_t)__builtin_amdgcn_readlane((int)mycol, j);
            float* row = const_cast<float*>(row_c);
            if (!row) {  // paged, no pool row yet: regenerate the initial values, then load
                row = sp_perm_row<PAGED_OK, true>(c, b, s, (int)col, scratch);
                if (row) load(j, row, pw_c, a0, a1);
            }
            // the next column's loads go out before this column is updated
            uint32_t pw_n = 0u;
            float4 b0 = make_float4(0.f, 0.f, 0.f, 0.f), b1 = b0;
            const float* row_n = nullptr;
            if (j + 1 < kn) {
                row_n = rowp(j + 1);
                if (row_n) load(j + 1, row_n, pw_n, b0, b1);
            }
            if (row) {
                // stage the row, then each lane takes its ranks
                st4[2 * l] = a0;
                st4[2 * l + 1] = a1;
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                const uint32_t byte = (pw_c >> ((l & 3) * 8)) & 0xFFu;
                const uint32_t pc = __popc(byte);
                const uint32_t incl = wave_incl_scan(pc);
                const uint32_t r0 = incl - pc;
                const float* sf = reinterpret_cast<const float*>(scratch);
                float pv[8];
#pragma unroll
                for (int k = 0; k < 8; k++) pv[k] = (uint32_t)k < pc ? sf[r0 + k] : 0.0f;
                const uint32_t cw = col >> 5, cb = 1u << (col & 31);
                float* sfw = reinterpret_cast<float*>(scratch);
                uint32_t x = byte;
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    if ((uint32_t)k < pc) {
                        const int jb = __ffs(x) - 1;
                        x &= x - 1;
                        const int input = (l >> 2) * 32 + (l & 3) * 8 + jb;
                        float p = pv[k];
                        const bool oldc = p >= c.sp_conn_thr;
                        if (mode == 0) p = p + (((ibyte >> jb) & 1u) ? c.sp_inc : -1 * c.sp_dec);
                        else p = p + c.sp_below_inc;
                        bool newc;
                        p = sp_update_perm(c, p, mode == 0, newc);
#ifdef HTM_SP_RANK_STORES  // (A/B builds: the round-5 per-rank stores)
                        row[r0 + k] = p;
#endif
                        sfw[r0 + k] = p;  // (in place: each lane rewrites its own ranks)
                        if (oldc != newc) atomicXor(&connT[(size_t)input * c.nw + cw], cb);
                    }
                }
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                // the row written back from the scratch with each store
                // instruction covering one contiguous run: float4 q = lane +
                // 64 i (1 KiB per instruction, whole 128-byte lines of a pool
                // row -- its padding past n_potential gets the staged zeros;
                // per-rank 4-byte stores left 64-byte partial-line writes,
                // 1.5x the row's bytes, profiles/r05_end); scalar runs when
                // the row is not 16-byte aligned (dense rows, npot % 4 != 0)
#ifdef HTM_SP_RANK_STORES
                if (false) {
#else
                if (vec) {
#endif
                    const int n4 = paged ? c.pool_stride >> 2 : npot >> 2;
                    float4* row4 = reinterpret_cast<float4*>(row);
                    for (int q = l; q < n4; q += 64) row4[q] = st4[q];
                } else {
#ifndef HTM_SP_RANK_STORES
                    for (int q = l; q < npot; q += 64) row[q] = sfw[q];
#endif
                }
                __builtin_amdgcn_wave_barrier();  // (the scratch is restaged next)
            }
            row_c = row_n;
            pw_c = pw_n;
            a0 = b0;
            a1 = b1;
        }
    }
}

// SP bookkeeping of one compute (updateBookeepingVars_), by one thread
template <bool LEARN, class SH>
__device__ __forceinline__ void sp_count_iteration(const SpBufs& b, int s, SH& sh) {
    uint32_t* sc = b.scalars + (size_t)s * 4;
    uint32_t it = sc[0] + 1;
    sc[0] = it;
    if (LEARN) sc[1] = sc[1] + 1;
    sh.iter = it;
}

// Input stage, encoder: RecordSensor -> MultiEncoder.encodeIntoArray.  A
// ScalarEncoder is computed here; RDSE engines read the list
// rdse_encode_kernel made for this step (enc: [S][enc_list], count first).
template <bool LEARN>
__device__ __forceinline__ void sp_load_input(const DevCfg& c, const SpBufs& b, const double* values, int s,
                                              SpShared& sh, const uint16_t* enc = nullptr) {
    const int t = threadIdx.x;
    if (t < 64) sh.in[t] = 0;
    if (t == 0) {
        int n = 0;
        if (enc) {
            const uint16_t* e = enc + (size_t)s * c.enc_list;
            n = e[0];
            for (int k = 0; k < n; k++) sh.act_inputs[k] = e[1 + k];
        } else {
            for (int f = 0; f < c.n_fields; f++) {
                int bkt = enc_first_on_bit(c, f, values[(size_t)s * c.n_fields + f]);
                b.enc_bucket[(size_t)s * 4 + f] = bkt;
                if (bkt < 0) continue;
                for (int k = 0; k < c.enc_w; k++) sh.act_inputs[n++] = f * c.enc_n + bkt + k;
            }
        }
        sh.n_act_inputs = n;
        sp_count_iteration<LEARN>(b, s, sh);
    }
    __syncthreads();
    for (int k = t; k < sh.n_act_inputs; k += blockDim.x) {
        int i = sh.act_inputs[k];
        atomicOr(&sh.in[i >> 5], 1u << (i & 31));
    }
}

// Input stage, external SDR: row s of a [n_streams][nin_pad/32] bitmap (bits
// past nin are ignored: the link carries exactly inputWidth elements)
template <bool LEARN>
__device__ __forceinline__ void sp_load_input(const DevCfg& c, const SpBufs& b, const uint32_t* sdr, int s,
                                              SpSharedSdr& sh, const uint16_t* = nullptr) {
    const int pw = c.nin_pad >> 5;
    const uint32_t* row = sdr + (size_t)s * pw;
    for (int w = threadIdx.x; w < pw; w += blockDim.x) {
        const int lo = w * 32;
        uint32_t x = row[w];
        if (lo + 32 > c.nin) x &= (1u << (c.nin - lo)) - 1u;
        sh.in[w] = x;
    }
    if (threadIdx.x == 0) sp_count_iteration<LEARN>(b, s, sh);
}

// One SpatialPooler.compute of stream s by the calling workgroup (>= 64
// threads; learning uses every wave).  sh may live in static or dynamic LDS;
// `input` is the encoder values (SpShared) or the input SDR (SpSharedSdr).
// PAGED_OK = false compiles the paged-permanence path out (kernels that
// never run paged engines: the frozen-inference bench kernel).
// bkey: LDS for the boosted inhibition, (nw + 1) * 32 words (used when
// learning with boostStrength != 0); enc: RDSE engines' encoded lists of the step.
// planes: LDS for the waves' partial overlaps (SP_PLANE_WORDS; SpShared input
// only), or null for the one-wave overlap.
template <bool LEARN, bool PAGED_OK = true, bool PLANES = false, class SH, class IN>
__device__ __forceinline__ void sp_step_body(const DevCfg& c, const SpBufs& b, const IN* input, int s,
                                             SH& sh, int write_overlaps, uint32_t* bkey = nullptr,
                                             const uint16_t* enc = nullptr, uint32_t* planes = nullptr) {
    const int t = threadIdx.x;
    const bool boosted = LEARN && bkey && c.sp_boost != 0.0f;
    sp_load_input<LEARN>(c, b, input, s, sh, enc);
    if (boosted) {  // boostFactors_ of the stream -> bkey (float bits)
        const float* bf = b.boost + (size_t)model_stream(c, s) * c.ncol;
        for (int col = t; col < c.ncol; col += blockDim.x) bkey[bkey_at(c, col)] = __float_as_uint(bf[col]);
    }
    __syncthreads();
    if constexpr (std::is_same<SH, SpShared>::value) {
        if (planes) {
            sp_overlap_partial(c, b, s, sh, planes);
            __syncthreads();
        }
    } else {
        planes = nullptr;
    }
    if (t < 64) sp_overlap_inhibit(c, b, s, sh, write_overlaps, boosted ? bkey : nullptr, planes);
    __syncthreads();
    const int nact = sh.nact < HTM_MAXACT ? sh.nact : HTM_MAXACT;
    if (t < nact) b.act[(size_t)s * HTM_MAXACT + t] = sh.actlist[t];
    if (t == 0) b.nact[s] = (uint32_t)nact;
#ifdef HTM_STAMPS
    if constexpr (std::is_same<SH, SpShared>::value) {
        if (t == 0) sh.st_t_learn = LEARN ? __builtin_amdgcn_s_memtime() : 0ull;
    }
#endif
    if (!LEARN) return;  // (callers synchronise before reading b.act)
    // ---- adaptSynapses_: one wave per active column (a paged column's first
    // change replays its initial values through the wave's share of the
    // overlap planes, free now: 512 words per wave)
    constexpr bool LB = PLANES && std::is_same<SH, SpShared>::value;  // (PLANES: the fused kernels' planes)
    static_assert(!LB || (TM_NT / 64) * 512 <= SP_PLANE_WORDS, "replay scratch: 512 words per wave");
    uint32_t* scratch = LB ? planes + wave_id() * 512u : nullptr;
    if (LB && c.nin_pad <= 512 && c.n_potential <= 512) {
        sp_adapt_wave<PAGED_OK>(c, b, s, sh.actlist, nact, sh.in, 0, scratch);
    } else {
        for (int a = wave_id(); a < nact; a += blockDim.x >> 6)
            sp_adapt_column<PAGED_OK, LB>(c, b, s, sh.actlist[a], sh.in, 0, scratch);
    }
    __syncthreads();
    // ---- updateDutyCycles_ (period = min(dutyCyclePeriod, iterationNum))
    float* odc = b.duty + (size_t)model_stream(c, s) * 2 * c.ncol;
    float* adc = odc + c.ncol;
    const uint32_t period = (uint32_t)c.dc_period > sh.iter ? sh.iter : (uint32_t)c.dc_period;
    const float pm1 = (float)(period - 1), pf = (float)period;
    float min_odc = __uint_as_float(b.scalars[(size_t)s * 4 + 2]);
    if (t == 0) sh.nbump = 0;
    __syncthreads();
    float mx = 0.0f;
    float* bf = b.boost + (size_t)model_stream(c, s) * c.ncol;
    for (int col = t; col < c.ncol; col += blockDim.x) {
        float ov = (float)((sh.ovnz[col >> 5] >> (col & 31)) & 1u);
        float ac = (float)((sh.act[col >> 5] >> (col & 31)) & 1u);
        float o = (odc[col] * pm1 + ov) / pf;
        float a = (adc[col] * pm1 + ac) / pf;
        odc[col] = o;
        adc[col] = a;
        // updateBoostFactorsGlobal_ (after bumpUpWeakColumns_, which leaves the
        // duty cycles alone): exp((targetDensity - activeDutyCycle) * strength)
        if (c.sp_boost != 0.0f) bf[col] = exp_det((c.sp_target - a) * c.sp_boost);
        mx = o > mx ? o : mx;
        if (o < min_odc) {  // bumpUpWeakColumns_ candidates
            int k = atomicAdd(&sh.nbump, 1);
            sh.bump[k] = (uint16_t)col;
        }
    }
    // (boostStrength 0: the factors stay exp(0) == 1)
    __syncthreads();
    const int nb = sh.nbump;
    if (nb > 0) {
        // ascending order is irrelevant: each column is updated independently
        if (LB && c.nin_pad <= 512 && c.n_potential <= 512) {
            sp_adapt_wave<PAGED_OK>(c, b, s, sh.bump, nb, sh.in, 1, scratch);
        } else {
            for (int k = wave_id(); k < nb; k += blockDim.x >> 6)
                sp_adapt_column<PAGED_OK, LB>(c, b, s, sh.bump[k], sh.in, 1, scratch);
        }
    }
    // ---- isUpdateRound_: updateMinDutyCyclesGlobal_
    if (sh.iter % (uint32_t)c.update_period == 0) {
        mx = __uint_as_float(wave_max_u32(__float_as_uint(mx)));  // non-negative floats order as uints
        if (lane_id() == 0) sh.red[wave_id()] = mx;
        __syncthreads();
        if (t == 0) {
            float m = sh.red[0];
            for (int w = 1; w < (int)(blockDim.x >> 6); w++) m = sh.red[w] > m ? sh.red[w] : m;
            b.scalars[(size_t)s * 4 + 2] = __float_as_uint(c.sp_min_pct_odc * m);
        }
    }
}

