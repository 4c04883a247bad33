// tm_core.h -- BacktrackingTM (TMRegion, temporalImp "cpp") + raw anomaly for
// N streams on gfx950, one 256-thread workgroup per stream per step.
//
// Reference path: TMRegion.compute -> BacktrackingTMCPP.compute -> Cells4
// (params ML/HTM/NetworkUtils.py:44-64,140-153; anomaly read at
// ML/HTM/NetworkModel.py:133).  Control flow restates NuPIC's BacktrackingTM
// (updateInferenceState / inferPhase1 / inferPhase2 / inferBacktrack,
// updateLearningState / learnPhase1 / learnPhase2 / learnBacktrack,
// processSegmentUpdates, adaptSegment, getBestMatchingCell,
// getCellForNewSegment, chooseCellsToLearnFrom) exactly as oracle/htm_oracle.c
// does.
//
// MI355X design:
//   * the whole step of one stream runs inside one workgroup: its bitmaps
//     (cells x 1 bit), column confidences and bookkeeping live in LDS;
//     segment state streams from HBM;
//   * inference phase 2 (the hot loop) has two forms with identical results:
//       - learning on:  a coalesced scan of the segment pool (4 lanes per
//         segment, 16 B of synapse sources each) probing the LDS bitmap;
//       - learning off: forward propagation over a frozen cell -> segment
//         index (what Cells4's _outSynapses does), counting active synapses
//         per segment with LDS atomics in windows of the slot space, so a
//         step reads only the out-synapses of the active cells;
//   * the float32 column confidences are summed in NuPIC's (column, cell,
//     segment) order (bucket sort of the qualifying segments), so they are
//     bit-identical to the oracle;
//   * the data-dependent nupic::Random draws of learning run on lane 0 of
//     wave 0 in NuPIC order; everything else is wave- or workgroup-parallel.
#pragma once
#include "sp_dev.h"

static __constant__ float kDcAlpha[9] = {0.0f, 0.0032f, 0.0010f, 0.00032f, 0.00010f, 0.000032f, 0.00001f, 0.0000032f, 0.0000010f};
static __constant__ uint32_t kDcTier[9] = {0, 100, 320, 1000, 3200, 10000, 32000, 100000, 320000};

struct __attribute__((aligned(16))) TmSh {
    double avg_dens, avg_lsl;
    unsigned long long bytes;      // algorithmic HBM bytes of this step (thread 0 / LDS atomics)
    unsigned long long bytes_acc;  // ... of the earlier steps of a run kept in LDS
    uint32_t lrn_iter, iter;
    int32_t pam, lsl, reset, have_avg;
    uint32_t rng[31];
    int32_t rf, rr;
    uint32_t hwm, nlive;
    int32_t n_inf_pat, n_lrn_pat, inf_head, lrn_head;
    uint16_t inf_len[HTM_MAXPAT], lrn_len[HTM_MAXPAT];
    int32_t n_upd;
    uint32_t err;
    uint32_t st[4];
    int32_t nA;
    int32_t qn;
    int32_t ncand;
    int32_t ti[8];
    int32_t npc_known;  // numPredictedCols of the current frozen phase 2 once counted, else -1
    int32_t fx_na;      // active cells listed by the last frozen collection (U: the cell list)
    uint32_t p1_off;    // LDS offset of the active columns (ascending) phase 1 built infA from
    int32_t p1_n;       // their number, or -1 when infA is not phase 1's
    int32_t lp2p;       // the previous step's final learnPhase2 is pending (lp2_finish)
    int32_t lp2s;       // ... and this step's first pool scan has counted its best matches (Tm::lkey)
    float tf[4];
    uint32_t red[3 * TM_NWAVES];
    uint32_t nz_valid;  // the loaded nonzero-column bitmap of colConfidence(t-1) is current (first step)
    uint32_t acc[3];    // wg_sum1's rotating accumulators
    uint16_t act[HTM_MAXACT];
    uint32_t cand[HTM_MAXACT];
    uint32_t newsrc[HTM_MAXSYN];
    __attribute__((aligned(16))) uint16_t inf_pat[HTM_MAXPAT][HTM_MAXACT];
#ifdef HTM_STAMPS
    uint64_t st_acc[HTM_NSTAMP], st_cnt[HTM_NSTAMP], st_last, st_start, st_sp0;
#endif
};

struct Tm {
    DevCfg c;
    int s;
    TmSh* sh;
    // LDS regions
    uint32_t *infA, *infP, *infP1, *lrnA, *lrnA1, *lrnP, *lrnP1;
    float* colconf;
    uint32_t* flags;   // ncol bits
    uint32_t* U;       // union region
    uint32_t* lkey;    // learning: the deferred learnPhase2's best-match keys, u32 [ncol] (lp2_finish)
    uint16_t (*lrnpat)[HTM_MAXACT];  // learn-state pattern ring (learning layouts only)
    // global, this stream
    uint32_t* meta;
    uint16_t* src;
    float* perm;
    uint32_t* conn;
    uint32_t* duty;
    uint8_t* nseg;
    htm_tm_update* upd;
    uint32_t* sbm;     // scratch bitmaps [5][cw]
    float* sconf;
    uint32_t* q1;
    uint32_t* q2;
    const uint32_t* fxoff;
    const uint4* fxent;
    const uint2* fxrec;
    const uint32_t* fxrslot;
    const uint16_t* fxpcell;
    uint32_t np;       // predictive-capable segments (pids) of this stream
    uint32_t nr;       // ranks (live segments) of the frozen index
    const TmBufs* tb;  // the engine's buffers (deferred-duty log)
    bool defer;        // discarded frozen phase 2s log their active cells (TmBufs::fx_dlog)
    uint32_t dn, df;   // deferred log: entries logged, entries flushed (every thread's copy)
    uint32_t rh, rl;   // hash and length of the set in ring slot (threadIdx.x % 64) (slots < fx_dcap)
    uint32_t nsum;     // wg_sum1 calls so far (every thread's copy)
};

// stamp buckets (HTM_STAMPS): where one stream-step's cycles go
enum {
    SB_LOAD = 0, SB_P1, SB_LIST, SB_WINPRE, SB_STREAM, SB_QSCAN, SB_FIN1, SB_FIN2, SB_BT, SB_LEARN, SB_WB,
    SB_SCAN, SB_SORT, SB_SUMS, SB_OWNER, SB_SLOAD, SB_COUNT, SB_FCLR, SB_CPC, SB_DEFER, SB_SP, SB_NORM,
    // learning (round 4): learn-phase pool scans (scan_best), queued segment
    // updates, wave 0's serial adapt / create / update-building, the learn
    // backtrack's state copies, pool compaction, the SP's learning part
    // (adaptSynapses_ incl. paged-row replays, duty cycles, weak-column bumps)
    SB_LSCAN, SB_LUPD, SB_LW, SB_LBT, SB_COMPACT, SB_SPL,
    // (round 5) the learning loops split: update building (active-synapse
    // masks, candidate filters), generator draws (sampling, getCellForNewSegment),
    // segment writes (adapt, trim, create, queued-update appends)
    SB_LWB, SB_LWS, SB_LWW,
    SB_NCMP  // the normaliser's run-head compaction (frozen ranked tail)
};
// event counts: phase2 calls, windows, out-list blocks, qualifying segments, active cells
// and a histogram of whole-step cycles: SC_HIST + b counts steps of
// [2^(15+b), 2^(16+b)) cycles (b = 0 also holds shorter ones, b = 8 longer)
enum { SC_P2 = 0, SC_WIN, SC_BLK, SC_QN, SC_NACT, SC_TNZ, SC_STEPS, SC_HIST };
// (SC_HIST .. SC_HIST + 8 are the histogram) learning counts: pool scans and
// the slots they swept, SP paged-row replays and the lane-0 cycles they took
// (summed over waves; filled in by htm_debug_stamps from SpBufs::dbg)
enum { SC_NSCAN = 16, SC_SCANSLOTS, SC_REPLAY, SC_REPLAYCYC, SC_REPLAYSAMPLE, SC_REPLAYSKIP,
       // learning loops: columns of learn phase 1 / 2, sampling calls, draws consumed,
       // the cycles inside the samples, generator blocks made
       SC_LP1COLS, SC_LP2COLS, SC_LSAMPLES, SC_LDRAWS, SC_LSAMPLECYC, SC_LBLOCKS };

// learning loops (wave-parallel, round 5): column records per pass (learn
// phase 1: <= HTM_MAXACT columns; phase 2 in batches) and their LDS words
// (48-byte records, then each wave's new-source list)
#define LREC_N 64
#define LREC_WORDS (LREC_N * 12 + TM_NWAVES * HTM_MAXSYN)

// ---------------------------------------------------------------------------
// LDS layout
struct TmLayout {
    size_t off_lpat, off_bm, off_conf, off_flags, off_lkey, off_U, total;
    int nbm;
    size_t u_words;
};

__host__ __device__ inline size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

// nosp: a TM-only launch (the SP kernel ran first): no SP step in the union
__host__ __device__ inline TmLayout tm_layout(const DevCfg& c, int learn, int frozen, int nosp = 0) {
    TmLayout L;
    L.nbm = learn ? 7 : 3;
    size_t o = align16(sizeof(TmSh));
    L.off_lpat = o;  // the learn-state pattern ring: learning only
    if (learn) o = align16(o + (size_t)HTM_MAXPAT * HTM_MAXACT * 2);
    L.off_bm = o;
    o = align16(o + (size_t)L.nbm * c.cw * 4);
    L.off_conf = o;
    o = align16(o + (size_t)c.ncol * 4);
    L.off_flags = o;
    o = align16(o + (size_t)c.nw * 4);
    L.off_lkey = o;  // learning only: the deferred learnPhase2's keys
    if (learn) o = align16(o + (size_t)c.ncol * 4);
    L.off_U = o;
    // union of phase-local arrays:
    //  finish: colcnt[ncol] u32, nzcol[ncol] u16, nzstart[ncol+1] u32, and the
    //          qualifying-segment buffers qkey/qdc/skey/sdc[q_lds]
    //  keys (learning): best-match keys u64[ncol], the learning loops' column
    //          records and new-source lists (LREC_WORDS), phase 2's key columns u16[ncol]
    //  frozen collection: u8 counters[fx_win], active cells u16[max_act_cells],
    //          block prefix u32[max_act_cells+1], list starts u32[max_act_cells],
    //          block -> list map u16[FX_OWN]
    //  trim flags (learning): u32[upd_cap]
    //  (the frozen tail is phase2_finish_ranked's, in the frozen collection's
    //  words: no finish arrays)
    size_t fin = frozen && !learn ? 0
                                  : (size_t)c.ncol + (size_t)(c.ncol + 1) / 2 + (size_t)c.ncol + 1 + 4 * (size_t)c.q_lds +
                                        (size_t)(c.q_lds + 1) / 2 + (size_t)c.nw;
    size_t keys = learn ? 2 * (size_t)c.ncol + LREC_WORDS + ((size_t)c.ncol + 1) / 2 : 0;
    size_t col = frozen ? (size_t)c.fx_win / 4 + 64 + (size_t)(c.max_act_cells + 1) / 2 + 2 * (size_t)c.max_act_cells +
                              1 + FX_OWN / 2
                        : 0;
    size_t trim = learn ? (size_t)c.upd_cap : 0;
    // the fused kernels' SP step, and the boosted-inhibition keys after it
    size_t spw = nosp ? 0 : align16(sizeof(SpShared)) / 4 + (c.sp_boost != 0.0f ? ((size_t)c.nw + 1) * 32 : 0) + SP_PLANE_WORDS;
    size_t u = fin;
    if (spw > u) u = spw;
    if (keys > u) u = keys;
    if (col > u) u = col;
    if (trim > u) u = trim;
    L.u_words = u;
    o = align16(o + u * 4);
    L.total = o;
    return L;
}


// ---------------------------------------------------------------------------
// workgroup helpers
__device__ __forceinline__ void wg_clear(uint32_t* p, int n) {
    if ((((uintptr_t)p) & 15) == 0 && (n & 3) == 0) {
        uint4* p4 = reinterpret_cast<uint4*>(p);
        for (int i = threadIdx.x; i < (n >> 2); i += TM_NT) p4[i] = make_uint4(0u, 0u, 0u, 0u);
    } else {
        for (int i = threadIdx.x; i < n; i += TM_NT) p[i] = 0;
    }
}
__device__ __forceinline__ void wg_copy(uint32_t* d, const uint32_t* s, int n) {
    for (int i = threadIdx.x; i < n; i += TM_NT) d[i] = s[i];
}
// sum over the workgroup (contains barriers; call uniformly)
__device__ __forceinline__ uint32_t wg_sum(TmSh* sh, uint32_t v) {
    v = wave_sum_u32(v);
    __syncthreads();
    if (lane_id() == 0) sh->red[wave_id()] = v;
    __syncthreads();
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < TM_NWAVES; w++) t += sh->red[w];
    __syncthreads();
    return t;
}
// Sum over the workgroup with ONE barrier: the waves add into one of three
// rotating LDS accumulators; after the barrier every thread reads it and
// thread 0 zeroes the slot the call after next uses (its last readers read it
// before this call's barrier).  tm_bind zeroes the slots; every thread counts
// the calls (t.nsum).  Call uniformly.
__device__ __forceinline__ uint32_t wg_sum1(Tm& t, uint32_t v);

// The same with one barrier, through its own slots of sh->red: callers must
// have passed another barrier since the previous call read them.
__device__ __forceinline__ uint32_t wg_excl_scan1(TmSh* sh, uint32_t v, uint32_t* total);

// exclusive prefix over the workgroup in thread order; *total gets the sum
__device__ __forceinline__ uint32_t wg_excl_scan(TmSh* sh, uint32_t v, uint32_t* total) {
    uint32_t incl = wave_incl_scan(v);
    __syncthreads();
    if (lane_id() == 63) sh->red[wave_id()] = incl;
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < TM_NWAVES; w++) {
        if (w < wave_id()) base += sh->red[w];
        tot += sh->red[w];
    }
    __syncthreads();
    *total = tot;
    return base + incl - v;
}

__device__ __forceinline__ uint32_t wg_excl_scan1(TmSh* sh, uint32_t v, uint32_t* total) {
    const uint32_t incl = wave_incl_scan(v);
    if (lane_id() == 63) sh->red[2 * TM_NWAVES + wave_id()] = incl;
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < TM_NWAVES; w++) {
        const uint32_t x = sh->red[2 * TM_NWAVES + w];
        if (w < (int)wave_id()) base += x;
        tot += x;
    }
    *total = tot;
    return base + incl - v;
}

__device__ __forceinline__ uint32_t wg_sum1(Tm& t, uint32_t v) {
    uint32_t* acc = t.sh->acc;
    const uint32_t k = t.nsum % 3u;
    v = wave_sum_u32(v);
    if (lane_id() == 0 && v) atomicAdd(&acc[k], v);
    __syncthreads();
    const uint32_t r = acc[k];
    if (threadIdx.x == 0) acc[(k + 2u) % 3u] = 0u;
    t.nsum++;
    return r;
}

__device__ __forceinline__ uint32_t col_of(const DevCfg& c, uint32_t cell) { return __umulhi(cell, c.kmagic); }
__device__ __forceinline__ uint32_t kmask(int K) { return K >= 32 ? 0xFFFFFFFFu : ((1u << K) - 1u); }

// Segment::dutyCycle(iteration, active, readOnly=false) on the pool entry
__device__ __forceinline__ float seg_dc_update(uint32_t* duty, uint32_t slot, uint32_t it, bool active) {
    uint32_t* d = duty + (size_t)slot * 3;
    float dc;
    if (it <= kDcTier[1]) {
        dc = (float)d[0] / (float)it;
        d[1] = __float_as_uint(dc);
        d[2] = it;
        return dc;
    }
    uint32_t age = it - d[2];
    float last = __uint_as_float(d[1]);
    if (age == 0 && !active) return last;
    float alpha = 0.0f;
    for (int t = 8; t > 0; t--) {
        if (it > kDcTier[t]) { alpha = kDcAlpha[t]; break; }
    }
    dc = pow_det((float)(1.0 - (double)alpha), age) * last;
    if (active) dc += alpha;
    d[1] = __float_as_uint(dc);
    d[2] = it;
    return dc;
}

// ---------------------------------------------------------------------------
// cell list of a bitmap (ascending) into dst; returns count (uniform)
__device__ __forceinline__ uint32_t wg_bitmap_list(Tm& t, const uint32_t* bm, uint32_t* dst32, uint16_t* dst16, uint32_t cap) {
    const int cw = t.c.cw;
    const int per = (cw + TM_NT - 1) / TM_NT;
    const int w0 = threadIdx.x * per;
    uint32_t cnt = 0;
    for (int k = 0; k < per; k++)
        if (w0 + k < cw) cnt += __popc(bm[w0 + k]);
    uint32_t total;
    uint32_t pos = wg_excl_scan(t.sh, cnt, &total);
    for (int k = 0; k < per; k++) {
        int w = w0 + k;
        if (w >= cw) break;
        for (uint32_t x = bm[w]; x; x &= x - 1) {
            uint32_t cell = (uint32_t)w * 32 + __ffs(x) - 1;
            if (pos < cap) {
                if (dst32) dst32[pos] = cell;
                if (dst16) dst16[pos] = (uint16_t)cell;
            }
            pos++;
        }
    }
    __syncthreads();
    return total;
}

// ---------------------------------------------------------------------------
// Inference
// _inferPhase1(activeColumns, useStartCells)
// prevP: the predicted state it reads (default infPredictedState(t-1); a
// backtrack replay passes the previous replay's infP directly)
__device__ __forceinline__ bool infer_phase1(Tm& t, const uint16_t* cols, int nA, bool use_start,
                                             const uint32_t* prevP = nullptr) {
    const int K = t.c.K;
    if (threadIdx.x == 0) {  // (collect_frozen lists the active cells column by column)
        t.sh->p1_off = (uint32_t)(reinterpret_cast<const char*>(cols) - reinterpret_cast<const char*>(t.sh));
        t.sh->p1_n = nA;
    }
    wg_clear(t.infA, t.c.cw);
    __syncthreads();
    uint32_t npc = 0;
    for (int a = threadIdx.x; a < nA; a += TM_NT) {
        uint32_t lo = (uint32_t)cols[a] * K;
        if (use_start) {
            bm_or_field(t.infA, lo, 1, 1u);
        } else {
            uint32_t f = bm_field(prevP ? prevP : t.infP1, lo, K);
            if (f) {
                bm_or_field(t.infA, lo, K, f);
                npc++;
            } else {
                bm_or_field(t.infA, lo, K, kmask(K));
            }
        }
    }
    npc = wg_sum1(t, npc);
    STAMP(t, SB_P1);
    return use_start || (double)npc >= 0.50 * (double)nA;
}

// collect slots of segments with >= thr synapses onto active cells of
// `state` by scanning the pool (learning-on form)
// Scan the segment pool (4 lanes per segment, 16 B of synapse sources each)
// against the cell bitmap `state`: for every slot, f(slot, meta, eligible,
// mask of synapses onto cells on in `state`) on all 4 lanes (mask reduced
// across them).  Only segments with elig(meta) load their rows.  SC_DEPTH
// batches of 64 segments are in flight per workgroup: meta loads of the
// batch first, then the row loads, so a pass over the pool costs two HBM
// round trips per SC_DEPTH x 64 segments.  SPEC (a scan whose every live
// segment is eligible: elig must then return true): the rows are loaded with
// the meta words, not after them -- one round trip per batch; rows of dead
// slots and lanes past a segment's synapses are loaded and ignored.  Returns
// this thread's bytes.
#ifndef SC_DEPTH
#define SC_DEPTH 8
#endif
// one segment's lane of a pool scan: the mask of its synapses (this lane's
// eight) onto cells on in `state`, OR-ed over the segment's four lanes
__device__ __forceinline__ uint32_t scan_seg_mask(const uint32_t* state, uint32_t cwm1, uint32_t sub, uint32_t m,
                                                  bool el, uint4 v, uint32_t& nb) {
    const uint32_t nsyn = meta_nsyn(m);
    uint32_t mask = 0;
    if (el && sub * 8u < nsyn) {
        nb += 16;
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        // all eight state words read unconditionally (one LDS round trip; a
        // per-synapse `j < nsyn &&` test made a branch and a wait per read),
        // entries past nsyn clamped into the bitmap and masked off afterwards
        uint32_t sw[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint32_t wi = (w[k >> 1] >> ((k & 1) * 16 + 5)) & 0x7FFu;
            sw[k] = state[wi < cwm1 ? wi : cwm1];
        }
        uint32_t bits = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) bits |= ((sw[k] >> ((w[k >> 1] >> ((k & 1) * 16)) & 31u)) & 1u) << k;
        const uint32_t left = nsyn - sub * 8u;
        mask = (bits & (left >= 8u ? 0xFFu : (1u << left) - 1u)) << (sub * 8u);
    }
    // OR over the segment's four lanes: DPP quad permutes (a __shfl_xor is a
    // ds_bpermute, an LDS round trip)
    mask |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mask, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    mask |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mask, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    return mask;
}

template <bool SPEC = false, typename E, typename F>
__device__ __forceinline__ uint32_t scan_pool(Tm& t, const uint32_t* state, E elig, F f) {
    const uint32_t hwm = t.sh->hwm;
    COUNT(t, SC_NSCAN, 1);
    COUNT(t, SC_SCANSLOTS, hwm);
    const uint32_t g = threadIdx.x >> 2, sub = threadIdx.x & 3;
    const uint32_t cwm1 = (uint32_t)t.c.cw - 1u;
    uint32_t nb = 0;
    for (uint32_t base = 0; base < hwm; base += SC_DEPTH * (TM_NT / 4)) {
        uint32_t m[SC_DEPTH];
#pragma unroll
        for (int d = 0; d < SC_DEPTH; d++) {
            const uint32_t slot = base + d * (TM_NT / 4) + g;
            m[d] = slot < hwm ? t.meta[slot] : 0u;
        }
        uint4 v[SC_DEPTH];
        bool el[SC_DEPTH];
#pragma unroll
        for (int d = 0; d < SC_DEPTH; d++) {
            const uint32_t slot = base + d * (TM_NT / 4) + g;
            if (SPEC) {
                v[d] = slot < hwm ? *reinterpret_cast<const uint4*>(t.src + (size_t)slot * HTM_MAXSYN + sub * 8)
                                  : make_uint4(0u, 0u, 0u, 0u);
            } else {
                el[d] = meta_live(m[d]) && elig(m[d]);
                v[d] = make_uint4(0u, 0u, 0u, 0u);
                if (el[d] && sub * 8u < meta_nsyn(m[d]))
                    v[d] = *reinterpret_cast<const uint4*>(t.src + (size_t)slot * HTM_MAXSYN + sub * 8);
            }
        }
        if (SPEC) {
#pragma unroll
            for (int d = 0; d < SC_DEPTH; d++) el[d] = meta_live(m[d]) && elig(m[d]);
        }
#pragma unroll
        for (int d = 0; d < SC_DEPTH; d++) {
            const uint32_t slot = base + d * (TM_NT / 4) + g;
            if (slot < hwm && sub == 0) nb += 4;
            const uint32_t mask = scan_seg_mask(state, cwm1, sub, m[d], el[d], v[d], nb);
            f(slot, m[d], el[d], mask);
        }
    }
    return nb;
}

// scan_pool<true> against two cell bitmaps at once: f(slot, meta, live,
// mask onto `state`, mask onto `state2`) -- one pass over the pool for two
// counts (an inference phase 2 and the previous step's deferred learn phase 2,
// collect_scan).  Returns this thread's bytes (the rows counted once).
template <typename F>
__device__ __forceinline__ uint32_t scan_pool2(Tm& t, const uint32_t* state, const uint32_t* state2, F f) {
    const uint32_t hwm = t.sh->hwm;
    COUNT(t, SC_NSCAN, 1);
    COUNT(t, SC_SCANSLOTS, hwm);
    const uint32_t g = threadIdx.x >> 2, sub = threadIdx.x & 3;
    const uint32_t cwm1 = (uint32_t)t.c.cw - 1u;
    uint32_t nb = 0, nb2 = 0;
    for (uint32_t base = 0; base < hwm; base += SC_DEPTH * (TM_NT / 4)) {
        uint32_t m[SC_DEPTH];
        uint4 v[SC_DEPTH];
#pragma unroll
        for (int d = 0; d < SC_DEPTH; d++) {
            const uint32_t slot = base + d * (TM_NT / 4) + g;
            m[d] = slot < hwm ? t.meta[slot] : 0u;
            v[d] = slot < hwm ? *reinterpret_cast<const uint4*>(t.src + (size_t)slot * HTM_MAXSYN + sub * 8)
                              : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int d = 0; d < SC_DEPTH; d++) {
            const uint32_t slot = base + d * (TM_NT / 4) + g;
            if (slot < hwm && sub == 0) nb += 4;
            const bool el = meta_live(m[d]);
            const uint32_t mask = scan_seg_mask(state, cwm1, sub, m[d], el, v[d], nb);
            const uint32_t mask2 = scan_seg_mask(state2, cwm1, sub, m[d], el, v[d], nb2);
            f(slot, m[d], el, mask, mask2);
        }
    }
    return nb;
}

// A scan whose eligible segments are few (learn phase 1: the segments of a
// handful of flagged columns): the meta words are streamed SCS_META per thread
// per round trip and the eligible slots listed in LDS (elist[0] the count,
// elist[1..ecap] the slots), then only their rows are read, four lanes per
// segment -- two or three round trips for the pool instead of two per
// SC_DEPTH x 64 slots.  f(slot, meta, true, mask) for the eligible slots only
// (the callers ignore ineligible ones).  Sets *overflow (uniform) and calls no
// f when more than ecap slots are eligible: the caller then runs scan_pool.
// Contains barriers: call uniformly.  Returns this thread's bytes.
#ifndef SCS_META
#define SCS_META 16
#endif
template <typename E, typename F>
__device__ __forceinline__ uint32_t scan_pool_sparse(Tm& t, const uint32_t* state, E elig, F f, uint32_t* elist,
                                                     uint32_t ecap, bool* overflow) {
    const uint32_t hwm = t.sh->hwm;
    COUNT(t, SC_NSCAN, 1);
    COUNT(t, SC_SCANSLOTS, hwm);
    uint32_t nb = 0;
    if (threadIdx.x == 0) elist[0] = 0u;
    __syncthreads();
    for (uint32_t base = 0; base < hwm; base += SCS_META * TM_NT) {
        uint32_t m[SCS_META];
#pragma unroll
        for (int d = 0; d < SCS_META; d++) {
            const uint32_t slot = base + d * TM_NT + threadIdx.x;
            m[d] = slot < hwm ? t.meta[slot] : 0u;
        }
#pragma unroll
        for (int d = 0; d < SCS_META; d++) {
            const uint32_t slot = base + d * TM_NT + threadIdx.x;
            if (slot < hwm) nb += 4;
            if (meta_live(m[d]) && elig(m[d])) {
                const uint32_t k = atomicAdd(&elist[0], 1u);
                if (k < ecap) elist[1 + k] = slot;
            }
        }
    }
    __syncthreads();
    const uint32_t ne = elist[0];
    *overflow = ne > ecap;
    if (ne > ecap) return nb;
    const uint32_t g = threadIdx.x >> 2, sub = threadIdx.x & 3;
    const uint32_t cwm1 = (uint32_t)t.c.cw - 1u;
    for (uint32_t e0 = 0; e0 < ne; e0 += 2u * (TM_NT / 4)) {  // (two segments per quad in flight)
        uint32_t sl[2], mm[2];
        uint4 v[2];
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const uint32_t e = e0 + (uint32_t)u * (TM_NT / 4) + g;
            sl[u] = e < ne ? elist[1 + e] : 0u;
            mm[u] = e < ne ? t.meta[sl[u]] : 0u;
        }
#pragma unroll
        for (int u = 0; u < 2; u++)
            v[u] = sub * 8u < meta_nsyn(mm[u])
                       ? *reinterpret_cast<const uint4*>(t.src + (size_t)sl[u] * HTM_MAXSYN + sub * 8)
                       : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const uint32_t e = e0 + (uint32_t)u * (TM_NT / 4) + g;
            const bool in = e < ne;
            const uint32_t mask = scan_seg_mask(state, cwm1, sub, mm[u], in, v[u], nb);
            if (in) f(sl[u], mm[u], true, mask);
        }
    }
    return nb;
}

// collect slots of segments with >= thr synapses onto active cells of
// `state` by scanning the pool (learning-on form)
// The first pool scan of a learning step also counts the previous step's
// deferred learn phase 2 (lp2_finish): every live segment's synapses onto
// lrnActiveState(t-1), its key (activity, cellInColumn, first slot) kept per
// column in Tm::lkey -- the pool between the two is the same (the deferred
// phase writes no segment, and an inference phase 2 writes only dutyCycle
// records, which it does not read).
__device__ __forceinline__ void collect_scan(Tm& t, const uint32_t* state, int thr) {
    const DevCfg& c = t.c;
    const uint32_t sub = threadIdx.x & 3;
    // a qualifying segment's slot to q1 and its active-synapse mask to q2
    // (pass 1 reads the mask instead of the segment's row again)
    auto qual = [&](uint32_t slot, bool el, uint32_t mask) {
        if (el && sub == 0 && __popc(mask) >= (uint32_t)thr) {
            const uint32_t i = (uint32_t)atomicAdd(&t.sh->qn, 1);
            if (i < (uint32_t)c.q_cap) {
                t.q1[i] = slot;
                t.q2[i] = mask;
            }
        }
    };
    uint32_t nb;
    const bool lp2 = t.lkey != nullptr && t.sh->lp2p && !t.sh->lp2s;  // (LDS flags: uniform)
    if (lp2) {
        nb = scan_pool2(t, state, t.lrnA1, [&](uint32_t slot, uint32_t m, bool el, uint32_t mask, uint32_t mask2) {
            qual(slot, el, mask);
            const uint32_t n2 = __popc(mask2);
            if (el && sub == 0 && n2 >= (uint32_t)c.act_thr) {
                const uint32_t cell = meta_cell(m), col = col_of(c, cell);
                // scan_best's key order in 32 bits (slots < 2^21, DevCfg::lp2_defer)
                atomicMax(&t.lkey[col], (n2 << 26) | ((cell - col * c.K) << 21) | (0x1FFFFFu - slot));
            }
        });
    } else {
        nb = scan_pool<true>(t, state, [](uint32_t) { return true; },
                             [&](uint32_t slot, uint32_t, bool el, uint32_t mask) { qual(slot, el, mask); });
    }
    nb = wg_sum(t.sh, nb);
    if (threadIdx.x == 0) {
        t.sh->bytes += nb;
        if (lp2) t.sh->lp2s = 1;  // (every thread has read the flags: wg_sum's barriers)
    }
    STAMP(t, SB_SCAN);
}

// one 16-byte block of a frozen out-list: 8 window-relative u16 ranks,
// 0xFFFF = padding; bump the rank's u8 counter with non-returning LDS
// atomics (padding is counted branch-free into a per-lane spare word past
// the counters, cnt[dummy + lane], so sink updates never collide)
__device__ __forceinline__ void fx_count_block(uint32_t* cnt, uint4 v, uint32_t dummy) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int h = 0; h < 8; h++) {
        const uint32_t rel = (w[h >> 1] >> ((h & 1) * 16)) & 0xFFFFu;
        atomicAdd(&cnt[rel != 0xFFFFu ? (rel >> 2) : dummy + (threadIdx.x & 63)], 1u << ((rel & 3) * 8));
    }
}

// block -> list map of the blocks [lo, hi): owner[x - lo] = the list holding block x
__device__ __forceinline__ void fx_owner_map(const uint32_t* pstart, uint32_t na, uint32_t lo, uint32_t hi,
                                             uint16_t* owner) {
    for (uint32_t k = threadIdx.x; k < na; k += TM_NT) {
        const uint32_t a = pstart[k] > lo ? pstart[k] : lo;
        const uint32_t z = pstart[k + 1] < hi ? pstart[k + 1] : hi;
        for (uint32_t x = a; x < z; x++) owner[x - lo] = (uint16_t)k;
    }
}

// Stream the 16-byte blocks of lists k < na -- list k is the block range
// [plo[k], plo[k] + n_k) of ent, pstart the exclusive prefix of n_k with
// pstart[na] = B -- and count every u16 entry into the u8 counters.  Per
// pass of FX_OWN blocks every thread issues its FX_DEPTH block loads (their
// lists from a block -> list map in LDS) before counting any, so one HBM
// round trip covers FX_OWN blocks whatever the list lengths; the next pass's
// map is built while those loads are in flight (a barrier once every thread
// has read the map for its addresses -- LDS reads only: the loads stay in
// flight), not before the next loads.  The first pass's map is the
// caller's (collect_frozen writes it with the list starts, before its
// barrier), or, `sep` (DevCfg::fx_own_sep), built here as in round 5.
__device__ __forceinline__ void fx_stream(const uint4* ent, const uint32_t* plo, const uint32_t* pstart, uint32_t na,
                                          uint32_t B, uint32_t* cnt, uint16_t* owner, uint32_t dummy, bool sep,
                                          TmSh* shp = nullptr) {
    if (B == 0) return;
    if (sep) {
        fx_owner_map(pstart, na, 0u, B < FX_OWN ? B : FX_OWN, owner);
        __syncthreads();
    }
    STAMP_SH(shp, SB_OWNER);
    for (uint32_t lo = 0; lo < B; lo += FX_OWN) {
        const uint32_t hi = B - lo < FX_OWN ? B : lo + FX_OWN;
        uint4 v[FX_DEPTH];
#pragma unroll
        for (int j = 0; j < FX_DEPTH; j++) {
            const uint32_t x = lo + j * TM_NT + threadIdx.x;
            v[j] = make_uint4(~0u, ~0u, ~0u, ~0u);
            if (x < hi) {
                const uint32_t k = owner[x - lo];
                v[j] = ent[plo[k] + (x - pstart[k])];
            }
        }
        if (hi < B) {
            __syncthreads();  // (every thread's map reads done)
            fx_owner_map(pstart, na, hi, B - hi < FX_OWN ? B : hi + FX_OWN, owner);
        }
        STAMP_SH(shp, SB_OWNER);
#pragma unroll
        for (int j = 0; j < FX_DEPTH; j++) {
#ifdef HTM_STAMPS
            if (j == 0 && threadIdx.x == 0) {
                __builtin_amdgcn_s_waitcnt(0);  // diagnostic: charge the block loads' latency to SB_SLOAD
                STAMP_SH(shp, SB_SLOAD);
            }
#endif
            fx_count_block(cnt, v[j], dummy);
        }
        STAMP_SH(shp, SB_COUNT);
        __syncthreads();
    }
}

// Every counter byte >= thr (1..127) of cnt[0 .. nbytes), nbytes a multiple
// of 16: f(index).  Counters never exceed 32, so byte + (128 - thr) sets bit
// 7 exactly when byte >= thr, without carries between bytes.
template <typename F>
__device__ __forceinline__ void fx_qualify(const uint32_t* cnt, uint32_t nbytes, uint32_t thr, F f) {
    const uint32_t add = 0x01010101u * (128u - thr);
    const uint4* c4 = reinterpret_cast<const uint4*>(cnt);
    for (uint32_t i = threadIdx.x; i < nbytes / 16; i += TM_NT) {
        const uint4 x = c4[i];
        const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int q = 0; q < 4; q++) {
            for (uint32_t m = (w[q] + add) & 0x80808080u; m; m &= m - 1) f(16 * i + 4 * q + ((__ffs(m) - 1) >> 3));
        }
    }
}

// The counter bytes >= thr of the nquads 16-byte quads at cnt, as ranks
// base + index, appended to dst at sh->qn in ASCENDING order (each thread
// sweeps a contiguous run of quads; one workgroup scan places the runs), so
// the qualifying list comes out in rank = (cell, creation) order.  Counters
// never exceed 32 (see fx_qualify).  Contains barriers: call uniformly.
#ifndef FX_CQ
#define FX_CQ 16  // counter quads one thread sweeps (W <= 16 x 16 x TM_NT bytes)
#endif

__device__ __forceinline__ void fx_collect_ordered(const uint32_t* cnt, uint32_t nquads, uint32_t thr, uint32_t base,
                                                   TmSh* sh, uint32_t* dst, uint32_t qcap) {
    const uint32_t add = 0x01010101u * (128u - thr);
    const uint4* c4 = reinterpret_cast<const uint4*>(cnt);
    const uint32_t per = (nquads + TM_NT - 1) / TM_NT;  // <= FX_CQ (fx_win <= 64512)
    const uint32_t q0 = threadIdx.x * per;
    // one sweep: every quad of the thread's run loaded at once; the hits of a
    // quad counted from its masked words (byte + (128 - thr) sets bit 7
    // exactly when byte >= thr), and only a bit per quad kept -- hits are
    // rare (a few hundred of the window's ranks), so the quads that have
    // them are read again to place them
    uint32_t any = 0, mine = 0;
    const uint32_t nq = q0 < nquads ? (nquads - q0 < per ? nquads - q0 : per) : 0u;
    for (uint32_t i0 = 0; i0 < nq; i0 += 4) {  // (four quads' reads in flight)
        uint4 x[4];
#pragma unroll
        for (int u = 0; u < 4; u++) x[u] = i0 + u < nq ? c4[q0 + i0 + u] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint32_t h = __popc((x[u].x + add) & 0x80808080u) + __popc((x[u].y + add) & 0x80808080u) +
                               __popc((x[u].z + add) & 0x80808080u) + __popc((x[u].w + add) & 0x80808080u);
            mine += h;
            any |= (h ? 1u : 0u) << (i0 + u);
        }
    }
    // exclusive prefix over the workgroup in thread order (one barrier)
    const uint32_t qn0 = (uint32_t)sh->qn;  // thread 0 updates it only after the barrier
    const uint32_t incl = wave_incl_scan(mine);
    if (lane_id() == 63) sh->red[TM_NWAVES + wave_id()] = incl;
    __syncthreads();
    uint32_t pos = qn0 + incl - mine, tot = 0;
#pragma unroll
    for (int v = 0; v < TM_NWAVES; v++) {
        const uint32_t x = sh->red[TM_NWAVES + v];
        if (v < (int)wave_id()) pos += x;
        tot += x;
    }
    for (uint32_t a = any; a; a &= a - 1) {
        const uint32_t i = __ffs(a) - 1;
        const uint4 x = c4[q0 + i];
        const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
            for (uint32_t m = (w[j] + add) & 0x80808080u; m; m &= m - 1) {
                const uint32_t b = (uint32_t)(__ffs(m) - 1) >> 3;  // byte of the word
                if (pos < qcap) dst[pos] = base + 16 * (q0 + i) + 4 * j + b;
                pos++;
            }
        }
    }
    if (threadIdx.x == 0) sh->qn = (int32_t)(qn0 + tot);
}

// zero n 16-byte quads of LDS
__device__ __forceinline__ void wg_clear4(uint32_t* p, uint32_t nquads) {
    uint4* p4 = reinterpret_cast<uint4*>(p);
    for (uint32_t i = threadIdx.x; i < nquads; i += TM_NT) p4[i] = make_uint4(0u, 0u, 0u, 0u);
}

// learning-off form: forward propagation over the frozen cell->segment index
// (what Cells4's _outSynapses does).  Pass 0 counts CONNECTED active
// synapses of the predictive-capable segments (pid lists; counter >=
// activationThreshold predicts the segment's cell); then, per window of the
// slot space, all active synapses of every segment (counter >= thr: the
// segment qualifies for the confidence sum).
// what collect_frozen counts: the pid pass and every rank window, the pid pass
// only, or the rank windows only (listing the active cells, or reusing the
// list a pid-only call left in U)
enum { FX_ALL = 0, FX_PID = 1, FX_WIN = 2, FX_WIN_REUSE = 3 };

// win >= 0 (FX_WIN only): count that one rank window (the flush's per-window jobs)
__device__ __forceinline__ void collect_frozen(Tm& t, int thr, int mode = FX_ALL, int win = -1) {
    const DevCfg& c = t.c;
    TmSh* sh = t.sh;
    const uint32_t W = (uint32_t)c.fx_win;
    const uint32_t mac = (uint32_t)c.max_act_cells;
    uint32_t* cnt = t.U;  // W / 4 counter words + 64 spare (padding sinks)
    const uint32_t dummy = W / 4;
    uint16_t* cells = reinterpret_cast<uint16_t*>(t.U + W / 4 + 64);
    uint32_t* pstart = t.U + W / 4 + 64 + (mac + 1) / 2;
    uint32_t* plo = pstart + mac + 1;
    uint16_t* owner = reinterpret_cast<uint16_t*>(plo + mac);
    uint32_t na;
    if (mode == FX_WIN_REUSE) {
        na = (uint32_t)sh->fx_na;
    } else if (sh->p1_n >= 0 && sh->p1_n <= 64) {
        // infA is phase 1's: each active column's cells (ascending columns,
        // ascending cells = the bitmap's order), listed by wave 0, one lane per column
        if (wave_id() == 0) {
            const int a = lane_id();
            const int K = c.K;
            const int p1n = sh->p1_n;
            const uint16_t* p1c = reinterpret_cast<const uint16_t*>(reinterpret_cast<const char*>(sh) + sh->p1_off);
            const uint32_t col = a < p1n ? p1c[a] : 0u;
            const uint32_t f = a < p1n ? bm_field(t.infA, col * (uint32_t)K, (uint32_t)K) : 0u;
            const uint32_t n1 = (uint32_t)__popc(f);
            const uint32_t incl = wave_incl_scan(n1);
            uint32_t pos = incl - n1;
            for (uint32_t x = f; x; x &= x - 1) {
                if (pos < mac) cells[pos] = (uint16_t)(col * (uint32_t)K + (uint32_t)(__ffs(x) - 1));
                pos++;
            }
            const uint32_t tot = lane63(incl);
            if (a == 0) sh->fx_na = (int32_t)(tot < mac ? tot : mac);
        }
        __syncthreads();
        na = (uint32_t)sh->fx_na;
    } else {
        const uint32_t nact = wg_bitmap_list(t, t.infA, nullptr, cells, mac);
        na = nact < mac ? nact : mac;
        if (threadIdx.x == 0) sh->fx_na = (int32_t)na;
    }
    const uint32_t nr = t.nr;
    STAMP(t, SB_LIST);
    COUNT(t, SC_NACT, na);
    const uint32_t nw = (nr + W - 1) / W;
    const bool pid_ok = t.np <= (uint32_t)c.fx_pcap;
    const uint32_t per = (na + TM_NT - 1) / TM_NT;  // <= FX_MAXPER (na <= 64 x 32)
    const uint32_t k0 = threadIdx.x * per;
    uint32_t nblk = 0;
    // block ranges of this thread's cells in pass w: the first FX_PF of them
    // loaded one pass ahead (registers), any further ones (more than
    // FX_PF x TM_NT active cells: K > 12) loaded in the pass
    constexpr uint32_t FX_PF = 2;
    uint32_t olo[FX_PF], ohi[FX_PF];
    auto off_idx = [&](int w, uint32_t k) {
        return FX_LIST(c, w, cells[k]);
    };
    auto load_offsets = [&](int w) {
#pragma unroll
        for (uint32_t j = 0; j < FX_PF; j++) {
            const uint32_t k = k0 + j;
            if (j < per && k < na) {
                const size_t idx = off_idx(w, k);
                olo[j] = t.fxoff[idx];
                ohi[j] = t.fxoff[idx + 1];
            }
        }
    };
    const int w_first = (pid_ok && t.np > 0 && mode != FX_WIN && mode != FX_WIN_REUSE) ? -1 : win >= 0 ? win : 0;
    const int w_end = mode == FX_PID ? 0 : win >= 0 ? (win < (int)nw ? win + 1 : win) : (int)nw;
    if (w_first < w_end) load_offsets(w_first);
    // this thread's lists of pass w: plo = the first block, pstart = the block
    // count (the exclusive prefix replaces it once the workgroup total is
    // known); returns their block total.  olo/ohi hold pass w's first FX_PF
    // offsets (loaded a pass ahead); pass w + 1's are requested here.
    auto store_lists = [&](int w) {
        uint32_t lsum = 0;
#pragma unroll
        for (uint32_t j = 0; j < FX_PF; j++) {
            const uint32_t k = k0 + j;
            if (j < per && k < na) {
                plo[k] = olo[j];
                pstart[k] = ohi[j] - olo[j];
                lsum += ohi[j] - olo[j];
            }
        }
        for (uint32_t j = FX_PF; j < per; j++) {
            const uint32_t k = k0 + j;
            if (k >= na) break;
            const size_t idx = off_idx(w, k);
            const uint32_t lo = t.fxoff[idx], hi = t.fxoff[idx + 1];
            plo[k] = lo;
            pstart[k] = hi - lo;
            lsum += hi - lo;
        }
        if (w + 1 < w_end) load_offsets(w + 1);
        return lsum;
    };
    // the lists' starts from this thread's exclusive prefix pos, and
    // fx_stream's first block -> list map from the starts in hand
    const bool own_sep = c.fx_own_sep != 0;
    auto place_lists = [&](uint32_t pos, uint32_t B) {
        for (uint32_t j = 0; j < per; j++) {
            const uint32_t k = k0 + j;
            if (k >= na) break;
            const uint32_t n = pstart[k];
            pstart[k] = pos;
            if (!own_sep) {
                const uint32_t e = pos + n < FX_OWN ? pos + n : FX_OWN;
                for (uint32_t x = pos; x < e; x++) owner[x] = (uint16_t)k;
            }
            pos += n;
        }
        if (threadIdx.x == 0) pstart[na] = B;
    };
    for (int w = w_first; w < w_end; w++) {
        // counters cover the pids (pass -1) or this window's ranks
        const uint32_t span = w < 0 ? t.np : (nr - (uint32_t)w * W < W ? nr - (uint32_t)w * W : W);
        const uint32_t nbytes = (span + 15u) & ~15u;
        const uint32_t lsum = store_lists(w);
        uint32_t B;
        const uint32_t pos = wg_excl_scan1(sh, lsum, &B);
        place_lists(pos, B);
        wg_clear4(cnt, nbytes / 16);
        __syncthreads();
        nblk += B;
        STAMP(t, SB_WINPRE);
        COUNT(t, SC_WIN, 1);
        COUNT(t, SC_BLK, B);
        fx_stream(t.fxent, plo, pstart, na, B, cnt, owner, dummy, own_sep, sh);
        STAMP(t, SB_STREAM);
        if (w >= 0) {
            fx_collect_ordered(cnt, nbytes / 16, (uint32_t)thr, (uint32_t)w * W, sh, t.q1, (uint32_t)c.q_cap);
        } else {
            // pid counter >= activationThreshold: the segment's cell is predicted
            const uint32_t np = t.np;
            uint32_t* infP = t.infP;
            const uint16_t* pcell = t.fxpcell;
            fx_qualify(cnt, nbytes, (uint32_t)c.act_thr, [&](uint32_t pid) {
                if (pid < np) {
                    const uint32_t cell = pcell[pid];
                    atomicOr(&infP[cell >> 5], 1u << (cell & 31));
                }
            });
            __syncthreads();
        }
        STAMP(t, SB_QSCAN);
    }
    // out-list blocks + the two block offsets of every (active cell, pass)
    if (threadIdx.x == 0 && w_end > w_first) sh->bytes += 16ull * nblk + 8ull * na * (uint32_t)(w_end - w_first);
}

// Pass 1 of _inferPhase2 over the qn qualifying segments in t.q1: the
// predicted cells (rows path; the frozen pid path predicted them while
// counting), the dutyCycle() each contributes, emit(k, slot, cell, dc).
// Returns this thread's algorithmic bytes.
// connected synapses of pool slot `slot` onto active cells (>= activationThreshold
// predicts the segment's cell); adds the bytes read to nb
__device__ __forceinline__ uint32_t seg_connected_activity(Tm& t, uint32_t slot, uint32_t nsyn, uint32_t& nb) {
    nb += 4u + 16u * ((nsyn + 7u) / 8u);
    const uint32_t cm = t.conn[slot];
    const uint4* row = reinterpret_cast<const uint4*>(t.src + (size_t)slot * HTM_MAXSYN);
    const uint32_t cwm1 = (uint32_t)t.c.cw - 1u;
    // the row's used quads loaded before any is read (one round trip), the
    // state words read unconditionally (entries past nsyn clamped, masked below)
    uint4 v[4];
#pragma unroll
    for (int q = 0; q < 4; q++) v[q] = (uint32_t)q * 8u < nsyn ? row[q] : make_uint4(0u, 0u, 0u, 0u);
    uint32_t bits = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint32_t w[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
        for (int k2 = 0; k2 < 8; k2++) {
            const uint32_t sid = (w[k2 >> 1] >> ((k2 & 1) * 16)) & 0xFFFFu;
            const uint32_t wi = sid >> 5;
            bits |= ((t.infA[wi < cwm1 ? wi : cwm1] >> (sid & 31)) & 1u) << (q * 8 + k2);
        }
    }
    return (uint32_t)__popc(bits & cm & (nsyn >= 32u ? 0xFFFFFFFFu : (1u << nsyn) - 1u));
}

template <bool FROZEN, typename F>
__device__ __forceinline__ uint32_t phase2_pass1(Tm& t, uint32_t qn, F emit) {
    const DevCfg& c = t.c;
    TmSh* sh = t.sh;
    uint32_t nb = 0;
    // frozen: the cells the pid counters did not predict (more pids than
    // fx_pcap) come from the segments' synapse rows
    const bool rows = FROZEN && t.np > (uint32_t)c.fx_pcap;
    // frozen index: cell and the (frozen-iteration) dutyCycle of the segment
    // of rank q1[k].  Four entries per thread per round: their ranks, then
    // their records, are loaded before any is used (two round trips per four
    // instead of two per entry).  The dutyCycle() state update is a store of
    // the value it returns; the value read never comes from the pool's record,
    // which streams sharing a model (fleet) may be refreshing.
    constexpr uint32_t P1B = 4;
    for (uint32_t k0 = threadIdx.x; k0 < qn && FROZEN; k0 += P1B * TM_NT) {
        uint32_t rk[P1B];
        uint2 rc[P1B];
#pragma unroll
        for (uint32_t u = 0; u < P1B; u++) {
            const uint32_t k = k0 + u * TM_NT;
            rk[u] = k < qn ? t.q1[k] : 0u;
        }
#pragma unroll
        for (uint32_t u = 0; u < P1B; u++) {
            const uint32_t k = k0 + u * TM_NT;
            rc[u] = k < qn ? t.fxrec[rk[u]] : make_uint2(FX_FRESH, 0u);
        }
#pragma unroll
        for (uint32_t u = 0; u < P1B; u++) {
            const uint32_t k = k0 + u * TM_NT;
            if (k >= qn) break;
            const uint32_t rank = rk[u];
            const uint2 rec = rc[u];
            const uint32_t cell = rec.x & 0xFFFFu;
            // the dutyCycle() state write stores the same value every time while
            // the iteration counter is frozen: only the first one after the index
            // build changes the record (FX_FRESH marks it done, or never needed)
            uint32_t slot = ~0u;
            if (!(rec.x & FX_FRESH) || rows) {
                slot = t.fxrslot[rank];
                nb += 4u;
            }
            if (!(rec.x & FX_FRESH)) {
                t.duty[(size_t)slot * 3 + 1] = rec.y;
                t.duty[(size_t)slot * 3 + 2] = sh->lrn_iter;
                atomicOr(const_cast<uint32_t*>(&t.fxrec[rank].x), FX_FRESH);
                nb += 8u;
            }
            nb += 8u;
            if (rows) {
                const uint32_t nsyn = meta_nsyn(t.meta[slot]);
                if (seg_connected_activity(t, slot, nsyn, nb) >= (uint32_t)c.act_thr)
                    atomicOr(&t.infP[cell >> 5], 1u << (cell & 31));
                nb += 4u;
            }
            emit(k, rank, cell, __uint_as_float(rec.y));
        }
    }
    for (uint32_t k = threadIdx.x; k < qn && !FROZEN; k += TM_NT) {
        // pool scan (collect_scan): the slot and the mask of its synapses onto
        // active cells; connected ones = mask & the connected-synapse mask
        const uint32_t slot = t.q1[k], amask = t.q2[k];
        const uint32_t m = t.meta[slot], cm = t.conn[slot];
        const uint32_t cell = meta_cell(m), nsyn = meta_nsyn(m);
        // slot + mask + meta + conn + duty-cycle record read and written
        nb += 4u + 4u + 4u + 4u + 12u + 8u;
#ifdef HTM_PASS1_ROWS  // (A/B builds: the row read again, round 5)
        (void)amask;
        (void)cm;
        if (seg_connected_activity(t, slot, nsyn, nb) >= (uint32_t)c.act_thr)
#else
        if ((uint32_t)__popc(amask & cm & (nsyn >= 32u ? 0xFFFFFFFFu : (1u << nsyn) - 1u)) >= (uint32_t)c.act_thr)
#endif
            atomicOr(&t.infP[cell >> 5], 1u << (cell & 31));
        emit(k, slot, cell, seg_dc_update(t.duty, slot, sh->lrn_iter, false));
    }
    return nb;
}

// numPredictedCols: columns with a predicted cell (uniform; has barriers)
__device__ __forceinline__ uint32_t count_predicted_cols(Tm& t) {
    const DevCfg& c = t.c;
    uint32_t n = 0;
    for (int col = threadIdx.x; col < c.ncol; col += TM_NT)
        if (bm_field(t.infP, (uint32_t)col * c.K, c.K)) n++;
    return wg_sum1(t, n);
}

// Tail of _inferPhase2 for qn <= q_lds (<= 1024) qualifying segments: the
// keys col:12 | cellInColumn:5 | slot:27 | k:10 are bitonic-sorted in LDS,
// each column's confidence is summed over its run in that order -- NuPIC's
// (column, cell, segment) order -- and the normaliser is folded over the
// columns in ascending order, so the float32 results are bit-identical to
// the oracle.  Returns numPredictedCols.
template <bool FROZEN>
__device__ __forceinline__ uint32_t phase2_finish_sorted(Tm& t, uint32_t qn) {
    const DevCfg& c = t.c;
    TmSh* sh = t.sh;
    const int K = c.K;
    const uint32_t ql = (uint32_t)c.q_lds;
    uint64_t* qk = reinterpret_cast<uint64_t*>(t.U);     // [ql] keys, sorted in place
    float* qd = reinterpret_cast<float*>(t.U + 2 * ql);  // [ql] dutyCycle by pass-1 index k
    float* rs = reinterpret_cast<float*>(t.U + 3 * ql);  // [ql] run sums at run heads, -1 elsewhere
    uint32_t nb = phase2_pass1<FROZEN>(t, qn, [&](uint32_t k, uint32_t slot, uint32_t cell, float dc) {
        const uint32_t col = col_of(c, cell);
        qk[k] = ((uint64_t)col << 42) | ((uint64_t)(cell - col * K) << 37) | ((uint64_t)slot << 10) | k;
        qd[k] = dc;
    });
    uint32_t n2 = 1;  // pad to a power of two with +inf keys
    while (n2 < qn) n2 <<= 1;
    for (uint32_t k = qn + threadIdx.x; k < n2; k += TM_NT) qk[k] = ~0ull;
    nb = wg_sum(sh, nb);
    if (threadIdx.x == 0) sh->bytes += nb;
    STAMP(t, SB_FIN1);
    COUNT(t, SC_QN, qn);
    COUNT(t, SC_P2, 1);
    for (uint32_t size = 2; size <= n2; size <<= 1) {
        for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
            for (uint32_t i = threadIdx.x; i < n2 / 2; i += TM_NT) {
                const uint32_t lo = 2 * i - (i & (stride - 1));
                const uint32_t hi = lo + stride;
                const uint64_t a = qk[lo], b = qk[hi];
                if ((a > b) == ((lo & size) == 0)) {
                    qk[lo] = b;
                    qk[hi] = a;
                }
            }
            __syncthreads();
        }
    }
    STAMP(t, SB_SORT);
    // run heads sum their column in order; -1 marks the other entries
    for (uint32_t k = threadIdx.x; k < qn; k += TM_NT) {
        const uint32_t col = (uint32_t)(qk[k] >> 42);
        if (k > 0 && (uint32_t)(qk[k - 1] >> 42) == col) {
            rs[k] = -1.0f;
            continue;
        }
        float sum = 0.0f;
        for (uint32_t j = k; j < qn && (uint32_t)(qk[j] >> 42) == col; j++) sum += qd[qk[j] & 1023u];
        t.colconf[col] = sum;
        rs[k] = sum;
    }
    __syncthreads();
    STAMP(t, SB_SUMS);
    // normaliser: sequential sum over the nonzero columns, ascending (the
    // -1 markers of non-head entries add +0.0f, which leaves the sum exact)
    if (threadIdx.x == 0) {
        float tot = 0.0f;
#pragma unroll 8
        for (uint32_t k = 0; k < qn; k++) tot += fmaxf(rs[k], 0.0f);
        sh->tf[0] = tot;
    }
    __syncthreads();
    const float tot = sh->tf[0];
    if (tot > 0.0f)
        for (uint32_t k = threadIdx.x; k < qn; k += TM_NT)
            if (rs[k] >= 0.0f) t.colconf[(uint32_t)(qk[k] >> 42)] = rs[k] / tot;
    const uint32_t npcol = count_predicted_cols(t);
    STAMP(t, SB_FIN2);
    return npcol;
}

// Tail of the frozen _inferPhase2: the qualifying segments arrive in rank =
// (column, cell, creation) order -- NuPIC's summation order -- so each
// column's confidence is the in-order float sum over its run of the list and
// the normaliser folds the run sums in ascending column order: bit-identical
// to the oracle without sorting.  Column and dutyCycle of entry k live in
// LDS (qn <= q_lds) or, past that, in the HBM scratch (q1 / q2).  Returns
// numPredictedCols.
__device__ __forceinline__ uint32_t phase2_finish_ranked(Tm& t) {
    const DevCfg& c = t.c;
    TmSh* sh = t.sh;
    const uint32_t qn = (uint32_t)sh->qn;
    const uint32_t ql = (uint32_t)c.q_lds_fx;
    const bool in_lds = qn + 256u <= ql;  // (the normaliser keeps 256 words past the entries)
    uint16_t* lcol = reinterpret_cast<uint16_t*>(t.U);  // [ql]
    float* ldc = reinterpret_cast<float*>(t.U + (ql + 1) / 2);  // [ql]
    uint32_t* gcol = t.q1;
    float* gdc = reinterpret_cast<float*>(t.q2);
    uint32_t nb = phase2_pass1<true>(t, qn, [&](uint32_t k, uint32_t, uint32_t cell, float dc) {
        const uint32_t col = col_of(c, cell);
        if (in_lds) {
            lcol[k] = (uint16_t)col;
            ldc[k] = dc;
        } else {  // q1[k] (the rank) has been read: reuse the entry
            gcol[k] = col;
            gdc[k] = dc;
        }
    });
    nb = wg_sum1(t, nb);  // (a barrier)
    if (threadIdx.x == 0) sh->bytes += nb;
    STAMP(t, SB_FIN1);
    COUNT(t, SC_QN, qn);
    COUNT(t, SC_P2, 1);
    auto col_at = [&](uint32_t k) -> uint32_t { return in_lds ? (uint32_t)lcol[k] : gcol[k]; };
    auto dc_at = [&](uint32_t k) -> float { return in_lds ? ldc[k] : gdc[k]; };
    // run heads sum their column in list order (the adds stay sequential:
    // NuPIC's float order).  In LDS a run is read in aligned groups of eight
    // entries -- one 16-byte read of the columns, two of the dutyCycles --
    // with the next group's reads issued before this group's adds: a bursting
    // step's longest runs (hundreds of a popular column's segments) were a
    // chain of four-entry rounds of scalar reads (tail stamps: sums 38 K
    // cycles, profiles/r05_ab); wider scalar prefetches measured slower (LDS
    // issue, profiles/r06_ab/run_sums)
#ifndef HTM_SUMS_OLD
    if (in_lds) {
        const uint4* lc4 = reinterpret_cast<const uint4*>(lcol);  // (U and ql/2 words: 16-byte aligned)
        const float4* ld4 = reinterpret_cast<const float4*>(ldc);
        for (uint32_t k = threadIdx.x; k < qn; k += TM_NT) {
            const uint32_t col = lcol[k];
            if (k > 0 && lcol[k - 1] == col) continue;
            float sum = 0.0f;
            uint32_t a = k & ~7u;  // the group holding k
            uint4 cg = lc4[a >> 3];
            float4 d0 = ld4[a >> 2], d1 = ld4[(a >> 2) + 1];
            uint32_t i = k - a;  // the first entry of the run in the group
            for (;;) {
                const bool more = a + 8u < qn;
                uint4 cgn = make_uint4(0u, 0u, 0u, 0u);
                float4 d0n = make_float4(0.f, 0.f, 0.f, 0.f), d1n = d0n;
                if (more) {
                    cgn = lc4[(a >> 3) + 1];
                    d0n = ld4[(a >> 2) + 2];
                    d1n = ld4[(a >> 2) + 3];
                }
                const uint32_t cw[4] = {cg.x, cg.y, cg.z, cg.w};
                const float dv[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
                bool stop = false;
#pragma unroll
                for (uint32_t u = 0; u < 8; u++) {
                    if (u < i) continue;
                    const uint32_t cu = (cw[u >> 1] >> ((u & 1) * 16)) & 0xFFFFu;
                    if (!stop && a + u < qn && cu == col) sum += dv[u];
                    else stop = true;
                }
                if (stop || !more) break;
                a += 8u;
                i = 0u;
                cg = cgn;
                d0 = d0n;
                d1 = d1n;
            }
            t.colconf[col] = sum;
        }
    } else
#endif
    for (uint32_t k = threadIdx.x; k < qn; k += TM_NT) {
        const uint32_t col = col_at(k);
        if (k > 0 && col_at(k - 1) == col) continue;
        float sum = 0.0f;
        for (uint32_t j = k;; j += 4) {
            uint32_t cc[4];
            float dd[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const bool in = j + u < qn;
                cc[u] = in ? col_at(j + u) : 0xFFFFFFFFu;
                dd[u] = in ? dc_at(j + u) : 0.0f;
            }
            bool stop = false;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                if (!stop && cc[u] == col) sum += dd[u];
                else stop = true;
            }
            if (stop) break;
        }
        t.colconf[col] = sum;
    }
    __syncthreads();
    STAMP(t, SB_SUMS);
    // normaliser: sequential over the columns with a qualifying segment,
    // ascending (= run-head order; zeros in between would add nothing).  In
    // LDS: every wave takes 64-entry chunks, and the run heads of a chunk write
    // their column sums, compacted in order, to the chunk's own slots of ldc
    // (free once the sums are made) with the count in a side array; then wave
    // 0 folds the chunks in order, each one vector load and `count`
    // lane-by-lane adds, the next chunk loaded while one is folded.
    if (in_lds) {
        float* hv = ldc;
        uint32_t* cnt = reinterpret_cast<uint32_t*>(ldc + (ql - 256u));
        const uint32_t nch = (qn + 63u) / 64u;
        for (uint32_t ch = wave_id(); ch < nch; ch += TM_NWAVES) {
            const uint32_t i = ch * 64u + lane_id();
            bool head = false;
            float v = 0.0f;
            if (i < qn) {
                const uint32_t col = lcol[i];
                head = i == 0 || lcol[i - 1] != col;
                if (head) v = t.colconf[col];
            }
            const uint64_t m = __ballot(head);
            if (head) hv[ch * 64u + (uint32_t)__popcll(m & ((1ull << lane_id()) - 1ull))] = v;
            if (lane_id() == 0) cnt[ch] = (uint32_t)__popcll(m);
        }
        __syncthreads();
        STAMP(t, SB_NCMP);
        if (wave_id() == 0) {
            // wave 0 folds the heads from LDS (every lane the same chain, the
            // reads broadcast): a chain of dependent adds (a readlane per head moved every value through an SGPR,
            // ~100 cycles each: profiles/r05_mid); entries past a chunk's
            // count add +0.0f, which leaves the (non-negative) sum unchanged
            // (16 heads per round: four 16-byte reads issued together, then the
            // adds -- a chunk holds 64 slots, so reads past its count stay in it)
            float tot = 0.0f;
            auto fold16 = [&](const float4 (&x)[4], uint32_t j, uint32_t nn) {
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const uint32_t k = j + 4u * u;
                    tot += k < nn ? x[u].x : 0.0f;
                    tot += k + 1 < nn ? x[u].y : 0.0f;
                    tot += k + 2 < nn ? x[u].z : 0.0f;
                    tot += k + 3 < nn ? x[u].w : 0.0f;
                }
            };
            uint32_t nn1 = nch ? cnt[0] : 0u;
            for (uint32_t ch = 0; ch < nch; ch++) {
                const uint32_t nn = nn1;
                nn1 = ch + 1 < nch ? cnt[ch + 1] : 0u;
                const float4* p = reinterpret_cast<const float4*>(hv + ch * 64u);
                for (uint32_t j = 0; j < nn; j += 16) {
                    float4 x[4];
#pragma unroll
                    for (int u = 0; u < 4; u++) x[u] = p[(j >> 2) + u];
                    fold16(x, j, nn);
                }
            }
            if (lane_id() == 0) sh->tf[0] = tot;
        }
    } else if (wave_id() == 0) {
        float tot = 0.0f;
        for (uint32_t base = 0; base < qn; base += 64) {
            const uint32_t i = base + lane_id();
            float v = 0.0f;
            bool head = false;
            if (i < qn) {
                const uint32_t col = col_at(i);
                head = i == 0 || col_at(i - 1) != col;
                if (head) v = t.colconf[col];
            }
            const int vi = __float_as_int(v);
            for (uint64_t m = __ballot(head); m; m &= m - 1)
                tot += __int_as_float(__builtin_amdgcn_readlane(vi, (int)__builtin_ctzll(m)));
        }
        if (lane_id() == 0) sh->tf[0] = tot;
    }
    __syncthreads();
    STAMP(t, SB_NORM);
    const float tot = sh->tf[0];
    if (tot > 0.0f)
        for (uint32_t k = threadIdx.x; k < qn; k += TM_NT) {
            const uint32_t col = col_at(k);
            if (k == 0 || col_at(k - 1) != col) t.colconf[col] /= tot;
        }
    // numPredictedCols: counted by infer_phase2 before the tail when the pid
    // counters predicted the cells; from the rows read in pass 1 otherwise
    const uint32_t npcol = t.np > (uint32_t)c.fx_pcap ? count_predicted_cols(t) : (uint32_t)sh->npc_known;
    STAMP(t, SB_FIN2);
    return npcol;
}

// Shared tail of _inferPhase2: predicted cells, duty cycles, confidences in
// NuPIC order, normalisation.  Returns numPredictedCols (uniform).
template <bool FROZEN>
__device__ __forceinline__ uint32_t phase2_finish(Tm& t) {
    if (FROZEN) return phase2_finish_ranked(t);
    if (t.c.fin_mode == 1 && (uint32_t)t.sh->qn <= (uint32_t)t.c.q_lds)
        return phase2_finish_sorted<FROZEN>(t, (uint32_t)t.sh->qn);
    const DevCfg& c = t.c;
    TmSh* sh = t.sh;
    const int K = c.K;
    const uint32_t qn = (uint32_t)sh->qn;
    uint32_t* colcnt = t.U;
    uint16_t* nzcol = reinterpret_cast<uint16_t*>(t.U + c.ncol);
    uint32_t* nzstart = t.U + c.ncol + (c.ncol + 1) / 2;
    // qualifying segments (<= q_lds of them): key, dutyCycle, column; and
    // the same sorted by column bucket
    const uint32_t ql = (uint32_t)c.q_lds;
    uint32_t* qkey = nzstart + c.ncol + 1;
    float* qdc = reinterpret_cast<float*>(qkey + ql);
    uint32_t* skey = qkey + 2 * ql;
    float* sdc = reinterpret_cast<float*>(qkey + 3 * ql);
    uint16_t* qcol = reinterpret_cast<uint16_t*>(qkey + 4 * ql);
    uint32_t* colbits = qkey + 4 * ql + (ql + 1) / 2;  // [nw] nonzero columns (fin_mode 2)
    const bool in_lds = qn <= ql;
    const bool bitmap = c.fin_mode == 2;
    wg_clear(colcnt, c.ncol);
    if (bitmap) wg_clear(colbits, c.nw);
    __syncthreads();
    STAMP(t, SB_FCLR);
    // pass 1: connected activity -> predicted; dutyCycle(); bucket counts
    uint32_t nb = phase2_pass1<FROZEN>(t, qn, [&](uint32_t k, uint32_t slot, uint32_t cell, float dc) {
        const uint32_t col = col_of(c, cell);
        atomicAdd(&colcnt[col], 1u);
        if (bitmap) atomicOr(&colbits[col >> 5], 1u << (col & 31));
        if (in_lds) {
            qkey[k] = ((cell - col * K) << 27) | slot;
            qdc[k] = dc;
            qcol[k] = (uint16_t)col;
        }
    });
    nb = wg_sum(sh, nb);
    if (threadIdx.x == 0) sh->bytes += nb;
    STAMP(t, SB_FIN1);
    COUNT(t, SC_QN, qn);
    COUNT(t, SC_P2, 1);
    // exclusive scan of bucket counts + nonzero column list (ascending)
    uint32_t tsum, tnz;
    if (bitmap) {
        // wave 0 walks the nonzero-column bitmap (lane l: words l, l + 64)
        if (wave_id() == 0) {
            const uint32_t l = lane_id();
            uint32_t zbase = 0, obase = 0;
            for (int r = 0; r < 2; r++) {
                const uint32_t wi = l + 64u * r;
                const uint32_t bits = wi < (uint32_t)c.nw ? colbits[wi] : 0u;
                uint32_t s = 0;
                for (uint32_t x = bits; x; x &= x - 1) s += colcnt[wi * 32 + __ffs(x) - 1];
                const uint32_t nz = __popc(bits);
                const uint32_t iz = wave_incl_scan(nz), is = wave_incl_scan(s);
                uint32_t zo = zbase + iz - nz, off = obase + is - s;
                for (uint32_t x = bits; x; x &= x - 1) {
                    const uint32_t col = wi * 32 + __ffs(x) - 1;
                    const uint32_t n = colcnt[col];
                    nzcol[zo] = (uint16_t)col;
                    nzstart[zo] = off;
                    colcnt[col] = off;
                    zo++;
                    off += n;
                }
                zbase += lane63(iz);
                obase += lane63(is);
            }
            if (l == 0) {
                nzstart[zbase] = obase;
                sh->ti[2] = (int32_t)zbase;
                sh->ti[3] = (int32_t)obase;
            }
        }
        __syncthreads();
        STAMP(t, SB_SORT);
        tnz = (uint32_t)sh->ti[2];
        tsum = (uint32_t)sh->ti[3];
    } else {
        const int per = (c.ncol + TM_NT - 1) / TM_NT;
        const int c0 = threadIdx.x * per;
        uint32_t lsum = 0, lnz = 0;
        for (int k = 0; k < per; k++) {
            int col = c0 + k;
            if (col < c.ncol && colcnt[col]) { lsum += colcnt[col]; lnz++; }
        }
        uint32_t off = wg_excl_scan(sh, lsum, &tsum);
        uint32_t zo = wg_excl_scan(sh, lnz, &tnz);
        for (int k = 0; k < per; k++) {
            int col = c0 + k;
            if (col >= c.ncol) break;
            uint32_t n = colcnt[col];
            if (n) {
                nzcol[zo] = (uint16_t)col;
                nzstart[zo] = off;
                zo++;
            }
            colcnt[col] = off;
            off += n;
        }
        if (threadIdx.x == 0) nzstart[tnz] = tsum;
        __syncthreads();
    }
    (void)tsum;
    // pass 2: scatter keys (cellInColumn << 27 | slot) into column buckets
    if (in_lds) {
        for (uint32_t k = threadIdx.x; k < qn; k += TM_NT) {
            const uint32_t pos = atomicAdd(&colcnt[qcol[k]], 1u);
            skey[pos] = qkey[k];
            sdc[pos] = qdc[k];
        }
    } else {
        for (uint32_t k = threadIdx.x; k < qn; k += TM_NT) {
            uint32_t slot = t.q1[k];
            uint32_t cell = meta_cell(t.meta[slot]);
            uint32_t col = col_of(c, cell);
            uint32_t pos = atomicAdd(&colcnt[col], 1u);
            t.q2[pos] = ((cell - col * K) << 27) | slot;
        }
    }
    __syncthreads();
    // pass 3a (LDS path): each entry's rank inside its column bucket (keys are
    // unique: they hold the slot) places its dutyCycle in (cell, slot) order
    // into qdc, dead since the scatter.  Entry-parallel with independent loads:
    // a bucket of m entries costs m loads per entry instead of an O(m^2)
    // dependent insertion sort on one thread.
    if (in_lds) {
        for (uint32_t p = threadIdx.x; p < qn; p += TM_NT) {
            uint32_t lo = 0, hi = tnz;  // last z with nzstart[z] <= p
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (nzstart[mid] <= p) lo = mid;
                else hi = mid;
            }
            const uint32_t b0 = nzstart[lo], b1 = nzstart[lo + 1];
            const uint32_t key = skey[p];
            uint32_t r = 0;
            for (uint32_t j = b0; j < b1; j++) r += skey[j] < key ? 1u : 0u;
            qdc[b0 + r] = sdc[p];
        }
        __syncthreads();
    }
    // pass 3: per column, (cell, slot) order; float sum in that order
    uint32_t npcol = 0;
    for (uint32_t k = threadIdx.x; k < tnz; k += TM_NT) {
        uint32_t col = nzcol[k], lo = nzstart[k], hi = nzstart[k + 1];
        float sum = 0.0f;
        if (in_lds) {
            for (uint32_t i = lo; i < hi; i++) sum += qdc[i];
        } else {
            for (uint32_t i = lo + 1; i < hi; i++) {
                uint32_t key = t.q2[i];
                uint32_t j = i;
                while (j > lo && t.q2[j - 1] > key) { t.q2[j] = t.q2[j - 1]; j--; }
                t.q2[j] = key;
            }
            for (uint32_t i = lo; i < hi; i++) {
                uint32_t slot = t.q2[i] & 0x7FFFFFFu;
                sum += __uint_as_float(t.duty[(size_t)slot * 3 + 1]);
            }
        }
        t.colconf[col] = sum;
        if (bm_field(t.infP, col * K, K)) npcol++;
    }
    npcol = wg_sum(sh, npcol);
    STAMP(t, SB_SUMS);
    // total in nonzero-column order (ascending), sequentially as NuPIC sums it:
    // wave 0 loads 64 column sums at a time and folds them lane by lane
    // (zero padding adds +0.0f, which leaves the sum unchanged; a one-lane
    // fold reading them from LDS measured slower here: fin2 8 K -> 28 K cycles
    // per learning stream-step, profiles/r05_ab)
    if (wave_id() == 0) {
        float tot = 0.0f;
        for (uint32_t base = 0; base < tnz; base += 64) {
            const uint32_t i = base + lane_id();
            const float v = i < tnz ? t.colconf[nzcol[i]] : 0.0f;
            const int vi = __float_as_int(v);
#pragma unroll
            for (int j = 0; j < 64; j++) tot += __int_as_float(__builtin_amdgcn_readlane(vi, j));
        }
        if (lane_id() == 0) sh->tf[0] = tot;
    }
    __syncthreads();
    float tot = sh->tf[0];
    if (tot > 0.0f)
        for (uint32_t k = threadIdx.x; k < tnz; k += TM_NT) t.colconf[nzcol[k]] /= tot;
    __syncthreads();
    STAMP(t, SB_FIN2);
    COUNT(t, SC_TNZ, tnz);
    return npcol;
}

// The confidences a frozen phase 2 computes matter only if its state is the
// one the step keeps: P2_DISCARD -- a backtrack replay before the current
// pattern (its phase 1 reads only the predicted cells); P2_IF_IN_SEQ -- the
// step's own phase 2 or a replay's last one (kept exactly when in sequence,
// otherwise a backtrack or the next start recomputes); P2_KEEP -- always.
// Skipped confidence sums leave colConfidence zero.  The segments' dutyCycle()
// state updates happen in every case, as in NuPIC.
enum { P2_DISCARD = 0, P2_IF_IN_SEQ = 1, P2_KEEP = 2 };

// frozen phase 2 whose confidences are discarded: the dutyCycle() state
// updates of the qualifying segments only
__device__ __forceinline__ void phase2_duty_only(Tm& t) {
    const uint32_t qn = (uint32_t)t.sh->qn;
    const uint32_t nb = phase2_pass1<true>(t, qn, [](uint32_t, uint32_t, uint32_t, float) {});
    if (nb) atomicAdd(&t.sh->bytes, (unsigned long long)nb);
    COUNT(t, SC_QN, qn);
    COUNT(t, SC_P2, 1);
}

// murmur3's finaliser: the per-cell term of an active set's hash
__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}

// Log the active cells of a frozen phase 2 whose confidences are discarded
// (the list a pid-only collection left in U) for tm_fx_flush_kernel, which
// makes its qualifying segments' dutyCycle() record writes.  The log is a
// ring of fx_dcap entries per stream; an active set equal to one still in the
// ring (flushed or not: backtrack replays recur from step to step) is not
// logged again -- its writes are made or pending.  The ring's hashes and
// lengths live in registers (lane l of every wave holds slot l's, loaded with
// the state), so finding the candidate costs no memory access; only the
// newest candidate's cells are read back and compared in full.  False when
// the ring holds fx_dcap unflushed entries: the caller then counts the rank
// windows itself.  Contains barriers: call uniformly.
__device__ __forceinline__ bool defer_phase2(Tm& t) {
    const DevCfg& c = t.c;
    TmSh* sh = t.sh;
    const TmBufs& b = *t.tb;
    const uint32_t dcap = (uint32_t)c.fx_dcap;
    const uint32_t na = (uint32_t)sh->fx_na;
    const uint16_t* cells = reinterpret_cast<const uint16_t*>(t.U + c.fx_win / 4 + 64);
    const size_t stride = fx_dstride(c);
    // order-independent hash of the set
    uint32_t h = 0;
    for (uint32_t k = threadIdx.x; k < na; k += TM_NT) h += fmix32(cells[k] + 0x9e3779b9u);
    h = fmix32(wg_sum1(t, h) ^ na);
    const uint32_t n = t.dn;
    // the newest resident entry with this hash and length (every wave finds
    // the same: lane l of each wave holds slot l)
    const uint32_t l = lane_id();
    const uint32_t resident = n < dcap ? n : dcap;
    uint32_t age = 0xFFFFFFFFu;  // n - 1 - entry in slot l
    if (l < dcap && resident) {
        const uint32_t a = (n - 1u - l) % dcap;
        if (a < resident && t.rh == h && t.rl == na) age = a;
    }
    age = ~wave_max_u32(~age);  // the minimum: the newest entry
    if (age != 0xFFFFFFFFu) {
        const uint16_t* old = b.fx_dlog + ((size_t)t.s * dcap + (n - 1u - age) % dcap) * stride;
        uint32_t diff = 0;
        for (uint32_t k = threadIdx.x; k < na; k += TM_NT) diff |= old[k] != cells[k] ? 1u : 0u;
        if (wg_sum1(t, diff) == 0) {
            if (threadIdx.x == 0) sh->bytes += 2ull * na;
            return true;  // the same set is logged already
        }
    }
    if (n - t.df >= dcap) return false;
    const uint32_t sl = n % dcap;
    const size_t slot = (size_t)t.s * dcap + sl;
    uint16_t* dst = b.fx_dlog + slot * stride;
    for (uint32_t k = threadIdx.x; k < na; k += TM_NT) dst[k] = cells[k];
    if (threadIdx.x == 0) {
        b.fx_dlen[slot] = (uint16_t)na;
        b.fx_dhash[slot] = h;
        sh->bytes += 2ull * na + 6ull;
    }
    if (l == sl) {
        t.rh = h;
        t.rl = na;
    }
    t.dn = n + 1u;
    return true;
}

// _inferPhase2()
template <bool FROZEN>
__device__ __forceinline__ bool infer_phase2(Tm& t, int need = P2_KEEP) {
    TmSh* sh = t.sh;
    if (threadIdx.x == 0) {
        sh->st[0]++;
        sh->qn = 0;
        sh->npc_known = -1;
    }
    wg_clear(t.infP, t.c.cw);
    wg_clear(reinterpret_cast<uint32_t*>(t.colconf), t.c.ncol);
    // (frozen: collect_frozen's cell listing ends with a barrier before any
    // infP / colConfidence write or qn read)
    if (!FROZEN) __syncthreads();
    if (FROZEN && t.defer && need != P2_KEEP && t.np <= (uint32_t)t.c.fx_pcap) {
        // the predicted cells first (pid pass): a phase 2 whose confidences the
        // step discards needs nothing else now -- its segments' one-time
        // dutyCycle() record writes are logged for tm_fx_flush_kernel
        collect_frozen(t, t.c.act_thr, FX_PID);
        __syncthreads();
        const uint32_t npc = count_predicted_cols(t);
        STAMP(t, SB_CPC);
        const bool inSeq = (double)npc >= 0.5 * sh->avg_dens;
        const bool keep = need == P2_IF_IN_SEQ && inSeq;
        if (!keep) {
            const bool logged = defer_phase2(t);
            STAMP(t, SB_DEFER);
            if (logged) return inSeq;
        }
        collect_frozen(t, t.c.act_thr, FX_WIN_REUSE);
        __syncthreads();
        if (threadIdx.x == 0 && (uint32_t)sh->qn > (uint32_t)t.c.q_cap) {
            sh->err |= 16u;
            sh->qn = t.c.q_cap;
        }
        __syncthreads();
        if (keep) {
            if (threadIdx.x == 0) sh->npc_known = (int32_t)npc;
            __syncthreads();
            (void)phase2_finish<FROZEN>(t);
        } else {
            phase2_duty_only(t);
        }
        __syncthreads();
        return inSeq;
    }
    if (FROZEN) collect_frozen(t, t.c.act_thr);
    else collect_scan(t, t.infA, t.c.act_thr);
    __syncthreads();
    if (threadIdx.x == 0 && (uint32_t)sh->qn > (uint32_t)t.c.q_cap) {
        sh->err |= 16u;  // qualifying-segment list overflow (fleet q_capacity): results invalid
        sh->qn = t.c.q_cap;
    }
    __syncthreads();
    if (FROZEN && t.np <= (uint32_t)t.c.fx_pcap) {
        // the pid counters have predicted the cells: decide first
        const uint32_t npc = count_predicted_cols(t);
        const bool inSeq = (double)npc >= 0.5 * sh->avg_dens;
        if (need == P2_KEEP || (need == P2_IF_IN_SEQ && inSeq)) {
            if (threadIdx.x == 0) sh->npc_known = (int32_t)npc;
            __syncthreads();
            (void)phase2_finish<FROZEN>(t);
        } else {
            phase2_duty_only(t);
        }
        __syncthreads();
        return inSeq;
    }
    uint32_t npc = phase2_finish<FROZEN>(t);
    return (double)npc >= 0.5 * sh->avg_dens;
}

__device__ __forceinline__ const uint16_t* inf_pat(Tm& t, int k) {
    return t.sh->inf_pat[(t.sh->inf_head + k) % HTM_MAXPAT];
}
__device__ __forceinline__ int inf_len(Tm& t, int k) { return t.sh->inf_len[(t.sh->inf_head + k) % HTM_MAXPAT]; }
__device__ __forceinline__ const uint16_t* lrn_pat(Tm& t, int k) {
    return t.lrnpat[(t.sh->lrn_head + k) % HTM_MAXPAT];
}
__device__ __forceinline__ int lrn_len(Tm& t, int k) { return t.sh->lrn_len[(t.sh->lrn_head + k) % HTM_MAXPAT]; }

// _inferBacktrack(activeColumns).  NuPIC copies infPredictedState t -> t-1
// before every replay's phase 1 and restores t-1 from a backup afterwards;
// here a replay's phase 1 reads the previous replay's infP directly (its
// phase 2 clears infP only after phase 1's barriers), so infP(t-1) (infP1) is
// never touched and needs no backup.  NuPIC's saved candidate state is not
// copied: the loop stops at the candidate, so the live state already is it;
// and with no candidate the current pattern's phase 1 is recomputed from
// infP(t-1) instead of restoring a saved infActiveState (same state,
// computed the same way).
template <bool FROZEN>
__device__ __forceinline__ void infer_backtrack(Tm& t) {
    TmSh* sh = t.sh;
    const int numPrev = sh->n_inf_pat;
    if (numPrev <= 0) return;
    const int cur = numPrev - 1;
    if (threadIdx.x == 0) sh->st[1]++;
    uint32_t bad = 0;
    bool haveCand = false;
    int candStart = -1;
    for (int start = 0; start < numPrev; start++) {
        if (start == cur && haveCand) break;
        bool inSeq = false;
        for (int off = start; off < numPrev; off++) {
            STAMP(t, SB_BT);
            inSeq = infer_phase1(t, inf_pat(t, off), inf_len(t, off), off == start, t.infP);
            if (!inSeq) break;
            inSeq = infer_phase2<FROZEN>(t, off == cur ? P2_IF_IN_SEQ : P2_DISCARD);
            if (!inSeq) break;
        }
        if (!inSeq) {
            bad |= 1u << start;
            continue;
        }
        haveCand = true;
        candStart = start;
        break;
    }
    if (!haveCand) {
        (void)infer_phase1(t, sh->act, sh->nA, sh->reset != 0);
        (void)infer_phase2<FROZEN>(t);
    }
    if (threadIdx.x == 0) {
        int npop = 0;
        for (int i = 0; i < numPrev; i++) {
            if (((bad >> i) & 1u) || (haveCand && i <= candStart)) npop++;
            else break;
        }
        sh->inf_head = (sh->inf_head + npop) % HTM_MAXPAT;
        sh->n_inf_pat -= npop;
    }
    STAMP(t, SB_BT);
}

// _updateInferenceState(activeColumns)
template <bool FROZEN>
__device__ __forceinline__ void update_inference(Tm& t) {
    TmSh* sh = t.sh;
    if (threadIdx.x == 0) {
        if (t.c.max_inf_bt > 0) {
            if (sh->n_inf_pat > t.c.max_inf_bt) {
                sh->inf_head = (sh->inf_head + 1) % HTM_MAXPAT;
                sh->n_inf_pat--;
            }
            int slot = (sh->inf_head + sh->n_inf_pat) % HTM_MAXPAT;
            sh->inf_len[slot] = (uint16_t)sh->nA;
            sh->ti[0] = slot;
            sh->n_inf_pat++;
        } else {
            sh->ti[0] = -1;
        }
    }
    __syncthreads();
    if (sh->ti[0] >= 0)
        for (int a = threadIdx.x; a < sh->nA; a += TM_NT) sh->inf_pat[sh->ti[0]][a] = sh->act[a];
    __syncthreads();
    bool inSeq = infer_phase1(t, sh->act, sh->nA, sh->reset != 0);
    if (!inSeq) {
        infer_backtrack<FROZEN>(t);
        return;
    }
    // with a pattern history, a phase 2 out of sequence is redone by the backtrack
    inSeq = infer_phase2<FROZEN>(t, sh->n_inf_pat > 0 ? P2_IF_IN_SEQ : P2_KEEP);
    if (!inSeq) infer_backtrack<FROZEN>(t);
}

// ---------------------------------------------------------------------------
// Learning (wave-0 sequential helpers run with all 64 lanes of wave 0)

// per-column best (activity, cellInColumn, first segment) key over the pool
// for segments with >= thr synapses onto `state`; only columns flagged in
// `colflags` when it is non-null.  _getBestMatchingCell for many columns.
__device__ __forceinline__ void scan_best(Tm& t, const uint32_t* state, int thr, const uint32_t* colflags) {
    const DevCfg& c = t.c;
    unsigned long long* keys = reinterpret_cast<unsigned long long*>(t.U);
    const uint32_t sub = threadIdx.x & 3;
    auto best = [&](uint32_t slot, uint32_t m, bool el, uint32_t mask) {
        const uint32_t n = __popc(mask);
        if (el && sub == 0 && n >= (uint32_t)thr) {
            const uint32_t cell = meta_cell(m), col = col_of(c, cell);
            const uint32_t cic = cell - col * c.K;
            const unsigned long long key = ((unsigned long long)n << 40) | ((unsigned long long)cic << 32) |
                                           (unsigned long long)(0xFFFFFFFFu - slot);
            atomicMax(&keys[col], key);
        }
    };
    // every column (learn phase 2): rows loaded with the meta words; flagged
    // columns only (learn phase 1): the eligible slots listed first (in the
    // learning records' LDS, free until the records are built), then their
    // rows -- the whole pool's scan only if the list overflows
    auto flagged = [&](uint32_t m) {
        const uint32_t col = col_of(c, meta_cell(m));
        return ((colflags[col >> 5] >> (col & 31)) & 1u) != 0u;
    };
    uint32_t nb;
    if (colflags) {
        bool over = false;
        nb = scan_pool_sparse(t, state, flagged, best, t.U + 2 * c.ncol, (uint32_t)LREC_WORDS - 1u, &over);
        if (over) nb += scan_pool<false>(t, state, flagged, best);
    } else {
        nb = scan_pool<true>(t, state, [](uint32_t) { return true; }, best);
    }
    nb = wg_sum(t.sh, nb);
    if (threadIdx.x == 0) t.sh->bytes += nb;
}

__device__ __forceinline__ uint32_t key_slot(unsigned long long k) { return 0xFFFFFFFFu - (uint32_t)k; }
__device__ __forceinline__ uint32_t key_cic(unsigned long long k) { return (uint32_t)(k >> 32) & 0xFFu; }
__device__ __forceinline__ uint32_t key_act(unsigned long long k) { return (uint32_t)(k >> 40); }

// ---- nupic::Random draws by a whole wave (learning's wave-0 helpers).
// The generator (TmSh::rng, rf, rr: glibc random_r TYPE_3, r == f - 3 mod 31)
// is x[n] = x[n-31] + x[n-3]; buffer slot (f + j) % 31 holds x[n-31+j].  The
// next 31 values y[j] = x[n+j] = v[j] + (j >= 3 ? y[j-3] : v[28+j]) are a
// stride-3 inclusive scan of v plus v[28 + j % 3]: four cross-lane adds, the
// block in lanes 0..30 at once instead of 31 dependent LDS round trips.
// w_rng_peek returns lane j's upcoming raw draw j (the value rng_raw would
// return; lanes >= 31: 0) without consuming it, w_rng_commit(k) consumes the
// first k (<= 31) -- the generator then stands exactly where k rng_raw calls
// leave it.  Call with every lane of the wave.
__device__ __forceinline__ uint32_t w_rng_peek(Tm& t, uint32_t& y) {
    TmSh* sh = t.sh;
    const uint32_t l = (uint32_t)lane_id();
    const uint32_t f = (uint32_t)__builtin_amdgcn_readfirstlane(sh->rf);
    uint32_t fj = f + l;
    fj = fj >= 31u ? fj - 31u : fj;
    const uint32_t v = l < 31u ? sh->rng[fj < 31u ? fj : 0u] : 0u;
    uint32_t p = v;
#pragma unroll
    for (int d = 3; d < 31; d *= 2) {
        const uint32_t up = (uint32_t)__shfl_up((int)p, d, 64);
        if (l >= (uint32_t)d) p += up;
    }
    const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 28);
    const uint32_t b1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 29);
    const uint32_t b2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 30);
    const uint32_t m3 = l % 3u;
    y = p + (m3 == 0u ? b0 : m3 == 1u ? b1 : b2);
    return l < 31u ? ((y >> 1) & 0x7fffffffu) : 0u;
}

__device__ __forceinline__ void w_rng_commit(Tm& t, uint32_t y, uint32_t k) {
    TmSh* sh = t.sh;
    const uint32_t l = (uint32_t)lane_id();
    const uint32_t f = (uint32_t)__builtin_amdgcn_readfirstlane(sh->rf);
    __builtin_amdgcn_wave_barrier();  // every lane has read the state (w_rng_peek)
    if (l < k) {
        uint32_t fj = f + l;
        fj = fj >= 31u ? fj - 31u : fj;
        sh->rng[fj] = y;
    }
    COUNT(t, SC_LDRAWS, k);
    if (l == 0) {
        const uint32_t nf = (f + k) % 31u;
        sh->rf = (int32_t)nf;
        sh->rr = (int32_t)((nf + 28u) % 31u);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// _chooseCellsToLearnFrom's sample of n of the m candidates (m > n >= 1):
// bit i of the result = candidate i chosen.  n == 1: one draw, index
// getUInt32(m); else candidate i is taken when getUInt32(m - i) < n - taken,
// until n are taken -- the draws of up to 31 candidates and their residues
// are computed across the lanes at once, the (cheap) sequential decisions
// read them lane by lane, and exactly the draws the sequential loop makes
// are consumed.
__device__ __forceinline__ uint64_t w_rng_sample(Tm& t, uint32_t m, uint32_t n) {
    const uint32_t l = (uint32_t)lane_id();
    uint64_t ch = 0;
    uint32_t cnt = 0, i0 = 0;
    for (;;) {
        uint32_t y;
        const uint32_t raw = w_rng_peek(t, y);
        if (n == 1u) {
            const uint32_t u0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(raw % m));
            w_rng_commit(t, y, 1u);
            return 1ull << u0;
        }
        const uint32_t i = i0 + l;
        const uint32_t u = (l < 31u && i < m) ? raw % (m - i) : 0u;
        const uint32_t lim = m - i0 < 31u ? m - i0 : 31u;
        uint32_t k = 0;
        bool done = false;
        for (uint32_t j = 0; j < lim; j++) {
            const uint32_t uj = (uint32_t)__builtin_amdgcn_readlane((int)u, (int)j);
            k = j + 1u;
            if (uj < n - cnt) {
                ch |= 1ull << (i0 + j);
                if (++cnt == n) {
                    done = true;
                    break;
                }
            }
        }
        w_rng_commit(t, y, k);
        i0 += k;
        if (done || i0 >= m) return ch;
    }
}

// ---- the generator in wave 0's registers for a whole draw pass (round 5:
// the learning loops' draws).  Lane j < 31 holds the raw sums of the current
// block of 31 draws (x[n0 + 31 b + j], before the >> 1), `prev` the block
// before it -- initially the loaded state x[n0 - 31 .. n0 - 1], taken as block
// -1, fully consumed; pos = draws consumed in the current block.  A block
// follows from the previous one v by y[j] = v[j] + (j >= 3 ? y[j-3] : v[28+j]):
// lanes 0..2 get their base v[28 + j] added, then an inclusive scan over
// stride 3 inside each 16-lane row (DPP row_shr 3, 6, 12: residue classes
// never mix), and row 0's totals per residue (lanes 15, 13, 14) carried into
// row 1 by a second such scan -- no LDS round trip (w_rng_peek takes four
// ds_bpermute's and two LDS reads per block, and commits to LDS).
// The LDS generator (TmSh::rng, rf, rr) is loaded once and written back once.
struct WGen {
    uint32_t cur, prev;  // per lane
    uint32_t pos;        // draws consumed in the current block (uniform)
    uint32_t total;      // draws consumed since the load (uniform)
    uint32_t f0;         // the loaded state's front pointer (uniform)
};

__device__ __forceinline__ WGen wgen_load(Tm& t) {
    TmSh* sh = t.sh;
    const uint32_t l = (uint32_t)lane_id();
    WGen g;
    g.f0 = (uint32_t)__builtin_amdgcn_readfirstlane(sh->rf);
    uint32_t fj = g.f0 + l;
    fj = fj >= 31u ? fj - 31u : fj;
    g.cur = l < 31u ? sh->rng[fj < 31u ? fj : 0u] : 0u;
    g.prev = 0u;
    g.pos = 31u;
    g.total = 0u;
    return g;
}

__device__ __forceinline__ void wgen_ensure(WGen& g) {
    if (g.pos == 31u) {
        g.prev = g.cur;
        g.cur = rng_block_lanes(g.prev);
        g.pos = 0u;
    }
}

// one rng_raw() draw
__device__ __forceinline__ uint32_t wgen_raw(WGen& g) {
    wgen_ensure(g);
    const uint32_t y = (uint32_t)__builtin_amdgcn_readlane((int)g.cur, (int)g.pos);
    g.pos++;
    g.total++;
    return (y >> 1) & 0x7fffffffu;
}

// _chooseCellsToLearnFrom's sample of n of the m candidates (m > n >= 1),
// as w_rng_sample: candidate i is taken when getUInt32(m - i) < n - taken.
// Within a block the residues u are computed across the lanes; the taken
// set T of the block is the fixed point of
//     T = { lane l : u_l + |T below l| < need },
// found by iterating from T = { u < need } (each round re-counts every lane's
// takes below it with one mbcnt and re-ballots): the lanes before the first
// lane where an iterate differs from the sequential result are exact, so the
// next iterate is exact one lane further at least, and the iteration stops
// exactly at the sequential result (a fixed point satisfies the recurrence
// lane by lane).  A few rounds per block instead of a scalar step per take
// (round 5 first: ~2,900 cycles per sample).  When the block holds the
// need-th take, the candidates after it are not examined (their draws stay
// unconsumed), as in the loop.
__device__ __forceinline__ unsigned long long wgen_sample(WGen& g, uint32_t m, uint32_t n) {
    if (n == 1u) return 1ull << (wgen_raw(g) % m);
    const uint32_t l = (uint32_t)lane_id();
    const uint64_t below = (l == 0u) ? 0ull : (~0ull >> (64u - l));
    unsigned long long ch = 0ull;
    uint32_t need = n, i0 = 0u;
    for (;;) {
        wgen_ensure(g);
        const uint32_t pos = g.pos;
        const uint32_t avail = 31u - pos, left = m - i0;
        const uint32_t lim = left < avail ? left : avail;
        const bool valid = l >= pos && l < pos + lim;
        // (residues are < m <= 64; a lane outside the window can never be taken)
        const uint32_t u = valid ? ((g.cur >> 1) & 0x7fffffffu) % (m - (i0 + l - pos)) : 0x40000000u;
        uint64_t T = __ballot(u < need);
        for (;;) {
            const uint64_t Tn = __ballot(u + (uint32_t)__popcll(T & below) < need);
            if (Tn == T) break;
            T = Tn;
        }
        const uint32_t nt = (uint32_t)__popcll(T);
        uint32_t p;
        if (nt == need) {  // (at most need: no lane past the need-th take passes)
            p = 64u - (uint32_t)__clzll((unsigned long long)T);  // one past the last take
            need = 0u;
        } else {
            p = pos + lim;
            need -= nt;
        }
        ch |= (T >> pos) << i0;
        const uint32_t k = p - pos;
        g.pos = p;
        g.total += k;
        i0 += k;
        if (need == 0u || i0 >= m) return ch;
    }
}

// write the generator back to TmSh::rng / rf / rr: slot (f0 + total + j) % 31
// gets x[n0 + total - 31 + j], the last 31 raw sums (prev[pos..30] then
// cur[0..pos-1])
__device__ __forceinline__ void wgen_store(Tm& t, const WGen& g) {
    TmSh* sh = t.sh;
    const uint32_t l = (uint32_t)lane_id();
    const uint32_t split = 31u - g.pos;
    const uint32_t a = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((g.pos + l) & 63u) << 2), (int)g.prev);
    const uint32_t b = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((l + g.pos - 31u) & 63u) << 2), (int)g.cur);
    const uint32_t x = l < split ? a : b;
    const uint32_t f1 = (g.f0 + g.total) % 31u;
    __builtin_amdgcn_wave_barrier();
    if (l < 31u) {
        uint32_t fj = f1 + l;
        fj = fj >= 31u ? fj - 31u : fj;
        sh->rng[fj] = x;
    }
    if (l == 0u) {
        sh->rf = (int32_t)f1;
        sh->rr = (int32_t)((f1 + 28u) % 31u);
    }
    COUNT(t, SC_LDRAWS, g.total);
    COUNT(t, SC_LBLOCKS, (g.total + 30u) / 31u);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

struct WUpd {
    uint32_t mask;   // active existing synapse positions
    uint32_t n_new;  // new sources
    uint32_t my_new; // lane k (< n_new): k-th new source
};

// _getSegmentActiveSynapses(c, i, s, activeState, newSynapses) with
// _chooseCellsToLearnFrom; candidates = sh->cand (cells on in `state`).
// slot == 0xFFFFFFFF: new segment.
__device__ __forceinline__ WUpd w_build_update(Tm& t, uint32_t slot, const uint32_t* state, bool want_new) {
    TmSh* sh = t.sh;
    const int l = lane_id();
    const bool exist = slot != 0xFFFFFFFFu;
    uint32_t nsyn = exist ? meta_nsyn(t.meta[slot]) : 0u;
    uint32_t mysrc = (exist && (uint32_t)l < nsyn) ? (uint32_t)t.src[(size_t)slot * HTM_MAXSYN + l] : 0xFFFFFFFFu;
    bool act = (exist && (uint32_t)l < nsyn) && bm_get(state, mysrc);
    WUpd u;
    u.mask = (uint32_t)__ballot(act);
    u.n_new = 0;
    u.my_new = 0;
    if (l == 0 && exist) atomicAdd(&sh->bytes, (unsigned long long)(4 + 2 * nsyn));
    int n = want_new ? t.c.new_syn - __popc(u.mask) : 0;
    if (n <= 0) return u;
    const int ncand = sh->ncand;
    uint32_t cv = l < ncand ? sh->cand[l] : 0xFFFFFFFEu;
    bool ok = l < ncand;
    for (uint32_t j = 0; j < nsyn; j++) {  // (j uniform: a register read, not an LDS permute)
        const uint32_t sj = (uint32_t)__builtin_amdgcn_readlane((int)mysrc, (int)j);
        if (cv == sj) ok = false;
    }
    uint64_t keep = __ballot(ok);
    const uint32_t m = (uint32_t)__popcll(keep);
    if (m == 0) return u;
    const uint32_t pos = ballot_rank(keep);
    uint64_t chosen;
    if (m <= (uint32_t)n) {
        chosen = (m == 64) ? ~0ull : ((1ull << m) - 1ull);
    } else {
        STAMP(t, SB_LWB);
        chosen = w_rng_sample(t, m, (uint32_t)n);
        COUNT(t, SC_LSAMPLES, 1);
        STAMP(t, SB_LWS);
    }
    if (ok && ((chosen >> pos) & 1ull)) {
        uint32_t op = (uint32_t)__popcll(chosen & ((1ull << pos) - 1ull));
        sh->newsrc[op] = cv;
    }
    u.n_new = (uint32_t)__popcll(chosen);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    u.my_new = (uint32_t)l < u.n_new ? sh->newsrc[l] : 0u;
    return u;
}

__device__ __forceinline__ uint32_t wave_or_u32(uint32_t v) { return wave_or_dpp(v); }

// _adaptSegment on an existing segment; returns trimSegment (wave-uniform)
__device__ __forceinline__ bool w_adapt_existing(Tm& t, uint32_t slot, uint32_t amask, uint32_t n_new, uint32_t my_new) {
    const DevCfg& c = t.c;
    const int l = lane_id();
    const uint32_t m = t.meta[slot];
    const uint32_t nsyn = meta_nsyn(m);
    uint16_t* srow = t.src + (size_t)slot * HTM_MAXSYN;
    float* prow = t.perm + (size_t)slot * HTM_MAXSYN;
    if (l == 0) {
        t.duty[(size_t)slot * 3] += 1u;  // positiveActivations
        (void)seg_dc_update(t.duty, slot, t.sh->lrn_iter, true);
        // meta, duty (r/w), sources + permanences (r/w), conn
        atomicAdd(&t.sh->bytes, (unsigned long long)(4 + 24 + 2 * 6 * (nsyn + n_new) + 8));
    }
    const bool in = (uint32_t)l < nsyn;
    uint32_t sj = in ? srow[l] : 0u;
    float p = in ? prow[l] : 0.0f;
    const bool isact = in && ((amask >> l) & 1u);
    const bool inact = in && !isact;
    bool hit0 = false;
    if (inact) {
        float nv = p + (-c.tm_dec);
        p = nv;
        if (nv <= 0.0f) { p = 0.0f; hit0 = true; }
    }
    if (isact) {
        float nv = p + c.tm_inc;
        p = nv;
        if (nv > c.tm_max) p = c.tm_max;
    }
    const bool trim = __ballot(hit0) != 0ull;
    bool del = false;
    if (nsyn + n_new > (uint32_t)c.max_syn) {
        const uint32_t numToFree = nsyn + n_new - (uint32_t)c.max_syn;
        uint32_t rin = 0, rac = 0;
        for (int k = 0; k < 32; k++) {
            const float pk = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p), k));
            const int ik = __builtin_amdgcn_readlane((int)inact, k);
            const int ak = __builtin_amdgcn_readlane((int)isact, k);
            bool lt = (pk < p) || (pk == p && k < l);
            if (ik && lt) rin++;
            if (ak && lt) rac++;
        }
        const uint32_t ninact = (uint32_t)__popcll(__ballot(inact));
        if (inact && rin < numToFree) del = true;
        if (numToFree > ninact && isact && rac < numToFree - ninact) del = true;
    }
    const bool keep = in && !del;
    const uint64_t kb = __ballot(keep);
    const uint32_t nkeep = (uint32_t)__popcll(kb);
    const uint32_t np = ballot_rank(kb);
    uint32_t cbits = 0;
    if (keep) {
        srow[np] = (uint16_t)sj;
        prow[np] = p;
        if (p >= c.tm_conn) cbits |= 1u << np;
    }
    if ((uint32_t)l < n_new) {
        srow[nkeep + l] = (uint16_t)my_new;
        prow[nkeep + l] = c.init_perm;
        if (c.init_perm >= c.tm_conn) cbits |= 1u << (nkeep + l);
    }
    cbits = wave_or_u32(cbits);
    if (l == 0) {
        t.conn[slot] = cbits;
        t.meta[slot] = (m & ~(0x3Fu << 16)) | ((nkeep + n_new) << 16);
    }
    return trim;
}

// _trimSegmentsInCell(c, i, [s], minPermanence=0.00001, minNumSyns=0)
__device__ __forceinline__ void w_trim_segment(Tm& t, uint32_t slot) {
    const DevCfg& c = t.c;
    const int l = lane_id();
    const uint32_t m = t.meta[slot];
    const uint32_t nsyn = meta_nsyn(m), cell = meta_cell(m);
    uint16_t* srow = t.src + (size_t)slot * HTM_MAXSYN;
    float* prow = t.perm + (size_t)slot * HTM_MAXSYN;
    const bool in = (uint32_t)l < nsyn;
    uint32_t sj = in ? srow[l] : 0u;
    float p = in ? prow[l] : 0.0f;
    const bool del = in && p < 0.00001f;
    const uint32_t ndel = (uint32_t)__popcll(__ballot(del));
    if (l == 0) atomicAdd(&t.sh->bytes, (unsigned long long)(4 + 6 * nsyn + (ndel ? 8 + 6 * (nsyn - ndel) : 0)));
    if (ndel == nsyn) {
        if (l == 0) {
            t.meta[slot] = m & ~(1u << 23);
            t.nseg[cell] -= 1;
            atomicSub(&t.sh->nlive, 1u);
        }
        return;
    }
    if (ndel == 0) return;
    const bool keep = in && !del;
    const uint64_t kb = __ballot(keep);
    const uint32_t np = ballot_rank(kb);
    uint32_t cbits = 0;
    if (keep) {
        srow[np] = (uint16_t)sj;
        prow[np] = p;
        if (p >= c.tm_conn) cbits |= 1u << np;
    }
    cbits = wave_or_u32(cbits);
    if (l == 0) {
        t.conn[slot] = cbits;
        t.meta[slot] = (m & ~(0x3Fu << 16)) | ((nsyn - ndel) << 16);
    }
}

// new sequence segment on `cell` with the chosen sources
__device__ __forceinline__ void w_create_segment(Tm& t, uint32_t cell, uint32_t n_new, uint32_t my_new) {
    const DevCfg& c = t.c;
    TmSh* sh = t.sh;
    const int l = lane_id();
    uint32_t slot = sh->hwm;
    if (slot >= (uint32_t)c.seg_cap) {
        if (l == 0) sh->err |= 1u;
        return;
    }
    if ((uint32_t)l < n_new) {
        t.src[(size_t)slot * HTM_MAXSYN + l] = (uint16_t)my_new;
        t.perm[(size_t)slot * HTM_MAXSYN + l] = c.init_perm;
    }
    if (l == 0) {
        uint32_t cm = 0;
        if (c.init_perm >= c.tm_conn) cm = n_new >= 32 ? 0xFFFFFFFFu : ((1u << n_new) - 1u);
        t.conn[slot] = cm;
        t.meta[slot] = make_meta(cell, n_new, 1u, 1u);
        uint32_t* d = t.duty + (size_t)slot * 3;
        d[0] = 1u;
        d[1] = __float_as_uint((float)(1.0 / (double)sh->lrn_iter));
        d[2] = sh->lrn_iter;
        atomicAdd(&sh->bytes, (unsigned long long)(4 + 4 + 12 + 6 * n_new + 1));
        t.nseg[cell] += 1;
        sh->hwm = slot + 1;
        sh->nlive += 1;
    }
    __builtin_amdgcn_wave_barrier();
}

// the new segment of a wave-parallel learning loop at the slot wave 0 gave it
// (hwm and the live count were advanced there, in column order)
__device__ __forceinline__ void w_create_segment_at(Tm& t, uint32_t slot, uint32_t cell, uint32_t n_new,
                                                    uint32_t my_new) {
    const DevCfg& c = t.c;
    TmSh* sh = t.sh;
    const int l = lane_id();
    if ((uint32_t)l < n_new) {
        t.src[(size_t)slot * HTM_MAXSYN + l] = (uint16_t)my_new;
        t.perm[(size_t)slot * HTM_MAXSYN + l] = c.init_perm;
    }
    if (l == 0) {
        uint32_t cm = 0;
        if (c.init_perm >= c.tm_conn) cm = n_new >= 32 ? 0xFFFFFFFFu : ((1u << n_new) - 1u);
        t.conn[slot] = cm;
        t.meta[slot] = make_meta(cell, n_new, 1u, 1u);
        uint32_t* d = t.duty + (size_t)slot * 3;
        d[0] = 1u;
        d[1] = __float_as_uint((float)(1.0 / (double)sh->lrn_iter));
        d[2] = sh->lrn_iter;
        atomicAdd(&sh->bytes, (unsigned long long)(4 + 4 + 12 + 6 * n_new + 1));
        t.nseg[cell] += 1;
    }
    __builtin_amdgcn_wave_barrier();
}

// cells of column col a new segment may go to (getCellForNewSegment's
// candidates: not cell 0 unless K == 1, fewer than maxSegmentsPerCell
// segments), bit = cell in column (wave-uniform)
__device__ __forceinline__ uint32_t w_new_segment_cells(Tm& t, uint32_t col) {
    const DevCfg& c = t.c;
    const int l = lane_id();
    const int K = c.K;
    const int minIdx = K == 1 ? 0 : 1, maxIdx = K == 1 ? 0 : K - 1;
    const bool ok = l >= minIdx && l <= maxIdx && (int)t.nseg[col * K + l] < c.max_segs_per_cell;
    return (uint32_t)__ballot(ok);
}

// getCellForNewSegment with every cell of the column full: free its
// least-used segment (smallest refreshed dutyCycle, then lower cell, then
// slot) and return that cell (minIdx when none qualifies)
__device__ __forceinline__ uint32_t w_cell_full(Tm& t, uint32_t col) {
    const DevCfg& c = t.c;
    TmSh* sh = t.sh;
    const int l = lane_id();
    const int K = c.K;
    const int minIdx = K == 1 ? 0 : 1;
    unsigned long long best = ~0ull;
    const uint32_t hwm = sh->hwm;
    for (uint32_t slot = l; slot < hwm; slot += 64) {
        uint32_t mm = t.meta[slot];
        if (!meta_live(mm)) continue;
        uint32_t cell = meta_cell(mm);
        if (col_of(c, cell) != col) continue;
        uint32_t cic = cell - col * K;
        if ((int)cic < minIdx) continue;
        float dc = seg_dc_update(t.duty, slot, sh->lrn_iter, false);
        unsigned long long key = ((unsigned long long)__float_as_uint(dc) << 32) | ((unsigned long long)cic << 27) | slot;
        best = key < best ? key : best;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        unsigned long long tt = __shfl_xor(best, o, 64);
        best = tt < best ? tt : best;
    }
    if (best == ~0ull || __uint_as_float((uint32_t)(best >> 32)) >= 1.0f) return (uint32_t)minIdx;
    uint32_t slot = (uint32_t)best & 0x7FFFFFFu;
    uint32_t cic = (uint32_t)(best >> 27) & 0x1Fu;
    if (l == 0) {
        uint32_t mm = t.meta[slot];
        t.meta[slot] = mm & ~(1u << 23);
        t.nseg[meta_cell(mm)] -= 1;
        sh->nlive -= 1;
    }
    __builtin_amdgcn_wave_barrier();
    return cic;
}

// _getCellForNewSegment(colIdx) given its candidate cells b
// (w_new_segment_cells); returns the cell index within the column
__device__ __forceinline__ uint32_t w_cell_pick(Tm& t, uint32_t col, uint64_t b) {
    TmSh* sh = t.sh;
    const int l = lane_id();
    uint32_t m = (uint32_t)__popcll(b);
    if (m > 0) {
        uint32_t idx = 0;
        if (l == 0) {
            int32_t f = sh->rf, r = sh->rr;
            idx = rng_u32(sh->rng, f, r, m);
            sh->rf = f;
            sh->rr = r;
        }
        idx = (uint32_t)__builtin_amdgcn_readfirstlane((int)idx);
        // position of the idx-th set bit of b
        uint64_t x = b;
        for (uint32_t k = 0; k < idx; k++) x &= x - 1ull;
        return (uint32_t)(__ffsll((unsigned long long)x) - 1);
    }
    return w_cell_full(t, col);
}

// the same with the draw from the wave's register generator (draw pass)
__device__ __forceinline__ uint32_t w_cell_pick(Tm& t, WGen& g, uint32_t col, uint64_t b) {
    const uint32_t m = (uint32_t)__popcll(b);
    if (m > 0) {
        // Random::getUInt32(m): raw draws are < 2^31, so the rejection never fires
        const uint32_t idx = wgen_raw(g) % m;
        uint64_t x = b;
        for (uint32_t k = 0; k < idx; k++) x &= x - 1ull;
        return (uint32_t)(__ffsll((unsigned long long)x) - 1);
    }
    return w_cell_full(t, col);
}

// _getCellForNewSegment(colIdx); returns the cell index within the column
__device__ __forceinline__ uint32_t w_cell_for_new_segment(Tm& t, uint32_t col) {
    return w_cell_pick(t, col, w_new_segment_cells(t, col));
}

// cells on in `bm` -> sh->cand (<= HTM_MAXACT, ascending)
__device__ __forceinline__ void build_cand(Tm& t, const uint32_t* bm) {
    uint32_t n = wg_bitmap_list(t, bm, t.sh->cand, nullptr, HTM_MAXACT);
    if (threadIdx.x == 0) {
        if (n > HTM_MAXACT) { t.sh->err |= 8u; n = HTM_MAXACT; }
        t.sh->ncand = (int32_t)n;
    }
    __syncthreads();
}

// ---- wave-parallel learning loops (round 5).  A learn phase 1 / 2 loop over
// columns runs in three barrier-separated passes over one record per column:
//   build (every wave, columns round-robin): the RNG-free part -- the best
//       segment's active-synapse mask and the candidates not already on it
//       (_getSegmentActiveSynapses / _chooseCellsToLearnFrom's filter), or a new
//       segment's candidate cells (getCellForNewSegment's filter);
//   draw (wave 0, in NuPIC's column order): only the nupic::Random draws (the new
//       segment's cell, the sample of new synapses) and the ordered appends (the
//       new segment's slot at hwm, the queued update's index);
//   write (every wave): the segment adapt / trim / create, the queued update.
// Columns touch only their own segments and cells, so only the draws and the
// appends need the column order; results are those of the serial loop.
struct __attribute__((aligned(16))) LRec {
    unsigned long long keep;    // candidates (sh->cand positions) not on the segment
    unsigned long long chosen;  // bit i: the i-th kept candidate becomes a new synapse
    uint32_t slot;              // the segment: best match, or the new segment's slot (0xFFFFFFFF: none)
    uint32_t mask;              // active existing synapses; LR_NEW: the candidate cells of the column
    uint32_t idx;               // LR_QUEUE: queued-update index (0xFFFFFFFF: not queued)
    uint16_t col;
    uint8_t kind;               // LR_ADAPT, LR_NEW, LR_QUEUE
    uint8_t cic;                // cell in column
    uint8_t n;                  // new synapses wanted (0: none)
};
static_assert(sizeof(LRec) == 48, "LRec: 12 words (LREC_WORDS)");
enum { LR_ADAPT = 0, LR_NEW = 1, LR_QUEUE = 2 };
// learning scratch in the union region, past the best-match keys (u64[ncol]):
// the records, each wave's new-source list, phase 2's key-column list (u16[ncol])
__device__ __forceinline__ LRec* lrecs(Tm& t) { return reinterpret_cast<LRec*>(t.U + 2 * t.c.ncol); }
__device__ __forceinline__ uint32_t* lnewsrc(Tm& t) {
    return t.U + 2 * t.c.ncol + LREC_N * 12 + wave_id() * HTM_MAXSYN;
}
__device__ __forceinline__ uint16_t* lkeycols(Tm& t) {
    return reinterpret_cast<uint16_t*>(t.U + 2 * t.c.ncol + LREC_WORDS);
}

// build pass of one record: segment `slot` (meta word mw; 0xFFFFFFFF: a new
// segment) against `state`; the wave's lane 0 stores the record
__device__ __forceinline__ void w_rec_build(Tm& t, LRec* r, uint32_t kind, uint32_t col, uint32_t cic, uint32_t slot,
                                            uint32_t mw, const uint32_t* state, bool want_new) {
    TmSh* sh = t.sh;
    const int l = lane_id();
    const bool exist = slot != 0xFFFFFFFFu;
    const uint32_t nsyn = exist ? meta_nsyn(mw) : 0u;
    const uint32_t mysrc = (exist && (uint32_t)l < nsyn) ? (uint32_t)t.src[(size_t)slot * HTM_MAXSYN + l] : 0xFFFFFFFFu;
    const bool act = (exist && (uint32_t)l < nsyn) && bm_get(state, mysrc);
    uint32_t mask = (uint32_t)__ballot(act);
    if (l == 0 && exist) atomicAdd(&sh->bytes, (unsigned long long)(4 + 2 * nsyn));
    const int nw = want_new ? t.c.new_syn - __popc(mask) : 0;
    unsigned long long keep = 0ull;
    if (nw > 0) {
        const int ncand = sh->ncand;
        const uint32_t cv = l < ncand ? sh->cand[l] : 0xFFFFFFFEu;
        bool ok = l < ncand;
        for (uint32_t j = 0; j < nsyn; j++) {  // (j uniform: a register read, not an LDS permute)
            const uint32_t sj = (uint32_t)__builtin_amdgcn_readlane((int)mysrc, (int)j);
            if (cv == sj) ok = false;
        }
        keep = __ballot(ok);
    }
    if (kind == LR_NEW) mask = w_new_segment_cells(t, col);
    if (l == 0) {
        r->keep = keep;
        r->chosen = 0ull;
        r->slot = slot;
        r->mask = mask;
        r->idx = 0xFFFFFFFFu;
        r->col = (uint16_t)col;
        r->kind = (uint8_t)kind;
        r->cic = (uint8_t)cic;
        r->n = (uint8_t)(nw > 0 ? nw : 0);
    }
}

// draw pass (wave 0): records [0, nr) in order
__device__ __forceinline__ void w_rec_draw(Tm& t, LRec* recs, int nr) {
    const DevCfg& c = t.c;
    TmSh* sh = t.sh;
    const int l = lane_id();
    // lane j < nr holds record j's inputs (one LDS round trip for all) and
    // collects its outputs; the appends' counters stay in scalar registers
    unsigned long long kk = 0ull;
    uint32_t kmask = 0u, kcol = 0u, kkn = 0u;
    if (l < nr) {
        const LRec& r = recs[l];
        kk = r.keep;
        kmask = r.mask;
        kcol = r.col;
        kkn = (uint32_t)r.kind | ((uint32_t)r.n << 8);
    }
    unsigned long long och = 0ull;
    uint32_t oslot = 0xFFFFFFFFu, ocic = 0u, oidx = 0xFFFFFFFFu;
    uint32_t hwm = (uint32_t)__builtin_amdgcn_readfirstlane(sh->hwm);
    uint32_t nupd = (uint32_t)__builtin_amdgcn_readfirstlane(sh->n_upd);
    uint32_t nnew = 0u, err = 0u;
    WGen g = wgen_load(t);
    for (int j = 0; j < nr; j++) {
        const uint32_t kj = (uint32_t)__builtin_amdgcn_readlane((int)kkn, j);
        const uint32_t kind = kj & 0xFFu, n = kj >> 8;
        const unsigned long long keep =
            (unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)kk, j) |
            ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(kk >> 32), j) << 32);
        const uint32_t mask = (uint32_t)__builtin_amdgcn_readlane((int)kmask, j);
        uint32_t slot = 0xFFFFFFFFu, cic = 0u;
        if (kind == LR_NEW) {
            const uint32_t col = (uint32_t)__builtin_amdgcn_readlane((int)kcol, j);
            cic = w_cell_pick(t, g, col, (uint64_t)mask);  // (the all-cells-full path reads sh->hwm)
            if (hwm >= (uint32_t)c.seg_cap) {
                err |= 1u;
            } else {
                slot = hwm++;
                nnew++;
                if (l == 0) sh->hwm = hwm;
            }
        }
        const uint32_t m = (uint32_t)__popcll(keep);
        unsigned long long chosen = 0ull;
        if (n > 0u && m > 0u) {
            if (m <= n) {
                chosen = (m == 64) ? ~0ull : ((1ull << m) - 1ull);
            } else {
#ifdef HTM_STAMPS
                const uint64_t ts0_ = __builtin_amdgcn_s_memtime();
#endif
                chosen = wgen_sample(g, m, n);
                COUNT(t, SC_LSAMPLES, 1);
#ifdef HTM_STAMPS
                COUNT(t, SC_LSAMPLECYC, __builtin_amdgcn_s_memtime() - ts0_);
#endif
            }
        }
        uint32_t idx = 0xFFFFFFFFu;
        if (kind == LR_QUEUE && (mask != 0u || chosen != 0ull)) {
            if (nupd >= (uint32_t)c.upd_cap) err |= 2u;
            else idx = nupd++;
        }
        if (l == j) {
            och = chosen;
            oslot = slot;
            ocic = cic;
            oidx = idx;
        }
    }
    wgen_store(t, g);
    if (l < nr) {
        LRec& r = recs[l];
        r.chosen = och;
        r.idx = oidx;
        if ((kkn & 0xFFu) == LR_NEW) {
            r.slot = oslot;
            r.cic = (uint8_t)ocic;
        }
    }
    if (l == 0) {
        sh->hwm = hwm;
        sh->nlive += nnew;
        sh->n_upd = (int32_t)nupd;
        if (err) sh->err |= err;
    }
}

// the new sources of a drawn record: lane k (< *n_new) gets the k-th chosen
// candidate (ascending, as _chooseCellsToLearnFrom lists them)
__device__ __forceinline__ uint32_t w_rec_sources(Tm& t, unsigned long long keep, unsigned long long chosen,
                                                  uint32_t* n_new) {
    const int l = lane_id();
    uint32_t* ns = lnewsrc(t);
    const bool kept = l < t.sh->ncand && ((keep >> l) & 1ull);
    const uint32_t pos = ballot_rank(keep);
    const bool sel = kept && ((chosen >> pos) & 1ull);
    const uint64_t sb = __ballot(sel);
    *n_new = (uint32_t)__popcll(sb);
    if (sel) ns[ballot_rank(sb)] = t.sh->cand[l];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const uint32_t v = (uint32_t)l < *n_new ? ns[l] : 0u;
    __builtin_amdgcn_wave_barrier();  // (the next record's list overwrites ns)
    return v;
}

// _processSegmentUpdates(activeColumns)
__device__ __forceinline__ void process_segment_updates(Tm& t, const uint16_t* cols, int nA) {
    const DevCfg& c = t.c;
    TmSh* sh = t.sh;
    wg_clear(t.flags, c.nw);
    __syncthreads();
    for (int a = threadIdx.x; a < nA; a += TM_NT) atomicOr(&t.flags[cols[a] >> 5], 1u << (cols[a] & 31));
    __syncthreads();
    const int n = sh->n_upd;
    uint32_t* tflag = t.U;
    for (int k = wave_id(); k < n; k += TM_NWAVES) {
        const htm_tm_update& e = t.upd[k];
        uint32_t col = e.col;
        bool doit = ((t.flags[col >> 5] >> (col & 31)) & 1u) && (sh->lrn_iter - e.date <= (uint32_t)c.upd_valid);
        bool trim = false;
        if (doit) {
            uint32_t nn = e.n_new;
            uint32_t my_new = (uint32_t)lane_id() < nn ? e.new_src[lane_id()] : 0u;
            trim = w_adapt_existing(t, e.slot, e.active_mask, nn, my_new);
        }
        if (lane_id() == 0) tflag[k] = trim ? 1u : 0u;
    }
    __syncthreads();
    for (int k = wave_id(); k < n; k += TM_NWAVES)
        if (tflag[k]) w_trim_segment(t, t.upd[k].slot);
    __syncthreads();
    if (threadIdx.x == 0) sh->n_upd = 0;
    __syncthreads();
}

// _learnPhase1(activeColumns, readOnly)
__device__ __forceinline__ bool learn_phase1(Tm& t, const uint16_t* cols, int nA, bool ro) {
    const DevCfg& c = t.c;
    TmSh* sh = t.sh;
    const int K = c.K;
    wg_clear(t.lrnA, c.cw);
    wg_clear(t.flags, c.nw);
    __syncthreads();
    uint32_t nun = 0;
    for (int a = threadIdx.x; a < nA; a += TM_NT) {
        uint32_t col = cols[a];
        uint32_t f = bm_field(t.lrnP1, col * K, K);
        int pc = __popc(f);
        if (pc == 1) {
            bm_or_field(t.lrnA, col * K, K, f);
        } else {
            nun++;
            atomicOr(&t.flags[col >> 5], 1u << (col & 31));
            if (pc > 1) atomicOr(&sh->err, 4u);
        }
    }
    nun = wg_sum(sh, nun);
    const bool inSeq = (int)nun < nA / 2;
    if (ro || nun == 0) return inSeq;
    wg_clear(t.U, 2 * c.ncol);
    __syncthreads();
    STAMP(t, SB_LEARN);
    scan_best(t, t.lrnA1, c.min_thr, t.flags);
    __syncthreads();
    STAMP(t, SB_LSCAN);
    build_cand(t, t.lrnA1);
    STAMP(t, SB_LEARN);
    const unsigned long long* keys = reinterpret_cast<const unsigned long long*>(t.U);
#ifdef HTM_LEARN_SERIAL
    // (A/B builds: the round-4 loop, wave 0 doing every column in turn)
    if (wave_id() == 0) {
        for (int a = 0; a < nA; a++) {
            uint32_t col = cols[a];
            if (!((t.flags[col >> 5] >> (col & 31)) & 1u)) continue;
            unsigned long long key = keys[col];
            bool seqseg = false;
            uint32_t slot = 0, cic = 0;
            if (key) {
                slot = key_slot(key);
                cic = key_cic(key);
                seqseg = meta_seq(t.meta[slot]) != 0u;
            }
            COUNT(t, SC_LP1COLS, 1);
            STAMP(t, SB_LW);
            if (key && seqseg) {
                if (lane_id() == 0) bm_or_field(t.lrnA, col * K + cic, 1, 1u);
                WUpd u = w_build_update(t, slot, t.lrnA1, true);
                STAMP(t, SB_LWB);
                bool trim = w_adapt_existing(t, slot, u.mask, u.n_new, u.my_new);
                if (trim) w_trim_segment(t, slot);
                STAMP(t, SB_LWW);
            } else {
                cic = w_cell_for_new_segment(t, col);
                STAMP(t, SB_LWS);
                if (lane_id() == 0) bm_or_field(t.lrnA, col * K + cic, 1, 1u);
                WUpd u = w_build_update(t, 0xFFFFFFFFu, t.lrnA1, true);
                STAMP(t, SB_LWB);
                w_create_segment(t, col * K + cic, u.n_new, u.my_new);
                STAMP(t, SB_LWW);
            }
        }
    }
#else
    // the flagged columns in cols order (nA <= 64: one ballot; every wave the same)
    LRec* recs = lrecs(t);
    const int l = lane_id();
    const uint64_t fb =
        __ballot(l < nA && ((t.flags[cols[l < nA ? l : 0] >> 5] >> (cols[l < nA ? l : 0] & 31)) & 1u));
    const int nf = __popcll(fb);
    {
        uint64_t x = fb;
        for (int j = 0; x; j++, x &= x - 1ull) {
            if ((j & (TM_NWAVES - 1)) != wave_id()) continue;
            const uint32_t col = cols[__ffsll((unsigned long long)x) - 1];
            const unsigned long long key = keys[col];
            uint32_t slot = 0xFFFFFFFFu, cic = 0, mw = 0, kind = LR_NEW;
            if (key) {
                const uint32_t ks = key_slot(key);
                mw = t.meta[ks];
                if (meta_seq(mw)) {
                    kind = LR_ADAPT;
                    slot = ks;
                    cic = key_cic(key);
                }
            }
            w_rec_build(t, &recs[j], kind, col, cic, slot, mw, t.lrnA1, true);
            COUNT(t, SC_LP1COLS, 1);
        }
    }
    __syncthreads();
    STAMP(t, SB_LWB);
    if (wave_id() == 0) w_rec_draw(t, recs, nf);
    __syncthreads();
    STAMP(t, SB_LWS);
    for (int j = wave_id(); j < nf; j += TM_NWAVES) {
        const LRec& r = recs[j];
        const uint32_t col = r.col, cic = r.cic, slot = r.slot;
        uint32_t nn;
        const uint32_t my_new = w_rec_sources(t, r.keep, r.chosen, &nn);
        if (l == 0) bm_or_field(t.lrnA, col * K + cic, 1, 1u);
        if (r.kind == LR_ADAPT) {
            if (w_adapt_existing(t, slot, r.mask, nn, my_new)) w_trim_segment(t, slot);
        } else if (slot != 0xFFFFFFFFu) {
            w_create_segment_at(t, slot, col * K + cic, nn, my_new);
        }
    }
    __syncthreads();
    STAMP(t, SB_LWW);
#endif
    __syncthreads();
    STAMP(t, SB_LW);
    return inSeq;
}

// The rest of _learnPhase2 once its best-match keys are in U (u64 [ncol]):
// lrnPredictedState into `out` (cleared by the caller) and, unless read-only,
// the queued segment updates of the columns with a key -- active synapses and
// new-synapse candidates against `state` (lrnActiveState of the step the phase
// belongs to), dated `date`.  The step's own phase: (lrnA, lrnP, lrn_iter); the
// previous step's deferred one (lp2_finish): (lrnA1, lrnP1, lrn_iter - 1).
__device__ __forceinline__ void learn_phase2_post(Tm& t, const uint32_t* state, uint32_t* out, uint32_t date,
                                                  bool ro) {
    const DevCfg& c = t.c;
    TmSh* sh = t.sh;
    const int K = c.K;
    const unsigned long long* keys = reinterpret_cast<const unsigned long long*>(t.U);
    for (int col = threadIdx.x; col < c.ncol; col += TM_NT) {
        unsigned long long key = keys[col];
        if (key) bm_or_field(out, (uint32_t)col * K + key_cic(key), 1, 1u);
    }
    __syncthreads();
    if (ro) return;
    build_cand(t, state);
    STAMP(t, SB_LEARN);
#ifdef HTM_LEARN_SERIAL
    if (wave_id() == 0) {
        for (int base = 0; base < c.ncol; base += 64) {
            uint64_t b = __ballot(keys[base + lane_id()] != 0ull);
            while (b) {
                int bit = __ffsll((unsigned long long)b) - 1;
                b &= b - 1ull;
                uint32_t col = (uint32_t)(base + bit);
                unsigned long long key = keys[col];
                uint32_t slot = key_slot(key), act = key_act(key);
                COUNT(t, SC_LP2COLS, 1);
                STAMP(t, SB_LW);
                WUpd u = w_build_update(t, slot, state, act < (uint32_t)c.new_syn);
                STAMP(t, SB_LWB);
                if (u.mask == 0u && u.n_new == 0u) continue;
                int idx = sh->n_upd;
                if (idx >= c.upd_cap) {
                    if (lane_id() == 0) sh->err |= 2u;
                    continue;
                }
                htm_tm_update& e = t.upd[idx];
                if ((uint32_t)lane_id() < u.n_new) e.new_src[lane_id()] = (uint16_t)u.my_new;
                if (lane_id() == 0) {
                    e.slot = slot;
                    e.col = (uint16_t)col;
                    e.cell = (uint8_t)key_cic(key);
                    e.n_new = (uint8_t)u.n_new;
                    e.active_mask = u.mask;
                    e.date = date;
                    sh->n_upd = idx + 1;
                    // queued entry written now and read back at the next step
                    atomicAdd(&sh->bytes, (unsigned long long)(2 * (16 + 2 * u.n_new)));
                }
                __builtin_amdgcn_wave_barrier();
                STAMP(t, SB_LWW);
            }
        }
    }
#else
    // the columns with a best segment, ascending: thread x lists columns
    // [x * per, (x + 1) * per)
    uint16_t* kc = lkeycols(t);
    const int per = (c.ncol + TM_NT - 1) / TM_NT;
    const int c0 = threadIdx.x * per;
    uint32_t cnt = 0;
    for (int k = 0; k < per; k++)
        if (c0 + k < c.ncol && keys[c0 + k] != 0ull) cnt++;
    uint32_t nk;
    uint32_t pos = wg_excl_scan(sh, cnt, &nk);
    for (int k = 0; k < per; k++)
        if (c0 + k < c.ncol && keys[c0 + k] != 0ull) kc[pos++] = (uint16_t)(c0 + k);
    __syncthreads();
    LRec* recs = lrecs(t);
    const int l = lane_id();
    for (uint32_t b0 = 0; b0 < nk; b0 += LREC_N) {
        const int nb = nk - b0 < LREC_N ? (int)(nk - b0) : LREC_N;
        for (int j = wave_id(); j < nb; j += TM_NWAVES) {
            const uint32_t col = kc[b0 + j];
            const unsigned long long key = keys[col];
            const uint32_t slot = key_slot(key);
            w_rec_build(t, &recs[j], LR_QUEUE, col, key_cic(key), slot, t.meta[slot], state,
                        key_act(key) < (uint32_t)c.new_syn);
            COUNT(t, SC_LP2COLS, 1);
        }
        __syncthreads();
        STAMP(t, SB_LWB);
        if (wave_id() == 0) w_rec_draw(t, recs, nb);
        __syncthreads();
        STAMP(t, SB_LWS);
        for (int j = wave_id(); j < nb; j += TM_NWAVES) {
            const LRec& r = recs[j];
            const uint32_t idx = r.idx;
            uint32_t nn;
            const uint32_t my_new = w_rec_sources(t, r.keep, r.chosen, &nn);
            if (idx == 0xFFFFFFFFu) continue;
            htm_tm_update& e = t.upd[idx];
            if ((uint32_t)l < nn) e.new_src[l] = (uint16_t)my_new;
            if (l == 0) {
                e.slot = r.slot;
                e.col = r.col;
                e.cell = r.cic;
                e.n_new = (uint8_t)nn;
                e.active_mask = r.mask;
                e.date = date;
                // queued entry written now and read back at the next step
                atomicAdd(&sh->bytes, (unsigned long long)(2 * (16 + 2 * nn)));
            }
        }
        __syncthreads();
        STAMP(t, SB_LWW);
    }
#endif
    __syncthreads();
    STAMP(t, SB_LW);
}

// _learnPhase2(readOnly).  A read-only pass of a learn backtrack (`next`: the
// columns of the pattern after it) computes lrnPredictedState only for those
// columns: its one reader is the next pattern's read-only _learnPhase1, which
// looks at the next pattern's columns alone (learn_backtrack_from); every
// pass that writes recomputes lrnP in full before anything else reads it.
// The best-match search then reads the rows of those columns' segments only
// (scan_best's flagged form) instead of the whole pool.
__device__ __forceinline__ void learn_phase2(Tm& t, bool ro, const uint16_t* next = nullptr, int nnext = 0) {
    const DevCfg& c = t.c;
    TmSh* sh = t.sh;
    if (threadIdx.x == 0) sh->st[2]++;
    wg_clear(t.lrnP, c.cw);
    wg_clear(t.U, 2 * c.ncol);
    const bool part = ro && next != nullptr;
    if (part) {
        wg_clear(t.flags, c.nw);
        __syncthreads();
        for (int a = threadIdx.x; a < nnext; a += TM_NT) atomicOr(&t.flags[next[a] >> 5], 1u << (next[a] & 31));
    }
    __syncthreads();
    STAMP(t, SB_LEARN);
    scan_best(t, t.lrnA, c.act_thr, part ? t.flags : nullptr);
    __syncthreads();
    STAMP(t, SB_LSCAN);
    learn_phase2_post(t, t.lrnA, t.lrnP, sh->lrn_iter, ro);
}

// The final _learnPhase2 of a learning step is deferred (DevCfg::lp2_defer):
// the step ends with it pending (TmSh::lp2p, htm_tm_header::lp2_pending) and
// the next step completes it -- its best-match count rides on that step's
// first pool scan (collect_scan, keys in Tm::lkey), its lrnPredictedState
// goes straight into lrnP1, and its queued updates and nupic::Random draws
// happen after that step's inference and before its learning.  Nothing in
// between reads or writes what the phase reads or writes: inference touches
// no learn state, queue or generator, and only dutyCycle records of the
// segments; a step's learning starts with processSegmentUpdates, after this.
// Saves one full pool scan per learning step.  `date`: the deferred phase's
// lrn_iter.  A pending phase whose keys were not counted (no pool scan ran)
// scans here.  The engine completes a pending phase (tm_lp2_finish_kernel)
// before anything reads the state or steps without learning.
__device__ __forceinline__ void lp2_finish(Tm& t, uint32_t date) {
    const DevCfg& c = t.c;
    TmSh* sh = t.sh;
    if (threadIdx.x == 0) sh->st[2]++;
    wg_clear(t.lrnP1, c.cw);
    unsigned long long* keys = reinterpret_cast<unsigned long long*>(t.U);
    if (!sh->lp2s) {
        wg_clear(t.U, 2 * c.ncol);
        __syncthreads();
        scan_best(t, t.lrnA1, c.act_thr, nullptr);
    } else {
        for (int col = threadIdx.x; col < c.ncol; col += TM_NT) {
            const uint32_t k = t.lkey[col];
            keys[col] = k ? ((unsigned long long)(k >> 26) << 40) | ((unsigned long long)((k >> 21) & 31u) << 32) |
                                (unsigned long long)(0xFFFFFFFFu - (0x1FFFFFu - (k & 0x1FFFFFu)))
                          : 0ull;
        }
    }
    __syncthreads();
    STAMP(t, SB_LSCAN);
    learn_phase2_post(t, t.lrnA1, t.lrnP1, date, false);
    if (threadIdx.x == 0) {
        sh->lp2p = 0;
        sh->lp2s = 0;
    }
    __syncthreads();
}

// start cells (cell 0) of the given columns into lrnA
__device__ __forceinline__ void set_start_cells(Tm& t, uint32_t* bm, const uint16_t* cols, int nA) {
    wg_clear(bm, t.c.cw);
    __syncthreads();
    for (int a = threadIdx.x; a < nA; a += TM_NT) bm_or_field(bm, (uint32_t)cols[a] * t.c.K, 1, 1u);
    __syncthreads();
}

// _learnBacktrackFrom(startOffset, readOnly)
__device__ __forceinline__ bool learn_backtrack_from(Tm& t, int start, bool ro) {
    TmSh* sh = t.sh;
    const int cw = t.c.cw;
    const int numPrev = sh->n_lrn_pat;
    const int cur = numPrev - 1;
    if (!ro) {
        if (threadIdx.x == 0) sh->n_upd = 0;
        __syncthreads();
    }
    bool inSeq = true;
    for (int off = start; off < numPrev; off++) {
        STAMP(t, SB_LEARN);
        wg_copy(t.lrnP1, t.lrnP, cw);
        wg_copy(t.lrnA1, t.lrnA, cw);
        __syncthreads();
        STAMP(t, SB_LBT);
        const uint16_t* pat = lrn_pat(t, off);
        const int len = lrn_len(t, off);
        if (!ro) {
            process_segment_updates(t, pat, len);
            STAMP(t, SB_LUPD);
        }
        if (off == start) {
            set_start_cells(t, t.lrnA, pat, len);
            inSeq = true;
        } else {
            inSeq = learn_phase1(t, pat, len, ro);
        }
        if (!inSeq || off == cur) break;
#ifdef HTM_LP2_FULL_RO  // (A/B builds: read-only passes over every column)
        learn_phase2(t, ro);
#else
        if (ro) learn_phase2(t, true, lrn_pat(t, off + 1), lrn_len(t, off + 1));
        else learn_phase2(t, false);
#endif
    }
    return inSeq;
}

// _learnBacktrack(): steps backtracked, 0 on failure
__device__ __forceinline__ int learn_backtrack(Tm& t) {
    TmSh* sh = t.sh;
    const int numPrev = sh->n_lrn_pat - 1;
    if (numPrev <= 0) return 0;
    if (threadIdx.x == 0) sh->st[3]++;
    uint32_t bad = 0;
    bool inSeq = false;
    int start;
    for (start = 0; start < numPrev; start++) {
        inSeq = learn_backtrack_from(t, start, true);
        if (inSeq) break;
        bad |= 1u << start;
    }
    if (!inSeq) {
        if (threadIdx.x == 0) sh->n_lrn_pat = 0;
        __syncthreads();
        return 0;
    }
    (void)learn_backtrack_from(t, start, false);
    if (threadIdx.x == 0) {
        int npop = 0;
        for (int i = 0; i < numPrev; i++) {
            if (((bad >> i) & 1u) || i <= start) npop++;
            else break;
        }
        sh->lrn_head = (sh->lrn_head + npop) % HTM_MAXPAT;
        sh->n_lrn_pat -= npop;
    }
    __syncthreads();
    return numPrev - start;
}

// _updateLearningState(activeColumns)
__device__ __forceinline__ void update_learning(Tm& t) {
    const DevCfg& c = t.c;
    TmSh* sh = t.sh;
    // lrnA1 / lrnP1 hold time t-1 (loaded at entry)
    if (threadIdx.x == 0) {
        if (c.max_lrn_bt > 0) {
            if (sh->n_lrn_pat > c.max_lrn_bt) {
                sh->lrn_head = (sh->lrn_head + 1) % HTM_MAXPAT;
                sh->n_lrn_pat--;
            }
            int slot = (sh->lrn_head + sh->n_lrn_pat) % HTM_MAXPAT;
            sh->lrn_len[slot] = (uint16_t)sh->nA;
            sh->ti[1] = slot;
            sh->n_lrn_pat++;
        } else {
            sh->ti[1] = -1;
        }
    }
    __syncthreads();
    if (sh->ti[1] >= 0)
        for (int a = threadIdx.x; a < sh->nA; a += TM_NT) t.lrnpat[sh->ti[1]][a] = sh->act[a];
    __syncthreads();
    STAMP(t, SB_LEARN);
    process_segment_updates(t, sh->act, sh->nA);
    STAMP(t, SB_LUPD);
    if (threadIdx.x == 0) {
        if (sh->pam > 0) sh->pam--;
        sh->lsl++;
    }
    __syncthreads();
    if (!sh->reset) {
        bool inSeq = learn_phase1(t, sh->act, sh->nA, false);
        if (inSeq && threadIdx.x == 0) sh->pam = c.pam_len;
        __syncthreads();
    }
    if (sh->reset || sh->pam == 0 || (c.max_seq_len != 0 && sh->lsl >= c.max_seq_len)) {
        if (threadIdx.x == 0) {
            int seqLength = sh->pam == 0 ? sh->lsl - c.pam_len : sh->lsl;
            double alpha = sh->lrn_iter < 100 ? 0.5 : 0.1;
            sh->avg_lsl = (1.0 - alpha) * sh->avg_lsl + alpha * (double)seqLength;
        }
        __syncthreads();
        int backSteps = 0;
        if (!sh->reset) backSteps = learn_backtrack(t);
        if (sh->reset || backSteps == 0) {
            backSteps = 0;
            set_start_cells(t, t.lrnA, sh->act, sh->nA);
            if (threadIdx.x == 0) sh->n_lrn_pat = 0;
        }
        if (threadIdx.x == 0) {
            sh->pam = c.pam_len;
            sh->lsl = backSteps;
            sh->n_upd = 0;
        }
        __syncthreads();
    }
    if (c.lp2_defer) {
        // the final learn phase 2: completed by the next step (lp2_finish)
        if (threadIdx.x == 0) {
            sh->lp2p = 1;
            sh->lp2s = 0;
        }
        __syncthreads();
    } else {
        learn_phase2(t, false);
    }
}

// stable compaction of live segments (slot order preserved) so that a
// learning step always has seg_reserve free slots
__device__ __forceinline__ void compact_pool(Tm& t) {
    TmSh* sh = t.sh;
    const uint32_t hwm = sh->hwm;
    uint32_t base = 0;
    // pass 1: new slot of every live segment -> q1
    for (uint32_t c0 = 0; c0 < hwm; c0 += TM_NT) {
        uint32_t slot = c0 + threadIdx.x;
        bool live = slot < hwm && meta_live(t.meta[slot]);
        uint32_t tot;
        uint32_t pos = wg_excl_scan(sh, live ? 1u : 0u, &tot);
        if (slot < hwm) t.q1[slot] = live ? base + pos : 0xFFFFFFFFu;
        base += tot;
    }
    __syncthreads();
    // pass 2: move in increasing slot order (destinations never exceed sources)
    for (uint32_t c0 = 0; c0 < hwm; c0 += TM_NT) {
        uint32_t slot = c0 + threadIdx.x;
        uint32_t ns = slot < hwm ? t.q1[slot] : 0xFFFFFFFFu;
        uint32_t mm = 0, cm = 0, d0 = 0, d1 = 0, d2 = 0;
        uint4 sv[4];
        float4 pv[8];
#pragma unroll
        for (int k = 0; k < 4; k++) sv[k] = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int k = 0; k < 8; k++) pv[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ns != 0xFFFFFFFFu) {
            mm = t.meta[slot];
            cm = t.conn[slot];
            d0 = t.duty[(size_t)slot * 3];
            d1 = t.duty[(size_t)slot * 3 + 1];
            d2 = t.duty[(size_t)slot * 3 + 2];
            const uint4* sr = reinterpret_cast<const uint4*>(t.src + (size_t)slot * HTM_MAXSYN);
            const float4* pr = reinterpret_cast<const float4*>(t.perm + (size_t)slot * HTM_MAXSYN);
#pragma unroll
            for (int k = 0; k < 4; k++) sv[k] = sr[k];
#pragma unroll
            for (int k = 0; k < 8; k++) pv[k] = pr[k];
        }
        __syncthreads();
        if (ns != 0xFFFFFFFFu && ns != slot) {
            t.meta[ns] = mm;
            t.conn[ns] = cm;
            t.duty[(size_t)ns * 3] = d0;
            t.duty[(size_t)ns * 3 + 1] = d1;
            t.duty[(size_t)ns * 3 + 2] = d2;
            uint4* sw = reinterpret_cast<uint4*>(t.src + (size_t)ns * HTM_MAXSYN);
            float4* pw = reinterpret_cast<float4*>(t.perm + (size_t)ns * HTM_MAXSYN);
#pragma unroll
            for (int k = 0; k < 4; k++) sw[k] = sv[k];
#pragma unroll
            for (int k = 0; k < 8; k++) pw[k] = pv[k];
        }
        __syncthreads();
    }
    // queued updates follow their segments
    for (int k = threadIdx.x; k < sh->n_upd; k += TM_NT) t.upd[k].slot = t.q1[t.upd[k].slot];
    for (uint32_t slot = base + threadIdx.x; slot < hwm; slot += TM_NT) t.meta[slot] = 0u;
    __syncthreads();
    if (threadIdx.x == 0) sh->hwm = base;
    __syncthreads();
}

// ---------------------------------------------------------------------------
// One BacktrackingTM.compute + raw anomaly of stream s by the calling
// workgroup (TM_NT threads), LDS at `lds` (tm_layout).
// Bind the LDS regions and stream s's buffers: the model (SP, segment pool,
// frozen index) of stream s (the fleet's shared instance), the per-stream
// scratch (qualifying lists, backtrack backups) of stream `scr` -- a helper
// replaying another stream's backtrack uses its own scratch.
template <bool LEARN, bool FROZEN>
__device__ __forceinline__ void tm_bind(Tm& t, const DevCfg& c, const TmBufs& b, int s, int scr, uint8_t* lds) {
    const TmLayout L = tm_layout(c, LEARN, FROZEN);
    t.c = c;
    t.s = s;
    t.sh = reinterpret_cast<TmSh*>(lds);
    uint32_t* bmr = reinterpret_cast<uint32_t*>(lds + L.off_bm);
    t.infA = bmr;
    t.infP = bmr + c.cw;
    t.infP1 = bmr + 2 * c.cw;
    t.lrnA = LEARN ? bmr + 3 * c.cw : nullptr;
    t.lrnA1 = LEARN ? bmr + 4 * c.cw : nullptr;
    t.lrnP = LEARN ? bmr + 5 * c.cw : nullptr;
    t.lrnP1 = LEARN ? bmr + 6 * c.cw : nullptr;
    t.colconf = reinterpret_cast<float*>(lds + L.off_conf);
    t.flags = reinterpret_cast<uint32_t*>(lds + L.off_flags);
    t.U = reinterpret_cast<uint32_t*>(lds + L.off_U);
    t.lkey = LEARN ? reinterpret_cast<uint32_t*>(lds + L.off_lkey) : nullptr;
    t.lrnpat = LEARN ? reinterpret_cast<uint16_t(*)[HTM_MAXACT]>(lds + L.off_lpat) : nullptr;
    const size_t sc = (size_t)c.seg_cap;
    // model buffers: the stream's own, or the fleet's shared instance 0
    // (frozen inference writes only the segments' dutyCycle cache, with the
    // value every stream computes for it, so sharing is race-free)
    const size_t ms = (size_t)model_stream(c, s);
    t.meta = b.seg_meta + ms * sc;
    t.src = b.seg_src + ms * sc * HTM_MAXSYN;
    t.perm = b.seg_perm + ms * sc * HTM_MAXSYN;
    t.conn = b.seg_conn + ms * sc;
    t.duty = b.seg_duty + ms * sc * 3;
    t.nseg = b.cell_nseg + ms * c.ncells;
    t.upd = b.upd + ms * c.upd_cap;
    t.sbm = b.scr_bm + (size_t)scr * 5 * c.cw;
    t.sconf = b.scr_conf + (size_t)scr * c.ncol;
    t.q1 = b.scr_q + (size_t)scr * c.q_cap;
    t.q2 = b.scr_q2 + (size_t)scr * c.q_cap;
    if (FROZEN) {
        t.fxoff = b.fx_off + ms * (size_t)c.fx_noff;
        t.fxent = b.fx_ent + b.fx_base[ms];
        t.fxrec = b.fx_rec + ms * sc;
        t.fxrslot = b.fx_rslot + ms * sc;
        t.fxpcell = b.fx_pcell + ms * c.fx_pcap;
        t.np = b.fx_np[ms];
        t.nr = b.fx_nr[ms];
    } else {
        t.fxoff = nullptr;
        t.fxent = nullptr;
        t.fxrec = nullptr;
        t.fxrslot = nullptr;
        t.fxpcell = nullptr;
        t.np = 0;
        t.nr = 0;
    }
    t.tb = &b;
    t.defer = FROZEN && b.fx_dlog != nullptr;
    t.dn = t.df = 0;
    t.rh = t.rl = 0;
    t.nsum = 0;
    if (threadIdx.x == 0) t.sh->acc[0] = t.sh->acc[1] = t.sh->acc[2] = 0u;  // (a barrier follows before any use)
}

// Replay one deferred-log entry of stream s (ring slot i, `len` cells): its
// active cells, the counting of rank window `win` (-1: every window), the
// qualifying segments' first dutyCycle() record writes (phase2_duty_only).
// The calling workgroup's qualifying list is fx_fq's row `worker`.  Used by
// tm_fx_flush_kernel.
__device__ __forceinline__ void fx_replay_entry(const DevCfg& c, const TmBufs& b, int s, uint32_t i, uint32_t len,
                                                int win, uint32_t worker, uint8_t* lds) {
    Tm t;
    tm_bind<false, true>(t, c, b, s, s, lds);
    t.q1 = b.fx_fq + (size_t)worker * c.q_cap;
    t.defer = false;
    TmSh* sh = t.sh;
    if (threadIdx.x == 0) {
        sh->qn = 0;
        sh->bytes = 0;
        sh->lrn_iter = b.hdr[s].lrn_iter;  // frozen while TM learning is off
        sh->p1_n = -1;                      // infA comes from the log, not from a phase 1
    }
    wg_clear(t.infA, c.cw);
    __syncthreads();
    const uint16_t* cl = b.fx_dlog + ((size_t)s * (uint32_t)c.fx_dcap + i) * fx_dstride(c);
    for (uint32_t k = threadIdx.x; k < len; k += TM_NT) {
        const uint32_t cell = cl[k];
        if (cell < (uint32_t)c.ncells) atomicOr(&t.infA[cell >> 5], 1u << (cell & 31));
    }
    __syncthreads();
    collect_frozen(t, c.act_thr, FX_WIN, win);
    __syncthreads();
    if (threadIdx.x == 0 && (uint32_t)sh->qn > (uint32_t)c.q_cap) {
        atomicOr(&b.fx_fwork[1], FX_ERR_QCAP);  // qualifying-list overflow, as in the step (htm_status)
        sh->qn = c.q_cap;
    }
    __syncthreads();
    phase2_duty_only(t);
}

// Write the inference state back to HBM without reading anything: the
// infActiveState and infPredictedState bitmaps whole (coalesced 16-byte
// stores; a step changes the words of ~80 columns of each, which as scattered
// 4-byte stores cost a 32-byte sector apiece -- the same bytes, plus a read of
// the old words to find them), and colConfidence PACKED: gnz[0..nw) is the
// bitmap of its nonzero columns and gval[0..n) their values in ascending
// column order (one contiguous run of stores, not a scatter over the dense
// columns); gnz[nw] == 1 says the packed form is current (the host densifies
// it into TmBufs::colconf before it reads or replaces the state, then clears
// the flag, and the next step starts from the dense copy).  Uses t.flags and
// the head of t.U (free after the TM step).  Returns the bytes this thread
// moved.  Contains barriers.
// (A/B builds, -DHTM_WB_SC1: the write-back's stores as agent-scope relaxed
// atomic stores -- global_store sc1, which leave the XCD L2 at once instead of
// staying dirty for the end-of-kernel writeback)
#ifdef HTM_WB_SC1
#define WB_ST(p, v) __hip_atomic_store((p), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
#else
#define WB_ST(p, v) (*(p) = (v))
#endif
__device__ __forceinline__ uint32_t write_back_inference(Tm& t, uint32_t* gbm, float* gval, uint32_t* gnz) {
    const DevCfg& c = t.c;
    uint32_t* nzb = t.flags;  // the new bitmap
    uint32_t* woff = t.U;     // packed position of each bitmap word's first column
    // nonzero-column bitmap of the LDS colConfidence (ballots over 64 columns)
    for (int col0 = wave_id() * 64; col0 < c.ncol; col0 += TM_NT) {
        const int col = col0 + lane_id();
        const uint64_t bal = __ballot(col < c.ncol && t.colconf[col] != 0.0f);
        if (lane_id() == 0) {
            nzb[col0 >> 5] = (uint32_t)bal;
            if (col0 + 32 < c.ncol) nzb[(col0 >> 5) + 1] = (uint32_t)(bal >> 32);
        }
    }
    // the cell bitmaps meanwhile (they are final): consecutive words per lane,
    // 256 contiguous bytes per wave store (16-byte lanes through these LDS
    // pointers trip an LLVM gfx950 verifier error in the paged kernel)
    uint32_t wb = 0;
    for (int w = threadIdx.x; w < c.cw; w += TM_NT) {
        WB_ST(&gbm[w], t.infA[w]);
        WB_ST(&gbm[c.cw + w], t.infP[w]);
        wb += 8;
    }
    __syncthreads();
    // word offsets: exclusive prefix of the words' popcounts (nw <= 128 < TM_NT)
    uint32_t tot;
    const uint32_t mine = threadIdx.x < (uint32_t)c.nw ? (uint32_t)__popc(nzb[threadIdx.x]) : 0u;
    const uint32_t off = wg_excl_scan(t.sh, mine, &tot);
    if (threadIdx.x < (uint32_t)c.nw) {
        woff[threadIdx.x] = off;
        WB_ST(&gnz[threadIdx.x], nzb[threadIdx.x]);
        wb += 4;
    }
    if (threadIdx.x == 0) {
        gnz[c.nw] = 1u;
        wb += 4;
    }
    __syncthreads();
    for (int col = threadIdx.x; col < c.ncol; col += TM_NT) {
        const uint32_t w = nzb[col >> 5];
        if ((w >> (col & 31)) & 1u) {
            WB_ST(&gval[woff[col >> 5] + __popc(w & ((1u << (col & 31)) - 1u))], t.colconf[col]);
            wb += 4;
        }
    }
    return wb;
}

template <bool LEARN, bool FROZEN>
// first / last: the step opens / closes a run of steps by this workgroup.
// Between them the stream's TM state (cell bitmaps, colConfidence, header,
// pattern history, RNG) stays in LDS: only the first step loads it from HBM
// and only the last writes it back.
__device__ __forceinline__ void tm_step_body(const DevCfg& c, const TmBufs& b, const SpBufs& sp, float* scores,
                                             int keep_prev, int s, uint8_t* lds, int first = 1, int last = 1) {
    Tm t;
    tm_bind<LEARN, FROZEN>(t, c, b, s, s, lds);
    TmSh* sh = t.sh;
    if (threadIdx.x == 0) sh->p1_n = -1;  // (no phase 1 yet this step)
#ifdef HTM_STAMPS
    if (threadIdx.x == 0) {
        for (int k = 0; k < HTM_NSTAMP; k++) sh->st_acc[k] = sh->st_cnt[k] = 0;
        sh->st_last = __builtin_amdgcn_s_memtime();
        sh->st_start = sh->st_last;
        if (sh->st_sp0 && sh->st_sp0 < sh->st_last) {  // the fused SP: inference part, learning part
            const uint64_t tl = reinterpret_cast<const SpShared*>(lds + tm_layout(c, LEARN, FROZEN).off_U)->st_t_learn;
            if (tl > sh->st_sp0 && tl < sh->st_last) {
                sh->st_acc[SB_SP] = tl - sh->st_sp0;
                sh->st_acc[SB_SPL] = sh->st_last - tl;
            } else {
                sh->st_acc[SB_SP] = sh->st_last - sh->st_sp0;
            }
        }
        sh->st_sp0 = 0;
    }
#endif
    htm_tm_header* hdr = b.hdr + s;
    uint32_t* gbm = b.bm + (size_t)s * 4 * c.cw;
    float* gconf = b.colconf + (size_t)s * c.ncol;  // dense colConfidence (host-written state)
    float* gval = b.colval + (size_t)s * c.ncol;    // packed colConfidence (the kernels' write-back)
    const uint32_t* gnzr = b.colnz + (size_t)s * (c.nw + 1);
    uint16_t* gpat = b.pat + (size_t)s * 2 * HTM_MAXPAT * HTM_MAXACT;
    // ---- load state
    if (!first) {
        // continuing in LDS: t -> t-1 rotation of the predicted / learn states
        if (threadIdx.x == 0) {
            const uint32_t na = sp.nact[s];
            sh->nA = (int32_t)(na < HTM_MAXACT ? na : HTM_MAXACT);
            sh->bytes = 4ull;
        }
        if (threadIdx.x < HTM_MAXACT) sh->act[threadIdx.x] = sp.act[(size_t)s * HTM_MAXACT + threadIdx.x];
        wg_copy(t.infP1, t.infP, c.cw);
        if (LEARN) {
            wg_copy(t.lrnA1, t.lrnA, c.cw);
            wg_copy(t.lrnP1, t.lrnP, c.cw);
        }
        __syncthreads();
        if (threadIdx.x == 0) sh->bytes += 2ull * sh->nA;
    }
    if (first) {
        // every load of the state is issued before any is used (one round
        // trip): header scalars, RNG, the whole pattern ring(s) (2 KiB each,
        // 16-byte loads; dead slots come along), infP(t-1), and the
        // nonzero-column bitmap of colConfidence(t-1) with its valid flag
        if (threadIdx.x == 0) {
            sh->bytes_acc = 0;
            sh->avg_dens = hdr->avg_input_density;
            sh->avg_lsl = hdr->avg_learned_seq_length;
            sh->lrn_iter = hdr->lrn_iter;
            sh->iter = hdr->iter;
            sh->pam = hdr->pam_counter;
            sh->lsl = hdr->learned_seq_length;
            sh->reset = hdr->reset_called;
            sh->have_avg = hdr->have_avg_density;
            sh->rf = hdr->rng_f;
            sh->rr = hdr->rng_r;
            sh->hwm = hdr->seg_hwm;
            sh->nlive = hdr->seg_live;
            sh->n_inf_pat = hdr->n_inf_pat;
            sh->n_lrn_pat = hdr->n_lrn_pat;
            sh->inf_head = hdr->inf_pat_head;
            sh->lrn_head = hdr->lrn_pat_head;
            sh->n_upd = hdr->n_upd;
            sh->err = hdr->error;
            sh->st[0] = hdr->stat_inf_phase2;
            sh->st[1] = hdr->stat_inf_backtrack;
            sh->st[2] = hdr->stat_lrn_phase2;
            sh->st[3] = hdr->stat_lrn_backtrack;
            sh->lp2p = LEARN ? (int32_t)hdr->lp2_pending : 0;
            sh->lp2s = 0;
            uint32_t na = sp.nact[s];
            sh->nA = (int32_t)(na < HTM_MAXACT ? na : HTM_MAXACT);
            sh->nz_valid = gnzr[c.nw];
        }
        if (threadIdx.x < 31) sh->rng[threadIdx.x] = hdr->rng_state[threadIdx.x];
        if (threadIdx.x < HTM_MAXPAT) {
            sh->inf_len[threadIdx.x] = hdr->inf_pat_len[threadIdx.x];
            sh->lrn_len[threadIdx.x] = hdr->lrn_pat_len[threadIdx.x];
        }
        if (threadIdx.x < HTM_MAXACT) sh->act[threadIdx.x] = sp.act[(size_t)s * HTM_MAXACT + threadIdx.x];
        constexpr int RINGW = HTM_MAXPAT * HTM_MAXACT / 2;  // 32-bit words per ring
        const uint32_t* gpw = reinterpret_cast<const uint32_t*>(gpat);
        for (int i = threadIdx.x; i < RINGW; i += TM_NT) {
            reinterpret_cast<uint32_t*>(&sh->inf_pat[0][0])[i] = gpw[i];
            if (LEARN) reinterpret_cast<uint32_t*>(&t.lrnpat[0][0])[i] = gpw[RINGW + i];
        }
        for (int w = threadIdx.x; w < c.cw; w += TM_NT) {
            const uint32_t p = gbm[c.cw + w];  // infPredictedState t -> t-1
            t.infP1[w] = p;
            t.infP[w] = p;
            if (LEARN) {
                const uint32_t la = gbm[2 * c.cw + w], lp = gbm[3 * c.cw + w];
                t.lrnA1[w] = la;  // lrnActiveState t -> t-1
                t.lrnA[w] = la;
                t.lrnP1[w] = lp;  // lrnPredictedState t -> t-1
                t.lrnP[w] = lp;
            }
        }
        if (threadIdx.x < (uint32_t)c.nw) t.flags[threadIdx.x] = gnzr[threadIdx.x];
        if (t.defer) {  // the deferred log's counters (every thread keeps a copy) and ring metadata
            t.dn = b.fx_dn[s];
            t.df = b.fx_dflushed[s];
            const uint32_t l = lane_id();
            if (l < (uint32_t)c.fx_dcap) {
                t.rh = b.fx_dhash[(size_t)s * c.fx_dcap + l];
                t.rl = b.fx_dlen[(size_t)s * c.fx_dcap + l];
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            // header in/out, active list, pattern ring(s), bitmaps in (t-1), the
            // nonzero-column bitmap of colConfidence(t-1) + flag
            sh->bytes = (LEARN ? 2ull : 1ull) * 4ull * RINGW + 2ull * sizeof(htm_tm_header) + 2ull * sh->nA + 4ull +
                        (LEARN ? 3ull : 1ull) * 4ull * c.cw + 4ull * (c.nw + 1);
        }
    }
    const int nA = sh->nA;
    // ---- anomaly input: prevPredictedColumns = nonzero(colConfidence(t-1)):
    // on the first step of a run its nonzero-column bitmap (loaded into
    // t.flags; after the host changed the state, the dense copy in HBM); from
    // LDS after it
    const bool from_bm = first && sh->nz_valid == 1u;
    const float* pconf = first ? gconf : t.colconf;
    auto prev_nz = [&](int col) -> bool {
        return from_bm ? ((t.flags[col >> 5] >> (col & 31)) & 1u) != 0u : pconf[col] != 0.0f;
    };
    uint32_t hit = 0;
    for (int a = threadIdx.x; a < nA; a += TM_NT) hit += prev_nz(sh->act[a]) ? 1u : 0u;
    if (keep_prev)
        for (int col = threadIdx.x; col < c.ncol; col += TM_NT)
            b.prev_pred[(size_t)s * c.ncol + col] = prev_nz(col) ? 1 : 0;
    hit = wg_sum(sh, hit);
    if (threadIdx.x == 0) {
        // computeRawAnomalyScore -> Real32 output
        scores[s] = nA > 0 ? (float)((double)(nA - (int)hit) / (double)nA) : 0.0f;
        if (LEARN) sh->lrn_iter++;
        sh->iter++;
        if (!sh->have_avg) {
            sh->avg_dens = (double)nA;
            sh->have_avg = 1;
        } else {
            sh->avg_dens = 0.99 * sh->avg_dens + 0.01 * (double)nA;
        }
    }
    __syncthreads();
    if (LEARN && sh->lp2p) {  // the deferred learn phase 2's keys (collect_scan)
        wg_clear(t.lkey, c.ncol);
        __syncthreads();
    }
    STAMP(t, SB_LOAD);
    if (LEARN && sh->hwm + (uint32_t)c.seg_reserve > (uint32_t)c.seg_cap) {
        compact_pool(t);
        STAMP(t, SB_COMPACT);
    }
    // ---- BacktrackingTM.compute(input, learn, infer=True)
    update_inference<FROZEN>(t);
    STAMP(t, SB_BT);
    if (LEARN && sh->lp2p) lp2_finish(t, sh->lrn_iter - 1u);  // (the previous step's lrn_iter)
    if (LEARN) update_learning(t);
    STAMP(t, SB_LEARN);
    // ---- write back (last step of the run only)
    __syncthreads();
    if (!last) {
        if (threadIdx.x == 0) {
            sh->bytes_acc += sh->bytes;
            sh->reset = 0;  // reset_called is consumed by the step after the reset
        }
#ifdef HTM_STAMPS
        __syncthreads();
        STAMP(t, SB_WB);
        COUNT(t, SC_STEPS, 1);
        if (threadIdx.x == 0) {
            uint64_t x = (sh->st_last - sh->st_start) >> 16;
            int hb = 0;
            while (x && hb < 8) { hb++; x >>= 1; }
            sh->st_cnt[SC_HIST + hb] += 1;
            uint64_t* d = b.dbg + (size_t)s * 4 * HTM_NSTAMP;
            const bool tail = sh->st_last - sh->st_start >= (1ull << 18);
            for (int k = 0; k < HTM_NSTAMP; k++) {
                d[k] += sh->st_acc[k];
                d[HTM_NSTAMP + k] += sh->st_cnt[k];
                if (tail) {
                    d[2 * HTM_NSTAMP + k] += sh->st_acc[k];
                    d[3 * HTM_NSTAMP + k] += sh->st_cnt[k];
                }
            }
        }
#endif
        return;
    }
    // cell bitmaps whole, colConfidence packed (no reads)
    uint32_t wb = write_back_inference(t, gbm, gval, b.colnz + (size_t)s * (c.nw + 1));
    if (LEARN) {
        wg_copy(gbm + 2 * c.cw, t.lrnA, c.cw);
        wg_copy(gbm + 3 * c.cw, t.lrnP, c.cw);
        if (threadIdx.x == 0) wb += 8 * c.cw;
    }
    // patterns: a single step changes only the slot it pushed (pops move
    // the heads); a run of steps writes back every live slot
    if (first) {
        if (sh->ti[0] >= 0)
            for (int a = threadIdx.x; a < sh->nA; a += TM_NT)
                gpat[sh->ti[0] * HTM_MAXACT + a] = sh->inf_pat[sh->ti[0]][a];
        if (LEARN && sh->ti[1] >= 0)
            for (int a = threadIdx.x; a < sh->nA; a += TM_NT)
                gpat[(HTM_MAXPAT + sh->ti[1]) * HTM_MAXACT + a] = t.lrnpat[sh->ti[1]][a];
    } else {
        const int ni = sh->n_inf_pat, nl = LEARN ? sh->n_lrn_pat : 0;
        for (int i = threadIdx.x; i < (ni + nl) * HTM_MAXACT; i += TM_NT) {
            const int k = i / HTM_MAXACT, a = i % HTM_MAXACT;
            if (k < ni) {
                const int slot = (sh->inf_head + k) % HTM_MAXPAT;
                if (a < sh->inf_len[slot]) gpat[slot * HTM_MAXACT + a] = sh->inf_pat[slot][a];
            } else {
                const int slot = (sh->lrn_head + k - ni) % HTM_MAXPAT;
                if (a < sh->lrn_len[slot]) gpat[(HTM_MAXPAT + slot) * HTM_MAXACT + a] = t.lrnpat[slot][a];
            }
        }
    }
    wb = wg_sum(sh, wb);
    if (threadIdx.x == 0) {
        // bitmaps out (changed words; infA's old words read), colConfidence
        // out (sparse), nonzero-column map, pushed patterns, score
        sh->bytes += wb + (LEARN ? 4ull : 2ull) * sh->nA + 4ull;
        hdr->stat_bytes += sh->bytes_acc + sh->bytes;
    }
    // the RNG moves only when learning; a single step changes one ring slot's length
    if (LEARN && threadIdx.x < 31) hdr->rng_state[threadIdx.x] = sh->rng[threadIdx.x];
    if (threadIdx.x < HTM_MAXPAT) {
        if (!first || (int)threadIdx.x == sh->ti[0]) hdr->inf_pat_len[threadIdx.x] = sh->inf_len[threadIdx.x];
        if (LEARN && (!first || (int)threadIdx.x == sh->ti[1])) hdr->lrn_pat_len[threadIdx.x] = sh->lrn_len[threadIdx.x];
    }
    if (threadIdx.x == 0) {
        if (t.defer) b.fx_dn[s] = t.dn;
        hdr->avg_input_density = sh->avg_dens;
        hdr->avg_learned_seq_length = sh->avg_lsl;
        hdr->lrn_iter = sh->lrn_iter;
        hdr->iter = sh->iter;
        hdr->pam_counter = sh->pam;
        hdr->learned_seq_length = sh->lsl;
        hdr->reset_called = 0;
        hdr->have_avg_density = sh->have_avg;
        hdr->rng_f = sh->rf;
        hdr->rng_r = sh->rr;
        hdr->seg_hwm = sh->hwm;
        hdr->seg_live = sh->nlive;
        hdr->n_inf_pat = sh->n_inf_pat;
        hdr->n_lrn_pat = sh->n_lrn_pat;
        hdr->inf_pat_head = (uint16_t)sh->inf_head;
        hdr->lrn_pat_head = (uint16_t)sh->lrn_head;
        hdr->n_upd = sh->n_upd;
        hdr->error = sh->err;
        hdr->stat_inf_phase2 = sh->st[0];
        hdr->stat_inf_backtrack = sh->st[1];
        hdr->stat_lrn_phase2 = sh->st[2];
        hdr->stat_lrn_backtrack = sh->st[3];
        if (LEARN) hdr->lp2_pending = (uint32_t)sh->lp2p;
    }
#ifdef HTM_STAMPS
    __syncthreads();
    STAMP(t, SB_WB);
    COUNT(t, SC_STEPS, 1);
    if (threadIdx.x == 0) {
        uint64_t x = (sh->st_last - sh->st_start) >> 16;
        int hb = 0;
        while (x && hb < 8) { hb++; x >>= 1; }
        sh->st_cnt[SC_HIST + hb] += 1;
    }
    if (threadIdx.x == 0 && b.dbg) {
        uint64_t* d = b.dbg + (size_t)s * 4 * HTM_NSTAMP;
        const bool tail = sh->st_last - sh->st_start >= (1ull << 18);
        for (int k = 0; k < HTM_NSTAMP; k++) {
            d[k] += sh->st_acc[k];
            d[HTM_NSTAMP + k] += sh->st_cnt[k];
            if (tail) {
                d[2 * HTM_NSTAMP + k] += sh->st_acc[k];
                d[3 * HTM_NSTAMP + k] += sh->st_cnt[k];
            }
        }
    }
#endif
}

// Fused network.run(1) x n_steps: each work unit steps one stream through
// encoder -> SP -> TM -> anomaly for up to unit_steps consecutive records,
// its state LDS-resident between them (streams are independent; every
// stream's result is the one per-step launches give).  The SP's LDS aliases
// the TM union region, which is free between steps.
//
// Persistent work queue: a grid of at most (resident workgroups) dequeues
// units u = block * n + stream in order from wq[0]; unit (s, b) waits until
// wq[1 + s] -- stream s's completed blocks -- reaches b.  Its predecessor
// (s, b - 1) was dequeued n units earlier by a running workgroup, so the
// wait always ends; every workgroup exits once the counter passes the last
// unit.  This balances streams of unequal cost (backtracks) and removes the
// quantisation of n streams over the resident slots.  State handed between
// units goes through HBM: agent-scope fences on both sides (the XCDs' L2s
// are not coherent with each other).
// SPL = false compiles SP learning out (the frozen bench kernel: inference only)
#ifndef HTM_SPL_PLANES
#define HTM_SPL_PLANES 1
#endif
// NOSP compiles the SP out (TM-only launches: the SP kernel ran first)
template <bool LEARN, bool FROZEN, bool PAGED_OK, bool SPL = true, bool NOSP = false>
__device__ __forceinline__ void htm_run_body(const DevCfg& c, const TmBufs& b, const SpBufs& sp, const double* values,
                                             float* scores, int n_steps, int sp_learn, int keep_prev,
                                             int keep_overlaps, uint32_t* wq, int unit_steps, int n) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    __shared__ uint32_t unit_sh[3];  // unit, its stream, its block
    SpShared& ssh = *reinterpret_cast<SpShared*>(lds + tm_layout(c, LEARN, FROZEN).off_U);
    uint32_t* bkey = c.sp_boost != 0.0f
                         ? reinterpret_cast<uint32_t*>(lds + tm_layout(c, LEARN, FROZEN).off_U + align16(sizeof(SpShared)))
                         : nullptr;
    // the waves' partial overlaps, past SpShared and the boost keys
    uint32_t* planes = reinterpret_cast<uint32_t*>(lds + tm_layout(c, LEARN, FROZEN).off_U + align16(sizeof(SpShared))) +
                       (c.sp_boost != 0.0f ? ((size_t)c.nw + 1) * 32 : 0);
    const uint32_t nblk = (uint32_t)((n_steps + unit_steps - 1) / unit_steps);
    const uint32_t total = (uint32_t)n * nblk;
    // one flat loop over (unit, step) so the compiler sees the same single
    // step loop as a one-stream run (no invariants hoisted across units)
    // one unit per stream (n_steps <= unit_steps, e.g. every htm_step): no
    // hand-offs, so no queue and no fences -- workgroup b runs stream b
    const bool direct = nblk == 1;
#ifdef HTM_AB_KNOBS
    const unsigned long long wg_t0 = __builtin_amdgcn_s_memrealtime();
#endif
    uint32_t u = 0xFFFFFFFFu;
    int s = 0, k = 0, k0 = 0, k1 = 0;
    for (;;) {
        if (k == k1 && direct) {
            if (u != 0xFFFFFFFFu || blockIdx.x >= (uint32_t)n) break;
            u = blockIdx.x;
            s = b.ord ? (int)__builtin_amdgcn_readfirstlane(b.ord[blockIdx.x]) : (int)blockIdx.x;
            if (s >= n) break;  // (never: ord lists streams)
            k0 = k = 0;
            k1 = n_steps;
        }
        if (k == k1) {
            if (u != 0xFFFFFFFFu) {
                __threadfence();  // release this unit's state writes
                __syncthreads();
                if (threadIdx.x == 0)
                    __hip_atomic_store(&wq[1 + s], (uint32_t)(k0 / unit_steps) + 1u, __ATOMIC_RELEASE,
                                       __HIP_MEMORY_SCOPE_AGENT);
            }
            if (threadIdx.x == 0) {
                const uint32_t x = atomicAdd(&wq[0], 1u);
                if (x < total && x >= (uint32_t)n) {
                    const uint32_t xs = x % (uint32_t)n, blk = x / (uint32_t)n;
                    while (__hip_atomic_load(&wq[1 + xs], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < blk)
                        __builtin_amdgcn_s_sleep(8);
                }
                unit_sh[0] = x;
                unit_sh[1] = x % (uint32_t)n;
                unit_sh[2] = x / (uint32_t)n;
            }
            __syncthreads();
            // SGPR copies: the stream index must stay scalar (a VALU division
            // result would move every per-stream address into VGPRs)
            u = __builtin_amdgcn_readfirstlane(unit_sh[0]);
            if (u >= total) break;
            __threadfence();  // acquire the previous unit's state writes (all threads)
            s = (int)__builtin_amdgcn_readfirstlane(unit_sh[1]);
            k0 = (int)__builtin_amdgcn_readfirstlane(unit_sh[2]) * unit_steps;
            k1 = n_steps - k0 < unit_steps ? n_steps : k0 + unit_steps;
            k = k0;
        }
        const double* v = values + (size_t)k * c.n_streams * c.n_fields;
        const uint16_t* enc = c.enc_type == HTM_ENC_RDSE ? sp.enc_in + (size_t)k * c.n_streams * c.enc_list : nullptr;
#ifdef HTM_STAMPS
        if (threadIdx.x == 0) reinterpret_cast<TmSh*>(lds)->st_sp0 = __builtin_amdgcn_s_memtime();
#endif
        if constexpr (!NOSP) {  // (TM-only kernels: the SP code is not instantiated)
            if (!b.tm_only) {
                if (SPL && sp_learn)
                    sp_step_body<true, PAGED_OK, PAGED_OK || LEARN || HTM_SPL_PLANES>(c, sp, v, s, ssh, keep_overlaps,
                                                                                     bkey, enc, planes);
                else sp_step_body<false, PAGED_OK, true>(c, sp, v, s, ssh, keep_overlaps, nullptr, enc, planes);
                __syncthreads();
            }
        }
        tm_step_body<LEARN, FROZEN>(c, b, sp, scores + (size_t)k * c.n_streams, keep_prev, s, lds, k == k0,
                                    k == k1 - 1);
        __syncthreads();
        k++;
    }
#ifdef HTM_AB_KNOBS
    // A/B builds: the workgroup timeline of a lockstep launch (tools/wg_timeline.py)
    if (b.wg_trace && direct) {
        const uint32_t* infA = reinterpret_cast<const uint32_t*>(lds + tm_layout(c, LEARN, FROZEN).off_bm);
        uint32_t pc = 0;
        if (blockIdx.x < (uint32_t)n)
            for (int i = threadIdx.x; i < c.cw; i += TM_NT) pc += __popc(infA[i]);
        pc = wave_sum_u32(pc);
        __syncthreads();
        if (lane_id() == 0 && wave_id() < 3) unit_sh[wave_id()] = pc;
        __syncthreads();
        const uint32_t tot = unit_sh[0] + unit_sh[1] + unit_sh[2];
        __syncthreads();
        if (wave_id() == 3 && lane_id() == 0) unit_sh[0] = tot + pc;
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long* p = b.wg_trace + (size_t)blockIdx.x * 8;
            p[0] = wg_t0;
            p[1] = __builtin_amdgcn_s_memrealtime();
            p[2] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
            p[3] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
            p[4] = blockIdx.x < (uint32_t)n ? reinterpret_cast<TmSh*>(lds)->bytes : 0ull;
            p[5] = unit_sh[0];
        }
    }
#endif
}

#define HTM_RUN_ARGS                                                                                          \
    DevCfg c, TmBufs b, SpBufs sp, const double *values, float *scores, int n_steps, int sp_learn, int keep_prev, \
        int keep_overlaps, uint32_t *wq, int unit_steps, int n
#define HTM_RUN_PASS c, b, sp, values, scores, n_steps, sp_learn, keep_prev, keep_overlaps, wq, unit_steps, n

// The kernels live in their own translation units (tm_k_*.hip, compiled in
// parallel); each exports its kernel's address, a launcher and the dynamic-LDS
// attribute setter through these.
#define TM_RUN_KERNEL_EXPORTS(name, kern)                                                            \
    const void* tmk_fn_##name() { return (const void*)kern; }                                       \
    int tmk_launch_##name(int grid, size_t lds, hipStream_t st, HTM_RUN_ARGS) {                      \
        hipLaunchKernelGGL(kern, dim3(grid), dim3(TM_NT), lds, st, HTM_RUN_PASS);                     \
        return hipGetLastError() == hipSuccess ? 0 : -1;                                              \
    }                                                                                                 \
    int tmk_attr_##name(size_t lds) {                                                                 \
        return hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == \
                       hipSuccess ? 0 : -1;                                                           \
    }
#define TM_RUN_KERNEL_DECL(name)                                                                     \
    const void* tmk_fn_##name();                                                                      \
    int tmk_launch_##name(int grid, size_t lds, hipStream_t st, HTM_RUN_ARGS);                       \
    int tmk_attr_##name(size_t lds);
TM_RUN_KERNEL_DECL(run_frozen)
TM_RUN_KERNEL_DECL(run_frozen_tm)
TM_RUN_KERNEL_DECL(run_frozen_spl)
TM_RUN_KERNEL_DECL(run_frozen_paged)
TM_RUN_KERNEL_DECL(run_learn)
TM_RUN_KERNEL_DECL(run_learn_tm)
TM_RUN_KERNEL_DECL(run_infer)
// unfused TM step kernels (learn, frozen index, pool scan)
int tmk_launch_step(int learn, int frozen, int grid, size_t lds, hipStream_t st, DevCfg c, TmBufs b, SpBufs sp,
                    float* scores);
int tmk_attr_step(size_t lds_learn, size_t lds_frozen, size_t lds_scan);

