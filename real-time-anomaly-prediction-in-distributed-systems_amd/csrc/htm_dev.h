// htm_dev.h -- device-side layout and helpers of the MI355X HTM engine.
//
// Memory is laid out per stream (structure-of-arrays per field, streams
// contiguous), sized for 288 GB HBM: the SP keeps only potential synapses
// (float32, potential order) plus an input-major connected bitmap, the TM a
// slot-indexed segment pool (append-only; slot order == creation order, so
// a cell's segment list order is slot order) and, while TM learning is off,
// a forward index cell -> (segment, connected) used by frozen inference.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/htm_amd.h"

#define HTM_MAXSYN 32     // synapse slots per TM segment
#define HTM_MAXACT 64     // SP active columns (numActiveColumnsPerInhArea)
#define HTM_MAXK 32       // cells per column
#define HTM_MAXPAT 16     // backtrack pattern history slots
#define HTM_NPLANES 7     // bit-sliced overlap planes (overlap <= 127)
#define HTM_MAX_SDR 32768 // SDR-input SP: input bits (Models 2/3 level 2: 2048 x 12)
#define HTM_MAXNW 128     // ncol/32 words (ncol <= 4096)
#ifndef TM_NT
#define TM_NT 256                  // threads of the TM workgroup (one stream)
#endif
#define TM_NWAVES (TM_NT / 64)
#ifndef FX_DEPTH
#define FX_DEPTH 4                 // frozen index: out-list blocks in flight per thread
#endif
#define FX_OWN (FX_DEPTH * TM_NT)  // blocks streamed per pass (block -> list map in LDS)
// index of the block-list offset of (list w, cell x): w = -1 the cell's pid
// list, w >= 0 its rank window w.  Cell-major: a cell's pid list and window
// lists are one contiguous run of blocks and their offsets are adjacent words,
// so the passes of a phase 2 after the first find both in cache (same-box A/B
// vs window-major: same time, HBM traffic 1.99x vs 2.11x the algorithmic
// bytes, profiles/r03_ab).  FX_WINDOW_MAJOR (A/B builds only) restores the
// round-3 [window][cell] order.
#ifdef FX_WINDOW_MAJOR
#define FX_LIST(c, w, x) ((w) < 0 ? (size_t)(c).ncells * (c).fx_nwin + (size_t)(x) : (size_t)(w) * (c).ncells + (size_t)(x))
#else
#define FX_LIST(c, w, x) ((size_t)(x) * ((size_t)(c).fx_nwin + 1) + (size_t)((int)(w) + 1))
#endif
#define FX_MAXPER ((HTM_MAXACT * HTM_MAXK + TM_NT - 1) / TM_NT)  // active cells per thread

// Derived, immutable engine constants (kernel argument).
struct DevCfg {
    // encoder
    int32_t n_fields, enc_n, enc_w, enc_clip;
    double enc_min[4], enc_max[4], enc_resolution[4];  // per field
    int32_t enc_halfwidth;
    // SP
    int32_t nin, nin_pad, ncol, nw;      // nw = ncol/32
    int32_t n_potential;                  // potential synapses per column
    int32_t num_desired;                  // winners per step
    int32_t stim_thr, dc_period, update_period;
    float sp_conn;                        // synPermConnected
    float sp_conn_thr;                    // synPermConnected - PERMANENCE_EPSILON
    float sp_inc, sp_dec, sp_trim, sp_below_inc, sp_min_pct_odc;
    // TM
    int32_t K, ncells, cw;                // cw = ncells/32
    uint32_t kmagic;                      // ceil(2^32 / K): cell / K == umulhi(cell, kmagic)
    int32_t new_syn, max_syn, max_segs_per_cell;
    float init_perm, tm_conn, tm_inc, tm_dec, tm_max;
    int32_t min_thr, act_thr, pam_len, max_inf_bt, max_lrn_bt, max_seq_len, upd_valid;
    int32_t seg_cap, upd_cap;
    int32_t seg_reserve;                  // free slots needed before a learning step
    int32_t fx_win;                       // frozen index: segments per LDS counter window (<= 65536)
    int32_t fx_nwin;                      // windows covering seg_cap
    int32_t fx_pcap;                      // frozen index: max predictive-capable segments (pid space)
    int32_t fx_noff;                      // fx_off entries per stream: ncells*fx_nwin + ncells + 1
    int32_t q_lds;                        // qualifying segments sorted in LDS (more: global path)
    int32_t q_lds_fx;                     // ... of a frozen phase 2 ranked in LDS (column u16 + dutyCycle f32
                                          // in the whole union region; more: the HBM scratch)
    int32_t lp2_defer;                    // learning steps defer their final learnPhase2 (tm_core.h lp2_finish)
    int32_t fx_own_sep;                   // frozen windows: the first block -> list map built by fx_stream after
                                          // the list starts' barrier (1), or by collect_frozen with them (0)
    int32_t fin_mode;                     // phase-2 tail: 0 column buckets (scans over all columns),
                                          // 1 bitonic key sort, 2 buckets over the nonzero-column bitmap
    int32_t max_act_cells;                // num_desired * K (frozen collection cell list)
    int32_t n_streams;
    int32_t shared_model;                 // fleet: every stream reads model instance 0 (SP + TM frozen)
    int32_t q_cap;                        // per-stream capacity of the qualifying-segment scratch lists
    int32_t sdr_in;                       // the SP reads an external input SDR of nin bits (no encoder)
    int32_t fx_dcap;                      // deferred phase-2 log entries per stream (TmBufs::fx_dlog)
    // paged SP permanences (htm_config.sp_perm_rows > 0)
    int32_t sp_paged;                     // 1: rows from SpBufs::pool on first change, else init values
    int32_t n_ckpt;                       // nupic::Random checkpoints per stream (ncol / SP_CKPT_COLS)
    int32_t pool_stride;                  // floats per pool row: n_potential rounded up to 128 B
    int32_t enc_list;                     // u16 words per (step, stream) encoded input list (RDSE):
                                          // count + n_fields * enc_w, rounded up to 8
    uint64_t pool_rows;                   // rows in SpBufs::pool
    // boosting (updateBoostFactorsGlobal_): strength (0: factors stay 1.0, the
    // integer inhibition path) and the target density numActive / area
    float sp_boost, sp_target;
    // encoder: HTM_ENC_SCALAR or HTM_ENC_RDSE (then the active input bits of a
    // step come from rdse_encode_kernel through SpBufs::enc_in)
    int32_t enc_type;
    int32_t rdse_block;                   // bytes of one field's RDSE state (header + bucket map)
    double rdse_res;                      // RDSE resolution
};

// deferred-log slot stride in cells: max_act_cells rounded up to 8, so every
// slot starts 16-byte aligned (the flush's job builder compares slots in
// 16-byte loads)
__host__ __device__ inline size_t fx_dstride(const DevCfg& c) { return ((size_t)c.max_act_cells + 7) & ~(size_t)7; }

#define RDSE_HDR_WORDS 64   // int32 words of an RDSE field header (HTM_ST_ENC_RDSE)

#define SP_JUMP_POW 16      // jump tables: skips of up to 2^16 - 1 blocks (an 8-column group needs < 2^10)
#ifndef SP_CKPT_COLS
#define SP_CKPT_COLS 8      // columns per SP-initialisation checkpoint (paged permanences; <= 8)
#endif
#define SP_CKPT_WORDS 64    // words per checkpoint: st[31], idx, pending draws buf[31], pad
#define SP_ROW_NONE 0xFFFFFFFFu
#define SP_ERR_POOL 32u     // error flag: paged SP row pool exhausted (results invalid)

// instance of the model buffers (SP permanences/connections, TM segment
// pool, frozen index) stream s reads: its own, or the fleet's shared one
__device__ __forceinline__ int model_stream(const DevCfg& c, int s) { return c.shared_model ? 0 : s; }

// Device buffers (all per-stream strided).
struct SpBufs {
    uint32_t* connT;    // [S][nin_pad][nw]
    uint32_t* potmask;  // [S][ncol][nin_pad/32]
    float* perm;        // [S][ncol][n_potential]
    float* duty;        // [S][2][ncol]: overlap dc, active dc
    uint32_t* scalars;  // [S][4]: iter, iter_learn, min_odc bits, pad
    uint16_t* act;      // [S][HTM_MAXACT] active columns (ascending)
    uint32_t* nact;     // [S]
    int32_t* overlaps;  // [S][ncol]
    uint64_t* seeds;    // [S] SP seed per stream
    // paged permanences (DevCfg::sp_paged; perm is null then)
    uint32_t* prow;     // [S][ncol] pool row of the column, SP_ROW_NONE: initial values
    float* pool;        // [pool_rows][pool_stride]
    unsigned long long* pool_next;  // [1] rows handed out
    uint32_t* ckpt;     // [S][n_ckpt][SP_CKPT_WORDS] RNG state at columns 0, 8, 16, ... of sp_init
    const uint32_t* jump;  // [SP_JUMP_POW][31][32] the 31-draw block map of nupic::Random raised to 2^p
                           //     (rows padded to 32 words): skipping whole blocks by matrix powers
    uint32_t* err;      // [S] SP error flags (SP_ERR_POOL)
    float* boost;       // [S][ncol] boostFactors_ (1.0 at init)
    // RDSE encoders (DevCfg::enc_type == HTM_ENC_RDSE): per stream, per field
    // a block of rdse_block bytes (header int32[RDSE_HDR_WORDS], then the
    // int16 [HTM_RDSE_BUCKETS][enc_w] bucket map); the encoded active-input
    // lists of the steps of one launch [steps][S][enc_list] (word 0 = count);
    // the last record's bucket per field (HTM_OUT_BUCKETS)
    uint8_t* rdse;
    uint16_t* enc_in;
    int32_t* enc_bucket;  // [S][4]
    uint64_t* rdse_seeds; // [S] RDSE seed per stream
    uint64_t* dbg;        // [S][4] paged-row replays, their cycles, of which sampling-draw count and block
                          // skip (HTM_STAMPS builds only, else null)
};

struct TmBufs {
    htm_tm_header* hdr;     // [S]
    uint32_t* bm;           // [S][4][cw]: infA, infP, lrnA, lrnP (time t)
    float* colconf;         // [S][ncol]
    uint16_t* pat;          // [S][2*HTM_MAXPAT][HTM_MAXACT]: inf then lrn
    uint32_t* seg_meta;     // [S][seg_cap]
    uint16_t* seg_src;      // [S][seg_cap][32]
    float* seg_perm;        // [S][seg_cap][32]
    uint32_t* seg_conn;     // [S][seg_cap]
    uint32_t* seg_duty;     // [S][seg_cap][3]: posAct, lastDC bits, lastDCIter
    uint8_t* cell_nseg;     // [S][ncells]
    htm_tm_update* upd;     // [S][upd_cap]
    // scratch (per stream)
    uint32_t* scr_bm;       // [S][5][cw]: infA backup, infP(t-1) backup, infA cand, infP cand, spare
    float* scr_conf;        // [S][ncol]: colConf candidate
    uint32_t* scr_q;        // [S][q_cap]: qualifying segment keys
    uint32_t* scr_q2;       // [S][q_cap] (>= seg_cap entries): bucket-sorted keys / index-build pid map
    uint8_t* prev_pred;     // [S][ncol] nonzero(colConf(t-1)) captured before compute
    uint32_t* colnz;        // [S][nw + 1]: nonzero columns of colconf, word nw = 1 when the packed form is current
    float* colval;          // [S][ncol]: packed colConfidence, the nonzero columns' values in column order
    uint32_t* scr_cur;      // [S][ncells*fx_nwin] frozen-index fill cursors
    // frozen forward index (valid while TM learning is off).  Live segments
    // are numbered by RANK in NuPIC's (cell, creation) order -- the order
    // _inferPhase2 sums confidences in -- so segments that qualify, found by a
    // sweep over rank-ordered counters, come out already in summation order.
    // For stream s, counter window w (a range of fx_win ranks) and cell x, the
    // window-relative ranks (u16) of the segments with a synapse from x fill
    // the 16-byte blocks fx_ent[fx_base[s] + fx_off[s][w][x] .. fx_off[s][w][x+1]),
    // padded with 0xFFFF, so one uint4 load delivers 8 entries of one list.
    // Window-major: within a window the lists of consecutive cells are
    // adjacent, so a bursting column's cells stream as one contiguous run
    // The same block pool also holds, per cell, the list of predictive-
    // capable segment ids (pid: live segments with >= activationThreshold
    // connected synapses, numbered densely in slot order) that the cell
    // feeds through a CONNECTED synapse, so frozen phase 2 counts connected
    // activity without reading synapse rows.  fx_rec holds what phase 2
    // needs of a qualifying segment: its cell and the dutyCycle value it
    // reads while learning is off (the iteration counter is frozen).
    uint64_t* fx_base;      // [S] first block of the stream
    uint32_t* fx_off;       // [S][fx_noff]: block offsets of the lists in FX_LIST order ([cell][pid, windows]), then the end
    uint4* fx_ent;          // [total blocks] 8 x u16 entries each
    uint2* fx_rec;          // [S][seg_cap] by rank: {cell | FX_FRESH, dutyCycle bits}
    uint32_t* fx_rslot;     // [S][seg_cap] pool slot of each rank
    uint32_t* fx_nr;        // [S] ranks (live segments)
    uint16_t* fx_pcell;     // [S][fx_pcap] cell of each pid
    uint32_t* fx_np;        // [S] number of pids (> fx_pcap: pid lists not built, rows are read)
    uint64_t* dbg;          // [S][32] phase stamps + event counts (HTM_STAMPS builds only, else null)
    // Deferred dutyCycle() writes (frozen lockstep launches; null: off).  A
    // frozen phase 2 whose confidences the step discards needs only the
    // predicted cells (the pid pass) for what follows; its one remaining effect,
    // the first dutyCycle() record write of each qualifying segment (FX_FRESH),
    // is deferred: the phase 2's active cells are logged, and
    // tm_fx_flush_kernel replays the log before anything reads the records.
    uint16_t* fx_dlog;             // [S][fx_dcap][max_act_cells] active cells of a deferred phase 2
    uint16_t* fx_dlen;             // [S][fx_dcap] their number (a ring: entry e in slot e % fx_dcap)
    uint32_t* fx_dhash;            // [S][fx_dcap] hash of the set
    uint32_t* fx_dn;               // [S] entries logged (monotonic)
    uint32_t* fx_dflushed;         // [S] entries flushed
    uint32_t* fx_dsnap;            // [S] fx_dn when the latest flush was enqueued (step stream)
    uint32_t* fx_dupto;            // [S] the bound the running flush's job builder took from fx_dsnap:
                                   //     the flush replays [fx_dflushed, fx_dupto) and its done kernel
                                   //     advances fx_dflushed to exactly that (never to a later snapshot)
    uint32_t* fx_fq;               // [FX_FLUSH_WG][q_cap] the flush workgroups' qualifying lists
    uint32_t* fx_fwork;            // [4] flush job counter, error flags (FX_ERR_*), jobs
    uint32_t* fx_fjobs;            // [S * fx_dcap * fx_nwin] the running flush's jobs:
                                   //     (stream * fx_dcap + ring slot) * (fx_nwin + 1) + rank window
                                   //     (fx_nwin: every window of the entry)
    unsigned long long* wg_trace;  // A/B builds (HTM_WG_TRACE): [grid][8] start / end (s_memrealtime),
                                   //     HW_ID, XCC_ID, step bytes, final active cells; else null
    // Ordered lockstep launches (HTM_OPT_ORDERED): the SP kernel has run every
    // stream's SP, ord_sort_kernel has listed the streams heaviest TM step
    // first (the active cells phase 1 will list), and the fused kernel runs
    // the TM steps only, workgroup b taking stream ord[b]: the hardware
    // dispatches workgroups in order, so the launch's longest steps start first
    // instead of wherever the stream order puts them.
    const uint32_t* ord;           // [S] stream of each workgroup (null: workgroup b runs stream b)
    int32_t tm_only;               // 1: the launch skips the SP (ordered launches)
};
#define FX_FWORK_WORDS 4
#define ORD_NB 64                  // cost buckets of the ordering (active-cell estimate / (max_act_cells / 64))
// the cost bucket of an active-cell estimate (ord_sort_kernel)
__host__ __device__ inline uint32_t ord_bucket(uint32_t est, uint32_t mac) {
    const uint32_t q = (uint32_t)(((unsigned long long)est * 64u) / (mac + 1u));
    return q < 64u ? q : 63u;
}
#define ORD_MAX_STREAMS 16384      // ordered lockstep launches: ord_sort_kernel's one workgroup (n bytes of LDS)

// deferred-log flush error flags (fx_fwork[1]; htm_status / htm_counters)
#define FX_ERR_QCAP 16u   // a replayed phase 2 overflowed q_cap (as in the step: results invalid)
#define FX_ERR_RING 64u   // fx_dupto - fx_dflushed > fx_dcap: ring counters inconsistent (entries skipped)
#define FX_ERR_JOBS 128u  // the job list would pass S * fx_dcap entries (entries skipped)
#define FX_ERR_JOB 256u   // a job names a stream >= n, a slot >= fx_dcap or a set longer than
                          // max_act_cells (job skipped)

#define FX_FLUSH_WG 1024  // persistent workgroups of tm_fx_flush_kernel (each has its own scratch list)

#define FX_FRESH 0x80000000u  // fx_rec.x: the segment's dutyCycle record holds its frozen value

// Diagnostic phase stamps (HTM_STAMPS builds only): thread 0 charges the
// shader cycles since its previous stamp to bucket k.  Compiled out of the
// product library.
#define HTM_NSTAMP 32  // stamp buckets; the debug record per stream is 4 x HTM_NSTAMP words
#ifdef HTM_STAMPS
#define STAMP(t, k)                                                     \
    do {                                                                \
        if (threadIdx.x == 0) {                                         \
            const uint64_t now_ = __builtin_amdgcn_s_memtime();         \
            (t).sh->st_acc[(k)] += now_ - (t).sh->st_last;              \
            (t).sh->st_last = now_;                                     \
        }                                                               \
    } while (0)
#define COUNT(t, k, v)                                                  \
    do {                                                                \
        if (threadIdx.x == 0) (t).sh->st_cnt[(k)] += (uint64_t)(v);     \
    } while (0)
#define STAMP_SH(sh, k)                                                 \
    do {                                                                \
        if (threadIdx.x == 0) {                                         \
            const uint64_t now_ = __builtin_amdgcn_s_memtime();         \
            (sh)->st_acc[(k)] += now_ - (sh)->st_last;                  \
            (sh)->st_last = now_;                                       \
        }                                                               \
    } while (0)
#else
#define STAMP(t, k) do { } while (0)
#define COUNT(t, k, v) do { } while (0)
#define STAMP_SH(sh, k) do { } while (0)
#endif

// ---------------------------------------------------------------------------
// segment meta word
__device__ __forceinline__ uint32_t meta_cell(uint32_t m) { return m & 0xFFFFu; }
__device__ __forceinline__ uint32_t meta_nsyn(uint32_t m) { return (m >> 16) & 0x3Fu; }
__device__ __forceinline__ uint32_t meta_seq(uint32_t m) { return (m >> 22) & 1u; }
__device__ __forceinline__ uint32_t meta_live(uint32_t m) { return (m >> 23) & 1u; }
__device__ __forceinline__ uint32_t make_meta(uint32_t cell, uint32_t nsyn, uint32_t seq, uint32_t live) {
    return cell | (nsyn << 16) | (seq << 22) | (live << 23);
}

// ---------------------------------------------------------------------------
// nupic::Random (BSD random() TYPE_3), state held in LDS or registers.
struct Rng {
    uint32_t s[31];
    int32_t f, r;
};

__device__ __forceinline__ uint32_t rng_raw(uint32_t* s, int32_t& f, int32_t& r) {
    s[f] += s[r];
    uint32_t i = (s[f] >> 1) & 0x7fffffffu;
    if (++f >= 31) { f = 0; ++r; }
    else if (++r >= 31) { r = 0; }
    return i;
}

__device__ __forceinline__ void rng_seed(uint32_t* s, int32_t& f, int32_t& r, uint64_t seed) {
    int32_t x = (int32_t)(seed % 2147483646ull + 1ull);
    s[0] = (uint32_t)x;
    for (int i = 1; i < 31; i++) {
        int32_t hi = x / 127773, lo = x % 127773;
        x = 16807 * lo - 2836 * hi;
        if (x < 0) x += 2147483647;
        s[i] = (uint32_t)x;
    }
    f = 3;
    r = 0;
    for (int i = 0; i < 310; i++) (void)rng_raw(s, f, r);
}

// Random::getUInt32(max): raw draws are < 2^31 so the rejection never fires.
__device__ __forceinline__ uint32_t rng_u32(uint32_t* s, int32_t& f, int32_t& r, uint32_t max) {
    uint32_t smax = 0xFFFFFFFFu - (0xFFFFFFFFu % max);
    uint32_t v;
    do { v = rng_raw(s, f, r); } while (v > smax);
    return v % max;
}

__device__ __forceinline__ double rng_real64(uint32_t* s, int32_t& f, int32_t& r) {
    // getUInt64(2^48): lo | hi<<32, % 2^48 (never rejected)
    uint64_t lo = rng_raw(s, f, r);
    uint64_t hi = rng_raw(s, f, r);
    uint64_t v = (lo | (hi << 32)) & ((1ull << 48) - 1ull);
    return (double)v * (1.0 / 281474976710656.0);  // ldexp(v, -48), exact
}

// ---------------------------------------------------------------------------
// bitmaps
__device__ __forceinline__ bool bm_get(const uint32_t* bm, uint32_t i) { return (bm[i >> 5] >> (i & 31)) & 1u; }

// bits [lo, lo+len) of a bitmap (len <= 32), returned in the low bits
__device__ __forceinline__ uint32_t bm_field(const uint32_t* bm, uint32_t lo, uint32_t len) {
    uint32_t w = lo >> 5, b = lo & 31;
    uint64_t x = (uint64_t)bm[w];
    if (b + len > 32) x |= (uint64_t)bm[w + 1] << 32;
    x >>= b;
    return (uint32_t)(x & ((len == 32) ? 0xFFFFFFFFull : ((1ull << len) - 1ull)));
}

// OR `bits` (len <= 32) into bitmap at [lo, lo+len) with LDS atomics
__device__ __forceinline__ void bm_or_field(uint32_t* bm, uint32_t lo, uint32_t len, uint32_t bits) {
    if (!bits) return;
    uint32_t w = lo >> 5, b = lo & 31;
    uint64_t x = (uint64_t)bits << b;
    if ((uint32_t)x) atomicOr(&bm[w], (uint32_t)x);
    if (b + len > 32 && (uint32_t)(x >> 32)) atomicOr(&bm[w + 1], (uint32_t)(x >> 32));
}

// ---------------------------------------------------------------------------
// wave helpers (wave64)
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

// inclusive prefix sum over the wave with DPP (no LDS traffic): Hillis-
// Steele within each 16-lane row (row_shr 1/2/4/8), then the row totals
// carried across rows with row_bcast:15 / row_bcast:31 (gfx9 DPP).  Lanes a
// DPP move does not reach add the `old` operand, 0.
#ifndef HTM_SCAN_SHFL
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return v;
}
#else
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    int l = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t t = __shfl_up(v, o, 64);
        if (l >= o) v += t;
    }
    return v;
}
#endif

// the value of lane 63 (uniform: a scalar register)
__device__ __forceinline__ uint32_t lane63(uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)v, 63); }

// sum / max over the wave (all 64 lanes active): a DPP scan and lane 63's
// result -- no LDS round trips (a __shfl_xor butterfly is six ds_bpermute's)
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) { return lane63(wave_incl_scan(v)); }

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    // lanes a DPP move does not reach take `old` = 0, neutral for unsigned max
    uint32_t t;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v = t > v ? t : v;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v = t > v ? t : v;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v = t > v ? t : v;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v = t > v ? t : v;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v = t > v ? t : v;
    t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    v = t > v ? t : v;
    return lane63(v);
}

// v with lane `lane` replaced by the wave-uniform x (v_writelane_b32: no
// per-lane mask; clang has no builtin for it)
template <int LANE>
__device__ __forceinline__ uint32_t writelane_u32(uint32_t v, uint32_t x) {
    const uint32_t xs = (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
    asm volatile("s_nop 4\n\tv_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(xs), "i"(LANE));
    return v;
}

// nupic::Random's next block of 31 raw sums across the lanes: lane j < 31
// holds v[j] = x[n-31+j] of the window and gets y[j] = x[n+j] = v[j] +
// (j >= 3 ? y[j-3] : v[28+j]) (TM learning's draw pass, the SP's paged-row
// replay).  Lanes 0..2 get their base v[28 + j] added, then an inclusive scan
// over stride 3 inside each 16-lane row (DPP row_shr 3, 6, 12: residue
// classes never mix), and row 0's per-residue totals (lanes 15, 13, 14) are
// carried into row 1 by a second such scan.  No LDS round trip, no per-lane
// masks.  Call with every lane of the wave.
__device__ __forceinline__ uint32_t rng_block_lanes(uint32_t v) {
    // lanes 0..2 start from v[j] + v[28 + j] (the recurrence's base), so the
    // stride-3 scan carries it into every later lane of the residue; no
    // per-residue lane masks (as loop-invariant SGPR masks they were spilled)
    uint32_t p = v;
    p = writelane_u32<0>(p, (uint32_t)__builtin_amdgcn_readlane((int)v, 0) + (uint32_t)__builtin_amdgcn_readlane((int)v, 28));
    p = writelane_u32<1>(p, (uint32_t)__builtin_amdgcn_readlane((int)v, 1) + (uint32_t)__builtin_amdgcn_readlane((int)v, 29));
    p = writelane_u32<2>(p, (uint32_t)__builtin_amdgcn_readlane((int)v, 2) + (uint32_t)__builtin_amdgcn_readlane((int)v, 30));
    p += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)p, 0x113, 0xF, 0xF, false);  // row_shr:3
    p += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)p, 0x116, 0xF, 0xF, false);  // row_shr:6
    p += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)p, 0x11C, 0xF, 0xF, false);  // row_shr:12
    // row 0's totals per residue (lanes 15, 13, 14) enter row 1 at its first
    // lane of that residue (18, 16, 17) and are carried by the same scan
    uint32_t q = 0u;
    q = writelane_u32<16>(q, (uint32_t)__builtin_amdgcn_readlane((int)p, 13));
    q = writelane_u32<17>(q, (uint32_t)__builtin_amdgcn_readlane((int)p, 14));
    q = writelane_u32<18>(q, (uint32_t)__builtin_amdgcn_readlane((int)p, 15));
    q += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q, 0x113, 0xF, 0xF, false);
    q += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q, 0x116, 0xF, 0xF, false);
    q += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q, 0x11C, 0xF, 0xF, false);
    return p + q;
}

// OR over the wave (all 64 lanes active): a DPP scan read from lane 63
__device__ __forceinline__ uint32_t wave_or_dpp(uint32_t v) {
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return lane63(v);
}

// number of set bits of a 64-bit ballot below this lane
__device__ __forceinline__ uint32_t ballot_rank(uint64_t ball) {
    uint64_t m = (lane_id() == 0) ? 0ull : (~0ull >> (64 - lane_id()));
    return (uint32_t)__popcll(ball & m);
}

// exp(x) in double by a fixed sequence of IEEE operations (range reduction by
// ln 2 in two parts, degree-13 Taylor polynomial, exact power-of-two scaling),
// rounded to float: the SP boost factor exp((target - activeDutyCycle) *
// strength) of updateBoostFactorsGlobal_.  oracle/htm_oracle.c exp_det runs
// the same operations, so both agree bit for bit (and with the correctly
// rounded expf wherever double rounding does not intervene).
__device__ __forceinline__ float exp_det(float xf) {
    const double x = (double)xf;
    if (!(x == x)) return xf;
    if (x > 88.8) return __int_as_float(0x7f800000);
    if (x < -104.0) return 0.0f;
    const double inv_ln2 = 1.4426950408889634, ln2_hi = 6.93147180369123816490e-01,
                 ln2_lo = 1.90821492927058770002e-10;
    const double kd = __dmul_rn(x, inv_ln2);
    const int k = (int)(kd < 0.0 ? __dadd_rn(kd, -0.5) : __dadd_rn(kd, 0.5));
    const double r = __dadd_rn(__dadd_rn(x, -__dmul_rn((double)k, ln2_hi)), -__dmul_rn((double)k, ln2_lo));
    const double inv_fact[14] = {1.0, 1.0, 0.5, 1.0 / 6.0, 1.0 / 24.0, 1.0 / 120.0, 1.0 / 720.0,
                                 1.0 / 5040.0, 1.0 / 40320.0, 1.0 / 362880.0, 1.0 / 3628800.0,
                                 1.0 / 39916800.0, 1.0 / 479001600.0, 1.0 / 6227020800.0};
    double p = inv_fact[13];
#pragma unroll
    for (int i = 12; i >= 0; i--) p = __dadd_rn(__dmul_rn(p, r), inv_fact[i]);
    return (float)__dmul_rn(p, __longlong_as_double((long long)(1023 + k) << 52));
}

// pow(b, e) for integer e by binary exponentiation in double, rounded to
// float: deterministic on host and device (the oracle uses the same rule).
__device__ __forceinline__ float pow_det(float b, uint32_t e) {
    double r = 1.0, x = (double)b;
    while (e) {
        if (e & 1u) r = __dmul_rn(r, x);
        x = __dmul_rn(x, x);
        e >>= 1;
    }
    return (float)r;
}

// sets htm_last_error()'s message and returns code (engine.cpp)
int htm_fail(int code, const char* fmt, ...);

// host launch wrappers (defined in sp.hip / tm.hip)
int launch_sp_init(const DevCfg& c, const SpBufs& b, int n, hipStream_t st);
int launch_sp_perm_export(const DevCfg& c, const SpBufs& b, float* dst, int s0, int m, hipStream_t st);
int launch_sp_perm_import(const DevCfg& c, const SpBufs& b, const float* src, size_t src_stride, int s0, int m,
                          hipStream_t st);
int launch_sp_step(const DevCfg& c, const SpBufs& b, const double* values, int learn, int n, int keep_overlaps,
                   hipStream_t st);
int launch_rdse_init(const DevCfg& c, const SpBufs& b, int n, hipStream_t st);
int launch_rdse_encode(const DevCfg& c, const SpBufs& b, const double* values, int n_steps, int n, hipStream_t st);
int launch_sp_step_sdr(const DevCfg& c, const SpBufs& b, const uint32_t* sdr, int learn, int n, int keep_overlaps,
                       hipStream_t st);
int launch_tm_fx_rank(const DevCfg& c, const TmBufs& b, int n, hipStream_t st);
int launch_tm_init(const DevCfg& c, const TmBufs& b, const uint64_t* seeds, int n, hipStream_t st);
int launch_tm_step(const DevCfg& c, const TmBufs& b, const SpBufs& sp, float* scores, int learn, int frozen,
                   int n, hipStream_t st);
int launch_htm_run(const DevCfg& c, const TmBufs& b, const SpBufs& sp, const double* values, float* scores,
                   int n_steps, int sp_learn, int tm_learn, int frozen, int keep_prev, int keep_overlaps, int n,
                   uint32_t* wq, int unit_steps, hipStream_t st);
int launch_tm_fx_count(const DevCfg& c, const TmBufs& b, uint64_t* counts, int n, hipStream_t st);
int launch_tm_fx_fill(const DevCfg& c, const TmBufs& b, int n, hipStream_t st);
int launch_tm_fx_flush(const DevCfg& c, const TmBufs& b, int n, int max_wg, hipStream_t st, int from_dn, int split);
int launch_tm_fx_snap(const TmBufs& b, int n, hipStream_t st);
int launch_ord_sort(const DevCfg& c, const uint16_t* est, uint32_t* ord, int n, hipStream_t st);
int launch_sp_step_ord(const DevCfg& c, const SpBufs& b, const double* values, int learn, int n, int keep_overlaps,
                       const uint32_t* tm_bm, uint16_t* est, hipStream_t st);
int launch_tm_reset(const DevCfg& c, const TmBufs& b, int n, hipStream_t st);
int launch_tm_lp2_finish(const DevCfg& c, const TmBufs& b, int n, hipStream_t st);
int launch_tm_compact(const DevCfg& c, const TmBufs& b, int n, hipStream_t st);
size_t tm_step_lds_bytes(const DevCfg& c, int learn, int frozen, int nosp = 0);
size_t tm_step_lds_base(const DevCfg& c, int learn, int frozen);  // offset of the union region
int tm_configure_lds(const DevCfg& c);
int launch_prev_pred(const DevCfg& c, const TmBufs& b, int n, hipStream_t st);
