// tm.hip -- host launchers of the TM kernels, the per-stream init / reset
// kernels, the frozen-index build (rank / count / fill) and the deferred
// dutyCycle() flush.  The step kernels themselves are in tm_k_*.hip, their
// device code in tm_core.h (BacktrackingTM + raw anomaly, see its header).
#include <algorithm>

#include "tm_core.h"

size_t tm_step_lds_bytes(const DevCfg& c, int learn, int frozen, int nosp) { return tm_layout(c, learn, frozen, nosp).total; }
size_t tm_step_lds_base(const DevCfg& c, int learn, int frozen) { return tm_layout(c, learn, frozen).off_U; }

static int run_grid(const void* fn, size_t lds, int total) {
    // resident workgroups: cached per (kernel, LDS size)
    static const void* kf[8];
    static size_t kl[8];
    static int kg[8], nk = 0;
    for (int i = 0; i < nk; i++)
        if (kf[i] == fn && kl[i] == lds) return total < kg[i] ? total : kg[i];
    int per_cu = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, TM_NT, lds) != hipSuccess || per_cu < 1) per_cu = 1;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
        cus = 256;
    const int g = per_cu * cus;
    if (nk < 8) {
        kf[nk] = fn;
        kl[nk] = lds;
        kg[nk] = g;
        nk++;
    }
    return total < g ? total : g;
}

int launch_htm_run(const DevCfg& c, const TmBufs& b, const SpBufs& sp, const double* values, float* scores,
                   int n_steps, int sp_learn, int tm_learn, int frozen, int keep_prev, int keep_overlaps, int n,
                   uint32_t* wq, int unit_steps, hipStream_t st) {
    if (n <= 0 || n_steps <= 0) return 0;
    if (unit_steps < 1) unit_steps = 1;
    // (a TM-only launch needs no SP words: its own, smaller, LDS request)
    size_t lds = tm_step_lds_bytes(c, tm_learn, frozen, b.tm_only ? 1 : 0);
    const long nblk = (n_steps + unit_steps - 1) / unit_steps;
    if ((long)n * nblk >= 0x7FFFFFFFL) return -1;
    const int total = (int)(n * nblk);
    // a single unit per stream runs on the hardware dispatcher (grid = streams)
    if (nblk > 1 && hipMemsetAsync(wq, 0, ((size_t)n + 1) * sizeof(uint32_t), st) != hipSuccess) return -1;
    // a TM-only launch (ordered lockstep steps: the SP kernel ran first, with
    // its learning) needs no SP code: the inference-only frozen kernel
    const int which = tm_learn ? (b.tm_only ? 5 : 0)
                               : frozen ? (c.sp_paged ? 2 : (sp_learn && !b.tm_only) ? 4 : 1) : 3;
    // TM-only frozen launches (ordered lockstep steps): the kernel with the SP
    // compiled out (fewer registers: 153 VGPRs vs 166)
#ifdef HTM_NO_TMONLY_KERNEL  // (A/B builds: TM-only launches on the fused kernel)
    const bool tmo = false;
#else
    const bool tmo = which == 1 && b.tm_only;
#endif
    const void* fn = which == 0 ? tmk_fn_run_learn() : which == 1 ? (tmo ? tmk_fn_run_frozen_tm() : tmk_fn_run_frozen())
                     : which == 2 ? tmk_fn_run_frozen_paged() : which == 4 ? tmk_fn_run_frozen_spl()
                     : which == 5 ? tmk_fn_run_learn_tm() : tmk_fn_run_infer();
    const int grid = nblk == 1 ? total : run_grid(fn, lds, total);
    switch (which) {
        case 0: return tmk_launch_run_learn(grid, lds, st, HTM_RUN_PASS);
        case 1: return tmo ? tmk_launch_run_frozen_tm(grid, lds, st, HTM_RUN_PASS)
                           : tmk_launch_run_frozen(grid, lds, st, HTM_RUN_PASS);
        case 2: return tmk_launch_run_frozen_paged(grid, lds, st, HTM_RUN_PASS);
        case 4: return tmk_launch_run_frozen_spl(grid, lds, st, HTM_RUN_PASS);
        case 5: return tmk_launch_run_learn_tm(grid, lds, st, HTM_RUN_PASS);
        default: return tmk_launch_run_infer(grid, lds, st, HTM_RUN_PASS);
    }
}

int launch_tm_step(const DevCfg& c, const TmBufs& b, const SpBufs& sp, float* scores, int learn, int frozen, int n,
                   hipStream_t st) {
    return tmk_launch_step(learn, frozen, n, tm_step_lds_bytes(c, learn, frozen), st, c, b, sp, scores);
}

// ---------------------------------------------------------------------------
// init / reset
__global__ void tm_init_kernel(DevCfg c, TmBufs b, const uint64_t* seeds, int n) {
    int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    htm_tm_header* h = b.hdr + s;
    uint32_t st[31];
    int32_t f, r;
    rng_seed(st, f, r, seeds[s]);
    for (int i = 0; i < 31; i++) h->rng_state[i] = st[i];
    h->rng_f = f;
    h->rng_r = r;
    h->pam_counter = c.pam_len;
}

int launch_tm_init(const DevCfg& c, const TmBufs& b, const uint64_t* seeds, int n, hipStream_t st) {
    hipLaunchKernelGGL(tm_init_kernel, dim3((n + 63) / 64), dim3(64), 0, st, c, b, seeds, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Complete the pending final learn phase 2 of every stream whose last
// learning step deferred it (htm_tm_header::lp2_pending; tm_core.h
// lp2_finish): lrnPredictedState, the queued updates and the generator, as
// the step itself would have left them.  One workgroup per stream; streams
// with nothing pending return at once.
__global__ __launch_bounds__(TM_NT) void tm_lp2_finish_kernel(DevCfg c, TmBufs b) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int s = blockIdx.x;
    htm_tm_header* hdr = b.hdr + s;
    if (__builtin_amdgcn_readfirstlane(hdr->lp2_pending) == 0u) return;
    Tm t;
    tm_bind<true, false>(t, c, b, s, s, lds);
    TmSh* sh = t.sh;
    uint32_t* gbm = b.bm + (size_t)s * 4 * c.cw;
    if (threadIdx.x == 0) {
        sh->lrn_iter = hdr->lrn_iter;
        sh->rf = hdr->rng_f;
        sh->rr = hdr->rng_r;
        sh->hwm = hdr->seg_hwm;
        sh->nlive = hdr->seg_live;
        sh->n_upd = hdr->n_upd;
        sh->err = hdr->error;
        sh->st[2] = hdr->stat_lrn_phase2;
        sh->lp2p = 1;
        sh->lp2s = 0;
        sh->bytes = 0;
    }
    if (threadIdx.x < 31) sh->rng[threadIdx.x] = hdr->rng_state[threadIdx.x];
    for (int w = threadIdx.x; w < c.cw; w += TM_NT) t.lrnA1[w] = gbm[2 * c.cw + w];  // lrnActiveState of that step
    __syncthreads();
    lp2_finish(t, sh->lrn_iter);
    for (int w = threadIdx.x; w < c.cw; w += TM_NT) gbm[3 * c.cw + w] = t.lrnP1[w];
    if (threadIdx.x < 31) hdr->rng_state[threadIdx.x] = sh->rng[threadIdx.x];
    if (threadIdx.x == 0) {
        hdr->rng_f = sh->rf;
        hdr->rng_r = sh->rr;
        hdr->seg_hwm = sh->hwm;
        hdr->seg_live = sh->nlive;
        hdr->n_upd = sh->n_upd;
        hdr->error = sh->err;
        hdr->stat_lrn_phase2 = sh->st[2];
        hdr->stat_bytes += sh->bytes;
        hdr->lp2_pending = 0u;
    }
}

int launch_tm_lp2_finish(const DevCfg& c, const TmBufs& b, int n, hipStream_t st) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(tm_lp2_finish_kernel, dim3(n), dim3(TM_NT), tm_step_lds_bytes(c, 1, 0), st, c, b);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// BacktrackingTM.reset(): clears t and t-1 states (colConfidence is kept),
// flushes the update queue and the pattern histories
__global__ void tm_reset_kernel(DevCfg c, TmBufs b) {
    int s = blockIdx.x;
    uint32_t* gbm = b.bm + (size_t)s * 4 * c.cw;
    for (int i = threadIdx.x; i < 4 * c.cw; i += blockDim.x) gbm[i] = 0u;
    if (threadIdx.x == 0) {
        htm_tm_header* h = b.hdr + s;
        h->n_upd = 0;
        h->reset_called = 1;
        h->n_inf_pat = 0;
        h->n_lrn_pat = 0;
    }
}

int launch_tm_reset(const DevCfg& c, const TmBufs& b, int n, hipStream_t st) {
    hipLaunchKernelGGL(tm_reset_kernel, dim3(n), dim3(256), 0, st, c, b);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---------------------------------------------------------------------------
// Frozen forward index build.  counts[s] = total blocks of stream s.
// fx_off[s] doubles as the per-list entry counter array; scr_q2[s] holds the
// pid of each slot (~0u: not predictive-capable) between count and fill.

// Segment::dutyCycle(it, active=false) without the state update: the value
// the frozen phase 2 reads for the segment (seg_dc_update's arithmetic).
__device__ __forceinline__ float seg_dc_peek(const uint32_t* duty, uint32_t slot, uint32_t it) {
    const uint32_t* d = duty + (size_t)slot * 3;
    if (it <= kDcTier[1]) return (float)d[0] / (float)it;
    const uint32_t age = it - d[2];
    const float last = __uint_as_float(d[1]);
    if (age == 0) return last;
    float alpha = 0.0f;
    for (int t = 8; t > 0; t--) {
        if (it > kDcTier[t]) { alpha = kDcAlpha[t]; break; }
    }
    return pow_det((float)(1.0 - (double)alpha), age) * last;
}

// Ranks: live segments in (cell, slot) order -- slot order within a cell is
// creation order, NuPIC's segment list order.  Counting sort by cell (counts
// and cursors in scr_cur), then each cell's few slots sorted in place.
__global__ void tm_fx_rank_kernel(DevCfg c, TmBufs b) {
    const int s = blockIdx.x;
    const size_t sc = (size_t)c.seg_cap;
    const uint32_t* meta = b.seg_meta + (size_t)s * sc;
    uint32_t* cnt = b.scr_cur + (size_t)s * c.fx_noff;  // ncells + 1 <= fx_noff
    uint32_t* rslot = b.fx_rslot + (size_t)s * sc;
    const uint32_t hwm = b.hdr[s].seg_hwm;
    const uint32_t nc = (uint32_t)c.ncells;
    __shared__ uint32_t part[256];
    __shared__ uint32_t tot;
    for (uint32_t i = threadIdx.x; i < nc; i += blockDim.x) cnt[i] = 0u;
    __syncthreads();
    for (uint32_t slot = threadIdx.x; slot < hwm; slot += blockDim.x) {
        const uint32_t m = meta[slot];
        if (meta_live(m)) atomicAdd(&cnt[meta_cell(m)], 1u);
    }
    __syncthreads();
    const uint32_t per = (nc + blockDim.x - 1) / blockDim.x;
    const uint32_t i0 = threadIdx.x * per;
    uint32_t sum = 0;
    for (uint32_t k = 0; k < per && i0 + k < nc; k++) sum += cnt[i0 + k];
    part[threadIdx.x] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (int k = 0; k < (int)blockDim.x; k++) { uint32_t v = part[k]; part[k] = run; run += v; }
        tot = run;
        b.fx_nr[s] = run;
    }
    __syncthreads();
    uint32_t run = part[threadIdx.x];
    for (uint32_t k = 0; k < per && i0 + k < nc; k++) {
        const uint32_t v = cnt[i0 + k];
        cnt[i0 + k] = run;
        run += v;
    }
    __syncthreads();
    for (uint32_t slot = threadIdx.x; slot < hwm; slot += blockDim.x) {
        const uint32_t m = meta[slot];
        if (meta_live(m)) rslot[atomicAdd(&cnt[meta_cell(m)], 1u)] = slot;
    }
    __syncthreads();
    // cnt[x] is now the end of cell x's rank range
    for (uint32_t x = threadIdx.x; x < nc; x += blockDim.x) {
        const uint32_t lo = x ? cnt[x - 1] : 0u, hi = cnt[x];
        for (uint32_t i = lo + 1; i < hi; i++) {
            const uint32_t v = rslot[i];
            uint32_t j = i;
            while (j > lo && rslot[j - 1] > v) { rslot[j] = rslot[j - 1]; j--; }
            rslot[j] = v;
        }
    }
    (void)tot;
}

int launch_tm_fx_rank(const DevCfg& c, const TmBufs& b, int n, hipStream_t st) {
    hipLaunchKernelGGL(tm_fx_rank_kernel, dim3(n), dim3(256), 0, st, c, b);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

__global__ void tm_fx_count_kernel(DevCfg c, TmBufs b, uint64_t* counts) {
    const int s = blockIdx.x;
    const size_t sc = (size_t)c.seg_cap;
    const uint32_t* meta = b.seg_meta + (size_t)s * sc;
    const uint16_t* src = b.seg_src + (size_t)s * sc * HTM_MAXSYN;
    const uint32_t* conn = b.seg_conn + (size_t)s * sc;
    const uint32_t* rslot = b.fx_rslot + (size_t)s * sc;
    const size_t noff = (size_t)c.fx_noff;
    uint32_t* off = b.fx_off + (size_t)s * noff;
    uint32_t* pid = b.scr_q2 + (size_t)s * sc;  // by rank
    uint16_t* pcell = b.fx_pcell + (size_t)s * c.fx_pcap;
    const uint32_t nr = b.fx_nr[s];
    __shared__ uint32_t part[256];
    __shared__ uint32_t tot;
    for (size_t i = threadIdx.x; i < noff; i += blockDim.x) off[i] = 0u;
    __syncthreads();
    // window-list entry counts; predictive-capable flags over a contiguous
    // chunk of ranks per thread (pids are dense in rank order)
    const uint32_t rper = (nr + blockDim.x - 1) / blockDim.x;
    const uint32_t r0 = threadIdx.x * rper, r1 = r0 + rper < nr ? r0 + rper : nr;
    uint32_t ncap = 0;
    for (uint32_t r = r0; r < r1; r++) {
        const uint32_t slot = rslot[r];
        const uint32_t m = meta[slot];
        const uint32_t nsyn = meta_nsyn(m), w = r / (uint32_t)c.fx_win;
        for (uint32_t j = 0; j < nsyn; j++)
            atomicAdd(&off[FX_LIST(c, (int)w, src[(size_t)slot * HTM_MAXSYN + j])], 1u);
        const uint32_t cm = conn[slot] & (nsyn >= 32 ? ~0u : ((1u << nsyn) - 1u));
        uint32_t p = ~0u;
        if (__popc(cm) >= (uint32_t)c.act_thr) {
            p = 0u;
            ncap++;
        }
        pid[r] = p;
    }
    part[threadIdx.x] = ncap;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (int k = 0; k < (int)blockDim.x; k++) { uint32_t v = part[k]; part[k] = run; run += v; }
        tot = run;
        b.fx_np[s] = run;
    }
    __syncthreads();
    const uint32_t np = tot;
    if (np <= (uint32_t)c.fx_pcap) {
        uint32_t next = part[threadIdx.x];
        for (uint32_t r = r0; r < r1; r++) {
            if (pid[r] == ~0u) continue;
            const uint32_t slot = rslot[r];
            const uint32_t m = meta[slot], nsyn = meta_nsyn(m), cm = conn[slot];
            pid[r] = next;
            pcell[next] = (uint16_t)meta_cell(m);
            next++;
            for (uint32_t j = 0; j < nsyn; j++)
                if ((cm >> j) & 1u) atomicAdd(&off[FX_LIST(c, -1, src[(size_t)slot * HTM_MAXSYN + j])], 1u);
        }
    }
    __syncthreads();
    // entries -> 16-byte blocks of 8, then exclusive scan (chunked per thread)
    const size_t per = (noff + blockDim.x - 1) / blockDim.x;
    const size_t i0 = threadIdx.x * per;
    uint32_t sum = 0;
    for (size_t k = 0; k < per && i0 + k < noff; k++) {
        const uint32_t nb = (off[i0 + k] + 7u) >> 3;
        off[i0 + k] = nb;
        sum += nb;
    }
    __syncthreads();
    part[threadIdx.x] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (int k = 0; k < (int)blockDim.x; k++) { uint32_t v = part[k]; part[k] = run; run += v; }
        tot = run;
    }
    __syncthreads();
    uint32_t run = part[threadIdx.x];
    for (size_t k = 0; k < per && i0 + k < noff; k++) {
        uint32_t v = off[i0 + k];
        off[i0 + k] = run;
        run += v;
    }
    if (threadIdx.x == 0) counts[s] = tot;
}

int launch_tm_fx_count(const DevCfg& c, const TmBufs& b, uint64_t* counts, int n, hipStream_t st) {
    hipLaunchKernelGGL(tm_fx_count_kernel, dim3(n), dim3(256), 0, st, c, b, counts);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// fill: per-list entry cursors in scr_cur; fx_ent was set to 0xFF.. by the
// host, so the tail of each list's last block stays padding
__global__ void tm_fx_fill_kernel(DevCfg c, TmBufs b) {
    const int s = blockIdx.x;
    const size_t sc = (size_t)c.seg_cap;
    const uint32_t* meta = b.seg_meta + (size_t)s * sc;
    const uint16_t* src = b.seg_src + (size_t)s * sc * HTM_MAXSYN;
    const uint32_t* conn = b.seg_conn + (size_t)s * sc;
    const uint32_t* duty = b.seg_duty + (size_t)s * sc * 3;
    const uint32_t* pid = b.scr_q2 + (size_t)s * sc;
    const uint32_t* rslot = b.fx_rslot + (size_t)s * sc;
    const size_t noff = (size_t)c.fx_noff;
    const uint32_t* off = b.fx_off + (size_t)s * noff;
    uint32_t* cur = b.scr_cur + (size_t)s * noff;
    uint16_t* ent = reinterpret_cast<uint16_t*>(b.fx_ent + b.fx_base[s]);
    uint2* rec = b.fx_rec + (size_t)s * sc;
    const uint32_t nr = b.fx_nr[s];
    const uint32_t it = b.hdr[s].lrn_iter;
    const bool pid_ok = b.fx_np[s] <= (uint32_t)c.fx_pcap;
    const uint32_t W = (uint32_t)c.fx_win;
    for (size_t i = threadIdx.x; i + 1 < noff; i += blockDim.x) cur[i] = off[i] * 8u;
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < nr; r += blockDim.x) {
        const uint32_t slot = rslot[r];
        const uint32_t m = meta[slot];
        const uint32_t nsyn = meta_nsyn(m), w = r / W;
        for (uint32_t j = 0; j < nsyn; j++) {
            uint32_t pos = atomicAdd(&cur[FX_LIST(c, (int)w, src[(size_t)slot * HTM_MAXSYN + j])], 1u);
            ent[pos] = (uint16_t)(r - w * W);
        }
        // FX_FRESH: the record already holds what a frozen dutyCycle() stores
        // (lastDCIter == it past the first tier: age 0 returns without a write)
        const uint32_t fresh = (it > kDcTier[1] && duty[(size_t)slot * 3 + 2] == it) ? FX_FRESH : 0u;
        rec[r] = make_uint2(meta_cell(m) | fresh, __float_as_uint(seg_dc_peek(duty, slot, it)));
        const uint32_t p = pid[r];
        if (pid_ok && p != ~0u) {
            const uint32_t cm = conn[slot];
            for (uint32_t j = 0; j < nsyn; j++) {
                if (!((cm >> j) & 1u)) continue;
                uint32_t pos = atomicAdd(&cur[FX_LIST(c, -1, src[(size_t)slot * HTM_MAXSYN + j])], 1u);
                ent[pos] = (uint16_t)p;
            }
        }
    }
}

__global__ __launch_bounds__(TM_NT) void tm_fx_flush_kernel(DevCfg c, TmBufs b, int n);

int tm_configure_lds(const DevCfg& c) {
    // the frozen variant may exceed the default 64 KiB dynamic LDS limit
    size_t b0 = tm_step_lds_bytes(c, 1, 0), b1 = tm_step_lds_bytes(c, 0, 1), b2 = tm_step_lds_bytes(c, 0, 0);
    int r = tmk_attr_step(b0, b1, b2);
    r |= tmk_attr_run_learn(b0) | tmk_attr_run_frozen(b1) | tmk_attr_run_infer(b2) | tmk_attr_run_frozen_paged(b1) |
         tmk_attr_run_frozen_tm(tm_step_lds_bytes(c, 0, 1, 1)) |
         tmk_attr_run_frozen_spl(b1) | tmk_attr_run_learn_tm(b0);
    r |= hipFuncSetAttribute((const void*)tm_fx_flush_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)b1) ==
                 hipSuccess ? 0 : -1;
    r |= hipFuncSetAttribute((const void*)tm_lp2_finish_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)b0) ==
                 hipSuccess ? 0 : -1;
    (void)hipGetLastError();
    return r ? -1 : 0;
}

// Deferred dutyCycle() writes of frozen lockstep launches (TmBufs::fx_dlog):
// each logged phase 2 is replayed -- its active cells, the rank windows'
// counting, the first record write of every qualifying segment not yet
// written (FX_FRESH) -- by persistent workgroups claiming (stream, entry)
// pairs, each with its own qualifying list.  Entries of one stream may run
// concurrently: the writes store the value every replay computes.  The bytes
// are not added to the streams' counters (the step kernel's roofline counts
// its own work).  tm_fx_flush_done_kernel then marks the entries flushed and
// clears fx_fwork[0] (zero at allocation) for the next flush.
// The flush runs on its own stream beside later steps: it replays the entries
// [fx_dflushed, fx_dupto) -- fx_dupto is the value of fx_dsnap (the snapshot
// of fx_dn taken on the step stream when a flush was enqueued) its job
// builder read -- and the steps only append to ring slots outside that range
// (a step reads fx_dflushed, which moves only when a flush is complete, and
// only to that flush's fx_dupto; a stale read leaves it fewer free slots,
// never more).  Every job is checked before use (FX_ERR_JOB): a bad one is
// skipped and flagged, never dereferenced.
// A job is one logged entry, or (split flushes) one rank window of it: split,
// the windows of a bursting set (the longest jobs) run on separate workgroups,
// so the flush takes about one window's counting -- what a flush that a
// caller waits for wants (htm_flush, the end of a timed region); unsplit, the
// per-job setup is paid once per entry -- what the periodic flushes want
// (profiles/r04_ab/flush_split.txt).
__global__ __launch_bounds__(TM_NT) void tm_fx_flush_kernel(DevCfg c, TmBufs b, int n) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    __shared__ uint32_t job;
    const uint32_t dcap = (uint32_t)c.fx_dcap, nwin = (uint32_t)c.fx_nwin, stride = nwin + 1u;
    const uint32_t cap = (uint32_t)n * dcap * nwin;
    uint32_t total = b.fx_fwork[2];  // the job list (tm_fx_jobs_kernel, the launch before)
    if (total > cap) {
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(&b.fx_fwork[1], FX_ERR_JOBS);
        total = cap;
    }
    for (;;) {
        __syncthreads();
        if (threadIdx.x == 0) job = atomicAdd(&b.fx_fwork[0], 1u);
        __syncthreads();
        const uint32_t jj = __builtin_amdgcn_readfirstlane(job);
        if (jj >= total) break;
        // (stream * dcap + ring slot) * (nwin + 1) + window (nwin: every window)
        const uint32_t jw = __builtin_amdgcn_readfirstlane(b.fx_fjobs[jj]);
        const uint32_t win = jw % stride, j = jw / stride;
        const uint32_t su = j / dcap;
        const uint32_t i = j % dcap;
        const uint32_t len0 = su < (uint32_t)n ? (uint32_t)b.fx_dlen[(size_t)su * dcap + i] : 0xFFFFFFFFu;
        if (su >= (uint32_t)n || len0 > (uint32_t)c.max_act_cells) {
            if (threadIdx.x == 0) atomicOr(&b.fx_fwork[1], FX_ERR_JOB);
            continue;
        }
        fx_replay_entry(c, b, (int)su, i, len0, win < nwin ? (int)win : -1, blockIdx.x, lds);
    }
}

// Ordered lockstep launches (TmBufs::ord): after the SP kernel
// (sp_step_ord_kernel: est[s], the active cells TM phase 1 will list -- what a
// step's cost follows, profiles/r04_ab/lpt_sim.txt), list the streams heaviest
// first: a counting sort over ORD_NB cost buckets by one workgroup (streams
// within a bucket in no particular order -- streams are independent, so the
// order never changes a result).
__global__ __launch_bounds__(1024) void ord_sort_kernel(DevCfg c, const uint16_t* est, uint32_t* ord, int n) {
    __shared__ uint32_t hist[ORD_NB], at[ORD_NB];
    extern __shared__ uint8_t bkt[];  // [n] bucket of each stream
    const uint32_t mac = (uint32_t)c.max_act_cells;
    for (int q = threadIdx.x; q < ORD_NB; q += blockDim.x) hist[q] = 0;
    for (int s = threadIdx.x; s < n; s += blockDim.x) bkt[s] = (uint8_t)ord_bucket(est[s], mac);
    __syncthreads();
    for (int s = threadIdx.x; s < n; s += blockDim.x) atomicAdd(&hist[bkt[s]], 1u);
    __syncthreads();
    static_assert(ORD_NB == 64, "one lane per bucket");
    if (threadIdx.x < 64) {  // exclusive prefix, heaviest bucket first (lane l: bucket 63 - l)
        const uint32_t h = hist[63 - threadIdx.x];
        at[63 - threadIdx.x] = wave_incl_scan(h) - h;
    }
    __syncthreads();
    for (int s = threadIdx.x; s < n; s += blockDim.x) ord[atomicAdd(&at[bkt[s]], 1u)] = (uint32_t)s;
}

int launch_ord_sort(const DevCfg& c, const uint16_t* est, uint32_t* ord, int n, hipStream_t st) {
    if (n <= 0 || n > ORD_MAX_STREAMS) return -1;  // (n + 512 bytes of LDS)
    hipLaunchKernelGGL(ord_sort_kernel, dim3(1), dim3(1024), (size_t)n, st, c, est, ord, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Before a flush (on the flush's stream): the entries [fx_dflushed, fx_dsnap)
// of every stream as a compact job list.  Steps append to the ring beside
// this kernel but never into [fx_dflushed, fx_dsnap), so the batch is stable.
// The bound taken is stored in fx_dupto: a later snapshot the step stream
// takes while this flush runs (flushes every few steps, a flush slower than
// that) moves fx_dsnap, not what this flush completes -- its done kernel
// advances fx_dflushed to fx_dupto, so no entry is marked flushed without
// having been replayed.  One thread per stream.  No repeats to drop: a step
// logs no set equal to one still in the ring (defer_phase2), and the ring
// holds more entries than a batch (round 4 hashed every batch's cells here to
// find repeats; it found none -- 14.7 us of every flush's critical path).
// from_dn: the flush runs on the step stream after the steps (nothing appends
// meanwhile), so the bound is fx_dn itself -- no snapshot launch.
__global__ __launch_bounds__(256) void tm_fx_jobs_kernel(DevCfg c, TmBufs b, int n, int from_dn, int split) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    const uint32_t dcap = (uint32_t)c.fx_dcap;
    const uint32_t f = b.fx_dflushed[s], u = from_dn ? b.fx_dn[s] : b.fx_dsnap[s], p = u - f;
    // the ring invariant: fx_dflushed <= fx_dsnap <= fx_dflushed + fx_dcap
    // (a step appends only while fewer than fx_dcap entries are unflushed)
    const bool bad = p > dcap;
    b.fx_dupto[s] = bad ? f : u;
    if (bad) atomicOr(&b.fx_fwork[1], FX_ERR_RING);
    if (p == 0 || bad) return;
    // one job per entry, or per (entry, rank window of the stream's model) when split
    const uint32_t nwin = (uint32_t)c.fx_nwin, W = (uint32_t)c.fx_win;
    const uint32_t nr = b.fx_nr[model_stream(c, s)];
    uint32_t nw = (nr + W - 1u) / W;
    nw = nw < nwin ? nw : nwin;
    if (!split) nw = 1u;
    uint32_t base = atomicAdd(&b.fx_fwork[2], p * nw);
    const uint32_t cap = (uint32_t)n * dcap * nwin;
    for (uint32_t i = 0; i < p; i++) {
        const uint32_t e = (uint32_t)s * dcap + (f + i) % dcap;
        for (uint32_t w = 0; w < nw; w++, base++) {
            if (base < cap) b.fx_fjobs[base] = e * (nwin + 1u) + (split ? w : nwin);
            else atomicOr(&b.fx_fwork[1], FX_ERR_JOBS);
        }
    }
}

// after a flush: the entries its job builder took are flushed; the counters restart
__global__ void tm_fx_flush_done_kernel(TmBufs b, int n) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < n) b.fx_dflushed[s] = b.fx_dupto[s];
    if (s == 0) {
        b.fx_fwork[0] = 0u;
        b.fx_fwork[2] = 0u;
    }
}

// the entries a flush enqueued now covers (on the step stream, after the steps)
__global__ void tm_fx_snap_kernel(TmBufs b, int n) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < n) b.fx_dsnap[s] = b.fx_dn[s];
}

int launch_tm_fx_snap(const TmBufs& b, int n, hipStream_t st) {
    if (n <= 0 || !b.fx_dlog) return 0;
    hipLaunchKernelGGL(tm_fx_snap_kernel, dim3((n + 255) / 256), dim3(256), 0, st, b, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_tm_fx_flush(const DevCfg& c, const TmBufs& b, int n, int max_wg, hipStream_t st, int from_dn, int split) {
    if (n <= 0 || !b.fx_dlog) return 0;
    const size_t lds = tm_step_lds_bytes(c, 0, 1);
    const int total = n * c.fx_dcap * (split ? c.fx_nwin : 1);
    int grid = run_grid((const void*)tm_fx_flush_kernel, lds, total);
    if (grid > FX_FLUSH_WG) grid = FX_FLUSH_WG;
    if (max_wg > 0 && grid > max_wg) grid = max_wg;
    hipLaunchKernelGGL(tm_fx_jobs_kernel, dim3((n + 255) / 256), dim3(256), 0, st, c, b, n, from_dn, split);
    hipLaunchKernelGGL(tm_fx_flush_kernel, dim3(grid), dim3(TM_NT), lds, st, c, b, n);
    hipLaunchKernelGGL(tm_fx_flush_done_kernel, dim3((n + 255) / 256), dim3(256), 0, st, b, n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_tm_fx_fill(const DevCfg& c, const TmBufs& b, int n, hipStream_t st) {
    hipLaunchKernelGGL(tm_fx_fill_kernel, dim3(n), dim3(256), 0, st, c, b);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
