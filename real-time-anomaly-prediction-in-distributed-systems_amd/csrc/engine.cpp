// engine.cpp -- host side of the C ABI (include/htm_amd.h).
//
// Owns the device memory of all streams (one hipMalloc per buffer, sized
// from the config), derives the immutable kernel constants, and sequences
// the per-step launches: SP kernel then TM kernel on the caller's stream.
// The TM kernel variant follows the learning flags: learning on -> pool
// scans; learning off -> frozen forward index (built on the first frozen
// step after learning, one count/scan/fill pass per stream).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "htm_dev.h"

static thread_local std::string g_err;

// the message htm_last_error() returns; every HTM_E_* return of the library
// goes through here (engine.cpp and the slo / likelihood / classifier units)
int htm_fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

namespace {

#define HIP_TRY(x)                                                                          \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) return htm_fail(HTM_E_HIP, "%s: %s", #x, hipGetErrorString(e_)); \
    } while (0)

size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

}  // namespace

struct Region {
    void* base;
    size_t per_stream;
    bool model;  // part of the model (SP permanences/connections, TM segment pool): one instance in a fleet
};

// lockstep launches between two flushes of the deferred log, and the grid of
// a flush that runs beside the steps: a part of the chip fills the gaps the
// steps' tails leave; a full-width flush beside them takes the slots the next
// step's workgroups need (measured on config 2, 256-step regions ending with
// htm_flush, profiles/r03_flush: 1,024 workgroups every 8 steps 0.319 ms per
// step, 128 / 16 0.244, 256 / 8 0.243, the round-2 full-width flush on the
// step stream every 32 steps 0.246; 20-step regions 0.278 / 0.258 / 0.269).
// With ordered lockstep steps the TM launch's tail leaves more of the chip idle
// and a wider flush fills it: 768 workgroups 0.1763 ms per step vs 256 0.1801
// (512: 0.1764; 128-step regions), 20-step regions 0.1887 vs 0.1903
// (profiles/r04_ab/flush_wg.txt).  Round 6, the flush started beside the next
// TM launch at the lowest stream priority: every 4 launches 0.1515 ms per step,
// 6 0.1508, 8 0.1525, 2 0.1532 (2,324-step regions); 20-step regions 0.1618
// (4) vs 0.1646 (8) (profiles/r06_ab/flush_cadence/).  Measured again with
// 12 20-step regions per process: 6 0.1586, 4 0.1592, 8 0.1599, 10 0.1630;
// 2,324-step regions 6 0.1499 vs 4 0.1516 -- the end flush's time is not set
// by how many logged steps it covers (profiles/r06_ab/final_flush/, flush_cadence/)
#define FLUSH_EVERY 6
#define FLUSH_WG 768

struct htm_engine {
    htm_config cfg;
    DevCfg dc;
    int32_t n;
    int32_t nm = 0;      // model instances: n, or 1 in a fleet (shared model)
    bool fleet = false;
    int32_t device;
    SpBufs sp;
    TmBufs tm;
    std::vector<void*> allocs;
    size_t bytes = 0;
    int32_t sp_learn = 1, tm_learn = 1;
    int32_t use_frozen = 1;
    int32_t keep_prev = 0;
    int32_t keep_overlaps = 0;
    bool fx_valid = false;
    size_t fx_cap = 0;
    uint64_t* d_counts = nullptr;
    Region regions[HTM_ST_COUNT + 1];
    int32_t profile = 0;            // HTM_OPT_PROFILE: 0 off, N: HIP events around every N-th launch
    uint32_t prof_seq = 0;          // launches since profiling was switched on
    std::vector<hipEvent_t> ev_pool;
    std::vector<int32_t> ev_steps;  // steps covered by each profiled event triple
    std::vector<char> ev_fused;     // the triple's first event is unused (fused launch: no SP kernel)
    size_t ev_used = 0;
    int32_t fused = 1;              // HTM_OPT_FUSED
    int32_t run_chunk = 256;        // steps per fused htm_run launch
    int32_t run_unit = 0;           // steps per work unit of the fused kernel's queue (0: auto)
    uint32_t* wq = nullptr;         // the fused kernel's work queue: next unit + per-stream done blocks
    int32_t defer = 1;              // HTM_OPT_DEFER_DUTY: frozen lockstep steps defer discarded phase 2s' duty writes
    int32_t defer_steps = 0;        // lockstep launches since the last flush of the deferred log
    int32_t flush_every = 0;        // lockstep launches between flushes (0: FLUSH_EVERY)
    // the flush of the deferred log runs on its own stream, concurrently with
    // the next steps (they never read the records it writes): a snapshot of
    // the log counters on the step stream, the flush on fstream after it
    hipStream_t fstream = nullptr;
    hipEvent_t ev_logged = nullptr;   // step stream: the snapshot of the log counters
    hipEvent_t ev_flushed = nullptr;  // fstream: the last enqueued flush is complete
    bool flush_pending = false;       // ev_flushed not yet waited for by a step stream or the host
    int32_t final_split = 1;          // htm_flush's flush: jobs per (entry, rank window) (A/B knob HTM_FINAL_SPLIT)
    int32_t flush_mode = 0;           // 0: flush stream beside the steps; 1: on the step stream
    int32_t flush_wg = FLUSH_WG;      // grid of a flush beside the steps
    int32_t flush_prio = 1;           // 1: the flush stream at the lowest priority (round 6: config 2
                                      // 0.1548 -> 0.1529 ms/step same box, profiles/r06_ab/flush_stream/)
    size_t enc_cap = 0;               // steps SpBufs::enc_in holds (RDSE engines)
    bool conf_packed = false;         // a step kernel wrote colConfidence packed since the last densify
    bool lp2_pending = false;         // a learning step may have left its final learn phase 2 pending
    int32_t ordered = 1;              // HTM_OPT_ORDERED: frozen lockstep steps run their TM steps heaviest first
    int32_t split_learn = 1;          // HTM_OPT_SPLIT_LEARN: learning lockstep steps run the SP kernel, then TM-only
    uint32_t* ord = nullptr;          // [n] the ordered launch's stream of each workgroup
    uint16_t* ord_est = nullptr;      // [n] each stream's TM cost estimate (sp_step_ord_kernel)
    unsigned long long* wg_trace = nullptr;  // A/B builds: HTM_WG_TRACE timeline of the latest lockstep launch
    size_t wg_trace_cap = 0;
};


// A/B and tuning knobs read from the environment exist only in the A/B build
// (make ab -> libhtm_amd_ab.so, -DHTM_AB_KNOBS; tools/ab_libs.py loads it);
// the product library ignores the environment.
static const char* ab_knob(const char* name) {
#ifdef HTM_AB_KNOBS
    return std::getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

static int flush_deferred(htm_engine* e, hipStream_t st);
static int flush_sync(htm_engine* e);
static int grow_enc(htm_engine* e, size_t steps, hipStream_t st);
static int densify_conf(htm_engine* e, hipStream_t st);

extern "C" {

void htm_default_config(htm_config* c) {
    std::memset(c, 0, sizeof(*c));
    c->n_fields = 1;
    c->enc_n = 500;
    c->enc_w = 21;
    c->enc_minval = 0.0;
    c->enc_maxval = 100.0;
    c->enc_clip = 1;
    c->sp_columns = 2048;
    c->sp_num_active = 40;
    c->sp_potential_pct = 0.8f;
    c->sp_perm_connected = 0.1f;
    c->sp_perm_active_inc = 0.0001f;
    c->sp_perm_inactive_dec = 0.0005f;
    c->sp_min_pct_overlap_dc = 0.001f;
    c->sp_duty_cycle_period = 1000;
    c->sp_boost_strength = 0.0f;
    c->sp_stimulus_threshold = 0;
    c->sp_update_period = 50;
    c->sp_seed = 2045;
    c->tm_cells_per_col = 12;
    c->tm_new_syn_count = 20;
    c->tm_max_syn_per_seg = 32;
    c->tm_max_segs_per_cell = 128;
    c->tm_initial_perm = 0.21f;
    c->tm_connected_perm = 0.5f;
    c->tm_perm_inc = 0.1f;
    c->tm_perm_dec = 0.1f;
    c->tm_perm_max = 1.0f;
    c->tm_min_threshold = 9;
    c->tm_activation_threshold = 12;
    c->tm_pam_length = 3;
    c->tm_max_inf_backtrack = 10;
    c->tm_max_lrn_backtrack = 5;
    c->tm_max_seq_length = 32;
    c->tm_seg_update_valid_duration = 5;
    c->tm_seed = 2045;
    c->seg_capacity = 1 << 17;
    c->upd_capacity = 2048;
    c->seed_stride = 0;
    c->enc_type = HTM_ENC_SCALAR;
    c->rdse_resolution = 0.88;
    c->rdse_seed = 1;
}

}  // extern "C"

static int derive(const htm_config& c, int32_t n, size_t lds_budget, DevCfg& d) {
    const bool sdr = c.sdr_bits != 0;
    if (sdr) {
        if (c.sdr_bits < 1 || c.sdr_bits > HTM_MAX_SDR)
            return htm_fail(HTM_E_INVALID, "sdr_bits must be 0 (encoder input) or 1..%d", HTM_MAX_SDR);
    } else {
        if (c.n_fields < 1 || c.n_fields > 4) return htm_fail(HTM_E_INVALID, "n_fields must be 1..4");
        if (c.enc_w < 1 || c.enc_w >= c.enc_n || c.enc_n * c.n_fields > 2048)
            return htm_fail(HTM_E_INVALID, "encoder n/w out of range");
        if (c.n_fields * c.enc_w >= 128) return htm_fail(HTM_E_INVALID, "n_fields*w must be < 128");
        if (c.enc_type != HTM_ENC_SCALAR && c.enc_type != HTM_ENC_RDSE)
            return htm_fail(HTM_E_INVALID, "enc_type must be HTM_ENC_SCALAR or HTM_ENC_RDSE");
        // RandomDistributedScalarEncoder.__init__'s checks (w odd, n > 6 w,
        // resolution > 0); n <= 500 w lets the init shuffle run in the map rows
        if (c.enc_type == HTM_ENC_RDSE &&
            (c.enc_w % 2 == 0 || c.enc_n <= 6 * c.enc_w || c.enc_n > (HTM_RDSE_BUCKETS / 2) * c.enc_w ||
             !(c.rdse_resolution > 0.0)))
            return htm_fail(HTM_E_INVALID, "RDSE needs an odd w, 6 w < n <= 500 w and resolution > 0");
    }
    if (c.sp_columns < 64 || c.sp_columns % 64 != 0 || c.sp_columns > 4096)
        return htm_fail(HTM_E_INVALID, "sp_columns must be a multiple of 64 in [64, 4096]");
    if (c.sp_num_active < 1 || c.sp_num_active > HTM_MAXACT) return htm_fail(HTM_E_INVALID, "sp_num_active must be 1..64");
    if (!(c.sp_boost_strength >= 0.0f) || c.sp_boost_strength > 1000.0f)
        return htm_fail(HTM_E_INVALID, "boostStrength must be in [0, 1000]");
    if (c.sp_stimulus_threshold < 0 || c.sp_stimulus_threshold > 127) return htm_fail(HTM_E_INVALID, "stimulus threshold");
    if (c.tm_cells_per_col < 2 || c.tm_cells_per_col > HTM_MAXK) return htm_fail(HTM_E_INVALID, "cells_per_col must be 2..32");
    if ((int64_t)c.sp_columns * c.tm_cells_per_col > 65536) return htm_fail(HTM_E_INVALID, "columns*cells must be <= 65536");
    if (c.tm_max_syn_per_seg < 1 || c.tm_max_syn_per_seg > HTM_MAXSYN) return htm_fail(HTM_E_INVALID, "max_syn_per_seg 1..32");
    if (c.tm_new_syn_count < 1 || c.tm_new_syn_count > c.tm_max_syn_per_seg)
        return htm_fail(HTM_E_INVALID, "new_syn_count must be 1..max_syn_per_seg");
    if (c.tm_max_segs_per_cell < 1 || c.tm_max_segs_per_cell > 255) return htm_fail(HTM_E_INVALID, "max_segs_per_cell 1..255");
    if (c.tm_max_inf_backtrack < 0 || c.tm_max_inf_backtrack > HTM_MAXPAT - 1 || c.tm_max_lrn_backtrack < 0 ||
        c.tm_max_lrn_backtrack > HTM_MAXPAT - 1)
        return htm_fail(HTM_E_INVALID, "backtrack depth must be 0..15");
    if (c.tm_pam_length < 1) return htm_fail(HTM_E_INVALID, "pamLength must be > 0");
    if (c.tm_activation_threshold < 1 || c.tm_activation_threshold > HTM_MAXSYN || c.tm_min_threshold < 1 ||
        c.tm_min_threshold > HTM_MAXSYN)
        return htm_fail(HTM_E_INVALID, "activation/min thresholds must be 1..32");
    if (c.seg_capacity < 64 || c.seg_capacity > (1 << 27)) return htm_fail(HTM_E_INVALID, "seg_capacity");
    if (c.upd_capacity < 1 || c.upd_capacity > 65535) return htm_fail(HTM_E_INVALID, "upd_capacity");
    std::memset(&d, 0, sizeof(d));
    d.n_fields = sdr ? 0 : c.n_fields;
    d.enc_type = sdr ? HTM_ENC_SCALAR : c.enc_type;
    d.rdse_res = c.rdse_resolution;
    d.rdse_block = (int32_t)(RDSE_HDR_WORDS * 4 + round_up((size_t)HTM_RDSE_BUCKETS * c.enc_w * 2, 16));
    d.enc_list = (int32_t)round_up((size_t)c.n_fields * c.enc_w + 1, 8);
    d.enc_n = c.enc_n;
    d.enc_w = c.enc_w;
    d.enc_clip = c.enc_clip;
    for (int f = 0; f < 4; f++) {
        const bool own = c.field_maxval[f] > c.field_minval[f];
        d.enc_min[f] = own ? c.field_minval[f] : c.enc_minval;
        d.enc_max[f] = own ? c.field_maxval[f] : c.enc_maxval;
        d.enc_resolution[f] = (d.enc_max[f] - d.enc_min[f]) / (double)(c.enc_n - c.enc_w);
    }
    d.enc_halfwidth = (c.enc_w - 1) / 2;
    d.nin = sdr ? c.sdr_bits : c.n_fields * c.enc_n;
    d.sdr_in = sdr ? 1 : 0;
    d.nin_pad = (int32_t)round_up((size_t)d.nin, 32);
    d.ncol = c.sp_columns;
    d.nw = c.sp_columns / 32;
    // mapPotential_: WrappingNeighborhood(radius = inputWidth) covers all inputs
    d.n_potential = (int32_t)roundf((float)d.nin * c.sp_potential_pct);
    // paged permanences: a shared pool of n * sp_perm_rows rows (row index u32)
    if (c.sp_perm_rows < 0 || (uint64_t)c.sp_perm_rows * (uint64_t)n >= 0xFFFFFFFFull)
        return htm_fail(HTM_E_INVALID, "sp_perm_rows must be >= 0 and n_streams * sp_perm_rows < 2^32");
    d.sp_paged = c.sp_perm_rows > 0 ? 1 : 0;
    d.n_ckpt = (c.sp_columns + SP_CKPT_COLS - 1) / SP_CKPT_COLS;
    d.pool_stride = (int32_t)round_up((size_t)d.n_potential, 32);
    d.pool_rows = (uint64_t)c.sp_perm_rows * (uint64_t)n;
    // inhibitColumns_: inhibitionRadius = max(columnDimensions) (global)
    uint32_t area = (uint32_t)powf((float)(2 * c.sp_columns + 1), 1.0f);
    if (area > (uint32_t)c.sp_columns) area = (uint32_t)c.sp_columns;
    float density = (float)c.sp_num_active / (float)area;
    if (density > 0.5f) density = 0.5f;
    d.num_desired = (int32_t)(uint32_t)(density * (float)c.sp_columns);
    // updateBoostFactorsGlobal_: the same target density (global inhibition)
    d.sp_boost = c.sp_boost_strength;
    d.sp_target = density;
    if (d.num_desired > HTM_MAXACT) return htm_fail(HTM_E_INVALID, "too many winners");
    d.stim_thr = c.sp_stimulus_threshold;
    d.dc_period = c.sp_duty_cycle_period;
    d.update_period = c.sp_update_period;
    d.sp_conn = c.sp_perm_connected;
    d.sp_conn_thr = c.sp_perm_connected - 0.000001f;
    d.sp_inc = c.sp_perm_active_inc;
    d.sp_dec = c.sp_perm_inactive_dec;
    d.sp_trim = (float)((double)c.sp_perm_active_inc / 2.0);
    d.sp_below_inc = (float)((double)c.sp_perm_connected / 10.0);
    d.sp_min_pct_odc = c.sp_min_pct_overlap_dc;
    d.K = c.tm_cells_per_col;
    d.ncells = c.sp_columns * c.tm_cells_per_col;
    d.cw = d.ncells / 32;
    d.kmagic = (uint32_t)((4294967296ull + (uint64_t)d.K - 1) / (uint64_t)d.K);
    d.new_syn = c.tm_new_syn_count;
    d.max_syn = c.tm_max_syn_per_seg;
    d.max_segs_per_cell = c.tm_max_segs_per_cell;
    d.init_perm = c.tm_initial_perm;
    d.tm_conn = c.tm_connected_perm;
    d.tm_inc = c.tm_perm_inc;
    d.tm_dec = c.tm_perm_dec;
    d.tm_max = c.tm_perm_max;
    d.min_thr = c.tm_min_threshold;
    d.act_thr = c.tm_activation_threshold;
    d.pam_len = c.tm_pam_length;
    d.max_inf_bt = c.tm_max_inf_backtrack;
    d.max_lrn_bt = c.tm_max_lrn_backtrack;
    d.max_seq_len = c.tm_max_seq_length;
    d.upd_valid = c.tm_seg_update_valid_duration;
    d.seg_cap = c.seg_capacity;
    d.upd_cap = c.upd_capacity;
    d.seg_reserve = (c.tm_max_lrn_backtrack + 2) * c.sp_num_active;
    if (d.seg_reserve >= d.seg_cap) return htm_fail(HTM_E_INVALID, "seg_capacity too small for one learning step");
    d.n_streams = n;
    d.shared_model = 0;
    d.q_cap = d.seg_cap;
    d.max_act_cells = d.num_desired * d.K;
    // qualifying segments ranked in LDS: as many (<= 1024) as the phase-2
    // bucket arrays leave room for in the LDS budget; more go through HBM
    {
        // (the finish arrays are the learning / pool-scan layouts': sized as at
        // three frozen workgroups per CU whatever the frozen budget)
        const size_t qb = std::max(lds_budget, (size_t)52 * 1024);
        const size_t off_u0 = tm_step_lds_base(d, 0, 1);
        const size_t avail0 = qb > off_u0 ? (qb - off_u0) / 4 : 0;
        const size_t fixed = (size_t)d.ncol + (size_t)(d.ncol + 1) / 2 + (size_t)d.ncol + 1 + (size_t)d.nw;
        size_t q = avail0 > fixed ? (avail0 - fixed) * 2 / 9 : 0;
        q = q / 64 * 64;
        if (q > 1024) q = 1024;
        if (q < 64) return htm_fail(HTM_E_INVALID, "LDS budget %zu too small for the phase-2 buckets", qb);
        d.q_lds = (int32_t)q;
    }
    // measured (profiles/r01_ab): the nonzero-column bitmap beats column buckets (+1.5%) and the
    // bitonic key sort at Model-1 sizes
    d.fin_mode = 2;
    // learning steps defer their final learn phase 2 into the next step's first
    // pool scan (tm_core.h lp2_finish): 32-bit keys hold slots < 2^21
    d.lp2_defer = d.seg_cap <= (1 << 21) ? 1 : 0;
#ifdef HTM_NO_LP2_DEFER  // (A/B builds)
    d.lp2_defer = 0;
#endif
    // the first block -> list map of a frozen window: written with the list
    // starts (one barrier less) at Model-1's 12 cells per column (config 2
    // 0.1546 -> 0.1531 ms/step); after their barrier at 32 (model.yaml fleet
    // 23.31 -> 22.35 ms/step), where a thread's run of list starts is long
    // (profiles/r06_ab/owner_map/)
    d.fx_own_sep = d.K > 16 ? 1 : 0;
    if (const char* env = ab_knob("HTM_FX_OWN_SEP")) d.fx_own_sep = std::atoi(env) ? 1 : 0;  // A/B knob
    if (const char* env = ab_knob("HTM_TM_FIN"))
        d.fin_mode = std::strcmp(env, "sorted") == 0 ? 1 : std::strcmp(env, "buckets") == 0 ? 0 : 2;
    // frozen-inference counter window: the union region holds the u8
    // counters (fx_win bytes) plus the active-cell list and its block prefix;
    // fill the LDS budget (two workgroups per CU by default).  Out-list
    // entries are window-relative u16 with 0xFFFF as padding.
    const size_t off_u = tm_step_lds_base(d, 0, 1);
    const size_t cell_words = 64 + (size_t)(d.max_act_cells + 1) / 2 + 2 * (size_t)d.max_act_cells + 1 + FX_OWN / 2;
    size_t avail = lds_budget > off_u ? (lds_budget - off_u) / 4 : 0;
    size_t win = avail > cell_words ? (avail - cell_words) * 4 : 0;
    // 64-slot granularity (counter sweeps work in 16-byte quads): a window a
    // few hundred slots wider can save a whole pass per phase 2 (config 2:
    // 68,376 live segments fit 3 windows of 22,976, not of 22,528)
    size_t gran = 64;
    if (const char* env = ab_knob("HTM_FX_GRAN")) gran = (size_t)std::max(64, std::atoi(env)) / 64 * 64;  // A/B knob
    win = (win / gran) * gran;
    if (win < 1024) win = 1024;
    if (win > 64512) win = 64512;
    if (const char* env = ab_knob("HTM_FX_WIN_MAX"))  // A/B knob: a narrower window (occupancy study)
        win = std::min(win, (size_t)std::max(1024, std::atoi(env)) / 64 * 64);
    size_t capr = round_up((size_t)d.seg_cap, 64);
    if (win > capr) win = capr;
    d.fx_win = (int32_t)win;
    d.fx_nwin = (int32_t)((d.seg_cap + d.fx_win - 1) / d.fx_win);
    d.fx_pcap = d.fx_win < 65535 ? d.fx_win : 65535;
    if (const char* env = ab_knob("HTM_FX_PID"))  // A/B knob: 0 = no pid lists (rows path)
        if (std::atoi(env) == 0) d.fx_pcap = 0;
    d.fx_noff = d.ncells * d.fx_nwin + d.ncells + 1;
    // deferred phase-2 log entries per stream (lockstep): a flush every
    // fx_dcap / 2 steps keeps them from filling (a full log falls back to
    // counting in the step); measured on config 2 (profiles/r02_defer):
    // 64 entries flushed every 32 steps 0.273 ms/step, 32 / 16 0.276, 16 / 8 0.304
    d.fx_dcap = n <= 16384 ? 64 : 8;
    if (const char* env = ab_knob("HTM_DEFER_CAP")) d.fx_dcap = std::min(64, std::max(1, std::atoi(env)));  // A/B knob (the flush's job builder handles <= 64)
    // the ranked phase-2 tail keeps a u16 column and a f32 dutyCycle per
    // qualifying segment in the union region (free once the counting is
    // done): bursting steps (~1,500-2,000 qualifying segments on config 2) stay
    // in LDS instead of taking the HBM-scratch path
    {
        // (the TM-only launch's union: no SP words -- the smaller of the two frozen layouts)
        const size_t uw = (tm_step_lds_bytes(d, 0, 1, 1) - tm_step_lds_base(d, 0, 1)) / 4;
        d.q_lds_fx = (int32_t)(uw * 2 / 3 / 64 * 64);
    }
    return HTM_OK;
}

static int dalloc(htm_engine* e, void** p, size_t bytes) {
    if (bytes == 0) bytes = 16;
    hipError_t err = hipMalloc(p, bytes);
    if (err != hipSuccess) return htm_fail(HTM_E_HIP, "hipMalloc(%zu): %s", bytes, hipGetErrorString(err));
    err = hipMemset(*p, 0, bytes);
    if (err != hipSuccess) return htm_fail(HTM_E_HIP, "hipMemset: %s", hipGetErrorString(err));
    e->allocs.push_back(*p);
    e->bytes += bytes;
    return HTM_OK;
}

#define ALLOC(field, T, count)                                                     \
    do {                                                                           \
        void* p_ = nullptr;                                                        \
        int r_ = dalloc(e, &p_, (size_t)(count) * sizeof(T));                      \
        if (r_) return r_;                                                         \
        field = reinterpret_cast<T*>(p_);                                          \
    } while (0)

// B^(2^p), p < SP_JUMP_POW, of the block map st[(3 + j) % 31] += st[j] (j = 0..30),
// row j column i = the weight of st[i] in the new st[j]; rows padded to 32 words
static void sp_jump_tables(std::vector<uint32_t>& out) {
    std::vector<uint32_t> m(31 * 31), t(31 * 31);
    for (int i = 0; i < 31; i++) {
        uint32_t st[31] = {0};
        st[i] = 1u;
        for (int j = 0; j < 31; j++) st[(3 + j) % 31] += st[j];
        for (int j = 0; j < 31; j++) m[j * 31 + i] = st[j];
    }
    out.assign((size_t)SP_JUMP_POW * 31 * 32, 0u);
    for (int p = 0; p < SP_JUMP_POW; p++) {
        for (int j = 0; j < 31; j++)
            for (int i = 0; i < 31; i++) out[((size_t)p * 31 + j) * 32 + i] = m[j * 31 + i];
        for (int j = 0; j < 31; j++)  // m = m * m (mod 2^32)
            for (int i = 0; i < 31; i++) {
                uint32_t a = 0;
                for (int k = 0; k < 31; k++) a += m[j * 31 + k] * m[k * 31 + i];
                t[j * 31 + i] = a;
            }
        m.swap(t);
    }
}

static int allocate(htm_engine* e) {
    const DevCfg& d = e->dc;
    const size_t S = (size_t)e->n;
    const size_t M = (size_t)e->nm;  // model instances
    const size_t cap = (size_t)d.seg_cap;
    ALLOC(e->wq, uint32_t, S + 1);
    ALLOC(e->sp.connT, uint32_t, M * d.nin_pad * d.nw);
    ALLOC(e->sp.potmask, uint32_t, M * d.ncol * (d.nin_pad / 32));
    if (d.sp_paged) {
        e->sp.perm = nullptr;
        ALLOC(e->sp.prow, uint32_t, M * d.ncol);
        HIP_TRY(hipMemset(e->sp.prow, 0xFF, M * d.ncol * 4));  // SP_ROW_NONE: initial values
        ALLOC(e->sp.pool, float, (size_t)d.pool_rows * d.pool_stride);
        ALLOC(e->sp.pool_next, unsigned long long, 1);
        ALLOC(e->sp.ckpt, uint32_t, M * d.n_ckpt * SP_CKPT_WORDS);
        {
            // jump tables of the replays' skip (sp_jump_blocks): B^(2^p), B the
            // 31-draw block map of nupic::Random's state, linear over Z/2^32
            std::vector<uint32_t> jt;
            sp_jump_tables(jt);
            uint32_t* dj = nullptr;
            ALLOC(dj, uint32_t, jt.size());
            HIP_TRY(hipMemcpy(dj, jt.data(), jt.size() * 4, hipMemcpyHostToDevice));
            e->sp.jump = dj;
        }
    } else {
        ALLOC(e->sp.perm, float, M * d.ncol * d.n_potential);
    }
    ALLOC(e->sp.err, uint32_t, S);
    ALLOC(e->sp.duty, float, M * 2 * d.ncol);
    ALLOC(e->sp.boost, float, M * d.ncol);
    ALLOC(e->sp.enc_bucket, int32_t, S * 4);
    const size_t rdse_per = d.enc_type == HTM_ENC_RDSE ? (size_t)d.n_fields * d.rdse_block : 0;
    if (rdse_per) {
        ALLOC(e->sp.rdse, uint8_t, S * rdse_per);
        ALLOC(e->sp.rdse_seeds, uint64_t, S);
    } else {
        e->sp.rdse = nullptr;
        e->sp.rdse_seeds = nullptr;
    }
    e->sp.enc_in = nullptr;
    ALLOC(e->sp.scalars, uint32_t, S * 4);
    ALLOC(e->sp.act, uint16_t, S * HTM_MAXACT);
    ALLOC(e->sp.nact, uint32_t, S);
    ALLOC(e->sp.overlaps, int32_t, S * d.ncol);
    ALLOC(e->sp.seeds, uint64_t, S);
    ALLOC(e->tm.hdr, htm_tm_header, S);
    ALLOC(e->tm.bm, uint32_t, S * 4 * d.cw);
    ALLOC(e->tm.colconf, float, S * d.ncol);
    ALLOC(e->tm.pat, uint16_t, S * 2 * HTM_MAXPAT * HTM_MAXACT);
    ALLOC(e->tm.seg_meta, uint32_t, M * cap);
    ALLOC(e->tm.seg_src, uint16_t, M * cap * HTM_MAXSYN);
    ALLOC(e->tm.seg_perm, float, M * cap * HTM_MAXSYN);
    ALLOC(e->tm.seg_conn, uint32_t, M * cap);
    ALLOC(e->tm.seg_duty, uint32_t, M * cap * 3);
    ALLOC(e->tm.cell_nseg, uint8_t, M * d.ncells);
    ALLOC(e->tm.upd, htm_tm_update, M * d.upd_cap);
    ALLOC(e->tm.scr_bm, uint32_t, S * 5 * d.cw);
    ALLOC(e->tm.scr_conf, float, S * d.ncol);
    ALLOC(e->tm.scr_q, uint32_t, S * (size_t)d.q_cap);
    ALLOC(e->tm.scr_q2, uint32_t, std::max(S * (size_t)d.q_cap, cap));
    ALLOC(e->tm.prev_pred, uint8_t, S * d.ncol);
    ALLOC(e->tm.colnz, uint32_t, S * ((size_t)d.nw + 1));
    ALLOC(e->tm.colval, float, S * d.ncol);
    ALLOC(e->tm.fx_base, uint64_t, S);
    ALLOC(e->d_counts, uint64_t, S);
#ifdef HTM_STAMPS
    ALLOC(e->tm.dbg, uint64_t, S * 4 * HTM_NSTAMP);
    ALLOC(e->sp.dbg, uint64_t, S * 4);
#endif
    e->tm.fx_ent = nullptr;
    // region table for export / import / save / load / replicate
    Region* r = e->regions;
    for (int i = 0; i <= HTM_ST_COUNT; i++) r[i] = Region{nullptr, 0, false};
    r[HTM_ST_SP_CONNT] = {e->sp.connT, (size_t)d.nin_pad * d.nw * 4, true};
    r[HTM_ST_SP_POTMASK] = {e->sp.potmask, (size_t)d.ncol * (d.nin_pad / 32) * 4, true};
    // paged engines: no base (export/import convert to and from the dense layout)
    r[HTM_ST_SP_PERM] = {e->sp.perm, (size_t)d.ncol * d.n_potential * 4, true};
    r[HTM_ST_SP_PERM_CKPT] = {e->sp.ckpt, d.sp_paged ? (size_t)d.n_ckpt * SP_CKPT_WORDS * 4 : 0, true};
    r[HTM_ST_SP_DUTY] = {e->sp.duty, (size_t)2 * d.ncol * 4, true};
    r[HTM_ST_SP_BOOST] = {e->sp.boost, (size_t)d.ncol * 4, true};
    r[HTM_ST_ENC_RDSE] = {e->sp.rdse, rdse_per, false};
    r[HTM_ST_SP_SCALARS] = {e->sp.scalars, 16, false};
    r[HTM_ST_TM_HEADER] = {e->tm.hdr, sizeof(htm_tm_header), false};
    r[HTM_ST_TM_BITMAPS] = {e->tm.bm, (size_t)4 * d.cw * 4, false};
    r[HTM_ST_TM_COLCONF] = {e->tm.colconf, (size_t)d.ncol * 4, false};
    r[HTM_ST_TM_SEG_META] = {e->tm.seg_meta, cap * 4, true};
    r[HTM_ST_TM_SEG_SRC] = {e->tm.seg_src, cap * HTM_MAXSYN * 2, true};
    r[HTM_ST_TM_SEG_PERM] = {e->tm.seg_perm, cap * HTM_MAXSYN * 4, true};
    r[HTM_ST_TM_SEG_CONN] = {e->tm.seg_conn, cap * 4, true};
    r[HTM_ST_TM_SEG_DUTY] = {e->tm.seg_duty, cap * 12, true};
    r[HTM_ST_TM_CELL_NSEG] = {e->tm.cell_nseg, (size_t)d.ncells, true};
    r[HTM_ST_TM_PATTERNS] = {e->tm.pat, (size_t)2 * HTM_MAXPAT * HTM_MAXACT * 2, false};
    r[HTM_ST_TM_UPDATES] = {e->tm.upd, (size_t)d.upd_cap * sizeof(htm_tm_update), true};
    return HTM_OK;
}

static int query_lds_optin() {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeSharedMemPerBlockOptin, dev) != hipSuccess || v <= 0) {
        (void)hipGetLastError();
        v = 65536;
        (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, dev);
    }
    return v;
}

static int check_lds(const DevCfg& d) {
    int maxlds = query_lds_optin();
    for (int learn = 0; learn < 2; learn++)
        for (int fz = 0; fz < 2; fz++) {
            if (learn && fz) continue;
            size_t b = tm_step_lds_bytes(d, learn, fz);
            if (b > (size_t)maxlds) return htm_fail(HTM_E_INVALID, "TM kernel needs %zu B LDS > %d", b, maxlds);
        }
    return HTM_OK;
}

static int create_uninit(const htm_config* cfg, int32_t n_streams, int32_t device, htm_engine** out,
                         int32_t fleet_q_cap = 0) {
    if (!cfg || !out || n_streams < 1) return htm_fail(HTM_E_INVALID, "bad arguments");
    *out = nullptr;
    HIP_TRY(hipSetDevice(device));
    htm_engine* e = new htm_engine();
    e->cfg = *cfg;
    e->n = n_streams;
    e->fleet = fleet_q_cap > 0;
    e->nm = e->fleet ? 1 : n_streams;
    e->device = device;
    int optin = query_lds_optin();
    // three frozen-inference workgroups per CU (HTM_RUN_WAVES): 160 KiB / 3,
    // less the run kernel's static LDS, rounded down to 1 KiB
    size_t budget = optin >= 54 * 1024 ? (size_t)52 * 1024 : (size_t)optin - 2048;
#ifdef HTM_TM_LDS_BUDGET_DEFAULT
    // (experiment builds, e.g. four frozen TM-only workgroups per CU: 40 KiB)
    budget = std::min(budget, (size_t)HTM_TM_LDS_BUDGET_DEFAULT);
#endif
    if (const char* env = ab_knob("HTM_TM_LDS_BUDGET")) {  // tuning knob (bytes)
        long v = std::strtol(env, nullptr, 10);
        if (v >= 16384 && v <= optin) budget = (size_t)v;
    }
    if (const char* env = ab_knob("HTM_FUSED")) e->fused = std::atoi(env) != 0;  // A/B knob
    if (const char* env = ab_knob("HTM_RUN_UNIT")) e->run_unit = std::max(1, std::atoi(env));  // A/B knob
    if (const char* env = ab_knob("HTM_DEFER_DUTY")) e->defer = std::atoi(env) != 0;            // A/B knob
    if (const char* env = ab_knob("HTM_DEFER_FLUSH_EVERY")) e->flush_every = std::max(1, std::atoi(env));  // test knob
    // fleet-sized engines (8-entry logs, a flush every 4 steps) flush on the
    // step stream: beside the steps, 131,072-stream fleets ran bimodal (15 or
    // 30 ms per step) and faulted (illegal address) in some runs; on the step
    // stream 14.7 ms (Model-1) / 23.5 ms (model.yaml), clean in every run
    // (profiles/r03_ab/fleet_flush_mode.txt)
    if (n_streams > 16384) e->flush_mode = 1;
    if (const char* env = ab_knob("HTM_FLUSH_MODE")) e->flush_mode = std::atoi(env);                 // A/B knob
    if (const char* env = ab_knob("HTM_FLUSH_WG")) e->flush_wg = std::max(0, std::atoi(env));         // A/B knob
    if (const char* env = ab_knob("HTM_ORDERED")) e->ordered = std::atoi(env) ? 1 : 0;               // A/B knob
    if (const char* env = ab_knob("HTM_FLUSH_PRIO")) e->flush_prio = std::atoi(env);                 // A/B knob
    if (const char* env = ab_knob("HTM_FINAL_SPLIT")) e->final_split = std::atoi(env) ? 1 : 0;       // A/B knob
    int r = derive(*cfg, n_streams, budget, e->dc);
    if (r && !ab_knob("HTM_TM_LDS_BUDGET") && optin >= 78 * 1024) {
        // shapes whose fixed LDS state leaves no room at 3 workgroups per CU
        // (e.g. 32 cells per column) run at 2
        budget = (size_t)76 * 1024;
        r = derive(*cfg, n_streams, budget, e->dc);
    }
    if (r && !ab_knob("HTM_TM_LDS_BUDGET") && optin > 78 * 1024) {
        // 4096 columns (config 5): one workgroup per CU
        budget = (size_t)optin - 2048;
        r = derive(*cfg, n_streams, budget, e->dc);
    }
    if (!r && e->dc.sdr_in) e->fused = 0;  // SDR input: SP kernel + TM kernel per step
    if (!r && e->fleet) {
        e->dc.shared_model = 1;
        e->dc.q_cap = std::min(fleet_q_cap, e->dc.seg_cap);
        e->sp_learn = e->tm_learn = 0;
    }
    if (!r) r = check_lds(e->dc);
    if (!r) r = allocate(e);
    if (!r) r = grow_enc(e, 1, nullptr);  // RDSE engines: one step's lists now (longer launches grow them)
    if (!r && tm_configure_lds(e->dc)) {
        size_t mx = std::max(tm_step_lds_bytes(e->dc, 0, 1),
                             std::max(tm_step_lds_bytes(e->dc, 1, 0), tm_step_lds_bytes(e->dc, 0, 0)));
        if (mx > 65536) r = htm_fail(HTM_E_HIP, "cannot raise the dynamic LDS limit to %zu B", mx);
    }
    if (r) {
        for (void* p : e->allocs) (void)hipFree(p);
        if (e->sp.enc_in) (void)hipFree(e->sp.enc_in);
        delete e;
        return r;
    }
    *out = e;
    return HTM_OK;
}

extern "C" {

// NuPIC initialisation of a created engine (SP pools/permanences, TM RNG)
static int init_streams(htm_engine* e, const htm_config* cfg, int32_t n_streams, uint64_t** dseeds) {
    std::vector<uint64_t> seeds((size_t)n_streams);
    for (int s = 0; s < n_streams; s++) seeds[s] = cfg->sp_seed + (uint64_t)s * (uint64_t)cfg->seed_stride;
    HIP_TRY(hipMemcpy(e->sp.seeds, seeds.data(), seeds.size() * 8, hipMemcpyHostToDevice));
    if (launch_sp_init(e->dc, e->sp, n_streams, 0)) return htm_fail(HTM_E_HIP, "sp_init launch failed");
    if (e->sp.rdse) {
        std::vector<uint64_t> rs((size_t)n_streams);
        for (int s = 0; s < n_streams; s++) rs[s] = cfg->rdse_seed + (uint64_t)s * (uint64_t)cfg->seed_stride;
        HIP_TRY(hipMemcpy(e->sp.rdse_seeds, rs.data(), rs.size() * 8, hipMemcpyHostToDevice));
        if (launch_rdse_init(e->dc, e->sp, n_streams, 0)) return htm_fail(HTM_E_HIP, "rdse_init launch failed");
    }
    for (int s = 0; s < n_streams; s++) seeds[s] = cfg->tm_seed + (uint64_t)s * (uint64_t)cfg->seed_stride;
    HIP_TRY(hipMalloc(dseeds, seeds.size() * 8));
    HIP_TRY(hipMemcpy(*dseeds, seeds.data(), seeds.size() * 8, hipMemcpyHostToDevice));
    if (launch_tm_init(e->dc, e->tm, *dseeds, n_streams, 0)) return htm_fail(HTM_E_HIP, "tm_init launch failed");
    HIP_TRY(hipDeviceSynchronize());
    return HTM_OK;
}

int htm_create(const htm_config* cfg, int32_t n_streams, int32_t device, htm_engine** out) {
    int r = create_uninit(cfg, n_streams, device, out);
    if (r) return r;
    uint64_t* dseeds = nullptr;
    r = init_streams(*out, cfg, n_streams, &dseeds);
    if (dseeds) (void)hipFree(dseeds);
    if (r) {  // no half-initialised handle escapes: free everything, *out = NULL
        htm_destroy(*out);
        *out = nullptr;
    }
    return r;
}

int htm_destroy(htm_engine* e) {
    if (!e) return HTM_OK;
    (void)hipSetDevice(e->device);
    (void)hipDeviceSynchronize();
    for (void* p : e->allocs) (void)hipFree(p);
    if (e->tm.fx_ent) (void)hipFree(e->tm.fx_ent);
    if (e->sp.enc_in) (void)hipFree(e->sp.enc_in);
    for (hipEvent_t x : e->ev_pool) (void)hipEventDestroy(x);
    if (e->ev_logged) (void)hipEventDestroy(e->ev_logged);
    if (e->ev_flushed) (void)hipEventDestroy(e->ev_flushed);
    if (e->fstream) (void)hipStreamDestroy(e->fstream);
    delete e;
    return HTM_OK;
}

int htm_set_learning(htm_engine* e, int32_t sp_learn, int32_t tm_learn) {
    if (!e) return htm_fail(HTM_E_INVALID, "null engine");
    if (int r = flush_sync(e)) return r;
    if (e->fleet && (sp_learn || tm_learn))
        return htm_fail(HTM_E_STATE, "a fleet engine shares one frozen model: learning stays off");
    e->sp_learn = sp_learn ? 1 : 0;
    if (tm_learn && !e->tm_learn) e->fx_valid = false;
    e->tm_learn = tm_learn ? 1 : 0;
    return HTM_OK;
}

int htm_set_option(htm_engine* e, int32_t opt, int32_t value) {
    if (!e) return htm_fail(HTM_E_INVALID, "null engine");
    if (opt == HTM_OPT_FROZEN_INDEX) {
        // a fleet's streams share the model's segment records: only the frozen
        // index reads them race-free (the pool scan's dutyCycle() reads and
        // writes the shared records)
        if (!value && e->fleet) return htm_fail(HTM_E_INVALID, "fleet engines always run the frozen index");
        e->use_frozen = value ? 1 : 0;
    }
    else if (opt == HTM_OPT_KEEP_PREV) e->keep_prev = value ? 1 : 0;
    else if (opt == HTM_OPT_KEEP_OVERLAPS) e->keep_overlaps = value ? 1 : 0;
    else if (opt == HTM_OPT_PROFILE) {
        if (value < 0) return htm_fail(HTM_E_INVALID, "profile: 0 off, N >= 1 every N-th launch");
        e->profile = value;
        e->prof_seq = 0;
        e->ev_used = 0;
        e->ev_steps.clear();
        e->ev_fused.clear();
    }
    else if (opt == HTM_OPT_FUSED) {
        if (value && e->dc.sdr_in) return htm_fail(HTM_E_INVALID, "SDR-input engines run unfused");
        e->fused = value ? 1 : 0;
    }
    else if (opt == HTM_OPT_RUN_CHUNK) {
        if (value < 1) return htm_fail(HTM_E_INVALID, "run chunk must be >= 1");
        e->run_chunk = value;
    }
    else if (opt == HTM_OPT_DEFER_DUTY) {
        if (!value) {
            if (int r = flush_sync(e)) return r;
        }
        e->defer = value ? 1 : 0;
    }
    else if (opt == HTM_OPT_FLUSH_MODE) {
        if (value < 0 || value > 1)
            return htm_fail(HTM_E_INVALID, "flush mode must be 0 (beside the steps) or 1 (on the step stream)");
        if (int r = flush_sync(e)) return r;
        e->flush_mode = value;
    }
    else if (opt == HTM_OPT_ORDERED) e->ordered = value ? 1 : 0;
    else if (opt == HTM_OPT_SPLIT_LEARN) e->split_learn = value ? 1 : 0;
    else if (opt == HTM_OPT_FLUSH_EVERY) {
        if (value < 0) return htm_fail(HTM_E_INVALID, "flush cadence: 0 (default) or N >= 1 lockstep steps");
        if (int r = flush_sync(e)) return r;
        e->flush_every = value;
    }
    else if (opt == HTM_OPT_RUN_UNIT) {
        if (value < 0) return htm_fail(HTM_E_INVALID, "run unit must be >= 0 (0: auto)");
        e->run_unit = value;
    }
    else return htm_fail(HTM_E_INVALID, "unknown option %d", opt);
    return HTM_OK;
}

}  // extern "C"

// The frozen index's per-stream tables are allocated on first use, so an
// engine that only learns (config 3) does not pay for them.
static int alloc_fx(htm_engine* e) {
    if (e->tm.fx_off) return HTM_OK;
    const DevCfg& d = e->dc;
    const size_t M = (size_t)e->nm;
    ALLOC(e->tm.scr_cur, uint32_t, M * (size_t)d.fx_noff);
    ALLOC(e->tm.fx_off, uint32_t, M * (size_t)d.fx_noff);
    ALLOC(e->tm.fx_rec, uint2, M * (size_t)d.seg_cap);
    ALLOC(e->tm.fx_rslot, uint32_t, M * (size_t)d.seg_cap);
    ALLOC(e->tm.fx_nr, uint32_t, M);
    ALLOC(e->tm.fx_pcell, uint16_t, M * (size_t)d.fx_pcap);
    ALLOC(e->tm.fx_np, uint32_t, M);
    return HTM_OK;
}

// The deferred dutyCycle() log of lockstep steps (a ring per stream), the
// flush kernel's per-workgroup qualifying lists, and the flush stream:
// allocated on the first deferring launch, so engines that never step frozen
// in lockstep (learning, htm_run replays, HTM_OPT_DEFER_DUTY 0) do not pay.
static int alloc_dlog(htm_engine* e) {
    if (e->tm.fx_dlog) return HTM_OK;
    const DevCfg& d = e->dc;
    const size_t S = (size_t)e->n;
    ALLOC(e->tm.fx_dlen, uint16_t, S * (size_t)d.fx_dcap);
    ALLOC(e->tm.fx_dhash, uint32_t, S * (size_t)d.fx_dcap);
    ALLOC(e->tm.fx_dn, uint32_t, S);
    ALLOC(e->tm.fx_dflushed, uint32_t, S);
    ALLOC(e->tm.fx_dsnap, uint32_t, S);
    ALLOC(e->tm.fx_dupto, uint32_t, S);
    ALLOC(e->tm.fx_fq, uint32_t, (size_t)FX_FLUSH_WG * (size_t)d.q_cap);
    ALLOC(e->tm.fx_fwork, uint32_t, FX_FWORK_WORDS);
    // a split job's id is (stream * fx_dcap + slot) * (fx_nwin + 1) + window (uint32)
    if (S * (size_t)d.fx_dcap * ((size_t)d.fx_nwin + 1) >= ((size_t)1 << 32))
        return htm_fail(HTM_E_CAPACITY, "deferred-write flush: %zu streams x %d ring slots x %d windows overflow the "
                        "32-bit job ids", S, d.fx_dcap, d.fx_nwin + 1);
    ALLOC(e->tm.fx_fjobs, uint32_t, S * (size_t)d.fx_dcap * (size_t)d.fx_nwin);
    if (e->flush_prio) {
        int least = 0, greatest = 0;
        HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
        HIP_TRY(hipStreamCreateWithPriority(&e->fstream, hipStreamNonBlocking, least));
    } else {
        HIP_TRY(hipStreamCreateWithFlags(&e->fstream, hipStreamNonBlocking));
    }
    HIP_TRY(hipEventCreateWithFlags(&e->ev_logged, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&e->ev_flushed, hipEventDisableTiming));
    ALLOC(e->tm.fx_dlog, uint16_t, S * (size_t)d.fx_dcap * fx_dstride(d));  // last: the "allocated" test
    return HTM_OK;
}

// Flush of the deferred dutyCycle() writes logged by lockstep steps.
// flush_async: snapshot the log counters on the step stream `st` (the entries
// logged so far), then replay those entries on the flush stream, which waits
// for the snapshot only -- later steps run beside the flush (they append to
// the ring's free slots and never read the segment records it writes).
static int flush_async(htm_engine* e, hipStream_t st) {
    if (!e->tm.fx_dlog || !e->defer_steps) return HTM_OK;
    if (e->flush_mode == 1 || st == e->fstream) {
        // on the stream of the steps, after them: the bound is fx_dn itself
        if (launch_tm_fx_flush(e->dc, e->tm, e->n, 0, st, 1, 0))
            return htm_fail(HTM_E_HIP, "flush launch: %s", hipGetErrorString(hipGetLastError()));
        e->defer_steps = 0;
        return HTM_OK;
    }
    if (launch_tm_fx_snap(e->tm, e->n, st)) return htm_fail(HTM_E_HIP, "flush snapshot launch");
    HIP_TRY(hipEventRecord(e->ev_logged, st));
    HIP_TRY(hipStreamWaitEvent(e->fstream, e->ev_logged, 0));
    if (launch_tm_fx_flush(e->dc, e->tm, e->n, e->flush_wg, e->fstream, 0, 0))
        return htm_fail(HTM_E_HIP, "flush launch: %s", hipGetErrorString(hipGetLastError()));
    HIP_TRY(hipEventRecord(e->ev_flushed, e->fstream));
    e->defer_steps = 0;
    e->flush_pending = true;
    return HTM_OK;
}

// Flush and order `st` after it: work enqueued on `st` afterwards sees every
// record write of the steps enqueued before (stream-ordered, asynchronous).
// The flush beside the steps, if one is running, is waited for; the entries
// logged since are flushed on `st` itself, full width (nothing runs beside).
static int flush_deferred(htm_engine* e, hipStream_t st) {
    if (e->flush_pending) {
        HIP_TRY(hipStreamWaitEvent(st, e->ev_flushed, 0));
        e->flush_pending = false;
    }
    if (!e->tm.fx_dlog || !e->defer_steps) return HTM_OK;
    // (the caller waits on it: split per rank window, the latency of one window)
    if (launch_tm_fx_flush(e->dc, e->tm, e->n, 0, st, 1, e->final_split))
        return htm_fail(HTM_E_HIP, "flush launch: %s", hipGetErrorString(hipGetLastError()));
    e->defer_steps = 0;
    return HTM_OK;
}

// Host-side flush before the host reads or replaces the state: every stream
// of the device is drained first (the steps may have been issued on any
// stream, e.g. torch's current one), then the flush runs to completion.
// Complete the learning steps' pending final learn phase 2s (enqueued on st).
static int finish_lp2(htm_engine* e, hipStream_t st) {
    if (!e->lp2_pending) return HTM_OK;
    if (launch_tm_lp2_finish(e->dc, e->tm, e->nm, st)) return htm_fail(HTM_E_HIP, "lp2 finish launch");
    e->lp2_pending = false;
    return HTM_OK;
}

static int flush_sync(htm_engine* e) {
    if (e->lp2_pending) {
        HIP_TRY(hipDeviceSynchronize());
        if (int r = finish_lp2(e, nullptr)) return r;
        HIP_TRY(hipDeviceSynchronize());
    }
    if (!e->tm.fx_dlog) return HTM_OK;
    HIP_TRY(hipDeviceSynchronize());
    if (e->defer_steps) {
        if (int r = flush_async(e, e->fstream)) return r;
        HIP_TRY(hipStreamSynchronize(e->fstream));
    }
    e->flush_pending = false;
    return HTM_OK;
}

static int build_fx(htm_engine* e, hipStream_t st) {
    const DevCfg& d = e->dc;
    int ra = flush_sync(e);  // the log refers to the index being replaced
    if (!ra) ra = alloc_fx(e);
    if (ra) return ra;
    if (e->tm.fx_dlog) {
        // the logged sets were recorded against the old records and iteration:
        // an empty ring, so no later set is taken for one already written
        HIP_TRY(hipMemsetAsync(e->tm.fx_dn, 0, (size_t)e->n * 4, st));
        HIP_TRY(hipMemsetAsync(e->tm.fx_dflushed, 0, (size_t)e->n * 4, st));
        HIP_TRY(hipMemsetAsync(e->tm.fx_dsnap, 0, (size_t)e->n * 4, st));
        HIP_TRY(hipMemsetAsync(e->tm.fx_dupto, 0, (size_t)e->n * 4, st));
    }
    if (launch_tm_fx_rank(d, e->tm, e->nm, st)) return htm_fail(HTM_E_HIP, "fx rank launch");
    if (launch_tm_fx_count(d, e->tm, e->d_counts, e->nm, st)) return htm_fail(HTM_E_HIP, "fx count launch");
    std::vector<uint64_t> counts((size_t)e->nm);
    HIP_TRY(hipMemcpyAsync(counts.data(), e->d_counts, counts.size() * 8, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    std::vector<uint64_t> base((size_t)e->nm);
    uint64_t tot = 0;
    for (int s = 0; s < e->nm; s++) {
        base[s] = tot;
        tot += counts[s];
    }
    if (tot == 0) tot = 1;
    if (tot > e->fx_cap) {  // capacity in 16-byte blocks
        if (e->tm.fx_ent) HIP_TRY(hipFree(e->tm.fx_ent));
        e->tm.fx_ent = nullptr;
        size_t cap = (size_t)(tot + tot / 8 + 1024);
        HIP_TRY(hipMalloc(&e->tm.fx_ent, cap * 16));
        e->fx_cap = cap;
    }
    HIP_TRY(hipMemsetAsync(e->tm.fx_ent, 0xFF, (size_t)tot * 16, st));
    HIP_TRY(hipMemcpyAsync(e->tm.fx_base, base.data(), base.size() * 8, hipMemcpyHostToDevice, st));
    if (launch_tm_fx_fill(d, e->tm, e->nm, st)) return htm_fail(HTM_E_HIP, "fx fill launch");
    HIP_TRY(hipStreamSynchronize(st));
    e->fx_valid = true;
    return HTM_OK;
}

extern "C" {

// HTM_OPT_PROFILE N: the events bracket every N-th launch (a timed event
// record between two dependent launches holds the queue ~12 us -- measured in
// a 20-step lockstep trace, profiles/r04_b -- so sampling keeps the timed
// region close to the unprofiled one; the average is over the sampled launches)
static bool profiled_launch(htm_engine* e) {
    if (!e->profile) return false;
    return e->prof_seq++ % (uint32_t)e->profile == 0;
}

static int next_events(htm_engine* e, hipEvent_t* ev, int32_t steps) {
    // three events per profiled step: before SP, between SP and TM, after TM
    while (e->ev_pool.size() < e->ev_used + 3) {
        hipEvent_t x;
        HIP_TRY(hipEventCreate(&x));
        e->ev_pool.push_back(x);
    }
    for (int k = 0; k < 3; k++) ev[k] = e->ev_pool[e->ev_used + k];
    e->ev_used += 3;
    e->ev_steps.push_back(steps);
    e->ev_fused.push_back(0);
    return HTM_OK;
}

// Mode of the next steps: the TM kernel variant follows the learning flags;
// with TM learning off the frozen forward index is (re)built first.
static int prepare_step(htm_engine* e, hipStream_t st, int* frozen) {
    *frozen = 0;
    // a step without TM learning completes what the last learning step deferred
    if (!e->tm_learn && e->lp2_pending) {
        int r = finish_lp2(e, st);
        if (r) return r;
    }
    if (e->tm_learn && e->dc.lp2_defer) e->lp2_pending = true;
    if (e->tm_learn || !e->use_frozen) {
        // the pool scans read the segments' dutyCycle records
        int r = flush_deferred(e, st);
        if (r) return r;
    }
    if (e->tm_learn) {
        e->fx_valid = false;
    } else if (e->use_frozen) {
        if (!e->fx_valid) {
            int r = build_fx(e, st);
            if (r) return r;
        }
        *frozen = 1;
    }
    return HTM_OK;
}

// RDSE engines: the encoder kernel runs the streams' encoders through the
// launch's n_steps records first.  Their lists (count + n_fields * enc_w bits,
// DevCfg::enc_list words per stream-step) are allocated at creation for one
// step (a lockstep engine never needs more; a 131,072-stream model.yaml fleet
// would hold 1.6 GB for run_chunk steps); the first longer launch grows the
// buffer (synchronising) to its length.
static int grow_enc(htm_engine* e, size_t steps, hipStream_t st) {
    if (e->dc.enc_type != HTM_ENC_RDSE || steps <= e->enc_cap) return HTM_OK;
    const size_t per = (size_t)e->n * e->dc.enc_list * 2;
    if (e->sp.enc_in) {
        HIP_TRY(hipStreamSynchronize(st));
        HIP_TRY(hipFree(e->sp.enc_in));
        e->bytes -= e->enc_cap * per;
        e->sp.enc_in = nullptr;
        e->enc_cap = 0;
    }
    HIP_TRY(hipMalloc(&e->sp.enc_in, steps * per));
    e->enc_cap = steps;
    e->bytes += e->enc_cap * per;
    return HTM_OK;
}

static int encode_rdse(htm_engine* e, const double* d_values, int32_t n_steps, hipStream_t st) {
    if (e->dc.enc_type != HTM_ENC_RDSE) return HTM_OK;
    if (int r = grow_enc(e, (size_t)n_steps, st)) return r;
    if (launch_rdse_encode(e->dc, e->sp, d_values, n_steps, e->n, st)) return htm_fail(HTM_E_HIP, "rdse encode launch");
    return HTM_OK;
}

// n_steps network.run(1) of every stream in one fused SP+TM launch.
static int run_fused(htm_engine* e, int32_t n_steps, const double* d_values, float* d_scores, hipStream_t st,
                     int frozen) {
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    const bool prof = profiled_launch(e);
    // ordered lockstep step (HTM_OPT_ORDERED; frozen, one step, dense SP, at
    // most 16,384 streams): the SP kernel, the cost-ordered stream list, then
    // the fused kernel's TM steps in that order
    const bool ordered = frozen && n_steps == 1 && !e->tm_learn && e->ordered && !e->dc.sp_paged && e->n <= ORD_MAX_STREAMS;
    // split learning step (HTM_OPT_SPLIT_LEARN; TM learning on, one step): the
    // SP kernel (its learning, paged rows included, at the SP kernel's own
    // occupancy), then the TM-only learning kernel (the SP compiled out)
    const bool split = e->tm_learn && n_steps == 1 && e->split_learn && !e->dc.sdr_in;
    if (prof) {
        int r = next_events(e, ev, n_steps);
        if (r) return r;
        // one event before and one after the fused kernel (an event record is
        // a few microseconds of the queue's time: no empty "SP" interval);
        // ordered: around the TM launch only (its SP kernel and sort untimed);
        // split learning: the SP kernel and the TM kernel each
        e->ev_fused.back() = split ? 0 : 1;
        if (split) HIP_TRY(hipEventRecord(ev[0], st));
        else if (!ordered) HIP_TRY(hipEventRecord(ev[1], st));
    }
    // auto unit: a stream keeps its TM state in LDS for a unit's steps; longer
    // units save state round trips and queue handoffs, shorter ones balance
    // the launch's tail (measured on config 2, profiles/r01_s4/ab_unit.txt:
    // 256-step launches best at 32, 2324-step launches flat over 48..96)
    const int32_t unit = e->run_unit > 0 ? e->run_unit : std::max(16, std::min(64, n_steps / 8));
    if (int r = encode_rdse(e, d_values, n_steps, st)) return r;
    // deferred dutyCycle() writes: frozen lockstep launches (one step)
    const bool defer = frozen && n_steps == 1 && e->defer;
    const int32_t cadence = e->flush_every ? e->flush_every : std::min(FLUSH_EVERY, e->dc.fx_dcap / 2);
    TmBufs tb = e->tm;
    if (defer) {
        if (int r = alloc_dlog(e)) return r;
        tb = e->tm;
    } else {
        tb.fx_dlog = nullptr;
    }
    if (ordered) {
        if (!e->ord) {
            ALLOC(e->ord, uint32_t, e->n);
            ALLOC(e->ord_est, uint16_t, e->n);
        }
        if (launch_sp_step_ord(e->dc, e->sp, d_values, e->sp_learn, e->n, e->keep_overlaps, e->tm.bm, e->ord_est, st))
            return htm_fail(HTM_E_HIP, "sp_step launch");
        tb.ord = e->ord;
        tb.tm_only = 1;
        if (launch_ord_sort(e->dc, e->ord_est, e->ord, e->n, st))
            return htm_fail(HTM_E_HIP, "ord_sort launch");
#ifndef HTM_FLUSH_AFTER_STEP
        // a due flush of the deferred log starts here, after this step's SP
        // kernel and sort: its workgroups and the TM launch's become ready
        // together and the flush stream's low priority dispatches the launch's
        // first (issued after the previous step's launch, the flush took the
        // CUs during this SP kernel and sort and delayed the whole launch)
        if (defer && e->defer_steps >= cadence)
            if (int r = flush_async(e, st)) return r;
#endif
        if (prof) HIP_TRY(hipEventRecord(ev[1], st));  // (the 256-thread TM launch's start)
    } else if (split) {
        if (launch_sp_step_ord(e->dc, e->sp, d_values, e->sp_learn, e->n, e->keep_overlaps, nullptr, nullptr, st))
            return htm_fail(HTM_E_HIP, "sp_step launch");
        if (prof) HIP_TRY(hipEventRecord(ev[1], st));
        tb.tm_only = 1;
    }
#ifdef HTM_AB_KNOBS
    // A/B builds: every workgroup's start / end time of the latest lockstep launch
    if (ab_knob("HTM_WG_TRACE") && n_steps == 1) {
        if (!e->wg_trace) {
            e->wg_trace_cap = (size_t)e->n;
            HIP_TRY(hipMalloc(&e->wg_trace, e->wg_trace_cap * 64));
            e->allocs.push_back(e->wg_trace);
        }
        HIP_TRY(hipMemsetAsync(e->wg_trace, 0, e->wg_trace_cap * 64, st));
        tb.wg_trace = e->wg_trace;
    }
#endif
    if (launch_htm_run(e->dc, tb, e->sp, d_values, d_scores, n_steps, e->sp_learn, e->tm_learn, frozen,
                       e->keep_prev, e->keep_overlaps, e->n, e->wq, unit, st))
        return htm_fail(HTM_E_HIP, "htm_run launch: %s", hipGetErrorString(hipGetLastError()));
    e->conf_packed = true;
    if (prof) HIP_TRY(hipEventRecord(ev[2], st));  // (the step kernel only: a flush is its own kernel)
    // (an explicit cadence, HTM_OPT_FLUSH_EVERY, is taken as given: past the ring the log fills)
    if (defer && ++e->defer_steps >= cadence) {
#ifndef HTM_FLUSH_AFTER_STEP
        if (ordered) return HTM_OK;  // (the next ordered step starts it before its TM launch)
#endif
        int r = flush_async(e, st);  // beside the next steps
        if (r) return r;
    }
    return HTM_OK;
}

// One unfused step: the SP kernel (encoder values or input SDR), then the TM kernel.
static int step_unfused(htm_engine* e, const double* d_values, const uint32_t* d_sdr, float* d_scores,
                        hipStream_t st, int frozen) {
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    int r;
    const bool prof = profiled_launch(e);
    if (prof) {
        r = next_events(e, ev, 1);
        if (r) return r;
        HIP_TRY(hipEventRecord(ev[0], st));
    }
    if (!d_sdr && encode_rdse(e, d_values, 1, st)) return HTM_E_HIP;
    if (d_sdr ? launch_sp_step_sdr(e->dc, e->sp, d_sdr, e->sp_learn, e->n, e->keep_overlaps, st)
              : launch_sp_step(e->dc, e->sp, d_values, e->sp_learn, e->n, e->keep_overlaps, st))
        return htm_fail(HTM_E_HIP, "sp_step launch");
    if (e->keep_prev) {
        // prevPredictedColumns (nonzero colConfidence before compute)
        if (launch_prev_pred(e->dc, e->tm, e->n, st)) return htm_fail(HTM_E_HIP, "prev_pred launch");
    }
    if (prof) HIP_TRY(hipEventRecord(ev[1], st));
    TmBufs tb = e->tm;
    tb.fx_dlog = nullptr;  // (deferred duty writes: fused lockstep launches only)
    if (launch_tm_step(e->dc, tb, e->sp, d_scores, e->tm_learn, frozen, e->n, st))
        return htm_fail(HTM_E_HIP, "tm_step launch: %s", hipGetErrorString(hipGetLastError()));
    e->conf_packed = true;
    if (prof) HIP_TRY(hipEventRecord(ev[2], st));
    return HTM_OK;
}

int htm_step(htm_engine* e, const double* d_values, float* d_scores, void* stream) {
    if (!e || !d_values || !d_scores) return htm_fail(HTM_E_INVALID, "bad arguments");
    if (e->dc.sdr_in) return htm_fail(HTM_E_INVALID, "this engine reads an input SDR: use htm_step_sdr");
    hipStream_t st = (hipStream_t)stream;
    int frozen = 0;
    int r = prepare_step(e, st, &frozen);
    if (r) return r;
    if (e->fused) return run_fused(e, 1, d_values, d_scores, st, frozen);
    return step_unfused(e, d_values, nullptr, d_scores, st, frozen);
}

int htm_step_sdr(htm_engine* e, const uint32_t* d_sdr, float* d_scores, void* stream) {
    if (!e || !d_sdr || !d_scores) return htm_fail(HTM_E_INVALID, "bad arguments");
    if (!e->dc.sdr_in) return htm_fail(HTM_E_INVALID, "this engine reads encoder values: use htm_step");
    hipStream_t st = (hipStream_t)stream;
    int frozen = 0;
    int r = prepare_step(e, st, &frozen);
    if (r) return r;
    return step_unfused(e, nullptr, d_sdr, d_scores, st, frozen);
}

int htm_run_sdr(htm_engine* e, int32_t n_steps, const uint32_t* d_sdr, float* d_scores, void* stream) {
    if (!e) return htm_fail(HTM_E_INVALID, "null engine");
    if (n_steps < 0 || (n_steps > 0 && (!d_sdr || !d_scores))) return htm_fail(HTM_E_INVALID, "bad arguments");
    const size_t stride = (size_t)e->n * (e->dc.nin_pad / 32);
    for (int32_t k = 0; k < n_steps; k++) {
        int r = htm_step_sdr(e, d_sdr + (size_t)k * stride, d_scores + (size_t)k * e->n, stream);
        if (r) return r;
    }
    return HTM_OK;
}

// Kernel times of the profiled steps since the last read:
// out4 = {SP kernel ms, TM kernel ms, steps, 0}
int htm_profile_read(htm_engine* e, double* out4) {
    if (!e || !out4) return htm_fail(HTM_E_INVALID, "bad arguments");
    HIP_TRY(hipDeviceSynchronize());
    double sp = 0.0, tm = 0.0;
    for (size_t k = 0; k + 2 < e->ev_used + 1 && k < e->ev_used; k += 3) {
        float a = 0.f, b = 0.f;
        if (!e->ev_fused[k / 3]) HIP_TRY(hipEventElapsedTime(&a, e->ev_pool[k], e->ev_pool[k + 1]));
        HIP_TRY(hipEventElapsedTime(&b, e->ev_pool[k + 1], e->ev_pool[k + 2]));
        sp += a;
        tm += b;
    }
    double steps = 0.0;
    for (int32_t x : e->ev_steps) steps += x;
    out4[0] = sp;
    out4[1] = tm;
    out4[2] = steps;
    out4[3] = (double)(e->ev_used / 3);
    e->ev_used = 0;
    e->ev_steps.clear();
    e->ev_fused.clear();
    return HTM_OK;
}

// error flags of the deferred-duty flushes (host; the device is idle)
static uint32_t flush_error(htm_engine* e) {
    uint32_t x = 0;
    if (e->tm.fx_fwork && hipMemcpy(&x, e->tm.fx_fwork + 1, 4, hipMemcpyDeviceToHost) != hipSuccess) x = 0;
    return x;
}

// Sum of the per-stream TM counters: out8 = {algorithmic bytes, inferPhase2
// calls, inferBacktracks, learnPhase2 calls, learnBacktracks, live segments,
// pool high-water marks, OR of error flags}
int htm_counters(htm_engine* e, uint64_t* out8) {
    if (!e || !out8) return htm_fail(HTM_E_INVALID, "bad arguments");
    if (int r = flush_sync(e)) return r;
    HIP_TRY(hipDeviceSynchronize());
    std::vector<htm_tm_header> h((size_t)e->n);
    HIP_TRY(hipMemcpy(h.data(), e->tm.hdr, h.size() * sizeof(htm_tm_header), hipMemcpyDeviceToHost));
    for (int k = 0; k < 8; k++) out8[k] = 0;
    std::vector<uint32_t> spe((size_t)e->n);
    HIP_TRY(hipMemcpy(spe.data(), e->sp.err, spe.size() * 4, hipMemcpyDeviceToHost));
    for (uint32_t x : spe) out8[7] |= x;
    out8[7] |= flush_error(e);
    for (const auto& x : h) {
        out8[0] += x.stat_bytes;
        out8[1] += x.stat_inf_phase2;
        out8[2] += x.stat_inf_backtrack;
        out8[3] += x.stat_lrn_phase2;
        out8[4] += x.stat_lrn_backtrack;
        out8[5] += x.seg_live;
        out8[6] += x.seg_hwm;
        out8[7] |= x.error;
    }
    return HTM_OK;
}

// count slots of the SP paged-row replays (tm_core.h SC_REPLAY, SC_REPLAYCYC)
#define SC_REPLAY_IDX 18

int htm_debug_stamps(htm_engine* e, uint64_t* out128) {
    if (!e || !out128) return htm_fail(HTM_E_INVALID, "bad arguments");
    if (!e->tm.dbg) return htm_fail(HTM_E_STATE, "not a stamps build (HTM_STAMPS)");
    HIP_TRY(hipDeviceSynchronize());
    const int W = 4 * HTM_NSTAMP;
    std::vector<uint64_t> h((size_t)e->n * W), r((size_t)e->n * 4);
    HIP_TRY(hipMemcpy(h.data(), e->tm.dbg, h.size() * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(r.data(), e->sp.dbg, r.size() * 8, hipMemcpyDeviceToHost));
    for (int k = 0; k < W; k++) out128[k] = 0;
    for (int s = 0; s < e->n; s++) {
        for (int k = 0; k < W; k++) out128[k] += h[(size_t)s * W + k];
        // SP paged-row replays (not attributable to tail steps)
        for (int k = 0; k < 4; k++) out128[HTM_NSTAMP + SC_REPLAY_IDX + k] += r[(size_t)s * 4 + k];
    }
    HIP_TRY(hipMemset(e->tm.dbg, 0, h.size() * 8));
    HIP_TRY(hipMemset(e->sp.dbg, 0, r.size() * 8));
    return HTM_OK;
}

int htm_run(htm_engine* e, int32_t n_steps, const double* d_values, float* d_scores, void* stream) {
    if (!e) return htm_fail(HTM_E_INVALID, "null engine");
    if (e->dc.sdr_in) return htm_fail(HTM_E_INVALID, "this engine reads an input SDR: use htm_run_sdr");
    if (n_steps < 0 || (n_steps > 0 && (!d_values || !d_scores))) return htm_fail(HTM_E_INVALID, "bad arguments");
    const size_t stride = (size_t)e->n * e->cfg.n_fields;
    if (e->fused) {
        hipStream_t st = (hipStream_t)stream;
        int frozen = 0;
        int r = prepare_step(e, st, &frozen);
        if (r) return r;
        for (int32_t k = 0; k < n_steps; k += e->run_chunk) {
            const int32_t m = n_steps - k < e->run_chunk ? n_steps - k : e->run_chunk;
            r = run_fused(e, m, d_values + (size_t)k * stride, d_scores + (size_t)k * e->n, st, frozen);
            if (r) return r;
        }
        return HTM_OK;
    }
    for (int32_t k = 0; k < n_steps; k++) {
        int r = htm_step(e, d_values + (size_t)k * stride, d_scores + (size_t)k * e->n, stream);
        if (r) return r;
    }
    return HTM_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// outputs
__global__ void out_kernel(DevCfg c, SpBufs sp, TmBufs tm, int which, uint8_t* dst) {
    const int s = blockIdx.x;
    if (which == HTM_OUT_ACTIVE_COLUMNS) {
        uint8_t* o = dst + (size_t)s * c.ncol;
        for (int i = threadIdx.x; i < c.ncol; i += blockDim.x) o[i] = 0;
        __syncthreads();
        uint32_t n = sp.nact[s];
        for (uint32_t i = threadIdx.x; i < n && i < HTM_MAXACT; i += blockDim.x) o[sp.act[(size_t)s * HTM_MAXACT + i]] = 1;
    } else if (which == HTM_OUT_PREV_PRED_COLS) {
        uint8_t* o = dst + (size_t)s * c.ncol;
        for (int i = threadIdx.x; i < c.ncol; i += blockDim.x) o[i] = tm.prev_pred[(size_t)s * c.ncol + i];
    } else if (which == HTM_OUT_TM_OUTPUT) {
        uint32_t* o = reinterpret_cast<uint32_t*>(dst) + (size_t)s * c.cw;
        const uint32_t* bm = tm.bm + (size_t)s * 4 * c.cw;
        for (int i = threadIdx.x; i < c.cw; i += blockDim.x) o[i] = bm[i] | bm[c.cw + i];
    } else if (which == HTM_OUT_PRED_COLS) {
        uint8_t* o = dst + (size_t)s * c.ncol;
        const uint32_t* nz = tm.colnz + (size_t)s * (c.nw + 1);
        const bool packed = nz[c.nw] == 1u;  // the bitmap is current (else the dense copy is)
        for (int i = threadIdx.x; i < c.ncol; i += blockDim.x)
            o[i] = packed ? (uint8_t)((nz[i >> 5] >> (i & 31)) & 1u) : (tm.colconf[(size_t)s * c.ncol + i] != 0.0f ? 1 : 0);
    }
}

__global__ void prev_pred_kernel(DevCfg c, TmBufs tm) {
    const int s = blockIdx.x;
    const uint32_t* nz = tm.colnz + (size_t)s * (c.nw + 1);
    const bool packed = nz[c.nw] == 1u;  // the bitmap is current (else the dense copy is)
    for (int i = threadIdx.x; i < c.ncol; i += blockDim.x)
        tm.prev_pred[(size_t)s * c.ncol + i] =
            packed ? (uint8_t)((nz[i >> 5] >> (i & 31)) & 1u) : (tm.colconf[(size_t)s * c.ncol + i] != 0.0f ? 1 : 0);
}

int launch_prev_pred(const DevCfg& c, const TmBufs& b, int n, hipStream_t st) {
    hipLaunchKernelGGL(prev_pred_kernel, dim3(n), dim3(256), 0, st, c, b);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" {

size_t htm_output_bytes(const htm_engine* e, int32_t which) {
    if (!e) return 0;
    const DevCfg& d = e->dc;
    switch (which) {
        case HTM_OUT_ACTIVE_COLUMNS:
        case HTM_OUT_PREV_PRED_COLS:
        case HTM_OUT_PRED_COLS: return (size_t)d.ncol;
        case HTM_OUT_INF_ACTIVE:
        case HTM_OUT_INF_PREDICTED:
        case HTM_OUT_LRN_ACTIVE:
        case HTM_OUT_LRN_PREDICTED:
        case HTM_OUT_TM_OUTPUT: return (size_t)d.cw * 4;
        case HTM_OUT_COL_CONFIDENCE: return (size_t)d.ncol * 4;
        case HTM_OUT_SP_OVERLAPS: return (size_t)d.ncol * 4;
        case HTM_OUT_BUCKETS: return 16;
        default: return 0;
    }
}

int htm_get_output(htm_engine* e, int32_t which, void* d_dst, size_t bytes, void* stream) {
    if (!e || !d_dst) return htm_fail(HTM_E_INVALID, "bad arguments");
    size_t per = htm_output_bytes(e, which);
    if (!per) return htm_fail(HTM_E_INVALID, "unknown output %d", which);
    if (bytes < per * e->n) return htm_fail(HTM_E_INVALID, "output buffer too small (%zu < %zu)", bytes, per * e->n);
    hipStream_t st = (hipStream_t)stream;
    const DevCfg& d = e->dc;
    switch (which) {
        case HTM_OUT_ACTIVE_COLUMNS:
        case HTM_OUT_PREV_PRED_COLS:
        case HTM_OUT_TM_OUTPUT:
        case HTM_OUT_PRED_COLS:
            if (which == HTM_OUT_PREV_PRED_COLS && !e->keep_prev)
                return htm_fail(HTM_E_STATE, "prev-predicted columns need htm_set_option(KEEP_PREV)");
            hipLaunchKernelGGL(out_kernel, dim3(e->n), dim3(256), 0, st, d, e->sp, e->tm, which, (uint8_t*)d_dst);
            HIP_TRY(hipGetLastError());
            return HTM_OK;
        case HTM_OUT_INF_ACTIVE:
        case HTM_OUT_INF_PREDICTED:
        case HTM_OUT_LRN_ACTIVE:
        case HTM_OUT_LRN_PREDICTED: {
            int k = which - HTM_OUT_INF_ACTIVE;
            HIP_TRY(hipMemcpy2DAsync(d_dst, per, e->tm.bm + (size_t)k * d.cw, (size_t)4 * d.cw * 4, per, e->n,
                                     hipMemcpyDeviceToDevice, st));
            return HTM_OK;
        }
        case HTM_OUT_COL_CONFIDENCE:
            if (int r = densify_conf(e, st)) return r;
            HIP_TRY(hipMemcpyAsync(d_dst, e->tm.colconf, per * e->n, hipMemcpyDeviceToDevice, st));
            return HTM_OK;
        case HTM_OUT_SP_OVERLAPS:
            if (!e->keep_overlaps) return htm_fail(HTM_E_STATE, "SP overlaps need htm_set_option(KEEP_OVERLAPS)");
            HIP_TRY(hipMemcpyAsync(d_dst, e->sp.overlaps, per * e->n, hipMemcpyDeviceToDevice, st));
            return HTM_OK;
        case HTM_OUT_BUCKETS:
            if (d.sdr_in) return htm_fail(HTM_E_STATE, "an SDR-input engine has no encoder");
            HIP_TRY(hipMemcpyAsync(d_dst, e->sp.enc_bucket, per * e->n, hipMemcpyDeviceToDevice, st));
            return HTM_OK;
    }
    return htm_fail(HTM_E_INVALID, "unknown output");
}

size_t htm_state_bytes(const htm_engine* e, int32_t region) {
    if (!e || region < 1 || region > HTM_ST_COUNT) return 0;
    return e->regions[region].per_stream;
}

// instances of a region: streams, or (model regions of a fleet) the one shared model
static int32_t region_count(const htm_engine* e, int32_t region) {
    return e->regions[region].model ? e->nm : e->n;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Paged SP permanences <-> the dense HTM_ST_SP_PERM layout, a chunk of
// streams at a time through a device staging buffer (<= 256 MiB).
static size_t paged_chunk(const htm_engine* e) {
    const size_t per = e->regions[HTM_ST_SP_PERM].per_stream;
    return std::max<size_t>(1, ((size_t)256 << 20) / per);
}

// streams [s0, s0+n) into h_dst (host) or d_dst (device), dense
static int paged_perm_export(htm_engine* e, int32_t s0, int32_t n, void* h_dst, float* d_dst) {
    const size_t per = e->regions[HTM_ST_SP_PERM].per_stream;
    if (d_dst) {
        if (launch_sp_perm_export(e->dc, e->sp, d_dst, s0, n, nullptr)) return htm_fail(HTM_E_HIP, "perm export launch");
        HIP_TRY(hipDeviceSynchronize());
        return HTM_OK;
    }
    const int32_t chunk = (int32_t)std::min<size_t>((size_t)n, paged_chunk(e));
    float* tmp = nullptr;
    HIP_TRY(hipMalloc(&tmp, per * chunk));
    int rc = HTM_OK;
    for (int32_t k = 0; k < n && !rc; k += chunk) {
        const int32_t m = std::min(chunk, n - k);
        if (launch_sp_perm_export(e->dc, e->sp, tmp, s0 + k, m, nullptr)) rc = htm_fail(HTM_E_HIP, "perm export launch");
        else if (hipMemcpy((uint8_t*)h_dst + per * k, tmp, per * m, hipMemcpyDeviceToHost) != hipSuccess)
            rc = htm_fail(HTM_E_HIP, "perm export copy: %s", hipGetErrorString(hipGetLastError()));
    }
    (void)hipFree(tmp);
    return rc;
}

// dense rows from h_src (host) or d_src (device, d_stride floats between
// streams: 0 = the same row set for every stream) into streams [s0, s0+n)
static int paged_perm_import(htm_engine* e, int32_t s0, int32_t n, const void* h_src, const float* d_src,
                             size_t d_stride) {
    const size_t per = e->regions[HTM_ST_SP_PERM].per_stream;
    if (d_src) {
        if (launch_sp_perm_import(e->dc, e->sp, d_src, d_stride, s0, n, nullptr)) return htm_fail(HTM_E_HIP, "perm import launch");
        HIP_TRY(hipDeviceSynchronize());
        return HTM_OK;
    }
    const int32_t chunk = (int32_t)std::min<size_t>((size_t)n, paged_chunk(e));
    float* tmp = nullptr;
    HIP_TRY(hipMalloc(&tmp, per * chunk));
    int rc = HTM_OK;
    for (int32_t k = 0; k < n && !rc; k += chunk) {
        const int32_t m = std::min(chunk, n - k);
        if (hipMemcpy(tmp, (const uint8_t*)h_src + per * k, per * m, hipMemcpyHostToDevice) != hipSuccess)
            rc = htm_fail(HTM_E_HIP, "perm import copy: %s", hipGetErrorString(hipGetLastError()));
        else if (launch_sp_perm_import(e->dc, e->sp, tmp, per / 4, s0 + k, m, nullptr) ||
                 hipDeviceSynchronize() != hipSuccess)
            rc = htm_fail(HTM_E_HIP, "perm import launch");
    }
    (void)hipFree(tmp);
    return rc;
}

// New checkpoints or potential masks (what the initial values of columns
// without a row are replayed from) for streams [s0, s0+n): their permanences
// keep their values -- exported against the old initial values, re-imported
// against the new.
static int paged_rebase_import(htm_engine* e, int32_t region, int32_t s0, int32_t n, const void* h_src) {
    const size_t per = e->regions[HTM_ST_SP_PERM].per_stream;
    const size_t cper = e->regions[region].per_stream;
    uint8_t* base = (uint8_t*)e->regions[region].base;
    const int32_t chunk = (int32_t)std::min<size_t>((size_t)n, paged_chunk(e));
    float* tmp = nullptr;
    HIP_TRY(hipMalloc(&tmp, per * chunk));
    int rc = HTM_OK;
    for (int32_t k = 0; k < n && !rc; k += chunk) {
        const int32_t m = std::min(chunk, n - k);
        rc = paged_perm_export(e, s0 + k, m, nullptr, tmp);
        if (!rc && hipMemcpy(base + cper * (s0 + k), (const uint8_t*)h_src + cper * k, cper * m,
                             hipMemcpyHostToDevice) != hipSuccess)
            rc = htm_fail(HTM_E_HIP, "region %d import copy", region);
        if (!rc) rc = paged_perm_import(e, s0 + k, m, nullptr, tmp, per / 4);
    }
    (void)hipFree(tmp);
    return rc;
}

extern "C" {

int htm_export_state(htm_engine* e, int32_t region, int32_t s0, int32_t n, void* h_dst, size_t bytes) {
    if (!e || region < 1 || region > HTM_ST_COUNT || s0 < 0 || n < 1 || s0 + n > region_count(e, region))
        return htm_fail(HTM_E_INVALID, "bad export arguments");
    const Region& r = e->regions[region];
    if (bytes < r.per_stream * n) return htm_fail(HTM_E_INVALID, "export buffer too small");
    if (int rf = flush_sync(e)) return rf;
    if (int rd = densify_conf(e, nullptr)) return rd;
    HIP_TRY(hipDeviceSynchronize());
    if (r.per_stream == 0) return HTM_OK;
    if (region == HTM_ST_SP_PERM && e->dc.sp_paged) return paged_perm_export(e, s0, n, h_dst, nullptr);
    HIP_TRY(hipMemcpy(h_dst, (uint8_t*)r.base + r.per_stream * s0, r.per_stream * n, hipMemcpyDeviceToHost));
    return HTM_OK;
}

// The kernels write colConfidence back packed (TmBufs::colnz bitmap +
// colval values); the dense per-stream copy (HTM_ST_TM_COLCONF, colconf) is
// rebuilt from it before the host reads or replaces any state: one workgroup
// per stream whose packed form is current.
__global__ void conf_densify_kernel(DevCfg c, TmBufs b) {
    const int s = blockIdx.x;
    const uint32_t* nz = b.colnz + (size_t)s * (c.nw + 1);
    if (nz[c.nw] != 1u) return;  // the dense copy is current
    __shared__ uint32_t woff[HTM_MAXNW];
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (int w = 0; w < c.nw; w++) {
            woff[w] = run;
            run += (uint32_t)__popc(nz[w]);
        }
    }
    __syncthreads();
    const float* v = b.colval + (size_t)s * c.ncol;
    float* d = b.colconf + (size_t)s * c.ncol;
    for (int col = threadIdx.x; col < c.ncol; col += blockDim.x) {
        const uint32_t w = nz[col >> 5];
        d[col] = ((w >> (col & 31)) & 1u) ? v[woff[col >> 5] + __popc(w & ((1u << (col & 31)) - 1u))] : 0.0f;
    }
}

static int densify_conf(htm_engine* e, hipStream_t st) {
    if (!e->conf_packed) return HTM_OK;
    hipLaunchKernelGGL(conf_densify_kernel, dim3(e->n), dim3(256), 0, st, e->dc, e->tm);
    HIP_TRY(hipGetLastError());
    e->conf_packed = false;
    return HTM_OK;
}

// Any host-side change of the TM state: the dense colConfidence becomes the
// current copy (densified first) and the packed form is marked stale, so the
// next step starts from the dense copy and writes back in full.
static int invalidate_colnz(htm_engine* e, void* stream) {
    if (int r = densify_conf(e, (hipStream_t)stream)) return r;
    const size_t bytes = (size_t)e->n * ((size_t)e->dc.nw + 1) * 4;
    if (hipMemsetAsync(e->tm.colnz, 0, bytes, (hipStream_t)stream) != hipSuccess)
        return htm_fail(HTM_E_HIP, "colnz reset: %s", hipGetErrorString(hipGetLastError()));
    return HTM_OK;
}

// rebase = false: plain copies of the checkpoints / potential masks (htm_load,
// whose fresh engine holds no permanences yet)
static int import_region(htm_engine* e, int32_t region, int32_t s0, int32_t n, const void* h_src, size_t bytes,
                         bool rebase) {
    if (!e || region < 1 || region > HTM_ST_COUNT || s0 < 0 || n < 1 || s0 + n > region_count(e, region))
        return htm_fail(HTM_E_INVALID, "bad import arguments");
    const Region& r = e->regions[region];
    // no checkpoints (an export of a dense engine): the streams keep their own
    if (region == HTM_ST_SP_PERM_CKPT && (bytes == 0 || r.per_stream == 0)) return HTM_OK;
    if (bytes < r.per_stream * n) return htm_fail(HTM_E_INVALID, "import buffer too small");
    if (r.per_stream == 0) return HTM_OK;  // (a region this engine does not have, e.g. RDSE state)
    if (int rf = flush_sync(e)) return rf;
    if (int rd = densify_conf(e, nullptr)) return rd;  // (before the dense copy may be overwritten)
    HIP_TRY(hipDeviceSynchronize());
    if (region == HTM_ST_SP_PERM && e->dc.sp_paged) return paged_perm_import(e, s0, n, h_src, nullptr, 0);
    if (rebase && e->dc.sp_paged && (region == HTM_ST_SP_PERM_CKPT || region == HTM_ST_SP_POTMASK))
        return paged_rebase_import(e, region, s0, n, h_src);
    HIP_TRY(hipMemcpy((uint8_t*)r.base + r.per_stream * s0, h_src, r.per_stream * n, hipMemcpyHostToDevice));
    if (region >= HTM_ST_TM_HEADER && region <= HTM_ST_TM_UPDATES) e->fx_valid = false;
    return invalidate_colnz(e, nullptr);
}

int htm_import_state(htm_engine* e, int32_t region, int32_t s0, int32_t n, const void* h_src, size_t bytes) {
    return import_region(e, region, s0, n, h_src, bytes, true);
}

int htm_reset_tm(htm_engine* e, void* stream) {
    if (!e) return htm_fail(HTM_E_INVALID, "null engine");
    if (int r = finish_lp2(e, (hipStream_t)stream)) return r;  // (the deferred phase precedes the reset)
    if (launch_tm_reset(e->dc, e->tm, e->n, (hipStream_t)stream)) return htm_fail(HTM_E_HIP, "reset launch");
    return invalidate_colnz(e, stream);
}

// Broadcast one stream's slice of a per-stream region into every other
// stream: a grid-stride copy in 16-byte (or 4-byte / 1-byte) units.
__global__ void replicate_kernel(uint8_t* base, size_t per, int32_t src, int32_t n, int unit) {
    const size_t m = per / (size_t)unit;  // units per stream
    const size_t total = m * (size_t)n;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const size_t s = i / m, k = i - s * m;
        if ((int32_t)s == src) continue;
        if (unit == 16)
            reinterpret_cast<uint4*>(base + per * s)[k] = reinterpret_cast<const uint4*>(base + per * src)[k];
        else if (unit == 4)
            reinterpret_cast<uint32_t*>(base + per * s)[k] = reinterpret_cast<const uint32_t*>(base + per * src)[k];
        else
            base[per * s + k] = base[per * src + k];
    }
}

static int replicate_region(uint8_t* base, size_t per, int32_t src, int32_t n, hipStream_t st) {
    const int unit = (per % 16 == 0 && ((uintptr_t)base % 16) == 0) ? 16 : (per % 4 == 0 ? 4 : 1);
    const size_t total = per / unit * (size_t)n;
    size_t blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(replicate_kernel, dim3((unsigned)blocks), dim3(256), 0, st, base, per, src, n, unit);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int htm_replicate_stream(htm_engine* e, int32_t src, void* stream) {
    if (!e || src < 0 || src >= e->n) return htm_fail(HTM_E_INVALID, "bad source stream");
    hipStream_t st = (hipStream_t)stream;
    if (int rf = flush_sync(e)) return rf;
    if (int rd = densify_conf(e, st)) return rd;
    for (int id = 1; id <= HTM_ST_COUNT; id++) {
        const Region& r = e->regions[id];
        if (!r.base || !r.per_stream) continue;
        const int32_t cnt = region_count(e, id);
        if (cnt < 2) continue;
        if (replicate_region((uint8_t*)r.base, r.per_stream, src, cnt, st)) return htm_fail(HTM_E_HIP, "replicate launch");
    }
    if (e->dc.sp_paged && e->nm > 1) {
        // the source's permanences (dense, once) imported into every stream,
        // whose checkpoints (the initial values) are the source's now
        HIP_TRY(hipStreamSynchronize(st));
        float* tmp = nullptr;
        HIP_TRY(hipMalloc(&tmp, e->regions[HTM_ST_SP_PERM].per_stream));
        int rc = paged_perm_export(e, src, 1, nullptr, tmp);
        if (!rc) rc = paged_perm_import(e, 0, e->n, nullptr, tmp, 0);
        (void)hipFree(tmp);
        if (rc) return rc;
    }
    // SP active list of the last step too (the TM reads it)
    if (replicate_region((uint8_t*)e->sp.act, HTM_MAXACT * 2, src, e->n, st) ||
        replicate_region((uint8_t*)e->sp.nact, 4, src, e->n, st))
        return htm_fail(HTM_E_HIP, "replicate launch");
    if (invalidate_colnz(e, stream)) return HTM_E_HIP;
    HIP_TRY(hipStreamSynchronize(st));
    e->fx_valid = false;
    return HTM_OK;
}

int htm_create_fleet(const htm_engine* model, int32_t model_stream, int32_t n_streams, int32_t q_capacity,
                     int32_t device, htm_engine** out) {
    if (!model || !out || n_streams < 1 || q_capacity < 64) return htm_fail(HTM_E_INVALID, "bad arguments");
    if (model->fleet) return htm_fail(HTM_E_INVALID, "the model must be an ordinary engine, not a fleet");
    if (model->dc.sdr_in) return htm_fail(HTM_E_INVALID, "fleets are built from encoder-input engines");
    if (model_stream < 0 || model_stream >= model->n) return htm_fail(HTM_E_INVALID, "bad model stream");
    *out = nullptr;
    HIP_TRY(hipSetDevice(model->device));
    if (int rf = flush_sync(const_cast<htm_engine*>(model))) return rf;
    if (int rd = densify_conf(const_cast<htm_engine*>(model), nullptr)) return rd;
    HIP_TRY(hipDeviceSynchronize());
    htm_engine* e = nullptr;
    htm_config fcfg = model->cfg;
    fcfg.sp_perm_rows = 0;  // the fleet's one SP instance is dense (never learns)
    int r = create_uninit(&fcfg, n_streams, device, &e, q_capacity);
    if (r) return r;
    // model regions -> the shared instance, per-stream regions -> stream 0 (then every stream)
    for (int id = 1; id <= HTM_ST_COUNT && !r; id++) {
        const Region& src = model->regions[id];
        const Region& dst = e->regions[id];
        if (id == HTM_ST_SP_PERM_CKPT) continue;
        if (src.per_stream == 0 && dst.per_stream == 0) continue;  // (no RDSE state: a ScalarEncoder model)
        if (id == HTM_ST_SP_PERM && model->dc.sp_paged) {
            std::vector<uint8_t> buf(src.per_stream);
            r = htm_export_state(const_cast<htm_engine*>(model), id, model_stream, 1, buf.data(), buf.size());
            if (!r) r = htm_import_state(e, id, 0, 1, buf.data(), buf.size());
            continue;
        }
        if (!src.base || !dst.base || src.per_stream != dst.per_stream) {
            r = htm_fail(HTM_E_STATE, "region %d layout differs", id);
            break;
        }
        if (hipMemcpy(dst.base, (const uint8_t*)src.base + src.per_stream * model_stream, src.per_stream,
                      hipMemcpyDefault) != hipSuccess)
            r = htm_fail(HTM_E_HIP, "fleet copy of region %d", id);
    }
    if (!r && (hipMemcpy(e->sp.act, model->sp.act + (size_t)model_stream * HTM_MAXACT, HTM_MAXACT * 2,
                         hipMemcpyDefault) != hipSuccess ||
               hipMemcpy(e->sp.nact, model->sp.nact + model_stream, 4, hipMemcpyDefault) != hipSuccess))
        r = htm_fail(HTM_E_HIP, "fleet copy of the SP output");
    if (!r) r = htm_replicate_stream(e, 0, nullptr);
    if (r) {
        htm_destroy(e);
        return r;
    }
    e->sp_learn = e->tm_learn = 0;
    *out = e;
    return HTM_OK;
}

int32_t htm_is_fleet(const htm_engine* e) { return e && e->fleet ? 1 : 0; }

int htm_flush(htm_engine* e, void* stream) {
    if (!e) return htm_fail(HTM_E_INVALID, "null engine");
    return flush_deferred(e, (hipStream_t)stream);
}

int32_t htm_n_streams(const htm_engine* e) { return e ? e->n : 0; }

int htm_get_config(const htm_engine* e, htm_config* out) {
    if (!e || !out) return htm_fail(HTM_E_INVALID, "bad arguments");
    *out = e->cfg;
    return HTM_OK;
}

size_t htm_device_bytes(const htm_engine* e) { return e ? e->bytes + e->fx_cap * 16 : 0; }

uint64_t htm_sp_perm_rows_used(htm_engine* e) {
    if (!e || !e->dc.sp_paged) return 0;
    unsigned long long x = 0;
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(&x, e->sp.pool_next, sizeof(x), hipMemcpyDeviceToHost) != hipSuccess)
        return 0;
    return std::min<unsigned long long>(x, e->dc.pool_rows);
}

#ifdef HTM_AB_KNOBS
// A/B builds only (not in htm_amd.h): the HTM_WG_TRACE timeline of the latest
// lockstep launch, [workgroup][8] (start, end, HW_ID, XCC_ID, step bytes, final
// active cells); returns the rows copied.
int64_t htm_ab_wg_trace(htm_engine* e, unsigned long long* out, int64_t max_rows) {
    if (!e || !e->wg_trace || !out) return 0;
    const int64_t rows = std::min<int64_t>(max_rows, (int64_t)e->wg_trace_cap);
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(out, e->wg_trace, (size_t)rows * 64, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    return rows;
}
#endif

int32_t htm_frozen_index_valid(const htm_engine* e) { return e && e->fx_valid ? 1 : 0; }

const char* htm_last_error(void) { return g_err.c_str(); }

int32_t htm_abi_version(void) { return HTM_ABI_VERSION; }

// Synchronise and report per-stream error flags (pool/queue overflow).
int htm_status(htm_engine* e) {
    if (!e) return htm_fail(HTM_E_INVALID, "null engine");
    if (int r = flush_sync(e)) return r;
    HIP_TRY(hipDeviceSynchronize());
    std::vector<htm_tm_header> h((size_t)e->n);
    HIP_TRY(hipMemcpy(h.data(), e->tm.hdr, h.size() * sizeof(htm_tm_header), hipMemcpyDeviceToHost));
    std::vector<uint32_t> spe((size_t)e->n);
    HIP_TRY(hipMemcpy(spe.data(), e->sp.err, spe.size() * 4, hipMemcpyDeviceToHost));
    if (uint32_t fe = flush_error(e))
        return htm_fail(HTM_E_CAPACITY, "deferred-duty flush error flags 0x%x (16: qualifying-segment list overflow, "
                        "results invalid -- raise q_capacity)", fe);
    for (int s = 0; s < e->n; s++) {
        if (spe[s] & SP_ERR_POOL)
            return htm_fail(HTM_E_CAPACITY, "stream %d error flag 0x20: SP permanence row pool exhausted -- updates "
                            "were dropped, results invalid; raise sp_perm_rows", s);
        if (h[s].error) return htm_fail(HTM_E_CAPACITY, "stream %d error flags 0x%x (1: segment pool full -- new segments were dropped, raise seg_capacity; 2: segment-update queue full; 4: >1 learn-predicted cell in a column; 8: learn-active cell list overflow; 16: qualifying-segment list overflow, results invalid -- raise q_capacity)", s, h[s].error);
    }
    return HTM_OK;
}

// ---------------------------------------------------------------------------
// save / load: "HTMAMD01", abi, config, n, learning flags, then regions --
// the SP checkpoints first, so a paged engine's permanences are imported
// against the initial values they were exported with.  A fleet's file starts
// "HTMFLT01" and carries its q_capacity after the flags; its model regions
// (SP permanences / connections, the TM segment pool) are stored once, its
// per-stream regions (TM state, RDSE maps, SP counters) for every stream.
static int save_order(int k) { return k == 0 ? HTM_ST_SP_PERM_CKPT : k < HTM_ST_SP_PERM_CKPT ? k : k + 1; }

int htm_save(htm_engine* e, const char* path) {
    if (!e || !path) return htm_fail(HTM_E_INVALID, "bad arguments");
    if (int rf = flush_sync(e)) return rf;  // the deferred dutyCycle() writes are part of the state
    FILE* f = std::fopen(path, "wb");
    if (!f) return htm_fail(HTM_E_IO, "cannot open %s", path);
    const char magic[8] = {'H', 'T', 'M', e->fleet ? 'F' : 'A', e->fleet ? 'L' : 'M', e->fleet ? 'T' : 'D', '0', '1'};
    int32_t abi = HTM_ABI_VERSION;
    bool ok = std::fwrite(magic, 8, 1, f) == 1 && std::fwrite(&abi, 4, 1, f) == 1 &&
              std::fwrite(&e->cfg, sizeof(htm_config), 1, f) == 1 && std::fwrite(&e->n, 4, 1, f) == 1 &&
              std::fwrite(&e->sp_learn, 4, 1, f) == 1 && std::fwrite(&e->tm_learn, 4, 1, f) == 1;
    if (ok && e->fleet) ok = std::fwrite(&e->dc.q_cap, 4, 1, f) == 1;
    std::vector<uint8_t> buf;
    for (int k = 0; ok && k < HTM_ST_COUNT; k++) {
        const int id = save_order(k);
        const Region& r = e->regions[id];
        const int32_t cnt = region_count(e, id);
        uint64_t nb = (uint64_t)r.per_stream * cnt;
        buf.resize(nb);
        if (htm_export_state(e, id, 0, cnt, buf.data(), nb)) { ok = false; break; }
        int32_t rid = id;
        ok = std::fwrite(&rid, 4, 1, f) == 1 && std::fwrite(&nb, 8, 1, f) == 1 && std::fwrite(buf.data(), 1, nb, f) == nb;
    }
    // last SP output (the TM of the next step does not need it, kept for outputs)
    std::fclose(f);
    if (!ok) return htm_fail(HTM_E_IO, "write failed: %s", path);
    return HTM_OK;
}

int htm_load(const char* path, int32_t device, htm_engine** out) {
    if (!path || !out) return htm_fail(HTM_E_INVALID, "bad arguments");
    FILE* f = std::fopen(path, "rb");
    if (!f) return htm_fail(HTM_E_IO, "cannot open %s", path);
    char magic[8];
    int32_t abi = 0, n = 0, spl = 1, tml = 1, qcap = 0;
    htm_config cfg;
    bool ok = std::fread(magic, 8, 1, f) == 1 &&
              (std::memcmp(magic, "HTMAMD01", 8) == 0 || std::memcmp(magic, "HTMFLT01", 8) == 0) &&
              std::fread(&abi, 4, 1, f) == 1 && abi == HTM_ABI_VERSION &&
              std::fread(&cfg, sizeof(cfg), 1, f) == 1 && std::fread(&n, 4, 1, f) == 1 &&
              std::fread(&spl, 4, 1, f) == 1 && std::fread(&tml, 4, 1, f) == 1;
    const bool fleet = ok && magic[3] == 'F';
    if (ok && fleet) ok = std::fread(&qcap, 4, 1, f) == 1 && qcap >= 64;
    if (!ok) {
        std::fclose(f);
        return htm_fail(HTM_E_IO, "%s is not an engine file of ABI %d", path, HTM_ABI_VERSION);
    }
    htm_engine* e = nullptr;
    int r = create_uninit(&cfg, n, device, &e, fleet ? qcap : 0);
    if (r) {
        std::fclose(f);
        return r;
    }
    std::vector<uint8_t> buf;
    for (int i = 0; ok && i < HTM_ST_COUNT; i++) {
        const int k = save_order(i);
        const int32_t cnt = region_count(e, k);
        int32_t rid;
        uint64_t nb;
        ok = std::fread(&rid, 4, 1, f) == 1 && std::fread(&nb, 8, 1, f) == 1 && rid == k &&
             nb == (uint64_t)e->regions[k].per_stream * cnt;
        if (!ok) break;
        buf.resize(nb);
        ok = std::fread(buf.data(), 1, nb, f) == nb;
        if (ok && import_region(e, k, 0, cnt, buf.data(), nb, false)) ok = false;
    }
    std::fclose(f);
    if (!ok) {
        htm_destroy(e);
        return htm_fail(HTM_E_IO, "truncated or inconsistent engine file %s", path);
    }
    e->sp_learn = fleet ? 0 : spl;
    e->tm_learn = fleet ? 0 : tml;
    *out = e;
    return HTM_OK;
}

}  // extern "C"
