/*
 * htm_amd.h -- C ABI of the MI355X-native batched HTM engine.
 *
 * One engine = N independent metric streams, each a Model-1 network
 * (ScalarEncoder -> SpatialPooler -> BacktrackingTM -> raw anomaly), stepped
 * in lockstep on one GPU.  Plain pointers and sizes only; no C++ exceptions
 * cross this boundary; every entry point returns 0 on success or a negative
 * HTM_E* code, with htm_last_error() describing the failure.
 *
 * Reference interfaces each entry point replaces (paths relative to the
 * reference repo root; NuPIC symbols are the external library the reference
 * calls):
 *   htm_create        Network() + addRegion(RecordSensor/SPRegion/TMRegion)
 *                     + link(): ML/HTM/NetworkModel.py:48-110,
 *                     ML/HTM/NetworkUtils.py:111-153 (params :25-64, :77-88)
 *   htm_set_learning  region.setParameter("learningMode", b):
 *                     ML/HTM/NetworkUtils.py:132,147, ML/HTM/NetworkModel.py:40-44
 *                     (SP and TM flags are independent: the reference keeps
 *                     SP learning on while TM learning is off)
 *   htm_step          dataSource.setData(v) + network.run(1) +
 *                     getOutputData("anomalyScore")[0]:
 *                     ML/HTM/NetworkModel.py:35-46,112-133,
 *                     ML/HTM/StreamReader.py:157-161
 *   htm_get_output    region.getOutputData(...): NetworkModel.py:129,133
 *   htm_save/htm_load network.save(path) / Network(path):
 *                     ML/HTM/NetworkUtils.py:156-163, ModelTesting.py:176
 *   htm_reset_tm      TMRegion resetIn -> BacktrackingTM.reset() [ext]
 *   htm_last_error    NTA_THROW -> RuntimeError convention [ext]
 */
#ifndef HTM_AMD_H
#define HTM_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HTM_ABI_VERSION 6

/* error codes */
#define HTM_OK 0
#define HTM_E_INVALID (-1)   /* bad argument / unsupported parameter */
#define HTM_E_HIP (-2)       /* HIP runtime failure */
#define HTM_E_CAPACITY (-3)  /* a per-stream pool overflowed (see last_error) */
#define HTM_E_IO (-4)        /* save/load failure */
#define HTM_E_STATE (-5)     /* call not valid in the current engine state */

/* Network parameters of one stream.  Field meaning, units and defaults are
 * the reference's (htm_default_config): encoder NetworkUtils.py:77-88,
 * SP_PARAMS NetworkUtils.py:26-41, TM_PARAMS NetworkUtils.py:44-64, plus the
 * NuPIC defaults the reference relies on. */
typedef struct {
    /* ScalarEncoder per field (MultiEncoder: fields in sorted name order) */
    int32_t n_fields;            /* 1 (Model 1: cpu) .. 4 */
    int32_t enc_n;               /* 500 */
    int32_t enc_w;               /* 21 */
    double enc_minval;           /* 0.0 */
    double enc_maxval;           /* 100.0 */
    int32_t enc_clip;            /* 1 */
    /* SpatialPooler */
    int32_t sp_columns;          /* 2048 (multiple of 64, <= 4096) */
    int32_t sp_num_active;       /* 40 (<= 64) */
    float sp_potential_pct;      /* 0.8 */
    float sp_perm_connected;     /* 0.1 */
    float sp_perm_active_inc;    /* 0.0001 */
    float sp_perm_inactive_dec;  /* 0.0005 */
    float sp_min_pct_overlap_dc; /* 0.001 */
    int32_t sp_duty_cycle_period;/* 1000 */
    float sp_boost_strength;     /* 0.0 (NetworkUtils.py:41); model.yaml:41 uses 3.0:
                                    boostFactors = exp((targetDensity - activeDutyCycle) * strength)
                                    after every learning step, boosted overlaps select the winners */
    int32_t sp_stimulus_threshold; /* 0 */
    int32_t sp_update_period;    /* 50 */
    uint64_t sp_seed;            /* 2045 */
    /* BacktrackingTM */
    int32_t tm_cells_per_col;    /* 12 (<= 32) */
    int32_t tm_new_syn_count;    /* 20 (<= 32) */
    int32_t tm_max_syn_per_seg;  /* 32 (<= 32) */
    int32_t tm_max_segs_per_cell;/* 128 (<= 255) */
    float tm_initial_perm;       /* 0.21 */
    float tm_connected_perm;     /* 0.5 */
    float tm_perm_inc;           /* 0.1 */
    float tm_perm_dec;           /* 0.1 */
    float tm_perm_max;           /* 1.0 */
    int32_t tm_min_threshold;    /* 9 */
    int32_t tm_activation_threshold; /* 12 */
    int32_t tm_pam_length;       /* 3 */
    int32_t tm_max_inf_backtrack;/* 10 (<= 15) */
    int32_t tm_max_lrn_backtrack;/* 5 (<= 15) */
    int32_t tm_max_seq_length;   /* 32 */
    int32_t tm_seg_update_valid_duration; /* 5 */
    uint64_t tm_seed;            /* 2045 */
    /* engine capacities (per stream) */
    int32_t seg_capacity;        /* segment pool slots per stream */
    int32_t upd_capacity;        /* queued segment updates per stream */
    int32_t seed_stride;         /* stream s uses seeds sp_seed + s*stride,
                                    tm_seed + s*stride (0: all identical) */
    /* > 0: the SP reads an external input SDR of sdr_bits bits instead of the
     * encoder -- the second level of the reference's Models 2/3, whose L2
     * SPRegion is fed the L1 TMRegion's bottomUpOut (MultiLevelNetworkModel.py:92-97,
     * MultiLevelNetworkAnomaly.py:112-116); steps go through htm_step_sdr /
     * htm_run_sdr.  <= 32768 */
    int32_t sdr_bits;
    /* Per-field encoder range: field f uses [field_minval[f], field_maxval[f]]
     * when field_maxval[f] > field_minval[f], else [enc_minval, enc_maxval] --
     * the 4-field aggregate of StreamAggregator.py:101-115 (cpu %, mem %, mean
     * and max response time) does not share one range.  n, w and clipInput
     * stay shared.  Zero (htm_default_config) = the shared range. */
    double field_minval[4];
    double field_maxval[4];
    /* SP permanence storage.  0 (htm_default_config): dense, ncol rows of
     * n_potential floats per stream.  > 0: paged -- one pool of
     * n_streams * sp_perm_rows rows shared by all streams; a column gets a
     * row on its first permanence change (adaptSynapses_ / bumpUpWeakColumns_),
     * until then its permanences are the NuPIC initial values, regenerated on
     * the GPU from per-stream nupic::Random checkpoints (one per 8 columns).
     * Fresh learning streams touch ~25-30 % of their columns in 256 steps,
     * so config 3 (65,536 learning streams, BASELINE.json configs[2]) fits one
     * GPU.  Results are identical to the dense layout; an exhausted pool sets
     * error flag 32 (htm_status: HTM_E_CAPACITY, results invalid). */
    int32_t sp_perm_rows;
    int32_t reserved0;           /* 0 */
    /* Encoder of every field: HTM_ENC_SCALAR (the reference's ScalarEncoder,
     * NetworkUtils.py:77-88) or HTM_ENC_RDSE -- NuPIC's
     * RandomDistributedScalarEncoder of the model.yaml parameter set
     * (ML/HTM/params/model.yaml:15-21: resolution 0.88, seed 1; n = enc_n
     * (NuPIC default 400), w = enc_w (21, odd), n > 6 w).  An RDSE is stateful
     * per stream and field: its bucket map grows on demand and its offset is
     * the first value it encodes (state region HTM_ST_ENC_RDSE). */
    int32_t enc_type;
    int32_t reserved1;           /* 0 */
    double rdse_resolution;      /* 0.88 */
    uint64_t rdse_seed;          /* 1; stream s uses rdse_seed + s * seed_stride */
} htm_config;

#define HTM_ENC_SCALAR 0
#define HTM_ENC_RDSE 1
#define HTM_RDSE_BUCKETS 1000    /* RandomDistributedScalarEncoder INITIAL_BUCKETS */

typedef struct htm_engine htm_engine;

/* Fill *cfg with the reference's Model-1 parameters. */
void htm_default_config(htm_config* cfg);

/* Create an engine of n_streams streams on HIP device `device`, running
 * the NuPIC initialisation (SP potential pools / permanences from
 * nupic::Random(seed)) on the GPU.  *out receives the handle. */
int htm_create(const htm_config* cfg, int32_t n_streams, int32_t device, htm_engine** out);
int htm_destroy(htm_engine* eng);

/* Independent SP / TM learning flags (both start on, like the regions). */
int htm_set_learning(htm_engine* eng, int32_t sp_learn, int32_t tm_learn);

/* Engine options. */
#define HTM_OPT_FROZEN_INDEX 1 /* 1 (default): while TM learning is off, infer through the
                                  frozen cell->segment forward index; 0: scan the pool */
#define HTM_OPT_KEEP_PREV 2    /* 1: retain prevPredictedColumns for HTM_OUT_PREV_PRED_COLS */
#define HTM_OPT_KEEP_OVERLAPS 3 /* 1: retain SP overlaps for HTM_OUT_SP_OVERLAPS */
#define HTM_OPT_PROFILE 4       /* N >= 1: bracket the SP and TM kernels of every N-th launch with HIP
                                   events (1: every launch; htm_profile_read averages the sampled ones) */
#define HTM_OPT_FUSED 5         /* 1 (default): one fused SP+TM kernel per htm_step and per
                                   chunk of htm_run steps (each stream runs its chunk without
                                   waiting for the others); 0: separate SP and TM launches */
#define HTM_OPT_RUN_CHUNK 6     /* steps per fused htm_run launch (default 256) */
#define HTM_OPT_RUN_UNIT 7      /* steps per work-queue unit of a fused htm_run launch (0, the
                                   default: launch steps / 8 clamped to [16, 64]); a stream's
                                   TM state stays in LDS for a unit's steps */
/* 8, 9: retired (round-2 backtrack assist, measured no faster; removed from the kernels) */
#define HTM_OPT_DEFER_DUTY 10   /* 1 (default): in frozen lockstep steps (htm_step), a phase 2 whose
                                   confidences the step discards (backtrack replays, out-of-sequence
                                   results) computes only the predicted cells; the first dutyCycle()
                                   record write of its qualifying segments is deferred to a flush kernel
                                   that runs on the engine's own HIP stream beside the next steps (every
                                   8 steps), and completes before any call that reads the records: export,
                                   save, learning on, htm_status / htm_counters, htm_flush.  Results and
                                   state are those of the undeferred step.  0: count every phase 2 in full */
#define HTM_OPT_FLUSH_MODE 11   /* where the deferred-write flush runs: 0 on the engine's own HIP stream
                                   beside the next steps, 1 on the step stream after them (full width).
                                   Results are identical; the default is chosen by measurement from the
                                   engine size (deferred dutyCycle() writes).  (ABI 5's mode 2,
                                   a flush in the tail of the next ordered launch, measured slower and
                                   was removed in ABI 6) */
#define HTM_OPT_ORDERED 12      /* 1 (default): a frozen lockstep step (htm_step) of a dense-SP engine of
                                   at most 16,384 streams runs the SP kernel, lists the streams by the
                                   cost of their TM step (the active cells phase 1 will list), and runs
                                   the TM steps heaviest first; results are identical.  0: one fused
                                   SP+TM workgroup per stream in stream order */
#define HTM_OPT_FLUSH_EVERY 13  /* lockstep steps between the periodic flushes of the deferred dutyCycle()
                                   writes (0: the default, 6, at most half the log ring); a cadence past
                                   the ring makes the log fill, and a full log makes a step count its
                                   discarded phase 2s in full (results identical) */
#define HTM_OPT_SPLIT_LEARN 14  /* 1 (default): a lockstep htm_step with TM learning on runs the SP kernel (its
                                   learning included) and then the TM learning kernel with the SP compiled out
                                   (each at its own occupancy); results are identical.  0: one fused SP+TM
                                   learning kernel */
/* 15: retired in ABI 6 (HTM_OPT_WIDE: the heaviest ordered steps by 768-thread workgroups, measured
   slower); setting it returns HTM_E_INVALID */
int htm_set_option(htm_engine* eng, int32_t opt, int32_t value);

/* Complete the deferred dutyCycle() writes (HTM_OPT_DEFER_DUTY): work enqueued
 * on `stream` afterwards sees them (asynchronous w.r.t. the host); a
 * benchmark's timed region ends with it. */
int htm_flush(htm_engine* eng, void* stream);

/* Kernel times of the profiled launches since the last call (synchronises):
 * out4 = {SP kernel ms, TM (or fused SP+TM) kernel ms, steps covered,
 * profiled launches}.  Fused launches report their whole time as TM. */
int htm_profile_read(htm_engine* eng, double* out4);

/* Sum over streams of the TM counters (synchronises): out8 = {algorithmic HBM
 * bytes moved by the TM kernel, inferPhase2 calls, inferBacktracks,
 * learnPhase2 calls, learnBacktracks, live segments, pool high-water marks,
 * OR of error flags}. */
int htm_counters(htm_engine* eng, uint64_t* out8);

/* Diagnostic builds only (libhtm_amd_stamps.so, -DHTM_STAMPS): per-phase
 * shader-cycle stamps of the TM kernel summed over streams since the last
 * call (out128[0..31]) and event counts (out128[32..63]), then the same over
 * the tail steps only -- stream-steps whose TM part took >= 2^18 cycles
 * (out128[64..127]); HTM_E_STATE in the product library. */
int htm_debug_stamps(htm_engine* eng, uint64_t* out128);

/* Synchronise and check every stream's overflow flags (HTM_E_CAPACITY). */
int htm_status(htm_engine* eng);

/* One network.run(1) for every stream.  d_values: device pointer to
 * n_streams * n_fields doubles (NaN = missing value).  d_scores: device
 * pointer to n_streams floats receiving the raw anomaly score.  stream: a
 * hipStream_t (NULL = default stream).  Asynchronous w.r.t. the host. */
int htm_step(htm_engine* eng, const double* d_values, float* d_scores, void* stream);

/* Run n_steps steps back to back: d_values is [n_steps][n_streams][n_fields],
 * d_scores is [n_steps][n_streams]. */
int htm_run(htm_engine* eng, int32_t n_steps, const double* d_values, float* d_scores, void* stream);

/* The same for an engine whose SP reads an input SDR (sdr_bits > 0): d_sdr is a
 * DEVICE uint32 bitmap [n_streams][ceil(sdr_bits/32)] (e.g. another engine's
 * HTM_OUT_TM_OUTPUT: L1 TM bottomUpOut -> L2 SPRegion bottomUpIn,
 * MultiLevelNetworkModel.py:94), or [n_steps][n_streams][words] for htm_run_sdr. */
int htm_step_sdr(htm_engine* eng, const uint32_t* d_sdr, float* d_scores, void* stream);
int htm_run_sdr(htm_engine* eng, int32_t n_steps, const uint32_t* d_sdr, float* d_scores, void* stream);

/* Output selectors for htm_get_output (all per stream, concatenated over
 * streams, written to a DEVICE buffer of `bytes` bytes on `stream`). */
#define HTM_OUT_ACTIVE_COLUMNS 1   /* uint8 [ncol]  SP bottomUpOut */
#define HTM_OUT_PREV_PRED_COLS 2   /* uint8 [ncol]  nonzero(colConfidence(t-1)) */
#define HTM_OUT_INF_ACTIVE 3       /* uint32 bitmap [ncells/32] infActiveState t */
#define HTM_OUT_INF_PREDICTED 4    /* uint32 bitmap [ncells/32] infPredictedState t */
#define HTM_OUT_LRN_ACTIVE 5       /* uint32 bitmap [ncells/32] lrnActiveState t */
#define HTM_OUT_LRN_PREDICTED 6    /* uint32 bitmap [ncells/32] lrnPredictedState t */
#define HTM_OUT_COL_CONFIDENCE 7   /* float [ncol]  colConfidence t (topDownOut) */
#define HTM_OUT_TM_OUTPUT 8        /* uint32 bitmap [ncells/32] bottomUpOut = infP|infA */
#define HTM_OUT_SP_OVERLAPS 9      /* int32 [ncol] SP overlaps of the last step */
#define HTM_OUT_BUCKETS 10         /* int32 [4] the encoders' bucket index per field of the last
                                      record (-1: missing value): the sensor's bucketIdxOut
                                      (NetworkModel.py:88-95) */
#define HTM_OUT_PRED_COLS 11       /* uint8 [ncol]  nonzero(colConfidence t): the predicted columns the
                                      next step's raw anomaly reads (NetworkModel.py:133 via
                                      prevPredictedColumns); read from the packed state, the
                                      state is not changed (HTM_OUT_COL_CONFIDENCE densifies it) */
int htm_get_output(htm_engine* eng, int32_t which, void* d_dst, size_t bytes, void* stream);
/* Bytes per stream of an output selector (0 if unknown). */
size_t htm_output_bytes(const htm_engine* eng, int32_t which);

/* Raw per-stream state export/import (host buffers), used by save/load and
 * by the parity tests.  Region ids and layouts are documented in DESIGN.md
 * §State layout; htm_state_bytes gives the per-stream size of a region. */
#define HTM_ST_SP_CONNT 1      /* uint32 [nin_pad][ncol/32] connected, input-major */
#define HTM_ST_SP_POTMASK 2    /* uint32 [ncol][nin_pad/32] potential pool */
#define HTM_ST_SP_PERM 3       /* float  [ncol][n_potential] potential order */
#define HTM_ST_SP_DUTY 4       /* float  [2][ncol] overlap, active duty cycles */
#define HTM_ST_SP_SCALARS 5    /* uint32 [4] iter, iter_learn, min_overlap_dc bits, 0 */
#define HTM_ST_TM_HEADER 6     /* struct htm_tm_header */
#define HTM_ST_TM_BITMAPS 7    /* uint32 [4][ncells/32] infA, infP, lrnA, lrnP */
#define HTM_ST_TM_COLCONF 8    /* float [ncol] */
#define HTM_ST_TM_SEG_META 9   /* uint32 [seg_capacity] cell | nsyn<<16 | seq<<22 | live<<23 */
#define HTM_ST_TM_SEG_SRC 10   /* uint16 [seg_capacity][32] */
#define HTM_ST_TM_SEG_PERM 11  /* float [seg_capacity][32] */
#define HTM_ST_TM_SEG_CONN 12  /* uint32 [seg_capacity] connected-synapse mask */
#define HTM_ST_TM_SEG_DUTY 13  /* uint32 [seg_capacity][3] posAct, lastDC bits, lastDCIter */
#define HTM_ST_TM_CELL_NSEG 14 /* uint8 [ncells] segments per cell */
#define HTM_ST_TM_PATTERNS 15  /* uint16 [inf 16 + lrn 16][64] pattern history rings */
#define HTM_ST_TM_UPDATES 16   /* htm_tm_update [upd_capacity] */
#define HTM_ST_SP_PERM_CKPT 17 /* paged engines (sp_perm_rows > 0) only, else 0 bytes:
                                  uint32 [ncol/8][64] nupic::Random checkpoints of the SP
                                  initialisation, one per 8 columns (the initial permanences
                                  of columns without a pool row).  Importing it re-bases the
                                  stream (its permanences keep their values); importing 0
                                  bytes keeps the stream's own. */
#define HTM_ST_SP_BOOST 18     /* float [ncol] boostFactors (1.0 until a learning step with
                                  boostStrength != 0) */
#define HTM_ST_ENC_RDSE 19     /* RDSE engines (enc_type HTM_ENC_RDSE) only, else 0 bytes: per
                                  field, int32 [64] {minIndex, maxIndex, has_offset, numTries,
                                  offset (double, 2 words), nupic::Random state [31], fptr, rptr,
                                  0...} then int16 [HTM_RDSE_BUCKETS][enc_w] bucket map rows
                                  (rows outside [minIndex, maxIndex] are unused), padded to 16 B */
#define HTM_ST_COUNT 19
size_t htm_state_bytes(const htm_engine* eng, int32_t region);
int htm_export_state(htm_engine* eng, int32_t region, int32_t stream_begin, int32_t n,
                     void* h_dst, size_t bytes);
int htm_import_state(htm_engine* eng, int32_t region, int32_t stream_begin, int32_t n,
                     const void* h_src, size_t bytes);

/* Per-stream TM bookkeeping (HTM_ST_TM_HEADER layout). */
typedef struct {
    uint32_t lrn_iter, iter;
    int32_t pam_counter, learned_seq_length, reset_called, have_avg_density;
    double avg_input_density, avg_learned_seq_length;
    uint32_t rng_state[31];
    int32_t rng_f, rng_r;
    uint32_t seg_hwm, seg_live;
    int32_t n_inf_pat, n_lrn_pat;
    uint16_t inf_pat_len[16];
    uint16_t lrn_pat_len[16];
    int32_t n_upd;
    uint32_t error;          /* bit 0 seg pool full, bit 1 update queue full */
    uint32_t stat_inf_phase2, stat_inf_backtrack, stat_lrn_phase2, stat_lrn_backtrack;
    uint16_t inf_pat_head, lrn_pat_head; /* ring-buffer heads of the histories */
    uint32_t lp2_pending;    /* engine-internal: the last learning step's final learnPhase2 is deferred
                                into the next step's first pool scan; always 0 in exported / saved state */
    uint64_t stat_bytes;     /* algorithmic HBM bytes moved by the TM kernel (accumulated) */
} htm_tm_header;

/* A queued segment update (BacktrackingTM segmentUpdates entry). */
typedef struct {
    uint32_t slot;           /* segment slot */
    uint16_t col;
    uint8_t cell;            /* cell index within the column */
    uint8_t n_new;           /* new synapse sources */
    uint32_t active_mask;    /* existing synapse positions to reinforce */
    uint32_t date;           /* lrn_iter when queued */
    uint16_t new_src[32];
} htm_tm_update;

/* TM reset (BacktrackingTM.reset) of every stream. */
int htm_reset_tm(htm_engine* eng, void* stream);

/* Save / load the whole engine (config + every region) to one file.  The
 * deferred dutyCycle() writes are completed first.  A fleet (htm_create_fleet)
 * saves its shared model once and every stream's own state, and loads back as
 * a fleet: a run saved mid-way continues bit-exactly from the loaded file
 * (NetworkModel.py:123-125 saves before the step, ModelTesting.py:176 reloads). */
int htm_save(htm_engine* eng, const char* path);
int htm_load(const char* path, int32_t device, htm_engine** out);

/* Replicate stream `src` into every stream of the engine (config-2 setup:
 * every stream starts from the same trained Model-1 state). */
int htm_replicate_stream(htm_engine* eng, int32_t src, void* stream);

/* Fleet mode: n_streams streams that share ONE
 * frozen model -- the SP and the TM segment pool of stream `model_stream` of
 * `model` -- each with its own TM state (cell bitmaps, confidences, pattern
 * history, counters), every stream starting from the model stream's state.
 * Learning stays off (htm_set_learning with a flag on: HTM_E_STATE); with
 * learning off replicated models never diverge, so a fleet's results equal
 * those of an ordinary engine holding n_streams copies of the model, at a
 * fraction of the memory.  q_capacity bounds each stream's list of
 * qualifying segments per inference pass (overflow: htm_status reports
 * error flag 16). */
int htm_create_fleet(const htm_engine* model, int32_t model_stream, int32_t n_streams, int32_t q_capacity,
                     int32_t device, htm_engine** out);
int32_t htm_is_fleet(const htm_engine* eng);

/* Engine introspection */
int32_t htm_n_streams(const htm_engine* eng);
int htm_get_config(const htm_engine* eng, htm_config* out);
/* Bytes of device memory held by the engine. */
size_t htm_device_bytes(const htm_engine* eng);
/* Paged SP permanences: pool rows handed out so far (synchronises; 0 for a
 * dense engine).  Rows never return to the pool. */
uint64_t htm_sp_perm_rows_used(htm_engine* eng);
/* 1 when the frozen-TM forward index (used while TM learning is off) is
 * current. */
int32_t htm_frozen_index_valid(const htm_engine* eng);

/* ---- SLO-violation prediction harness, batched over streams ----------------
 * ML/HTM/ModelTesting.py runModel :36-107, processpredictionList :113-146,
 * getModelStats :148-171.  Per stream and record: the
 * window of 1 + lookahead anomaly scores, the record's violation count and
 * int(mean response time); a record with a missing metric is skipped
 * (valid = 0).  Threshold 0.85 in the code, 0.98/0.99 in the README sweep;
 * max_lead 50; slo_response 70 (ms). */
typedef struct htm_slo htm_slo;
int htm_slo_create(int32_t n_streams, double threshold, int32_t max_lead, int32_t slo_response, int32_t device,
                   htm_slo** out);
int htm_slo_destroy(htm_slo* slo);
/* d_scores: DEVICE float [window][n_streams] (the engine's htm_run output
 * rows of the record's steps); d_violations, d_means: DEVICE int32
 * [n_streams]; d_valid: DEVICE uint8 [n_streams] or NULL (all valid). */
int htm_slo_record(htm_slo* slo, const float* d_scores, int32_t window, const int32_t* d_violations,
                   const int32_t* d_means, const uint8_t* d_valid, void* stream);
/* getModelStats per stream into HOST h_out5[n_streams][5] = {TP, FP, TN, FN,
 * lead-time sum} over the prediction list minus its last max_lead items. */
int htm_slo_stats(htm_slo* slo, int64_t* h_out5, void* stream);

/* ---- AnomalyLikelihood, batched over streams (north-star extension; the
 * reference never computes it, parity unpinned) ------------------------------
 * NuPIC 1.0.x AnomalyLikelihood semantics (oracle/likelihood_reference.py):
 * learning_period 288, estimation_samples 100, historic_window 8640 (<= 8640),
 * reestimation_period 100 are NuPIC's defaults. */
typedef struct htm_likelihood htm_likelihood;
int htm_likelihood_create(int32_t n_streams, int32_t learning_period, int32_t estimation_samples,
                          int32_t historic_window, int32_t reestimation_period, int32_t device, htm_likelihood** out);
int htm_likelihood_destroy(htm_likelihood* lk);
/* anomalyProbability(value, anomalyScore) of every stream: d_values DEVICE
 * double, stream s's metric at d_values[s * value_stride]; d_scores DEVICE
 * float [n] (the engine's raw scores); d_out DEVICE double [n]. */
int htm_likelihood_step(htm_likelihood* lk, const double* d_values, int32_t value_stride, const float* d_scores,
                        double* d_out, void* stream);

/* ---- SDRClassifier, batched over streams ---------------
 * Replaces the "py.SDRClassifierRegion" the reference adds with alpha 0.005,
 * steps "1,2,3,4,5,6,7" (ML/HTM/NetworkModel.py:70-97): its compute() over
 * TM bottomUpOut + the sensor's bucketIdxOut / actValueOut (:88-95), read by
 * getOutputData("actualValues" / "probabilities") in
 * NetworkUtils.getPredictionResults (ML/HTM/NetworkUtils.py:166-184).
 * NuPIC 1.0.x SDRClassifier semantics (oracle/sdr_classifier_reference.py;
 * parity unpinned w.r.t. NuPIC).  n_inputs = TM cells (multiple of 32),
 * n_buckets = the predicted field's bucket count (<= 1024), steps distinct,
 * <= 16 of them.  Weights are float64 [steps][n_inputs][n_buckets] per stream. */
typedef struct htm_classifier htm_classifier;
int htm_cls_create(int32_t n_streams, int32_t n_inputs, int32_t n_buckets, const int32_t* steps, int32_t n_steps,
                   double alpha, double act_value_alpha, int32_t device, htm_classifier** out);
int htm_cls_destroy(htm_classifier* cls);
/* One SDRClassifierRegion.compute of every stream.  d_pattern: DEVICE uint32
 * bitmap [n_streams][n_inputs/32] (HTM_OUT_TM_OUTPUT); d_bucket DEVICE int32
 * [n] (< 0: no learning for that stream) and d_act_value DEVICE double [n]
 * (needed when learn); outputs (needed when infer): d_probabilities DEVICE
 * double [n][n_steps][n_buckets] (zeros above maxBucketIdx), d_actual_values
 * DEVICE double [n][n_buckets] (the region's actualValues output). */
int htm_cls_compute(htm_classifier* cls, const uint32_t* d_pattern, const int32_t* d_bucket, const double* d_act_value,
                    int32_t learn, int32_t infer, double* d_probabilities, double* d_actual_values, void* stream);
/* Synchronise; OR of per-stream flags: 1 empty pattern, 2 bucket >= n_buckets. */
int htm_cls_status(htm_classifier* cls, int32_t* out_flags);
/* State regions (per stream) for save/load and tests. */
#define HTM_CLS_ST_SCALARS 1   /* int32 [12] recordNum, maxInputIdx, maxBucketIdx, ... */
#define HTM_CLS_ST_ACTUAL 2    /* double [n_buckets] actual-value EMA */
#define HTM_CLS_ST_ACTUAL_OK 3 /* int32 [n_buckets] 1 where the EMA holds a value */
#define HTM_CLS_ST_HIST_REC 4  /* int32 [max(steps)+1] history record numbers */
#define HTM_CLS_ST_HIST_LEN 5  /* int32 [max(steps)+1] history pattern lengths */
#define HTM_CLS_ST_HIST_IDX 6  /* uint16 [max(steps)+1][n_inputs] history patterns */
#define HTM_CLS_ST_WEIGHTS 7   /* double [n_steps][n_inputs][n_buckets] */
size_t htm_cls_state_bytes(const htm_classifier* cls, int32_t region);
int htm_cls_export_state(htm_classifier* cls, int32_t region, int32_t stream_begin, int32_t n, void* h_dst,
                         size_t bytes);
int htm_cls_import_state(htm_classifier* cls, int32_t region, int32_t stream_begin, int32_t n, const void* h_src,
                         size_t bytes);

const char* htm_last_error(void);
int32_t htm_abi_version(void);
/* How the library was built: "<unit> <optimisation level>;..." for every
 * translation unit (LLVM's gfx950 verifier has rejected some units at -O3;
 * those build at -O2 or -O1, csrc/cc.sh), then the compiler and the target. */
const char* htm_build_info(void);

#ifdef __cplusplus
}
#endif
#endif
