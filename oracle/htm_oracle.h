/*
 * htm_oracle.h -- CPU restatement of the reference's HTM hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle for the MI355X engine
 * (and the timed "port" CPU baseline in bench.py).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The
 * product path never links or calls it.
 *
 * PARITY UNPINNED (w.r.t. NuPIC): the reference delegates all arithmetic to
 * NuPIC 1.0.x (nupic + nupic.bindings), which is not vendored, not installed
 * and Python-2-only.  This file restates the algorithm as
 * wired by the reference (ML/HTM/NetworkUtils.py:25-64,77-153,
 * ML/HTM/NetworkModel.py:35-157) with NuPIC semantics taken from SURVEY.md
 * Appendix A.  The only end-to-end pins the reference holds are the input
 * traces (ML/Data/{Training,Testing}Data.txt) and the threshold sweep in ML/Data/result_model1.txt,
 * which pins the score quantisation float32((40-k)/40).
 */
#ifndef HTM_ORACLE_H
#define HTM_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Parameters of one Model-1 style stream: encoder -> SP -> TM -> raw anomaly.
 * Defaults (orc_default_params) are the reference's: NetworkUtils.py:26-64,
 * encoder NetworkUtils.py:77-88. */
typedef struct {
    /* ScalarEncoder (one per field, fields concatenated in sorted name order) */
    int32_t n_fields;          /* 1 for Model 1 (cpu), 2 for Model 3 (cpu, mem) */
    int32_t enc_n;             /* 500 */
    int32_t enc_w;             /* 21 */
    double enc_minval;         /* 0 */
    double enc_maxval;         /* 100 */
    int32_t enc_clip;          /* clipInput True */
    /* SpatialPooler */
    int32_t sp_columns;        /* 2048 */
    int32_t sp_num_active;     /* numActiveColumnsPerInhArea 40 */
    float sp_potential_pct;    /* 0.8 */
    float sp_perm_connected;   /* 0.1 */
    float sp_perm_active_inc;  /* 0.0001 */
    float sp_perm_inactive_dec;/* 0.0005 */
    float sp_min_pct_overlap_dc; /* 0.001 (NuPIC default) */
    int32_t sp_duty_cycle_period; /* 1000 (NuPIC default) */
    float sp_boost_strength;   /* 0.0 */
    int32_t sp_stimulus_threshold; /* 0 (NuPIC default) */
    int32_t sp_update_period;  /* 50 (NuPIC constant) */
    uint64_t sp_seed;          /* 2045 */
    /* BacktrackingTM / Cells4 */
    int32_t tm_cells_per_col;  /* 12 */
    int32_t tm_new_syn_count;  /* 20 */
    int32_t tm_max_syn_per_seg;/* 32 */
    int32_t tm_max_segs_per_cell; /* 128 */
    float tm_initial_perm;     /* 0.21 */
    float tm_connected_perm;   /* 0.5 (NuPIC default) */
    float tm_perm_inc;         /* 0.1 */
    float tm_perm_dec;         /* 0.1 */
    float tm_perm_max;         /* 1.0 */
    int32_t tm_min_threshold;  /* 9 */
    int32_t tm_activation_threshold; /* 12 */
    int32_t tm_pam_length;     /* 3 */
    int32_t tm_max_inf_backtrack; /* 10 */
    int32_t tm_max_lrn_backtrack; /* 5 */
    int32_t tm_max_seq_length; /* 32 */
    int32_t tm_seg_update_valid_duration; /* 5 */
    uint64_t tm_seed;          /* 2045 */
    /* Alternatives for the Appendix A [L]/[M] choices (ORC_VAR_* bits; 0 = the
     * frozen restatement the HIP engine is held bit-exact to).  Only used by
     * oracle/variant_sweep.py to A/B them against ML/Data/result_model1.txt. */
    uint32_t variant;
    /* > 0: the SP input is an external SDR of this many bits (a second-level SP
     * fed a TM's bottomUpOut, MultiLevelNetworkModel.py:92-94); the encoder is
     * unused and steps go through orc_step_sdr */
    int32_t sdr_bits;
    /* per-field ScalarEncoder range (the aggregate's cpu %, mem %, mean and max
     * response time, StreamAggregator.py:101-115): field f uses
     * [field_minval[f], field_maxval[f]] when field_maxval[f] > field_minval[f],
     * else [enc_minval, enc_maxval] */
    double field_minval[4];
    double field_maxval[4];
    /* encoder type: ORC_ENC_SCALAR (0, NetworkUtils.py:77-88) or ORC_ENC_RDSE --
     * NuPIC's RandomDistributedScalarEncoder, the encoder of the reference's
     * model.yaml parameter set (ML/HTM/params/model.yaml:15-21: resolution 0.88,
     * seed 1; NuPIC defaults w = enc_w = 21, n = enc_n = 400) */
    int32_t enc_type;
    int32_t pad0;
    double rdse_resolution;
    uint64_t rdse_seed;
} orc_params;

#define ORC_ENC_SCALAR 0
#define ORC_ENC_RDSE 1
#define ORC_RDSE_BUCKETS 1000   /* RandomDistributedScalarEncoder INITIAL_BUCKETS (maxBuckets) */

#define ORC_VAR_SP_TIE_LOW       0x001u /* global inhibition: ties -> LOWER index (strict '>' admission) */
#define ORC_VAR_SP_NO_TIEBREAKER 0x002u /* SP init draws no 2048-entry tieBreaker before the pools */
#define ORC_VAR_SP_INIT_DOUBLE   0x004u /* initPermConnected_: 0.1f + span*u summed in double (C++ promotion) */
#define ORC_VAR_SP_POOL_ASCEND   0x008u /* potential-pool population in ascending input order (no wrap centre) */
#define ORC_VAR_TM_BMC_SEG_GE    0x010u /* getBestMatchingCell: last segment with '>=' over the column (Cells4 form) */
#define ORC_VAR_TM_DC_TIERS      0x020u /* refresh every segment's duty cycle when lrnIter crosses a tier */
#define ORC_VAR_TM_DC_READONLY   0x040u /* inferPhase2 reads segment duty cycles read-only */
#define ORC_VAR_TM_FREE_LATE     0x080u /* freeNSynapses: equal-permanence ties free the LATER synapse first */
#define ORC_VAR_TM_BT_LAST_START 0x100u /* inferBacktrack: prefer the in-sequence start CLOSEST to now */

typedef struct orc_model orc_model;

void orc_default_params(orc_params* p);
orc_model* orc_create(const orc_params* p);
orc_model* orc_clone(const orc_model* m);
void orc_free(orc_model* m);

/* One network.run(1): encode values[n_fields] -> SP.compute -> TM.compute
 * (infer on) -> raw anomaly.  Returns the float32 anomaly score that
 * TMRegion writes to getOutputData('anomalyScore')[0]. */
float orc_step(orc_model* m, const double* values, int sp_learn, int tm_learn);
/* Batch form for the CPU baseline: models[i] consumes values[i*n_fields..],
 * OpenMP across streams when built with -fopenmp. */
void orc_step_batch(orc_model** models, int n, const double* values,
                    int sp_learn, int tm_learn, float* scores, int n_threads);
void orc_tm_reset(orc_model* m);
/* One step of a model whose SP reads an external SDR (sdr_bits > 0):
 * input[sdr_bits] 0/1 -> SP -> TM -> raw anomaly (NetworkModel-style order) */
float orc_step_sdr(orc_model* m, const uint8_t* input, int sp_learn, int tm_learn);
/* TMRegion bottomUpOut (outputType 'normal'): infActive | infPredicted, 0/1 per cell */
void orc_tm_output(const orc_model* m, uint8_t* out);

/* ---- introspection (state dumps for parity tests) ---- */
int orc_num_inputs(const orc_model* m);
int orc_num_cells(const orc_model* m);
void orc_encode(orc_model* m, const double* values, uint8_t* out);  /* (RDSE: advances the encoder) */
/* active columns of the last step, ascending; returns count */
int orc_active_columns(const orc_model* m, int32_t* out);
/* columns with nonzero colConfidence before the last step (anomaly input) */
int orc_prev_pred_columns(const orc_model* m, int32_t* out);
/* per-cell 0/1 states at 't' */
void orc_tm_states(const orc_model* m, uint8_t* inf_active, uint8_t* inf_pred,
                   uint8_t* lrn_active, uint8_t* lrn_pred);
void orc_col_confidence(const orc_model* m, float* out);
void orc_cell_confidence(const orc_model* m, float* out);
/* scalar TM bookkeeping: [lrnIter, iter, pamCounter, learnedSeqLength,
 * n_prev_inf, n_prev_lrn, n_updates, n_segments, n_synapses] */
void orc_tm_scalars(const orc_model* m, int64_t* out9);
double orc_tm_avg_input_density(const orc_model* m);
/* work counters: [inferPhase2 calls, inferBacktracks, lrnPhase2 calls, lrnBacktracks,
 * inferPhase2 calls on the critical path were backtrack start offsets replayed in parallel] */
void orc_tm_stats(const orc_model* m, int64_t* out5);
/* Segments in canonical order (column, cell, position in cell list).
 * seg_info[k*5+{0..4}] = {cell, isSequence, posActivations, lastDCIter, nsyn}
 * seg_dc[k] = lastPosDutyCycle; syn_src/syn_perm hold max_syn entries per
 * segment (unused slots 0).  Returns n_segments (call with NULL to size). */
int orc_tm_segments(const orc_model* m, int32_t* seg_info, float* seg_dc,
                    int32_t* syn_src, float* syn_perm, int max_syn);
/* SP state: perm dense [columns][inputs], potential [columns][inputs] 0/1,
 * connected [columns][inputs] 0/1, duty cycles, scalars */
void orc_sp_state(const orc_model* m, float* perm, uint8_t* potential,
                  uint8_t* connected, float* overlap_dc, float* active_dc,
                  float* min_overlap_dc, float* boost, int64_t* iters2);
void orc_sp_overlaps(const orc_model* m, int32_t* out);
/* RNG known-answer helpers (nupic::Random restatement) */
void orc_rng_stream(uint64_t seed, int n, uint32_t* out);
void orc_rng_real64(uint64_t seed, int n, double* out);
/* TM RNG state of a model (31 words + fptr + rptr) */
void orc_tm_rng_state(const orc_model* m, uint32_t* out33);
/* RDSE encoder state of field f: scalars {minIndex, maxIndex, has_offset,
 * numTries}, *offset, and the bucket map rows [ORC_RDSE_BUCKETS][w] (rows
 * outside [minIndex, maxIndex] are zero) */
void orc_rdse_state(const orc_model* m, int f, int32_t* scalars4, double* offset, int32_t* map);
/* bucket index of field f of the last encoded record (-1: missing) */
int orc_bucket(const orc_model* m, int f);
/* boost factor exp((target - activeDutyCycle) * boostStrength) as the SP
 * computes it (a deterministic double evaluation rounded to float) */
float orc_exp_det(float x);

#ifdef __cplusplus
}
#endif
#endif
