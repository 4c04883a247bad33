/*
 * htm_oracle.c -- CPU restatement of the reference's HTM hot path
 * (encoder -> SPRegion compute -> TMRegion compute -> raw anomaly).
 *
 * TEST INFRASTRUCTURE ONLY (parity oracle + "port" CPU baseline); see
 * htm_oracle.h.  PARITY UNPINNED w.r.t. NuPIC: the reference calls NuPIC
 * 1.0.x, which is absent; semantics follow SURVEY.md
 * Appendix A and the NuPIC 1.0.x algorithms the reference instantiates:
 *   - ScalarEncoder           NetworkUtils.py:77-88        (Appendix A.1)
 *   - RandomDistributedScalarEncoder  params/model.yaml:15-21 (the 32-cell
 *     model.yaml shape; NuPIC 1.0.x nupic/encoders/random_distributed_scalar.py)
 *   - SpatialPooler (cpp)     NetworkUtils.py:26-41,126-136 (Appendix A.2)
 *   - BacktrackingTM(CPP)     NetworkUtils.py:44-64,140-153 (Appendix A.3)
 *   - computeRawAnomalyScore  read at NetworkModel.py:133 (Appendix A.4)
 * The control flow of the TM mirrors NuPIC's BacktrackingTM (py), which
 * NuPIC kept bit-compatible with Cells4 (same nupic::Random draw order);
 * arithmetic is float32 as in Cells4 (Real = float).
 *
 * Frozen [L]/[M] choices (documented in DESIGN.md §Oracle):
 *   - Random seeding s0 = seed % 2147483646 + 1 (Appendix A.2).
 *   - SP init draws a 2048-entry tieBreaker before the per-column loop.
 *   - Global inhibition: insertion with >=, i.e. ties -> higher column wins.
 *   - freeNSynapses: stable (permanence, index) order.
 *   - An empty segment is created when a new segment has no source cells.
 *   - Segment duty-cycle pow(1-alpha, age) evaluated by binary
 *     exponentiation in double, rounded to float (deterministic; equals the
 *     correctly rounded powf except in double-rounding corner cases).
 *   - SP boost factors exp(x) (std::exp(float) in updateBoostFactorsGlobal_)
 *     evaluated in double by a fixed operation sequence, rounded to float
 *     (exp_det; equals the correctly rounded expf except in double-rounding
 *     corner cases).
 *   - RDSE: Random::shuffle is the Fisher-Yates form of nupic.core's
 *     Random.hpp (swap(first[0], first[getUInt32(n)]), n decreasing); Python
 *     2's round() rounds halves away from zero.
 *
 * Build: cc -O2 -ffp-contract=off -fopenmp -shared -fPIC (oracle/Makefile).
 */
#include "htm_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_MAXSYN 64

/* =====================================================================
 * nupic::Random  (nupic.core utils/Random.cpp)
 * BSD random() TYPE_3 additive generator, 31 words, sep 3.
 * ===================================================================== */
typedef struct { uint32_t s[31]; int f, r; } rng_t;

static uint32_t rng_raw(rng_t* g) {
    g->s[g->f] += g->s[g->r];
    uint32_t i = (g->s[g->f] >> 1) & 0x7fffffffu; /* chucking least random bit */
    if (++g->f >= 31) { g->f = 0; ++g->r; }
    else if (++g->r >= 31) { g->r = 0; }
    return i;
}

static void rng_seed(rng_t* g, uint64_t seed) {
    int32_t x = (int32_t)(seed % 2147483646ULL + 1ULL);
    g->s[0] = (uint32_t)x;
    for (int i = 1; i < 31; i++) {
        /* state[i] = 16807 * state[i-1] % 2147483647 without overflow */
        int32_t hi = x / 127773, lo = x % 127773;
        x = 16807 * lo - 2836 * hi;
        if (x < 0) x += 2147483647;
        g->s[i] = (uint32_t)x;
    }
    g->f = 3; g->r = 0;
    for (int i = 0; i < 10 * 31; i++) (void)rng_raw(g);
}

/* Random::getUInt32(max): rejection on MAX32 - MAX32 % max, then % max */
static uint32_t rng_u32(rng_t* g, uint32_t max) {
    uint32_t smax = 0xFFFFFFFFu - (0xFFFFFFFFu % max);
    uint32_t v;
    do { v = rng_raw(g); } while (v > smax);
    return v % max;
}

/* Random::getUInt64(max): lo | hi << 32 */
static uint64_t rng_u64(rng_t* g, uint64_t max) {
    uint64_t smax = 0xFFFFFFFFFFFFFFFFull - (0xFFFFFFFFFFFFFFFFull % max);
    uint64_t v;
    do {
        uint64_t lo = rng_raw(g);
        uint64_t hi = rng_raw(g);
        v = lo | (hi << 32);
    } while (v > smax);
    return v % max;
}

/* Random::getReal64(): 48 mantissa bits */
static double rng_real64(rng_t* g) {
    return ldexp((double)rng_u64(g, 1ull << 48), -48);
}

/* Random::sample: Knuth selection sampling, keeps population order */
static void rng_sample(rng_t* g, const uint32_t* pop, uint32_t n, uint32_t* out, uint32_t k) {
    if (k == 0) return;
    uint32_t next = 0;
    for (uint32_t i = 0; i < n; i++) {
        if (rng_u32(g, n - i) < k - next) {
            out[next++] = pop[i];
            if (next == k) break;
        }
    }
}

/* exp(x) in double by a fixed sequence of IEEE operations (range reduction by
 * ln 2 in two parts, degree-13 Taylor polynomial, exact power-of-two
 * scaling), rounded to float: the SP boost factor std::exp((Real)...) of
 * updateBoostFactorsGlobal_.  The HIP engine evaluates the same sequence
 * (sp_dev.h exp_det), so both agree bit for bit. */
static float exp_det(float xf) {
    const double x = (double)xf;
    if (!(x == x)) return xf;
    if (x > 88.8) return INFINITY;
    if (x < -104.0) return 0.0f;
    const double inv_ln2 = 1.4426950408889634, ln2_hi = 6.93147180369123816490e-01,
                 ln2_lo = 1.90821492927058770002e-10;
    const double kd = x * inv_ln2;
    const int k = (int)(kd < 0.0 ? kd - 0.5 : kd + 0.5);
    const double r = (x - (double)k * ln2_hi) - (double)k * ln2_lo;
    static const double inv_fact[14] = {1.0, 1.0, 0.5, 1.0 / 6.0, 1.0 / 24.0, 1.0 / 120.0, 1.0 / 720.0,
                                        1.0 / 5040.0, 1.0 / 40320.0, 1.0 / 362880.0, 1.0 / 3628800.0,
                                        1.0 / 39916800.0, 1.0 / 479001600.0, 1.0 / 6227020800.0};
    double p = inv_fact[13];
    for (int i = 12; i >= 0; i--) p = p * r + inv_fact[i];
    union { double d; uint64_t u; } sc;
    sc.u = (uint64_t)(1023 + k) << 52;
    return (float)(p * sc.d);
}

float orc_exp_det(float x) { return exp_det(x); }

/* =====================================================================
 * ScalarEncoder (nupic.encoders.scalar; Appendix A.1), fields concatenated
 * in sorted name order by MultiEncoder (NetworkUtils.py:77-108).
 * ===================================================================== */
/* returns the first on-bit (bucket index) or -1 for a missing value */
static int enc_first_on_bit(const orc_params* p, int f, double x) {
    if (isnan(x)) return -1; /* SENTINEL_VALUE_FOR_MISSING_DATA -> all zeros */
    const int own = p->field_maxval[f] > p->field_minval[f];
    const double minval = own ? p->field_minval[f] : p->enc_minval;
    const double maxval = own ? p->field_maxval[f] : p->enc_maxval;
    double rangeInternal = maxval - minval;
    double resolution = rangeInternal / (double)(p->enc_n - p->enc_w);
    int halfwidth = (p->enc_w - 1) / 2;
    int padding = halfwidth;
    if (x < minval) {
        if (!p->enc_clip) return -1;
        x = minval;
    }
    if (x > maxval) {
        if (!p->enc_clip) return -1;
        x = maxval;
    }
    int centerbin = (int)(((x - minval) + resolution / 2.0) / resolution) + padding;
    return centerbin - halfwidth;
}

static void enc_encode(const orc_params* p, const double* values, uint8_t* out) {
    int nin = p->n_fields * p->enc_n;
    memset(out, 0, (size_t)nin);
    for (int f = 0; f < p->n_fields; f++) {
        int b = enc_first_on_bit(p, f, values[f]);
        if (b < 0) continue;
        for (int k = 0; k < p->enc_w; k++) out[f * p->enc_n + b + k] = 1;
    }
}

/* =====================================================================
 * RandomDistributedScalarEncoder (NuPIC 1.0.x
 * nupic/encoders/random_distributed_scalar.py), the encoder of the
 * reference's model.yaml parameter set (ML/HTM/params/model.yaml:15-21).
 * State per field: the bucket map (bucket index -> w bit positions, grown on
 * demand one neighbour at a time), the index range [minIndex, maxIndex],
 * the offset (the first value encoded), and the encoder's own
 * nupic::Random(seed).
 * ===================================================================== */
typedef struct {
    int32_t min_idx, max_idx, has_offset, num_tries;
    double offset;
    rng_t rng;
    int32_t* map; /* [ORC_RDSE_BUCKETS][w] */
} rdse_t;

/* __init__ -> _initializeBucketMap(INITIAL_BUCKETS, offset=None): the middle
 * bucket is _permutation(n)[0:w], numpy.arange(n) shuffled by Random.shuffle */
static void rdse_init(const orc_params* p, rdse_t* r, uint64_t seed) {
    const int n = p->enc_n, w = p->enc_w;
    rng_seed(&r->rng, seed);
    r->min_idx = r->max_idx = ORC_RDSE_BUCKETS / 2;
    r->has_offset = 0;
    r->offset = 0.0;
    r->num_tries = 0;
    r->map = (int32_t*)calloc((size_t)ORC_RDSE_BUCKETS * w, sizeof(int32_t));
    uint32_t* perm = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)n);
    for (int i = 0; i < n; i++) perm[i] = (uint32_t)i;
    uint32_t left = (uint32_t)n;
    for (int i = 0; i < n; i++, left--) {
        const uint32_t j = rng_u32(&r->rng, left);
        const uint32_t t = perm[i];
        perm[i] = perm[i + j];
        perm[i + j] = t;
    }
    for (int k = 0; k < w; k++) r->map[(size_t)r->min_idx * w + k] = (int32_t)perm[k];
    free(perm);
}

static void rdse_copy(const orc_params* p, rdse_t* d, const rdse_t* s) {
    *d = *s;
    const size_t nb = (size_t)ORC_RDSE_BUCKETS * p->enc_w * sizeof(int32_t);
    d->map = (int32_t*)malloc(nb);
    memcpy(d->map, s->map, nb);
}

/* Python 2 round(): halves away from zero (exact: v - trunc(v) is exact) */
static double round_half_away(double v) {
    const double t = trunc(v);
    const double fr = v - t;
    if (fr >= 0.5) return t + 1.0;
    if (fr <= -0.5) return t - 1.0;
    return t;
}

/* getBucketIndices(x): maxBuckets/2 + int(round((x - offset) / resolution)),
 * clipped to [0, maxBuckets); the first value seen becomes the offset; a
 * missing value (NaN) is bucket None (-1) and does not set the offset */
static int rdse_bucket(const orc_params* p, rdse_t* r, double x) {
    if (isnan(x)) return -1;
    if (!r->has_offset) {
        r->offset = x;
        r->has_offset = 1;
    }
    const double q = round_half_away((x - r->offset) / p->rdse_resolution);
    double b = (double)(ORC_RDSE_BUCKETS / 2) + q;
    if (b < 0.0) b = 0.0;
    if (b > (double)(ORC_RDSE_BUCKETS - 1)) b = (double)(ORC_RDSE_BUCKETS - 1);
    return (int)b;
}

/* _overlapOK(i, j, overlap) with _maxOverlap = 2 */
static int rdse_overlap_ok(int w, int i, int j, int overlap) {
    const int d = i > j ? i - j : j - i;
    return d < w ? overlap == w - d : overlap <= 2;
}

/* _newRepresentationOK(newRep, newIndex): running overlap of newRep with every
 * existing bucket, minIndex .. maxIndex (adjacent buckets differ in one
 * position: (i-1) % w below the middle, i % w above) */
static int rdse_rep_ok(const orc_params* p, const rdse_t* r, const int32_t* rep, const uint8_t* bin, int new_idx) {
    const int w = p->enc_w, mid = ORC_RDSE_BUCKETS / 2;
    (void)rep;
    const int32_t* m = r->map;
    int run = 0;
    for (int k = 0; k < w; k++) run += bin[m[(size_t)r->min_idx * w + k]];
    if (!rdse_overlap_ok(w, r->min_idx, new_idx, run)) return 0;
    for (int i = r->min_idx + 1; i <= mid; i++) {
        const int nb = (i - 1) % w;
        run -= bin[m[(size_t)(i - 1) * w + nb]];
        run += bin[m[(size_t)i * w + nb]];
        if (!rdse_overlap_ok(w, i, new_idx, run)) return 0;
    }
    for (int i = mid + 1; i <= r->max_idx; i++) {
        const int nb = i % w;
        run -= bin[m[(size_t)(i - 1) * w + nb]];
        run += bin[m[(size_t)i * w + nb]];
        if (!rdse_overlap_ok(w, i, new_idx, run)) return 0;
    }
    return 1;
}

/* _newRepresentation(index, newIndex): the neighbour's bits with position
 * newIndex % w redrawn (getUInt32(n)) until the bit is new to the neighbour
 * and the overlap rules hold against every existing bucket */
static void rdse_new_rep(const orc_params* p, rdse_t* r, int from, int new_idx) {
    const int n = p->enc_n, w = p->enc_w;
    int32_t* rep = r->map + (size_t)new_idx * w;
    const int32_t* nbr = r->map + (size_t)from * w;
    memcpy(rep, nbr, sizeof(int32_t) * (size_t)w);
    const int ri = new_idx % w;
    uint8_t* bin = (uint8_t*)malloc((size_t)n);
    for (;;) {
        const int32_t bit = (int32_t)rng_u32(&r->rng, (uint32_t)n);
        rep[ri] = bit;
        int in_nbr = 0;
        for (int k = 0; k < w; k++) in_nbr |= nbr[k] == bit;
        if (!in_nbr) {
            memset(bin, 0, (size_t)n);
            for (int k = 0; k < w; k++) bin[rep[k]] = 1;
            if (rdse_rep_ok(p, r, rep, bin, new_idx)) break;
        }
        r->num_tries++;
    }
    free(bin);
}

/* mapBucketIndexToNonZeroBits(index): _createBucket grows the map one
 * neighbour at a time towards the index (the recursion's order) */
static const int32_t* rdse_bits(const orc_params* p, rdse_t* r, int idx) {
    if (idx < r->min_idx) {
        for (int i = r->min_idx - 1; i >= idx; i--) {
            rdse_new_rep(p, r, r->min_idx, i);
            r->min_idx = i;
        }
    } else if (idx > r->max_idx) {
        for (int i = r->max_idx + 1; i <= idx; i++) {
            rdse_new_rep(p, r, r->max_idx, i);
            r->max_idx = i;
        }
    }
    return r->map + (size_t)idx * p->enc_w;
}

/* =====================================================================
 * SpatialPooler (nupic.core algorithms/SpatialPooler.cpp; Appendix A.2)
 * Dense restatement: perm[c][i] float32, potential/connected 0/1.
 * ===================================================================== */
typedef struct {
    int nin, ncol;
    uint8_t* potential;
    float* perm;
    uint8_t* connected;
    int32_t* conn_count;
    float* overlap_dc;
    float* active_dc;
    float* min_overlap_dc;
    float* boost;
    float* tie_breaker;
    int32_t* overlaps;
    float* boosted;
    int64_t iter, iter_learn;
    uint32_t inhibition_radius;
    float perm_trim, perm_below_stim_inc, perm_min, perm_max;
    int32_t* active_sorted; /* ascending */
    int n_active;
    uint8_t* active_dense;
    rng_t rng;
    float* scratch; /* nin */
} sp_t;

static const float PERMANENCE_EPSILON = 0.000001f;

static void sp_clip(const sp_t* sp, float* perm, int trim) {
    float minVal = trim ? sp->perm_trim : sp->perm_min;
    for (int i = 0; i < sp->nin; i++) {
        float e = perm[i];
        e = e > sp->perm_max ? sp->perm_max : e;
        e = e < minVal ? sp->perm_min : e;
        perm[i] = e;
    }
}

/* updatePermanencesForColumn_(perm, column, raisePerm) */
static void sp_update_perm_for_column(const orc_params* p, sp_t* sp, float* perm, int c, int raise) {
    const uint8_t* pot = sp->potential + (size_t)c * sp->nin;
    if (raise) {
        /* raisePermanencesToThreshold_: clip (no trim), then bump until
         * numConnected >= stimulusThreshold (never loops at threshold 0) */
        sp_clip(sp, perm, 0);
        for (;;) {
            int nconn = 0;
            for (int i = 0; i < sp->nin; i++)
                if (perm[i] > p->sp_perm_connected - PERMANENCE_EPSILON) nconn++;
            if (nconn >= p->sp_stimulus_threshold) break;
            for (int i = 0; i < sp->nin; i++)
                if (pot[i]) perm[i] += sp->perm_below_stim_inc;
        }
    }
    int nconn = 0;
    uint8_t* conn = sp->connected + (size_t)c * sp->nin;
    float thr = p->sp_perm_connected - PERMANENCE_EPSILON;
    for (int i = 0; i < sp->nin; i++) {
        conn[i] = perm[i] >= thr ? 1 : 0;
        nconn += conn[i];
    }
    sp_clip(sp, perm, 1);
    memcpy(sp->perm + (size_t)c * sp->nin, perm, sizeof(float) * (size_t)sp->nin);
    sp->conn_count[c] = nconn;
}

static float sp_init_perm_connected(const orc_params* p, sp_t* sp) {
    float span = sp->perm_max - p->sp_perm_connected;
    float q;
    if (p->variant & ORC_VAR_SP_INIT_DOUBLE)
        q = (float)((double)p->sp_perm_connected + (double)span * rng_real64(&sp->rng));
    else
        q = p->sp_perm_connected + (float)((double)span * rng_real64(&sp->rng));
    q = (float)((double)(int32_t)(q * 100000.0f) / 100000.0);
    return q;
}

static float sp_init_perm_nonconnected(const orc_params* p, sp_t* sp) {
    float q = p->sp_perm_connected * (float)rng_real64(&sp->rng);
    q = (float)((double)(int32_t)(q * 100000.0f) / 100000.0);
    return q;
}

static float sp_density(const orc_params* p, const sp_t* sp) {
    /* inhibitColumns_: area = min((2r+1)^1, ncol), density = min(k/area, 0.5) */
    uint32_t area = (uint32_t)powf((float)(2 * sp->inhibition_radius + 1), 1.0f);
    if (area > (uint32_t)sp->ncol) area = (uint32_t)sp->ncol;
    float density = (float)p->sp_num_active / (float)area;
    if (density > 0.5f) density = 0.5f;
    return density;
}

static void sp_init(const orc_params* p, sp_t* sp) {
    int nin = p->sdr_bits > 0 ? p->sdr_bits : p->n_fields * p->enc_n, ncol = p->sp_columns;
    sp->nin = nin;
    sp->ncol = ncol;
    sp->potential = (uint8_t*)calloc((size_t)ncol * nin, 1);
    sp->perm = (float*)calloc((size_t)ncol * nin, sizeof(float));
    sp->connected = (uint8_t*)calloc((size_t)ncol * nin, 1);
    sp->conn_count = (int32_t*)calloc((size_t)ncol, sizeof(int32_t));
    sp->overlap_dc = (float*)calloc((size_t)ncol, sizeof(float));
    sp->active_dc = (float*)calloc((size_t)ncol, sizeof(float));
    sp->min_overlap_dc = (float*)calloc((size_t)ncol, sizeof(float));
    sp->boost = (float*)malloc(sizeof(float) * (size_t)ncol);
    sp->tie_breaker = (float*)malloc(sizeof(float) * (size_t)ncol);
    sp->overlaps = (int32_t*)calloc((size_t)ncol, sizeof(int32_t));
    sp->boosted = (float*)calloc((size_t)ncol, sizeof(float));
    sp->active_sorted = (int32_t*)calloc((size_t)ncol, sizeof(int32_t));
    sp->active_dense = (uint8_t*)calloc((size_t)ncol, 1);
    sp->scratch = (float*)calloc((size_t)nin, sizeof(float));
    for (int c = 0; c < ncol; c++) sp->boost[c] = 1.0f;
    sp->iter = sp->iter_learn = 0;
    sp->n_active = 0;
    sp->perm_trim = (float)((double)p->sp_perm_active_inc / 2.0);
    sp->perm_below_stim_inc = (float)((double)p->sp_perm_connected / 10.0);
    sp->perm_min = 0.0f;
    sp->perm_max = 1.0f;
    rng_seed(&sp->rng, p->sp_seed);

    /* potentialRadius = inputWidth (SPRegion), capped at numInputs */
    uint32_t radius = (uint32_t)nin;
    for (int c = 0; c < ncol; c++)
        sp->tie_breaker[c] = (p->variant & ORC_VAR_SP_NO_TIEBREAKER) ? 0.0f : (float)(0.01 * rng_real64(&sp->rng));

    uint32_t* pop = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)nin);
    uint32_t* sel = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)nin);
    float* perm = (float*)malloc(sizeof(float) * (size_t)nin);
    for (int c = 0; c < ncol; c++) {
        /* mapColumn_: centre input = floor((c + 0.5) * (nin / ncol)) */
        float ratio = (float)nin / (float)ncol;
        float coord = (float)(((double)c + 0.5) * (double)ratio);
        int32_t center = (int32_t)floorf(coord);
        /* WrappingNeighborhood(center, radius, [nin]) iteration order */
        uint32_t count = 2 * radius + 1;
        if (count > (uint32_t)nin) count = (uint32_t)nin;
        for (uint32_t k = 0; k < count; k++) {
            int32_t coordk = (center - (int32_t)radius + (int32_t)k) % nin;
            if (coordk < 0) coordk += nin;
            if (p->variant & ORC_VAR_SP_POOL_ASCEND) coordk = (int32_t)k;
            pop[k] = (uint32_t)coordk;
        }
        uint32_t numPotential = (uint32_t)roundf((float)count * p->sp_potential_pct);
        rng_sample(&sp->rng, pop, count, sel, numPotential);
        uint8_t* pot = sp->potential + (size_t)c * nin;
        for (uint32_t k = 0; k < numPotential; k++) pot[sel[k]] = 1;
        /* initPermanence_(potential, initConnectedPct = 0.5) */
        for (int i = 0; i < nin; i++) {
            perm[i] = 0.0f;
            if (!pot[i]) continue;
            if (rng_real64(&sp->rng) <= 0.5f)
                perm[i] = sp_init_perm_connected(p, sp);
            else
                perm[i] = sp_init_perm_nonconnected(p, sp);
            perm[i] = perm[i] < sp->perm_trim ? 0.0f : perm[i];
        }
        sp_update_perm_for_column(p, sp, perm, c, 1);
    }
    free(pop);
    free(sel);
    free(perm);
    /* updateInhibitionRadius_: global inhibition -> max(columnDimensions) */
    sp->inhibition_radius = (uint32_t)ncol;
}

static void sp_free(sp_t* sp) {
    free(sp->potential); free(sp->perm); free(sp->connected); free(sp->conn_count);
    free(sp->overlap_dc); free(sp->active_dc); free(sp->min_overlap_dc);
    free(sp->boost); free(sp->tie_breaker); free(sp->overlaps); free(sp->boosted);
    free(sp->active_sorted); free(sp->active_dense); free(sp->scratch);
}

static void sp_copy(sp_t* d, const sp_t* s) {
    size_t ci = (size_t)s->ncol * s->nin, nc = (size_t)s->ncol;
    *d = *s;
    d->potential = (uint8_t*)malloc(ci); memcpy(d->potential, s->potential, ci);
    d->perm = (float*)malloc(ci * 4); memcpy(d->perm, s->perm, ci * 4);
    d->connected = (uint8_t*)malloc(ci); memcpy(d->connected, s->connected, ci);
#define DUP(f, T) d->f = (T*)malloc(nc * sizeof(T)); memcpy(d->f, s->f, nc * sizeof(T));
    DUP(conn_count, int32_t) DUP(overlap_dc, float) DUP(active_dc, float)
    DUP(min_overlap_dc, float) DUP(boost, float) DUP(tie_breaker, float)
    DUP(overlaps, int32_t) DUP(boosted, float) DUP(active_sorted, int32_t)
    DUP(active_dense, uint8_t)
#undef DUP
    d->scratch = (float*)calloc((size_t)s->nin, sizeof(float));
}

/* inhibitColumnsGlobal_: insertion list, ">=" so ties go to the later
 * (higher) column index; returns winners ordered by (overlap desc, idx desc) */
static int sp_inhibit_global(const orc_params* p, const sp_t* sp, const float* ov, int32_t* winners) {
    float density = sp_density(p, sp);
    uint32_t numDesired = (uint32_t)(density * (float)sp->ncol);
    int n = 0;
    for (int i = 0; i < sp->ncol; i++) {
        if (ov[i] < (float)p->sp_stimulus_threshold) continue;
        int low = (p->variant & ORC_VAR_SP_TIE_LOW) != 0;
        if ((uint32_t)n < numDesired || ov[i] > ov[winners[n - 1]] || (!low && ov[i] == ov[winners[n - 1]])) {
            int pos = 0;
            if (low) while (pos < n && !(ov[i] > ov[winners[pos]])) pos++;
            else while (pos < n && !(ov[i] >= ov[winners[pos]])) pos++;
            memmove(winners + pos + 1, winners + pos, sizeof(int32_t) * (size_t)(n - pos));
            winners[pos] = i;
            n++;
            if ((uint32_t)n > numDesired) n--;
        }
    }
    return n;
}

static int cmp_i32(const void* a, const void* b) {
    int32_t x = *(const int32_t*)a, y = *(const int32_t*)b;
    return (x > y) - (x < y);
}

static void sp_compute(const orc_params* p, sp_t* sp, const uint8_t* input, int learn) {
    int nin = sp->nin, ncol = sp->ncol;
    /* updateBookeepingVars_ */
    sp->iter++;
    if (learn) sp->iter_learn++;
    /* calculateOverlap_ */
    for (int c = 0; c < ncol; c++) {
        const uint8_t* conn = sp->connected + (size_t)c * nin;
        int32_t o = 0;
        for (int i = 0; i < nin; i++) o += (conn[i] & input[i]);
        sp->overlaps[c] = o;
    }
    /* boostOverlaps_ when learning */
    for (int c = 0; c < ncol; c++)
        sp->boosted[c] = learn ? sp->boost[c] * (float)sp->overlaps[c] : (float)sp->overlaps[c];
    int32_t* winners = (int32_t*)malloc(sizeof(int32_t) * (size_t)(ncol + 1));
    int nw = sp_inhibit_global(p, sp, sp->boosted, winners);
    memset(sp->active_dense, 0, (size_t)ncol);
    for (int k = 0; k < nw; k++) sp->active_dense[winners[k]] = 1;
    if (learn) {
        /* adaptSynapses_ */
        float* permChanges = sp->scratch;
        for (int i = 0; i < nin; i++)
            permChanges[i] = input[i] > 0 ? p->sp_perm_active_inc : -1 * p->sp_perm_inactive_dec;
        float* perm = (float*)malloc(sizeof(float) * (size_t)nin);
        for (int k = 0; k < nw; k++) {
            int c = winners[k];
            const uint8_t* pot = sp->potential + (size_t)c * nin;
            memcpy(perm, sp->perm + (size_t)c * nin, sizeof(float) * (size_t)nin);
            for (int i = 0; i < nin; i++)
                if (pot[i] > 0) perm[i] += permChanges[i];
            sp_update_perm_for_column(p, sp, perm, c, 1);
        }
        /* updateDutyCycles_ */
        uint32_t period = (uint32_t)p->sp_duty_cycle_period > (uint64_t)sp->iter
                              ? (uint32_t)sp->iter : (uint32_t)p->sp_duty_cycle_period;
        for (int c = 0; c < ncol; c++) {
            uint32_t ov = sp->overlaps[c] > 0 ? 1u : 0u;
            uint32_t ac = sp->active_dense[c] > 0 ? 1u : 0u;
            sp->overlap_dc[c] = (sp->overlap_dc[c] * (float)(period - 1) + (float)ov) / (float)period;
            sp->active_dc[c] = (sp->active_dc[c] * (float)(period - 1) + (float)ac) / (float)period;
        }
        /* bumpUpWeakColumns_ */
        for (int c = 0; c < ncol; c++) {
            if (sp->overlap_dc[c] >= sp->min_overlap_dc[c]) continue;
            const uint8_t* pot = sp->potential + (size_t)c * nin;
            memcpy(perm, sp->perm + (size_t)c * nin, sizeof(float) * (size_t)nin);
            for (int i = 0; i < nin; i++)
                if (pot[i] > 0) perm[i] += sp->perm_below_stim_inc;
            sp_update_perm_for_column(p, sp, perm, c, 0);
        }
        free(perm);
        /* updateBoostFactorsGlobal_ */
        float target = sp_density(p, sp);
        for (int c = 0; c < ncol; c++)
            sp->boost[c] = exp_det((target - sp->active_dc[c]) * p->sp_boost_strength);
        /* isUpdateRound_: updateInhibitionRadius_ (global: constant) and
         * updateMinDutyCyclesGlobal_ */
        if (sp->iter % p->sp_update_period == 0) {
            sp->inhibition_radius = (uint32_t)ncol;
            float mx = sp->overlap_dc[0];
            for (int c = 1; c < ncol; c++) if (sp->overlap_dc[c] > mx) mx = sp->overlap_dc[c];
            for (int c = 0; c < ncol; c++) sp->min_overlap_dc[c] = p->sp_min_pct_overlap_dc * mx;
        }
    }
    memcpy(sp->active_sorted, winners, sizeof(int32_t) * (size_t)nw);
    qsort(sp->active_sorted, (size_t)nw, sizeof(int32_t), cmp_i32);
    sp->n_active = nw;
    free(winners);
}

/* =====================================================================
 * BacktrackingTM (nupic.algorithms.backtracking_tm[_cpp] / Cells4;
 * Appendix A.3).  Cells are (column, index) pairs flattened to
 * cell = column * cellsPerColumn + index; synapse sources likewise.
 * ===================================================================== */
typedef struct { uint32_t src; float perm; } syn_t;

typedef struct {
    int is_seq;
    uint32_t pos_act, tot_act, last_active_it;
    float last_dc;
    uint32_t last_dc_it;
    int nsyn, cap;
    syn_t* syn;
} seg_t;

typedef struct { int n, cap; seg_t** s; } cell_t;

typedef struct {
    int col, cell;
    seg_t* seg;      /* NULL: create a new segment */
    int n_idx;       /* indices of existing synapses to reinforce */
    int32_t idx[ORC_MAXSYN];
    int n_new;       /* new synapse sources (flat cell) */
    uint32_t newsrc[ORC_MAXSYN];
    int seq_flag;
} segupd_t;

typedef struct { uint32_t date; segupd_t u; } dupd_t;
typedef struct { int col, cell, n, cap; dupd_t* it; } updlist_t;

typedef struct { int n; int32_t* cols; } pattern_t;

typedef struct {
    int ncol, K, ncells;
    cell_t* cells;
    uint8_t *infA_t, *infA_t1, *infA_backup, *infA_cand;
    uint8_t *infP_t, *infP_t1, *infP_backup, *infP_cand;
    uint8_t *lrnA_t, *lrnA_t1, *lrnP_t, *lrnP_t1;
    float *cellConf_t, *cellConf_t1, *cellConf_cand;
    float *colConf_t, *colConf_t1, *colConf_cand;
    pattern_t* inf_pat; int n_inf_pat;
    pattern_t* lrn_pat; int n_lrn_pat;
    updlist_t* upd; int n_upd, cap_upd;
    uint32_t lrn_iter, iter;
    int pam_counter, learned_seq_length, reset_called;
    int have_avg_density;
    double avg_input_density, avg_learned_seq_length;
    rng_t rng;
    uint8_t* colmask; /* scratch: active-column membership */
    uint32_t* cand;   /* scratch: candidate cells */
    uint32_t* cand2;
    int64_t stats[5]; /* inferPhase2 calls, inferBacktracks, lrnPhase2 calls, lrnBacktracks,
                         inferPhase2 calls on the critical path if backtrack start offsets ran in parallel */
    int bt_crit;      /* scratch: the last inferBacktrack's critical-path phase-2 calls */
    uint32_t variant;
} tm_t;

static const uint32_t DC_TIERS[9] = {0, 100, 320, 1000, 3200, 10000, 32000, 100000, 320000};
static const float DC_ALPHAS[9] = {0.0f, 0.0032f, 0.0010f, 0.00032f, 0.00010f,
                                   0.000032f, 0.00001f, 0.0000032f, 0.0000010f};

/* pow(b, e) for integer e >= 0 by binary exponentiation in double */
static float pow_det(float b, uint32_t e) {
    double r = 1.0, x = (double)b;
    while (e) {
        if (e & 1u) r *= x;
        x *= x;
        e >>= 1;
    }
    return (float)r;
}

/* Segment::dutyCycle(iteration, active, readOnly) */
static float seg_duty_cycle(seg_t* s, uint32_t it, int active, int read_only) {
    float dc;
    if (it <= DC_TIERS[1]) {
        dc = (float)s->pos_act / (float)it;
        if (!read_only) { s->last_dc_it = it; s->last_dc = dc; }
        return dc;
    }
    uint32_t age = it - s->last_dc_it;
    if (age == 0 && !active) return s->last_dc;
    float alpha = 0.0f;
    for (int t = 8; t > 0; t--) {
        if (it > DC_TIERS[t]) { alpha = DC_ALPHAS[t]; break; }
    }
    dc = pow_det((float)(1.0 - (double)alpha), age) * s->last_dc;
    if (active) dc += alpha;
    if (!read_only) { s->last_dc_it = it; s->last_dc = dc; }
    return dc;
}

static seg_t* seg_new(const orc_params* p, uint32_t lrn_iter, int is_seq) {
    seg_t* s = (seg_t*)calloc(1, sizeof(seg_t));
    s->is_seq = is_seq;
    s->pos_act = 1;
    s->tot_act = 1;
    s->last_active_it = lrn_iter;
    s->last_dc = (float)(1.0 / (double)lrn_iter);
    s->last_dc_it = lrn_iter;
    s->cap = p->tm_max_syn_per_seg > 0 ? p->tm_max_syn_per_seg + ORC_MAXSYN : ORC_MAXSYN;
    s->syn = (syn_t*)malloc(sizeof(syn_t) * (size_t)s->cap);
    return s;
}

static void seg_free(seg_t* s) { free(s->syn); free(s); }

static void seg_add_syn(seg_t* s, uint32_t src, float perm) {
    if (s->nsyn == s->cap) {
        s->cap *= 2;
        s->syn = (syn_t*)realloc(s->syn, sizeof(syn_t) * (size_t)s->cap);
    }
    s->syn[s->nsyn].src = src;
    s->syn[s->nsyn].perm = perm;
    s->nsyn++;
}

static void seg_remove_idx(seg_t* s, int k) {
    memmove(s->syn + k, s->syn + k + 1, sizeof(syn_t) * (size_t)(s->nsyn - k - 1));
    s->nsyn--;
}

static void cell_append(cell_t* c, seg_t* s) {
    if (c->n == c->cap) {
        c->cap = c->cap ? 2 * c->cap : 4;
        c->s = (seg_t**)realloc(c->s, sizeof(seg_t*) * (size_t)c->cap);
    }
    c->s[c->n++] = s;
}

static void cell_remove(cell_t* c, seg_t* s) {
    for (int k = 0; k < c->n; k++) {
        if (c->s[k] == s) {
            memmove(c->s + k, c->s + k + 1, sizeof(seg_t*) * (size_t)(c->n - k - 1));
            c->n--;
            return;
        }
    }
}

/* _getSegmentActivityLevel(s, activeState, connectedSynapsesOnly=False) */
static int seg_activity(const seg_t* s, const uint8_t* state) {
    int n = 0;
    for (int k = 0; k < s->nsyn; k++) n += state[s->syn[k].src] ? 1 : 0;
    return n;
}

/* _isSegmentActive: connected (perm >= connectedPerm) synapses on active cells */
static int seg_is_active(const orc_params* p, const seg_t* s, const uint8_t* state) {
    int n = 0;
    for (int k = 0; k < s->nsyn; k++)
        if (state[s->syn[k].src] && s->syn[k].perm >= p->tm_connected_perm) n++;
    return n >= p->tm_activation_threshold;
}

static void tm_init(const orc_params* p, tm_t* tm) {
    memset(tm, 0, sizeof(*tm));
    tm->ncol = p->sp_columns;
    tm->K = p->tm_cells_per_col;
    tm->ncells = tm->ncol * tm->K;
    size_t nc = (size_t)tm->ncells;
    tm->cells = (cell_t*)calloc(nc, sizeof(cell_t));
#define AL8(f) tm->f = (uint8_t*)calloc(nc, 1);
    AL8(infA_t) AL8(infA_t1) AL8(infA_backup) AL8(infA_cand)
    AL8(infP_t) AL8(infP_t1) AL8(infP_backup) AL8(infP_cand)
    AL8(lrnA_t) AL8(lrnA_t1) AL8(lrnP_t) AL8(lrnP_t1)
#undef AL8
    tm->cellConf_t = (float*)calloc(nc, 4);
    tm->cellConf_t1 = (float*)calloc(nc, 4);
    tm->cellConf_cand = (float*)calloc(nc, 4);
    tm->colConf_t = (float*)calloc((size_t)tm->ncol, 4);
    tm->colConf_t1 = (float*)calloc((size_t)tm->ncol, 4);
    tm->colConf_cand = (float*)calloc((size_t)tm->ncol, 4);
    tm->inf_pat = (pattern_t*)calloc((size_t)p->tm_max_inf_backtrack + 2, sizeof(pattern_t));
    tm->lrn_pat = (pattern_t*)calloc((size_t)p->tm_max_lrn_backtrack + 2, sizeof(pattern_t));
    for (int k = 0; k < p->tm_max_inf_backtrack + 2; k++)
        tm->inf_pat[k].cols = (int32_t*)calloc((size_t)tm->ncol, 4);
    for (int k = 0; k < p->tm_max_lrn_backtrack + 2; k++)
        tm->lrn_pat[k].cols = (int32_t*)calloc((size_t)tm->ncol, 4);
    tm->pam_counter = p->tm_pam_length;
    tm->variant = p->variant;
    tm->colmask = (uint8_t*)calloc((size_t)tm->ncol, 1);
    tm->cand = (uint32_t*)calloc(nc, 4);
    tm->cand2 = (uint32_t*)calloc(nc, 4);
    rng_seed(&tm->rng, p->tm_seed);
}

static void tm_free(const orc_params* p, tm_t* tm) {
    for (int c = 0; c < tm->ncells; c++) {
        for (int k = 0; k < tm->cells[c].n; k++) seg_free(tm->cells[c].s[k]);
        free(tm->cells[c].s);
    }
    free(tm->cells);
    free(tm->infA_t); free(tm->infA_t1); free(tm->infA_backup); free(tm->infA_cand);
    free(tm->infP_t); free(tm->infP_t1); free(tm->infP_backup); free(tm->infP_cand);
    free(tm->lrnA_t); free(tm->lrnA_t1); free(tm->lrnP_t); free(tm->lrnP_t1);
    free(tm->cellConf_t); free(tm->cellConf_t1); free(tm->cellConf_cand);
    free(tm->colConf_t); free(tm->colConf_t1); free(tm->colConf_cand);
    for (int k = 0; k < p->tm_max_inf_backtrack + 2; k++) free(tm->inf_pat[k].cols);
    for (int k = 0; k < p->tm_max_lrn_backtrack + 2; k++) free(tm->lrn_pat[k].cols);
    free(tm->inf_pat); free(tm->lrn_pat);
    for (int k = 0; k < tm->n_upd; k++) free(tm->upd[k].it);
    free(tm->upd);
    free(tm->colmask); free(tm->cand); free(tm->cand2);
}

static void tm_copy(const orc_params* p, tm_t* d, const tm_t* s) {
    size_t nc = (size_t)s->ncells, ncol = (size_t)s->ncol;
    tm_init(p, d);
    /* segments: deep copy; remember old->new pointers for the update queue */
    int nseg = 0;
    for (size_t c = 0; c < nc; c++) nseg += s->cells[c].n;
    seg_t** from = (seg_t**)malloc(sizeof(seg_t*) * (size_t)(nseg + 1));
    seg_t** to = (seg_t**)malloc(sizeof(seg_t*) * (size_t)(nseg + 1));
    int k = 0;
    for (size_t c = 0; c < nc; c++) {
        for (int j = 0; j < s->cells[c].n; j++) {
            seg_t* os = s->cells[c].s[j];
            seg_t* ns = (seg_t*)malloc(sizeof(seg_t));
            *ns = *os;
            ns->syn = (syn_t*)malloc(sizeof(syn_t) * (size_t)os->cap);
            memcpy(ns->syn, os->syn, sizeof(syn_t) * (size_t)os->nsyn);
            cell_append(&d->cells[c], ns);
            from[k] = os;
            to[k] = ns;
            k++;
        }
    }
#define CP8(f) memcpy(d->f, s->f, nc);
    CP8(infA_t) CP8(infA_t1) CP8(infA_backup) CP8(infA_cand)
    CP8(infP_t) CP8(infP_t1) CP8(infP_backup) CP8(infP_cand)
    CP8(lrnA_t) CP8(lrnA_t1) CP8(lrnP_t) CP8(lrnP_t1)
#undef CP8
    memcpy(d->cellConf_t, s->cellConf_t, nc * 4);
    memcpy(d->cellConf_t1, s->cellConf_t1, nc * 4);
    memcpy(d->cellConf_cand, s->cellConf_cand, nc * 4);
    memcpy(d->colConf_t, s->colConf_t, ncol * 4);
    memcpy(d->colConf_t1, s->colConf_t1, ncol * 4);
    memcpy(d->colConf_cand, s->colConf_cand, ncol * 4);
    d->n_inf_pat = s->n_inf_pat;
    for (int i = 0; i < s->n_inf_pat; i++) {
        d->inf_pat[i].n = s->inf_pat[i].n;
        memcpy(d->inf_pat[i].cols, s->inf_pat[i].cols, 4 * (size_t)s->inf_pat[i].n);
    }
    d->n_lrn_pat = s->n_lrn_pat;
    for (int i = 0; i < s->n_lrn_pat; i++) {
        d->lrn_pat[i].n = s->lrn_pat[i].n;
        memcpy(d->lrn_pat[i].cols, s->lrn_pat[i].cols, 4 * (size_t)s->lrn_pat[i].n);
    }
    for (int i = 0; i < s->n_upd; i++) {
        const updlist_t* ul = &s->upd[i];
        if (d->n_upd == d->cap_upd) {
            d->cap_upd = d->cap_upd ? 2 * d->cap_upd : 16;
            d->upd = (updlist_t*)realloc(d->upd, sizeof(updlist_t) * (size_t)d->cap_upd);
        }
        updlist_t* nl = &d->upd[d->n_upd++];
        *nl = *ul;
        nl->it = (dupd_t*)malloc(sizeof(dupd_t) * (size_t)(ul->cap ? ul->cap : 1));
        memcpy(nl->it, ul->it, sizeof(dupd_t) * (size_t)ul->n);
        for (int j = 0; j < nl->n; j++) {
            for (int q = 0; q < k; q++)
                if (nl->it[j].u.seg == from[q]) { nl->it[j].u.seg = to[q]; break; }
        }
    }
    free(from);
    free(to);
    d->lrn_iter = s->lrn_iter;
    d->iter = s->iter;
    d->variant = s->variant;
    d->pam_counter = s->pam_counter;
    d->learned_seq_length = s->learned_seq_length;
    d->reset_called = s->reset_called;
    d->have_avg_density = s->have_avg_density;
    d->avg_input_density = s->avg_input_density;
    d->avg_learned_seq_length = s->avg_learned_seq_length;
    d->rng = s->rng;
}

/* ---------------- segment update queue (dict keyed by (c,i)) ---------------- */
static void tm_remove_updlist(tm_t* tm, int k) {
    free(tm->upd[k].it);
    memmove(tm->upd + k, tm->upd + k + 1, sizeof(updlist_t) * (size_t)(tm->n_upd - k - 1));
    tm->n_upd--;
}

/* _addToSegmentUpdates */
static void tm_add_to_updates(tm_t* tm, int c, int i, const segupd_t* u) {
    if (u->n_idx + u->n_new == 0) return;
    updlist_t* l = NULL;
    for (int k = 0; k < tm->n_upd; k++)
        if (tm->upd[k].col == c && tm->upd[k].cell == i) { l = &tm->upd[k]; break; }
    if (!l) {
        if (tm->n_upd == tm->cap_upd) {
            tm->cap_upd = tm->cap_upd ? 2 * tm->cap_upd : 16;
            tm->upd = (updlist_t*)realloc(tm->upd, sizeof(updlist_t) * (size_t)tm->cap_upd);
        }
        l = &tm->upd[tm->n_upd++];
        l->col = c; l->cell = i; l->n = 0; l->cap = 0; l->it = NULL;
    }
    if (l->n == l->cap) {
        l->cap = l->cap ? 2 * l->cap : 2;
        l->it = (dupd_t*)realloc(l->it, sizeof(dupd_t) * (size_t)l->cap);
    }
    l->it[l->n].date = tm->lrn_iter;
    l->it[l->n].u = *u;
    l->n++;
}

static void tm_clear_updates(tm_t* tm) {
    for (int k = 0; k < tm->n_upd; k++) free(tm->upd[k].it);
    tm->n_upd = 0;
}

/* _cleanUpdatesList(col, cellIdx, seg) */
static void tm_clean_updates_list(tm_t* tm, int col, int cell, const seg_t* seg) {
    for (int k = 0; k < tm->n_upd; k++) {
        updlist_t* l = &tm->upd[k];
        if (l->col != col || l->cell != cell) continue;
        for (int j = 0; j < l->n;) {
            if (l->it[j].u.seg == seg) {
                memmove(l->it + j, l->it + j + 1, sizeof(dupd_t) * (size_t)(l->n - j - 1));
                l->n--;
            } else {
                j++;
            }
        }
    }
}

/* _trimSegmentsInCell(colIdx, cellIdx, [seg], minPermanence, minNumSyns) */
static void tm_trim_segment(tm_t* tm, int c, int i, seg_t* seg, float min_perm, int min_syns) {
    int ndel = 0;
    for (int k = 0; k < seg->nsyn; k++) ndel += seg->syn[k].perm < min_perm ? 1 : 0;
    int del_seg = 0;
    if (ndel == seg->nsyn) {
        del_seg = 1;
    } else {
        for (int k = 0; k < seg->nsyn;) {
            if (seg->syn[k].perm < min_perm) seg_remove_idx(seg, k);
            else k++;
        }
        if (seg->nsyn < min_syns) del_seg = 1;
    }
    if (del_seg) {
        tm_clean_updates_list(tm, c, i, seg);
        cell_remove(&tm->cells[c * tm->K + i], seg);
        seg_free(seg);
    }
}

/* _chooseCellsToLearnFrom(c, i, s, n, activeState): appends to u->newsrc */
static void tm_choose_cells_to_learn_from(tm_t* tm, const seg_t* s, int n, const uint8_t* state, segupd_t* u) {
    if (n <= 0) return;
    int nc = 0;
    for (int k = 0; k < tm->ncells; k++) {
        if (!state[k]) continue;
        int dup = 0;
        if (s) {
            for (int j = 0; j < s->nsyn; j++)
                if (s->syn[j].src == (uint32_t)k) { dup = 1; break; }
        }
        if (!dup) tm->cand[nc++] = (uint32_t)k;
    }
    if (nc == 0) return;
    if (nc <= n) {
        for (int k = 0; k < nc; k++) u->newsrc[u->n_new++] = tm->cand[k];
        return;
    }
    if (n == 1) {
        uint32_t idx = rng_u32(&tm->rng, (uint32_t)nc);
        u->newsrc[u->n_new++] = tm->cand[idx];
        return;
    }
    /* sample indices 0..nc-1, order preserving -> already sorted by cell */
    for (int k = 0; k < nc; k++) tm->cand2[k] = (uint32_t)k;
    uint32_t pick[ORC_MAXSYN];
    rng_sample(&tm->rng, tm->cand2, (uint32_t)nc, pick, (uint32_t)n);
    for (int k = 0; k < n; k++) u->newsrc[u->n_new++] = tm->cand[pick[k]];
}

/* _getSegmentActiveSynapses(c, i, s, activeState, newSynapses) */
static void tm_get_segment_active_synapses(const orc_params* p, tm_t* tm, int c, int i, seg_t* s,
                                           const uint8_t* state, int new_synapses, segupd_t* u) {
    memset(u, 0, sizeof(*u));
    u->col = c;
    u->cell = i;
    u->seg = s;
    if (s) {
        for (int k = 0; k < s->nsyn; k++)
            if (state[s->syn[k].src]) u->idx[u->n_idx++] = k;
    }
    if (new_synapses) {
        int n = p->tm_new_syn_count - u->n_idx;
        tm_choose_cells_to_learn_from(tm, s, n, state, u);
    }
}

/* _getBestMatchingCell(c, activeState, minThreshold) */
static int tm_best_matching_cell(tm_t* tm, int c, const uint8_t* state, int min_threshold,
                                 seg_t** best_seg, int* best_act) {
    int bestActivityInCol = min_threshold, bestSegIdxInCol = -1, bestCellInCol = -1;
    if (tm->variant & ORC_VAR_TM_BMC_SEG_GE) {
        for (int i = 0; i < tm->K; i++) {
            cell_t* cl = &tm->cells[c * tm->K + i];
            for (int j = 0; j < cl->n; j++) {
                int a = seg_activity(cl->s[j], state);
                if (a >= bestActivityInCol) { bestActivityInCol = a; bestSegIdxInCol = j; bestCellInCol = i; }
            }
        }
        if (bestCellInCol == -1) { *best_seg = NULL; *best_act = 0; return -1; }
        *best_seg = tm->cells[c * tm->K + bestCellInCol].s[bestSegIdxInCol];
        *best_act = bestActivityInCol;
        return bestCellInCol;
    }
    for (int i = 0; i < tm->K; i++) {
        cell_t* cl = &tm->cells[c * tm->K + i];
        int maxSegActivity = 0, maxSegIdx = 0;
        for (int j = 0; j < cl->n; j++) {
            int a = seg_activity(cl->s[j], state);
            if (a > maxSegActivity) { maxSegActivity = a; maxSegIdx = j; }
        }
        if (maxSegActivity >= bestActivityInCol) {
            bestActivityInCol = maxSegActivity;
            bestSegIdxInCol = maxSegIdx;
            bestCellInCol = i;
        }
    }
    if (bestCellInCol == -1) { *best_seg = NULL; *best_act = 0; return -1; }
    *best_seg = tm->cells[c * tm->K + bestCellInCol].s[bestSegIdxInCol];
    *best_act = bestActivityInCol;
    (void)bestSegIdxInCol;
    return bestCellInCol;
}

/* _getCellForNewSegment(colIdx) */
static int tm_cell_for_new_segment(const orc_params* p, tm_t* tm, int c) {
    int K = tm->K;
    if (p->tm_max_segs_per_cell < 0) {
        if (K > 1) return (int)rng_u32(&tm->rng, (uint32_t)(K - 1)) + 1;
        return 0;
    }
    int minIdx = K == 1 ? 0 : 1, maxIdx = K == 1 ? 0 : K - 1;
    int cand[64], nc = 0;
    for (int i = minIdx; i <= maxIdx; i++)
        if (tm->cells[c * K + i].n < p->tm_max_segs_per_cell) cand[nc++] = i;
    if (nc > 0) return cand[rng_u32(&tm->rng, (uint32_t)nc)];
    /* all full: free the least-used segment in the column */
    seg_t* candSeg = NULL;
    float candDC = 1.0f;
    int candCell = -1;
    for (int i = minIdx; i <= maxIdx; i++) {
        cell_t* cl = &tm->cells[c * K + i];
        for (int j = 0; j < cl->n; j++) {
            float dc = seg_duty_cycle(cl->s[j], tm->lrn_iter, 0, 0);
            if (dc < candDC) { candCell = i; candDC = dc; candSeg = cl->s[j]; }
        }
    }
    if (!candSeg) return minIdx; /* unreachable in practice (NuPIC would raise) */
    tm_clean_updates_list(tm, c, candCell, candSeg);
    cell_remove(&tm->cells[c * K + candCell], candSeg);
    seg_free(candSeg);
    return candCell;
}

static int cmp_perm_idx(const void* a, const void* b) {
    const float* x = (const float*)a;
    const float* y = (const float*)b;
    if (x[0] < y[0]) return -1;
    if (x[0] > y[0]) return 1;
    return (x[1] > y[1]) - (x[1] < y[1]);
}

static int cmp_perm_idx_late(const void* a, const void* b) {
    const float* x = (const float*)a;
    const float* y = (const float*)b;
    if (x[0] < y[0]) return -1;
    if (x[0] > y[0]) return 1;
    return (x[1] < y[1]) - (x[1] > y[1]);
}

/* Segment.freeNSynapses(numToFree, inactiveSynapseIndices) */
static void seg_free_n_synapses(seg_t* s, int num_to_free, const uint8_t* inactive, int late) {
    int (*cmp)(const void*, const void*) = late ? cmp_perm_idx_late : cmp_perm_idx;
    float keys[2 * ORC_MAXSYN * 2];
    int cands[ORC_MAXSYN * 2], ncand = 0;
    /* lowest-permanence inactive synapses first (stable by index) */
    int ni = 0;
    for (int k = 0; k < s->nsyn; k++)
        if (inactive[k]) { keys[2 * ni] = s->syn[k].perm; keys[2 * ni + 1] = (float)k; ni++; }
    qsort(keys, (size_t)ni, 2 * sizeof(float), cmp);
    for (int k = 0; k < ni && ncand < num_to_free; k++) cands[ncand++] = (int)keys[2 * k + 1];
    if (ncand < num_to_free) {
        int na = 0;
        for (int k = 0; k < s->nsyn; k++)
            if (!inactive[k]) { keys[2 * na] = s->syn[k].perm; keys[2 * na + 1] = (float)k; na++; }
        qsort(keys, (size_t)na, 2 * sizeof(float), cmp);
        for (int k = 0; k < na && ncand < num_to_free; k++) cands[ncand++] = (int)keys[2 * k + 1];
    }
    uint8_t del[ORC_MAXSYN * 2];
    memset(del, 0, sizeof(del));
    for (int k = 0; k < ncand; k++) del[cands[k]] = 1;
    int w = 0;
    for (int k = 0; k < s->nsyn; k++)
        if (!del[k]) s->syn[w++] = s->syn[k];
    s->nsyn = w;
}

/* _adaptSegment(segUpdate); returns trimSegment */
static int tm_adapt_segment(const orc_params* p, tm_t* tm, const segupd_t* u) {
    int trim = 0;
    seg_t* s = u->seg;
    if (s) {
        s->last_active_it = tm->lrn_iter;
        s->pos_act += 1;
        (void)seg_duty_cycle(s, tm->lrn_iter, 1, 0);
        uint8_t inactive[ORC_MAXSYN * 2];
        int last = s->nsyn;
        for (int k = 0; k < last; k++) inactive[k] = 1;
        for (int k = 0; k < u->n_idx; k++) inactive[u->idx[k]] = 0;
        /* decrement inactive synapses, floor at 0 */
        for (int k = 0; k < last; k++) {
            if (!inactive[k]) continue;
            float nv = s->syn[k].perm + (-p->tm_perm_dec);
            s->syn[k].perm = nv;
            if (nv <= 0.0f) { s->syn[k].perm = 0.0f; trim = 1; }
        }
        /* increment active synapses, cap at permanenceMax */
        for (int k = 0; k < last; k++) {
            if (inactive[k]) continue;
            float nv = s->syn[k].perm + p->tm_perm_inc;
            s->syn[k].perm = nv;
            if (nv > p->tm_perm_max) s->syn[k].perm = p->tm_perm_max;
        }
        if (p->tm_max_syn_per_seg > 0 && u->n_new + s->nsyn > p->tm_max_syn_per_seg) {
            int num_to_free = s->nsyn + u->n_new - p->tm_max_syn_per_seg;
            seg_free_n_synapses(s, num_to_free, inactive, (tm->variant & ORC_VAR_TM_FREE_LATE) != 0);
        }
        for (int k = 0; k < u->n_new; k++) seg_add_syn(s, u->newsrc[k], p->tm_initial_perm);
    } else {
        seg_t* ns = seg_new(p, tm->lrn_iter, u->seq_flag);
        for (int k = 0; k < u->n_new; k++) seg_add_syn(ns, u->newsrc[k], p->tm_initial_perm);
        cell_append(&tm->cells[u->col * tm->K + u->cell], ns);
    }
    return trim;
}

/* _processSegmentUpdates(activeColumns) */
static void tm_process_segment_updates(const orc_params* p, tm_t* tm, const int32_t* active, int nA) {
    memset(tm->colmask, 0, (size_t)tm->ncol);
    for (int k = 0; k < nA; k++) tm->colmask[active[k]] = 1;
    /* trims collected, applied after all updates */
    int ntrim = 0, captrim = 16;
    segupd_t* trims = (segupd_t*)malloc(sizeof(segupd_t) * (size_t)captrim);
    for (int k = 0; k < tm->n_upd;) {
        updlist_t* l = &tm->upd[k];
        int c = l->col;
        int update = tm->colmask[c] ? 1 : 0; /* doPooling False: 'remove' otherwise */
        if (update) {
            for (int j = 0; j < l->n; j++) {
                if (tm->lrn_iter - l->it[j].date > (uint32_t)p->tm_seg_update_valid_duration) continue;
                if (tm_adapt_segment(p, tm, &l->it[j].u)) {
                    if (ntrim == captrim) {
                        captrim *= 2;
                        trims = (segupd_t*)realloc(trims, sizeof(segupd_t) * (size_t)captrim);
                    }
                    trims[ntrim++] = l->it[j].u;
                }
            }
        }
        /* updateListKeep is empty for both 'update' and 'remove' */
        tm_remove_updlist(tm, k);
    }
    for (int k = 0; k < ntrim; k++)
        tm_trim_segment(tm, trims[k].col, trims[k].cell, trims[k].seg, 0.00001f, 0);
    free(trims);
}

/* _learnPhase1(activeColumns, readOnly) */
static int tm_learn_phase1(const orc_params* p, tm_t* tm, const int32_t* active, int nA, int read_only) {
    int K = tm->K;
    memset(tm->lrnA_t, 0, (size_t)tm->ncells);
    int numUnpredicted = 0;
    for (int a = 0; a < nA; a++) {
        int c = active[a];
        int npred = 0, predcell = -1;
        for (int i = 0; i < K; i++)
            if (tm->lrnP_t1[c * K + i] == 1) { npred++; predcell = i; }
        if (npred == 1) {
            tm->lrnA_t[c * K + predcell] = 1;
            continue;
        }
        numUnpredicted++;
        if (read_only) continue;
        seg_t* s;
        int act;
        int i = tm_best_matching_cell(tm, c, tm->lrnA_t1, p->tm_min_threshold, &s, &act);
        segupd_t u;
        if (s && s->is_seq) {
            tm->lrnA_t[c * K + i] = 1;
            tm_get_segment_active_synapses(p, tm, c, i, s, tm->lrnA_t1, 1, &u);
            s->tot_act += 1;
            if (tm_adapt_segment(p, tm, &u)) tm_trim_segment(tm, c, i, s, 0.00001f, 0);
        } else {
            i = tm_cell_for_new_segment(p, tm, c);
            tm->lrnA_t[c * K + i] = 1;
            tm_get_segment_active_synapses(p, tm, c, i, NULL, tm->lrnA_t1, 1, &u);
            u.seq_flag = 1;
            tm_adapt_segment(p, tm, &u);
        }
    }
    return numUnpredicted < nA / 2;
}

/* _learnPhase2(readOnly) */
static void tm_learn_phase2(const orc_params* p, tm_t* tm, int read_only) {
    int K = tm->K;
    tm->stats[2]++;
    memset(tm->lrnP_t, 0, (size_t)tm->ncells);
    for (int c = 0; c < tm->ncol; c++) {
        seg_t* s;
        int act;
        int i = tm_best_matching_cell(tm, c, tm->lrnA_t, p->tm_activation_threshold, &s, &act);
        if (i < 0) continue;
        tm->lrnP_t[c * K + i] = 1;
        if (read_only) continue;
        segupd_t u;
        tm_get_segment_active_synapses(p, tm, c, i, s, tm->lrnA_t, act < p->tm_new_syn_count, &u);
        s->tot_act += 1;
        tm_add_to_updates(tm, c, i, &u);
    }
}

static void pat_push(pattern_t* pats, int* n, int maxbt, const int32_t* cols, int nA) {
    if (*n > maxbt) {
        /* pop(0): rotate the storage */
        int32_t* keep = pats[0].cols;
        memmove(pats, pats + 1, sizeof(pattern_t) * (size_t)(*n - 1));
        pats[*n - 1].cols = keep;
        (*n)--;
    }
    pats[*n].n = nA;
    memcpy(pats[*n].cols, cols, 4 * (size_t)nA);
    (*n)++;
}

static void pat_pop_front(pattern_t* pats, int* n) {
    int32_t* keep = pats[0].cols;
    memmove(pats, pats + 1, sizeof(pattern_t) * (size_t)(*n - 1));
    pats[*n - 1].cols = keep;
    pats[*n - 1].n = 0;
    (*n)--;
}

/* _learnBacktrackFrom(startOffset, readOnly) */
static int tm_learn_backtrack_from(const orc_params* p, tm_t* tm, int start, int read_only) {
    int numPrev = tm->n_lrn_pat;
    int cur = numPrev - 1;
    if (!read_only) tm_clear_updates(tm);
    int inSeq = 1;
    for (int off = start; off < numPrev; off++) {
        memcpy(tm->lrnP_t1, tm->lrnP_t, (size_t)tm->ncells);
        memcpy(tm->lrnA_t1, tm->lrnA_t, (size_t)tm->ncells);
        const pattern_t* pat = &tm->lrn_pat[off];
        if (!read_only) tm_process_segment_updates(p, tm, pat->cols, pat->n);
        if (off == start) {
            memset(tm->lrnA_t, 0, (size_t)tm->ncells);
            for (int a = 0; a < pat->n; a++) tm->lrnA_t[pat->cols[a] * tm->K] = 1;
            inSeq = 1;
        } else {
            inSeq = tm_learn_phase1(p, tm, pat->cols, pat->n, read_only);
        }
        if (!inSeq || off == cur) break;
        tm_learn_phase2(p, tm, read_only);
    }
    return inSeq;
}

/* _learnBacktrack(); returns number of steps backtracked (0 = failure) */
static int tm_learn_backtrack(const orc_params* p, tm_t* tm) {
    int numPrev = tm->n_lrn_pat - 1;
    tm->stats[3]++;
    if (numPrev <= 0) return 0;
    uint8_t bad[64];
    memset(bad, 0, sizeof(bad));
    int inSeq = 0, start;
    for (start = 0; start < numPrev; start++) {
        inSeq = tm_learn_backtrack_from(p, tm, start, 1);
        if (inSeq) break;
        bad[start] = 1;
    }
    if (!inSeq) {
        tm->n_lrn_pat = 0;
        return 0;
    }
    tm_learn_backtrack_from(p, tm, start, 0);
    for (int i = 0; i < numPrev; i++) {
        if (bad[i] || i <= start) pat_pop_front(tm->lrn_pat, &tm->n_lrn_pat);
        else break;
    }
    return numPrev - start;
}

/* _updateAvgLearnedSeqLength */
static void tm_update_avg_learned_seq_length(tm_t* tm, int prevSeqLength) {
    double alpha = tm->lrn_iter < 100 ? 0.5 : 0.1;
    tm->avg_learned_seq_length = (1.0 - alpha) * tm->avg_learned_seq_length + alpha * prevSeqLength;
}

/* _updateLearningState(activeColumns) */
static void tm_update_learning_state(const orc_params* p, tm_t* tm, const int32_t* active, int nA) {
    memcpy(tm->lrnP_t1, tm->lrnP_t, (size_t)tm->ncells);
    memcpy(tm->lrnA_t1, tm->lrnA_t, (size_t)tm->ncells);
    if (p->tm_max_lrn_backtrack > 0) pat_push(tm->lrn_pat, &tm->n_lrn_pat, p->tm_max_lrn_backtrack, active, nA);
    tm_process_segment_updates(p, tm, active, nA);
    if (tm->pam_counter > 0) tm->pam_counter--;
    tm->learned_seq_length++;
    if (!tm->reset_called) {
        int inSeq = tm_learn_phase1(p, tm, active, nA, 0);
        if (inSeq) tm->pam_counter = p->tm_pam_length;
    }
    if (tm->reset_called || tm->pam_counter == 0 ||
        (p->tm_max_seq_length != 0 && tm->learned_seq_length >= p->tm_max_seq_length)) {
        int seqLength = tm->pam_counter == 0 ? tm->learned_seq_length - p->tm_pam_length
                                             : tm->learned_seq_length;
        tm_update_avg_learned_seq_length(tm, seqLength);
        int backSteps = 0;
        if (!tm->reset_called) backSteps = tm_learn_backtrack(p, tm);
        if (tm->reset_called || backSteps == 0) {
            backSteps = 0;
            memset(tm->lrnA_t, 0, (size_t)tm->ncells);
            for (int a = 0; a < nA; a++) tm->lrnA_t[active[a] * tm->K] = 1;
            tm->n_lrn_pat = 0;
        }
        tm->pam_counter = p->tm_pam_length;
        tm->learned_seq_length = backSteps;
        tm_clear_updates(tm);
    }
    tm_learn_phase2(p, tm, 0);
}

/* _inferPhase1(activeColumns, useStartCells) */
static int tm_infer_phase1(tm_t* tm, const int32_t* active, int nA, int use_start) {
    int K = tm->K;
    memset(tm->infA_t, 0, (size_t)tm->ncells);
    int numPredictedColumns = 0;
    if (use_start) {
        for (int a = 0; a < nA; a++) tm->infA_t[active[a] * K] = 1;
    } else {
        for (int a = 0; a < nA; a++) {
            int c = active[a], npc = 0;
            for (int i = 0; i < K; i++)
                if (tm->infP_t1[c * K + i] == 1) { tm->infA_t[c * K + i] = 1; npc++; }
            if (npc > 0) numPredictedColumns++;
            else for (int i = 0; i < K; i++) tm->infA_t[c * K + i] = 1;
        }
    }
    return use_start || (double)numPredictedColumns >= 0.50 * (double)nA;
}

/* _inferPhase2() */
static int tm_infer_phase2(const orc_params* p, tm_t* tm) {
    int K = tm->K;
    tm->stats[0]++;
    memset(tm->infP_t, 0, (size_t)tm->ncells);
    memset(tm->cellConf_t, 0, sizeof(float) * (size_t)tm->ncells);
    memset(tm->colConf_t, 0, sizeof(float) * (size_t)tm->ncol);
    for (int c = 0; c < tm->ncol; c++) {
        for (int i = 0; i < K; i++) {
            cell_t* cl = &tm->cells[c * K + i];
            for (int j = 0; j < cl->n; j++) {
                seg_t* s = cl->s[j];
                int nact = seg_activity(s, tm->infA_t);
                if (nact < p->tm_activation_threshold) continue;
                float dc = seg_duty_cycle(s, tm->lrn_iter, 0, (tm->variant & ORC_VAR_TM_DC_READONLY) != 0);
                tm->cellConf_t[c * K + i] += dc;
                tm->colConf_t[c] += dc;
                if (seg_is_active(p, s, tm->infA_t)) tm->infP_t[c * K + i] = 1;
            }
        }
    }
    float sum = 0.0f;
    for (int c = 0; c < tm->ncol; c++) sum += tm->colConf_t[c];
    if (sum > 0.0f) {
        for (int c = 0; c < tm->ncol; c++) tm->colConf_t[c] /= sum;
        for (int k = 0; k < tm->ncells; k++) tm->cellConf_t[k] /= sum;
    }
    int numPredictedCols = 0;
    for (int c = 0; c < tm->ncol; c++) {
        for (int i = 0; i < K; i++)
            if (tm->infP_t[c * K + i]) { numPredictedCols++; break; }
    }
    return (double)numPredictedCols >= 0.5 * tm->avg_input_density;
}

/* _inferBacktrack(activeColumns) */
static void tm_infer_backtrack(const orc_params* p, tm_t* tm) {
    int numPrev = tm->n_inf_pat;
    tm->stats[1]++;
    if (numPrev <= 0) return;
    int cur = numPrev - 1;
    size_t nc = (size_t)tm->ncells;
    memcpy(tm->infA_backup, tm->infA_t, nc);
    memcpy(tm->infP_backup, tm->infP_t1, nc);
    uint8_t bad[64];
    memset(bad, 0, sizeof(bad));
    int inSeq = 0, haveCand = 0, candStart = -1, maxlen = 0;
    for (int start = 0; start < numPrev; start++) {
        if (start == cur && haveCand) break;
        inSeq = 0;
        int len = 0;
        for (int off = start; off < numPrev; off++) {
            memcpy(tm->infP_t1, tm->infP_t, nc);
            inSeq = tm_infer_phase1(tm, tm->inf_pat[off].cols, tm->inf_pat[off].n, off == start);
            if (!inSeq) break;
            inSeq = tm_infer_phase2(p, tm);
            len++;
            if (!inSeq) break;
        }
        if (len > maxlen) maxlen = len;
        if (!inSeq) { bad[start] = 1; continue; }
        haveCand = 1;
        candStart = start;
        if (candStart == cur) break;
        memcpy(tm->infA_cand, tm->infA_t, nc);
        memcpy(tm->infP_cand, tm->infP_t, nc);
        memcpy(tm->cellConf_cand, tm->cellConf_t, nc * 4);
        memcpy(tm->colConf_cand, tm->colConf_t, (size_t)tm->ncol * 4);
        if (!(tm->variant & ORC_VAR_TM_BT_LAST_START)) break;
    }
    tm->bt_crit = maxlen + (haveCand ? 0 : 1);
    if (!haveCand) {
        memcpy(tm->infA_t, tm->infA_backup, nc);
        tm_infer_phase2(p, tm);
    } else if (candStart != cur) {
        memcpy(tm->infA_t, tm->infA_cand, nc);
        memcpy(tm->infP_t, tm->infP_cand, nc);
        memcpy(tm->cellConf_t, tm->cellConf_cand, nc * 4);
        memcpy(tm->colConf_t, tm->colConf_cand, (size_t)tm->ncol * 4);
    }
    for (int i = 0; i < numPrev; i++) {
        if (bad[i] || (haveCand && i <= candStart)) pat_pop_front(tm->inf_pat, &tm->n_inf_pat);
        else break;
    }
    memcpy(tm->infP_t1, tm->infP_backup, nc);
}

/* _updateInferenceState(activeColumns) */
static void tm_update_inference_state(const orc_params* p, tm_t* tm, const int32_t* active, int nA) {
    size_t nc = (size_t)tm->ncells;
    memcpy(tm->infA_t1, tm->infA_t, nc);
    memcpy(tm->infP_t1, tm->infP_t, nc);
    memcpy(tm->cellConf_t1, tm->cellConf_t, nc * 4);
    memcpy(tm->colConf_t1, tm->colConf_t, (size_t)tm->ncol * 4);
    if (p->tm_max_inf_backtrack > 0) pat_push(tm->inf_pat, &tm->n_inf_pat, p->tm_max_inf_backtrack, active, nA);
    int inSeq = tm_infer_phase1(tm, active, nA, tm->reset_called);
    tm->bt_crit = 0;
    if (!inSeq) {
        tm_infer_backtrack(p, tm);
        tm->stats[4] += tm->bt_crit;
        return;
    }
    inSeq = tm_infer_phase2(p, tm);
    if (!inSeq) tm_infer_backtrack(p, tm);
    tm->stats[4] += 1 + tm->bt_crit;
}

/* BacktrackingTM.compute(bottomUpInput, enableLearn, enableInference=True) */
static void tm_compute(const orc_params* p, tm_t* tm, const int32_t* active, int nA, int learn) {
    if (learn) tm->lrn_iter++;
    tm->iter++;
    if (learn && (tm->variant & ORC_VAR_TM_DC_TIERS)) {
        int tier = 0;
        for (int t = 1; t < 9; t++) tier |= tm->lrn_iter == DC_TIERS[t];
        if (tier)
            for (int c = 0; c < tm->ncells; c++)
                for (int j = 0; j < tm->cells[c].n; j++) (void)seg_duty_cycle(tm->cells[c].s[j], tm->lrn_iter, 0, 0);
    }
    if (!tm->have_avg_density) {
        tm->avg_input_density = (double)nA;
        tm->have_avg_density = 1;
    } else {
        tm->avg_input_density = 0.99 * tm->avg_input_density + 0.01 * (double)nA;
    }
    tm_update_inference_state(p, tm, active, nA);
    if (learn) tm_update_learning_state(p, tm, active, nA);
    tm->reset_called = 0;
}

/* BacktrackingTM.reset() */
static void tm_reset(tm_t* tm) {
    size_t nc = (size_t)tm->ncells;
    memset(tm->lrnA_t1, 0, nc); memset(tm->lrnA_t, 0, nc);
    memset(tm->lrnP_t1, 0, nc); memset(tm->lrnP_t, 0, nc);
    memset(tm->infA_t1, 0, nc); memset(tm->infA_t, 0, nc);
    memset(tm->infP_t1, 0, nc); memset(tm->infP_t, 0, nc);
    memset(tm->cellConf_t1, 0, nc * 4); memset(tm->cellConf_t, 0, nc * 4);
    tm_clear_updates(tm);
    tm->reset_called = 1;
    tm->n_inf_pat = 0;
    tm->n_lrn_pat = 0;
}

/* =====================================================================
 * Model: encoder -> SP -> TM -> raw anomaly
 * ===================================================================== */
struct orc_model {
    orc_params p;
    rdse_t rdse[4];
    int32_t bucket[4];
    sp_t sp;
    tm_t tm;
    uint8_t* input;
    int32_t* prev_pred;
    int n_prev_pred;
};

void orc_default_params(orc_params* p) {
    memset(p, 0, sizeof(*p));
    p->n_fields = 1;
    p->enc_n = 500;
    p->enc_w = 21;
    p->enc_minval = 0.0;
    p->enc_maxval = 100.0;
    p->enc_clip = 1;
    p->sp_columns = 2048;
    p->sp_num_active = 40;
    p->sp_potential_pct = 0.8f;
    p->sp_perm_connected = 0.1f;
    p->sp_perm_active_inc = 0.0001f;
    p->sp_perm_inactive_dec = 0.0005f;
    p->sp_min_pct_overlap_dc = 0.001f;
    p->sp_duty_cycle_period = 1000;
    p->sp_boost_strength = 0.0f;
    p->sp_stimulus_threshold = 0;
    p->sp_update_period = 50;
    p->sp_seed = 2045;
    p->tm_cells_per_col = 12;
    p->tm_new_syn_count = 20;
    p->tm_max_syn_per_seg = 32;
    p->tm_max_segs_per_cell = 128;
    p->tm_initial_perm = 0.21f;
    p->tm_connected_perm = 0.5f;
    p->tm_perm_inc = 0.1f;
    p->tm_perm_dec = 0.1f;
    p->tm_perm_max = 1.0f;
    p->tm_min_threshold = 9;
    p->tm_activation_threshold = 12;
    p->tm_pam_length = 3;
    p->tm_max_inf_backtrack = 10;
    p->tm_max_lrn_backtrack = 5;
    p->tm_max_seq_length = 32;
    p->tm_seg_update_valid_duration = 5;
    p->tm_seed = 2045;
}

orc_model* orc_create(const orc_params* p) {
    if (p->sdr_bits < 0 || (p->tm_max_inf_backtrack > 60 || p->tm_max_lrn_backtrack > 60 ||
        p->tm_max_syn_per_seg > ORC_MAXSYN || p->tm_new_syn_count > ORC_MAXSYN ||
        p->tm_cells_per_col > 64))
        return NULL;
    if (p->enc_type == ORC_ENC_RDSE &&
        (p->sdr_bits > 0 || p->enc_w < 1 || p->enc_w % 2 == 0 || p->enc_n <= 6 * p->enc_w || !(p->rdse_resolution > 0.0)))
        return NULL;
    orc_model* m = (orc_model*)calloc(1, sizeof(orc_model));
    m->p = *p;
    if (p->enc_type == ORC_ENC_RDSE)
        for (int f = 0; f < p->n_fields; f++) rdse_init(&m->p, &m->rdse[f], p->rdse_seed);
    for (int f = 0; f < 4; f++) m->bucket[f] = -1;
    sp_init(&m->p, &m->sp);
    tm_init(&m->p, &m->tm);
    m->input = (uint8_t*)calloc((size_t)m->sp.nin, 1);
    m->prev_pred = (int32_t*)calloc((size_t)m->sp.ncol, 4);
    return m;
}

orc_model* orc_clone(const orc_model* s) {
    orc_model* m = (orc_model*)calloc(1, sizeof(orc_model));
    m->p = s->p;
    if (s->p.enc_type == ORC_ENC_RDSE)
        for (int f = 0; f < s->p.n_fields; f++) rdse_copy(&s->p, &m->rdse[f], &s->rdse[f]);
    memcpy(m->bucket, s->bucket, sizeof(m->bucket));
    sp_copy(&m->sp, &s->sp);
    tm_copy(&m->p, &m->tm, &s->tm);
    m->input = (uint8_t*)malloc((size_t)s->sp.nin);
    memcpy(m->input, s->input, (size_t)s->sp.nin);
    m->prev_pred = (int32_t*)malloc((size_t)s->sp.ncol * 4);
    memcpy(m->prev_pred, s->prev_pred, (size_t)s->sp.ncol * 4);
    m->n_prev_pred = s->n_prev_pred;
    return m;
}

void orc_free(orc_model* m) {
    if (!m) return;
    if (m->p.enc_type == ORC_ENC_RDSE)
        for (int f = 0; f < m->p.n_fields; f++) free(m->rdse[f].map);
    sp_free(&m->sp);
    tm_free(&m->p, &m->tm);
    free(m->input);
    free(m->prev_pred);
    free(m);
}

static float step_after_encode(orc_model* m, int sp_learn, int tm_learn);

/* RecordSensor -> MultiEncoder.encodeIntoArray: fields in sorted name order,
 * each encoder's n bits */
static void model_encode(orc_model* m, const double* values, uint8_t* out) {
    const orc_params* p = &m->p;
    if (p->enc_type != ORC_ENC_RDSE) {
        enc_encode(p, values, out);
        for (int f = 0; f < p->n_fields; f++) m->bucket[f] = enc_first_on_bit(p, f, values[f]);
        return;
    }
    memset(out, 0, (size_t)p->n_fields * p->enc_n);
    for (int f = 0; f < p->n_fields; f++) {
        const int b = rdse_bucket(p, &m->rdse[f], values[f]);
        m->bucket[f] = b;
        if (b < 0) continue;
        const int32_t* bits = rdse_bits(p, &m->rdse[f], b);
        for (int k = 0; k < p->enc_w; k++) out[f * p->enc_n + bits[k]] = 1;
    }
}

float orc_step(orc_model* m, const double* values, int sp_learn, int tm_learn) {
    model_encode(m, values, m->input);
    return step_after_encode(m, sp_learn, tm_learn);
}

float orc_step_sdr(orc_model* m, const uint8_t* input, int sp_learn, int tm_learn) {
    for (int i = 0; i < m->sp.nin; i++) m->input[i] = input[i] ? 1 : 0;
    return step_after_encode(m, sp_learn, tm_learn);
}

void orc_tm_output(const orc_model* m, uint8_t* out) {
    for (int k = 0; k < m->tm.ncells; k++) out[k] = (m->tm.infA_t[k] | m->tm.infP_t[k]) ? 1 : 0;
}

static float step_after_encode(orc_model* m, int sp_learn, int tm_learn) {
    sp_compute(&m->p, &m->sp, m->input, sp_learn);
    /* TMRegion (anomalyMode): prevPredictedColumns = nonzero(topDownCompute())
     * captured before compute */
    int np = 0;
    for (int c = 0; c < m->tm.ncol; c++)
        if (m->tm.colConf_t[c] != 0.0f) m->prev_pred[np++] = c;
    m->n_prev_pred = np;
    tm_compute(&m->p, &m->tm, m->sp.active_sorted, m->sp.n_active, tm_learn);
    /* computeRawAnomalyScore(activeColumns, prevPredictedColumns) */
    int nA = m->sp.n_active;
    if (nA == 0) return 0.0f;
    int hit = 0;
    for (int a = 0, k = 0; a < nA; a++) {
        while (k < np && m->prev_pred[k] < m->sp.active_sorted[a]) k++;
        if (k < np && m->prev_pred[k] == m->sp.active_sorted[a]) hit++;
    }
    double score = (double)(nA - hit) / (double)nA;
    return (float)score;
}

void orc_step_batch(orc_model** models, int n, const double* values, int sp_learn, int tm_learn,
                    float* scores, int n_threads) {
#ifdef _OPENMP
    if (n_threads <= 0) n_threads = omp_get_max_threads();
#pragma omp parallel for num_threads(n_threads) schedule(dynamic, 1)
#else
    (void)n_threads;
#endif
    for (int i = 0; i < n; i++) {
        int nf = models[i]->p.n_fields;
        scores[i] = orc_step(models[i], values + (size_t)i * nf, sp_learn, tm_learn);
    }
}

void orc_tm_reset(orc_model* m) { tm_reset(&m->tm); }

/* ---------------- introspection ---------------- */
int orc_num_inputs(const orc_model* m) { return m->sp.nin; }
int orc_num_cells(const orc_model* m) { return m->tm.ncells; }

void orc_encode(orc_model* m, const double* values, uint8_t* out) { model_encode(m, values, out); }

int orc_bucket(const orc_model* m, int f) { return (f >= 0 && f < 4) ? m->bucket[f] : -1; }

void orc_rdse_state(const orc_model* m, int f, int32_t* sc4, double* offset, int32_t* map) {
    const rdse_t* r = &m->rdse[f];
    if (m->p.enc_type != ORC_ENC_RDSE || f < 0 || f >= m->p.n_fields) return;
    sc4[0] = r->min_idx;
    sc4[1] = r->max_idx;
    sc4[2] = r->has_offset;
    sc4[3] = r->num_tries;
    *offset = r->offset;
    const int w = m->p.enc_w;
    memset(map, 0, sizeof(int32_t) * (size_t)ORC_RDSE_BUCKETS * w);
    for (int i = r->min_idx; i <= r->max_idx; i++)
        memcpy(map + (size_t)i * w, r->map + (size_t)i * w, sizeof(int32_t) * (size_t)w);
}

int orc_active_columns(const orc_model* m, int32_t* out) {
    memcpy(out, m->sp.active_sorted, 4 * (size_t)m->sp.n_active);
    return m->sp.n_active;
}

int orc_prev_pred_columns(const orc_model* m, int32_t* out) {
    memcpy(out, m->prev_pred, 4 * (size_t)m->n_prev_pred);
    return m->n_prev_pred;
}

void orc_tm_states(const orc_model* m, uint8_t* ia, uint8_t* ip, uint8_t* la, uint8_t* lp) {
    size_t nc = (size_t)m->tm.ncells;
    if (ia) memcpy(ia, m->tm.infA_t, nc);
    if (ip) memcpy(ip, m->tm.infP_t, nc);
    if (la) memcpy(la, m->tm.lrnA_t, nc);
    if (lp) memcpy(lp, m->tm.lrnP_t, nc);
}

void orc_col_confidence(const orc_model* m, float* out) {
    memcpy(out, m->tm.colConf_t, 4 * (size_t)m->tm.ncol);
}

void orc_cell_confidence(const orc_model* m, float* out) {
    memcpy(out, m->tm.cellConf_t, 4 * (size_t)m->tm.ncells);
}

void orc_tm_scalars(const orc_model* m, int64_t* o) {
    int nseg = 0, nsyn = 0;
    for (int c = 0; c < m->tm.ncells; c++) {
        nseg += m->tm.cells[c].n;
        for (int j = 0; j < m->tm.cells[c].n; j++) nsyn += m->tm.cells[c].s[j]->nsyn;
    }
    int nupd = 0;
    for (int k = 0; k < m->tm.n_upd; k++) nupd += m->tm.upd[k].n;
    o[0] = m->tm.lrn_iter;
    o[1] = m->tm.iter;
    o[2] = m->tm.pam_counter;
    o[3] = m->tm.learned_seq_length;
    o[4] = m->tm.n_inf_pat;
    o[5] = m->tm.n_lrn_pat;
    o[6] = nupd;
    o[7] = nseg;
    o[8] = nsyn;
}

double orc_tm_avg_input_density(const orc_model* m) { return m->tm.avg_input_density; }

void orc_tm_stats(const orc_model* m, int64_t* out5) { memcpy(out5, m->tm.stats, sizeof(m->tm.stats)); }

int orc_tm_segments(const orc_model* m, int32_t* info, float* dc, int32_t* src, float* perm, int max_syn) {
    int k = 0;
    for (int c = 0; c < m->tm.ncells; c++) {
        const cell_t* cl = &m->tm.cells[c];
        for (int j = 0; j < cl->n; j++, k++) {
            const seg_t* s = cl->s[j];
            if (!info) continue;
            info[k * 5 + 0] = c;
            info[k * 5 + 1] = s->is_seq;
            info[k * 5 + 2] = (int32_t)s->pos_act;
            info[k * 5 + 3] = (int32_t)s->last_dc_it;
            info[k * 5 + 4] = s->nsyn;
            dc[k] = s->last_dc;
            for (int q = 0; q < max_syn; q++) {
                src[(size_t)k * max_syn + q] = q < s->nsyn ? (int32_t)s->syn[q].src : 0;
                perm[(size_t)k * max_syn + q] = q < s->nsyn ? s->syn[q].perm : 0.0f;
            }
        }
    }
    return k;
}

void orc_sp_state(const orc_model* m, float* perm, uint8_t* pot, uint8_t* conn, float* odc,
                  float* adc, float* minodc, float* boost, int64_t* it2) {
    size_t ci = (size_t)m->sp.ncol * m->sp.nin, nc = (size_t)m->sp.ncol;
    if (perm) memcpy(perm, m->sp.perm, ci * 4);
    if (pot) memcpy(pot, m->sp.potential, ci);
    if (conn) memcpy(conn, m->sp.connected, ci);
    if (odc) memcpy(odc, m->sp.overlap_dc, nc * 4);
    if (adc) memcpy(adc, m->sp.active_dc, nc * 4);
    if (minodc) memcpy(minodc, m->sp.min_overlap_dc, nc * 4);
    if (boost) memcpy(boost, m->sp.boost, nc * 4);
    if (it2) { it2[0] = m->sp.iter; it2[1] = m->sp.iter_learn; }
}

void orc_sp_overlaps(const orc_model* m, int32_t* out) {
    memcpy(out, m->sp.overlaps, 4 * (size_t)m->sp.ncol);
}

void orc_rng_stream(uint64_t seed, int n, uint32_t* out) {
    rng_t g;
    rng_seed(&g, seed);
    for (int i = 0; i < n; i++) out[i] = rng_raw(&g);
}

void orc_rng_real64(uint64_t seed, int n, double* out) {
    rng_t g;
    rng_seed(&g, seed);
    for (int i = 0; i < n; i++) out[i] = rng_real64(&g);
}

void orc_tm_rng_state(const orc_model* m, uint32_t* out33) {
    memcpy(out33, m->tm.rng.s, 31 * 4);
    out33[31] = (uint32_t)m->tm.rng.f;
    out33[32] = (uint32_t)m->tm.rng.r;
}
