// classifier.hip -- SDRClassifier for N streams.
//
// Restates NuPIC 1.0.x SDRClassifier (implementation 'py') behind
// SDRClassifierRegion.compute, as oracle/sdr_classifier_reference.py
// describes: the region the reference adds with alpha 0.005 and steps 1..7
// (ML/HTM/NetworkModel.py:70-97), fed TM bottomUpOut, the sensor's bucket
// index and actual value; its probabilities feed getPredictionResults
// (ML/HTM/NetworkUtils.py:166-184).  It never affects the anomaly score.
//
// Per stream: float64 weights [steps][ncells][nbuckets] (the lazily grown
// NuPIC matrix, zero-padded to its final size: rows above maxInputIdx and
// columns above maxBucketIdx stay zero and are never read), the actual-value
// EMA per bucket, and the pattern history ring (max(steps) + 1 entries of
// u16 cell indices).
//
// MI355X design: two launches per record.
//   cls_prep_kernel  one workgroup per stream: compacts the TM output bitmap
//                    into the history ring (block scan of per-thread word
//                    popcounts, ascending cell order), grows maxInputIdx,
//                    writes the inference's actual values, then updates the
//                    bucket bound and the actual-value EMA.
//   cls_step_kernel  one workgroup per (stream, step): each thread owns
//                    bucket columns and adds the pattern's weight rows in
//                    pattern order (numpy's axis-0 reduce order, coalesced
//                    8-byte loads across buckets), softmax with the sum in
//                    numpy's pairwise order; learning computes the error of
//                    the history entry of that age before updating its rows.
// Bucket columns per row are contiguous, so a row update is one coalesced
// read-modify-write per 256 buckets; traffic per stream-record is
// (inference + error + update) ~ steps x |pattern| x nbuckets x 8 B x 4.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "htm_dev.h"

#define CLS_NT 256
#define CLS_MAX_STEPS 16
#define CLS_NB_MAX 1024

struct ClsState {
    int32_t record_num;     // next record number (SDRClassifierRegion.recordNum)
    int32_t max_input;      // maxInputIdx
    int32_t max_bucket;     // maxBucketIdx (after this record's learning)
    int32_t infer_buckets;  // maxBucketIdx + 1 seen by this record's inference
    int32_t hist_n, hist_head;
    int32_t cur_rec, cur_slot;  // this record's number and history slot
    int32_t err;            // 1: THIS record's pattern is empty (NuPIC max() of an empty list; the record
                            //    is skipped, later records run), 2: bucket >= nbuckets (sticky)
    int32_t learn_bucket;   // this record's bucket (-1: no learning)
    int32_t pad[2];
};

struct ClsBufs {
    ClsState* st;      // [S]
    double* actv;      // [S][nb]
    int32_t* act_ok;   // [S][nb]
    int32_t* hrec;     // [S][H]
    int32_t* hlen;     // [S][H]
    uint16_t* hidx;    // [S][H][ncells]
    double* w;         // [S][nsteps][ncells][nb]
    int32_t n, ncells, nb, nsteps, H;
    int32_t steps[CLS_MAX_STEPS];
    double alpha, act_alpha;
};

struct htm_classifier {
    ClsBufs b;
    int device;
};

// numpy's float64 add.reduce of a contiguous vector: pairwise with blocks of 8
template <int D>
__device__ double np_pairwise(const double* a, int n) {
    if (n < 8) {
        double r = 0.0;
        for (int i = 0; i < n; i++) r += a[i];
        return r;
    }
    if (n <= 128 || D == 0) {
        double r[8];
#pragma unroll
        for (int j = 0; j < 8; j++) r[j] = a[j];
        int i = 8;
        for (; i < n - (n % 8); i += 8) {
#pragma unroll
            for (int j = 0; j < 8; j++) r[j] += a[i + j];
        }
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i];
        return res;
    }
    int n2 = n / 2;
    n2 -= n2 % 8;
    return np_pairwise<(D > 0 ? D - 1 : 0)>(a, n2) + np_pairwise<(D > 0 ? D - 1 : 0)>(a + n2, n - n2);
}

__device__ __forceinline__ double wg_max(double v, double* red) {
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[wv] = v;
    __syncthreads();
    double m = red[0];
    for (int i = 1; i < CLS_NT / 64; i++) m = fmax(m, red[i]);
    __syncthreads();
    return m;
}

// softmax of the pattern's activation over buckets [0, B): e[] (LDS) receives
// the distribution.  Rows are added in pattern order, per bucket column.
__device__ void cls_infer(const double* __restrict__ W, const uint16_t* __restrict__ pat, int plen, int nb, int B,
                          double* e, double* red, double* sum_sh) {
    double mloc = -INFINITY;
    for (int b = threadIdx.x; b < B; b += CLS_NT) {
        double a = W[(size_t)pat[0] * nb + b];
        for (int i = 1; i < plen; i++) a += W[(size_t)pat[i] * nb + b];
        e[b] = a;
        mloc = fmax(mloc, a);
    }
    const double m = wg_max(mloc, red);
    for (int b = threadIdx.x; b < B; b += CLS_NT) e[b] = exp(e[b] - m);
    __syncthreads();
    if (threadIdx.x == 0) *sum_sh = np_pairwise<6>(e, B);
    __syncthreads();
    const double s = *sum_sh;
    for (int b = threadIdx.x; b < B; b += CLS_NT) e[b] = e[b] / s;
    __syncthreads();
}

__global__ void __launch_bounds__(CLS_NT) cls_prep_kernel(ClsBufs c, const uint32_t* __restrict__ pattern,
                                                           const int32_t* __restrict__ bucket,
                                                           const double* __restrict__ actval, int learn, int infer,
                                                           double* __restrict__ out_actual) {
    __shared__ int32_t scan[CLS_NT];
    __shared__ int32_t sh_slot, sh_max;
    const int s = blockIdx.x;
    ClsState* st = c.st + s;
    const int words = c.ncells / 32;
    const uint32_t* row = pattern + (size_t)s * words;
    if (threadIdx.x == 0) {
        int slot;
        if (st->hist_n < c.H) {
            slot = (st->hist_head + st->hist_n) % c.H;
            st->hist_n++;
        } else {
            slot = st->hist_head;
            st->hist_head = (st->hist_head + 1) % c.H;
        }
        sh_slot = slot;
        sh_max = -1;
    }
    // contiguous word chunk per thread, block-exclusive scan of the popcounts
    const int per = (words + CLS_NT - 1) / CLS_NT;
    const int w0 = threadIdx.x * per;
    const int w1 = min(words, w0 + per);
    int cnt = 0;
    for (int w = w0; w < w1; w++) cnt += __popc(row[w]);
    scan[threadIdx.x] = cnt;
    __syncthreads();
    for (int o = 1; o < CLS_NT; o <<= 1) {
        const int v = (int)threadIdx.x >= o ? scan[threadIdx.x - o] : 0;
        __syncthreads();
        scan[threadIdx.x] += v;
        __syncthreads();
    }
    const int total = scan[CLS_NT - 1];
    const int slot = sh_slot;
    uint16_t* dst = c.hidx + ((size_t)s * c.H + slot) * c.ncells;
    int pos = scan[threadIdx.x] - cnt;
    int last = -1;
    for (int w = w0; w < w1; w++) {
        uint32_t x = row[w];
        while (x) {
            const int bit = __ffs(x) - 1;
            x &= x - 1;
            dst[pos++] = (uint16_t)(w * 32 + bit);
            last = w * 32 + bit;
        }
    }
    if (last >= 0) atomicMax(&sh_max, last);
    __syncthreads();
    const int rec = st->record_num;
    const int old_b = st->max_bucket;
    // inference's actual values (before this record's learning): buckets that
    // never had a value take actValueList[0] (the region's dummy 0 when not learning)
    if (infer) {
        const double dflt = (c.steps[0] == 0 || !learn) ? 0.0 : actval[s];
        for (int b = threadIdx.x; b < c.nb; b += CLS_NT) {
            const size_t k = (size_t)s * c.nb + b;
            out_actual[k] = b <= old_b ? (c.act_ok[k] ? c.actv[k] : dflt) : 0.0;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        c.hrec[(size_t)s * c.H + slot] = rec;
        c.hlen[(size_t)s * c.H + slot] = total;
        st->cur_rec = rec;
        st->cur_slot = slot;
        st->record_num = rec + 1;
        st->infer_buckets = old_b + 1;
        st->learn_bucket = -1;
        st->err &= ~1;  // per-record flag: an empty pattern skips only this record
        if (total == 0) {
            st->err |= 1;
        } else {
            if (sh_max > st->max_input) st->max_input = sh_max;
            const int bk = learn ? bucket[s] : -1;
            if (bk >= c.nb) {
                st->err |= 2;
            } else if (bk >= 0) {
                if (bk > st->max_bucket) st->max_bucket = bk;
                const size_t k = (size_t)s * c.nb + bk;
                const double v = actval[s];
                if (!c.act_ok[k]) {
                    c.actv[k] = v;
                    c.act_ok[k] = 1;
                } else {
                    const double t1 = (1.0 - c.act_alpha) * c.actv[k];
                    const double t2 = c.act_alpha * v;
                    c.actv[k] = t1 + t2;
                }
                st->learn_bucket = bk;
            }
        }
    }
}

__global__ void __launch_bounds__(CLS_NT) cls_step_kernel(ClsBufs c, int infer, double* __restrict__ out_prob) {
    __shared__ double e[CLS_NB_MAX];
    __shared__ double red[CLS_NT / 64];
    __shared__ double sum_sh;
    const int s = blockIdx.x, y = blockIdx.y;
    const int k = c.steps[y];
    const ClsState st = c.st[s];
    double* W = c.w + ((size_t)s * c.nsteps + y) * (size_t)c.ncells * c.nb;
    const uint16_t* hidx = c.hidx + (size_t)s * c.H * c.ncells;
    double* prob = out_prob + ((size_t)s * c.nsteps + y) * c.nb;
    if (st.err & 1) return;
    if (infer) {
        const int B = st.infer_buckets;
        cls_infer(W, hidx + (size_t)st.cur_slot * c.ncells, c.hlen[(size_t)s * c.H + st.cur_slot], c.nb, B, e, red,
                  &sum_sh);
        for (int b = threadIdx.x; b < c.nb; b += CLS_NT) prob[b] = b < B ? e[b] : 0.0;
        __syncthreads();
    }
    const int bk = st.learn_bucket;
    if (bk < 0) return;
    // the history entry of age k (at most one)
    int slot = -1;
    for (int h = 0; h < st.hist_n; h++) {
        const int sl = (st.hist_head + h) % c.H;
        if (st.cur_rec - c.hrec[(size_t)s * c.H + sl] == k) slot = sl;
    }
    if (slot < 0) return;
    const int B = st.max_bucket + 1;
    const uint16_t* pat = hidx + (size_t)slot * c.ncells;
    const int plen = c.hlen[(size_t)s * c.H + slot];
    cls_infer(W, pat, plen, c.nb, B, e, red, &sum_sh);
    for (int b = threadIdx.x; b < B; b += CLS_NT) {
        const double err = (b == bk ? 1.0 : 0.0) - e[b];
        const double d = c.alpha * err;
        for (int i = 0; i < plen; i++) {
            double* p = W + (size_t)pat[i] * c.nb + b;
            *p = *p + d;
        }
    }
}

extern "C" {

int htm_cls_destroy(htm_classifier* h) {
    if (!h) return HTM_OK;
    (void)hipSetDevice(h->device);
    (void)hipDeviceSynchronize();
    void* ps[] = {h->b.st, h->b.actv, h->b.act_ok, h->b.hrec, h->b.hlen, h->b.hidx, h->b.w};
    for (void* p : ps)
        if (p) (void)hipFree(p);
    delete h;
    return HTM_OK;
}

int htm_cls_create(int32_t n_streams, int32_t n_inputs, int32_t n_buckets, const int32_t* steps, int32_t n_steps,
                   double alpha, double act_value_alpha, int32_t device, htm_classifier** out) {
    if (!out || !steps || n_streams < 1 || n_inputs < 32 || n_inputs % 32 || n_inputs > 65536 || n_buckets < 1 ||
        n_buckets > CLS_NB_MAX || n_steps < 1 || n_steps > CLS_MAX_STEPS)
        return htm_fail(HTM_E_INVALID, "%s: invalid argument", __func__);
    int mx = 0;
    for (int i = 0; i < n_steps; i++) {
        if (steps[i] < 0 || steps[i] > 1000) return htm_fail(HTM_E_INVALID, "%s: invalid argument", __func__);
        for (int j = 0; j < i; j++)
            if (steps[j] == steps[i]) return htm_fail(HTM_E_INVALID, "%s: invalid argument", __func__);
        mx = steps[i] > mx ? steps[i] : mx;
    }
    *out = nullptr;
    if (hipSetDevice(device) != hipSuccess) return htm_fail(HTM_E_HIP, "%s: %s", __func__, hipGetErrorString(hipGetLastError()));
    htm_classifier* h = new htm_classifier();
    h->device = device;
    ClsBufs& b = h->b;
    b.n = n_streams;
    b.ncells = n_inputs;
    b.nb = n_buckets;
    b.nsteps = n_steps;
    b.H = mx + 1;
    for (int i = 0; i < n_steps; i++) b.steps[i] = steps[i];
    b.alpha = alpha;
    b.act_alpha = act_value_alpha;
    const size_t n = (size_t)n_streams;
    struct {
        void** p;
        size_t bytes;
    } al[] = {{(void**)&b.st, n * sizeof(ClsState)},
              {(void**)&b.actv, n * n_buckets * 8},
              {(void**)&b.act_ok, n * n_buckets * 4},
              {(void**)&b.hrec, n * b.H * 4},
              {(void**)&b.hlen, n * b.H * 4},
              {(void**)&b.hidx, n * b.H * (size_t)n_inputs * 2},
              {(void**)&b.w, n * n_steps * (size_t)n_inputs * n_buckets * 8}};
    for (auto& a : al) {
        if (hipMalloc(a.p, a.bytes) != hipSuccess || hipMemset(*a.p, 0, a.bytes) != hipSuccess) {
            (void)hipGetLastError();
            htm_cls_destroy(h);
            return htm_fail(HTM_E_HIP, "%s: %s", __func__, hipGetErrorString(hipGetLastError()));
        }
    }
    *out = h;
    return HTM_OK;
}

int htm_cls_compute(htm_classifier* h, const uint32_t* d_pattern, const int32_t* d_bucket, const double* d_act_value,
                    int32_t learn, int32_t infer, double* d_probabilities, double* d_actual_values, void* stream) {
    if (!h || !d_pattern || (learn && (!d_bucket || !d_act_value)) || (infer && (!d_probabilities || !d_actual_values)))
        return htm_fail(HTM_E_INVALID, "%s: invalid argument", __func__);
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(cls_prep_kernel, dim3(h->b.n), dim3(CLS_NT), 0, st, h->b, d_pattern, d_bucket, d_act_value,
                       learn ? 1 : 0, infer ? 1 : 0, d_actual_values);
    hipLaunchKernelGGL(cls_step_kernel, dim3(h->b.n, h->b.nsteps), dim3(CLS_NT), 0, st, h->b, infer ? 1 : 0,
                       d_probabilities);
    return hipGetLastError() == hipSuccess ? HTM_OK : htm_fail(HTM_E_HIP, "%s: HIP launch/sync failed", __func__);
}

static int cls_region(const htm_classifier* h, int32_t region, void** base, size_t* per) {
    const ClsBufs& b = h->b;
    switch (region) {
        case HTM_CLS_ST_SCALARS: *base = b.st; *per = sizeof(ClsState); return HTM_OK;
        case HTM_CLS_ST_ACTUAL: *base = b.actv; *per = (size_t)b.nb * 8; return HTM_OK;
        case HTM_CLS_ST_ACTUAL_OK: *base = b.act_ok; *per = (size_t)b.nb * 4; return HTM_OK;
        case HTM_CLS_ST_HIST_REC: *base = b.hrec; *per = (size_t)b.H * 4; return HTM_OK;
        case HTM_CLS_ST_HIST_LEN: *base = b.hlen; *per = (size_t)b.H * 4; return HTM_OK;
        case HTM_CLS_ST_HIST_IDX: *base = b.hidx; *per = (size_t)b.H * b.ncells * 2; return HTM_OK;
        case HTM_CLS_ST_WEIGHTS: *base = b.w; *per = (size_t)b.nsteps * b.ncells * b.nb * 8; return HTM_OK;
        default: return htm_fail(HTM_E_INVALID, "%s: invalid argument", __func__);
    }
}

size_t htm_cls_state_bytes(const htm_classifier* h, int32_t region) {
    void* base;
    size_t per;
    if (!h || cls_region(h, region, &base, &per)) return 0;
    return per;
}

static int cls_copy(htm_classifier* h, int32_t region, int32_t s0, int32_t n, void* host, size_t bytes, int to_dev) {
    void* base;
    size_t per;
    if (!h || !host || s0 < 0 || n < 1 || s0 + n > h->b.n || cls_region(h, region, &base, &per)) return htm_fail(HTM_E_INVALID, "%s: invalid argument", __func__);
    if (bytes != per * n) return htm_fail(HTM_E_INVALID, "%s: invalid argument", __func__);
    if (hipSetDevice(h->device) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return htm_fail(HTM_E_HIP, "%s: %s", __func__, hipGetErrorString(hipGetLastError()));
    char* d = (char*)base + per * s0;
    hipError_t e = to_dev ? hipMemcpy(d, host, bytes, hipMemcpyHostToDevice)
                          : hipMemcpy(host, d, bytes, hipMemcpyDeviceToHost);
    return e == hipSuccess ? HTM_OK : htm_fail(HTM_E_HIP, "%s: HIP launch/sync failed", __func__);
}

int htm_cls_export_state(htm_classifier* h, int32_t region, int32_t s0, int32_t n, void* h_dst, size_t bytes) {
    return cls_copy(h, region, s0, n, h_dst, bytes, 0);
}

int htm_cls_import_state(htm_classifier* h, int32_t region, int32_t s0, int32_t n, const void* h_src, size_t bytes) {
    return cls_copy(h, region, s0, n, const_cast<void*>(h_src), bytes, 1);
}

int htm_cls_status(htm_classifier* h, int32_t* out_flags) {
    if (!h || !out_flags) return htm_fail(HTM_E_INVALID, "%s: invalid argument", __func__);
    if (hipSetDevice(h->device) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return htm_fail(HTM_E_HIP, "%s: %s", __func__, hipGetErrorString(hipGetLastError()));
    ClsState* hs = new ClsState[h->b.n];
    const hipError_t e = hipMemcpy(hs, h->b.st, sizeof(ClsState) * h->b.n, hipMemcpyDeviceToHost);
    int32_t f = 0;
    for (int s = 0; s < h->b.n; s++) f |= hs[s].err;
    delete[] hs;
    if (e != hipSuccess) return htm_fail(HTM_E_HIP, "%s: %s", __func__, hipGetErrorString(hipGetLastError()));
    *out_flags = f;
    return HTM_OK;
}

}  // extern "C"
