// likelihood.hip -- AnomalyLikelihood for N streams (north-star extension,
// SURVEY.md §8(a) row a13; parity unpinned: the reference never computes it).
//
// Restates NuPIC 1.0.x nupic/algorithms/anomaly_likelihood.py as described
// in oracle/likelihood_reference.py: a probation period returning 0.5, a
// normal distribution of the raw score's 10-record moving average
// re-estimated every `reestimation` records from the last `historic`
// records (minus a learning-period prefix), the Gaussian tail probability of
// each new moving average, NuPIC's red/yellow filter, likelihood = 1 - tail.
//
// MI355X design: one 256-thread workgroup per stream.  The per-record update
// is a handful of double operations on thread 0; the re-estimation (every
// 100 records, over up to 8,640 records) stages the stream's score ring in
// LDS and reduces the moving averages' and metric values' moments across the
// workgroup in double.  Moving averages are fresh 10-term sums, not NuPIC's
// running total (differences ~1e-16 relative; the contract is 1e-6).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "htm_dev.h"

#define LK_WIN 10
#define LK_HWCAP 8640
#define LK_RED (1.0 - 0.99999)
#define LK_YELLOW (1.0 - 0.999)

struct LkState {
    int32_t iteration, n_hist, head, have_dist;
    int32_t ma_n, ma_start, hl_n, hl_start;
    double mean, stdev, ma_total;
    double ma_vals[LK_WIN];  // ring, oldest at ma_start
    double hl[LK_WIN];       // unfiltered tail probabilities, ring, oldest at hl_start
};

struct LkBufs {
    LkState* st;    // [S]
    float* hs;      // [S][hw] raw scores (ring)
    double* hv;     // [S][hw] metric values (ring)
    int32_t lp, es, hw, rp, n;
};

__device__ __forceinline__ double lk_tail(double x, double mean, double stdev) {
    if (x < mean) x = 2.0 * mean - x;
    const double z = (x - mean) / stdev;
    return 0.5 * erfc(z / 1.4142);
}

// workgroup sum of doubles (256 threads)
__device__ __forceinline__ double lk_sum(double v, double* red) {
    red[threadIdx.x] = v;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    const double r = red[0];
    __syncthreads();
    return r;
}

__global__ __launch_bounds__(256) void lk_step_kernel(LkBufs b, const double* values, int vstride,
                                                      const float* scores, double* out) {
    const int s = blockIdx.x;
    __shared__ LkState L;
    __shared__ float sc[LK_HWCAP];
    __shared__ double red[256];
    if (threadIdx.x == 0) L = b.st[s];
    __syncthreads();
    const bool probation = L.iteration < b.lp + b.es;
    const bool est = !probation && (!L.have_dist || L.iteration % b.rp == 0);
    if (est) {
        const int n = L.n_hist;
        const int shifted = L.iteration - b.hw > 0 ? L.iteration - b.hw : 0;
        int skip = b.lp - shifted > 0 ? b.lp - shifted : 0;
        skip = skip < L.iteration ? skip : L.iteration;
        const float* hs = b.hs + (size_t)s * b.hw;
        const double* hv = b.hv + (size_t)s * b.hw;
        for (int j = threadIdx.x; j < n; j += 256) sc[j] = hs[(L.head + j) % b.hw];  // oldest first
        __syncthreads();
        double sa = 0.0, sv = 0.0;
        for (int j = skip + (int)threadIdx.x; j < n; j += 256) {
            const int j0 = j - (LK_WIN - 1) > 0 ? j - (LK_WIN - 1) : 0;
            double t = 0.0;
            for (int k = j0; k <= j; k++) t += (double)sc[k];
            sa += t / (double)(j - j0 + 1);
            sv += hv[(L.head + j) % b.hw];
        }
        const int m = n - skip;
        const double mean_a = m > 0 ? lk_sum(sa, red) / m : 0.0;
        const double mean_v = m > 0 ? lk_sum(sv, red) / m : 0.0;
        double qa = 0.0, qv = 0.0;
        for (int j = skip + (int)threadIdx.x; j < n; j += 256) {
            const int j0 = j - (LK_WIN - 1) > 0 ? j - (LK_WIN - 1) : 0;
            double t = 0.0;
            for (int k = j0; k <= j; k++) t += (double)sc[k];
            const double a = t / (double)(j - j0 + 1) - mean_a;
            const double v = hv[(L.head + j) % b.hw] - mean_v;
            qa += a * a;
            qv += v * v;
        }
        const double var_a = m > 0 ? lk_sum(qa, red) / m : 0.0;
        const double var_v = m > 0 ? lk_sum(qv, red) / m : 0.0;
        if (threadIdx.x == 0) {
            if (m <= 0 || var_v < 1.5e-5) {  // nullDistribution
                L.mean = 0.5;
                L.stdev = 1e3;
            } else {
                L.mean = mean_a < 0.03 ? 0.03 : mean_a;
                L.stdev = sqrt(var_a < 0.0003 ? 0.0003 : var_a);
            }
            L.have_dist = 1;
            // the moving-average window continues from the history's last records
            const int w = n < LK_WIN ? n : LK_WIN;
            L.ma_n = w;
            L.ma_start = 0;
            double tot = 0.0;
            for (int k = 0; k < w; k++) {
                L.ma_vals[k] = (double)sc[n - w + k];
                tot += L.ma_vals[k];
            }
            L.ma_total = tot;
            // tail probabilities of the history's last (<= 10) moving averages
            L.hl_n = w;
            L.hl_start = 0;
            for (int k = 0; k < w; k++) {
                const int j = n - w + k;
                const int j0 = j - (LK_WIN - 1) > 0 ? j - (LK_WIN - 1) : 0;
                double t = 0.0;
                for (int q = j0; q <= j; q++) t += (double)sc[q];
                L.hl[k] = lk_tail(t / (double)(j - j0 + 1), L.mean, L.stdev);
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const double score = (double)scores[s];
        const double value = values[(size_t)s * vstride];
        double lik = 0.5;
        if (!probation) {
            // MovingAverage.compute
            if (L.ma_n == LK_WIN) {
                L.ma_total -= L.ma_vals[L.ma_start];
                L.ma_start = (L.ma_start + 1) % LK_WIN;
                L.ma_n--;
            }
            L.ma_vals[(L.ma_start + L.ma_n) % LK_WIN] = score;
            L.ma_n++;
            L.ma_total += score;
            const double avg = L.ma_total / (double)L.ma_n;
            const double p = lk_tail(avg, L.mean, L.stdev);
            double filt = p;
            if (L.hl_n > 0 && p <= LK_RED) {
                const double prev = L.hl[(L.hl_start + L.hl_n - 1) % LK_WIN];
                filt = prev > LK_RED ? p : LK_YELLOW;
            }
            if (L.hl_n == LK_WIN) {
                L.hl_start = (L.hl_start + 1) % LK_WIN;
                L.hl_n--;
            }
            L.hl[(L.hl_start + L.hl_n) % LK_WIN] = p;
            L.hl_n++;
            lik = 1.0 - filt;
        }
        // history deque (maxlen hw)
        int idx;
        if (L.n_hist < b.hw) {
            idx = (L.head + L.n_hist) % b.hw;
            L.n_hist++;
        } else {
            idx = L.head;
            L.head = (L.head + 1) % b.hw;
        }
        b.hs[(size_t)s * b.hw + idx] = (float)score;
        b.hv[(size_t)s * b.hw + idx] = value;
        L.iteration++;
        out[s] = lik;
        b.st[s] = L;
    }
}

struct htm_likelihood {
    LkBufs b;
    int32_t device;
};

extern "C" {

int htm_likelihood_create(int32_t n_streams, int32_t learning_period, int32_t estimation_samples,
                          int32_t historic_window, int32_t reestimation_period, int32_t device, htm_likelihood** out) {
    if (!out || n_streams < 1 || learning_period < 0 || estimation_samples < 0 || historic_window < 1 ||
        historic_window > LK_HWCAP || reestimation_period < 1)
        return htm_fail(HTM_E_INVALID, "%s: invalid argument", __func__);
    *out = nullptr;
    if (hipSetDevice(device) != hipSuccess) return htm_fail(HTM_E_HIP, "%s: %s", __func__, hipGetErrorString(hipGetLastError()));
    htm_likelihood* h = new htm_likelihood();
    h->device = device;
    h->b.lp = learning_period;
    h->b.es = estimation_samples;
    h->b.hw = historic_window;
    h->b.rp = reestimation_period;
    h->b.n = n_streams;
    const size_t n = (size_t)n_streams, hw = (size_t)historic_window;
    bool ok = hipMalloc(&h->b.st, n * sizeof(LkState)) == hipSuccess &&
              hipMalloc(&h->b.hs, n * hw * 4) == hipSuccess && hipMalloc(&h->b.hv, n * hw * 8) == hipSuccess;
    ok = ok && hipMemset(h->b.st, 0, n * sizeof(LkState)) == hipSuccess;
    if (!ok) {
        htm_likelihood_destroy(h);
        return htm_fail(HTM_E_HIP, "%s: %s", __func__, hipGetErrorString(hipGetLastError()));
    }
    *out = h;
    return HTM_OK;
}

int htm_likelihood_destroy(htm_likelihood* h) {
    if (!h) return HTM_OK;
    (void)hipSetDevice(h->device);
    (void)hipDeviceSynchronize();
    if (h->b.st) (void)hipFree(h->b.st);
    if (h->b.hs) (void)hipFree(h->b.hs);
    if (h->b.hv) (void)hipFree(h->b.hv);
    delete h;
    return HTM_OK;
}

int htm_likelihood_step(htm_likelihood* h, const double* d_values, int32_t value_stride, const float* d_scores,
                        double* d_out, void* stream) {
    if (!h || !d_values || !d_scores || !d_out || value_stride < 1) return htm_fail(HTM_E_INVALID, "%s: invalid argument", __func__);
    hipLaunchKernelGGL(lk_step_kernel, dim3(h->b.n), dim3(256), 0, (hipStream_t)stream, h->b, d_values,
                       value_stride, d_scores, d_out);
    return hipGetLastError() == hipSuccess ? HTM_OK : htm_fail(HTM_E_HIP, "%s: HIP launch/sync failed", __func__);
}

}  // extern "C"
