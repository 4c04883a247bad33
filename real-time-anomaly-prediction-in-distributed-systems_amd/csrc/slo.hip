// slo.hip -- the reference's SLO-violation prediction harness, batched over
// streams.
//
// Reference: ML/HTM/ModelTesting.py runModel :36-107 (per record: the 1 + 7
// anomaly scores of the network steps, any score > threshold -> predict 'A'
// unless it is the first record; SLO violation = violations > 0 or
// int(mean) >= 70), processpredictionList :113-146 (resolve pending
// predictions against the violation state within MAX_LEAD_TIME = 50
// records, TP lead time, the FN -> TN rewrite of the last 50 records) and
// getModelStats :148-171 (TP/FP/TN/FN and lead over predictionList[:-50]).
//
// MI355X design: one lane per stream (the harness is a short sequential
// state machine per stream; streams are independent).  The unbounded
// predictionList becomes a 64-entry ring of the newest items per stream
// (items older than 50 records can no longer change except by the pending
// -> FP/TN resolution, which is order-free and kept as two counters), in
// [64][streams] layout so each ring access is coalesced across lanes.
// Scores arrive as the engine writes them ([window][streams] float32) and
// are compared as double against the double threshold, like Python does
// with the Real32 output.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "htm_dev.h"

// item: bit 0 kind (1 = 'A'), bit 1 pending, bits 2-3 label, bits 8-15 lead
#define SLO_RING 64
enum { L_TP = 0, L_TN = 1, L_FP = 2, L_FN = 3 };

struct SloState {
    uint32_t* ring;      // [SLO_RING][n]
    int32_t* rcount;     // [n]
    int64_t* acc;        // [n][7]: tp, fp, tn, fn, lead sum, pending-A out of ring, pending-N out of ring
};

__device__ __forceinline__ uint32_t it_kind(uint32_t x) { return x & 1u; }
__device__ __forceinline__ uint32_t it_pending(uint32_t x) { return (x >> 1) & 1u; }
__device__ __forceinline__ uint32_t it_label(uint32_t x) { return (x >> 2) & 3u; }
__device__ __forceinline__ uint32_t it_make(uint32_t kind, uint32_t pending, uint32_t label, uint32_t lead) {
    return kind | (pending << 1) | (label << 2) | (lead << 8);
}

__global__ void slo_record_kernel(SloState st, int n, const float* scores, int w, const int32_t* violations,
                                  const int32_t* means, const uint8_t* valid, double threshold, int max_lead,
                                  int32_t slo_response) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    if (valid && !valid[s]) return;  // null cpu/mem: the record is skipped before rcount += 1 (:51-53)
    const int32_t rc = st.rcount[s] + 1;  // :62
    st.rcount[s] = rc;
    int nover = 0;  // :75-77
    for (int j = 0; j < w; j++) nover += ((double)scores[(size_t)j * n + s] > threshold) ? 1 : 0;
    const bool violation = violations[s] > 0 || means[s] >= slo_response;  // :57-60
    int64_t* acc = st.acc + (size_t)s * 7;
    // the item leaving the ring (record rc - 64) is final unless pending
    const int slot = (rc - 1) % SLO_RING;
    if (rc > SLO_RING) {
        const uint32_t old = st.ring[(size_t)slot * n + s];
        if (it_pending(old)) {
            acc[it_kind(old) ? 5 : 6] += 1;
        } else {
            const uint32_t lb = it_label(old);
            acc[lb == L_TP ? 0 : lb == L_FP ? 1 : lb == L_TN ? 2 : 3] += 1;
            if (lb == L_TP) acc[4] += old >> 8;
        }
    }
    // append (:81-99): 'A' (initial label TP) or 'N' (initial label TN), pending
    const uint32_t kindA = (nover > 0 && rc > 1) ? 1u : 0u;
    st.ring[(size_t)slot * n + s] = it_make(kindA, 1u, kindA ? L_TP : L_TN, 0u);
    // processpredictionList(state, rc) in list order, oldest first (:113-146)
    const int nring = rc < SLO_RING ? rc : SLO_RING;
    if (violation) {
        for (int a = nring - 1; a >= 0; a--) {  // a = age = rc - item's rcount
            const int sl = (rc - 1 - a) % SLO_RING;
            uint32_t x = st.ring[(size_t)sl * n + s];
            if (!it_pending(x) || a > max_lead) continue;
            if (!it_kind(x)) {
                st.ring[(size_t)sl * n + s] = it_make(0u, 0u, L_FN, 0u);
                continue;
            }
            st.ring[(size_t)sl * n + s] = it_make(1u, 0u, L_TP, (uint32_t)(max_lead - a));
            // predictionList[max(rc - max_lead, 0) : rc]: the items of age < max_lead
            for (int b = 0; b < max_lead && b < nring; b++) {
                const int sb = (rc - 1 - b) % SLO_RING;
                const uint32_t y = st.ring[(size_t)sb * n + s];
                if (it_label(y) == L_FN) st.ring[(size_t)sb * n + s] = (y & ~(3u << 2)) | ((uint32_t)L_TN << 2);
            }
        }
    } else {
        // pending items older than max_lead resolve: 'A' -> FP, 'N' -> TN
        acc[1] += acc[5];
        acc[2] += acc[6];
        acc[5] = 0;
        acc[6] = 0;
        for (int a = nring - 1; a > max_lead; a--) {
            const int sl = (rc - 1 - a) % SLO_RING;
            const uint32_t x = st.ring[(size_t)sl * n + s];
            if (!it_pending(x)) continue;
            st.ring[(size_t)sl * n + s] = it_kind(x) ? it_make(1u, 0u, L_FP, 0u) : it_make(0u, 0u, L_TN, 0u);
        }
    }
}

// getModelStats over predictionList[:-max_lead]: out[s] = {tp, fp, tn, fn, lead sum}
__global__ void slo_stats_kernel(SloState st, int n, int max_lead, int64_t* out) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    const int64_t* acc = st.acc + (size_t)s * 7;
    // out-of-ring items; pending ones still carry their initial label
    int64_t tp = acc[0] + acc[5], fp = acc[1], tn = acc[2] + acc[6], fn = acc[3], lead = acc[4];
    const int32_t rc = st.rcount[s];
    const int nring = rc < SLO_RING ? rc : SLO_RING;
    for (int a = nring - 1; a >= max_lead; a--) {  // items with index < rc - max_lead
        const uint32_t x = st.ring[(size_t)((rc - 1 - a) % SLO_RING) * n + s];
        const uint32_t lb = it_label(x);
        if (lb == L_TP) {
            tp++;
            lead += x >> 8;
        } else if (lb == L_FP) {
            fp++;
        } else if (lb == L_TN) {
            tn++;
        } else {
            fn++;
        }
    }
    int64_t* o = out + (size_t)s * 5;
    o[0] = tp;
    o[1] = fp;
    o[2] = tn;
    o[3] = fn;
    o[4] = lead;
}

struct htm_slo {
    int32_t n, device, max_lead, slo_response;
    double threshold;
    SloState st;
    int64_t* d_out;
};

extern "C" {

int htm_slo_create(int32_t n_streams, double threshold, int32_t max_lead, int32_t slo_response, int32_t device,
                   htm_slo** out) {
    if (!out || n_streams < 1 || max_lead < 0 || max_lead > SLO_RING - 2) return htm_fail(HTM_E_INVALID, "%s: invalid argument", __func__);
    *out = nullptr;
    if (hipSetDevice(device) != hipSuccess) return htm_fail(HTM_E_HIP, "%s: %s", __func__, hipGetErrorString(hipGetLastError()));
    htm_slo* h = new htm_slo();
    h->n = n_streams;
    h->device = device;
    h->max_lead = max_lead;
    h->slo_response = slo_response;
    h->threshold = threshold;
    const size_t n = (size_t)n_streams;
    bool ok = hipMalloc(&h->st.ring, n * SLO_RING * 4) == hipSuccess &&
              hipMalloc(&h->st.rcount, n * 4) == hipSuccess && hipMalloc(&h->st.acc, n * 7 * 8) == hipSuccess &&
              hipMalloc(&h->d_out, n * 5 * 8) == hipSuccess;
    ok = ok && hipMemset(h->st.ring, 0, n * SLO_RING * 4) == hipSuccess &&
         hipMemset(h->st.rcount, 0, n * 4) == hipSuccess && hipMemset(h->st.acc, 0, n * 7 * 8) == hipSuccess;
    if (!ok) {
        htm_slo_destroy(h);
        return htm_fail(HTM_E_HIP, "%s: %s", __func__, hipGetErrorString(hipGetLastError()));
    }
    *out = h;
    return HTM_OK;
}

int htm_slo_destroy(htm_slo* h) {
    if (!h) return HTM_OK;
    (void)hipSetDevice(h->device);
    (void)hipDeviceSynchronize();
    if (h->st.ring) (void)hipFree(h->st.ring);
    if (h->st.rcount) (void)hipFree(h->st.rcount);
    if (h->st.acc) (void)hipFree(h->st.acc);
    if (h->d_out) (void)hipFree(h->d_out);
    delete h;
    return HTM_OK;
}

int htm_slo_record(htm_slo* h, const float* d_scores, int32_t window, const int32_t* d_violations,
                   const int32_t* d_means, const uint8_t* d_valid, void* stream) {
    if (!h || !d_scores || window < 1 || !d_violations || !d_means) return htm_fail(HTM_E_INVALID, "%s: invalid argument", __func__);
    hipLaunchKernelGGL(slo_record_kernel, dim3((h->n + 255) / 256), dim3(256), 0, (hipStream_t)stream, h->st, h->n,
                       d_scores, window, d_violations, d_means, d_valid, h->threshold, h->max_lead,
                       h->slo_response);
    return hipGetLastError() == hipSuccess ? HTM_OK : htm_fail(HTM_E_HIP, "%s: HIP launch/sync failed", __func__);
}

int htm_slo_stats(htm_slo* h, int64_t* h_out5, void* stream) {
    if (!h || !h_out5) return htm_fail(HTM_E_INVALID, "%s: invalid argument", __func__);
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(slo_stats_kernel, dim3((h->n + 255) / 256), dim3(256), 0, st, h->st, h->n, h->max_lead,
                       h->d_out);
    if (hipGetLastError() != hipSuccess) return htm_fail(HTM_E_HIP, "%s: %s", __func__, hipGetErrorString(hipGetLastError()));
    if (hipMemcpyAsync(h_out5, h->d_out, (size_t)h->n * 5 * 8, hipMemcpyDeviceToHost, st) != hipSuccess)
        return htm_fail(HTM_E_HIP, "%s: %s", __func__, hipGetErrorString(hipGetLastError()));
    return hipStreamSynchronize(st) == hipSuccess ? HTM_OK : htm_fail(HTM_E_HIP, "%s: HIP launch/sync failed", __func__);
}

}  // extern "C"
