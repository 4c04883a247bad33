// fetch_calib.hip -- calibration of the HBM byte counters on gfx950 for the
// access widths the frozen TM kernel issues (MI355X_MICROARCH.md, HBM
// section: "other access widths are uncalibrated: calibrate on a known byte
// count in your own access pattern").  Each kernel is one dispatch with a
// known request pattern over buffers far larger than L2; rocprofv3 --pmc
// passes record FETCH_SIZE / WRITE_SIZE and the L2 memory-side request
// counters by size (TCC_EA0_RDREQ_{32B,64B,128B}, TCC_EA0_WRREQ{,_64B}),
// and tools/pmc_summary.py --calib compares them with the bytes printed here.
//
// Patterns (the frozen kernel's mix):
//   cal_stream16  coalesced 16 B/lane loads (the guide's calibrated case)
//   cal_runs16    runs of 8 consecutive 16 B blocks at random 128 B-aligned
//                 starts, 8 lanes per run (out-list blocks)
//   cal_gather8   one random 8 B load per lane (fx_off offset pairs, fx_rec)
//   cal_gather4   one random 4 B load per lane (meta words, rslot)
//   cal_stream4   coalesced 4 B/lane loads
//   cal_wstream16 coalesced 16 B/lane stores
//   cal_wscatter4 one random 4 B store per lane (duty-cycle record writes)
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            std::exit(1);                                                          \
        }                                                                          \
    } while (0)

__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

// a data-dependent store that never happens keeps every load live without
// adding write traffic
__device__ __forceinline__ void sink(unsigned* out, unsigned v) {
    if (v == 0x9e3779b9u) out[threadIdx.x & 1023] = v;
}

__global__ void cal_stream16(const uint4* a, size_t n, unsigned* out) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    sink(out, acc);
}

__global__ void cal_runs16(const uint4* a, size_t nruns_space, size_t nruns, unsigned* out) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nruns * 8; i += (size_t)gridDim.x * blockDim.x) {
        const size_t run = i >> 3;
        const size_t start = (mix64(run) % nruns_space) * 8;  // 128 B aligned
        const uint4 v = a[start + (i & 7)];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    sink(out, acc);
}

__global__ void cal_gather8(const uint2* a, size_t space, size_t n, unsigned* out) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint2 v = a[mix64(i + 0x1234567ull) % space];
        acc += v.x ^ v.y;
    }
    sink(out, acc);
}

__global__ void cal_gather4(const unsigned* a, size_t space, size_t n, unsigned* out) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc += a[mix64(i + 0x89abcdefull) % space];
    sink(out, acc);
}

__global__ void cal_stream4(const unsigned* a, size_t n, unsigned* out) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc += a[i];
    sink(out, acc);
}

__global__ void cal_wstream16(uint4* a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = make_uint4((unsigned)i, 1u, 2u, 3u);
}

__global__ void cal_wscatter4(unsigned* a, size_t space, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[mix64(i + 0x55aa55aaull) % space] = (unsigned)i;
}

int main() {
    const size_t big = (size_t)1 << 30;   // 1 GiB random-access space
    const size_t strm = (size_t)1 << 28;  // 256 MiB streams
    void *A = nullptr, *B = nullptr;
    unsigned* out = nullptr;
    CHECK(hipMalloc(&A, big));
    CHECK(hipMalloc(&B, strm));
    CHECK(hipMalloc(&out, 1024 * 4));
    CHECK(hipMemset(A, 1, big));
    CHECK(hipMemset(B, 2, strm));
    CHECK(hipMemset(out, 0, 1024 * 4));
    CHECK(hipDeviceSynchronize());
    const dim3 grid(8192), blk(256);
    const size_t nruns = (size_t)1 << 20, ngath = (size_t)1 << 23;
    hipLaunchKernelGGL(cal_stream16, grid, blk, 0, 0, (const uint4*)B, strm / 16, out);
    hipLaunchKernelGGL(cal_runs16, grid, blk, 0, 0, (const uint4*)A, big / 128, nruns, out);
    hipLaunchKernelGGL(cal_gather8, grid, blk, 0, 0, (const uint2*)A, big / 8, ngath, out);
    hipLaunchKernelGGL(cal_gather4, grid, blk, 0, 0, (const unsigned*)A, big / 4, ngath, out);
    hipLaunchKernelGGL(cal_stream4, grid, blk, 0, 0, (const unsigned*)B, strm / 4, out);
    hipLaunchKernelGGL(cal_wstream16, grid, blk, 0, 0, (uint4*)B, strm / 16);
    hipLaunchKernelGGL(cal_wscatter4, grid, blk, 0, 0, (unsigned*)A, big / 4, ngath);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    // requested bytes per kernel (loads / stores issued by the lanes); the
    // random patterns touch (almost) one distinct line per request
    std::printf("{\"cal_stream16\": {\"read\": %zu}, \"cal_runs16\": {\"read\": %zu}, "
                "\"cal_gather8\": {\"read\": %zu}, \"cal_gather4\": {\"read\": %zu}, "
                "\"cal_stream4\": {\"read\": %zu}, \"cal_wstream16\": {\"write\": %zu}, "
                "\"cal_wscatter4\": {\"write\": %zu}}\n",
                strm, nruns * 128, ngath * 8, ngath * 4, strm, strm, ngath * 4);
    CHECK(hipFree(A));
    CHECK(hipFree(B));
    CHECK(hipFree(out));
    return 0;
}
