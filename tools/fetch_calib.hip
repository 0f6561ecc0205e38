// fetch_calib.hip — calibrates rocprofv3's FETCH_SIZE against known byte counts for the
// load widths and access shapes of the postings scan (K5, pf_kernels.hip), as
// MI355X_MICROARCH.md (HBM section) asks before an absolute is trusted: "Other access
// widths are uncalibrated: calibrate on a known byte count in your own access pattern".
//
// Every kernel reads a distinct region of a 2 GiB buffer (past the 256 MiB Infinity Cache,
// so no re-read is served on-die) exactly once and writes one word per workgroup:
//   w4_stream   4 B / lane, one coalesced stream            (list entries, long lists)
//   w8_stream   8 B / lane, one coalesced stream            (entry norms, long lists)
//   w16_stream 16 B / lane, one coalesced stream            (the guide's calibrated case)
//   w4_runs     4 B / lane, runs of 32 entries at scattered 128-B-aligned offsets
//   w8_runs     8 B / lane, runs of 32 entries at scattered offsets (norms of short lists)
// It prints one JSON line: kernel -> bytes read per launch.  tools/fetch_calib.py joins it
// with the FETCH_SIZE rows of the rocprofv3 pass and reports bytes / (FETCH_SIZE KiB * 1024).
//
//   hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/fetch_calib
//   rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d OUT -o run -- tools/fetch_calib
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            return 1;                                                             \
        }                                                                         \
    } while (0)

constexpr int kThreads = 256;

template <class T>
__device__ __forceinline__ uint32_t fold(const T& v);
template <>
__device__ __forceinline__ uint32_t fold<uint32_t>(const uint32_t& v) { return v; }
template <>
__device__ __forceinline__ uint32_t fold<uint2>(const uint2& v) { return v.x ^ v.y; }
template <>
__device__ __forceinline__ uint32_t fold<uint4>(const uint4& v) { return v.x ^ v.y ^ v.z ^ v.w; }

// elements [0, n) of p, grid-stride, one element per lane per step
template <class T>
__device__ __forceinline__ void stream_body(const T* __restrict__ p, uint64_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kThreads)
        acc ^= fold(p[i]);
    acc = __reduce_or_sync(0xFFFFFFFFFFFFFFFFull, acc);
    if (threadIdx.x == 0) out[blockIdx.x] = acc;
}

// runs of 32 elements starting at run_off[r] (element index), one run per half-wave
template <class T>
__device__ __forceinline__ void runs_body(const T* __restrict__ p, const uint64_t* __restrict__ run_off,
                                          uint32_t nruns, uint32_t* out) {
    uint32_t acc = 0;
    const uint32_t per_block = kThreads / 32;
    for (uint32_t r0 = blockIdx.x * per_block; r0 < nruns; r0 += gridDim.x * per_block) {
        const uint32_t r = r0 + threadIdx.x / 32;
        if (r < nruns) acc ^= fold(p[run_off[r] + (threadIdx.x & 31)]);
    }
    acc = __reduce_or_sync(0xFFFFFFFFFFFFFFFFull, acc);
    if (threadIdx.x == 0) out[blockIdx.x] = acc;
}

__global__ __launch_bounds__(kThreads) void w4_stream(const uint32_t* p, uint64_t n, uint32_t* out) { stream_body(p, n, out); }
__global__ __launch_bounds__(kThreads) void w8_stream(const uint2* p, uint64_t n, uint32_t* out) { stream_body(p, n, out); }
__global__ __launch_bounds__(kThreads) void w16_stream(const uint4* p, uint64_t n, uint32_t* out) { stream_body(p, n, out); }
__global__ __launch_bounds__(kThreads) void w4_runs(const uint32_t* p, const uint64_t* o, uint32_t nr, uint32_t* out) {
    runs_body(p, o, nr, out);
}
__global__ __launch_bounds__(kThreads) void w8_runs(const uint2* p, const uint64_t* o, uint32_t nr, uint32_t* out) {
    runs_body(p, o, nr, out);
}

int main() {
    const size_t buf = (size_t)2 << 30;  // 2 GiB: each kernel reads its own 384 MiB region
    const size_t region = (size_t)384 << 20;
    uint8_t* d = nullptr;
    uint32_t* out = nullptr;
    CK(hipMalloc(&d, buf));
    CK(hipMemset(d, 0x5A, buf));
    CK(hipMalloc(&out, 1 << 20));
    const int grid = 4096;
    // scattered runs: 32 elements each, at 128-B-aligned offsets spread over a region
    auto make_runs = [&](size_t elem, size_t nruns, uint64_t seed) {
        std::vector<uint64_t> off(nruns);
        const size_t span = region / elem - 32;
        uint64_t x = seed;
        for (size_t r = 0; r < nruns; ++r) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            off[r] = ((x >> 17) % (span / (128 / elem))) * (128 / elem);
        }
        return off;
    };
    // runs kept sparse enough that two runs rarely share a 128-B line (1 run per ~4 KiB)
    const size_t nruns4 = region / 4096, nruns8 = region / 4096;
    std::vector<uint64_t> r4 = make_runs(4, nruns4, 1), r8 = make_runs(8, nruns8, 2);
    uint64_t *d_r4 = nullptr, *d_r8 = nullptr;
    CK(hipMalloc(&d_r4, r4.size() * 8));
    CK(hipMalloc(&d_r8, r8.size() * 8));
    CK(hipMemcpy(d_r4, r4.data(), r4.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_r8, r8.data(), r8.size() * 8, hipMemcpyHostToDevice));
    // distinct lines touched by the runs (what a line-granular fetch must move)
    auto lines_of = [&](const std::vector<uint64_t>& off, size_t elem) {
        std::vector<uint64_t> ls;
        for (uint64_t o : off)
            for (uint64_t b = o * elem / 128; b <= ((o + 32) * elem - 1) / 128; ++b) ls.push_back(b);
        std::sort(ls.begin(), ls.end());
        return (uint64_t)(std::unique(ls.begin(), ls.end()) - ls.begin());
    };
    const uint64_t lines4 = lines_of(r4, 4), lines8 = lines_of(r8, 8);
    const int reps = 5;
    for (int rep = 0; rep < reps; ++rep) {
        hipLaunchKernelGGL(w4_stream, dim3(grid), dim3(kThreads), 0, 0,
                           reinterpret_cast<const uint32_t*>(d + 0 * region), region / 4, out);
        hipLaunchKernelGGL(w8_stream, dim3(grid), dim3(kThreads), 0, 0,
                           reinterpret_cast<const uint2*>(d + 1 * region), region / 8, out);
        hipLaunchKernelGGL(w16_stream, dim3(grid), dim3(kThreads), 0, 0,
                           reinterpret_cast<const uint4*>(d + 2 * region), region / 16, out);
        hipLaunchKernelGGL(w4_runs, dim3(grid), dim3(kThreads), 0, 0,
                           reinterpret_cast<const uint32_t*>(d + 3 * region), d_r4, (uint32_t)nruns4, out);
        hipLaunchKernelGGL(w8_runs, dim3(grid), dim3(kThreads), 0, 0,
                           reinterpret_cast<const uint2*>(d + 4 * region), d_r8, (uint32_t)nruns8, out);
        CK(hipDeviceSynchronize());
    }
    // the stream kernels read `region` bytes; the runs kernels 32 elements per run plus the
    // 8-B run offsets (read coalesced); lines_* = 128-B lines the runs touch
    printf("{\"w4_stream\": {\"bytes\": %zu}, \"w8_stream\": {\"bytes\": %zu}, \"w16_stream\": {\"bytes\": %zu}, "
           "\"w4_runs\": {\"bytes\": %zu, \"line_bytes\": %llu}, "
           "\"w8_runs\": {\"bytes\": %zu, \"line_bytes\": %llu}, \"reps\": %d}\n",
           region, region, region, nruns4 * (32 * 4 + 8), (unsigned long long)(lines4 * 128 + nruns4 * 8),
           nruns8 * (32 * 8 + 8), (unsigned long long)(lines8 * 128 + nruns8 * 8), reps);
    CK(hipFree(d));
    CK(hipFree(out));
    CK(hipFree(d_r4));
    CK(hipFree(d_r8));
    return 0;
}
