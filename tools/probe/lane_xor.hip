// Device check of pf_device.h's lane_xor32 / wave_sort64 / wave_min64 (DPP + permlane swaps):
// prints OK or the first mismatch.  hipcc --offload-arch=gfx950 -O3 -I csrc tools/probe/lane_xor.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>
#include "pf_device.h"
using namespace pf;
__global__ void probe(uint32_t* ox, uint64_t* os, uint64_t* om, const uint64_t* in) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int ms[7] = {1, 2, 4, 8, 15, 16, 32};
#pragma unroll
    for (int i = 0; i < 7; ++i) ox[(w * 7 + i) * 64 + lane] = lane_xor32((uint32_t)threadIdx.x, ms[i]);
    const uint64_t x = in[threadIdx.x];
    os[threadIdx.x] = wave_sort64(x, lane);
    om[threadIdx.x] = wave_min64(x);
}
int main() {
    const int n = 128;
    std::vector<uint64_t> in(n);
    srand(7);
    for (auto& v : in) v = ((uint64_t)rand() << 33) ^ ((uint64_t)rand() << 10) ^ (uint64_t)rand();
    in[5] = in[9];
    uint32_t* dx; uint64_t *ds, *dm, *di;
    hipMalloc(&dx, 2 * 7 * 64 * 4); hipMalloc(&ds, n * 8); hipMalloc(&dm, n * 8); hipMalloc(&di, n * 8);
    hipMemcpy(di, in.data(), n * 8, hipMemcpyHostToDevice);
    probe<<<1, n>>>(dx, ds, dm, di);
    std::vector<uint32_t> hx(2 * 7 * 64); std::vector<uint64_t> hs(n), hm(n);
    hipMemcpy(hx.data(), dx, hx.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(hs.data(), ds, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(hm.data(), dm, n * 8, hipMemcpyDeviceToHost);
    const int ms[7] = {1, 2, 4, 8, 15, 16, 32};
    int bad = 0;
    for (int w = 0; w < 2; ++w)
        for (int i = 0; i < 7; ++i)
            for (int l = 0; l < 64; ++l) {
                const uint32_t want = (uint32_t)(w * 64 + (l ^ ms[i])), got = hx[(w * 7 + i) * 64 + l];
                if (got != want && bad++ < 10) printf("xor %d lane %d: %u want %u\n", ms[i], w * 64 + l, got, want);
            }
    for (int w = 0; w < 2; ++w) {
        std::vector<uint64_t> v(in.begin() + 64 * w, in.begin() + 64 * (w + 1));
        std::sort(v.begin(), v.end());
        for (int l = 0; l < 64; ++l) {
            if (hs[64 * w + l] != v[l] && bad++ < 20) printf("sort wave %d lane %d\n", w, l);
            if (hm[64 * w + l] != v[0] && bad++ < 20) printf("min wave %d lane %d\n", w, l);
        }
    }
    printf(bad ? "FAIL %d\n" : "OK\n", bad);
    return bad ? 1 : 0;
}
