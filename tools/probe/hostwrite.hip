// Probe: can the host write device memory directly (fine-grained device allocation), and what does a
// per-launch 9-KB upload cost that way vs hipMemcpyAsync from pinned memory?  Prints timings.
// hipcc --offload-arch=gfx950 -O2 tools/probe/hostwrite.hip -o tools/probe/hostwrite
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>
__global__ void consume(const unsigned* img, unsigned n, unsigned* out, unsigned step) {
    __shared__ unsigned acc;
    if (threadIdx.x == 0) acc = 0;
    __syncthreads();
    unsigned s = 0;
    for (unsigned i = threadIdx.x; i < n; i += blockDim.x) s += img[i];
    atomicAdd(&acc, s);
    __syncthreads();
    if (threadIdx.x == 0 && blockIdx.x == 0) out[step] = acc;
}
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("ERR %s at %d: %s\n", #x, __LINE__, hipGetErrorString(e)); return 1; } } while (0)
int main() {
    const unsigned n = 9 * 1024 / 4, steps = 200;
    hipStream_t s; CK(hipStreamCreate(&s));
    unsigned *dev, *out, *pin, *fg = nullptr;
    CK(hipMalloc(&dev, n * 4)); CK(hipMalloc(&out, steps * 4));
    CK(hipHostMalloc(&pin, n * 4));
    hipError_t e = hipExtMallocWithFlags((void**)&fg, n * 4 * 4, hipDeviceMallocFinegrained);
    printf("fine-grained alloc: %s\n", hipGetErrorString(e));
    hipPointerAttribute_t at{};
    if (e == hipSuccess && hipPointerGetAttributes(&at, fg) == hipSuccess)
        printf("attrs: type %d hostPointer %p devicePointer %p\n", (int)at.type, at.hostPointer, at.devicePointer);
    std::vector<unsigned> want(steps);
    unsigned* pins[4];
    for (auto& q : pins) CK(hipHostMalloc(&q, n * 4));
    hipEvent_t ev[4];
    for (auto& x : ev) CK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
    auto run = [&](int mode) -> double {
        CK(hipDeviceSynchronize());
        auto t0 = std::chrono::steady_clock::now();
        for (unsigned i = 0; i < steps; ++i) {
            unsigned sum = 0;
            const int r = i & 3;
            if (i >= 4) CK(hipEventSynchronize(ev[r]));  // the slot's previous launch is done
            unsigned* hostw = mode == 0 ? pins[r] : fg + r * n;
            for (unsigned j = 0; j < n; ++j) { hostw[j] = i + j; sum += i + j; }
            if (mode == 0) {
                CK(hipMemcpyAsync(dev + 0, pins[r], n * 4, hipMemcpyHostToDevice, s));
                consume<<<1024, 256, 0, s>>>(dev, n, out, i);
            } else {
                __atomic_thread_fence(__ATOMIC_SEQ_CST);
                consume<<<1024, 256, 0, s>>>(fg + r * n, n, out, i);
            }
            CK(hipEventRecord(ev[r], s));
            want[i] = sum;
        }
        CK(hipStreamSynchronize(s));
        auto t1 = std::chrono::steady_clock::now();
        std::vector<unsigned> got(steps);
        CK(hipMemcpy(got.data(), out, steps * 4, hipMemcpyDeviceToHost));
        int bad = 0;
        for (unsigned i = 0; i < steps; ++i) bad += got[i] != want[i];
        printf("mode %d: %.2f us/step, mismatches %d\n", mode, std::chrono::duration<double, std::micro>(t1 - t0).count() / steps, bad);
        return 0;
    };
    run(0); run(0);
    if (e == hipSuccess) { run(1); run(1); }
    printf("done\n");
    return 0;
}
