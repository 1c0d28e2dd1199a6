// mall_rw.hip -- calibration microbenchmark (not part of the product): does a buffer one
// kernel has just written come back faster than HBM when the next kernel reads it, i.e.
// does the 256 MB Infinity Cache (MALL) keep the Viterbi's decision words between k_acs2
// and k_traceback2?  For each size N: a streaming write of N bytes
// (16-byte stores, every CU), then a streaming read of the same N bytes; read bandwidth
// against a read of N bytes that were last written 2 GB of traffic ago (evicted).
// Prints N, the read-after-write rate, the cold read rate, the write rate (GB/s).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>
#include <algorithm>
#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; }      \
    } while (0)

__global__ __launch_bounds__(256) void k_write(uint4 *p, int64_t n, uint32_t v) {
    for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        p[i] = make_uint4(v, (uint32_t)i, v ^ 1u, (uint32_t)(i >> 32));
}
__global__ __launch_bounds__(256) void k_read(const uint4 *p, int64_t n, uint32_t *sink) {
    uint32_t acc = 0;
    for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;            // keeps the loads
}

int main() {
    const int64_t big = 2LL << 30;                       // the evicting buffer
    const std::vector<int64_t> sizes = {32LL << 20, 64LL << 20, 128LL << 20, 192LL << 20, 256LL << 20,
                                        384LL << 20, 512LL << 20, 1LL << 30, 3LL << 29};
    uint4 *buf = nullptr, *ev = nullptr;
    uint32_t *sink = nullptr;
    CK(hipMalloc(&buf, sizes.back()));
    CK(hipMalloc(&ev, big));
    CK(hipMalloc(&sink, 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const dim3 grid(256 * 8), blk(256);
    auto timed = [&](auto launch) -> float {
        float ms = 0;
        (void)hipEventRecord(a, 0);
        launch();
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
        return ms;
    };
    printf("%10s %14s %14s %14s   (GB/s, median of 7)\n", "MB", "read-after-write", "read-evicted", "write");
    for (int64_t n : sizes) {
        const int64_t nv = n / 16;
        std::vector<float> raw, cold, wr;
        for (int rep = 0; rep < 7; rep++) {
            wr.push_back(timed([&] { hipLaunchKernelGGL(k_write, grid, blk, 0, 0, buf, nv, (uint32_t)rep); }));
            raw.push_back(timed([&] { hipLaunchKernelGGL(k_read, grid, blk, 0, 0, buf, nv, sink); }));
            hipLaunchKernelGGL(k_write, grid, blk, 0, 0, ev, big / 16, (uint32_t)rep);     // evict
            hipLaunchKernelGGL(k_read, grid, blk, 0, 0, ev, big / 16, sink);
            cold.push_back(timed([&] { hipLaunchKernelGGL(k_read, grid, blk, 0, 0, buf, nv, sink); }));
        }
        CK(hipDeviceSynchronize());
        auto med = [](std::vector<float> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
        auto gbs = [&](float ms) { return (double)n / (ms * 1e-3) / 1e9; };
        printf("%10lld %14.0f %14.0f %14.0f\n", (long long)(n >> 20), gbs(med(raw)), gbs(med(cold)), gbs(med(wr)));
    }
    CK(hipFree(buf));
    CK(hipFree(ev));
    CK(hipFree(sink));
    return 0;
}
