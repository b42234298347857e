// tools/microbench/memlat.hip -- what a box's memory system does for the search's access pattern, to compare
// boxes (the same search build runs 149-171 ms at C5 on different MI355X boxes):
//   * dependent random 8-B loads (a pointer chase per wave, 5120 waves like the search grid) over footprints of
//     256 MB .. 32 GB: average latency per hop in ns (TLB reach and DRAM latency show up as the footprint grows);
//   * a streaming read of 8 GB: GB/s.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                                  \
    do {                                                                                                       \
        hipError_t err_ = (x);                                                                                 \
        if (err_ != hipSuccess) {                                                                              \
            std::printf("%s: %s\n", #x, hipGetErrorString(err_));                                              \
            std::exit(1);                                                                                      \
        }                                                                                                      \
    } while (0)

// one chain per wave (lane 0 drives, the other lanes idle), `hops` dependent loads; bounded loop
__global__ void chase(const uint64_t *buf, uint64_t nwords, int hops, uint64_t *sink)
{
    uint64_t idx = ((uint64_t)blockIdx.x * 0x9E3779B97F4A7C15ull) % nwords;
    uint64_t acc = 0;
    if (threadIdx.x == 0) {
        for (int h = 0; h < hops; ++h) {
            const uint64_t v = __hip_atomic_load(buf + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            acc += v;
            idx = (v ^ (idx * 0x2545F4914F6CDD1Dull)) % nwords;
        }
        sink[blockIdx.x] = acc;
    }
}

__global__ void fill(uint64_t *buf, uint64_t n)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        buf[i] = i * 0x9E3779B97F4A7C15ull + 12345;
}

__global__ void stream(const uint4 *buf, uint64_t n, uint32_t *sink)
{
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 v = buf[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u)
        sink[0] = acc;
}

int main()
{
    const uint64_t max_bytes = 32ull << 30;
    uint64_t *buf = nullptr, *sink = nullptr;
    CK(hipMalloc(&buf, max_bytes));
    CK(hipMalloc(&sink, sizeof(uint64_t) * 8192));
    hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, buf, max_bytes / 8);
    CK(hipDeviceSynchronize());
    const int waves = 5120, hops = 2000;
    for (uint64_t fp = 256ull << 20; fp <= max_bytes; fp *= 4) {
        hipLaunchKernelGGL(chase, dim3(waves), dim3(64), 0, 0, buf, fp / 8, 50, sink); // warm
        CK(hipDeviceSynchronize());
        const auto t0 = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(chase, dim3(waves), dim3(64), 0, 0, buf, fp / 8, hops, sink);
        CK(hipDeviceSynchronize());
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::printf("pointer chase, %d waves, footprint %6.2f GB: %.0f ns per dependent load, %.2f G loads/s\n", waves,
                    fp / 1073741824.0, s / hops * 1e9, (double)waves * hops / s / 1e9);
    }
    const uint64_t sb = 8ull << 30;
    hipLaunchKernelGGL(stream, dim3(8192), dim3(256), 0, 0, (const uint4 *)buf, sb / 16, (uint32_t *)sink);
    CK(hipDeviceSynchronize());
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < 5; ++r)
        hipLaunchKernelGGL(stream, dim3(8192), dim3(256), 0, 0, (const uint4 *)buf, sb / 16, (uint32_t *)sink);
    CK(hipDeviceSynchronize());
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("streaming read 8 GB: %.0f GB/s\n", 5.0 * sb / s / 1e9);
    return 0;
}
