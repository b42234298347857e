// tools/microbench/concurrency.hip -- do two kernels on two HIP streams run at the same time on this box?
// Each kernel is one workgroup that spins ~T ms on the shader clock (s_memrealtime, 100 MHz): run serially the
// pair takes ~2T, concurrently ~T. Variants: non-blocking streams, default streams, and with timing events
// recorded around each launch (as the executor records them).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                                  \
    do {                                                                                                       \
        hipError_t err_ = (x);                                                                                    \
        if (err_ != hipSuccess) {                                                                                 \
            std::printf("%s: %s\n", #x, hipGetErrorString(err_));                                                 \
            std::exit(1);                                                                                      \
        }                                                                                                      \
    } while (0)

__global__ void spin(unsigned long long ticks, int *out)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long t = t0;
    int n = 0;
    while (t - t0 < ticks) { // bounded: every wave leaves after `ticks` of the 100 MHz clock
        t = __builtin_amdgcn_s_memrealtime();
        ++n;
    }
    if (threadIdx.x == 0)
        out[blockIdx.x] = n;
}

static double run(hipStream_t a, hipStream_t b, int blocks, unsigned long long ticks, int *d, bool events)
{
    hipEvent_t e[4];
    for (auto &x : e)
        CK(hipEventCreate(&x));
    CK(hipDeviceSynchronize());
    const auto t0 = std::chrono::steady_clock::now();
    if (events)
        CK(hipEventRecord(e[0], a));
    hipLaunchKernelGGL(spin, dim3(blocks), dim3(64), 0, a, ticks, d);
    if (events) {
        CK(hipEventRecord(e[1], a));
        CK(hipEventRecord(e[2], b));
    }
    hipLaunchKernelGGL(spin, dim3(blocks), dim3(64), 0, b, ticks, d + blocks);
    if (events)
        CK(hipEventRecord(e[3], b));
    CK(hipDeviceSynchronize());
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    for (auto &x : e)
        CK(hipEventDestroy(x));
    return ms;
}

int main()
{
    int *d = nullptr;
    CK(hipMalloc(&d, sizeof(int) * 1 << 20));
    const unsigned long long ticks = 100000ull * 50; // 50 ms at 100 MHz
    hipStream_t n1, n2, b1, b2;
    CK(hipStreamCreateWithFlags(&n1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&n2, hipStreamNonBlocking));
    CK(hipStreamCreate(&b1));
    CK(hipStreamCreate(&b2));
    run(n1, n2, 1, ticks / 10, d, false); // warm-up
    const char *env[] = {"GPU_MAX_HW_QUEUES", "AMD_SERIALIZE_KERNEL", "AMD_SERIALIZE_COPY", "HIP_LAUNCH_BLOCKING",
                         "HIP_VISIBLE_DEVICES", "HSA_ENABLE_SDMA", "GPU_ENABLE_LC", "HSA_CU_MASK"};
    for (const char *k : env)
        std::printf("%s=%s\n", k, std::getenv(k) ? std::getenv(k) : "(unset)");
    std::printf("one kernel alone (50 ms): %.1f ms\n", run(n1, n1, 1, ticks, d, false) / 2.0);
    std::printf("non-blocking streams, 1 WG each: %.1f ms (serial ~100, concurrent ~50)\n", run(n1, n2, 1, ticks, d, false));
    std::printf("non-blocking streams + timing events: %.1f ms\n", run(n1, n2, 1, ticks, d, true));
    std::printf("blocking streams: %.1f ms\n", run(b1, b2, 1, ticks, d, false));
    std::printf("non-blocking streams, 256 WG each: %.1f ms\n", run(n1, n2, 256, ticks, d, false));
    std::printf("non-blocking streams, 2048 WG each: %.1f ms\n", run(n1, n2, 2048, ticks, d, false));
    // many streams: is the k-th stream on the same hardware queue as the first?
    hipStream_t s[8];
    for (auto &x : s)
        CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    for (int k = 1; k < 8; ++k)
        std::printf("stream 0 + stream %d: %.1f ms\n", k, run(s[0], s[k], 1, ticks, d, false));
    // a high-priority stream and a CU-masked stream (all CUs): do they get a hardware queue of their own?
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    hipStream_t hp, cm;
    CK(hipStreamCreateWithPriority(&hp, hipStreamNonBlocking, hi));
    std::vector<uint32_t> mask(8, 0xFFFFFFFFu);
    CK(hipExtStreamCreateWithCUMask(&cm, (uint32_t)mask.size(), mask.data()));
    std::printf("priority range [%d, %d]\n", lo, hi);
    for (int k = 0; k < 4; ++k)
        std::printf("high-priority + stream %d: %.1f ms; CU-masked + stream %d: %.1f ms\n", k,
                    run(hp, s[k], 1, ticks, d, false), k, run(cm, s[k], 1, ticks, d, false));
    std::printf("high-priority + CU-masked: %.1f ms\n", run(hp, cm, 1, ticks, d, false));
    return 0;
}
