// tools/microbench/placement.hip -- where do one-wave workgroups land? Every wave spins 20 ms (so the whole
// grid is resident at once) and records its hardware id (s_getreg HW_ID: SIMD, CU, SE; XCC_ID); the host prints
// how many waves share a SIMD, for grids of 1-wave and 4-wave workgroups at 1 and 2 waves per SIMD.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

#define CK(x)                                                                                                  \
    do {                                                                                                       \
        hipError_t err_ = (x);                                                                                 \
        if (err_ != hipSuccess) {                                                                              \
            std::printf("%s: %s\n", #x, hipGetErrorString(err_));                                              \
            std::exit(1);                                                                                      \
        }                                                                                                      \
    } while (0)

__global__ void where(unsigned long long ticks, unsigned *out)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    }
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20); // HW_REG_XCC_ID
    if ((threadIdx.x & 63) == 0)
        out[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = (hw & 0xFFFFu) | ((xcc & 0xFu) << 16);
}

static void run(int blocks, int threads)
{
    const int waves = blocks * threads / 64;
    unsigned *d = nullptr;
    CK(hipMalloc(&d, sizeof(unsigned) * waves));
    hipLaunchKernelGGL(where, dim3(blocks), dim3(threads), 0, 0, 100000ull * 20, d);
    CK(hipDeviceSynchronize());
    std::vector<unsigned> h(waves);
    CK(hipMemcpy(h.data(), d, sizeof(unsigned) * waves, hipMemcpyDeviceToHost));
    CK(hipFree(d));
    std::map<unsigned, int> per_simd, per_cu;
    for (unsigned v : h) {
        const unsigned simd = (v >> 4) & 3, cu = (v >> 8) & 15, sh = (v >> 12) & 1, se = (v >> 13) & 7, xcc = v >> 16;
        const unsigned cuid = (((xcc * 8 + se) * 2 + sh) * 16 + cu);
        per_simd[cuid * 4 + simd]++;
        per_cu[cuid]++;
    }
    std::map<int, int> hs, hc;
    for (auto &p : per_simd)
        hs[p.second]++;
    for (auto &p : per_cu)
        hc[p.second]++;
    std::printf("%d blocks x %d threads: %zu CUs, %zu SIMDs used; waves per SIMD histogram:", blocks, threads,
                per_cu.size(), per_simd.size());
    for (auto &p : hs)
        std::printf(" %d:%d", p.first, p.second);
    std::printf("; waves per CU:");
    for (auto &p : hc)
        std::printf(" %d:%d", p.first, p.second);
    std::printf("\n");
}

int main()
{
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    std::printf("CUs: %d\n", cus);
    run(cus * 4, 64);   // one-wave workgroups, 4 per CU
    run(cus * 8, 64);   // 8 per CU
    run(cus, 256);      // one 4-wave workgroup per CU
    run(cus * 2, 256);  // two per CU
    run(cus * 12, 64);  // the search grid's 12 per CU
    return 0;
}
