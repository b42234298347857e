// tools/microbench/vispattern.hip -- the search's per-hop memory pattern with two visited-set layouts, to price
// a compact per-query visited table before building it into hnsw_pq_fast_kernel:
//   * every wave (5,120, the search grid) runs `hops` iterations of: issue the prefetch of a random 384-B row
//     (ids + codes, consumed one iteration later), the visited test of 8 random links, a dependent chain of
//     cross-lane work standing in for the ADC + push loop, then the marks of the 8 links;
//   * layout 0 = today's tagged words: a 4-B load per link in the slot's own ntotal/16-word region (12.5 MB at C5),
//     marks by atomic max + atomic or on the same word;
//   * layout 1 = a compact table: a 16-B load per link half (lanes j and j + 32) in the slot's 64 KB table,
//     marks by one plain 4-B store;
//   * layout 2 = layout 0 with plain-store marks (what the atomics cost);
//   * layout 3 = layout 0 without marks.
// Prints ns per hop for each layout and amount of stand-in work.
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

__device__ __forceinline__ uint32_t mix(uint32_t x)
{
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

// ORDER (layout 0 words, atomic marks): 0 = marks right after the visited answer, log store at the end of the hop
// (the kernel today); 1 = log store deferred until after the next hop's loads; 2 = marks and log store deferred;
// 3 = no marks, no log stores (the floor); 4 = as 0 with branchy marks / log store (as the search kernel)
template <int LAYOUT, int ORDER = 0>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(5))) void hops_kernel(
    const int32_t *rows, uint64_t nrows, uint32_t *vis, uint64_t vis_words, uint32_t *tab, int hops, int work,
    uint32_t *sink, uint64_t *logs)
{
    __shared__ uint32_t pad[2048]; // the LUT's 8 KB: 20 waves per CU, as the search
    const int lane = threadIdx.x;
    pad[lane] = lane;
    uint32_t *myvis = vis + (size_t)blockIdx.x * vis_words;
    uint32_t *mytab = tab + (size_t)blockIdx.x * (64 * 1024 / 4);
    uint64_t *mylog = logs + (size_t)blockIdx.x * 4096;
    uint32_t *scratch = reinterpret_cast<uint32_t *>(logs + (size_t)gridDim.x * 4096) + (size_t)blockIdx.x * 256;
    uint32_t seed = mix(blockIdx.x * 7919u + 17u);
    uint32_t acc = 0;
    uint64_t r = mix(seed) % nrows;
    int32_t id = 0;
    uint2 cd = make_uint2(0u, 0u);
    uint32_t *paddr = nullptr; // deferred marks
    bool pmark = false;
    uint32_t ph = 0;
    int logn = 0;
    bool plog = false;
    for (int h = 0; h < hops; ++h) {
        // pop_min stand-in
        uint32_t w0 = acc + (uint32_t)lane;
        for (int i = 0; i < 4; ++i)
            w0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((w0 & 63u) << 2), (int)w0) * 3u + 1u;
        acc += __builtin_amdgcn_readfirstlane(w0) & 1u;
        seed = mix(seed + (uint32_t)h);
        r = ((uint64_t)seed * 2654435761ull + (uint64_t)__builtin_amdgcn_readfirstlane(acc & 1u)) % nrows;
        id = rows[r * 96 + (lane & 31)];
        cd = reinterpret_cast<const uint2 *>(rows + r * 96 + 32)[lane & 31];
        const uint32_t link = mix(seed ^ (uint32_t)(lane & 31) * 0x9E3779B9u);
        const bool act = (lane & 31) < 8 && (LAYOUT == 1 || lane < 32);
        uint32_t old = 0;
        uint32_t *addr = nullptr;
        if (LAYOUT == 1) {
            const uint32_t b = link % (64 * 1024 / 32);
            const uint4 *p = reinterpret_cast<const uint4 *>(mytab + b * 8 + (lane >= 32 ? 4 : 0));
            const uint4 v = *(act ? p : reinterpret_cast<const uint4 *>(scratch + 192) + (lane & 15));
            old = act ? (v.x ^ v.y ^ v.z ^ v.w) : 1u;
            addr = mytab + b * 8 + (link >> 29);
        } else {
            addr = myvis + (link % vis_words);
            old = __hip_atomic_load(act ? addr : scratch + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            old = act ? old : 1u;
        }
        // deferred stores of the previous hop go out after this hop's loads
        if (ORDER == 2) {
            uint32_t *ma = pmark ? paddr : scratch + lane;
            __hip_atomic_fetch_max(ma, pmark ? ph << 16 : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_or(ma, pmark ? 2u : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (ORDER == 1 || ORDER == 2)
            __hip_atomic_store(plog ? mylog + ((logn + lane) & 4095) : (uint64_t *)(scratch + 64) + lane, (uint64_t)acc,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // the visited answer (the row issued before it has arrived too)
        acc += (uint32_t)id + cd.x;
        const bool fresh = act && (old & 1u) == 0u;
        if (ORDER == 4 && fresh) {
            __hip_atomic_fetch_max(addr, (uint32_t)h << 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_or(addr, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (ORDER <= 1) {
            if (LAYOUT == 0) {
                uint32_t *ma = fresh ? addr : scratch + lane;
                __hip_atomic_fetch_max(ma, fresh ? (uint32_t)h << 16 : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_or(ma, fresh ? 2u : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else {
                __hip_atomic_store(fresh && lane < 32 ? addr : scratch + lane, (uint32_t)h << 1, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        pmark = fresh;
        paddr = addr;
        ph = (uint32_t)h;
        // push-loop stand-in: a dependent chain of cross-lane round trips
        uint32_t w = old + (uint32_t)lane;
        for (int i = 0; i < work; ++i) {
            w = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((w & 63u) << 2), (int)w);
            w = w * 3u + 1u;
        }
        acc += w;
        // log store of ~2 accepted pushes
        const bool lg = lane < 2;
        if (ORDER == 0)
            __hip_atomic_store(lg ? mylog + ((logn + lane) & 4095) : (uint64_t *)(scratch + 64) + lane, (uint64_t)acc,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (ORDER == 4 && lg)
            __hip_atomic_store(mylog + ((logn + lane) & 4095), (uint64_t)acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        plog = lg;
        logn += 2;
    }
    if (acc == 0x12345678u)
        sink[blockIdx.x] = acc + pad[lane];
}

__global__ void fill(uint32_t *buf, uint64_t n, uint32_t mod)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        buf[i] = mod ? (uint32_t)((i * 2654435761ull) % mod) : 0u;
}

int main(int argc, char **argv)
{
    const uint64_t ntotal = 50000000ull, nrows = ntotal;
    const int waves = argc > 1 ? std::atoi(argv[1]) : 5120;
    const int hops = argc > 2 ? std::atoi(argv[2]) : 400;
    const uint64_t vis_words = (ntotal + 15) / 16;
    int32_t *rows = nullptr;
    uint32_t *vis = nullptr, *tab = nullptr, *sink = nullptr;
    CK(hipMalloc(&rows, nrows * 96 * sizeof(int32_t)));
    CK(hipMalloc(&vis, (size_t)waves * vis_words * sizeof(uint32_t)));
    CK(hipMalloc(&tab, (size_t)waves * 64 * 1024));
    CK(hipMalloc(&sink, sizeof(uint32_t) * waves));
    hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, (uint32_t *)rows, nrows * 96, (uint32_t)ntotal);
    hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, vis, (uint64_t)waves * vis_words, 0u);
    hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, tab, (uint64_t)waves * 16 * 1024, 0u);
    CK(hipDeviceSynchronize());
    uint64_t *logs = nullptr;
    CK(hipMalloc(&logs, (size_t)waves * 4096 * 8 + (size_t)waves * 1024));
    CK(hipMemset(logs, 0, (size_t)waves * 4096 * 8 + (size_t)waves * 1024));
    // footprints: rows over nrows_sel nodes, visited words over vw_sel words per slot (branchy atomic marks, ORDER 4)
    const uint64_t row_sel[2] = {nrows, 100000ull};
    const uint64_t vw_sel[2] = {vis_words, 16384ull};
    for (int work : {0, 16}) {
        for (int ri = 0; ri < 2; ++ri) {
            for (int vi = 0; vi < 2; ++vi) {
                auto launch = [&](int hp) {
                    hipLaunchKernelGGL((hops_kernel<0, 4>), dim3(waves), dim3(64), 0, 0, rows, row_sel[ri], vis, vw_sel[vi], tab, hp,
                                       work, sink, logs);
                };
                launch(20);
                CK(hipDeviceSynchronize());
                const auto t0 = std::chrono::steady_clock::now();
                launch(hops);
                CK(hipDeviceSynchronize());
                const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                std::printf("work %2d  rows over %8.3f GB, visited %8.3f MB per slot (%.1f GB in all): %6.0f ns per hop\n", work,
                            row_sel[ri] * 384.0 / 1e9, vw_sel[vi] * 4.0 / 1e6, vw_sel[vi] * 4.0 * waves / 1e9, sec / hops * 1e9);
            }
        }
    }
    return 0;
}
