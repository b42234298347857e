// deepreadmapper_amd/csrc/hnsw_search_lds.hip -- general-size fallback of the HNSW-PQ search kernel
// (heaps in LDS, replayed on lane 0), used when max(efSearch, k) > 512. Same semantics and results as
// hnsw_search.hip; see that file for the fast register-resident path.
//
// Original notes:
//
// Replaces the hot loop behind faiss_search (src/hnswpq/search.cpp:39-40): faiss
// IndexHNSW::search -> HNSW::search (greedy upper levels + search_from_candidates at level 0)
// with PQDistanceComputer (ADC over an 8 x 256 LUT) [upstream faiss >= 1.8, restated in
// oracle/drm_oracle.c]. Results are bit-identical to that restatement: same ids, same fp32
// distances (same op order, no FMA contraction), same ndis / nhops.
//
// Mapping (DESIGN.md "HNSW kernel"):
//   * one 64-lane wave = one query; persistent grid of `n_slots` one-wave workgroups pulling
//     query indices from an atomic work queue (every wave exits once the queue is drained);
//   * LDS per wave: the query's PQ LUT (M*ksub f32 = 8 KB), the MinimaxHeap (ef x {f32,i32}),
//     the k-result heap, the query vector and a 64-entry scratch for one expansion;
//   * one level-0 neighbour row (2*M_hnsw int32 = 128 B) is one coalesced load, lane j = link j;
//   * visited set = a per-slot bitmap in HBM (ntotal bits), test-and-set with one atomicOr per
//     link, cleared after the query from the list of bits it set (exact, no false positives);
//   * pop_min and count_below are wave-parallel (64-bit key min-reduction / ballot+popcount);
//     heap pushes/pops and result-heap updates replay faiss's exact array layout on lane 0,
//     because the traversal order under equal distances depends on it.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>

#include "drm_device.h"

#pragma clang fp contract(off)

namespace drm {
namespace {

struct DI {
    float d;
    int32_t i;
};

__device__ __forceinline__ uint32_t ord32(float f)
{
    uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        uint32_t lo = __shfl_xor((uint32_t)v, off, 64);
        uint32_t hi = __shfl_xor((uint32_t)(v >> 32), off, 64);
        uint64_t o = ((uint64_t)hi << 32) | lo;
        v = o < v ? o : v;
    }
    return v;
}

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

__device__ __forceinline__ int prefix_count(uint64_t mask, int lane)
{
    return __popcll(mask & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
}

// faiss::CMax<float, TI>::cmp2
__device__ __forceinline__ bool cmp2(float v1, float v2, int32_t i1, int32_t i2)
{
    return (v1 > v2) || ((v1 == v2) && (i1 > i2));
}

// faiss heap_push<CMax<float,int32>>(k, ...) on a 0-based LDS array (1-based internally)
__device__ void heap_push(DI *h, int k, float val, int32_t id)
{
    int i = k;
    while (i > 1) {
        int f = i >> 1;
        DI pf = h[f - 1];
        if (!cmp2(val, pf.d, id, pf.i))
            break;
        h[i - 1] = pf;
        i = f;
    }
    h[i - 1] = DI{val, id};
}

// faiss heap_pop<CMax<float,int32>>(k, ...)
__device__ void heap_pop(DI *h, int k)
{
    DI last = h[k - 1];
    int i = 1;
    for (;;) {
        int i1 = i << 1, i2 = i1 + 1;
        if (i1 > k)
            break;
        DI c1 = h[i1 - 1];
        DI c2 = (i2 <= k) ? h[i2 - 1] : c1;
        if ((i2 == k + 1) || cmp2(c1.d, c2.d, c1.i, c2.i)) {
            if (cmp2(last.d, c1.d, last.i, c1.i))
                break;
            h[i - 1] = c1;
            i = i1;
        } else {
            if (cmp2(last.d, c2.d, last.i, c2.i))
                break;
            h[i - 1] = c2;
            i = i2;
        }
    }
    h[i - 1] = h[k - 1];
}

// faiss heap_replace_top<CMax<float,int64>>(k, ...) -- labels are storage ids (< 2^31)
__device__ void heap_replace_top(DI *h, int k, float val, int32_t id)
{
    int i = 1;
    for (;;) {
        int i1 = i << 1, i2 = i1 + 1;
        if (i1 > k)
            break;
        DI c1 = h[i1 - 1];
        DI c2 = (i2 <= k) ? h[i2 - 1] : c1;
        if ((i2 == k + 1) || cmp2(c1.d, c2.d, c1.i, c2.i)) {
            if (cmp2(val, c1.d, id, c1.i))
                break;
            h[i - 1] = c1;
            i = i1;
        } else {
            if (cmp2(val, c2.d, id, c2.i))
                break;
            h[i - 1] = c2;
            i = i2;
        }
    }
    h[i - 1] = DI{val, id};
}

// PQ ADC distance of node v: sequential fp32 sum over sub-quantizers starting from 0
// (distance_single_code / distance_four_codes for M < 16) [upstream faiss].
template <bool FAST8>
__device__ __forceinline__ float pq_distance(const SearchArgs &a, const float *lut, int32_t v)
{
    float r = 0.0f;
    if (FAST8) { // M == 8, nbits == 8: one 8-byte code load
        const uint2 c = *reinterpret_cast<const uint2 *>(a.codes + (size_t)v * 8);
#pragma unroll
        for (int m = 0; m < 4; ++m)
            r = __fadd_rn(r, lut[m * 256 + ((c.x >> (8 * m)) & 255u)]);
#pragma unroll
        for (int m = 0; m < 4; ++m)
            r = __fadd_rn(r, lut[(m + 4) * 256 + ((c.y >> (8 * m)) & 255u)]);
        return r;
    }
    const uint8_t *code = a.codes + (size_t)v * a.code_size;
    for (int m = 0; m < a.M; ++m) {
        uint32_t idx;
        if (a.nbits == 8) {
            idx = code[m];
        } else {
            uint32_t bitpos = (uint32_t)m * (uint32_t)a.nbits;
            uint32_t byte = bitpos >> 3, shift = bitpos & 7;
            uint32_t need = shift + (uint32_t)a.nbits;
            uint32_t acc = 0;
            for (uint32_t b = 0; b * 8 < need; ++b)
                acc |= (uint32_t)code[byte + b] << (8 * b);
            idx = (acc >> shift) & ((1u << a.nbits) - 1u);
        }
        r = __fadd_rn(r, lut[m * a.ksub + (int)idx]);
    }
    return r;
}

template <bool FAST8>
__global__ __launch_bounds__(64) void hnsw_pq_search_lds_kernel(SearchArgs a)
{
    extern __shared__ __align__(16) unsigned char smem[];
    const int lane = lane_id();
    // LDS carve-up (all offsets 16-byte aligned by construction on the host)
    float *lut = reinterpret_cast<float *>(smem);
    float *qv = lut + a.M * a.ksub;
    DI *cand = reinterpret_cast<DI *>(qv + ((a.d + 3) & ~3));
    DI *res = cand + ((a.ef + 1) & ~1);
    DI *nb = res + a.kpad;                                // 64 entries
    uint64_t *keys = reinterpret_cast<uint64_t *>(res);  // sort image, aliases res
    uint32_t *vis = a.visited + (size_t)blockIdx.x * (size_t)a.vis_words;
    int32_t *clr = a.clear_list + (size_t)blockIdx.x * (size_t)a.clear_cap;

    int64_t taken = 0;
    for (;;) {
        const int64_t q = wave_next_item(a.counter, lane);
        if (q >= a.n)
            break;
        if (++taken > a.item_bound) { // more items than the queue holds: a broken work-queue fetch
            if (lane == 0)
                atomicAdd(a.errors, 1u);
            break;
        }

        int32_t ndis = 0, nhops = 0;
        // --- HeapBlockResultHandler::begin: heapify k x (+inf, -1)
        for (int j = lane; j < a.k; j += 64)
            res[j] = DI{INFINITY, -1};
        if (a.entry_point < 0 || a.ntotal == 0) {
            for (int j = lane; j < a.k; j += 64) {
                a.D[q * a.k + j] = INFINITY;
                a.I[q * a.k + j] = -1;
            }
            if (lane == 0) {
                a.ndis[q] = 0;
                a.nhops[q] = 0;
                if (a.nhops_upper)
                    a.nhops_upper[q] = 0;
            }
            continue;
        }
        // --- set_query: query vector to LDS, then LUT[m][c] = sum_t (x - c)^2 (sequential t)
        for (int t = lane; t < a.d; t += 64)
            qv[t] = a.x[q * a.d + t];
        __syncthreads();
        for (int e = lane; e < a.M * a.ksub; e += 64) {
            const int m = e / a.ksub;
            const float *cen = a.centroids + (size_t)e * a.dsub;
            const float *xs = qv + m * a.dsub;
            float acc = 0.0f;
            for (int t = 0; t < a.dsub; ++t) {
                float diff = __fsub_rn(xs[t], cen[t]);
                acc = __fadd_rn(acc, __fmul_rn(diff, diff));
            }
            lut[e] = acc;
        }
        __syncthreads();

        // --- greedy descent on levels max_level .. 1 (greedy_update_nearest)
        int32_t nearest = a.entry_point;
        float d_nearest = pq_distance<FAST8>(a, lut, nearest);
        for (int level = a.max_level; level >= 1; --level) {
            const int cnt = a.cum[level + 1] - a.cum[level];
            for (;;) {
                const int32_t prev = nearest;
                const uint32_t base = a.upper_off[nearest] + (uint32_t)(a.cum[level] - a.cum[1]);
                int32_t v = (lane < cnt) ? a.upper_nbr[base + lane] : -1;
                const uint64_t neg = __ballot(lane < cnt && v < 0);
                const int nvalid = neg ? (__ffsll((unsigned long long)neg) - 1) : cnt;
                float dd = INFINITY;
                if (lane < nvalid)
                    dd = pq_distance<FAST8>(a, lut, v);
                ndis += nvalid;
                nhops += 1;
                // sequential `if (dis < d_nearest)` in link order == first lane holding the minimum
                uint64_t key = (lane < nvalid) ? (((uint64_t)ord32(dd) << 32) | (uint32_t)lane) : ~0ull;
                key = wave_min_u64(key);
                if (key != ~0ull) {
                    const int bl = (int)(key & 63);
                    const float bd = __shfl(dd, bl, 64);
                    const int32_t bv = __shfl(v, bl, 64);
                    if (bd < d_nearest) {
                        d_nearest = bd;
                        nearest = bv;
                    }
                }
                if (nearest == prev)
                    break;
            }
        }

        // --- level 0: MinimaxHeap candidates(ef); push(nearest); seed result + visited
        int kc = 1, nvalid = 1;
        if (lane == 0)
            cand[0] = DI{d_nearest, nearest};
        float thr = INFINITY;
        if (lane == 0) {
            if (d_nearest < thr) {
                heap_replace_top(res, a.k, d_nearest, nearest);
                thr = res[0].d;
            }
        }
        thr = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(thr)));
        int clear_n = 0;
        if (lane == 0) {
            atomicOr(&vis[nearest >> 5], 1u << (nearest & 31));
            if (a.clear_cap > 0)
                clr[0] = nearest;
        }
        clear_n = 1;
        __syncthreads();

        int nstep = 0, ndis0 = 0;
        bool overrun = false;
        while (nvalid > 0) {
            if (nstep > a.hop_bound) { // a node is expanded at most once: past the bound the bookkeeping is broken
                overrun = true;
                break;
            }
            // pop_min: min distance over valid slots, ties -> highest slot
            uint64_t best = ~0ull;
            for (int s = lane; s < kc; s += 64) {
                const DI e = cand[s];
                if (e.i != -1) {
                    uint64_t key = ((uint64_t)ord32(e.d) << 32) | (uint32_t)(0xFFFFFFFFu - (uint32_t)s);
                    best = key < best ? key : best;
                }
            }
            best = wave_min_u64(best);
            const int imin = (int)(0xFFFFFFFFu - (uint32_t)best);
            const DI pm = cand[imin];
            const float d0 = pm.d;
            const int32_t v0 = pm.i;
            __syncthreads();
            if (lane == 0)
                cand[imin].i = -1;
            nvalid--;
            // count_below(d0): every slot < kc, popped ones included
            int below = 0;
            for (int base = 0; base < kc; base += 64) {
                const int s = base + lane;
                const bool b = (s < kc) && (cand[s].d < d0);
                below += __popcll(__ballot(b));
            }
            if (below >= a.efSearch)
                break;

            // expand v0's level-0 row
            const int32_t *row = a.nbr0 + (size_t)v0 * (size_t)a.deg0;
            const int32_t v1 = (lane < a.deg0) ? row[lane] : -1;
            const uint64_t negm = __ballot(lane < a.deg0 && v1 < 0);
            const int jmax = negm ? (__ffsll((unsigned long long)negm) - 1) : a.deg0;
            bool fresh = false;
            if (lane < jmax) {
                const uint32_t bit = 1u << (v1 & 31);
                const uint32_t old = atomicOr(&vis[v1 >> 5], bit);
                fresh = (old & bit) == 0u;
            }
            if (a.check_dups) { // a repeated id in one row: only its first occurrence is fresh
                for (int j = 0; j < jmax; ++j) {
                    const int32_t vj = __shfl(v1, j, 64);
                    if (j < lane && vj == v1)
                        fresh = false;
                }
            }
            const uint64_t fm = __ballot(fresh);
            const int nf = __popcll(fm);
            const int pos = prefix_count(fm, lane);
            if (fresh) {
                if (clear_n + pos < a.clear_cap)
                    clr[clear_n + pos] = v1;
                const float dd = pq_distance<FAST8>(a, lut, v1);
                nb[pos] = DI{dd, v1};
            }
            clear_n += nf;
            ndis0 += nf;
            __syncthreads();
            if (lane == 0) {
                // add_to_heap for each fresh link, in row order
                for (int t = 0; t < nf; ++t) {
                    const DI e = nb[t];
                    if (e.d < thr) {
                        heap_replace_top(res, a.k, e.d, e.i);
                        thr = res[0].d;
                    }
                    // MinimaxHeap::push
                    if (kc == a.ef) {
                        const DI top = cand[0];
                        if (e.d >= top.d)
                            continue;
                        if (top.i != -1)
                            --nvalid;
                        heap_pop(cand, kc--);
                    }
                    heap_push(cand, ++kc, e.d, e.i);
                    ++nvalid;
                }
            }
            kc = __builtin_amdgcn_readfirstlane(kc);
            nvalid = __builtin_amdgcn_readfirstlane(nvalid);
            thr = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(thr)));
            __syncthreads();
            nstep++;
        }

        // --- SingleResultHandler::end (heap_reorder): ascending (distance, id), (+inf,-1) padding
        __syncthreads();
        for (int j = lane; j < a.kpad; j += 64) { // in place: keys[j] aliases res[j] (both 8 bytes)
            const DI e = (j < a.k) ? res[j] : DI{INFINITY, -1};
            keys[j] = (e.i >= 0) ? (((uint64_t)ord32(e.d) << 32) | (uint32_t)e.i) : ~0ull;
        }
        __syncthreads();
        for (int size = 2; size <= a.kpad; size <<= 1) {
            for (int stride = size >> 1; stride > 0; stride >>= 1) {
                for (int t = lane; t < (a.kpad >> 1); t += 64) {
                    const int i = 2 * t - (t & (stride - 1));
                    const int j = i + stride;
                    const bool asc = (i & size) == 0;
                    const uint64_t x = keys[i], y = keys[j];
                    if ((x > y) == asc) {
                        keys[i] = y;
                        keys[j] = x;
                    }
                }
                __syncthreads();
            }
        }
        for (int j = lane; j < a.k; j += 64) {
            const uint64_t key = keys[j];
            if (key == ~0ull) {
                a.D[q * a.k + j] = INFINITY;
                a.I[q * a.k + j] = -1;
            } else {
                const uint32_t o = (uint32_t)(key >> 32);
                const uint32_t u = (o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o;
                a.D[q * a.k + j] = __uint_as_float(u);
                a.I[q * a.k + j] = (int64_t)(uint32_t)key;
            }
        }
        if (lane == 0) {
            a.ndis[q] = overrun ? -1 : ndis + ndis0;
            a.nhops[q] = overrun ? -1 : nhops + nstep;
            if (a.nhops_upper)
                a.nhops_upper[q] = nhops;
            if (overrun)
                atomicAdd(a.errors, 1u);
        }

        // --- VisitedTable::advance: clear exactly the bits this query set
        if (clear_n <= a.clear_cap) {
            for (int t = lane; t < clear_n; t += 64)
                vis[clr[t] >> 5] = 0u;
        } else {
            for (int64_t w = lane; w < a.vis_words; w += 64)
                vis[w] = 0u;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
}

} // namespace

void launch_hnsw_search_lds(DeviceIndex &ix, const float *d_x, int64_t n, int k, int ef, float *d_D, int64_t *d_I,
                        int32_t *d_ndis, int32_t *d_nhops, int32_t *d_nhops_upper, hipStream_t stream)
{
    if (n <= 0)
        return;
    if (k < 1 || k > 1024)
        throw Error(DRM_ERR_UNSUPPORTED, "k must be in [1, 1024] on the GPU path, got " + std::to_string(k));
    if (ef < 1)
        ef = 1;
    const int efc = std::max(ef, k);
    if (efc > 4096)
        throw Error(DRM_ERR_UNSUPPORTED, "max(efSearch, k) must be <= 4096 on the GPU path");
    if (ix.deg0 > 64)
        throw Error(DRM_ERR_UNSUPPORTED, "level-0 degree 2*M_hnsw must be <= 64 on the GPU path");
    for (int l = 1; l < ix.n_levels; ++l)
        if (ix.cum[l + 1] - ix.cum[l] > 64)
            throw Error(DRM_ERR_UNSUPPORTED, "upper-level degree must be <= 64");
    if ((size_t)ix.pq_M * (size_t)ix.ksub > 16384)
        throw Error(DRM_ERR_UNSUPPORTED, "PQ LUT M*2^nbits must be <= 16384 entries (64 KB LDS)");

    int kpad = 64;
    while (kpad < k)
        kpad <<= 1;
    const size_t lds = sizeof(float) * (size_t)ix.pq_M * ix.ksub + sizeof(float) * (size_t)((ix.d + 3) & ~3) +
                       sizeof(DI) * (size_t)((efc + 1) & ~1) + sizeof(DI) * (size_t)kpad + sizeof(DI) * 64;
    if (lds > 160 * 1024)
        throw Error(DRM_ERR_UNSUPPORTED, "search workspace does not fit in LDS");

    int cus = 0;
    DRM_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ix.device));
    int per_cu = std::max(1, std::min(16, (int)((160 * 1024) / lds)));
    int slots = (int)std::min<int64_t>(n, (int64_t)cus * per_cu);
    // (re)allocate per-slot workspace
    const int64_t words = (ix.ntotal + 31) / 32;
    if (slots > ix.n_slots || words != ix.vis_words) {
        if (ix.visited)
            DRM_HIP_CHECK(hipFree(ix.visited));
        if (ix.clear_list)
            DRM_HIP_CHECK(hipFree(ix.clear_list));
        ix.visited = nullptr;
        ix.clear_list = nullptr;
        const int alloc_slots = std::max(slots, (int)std::min<int64_t>((int64_t)cus * per_cu, 1 << 20));
        ix.vis_words = std::max<int64_t>(words, 1);
        ix.clear_cap = 16384;
        DRM_HIP_CHECK(malloc_big((void **)&ix.visited, sizeof(uint32_t) * (size_t)alloc_slots * (size_t)ix.vis_words, kBigVisited));
        DRM_HIP_CHECK(hipMemset(ix.visited, 0, sizeof(uint32_t) * (size_t)alloc_slots * (size_t)ix.vis_words));
        DRM_HIP_CHECK(hipMalloc(&ix.clear_list, sizeof(int32_t) * (size_t)alloc_slots * (size_t)ix.clear_cap));
        ix.n_slots = alloc_slots;
    }
    if (!ix.counter)
        DRM_HIP_CHECK(hipMalloc(&ix.counter, 4 * sizeof(uint32_t)));

    SearchArgs a{};
    a.x = d_x;
    a.n = n;
    a.d = ix.d;
    a.M = ix.pq_M;
    a.nbits = ix.pq_nbits;
    a.ksub = ix.ksub;
    a.dsub = ix.dsub;
    a.code_size = ix.code_size;
    a.centroids = ix.centroids;
    a.codes = ix.codes;
    a.nbr0 = ix.nbr0;
    a.deg0 = ix.deg0;
    a.upper_off = ix.upper_off;
    a.upper_nbr = ix.upper_nbr;
    for (int l = 0; l <= kMaxLevels; ++l)
        a.cum[l] = ix.cum[l];
    a.max_level = ix.max_level;
    a.entry_point = ix.entry_point;
    a.ntotal = ix.ntotal;
    a.k = k;
    a.efSearch = ef;
    a.ef = efc;
    a.kpad = kpad;
    a.D = d_D;
    a.I = d_I;
    a.ndis = d_ndis;
    a.nhops = d_nhops;
    a.nhops_upper = d_nhops_upper;
    a.visited = ix.visited;
    a.vis_words = ix.vis_words;
    a.clear_list = ix.clear_list;
    a.clear_cap = ix.clear_cap;
    a.counter = ix.counter;
    a.errors = ix.counter + 3;
    a.hop_bound = search_hop_bound(ix);
    a.item_bound = search_item_bound(ix, n);
    a.check_dups = ix.has_dup_links;

    DRM_HIP_CHECK(hipMemsetAsync(ix.counter, 0, 4 * sizeof(uint32_t), stream)); // queue head and error count
    const bool fast8 = (ix.pq_M == 8 && ix.pq_nbits == 8 && ix.code_size == 8);
    if (fast8)
        hipLaunchKernelGGL(hnsw_pq_search_lds_kernel<true>, dim3(slots), dim3(64), lds, stream, a);
    else
        hipLaunchKernelGGL(hnsw_pq_search_lds_kernel<false>, dim3(slots), dim3(64), lds, stream, a);
    DRM_HIP_CHECK(hipGetLastError());
}

} // namespace drm
