// deepreadmapper_amd/csrc/hnsw_flat_search.hip -- hnswlib fp32-L2 search for gfx950.
//
// Replaces search(index, queries, k, ef) (src/hnswlib_dir/search.cpp:7-52): per query
// HierarchicalNSW<float>::searchKnnCloserFirst -> searchKnn -> searchBaseLayerST<bare_bone>
// [upstream hnswlib, restated in oracle/hnswlib_oracle.cpp]. Results are bit-identical to that
// restatement: same labels, same fp32 distances (hnswlib's 8-accumulator L2SqrSIMD16ExtAVX order,
// no FMA), same ndis / nhops.
//
// Mapping (DESIGN.md "fp32 HNSW kernel"):
//   * one 64-lane wave = one query, persistent grid pulling query ids from an atomic counter;
//   * a level-0 row (maxM0 = 2M = 128 links at the reference's M = 64) is one coalesced 512-B load;
//     visited = per-slot HBM bitmap, one atomicOr per link, cleared from a clear list;
//   * distances: 8 lanes per fresh neighbour, lane i owning hnswlib's AVX accumulator i (dims
//     i, i+8, ...), 8 neighbours per pass; the accumulators are summed left to right by a DPP chain;
//   * top_candidates and candidate_set are libstdc++ binary heaps (std::priority_queue with
//     CompareByFirst) replayed exactly -- __push_heap / __adjust_heap -- in LDS by lane 0, with the
//     unbounded candidate_set spilling past `cand_lds` entries into a per-slot global array.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "drm_device.h"

#pragma clang fp contract(off)

namespace drm {
namespace {

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

// Heap array accessor: LDS part, plus (OVF) a per-slot global continuation past lds_cap entries.
template <bool OVF> struct HeapRef {
    float *k;         // LDS keys [lds_cap]
    uint32_t *i;      // LDS ids
    int lds_cap;
    float *ok;        // overflow keys (global), OVF only
    uint32_t *oi;     // overflow ids
    __device__ float key(int t) const { return (!OVF || t < lds_cap) ? k[t] : ok[t - lds_cap]; }
    __device__ uint32_t id(int t) const { return (!OVF || t < lds_cap) ? i[t] : oi[t - lds_cap]; }
    __device__ void set(int t, float kk, uint32_t ii) const
    {
        if (!OVF || t < lds_cap) {
            k[t] = kk;
            i[t] = ii;
        } else {
            ok[t - lds_cap] = kk;
            oi[t - lds_cap] = ii;
        }
    }
};

// std::priority_queue::emplace = push_back + std::push_heap -> __push_heap(first, len-1, 0, value),
// comparator CompareByFirst: a.first < b.first (libstdc++ bits/stl_heap.h)
template <bool OVF> __device__ void stl_push(const HeapRef<OVF> &h, int len, float vk, uint32_t vi)
{
    int hole = len - 1;
    int parent = (hole - 1) / 2;
    while (hole > 0 && h.key(parent) < vk) {
        h.set(hole, h.key(parent), h.id(parent));
        hole = parent;
        parent = (hole - 1) / 2;
    }
    h.set(hole, vk, vi);
}

// std::priority_queue::pop = std::pop_heap + pop_back: the last element is re-inserted through
// __adjust_heap(first, 0, len - 1, value) (hole to a leaf along the larger child, ties -> right),
// then __push_heap back up
template <bool OVF> __device__ void stl_pop(const HeapRef<OVF> &h, int len)
{
    if (len <= 1)
        return;
    const float vk = h.key(len - 1);
    const uint32_t vi = h.id(len - 1);
    const int L = len - 1;
    int hole = 0, second = 0;
    while (second < (L - 1) / 2) {
        second = 2 * (second + 1);
        if (h.key(second) < h.key(second - 1))
            second--;
        h.set(hole, h.key(second), h.id(second));
        hole = second;
    }
    if ((L & 1) == 0 && second == (L - 2) / 2) {
        second = 2 * (second + 1);
        h.set(hole, h.key(second - 1), h.id(second - 1));
        hole = second - 1;
    }
    int parent = (hole - 1) / 2;
    while (hole > 0 && h.key(parent) < vk) {
        h.set(hole, h.key(parent), h.id(parent));
        hole = parent;
        parent = (hole - 1) / 2;
    }
    h.set(hole, vk, vi);
}

__device__ __forceinline__ uint32_t dpp_row_shr1(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);
}

// L2 of the query (LDS) against `nitem` vectors: item f handled by lane group f & 7 in pass f >> 3.
// Lane i of a group accumulates dims i, i+8, ... in order (hnswlib L2SqrSIMD16ExtAVX accumulator i);
// the 8 accumulators are then added left to right. Results go to out[f] (LDS).
__device__ void l2_items(const FlatArgs &a, const float *q, const uint32_t *ids, int nitem, float *out)
{
    const int lane = lane_id(), grp = lane >> 3, sub = lane & 7;
    for (int base = 0; base < nitem; base += 8) {
        const int f = base + grp;
        const bool act = f < nitem;
        float acc = 0.0f;
        if (act) {
            const float *v = a.vec + (size_t)ids[f] * (size_t)a.d;
            for (int t = sub; t < a.d; t += 8) {
                const float df = __fsub_rn(q[t], v[t]);
                acc = __fadd_rn(acc, __fmul_rn(df, df));
            }
        }
        // prefix chain: after step s, lane sub == s holds acc0 + ... + acc_s (left to right)
        uint32_t p = __float_as_uint(acc);
#pragma unroll
        for (int s = 1; s < 8; ++s) {
            const uint32_t t = dpp_row_shr1(p);
            if (sub == s)
                p = __float_as_uint(__fadd_rn(__uint_as_float(t), __uint_as_float(p)));
        }
        if (act && sub == 7)
            out[f] = __uint_as_float(p);
    }
    __syncthreads();
}

__global__ __launch_bounds__(64) void hnsw_flat_search_kernel(FlatArgs a)
{
    extern __shared__ __align__(16) unsigned char smem[];
    const int lane = lane_id();
    float *q = reinterpret_cast<float *>(smem);                      // [d]
    float *topk = q + a.d;                                           // [top_lds]
    uint32_t *topi = reinterpret_cast<uint32_t *>(topk + a.top_lds); // [top_lds]
    float *cdk = reinterpret_cast<float *>(topi + a.top_lds);        // [cand_lds]
    uint32_t *cdi = reinterpret_cast<uint32_t *>(cdk + a.cand_lds); // [cand_lds]
    uint32_t *fid = cdi + a.cand_lds;                               // [maxM0] fresh ids / upper links
    float *fd = reinterpret_cast<float *>(fid + a.maxM0);           // [maxM0] their distances
    int *sh = reinterpret_cast<int *>(fd + a.maxM0);                // [4] broadcast scalars
    uint32_t *vis = a.visited + (size_t)blockIdx.x * (size_t)a.vis_words;
    int32_t *clr = a.clear_list + (size_t)blockIdx.x * (size_t)a.clear_cap;
    const HeapRef<true> top{topk, topi, a.top_lds, a.top_ovf_k + (size_t)blockIdx.x * (size_t)a.top_ovf_cap,
                            a.top_ovf_i + (size_t)blockIdx.x * (size_t)a.top_ovf_cap};
    const HeapRef<true> cand{cdk, cdi, a.cand_lds, a.cand_ovf_k + (size_t)blockIdx.x * (size_t)a.cand_ovf_cap,
                       a.cand_ovf_i + (size_t)blockIdx.x * (size_t)a.cand_ovf_cap};
    const int cand_cap = a.cand_lds + (int)a.cand_ovf_cap;

    for (;;) {
        int qi = 0;
        if (lane == 0)
            qi = (int)atomicAdd(a.counter, 1u);
        qi = __builtin_amdgcn_readfirstlane(qi);
        if ((int64_t)qi >= a.n)
            break;
        float *Dq = a.D + (int64_t)qi * a.k;
        uint64_t *Lq = a.L + (int64_t)qi * a.k;
        if (a.ntotal == 0) {
            for (int j = lane; j < a.k; j += 64) {
                Dq[j] = INFINITY;
                Lq[j] = ~0ull;
            }
            if (lane == 0) {
                a.ndis[qi] = 0;
                a.nhops[qi] = 0;
                if (a.nhops_upper)
                    a.nhops_upper[qi] = 0;
            }
            continue;
        }
        for (int t = lane; t < a.d; t += 64)
            q[t] = a.x[(int64_t)qi * a.d + t];
        __syncthreads();
        int ndis = 0, nhops = 0;
        // --- searchKnn: greedy descent on levels maxlevel .. 1
        uint32_t cur = a.ep;
        if (lane == 0)
            fid[0] = cur;
        __syncthreads();
        l2_items(a, q, fid, 1, fd);
        float curdist = fd[0];
        ndis++;
        int nhops_up = 0;
        for (int level = a.maxlevel; level > 0; --level) {
            for (;;) {
                const uint32_t *blk = a.up + a.up_off[cur] + (int64_t)(level - 1) * (1 + a.maxM);
                const int size = (int)(blk[0] & 0xFFFFu);
                for (int j = lane; j < size; j += 64)
                    fid[j] = blk[1 + j];
                __syncthreads();
                nhops++;
                nhops_up++;
                ndis += size;
                l2_items(a, q, fid, size, fd);
                bool changed = false;
                for (int j = 0; j < size; ++j) { // sequential `if (d < curdist)` (uniform)
                    const float dd = fd[j];
                    if (dd < curdist) {
                        curdist = dd;
                        cur = fid[j];
                        changed = true;
                    }
                }
                __syncthreads();
                if (!changed)
                    break;
            }
        }
        // --- searchBaseLayerST<bare_bone_search = true>(cur, q, max(ef, k))
        int top_len = 1, cand_len = 1, clear_n = 1;
        float lowerBound = curdist;
        bool overflow = false;
        if (lane == 0) {
            top.set(0, curdist, cur);
            cand.set(0, -curdist, cur);
            atomicOr(&vis[cur >> 5], 1u << (cur & 31));
            if (a.clear_cap > 0)
                clr[0] = (int32_t)cur;
        }
        __syncthreads();
        while (cand_len > 0) {
            const float cdist = -cand.key(0);
            if (cdist > lowerBound)
                break;
            const uint32_t c = cand.id(0);
            __syncthreads();
            if (lane == 0)
                stl_pop(cand, cand_len);
            cand_len--;
            nhops++;
            // the row of c: maxM0 links, lane j holds links j, j + 64, ...
            const int cnt = (int)(a.l0cnt[c] & 0xFFFFu);
            const uint32_t *row = a.l0 + (size_t)c * (size_t)a.maxM0;
            int nf = 0;
            for (int base = 0; base < cnt; base += 64) {
                const int j = base + lane;
                const bool act = j < cnt;
                const uint32_t v = act ? row[j] : 0u;
                bool fresh = false;
                if (act) {
                    const uint32_t bit = 1u << (v & 31);
                    fresh = (atomicOr(&vis[v >> 5], bit) & bit) == 0u;
                }
                if (a.check_dups) { // a repeated link in one row: only its first occurrence is fresh
                    for (int jj = 0; jj < cnt; ++jj) {
                        const uint32_t vj = row[jj];
                        if (jj < j && vj == v)
                            fresh = false;
                    }
                }
                const uint64_t fm = __ballot(fresh);
                if (fresh) {
                    const int p = nf + __popcll(fm & (lane ? (~0ull >> (64 - lane)) : 0ull));
                    fid[p] = v;
                    if (clear_n + p < a.clear_cap)
                        clr[clear_n + p] = (int32_t)v;
                }
                nf += __popcll(fm);
            }
            clear_n += nf;
            __syncthreads();
            l2_items(a, q, fid, nf, fd);
            ndis += nf;
            // sequential consideration in link order (lane 0 owns both heaps)
            if (lane == 0) {
                int tl = top_len, cl = cand_len;
                float lb = lowerBound;
                for (int f = 0; f < nf; ++f) {
                    const float dist = fd[f];
                    if (tl < a.ef || lb > dist) {
                        if (cl >= cand_cap) {
                            overflow = true;
                            break;
                        }
                        cand.set(cl, -dist, fid[f]);
                        stl_push(cand, ++cl, -dist, fid[f]);
                        top.set(tl, dist, fid[f]);
                        stl_push(top, ++tl, dist, fid[f]);
                        while (tl > a.ef) {
                            stl_pop(top, tl);
                            tl--;
                        }
                        lb = top.key(0);
                    }
                }
                sh[0] = tl;
                sh[1] = cl;
                sh[2] = __float_as_int(lb);
                sh[3] = overflow ? 1 : 0;
            }
            __syncthreads();
            top_len = sh[0];
            cand_len = sh[1];
            lowerBound = __int_as_float(sh[2]);
            if (sh[3])
                break;
            __syncthreads();
        }
        if (lane == 0 && overflow)
            atomicAdd(a.counter + 1, 1u); // candidate_set overflow: reported by the host entry points
        // --- while (top.size() > k) top.pop(); then order survivors by (dist, label)
        if (lane == 0) {
            int tl = top_len;
            while (tl > a.k) {
                stl_pop(top, tl);
                tl--;
            }
            sh[0] = tl;
        }
        __syncthreads();
        const int nres = sh[0];
        // searchKnnCloserFirst order: ascending (dist, label) -- rank by counting, labels staged in
        // the (now idle) candidate-heap LDS when they fit
        uint64_t *lab = reinterpret_cast<uint64_t *>(cdk);
        const bool staged = nres <= a.cand_lds;
        if (staged)
            for (int e = lane; e < nres; e += 64)
                lab[e] = a.labels[top.id(e)];
        __syncthreads();
        for (int e = lane; e < nres; e += 64) {
            const float de = top.key(e);
            const uint64_t le = staged ? lab[e] : a.labels[top.id(e)];
            int rank = 0;
            for (int o = 0; o < nres; ++o) {
                const float dq = top.key(o);
                const uint64_t lo = staged ? lab[o] : a.labels[top.id(o)];
                rank += (dq < de) || (dq == de && lo < le);
            }
            Dq[rank] = de;
            Lq[rank] = le;
        }
        for (int j = nres + lane; j < a.k; j += 64) {
            Dq[j] = INFINITY;
            Lq[j] = ~0ull;
        }
        if (lane == 0) {
            a.ndis[qi] = ndis;
            a.nhops[qi] = nhops;
            if (a.nhops_upper)
                a.nhops_upper[qi] = nhops_up;
        }
        // VisitedTable reset: clear exactly the bits this query set
        if (clear_n <= a.clear_cap) {
            for (int t = lane; t < clear_n; t += 64)
                vis[(uint32_t)clr[t] >> 5] = 0u;
        } else {
            for (int64_t w = lane; w < a.vis_words; w += 64)
                vis[w] = 0u;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
}

} // namespace

void launch_hnsw_flat_search(DeviceFlatIndex &ix, const float *d_x, int64_t n, int k, int ef, float *d_D,
                             uint64_t *d_L, int32_t *d_ndis, int32_t *d_nhops, int32_t *d_nhops_upper,
                             hipStream_t stream)
{
    if (n <= 0)
        return;
    if (k < 1 || k > 4096)
        throw Error(DRM_ERR_UNSUPPORTED, "k must be in [1, 4096] on the GPU path");
    const int efc = std::max(std::max(ef, 1), k); // searchKnn: searchBaseLayerST(..., max(ef_, k))
    if (ix.d % 16 != 0 || ix.d > 4096)
        throw Error(DRM_ERR_UNSUPPORTED, "fp32 search needs d % 16 == 0 (hnswlib L2SqrSIMD16Ext)");
    int cus = 0;
    DRM_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ix.device));
    const int cand_lds = 512;
    const int top_lds = std::min(efc + 1, 1024); // top_candidates beyond this continue in global memory
    const int64_t top_ovf = (int64_t)efc + 1 - top_lds;
    const size_t lds = sizeof(float) * (size_t)ix.d + 8 * (size_t)top_lds + 8 * (size_t)cand_lds +
                       8 * (size_t)ix.maxM0 + 16;
    if (lds > 160 * 1024)
        throw Error(DRM_ERR_UNSUPPORTED, "fp32 search workspace does not fit in LDS (ef too large)");
    const int per_cu = std::max(1, std::min(ix.waves_per_cu, (int)((160 * 1024) / lds)));
    const int slots = (int)std::min<int64_t>(n, (int64_t)cus * per_cu);
    const int64_t words = (ix.ntotal + 31) / 32;
    const int64_t ovf_cap = 16384;
    if (slots > ix.n_slots || words != ix.vis_words || top_ovf > ix.top_ovf_cap) {
        for (void *p : {(void *)ix.visited, (void *)ix.clear_list, (void *)ix.cand_ovf_k, (void *)ix.cand_ovf_i,
                        (void *)ix.top_ovf_k, (void *)ix.top_ovf_i})
            if (p)
                DRM_HIP_CHECK(hipFree(p));
        const int alloc = std::max(slots, cus * per_cu);
        ix.vis_words = std::max<int64_t>(words, 1);
        ix.clear_cap = 16384;
        ix.cand_ovf_cap = ovf_cap;
        DRM_HIP_CHECK(hipMalloc(&ix.visited, sizeof(uint32_t) * (size_t)alloc * (size_t)ix.vis_words));
        DRM_HIP_CHECK(hipMemset(ix.visited, 0, sizeof(uint32_t) * (size_t)alloc * (size_t)ix.vis_words));
        DRM_HIP_CHECK(hipMalloc(&ix.clear_list, sizeof(int32_t) * (size_t)alloc * (size_t)ix.clear_cap));
        DRM_HIP_CHECK(hipMalloc(&ix.cand_ovf_k, sizeof(float) * (size_t)alloc * (size_t)ovf_cap));
        DRM_HIP_CHECK(hipMalloc(&ix.cand_ovf_i, sizeof(uint32_t) * (size_t)alloc * (size_t)ovf_cap));
        ix.top_ovf_cap = std::max<int64_t>(top_ovf, 1);
        DRM_HIP_CHECK(hipMalloc(&ix.top_ovf_k, sizeof(float) * (size_t)alloc * (size_t)ix.top_ovf_cap));
        DRM_HIP_CHECK(hipMalloc(&ix.top_ovf_i, sizeof(uint32_t) * (size_t)alloc * (size_t)ix.top_ovf_cap));
        ix.n_slots = alloc;
    }
    if (!ix.counter)
        DRM_HIP_CHECK(hipMalloc(&ix.counter, 4 * sizeof(uint32_t)));
    FlatArgs a{};
    a.x = d_x;
    a.n = n;
    a.d = ix.d;
    a.vec = ix.vec;
    a.l0 = ix.l0;
    a.l0cnt = ix.l0cnt;
    a.maxM0 = ix.maxM0;
    a.up_off = ix.up_off;
    a.up = ix.up;
    a.maxM = ix.maxM;
    a.maxlevel = ix.maxlevel;
    a.ep = ix.ep;
    a.ntotal = ix.ntotal;
    a.labels = ix.labels;
    a.k = k;
    a.ef = efc;
    a.D = d_D;
    a.L = d_L;
    a.ndis = d_ndis;
    a.nhops = d_nhops;
    a.nhops_upper = d_nhops_upper;
    a.visited = ix.visited;
    a.vis_words = ix.vis_words;
    a.clear_list = ix.clear_list;
    a.clear_cap = ix.clear_cap;
    a.counter = ix.counter;
    a.check_dups = ix.has_dup_links;
    a.cand_lds = cand_lds;
    a.cand_ovf_k = ix.cand_ovf_k;
    a.cand_ovf_i = ix.cand_ovf_i;
    a.cand_ovf_cap = ix.cand_ovf_cap;
    a.top_lds = top_lds;
    a.top_ovf_k = ix.top_ovf_k;
    a.top_ovf_i = ix.top_ovf_i;
    a.top_ovf_cap = ix.top_ovf_cap;
    DRM_HIP_CHECK(hipMemsetAsync(ix.counter, 0, 2 * sizeof(uint32_t), stream));
    hipLaunchKernelGGL(hnsw_flat_search_kernel, dim3(slots), dim3(64), lds, stream, a);
    DRM_HIP_CHECK(hipGetLastError());
}

} // namespace drm
