// deepreadmapper_amd/csrc/hnsw_search.hip -- wavefront-per-query HNSW-PQ search for gfx950.
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
#include "pq_common.h"

#pragma clang fp contract(off)

namespace drm {
namespace {

struct DI {
    float d;
    int32_t i;
};

// Register-resident arrays of 64*R slots: slot s lives in lane (s & 63), register (s >> 6).
// rd/wr take a wave-uniform slot: rd compiles to v_readlane, wr to a lane-masked v_cndmask.
template <int R> __device__ __forceinline__ uint32_t rd(const uint32_t (&a)[R], int s)
{
    const int l = s & 63, r = s >> 6;
    uint32_t out = 0;
#pragma unroll
    for (int i = 0; i < R; ++i) {
        const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)a[i], l);
        out = (r == i) ? x : out;
    }
    return out;
}
template <int R> __device__ __forceinline__ void wr(uint32_t (&a)[R], int s, uint32_t v)
{
    const int l = s & 63, r = s >> 6;
    const bool mine = (int)(threadIdx.x & 63) == l; // v_cmp + v_cndmask (no writelane builtin in HIP)
#pragma unroll
    for (int i = 0; i < R; ++i)
        if (r == i)
            a[i] = mine ? v : a[i];
}

// faiss heap_push<CMax<float,int32>>(k, ...) -- the MinimaxHeap layout, replayed exactly
template <int R> __device__ void heap_push(uint32_t (&hk)[R], uint32_t (&hi)[R], int k, uint32_t key, int32_t id)
{
    int i = k;
    while (i > 1) {
        const int f = i >> 1;
        const uint32_t pk = rd(hk, f - 1);
        const int32_t pi = (int32_t)rd(hi, f - 1);
        if (!cmp2(key, pk, id, pi))
            break;
        wr(hk, i - 1, pk);
        wr(hi, i - 1, (uint32_t)pi);
        i = f;
    }
    wr(hk, i - 1, key);
    wr(hi, i - 1, (uint32_t)id);
}

// faiss heap_pop<CMax<float,int32>>(k, ...)
template <int R> __device__ void heap_pop(uint32_t (&hk)[R], uint32_t (&hi)[R], int k)
{
    const uint32_t lk = rd(hk, k - 1);
    const int32_t li = (int32_t)rd(hi, k - 1);
    int i = 1;
    for (;;) {
        const int i1 = i << 1, i2 = i1 + 1;
        if (i1 > k)
            break;
        const uint32_t k1 = rd(hk, i1 - 1);
        const int32_t d1 = (int32_t)rd(hi, i1 - 1);
        uint32_t k2 = k1;
        int32_t d2 = d1;
        if (i2 <= k) {
            k2 = rd(hk, i2 - 1);
            d2 = (int32_t)rd(hi, i2 - 1);
        }
        if ((i2 == k + 1) || cmp2(k1, k2, d1, d2)) {
            if (cmp2(lk, k1, li, d1))
                break;
            wr(hk, i - 1, k1);
            wr(hi, i - 1, (uint32_t)d1);
            i = i1;
        } else {
            if (cmp2(lk, k2, li, d2))
                break;
            wr(hk, i - 1, k2);
            wr(hi, i - 1, (uint32_t)d2);
            i = i2;
        }
    }
    wr(hk, i - 1, lk);
    wr(hi, i - 1, (uint32_t)li);
}

// lexicographic min of (hi, lo) over the wave
__device__ __forceinline__ uint64_t wave_min_pair(uint32_t hi, uint32_t lo)
{
    const uint32_t mh = wave_min_u32(hi);
    const uint32_t ml = wave_min_u32(hi == mh ? lo : 0xFFFFFFFFu);
    return ((uint64_t)mh << 32) | ml;
}
// lane i <- lane i-1 (lane 0 <- old)
__device__ __forceinline__ uint32_t wave_shr1(uint32_t old, uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xF, 0xF, false);
}

// value of register array `a` at a per-lane slot (ds_bpermute per register)
template <int R> __device__ __forceinline__ uint32_t fetch(const uint32_t (&a)[R], int slot)
{
    const int sl = slot & 63, sr = slot >> 6;
    uint32_t out = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t x = (uint32_t)__shfl((int)a[r], sl, 64);
        out = (sr == r) ? x : out;
    }
    return out;
}

// faiss heap_push<CMax<float,int32>>(k, val, id), wave-parallel (R <= 2, k <= 64R <= 128):
// lane l >= 1 holds the ancestor at level l; the sift-up stops at the first ancestor that does
// not compare below val; every lane then pulls the new contents of its path slots.
template <int R> __device__ void heap_push_par(uint32_t (&hk)[R], uint32_t (&hi)[R], int k, uint32_t key, int32_t id)
{
    const int lane = lane_id();
    const int anc = (lane < 16) ? (k >> lane) : 0;
    const bool exists = lane >= 1 && anc >= 1;
    const int src = exists ? anc - 1 : 0;
    const uint32_t ak = fetch(hk, src);
    const int32_t ai = (int32_t)fetch(hi, src);
    const bool moves = exists && cmp2(key, ak, id, ai);
    const uint64_t stopm = __ballot(lane >= 1 && !moves);
    const int h = __builtin_ctzll(stopm) - 1; // parents moved down; val lands at k >> h
    const int bk = 32 - __builtin_clz((unsigned)k);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int p = lane + 64 * r + 1;
        const int m = bk - (32 - __builtin_clz((unsigned)p));
        const bool on = m >= 0 && m <= h && (k >> m) == p;
        const int srcl = (m + 1) & 63;
        const uint32_t vk = (uint32_t)__shfl((int)ak, srcl, 64);
        const int32_t vi = __shfl(ai, srcl, 64);
        if (on) {
            hk[r] = (m == h) ? key : vk;
            hi[r] = (m == h) ? (uint32_t)id : (uint32_t)vi;
        }
    }
}

// faiss heap_pop<CMax<float,int32>>(k), wave-parallel (R <= 2): lane p-1 decides which child the
// sift-down takes at internal node p, lane l walks to the path node at depth l, the hole stops at
// the first child that `last` does not compare below, and owners pull their new slot contents.
template <int R> __device__ void heap_pop_par(uint32_t (&hk)[R], uint32_t (&hi)[R], int k)
{
    const int lane = lane_id();
    const uint32_t lk = rd(hk, k - 1);
    const int32_t li = (int32_t)rd(hi, k - 1);
    const int c1 = 2 * (lane + 1), c2 = c1 + 1;
    const int s1 = min(c1, 64 * R) - 1, s2 = min(c2, 64 * R) - 1;
    const uint32_t k1 = fetch(hk, s1), k2 = fetch(hk, s2);
    const int32_t i1 = (int32_t)fetch(hi, s1), i2 = (int32_t)fetch(hi, s2);
    const uint64_t lm = __ballot((c2 == k + 1) || cmp2(k1, k2, i1, i2)); // bit p-1: take left child
    // uniform (scalar) walk of the max-child path down to its last node `leaf` at depth `depth`;
    // the path node at depth l is the leaf's ancestor leaf >> (depth - l)
    int leaf = 1, depth = 0;
    while (2 * leaf <= k) {
        leaf = 2 * leaf + (int)(((lm >> (leaf - 1)) & 1ull) ^ 1ull);
        ++depth;
    }
    const bool onpath = lane <= depth;
    const int pl = onpath ? (leaf >> (depth - lane)) : 0;
    const int src = onpath ? pl - 1 : 0;
    const uint32_t ak = fetch(hk, src);
    const int32_t ai = (int32_t)fetch(hi, src);
    const uint64_t sm = __ballot(lane >= 1 && (!onpath || cmp2(lk, ak, li, ai)));
    const int h = __builtin_ctzll(sm) - 1; // the hole ends at path depth h
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int pos = lane + 64 * r + 1;
        const int m = 31 - __builtin_clz((unsigned)pos);
        const bool on = m <= h && (leaf >> (depth - m)) == pos;
        const int srcl = (m + 1) & 63;
        const uint32_t vk = (uint32_t)__shfl((int)ak, srcl, 64);
        const int32_t vi = __shfl(ai, srcl, 64);
        if (on) {
            hk[r] = (m == h) ? lk : vk;
            hi[r] = (m == h) ? (uint32_t)li : (uint32_t)vi;
        }
    }
}


// Candidate heap (faiss MinimaxHeap arrays; 1-based heap index i = slot + 1) for ef <= 128 in the
// sibling-pair layout: lane p holds the two children of node slot p, slots 2p+1 (L) and 2p+2 (R).
// Slot 0, the root, sits in lane 63's R half (node 63's right child would be slot 128 >= ef).
// A sift-down then picks every node's larger child inside its own lane, the path values are one
// ds_bpermute of the chosen children, and each pair's new contents come from one source lane.
struct PairHeap {
    uint32_t kL, kR, iL, iR;

    __device__ __forceinline__ void init()
    {
        kL = kR = 0u;
        iL = iR = 0xFFFFFFFFu;
    }
    static __device__ __forceinline__ int lane_of(int s) { return s == 0 ? 63 : (s - 1) >> 1; }
    static __device__ __forceinline__ bool right_of(int s) { return s == 0 || ((s - 1) & 1); }
    // (values are selected, never members: a member chosen at run time would be spilled to scratch)
    __device__ __forceinline__ uint32_t key(int s) const
    {
        const int l = lane_of(s);
        const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)kL, l);
        const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)kR, l);
        return right_of(s) ? b : a;
    }
    __device__ __forceinline__ uint32_t id(int s) const
    {
        const int l = lane_of(s);
        const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)iL, l);
        const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)iR, l);
        return right_of(s) ? b : a;
    }
    __device__ __forceinline__ void set(int s, uint32_t k, uint32_t i)
    {
        const bool mine = lane_id() == lane_of(s);
        const bool r = right_of(s);
        const bool mr = mine && r, ml = mine && !r;
        kR = mr ? k : kR;
        iR = mr ? i : iR;
        kL = ml ? k : kL;
        iL = ml ? i : iL;
    }
    __device__ __forceinline__ void set_id(int s, uint32_t i)
    {
        const bool mine = lane_id() == lane_of(s);
        const bool r = right_of(s);
        iR = (mine && r) ? i : iR;
        iL = (mine && !r) ? i : iL;
    }
    __device__ __forceinline__ uint32_t root_key() const { return (uint32_t)__builtin_amdgcn_readlane((int)kR, 63); }
    __device__ __forceinline__ uint32_t root_id() const { return (uint32_t)__builtin_amdgcn_readlane((int)iR, 63); }

    // faiss heap_push<CMax<float,int32>>(k, key, id): the new element starts at 1-based index k
    __device__ __forceinline__ void push(int k, uint32_t key_, int32_t id_)
    {
        if (k == 1 || !cmp2(key_, key((k >> 1) - 1), id_, (int32_t)id((k >> 1) - 1))) {
            set(k - 1, key_, (uint32_t)id_); // most pushes stay at the bottom
            return;
        }
        const int lane = lane_id();
        // lane l >= 1: the ancestor k >> l; the sift-up passes every ancestor below the new element
        const int anc = (lane < 16) ? (k >> lane) : 0;
        const bool exists = lane >= 1 && anc >= 1;
        const int sa = exists ? anc - 1 : 0;
        const int sl = lane_of(sa);
        const bool sr = right_of(sa);
        const uint32_t akL = (uint32_t)__shfl((int)kL, sl, 64), akR = (uint32_t)__shfl((int)kR, sl, 64);
        const uint32_t aiL = (uint32_t)__shfl((int)iL, sl, 64), aiR = (uint32_t)__shfl((int)iR, sl, 64);
        const uint32_t ak = sr ? akR : akL, ai = sr ? aiR : aiL;
        const bool moves = exists && cmp2(key_, ak, id_, (int32_t)ai);
        const int h = __builtin_ctzll(__ballot(lane >= 1 && !moves)) - 1; // ancestors 1..h move down
        const int bk = 32 - __builtin_clz((unsigned)k);
        // chain index m holds the node k >> m; it receives chain m+1's value, chain h the new one
        {
            const int m = bk - 1; // the root
            if (m <= h) {
                const uint32_t nk = (m == h) ? key_ : (uint32_t)__builtin_amdgcn_readlane((int)ak, m + 1);
                const uint32_t ni = (m == h) ? (uint32_t)id_ : (uint32_t)__builtin_amdgcn_readlane((int)ai, m + 1);
                kR = (lane == 63) ? nk : kR;
                iR = (lane == 63) ? ni : iR;
            }
        }
        const int iLx = 2 * lane + 2; // 1-based index of this lane's L slot (R = iLx + 1)
        const int m = bk - (32 - __builtin_clz((unsigned)iLx));
        const bool inrange = m >= 0 && m <= h;
        const int tgt = inrange ? (k >> m) : 0;
        const bool onL = inrange && tgt == iLx;
        const bool onR = inrange && tgt == iLx + 1 && lane != 63;
        const int src = (m + 1) & 63;
        const uint32_t vk = (uint32_t)__shfl((int)ak, src, 64), vi = (uint32_t)__shfl((int)ai, src, 64);
        const uint32_t nk = (m == h) ? key_ : vk, ni = (m == h) ? (uint32_t)id_ : vi;
        if (onL) {
            kL = nk;
            iL = ni;
        }
        if (onR) {
            kR = nk;
            iR = ni;
        }
    }

    // faiss heap_pop<CMax<float,int32>>(k): the element at 1-based k is sifted down from the root
    __device__ __forceinline__ void pop(int k)
    {
        const int lane = lane_id();
        const uint32_t vk = key(k - 1);
        const int32_t vi = (int32_t)id(k - 1);
        // node `lane` (1-based lane+1) has children 2*lane+2 (L) and 2*lane+3 (R); node 63's only
        // possible child is 128
        const bool takeL = (lane == 63) || (2 * lane + 3 == k + 1) || cmp2(kL, kR, (int32_t)iL, (int32_t)iR);
        const uint64_t lm = __ballot(takeL);
        const uint32_t mk = takeL ? kL : kR, mi = takeL ? iL : iR;
        (void)lm;
        // The max-child path by pointer doubling (VALU + ds_bpermute instead of a scalar walk):
        // N1(p) = chosen child slot of node slot p (p itself once p has no children; slots >= 64
        // are leaves), N2 = N1.N1, N4 = N2.N2; lane d then composes its depth-d node from d's bits.
        const int n1 = (2 * lane + 2 <= k) ? (takeL ? 2 * lane + 1 : 2 * lane + 2) : lane;
        const int n1n1 = __shfl(n1, n1 & 63, 64);
        const int n2 = (n1 < 64) ? n1n1 : n1;
        const int n2n2 = __shfl(n2, n2 & 63, 64);
        const int n4 = (n2 < 64) ? n2n2 : n2;
        const int root_child = __builtin_amdgcn_readlane(n1, 0); // explicit lane (readfirstlane would follow exec)
        int sd = (lane & 1) ? root_child : 0;
        {
            const int t = __shfl(n2, sd & 63, 64);
            sd = ((lane & 2) && sd < 64) ? t : sd;
            const int u = __shfl(n4, sd & 63, 64);
            sd = ((lane & 4) && sd < 64) ? u : sd;
        }
        // sd = 0-based path slot at depth `lane` (lanes 0..7); the previous depth's via DPP row_shr:1
        const int sprev = (int)dpp_u32(0u, (uint32_t)sd, 0x111, 0xF);
        const int depth = __popcll(__ballot(lane >= 1 && lane <= 7 && sd != sprev));
        const int leaf = __builtin_amdgcn_readlane(sd, 7) + 1; // 1-based
        // lane l in [1, depth]: the path node at depth l = the chosen child of the node above it
        const bool onpath = lane >= 1 && lane <= depth;
        const int par = onpath ? sprev : 0;
        const uint32_t ak = (uint32_t)__shfl((int)mk, par, 64), ai = (uint32_t)__shfl((int)mi, par, 64);
        const int h = __builtin_ctzll(__ballot(lane >= 1 && (!onpath || cmp2(vk, ak, vi, (int32_t)ai)))) - 1;
        // depth m takes depth m+1's value for m < h; depth h takes the sifted element
        {
            const uint32_t nk = (h == 0) ? vk : (uint32_t)__builtin_amdgcn_readlane((int)ak, 1);
            const uint32_t ni = (h == 0) ? (uint32_t)vi : (uint32_t)__builtin_amdgcn_readlane((int)ai, 1);
            kR = (lane == 63) ? nk : kR;
            iR = (lane == 63) ? ni : iR;
        }
        const int iLx = 2 * lane + 2;
        const int m = 31 - __builtin_clz((unsigned)iLx); // depth of this lane's pair
        const bool inrange = m <= h;
        const int tgt = inrange ? (leaf >> (depth - m)) : 0;
        const bool onL = inrange && tgt == iLx;
        const bool onR = inrange && tgt == iLx + 1 && lane != 63;
        const int src = (m + 1) & 63;
        const uint32_t wk = (uint32_t)__shfl((int)ak, src, 64), wi = (uint32_t)__shfl((int)ai, src, 64);
        const uint32_t nk = (m == h) ? vk : wk, ni = (m == h) ? (uint32_t)vi : wi;
        if (onL) {
            kL = nk;
            iL = ni;
        }
        if (onR) {
            kR = nk;
            iR = ni;
        }
    }
};


// The visited set is a per-slot HBM bitmap (atomicOr test-and-set), cleared from a list after each query.
// Bounded: a query past a.hop_bound level-0 hops, or a wave past a.item_bound work items, ends with an error count
// (a.errors; drm_search returns DRM_ERR_INTERNAL) instead of looping.
// STAMPS (diagnostic builds only): per-section s_memtime sums -> a.stamps[section], for time shares.
#define DRM_STAMP(idx)                                                                                      \
    do {                                                                                                    \
        if (STAMPS) {                                                                                       \
            __builtin_amdgcn_sched_barrier(0);                                                              \
            const uint64_t _t = __builtin_amdgcn_s_memtime();                                               \
            __builtin_amdgcn_sched_barrier(0);                                                              \
            st_acc[idx] += _t - st_last;                                                                    \
            st_last = _t;                                                                                   \
        }                                                                                                   \
    } while (0)

template <int R, bool FAST8, bool STAMPS = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void hnsw_pq_search_kernel(SearchArgs a)
{
    extern __shared__ __align__(16) unsigned char smem[];
    uint64_t st_acc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t st_last = STAMPS ? __builtin_amdgcn_s_memtime() : 0;
    const int lane = lane_id();
    float *lut = reinterpret_cast<float *>(smem);
    uint32_t *vis = a.visited + (size_t)blockIdx.x * (size_t)a.vis_words;
    int32_t *clr = a.clear_list + (size_t)blockIdx.x * (size_t)a.clear_cap;
    const uint32_t kInfKey = ord32(INFINITY);
    int64_t taken = 0;
    for (;;) {
        const int q = wave_next_item(a.counter, lane);
        if ((int64_t)q >= a.n)
            break;
        if (++taken > a.item_bound) { // more items than the queue holds: a broken work-queue fetch
            if (lane == 0)
                atomicAdd(a.errors, 1u);
            break;
        }

        if (a.entry_point < 0 || a.ntotal == 0) {
            for (int j = lane; j < a.k; j += 64) {
                a.D[(int64_t)q * a.k + j] = INFINITY;
                a.I[(int64_t)q * a.k + j] = -1;
            }
            if (lane == 0) {
                a.ndis[q] = 0;
                a.nhops[q] = 0;
                if (a.nhops_upper)
                    a.nhops_upper[q] = 0;
            }
            continue;
        }
        DRM_STAMP(7);
        // --- set_query
        build_lut(a, q, lut, lane);
        DRM_STAMP(0);
        int32_t nearest;
        uint32_t dn;
        int ndis, nhops;
        greedy_upper<FAST8>(a, lut, lane, nearest, dn, ndis, nhops);
        const int nhops_upper = nhops;

        DRM_STAMP(1);
        // --- level 0. Result handler: k slots of (+inf,-1) (HeapBlockResultHandler::begin)
        constexpr bool PAIR = R <= 2; // candidate heap in the sibling-pair layout (ef <= 128)
        uint32_t rk[R], ri[R], ck[PAIR ? 1 : R], ci[PAIR ? 1 : R];
        PairHeap ph;
        ph.init();
#pragma unroll
        for (int r = 0; r < R; ++r) {
            rk[r] = kInfKey;
            ri[r] = 0xFFFFFFFFu;
        }
#pragma unroll
        for (int r = 0; r < (PAIR ? 1 : R); ++r) {
            ck[r] = 0;
            ci[r] = 0xFFFFFFFFu;
        }
        // Result set kept sorted by (key, id) in slots 0..k-1: inserting below the max (slot k-1)
        // evicts the max, which is exactly heap_replace_top's effect on the k-set; the output order
        // is heap_reorder's (valid entries ascending, then (+inf,-1)).
        uint32_t thr = kInfKey;
        auto add_result = [&](uint32_t key, int32_t id) {
            if (key < thr) { // SingleResultHandler::add_result: strict on distance
                int pos = 0;
                uint32_t pk[R], pi[R];
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    pos += __popcll(__ballot((lane + 64 * r) < a.k && cmp2(key, rk[r], id, (int32_t)ri[r])));
                    const uint32_t carry_k = r ? (uint32_t)__builtin_amdgcn_readlane((int)rk[r - 1], 63) : 0u;
                    const uint32_t carry_i = r ? (uint32_t)__builtin_amdgcn_readlane((int)ri[r - 1], 63) : 0u;
                    pk[r] = wave_shr1(carry_k, rk[r]);
                    pi[r] = wave_shr1(carry_i, ri[r]);
                }
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int s = lane + 64 * r;
                    if (s > pos) {
                        rk[r] = pk[r];
                        ri[r] = pi[r];
                    } else if (s == pos) {
                        rk[r] = key;
                        ri[r] = (uint32_t)id;
                    }
                }
                thr = rd(rk, a.k - 1);
            }
        };
        // MinimaxHeap candidates(ef); push(nearest, d_nearest); seed result + visited set
        int kc = 1, nvalid = 1;
        if constexpr (PAIR) {
            ph.set(0, dn, (uint32_t)nearest);
        } else {
            wr(ck, 0, dn);
            wr(ci, 0, (uint32_t)nearest);
        }
        add_result(dn, nearest);
        int clear_n = 1;
        if (lane == 0) {
            vis_test_set(&vis[nearest >> 5], 1u << (nearest & 31));
            if (a.clear_cap > 0)
                clr[0] = nearest;
        }
        __syncthreads();

        int nstep = 0, ndis0 = 0;
        bool overrun = false;
        int32_t pred = -1, v1_pref = -1; // row of the node predicted to be popped next, loaded early
        while (nvalid > 0) {
            if (nstep > a.hop_bound) { // a node is expanded at most once: past the bound the bookkeeping is broken
                overrun = true;
                break;
            }
            // pop_min: smallest distance among valid slots, ties -> highest slot
            uint32_t bh = 0xFFFFFFFFu, bl = 0xFFFFFFFFu;
            const int sL = 2 * lane + 1, sR = (lane == 63) ? 0 : 2 * lane + 2; // PAIR slots of this lane
            if constexpr (PAIR) {
                if (sR < kc && ph.iR != 0xFFFFFFFFu) {
                    bh = ph.kR;
                    bl = 0xFFFFFFFFu - (uint32_t)sR;
                }
                if (sL < kc && ph.iL != 0xFFFFFFFFu) {
                    const uint32_t lo = 0xFFFFFFFFu - (uint32_t)sL;
                    if (ph.kL < bh || (ph.kL == bh && lo < bl)) {
                        bh = ph.kL;
                        bl = lo;
                    }
                }
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int s = lane + 64 * r;
                    if (s < kc && ci[r] != 0xFFFFFFFFu) {
                        const uint32_t lo = 0xFFFFFFFFu - (uint32_t)s;
                        if (ck[r] < bh || (ck[r] == bh && lo < bl)) {
                            bh = ck[r];
                            bl = lo;
                        }
                    }
                }
            }
            const uint64_t best = wave_min_pair(bh, bl);
            const int imin = (int)ufirst(0xFFFFFFFFu - (uint32_t)best);
            const uint32_t d0 = ufirst((uint32_t)(best >> 32));
            int32_t v0;
            if constexpr (PAIR) {
                v0 = (int32_t)ph.id(imin);
                ph.set_id(imin, 0xFFFFFFFFu);
            } else {
                v0 = (int32_t)rd(ci, imin);
                wr(ci, imin, 0xFFFFFFFFu);
            }
            nvalid--;
            // count_below(d0): every slot < kc, popped ones included
            int below = 0;
            if constexpr (PAIR) {
                below = __popcll(__ballot(sL < kc && ph.kL < d0)) + __popcll(__ballot(sR < kc && ph.kR < d0));
            } else {
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const int s = lane + 64 * r;
                    below += __popcll(__ballot(s < kc && ck[r] < d0));
                }
            }
            if (below >= a.efSearch)
                break;

            DRM_STAMP(2);
            // expand v0's level-0 row (one coalesced 128-B load at M_hnsw = 16)
            int32_t v1 = v1_pref;
            if (v0 != pred)
                v1 = (lane < a.deg0) ? a.nbr0[(size_t)v0 * (size_t)a.deg0 + lane] : -1;
            const uint64_t negm = __ballot(lane < a.deg0 && v1 < 0);
            const int jmax = negm ? (__ffsll((unsigned long long)negm) - 1) : a.deg0;
            const bool act = lane < jmax;
            uint2 c8 = make_uint2(0u, 0u);
            if (FAST8 && act)
                c8 = load_code8<FAST8>(a, v1); // issued before the visited test: overlaps its latency
            bool fresh = false;
            if (act) {
                const uint32_t bit = 1u << (v1 & 31);
                const uint32_t old = vis_test_set(&vis[v1 >> 5], bit);
                fresh = (old & bit) == 0u;
            }
            if (a.check_dups) { // a repeated id in one row: only its first occurrence is fresh
                for (int j = 0; j < jmax; ++j) {
                    const int32_t vj = __shfl(v1, j, 64);
                    if (j < lane && vj == v1)
                        fresh = false;
                }
            }
            DRM_STAMP(3);
            const uint64_t fm = __ballot(fresh);
            const int nf = __popcll(fm);
            const int clear_base = clear_n;
            clear_n += nf;
            uint32_t dk = 0;
            if (fresh) {
                if (!FAST8)
                    c8 = load_code8<FAST8>(a, v1);
                dk = ord32(pq_distance_code<FAST8>(a, lut, v1, c8));
            }
            ndis0 += nf;
            {
                // Predict the next pop_min (smallest valid candidate after this row's pushes) and
                // start loading its row now, so the load overlaps the heap updates below. A wrong
                // prediction (ties, evictions) only costs a reload.
                uint32_t mk = fresh ? dk : 0xFFFFFFFFu;
                uint32_t mid = (uint32_t)v1;
                if constexpr (PAIR) {
                    const int sL = 2 * lane + 1, sR = (lane == 63) ? 0 : 2 * lane + 2;
                    if (sL < kc && ph.iL != 0xFFFFFFFFu && ph.kL < mk) {
                        mk = ph.kL;
                        mid = ph.iL;
                    }
                    if (sR < kc && ph.iR != 0xFFFFFFFFu && ph.kR < mk) {
                        mk = ph.kR;
                        mid = ph.iR;
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const int s = lane + 64 * r;
                        if (s < kc && ci[r] != 0xFFFFFFFFu && ck[r] < mk) {
                            mk = ck[r];
                            mid = ci[r];
                        }
                    }
                }
                const uint32_t m = wave_min_u32(mk);
                pred = -1;
                if (m != 0xFFFFFFFFu) {
                    pred = __builtin_amdgcn_readlane((int)mid, __builtin_ctzll(__ballot(mk == m)));
                    v1_pref = (lane < a.deg0) ? a.nbr0[(size_t)pred * (size_t)a.deg0 + lane] : -1;
                }
            }
            // clear-list entries are stored after the loads above so that no wait covers them
            if (fresh) {
                const int p = clear_base + __popcll(fm & lanes_below(lane));
                if (p < a.clear_cap)
                    clr[p] = v1;
            }
            DRM_STAMP(4);
            // add_to_heap for each fresh link in row order (wave-uniform scalar loop)
            uint64_t rem = fm;
            while (rem) {
                const int l = __builtin_ctzll(rem);
                rem &= rem - 1;
                const uint32_t key = (uint32_t)__builtin_amdgcn_readlane((int)dk, l);
                const int32_t id = __builtin_amdgcn_readlane(v1, l);
                DRM_STAMP(5);
                add_result(key, id);
                DRM_STAMP(8);
                if (kc == a.ef) { // MinimaxHeap::push on a full heap
                    if constexpr (PAIR) {
                        if (key >= ph.root_key())
                            continue;
                        if (ph.root_id() != 0xFFFFFFFFu)
                            --nvalid;
                        ph.pop(kc);
                        DRM_STAMP(9);
                    } else {
                        if (key >= (uint32_t)__builtin_amdgcn_readlane((int)ck[0], 0))
                            continue;
                        if ((uint32_t)__builtin_amdgcn_readlane((int)ci[0], 0) != 0xFFFFFFFFu)
                            --nvalid;
                        heap_pop(ck, ci, kc);
                    }
                    kc--;
                }
                kc++;
                if constexpr (PAIR)
                    ph.push(kc, key, id);
                else
                    heap_push(ck, ci, kc, key, id);
                ++nvalid;
                DRM_STAMP(10);
            }
            nstep++;
            DRM_STAMP(5);
        }

        DRM_STAMP(2);
        // --- SingleResultHandler::end (heap_reorder): the sorted slots are already its output
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int j = lane + 64 * r;
            if (j < a.k) {
                const int64_t o = (int64_t)q * a.k + j;
                const bool valid = (int32_t)ri[r] >= 0;
                a.D[o] = valid ? unord32(rk[r]) : INFINITY;
                a.I[o] = valid ? (int64_t)(int32_t)ri[r] : (int64_t)-1;
            }
        }
        if (lane == 0) {
            a.ndis[q] = overrun ? -1 : ndis + ndis0;
            a.nhops[q] = overrun ? -1 : nhops + nstep;
            if (a.nhops_upper)
                a.nhops_upper[q] = nhops_upper;
            if (overrun)
                atomicAdd(a.errors, 1u);
        }

        // --- VisitedTable::advance: clear exactly the HBM bits this query set
        if (clear_n <= a.clear_cap) {
            for (int t = lane; t < clear_n; t += 64)
                vis[clr[t] >> 5] = 0u;
        } else {
            for (int64_t w = lane; w < a.vis_words; w += 64)
                vis[w] = 0u;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        DRM_STAMP(6);
    }
    if (STAMPS && lane_id() == 0 && a.stamps)
        for (int i = 0; i < 12; ++i)
            atomicAdd(reinterpret_cast<unsigned long long *>(a.stamps) + i, (unsigned long long)st_acc[i]);
}


} // namespace

// Per-slot search workspace (visited bitmaps, clear lists, queue counters, the lean kernel's push log)
// for a full-occupancy grid, allocated once at index load so that no search pays for it (at C5 a bitmap
// workspace is 32 GB). Searches that need more (other LUT sizes, larger logs) still grow it. The lean kernel
// keeps no visited table: with inline rows the bitmap waits for a search that needs it (another kernel, or
// exact statistics).
void reserve_search_scratch(DeviceIndex &ix)
{
    int cus = 0;
    DRM_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ix.device));
    const size_t lds = sizeof(float) * (size_t)ix.pq_M * ix.ksub;
    if (lds == 0 || lds > 160 * 1024)
        return;
    const int per_cu = std::max(1, std::min(ix.waves_per_cu, (int)((160 * 1024) / lds)));
    const int slots = cus * per_cu;
    if (!ix.rows) {
        ix.vis_words = std::max<int64_t>((ix.ntotal + 31) / 32, 1);
        ix.clear_cap = 16384;
        DRM_HIP_CHECK(malloc_big((void **)&ix.visited, sizeof(uint32_t) * (size_t)slots * (size_t)ix.vis_words, kBigVisited));
        DRM_HIP_CHECK(hipMemset(ix.visited, 0, sizeof(uint32_t) * (size_t)slots * (size_t)ix.vis_words));
        DRM_HIP_CHECK(hipMalloc(&ix.clear_list, sizeof(int32_t) * (size_t)slots * (size_t)ix.clear_cap));
        ix.n_slots = slots;
        ix.device_bytes += (int64_t)sizeof(uint32_t) * slots * ix.vis_words + (int64_t)sizeof(int32_t) * slots * ix.clear_cap;
    }
    DRM_HIP_CHECK(hipMalloc(&ix.counter, 4 * sizeof(uint32_t)));
    DRM_HIP_CHECK(hipMemset(ix.counter, 0, 4 * sizeof(uint32_t)));
    const int cap = std::max(ix.log_cap_req, 128 + 128); // what the lean kernel asks for at ef = 128
    if (ix.log)
        DRM_HIP_CHECK(hipFree(ix.log));
    DRM_HIP_CHECK(hipMalloc(&ix.log, sizeof(uint64_t) * (size_t)slots * (size_t)cap));
    ix.log_cap = cap;
    ix.log_slots = slots;
    ix.device_bytes += (int64_t)sizeof(uint64_t) * slots * cap;
}

void check_search_errors(DeviceIndex &ix)
{
    if (!ix.counter)
        return;
    uint32_t c[4] = {0, 0, 0, 0};
    DRM_HIP_CHECK(hipMemcpy(c, ix.counter, sizeof(c), hipMemcpyDeviceToHost));
    if (c[3]) {
        DRM_HIP_CHECK(hipMemset(ix.counter + 3, 0, sizeof(uint32_t))); // reported once
        throw Error(DRM_ERR_INTERNAL, std::to_string(c[3]) + " queries exceeded the search's hop bound or waves their "
                                                             "work-item bound (DESIGN.md sec. 4.1): search state broken");
    }
}

int64_t search_hop_bound(const DeviceIndex &ix) { return ix.hop_bound > 0 ? std::min(ix.hop_bound, ix.ntotal) : ix.ntotal; }
int64_t search_item_bound(const DeviceIndex &ix, int64_t n) { return ix.item_bound > 0 ? std::min(ix.item_bound, n) : n; }

void launch_hnsw_search(DeviceIndex &ix, const float *d_x, int64_t n, int k, int ef, float *d_D, int64_t *d_I,
                        int32_t *d_ndis, int32_t *d_nhops, int32_t *d_nhops_upper, hipStream_t stream)
{
    if (n <= 0)
        return;
    if (k < 1 || k > 1024)
        throw Error(DRM_ERR_UNSUPPORTED, "k must be in [1, 1024] on the GPU path, got " + std::to_string(k));
    if (ef < 1)
        ef = 1;
    const int efc = std::max(ef, k);
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
    const int R = (std::max(efc, k) + 63) / 64;
    if (R > 8 || ix.force_lds_kernel) { // large ef / k: LDS-heap kernel
        launch_hnsw_search_lds(ix, d_x, n, k, ef, d_D, d_I, d_ndis, d_nhops, d_nhops_upper, stream);
        return;
    }
    const size_t lds = sizeof(float) * (size_t)ix.pq_M * ix.ksub; // the LUT
    if (lds > 160 * 1024)
        throw Error(DRM_ERR_UNSUPPORTED, "search workspace does not fit in LDS");

    int cus = 0;
    DRM_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ix.device));
    int per_cu = std::max(1, std::min(ix.waves_per_cu, (int)((160 * 1024) / lds)));
    int slots = (int)std::min<int64_t>(n, (int64_t)cus * per_cu);
    // (re)allocate per-slot workspace: the lean kernel needs the bitmap only to count faiss's ndis
    const bool fast_path = ix.use_fast && hnsw_pq_fast_supported(ix, k, efc);
    const bool need_bitmap = !fast_path || ix.exact_stats;
    const int64_t words = (ix.ntotal + 31) / 32;
    if (need_bitmap && (slots > ix.n_slots || words != ix.vis_words)) {
        if (ix.visited) {
            DRM_HIP_CHECK(hipFree(ix.visited));
            ix.device_bytes -= (int64_t)sizeof(uint32_t) * ix.n_slots * ix.vis_words;
        }
        if (ix.clear_list) {
            DRM_HIP_CHECK(hipFree(ix.clear_list));
            ix.device_bytes -= (int64_t)sizeof(int32_t) * ix.n_slots * ix.clear_cap;
        }
        ix.visited = nullptr;
        ix.clear_list = nullptr;
        const int alloc_slots = std::max(slots, (int)std::min<int64_t>((int64_t)cus * per_cu, 1 << 20));
        ix.vis_words = std::max<int64_t>(words, 1);
        ix.clear_cap = 16384;
        size_t free_b = 0, total_b = 0;
        DRM_HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
        const size_t need_b = sizeof(uint32_t) * (size_t)alloc_slots * (size_t)ix.vis_words +
                              sizeof(int32_t) * (size_t)alloc_slots * (size_t)ix.clear_cap;
        if (need_b > free_b)
            throw Error(DRM_ERR_UNSUPPORTED, "the search's visited bitmaps need " + std::to_string(need_b >> 20) +
                                                 " MiB of device memory, " + std::to_string(free_b >> 20) + " MiB free");
        DRM_HIP_CHECK(malloc_big((void **)&ix.visited, sizeof(uint32_t) * (size_t)alloc_slots * (size_t)ix.vis_words, kBigVisited));
        DRM_HIP_CHECK(hipMemset(ix.visited, 0, sizeof(uint32_t) * (size_t)alloc_slots * (size_t)ix.vis_words));
        DRM_HIP_CHECK(hipMalloc(&ix.clear_list, sizeof(int32_t) * (size_t)alloc_slots * (size_t)ix.clear_cap));
        ix.n_slots = alloc_slots;
        ix.device_bytes += (int64_t)(need_b);
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
    a.stamps = ix.stamps;
    a.trace = ix.trace;
    a.x_aligned16 = ((uintptr_t)d_x % 16) == 0;

    const bool fast8 = (ix.pq_M == 8 && ix.pq_nbits == 8 && ix.code_size == 8);
    if (fast_path) {
        // the lean kernel (hnsw_pq_fast.hip); k == ef logs accepted pushes per slot
        // a compacted log holds <= k <= ef entries; then up to 64 staged evictions, or the ef heap entries at the end
        const int cap = std::max(ix.log_cap_req, efc + std::max(efc, 64));
        const int need = std::max(ix.log_slots, slots);
        if (!ix.log || ix.log_cap != cap || ix.log_slots < need) {
            if (ix.log) {
                DRM_HIP_CHECK(hipFree(ix.log));
                ix.device_bytes -= (int64_t)sizeof(uint64_t) * ix.log_slots * ix.log_cap;
            }
            ix.log = nullptr;
            DRM_HIP_CHECK(hipMalloc(&ix.log, sizeof(uint64_t) * (size_t)need * (size_t)cap));
            ix.log_cap = cap;
            ix.log_slots = need;
            ix.device_bytes += (int64_t)sizeof(uint64_t) * need * cap;
        }
        a.log = ix.log;
        a.log_cap = ix.log_cap;
        a.rows = ix.rows;
        a.row_words = ix.row_words;
        a.upper_codes = ix.upper_codes;
        a.exact_stats = ix.exact_stats;
        DRM_HIP_CHECK(hipMemsetAsync(ix.counter, 0, 4 * sizeof(uint32_t), stream));
        launch_hnsw_pq_fast(a, slots, ix.stamps != nullptr, stream);
        return;
    }
    DRM_HIP_CHECK(hipMemsetAsync(ix.counter, 0, 4 * sizeof(uint32_t), stream));
#define DRM_LAUNCH_EXACT(RR, F8)                                                                               \
    hipLaunchKernelGGL((hnsw_pq_search_kernel<RR, F8>), dim3(slots), dim3(64), lds, stream, a)
#define DRM_LAUNCH_EXACT_R(F8)                                                                                 \
    switch (R) {                                                                                                \
    case 1: DRM_LAUNCH_EXACT(1, F8); break;                                                                     \
    case 2: DRM_LAUNCH_EXACT(2, F8); break;                                                                     \
    case 3: case 4: DRM_LAUNCH_EXACT(4, F8); break;                                                             \
    default: DRM_LAUNCH_EXACT(8, F8); break;                                                                    \
    }
    if (fast8 && ix.stamps && R == 2) {
        hipLaunchKernelGGL((hnsw_pq_search_kernel<2, true, true>), dim3(slots), dim3(64), lds, stream, a);
    } else if (fast8) {
        DRM_LAUNCH_EXACT_R(true)
    } else {
        DRM_LAUNCH_EXACT_R(false)
    }
#undef DRM_LAUNCH_EXACT_R
#undef DRM_LAUNCH_EXACT
    DRM_HIP_CHECK(hipGetLastError());
}

} // namespace drm
