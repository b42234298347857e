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

// The lane id as an opaque value: per-lane index arithmetic derived from it is recomputed where it
// is used instead of being hoisted out of the hop loop, where it would pin VGPRs (occupancy).
__device__ __forceinline__ int lane_id_local()
{
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

// Heap entries live in LDS as interleaved (key bits, id) pairs: one 8-byte access per entry, and a
// node's two children (slots 2p+1, 2p+2) are one ds_read2_b64.
typedef uint2 KV;
__device__ __forceinline__ float kv_key(KV e) { return __uint_as_float(e.x); }
__device__ __forceinline__ KV kv_make(float k, uint32_t i) { return make_uint2(__float_as_uint(k), i); }
// One 8-byte LDS read whose both halves are live right away. Left alone, the compiler reads the key,
// waits, and fetches the id later only in the lanes that move it -- a second dependent LDS round
// trip in every heap operation.
__device__ __forceinline__ KV kv_load(const KV *p)
{
    KV e = *p;
    asm volatile("" : "+v"(e.x), "+v"(e.y));
    return e;
}

// Address-space-qualified pointers: an access that may go to either part stays a branch between an
// LDS and a global instruction. Generic pointers would let the compiler fold the two into one flat_*
// access, and flat accesses count against both vmcnt and lgkmcnt -- every LDS wait after one would
// then also wait for the outstanding row prefetch.
#define DRM_LDS __attribute__((address_space(3)))
#define DRM_GLOBAL __attribute__((address_space(1)))

#ifndef DRM_FLAT_MW
#define DRM_FLAT_MW 1 // 1: heap ops write their moved entries and the new one in one write phase
#endif

// Heap array accessor: LDS part, plus (OVF) a per-slot global continuation past lds_cap entries.
template <bool OVF> struct HeapRef {
    DRM_LDS uint64_t *kv;    // LDS entries [lds_cap], the KV pairs as (id << 32 | key bits)
    int lds_cap;
    DRM_GLOBAL float *ok;    // overflow keys (global), OVF only
    DRM_GLOBAL uint32_t *oi; // overflow ids
    __device__ float key(int t) const
    {
        return (!OVF || t < lds_cap) ? __uint_as_float((uint32_t)kv[t]) : ok[t - lds_cap];
    }
    __device__ uint32_t id(int t) const { return (!OVF || t < lds_cap) ? (uint32_t)(kv[t] >> 32) : oi[t - lds_cap]; }
    __device__ void set(int t, float kk, uint32_t ii) const
    {
        if (!OVF || t < lds_cap) {
            kv[t] = (uint64_t)__float_as_uint(kk) | ((uint64_t)ii << 32);
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

// ---- wave-parallel versions of the same two heap operations, for a heap held entirely in LDS.
// They leave exactly the layout the serial replay above leaves (so every later tie resolves the same
// way), but cost one LDS round trip plus a few ballots instead of one dependent LDS access per level.
// ballot of a bool straight from its compare mask (HIP's int __ballot adds a select + compare)
__device__ __forceinline__ uint64_t bal(bool b) { return __builtin_amdgcn_ballot_w64(b); }

__device__ __forceinline__ int heap_depth(int slot) { return 31 - __builtin_clz((unsigned)slot + 1u); }

// __push_heap for the element just appended at slot len-1. Along the ancestor chain keys only grow
// (parent >= child), so the ancestors that move down are exactly those with key < vk: lane j reads
// ancestor j+1, one ballot counts them (h), they shift down one level and vk lands at ancestor h.
// Returns true when vk became the root.
__device__ __forceinline__ bool par_push(KV *H, int len, float vk, uint32_t vi)
{
    const int lane = lane_id_local();
    const int hole = len - 1;
    const int m = heap_depth(hole);
    const int j = lane + 1;
    const bool valid = j <= m;
    const int anc = valid ? ((hole + 1) >> j) - 1 : 0;
    const KV ae = kv_load(H + anc);
    const bool lt = valid && kv_key(ae) < vk;
    const int h = __popcll(bal(lt));
#if DRM_FLAT_MW
    // the lanes that move are a prefix (0 .. h-1): lane i < h writes ancestor i+1 into ancestor i's
    // place, lane h writes vk into ancestor h -- one write phase
    if (lane <= h)
        H[((hole + 1) >> lane) - 1] = lane < h ? ae : kv_make(vk, vi);
#else
    if (lt) // ancestor j moves into ancestor j-1's place (ancestor 0 = the hole)
        H[((hole + 1) >> (j - 1)) - 1] = ae;
    if (lane == 0)
        H[((hole + 1) >> h) - 1] = kv_make(vk, vi);
#endif
    return h == m;
}

// candidate_set.emplace(-dist, id) then top_candidates.emplace(dist, id) (par_push twice): the two
// heaps are disjoint, so both ancestor reads go out in one LDS round trip. Returns true when dist
// became top_candidates' root.
__device__ __forceinline__ bool par_push2(KV *Cd, int clen, KV *T, int tlen, float dist, uint32_t id)
{
    const int lane = lane_id_local();
    const int j = lane + 1;
    const int chole = clen - 1, cm = heap_depth(chole);
    const int thole = tlen - 1, tm = heap_depth(thole);
    const bool cvalid = j <= cm, tvalid = j <= tm;
    KV ca = Cd[cvalid ? ((chole + 1) >> j) - 1 : 0];
    KV ta = T[tvalid ? ((thole + 1) >> j) - 1 : 0];
    asm volatile("" : "+v"(ca.x), "+v"(ca.y), "+v"(ta.x), "+v"(ta.y));
    const bool clt = cvalid && kv_key(ca) < -dist;
    const int hc = __popcll(bal(clt));
    const bool tlt = tvalid && kv_key(ta) < dist;
    const int ht = __popcll(bal(tlt));
#if DRM_FLAT_MW
    if (lane <= hc)
        Cd[((chole + 1) >> lane) - 1] = lane < hc ? ca : kv_make(-dist, id);
    if (lane <= ht)
        T[((thole + 1) >> lane) - 1] = lane < ht ? ta : kv_make(dist, id);
#else
    if (clt)
        Cd[((chole + 1) >> (j - 1)) - 1] = ca;
    if (lane == 0)
        Cd[((chole + 1) >> hc) - 1] = kv_make(-dist, id);
    if (tlt)
        T[((thole + 1) >> (j - 1)) - 1] = ta;
    if (lane == 0)
        T[((thole + 1) >> ht) - 1] = kv_make(dist, id);
#endif
    return ht == tm;
}

// pop_heap + pop_back for len > 1 (libstdc++ __adjust_heap then __push_heap of the old last
// element): the hole walks from the root to a leaf along the larger child (ties -> right child, a
// lone left child taken), then the old last element v sifts back up that same path. Net effect on
// the path P_0 = root .. P_m = leaf: with h = #{i >= 1 : key(P_i) < v}, P_0 .. P_{m-h-1} each take
// their successor's entry, P_{m-h} takes v, the rest stay (keys along the path only fall, so those
// P_i are a suffix). Lanes own nodes p = lane + 64 jj and read both children of p, so the child
// choices are one ballot per 64 nodes; the leaf is found by a scalar walk over those bits (heap_walk);
// then lane i reads P_{i+1} (the entry that moves up into P_i), one ballot gives h, one write phase.
// NN = node groups (L <= 128 NN + 1). Children are read without a bounds select: slots up to 128 NN
// stay inside the wave's LDS (the heap regions are followed by others) and entries past L never take
// part. Returns the new root key.
template <int NN> __device__ __forceinline__ int heap_walk(const uint64_t (&bits)[NN], int L)
{
    // u = node + 1; node u - 1 has a child iff 2u <= L. Nodes 0 .. 63 are all in bits[0].
    int u = 1;
#pragma unroll
    for (int d = 0; d < 7; ++d)
        if (2 * u <= L && (NN == 1 || u <= 64))
            u = 2 * u + (int)((bits[0] >> (u - 1)) & 1ull);
    if constexpr (NN > 1) {
        while (2 * u <= L) {
            const int p = u - 1;
            uint64_t mk = bits[0];
#pragma unroll
            for (int jj = 1; jj < NN; ++jj)
                if ((p >> 6) == jj)
                    mk = bits[jj];
            u = 2 * u + (int)((mk >> (p & 63)) & 1ull);
        }
    }
    return u - 1;
}

template <int NN> __device__ __forceinline__ float par_pop(KV *H, int len)
{
    const int lane = lane_id_local();
    const int L = len - 1;
    // every read of this round trip is issued before the first use: one LDS wait instead of one per
    // read (left alone, the compiler waits for ve, then serialises the child reads on few VGPRs)
    KV ve = H[L];
    uint32_t lk[NN], rk[NN];
#pragma unroll
    for (int jj = 0; jj < NN; ++jj) {
        const int p = lane + 64 * jj;
        lk[jj] = H[2 * p + 1].x;
        rk[jj] = H[2 * p + 2].x;
    }
    asm volatile("" : "+v"(ve.x), "+v"(ve.y), "+v"(lk[0]), "+v"(rk[0]));
    if constexpr (NN > 1) {
        asm volatile("" : "+v"(lk[1]), "+v"(rk[1]), "+v"(lk[NN - 1]), "+v"(rk[NN - 1]));
        if constexpr (NN > 3)
            asm volatile("" : "+v"(lk[2]), "+v"(rk[2]));
    }
    const float vk = __uint_as_float(__builtin_amdgcn_readfirstlane(ve.x)); // uniform (ve is opaque)
    uint64_t bits[NN];
#pragma unroll
    for (int jj = 0; jj < NN; ++jj) {
        const int p = lane + 64 * jj;
        bits[jj] = bal((2 * p + 2 < L) & !(__uint_as_float(rk[jj]) < __uint_as_float(lk[jj])));
    }
    const int leaf = heap_walk<NN>(bits, L);
    const int m = heap_depth(leaf);
    const int j = lane + 1;
    const bool valid = j <= m;
    const KV ce = kv_load(H + (valid ? ((leaf + 1) >> (m - j)) - 1 : 0)); // P_{lane + 1}
    const int h = __popcll(bal(valid & (kv_key(ce) < vk)));
    const int t = m - h; // depth where v lands
#if DRM_FLAT_MW
    if (lane <= t) // P_i takes P_{i+1} for i < t, P_t takes v
        H[((leaf + 1) >> (m - lane)) - 1] = lane < t ? ce : ve;
#else
    if (lane < t)
        H[((leaf + 1) >> (m - lane)) - 1] = ce;
    if (lane == 0)
        H[((leaf + 1) >> h) - 1] = ve;
#endif
    return t > 0 ? __uint_as_float(__builtin_amdgcn_readlane(ce.x, 0)) : vk;
}

#ifndef DRM_FLAT_POP3
#define DRM_FLAT_POP3 1 // 1: three node groups for 129 .. 385-entry heaps (one child read fewer than four)
#endif
// heaps of up to 513 entries (the callers take the serial replay beyond)
__device__ __forceinline__ float par_pop_any(KV *H, int len)
{
    const int L = len - 1;
    if (L <= 128)
        return par_pop<1>(H, len);
#if DRM_FLAT_POP3
    if (L <= 384) // nodes 0 .. 191 (the candidate_set LDS part, 376 entries, stays below)
        return par_pop<3>(H, len);
#endif
    return par_pop<4>(H, len);
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

// Same distances with the query slice in registers (qr[r] = q[sub + 8r], NV = d / 8 per lane) and
// every load of a pass issued before the first use: 16 items per pass, two per lane group, so a
// hop's distances cost one memory round trip instead of one per dimension step.
#ifndef DRM_FLAT_WAVES
#define DRM_FLAT_WAVES 8 // resident waves per SIMD the kernel is register-budgeted for (4x per CU)
#endif
#ifndef DRM_FLAT_CAND_LDS
#define DRM_FLAT_CAND_LDS 376 // candidate_set entries in LDS (5 KB per wave at 8 waves/SIMD); ~2 % of C3 queries outgrow it and finish in the slow loop
#endif
#ifndef DRM_FLAT_VIS_LOAD
#define DRM_FLAT_VIS_LOAD 1 // 1: visited test by L2 loads + marking of fresh links only; 0: returning atomicOr per link
#endif
#ifndef DRM_FLAT_PUSH2
#define DRM_FLAT_PUSH2 1 // 1: both pushes of an accepted link share one LDS round trip (par_push2)
#endif
#ifndef DRM_FLAT_TWO_SETS
#define DRM_FLAT_TWO_SETS 0 // 1: 16 items per pass (two per lane group); 0: 8 (fewer VGPRs)
#endif
#ifndef DRM_FLAT_Q_REGS
#define DRM_FLAT_Q_REGS 1 // 1: the query slice stays in 16 VGPRs; 0: re-read from LDS per pass (occupancy)
#endif
#ifndef DRM_FLAT_PK
#define DRM_FLAT_PK 0 // 1: packed-fp32 differences and squares (v_pk_add_f32 / v_pk_mul_f32): fewer
                      // instructions but measured slower (12.8 vs 12.45 ms in one-box A/B), so off
#endif
typedef float f32x2 __attribute__((ext_vector_type(2)));
template <int NV>
__device__ __forceinline__ void l2_items_reg(const FlatArgs &a, const float *q, const float (&qreg)[NV],
                                             const uint32_t *ids, int nitem, float *out)
{
    const int lane = lane_id_local(), grp = lane >> 3, sub = lane & 7;
    for (int base = 0; base < nitem; base += DRM_FLAT_TWO_SETS ? 16 : 8) {
        float qr[NV];
#pragma unroll
        for (int r = 0; r < NV; ++r)
            qr[r] = DRM_FLAT_Q_REGS ? qreg[r] : q[sub + 8 * r];
        const int f0 = base + grp, f1 = base + 8 + grp;
        const bool two = DRM_FLAT_TWO_SETS && base + 8 < nitem; // wave-uniform
        const float *v0 = a.vec + (size_t)ids[min(f0, nitem - 1)] * (size_t)(8 * NV) + sub;
        const float *v1 = a.vec + (size_t)ids[min(f1, nitem - 1)] * (size_t)(8 * NV) + sub;
        float t0[NV], t1[NV];
#pragma unroll
        for (int r = 0; r < NV; ++r)
            t0[r] = v0[8 * r];
        if (two) {
#pragma unroll
            for (int r = 0; r < NV; ++r)
                t1[r] = v1[8 * r];
        }
        float acc0 = 0.0f, acc1 = 0.0f;
#if DRM_FLAT_PK
        // dims r, r + 1 of the lane's accumulator: the differences and squares as v_pk_add_f32 /
        // v_pk_mul_f32 (two IEEE ops per lane, the same roundings), the adds stay sequential
#pragma unroll
        for (int r = 0; r + 1 < NV; r += 2) {
            const f32x2 qq = {qr[r], qr[r + 1]};
            const f32x2 tt = {t0[r], t0[r + 1]};
            const f32x2 df = qq - tt;
            const f32x2 sq = df * df;
            acc0 = __fadd_rn(acc0, sq.x);
            acc0 = __fadd_rn(acc0, sq.y);
        }
        if (NV & 1) {
            const float df = __fsub_rn(qr[NV - 1], t0[NV - 1]);
            acc0 = __fadd_rn(acc0, __fmul_rn(df, df));
        }
#else
#pragma unroll
        for (int r = 0; r < NV; ++r) {
            const float df = __fsub_rn(qr[r], t0[r]);
            acc0 = __fadd_rn(acc0, __fmul_rn(df, df));
        }
#endif
        uint32_t p0 = __float_as_uint(acc0);
#pragma unroll
        for (int s = 1; s < 8; ++s) {
            const uint32_t t = dpp_row_shr1(p0);
            if (sub == s)
                p0 = __float_as_uint(__fadd_rn(__uint_as_float(t), __uint_as_float(p0)));
        }
        if (f0 < nitem && sub == 7)
            out[f0] = __uint_as_float(p0);
        if (two) {
#pragma unroll
            for (int r = 0; r < NV; ++r) {
                const float df = __fsub_rn(qr[r], t1[r]);
                acc1 = __fadd_rn(acc1, __fmul_rn(df, df));
            }
            uint32_t p1 = __float_as_uint(acc1);
#pragma unroll
            for (int s = 1; s < 8; ++s) {
                const uint32_t t = dpp_row_shr1(p1);
                if (sub == s)
                    p1 = __float_as_uint(__fadd_rn(__uint_as_float(t), __uint_as_float(p1)));
            }
            if (f1 < nitem && sub == 7)
                out[f1] = __uint_as_float(p1);
        }
    }
    __syncthreads();
}

template <int NV>
__device__ __forceinline__ void l2_dispatch(const FlatArgs &a, const float *q, const float (&qr)[NV > 0 ? NV : 1],
                                            const uint32_t *ids, int nitem, float *out)
{
    if constexpr (NV > 0)
        l2_items_reg<NV>(a, q, qr, ids, nitem, out);
    else
        l2_items(a, q, ids, nitem, out);
}

// ---- Out-of-line slow paths: heaps that reach past their LDS part (candidate_set beyond cand_lds
// entries, or top_candidates at large ef) take the serial replay on lane 0. Kept out of line so that
// no global-memory access sits inside the common path's loops: the wait for one would also wait for
// the outstanding row prefetch (vmcnt is in order).
struct ConsState {
    int top_len, cand_len;
    float lb;
    int overflow;
};

__device__ __forceinline__ void serial_cand_pop(HeapRef<true> cand, int len)
{
    if (lane_id() == 0)
        stl_pop(cand, len);
    __syncthreads();
}

// consideration of the fresh links from chunk `base` (remaining candidates `mask`) onward, any heap
// sizes: the same test and heap updates as the fast loop, serial where a heap leaves LDS
__device__ __forceinline__ ConsState slow_consider(const float *fd, const uint32_t *fid, int nf, int base0,
                                                             uint64_t mask0, ConsState st, HeapRef<true> top,
                                                             HeapRef<true> cand, KV *topkv, KV *cdkv, int ef,
                                                             int cand_lds, int cand_cap, bool top_par, int *sh)
{
    const int lane = lane_id();
    for (int base = base0; base < nf; base += 64) {
        const int f = base + lane;
        const float dl = f < nf ? fd[f] : INFINITY;
        const uint32_t il = f < nf ? fid[f] : 0u;
        uint64_t mask = base == base0 ? mask0 : bal(f < nf && (st.top_len < ef || st.lb > dl));
        while (mask) {
            const int b = __builtin_ctzll(mask);
            mask &= mask - 1;
            const float dist = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(dl), b));
            if (!(st.top_len < ef || st.lb > dist))
                continue;
            if (st.cand_len >= cand_cap) {
                st.overflow = 1;
                return st;
            }
            const uint32_t id = __builtin_amdgcn_readlane(il, b);
            if (++st.cand_len <= cand_lds) {
                par_push(cdkv, st.cand_len, -dist, id);
            } else {
                if (lane == 0) {
                    cand.set(st.cand_len - 1, -dist, id);
                    stl_push(cand, st.cand_len, -dist, id);
                }
                __syncthreads();
            }
            ++st.top_len;
            if (top_par) {
                if (par_push(topkv, st.top_len, dist, id))
                    st.lb = dist;
                while (st.top_len > ef)
                    st.lb = par_pop_any(topkv, st.top_len--);
            } else {
                if (lane == 0) {
                    top.set(st.top_len - 1, dist, id);
                    stl_push(top, st.top_len, dist, id);
                    int tl = st.top_len;
                    while (tl > ef)
                        stl_pop(top, tl--);
                    sh[2] = __float_as_int(top.key(0));
                }
                __syncthreads();
                st.top_len = min(st.top_len, ef);
                st.lb = __int_as_float(sh[2]);
            }
        }
    }
    return st;
}

// Links of c not yet visited, in row order -> fid[0 .. nf), each marked in the visited bitmap. Row
// slots past the link count hold ~0u (drm_flat_index_load), so the first 128 slots need no count;
// the caller may have issued their loads already (have_pf: pf_w0 / pf_w1 = slots lane, 64 + lane).
__device__ __forceinline__ int expand_row(const FlatArgs &a, uint32_t c, uint32_t *vis, uint32_t *fid, bool have_pf,
                                          uint32_t pf_w0, uint32_t pf_w1)
{
    const int lane = lane_id_local();
    const uint32_t *row = a.l0 + (size_t)c * (size_t)a.maxM0;
    uint32_t r0, r1;
    if (have_pf) {
        r0 = lane < a.maxM0 ? pf_w0 : ~0u; // the loads were clamped to the row (see the hop loop)
        r1 = 64 + lane < a.maxM0 ? pf_w1 : ~0u;
    } else {
        r0 = lane < a.maxM0 ? row[lane] : ~0u;
        r1 = 64 + lane < a.maxM0 ? row[64 + lane] : ~0u;
    }
    const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
    const int nbase = a.maxM0 <= 128 ? 128 : (int)(a.l0cnt[c] & 0xFFFFu);
    int nf = 0;
    for (int base = 0; base < nbase; base += 128) { // one pass when maxM0 <= 128
        const int j0 = base + lane, j1 = base + 64 + lane;
        const uint32_t v0 = base == 0 ? r0 : (j0 < a.maxM0 ? row[j0] : ~0u);
        const uint32_t v1 = base == 0 ? r1 : (j1 < a.maxM0 ? row[j1] : ~0u);
        const bool act0 = v0 != ~0u, act1 = v1 != ~0u;
        const uint32_t b0 = 1u << (v0 & 31), b1 = 1u << (v1 & 31);
        uint32_t o0 = ~0u, o1 = ~0u;
#if DRM_FLAT_VIS_LOAD
        // test with plain L2 loads, mark only the fresh links (non-returning atomics). The wave's
        // earlier marks are all performed: VMEM completes in order and the row these ids came from
        // was issued after them.
        if (act0)
            o0 = __hip_atomic_load(&vis[v0 >> 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (act1)
            o1 = __hip_atomic_load(&vis[v1 >> 5], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
        if (act0)
            o0 = atomicOr(&vis[v0 >> 5], b0);
        if (act1)
            o1 = atomicOr(&vis[v1 >> 5], b1);
#endif
        bool fresh0 = (o0 & b0) == 0u, fresh1 = (o1 & b1) == 0u;
        if (a.check_dups) { // a repeated link in one row: only its first occurrence is fresh
            const int cnt = (int)(a.l0cnt[c] & 0xFFFFu);
            for (int jj = 0; jj < cnt; ++jj) {
                const uint32_t vj = row[jj];
                fresh0 = fresh0 && !(jj < j0 && vj == v0);
                fresh1 = fresh1 && !(jj < j1 && vj == v1);
            }
        }
#if DRM_FLAT_VIS_LOAD
        if (fresh0)
            __hip_atomic_fetch_or(&vis[v0 >> 5], b0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (fresh1)
            __hip_atomic_fetch_or(&vis[v1 >> 5], b1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
        const uint64_t fm0 = bal(fresh0), fm1 = bal(fresh1);
        const int n0 = __popcll(fm0);
        if (fresh0)
            fid[nf + __popcll(fm0 & below)] = v0;
        if (fresh1)
            fid[nf + n0 + __popcll(fm1 & below)] = v1;
        nf += n0 + __popcll(fm1);
    }
    __syncthreads();
    return nf;
}

// VisitedTable reset list: this hop's fresh ids, appended once the hop's bookkeeping is done, so the
// stores' acknowledgements overlap the next hop's row load and visited atomics (which wait on vmcnt
// anyway) instead of stalling this hop's distance loads.
__device__ __forceinline__ int append_clear(const FlatArgs &a, int32_t *clr, int clear_n, const uint32_t *fid, int nf)
{
    for (int f = lane_id_local(); f < nf; f += 64)
        if (clear_n + f < a.clear_cap)
            clr[clear_n + f] = (int32_t)fid[f];
    return clear_n + nf;
}

// Ascending (key, label) order of 128 pairs held as element i = lane + 64 r in register r: a bitonic
// network, partners across lanes by ds_bpermute (j < 64) or within the lane (j = 64). Equal pairs
// (only the +inf padding) may swap freely.
__device__ __forceinline__ bool kl_less(float ka, uint64_t la, float kb, uint64_t lb)
{
    return ka < kb || (ka == kb && la < lb);
}

__device__ __forceinline__ void bitonic128(float (&k)[2], uint64_t (&l)[2])
{
    const int lane = lane_id_local();
#pragma unroll
    for (int kk = 2; kk <= 128; kk <<= 1) {
#pragma unroll
        for (int j = kk >> 1; j > 0; j >>= 1) {
            if (j == 64) { // kk == 128: ascending
                if (kl_less(k[1], l[1], k[0], l[0])) {
                    const float tk = k[0];
                    const uint64_t tl = l[0];
                    k[0] = k[1];
                    l[0] = l[1];
                    k[1] = tk;
                    l[1] = tl;
                }
                continue;
            }
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const float pk = __shfl_xor(k[r], j);
                const uint64_t pl = __shfl_xor(l[r], j);
                const bool lower = (lane & j) == 0;
                const bool asc = ((lane + 64 * r) & kk) == 0;
                const bool take = lower == asc ? kl_less(pk, pl, k[r], l[r]) : kl_less(k[r], l[r], pk, pl);
                k[r] = take ? pk : k[r];
                l[r] = take ? pl : l[r];
            }
        }
    }
}

#define FLAT_STAMP(idx)                                                                                     \
    do {                                                                                                    \
        if (STAMPS) {                                                                                       \
            __builtin_amdgcn_sched_barrier(0);                                                              \
            const uint64_t _t = __builtin_amdgcn_s_memtime();                                               \
            __builtin_amdgcn_sched_barrier(0);                                                              \
            st_acc[idx] += _t - st_last;                                                                    \
            st_last = _t;                                                                                   \
        }                                                                                                   \
    } while (0)

// NV = d / 8 when the query slice lives in registers (d = 128 -> 16), 0 for the generic LDS path. Both
// libstdc++ heaps are replayed exactly (any input, ties included).
// Bounded: a query past a.hop_bound level-0 hops, or a wave past a.item_bound work items, ends with an error count
// (a.errors; drm_flat_search returns DRM_ERR_INTERNAL) instead of looping.
// MODE 0: the whole search. MODE 1: the same with the common shape as compile-time constants
// (d = 128, k = ef = 128, maxM0 = 128, maxM = 64, no repeated links, top heap fully in LDS): fewer
// live SGPRs and no kernel-argument reloads in the hop loop.
template <int NV, bool STAMPS, int MODE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(DRM_FLAT_WAVES))) void hnsw_flat_search_kernel(FlatArgs a_in)
{
    FlatArgs a = a_in;
    if (MODE == 1) {
        a.d = 128;
        a.k = 128;
        a.ef = 128;
        a.maxM0 = 128;
        a.maxM = 64;
        a.top_lds = 129;
        a.top_ovf_cap = 0;
        a.cand_lds = DRM_FLAT_CAND_LDS;
        a.check_dups = 0;
    }
    extern __shared__ __align__(16) unsigned char smem[];
    const int lane = lane_id();
    uint64_t st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t st_last = STAMPS ? __builtin_amdgcn_s_memtime() : 0;
    constexpr bool q_lds = NV == 0 || !DRM_FLAT_Q_REGS;               // query slice in registers otherwise
    float *q = reinterpret_cast<float *>(smem);                      // [d] (q_lds)
    KV *topkv = reinterpret_cast<KV *>(q + (q_lds ? a.d : 0));      // [top_lds] (d % 16 == 0: aligned)
    KV *cdkv = topkv + a.top_lds;                                   // [cand_lds]
    uint32_t *fid = reinterpret_cast<uint32_t *>(cdkv + a.cand_lds); // [maxM0] fresh ids / upper links
    float *fd = reinterpret_cast<float *>(fid + a.maxM0);           // [maxM0] their distances
    int *sh = reinterpret_cast<int *>(fd + a.maxM0);                // [4] broadcast scalars
    uint32_t *vis = a.visited + (size_t)blockIdx.x * (size_t)a.vis_words;
    int32_t *clr = a.clear_list + (size_t)blockIdx.x * (size_t)a.clear_cap;
    const HeapRef<true> top{(DRM_LDS uint64_t *)topkv, a.top_lds,
                            (DRM_GLOBAL float *)(a.top_ovf_k + (size_t)blockIdx.x * (size_t)a.top_ovf_cap),
                            (DRM_GLOBAL uint32_t *)(a.top_ovf_i + (size_t)blockIdx.x * (size_t)a.top_ovf_cap)};
    const HeapRef<true> cand{(DRM_LDS uint64_t *)cdkv, a.cand_lds,
                             (DRM_GLOBAL float *)(a.cand_ovf_k + (size_t)blockIdx.x * (size_t)a.cand_ovf_cap),
                             (DRM_GLOBAL uint32_t *)(a.cand_ovf_i + (size_t)blockIdx.x * (size_t)a.cand_ovf_cap)};
    const int cand_cap = a.cand_lds + (int)a.cand_ovf_cap;
    int64_t taken = 0;
    for (;;) {
        const int qi = wave_next_item(a.counter, lane);
        if ((int64_t)qi >= a.n)
            break;
        if (++taken > a.item_bound) { // more items than the queue holds: a broken work-queue fetch
            if (lane == 0)
                atomicAdd(a.errors, 1u);
            break;
        }
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
        float qr[NV > 0 ? NV : 1];
        if constexpr (NV > 0 && DRM_FLAT_Q_REGS) {
#pragma unroll
            for (int r = 0; r < NV; ++r)
                qr[r] = a.x[(int64_t)qi * a.d + (lane & 7) + 8 * r];
        } else {
            for (int t = lane; t < a.d; t += 64)
                q[t] = a.x[(int64_t)qi * a.d + t];
        }
        __syncthreads();
        int ndis = 0, nhops = 0;
        // --- searchKnn: greedy descent on levels maxlevel .. 1
        uint32_t cur = a.ep;
        float curdist = 0.0f;
        int nhops_up = 0;
        {
            if (lane == 0)
                fid[0] = cur;
            __syncthreads();
            l2_dispatch<NV>(a, q, qr, fid, 1, fd);
            curdist = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(fd[0])));
            ndis++;
        }
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
                l2_dispatch<NV>(a, q, qr, fid, size, fd);
                bool changed = false;
                for (int j = 0; j < size; ++j) { // sequential `if (d < curdist)` (uniform)
                    const float dd = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(fd[j])));
                    if (dd < curdist) {
                        curdist = dd;
                        cur = (uint32_t)__builtin_amdgcn_readfirstlane((int)fid[j]);
                        changed = true;
                    }
                }
                __syncthreads();
                if (!changed)
                    break;
            }
        }
        {
        // --- searchBaseLayerST<bare_bone_search = true>(cur, q, max(ef, k))
        int clear_n = 1;
        if (lane == 0) {
            atomicOr(&vis[cur >> 5], 1u << (cur & 31));
            if (a.clear_cap > 0)
                clr[0] = (int32_t)cur;
        }
        int nres = 0;
        bool overrun = false;
        {
            int top_len = 1, cand_len = 1;
            float lowerBound = curdist;
            bool overflow = false;
            if (lane == 0) {
                top.set(0, curdist, cur);
                cand.set(0, -curdist, cur);
            }
            __syncthreads();
            FLAT_STAMP(0); // query setup + upper levels
            const bool top_par = a.ef + 1 <= min(a.top_lds, 513); // top_candidates in LDS, parallel ops
            // Fast hop loop: both heaps entirely in LDS, wave-parallel heap ops, no global access but
            // the row / visited / distance / prefetch traffic itself. The first link that would take
            // candidate_set past its LDS part ends it; the query then finishes in the slow loop below
            // (also taken from the start when top_candidates does not fit). Keeping the serial
            // replay's global accesses out of this loop keeps its waits off the row prefetch.
            bool slow = !top_par;
            int slow_base = -1, slow_nf = 0;
            uint64_t slow_mask = 0;
            while (!slow && cand_len > 0) {
                if (nhops - nhops_up > a.hop_bound) { // a node is expanded at most once: the bookkeeping is broken
                    overrun = true;
                    break;
                }
                const KV croot = kv_load(cdkv); // slot 0 is always in LDS
                const float cdist = -__uint_as_float(__builtin_amdgcn_readfirstlane(croot.x));
                if (cdist > lowerBound)
                    break;
                const uint32_t c = __builtin_amdgcn_readfirstlane(croot.y);
                // the row loads go out before the pop, which then overlaps their latency
                const uint32_t *crow = a.l0 + (size_t)c * (size_t)a.maxM0;
                // unconditional (clamped) loads, masked when used: no register init that would wait
                // for the VMEM counter to drain first
                const uint32_t w0 = crow[min(lane, a.maxM0 - 1)];
                const uint32_t w1 = crow[min(64 + lane, a.maxM0 - 1)];
                __syncthreads();
                if (cand_len > 1)
                    par_pop_any(cdkv, cand_len);
                cand_len--;
                nhops++;
                FLAT_STAMP(1); // candidate_set pop
                const int nf = expand_row(a, c, vis, fid, true, w0, w1);
                FLAT_STAMP(2); // row + visited
                l2_dispatch<NV>(a, q, qr, fid, nf, fd);
                ndis += nf;
                FLAT_STAMP(3); // distances
                // consideration in link order: `if (top.size() < ef || lowerBound > dist)` push both
                // heaps, trim top to ef. lowerBound only falls once top is full, so one ballot per 64
                // links picks a superset of the accepted ones (the exact test is rechecked).
                for (int base = 0; base < nf && !slow; base += 64) {
                    const int f = base + lane;
                    const float dl = f < nf ? fd[f] : INFINITY;
                    const uint32_t il = f < nf ? fid[f] : 0u;
                    uint64_t mask = bal(f < nf && (top_len < a.ef || lowerBound > dl));
                    while (mask) {
                        const int b = __builtin_ctzll(mask);
                        const float dist = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(dl), b));
                        if (!(top_len < a.ef || lowerBound > dist)) {
                            mask &= mask - 1;
                            continue;
                        }
                        if (cand_len + 1 > a.cand_lds) { // hand the rest of this hop to the slow loop
                            slow = true;
                            slow_base = base;
                            slow_mask = mask;
                            slow_nf = nf;
                            break;
                        }
                        mask &= mask - 1;
                        const uint32_t id = __builtin_amdgcn_readlane(il, b);
#if DRM_FLAT_PUSH2
                        if (par_push2(cdkv, ++cand_len, topkv, ++top_len, dist, id))
                            lowerBound = dist;
#else
                        par_push(cdkv, ++cand_len, -dist, id);
                        if (par_push(topkv, ++top_len, dist, id))
                            lowerBound = dist;
#endif
                        while (top_len > a.ef)
                            lowerBound = par_pop_any(topkv, top_len--);
                    }
                }
                clear_n = append_clear(a, clr, clear_n, fid, nf);
                __syncthreads();
                FLAT_STAMP(4); // consideration: heap pushes / pops
            }
            if (slow && !overrun) {
                ConsState st{top_len, cand_len, lowerBound, 0};
                if (slow_base >= 0) { // the rest of the interrupted hop (its fresh links are still in LDS)
                    st = slow_consider(fd, fid, slow_nf, slow_base, slow_mask, st, top, cand, topkv, cdkv, a.ef,
                                       a.cand_lds, cand_cap, top_par, sh);
                    clear_n = append_clear(a, clr, clear_n, fid, slow_nf);
                }
                while (!st.overflow && st.cand_len > 0) {
                    if (nhops - nhops_up > a.hop_bound) {
                        overrun = true;
                        break;
                    }
                    const float cdist = -cand.key(0);
                    if (cdist > st.lb)
                        break;
                    const uint32_t c = cand.id(0);
                    __syncthreads();
                    if (st.cand_len > 1) {
                        if (st.cand_len <= a.cand_lds)
                            par_pop_any(cdkv, st.cand_len);
                        else
                            serial_cand_pop(cand, st.cand_len);
                    }
                    st.cand_len--;
                    nhops++;
                    const int nf = expand_row(a, c, vis, fid, false, 0u, 0u);
                    l2_dispatch<NV>(a, q, qr, fid, nf, fd);
                    ndis += nf;
                    const int f = lane;
                    const float dl = f < nf ? fd[f] : INFINITY;
                    st = slow_consider(fd, fid, nf, 0, bal(f < nf && (st.top_len < a.ef || st.lb > dl)), st, top,
                                       cand, topkv, cdkv, a.ef, a.cand_lds, cand_cap, top_par, sh);
                    clear_n = append_clear(a, clr, clear_n, fid, nf);
                    __syncthreads();
                }
                top_len = st.top_len;
                cand_len = st.cand_len;
                lowerBound = st.lb;
                overflow = st.overflow != 0;
            }
            if (lane == 0 && overflow)
                atomicAdd(a.overflow, 1u); // candidate_set overflow: reported by the host entry points
            // --- while (top.size() > k) top.pop(); then order survivors by (dist, label)
            if (top_par) {
                while (top_len > a.k)
                    par_pop_any(topkv, top_len--);
            } else {
                if (lane == 0) {
                    int tl = top_len;
                    while (tl > a.k)
                        stl_pop(top, tl--);
                }
                top_len = min(top_len, a.k);
            }
            __syncthreads();
            nres = top_len;
            // searchKnnCloserFirst order: ascending (dist, label)
            if (top_par && nres <= 128) { // wave bitonic sort of the (at most 128) survivors
                float sk[2];
                uint64_t sl[2];
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    const int e = lane + 64 * r;
                    const bool v = e < nres;
                    const KV te = topkv[v ? e : 0];
                    sk[r] = v ? kv_key(te) : INFINITY;
                    sl[r] = v ? a.labels[te.y] : ~0ull;
                }
                bitonic128(sk, sl);
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    const int e = lane + 64 * r;
                    if (e < nres) {
                        Dq[e] = sk[r];
                        Lq[e] = sl[r];
                    }
                }
            } else { // rank by counting, labels staged in the (now idle) candidate-heap LDS when they fit
                uint64_t *lab = reinterpret_cast<uint64_t *>(cdkv);
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
            }
        }
        for (int j = nres + lane; j < a.k; j += 64) {
            Dq[j] = INFINITY;
            Lq[j] = ~0ull;
        }
        if (lane == 0) {
            a.ndis[qi] = overrun ? -1 : ndis;
            a.nhops[qi] = overrun ? -1 : nhops;
            if (a.nhops_upper)
                a.nhops_upper[qi] = nhops_up;
            if (overrun)
                atomicAdd(a.errors, 1u);
        }
        // VisitedTable reset: clear exactly the bits this query set
        // (no wait for these stores: VMEM completes in order, so the next query's first visited test,
        // which waits for loads issued after them, already sees them performed)
        if (clear_n <= a.clear_cap) {
#pragma unroll 4
            for (int t = lane; t < clear_n; t += 64)
                vis[(uint32_t)clr[t] >> 5] = 0u;
        } else {
            for (int64_t w = lane; w < a.vis_words; w += 64)
                vis[w] = 0u;
        }
        __syncthreads();
        FLAT_STAMP(5); // result ordering + reset
        }
    }
    if (STAMPS && lane == 0 && a.stamps)
        for (int i = 0; i < 8; ++i)
            atomicAdd(reinterpret_cast<unsigned long long *>(a.stamps) + i, (unsigned long long)st_acc[i]);
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
    const int cand_lds = DRM_FLAT_CAND_LDS;
    const int top_lds = std::min(efc + 1, 1024); // top_candidates beyond this continue in global memory
    const int64_t top_ovf = (int64_t)efc + 1 - top_lds;
    const bool q_lds = ix.d != 128 || !DRM_FLAT_Q_REGS; // the d = 128 kernel keeps the query in VGPRs
    const size_t lds = sizeof(float) * (q_lds ? (size_t)ix.d : 0) + 8 * (size_t)top_lds + 8 * (size_t)cand_lds +
                       8 * (size_t)ix.maxM0 + 16;
    if (lds > 160 * 1024)
        throw Error(DRM_ERR_UNSUPPORTED, "fp32 search workspace does not fit in LDS (ef too large)");
    const int per_cu = std::max(1, std::min(std::min(ix.waves_per_cu, 4 * DRM_FLAT_WAVES), (int)((160 * 1024) / lds)));
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
        DRM_HIP_CHECK(malloc_big((void **)&ix.visited, sizeof(uint32_t) * (size_t)alloc * (size_t)ix.vis_words, kBigVisited));
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
        DRM_HIP_CHECK(hipMalloc(&ix.counter, 8 * sizeof(uint32_t)));
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
    a.overflow = ix.counter + 1;
    a.errors = ix.counter + 3;
    a.hop_bound = ix.hop_bound > 0 ? std::min(ix.hop_bound, ix.ntotal) : ix.ntotal;
    a.item_bound = ix.item_bound > 0 ? std::min(ix.item_bound, n) : n;
    a.check_dups = ix.has_dup_links;
    a.cand_lds = cand_lds;
    a.cand_ovf_k = ix.cand_ovf_k;
    a.cand_ovf_i = ix.cand_ovf_i;
    a.cand_ovf_cap = ix.cand_ovf_cap;
    a.top_lds = top_lds;
    a.top_ovf_k = ix.top_ovf_k;
    a.top_ovf_i = ix.top_ovf_i;
    a.top_ovf_cap = ix.top_ovf_cap;
    DRM_HIP_CHECK(hipMemsetAsync(ix.counter, 0, 8 * sizeof(uint32_t), stream));
    a.stamps = ix.stamps;
#define DRM_FLAT_MAIN(M_)                                                                                      \
    if (ix.d == 128) {                                                                                          \
        if (a.stamps)                                                                                           \
            hipLaunchKernelGGL((hnsw_flat_search_kernel<16, true, M_>), dim3(slots), dim3(64), lds, stream, a); \
        else                                                                                                    \
            hipLaunchKernelGGL((hnsw_flat_search_kernel<16, false, M_>), dim3(slots), dim3(64), lds, stream, a); \
    } else {                                                                                                    \
        if (a.stamps)                                                                                           \
            hipLaunchKernelGGL((hnsw_flat_search_kernel<0, true, M_>), dim3(slots), dim3(64), lds, stream, a); \
        else                                                                                                    \
            hipLaunchKernelGGL((hnsw_flat_search_kernel<0, false, M_>), dim3(slots), dim3(64), lds, stream, a); \
    }
    const bool fixed = ix.d == 128 && k == 128 && efc == 128 && ix.maxM0 == 128 && ix.maxM == 64 && top_lds == 129 &&
                       !ix.has_dup_links && !a.stamps && DRM_FLAT_Q_REGS;
    if (fixed)
        hipLaunchKernelGGL((hnsw_flat_search_kernel<16, false, 1>), dim3(slots), dim3(64), lds, stream, a);
    else {
        DRM_FLAT_MAIN(0)
    }
#undef DRM_FLAT_MAIN
    DRM_HIP_CHECK(hipGetLastError());
}

} // namespace drm
