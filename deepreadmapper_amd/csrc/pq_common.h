// deepreadmapper_amd/csrc/pq_common.h -- device helpers shared by the HNSW-PQ search kernels
// (hnsw_search.hip: the general exact kernel; hnsw_pq_fast.hip: the lean ef <= 128 kernel).
// set_query / compute_distance_table, the PQ-ADC distance and greedy_update_nearest restate upstream
// faiss (IndexPQ.cpp, ProductQuantizer.cpp, HNSW.cpp) with a fixed fp32 op order and no FMA; the
// oracle (oracle/drm_oracle.c) uses the same order, so results are bit-identical to it.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

#include "drm_device.h"

#pragma clang fp contract(off)

namespace drm {
namespace {

// Distances are compared through an order-preserving uint32 image (ord32), so every heap
// comparison is integer and runs on the scalar unit: float a < b  <=>  ord32(a) < ord32(b)
// (no NaN, and +0 only: distances are sums of squares starting from +0.0f).
__device__ __forceinline__ uint32_t ord32(float f)
{
    uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
// ord32 of a value known to have its sign bit clear (a PQ-ADC distance: a sum of non-negative LUT entries from +0.0)
__device__ __forceinline__ uint32_t ord32_nonneg(float f) { return __float_as_uint(f) | 0x80000000u; }
__device__ __forceinline__ float unord32(uint32_t o)
{
    return __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o);
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
    // every lane holds the minimum now; readfirstlane tells the compiler so (a shuffle result is a
    // divergent value to its uniformity analysis, and branches on it would become exec-masked)
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }
__device__ __forceinline__ uint64_t lanes_below(int lane) { return lane == 0 ? 0ull : (~0ull >> (64 - lane)); }
__device__ __forceinline__ uint32_t ufirst(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }

// faiss::CMax<float, TI>::cmp2 on (ord32 key, id)
__device__ __forceinline__ bool cmp2(uint32_t k1, uint32_t k2, int32_t i1, int32_t i2)
{
    return (k1 > k2) || ((k1 == k2) && (i1 > i2));
}

// ---- DPP wave reductions (gfx9 DPP: row_shr:1/2/4/8, row_bcast:15/31, wave_shr:1)
__device__ __forceinline__ uint32_t dpp_u32(uint32_t old, uint32_t v, int ctrl, int row_mask)
{
    switch (ctrl) { // the builtin needs compile-time controls
    case 0x111: return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x111, 0xF, 0xF, false);
    case 0x112: return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x112, 0xF, 0xF, false);
    case 0x114: return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x114, 0xF, 0xF, false);
    case 0x118: return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x118, 0xF, 0xF, false);
    case 0x142: return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x142, 0xA, 0xF, false);
    default: return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x143, 0xC, 0xF, false);
    }
}
// min over the 64 lanes, returned wave-uniform
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v)
{
    // row rotations (row_ror:1/2/4/8) first: every lane of a row reads a valid lane (bound_ctrl's zero-fill never
    // applies), so no identity "old" value -- and no v_mov to initialise one -- is needed, and each stage is one
    // v_min_u32_dpp; after them every lane holds its row's minimum
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x121, 0xF, 0xF, true));
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x122, 0xF, 0xF, true));
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xF, 0xF, true));
    v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, true));
    v = min(v, dpp_u32(0xFFFFFFFFu, v, 0x142, 0xA));
    v = min(v, dpp_u32(0xFFFFFFFFu, v, 0x143, 0xC));
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
// PQ ADC distance of node v: sequential fp32 sum over sub-quantizers starting from 0
// (distance_single_code / distance_four_codes for M < 16) [upstream faiss].
template <bool FAST8>
__device__ __forceinline__ float pq_distance_code(const SearchArgs &a, const float *lut, int32_t v, uint2 c8)
{
    float r = 0.0f;
    if (FAST8) { // M == 8, nbits == 8: the 8-byte code is already in c8
        // +0.0 + x == x for a LUT entry (never -0.0): the sum starts at the first entry, the same bits
        r = lut[c8.x & 255u];
#pragma unroll
        for (int m = 1; m < 4; ++m)
            r = __fadd_rn(r, lut[m * 256 + ((c8.x >> (8 * m)) & 255u)]);
#pragma unroll
        for (int m = 0; m < 4; ++m)
            r = __fadd_rn(r, lut[(m + 4) * 256 + ((c8.y >> (8 * m)) & 255u)]);
        return r;
    }
    const uint8_t *code = a.codes + (size_t)v * a.code_size;
    for (int m = 0; m < a.M; ++m) {
        uint32_t idx;
        if (a.nbits == 8) {
            idx = code[m];
        } else {
            const uint32_t bitpos = (uint32_t)m * (uint32_t)a.nbits;
            const uint32_t byte = bitpos >> 3, shift = bitpos & 7;
            const uint32_t need = shift + (uint32_t)a.nbits;
            uint32_t acc = 0;
            for (uint32_t b = 0; b * 8 < need; ++b)
                acc |= (uint32_t)code[byte + b] << (8 * b);
            idx = (acc >> shift) & ((1u << a.nbits) - 1u);
        }
        r = __fadd_rn(r, lut[m * a.ksub + (int)idx]);
    }
    return r;
}

template <bool FAST8> __device__ __forceinline__ uint2 load_code8(const SearchArgs &a, int32_t v)
{
    if (FAST8)
        return *reinterpret_cast<const uint2 *>(a.codes + (size_t)v * 8);
    return make_uint2(0u, 0u);
}

// set_query: LUT[m][c] = sum_t (x - c)^2 over the sub-vector, sequential t, no FMA
// (PQDistanceComputer::set_query -> compute_distance_table) [upstream faiss]. The query is read
// straight from global memory (every lane of a pass reads the same 64 B: one L1 broadcast), so the
// only LDS a wave owns is its LUT -- 8 KB, i.e. 20 resident waves per CU.
__device__ __forceinline__ void build_lut(const SearchArgs &a, int64_t q, float *lut, int lane)
{
    const float *qv = a.x + q * a.d;
    if (a.dsub == 16 && (a.ksub & 127) == 0 && a.x_aligned16) {
        // 2 entries of one sub-quantizer per lane per pass, 8 float4 loads in flight
        for (int e0 = lane; e0 < a.M * a.ksub; e0 += 128) {
            const int m = e0 / a.ksub;
            const float4 *xs = reinterpret_cast<const float4 *>(qv + m * 16);
            float4 c[2][4];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const float4 *cp = reinterpret_cast<const float4 *>(a.centroids + (size_t)(e0 + 64 * u) * 16);
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    c[u][i] = cp[i];
            }
            float acc[2] = {0.0f, 0.0f};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float4 x = xs[i];
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    float df = __fsub_rn(x.x, c[u][i].x);
                    acc[u] = __fadd_rn(acc[u], __fmul_rn(df, df));
                    df = __fsub_rn(x.y, c[u][i].y);
                    acc[u] = __fadd_rn(acc[u], __fmul_rn(df, df));
                    df = __fsub_rn(x.z, c[u][i].z);
                    acc[u] = __fadd_rn(acc[u], __fmul_rn(df, df));
                    df = __fsub_rn(x.w, c[u][i].w);
                    acc[u] = __fadd_rn(acc[u], __fmul_rn(df, df));
                }
            }
#pragma unroll
            for (int u = 0; u < 2; ++u)
                lut[e0 + 64 * u] = acc[u];
        }
    } else
    for (int e = lane; e < a.M * a.ksub; e += 64) {
        const int m = e / a.ksub;
        const float *cen = a.centroids + (size_t)e * a.dsub;
        const float *xs = qv + m * a.dsub;
        float acc = 0.0f;
        for (int t = 0; t < a.dsub; ++t) {
            const float diff = __fsub_rn(xs[t], cen[t]);
            acc = __fadd_rn(acc, __fmul_rn(diff, diff));
        }
        lut[e] = acc;
    }
    __syncthreads();

}

// set_query for the lean kernel (M = 8, ksub = 256, dsub = 16, 16-B aligned queries): the same
// per-entry op order as build_lut, with the query sub-vector made wave-uniform (SGPRs) so that only
// the centroids a lane works on occupy VGPRs. A lane sums 2 H entries of a sub-quantizer at once, their 8 H
// centroid loads issued together: 16 / H load round trips per LUT. H = 2 measured 96.0 -> 95.6 ms at C5
// (profiles/r05/ab_search_lut_unroll.txt) but read 13 GB more from HBM per launch (FETCH_SIZE 35.9 -> 48.9 GB,
// profiles/r05/fetch_lut_halves.txt) and ran no faster under the profiler, so both the search and the builder take
// H = 1.
template <int H>
__device__ __forceinline__ void build_lut_m8_ptr(const float *qv, const float *centroids, float *lut, int lane)
{
    typedef float f2 __attribute__((ext_vector_type(2)));
    for (int m = 0; m < 8; ++m) {
        float xs[16];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float4 t = reinterpret_cast<const float4 *>(qv + m * 16)[i];
            xs[4 * i + 0] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, t.x)));
            xs[4 * i + 1] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, t.y)));
            xs[4 * i + 2] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, t.z)));
            xs[4 * i + 3] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, t.w)));
        }
#pragma unroll 1
        for (int c0 = 0; c0 < 256; c0 += 128 * H) {
        const float4 *cq = reinterpret_cast<const float4 *>(centroids) + ((size_t)m * 256 + c0 + lane) * 4;
        float4 u[H][4], w[H][4];
#pragma unroll
        for (int h = 0; h < H; ++h)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                u[h][i] = cq[h * 512 + i];
                w[h][i] = cq[h * 512 + 256 + i];
            }
        // two entries' chains side by side in the halves of packed fp32 ops (v_pk_add_f32 / v_pk_mul_f32): each
        // entry keeps its own sequence of IEEE round-to-nearest subtract, multiply, add (no contraction)
#pragma unroll
        for (int h = 0; h < H; ++h) {
            f2 acc = {0.0f, 0.0f};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float cu[4] = {u[h][i].x, u[h][i].y, u[h][i].z, u[h][i].w};
                const float cw[4] = {w[h][i].x, w[h][i].y, w[h][i].z, w[h][i].w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const f2 x2 = {xs[4 * i + j], xs[4 * i + j]};
                    const f2 c2 = {cu[j], cw[j]};
                    const f2 d = x2 - c2;
                    acc = acc + d * d;
                }
            }
            const int e0 = m * 256 + c0 + h * 128 + lane;
            lut[e0] = acc.x;
            lut[e0 + 64] = acc.y;
        }
        }
    }
    __syncthreads();
}
__device__ __forceinline__ void build_lut_m8(const SearchArgs &a, int64_t q, float *lut, int lane)
{
    build_lut_m8_ptr<1>(a.x + q * a.d, a.centroids, lut, lane);
}

// greedy_update_nearest on levels max_level .. 1 (HNSW::search, upper levels) [upstream faiss]
template <bool FAST8>
__device__ __forceinline__ void greedy_upper(const SearchArgs &a, const float *lut, int lane, int32_t &nearest_out,
                                             uint32_t &dn_out, int &ndis_out, int &nhops_out)
{
    int32_t nearest = a.entry_point;
    uint32_t dn = ufirst(ord32(pq_distance_code<FAST8>(a, lut, nearest, load_code8<FAST8>(a, nearest))));
    int ndis = 0, nhops = 0;
    for (int level = a.max_level; level >= 1; --level) {
        const int cnt = a.cum[level + 1] - a.cum[level];
        for (;;) {
            const int32_t prev = nearest;
            const uint32_t base = a.upper_off[nearest] + (uint32_t)(a.cum[level] - a.cum[1]);
            const int32_t v = (lane < cnt) ? a.upper_nbr[base + lane] : -1;
            const uint64_t neg = __ballot(lane < cnt && v < 0);
            const int nvalid = neg ? (__ffsll((unsigned long long)neg) - 1) : cnt;
            uint32_t dk = 0xFFFFFFFFu;
            if (lane < nvalid)
                dk = ord32(pq_distance_code<FAST8>(a, lut, v, load_code8<FAST8>(a, v)));
            ndis += nvalid;
            nhops += 1;
            // sequential `if (dis < d_nearest)` in link order == first lane holding the minimum
            uint64_t key = (lane < nvalid) ? (((uint64_t)dk << 32) | (uint32_t)lane) : ~0ull;
            key = wave_min_u64(key);
            if (key != ~0ull) {
                const uint32_t bk = (uint32_t)(key >> 32);
                if (bk < dn) {
                    dn = bk;
                    nearest = __builtin_amdgcn_readlane(v, (int)(key & 63));
                }
            }
            if (nearest == prev)
                break;
        }
    }
    nearest_out = nearest;
    dn_out = dn;
    ndis_out = ndis;
    nhops_out = nhops;
}

// Each bitmap slot is owned by exactly one workgroup (one wave) for the whole launch, so a
// workgroup-scope atomic is sufficient: it is performed in the XCD's L2 instead of memory-side.
__device__ __forceinline__ uint32_t vis_test_set(uint32_t *w, uint32_t bit)
{
    return __hip_atomic_fetch_or(w, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

} // namespace
} // namespace drm
