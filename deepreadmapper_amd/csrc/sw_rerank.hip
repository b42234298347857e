// deepreadmapper_amd/csrc/sw_rerank.hip -- Smith-Waterman rerank for gfx950.
//
// Replaces post_process_sw_static (src/utils/post_processor.cpp:454-549) -> find_sequences
// (static, :204-336) -> sw_reranker (src/utils/reranker.cpp:3-51) -> calc_sw_score
// (src/utils/metrics.cpp:10-45). Scores are bit-exact (integer DP), and the top-k order is
// libstdc++ std::partial_sort's, replayed on the device (ties included).
//
// DP mapping (DESIGN.md "SW kernel"): inter-task -- one lane = one (candidate, query) pair, all
// lanes of a workgroup share the query. The DP row over the query (<= LQ columns) lives in LQ
// VGPRs; the loop runs over candidate bytes. The substitution score comes from a query profile
// in LDS: for each byte value b a bit-vector over query positions, bit 2j+1 set iff q[j] == b,
// so `(w >> 2j) & 2` is 2*match and one cell is
//     h = max(0, max3(diag + 2*match, up, left) - 1)
// which equals max(0, diag +/- 1, up - 1, left - 1) of metrics.cpp:34-37. Padding (ragged query
// tails, rows past a candidate's end) uses an all-zero profile row: such cells can never exceed
// an already-counted neighbour, so the running maximum is unchanged. No MFMA: SW is not a dense
// contraction; the bound is integer VALU issue.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "drm_device.h"

namespace drm {
namespace {

constexpr int kPadRow = 256; // profile row index for "matches nothing"

// One DP row update for the full register row H[0..LQ).
template <int LQ>
__device__ __forceinline__ void sw_row(int (&H)[LQ], const uint32_t (&bv)[LQ / 16], int &best)
{
    int diag = 0, left = 0;
#pragma unroll
    for (int j = 0; j < LQ; ++j) {
        const uint32_t m2 = (bv[j >> 4] >> (2 * (j & 15))) & 2u;
        const int up = H[j];
        int h = max(max((int)(diag + (int)m2), up), left);
        h = max(h - 1, 0);
        diag = up;
        H[j] = h;
        left = h;
        best = max(best, h);
    }
}

template <int LQ>
__device__ __forceinline__ void load_profile(const uint32_t *prof, int ch, uint32_t (&bv)[LQ / 16])
{
    constexpr int NW = LQ / 16;
    constexpr int NWP = (NW + 3) & ~3;
    const uint4 *p = reinterpret_cast<const uint4 *>(prof + (size_t)ch * NWP);
#pragma unroll
    for (int w = 0; w < NW; w += 4) {
        const uint4 v = p[w / 4];
        bv[w] = v.x;
        if (w + 1 < NW)
            bv[w + 1] = v.y;
        if (w + 2 < NW)
            bv[w + 2] = v.z;
        if (w + 3 < NW)
            bv[w + 3] = v.w;
    }
}

// Build the query profile: prof[b][w] bit (2*(j%16)+1) of word j/16 set iff q[j] == b, b < 256.
template <int LQ>
__device__ void build_profile(uint32_t *prof, const uint8_t *q, int qlen)
{
    constexpr int NW = LQ / 16;
    constexpr int NWP = (NW + 3) & ~3;
    for (int e = threadIdx.x; e < 257 * NWP; e += blockDim.x) {
        const int b = e / NWP, w = e % NWP;
        uint32_t bits = 0;
        if (b < 256 && w < NW) {
            for (int t = 0; t < 16; ++t) {
                const int j = w * 16 + t;
                if (j < qlen && q[j] == (uint8_t)b)
                    bits |= 2u << (2 * t);
            }
        }
        prof[e] = bits;
    }
}

// ------------------------------------------------------------------------ partial_sort replay
// libstdc++ std::partial_sort(first, middle, last, comp) with comp(a,b) = score[a] > score[b]
// (reranker.cpp:38-40) on packed elements e = (score << 16) | index: comp only looks at score.
__device__ __forceinline__ bool ps_comp(uint32_t a, uint32_t b) { return (a >> 16) > (b >> 16); }

__device__ void ps_adjust_heap(uint32_t *first, int hole, int len, uint32_t value)
{
    const int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (ps_comp(first[second], first[second - 1]))
            second--;
        first[hole] = first[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        first[hole] = first[second - 1];
        hole = second - 1;
    }
    int parent = (hole - 1) / 2;
    while (hole > top && ps_comp(first[parent], value)) {
        first[hole] = first[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    first[hole] = value;
}

__device__ void ps_partial_sort(uint32_t *e, int n, int k)
{
    if (k >= 2) { // __make_heap(first, middle)
        int parent = (k - 2) / 2;
        for (;;) {
            ps_adjust_heap(e, parent, k, e[parent]);
            if (parent == 0)
                break;
            parent--;
        }
    }
    for (int i = k; i < n; ++i) // rest of __heap_select
        if (ps_comp(e[i], e[0])) {
            const uint32_t v = e[i];
            e[i] = e[0];
            ps_adjust_heap(e, 0, k, v);
        }
    for (int last = k - 1; last > 0; --last) { // __sort_heap
        const uint32_t v = e[last];
        e[last] = e[0];
        ps_adjust_heap(e, 0, last, v);
    }
}

template <int LQ>
__global__ __launch_bounds__(128) void sw_rerank_kernel(RerankArgs a)
{
    constexpr int NW = LQ / 16;
    constexpr int NWP = (NW + 3) & ~3;
    __shared__ __align__(16) uint32_t prof[257 * NWP];
    __shared__ __align__(16) uint8_t qbuf[LQ];
    __shared__ uint64_t cand[kMaxCands];
    __shared__ uint32_t elem[kMaxCands];
    __shared__ int ncand_s;

    const int tid = threadIdx.x;
    for (int64_t q = blockIdx.x; q < a.nq; q += gridDim.x) {
        const int qlen = a.q_len[q];
        // --- candidate list (find_sequences static): dense keeps ids < n_ref in order; sparse
        //     expands sparse_id*stride to [pos-stride+1, pos+stride) with duplicates kept.
        if (tid == 0) {
            const int nsel = min(a.k_clusters, a.kk);
            const int64_t *nb = a.neighbors + q * a.kk;
            int nc = 0;
            bool overflow = false;
            for (int i = 0; i < nsel && !overflow; ++i) {
                const uint64_t id = (uint64_t)nb[i];
                if (a.stride == 1) {
                    if (id < (uint64_t)a.n_ref) {
                        if (nc >= kMaxCands)
                            overflow = true;
                        else
                            cand[nc++] = id;
                    }
                } else {
                    const uint64_t s = (uint64_t)a.stride;
                    const uint64_t actual = id * s;
                    if (actual >= (uint64_t)a.n_ref)
                        continue;
                    const uint64_t start = (actual >= s - 1) ? actual - s + 1 : 0;
                    const uint64_t end = min(actual + s, (uint64_t)a.n_ref);
                    for (uint64_t pos = start; pos < end; ++pos) {
                        if (nc >= kMaxCands) {
                            overflow = true;
                            break;
                        }
                        cand[nc++] = pos;
                    }
                }
            }
            ncand_s = overflow ? -1 : nc;
        }
        for (int t = tid; t < LQ; t += blockDim.x)
            qbuf[t] = (t < qlen) ? a.queries[q * a.q_stride + t] : 0;
        __syncthreads();
        build_profile<LQ>(prof, qbuf, qlen);
        __syncthreads();
        const int ncand = (qlen > LQ) ? -3 : ncand_s; // -3: query longer than this build's LQ

        if (ncand > 0) {
            // --- SW scores, one lane per candidate
            for (int c = tid; c < ncand; c += blockDim.x) {
                int H[LQ];
#pragma unroll
                for (int j = 0; j < LQ; ++j)
                    H[j] = 0;
                int best = 0;
                const uint8_t *win = a.refs + (size_t)cand[c] * (size_t)a.row_stride;
                const uint32_t *w32 = reinterpret_cast<const uint32_t *>(win); // rows are 16-B aligned
                const int L = a.ref_len;
                uint32_t nxt = (L > 0) ? w32[0] : 0u;
                for (int i0 = 0; i0 < L; i0 += 4) {
                    const uint32_t cur = nxt;
                    if (i0 + 4 < L)
                        nxt = w32[(i0 >> 2) + 1]; // prefetch the next 4 candidate bytes
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const int ch = (i0 + t < L) ? (int)((cur >> (8 * t)) & 255u) : kPadRow;
                        uint32_t bv[NW];
                        load_profile<LQ>(prof, ch, bv);
                        sw_row<LQ>(H, bv, best);
                    }
                }
                elem[c] = ((uint32_t)best << 16) | (uint32_t)c;
            }
        }
        __syncthreads();
        // --- sw_reranker ordering + outputs
        if (tid == 0) {
            int status;
            if (ncand < 0)
                status = ncand == -3 ? -3 : -2; // -2: > kMaxCands candidates, -3: query > LQ bytes
            else if (ncand == 0 || a.k == 0)
                status = 0; // reranker.cpp:10-11: empty result for this query
            else if (ncand < a.k)
                status = -1; // reranker.cpp:26-29
            else {
                ps_partial_sort(elem, ncand, a.k);
                status = a.k;
            }
            a.status[q] = status;
        }
        __syncthreads();
        const int st = a.status[q];
        for (int j = tid; j < a.k; j += blockDim.x) {
            if (st > 0) {
                const uint32_t e = elem[j];
                a.top_scores[q * a.k + j] = (int32_t)(e >> 16);
                a.top_ids[q * a.k + j] = cand[e & 0xFFFFu];
            } else {
                a.top_scores[q * a.k + j] = -1;
                a.top_ids[q * a.k + j] = ~0ull;
            }
        }
        __syncthreads();
    }
}

// Generic batched calc_sw_score: one 64-lane wave per pair builds the profile of seq2 and
// lane 0 runs the DP over seq1 (correctness path for the drm_sw_scores API).
template <int LQ>
__global__ __launch_bounds__(64) void sw_pairs_kernel(const uint8_t *s1, const int64_t *off1, const int32_t *len1,
                                                      const uint8_t *s2, const int64_t *off2, const int32_t *len2,
                                                      int64_t npairs, int32_t *scores)
{
    constexpr int NW = LQ / 16;
    constexpr int NWP = (NW + 3) & ~3;
    __shared__ __align__(16) uint32_t prof[257 * NWP];
    __shared__ __align__(16) uint8_t qbuf[LQ];
    for (int64_t p = blockIdx.x; p < npairs; p += gridDim.x) {
        const int l2 = len2[p];
        for (int t = threadIdx.x; t < LQ; t += blockDim.x)
            qbuf[t] = (t < l2) ? s2[off2[p] + t] : 0;
        __syncthreads();
        build_profile<LQ>(prof, qbuf, l2);
        __syncthreads();
        if (threadIdx.x == 0) {
            int H[LQ];
#pragma unroll
            for (int j = 0; j < LQ; ++j)
                H[j] = 0;
            int best = 0;
            const int l1 = len1[p];
            const uint8_t *a = s1 + off1[p];
            for (int i = 0; i < l1; ++i) {
                uint32_t bv[NW];
                load_profile<LQ>(prof, a[i], bv);
                sw_row<LQ>(H, bv, best);
            }
            scores[p] = (l1 > 0 && l2 > 0) ? best : 0;
        }
        __syncthreads();
    }
}

} // namespace

static int pick_lq(int max_qlen)
{
    if (max_qlen <= 64)
        return 64;
    if (max_qlen <= 160)
        return 160;
    if (max_qlen <= 256)
        return 256;
    throw Error(DRM_ERR_UNSUPPORTED,
                "query length " + std::to_string(max_qlen) + " > 256 is not supported by the GPU SW kernel yet");
}

void launch_sw_rerank(const DeviceRefs &refs, const RerankArgs &a, int max_qlen, hipStream_t stream)
{
    if (a.nq <= 0)
        return;
    if (a.k > kMaxCands)
        throw Error(DRM_ERR_UNSUPPORTED, "k > 1024 not supported by the GPU rerank kernel");
    if (refs.row_stride % 16 != 0)
        throw Error(DRM_ERR_ARG, "window table row stride must be a multiple of 16");
    const int grid = (int)std::min<int64_t>(a.nq, 65536);
    switch (pick_lq(max_qlen)) {
    case 64:
        hipLaunchKernelGGL(sw_rerank_kernel<64>, dim3(grid), dim3(128), 0, stream, a);
        break;
    case 160:
        hipLaunchKernelGGL(sw_rerank_kernel<160>, dim3(grid), dim3(128), 0, stream, a);
        break;
    default:
        hipLaunchKernelGGL(sw_rerank_kernel<256>, dim3(grid), dim3(128), 0, stream, a);
        break;
    }
    DRM_HIP_CHECK(hipGetLastError());
}

void launch_sw_pairs(const uint8_t *d_s1, const int64_t *d_off1, const int32_t *d_len1, const uint8_t *d_s2,
                     const int64_t *d_off2, const int32_t *d_len2, int64_t npairs, int32_t *d_scores, int max_len2,
                     hipStream_t stream)
{
    if (npairs <= 0)
        return;
    const int grid = (int)std::min<int64_t>(npairs, 65536);
    switch (pick_lq(max_len2)) {
    case 64:
        hipLaunchKernelGGL(sw_pairs_kernel<64>, dim3(grid), dim3(64), 0, stream, d_s1, d_off1, d_len1, d_s2, d_off2,
                           d_len2, npairs, d_scores);
        break;
    case 160:
        hipLaunchKernelGGL(sw_pairs_kernel<160>, dim3(grid), dim3(64), 0, stream, d_s1, d_off1, d_len1, d_s2,
                           d_off2, d_len2, npairs, d_scores);
        break;
    default:
        hipLaunchKernelGGL(sw_pairs_kernel<256>, dim3(grid), dim3(64), 0, stream, d_s1, d_off1, d_len1, d_s2,
                           d_off2, d_len2, npairs, d_scores);
        break;
    }
    DRM_HIP_CHECK(hipGetLastError());
}

} // namespace drm
