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
#include <cstdlib>

#include "drm_device.h"

namespace drm {
namespace {

constexpr int kPadRow = 256; // profile row index for "matches nothing"
constexpr uint32_t kNoWindow = 0xFFFFFFFFu; // dynamic lookup: an id whose window lies outside the genome

// comp_table of the reference (src/utils/parse_inputs.cpp:5-14): A<->T, C<->G, N->N, anything else 0
__device__ __forceinline__ int comp_byte(int c)
{
    return c == 'A' ? 'T' : c == 'T' ? 'A' : c == 'C' ? 'G' : c == 'G' ? 'C' : c == 'N' ? 'N' : 0;
}

// Bytes of one candidate window: the static table row, or (dynamic lookup, find_sequence
// src/utils/post_processor.cpp:47-64) genome[w / 2 ..+ ref_len), reverse-complemented for odd w;
// a window past the genome end is the empty string (every row reads as the pad byte -1).
struct CandRow {
    const uint8_t *p;
    int rc;
    __device__ __forceinline__ CandRow(const RerankArgs &a, uint64_t w)
    {
        if (a.genome) {
            const uint64_t pos = w >> 1;
            const bool ok = w != (uint64_t)kNoWindow && pos + (uint64_t)a.ref_len <= (uint64_t)a.glen;
            rc = (int)(w & 1u);
            p = ok ? a.genome + pos + (rc ? a.ref_len - 1 : 0) : nullptr;
        } else {
            p = a.refs + w * (uint64_t)a.row_stride;
            rc = 0;
        }
    }
    __device__ __forceinline__ int at(int i) const
    {
        if (!p)
            return -1;
        return rc ? comp_byte(p[-i]) : (int)p[i];
    }
};

// find_sequences' candidate list of query q into cand[] (one thread); returns the count, -2 past
// kMaxCands. Static (:204-336): dense ids >= n_ref are dropped; sparse expansions are clipped to n_ref.
// Dynamic (:72-201): dense keeps every id (out-of-genome windows are empty); the sparse expansion is
// checked against the genome length. Duplicates are kept (the mapping restores the original count).
template <typename T>
__device__ int find_candidates(const RerankArgs &a, const int64_t *nb, int nsel, T *cand, int cap = kMaxCands)
{
    const uint64_t limit = a.genome ? (uint64_t)a.glen : (uint64_t)a.n_ref;
    int nc = 0;
    for (int i = 0; i < nsel; ++i) {
        const uint64_t id = (uint64_t)nb[i];
        if (a.stride == 1) {
            if (a.genome || id < limit) {
                if (nc >= cap)
                    return -2;
                cand[nc++] = a.genome ? (T)(id < (uint64_t)kNoWindow ? id : kNoWindow) : (T)id;
            }
            continue;
        }
        const uint64_t s = (uint64_t)a.stride;
        const uint64_t actual = id * s;
        if (actual >= limit)
            continue;
        const uint64_t start = (actual >= s - 1) ? actual - s + 1 : 0;
        const uint64_t end = min(actual + s, limit);
        for (uint64_t pos = start; pos < end; ++pos) {
            if (nc >= cap)
                return -2;
            cand[nc++] = (T)pos;
        }
    }
    return nc;
}

// One DP row update for the full register row H[0..LQ).
template <int LQ>
__device__ __forceinline__ void sw_row(int (&H)[LQ], const uint32_t (&bv)[(LQ + 15) / 16], int &best)
{
    // The next cell's diagonal term (old H[j] + 2*match) is formed before H[j] is overwritten, so the
    // old and new H[j] never overlap and stay in one register (no per-cell v_mov).
    int t_next = (int)__builtin_amdgcn_ubfe(bv[0], 0u, 2u); // diag of column 0 is the zero border
    int left = 0;
#pragma unroll
    for (int j = 0; j < LQ; ++j) {
        const int t = t_next;
        const int up = H[j];
        if (j + 1 < LQ)
            t_next = up + (int)__builtin_amdgcn_ubfe(bv[(j + 1) >> 4], 2u * ((j + 1) & 15), 2u); // bit 2t is 0
        int h = max(max(t, up), left);
        h = max(h - 1, 0);
        H[j] = h;
        left = h;
        best = max(best, h);
    }
}

typedef unsigned short us2 __attribute__((ext_vector_type(2)));

// Two candidates per lane in 16-bit halves (lo = candidate a, hi = candidate b). pw[g] carries the
// match bits of query positions 8g..8g+7 for both candidates (bit 2t+1 of each half), so one 32-bit
// shift + mask yields 2*match for both; scores <= 256 never carry across halves.
template <int LQ>
__device__ __forceinline__ void sw_row_pk(uint32_t (&H)[LQ], const uint32_t (&pw)[(LQ + 7) / 8], us2 &best)
{
    uint32_t t_next = pw[0] & 0x00020002u; // diag of column 0 is the zero border
    us2 left = {0, 0};
#pragma unroll
    for (int j = 0; j < LQ; ++j) {
        const uint32_t t = t_next;
        const uint32_t up = H[j];
        if (j + 1 < LQ)
            t_next = up + ((pw[(j + 1) >> 3] >> (2 * ((j + 1) & 7))) & 0x00020002u);
        us2 h = __builtin_elementwise_max(__builtin_elementwise_max(__builtin_bit_cast(us2, t),
                                                                    __builtin_bit_cast(us2, up)),
                                          left);
        h = __builtin_elementwise_sub_sat(h, (us2){1, 1});
        H[j] = __builtin_bit_cast(uint32_t, h);
        left = h;
        best = __builtin_elementwise_max(best, h);
    }
}

// Interleave the profile rows of two candidate bytes into pw (see sw_row_pk).
template <int LQ>
__device__ __forceinline__ void load_profile_pk(const uint32_t *prof, int ca, int cb, uint32_t (&pw)[(LQ + 7) / 8])
{
    constexpr int NW = (LQ + 15) / 16;
    constexpr int NWP = (NW + 3) & ~3;
    constexpr int NG = (LQ + 7) / 8;
    const uint4 *pa = reinterpret_cast<const uint4 *>(prof + (size_t)ca * NWP);
    const uint4 *pb = reinterpret_cast<const uint4 *>(prof + (size_t)cb * NWP);
#pragma unroll
    for (int w4 = 0; w4 < NWP / 4; ++w4) {
        const uint4 va = pa[w4], vb = pb[w4];
        const uint32_t wa[4] = {va.x, va.y, va.z, va.w};
        const uint32_t wb[4] = {vb.x, vb.y, vb.z, vb.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int w = w4 * 4 + e;
            if (2 * w < NG)
                pw[2 * w] = __builtin_amdgcn_perm(wb[e], wa[e], 0x05040100u);
            if (2 * w + 1 < NG)
                pw[2 * w + 1] = __builtin_amdgcn_perm(wb[e], wa[e], 0x07060302u);
        }
    }
}

template <int LQ>
__device__ __forceinline__ void load_profile(const uint32_t *prof, int ch, uint32_t (&bv)[(LQ + 15) / 16])
{
    constexpr int NW = (LQ + 15) / 16;
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
    constexpr int NW = (LQ + 15) / 16;
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
// (reranker.cpp:38-40) on packed elements e = (score << S) | index: comp only looks at score. T = uint32_t, S = 16 in
// general; T = uint16_t, S = 8 when every score and candidate index fits a byte (half the LDS per query).
template <typename T, int S>
__device__ __forceinline__ bool ps_comp(T a, T b) { return (a >> S) > (b >> S); }

template <typename T, int S>
__device__ void ps_adjust_heap(T *first, int hole, int len, T value)
{
    const int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (ps_comp<T, S>(first[second], first[second - 1]))
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
    while (hole > top && ps_comp<T, S>(first[parent], value)) {
        first[hole] = first[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    first[hole] = value;
}

template <typename T, int S>
__device__ void ps_partial_sort(T *e, int n, int k)
{
    if (k >= 2) { // __make_heap(first, middle)
        int parent = (k - 2) / 2;
        for (;;) {
            ps_adjust_heap<T, S>(e, parent, k, e[parent]);
            if (parent == 0)
                break;
            parent--;
        }
    }
    for (int i = k; i < n; ++i) // rest of __heap_select
        if (ps_comp<T, S>(e[i], e[0])) {
            const T v = e[i];
            e[i] = e[0];
            ps_adjust_heap<T, S>(e, 0, k, v);
        }
    for (int last = k - 1; last > 0; --last) { // __sort_heap
        const T v = e[last];
        e[last] = e[0];
        ps_adjust_heap<T, S>(e, 0, last, v);
    }
}

// Kernel 1 of the rerank: candidate lists (find_sequences static) + one SW score per candidate.
// One 64-lane workgroup per query (grid-stride); each lane scores two candidates (16-bit halves).
template <int LQ, bool ONLY_FLAGGED = false>
__global__ __launch_bounds__(64) void sw_score_kernel(RerankArgs a)
{
    constexpr int NW = (LQ + 15) / 16;
    constexpr int NWP = (NW + 3) & ~3;
    __shared__ __align__(16) uint32_t prof[257 * NWP];
    __shared__ __align__(16) uint8_t qbuf[LQ];
    __shared__ uint64_t cand[kMaxCands];
    __shared__ int ncand_s;

    const int tid = threadIdx.x; // one wave per workgroup
    const int lane = tid & 63;
    for (int64_t q = blockIdx.x; q < a.nq; q += gridDim.x) {
        if (ONLY_FLAGGED && a.ncand[q] != -4)
            continue; // scored by sw_score_f16_kernel
        const int qlen = a.q_len[q];
        const int nsel = min(a.k_clusters, a.kk);
        const int64_t *nb = a.neighbors + q * a.kk;
        if (a.stride == 1 && nsel <= kMaxCands && !a.genome) {
            // dense (post_processor.cpp:215-236): keep ids < n_ref, in order -- ballot compaction
            int base = 0;
            for (int c = 0; c < nsel; c += 64) {
                const int i = c + lane;
                const uint64_t id = (i < nsel) ? (uint64_t)nb[i] : ~0ull;
                const bool keep = id < (uint64_t)a.n_ref;
                const uint64_t m = __ballot(keep);
                if (keep)
                    cand[base + __popcll(m & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))))] = id;
                base += __popcll(m);
            }
            if (tid == 0)
                ncand_s = base;
        } else if (tid == 0) {
            ncand_s = find_candidates(a, nb, nsel, cand);
        }
        for (int t = tid; t < LQ; t += blockDim.x)
            qbuf[t] = (t < qlen) ? a.queries[q * a.q_stride + t] : 0;
        __syncthreads();
        build_profile<LQ>(prof, qbuf, qlen);
        __syncthreads();
        const int ncand = (qlen > LQ) ? -3 : ncand_s;
        if (tid == 0)
            a.ncand[q] = ncand;
        // two candidates per lane: c and c + blockDim.x
        for (int c0 = tid; c0 < ncand; c0 += 2 * blockDim.x) {
            const int c1 = c0 + (int)blockDim.x;
            const bool has_b = c1 < ncand;
            uint32_t H[LQ];
#pragma unroll
            for (int j = 0; j < LQ; ++j)
                H[j] = 0u;
            us2 best = {0, 0};
            const uint64_t wa = cand[c0], wb = has_b ? cand[c1] : cand[c0];
            const CandRow ra(a, wa), rb(a, wb);
            const int L = a.ref_len;
            auto code = [](int c) { return c < 0 ? kPadRow : c; };
            int na = (L > 0) ? code(ra.at(0)) : kPadRow;
            int nb2 = (L > 0 && has_b) ? code(rb.at(0)) : kPadRow;
            for (int i = 0; i < L; ++i) {
                const int ca = na, cb = nb2;
                if (i + 1 < L) { // prefetch the next row's bytes
                    na = code(ra.at(i + 1));
                    nb2 = has_b ? code(rb.at(i + 1)) : kPadRow;
                }
                uint32_t pw[(LQ + 7) / 8];
                load_profile_pk<LQ>(prof, ca, cb, pw);
                sw_row_pk<LQ>(H, pw, best);
            }
            // dense dynamic lookup reports the search's own id (e.g. -1 as 2^64-1, post_processor.cpp:95-101)
            const bool dense_dyn = a.genome && a.stride == 1;
            a.cand_ids[q * a.cmax + c0] = dense_dyn ? (uint64_t)nb[c0] : wa;
            a.cand_scores[q * a.cmax + c0] = (int32_t)best.x;
            if (has_b) {
                a.cand_ids[q * a.cmax + c1] = dense_dyn ? (uint64_t)nb[c1] : wb;
                a.cand_scores[q * a.cmax + c1] = (int32_t)best.y;
            }
        }
        __syncthreads();
    }
}


// ------------------------------------------------------------------------ fp16 DP (fast path)
// Scores are carried as fp16 multiples of 2^-10 (exact: every value is an integer <= ~300, far
// below 1024), two candidates per lane in the halves of one register. One cell pair is
//     t = diag + term                         v_pk_add_f16   (term = 2^-9 on a match, else 0)
//     h = clamp01(max3(t, up, left) - 2^-10)  v_pk_maximum3_f16, v_pk_add_f16 ... clamp
// i.e. h = max(0, max3(diag + 2*match, up, left) - 1) scaled by 2^-10 (metrics.cpp:34-37); the
// f16 clamp modifier (to [0, 1]) is the max with 0, and the running best takes two columns per
// v_pk_maximum3_f16 -- 3.5 VALU per cell pair.
//
// The match terms come ready-paired from LDS: for candidate-byte codes a, b in 0..4 (A, C, G, T,
// 4 = "a byte the query does not contain") `pprof` row (a, b) (at a * GST + b * PST words, a layout
// whose 16 A/C/G/T rows fall on distinct bank quads of every ds_read_b128 lane group) holds the words
// (q[j]==a ? 0x1800 : 0) | (q[j]==b ? 0x18000000 : 0) (0x1800 = 2^-9 in fp16). A candidate byte that
// is not A/C/G/T but does occur in the query (e.g. N against N) cannot be coded; the query is then
// flagged (ncand = kNeedBitProfile) and the bit-profile kernel re-scores it exactly.
constexpr int kNeedBitProfile = -4;

typedef _Float16 h2 __attribute__((ext_vector_type(2)));

#ifndef DRM_SW_ROWS
#define DRM_SW_ROWS 2 // DP rows in flight per pass over the columns (sw_rows_i16); 2 measured fastest of 2-5
#endif
#ifndef DRM_SW_PF
#define DRM_SW_PF 1 // profile groups (4 columns each) read ahead of the one in use, per row (1-4 measured: 1 best by <1 %)
#endif

// ---- integer cells. A score s (0 <= s <= 1023) is the 16-bit pattern s, i.e. the fp16 subnormal s * 2^-24: fp16
// ordering of non-negative patterns below 0x7C00 is the integer ordering (subnormals included: fp16 denormals are
// kept, the default FP mode), so v_pk_maximum3_f16 is an exact integer max3. The diagonal term (+2 on a match) is
// added by v_add_u32 across both halves: the low half stays below 2^16 (s <= 1023 + 2), so no carry crosses. One
// cell pair costs a 32-bit add (2 cycles per wave64 instruction on gfx950), a packed max3 and a packed saturating
// subtract (4 each), and half a packed max3 for the best: 12 issue cycles (profiles/r02/valu_rate_probe.txt).
__device__ __forceinline__ uint32_t imax3(uint32_t a, uint32_t b, uint32_t c)
{
    const h2 r = __builtin_elementwise_maximum(__builtin_elementwise_maximum(__builtin_bit_cast(h2, a), __builtin_bit_cast(h2, b)),
                                               __builtin_bit_cast(h2, c));
    return __builtin_bit_cast(uint32_t, r);
}
__device__ __forceinline__ uint32_t idec(uint32_t a) // max(0, s - 1) in both halves: v_pk_sub_u16 ... clamp
{
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(__builtin_bit_cast(u16x2, a), (u16x2){1, 1}));
}

// R DP rows in one pass over the LQ columns (rows = consecutive candidate bytes i .. i + R - 1): at step j row r
// computes column j - r, from the value the row above it wrote there one step earlier, so one wave issues from R
// independent left-to-right chains (max3 -> subtract -> the next column's max3) instead of one. The DP row lives
// in H (one register per column, two candidates per register) and is updated in place: a cell's next-column
// diagonal term is formed from H[c] before the cell overwrites it. The issue rate of this DP is set by the number
// of such chains a SIMD holds (one wave per SIMD ran at 46 % of two; the 150-register row
// leaves room for two waves only), so R is the lever. Per row, the profile words of PF groups of 4 columns are
// read ahead of the one in use (one ds_read_b128 each), and a group's slot is refilled once the last row is past
// it. The best takes one max3 per two cells. pp[r]: the pair-profile row of DP row i + r (match terms of the two
// candidates' bytes against every query column).
template <int LQ, int R, int PF>
__device__ __forceinline__ void sw_rows_i16(uint32_t (&H)[LQ], const uint32_t *const (&pp)[R], uint32_t &best)
{
    constexpr int NG = (LQ + 3) / 4, NS = PF + 1, LAG = R - 2;
    uint4 P[R][NS];
#pragma unroll
    for (int g = 0; g < NS; ++g)
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (g < NG)
                P[r][g] = *reinterpret_cast<const uint4 *>(pp[r] + 4 * g);
    auto word = [](const uint4 &v, int e) { return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w; };
    uint32_t td[R], left[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        td[r] = P[r][0].x; // column 0: the diagonal is the zero border
        left[r] = 0u;
    }
    uint32_t pend = 0u; // R odd: the last row's value of an even step, paired with the next step's
#pragma clang loop unroll(full)
    for (int j = 0; j < LQ + R - 1; ++j) {
        if (j - LAG >= 4 && ((j - LAG) & 3) == 0) { // group gd is done for every row: refill its slot
            const int gd = ((j - LAG) >> 2) - 1, gn = gd + NS;
            if (gn < NG) {
#pragma unroll
                for (int r = 0; r < R; ++r)
                    P[r][gd % NS] = *reinterpret_cast<const uint4 *>(pp[r] + 4 * gn);
            }
            __builtin_amdgcn_sched_barrier(0); // keep the reads here, ahead of the columns that consume them
        }
        uint32_t h[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int c = j - r;
            h[r] = 0u;
            if (c >= 0 && c < LQ) {
                const uint32_t up = H[c];
                uint32_t tn = 0u;
                if (c + 1 < LQ)
                    tn = up + word(P[r][((c + 1) >> 2) % NS], (c + 1) & 3);
                const uint32_t v = idec(imax3(td[r], up, left[r]));
                H[c] = v;
                left[r] = v;
                td[r] = tn;
                h[r] = v;
            }
        }
#pragma unroll
        for (int r = 0; r + 1 < R; r += 2)
            best = imax3(best, h[r], h[r + 1]);
        if (R & 1) {
            if (j & 1)
                best = imax3(best, pend, h[R - 1]);
            else
                pend = h[R - 1];
        }
    }
    if (R & 1)
        best = imax3(best, pend, pend);
}

__device__ __forceinline__ int acgt_code(int c) // A,C,G,T -> 0..3, anything else -> -1
{
    const int k = (c >> 1) & 3; // A=0x41 -> 0, C=0x43 -> 1, T=0x54 -> 2, G=0x47 -> 3
    return (((0x47544341u >> (8 * k)) & 0xFFu) == (uint32_t)c) ? k : -1;
}
__device__ __forceinline__ int acgt_byte(int k) { return k < 4 ? (int)((0x47544341u >> (8 * k)) & 0xFFu) : -1; }
// pair-profile row of candidate codes (ka, kb) (sw_score_f16_kernel): the A/C/G/T pairs first, 4 ka + kb
__device__ __forceinline__ int pair_row(int ka, int kb)
{
    return ka < 4 ? (kb < 4 ? 4 * ka + kb : 16 + ka) : (kb < 4 ? 20 + kb : 24);
}

// Kernel 1 (fast path) of the rerank: candidate lists (find_sequences static) + one SW score per
// candidate; same contract as sw_score_kernel. One 64-lane workgroup per query (grid-stride).
template <int LQ>
__global__ __launch_bounds__(64) void sw_score_f16_kernel(RerankArgs a)
{
    // Pair-profile layout: the row of candidate codes (ka, kb) (0..3 = A, C, T, G; 4 = none) is row
    // p = pair_row(ka, kb) at p * PST words: the 16 A/C/G/T pairs are p = 4 ka + kb = 0..15, the pairs with a
    // 'none' code follow (16 + ka, 20 + kb, 24). A ds_read_b128 lane group (16 lanes) is conflict-free when the
    // 16-byte chunk index (address / 16) mod 16 differs between distinct rows: with PST / 4 odd, p * PST / 4 mod 16
    // is distinct for p = 0..15 (MI355X_MICROARCH.md, LDS banking). And p = 4 ka + kb of four rows at once is two
    // byte-wise (SWAR) operations on the candidates' code words (the fast path below).
    constexpr int PST = ((LQ + 3) & ~3) + 4 + (((((LQ + 3) & ~3) + 4) / 4) % 2 == 0 ? 4 : 0);
    static_assert((PST / 4) % 2 == 1, "pair-profile bank spread");
    constexpr int PPROF = 25 * PST;
    __shared__ __align__(16) uint32_t pprof[PPROF];
    // the query as given (up to LQ + 2 bytes: the tags of a 150 bp read around LQ = 150 DP columns)
    constexpr int QB = (LQ + 2 + 15) & ~15;
    __shared__ __align__(16) uint8_t qbuf[QB];
    __shared__ int lead_s, qe_s;
    __shared__ uint32_t qmask[8]; // bytes present in the query
    extern __shared__ uint32_t cand[]; // [a.cmax]
    __shared__ int ncand_s, flag_s;

    const int tid = threadIdx.x; // one wave per workgroup
    const int lane = tid & 63;
    for (int64_t q = blockIdx.x; q < a.nq; q += gridDim.x) {
        const int qlen = a.q_len[q];
        const int nsel = min(a.k_clusters, a.kk);
        const int64_t *nb = a.neighbors + q * a.kk;
        if (a.stride == 1 && nsel <= kMaxCands && !a.genome) {
            // dense (post_processor.cpp:215-236): keep ids < n_ref, in order -- ballot compaction
            int base = 0;
            for (int c = 0; c < nsel; c += 64) {
                const int i = c + lane;
                const uint64_t id = (i < nsel) ? (uint64_t)nb[i] : ~0ull;
                const bool keep = id < (uint64_t)a.n_ref;
                const uint64_t m = __ballot(keep);
                if (keep)
                    cand[base + __popcll(m & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))))] = (uint32_t)id;
                base += __popcll(m);
            }
            if (tid == 0)
                ncand_s = base;
        } else if (tid == 0) {
            // sparse (:238-335) or dynamic lookup: expand, duplicates kept (:502-507)
            ncand_s = find_candidates(a, nb, nsel, cand, a.cmax);
        }
        for (int t = tid; t < QB; t += 64)
            qbuf[t] = (t < qlen && t < QB) ? a.queries[q * a.q_stride + t] : 0;
        if (tid < 8)
            qmask[tid] = 0u;
        if (tid == 0)
            flag_s = 0;
        __syncthreads();
        for (int t = tid; t < qlen && t < QB; t += 64)
            atomicOr(&qmask[qbuf[t] >> 5], 1u << (qbuf[t] & 31));
        // Leading and trailing query bytes that are not A/C/G/T (the "<" / ">" tags) are dropped from the DP: on
        // this path no candidate byte matches them (a candidate byte equal to a non-ACGT query byte flags the query
        // for the bit-profile kernel), so a leading such column holds 0 in every row -- the zero border the next
        // column sees anyway -- and a trailing one never exceeds the best of the columns to its left (each of its
        // cells is a neighbour minus 1, or 0). The DP over the remaining qe columns gives the same score.
        if (tid == 0) {
            const int n = qlen < QB ? qlen : QB;
            int lo = 0, hi = n;
            while (lo < hi && acgt_code(qbuf[lo]) < 0)
                ++lo;
            while (hi > lo && acgt_code(qbuf[hi - 1]) < 0)
                --hi;
            lead_s = lo;
            qe_s = hi - lo;
        }
        __syncthreads();
        const int lead = lead_s, qe = qe_s;
        // one column per lane: its query byte is tested once against A, C, G, T and written to the 25 rows
        for (int j = tid; j < PST; j += 64) {
            const int c = (j < qe && j < LQ) ? (int)qbuf[lead + j] : -1; // past the query: matches nothing
            // the diagonal term: +2 on a match (the -1 every cell takes makes it +1); code 4 matches nothing
            uint32_t m[5];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                m[k] = c == acgt_byte(k) ? 0x0002u : 0u;
            m[4] = 0u;
#pragma unroll
            for (int ka = 0; ka < 5; ++ka)
#pragma unroll
                for (int kb = 0; kb < 5; ++kb)
                    pprof[pair_row(ka, kb) * PST + j] = m[ka] | (m[kb] << 16);
        }
        __syncthreads();
        // longer than the buffer: unsupported here (-3); more than LQ columns left after the tags: the bit-profile
        // kernel scores the query (flagged)
        const int ncand = (qlen > QB) ? -3 : ncand_s;
        bool flagged = qe > LQ;
        // two candidates per lane: c and c + 64
        for (int c0 = tid; c0 < (qe > LQ ? 0 : ncand); c0 += 128) {
            const int c1 = c0 + 64;
            const bool has_b = c1 < ncand;
            uint32_t H[LQ];
#pragma unroll
            for (int j = 0; j < LQ; ++j)
                H[j] = 0u;
            uint32_t best = 0u;
            const uint32_t wa = cand[c0], wb = has_b ? cand[c1] : cand[c0];
            // the candidate rows arrive 16 bytes per lane per 16 DP rows (one aligned load each, the next
            // block in flight while the current one is consumed), not one byte load per row
            // the candidate rows arrive 16 bytes per lane per 16 DP rows (one aligned load each, the next
            // block in flight while the current one is consumed), not one byte load per row; dynamic lookup reads
            // unaligned genome windows one byte per row (genome bytes are ACGTN)
            const CandRow ra(a, wa), rb(a, wb);
            const uint4 *pa = reinterpret_cast<const uint4 *>(a.refs + (size_t)wa * (size_t)a.row_stride);
            const uint4 *pb = reinterpret_cast<const uint4 *>(a.refs + (size_t)wb * (size_t)a.row_stride);
            const int L = a.ref_len;
            const int nblk = (int)(a.row_stride >> 4); // row_stride is a multiple of 16, >= ref_len
            uint4 ba = make_uint4(0u, 0u, 0u, 0u), bb = ba, na4 = ba, nb4 = ba;
            if (L > 0 && !a.genome) {
                na4 = pa[0];
                nb4 = pb[0];
            }
            // profile row of candidate bytes (ca, cb) (-1: past the window / no second candidate): a byte that is not
            // A/C/G/T takes the 'none' code 4, unless the query holds it (e.g. N against N): the query is then flagged
            // for the bit-profile kernel
            auto prow = [&](int ca, int cb) -> const uint32_t * {
                int ka = acgt_code(ca), kb = acgt_code(cb);
                if (ka < 0) {
                    flagged |= ca >= 0 && ((qmask[ca >> 5] >> (ca & 31)) & 1u) != 0u;
                    ka = 4;
                }
                if (kb < 0) {
                    flagged |= cb >= 0 && ((qmask[cb >> 5] >> (cb & 31)) & 1u) != 0u;
                    kb = 4;
                }
                return pprof + pair_row(ka, kb) * PST;
            };
            if (a.genome) {
                // dynamic lookup: window bytes one at a time (reverse-complemented for odd ids)
                int i = 0;
                for (; i + DRM_SW_ROWS <= L; i += DRM_SW_ROWS) {
                    const uint32_t *pr[DRM_SW_ROWS];
#pragma unroll
                    for (int r = 0; r < DRM_SW_ROWS; ++r)
                        pr[r] = prow(ra.at(i + r), has_b ? rb.at(i + r) : -1);
                    sw_rows_i16<LQ, DRM_SW_ROWS, DRM_SW_PF>(H, pr, best);
                }
                for (; i < L; ++i) {
                    const uint32_t *pr[1] = {prow(ra.at(i), has_b ? rb.at(i) : -1)};
                    sw_rows_i16<LQ, 1, DRM_SW_PF>(H, pr, best);
                }
            } else {
                // static table: each 4-byte word of a candidate's 16-byte block holds 4 DP rows. Fast path: when every
                // byte of the word is A/C/G/T in every lane, the codes of its 4 rows come from two byte-wise operations
                // (k = (c >> 1) & 3, checked against the A/C/T/G table by one v_perm) and their profile rows are
                // p = 4 ka + kb, one byte each of p4 -- a bit-field extract and a multiply-add per row instead of the
                // per-row code tests
                uint32_t wa4 = 0u, wb4 = 0u, p4 = 0u;
                bool fast = false;
                auto row = [&](int i) -> const uint32_t * {
                    if ((i & 3) == 0) { // wave-uniform: the next word of each block (register moves, no indexing)
                        if ((i & 15) == 0) { // the next block becomes current, prefetch the one after
                            ba = na4;
                            bb = nb4;
                            const int nx = (i >> 4) + 1;
                            if (nx < nblk && 16 * nx < L) {
                                na4 = pa[nx];
                                nb4 = pb[nx];
                            }
                        }
                        wa4 = ba.x;
                        wb4 = has_b ? bb.x : 0u;
                        ba = make_uint4(ba.y, ba.z, ba.w, 0u);
                        bb = make_uint4(bb.y, bb.z, bb.w, 0u);
                        const uint32_t ka4 = (wa4 >> 1) & 0x03030303u, kb4 = (wb4 >> 1) & 0x03030303u;
                        const uint32_t bad = (__builtin_amdgcn_perm(0u, 0x47544341u, ka4) ^ wa4) |
                                             (has_b ? (__builtin_amdgcn_perm(0u, 0x47544341u, kb4) ^ wb4) : 0u);
                        fast = i + 4 <= L && __ballot(bad != 0u) == 0ull;
                        p4 = has_b ? (ka4 << 2) + kb4 : ka4 + 0x10101010u; // (ka, 'none'): 16 + ka
                    }
                    const uint32_t sh = 8u * (uint32_t)(i & 3);
                    if (fast)
                        return pprof + __builtin_amdgcn_ubfe(p4, sh, 8u) * PST;
                    return prow((int)((wa4 >> sh) & 255u), has_b ? (int)((wb4 >> sh) & 255u) : -1);
                };
                int i = 0;
                for (; i + DRM_SW_ROWS <= L; i += DRM_SW_ROWS) {
                    const uint32_t *pr[DRM_SW_ROWS];
#pragma unroll
                    for (int r = 0; r < DRM_SW_ROWS; ++r)
                        pr[r] = row(i + r); // in row order: row() steps through the candidate bytes
                    sw_rows_i16<LQ, DRM_SW_ROWS, DRM_SW_PF>(H, pr, best);
                }
                for (; i < L; ++i) {
                    const uint32_t *pr[1] = {row(i)};
                    sw_rows_i16<LQ, 1, DRM_SW_PF>(H, pr, best);
                }
            }
            const int score_a = (int)(best & 0xFFFFu), score_b = (int)(best >> 16);
            const bool dense_dyn = a.genome && a.stride == 1; // the search's own id (post_processor.cpp:95-101)
            a.cand_ids[q * a.cmax + c0] = dense_dyn ? (uint64_t)nb[c0] : wa;
            a.cand_scores[q * a.cmax + c0] = score_a;
            if (has_b) {
                a.cand_ids[q * a.cmax + c1] = dense_dyn ? (uint64_t)nb[c1] : wb;
                a.cand_scores[q * a.cmax + c1] = score_b;
            }
        }
        if (__ballot(flagged) != 0ull && lane == 0)
            flag_s = 1;
        __syncthreads();
        if (tid == 0)
            a.ncand[q] = (ncand >= 0 && flag_s) ? kNeedBitProfile : ncand;
        __syncthreads();
    }
}

// ------------------------------------------------------------------------ banded DP (opt-in, non-parity)
// The reference leaves banding as a TODO (includes/utils/reranker.hpp:12) and scores the full DP, so this is an
// opt-in mode of this implementation (drm_refs_set_sw_band), never the default: the recurrence of metrics.cpp:30-41
// restricted to the cells |i - j| <= W (row i over the candidate, column j over the query, both 0-based), a cell
// outside the band being 0 (oracle_calc_sw_score_banded). The score is at most the full one and equal to it when the
// best local alignment lies inside the band.
//
// Layout: one wave per query, two candidates per lane (16-bit halves, integer cells as in sw_rows_i16). The band of
// row i is B = 2W + 1 registers, cell k holding column j = i - W + k, so a row's update is the full kernel's with
// static indices: diag = the old cell k, up = the old cell k + 1 (0 past the band), left = the new cell k - 1. The
// match terms come from a byte profile in LDS: per query byte code c (the query's distinct bytes, at most 7, plus an
// 'absent' code that matches nothing) one byte per query position (2 on a match), padded by W zero positions on the
// left, in 4 copies shifted by 0..3 bytes so that a row's band starts on a word boundary of copy i & 3. One v_perm
// per cell pair takes candidate a's byte into the low half and candidate b's into the high half: 4.5 VALU per cell
// pair. Positions left of the query (j < 0) are 0 in every row (the zero border); positions right of it match
// nothing, and such cells never exceed a cell to their left, so the running best is unchanged (the same argument as
// the padding of sw_score_kernel); rows past qlen + W - 1 hold only such cells and are skipped.
constexpr int kBandQMax = 256; // longest query the banded kernel takes (longer: status -3, unsupported)
constexpr int kBandCodes = 8;  // per query: up to 7 distinct query bytes + 'absent'

__host__ __device__ constexpr int band_words(int w) { return (2 * w + 1 + 3) / 4; }

template <int W>
__global__ __launch_bounds__(64) void sw_score_band_kernel(RerankArgs a, int rsw)
{
    constexpr int B = 2 * W + 1;
    constexpr int NWB = band_words(W);
    __shared__ __align__(16) uint8_t qbuf[kBandQMax];
    __shared__ uint8_t code_of[256];
    __shared__ uint32_t qmask[8];
    __shared__ int ncand_s;
    extern __shared__ __align__(16) uint32_t band_lds[];
    uint32_t *bprof = band_lds;                       // [4 copies][kBandCodes][rsw]
    uint32_t *cand = band_lds + 4 * kBandCodes * rsw; // [a.cmax]
    const int lane = threadIdx.x & 63;
    for (int64_t q = blockIdx.x; q < a.nq; q += gridDim.x) {
        const int qlen = a.q_len[q];
        const int nsel = min(a.k_clusters, a.kk);
        const int64_t *nb = a.neighbors + q * a.kk;
        if (a.stride == 1 && nsel <= kMaxCands && !a.genome) {
            // dense (post_processor.cpp:215-236): keep ids < n_ref, in order -- ballot compaction
            int base = 0;
            for (int c = 0; c < nsel; c += 64) {
                const int i = c + lane;
                const uint64_t id = (i < nsel) ? (uint64_t)nb[i] : ~0ull;
                const bool keep = id < (uint64_t)a.n_ref;
                const uint64_t m = __ballot(keep);
                if (keep)
                    cand[base + __popcll(m & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))))] = (uint32_t)id;
                base += __popcll(m);
            }
            if (lane == 0)
                ncand_s = base;
        } else if (lane == 0) {
            ncand_s = find_candidates(a, nb, nsel, cand, a.cmax); // sparse or dynamic lookup
        }
        for (int t = lane; t < kBandQMax; t += 64)
            qbuf[t] = t < qlen ? a.queries[q * a.q_stride + t] : 0;
        if (lane < 8)
            qmask[lane] = 0u;
        __syncthreads();
        for (int t = lane; t < qlen && t < kBandQMax; t += 64)
            atomicOr(&qmask[qbuf[t] >> 5], 1u << (qbuf[t] & 31));
        __syncthreads();
        // byte codes: the query's distinct bytes in ascending order take 0, 1, ...; every other byte is 'absent'
        int ndist = 0;
#pragma unroll
        for (int w = 0; w < 8; ++w)
            ndist += __popc(qmask[w]);
        for (int b = lane; b < 256; b += 64) {
            int rank = 0;
            for (int w = 0; w < (b >> 5); ++w)
                rank += __popc(qmask[w]);
            const uint32_t m = qmask[b >> 5];
            rank += __popc(m & ((1u << (b & 31)) - 1u));
            const bool in_q = ((m >> (b & 31)) & 1u) != 0u;
            code_of[b] = (uint8_t)(in_q && rank < kBandCodes - 1 ? rank : kBandCodes - 1);
        }
        __syncthreads();
        // the byte profile: copy s, word x holds positions 4x + s .. 4x + s + 3 (query column position - W)
        const int qn = min(qlen, kBandQMax); // a longer query is refused below; its profile is never read
        for (int it = lane; it < 4 * rsw; it += 64) {
            const int s = it / rsw, x = it - s * rsw;
            uint32_t cq = 0u; // the 4 positions' codes, 0xFF outside the query
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int j = 4 * x + e + s - W;
                const uint32_t c = (j >= 0 && j < qn) ? (uint32_t)code_of[qbuf[j]] : 0xFFu;
                cq |= c << (8 * e);
            }
#pragma unroll
            for (int c = 0; c < kBandCodes; ++c) {
                uint32_t w = 0u;
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    w |= ((cq >> (8 * e)) & 255u) == (uint32_t)c && c != kBandCodes - 1 ? 2u << (8 * e) : 0u;
                bprof[(s * kBandCodes + c) * rsw + x] = w;
            }
        }
        __syncthreads();
        const bool unsupported = qlen > kBandQMax || ndist > kBandCodes - 1;
        const int ncand = unsupported ? -3 : ncand_s;
        const int L = a.ref_len;
        const int rows = min(L, qlen + W); // later rows hold only cells right of the query
        for (int c0 = lane; c0 < ncand; c0 += 128) {
            const int c1 = c0 + 64;
            const bool has_b = c1 < ncand;
            uint32_t H[B];
#pragma unroll
            for (int k = 0; k < B; ++k)
                H[k] = 0u;
            uint32_t best = 0u;
            const uint32_t wa = cand[c0], wb = has_b ? cand[c1] : cand[c0];
            const CandRow ra(a, wa), rb(a, wb);
            // static table: 16 candidate bytes per load (rows i .. i + 15), the next block in flight; dynamic lookup:
            // one byte per row, one row ahead
            const uint4 *pa = reinterpret_cast<const uint4 *>(a.refs + (size_t)wa * (size_t)a.row_stride);
            const uint4 *pb = reinterpret_cast<const uint4 *>(a.refs + (size_t)wb * (size_t)a.row_stride);
            const int nblk = (int)(a.row_stride >> 4);
            uint4 ba = make_uint4(0u, 0u, 0u, 0u), bb = ba, na4 = ba, nb4 = ba;
            uint32_t wa4 = 0u, wb4 = 0u;
            int nca = -1, ncb = -1;
            if (rows > 0) {
                if (a.genome) {
                    nca = ra.at(0);
                    ncb = has_b ? rb.at(0) : -1;
                } else {
                    na4 = pa[0];
                    nb4 = pb[0];
                }
            }
            for (int i = 0; i < rows; ++i) {
                int ca, cb;
                if (a.genome) {
                    ca = nca;
                    cb = ncb;
                    if (i + 1 < rows) {
                        nca = ra.at(i + 1);
                        ncb = has_b ? rb.at(i + 1) : -1;
                    }
                } else {
                    if ((i & 3) == 0) {
                        if ((i & 15) == 0) {
                            ba = na4;
                            bb = nb4;
                            const int nx = (i >> 4) + 1;
                            if (nx < nblk && 16 * nx < rows) {
                                na4 = pa[nx];
                                nb4 = pb[nx];
                            }
                        }
                        wa4 = ba.x;
                        wb4 = bb.x;
                        ba = make_uint4(ba.y, ba.z, ba.w, 0u);
                        bb = make_uint4(bb.y, bb.z, bb.w, 0u);
                    }
                    const uint32_t sh = 8u * (uint32_t)(i & 3);
                    ca = (int)((wa4 >> sh) & 255u);
                    cb = has_b ? (int)((wb4 >> sh) & 255u) : -1;
                }
                const int ka = ca < 0 ? kBandCodes - 1 : (int)code_of[ca];
                const int kb = cb < 0 ? kBandCodes - 1 : (int)code_of[cb];
                // the band of row i starts at padded position i: copy i & 3, word i >> 2
                const uint32_t *qa = bprof + ((i & 3) * kBandCodes + ka) * rsw + (i >> 2);
                const uint32_t *qb = bprof + ((i & 3) * kBandCodes + kb) * rsw + (i >> 2);
                uint32_t xa[NWB], xb[NWB];
#pragma unroll
                for (int n = 0; n < NWB; ++n) {
                    xa[n] = qa[n];
                    xb[n] = qb[n];
                }
                uint32_t left = 0u, prev = 0u;
#pragma unroll
                for (int k = 0; k < B; ++k) {
                    const uint32_t e = (uint32_t)(k & 3);
                    // bytes: [a's term, 0, b's term, 0]
                    const uint32_t term = __builtin_amdgcn_perm(xb[k >> 2], xa[k >> 2], 0x0C000C00u | ((4u + e) << 16) | e);
                    const uint32_t t = H[k] + term;
                    const uint32_t up = k + 1 < B ? H[k + 1] : 0u;
                    const uint32_t h = idec(imax3(t, up, left));
                    H[k] = h;
                    left = h;
                    if (k & 1)
                        best = imax3(best, prev, h);
                    else if (k == B - 1)
                        best = imax3(best, h, h);
                    prev = h;
                }
            }
            const bool dense_dyn = a.genome && a.stride == 1; // the search's own id (post_processor.cpp:95-101)
            a.cand_ids[q * a.cmax + c0] = dense_dyn ? (uint64_t)nb[c0] : wa;
            a.cand_scores[q * a.cmax + c0] = (int)(best & 0xFFFFu);
            if (has_b) {
                a.cand_ids[q * a.cmax + c1] = dense_dyn ? (uint64_t)nb[c1] : wb;
                a.cand_scores[q * a.cmax + c1] = (int)(best >> 16);
            }
        }
        __syncthreads();
        if (lane == 0)
            a.ncand[q] = ncand;
        __syncthreads();
    }
}

// Kernel 2 of the rerank: sw_reranker's std::partial_sort + output, one thread per query. Each
// thread replays libstdc++'s heap algorithm on its own padded LDS array (stride: an odd number of words, so
// threads touching the same heap index hit different banks). The block loads its queries' score rows and writes
// their results cooperatively (one query row at a time, lanes along the row: coalesced), around the per-thread sort.
// T / S: the packed element (see ps_comp); stride in elements.
template <typename T, int S>
__global__ __launch_bounds__(64) void sw_topk_kernel(RerankArgs a, int stride)
{
    extern __shared__ __align__(16) unsigned char topk_lds[];
    T *heap_lds = reinterpret_cast<T *>(topk_lds);
    __shared__ int ncand_s[64], status_s[64];
    const int tpb = (int)blockDim.x, t = (int)threadIdx.x;
    const int64_t q0 = (int64_t)blockIdx.x * tpb;
    const int nqb = (int)((a.nq - q0) < tpb ? (a.nq - q0) : tpb);
    if (t < nqb) {
        const int ncand = a.ncand[q0 + t];
        int status;
        if (ncand < 0)
            status = ncand; // -2: > kMaxCands candidates, -3: query longer than the SW build
        else if (ncand == 0 || a.k == 0)
            status = 0; // reranker.cpp:10-11: empty result for this query
        else if (ncand < a.k)
            status = -1; // reranker.cpp:26-29
        else
            status = a.k;
        ncand_s[t] = ncand;
        status_s[t] = status;
        a.status[q0 + t] = status;
    }
    __syncthreads();
    for (int r = 0; r < nqb; ++r) { // the rows' (score, candidate) words, packed as the sort compares them
        if (status_s[r] <= 0)
            continue;
        const int nc = ncand_s[r];
        for (int c = t; c < nc; c += tpb)
            heap_lds[(size_t)r * stride + c] = (T)(((uint32_t)a.cand_scores[(q0 + r) * a.cmax + c] << S) | (uint32_t)c);
    }
    __syncthreads();
    if (t < nqb && status_s[t] > 0)
        ps_partial_sort<T, S>(heap_lds + (size_t)t * stride, ncand_s[t], a.k);
    __syncthreads();
    for (int r = 0; r < nqb; ++r) {
        const int64_t q = q0 + r;
        const bool ok = status_s[r] > 0;
        for (int j = t; j < a.k; j += tpb) {
            const uint32_t v = ok ? (uint32_t)heap_lds[(size_t)r * stride + j] : 0u;
            a.top_scores[q * a.k + j] = ok ? (int32_t)(v >> S) : -1;
            a.top_ids[q * a.k + j] = ok ? a.cand_ids[q * a.cmax + (v & ((1u << S) - 1u))] : ~0ull;
        }
    }
}

// Generic batched calc_sw_score: one 64-lane wave per pair builds the profile of seq2 and
// lane 0 runs the DP over seq1 (correctness path for the drm_sw_scores API).
template <int LQ>
__global__ __launch_bounds__(64) void sw_pairs_kernel(const uint8_t *s1, const int64_t *off1, const int32_t *len1,
                                                      const uint8_t *s2, const int64_t *off2, const int32_t *len2,
                                                      int64_t npairs, int32_t *scores)
{
    constexpr int NW = (LQ + 15) / 16;
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
    if (max_qlen <= 152) // 150 bp reads + "<" ">" tags (format_fastq)
        return 152;
    if (max_qlen <= 256)
        return 256;
    throw Error(DRM_ERR_UNSUPPORTED,
                "query length " + std::to_string(max_qlen) + " > 256 is not supported by the GPU SW kernel yet");
}

void launch_sw_rerank(DeviceRefs &refs, RerankArgs a, int max_qlen, hipStream_t stream)
{
    if (a.nq <= 0)
        return;
    if (a.k > kMaxCands)
        throw Error(DRM_ERR_UNSUPPORTED, "k > 1024 not supported by the GPU rerank kernel");
    if (refs.row_stride % 16 != 0)
        throw Error(DRM_ERR_ARG, "window table row stride must be a multiple of 16");
    const int64_t nsel = std::min(a.k_clusters, a.kk);
    const int64_t cmax = std::max<int64_t>(1, std::min<int64_t>(kMaxCands, a.stride == 1 ? nsel : nsel * (2 * a.stride - 1)));
    const size_t need = (size_t)a.nq * (size_t)cmax;
    if (need > refs.ws_elems || !refs.ws_ncand || (size_t)a.nq > refs.ws_nq) {
        if (refs.ws_ids)
            DRM_HIP_CHECK(hipFree(refs.ws_ids));
        if (refs.ws_scores)
            DRM_HIP_CHECK(hipFree(refs.ws_scores));
        if (refs.ws_ncand)
            DRM_HIP_CHECK(hipFree(refs.ws_ncand));
        refs.ws_ids = nullptr;
        refs.ws_scores = nullptr;
        refs.ws_ncand = nullptr;
        DRM_HIP_CHECK(hipMalloc(&refs.ws_ids, sizeof(uint64_t) * need));
        DRM_HIP_CHECK(hipMalloc(&refs.ws_scores, sizeof(int32_t) * need));
        DRM_HIP_CHECK(hipMalloc(&refs.ws_ncand, sizeof(int32_t) * (size_t)a.nq));
        refs.ws_elems = need;
        refs.ws_nq = (size_t)a.nq;
    }
    a.cmax = (int32_t)cmax;
    a.cand_ids = refs.ws_ids;
    a.cand_scores = refs.ws_scores;
    a.ncand = refs.ws_ncand;
    // the bit-profile kernel: one one-wave workgroup per query up to 65536 (grid-stride beyond)
    const int grid = (int)std::min<int64_t>(a.nq, 65536);
#ifndef DRM_SW_F16_GRID_CAP
#define DRM_SW_F16_GRID_CAP (1 << 30)
#endif
    // the pair-profile kernel: one workgroup per query (a query is ~270k issue cycles of one wave, so the grid's
    // tail is one query, not the 19-20 a 65536-wave grid-stride hands each wave at C5)
    const int grid_f16 = (int)std::min<int64_t>(a.nq, (int64_t)DRM_SW_F16_GRID_CAP);
    const size_t cand_lds = sizeof(uint32_t) * (size_t)cmax; // sw_score_f16_kernel's candidate list
    // fp16 pair-profile kernel for queries up to 152 bytes; the bit-profile kernel re-scores the
    // queries it flagged, and takes longer queries (or everything when DRM_SW_BITPROFILE=1).
    if (refs.sw_band > 0) {
        // opt-in banded DP (non-parity): one kernel for every query (status -3 past its limits)
        const int W = refs.sw_band;
        const int qm = std::max(1, std::min(max_qlen, kBandQMax));
        const int rsw = (((qm + W - 1) >> 2) + band_words(W)) | 1; // odd: the copies' rows spread over the banks
        const size_t lds = sizeof(uint32_t) * ((size_t)4 * kBandCodes * (size_t)rsw + (size_t)cmax);
        switch (W) {
        case 8:
            hipLaunchKernelGGL((sw_score_band_kernel<8>), dim3(grid_f16), dim3(64), lds, stream, a, rsw);
            break;
        case 16:
            hipLaunchKernelGGL((sw_score_band_kernel<16>), dim3(grid_f16), dim3(64), lds, stream, a, rsw);
            break;
        case 32:
            hipLaunchKernelGGL((sw_score_band_kernel<32>), dim3(grid_f16), dim3(64), lds, stream, a, rsw);
            break;
        default:
            throw Error(DRM_ERR_ARG, "SW band must be 8, 16 or 32");
        }
    } else {
    static const bool force_bits = [] {
        const char *e = std::getenv("DRM_SW_BITPROFILE");
        return e && std::atoi(e) != 0;
    }();
    switch (pick_lq(max_qlen)) {
    case 64:
        if (force_bits) {
            hipLaunchKernelGGL((sw_score_kernel<64>), dim3(grid), dim3(64), 0, stream, a);
        } else {
            hipLaunchKernelGGL((sw_score_f16_kernel<64>), dim3(grid_f16), dim3(64), cand_lds, stream, a);
            hipLaunchKernelGGL((sw_score_kernel<64, true>), dim3(grid), dim3(64), 0, stream, a);
        }
        break;
    case 152:
        if (force_bits) {
            hipLaunchKernelGGL((sw_score_kernel<152>), dim3(grid), dim3(64), 0, stream, a);
        } else {
            // 150 DP columns: the read's bases; the "<" / ">" tags are dropped in the kernel (a query with more
            // than 150 columns left after its non-ACGT ends is flagged and scored by the bit-profile kernel)
            hipLaunchKernelGGL((sw_score_f16_kernel<150>), dim3(grid_f16), dim3(64), cand_lds, stream, a);
            hipLaunchKernelGGL((sw_score_kernel<152, true>), dim3(grid), dim3(64), 0, stream, a);
        }
        break;
    default:
        hipLaunchKernelGGL((sw_score_kernel<256>), dim3(grid), dim3(64), 0, stream, a);
        break;
    }
    }
    DRM_HIP_CHECK(hipGetLastError());
    // 16-bit elements when every score (<= the window length) and every candidate index fits a byte: half the LDS
    // per query, twice the queries in flight for the latency-bound heap walk
    const bool small = a.ref_len <= 255 && cmax <= 256;
    const size_t esz = small ? 2 : 4;
    const int stride_words = (int)(((size_t)(cmax + 1) * esz + 3) / 4) | 1; // odd: lanes at one index, distinct banks
    const int stride = (int)((size_t)stride_words * 4 / esz);
    int tpb = 64;
    while (tpb > 1 && (size_t)tpb * (size_t)stride * esz > 65536)
        tpb >>= 1;
    const int64_t blocks = (a.nq + tpb - 1) / tpb;
    if (small)
        hipLaunchKernelGGL((sw_topk_kernel<uint16_t, 8>), dim3((unsigned)blocks), dim3(tpb), (size_t)tpb * stride * esz,
                           stream, a, stride);
    else
        hipLaunchKernelGGL((sw_topk_kernel<uint32_t, 16>), dim3((unsigned)blocks), dim3(tpb), (size_t)tpb * stride * esz,
                           stream, a, stride);
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
    case 152:
        hipLaunchKernelGGL(sw_pairs_kernel<152>, dim3(grid), dim3(64), 0, stream, d_s1, d_off1, d_len1, d_s2,
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
