// deepreadmapper_amd/csrc/l2_rerank.hip -- L2 rerank for gfx950 (the reference's live post-processing).
//
// Replaces post_process_l2_static (src/utils/post_processor.cpp:1023-1162; called from
// src/main.cpp:330) -> find_sequences (static, :204-336) -> Vectorizer::vectorize of the candidate
// windows -> batch_reranker (src/utils/reranker.cpp:98-195) -> calc_l2_dist (src/utils/metrics.cpp:48-61).
//
// Candidate embeddings come from a device-resident table of every window's embedding, filled once by
// the GRU encoder (drm_refs_embed). The encoder is a deterministic function of the window bytes, so the
// table row equals what the reference recomputes per run for the same window (4 * d bytes per window:
// 25.6 GB at C5's 50M windows, resident beside the index in 288 GB of HBM).
//
// Distance: calc_l2_dist's loop `diff = a[i] - b[i]; sum += diff * diff` as g++ -O3 -march=native compiles
// it for the reference (build.zig:48-57). Read off the reference's own metrics.cpp built with -mavx2 -mfma
// (oracle/_ref): vsubps/vmulps over blocks of 8 floats, each rounded square then added to `sum` in index
// order (an in-order reduction, no contraction); only a tail of <= 3 elements is fused, and d = 128 has no
// tail. So: sum = sum + round(diff * diff) sequentially, then sqrtf (this file builds with
// -ffp-contract=off). One lane runs one candidate's sum in that order; the squares are formed beforehand
// from coalesced row loads and staged in LDS.
// Top-k: libstdc++ std::partial_sort(first, first + k, last, l2[a] < l2[b]) replayed per query (ties
// included), as the SW rerank does (sw_rerank.hip).
//
// Candidate lists (post_process_l2_static):
//  - dense (stride 1): query q's candidates are its kk labels; find_sequences drops ids >= n_ref while the
//    query boundaries still count kk per query, which makes the reference throw ("Invalid mapping index in
//    expansion", :1100-1106) or read past its arrays -- status -4 here, an error for the call.
//  - sparse (stride > 1): find_sequences expands every label over the whole call into one stream of up to
//    2*stride - 1 windows per label, but the query boundaries advance by kk*stride per query (:1063-1071),
//    so query q reranks stream entries [q*kk*stride, (q+1)*kk*stride) -- windows that may belong to
//    neighbouring queries. That is the reference's result and it is reproduced exactly: the stream offsets
//    are a prefix sum over the call (so a stride > 1 call cannot be split into batches), and a query whose
//    range runs past the stream's end (the reference reads out of bounds there) gets status -4.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "drm_device.h"

namespace drm {
namespace {

constexpr int kBadId = -4;

// find_sequences' sparse expansion of one label (post_processor.cpp:248-258), size_t arithmetic
__device__ __forceinline__ void expand(uint64_t id, uint64_t s, uint64_t n, uint64_t &start, uint64_t &cnt)
{
    const uint64_t actual = id * s; // wraps like the reference's size_t product
    if (actual >= n) {
        start = 0;
        cnt = 0;
        return;
    }
    start = actual >= s - 1 ? actual - s + 1 : 0;
    cnt = min(actual + s, n) - start;
}

// per-query total of the sparse expansion
__global__ __launch_bounds__(256) void l2_expand_count_kernel(L2Args a, uint64_t *qcount)
{
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= a.nq)
        return;
    uint64_t tot = 0;
    for (int j = 0; j < a.lpq; ++j) {
        uint64_t st, c;
        expand((uint64_t)a.neighbors[q * a.kk + j], (uint64_t)a.stride, (uint64_t)a.limit, st, c);
        tot += c;
    }
    qcount[q] = tot;
}

// Kernel 1: one wave per (query, 64 candidates); cand_dist/cand_ids: [nq][cmax] workspace, ncand[q] = status
// (-4 for an invalid label / range; qoff, sparse only: exclusive prefix of the per-query expansion totals). The squares are independent of
// the summation order, so they are formed from coalesced loads -- 32 lanes read 128 contiguous bytes of one
// row, two rows per instruction -- and parked in LDS as [row][32 dims] (row stride 33 words: conflict-free);
// then lane l adds row l's 32 squares in index order to its running sum. Four 32-dim chunks cover d = 128.
constexpr int kStageRows = 64, kStageDims = 32, kStagePitch = kStageDims + 1;

__device__ __forceinline__ bool l2_candidate(const L2Args &a, int64_t q, int c, int nc, const uint64_t *qoff,
                                             uint64_t &pos)
{
    pos = 0;
    if (c >= nc)
        return false;
    if (a.stride == 1) {
        pos = (uint64_t)a.neighbors[q * a.kk + c];
        return pos < (uint64_t)a.limit;
    }
    const uint64_t g = (uint64_t)q * (uint64_t)nc + (uint64_t)c;
    if (g >= qoff[a.nq])
        return false;
    int64_t lo = 0, hi = a.nq;
    while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if (qoff[mid] <= g)
            lo = mid;
        else
            hi = mid;
    }
    uint64_t rem = g - qoff[lo];
    for (int j = 0; j < a.lpq; ++j) {
        uint64_t st, cn;
        expand((uint64_t)a.neighbors[lo * a.kk + j], (uint64_t)a.stride, (uint64_t)a.limit, st, cn);
        if (rem < cn) {
            pos = st + rem;
            break;
        }
        rem -= cn;
    }
    return true;
}

__global__ __launch_bounds__(64) void l2_dist_staged_kernel(L2Args a, int cmax, int chunks, const uint64_t *qoff,
                                                            float *cand_dist, uint64_t *cand_ids, int32_t *ncand)
{
    __shared__ float sq[kStageRows * kStagePitch];
    __shared__ uint32_t row_lo[kStageRows], row_hi[kStageRows];
    const int lane = threadIdx.x;
    const int64_t q = blockIdx.x / chunks;
    const int c = (int)(blockIdx.x - q * chunks) * kStageRows + lane;
    const int nc = a.nc;
    uint64_t pos;
    const bool ok = l2_candidate(a, q, c, nc, qoff, pos);
    if (c < nc && !ok)
        ncand[q] = kBadId;
    const uint64_t rpos = ok ? pos : 0; // rows of absent / invalid candidates: row 0, never stored
    row_lo[lane] = (uint32_t)rpos;
    row_hi[lane] = (uint32_t)(rpos >> 32);
    __syncthreads();
    const int half = lane >> 5, col = lane & 31;
    const float *qv = a.query_emb + q * (int64_t)a.d;
    float sum = 0.0f;
    for (int k0 = 0; k0 < a.d; k0 += kStageDims) {
        const float qx = qv[k0 + col];
        float x[kStageRows / 2];
#pragma unroll
        for (int rr = 0; rr < kStageRows / 2; ++rr) {
            const int r = 2 * rr + half;
            const uint64_t p = ((uint64_t)row_hi[r] << 32) | row_lo[r];
            x[rr] = __builtin_nontemporal_load(a.emb + p * (uint64_t)a.d + k0 + col);
        }
#pragma unroll
        for (int rr = 0; rr < kStageRows / 2; ++rr) {
            const float t = x[rr] - qx; // vec1 = candidate, vec2 = query (batch_reranker :150)
            sq[(2 * rr + half) * kStagePitch + col] = t * t;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kStageDims; ++j)
            sum = sum + sq[lane * kStagePitch + j];
        __syncthreads();
    }
    if (ok) {
        cand_ids[q * cmax + c] = pos;
        cand_dist[q * cmax + c] = __builtin_sqrtf(sum);
    }
}

// libstdc++ partial_sort on packed (distance bits << 32 | index), comp(a, b) = dist[a] < dist[b]. Distances
// are sqrtf of a sum of squares: non-negative (or NaN, not produced by finite embeddings), so their bit
// patterns order like the floats.
__device__ __forceinline__ bool l2_comp(uint64_t x, uint64_t y) { return (x >> 32) < (y >> 32); }

__device__ void l2_adjust_heap(uint64_t *first, int hole, int len, uint64_t value)
{
    const int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (l2_comp(first[second], first[second - 1]))
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
    while (hole > top && l2_comp(first[parent], value)) {
        first[hole] = first[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    first[hole] = value;
}

__device__ void l2_partial_sort(uint64_t *e, int n, int k)
{
    if (k >= 2) {
        int parent = (k - 2) / 2;
        for (;;) {
            l2_adjust_heap(e, parent, k, e[parent]);
            if (parent == 0)
                break;
            parent--;
        }
    }
    for (int i = k; i < n; ++i)
        if (l2_comp(e[i], e[0])) {
            const uint64_t v = e[i];
            e[i] = e[0];
            l2_adjust_heap(e, 0, k, v);
        }
    for (int last = k - 1; last > 0; --last) {
        const uint64_t v = e[last];
        e[last] = e[0];
        l2_adjust_heap(e, 0, last, v);
    }
}

// batch_reranker's partial_sort + output of one query on its own padded LDS array
__device__ void l2_replay_one(const L2Args &a, int cmax, const float *cand_dist, const uint64_t *cand_ids, int64_t q,
                              uint64_t *e)
{
    const int nc = a.nc;
    a.status[q] = a.k; // only complete queries with a tie reach the replay
    for (int c = 0; c < nc; ++c)
        e[c] = ((uint64_t)__float_as_uint(cand_dist[q * cmax + c]) << 32) | (uint32_t)c;
    l2_partial_sort(e, nc, a.k);
    for (int j = 0; j < a.k; ++j) {
        const uint64_t v = e[j];
        a.top_dists[q * a.k + j] = __uint_as_float((uint32_t)(v >> 32));
        a.top_ids[q * a.k + j] = cand_ids[q * cmax + (uint32_t)v];
    }
}


// Kernel 2 (fast path): one wave per query sorts the (distance bits << 32 | index) keys of its candidates in
// registers (E keys per lane, a bitonic network over 64*E slots, partners across lanes by shuffles). With
// distinct distances over the first k + 1 sorted positions, the k smallest form a unique ordered set and
// partial_sort returns exactly it, so the rows are written here. A query with an exact distance tie there is
// appended to the replay list (replay[0] = count), and the heap replay decides its tie order.

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m)
{
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m), hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src)
{
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src), hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}

// ascending bitonic sort of 64*E keys held E per lane (slot i = lane + 64 * h)
template <int E> __device__ __forceinline__ void bitonic_sort(uint64_t (&e)[E], int lane)
{
    constexpr int N = 64 * E;
#pragma unroll
    for (int size = 2; size <= N; size <<= 1) {
#pragma unroll
        for (int j = size >> 1; j > 0; j >>= 1) {
            if (j >= 64) { // partner in the same lane, slot h ^ (j / 64)
#pragma unroll
                for (int h = 0; h < E; ++h) {
                    const int hp = h ^ (j >> 6);
                    if (hp > h) {
                        const int i = lane + 64 * h;
                        const bool up = (i & size) == 0;
                        const uint64_t x = e[h], y = e[hp];
                        const bool sw = up ? (x > y) : (x < y);
                        e[h] = sw ? y : x;
                        e[hp] = sw ? x : y;
                    }
                }
            } else {
#pragma unroll
                for (int h = 0; h < E; ++h) {
                    const int i = lane + 64 * h;
                    const uint64_t y = shfl_xor_u64(e[h], j);
                    const bool up = (i & size) == 0;
                    const bool lower = (lane & j) == 0;
                    // the lower slot keeps the smaller key when ascending, the larger when descending
                    const bool keep_min = lower == up;
                    e[h] = keep_min ? (e[h] < y ? e[h] : y) : (e[h] > y ? e[h] : y);
                }
            }
        }
    }
}

// an exact distance tie among sorted positions [0, k] (next(i) = i + 1), for the whole wave
template <int E> __device__ __forceinline__ bool sorted_tie(const uint64_t (&e)[E], int lane, int k, int nc)
{
    // exact distance ties among sorted positions [0, k]: next(i) = i + 1
    bool tie = false;
#pragma unroll
    for (int h = 0; h < E; ++h) {
        const uint64_t nx_same = shfl_u64(e[h], (lane + 1) & 63);
        const uint64_t nx_wrap = h + 1 < E ? shfl_u64(e[h + 1 < E ? h + 1 : h], 0) : ~0ull;
        const uint64_t nx = lane < 63 ? nx_same : nx_wrap;
        const int i = lane + 64 * h;
        if (i < k && i + 1 < nc && (uint32_t)(nx >> 32) == (uint32_t)(e[h] >> 32))
            tie = true;
    }
    return __any(tie);
}

template <int E>
__global__ __launch_bounds__(64) void l2_sort_kernel(L2Args a, int cmax, const float *cand_dist,
                                                     const uint64_t *cand_ids, int32_t *ncand, uint32_t *replay)
{
    const int64_t q = blockIdx.x;
    const int lane = threadIdx.x;
    const int nc = a.nc;
    const int st0 = ncand[q];
    int status;
    if (st0 == kBadId)
        status = kBadId;
    else if (nc == 0)
        status = 0;
    else if (nc < a.k)
        status = -1;
    else
        status = a.k;
    if (status <= 0) {
        if (lane == 0)
            a.status[q] = status;
        for (int j = lane; j < a.k; j += 64) {
            a.top_dists[q * a.k + j] = -1.0f;
            a.top_ids[q * a.k + j] = ~0ull;
        }
        return;
    }
    uint64_t e[E]; // slot i = lane + 64 * h
#pragma unroll
    for (int h = 0; h < E; ++h) {
        const int i = lane + 64 * h;
        e[h] = i < nc ? ((uint64_t)__float_as_uint(cand_dist[q * cmax + i]) << 32) | (uint32_t)i : ~0ull;
    }
    bitonic_sort<E>(e, lane);
    const bool tie = sorted_tie<E>(e, lane, a.k, nc);
    if (tie) {
        if (lane == 0) // replay[0] = count, replay[1 + j] = the j-th handed-over query
            replay[1 + atomicAdd(replay, 1u)] = (uint32_t)q;
        return;
    }
    if (lane == 0)
        a.status[q] = status;
#pragma unroll
    for (int h = 0; h < E; ++h) {
        const int i = lane + 64 * h;
        if (i < a.k) {
            a.top_dists[q * a.k + i] = __uint_as_float((uint32_t)(e[h] >> 32));
            a.top_ids[q * a.k + i] = cand_ids[q * cmax + (uint32_t)e[h]];
        }
    }
}

// Kernels 1 + 2 fused for queries of at most 128 candidates (the pipeline's K = 128): a 128-lane block stages
// and sums the distances of its query (one wave per 64 candidates, as l2_dist_staged_kernel), the keys meet in
// LDS, and the first wave sorts them (as l2_sort_kernel). The workspace is written only for a query with a tie,
// for the replay.
__global__ __launch_bounds__(128) void l2_fused_kernel(L2Args a, int cmax, const uint64_t *qoff, float *cand_dist,
                                                       uint64_t *cand_ids, uint32_t *replay)
{
    __shared__ float sq[2][kStageRows * kStagePitch];
    __shared__ uint32_t row_lo[128], row_hi[128];
    __shared__ uint64_t keys[128], cpos[128];
    __shared__ int bad;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int64_t q = blockIdx.x;
    const int nc = a.nc;
    if (tid == 0)
        bad = 0;
    __syncthreads();
    uint64_t pos;
    const bool ok = l2_candidate(a, q, tid, nc, qoff, pos);
    if (tid < nc && !ok)
        bad = 1;
    const uint64_t rpos = ok ? pos : 0;
    row_lo[tid] = (uint32_t)rpos;
    row_hi[tid] = (uint32_t)(rpos >> 32);
    cpos[tid] = pos;
    __syncthreads();
    const int half = lane >> 5, col = lane & 31;
    const float *qv = a.query_emb + q * (int64_t)a.d;
    float *sw = sq[w];
    float sum = 0.0f;
    for (int k0 = 0; k0 < a.d; k0 += kStageDims) {
        const float qx = qv[k0 + col];
        float x[kStageRows / 2];
#pragma unroll
        for (int rr = 0; rr < kStageRows / 2; ++rr) {
            const int r = w * kStageRows + 2 * rr + half;
            const uint64_t p = ((uint64_t)row_hi[r] << 32) | row_lo[r];
            x[rr] = __builtin_nontemporal_load(a.emb + p * (uint64_t)a.d + k0 + col);
        }
#pragma unroll
        for (int rr = 0; rr < kStageRows / 2; ++rr) {
            const float t = x[rr] - qx; // vec1 = candidate, vec2 = query (batch_reranker :150)
            sw[(2 * rr + half) * kStagePitch + col] = t * t;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kStageDims; ++j)
            sum = sum + sw[lane * kStagePitch + j];
        __syncthreads();
    }
    const float dist = __builtin_sqrtf(sum);
    keys[tid] = ok ? ((uint64_t)__float_as_uint(dist) << 32) | (uint32_t)tid : ~0ull;
    __syncthreads();
    if (w != 0)
        return; // no block barrier below this point
    int status;
    if (bad)
        status = kBadId;
    else if (nc == 0)
        status = 0;
    else if (nc < a.k)
        status = -1;
    else
        status = a.k;
    if (status <= 0) {
        if (lane == 0)
            a.status[q] = status;
        for (int j = lane; j < a.k; j += 64) {
            a.top_dists[q * a.k + j] = -1.0f;
            a.top_ids[q * a.k + j] = ~0ull;
        }
        return;
    }
    uint64_t e[2] = {keys[lane], keys[lane + 64]};
    bitonic_sort<2>(e, lane);
    if (sorted_tie<2>(e, lane, a.k, nc)) {
        for (int c = lane; c < nc; c += 64) { // the replay reads the query's distances and ids
            cand_dist[q * cmax + c] = __uint_as_float((uint32_t)(keys[c] >> 32));
            cand_ids[q * cmax + c] = cpos[c];
        }
        if (lane == 0)
            replay[1 + atomicAdd(replay, 1u)] = (uint32_t)q;
        return;
    }
    if (lane == 0)
        a.status[q] = status;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int i = lane + 64 * h;
        if (i < a.k) {
            a.top_dists[q * a.k + i] = __uint_as_float((uint32_t)(e[h] >> 32));
            a.top_ids[q * a.k + i] = cpos[(uint32_t)e[h]];
        }
    }
}

// Kernel 3 (tie replay): the queries l2_sort_kernel handed over, one thread each; the grid is sized for the
// worst case but every thread stops at the device-side count
__global__ __launch_bounds__(64) void l2_topk_kernel(L2Args a, int cmax, const float *cand_dist,
                                                     const uint64_t *cand_ids, const uint32_t *replay)
{
    extern __shared__ uint64_t l2_heap[];
    const uint32_t n_replay = replay[0];
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < n_replay; r += gridDim.x * blockDim.x)
        l2_replay_one(a, cmax, cand_dist, cand_ids, (int64_t)replay[1 + r],
                      l2_heap + (size_t)threadIdx.x * (size_t)(cmax + 1));
}

__global__ void l2_fill_status_kernel(int32_t *ncand, int64_t nq)
{
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q < nq)
        ncand[q] = 0;
}

} // namespace

namespace {
__device__ __forceinline__ uint8_t comp_base(uint8_t c) // comp_table, src/utils/parse_inputs.cpp:5-14
{
    return c == 'A' ? 'T' : c == 'T' ? 'A' : c == 'C' ? 'G' : c == 'G' ? 'C' : c == 'N' ? 'N' : 0;
}

// one thread per output byte: row w of the dynamic lookup (find_sequence, src/utils/post_processor.cpp:47-64)
__global__ void genome_rows_kernel(const uint8_t *genome, int64_t glen, int32_t ref_len, int64_t w0, int64_t n,
                                   uint8_t *rows, int64_t row_stride, int32_t *lens)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t r = t / row_stride;
    const int j = (int)(t - r * row_stride);
    if (r >= n)
        return;
    const uint64_t w = (uint64_t)(w0 + r), pos = w >> 1;
    const bool ok = pos + (uint64_t)ref_len <= (uint64_t)glen;
    uint8_t v = 0;
    if (ok && j < ref_len)
        v = (w & 1) ? comp_base(genome[pos + ref_len - 1 - j]) : genome[pos + j];
    rows[r * row_stride + j] = v;
    if (j == 0)
        lens[r] = ok ? ref_len : 0;
}
} // namespace

void launch_genome_rows(const DeviceRefs &refs, int64_t w0, int64_t n, uint8_t *rows, int64_t row_stride,
                        int32_t *lens, hipStream_t stream)
{
    const int64_t threads = n * row_stride;
    if (threads <= 0)
        return;
    hipLaunchKernelGGL(genome_rows_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, stream,
                       refs.genome, refs.glen, refs.ref_len, w0, n, rows, row_stride, lens);
    DRM_HIP_CHECK(hipGetLastError());
}

void launch_l2_rerank(DeviceRefs &refs, L2Args a, hipStream_t stream)
{
    if (a.nq <= 0)
        return;
    if (a.d <= 0 || a.d % kStageDims != 0)
        throw Error(DRM_ERR_ARG, "embedding dimension must be a positive multiple of 32");
    const int64_t nc = a.nc;
    if (nc > kMaxCands)
        throw Error(DRM_ERR_UNSUPPORTED, "more than 1024 candidates per query in the GPU L2 rerank");
    if (a.k > kMaxCands)
        throw Error(DRM_ERR_UNSUPPORTED, "k > 1024 not supported by the GPU L2 rerank");
    const int64_t cmax = std::max<int64_t>(1, nc);
    const size_t need = (size_t)a.nq * (size_t)cmax;
    // the SW workspace, reused: ws_scores holds the distances' bits
    if (need > refs.ws_elems || !refs.ws_ncand || (size_t)a.nq > refs.ws_nq) {
        for (void *p : {(void *)refs.ws_ids, (void *)refs.ws_scores, (void *)refs.ws_ncand})
            if (p)
                DRM_HIP_CHECK(hipFree(p));
        refs.ws_ids = nullptr;
        refs.ws_scores = nullptr;
        refs.ws_ncand = nullptr;
        DRM_HIP_CHECK(hipMalloc(&refs.ws_ids, sizeof(uint64_t) * need));
        DRM_HIP_CHECK(hipMalloc(&refs.ws_scores, sizeof(int32_t) * need));
        DRM_HIP_CHECK(hipMalloc(&refs.ws_ncand, sizeof(int32_t) * (size_t)a.nq));
        refs.ws_elems = need;
        refs.ws_nq = (size_t)a.nq;
    }
    float *cand_dist = reinterpret_cast<float *>(refs.ws_scores);
    if (nc > 128) // the staged distance kernel reports invalid labels through ncand
        hipLaunchKernelGGL(l2_fill_status_kernel, dim3((unsigned)((a.nq + 255) / 256)), dim3(256), 0, stream,
                           refs.ws_ncand, a.nq);
    uint64_t *qoff = nullptr;
    void *scan_tmp = nullptr;
    if (a.stride > 1) {
        // per-query expansion totals -> exclusive prefix qoff[0..nq], qoff[nq] = the stream length
        DRM_HIP_CHECK(hipMallocAsync((void **)&qoff, sizeof(uint64_t) * (size_t)(a.nq + 1), stream));
        DRM_HIP_CHECK(hipMemsetAsync(qoff, 0, sizeof(uint64_t) * (size_t)(a.nq + 1), stream));
        hipLaunchKernelGGL(l2_expand_count_kernel, dim3((unsigned)((a.nq + 255) / 256)), dim3(256), 0, stream, a,
                           qoff);
        size_t tmp_bytes = 0;
        DRM_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, qoff, qoff, (int)(a.nq + 1), stream));
        DRM_HIP_CHECK(hipMallocAsync(&scan_tmp, std::max<size_t>(tmp_bytes, 16), stream));
        DRM_HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(scan_tmp, tmp_bytes, qoff, qoff, (int)(a.nq + 1), stream));
    }
    uint32_t *replay = nullptr; // [0] = count, then the handed-over queries
    DRM_HIP_CHECK(hipMallocAsync((void **)&replay, sizeof(uint32_t) * (size_t)(a.nq + 1), stream));
    DRM_HIP_CHECK(hipMemsetAsync(replay, 0, sizeof(uint32_t), stream));
    if (nc <= 128) {
        hipLaunchKernelGGL(l2_fused_kernel, dim3((unsigned)a.nq), dim3(128), 0, stream, a, (int)cmax, qoff, cand_dist,
                           refs.ws_ids, replay);
    } else {
        const int chunks = (int)((nc + kStageRows - 1) / kStageRows);
        hipLaunchKernelGGL(l2_dist_staged_kernel, dim3((unsigned)(a.nq * chunks)), dim3(kStageRows), 0, stream, a,
                           (int)cmax, chunks, qoff, cand_dist, refs.ws_ids, refs.ws_ncand);
        DRM_HIP_CHECK(hipGetLastError());
        switch (cmax <= 256 ? 4 : cmax <= 512 ? 8 : 16) {
        case 4:
            hipLaunchKernelGGL(l2_sort_kernel<4>, dim3((unsigned)a.nq), dim3(64), 0, stream, a, (int)cmax, cand_dist,
                               refs.ws_ids, refs.ws_ncand, replay);
            break;
        case 8:
            hipLaunchKernelGGL(l2_sort_kernel<8>, dim3((unsigned)a.nq), dim3(64), 0, stream, a, (int)cmax, cand_dist,
                               refs.ws_ids, refs.ws_ncand, replay);
            break;
        default:
            hipLaunchKernelGGL(l2_sort_kernel<16>, dim3((unsigned)a.nq), dim3(64), 0, stream, a, (int)cmax,
                               cand_dist, refs.ws_ids, refs.ws_ncand, replay);
            break;
        }
    }
    DRM_HIP_CHECK(hipGetLastError());
    int tpb = 64;
    while (tpb > 1 && (size_t)tpb * (size_t)(cmax + 1) * 8 > 65536)
        tpb >>= 1;
    const int64_t blocks = std::min<int64_t>((a.nq + tpb - 1) / tpb, 128); // ties are rare: a small grid drains the list
    hipLaunchKernelGGL(l2_topk_kernel, dim3((unsigned)blocks), dim3(tpb), (size_t)tpb * (size_t)(cmax + 1) * 8,
                       stream, a, (int)cmax, cand_dist, refs.ws_ids, replay);
    DRM_HIP_CHECK(hipGetLastError());
    DRM_HIP_CHECK(hipFreeAsync(replay, stream));
    if (qoff) {
        DRM_HIP_CHECK(hipFreeAsync(scan_tmp, stream));
        DRM_HIP_CHECK(hipFreeAsync(qoff, stream));
    }
}

} // namespace drm
