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
// -ffp-contract=off). One lane runs one candidate's chain in that order.
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
    for (int j = 0; j < a.kk; ++j) {
        uint64_t st, c;
        expand((uint64_t)a.neighbors[q * a.kk + j], (uint64_t)a.stride, (uint64_t)a.n_ref, st, c);
        tot += c;
    }
    qcount[q] = tot;
}

// calc_l2_dist of one candidate: rounded squares added in index order over d dims, row read as float4s
__device__ __forceinline__ float l2_chain(const float *__restrict__ row, const float *__restrict__ qv, int d)
{
    float sum = 0.0f;
    typedef float v4f __attribute__((ext_vector_type(4)));
    const v4f *r4 = reinterpret_cast<const v4f *>(row);
    const v4f *q4 = reinterpret_cast<const v4f *>(qv);
    for (int i = 0; i < d / 4; ++i) {
        const v4f x = __builtin_nontemporal_load(r4 + i);
        const v4f y = q4[i];
        float t;
        t = x.x - y.x; // vec1 = candidate, vec2 = query (batch_reranker :150)
        sum = sum + t * t;
        t = x.y - y.y;
        sum = sum + t * t;
        t = x.z - y.z;
        sum = sum + t * t;
        t = x.w - y.w;
        sum = sum + t * t;
    }
    return __builtin_sqrtf(sum);
}

// Kernel 1: one lane per (query, candidate). cand_dist/cand_ids: [nq][cmax] workspace; ncand[q] = status.
// qoff (sparse only): exclusive prefix of the per-query expansion totals, total = qoff[nq].
__global__ __launch_bounds__(256) void l2_dist_kernel(L2Args a, int cmax, const uint64_t *qoff, float *cand_dist,
                                                      uint64_t *cand_ids, int32_t *ncand)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t q = t / cmax;
    const int c = (int)(t - q * cmax);
    if (q >= a.nq)
        return;
    const int nc = (int)(a.stride == 1 ? a.kk : (int64_t)a.kk * a.stride);
    if (c >= nc)
        return;
    uint64_t pos;
    bool ok;
    if (a.stride == 1) {
        pos = (uint64_t)a.neighbors[q * a.kk + c];
        ok = pos < (uint64_t)a.n_ref;
    } else {
        // global stream entry g of the call; owning query by binary search over qoff, then its label
        const uint64_t g = (uint64_t)q * (uint64_t)nc + (uint64_t)c;
        ok = g < qoff[a.nq];
        pos = 0;
        if (ok) {
            int64_t lo = 0, hi = a.nq; // last qq with qoff[qq] <= g
            while (hi - lo > 1) {
                const int64_t mid = (lo + hi) >> 1;
                if (qoff[mid] <= g)
                    lo = mid;
                else
                    hi = mid;
            }
            uint64_t rem = g - qoff[lo];
            for (int j = 0; j < a.kk; ++j) {
                uint64_t st, cn;
                expand((uint64_t)a.neighbors[lo * a.kk + j], (uint64_t)a.stride, (uint64_t)a.n_ref, st, cn);
                if (rem < cn) {
                    pos = st + rem;
                    break;
                }
                rem -= cn;
            }
        }
    }
    if (!ok) {
        ncand[q] = kBadId; // every writer stores the same value
        return;
    }
    cand_ids[q * cmax + c] = pos;
    cand_dist[q * cmax + c] = l2_chain(a.emb + pos * (uint64_t)a.d, a.query_emb + q * (int64_t)a.d, a.d);
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

// Kernel 2: batch_reranker's partial_sort + output, one thread per query on a padded LDS array
__global__ __launch_bounds__(64) void l2_topk_kernel(L2Args a, int cmax, const float *cand_dist,
                                                     const uint64_t *cand_ids, const int32_t *ncand)
{
    extern __shared__ uint64_t l2_heap[];
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= a.nq)
        return;
    uint64_t *e = l2_heap + (size_t)threadIdx.x * (size_t)(cmax + 1);
    const int nc = (int)(a.stride == 1 ? a.kk : (int64_t)a.kk * a.stride);
    int status;
    if (ncand[q] == kBadId)
        status = kBadId;
    else if (nc == 0)
        status = 0; // :131-140: empty result
    else if (nc < a.k)
        status = -1; // :154-158
    else
        status = a.k;
    a.status[q] = status;
    if (status > 0) {
        for (int c = 0; c < nc; ++c)
            e[c] = ((uint64_t)__float_as_uint(cand_dist[q * cmax + c]) << 32) | (uint32_t)c;
        l2_partial_sort(e, nc, a.k);
        for (int j = 0; j < a.k; ++j) {
            const uint64_t v = e[j];
            a.top_dists[q * a.k + j] = __uint_as_float((uint32_t)(v >> 32));
            a.top_ids[q * a.k + j] = cand_ids[q * cmax + (uint32_t)v];
        }
    } else {
        for (int j = 0; j < a.k; ++j) {
            a.top_dists[q * a.k + j] = -1.0f;
            a.top_ids[q * a.k + j] = ~0ull;
        }
    }
}

__global__ void l2_fill_status_kernel(int32_t *ncand, int64_t nq)
{
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q < nq)
        ncand[q] = 0;
}

} // namespace

void launch_l2_rerank(DeviceRefs &refs, L2Args a, hipStream_t stream)
{
    if (a.nq <= 0)
        return;
    if (a.d <= 0 || a.d % 4 != 0)
        throw Error(DRM_ERR_ARG, "embedding dimension must be a positive multiple of 4");
    const int64_t nc = a.stride == 1 ? a.kk : (int64_t)a.kk * a.stride;
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
    const int64_t threads = a.nq * cmax;
    hipLaunchKernelGGL(l2_dist_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, stream, a, (int)cmax,
                       qoff, cand_dist, refs.ws_ids, refs.ws_ncand);
    DRM_HIP_CHECK(hipGetLastError());
    int tpb = 64;
    while (tpb > 1 && (size_t)tpb * (size_t)(cmax + 1) * 8 > 65536)
        tpb >>= 1;
    const int64_t blocks = (a.nq + tpb - 1) / tpb;
    hipLaunchKernelGGL(l2_topk_kernel, dim3((unsigned)blocks), dim3(tpb), (size_t)tpb * (size_t)(cmax + 1) * 8,
                       stream, a, (int)cmax, cand_dist, refs.ws_ids, refs.ws_ncand);
    DRM_HIP_CHECK(hipGetLastError());
    if (qoff) {
        DRM_HIP_CHECK(hipFreeAsync(scan_tmp, stream));
        DRM_HIP_CHECK(hipFreeAsync(qoff, stream));
    }
}

} // namespace drm
