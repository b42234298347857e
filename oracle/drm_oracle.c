/*
 * oracle/drm_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's query hot path, used (a) as the parity checker for the HIP
 * path and (b) as the OpenMP CPU baseline timed by bench.py. Never linked into the product.
 * Compile with -ffp-contract=off: every fp32 product/sum below is rounded separately, in the
 * order written, which is the order the HIP kernels use (DESIGN.md "fixed fp32 op order").
 *
 * Citations are to /root/reference (DeepReadMapper) unless marked [upstream faiss], in which case
 * the code restates faiss >= 1.8 semantics (faiss is not vendored in the reference nor installed
 * here): faiss/impl/HNSW.cpp, faiss/utils/Heap.h, faiss/IndexHNSW.cpp,
 * faiss/IndexPQ.cpp, faiss/impl/ProductQuantizer.cpp, faiss/impl/code_distance/.
 */
#include "drm_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static inline int imax(int a, int b) { return a > b ? a : b; }

/* ========================================================================================
 * Smith-Waterman score. Restates calc_sw_score, src/utils/metrics.cpp:10-45:
 *   match +1, mismatch -1, linear gap -1 (:18-20), dp[i][j] = max(0, diag+s, up-1, left-1)
 *   (:30-41), running max over all cells. Raw byte equality (case-sensitive, 'N'=='N').
 * The full (len1+1)x(len2+1) matrix of :26 is replaced by one rolling row: same values.
 * ====================================================================================== */
int oracle_calc_sw_score(const uint8_t *s1, int64_t len1, const uint8_t *s2, int64_t len2)
{
    if (len1 <= 0 || len2 <= 0)
        return 0;
    int stack_row[1024];
    int *row = (len2 + 1 <= 1024) ? stack_row : (int *)malloc(sizeof(int) * (size_t)(len2 + 1));
    for (int64_t j = 0; j <= len2; ++j)
        row[j] = 0;
    int best = 0;
    for (int64_t i = 1; i <= len1; ++i) {
        const uint8_t c1 = s1[i - 1];
        int diag = 0; /* dp[i-1][0] */
        int left = 0; /* dp[i][0]   */
        for (int64_t j = 1; j <= len2; ++j) {
            const int up = row[j];
            const int sm = diag + (c1 == s2[j - 1] ? 1 : -1);
            int h = imax(imax(0, sm), imax(up - 1, left - 1));
            diag = up;
            row[j] = h;
            left = h;
            best = imax(best, h);
        }
    }
    if (row != stack_row)
        free(row);
    return best;
}

/* ========================================================================================
 * Banded Smith-Waterman: an opt-in, NON-PARITY mode of this implementation (the reference has only
 * a TODO for it, includes/utils/reranker.hpp:12). The recurrence of calc_sw_score restricted to
 * the cells with |i - j| <= band (1-based row i over s1, column j over s2); a cell outside the
 * band is 0, so an alignment path stays inside it. band <= 0 is the full DP above. The score is
 * at most the full one and equals it when the best local alignment lies inside the band.
 * ====================================================================================== */
int oracle_calc_sw_score_banded(const uint8_t *s1, int64_t len1, const uint8_t *s2, int64_t len2, int64_t band)
{
    if (band <= 0)
        return oracle_calc_sw_score(s1, len1, s2, len2);
    if (len1 <= 0 || len2 <= 0)
        return 0;
    int *row = (int *)calloc((size_t)(len2 + 1), sizeof(int)); /* dp[i-1][*]; out-of-band cells hold 0 */
    int best = 0;
    for (int64_t i = 1; i <= len1; ++i) {
        const uint8_t c1 = s1[i - 1];
        int diag = 0, left = 0;
        for (int64_t j = 1; j <= len2; ++j) {
            const int up = row[j];
            int h = 0;
            if (j - i <= band && i - j <= band)
                h = imax(imax(0, diag + (c1 == s2[j - 1] ? 1 : -1)), imax(up - 1, left - 1));
            diag = up;
            row[j] = h;
            left = h;
            best = imax(best, h);
        }
    }
    free(row);
    return best;
}

/* ========================================================================================
 * libstdc++ std::partial_sort with comp(a, b) := scores[a] > scores[b], the exact call of
 * src/utils/reranker.cpp:38-40. Restates __partial_sort = __heap_select + __sort_heap and the
 * helpers __make_heap / __adjust_heap / __push_heap / __pop_heap (bits/stl_heap.h,
 * bits/stl_algo.h, GCC 11). Tie order among equal scores follows the heap mechanics exactly.
 * ====================================================================================== */
#define PS_COMP(a, b) (scores[(a)] > scores[(b)])

static void ps_adjust_heap(int64_t *first, int64_t hole, int64_t len, int64_t value, const int32_t *scores)
{
    const int64_t top = hole;
    int64_t second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (PS_COMP(first[second], first[second - 1]))
            second--;
        first[hole] = first[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        first[hole] = first[second - 1];
        hole = second - 1;
    }
    /* __push_heap(first, hole, top, value) with comp(*parent, value) */
    int64_t parent = (hole - 1) / 2;
    while (hole > top && PS_COMP(first[parent], value)) {
        first[hole] = first[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    first[hole] = value;
}

static void ps_make_heap(int64_t *first, int64_t len, const int32_t *scores)
{
    if (len < 2)
        return;
    int64_t parent = (len - 2) / 2;
    for (;;) {
        int64_t value = first[parent];
        ps_adjust_heap(first, parent, len, value, scores);
        if (parent == 0)
            return;
        parent--;
    }
}

/* __pop_heap(first, first+len, result) */
static void ps_pop_heap(int64_t *first, int64_t len, int64_t *result, const int32_t *scores)
{
    int64_t value = *result;
    *result = first[0];
    ps_adjust_heap(first, 0, len, value, scores);
}

void oracle_partial_sort_desc(int64_t *idx, int64_t n, int64_t k, const int32_t *scores)
{
    if (k <= 0)
        return;
    /* __heap_select(first, middle, last) */
    ps_make_heap(idx, k, scores);
    for (int64_t i = k; i < n; ++i)
        if (PS_COMP(idx[i], idx[0]))
            ps_pop_heap(idx, k, idx + i, scores);
    /* __sort_heap(first, middle) */
    int64_t last = k;
    while (last > 1) {
        --last;
        ps_pop_heap(idx, last, idx + last, scores);
    }
}

/* ========================================================================================
 * post_process_sw_static (src/utils/post_processor.cpp:454-549) + find_sequences static
 * (:204-336) + sw_reranker (src/utils/reranker.cpp:3-51).
 * ====================================================================================== */
static int64_t pp_one_query(const int64_t *nb, int64_t kk, const uint8_t *refs, int64_t n_ref, int64_t ref_len,
                            int64_t ref_stride, const uint8_t *q, int32_t qlen, int64_t stride, int64_t k,
                            int64_t k_clusters, int64_t band, int32_t *out_scores, uint64_t *out_ids)
{
    /* :494-495  first min(k_clusters, n_i) neighbour ids, converted long -> size_t (:339-355) */
    const int64_t nsel = k_clusters < kk ? k_clusters : kk;
    int64_t cap = (stride == 1) ? (nsel > 0 ? nsel : 1) : (nsel * (2 * stride) + 1);
    uint64_t *cand = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)cap);
    int64_t ncand = 0;
    if (stride == 1) {
        /* dense branch :215-236 -- ids >= ref_seqs.size() (e.g. -1 -> 2^64-1) are dropped */
        for (int64_t i = 0; i < nsel; ++i) {
            uint64_t id = (uint64_t)nb[i];
            if (id < (uint64_t)n_ref)
                cand[ncand++] = id;
        }
    } else {
        /* sparse branch :238-335: expand sparse_id*stride to [pos-stride+1, pos+stride), the
         * mapping keeps every expansion (duplicates included) in original order. */
        for (int64_t i = 0; i < nsel; ++i) {
            uint64_t actual = (uint64_t)nb[i] * (uint64_t)stride; /* size_t arithmetic, wraps */
            if (actual >= (uint64_t)n_ref)
                continue;
            uint64_t start = (actual >= (uint64_t)(stride - 1)) ? actual - (uint64_t)stride + 1 : 0;
            uint64_t end = actual + (uint64_t)stride;
            if (end > (uint64_t)n_ref)
                end = (uint64_t)n_ref;
            for (uint64_t pos = start; pos < end; ++pos)
                cand[ncand++] = pos;
        }
    }
    if (ncand == 0 || k == 0) { /* reranker.cpp:10-11 returns empty: the query contributes 0 rows */
        free(cand);
        return 0;
    }
    int32_t *scores = (int32_t *)malloc(sizeof(int32_t) * (size_t)ncand);
    for (int64_t c = 0; c < ncand; ++c)
        scores[c] = oracle_calc_sw_score_banded(refs + cand[c] * (uint64_t)ref_stride, ref_len, q, qlen, band);
    if (ncand < k) { /* reranker.cpp:26-29 */
        free(scores);
        free(cand);
        return -1;
    }
    int64_t *idx = (int64_t *)malloc(sizeof(int64_t) * (size_t)ncand);
    for (int64_t c = 0; c < ncand; ++c)
        idx[c] = c;
    oracle_partial_sort_desc(idx, ncand, k, scores);
    for (int64_t j = 0; j < k; ++j) {
        out_scores[j] = scores[idx[j]];
        out_ids[j] = cand[idx[j]];
    }
    free(idx);
    free(scores);
    free(cand);
    return k;
}

int64_t oracle_post_process_sw_static_banded(const int64_t *neighbors, int64_t nq, int64_t kk, const uint8_t *refs,
                                             int64_t n_ref, int64_t ref_len, int64_t ref_stride, const uint8_t *queries,
                                             const int32_t *q_len, int64_t q_stride, int64_t stride, int64_t k,
                                             int64_t k_clusters, int64_t band, int nthreads, int32_t *top_scores,
                                             uint64_t *top_ids, int32_t *counts)
{
    if (k > k_clusters * 2 * stride) /* :486-489 */
        return -1000000000;
    int64_t first_bad = -1;
#ifdef _OPENMP
    if (nthreads <= 0)
        nthreads = omp_get_max_threads();
#pragma omp parallel for num_threads(nthreads) schedule(dynamic)
#endif
    for (int64_t i = 0; i < nq; ++i) {
        for (int64_t j = 0; j < k; ++j) {
            top_scores[i * k + j] = -1;
            top_ids[i * k + j] = UINT64_MAX;
        }
        int64_t r = pp_one_query(neighbors + i * kk, kk, refs, n_ref, ref_len, ref_stride, queries + i * q_stride,
                                 q_len[i], stride, k, k_clusters, band, top_scores + i * k, top_ids + i * k);
        counts[i] = r < 0 ? 0 : (int32_t)r;
        if (r < 0) {
#ifdef _OPENMP
#pragma omp critical
#endif
            {
                if (first_bad < 0 || i < first_bad)
                    first_bad = i;
            }
        }
    }
    return first_bad >= 0 ? -(1 + first_bad) : 0;
}

int64_t oracle_post_process_sw_static(const int64_t *neighbors, int64_t nq, int64_t kk, const uint8_t *refs,
                                      int64_t n_ref, int64_t ref_len, int64_t ref_stride, const uint8_t *queries,
                                      const int32_t *q_len, int64_t q_stride, int64_t stride, int64_t k,
                                      int64_t k_clusters, int nthreads, int32_t *top_scores, uint64_t *top_ids,
                                      int32_t *counts)
{
    return oracle_post_process_sw_static_banded(neighbors, nq, kk, refs, n_ref, ref_len, ref_stride, queries, q_len,
                                                q_stride, stride, k, k_clusters, 0, nthreads, top_scores, top_ids,
                                                counts);
}

/* ========================================================================================
 * post_process_sw_dynamic (src/utils/post_processor.cpp:357-452): candidate windows cut from the
 * genome string (extract_FASTA_sequence, src/utils/parse_inputs.cpp:174-220) by find_sequences
 * dynamic (:72-201) / find_sequence (:47-64), then sw_reranker.
 *   dense (stride 1): every one of the first min(k_clusters, n) ids is a candidate (no range check;
 *     an id whose window runs past the genome -- e.g. -1 -> 2^64-1 -- is the empty string, score 0);
 *   sparse: actual = id * stride is checked against the GENOME LENGTH and the expansion
 *     [actual - stride + 1, actual + stride) is clipped to it (the reference's quirk), duplicates kept.
 * find_sequence: window id -> position id / 2, reverse complement (comp_table :5-14) when id is odd.
 * ====================================================================================== */
static uint8_t comp_byte(uint8_t c)
{
    switch (c) {
    case 'A': return 'T';
    case 'T': return 'A';
    case 'C': return 'G';
    case 'G': return 'C';
    case 'N': return 'N';
    default: return 0;
    }
}

/* find_sequence: the window of dense id `id` into buf (ref_len bytes), returns its length (0 = "") */
static int64_t find_sequence_dyn(const uint8_t *g, int64_t glen, uint64_t id, int64_t ref_len, uint8_t *buf)
{
    const uint64_t pos = id / 2;
    if (pos + (uint64_t)ref_len > (uint64_t)glen)
        return 0;
    if (id % 2 == 1)
        for (int64_t i = 0; i < ref_len; ++i)
            buf[i] = comp_byte(g[pos + (uint64_t)(ref_len - 1 - i)]);
    else
        memcpy(buf, g + pos, (size_t)ref_len);
    return ref_len;
}

static int64_t ppd_one_query(const int64_t *nb, int64_t kk, const uint8_t *g, int64_t glen, int64_t ref_len,
                             const uint8_t *q, int32_t qlen, int64_t stride, int64_t k, int64_t k_clusters,
                             int64_t band, int32_t *out_scores, uint64_t *out_ids)
{
    const int64_t nsel = k_clusters < kk ? k_clusters : kk;
    int64_t cap = (stride == 1) ? (nsel > 0 ? nsel : 1) : (nsel * (2 * stride) + 1);
    uint64_t *cand = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)cap);
    int64_t ncand = 0;
    if (stride == 1) {
        for (int64_t i = 0; i < nsel; ++i)
            cand[ncand++] = (uint64_t)nb[i];
    } else {
        for (int64_t i = 0; i < nsel; ++i) {
            uint64_t actual = (uint64_t)nb[i] * (uint64_t)stride;
            if (actual >= (uint64_t)glen)
                continue;
            uint64_t start = (actual >= (uint64_t)(stride - 1)) ? actual - (uint64_t)stride + 1 : 0;
            uint64_t end = actual + (uint64_t)stride;
            if (end > (uint64_t)glen)
                end = (uint64_t)glen;
            for (uint64_t pos = start; pos < end; ++pos)
                cand[ncand++] = pos;
        }
    }
    if (ncand == 0 || k == 0) {
        free(cand);
        return 0;
    }
    int32_t *scores = (int32_t *)malloc(sizeof(int32_t) * (size_t)ncand);
    uint8_t *buf = (uint8_t *)malloc((size_t)(ref_len > 0 ? ref_len : 1));
    for (int64_t c = 0; c < ncand; ++c) {
        const int64_t len = find_sequence_dyn(g, glen, cand[c], ref_len, buf);
        scores[c] = oracle_calc_sw_score_banded(buf, len, q, qlen, band);
    }
    free(buf);
    if (ncand < k) {
        free(scores);
        free(cand);
        return -1;
    }
    int64_t *idx = (int64_t *)malloc(sizeof(int64_t) * (size_t)ncand);
    for (int64_t c = 0; c < ncand; ++c)
        idx[c] = c;
    oracle_partial_sort_desc(idx, ncand, k, scores);
    for (int64_t j = 0; j < k; ++j) {
        out_scores[j] = scores[idx[j]];
        out_ids[j] = cand[idx[j]];
    }
    free(idx);
    free(scores);
    free(cand);
    return k;
}

int64_t oracle_post_process_sw_dynamic_banded(const int64_t *neighbors, int64_t nq, int64_t kk,
                                              const uint8_t *genome, int64_t glen, int64_t ref_len,
                                              const uint8_t *queries, const int32_t *q_len, int64_t q_stride,
                                              int64_t stride, int64_t k, int64_t k_clusters, int64_t band,
                                              int nthreads, int32_t *top_scores, uint64_t *top_ids, int32_t *counts)
{
    if (k > k_clusters * 2 * stride) /* :390-393 */
        return -1000000000;
    int64_t first_bad = -1;
#ifdef _OPENMP
    if (nthreads <= 0)
        nthreads = omp_get_max_threads();
#pragma omp parallel for num_threads(nthreads) schedule(dynamic)
#endif
    for (int64_t i = 0; i < nq; ++i) {
        for (int64_t j = 0; j < k; ++j) {
            top_scores[i * k + j] = -1;
            top_ids[i * k + j] = UINT64_MAX;
        }
        int64_t r = ppd_one_query(neighbors + i * kk, kk, genome, glen, ref_len, queries + i * q_stride, q_len[i],
                                  stride, k, k_clusters, band, top_scores + i * k, top_ids + i * k);
        counts[i] = r < 0 ? 0 : (int32_t)r;
        if (r < 0) {
#ifdef _OPENMP
#pragma omp critical
#endif
            {
                if (first_bad < 0 || i < first_bad)
                    first_bad = i;
            }
        }
    }
    return first_bad >= 0 ? -(1 + first_bad) : 0;
}

int64_t oracle_post_process_sw_dynamic(const int64_t *neighbors, int64_t nq, int64_t kk, const uint8_t *genome,
                                       int64_t glen, int64_t ref_len, const uint8_t *queries, const int32_t *q_len,
                                       int64_t q_stride, int64_t stride, int64_t k, int64_t k_clusters, int nthreads,
                                       int32_t *top_scores, uint64_t *top_ids, int32_t *counts)
{
    return oracle_post_process_sw_dynamic_banded(neighbors, nq, kk, genome, glen, ref_len, queries, q_len, q_stride,
                                                 stride, k, k_clusters, 0, nthreads, top_scores, top_ids, counts);
}

/* ========================================================================================
 * faiss IndexHNSWPQ search [upstream faiss >= 1.8].
 * ====================================================================================== */

/* operation counters (diagnostic; summed over all queries of the last oracle_hnswpq_search call) */
static int64_t g_cnt_push, g_cnt_pop, g_cnt_reject, g_cnt_result, g_cnt_tiepop, g_cnt_tieq;
/* per-thread tallies, folded into the globals once per thread (no atomics in the hot loop) */
static _Thread_local int64_t t_push, t_pop, t_reject, t_result, t_tiepop, t_tieq;
/* faiss::CMax<T,TI>::cmp2 -- (a1 > b1) || (a1 == b1 && a2 > b2) */
#define CMP2(v1, v2, i1, i2) (((v1) > (v2)) || (((v1) == (v2)) && ((i1) > (i2))))

/* faiss/utils/Heap.h heap_push<CMax<float,int32>> (1-based internally) */
static void heap_push_i32(size_t k, float *bh_val, int32_t *bh_ids, float val, int32_t id)
{
    bh_val--;
    bh_ids--;
    size_t i = k, i_father;
    while (i > 1) {
        i_father = i >> 1;
        if (!CMP2(val, bh_val[i_father], id, bh_ids[i_father]))
            break;
        bh_val[i] = bh_val[i_father];
        bh_ids[i] = bh_ids[i_father];
        i = i_father;
    }
    bh_val[i] = val;
    bh_ids[i] = id;
}

/* faiss/utils/Heap.h heap_pop<CMax<float,int32>> */
static void heap_pop_i32(size_t k, float *bh_val, int32_t *bh_ids)
{
    bh_val--;
    bh_ids--;
    float val = bh_val[k];
    int32_t id = bh_ids[k];
    size_t i = 1, i1, i2;
    for (;;) {
        i1 = i << 1;
        i2 = i1 + 1;
        if (i1 > k)
            break;
        if ((i2 == k + 1) || CMP2(bh_val[i1], bh_val[i2], bh_ids[i1], bh_ids[i2])) {
            if (CMP2(val, bh_val[i1], id, bh_ids[i1]))
                break;
            bh_val[i] = bh_val[i1];
            bh_ids[i] = bh_ids[i1];
            i = i1;
        } else {
            if (CMP2(val, bh_val[i2], id, bh_ids[i2]))
                break;
            bh_val[i] = bh_val[i2];
            bh_ids[i] = bh_ids[i2];
            i = i2;
        }
    }
    bh_val[i] = bh_val[k];
    bh_ids[i] = bh_ids[k];
}

/* faiss/utils/Heap.h heap_replace_top<CMax<float,int64>> */
static void heap_replace_top_i64(size_t k, float *bh_val, int64_t *bh_ids, float val, int64_t id)
{
    bh_val--;
    bh_ids--;
    size_t i = 1, i1, i2;
    for (;;) {
        i1 = i << 1;
        i2 = i1 + 1;
        if (i1 > k)
            break;
        if ((i2 == k + 1) || CMP2(bh_val[i1], bh_val[i2], bh_ids[i1], bh_ids[i2])) {
            if (CMP2(val, bh_val[i1], id, bh_ids[i1]))
                break;
            bh_val[i] = bh_val[i1];
            bh_ids[i] = bh_ids[i1];
            i = i1;
        } else {
            if (CMP2(val, bh_val[i2], id, bh_ids[i2]))
                break;
            bh_val[i] = bh_val[i2];
            bh_ids[i] = bh_ids[i2];
            i = i2;
        }
    }
    bh_val[i] = val;
    bh_ids[i] = id;
}

/* heap_pop<CMax<float,int64>> used by heap_reorder */
static void heap_pop_i64(size_t k, float *bh_val, int64_t *bh_ids)
{
    bh_val--;
    bh_ids--;
    float val = bh_val[k];
    int64_t id = bh_ids[k];
    size_t i = 1, i1, i2;
    for (;;) {
        i1 = i << 1;
        i2 = i1 + 1;
        if (i1 > k)
            break;
        if ((i2 == k + 1) || CMP2(bh_val[i1], bh_val[i2], bh_ids[i1], bh_ids[i2])) {
            if (CMP2(val, bh_val[i1], id, bh_ids[i1]))
                break;
            bh_val[i] = bh_val[i1];
            bh_ids[i] = bh_ids[i1];
            i = i1;
        } else {
            if (CMP2(val, bh_val[i2], id, bh_ids[i2]))
                break;
            bh_val[i] = bh_val[i2];
            bh_ids[i] = bh_ids[i2];
            i = i2;
        }
    }
    bh_val[i] = bh_val[k];
    bh_ids[i] = bh_ids[k];
}

/* faiss/utils/Heap.h heap_reorder<CMax<float,int64>> */
static void heap_reorder_i64(size_t k, float *bh_val, int64_t *bh_ids)
{
    size_t i, ii;
    for (i = 0, ii = 0; i < k; i++) {
        float val = bh_val[0];
        int64_t id = bh_ids[0];
        heap_pop_i64(k - i, bh_val, bh_ids);
        bh_val[k - ii - 1] = val;
        bh_ids[k - ii - 1] = id;
        if (id != -1)
            ii++;
    }
    memmove(bh_val, bh_val + k - ii, ii * sizeof(*bh_val));
    memmove(bh_ids, bh_ids + k - ii, ii * sizeof(*bh_ids));
    for (; ii < k; ii++) {
        bh_val[ii] = INFINITY;
        bh_ids[ii] = -1;
    }
}

/* HNSW::MinimaxHeap [upstream faiss/impl/HNSW.{h,cpp}] */
typedef struct {
    int n, k, nvalid;
    int32_t *ids;
    float *dis;
} minimax_t;

static void mm_push(minimax_t *h, int32_t i, float v)
{
    if (h->k == h->n) {
        if (v >= h->dis[0]) {
            t_reject++;
            return;
        }
        t_pop++;
        if (h->ids[0] != -1)
            --h->nvalid;
        heap_pop_i32((size_t)h->k--, h->dis, h->ids);
    }
    heap_push_i32((size_t)++h->k, h->dis, h->ids, v, i);
    ++h->nvalid;
    t_push++;
}

/* pop_min: minimum dis among valid slots, ties -> highest slot index (the scalar version scans
 * from k-1 down with strict <; the AVX2 version tracks the rightmost min -- same result). */
static int32_t mm_pop_min(minimax_t *h, float *vmin_out)
{
    int i = h->k - 1;
    while (i >= 0) {
        if (h->ids[i] != -1)
            break;
        i--;
    }
    if (i == -1)
        return -1;
    int imin = i;
    float vmin = h->dis[i];
    i--;
    while (i >= 0) {
        if (h->ids[i] != -1 && h->dis[i] < vmin) {
            vmin = h->dis[i];
            imin = i;
        }
        i--;
    }
    if (vmin_out)
        *vmin_out = vmin;
    for (int j = 0; j < h->k; ++j) /* diagnostic: another valid slot holds the same minimum */
        if (j != imin && h->ids[j] != -1 && h->dis[j] == vmin) {
            t_tiepop++;
            break;
        }
    int32_t ret = h->ids[imin];
    h->ids[imin] = -1;
    --h->nvalid;
    return ret;
}

/* count_below: counts every slot < k (popped ones included) with dis < thresh */
static int mm_count_below(const minimax_t *h, float thresh)
{
    int n_below = 0;
    for (int i = 0; i < h->k; i++)
        if (h->dis[i] < thresh)
            n_below++;
    return n_below;
}

/* PQ code reader: faiss PQDecoder8 / PQDecoderGeneric (LSB-first bit packing). */
static inline uint32_t pq_decode(const uint8_t *code, int m, int nbits)
{
    if (nbits == 8)
        return code[m];
    uint64_t bitpos = (uint64_t)m * (uint64_t)nbits;
    uint64_t byte = bitpos >> 3;
    int shift = (int)(bitpos & 7);
    uint64_t acc = 0;
    int need = shift + nbits;
    for (int b = 0; b * 8 < need; ++b)
        acc |= (uint64_t)code[byte + b] << (8 * b);
    return (uint32_t)((acc >> shift) & ((1ull << nbits) - 1));
}

/* Sum order of one LUT entry ||x_m - c||^2 over the dsub dims (oracle_set_lut_order). faiss computes it
 * with fvec_L2sqr under FAISS_PRAGMA_IMPRECISE_LOOP, so the order is whatever the compiler's
 * vectorizer makes of it on the build host (the reference builds with -march=native, build.zig:48-57):
 *   0 (default, the GPU kernel's): sequential, mul then add, no FMA;
 *   1: 8 AVX2 lanes, lane i sums dims i, i+8, ... with FMA, then the tree (i, i+4), (i, i+2), (0, 1);
 *   2: 16 AVX-512 lanes with FMA, then the tree 16 -> 8 -> 4 -> 2 -> 1;
 *   3: 8 AVX2 lanes without FMA (mul, add), same tree as 1.
 * Orders 1-3 bound how far a faiss build on an AVX2 / AVX-512 host can move from order 0. */
static int g_lut_order = 0;
void oracle_set_lut_order(int order) { g_lut_order = order; }

static float l2_lanes(const float *x, const float *y, int d, int lanes, int fma_on)
{
    float acc[16] = {0};
    for (int j = 0; j < d; j += lanes)
        for (int i = 0; i < lanes && j + i < d; ++i) {
            float t = x[j + i] - y[j + i];
            if (fma_on)
                acc[i] = fmaf(t, t, acc[i]);
            else {
                float sq = t * t;
                acc[i] = acc[i] + sq;
            }
        }
    for (int w = lanes / 2; w >= 1; w /= 2)
        for (int i = 0; i < w; ++i)
            acc[i] = acc[i] + acc[i + w];
    return acc[0];
}

void oracle_pq_distance_table(const oracle_hnswpq_t *ix, const float *x, float *lut)
{
    const int M = ix->pq_M, ksub = ix->ksub, dsub = ix->dsub;
    for (int m = 0; m < M; ++m) {
        const float *xs = x + (size_t)m * dsub;
        for (int c = 0; c < ksub; ++c) {
            const float *cen = ix->centroids + ((size_t)m * ksub + c) * dsub;
            float acc = 0.0f;
            if (g_lut_order == 1)
                acc = l2_lanes(xs, cen, dsub, 8, 1);
            else if (g_lut_order == 2)
                acc = l2_lanes(xs, cen, dsub, 16, 1);
            else if (g_lut_order == 3)
                acc = l2_lanes(xs, cen, dsub, 8, 0);
            else
                for (int t = 0; t < dsub; ++t) {
                    float diff = xs[t] - cen[t];
                    float sq = diff * diff;
                    acc = acc + sq;
                }
            lut[(size_t)m * ksub + c] = acc;
        }
    }
}

/* distance_single_code / distance_four_codes for M < 16: sequential fp32 sum from 0 */
static inline float pq_dis(const oracle_hnswpq_t *ix, const float *lut, int64_t node)
{
    const uint8_t *code = ix->codes + (size_t)node * ix->code_size;
    float r = 0.0f;
    for (int m = 0; m < ix->pq_M; ++m)
        r = r + lut[(size_t)m * ix->ksub + pq_decode(code, m, ix->pq_nbits)];
    return r;
}

void oracle_hnsw_counters(int64_t *out6)
{
    out6[0] = g_cnt_push;
    out6[1] = g_cnt_pop;
    out6[2] = g_cnt_reject;
    out6[3] = g_cnt_result;
    out6[4] = g_cnt_tiepop;
    out6[5] = g_cnt_tieq;
}

typedef struct {
    float *lut;
    uint8_t *visited;
    uint8_t visno;
    minimax_t cand;
} hnsw_scratch_t;

/* HNSW::search + greedy_update_nearest + search_from_candidates (level 0, bounded queue,
 * check_relative_distance = true, upper_beam = 1, no IDSelector). */
static void hnsw_search_one(const oracle_hnswpq_t *ix, const float *x, int k, int efSearch, float *D, int64_t *I,
                            int32_t *ndis_out, int32_t *nhops_out, hnsw_scratch_t *s)
{
    int64_t ndis = 0, nhops = 0;
    /* HeapBlockResultHandler::SingleResultHandler::begin: heap_heapify(k) -> (+inf, -1) */
    for (int j = 0; j < k; ++j) {
        D[j] = INFINITY;
        I[j] = -1;
    }
    float threshold = D[0];

    if (ix->entry_point == -1 || ix->ntotal == 0) {
        heap_reorder_i64((size_t)k, D, I);
        *ndis_out = 0;
        *nhops_out = 0;
        return;
    }
    oracle_pq_distance_table(ix, x, s->lut); /* PQDistanceComputer::set_query */

    int32_t nearest = ix->entry_point;
    float d_nearest = pq_dis(ix, s->lut, nearest);

    for (int level = ix->max_level; level >= 1; level--) {
        /* greedy_update_nearest */
        for (;;) {
            int32_t prev_nearest = nearest;
            size_t o = ix->offsets[nearest];
            size_t begin = o + (size_t)ix->cum_nneighbor_per_level[level];
            size_t end = o + (size_t)ix->cum_nneighbor_per_level[level + 1];
            for (size_t j = begin; j < end; j++) {
                int32_t v = ix->neighbors[j];
                if (v < 0)
                    break;
                ndis += 1;
                float dis = pq_dis(ix, s->lut, v);
                if (dis < d_nearest) {
                    nearest = v;
                    d_nearest = dis;
                }
            }
            nhops += 1;
            if (nearest == prev_nearest)
                break;
        }
    }

    const int ef = efSearch > k ? efSearch : k;
    minimax_t *cand = &s->cand;
    cand->n = ef;
    cand->k = 0;
    cand->nvalid = 0;
    mm_push(cand, nearest, d_nearest);

    /* search_from_candidates(level 0) */
    for (int i = 0; i < cand->nvalid; i++) {
        int32_t v1 = cand->ids[i];
        float d = cand->dis[i];
        if (d < threshold) {
            heap_replace_top_i64((size_t)k, D, I, d, v1);
            threshold = D[0];
        }
        s->visited[v1] = s->visno;
    }

    int nstep = 0;
    const size_t deg0 = (size_t)(ix->cum_nneighbor_per_level[1] - ix->cum_nneighbor_per_level[0]);
    while (cand->nvalid > 0) {
        float d0 = 0;
        int32_t v0 = mm_pop_min(cand, &d0);
        int n_dis_below = mm_count_below(cand, d0);
        if (n_dis_below >= efSearch)
            break;
        size_t begin = ix->offsets[v0] + (size_t)ix->cum_nneighbor_per_level[0];
        size_t end = begin + deg0;
        threshold = D[0];
        for (size_t j = begin; j < end; j++) {
            int32_t v1 = ix->neighbors[j];
            if (v1 < 0)
                break;
            int vget = s->visited[v1] == s->visno;
            s->visited[v1] = s->visno;
            if (vget)
                continue;
            float dis = pq_dis(ix, s->lut, v1);
            ndis += 1;
            /* add_to_heap */
            if (dis < threshold) {
                t_result++;
                heap_replace_top_i64((size_t)k, D, I, dis, v1);
                threshold = D[0];
            }
            mm_push(cand, v1, dis);
        }
        nstep++;
    }
    nhops += nstep;

    /* VisitedTable::advance */
    s->visno++;
    if (s->visno == 250) {
        memset(s->visited, 0, (size_t)ix->ntotal);
        s->visno = 1;
    }
    /* SingleResultHandler::end -> heap_reorder */
    heap_reorder_i64((size_t)k, D, I);
    *ndis_out = (int32_t)ndis;
    *nhops_out = (int32_t)nhops;
}

int oracle_hnswpq_search(const oracle_hnswpq_t *ix, const float *x, int64_t n, int k, int efSearch, float *D,
                         int64_t *I, int32_t *ndis, int32_t *nhops, int nthreads)
{
    if (k <= 0)
        return -1;
    g_cnt_push = g_cnt_pop = g_cnt_reject = g_cnt_result = g_cnt_tiepop = g_cnt_tieq = 0;
    const int ef = efSearch > k ? efSearch : k;
#ifdef _OPENMP
    if (nthreads <= 0)
        nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads)
#endif
    {
        hnsw_scratch_t s;
        s.lut = (float *)malloc(sizeof(float) * (size_t)ix->pq_M * (size_t)ix->ksub);
        s.visited = (uint8_t *)calloc((size_t)(ix->ntotal > 0 ? ix->ntotal : 1), 1);
        s.visno = 1;
        s.cand.ids = (int32_t *)malloc(sizeof(int32_t) * (size_t)ef);
        s.cand.dis = (float *)malloc(sizeof(float) * (size_t)ef);
        t_push = t_pop = t_reject = t_result = t_tiepop = t_tieq = 0;
#ifdef _OPENMP
#pragma omp for schedule(guided)
#endif
        for (int64_t i = 0; i < n; ++i) {
            const int64_t tp0 = t_tiepop;
            hnsw_search_one(ix, x + i * ix->d, k, efSearch, D + i * k, I + i * k, ndis + i, nhops + i, &s);
            t_tieq += t_tiepop != tp0;
        }
#ifdef _OPENMP
#pragma omp critical
#endif
        {
            g_cnt_push += t_push;
            g_cnt_pop += t_pop;
            g_cnt_reject += t_reject;
            g_cnt_result += t_result;
            g_cnt_tiepop += t_tiepop;
            g_cnt_tieq += t_tieq;
        }
        free(s.lut);
        free(s.visited);
        free(s.cand.ids);
        free(s.cand.dis);
    }
    return 0;
}

/* ========================================================================================
 * L2 rerank: post_process_l2_static (src/utils/post_processor.cpp:1023-1162) -> find_sequences
 * (static, :204-336) -> batch_reranker (src/utils/reranker.cpp:98-195, k = k_clusters) ->
 * calc_l2_dist (src/utils/metrics.cpp:48-61). Candidate embeddings are rows of emb[n_ref x d].
 * ====================================================================================== */

/* calc_l2_dist as g++ -O3 -march=native builds the reference (build.zig:48-57), read off the reference's own
 * metrics.cpp compiled with -mavx2 -mfma (oracle/_ref): the loop is vectorized as vsubps + vmulps over
 * 8-float blocks (then one 4-float block) whose squares are added to `sum` one at a time in index order
 * (vaddss: an in-order reduction, no contraction); only the last <= 3 elements run as scalar
 * vfmadd231ss. mode 0: every square rounded, then added (the vector body; all of d = 128);
 * mode 1: every element fused; mode 2: the -mavx2 schedule above (fused scalar tail). */
float oracle_calc_l2_dist(const float *cand, const float *query, int64_t d, int mode)
{
    int64_t n_unfused = d;
    if (mode == 1)
        n_unfused = 0;
    else if (mode == 2) {
        const int64_t n8 = d >= 8 ? d / 8 * 8 : 0;
        n_unfused = n8 + (d - n8 >= 4 ? 4 : 0);
    }
    float sum = 0.0f;
    for (int64_t i = 0; i < d; ++i) {
        const float diff = cand[i] - query[i];
        if (i >= n_unfused)
            sum = fmaf(diff, diff, sum);
        else {
            const float sq = diff * diff;
            sum = sum + sq;
        }
    }
    return sqrtf(sum);
}

/* libstdc++ std::partial_sort with comp(a, b) := dists[a] < dists[b] (reranker.cpp:165-166) */
#define PSL_COMP(a, b) (dists[(a)] < dists[(b)])

static void psl_adjust_heap(int64_t *first, int64_t hole, int64_t len, int64_t value, const float *dists)
{
    const int64_t top = hole;
    int64_t second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (PSL_COMP(first[second], first[second - 1]))
            second--;
        first[hole] = first[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        first[hole] = first[second - 1];
        hole = second - 1;
    }
    int64_t parent = (hole - 1) / 2;
    while (hole > top && PSL_COMP(first[parent], value)) {
        first[hole] = first[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    first[hole] = value;
}

void oracle_partial_sort_asc_f32(int64_t *idx, int64_t n, int64_t k, const float *dists)
{
    if (k <= 0)
        return;
    if (k >= 2) {
        int64_t parent = (k - 2) / 2;
        for (;;) {
            psl_adjust_heap(idx, parent, k, idx[parent], dists);
            if (parent == 0)
                break;
            parent--;
        }
    }
    for (int64_t i = k; i < n; ++i)
        if (PSL_COMP(idx[i], idx[0])) {
            const int64_t v = idx[i];
            idx[i] = idx[0];
            psl_adjust_heap(idx, 0, k, v, dists);
        }
    for (int64_t last = k - 1; last > 0; --last) {
        const int64_t v = idx[last];
        idx[last] = idx[0];
        psl_adjust_heap(idx, 0, last, v, dists);
    }
}

/* find_sequences' sparse expansion of one label (size_t arithmetic, :248-258) */
static void l2_expand(uint64_t id, uint64_t s, uint64_t n, uint64_t *start, uint64_t *cnt)
{
    const uint64_t actual = id * s;
    if (actual >= n) {
        *start = 0;
        *cnt = 0;
        return;
    }
    *start = actual >= s - 1 ? actual - s + 1 : 0;
    *cnt = (actual + s < n ? actual + s : n) - *start;
}

/* Shared by the static and dynamic L2 post-processing: each query contributes its first lpq labels to one
 * expansion stream (stride > 1; positions < limit) and reranks the stream entries [q*nc, (q+1)*nc) with
 * batch_reranker(k); at stride 1 its candidates are its kk labels (each < limit).
 * Returns 0, or -(q+1) for the first query whose candidate range is invalid (a dense label >= limit,
 * or a sparse range past the expanded stream), or -(nq+1+q) for the first query with fewer than
 * k candidates. Outputs [nq x k]; status[q] = k / 0 / -1 / -4 as the device. */
static int64_t l2_rerank_common(const float *emb, int64_t limit, int64_t d, const int64_t *neighbors, int64_t nq,
                                int64_t kk, int64_t lpq, int64_t nc, const float *query_emb, int64_t stride,
                                int64_t k_clusters, int mode, float *top_dists, uint64_t *top_ids, int32_t *status)
{
    const int64_t n_ref = limit;
    /* the global expansion stream of the whole call (sparse): one entry per expanded window */
    uint64_t *stream = NULL;
    uint64_t total = 0;
    if (stride > 1) {
        for (int64_t q = 0; q < nq; ++q)
            for (int64_t j = 0; j < lpq; ++j) {
                uint64_t st, c;
                l2_expand((uint64_t)neighbors[q * kk + j], (uint64_t)stride, (uint64_t)n_ref, &st, &c);
                total += c;
            }
        stream = (uint64_t *)malloc(sizeof(uint64_t) * (total ? total : 1));
        uint64_t w = 0;
        for (int64_t q = 0; q < nq; ++q)
            for (int64_t j = 0; j < lpq; ++j) {
                uint64_t st, c;
                l2_expand((uint64_t)neighbors[q * kk + j], (uint64_t)stride, (uint64_t)n_ref, &st, &c);
                for (uint64_t t = 0; t < c; ++t)
                    stream[w++] = st + t;
            }
    }
    float *dists = (float *)malloc(sizeof(float) * (nc ? nc : 1));
    uint64_t *cand = (uint64_t *)malloc(sizeof(uint64_t) * (nc ? nc : 1));
    int64_t *idx = (int64_t *)malloc(sizeof(int64_t) * (nc ? nc : 1));
    int64_t first_invalid = -1, first_short = -1;
    for (int64_t q = 0; q < nq; ++q) {
        int ok = 1;
        for (int64_t c = 0; c < nc && ok; ++c) {
            if (stride == 1) {
                cand[c] = (uint64_t)neighbors[q * kk + c];
                ok = cand[c] < (uint64_t)n_ref;
            } else {
                const uint64_t g = (uint64_t)q * (uint64_t)nc + (uint64_t)c;
                ok = g < total;
                if (ok)
                    cand[c] = stream[g];
            }
        }
        int32_t st;
        if (!ok)
            st = -4;
        else if (nc == 0)
            st = 0;
        else if (nc < k_clusters)
            st = -1;
        else
            st = (int32_t)k_clusters;
        status[q] = st;
        if (st == -4 && first_invalid < 0)
            first_invalid = q;
        if (st == -1 && first_short < 0)
            first_short = q;
        if (st > 0) {
            for (int64_t c = 0; c < nc; ++c) {
                dists[c] = oracle_calc_l2_dist(emb + cand[c] * (uint64_t)d, query_emb + q * d, d, mode);
                idx[c] = c;
            }
            oracle_partial_sort_asc_f32(idx, nc, k_clusters, dists);
            for (int64_t j = 0; j < k_clusters; ++j) {
                top_dists[q * k_clusters + j] = dists[idx[j]];
                top_ids[q * k_clusters + j] = cand[idx[j]];
            }
        } else {
            for (int64_t j = 0; j < k_clusters; ++j) {
                top_dists[q * k_clusters + j] = -1.0f;
                top_ids[q * k_clusters + j] = ~0ull;
            }
        }
    }
    free(stream);
    free(dists);
    free(cand);
    free(idx);
    if (first_invalid >= 0)
        return -(first_invalid + 1);
    if (first_short >= 0)
        return -(nq + 1 + first_short);
    return 0;
}

/* post_process_l2_static (src/utils/post_processor.cpp:1023-1162): all kk labels, boundaries kk*stride per
 * query, batch_reranker(k = k_clusters) */
int64_t oracle_post_process_l2_static(const float *emb, int64_t n_ref, int64_t d, const int64_t *neighbors, int64_t nq,
                                      int64_t kk, const float *query_emb, int64_t stride, int64_t k_clusters,
                                      int mode, float *top_dists, uint64_t *top_ids, int32_t *status)
{
    return l2_rerank_common(emb, n_ref, d, neighbors, nq, kk, kk, stride == 1 ? kk : kk * stride, query_emb, stride,
                            k_clusters, mode, top_dists, top_ids, status);
}

/* post_process_l2_dynamic(_streaming), stride > 1 (:575-590, :617-627, :884-1010): the first min(k_clusters, kk)
 * labels, boundaries (2*stride - 1) per label, positions checked against the genome length, batch_reranker(k);
 * emb rows are the dynamic-lookup windows 0 .. glen-1 */
int64_t oracle_post_process_l2_dynamic(const float *emb, int64_t glen, int64_t d, const int64_t *neighbors,
                                       int64_t nq, int64_t kk, const float *query_emb, int64_t stride, int64_t k,
                                       int64_t k_clusters, int mode, float *top_dists, uint64_t *top_ids,
                                       int32_t *status)
{
    const int64_t lpq = k_clusters < kk ? k_clusters : kk;
    return l2_rerank_common(emb, glen, d, neighbors, nq, kk, lpq, lpq * (2 * stride - 1), query_emb, stride, k,
                            mode, top_dists, top_ids, status);
}
