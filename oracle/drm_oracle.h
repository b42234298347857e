/*
 * oracle/drm_oracle.h -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * A plain-C restatement of the reference hot path:
 *   - calc_sw_score            src/utils/metrics.cpp:10-45
 *   - sw_reranker's ordering   src/utils/reranker.cpp:3-51 (std::partial_sort, libstdc++ heap order)
 *   - post_process_sw_static   src/utils/post_processor.cpp:454-549 (+ find_sequences :204-336)
 *   - faiss IndexHNSWPQ::search, the backend behind faiss_search (src/hnswpq/search.cpp:6-56)
 *     [upstream faiss >= 1.8 semantics, restated; faiss is absent from this image, see DESIGN.md]
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library.
 * The product (deepreadmapper_amd / libdrm_hip.so) never links or calls it.
 */
#ifndef DRM_ORACLE_H
#define DRM_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- Smith-Waterman (src/utils/metrics.cpp:10-45) ---- */
int oracle_calc_sw_score(const uint8_t *seq1, int64_t len1, const uint8_t *seq2, int64_t len2);

/* Banded SW (an opt-in, non-parity mode of this implementation; the reference has only a TODO,
 * includes/utils/reranker.hpp:12): cells with |i - j| <= band, 0 outside; band <= 0 = full DP. */
int oracle_calc_sw_score_banded(const uint8_t *seq1, int64_t len1, const uint8_t *seq2, int64_t len2, int64_t band);

/* libstdc++ std::partial_sort(idx, idx+k, idx+n, [](a,b){return scores[a] > scores[b];})
 * (src/utils/reranker.cpp:35-40). idx must hold the iota sequence on entry. */
void oracle_partial_sort_desc(int64_t *idx, int64_t n, int64_t k, const int32_t *scores);

/* post_process_sw_static (src/utils/post_processor.cpp:454-549) for one batch.
 *   neighbors [nq x kk] int64 (faiss labels, -1 allowed)
 *   refs      [n_ref x ref_stride] bytes, window r is refs[r*ref_stride .. +ref_len)
 *   queries   [nq x q_stride] bytes with lengths q_len[i] (tagged "<" + read + ">")
 * Outputs per query (k each): top_scores (int32), top_ids (uint64 dense window id), counts[i] = rows
 * the reference emits for query i (k, or 0 when it has no candidate at all: reranker.cpp:10-11).
 * Unfilled rows hold score -1 / id UINT64_MAX.
 * Returns 0, or -(1 + query index) when a query has fewer than k candidates
 * (the reference throws "Not enough candidates (n < k)", src/utils/reranker.cpp:26-29),
 * or -1000000000 when k > k_clusters*2*stride (post_processor.cpp:486-489). */
int64_t oracle_post_process_sw_static(const int64_t *neighbors, int64_t nq, int64_t kk,
                                      const uint8_t *refs, int64_t n_ref, int64_t ref_len, int64_t ref_stride,
                                      const uint8_t *queries, const int32_t *q_len, int64_t q_stride,
                                      int64_t stride, int64_t k, int64_t k_clusters, int nthreads,
                                      int32_t *top_scores, uint64_t *top_ids, int32_t *counts);
/* post_process_sw_dynamic (src/utils/post_processor.cpp:357-452) over the genome string */
int64_t oracle_post_process_sw_dynamic(const int64_t *neighbors, int64_t nq, int64_t kk, const uint8_t *genome,
                                       int64_t glen, int64_t ref_len, const uint8_t *queries, const int32_t *q_len,
                                       int64_t q_stride, int64_t stride, int64_t k, int64_t k_clusters, int nthreads,
                                       int32_t *top_scores, uint64_t *top_ids, int32_t *counts);

/* the same two with the banded SW score (band <= 0: identical to the full ones) */
int64_t oracle_post_process_sw_static_banded(const int64_t *neighbors, int64_t nq, int64_t kk, const uint8_t *refs,
                                             int64_t n_ref, int64_t ref_len, int64_t ref_stride, const uint8_t *queries,
                                             const int32_t *q_len, int64_t q_stride, int64_t stride, int64_t k,
                                             int64_t k_clusters, int64_t band, int nthreads, int32_t *top_scores,
                                             uint64_t *top_ids, int32_t *counts);
int64_t oracle_post_process_sw_dynamic_banded(const int64_t *neighbors, int64_t nq, int64_t kk,
                                              const uint8_t *genome, int64_t glen, int64_t ref_len,
                                              const uint8_t *queries, const int32_t *q_len, int64_t q_stride,
                                              int64_t stride, int64_t k, int64_t k_clusters, int64_t band,
                                              int nthreads, int32_t *top_scores, uint64_t *top_ids, int32_t *counts);

/* ---- faiss IndexHNSWPQ (upstream semantics, see DESIGN.md "oracle") ---- */
typedef struct {
    int32_t d;
    int64_t ntotal;
    int32_t pq_M, pq_nbits, dsub, ksub, code_size;
    const float *centroids;            /* [pq_M][ksub][dsub] */
    const uint8_t *codes;              /* [ntotal][code_size] */
    const int32_t *levels;             /* [ntotal], level+1 */
    const uint64_t *offsets;           /* [ntotal+1] */
    const int32_t *neighbors;          /* [offsets[ntotal]] */
    const int32_t *cum_nneighbor_per_level; /* [n_cum] */
    int32_t n_cum;
    int32_t entry_point, max_level;
} oracle_hnswpq_t;

/* ProductQuantizer::compute_distance_table: lut[m*ksub + c] = sum_t (x[m*dsub+t]-C[m][c][t])^2,
 * summed t = 0..dsub-1 sequentially, products and sums rounded separately (no FMA). */
void oracle_pq_distance_table(const oracle_hnswpq_t *ix, const float *x, float *lut);
/* LUT sum order variant (0 = default sequential; 1 AVX2+FMA, 2 AVX-512+FMA, 3 AVX2 no FMA) */
void oracle_set_lut_order(int order);

/* IndexHNSW::search for n queries. D [n x k] float, I [n x k] int64, per-query ndis / nhops
 * (HNSWStats as accumulated by HNSW::search). nthreads <= 0 -> all OpenMP threads. */
int oracle_hnswpq_search(const oracle_hnswpq_t *ix, const float *x, int64_t n, int k, int efSearch,
                         float *D, int64_t *I, int32_t *ndis, int32_t *nhops, int nthreads);

/* diagnostic: {candidate pushes, pops on full heap, rejected pushes, result insertions} of the last search */
/* diagnostic op counts of the last oracle_hnswpq_search: push, pop(evict), reject, result insert,
 * pop_min calls facing an equal valid minimum, queries with at least one such pop_min */
void oracle_hnsw_counters(int64_t *out6);

/* L2 rerank: post_process_l2_static -> batch_reranker -> calc_l2_dist (see drm_oracle.c) */
float oracle_calc_l2_dist(const float *cand, const float *query, int64_t d, int mode);
void oracle_partial_sort_asc_f32(int64_t *idx, int64_t n, int64_t k, const float *dists);
int64_t oracle_post_process_l2_static(const float *emb, int64_t n_ref, int64_t d, const int64_t *neighbors, int64_t nq,
                                      int64_t kk, const float *query_emb, int64_t stride, int64_t k_clusters,
                                      int mode, float *top_dists, uint64_t *top_ids, int32_t *status);
int64_t oracle_post_process_l2_dynamic(const float *emb, int64_t glen, int64_t d, const int64_t *neighbors,
                                       int64_t nq, int64_t kk, const float *query_emb, int64_t stride, int64_t k,
                                       int64_t k_clusters, int mode, float *top_dists, uint64_t *top_ids,
                                       int32_t *status);

#ifdef __cplusplus
}
#endif
#endif
