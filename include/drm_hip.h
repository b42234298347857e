/*
 * include/drm_hip.h -- C ABI of libdrm_hip.so, the MI355X-native drop-in for DeepReadMapper's
 * query hot path (HNSW-PQ candidate search + Smith-Waterman rerank).
 *
 * Every entry point is plain C: pointers + sizes, no C++/torch types. Return value 0 = success,
 * negative = error (message via drm_last_error(), thread-local), mirroring the reference's
 * exception + "Error: ..." convention (src/main.cpp:439-448). All citations are to the reference
 * (/root/reference, hunglongtrangithub/DeepReadMapper) unless marked [faiss].
 */
#ifndef DRM_HIP_H
#define DRM_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DRM_OK 0
#define DRM_ERR_ARG (-1)       /* bad argument (std::invalid_argument / runtime_error in reference) */
#define DRM_ERR_IO (-2)        /* file missing / unreadable                                          */
#define DRM_ERR_FORMAT (-3)    /* index file not an IndexHNSWPQ we can read                          */
#define DRM_ERR_HIP (-4)       /* HIP runtime error                                                  */
#define DRM_ERR_CANDS (-5)     /* "Not enough candidates (n < k)"  src/utils/reranker.cpp:26-29      */
#define DRM_ERR_K (-6)         /* "Final k too large..."           src/utils/post_processor.cpp:486-489 */
#define DRM_ERR_UNSUPPORTED (-7)
#define DRM_ERR_INTERNAL (-8)  /* a kernel detected broken bookkeeping (e.g. a search past its hop bound)   */

/* Threading: every handle (drm_index, drm_flat_index, drm_refs) owns mutable device scratch (visited
 * bitmaps, clear lists, queue counters, rerank workspace). A handle is single-stream: its calls must be
 * serialised in stream order (one in-flight call per handle). Concurrent work on one device uses one
 * handle per stream; multi-device fan-out (drm_multi_*) keeps one handle per device. The diagnostic
 * counters (drm_*_overflows / _fallbacks) describe the handle's most recent search. */
typedef struct drm_index drm_index; /* device-resident IndexHNSWPQ */
typedef struct drm_refs drm_refs;   /* device-resident static window table (ref_seqs) */
typedef struct drm_encoder drm_encoder; /* device-resident GRU read encoder */

typedef struct {
    int32_t d;             /* vector dimension                                  */
    int64_t ntotal;        /* number of indexed vectors                         */
    int32_t pq_M;          /* PQ sub-quantizers (M_pq)                          */
    int32_t pq_nbits;      /* bits per sub-quantizer code                       */
    int32_t M_hnsw;        /* HNSW M; level-0 degree = 2*M_hnsw                 */
    int32_t max_level;     /* HNSW max_level                                    */
    int32_t entry_point;   /* HNSW entry point                                  */
    int32_t efConstruction;
    int32_t efSearch;      /* value stored in the file                          */
    int32_t metric_type;   /* 1 = METRIC_L2 (the only one the reference builds) */
    int64_t device_bytes;  /* HBM held by the index on its device              */
    int32_t device;        /* HIP device the index lives on                     */
} drm_index_info;

typedef struct {
    int64_t nq;            /* queries searched                                       */
    int64_t ndis;          /* sum of HNSWStats.ndis  [faiss hnsw_stats]               */
    int64_t nhops;         /* sum of HNSWStats.nhops                                  */
    double kernel_ms;      /* device time of the search kernel(s) (hipEvent)          */
} drm_search_stats;

/* ---------------------------------------------------------------- runtime / errors */
const char *drm_last_error(void);
int drm_version(void); /* major*10000 + minor*100 + patch */
int drm_device_count(int *n);
int drm_set_device(int device);
/* The device's shape, read at run time (hipGetDeviceProperties): compute units, peak engine clock (kHz), HBM
 * bytes, LDS bytes per CU, architecture name. bench.py prices its issue ceilings with these. */
typedef struct {
    int32_t cu_count;
    int32_t clock_khz;
    int64_t total_mem;
    int32_t lds_per_cu;
    char arch[64];
} drm_device_props;
int drm_device_get_props(int device, drm_device_props *out);
int drm_device_sync(void);
int drm_malloc(void **ptr, size_t bytes);
int drm_free(void *ptr);
int drm_memset(void *ptr, int value, size_t bytes);
int drm_memcpy_h2d(void *dst, const void *src, size_t bytes);
/* A 64-bit checksum of nbytes of device memory (8-byte aligned): the sum, mod 2^64, over the little-endian 8-byte
 * words w_i (the last one zero-padded) of splitmix64(w_i + i * 0x9E3779B97F4A7C15). Position-dependent, so rows
 * landing at the wrong offset change it; used to verify the RCCL result gather (bench.py) and the index broadcast
 * without copying the rows to the host. It reads the buffer after all device work this process enqueued before the
 * call has finished, on any stream (a device synchronisation), then runs on `stream`, which it synchronises. No
 * reference counterpart (a tool). */
int drm_device_checksum(const void *d_ptr, int64_t nbytes, uint64_t *out, void *stream);
int drm_memcpy_d2h(void *dst, const void *src, size_t bytes);
/* A measurement tool (no reference counterpart): the latency of the search's dependent row load on this device.
 * `waves` waves (one per workgroup) each walk `hops` 384-B rows -- the lean kernel's level-0 row, 12 B per lane on
 * 32 lanes -- of a footprint_bytes table of random contents, each next row chosen by the row just read; returns the
 * device time per hop in ns (hipEvent). bench.py prices its search latency floor with it. */
int drm_device_chase_latency(int device, int64_t footprint_bytes, int32_t waves, int32_t hops, double *ns_per_load);
/* The same walk loading only the first row_lines (1..3) 128-B lines of each 384-B row (10, 21 or 32 links): prices a
 * row load gated on the row's valid link count. drm_device_chase_latency is row_lines = 3. */
int drm_device_chase_rows(int device, int64_t footprint_bytes, int32_t waves, int32_t hops, int32_t row_lines,
                          double *ns_per_load);
int drm_stream_create(void **stream);
int drm_stream_destroy(void *stream);
int drm_stream_sync(void *stream);
int drm_event_create(void **ev);
int drm_event_destroy(void *ev);
int drm_event_record(void *ev, void *stream);
/* Work enqueued on `stream` after this call waits for `ev` (pipelining search and rerank on two streams). */
int drm_stream_wait_event(void *stream, void *ev);
int drm_event_elapsed_ms(void *start, void *stop, float *ms);

/* ---------------------------------------------------------------- index (search side)
 * drm_index_load replaces `faiss::read_index(index_file) + dynamic_cast<faiss::IndexHNSWPQ*>`
 * (src/main.cpp:236-237). It parses the faiss "IHNp" file [faiss impl/index_read.cpp], validates
 * it, re-lays it out for HBM (dense level-0 rows, compact upper levels) and uploads it to
 * `device`. drm_index_free replaces `delete alg_hnsw` (src/main.cpp:299). */
int drm_index_load(const char *path, int device, drm_index **out);
int drm_index_free(drm_index *index);
/* drm_index_clone: a replica of a loaded index on `device` (device-to-device copies of its buffers, over xGMI
 * between GPUs, the inline rows derived on the target), for one process driving several GPUs: the file is parsed
 * once (drm_multi_create does this). The source is not changed. */
int drm_index_clone(const drm_index *src, int device, drm_index **out);
int drm_index_get_info(const drm_index *index, drm_index_info *info);

/* drm_search replaces faiss_search(index, query_data, k, ef) (includes/hnswpq/search.hpp:18-21,
 * src/hnswpq/search.cpp:6-56), i.e. `index->hnsw.efSearch = ef; index->search(n, x, k, D, I)`.
 * Host pointers: x [n x d] f32 row-major; D [n x k] f32 and I [n x k] int64 are caller-owned and
 * filled like faiss (ascending distance, ties by id, missing slots (+inf, -1)).
 * Throws-equivalent: n == 0 -> DRM_ERR_ARG "Query data is empty" (search.cpp:16-19).
 * stats may be NULL. */
int drm_search(drm_index *index, const float *x, int64_t n, int32_t d, int32_t k, int32_t ef, float *D, int64_t *I,
               drm_search_stats *stats);

/* Same search on device-resident buffers, enqueued on `stream` (a hipStream_t, NULL = default).
 * ndis / nhops ([n] int32, may be NULL) receive the per-query HNSWStats the kernel measured: nhops always as
 * faiss counts it; ndis as faiss counts it (links never seen before) with drm_index_set_exact_stats on, else, on
 * the PQ 8x8 lean kernel, the distances the kernel computed. A query that exceeded its hop bound (broken
 * bookkeeping, never expected) reports nhops = ndis = -1; drm_search turns that into DRM_ERR_INTERNAL. */
int drm_search_device(drm_index *index, const float *d_x, int64_t n, int32_t k, int32_t ef, float *d_D,
                      int64_t *d_I, int32_t *d_ndis, int32_t *d_nhops, void *stream);
/* As drm_search_device, plus d_nhops_upper[n] (may be NULL): the greedy hops on levels >= 1
 * contained in nhops (they read M_hnsw-wide rows instead of 2*M_hnsw-wide ones). */
int drm_search_device_ex(drm_index *index, const float *d_x, int64_t n, int32_t k, int32_t ef, float *d_D,
                         int64_t *d_I, int32_t *d_ndis, int32_t *d_nhops, int32_t *d_nhops_upper, void *stream);
/* Tuning (no reference counterpart): resident search waves per CU of this index's persistent search grid
 * (0 = the default, 20: every CU's LDS holds 20 PQ lookup tables of 8 KB). Used by the occupancy scans of
 * DESIGN.md sec. 4.1. Results do not depend on it. */
int drm_index_set_search_waves(drm_index *index, int32_t waves_per_cu);
/* Statistics (no reference counterpart): on (1), ndis counts faiss's HNSWStats.ndis exactly -- the links each
 * hop finds not yet visited -- with a per-slot visited bitmap kept beside the search (the lean kernel needs none
 * for its results). Off (0, the default; DRM_SEARCH_EXACT_STATS=1 at load sets it) the lean
 * kernel reports the distances it computed. Results (D, I, nhops) do not depend on it. */
int drm_index_set_exact_stats(drm_index *index, int32_t on);
/* Safety (no reference counterpart): every search kernel bounds its loops -- a query past ntotal level-0 hops, or
 * a persistent wave past n work items, means broken search state, and ends with nhops = ndis = -1 for the query
 * and an error count instead of a hang. drm_search returns DRM_ERR_INTERNAL when the count
 * is non-zero; callers of the device entry points (drm_search_device[_ex]) read it here. Synchronizes the
 * device and resets the count. */
int drm_index_search_errors(drm_index *index, int64_t *count);

/* ---------------------------------------------------------------- fp32-L2 index (hnswlib)
 * The reference's hnswlib backend (BASELINE configs[1] "HIP L2 HNSW
 * search"): an hnswlib HierarchicalNSW<float> file searched with fp32 squared-L2 distances. */
typedef struct drm_flat_index drm_flat_index;

typedef struct {
    int32_t d;
    int64_t ntotal;
    int32_t M, maxM0, maxM; /* hnswlib M_, maxM0_ (level 0), maxM_ (levels >= 1) */
    int32_t max_level;
    uint32_t entry_point;
    int32_t efConstruction;
    int64_t device_bytes;
} drm_flat_index_info;

/* new hnswlib::HierarchicalNSW<float>(&space, index_file) (src/hnswlib_dir/test_search.cpp:33):
 * parses and validates an hnswlib saveIndex file, uploads it to `device`. */
int drm_flat_index_load(const char *path, int device, drm_flat_index **out);
int drm_flat_index_free(drm_flat_index *index);
int drm_flat_index_get_info(const drm_flat_index *index, drm_flat_index_info *info);

/* search(index, query_data, k, ef) (src/hnswlib_dir/search.cpp:7-52, includes/hnswlib_dir/search.hpp):
 * setEf(ef) then searchKnnCloserFirst(q, k) per query. x: [n][d] f32 host; outputs caller-owned
 * [n][k]: D = squared L2 ascending, labels = hnswlib labels (u64); a short result is padded with
 * (+inf, 2^64-1). Throws "Query data is empty" (-1) for n == 0 (search.cpp:20-23). */
int drm_flat_search(drm_flat_index *index, const float *x, int64_t n, int32_t d, int32_t k, int32_t ef, float *D,
                    uint64_t *labels, drm_search_stats *stats);
/* Same on device buffers, enqueued on `stream`; d_ndis/d_nhops [n] receive per-query counts,
 * d_nhops_upper [n] (may be NULL) the hops on levels >= 1 contained in nhops. */
int drm_flat_search_device(drm_flat_index *index, const float *d_x, int64_t n, int32_t k, int32_t ef, float *d_D,
                           uint64_t *d_labels, int32_t *d_ndis, int32_t *d_nhops, int32_t *d_nhops_upper,
                           void *stream);
/* Diagnostic: queries of the last search whose candidate_set outgrew the GPU heap (their outputs
 * are invalid; drm_flat_search reports it as an error). Synchronizes the device. */
int drm_flat_search_overflows(drm_flat_index *index, int64_t *count);
/* As drm_index_search_errors for the fp32 index (drm_flat_search returns DRM_ERR_INTERNAL on a non-zero count). */
int drm_flat_search_errors(drm_flat_index *index, int64_t *count);

/* ---------------------------------------------------------------- Smith-Waterman rerank */
/* Batched calc_sw_score(seq1, seq2) (includes/utils/metrics.hpp:22, src/utils/metrics.cpp:10-45):
 * pair p scores s1[off1[p] .. +len1[p]) against s2[off2[p] .. +len2[p]). Host pointers. */
int drm_sw_scores(const uint8_t *s1, const int64_t *off1, const int32_t *len1, const uint8_t *s2,
                  const int64_t *off2, const int32_t *len2, int64_t npairs, int32_t *scores);

/* The static reference window table `ref_seqs` (read_file(ref, ref_len, 1, lookup=true),
 * src/main.cpp:190): n_ref windows of ref_len bytes, window r at windows[r*row_stride]. */
int drm_refs_create(const uint8_t *windows, int64_t n_ref, int32_t ref_len, int64_t row_stride, int device,
                    drm_refs **out);
int drm_refs_free(drm_refs *refs);
/* Dynamic lookup (pipeline's use_dynamic, src/main.cpp:182-185): the genome string itself
 * (extract_FASTA_sequence, src/utils/parse_inputs.cpp:174-220 -- drm_extract_fasta_sequence) on the
 * device instead of the 2*(L - ref_len + 1)-window table: window id w is genome[w/2 ..+ ref_len),
 * reverse-complemented (comp_table) when w is odd (find_sequence, src/utils/post_processor.cpp:47-64).
 * Genomes of up to 2^31 - 1 bases. */
int drm_refs_create_genome(const uint8_t *genome, int64_t len, int32_t ref_len, int device, drm_refs **out);
int drm_refs_is_genome(const drm_refs *refs, int *is_genome);
/* extract_FASTA_sequence: the file's first line is skipped, whitespace dropped, letters upper-cased
 * and only A/C/G/T/N kept (from every later line, headers included -- the reference's behaviour).
 * Two calls: *len receives the length (out may be NULL), then out[0 .. *len) the sequence. */
int drm_extract_fasta_sequence(const char *path, uint8_t *out, int64_t *len);
/* Shape and device of a window table (any out-pointer may be NULL). */
int drm_refs_get_info(const drm_refs *refs, int64_t *n_ref, int32_t *ref_len, int *device);
/* Opt-in banded Smith-Waterman for every rerank on this handle (an extension: the reference scores the full DP and
 * leaves banding as a TODO, includes/utils/reranker.hpp:12). band 0 = the full DP, bit-exact with calc_sw_score
 * (the default); band 8, 16 or 32 = only the cells with |i - j| <= band (row i over the window, column j over the
 * query, both 0-based), a cell outside the band being 0: the score is at most the full one and equal to it when the
 * best local alignment stays inside the band (NOT parity with the reference). Other values: DRM_ERR_ARG. A new handle
 * starts at $DRM_SW_BAND (unset: 0). Banded queries are limited to 256 bytes and 7 distinct byte values (otherwise
 * the rerank fails with DRM_ERR_UNSUPPORTED). */
int drm_refs_set_sw_band(drm_refs *refs, int32_t band);
int drm_refs_get_sw_band(const drm_refs *refs, int32_t *band);

/* post_process_sw_static (src/utils/post_processor.cpp:454-549) -> find_sequences (static,
 * :204-336) -> sw_reranker (src/utils/reranker.cpp:3-51) -> calc_sw_score, for nq queries.
 *   neighbors [nq x kk] int64 faiss labels (-1 allowed), queries [nq x q_stride] bytes, q_len[nq]
 *   (the tagged "<"+read+">" strings of format_fastq, src/utils/parse_inputs.cpp:843-950).
 * Outputs [nq x k]: top_scores (SW score), top_ids (dense window id, size_t), counts[nq] (k, or 0
 * when the query had no candidate at all: reranker.cpp:10-11). Ordering among equal scores is
 * libstdc++ std::partial_sort's (reranker.cpp:38-40).
 * Errors: DRM_ERR_K (k > k_clusters*2*stride), DRM_ERR_CANDS (some query has 0 < n_cands < k;
 * *bad_query receives the first such query index when bad_query != NULL). Host pointers. */
int drm_post_process_sw_static(drm_refs *refs, const int64_t *neighbors, int64_t nq, int32_t kk,
                               const uint8_t *queries, const int32_t *q_len, int32_t q_stride, int64_t stride,
                               int32_t k, int32_t k_clusters, int32_t *top_scores, uint64_t *top_ids,
                               int32_t *counts, int64_t *bad_query);

/* Device-buffer form, enqueued on `stream`. d_status[nq] receives per-query status
 * (k or 0 = rows emitted, -1 = not enough candidates, -2 = more than 1024 candidates,
 * -3 = query longer than q_stride's SW build). Host must check d_status. */
int drm_post_process_sw_static_device(drm_refs *refs, const int64_t *d_neighbors, int64_t nq, int32_t kk,
                                      const uint8_t *d_queries, const int32_t *d_q_len, int32_t q_stride,
                                      int64_t stride, int32_t k, int32_t k_clusters, int32_t *d_top_scores,
                                      uint64_t *d_top_ids, int32_t *d_status, void *stream);

/* ---------------------------------------------------------------- L2 rerank (the reference's live path)
 * post_process_l2_static (src/utils/post_processor.cpp:1023-1162, called at src/main.cpp:330) ->
 * find_sequences (static) -> Vectorizer::vectorize of the candidate windows -> batch_reranker(k = k_clusters)
 * (src/utils/reranker.cpp:98-195) -> calc_l2_dist (src/utils/metrics.cpp:48-61).
 * drm_refs_embed fills a device table of every window's embedding with the read encoder (the reference
 * re-embeds each candidate window per run; the encoder is a deterministic function of the window, so the
 * table row is the same vector) -- n_ref x 128 f32 of HBM, synchronous on `stream`. Encoder and window
 * table must be on the same device. drm_refs_embeddings returns the table's device pointer (NULL before
 * drm_refs_embed) and its width. */
int drm_refs_embed(drm_refs *refs, drm_encoder *enc, void *stream);
int drm_refs_embeddings(drm_refs *refs, const float **d_emb, int32_t *dim);
/* neighbors [nq x kk] (every label is a candidate, as in the reference), query_emb [nq x d] f32 (the search's
 * query embeddings). Outputs [nq x k_clusters]: top_dists (sqrtf of the rounded squares summed in index order, ascending,
 * libstdc++ std::partial_sort's order among ties), top_ids (window ids), counts[nq] (k_clusters, or 0 for
 * kk == 0). stride > 1 reproduces the reference's global expansion stream (query q reranks stream entries
 * [q*kk*stride, (q+1)*kk*stride) of the whole call), so such a call must not be split into batches.
 * Errors: DRM_ERR_ARG "Invalid mapping index in expansion" (a label outside the table, or a range past the
 * stream: the reference throws or reads out of bounds), DRM_ERR_CANDS (kk*stride < k_clusters); *bad_query
 * receives the first offending query. Host pointers. */
int drm_post_process_l2_static(drm_refs *refs, const int64_t *neighbors, int64_t nq, int32_t kk,
                               const float *query_emb, int32_t d, int64_t stride, int32_t k_clusters,
                               float *top_dists, uint64_t *top_ids, int32_t *counts, int64_t *bad_query);
/* Device-buffer form on `stream`; d_status[nq]: k_clusters or 0 = rows emitted, -1 = not enough candidates,
 * -4 = invalid label / range past the stream. */
int drm_post_process_l2_static_device(drm_refs *refs, const int64_t *d_neighbors, int64_t nq, int32_t kk,
                                      const float *d_query_emb, int32_t d, int64_t stride, int32_t k_clusters,
                                      float *d_top_dists, uint64_t *d_top_ids, int32_t *d_status, void *stream);
/* post_process_l2_dynamic / post_process_l2_dynamic_streaming's rerank (src/utils/post_processor.cpp:553-750,
 * :752-1021) on a genome handle embedded with drm_refs_embed (a genome handle embeds windows [0, glen): the
 * positions the sparse expansion can reach, window w = genome[w/2 ..+ ref_len), reverse-complemented for odd
 * w). stride > 1 only -- at stride 1 the reference reranks nothing and returns the first min(k, k_clusters)
 * search neighbours with their search distances (DRM_ERR_ARG here). Each query contributes its first
 * min(k_clusters, kk) labels to one global expansion stream (positions checked against the genome length)
 * and reranks the stream entries [q*nc, (q+1)*nc), nc = min(k_clusters, kk) * (2*stride - 1), keeping k rows
 * ([nq x k] outputs). Errors as drm_post_process_l2_static, plus DRM_ERR_K (k > k_clusters*2*stride). */
int drm_post_process_l2_dynamic(drm_refs *refs, const int64_t *neighbors, int64_t nq, int32_t kk,
                                const float *query_emb, int32_t d, int64_t stride, int32_t k, int32_t k_clusters,
                                float *top_dists, uint64_t *top_ids, int32_t *counts, int64_t *bad_query);
int drm_post_process_l2_dynamic_device(drm_refs *refs, const int64_t *d_neighbors, int64_t nq, int32_t kk,
                                       const float *d_query_emb, int32_t d, int64_t stride, int32_t k,
                                       int32_t k_clusters, float *d_top_dists, uint64_t *d_top_ids, int32_t *d_status,
                                       void *stream);

/* ---------------------------------------------------------------- batch executor (exec.cpp)
 * Pinned host memory: buffers from drm_host_alloc make the executor's host <-> device copies DMA
 * transfers that overlap the kernels; ordinary (pageable) buffers work too, staged by the runtime. */
int drm_host_alloc(void **ptr, size_t bytes);
int drm_host_free(void *ptr);

/* The fused search -> SW rerank of one batch driver pass (SURVEY.md sec. 8b `drm_search_rerank`): the
 * reference's faiss_search(index, emb, k_clusters, ef) followed by post_process_sw_static(neighbors,
 * distances, ref_seqs, query_seqs, ref_len, stride, k, k_clusters) (src/main.cpp:278, :333-341), run as
 * batches streamed through the device (host->device copies, kernels and device->host copies of
 * consecutive batches overlap on two streams; batch size DRM_BATCH, default 262144 queries).
 * Host pointers throughout:
 *   x [n x d] f32 -> D [n x k_clusters] f32, I [n x k_clusters] int64 (drm_search's outputs);
 *   refs == NULL: search only (queries ... status ignored); a genome handle (drm_refs_create_genome)
 *   reranks with the dynamic lookup (post_process_sw_dynamic), a window table with the static one;
 *   else queries [n x q_stride] bytes with q_len[n] -> sw_scores / sw_ids [n x k] and status[n]
 *   (drm_post_process_sw_static_device's per-query status: k or 0 rows emitted, -1 not enough
 *   candidates, -2 / -3 candidate or length limits).
 * Errors: those of drm_search, plus DRM_ERR_K / DRM_ERR_CANDS / DRM_ERR_UNSUPPORTED as
 * drm_post_process_sw_static reports them (the outputs of the other queries are still written).
 * stats->kernel_ms is the device span of the compute stream. */
int drm_search_rerank(drm_index *index, drm_refs *refs, const float *x, int64_t n, int32_t d, int32_t k_clusters,
                      int32_t ef, const uint8_t *queries, const int32_t *q_len, int32_t q_stride, int64_t stride,
                      int32_t k, float *D, int64_t *I, int32_t *sw_scores, uint64_t *sw_ids, int32_t *status,
                      drm_search_stats *stats);

/* The same search -> SW rerank on DEVICE-resident buffers (shapes as drm_search_rerank; d_ndis, d_nhops,
 * d_nhops_upper may be NULL), enqueued on `stream`: the search, then the rerank, each with the whole chip
 * (co-scheduling them on shared CUs measured slower at C5 and was removed in round 5). The
 * outputs equal those of drm_search_device + drm_post_process_sw_static_device (or _dynamic_device for a genome
 * handle). d_status must be checked by the caller, and search errors read with drm_index_search_errors. stats
 * (may be NULL) makes the call synchronous and returns the device span and the search / rerank spans
 * (n_batches = 1; first_search_ms = search_ms, last_sw_ms = sw_ms). */
typedef struct {
    int64_t nq;
    int32_t n_batches;
    double kernel_ms;       /* device span: first search start -> last rerank end */
    double search_ms;       /* the search's span */
    double sw_ms;           /* the rerank's span */
    double first_search_ms; /* = search_ms (one batch) */
    double last_sw_ms;      /* = sw_ms (one batch) */
} drm_pipeline_stats;
int drm_search_rerank_device(drm_index *index, drm_refs *refs, const float *d_x, int64_t n, int32_t k_clusters,
                             int32_t ef, const uint8_t *d_queries, const int32_t *d_q_len, int32_t q_stride,
                             int64_t stride, int32_t k, float *d_D, int64_t *d_I, int32_t *d_ndis, int32_t *d_nhops,
                             int32_t *d_nhops_upper, int32_t *d_sw_scores, uint64_t *d_sw_ids, int32_t *d_status,
                             void *stream, drm_pipeline_stats *stats);

/* Optional: set up drm_search_rerank's streams and device buffers for a batch of n queries ahead of the
 * call (q_stride = 0: search only), and do the first-use work there (the copy engines' first DMA, the
 * search kernel's first launch), so the call itself only streams data and runs kernels. */
int drm_search_rerank_prepare(drm_index *index, int64_t n, int32_t d, int32_t k_clusters, int32_t k, int32_t q_stride);

/* ---------------------------------------------------------------- multi-GPU fan-out
 * One index replica (and window table, when windows != NULL) per entry of devices[ndev] -- the same
 * device may appear more than once. drm_multi_search_rerank splits the n queries into contiguous
 * shards [r*n/ndev, (r+1)*n/ndev), runs drm_search_rerank for shard r on devices[r] from its own host
 * thread, and writes every shard straight into the caller's outputs (same arguments and outputs as
 * drm_search_rerank; stats summed, kernel_ms the slowest shard). Outputs are byte-identical to a
 * one-device run: queries are independent (src/utils/post_processor.cpp:491). */
typedef struct drm_multi drm_multi;
int drm_multi_create(const char *index_path, const int *devices, int ndev, const uint8_t *windows, int64_t n_ref,
                     int32_t ref_len, int64_t row_stride, drm_multi **out);
/* The same with the dynamic lookup: a genome handle per device (drm_refs_create_genome). */
int drm_multi_create_genome(const char *index_path, const int *devices, int ndev, const uint8_t *genome, int64_t len,
                            int32_t ref_len, drm_multi **out);
int drm_multi_free(drm_multi *m);
int drm_multi_get_index_info(const drm_multi *m, drm_index_info *info); /* replica 0's info */
int drm_multi_search_rerank(drm_multi *m, const float *x, int64_t n, int32_t d, int32_t k_clusters, int32_t ef,
                            const uint8_t *queries, const int32_t *q_len, int32_t q_stride, int64_t stride, int32_t k,
                            float *D, int64_t *I, int32_t *sw_scores, uint64_t *sw_ids, int32_t *status,
                            drm_search_stats *stats);

/* ---------------------------------------------------------------- RCCL result gather (one process per GPU)
 * A communicator over the nranks processes of a job (rank 0 creates the id with drm_comm_unique_id and
 * hands it to the others out of band, e.g. over the job's gloo/TCP control plane).
 * drm_comm_gather_rows: rank r holds rows [r*n_total/nranks, (r+1)*n_total/nranks) of a row-major
 * [n_total x row_bytes] result in d_send (device memory); the root receives all n_total rows in d_recv
 * over RCCL point-to-point transfers (xGMI), enqueued on `stream`. */
#define DRM_COMM_ID_BYTES 128
typedef struct drm_comm drm_comm;
int drm_comm_unique_id(uint8_t *id);
int drm_comm_init(const uint8_t *id, int nranks, int rank, int device, drm_comm **out);
int drm_comm_free(drm_comm *comm);
int drm_comm_gather_rows(drm_comm *comm, const void *d_send, int64_t n_total, int64_t row_bytes, void *d_recv, int root,
                         void *stream);
/* drm_index_broadcast: the index replicated from one GPU to every rank over RCCL ("index
 * broadcast from GPU0"), in place of every rank parsing the IHNp file (drm_index_load; src/main.cpp:236-237 is
 * the load it replaces on ranks != root). Collective: every rank of `comm` calls it, on the communicator's device.
 * The root passes its loaded index in root_index (other ranks pass NULL); every other rank receives a new index in
 * *out. At the root `out` may be NULL (its index is the replica) or non-NULL for a separate copy (what a
 * one-rank job uses to exercise the receive side). The header goes first (shape, levels, entry point, kept
 * metadata, and the root's checksum of each buffer), then the PQ centroids, codes, level-0 rows and upper-level
 * lists in one grouped ncclBroadcast; each receiver checks the checksums, derives the lean kernel's inline rows
 * itself and applies its own DRM_SEARCH_* load-time knobs. An argument, allocation or checksum failure on any rank
 * fails the call on every rank (an agreement step precedes each transfer, so none is left waiting). Synchronous. */
int drm_index_broadcast(drm_comm *comm, drm_index *root_index, int root, drm_index **out);

/* post_process_sw_dynamic (src/utils/post_processor.cpp:357-452) on a genome handle: the same
 * contract as drm_post_process_sw_static, with find_sequences' dynamic candidate rules (dense: every
 * one of the first min(k_clusters, kk) ids, an out-of-genome window scoring 0 and keeping its id;
 * sparse: the expansion checked against the genome length). */
int drm_post_process_sw_dynamic(drm_refs *refs, const int64_t *neighbors, int64_t nq, int32_t kk,
                                const uint8_t *queries, const int32_t *q_len, int32_t q_stride, int64_t stride,
                                int32_t k, int32_t k_clusters, int32_t *top_scores, uint64_t *top_ids,
                                int32_t *counts, int64_t *bad_query);
int drm_post_process_sw_dynamic_device(drm_refs *refs, const int64_t *d_neighbors, int64_t nq, int32_t kk,
                                       const uint8_t *d_queries, const int32_t *d_q_len, int32_t q_stride,
                                       int64_t stride, int32_t k, int32_t k_clusters, int32_t *d_top_scores,
                                       uint64_t *d_top_ids, int32_t *d_status, void *stream);

/* ---------------------------------------------------------------- index build (hnswpq_index)
 * build_faiss_index (src/hnswpq/index.cpp:86-193): trains PQ on an evenly spaced sample of
 * sample_rate*n vectors (create_training_set :57-84, Config::Build::SAMPLE_RATE = 0.5), builds the
 * HNSW graph (M_hnsw, efConstruction) with PQ-ADC distances and writes a faiss "IHNp" file.
 * nthreads <= 0 -> all cores; nthreads == 1 gives a deterministic graph. */
int drm_build_hnswpq(const float *x, int64_t n, int32_t d, int32_t M_pq, int32_t nbits, int32_t M_hnsw,
                     int32_t efConstruction, double sample_rate, int32_t nthreads, uint64_t seed,
                     const char *index_path);

/* The same build on one GPU (builder_gpu.hip), from DEVICE-resident vectors d_x [n x d] f32 (d = 128,
 * M_pq = 8, nbits = 8): PQ trained on the host on the same sample as drm_build_hnswpq, codes and the
 * graph built on `device` (batched insertion, ef = min(efConstruction, 256) beams, closest-first
 * neighbour selection), written as the same faiss "IHNp" file. For the 10M-50M synthetic configurations
 * (BASELINE.json configs[3..4]) that the host builder cannot produce inside a run. */
int drm_build_hnswpq_device(const float *d_x, int64_t n, int32_t d, int32_t M_pq, int32_t nbits, int32_t M_hnsw,
                            int32_t efConstruction, double sample_rate, uint64_t seed, int device,
                            const char *index_path);

/* build_index (src/hnswlib_dir/index.cpp:3-49): hnswlib HierarchicalNSW<float>(L2Space(d), n, M,
 * efConstruction), addPoint(x[i], label i) for all i, saveIndex -> an hnswlib file (the reference's
 * defaults: M = Config::Build::GPH_DEG = 64, EFC = 128, includes/utils/config.hpp:30-31). The graph
 * follows hnswlib's construction algorithm; it need not equal hnswlib's bit for bit. */
int drm_build_hnsw_flat(const float *x, int64_t n, int32_t d, int32_t M, int32_t efConstruction, int32_t nthreads,
                        uint64_t seed, const char *index_path);

/* ---------------------------------------------------------------- synthetic embedder
 * Stand-in for the OpenVINO read encoder (Vectorizer::vectorize, src/inference/vectorize.cpp:34-141,
 * OUT OF SCOPE): e(s) = normalize(sum_t R[3-mer(s, t)]) over ACGT 3-mers, R a [64 x dim] N(0,1)
 * matrix drawn from splitmix64(seed). Deterministic; used by the CLIs and the synthetic workloads so
 * that reads land near their source windows. seqs: n strings at seqs[off[i] .. +len[i]). */
int drm_embed_kmer3(const uint8_t *seqs, const int64_t *off, const int32_t *len, int64_t n, int32_t dim,
                    uint64_t seed, float *out);

/* drm_embed_kmer3 on the device for n fixed-length rows (d_rows[i * row_stride .. + len), len <= 512,
 * dim = 128), enqueued on `stream` and synchronised; bit-identical to drm_embed_kmer3. */
int drm_embed_kmer3_device(const uint8_t *d_rows, int64_t n, int32_t len, int64_t row_stride, int32_t dim,
                           uint64_t seed, float *d_out, void *stream);

/* ---------------------------------------------------------------------------------------------
 * Read encoder: Vectorizer (src/inference/vectorize.cpp:4-141) =
 * Preprocessor::preprocess tokens (src/inference/preprocess.cpp:20-42) + the OpenVINO GRU model
 * (src/inference/fast_model.cpp:3-68, models/finetuned_sgn33-new-a-Apr6.xml) on the GPU.
 * -------------------------------------------------------------------------------------------*/
typedef struct {
    int32_t hidden, emb_dim, max_len, out_dim; /* 64, 64, 123 (config.hpp:21), 128 (config.hpp:22) */
    int32_t n_token_rows;                     /* 97: padding + the 96 _Tok2Index tokens */
    int32_t device;
    float h0;
    int64_t device_bytes;
} drm_encoder_info;

/* model_path: the reference's IR (.xml; weights from the sibling .bin, as core.read_model does,
 * fast_model.cpp:15) or a .drmenc file written by drm_encoder_export. DRM_ERR_UNSUPPORTED for any
 * graph other than embedding -> 2 x bidirectional GRU(64, linear_before_reset) with f16 weights. */
int drm_encoder_load(const char *model_path, int device, drm_encoder **out);
int drm_encoder_export(const char *model_path, const char *out_path); /* host only */
int drm_encoder_free(drm_encoder *enc);
int drm_encoder_get_info(const drm_encoder *enc, drm_encoder_info *info);
/* Preprocessor::preprocess + prepareBatch padding: tokens [n][max_len] model-input vocabulary ids
 * (0 = padding; -1 where the reference's hashToken indexes past its 96-entry table, which is
 * undefined behaviour there). seqs: n rows of `stride` bytes, lens[i] >= 2 (DRM_ERR_ARG otherwise). */
int drm_tokenize(drm_encoder *enc, const uint8_t *seqs, const int32_t *lens, int64_t n, int64_t stride, int32_t *tokens);
/* Vectorizer::vectorize: out [n][128] f32. n_undefined (optional): tokens that hit the reference's
 * undefined table read (encoded with the padding row). */
int drm_vectorize(drm_encoder *enc, const uint8_t *seqs, const int32_t *lens, int64_t n, int64_t stride, float *out,
                  int64_t *n_undefined);
/* device buffers + stream, asynchronous; lens must be >= 2 (shorter sequences encode as padding and
 * are counted by drm_encoder_flags). Like the index handles, an encoder handle is single-stream: its
 * layer-1 workspace is reused by every call, so calls must be serialised in stream order. */
int drm_vectorize_device(drm_encoder *enc, const uint8_t *d_seqs, const int32_t *d_lens, int64_t n, int64_t stride,
                         float *d_out, void *stream);
/* counters accumulated by drm_vectorize_device since the last call (synchronises the device) */
int drm_encoder_flags(drm_encoder *enc, int64_t *n_undefined, int64_t *n_short);

#ifdef __cplusplus
}
#endif
#endif
