// deepreadmapper_amd/csrc/drm_device.h -- device-side data structures + kernel launchers.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "drm_internal.h"

#define DRM_HIP_CHECK(expr)                                                                                 \
    do {                                                                                                    \
        hipError_t _e = (expr);                                                                             \
        if (_e != hipSuccess)                                                                               \
            throw ::drm::Error(DRM_ERR_HIP, std::string(#expr) + " failed: " + hipGetErrorString(_e) + " (" + \
                                                __FILE__ + ":" + std::to_string(__LINE__) + ")");            \
    } while (0)

namespace drm {

// Large, randomly accessed device arrays (index rows and codes, visited bitmaps, window table): plain hipMalloc.
// (Physically contiguous placement, hipDeviceMallocContiguous, measured slower for the C5 search in round 3 and was
// removed in round 5) The kind names what the allocation holds.
enum BigKind { kBigIndex = 1, kBigVisited = 2, kBigWindows = 4 };
inline hipError_t malloc_big(void **p, size_t bytes, BigKind) { return hipMalloc(p, bytes); }

constexpr int kMaxLevels = 24; // HNSW levels representable in SearchArgs::cum
constexpr int64_t kTraceWords = 8 + 8 * (1 << 20); // diagnostic trace: a count, then 8-word records

// HBM image of an IndexHNSWPQ (DESIGN.md "data layout in HBM").
struct DeviceIndex {
    int device = 0;
    int32_t d = 0, pq_M = 0, pq_nbits = 0, dsub = 0, ksub = 0, code_size = 0;
    int64_t ntotal = 0;
    int32_t deg0 = 0, n_levels = 0, max_level = -1, entry_point = -1;
    int32_t cum[kMaxLevels + 1] = {};
    int32_t has_dup_links = 0; // some neighbour row lists one id twice
    // safety bounds: a query past hop_bound level-0 hops, or a persistent wave past item_bound
    // work items, ends with an error count (DRM_ERR_INTERNAL); 0 = the natural bounds (ntotal hops, n items), set
    // lower only by tests (DRM_SEARCH_HOP_BOUND, DRM_WAVE_ITEM_BOUND, read at load)
    int64_t hop_bound = 0, item_bound = 0;
    int32_t waves_per_cu = 20; // resident search waves per CU (LDS allows 20 at 8 KB of LUT each)
    int32_t waves_per_cu_load = 20; // the value set at load (DRM_SEARCH_WAVES_PER_CU or 20): what 0 restores
    int32_t exact_stats = 0;   // lean kernel: count faiss's ndis with a visited bitmap (DRM_SEARCH_EXACT_STATS)
    int32_t force_lds_kernel = 0; // use the general LDS-heap kernel (hnsw_search_lds.hip)
    uint64_t *stamps = nullptr;   // diagnostic: 8 section-cycle sums (DRM_SEARCH_STAMPS=1)
    uint32_t *trace = nullptr;    // diagnostic: host-mapped trace of a DRM_PQ_DEBUG build (DRM_SEARCH_TRACE=1)
    float *centroids = nullptr;    // [M][ksub][dsub] f32
    uint8_t *codes = nullptr;      // [ntotal][code_size]
    int32_t *nbr0 = nullptr;       // [ntotal][deg0] level-0 rows (128 B each at M_hnsw=16)
    // lean kernel's level-0 rows with the neighbours' PQ codes inline: node i's row is, per link, its id (int32) and
    // its 8-byte code (12 B per link), row_words int32 per row (384 B at M_hnsw = 16), so one dwordx3 load brings a
    // hop its links and the codes its distances need; null when the index shape has no such
    // layout (PQ != 8 x 8)
    int32_t *rows = nullptr;
    int32_t row_words = 0;
    uint2 *upper_codes = nullptr;  // the code of every upper_nbr entry (0 for -1): greedy hops fetch ids + codes together
    int32_t use_inline = 1;        // DRM_SEARCH_INLINE=0: the lean kernel reads nbr0 + codes instead
    uint32_t *upper_off = nullptr; // [ntotal] start of node's level>=1 lists in upper_nbr, ~0u if none
    int32_t *upper_nbr = nullptr;  // concatenated level>=1 lists
    int64_t upper_len = 0;
    // search workspace (per resident wave slot), grown on demand
    int32_t n_slots = 0;
    int64_t vis_words = 0;         // bitmap words per slot
    uint32_t *visited = nullptr;   // [n_slots][vis_words]
    int32_t clear_cap = 0;
    int32_t *clear_list = nullptr; // [n_slots][clear_cap]
    uint32_t *counter = nullptr;   // [0] work queue head, [3] error count (hop / item bounds)
    int32_t use_fast = 1;          // lean kernel (hnsw_pq_fast.hip) where it applies; DRM_SEARCH_FAST=0 off
    uint64_t *log = nullptr;       // [n_slots][log_cap] accepted pushes (lean kernel, k == ef)
    int32_t log_cap = 0, log_slots = 0;
    int32_t log_cap_req = 512;     // entries per slot (DRM_SEARCH_LOG_CAP; >= ef + max(ef, 64), compaction beyond)
    // the lean kernel keeps no visited table (its heap is the visited set): the bitmap above
    // is allocated only for the other kernels, or for exact_stats
    int64_t device_bytes = 0;
    HnswPqHost meta; // header fields kept for drm_index_get_info (vectors released)
};

struct SearchArgs {
    const float *x;
    int64_t n;
    int32_t d, M, nbits, ksub, dsub, code_size;
    const float *centroids;
    const uint8_t *codes;
    const int32_t *nbr0;
    int32_t deg0;
    const uint32_t *upper_off;
    const int32_t *upper_nbr;
    int32_t cum[kMaxLevels + 1];
    int32_t max_level, entry_point;
    int64_t ntotal;
    int32_t k, efSearch, ef, kpad;
    float *D;
    int64_t *I;
    int32_t *ndis;
    int32_t *nhops;
    int32_t *nhops_upper; // optional: greedy hops on levels >= 1 (for the bytes model)
    uint32_t *visited;
    int64_t vis_words;
    int32_t *clear_list;
    int32_t clear_cap;
    uint32_t *counter;     // work queue head
    uint32_t *errors;      // queries past hop_bound + waves past item_bound (drm_search: DRM_ERR_INTERNAL)
    int64_t hop_bound;     // level-0 hops per query (ntotal unless a test lowers it)
    int64_t item_bound;    // work items per wave (n unless a test lowers it)
    int32_t check_dups;
    int32_t x_aligned16; // queries 16-B aligned: float4 loads in the LUT build
    uint64_t *stamps; // diagnostic section timers (DRM_SEARCH_STAMPS=1), else null
    uint64_t *log;         // lean kernel: per-slot log of accepted MinimaxHeap pushes
    int32_t log_cap;
    const int32_t *rows;   // lean kernel, inline layout: [ntotal][row_words] ids + codes (DeviceIndex::rows)
    int32_t row_words;
    const uint2 *upper_codes; // lean kernel, inline layout: codes beside upper_nbr (DeviceIndex::upper_codes)
    int32_t exact_stats;      // lean kernel: faiss's ndis counted with `visited` (else the distances computed)
    uint32_t *trace;          // diagnostic (DRM_PQ_DEBUG builds): host-mapped records, [0] = count
};

// lean kernel (hnsw_pq_fast.hip): inline rows, PQ 8x8, level-0 degree <= 64, ef <= 128, k == ef or k <= 64
bool hnsw_pq_fast_supported(const DeviceIndex &ix, int k, int efc);
void launch_hnsw_pq_fast(const SearchArgs &a, int slots, bool stamps, hipStream_t stream);
// DeviceIndex::rows from nbr0 + codes (PQ 8 x 8, deg0 <= 64), on the device
void build_inline_rows(DeviceIndex &ix);

void reserve_search_scratch(DeviceIndex &ix);
// after a synchronised search: DRM_ERR_INTERNAL if a query of it ended on the hop bound or a wave on its item bound
// (counter[3], reset once reported)
void check_search_errors(DeviceIndex &ix);
int64_t search_hop_bound(const DeviceIndex &ix);
int64_t search_item_bound(const DeviceIndex &ix, int64_t n);
void launch_hnsw_search(DeviceIndex &ix, const float *d_x, int64_t n, int k, int ef, float *d_D, int64_t *d_I,
                        int32_t *d_ndis, int32_t *d_nhops, int32_t *d_nhops_upper, hipStream_t stream);
void launch_hnsw_search_lds(DeviceIndex &ix, const float *d_x, int64_t n, int k, int ef, float *d_D, int64_t *d_I,
                            int32_t *d_ndis, int32_t *d_nhops, int32_t *d_nhops_upper, hipStream_t stream);

// ---------------------------------------------------------------------- fp32 (hnswlib) index
// HBM image of an hnswlib HierarchicalNSW<float> (DESIGN.md "fp32 mode").
struct DeviceFlatIndex {
    int device = 0;
    int32_t d = 0, maxM0 = 0, maxM = 0, maxlevel = -1, M = 0, efc = 0;
    uint32_t ep = 0;
    int64_t ntotal = 0;
    int32_t has_dup_links = 0;
    int32_t waves_per_cu = 32;  // cap on resident search waves per CU (the kernel build sets the real one)
    int64_t hop_bound = 0, item_bound = 0; // as DeviceIndex (DRM_SEARCH_HOP_BOUND, DRM_WAVE_ITEM_BOUND)
    float *vec = nullptr;      // [ntotal][d] f32 (512-B rows at d = 128)
    uint32_t *l0 = nullptr;    // [ntotal][maxM0] level-0 links (512-B rows at maxM0 = 128)
    uint32_t *l0cnt = nullptr; // [ntotal] link counts
    int64_t *up_off = nullptr; // [ntotal] first word of the node's upper blocks, -1 if none
    uint32_t *up = nullptr;    // blocks of (1 + maxM) words: count, links
    uint64_t *labels = nullptr;
    // search workspace (per resident wave slot), grown on demand
    int32_t n_slots = 0;
    int64_t vis_words = 0;
    uint32_t *visited = nullptr;
    int32_t clear_cap = 0;
    int32_t *clear_list = nullptr;
    int64_t cand_ovf_cap = 0;       // candidate_set entries beyond the LDS part, per slot
    float *cand_ovf_k = nullptr;
    uint32_t *cand_ovf_i = nullptr;
    int64_t top_ovf_cap = 0;        // top_candidates entries beyond the LDS part (large ef), per slot
    float *top_ovf_k = nullptr;
    uint32_t *top_ovf_i = nullptr;
    uint32_t *counter = nullptr;    // [0] queue head, [1] candidate_set overflows, [3] error count (bounds)
    uint64_t *stamps = nullptr;     // diagnostic: 8 section-cycle sums (DRM_SEARCH_STAMPS=1)
    int64_t device_bytes = 0;
    HnswFlatHost meta;              // header fields for drm_flat_index_get_info (arrays released)
};

struct FlatArgs {
    const float *x;
    int64_t n;
    int32_t d;
    const float *vec;
    const uint32_t *l0;
    const uint32_t *l0cnt;
    int32_t maxM0;
    const int64_t *up_off;
    const uint32_t *up;
    int32_t maxM, maxlevel;
    uint32_t ep;
    int64_t ntotal;
    const uint64_t *labels;
    int32_t k, ef;
    float *D;
    uint64_t *L;
    int32_t *ndis, *nhops;
    int32_t *nhops_upper; // optional: greedy hops on levels >= 1 (for the bytes model)
    uint32_t *visited;
    int64_t vis_words;
    int32_t *clear_list;
    int32_t clear_cap;
    uint32_t *counter;     // work queue head
    uint32_t *errors;      // queries past hop_bound + waves past item_bound (drm_flat_search: DRM_ERR_INTERNAL)
    int64_t hop_bound, item_bound;
    int32_t check_dups;
    int32_t cand_lds;
    float *cand_ovf_k;
    uint32_t *cand_ovf_i;
    int64_t cand_ovf_cap;
    int32_t top_lds;
    float *top_ovf_k;
    uint32_t *top_ovf_i;
    int64_t top_ovf_cap;
    uint64_t *stamps;     // diagnostic section timers (DRM_SEARCH_STAMPS=1)
    uint32_t *overflow;   // candidate_set overflow count (counter[1])
};

void launch_hnsw_flat_search(DeviceFlatIndex &ix, const float *d_x, int64_t n, int k, int ef, float *d_D,
                             uint64_t *d_L, int32_t *d_ndis, int32_t *d_nhops, int32_t *d_nhops_upper,
                             hipStream_t stream);

// ---------------------------------------------------------------------------------- SW rerank
struct DeviceRefs {
    int device = 0;
    uint8_t *windows = nullptr; // [n_ref][row_stride], row_stride % 16 == 0
    int64_t n_ref = 0;
    int32_t ref_len = 0;
    int64_t row_stride = 0;
    // rerank workspace (grown on demand): candidate ids / SW scores / candidate counts per query
    uint64_t *ws_ids = nullptr;
    int32_t *ws_scores = nullptr;
    int32_t *ws_ncand = nullptr;
    size_t ws_elems = 0, ws_nq = 0;
    // dynamic lookup (use_dynamic, post_process_sw_dynamic): the genome string instead of a window
    // table; window id w is genome[w / 2 ..+ ref_len), reverse-complemented when w is odd
    uint8_t *genome = nullptr;
    int64_t glen = 0;
    // L2 rerank (post_process_l2_*): the read encoder's embedding of every window, [emb_rows][emb_dim] f32,
    // filled once by drm_refs_embed (l2_rerank.hip); emb_rows = n_ref, or glen for a genome handle
    float *emb = nullptr;
    int32_t emb_dim = 0;
    int64_t emb_rows = 0;
    // opt-in banded SW (drm_refs_set_sw_band): 0 = the full DP of the reference (default), else the band half-width
    int32_t sw_band = 0;
};

struct RerankArgs {
    const uint8_t *refs;
    int64_t n_ref;
    int32_t ref_len;
    int64_t row_stride;
    const int64_t *neighbors;
    int32_t kk, k_clusters;
    int64_t stride;
    const uint8_t *queries;
    const int32_t *q_len;
    int32_t q_stride;
    int32_t k;
    int64_t nq;
    int32_t *top_scores;
    uint64_t *top_ids;
    int32_t *status;
    // dynamic lookup (post_process_sw_dynamic): genome != nullptr replaces the window table
    const uint8_t *genome;
    int64_t glen;
    // workspace (set by launch_sw_rerank)
    int32_t cmax;
    uint64_t *cand_ids;
    int32_t *cand_scores;
    int32_t *ncand;
};

constexpr int kMaxCands = 1024; // candidates per query kept in LDS

void launch_sw_rerank(DeviceRefs &refs, RerankArgs a, int max_qlen, hipStream_t stream);

// generic batched calc_sw_score: one wave per pair
void launch_sw_pairs(const uint8_t *d_s1, const int64_t *d_off1, const int32_t *d_len1, const uint8_t *d_s2,
                     const int64_t *d_off2, const int32_t *d_len2, int64_t npairs, int32_t *d_scores, int max_len2,
                     hipStream_t stream);

// L2 rerank (post_process_l2_static -> batch_reranker, src/utils/post_processor.cpp:1023-1162,
// src/utils/reranker.cpp:98-195): distances from the window embedding table, libstdc++ partial_sort
struct L2Args {
    const float *emb;          // [limit][d] window embeddings (row = window id)
    int64_t limit;             // ids / expanded positions must be < limit: n_ref, or the genome length (dynamic)
    int32_t d;
    const int64_t *neighbors;  // [nq][kk]
    int32_t kk;
    int32_t lpq;               // labels used per query: kk (static), min(k_clusters, kk) (dynamic sparse)
    int32_t nc;                // candidates per query: kk at stride 1, else the boundary width of the caller
    int64_t stride;
    const float *query_emb;    // [nq][d]
    int32_t k;                 // rows kept per query (batch_reranker's k)
    int64_t nq;
    float *top_dists;          // [nq][k]
    uint64_t *top_ids;         // [nq][k]
    int32_t *status;           // [nq]
};
void launch_l2_rerank(DeviceRefs &refs, L2Args a, hipStream_t stream);
// genome windows w in [0, n) as rows of ref_len bytes (w / 2 .. + ref_len, reverse-complemented when w is odd;
// lens[w] = 0 past the genome end), the input of the encoder for a genome handle's embedding table
void launch_genome_rows(const DeviceRefs &refs, int64_t w0, int64_t n, uint8_t *rows, int64_t row_stride,
                        int32_t *lens, hipStream_t stream);

// ---------------------------------------------------------------------------------- read encoder
// HBM image of the GRU read encoder (encoder_gru.hip)
struct DeviceEncoder {
    int device = 0;
    float h0 = 0.f;
    uint16_t *emb = nullptr;   // [97][64] f16: row 0 = padding id 0, row 1 + h = _Tok2Index[h]
    uint16_t *vocab = nullptr; // [97] vocabulary id per row (drm_tokenize output)
    uint16_t *W[2] = {}, *R[2] = {}; // f16 [2 dirs][192][in], [2][192][64] (gate order z, r, n)
    float *B[2] = {};          // [2][256] f32: b_z, b_r, Wb_n, Rb_n
    uint16_t *y1 = nullptr;    // layer-1 outputs of the tiles in flight (hi/lo f16), grown on demand
    int64_t y1_tiles = 0;
    // 32 reads each; 2 MB of layer-1 output per tile (DRM_ENC_TILES). 3,072: 79.2 -> 78.4 ms at C5 against 2,048;
    // chunks of whole workgroup rounds (1,920 / 2,304) measured no different (profiles/r06/ab_enc_tiles.txt)
    int64_t max_tiles_per_launch = 3072;
    uint32_t *flags = nullptr; // [0] tokens past _Tok2Index, [1] sequences shorter than 2 bytes
    int64_t device_bytes = 0;
};
int64_t encoder_tile_bytes();
void encoder_upload(DeviceEncoder &d, const EncoderHost &h, int device);
void encoder_release(DeviceEncoder &d);
void launch_encode(DeviceEncoder &d, const uint8_t *d_seqs, const int32_t *d_lens, int64_t n, int64_t stride,
                   float *d_out, hipStream_t stream);
void launch_tokenize(const DeviceEncoder &d, const uint8_t *d_seqs, const int32_t *d_lens, int64_t n, int64_t stride,
                     int32_t *d_tokens, hipStream_t stream);

} // namespace drm

#if defined(__HIP__)
namespace drm {
// The wave's next item from a persistent kernel's atomic work queue (counter[0]). Every lane executes the atomic
// (lane 0 adds 1, the others 0) and the wave takes lane 0's old value: no branch on the lane id sits in front of the
// readfirstlane. With the usual `if (lane == 0) q = atomicAdd(..)` a search kernel whose loop body also ends in
// `if (lane == 0)` stores was compiled into two loops split on the lane id (lane 0 left to fetch the next item,
// lanes 1..63 looped back with q = 0 and re-ran item 0 forever): a hang, seen in round 4.
__device__ __forceinline__ int wave_next_item(uint32_t *counter, int lane)
{
    const uint32_t old = __hip_atomic_fetch_add(counter, lane == 0 ? 1u : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return __builtin_amdgcn_readfirstlane((int)old);
}
} // namespace drm
#endif
