// deepreadmapper_amd/csrc/builder_gpu.hip -- IndexHNSWPQ construction on one MI355X (SURVEY.md sec. 8f
// row 2), writing the same faiss "IHNp" file as the host builder (builder.cpp) and `hnswpq_index`
// (build_faiss_index, src/hnswpq/index.cpp:86-193). faiss is absent and build parity with it is not
// required: what must hold is a valid HNSW graph over PQ codes in faiss's layout,
// which drm_index_load validates and the search parity tests then use.
//
// Pipeline:
//   1. PQ training on the host, on create_training_set's sample (pq_training_rows / pq_train_subspaces,
//      the same code and sample as the host builder); the sample rows are gathered on the device;
//   2. PQ encoding on the device (one thread per vector and sub-quantizer, codebook slice in LDS; the
//      host encoder's op order, so codes are identical);
//   3. levels from the host builder's random_level (hnsw_assign_levels), insertion order = level
//      descending, shuffled within a level (hnsw_add_vertices); the first node is the entry point;
//   4. batched insertion, batch b = order[2^b, 2^(b+1)) capped at kMaxBatch: one wave per new node
//      builds its PQ LUT, descends greedily through the levels above its own, and on each of its levels
//      runs an ef-bounded best-first beam (efConstruction, <= 256 in registers) over the nodes already
//      inserted (ADC distances, per-slot visited bitmap as in the search kernel); it links to the
//      candidates the neighbour heuristic keeps (below). A second kernel adds the reverse links: each target list keeps
//      its degree-many closest entries (one 64-bit CAS on the (distance, id) pair that is the current
//      maximum; retried on conflict). Neighbours of one batch do not see each other; the growing
//      batches keep that effect small, as in other batched GPU HNSW builders;
//   5. lists sorted by distance, packed into faiss's offsets/neighbors layout, file written on the host.
// Forward links follow faiss's shrink_neighbor_list heuristic with symmetric PQ distances (sdc_table),
// applied to the 64 nearest candidates (faiss scans all efC); reverse links keep the closest entries
// instead of re-running the heuristic on the target's list. The graph is therefore not faiss's graph;
// the file format, levels, entry point and PQ are.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "drm_device.h"
#include "pq_common.h"

#pragma clang fp contract(off)

namespace drm {
namespace {

constexpr int64_t kMaxBatch = 1 << 21;

__device__ __forceinline__ uint64_t bballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ uint64_t bpack(uint32_t key, int32_t id) { return ((uint64_t)key << 32) | (uint32_t)id; }
__device__ __forceinline__ int32_t bid(uint64_t e) { return e == ~0ull ? -1 : (int32_t)(uint32_t)e; }

// ------------------------------------------------------------------ PQ encode (ProductQuantizer::compute_codes)
// grid (ceil(n / 256), M), 256 threads: thread = vector, blockIdx.y = sub-quantizer, its codebook in LDS.
template <int dsub>
__global__ __launch_bounds__(256) void pq_encode_kernel(const float *x, int64_t n, int d, const float *centroids,
                                                         uint8_t *codes, int M)
{
    extern __shared__ float cb[]; // [256][dsub]
    const int m = blockIdx.y;
    for (int e = threadIdx.x; e < 256 * dsub; e += 256)
        cb[e] = centroids[(size_t)m * 256 * dsub + e];
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n)
        return;
    float xs[dsub];
#pragma unroll
    for (int t = 0; t < dsub; ++t)
        xs[t] = x[i * d + (int64_t)m * dsub + t];
    int best = 0;
    float bd = INFINITY;
    for (int c = 0; c < 256; ++c) {
        float acc = 0.0f;
#pragma unroll
        for (int t = 0; t < dsub; ++t) {
            const float df = __fsub_rn(xs[t], cb[c * dsub + t]);
            acc = __fadd_rn(acc, __fmul_rn(df, df));
        }
        if (acc < bd) {
            bd = acc;
            best = c;
        }
    }
    codes[i * M + m] = (uint8_t)best;
}

__global__ void gather_rows_kernel(const float *x, const int64_t *idx, int64_t m, int d, float *out)
{
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m * d; e += (int64_t)gridDim.x * blockDim.x)
        out[e] = x[idx[e / d] * d + e % d];
}

struct BuildArgs {
    const float *x;
    int32_t d;
    const float *centroids;
    const uint8_t *codes;
    const float *sdc;    // [M][256][256] symmetric sub-distances (PQ sdc_table)
    uint64_t *link0;     // [n][deg0] packed (ord32(dist) << 32 | id), ~0 = empty
    uint64_t *linkU;     // level l >= 1 list of node i at uoff[i] + (l - 1) * degU
    const int64_t *uoff; // [n], -1 for level-0-only nodes
    const int32_t *levels;
    int32_t deg0, degU;
    int32_t entry_point, max_level;
    const int32_t *order;
    int64_t start, count;
    int32_t ef;
    uint32_t *visited;
    int64_t vis_words;
    int32_t *clear_list;
    int32_t clear_cap;
    uint32_t *counter;
    uint32_t *errors;            // waves past item_bound + beams past hop_bound: the build fails (DRM_ERR_INTERNAL)
    int64_t item_bound, hop_bound; // count (a batch's nodes) and n (each node is expanded once) unless a test lowers them
};

__device__ __forceinline__ uint32_t adc8(const float *lut, const uint8_t *codes, int32_t v)
{
    const uint2 c8 = *reinterpret_cast<const uint2 *>(codes + (size_t)v * 8);
    float r = 0.0f;
#pragma unroll
    for (int m = 0; m < 4; ++m)
        r = __fadd_rn(r, lut[m * 256 + ((c8.x >> (8 * m)) & 255u)]);
#pragma unroll
    for (int m = 0; m < 4; ++m)
        r = __fadd_rn(r, lut[(m + 4) * 256 + ((c8.y >> (8 * m)) & 255u)]);
    return ord32(r);
}

__device__ __forceinline__ const uint64_t *list_at(const BuildArgs &a, int32_t v, int l)
{
    return l == 0 ? a.link0 + (size_t)v * a.deg0 : a.linkU + a.uoff[v] + (int64_t)(l - 1) * a.degU;
}

// One wave per new node: greedy descent, then an ef-bounded beam on each of the node's levels, and the
// closest deg candidates become its forward links. W = sorted register array (slot s: lane s & 63,
// register s >> 6), bit 0 of `ex[r]` marks an expanded entry.
template <int R>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void hnsw_build_insert_kernel(BuildArgs a)
{
    extern __shared__ __align__(16) float lut[];
    const int lane = lane_id();
    uint32_t *vis = a.visited + (size_t)blockIdx.x * (size_t)a.vis_words;
    int32_t *clr = a.clear_list + (size_t)blockIdx.x * (size_t)a.clear_cap;
    int64_t taken = 0;
    for (;;) {
        const int qi = wave_next_item(a.counter, lane);
        if ((int64_t)qi >= a.count)
            break;
        if (++taken > a.item_bound) { // more items than the batch holds: a broken work-queue fetch
            if (lane == 0)
                atomicAdd(a.errors, 1u);
            break;
        }
        const int32_t u = a.order[a.start + qi];
        build_lut_m8_ptr<1>(a.x + (size_t)u * a.d, a.centroids, lut, lane);
        const int ul = a.levels[u];
        int32_t cur = a.entry_point;
        uint32_t dcur = __builtin_amdgcn_readfirstlane(adc8(lut, a.codes, cur));
        // greedy_update_nearest on the levels above the node's own
        for (int l = a.max_level; l > ul; --l) {
            for (;;) {
                const uint64_t e = lane < a.degU ? list_at(a, cur, l)[lane] : ~0ull;
                const int32_t v = bid(e);
                uint32_t dk = v >= 0 ? adc8(lut, a.codes, v) : 0xFFFFFFFFu;
                const uint32_t mn = wave_min_u32(dk);
                if (mn >= dcur)
                    break;
                dcur = mn;
                cur = __builtin_amdgcn_readlane(v, __builtin_ctzll(bballot(dk == mn)));
            }
        }
        for (int l = min(ul, a.max_level); l >= 0; --l) {
            const int deg = l == 0 ? a.deg0 : a.degU;
            uint64_t W[R];
            bool ex[R];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                W[r] = ~0ull;
                ex[r] = false;
            }
            if (lane == 0)
                W[0] = bpack(dcur, cur);
            int nw = 1, clear_n = 1;
            int64_t hops = 0;
            if (lane == 0) {
                atomicOr(&vis[cur >> 5], 1u << (cur & 31));
                clr[0] = cur;
            }
            for (;;) {
                if (++hops > a.hop_bound) { // every node is expanded at most once: the beam's state is broken
                    if (lane == 0)
                        atomicAdd(a.errors, 1u);
                    break;
                }
                // the nearest unexpanded entry (W is sorted: the first one)
                int s = -1;
#pragma unroll
                for (int r = R - 1; r >= 0; --r) {
                    const uint64_t m = bballot(W[r] != ~0ull && !ex[r]);
                    if (m)
                        s = 64 * r + __builtin_ctzll(m);
                }
                if (s < 0)
                    break;
                int32_t v = 0;
#pragma unroll
                for (int r = 0; r < R; ++r)
                    if ((s >> 6) == r) {
                        v = (int32_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)W[r], s & 63);
                        if (lane == (s & 63))
                            ex[r] = true;
                    }
                const uint64_t e = lane < deg ? list_at(a, v, l)[lane] : ~0ull;
                const int32_t w = bid(e);
                bool fresh = false;
                uint32_t dk = 0xFFFFFFFFu;
                if (w >= 0) {
                    const uint32_t bit = 1u << (w & 31);
                    fresh = (atomicOr(&vis[w >> 5], bit) & bit) == 0u;
                    if (fresh)
                        dk = adc8(lut, a.codes, w);
                }
                const uint64_t fm = bballot(fresh);
                if (fresh) {
                    const int p = clear_n + __builtin_popcountll(fm & lanes_below(lane));
                    if (p < a.clear_cap)
                        clr[p] = w;
                }
                clear_n += __builtin_popcountll(fm);
                // insert the fresh candidates that beat the current ef-th entry
                uint64_t rem = fm;
                while (rem) {
                    const int l2 = __builtin_ctzll(rem);
                    rem &= rem - 1;
                    const uint64_t val = bpack((uint32_t)__builtin_amdgcn_readlane((int)dk, l2),
                                               __builtin_amdgcn_readlane(w, l2));
                    if (nw == a.ef) {
                        const int lr = (a.ef - 1) >> 6, ll = (a.ef - 1) & 63;
                        uint64_t last = 0;
#pragma unroll
                        for (int r = 0; r < R; ++r)
                            if (r == lr)
                                last = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(W[r] >> 32), ll) << 32) |
                                       (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)W[r], ll);
                        if (val >= last)
                            continue;
                    } else {
                        ++nw;
                    }
                    int pos = 0;
#pragma unroll
                    for (int r = 0; r < R; ++r)
                        pos += __builtin_popcountll(bballot(W[r] < val));
                    // shift slots >= pos up by one (the ef-th falls off), put val at pos
                    uint64_t carryW = 0;
                    bool carryE = false;
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const uint32_t ch = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(carryW >> 32),
                                                                                  (int)(uint32_t)(W[r] >> 32), 0x138,
                                                                                  0xF, 0xF, false);
                        const uint32_t cl = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)carryW,
                                                                                  (int)(uint32_t)W[r], 0x138, 0xF, 0xF,
                                                                                  false);
                        const int ce = __builtin_amdgcn_update_dpp((int)carryE, (int)ex[r], 0x138, 0xF, 0xF, false);
                        const uint64_t nextW = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(W[r] >> 32), 63)
                                                << 32) |
                                               (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)W[r], 63);
                        const bool nextE = __builtin_amdgcn_readlane((int)ex[r], 63) != 0;
                        const int sidx = 64 * r + lane;
                        const uint64_t shW = ((uint64_t)ch << 32) | cl;
                        if (sidx > pos) {
                            W[r] = shW;
                            ex[r] = ce != 0;
                        } else if (sidx == pos) {
                            W[r] = val;
                            ex[r] = false;
                        }
                        carryW = nextW;
                        carryE = nextE;
                    }
#pragma unroll
                    for (int r = 0; r < R; ++r)
                        if (64 * r + lane >= a.ef)
                            W[r] = ~0ull;
                }
            }
            // HNSW::shrink_neighbor_list over the 64 nearest candidates: candidate c (lane c, in distance
            // order) is kept unless an already kept k is closer to it than the new node is
            // (symmetric PQ distance sdc(k, c) < d(q, c)); at most deg are kept.
            const bool has = W[0] != ~0ull;
            const int32_t cid = has ? (int32_t)(uint32_t)W[0] : 0;
            const uint2 cc = has ? *reinterpret_cast<const uint2 *>(a.codes + (size_t)cid * 8) : make_uint2(0u, 0u);
            const float dq = unord32((uint32_t)(W[0] >> 32));
            const int T = __builtin_popcountll(bballot(has));
            uint64_t dom = 0;
#pragma unroll 4
            for (int k = 0; k + 1 < T; ++k) {
                const uint32_t kx = (uint32_t)__builtin_amdgcn_readlane((int)cc.x, k);
                const uint32_t ky = (uint32_t)__builtin_amdgcn_readlane((int)cc.y, k);
                if (k < lane && has) {
                    float sd = 0.0f;
#pragma unroll
                    for (int m = 0; m < 4; ++m)
                        sd = __fadd_rn(sd, a.sdc[((m * 256 + ((kx >> (8 * m)) & 255u)) << 8) + ((cc.x >> (8 * m)) & 255u)]);
#pragma unroll
                    for (int m = 0; m < 4; ++m)
                        sd = __fadd_rn(sd, a.sdc[(((m + 4) * 256 + ((ky >> (8 * m)) & 255u)) << 8) +
                                                 ((cc.y >> (8 * m)) & 255u)]);
                    if (sd < dq)
                        dom |= 1ull << k;
                }
            }
            uint64_t kept = 0;
            int nk = 0;
            for (int c = 0; c < T && nk < deg; ++c) {
                const uint64_t dc = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(dom >> 32), c) << 32) |
                                    (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)dom, c);
                if ((dc & kept) == 0) {
                    kept |= 1ull << c;
                    ++nk;
                }
            }
            // forward links: the kept candidates in distance order, then empty slots
            uint64_t *mine = l == 0 ? a.link0 + (size_t)u * a.deg0 : a.linkU + a.uoff[u] + (int64_t)(l - 1) * a.degU;
            if ((kept >> lane) & 1ull)
                mine[__builtin_popcountll(kept & lanes_below(lane))] = W[0];
            if (lane >= nk && lane < deg)
                mine[lane] = ~0ull;
            // the next level starts from the nearest candidate found here
            cur = (int32_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)W[0], 0);
            dcur = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(W[0] >> 32), 0);
            // VisitedTable::advance
            if (clear_n <= a.clear_cap) {
                for (int t = lane; t < clear_n; t += 64)
                    vis[clr[t] >> 5] = 0u;
            } else {
                for (int64_t t = lane; t < a.vis_words; t += 64)
                    vis[t] = 0u;
            }
            __builtin_amdgcn_s_waitcnt(0);
        }
        __syncthreads();
    }
}

// Reverse links of one batch: thread = (new node, level, slot). The target keeps its deg closest
// entries: replace the current maximum (lowest slot among equal maxima, so valid entries stay a
// prefix) by one 64-bit CAS, retried when another thread changed the list in between.
__global__ void hnsw_build_reverse_kernel(BuildArgs a, int level)
{
    const int deg = level == 0 ? a.deg0 : a.degU;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.count * deg)
        return;
    const int32_t u = a.order[a.start + t / deg];
    if (a.levels[u] < level)
        return;
    const uint64_t e = list_at(a, u, level)[t % deg];
    const int32_t v = bid(e);
    if (v < 0)
        return;
    const uint64_t nv = bpack((uint32_t)(e >> 32), u);
    uint64_t *lst = const_cast<uint64_t *>(list_at(a, v, level));
    for (int attempt = 0; attempt < 1024; ++attempt) {
        uint64_t mx = 0;
        int ms = 0;
        for (int j = 0; j < deg; ++j) {
            const uint64_t x = __hip_atomic_load(lst + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((uint32_t)x == (uint32_t)u && x != ~0ull)
                return; // already linked
            if (x > mx) {
                mx = x;
                ms = j;
            }
        }
        if (nv >= mx)
            return;
        uint64_t expect = mx;
        if (__hip_atomic_compare_exchange_strong(lst + ms, &expect, nv, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT))
            return;
    }
}

// Final pass: every list sorted by (distance, id), ids unpacked (-1 padding at the end). One thread per
// list, insertion sort in its own LDS row (deg <= 64).
__global__ __launch_bounds__(64) void hnsw_build_finish_kernel(const uint64_t *links, int64_t nlists, int deg,
                                                                int32_t *out)
{
    __shared__ uint64_t rows[64 * 64];
    const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (i >= nlists)
        return;
    uint64_t *v = rows + threadIdx.x * 64;
    for (int j = 0; j < deg; ++j)
        v[j] = links[i * deg + j];
    for (int j = 1; j < deg; ++j) {
        const uint64_t x = v[j];
        int k = j - 1;
        while (k >= 0 && v[k] > x) {
            v[k + 1] = v[k];
            --k;
        }
        v[k + 1] = x;
    }
    for (int j = 0; j < deg; ++j)
        out[i * deg + j] = bid(v[j]);
}

template <typename T> struct DevArr {
    T *p = nullptr;
    explicit DevArr(size_t n) { DRM_HIP_CHECK(hipMalloc(&p, sizeof(T) * std::max<size_t>(n, 1))); }
    ~DevArr()
    {
        if (p)
            (void)hipFree(p);
    }
    DevArr(const DevArr &) = delete;
};

double secs_since(std::chrono::steady_clock::time_point t0)
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

} // namespace

void build_hnswpq_gpu(const float *d_x, int64_t n, int d, int M_pq, int nbits, int M_hnsw, int efc,
                      double sample_rate, uint64_t seed, int device, const std::string &path)
{
    if (n <= 0)
        throw Error(DRM_ERR_ARG, "Input data is empty");
    if (d != 128 || M_pq != 8 || nbits != 8)
        throw Error(DRM_ERR_UNSUPPORTED, "the GPU builder supports d = 128, M_pq = 8, nbits = 8 (the reference's "
                                         "configuration); use the host builder for other shapes");
    if (M_hnsw < 2 || 2 * M_hnsw > 64 || efc < 1)
        throw Error(DRM_ERR_ARG, "invalid build parameters (M_hnsw in [2, 32], efConstruction >= 1)");
    if (n >= ((int64_t)1 << 31))
        throw Error(DRM_ERR_UNSUPPORTED, "more than 2^31-1 vectors");
    const bool verbose = std::getenv("DRM_BUILD_VERBOSE") && std::atoi(std::getenv("DRM_BUILD_VERBOSE"));
    auto t0 = std::chrono::steady_clock::now();
    DRM_HIP_CHECK(hipSetDevice(device));
    const int ksub = 256, dsub = d / M_pq;

    HnswPqHost ix;
    ix.hdr.d = d;
    ix.hdr.ntotal = n;
    ix.storage_hdr = ix.hdr;
    ix.pq_d = (uint64_t)d;
    ix.pq_M = (uint64_t)M_pq;
    ix.pq_nbits = (uint64_t)nbits;
    ix.centroids.resize((size_t)d * ksub);
    // 1. PQ training on the host builder's sample
    {
        const std::vector<size_t> rows = pq_training_rows(n, sample_rate, ksub, seed);
        std::vector<int64_t> ri(rows.begin(), rows.end());
        DevArr<int64_t> didx(ri.size());
        DevArr<float> dtr(ri.size() * (size_t)d);
        DRM_HIP_CHECK(hipMemcpy(didx.p, ri.data(), sizeof(int64_t) * ri.size(), hipMemcpyHostToDevice));
        hipLaunchKernelGGL(gather_rows_kernel, dim3(1024), dim3(256), 0, nullptr, d_x, didx.p, (int64_t)ri.size(), d,
                           dtr.p);
        DRM_HIP_CHECK(hipGetLastError());
        std::vector<float> tr(ri.size() * (size_t)d);
        DRM_HIP_CHECK(hipMemcpy(tr.data(), dtr.p, sizeof(float) * tr.size(), hipMemcpyDeviceToHost));
        pq_train_subspaces(tr.data(), ri.size(), d, M_pq, nbits, seed, 0, ix.centroids.data());
    }
    if (verbose)
        std::fprintf(stderr, "[gpu build] PQ trained %.1fs\n", secs_since(t0));
    // PQ sdc_table [M][ksub][ksub] (ProductQuantizer::compute_sdc_table), for the neighbour heuristic
    std::vector<float> sdc((size_t)M_pq * ksub * ksub);
    for (int m = 0; m < M_pq; ++m)
        for (int i = 0; i < ksub; ++i)
            for (int j = 0; j < ksub; ++j) {
                const float *ci = &ix.centroids[((size_t)m * ksub + i) * dsub];
                const float *cj = &ix.centroids[((size_t)m * ksub + j) * dsub];
                float acc = 0.f;
                for (int t = 0; t < dsub; ++t) {
                    const float df = ci[t] - cj[t];
                    acc += df * df;
                }
                sdc[((size_t)m * ksub + i) * ksub + j] = acc;
            }
    DevArr<float> dsdc(sdc.size());
    DRM_HIP_CHECK(hipMemcpy(dsdc.p, sdc.data(), sizeof(float) * sdc.size(), hipMemcpyHostToDevice));
    DevArr<float> dcent(ix.centroids.size());
    DRM_HIP_CHECK(hipMemcpy(dcent.p, ix.centroids.data(), sizeof(float) * ix.centroids.size(), hipMemcpyHostToDevice));
    // 2. codes
    DevArr<uint8_t> dcodes((size_t)n * M_pq);
    hipLaunchKernelGGL((pq_encode_kernel<16>), dim3((unsigned)((n + 255) / 256), (unsigned)M_pq), dim3(256),
                       sizeof(float) * ksub * dsub, nullptr, d_x, n, d, dcent.p, dcodes.p, M_pq);
    DRM_HIP_CHECK(hipGetLastError());
    // 3. levels and insertion order
    ix.efConstruction = efc;
    ix.efSearch = 16;
    const int top_level = hnsw_assign_levels(ix, n, M_hnsw, seed);
    const int deg0 = 2 * M_hnsw, degU = M_hnsw;
    std::vector<int32_t> order;
    order.reserve((size_t)n);
    {
        std::vector<std::vector<int32_t>> buckets((size_t)top_level + 1);
        for (int64_t i = 0; i < n; ++i)
            buckets[(size_t)ix.levels[i] - 1].push_back((int32_t)i);
        std::mt19937 orng((uint32_t)(789 + seed));
        for (int pl = top_level; pl >= 0; --pl) {
            auto &bk = buckets[(size_t)pl];
            for (size_t j = 0; j + 1 < bk.size(); ++j)
                std::swap(bk[j], bk[j + orng() % (bk.size() - j)]);
            order.insert(order.end(), bk.begin(), bk.end());
        }
    }
    ix.entry_point = order[0];
    ix.max_level = ix.levels[order[0]] - 1;
    std::vector<int64_t> uoff((size_t)n, -1);
    int64_t upper_len = 0;
    std::vector<int32_t> lev0((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        lev0[(size_t)i] = ix.levels[i] - 1;
        if (lev0[(size_t)i] > 0) {
            uoff[(size_t)i] = upper_len;
            upper_len += (int64_t)lev0[(size_t)i] * degU;
        }
    }
    DevArr<uint64_t> dl0((size_t)n * deg0), dlu((size_t)upper_len);
    DRM_HIP_CHECK(hipMemset(dl0.p, 0xFF, sizeof(uint64_t) * (size_t)n * deg0));
    DRM_HIP_CHECK(hipMemset(dlu.p, 0xFF, sizeof(uint64_t) * (size_t)std::max<int64_t>(upper_len, 1)));
    DevArr<int64_t> duoff((size_t)n);
    DevArr<int32_t> dlev((size_t)n), dorder((size_t)n);
    DRM_HIP_CHECK(hipMemcpy(duoff.p, uoff.data(), sizeof(int64_t) * (size_t)n, hipMemcpyHostToDevice));
    DRM_HIP_CHECK(hipMemcpy(dlev.p, lev0.data(), sizeof(int32_t) * (size_t)n, hipMemcpyHostToDevice));
    DRM_HIP_CHECK(hipMemcpy(dorder.p, order.data(), sizeof(int32_t) * (size_t)n, hipMemcpyHostToDevice));
    // 4. batched insertion
    int cus = 0;
    DRM_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    const int slots = cus * 16;
    const int64_t vis_words = (n + 31) / 32;
    const int clear_cap = 16384;
    DevArr<uint32_t> dvis((size_t)slots * (size_t)vis_words);
    DRM_HIP_CHECK(hipMemset(dvis.p, 0, sizeof(uint32_t) * (size_t)slots * (size_t)vis_words));
    DevArr<int32_t> dclr((size_t)slots * clear_cap);
    DevArr<uint32_t> dcounter(2); // [0] work queue head, [1] error count
    const int ef = std::min(efc, 256);
    BuildArgs a{};
    a.x = d_x;
    a.d = d;
    a.centroids = dcent.p;
    a.codes = dcodes.p;
    a.sdc = dsdc.p;
    a.link0 = dl0.p;
    a.linkU = dlu.p;
    a.uoff = duoff.p;
    a.levels = dlev.p;
    a.deg0 = deg0;
    a.degU = degU;
    a.entry_point = ix.entry_point;
    a.max_level = ix.max_level;
    a.order = dorder.p;
    a.ef = std::max(ef, deg0);
    a.visited = dvis.p;
    a.vis_words = vis_words;
    a.clear_list = dclr.p;
    a.clear_cap = clear_cap;
    a.counter = dcounter.p;
    a.errors = dcounter.p + 1;
    auto env_bound = [](const char *k, int64_t dflt) {
        const char *e = std::getenv(k);
        const int64_t v = e ? std::atoll(e) : 0;
        return v > 0 ? std::min(v, dflt) : dflt;
    };
    a.hop_bound = env_bound("DRM_BUILD_HOP_BOUND", n);
    DRM_HIP_CHECK(hipMemset(dcounter.p, 0, 2 * sizeof(uint32_t)));
    const size_t lds = sizeof(float) * 8 * 256;
    for (int64_t start = 1; start < n;) {
        const int64_t cnt = std::min(std::min(start, kMaxBatch), n - start);
        a.start = start;
        a.count = cnt;
        a.item_bound = env_bound("DRM_BUILD_ITEM_BOUND", cnt);
        DRM_HIP_CHECK(hipMemsetAsync(dcounter.p, 0, sizeof(uint32_t), nullptr));
        const int grid = (int)std::min<int64_t>(cnt, slots);
        if (a.ef <= 128)
            hipLaunchKernelGGL((hnsw_build_insert_kernel<2>), dim3(grid), dim3(64), lds, nullptr, a);
        else
            hipLaunchKernelGGL((hnsw_build_insert_kernel<4>), dim3(grid), dim3(64), lds, nullptr, a);
        DRM_HIP_CHECK(hipGetLastError());
        for (int l = 0; l <= ix.max_level; ++l) {
            const int deg = l == 0 ? deg0 : degU;
            const int64_t th = cnt * deg;
            hipLaunchKernelGGL(hnsw_build_reverse_kernel, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, nullptr, a,
                               l);
            DRM_HIP_CHECK(hipGetLastError());
        }
        start += cnt;
        if (verbose && (cnt >= kMaxBatch || start >= n)) {
            DRM_HIP_CHECK(hipDeviceSynchronize());
            std::fprintf(stderr, "[gpu build] %lld / %lld inserted %.1fs\n", (long long)start, (long long)n,
                         secs_since(t0));
        }
    }
    DRM_HIP_CHECK(hipDeviceSynchronize());
    uint32_t nerr = 0;
    DRM_HIP_CHECK(hipMemcpy(&nerr, dcounter.p + 1, sizeof(nerr), hipMemcpyDeviceToHost));
    if (nerr)
        throw Error(DRM_ERR_INTERNAL, std::to_string(nerr) + " insertion waves exceeded their work-item or beam-hop "
                                                             "bound: build state broken");
    if (verbose)
        std::fprintf(stderr, "[gpu build] graph built %.1fs\n", secs_since(t0));
    // 5. faiss layout
    std::vector<int32_t> l0((size_t)n * deg0), lu((size_t)upper_len);
    {
        DevArr<int32_t> o0((size_t)n * deg0);
        hipLaunchKernelGGL(hnsw_build_finish_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, nullptr, dl0.p, n,
                           deg0, o0.p);
        DRM_HIP_CHECK(hipGetLastError());
        DRM_HIP_CHECK(hipMemcpy(l0.data(), o0.p, sizeof(int32_t) * l0.size(), hipMemcpyDeviceToHost));
        if (upper_len > 0) {
            DevArr<int32_t> ou((size_t)upper_len);
            const int64_t nl = upper_len / degU;
            hipLaunchKernelGGL(hnsw_build_finish_kernel, dim3((unsigned)((nl + 63) / 64)), dim3(64), 0, nullptr,
                               dlu.p, nl, degU, ou.p);
            DRM_HIP_CHECK(hipGetLastError());
            DRM_HIP_CHECK(hipMemcpy(lu.data(), ou.p, sizeof(int32_t) * lu.size(), hipMemcpyDeviceToHost));
        }
    }
    ix.codes.resize((size_t)n * M_pq);
    DRM_HIP_CHECK(hipMemcpy(ix.codes.data(), dcodes.p, ix.codes.size(), hipMemcpyDeviceToHost));
    ix.neighbors.assign(ix.offsets.back(), -1);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        int32_t *dst = ix.neighbors.data() + ix.offsets[i];
        std::memcpy(dst, &l0[(size_t)i * deg0], sizeof(int32_t) * deg0);
        if (uoff[(size_t)i] >= 0)
            std::memcpy(dst + deg0, &lu[(size_t)uoff[(size_t)i]], sizeof(int32_t) * (size_t)lev0[(size_t)i] * degU);
    }
    write_hnswpq(ix, path);
    if (verbose)
        std::fprintf(stderr, "[gpu build] written %.1fs\n", secs_since(t0));
}

} // namespace drm

extern "C" int drm_build_hnswpq_device(const float *d_x, int64_t n, int32_t d, int32_t M_pq, int32_t nbits,
                                       int32_t M_hnsw, int32_t efConstruction, double sample_rate, uint64_t seed,
                                       int device, const char *index_path)
{
    try {
        if (!d_x || !index_path)
            throw drm::Error(DRM_ERR_ARG, "null argument");
        drm::build_hnswpq_gpu(d_x, n, d, M_pq, nbits, M_hnsw, efConstruction, sample_rate, seed, device, index_path);
        return DRM_OK;
    } catch (const drm::Error &e) {
        drm::set_last_error(e.what());
        return e.code;
    } catch (const std::exception &e) {
        drm::set_last_error(e.what());
        return DRM_ERR_ARG;
    }
}
