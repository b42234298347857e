// deepreadmapper_amd/csrc/exec.cpp -- the batch executor of the query hot path, on top of the C ABI:
//
//   * drm_search_rerank: the fused search -> SW rerank entry proposed in SURVEY.md sec. 8b. It replaces
//     the reference's staged loop faiss_search(...) then post_process_sw_static(...) (src/main.cpp:270-341)
//     with batches that stream through the device: host -> device copies of batch b+1, the search and
//     rerank kernels of batch b and the device -> host copies of batch b-1 overlap on three HIP streams
//     (two device buffer sets, ping-pong). Copies are DMA when the caller's buffers are pinned
//     (drm_host_alloc), staged by the HIP runtime otherwise;
//   * drm_multi_*: the multi-GPU fan-out "inside the call" (SURVEY.md sec. 8b Threading, sec. 8e): one
//     index replica and window table per device, contiguous query shards [r*n/G, (r+1)*n/G), one host
//     thread per device running drm_search_rerank on its shard straight into the caller's outputs.
//     Queries are independent (#pragma omp over queries in faiss, src/utils/post_processor.cpp:491), so
//     there is no exchange on the data path and the outputs are byte-identical to one device's;
//   * drm_comm_*: for jobs run as one process per GPU (bench.py under torch.distributed.run), the one
//     real exchange step of the path -- every rank's device-resident result rows gathered to the root
//     rank over RCCL (xGMI point-to-point sends, grouped), sec. 8e.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "drm_hip.h"
#include "drm_internal.h"

using drm::Error;

namespace {

void hip_check(hipError_t e, const char *what)
{
    if (e != hipSuccess)
        throw Error(DRM_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}
#define HC(x) hip_check((x), #x)

void abi_check(int rc)
{
    if (rc != DRM_OK)
        throw Error(rc, drm_last_error());
}

template <class F> int guard(F &&f)
{
    try {
        f();
        return DRM_OK;
    } catch (const Error &e) {
        drm::set_last_error(e.what());
        return e.code;
    } catch (const std::bad_alloc &) {
        drm::set_last_error("out of host memory");
        return DRM_ERR_ARG;
    } catch (const std::exception &e) {
        drm::set_last_error(e.what());
        return DRM_ERR_ARG;
    }
}

struct DevMem {
    void *p = nullptr;
    DevMem() = default;
    explicit DevMem(size_t bytes) { HC(hipMalloc(&p, std::max<size_t>(bytes, 1))); }
    ~DevMem()
    {
        if (p)
            (void)hipFree(p);
    }
    DevMem(const DevMem &) = delete;
    DevMem &operator=(const DevMem &) = delete;
    template <class T> T *as() const { return static_cast<T *>(p); }
};

// One device buffer set of the batch pipeline.
struct Span {
    void *p = nullptr;
    template <class T> T *as() const { return static_cast<T *>(p); }
};
struct BatchSet {
    Span x, q, ql, D, I, nd, nh, sc, id, st; // slices of the cache's one device arena
    hipEvent_t search_done = nullptr, comp_done = nullptr, out_done = nullptr;
    bool busy = false;
};

constexpr int kSets = 3;

// Streams, events and device buffers of the executor, kept per index handle between calls (an index
// handle is single-stream, so one executor per handle never races), grown when a call needs more.
struct ExecCache {
    int device = -1;
    hipStream_t s_search = nullptr, s_sw = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    BatchSet sets[kSets];
    int64_t B = 0, d = 0, kc = 0, kr = 0, q_stride = 0;
    bool rr = false;
    std::unique_ptr<DevMem> arena;
    // pinned host staging of the per-query ndis / nhops (a copy into pageable memory would block the
    // host thread until the kernels before it finish, serialising the batch loop)
    int32_t *h_stats = nullptr;
    int64_t h_stats_n = 0;
    // drm_search_rerank_device: per-batch timing events (search start/end, rerank start/end) and the join
    std::vector<hipEvent_t> ev_ss, ev_se, ev_we;
    hipEvent_t join = nullptr;
    void reserve_events(size_t nb)
    {
        for (auto *v : {&ev_ss, &ev_se, &ev_we})
            while (v->size() < nb) {
                hipEvent_t e;
                HC(hipEventCreate(&e));
                v->push_back(e);
            }
        if (!join)
            HC(hipEventCreateWithFlags(&join, hipEventDisableTiming));
    }
    void reserve_stats(int64_t n)
    {
        if (n <= h_stats_n)
            return;
        if (h_stats)
            HC(hipHostFree(h_stats));
        h_stats = nullptr;
        HC(hipHostMalloc((void **)&h_stats, sizeof(int32_t) * 2 * (size_t)n, hipHostMallocDefault));
        h_stats_n = n;
    }

    void init(int dev)
    {
        device = dev;
        HC(hipSetDevice(dev));
        // two non-blocking streams (no implicit synchronisation with the legacy null stream). HIP deals its
        // streams round-robin over GPU_MAX_HW_QUEUES hardware queues (4 on the box) and two streams on one queue
        // run in submission order (tools/microbench/concurrency.hip); the executor's own two streams are created
        // together, so they land on different queues. Either may share its queue with a stream the process made
        // earlier (the caller's, RCCL's, torch's). That is acceptable here: the executor orders itself behind the
        // caller's stream anyway (an event at entry, the caller waits on ours at exit), RCCL and torch streams carry
        // no work while a search runs in this library's callers (the bench's gather runs after its timed region),
        // and a queue shared with an idle stream costs nothing. Round 3 gave each stream a queue of its own with a
        // full CU mask (hipExtStreamCreateWithCUMask), but such streams synchronise with the null stream; round-3
        // advice asked for non-blocking ones, and the measured overlap of search and rerank batches
        // (profiles/r02/pipe_c3/timeline_2streams.txt) does not depend on it.
        for (hipStream_t *s : {&s_search, &s_sw})
            HC(hipStreamCreateWithFlags(s, hipStreamNonBlocking));
        HC(hipEventCreate(&e0));
        HC(hipEventCreate(&e1));
        for (auto &b : sets)
            for (hipEvent_t *e : {&b.search_done, &b.comp_done, &b.out_done})
                HC(hipEventCreateWithFlags(e, hipEventDisableTiming));
    }
    void reserve(int64_t B_, int64_t d_, int64_t kc_, int64_t kr_, int64_t qs_, bool rr_)
    {
        if (B_ <= B && d_ == d && kc_ <= kc && kr_ <= kr && qs_ <= q_stride && (rr == rr_ || !rr_))
            return;
        B = std::max(B, B_);
        d = d_;
        kc = std::max(kc, kc_);
        kr = std::max(kr, kr_);
        q_stride = std::max(q_stride, qs_);
        rr = rr || rr_;
        // one allocation for all sets (each hipMalloc maps its pages up front; ten per set cost ms)
        const size_t qsz = (size_t)std::max<int64_t>(q_stride, 1), ksz = (size_t)std::max<int64_t>(kr, 1);
        const size_t sizes[10] = {sizeof(float) * (size_t)B * d, sizeof(float) * (size_t)B * kc,
                                  sizeof(int64_t) * (size_t)B * kc, sizeof(int32_t) * (size_t)B,
                                  sizeof(int32_t) * (size_t)B, rr ? (size_t)B * qsz : 0,
                                  rr ? sizeof(int32_t) * (size_t)B : 0, rr ? sizeof(int32_t) * (size_t)B * ksz : 0,
                                  rr ? sizeof(uint64_t) * (size_t)B * ksz : 0, rr ? sizeof(int32_t) * (size_t)B : 0};
        size_t per_set = 0;
        for (size_t z : sizes)
            per_set += (z + 255) & ~(size_t)255;
        arena.reset(); // release the old arena first (the sets are idle between calls)
        arena.reset(new DevMem(per_set * kSets));
        uint8_t *base = arena->as<uint8_t>();
        for (auto &s : sets) {
            Span *dst[10] = {&s.x, &s.D, &s.I, &s.nd, &s.nh, &s.q, &s.ql, &s.sc, &s.id, &s.st};
            for (int i = 0; i < 10; ++i) {
                dst[i]->p = sizes[i] ? base : nullptr;
                base += (sizes[i] + 255) & ~(size_t)255;
            }
        }
    }
    void drain()
    {
        for (hipStream_t s : {s_search, s_sw})
            if (s)
                (void)hipStreamSynchronize(s);
        for (auto &b : sets)
            b.busy = false;
    }
    ~ExecCache()
    {
        if (device < 0)
            return;
        (void)hipSetDevice(device);
        drain();
        for (auto &b : sets)
            for (hipEvent_t e : {b.search_done, b.comp_done, b.out_done})
                if (e)
                    (void)hipEventDestroy(e);
        for (hipEvent_t e : {e0, e1, join})
            if (e)
                (void)hipEventDestroy(e);
        for (auto *v : {&ev_ss, &ev_se, &ev_we})
            for (hipEvent_t e : *v)
                (void)hipEventDestroy(e);
        for (hipStream_t s : {s_search, s_sw})
            if (s)
                (void)hipStreamDestroy(s);
        if (h_stats)
            (void)hipHostFree(h_stats);
    }
};

std::mutex g_exec_mu;
// never destroyed: HIP calls from static destructors at process exit are unsafe; handles are released
// explicitly through drm_index_free
std::map<const void *, std::unique_ptr<ExecCache>> &g_exec = *new std::map<const void *, std::unique_ptr<ExecCache>>();

ExecCache &exec_for(const drm_index *ix, int device)
{
    std::lock_guard<std::mutex> lk(g_exec_mu);
    auto &p = g_exec[ix];
    if (!p || p->device != device) {
        p.reset(new ExecCache());
        p->init(device);
    }
    return *p;
}

// The batches of an n-query call: (first query, count). Equal batches of at most Bmax, except that with four or more
// of them the first and the last are a quarter of the others: the first upload and the last batch's result download
// are the only copies no kernel hides (at C5: 167 MB in, 771 MB out per 250k-query batch), and they shrink with them
std::vector<std::pair<int64_t, int64_t>> batch_plan(int64_t n, int64_t Bmax)
{
    std::vector<std::pair<int64_t, int64_t>> plan;
    Bmax = std::max<int64_t>(1, std::min(Bmax, n));
    int64_t nb = (n + Bmax - 1) / Bmax;
    int64_t edge = 0;
    if (nb >= 4 && !std::getenv("DRM_BATCH")) {
        edge = std::max<int64_t>(1, Bmax / 4);
        const int64_t mid = n - 2 * edge;
        nb = (mid + Bmax - 1) / Bmax;
        const int64_t B = (mid + nb - 1) / nb;
        plan.emplace_back(0, edge);
        for (int64_t lo = edge; lo < n - edge; lo += B)
            plan.emplace_back(lo, std::min(B, n - edge - lo));
        plan.emplace_back(n - edge, edge);
        return plan;
    }
    const int64_t B = (n + nb - 1) / nb; // equal batches, none tiny
    for (int64_t lo = 0; lo < n; lo += B)
        plan.emplace_back(lo, std::min(B, n - lo));
    return plan;
}

int64_t batch_size_for(int64_t n)
{
    if (const char *e = std::getenv("DRM_BATCH"))
        return std::max<int64_t>(1, std::atoll(e));
    // at least four batches for the copy / compute overlap, none below 32k queries (each kernel
    // launch drains its persistent grid at the end) nor above 256k (~1 GB of buffers per set)
    return std::min<int64_t>(262144, std::max<int64_t>(32768, (n + 3) / 4));
}

// status -> error, as drm_post_process_sw_static reports it (reranker.cpp:26-29, post_processor.cpp:486-489)
void check_status(const int32_t *status, int64_t n, int32_t k)
{
    int64_t first_bad = -1, first_over = -1;
    for (int64_t i = 0; i < n && (first_bad < 0 || first_over < 0); ++i) {
        if (status[i] == -1 && first_bad < 0)
            first_bad = i;
        if ((status[i] == -2 || status[i] == -3) && first_over < 0)
            first_over = i;
    }
    if (first_over >= 0)
        throw Error(DRM_ERR_UNSUPPORTED, "query " + std::to_string(first_over) +
                                             " expands to more than 1024 candidates or exceeds the SW kernels' limits (query"
                                             " length; banded: 256 bytes, 7 distinct query bytes)");
    if (first_bad >= 0)
        throw Error(DRM_ERR_CANDS, "Not enough candidates (query " + std::to_string(first_bad) + ": fewer than " +
                                       std::to_string(k) + ")");
}

void search_rerank(drm_index *index, drm_refs *refs, const float *x, int64_t n, int32_t d, int32_t k_clusters,
                   int32_t ef, const uint8_t *queries, const int32_t *q_len, int32_t q_stride, int64_t stride,
                   int32_t k, float *D, int64_t *I, int32_t *sw_scores, uint64_t *sw_ids, int32_t *status,
                   drm_search_stats *stats)
{
    if (!index || !x || !D || !I)
        throw Error(DRM_ERR_ARG, "null argument");
    if (n <= 0)
        throw Error(DRM_ERR_ARG, "Query data is empty"); // src/hnswpq/search.cpp:16-19
    drm_index_info info;
    abi_check(drm_index_get_info(index, &info));
    if (d != info.d)
        throw Error(DRM_ERR_ARG, "query dimension " + std::to_string(d) + " != index dimension " + std::to_string(info.d));
    if (k_clusters <= 0)
        throw Error(DRM_ERR_ARG, "k must be > 0");
    const bool rr = refs != nullptr;
    int genome_mode = 0;
    if (rr) {
        if (!queries || !q_len || !sw_scores || !sw_ids || !status)
            throw Error(DRM_ERR_ARG, "null rerank argument");
        if (stride < 1 || k < 0)
            throw Error(DRM_ERR_ARG, "invalid stride / k");
        if ((int64_t)k > (int64_t)k_clusters * 2 * stride) // post_processor.cpp:486-489
            throw Error(DRM_ERR_K, "Final k too large. Ensure k < k_clusters * 2 * stride to have enough candidates.");
        for (int64_t i = 0; i < n; ++i)
            if (q_len[i] < 0 || q_len[i] > q_stride)
                throw Error(DRM_ERR_ARG, "query length outside [0, q_stride]");
        int dev_r = -1;
        abi_check(drm_refs_get_info(refs, nullptr, nullptr, &dev_r));
        abi_check(drm_refs_is_genome(refs, &genome_mode));
        if (dev_r != info.device)
            throw Error(DRM_ERR_ARG, "index and window table live on different devices");
    }
    static const bool verbose = std::getenv("DRM_EXEC_VERBOSE") && std::atoi(std::getenv("DRM_EXEC_VERBOSE"));
    const auto t_start = std::chrono::steady_clock::now();
    auto ms_since = [&] {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    };
    HC(hipSetDevice(info.device));
    const std::vector<std::pair<int64_t, int64_t>> plan = batch_plan(n, batch_size_for(n));
    int64_t B = 0;
    for (const auto &pb : plan)
        B = std::max(B, pb.second);
    // DRM_EXEC_OVERLAP=1: the round-2 schedule, where batch b+1's search may start while batch b's rerank runs
    // (the two kernels then share the CUs, measured slower than one after the other)
    static const bool overlap = std::getenv("DRM_EXEC_OVERLAP") && std::atoi(std::getenv("DRM_EXEC_OVERLAP"));
    const size_t kc = (size_t)k_clusters, kr = rr ? (size_t)k : 0;
    ExecCache &ex = exec_for(index, info.device);
    try {
        ex.reserve(B, d, (int64_t)kc, (int64_t)kr, rr ? q_stride : 0, rr);
        ex.reserve_stats(n);
        int32_t *nd_host = ex.h_stats, *nh_host = ex.h_stats + n;
        if (verbose)
            std::fprintf(stderr, "[exec] %lld queries, batch %lld: setup %.2f ms\n", (long long)n, (long long)B, ms_since());
        HC(hipEventRecord(ex.e0, ex.s_search));
        // Two streams: s_search (uploads, search, downloads) and s_sw (rerank). HIP maps streams onto a few
        // hardware queues per device (GPU_MAX_HW_QUEUES, 4 by default, the null stream and the caller's own
        // streams included); two streams that land on one queue run in submission order, so a separate
        // download stream that shared the rerank's queue put each batch's downloads between two reranks.
        // With a rerank, a batch's search results are downloaded on s_search right after its search, and
        // its rerank results one batch late, after the next search: the search stream waits for the
        // rerank there, and has the slack for it (a search is shorter than a rerank). Without a rerank,
        // s_sw is the download stream.
        hipStream_t s_out = rr ? ex.s_search : ex.s_sw;
        auto download_search = [&](BatchSet &s, int64_t lo, size_t m) {
            HC(hipStreamWaitEvent(s_out, s.search_done, 0));
            HC(hipMemcpyAsync(D + (size_t)lo * kc, s.D.p, sizeof(float) * m * kc, hipMemcpyDeviceToHost, s_out));
            HC(hipMemcpyAsync(I + (size_t)lo * kc, s.I.p, sizeof(int64_t) * m * kc, hipMemcpyDeviceToHost, s_out));
            HC(hipMemcpyAsync(nd_host + lo, s.nd.p, sizeof(int32_t) * m, hipMemcpyDeviceToHost, s_out));
            HC(hipMemcpyAsync(nh_host + lo, s.nh.p, sizeof(int32_t) * m, hipMemcpyDeviceToHost, s_out));
        };
        auto download_rerank = [&](BatchSet &s, int64_t lo, size_t m) {
            HC(hipStreamWaitEvent(s_out, s.comp_done, 0));
            HC(hipMemcpyAsync(sw_scores + (size_t)lo * kr, s.sc.p, sizeof(int32_t) * m * kr, hipMemcpyDeviceToHost,
                              s_out));
            HC(hipMemcpyAsync(sw_ids + (size_t)lo * kr, s.id.p, sizeof(uint64_t) * m * kr, hipMemcpyDeviceToHost,
                              s_out));
            HC(hipMemcpyAsync(status + lo, s.st.p, sizeof(int32_t) * m, hipMemcpyDeviceToHost, s_out));
            HC(hipEventRecord(s.out_done, s_out));
        };
        int64_t b = 0, prev_lo = 0;
        size_t prev_m = 0;
        for (const auto &pb : plan) {
            const int64_t lo = pb.first, nb = pb.second;
            BatchSet &s = ex.sets[b % kSets];
            if (s.busy) // the set's previous batch has left the device
                HC(hipEventSynchronize(s.out_done));
            s.busy = true;
            const size_t m = (size_t)nb;
            HC(hipMemcpyAsync(s.x.p, x + (size_t)lo * d, sizeof(float) * m * d, hipMemcpyHostToDevice, ex.s_search));
            if (rr) {
                HC(hipMemcpyAsync(s.q.p, queries + (size_t)lo * q_stride, m * q_stride, hipMemcpyHostToDevice,
                                  ex.s_search));
                HC(hipMemcpyAsync(s.ql.p, q_len + lo, sizeof(int32_t) * m, hipMemcpyHostToDevice, ex.s_search));
            }
            // search (s_search, behind its uploads, and behind the previous batch's rerank: each kernel has the
            // whole chip, while the copy engines move batch b+1's inputs and batch b-1's results), then rerank (s_sw)
            if (rr && b > 0 && !overlap)
                HC(hipStreamWaitEvent(ex.s_search, ex.sets[(b - 1) % kSets].comp_done, 0));
            abi_check(drm_search_device_ex(index, s.x.as<float>(), nb, k_clusters, ef, s.D.as<float>(),
                                           s.I.as<int64_t>(), s.nd.as<int32_t>(), s.nh.as<int32_t>(), nullptr,
                                           ex.s_search));
            HC(hipEventRecord(s.search_done, ex.s_search));
            if (rr) {
                HC(hipStreamWaitEvent(ex.s_sw, s.search_done, 0));
                auto *pp = genome_mode ? drm_post_process_sw_dynamic_device : drm_post_process_sw_static_device;
                abi_check(pp(refs, s.I.as<int64_t>(), nb, k_clusters, s.q.as<uint8_t>(), s.ql.as<int32_t>(), q_stride,
                             stride, k, k_clusters, s.sc.as<int32_t>(), s.id.as<uint64_t>(), s.st.as<int32_t>(),
                             ex.s_sw));
                HC(hipEventRecord(s.comp_done, ex.s_sw));
                download_search(s, lo, m);
                if (b > 0)
                    download_rerank(ex.sets[(b - 1) % kSets], prev_lo, prev_m);
            } else {
                download_search(s, lo, m);
                HC(hipEventRecord(s.out_done, s_out));
            }
            prev_lo = lo;
            prev_m = m;
            if (verbose)
                std::fprintf(stderr, "[exec] batch %lld enqueued %.2f ms\n", (long long)b, ms_since());
            ++b;
        }
        // e1: the end of the last batch's compute (the device span excludes its download)
        HC(hipStreamWaitEvent(ex.s_search, ex.sets[(b - 1) % kSets].comp_done, 0));
        HC(hipEventRecord(ex.e1, ex.s_search));
        if (rr)
            download_rerank(ex.sets[(b - 1) % kSets], prev_lo, prev_m);
        HC(hipStreamSynchronize(s_out));
        HC(hipEventSynchronize(ex.e1));
        ex.drain();
        float ms = 0.f;
        HC(hipEventElapsedTime(&ms, ex.e0, ex.e1));
        if (verbose)
            std::fprintf(stderr, "[exec] done %.2f ms (device span %.2f ms)\n", ms_since(), ms);
        if (stats) {
            stats->nq = n;
            stats->ndis = 0;
            stats->nhops = 0;
            for (int64_t i = 0; i < n; ++i) {
                stats->ndis += nd_host[i];
                stats->nhops += nh_host[i];
            }
            stats->kernel_ms = ms; // device span from the first search to the last rerank
        }
    } catch (...) {
        ex.drain();
        throw;
    }
    int64_t nerr = 0; // a query past the hop bound has nhops = -1 and partial rows: fail the call
    abi_check(drm_index_search_errors(index, &nerr));
    if (nerr)
        throw Error(DRM_ERR_INTERNAL, std::to_string(nerr) + " queries exceeded the search's hop bound or waves their "
                                                            "work-item bound: search state broken");
    if (rr)
        check_status(status, n, k);
}

// ---------------------------------------------------------------------------------------------------------
// drm_search_rerank_device: the same search -> SW rerank on device-resident buffers, on the caller's stream: the
// search with the whole chip, then the rerank with the whole chip. (Round 3 ran search(b) beside rerank(b-1) on
// shared CUs with capped grids; it measured slower at C5 -- a rerank wave alone on its SIMD issues at half rate
// and no search wave fits beside two of them -- and was removed in round 5)
void search_rerank_device(drm_index *index, drm_refs *refs, const float *d_x, int64_t n, int32_t k_clusters,
                          int32_t ef, const uint8_t *d_queries, const int32_t *d_q_len, int32_t q_stride,
                          int64_t stride, int32_t k, float *d_D, int64_t *d_I, int32_t *d_ndis, int32_t *d_nhops,
                          int32_t *d_nhops_upper, int32_t *d_sw_scores, uint64_t *d_sw_ids, int32_t *d_status,
                          hipStream_t stream, drm_pipeline_stats *stats)
{
    if (!index || !refs || !d_x || !d_D || !d_I || !d_queries || !d_q_len || !d_sw_scores || !d_sw_ids || !d_status)
        throw Error(DRM_ERR_ARG, "null argument");
    if (n <= 0)
        throw Error(DRM_ERR_ARG, "Query data is empty"); // src/hnswpq/search.cpp:16-19
    if (k_clusters <= 0 || k < 0 || stride < 1)
        throw Error(DRM_ERR_ARG, "invalid k / k_clusters / stride");
    if ((int64_t)k > (int64_t)k_clusters * 2 * stride) // post_processor.cpp:486-489
        throw Error(DRM_ERR_K, "Final k too large. Ensure k < k_clusters * 2 * stride to have enough candidates.");
    drm_index_info info;
    abi_check(drm_index_get_info(index, &info));
    int dev_r = -1, genome_mode = 0;
    abi_check(drm_refs_get_info(refs, nullptr, nullptr, &dev_r));
    abi_check(drm_refs_is_genome(refs, &genome_mode));
    if (dev_r != info.device)
        throw Error(DRM_ERR_ARG, "index and window table live on different devices");
    HC(hipSetDevice(info.device));
    ExecCache &ex = exec_for(index, info.device);
    ex.reserve_events(1);
    auto *pp = genome_mode ? drm_post_process_sw_dynamic_device : drm_post_process_sw_static_device;
    HC(hipEventRecord(ex.ev_ss[0], stream));
    abi_check(drm_search_device_ex(index, d_x, n, k_clusters, ef, d_D, d_I, d_ndis, d_nhops, d_nhops_upper, stream));
    HC(hipEventRecord(ex.ev_se[0], stream));
    abi_check(pp(refs, d_I, n, k_clusters, d_queries, d_q_len, q_stride, stride, k, k_clusters, d_sw_scores, d_sw_ids,
                  d_status, stream));
    HC(hipEventRecord(ex.ev_we[0], stream));
    if (stats) {
        HC(hipEventSynchronize(ex.ev_we[0]));
        *stats = drm_pipeline_stats{};
        stats->nq = n;
        stats->n_batches = 1;
        float ms = 0.f;
        HC(hipEventElapsedTime(&ms, ex.ev_ss[0], ex.ev_se[0]));
        stats->search_ms = stats->first_search_ms = ms;
        HC(hipEventElapsedTime(&ms, ex.ev_se[0], ex.ev_we[0]));
        stats->sw_ms = stats->last_sw_ms = ms;
        HC(hipEventElapsedTime(&ms, ex.ev_ss[0], ex.ev_we[0]));
        stats->kernel_ms = ms;
    }
}

} // namespace

namespace drm {
// drm_index_free calls this: the executor state kept for the handle goes with it
void exec_release(const void *index)
{
    std::lock_guard<std::mutex> lk(g_exec_mu);
    g_exec.erase(index);
}
} // namespace drm

// ------------------------------------------------------------------------------------ C ABI
extern "C" {

int drm_host_alloc(void **ptr, size_t bytes)
{
    return guard([&] {
        if (!ptr)
            throw Error(DRM_ERR_ARG, "null argument");
        HC(hipHostMalloc(ptr, std::max<size_t>(bytes, 1), hipHostMallocDefault));
    });
}

int drm_host_free(void *ptr)
{
    return guard([&] {
        if (ptr)
            HC(hipHostFree(ptr));
    });
}

int drm_search_rerank_device(drm_index *index, drm_refs *refs, const float *d_x, int64_t n, int32_t k_clusters,
                             int32_t ef, const uint8_t *d_queries, const int32_t *d_q_len, int32_t q_stride,
                             int64_t stride, int32_t k, float *d_D, int64_t *d_I, int32_t *d_ndis, int32_t *d_nhops,
                             int32_t *d_nhops_upper, int32_t *d_sw_scores, uint64_t *d_sw_ids, int32_t *d_status,
                             void *stream, drm_pipeline_stats *stats)
{
    return guard([&] {
        search_rerank_device(index, refs, d_x, n, k_clusters, ef, d_queries, d_q_len, q_stride, stride, k, d_D, d_I,
                             d_ndis, d_nhops, d_nhops_upper, d_sw_scores, d_sw_ids, d_status, (hipStream_t)stream,
                             stats);
    });
}

int drm_search_rerank_prepare(drm_index *index, int64_t n, int32_t d, int32_t k_clusters, int32_t k, int32_t q_stride)
{
    return guard([&] {
        if (!index || n <= 0 || d <= 0 || k_clusters <= 0)
            throw Error(DRM_ERR_ARG, "invalid prepare arguments");
        drm_index_info info;
        abi_check(drm_index_get_info(index, &info));
        HC(hipSetDevice(info.device));
        ExecCache &ex = exec_for(index, info.device);
        const bool rr = q_stride > 0;
        ex.reserve(std::min<int64_t>(n, batch_size_for(n)), d, k_clusters, rr ? k : 0, q_stride, rr);
        ex.reserve_stats(n);
        // first use of the copy engines and the arena: copies on both streams, large enough
        // to take the DMA-engine path the batch copies take (a small copy goes another way)
        const size_t wb = std::min(sizeof(int32_t) * 2 * (size_t)n, sizeof(float) * (size_t)ex.B * ex.kc);
        HC(hipMemcpyAsync(ex.sets[0].D.p, ex.h_stats, wb, hipMemcpyHostToDevice, ex.s_search));
        HC(hipStreamSynchronize(ex.s_search));
        HC(hipMemcpyAsync(ex.h_stats, ex.sets[0].D.p, wb, hipMemcpyDeviceToHost, ex.s_search));
        HC(hipStreamSynchronize(ex.s_search));
        HC(hipMemcpyAsync(ex.h_stats, ex.sets[0].D.p, wb, hipMemcpyDeviceToHost, ex.s_sw));
        HC(hipStreamSynchronize(ex.s_sw));
        // first launch of the search kernel (code object load, scratch and the index's first touch): one
        // small batch of zero queries whose results are dropped, so the first timed batch runs at speed
        const int64_t nw = std::min<int64_t>(std::min<int64_t>(n, batch_size_for(n)), 1024);
        BatchSet &s = ex.sets[0];
        HC(hipMemsetAsync(s.x.p, 0, sizeof(float) * (size_t)nw * d, ex.s_search));
        abi_check(drm_search_device_ex(index, s.x.as<float>(), nw, k_clusters, std::max(k_clusters, 16),
                                       s.D.as<float>(), s.I.as<int64_t>(), s.nd.as<int32_t>(), s.nh.as<int32_t>(),
                                       nullptr, ex.s_search));
        ex.drain();
    });
}

int drm_search_rerank(drm_index *index, drm_refs *refs, const float *x, int64_t n, int32_t d, int32_t k_clusters,
                      int32_t ef, const uint8_t *queries, const int32_t *q_len, int32_t q_stride, int64_t stride,
                      int32_t k, float *D, int64_t *I, int32_t *sw_scores, uint64_t *sw_ids, int32_t *status,
                      drm_search_stats *stats)
{
    return guard([&] {
        search_rerank(index, refs, x, n, d, k_clusters, ef, queries, q_len, q_stride, stride, k, D, I, sw_scores,
                      sw_ids, status, stats);
    });
}

} // extern "C"

// ------------------------------------------------------------------------------------ multi-GPU
struct drm_multi {
    std::vector<int> devices;
    std::vector<drm_index *> index;
    std::vector<drm_refs *> refs;
};

namespace {
// runs f(r) on one host thread per replica; the first error (lowest replica) is rethrown
template <class F> void fan_out(int g, F &&f)
{
    std::vector<std::thread> th;
    std::vector<int> rc((size_t)g, DRM_OK);
    std::vector<std::string> msg((size_t)g);
    for (int r = 0; r < g; ++r)
        th.emplace_back([&, r] {
            try {
                f(r);
            } catch (const Error &e) {
                rc[(size_t)r] = e.code;
                msg[(size_t)r] = e.what();
            } catch (const std::exception &e) {
                rc[(size_t)r] = DRM_ERR_ARG;
                msg[(size_t)r] = e.what();
            }
        });
    for (auto &t : th)
        t.join();
    for (int r = 0; r < g; ++r)
        if (rc[(size_t)r] != DRM_OK)
            throw Error(rc[(size_t)r], "device " + std::to_string(r) + ": " + msg[(size_t)r]);
}

inline int64_t shard_lo(int64_t n, int r, int g) { return n * r / g; }

void free_multi(drm_multi *m)
{
    for (auto *ix : m->index)
        if (ix)
            drm_index_free(ix);
    for (auto *rf : m->refs)
        if (rf)
            drm_refs_free(rf);
}
} // namespace

extern "C" {

} // extern "C"

namespace {
// the index replicas of a drm_multi: the file parsed once, on the first device, and cloned device to device to
// the others (drm_index_clone), in parallel -- not one host parse and one host image per device
void load_replicas(const char *index_path, drm_multi *m)
{
    const int ndev = (int)m->devices.size();
    abi_check(drm_index_load(index_path, m->devices[0], &m->index[0]));
    if (ndev > 1)
        fan_out(ndev - 1, [&](int r) {
            abi_check(drm_index_clone(m->index[0], m->devices[(size_t)r + 1], &m->index[(size_t)r + 1]));
        });
}
} // namespace

extern "C" {

int drm_multi_create(const char *index_path, const int *devices, int ndev, const uint8_t *windows, int64_t n_ref,
                     int32_t ref_len, int64_t row_stride, drm_multi **out)
{
    return guard([&] {
        if (!index_path || !devices || !out || ndev <= 0)
            throw Error(DRM_ERR_ARG, "null argument or no device");
        *out = nullptr;
        std::unique_ptr<drm_multi> m(new drm_multi());
        m->devices.assign(devices, devices + ndev);
        m->index.assign((size_t)ndev, nullptr);
        m->refs.assign((size_t)ndev, nullptr);
        try {
            load_replicas(index_path, m.get());
            fan_out(ndev, [&](int r) {
                if (windows)
                    abi_check(drm_refs_create(windows, n_ref, ref_len, row_stride, m->devices[(size_t)r],
                                              &m->refs[(size_t)r]));
            });
        } catch (...) {
            free_multi(m.get());
            throw;
        }
        *out = m.release();
    });
}

int drm_multi_create_genome(const char *index_path, const int *devices, int ndev, const uint8_t *genome, int64_t len,
                            int32_t ref_len, drm_multi **out)
{
    return guard([&] {
        if (!index_path || !devices || !out || ndev <= 0 || (!genome && len > 0))
            throw Error(DRM_ERR_ARG, "null argument or no device");
        *out = nullptr;
        std::unique_ptr<drm_multi> m(new drm_multi());
        m->devices.assign(devices, devices + ndev);
        m->index.assign((size_t)ndev, nullptr);
        m->refs.assign((size_t)ndev, nullptr);
        try {
            load_replicas(index_path, m.get());
            fan_out(ndev, [&](int r) {
                abi_check(drm_refs_create_genome(genome, len, ref_len, m->devices[(size_t)r], &m->refs[(size_t)r]));
            });
        } catch (...) {
            free_multi(m.get());
            throw;
        }
        *out = m.release();
    });
}

int drm_multi_free(drm_multi *m)
{
    return guard([&] {
        if (!m)
            return;
        free_multi(m);
        delete m;
    });
}

int drm_multi_get_index_info(const drm_multi *m, drm_index_info *info)
{
    return guard([&] {
        if (!m || m->index.empty())
            throw Error(DRM_ERR_ARG, "null argument");
        abi_check(drm_index_get_info(m->index[0], info));
    });
}

int drm_multi_search_rerank(drm_multi *m, const float *x, int64_t n, int32_t d, int32_t k_clusters, int32_t ef,
                            const uint8_t *queries, const int32_t *q_len, int32_t q_stride, int64_t stride, int32_t k,
                            float *D, int64_t *I, int32_t *sw_scores, uint64_t *sw_ids, int32_t *status,
                            drm_search_stats *stats)
{
    return guard([&] {
        if (!m)
            throw Error(DRM_ERR_ARG, "null argument");
        if (n <= 0)
            throw Error(DRM_ERR_ARG, "Query data is empty");
        const int g = (int)m->devices.size();
        const bool rr = m->refs[0] != nullptr && queries != nullptr;
        std::vector<drm_search_stats> st((size_t)g);
        const size_t kc = (size_t)k_clusters, kr = (size_t)std::max(k, 0);
        fan_out(g, [&](int r) {
            const int64_t lo = shard_lo(n, r, g), hi = shard_lo(n, r + 1, g);
            if (hi <= lo)
                return;
            // contiguous shard [lo, hi), outputs written in place (no exchange)
            search_rerank(m->index[(size_t)r], rr ? m->refs[(size_t)r] : nullptr, x + (size_t)lo * d, hi - lo, d,
                          k_clusters, ef, rr ? queries + (size_t)lo * q_stride : nullptr, rr ? q_len + lo : nullptr,
                          q_stride, stride, k, D + (size_t)lo * kc, I + (size_t)lo * kc,
                          rr ? sw_scores + (size_t)lo * kr : nullptr, rr ? sw_ids + (size_t)lo * kr : nullptr,
                          rr ? status + lo : nullptr, &st[(size_t)r]);
        });
        if (stats) {
            *stats = drm_search_stats{};
            for (auto &s : st) {
                stats->nq += s.nq;
                stats->ndis += s.ndis;
                stats->nhops += s.nhops;
                stats->kernel_ms = std::max(stats->kernel_ms, s.kernel_ms);
            }
        }
    });
}

} // extern "C"

// ------------------------------------------------------------------------------------ RCCL gather
struct drm_comm {
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0, device = 0;
};

namespace {
void nccl_check(ncclResult_t r, const char *what)
{
    if (r != ncclSuccess)
        throw Error(DRM_ERR_HIP, std::string(what) + ": " + ncclGetErrorString(r));
}
} // namespace

namespace drm {
int comm_rank(const drm_comm *c) { return c->rank; }
int comm_nranks(const drm_comm *c) { return c->nranks; }
int comm_device(const drm_comm *c) { return c->device; }

void comm_broadcast(drm_comm *c, const BcastItem *items, int n, int root, void *stream)
{
    hipStream_t s = (hipStream_t)stream;
    HC(hipSetDevice(c->device));
    nccl_check(ncclGroupStart(), "ncclGroupStart");
    for (int i = 0; i < n; ++i)
        if (items[i].bytes > 0)
            nccl_check(ncclBroadcast(c->rank == root ? items[i].send : nullptr, items[i].recv, items[i].bytes, ncclUint8,
                                     root, c->comm, s),
                       "ncclBroadcast");
    nccl_check(ncclGroupEnd(), "ncclGroupEnd");
    HC(hipStreamSynchronize(s));
}

int comm_all_ok(drm_comm *c, bool ok, void *stream)
{
    // plain allocation and synchronous copies around the one collective (see device_checksum, capi.cpp)
    hipStream_t s = (hipStream_t)stream;
    HC(hipSetDevice(c->device));
    DevMem d(sizeof(int32_t));
    const int32_t h = ok ? 1 : 0;
    HC(hipMemcpy(d.p, &h, sizeof(h), hipMemcpyHostToDevice));
    nccl_check(ncclAllReduce(d.p, d.p, 1, ncclInt32, ncclMin, c->comm, s), "ncclAllReduce");
    HC(hipStreamSynchronize(s));
    int32_t r = 0;
    HC(hipMemcpy(&r, d.p, sizeof(r), hipMemcpyDeviceToHost));
    return r;
}
} // namespace drm

extern "C" {

int drm_comm_unique_id(uint8_t *id)
{
    return guard([&] {
        if (!id)
            throw Error(DRM_ERR_ARG, "null argument");
        static_assert(sizeof(ncclUniqueId) == DRM_COMM_ID_BYTES, "RCCL unique id size");
        ncclUniqueId u;
        nccl_check(ncclGetUniqueId(&u), "ncclGetUniqueId");
        std::memcpy(id, &u, sizeof(u));
    });
}

int drm_comm_init(const uint8_t *id, int nranks, int rank, int device, drm_comm **out)
{
    return guard([&] {
        if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks)
            throw Error(DRM_ERR_ARG, "invalid communicator arguments");
        *out = nullptr;
        HC(hipSetDevice(device));
        std::unique_ptr<drm_comm> c(new drm_comm());
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        const ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
        // RCCL needs one GPU per rank: ranks that share a device (a rehearsal of N ranks on fewer GPUs) are
        // refused by it as "invalid usage"; say what it means instead
        if (r == ncclInvalidUsage)
            throw Error(DRM_ERR_UNSUPPORTED, "ncclCommInitRank: invalid usage -- RCCL needs one GPU per rank, and "
                                             "rank " + std::to_string(rank) + " of " + std::to_string(nranks) +
                                             " shares device " + std::to_string(device) + " with another rank");
        nccl_check(r, "ncclCommInitRank");
        c->nranks = nranks;
        c->rank = rank;
        c->device = device;
        *out = c.release();
    });
}

int drm_comm_free(drm_comm *c)
{
    return guard([&] {
        if (!c)
            return;
        if (c->comm)
            (void)ncclCommDestroy(c->comm);
        delete c;
    });
}

int drm_comm_gather_rows(drm_comm *c, const void *d_send, int64_t n_total, int64_t row_bytes, void *d_recv, int root,
                         void *stream)
{
    return guard([&] {
        if (!c || n_total < 0 || row_bytes <= 0 || root < 0 || root >= c->nranks)
            throw Error(DRM_ERR_ARG, "invalid gather arguments");
        if (c->rank == root && !d_recv)
            throw Error(DRM_ERR_ARG, "root needs a receive buffer");
        HC(hipSetDevice(c->device));
        hipStream_t s = (hipStream_t)stream;
        const int g = c->nranks;
        auto cnt = [&](int r) { return (size_t)(shard_lo(n_total, r + 1, g) - shard_lo(n_total, r, g)) * (size_t)row_bytes; };
        auto off = [&](int r) { return (size_t)shard_lo(n_total, r, g) * (size_t)row_bytes; };
        if (c->rank == root && cnt(root) > 0)
            HC(hipMemcpyAsync(static_cast<uint8_t *>(d_recv) + off(root), d_send, cnt(root), hipMemcpyDeviceToDevice, s));
        nccl_check(ncclGroupStart(), "ncclGroupStart");
        if (c->rank == root) {
            for (int r = 0; r < g; ++r)
                if (r != root && cnt(r) > 0)
                    nccl_check(ncclRecv(static_cast<uint8_t *>(d_recv) + off(r), cnt(r), ncclUint8, r, c->comm, s),
                               "ncclRecv");
        } else if (cnt(c->rank) > 0) {
            nccl_check(ncclSend(d_send, cnt(c->rank), ncclUint8, root, c->comm, s), "ncclSend");
        }
        nccl_check(ncclGroupEnd(), "ncclGroupEnd");
    });
}

} // extern "C"
