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
#include <cstdlib>
#include <cstring>
#include <memory>
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

// One device buffer set of the ping-pong pipeline.
struct BatchSet {
    std::unique_ptr<DevMem> x, q, ql, D, I, nd, nh, sc, id, st;
    hipEvent_t in_done = nullptr, comp_done = nullptr, out_done = nullptr;
    int64_t lo = 0, n = 0; // queries of the batch in flight in this set
    bool busy = false;
};

int64_t batch_size_default()
{
    if (const char *e = std::getenv("DRM_BATCH"))
        return std::max<int64_t>(1, std::atoll(e));
    return 262144; // ~1 GB of device buffers per set at K = 128
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
                                             " expands to more than 1024 candidates or exceeds the SW length limit");
    if (first_bad >= 0)
        throw Error(DRM_ERR_CANDS, "Not enough candidates (query " + std::to_string(first_bad) + ": fewer than " +
                                       std::to_string(k) + ")");
}

void search_rerank(drm_index *index, drm_refs *refs, const float *x, int64_t n, int32_t d, int32_t k_clusters,
                   int32_t ef, const uint8_t *queries, const int32_t *q_len, int32_t q_stride, int64_t stride,
                   int32_t k, float *D, int64_t *I, int32_t *sw_scores, uint64_t *sw_ids, int32_t *status,
                   drm_search_stats *stats, int64_t batch)
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
        if (dev_r != info.device)
            throw Error(DRM_ERR_ARG, "index and window table live on different devices");
    }
    HC(hipSetDevice(info.device));
    const int64_t B = std::min<int64_t>(n, batch > 0 ? batch : batch_size_default());
    const size_t kc = (size_t)k_clusters, kr = rr ? (size_t)k : 0;
    hipStream_t s_in, s_comp, s_out;
    HC(hipStreamCreateWithFlags(&s_in, hipStreamNonBlocking));
    HC(hipStreamCreateWithFlags(&s_comp, hipStreamNonBlocking));
    HC(hipStreamCreateWithFlags(&s_out, hipStreamNonBlocking));
    std::vector<BatchSet> sets(n > B ? 2 : 1);
    std::vector<int32_t> nd_host((size_t)n), nh_host((size_t)n);
    hipEvent_t e0, e1;
    HC(hipEventCreate(&e0));
    HC(hipEventCreate(&e1));
    auto cleanup = [&] {
        (void)hipStreamSynchronize(s_in);
        (void)hipStreamSynchronize(s_comp);
        (void)hipStreamSynchronize(s_out);
        for (auto &s : sets)
            for (hipEvent_t e : {s.in_done, s.comp_done, s.out_done})
                if (e)
                    (void)hipEventDestroy(e);
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        (void)hipStreamDestroy(s_in);
        (void)hipStreamDestroy(s_comp);
        (void)hipStreamDestroy(s_out);
    };
    try {
        for (auto &s : sets) {
            s.x.reset(new DevMem(sizeof(float) * (size_t)B * d));
            s.D.reset(new DevMem(sizeof(float) * (size_t)B * kc));
            s.I.reset(new DevMem(sizeof(int64_t) * (size_t)B * kc));
            s.nd.reset(new DevMem(sizeof(int32_t) * (size_t)B));
            s.nh.reset(new DevMem(sizeof(int32_t) * (size_t)B));
            if (rr) {
                s.q.reset(new DevMem((size_t)B * q_stride));
                s.ql.reset(new DevMem(sizeof(int32_t) * (size_t)B));
                s.sc.reset(new DevMem(sizeof(int32_t) * (size_t)B * kr));
                s.id.reset(new DevMem(sizeof(uint64_t) * (size_t)B * kr));
                s.st.reset(new DevMem(sizeof(int32_t) * (size_t)B));
            }
            HC(hipEventCreateWithFlags(&s.in_done, hipEventDisableTiming));
            HC(hipEventCreateWithFlags(&s.comp_done, hipEventDisableTiming));
            HC(hipEventCreateWithFlags(&s.out_done, hipEventDisableTiming));
        }
        HC(hipEventRecord(e0, s_comp));
        int64_t b = 0;
        for (int64_t lo = 0; lo < n; lo += B, ++b) {
            BatchSet &s = sets[(size_t)(b % (int64_t)sets.size())];
            if (s.busy) // the set's previous batch has left the device
                HC(hipEventSynchronize(s.out_done));
            s.lo = lo;
            s.n = std::min(B, n - lo);
            s.busy = true;
            const size_t m = (size_t)s.n;
            // host -> device (stream s_in)
            HC(hipMemcpyAsync(s.x->p, x + (size_t)lo * d, sizeof(float) * m * d, hipMemcpyHostToDevice, s_in));
            if (rr) {
                HC(hipMemcpyAsync(s.q->p, queries + (size_t)lo * q_stride, m * q_stride, hipMemcpyHostToDevice, s_in));
                HC(hipMemcpyAsync(s.ql->p, q_len + lo, sizeof(int32_t) * m, hipMemcpyHostToDevice, s_in));
            }
            HC(hipEventRecord(s.in_done, s_in));
            // search + rerank (stream s_comp)
            HC(hipStreamWaitEvent(s_comp, s.in_done, 0));
            abi_check(drm_search_device_ex(index, s.x->as<float>(), s.n, k_clusters, ef, s.D->as<float>(),
                                           s.I->as<int64_t>(), s.nd->as<int32_t>(), s.nh->as<int32_t>(), nullptr,
                                           s_comp));
            if (rr)
                abi_check(drm_post_process_sw_static_device(refs, s.I->as<int64_t>(), s.n, k_clusters,
                                                            s.q->as<uint8_t>(), s.ql->as<int32_t>(), q_stride, stride,
                                                            k, k_clusters, s.sc->as<int32_t>(), s.id->as<uint64_t>(),
                                                            s.st->as<int32_t>(), s_comp));
            HC(hipEventRecord(s.comp_done, s_comp));
            // device -> host (stream s_out)
            HC(hipStreamWaitEvent(s_out, s.comp_done, 0));
            HC(hipMemcpyAsync(D + (size_t)lo * kc, s.D->p, sizeof(float) * m * kc, hipMemcpyDeviceToHost, s_out));
            HC(hipMemcpyAsync(I + (size_t)lo * kc, s.I->p, sizeof(int64_t) * m * kc, hipMemcpyDeviceToHost, s_out));
            HC(hipMemcpyAsync(nd_host.data() + lo, s.nd->p, sizeof(int32_t) * m, hipMemcpyDeviceToHost, s_out));
            HC(hipMemcpyAsync(nh_host.data() + lo, s.nh->p, sizeof(int32_t) * m, hipMemcpyDeviceToHost, s_out));
            if (rr) {
                HC(hipMemcpyAsync(sw_scores + (size_t)lo * kr, s.sc->p, sizeof(int32_t) * m * kr, hipMemcpyDeviceToHost,
                                  s_out));
                HC(hipMemcpyAsync(sw_ids + (size_t)lo * kr, s.id->p, sizeof(uint64_t) * m * kr, hipMemcpyDeviceToHost,
                                  s_out));
                HC(hipMemcpyAsync(status + lo, s.st->p, sizeof(int32_t) * m, hipMemcpyDeviceToHost, s_out));
            }
            HC(hipEventRecord(s.out_done, s_out));
        }
        HC(hipEventRecord(e1, s_comp));
        HC(hipStreamSynchronize(s_out));
        HC(hipEventSynchronize(e1));
        float ms = 0.f;
        HC(hipEventElapsedTime(&ms, e0, e1));
        if (stats) {
            stats->nq = n;
            stats->ndis = 0;
            stats->nhops = 0;
            for (int64_t i = 0; i < n; ++i) {
                stats->ndis += nd_host[(size_t)i];
                stats->nhops += nh_host[(size_t)i];
            }
            stats->kernel_ms = ms; // device span of the compute stream (search + rerank of all batches)
        }
    } catch (...) {
        cleanup();
        throw;
    }
    cleanup();
    if (rr)
        check_status(status, n, k);
}

} // namespace

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

int drm_search_rerank(drm_index *index, drm_refs *refs, const float *x, int64_t n, int32_t d, int32_t k_clusters,
                      int32_t ef, const uint8_t *queries, const int32_t *q_len, int32_t q_stride, int64_t stride,
                      int32_t k, float *D, int64_t *I, int32_t *sw_scores, uint64_t *sw_ids, int32_t *status,
                      drm_search_stats *stats)
{
    return guard([&] {
        search_rerank(index, refs, x, n, d, k_clusters, ef, queries, q_len, q_stride, stride, k, D, I, sw_scores,
                      sw_ids, status, stats, 0);
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
            fan_out(ndev, [&](int r) {
                abi_check(drm_index_load(index_path, m->devices[(size_t)r], &m->index[(size_t)r]));
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
                          rr ? status + lo : nullptr, &st[(size_t)r], 0);
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
        nccl_check(ncclCommInitRank(&c->comm, nranks, u, rank), "ncclCommInitRank");
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
