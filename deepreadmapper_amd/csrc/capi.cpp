// deepreadmapper_amd/csrc/capi.cpp -- implementation of include/drm_hip.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <numeric>
#include <thread>
#include <unordered_set>

#include "drm_device.h"

namespace drm {
void exec_release(const void *index); // exec.cpp
static thread_local std::string g_last_error;
void set_last_error(const std::string &msg) { g_last_error = msg; }
} // namespace drm

struct drm_index {
    drm::DeviceIndex dev;
};
struct drm_refs {
    drm::DeviceRefs dev;
};
struct drm_flat_index {
    drm::DeviceFlatIndex dev;
};
struct drm_encoder {
    drm::DeviceEncoder dev;
};

using drm::Error;

template <class F> static int guarded(F &&f)
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

namespace {
template <class T> struct DevBuf { // RAII device buffer for host-pointer entry points
    T *p = nullptr;
    size_t n = 0;
    explicit DevBuf(size_t count) : n(count)
    {
        if (count)
            DRM_HIP_CHECK(hipMalloc(&p, sizeof(T) * count));
    }
    ~DevBuf()
    {
        if (p)
            (void)hipFree(p);
    }
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    void upload(const T *h) { DRM_HIP_CHECK(hipMemcpy(p, h, sizeof(T) * n, hipMemcpyHostToDevice)); }
    void download(T *h) const { DRM_HIP_CHECK(hipMemcpy(h, p, sizeof(T) * n, hipMemcpyDeviceToHost)); }
};

// drm_device_checksum: sum over the 8-byte little-endian words w_i of a buffer (the tail zero-padded) of
// splitmix64(w_i + i * 0x9E3779B97F4A7C15), mod 2^64 -- position-dependent, order-free, so a grid-stride sum with
// one atomic per wave computes it (deepreadmapper_amd.device.host_checksum is the same function on the host)
__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// one partial sum per wave, stored (no atomics, no zero-fill to order before them); the host adds the partials
__global__ __launch_bounds__(256) void checksum_kernel(const uint8_t *p, int64_t nbytes, unsigned long long *partial)
{
    const int64_t nw = (nbytes + 7) >> 3;
    uint64_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nw; i += (int64_t)gridDim.x * 256) {
        uint64_t w;
        if (8 * i + 8 <= nbytes) {
            w = reinterpret_cast<const uint64_t *>(p)[i];
        } else {
            w = 0;
            for (int64_t b = 8 * i; b < nbytes; ++b)
                w |= (uint64_t)p[b] << (8 * (b - 8 * i));
        }
        acc += mix64(w + (uint64_t)i * 0x9E3779B97F4A7C15ull);
    }
    for (int o = 32; o > 0; o >>= 1)
        acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0)
        partial[blockIdx.x * 4 + (threadIdx.x >> 6)] = (unsigned long long)acc;
}

// --- diagnostics for the replica checksum's stale sums (not part of include/drm_hip.h) ---
// the first form of drm_device_checksum (round 5, until dd29dac), kept to reproduce what it returned: one atomic per
// wave into a stream-ordered pool allocation zeroed by hipMemsetAsync, an async copy into pageable host memory
__global__ __launch_bounds__(256) void checksum_atomic_kernel(const uint8_t *p, int64_t nbytes, unsigned long long *out)
{
    const int64_t nw = (nbytes + 7) >> 3;
    uint64_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nw; i += (int64_t)gridDim.x * 256) {
        uint64_t w;
        if (8 * i + 8 <= nbytes) {
            w = reinterpret_cast<const uint64_t *>(p)[i];
        } else {
            w = 0;
            for (int64_t b = 8 * i; b < nbytes; ++b)
                w |= (uint64_t)p[b] << (8 * (b - 8 * i));
        }
        acc += mix64(w + (uint64_t)i * 0x9E3779B97F4A7C15ull);
    }
    for (int o = 32; o > 0; o >>= 1)
        acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0)
        atomicAdd(out, (unsigned long long)acc);
}

// a writer that holds its stream for delay_us microseconds of device time (the 100 MHz real-time counter, bounded
// loop) and then fills nbytes with the byte `value`: issued on one stream, it lets a test read the buffer from
// another stream before the write lands
__global__ __launch_bounds__(256) void delayed_fill_kernel(uint32_t *p, int64_t nwords, uint32_t v, uint64_t ticks)
{
    if (ticks) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (int i = 0; i < (1 << 24); ++i) {
            if (__builtin_amdgcn_s_memrealtime() - t0 >= ticks)
                break;
            __builtin_amdgcn_s_sleep(64);
        }
    }
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nwords; i += (int64_t)gridDim.x * 256)
        p[i] = v;
}

// drm_device_checksum's sum, on `s`; returns once it is known. It first waits for every piece of work this process
// has enqueued on the device, on any stream: a checksum enqueued on `s` alone reads the buffer while writes issued on
// another stream without an event may still be in flight, and returns the sum of the old contents -- the stale sums
// of round 5 (tests/test_gpu_checksum.py reproduces it with a delayed writer). Partials per wave into
// a plain allocation, added on the host.
uint64_t device_checksum(const void *d_ptr, int64_t nbytes, hipStream_t s)
{
    const int64_t nw = (nbytes + 7) >> 3;
    if (nw == 0)
        return 0;
    DRM_HIP_CHECK(hipDeviceSynchronize());
    const int64_t blocks = std::min<int64_t>((nw + 255) / 256, 4096);
    DevBuf<unsigned long long> partial((size_t)blocks * 4);
    hipLaunchKernelGGL(checksum_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const uint8_t *)d_ptr, nbytes, partial.p);
    DRM_HIP_CHECK(hipGetLastError());
    DRM_HIP_CHECK(hipStreamSynchronize(s));
    std::vector<unsigned long long> h((size_t)blocks * 4);
    partial.download(h.data());
    uint64_t sum = 0;
    for (unsigned long long v : h)
        sum += (uint64_t)v;
    return sum;
}

// drm_device_chase_latency / drm_device_chase_rows: the search's dependent row load alone. Each wave walks `hops` rows
// of a 384-B stride (the lean kernel's level-0 row: link j's 12 B on lane j), loading the first `lanes` links of each
// (32: the whole row, 3 lines; 21: the first 2 lines; 10: the first line), the next row's index a function of the row
// just read, over `nrows` rows of random contents; lanes past `lanes` read link 0 (the search kernel's form for lanes
// past a row's end: no branch, no extra line); bounded loop, one store per lane at the end (keeps the loads live)
__global__ __launch_bounds__(64) void chase_rows_kernel(const uint32_t *rows, int64_t nrows, int hops, int lanes,
                                                        uint32_t *sink)
{
    const int lane = threadIdx.x;
    const int l = lane < lanes ? lane : 0;
    uint64_t r = ((uint64_t)blockIdx.x * 0x9E3779B97F4A7C15ull) % (uint64_t)nrows;
    uint32_t acc = 0;
    for (int h = 0; h < hops; ++h) {
        const uint32_t *row = rows + r * 96u;
        const uint32_t x = row[3 * l], y = row[3 * l + 1], z = row[3 * l + 2];
        acc ^= x ^ y ^ z;
        // the next row from the row just read, salted with the wave and the hop: two waves that meet on a row part
        // again at once (an unsalted walk is a function of the row alone, so met walks merge and re-read each
        // other's rows from the caches), and no wave walks a cycle
        const uint32_t k = (uint32_t)__builtin_amdgcn_readfirstlane((int)x) ^ ((uint32_t)h * 0x9E3779B9u);
        r = ((uint64_t)k * 0x2545F4914F6CDD1Dull + r + 1 + (uint64_t)blockIdx.x * 0xD1B54A32D192ED03ull) % (uint64_t)nrows;
    }
    sink[(size_t)blockIdx.x * 64 + lane] = acc;
}

__global__ __launch_bounds__(256) void fill_random_kernel(uint32_t *p, int64_t n)
{
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        p[i] = (uint32_t)(mix64((uint64_t)i) >> 17);
}

template <class T> T *upload_vec(const std::vector<T> &v, int64_t &bytes)
{
    T *p = nullptr;
    size_t nb = sizeof(T) * std::max<size_t>(v.size(), 1);
    DRM_HIP_CHECK(drm::malloc_big((void **)&p, nb, drm::kBigIndex));
    if (!v.empty())
        DRM_HIP_CHECK(hipMemcpy(p, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice));
    bytes += (int64_t)nb;
    return p;
}

// tuning knobs read when an index is loaded or received: kernel choice, occupancy, diagnostics, the
// safety bounds (tests lower them)
void apply_load_env(drm::DeviceIndex &d)
{
    if (const char *e = std::getenv("DRM_SEARCH_HOP_BOUND"))
        d.hop_bound = std::max<int64_t>(0, std::atoll(e));
    if (const char *e = std::getenv("DRM_WAVE_ITEM_BOUND"))
        d.item_bound = std::max<int64_t>(0, std::atoll(e));
    if (const char *e = std::getenv("DRM_SEARCH_WAVES_PER_CU"))
        d.waves_per_cu = std::max(1, std::atoi(e));
    d.waves_per_cu_load = d.waves_per_cu;
    if (const char *e = std::getenv("DRM_SEARCH_EXACT_STATS"))
        d.exact_stats = std::atoi(e) ? 1 : 0;
    if (const char *e = std::getenv("DRM_SEARCH_LOG_CAP"))
        d.log_cap_req = std::max(1, std::atoi(e));
    if (const char *e = std::getenv("DRM_SEARCH_FAST"))
        d.use_fast = std::atoi(e) ? 1 : 0;
    if (const char *e = std::getenv("DRM_SEARCH_INLINE"))
        d.use_inline = std::atoi(e) ? 1 : 0;
    if (const char *e = std::getenv("DRM_SEARCH_LDS_KERNEL"))
        d.force_lds_kernel = std::atoi(e) ? 1 : 0;
    if (const char *e = std::getenv("DRM_SEARCH_STAMPS"))
        if (std::atoi(e)) {
            DRM_HIP_CHECK(hipMalloc(&d.stamps, 16 * sizeof(uint64_t)));
            DRM_HIP_CHECK(hipMemset(d.stamps, 0, 16 * sizeof(uint64_t)));
        }
    if (const char *e = std::getenv("DRM_SEARCH_TRACE"))
        if (std::atoi(e)) { // host memory the device writes through: readable while a kernel runs (or hangs)
            DRM_HIP_CHECK(hipHostMalloc((void **)&d.trace, sizeof(uint32_t) * drm::kTraceWords,
                                        hipHostMallocMapped | hipHostMallocCoherent));
            std::memset(d.trace, 0, sizeof(uint32_t) * drm::kTraceWords);
        }
}

void free_index(drm::DeviceIndex &d)
{
    if (d.trace)
        (void)hipHostFree(d.trace);
    void *ptrs[] = {d.centroids, d.codes,   d.nbr0,   d.upper_off, d.upper_nbr, d.visited,
                    d.clear_list, d.counter, d.stamps,   d.log,       d.rows,      d.upper_codes};
    for (void *p : ptrs)
        if (p)
            (void)hipFree(p);
}
} // namespace

extern "C" {

const char *drm_last_error(void) { return drm::g_last_error.c_str(); }
int drm_version(void) { return 100; /* 0.1.0 */ }

int drm_device_count(int *n)
{
    return guarded([&] { DRM_HIP_CHECK(hipGetDeviceCount(n)); });
}
int drm_device_get_props(int device, drm_device_props *out)
{
    return guarded([&] {
        if (!out)
            throw Error(DRM_ERR_ARG, "null argument");
        hipDeviceProp_t p;
        DRM_HIP_CHECK(hipGetDeviceProperties(&p, device));
        *out = drm_device_props{};
        out->cu_count = p.multiProcessorCount;
        out->clock_khz = p.clockRate;
        out->total_mem = (int64_t)p.totalGlobalMem;
        out->lds_per_cu = (int32_t)p.maxSharedMemoryPerMultiProcessor;
        std::snprintf(out->arch, sizeof(out->arch), "%s", p.gcnArchName);
    });
}
int drm_set_device(int device)
{
    return guarded([&] { DRM_HIP_CHECK(hipSetDevice(device)); });
}
int drm_device_sync(void)
{
    return guarded([&] { DRM_HIP_CHECK(hipDeviceSynchronize()); });
}
int drm_malloc(void **ptr, size_t bytes)
{
    return guarded([&] { DRM_HIP_CHECK(hipMalloc(ptr, std::max<size_t>(bytes, 1))); });
}
int drm_free(void *ptr)
{
    return guarded([&] {
        if (ptr)
            DRM_HIP_CHECK(hipFree(ptr));
    });
}
int drm_memset(void *ptr, int value, size_t bytes)
{
    return guarded([&] { DRM_HIP_CHECK(hipMemset(ptr, value, bytes)); });
}
int drm_device_checksum(const void *d_ptr, int64_t nbytes, uint64_t *out, void *stream)
{
    return guarded([&] {
        if (!out || nbytes < 0 || (nbytes > 0 && (!d_ptr || ((uintptr_t)d_ptr & 7u) != 0u)))
            throw Error(DRM_ERR_ARG, "drm_device_checksum: needs an 8-byte aligned device pointer and an output");
        *out = device_checksum(d_ptr, nbytes, (hipStream_t)stream);
    });
}
int drm_device_chase_rows(int device, int64_t footprint_bytes, int32_t waves, int32_t hops, int32_t row_lines,
                          double *ns_per_load)
{
    return guarded([&] {
        if (!ns_per_load || footprint_bytes < 384 || waves < 1 || waves > (1 << 20) || hops < 1 || hops > 100000 ||
            row_lines < 1 || row_lines > 3)
            throw Error(DRM_ERR_ARG, "drm_device_chase_rows: footprint >= 384 B, 1..2^20 waves, 1..1e5 hops, 1..3 lines");
        DRM_HIP_CHECK(hipSetDevice(device));
        const int64_t nrows = footprint_bytes / 384;
        const int lanes = row_lines * 128 / 12; // links whose 12 B lie in the first row_lines 128-B lines: 10, 21, 32
        DevBuf<uint32_t> rows((size_t)nrows * 96), sink((size_t)waves * 64);
        hipLaunchKernelGGL(fill_random_kernel, dim3(8192), dim3(256), 0, 0, rows.p, nrows * 96);
        DRM_HIP_CHECK(hipGetLastError());
        hipEvent_t e0, e1;
        DRM_HIP_CHECK(hipEventCreate(&e0));
        DRM_HIP_CHECK(hipEventCreate(&e1));
        hipLaunchKernelGGL(chase_rows_kernel, dim3((unsigned)waves), dim3(64), 0, 0, rows.p, nrows, std::min(hops, 50),
                           lanes, sink.p); // warm-up
        DRM_HIP_CHECK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(chase_rows_kernel, dim3((unsigned)waves), dim3(64), 0, 0, rows.p, nrows, hops, lanes, sink.p);
        DRM_HIP_CHECK(hipEventRecord(e1, 0));
        DRM_HIP_CHECK(hipGetLastError());
        DRM_HIP_CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        DRM_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        *ns_per_load = (double)ms * 1e6 / hops;
    });
}
int drm_device_chase_latency(int device, int64_t footprint_bytes, int32_t waves, int32_t hops, double *ns_per_load)
{
    return drm_device_chase_rows(device, footprint_bytes, waves, hops, 3, ns_per_load);
}
int drm_memcpy_h2d(void *dst, const void *src, size_t bytes)
{
    return guarded([&] { DRM_HIP_CHECK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice)); });
}
int drm_memcpy_d2h(void *dst, const void *src, size_t bytes)
{
    return guarded([&] { DRM_HIP_CHECK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost)); });
}
int drm_stream_create(void **stream)
{
    return guarded([&] {
        hipStream_t s;
        DRM_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        *stream = (void *)s;
    });
}
int drm_stream_destroy(void *stream)
{
    return guarded([&] { DRM_HIP_CHECK(hipStreamDestroy((hipStream_t)stream)); });
}
int drm_stream_sync(void *stream)
{
    return guarded([&] { DRM_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream)); });
}
int drm_event_create(void **ev)
{
    return guarded([&] {
        hipEvent_t e;
        DRM_HIP_CHECK(hipEventCreate(&e));
        *ev = (void *)e;
    });
}
int drm_event_destroy(void *ev)
{
    return guarded([&] { DRM_HIP_CHECK(hipEventDestroy((hipEvent_t)ev)); });
}
int drm_event_record(void *ev, void *stream)
{
    return guarded([&] { DRM_HIP_CHECK(hipEventRecord((hipEvent_t)ev, (hipStream_t)stream)); });
}
int drm_stream_wait_event(void *stream, void *ev)
{
    return guarded([&] { DRM_HIP_CHECK(hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)ev, 0)); });
}
int drm_event_elapsed_ms(void *start, void *stop, float *ms)
{
    return guarded([&] {
        DRM_HIP_CHECK(hipEventSynchronize((hipEvent_t)stop));
        DRM_HIP_CHECK(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop));
    });
}

// ------------------------------------------------------------------------------------ index
int drm_index_load(const char *path, int device, drm_index **out)
{
    return guarded([&] {
        if (!path || !out)
            throw Error(DRM_ERR_ARG, "null argument");
        *out = nullptr;
        drm::HnswPqHost h = drm::read_hnswpq(path);
        if ((int)h.cum_nneighbor_per_level.size() - 1 > drm::kMaxLevels)
            throw Error(DRM_ERR_UNSUPPORTED, "more than 24 HNSW levels");
        DRM_HIP_CHECK(hipSetDevice(device));
        std::unique_ptr<drm_index> ix(new drm_index());
        drm::DeviceIndex &d = ix->dev;
        d.device = device;
        d.d = h.hdr.d;
        d.ntotal = h.hdr.ntotal;
        d.pq_M = (int)h.pq_M;
        d.pq_nbits = (int)h.pq_nbits;
        d.dsub = h.dsub();
        d.ksub = h.ksub();
        d.code_size = h.code_size();
        d.deg0 = h.deg0();
        d.n_levels = (int)h.cum_nneighbor_per_level.size() - 1;
        d.max_level = h.max_level;
        d.entry_point = h.entry_point;
        for (size_t l = 0; l < h.cum_nneighbor_per_level.size(); ++l)
            d.cum[l] = h.cum_nneighbor_per_level[l];
        // level-0 rows, dense [ntotal][deg0]
        const int64_t n = h.hdr.ntotal;
        std::vector<int32_t> nbr0((size_t)n * d.deg0);
        std::vector<uint32_t> upper_off((size_t)n, ~0u);
        std::vector<int32_t> upper;
        // level-0 rows and the duplicate-link check in parallel (tens of millions of rows at C5)
        {
            const int nt = (int)std::max(1u, std::min(32u, std::thread::hardware_concurrency()));
            std::vector<int> dup(nt, 0);
            std::vector<std::thread> pool;
            for (int t = 0; t < nt; ++t)
                pool.emplace_back([&, t] {
                    for (int64_t i = n * t / nt; i < n * (t + 1) / nt; ++i) {
                        const uint64_t o = h.offsets[(size_t)i];
                        int32_t *r = &nbr0[(size_t)i * d.deg0];
                        std::memcpy(r, &h.neighbors[o + h.cum_nneighbor_per_level[0]], sizeof(int32_t) * d.deg0);
                        // a row listing one id twice changes visited-set semantics: flag it for the kernel
                        for (int a = 0; a < d.deg0 && r[a] >= 0 && !dup[t]; ++a)
                            for (int b = a + 1; b < d.deg0 && r[b] >= 0; ++b)
                                if (r[a] == r[b]) {
                                    dup[t] = 1;
                                    break;
                                }
                    }
                });
            for (auto &th : pool)
                th.join();
            d.has_dup_links = *std::max_element(dup.begin(), dup.end());
        }
        for (int64_t i = 0; i < n; ++i) {
            const int lv = h.levels[(size_t)i];
            if (lv > 1) {
                const uint64_t o = h.offsets[(size_t)i];
                if (upper.size() > 0xF0000000ull)
                    throw Error(DRM_ERR_UNSUPPORTED, "upper-level link table exceeds 32-bit offsets");
                upper_off[(size_t)i] = (uint32_t)upper.size();
                upper.insert(upper.end(), h.neighbors.begin() + (o + h.cum_nneighbor_per_level[1]),
                             h.neighbors.begin() + (o + h.cum_nneighbor_per_level[lv]));
            }
        }
        d.upper_len = (int64_t)upper.size();
        apply_load_env(d);
        try {
            d.centroids = upload_vec(h.centroids, d.device_bytes);
            d.codes = upload_vec(h.codes, d.device_bytes);
            d.nbr0 = upload_vec(nbr0, d.device_bytes);
            d.upper_off = upload_vec(upper_off, d.device_bytes);
            d.upper_nbr = upload_vec(upper, d.device_bytes);
            if (d.use_inline)
                drm::build_inline_rows(d); // ids + inline codes per level-0 row (lean kernel)
            drm::reserve_search_scratch(d); // the per-slot search workspace, once, outside any search
        } catch (...) {
            free_index(d);
            throw;
        }
        // keep header metadata only
        d.meta.hdr = h.hdr;
        d.meta.efConstruction = h.efConstruction;
        d.meta.efSearch = h.efSearch;
        d.meta.entry_point = h.entry_point;
        d.meta.max_level = h.max_level;
        d.meta.pq_M = h.pq_M;
        d.meta.pq_nbits = h.pq_nbits;
        d.meta.cum_nneighbor_per_level = h.cum_nneighbor_per_level;
        *out = ix.release();
    });
}

} // extern "C"

// drm_index_broadcast: the wire header the root sends first -- every scalar a DeviceIndex and its kept metadata hold,
// the byte size of each buffer that follows, and the root's checksum of each (receivers verify what arrived)
namespace {
constexpr uint64_t kBcastMagic = 0x3143425849524444ull; // "DDRIXBC1"
constexpr int kBcastBufs = 5;                          // centroids, codes, nbr0, upper_off, upper_nbr
struct IndexWire {
    uint64_t magic;
    int32_t d, pq_M, pq_nbits, dsub, ksub, code_size, deg0, n_levels, max_level, entry_point, has_dup_links;
    int32_t cum[drm::kMaxLevels + 1];
    int64_t ntotal, upper_len;
    int32_t hdr_d, hdr_metric_type;
    int64_t hdr_ntotal;
    float hdr_metric_arg;
    int32_t hdr_is_trained, efConstruction, efSearch;
    uint64_t meta_pq_M, meta_pq_nbits;
    uint64_t bytes[kBcastBufs], sums[kBcastBufs];
};

// the byte size upload_vec gives each buffer (at least one element)
void index_buffer_sizes(const drm::DeviceIndex &d, uint64_t *bytes)
{
    bytes[0] = sizeof(float) * (uint64_t)std::max<int64_t>((int64_t)d.pq_M * d.ksub * d.dsub, 1);
    bytes[1] = (uint64_t)std::max<int64_t>(d.ntotal * d.code_size, 1);
    bytes[2] = sizeof(int32_t) * (uint64_t)std::max<int64_t>(d.ntotal * d.deg0, 1);
    bytes[3] = sizeof(uint32_t) * (uint64_t)std::max<int64_t>(d.ntotal, 1);
    bytes[4] = sizeof(int32_t) * (uint64_t)std::max<int64_t>(d.upper_len, 1);
}
void **index_buffers(drm::DeviceIndex &d, void **out)
{
    out[0] = d.centroids;
    out[1] = d.codes;
    out[2] = d.nbr0;
    out[3] = d.upper_off;
    out[4] = d.upper_nbr;
    return out;
}

// the header of an index (no checksums)
IndexWire index_to_wire(const drm::DeviceIndex &r)
{
    IndexWire w{};
    w.magic = kBcastMagic;
    w.d = r.d, w.pq_M = r.pq_M, w.pq_nbits = r.pq_nbits, w.dsub = r.dsub, w.ksub = r.ksub;
    w.code_size = r.code_size, w.deg0 = r.deg0, w.n_levels = r.n_levels, w.max_level = r.max_level;
    w.entry_point = r.entry_point, w.has_dup_links = r.has_dup_links;
    std::memcpy(w.cum, r.cum, sizeof(w.cum));
    w.ntotal = r.ntotal, w.upper_len = r.upper_len;
    w.hdr_d = r.meta.hdr.d, w.hdr_metric_type = r.meta.hdr.metric_type, w.hdr_ntotal = r.meta.hdr.ntotal;
    w.hdr_metric_arg = r.meta.hdr.metric_arg, w.hdr_is_trained = r.meta.hdr.is_trained;
    w.efConstruction = r.meta.efConstruction, w.efSearch = r.meta.efSearch;
    w.meta_pq_M = r.meta.pq_M, w.meta_pq_nbits = r.meta.pq_nbits;
    index_buffer_sizes(r, w.bytes);
    return w;
}

// a new index on `device` from a header: validated, the load-time knobs applied, its five buffers allocated (not
// filled); throws Error
std::unique_ptr<drm_index> index_from_wire(const IndexWire &w, int device)
{
    uint64_t expect[kBcastBufs];
    drm::DeviceIndex probe;
    probe.pq_M = w.pq_M, probe.ksub = w.ksub, probe.dsub = w.dsub, probe.ntotal = w.ntotal;
    probe.code_size = w.code_size, probe.deg0 = w.deg0, probe.upper_len = w.upper_len;
    if (w.magic != kBcastMagic || w.ntotal <= 0 || w.deg0 < 1 || w.n_levels < 1 || w.n_levels > drm::kMaxLevels ||
        w.upper_len < 0 || w.pq_M < 1 || w.ksub < 1 || w.dsub < 1)
        throw Error(DRM_ERR_FORMAT, "malformed index header");
    index_buffer_sizes(probe, expect);
    if (std::memcmp(expect, w.bytes, sizeof(expect)) != 0)
        throw Error(DRM_ERR_FORMAT, "index header sizes disagree");
    DRM_HIP_CHECK(hipSetDevice(device));
    std::unique_ptr<drm_index> ix(new drm_index());
    drm::DeviceIndex &d = ix->dev;
    d.device = device;
    d.d = w.d, d.pq_M = w.pq_M, d.pq_nbits = w.pq_nbits, d.dsub = w.dsub, d.ksub = w.ksub;
    d.code_size = w.code_size, d.deg0 = w.deg0, d.n_levels = w.n_levels, d.max_level = w.max_level;
    d.entry_point = w.entry_point, d.has_dup_links = w.has_dup_links;
    std::memcpy(d.cum, w.cum, sizeof(d.cum));
    d.ntotal = w.ntotal, d.upper_len = w.upper_len;
    d.meta.hdr.d = w.hdr_d, d.meta.hdr.metric_type = w.hdr_metric_type, d.meta.hdr.ntotal = w.hdr_ntotal;
    d.meta.hdr.metric_arg = w.hdr_metric_arg, d.meta.hdr.is_trained = (uint8_t)w.hdr_is_trained;
    d.meta.efConstruction = w.efConstruction, d.meta.efSearch = w.efSearch;
    d.meta.entry_point = w.entry_point, d.meta.max_level = w.max_level;
    d.meta.pq_M = w.meta_pq_M, d.meta.pq_nbits = w.meta_pq_nbits;
    d.meta.cum_nneighbor_per_level.assign(w.cum, w.cum + w.n_levels + 1);
    try {
        apply_load_env(d);
        void **slots[kBcastBufs] = {(void **)&d.centroids, (void **)&d.codes, (void **)&d.nbr0, (void **)&d.upper_off,
                                    (void **)&d.upper_nbr};
        for (int b = 0; b < kBcastBufs; ++b) {
            DRM_HIP_CHECK(drm::malloc_big(slots[b], w.bytes[b], drm::kBigIndex));
            d.device_bytes += (int64_t)w.bytes[b];
        }
    } catch (...) {
        free_index(d);
        throw;
    }
    return ix;
}

// after the five buffers are filled: the lean kernel's inline rows (a function of nbr0 + codes) and the search
// scratch, as drm_index_load makes them; frees the index and rethrows on failure
void index_finish(drm_index *ix)
{
    try {
        drm::DeviceIndex &d = ix->dev;
        DRM_HIP_CHECK(hipSetDevice(d.device));
        if (d.use_inline)
            drm::build_inline_rows(d);
        drm::reserve_search_scratch(d);
    } catch (...) {
        free_index(ix->dev);
        throw;
    }
}
} // namespace

extern "C" {

int drm_index_broadcast(drm_comm *comm, drm_index *root_index, int root, drm_index **out)
{
    // every rank of the job runs every collective below in the same order whatever fails locally: a failure before a
    // data transfer is carried through comm_all_ok, so no rank is left waiting in a broadcast another rank skipped
    return guarded([&] {
        if (!comm)
            throw Error(DRM_ERR_ARG, "drm_index_broadcast: null communicator");
        const int rank = drm::comm_rank(comm), nranks = drm::comm_nranks(comm), device = drm::comm_device(comm);
        if (root < 0 || root >= nranks)
            throw Error(DRM_ERR_ARG, "drm_index_broadcast: root out of range");
        if (out)
            *out = nullptr;
        DRM_HIP_CHECK(hipSetDevice(device));
        hipStream_t s;
        DRM_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        struct StreamGuard {
            hipStream_t s;
            ~StreamGuard() { (void)hipStreamDestroy(s); }
        } sg{s};
        const bool is_root = rank == root;
        std::string why;
        // 1. the root's header (with its buffer checksums)
        IndexWire w{};
        if (is_root) {
            if (!root_index)
                why = "the root passes its loaded index";
            else if (root_index->dev.device != device)
                why = "the root's index lives on device " + std::to_string(root_index->dev.device) +
                      ", its communicator on device " + std::to_string(device);
            else {
                drm::DeviceIndex &r = root_index->dev;
                w = index_to_wire(r);
                void *bufs[kBcastBufs];
                index_buffers(r, bufs);
                for (int b = 0; b < kBcastBufs; ++b)
                    w.sums[b] = device_checksum(bufs[b], (int64_t)w.bytes[b], s);
            }
        } else if (!out) {
            why = "a receiving rank passes `out`";
        }
        if (!drm::comm_all_ok(comm, why.empty(), s))
            throw Error(DRM_ERR_ARG, "drm_index_broadcast: " + (why.empty() ? std::string("another rank's arguments were refused") : why));
        {
            DevBuf<uint8_t> dw(sizeof(IndexWire));
            if (is_root)
                dw.upload(reinterpret_cast<const uint8_t *>(&w));
            const drm::BcastItem hdr{dw.p, dw.p, sizeof(IndexWire)};
            drm::comm_broadcast(comm, &hdr, 1, root, s);
            dw.download(reinterpret_cast<uint8_t *>(&w));
        }
        // 2. the receiver's index (a root asking for a copy receives too)
        std::unique_ptr<drm_index> ix;
        const bool receive = out != nullptr;
        if (receive) {
            try {
                ix = index_from_wire(w, device);
            } catch (const std::exception &e) {
                why = e.what();
            }
        }
        if (!drm::comm_all_ok(comm, why.empty(), s)) {
            if (ix)
                free_index(ix->dev);
            throw Error(DRM_ERR_HIP, "drm_index_broadcast: " + (why.empty() ? std::string("another rank could not take the index") : why));
        }
        // 3. the buffers, in one grouped broadcast; each receiver checks what arrived against the root's checksums
        //    and derives the lean kernel's inline rows locally (they are a function of nbr0 + codes)
        drm::BcastItem items[kBcastBufs];
        void *src[kBcastBufs] = {};
        if (is_root)
            index_buffers(root_index->dev, src);
        void *dst[kBcastBufs] = {};
        if (receive)
            index_buffers(ix->dev, dst);
        for (int b = 0; b < kBcastBufs; ++b)
            items[b] = drm::BcastItem{src[b], receive ? dst[b] : src[b], (size_t)w.bytes[b]};
        try {
            drm::comm_broadcast(comm, items, kBcastBufs, root, s);
        } catch (...) {
            if (ix)
                free_index(ix->dev);
            throw;
        }
        if (receive) {
            try {
                for (int b = 0; b < kBcastBufs; ++b) {
                    const uint64_t got = device_checksum(dst[b], (int64_t)w.bytes[b], s);
                    if (got != w.sums[b]) {
                        char msg[160];
                        std::snprintf(msg, sizeof msg, "buffer %d (%llu bytes) arrived with checksum %016llx, the root's is "
                                      "%016llx", b, (unsigned long long)w.bytes[b], (unsigned long long)got,
                                      (unsigned long long)w.sums[b]);
                        throw Error(DRM_ERR_INTERNAL, msg);
                    }
                }
            } catch (const std::exception &e) {
                why = e.what();
                free_index(ix->dev);
                ix.reset();
            }
            if (ix) {
                try {
                    index_finish(ix.get());
                } catch (const std::exception &e) {
                    why = e.what();
                    ix.reset(); // index_finish freed its buffers
                }
            }
        }
        if (!drm::comm_all_ok(comm, why.empty(), s)) {
            if (ix)
                free_index(ix->dev);
            throw Error(DRM_ERR_INTERNAL, "drm_index_broadcast: " + (why.empty() ? std::string("another rank failed to verify the index") : why));
        }
        if (receive)
            *out = ix.release();
    });
}

int drm_index_clone(const drm_index *src, int device, drm_index **out)
{
    return guarded([&] {
        if (!src || !out)
            throw Error(DRM_ERR_ARG, "null argument");
        *out = nullptr;
        drm::DeviceIndex &r = const_cast<drm_index *>(src)->dev;
        const IndexWire w = index_to_wire(r);
        std::unique_ptr<drm_index> ix = index_from_wire(w, device);
        void *from[kBcastBufs], *to[kBcastBufs];
        index_buffers(r, from);
        index_buffers(ix->dev, to);
        try {
            // device to device (peer copies over xGMI when the devices differ; the runtime stages them if peer
            // access is off), from the source's device
            DRM_HIP_CHECK(hipSetDevice(r.device));
            DRM_HIP_CHECK(hipDeviceSynchronize());
            for (int b = 0; b < kBcastBufs; ++b)
                DRM_HIP_CHECK(hipMemcpyPeer(to[b], device, from[b], r.device, w.bytes[b]));
            DRM_HIP_CHECK(hipDeviceSynchronize());
        } catch (...) {
            free_index(ix->dev);
            throw;
        }
        index_finish(ix.get());
        *out = ix.release();
    });
}

int drm_index_free(drm_index *index)
{
    drm::exec_release(index);
    return guarded([&] {
        if (!index)
            return;
        (void)hipSetDevice(index->dev.device);
        free_index(index->dev);
        delete index;
    });
}

// diagnostics (not part of include/drm_hip.h): the round-5 first form of drm_device_checksum, and
// a delayed writer (nbytes a multiple of 4)
int drm_debug_checksum_pool(const void *d_ptr, int64_t nbytes, uint64_t *out, void *stream)
{
    return guarded([&] {
        if (!out || nbytes < 0 || (nbytes > 0 && (!d_ptr || ((uintptr_t)d_ptr & 7u) != 0u)))
            throw Error(DRM_ERR_ARG, "drm_debug_checksum_pool: needs an 8-byte aligned device pointer and an output");
        hipStream_t s = (hipStream_t)stream;
        unsigned long long *d_out = nullptr;
        DRM_HIP_CHECK(hipMallocAsync((void **)&d_out, sizeof(*d_out), s));
        DRM_HIP_CHECK(hipMemsetAsync(d_out, 0, sizeof(*d_out), s));
        const int64_t nw = (nbytes + 7) >> 3;
        if (nw > 0) {
            const int64_t blocks = std::min<int64_t>((nw + 255) / 256, 4096);
            hipLaunchKernelGGL(checksum_atomic_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const uint8_t *)d_ptr,
                               nbytes, d_out);
            DRM_HIP_CHECK(hipGetLastError());
        }
        unsigned long long h = 0;
        DRM_HIP_CHECK(hipMemcpyAsync(&h, d_out, sizeof(h), hipMemcpyDeviceToHost, s));
        DRM_HIP_CHECK(hipFreeAsync(d_out, s));
        DRM_HIP_CHECK(hipStreamSynchronize(s));
        *out = (uint64_t)h;
    });
}
int drm_debug_malloc_async(void **ptr, size_t bytes, void *stream)
{
    return guarded([&] { DRM_HIP_CHECK(hipMallocAsync(ptr, std::max<size_t>(bytes, 1), (hipStream_t)stream)); });
}
int drm_debug_free_async(void *ptr, void *stream)
{
    return guarded([&] { DRM_HIP_CHECK(hipFreeAsync(ptr, (hipStream_t)stream)); });
}
int drm_debug_delayed_fill(void *d_ptr, int64_t nbytes, int32_t value, int64_t delay_us, void *stream)
{
    return guarded([&] {
        if (!d_ptr || nbytes < 0 || (nbytes & 3) || delay_us < 0 || delay_us > 10000000)
            throw Error(DRM_ERR_ARG, "drm_debug_delayed_fill: a device pointer, nbytes % 4 == 0, delay <= 10 s");
        const uint32_t b = (uint32_t)value & 0xFFu;
        const int64_t nw = nbytes >> 2;
        hipLaunchKernelGGL(delayed_fill_kernel, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((nw + 255) / 256, 1024))),
                           dim3(256), 0, (hipStream_t)stream, (uint32_t *)d_ptr, nw, b * 0x01010101u,
                           (uint64_t)delay_us * 100u);
        DRM_HIP_CHECK(hipGetLastError());
    });
}

// diagnostic (not part of include/drm_hip.h): read and reset the section timers of a stamps build
int drm_debug_search_stamps(drm_index *index, uint64_t *out16)
{
    return guarded([&] {
        if (!index || !index->dev.stamps)
            throw Error(DRM_ERR_ARG, "index was not loaded with DRM_SEARCH_STAMPS=1");
        DRM_HIP_CHECK(hipMemcpy(out16, index->dev.stamps, 16 * sizeof(uint64_t), hipMemcpyDeviceToHost));
        DRM_HIP_CHECK(hipMemset(index->dev.stamps, 0, 16 * sizeof(uint64_t)));
    });
}

// diagnostic (not part of include/drm_hip.h): the host-mapped trace of a DRM_PQ_DEBUG build (DRM_SEARCH_TRACE=1)
int drm_debug_search_trace(drm_index *index, uint32_t **ptr, int64_t *words)
{
    return guarded([&] {
        if (!index || !ptr || !words)
            throw Error(DRM_ERR_ARG, "null argument");
        *ptr = index->dev.trace;
        *words = index->dev.trace ? drm::kTraceWords : 0;
    });
}

int drm_index_search_errors(drm_index *index, int64_t *count)
{
    return guarded([&] {
        if (!index || !count)
            throw Error(DRM_ERR_ARG, "null argument");
        uint32_t c[4] = {0, 0, 0, 0};
        if (index->dev.counter) {
            DRM_HIP_CHECK(hipDeviceSynchronize());
            DRM_HIP_CHECK(hipMemcpy(c, index->dev.counter, sizeof(c), hipMemcpyDeviceToHost));
            DRM_HIP_CHECK(hipMemset(index->dev.counter + 3, 0, sizeof(uint32_t)));
        }
        *count = (int64_t)c[3];
    });
}

int drm_index_set_search_waves(drm_index *index, int32_t waves_per_cu)
{
    return guarded([&] {
        if (!index || waves_per_cu < 0)
            throw Error(DRM_ERR_ARG, "invalid argument");
        // the per-slot workspace was reserved at load for index->dev.waves_per_cu; more slots grow it on
        // the next search, fewer use a prefix of it; 0 restores the value the index was loaded with
        index->dev.waves_per_cu = waves_per_cu > 0 ? waves_per_cu : index->dev.waves_per_cu_load;
    });
}

int drm_index_set_exact_stats(drm_index *index, int32_t on)
{
    return guarded([&] {
        if (!index)
            throw Error(DRM_ERR_ARG, "null index");
        drm::DeviceIndex &d = index->dev;
        d.exact_stats = on ? 1 : 0;
        // switched off on an index whose searches take the lean kernel: the per-slot visited bitmap (32 GB at C5) was
        // there for the count only -- release it (a search that needs it again, another kernel or exact statistics,
        // allocates it anew)
        if (!on && d.rows && d.visited) {
            DRM_HIP_CHECK(hipSetDevice(d.device));
            DRM_HIP_CHECK(hipDeviceSynchronize());
            DRM_HIP_CHECK(hipFree(d.visited));
            d.visited = nullptr;
            d.device_bytes -= (int64_t)sizeof(uint32_t) * d.n_slots * d.vis_words;
            if (d.clear_list) {
                DRM_HIP_CHECK(hipFree(d.clear_list));
                d.clear_list = nullptr;
                d.device_bytes -= (int64_t)sizeof(int32_t) * d.n_slots * d.clear_cap;
            }
            d.n_slots = 0;
            d.vis_words = 0;
        }
    });
}

int drm_index_get_info(const drm_index *index, drm_index_info *info)
{
    return guarded([&] {
        if (!index || !info)
            throw Error(DRM_ERR_ARG, "null argument");
        const drm::DeviceIndex &d = index->dev;
        info->d = d.d;
        info->ntotal = d.ntotal;
        info->pq_M = d.pq_M;
        info->pq_nbits = d.pq_nbits;
        info->M_hnsw = d.deg0 / 2;
        info->max_level = d.max_level;
        info->entry_point = d.entry_point;
        info->efConstruction = d.meta.efConstruction;
        info->efSearch = d.meta.efSearch;
        info->metric_type = d.meta.hdr.metric_type;
        info->device_bytes = d.device_bytes;
        info->device = d.device;
    });
}

int drm_search_device(drm_index *index, const float *d_x, int64_t n, int32_t k, int32_t ef, float *d_D,
                      int64_t *d_I, int32_t *d_ndis, int32_t *d_nhops, void *stream)
{
    return drm_search_device_ex(index, d_x, n, k, ef, d_D, d_I, d_ndis, d_nhops, nullptr, stream);
}

int drm_search_device_ex(drm_index *index, const float *d_x, int64_t n, int32_t k, int32_t ef, float *d_D,
                         int64_t *d_I, int32_t *d_ndis, int32_t *d_nhops, int32_t *d_nhops_upper, void *stream)
{
    return guarded([&] {
        if (!index)
            throw Error(DRM_ERR_ARG, "null index");
        if (n <= 0)
            throw Error(DRM_ERR_ARG, "Query data is empty");
        if (n >= (int64_t)1 << 31)
            throw Error(DRM_ERR_ARG, "more than 2^31-1 queries in one call");
        DRM_HIP_CHECK(hipSetDevice(index->dev.device));
        int32_t *nd = d_ndis, *nh = d_nhops;
        std::unique_ptr<DevBuf<int32_t>> tmp;
        if (!nd || !nh) {
            tmp.reset(new DevBuf<int32_t>((size_t)n * 2));
            if (!nd)
                nd = tmp->p;
            if (!nh)
                nh = tmp->p + n;
        }
        drm::launch_hnsw_search(index->dev, d_x, n, k, ef, d_D, d_I, nd, nh, d_nhops_upper, (hipStream_t)stream);
        if (tmp)
            DRM_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
    });
}

int drm_search(drm_index *index, const float *x, int64_t n, int32_t d, int32_t k, int32_t ef, float *D, int64_t *I,
               drm_search_stats *stats)
{
    return guarded([&] {
        if (!index || !x || !D || !I)
            throw Error(DRM_ERR_ARG, "null argument");
        if (n <= 0)
            throw Error(DRM_ERR_ARG, "Query data is empty"); // src/hnswpq/search.cpp:16-19
        if (d != index->dev.d)
            throw Error(DRM_ERR_ARG, "query dimension " + std::to_string(d) + " != index dimension " +
                                         std::to_string(index->dev.d));
        if (k <= 0)
            throw Error(DRM_ERR_ARG, "k must be > 0");
        DRM_HIP_CHECK(hipSetDevice(index->dev.device));
        DevBuf<float> dx((size_t)n * d), dD((size_t)n * k);
        DevBuf<int64_t> dI((size_t)n * k);
        DevBuf<int32_t> dst((size_t)n * 2);
        dx.upload(x);
        hipEvent_t e0, e1;
        DRM_HIP_CHECK(hipEventCreate(&e0));
        DRM_HIP_CHECK(hipEventCreate(&e1));
        DRM_HIP_CHECK(hipEventRecord(e0, nullptr));
        drm::launch_hnsw_search(index->dev, dx.p, n, k, ef, dD.p, dI.p, dst.p, dst.p + n, nullptr, nullptr);
        DRM_HIP_CHECK(hipEventRecord(e1, nullptr));
        DRM_HIP_CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        DRM_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        drm::check_search_errors(index->dev);
        dD.download(D);
        dI.download(I);
        if (stats) {
            std::vector<int32_t> st((size_t)n * 2);
            dst.download(st.data());
            stats->nq = n;
            stats->ndis = std::accumulate(st.begin(), st.begin() + n, (int64_t)0);
            stats->nhops = std::accumulate(st.begin() + n, st.end(), (int64_t)0);
            stats->kernel_ms = ms;
        }
    });
}

// ------------------------------------------------------------------------ fp32 (hnswlib) index
namespace {
void free_flat(drm::DeviceFlatIndex &d)
{
    void *ptrs[] = {d.vec,        d.l0,         d.l0cnt,      d.up_off,    d.up,        d.labels,  d.visited,
                    d.clear_list, d.cand_ovf_k, d.cand_ovf_i, d.top_ovf_k, d.top_ovf_i, d.counter, d.stamps,
                    };
    for (void *p : ptrs)
        if (p)
            (void)hipFree(p);
}
} // namespace

int drm_flat_index_load(const char *path, int device, drm_flat_index **out)
{
    return guarded([&] {
        if (!path || !out)
            throw Error(DRM_ERR_ARG, "null argument");
        *out = nullptr;
        drm::HnswFlatHost h = drm::read_hnswlib(path);
        if (h.d % 16 != 0)
            throw Error(DRM_ERR_UNSUPPORTED, "fp32 GPU search needs d % 16 == 0 (hnswlib L2SqrSIMD16Ext)");
        if (h.maxM0 > 4096 || h.maxM > 4096)
            throw Error(DRM_ERR_UNSUPPORTED, "maxM0/maxM > 4096");
        if (h.n > 0xFFFFFFFFll)
            throw Error(DRM_ERR_UNSUPPORTED, "more than 2^32 elements");
        DRM_HIP_CHECK(hipSetDevice(device));
        std::unique_ptr<drm_flat_index, void (*)(drm_flat_index *)> ix(new drm_flat_index(), [](drm_flat_index *p) {
            free_flat(p->dev);
            delete p;
        });
        drm::DeviceFlatIndex &d = ix->dev;
        d.device = device;
        d.d = h.d;
        d.ntotal = h.n;
        d.maxM0 = (int32_t)h.maxM0;
        d.maxM = (int32_t)h.maxM;
        d.M = (int32_t)h.M;
        d.efc = (int32_t)h.efc;
        d.maxlevel = h.maxlevel;
        d.ep = h.ep;
        const int64_t n = h.n;
        std::vector<uint32_t> l0((size_t)n * d.maxM0, 0u), cnt((size_t)n);
        for (int64_t i = 0; i < n; ++i) {
            const uint32_t *row = &h.l0[(size_t)i * (1 + h.maxM0)];
            cnt[(size_t)i] = row[0] & 0xFFFFu;
            std::memcpy(&l0[(size_t)i * d.maxM0], row + 1, sizeof(uint32_t) * cnt[(size_t)i]);
            // slots past the count hold ~0u: the kernel's row step needs no count (ids < 2^32 - 1)
            std::fill(l0.begin() + (int64_t)i * d.maxM0 + cnt[(size_t)i], l0.begin() + (int64_t)(i + 1) * d.maxM0,
                      0xFFFFFFFFu);
            if (!d.has_dup_links) { // a row listing one id twice: only its first occurrence is fresh
                std::unordered_set<uint32_t> seen;
                for (uint32_t j = 0; j < cnt[(size_t)i]; ++j)
                    if (!seen.insert(row[1 + j]).second) {
                        d.has_dup_links = 1;
                        break;
                    }
            }
        }
        if (const char *e = std::getenv("DRM_SEARCH_WAVES_PER_CU"))
            d.waves_per_cu = std::max(1, std::atoi(e));
        if (const char *e = std::getenv("DRM_SEARCH_HOP_BOUND"))
            d.hop_bound = std::max<int64_t>(0, std::atoll(e));
        if (const char *e = std::getenv("DRM_WAVE_ITEM_BOUND"))
            d.item_bound = std::max<int64_t>(0, std::atoll(e));
        if (const char *e = std::getenv("DRM_SEARCH_STAMPS"))
            if (std::atoi(e)) {
                DRM_HIP_CHECK(hipMalloc(&d.stamps, 8 * sizeof(uint64_t)));
                DRM_HIP_CHECK(hipMemset(d.stamps, 0, 8 * sizeof(uint64_t)));
            }
        d.vec = upload_vec(h.vec, d.device_bytes);
        d.l0 = upload_vec(l0, d.device_bytes);
        d.l0cnt = upload_vec(cnt, d.device_bytes);
        d.up_off = upload_vec(h.up_off, d.device_bytes);
        d.up = upload_vec(h.up.empty() ? std::vector<uint32_t>(1, 0u) : h.up, d.device_bytes);
        d.labels = upload_vec(h.labels, d.device_bytes);
        h.vec.clear();
        h.vec.shrink_to_fit();
        h.l0.clear();
        h.l0.shrink_to_fit();
        h.up.clear();
        h.up.shrink_to_fit();
        d.meta = std::move(h);
        *out = ix.release();
    });
}

int drm_flat_index_free(drm_flat_index *index)
{
    return guarded([&] {
        if (!index)
            return;
        free_flat(index->dev);
        delete index;
    });
}

int drm_flat_index_get_info(const drm_flat_index *index, drm_flat_index_info *info)
{
    return guarded([&] {
        if (!index || !info)
            throw Error(DRM_ERR_ARG, "null argument");
        const drm::DeviceFlatIndex &d = index->dev;
        info->d = d.d;
        info->ntotal = d.ntotal;
        info->M = d.M;
        info->maxM0 = d.maxM0;
        info->maxM = d.maxM;
        info->max_level = d.maxlevel;
        info->entry_point = d.ep;
        info->efConstruction = d.efc;
        info->device_bytes = d.device_bytes;
    });
}

int drm_flat_search_device(drm_flat_index *index, const float *d_x, int64_t n, int32_t k, int32_t ef, float *d_D,
                           uint64_t *d_labels, int32_t *d_ndis, int32_t *d_nhops, int32_t *d_nhops_upper,
                           void *stream)
{
    return guarded([&] {
        if (!index || (n > 0 && (!d_x || !d_D || !d_labels || !d_ndis || !d_nhops)))
            throw Error(DRM_ERR_ARG, "null argument");
        if (n <= 0)
            throw Error(DRM_ERR_ARG, "Query data is empty"); // src/hnswlib_dir/search.cpp:20-23
        if (n >= (int64_t)1 << 31)
            throw Error(DRM_ERR_ARG, "more than 2^31-1 queries in one call");
        DRM_HIP_CHECK(hipSetDevice(index->dev.device));
        drm::launch_hnsw_flat_search(index->dev, d_x, n, k, ef, d_D, d_labels, d_ndis, d_nhops, d_nhops_upper,
                                     (hipStream_t)stream);
    });
}

int drm_debug_flat_stamps(drm_flat_index *index, uint64_t *out8)
{
    return guarded([&] {
        if (!index || !index->dev.stamps)
            throw Error(DRM_ERR_ARG, "index was not loaded with DRM_SEARCH_STAMPS=1");
        DRM_HIP_CHECK(hipMemcpy(out8, index->dev.stamps, 8 * sizeof(uint64_t), hipMemcpyDeviceToHost));
        DRM_HIP_CHECK(hipMemset(index->dev.stamps, 0, 8 * sizeof(uint64_t)));
    });
}

int drm_flat_search_overflows(drm_flat_index *index, int64_t *count)
{
    return guarded([&] {
        if (!index || !count)
            throw Error(DRM_ERR_ARG, "null argument");
        uint32_t c[2] = {0, 0};
        if (index->dev.counter) {
            DRM_HIP_CHECK(hipDeviceSynchronize());
            DRM_HIP_CHECK(hipMemcpy(c, index->dev.counter, sizeof(c), hipMemcpyDeviceToHost));
        }
        *count = (int64_t)c[1];
    });
}

int drm_flat_search_errors(drm_flat_index *index, int64_t *count)
{
    return guarded([&] {
        if (!index || !count)
            throw Error(DRM_ERR_ARG, "null argument");
        uint32_t c[4] = {0, 0, 0, 0};
        if (index->dev.counter) {
            DRM_HIP_CHECK(hipDeviceSynchronize());
            DRM_HIP_CHECK(hipMemcpy(c, index->dev.counter, sizeof(c), hipMemcpyDeviceToHost));
            DRM_HIP_CHECK(hipMemset(index->dev.counter + 3, 0, sizeof(uint32_t)));
        }
        *count = (int64_t)c[3];
    });
}

int drm_flat_search(drm_flat_index *index, const float *x, int64_t n, int32_t d, int32_t k, int32_t ef, float *D,
                    uint64_t *labels, drm_search_stats *stats)
{
    return guarded([&] {
        if (!index || !x || !D || !labels)
            throw Error(DRM_ERR_ARG, "null argument");
        if (n <= 0)
            throw Error(DRM_ERR_ARG, "Query data is empty"); // src/hnswlib_dir/search.cpp:20-23
        if (n >= (int64_t)1 << 31)
            throw Error(DRM_ERR_ARG, "more than 2^31-1 queries in one call");
        if (d != index->dev.d)
            throw Error(DRM_ERR_ARG, "query dimension " + std::to_string(d) + " != index dimension " +
                                         std::to_string(index->dev.d));
        if (k <= 0)
            throw Error(DRM_ERR_ARG, "k must be > 0");
        DRM_HIP_CHECK(hipSetDevice(index->dev.device));
        DevBuf<float> dx((size_t)n * d), dD((size_t)n * k);
        DevBuf<uint64_t> dL((size_t)n * k);
        DevBuf<int32_t> dst((size_t)n * 2);
        dx.upload(x);
        hipEvent_t e0, e1;
        DRM_HIP_CHECK(hipEventCreate(&e0));
        DRM_HIP_CHECK(hipEventCreate(&e1));
        DRM_HIP_CHECK(hipEventRecord(e0, nullptr));
        drm::launch_hnsw_flat_search(index->dev, dx.p, n, k, ef, dD.p, dL.p, dst.p, dst.p + n, nullptr, nullptr);
        DRM_HIP_CHECK(hipEventRecord(e1, nullptr));
        DRM_HIP_CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        DRM_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        uint32_t c[4] = {0, 0, 0, 0};
        DRM_HIP_CHECK(hipMemcpy(c, index->dev.counter, sizeof(c), hipMemcpyDeviceToHost));
        if (c[3]) {
            DRM_HIP_CHECK(hipMemset(index->dev.counter + 3, 0, sizeof(uint32_t)));
            throw Error(DRM_ERR_INTERNAL, std::to_string(c[3]) + " queries exceeded the search's hop bound or waves "
                                                                 "their work-item bound: search state broken");
        }
        if (c[1])
            throw Error(DRM_ERR_UNSUPPORTED, std::to_string(c[1]) + " queries outgrew the GPU candidate heap");
        dD.download(D);
        dL.download(labels);
        if (stats) {
            std::vector<int32_t> st((size_t)n * 2);
            dst.download(st.data());
            stats->nq = n;
            stats->ndis = std::accumulate(st.begin(), st.begin() + n, (int64_t)0);
            stats->nhops = std::accumulate(st.begin() + n, st.end(), (int64_t)0);
            stats->kernel_ms = ms;
        }
    });
}

// ------------------------------------------------------------------------------------ SW
int drm_sw_scores(const uint8_t *s1, const int64_t *off1, const int32_t *len1, const uint8_t *s2,
                  const int64_t *off2, const int32_t *len2, int64_t npairs, int32_t *scores)
{
    return guarded([&] {
        if (npairs <= 0)
            return;
        if (!s1 || !off1 || !len1 || !s2 || !off2 || !len2 || !scores)
            throw Error(DRM_ERR_ARG, "null argument");
        int64_t n1 = 0, n2 = 0;
        int max2 = 0;
        for (int64_t p = 0; p < npairs; ++p) {
            if (len1[p] < 0 || len2[p] < 0)
                throw Error(DRM_ERR_ARG, "negative length");
            n1 = std::max(n1, off1[p] + len1[p]);
            n2 = std::max(n2, off2[p] + len2[p]);
            max2 = std::max(max2, len2[p]);
        }
        DevBuf<uint8_t> d1((size_t)std::max<int64_t>(n1, 1)), d2((size_t)std::max<int64_t>(n2, 1));
        DevBuf<int64_t> do1((size_t)npairs), do2((size_t)npairs);
        DevBuf<int32_t> dl1((size_t)npairs), dl2((size_t)npairs), ds((size_t)npairs);
        if (n1)
            DRM_HIP_CHECK(hipMemcpy(d1.p, s1, (size_t)n1, hipMemcpyHostToDevice));
        if (n2)
            DRM_HIP_CHECK(hipMemcpy(d2.p, s2, (size_t)n2, hipMemcpyHostToDevice));
        do1.upload(off1);
        do2.upload(off2);
        dl1.upload(len1);
        dl2.upload(len2);
        drm::launch_sw_pairs(d1.p, do1.p, dl1.p, d2.p, do2.p, dl2.p, npairs, ds.p, max2, nullptr);
        DRM_HIP_CHECK(hipDeviceSynchronize());
        ds.download(scores);
    });
}

namespace {
// the opt-in banded SW (drm_refs_set_sw_band): 0 (full DP, the reference's) or 8 / 16 / 32
void check_sw_band(int32_t band)
{
    if (band != 0 && band != 8 && band != 16 && band != 32)
        throw Error(DRM_ERR_ARG, "SW band must be 0 (full DP), 8, 16 or 32, got " + std::to_string(band));
}
// the initial band of a new handle: DRM_SW_BAND (unset: 0), so that the pipeline CLI can opt in without new argv
int32_t env_sw_band()
{
    const char *e = std::getenv("DRM_SW_BAND");
    const int32_t band = e ? (int32_t)std::atoi(e) : 0;
    check_sw_band(band);
    return band;
}
} // namespace

int drm_refs_create(const uint8_t *windows, int64_t n_ref, int32_t ref_len, int64_t row_stride, int device,
                    drm_refs **out)
{
    return guarded([&] {
        if (!out || (!windows && n_ref > 0))
            throw Error(DRM_ERR_ARG, "null argument");
        if (n_ref < 0 || ref_len < 0 || row_stride < ref_len)
            throw Error(DRM_ERR_ARG, "invalid window table shape");
        DRM_HIP_CHECK(hipSetDevice(device));
        std::unique_ptr<drm_refs> r(new drm_refs());
        r->dev.device = device;
        r->dev.sw_band = env_sw_band();
        r->dev.n_ref = n_ref;
        r->dev.ref_len = ref_len;
        r->dev.row_stride = std::max<int64_t>(16, ((int64_t)ref_len + 15) / 16 * 16);
        const size_t bytes = (size_t)std::max<int64_t>(n_ref, 1) * (size_t)r->dev.row_stride;
        DRM_HIP_CHECK(drm::malloc_big((void **)&r->dev.windows, bytes, drm::kBigWindows));
        DRM_HIP_CHECK(hipMemset(r->dev.windows, 0, bytes));
        if (n_ref > 0 && ref_len > 0) {
            // pageable host rows of ref_len bytes: a 2D host-to-device copy of tens of millions of short
            // rows is slow, so contiguous chunks go up in 1D copies and are re-pitched on the device
            const int64_t chunk = std::max<int64_t>(1, ((int64_t)256 << 20) / row_stride);
            uint8_t *stage = nullptr;
            DRM_HIP_CHECK(hipMalloc(&stage, (size_t)std::min(chunk, n_ref) * (size_t)row_stride));
            for (int64_t r0 = 0; r0 < n_ref; r0 += chunk) {
                const int64_t nr = std::min(chunk, n_ref - r0);
                DRM_HIP_CHECK(hipMemcpy(stage, windows + r0 * row_stride, (size_t)nr * (size_t)row_stride,
                                        hipMemcpyHostToDevice));
                DRM_HIP_CHECK(hipMemcpy2D(r->dev.windows + r0 * r->dev.row_stride, (size_t)r->dev.row_stride, stage,
                                          (size_t)row_stride, (size_t)ref_len, (size_t)nr, hipMemcpyDeviceToDevice));
            }
            DRM_HIP_CHECK(hipFree(stage));
        }
        *out = r.release();
    });
}

int drm_refs_create_genome(const uint8_t *genome, int64_t len, int32_t ref_len, int device, drm_refs **out)
{
    return guarded([&] {
        if (!out || (!genome && len > 0))
            throw Error(DRM_ERR_ARG, "null argument");
        if (len < 0 || ref_len < 0)
            throw Error(DRM_ERR_ARG, "invalid genome / ref_len");
        if (len >= ((int64_t)1 << 31))
            throw Error(DRM_ERR_UNSUPPORTED, "genomes of 2^31 bases or more are not supported (32-bit window ids)");
        DRM_HIP_CHECK(hipSetDevice(device));
        std::unique_ptr<drm_refs> r(new drm_refs());
        r->dev.device = device;
        r->dev.sw_band = env_sw_band();
        r->dev.ref_len = ref_len;
        r->dev.row_stride = 16;
        r->dev.glen = len;
        r->dev.n_ref = len >= ref_len ? 2 * (len - ref_len + 1) : 0;
        DRM_HIP_CHECK(drm::malloc_big((void **)&r->dev.genome, (size_t)std::max<int64_t>(len, 1), drm::kBigWindows));
        if (len > 0)
            DRM_HIP_CHECK(hipMemcpy(r->dev.genome, genome, (size_t)len, hipMemcpyHostToDevice));
        *out = r.release();
    });
}

int drm_refs_is_genome(const drm_refs *refs, int *is_genome)
{
    return guarded([&] {
        if (!refs || !is_genome)
            throw Error(DRM_ERR_ARG, "null argument");
        *is_genome = refs->dev.genome ? 1 : 0;
    });
}

int drm_refs_get_info(const drm_refs *refs, int64_t *n_ref, int32_t *ref_len, int *device)
{
    return guarded([&] {
        if (!refs)
            throw Error(DRM_ERR_ARG, "null argument");
        if (n_ref)
            *n_ref = refs->dev.n_ref;
        if (ref_len)
            *ref_len = refs->dev.ref_len;
        if (device)
            *device = refs->dev.device;
    });
}

int drm_refs_set_sw_band(drm_refs *refs, int32_t band)
{
    return guarded([&] {
        if (!refs)
            throw Error(DRM_ERR_ARG, "null argument");
        check_sw_band(band);
        refs->dev.sw_band = band;
    });
}

int drm_refs_get_sw_band(const drm_refs *refs, int32_t *band)
{
    return guarded([&] {
        if (!refs || !band)
            throw Error(DRM_ERR_ARG, "null argument");
        *band = refs->dev.sw_band;
    });
}

int drm_refs_free(drm_refs *refs)
{
    return guarded([&] {
        if (!refs)
            return;
        (void)hipSetDevice(refs->dev.device);
        for (void *p : {(void *)refs->dev.windows, (void *)refs->dev.ws_ids, (void *)refs->dev.ws_scores,
                        (void *)refs->dev.ws_ncand, (void *)refs->dev.genome, (void *)refs->dev.emb})
            if (p)
                (void)hipFree(p);
        delete refs;
    });
}

static drm::RerankArgs make_rerank_args(drm_refs *refs, const int64_t *nb, int64_t nq, int32_t kk, const uint8_t *q,
                                        const int32_t *ql, int32_t q_stride, int64_t stride, int32_t k,
                                        int32_t k_clusters, int32_t *ts, uint64_t *ti, int32_t *st)
{
    if (!refs)
        throw Error(DRM_ERR_ARG, "null refs");
    if (stride < 1)
        throw Error(DRM_ERR_ARG, "stride must be >= 1");
    if (k < 0 || k_clusters < 0 || kk < 0)
        throw Error(DRM_ERR_ARG, "negative k / k_clusters / kk");
    if ((int64_t)k > (int64_t)k_clusters * 2 * stride) // post_processor.cpp:486-489
        throw Error(DRM_ERR_K, "Final k too large. Ensure k < k_clusters * 2 * stride to have enough candidates.");
    drm::RerankArgs a{};
    a.genome = refs->dev.genome;
    a.glen = refs->dev.glen;
    a.refs = refs->dev.windows;
    a.n_ref = refs->dev.n_ref;
    a.ref_len = refs->dev.ref_len;
    a.row_stride = refs->dev.row_stride;
    a.neighbors = nb;
    a.kk = kk;
    a.k_clusters = k_clusters;
    a.stride = stride;
    a.queries = q;
    a.q_len = ql;
    a.q_stride = q_stride;
    a.k = k;
    a.nq = nq;
    a.top_scores = ts;
    a.top_ids = ti;
    a.status = st;
    return a;
}

static void require_mode(const drm_refs *refs, bool dynamic)
{
    if (!refs)
        throw Error(DRM_ERR_ARG, "null refs");
    if (dynamic && !refs->dev.genome)
        throw Error(DRM_ERR_ARG, "post_process_sw_dynamic needs a genome handle (drm_refs_create_genome)");
    if (!dynamic && refs->dev.genome)
        throw Error(DRM_ERR_ARG, "post_process_sw_static needs a window table (drm_refs_create), not a genome");
}

static int post_process_device(bool dynamic, drm_refs *refs, const int64_t *d_neighbors, int64_t nq, int32_t kk,
                               const uint8_t *d_queries, const int32_t *d_q_len, int32_t q_stride, int64_t stride,
                               int32_t k, int32_t k_clusters, int32_t *d_top_scores, uint64_t *d_top_ids,
                               int32_t *d_status, void *stream)
{
    return guarded([&] {
        require_mode(refs, dynamic);
        drm::RerankArgs a = make_rerank_args(refs, d_neighbors, nq, kk, d_queries, d_q_len, q_stride, stride, k,
                                             k_clusters, d_top_scores, d_top_ids, d_status);
        DRM_HIP_CHECK(hipSetDevice(refs->dev.device));
        // max query length bounded by the row stride of the query buffer
        drm::launch_sw_rerank(refs->dev, a, q_stride, (hipStream_t)stream);
    });
}

int drm_post_process_sw_static_device(drm_refs *refs, const int64_t *d_neighbors, int64_t nq, int32_t kk,
                                      const uint8_t *d_queries, const int32_t *d_q_len, int32_t q_stride,
                                      int64_t stride, int32_t k, int32_t k_clusters, int32_t *d_top_scores,
                                      uint64_t *d_top_ids, int32_t *d_status, void *stream)
{
    return post_process_device(false, refs, d_neighbors, nq, kk, d_queries, d_q_len, q_stride, stride, k, k_clusters,
                               d_top_scores, d_top_ids, d_status, stream);
}

int drm_post_process_sw_dynamic_device(drm_refs *refs, const int64_t *d_neighbors, int64_t nq, int32_t kk,
                                       const uint8_t *d_queries, const int32_t *d_q_len, int32_t q_stride,
                                       int64_t stride, int32_t k, int32_t k_clusters, int32_t *d_top_scores,
                                       uint64_t *d_top_ids, int32_t *d_status, void *stream)
{
    return post_process_device(true, refs, d_neighbors, nq, kk, d_queries, d_q_len, q_stride, stride, k, k_clusters,
                               d_top_scores, d_top_ids, d_status, stream);
}

static int post_process_host(bool dynamic, drm_refs *refs, const int64_t *neighbors, int64_t nq, int32_t kk,
                             const uint8_t *queries, const int32_t *q_len, int32_t q_stride, int64_t stride,
                             int32_t k, int32_t k_clusters, int32_t *top_scores, uint64_t *top_ids, int32_t *counts,
                             int64_t *bad_query)
{
    return guarded([&] {
        require_mode(refs, dynamic);
        if (bad_query)
            *bad_query = -1;
        if (nq <= 0)
            return;
        if (!neighbors || !queries || !q_len || !top_scores || !top_ids || !counts)
            throw Error(DRM_ERR_ARG, "null argument");
        int max_q = 0;
        for (int64_t i = 0; i < nq; ++i) {
            if (q_len[i] < 0 || q_len[i] > q_stride)
                throw Error(DRM_ERR_ARG, "query length outside [0, q_stride]");
            max_q = std::max(max_q, q_len[i]);
        }
        drm::RerankArgs a = make_rerank_args(refs, nullptr, nq, kk, nullptr, nullptr, q_stride, stride, k,
                                             k_clusters, nullptr, nullptr, nullptr);
        DRM_HIP_CHECK(hipSetDevice(refs->dev.device));
        DevBuf<int64_t> dn((size_t)nq * kk);
        DevBuf<uint8_t> dq((size_t)nq * q_stride);
        DevBuf<int32_t> dl((size_t)nq), dst((size_t)nq), ds((size_t)nq * k);
        DevBuf<uint64_t> di((size_t)nq * k);
        if (dn.n)
            dn.upload(neighbors);
        if (dq.n)
            dq.upload(queries);
        dl.upload(q_len);
        a.neighbors = dn.p;
        a.queries = dq.p;
        a.q_len = dl.p;
        a.top_scores = ds.p;
        a.top_ids = di.p;
        a.status = dst.p;
        drm::launch_sw_rerank(refs->dev, a, max_q, nullptr);
        DRM_HIP_CHECK(hipDeviceSynchronize());
        std::vector<int32_t> st((size_t)nq);
        dst.download(st.data());
        if (ds.n) {
            ds.download(top_scores);
            di.download(top_ids);
        }
        int64_t first_bad = -1, first_over = -1;
        for (int64_t i = 0; i < nq; ++i) {
            counts[i] = st[(size_t)i] > 0 ? st[(size_t)i] : 0;
            if (st[(size_t)i] == -1 && first_bad < 0)
                first_bad = i;
            if ((st[(size_t)i] == -2 || st[(size_t)i] == -3) && first_over < 0)
                first_over = i;
        }
        if (first_over >= 0)
            throw Error(DRM_ERR_UNSUPPORTED, "query " + std::to_string(first_over) + " expands to more than " +
                                                 std::to_string(drm::kMaxCands) +
                                                 " candidates or exceeds the SW kernels' limits (query length; banded: 256"
                                                 " bytes, 7 distinct query bytes)");
        if (first_bad >= 0) {
            if (bad_query)
                *bad_query = first_bad;
            // count the candidates of the offending query for the reference's message
            const int64_t *nb = neighbors + first_bad * kk;
            int64_t nc = 0;
            // static lookup checks ids against the window count, dynamic against the genome length
            const uint64_t limit = dynamic ? (uint64_t)refs->dev.glen : (uint64_t)refs->dev.n_ref;
            for (int i = 0; i < std::min(k_clusters, kk); ++i) {
                uint64_t id = (uint64_t)nb[i];
                if (stride == 1) {
                    nc += dynamic || id < limit;
                } else {
                    uint64_t act = id * (uint64_t)stride;
                    if (act >= limit)
                        continue;
                    uint64_t s0 = act >= (uint64_t)(stride - 1) ? act - stride + 1 : 0;
                    nc += (int64_t)(std::min<uint64_t>(act + stride, limit) - s0);
                }
            }
            throw Error(DRM_ERR_CANDS,
                        "Not enough candidates (" + std::to_string(nc) + " < " + std::to_string(k) + ")");
        }
    });
}

int drm_post_process_sw_static(drm_refs *refs, const int64_t *neighbors, int64_t nq, int32_t kk,
                               const uint8_t *queries, const int32_t *q_len, int32_t q_stride, int64_t stride,
                               int32_t k, int32_t k_clusters, int32_t *top_scores, uint64_t *top_ids,
                               int32_t *counts, int64_t *bad_query)
{
    return post_process_host(false, refs, neighbors, nq, kk, queries, q_len, q_stride, stride, k, k_clusters,
                             top_scores, top_ids, counts, bad_query);
}

int drm_post_process_sw_dynamic(drm_refs *refs, const int64_t *neighbors, int64_t nq, int32_t kk,
                                const uint8_t *queries, const int32_t *q_len, int32_t q_stride, int64_t stride,
                                int32_t k, int32_t k_clusters, int32_t *top_scores, uint64_t *top_ids,
                                int32_t *counts, int64_t *bad_query)
{
    return post_process_host(true, refs, neighbors, nq, kk, queries, q_len, q_stride, stride, k, k_clusters,
                             top_scores, top_ids, counts, bad_query);
}

// ------------------------------------------------------------------------------- L2 rerank
static drm::L2Args make_l2_args(drm_refs *refs, bool dynamic, const int64_t *nb, int64_t nq, int32_t kk,
                                const float *qe, int32_t d, int64_t stride, int32_t k, int32_t k_clusters, float *td,
                                uint64_t *ti, int32_t *st)
{
    require_mode(refs, dynamic);
    if (!refs->dev.emb)
        throw Error(DRM_ERR_ARG, "the window table has no embeddings: call drm_refs_embed first");
    if (d != refs->dev.emb_dim)
        throw Error(DRM_ERR_ARG, "Vector sizes mismatch: " + std::to_string(refs->dev.emb_dim) + " vs " +
                                     std::to_string(d)); // calc_l2_dist, metrics.cpp:50-53
    if (stride < 1)
        throw Error(DRM_ERR_ARG, "stride must be >= 1");
    if (nq < 0 || kk < 0 || k_clusters < 0 || k < 0)
        throw Error(DRM_ERR_ARG, "negative nq / kk / k / k_clusters");
    drm::L2Args a{};
    a.emb = refs->dev.emb;
    a.d = d;
    a.neighbors = nb;
    a.kk = kk;
    a.stride = stride;
    a.query_emb = qe;
    a.nq = nq;
    a.top_dists = td;
    a.top_ids = ti;
    a.status = st;
    if (!dynamic) { // post_process_l2_static: every label, kk*stride boundaries, batch_reranker k = k_clusters
        a.limit = refs->dev.n_ref;
        a.lpq = kk;
        a.nc = (int32_t)(stride == 1 ? kk : (int64_t)kk * stride);
        a.k = k_clusters;
    } else { // post_process_l2_dynamic(_streaming), stride > 1 (:575-590, :617-627): min(k_clusters, kk) labels,
             // (2*stride - 1) boundaries per label, positions checked against the genome length, k rows
        if (stride == 1)
            throw Error(DRM_ERR_ARG, "post_process_l2_dynamic at stride 1 reranks nothing: its rows are the first "
                                     "min(k, k_clusters) search neighbours with their search distances");
        if ((int64_t)k > (int64_t)k_clusters * 2 * stride) // :566-569
            throw Error(DRM_ERR_K, "Final k too large. Ensure k < k_clusters * 2 * stride to have enough candidates.");
        a.limit = refs->dev.glen;
        a.lpq = std::min(k_clusters, kk);
        a.nc = (int32_t)((int64_t)a.lpq * (2 * stride - 1));
        a.k = k;
    }
    if ((int64_t)a.nc > drm::kMaxCands)
        throw Error(DRM_ERR_UNSUPPORTED, "more than 1024 candidates per query in the GPU L2 rerank");
    return a;
}

static int l2_device(bool dynamic, drm_refs *refs, const int64_t *d_neighbors, int64_t nq, int32_t kk,
                     const float *d_query_emb, int32_t d, int64_t stride, int32_t k, int32_t k_clusters,
                     float *d_top_dists, uint64_t *d_top_ids, int32_t *d_status, void *stream)
{
    return guarded([&] {
        drm::L2Args a = make_l2_args(refs, dynamic, d_neighbors, nq, kk, d_query_emb, d, stride, k, k_clusters,
                                     d_top_dists, d_top_ids, d_status);
        DRM_HIP_CHECK(hipSetDevice(refs->dev.device));
        drm::launch_l2_rerank(refs->dev, a, (hipStream_t)stream);
    });
}

static int l2_host(bool dynamic, drm_refs *refs, const int64_t *neighbors, int64_t nq, int32_t kk,
                   const float *query_emb, int32_t d, int64_t stride, int32_t k, int32_t k_clusters, float *top_dists,
                   uint64_t *top_ids, int32_t *counts, int64_t *bad_query)
{
    return guarded([&] {
        drm::L2Args a = make_l2_args(refs, dynamic, nullptr, nq, kk, nullptr, d, stride, k, k_clusters, nullptr,
                                     nullptr, nullptr);
        if (bad_query)
            *bad_query = -1;
        if (nq <= 0)
            return;
        if (!neighbors || !query_emb || !top_dists || !top_ids || !counts)
            throw Error(DRM_ERR_ARG, "null argument");
        DRM_HIP_CHECK(hipSetDevice(refs->dev.device));
        const size_t rows = (size_t)nq * (size_t)a.k;
        DevBuf<int64_t> dn((size_t)nq * kk);
        DevBuf<float> dqe((size_t)nq * d), dd(rows);
        DevBuf<int32_t> dst((size_t)nq);
        DevBuf<uint64_t> di(rows);
        if (dn.n)
            dn.upload(neighbors);
        dqe.upload(query_emb);
        a.neighbors = dn.p;
        a.query_emb = dqe.p;
        a.top_dists = dd.p;
        a.top_ids = di.p;
        a.status = dst.p;
        drm::launch_l2_rerank(refs->dev, a, nullptr);
        DRM_HIP_CHECK(hipDeviceSynchronize());
        std::vector<int32_t> st((size_t)nq);
        dst.download(st.data());
        if (dd.n) {
            dd.download(top_dists);
            di.download(top_ids);
        }
        int64_t first_bad = -1, first_ids = -1;
        for (int64_t i = 0; i < nq; ++i) {
            counts[i] = st[(size_t)i] > 0 ? st[(size_t)i] : 0;
            if (st[(size_t)i] == -1 && first_bad < 0)
                first_bad = i;
            if (st[(size_t)i] == -4 && first_ids < 0)
                first_ids = i;
        }
        if (first_ids >= 0) {
            if (bad_query)
                *bad_query = first_ids;
            throw Error(DRM_ERR_ARG, "Invalid mapping index in expansion (query " + std::to_string(first_ids) +
                                         ": a label outside the window table, or a candidate range past the "
                                         "expanded stream)"); // post_processor.cpp:1100-1106
        }
        if (first_bad >= 0) {
            if (bad_query)
                *bad_query = first_bad;
            throw Error(DRM_ERR_CANDS, "Not enough candidates (" + std::to_string(a.nc) + " < " +
                                           std::to_string(a.k) + ") for query " +
                                           std::to_string(first_bad)); // reranker.cpp:154-158
        }
    });
}

int drm_refs_embed(drm_refs *refs, drm_encoder *enc, void *stream)
{
    return guarded([&] {
        if (!refs || !enc)
            throw Error(DRM_ERR_ARG, "null argument");
        if (refs->dev.device != enc->dev.device)
            throw Error(DRM_ERR_ARG, "window table and encoder live on different devices");
        if (refs->dev.ref_len < 2)
            throw Error(DRM_ERR_ARG, "windows shorter than 2 bytes cannot be vectorized");
        DRM_HIP_CHECK(hipSetDevice(refs->dev.device));
        hipStream_t s = (hipStream_t)stream;
        const bool genome = refs->dev.genome != nullptr;
        // a genome handle: windows [0, glen), the positions the dynamic sparse expansion can reach
        const int64_t n = genome ? refs->dev.glen : refs->dev.n_ref, d = 128;
        if (refs->dev.emb && refs->dev.emb_rows != n) {
            DRM_HIP_CHECK(hipFree(refs->dev.emb));
            refs->dev.emb = nullptr;
        }
        if (!refs->dev.emb) {
            // n x 512 B: a genome handle embeds one row per base (a 3 Gbp genome would need ~1.5 TB), so the table
            // is checked against the device's free memory before it is asked for
            const size_t bytes = sizeof(float) * (size_t)std::max<int64_t>(n, 1) * d;
            size_t free_b = 0, total_b = 0;
            DRM_HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
            if (bytes > free_b)
                throw Error(DRM_ERR_UNSUPPORTED,
                            "window-embedding table of " + std::to_string(n) + " rows needs " +
                                std::to_string(bytes >> 30) + " GiB of device memory, " + std::to_string(free_b >> 30) +
                                " GiB are free (a genome handle embeds one window per base)");
            DRM_HIP_CHECK(drm::malloc_big((void **)&refs->dev.emb, bytes, drm::kBigWindows));
        }
        refs->dev.emb_dim = (int32_t)d;
        refs->dev.emb_rows = n;
        const int64_t chunk = std::min<int64_t>(std::max<int64_t>(n, 1), (int64_t)4 << 20);
        DevBuf<int32_t> lens((size_t)chunk);
        const int64_t rs = std::max<int64_t>(16, ((int64_t)refs->dev.ref_len + 15) / 16 * 16);
        DevBuf<uint8_t> rows(genome ? (size_t)chunk * (size_t)rs : 0);
        if (!genome) {
            std::vector<int32_t> h((size_t)chunk, refs->dev.ref_len);
            lens.upload(h.data());
        }
        for (int64_t r0 = 0; r0 < n; r0 += chunk) {
            const int64_t m = std::min(chunk, n - r0);
            if (genome) {
                drm::launch_genome_rows(refs->dev, r0, m, rows.p, rs, lens.p, s);
                drm::launch_encode(enc->dev, rows.p, lens.p, m, rs, refs->dev.emb + r0 * d, s);
            } else {
                drm::launch_encode(enc->dev, refs->dev.windows + r0 * refs->dev.row_stride, lens.p, m,
                                   refs->dev.row_stride, refs->dev.emb + r0 * d, s);
            }
        }
        DRM_HIP_CHECK(hipStreamSynchronize(s));
    });
}

int drm_refs_embeddings(drm_refs *refs, const float **d_emb, int32_t *dim)
{
    return guarded([&] {
        if (!refs || !d_emb)
            throw Error(DRM_ERR_ARG, "null argument");
        *d_emb = refs->dev.emb;
        if (dim)
            *dim = refs->dev.emb_dim;
    });
}

int drm_post_process_l2_static_device(drm_refs *refs, const int64_t *d_neighbors, int64_t nq, int32_t kk,
                                      const float *d_query_emb, int32_t d, int64_t stride, int32_t k_clusters,
                                      float *d_top_dists, uint64_t *d_top_ids, int32_t *d_status, void *stream)
{
    return l2_device(false, refs, d_neighbors, nq, kk, d_query_emb, d, stride, k_clusters, k_clusters, d_top_dists,
                     d_top_ids, d_status, stream);
}

int drm_post_process_l2_static(drm_refs *refs, const int64_t *neighbors, int64_t nq, int32_t kk,
                               const float *query_emb, int32_t d, int64_t stride, int32_t k_clusters,
                               float *top_dists, uint64_t *top_ids, int32_t *counts, int64_t *bad_query)
{
    return l2_host(false, refs, neighbors, nq, kk, query_emb, d, stride, k_clusters, k_clusters, top_dists, top_ids,
                   counts, bad_query);
}

int drm_post_process_l2_dynamic_device(drm_refs *refs, const int64_t *d_neighbors, int64_t nq, int32_t kk,
                                       const float *d_query_emb, int32_t d, int64_t stride, int32_t k,
                                       int32_t k_clusters, float *d_top_dists, uint64_t *d_top_ids, int32_t *d_status,
                                       void *stream)
{
    return l2_device(true, refs, d_neighbors, nq, kk, d_query_emb, d, stride, k, k_clusters, d_top_dists, d_top_ids,
                     d_status, stream);
}

int drm_post_process_l2_dynamic(drm_refs *refs, const int64_t *neighbors, int64_t nq, int32_t kk,
                                const float *query_emb, int32_t d, int64_t stride, int32_t k, int32_t k_clusters,
                                float *top_dists, uint64_t *top_ids, int32_t *counts, int64_t *bad_query)
{
    return l2_host(true, refs, neighbors, nq, kk, query_emb, d, stride, k, k_clusters, top_dists, top_ids, counts,
                   bad_query);
}

} // extern "C"

// ------------------------------------------------------------------------------- read encoder
static void check_seqs(const uint8_t *seqs, const int32_t *lens, int64_t n, int64_t stride)
{
    if (n < 0 || (n > 0 && (!seqs || !lens)) || stride <= 0) throw Error(DRM_ERR_ARG, "invalid sequence batch");
    for (int64_t i = 0; i < n; ++i)
        if (lens[i] < 2 || lens[i] > stride)
            throw Error(DRM_ERR_ARG, "sequence " + std::to_string(i) + " has length " + std::to_string(lens[i]) +
                                         " (need 2 <= len <= stride)");
}

extern "C" int drm_encoder_load(const char *model_path, int device, drm_encoder **out)
{
    return guarded([&] {
        if (!model_path || !out) throw Error(DRM_ERR_ARG, "null argument");
        drm::EncoderHost h = drm::read_encoder(model_path);
        auto e = std::make_unique<drm_encoder>();
        try {
            drm::encoder_upload(e->dev, h, device);
        } catch (...) {
            drm::encoder_release(e->dev);
            throw;
        }
        if (const char *v = getenv("DRM_ENC_TILES")) e->dev.max_tiles_per_launch = std::max(1, atoi(v));
        *out = e.release();
    });
}

extern "C" int drm_encoder_export(const char *model_path, const char *out_path)
{
    return guarded([&] {
        if (!model_path || !out_path) throw Error(DRM_ERR_ARG, "null argument");
        drm::write_encoder(drm::read_encoder(model_path), out_path);
    });
}

extern "C" int drm_encoder_free(drm_encoder *enc)
{
    return guarded([&] {
        if (!enc) return;
        drm::encoder_release(enc->dev);
        delete enc;
    });
}

extern "C" int drm_encoder_get_info(const drm_encoder *enc, drm_encoder_info *info)
{
    return guarded([&] {
        if (!enc || !info) throw Error(DRM_ERR_ARG, "null argument");
        *info = drm_encoder_info{64, 64, 123, 128, 1 + drm::kTokenHashes, enc->dev.device, enc->dev.h0,
                                 enc->dev.device_bytes + enc->dev.y1_tiles * drm::encoder_tile_bytes()};
    });
}

extern "C" int drm_tokenize(drm_encoder *enc, const uint8_t *seqs, const int32_t *lens, int64_t n, int64_t stride,
                            int32_t *tokens)
{
    return guarded([&] {
        if (!enc || (n > 0 && !tokens)) throw Error(DRM_ERR_ARG, "null argument");
        check_seqs(seqs, lens, n, stride);
        if (n == 0) return;
        DRM_HIP_CHECK(hipSetDevice(enc->dev.device));
        DevBuf<uint8_t> d_s(n * stride);
        DevBuf<int32_t> d_l(n), d_t(n * 123);
        DRM_HIP_CHECK(hipMemcpy(d_s.p, seqs, n * stride, hipMemcpyHostToDevice));
        DRM_HIP_CHECK(hipMemcpy(d_l.p, lens, n * 4, hipMemcpyHostToDevice));
        drm::launch_tokenize(enc->dev, d_s.p, d_l.p, n, stride, d_t.p, nullptr);
        DRM_HIP_CHECK(hipMemcpy(tokens, d_t.p, n * 123 * 4, hipMemcpyDeviceToHost));
    });
}

static void read_flags(drm_encoder *enc, int64_t *undef, int64_t *shorts)
{
    uint32_t f[2];
    DRM_HIP_CHECK(hipMemcpy(f, enc->dev.flags, 8, hipMemcpyDeviceToHost));
    DRM_HIP_CHECK(hipMemset(enc->dev.flags, 0, 8));
    if (undef) *undef = f[0];
    if (shorts) *shorts = f[1];
}

extern "C" int drm_vectorize(drm_encoder *enc, const uint8_t *seqs, const int32_t *lens, int64_t n, int64_t stride,
                             float *out, int64_t *n_undefined)
{
    return guarded([&] {
        if (!enc || (n > 0 && !out)) throw Error(DRM_ERR_ARG, "null argument");
        check_seqs(seqs, lens, n, stride);
        if (n_undefined) *n_undefined = 0;
        if (n == 0) return;
        DRM_HIP_CHECK(hipSetDevice(enc->dev.device));
        DevBuf<uint8_t> d_s(n * stride);
        DevBuf<int32_t> d_l(n);
        DevBuf<float> d_o(n * 128);
        DRM_HIP_CHECK(hipMemcpy(d_s.p, seqs, n * stride, hipMemcpyHostToDevice));
        DRM_HIP_CHECK(hipMemcpy(d_l.p, lens, n * 4, hipMemcpyHostToDevice));
        read_flags(enc, nullptr, nullptr);
        drm::launch_encode(enc->dev, d_s.p, d_l.p, n, stride, d_o.p, nullptr);
        DRM_HIP_CHECK(hipMemcpy(out, d_o.p, n * 128 * 4, hipMemcpyDeviceToHost));
        read_flags(enc, n_undefined, nullptr);
    });
}

extern "C" int drm_vectorize_device(drm_encoder *enc, const uint8_t *d_seqs, const int32_t *d_lens, int64_t n,
                                    int64_t stride, float *d_out, void *stream)
{
    return guarded([&] {
        if (!enc || n < 0 || stride <= 0 || (n > 0 && (!d_seqs || !d_lens || !d_out)))
            throw Error(DRM_ERR_ARG, "invalid argument");
        DRM_HIP_CHECK(hipSetDevice(enc->dev.device));
        drm::launch_encode(enc->dev, d_seqs, d_lens, n, stride, d_out, (hipStream_t)stream);
    });
}

extern "C" int drm_encoder_flags(drm_encoder *enc, int64_t *n_undefined, int64_t *n_short)
{
    return guarded([&] {
        if (!enc) throw Error(DRM_ERR_ARG, "null argument");
        DRM_HIP_CHECK(hipSetDevice(enc->dev.device));
        DRM_HIP_CHECK(hipDeviceSynchronize());
        read_flags(enc, n_undefined, n_short);
    });
}
