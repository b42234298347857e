// deepreadmapper_amd/csrc/builder_flat.cpp -- fp32-L2 HNSW builder writing hnswlib's file format.
//
// Replaces the reference's build_index (src/hnswlib_dir/index.cpp:3-49): HierarchicalNSW<float>
// (L2Space(dim), max_elements = n, M, ef_construction) + addPoint(x[i], label i) for every i +
// saveIndex. Construction follows hnswlib's algorithm (maxM = M, maxM0 = 2M, mult = 1/ln M,
// greedy descent, searchBaseLayer with ef_construction, getNeighborsByHeuristic2,
// mutuallyConnectNewElement); the graph itself need not equal hnswlib's (build parity is not a
// requirement), but the file is one hnswlib loads.
// Threads insert elements concurrently with per-node locks, as hnswlib's parallel addPoint does.
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <mutex>
#include <queue>

#include "drm_internal.h"

namespace drm {
namespace {

inline float l2(const float *a, const float *b, int d)
{
    float s = 0.f;
    for (int j = 0; j < d; ++j) {
        const float t = a[j] - b[j];
        s += t * t;
    }
    return s;
}

typedef std::pair<float, uint32_t> DI;
struct ByFirst {
    bool operator()(const DI &a, const DI &b) const { return a.first < b.first; }
};
typedef std::priority_queue<DI, std::vector<DI>, ByFirst> MaxQ; // top = farthest

uint64_t splitmix(uint64_t &s)
{
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct FlatBuilder {
    HnswFlatHost &ix;
    const float *x;
    std::vector<omp_lock_t> locks;
    std::mutex global;

    FlatBuilder(HnswFlatHost &i, const float *xx) : ix(i), x(xx) {}
    const float *v(uint32_t i) const { return x + (size_t)i * ix.d; }
    uint32_t *links(uint32_t i, int level)
    {
        if (level == 0)
            return &ix.l0[(size_t)i * (1 + ix.maxM0)];
        return &ix.up[(size_t)ix.up_off[i] + (size_t)(level - 1) * (1 + ix.maxM)];
    }

    MaxQ search_layer(uint32_t ep, const float *q, int level, std::vector<uint32_t> &vis, uint32_t &tag)
    {
        if (++tag == 0) {
            std::fill(vis.begin(), vis.end(), 0u);
            tag = 1;
        }
        MaxQ top, cand;
        float lb = l2(q, v(ep), ix.d);
        top.emplace(lb, ep);
        cand.emplace(-lb, ep);
        vis[ep] = tag;
        while (!cand.empty()) {
            const DI c = cand.top();
            if (-c.first > lb && top.size() == ix.efc)
                break;
            cand.pop();
            std::vector<uint32_t> nb;
            omp_set_lock(&locks[c.second]);
            const uint32_t *ll = links(c.second, level);
            nb.assign(ll + 1, ll + 1 + (ll[0] & 0xFFFFu));
            omp_unset_lock(&locks[c.second]);
            for (uint32_t w : nb) {
                if (vis[w] == tag)
                    continue;
                vis[w] = tag;
                const float dd = l2(q, v(w), ix.d);
                if (top.size() < ix.efc || lb > dd) {
                    cand.emplace(-dd, w);
                    top.emplace(dd, w);
                    if (top.size() > ix.efc)
                        top.pop();
                    if (!top.empty())
                        lb = top.top().first;
                }
            }
        }
        return top;
    }

    // getNeighborsByHeuristic2: keep a candidate unless an already kept one is closer to it than
    // the base element is
    void heuristic(MaxQ &top, size_t M)
    {
        if (top.size() < M)
            return;
        std::priority_queue<DI> closest; // (-dist, id): top = nearest
        while (!top.empty()) {
            closest.emplace(-top.top().first, top.top().second);
            top.pop();
        }
        std::vector<DI> keep;
        while (!closest.empty() && keep.size() < M) {
            const DI c = closest.top();
            closest.pop();
            bool good = true;
            for (const DI &k : keep)
                if (l2(v(k.second), v(c.second), ix.d) < -c.first) {
                    good = false;
                    break;
                }
            if (good)
                keep.push_back(c);
        }
        for (const DI &k : keep)
            top.emplace(-k.first, k.second);
    }

    uint32_t connect(uint32_t cur, MaxQ &top, int level)
    {
        const size_t mmax = level ? ix.maxM : ix.maxM0;
        heuristic(top, ix.M);
        std::vector<uint32_t> sel;
        while (!top.empty()) {
            sel.push_back(top.top().second);
            top.pop();
        }
        const uint32_t next = sel.back(); // the closest one
        {
            omp_set_lock(&locks[cur]);
            uint32_t *ll = links(cur, level);
            ll[0] = (uint32_t)sel.size();
            for (size_t j = 0; j < sel.size(); ++j)
                ll[1 + j] = sel[j];
            omp_unset_lock(&locks[cur]);
        }
        for (uint32_t s : sel) {
            omp_set_lock(&locks[s]);
            uint32_t *ll = links(s, level);
            const uint32_t sz = ll[0] & 0xFFFFu;
            if (sz < mmax) {
                ll[1 + sz] = cur;
                ll[0] = sz + 1;
            } else {
                MaxQ cands;
                cands.emplace(l2(v(s), v(cur), ix.d), cur);
                for (uint32_t j = 0; j < sz; ++j)
                    cands.emplace(l2(v(s), v(ll[1 + j]), ix.d), ll[1 + j]);
                heuristic(cands, mmax);
                uint32_t k = 0;
                while (!cands.empty()) {
                    ll[1 + k++] = cands.top().second;
                    cands.pop();
                }
                ll[0] = k;
            }
            omp_unset_lock(&locks[s]);
        }
        return next;
    }
};

} // namespace

void build_hnsw_flat(const float *x, int64_t n, int d, int M, int efc, int nthreads, uint64_t seed,
                     const std::string &path)
{
    if (n <= 0)
        throw Error(DRM_ERR_ARG, "Input data is empty"); // index.cpp:12-15
    if (d <= 0 || M < 2 || M > 32767 || efc < 1)
        throw Error(DRM_ERR_ARG, "invalid build parameters");
    if (n > (int64_t)0xFFFFFFFEll)
        throw Error(DRM_ERR_UNSUPPORTED, "more than 2^32-2 elements");
    if (nthreads <= 0)
        nthreads = omp_get_max_threads();
    HnswFlatHost ix;
    ix.d = d;
    ix.n = n;
    ix.max_elements = (uint64_t)n;
    ix.M = (uint64_t)M;
    ix.maxM = (uint64_t)M;
    ix.maxM0 = 2 * (uint64_t)M;
    ix.mult = 1.0 / std::log(1.0 * M);
    ix.efc = (uint64_t)std::max(M, efc); // hnswlib: ef_construction_ = std::max(ef_construction, M)
    ix.vec.assign(x, x + (size_t)n * d);
    ix.labels.resize(n);
    ix.levels.resize(n);
    ix.up_off.assign(n, -1);
    ix.l0.assign((size_t)n * (1 + ix.maxM0), 0u);
    uint64_t s = seed ^ 0x5DEECE66Dull;
    int64_t words = 0;
    for (int64_t i = 0; i < n; ++i) {
        ix.labels[i] = (uint64_t)i;
        const double u = ((splitmix(s) >> 11) + 1) * (1.0 / 9007199254740993.0); // (0, 1]
        ix.levels[i] = (int32_t)(-std::log(u) * ix.mult);
        if (ix.levels[i] > 0) {
            ix.up_off[i] = words;
            words += (int64_t)ix.levels[i] * (int64_t)(1 + ix.maxM);
        }
    }
    ix.up.assign((size_t)std::max<int64_t>(words, 1), 0u);
    FlatBuilder b(ix, x);
    b.locks.resize(n);
    for (auto &l : b.locks)
        omp_init_lock(&l);
    ix.ep = 0;
    ix.maxlevel = ix.levels[0];
    // hnswlib inserts serially when single-threaded; a handful of elements go first serially so the
    // parallel phase starts from a connected core
    const int64_t serial = std::min<int64_t>(n, 256);
    std::vector<uint32_t> vis0((size_t)n, 0u);
    uint32_t tag0 = 0;
    auto insert = [&](int64_t i, std::vector<uint32_t> &vis, uint32_t &tag) {
        const int lvl = ix.levels[i];
        std::unique_lock<std::mutex> g(b.global);
        const int maxlevel = ix.maxlevel;
        if (lvl <= maxlevel)
            g.unlock();
        uint32_t cur = ix.ep;
        const float *q = b.v((uint32_t)i);
        if (lvl < maxlevel) {
            float curd = l2(q, b.v(cur), d);
            for (int level = maxlevel; level > lvl; --level) {
                bool changed = true;
                while (changed) {
                    changed = false;
                    omp_set_lock(&b.locks[cur]);
                    const uint32_t *ll = b.links(cur, level);
                    std::vector<uint32_t> nb(ll + 1, ll + 1 + (ll[0] & 0xFFFFu));
                    omp_unset_lock(&b.locks[cur]);
                    for (uint32_t w : nb) {
                        const float dd = l2(q, b.v(w), d);
                        if (dd < curd) {
                            curd = dd;
                            cur = w;
                            changed = true;
                        }
                    }
                }
            }
        }
        for (int level = std::min(lvl, maxlevel); level >= 0; --level) {
            MaxQ top = b.search_layer(cur, q, level, vis, tag);
            cur = b.connect((uint32_t)i, top, level);
        }
        if (lvl > maxlevel) {
            ix.ep = (uint32_t)i;
            ix.maxlevel = lvl;
        }
    };
    for (int64_t i = 1; i < serial; ++i)
        insert(i, vis0, tag0);
#pragma omp parallel num_threads(nthreads)
    {
        std::vector<uint32_t> vis((size_t)n, 0u);
        uint32_t tag = 0;
#pragma omp for schedule(dynamic, 64)
        for (int64_t i = serial; i < n; ++i)
            insert(i, vis, tag);
    }
    for (auto &l : b.locks)
        omp_destroy_lock(&l);
    write_hnswlib(ix, path);
}

} // namespace drm

extern "C" int drm_build_hnsw_flat(const float *x, int64_t n, int32_t d, int32_t M, int32_t efc, int32_t nthreads,
                                   uint64_t seed, const char *path)
{
    try {
        if (!x || !path)
            throw drm::Error(DRM_ERR_ARG, "null argument");
        drm::build_hnsw_flat(x, n, d, M, efc, nthreads, seed, path);
        return DRM_OK;
    } catch (const drm::Error &e) {
        drm::set_last_error(e.what());
        return e.code;
    } catch (const std::exception &e) {
        drm::set_last_error(e.what());
        return DRM_ERR_IO;
    }
}
