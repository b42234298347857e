// oracle/hnswlib_oracle.cpp -- TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py cpu_baseline).
//
// CPU restatement of hnswlib's fp32-L2 search as the reference drives it:
//   search(index, queries, k, ef)          src/hnswlib_dir/search.cpp:7-52 (setEf, then per query
//   -> searchKnnCloserFirst(q, k)          searchKnnCloserFirst, OpenMP over queries)
//   -> HierarchicalNSW::searchKnn          [upstream hnswlib, unvendored submodule, no pinned commit;
//   -> searchBaseLayerST<bare_bone=true>    restated from the v0.7/v0.8 algorithm -- parity unpinned]
//
// Semantics kept exactly:
//   * greedy descent on levels maxlevel..1: scan the level's link list, `if (d < curdist)` moves;
//     repeat while the node changed;
//   * level 0: top_candidates and candidate_set are std::priority_queue<pair<float, id>> ordered by
//     CompareByFirst (a.first < b.first) -- this file uses libstdc++'s own priority_queue, so the
//     heap layout and hence every tie order is libstdc++'s; candidate_set holds (-dist, id);
//     stop when -candidate_set.top().first > lowerBound; a fresh link is considered iff
//     top_candidates.size() < ef || lowerBound > dist; top_candidates is trimmed to ef by pop();
//   * searchKnn pops top_candidates down to k, then orders the survivors by (dist, label) through
//     std::priority_queue<pair<float, label>> (std::less on pairs); searchKnnCloserFirst returns
//     them closest first.
// L2: hnswlib's L2SqrSIMD16ExtAVX order for d % 16 == 0 -- eight accumulators, accumulator i sums
// (x[j]-y[j])^2 over j = i, i+8, i+16, ... in order (mul then add, no FMA), then
// acc0 + acc1 + ... + acc7 left to right.
#include <cmath>
#include <cstdint>
#include <algorithm>
#include <cstring>
#include <queue>
#include <utility>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

namespace {
thread_local size_t t_maxcand = 0; // diagnostic: largest candidate_set of the thread's queries
thread_local int64_t t_tieq[3] = {0, 0, 0}; // diagnostic: queries with a tied eviction / tied pop / any

struct Flat {
    int d;
    int64_t n;
    int maxM0, maxM, maxlevel;
    uint32_t ep;
    const float *vec;        // [n][d]
    const uint32_t *l0;      // [n][1 + maxM0]: count, links
    const int64_t *up_off;   // [n]: start of node's level>=1 blocks in `up` (uint32 units), -1 if none
    const uint32_t *up;      // blocks of (1 + maxM): count, links; block l-1 for level l
    const uint64_t *labels;  // [n]
};

#pragma GCC push_options
#pragma GCC optimize("fp-contract=off")
// Sum order (oracle_set_l2_order), the hnswlib kernels a -march=native build (build.zig:48-57) can pick:
//   0 (default, the GPU kernel's): L2SqrSIMD16ExtAVX, 8 accumulators, mul then add;
//   1: L2SqrSIMD16ExtAVX with the mul/add pair contracted to FMA (GCC contracts intrinsics);
//   2: L2SqrSIMD16ExtAVX512, 16 accumulators, mul then add, TmpRes[0] + ... + TmpRes[15];
//   3: L2SqrSIMD16ExtAVX512 with FMA.
int g_l2_order = 0;
float l2_lanes(const float *x, const float *y, int d, int lanes, bool fma_on)
{
    float acc[16] = {0};
    for (int j = 0; j < d; j += lanes)
        for (int i = 0; i < lanes; ++i) {
            const float t = x[j + i] - y[j + i];
            if (fma_on) {
                acc[i] = std::fma(t, t, acc[i]);
            } else {
                const float sq = t * t;
                acc[i] = acc[i] + sq;
            }
        }
    float r = acc[0];
    for (int i = 1; i < lanes; ++i)
        r = r + acc[i];
    return r;
}
float l2_avx(const float *x, const float *y, int d)
{
    switch (g_l2_order) {
    case 1: return l2_lanes(x, y, d, 8, true);
    case 2: return l2_lanes(x, y, d, 16, false);
    case 3: return l2_lanes(x, y, d, 16, true);
    default: return l2_lanes(x, y, d, 8, false);
    }
}
#pragma GCC pop_options

struct CompareByFirst {
    bool operator()(const std::pair<float, uint32_t> &a, const std::pair<float, uint32_t> &b) const
    {
        return a.first < b.first;
    }
};
typedef std::priority_queue<std::pair<float, uint32_t>, std::vector<std::pair<float, uint32_t>>, CompareByFirst>
    PQ;

void search_one(const Flat &ix, const float *q, int k, int ef_, float *D, int64_t *I, int32_t *ndis_out,
                int32_t *nhops_out, std::vector<uint32_t> &vis, uint32_t &tag)
{
    int64_t ndis = 0, nhops = 0;
    for (int j = 0; j < k; ++j) {
        D[j] = INFINITY;
        I[j] = -1;
    }
    if (ix.n == 0) {
        *ndis_out = 0;
        *nhops_out = 0;
        return;
    }
    uint32_t cur = ix.ep;
    float curdist = l2_avx(q, ix.vec + (size_t)cur * ix.d, ix.d);
    ndis++;
    for (int level = ix.maxlevel; level > 0; level--) {
        bool changed = true;
        while (changed) {
            changed = false;
            const uint32_t *blk = ix.up + ix.up_off[cur] + (size_t)(level - 1) * (1 + ix.maxM);
            const int size = (int)(blk[0] & 0xFFFFu);
            nhops++;
            ndis += size;
            for (int i = 0; i < size; ++i) {
                const uint32_t c = blk[1 + i];
                const float dd = l2_avx(q, ix.vec + (size_t)c * ix.d, ix.d);
                if (dd < curdist) {
                    curdist = dd;
                    cur = c;
                    changed = true;
                }
            }
        }
    }
    const size_t ef = (size_t)(ef_ > k ? ef_ : k);
    // searchBaseLayerST<bare_bone_search = true>
    if (++tag == 0) {
        std::fill(vis.begin(), vis.end(), 0u);
        tag = 1;
    }
    PQ top, cand;
    bool tie_evict = false, tie_pop = false;
    float lowerBound = curdist;
    top.emplace(curdist, cur);
    cand.emplace(-curdist, cur);
    vis[cur] = tag;
    while (!cand.empty()) {
        const std::pair<float, uint32_t> cp = cand.top();
        const float cdist = -cp.first;
        if (cdist > lowerBound)
            break;
        if (cand.size() > t_maxcand)
            t_maxcand = cand.size();
        cand.pop();
        if (!cand.empty() && cand.top().first == cp.first)
            tie_pop = true;
        nhops++;
        const uint32_t *row = ix.l0 + (size_t)cp.second * (1 + ix.maxM0);
        const int size = (int)(row[0] & 0xFFFFu);
        for (int j = 1; j <= size; ++j) {
            const uint32_t c = row[j];
            if (vis[c] == tag)
                continue;
            vis[c] = tag;
            const float dist = l2_avx(q, ix.vec + (size_t)c * ix.d, ix.d);
            ndis++;
            if (top.size() < ef || lowerBound > dist) {
                cand.emplace(-dist, c);
                top.emplace(dist, c);
                while (top.size() > ef) {
                    const float ev = top.top().first;
                    top.pop();
                    if (top.top().first == ev)
                        tie_evict = true;
                }
                if (!top.empty())
                    lowerBound = top.top().first;
            }
        }
    }
    t_tieq[0] += tie_evict;
    t_tieq[1] += tie_pop;
    t_tieq[2] += tie_evict || tie_pop;
    while (top.size() > (size_t)k)
        top.pop();
    std::priority_queue<std::pair<float, uint64_t>> result;
    while (!top.empty()) {
        result.push(std::pair<float, uint64_t>(top.top().first, ix.labels[top.top().second]));
        top.pop();
    }
    size_t sz = result.size();
    std::vector<std::pair<float, uint64_t>> out(sz);
    while (!result.empty()) {
        out[--sz] = result.top();
        result.pop();
    }
    for (size_t j = 0; j < out.size() && j < (size_t)k; ++j) {
        D[j] = out[j].first;
        I[j] = (int64_t)out[j].second;
    }
    *ndis_out = (int32_t)ndis;
    *nhops_out = (int32_t)nhops;
}

} // namespace

extern "C" {
void oracle_set_l2_order(int order) { g_l2_order = order; }


static size_t g_maxcand = 0;
static int64_t g_tieq[3] = {0, 0, 0};
// diagnostic: queries of the last oracle_hnswlib_search call with a tie at an eviction of
// top_candidates / at a candidate_set pop / either (where heap layouts decide the traversal)
void oracle_hnswlib_tie_queries(int64_t *out3)
{
    for (int i = 0; i < 3; ++i)
        out3[i] = g_tieq[i];
}
// diagnostic: the largest candidate_set size seen by the last oracle_hnswlib_search call
size_t oracle_hnswlib_maxcand() { return g_maxcand; }

float oracle_l2_avx(const float *x, const float *y, int d) { return l2_avx(x, y, d); }

// Search n queries x[n][d]; D/I [n][k] (closest first, padded (+inf, -1)); ndis/nhops per query.
int oracle_hnswlib_search(int d, int64_t ntotal, int maxM0, int maxM, int maxlevel, uint32_t ep, const float *vec,
                          const uint32_t *l0, const int64_t *up_off, const uint32_t *up, const uint64_t *labels,
                          const float *x, int64_t n, int k, int ef, float *D, int64_t *I, int32_t *ndis,
                          int32_t *nhops, int nthreads)
{
    if (k <= 0 || d % 16 != 0)
        return -1;
    Flat ix{d, ntotal, maxM0, maxM, maxlevel, ep, vec, l0, up_off, up, labels};
    g_maxcand = 0;
    g_tieq[0] = g_tieq[1] = g_tieq[2] = 0;
#ifdef _OPENMP
    if (nthreads <= 0)
        nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads)
#endif
    {
        std::vector<uint32_t> vis((size_t)(ntotal > 0 ? ntotal : 1), 0u);
        uint32_t tag = 0;
        t_maxcand = 0;
        t_tieq[0] = t_tieq[1] = t_tieq[2] = 0;
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int64_t i = 0; i < n; ++i)
            search_one(ix, x + i * d, k, ef, D + i * k, I + i * k, ndis + i, nhops + i, vis, tag);
#ifdef _OPENMP
#pragma omp critical
#endif
        {
            g_maxcand = std::max(g_maxcand, t_maxcand);
            for (int i = 0; i < 3; ++i)
                g_tieq[i] += t_tieq[i];
        }
    }
    return 0;
}

} // extern "C"
