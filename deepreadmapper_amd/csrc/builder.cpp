// deepreadmapper_amd/csrc/builder.cpp -- `hnswpq_index` back end: build an IndexHNSWPQ and write
// it in faiss's on-disk format. Follows build_faiss_index (src/hnswpq/index.cpp:86-193):
//   1. training set = n*SAMPLE_RATE vectors sampled at evenly spaced indices (create_training_set
//      :57-84, Config::Build::SAMPLE_RATE = 0.5 includes/utils/config.hpp:35)
//   2. IndexHNSWPQ(dim, M_pq, M_hnsw, nbits), efConstruction = EFC (:111-113), train (:122)
//   3. add all vectors (:160-175), write_index (:188)
// faiss itself is absent, so PQ training (k-means, 25 iterations, <= 256
// points per centroid) and HNSW insertion (greedy descent + efConstruction beam + the
// shrink_neighbor_list heuristic with symmetric PQ distances, as [faiss impl/HNSW.cpp] does) are
// implemented here. Build parity with faiss is NOT required: search parity is "same index file
// in, same results out" (SURVEY.md sec. 7 step 9). nthreads == 1 gives a deterministic graph.
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <queue>
#include <random>

#include "drm_internal.h"

namespace drm {
namespace {

inline float l2sqr(const float *a, const float *b, int d)
{
    float acc = 0.f;
    for (int t = 0; t < d; ++t) {
        float diff = a[t] - b[t];
        acc += diff * diff;
    }
    return acc;
}

struct PQ {
    int d, M, nbits, dsub, ksub, code_size;
    std::vector<float> centroids; // [M][ksub][dsub]
    std::vector<float> sdc;       // [M][ksub][ksub]

    uint32_t decode(const uint8_t *code, int m) const
    {
        if (nbits == 8)
            return code[m];
        uint64_t bitpos = (uint64_t)m * nbits, byte = bitpos >> 3;
        int shift = int(bitpos & 7), need = shift + nbits;
        uint64_t acc = 0;
        for (int b = 0; b * 8 < need; ++b)
            acc |= (uint64_t)code[byte + b] << (8 * b);
        return uint32_t((acc >> shift) & ((1ull << nbits) - 1));
    }
    void encode(const float *x, uint8_t *code) const
    {
        std::memset(code, 0, (size_t)code_size);
        uint64_t bitpos = 0;
        for (int m = 0; m < M; ++m) {
            const float *cm = centroids.data() + (size_t)m * ksub * dsub;
            int best = 0;
            float bd = std::numeric_limits<float>::infinity();
            for (int c = 0; c < ksub; ++c) {
                float dd = l2sqr(x + (size_t)m * dsub, cm + (size_t)c * dsub, dsub);
                if (dd < bd) {
                    bd = dd;
                    best = c;
                }
            }
            for (int b = 0; b < nbits; ++b, ++bitpos)
                if (best >> b & 1)
                    code[bitpos >> 3] |= uint8_t(1u << (bitpos & 7));
        }
    }
    void lut(const float *x, float *tab) const
    {
        for (int m = 0; m < M; ++m)
            for (int c = 0; c < ksub; ++c)
                tab[(size_t)m * ksub + c] =
                    l2sqr(x + (size_t)m * dsub, centroids.data() + ((size_t)m * ksub + c) * dsub, dsub);
    }
};

// Lloyd k-means on one sub-space [faiss Clustering::train, restated loosely]
void kmeans(const float *x, size_t n, int d, int k, int niter, uint64_t seed, float *cent, int nthreads)
{
    std::mt19937 rng((uint32_t)seed);
    std::vector<size_t> perm(n);
    for (size_t i = 0; i < n; ++i)
        perm[i] = i;
    for (size_t i = 0; i + 1 < n; ++i)
        std::swap(perm[i], perm[i + rng() % (n - i)]);
    for (int c = 0; c < k; ++c)
        std::memcpy(cent + (size_t)c * d, x + perm[(size_t)c % n] * d, sizeof(float) * d);
    std::vector<int> assign(n);
    std::vector<double> sum((size_t)k * d);
    std::vector<size_t> cnt(k);
    for (int it = 0; it < niter; ++it) {
#pragma omp parallel for num_threads(nthreads) schedule(static)
        for (int64_t i = 0; i < (int64_t)n; ++i) {
            int best = 0;
            float bd = std::numeric_limits<float>::infinity();
            for (int c = 0; c < k; ++c) {
                float dd = l2sqr(x + (size_t)i * d, cent + (size_t)c * d, d);
                if (dd < bd) {
                    bd = dd;
                    best = c;
                }
            }
            assign[i] = best;
        }
        std::fill(sum.begin(), sum.end(), 0.0);
        std::fill(cnt.begin(), cnt.end(), 0);
        for (size_t i = 0; i < n; ++i) {
            cnt[assign[i]]++;
            for (int t = 0; t < d; ++t)
                sum[(size_t)assign[i] * d + t] += x[i * d + t];
        }
        for (int c = 0; c < k; ++c)
            if (cnt[c])
                for (int t = 0; t < d; ++t)
                    cent[(size_t)c * d + t] = float(sum[(size_t)c * d + t] / (double)cnt[c]);
        // empty clusters: split the largest one (faiss split_clusters, symmetric perturbation)
        for (int c = 0; c < k; ++c) {
            if (cnt[c])
                continue;
            int big = int(std::max_element(cnt.begin(), cnt.end()) - cnt.begin());
            if (cnt[big] < 2)
                continue;
            for (int t = 0; t < d; ++t) {
                float v = cent[(size_t)big * d + t];
                float eps = (t % 2 == 0) ? 1.f / 1024 : -1.f / 1024;
                cent[(size_t)c * d + t] = v * (1 + eps);
                cent[(size_t)big * d + t] = v * (1 - eps);
            }
            cnt[c] = cnt[big] / 2;
            cnt[big] -= cnt[c];
        }
    }
}

typedef std::pair<float, int32_t> DN; // (distance, id)
struct Closer {                       // priority_queue top = farthest (NodeDistCloser)
    bool operator()(const DN &a, const DN &b) const { return a.first < b.first; }
};
struct Farther { // top = nearest (NodeDistFarther)
    bool operator()(const DN &a, const DN &b) const { return a.first > b.first; }
};

struct Builder {
    HnswPqHost &ix;
    const PQ &pq;
    std::vector<omp_lock_t> locks;
    Builder(HnswPqHost &i, const PQ &p) : ix(i), pq(p) {}

    const uint8_t *code(int32_t v) const { return ix.codes.data() + (size_t)v * pq.code_size; }
    float adc(const float *tab, int32_t v) const
    {
        const uint8_t *c = code(v);
        float r = 0.f;
        for (int m = 0; m < pq.M; ++m)
            r += tab[(size_t)m * pq.ksub + pq.decode(c, m)];
        return r;
    }
    float sdc(int32_t a, int32_t b) const
    {
        const uint8_t *ca = code(a), *cb = code(b);
        float r = 0.f;
        for (int m = 0; m < pq.M; ++m)
            r += pq.sdc[((size_t)m * pq.ksub + pq.decode(ca, m)) * pq.ksub + pq.decode(cb, m)];
        return r;
    }
    void range(int32_t no, int level, size_t &b, size_t &e) const
    {
        size_t o = ix.offsets[no];
        b = o + ix.cum_nneighbor_per_level[level];
        e = o + ix.cum_nneighbor_per_level[level + 1];
    }
    void greedy(const float *tab, int level, int32_t &nearest, float &dn) const
    {
        for (;;) {
            int32_t prev = nearest;
            size_t b, e;
            range(nearest, level, b, e);
            for (size_t j = b; j < e; ++j) {
                int32_t v = ix.neighbors[j];
                if (v < 0)
                    break;
                float dd = adc(tab, v);
                if (dd < dn) {
                    dn = dd;
                    nearest = v;
                }
            }
            if (nearest == prev)
                return;
        }
    }
    // HNSW::shrink_neighbor_list: keep v1 unless some kept v2 is closer to v1 than the query is
    void shrink(std::vector<DN> &cands_sorted_near_first, size_t max_size, std::vector<DN> &out) const
    {
        out.clear();
        for (const DN &v1 : cands_sorted_near_first) {
            bool good = true;
            for (const DN &v2 : out)
                if (sdc(v2.second, v1.second) < v1.first) {
                    good = false;
                    break;
                }
            if (good) {
                out.push_back(v1);
                if (out.size() >= max_size)
                    return;
            }
        }
    }
    void add_link(int32_t src, int32_t dest, int level)
    {
        size_t b, e;
        range(src, level, b, e);
        if (ix.neighbors[e - 1] == -1) {
            size_t i = e;
            while (i > b) {
                if (ix.neighbors[i - 1] != -1)
                    break;
                i--;
            }
            ix.neighbors[i] = dest;
            return;
        }
        std::vector<DN> all;
        all.emplace_back(sdc(src, dest), dest);
        for (size_t i = b; i < e; ++i)
            all.emplace_back(sdc(src, ix.neighbors[i]), ix.neighbors[i]);
        std::stable_sort(all.begin(), all.end(), [](const DN &x, const DN &y) { return x.first < y.first; });
        std::vector<DN> kept;
        if (all.size() < e - b)
            kept = all;
        else
            shrink(all, e - b, kept);
        size_t i = b;
        for (const DN &d : kept)
            ix.neighbors[i++] = d.second;
        while (i < e)
            ix.neighbors[i++] = -1;
    }
    void search_to_add(const float *tab, int32_t ep, float dep, int level, std::vector<uint32_t> &vt, uint32_t &vno,
                       std::vector<DN> &result_near_first) const
    {
        std::priority_queue<DN, std::vector<DN>, Farther> cand;
        std::priority_queue<DN, std::vector<DN>, Closer> res;
        cand.emplace(dep, ep);
        res.emplace(dep, ep);
        vt[ep] = vno;
        const size_t efc = (size_t)ix.efConstruction;
        while (!cand.empty()) {
            DN cur = cand.top();
            if (cur.first > res.top().first)
                break;
            cand.pop();
            size_t b, e;
            range(cur.second, level, b, e);
            for (size_t j = b; j < e; ++j) {
                int32_t v = ix.neighbors[j];
                if (v < 0)
                    break;
                if (vt[v] == vno)
                    continue;
                vt[v] = vno;
                float dd = adc(tab, v);
                if (res.size() < efc || res.top().first > dd) {
                    res.emplace(dd, v);
                    cand.emplace(dd, v);
                    if (res.size() > efc)
                        res.pop();
                }
            }
        }
        if (++vno == 0) {
            std::fill(vt.begin(), vt.end(), 0u);
            vno = 1;
        }
        result_near_first.clear();
        while (!res.empty()) {
            result_near_first.push_back(res.top());
            res.pop();
        }
        std::reverse(result_near_first.begin(), result_near_first.end());
    }
};

} // namespace

std::vector<size_t> pq_training_rows(int64_t n, double sample_rate, int ksub, uint64_t seed)
{
    // create_training_set (src/hnswpq/index.cpp:57-84): evenly spaced, n_train = n * sample_rate
    size_t n_train = (size_t)((double)n * sample_rate);
    if (n_train < 1)
        n_train = 1;
    const double step = (double)n / (double)n_train;
    // faiss Clustering subsamples to max_points_per_centroid (256) * k points
    const size_t n_fit = std::min(n_train, (size_t)256 * ksub);
    std::vector<size_t> idx(n_train);
    for (size_t i = 0; i < n_train; ++i)
        idx[i] = std::min((size_t)((double)i * step), (size_t)n - 1);
    if (n_fit < n_train) {
        std::mt19937 rng((uint32_t)(seed * 2654435761u + 1234));
        for (size_t i = 0; i < n_fit; ++i)
            std::swap(idx[i], idx[i + rng() % (n_train - i)]);
        idx.resize(n_fit);
    }
    return idx;
}

void pq_train_subspaces(const float *rows, size_t n_fit, int d, int M, int nbits, uint64_t seed, int nthreads,
                        float *centroids)
{
    const int dsub = d / M, ksub = 1 << nbits;
    if (nthreads <= 0)
        nthreads = omp_get_max_threads();
    std::vector<float> sub(n_fit * (size_t)dsub);
    for (int m = 0; m < M; ++m) {
        for (size_t i = 0; i < n_fit; ++i)
            std::memcpy(&sub[i * dsub], rows + i * d + (size_t)m * dsub, sizeof(float) * dsub);
        kmeans(sub.data(), n_fit, dsub, ksub, 25, seed + 1234 + (uint64_t)m, centroids + (size_t)m * ksub * dsub,
               nthreads);
    }
}

int hnsw_assign_levels(HnswPqHost &ix, int64_t n, int M_hnsw, uint64_t seed)
{
    // HNSW(M): default probas, levels ~ random_level() [faiss HNSW::prepare_level_tab]
    hnsw_default_probas(M_hnsw, ix.assign_probas, ix.cum_nneighbor_per_level);
    std::mt19937 lrng((uint32_t)(12345 + seed));
    ix.levels.resize((size_t)n);
    ix.offsets.assign((size_t)n + 1, 0);
    int top_level = 0;
    for (int64_t i = 0; i < n; ++i) {
        double f = lrng() / double(lrng.max());
        int level = (int)ix.assign_probas.size() - 1;
        for (int l = 0; l < (int)ix.assign_probas.size(); ++l) {
            if (f < ix.assign_probas[l]) {
                level = l;
                break;
            }
            f -= ix.assign_probas[l];
        }
        ix.levels[i] = level + 1;
        top_level = std::max(top_level, level);
        ix.offsets[i + 1] = ix.offsets[i] + (uint64_t)ix.cum_nneighbor_per_level[level + 1];
    }
    return top_level;
}

void build_hnswpq(const float *x, int64_t n, int d, int M_pq, int nbits, int M_hnsw, int efc, double sample_rate,
                  int nthreads, uint64_t seed, const std::string &path)
{
    if (n <= 0)
        throw Error(DRM_ERR_ARG, "Input data is empty");
    if (M_pq <= 0 || d % M_pq != 0)
        throw Error(DRM_ERR_ARG, "M_pq must divide the dimension");
    if (nbits < 1 || nbits > 16 || M_hnsw < 2 || efc < 1)
        throw Error(DRM_ERR_ARG, "invalid build parameters");
    if (nthreads <= 0)
        nthreads = omp_get_max_threads();

    PQ pq;
    pq.d = d;
    pq.M = M_pq;
    pq.nbits = nbits;
    pq.dsub = d / M_pq;
    pq.ksub = 1 << nbits;
    pq.code_size = (M_pq * nbits + 7) / 8;
    pq.centroids.resize((size_t)d * pq.ksub);

    {
        const std::vector<size_t> rows = pq_training_rows(n, sample_rate, pq.ksub, seed);
        std::vector<float> tx(rows.size() * (size_t)d);
        for (size_t i = 0; i < rows.size(); ++i)
            std::memcpy(&tx[i * d], x + rows[i] * d, sizeof(float) * d);
        pq_train_subspaces(tx.data(), rows.size(), d, M_pq, nbits, seed, nthreads, pq.centroids.data());
    }
    pq.sdc.resize((size_t)M_pq * pq.ksub * pq.ksub);
    for (int m = 0; m < M_pq; ++m)
        for (int a = 0; a < pq.ksub; ++a)
            for (int b = 0; b < pq.ksub; ++b)
                pq.sdc[((size_t)m * pq.ksub + a) * pq.ksub + b] =
                    l2sqr(&pq.centroids[((size_t)m * pq.ksub + a) * pq.dsub],
                          &pq.centroids[((size_t)m * pq.ksub + b) * pq.dsub], pq.dsub);

    HnswPqHost ix;
    ix.hdr.d = d;
    ix.hdr.ntotal = n;
    ix.storage_hdr = ix.hdr;
    ix.pq_d = (uint64_t)d;
    ix.pq_M = (uint64_t)M_pq;
    ix.pq_nbits = (uint64_t)nbits;
    ix.centroids = pq.centroids;
    ix.codes.resize((size_t)n * pq.code_size);
#pragma omp parallel for num_threads(nthreads) schedule(static)
    for (int64_t i = 0; i < n; ++i)
        pq.encode(x + (size_t)i * d, ix.codes.data() + (size_t)i * pq.code_size);

    ix.efConstruction = efc;
    ix.efSearch = 16;
    const int top_level = hnsw_assign_levels(ix, n, M_hnsw, seed);
    ix.neighbors.assign(ix.offsets.back(), -1);

    Builder B(ix, pq);
    B.locks.resize((size_t)n);
    for (auto &l : B.locks)
        omp_init_lock(&l);

    // hnsw_add_vertices: bucket by level, insert highest levels first, random order within a level
    std::vector<std::vector<int32_t>> buckets((size_t)top_level + 1);
    for (int64_t i = 0; i < n; ++i)
        buckets[(size_t)ix.levels[i] - 1].push_back((int32_t)i);
    std::mt19937 orng((uint32_t)(789 + seed));
    ix.entry_point = -1;
    ix.max_level = -1;
    for (int pl = top_level; pl >= 0; --pl) {
        auto &bk = buckets[(size_t)pl];
        for (size_t j = 0; j + 1 < bk.size(); ++j)
            std::swap(bk[j], bk[j + orng() % (bk.size() - j)]);
        size_t start = 0;
        if (ix.entry_point < 0 && !bk.empty()) { // first point becomes the entry point
            ix.entry_point = bk[0];
            ix.max_level = pl;
            start = 1;
        }
#pragma omp parallel num_threads(nthreads)
        {
            std::vector<float> tab((size_t)pq.M * pq.ksub);
            std::vector<uint32_t> vt((size_t)n, 0u);
            uint32_t vno = 1;
            std::vector<DN> found, kept;
#pragma omp for schedule(dynamic, 64)
            for (int64_t bi = (int64_t)start; bi < (int64_t)bk.size(); ++bi) {
                int32_t pt = bk[(size_t)bi];
                pq.lut(x + (size_t)pt * d, tab.data());
                int32_t nearest = ix.entry_point;
                float dn = B.adc(tab.data(), nearest);
                int level = ix.max_level;
                omp_set_lock(&B.locks[pt]);
                for (; level > pl; --level)
                    B.greedy(tab.data(), level, nearest, dn);
                for (; level >= 0; --level) {
                    B.search_to_add(tab.data(), nearest, dn, level, vt, vno, found);
                    size_t M = (size_t)ix.nb_at(level);
                    if (found.size() < M)
                        kept = found;
                    else
                        B.shrink(found, M, kept);
                    for (const DN &o : kept)
                        B.add_link(pt, o.second, level);
                    omp_unset_lock(&B.locks[pt]);
                    for (const DN &o : kept) {
                        omp_set_lock(&B.locks[o.second]);
                        B.add_link(o.second, pt, level);
                        omp_unset_lock(&B.locks[o.second]);
                    }
                    omp_set_lock(&B.locks[pt]);
                    // next level starts from the nearest found at this one
                    if (!found.empty()) {
                        nearest = found[0].second;
                        dn = found[0].first;
                    }
                }
                omp_unset_lock(&B.locks[pt]);
            }
        }
    }
    for (auto &l : B.locks)
        omp_destroy_lock(&l);
    write_hnswpq(ix, path);
}

} // namespace drm

extern "C" int drm_build_hnswpq(const float *x, int64_t n, int32_t d, int32_t M_pq, int32_t nbits, int32_t M_hnsw,
                                int32_t efConstruction, double sample_rate, int32_t nthreads, uint64_t seed,
                                const char *index_path)
{
    try {
        if (!x || !index_path)
            throw drm::Error(DRM_ERR_ARG, "null argument");
        drm::build_hnswpq(x, n, d, M_pq, nbits, M_hnsw, efConstruction, sample_rate, nthreads, seed, index_path);
        return DRM_OK;
    } catch (const drm::Error &e) {
        drm::set_last_error(e.what());
        return e.code;
    } catch (const std::exception &e) {
        drm::set_last_error(e.what());
        return DRM_ERR_ARG;
    }
}
