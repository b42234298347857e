// oracle/ref_shim.cpp -- TEST INFRASTRUCTURE ONLY.
// extern "C" wrapper around the REFERENCE's own calc_sw_score (src/utils/metrics.cpp:10-45),
// compiled together with /root/reference/src/utils/metrics.cpp where it lies (see oracle/Makefile).
// The resulting oracle/_ref/libdrm_ref.so is the "reference" leg of the SW parity tests and the
// SW-only reference CPU baseline. No reference source is copied into this repository.
#include <cstdint>
#include <string>
#include "metrics.hpp"

extern "C" int ref_calc_sw_score(const uint8_t *s1, int64_t l1, const uint8_t *s2, int64_t l2)
{
    std::string a(reinterpret_cast<const char *>(s1), (size_t)l1);
    std::string b(reinterpret_cast<const char *>(s2), (size_t)l2);
    return calc_sw_score(a, b);
}

// The reference's own calc_l2_dist (src/utils/metrics.cpp:48-61). oracle/Makefile builds this library with
// -mavx2 -mfma (the features -march=native gives the reference on any current x86 host), so the loop is
// vectorized and contracted the way the reference's own build compiles it.
#include <vector>
extern "C" float ref_calc_l2_dist(const float *a, const float *b, int64_t d)
{
    std::vector<float> v1(a, a + d), v2(b, b + d);
    return calc_l2_dist(v1, v2);
}

// The CPU baseline's SW half on the reference's own scorer (bench.py cpu_baseline): per query, calc_sw_score of each of
// its kk candidate windows against the query as given, then the reranker's ordering -- std::partial_sort of the
// candidate indices by score, descending (src/utils/reranker.cpp:16-40) -- OpenMP over queries as
// post_process_sw_static runs them (src/utils/post_processor.cpp:491). Scores land in `scores` [nq][kk] in sorted order,
// the candidates' positions in `order` [nq][kk]. Ids at or past n_ref are skipped (find_sequences, dense).
#include <algorithm>
#include <numeric>
#include <omp.h>
extern "C" int ref_sw_rerank_rows(const uint8_t *refs, int64_t n_ref, int64_t ref_stride, int64_t ref_len,
                                  const int64_t *nb, int64_t nq, int64_t kk, const uint8_t *queries, int64_t q_stride,
                                  const int32_t *q_len, int32_t *scores, int32_t *order, int nthreads)
{
    if (nthreads > 0)
        omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic)
    for (int64_t q = 0; q < nq; ++q) {
        const std::string query(reinterpret_cast<const char *>(queries + q * q_stride), (size_t)q_len[q]);
        std::vector<int> sc;
        std::vector<int32_t> pos;
        for (int64_t c = 0; c < kk; ++c) {
            const int64_t id = nb[q * kk + c];
            if (id < 0 || id >= n_ref)
                continue;
            const std::string cand(reinterpret_cast<const char *>(refs + id * ref_stride), (size_t)ref_len);
            sc.push_back(calc_sw_score(cand, query));
            pos.push_back((int32_t)c);
        }
        std::vector<size_t> idx(sc.size());
        std::iota(idx.begin(), idx.end(), 0);
        std::partial_sort(idx.begin(), idx.end(), idx.end(), [&](size_t a, size_t b) { return sc[a] > sc[b]; });
        for (int64_t j = 0; j < kk; ++j) {
            scores[q * kk + j] = j < (int64_t)idx.size() ? sc[idx[j]] : -1;
            order[q * kk + j] = j < (int64_t)idx.size() ? pos[idx[j]] : -1;
        }
    }
    return 0;
}
