// oracle/stl_partial_sort.cpp -- TEST INFRASTRUCTURE ONLY.
// The host C++ standard library's std::partial_sort, called exactly as the reference calls it
// (src/utils/reranker.cpp:35-40: iota indices, comparator scores[a] > scores[b]).
// Used to pin oracle_partial_sort_desc (the C restatement) and the device emulation.
#include <algorithm>
#include <cstdint>
#include <numeric>
#include <vector>

extern "C" void stl_partial_sort_desc(int64_t *idx, int64_t n, int64_t k, const int32_t *scores)
{
    std::vector<size_t> indices((size_t)n);
    std::iota(indices.begin(), indices.end(), 0);
    std::partial_sort(indices.begin(), indices.begin() + k, indices.end(),
                      [&scores](size_t i1, size_t i2) { return scores[i1] > scores[i2]; });
    for (int64_t i = 0; i < n; ++i)
        idx[i] = (int64_t)indices[(size_t)i];
}

// batch_reranker's call (src/utils/reranker.cpp:162-166): comparator l2_dists[a] < l2_dists[b]
extern "C" void stl_partial_sort_asc_f32(int64_t *idx, int64_t n, int64_t k, const float *dists)
{
    std::vector<size_t> indices((size_t)n);
    std::iota(indices.begin(), indices.end(), 0);
    std::partial_sort(indices.begin(), indices.begin() + k, indices.end(),
                      [&dists](size_t i1, size_t i2) { return dists[i1] < dists[i2]; });
    for (int64_t i = 0; i < n; ++i)
        idx[i] = (int64_t)indices[(size_t)i];
}
