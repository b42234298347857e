// deepreadmapper_amd/csrc/query_order.hip -- device radix sort of (u32 key, i32 value) pairs.
//
// Used by the fp32 search (hnsw_flat_search.hip) to order the level-0 queue: after a descent-only
// pass, the queries are sorted by the node id of their level-0 entry point, so the waves resident at
// any moment search neighbouring regions of the graph and share its rows and vectors in L2 and the
// Infinity Cache. The order never changes a result: each query's search is independent (the
// reference runs them under an OpenMP `schedule(guided)` loop in any order).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "drm_device.h"

namespace drm {

size_t sort_pairs_temp_bytes(int64_t n, int bits)
{
    size_t bytes = 0;
    DRM_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                                                     (const int32_t *)nullptr, (int32_t *)nullptr, (int)n, 0, bits));
    return bytes;
}

void sort_pairs(void *temp, size_t temp_bytes, const uint32_t *kin, uint32_t *kout, const int32_t *vin, int32_t *vout,
                int64_t n, int bits, hipStream_t stream)
{
    DRM_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, kin, kout, vin, vout, (int)n, 0, bits, stream));
}

} // namespace drm
