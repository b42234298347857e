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
