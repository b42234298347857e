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
