// deepreadmapper_amd/csrc/embed.cpp -- deterministic 3-mer random-projection embedder.
// Stand-in for the OpenVINO GRU encoder (src/inference/*, OUT OF SCOPE per SURVEY.md sec. 2 row 11),
// so that `pipeline`/`hnswpq_index` accept sequence files end to end and the synthetic workloads of
// BASELINE.json (C1, C3, C4) have locality: a read embeds next to the window it was drawn from.
#include <cmath>
#include <vector>

#include "drm_internal.h"

namespace drm {

static inline uint64_t splitmix64(uint64_t &s)
{
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

std::vector<double> kmer3_matrix(int dim, uint64_t seed)
{
    std::vector<double> R((size_t)64 * dim);
    uint64_t s = seed;
    const double two_pi = 6.283185307179586476925286766559;
    for (size_t i = 0; i < R.size(); ++i) {
        double u1 = ((splitmix64(s) >> 11) + 1.0) * (1.0 / 9007199254740993.0); // (0, 1]
        double u2 = (splitmix64(s) >> 11) * (1.0 / 9007199254740992.0);         // [0, 1)
        R[i] = std::sqrt(-2.0 * std::log(u1)) * std::cos(two_pi * u2);
    }
    return R;
}

static inline int base2(uint8_t c)
{
    switch (c) {
    case 'A':
        return 0;
    case 'C':
        return 1;
    case 'G':
        return 2;
    case 'T':
        return 3;
    default:
        return -1;
    }
}

void embed_kmer3(const uint8_t *seqs, const int64_t *off, const int32_t *len, int64_t n, int dim, uint64_t seed,
                 float *out)
{
    const std::vector<double> R = kmer3_matrix(dim, seed);
#pragma omp parallel
    {
        std::vector<double> acc((size_t)dim);
#pragma omp for schedule(static)
        for (int64_t i = 0; i < n; ++i) {
            std::fill(acc.begin(), acc.end(), 0.0);
            const uint8_t *s = seqs + off[i];
            const int L = len[i];
            for (int t = 0; t + 3 <= L; ++t) {
                int a = base2(s[t]), b = base2(s[t + 1]), c = base2(s[t + 2]);
                if (a < 0 || b < 0 || c < 0)
                    continue;
                const double *r = &R[(size_t)(16 * a + 4 * b + c) * dim];
                for (int j = 0; j < dim; ++j)
                    acc[j] += r[j];
            }
            double nrm = 0.0;
            for (int j = 0; j < dim; ++j)
                nrm += acc[j] * acc[j];
            nrm = std::sqrt(nrm);
            float *o = out + (size_t)i * dim;
            for (int j = 0; j < dim; ++j)
                o[j] = nrm > 0.0 ? (float)(acc[j] / nrm) : 0.0f;
        }
    }
}

} // namespace drm

extern "C" int drm_embed_kmer3(const uint8_t *seqs, const int64_t *off, const int32_t *len, int64_t n, int32_t dim,
                               uint64_t seed, float *out)
{
    if (n < 0 || dim <= 0 || (n > 0 && (!seqs || !off || !len || !out))) {
        drm::set_last_error("drm_embed_kmer3: invalid argument");
        return DRM_ERR_ARG;
    }
    drm::embed_kmer3(seqs, off, len, n, dim, seed, out);
    return DRM_OK;
}
