// deepreadmapper_amd/csrc/embed_gpu.hip -- the stand-in 3-mer embedder of embed.cpp on the device, for
// tables of fixed-length rows (the window table of a synthetic genome: 50M rows at C5 would take the
// host minutes). Stand-in for the OpenVINO encoder (src/inference/vectorize.cpp:34-141), used by the
// synthetic workloads only. fp64 sums in the host's order, correctly rounded sqrt and division: the
// outputs are bit-identical to drm_embed_kmer3.
#include <hip/hip_runtime.h>

#include <vector>

#include "drm_device.h"

#pragma clang fp contract(off)

namespace drm {
namespace {

constexpr int kRowsPerBlock = 16;

__device__ __forceinline__ int base2_d(uint8_t c)
{
    return c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : c == 'T' ? 3 : -1;
}

// One 64-lane block per group of 16 rows: lane j accumulates dims j and j + 64 of one row at a time
// (3-mers in sequence order), then lane r < 16 forms row r's norm sequentially over the 128 dims.
__global__ __launch_bounds__(64) void embed_rows_kernel(const uint8_t *rows, int64_t n, int len, int64_t stride,
                                                        const double *R, float *out)
{
    __shared__ double acc_s[kRowsPerBlock][129]; // padded: lane r reads row r's column t conflict-free
    __shared__ double nrm_s[kRowsPerBlock];
    __shared__ uint8_t seq_s[512];
    const int lane = threadIdx.x;
    for (int64_t base = (int64_t)blockIdx.x * kRowsPerBlock; base < n; base += (int64_t)gridDim.x * kRowsPerBlock) {
        const int cnt = (int)min((int64_t)kRowsPerBlock, n - base);
        for (int r = 0; r < cnt; ++r) {
            const uint8_t *s = rows + (base + r) * stride;
            for (int t = lane; t < len; t += 64)
                seq_s[t] = s[t];
            __syncthreads();
            double a0 = 0.0, a1 = 0.0;
            for (int t = 0; t + 3 <= len; ++t) {
                const int b0 = base2_d(seq_s[t]), b1 = base2_d(seq_s[t + 1]), b2 = base2_d(seq_s[t + 2]);
                if (b0 < 0 || b1 < 0 || b2 < 0)
                    continue;
                const double *rr = R + (size_t)(16 * b0 + 4 * b1 + b2) * 128;
                a0 = __dadd_rn(a0, rr[lane]);
                a1 = __dadd_rn(a1, rr[lane + 64]);
            }
            acc_s[r][lane] = a0;
            acc_s[r][lane + 64] = a1;
            __syncthreads();
        }
        if (lane < cnt) {
            double s = 0.0;
            for (int j = 0; j < 128; ++j)
                s = __dadd_rn(s, __dmul_rn(acc_s[lane][j], acc_s[lane][j]));
            nrm_s[lane] = __dsqrt_rn(s);
        }
        __syncthreads();
        for (int r = 0; r < cnt; ++r) {
            const double nrm = nrm_s[r];
            float *o = out + (base + r) * 128;
            o[lane] = nrm > 0.0 ? (float)__ddiv_rn(acc_s[r][lane], nrm) : 0.0f;
            o[lane + 64] = nrm > 0.0 ? (float)__ddiv_rn(acc_s[r][lane + 64], nrm) : 0.0f;
        }
        __syncthreads();
    }
}

} // namespace
} // namespace drm

extern "C" int drm_embed_kmer3_device(const uint8_t *d_rows, int64_t n, int32_t len, int64_t row_stride, int32_t dim,
                                      uint64_t seed, float *d_out, void *stream)
{
    try {
        if (n < 0 || len < 0 || len > 512 || row_stride < len || (n > 0 && (!d_rows || !d_out)))
            throw drm::Error(DRM_ERR_ARG, "drm_embed_kmer3_device: invalid argument (rows of <= 512 bytes)");
        if (dim != 128)
            throw drm::Error(DRM_ERR_UNSUPPORTED, "drm_embed_kmer3_device: dim must be 128");
        if (n == 0)
            return DRM_OK;
        const std::vector<double> R = drm::kmer3_matrix(dim, seed);
        double *dR = nullptr;
        DRM_HIP_CHECK(hipMalloc(&dR, sizeof(double) * R.size()));
        DRM_HIP_CHECK(hipMemcpy(dR, R.data(), sizeof(double) * R.size(), hipMemcpyHostToDevice));
        const int64_t groups = (n + drm::kRowsPerBlock - 1) / drm::kRowsPerBlock;
        const int grid = (int)std::min<int64_t>(groups, 65536);
        hipLaunchKernelGGL(drm::embed_rows_kernel, dim3(grid), dim3(64), 0, (hipStream_t)stream, d_rows, n, len,
                           row_stride, dR, d_out);
        const hipError_t e = hipGetLastError();
        DRM_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
        (void)hipFree(dR);
        if (e != hipSuccess)
            throw drm::Error(DRM_ERR_HIP, std::string("embed_rows_kernel launch: ") + hipGetErrorString(e));
        return DRM_OK;
    } catch (const drm::Error &e) {
        drm::set_last_error(e.what());
        return e.code;
    }
}
