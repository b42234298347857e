// deepreadmapper_amd/csrc/encoder_gru.hip -- the read encoder on gfx950:
// Vectorizer::vectorize (src/inference/vectorize.cpp:34-141) = Preprocessor tokens
// (src/inference/preprocess.cpp:20-42) -> embedding -> 2 x bidirectional GRU (hidden 64,
// linear_before_reset) -> concat(final fwd h, final bwd h) of layer 2, as the IR
// models/finetuned_sgn33-new-a-Apr6.xml runs it under OpenVINO (src/inference/fast_model.cpp).
//
// Two kernels per chunk of tiles (32 reads each): layer 1, then layer 2; one workgroup = one (tile,
// direction), 4 waves, wave w owning hidden units [16w, +16), so 3 independent workgroups share a CU
// and their barriers and gate math overlap each other's MFMA chains. Each recurrence step is a [32 x K] x [K x 16]
// product per gate on the 16x16x32 f16 MFMA: the weights are f16 in the IR (exact B operands, held in
// VGPRs for the whole layer); the f32 state h enters as two f16 terms hi = f16(h), lo = f16(h - hi)
// (~22 significant bits, f32 accumulation), so the recurrence stays f32-grade at the f16 matrix rate.
// Layer 1's input x_t is the token's embedding row (f16-exact, K = 64, fused into the same chains);
// layer 2's input is layer 1's output [fwd | bwd] at t, written to HBM as hi/lo f16 by layer 1 and
// staged back through LDS one step ahead. Gate math per (read, unit):
//   z = s(x Wz' + h Rz' + bz), r = s(x Wr' + h Rr' + br), n = tanh(x Wn' + Wbn + r (h Rn' + Rbn)),
//   h' = n + z (h - n)                                       (OpenVINO GRUCell, linear_before_reset)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "drm_device.h"

namespace drm {
namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kT = 32;   // reads per tile: two 16-row MFMA blocks
constexpr int kL = 123;  // recurrence steps = Config::Inference::MAX_LEN (config.hpp:21)
constexpr int kH = 64;   // hidden units
constexpr int kHS = 72;  // LDS row stride (halfs) of h images: 144-B rows, conflict-free ds_read_b128
constexpr int kES = 72;  // LDS row stride (halfs) of embedding rows
// LDS row stride (halfs) of staged layer-1 outputs: 544-B rows = 34 16-B slots. A ds_read_b128 lane group (rows
// ar = lane & 15, chunk + kq = lane >> 4) then hits 16 distinct slots of the 256-B bank row (row stride = 2 slots mod
// 16; 528-B rows, 1 slot mod 16, put two lanes of each group on one slot: 2-way, profiles/r06/prof_enc)
constexpr int kXS = 272;
constexpr int kYR = 256; // layer-1 output row in HBM: hi[fwd 64 | bwd 64] | lo[fwd 64 | bwd 64]
constexpr int kRows = 1 + kTokenHashes;
// bytes per tile row of the staged token ids: 132 = 33 dwords, so the 16 rows a ds_read_u8 of one step reads fall on
// 16 different banks (128-B rows put all 16 on one bank: 16-way, profiles/r06/prof_enc)
constexpr int kTokStride = 132;
static_assert(kRows * kES * 2 <= 16384, "embedding rows fit their LDS slot");

__device__ __forceinline__ int lower(int c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }

__device__ __forceinline__ int cval(int c) // char2Val (preprocess.hpp:10-25), c lower-cased
{
    return c == 'a' ? 0 : c == 'c' ? 1 : c == 'g' ? 2 : c == 't' ? 3 : 7;
}

// hashToken (preprocess.hpp:32-49) of token t of a sequence of len >= 2 bytes, as
// Preprocessor::preprocess places it (preprocess.cpp:25-40); -1 past the sequence's tokens
__device__ __forceinline__ int token_hash(const uint8_t *s, int len, int t)
{
    const int n = min(kL, len);
    if (t >= n) return -1;
    int c0, c1, c2;
    if (t == n - 1) { // result[len - 1]: seq[len-2], seq[len-1], then seq[len] or '>'
        c0 = s[n - 2];
        c1 = s[n - 1];
        c2 = n < len ? s[n] : '>';
    } else if (t == 0) { // result[0]: '<', seq[0], seq[1] (seq[0] is the tag itself in tagged reads)
        c0 = '<';
        c1 = s[0];
        c2 = s[1];
    } else {
        c0 = s[t - 1];
        c1 = s[t];
        c2 = s[t + 1];
    }
    c0 = lower(c0);
    c1 = lower(c1);
    c2 = lower(c2);
    if (c0 == '<') return (cval(c1) << 2) + cval(c2);
    if (c2 == '>') return 16 + (cval(c0) << 2) + cval(c1);
    return 32 + (cval(c0) << 4) + (cval(c1) << 2) + cval(c2);
}

__device__ __forceinline__ float sigm(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float tanh_(float x) { return 2.f * __builtin_amdgcn_rcpf(1.f + __expf(-2.f * x)) - 1.f; }

__device__ __forceinline__ f4 mfma(h8 a, h8 b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }

struct EncArgs {
    const uint8_t *seqs;
    const int32_t *lens;
    int64_t stride, n, first_tile;
    const _Float16 *emb; // [kRows][64] (row 0 = padding id 0, row 1 + h = _Tok2Index[h])
    const _Float16 *W1, *R1, *W2, *R2;
    const float *B1, *B2; // [2][256] zrh: b_z, b_r, Wb_n, Rb_n
    _Float16 *y1;         // [tiles of this launch][kL][kT][kYR]
    float *out;           // [n][128]
    float h0;
    uint32_t *flags;      // [0] tokens past _Tok2Index (reference UB), [1] sequences shorter than 2
};

// Gate epilogue for one 16-row block: C layout col = lane & 15 (unit j), row = 4 (lane >> 4) + q.
__device__ __forceinline__ void gates(const f4 &z, const f4 &r, const f4 &gx, const f4 &gh, float *hp, int row0, int j,
                                      _Float16 *nh, _Float16 *nl)
{
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float zz = sigm(z[q]), rr = sigm(r[q]);
        const float nn = tanh_(gx[q] + rr * gh[q]);
        const float h = nn + zz * (hp[q] - nn);
        hp[q] = h;
        const _Float16 hi = (_Float16)h;
        const _Float16 lo = (_Float16)(h - (float)hi);
        nh[(row0 + q) * kHS + j] = hi;
        nl[(row0 + q) * kHS + j] = lo;
    }
}

// one h image = 32 rows of kHS halfs + 64 halfs of pad, so the hi and lo images of a buffer sit 32 banks
// apart (the layer-1 row copy reads both in one ds_read_b128 lane group)
constexpr int kImg = kT * kHS + 64;
constexpr size_t kHbDirBytes = size_t(2) * 2 * kImg * 2; // [buf][hi/lo] images of one direction
constexpr size_t kXbDirBytes = size_t(2) * kT * kXS * 2;     // [buf] staged layer-1 rows of one direction

// Layer 1 of one direction (blockIdx.y) for one tile (blockIdx.x): input = the tokens' embedding rows.
// 4 waves, wave w owning units [16w, +16); writes h_t (hi, lo) of every step to the tile's layer-1 rows.
#ifndef DRM_ENC_L1_WAVES
#define DRM_ENC_L1_WAVES 3 // waves per SIMD of layer 1 (its two row blocks' accumulators are live together)
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DRM_ENC_L1_WAVES))) void gru_layer1_kernel(EncArgs a)
{
    __shared__ __attribute__((aligned(16))) uint8_t smem[kHbDirBytes + 16384 + kT * kTokStride];
    _Float16 *hb = (_Float16 *)smem;
    _Float16 *embs = (_Float16 *)(smem + kHbDirBytes);
    uint8_t *toks = smem + kHbDirBytes + 16384;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int dir = blockIdx.y, j = (wave << 4) + (lane & 15), kq = lane >> 4, c16 = lane & 15;
    const int64_t r0 = (a.first_tile + blockIdx.x) * kT;
    _Float16 *y1 = a.y1 + (int64_t)blockIdx.x * kL * kT * kYR;
    auto himg = [&](int buf, int hl) { return hb + (buf * 2 + hl) * kImg; };

    for (int i = tid; i < kT * kTokStride; i += 256) {
        const int row = i / kTokStride, t = i % kTokStride;
        const int64_t r = r0 + row;
        int v = 0;
        if (r < a.n && t < kL) {
            const int len = a.lens[r];
            if (len >= 2) {
                const int h = token_hash(a.seqs + r * a.stride, len, t);
                if (dir == 0 && h >= kTokenHashes) atomicAdd(&a.flags[0], 1u);
                v = (h >= 0 && h < kTokenHashes) ? h + 1 : 0;
            } else if (t == 0 && dir == 0) {
                atomicAdd(&a.flags[1], 1u);
            }
        }
        toks[i] = (uint8_t)v;
    }
    for (int i = tid; i < kRows * 8; i += 256)
        *(h8 *)(embs + (i >> 3) * kES + (i & 7) * 8) = *(const h8 *)(a.emb + i * 8);
    const _Float16 h0hi = (_Float16)a.h0, h0lo = (_Float16)(a.h0 - (float)h0hi);
    for (int i = tid; i < kT * kH; i += 256) {
        himg(0, 0)[(i / kH) * kHS + i % kH] = h0hi;
        himg(0, 1)[(i / kH) * kHS + i % kH] = h0lo;
    }
    float hp[2][4];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int q = 0; q < 4; ++q) hp[rb][q] = a.h0;

    const _Float16 *R = a.R1 + dir * 3 * kH * kH, *W = a.W1 + dir * 3 * kH * 64;
    h8 rf[3][2], wf[3][2];
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            rf[g][c] = *(const h8 *)(R + (g * kH + j) * kH + c * 32 + kq * 8);
            wf[g][c] = *(const h8 *)(W + (g * kH + j) * 64 + c * 32 + kq * 8);
        }
    const float *B = a.B1 + dir * 4 * kH;
    const float bz = B[j], br = B[kH + j], bxn = B[2 * kH + j], bhn = B[3 * kH + j];
    __syncthreads();
    for (int s = 0; s < kL; ++s) {
        const int t = dir ? kL - 1 - s : s, cur = s & 1;
        const _Float16 *hh = himg(cur, 0), *hl = himg(cur, 1);
        _Float16 *nh = himg(cur ^ 1, 0), *nl = himg(cur ^ 1, 1);
        // both row blocks' MFMA chains first, then both gate epilogues: the second block's MFMAs
        // execute while the first block's gate math issues
        f4 z[2], r[2], gx[2], gh[2];
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
            const int ar = rb * 16 + c16;
            const h8 ah0 = *(const h8 *)(hh + ar * kHS + kq * 8), ah1 = *(const h8 *)(hh + ar * kHS + 32 + kq * 8);
            const h8 al0 = *(const h8 *)(hl + ar * kHS + kq * 8), al1 = *(const h8 *)(hl + ar * kHS + 32 + kq * 8);
            const int tr = toks[ar * kTokStride + t];
            const h8 ax0 = *(const h8 *)(embs + tr * kES + kq * 8), ax1 = *(const h8 *)(embs + tr * kES + 32 + kq * 8);
            z[rb] = f4{bz, bz, bz, bz};
            r[rb] = f4{br, br, br, br};
            gx[rb] = f4{bxn, bxn, bxn, bxn};
            gh[rb] = f4{bhn, bhn, bhn, bhn};
            z[rb] = mfma(ax0, wf[0][0], z[rb]);
            r[rb] = mfma(ax0, wf[1][0], r[rb]);
            gx[rb] = mfma(ax0, wf[2][0], gx[rb]);
            gh[rb] = mfma(ah0, rf[2][0], gh[rb]);
            z[rb] = mfma(ax1, wf[0][1], z[rb]);
            r[rb] = mfma(ax1, wf[1][1], r[rb]);
            gx[rb] = mfma(ax1, wf[2][1], gx[rb]);
            gh[rb] = mfma(ah1, rf[2][1], gh[rb]);
            z[rb] = mfma(ah0, rf[0][0], z[rb]);
            r[rb] = mfma(ah0, rf[1][0], r[rb]);
            gh[rb] = mfma(al0, rf[2][0], gh[rb]);
            z[rb] = mfma(ah1, rf[0][1], z[rb]);
            r[rb] = mfma(ah1, rf[1][1], r[rb]);
            gh[rb] = mfma(al1, rf[2][1], gh[rb]);
            z[rb] = mfma(al0, rf[0][0], z[rb]);
            r[rb] = mfma(al0, rf[1][0], r[rb]);
            z[rb] = mfma(al1, rf[0][1], z[rb]);
            r[rb] = mfma(al1, rf[1][1], r[rb]);
        }
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
            gates(z[rb], r[rb], gx[rb], gh[rb], hp[rb], rb * 16 + kq * 4, j, nh, nl);
        __syncthreads();
        // h_t (hi, lo) of this direction -> the tile's layer-1 row t: 32 rows x 2 x 128 B, 2 x 16 B per thread
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int c = tid + 256 * i, row = c >> 4, hlsel = (c >> 3) & 1, seg = c & 7;
            *(h8 *)(y1 + ((int64_t)t * kT + row) * kYR + hlsel * 128 + dir * kH + seg * 8) =
                *(const h8 *)((hlsel ? nl : nh) + row * kHS + seg * 8);
        }
    }
}

// Layer 2 of one direction (blockIdx.y) for one tile: input = layer 1's [fwd | bwd] rows (hi/lo),
// staged through LDS one step ahead; writes the final state to out[:, 64 dir ..].
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void gru_layer2_kernel(EncArgs a)
{
    __shared__ __attribute__((aligned(16))) uint8_t smem[kHbDirBytes + kXbDirBytes];
    _Float16 *hb = (_Float16 *)smem;
    _Float16 *xb = (_Float16 *)(smem + kHbDirBytes);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int dir = blockIdx.y, j = (wave << 4) + (lane & 15), kq = lane >> 4, c16 = lane & 15;
    const int64_t r0 = (a.first_tile + blockIdx.x) * kT;
    const _Float16 *y1 = a.y1 + (int64_t)blockIdx.x * kL * kT * kYR;
    auto himg = [&](int buf, int hl) { return hb + (buf * 2 + hl) * kImg; };

    const _Float16 *R = a.R2 + dir * 3 * kH * kH, *W = a.W2 + dir * 3 * kH * 2 * kH;
    h8 rf[3][2], wf[3][4];
#pragma unroll
    for (int g = 0; g < 3; ++g) {
#pragma unroll
        for (int c = 0; c < 2; ++c) rf[g][c] = *(const h8 *)(R + (g * kH + j) * kH + c * 32 + kq * 8);
#pragma unroll
        for (int c = 0; c < 4; ++c) wf[g][c] = *(const h8 *)(W + (g * kH + j) * 2 * kH + c * 32 + kq * 8);
    }
    const float *B = a.B2 + dir * 4 * kH;
    const float bz = B[j], br = B[kH + j], bxn = B[2 * kH + j], bhn = B[3 * kH + j];
    float hp[2][4];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int q = 0; q < 4; ++q) hp[rb][q] = a.h0;
    const _Float16 h0hi = (_Float16)a.h0, h0lo = (_Float16)(a.h0 - (float)h0hi);
    for (int i = tid; i < kT * kH; i += 256) {
        himg(0, 0)[(i / kH) * kHS + i % kH] = h0hi;
        himg(0, 1)[(i / kH) * kHS + i % kH] = h0lo;
    }
    // 32 rows x 512 B of layer-1 output per step: 4 x 16 B per thread
    h8 xr[4];
    auto load_x = [&](int t) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int c = tid + 256 * i, row = c >> 5, seg = c & 31;
            xr[i] = *(const h8 *)(y1 + ((int64_t)t * kT + row) * kYR + seg * 8);
        }
    };
    auto store_x = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int c = tid + 256 * i, row = c >> 5, seg = c & 31;
            *(h8 *)(xb + buf * kT * kXS + row * kXS + seg * 8) = xr[i];
        }
    };
    load_x(dir ? kL - 1 : 0);
    store_x(0);
    __syncthreads();
    for (int s = 0; s < kL; ++s) {
        const int cur = s & 1;
        if (s + 1 < kL) load_x(dir ? kL - 2 - s : s + 1);
        const _Float16 *hh = himg(cur, 0), *hl = himg(cur, 1);
        _Float16 *nh = himg(cur ^ 1, 0), *nl = himg(cur ^ 1, 1);
        const _Float16 *xs = xb + cur * kT * kXS;
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
            const int ar = rb * 16 + c16;
            const h8 ah0 = *(const h8 *)(hh + ar * kHS + kq * 8), ah1 = *(const h8 *)(hh + ar * kHS + 32 + kq * 8);
            const h8 al0 = *(const h8 *)(hl + ar * kHS + kq * 8), al1 = *(const h8 *)(hl + ar * kHS + 32 + kq * 8);
            f4 z = {bz, bz, bz, bz}, r = {br, br, br, br}, gx = {bxn, bxn, bxn, bxn}, gh = {bhn, bhn, bhn, bhn};
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const h8 xh = *(const h8 *)(xs + ar * kXS + c * 32 + kq * 8);
                const h8 xl = *(const h8 *)(xs + ar * kXS + 128 + c * 32 + kq * 8);
                z = mfma(xh, wf[0][c], z);
                r = mfma(xh, wf[1][c], r);
                gx = mfma(xh, wf[2][c], gx);
                z = mfma(xl, wf[0][c], z);
                r = mfma(xl, wf[1][c], r);
                gx = mfma(xl, wf[2][c], gx);
            }
            gh = mfma(ah0, rf[2][0], gh);
            z = mfma(ah0, rf[0][0], z);
            r = mfma(ah0, rf[1][0], r);
            gh = mfma(ah1, rf[2][1], gh);
            z = mfma(ah1, rf[0][1], z);
            r = mfma(ah1, rf[1][1], r);
            gh = mfma(al0, rf[2][0], gh);
            z = mfma(al0, rf[0][0], z);
            r = mfma(al0, rf[1][0], r);
            gh = mfma(al1, rf[2][1], gh);
            z = mfma(al1, rf[0][1], z);
            r = mfma(al1, rf[1][1], r);
            gates(z, r, gx, gh, hp[rb], rb * 16 + kq * 4, j, nh, nl);
        }
        if (s + 1 < kL) store_x(cur ^ 1);
        __syncthreads();
    }
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t r = r0 + rb * 16 + kq * 4 + q;
            if (r < a.n) a.out[r * 128 + dir * kH + j] = hp[rb][q];
        }
}

// Preprocessor::preprocess + Vectorizer::prepareBatch's zero padding as model-input ids: one thread
// per (sequence, position); -1 where the reference indexes past _Tok2Index.
__global__ void tokenize_kernel(const uint8_t *seqs, const int32_t *lens, int64_t stride, int64_t n,
                                const uint16_t *vocab, int32_t *tokens)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * kL) return;
    const int64_t r = i / kL;
    const int t = int(i % kL);
    const int len = lens[r];
    int v = 0;
    if (len >= 2) {
        const int h = token_hash(seqs + r * stride, len, t);
        v = h < 0 ? 0 : h < kTokenHashes ? vocab[1 + h] : -1;
    }
    tokens[i] = v;
}

} // namespace

int64_t encoder_tile_bytes() { return int64_t(kL) * kT * kYR * 2; }

void encoder_upload(DeviceEncoder &d, const EncoderHost &h, int device)
{
    if ((int)h.emb_rows.size() != kRows * 64 || h.hidden != kH || h.emb_dim != 64 || h.max_len != kL)
        throw Error(DRM_ERR_UNSUPPORTED, "encoder: unsupported model shape");
    d.device = device;
    d.h0 = h.h0;
    DRM_HIP_CHECK(hipSetDevice(device));
    auto up16 = [&](const std::vector<uint16_t> &v, uint16_t **p) {
        DRM_HIP_CHECK(hipMalloc(p, v.size() * 2));
        DRM_HIP_CHECK(hipMemcpy(*p, v.data(), v.size() * 2, hipMemcpyHostToDevice));
        d.device_bytes += v.size() * 2;
    };
    up16(h.emb_rows, &d.emb);
    up16(h.vocab_rows, &d.vocab);
    for (int l = 0; l < 2; ++l) {
        up16(h.W[l], &d.W[l]);
        up16(h.R[l], &d.R[l]);
        std::vector<float> b(h.B[l].size());
        for (size_t i = 0; i < b.size(); ++i) {
            _Float16 x;
            memcpy(&x, &h.B[l][i], 2);
            b[i] = (float)x;
        }
        DRM_HIP_CHECK(hipMalloc(&d.B[l], b.size() * 4));
        DRM_HIP_CHECK(hipMemcpy(d.B[l], b.data(), b.size() * 4, hipMemcpyHostToDevice));
    }
    DRM_HIP_CHECK(hipMalloc(&d.flags, 16));
    DRM_HIP_CHECK(hipMemset(d.flags, 0, 16));
}

void encoder_release(DeviceEncoder &d)
{
    (void)hipSetDevice(d.device);
    for (void *p : {(void *)d.emb, (void *)d.vocab, (void *)d.W[0], (void *)d.W[1], (void *)d.R[0], (void *)d.R[1],
                    (void *)d.B[0], (void *)d.B[1], (void *)d.y1, (void *)d.flags})
        if (p) (void)hipFree(p);
    d = DeviceEncoder{};
}

void launch_encode(DeviceEncoder &d, const uint8_t *d_seqs, const int32_t *d_lens, int64_t n, int64_t stride,
                   float *d_out, hipStream_t stream)
{
    if (n <= 0) return;
    const int64_t tiles = (n + kT - 1) / kT;
    int64_t per = std::min<int64_t>(tiles, d.max_tiles_per_launch);
    if (d.y1_tiles < per) {
        if (d.y1) DRM_HIP_CHECK(hipFree(d.y1));
        d.y1 = nullptr;
        DRM_HIP_CHECK(hipMalloc(&d.y1, per * encoder_tile_bytes()));
        d.y1_tiles = per;
    }
    EncArgs a{};
    a.seqs = d_seqs;
    a.lens = d_lens;
    a.stride = stride;
    a.n = n;
    a.emb = (const _Float16 *)d.emb;
    a.W1 = (const _Float16 *)d.W[0];
    a.R1 = (const _Float16 *)d.R[0];
    a.W2 = (const _Float16 *)d.W[1];
    a.R2 = (const _Float16 *)d.R[1];
    a.B1 = d.B[0];
    a.B2 = d.B[1];
    a.y1 = (_Float16 *)d.y1;
    a.out = d_out;
    a.h0 = d.h0;
    a.flags = d.flags;
    for (int64_t t0 = 0; t0 < tiles; t0 += per) {
        a.first_tile = t0;
        const int64_t nt = std::min(per, tiles - t0);
        hipLaunchKernelGGL(gru_layer1_kernel, dim3((unsigned)nt, 2), dim3(256), 0, stream, a);
        DRM_HIP_CHECK(hipGetLastError());
        hipLaunchKernelGGL(gru_layer2_kernel, dim3((unsigned)nt, 2), dim3(256), 0, stream, a);
        DRM_HIP_CHECK(hipGetLastError());
    }
}

void launch_tokenize(const DeviceEncoder &d, const uint8_t *d_seqs, const int32_t *d_lens, int64_t n, int64_t stride,
                     int32_t *d_tokens, hipStream_t stream)
{
    if (n <= 0) return;
    const int64_t total = n * kL;
    hipLaunchKernelGGL(tokenize_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, d_seqs, d_lens,
                       stride, n, d.vocab, d_tokens);
    DRM_HIP_CHECK(hipGetLastError());
}

} // namespace drm
