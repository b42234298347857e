// VALU issue-rate probe for gfx950: cycles per wave64 instruction per SIMD for
// packed fp16 / fp32 ops at 1..8 waves per SIMD, independent and dependent chains; modes 4-6: the SW rerank's
// cell-pair instruction mix (sw_rerank.hip sw_rows_i16), timed with the shader clock (s_memtime) inside the
// kernel as well as with events at the nominal clock.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef _Float16 h2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(64) void probe(float *out, unsigned long long *cyc, int iters)
{
    h2 a0 = {(_Float16)(threadIdx.x * 1e-3f), (_Float16)1.0f}, a1 = a0 + a0, a2 = a1 + a0, a3 = a2 + a0;
    h2 a4 = a3 + a0, a5 = a4 + a0, a6 = a5 + a0, a7 = a6 + a0;
    const h2 d = {(_Float16)-0.0009765625f, (_Float16)0.0009765625f};
    float f0 = threadIdx.x, f1 = f0 + 1, f2 = f0 + 2, f3 = f0 + 3, f4 = f0 + 4, f5 = f0 + 5, f6 = f0 + 6, f7 = f0 + 7;
    uint32_t x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    uint32_t t = threadIdx.x & 1 ? 0x20000u : 0x2u, u0 = 3u, u1 = 5u, bst = 0u;
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (MODE == 0) { // 8 independent v_pk_add_f16
#define P1(x) asm volatile("v_pk_add_f16 %0, %0, %1" : "+v"(x) : "v"(d));
                P1(a0) P1(a1) P1(a2) P1(a3) P1(a4) P1(a5) P1(a6) P1(a7)
            } else if (MODE == 1) { // 8 independent v_pk_maximum3_f16
#define P2(x, y) asm volatile("v_pk_maximum3_f16 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(d));
                P2(a0, d) P2(a1, d) P2(a2, d) P2(a3, d) P2(a4, d) P2(a5, d) P2(a6, d) P2(a7, d)
            } else if (MODE == 2) { // 8 independent v_add_f32
#define P3(x) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(f7));
                P3(f0) P3(f1) P3(f2) P3(f3) P3(f4) P3(f5) P3(f6) P3(f0)
            } else if (MODE == 3) { // one dependent v_pk_add_f16 chain
                P1(a0) P1(a0) P1(a0) P1(a0) P1(a0) P1(a0) P1(a0) P1(a0)
            } else if (MODE == 4 || MODE == 5) {
                // 8 SW cell pairs: diag add (MODE 4: v_add_u32, MODE 5: v_pk_add_u16), packed max3, packed saturating
                // subtract, and 4 packed max3 into the best: the per-cell-pair mix of the SW DP, 28 instructions per
                // 8 cell pairs (12 issue cycles per pair if the add takes 2 and the packed ops 4)
#define ADD(x) if (MODE == 4) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(t)); \
               else asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x) : "v"(t));
#define MX(x) asm volatile("v_pk_maximum3_f16 %0, %0, %1, %2" : "+v"(x) : "v"(u0), "v"(u1));
#define SB(x) asm volatile("v_pk_sub_u16 %0, %0, 1 op_sel_hi:[1,0] clamp" : "+v"(x));
#define BS(x, y) asm volatile("v_pk_maximum3_f16 %0, %0, %1, %2" : "+v"(bst) : "v"(x), "v"(y));
                ADD(x0) ADD(x1) ADD(x2) ADD(x3) ADD(x4) ADD(x5) ADD(x6) ADD(x7)
                MX(x0) MX(x1) MX(x2) MX(x3) MX(x4) MX(x5) MX(x6) MX(x7)
                SB(x0) SB(x1) SB(x2) SB(x3) SB(x4) SB(x5) SB(x6) SB(x7)
                BS(x0, x1) BS(x2, x3) BS(x4, x5) BS(x6, x7)
            } else { // 8 independent v_add_u32
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(x0) : "v"(t));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(x1) : "v"(t));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(x2) : "v"(t));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(x3) : "v"(t));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(x4) : "v"(t));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(x5) : "v"(t));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(x6) : "v"(t));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(x7) : "v"(t));
            }
        }
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
    h2 s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    out[blockIdx.x * 64 + threadIdx.x] = (float)s.x + (float)s.y + f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7 +
                                         (float)(x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7 ^ bst);
    if (threadIdx.x == 0)
        cyc[blockIdx.x] = c1 - c0; // this wave's loop, in shader clocks
}

int main(int argc, char **argv)
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    float *out;
    hipMalloc(&out, sizeof(float) * 64 * cus * 32);
    unsigned long long *cyc;
    hipMalloc(&cyc, sizeof(unsigned long long) * cus * 32);
    unsigned long long *hcyc = (unsigned long long *)std::malloc(sizeof(unsigned long long) * cus * 32);
    const int iters = 16384;
    const char *names[] = {"v_pk_add_f16 indep", "v_pk_maximum3_f16 indep", "v_add_f32 indep", "v_pk_add_f16 dep chain",
                           "SW mix (v_add_u32)", "SW mix (v_pk_add_u16)", "v_add_u32 indep"};
    const double per_iter[] = {64, 64, 64, 64, 8 * 28, 8 * 28, 64}; // instructions per loop iteration
    for (int mode = 0; mode < 7; ++mode)
        for (int wps = 1; wps <= 8; wps *= 2) {
            const int grid = cus * 4 * wps;
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(e0);
                if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(grid), dim3(64), 0, 0, out, cyc, iters);
                if (mode == 1) hipLaunchKernelGGL(probe<1>, dim3(grid), dim3(64), 0, 0, out, cyc, iters);
                if (mode == 2) hipLaunchKernelGGL(probe<2>, dim3(grid), dim3(64), 0, 0, out, cyc, iters);
                if (mode == 3) hipLaunchKernelGGL(probe<3>, dim3(grid), dim3(64), 0, 0, out, cyc, iters);
                if (mode == 4) hipLaunchKernelGGL(probe<4>, dim3(grid), dim3(64), 0, 0, out, cyc, iters);
                if (mode == 5) hipLaunchKernelGGL(probe<5>, dim3(grid), dim3(64), 0, 0, out, cyc, iters);
                if (mode == 6) hipLaunchKernelGGL(probe<6>, dim3(grid), dim3(64), 0, 0, out, cyc, iters);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
            }
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double ops_per_wave = (double)iters * per_iter[mode];
            const double ev_cyc = ms * 1e-3 * clk * 1e3; // clockRate in kHz
            hipMemcpy(hcyc, cyc, sizeof(unsigned long long) * grid, hipMemcpyDeviceToHost);
            double wc = 0;
            for (int g = 0; g < grid; ++g)
                wc += (double)hcyc[g];
            wc /= grid; // mean shader clocks of one wave's loop, all waves of a SIMD running together
            // waves per SIMD = wps; each SIMD ran wps waves x ops_per_wave instructions
            // the s_memtime figure is one wave's own loop: the SIMD's rate only when its waves run side by side for the
            // whole loop (exact at 1 wave per SIMD; at more, staggered waves make it read low)
            std::printf("%-26s waves/SIMD=%d  %.2f cycles per wave64 instr per SIMD at the nominal clock, %.2f by s_memtime"
                        " (%.3f ms, clk %d MHz, per-wave %.0f MHz)\n",
                        names[mode], wps, ev_cyc / (ops_per_wave * wps), wc / (ops_per_wave * wps), ms, clk / 1000,
                        wc / (ms * 1e-3) / 1e6);
        }
    return 0;
}
