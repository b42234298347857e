// VALU issue-rate probe for gfx950: cycles per wave64 instruction per SIMD for
// packed fp16 / fp32 ops at 1..8 waves per SIMD, independent and dependent chains.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef _Float16 h2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(64) void probe(float *out, int iters)
{
    h2 a0 = {(_Float16)(threadIdx.x * 1e-3f), (_Float16)1.0f}, a1 = a0 + a0, a2 = a1 + a0, a3 = a2 + a0;
    h2 a4 = a3 + a0, a5 = a4 + a0, a6 = a5 + a0, a7 = a6 + a0;
    const h2 d = {(_Float16)-0.0009765625f, (_Float16)0.0009765625f};
    float f0 = threadIdx.x, f1 = f0 + 1, f2 = f0 + 2, f3 = f0 + 3, f4 = f0 + 4, f5 = f0 + 5, f6 = f0 + 6, f7 = f0 + 7;
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
            } else { // one dependent v_pk_add_f16 chain
                P1(a0) P1(a0) P1(a0) P1(a0) P1(a0) P1(a0) P1(a0) P1(a0)
            }
        }
    }
    h2 s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    out[blockIdx.x * 64 + threadIdx.x] = (float)s.x + (float)s.y + f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7;
}

int main(int argc, char **argv)
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    float *out;
    hipMalloc(&out, sizeof(float) * 64 * cus * 32);
    const int iters = 4096;
    const char *names[] = {"v_pk_add_f16 indep", "v_pk_maximum3_f16 indep", "v_add_f32 indep", "v_pk_add_f16 dep chain"};
    for (int mode = 0; mode < 4; ++mode)
        for (int wps = 1; wps <= 8; wps *= 2) {
            const int grid = cus * 4 * wps;
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(e0);
                if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(grid), dim3(64), 0, 0, out, iters);
                if (mode == 1) hipLaunchKernelGGL(probe<1>, dim3(grid), dim3(64), 0, 0, out, iters);
                if (mode == 2) hipLaunchKernelGGL(probe<2>, dim3(grid), dim3(64), 0, 0, out, iters);
                if (mode == 3) hipLaunchKernelGGL(probe<3>, dim3(grid), dim3(64), 0, 0, out, iters);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
            }
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double ops_per_wave = (double)iters * 64; // 8 x 8 per iteration
            const double cyc = ms * 1e-3 * clk * 1e3;       // clockRate in kHz
            // waves per SIMD = wps; each SIMD ran wps waves x ops_per_wave instructions
            std::printf("%-26s waves/SIMD=%d  %.2f cycles per wave64 instr per SIMD (%.3f ms, clk %d MHz)\n", names[mode],
                        wps, cyc / (ops_per_wave * wps), ms, clk / 1000);
        }
    return 0;
}
