// Micro-benchmark: issue cost of v_pk_add_f32 vs v_add_f32 (wave64, gfx950), 8 independent
// chains per wave, 1 / 2 / 4 / 8 waves per SIMD.  Build: hipcc --offload-arch=gfx950 -O3 pk_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#define N_ITER 4096
template <int PK>
__global__ void k(float *out, float s) {
    float a0 = s + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
          a7 = a0 + 7, a8 = a0 + 8, a9 = a0 + 9, a10 = a0 + 10, a11 = a0 + 11, a12 = a0 + 12, a13 = a0 + 13,
          a14 = a0 + 14, a15 = a0 + 15;
    for (int i = 0; i < N_ITER; ++i) {
        if (PK) {
            asm volatile(
                "v_pk_add_f32 %0, %0, %0\n v_pk_add_f32 %1, %1, %1\n v_pk_add_f32 %2, %2, %2\n v_pk_add_f32 %3, %3, %3\n"
                "v_pk_add_f32 %4, %4, %4\n v_pk_add_f32 %5, %5, %5\n v_pk_add_f32 %6, %6, %6\n v_pk_add_f32 %7, %7, %7\n"
                : "+v"(*(double *)&a0), "+v"(*(double *)&a2), "+v"(*(double *)&a4), "+v"(*(double *)&a6),
                  "+v"(*(double *)&a8), "+v"(*(double *)&a10), "+v"(*(double *)&a12), "+v"(*(double *)&a14));
        } else {
            asm volatile(
                "v_add_f32 %0, %0, %0\n v_add_f32 %1, %1, %1\n v_add_f32 %2, %2, %2\n v_add_f32 %3, %3, %3\n"
                "v_add_f32 %4, %4, %4\n v_add_f32 %5, %5, %5\n v_add_f32 %6, %6, %6\n v_add_f32 %7, %7, %7\n"
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + a8 + a9 + a10 + a11 + a12 +
                                                 a13 + a14 + a15;
}
int main() {
    float *o;
    hipMalloc(&o, 256 * 8 * 256 * 4 * sizeof(float));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int wps : {1, 2, 4, 8}) {
        for (int pk = 0; pk < 2; ++pk) {
            dim3 grid(256), block(64 * 4 * wps);
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(e0);
                if (pk) hipLaunchKernelGGL(k<1>, grid, block, 0, 0, o, 1.0f);
                else hipLaunchKernelGGL(k<0>, grid, block, 0, 0, o, 1.0f);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
            }
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            double insts_per_simd = (double)N_ITER * 8 * wps;  // per SIMD
            double cyc = ms * 1e-3 * 2.4e9;                       // at 2.4 GHz nominal
            printf("waves/SIMD %d %s: %.3f ms  -> %.2f cycles per wave-instruction per SIMD (2.4 GHz)\n", wps,
                   pk ? "v_pk_add_f32" : "v_add_f32   ", ms, cyc / insts_per_simd);
        }
    }
    return 0;
}
