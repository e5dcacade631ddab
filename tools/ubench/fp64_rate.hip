// Micro-benchmark: issue cost of float64 VALU ops (v_add_f64, v_mul_f64, v_fma_f64) on gfx950,
// 8 independent chains per wave, 1 / 2 / 4 waves per SIMD; modes 3-4: the same FMA / add with one
// operand read from an SGPR pair (a wave-uniform constant, as the compiler places bconst-style
// coefficients).  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
#define N_ITER 4096
template <int MODE>
__global__ void k(double *out, double s) {
    double x[8], y = s * 1.0001, z = s * 0.5;
    const double ys = __builtin_bit_cast(double, __builtin_amdgcn_readfirstlane(0) == 0 ? __builtin_bit_cast(long long, s * 1.0001) : 0ll);
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = s + threadIdx.x + i;
    for (int i = 0; i < N_ITER; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (MODE == 0) asm volatile("v_add_f64 %0, %0, %1" : "+v"(x[j]) : "v"(y));
            if (MODE == 1) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(x[j]) : "v"(y));
            if (MODE == 2) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(x[j]) : "v"(y), "v"(z));
            if (MODE == 3) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(x[j]) : "s"(ys), "v"(z));
            if (MODE == 4) asm volatile("v_add_f64 %0, %0, %1" : "+v"(x[j]) : "s"(ys));
        }
    }
    double r = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r += x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
template <int MODE>
void run(double *o, hipEvent_t e0, hipEvent_t e1, const char *name) {
    for (int wps : {1, 2, 4}) {
        float ms = 0;
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(k<MODE>, dim3(256), dim3(64 * 4 * wps), 0, 0, o, 1.0);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
        }
        printf("%-10s waves/SIMD %d: %.3f ms -> %.2f cyc per wave-instruction per SIMD (2.4 GHz)\n", name, wps, ms,
               ms * 1e-3 * 2.4e9 / ((double)N_ITER * 8 * wps));
    }
}
int main() {
    double *o;
    (void)hipMalloc(&o, 256 * 1024 * sizeof(double));
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    run<0>(o, e0, e1, "v_add_f64");
    run<1>(o, e0, e1, "v_mul_f64");
    run<2>(o, e0, e1, "v_fma_f64");
    run<3>(o, e0, e1, "fma sgpr");
    run<4>(o, e0, e1, "add sgpr");
    return 0;
}
