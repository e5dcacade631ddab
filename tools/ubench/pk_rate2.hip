// Micro-benchmark 2: issue cost of packed f32 ops (v_pk_fma_f32 / v_pk_add_f32 / v_pk_mul_f32) with
// DISTINCT source registers (pk_rate.hip read both sources from the destination pair), vs
// v_fma_f32 / v_add_f32, 8 independent accumulator chains per wave, 1 / 2 / 4 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 pk_rate2.hip -o pk_rate2
#include <hip/hip_runtime.h>
#include <cstdio>
#define N_ITER 4096
typedef float f2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ void k(float *out, float s) {
    f2 a[8], b, c;
    b = f2{s * 1.0001f, s * 0.9999f};
    c = f2{s * 0.5f, s * 0.25f};
    float x[8], y = s * 1.0001f, z = s * 0.5f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        a[i] = f2{s + threadIdx.x + i, s - i};
        x[i] = s + threadIdx.x + i;
    }
    for (int i = 0; i < N_ITER; ++i) {
        if (MODE == 0) {
#pragma unroll
            for (int j = 0; j < 8; ++j) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[j]) : "v"(y), "v"(z));
        } else if (MODE == 1) {
#pragma unroll
            for (int j = 0; j < 8; ++j) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(a[j]) : "v"(b), "v"(c));
        } else if (MODE == 2) {
#pragma unroll
            for (int j = 0; j < 8; ++j) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
        } else if (MODE == 3) {
#pragma unroll
            for (int j = 0; j < 8; ++j) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
        } else if (MODE == 4) {
#pragma unroll
            for (int j = 0; j < 8; ++j) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[j]) : "v"(y));
        } else if (MODE == 5) {  // alternating packed / scalar
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(a[j]) : "v"(b), "v"(c));
                asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[j]) : "v"(y), "v"(z));
            }
        }
    }
    float r = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) r += a[i].x + a[i].y + x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int MODE>
void run(float *o, hipEvent_t e0, hipEvent_t e1, const char *name) {
    for (int wps : {1, 2, 4}) {
        dim3 grid(256), block(64 * 4 * wps);
        float ms = 0;
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(k<MODE>, grid, block, 0, 0, o, 1.0f);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&ms, e0, e1);
        }
        double insts = (double)N_ITER * 8 * wps;  // per SIMD
        printf("%-28s waves/SIMD %d: %.3f ms -> %.2f cyc per wave-instruction per SIMD (2.4 GHz)\n", name, wps, ms,
               ms * 1e-3 * 2.4e9 / insts);
    }
}

int main() {
    float *o;
    hipMalloc(&o, 256 * 1024 * sizeof(float));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    run<0>(o, e0, e1, "v_fma_f32");
    run<4>(o, e0, e1, "v_add_f32");
    run<1>(o, e0, e1, "v_pk_fma_f32 (distinct src)");
    run<2>(o, e0, e1, "v_pk_add_f32 (distinct src)");
    run<3>(o, e0, e1, "v_pk_mul_f32 (distinct src)");
    run<5>(o, e0, e1, "pk_fma / fma alternating");
    return 0;
}
