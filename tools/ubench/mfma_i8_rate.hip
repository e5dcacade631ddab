// Whole-chip int8 MFMA throughput on gfx950, timed with HIP events (the Welch int8
// kernel's ceiling).  r4's mfma_i8.hip timed one wave per SIMD with s_memtime; this one fills every
// CU with W waves per SIMD and reports TOPS against the 5 POPS dense int8 peak:
//  (a) v_mfma_i32_16x16x64_i8, NM independent accumulators per wave, W = 1..4 waves per SIMD;
//  (b) v_mfma_i32_32x32x32_i8 (same ops per instruction x 2, half the operand bytes per op);
//  (c) mixed waves: W MFMA waves per SIMD plus one wave per SIMD doing NV float64 FMAs per
//      iteration -- whether float64 work on another wave of the SIMD steals MFMA issue;
//  (d) the same with int32 VALU work (v_add / v_lshl_add) in place of the float64.
// Build: hipcc --offload-arch=gfx950 -O3 mfma_i8_rate.hip -o bin/mfma_i8_rate
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(3);                                                                  \
        }                                                                                  \
    } while (0)

// KIND 0: MFMA wave; waves with (wave index % 4 == 3 and MIX) do side work instead:
// MIX 1 float64 FMAs, MIX 2 int32 VALU
template <int NM, bool BIG, int MIX, int NV>
__global__ __launch_bounds__(1024) void k_rate(int *out, double *dout, int iters, int seed) {
    const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int nw = blockDim.x >> 6;
    // the side wave: the last 4 waves of the workgroup (one per SIMD)
    const bool side = MIX && wv >= nw - 4;
    if (!side) {
        v4i a = {seed + l, seed * 3 + l, l ^ seed, 7 * l}, b = {l, seed - l, 5 * l, seed};
        if (BIG) {
            v16i c[NM];
#pragma unroll
            for (int m = 0; m < NM; ++m) c[m] = v16i{} + m;
            for (int it = 0; it < iters; ++it) {
#pragma unroll
                for (int m = 0; m < NM; ++m) c[m] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c[m], 0, 0, 0);
            }
            int s = 0;
#pragma unroll
            for (int m = 0; m < NM; ++m)
#pragma unroll
                for (int r = 0; r < 16; ++r) s += c[m][r];
            out[blockIdx.x * blockDim.x + threadIdx.x] = s;
        } else {
            v4i c[NM];
#pragma unroll
            for (int m = 0; m < NM; ++m) c[m] = v4i{m, 0, 0, 0};
            for (int it = 0; it < iters; ++it) {
#pragma unroll
                for (int m = 0; m < NM; ++m) c[m] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c[m], 0, 0, 0);
            }
            int s = 0;
#pragma unroll
            for (int m = 0; m < NM; ++m) s += c[m][0] + c[m][1] + c[m][2] + c[m][3];
            out[blockIdx.x * blockDim.x + threadIdx.x] = s;
        }
    } else if (MIX == 1) {
        double d[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) d[i] = 1.0 + 1e-3 * (l + i);
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int v = 0; v < NV; ++v) d[v & 7] = __builtin_fma(d[v & 7], 0.999, 1e-7);
        }
        double ds = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) ds += d[i];
        dout[blockIdx.x * blockDim.x + threadIdx.x] = ds;
    } else {
        unsigned u[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) u[i] = seed * 7 + l + i;
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int v = 0; v < NV; ++v) u[v & 7] = (u[v & 7] << 3) + u[(v + 1) & 7];
        }
        unsigned s = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) s += u[i];
        out[blockIdx.x * blockDim.x + threadIdx.x] = (int)s;
    }
}

template <int NM, bool BIG, int MIX, int NV>
void run(const char *what, int cus, int w, int *d_out, double *d_dout, int iters) {
    const int threads = 256 * w + (MIX ? 256 : 0);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((k_rate<NM, BIG, MIX, NV>), dim3(cus), dim3(threads), 0, 0, d_out, d_dout, iters / 8, 3);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_rate<NM, BIG, MIX, NV>), dim3(cus), dim3(threads), 0, 0, d_out, d_dout, iters, 5);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double ops = 2.0 * 16 * 16 * 64 * (BIG ? 2 : 1) * NM * (double)iters * 4 * w * cus;
    const double mfma_per_simd = (double)NM * iters * w;
    std::printf("%-34s W=%d NM=%2d: %8.3f ms  %7.1f TOPS  %5.1f ns per MFMA per SIMD (16x16x64 units)\n", what, w,
                NM, ms, ops / (ms * 1e-3) / 1e12, ms * 1e6 / (mfma_per_simd * (BIG ? 2 : 1)));
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    int clk = 0;
    CK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0));
    std::printf("CUs %d, clock %d kHz; peak 16x16x64 i8 at 16 cycles: %.2f ns\n", cus, clk, 16.0 / (clk * 1e-6));
    int *d_out;
    double *d_dout;
    CK(hipMalloc(&d_out, sizeof(int) * cus * 1280));
    CK(hipMalloc(&d_dout, sizeof(double) * cus * 1280));
    const int it = 20000;
    run<4, false, 0, 0>("16x16x64", cus, 1, d_out, d_dout, it);
    run<8, false, 0, 0>("16x16x64", cus, 1, d_out, d_dout, it);
    run<16, false, 0, 0>("16x16x64", cus, 1, d_out, d_dout, it);
    run<4, false, 0, 0>("16x16x64", cus, 2, d_out, d_dout, it);
    run<8, false, 0, 0>("16x16x64", cus, 2, d_out, d_dout, it);
    run<4, false, 0, 0>("16x16x64", cus, 3, d_out, d_dout, it);
    run<8, false, 0, 0>("16x16x64", cus, 3, d_out, d_dout, it);
    run<4, false, 0, 0>("16x16x64", cus, 4, d_out, d_dout, it);
    run<2, true, 0, 0>("32x32x32", cus, 1, d_out, d_dout, it / 2);
    run<4, true, 0, 0>("32x32x32", cus, 1, d_out, d_dout, it / 2);
    run<4, true, 0, 0>("32x32x32", cus, 2, d_out, d_dout, it / 2);
    run<4, true, 0, 0>("32x32x32", cus, 3, d_out, d_dout, it / 2);
    run<8, false, 1, 16>("16x16x64 + f64 wave (16 fma/it)", cus, 2, d_out, d_dout, it);
    run<8, false, 1, 64>("16x16x64 + f64 wave (64 fma/it)", cus, 2, d_out, d_dout, it);
    run<8, false, 2, 16>("16x16x64 + i32 wave (16 op/it)", cus, 2, d_out, d_dout, it);
    run<8, false, 2, 64>("16x16x64 + i32 wave (64 op/it)", cus, 2, d_out, d_dout, it);
    return 0;
}
