// Micro-benchmark for the exact band-delta kernel's matrix step: int8 MFMA on gfx950.
//
//  (a) fragment map of v_mfma_i32_16x16x64_i8: random int8 A [16][64], B [64][16] loaded with the
//      hypothesis  lane l: A[l & 15][16 (l >> 4) + j], B[16 (l >> 4) + j][l & 15] (j = 0..15, byte j
//      of the lane's 4 VGPRs), C/D col = l & 15, row = 4 (l >> 4) + r; compared with the host GEMM.
//      (Any k order works for a GEMM as long as byte j of lane l is the same k in A and in B.)
//  (b) issue rate: NM independent MFMAs per iteration (one wave per SIMD, 4 waves per CU, every CU),
//      cycles per MFMA from s_memtime;
//  (c) co-issue: the same MFMAs with NV independent v_fma_f64 per iteration beside them (as the
//      delta kernel's float64 post-processing would run) -- time vs max(MFMA alone, VALU alone).
// Build: hipcc --offload-arch=gfx950 -O3 mfma_i8.hip -o mfma_i8
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(3);                                                                  \
        }                                                                                  \
    } while (0)

__global__ void k_map(const signed char *A, const signed char *B, int *C) {
    const int l = threadIdx.x;
    signed char a[16], b[16];
    for (int j = 0; j < 16; ++j) {
        a[j] = A[(l & 15) * 64 + 16 * (l >> 4) + j];
        b[j] = B[(16 * (l >> 4) + j) * 16 + (l & 15)];
    }
    v4i av, bv;
    __builtin_memcpy(&av, a, 16);
    __builtin_memcpy(&bv, b, 16);
    v4i c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) C[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

template <int NM, int NV>
__global__ __launch_bounds__(256) void k_rate(long long *cyc, int *out, double *dout, int iters, int seed) {
    const int l = threadIdx.x & 63;
    v4i a = {seed + l, seed * 3 + l, l ^ seed, 7 * l}, b = {l, seed - l, 5 * l, seed};
    v4i c[NM > 0 ? NM : 1];
#pragma unroll
    for (int m = 0; m < (NM > 0 ? NM : 1); ++m) c[m] = v4i{m, 0, 0, 0};
    double d[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = 1.0 + 1e-3 * (l + i);
    const double fa = 0.999, fb = 1e-7;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int m = 0; m < NM; ++m) {
            c[m] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c[m], 0, 0, 0);
#pragma unroll
            for (int v = 0; v < NV / (NM > 0 ? NM : 1); ++v) d[v & 7] = __builtin_fma(d[v & 7], fa, fb);
        }
        if (NM == 0) {
#pragma unroll
            for (int v = 0; v < NV; ++v) d[v & 7] = __builtin_fma(d[v & 7], fa, fb);
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    int s = 0;
#pragma unroll
    for (int m = 0; m < (NM > 0 ? NM : 1); ++m) s += c[m][0] + c[m][1] + c[m][2] + c[m][3];
    double ds = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) ds += d[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    dout[blockIdx.x * blockDim.x + threadIdx.x] = ds;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NM, int NV>
double run_rate(int cus, long long *d_cyc, int *d_out, double *d_dout, int iters) {
    // 4 waves per workgroup = one per SIMD, one workgroup per CU
    hipLaunchKernelGGL((k_rate<NM, NV>), dim3(cus), dim3(256), 0, 0, d_cyc, d_out, d_dout, iters, 3);
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL((k_rate<NM, NV>), dim3(cus), dim3(256), 0, 0, d_cyc, d_out, d_dout, iters, 5);
    CK(hipDeviceSynchronize());
    std::vector<long long> cyc(cus);
    CK(hipMemcpy(cyc.data(), d_cyc, sizeof(long long) * cus, hipMemcpyDeviceToHost));
    std::sort(cyc.begin(), cyc.end());
    // s_memtime counts at the shader clock's reference (100 MHz x ... ): report per iteration
    return (double)cyc[cus / 2] / iters;
}

int main() {
    std::mt19937 g(1);
    std::vector<signed char> A(16 * 64), B(64 * 16);
    for (auto &x : A) x = (signed char)(int)(g() % 256 - 128);
    for (auto &x : B) x = (signed char)(int)(g() % 256 - 128);
    signed char *dA, *dB;
    int *dC;
    CK(hipMalloc(&dA, A.size()));
    CK(hipMalloc(&dB, B.size()));
    CK(hipMalloc(&dC, 256 * 4));
    CK(hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_map, dim3(1), dim3(64), 0, 0, dA, dB, dC);
    CK(hipDeviceSynchronize());
    std::vector<int> C(256);
    CK(hipMemcpy(C.data(), dC, 256 * 4, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int m = 0; m < 16; ++m)
        for (int n = 0; n < 16; ++n) {
            int s = 0;
            for (int k = 0; k < 64; ++k) s += (int)A[m * 64 + k] * (int)B[k * 16 + n];
            bad += s != C[m * 16 + n];
        }
    std::printf("map: lane l A[l&15][16(l>>4)+j] B[16(l>>4)+j][l&15] C[4(l>>4)+r][l&15]: %s (%d of 256 wrong)\n",
                bad ? "WRONG" : "ok", bad);

    int dev = 0, cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    long long *d_cyc;
    int *d_out;
    double *d_dout;
    CK(hipMalloc(&d_cyc, sizeof(long long) * cus));
    CK(hipMalloc(&d_out, sizeof(int) * cus * 256));
    CK(hipMalloc(&d_dout, sizeof(double) * cus * 256));
    const int it = 4096;
    const double m8 = run_rate<8, 0>(cus, d_cyc, d_out, d_dout, it);
    const double m16 = run_rate<16, 0>(cus, d_cyc, d_out, d_dout, it);
    std::printf("s_memtime ticks per iteration: 8 MFMA %.1f (%.2f per MFMA), 16 MFMA %.1f (%.2f per MFMA)\n", m8,
                m8 / 8, m16, m16 / 16);
    const double v32 = run_rate<0, 32>(cus, d_cyc, d_out, d_dout, it);
    const double v64 = run_rate<0, 64>(cus, d_cyc, d_out, d_dout, it);
    std::printf("v_fma_f64 alone: 32 %.1f, 64 %.1f ticks per iteration\n", v32, v64);
    const double c32 = run_rate<16, 32>(cus, d_cyc, d_out, d_dout, it);
    const double c64 = run_rate<16, 64>(cus, d_cyc, d_out, d_dout, it);
    std::printf("16 MFMA + 32 fma_f64: %.1f (alone %.1f + %.1f); 16 MFMA + 64 fma_f64: %.1f (alone %.1f + %.1f)\n", c32,
                m16, v32, c64, m16, v64);
    return bad ? 1 : 0;
}
