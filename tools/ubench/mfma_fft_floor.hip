// Micro-benchmark: the issue floor of an MFMA-based 1024-point real STFT frame.
// Per frame: NM v_mfma_f32_32x32x16_f16 (36 = a 32 x 32 two-pass DFT with fp16 hi/lo operand
// splitting, three products per f32 product) plus NV independent VALU ops (the split
// conversions, twiddles, window and |X|^2 left on the VALU), W waves per SIMD.  Prints ms for
// the C3 frame count (8.1 M frames) next to the current stft1024_kernel (6.5 ms).
// Build: hipcc --offload-arch=gfx950 -O3 mfma_fft_floor.hip -o mfma_fft_floor
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

template <int NM, int NV>
__global__ __launch_bounds__(256) void k(float *out, long frames_per_wave, float s) {
    const int lane = threadIdx.x & 63;
    h8 a, b;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        a[i] = (_Float16)(s * (lane + i));
        b[i] = (_Float16)(s * (lane - i));
    }
    f16v acc[4] = {};
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = s + lane + i;
    for (long f = 0; f < frames_per_wave; ++f) {
#pragma unroll
        for (int m = 0; m < NM; ++m) {
            acc[m & 3] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[m & 3], 0, 0, 0);
#pragma unroll
            for (int j = 0; j < NV / NM; ++j) v[j & 7] = v[j & 7] * 1.0001f + 0.5f;
        }
    }
    float r = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) r += v[i];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < 16; ++i) r += acc[q][i];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int NM, int NV>
void run(int wps, const char *name) {
    const long frames = 8100000;
    int dev_cu = 256;
    const int blocks = dev_cu * wps;  // 4 waves per block = one per SIMD
    const long waves = (long)blocks * 4;
    const long fpw = (frames + waves - 1) / waves;
    float *out;
    (void)hipMalloc(&out, sizeof(float) * blocks * 256);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((k<NM, NV>), dim3(blocks), dim3(256), 0, 0, out, fpw, 1e-3f);
    (void)hipEventRecord(e0);
    for (int it = 0; it < 5; ++it) hipLaunchKernelGGL((k<NM, NV>), dim3(blocks), dim3(256), 0, 0, out, fpw, 1e-3f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%-28s waves/SIMD %d: %.3f ms per 8.1 M frames\n", name, wps, ms / 5);
    (void)hipFree(out);
}

int main() {
    for (int w = 1; w <= 4; w *= 2) {
        run<36, 0>(w, "36 MFMA, no VALU");
        run<36, 252>(w, "36 MFMA + 252 VALU");
        run<36, 396>(w, "36 MFMA + 396 VALU");
        run<24, 252>(w, "24 MFMA + 252 VALU");
    }
    return 0;
}
