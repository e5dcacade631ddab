// Micro-benchmark: HBM write bandwidth for the spectrogram's store pattern.
// 1440 files x 513 rows x ld floats (ld = 5632); a "tile" = 32 (or 64) consecutive
// columns of all 513 rows of one file.  Persistent workgroups (one per CU) walk
// contiguous tile ranges like stft1024_kernel.  Modes:
//   0: freq-major tiles, 128-B row segments (the kernel's pattern), float2 per lane
//   1: same with 256-B segments (64-column tiles)
//   2: contiguous streaming float4 writes of the same byte count
//   3: mode 0 with nontemporal stores
//   4: mode 0 with tiles assigned round-robin so that the 8 XCD-neighbour WGs write
//      adjacent tiles of the same rows (tile = wg + k*grid)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

constexpr int K = 513;
__global__ __launch_bounds__(1024) void wr(float *out, int64_t ld, int64_t tiles_per_file, int64_t ntiles,
                                           int64_t per, int tt, int mode) {
    const int tid = threadIdx.x;
    const int segs = tt / 2;  // float2 per row segment
    const int rows_per_pass = 1024 / segs;
    if (mode == 2) {
        const int64_t total4 = ntiles * (int64_t)K * tt / 4;
        float4 *o4 = reinterpret_cast<float4 *>(out);
        const int64_t b0 = blockIdx.x * per * (int64_t)K * tt / 4, b1 = b0 + per * (int64_t)K * tt / 4;
        for (int64_t i = b0 + tid; i < b1 && i < total4; i += 1024) o4[i] = make_float4(1.f, 2.f, 3.f, (float)i);
        return;
    }
    for (int64_t it = 0; it < per; ++it) {
        const int64_t tl = mode == 4 ? blockIdx.x + it * gridDim.x : blockIdx.x * per + it;
        if (tl >= ntiles) break;
        const int64_t f = tl / tiles_per_file, ti = tl % tiles_per_file;
        float *of = out + f * (int64_t)K * ld + ti * tt;
        const int q = tid % segs;
        for (int k0 = 0; k0 < K; k0 += rows_per_pass) {
            const int k = k0 + tid / segs;
            if (k < K) {
                float2 v = make_float2((float)k, (float)tl);
                float2 *p = reinterpret_cast<float2 *>(of + (int64_t)k * ld + 2 * q);
                if (mode == 3) {
                    typedef float f2v __attribute__((ext_vector_type(2)));
                    f2v vv = {v.x, v.y};
                    __builtin_nontemporal_store(vv, reinterpret_cast<f2v *>(p));
                } else {
                    *p = v;
                }
            }
        }
    }
}

int main() {
    const int64_t nfiles = 1440, ld = 5632;
    const size_t bytes = (size_t)nfiles * K * ld * 4;
    float *out;
    if (hipMalloc(&out, bytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[] = {"128B segments", "256B segments", "contiguous float4", "128B nontemporal", "128B XCD-adjacent"};
    for (int mode = 0; mode < 5; ++mode) {
        const int tt = mode == 1 ? 64 : 32;
        const int64_t tpf = ld / tt, ntiles = tpf * nfiles;
        const int grid = 256;
        const int64_t per = (ntiles + grid - 1) / grid;
        float best = 1e9;
        for (int rep = 0; rep < 4; ++rep) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(wr, dim3(grid), dim3(1024), 0, 0, out, ld, tpf, ntiles, per, tt, mode);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        printf("mode %d %-20s %.3f ms  %.0f GB/s\n", mode, names[mode], best, bytes / (best * 1e-3) / 1e9);
    }
    return 0;
}
