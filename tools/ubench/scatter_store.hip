// Micro-benchmark: can the STFT write its freq-major spectrogram straight from registers?
// Output = 1440 files x 513 rows x ld floats (ld = 5632), as stft1024_kernel writes it.
// A "tile" = 32 consecutive frames (columns) of all 513 rows.  Persistent workgroups walk
// contiguous tile ranges.  Modes:
//   0: LDS-tile pattern: 128-B row segments, 8 lanes x 16 B per row (stft1024_kernel today)
//   1: registers, 4 frames per wave: lane l writes rows l + 64 r (r = 0..8) as one 16-B
//      float4 (4 consecutive frames); 8 waves cover a 32-frame tile
//   2: registers, 2 frames per wave: float2 per row, 16 waves per tile
//   3: mode 1 with nontemporal stores
//   4: registers, 8 frames per wave (two float4 per row), 4 waves per tile
//   5: LDS-tile pattern with 16-frame tiles: 64-B row segments, 4 lanes x 16 B per row
//   6: LDS-tile pattern with 64-frame tiles: 256-B row segments, 16 lanes x 16 B per row
// Prints GB/s for each mode; the byte count is the spectrogram (16.6 GB).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int K = 513;
typedef float f4v __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(1024) void wr(float *out, int64_t ld, int64_t tiles_per_file, int64_t ntiles,
                                           int64_t per, int mode) {
    const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    for (int64_t it = 0; it < per; ++it) {
        const int64_t tl = blockIdx.x * per + it;
        if (tl >= ntiles) break;
        const int64_t f = tl / tiles_per_file, ti = tl % tiles_per_file;
        float *of = out + f * (int64_t)K * ld + ti * 32;
        if (mode == 0) {
            const int q = tid & 7;
            for (int k0 = 0; k0 < K; k0 += 128) {
                const int k = k0 + (tid >> 3);
                if (k < K) *reinterpret_cast<float4 *>(of + (int64_t)k * ld + 4 * q) = make_float4(k, tl, 1.f, 2.f);
            }
        } else if (mode == 1 || mode == 3) {
            if (w >= 8) continue;
            for (int r = 0; r < 9; ++r) {
                const int k = l + 64 * r;
                if (k < K) {
                    f4v v = {(float)k, (float)tl, 1.f, 2.f};
                    f4v *p = reinterpret_cast<f4v *>(of + (int64_t)k * ld + 4 * w);
                    if (mode == 3) __builtin_nontemporal_store(v, p);
                    else *p = v;
                }
            }
        } else if (mode == 2) {
            for (int r = 0; r < 9; ++r) {
                const int k = l + 64 * r;
                if (k < K) *reinterpret_cast<float2 *>(of + (int64_t)k * ld + 2 * w) = make_float2(k, tl);
            }
        } else if (mode == 5) {  // tile tl covers 16 frames: two per 32-frame "tile" index
            for (int h = 0; h < 2; ++h) {
                const int q = tid & 3;
                for (int k0 = 0; k0 < K; k0 += 256) {
                    const int k = k0 + (tid >> 2);
                    if (k < K)
                        *reinterpret_cast<float4 *>(of + (int64_t)k * ld + 16 * h + 4 * q) = make_float4(k, tl, 1.f, 2.f);
                }
            }
        } else if (mode == 6) {  // pairs of 32-frame tiles as one 64-frame tile
            if (it & 1) continue;
            const int q = tid & 15;
            for (int k0 = 0; k0 < K; k0 += 64) {
                const int k = k0 + (tid >> 4);
                if (k < K && ti + 1 < tiles_per_file)
                    *reinterpret_cast<float4 *>(of + (int64_t)k * ld + 4 * q) = make_float4(k, tl, 1.f, 2.f);
            }
        } else if (mode == 4) {
            if (w >= 4) continue;
            for (int r = 0; r < 9; ++r) {
                const int k = l + 64 * r;
                if (k < K) {
                    float4 *p = reinterpret_cast<float4 *>(of + (int64_t)k * ld + 8 * w);
                    p[0] = make_float4(k, tl, 1.f, 2.f);
                    p[1] = make_float4(k, tl, 3.f, 4.f);
                }
            }
        }
    }
}

int main() {
    const int64_t F = 1440, ld = 5632, tpf = ld / 32, ntiles = F * tpf;
    const size_t bytes = (size_t)F * K * ld * 4;
    float *out;
    if (hipMalloc(&out, bytes) != hipSuccess) return 1;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    for (int mode : {0, 5, 6}) {
        for (int wpc = 1; wpc <= 2; ++wpc) {
            const int64_t wgs = (int64_t)cus * wpc;
            const int64_t per = (ntiles + wgs - 1) / wgs;
            float best = 1e30f;
            for (int rep = 0; rep < 6; ++rep) {
                hipEventRecord(a);
                hipLaunchKernelGGL(wr, dim3((unsigned)wgs), dim3(1024), 0, 0, out, ld, tpf, ntiles, per, mode);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms;
                hipEventElapsedTime(&ms, a, b);
                if (rep > 0 && ms < best) best = ms;
            }
            printf("mode %d  wg/CU %d  %.3f ms  %.0f GB/s\n", mode, wpc, best, bytes / (best * 1e-3) / 1e9);
        }
    }
    hipFree(out);
    return 0;
}
