// Micro-benchmark for VERDICT r2 item 2's two untried stft1024 / cstft4096 levers:
//
//  (a) register transposes.  A lane holds 8 complex values (16 floats), the layout between two
//      radix-8 passes; the exchange of lane bits 3..5 with register bits 0..2 is done
//        lds   : as the kernels do now, 8 ds_write_b64 + 8 ds_read_b64 through a per-wave scratch;
//        p5    : lane bit 5 only, v_permlane32_swap (8 swaps: the cost of one exchanged bit);
//        p54   : lane bits 5 and 4, v_permlane32_swap + v_permlane16_swap (16 swaps);
//        reg   : the full 3-bit exchange, bits 5 and 4 as above and bit 3 by DPP row_ror:8 and
//                v_cndmask (no lane-bit-3 swap instruction exists);
//      each between NV independent FMAs over the same registers (a pass's worth of VALU work),
//      4 waves per SIMD, so a variant's cost is what it adds to a VALU-bound loop.
//  (b) MFMA co-issue.  NM independent v_mfma_f32_16x16x4_f32 (a dense real 16 x 16 = complex
//      8 x 8 DFT over 16 butterflies needs 4 of them per k-block, 16 per 64-butterfly pass)
//      interleaved with NV independent FMAs: if the matrix pipe runs beside the VALU, the time is
//      max(MFMA alone, VALU alone), and a pass moved to MFMA removes its VALU time.
//
// Cycles from s_memtime, per loop iteration per SIMD.  Build:
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize coissue_xpose.hip -o coissue_xpose
// (no SLP: packed v_pk_fma_f32 would issue at a different rate than the scalar FMAs compared)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <algorithm>

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void stamp(long long *cyc, long long t0, long long t1) {
    if (threadIdx.x == 0) {
        const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11));
        cyc[3 * blockIdx.x] = t0;
        cyc[3 * blockIdx.x + 1] = t1;
        cyc[3 * blockIdx.x + 2] = xcc;
    }
}

template <int NV>
__device__ __forceinline__ void valu_block(float (&v)[16], float a, float b) {
#pragma unroll
    for (int j = 0; j < NV; ++j) v[j & 15] = __builtin_fmaf(v[j & 15], a, b);
}

// (a) transposes: MODE 0 none, 1 lds, 2 p5, 3 p54, 4 reg
template <int MODE, int NV>
__global__ __launch_bounds__(1024) void k_xpose(long long *cyc, float *out, int iters, float a, float b) {
    __shared__ float2 scr[16][64 * 8 + 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = a * (lane + i);
    const bool b3 = lane & 8;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        valu_block<NV>(v, a, b);
        if (MODE == 1) {
            float2 *s = scr[wave];
            // write element (lane, r) at 8*lane + r, read (l + 64 r): lane bits 3..5 <-> r; pad
            // one float2 per 8 to spread the banks (what stft1024's phys() does)
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int e = 8 * lane + r;
                s[e + (e >> 3)] = make_float2(v[2 * r], v[2 * r + 1]);
            }
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int e = lane + 64 * r;
                const float2 x = s[e + (e >> 3)];
                v[2 * r] = x.x;
                v[2 * r + 1] = x.y;
            }
            __builtin_amdgcn_wave_barrier();
        } else if (MODE >= 2) {
            // bit 5 <-> register bit 2: pairs (r, r + 4), both floats of the complex value
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    auto x = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[2 * r + c]),
                                                              __float_as_uint(v[2 * r + 8 + c]), false, false);
                    v[2 * r + c] = __uint_as_float(x[0]);
                    v[2 * r + 8 + c] = __uint_as_float(x[1]);
                }
            if (MODE >= 3) {  // bit 4 <-> register bit 1: pairs (r, r + 2)
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    if (r & 2) continue;
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        auto x = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[2 * r + c]),
                                                                  __float_as_uint(v[2 * r + 4 + c]), false, false);
                        v[2 * r + c] = __uint_as_float(x[0]);
                        v[2 * r + 4 + c] = __uint_as_float(x[1]);
                    }
                }
            }
            if (MODE >= 4) {  // bit 3 <-> register bit 0: pairs (r, r + 1), DPP row_ror:8 = lane ^ 8
#pragma unroll
                for (int r = 0; r < 8; r += 2)
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        const float lo = v[2 * r + c], hi = v[2 * r + 2 + c];
                        const float t = b3 ? lo : hi;
                        const float u = __uint_as_float(
                            __builtin_amdgcn_update_dpp(0u, __float_as_uint(t), 0x128, 0xf, 0xf, false));
                        v[2 * r + c] = b3 ? u : lo;
                        v[2 * r + 2 + c] = b3 ? hi : u;
                    }
            }
        }
    }
    __syncthreads();
    const long long t1 = __builtin_amdgcn_s_memtime();
    stamp(cyc, t0, t1);
    float r = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) r += v[i];
    if (r == 1234.5f) out[threadIdx.x] = r;
}

// (b) NM MFMA + NV FMAs per iteration; IL: pin the interleave (1 MFMA, NV/NM FMAs, ...) in the
// instruction stream with sched_group_barrier (otherwise hipcc groups the MFMAs after the FMAs)
template <int NM, int NV, bool IL = false>
__global__ __launch_bounds__(1024) void k_coissue(long long *cyc, float *out, int iters, float a, float b) {
    const int lane = threadIdx.x & 63;
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = a * (lane + i);
    f4 acc[4] = {};
    const float ma = a * lane, mb = b * lane;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if (NM == 0) {
            valu_block<NV>(v, a, b);
        } else {
#pragma unroll
            for (int m = 0; m < NM; ++m) {
                acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(ma, mb, acc[m & 3], 0, 0, 0);
                valu_block<NV / (NM > 0 ? NM : 1)>(v, a, b);
                if (IL) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, NV / (NM > 0 ? NM : 1), 0);
                }
            }
        }
    }
    __syncthreads();
    const long long t1 = __builtin_amdgcn_s_memtime();
    stamp(cyc, t0, t1);
    float r = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) r += v[i];
#pragma unroll
    for (int q = 0; q < 4; ++q) r += acc[q][0] + acc[q][1] + acc[q][2] + acc[q][3];
    if (r == 1234.5f) out[threadIdx.x] = r;
}

// control for (b): the same loop with a bf16 MFMA (v_mfma_f32_16x16x32_bf16), which the guide
// documents as running beside VALU fillers -- shows the method sees co-issue where it exists
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
template <int NM, int NV>
__global__ __launch_bounds__(1024) void k_coissue_bf16(long long *cyc, float *out, int iters, float a, float b) {
    const int lane = threadIdx.x & 63;
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = a * (lane + i);
    f4 acc[4] = {};
    bf8 ma, mb;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        ma[i] = (__bf16)(a * (lane + i));
        mb[i] = (__bf16)(b * (lane - i));
    }
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int m = 0; m < NM; ++m) {
            acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ma, mb, acc[m & 3], 0, 0, 0);
            valu_block<NV / (NM > 0 ? NM : 1)>(v, a, b);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, NV / (NM > 0 ? NM : 1), 0);
        }
    }
    __syncthreads();
    const long long t1 = __builtin_amdgcn_s_memtime();
    stamp(cyc, t0, t1);
    float r = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) r += v[i];
#pragma unroll
    for (int q = 0; q < 4; ++q) r += acc[q][0] + acc[q][1] + acc[q][2] + acc[q][3];
    if (r == 1234.5f) out[threadIdx.x] = r;
}

static double run(void (*kern)(long long *, float *, int, float, float), long long *cyc, float *out, int cus,
                  int iters) {
    // per workgroup t1 - t0 (all workgroups run at once, one per CU), averaged; best of 3
    static long long h[3 * 4096];
    double best = 1e30;
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(kern, dim3(cus), dim3(1024), 0, 0, cyc, out, iters, 1.0001f, 0.5f);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(h, cyc, sizeof(long long) * 3 * cus, hipMemcpyDeviceToHost);
        double m = 0;
        for (int i = 0; i < cus; ++i) m += (double)(h[3 * i + 1] - h[3 * i]);
        best = std::min(best, m / cus);
    }
    return best / iters / 4.0;  // per iteration per wave (4 waves per SIMD share it)
}

int main() {
    long long *cyc;
    float *out;
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    (void)hipMalloc(&cyc, sizeof(long long) * cus * 3);
    (void)hipMalloc(&out, sizeof(float) * 1024);
    const int it = 2000;
    printf("# cycles per loop iteration per wave (4 waves/SIMD, 1 WG of 16 waves per CU)\n");
    printf("(a) transposes of 8 complex values per lane (lane bits 3..5 <-> register bits), between NV FMAs\n");
#define XP(NV)                                                                                              \
    {                                                                                                       \
        const double n0 = run(k_xpose<0, NV>, cyc, out, cus, it), l = run(k_xpose<1, NV>, cyc, out, cus, it); \
        const double p5 = run(k_xpose<2, NV>, cyc, out, cus, it), p54 = run(k_xpose<3, NV>, cyc, out, cus, it); \
        const double rg = run(k_xpose<4, NV>, cyc, out, cus, it);                                          \
        printf("NV=%4d  none %7.1f  lds %7.1f (+%5.1f)  p5 %7.1f (+%5.1f)  p54 %7.1f (+%5.1f)  reg %7.1f (+%5.1f)\n", \
               NV, n0, l, l - n0, p5, p5 - n0, p54, p54 - n0, rg, rg - n0);                                 \
    }
    XP(0) XP(64) XP(128) XP(256)
    printf("(b) NM v_mfma_f32_16x16x4_f32 + NV FMAs per iteration\n");
#define CO(NM, NV)                                                                                          \
    {                                                                                                       \
        const double m = run(k_coissue<NM, 0>, cyc, out, cus, it), v = run(k_coissue<0, NV>, cyc, out, cus, it); \
        const double mv = run(k_coissue<NM, NV>, cyc, out, cus, it);                                       \
        const double il = run(k_coissue<NM, NV, true>, cyc, out, cus, it);                                 \
        printf("NM=%3d NV=%4d  mfma alone %7.1f  valu alone %7.1f  both %7.1f  interleaved %7.1f  (max %7.1f, sum %7.1f)\n", \
               NM, NV, m, v, mv, il, std::max(m, v), m + v);                                                \
    }
    CO(16, 64) CO(16, 128) CO(16, 256) CO(32, 256) CO(32, 512) CO(64, 512)
    printf("(b') control: NM v_mfma_f32_16x16x32_bf16 + NV FMAs, interleaved\n");
#define CB(NM, NV)                                                                                          \
    {                                                                                                       \
        const double m = run(k_coissue_bf16<NM, 0>, cyc, out, cus, it), v = run(k_coissue<0, NV>, cyc, out, cus, it); \
        const double mv = run(k_coissue_bf16<NM, NV>, cyc, out, cus, it);                                  \
        printf("NM=%3d NV=%4d  mfma alone %7.1f  valu alone %7.1f  interleaved %7.1f  (max %7.1f, sum %7.1f)\n", NM, NV, \
               m, v, mv, std::max(m, v), m + v);                                                            \
    }
    CB(16, 64) CB(16, 128) CB(16, 256) CB(32, 512)
    (void)hipFree(cyc);
    (void)hipFree(out);
    return 0;
}
