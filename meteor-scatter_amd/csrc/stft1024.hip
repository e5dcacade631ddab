// Fast path of the STFT power spectrogram for nperseg = nfft = 1024 (the headline
// configuration: scipy.signal.spectrogram(x, fs, 'hann', 1024, 512) as called at
// dsp/src/main.py:52-54 / :132-133 and BASELINE configs C1-C4).
//
// One wave = one frame at a time, 64 lanes x 8 complex points, all three radix-8
// Stockham passes in registers:
//   load   lane j holds z[j + 64 r] = x[2(j+64r)] + i x[2(j+64r)+1] (r = 0..7): one
//          4-byte sample pair per lane per instruction, 256 B coalesced per wave;
//   detrend/window in registers (frame mean: exact integer wave reduction);
//   pass 1 (no twiddle) → LDS transpose → pass 2 → LDS transpose → pass 3 → lane j
//          holds Z[j + 64 r] in natural order;
//   post   conjugate partner Z[512-k] from lane (64-j) by ds_bpermute, real-spectrum
//          split, |X|^2 * scale (x2 off DC/Nyquist) → LDS tile [513][32+1];
// one workgroup = 16 waves = 32 frames per tile, 2 frames per wave; the tile is
// written out as 128-B row segments (one dword per lane).  Workgroups are persistent
// and walk a contiguous range of tiles, so the half-frame shared by neighbouring
// tiles is re-read from L2, and each wave prefetches its next frame's samples
// while computing the current one.
#include "msd_internal.h"

namespace msd {
namespace {

constexpr int F_NW = 16;             // waves per workgroup
constexpr int F_TT = 32;             // frames per tile
constexpr int F_FPW = F_TT / F_NW;   // frames per wave per tile (2)
constexpr int F_K = 513;             // one-sided bins
constexpr int F_PITCH = F_TT + 1;    // tile row pitch (floats): conflict-free dword writes
constexpr int F_SCR = 640;           // float2 per wave scratch (padded 512)
constexpr int F_TILE_BYTES = ((F_K * F_PITCH * 4 + 15) / 16) * 16;
constexpr int F_SCR_BYTES = F_NW * F_SCR * 8;
// per-lane tables, laid out [r][lane] so that every read is lane-contiguous:
// window pairs w[2(j+64r)], w[2(j+64r)+1]; pass-2 twiddles W64^{(j&7) r}; pass-3 W512^{j r}
constexpr int F_TAB_OFF = F_TILE_BYTES + F_SCR_BYTES;
constexpr int F_LDS = F_TAB_OFF + (8 + 7 + 7) * 64 * 8;
static_assert(F_LDS <= 160 * 1024, "LDS budget");

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 mul_mi(float2 a) { return make_float2(a.y, -a.x); }

__device__ __forceinline__ void dft4(float2 &a0, float2 &a1, float2 &a2, float2 &a3) {
    const float2 t0 = cadd(a0, a2), t1 = csub(a0, a2), t2 = cadd(a1, a3), t3 = mul_mi(csub(a1, a3));
    a0 = cadd(t0, t2);
    a1 = cadd(t1, t3);
    a2 = csub(t0, t2);
    a3 = csub(t1, t3);
}

// in-place forward DFT of 8 points, natural order in and out
__device__ __forceinline__ void dft8(float2 *v) {
    const float s = 0.70710678118654752440f;
    float2 a0 = cadd(v[0], v[4]), a1 = cadd(v[1], v[5]), a2 = cadd(v[2], v[6]), a3 = cadd(v[3], v[7]);
    float2 b0 = csub(v[0], v[4]), b1 = csub(v[1], v[5]), b2 = csub(v[2], v[6]), b3 = csub(v[3], v[7]);
    b1 = make_float2((b1.x + b1.y) * s, (b1.y - b1.x) * s);
    b2 = mul_mi(b2);
    b3 = make_float2((b3.y - b3.x) * s, -(b3.x + b3.y) * s);
    dft4(a0, a1, a2, a3);
    dft4(b0, b1, b2, b3);
    v[0] = a0; v[2] = a1; v[4] = a2; v[6] = a3;
    v[1] = b0; v[3] = b1; v[5] = b2; v[7] = b3;
}

__device__ __forceinline__ int phys(int n) { return n + ((n >> 3) << 1); }

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// raw sample pair storage per input type, and its conversion
template <typename T>
struct PairIO;
template <>
struct PairIO<int16_t> {
    using raw_t = uint32_t;
    static constexpr bool kInt = true;
    __device__ static raw_t load(const int16_t *p) { return *reinterpret_cast<const uint32_t *>(p); }
    __device__ static float lo(raw_t r) { return (float)(int16_t)(r & 0xffffu); }
    __device__ static float hi(raw_t r) { return (float)(int16_t)(r >> 16); }
    __device__ static int ilo(raw_t r) { return (int)(int16_t)(r & 0xffffu); }
    __device__ static int ihi(raw_t r) { return (int)(int16_t)(r >> 16); }
};
template <>
struct PairIO<uint8_t> {
    using raw_t = uint32_t;
    static constexpr bool kInt = true;
    __device__ static raw_t load(const uint8_t *p) { return *reinterpret_cast<const uint16_t *>(p); }
    __device__ static float lo(raw_t r) { return (float)(r & 0xffu); }
    __device__ static float hi(raw_t r) { return (float)((r >> 8) & 0xffu); }
    __device__ static int ilo(raw_t r) { return (int)(r & 0xffu); }
    __device__ static int ihi(raw_t r) { return (int)((r >> 8) & 0xffu); }
};
template <>
struct PairIO<float> {
    using raw_t = float2;
    static constexpr bool kInt = false;
    __device__ static raw_t load(const float *p) { return *reinterpret_cast<const float2 *>(p); }
    __device__ static float lo(raw_t r) { return r.x; }
    __device__ static float hi(raw_t r) { return r.y; }
    __device__ static int ilo(raw_t) { return 0; }
    __device__ static int ihi(raw_t) { return 0; }
};

template <typename T>
__global__ __launch_bounds__(F_NW * 64, 1) void stft1024_kernel(
    const T *__restrict__ x, const int64_t *__restrict__ off, const int64_t *__restrict__ len,
    int64_t tiles_per_file, int64_t ntiles, int64_t tiles_per_wg, int hop, float scale4,
    const float *__restrict__ g_win, const float2 *__restrict__ g_tw, const float2 *__restrict__ g_post,
    float *__restrict__ out, int64_t ld) {
    using IO = PairIO<T>;
    using raw_t = typename IO::raw_t;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float *tile = reinterpret_cast<float *>(smem);
    const int tid = threadIdx.x;
    const int j = tid & 63;
    const int wave = tid >> 6;
    float2 *scr = reinterpret_cast<float2 *>(smem + F_TILE_BYTES) + wave * F_SCR;

    // per-lane constant tables in LDS ([r][lane]): window pairs, pass-2/3 twiddles
    float2 *t_win = reinterpret_cast<float2 *>(smem + F_TAB_OFF);
    float2 *t_tw2 = t_win + 8 * 64 - 64;  // rows r = 1..7
    float2 *t_tw3 = t_tw2 + 7 * 64;
    for (int i = tid; i < 8 * 64; i += F_NW * 64) {
        const int r = i >> 6, l = i & 63;
        t_win[i] = *reinterpret_cast<const float2 *>(g_win + 2 * (l + 64 * r));
        if (r > 0) {
            t_tw2[i] = g_tw[8 * (l & 7) * r];
            t_tw3[i] = g_tw[l * r];
        }
    }
    __syncthreads();
    const float2 pb = g_post[j];  // exp(-2*pi*i*j/1024)
    const int partner = (64 - j) & 63;

    const int64_t tb = (int64_t)blockIdx.x * tiles_per_wg;
    const int64_t te = tb + tiles_per_wg < ntiles ? tb + tiles_per_wg : ntiles;

    // frame sequence of this wave: (tile, fb) for tile in [tb, te), fb in [0, F_FPW)
    auto frame_src = [&](int64_t tl, int fb, bool &valid) -> const T * {
        const int64_t f = tl / tiles_per_file;
        const int64_t t = (tl - f * tiles_per_file) * F_TT + wave * F_FPW + fb;
        const int64_t n = len[f];
        const int64_t nfr = n >= 1024 ? (n - 1024) / hop + 1 : 0;
        valid = t < nfr;
        return x + off[f] + t * (int64_t)hop;
    };
    raw_t cur[8], nxt[8];
    bool cur_ok = false, nxt_ok = false;
    if (tb < te) {
        const T *p = frame_src(tb, 0, cur_ok);
        if (cur_ok) {
#pragma unroll
            for (int r = 0; r < 8; ++r) cur[r] = IO::load(p + 2 * (j + 64 * r));
        }
    }

    for (int64_t tl = tb; tl < te; ++tl) {
#pragma unroll
        for (int fb = 0; fb < F_FPW; ++fb) {
            // prefetch the next frame of the sequence
            {
                const int64_t ntl = fb + 1 < F_FPW ? tl : tl + 1;
                const int nfb = fb + 1 < F_FPW ? fb + 1 : 0;
                nxt_ok = false;
                if (ntl < te) {
                    const T *p = frame_src(ntl, nfb, nxt_ok);
                    if (nxt_ok) {
#pragma unroll
                        for (int r = 0; r < 8; ++r) nxt[r] = IO::load(p + 2 * (j + 64 * r));
                    }
                }
            }
            float pw[9];
            if (cur_ok) {
                float2 v[8];
                float mean;
                if constexpr (IO::kInt) {
                    int s = 0;
#pragma unroll
                    for (int r = 0; r < 8; ++r) s += IO::ilo(cur[r]) + IO::ihi(cur[r]);
#pragma unroll
                    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
                    mean = (float)((double)s * (1.0 / 1024.0));
                } else {
                    float s = 0.f;
#pragma unroll
                    for (int r = 0; r < 8; ++r) s += IO::lo(cur[r]) + IO::hi(cur[r]);
#pragma unroll
                    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
                    mean = s * (1.0f / 1024.0f);
                }
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    const float2 w = t_win[r * 64 + j];
                    v[r] = make_float2((IO::lo(cur[r]) - mean) * w.x, (IO::hi(cur[r]) - mean) * w.y);
                }
                // pass 1 (Ns = 1): out[8 j + r]
                dft8(v);
#pragma unroll
                for (int r = 0; r < 8; r += 2)
                    *reinterpret_cast<float4 *>(&scr[phys(8 * j + r)]) = make_float4(v[r].x, v[r].y, v[r + 1].x,
                                                                                       v[r + 1].y);
                wave_sync();
#pragma unroll
                for (int r = 0; r < 8; ++r) v[r] = scr[phys(j + 64 * r)];
                wave_sync();
                // pass 2 (Ns = 8): out[64 (j>>3) + (j&7) + 8 r]
#pragma unroll
                for (int r = 1; r < 8; ++r) v[r] = cmul(v[r], t_tw2[r * 64 + j]);
                dft8(v);
                const int o2 = 64 * (j >> 3) + (j & 7);
#pragma unroll
                for (int r = 0; r < 8; ++r) scr[phys(o2 + 8 * r)] = v[r];
                wave_sync();
#pragma unroll
                for (int r = 0; r < 8; ++r) v[r] = scr[phys(j + 64 * r)];
                wave_sync();
                // pass 3 (Ns = 64): lane j holds Z[j + 64 r]
#pragma unroll
                for (int r = 1; r < 8; ++r) v[r] = cmul(v[r], t_tw3[r * 64 + j]);
                dft8(v);
                // X' = 2X = (Z + conj Zm) + W^k (-i)(Z - conj Zm), Zm = Z[(512 - k) mod 512] from lane
                // (64 - j) register 7 - r (lane 0 pairs with itself: register (8 - r) & 7); W^k = pb * W16^r
                float2 wk = pb;
                const float2 w16 = make_float2(0.92387953251128675613f, -0.38268343236508977173f);
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                    const float2 sv = v[7 - r];
                    float2 m = make_float2(__shfl(sv.x, partner, 64), __shfl(sv.y, partner, 64));
                    if (j == 0) m = v[(8 - r) & 7];
                    const float2 z = v[r];
                    const float2 e = make_float2(z.x + m.x, z.y - m.y);
                    const float2 o = make_float2(z.y + m.y, m.x - z.x);  // -i (z - conj m)
                    const float2 X = cadd(e, cmul(wk, o));
                    pw[r] = (X.x * X.x + X.y * X.y) * (2.0f * scale4);
                    if (r == 0 && j == 0) {
                        pw[0] = (X.x * X.x + X.y * X.y) * scale4;
                        const float2 Xn = csub(e, o);  // k = 512: W = -1
                        pw[8] = (Xn.x * Xn.x + Xn.y * Xn.y) * scale4;
                    }
                    wk = cmul(wk, w16);
                }
            } else {
#pragma unroll
                for (int r = 0; r < 9; ++r) pw[r] = 0.f;
            }
            {
                const int c = wave * F_FPW + fb;
#pragma unroll
                for (int r = 0; r < 8; ++r) tile[(j + 64 * r) * F_PITCH + c] = pw[r];
                if (j == 0) tile[512 * F_PITCH + c] = pw[8];
            }
            cur_ok = nxt_ok;
#pragma unroll
            for (int r = 0; r < 8; ++r) cur[r] = nxt[r];
        }
        __syncthreads();
        // write the tile: rows k = 0..512, 32 floats (128 B) each; one dword per lane,
        // conflict-free LDS reads at pitch 33, two full row segments per wave store
        {
            const int64_t f = tl / tiles_per_file;
            const int64_t t0 = (tl - f * tiles_per_file) * F_TT;
            float *of = out + f * (int64_t)F_K * ld + t0;
            const int q = tid & 31;
#pragma unroll
            for (int k0 = 0; k0 < F_K; k0 += F_NW * 64 / 32) {
                const int k = k0 + (tid >> 5);
                if (k < F_K) of[(int64_t)k * ld + q] = tile[k * F_PITCH + q];
            }
        }
        __syncthreads();
    }
}

template <typename T>
int launch_fast_t(msd_stft_plan *p, const void *x, const int64_t *off, const int64_t *len, int64_t nfiles, float *out,
                  int64_t ld) {
    auto kern = stft1024_kernel<T>;
    static bool attr_set = false;
    if (!attr_set) {
        MSD_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, F_LDS));
        attr_set = true;
    }
    int dev = p->ctx->device, cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int64_t tiles_per_file = ld / F_TT;
    const int64_t ntiles = tiles_per_file * nfiles;
    int64_t wgs = cus;  // one 16-wave workgroup per CU (LDS-bound residency)
    if (wgs > ntiles) wgs = ntiles;
    const int64_t per = (ntiles + wgs - 1) / wgs;
    wgs = (ntiles + per - 1) / per;
    hipLaunchKernelGGL(kern, dim3((unsigned)wgs), dim3(F_NW * 64), F_LDS, p->ctx->stream, static_cast<const T *>(x),
                       off, len, tiles_per_file, ntiles, per, p->hop, static_cast<float>(p->scale * 0.25),
                       p->d_window, p->d_tw, p->d_post, out, ld);
    MSD_HIP(hipGetLastError());
    return MSD_OK;
}

}  // namespace

// returns 1 if the fast path handled the launch, 0 if not applicable, <0 on error
int launch_stft1024(msd_stft_plan *p, const void *x, int dtype, const int64_t *off, const int64_t *len,
                    int64_t nfiles, float *out, int64_t ld) {
    if (p->nperseg != 1024 || (p->hop & 1)) return 0;
    int rc;
    switch (dtype) {
        case MSD_I16: rc = launch_fast_t<int16_t>(p, x, off, len, nfiles, out, ld); break;
        case MSD_F32: rc = launch_fast_t<float>(p, x, off, len, nfiles, out, ld); break;
        case MSD_U8: rc = launch_fast_t<uint8_t>(p, x, off, len, nfiles, out, ld); break;
        default: return 0;
    }
    return rc == MSD_OK ? 1 : rc;
}

}  // namespace msd
