// STFT power spectrogram on gfx950 — scipy.signal.spectrogram(mode='psd',
// scaling='density', window='hann', detrend='constant', one-sided) semantics, as
// called by the reference at dsp/src/main.py:52-54 and :132-133.
//
// Layout and mapping:
//   * one workgroup = NW waves = one tile of TT consecutive frames of one file;
//   * one wave = one frame at a time: the N real samples are loaded coalesced
//     (16 B per lane), detrended (frame mean via a wave reduction), windowed and
//     packed as M = N/2 complex points z[m] = x[2m] + i*x[2m+1] into the wave's LDS
//     scratch; a radix-8 Stockham FFT of size M runs in that scratch; the real
//     spectrum is recovered with the usual half-length post-twiddle;
//   * |X|^2 * scale (x2 on bins 1..M-1) goes to an LDS tile [K][TT] (freq-major);
//   * the tile is written out as TT-float (128 B) contiguous row segments with
//     16-B stores: out[file][k][t] with a padded row pitch ld (multiple of 32).
// HBM traffic per frame: hop*sizeof(sample) read (frames overlap; the overlap is
// served by L2) + K*4 B written.  No MFMA: the op is bandwidth/VALU bound.
#include "msd_internal.h"

namespace msd {
namespace {

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 mul_mi(float2 a) { return make_float2(a.y, -a.x); }  // a * (-i)

template <int R>
struct Dft;
template <>
struct Dft<2> {
    __device__ __forceinline__ static void run(float2 *v) {
        float2 a = v[0], b = v[1];
        v[0] = cadd(a, b);
        v[1] = csub(a, b);
    }
};
template <>
struct Dft<4> {
    __device__ __forceinline__ static void run(float2 *v) {
        float2 t0 = cadd(v[0], v[2]), t1 = csub(v[0], v[2]);
        float2 t2 = cadd(v[1], v[3]), t3 = mul_mi(csub(v[1], v[3]));
        v[0] = cadd(t0, t2);
        v[1] = cadd(t1, t3);
        v[2] = csub(t0, t2);
        v[3] = csub(t1, t3);
    }
};
template <>
struct Dft<8> {
    __device__ __forceinline__ static void run(float2 *v) {
        const float s = 0.70710678118654752440f;
        float2 a[4], b[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            a[r] = cadd(v[r], v[r + 4]);
            b[r] = csub(v[r], v[r + 4]);
        }
        b[1] = make_float2((b[1].x + b[1].y) * s, (b[1].y - b[1].x) * s);   // * W8^1
        b[2] = mul_mi(b[2]);                                                 // * W8^2
        b[3] = make_float2((b[3].y - b[3].x) * s, -(b[3].x + b[3].y) * s);  // * W8^3
        Dft<4>::run(a);
        Dft<4>::run(b);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            v[2 * r] = a[r];
            v[2 * r + 1] = b[r];
        }
    }
};

constexpr int ilog2(int v) { return v <= 1 ? 0 : 1 + ilog2(v / 2); }

// padded LDS index: 2 float2 of padding per 8 (keeps 16-B alignment of even
// indices and makes the staging ds_write_b128 and pass accesses conflict-light)
__device__ __forceinline__ constexpr int phys(int n) { return n + ((n >> 3) << 1); }

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One Stockham autosort pass of radix R over M points held in the wave's scratch
// S (in place: every lane loads all its butterflies before any lane stores).
template <int M, int R, int Ns>
__device__ __forceinline__ void stockham_pass(float2 *S, const float2 *tw, int lane) {
    constexpr int NBF = M / R;
    constexpr int PER = (NBF + 63) / 64;
    float2 v[PER][R];
#pragma unroll
    for (int b = 0; b < PER; ++b) {
        const int bf = lane + 64 * b;
        if (NBF % 64 == 0 || bf < NBF) {
#pragma unroll
            for (int r = 0; r < R; ++r) v[b][r] = S[phys(bf + r * NBF)];
        }
    }
    wave_sync();
#pragma unroll
    for (int b = 0; b < PER; ++b) {
        const int bf = lane + 64 * b;
        if (NBF % 64 == 0 || bf < NBF) {
            const int k = bf & (Ns - 1);
            if (Ns > 1) {
#pragma unroll
                for (int r = 1; r < R; ++r) v[b][r] = cmul(v[b][r], tw[k * r * (M / (Ns * R))]);
            }
            Dft<R>::run(v[b]);
            const int o = (bf - k) * R + k;
#pragma unroll
            for (int r = 0; r < R; ++r) S[phys(o + r * Ns)] = v[b][r];
        }
    }
    wave_sync();
}

template <int M, int PASS, int Ns>
__device__ __forceinline__ void fft_passes(float2 *S, const float2 *tw, int lane) {
    if constexpr (Ns < M) {
        constexpr int LOG = ilog2(M);
        constexpr int N8 = LOG / 3;
        constexpr int R = PASS < N8 ? 8 : (1 << (LOG % 3));
        stockham_pass<M, R, Ns>(S, tw, lane);
        fft_passes<M, PASS + 1, Ns * R>(S, tw, lane);
    }
}

template <typename T>
__device__ __forceinline__ float to_f(T v) {
    return static_cast<float>(v);
}

// load SPL consecutive samples starting at p into s[] as float
template <typename T, int SPL>
__device__ __forceinline__ void load_samples(const T *p, float *s) {
    constexpr int BYTES = SPL * (int)sizeof(T);
    if constexpr (BYTES % 16 == 0) {
        if ((reinterpret_cast<uintptr_t>(p) & 15) == 0) {
            const uint4 *q = reinterpret_cast<const uint4 *>(p);
            constexpr int PER = 16 / (int)sizeof(T);
#pragma unroll
            for (int i = 0; i < BYTES / 16; ++i) {
                uint4 u = q[i];
                const T *e = reinterpret_cast<const T *>(&u);
#pragma unroll
                for (int j = 0; j < PER; ++j) s[i * PER + j] = to_f(e[j]);
            }
            return;
        }
    }
#pragma unroll
    for (int i = 0; i < SPL; ++i) s[i] = to_f(p[i]);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <int M, int NW, int TT>
struct StftGeom {
    static constexpr int N = 2 * M;
    static constexpr int K = M + 1;
    static constexpr int PITCH = TT + 4;             // floats per tile row (16-B aligned rows)
    static constexpr int SCR = M + M / 4;            // float2 per wave scratch (phys range)
    static constexpr int TILE_F = K * PITCH;         // floats
    static constexpr int TW_OFF = TILE_F * 4;        // bytes
    static constexpr int POST_OFF = TW_OFF + M * 8;  // bytes
    static constexpr int WIN_OFF = POST_OFF + (M + 2) * 8;
    static constexpr int SCR_OFF = WIN_OFF + N * 4;
    static constexpr int LDS_BYTES = SCR_OFF + NW * SCR * 8;
    static_assert(TILE_F % 4 == 0, "tile must keep 16-B alignment");
};

template <int M, int NW, int TT, typename T>
__global__ __launch_bounds__(NW * 64) void stft_psd_kernel(const T *__restrict__ x, const int64_t *__restrict__ off,
                                                           const int64_t *__restrict__ len, int64_t tiles_per_file,
                                                           int hop, float scale, int detrend, const float *__restrict__ g_win,
                                                           const float2 *__restrict__ g_tw,
                                                           const float2 *__restrict__ g_post, float *__restrict__ out,
                                                           int64_t ld) {
    using G = StftGeom<M, NW, TT>;
    constexpr int N = G::N, K = G::K, PITCH = G::PITCH;
    constexpr int SPL = N / 64;  // real samples per lane
    constexpr int FPW = TT / NW; // frames per wave
    static_assert(TT % NW == 0, "frames per wave");
    static_assert(SPL % 2 == 0, "complex packing");

    extern __shared__ __attribute__((aligned(16))) char smem[];
    float *tile = reinterpret_cast<float *>(smem);
    float2 *tw = reinterpret_cast<float2 *>(smem + G::TW_OFF);
    float2 *post = reinterpret_cast<float2 *>(smem + G::POST_OFF);
    float *win = reinterpret_cast<float *>(smem + G::WIN_OFF);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    float2 *scr = reinterpret_cast<float2 *>(smem + G::SCR_OFF) + wave * G::SCR;

    const int64_t f = blockIdx.x / tiles_per_file;
    const int64_t t0 = (blockIdx.x % tiles_per_file) * TT;
    const int64_t n = len[f];
    const int64_t nfr = n >= N ? (n - N) / hop + 1 : 0;
    const T *xf = x + off[f];

    for (int i = tid; i < M; i += NW * 64) tw[i] = g_tw[i];
    for (int i = tid; i <= M; i += NW * 64) post[i] = g_post[i];
    for (int i = tid; i < N; i += NW * 64) win[i] = g_win[i];
    __syncthreads();

    for (int fb = 0; fb < FPW; ++fb) {
        const int c = wave * FPW + fb;
        const int64_t t = t0 + c;
        if (t < nfr) {
            float s[SPL];
            load_samples<T, SPL>(xf + t * hop + lane * SPL, s);
            // the per-lane sums accumulate x - xref, xref the frame's first sample: exact for integer
            // samples, and for float ones a DC offset does not enter their float rounding; the wave
            // sum in fp64.  The mean is subtracted as hi + lo (hi its float32 rounding, lo the rest),
            // so that the detrended sample is the float32 rounding of x - mean also where float(mean)
            // is not exact (|mean| >= 2^24 / N for integer input: a residual DC at bins 0, 1 otherwise)
            const float xref = __shfl(s[0], 0, 64);
            float ls = 0.f;
#pragma unroll
            for (int q = 0; q < SPL; ++q) ls += s[q] - xref;
            const double md = detrend ? (double)xref + wave_sum(static_cast<double>(ls)) / static_cast<double>(N)
                                      : 0.0;  // detrend_none: 0
            const float mean = static_cast<float>(md), mlo = static_cast<float>(md - static_cast<double>(mean));
            const float *w = win + lane * SPL;
#pragma unroll
            for (int q = 0; q < SPL / 2; ++q) {
                const int m = lane * (SPL / 2) + q;
                scr[phys(m)] = make_float2(((s[2 * q] - mean) - mlo) * w[2 * q],
                                           ((s[2 * q + 1] - mean) - mlo) * w[2 * q + 1]);
            }
            wave_sync();
            fft_passes<M, 0, 1>(scr, tw, lane);
#pragma unroll
            for (int i = 0; i < (K + 63) / 64; ++i) {
                const int k = lane + 64 * i;
                if (k <= M) {
                    const float2 zk = scr[phys(k & (M - 1))];
                    const float2 zm = scr[phys((M - k) & (M - 1))];
                    const float2 e = make_float2(0.5f * (zk.x + zm.x), 0.5f * (zk.y - zm.y));
                    const float2 o = make_float2(0.5f * (zk.y + zm.y), -0.5f * (zk.x - zm.x));
                    const float2 X = cadd(e, cmul(post[k], o));
                    float p = (X.x * X.x + X.y * X.y) * scale;
                    if (k != 0 && k != M) p *= 2.f;
                    tile[k * PITCH + c] = p;
                }
            }
            wave_sync();
        } else {
            for (int k = lane; k < K; k += 64) tile[k * PITCH + c] = 0.f;
        }
    }
    __syncthreads();

    float *of = out + f * (int64_t)K * ld + t0;
    constexpr int Q = TT / 4;
    for (int idx = tid; idx < K * Q; idx += NW * 64) {
        const int k = idx / Q, q = idx - (idx / Q) * Q;
        const float4 v = *reinterpret_cast<const float4 *>(&tile[k * PITCH + 4 * q]);
        *reinterpret_cast<float4 *>(&of[(int64_t)k * ld + 4 * q]) = v;
    }
}

template <int M, int NW, int TT, typename T>
int launch_t(msd_stft_plan *p, const void *x, const int64_t *off, const int64_t *len, int64_t nfiles, float *out,
             int64_t ld) {
    using G = StftGeom<M, NW, TT>;
    auto kern = stft_psd_kernel<M, NW, TT, T>;
    if (int rc = ensure_dyn_lds(reinterpret_cast<const void *>(kern), G::LDS_BYTES)) return rc;
    const int64_t tiles = ld / TT;
    const int64_t blocks = tiles * nfiles;
    if (blocks > 0x7fffffffLL) return fail(MSD_ERR_UNSUPPORTED, "stft: grid too large");
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(NW * 64), G::LDS_BYTES, p->ctx->stream,
                       static_cast<const T *>(x), off, len, tiles, p->hop, static_cast<float>(p->scale),
                       p->detrend, p->d_window, p->d_tw, p->d_post, out, ld);
    MSD_HIP(hipGetLastError());
    return MSD_OK;
}

template <int M, int NW, int TT>
int launch_m(msd_stft_plan *p, const void *x, int dtype, const int64_t *off, const int64_t *len, int64_t nfiles,
             float *out, int64_t ld) {
    switch (dtype) {
        case MSD_I16: return launch_t<M, NW, TT, int16_t>(p, x, off, len, nfiles, out, ld);
        case MSD_F32: return launch_t<M, NW, TT, float>(p, x, off, len, nfiles, out, ld);
        case MSD_U8: return launch_t<M, NW, TT, uint8_t>(p, x, off, len, nfiles, out, ld);
        default: return fail(MSD_ERR_UNSUPPORTED, "stft: dtype must be u8, i16 or f32 (float32 output)");
    }
}

}  // namespace

int launch_stft(msd_stft_plan *p, const void *x, int dtype, const int64_t *off, const int64_t *len, int64_t nfiles,
                int64_t max_frames, void *out, int64_t ld) {
    (void)max_frames;
    if (nfiles == 0) return MSD_OK;
    KernelTimer timer(p->ctx, K_STFT);
    // the tiled float32 kernels cover nperseg = nfft in {256, ..., 2048} for u8 / i16 / f32;
    // every other shape (and every float64 plan) goes to stft_any.hip
    const bool tiled_dtype = dtype == MSD_U8 || dtype == MSD_I16 || dtype == MSD_F32;
    if (p->precision != MSD_F32 || p->nfft != p->nperseg || !tiled_dtype)
        return launch_stft_any(p, x, dtype, off, len, nfiles, out, ld);
    if (!p->ctx->force_generic) {
        const int fast = launch_stft1024(p, x, dtype, off, len, nfiles, static_cast<float *>(out), ld);
        if (fast < 0) return fast;
        if (fast == 1) return MSD_OK;
    }
    float *o = static_cast<float *>(out);
    switch (p->nperseg) {
        case 256: return launch_m<128, 8, 32>(p, x, dtype, off, len, nfiles, o, ld);
        case 512: return launch_m<256, 8, 32>(p, x, dtype, off, len, nfiles, o, ld);
        case 1024: return launch_m<512, 8, 32>(p, x, dtype, off, len, nfiles, o, ld);
        case 2048: return launch_m<1024, 4, 16>(p, x, dtype, off, len, nfiles, o, ld);
        default: return launch_stft_any(p, x, dtype, off, len, nfiles, out, ld);
    }
}

}  // namespace msd
