// STFT power spectrogram for the shapes the tiled kernels do not cover: any segment length
// nperseg <= nfft, zero-padded to a power-of-two nfft up to 16384, any hop, in float32 or in
// float64 arithmetic.  Used by
//   * scipy.signal.spectrogram(x, fs, 'hann', nperseg, noverlap, nfft) with nperseg 4096 /
//     8192 (the whole-file debug spectrogram, dsp/src/main.py:127-133 with n_fft = 1024*4,
//     :278-300), nfft > nperseg (zero padding) and inputs shorter than nperseg (scipy shrinks
//     nperseg to the input length, _spectral_py.py _triage_segments);
//   * matplotlib.mlab.specgram in float64 (the legacy noise floor, prime_detection.py:65-91,
//     mlab.py:299-356: symmetric Hann, no detrend, pad_to = NFFT).
//
// Mapping: one 256-thread workgroup per (file, frame column).  The frame's nperseg samples are
// read coalesced, detrended (constant: mean in float64 from exact per-thread sums), windowed
// and packed as M = nfft/2 complex points z[m] = x[2m] + i x[2m+1] (zeros past nperseg) into
// LDS; radix-4 Stockham passes (one radix-2 pass when log2 M is odd) run between two LDS
// buffers; the real spectrum is split out with the half-length post-twiddle and |X|^2 * scale
// (x2 on bins 1..M-1) is stored to out[f][k][t].  These are debug / legacy sizes, not the
// bandwidth-bound headline path: the column stores are 4- or 8-B per row and rely on L2 to
// merge the neighbouring columns that concurrent workgroups write.
#include <type_traits>

#include "msd_internal.h"

namespace msd {
namespace {

constexpr int SA_THREADS = 256;

template <typename R>
struct Cx;
template <>
struct Cx<float> {
    using t = float2;
    __device__ static t make(float a, float b) { return make_float2(a, b); }
};
template <>
struct Cx<double> {
    using t = double2;
    __device__ static t make(double a, double b) { return make_double2(a, b); }
};

template <typename C>
__device__ __forceinline__ C cadd(C a, C b) {
    C r;
    r.x = a.x + b.x;
    r.y = a.y + b.y;
    return r;
}
template <typename C>
__device__ __forceinline__ C csub(C a, C b) {
    C r;
    r.x = a.x - b.x;
    r.y = a.y - b.y;
    return r;
}
template <typename C>
__device__ __forceinline__ C cmul(C a, C b) {
    C r;
    r.x = a.x * b.x - a.y * b.y;
    r.y = a.x * b.y + a.y * b.x;
    return r;
}
template <typename C>
__device__ __forceinline__ C mul_mi(C a) {  // a * (-i)
    C r;
    r.x = a.y;
    r.y = -a.x;
    return r;
}

template <typename T>
__device__ __forceinline__ double sample_d(const T *p, int64_t i) {
    return static_cast<double>(p[i]);
}

// one Stockham pass of radix R (4 or 2) over M points: src -> dst, Ns = product of the radices
// of the passes before (out[(j - k) R + k + r Ns] = sum_q in[j + q M/R] W^{...})
template <int R, typename C>
__device__ __forceinline__ void stockham(const C *__restrict__ src, C *__restrict__ dst, const C *__restrict__ tw,
                                         int M, int Ns) {
    const int nbf = M / R;
    for (int j = threadIdx.x; j < nbf; j += SA_THREADS) {
        const int k = j & (Ns - 1);
        C v[R];
#pragma unroll
        for (int q = 0; q < R; ++q) v[q] = src[j + q * nbf];
        if (Ns > 1) {
            const int step = M / (Ns * R);  // W_M^{k q M / (Ns R)} = W_{Ns R}^{k q}
#pragma unroll
            for (int q = 1; q < R; ++q) v[q] = cmul(v[q], tw[k * q * step]);
        }
        if constexpr (R == 4) {
            const C t0 = cadd(v[0], v[2]), t1 = csub(v[0], v[2]), t2 = cadd(v[1], v[3]), t3 = mul_mi(csub(v[1], v[3]));
            v[0] = cadd(t0, t2);
            v[1] = cadd(t1, t3);
            v[2] = csub(t0, t2);
            v[3] = csub(t1, t3);
        } else {
            const C a = v[0];
            v[0] = cadd(a, v[1]);
            v[1] = csub(a, v[1]);
        }
        const int o = (j - k) * R + k;
#pragma unroll
        for (int q = 0; q < R; ++q) dst[o + q * Ns] = v[q];
    }
}

// the same pass in place on one buffer (float64 at nfft 16384: two M-point buffers would need 256 KB
// of LDS, the workgroup has 160 KB): every thread first reads all its butterflies' inputs into
// registers (M <= 8192: at most 32 complex values), the workgroup synchronises, then writes
template <int R, typename C>
__device__ __forceinline__ void stockham_inplace(C *__restrict__ buf, const C *__restrict__ tw, int M, int Ns) {
    constexpr int NB = 32 / R;  // butterflies per thread at M = 8192
    const int nbf = M / R;
    C v[NB][R];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const int j = threadIdx.x + b * SA_THREADS;
        if (j < nbf)
#pragma unroll
            for (int q = 0; q < R; ++q) v[b][q] = buf[j + q * nbf];
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const int j = threadIdx.x + b * SA_THREADS;
        if (j >= nbf) continue;
        const int k = j & (Ns - 1);
        if (Ns > 1) {
            const int step = M / (Ns * R);
#pragma unroll
            for (int q = 1; q < R; ++q) v[b][q] = cmul(v[b][q], tw[k * q * step]);
        }
        if constexpr (R == 4) {
            const C t0 = cadd(v[b][0], v[b][2]), t1 = csub(v[b][0], v[b][2]), t2 = cadd(v[b][1], v[b][3]),
                    t3 = mul_mi(csub(v[b][1], v[b][3]));
            v[b][0] = cadd(t0, t2);
            v[b][1] = cadd(t1, t3);
            v[b][2] = csub(t0, t2);
            v[b][3] = csub(t1, t3);
        } else {
            const C a = v[b][0];
            v[b][0] = cadd(a, v[b][1]);
            v[b][1] = csub(a, v[b][1]);
        }
        const int o = (j - k) * R + k;
#pragma unroll
        for (int q = 0; q < R; ++q) buf[o + q * Ns] = v[b][q];
    }
}

// INPLACE: one M-point LDS buffer (stockham_inplace) instead of two
template <typename T, typename R, bool INPLACE>
__global__ __launch_bounds__(SA_THREADS) void stft_any_kernel(
    const T *__restrict__ x, const int64_t *__restrict__ off, const int64_t *__restrict__ len, int nperseg, int hop,
    int M, int logM, R scale, int detrend, const R *__restrict__ win, const typename Cx<R>::t *__restrict__ tw,
    const typename Cx<R>::t *__restrict__ post, R *__restrict__ out, int64_t ld) {
    using C = typename Cx<R>::t;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    C *A = reinterpret_cast<C *>(smem);
    C *B = INPLACE ? A : A + M;
    __shared__ double red[SA_THREADS / 64];

    const int64_t f = blockIdx.y;
    const int64_t t = blockIdx.x;
    const int64_t n = len[f];
    const int64_t nfr = n >= nperseg ? (n - nperseg) / hop + 1 : 0;
    const int K = M + 1;
    R *of = out + f * (int64_t)K * ld + t;
    if (t >= nfr) {  // padding column (t in [T_f, ld)): zeros
        for (int k = threadIdx.x; k < K; k += SA_THREADS) of[(int64_t)k * ld] = R(0);
        return;
    }
    const T *xf = x + off[f] + t * (int64_t)hop;

    // ---- constant detrend: the mean of the nperseg samples, float64 (exact for integer samples)
    double mean = 0.0;
    if (detrend) {
        double s = 0.0;
        for (int i = threadIdx.x; i < nperseg; i += SA_THREADS) s += sample_d(xf, i);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
        __syncthreads();
        double tot = 0.0;
#pragma unroll
        for (int w = 0; w < SA_THREADS / 64; ++w) tot += red[w];
        mean = tot / (double)nperseg;
    }
    // ---- windowed, zero-padded, packed into M complex points.  scipy's constant detrend runs in
    // float64 for every input but float32 (scipy.signal.detrend casts to 'd'): x - mean in float64,
    // then rounded to the working precision (a float32 mean of a large DC offset, e.g. uint16 input
    // around 32768, would leave up to half an ulp of 32768 in bins 0 and 1)
    constexpr bool f32_detrend = std::is_same<T, float>::value;
    auto centred = [&](int i) -> R {
        if constexpr (f32_detrend) return static_cast<R>(xf[i]) - static_cast<R>(mean);
        else return static_cast<R>(static_cast<double>(xf[i]) - mean);
    };
    for (int m = threadIdx.x; m < M; m += SA_THREADS) {
        const int i0 = 2 * m, i1 = 2 * m + 1;
        const R a = i0 < nperseg ? centred(i0) * win[i0] : R(0);
        const R b = i1 < nperseg ? centred(i1) * win[i1] : R(0);
        A[m] = Cx<R>::make(a, b);
    }
    __syncthreads();
    // ---- radix-4 passes (one radix-2 first when log2 M is odd), ping-pong A <-> B
    C *src = A, *dst = B;
    int Ns = 1;
    if constexpr (INPLACE) {
        if (logM & 1) {
            stockham_inplace<2>(A, tw, M, Ns);
            Ns *= 2;
            __syncthreads();
        }
        for (int p = 0; p < logM / 2; ++p) {
            stockham_inplace<4>(A, tw, M, Ns);
            Ns *= 4;
            __syncthreads();
        }
    } else {
    if (logM & 1) {
        stockham<2>(src, dst, tw, M, Ns);
        Ns *= 2;
        __syncthreads();
        C *tmp = src;
        src = dst;
        dst = tmp;
    }
    for (int p = 0; p < logM / 2; ++p) {
        stockham<4>(src, dst, tw, M, Ns);
        Ns *= 4;
        __syncthreads();
        C *tmp = src;
        src = dst;
        dst = tmp;
    }
    }
    // ---- real split: X[k] = (Z[k] + conj Z[M-k]) / 2 + W_{2M}^k (Z[k] - conj Z[M-k]) / (2i)
    for (int k = threadIdx.x; k < K; k += SA_THREADS) {
        const C zk = src[k & (M - 1)];
        const C zm = src[(M - k) & (M - 1)];
        const C e = Cx<R>::make(R(0.5) * (zk.x + zm.x), R(0.5) * (zk.y - zm.y));
        const C o = Cx<R>::make(R(0.5) * (zk.y + zm.y), R(-0.5) * (zk.x - zm.x));
        const C X = cadd(e, cmul(post[k], o));
        R p = (X.x * X.x + X.y * X.y) * scale;
        if (k != 0 && k != M) p *= R(2);
        of[(int64_t)k * ld] = p;
    }
}

template <typename T, typename R>
int launch_any_t(msd_stft_plan *p, const void *x, const int64_t *off, const int64_t *len, int64_t nfiles, R *out,
                 int64_t ld) {
    using C = typename Cx<R>::t;
    const int M = p->M;
    // two ping-pong buffers where they fit beside the static LDS, else one (in-place passes);
    // M <= 8192 (nfft <= 16384), so one buffer always fits (float64: 128 KB)
    constexpr int kLdsMax = 160 * 1024 - 1024;
    const bool inplace = 2 * M * (int)sizeof(C) > kLdsMax;
    if (M * (int)sizeof(C) > kLdsMax || M > 8192)
        return fail(MSD_ERR_UNSUPPORTED, "stft: nfft too large for one workgroup's LDS");
    const int lds = (inplace ? 1 : 2) * M * (int)sizeof(C);
    auto kern = inplace ? stft_any_kernel<T, R, true> : stft_any_kernel<T, R, false>;
    if (int rc = ensure_dyn_lds(reinterpret_cast<const void *>(kern), lds)) return rc;
    if (ld > 0x7fffffffLL || nfiles > 65535) return fail(MSD_ERR_UNSUPPORTED, "stft: grid too large for this shape");
    int logM = 0;
    while ((1 << logM) < M) ++logM;
    // the plan keeps its window and twiddles in the precision it computes in
    const R *win = static_cast<const R *>(p->precision == MSD_F64 ? (const void *)p->d_window64
                                                                  : (const void *)p->d_window);
    const C *tw = static_cast<const C *>(p->precision == MSD_F64 ? (const void *)p->d_tw64 : (const void *)p->d_tw);
    const C *post =
        static_cast<const C *>(p->precision == MSD_F64 ? (const void *)p->d_post64 : (const void *)p->d_post);
    hipLaunchKernelGGL(kern, dim3((unsigned)ld, (unsigned)nfiles), dim3(SA_THREADS), lds, p->ctx->stream,
                       static_cast<const T *>(x), off, len, p->nperseg, p->hop, M, logM, static_cast<R>(p->scale),
                       p->detrend, win, tw, post, out, ld);
    MSD_HIP(hipGetLastError());
    return MSD_OK;
}

template <typename R>
int launch_any_r(msd_stft_plan *p, const void *x, int dtype, const int64_t *off, const int64_t *len, int64_t nfiles,
                 R *out, int64_t ld) {
    switch (dtype) {
        case MSD_U8: return launch_any_t<uint8_t, R>(p, x, off, len, nfiles, out, ld);
        case MSD_I16: return launch_any_t<int16_t, R>(p, x, off, len, nfiles, out, ld);
        case MSD_I32: return launch_any_t<int32_t, R>(p, x, off, len, nfiles, out, ld);
        case MSD_F32: return launch_any_t<float, R>(p, x, off, len, nfiles, out, ld);
        case MSD_F64: return launch_any_t<double, R>(p, x, off, len, nfiles, out, ld);
        default: return fail(MSD_ERR_UNSUPPORTED, "stft: dtype must be u8, i16, i32, f32 or f64");
    }
}

}  // namespace

int launch_stft_any(msd_stft_plan *p, const void *x, int dtype, const int64_t *off, const int64_t *len,
                    int64_t nfiles, void *out, int64_t ld) {
    if (p->precision == MSD_F64) return launch_any_r<double>(p, x, dtype, off, len, nfiles, static_cast<double *>(out), ld);
    return launch_any_r<float>(p, x, dtype, off, len, nfiles, static_cast<float *>(out), ld);
}

}  // namespace msd
