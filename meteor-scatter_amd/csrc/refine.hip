// C5 certification, the refinement step: the band / noise dB delta of chosen STFT frames of an I/Q
// stream recomputed in float64 straight from the samples, for the frames whose detector decision
// the fp32 spectrogram's error bound cannot settle (and the frames of the windows their thresholds
// come from).  The quantity is the float64 reference's: scipy.signal.spectrogram of complex128
// input (periodic Hann, constant detrend, density) summed over the fftfreq band masks, 10*log10(E
// + 1e-12), band - noise (dsp/src/main.py:380-393 per frame).
//
// Only the band bins are needed, so no FFT: with the periodic Hann window w[n] = 1/2 - 1/4
// e^{2 pi i n/N} - 1/4 e^{-2 pi i n/N}, the windowed DFT of the detrended frame v = z - mean is
//   Y[k] = 1/2 V[k] - 1/4 V[k-1] - 1/4 V[k+1],   V[k] = Z[k] - N mean [k = 0 mod N],
// and a frame of N samples at hop H is R = N/D blocks of D = gcd(N, H) samples, so
//   Z_t[k] = sum_{j<R} e^{-2 pi i k j D / N} B_{tH/D + j}[k],  B_m[k] = sum_{n<D} z[mD + n] e^{-2 pi i k n/N}.
// Each block's B at the needed bins (band and noise bins +-1) is computed once (block_kernel: one
// wave per block, a float64 Goertzel recurrence over a contiguous segment per lane, rotated to the
// block origin and summed over the wave), then every frame combines its R blocks (frame_kernel).
// At C5 (N 4096, H 1024: D 1024, R 4) that is 1024 samples x 9 bins per frame instead of 4096 x 5
// for a per-frame DFT.
//
// The error bound written beside each delta (ed) covers both float64 computations (ours: the
// Goertzel chains and the combination; the reference's: pocketfft's 4 log2 N + 8 and the detrend /
// window roundings), against sum |v_n w_n| <= sum |z_n| + N |mean|: ~1e-12 dB, so a decision that
// stays uncertain after refinement is a genuine float64 near tie.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include <type_traits>
#include <vector>

#include "msd_internal.h"
#include "refine_i8.h"
#include "refine_plan.h"

namespace msd {
namespace {

template <typename T>
struct Samp;
template <>
struct Samp<int16_t> {
    __device__ static double2 at(const int16_t *x, int64_t i) {
        const uint32_t r = reinterpret_cast<const uint32_t *>(x)[i];
        return make_double2((double)(int16_t)(r & 0xffffu), (double)(int16_t)(r >> 16));
    }
};
template <>
struct Samp<float> {
    __device__ static double2 at(const float *x, int64_t i) {
        const float2 v = reinterpret_cast<const float2 *>(x)[i];
        return make_double2((double)v.x, (double)v.y);
    }
};

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }

// the range holding compact index g: ranges' compact starts cs[0..nr] (cs[nr] = total)
__device__ __forceinline__ int find_range(const int64_t *cs, int nr, int64_t g) {
    int lo = 0, hi = nr - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (cs[mid] <= g) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// double DPP moves (both halves), for row reductions of float64 values
template <int CTRL>
__device__ __forceinline__ double dpp_d(double x) {
    const long long v = __builtin_bit_cast(long long, x);
    const int lo = __builtin_amdgcn_mov_dpp((int)(v & 0xffffffffll), CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(v >> 32), CTRL, 0xf, 0xf, true);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
// every lane of a row of 16 gets the row's sum
__device__ __forceinline__ double row_sum_d(double v) {
    v += dpp_d<0xB1>(v);
    v += dpp_d<0x4E>(v);
    v += dpp_d<0x141>(v);
    v += dpp_d<0x140>(v);
    return v;
}

template <typename T>
struct Quad;  // four consecutive complex samples per load: raw() fetches, cvt() widens
template <>
struct Quad<int16_t> {
    using Raw = uint4;
    __device__ static Raw raw(const int16_t *x, int64_t i) {
        return *reinterpret_cast<const uint4 *>(reinterpret_cast<const uint32_t *>(x) + i);
    }
    __device__ static void cvt(const Raw &r, double2 (&z)[4]) {
        const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) z[e] = make_double2((double)(int16_t)(w[e] & 0xffffu), (double)(int16_t)(w[e] >> 16));
    }
};
template <>
struct Quad<float> {
    struct Raw {
        float4 a, b;
    };
    __device__ static Raw raw(const float *x, int64_t i) {
        return Raw{*reinterpret_cast<const float4 *>(x + 2 * i), *reinterpret_cast<const float4 *>(x + 2 * i + 4)};
    }
    __device__ static void cvt(const Raw &r, double2 (&z)[4]) {
        z[0] = make_double2(r.a.x, r.a.y);
        z[1] = make_double2(r.a.z, r.a.w);
        z[2] = make_double2(r.b.x, r.b.y);
        z[3] = make_double2(r.b.z, r.b.w);
    }
};

// D % 64 == 0 (RefineGeom::rows): sixteen lanes per block (a row of the wave), lane L the D/16 consecutive samples from
// L D/16; one pass over the samples runs the Goertzel recurrence of NK bins (the nk needed ones,
// padded with copies of bin 0 whose results are dropped: no per-bin branch in the loop), each
// segment's DFT is rotated to the block origin with two table twiddles, and the row sums the 16
// partials.  The next four samples are loaded before the current four are used.  Output
// bin-major (the frame kernel's neighbouring frames then read neighbouring addresses):
// out[b * nblocks + g] = B_g[k_b] for b < nk, then the block's sample sum (b = nk) and its sum of
// |re| + |im| (b = nk + 1, .x).
template <typename T, int NK>
__global__ __launch_bounds__(256) void block_kernel(const T *__restrict__ x, RefineGeom G, RefineBins K,
                                                    const int64_t *__restrict__ bstart, const int64_t *__restrict__ bcs,
                                                    int64_t nblocks, const double2 *__restrict__ W,
                                                    double2 *__restrict__ out) {
    const int l16 = threadIdx.x & 15;
    int64_t g = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
    const bool live = g < nblocks;
    if (!live) g = nblocks - 1;  // the row still takes part in nothing but its own DPP sums
    const int r = find_range(bcs, G.nr, g);
    const int64_t m = bstart[r] + (g - bcs[r]);
    const int S = G.D / 16;  // samples per lane (a multiple of 4)
    const int n0 = l16 * S;
    const int64_t base = m * (int64_t)G.D + n0;
    double c2[NK];
    double2 s1[NK], s2[NK];
#pragma unroll
    for (int b = 0; b < NK; ++b) {
        c2[b] = 2.0 * W[K.km[b < K.nk ? b : 0]].x;  // 2 cos(theta)
        s1[b] = make_double2(0.0, 0.0);
        s2[b] = make_double2(0.0, 0.0);
    }
    double2 sum = make_double2(0.0, 0.0);
    double l1 = 0.0;
    // the recurrence s_n = z_n + 2 cos(theta) s_{n-1} - s_{n-2}, two samples per step with the roles
    // of s1 / s2 alternating (no register moves): s2 <- fma(c2, s1, z0 - s2), s1 <- fma(c2, s2, z1 - s1)
    typename Quad<T>::Raw rn = Quad<T>::raw(x, base);
    for (int q = 0; q < S; q += 4) {
        double2 z[4];
        Quad<T>::cvt(rn, z);
        if (q + 4 < S) rn = Quad<T>::raw(x, base + q + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            sum = cadd(sum, z[e]);
            l1 += fabs(z[e].x) + fabs(z[e].y);
        }
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
#pragma unroll
            for (int b = 0; b < NK; ++b) {
                s2[b] = make_double2(fma(c2[b], s1[b].x, z[e].x - s2[b].x), fma(c2[b], s1[b].y, z[e].y - s2[b].y));
                s1[b] = make_double2(fma(c2[b], s2[b].x, z[e + 1].x - s1[b].x),
                                     fma(c2[b], s2[b].y, z[e + 1].y - s1[b].y));
            }
        }
    }
    double2 *o = out + g;  // bin-major: value b of block g at out[b * nblocks + g]
#pragma unroll
    for (int b = 0; b < NK; ++b) {
        if (b >= K.nk) continue;
        const int km = K.km[b];
        double2 c;
        if (km == 0) {
            c = sum;
        } else {  // sum_q z[n0 + q] W^{k (n0 + q)} = W^{k (n0 + S - 1)} s_{S-1} - W^{k (n0 + S)} s_{S-2}
            const double2 t1 = W[(int)(((uint32_t)km * (uint32_t)(n0 + S - 1)) % (uint32_t)G.N)];
            const double2 t2 = W[(int)(((uint32_t)km * (uint32_t)(n0 + S)) % (uint32_t)G.N)];
            c = csub(cmul(t1, s1[b]), cmul(t2, s2[b]));
        }
        c = make_double2(row_sum_d(c.x), row_sum_d(c.y));
        if (live && l16 == 0) o[b * nblocks] = c;
    }
    const double sx = row_sum_d(sum.x), sy = row_sum_d(sum.y), sl = row_sum_d(l1);
    if (live && l16 == 0) {
        o[K.nk * nblocks] = make_double2(sx, sy);
        o[(K.nk + 1) * nblocks] = make_double2(sl, 0.0);
    }
}

// D not a multiple of 64: one lane per block (a direct DFT over its D samples)
template <typename T>
__global__ __launch_bounds__(256) void block_small_kernel(const T *__restrict__ x, RefineGeom G, RefineBins K,
                                                          const int64_t *__restrict__ bstart,
                                                          const int64_t *__restrict__ bcs, int64_t nblocks,
                                                          const double2 *__restrict__ W, double2 *__restrict__ out) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nblocks) return;
    const int r = find_range(bcs, G.nr, g);
    const int64_t m = bstart[r] + (g - bcs[r]);
    const int64_t base = m * (int64_t)G.D;
    double2 sum = make_double2(0.0, 0.0);
    double l1 = 0.0;
    for (int q = 0; q < G.D; ++q) {
        const double2 z = Samp<T>::at(x, base + q);
        sum = cadd(sum, z);
        l1 += fabs(z.x) + fabs(z.y);
    }
    double2 *o = out + g;  // bin-major, as block_kernel
    for (int b = 0; b < K.nk; ++b) {
        const int km = K.km[b];
        if (km == 0) {
            o[b * nblocks] = sum;
            continue;
        }
        double2 acc = make_double2(0.0, 0.0);
        for (int q = 0; q < G.D; ++q)
            acc = cadd(acc, cmul(Samp<T>::at(x, base + q), W[(int)(((uint32_t)km * (uint32_t)q) % (uint32_t)G.N)]));
        o[b * nblocks] = acc;
    }
    o[K.nk * nblocks] = sum;
    o[(K.nk + 1) * nblocks] = make_double2(l1, 0.0);
}

// dB error of a band of n bins with energy E when every bin's amplitude is off by at most d
// (float64 computations on both sides)
__device__ __forceinline__ double band_db_bound64(double E, int n, double d) {
    if (n <= 0) return 0.0;
    const double u = 0x1p-53;
    const double dE = 2.0 * d * sqrt((double)n * E) + 3.0 * (double)n * d * d + 2.0 * ((double)n + 4.0) * u * E;
    const double den = E + 1e-12 - dE;
    if (!(den > 0.0)) return __builtin_inf();
    return 4.342944819032518 * dE / den * (1.0 + 1e-9);
}

// one thread per frame: combine the R blocks (rot[b][j] = W^{k_b j D}, host table, uniform reads),
// the Hann taps, |Y|^2 * scale, the band sums in np.sum order, 10 log10(E + 1e-12); delta and its bound.
// RC: R at compile time (C5: 4; a band bin's 3 R block loads then issue together: -0.033 ms of the
// 1.92 ms delta step, tools/i8_time.py against tools/experiments/r4_frame_kernel_old.patch) or 0 (runtime R).
// Loading the next bin's taps ahead did not pipeline: the compiler sinks the loads below the sums.
template <int RC>
__global__ __launch_bounds__(256) void frame_kernel(RefineGeom G, RefineBins K, const int64_t *__restrict__ fstart,
                                                    const int64_t *__restrict__ fcs, const int64_t *__restrict__ bstart,
                                                    const int64_t *__restrict__ bcs, int64_t nframes, int64_t nblocks,
                                                    const double2 *__restrict__ rot, const double2 *__restrict__ blk,
                                                    double *__restrict__ delta, double *__restrict__ ed,
                                                    double2 *__restrict__ fsum) {
    const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nframes) return;
    const int R = RC ? RC : G.R;
    const int r = find_range(fcs, G.nr, f);
    const int64_t t = fstart[r] + (f - fcs[r]);
    const int64_t m0 = t * (G.hop / G.D);  // first block of the frame (D = gcd(N, hop) divides hop)
    // bin-major blocks: neighbouring frames read neighbouring addresses
    const double2 *b0 = blk + (bcs[r] + (m0 - bstart[r]));
    const int64_t stride = nblocks;
    double2 sum = make_double2(0.0, 0.0);
    double l1 = 0.0;
#pragma unroll
    for (int j = 0; j < R; ++j) {
        sum = cadd(sum, b0[K.nk * stride + j]);
        l1 += b0[(K.nk + 1) * stride + j].x;
    }
    if (fsum) fsum[t] = sum;  // the frame's sample sums (exact for int16), for the spectrogram's detrend
    const double2 mean = make_double2(sum.x / G.N, sum.y / G.N);
    // V[k'] of the detrended frame at needed bin b from its R block values v
    const double2 dcm = make_double2(mean.x * G.N, mean.y * G.N);
    auto V = [&](int b, const double2 *v) {
        const double2 *rb = rot + b * R;
        double2 z = v[0];
#pragma unroll
        for (int j = 1; j < R; ++j) z = cadd(z, cmul(rb[j], v[j]));
        return b == K.dc ? csub(z, dcm) : z;
    };
    auto energy = [&](const int (*idx)[3], int n) {
        double E = 0.0;
        for (int q = 0; q < n; ++q) {
            double2 a, c, e;
            if constexpr (RC > 0) {  // the three taps' 3 R loads issued together, then the sums
                double2 v[3][RC];
#pragma unroll
                for (int i = 0; i < 3; ++i)
#pragma unroll
                    for (int j = 0; j < RC; ++j) v[i][j] = b0[idx[q][i] * stride + j];
                a = V(idx[q][0], v[0]), c = V(idx[q][1], v[1]), e = V(idx[q][2], v[2]);
            } else {
                auto Vb = [&](int b) { return V(b, b0 + b * stride); };
                a = Vb(idx[q][0]), c = Vb(idx[q][1]), e = Vb(idx[q][2]);
            }
            const double2 y = make_double2(0.5 * c.x - 0.25 * a.x - 0.25 * e.x, 0.5 * c.y - 0.25 * a.y - 0.25 * e.y);
            E += (y.x * y.x + y.y * y.y) * G.scale;
        }
        return E;
    };
    const double Eb = energy(K.bidx, K.nb), En = energy(K.nidx, K.nn);
    delta[t] = 10.0 * log10(Eb + 1e-12) - 10.0 * log10(En + 1e-12);
    // sum |v w| <= sum |z| + N |mean| (w <= 1); amplitude scale sqrt(scale) as P = |Y|^2 scale
    const double amp = (l1 + (double)G.N * (fabs(mean.x) + fabs(mean.y))) * sqrt(G.scale);
    const double d = G.chain * 0x1p-53 * amp;
    ed[t] = band_db_bound64(Eb, K.nb, d) + band_db_bound64(En, K.nn, d) + 1e-13;
}

// frame_kernel with a compile-time R = 4 (C5) or the runtime loop
inline void launch_frame(hipStream_t st, const RefineGeom &G, const RefineBins &K, const int64_t *fstart,
                         const int64_t *fcs, const int64_t *bstart, const int64_t *bcs, int64_t nframes,
                         int64_t nblocks, const double2 *rot, const double2 *blk, double *delta, double *ed,
                         double2 *fsum) {
    const dim3 grid((unsigned)((nframes + 255) / 256));
    auto kern = G.R == 4 ? frame_kernel<4> : frame_kernel<0>;
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, st, G, K, fstart, fcs, bstart, bcs, nframes, nblocks, rot, blk,
                       delta, ed, fsum);
}

}  // namespace
}  // namespace msd

using namespace msd;

extern "C" {

int msd_iq_delta64_path(int32_t nperseg, int64_t hop, double fs, int32_t band_lo, int32_t band_hi, int32_t noise_lo,
                        int32_t noise_hi, int32_t dtype) {
    if (dtype != MSD_CI16 && dtype != MSD_CF32) return fail(MSD_ERR_UNSUPPORTED, "msd_iq_delta64_path: CI16 or CF32");
    RefinePlan P;
    std::string msg;
    if (int rc = plan_refine(nperseg, hop, fs, band_lo, band_hi, noise_lo, noise_hi, nullptr, 0, 0, P, msg))
        return fail(rc, "msd_iq_delta64_path: " + msg);
    if (dtype == MSD_CI16 && i8_supported(P.G, P.K)) return MSD_REFINE_INT8_MFMA;
    return P.G.rows ? MSD_REFINE_GOERTZEL_ROWS : MSD_REFINE_DIRECT;
}

int msd_iq_delta64_dev(msd_ctx *ctx, const void *x, int32_t dtype, int64_t n_samples, int32_t nperseg, int64_t hop,
                       double fs, int32_t band_lo, int32_t band_hi, int32_t noise_lo, int32_t noise_hi,
                       const int64_t *ranges, int64_t nranges, double *delta, double *ed) {
    return msd_iq_delta64_sums_dev(ctx, x, dtype, n_samples, nperseg, hop, fs, band_lo, band_hi, noise_lo, noise_hi,
                                   ranges, nranges, delta, ed, nullptr);
}

int msd_iq_delta64_sums_dev(msd_ctx *ctx, const void *x, int32_t dtype, int64_t n_samples, int32_t nperseg,
                            int64_t hop, double fs, int32_t band_lo, int32_t band_hi, int32_t noise_lo,
                            int32_t noise_hi, const int64_t *ranges, int64_t nranges, double *delta, double *ed,
                            double *frame_sums) {
    double2 *fsum = reinterpret_cast<double2 *>(frame_sums);
    if (!ctx || (!x && n_samples) || !delta || !ed || (!ranges && nranges) || nranges < 0 || nperseg < 4 ||
        hop <= 0 || !(fs > 0))
        return fail(MSD_ERR_INVALID, "msd_iq_delta64_dev: bad args");
    if (dtype != MSD_CI16 && dtype != MSD_CF32) return fail(MSD_ERR_UNSUPPORTED, "msd_iq_delta64_dev: CI16 or CF32");
    RefinePlan P;
    std::string msg;
    if (int rc = plan_refine(nperseg, hop, fs, band_lo, band_hi, noise_lo, noise_hi, ranges, nranges, n_samples, P, msg))
        return fail(rc, "msd_iq_delta64_dev: " + msg);
    const int N = nperseg;
    RefineBins &K = P.K;
    RefineGeom &G = P.G;
    if (fsum && dtype == MSD_CI16 && !ctx->refine_goertzel && i8_supported(G, K) && K.nk <= 8)
        return fail(MSD_ERR_UNSUPPORTED, "msd_iq_delta64_sums_dev: this block step carries no sums (int8, <= 8 bins)");
    if (nranges == 0) return MSD_OK;
    const std::vector<int64_t> &fstart = P.fstart, &fcs = P.fcs, &bstart = P.bstart, &bcs = P.bcs;
    const int64_t nblocks = P.nblocks, nframes = P.nframes;
    DeviceGuard g(ctx->device);
    hipStream_t st = ctx->stream;
    // W^m (m < N): built and uploaded once per frame length (N sin / cos on the host cost
    // ~0.2 ms, more than the refinement's other host work), kept on the context
    if (ctx->rf_w_n != N) {
        std::vector<double2> W(N);
        for (int m = 0; m < N; ++m) {  // W^m = cos - i sin of 2 pi m / N, each within ~0.5 ulp
            long double c, sn;
            unit_root_ld(m, N, c, sn);
            W[m] = make_double2((double)c, -(double)sn);
        }
        MSD_HIP(hipStreamSynchronize(st));
        if (ctx->rf_w) MSD_HIP(hipFree(ctx->rf_w));
        ctx->rf_w = nullptr;
        ctx->rf_w_n = 0;
        MSD_HIP(hipMalloc(&ctx->rf_w, sizeof(double2) * N));
        MSD_HIP(hipMemcpy(ctx->rf_w, W.data(), sizeof(double2) * N, hipMemcpyHostToDevice));
        ctx->rf_w_n = N;
    }
    const double2 *Wd = ctx->rf_w;
    // per call: the per-bin block rotations rot[b][j] = W^{k_b j D} (j < R), and the ranges
    const int R = G.R;
    std::vector<double2> rt((size_t)K.nk * R);
    for (int b = 0; b < K.nk; ++b)
        for (int j = 0; j < R; ++j) {
            const int64_t m = (int64_t)G.D * (((int64_t)K.km[b] * j) % R);
            long double c, sn;
            unit_root_ld(m, N, c, sn);
            rt[(size_t)b * R + j] = make_double2((double)c, -(double)sn);
        }
    const size_t nb_blk = (sizeof(double2) * (size_t)nblocks * (K.nk + 2) + 255) / 256 * 256;
    const size_t nb_rot = (sizeof(double2) * rt.size() + 255) / 256 * 256;
    const size_t nb_meta = sizeof(int64_t) * (4 * (size_t)nranges + 2);
    void *d = nullptr;
    if (int rc = ctx_scratch(ctx, 4, nb_blk + nb_rot + nb_meta, &d)) return rc;  // grown once, kept
    auto *blk = static_cast<double2 *>(d);
    auto *rot = reinterpret_cast<double2 *>(static_cast<char *>(d) + nb_blk);
    auto *meta = reinterpret_cast<int64_t *>(static_cast<char *>(d) + nb_blk + nb_rot);
    std::vector<int64_t> hm;
    hm.insert(hm.end(), fstart.begin(), fstart.end());
    hm.insert(hm.end(), fcs.begin(), fcs.end());
    hm.insert(hm.end(), bstart.begin(), bstart.end());
    hm.insert(hm.end(), bcs.begin(), bcs.end());
    const int64_t *d_fstart = meta, *d_fcs = meta + nranges, *d_bstart = meta + 2 * nranges + 1,
                  *d_bcs = meta + 3 * nranges + 1;
    // both tables through a pinned staging block (the copies are truly async, so the call returns
    // while the kernels run); the previous call's copies have left it once its event has passed.
    // The same tables as the last call's, still in the same scratch block, are not copied again:
    // in the C5 step the two copies sat between the spectrogram's end and the delta's start.
    const size_t b_rt = sizeof(double2) * rt.size(), b_hm = sizeof(int64_t) * hm.size();
    const bool same = ctx->rf_last_dev == d && ctx->rf_last.size() == b_rt + b_hm &&
                      !std::memcmp(ctx->rf_last.data(), rt.data(), b_rt) &&
                      !std::memcmp(ctx->rf_last.data() + b_rt, hm.data(), b_hm);
    hipError_t e = hipSuccess;
    if (!same) {
        ctx->rf_last_dev = nullptr;  // set again once both copies are enqueued
        if (!ctx->rf_ev) MSD_HIP(hipEventCreateWithFlags(&ctx->rf_ev, hipEventDisableTiming));
        else MSD_HIP(hipEventSynchronize(ctx->rf_ev));
        if (ctx->rf_pin_bytes < b_rt + b_hm) {
            if (ctx->rf_pin) MSD_HIP(hipHostFree(ctx->rf_pin));
            ctx->rf_pin = nullptr;
            ctx->rf_pin_bytes = 0;
            const size_t want = std::max<size_t>(b_rt + b_hm, 4096);
            MSD_HIP(hipHostMalloc(&ctx->rf_pin, want, hipHostMallocDefault));
            ctx->rf_pin_bytes = want;
        }
        char *pin = static_cast<char *>(ctx->rf_pin);
        std::memcpy(pin, rt.data(), b_rt);
        std::memcpy(pin + b_rt, hm.data(), b_hm);
        e = hipMemcpyAsync(rot, pin, b_rt, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipMemcpyAsync(meta, pin + b_rt, b_hm, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipEventRecord(ctx->rf_ev, st);
        if (e == hipSuccess) {
            ctx->rf_last.assign(pin, pin + b_rt + b_hm);
            ctx->rf_last_dev = d;
        }
    }
    // int16 blocks of 1024 samples: the exact integer DFT on the matrix cores (refine_i8.hip), its
    // own (smaller) rounding chain in the bound
    RefineGeom GF = G;
    const bool i8 = dtype == MSD_CI16 && !ctx->refine_goertzel && i8_supported(G, K);
    if (i8) GF.chain = i8_chain_own() + G.chain_tail;
    if (e == hipSuccess && i8) {
        KernelTimer timer(ctx, K_REFINE);
        if (int rc = launch_refine_i8(ctx, static_cast<const int16_t *>(x), G, K, d_bstart, d_bcs, nblocks, blk))
            return rc;
        launch_frame(st, GF, K, d_fstart, d_fcs, d_bstart, d_bcs, nframes, nblocks, rot, blk, delta, ed, fsum);
        e = hipGetLastError();
    } else if (e == hipSuccess) {
        KernelTimer timer(ctx, K_REFINE);
        if (G.rows) {  // rows of 16 lanes, S = D/16 (a multiple of 4) samples per lane
            const unsigned grid = (unsigned)((nblocks + 15) / 16);
            auto go = [&](auto nkc, const auto *xp) {
                constexpr int NKC = decltype(nkc)::value;
                using T = std::remove_cv_t<std::remove_pointer_t<decltype(xp)>>;
                auto kern = block_kernel<T, NKC>;
                hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, st, xp, G, K, d_bstart, d_bcs, nblocks, Wd, blk);
            };
            auto by_nk = [&](const auto *xp) {  // register arrays sized to the bins (C5: 9)
                if (K.nk <= 3) go(std::integral_constant<int, 3>{}, xp);
                else if (K.nk <= 5) go(std::integral_constant<int, 5>{}, xp);
                else if (K.nk <= 7) go(std::integral_constant<int, 7>{}, xp);
                else if (K.nk <= 9) go(std::integral_constant<int, 9>{}, xp);
                else if (K.nk <= 12) go(std::integral_constant<int, 12>{}, xp);
                else if (K.nk <= 16) go(std::integral_constant<int, 16>{}, xp);
                else if (K.nk <= 24) go(std::integral_constant<int, 24>{}, xp);
                else go(std::integral_constant<int, RF_MAXK>{}, xp);
            };
            if (dtype == MSD_CI16) by_nk(static_cast<const int16_t *>(x));
            else by_nk(static_cast<const float *>(x));
        } else {
            const unsigned grid = (unsigned)((nblocks + 255) / 256);
            if (dtype == MSD_CI16)
                hipLaunchKernelGGL(block_small_kernel<int16_t>, dim3(grid), dim3(256), 0, st,
                                   static_cast<const int16_t *>(x), G, K, d_bstart, d_bcs, nblocks, Wd, blk);
            else
                hipLaunchKernelGGL(block_small_kernel<float>, dim3(grid), dim3(256), 0, st,
                                   static_cast<const float *>(x), G, K, d_bstart, d_bcs, nblocks, Wd, blk);
        }
        launch_frame(st, G, K, d_fstart, d_fcs, d_bstart, d_bcs, nframes, nblocks, rot, blk, delta, ed, fsum);
        e = hipGetLastError();
    }
    if (e != hipSuccess) return hip_fail(e, "msd_iq_delta64_dev");
    return MSD_OK;
}

}  // extern "C"
