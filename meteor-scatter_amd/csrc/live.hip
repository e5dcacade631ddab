// Phase-2 live detector of the reference (dsp/src/live/backend/processor.py), float64:
//   welch_bands_kernel  a8  per processing block: scipy.signal.welch(block, fs, nfft=n_fft)
//                           (processor.py:206) restricted to the bins of the three bands, and
//                           the band sums → dB (processor.py:349-369)
//   live_detect_kernel  a9  the over-noise value, its history threshold and the
//                           Init / Detection / Tracking state machine (processor.py:391-507)
//
// welch_bands_kernel: one 256-thread workgroup per block.  The block's samples are staged
// in LDS as float64 (times the soundfile scale); each Welch segment is detrended with its
// numpy-order mean (np_reduce.h) and windowed in LDS; then every (segment, bin) pair runs a
// float64 Goertzel recurrence over the nperseg samples — the band bins only, not the whole
// nfft-point rFFT (the zero padding to nfft only sets the bin spacing).  Tasks are laid out
// so that the 64 lanes of a wave share one segment (broadcast LDS reads).  Segment powers
// are averaged in scipy's order (sequential over segments, / nseg) and the band sums use
// numpy's pairwise order.
//
// live_detect_kernel: one workgroup per file.  The history thresholds mean + k*std of the
// previous W over-noise values do not depend on the state, so they are computed in
// parallel (one thread per block); one thread then runs the state machine.
#include <cmath>

#include "msd_internal.h"
#include "np_reduce.h"

#pragma clang fp contract(off)

namespace msd {
namespace {

constexpr int WL_THREADS = 256;
constexpr int WL_SLOT_CHUNK = 512;  // bins per pass (LDS for the segment powers)

template <typename T>
__device__ __forceinline__ double to_f64(T v) {
    return (double)v;
}

struct WelchArgs {
    int64_t nfiles, max_blocks, ld;
    int block_size, nperseg, step, nseg, nfft, nslots, nbands;
    int ypitch;  // doubles per windowed segment row in LDS
    double sample_scale, scale;
    int band_lo[MSD_WELCH_MAX_BANDS], band_hi[MSD_WELCH_MAX_BANDS];
    int band_slot0[MSD_WELCH_MAX_BANDS];  // first slot of each band
};

template <typename T>
__global__ __launch_bounds__(WL_THREADS) void welch_bands_kernel(const T *__restrict__ x,
                                                                 const int64_t *__restrict__ off,
                                                                 const int64_t *__restrict__ len, WelchArgs A,
                                                                 const double *__restrict__ g_win,
                                                                 const double *__restrict__ g_bins,
                                                                 double *__restrict__ band_db,
                                                                 double *__restrict__ psd_out) {
    extern __shared__ double sm[];
    const int64_t gb = blockIdx.x;
    const int64_t f = gb / A.max_blocks;
    const int64_t b = gb - f * A.max_blocks;
    if (f >= A.nfiles) return;
    const int64_t n = len[f];
    const int64_t nb = n >= A.block_size ? (n - A.block_size) / A.block_size + 1 : 0;
    if (b >= nb) return;  // whole workgroup (uniform)
    const int tid = threadIdx.x;
    const int span = (A.nseg - 1) * A.step + A.nperseg;  // samples the segments cover
    double *xs = sm;                                      // [span]
    double *ys = xs + ((span + 1) & ~1);                  // [nseg][ypitch]
    double *mean = ys + A.nseg * A.ypitch;                // [nseg] (padded to 8)
    double *psd = mean + 8;                               // [nslots]
    double *pw = psd + ((A.nslots + 1) & ~1);             // [nseg][WL_SLOT_CHUNK]

    const T *xb = x + off[f] + b * (int64_t)A.block_size;
    for (int i = tid; i < span; i += WL_THREADS) xs[i] = to_f64(xb[i]) * A.sample_scale;
    __syncthreads();
    // detrend='constant': d - np.mean(d, axis=-1) per segment (numpy pairwise order)
    if (tid < A.nseg) mean[tid] = np_sum(ArrRef{xs}, (int64_t)tid * A.step, A.nperseg) / (double)A.nperseg;
    __syncthreads();
    for (int i = tid; i < A.nseg * A.nperseg; i += WL_THREADS) {
        const int s = i / A.nperseg, m = i - s * A.nperseg;
        ys[s * A.ypitch + m] = g_win[m] * (xs[s * A.step + m] - mean[s]);  // win * detrended
    }
    __syncthreads();

    const int chunk_pad = (WL_SLOT_CHUNK + 63) & ~63;
    for (int c0 = 0; c0 < A.nslots; c0 += WL_SLOT_CHUNK) {
        const int cn = A.nslots - c0 < WL_SLOT_CHUNK ? A.nslots - c0 : WL_SLOT_CHUNK;
        const int cpad = (cn + 63) & ~63;  // slots per segment padded to whole waves
        (void)chunk_pad;
        for (int task = tid; task < A.nseg * cpad; task += WL_THREADS) {
            const int s = task / cpad, j = task - s * cpad;  // s is wave-uniform
            if (j >= cn) continue;
            const double *bc = g_bins + 4 * (c0 + j);
            const double cw = bc[0], sw = bc[1], c2 = bc[2], dbl = bc[3];
            const double *y = ys + s * A.ypitch;
            double s1 = 0.0, s2 = 0.0;
#pragma unroll 8
            for (int m = 0; m < A.nperseg; ++m) {
                const double s0 = __builtin_fma(c2, s1, y[m] - s2);
                s2 = s1;
                s1 = s0;
            }
            // X e^{i w (L-1)} = s1 - e^{-i w} s2: |X|^2 = re^2 + im^2
            const double re = s1 - cw * s2, im = sw * s2;
            double p = re * re + im * im;  // conj(X) * X (real part)
            p = p * A.scale;               // result *= scale
            p = p * dbl;                   // result[..., 1:-1] *= 2 (onesided, psd)
            pw[s * WL_SLOT_CHUNK + j] = p;
        }
        __syncthreads();
        for (int j = tid; j < cn; j += WL_THREADS) {  // Pxy.mean(axis=-1): sequential over segments
            double acc = pw[j];
            for (int s = 1; s < A.nseg; ++s) acc += pw[s * WL_SLOT_CHUNK + j];
            const double v = acc / (double)A.nseg;
            psd[c0 + j] = v;
            if (psd_out) psd_out[(f * A.ld + b) * (int64_t)A.nslots + c0 + j] = v;
        }
        __syncthreads();
    }
    if (tid < A.nbands) {
        const int w = A.band_hi[tid] - A.band_lo[tid] + 1;
        const double P = w > 0 ? np_sum(ArrRef{psd}, A.band_slot0[tid], w) : 0.0;  // np.sum(psd[mask])
        band_db[(f * A.nbands + tid) * A.ld + b] = P > 0.0 ? 10.0 * log10(P) : -INFINITY;
    }
}

struct LiveArgs {
    msd_live_cfg cfg;
    int64_t nfiles, ld, cap;
};

// Python's builtin min/max over a list (first element kept unless a later one compares
// strictly less / greater — NaN behaves as CPython's does)
__device__ __forceinline__ void py_minmax(const double *v, int64_t a, int64_t e, double &mn, double &mx) {
    mn = v[a];
    mx = v[a];
    for (int64_t i = a + 1; i < e; ++i) {
        if (v[i] < mn) mn = v[i];
        if (v[i] > mx) mx = v[i];
    }
}

__global__ __launch_bounds__(WL_THREADS) void live_detect_kernel(const double *__restrict__ band_db,
                                                                  const int64_t *__restrict__ nblocks, LiveArgs A,
                                                                  double *__restrict__ over, double *__restrict__ thr,
                                                                  msd_meteor *__restrict__ out,
                                                                  int64_t *__restrict__ counts,
                                                                  int32_t *__restrict__ status) {
    const int64_t f = blockIdx.x;
    if (f >= A.nfiles) return;
    const int64_t nb = nblocks[f];
    const int tid = threadIdx.x;
    const double *sig = band_db + (f * 3 + 0) * A.ld;
    const double *n1 = band_db + (f * 3 + 1) * A.ld;
    const double *n2 = band_db + (f * 3 + 2) * A.ld;
    double *ov = over + f * A.ld;
    double *th = thr + f * A.ld;
    const msd_live_cfg &C = A.cfg;
    // processor.py:391: block_db_2_ms = block_db_ms - np.mean([n1, n2])
    for (int64_t i = tid; i < nb; i += WL_THREADS) {
        const double m = (-0.0 + n1[i] + n2[i]) / 2.0;
        ov[i] = sig[i] - m;
    }
    __syncthreads();
    // processor.py:392-402: history = the previous min(W, b) values (W = 0 → all of them)
    for (int64_t i = tid; i < nb; i += WL_THREADS) {
        const int64_t W = C.avg_win_blocks;
        const int64_t h0 = W > 0 ? (i - W > 0 ? i - W : 0) : 0;
        const int64_t hn = i - h0;
        double mean = NAN, sd = NAN;
        if (hn > 0) np_mean_std(ov, h0, hn, mean, sd);
        th[i] = mean + C.k_std * sd;
    }
    __syncthreads();
    if (tid != 0) return;
    // the state machine (processor.py:404-507)
    int state = 0;  // 0 init, 1 detection, 2 tracking
    double lock = -1.0, until = -1.0, t_start = 0.0;
    int64_t trig = 0, cnt = 0;
    for (int64_t i = 0; i < nb; ++i) {
        const double t0 = (double)(i * (int64_t)C.block_size) / C.fs;
        const double t1 = (double)(i * (int64_t)C.block_size + C.block_size) / C.fs;
        const double fresh = th[i];
        double t = fresh;
        if (state == 2) t = lock;
        else if (state == 1 && until > t1) t = lock;
        th[i] = t;
        const double v = ov[i];
        if (state == 0) {
            if (t0 >= C.init_wait_sec) {
                state = 1;
                lock = -1.0;
                until = -1.0;
            }
        } else if (state == 1) {
            if (v > t) {
                // locked_threshold = thr + 0 * history_std (NaN if the std is)
                const int64_t W = C.avg_win_blocks;
                const int64_t h0 = W > 0 ? (i - W > 0 ? i - W : 0) : 0;
                double hm = NAN, hs = NAN;
                if (i - h0 > 0) np_mean_std(ov, h0, i - h0, hm, hs);
                lock = t + 0.0 * hs;
                t_start = t0;
                trig = i;
                state = 2;
            }
        } else {
            if (v < t) {  // history = over[trig+1 .. i]
                const double dur = t0 - t_start;
                double hm, hs;
                np_mean_std(ov, trig + 1, i - trig, hm, hs);
                if (hm >= C.min_db_mean && dur >= C.min_dur_sec) {
                    if (cnt < A.cap) {
                        msd_meteor m;
                        m.start_block = trig;
                        m.stop_block = i;
                        m.time_start = t_start;
                        m.time_stop = t0;
                        m.duration = dur;
                        py_minmax(ov, trig + 1, i + 1, m.db_min, m.db_max);
                        m.db_mean = hm;
                        m.db_std = hs;
                        out[f * A.cap + cnt] = m;
                    }
                    ++cnt;
                }
                state = 1;
                until = t0 + C.after_tracking_wait_sec;
            }
        }
    }
    counts[f] = cnt;
    if (status) status[f] = cnt > A.cap ? 3 : 0;
}

template <typename T>
int launch_welch_t(msd_welch_plan *p, const void *x, const int64_t *off, const int64_t *len, int64_t nfiles,
                   int64_t max_blocks, double *band_db, int64_t ld, double *psd) {
    const msd_welch_cfg &c = p->cfg;
    WelchArgs A{};
    A.nfiles = nfiles;
    A.max_blocks = max_blocks;
    A.ld = ld;
    A.block_size = c.block_size;
    A.nperseg = c.nperseg;
    A.step = p->step;
    A.nseg = p->nseg;
    A.nfft = c.nfft;
    A.nslots = p->nslots;
    A.nbands = c.nbands;
    A.ypitch = c.nperseg + 2;  // row offset of 2 doubles: segments start on different banks
    A.sample_scale = c.sample_scale;
    A.scale = c.scale;
    int slot = 0;
    for (int j = 0; j < c.nbands; ++j) {
        A.band_lo[j] = c.band_lo[j];
        A.band_hi[j] = c.band_hi[j];
        A.band_slot0[j] = slot;
        if (c.band_hi[j] >= c.band_lo[j]) slot += c.band_hi[j] - c.band_lo[j] + 1;
    }
    const int span = (p->nseg - 1) * p->step + c.nperseg;
    const size_t lds = sizeof(double) * (((span + 1) & ~1) + (size_t)p->nseg * A.ypitch + 8 +
                                         ((p->nslots + 1) & ~1) + (size_t)p->nseg * WL_SLOT_CHUNK);
    if (lds > 160 * 1024) return fail(MSD_ERR_UNSUPPORTED, "welch: block / segment configuration exceeds LDS");
    static bool attr = false;
    if (!attr) {
        MSD_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(welch_bands_kernel<T>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        attr = true;
    }
    const int64_t grid = nfiles * max_blocks;
    if (grid > 0x7fffffffLL) return fail(MSD_ERR_UNSUPPORTED, "welch: grid too large");
    KernelTimer timer(p->ctx, K_WELCH);
    hipLaunchKernelGGL(welch_bands_kernel<T>, dim3((unsigned)grid), dim3(WL_THREADS), lds, p->ctx->stream,
                       static_cast<const T *>(x), off, len, A, p->d_window, p->d_bins, band_db, psd);
    MSD_HIP(hipGetLastError());
    return MSD_OK;
}

int launch_welch(msd_welch_plan *p, const void *x, int dtype, const int64_t *off, const int64_t *len, int64_t nfiles,
                 int64_t max_blocks, double *band_db, int64_t ld, double *psd) {
    if (nfiles == 0 || max_blocks == 0) return MSD_OK;
    switch (dtype) {
        case MSD_U8: return launch_welch_t<uint8_t>(p, x, off, len, nfiles, max_blocks, band_db, ld, psd);
        case MSD_I16: return launch_welch_t<int16_t>(p, x, off, len, nfiles, max_blocks, band_db, ld, psd);
        case MSD_I32: return launch_welch_t<int32_t>(p, x, off, len, nfiles, max_blocks, band_db, ld, psd);
        case MSD_F32: return launch_welch_t<float>(p, x, off, len, nfiles, max_blocks, band_db, ld, psd);
        case MSD_F64: return launch_welch_t<double>(p, x, off, len, nfiles, max_blocks, band_db, ld, psd);
        default: return fail(MSD_ERR_INVALID, "welch: unknown dtype");
    }
}

int launch_live(msd_ctx *ctx, const double *band_db, const int64_t *nblocks, int64_t nfiles, int64_t ld,
                const msd_live_cfg *cfg, msd_meteor *out, int64_t cap, int64_t *counts, double *thr, double *over,
                int32_t *status) {
    if (nfiles == 0) return MSD_OK;
    LiveArgs A{};
    A.cfg = *cfg;
    A.nfiles = nfiles;
    A.ld = ld;
    A.cap = cap;
    KernelTimer timer(ctx, K_LIVE);
    hipLaunchKernelGGL(live_detect_kernel, dim3((unsigned)nfiles), dim3(WL_THREADS), 0, ctx->stream, band_db, nblocks,
                       A, over, thr, out, counts, status);
    MSD_HIP(hipGetLastError());
    return MSD_OK;
}

}  // namespace
}  // namespace msd

using namespace msd;

extern "C" {

int msd_welch_plan_create(msd_ctx *ctx, const msd_welch_cfg *cfg, const double *window, msd_welch_plan **out) {
    if (!ctx || !cfg || !window || !out) return fail(MSD_ERR_INVALID, "msd_welch_plan_create: null");
    *out = nullptr;
    const msd_welch_cfg &c = *cfg;
    if (c.block_size <= 0 || c.nperseg <= 0 || c.nperseg > c.block_size || c.noverlap < 0 ||
        c.noverlap >= c.nperseg || c.nfft < c.nperseg)
        return fail(MSD_ERR_INVALID, "msd_welch_plan_create: need 0 <= noverlap < nperseg <= block_size, nfft >= nperseg");
    if (c.nbands < 1 || c.nbands > MSD_WELCH_MAX_BANDS)
        return fail(MSD_ERR_INVALID, "msd_welch_plan_create: nbands out of range");
    std::vector<double> bins;
    int nslots = 0;
    for (int j = 0; j < c.nbands; ++j) {
        if (c.band_hi[j] < c.band_lo[j]) continue;
        if (c.band_lo[j] < 0 || c.band_hi[j] > c.nfft / 2)
            return fail(MSD_ERR_INVALID, "msd_welch_plan_create: band bins outside 0..nfft/2");
        for (int k = c.band_lo[j]; k <= c.band_hi[j]; ++k) {
            const double w = 2.0 * M_PI * (double)k / (double)c.nfft;
            const bool edge = k == 0 || (c.nfft % 2 == 0 && k == c.nfft / 2);
            bins.push_back(std::cos(w));
            bins.push_back(std::sin(w));
            bins.push_back(2.0 * std::cos(w));
            bins.push_back(edge ? 1.0 : 2.0);
            ++nslots;
        }
    }
    DeviceGuard g(ctx->device);
    auto *p = new msd_welch_plan();
    p->ctx = ctx;
    p->cfg = c;
    p->step = c.nperseg - c.noverlap;
    p->nseg = (c.block_size - c.nperseg) / p->step + 1;
    p->nslots = nslots;
    hipError_t e = hipMalloc(&p->d_window, sizeof(double) * c.nperseg);
    if (e == hipSuccess) e = hipMalloc(&p->d_bins, sizeof(double) * 4 * (nslots > 0 ? nslots : 1));
    if (e == hipSuccess) e = hipMemcpy(p->d_window, window, sizeof(double) * c.nperseg, hipMemcpyHostToDevice);
    if (e == hipSuccess && nslots)
        e = hipMemcpy(p->d_bins, bins.data(), sizeof(double) * bins.size(), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        msd_welch_plan_destroy(p);
        return hip_fail(e, "msd_welch_plan_create");
    }
    *out = p;
    return MSD_OK;
}

void msd_welch_plan_destroy(msd_welch_plan *p) {
    if (!p) return;
    DeviceGuard g(p->ctx->device);
    (void)hipStreamSynchronize(p->ctx->stream);
    if (p->d_window) (void)hipFree(p->d_window);
    if (p->d_bins) (void)hipFree(p->d_bins);
    delete p;
}

int msd_welch_bands_dev(msd_welch_plan *p, const void *x, int dtype, const int64_t *off, const int64_t *len,
                        int64_t nfiles, int64_t max_blocks, double *band_db, int64_t ld, double *psd) {
    if (!p || (nfiles > 0 && (!x || !off || !len || !band_db))) return fail(MSD_ERR_INVALID, "msd_welch_bands_dev: null");
    if (ld < max_blocks) return fail(MSD_ERR_INVALID, "msd_welch_bands_dev: ld < max_blocks");
    DeviceGuard g(p->ctx->device);
    return launch_welch(p, x, dtype, off, len, nfiles, max_blocks, band_db, ld, psd);
}

int msd_welch_bands(msd_welch_plan *p, const void *x, int dtype, int64_t n, double *band_db, int64_t *blocks) {
    if (!p || (!x && n) || !band_db) return fail(MSD_ERR_INVALID, "msd_welch_bands: null");
    const size_t es = dtype_size(dtype);
    if (!es) return fail(MSD_ERR_INVALID, "msd_welch_bands: unknown dtype");
    const int64_t B = p->cfg.block_size;
    const int64_t nb = n >= B ? (n - B) / B + 1 : 0;
    if (blocks) *blocks = nb;
    if (nb == 0) return MSD_OK;
    msd_ctx *ctx = p->ctx;
    DeviceGuard g(ctx->device);
    void *dx, *dmeta, *dout;
    int rc;
    const int nbands = p->cfg.nbands;
    if ((rc = ctx_scratch(ctx, 0, ((size_t)n * es + 255) / 256 * 256, &dx))) return rc;
    if ((rc = ctx_scratch(ctx, 1, 64, &dmeta))) return rc;
    if ((rc = ctx_scratch(ctx, 2, sizeof(double) * nbands * nb, &dout))) return rc;
    int64_t meta[2] = {0, n};
    MSD_HIP(hipMemcpyAsync(dx, x, (size_t)n * es, hipMemcpyHostToDevice, ctx->stream));
    MSD_HIP(hipMemcpyAsync(dmeta, meta, sizeof(meta), hipMemcpyHostToDevice, ctx->stream));
    const int64_t *doff = static_cast<const int64_t *>(dmeta);
    rc = launch_welch(p, dx, dtype, doff, doff + 1, 1, nb, static_cast<double *>(dout), nb, nullptr);
    if (rc) return rc;
    MSD_HIP(hipMemcpyAsync(band_db, dout, sizeof(double) * nbands * nb, hipMemcpyDeviceToHost, ctx->stream));
    MSD_HIP(hipStreamSynchronize(ctx->stream));
    return MSD_OK;
}

static int check_live_cfg(const msd_live_cfg *c) {
    if (!c) return fail(MSD_ERR_INVALID, "live: null cfg");
    if (c->block_size <= 0 || !(c->fs > 0) || c->avg_win_blocks < 0)
        return fail(MSD_ERR_INVALID, "live: block_size, fs must be > 0 and avg_win_blocks >= 0");
    return MSD_OK;
}

int msd_live_detect_dev(msd_ctx *ctx, const double *band_db, const int64_t *nblocks, int64_t nfiles, int64_t ld,
                        const msd_live_cfg *cfg, msd_meteor *out, int64_t cap, int64_t *counts, double *thresholds,
                        double *over, int32_t *status) {
    if (!ctx || (nfiles > 0 && (!band_db || !nblocks || !counts || !thresholds || !over || (!out && cap))))
        return fail(MSD_ERR_INVALID, "msd_live_detect_dev: null (thresholds and over are required scratch here)");
    int rc = check_live_cfg(cfg);
    if (rc) return rc;
    DeviceGuard g(ctx->device);
    return launch_live(ctx, band_db, nblocks, nfiles, ld, cfg, out, cap, counts, thresholds, over, status);
}

int msd_live_detect(msd_ctx *ctx, const double *band_db, int64_t nb, const msd_live_cfg *cfg, msd_meteor *out,
                    int64_t cap, int64_t *count, double *thresholds, double *over) {
    if (!ctx || (!band_db && nb) || (!out && cap) || !count) return fail(MSD_ERR_INVALID, "msd_live_detect: null");
    int rc = check_live_cfg(cfg);
    if (rc) return rc;
    DeviceGuard g(ctx->device);
    const int64_t ld = nb > 0 ? nb : 1;
    const int64_t dcap = cap > 0 ? cap : 1;
    // scratch: band_db[3*ld] | over[ld] | thr[ld] | nb | count | status(pad) | meteors[dcap]
    const size_t head = sizeof(double) * 5 * ld + 32;
    void *s;
    if ((rc = ctx_scratch(ctx, 3, head + sizeof(msd_meteor) * dcap, &s))) return rc;
    char *base = static_cast<char *>(s);
    double *dband = reinterpret_cast<double *>(base);
    double *dover = dband + 3 * ld;
    double *dthr = dover + ld;
    int64_t *dnb = reinterpret_cast<int64_t *>(dthr + ld);
    int64_t *dcount = dnb + 1;
    int32_t *dstatus = reinterpret_cast<int32_t *>(dcount + 1);
    msd_meteor *dmet = reinterpret_cast<msd_meteor *>(base + head);
    if (nb) MSD_HIP(hipMemcpyAsync(dband, band_db, sizeof(double) * 3 * nb, hipMemcpyHostToDevice, ctx->stream));
    MSD_HIP(hipMemcpyAsync(dnb, &nb, sizeof(int64_t), hipMemcpyHostToDevice, ctx->stream));
    // band_db rows were packed with ld = nb
    rc = launch_live(ctx, dband, dnb, 1, ld, cfg, dmet, dcap, dcount, dthr, dover, dstatus);
    if (rc) return rc;
    int64_t cnt = 0;
    MSD_HIP(hipMemcpyAsync(&cnt, dcount, sizeof(cnt), hipMemcpyDeviceToHost, ctx->stream));
    MSD_HIP(hipStreamSynchronize(ctx->stream));
    *count = cnt;
    const int64_t ncopy = cnt < cap ? cnt : cap;
    if (ncopy > 0)
        MSD_HIP(hipMemcpyAsync(out, dmet, sizeof(msd_meteor) * ncopy, hipMemcpyDeviceToHost, ctx->stream));
    if (thresholds && nb)
        MSD_HIP(hipMemcpyAsync(thresholds, dthr, sizeof(double) * nb, hipMemcpyDeviceToHost, ctx->stream));
    if (over && nb) MSD_HIP(hipMemcpyAsync(over, dover, sizeof(double) * nb, hipMemcpyDeviceToHost, ctx->stream));
    MSD_HIP(hipStreamSynchronize(ctx->stream));
    if (cnt > cap) return fail(MSD_ERR_CAPACITY, "live: more meteors than capacity");
    return MSD_OK;
}

}  // extern "C"
