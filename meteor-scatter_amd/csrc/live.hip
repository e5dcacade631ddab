// Phase-2 live detector of the reference (dsp/src/live/backend/processor.py), float64:
//   welch_bands_kernel  a8  per processing block: scipy.signal.welch(block, fs, nfft=n_fft)
//                           (processor.py:206) restricted to the bins of the three bands, and
//                           the band sums → dB (processor.py:349-369)
//   live_seg_*_kernel   a9  the over-noise value, its history threshold and the
//                           Init / Detection / Tracking state machine (processor.py:391-507)
//
// (int16 audio takes welch_i8.hip's exact integer GEMM instead of welch_bands_kernel by default.)
// welch_bands_kernel: one wave per block.  Each Welch segment's samples are staged in the
// wave's LDS as float64 (times the soundfile scale), detrended with the numpy-order mean and
// windowed; then every band bin (one lane each) runs a float64 Goertzel recurrence over the
// nperseg samples — the band bins only, not the whole nfft-point rFFT (the zero padding to
// nfft only sets the bin spacing).  Segment powers are averaged in scipy's order (sequential
// over segments, / nseg) and the band sums use numpy's pairwise order.
//
// live_over_kernel, live_history_kernel: the over-noise values, then the history thresholds
// mean + k*std of the previous W of them -- state-free, one thread per block of every file
// (the whole GPU, not one workgroup per file);
// live_seg_{init,scan,link,emit}_kernel: the state machine in 256-block time segments, one wave
// each over the whole GPU (ballots), rounds of scan + link to a fixed point over their entry states,
// then one emitting pass.
#include <cmath>

#include "msd_internal.h"
#include "np_reduce.h"

#pragma clang fp contract(off)

namespace msd {
namespace {

constexpr int WL_THREADS = 256;

// np.sum over LDS in numpy's exact order: one pairwise leaf inline up to 128 elements (the
// default 100 Hz bands: 103 bins at nfft 4096), numpy's full recursion beyond (bands wider
// than 128 bins, nperseg above 128)
__device__ __forceinline__ double lds_band_sum(const double *p, int64_t base, int64_t n) {
    return n <= 128 ? np_sum_small(ArrRef{p}, base, n) : np_sum(ArrRef{p}, base, n);
}

template <typename T>
__device__ __forceinline__ double to_f64(T v) {
    return (double)v;
}

struct WelchArgs {
    int64_t nfiles, max_blocks, ld;
    int block_size, nperseg, step, nseg, nfft, nslots, nbands;
    int wave_lds;  // doubles of LDS per wave: segment [nperseg, padded] + psd [nslots, padded]
    double sample_scale, scale;
    int band_lo[MSD_WELCH_MAX_BANDS], band_hi[MSD_WELCH_MAX_BANDS];
    int band_slot0[MSD_WELCH_MAX_BANDS];  // first slot of each band
};

template <int CTRL>
__device__ __forceinline__ double dpp_f64(double x) {
    const int2 v = __builtin_bit_cast(int2, x);
    int2 r;
    r.x = __builtin_amdgcn_mov_dpp(v.x, CTRL, 0xf, 0xf, true);
    r.y = __builtin_amdgcn_mov_dpp(v.y, CTRL, 0xf, 0xf, true);
    return __builtin_bit_cast(double, r);
}

__device__ __forceinline__ double readlane_f64(double x, int lane) {
    const int2 v = __builtin_bit_cast(int2, x);
    int2 r;
    r.x = __builtin_amdgcn_readlane(v.x, lane);
    r.y = __builtin_amdgcn_readlane(v.y, lane);
    return __builtin_bit_cast(double, r);
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// np.sum(seg[0:n]) by one wave, numpy's pairwise order.  n = 256 (scipy's default
// nperseg): two 128-element leaves, their 8 interleaved partial sums on lanes 0-7 / 8-15,
// combined as ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) by DPP; other n: lane 0 (lds_band_sum).
__device__ __forceinline__ double wave_np_sum(const double *seg, int n, int lane) {
    if (n == 256) {
        double r = 0.0;
        if (lane < 16) {
            const double *a = seg + (lane >> 3) * 128 + (lane & 7);
            r = a[0];
            for (int k = 1; k < 16; ++k) r += a[8 * k];
        }
        r += dpp_f64<0xB1>(r);   // lane ^ 1
        r += dpp_f64<0x4E>(r);   // lane ^ 2
        r += dpp_f64<0x141>(r);  // half-row mirror: lanes 0-3 meet 4-7 (8-11 meet 12-15)
        return 0.0 + (readlane_f64(r, 0) + readlane_f64(r, 8));
    }
    double v = 0.0;
    if (lane == 0) v = lds_band_sum(seg, 0, n);
    return readlane_f64(v, 0);
}

// Goertzel power of NB band bins per lane (bins j, j + 64, ...) over the staged, windowed
// segment, added into the wave's psd in segment order.  The arithmetic per bin is the same
// for any NB (bit-identical results).
template <int NB>
__device__ __forceinline__ void goertzel_bins(const double *seg, int L, const double *__restrict__ g_bins, int j,
                                              int nslots, double scale, double *psd, int s) {
    double cw[NB], sw[NB], c2[NB], dbl[NB], s1[NB], s2[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const int jb = j + 64 * b;
        const double *bc = g_bins + 4 * (jb < nslots ? jb : 0);
        cw[b] = bc[0], sw[b] = bc[1], c2[b] = bc[2], dbl[b] = bc[3];
        s1[b] = 0.0, s2[b] = 0.0;
    }
    const double2 *y2 = reinterpret_cast<const double2 *>(seg);
    int m = 0;
#pragma unroll 4
    for (; m + 2 <= L; m += 2) {
        const double2 y = y2[m >> 1];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            double s0 = __builtin_fma(c2[b], s1[b], y.x - s2[b]);
            s2[b] = s1[b];
            s1[b] = s0;
            s0 = __builtin_fma(c2[b], s1[b], y.y - s2[b]);
            s2[b] = s1[b];
            s1[b] = s0;
        }
    }
    if (m < L) {
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const double s0 = __builtin_fma(c2[b], s1[b], seg[m] - s2[b]);
            s2[b] = s1[b];
            s1[b] = s0;
        }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const int jb = j + 64 * b;
        // X e^{i w (L-1)} = s1 - e^{-i w} s2: |X|^2 = re^2 + im^2
        const double re = s1[b] - cw[b] * s2[b], im = sw[b] * s2[b];
        double p = re * re + im * im;  // conj(X) * X (real part)
        p = p * scale;                 // result *= scale
        p = p * dbl[b];                // result[..., 1:-1] *= 2 (onesided psd)
        if (jb < nslots) psd[jb] = s == 0 ? p : psd[jb] + p;  // Pxy.mean(axis=-1): segments in order
    }
}

// One wave per processing block: per Welch segment, stage + detrend + window the samples in
// the wave's LDS, then Goertzel over the segment for every band bin (lane = bin, broadcast
// LDS reads of the samples, two per ds_read_b128), accumulating the segment powers in the
// wave's LDS psd in segment order.  No workgroup barriers: the 4 waves of a workgroup work
// on independent blocks.
template <typename T>
__global__ __launch_bounds__(WL_THREADS) void welch_bands_kernel(const T *__restrict__ x,
                                                                 const int64_t *__restrict__ off,
                                                                 const int64_t *__restrict__ len, WelchArgs A,
                                                                 const double *__restrict__ g_win,
                                                                 const double *__restrict__ g_bins,
                                                                 double *__restrict__ band_db,
                                                                 double *__restrict__ psd_out) {
    extern __shared__ double sm[];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int64_t gb = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave;  // 1-4 waves per workgroup
    const int64_t f = gb / A.max_blocks;
    const int64_t b = gb - f * A.max_blocks;
    if (f >= A.nfiles) return;
    const int64_t n = len[f];
    const int64_t nb = n >= A.block_size ? (n - A.block_size) / A.block_size + 1 : 0;
    if (b >= nb) return;  // whole wave
    double *seg = sm + wave * A.wave_lds;                 // [nperseg (+pad)]
    double *psd = seg + ((A.nperseg + 1) & ~1);           // [nslots]
    const T *xb = x + off[f] + b * (int64_t)A.block_size;
    const int L = A.nperseg;

    for (int s = 0; s < A.nseg; ++s) {
        const T *xs = xb + s * A.step;
        for (int i = lane; i < L; i += 64) seg[i] = to_f64(xs[i]) * A.sample_scale;
        wave_sync();
        // detrend='constant': d - np.mean(d, axis=-1) (numpy pairwise order)
        const double mean = wave_np_sum(seg, L, lane) / (double)L;
        wave_sync();
        for (int i = lane; i < L; i += 64) seg[i] = g_win[i] * (seg[i] - mean);  // win * detrended
        wave_sync();
        // two bins per lane while 128 remain (one broadcast LDS read feeds both recurrences:
        // half the LDS reads per flop, two independent FMA chains), then one per lane
        int j0 = 0;
        for (; j0 + 128 <= A.nslots; j0 += 128) goertzel_bins<2>(seg, L, g_bins, j0 + lane, A.nslots, A.scale, psd, s);
        for (; j0 < A.nslots; j0 += 64) goertzel_bins<1>(seg, L, g_bins, j0 + lane, A.nslots, A.scale, psd, s);
        wave_sync();
    }
    for (int j = lane; j < A.nslots; j += 64) {
        const double v = psd[j] / (double)A.nseg;
        psd[j] = v;
        if (psd_out) psd_out[(f * A.ld + b) * (int64_t)A.nslots + j] = v;
    }
    wave_sync();
    if (lane < A.nbands) {
        const int w = A.band_hi[lane] - A.band_lo[lane] + 1;
        const double P = w > 0 ? lds_band_sum(psd, A.band_slot0[lane], w) : 0.0;  // np.sum(psd[mask])
        band_db[(f * A.nbands + lane) * A.ld + b] = P > 0.0 ? 10.0 * log10(P) : -INFINITY;
    }
}

struct LiveArgs {
    msd_live_cfg cfg;
    int64_t nfiles, ld, cap;
};

// Python's builtin min/max over a list (first element kept unless a later one compares
// strictly less / greater — NaN behaves as CPython's does)
__device__ __forceinline__ void py_minmax(gdouble_t *v, int64_t a, int64_t e, double &mn, double &mx) {
    mn = v[a];
    mx = v[a];
    for (int64_t i = a + 1; i < e; ++i) {
        if (v[i] < mn) mn = v[i];
        if (v[i] > mx) mx = v[i];
    }
}

struct LiveScan {
    int state = 0;  // 0 init, 1 detection, 2 tracking
    double lock = -1.0, until = -1.0, t_start = 0.0;
    int64_t trig = 0, cnt = 0;
};

// numpy mean/std of over[b, b+n), read from global memory as such (global loads: the event handlers
// are out of line, and a generic pointer there would be read with flat instructions, np_reduce.h)
__device__ __forceinline__ void hist_stats(const double *ov, int64_t b, int64_t n, double &mean, double &sd,
                                           double *mn, double *mx) {
    np_mean_std_global(ov, b, n, mean, sd);
    if (mn) py_minmax(as_global(ov), b, b + n, *mn, *mx);
}

// The two event handlers are out of line (they run once per meteor; inlined, their numpy sums
// would be copied into every scan).  The scan state travels by value and the history is read
// through global loads: no generic pointer -- to the caller's scratch, to LDS or to global memory --
// reaches them, so they hold no flat instruction (np_reduce.h, tests/test_build_check.py).

// Detection → Tracking (processor.py:462-472): locked_threshold = thr + 0 * history_std
__device__ __noinline__ LiveScan live_trigger(LiveScan sc, const double *ov, int64_t i, double t, double t0,
                                              int64_t W) {
    const int64_t h0 = W > 0 ? (i - W > 0 ? i - W : 0) : 0;
    double hm = NAN, hs = NAN;
    if (i - h0 > 0) hist_stats(ov, h0, i - h0, hm, hs, nullptr, nullptr);
    sc.lock = t + 0.0 * hs;
    sc.t_start = t0;
    sc.trig = i;
    sc.state = 2;
    return sc;
}

// Tracking ends (processor.py:474-504): history = over[trig+1 .. i]
__device__ __noinline__ LiveScan live_close(LiveScan sc, const double *ov, int64_t i, double t0, double min_db_mean,
                                            double min_dur_sec, double wait_sec, msd_meteor *out, int64_t cap,
                                            bool writer) {
    const double dur = t0 - sc.t_start;
    double hm, hs, mn, mx;
    hist_stats(ov, sc.trig + 1, i - sc.trig, hm, hs, &mn, &mx);
    if (hm >= min_db_mean && dur >= min_dur_sec) {
        if (writer && sc.cnt < cap) {
            typedef __attribute__((address_space(1))) int64_t gi64;
            typedef __attribute__((address_space(1))) double gf64;
            msd_meteor *m = out + sc.cnt;  // fields stored through global pointers (global_store)
            *(gi64 *)&m->start_block = sc.trig;
            *(gi64 *)&m->stop_block = i;
            *(gf64 *)&m->time_start = sc.t_start;
            *(gf64 *)&m->time_stop = t0;
            *(gf64 *)&m->duration = dur;
            *(gf64 *)&m->db_min = mn;
            *(gf64 *)&m->db_max = mx;
            *(gf64 *)&m->db_mean = hm;
            *(gf64 *)&m->db_std = hs;
        }
        ++sc.cnt;
    }
    sc.state = 1;
    sc.until = t0 + wait_sec;
    return sc;
}

// processor.py:391: block_db_2_ms = block_db_ms - np.mean([n1, n2])
__global__ __launch_bounds__(WL_THREADS) void live_over_kernel(const double *__restrict__ band_db,
                                                                const int64_t *__restrict__ nblocks, LiveArgs A,
                                                                double *__restrict__ over) {
    const int64_t f = blockIdx.y;
    const int64_t i = (int64_t)blockIdx.x * WL_THREADS + threadIdx.x;
    if (i >= A.ld || i >= nblocks[f]) return;
    const double *sig = band_db + (f * 3 + 0) * A.ld;
    const double *n1 = band_db + (f * 3 + 1) * A.ld;
    const double *n2 = band_db + (f * 3 + 2) * A.ld;
    const double m = (-0.0 + n1[i] + n2[i]) / 2.0;
    over[f * A.ld + i] = sig[i] - m;
}

// processor.py:392-402: history = the previous min(W, b) values (W = 0 → all of them)
__global__ __launch_bounds__(WL_THREADS) void live_history_kernel(const int64_t *__restrict__ nblocks, LiveArgs A,
                                                                   const double *__restrict__ over,
                                                                   double *__restrict__ thr) {
    const int64_t f = blockIdx.y;
    const int64_t i = (int64_t)blockIdx.x * WL_THREADS + threadIdx.x;
    if (i >= A.ld || i >= nblocks[f]) return;
    const int64_t W = A.cfg.avg_win_blocks;
    const int64_t h0 = W > 0 ? (i - W > 0 ? i - W : 0) : 0;
    const int64_t hn = i - h0;
    double mean = NAN, sd = NAN;
    if (hn > 0) np_mean_std(over + f * A.ld, h0, hn, mean, sd);
    thr[f * A.ld + i] = mean + A.cfg.k_std * sd;
}

// the state machine of one file, time-segmented: segment s scans blocks [s L, (s + 1) L) of its file
// (L = LV_SEGLEN; one wave per segment, every file's segments over the whole GPU).  Segment 0 starts
// from the true initial state (Init); the others from the memoryless Detection state (no lock),
// which is where a file spends most of its time.  After each round every segment whose entry
// differs from its predecessor's exit re-scans from that exit, until no entry changes (normally 2-3
// rounds); the final entries are then exact, and a last pass per segment writes the thresholds used
// and the meteors at offsets from the earlier segments' meteor counts.  A segment's scan: at position
// k lane j evaluates block k + j under the current state; the first block whose event condition holds
// (ballot) is where the state changes, so a 64-block span without events is one step.
// (Rounds 1-5 ran one 16-wave workgroup per file with the rounds inside it: 24 files used 24 CUs,
// 0.65-0.70 ms per day.)
// blocks per segment: 256 against 64 / 128 / 512 / 1024 measured 0.26-0.31 vs 0.55 / 0.34-0.35 /
// 0.31-0.32 / 0.42-0.47 ms per day for the state machine (profiles/r6_live_seglen_ab.txt)
#ifndef LV_SEGLEN_N
#define LV_SEGLEN_N 256
#endif
constexpr int LV_SEGLEN = LV_SEGLEN_N;
#ifndef LV_ROUNDS_N
#define LV_ROUNDS_N 4
#endif
constexpr int LV_ROUNDS = LV_ROUNDS_N;  // rounds launched before the convergence flag is read

__device__ __forceinline__ bool live_same_entry(const LiveScan &x, const LiveScan &y, double t1_first) {
    if (x.state != y.state) return false;
    if (x.state == 2)
        return __builtin_bit_cast(long long, x.lock) == __builtin_bit_cast(long long, y.lock) &&
               __builtin_bit_cast(long long, x.t_start) == __builtin_bit_cast(long long, y.t_start) && x.trig == y.trig;
    if (x.state == 1) {  // a lock that has run out before the first block's end is no lock
        const bool lx = x.until > t1_first, ly = y.until > t1_first;
        if (lx != ly) return false;
        return !lx || (__builtin_bit_cast(long long, x.lock) == __builtin_bit_cast(long long, y.lock) &&
                       __builtin_bit_cast(long long, x.until) == __builtin_bit_cast(long long, y.until));
    }
    return true;
}

struct LiveSegArgs {
    LiveArgs L;
    int64_t smax;  // segments per file slot: ceil(ld / LV_SEGLEN)
};

__device__ __forceinline__ double live_tblk(const msd_live_cfg &C, int64_t i) {
    return (double)(i * (int64_t)C.block_size) / C.fs;
}

// one wave's pass over blocks [a, b) of one file from sc; emit: write the thresholds used and the meteors
__device__ __forceinline__ void live_scan(LiveScan &sc, int64_t a, int64_t b, bool emit, const double *ov, double *th,
                                          const msd_live_cfg &C, msd_meteor *outf, int64_t cap, int lane) {
    int64_t k = a;
    while (k < b) {
        const int64_t kk = k + lane;
        const bool valid = kk < b;
        const int64_t kc = valid ? kk : b - 1;
        const double v = ov[kc], fresh = th[kc], t0 = live_tblk(C, kc), t1 = live_tblk(C, kc + 1);
        double t;
        bool cand;
        if (sc.state == 0) {
            t = fresh;
            cand = t0 >= C.init_wait_sec;
        } else if (sc.state == 1) {
            t = sc.until > t1 ? sc.lock : fresh;
            cand = v > t;
        } else {
            t = sc.lock;
            cand = v < t;
        }
        const uint64_t mask = __ballot(valid && cand);
        const int first = mask ? __builtin_ctzll(mask) : 64;
        if (emit && valid && lane <= first) th[kk] = t;  // thresholds used (processor.py:395-412)
        if (!mask) {
            k += 64;
            continue;
        }
        const int64_t e = k + first;  // event block
        const double te = __shfl(t, first), t0e = __shfl(t0, first);
        if (sc.state == 0) {
            sc.state = 1;
            sc.lock = -1.0;
            sc.until = -1.0;
        } else if (sc.state == 1) {
            sc = live_trigger(sc, ov, e, te, t0e, C.avg_win_blocks);
        } else {
            sc = live_close(sc, ov, e, t0e, C.min_db_mean, C.min_dur_sec, C.after_tracking_wait_sec, outf, cap,
                            emit && lane == 0);
        }
        k = e + 1;
    }
}

// the segments' states: in / out [nfiles][smax] (entry, exit), cnt (meteors), active
struct LiveSegState {
    LiveScan *in, *out;
    int64_t *cnt;
    int32_t *active;
    int32_t *changed;  // [1]: some entry changed in the last link
};

// entries of round 1: Init at each file's start, Detection elsewhere; counts / status of empty files
__global__ __launch_bounds__(256) void live_seg_init_kernel(const int64_t *__restrict__ nblocks, LiveSegArgs A,
                                                            LiveSegState S, int64_t *__restrict__ counts,
                                                            int32_t *__restrict__ status) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= A.L.nfiles * A.smax) return;
    const int64_t f = i / A.smax, s = i - f * A.smax;
    const int64_t nb = nblocks[f];
    LiveScan e0;
    if (s > 0) {
        e0.state = 1;
        e0.lock = -1.0;
        e0.until = -1.0;
    }
    S.in[i] = e0;
    S.active[i] = s * LV_SEGLEN < nb;
    if (s == 0 && nb <= 0) {  // no segment: no meteors
        counts[f] = 0;
        if (status) status[f] = 0;
    }
}

// one wave per active segment: scan from its entry, record its exit and meteor count
__global__ __launch_bounds__(256) void live_seg_scan_kernel(const int64_t *__restrict__ nblocks, LiveSegArgs A,
                                                            LiveSegState S, const double *__restrict__ over,
                                                            double *__restrict__ thr) {
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= A.L.nfiles * A.smax || !S.active[i]) return;  // wave-uniform
    const int lane = threadIdx.x & 63;
    const int64_t f = i / A.smax, s = i - f * A.smax;
    const int64_t nb = nblocks[f];
    const int64_t a = s * LV_SEGLEN, b = a + LV_SEGLEN < nb ? a + LV_SEGLEN : nb;
    LiveScan sc = S.in[i];
    sc.cnt = 0;
    live_scan(sc, a, b, false, over + f * A.L.ld, thr + f * A.L.ld, A.L.cfg, nullptr, 0, lane);
    if (lane == 0) {
        S.out[i] = sc;
        S.cnt[i] = sc.cnt;
    }
}

// a segment whose entry differs from its predecessor's exit re-scans from that exit next round
__global__ __launch_bounds__(256) void live_seg_link_kernel(const int64_t *__restrict__ nblocks, LiveSegArgs A,
                                                            LiveSegState S) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= A.L.nfiles * A.smax) return;
    const int64_t f = i / A.smax, s = i - f * A.smax;
    const int64_t a = s * LV_SEGLEN;
    int act = 0;
    if (s > 0 && a < nblocks[f]) {  // (an empty segment's exit is its entry: its scan does nothing)
        const LiveScan nw = S.out[i - 1];
        if (!live_same_entry(nw, S.in[i], live_tblk(A.L.cfg, a + 1))) {
            S.in[i] = nw;
            act = 1;
            *S.changed = 1;
        }
    }
    S.active[i] = act;
}

// final pass from the exact entries: the thresholds used and the meteors at the offsets of the
// earlier segments' counts; the file's last segment writes its count and status
__global__ __launch_bounds__(256) void live_seg_emit_kernel(const int64_t *__restrict__ nblocks, LiveSegArgs A,
                                                            LiveSegState S, const double *__restrict__ over,
                                                            double *__restrict__ thr, msd_meteor *__restrict__ out,
                                                            int64_t *__restrict__ counts,
                                                            int32_t *__restrict__ status) {
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= A.L.nfiles * A.smax) return;
    const int lane = threadIdx.x & 63;
    const int64_t f = i / A.smax, s = i - f * A.smax;
    const int64_t nb = nblocks[f];
    const int64_t a = s * LV_SEGLEN;
    if (a >= nb) return;  // wave-uniform
    const int64_t b = a + LV_SEGLEN < nb ? a + LV_SEGLEN : nb;
    int64_t off = 0;  // meteors of the file's earlier segments
    for (int64_t j = lane; j < s; j += 64) off += S.cnt[i - s + j];
    for (int o = 32; o > 0; o >>= 1) off += __shfl_xor(off, o, 64);
    LiveScan sc = S.in[i];
    sc.cnt = off;
    live_scan(sc, a, b, true, over + f * A.L.ld, thr + f * A.L.ld, A.L.cfg, out + f * A.L.cap, A.L.cap, lane);
    if (lane == 0 && b == nb) {
        counts[f] = sc.cnt;
        if (status) status[f] = sc.cnt > A.L.cap ? 3 : 0;
    }
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
    A.wave_lds = ((c.nperseg + 1) & ~1) + ((p->nslots + 1) & ~1);
    A.sample_scale = c.sample_scale;
    A.scale = c.scale;
    int slot = 0;
    for (int j = 0; j < c.nbands; ++j) {
        A.band_lo[j] = c.band_lo[j];
        A.band_hi[j] = c.band_hi[j];
        A.band_slot0[j] = slot;
        if (c.band_hi[j] >= c.band_lo[j]) slot += c.band_hi[j] - c.band_lo[j] + 1;
    }
    // waves per workgroup: 4 unless one wave's segment + PSD buffer needs more of the LDS
    // (e.g. nperseg 4096 with a full 2049-bin PSD: 3)
    const size_t wave_bytes = sizeof(double) * (size_t)A.wave_lds;
    const int nw = (int)std::min<size_t>(WL_THREADS / 64, (160 * 1024) / wave_bytes);
    if (nw < 1) return fail(MSD_ERR_UNSUPPORTED, "welch: nperseg + band bins exceed the LDS budget");
    const size_t lds = wave_bytes * nw;
    if (int rc = ensure_dyn_lds(reinterpret_cast<const void *>(welch_bands_kernel<T>), 160 * 1024)) return rc;
    const int64_t grid = (nfiles * max_blocks + nw - 1) / nw;  // a wave per block
    if (grid > 0x7fffffffLL) return fail(MSD_ERR_UNSUPPORTED, "welch: grid too large");
    KernelTimer timer(p->ctx, K_WELCH);
    hipLaunchKernelGGL(welch_bands_kernel<T>, dim3((unsigned)grid), dim3(64 * nw), lds, p->ctx->stream,
                       static_cast<const T *>(x), off, len, A, p->d_window, p->d_bins, band_db, psd);
    MSD_HIP(hipGetLastError());
    return MSD_OK;
}

int launch_welch(msd_welch_plan *p, const void *x, int dtype, const int64_t *off, const int64_t *len, int64_t nfiles,
                 int64_t max_blocks, double *band_db, int64_t ld, double *psd) {
    if (nfiles == 0 || max_blocks == 0) return MSD_OK;
    if (dtype == MSD_I16 && p->d_i8 && !p->ctx->welch_goertzel)  // the exact integer DFT (welch_i8.hip)
        return launch_welch_i8(p, static_cast<const int16_t *>(x), off, len, nfiles, max_blocks, band_db, ld, psd);
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
    if (ld > 0) {  // grid width: the leading dimension bounds every file's block count
        const dim3 grid((unsigned)((ld + WL_THREADS - 1) / WL_THREADS), (unsigned)nfiles);
        hipLaunchKernelGGL(live_over_kernel, grid, dim3(WL_THREADS), 0, ctx->stream, band_db, nblocks, A, over);
        hipLaunchKernelGGL(live_history_kernel, grid, dim3(WL_THREADS), 0, ctx->stream, nblocks, A, over, thr);
    }
    LiveSegArgs G{};
    G.L = A;
    G.smax = ld > 0 ? (ld + LV_SEGLEN - 1) / LV_SEGLEN : 1;
    const int64_t nseg = nfiles * G.smax;
    const size_t b_state = sizeof(LiveScan) * (size_t)nseg, b_cnt = sizeof(int64_t) * (size_t)nseg,
                 b_act = sizeof(int32_t) * (size_t)nseg;
    void *sp = nullptr;
    if (int rc = ctx_scratch(ctx, 6, 2 * b_state + b_cnt + b_act + 64, &sp)) return rc;
    char *base = static_cast<char *>(sp);
    LiveSegState S;
    S.in = reinterpret_cast<LiveScan *>(base);
    S.out = reinterpret_cast<LiveScan *>(base + b_state);
    S.cnt = reinterpret_cast<int64_t *>(base + 2 * b_state);
    S.active = reinterpret_cast<int32_t *>(base + 2 * b_state + b_cnt);
    S.changed = reinterpret_cast<int32_t *>(base + 2 * b_state + b_cnt + b_act);
    if (nseg > 0x7fffffffLL) return fail(MSD_ERR_UNSUPPORTED, "live: too many segments");
    const unsigned g_thr = (unsigned)((nseg + 255) / 256), g_wave = (unsigned)((nseg + 3) / 4);
    hipStream_t st = ctx->stream;
    hipLaunchKernelGGL(live_seg_init_kernel, dim3(g_thr), dim3(256), 0, st, nblocks, G, S, counts, status);
    // rounds: scan the active segments, then link every segment to its predecessor's exit.  The
    // first LV_ROUNDS go out unchecked (segments with nothing to do exit at once); then the flag of
    // the last link is read, and more rounds follow while it is set
    for (int64_t r = 0;; ++r) {
        hipLaunchKernelGGL(live_seg_scan_kernel, dim3(g_wave), dim3(256), 0, st, nblocks, G, S, over, thr);
        MSD_HIP(hipMemsetAsync(S.changed, 0, sizeof(int32_t), st));
        hipLaunchKernelGGL(live_seg_link_kernel, dim3(g_thr), dim3(256), 0, st, nblocks, G, S);
        if (r + 1 < LV_ROUNDS) continue;
        int32_t changed = 0;
        MSD_HIP(hipMemcpyAsync(&changed, S.changed, sizeof(int32_t), hipMemcpyDeviceToHost, st));
        MSD_HIP(hipStreamSynchronize(st));
        if (!changed) break;
        if (r > G.smax + LV_ROUNDS) return fail(MSD_ERR_HIP, "live: segment states did not converge");
    }
    hipLaunchKernelGGL(live_seg_emit_kernel, dim3(g_wave), dim3(256), 0, st, nblocks, G, S, over, thr, out, counts,
                       status);
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
    if (welch_i8_shape(c, p->nseg, nslots, window)) {  // int16 samples on the matrix cores
        if (int rc = welch_i8_build(p, window)) {
            msd_welch_plan_destroy(p);
            return rc;
        }
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
    if (p->d_i8) (void)hipFree(p->d_i8);
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

int msd_welch_psd(msd_welch_plan *p, const void *x, int dtype, int64_t n, double *psd, int64_t *blocks) {
    if (!p || (!x && n) || !psd) return fail(MSD_ERR_INVALID, "msd_welch_psd: null");
    const size_t es = dtype_size(dtype);
    if (!es) return fail(MSD_ERR_INVALID, "msd_welch_psd: unknown dtype");
    const int64_t B = p->cfg.block_size;
    const int64_t nb = n >= B ? (n - B) / B + 1 : 0;
    if (blocks) *blocks = nb;
    if (nb == 0) return MSD_OK;
    msd_ctx *ctx = p->ctx;
    DeviceGuard g(ctx->device);
    void *dx, *dmeta, *dout;
    int rc;
    const int nbands = p->cfg.nbands;
    const size_t band_bytes = sizeof(double) * nbands * nb, psd_bytes = sizeof(double) * (size_t)p->nslots * nb;
    if ((rc = ctx_scratch(ctx, 0, ((size_t)n * es + 255) / 256 * 256, &dx))) return rc;
    if ((rc = ctx_scratch(ctx, 1, 64, &dmeta))) return rc;
    if ((rc = ctx_scratch(ctx, 2, band_bytes + psd_bytes, &dout))) return rc;
    int64_t meta[2] = {0, n};
    MSD_HIP(hipMemcpyAsync(dx, x, (size_t)n * es, hipMemcpyHostToDevice, ctx->stream));
    MSD_HIP(hipMemcpyAsync(dmeta, meta, sizeof(meta), hipMemcpyHostToDevice, ctx->stream));
    const int64_t *doff = static_cast<const int64_t *>(dmeta);
    double *dband = static_cast<double *>(dout);
    double *dpsd = reinterpret_cast<double *>(static_cast<char *>(dout) + band_bytes);
    rc = launch_welch(p, dx, dtype, doff, doff + 1, 1, nb, dband, nb, dpsd);
    if (rc) return rc;
    MSD_HIP(hipMemcpyAsync(psd, dpsd, psd_bytes, hipMemcpyDeviceToHost, ctx->stream));
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
