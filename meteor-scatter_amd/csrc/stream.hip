// C5: the reference's threshold detectors over ONE long stream (a 24 h I/Q recording whose STFT
// frames are the detector's blocks), time-sharded over ranks.  get_detections_adaptive()
// dsp/src/main.py:450-522 and get_detections() :396-448, float64, numpy-exact.
//
// Per rank (one shard of the stream's frames), all on the context stream:
//   iq_band_delta_kernel   frame-major spectrogram [T][N] -> band / noise dB, delta (main.py:380-393)
//   chunk_sums_kernel      numpy's add.reduce over the whole stream is s = 0.0; s += pairwise(chunk)
//                          for 8192-element chunks in order: each wave sums one chunk that starts
//                          in the shard (wave_chunk_sum: each lane follows its bits down numpy's
//                          recursion, the tree folds back with xor shuffles); the host adds the
//                          chunk sums of all ranks in order
//   fresh_kernel           mean + k*std(delta[i-W:i]) for every frame i >= W.  The pairwise tree of
//                          a W-element window has the same shape for every i, so the host turns it
//                          into a program (leaf / add / chunk-end ops) that every lane runs on its
//                          own 8 consecutive frames: one LDS element feeds 8 frames' accumulators
//                          (register blocking), the leaves stream through double-buffered LDS
//   fresh_short_kernel     frames i < W (windows delta[0:i], a different tree per frame)
//   approx_kernel          every frame's threshold from prefix sums (the predictor) and, in
//                          decisions-only mode, a rounding-error bound on |predicted - numpy|
//   fresh_list_kernel      decisions-only mode: numpy-exact thresholds of the frames the scan
//                          listed (near ties, triggers), one wave per frame
//   scan_kernel            the freeze/run state machine, one wave per segment: lane j evaluates
//                          frame pos+j; with the freeze state fixed the decisions of 64 frames are
//                          two ballots (fresh threshold / held threshold), and only the frames
//                          where the freeze state changes are walked in scalar code
//   propagate_kernel       segment s+1 re-enters with segment s's exit state; repeated to a
//                          fixed point (normally 2 rounds: speculative clean start, then fix-up)
//   runs_kernel, db_kernel the shard's runs (merged over segment edges) and np.mean dB of each
// FP contraction is off: numpy rounds every add / multiply separately.
#include "msd_internal.h"
#include "np_program.h"
#include "np_reduce.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#pragma clang fp contract(off)

struct msd_stream_plan {
    msd_ctx *ctx = nullptr;
    msd_det_cfg cfg{};
    int64_t n_total = 0, frame0 = 0, n_local = 0;
    int64_t n_tail = 0, n_head = 0, head_cap = 0;
    int64_t seg_len = 0, nseg = 0, cap = 0;
    double *d_x = nullptr;      // [n_tail | n_local | head_cap] delta of the stream around the shard
    double *d_fresh = nullptr;  // [n_local]
    double *d_thr = nullptr;    // [n_local] thresholds used (scan output)
    void *d_state = nullptr;    // in[nseg], out[nseg] states
    int32_t *d_active = nullptr;  // [nseg] + changed counter + overflow flag
    msd_det *d_runs = nullptr;  // [nseg][cap]
    int32_t *d_nruns = nullptr; // [nseg]
    double *d_margin = nullptr; // [nseg]
    msd_det *d_out = nullptr;   // compacted runs [nseg*cap]
    int64_t *d_count = nullptr;
    int64_t *d_pos = nullptr;   // [nseg] runs emitted before each segment
    double *d_chunks = nullptr; // chunk sums [nchunk] + the local path's mean, thr0
    int4 *d_prog = nullptr;     // fresh-threshold leaf records for windows of exactly W frames
    int32_t *d_need = nullptr;  // [ntiles] a scan used fresh thresholds in the tile
    int32_t *d_done = nullptr;  // [ntiles] the tile's exact thresholds are computed (+1: counter)
    double2 *d_pre = nullptr;   // [nblk + 1] prefix sums of x, x^2 (the predictor)
    // decisions-only mode (msd_stream_set_exact_thresholds(plan, 0)): exact thresholds per frame,
    // only where a decision or a held threshold depends on them
    double *d_eps = nullptr;      // [n_local] bound on |predicted - numpy threshold|
    uint8_t *d_exact = nullptr;   // [n_local] fresh[j] is numpy-exact
    int32_t *d_list = nullptr;    // [n_local] frames the last marking pass needs exact
    bool decide = false;
    // certification against the float64 reference (msd_stream_set_certify): a bound on |delta -
    // delta_ref| per frame, the thresholds' error from it, and per segment the decisions the bounds
    // cannot settle
    bool certify = false;
    double *d_ed = nullptr;       // [n_tail | n_local | head_cap] delta error bound (as d_x)
    double *d_terr = nullptr;     // [n_local] bound on |numpy threshold(delta) - numpy threshold(delta_ref)|
    double2 *d_pre_e = nullptr;   // [nblk + 1] prefix sums of (ed, ed^2)
    longlong2 *d_unc = nullptr;   // [nseg][UCAP] uncertain decisions {local frame, threshold source frame}
    int32_t *d_ucnt = nullptr;    // [nseg] uncertain decisions of the segment's last scan
    double2 *d_slack = nullptr;   // [nseg] min over the segment of |delta - thr| - (ed + threshold error), max of
                                  // ed + threshold error
    double2 *d_esum = nullptr;    // [nchunk + 1] per-chunk (sum ed, sum ed^2), then the shard's total
    double terr0 = 0.0;           // bound for thr0 (whole-stream mean + k std)
    int64_t ntiles = 0, nblk = 0;
    int nleaf = 0;
    double thr0 = 0;
    bool scanned = false;
    // every segment's certificate entries (d_ucnt, d_slack) come from a scan that ran with
    // certification on: set by a scan over all segments with certify on, cleared by
    // msd_stream_set_certify and by any scan with it off (a stale or never-written certificate
    // must not read as "certified")
    bool cert_valid = false;
    bool cert_staged = false;  // the certificate's counts / slacks already in h_cert (detect_local)
    bool want_exact = true;  // msd_stream_set_exact_thresholds
    int32_t listed = -1;     // decisions only: frames listed by the last msd_stream_scan (host copy)
    // pinned host block for the small per-step readbacks (counters, exit state, margins, chunk
    // sums): the copies are asynchronous DMA and a decision point costs one stream sync, where a
    // pageable destination costs a staged, host-synchronous copy each (≈ 18 µs per copy in the C5
    // step's timeline)
    void *h_pin = nullptr;
    void *h_cert = nullptr;  // pinned staging of msd_stream_certificate
    size_t h_cert_bytes = 0;
};

namespace msd {
namespace {

constexpr int64_t CHUNK = NP_BUFSIZE;  // numpy's reduction buffer (8192 elements)

struct SState {  // msd_stream_state
    int64_t fz, last_stop;
    double thr;
    int64_t src;  // frame whose threshold `thr` is (-1: thr0)
    double terr;  // its error bound against the reference's (certification)
};
constexpr int UCAP = 32;  // uncertain decisions listed per segment and scan

struct PinHdr {  // head of msd_stream_plan::h_pin, then margins [nseg], then chunk sums
    int32_t changed, overflow;  // copied from d_active[nseg .. nseg + 1]
    int32_t listed, computed;
    int64_t count;
    SState ex;
};


// ---- the delta error bound of the fp32 spectrogram path (C5): |delta_gpu - delta_ref| <= ed for
// the float64 reference (scipy.signal.spectrogram of complex128 input, its band sums and dB).
// Standard model, per bin: the computed spectrum X^ of a linear FFT satisfies
// |X^_k - X_k| <= c u sum_n |v_n| with c the longest rounding chain from an input to an output
// (in units of u) and v the detrended, windowed frame: every operation multiplies the path terms
// through it by (1 + theta), |theta| <= u for an add, <= 2 sqrt 2 u for a complex multiply with FMA
// and sqrt 2 u more for a rounded twiddle, and each input reaches each bin by one path of unit
// weight.  cstft4096_kernel: detrend, window and its rounding (3), three passes of a 16-point DFT
// (radix-4 x 4: 2 + 2 adds and an internal twiddle multiply, 4 + 2.83 + 1.41 = 8.24 each) and the
// two inter-pass twiddles (4.24 each): 36.2, taken as IQ_CHAIN = 37 (second-order terms).  sum |v| <= sqrt(N) ||v||_2 =
// sqrt(S) with S = sum_k |X_k|^2 (Parseval), S from the kernel's energy partials (an upper bound
// after the factor 1.001: their own rounding is ~1e-4 relative).  The reference's float64 chain
// (pocketfft, 4 log2 N + 8, + 3 for detrend / window) adds its own, ~1e-9 of ours.  A band of n
// bins with computed energy E (fp64 sum of the fp32 powers, each |x|^2 + |y|^2 rounded twice)
// moves by dE <= 2 d sqrt(n E) + 3 n d^2 + (n + 4) u E, its dB by 10/ln 10 * dE / (E + 1e-12 - dE)
// (unbounded once dE >= E); delta by the sum of the two bands'.  A band touching bins -1..1 also
// carries the frame mean's rounding (the DC offset's transform): not bounded here, +inf.
constexpr double IQ_CHAIN = 37.0;

__device__ __forceinline__ double band_db_bound(double E, int n, double d) {
    if (n <= 0) return 0.0;  // empty band: 1e-12 on both sides
    const double u = 0x1p-24;
    const double dE = 2.0 * d * sqrt((double)n * E) + 3.0 * (double)n * d * d + ((double)n + 4.0) * u * E;
    const double den = E + 1e-12 - dE;
    if (!(den > 0.0)) return __builtin_inf();
    return 4.342944819032518 * dE / den * (1.0 + 1e-12);
}

__device__ __forceinline__ bool near_dc(int lo, int hi) { return hi >= lo && lo <= 1 && hi >= -1; }

// ------------------------------------------------------------------ band delta per frame
// one thread per frame: the band bins of a frame are one or two short contiguous runs of its row
// (~100-400 B), so a thread's loads are few and independent; thousands of frames in flight hide
// the latency.  Sums in float64, ascending bin order.
__device__ __forceinline__ double band_energy(const float *__restrict__ row, int N, int lo, int hi) {
    double acc = 0.0;
    for (int k = lo; k <= hi; ++k) acc += (double)__builtin_nontemporal_load(row + (k < 0 ? k + N : k));
    return acc;
}

// the same sum through 16-B loads of the aligned float4 chunks covering the band (fewer, wider
// memory instructions; same elements, same ascending order: C5's 0.21 → 0.13 ms).  A band across
// 0 Hz (its bins at both ends of the row) takes the scalar loop.
__device__ __forceinline__ double band_energy4(const float *__restrict__ row, int N, int lo, int hi) {
    if (hi < lo) return 0.0;
    if (lo < 0 && hi >= 0) return band_energy(row, N, lo, hi);
    const int ulo = lo < 0 ? lo + N : lo, uhi = hi < 0 ? hi + N : hi;
    double acc = 0.0;
    typedef float f4v __attribute__((ext_vector_type(4)));
    for (int c = ulo & ~3; c <= uhi; c += 4) {
        const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v *>(row + c));
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (c + e >= ulo && c + e <= uhi) acc += (double)v[e];
    }
    return acc;
}

// etot / ed (both or neither): the frame's 16 energy partials (cstft4096_kernel<EN>, [16][stride]) in,
// the delta error bound out (above)
__global__ __launch_bounds__(256) void iq_band_delta_kernel(const float *__restrict__ spec, int64_t nstreams,
                                                            int64_t max_frames, const int64_t *__restrict__ frames,
                                                            int N, int blo, int bhi, int nlo, int nhi,
                                                            double *__restrict__ band_db,
                                                            double *__restrict__ noise_db,
                                                            double *__restrict__ delta, int64_t ld,
                                                            const float *__restrict__ etot, double *__restrict__ ed) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nstreams * max_frames) return;
    const int64_t s = g / max_frames, t = g - s * max_frames;
    if (t >= frames[s]) return;
    const float *row = spec + (s * max_frames + t) * (int64_t)N;
    const double e0 = band_energy4(row, N, blo, bhi), e1 = band_energy4(row, N, nlo, nhi);
    const double bd = 10.0 * log10(e0 + 1e-12), nd = 10.0 * log10(e1 + 1e-12);
    if (band_db) band_db[s * ld + t] = bd;
    if (noise_db) noise_db[s * ld + t] = nd;
    delta[s * ld + t] = bd - nd;
    if (ed) {
        const int64_t es = (nstreams * max_frames + 3) / 4 * 4;  // msd_cstft_energy_stride
        double S = 0.0;
#pragma unroll
        for (int q = 0; q < 16; ++q) S += (double)__builtin_nontemporal_load(etot + q * es + s * max_frames + t);
        const double A = sqrt(S * 1.001);
        const double lg = log2((double)N);
        const double d = IQ_CHAIN * 0x1p-24 * A + (4.0 * lg + 11.0) * 0x1p-53 * sqrt((double)N) * A;
        double b = band_db_bound(e0, bhi - blo + 1, d) + band_db_bound(e1, nhi - nlo + 1, d);
        if (near_dc(blo, bhi) || near_dc(nlo, nhi) || !(S >= 0.0)) b = __builtin_inf();
        ed[s * ld + t] = b + 1e-12;
    }
}

// numpy's pairwise sum of one chunk a(cb .. cb+m), m <= 8192, by one wave.  Lane L follows the
// path of its 6 bits down numpy's recursion (bit 5 first: 0 = left half); the node where the path
// stops (a leaf of <= 128, or depth 6) is summed by the lane whose remaining bits are zero; the
// tree is then folded bottom-up with xor shuffles, adding only across nodes that were split.
// IEEE addition commutes, so left + right in either order gives numpy's bits.
template <typename A>
__device__ __forceinline__ double wave_chunk_sum(const A &a, int64_t cb, int64_t m) {
#pragma clang fp contract(off)
    const int L = threadIdx.x & 63;
    int64_t base = 0, size = m;
    int D = 6;  // depth of this lane's node
    for (int d = 0; d < 6; ++d) {
        if (size <= 128) {
            D = d;
            break;
        }
        int64_t n2 = size / 2;
        n2 -= n2 % 8;
        if ((L >> (5 - d)) & 1) {
            base += n2;
            size -= n2;
        } else {
            size = n2;
        }
    }
    const bool canon = (L & ((1 << (6 - D)) - 1)) == 0;
    double v = canon ? np_pairwise_rec<2>(a, cb + base, size) : 0.0;
    for (int d = 5; d >= 0; --d) {  // node at depth d split iff this lane's path went deeper
        const double o = __builtin_bit_cast(double, __shfl_xor(__builtin_bit_cast(long long, v), 1 << (5 - d), 64));
        if (D > d) v = v + o;
    }
    return __builtin_bit_cast(double, __shfl(__builtin_bit_cast(long long, v), 0, 64));
}

// np.sum of a(base .. base+n): s = 0.0; s += pairwise(chunk) over 8192-element chunks.  Inline: out of
// line, with the window read through global loads (GSqDevRef), the callee took 148 VGPRs and its
// callers 3 waves per SIMD instead of 4 -- the decisions-only fresh thresholds 5.1-5.5 -> 7.8-8.0 ms
// beside the C5 spectrogram, the step 11.7 -> 12.7 ms (profiles/r6_c5_fresh_inline_ab.txt)
template <typename A>
__device__ __forceinline__ double wave_np_sum(const A &a, int64_t base, int64_t n) {
#pragma clang fp contract(off)
    double s = 0.0;
    for (int64_t c = 0; c < n; c += NP_BUFSIZE) s += wave_chunk_sum(a, base + c, n - c < NP_BUFSIZE ? n - c : NP_BUFSIZE);
    return s;
}

// ------------------------------------------------------------------ chunk sums
// x: the stream around the shard (x[j] = frame x0 + j); chunk c covers frames [8192c, min(8192(c+1),
// n_total)).  One wave per chunk that starts in the shard.
template <bool SQ>
__global__ __launch_bounds__(256) void chunk_sums_kernel(const double *__restrict__ x, int64_t x0,
                                                         int64_t first_chunk, int64_t nchunks, int64_t n_total,
                                                         double mean_v, const double *__restrict__ mean_ptr,
                                                         double *__restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= nchunks) return;
    const double mean = mean_ptr ? *mean_ptr : mean_v;  // the local path keeps the mean on the device
    const int64_t g = (first_chunk + c) * CHUNK;
    const int64_t m = n_total - g < CHUNK ? n_total - g : CHUNK;
    const double *p = x + (g - x0);
    const double r = SQ ? wave_chunk_sum(GSqDevRef{as_global(p), mean}, 0, m) : wave_chunk_sum(GArrRef{as_global(p)}, 0, m);
    if (lane == 0) out[c] = r;
}

// the whole stream's np.mean / thr0 from its chunk sums, as the host forms them (s = 0.0; s += chunk
// sum, in order; mean = s / n; thr0 = mean + k * sqrt(s2 / n)), for the one-process path: no host
// round trip between the two passes.  stats[0] = mean (STAGE 0), stats[1] = thr0 (STAGE 1).
__global__ __launch_bounds__(256) void fresh_clear_kernel(int32_t *__restrict__ need, int64_t n_need, int32_t need_v,
                                                          int32_t *__restrict__ done, int64_t n_done,
                                                          uint8_t *__restrict__ exact, int64_t n_exact) {
    const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = i0; i < n_need; i += step) need[i] = need_v;
    for (int64_t i = i0; i < n_done; i += step) done[i] = 0;
    if (exact) {
        uint32_t *e4 = reinterpret_cast<uint32_t *>(exact);  // hipMalloc'd: 4-B aligned
        for (int64_t i = i0; i < n_exact / 4; i += step) e4[i] = 0u;
        for (int64_t i = (n_exact / 4) * 4 + i0; i < n_exact; i += step) exact[i] = 0;
    }
}

// The 256 threads stage the sums in LDS (independent loads), thread 0 adds them in order.
template <int STAGE>
__global__ __launch_bounds__(256) void stream_stats_kernel(const double *__restrict__ sums, int64_t nc, int64_t n,
                                                           double k, double *__restrict__ stats) {
    __shared__ double sh[2048];
    double s = 0.0;
    for (int64_t b = 0; b < nc; b += 2048) {
        const int64_t m = nc - b < 2048 ? nc - b : 2048;
        for (int64_t i = threadIdx.x; i < m; i += 256) sh[i] = sums[b + i];
        __syncthreads();
        if (threadIdx.x == 0)
            for (int64_t i = 0; i < m; ++i) s += sh[i];
        __syncthreads();
    }
    if (threadIdx.x != 0) return;
    if (STAGE == 0) stats[0] = s / (double)n;
    else stats[1] = stats[0] + k * sqrt(s / (double)n);
}

// ------------------------------------------------------------------ fresh thresholds
// the program: one record per leaf of numpy's tree over a W-element window, in order,
// {offset, length (<= 128), adds that follow it, 1 if a chunk ends after them}
constexpr int FR_MAXREC_LDS = 512;  // records kept in LDS (W up to ~32K); more are read from HBM

constexpr int FR_THREADS = 64;                   // a workgroup computes one tile
constexpr int FR_F = 8;                          // frames per lane
constexpr int FR_FRAMES = FR_THREADS * FR_F;     // frames per tile
constexpr int FR_STAGE = FR_FRAMES + 128;        // staged elements per leaf (leaf <= 128)
// pad (conflict-free 16-B LDS reads): 2 doubles per 8
constexpr int FR_PADDED = FR_STAGE + FR_STAGE / 4;
constexpr int FR_LOADS = (FR_STAGE + FR_THREADS - 1) / FR_THREADS;
constexpr int FR_DEPTH = 7;

__device__ __forceinline__ int padded(int q) { return q + 2 * (q >> 3); }

struct FreshParams {
    int64_t n_local, frame0, n_tail, x_len, W, F0;
    double k;
    int nleaf;
    int64_t pre_per;  // prefix blocks per thread of blockscan_kernel (error bound of the predictor)
    double eps_scale; // test hook (MSD_STREAM_EPS_SCALE): widens the bound, more frames made exact
};

// record i of the program through a pointer typed with its address space (LDS or global int32s, so
// that the loads are ds_read / global_load, never flat: np_reduce.h)
template <typename IntPtr>
__device__ __forceinline__ int4 load_rec(IntPtr recs, int i) {
    return make_int4(recs[4 * i], recs[4 * i + 1], recs[4 * i + 2], recs[4 * i + 3]);
}

// one pass of the program over this lane's 8 frames: out[f] = numpy np.sum of the window of frame f
// (SQ: of (x - mean[f])^2)
template <bool SQ, typename RecPtr>
__device__ __forceinline__ void fresh_pass(const double *__restrict__ x, int64_t xbase, int64_t x_len,
                                           RecPtr recs, int nleaf, double *stage,
                                           const double (&mean)[FR_F], double (&out)[FR_F]) {
    const int tid = threadIdx.x;
    // 8 frames: the pending partial sums live in scratch (a runtime-indexed array; 8 x 7 doubles
    // would not fit beside the 64 accumulators), touched once per leaf / add
    double stk_[FR_DEPTH + 1][FR_F];
    int sp = 0;
    auto top = [&](int d, int f) -> double & { return stk_[sp - 1 - d][f]; };
    auto push = [&](const double (&v)[FR_F]) {
#pragma unroll
        for (int f = 0; f < FR_F; ++f) stk_[sp][f] = v[f];
        ++sp;
    };
    auto pop = [&]() {  // removes stk[0] after an add folded it into stk[1] (or into acc)
        --sp;
    };
    auto add_top = [&]() {
#pragma unroll
        for (int f = 0; f < FR_F; ++f) top(1, f) = top(1, f) + top(0, f);
        pop();
    };
    double acc[FR_F];
#pragma unroll
    for (int f = 0; f < FR_F; ++f) acc[f] = 0.0;

    // prefetch registers for the next leaf's stage
    double pre[FR_LOADS];
    auto fetch = [&](int off) {
#pragma unroll
        for (int j = 0; j < FR_LOADS; ++j) {
            const int q = tid + j * FR_THREADS;
            int64_t idx = xbase + off + q;
            idx = idx < 0 ? 0 : (idx >= x_len ? x_len - 1 : idx);
            pre[j] = q < FR_STAGE ? x[idx] : 0.0;
        }
    };
    auto commit = [&](double *buf) {
#pragma unroll
        for (int j = 0; j < FR_LOADS; ++j) {
            const int q = tid + j * FR_THREADS;
            if (q < FR_STAGE) buf[padded(q)] = pre[j];
        }
    };
    int buf = 0;
    int4 cur = load_rec(recs, 0);
    fetch(cur.x);
    commit(stage);
    __syncthreads();
    for (int li = 0; li < nleaf; ++li) {
        // prefetch the following leaf while this one is summed
        const bool has_next = li + 1 < nleaf;
        const int4 nxt = has_next ? load_rec(recs, li + 1) : cur;
        if (has_next) fetch(nxt.x);
        const int len = cur.y;
        const double *st = stage + buf * FR_PADDED;
        const int l8 = tid * FR_F;  // this lane's first element (frame f reads st[l8 + f + m])
        auto elem = [&](int q) -> double { return st[padded(l8 + q)]; };
        double res[FR_F];
        if (len >= 8) {
            const int lim = len - (len & 7);
            const int G = lim >> 3;  // groups 0..G (G+1 groups: frame f spans q in [f, f+lim))
            double r[FR_F][8];
#pragma unroll
            for (int f = 0; f < FR_F; ++f)
#pragma unroll
                for (int k = 0; k < 8; ++k) r[f][k] = SQ ? 0.0 : -0.0;  // squares are >= +0: +0.0 is exact
            auto group = [&](int g, auto first, auto last) {
                double v[8];
                if constexpr (FR_F == 8) {
                    const double2 *vp = reinterpret_cast<const double2 *>(st + padded(l8 + 8 * g));
#pragma unroll
                    for (int h = 0; h < 4; ++h) {
                        const double2 t = vp[h];
                        v[2 * h] = t.x;
                        v[2 * h + 1] = t.y;
                    }
                } else {
#pragma unroll
                    for (int h = 0; h < 8; ++h) v[h] = st[padded(l8 + 8 * g + h)];
                }
#pragma unroll
                for (int f = 0; f < FR_F; ++f) {
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        if constexpr (decltype(first)::value) {
                            if (k < f) continue;
                        }
                        if constexpr (decltype(last)::value) {
                            if (k >= f) continue;
                        }
                        if constexpr (SQ) {
                            const double d = v[k] - mean[f];
                            r[f][(k - f) & 7] += d * d;
                        } else {
                            r[f][(k - f) & 7] += v[k];
                        }
                    }
                }
            };
            using T_ = std::integral_constant<bool, true>;
            using F_ = std::integral_constant<bool, false>;
            group(0, T_{}, F_{});
            for (int g = 1; g < G; ++g) group(g, F_{}, F_{});
            group(G, F_{}, T_{});
#pragma unroll
            for (int f = 0; f < FR_F; ++f) res[f] = ((r[f][0] + r[f][1]) + (r[f][2] + r[f][3])) +
                                                     ((r[f][4] + r[f][5]) + (r[f][6] + r[f][7]));
            for (int t = lim; t < len; ++t) {
#pragma unroll
                for (int f = 0; f < FR_F; ++f) {
                    const double v = elem(f + t);
                    if constexpr (SQ) {
                        const double d = v - mean[f];
                        res[f] += d * d;
                    } else {
                        res[f] += v;
                    }
                }
            }
        } else {
#pragma unroll
            for (int f = 0; f < FR_F; ++f) res[f] = -0.0;
            for (int t = 0; t < len; ++t) {
#pragma unroll
                for (int f = 0; f < FR_F; ++f) {
                    const double v = elem(f + t);
                    if constexpr (SQ) {
                        const double d = v - mean[f];
                        res[f] += d * d;
                    } else {
                        res[f] += v;
                    }
                }
            }
        }
        push(res);
        for (int a = 0; a < cur.z; ++a) add_top();  // the adds after the leaf: left + right
        if (cur.w) {  // chunk end: s += pairwise(chunk)
#pragma unroll
            for (int f = 0; f < FR_F; ++f) acc[f] = acc[f] + top(0, f);
            pop();
        }
        if (has_next) {
            commit(stage + (buf ^ 1) * FR_PADDED);
            buf ^= 1;
        }
        __syncthreads();
        cur = nxt;
    }
#pragma unroll
    for (int f = 0; f < FR_F; ++f) out[f] = acc[f];
}

// exact thresholds of the 512-frame tiles a scan used fresh thresholds in (need) and that are
// not computed yet (done); the others keep the predictor's values, which no final scan reads
__global__ __launch_bounds__(FR_THREADS) void fresh_kernel(const double *__restrict__ x, FreshParams P,
                                                           const int4 *__restrict__ prog,
                                                           double *__restrict__ fresh, const int32_t *__restrict__ need,
                                                           int32_t *__restrict__ done, int32_t *__restrict__ count) {
    __shared__ __attribute__((aligned(16))) double stage[2 * FR_PADDED];
    const int64_t wg = blockIdx.x;
    if (!need[wg] || done[wg]) return;
    if (threadIdx.x == 0) {
        done[wg] = 1;
        atomicAdd(count, 1);
    }
    if (P.frame0 + (wg + 1) * FR_FRAMES - 1 < P.W) return;  // short windows only: exact already
    const int64_t j0 = wg * FR_FRAMES + threadIdx.x * FR_F;  // this lane's first local frame
    // element m of the window of local frame j sits at x[n_tail + j - W + m]
    const int64_t xbase = P.n_tail + wg * FR_FRAMES - P.W;
    double mean[FR_F], s[FR_F];
#pragma unroll
    for (int f = 0; f < FR_F; ++f) mean[f] = 0.0;
    __shared__ int4 s_rec[FR_MAXREC_LDS];
    const bool in_lds = P.nleaf <= FR_MAXREC_LDS;
    if (in_lds)
        for (int i = threadIdx.x; i < P.nleaf; i += FR_THREADS) s_rec[i] = prog[i];
    __syncthreads();
    // the two passes instantiated on the LDS copy and on global memory, never on a pointer that may
    // be either (a generic pointer is read with flat instructions: np_reduce.h)
    // (typed pointers: the compiler may merge the two copies, but not loads of different address spaces)
    auto passes = [&](auto recs) {
        fresh_pass<false>(x, xbase, P.x_len, recs, P.nleaf, stage, mean, s);
#pragma unroll
        for (int f = 0; f < FR_F; ++f) mean[f] = s[f] / (double)P.W;
        fresh_pass<true>(x, xbase, P.x_len, recs, P.nleaf, stage, mean, s);
    };
    if (in_lds) passes((const __attribute__((address_space(3))) int *)s_rec);
    else passes((const __attribute__((address_space(1))) int *)prog);
#pragma unroll
    for (int f = 0; f < FR_F; ++f) {
        const int64_t j = j0 + f;
        const int64_t i = P.frame0 + j;
        if (j < P.n_local && i >= P.W && i >= P.F0) {
            const double sd = sqrt(s[f] / (double)P.W);
            fresh[j] = mean[f] + P.k * sd;
        }
    }
}

// ---- the predictor: mean + k*std of every window from prefix sums of x and x^2 (not numpy's
// rounding; it only tells the first scan which tiles need exact thresholds)
constexpr int PB = 256;  // elements per prefix block
// one wave per prefix block: each lane sums 4 elements, then an xor-shuffle tree (<= 10 additions
// per element, within the predictor's error bound)
__global__ __launch_bounds__(256) void blocksum_kernel(const double *__restrict__ x, int64_t x_len, int64_t nblk,
                                                       double2 *__restrict__ blk) {
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= nblk) return;
    double s = 0.0, q = 0.0;
#pragma unroll
    for (int r = 0; r < PB / 64; ++r) {
        const int64_t i = b * PB + r * 64 + lane;
        const double v = i < x_len ? x[i] : 0.0;
        s += v;
        q += v * v;
    }
    for (int o = 32; o > 0; o >>= 1) {
        s += __shfl_xor(s, o, 64);
        q += __shfl_xor(q, o, 64);
    }
    if (lane == 0) blk[b] = make_double2(s, q);
}

// exclusive prefix over the blocks, in place, one workgroup
__global__ __launch_bounds__(1024) void blockscan_kernel(double2 *__restrict__ blk, int64_t nblk) {
    __shared__ double2 tot[1024];
    const int tid = threadIdx.x;
    const int64_t per = (nblk + 1023) / 1024;
    const int64_t b0 = tid * per, b1 = b0 + per < nblk ? b0 + per : nblk;
    double2 acc = make_double2(0.0, 0.0);
    for (int64_t b = b0; b < b1; ++b) acc = make_double2(acc.x + blk[b].x, acc.y + blk[b].y);
    tot[tid] = acc;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const double2 v = tid >= o ? tot[tid - o] : make_double2(0.0, 0.0);
        __syncthreads();
        tot[tid] = make_double2(tot[tid].x + v.x, tot[tid].y + v.y);
        __syncthreads();
    }
    double2 run = tid > 0 ? tot[tid - 1] : make_double2(0.0, 0.0);
    for (int64_t b = b0; b < b1; ++b) {
        const double2 v = blk[b];
        blk[b] = run;
        run = make_double2(run.x + v.x, run.y + v.y);
    }
}

// eps (decisions-only mode): a bound on |predicted - numpy's threshold| from the rounding-error
// bounds of both (u = 2^-53; an element passes through at most d additions: |error of a sum| <=
// d u sum|x|, with sum|x| <= sqrt(len sum x^2)), times 4.  Frames whose |delta - predicted| exceeds it
// are decided exactly by the prediction.  NaN anywhere gives a NaN bound, which the scan treats as a
// near tie (exact threshold computed).
__device__ __forceinline__ double sd_err(double e, double sig_lo) {  // |sqrt(a) - sigma| given |a - sigma^2| <= e
    const double r = sqrt(e);
    return sig_lo > 0.0 ? fmin(r, e / sig_lo) : r;
}

__device__ __forceinline__ double2 d2add(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }

// exclusive block scan (256 threads, Hillis-Steele in LDS) of (x, x^2), plus base
__device__ __forceinline__ double2 block_exscan(double2 v, double2 base, double2 *sh) {
    const int t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
        const double2 w = t >= o ? sh[t - o] : make_double2(0.0, 0.0);
        __syncthreads();
        sh[t] = d2add(sh[t], w);
        __syncthreads();
    }
    const double2 r = t > 0 ? d2add(base, sh[t - 1]) : base;
    __syncthreads();
    return r;
}

// prefix sums of (x, x^2) over x[0 .. e): the block prefix plus the <= PB - 1 elements after the
// block start, summed by the workgroup as a tree (every thread gets it)
__device__ __forceinline__ double2 block_prefix(const double *__restrict__ x, const double2 *__restrict__ pre,
                                                int64_t e, double2 *sh) {
    const int t = threadIdx.x;
    const int64_t b = e / PB, q = b * PB + t;
    const double v = q < e ? x[q] : 0.0;
    sh[t] = make_double2(v, v * v);
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (t < o) sh[t] = d2add(sh[t], sh[t + o]);
        __syncthreads();
    }
    const double2 r = d2add(pre[b], sh[0]);
    __syncthreads();
    return r;
}

// a workgroup predicts 256 consecutive frames: the prefix sums at their window ends (and, for
// full windows, starts) are contiguous, so one block_prefix per range plus a block scan gives them
__global__ __launch_bounds__(256) void approx_kernel(const double *__restrict__ x, const double2 *__restrict__ pre,
                                                     FreshParams P, int64_t jbeg, double *__restrict__ fresh,
                                                     double *__restrict__ eps) {
    static_assert(PB == 256, "block_prefix: one element per thread of a 256-thread workgroup");
    __shared__ double2 sh[256];
    const int t = threadIdx.x;
    const int64_t j0 = jbeg + (int64_t)blockIdx.x * 256;
    const int64_t e0 = P.n_tail + j0, l0 = e0 - P.W;  // window end / start of a full window
    const double2 base_hi = block_prefix(x, pre, e0, sh);
    const double2 base_lo = l0 > 0 ? block_prefix(x, pre, l0, sh) : make_double2(0.0, 0.0);
    auto val = [&](int64_t q) {
        const double v = q >= 0 && q < P.x_len ? x[q] : 0.0;
        return make_double2(v, v * v);
    };
    const double2 hi = block_exscan(val(e0 + t), base_hi, sh);
    double2 lo = block_exscan(val(l0 + t), base_lo, sh);  // zeros before index 0
    const int64_t j = j0 + t;
    if (j >= P.n_local) return;
    const int64_t i = P.frame0 + j;
    if (i < P.F0) return;
    const int64_t e = e0 + t;
    const int64_t len = i < P.W ? i : P.W;  // windows before frame W are delta[0:i] (x index 0 = frame 0)
    if (len < P.W) lo = make_double2(0.0, 0.0);
    const double fl = (double)len;
    const double m = (hi.x - lo.x) / fl;
    double v = (hi.y - lo.y) / fl - m * m;
    v = v > 0.0 ? v : 0.0;
    const double sd = sqrt(v);
    const double thr = m + P.k * sd;
    fresh[j] = thr;
    if (!eps) return;
    const double u = 0x1p-53, ak = fabs(P.k);
    // predictor: prefix sums through <= PB (block sums) + per + 10 + per (block scan) + 8 + 1
    // (block_prefix) + 8 + 1 (block_exscan) additions, +1 rounding of x*x (2 PB + 20 + 2 per: ample)
    const double d2 = 2.0 * PB + 20.0 + 2.0 * (double)P.pre_per;
    const double S1 = hi.x - lo.x, S2 = hi.y - lo.y;
    const double eS1 = 1.01 * d2 * u * (sqrt((double)e * hi.y) + sqrt((double)(e - len) * lo.y)) + u * fabs(S1);
    const double eS2 = 1.01 * (d2 + 1.0) * u * (hi.y + lo.y) + u * fabs(S2);
    const double em_a = eS1 / fl + 2.0 * u * fabs(m);
    const double ev_a = (eS2 + u * fabs(S2)) / fl + em_a * (2.0 * fabs(m) + em_a) + u * m * m + 2.0 * u * v;
    const double sig_lo = sqrt(fmax(v - ev_a, 0.0));
    // numpy: s = 0.0; s += pairwise(8192-chunk): leaves of <= 128 (16 adds per accumulator, 3 to
    // combine, 7 remainder), <= 6 tree levels, one add per chunk
    const double d1 = 48.0 + fl / 8192.0;
    const double A = sqrt(fl * (S2 + eS2));  // >= sum |x| over the window
    const double em_np = d1 * u * A / fl + 2.0 * u * (fabs(m) + em_a);
    const double ev_np = 1.01 * (d1 + 4.0) * u * (v + ev_a + em_np * em_np) + em_np * em_np;
    const double es = sd_err(ev_a, sig_lo) + sd_err(ev_np, sig_lo) + 4.0 * u * (sd + sqrt(ev_a + ev_np));
    eps[j] = P.eps_scale * 4.0 * (em_a + em_np + ak * es + 4.0 * u * (fabs(thr) + ak * sd));
}

// certification: the threshold error of every frame from its window's delta error bounds.  mean +
// k std is (1 + k)-Lipschitz in the sense |mean(a) - mean(b)| <= mean|a - b| and |std(a) - std(b)|
// <= rms(a - b) (population std: the norm of the centred vector), so with |delta - delta_ref| <= ed
// per frame, |thr - thr_ref| <= mean(ed) + |k| rms(ed) over the window, plus numpy's own rounding
// on both sides (1e-10 absolute: ~1e-14 |thr| for these windows).  The window sums come from the
// prefix sums of (ed, ed^2) as the predictor's do (approx_kernel); their cancellation error
// (d u (hi + lo), nonnegative terms) is added.
constexpr double TERR_ABS = 1e-10;
__global__ __launch_bounds__(256) void terr_kernel(const double *__restrict__ ed, const double2 *__restrict__ pre,
                                                   FreshParams P, double *__restrict__ terr) {
    __shared__ double2 sh[256];
    const int t = threadIdx.x;
    const int64_t j0 = (int64_t)blockIdx.x * 256;
    const int64_t e0 = P.n_tail + j0, l0 = e0 - P.W;
    const double2 base_hi = block_prefix(ed, pre, e0, sh);
    const double2 base_lo = l0 > 0 ? block_prefix(ed, pre, l0, sh) : make_double2(0.0, 0.0);
    auto val = [&](int64_t q) {
        const double v = q >= 0 && q < P.x_len ? ed[q] : 0.0;
        return make_double2(v, v * v);
    };
    const double2 hi = block_exscan(val(e0 + t), base_hi, sh);
    double2 lo = block_exscan(val(l0 + t), base_lo, sh);
    const int64_t j = j0 + t;
    if (j >= P.n_local) return;
    const int64_t i = P.frame0 + j;
    const int64_t len = i < P.W ? i : P.W;
    if (len < P.W) lo = make_double2(0.0, 0.0);
    if (len <= 0) {  // empty window: NaN threshold on both sides
        terr[j] = 0.0;
        return;
    }
    const double fl = (double)len, u = 0x1p-53;
    const double d2 = 2.0 * PB + 20.0 + 2.0 * (double)P.pre_per;
    const double m1 = fmax(hi.x - lo.x, 0.0) / fl + 2.0 * d2 * u * (hi.x + lo.x) / fl;
    const double m2 = fmax(hi.y - lo.y, 0.0) / fl + 2.0 * d2 * u * (hi.y + lo.y) / fl;
    terr[j] = (m1 + fabs(P.k) * sqrt(m2)) * (1.0 + 1e-9) + TERR_ABS;
}

// sums of (ed, ed^2) over x[a .. b): one 256-thread workgroup per 8192 elements, then one
// workgroup adds the partials (out[nblocks] = total); deterministic order
__global__ __launch_bounds__(256) void ed_sums_kernel(const double *__restrict__ ed, int64_t a, int64_t b,
                                                      double2 *__restrict__ out) {
    __shared__ double2 sh[256];
    const int t = threadIdx.x;
    const int64_t c0 = a + (int64_t)blockIdx.x * CHUNK;
    double s1 = 0.0, s2 = 0.0;
    for (int64_t q = c0 + t; q < c0 + CHUNK && q < b; q += 256) {
        const double v = ed[q];
        s1 += v;
        s2 += v * v;
    }
    sh[t] = make_double2(s1, s2);
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (t < o) sh[t] = d2add(sh[t], sh[t + o]);
        __syncthreads();
    }
    if (t == 0) out[blockIdx.x] = sh[0];
}
__global__ __launch_bounds__(256) void ed_total_kernel(double2 *__restrict__ part, int64_t nb) {
    __shared__ double2 sh[256];
    const int t = threadIdx.x;
    double2 acc = make_double2(0.0, 0.0);
    for (int64_t q = t; q < nb; q += 256) acc = d2add(acc, part[q]);
    sh[t] = acc;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (t < o) sh[t] = d2add(sh[t], sh[t + o]);
        __syncthreads();
    }
    if (t == 0) part[nb] = sh[0];
}

// frames with i < W: window delta[0:i] (only the shard that holds the stream's first W frames)
// frames with i < W: window delta[0:i], a different tree per frame (only the shard that holds the
// stream's first W frames); one wave per frame
__global__ __launch_bounds__(256) void fresh_short_kernel(const double *__restrict__ x, FreshParams P,
                                                          int64_t jend, double *__restrict__ fresh) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int64_t j = (int64_t)blockIdx.x * 4 + w; j < jend; j += (int64_t)gridDim.x * 4) {
        const int64_t i = P.frame0 + j;
        if (i < P.F0) continue;
        const int64_t base = P.n_tail + j - i;  // x index of global frame 0 = n_tail - frame0
        const double m = wave_np_sum(GArrRef{as_global(x)}, base, i) / (double)i;
        const double v = wave_np_sum(GSqDevRef{as_global(x), m}, base, i);
        if (lane == 0) fresh[j] = m + P.k * sqrt(v / (double)i);
    }
}

// decisions-only mode: the frames the marking pass listed, numpy-exact, one 4-wave workgroup per
// frame: wave w sums the window's 8192-element chunks w, w + 4, ... (numpy's pairwise tree per
// chunk), and the chunk sums are added in order from 0.0 (s += chunk), as np.sum does; a window of
// more than FL_MAXCH chunks is summed by wave 0 alone (wave_np_sum, the same association)
constexpr int FL_MAXCH = 64;
__global__ __launch_bounds__(256) void fresh_list_kernel(const double *__restrict__ x, FreshParams P,
                                                         const int32_t *__restrict__ list,
                                                         const int32_t *__restrict__ count, double *__restrict__ fresh,
                                                         uint8_t *__restrict__ exact) {
#pragma clang fp contract(off)
    __shared__ double csum[2][FL_MAXCH];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t n = *count;
    for (int64_t q = blockIdx.x; q < n; q += gridDim.x) {
        const int64_t j = list[q];
        const int64_t i = P.frame0 + j;
        const int64_t len = i < P.W ? i : P.W;
        const int64_t base = P.n_tail + j - len;
        const int64_t nch = (len + NP_BUFSIZE - 1) / NP_BUFSIZE;
        if (nch > FL_MAXCH) {
            if (w == 0) {
                const double m = wave_np_sum(GArrRef{as_global(x)}, base, len) / (double)len;
                const double v = wave_np_sum(GSqDevRef{as_global(x), m}, base, len);
                if (lane == 0) {
                    fresh[j] = m + P.k * sqrt(v / (double)len);
                    exact[j] = 1;
                }
            }
            continue;
        }
        auto chunk_len = [&](int64_t c) { return len - c * NP_BUFSIZE < NP_BUFSIZE ? len - c * NP_BUFSIZE : NP_BUFSIZE; };
        for (int64_t c = w; c < nch; c += 4) {
            const double r = wave_chunk_sum(GArrRef{as_global(x)}, base + c * NP_BUFSIZE, chunk_len(c));
            if (lane == 0) csum[0][c] = r;
        }
        __syncthreads();
        double s = 0.0;
        for (int64_t c = 0; c < nch; ++c) s += csum[0][c];
        const double m = s / (double)len;
        for (int64_t c = w; c < nch; c += 4) {
            const double r = wave_chunk_sum(GSqDevRef{as_global(x), m}, base + c * NP_BUFSIZE, chunk_len(c));
            if (lane == 0) csum[1][c] = r;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            double v = 0.0;
            for (int64_t c = 0; c < nch; ++c) v += csum[1][c];
            fresh[j] = m + P.k * sqrt(v / (double)len);
            exact[j] = 1;
        }
        __syncthreads();  // csum is rewritten by the next frame
    }
}

// ------------------------------------------------------------------ scan
struct ScanParams {
    int64_t n_local, frame0, seg_len, nseg, cap, F0, Fa;
    double thr0;
    int32_t write_thr;
    double terr0;  // certification: thr0's error bound
};

// certification outputs (ed != nullptr): per segment the uncertain decisions of its last scan
struct CertOut {
    const double *ed;    // delta error bound, local frame index (nullptr: no certification)
    const double *terr;  // fresh threshold error bound, local frame index
    longlong2 *unc;      // [nseg][UCAP]
    int32_t *ucnt;       // [nseg]
    double2 *slack;      // [nseg] (min slack, max error zone)
};

__device__ __forceinline__ uint64_t bits_from(int p) { return p >= 64 ? 0ull : (~0ull << p); }
__device__ __forceinline__ uint64_t bits_upto(int e) { return e >= 63 ? ~0ull : ((1ull << (e + 1)) - 1ull); }
__device__ __forceinline__ int64_t shfl_i64(int64_t v, int l) {
    return __builtin_bit_cast(int64_t, __shfl(__builtin_bit_cast(long long, v), l, 64));
}

__global__ __launch_bounds__(64) void scan_kernel(const double *__restrict__ delta, const double *__restrict__ fresh,
                                                  ScanParams P, const SState *__restrict__ in_state,
                                                  SState *__restrict__ out_state, const int32_t *__restrict__ active,
                                                  msd_det *__restrict__ runs, int32_t *__restrict__ nruns,
                                                  double *__restrict__ seg_margin, double *__restrict__ thr_used,
                                                  int32_t *__restrict__ overflow, int32_t *__restrict__ need,
                                                  const double *__restrict__ eps, uint8_t *__restrict__ exact,
                                                  int32_t *__restrict__ list, int32_t *__restrict__ list_count,
                                                  int32_t *__restrict__ changed, CertOut cert) {
    const int64_t s = blockIdx.x;
    // the round's change counter, which the propagate kernel after this one increments (zeroed
    // here instead of by a separate memset launch per round)
    if (changed && s == 0 && threadIdx.x == 0) *changed = 0;
    if (!active[s]) return;
    const int lane = threadIdx.x;
    const int64_t a = s * P.seg_len;
    const int64_t b = a + P.seg_len < P.n_local ? a + P.seg_len : P.n_local;
    const SState in = in_state[s];
    int64_t fz = in.fz, last_stop = in.last_stop;
    double thr_cur = in.thr;
    int64_t src_cur = in.src;  // certification: where thr_cur comes from, and its error bound
    double terr_cur = in.terr;
    const double thr0 = P.thr0, terr0 = P.terr0;
    const bool cfy = cert.ed != nullptr;
    msd_det *rs = runs + s * P.cap;
    int64_t nr = 0, cur_start = 0;
    bool have = false;
    double min_margin = __builtin_inf();
    double min_slack = __builtin_inf(), max_zone = 0.0;
    int32_t nunc = 0;

    // the next step's delta and fresh threshold are loaded one step ahead (the loads do not depend
    // on the state), so the scalar walk of a step overlaps the memory latency of the next
    // (and, when listing, the bound and the exact flag; when certifying, the two error bounds)
    auto ld = [&](int64_t k, double &dv, double &fr, double &ep, uint8_t &ex, double &edv, double &trv) {
        const int64_t j = k + lane < b ? k + lane : (k < b ? k : a);
        dv = delta[j];
        fr = fresh[j];
        if (list) {
            ep = eps[j];
            ex = exact[j];
        }
        if (cfy) {
            edv = cert.ed[j];
            trv = cert.terr[j];
        }
    };
    // two steps in flight: the loads of step k + 128 are issued while step k is walked (deeper
    // rings, 8 steps unrolled, measured slower: the walk is bound by its own instruction latency)
    double dv_n, fr_n, ep_n = 0.0, dv_m, fr_m, ep_m = 0.0, ed_n = 0.0, ed_m = 0.0, tr_n = 0.0, tr_m = 0.0;
    uint8_t ex_n = 1, ex_m = 1;
    ld(a, dv_n, fr_n, ep_n, ex_n, ed_n, tr_n);
    ld(a + 64, dv_m, fr_m, ep_m, ex_m, ed_m, tr_m);
    for (int64_t k = a; k < b; k += 64) {
        const int nvalid = (int)(b - k < 64 ? b - k : 64);
        const bool valid = lane < nvalid;
        const int64_t j = valid ? k + lane : k;
        const int64_t gi = P.frame0 + j;  // global frame of this lane
        const int64_t pos = P.frame0 + k;
        const double dv = dv_n, fr = fr_n, ep = ep_n, edv = ed_n, trv = tr_n;
        const uint8_t ex = ex_n;
        dv_n = dv_m;
        fr_n = fr_m;
        ep_n = ep_m;
        ex_n = ex_m;
        ed_n = ed_m;
        tr_n = tr_m;
        ld(k + 128, dv_m, fr_m, ep_m, ex_m, ed_m, tr_m);
        const bool init = gi < P.F0;
        const double t_unf = init ? thr0 : fr;
        // certification: the fresh threshold's error against the reference's -- the window's delta
        // errors, plus the predictor's bound where the value is a prediction (decisions only)
        const double e_unf = init ? terr0 : trv + ((list && ex != 1) ? ep : 0.0);
        const int64_t s_unf = init ? -1 : gi;
        const uint64_t A_unf = __ballot(valid && dv > t_unf);
        double t_fin = t_unf, e_fin = e_unf;
        int64_t s_fin = s_unf;
        uint64_t D = 0, U = 0;  // detected, unfrozen (fresh threshold used)
        int p = 0;
        while (p < nvalid) {
            const int64_t i = pos + p;
            if (fz >= i) {  // frozen from p on: threshold held (thr0 before the fixed-init end)
                const int e = (int)(fz - pos < nvalid - 1 ? fz - pos : nvalid - 1);
                const bool h0 = i < P.F0;
                const double held = h0 ? thr0 : thr_cur;
                const double held_e = h0 ? terr0 : terr_cur;
                const int64_t held_s = h0 ? -1 : src_cur;
                const double t_h = init ? thr0 : held;
                const uint64_t rng = bits_from(p) & bits_upto(e);
                const uint64_t m = __ballot(valid && dv > t_h) & rng;
                if ((rng >> lane) & 1ull) {
                    t_fin = t_h;
                    e_fin = init ? terr0 : held_e;
                    s_fin = init ? -1 : held_s;
                }
                if ((pos + e) < P.F0) {
                    thr_cur = thr0;
                    terr_cur = terr0;
                    src_cur = -1;
                } else {
                    thr_cur = held;
                    terr_cur = held_e;
                    src_cur = held_s;
                }
                if (m) {
                    const int last = 63 - __builtin_clzll(m);
                    D |= m;
                    fz = pos + last + P.Fa;
                }
                p = e + 1;
            } else {  // unfrozen: fresh (or fixed) thresholds until the first detection
                const uint64_t m = A_unf & bits_from(p);
                if (!m) {
                    U |= bits_from(p);
                    thr_cur = __shfl(t_unf, nvalid - 1);
                    terr_cur = __shfl(e_unf, nvalid - 1);
                    src_cur = shfl_i64(s_unf, nvalid - 1);
                    p = nvalid;
                    break;
                }
                const int u = __builtin_ctzll(m);
                U |= bits_from(p) & bits_upto(u);
                D |= 1ull << u;
                thr_cur = __shfl(t_unf, u);
                terr_cur = __shfl(e_unf, u);
                src_cur = shfl_i64(s_unf, u);
                fz = pos + u + P.Fa;
                p = u + 1;
            }
        }
        if (need && (U & __ballot(valid && !init)) && lane == 0) need[k / FR_FRAMES] = 1;
        if (list) {  // decisions-only marking: near ties and triggers on predicted thresholds
            // exact[j]: 0 predicted, 2 listed (computed by the next refine), 1 exact; a frame is
            // listed once, whichever round (speculative or final) reads it first
            const bool unf = valid && !init && ((U >> lane) & 1ull);
            bool cand = false;
            if (unf && !ex) {
                const bool near = !(fabs(dv - fr) > ep);  // NaN: near
                cand = near || ((D >> lane) & 1ull);
                if (cand) exact[j] = 2;
            }
            const uint64_t mk = __ballot(cand);
            if (mk) {
                int base = 0;
                if (lane == 0) base = atomicAdd(list_count, __builtin_popcountll(mk));
                base = __shfl(base, 0);
                if (cand) list[base + __builtin_popcountll(mk & ((1ull << lane) - 1ull))] = (int32_t)j;
            }
        }
        if (valid) {
            const double mg = fabs(dv - t_fin);
            if (mg < min_margin) min_margin = mg;
            if (P.write_thr) thr_used[j] = t_fin;
        }
        if (cfy) {  // the decision dv > t_fin is the reference's when |dv - t_fin| exceeds both errors;
            // a NaN threshold (empty window) is NaN on both sides: no detection either way
            const double sl = t_fin != t_fin ? __builtin_inf() : fabs(dv - t_fin) - (edv + e_fin);
            const bool unc = valid && !(sl > 0.0);
            if (valid) {
                min_slack = fmin(min_slack, sl != sl ? -__builtin_inf() : sl);
                max_zone = fmax(max_zone, edv + e_fin);
            }
            const uint64_t mu = __ballot(unc);
            if (mu) {
                const int r = __builtin_popcountll(mu & ((1ull << lane) - 1ull));
                if (unc && nunc + r < UCAP) cert.unc[s * UCAP + nunc + r] = make_longlong2(j, s_fin);
                nunc += __builtin_popcountll(mu);
            }
        }
        // runs: maximal groups of consecutive detected frames (a new run iff i > last_stop + 1)
        while (D) {
            const int g0 = __builtin_ctzll(D);
            const uint64_t rest = ~(D >> g0);
            const int glen = rest ? __builtin_ctzll(rest) : 64 - g0;
            const int64_t ib = pos + g0, ie = ib + glen - 1;
            if (last_stop == ib - 1) {
                if (!have) {  // continues the previous segment's run
                    have = true;
                    cur_start = -1;
                }
            } else {
                if (have) {
                    if (lane == 0 && nr < P.cap) {
                        rs[nr].start = cur_start;
                        rs[nr].stop = last_stop + 1;
                    }
                    ++nr;
                }
                have = true;
                cur_start = ib;
            }
            last_stop = ie;
            D &= (glen + g0 >= 64) ? 0ull : (~0ull << (g0 + glen));
        }
    }
    if (have) {
        if (lane == 0 && nr < P.cap) {
            rs[nr].start = cur_start;
            rs[nr].stop = last_stop + 1;
        }
        ++nr;
    }
    for (int o = 32; o >= 1; o >>= 1) min_margin = fmin(min_margin, __shfl_xor(min_margin, o, 64));
    if (cfy)
        for (int o = 32; o >= 1; o >>= 1) {
            min_slack = fmin(min_slack, __shfl_xor(min_slack, o, 64));
            max_zone = fmax(max_zone, __shfl_xor(max_zone, o, 64));
        }
    if (lane == 0) {
        nruns[s] = (int32_t)(nr < P.cap ? nr : P.cap);
        if (nr > P.cap) atomicOr(overflow, 1);
        seg_margin[s] = min_margin;
        if (cfy) {
            cert.ucnt[s] = nunc;
            cert.slack[s] = make_double2(min_slack, max_zone);
        }
        SState o;
        o.fz = fz;
        o.last_stop = last_stop;
        o.thr = thr_cur;
        o.src = src_cur;
        o.terr = terr_cur;
        out_state[s] = o;
    }
}

// the states entering the segments before a scan: segment 0 gets the shard's entry state.
// reset 1: every other segment starts clean (speculative), all active; 2 (thresholds refined):
// every segment re-scans from its fixed-point entry state; 0 (the shard's entry changed): the
// others keep their states and only segment 0 is active
__global__ void scan_entry_kernel(SState *__restrict__ in_state, int32_t *__restrict__ active, int64_t nseg,
                                  SState entry, double thr0, double terr0, int32_t reset) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s < nseg) {
        if (s == 0) in_state[0] = entry;
        else if (reset == 1) in_state[s] = SState{-1, -2, thr0, -1, terr0};
        active[s] = (s == 0 || reset) ? 1 : 0;
    } else if (s < nseg + 2) {
        active[s] = 0;  // change counter, overflow flag
    }
}

// normalised equality of two states entering frame a (see msd_stream_state)
__device__ __forceinline__ bool same_state(const SState &x, const SState &y, int64_t a, int64_t F0) {
    const bool fx = x.fz >= a, fy = y.fz >= a;
    if (fx != fy) return false;
    if (fx) {
        if (x.fz != y.fz) return false;
        if (a >= F0 && (__builtin_bit_cast(long long, x.thr) != __builtin_bit_cast(long long, y.thr) || x.src != y.src))
            return false;
    }
    return (x.last_stop == a - 1) == (y.last_stop == a - 1);
}

__global__ void propagate_kernel(SState *__restrict__ in_state, const SState *__restrict__ out_state,
                                 int32_t *__restrict__ active, int64_t nseg, int64_t seg_len, int64_t frame0,
                                 int64_t F0, int32_t *__restrict__ changed) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nseg) return;
    if (s == 0) {
        active[0] = 0;
        return;
    }
    const SState nw = out_state[s - 1];
    if (same_state(nw, in_state[s], frame0 + s * seg_len, F0)) {
        active[s] = 0;
    } else {
        in_state[s] = nw;
        active[s] = 1;
        atomicAdd(changed, 1);
    }
}

// compaction: runs of segment s go to out[pos_s ..]; a continued first run of s >= 1 extends the
// last run of s-1 (or the run that one continues) instead.  One workgroup.
// 256 threads (was 1024): beside the persistent spectrogram (IQShardDetector overlap) a 16-wave
// workgroup found no CU with room until the spectrogram's last workgroups left (1.3 ms in the trace)
constexpr int RK_T = 256;
__global__ __launch_bounds__(RK_T) void runs_kernel(const msd_det *__restrict__ runs,
                                                    const int32_t *__restrict__ nruns, int64_t nseg, int64_t cap,
                                                    msd_det *__restrict__ out, int64_t *__restrict__ count,
                                                    int64_t *__restrict__ seg_pos) {
    __shared__ int64_t s_base;
    const int tid = threadIdx.x;
    if (tid == 0) s_base = 0;
    __syncthreads();
    for (int64_t c0 = 0; c0 < nseg; c0 += RK_T) {
        const int64_t s = c0 + tid;
        int64_t e = 0;
        bool cont = false;
        if (s < nseg) {
            const int64_t n = nruns[s];
            cont = s > 0 && n > 0 && runs[s * cap].start < 0;
            e = n - (cont ? 1 : 0);
        }
        // block-wide inclusive scan of e (Hillis-Steele in LDS)
        __shared__ int64_t sc[RK_T];
        sc[tid] = e;
        __syncthreads();
        for (int o = 1; o < RK_T; o <<= 1) {
            const int64_t v = tid >= o ? sc[tid - o] : 0;
            __syncthreads();
            sc[tid] += v;
            __syncthreads();
        }
        const int64_t pos = s_base + sc[tid] - e;
        if (s < nseg) {
            seg_pos[s] = pos;
            const int64_t n = nruns[s];
            for (int64_t r = cont ? 1 : 0; r < n; ++r) out[pos + r - (cont ? 1 : 0)] = runs[s * cap + r];
        }
        __syncthreads();
        if (tid == RK_T - 1) s_base += sc[RK_T - 1];
        __syncthreads();
    }
    if (tid == 0) *count = s_base;
    __syncthreads();
    // continued runs: the owner is the last emitted run before this segment
    for (int64_t s = 1 + tid; s < nseg; s += RK_T) {
        const int64_t n = nruns[s];
        if (n == 0 || runs[s * cap].start >= 0) continue;
        const int64_t before = seg_pos[s];  // runs emitted by the segments before s
        if (before > 0)
            atomicMax(reinterpret_cast<unsigned long long *>(&out[before - 1].stop),
                      (unsigned long long)runs[s * cap].stop);
    }
}

__global__ void db_kernel(const double *__restrict__ x, int64_t x0, msd_det *__restrict__ d, int64_t n) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const int64_t a = d[j].start, m = d[j].stop - d[j].start;
    d[j].db = np_sum(GArrRef{as_global(x)}, a - x0, m) / (double)m;
}

}  // namespace
}  // namespace msd

using namespace msd;

static PinHdr *pin_hdr(msd_stream_plan *p) { return static_cast<PinHdr *>(p->h_pin); }
static double *pin_margin(msd_stream_plan *p) { return reinterpret_cast<double *>(pin_hdr(p) + 1); }
static double *pin_chunks(msd_stream_plan *p) { return pin_margin(p) + (p->nseg > 0 ? p->nseg : 1); }
static SState *st_in(msd_stream_plan *p) { return reinterpret_cast<SState *>(p->d_state); }
static SState *st_out(msd_stream_plan *p) { return reinterpret_cast<SState *>(p->d_state) + p->nseg; }

extern "C" {

int msd_iq_band_delta_dev(msd_ctx *ctx, const float *spec, int64_t nstreams, int64_t max_frames,
                          const int64_t *frames, int32_t nperseg, int32_t band_lo, int32_t band_hi, int32_t noise_lo,
                          int32_t noise_hi, double *band_db, double *noise_db, double *delta, int64_t ld) {
    return msd_iq_band_delta_bound_dev(ctx, spec, nullptr, nstreams, max_frames, frames, nperseg, band_lo, band_hi,
                                       noise_lo, noise_hi, band_db, noise_db, delta, nullptr, ld);
}

int msd_iq_band_delta_bound_dev(msd_ctx *ctx, const float *spec, const float *etot, int64_t nstreams,
                                int64_t max_frames, const int64_t *frames, int32_t nperseg, int32_t band_lo,
                                int32_t band_hi, int32_t noise_lo, int32_t noise_hi, double *band_db, double *noise_db,
                                double *delta, double *ed, int64_t ld) {
    if (!ctx || !spec || !frames || !delta || nstreams < 0 || max_frames < 0 || nperseg <= 0 || ld < max_frames ||
        (!etot) != (!ed))
        return fail(MSD_ERR_INVALID, "msd_iq_band_delta_dev: bad args");
    const int h = nperseg / 2;
    auto ok = [&](int lo, int hi) { return hi < lo || (lo >= -h && hi <= nperseg - h - 1); };
    if (!ok(band_lo, band_hi) || !ok(noise_lo, noise_hi))
        return fail(MSD_ERR_INVALID, "msd_iq_band_delta_dev: band outside -N/2 .. N/2-1");
    if (nstreams == 0 || max_frames == 0) return MSD_OK;
    DeviceGuard g(ctx->device);
    KernelTimer timer(ctx, K_IQDELTA);
    const int64_t blocks = (nstreams * max_frames + 255) / 256;
    hipLaunchKernelGGL(iq_band_delta_kernel, dim3((unsigned)blocks), dim3(256), 0, ctx->stream, spec, nstreams,
                       max_frames, frames, (int)nperseg, band_lo, band_hi, noise_lo, noise_hi, band_db, noise_db,
                       delta, ld, etot, ed);
    MSD_HIP(hipGetLastError());
    return MSD_OK;
}

int msd_stream_plan_create(msd_ctx *ctx, const msd_det_cfg *cfg, int64_t n_total, int64_t frame0, int64_t n_local,
                           int64_t seg_len, int64_t cap_per_seg, int64_t head_frames, msd_stream_plan **out) {
    if (!ctx || !cfg || !out || n_total < 0 || frame0 < 0 || n_local < 0 || frame0 + n_local > n_total ||
        seg_len < 64 || seg_len % 64 || cap_per_seg <= 0 || head_frames < 0)
        return fail(MSD_ERR_INVALID, "msd_stream_plan_create: bad args");
    if (cfg->adaptive && (cfg->window_blocks < 0 || cfg->freeze_after_blocks < 0 || cfg->fixed_init_blocks < 0))
        return fail(MSD_ERR_INVALID, "msd_stream_plan_create: negative block counts");
    *out = nullptr;
    DeviceGuard g(ctx->device);
    auto *p = new msd_stream_plan();
    p->ctx = ctx;
    p->cfg = *cfg;
    p->n_total = n_total;
    p->frame0 = frame0;
    p->n_local = n_local;
    const int64_t W = cfg->adaptive ? cfg->window_blocks : 0;
    p->n_tail = W < frame0 ? W : frame0;
    const int64_t after = n_total - frame0 - n_local;
    p->head_cap = head_frames;
    p->n_head = head_frames < after ? head_frames : after;
    p->seg_len = seg_len;
    p->nseg = n_local > 0 ? (n_local + seg_len - 1) / seg_len : 0;
    p->cap = cap_per_seg;
    const int64_t nseg1 = p->nseg > 0 ? p->nseg : 1;
    const int64_t nl1 = n_local > 0 ? n_local : 1;
    const int64_t nchunk = n_local / CHUNK + 2;
    auto cleanup = [&](hipError_t e, const char *what) {
        msd_stream_plan_destroy(p);
        return hip_fail(e, what);
    };
    hipError_t e;
    if ((e = hipMalloc(&p->d_x, sizeof(double) * (p->n_tail + nl1 + p->head_cap))) != hipSuccess)
        return cleanup(e, "hipMalloc stream x");
    if ((e = hipMalloc(&p->d_fresh, sizeof(double) * nl1)) != hipSuccess) return cleanup(e, "hipMalloc fresh");
    if ((e = hipMalloc(&p->d_thr, sizeof(double) * nl1)) != hipSuccess) return cleanup(e, "hipMalloc thr");
    if ((e = hipMalloc(&p->d_state, sizeof(SState) * 2 * nseg1)) != hipSuccess) return cleanup(e, "hipMalloc state");
    if ((e = hipMalloc(&p->d_active, sizeof(int32_t) * (nseg1 + 2))) != hipSuccess)
        return cleanup(e, "hipMalloc active");
    if ((e = hipMalloc(&p->d_runs, sizeof(msd_det) * nseg1 * cap_per_seg)) != hipSuccess)
        return cleanup(e, "hipMalloc runs");
    if ((e = hipMalloc(&p->d_out, sizeof(msd_det) * nseg1 * cap_per_seg)) != hipSuccess)
        return cleanup(e, "hipMalloc out");
    if ((e = hipMalloc(&p->d_nruns, sizeof(int32_t) * nseg1)) != hipSuccess) return cleanup(e, "hipMalloc nruns");
    if ((e = hipMalloc(&p->d_margin, sizeof(double) * nseg1)) != hipSuccess) return cleanup(e, "hipMalloc margin");
    if ((e = hipMalloc(&p->d_count, sizeof(int64_t))) != hipSuccess) return cleanup(e, "hipMalloc count");
    if ((e = hipMalloc(&p->d_pos, sizeof(int64_t) * nseg1)) != hipSuccess) return cleanup(e, "hipMalloc pos");
    if ((e = hipMalloc(&p->d_chunks, sizeof(double) * (nchunk + 2))) != hipSuccess)
        return cleanup(e, "hipMalloc chunks");
    if ((e = hipHostMalloc(&p->h_pin, sizeof(PinHdr) + sizeof(double) * (nseg1 + nchunk + 4), hipHostMallocDefault)) !=
        hipSuccess)
        return cleanup(e, "hipHostMalloc stream readbacks");
    p->ntiles = (nl1 + FR_FRAMES - 1) / FR_FRAMES;
    p->nblk = (p->n_tail + nl1 + p->head_cap) / PB + 1;
    if ((e = hipMalloc(&p->d_need, sizeof(int32_t) * p->ntiles)) != hipSuccess) return cleanup(e, "hipMalloc need");
    if ((e = hipMalloc(&p->d_done, sizeof(int32_t) * (p->ntiles + 1))) != hipSuccess)
        return cleanup(e, "hipMalloc done");
    if ((e = hipMalloc(&p->d_pre, sizeof(double2) * (p->nblk + 1))) != hipSuccess) return cleanup(e, "hipMalloc pre");
    if ((e = hipMalloc(&p->d_eps, sizeof(double) * nl1)) != hipSuccess) return cleanup(e, "hipMalloc eps");
    if ((e = hipMalloc(&p->d_exact, nl1)) != hipSuccess) return cleanup(e, "hipMalloc exact");
    if ((e = hipMalloc(&p->d_list, sizeof(int32_t) * nl1)) != hipSuccess) return cleanup(e, "hipMalloc list");
    // certification buffers (used after msd_stream_set_certify); ed starts at 0 (delta exact)
    const int64_t xl = p->n_tail + nl1 + p->head_cap;
    if ((e = hipMalloc(&p->d_ed, sizeof(double) * xl)) != hipSuccess) return cleanup(e, "hipMalloc ed");
    if ((e = hipMemset(p->d_ed, 0, sizeof(double) * xl)) != hipSuccess) return cleanup(e, "hipMemset ed");
    if ((e = hipMalloc(&p->d_terr, sizeof(double) * nl1)) != hipSuccess) return cleanup(e, "hipMalloc terr");
    if ((e = hipMalloc(&p->d_pre_e, sizeof(double2) * (p->nblk + 1))) != hipSuccess)
        return cleanup(e, "hipMalloc pre_e");
    if ((e = hipMalloc(&p->d_unc, sizeof(longlong2) * nseg1 * UCAP)) != hipSuccess) return cleanup(e, "hipMalloc unc");
    if ((e = hipMalloc(&p->d_ucnt, sizeof(int32_t) * nseg1)) != hipSuccess) return cleanup(e, "hipMalloc ucnt");
    if ((e = hipMemset(p->d_ucnt, 0, sizeof(int32_t) * nseg1)) != hipSuccess) return cleanup(e, "hipMemset ucnt");
    if ((e = hipMalloc(&p->d_slack, sizeof(double2) * nseg1)) != hipSuccess) return cleanup(e, "hipMalloc slack");
    if ((e = hipMalloc(&p->d_esum, sizeof(double2) * (xl / CHUNK + 2))) != hipSuccess)
        return cleanup(e, "hipMalloc esum");
    if (W > 0) {
        std::vector<LeafRec> prog;  // np_program.h; LeafRec has int4's layout
        static_assert(sizeof(LeafRec) == sizeof(int4), "leaf record layout");
        build_program(W, prog);
        p->nleaf = (int)prog.size();
        if ((e = hipMalloc(&p->d_prog, sizeof(int4) * prog.size())) != hipSuccess) return cleanup(e, "hipMalloc prog");
        if ((e = hipMemcpy(p->d_prog, prog.data(), sizeof(int4) * prog.size(), hipMemcpyHostToDevice)) != hipSuccess)
            return cleanup(e, "hipMemcpy prog");
    }
    *out = p;
    return MSD_OK;
}

void msd_stream_plan_destroy(msd_stream_plan *p) {
    if (!p) return;
    DeviceGuard g(p->ctx->device);
    hipStreamSynchronize(p->ctx->stream);
    void *bufs[] = {p->d_x, p->d_fresh, p->d_thr, p->d_state, p->d_active, p->d_runs, p->d_out, p->d_nruns,
                    p->d_margin, p->d_count, p->d_pos, p->d_chunks, p->d_prog, p->d_need, p->d_done, p->d_pre,
                    p->d_eps, p->d_exact, p->d_list, p->d_ed, p->d_terr, p->d_pre_e, p->d_unc, p->d_ucnt,
                    p->d_slack, p->d_esum};
    for (void *b : bufs)
        if (b) hipFree(b);
    if (p->h_pin) hipHostFree(p->h_pin);
    if (p->h_cert) hipHostFree(p->h_cert);
    delete p;
}

int msd_stream_buffers(msd_stream_plan *p, double **delta, double **tail, int64_t *n_tail, double **head,
                       int64_t *n_head, double **thresholds) {
    if (!p) return fail(MSD_ERR_INVALID, "msd_stream_buffers: null plan");
    if (delta) *delta = p->d_x + p->n_tail;
    if (tail) *tail = p->d_x;
    if (n_tail) *n_tail = p->n_tail;
    if (head) *head = p->d_x + p->n_tail + p->n_local;
    if (n_head) *n_head = p->n_head;
    if (thresholds) *thresholds = p->d_thr;
    return MSD_OK;
}

int msd_stream_chunk_sums(msd_stream_plan *p, int32_t use_mean, double mean, double *sums, int64_t cap,
                          int64_t *nchunks, int64_t *first_chunk) {
    if (!p || !nchunks || !first_chunk) return fail(MSD_ERR_INVALID, "msd_stream_chunk_sums: null");
    const int64_t c0 = (p->frame0 + CHUNK - 1) / CHUNK;
    const int64_t end = p->frame0 + p->n_local;
    const int64_t c1 = end > 0 ? (end + CHUNK - 1) / CHUNK : 0;  // chunks starting before end
    const int64_t nc = c1 > c0 ? c1 - c0 : 0;
    *first_chunk = c0;
    *nchunks = nc;
    if (nc == 0) return MSD_OK;
    if (!sums || cap < nc) return fail(MSD_ERR_CAPACITY, "msd_stream_chunk_sums: sums buffer too small");
    const int64_t last_end = (c1 * CHUNK < p->n_total ? c1 * CHUNK : p->n_total);
    if (last_end > end + p->n_head)
        return fail(MSD_ERR_UNSUPPORTED, "msd_stream_chunk_sums: the shard's last chunk runs past the head halo");
    DeviceGuard g(p->ctx->device);
    const int64_t x0 = p->frame0 - p->n_tail;
    const unsigned blocks = (unsigned)((nc + 3) / 4);
    if (use_mean)
        hipLaunchKernelGGL(chunk_sums_kernel<true>, dim3(blocks), dim3(256), 0, p->ctx->stream, p->d_x, x0, c0, nc,
                           p->n_total, mean, nullptr, p->d_chunks);
    else
        hipLaunchKernelGGL(chunk_sums_kernel<false>, dim3(blocks), dim3(256), 0, p->ctx->stream, p->d_x, x0, c0, nc,
                           p->n_total, 0.0, nullptr, p->d_chunks);
    MSD_HIP(hipGetLastError());
    MSD_HIP(hipMemcpyAsync(pin_chunks(p), p->d_chunks, sizeof(double) * nc, hipMemcpyDeviceToHost, p->ctx->stream));
    MSD_HIP(hipStreamSynchronize(p->ctx->stream));
    std::memcpy(sums, pin_chunks(p), sizeof(double) * nc);
    return MSD_OK;
}

static void fresh_params(msd_stream_plan *p, FreshParams &P) {
    P.n_local = p->n_local;
    P.frame0 = p->frame0;
    P.n_tail = p->n_tail;
    P.x_len = p->n_tail + p->n_local + p->n_head;
    P.W = p->cfg.window_blocks;
    P.F0 = p->cfg.fixed_init_blocks;
    P.k = p->cfg.k_std;
    P.nleaf = p->nleaf;
    P.pre_per = (P.x_len / PB + 1 + 1023) / 1024;
    const char *es = getenv("MSD_STREAM_EPS_SCALE");
    P.eps_scale = es && atof(es) >= 1.0 ? atof(es) : 1.0;  // never narrower than the bound
}

int msd_stream_set_exact_thresholds(msd_stream_plan *p, int32_t on) {
    if (!p) return fail(MSD_ERR_INVALID, "msd_stream_set_exact_thresholds: null plan");
    p->want_exact = on != 0;
    return MSD_OK;
}

int msd_stream_predicted(msd_stream_plan *p, double *fresh, double *eps) {
    if (!p) return fail(MSD_ERR_INVALID, "msd_stream_predicted: null plan");
    if (!p->decide) return fail(MSD_ERR_INVALID, "msd_stream_predicted: plan not in decisions-only mode");
    if (p->n_local == 0) return MSD_OK;
    DeviceGuard g(p->ctx->device);
    hipStream_t st = p->ctx->stream;
    if (fresh) MSD_HIP(hipMemcpyAsync(fresh, p->d_fresh, sizeof(double) * p->n_local, hipMemcpyDeviceToHost, st));
    if (eps) MSD_HIP(hipMemcpyAsync(eps, p->d_eps, sizeof(double) * p->n_local, hipMemcpyDeviceToHost, st));
    MSD_HIP(hipStreamSynchronize(st));
    return MSD_OK;
}

int msd_stream_fresh(msd_stream_plan *p) {
    if (!p) return fail(MSD_ERR_INVALID, "msd_stream_fresh: null plan");
    if (!p->cfg.adaptive || p->n_local == 0) return MSD_OK;
    DeviceGuard g(p->ctx->device);
    hipStream_t st = p->ctx->stream;
    KernelTimer timer(p->ctx, K_FRESH);
    FreshParams P;
    fresh_params(p, P);
    // MSD_FRESH_ALL=1: every tile exact up front (A/B timing of the exact kernel; same results)
    static const bool all = [] {
        const char *e = getenv("MSD_FRESH_ALL");
        return e && e[0] == '1';
    }();
    // decisions-only: every frame predicted (with its error bound), exact ones listed by the scan
    p->decide = !p->want_exact && P.W > 0 && !(all || p->ctx->fresh_all);
    // need = 0 (1 with MSD_FRESH_ALL), done = 0, exact = 0 (decisions only): one launch
    hipLaunchKernelGGL(fresh_clear_kernel, dim3(512), dim3(256), 0, st, p->d_need, p->ntiles,
                       (all || p->ctx->fresh_all) ? 1 : 0, p->d_done, p->ntiles + 1, p->decide ? p->d_exact : nullptr,
                       p->n_local);
    // frames [0, jshort) have windows shorter than W: exact right away
    int64_t jshort = P.W - p->frame0;
    jshort = jshort < 0 ? 0 : (jshort > p->n_local ? p->n_local : jshort);
    if (P.W == 0) jshort = p->n_local;  // empty windows: NaN thresholds
    if (p->decide) jshort = 0;
    if (jshort > 0)
        hipLaunchKernelGGL(fresh_short_kernel, dim3((unsigned)std::min<int64_t>((jshort + 3) / 4, 4096)), dim3(256), 0,
                           st, p->d_x, P, jshort, p->d_fresh);
    if (jshort < p->n_local) {  // the predictor for full windows
        const int64_t nb = P.x_len / PB + 1;
        hipLaunchKernelGGL(blocksum_kernel, dim3((unsigned)((nb + 3) / 4)), dim3(256), 0, st, p->d_x, P.x_len,
                           nb, p->d_pre);
        hipLaunchKernelGGL(blockscan_kernel, dim3(1), dim3(1024), 0, st, p->d_pre, nb);
        const int64_t m = p->n_local - jshort;
        hipLaunchKernelGGL(approx_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, p->d_x, p->d_pre, P,
                           jshort, p->d_fresh, p->decide ? p->d_eps : nullptr);
    }
    if (p->certify) {  // the thresholds' error bounds from the windows' delta error bounds
        const int64_t nb = P.x_len / PB + 1;
        hipLaunchKernelGGL(blocksum_kernel, dim3((unsigned)((nb + 3) / 4)), dim3(256), 0, st, p->d_ed, P.x_len, nb,
                           p->d_pre_e);
        hipLaunchKernelGGL(blockscan_kernel, dim3(1), dim3(1024), 0, st, p->d_pre_e, nb);
        hipLaunchKernelGGL(terr_kernel, dim3((unsigned)((p->n_local + 255) / 256)), dim3(256), 0, st, p->d_ed,
                           p->d_pre_e, P, p->d_terr);
    }
    MSD_HIP(hipGetLastError());
    return MSD_OK;
}

int msd_stream_set_certify(msd_stream_plan *p, int32_t on) {
    if (!p) return fail(MSD_ERR_INVALID, "msd_stream_set_certify: null plan");
    p->certify = on != 0;
    p->cert_valid = false;  // the next full scan writes the certificate
    p->cert_staged = false;
    return MSD_OK;
}

int msd_stream_error_buffers(msd_stream_plan *p, double **ed, double **tail, double **head) {
    if (!p) return fail(MSD_ERR_INVALID, "msd_stream_error_buffers: null plan");
    if (ed) *ed = p->d_ed + p->n_tail;
    if (tail) *tail = p->d_ed;
    if (head) *head = p->d_ed + p->n_tail + p->n_local;
    return MSD_OK;
}

// (sum ed, sum ed^2) over [x0, x1) of the plan's x indexing, on the device at d_esum[nb]; returns nb
static int64_t ed_sums_async(msd_stream_plan *p, int64_t x0, int64_t x1) {
    const int64_t nb = x1 > x0 ? (x1 - x0 + CHUNK - 1) / CHUNK : 0;
    hipStream_t st = p->ctx->stream;
    if (nb > 0)
        hipLaunchKernelGGL(ed_sums_kernel, dim3((unsigned)nb), dim3(256), 0, st, p->d_ed, x0, x1, p->d_esum);
    hipLaunchKernelGGL(ed_total_kernel, dim3(1), dim3(256), 0, st, p->d_esum, nb);
    return nb;
}

int msd_stream_ed_sums(msd_stream_plan *p, double *s1, double *s2) {
    if (!p || !s1 || !s2) return fail(MSD_ERR_INVALID, "msd_stream_ed_sums: null");
    DeviceGuard g(p->ctx->device);
    const int64_t nb = ed_sums_async(p, p->n_tail, p->n_tail + p->n_local);
    MSD_HIP(hipGetLastError());
    double2 r;
    MSD_HIP(hipMemcpyAsync(pin_chunks(p), p->d_esum + nb, sizeof(double2), hipMemcpyDeviceToHost, p->ctx->stream));
    MSD_HIP(hipStreamSynchronize(p->ctx->stream));
    std::memcpy(&r, pin_chunks(p), sizeof(r));
    *s1 = r.x;
    *s2 = r.y;
    return MSD_OK;
}

// thr0's error bound from the whole stream's (sum ed, sum ed^2) over n frames
static double terr0_from(double s1, double s2, int64_t n, double k) {
    if (n <= 0) return 0.0;
    const double fl = (double)n;
    return (s1 / fl + fabs(k) * sqrt(s2 / fl)) * (1.0 + 1e-9) + TERR_ABS;
}

int msd_stream_set_terr0(msd_stream_plan *p, double s1, double s2) {
    if (!p) return fail(MSD_ERR_INVALID, "msd_stream_set_terr0: null plan");
    p->terr0 = terr0_from(s1, s2, p->n_total, p->cfg.k_std);
    return MSD_OK;
}

// pinned staging of the certificate (grown once): per-segment slacks, counts, then the lists
static int cert_staging(msd_stream_plan *p, double2 **sl, int32_t **cnt, longlong2 **u) {
    const size_t need =
        sizeof(double2) * p->nseg + sizeof(int32_t) * (p->nseg + 1) + sizeof(longlong2) * p->nseg * UCAP;
    if (p->h_cert_bytes < need) {
        if (p->h_cert) (void)hipHostFree(p->h_cert);
        p->h_cert = nullptr;
        p->h_cert_bytes = 0;
        MSD_HIP(hipHostMalloc(&p->h_cert, need, hipHostMallocDefault));
        p->h_cert_bytes = need;
    }
    *sl = static_cast<double2 *>(p->h_cert);
    *cnt = reinterpret_cast<int32_t *>(*sl + p->nseg);
    *u = reinterpret_cast<longlong2 *>(*cnt + p->nseg + (p->nseg & 1));
    return MSD_OK;
}

// the counts and slacks into the staging block (async, on the context stream)
static int cert_enqueue(msd_stream_plan *p) {
    double2 *sl;
    int32_t *cnt;
    longlong2 *u;
    if (int rc = cert_staging(p, &sl, &cnt, &u)) return rc;
    hipStream_t st = p->ctx->stream;
    MSD_HIP(hipMemcpyAsync(sl, p->d_slack, sizeof(double2) * p->nseg, hipMemcpyDeviceToHost, st));
    MSD_HIP(hipMemcpyAsync(cnt, p->d_ucnt, sizeof(int32_t) * p->nseg, hipMemcpyDeviceToHost, st));
    return MSD_OK;
}

int msd_stream_certificate(msd_stream_plan *p, int64_t *uncertain, double *min_slack, double *max_zone,
                           int64_t *frames, int64_t *srcs, int64_t cap, int64_t *listed) {
    if (!p || !uncertain || !min_slack || !max_zone || !listed)
        return fail(MSD_ERR_INVALID, "msd_stream_certificate: null");
    *uncertain = 0;
    *listed = 0;
    *min_slack = __builtin_inf();
    *max_zone = 0.0;
    if (!p->certify) return fail(MSD_ERR_INVALID, "msd_stream_certificate: certification is off");
    if (p->nseg == 0) return MSD_OK;
    if (!p->scanned || !p->cert_valid)
        return fail(MSD_ERR_INVALID, "msd_stream_certificate: call msd_stream_scan with certification on first");
    DeviceGuard g(p->ctx->device);
    hipStream_t st = p->ctx->stream;
    // counts and slacks in one round trip (already staged by msd_stream_detect_local's last sync),
    // the lists in a second one only when something is uncertain
    double2 *sl;
    int32_t *cnt;
    longlong2 *u;
    if (int rc = cert_staging(p, &sl, &cnt, &u)) return rc;
    if (!p->cert_staged) {
        if (int rc = cert_enqueue(p)) return rc;
        MSD_HIP(hipStreamSynchronize(st));
    }
    int64_t tot = 0;
    for (int64_t q = 0; q < p->nseg; ++q) {
        tot += cnt[q];
        *min_slack = sl[q].x < *min_slack || sl[q].x != sl[q].x ? sl[q].x : *min_slack;
        *max_zone = sl[q].y > *max_zone ? sl[q].y : *max_zone;
    }
    *uncertain = tot;
    if (tot == 0 || !frames || !srcs || cap <= 0) return MSD_OK;
    MSD_HIP(hipMemcpyAsync(u, p->d_unc, sizeof(longlong2) * p->nseg * UCAP, hipMemcpyDeviceToHost, st));
    MSD_HIP(hipStreamSynchronize(st));
    int64_t n = 0;
    for (int64_t q = 0; q < p->nseg && n < cap; ++q) {
        const int32_t m = cnt[q] < UCAP ? cnt[q] : UCAP;
        for (int32_t r = 0; r < m && n < cap; ++r, ++n) {
            frames[n] = p->frame0 + u[q * UCAP + r].x;  // global frame index
            srcs[n] = u[q * UCAP + r].y;
        }
    }
    *listed = n;
    return MSD_OK;
}

int msd_stream_refine(msd_stream_plan *p, int32_t *computed) {
    if (!p || !computed) return fail(MSD_ERR_INVALID, "msd_stream_refine: null");
    *computed = 0;
    if (!p->cfg.adaptive || p->n_local == 0 || p->cfg.window_blocks == 0) return MSD_OK;
    DeviceGuard g(p->ctx->device);
    hipStream_t st = p->ctx->stream;
    FreshParams P;
    fresh_params(p, P);
    int32_t *count = p->d_done + p->ntiles;
    if (p->decide && p->listed == 0) return MSD_OK;  // the last scan listed nothing
    if (p->decide) {  // the frames the scan rounds listed
        {
            KernelTimer timer(p->ctx, K_FRESH);
            hipLaunchKernelGGL(fresh_list_kernel, dim3(1024), dim3(256), 0, st, p->d_x, P, p->d_list, count,
                               p->d_fresh, p->d_exact);
        }
        MSD_HIP(hipGetLastError());
        MSD_HIP(hipMemcpyAsync(&pin_hdr(p)->computed, count, sizeof(int32_t), hipMemcpyDeviceToHost, st));
        MSD_HIP(hipMemsetAsync(count, 0, sizeof(int32_t), st));
        MSD_HIP(hipStreamSynchronize(st));
        *computed = pin_hdr(p)->computed;
        return MSD_OK;
    }
    MSD_HIP(hipMemsetAsync(count, 0, sizeof(int32_t), st));
    {
        KernelTimer timer(p->ctx, K_FRESH);
        hipLaunchKernelGGL(fresh_kernel, dim3((unsigned)p->ntiles), dim3(FR_THREADS), 0, st, p->d_x, P, p->d_prog,
                           p->d_fresh, p->d_need, p->d_done, count);
    }
    MSD_HIP(hipGetLastError());
    MSD_HIP(hipMemcpyAsync(&pin_hdr(p)->computed, count, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    MSD_HIP(hipStreamSynchronize(st));
    *computed = pin_hdr(p)->computed;
    return MSD_OK;
}

int msd_stream_scan(msd_stream_plan *p, double thr0, const msd_stream_state *entry, int32_t reset,
                    msd_stream_state *exit_state, int32_t *rounds) {
    if (!p || !entry) return fail(MSD_ERR_INVALID, "msd_stream_scan: null");
    DeviceGuard g(p->ctx->device);
    hipStream_t st = p->ctx->stream;
    int32_t nround = 0;
    const int32_t scan_mode = !p->scanned ? 1 : (reset == 1 || reset == 2 ? reset : 0);
    p->cert_staged = false;
    if (p->nseg == 0) {
        if (exit_state) *exit_state = *entry;
        if (rounds) *rounds = 0;
        return MSD_OK;
    }
    {  // entry states and active flags set on the device (kernel arguments: no host staging, no sync)
        SState e0;
        std::memcpy(&e0, entry, sizeof(SState));
        hipLaunchKernelGGL(scan_entry_kernel, dim3((unsigned)((p->nseg + 2 + 255) / 256)), dim3(256), 0, st, st_in(p),
                           p->d_active, p->nseg, e0, thr0, p->terr0, scan_mode);
        MSD_HIP(hipGetLastError());
    }
    p->thr0 = thr0;
    ScanParams P;
    P.n_local = p->n_local;
    P.frame0 = p->frame0;
    P.seg_len = p->seg_len;
    P.nseg = p->nseg;
    P.cap = p->cap;
    P.F0 = p->cfg.adaptive ? p->cfg.fixed_init_blocks : p->n_total;  // global mode: thr0 everywhere
    P.Fa = p->cfg.adaptive ? p->cfg.freeze_after_blocks : 0;
    P.thr0 = thr0;
    P.write_thr = p->decide ? 0 : 1;  // decisions only: the thresholds buffer is not an output
    P.terr0 = p->terr0;
    CertOut cert{nullptr, nullptr, nullptr, nullptr, nullptr};
    if (p->certify) cert = CertOut{p->d_ed + p->n_tail, p->d_terr, p->d_unc, p->d_ucnt, p->d_slack};
    int32_t *changed = p->d_active + p->nseg;
    int32_t *overflow = p->d_active + p->nseg + 1;
    // rounds are enqueued three at a time (a round with no active segment costs two empty
    // launches); the host checks the last round's change count, so a typical fixed point
    // (2-3 rounds) costs one round trip
    constexpr int R = 3;
    SState ex{};
    for (;;) {
        for (int r = 0; r < R; ++r) {
            {
                KernelTimer timer(p->ctx, K_SSCAN);
                hipLaunchKernelGGL(scan_kernel, dim3((unsigned)p->nseg), dim3(64), 0, st, p->d_x + p->n_tail,
                                   p->d_fresh, P, st_in(p), st_out(p), p->d_active, p->d_runs, p->d_nruns,
                                   p->d_margin, p->d_thr, overflow, nullptr, p->d_eps, p->d_exact,
                                   p->decide ? p->d_list : nullptr, p->d_done + p->ntiles, changed, cert);
            }
            MSD_HIP(hipGetLastError());
            ++nround;
            hipLaunchKernelGGL(propagate_kernel, dim3((unsigned)((p->nseg + 255) / 256)), dim3(256), 0, st, st_in(p),
                               st_out(p), p->d_active, p->nseg, p->seg_len, p->frame0, P.F0, changed);
            MSD_HIP(hipGetLastError());
        }
        PinHdr *h = pin_hdr(p);
        MSD_HIP(hipMemcpyAsync(&h->changed, changed, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, st));
        MSD_HIP(hipMemcpyAsync(&h->ex, st_out(p) + (p->nseg - 1), sizeof(SState), hipMemcpyDeviceToHost, st));
        if (p->decide)  // frames listed so far: a refine with none to compute needs no GPU round trip
            MSD_HIP(hipMemcpyAsync(&h->listed, p->d_done + p->ntiles, sizeof(int32_t), hipMemcpyDeviceToHost, st));
        MSD_HIP(hipStreamSynchronize(st));
        ex = h->ex;
        if (p->decide) p->listed = h->listed;
        if (h->overflow) return fail(MSD_ERR_CAPACITY, "msd_stream_scan: more runs in a segment than cap_per_seg");
        if (h->changed == 0) break;
        if (nround > p->nseg + 2 + R) return fail(MSD_ERR_INVALID, "msd_stream_scan: no fixed point");
    }
    if (p->cfg.adaptive && !p->decide) {
        // the tiles whose fresh thresholds the fixed point reads: one more pass over every segment
        // from its final entry state (same results), marking them -- the speculative rounds above
        // would also mark tiles that only a wrong entry state reads.  Decisions-only mode lists
        // frames (near ties and triggers on predicted thresholds) in every round instead, appended at
        // the counter after d_done, which msd_stream_refine consumes and clears: a speculative
        // round lists a few frames more, each once, and no extra pass is needed
        MSD_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(p->d_active), 1, p->nseg, st));
        {
            KernelTimer timer(p->ctx, K_SSCAN);
            hipLaunchKernelGGL(scan_kernel, dim3((unsigned)p->nseg), dim3(64), 0, st, p->d_x + p->n_tail, p->d_fresh, P,
                               st_in(p), st_out(p), p->d_active, p->d_runs, p->d_nruns, p->d_margin, p->d_thr,
                               overflow, p->d_need, nullptr, nullptr, nullptr, nullptr, nullptr, cert);
        }
        MSD_HIP(hipGetLastError());
        MSD_HIP(hipMemsetAsync(p->d_active, 0, sizeof(int32_t) * p->nseg, st));
    }
    p->scanned = true;
    // mode 1 / 2 scanned every segment: with certification on, every segment's entries are current;
    // mode 0 re-scans some and keeps the others' (valid only if they were)
    if (!p->certify) p->cert_valid = false;
    else if (scan_mode != 0) p->cert_valid = true;
    if (exit_state) std::memcpy(exit_state, &ex, sizeof(SState));
    if (rounds) *rounds = nround;
    return MSD_OK;
}

int msd_stream_runs(msd_stream_plan *p, msd_det *runs, int64_t cap, int64_t *count, double *margin) {
    if (!p || !count) return fail(MSD_ERR_INVALID, "msd_stream_runs: null");
    *count = 0;
    if (margin) *margin = __builtin_inf();
    if (p->nseg == 0) return MSD_OK;
    if (!p->scanned) return fail(MSD_ERR_INVALID, "msd_stream_runs: call msd_stream_scan first");
    DeviceGuard g(p->ctx->device);
    hipStream_t st = p->ctx->stream;
    hipLaunchKernelGGL(runs_kernel, dim3(1), dim3(RK_T), 0, st, p->d_runs, p->d_nruns, p->nseg, p->cap, p->d_out,
                       p->d_count, p->d_pos);
    MSD_HIP(hipGetLastError());
    MSD_HIP(hipMemcpyAsync(&pin_hdr(p)->count, p->d_count, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    MSD_HIP(hipMemcpyAsync(pin_margin(p), p->d_margin, sizeof(double) * p->nseg, hipMemcpyDeviceToHost, st));
    MSD_HIP(hipStreamSynchronize(st));
    const int64_t n = pin_hdr(p)->count;
    *count = n;
    if (margin)
        for (int64_t i = 0; i < p->nseg; ++i) *margin = pin_margin(p)[i] < *margin ? pin_margin(p)[i] : *margin;
    if (n > cap) return fail(MSD_ERR_CAPACITY, "msd_stream_runs: more runs than capacity");
    if (n > 0) {
        if (!runs) return fail(MSD_ERR_INVALID, "msd_stream_runs: null runs");
        MSD_HIP(hipMemcpy(runs, p->d_out, sizeof(msd_det) * n, hipMemcpyDeviceToHost));
    }
    return MSD_OK;
}

int msd_stream_db(msd_stream_plan *p, msd_det *dets, int64_t n) {
    if (!p || (!dets && n)) return fail(MSD_ERR_INVALID, "msd_stream_db: null");
    if (n == 0) return MSD_OK;
    const int64_t x0 = p->frame0 - p->n_tail, x1 = p->frame0 + p->n_local + p->n_head;
    for (int64_t j = 0; j < n; ++j)
        if (dets[j].start < x0 || dets[j].stop > x1 || dets[j].stop <= dets[j].start)
            return fail(MSD_ERR_UNSUPPORTED, "msd_stream_db: run outside the shard and its halos");
    DeviceGuard g(p->ctx->device);
    hipStream_t st = p->ctx->stream;
    void *d = nullptr;
    if (int rc = ctx_scratch(p->ctx, 3, sizeof(msd_det) * n, &d)) return rc;
    MSD_HIP(hipMemcpyAsync(d, dets, sizeof(msd_det) * n, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(db_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, p->d_x, x0,
                       reinterpret_cast<msd_det *>(d), n);
    MSD_HIP(hipGetLastError());
    MSD_HIP(hipMemcpyAsync(dets, d, sizeof(msd_det) * n, hipMemcpyDeviceToHost, st));
    MSD_HIP(hipStreamSynchronize(st));
    return MSD_OK;
}

// The whole protocol for one process holding the whole stream (meteorgpu/stream.py
// StreamDetector.run at world size 1, same results), natively: no halos, the chunk sums added
// in order on the host, the scan / refine loop, the runs, the global-mode end quirk and the dB
// means computed on the plan's own run buffer -- two host round trips fewer than the call
// sequence, and no interpreter between the calls.
int msd_stream_detect_local(msd_stream_plan *p, int32_t exact_thresholds, msd_det *out, int64_t cap, int64_t *count,
                            double *thr0_out, double *margin, int32_t *rounds, int32_t *refined) {
    if (!p || !count || !thr0_out || !margin || !rounds || !refined)
        return fail(MSD_ERR_INVALID, "msd_stream_detect_local: null");
    if (p->frame0 != 0 || p->n_local != p->n_total)
        return fail(MSD_ERR_UNSUPPORTED, "msd_stream_detect_local: the plan must hold the whole stream");
    *count = 0;
    *margin = __builtin_inf();
    *rounds = 0;
    *refined = 0;
    const int64_t n = p->n_total;
    const bool adaptive = p->cfg.adaptive != 0;
    if (n == 0) {
        *thr0_out = NAN;
        if (!adaptive) return fail(MSD_ERR_INDEX, "index 0 is out of bounds for axis 0 with size 0");  // main.py:412
        return MSD_OK;
    }
    int rc;
    if (adaptive) {
        if ((rc = msd_stream_set_exact_thresholds(p, exact_thresholds))) return rc;
        if ((rc = msd_stream_fresh(p))) return rc;
    }
    // np.mean / np.std of the whole stream (main.py:464-466, :399-400): s = 0.0; s += chunk sums,
    // both passes and the sums on the device (the protocol's msd_stream_chunk_sums does the same
    // through the host for N ranks), one readback of thr0
    double thr0;
    {
        DeviceGuard g(p->ctx->device);
        hipStream_t st = p->ctx->stream;
        const int64_t nc = (n + CHUNK - 1) / CHUNK;
        const unsigned blocks = (unsigned)((nc + 3) / 4);
        double *stats = p->d_chunks + (n / CHUNK + 2);
        hipLaunchKernelGGL(chunk_sums_kernel<false>, dim3(blocks), dim3(256), 0, st, p->d_x, (int64_t)0, (int64_t)0, nc,
                           n, 0.0, nullptr, p->d_chunks);
        hipLaunchKernelGGL(stream_stats_kernel<0>, dim3(1), dim3(256), 0, st, p->d_chunks, nc, n, p->cfg.k_std, stats);
        hipLaunchKernelGGL(chunk_sums_kernel<true>, dim3(blocks), dim3(256), 0, st, p->d_x, (int64_t)0, (int64_t)0, nc,
                           n, 0.0, stats, p->d_chunks);
        hipLaunchKernelGGL(stream_stats_kernel<1>, dim3(1), dim3(256), 0, st, p->d_chunks, nc, n, p->cfg.k_std, stats);
        int64_t nbe = 0;
        if (p->certify) nbe = ed_sums_async(p, 0, n);  // thr0's error bound from the whole stream's ed
        MSD_HIP(hipGetLastError());
        MSD_HIP(hipMemcpyAsync(pin_chunks(p), stats + 1, sizeof(double), hipMemcpyDeviceToHost, st));
        if (p->certify)
            MSD_HIP(hipMemcpyAsync(pin_chunks(p) + 1, p->d_esum + nbe, sizeof(double2), hipMemcpyDeviceToHost, st));
        MSD_HIP(hipStreamSynchronize(st));
        thr0 = pin_chunks(p)[0];
        if (p->certify) p->terr0 = terr0_from(pin_chunks(p)[1], pin_chunks(p)[2], n, p->cfg.k_std);
    }
    *thr0_out = thr0;
    // the freeze / run scan to its fixed point, refined until it reads exact thresholds only
    const msd_stream_state clean{-1, -2, thr0, -1, p->terr0};
    msd_stream_state ex{};
    int32_t r = 0;
    if ((rc = msd_stream_scan(p, thr0, &clean, 1, &ex, &r))) return rc;
    *rounds = 1;
    while (adaptive) {
        int32_t c = 0;
        if ((rc = msd_stream_refine(p, &c))) return rc;
        *refined += c;
        if (c == 0) break;
        if ((rc = msd_stream_scan(p, thr0, &clean, 2, &ex, &r))) return rc;
        ++*rounds;
    }
    // runs of the shard, compacted on the device
    DeviceGuard g(p->ctx->device);
    hipStream_t st = p->ctx->stream;
    hipLaunchKernelGGL(runs_kernel, dim3(1), dim3(RK_T), 0, st, p->d_runs, p->d_nruns, p->nseg, p->cap, p->d_out,
                       p->d_count, p->d_pos);
    MSD_HIP(hipGetLastError());
    MSD_HIP(hipMemcpyAsync(&pin_hdr(p)->count, p->d_count, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    MSD_HIP(hipMemcpyAsync(pin_margin(p), p->d_margin, sizeof(double) * p->nseg, hipMemcpyDeviceToHost, st));
    MSD_HIP(hipStreamSynchronize(st));
    const int64_t nr = pin_hdr(p)->count;
    for (int64_t i = 0; i < p->nseg; ++i) *margin = pin_margin(p)[i] < *margin ? pin_margin(p)[i] : *margin;
    *count = nr;
    if (nr > cap) return fail(MSD_ERR_CAPACITY, "msd_stream_detect_local: more runs than capacity");
    if (nr == 0) return MSD_OK;
    if (!out) return fail(MSD_ERR_INVALID, "msd_stream_detect_local: null out");
    if (!adaptive) MSD_HIP(hipMemcpy(out + (nr - 1), p->d_out + (nr - 1), sizeof(msd_det), hipMemcpyDeviceToHost));
    if (!adaptive && out[nr - 1].stop == n) {  // burst_stops gets len-1 (main.py:414-415)
        out[nr - 1].stop = n - 1;
        if (out[nr - 1].stop - out[nr - 1].start <= 0)
            return fail(MSD_ERR_ASSERT, "Detection duration must be greater than 0");  // main.py:437
        MSD_HIP(hipMemcpyAsync(p->d_out + (nr - 1), out + (nr - 1), sizeof(msd_det), hipMemcpyHostToDevice, st));
    }
    // np.mean dB of every run (main.py:422-423, :501-502) on the run buffer itself
    hipLaunchKernelGGL(db_kernel, dim3((unsigned)((nr + 255) / 256)), dim3(256), 0, st, p->d_x, (int64_t)0, p->d_out,
                       nr);
    MSD_HIP(hipGetLastError());
    MSD_HIP(hipMemcpyAsync(out, p->d_out, sizeof(msd_det) * nr, hipMemcpyDeviceToHost, st));
    // certifying: the certificate's counts and slacks ride on the same sync
    if (p->certify && p->cert_valid) {
        if (int rc2 = cert_enqueue(p)) return rc2;
    }
    MSD_HIP(hipStreamSynchronize(st));
    p->cert_staged = p->certify && p->cert_valid;
    return MSD_OK;
}

}  // extern "C"
