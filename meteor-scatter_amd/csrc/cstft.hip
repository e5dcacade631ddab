// Two-sided power spectrogram of complex (I/Q) input — BASELINE config C5 (192 kHz I/Q,
// 4096-point frames, 75 % overlap).  The quantity is scipy.signal.spectrogram(z, fs, 'hann',
// nperseg=N, noverlap=N-hop) for complex z (return_onesided switches to two-sided, bins in
// FFT order, |X|^2 / (fs * sum w^2), no doubling, complex64 arithmetic → float32 output).
//
// Mapping: one 256-thread workgroup transforms one frame at a time (persistent over a
// contiguous range of frames).  N = 4096 = 16 x 16 x 16:
//   pass 1  thread j holds z[j + 256 r] (r = 0..15, the coalesced load order): a 16-point
//           DFT over r in registers, then the twiddle W4096^(j q) (held in registers across
//           frames);
//   LDS     y[q][j] → thread (q, j1) gets y[q][j1 + 16 j2];
//   pass 2  16-point DFT over j2, twiddle W256^(j1 k2a) (LDS table);
//   LDS     → thread t = q + 16 k2a gets the 16 values over j1;
//   pass 3  16-point DFT over j1 → X[t + 256 k2b], k2b = 0..15.
// The powers leave frame-major, out[frame][k] (FFT order): 256 threads store 1 KB of
// consecutive bins per instruction, no output tile.  (A frequency-major [K][T] tile for
// K = 4096 would need 512 KB of LDS per 128-B row segment; scipy's [K][T] is the transpose of
// this layout.)  The window carries sqrt(scale), so |X|^2 is the density directly.
#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "msd_internal.h"

namespace msd {
namespace {

constexpr int CS_T = 256;              // threads per workgroup
constexpr int CS_N = 4096;             // frame length
// LDS layouts (float2 index) of the two transposes, chosen for the gfx950 bank model:
//   A (pass 1 → 2): y[q][c] at q*272 + c — the row pitch 272 ≡ 16 (mod 32) puts the two q rows
//     a half-wave reads into disjoint bank halves;
//   B (pass 2 → 3): u[q][c] at c*17 + q — column-major with an odd pitch: the pass-3 reads
//     (16 q values x 2 columns per half-wave) hit 64 distinct banks.
constexpr int CS_P = 272;
constexpr int CS_LDS_F2 = 16 * CS_P;   // float2 per frame buffer (= 256 * 17)

__device__ __forceinline__ float2 c_add(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 c_sub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 c_mul(float2 a, float2 b) {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 c_mi(float2 a) { return make_float2(a.y, -a.x); }  // a * (-i)

__device__ __forceinline__ void dft4(float2 &a0, float2 &a1, float2 &a2, float2 &a3) {
    const float2 t0 = c_add(a0, a2), t1 = c_sub(a0, a2), t2 = c_add(a1, a3), t3 = c_mi(c_sub(a1, a3));
    a0 = c_add(t0, t2);
    a1 = c_add(t1, t3);
    a2 = c_sub(t0, t2);
    a3 = c_sub(t1, t3);
}

// forward 16-point DFT, natural order in and out: n = n1 + 4 n2, k = k2 + 4 k1
__device__ __forceinline__ void dft16(float2 *v) {
    const float c1 = 0.92387953251128675613f, s1 = 0.38268343236508977173f, h = 0.70710678118654752440f;
#pragma unroll
    for (int n1 = 0; n1 < 4; ++n1) dft4(v[n1], v[n1 + 4], v[n1 + 8], v[n1 + 12]);  // v[n1 + 4 k2]
    // twiddles W16^(n1 k2)
    v[5] = c_mul(v[5], make_float2(c1, -s1));    // n1 1, k2 1: W^1
    v[9] = c_mul(v[9], make_float2(h, -h));      // n1 1, k2 2: W^2
    v[13] = c_mul(v[13], make_float2(s1, -c1));  // n1 1, k2 3: W^3
    v[6] = c_mul(v[6], make_float2(h, -h));      // n1 2, k2 1: W^2
    v[10] = c_mi(v[10]);                         // n1 2, k2 2: W^4 = -i
    v[14] = c_mul(v[14], make_float2(-h, -h));   // n1 2, k2 3: W^6
    v[7] = c_mul(v[7], make_float2(s1, -c1));    // n1 3, k2 1: W^3
    v[11] = c_mul(v[11], make_float2(-h, -h));   // n1 3, k2 2: W^6
    v[15] = c_mul(v[15], make_float2(-c1, s1));  // n1 3, k2 3: W^9
#pragma unroll
    for (int k2 = 0; k2 < 4; ++k2) dft4(v[4 * k2], v[4 * k2 + 1], v[4 * k2 + 2], v[4 * k2 + 3]);
    // v[4 k2 + k1] holds X[k2 + 4 k1]: reorder to natural
    float2 o[16];
#pragma unroll
    for (int k2 = 0; k2 < 4; ++k2)
#pragma unroll
        for (int k1 = 0; k1 < 4; ++k1) o[k2 + 4 * k1] = v[4 * k2 + k1];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = o[i];
}

template <typename T>
struct IQ;
template <>
struct IQ<int16_t> {  // interleaved int16 I, Q
    using raw_t = uint32_t;
    // non-temporal: 9.78 vs 9.86 ms for the C5 step's spectrogram (profiles/r5_cstft_nt_ab.txt)
    __device__ static raw_t load(const int16_t *p) {
        return __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(p));
    }
    __device__ static int re_i(raw_t r) { return (int)(int16_t)(r & 0xffffu); }
    __device__ static int im_i(raw_t r) { return (int)(int16_t)(r >> 16); }
    __device__ static float2 f(raw_t r) { return make_float2(cvt_i16_lo(r), cvt_i16_hi(r)); }
    using acc_t = int;
    __device__ static int wave_sum(int v) { return wave_sum_i(v); }
    // the thread's I and Q sums from the converted samples: float adds of integers stay exact
    // (|sum| <= 16 * 2^15 = 2^19), so full-rate v_add_f32 replace the quarter-rate v_dot2c
    template <int R0 = 0>
    __device__ static void thread_sums(const float2 *v, int &sr, int &si) {
        float a = 0.f, b = 0.f;
#pragma unroll
        for (int r = R0; r < 16; ++r) {
            a += v[r].x;
            b += v[r].y;
        }
        sr = (int)a;
        si = (int)b;
    }
    // the frame total from the four waves' exact sums (|total| < 2^28)
    __device__ static int total(const int *red) { return red[0] + red[1] + red[2] + red[3]; }
    // the same from an exact float64 total (msd_cstft_psd_fsums_dev: integer-valued)
    __device__ static int total_d(double t) { return (int)t; }
    // the mean total / 4096 as hi + lo, both exact: hi = float(total) / 4096 (float(total) rounds
    // the integer to 24 bits; |total| < 2^24, i.e. |mean| < 4096, is exact already and lo = 0), lo =
    // (total - float(total)) / 4096 (an integer of at most 4 bits / 4096)
    __device__ static void mean2(int tot, float &hi, float &lo) {
        const float f = (float)tot;
        hi = f * (1.0f / CS_N);
        lo = (float)(tot - (int)f) * (1.0f / CS_N);
    }
};
template <>
struct IQ<float> {  // interleaved float32 I, Q (complex64)
    using raw_t = float2;
    __device__ static raw_t load(const float *p) { return *reinterpret_cast<const float2 *>(p); }
    __device__ static float2 f(raw_t r) { return r; }
    using acc_t = float;
    __device__ static float wave_sum(float v) { return wave_sum_f(v); }
    template <int R0 = 0>
    __device__ static void thread_sums(const float2 *v, float &sr, float &si) {
        sr = 0.f;
        si = 0.f;
#pragma unroll
        for (int r = R0; r < 16; ++r) {
            sr += v[r].x;
            si += v[r].y;
        }
    }
    __device__ static double total(const float *red) {
        return (double)red[0] + (double)red[1] + (double)red[2] + (double)red[3];
    }
    __device__ static double total_d(double t) { return t; }
    // mean = hi + lo to float64 precision (hi its float32 rounding, lo the float32 of the rest)
    __device__ static void mean2(double tot, float &hi, float &lo) {
        const double m = tot * (1.0 / CS_N);
        hi = (float)m;
        lo = (float)(m - (double)hi);
    }
};

// int16 I/Q runs 4 waves per SIMD: 128 VGPRs with the [k][j1] pass-2 twiddle table (its reads need
// no per-k index registers; 8-68 B of spills, outside the frame loop) — A/B at hop 1024 (C5)
// 12.27 → 11.79 ms, hop 2048 6.38 → 6.19, hop 1000 13.05 → 12.53.  float32 I/Q keeps 3 waves and the
// W256^m table (at 4 waves it spills inside the loop, 12.33 → 14.55 ms; the [k][j1] table alone at 3
// waves is 2 % slower)
template <typename T, int SH>
struct CsTune {
    static constexpr bool kW4 = std::is_same<T, int16_t>::value;
    static constexpr int kWavesPerSimd = kW4 ? 4 : 1;  // launch-bounds minimum (1: no constraint)
};

// SH = hop / 256 when the hop is a multiple of 256 below N (C5: hop 1024 → 4), else 0.
// Thread j holds z[j + 256 r]; the next frame of the same stream needs z[j + 256 (r + SH)],
// so with SH > 0 it keeps raw[SH..15] (shifted down) and loads only raw[16-SH..15]: each
// sample is loaded once per workgroup instead of N / hop times.
// EN: also an upper bound of each frame's total power in 16 partials, etot[i][stride] (partial i =
// row r of 16 lanes of wave w at 4 w + r): by Parseval the input norm behind the fp32 FFT's per-bin
// error bound (the C5 detector's delta error bound, msd_iq_band_delta_bound_dev).  Each thread
// keeps the max of its 16 powers' sum over a group of 4 consecutive frames; at the group's last
// frame a row DPP reduction gives the row's partial (>= every frame's: a sum of maxima), stored for
// each frame of the group -- 16 adds and a max per thread and frame, the reduction and 4 stores per
// 4 frames (per frame: +5.6 % of the kernel, 12.03 -> 12.71 ms at C5)
// Detrend (scipy 'constant', before the window): the frame's complex mean m is subtracted from every
// sample in float32 as (x - hi) - lo, m = hi + lo both exact (IQ<T>::mean2), so the detrended sample
// is the float32 rounding of the float64 x - m.  A single float32 mean would leave the coherent error
// |m - float(m)| <= 2^-24 |m| in every sample, i.e. a residual DC of that size at bins 0, +-1 (for
// int16 I/Q from |m| >= 4096 on: up to 2e-3 relative per frame against scipy at a 16000 offset over
// quiet noise, tools/dbg/dc_precision.py); lo is zero below that and the frame then takes the
// one-subtraction path (a wave-uniform branch).  The round-4 post-FFT detrend (FFT of w x, bins 0,
// +-1 corrected afterwards) was cheaper but its rounding scales with the DC energy in EVERY bin:
// 2.7e-5 per frame at a 700 offset over sigma-3 noise; removed.
// PD 0: the sums in the kernel (exact integer DPP sums per wave, one LDS slot per wave, a barrier);
// PD 2 (msd_cstft_psd_fsums_dev): the frames' sums given (fsum[g], the exact delta step's): no
// reduction and no barrier before pass 1, the next frame's sums prefetched with its samples.
// DYN (C5's hop, the default): the workgroups take chunks of frames from a guided schedule (sched[k] ..
// sched[k + 1], sizes falling from ~total / (4 wgs) to 16 frames) by an atomic ticket instead of one
// fixed range each.  With fixed ranges the slowest workgroup sets the launch's end -- one on a slower
// CU, or one that started late because kernels on another stream (the C5 detector beside the
// spectrogram) held its slot when the grid was dispatched; with chunks the others take its share.
// Measured: 11.79 -> 10.62 ms alone, 10.35 ms beside the detector (bench C5, one box; chunks of 1 / (2
// wgs) of the rest), 9.73-9.81 ms with 1 / (4 wgs).
template <typename T, int SH, bool EN, int PD, bool DYN = false>
__global__ __launch_bounds__(CS_T, (CsTune<T, SH>::kWavesPerSimd)) void cstft4096_kernel(
    const T *__restrict__ x, const int64_t *__restrict__ off, const int64_t *__restrict__ len, int64_t nstreams,
    int64_t max_frames, int64_t total, int64_t per, int hop, int detrend, const float *__restrict__ g_win,
    const float2 *__restrict__ g_tw, float *__restrict__ out, float *__restrict__ etot, int64_t estride,
    const double2 *__restrict__ fsum, const int64_t *__restrict__ sched, int64_t nchunks,
    unsigned long long *__restrict__ ticket) {
    using io = IQ<T>;
    __shared__ float2 buf[CS_LDS_F2];
    // pass-2 twiddles W256^(j1 k).  kW4: at k * 16 + j1 — a half-wave reads 16 consecutive entries
    // (its two q values share them), conflict-free, the row an immediate offset, no index
    // registers; else W256^m at m = (j1 k) & 255 (2- to 8-way conflicts for even k: 10 extra LDS
    // cycles per wave and frame)
    constexpr bool W4 = CsTune<T, SH>::kW4;
    __shared__ float2 tw2[256];
    __shared__ typename io::acc_t red[2][CS_T / 64];
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < 256; i += CS_T)  // W256^x = W4096^(16 x)
        tw2[i] = g_tw[16 * (W4 ? ((i & 15) * (i >> 4)) & 255 : i)];
    // per-thread constants: window (x sqrt(scale)) and the pass-1 twiddles W4096^(j q)
    float wr[16];
    float2 tw1[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        wr[r] = g_win[tid + 256 * r];
        tw1[r] = g_tw[(tid * r) & (CS_N - 1)];
    }
    float *const ep = EN ? etot + (int64_t)(wave * 4 + (lane >> 4)) * estride : nullptr;  // this row's partials
    float emax = 0.f;  // EN: max over the frames of the current group of this thread's power sum
    const int q2 = tid >> 4, j1 = tid & 15;   // pass-2 thread: (q, j1)
    const int q3 = tid & 15, k2a = tid >> 4;  // pass-3 thread: t = q + 16 k2a
    __syncthreads();

    typename io::raw_t raw[16];
    // load rows [R0, 16) of frame t of the stream at element offset `base`
    auto load_rows = [&](int64_t base, int64_t t, auto r0c) {
        constexpr int R0 = decltype(r0c)::value;
        const T *p = x + 2 * uniform_i64(base + t * (int64_t)hop);
#pragma unroll
        for (int r = R0; r < 16; ++r) raw[r] = io::load(p + 2 * (tid + 256 * r));
    };
    // A range of frames [g0, g1) split at stream boundaries: per segment, the frames of the stream
    // [ga, gv) and then the frames past its end [gv, gb), written as zeros.  Within [ga, gv) the
    // prefetch of frame t + 1 is unconditional (clamped to the last frame at the end), so the
    // register rows never pass through data-dependent copies.
    auto run_range = [&](const int64_t g0, const int64_t g1) __attribute__((always_inline)) {
    for (int64_t ga = g0; ga < g1;) {
        const int64_t s = ga / max_frames;
        const int64_t gb = (s + 1) * max_frames < g1 ? (s + 1) * max_frames : g1;
        const int64_t n = len[s];
        const int64_t nfr = n >= CS_N ? (n - CS_N) / hop + 1 : 0;
        const int64_t ge = s * max_frames + nfr;  // end of the stream's frames
        const int64_t gv = ge < ga ? ga : ge > gb ? gb : ge;
        const int64_t base = off[s];
        float *of = out + ga * (int64_t)CS_N;
        // one frame: consumes raw (frame g), prefetches frame g + 1 into raw, writes `of`
        double2 fnext = make_double2(0.0, 0.0);  // PD 2: the sums of the frame raw holds
        // float32 I/Q, PD 0: the frame's first sample, subtracted before the float sums so that they
        // accumulate the variation, not the offset (a float sum of 4096 values near a DC m is off by
        // ~24 u |m|, which would leave that as a residual DC); the mean is then xref + sum / 4096
        constexpr bool REF = std::is_same<T, float>::value && PD == 0;
        float2 xnext = make_float2(0.f, 0.f);
        auto first_sample = [&](int64_t t) {
            return *reinterpret_cast<const float2 *>(x + 2 * uniform_i64(base + t * (int64_t)hop));
        };
        auto frame = [&](int64_t g, float *of) __attribute__((always_inline)) {
            float2 v[16];
            // ---- detrend: the frame's complex mean (scipy 'constant'): exact integer sums for
            // int16 I/Q (|sum| < 2^28), float sums for float32 I/Q; PD 0: per wave, then one LDS
            // slot per wave; PD 2: given
#pragma unroll
            for (int r = 0; r < 16; ++r) v[r] = io::f(raw[r]);
            const float2 xref = xnext;
            if constexpr (REF) {
                if (detrend) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) v[r] = c_sub(v[r], xref);
                }
            }
            if constexpr (PD == 0) {
                typename io::acc_t sr, si;
                io::thread_sums(v, sr, si);
                sr = io::wave_sum(sr);  // DPP row sums + readlane: no LDS round trips
                si = io::wave_sum(si);
                if (lane == 0) {
                    red[0][wave] = sr;
                    red[1][wave] = si;
                }
            }
            const double2 fcur = fnext;
            {  // prefetch frame t + 1 (raw is consumed); the segment's last frame reloads itself
                const int64_t tn = (g + 1 < gv ? g + 1 : g) - s * max_frames;
                if constexpr (SH > 0) {  // (after the segment's last frame raw is dead)
#pragma unroll
                    for (int r = 0; r < 16 - SH; ++r) raw[r] = raw[r + SH];
                    load_rows(base, tn, std::integral_constant<int, (SH > 0 ? 16 - SH : 0)>{});
                } else {
                    load_rows(base, tn, std::integral_constant<int, 0>{});
                }
                if constexpr (PD == 2) fnext = fsum[uniform_i64(s * max_frames + tn)];
                if constexpr (REF) xnext = first_sample(tn);
            }
            float mr = 0.f, lr = 0.f, mi = 0.f, li = 0.f;
            if constexpr (PD == 2) {
                io::mean2(io::total_d(fcur.x), mr, lr);
                io::mean2(io::total_d(fcur.y), mi, li);
            } else {
                lds_barrier();
                io::mean2(io::total(red[0]), mr, lr);
                io::mean2(io::total(red[1]), mi, li);
            }
            if (!detrend) mr = lr = mi = li = 0.f;
            // lo is wave-uniform: a branch, not a select -- frames with |mean| < 4096 (int16) pay one
            // subtraction per value
            if (__builtin_amdgcn_readfirstlane(lr != 0.f || li != 0.f)) {
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    v[r] = make_float2(((v[r].x - mr) - lr) * wr[r], ((v[r].y - mi) - li) * wr[r]);
            } else {
#pragma unroll
                for (int r = 0; r < 16; ++r) v[r] = make_float2((v[r].x - mr) * wr[r], (v[r].y - mi) * wr[r]);
            }
            // ---- pass 1: DFT over r, twiddle W4096^(j q), y[q][j]
            dft16(v);
#pragma unroll
            for (int q = 1; q < 16; ++q) v[q] = c_mul(v[q], tw1[q]);
            if constexpr (PD == 2) lds_barrier();  // everyone has read the previous frame's pass-2 layout
#pragma unroll
            for (int q = 0; q < 16; ++q) buf[q * CS_P + tid] = v[q];
            lds_barrier();
            // ---- pass 2: thread (q, j1): DFT over j2 of y[q][j1 + 16 j2], twiddle W256^(j1 k2a)
#pragma unroll
            for (int j2 = 0; j2 < 16; ++j2) v[j2] = buf[q2 * CS_P + j1 + 16 * j2];
            dft16(v);
#pragma unroll
            for (int k = 1; k < 16; ++k) v[k] = c_mul(v[k], tw2[W4 ? 16 * k + j1 : (j1 * k) & 255]);
            lds_barrier();  // everyone has read pass 1's layout
#pragma unroll
            for (int k = 0; k < 16; ++k) buf[(16 * k + j1) * 17 + q2] = v[k];  // u[q][k2a][j1], column-major
            lds_barrier();
            // ---- pass 3: thread t = q + 16 k2a: DFT over j1 → X[t + 256 k2b]
#pragma unroll
            for (int j = 0; j < 16; ++j) v[j] = buf[(16 * k2a + j) * 17 + q3];
            dft16(v);
            // the frame's 16 KB through a buffer resource on its (wave-uniform) base: the thread's
            // byte offset in a VGPR, the row offset 1 KB * k2b as the scalar offset, no per-lane
            // 64-bit address arithmetic; streaming (non-temporal) stores, written once (A/B: -1 to -2 %)
            const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
                reinterpret_cast<float *>(uniform_i64(reinterpret_cast<int64_t>(of))), 0, CS_N * 4, 0x00020000);
            float esum = 0.f;
#pragma unroll
            for (int k2b = 0; k2b < 16; ++k2b) {
                const float pw = v[k2b].x * v[k2b].x + v[k2b].y * v[k2b].y;
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, pw), rsrc, 4 * tid, 1024 * k2b, 2 /* nt */);
                if constexpr (EN) esum += pw;
            }
            if constexpr (EN) {
                emax = fmaxf(emax, esum);
                // groups of 4 frames from the workgroup's first (per is a multiple of 4): flush at
                // the group's last frame or the segment's
                const int64_t gr = g - g0;
                if ((gr & 3) == 3 || g + 1 == gv) {
                    const float e = row_sum_f(emax);
                    if ((lane & 15) == 0)  // the group's frames in this segment
                        for (int64_t q = (g - (gr & 3) > ga ? g - (gr & 3) : ga); q <= g; ++q) ep[q] = e;
                    emax = 0.f;
                }
            }
            // no barrier at the end: the next frame writes buf (and, PD 0, red) only after its first
            // barrier, which every wave reaches after its pass-3 reads of this frame
        };
        // The first frame is peeled off the loop: both ways into the loop then end with the
        // prefetch loads followed by this frame's 16 stores, so the compiler's wait for the
        // prefetched rows is vmcnt(16) — it never waits for the stores (gfx9 counts loads and
        // stores in one vmcnt; a loop entered straight after a load would wait vmcnt(0)).
        if (ga < gv) {
            load_rows(base, ga - s * max_frames, std::integral_constant<int, 0>{});
            if constexpr (PD == 2) fnext = fsum[uniform_i64(ga)];
            if constexpr (REF) xnext = first_sample(ga - s * max_frames);
            frame(ga, of);
            of += CS_N;
            for (int64_t g = ga + 1; g < gv; ++g, of += CS_N) frame(g, of);
        }
        for (int64_t g = gv; g < gb; ++g, of += CS_N)  // frames past a shorter stream's end
#pragma unroll
            for (int k2b = 0; k2b < 16; ++k2b) of[tid + 256 * k2b] = 0.f;
        ga = gb;
    }
    };
    if constexpr (!DYN) {
        const int64_t g0 = (int64_t)blockIdx.x * per;
        run_range(g0, g0 + per < total ? g0 + per : total);
    } else {
        // thread 0 draws the next chunk while the current one runs (double-buffered slot); the barrier
        // after a chunk publishes it and ends every wave's use of the chunk's LDS
        __shared__ int64_t slot[2];
        if (tid == 0) slot[0] = (int64_t)atomicAdd(ticket, 1ull);
        __syncthreads();
        int64_t k = uniform_i64(slot[0]);
        int par = 0;
        while (k < nchunks) {
            if (tid == 0) slot[par ^ 1] = (int64_t)atomicAdd(ticket, 1ull);
            run_range(uniform_i64(sched[k]), uniform_i64(sched[k + 1]));
            __syncthreads();
            k = uniform_i64(slot[par ^ 1]);
            par ^= 1;
        }
    }
}

}  // namespace
}  // namespace msd

struct msd_cstft_plan {
    msd_ctx *ctx = nullptr;
    int nperseg = 0, hop = 0, detrend = 1;
    float *d_win = nullptr;   // window x sqrt(scale)
    float2 *d_tw = nullptr;   // W4096^m, m = 0..4095
    // DYN: the guided chunk schedule for (sched_total frames, sched_wgs workgroups) and the ticket
    int64_t *d_sched = nullptr;
    int64_t sched_cap = 0, sched_total = -1, sched_wgs = -1, sched_n = 0;
    unsigned long long *d_ticket = nullptr;
};

using namespace msd;

extern "C" {

int msd_cstft_plan_create(msd_ctx *ctx, int32_t nperseg, int32_t hop, const float *window, double scale,
                          msd_cstft_plan **out) {
    if (!ctx || !window || !out) return fail(MSD_ERR_INVALID, "msd_cstft_plan_create: null");
    *out = nullptr;
    if (nperseg != CS_N) return fail(MSD_ERR_UNSUPPORTED, "cstft: nperseg must be 4096");
    if (hop <= 0 || hop > nperseg) return fail(MSD_ERR_INVALID, "cstft: need 0 < hop <= nperseg");
    if (!(scale > 0)) return fail(MSD_ERR_INVALID, "cstft: scale must be > 0");
    DeviceGuard g(ctx->device);
    auto *p = new msd_cstft_plan();
    p->ctx = ctx;
    p->nperseg = nperseg;
    p->hop = hop;
    std::vector<float> w(nperseg);
    const double rs = std::sqrt(scale);
    for (int i = 0; i < nperseg; ++i) w[i] = (float)((double)window[i] * rs);
    std::vector<float2> tw(CS_N);
    for (int m = 0; m < CS_N; ++m) {
        const double a = -2.0 * M_PI * (double)m / (double)CS_N;
        tw[m] = make_float2((float)std::cos(a), (float)std::sin(a));
    }
    hipError_t e = hipMalloc(&p->d_win, sizeof(float) * nperseg);
    if (e == hipSuccess) e = hipMalloc(&p->d_tw, sizeof(float2) * CS_N);
    if (e == hipSuccess) e = hipMemcpy(p->d_win, w.data(), sizeof(float) * nperseg, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(p->d_tw, tw.data(), sizeof(float2) * CS_N, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        msd_cstft_plan_destroy(p);
        return hip_fail(e, "msd_cstft_plan_create");
    }
    *out = p;
    return MSD_OK;
}

void msd_cstft_plan_destroy(msd_cstft_plan *p) {
    if (!p) return;
    DeviceGuard g(p->ctx->device);
    (void)hipStreamSynchronize(p->ctx->stream);
    if (p->d_win) (void)hipFree(p->d_win);
    if (p->d_tw) (void)hipFree(p->d_tw);
    if (p->d_sched) (void)hipFree(p->d_sched);
    if (p->d_ticket) (void)hipFree(p->d_ticket);
    delete p;
}

int msd_cstft_set_detrend(msd_cstft_plan *p, int detrend) {
    if (!p || (detrend != 0 && detrend != 1)) return fail(MSD_ERR_INVALID, "msd_cstft_set_detrend: bad args");
    p->detrend = detrend;
    return MSD_OK;
}

int64_t msd_cstft_frames(const msd_cstft_plan *p, int64_t n) {
    if (!p || n < p->nperseg) return 0;
    return (n - p->nperseg) / p->hop + 1;
}

int msd_cstft_psd_dev(msd_cstft_plan *p, const void *x, int dtype, const int64_t *off, const int64_t *len,
                      int64_t nstreams, int64_t max_frames, float *out) {
    return msd_cstft_psd_energy_dev(p, x, dtype, off, len, nstreams, max_frames, out, nullptr);
}

int64_t msd_cstft_energy_stride(int64_t nstreams, int64_t max_frames) { return (nstreams * max_frames + 3) / 4 * 4; }

int msd_cstft_psd_energy_dev(msd_cstft_plan *p, const void *x, int dtype, const int64_t *off, const int64_t *len,
                             int64_t nstreams, int64_t max_frames, float *out, float *etot) {
    return msd_cstft_psd_fsums_dev(p, x, dtype, off, len, nstreams, max_frames, out, etot, nullptr);
}

int msd_cstft_psd_fsums_dev(msd_cstft_plan *p, const void *x, int dtype, const int64_t *off, const int64_t *len,
                            int64_t nstreams, int64_t max_frames, float *out, float *etot, const double *frame_sums) {
    const double2 *fsum = reinterpret_cast<const double2 *>(frame_sums);
    if (!p || (nstreams > 0 && (!x || !off || !len || !out))) return fail(MSD_ERR_INVALID, "msd_cstft_psd_dev: null");
    if (dtype != MSD_CI16 && dtype != MSD_CF32) return fail(MSD_ERR_UNSUPPORTED, "cstft: dtype must be CI16 or CF32");
    if (nstreams == 0 || max_frames == 0) return MSD_OK;
    DeviceGuard g(p->ctx->device);
    const int64_t total = nstreams * max_frames;
    // persistent: as many workgroups as stay resident (registers and the 37 KB of LDS decide; the
    // compiler's register count sets 3 or 4 per CU), less the reserve
    auto grid = [&](auto kern) {
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, CS_T, 0) != hipSuccess || per_cu < 1)
            per_cu = 3;
        int64_t wgs = (int64_t)p->ctx->num_cu * per_cu - p->ctx->cstft_reserve;
        if (wgs < 1) wgs = 1;
        return wgs > total ? total : wgs;
    };
    auto launch = [&](auto kern, const auto *xp) -> int {
        int64_t wgs = grid(kern);
        int64_t per = (total + wgs - 1) / wgs;
        if (etot) per = (per + 3) / 4 * 4;  // energy groups of 4 frames start at every workgroup's first
        wgs = (total + per - 1) / per;
        KernelTimer timer(p->ctx, K_CSTFT);  // the FFT kernel alone: the roofline's
        hipLaunchKernelGGL(kern, dim3((unsigned)wgs), dim3(CS_T), 0, p->ctx->stream, xp, off, len, nstreams,
                           max_frames, total, per, p->hop, p->detrend, p->d_win, p->d_tw, out, etot,
                           msd_cstft_energy_stride(nstreams, max_frames), fsum, nullptr, (int64_t)0, nullptr);
        return MSD_OK;
    };
    // DYN: the guided schedule (multiples of 4 frames: the energy groups), built when (total, wgs)
    // change, and the ticket zeroed on the stream before every launch
    auto launch_dyn = [&](auto kern, const auto *xp) -> int {
        const int64_t wgs = grid(kern);
        if (p->sched_total != total || p->sched_wgs != wgs) {
            std::vector<int64_t> st(1, 0);
            // guided: each chunk 1 / (div * wgs) of what is left, at least cmin frames (A/B knobs:
            // MSD_CSTFT_GUIDE="cmin,div"; bench C5 on one box, profiles/r5_c5_sched_overlap.txt: div 1
            // 13.06 ms, 2 10.19, 4 9.73-9.81, 8 9.81, 16 9.88; fixed 16 / 32 / 64 / 128-frame chunks
            // 9.95 / 9.91 / 9.94 / 10.02 -- the workgroups working on nearby frames, not only the
            // balance, pays)
            int64_t cmin = 16, div = 4;
            if (const char *e = getenv("MSD_CSTFT_GUIDE")) {
                long a = 0, b = 0;
                if (sscanf(e, "%ld,%ld", &a, &b) == 2 && a >= 4 && b >= 1) cmin = a, div = b;
            }
            for (int64_t pos = 0; pos < total;) {
                int64_t sz = (total - pos) / (div * wgs);
                sz = (std::max<int64_t>(sz, cmin) + 3) / 4 * 4;
                pos = std::min(total, pos + sz);
                st.push_back(pos);
            }
            DeviceGuard dg(p->ctx->device);
            MSD_HIP(hipStreamSynchronize(p->ctx->stream));
            if ((int64_t)st.size() > p->sched_cap) {
                if (p->d_sched) MSD_HIP(hipFree(p->d_sched));
                p->d_sched = nullptr;
                p->sched_cap = 0;
                MSD_HIP(hipMalloc(&p->d_sched, sizeof(int64_t) * st.size()));
                p->sched_cap = (int64_t)st.size();
            }
            if (!p->d_ticket) MSD_HIP(hipMalloc(&p->d_ticket, sizeof(unsigned long long)));
            MSD_HIP(hipMemcpy(p->d_sched, st.data(), sizeof(int64_t) * st.size(), hipMemcpyHostToDevice));
            p->sched_total = total;
            p->sched_wgs = wgs;
            p->sched_n = (int64_t)st.size() - 1;
        }
        MSD_HIP(hipMemsetAsync(p->d_ticket, 0, sizeof(unsigned long long), p->ctx->stream));
        KernelTimer timer(p->ctx, K_CSTFT);
        hipLaunchKernelGGL(kern, dim3((unsigned)wgs), dim3(CS_T), 0, p->ctx->stream, xp, off, len, nstreams,
                           max_frames, total, (int64_t)0, p->hop, p->detrend, p->d_win, p->d_tw, out, etot,
                           msd_cstft_energy_stride(nstreams, max_frames), fsum, p->d_sched, p->sched_n,
                           p->d_ticket);
        return MSD_OK;
    };
    const int sh = p->hop % 256 == 0 ? p->hop / 256 : 0;
    // the given sums (PD 2) at C5's hop: the int16 exact delta step leaves them (frames that start
    // every 1024 samples); other hops compute their own
    const bool given = fsum && p->detrend && sh == 4;
    // the chunked kernels at C5's hop unless MSD_OPT_CSTFT_SCHED asks for fixed ranges: they balance
    // the workgroups' unequal speeds as well as late starts (A/B on one box, bench C5 exact mode:
    // 11.79 -> 10.62 ms for the kernel alone, profiles/r5_c5_sched_overlap.txt)
    const bool dyn = p->ctx->cstft_sched != 1;
    auto by_shift = [&](auto en, const auto *xp) -> int {
        constexpr bool EN = decltype(en)::value;
        using T = std::remove_cv_t<std::remove_pointer_t<decltype(xp)>>;
        if (sh == 4) {  // 75 % overlap (C5)
            if (dyn) return given ? launch_dyn(cstft4096_kernel<T, 4, EN, 2, true>, xp)
                                  : launch_dyn(cstft4096_kernel<T, 4, EN, 0, true>, xp);
            return given ? launch(cstft4096_kernel<T, 4, EN, 2>, xp) : launch(cstft4096_kernel<T, 4, EN, 0>, xp);
        }
        if (sh == 8) return launch(cstft4096_kernel<T, 8, EN, 0>, xp);  // 50 %
        return launch(cstft4096_kernel<T, 0, EN, 0>, xp);
    };
    auto by_energy = [&](const auto *xp) -> int {
        if (etot) return by_shift(std::integral_constant<bool, true>{}, xp);
        return by_shift(std::integral_constant<bool, false>{}, xp);
    };
    const int rc = dtype == MSD_CI16 ? by_energy(static_cast<const int16_t *>(x)) : by_energy(static_cast<const float *>(x));
    if (rc) return rc;
    MSD_HIP(hipGetLastError());
    return MSD_OK;
}

int msd_cstft_psd(msd_cstft_plan *p, const void *x, int dtype, int64_t n, float *out, int64_t *frames) {
    if (!p || (!x && n) || !out) return fail(MSD_ERR_INVALID, "msd_cstft_psd: null");
    const size_t es = dtype == MSD_CI16 ? 4 : dtype == MSD_CF32 ? 8 : 0;
    if (!es) return fail(MSD_ERR_UNSUPPORTED, "cstft: dtype must be CI16 or CF32");
    const int64_t T = msd_cstft_frames(p, n);
    if (frames) *frames = T;
    if (T == 0) return MSD_OK;
    msd_ctx *ctx = p->ctx;
    DeviceGuard g(ctx->device);
    void *dx, *dmeta, *dout;
    int rc;
    if ((rc = ctx_scratch(ctx, 0, ((size_t)n * es + 255) / 256 * 256, &dx))) return rc;
    if ((rc = ctx_scratch(ctx, 1, 64, &dmeta))) return rc;
    if ((rc = ctx_scratch(ctx, 2, sizeof(float) * CS_N * (size_t)T, &dout))) return rc;
    int64_t meta[2] = {0, n};
    MSD_HIP(hipMemcpyAsync(dx, x, (size_t)n * es, hipMemcpyHostToDevice, ctx->stream));
    MSD_HIP(hipMemcpyAsync(dmeta, meta, sizeof(meta), hipMemcpyHostToDevice, ctx->stream));
    const int64_t *doff = static_cast<const int64_t *>(dmeta);
    rc = msd_cstft_psd_dev(p, dx, dtype, doff, doff + 1, 1, T, static_cast<float *>(dout));
    if (rc) return rc;
    MSD_HIP(hipMemcpyAsync(out, dout, sizeof(float) * CS_N * (size_t)T, hipMemcpyDeviceToHost, ctx->stream));
    MSD_HIP(hipStreamSynchronize(ctx->stream));
    return MSD_OK;
}

}  // extern "C"
