// Internal declarations shared by the libmsdsp translation units.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/msdsp.h"

namespace msd {

void set_error(const std::string &msg);
int fail(int code, const std::string &msg);
int hip_fail(hipError_t e, const char *what);
// hipFuncAttributeMaxDynamicSharedMemorySize = bytes for `kernel` on the CURRENT device, once
// per (kernel, device); thread-safe (several contexts may launch from several threads)
int ensure_dyn_lds(const void *kernel, int bytes);

#define MSD_HIP(call)                                   \
    do {                                                \
        hipError_t e_ = (call);                         \
        if (e_ != hipSuccess) return hip_fail(e_, #call); \
    } while (0)

enum KernelId { K_STFT = 0, K_BLOCK = 1, K_DSTAT = 2, K_DSCAN = 3, K_WELCH = 4, K_LIVE = 5, K_CSTFT = 6, K_IQDELTA = 7, K_FRESH = 8, K_SSCAN = 9,
               K_REFINE = 10, K_CSTFT_DC = 11, K_COUNT = 12 };

struct EventPair {
    hipEvent_t a, b;
    int kernel;
};

}  // namespace msd

struct msd_ctx {
    int device = 0;
    int num_cu = 256;  // compute units (persistent-grid sizing)
    hipStream_t stream = nullptr;
    hipStream_t copy_stream = nullptr;  // host → HBM uploads (msd_memcpy_h2d_async), created on first use
    hipEvent_t fence_ev = nullptr;      // cross-stream ordering (msd_fence)
    hipEvent_t join_ev = nullptr;       // cross-context ordering (msd_stream_wait), this ctx signalling
    bool timing = false;
    uint32_t timing_mask = 0xffffffffu;  // msd_timing_select: kernel ids timed while timing is on
    bool force_generic = false;  // MSD_OPT_GENERIC_STFT
    bool fresh_all = false;      // MSD_OPT_FRESH_ALL
    std::vector<msd::EventPair> pending;  // recorded, not yet folded into totals
    std::vector<hipEvent_t> pool;         // reusable events
    double total_ms[msd::K_COUNT] = {};
    int64_t launches[msd::K_COUNT] = {};
    // scratch device buffers for the host-pointer convenience entry points
    // (slot 4: msd_iq_delta64_dev's block table, rotations and ranges; slot 5 unused since the
    // post-FFT detrend's side records went, round 5)
    void *scratch[8] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    size_t scratch_bytes[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // msd_iq_delta64_dev's twiddle table W^m (m < rf_w_n), built once per frame length
    double2 *rf_w = nullptr;
    int rf_w_n = 0;
    // its per-call tables staged in pinned memory (no stream sync), reusable once rf_ev has passed
    void *rf_pin = nullptr;
    size_t rf_pin_bytes = 0;
    hipEvent_t rf_ev = nullptr;
    // the tables of the last call as uploaded to scratch slot 4 (rf_last_dev): a call with the same
    // tables (every step of a stream of the same length) skips the two copies
    std::vector<char> rf_last;
    const void *rf_last_dev = nullptr;
    // the int8-MFMA block step's tables (refine_i8.hip): B fragments, column starts, lane twiddles,
    // built once per (frame length, bins)
    void *i8_tab = nullptr;
    uint64_t i8_key = 0;
    // ...and the exact (N, bins) they were built for: the hash only picks the candidate, a match
    // needs these equal (a hash collision must not reuse another geometry's tables)
    int i8_n = 0, i8_nk = 0;
    int i8_km[16] = {};
    bool refine_goertzel = false;  // MSD_OPT_REFINE_GOERTZEL: int16 refinement on the float64 Goertzel
    bool block_goertzel = false;   // MSD_OPT_BLOCK_GOERTZEL: int16 block energies on the float64 Goertzel
    bool welch_goertzel = false;   // MSD_OPT_WELCH_GOERTZEL: int16 Welch band powers on the float64 Goertzel
    int cstft_reserve = 0;         // MSD_OPT_CSTFT_RESERVE: workgroup slots the C5 spectrogram leaves free
    int cstft_sched = 0;           // MSD_OPT_CSTFT_SCHED: 0 / 2 chunks from a guided schedule, 1 fixed ranges
    int stft_sched = 0;            // MSD_OPT_STFT_SCHED: the same for stft1024_kernel (tiles)
    int num_cu_dev = 0;            // the device's CUs (num_cu: those the stream may use, MSD_OPT_STREAM_CUS)
    int stream_cus = 0;            // MSD_OPT_STREAM_CUS value in force
};

namespace msd {
// cos and sin of 2 pi j / N for any integer j, for host-built twiddle tables: j is reduced mod N into
// [-N/2, N/2] in exact integer arithmetic, the angle and the functions are evaluated in long double
// (x86-64: 64-bit significand), so each value rounded to double is within ~0.5 ulp of the exact one.
// (A double angle 2 pi m / N up to 2 pi is itself off by up to ~2 pi u, several u of twiddle error.)
inline void unit_root_ld(int64_t j, int64_t N, long double &c, long double &s) {
    int64_t r = j % N;
    if (r < 0) r += N;
    if (2 * r > N) r -= N;
    const long double a = 6.283185307179586476925286766559005768L * (long double)r / (long double)N;
    c = cosl(a);
    s = sinl(a);
}
}  // namespace msd

struct msd_stft_plan {
    msd_ctx *ctx = nullptr;
    int nperseg = 0, nfft = 0, hop = 0, M = 0;  // M = nfft/2 complex points, K = M + 1 bins
    int detrend = 1;                             // 1 constant (scipy), 0 none (matplotlib mlab)
    int precision = MSD_F32;                     // arithmetic and output type: MSD_F32 or MSD_F64
    double scale = 0;
    float *d_window = nullptr;   // [nperseg]  (MSD_F32 plans)
    float2 *d_tw = nullptr;      // [M]    exp(-2*pi*i*m/M)
    float2 *d_post = nullptr;    // [M+1]  exp(-2*pi*i*k/(2M))
    double *d_window64 = nullptr;  // the same three in float64 (MSD_F64 plans)
    double2 *d_tw64 = nullptr;
    double2 *d_post64 = nullptr;
    // stft1024_kernel's guided tile schedule (chunked, MSD_OPT_STFT_SCHED) and its ticket
    int64_t *d_sched = nullptr;
    int64_t sched_cap = 0, sched_total = -1, sched_wgs = -1, sched_n = 0;
    unsigned long long *d_ticket = nullptr;
    // stft1024_kernel, integer samples: the frame mean m = tot / 1024 = a + b / 1024 (a = floor) comes
    // off as the exact integer a before the FFT and as b / 1024 times the window's DFT after it, which
    // is exact when that DFT vanishes past bin 1 (periodic Hann: W_0 = N/2, W_1 = -N/4).  win_dft01:
    // W_0, W_1 of the float32 window in float64; win_dft_compact: max |W_k|, 2 <= k <= M, below
    // 1e-6 |W_0| (else integer input takes the generic kernel's exact two-part mean)
    double2 win_dft01[2] = {};
    int win_dft_compact = 0;
};

struct msd_block_plan {
    msd_ctx *ctx = nullptr;
    int64_t block_size = 0;
    int nfft = 0, L = 0;                  // L = min(B, nfft) samples used per block
    int band_lo = 0, band_hi = -1, noise_lo = 0, noise_hi = -1;
    int nbins = 0;                        // band bins + noise bins
    double *d_window = nullptr;           // [L]
    double2 *d_tw = nullptr;              // [nfft] exp(-2*pi*i*m/nfft)
    int *d_bins = nullptr;                // [nbins] bin indices, band first
    // fast path (nbins <= 64): per bin {2cos th, cos th, -sin th}, then per (bin, 16-lane
    // segment) the rotation exp(-i th (seg*SPL + SPL - 1)) — host-computed in float64
    double *d_bconst = nullptr;
    int spl = 0;                          // samples per lane segment of the fast path
    double2 *d_energy = nullptr;          // fast path: per block (band, noise) energy + 1e-12, grown
    size_t energy_cap = 0;                // blocks d_energy holds
    void *d_i8 = nullptr;                 // int16 blocks on the matrix cores (block_i8.hip): B fragments
                                          // + column constants, when block_i8_shape(L, nbins)
};

struct msd_welch_plan {
    msd_ctx *ctx = nullptr;
    msd_welch_cfg cfg{};
    int nseg = 0, step = 0;       // segments per block, nperseg - noverlap
    int nslots = 0;               // bins computed per block (band ranges concatenated)
    double *d_window = nullptr;   // [nperseg]
    double *d_bins = nullptr;     // [nslots][4]: cos w, sin w, 2 cos w, doubling factor (1 or 2)
    // int16 samples on the matrix cores (welch_i8.hip): B fragments and doubling factors of the
    // nct column tiles; null when the plan's shape does not take that path
    void *d_i8 = nullptr;
    int i8_nct = 0;
    bool i8_pairs = false;  // the accumulators' digit sums fit int32 pairs (welch_i8_build)
    bool i8_special = true;  // the live default's shape takes its own instantiation
};

namespace msd {

// workgroup barrier that orders LDS only: waits for this wave's LDS accesses, not for its
// global loads (prefetches) or stores still in flight.  __syncthreads() on gfx9 also waits
// vmcnt(0), which drains every outstanding prefetch and store at each barrier.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// a wave-uniform 64-bit value the compiler can keep in SGPRs (a load through x + uniform_i64(off) +
// lane offset then uses the scalar-base + 32-bit lane offset form, no per-lane 64-bit arithmetic)
__device__ __forceinline__ int64_t uniform_i64(int64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// DPP: v + v[lane ^ 1], v[lane ^ 2], mirrored half rows, mirrored rows → each lane
// holds the sum of its row of 16
__device__ __forceinline__ int row_sum_i(int v) {
    v += __builtin_amdgcn_mov_dpp(v, 0xB1, 0xf, 0xf, true);   // quad_perm [1,0,3,2]
    v += __builtin_amdgcn_mov_dpp(v, 0x4E, 0xf, 0xf, true);   // quad_perm [2,3,0,1]
    v += __builtin_amdgcn_mov_dpp(v, 0x141, 0xf, 0xf, true);  // row_half_mirror
    v += __builtin_amdgcn_mov_dpp(v, 0x140, 0xf, 0xf, true);  // row_mirror
    return v;
}
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), CTRL, 0xf, 0xf, true));
}
__device__ __forceinline__ float row_sum_f(float v) {
    v += dpp_f<0xB1>(v);
    v += dpp_f<0x4E>(v);
    v += dpp_f<0x141>(v);
    v += dpp_f<0x140>(v);
    return v;
}
// sum over the wave (uniform, in SGPRs): row sums by DPP, then the four rows by readlane
__device__ __forceinline__ int wave_sum_i(int v) {
    v = row_sum_i(v);
    return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
           __builtin_amdgcn_readlane(v, 48);
}
__device__ __forceinline__ float lane_f(float v, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
__device__ __forceinline__ float wave_sum_f(float v) {
    v = row_sum_f(v);
    return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
}

// int16 pairs packed in a 32-bit word (PCM16 samples, int16 I/Q): SDWA conversion of either half
// straight to float (no separate shift / bit-field extract), and integer sums by v_dot2 (one
// instruction adds both halves, or one of them, to an accumulator)
#ifndef MSD_NO_SDWA
__device__ __forceinline__ float cvt_i16_lo(uint32_t r) {
    float f;
    asm("v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0" : "=v"(f) : "v"(r));
    return f;
}
__device__ __forceinline__ float cvt_i16_hi(uint32_t r) {
    float f;
    asm("v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1" : "=v"(f) : "v"(r));
    return f;
}
typedef short msd_short2 __attribute__((ext_vector_type(2)));
template <int WLO, int WHI>
__device__ __forceinline__ int dot2_i16(uint32_t r, int acc) {
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(msd_short2, r), msd_short2{WLO, WHI}, acc, false);
}
#else
__device__ __forceinline__ float cvt_i16_lo(uint32_t r) { return (float)(int16_t)(r & 0xffffu); }
__device__ __forceinline__ float cvt_i16_hi(uint32_t r) { return (float)(int16_t)(r >> 16); }
template <int WLO, int WHI>
__device__ __forceinline__ int dot2_i16(uint32_t r, int acc) {
    return acc + WLO * (int)(int16_t)(r & 0xffffu) + WHI * (int)(int16_t)(r >> 16);
}
#endif

// makes `dev` current for the scope
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// scoped timing of one kernel launch on ctx->stream
struct KernelTimer {
    msd_ctx *ctx;
    int kernel;
    hipEvent_t a = nullptr, b = nullptr;
    KernelTimer(msd_ctx *c, int k);
    ~KernelTimer();
};

// a float constant held in a VGPR for the rest of the kernel: on gfx950 a VALU operand read from
// an SGPR issues at ~4.4 cycles per wave-instruction and a 32-bit literal at 2.65, a VGPR operand
// at 2.3 (VOP2) / 2.65 (VOP3) (tools/ubench/operand_rate.hip); the compiler hoists uniform constants
// into SGPRs or literals, the opaque move keeps this one in a VGPR
__device__ __forceinline__ float vgpr_f(float c) {
    float r;
    asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(c));
    return r;
}

// scratch buffer i of the context grown to at least `bytes`
int ctx_scratch(msd_ctx *ctx, int slot, size_t bytes, void **out);

// launchers (defined in the kernel translation units)
// out: float32 or float64 [nfiles][K][ld] by the plan's precision
int launch_stft(msd_stft_plan *plan, const void *x, int dtype, const int64_t *off, const int64_t *len, int64_t nfiles,
                int64_t max_frames, void *out, int64_t ld);
int launch_stft_any(msd_stft_plan *plan, const void *x, int dtype, const int64_t *off, const int64_t *len,
                    int64_t nfiles, void *out, int64_t ld);
int launch_stft1024(msd_stft_plan *plan, const void *x, int dtype, const int64_t *off, const int64_t *len,
                    int64_t nfiles, float *out, int64_t ld);
bool block_i8_shape(int64_t L, int nbins);
bool block_i8_window(const double *window, int64_t L);
bool welch_i8_shape(const msd_welch_cfg &c, int nseg, int nslots, const double *window);
int welch_i8_build(msd_welch_plan *p, const double *window);
int launch_welch_i8(msd_welch_plan *p, const int16_t *x, const int64_t *off, const int64_t *len, int64_t nfiles,
                    int64_t max_blocks, double *band_db, int64_t ld, double *psd);
int block_i8_build(msd_block_plan *p, const double *window, const int *bins, int nbins);
int launch_block_i8(msd_block_plan *p, const int16_t *x, const int64_t *off, const int64_t *len, int64_t nfiles,
                    int64_t max_blocks);
int launch_block_delta(msd_block_plan *plan, const void *x, int dtype, const int64_t *off, const int64_t *len,
                       int64_t nfiles, int64_t max_blocks, double *band_db, double *noise_db, double *delta,
                       int64_t ld);
int launch_detect(msd_ctx *ctx, const double *delta, const int64_t *nblocks, int64_t nfiles, int64_t ld,
                  const msd_det_cfg *cfg, msd_det *dets, int64_t cap, int64_t *counts, double *thresholds,
                  double *margin, int32_t *status, const msd_hist_cfg *hist);

inline size_t dtype_size(int dtype) {
    switch (dtype) {
        case MSD_U8: return 1;
        case MSD_I16: return 2;
        case MSD_I32: return 4;
        case MSD_F32: return 4;
        case MSD_F64: return 8;
        default: return 0;
    }
}

}  // namespace msd
