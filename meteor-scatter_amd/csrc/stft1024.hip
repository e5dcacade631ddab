// Fast path of the STFT power spectrogram for nperseg = nfft = 1024 (the headline
// configuration: scipy.signal.spectrogram(x, fs, 'hann', 1024, 512) as called at
// dsp/src/main.py:52-54 / :132-133 and BASELINE configs C1-C4).
//
// Mapping.  A wave transforms two frames at once (two independent
// instruction streams, interleaved by the compiler), 64 lanes x 8 complex points
// per frame, every radix-8 Stockham pass in registers:
//   load    lane l holds z[l + 64 r] = x[2(l+64r)] + i x[2(l+64r)+1] (r = 0..7): one
//           sample pair per lane per instruction, 256 B coalesced per wave;
//   detrend frame mean from an exact integer reduction: DPP adds inside each row of
//           16 lanes, then four v_readlane (no LDS round trip);
//   pass 1  → LDS transpose → pass 2 → LDS transpose → pass 3: lane l computes the
//           pass-3 butterfly pi(l) (a table: conjugate pairs j, 64-j in adjacent lanes,
//           pi(0)=0, pi(1)=32), so it holds Z[pi(l) + 64 r] and the conjugate partner
//           Z[512 - k] lives in lane l^1 (one DPP quad_perm per value);
//   post    real-spectrum split, |X|^2 * scale (x2 off DC / Nyquist) → LDS tile
//           [513][32] (row pitch 34, tile_at()).
// One workgroup = 16 waves (4 per SIMD: one wave alone issues a VALU op only every
// ~4 cycles, so the SIMD needs several) = one tile of 32 consecutive frames, one
// frame pair per wave.  The tile leaves as 128-B row segments.  Workgroups are
// persistent and walk a contiguous range of tiles (the half frame shared by
// neighbouring tiles is re-read from L2); each wave loads its next tile's frame pair
// into the sample registers as soon as the current pair is windowed.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "msd_internal.h"

#include <cmath>
#include <cstdlib>
#include <type_traits>

namespace msd {
namespace {

// The previous tile's write-out (row groups j = 0..4, rows 128 j + tid / 8) leaves in two bursts:
// groups [0, F_WO_SPLIT) after the first transposes, [F_WO_SPLIT, 5) after the second ones (the
// placement measured fastest among 13; the A/B variants live in tools/)
constexpr int F_WO_SPLIT = 2;
constexpr int F_NW = 16;                  // waves per workgroup (4 per SIMD)
constexpr int F_TT = 32;                  // frames per tile
constexpr int F_K = 513;                  // one-sided bins
constexpr int F_PITCH = F_TT + 2;         // tile row pitch (floats)
constexpr int F_SCRF = 576;               // float2 per frame scratch (phys(511) = 571)
constexpr int F_TILE_BYTES = ((F_K * F_PITCH * 4 + 15) / 16) * 16;
constexpr int F_SCR_OFF = F_TILE_BYTES;
constexpr int F_TAB_OFF = F_SCR_OFF + F_NW * F_SCRF * 8;
// per-lane constants, one 208-B row per lane [lane][26 float2]: window pairs w[2(l + 64 r)..] (r = 0..7,
// at 0), post twiddles W1024^{pi(l) + 64 r} (r = 0..3, at 8), pass-2 twiddles W64^{(l&7) r} (r = 1..7,
// at 12) and pass-3 twiddles W512^{pi(l) r} (r = 1..7, at 19).  Read as ds_read_b128 (4 LDS cycles
// per KB, the ds_read_b64 rate; the [r][lane] layout's reads were paired into ds_read2st64_b64 at
// 8 cycles per KB); the 52-dword row stride is 4 x odd, so a b128 lane group hits 16 disjoint
// 4-bank ranges (conflict-free)
constexpr int F_TABW = 26;
constexpr int F_LDS = F_TAB_OFF + F_TABW * 64 * 8;
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

// second half of a forward 8-point DFT: a_j = v_j + v_{j+4}, b_j = v_j - v_{j+4} given; s = sqrt(1/2)
// in a VGPR (vgpr_f: as an SGPR or literal operand its multiplies issue slower)
__device__ __forceinline__ void dft8_tail(float2 *v, float2 a0, float2 a1, float2 a2, float2 a3, float2 b0, float2 b1,
                                          float2 b2, float2 b3, float s) {
    b1 = make_float2((b1.x + b1.y) * s, (b1.y - b1.x) * s);
    b2 = mul_mi(b2);
    b3 = make_float2((b3.y - b3.x) * s, -(b3.x + b3.y) * s);
    dft4(a0, a1, a2, a3);
    dft4(b0, b1, b2, b3);
    v[0] = a0; v[2] = a1; v[4] = a2; v[6] = a3;
    v[1] = b0; v[3] = b1; v[5] = b2; v[7] = b3;
}

// in-place forward DFT of 8 points, natural order in and out
__device__ __forceinline__ void dft8(float2 *v, float s) {
    dft8_tail(v, cadd(v[0], v[4]), cadd(v[1], v[5]), cadd(v[2], v[6]), cadd(v[3], v[7]), csub(v[0], v[4]),
              csub(v[1], v[5]), csub(v[2], v[6]), csub(v[3], v[7]), s);
}

// dft8 of the windowed points d_j * w_j (componentwise), the window product of v_{j+4} shared
// by the first-stage sum and difference: 3 ops per component pair instead of 4
__device__ __forceinline__ void dft8_windowed(float2 *v, const float2 *d, const float2 *w, float s) {
    float2 a[4], b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float px = d[j + 4].x * w[j + 4].x, py = d[j + 4].y * w[j + 4].y;
        a[j] = make_float2(__builtin_fmaf(d[j].x, w[j].x, px), __builtin_fmaf(d[j].y, w[j].y, py));
        b[j] = make_float2(__builtin_fmaf(d[j].x, w[j].x, -px), __builtin_fmaf(d[j].y, w[j].y, -py));
    }
    dft8_tail(v, a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3], s);
}


// Transpose-scratch layout (float2 index): bit 4 of n flips bits 1 and 3, plus 4 float2 of
// padding per 32.  Together with the pass-3 lane table below it makes all four transpose
// access patterns (16-B pass-1 writes, 8-B reads, 8-B pass-2 writes, pass-3 reads) free of
// bank conflicts under the gfx950 LDS model — found by tools/lds_swizzle_search.py.
__device__ __forceinline__ int phys(int n) { return (n ^ (((n >> 4) & 1) * 10)) + ((n >> 5) << 2); }

// pass-3 butterfly of each lane: conjugate pairs (j, 64-j) in adjacent lanes, (0, 32) in
// lanes 0/1, grouped so that the pass-3 reads are conflict-free (tools/lds_swizzle_search.py)
__constant__ int8_t k_pass3_lane[64] = {0,  32, 1,  63, 3,  61, 5,  59, 6,  58, 7,  57, 12, 52, 14, 50,
                                        13, 51, 15, 49, 16, 48, 18, 46, 25, 39, 26, 38, 27, 37, 28, 36,
                                        2,  62, 4,  60, 8,  56, 9,  55, 10, 54, 11, 53, 17, 47, 19, 45,
                                        20, 44, 21, 43, 22, 42, 23, 41, 24, 40, 29, 35, 30, 34, 31, 33};

// Output tile: bin k, frame column c at k * 34 + ((c + rot(k)) & 31) (pitch 34 keeps rows 8-B
// aligned; an XOR-swizzled pitch-32 tile read by conflict-free ds_read_b128 measured 1.5 % slower).
// The half-row rotation of rows k = 32, 40, 48, 56 (mod 64) makes the post pass's tile writes
// conflict-free: a 16-lane ds_write_b64 group holds 8 conjugate pairs (j, 64 - j) of butterflies,
// whose rows 2k mod 32 banks cover 15 residues k mod 16 with one doubled (0 or 8, the pair
// j = 0 / 32, 16 / 48, 8 / 56 or 24 / 40), a 2-way conflict in every group (SQ_LDS_BANK_CONFLICT
// 1.30e8 = 32 cycles per wave-iteration, all of the kernel's); moving one row of each such pair
// by 16 banks fills the missing residue.  The write-out's rows 2m, 2m + 1 keep complementary
// banks (tools/lds_bank_model.py checks every access pattern of the kernel).
__device__ __forceinline__ int tile_rot(int k) { return (k & 39) == 32 ? 16 : 0; }
__device__ __forceinline__ int tile_at(int k, int c) { return k * F_PITCH + ((c + tile_rot(k)) & 31); }

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <typename T>
struct PairIO;
template <>
struct PairIO<int16_t> {
    using raw_t = uint32_t;
    static constexpr bool kInt = true;
    __device__ static raw_t load(const int16_t *p) { return *reinterpret_cast<const uint32_t *>(p); }
    __device__ static raw_t zero() { return 0u; }
    __device__ static int ilo(raw_t r) { return (int)(int16_t)(r & 0xffffu); }
    __device__ static int ihi(raw_t r) { return (int)(int16_t)(r >> 16); }
    __device__ static float lo(raw_t r) { return cvt_i16_lo(r); }
    __device__ static float hi(raw_t r) { return cvt_i16_hi(r); }
    __device__ static int sum2(raw_t r, int acc) { return dot2_i16<1, 1>(r, acc); }
};
template <>
struct PairIO<uint8_t> {
    using raw_t = uint32_t;
    static constexpr bool kInt = true;
    __device__ static raw_t load(const uint8_t *p) { return *reinterpret_cast<const uint16_t *>(p); }
    __device__ static raw_t zero() { return 0u; }
    __device__ static int ilo(raw_t r) { return (int)(r & 0xffu); }
    __device__ static int ihi(raw_t r) { return (int)((r >> 8) & 0xffu); }
    __device__ static float lo(raw_t r) { return (float)ilo(r); }
    __device__ static float hi(raw_t r) { return (float)ihi(r); }
    __device__ static int sum2(raw_t r, int acc) { return acc + ilo(r) + ihi(r); }
};
template <>
struct PairIO<float> {
    using raw_t = float2;
    static constexpr bool kInt = false;
    __device__ static raw_t load(const float *p) { return *reinterpret_cast<const float2 *>(p); }
    __device__ static raw_t zero() { return make_float2(0.f, 0.f); }
    __device__ static int ilo(raw_t) { return 0; }
    __device__ static int ihi(raw_t) { return 0; }
    __device__ static float lo(raw_t r) { return r.x; }
    __device__ static float hi(raw_t r) { return r.y; }
};

// per-file geometry kept in scalar registers while a workgroup walks its tiles
struct FileCur {
    int64_t f, ti;  // file, tile within file
    int64_t nfr;    // frames in the file
    int64_t base;   // element offset of the file
};

// sample-pair registers per lane for the wave's frame pair (t, t + 1): frame t in raw[0..7], frame
// t + 1 in raw[RB..RB+7].  SH (hop 512, integer samples): frame t + 1 starts at frame t's
// sample 512, so its first half IS raw[4..7] (RB = 4, 12 registers, 12 loads instead of 16)
template <bool SH>
struct PairRegs {
    static constexpr int RB = SH ? 4 : 8;
    static constexpr int N = RB + 8;
};


template <typename T, bool SH>
__device__ __forceinline__ void load_pair(const T *__restrict__ x, const FileCur &fc, int64_t t, int hop, int l,
                                          typename PairIO<T>::raw_t (&raw)[PairRegs<SH>::N]) {
    using IO = PairIO<T>;
    constexpr int RB = PairRegs<SH>::RB;
    if (t < fc.nfr) {  // wave-uniform
        const T *p = x + uniform_i64(fc.base + t * (int64_t)hop) + 2 * l;
#pragma unroll
        for (int r = 0; r < 8; ++r) raw[r] = IO::load(p + 128 * r);
    } else {
#pragma unroll
        for (int r = 0; r < 8; ++r) raw[r] = IO::zero();
    }
    constexpr int r0 = SH ? 4 : 0;  // SH: the second frame's first half is already in raw[4..7]
    if (t + 1 < fc.nfr) {
        const T *p = x + uniform_i64(fc.base + (t + 1) * (int64_t)hop) + 2 * l;
#pragma unroll
        for (int r = r0; r < 8; ++r) raw[RB + r] = IO::load(p + 128 * r);
    } else {
#pragma unroll
        for (int r = r0; r < 8; ++r) raw[RB + r] = IO::zero();
    }
}

// lanes 0 and 1 take their post-pass partner value from their own registers (a0 / a1 for lane 0,
// b0 / b1 for lane 1) instead of the DPP one: two exec-masked moves (full-rate v_mov_b32) instead
// of two v_cndmask_b32 selects (quarter-rate) per value.  The wave is fully active here.
__device__ __forceinline__ void lane01_fix(float &m0, float &m1, float &m2, float &m3, float a0, float a1, float a2,
                                           float a3, float b0, float b1, float b2, float b3) {
    asm volatile(
        "s_mov_b64 exec, 1\n\t"
        "v_mov_b32 %0, %4\n\tv_mov_b32 %1, %5\n\tv_mov_b32 %2, %6\n\tv_mov_b32 %3, %7\n\t"
        "s_mov_b64 exec, 2\n\t"
        "v_mov_b32 %0, %8\n\tv_mov_b32 %1, %9\n\tv_mov_b32 %2, %10\n\tv_mov_b32 %3, %11\n\t"
        "s_mov_b64 exec, -1"
        : "+v"(m0), "+v"(m1), "+v"(m2), "+v"(m3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3));
}

// WIDE: 64-bit output offsets (files of 2^20 frames and more); SH: hop 512 with integer samples
// DYN: the workgroups take chunks of consecutive tiles from a guided schedule (sched[k] .. sched[k+1],
// at least 2 tiles) by an atomic ticket instead of one fixed range each (as cstft4096_kernel, where it
// balances the workgroups' unequal speeds); the next chunk's ticket is drawn when a chunk starts and
// read at its last tile, at least one tile barrier later.
template <typename T, int WIDE, bool SH, bool DYN = false>
__global__ __launch_bounds__(F_NW * 64, 1) void stft1024_kernel(
    const T *__restrict__ x, const int64_t *__restrict__ off, const int64_t *__restrict__ len,
    int64_t tiles_per_file, int64_t ntiles, int64_t tiles_per_wg, int hop, float wscale, int detrend,
    const float *__restrict__ g_win, const float2 *__restrict__ g_tw, const float2 *__restrict__ g_post,
    float *__restrict__ out, int64_t ld, const int64_t *__restrict__ sched, int64_t nchunks,
    unsigned long long *__restrict__ ticket, float2 dcw0, float2 dcw1) {
    using IO = PairIO<T>;
    using raw_t = typename IO::raw_t;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float *tile = reinterpret_cast<float *>(smem);
    const int tid = threadIdx.x;
    const int l = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar frame addresses
    float2 *scr = reinterpret_cast<float2 *>(smem + F_SCR_OFF) + wave * F_SCRF;
    float2 *t_all = reinterpret_cast<float2 *>(smem + F_TAB_OFF);
    const float2 *tab = t_all + l * F_TABW;  // this lane's constants
    auto pi_of = [](int i) { return (int)k_pass3_lane[i]; };
    for (int i = tid; i < 64 * F_TABW; i += F_NW * 64) {
        const int li = i / F_TABW, c = i % F_TABW;
        float2 e;
        if (c < 8) {
            const float2 gw = *reinterpret_cast<const float2 *>(g_win + 2 * (li + 64 * c));
            e = make_float2(gw.x * wscale, gw.y * wscale);  // window * sqrt(scale / 2)
        } else if (c < 12) {
            e = g_post[pi_of(li) + 64 * (c - 8)];
        } else if (c < 19) {
            e = g_tw[8 * (li & 7) * (c - 11)];
        } else {
            e = g_tw[pi_of(li) * (c - 18)];
        }
        t_all[i] = e;
    }
    // the table entries as ds_read_b128 (two float2 each) / ds_read_b64
    auto tab4 = [&](int c) { return *reinterpret_cast<const float4 *>(tab + c); };
    const int pi = pi_of(l);
    // integer samples: the coefficient of the mean's fractional part b / 1024 at this lane's bin of
    // register 0 -- 2 ws W_k / 1024 at k = 0 (lane pi = 0) and k = 1 (pi = 1), zero elsewhere
    // (launch_fast_t: the window's DFT vanishes past bin 1)
    const float2 dcw = pi == 0 ? dcw0 : (pi == 1 ? dcw1 : make_float2(0.f, 0.f));
    __syncthreads();

    __shared__ int64_t slot[2];  // DYN: drawn chunk tickets
    int64_t tb, te;              // the current range of tiles
    int par = 0;
    if constexpr (DYN) {
        if (tid == 0) slot[0] = (int64_t)atomicAdd(ticket, 1ull);
        __syncthreads();
        const int64_t k = uniform_i64(slot[0]);
        if (k >= nchunks) return;
        tb = uniform_i64(sched[k]);
        te = uniform_i64(sched[k + 1]);
        if (tid == 0) slot[1] = (int64_t)atomicAdd(ticket, 1ull);  // the chunk after
        // published before any wave reads it: a one-tile first chunk (ntiles = 1, the schedule's only
        // chunk below cmin) reads slot[1] at its first loop head, with no tile barrier in between
        __syncthreads();
        par = 1;
    } else {
        tb = (int64_t)blockIdx.x * tiles_per_wg;
        te = tb + tiles_per_wg < ntiles ? tb + tiles_per_wg : ntiles;
        if (tb >= te) return;
    }
    auto file_at = [&](int64_t f, int64_t ti) {
        FileCur c;
        c.f = f;
        c.ti = ti;
        const int64_t n = len[f];
        c.nfr = n >= 1024 ? (n - 1024) / hop + 1 : 0;
        c.base = off[f];
        return c;
    };
    auto advance = [&](const FileCur &c) {
        return c.ti + 1 < tiles_per_file ? FileCur{c.f, c.ti + 1, c.nfr, c.base} : file_at(c.f + 1, 0);
    };
    FileCur cur = file_at(tb / tiles_per_file, tb % tiles_per_file);
    const int wcol = wave * 2;  // the two tile columns (frames) of this wave

    constexpr int RB = PairRegs<SH>::RB, NR = PairRegs<SH>::N;
    raw_t raw[NR];
    load_pair<T, SH>(x, cur, cur.ti * F_TT + wcol, hop, l, raw);
    bool b_ok = cur.ti * F_TT + wcol + 1 < cur.nfr;  // the pair's second frame exists (wave-uniform)
    // 32-bit byte offsets of this thread's write-out rows k = 128 j + tid / 8 from the tile's base
    uint32_t wo_off[5];
#pragma unroll
    for (int j = 0; j < 5; ++j)
        wo_off[j] = (uint32_t)(128 * j + (tid >> 3)) * ((uint32_t)ld * 4u) + 16u * (uint32_t)(tid & 7);
    // ---- tile → HBM: 513 rows x 32 floats (128 B), 8 lanes x 16 B per row.  Issued one
    // iteration late (in the middle of the next tile's transform), so the stores drain while
    // that tile computes; the next prefetch is issued before them, so the wait for it at the top
    // of the loop never waits for a tile's stores.
    auto write_out = [&](const FileCur &wc, auto j0c, auto j1c) {
        constexpr int J0 = decltype(j0c)::value, J1 = decltype(j1c)::value;
        // scalar base + lane offsets, 8 lanes x 16 B per row: two 8-B LDS reads → one 16-B
        // store.  WIDE = 0: 32-bit offsets (K*ld*4 < 2^31, i.e. ld < 2^20 frames); WIDE = 1:
        // 64-bit (longer files)
        char *of = reinterpret_cast<char *>(out + wc.f * (int64_t)F_K * ld + wc.ti * F_TT);
        const int qq = tid & 7;
        const int rw = tile_rot(tid >> 3);  // = tile_rot(k) for every j (k = 128 j + tid / 8)
        typedef float f4v __attribute__((ext_vector_type(4)));
        // WIDE = 0: a buffer resource on the tile's base and the precomputed 32-bit row offsets (no
        // per-store 64-bit address arithmetic)
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(of, 0, (int)((uint32_t)F_K * (uint32_t)ld * 4u), 0x00020000);
#pragma unroll
        for (int j = J0; j < J1; ++j) {
            const int k = 128 * j + (tid >> 3);
            if (k < F_K) {
                const int c0 = k * F_PITCH + ((4 * qq + rw) & 31);  // tile_at(k, 4 qq); + 2: tile_at(k, 4 qq + 2)
                const float2 a = *reinterpret_cast<const float2 *>(&tile[c0]);
                const float2 b = *reinterpret_cast<const float2 *>(&tile[c0 + 2]);
                const f4v v = f4v{a.x, a.y, b.x, b.y};
                // streaming (non-temporal) stores: written once, never re-read here (A/B: -1 to -2 %)
                if constexpr (WIDE)
                    __builtin_nontemporal_store(v, reinterpret_cast<f4v *>(of + ((int64_t)k * ld * 4 + 16 * qq)));
                else
                    __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, wo_off[j], 0, 2 /* nt */);
            }
        }
    };
    FileCur prev = cur;
    bool have_prev = false;
    const float hs = vgpr_f(0.70710678118654752440f);  // sqrt(1/2) of the DFT8s, in a VGPR

    for (int64_t tl = tb;;) {
        // the next tile: the next of this range, else (DYN) the first of the next drawn chunk
        bool has_next = tl + 1 < te, jump = false;
        int64_t ntl = tl + 1, nte = te;
        if constexpr (DYN) {
            if (!has_next) {
                const int64_t k2 = uniform_i64(slot[par]);
                if (k2 < nchunks) {
                    has_next = jump = true;
                    ntl = uniform_i64(sched[k2]);
                    nte = uniform_i64(sched[k2 + 1]);
                }
            }
        }
        const FileCur nxt = !has_next ? cur : jump ? file_at(ntl / tiles_per_file, ntl % tiles_per_file) : advance(cur);
        const bool b_cur = b_ok;
        float2 v[2][8], wv[8];
        // ---- detrend (consumes raw); the window is applied inside pass 1
        float rb[2] = {0.f, 0.f};  // integer samples: the mean's fractional part, times 1024
        {
            float mean[2], xr[2] = {0.f, 0.f};
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                if constexpr (IO::kInt) {
                    int s = 0;
                    if constexpr (SH) {  // frame sums from the three half sums (h1 shared)
                        int h[3] = {0, 0, 0};
#pragma unroll
                        for (int r = 0; r < 12; ++r) h[r >> 2] = IO::sum2(raw[r], h[r >> 2]);
                        s = h[q] + h[q + 1];
                    } else {
#pragma unroll
                        for (int r = 0; r < 8; ++r) s = IO::sum2(raw[RB * q + r], s);
                    }
                    s = row_sum_i(s);
                    const int tot = __builtin_amdgcn_readlane(s, 0) + __builtin_amdgcn_readlane(s, 16) +
                                    __builtin_amdgcn_readlane(s, 32) + __builtin_amdgcn_readlane(s, 48);
                    // the mean tot / 1024 = a + b / 1024 exactly (a = floor, 0 <= b < 1024): x - a is
                    // an exact integer (|x - a| < 2^16), so the frame is detrended by one subtraction
                    // at any offset, and b / 1024 times the window's DFT comes off bins 0 and 1 after
                    // the FFT (post pass).  (float(tot) / 1024, rounds 1-5, was exact only while
                    // |tot| < 2^24; the two-part mean hi + lo measured +7.9 % on this loop.)
                    mean[q] = detrend ? (float)(tot >> 10) : 0.f;
                    rb[q] = detrend ? (float)(tot & 1023) : 0.f;
                } else {
                    // float samples: the frame's first sample (lane 0's first value) comes off before
                    // the float sums, so that they accumulate the variation and not a DC offset (a
                    // float sum of 1024 values near m is off by ~10 u |m|: a residual DC otherwise);
                    // the mean is xref + the mean of x - xref
                    auto rl = [](float a, int lane) {
                        return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, a), lane));
                    };
                    const float xref = detrend ? rl(IO::lo(raw[RB * q]), 0) : 0.f;
                    float s = 0.f;
#pragma unroll
                    for (int r = 0; r < 8; ++r) s += (IO::lo(raw[RB * q + r]) - xref) + (IO::hi(raw[RB * q + r]) - xref);
                    s = row_sum_f(s);
                    const float tot = (rl(s, 0) + rl(s, 16)) + (rl(s, 32) + rl(s, 48));
                    mean[q] = detrend ? tot * (1.0f / 1024.0f) : 0.f;
                    xr[q] = xref;
                }
            }
            // each sample register converted once (SH: the shared half serves both frames); float
            // samples relative to their frame's xref
            float2 fr[NR];
#pragma unroll
            for (int i = 0; i < NR; ++i) {
                if constexpr (IO::kInt) fr[i] = make_float2(IO::lo(raw[i]), IO::hi(raw[i]));
                else fr[i] = make_float2(IO::lo(raw[i]) - xr[i / RB], IO::hi(raw[i]) - xr[i / RB]);
            }
#pragma unroll
            for (int r = 0; r < 8; r += 2) {
                const float4 w4 = tab4(r);
                wv[r] = make_float2(w4.x, w4.y);
                wv[r + 1] = make_float2(w4.z, w4.w);
            }
#pragma unroll
            for (int r = 0; r < 8; ++r) {
#pragma unroll
                for (int q = 0; q < 2; ++q)
                    v[q][r] = make_float2(fr[RB * q + r].x - mean[q], fr[RB * q + r].y - mean[q]);
            }
            if (SH && !b_cur) {  // no second frame: its tile column must be zero (the loads were not)
#pragma unroll
                for (int r = 0; r < 8; ++r) v[1][r] = make_float2(0.f, 0.f);
                rb[1] = 0.f;
            }
        }
        // ---- prefetch the next tile's frame pair into the (now free) sample registers
        if (has_next) {
            load_pair<T, SH>(x, nxt, nxt.ti * F_TT + wcol, hop, l, raw);
            b_ok = nxt.ti * F_TT + wcol + 1 < nxt.nfr;
        }

        // ---- pass 1 (Ns = 1): out[8 l + r].  One scratch per wave: frame A's transpose is
        // read back before frame B's is written (LDS executes a wave's accesses in order)
        dft8_windowed(v[0], v[0], wv, hs);
        dft8_windowed(v[1], v[1], wv, hs);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
#pragma unroll
            for (int r = 0; r < 8; r += 2)
                *reinterpret_cast<float4 *>(&scr[phys(8 * l + r)]) =
                    make_float4(v[q][r].x, v[q][r].y, v[q][r + 1].x, v[q][r + 1].y);
            wave_sync();
#pragma unroll
            for (int r = 0; r < 8; ++r) v[q][r] = scr[phys(l + 64 * r)];
            wave_sync();
        }
        // the previous tile's write-out, split between here (after the first transposes) and after
        // the second ones: its LDS reads and stores overlap the other waves' arithmetic in two
        // smaller bursts instead of one (A/B: all at the loop top +2 %, all here 0, half here and
        // half after the second transposes -3.4 %)
        if (have_prev) write_out(prev, std::integral_constant<int, 0>{}, std::integral_constant<int, F_WO_SPLIT>{});
        // ---- pass 2 (Ns = 8): out[64 (l>>3) + (l&7) + 8 r]
        const int o2 = 64 * (l >> 3) + (l & 7);
        float2 tw3_1;  // the first pass-3 twiddle shares the pass-2 table's last ds_read_b128
        {
            float2 w[8];  // pass-2 twiddles r = 1..7 at 12..18
#pragma unroll
            for (int r = 1; r < 8; r += 2) {
                const float4 w4 = tab4(11 + r);
                w[r] = make_float2(w4.x, w4.y);
                if (r < 7) w[r + 1] = make_float2(w4.z, w4.w);
                else tw3_1 = make_float2(w4.z, w4.w);
            }
#pragma unroll
            for (int r = 1; r < 8; ++r) {
                v[0][r] = cmul(v[0][r], w[r]);
                v[1][r] = cmul(v[1][r], w[r]);
            }
        }
        dft8(v[0], hs);
        dft8(v[1], hs);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
#pragma unroll
            for (int r = 0; r < 8; ++r) scr[phys(o2 + 8 * r)] = v[q][r];
            wave_sync();
#pragma unroll
            for (int r = 0; r < 8; ++r) v[q][r] = scr[phys(pi + 64 * r)];
            wave_sync();
        }
        if (have_prev) write_out(prev, std::integral_constant<int, F_WO_SPLIT>{}, std::integral_constant<int, 5>{});
        // ---- pass 3 (Ns = 64): butterfly pi(l) → lane holds Z[pi(l) + 64 r]
        {
            float2 w[8];  // pass-3 twiddles r = 1..7 at 19..25
            w[1] = tw3_1;
#pragma unroll
            for (int r = 2; r < 8; r += 2) {
                const float4 w4 = tab4(18 + r);
                w[r] = make_float2(w4.x, w4.y);
                w[r + 1] = make_float2(w4.z, w4.w);
            }
#pragma unroll
            for (int r = 1; r < 8; ++r) {
                v[0][r] = cmul(v[0][r], w[r]);
                v[1][r] = cmul(v[1][r], w[r]);
            }
        }
        dft8(v[0], hs);
        dft8(v[1], hs);
        // ---- post: X' = 2X = (Z + conj Zm) + W^k (-i)(Z - conj Zm), Zm = Z[(512 - k) mod 512],
        // and from the same e, o the mirror bin X'[512 - k] = conj(e - W^k o).  Lane l owns the
        // four pairs (k = pi(l) + 64 r, 512 - k), r = 0..3: Zm sits in lane l^1, register 7-r
        // (one DPP quad_perm per value); lane 1 (k = 32 + 64 r): own register 7-r; lane 0
        // (k = 64 r): own register (8-r)&7, its r = 0 pair being DC / Nyquist (no doubling), and
        // it alone also owns the self-mirrored bin 256.  W^k from the LDS table.  The powers stay
        // in registers until the tile is free (the previous tile's write-out has read it), so a
        // wave's transform overlaps the other waves' write-out.
        float pa[2][4], pb[2][4], p256[2];
        // the window carries sqrt(scale / 2): |X'|^2 is the doubled one-sided density; lane 0's
        // r = 0 pair (DC, Nyquist) is not doubled
        const float sc0 = l == 0 ? 0.5f : 1.0f;
        float2 wpost[4];  // post twiddles at 8..11: two ds_read_b128
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
            const float4 w4 = tab4(8 + r);
            wpost[r] = make_float2(w4.x, w4.y);
            wpost[r + 1] = make_float2(w4.z, w4.w);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float2 wk = wpost[r];
            float2 mm[2];
#pragma unroll
            for (int q = 0; q < 2; ++q) mm[q] = make_float2(dpp_f<0xB1>(v[q][7 - r].x), dpp_f<0xB1>(v[q][7 - r].y));
            lane01_fix(mm[0].x, mm[0].y, mm[1].x, mm[1].y, v[0][(8 - r) & 7].x, v[0][(8 - r) & 7].y,
                       v[1][(8 - r) & 7].x, v[1][(8 - r) & 7].y, v[0][7 - r].x, v[0][7 - r].y, v[1][7 - r].x,
                       v[1][7 - r].y);
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const float2 m = mm[q];
                const float2 z = v[q][r];
                const float2 e = make_float2(z.x + m.x, z.y - m.y);
                const float2 o = make_float2(z.y + m.y, m.x - z.x);  // -i (z - conj m)
                const float2 t = cmul(wk, o);
                float2 X1 = cadd(e, t);
                const float2 X2 = csub(e, t);
                if constexpr (IO::kInt) {
                    if (r == 0) {  // bins 0, 1: X' -= (b / 1024) 2 ws W_k, the mean's fractional part
                        X1.x = __builtin_fmaf(-rb[q], dcw.x, X1.x);
                        X1.y = __builtin_fmaf(-rb[q], dcw.y, X1.y);
                    }
                }
                pa[q][r] = X1.x * X1.x + X1.y * X1.y;
                pb[q][r] = X2.x * X2.x + X2.y * X2.y;
                if (r == 0) {
                    pa[q][r] *= sc0;
                    pb[q][r] *= sc0;
                }
            }
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {  // lane 0: X'[256] = 2 conj(Z[256]) → |X'|^2 = 4 |Z[256]|^2
            const float2 z = v[q][4];
            p256[q] = (z.x * z.x + z.y * z.y) * 4.0f;
        }
        lds_barrier();  // the previous tile's write-out has finished reading the tile
        // tile_at(pi + 64 r, wcol) and tile_at(512 - pi - 64 r, wcol): the rotations depend on the
        // row mod 64 only, i.e. on pi
        const int mb = (512 - pi) & 63;
        const int ta = tile_at(pi, wcol), tb = tile_at(mb, wcol) + (512 - pi - mb) * F_PITCH;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            *reinterpret_cast<float2 *>(&tile[ta + 64 * r * F_PITCH]) = make_float2(pa[0][r], pa[1][r]);
            *reinterpret_cast<float2 *>(&tile[tb - 64 * r * F_PITCH]) = make_float2(pb[0][r], pb[1][r]);
        }
        if (l == 0) *reinterpret_cast<float2 *>(&tile[tile_at(256, wcol)]) = make_float2(p256[0], p256[1]);
        lds_barrier();  // tile complete
        prev = cur;
        have_prev = true;
        cur = nxt;
        if (!has_next) break;
        if constexpr (DYN) {
            if (jump) {  // into the next chunk: draw the one after it
                par ^= 1;
                if (tid == 0) slot[par] = (int64_t)atomicAdd(ticket, 1ull);
            }
        }
        tl = ntl;
        te = nte;
    }
    write_out(prev, std::integral_constant<int, 0>{}, std::integral_constant<int, 5>{});  // the last tile (complete since the loop's final barrier)
}

template <typename T>
int launch_fast_t(msd_stft_plan *p, const void *x, const int64_t *off, const int64_t *len, int64_t nfiles, float *out,
                  int64_t ld) {
    const bool wide = (uint64_t)F_K * (uint64_t)ld * 4u >= (1ull << 31);
    const bool sh = PairIO<T>::kInt && p->hop == 512;
    auto kern = wide ? (sh ? stft1024_kernel<T, 1, PairIO<T>::kInt> : stft1024_kernel<T, 1, false>)
                     : (sh ? stft1024_kernel<T, 0, PairIO<T>::kInt> : stft1024_kernel<T, 0, false>);
    if (int rc = ensure_dyn_lds(reinterpret_cast<const void *>(kern), F_LDS)) return rc;
    const int cus = p->ctx->num_cu;  // queried once in msd_create
    const int64_t tiles_per_file = ld / F_TT;
    const int64_t ntiles = tiles_per_file * nfiles;
    int64_t wgs = cus;  // one 16-wave workgroup per CU (LDS-bound residency)
    if (wgs > ntiles) wgs = ntiles;
    const float ws = static_cast<float>(std::sqrt(p->scale * 0.5));
    // the mean's fractional part b / 1024 on bins 0, 1: X' = 2 ws X, so the coefficient is 2 ws W_k / 1024
    const double cf = 2.0 * std::sqrt(p->scale * 0.5) / 1024.0;
    const float2 dcw0 = make_float2((float)(cf * p->win_dft01[0].x), (float)(cf * p->win_dft01[0].y));
    const float2 dcw1 = make_float2((float)(cf * p->win_dft01[1].x), (float)(cf * p->win_dft01[1].y));
    if (p->ctx->stft_sched == 2) {
        // guided schedule of tile chunks (>= 2 tiles), rebuilt when (ntiles, wgs) change
        auto dkern = wide ? (sh ? stft1024_kernel<T, 1, PairIO<T>::kInt, true> : stft1024_kernel<T, 1, false, true>)
                          : (sh ? stft1024_kernel<T, 0, PairIO<T>::kInt, true> : stft1024_kernel<T, 0, false, true>);
        if (int rc = ensure_dyn_lds(reinterpret_cast<const void *>(dkern), F_LDS)) return rc;
        if (p->sched_total != ntiles || p->sched_wgs != wgs) {
            int64_t cmin = 2, div = 2;  // A/B knobs: MSD_STFT_GUIDE="cmin,div" (tiles)
            if (const char *e = getenv("MSD_STFT_GUIDE")) {
                long a = 0, b = 0;
                if (sscanf(e, "%ld,%ld", &a, &b) == 2 && a >= 2 && b >= 1) cmin = a, div = b;
            }
            std::vector<int64_t> st(1, 0);
            for (int64_t pos = 0; pos < ntiles;) {
                const int64_t sz = std::max<int64_t>((ntiles - pos) / (div * wgs), cmin);
                pos = std::min(ntiles, pos + sz);
                if (ntiles - pos > 0 && ntiles - pos < cmin) pos = ntiles;  // no chunk below cmin at the end
                st.push_back(pos);
            }
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
            p->sched_total = ntiles;
            p->sched_wgs = wgs;
            p->sched_n = (int64_t)st.size() - 1;
        }
        MSD_HIP(hipMemsetAsync(p->d_ticket, 0, sizeof(unsigned long long), p->ctx->stream));
        hipLaunchKernelGGL(dkern, dim3((unsigned)wgs), dim3(F_NW * 64), F_LDS, p->ctx->stream, static_cast<const T *>(x),
                           off, len, tiles_per_file, ntiles, (int64_t)0, p->hop, ws, p->detrend, p->d_window, p->d_tw,
                           p->d_post, out, ld, p->d_sched, p->sched_n, p->d_ticket, dcw0, dcw1);
        MSD_HIP(hipGetLastError());
        return MSD_OK;
    }
    const int64_t per = (ntiles + wgs - 1) / wgs;
    wgs = (ntiles + per - 1) / per;
    hipLaunchKernelGGL(kern, dim3((unsigned)wgs), dim3(F_NW * 64), F_LDS, p->ctx->stream, static_cast<const T *>(x),
                       off, len, tiles_per_file, ntiles, per, p->hop, ws, p->detrend, p->d_window, p->d_tw, p->d_post,
                       out, ld, nullptr, (int64_t)0, nullptr, dcw0, dcw1);
    MSD_HIP(hipGetLastError());
    return MSD_OK;
}

}  // namespace

// returns 1 if the fast path handled the launch, 0 if not applicable, <0 on error
int launch_stft1024(msd_stft_plan *p, const void *x, int dtype, const int64_t *off, const int64_t *len,
                    int64_t nfiles, float *out, int64_t ld) {
    if (p->nperseg != 1024 || (p->hop & 1)) return 0;
    // integer samples need a window whose DFT vanishes past bin 1 (the mean's fractional part is
    // corrected on bins 0, 1 only); others take the generic kernel's exact two-part mean
    if ((dtype == MSD_I16 || dtype == MSD_U8) && p->detrend && !p->win_dft_compact) return 0;
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
