// The live detector's Welch band powers (dsp/src/live/backend/processor.py:206, :349-369) for int16
// audio on the matrix cores.  Per processing block scipy.signal.welch detrends each nperseg-sample
// segment by its mean, windows it and takes the nfft-point rFFT; only the band bins are used.  For
// integer samples the detrended, windowed DFT at bin k is an integer-by-constant dot product,
//     X_k = sum_n (x_n - m) w_n e^{-2 pi i k n / nfft} = sum_n x_n c'_kn,
//     c'_kn = w_n e^{-2 pi i k n / nfft} - W_k / nperseg,  W_k = sum_n w_n e^{-2 pi i k n / nfft},
// because the mean m = sum_n x_n / nperseg is linear in the samples (the detrend folded into the
// coefficients: no per-segment mean, no second pass).  As in block_i8.hip, each real coefficient is
// T ~ c' 2^53 (|c'| <= 2) in seven balanced base-256 digits and each sample x = 256 h + l' + 128,
// so every inner sum is one v_mfma_i32_16x16x64_i8 accumulation, exact in int32.  The products of
// equal weight share an accumulator (h with digit b and l' with digit b + 1: weight 256^(7 - b)),
// eight per component.  The T of a component are rounded to sum exactly to zero (largest remainder),
// so the offset's term 128 sum_n T_n vanishes and the accumulators start at zero; the eight are
// combined exactly (as int32 pairs a_w + 256 a_(w+1) where the plan's bound allows, then two float64
// Horner groups below 2^49) and rounded once to float64: the result is
// round(sum_n (x_n - 128) T_n) = round(sum_n x_n T_n), zero for a silent block.  Error
// against the exact DFT: the quantisation (|T - c' 2^53| < 1: 2^-53 sum|x|) and two roundings of
// |X| <= 2 sum|x|, 5 u sum|x| -- inside margin.live_over_error's int8 term (18 u nperseg max|x|).
//
// GEMM: rows = segments (a 16-row tile holds bpt = 16 / nseg whole blocks, nseg rows each; the
// 5-segment instantiation walks units of 16 blocks = 5 full tiles, see SUPER),
// K = nperseg samples in steps of 64 (the lane's A fragment: 16 samples of its row, 8 at 8 g and 8 at
// 32 + 8 g of the step, g = lane >> 4, as block_i8.hip), columns = the components of the band bins
// (bin j's real part 2 j, imaginary part 2 j + 1), 16 per column tile.  The B fragments of all bins
// (7 digits x KS steps x 1 KB per column tile: 1.1 MB for the live default's 309 bins) do not fit
// one CU's LDS, so the column tiles are split into groups of cg (<= 144 KB of fragments) and each
// workgroup holds one group's fragments in LDS for its lifetime, walking the M tiles of its XCD:
// the workgroups of the column groups on one XCD walk the same tiles in the same order, so the
// samples come from HBM once per XCD and from its L2 for the other groups.  Per (M tile, column
// tile) a wave issues 14 MFMAs per K step (2 sample digits x 7 coefficient digits), combines the
// digits, forms |X|^2 * scale * (2 off DC / Nyquist) and averages each block's nseg segment rows in
// segment order (scipy: Pxy.mean(axis=-1)); the per-block PSD of the band bins goes to memory and
// welch_i8_bands_kernel takes numpy's pairwise band sums and 10 log10 (np.sum(psd[mask])).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "msd_internal.h"
#include "np_reduce.h"

#pragma clang fp contract(off)

namespace msd {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

constexpr int WI_ND = 7;                  // coefficient digits
constexpr int WI_NW = 8;                  // accumulator weights 256^0 .. 256^7
#ifndef WI_WAVES_N
#define WI_WAVES_N 12
#endif
// the digit combination in float64 (two exact Horner groups, one rounding) or in int64: 4.77-4.83
// vs 5.46-5.49 ms per day, the int64 form's 64-bit shifts and sign extensions cost more VALU issue
// than the float64 conversions they replace (profiles/r6_welch_i8_epi_ab.txt)
#ifndef WI_EPI_INT
#define WI_EPI_INT 0
#endif
// the MFMA with the coefficients as its A operand and the samples as B (the fragments' register
// layouts are the same): the output tile transposed, so a lane holds one segment's re and im of two
// bins and forms their powers itself (no partner exchange, no selects)
#ifndef WI_TRANS
#define WI_TRANS 1
#endif
// (the 5-segment instantiation only: the generic one spills 14 registers in this form)
#define WI_MFMA(samp, coef, acc)                                                                   \
    (TR ? __builtin_amdgcn_mfma_i32_16x16x64_i8(coef, samp, acc, 0, 0, 0)                         \
        : __builtin_amdgcn_mfma_i32_16x16x64_i8(samp, coef, acc, 0, 0, 0))
#ifndef WI_SUPER
#define WI_SUPER 1
#endif
#ifndef WI_SCHED
#define WI_SCHED 1
#endif
#ifndef WI_SPECIAL
#define WI_SPECIAL 1
#endif
// an M tile's samples are loaded at its start: prefetching the next tile's into 32 registers
// during this one measured 4.14-4.17 against 4.11-4.13 ms per day, the other waves hide the load
// (profiles/r6_welch_i8_epi_ab.txt)
// waves per workgroup: 12 = 3 per SIMD (<= 168 VGPRs).  Against 8 (2 per SIMD): 5.52-5.55 vs
// 5.97-6.04 ms per day in the first form (profiles/r6_welch_i8_ab.txt), 4.14-4.17 vs 4.31-4.33 in
// this one (profiles/r6_welch_i8_epi_ab.txt)
constexpr int WI_WAVES = WI_WAVES_N;
// waves per workgroup for KS K steps: 8 K steps (nperseg 512) need 236 VGPRs, 2 waves per SIMD
constexpr int wi_waves(int KS) { return KS <= 4 ? WI_WAVES : 8; }
constexpr int WI_PP = 9;                  // per-wave power scratch: 16 rows x 8 bins, pitch 9 doubles
constexpr int WI_PT = 17;                 // (transposed: 8 bins x 16 segment rows, pitch 17 doubles)
static_assert(8 * WI_PT <= 16 * WI_PP, "power scratch");
constexpr size_t WI_LDS = 160 * 1024;     // LDS of one workgroup: B fragments + per-wave power scratch
constexpr int WI_MAXKS = 8;               // nperseg <= 512 (16 K steps would spill)

struct WelchI8Args {
    int64_t nfiles, max_blocks, ld;
    int block_size, step, nseg, bpt;  // bpt: whole blocks per 16-row tile (bpt * nseg <= 16 rows)
    int nct, cg, ngroups, reps;       // column tiles, tiles per group, groups, workgroups per group and XCD
    int nslots;
    double xscale;  // 2^-53 x sample_scale: a component's value from its integer digit sum
    double pscale;  // the density scale 1 / (fs sum w^2), times xscale^2 when folded
    int fold;       // xscale a power of two: |X|^2 = xscale^2 (v^2 + q^2) exactly, folded into pscale
    int pairs;      // the accumulators combine in int32 pairs (digit_sum_pairs)
    double rnseg;   // 1 / nseg
};

template <int CTRL>
__device__ __forceinline__ double dpp64(double x) {
    const long long v = __builtin_bit_cast(long long, x);
    const int lo = __builtin_amdgcn_mov_dpp((int)(v & 0xffffffffll), CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(v >> 32), CTRL, 0xf, 0xf, true);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}

// A fragments of one K step from the lane's 16 samples (w[0..7], two per dword): h = x >> 8 and
// l' = (x & 255) - 128 (offset-binary byte ^ 0x80), as int8
__device__ __forceinline__ void digits(const uint32_t *w, v4i &hi, v4i &lo) {
#pragma unroll
    for (int o = 0; o < 4; ++o) {
        hi[o] = (int)__builtin_amdgcn_perm(w[2 * o + 1], w[2 * o], 0x07050301u);
        lo[o] = (int)(__builtin_amdgcn_perm(w[2 * o + 1], w[2 * o], 0x06040200u) ^ 0x80808080u);
    }
}

// sum_w 256^w a_w rounded once to float64: each group of four exact in int64 (|a| < 2^25: < 2^49),
// t = hi + (lo >> 32) and r = lo mod 2^32 give sum = t 2^32 + r; t converts exactly (|t| < 2^50)
#if WI_EPI_INT
__device__ __forceinline__ int64_t group4(int a0, int a1, int a2, int a3) {
    int64_t v = a3;
    v = (v << 8) + a2;
    v = (v << 8) + a1;
    return (v << 8) + a0;
}
#endif
__device__ __forceinline__ double digit_sum(int a0, int a1, int a2, int a3, int a4, int a5, int a6, int a7) {
#if WI_EPI_INT
    const int64_t lo = group4(a0, a1, a2, a3), hi = group4(a4, a5, a6, a7);
    const int64_t t = hi + (lo >> 32);
    const double tf = __builtin_fma((double)(int)(t >> 32), 0x1p32, (double)(uint32_t)t);
    return __builtin_fma(tf, 0x1p32, (double)(uint32_t)lo);
#else
    // the same value in float64: each group's Horner sum is exact (< 2^49), the last fma rounds once
    double lo = (double)a3, hi = (double)a7;
    lo = __builtin_fma(lo, 256.0, (double)a2);
    hi = __builtin_fma(hi, 256.0, (double)a6);
    lo = __builtin_fma(lo, 256.0, (double)a1);
    hi = __builtin_fma(hi, 256.0, (double)a5);
    lo = __builtin_fma(lo, 256.0, (double)a0);
    hi = __builtin_fma(hi, 256.0, (double)a4);
    return __builtin_fma(hi, 0x1p32, lo);
#endif
}

// the same value when the plan has checked |a_w| + 256 |a_(w+1)| < 2^31 for w = 0, 2, 4, 6 (every
// column's digit sums bound each accumulator, welch_i8_build): the pairs exact in int32, four
// conversions instead of eight, the same single rounding
__device__ __forceinline__ double digit_sum_pairs(int a0, int a1, int a2, int a3, int a4, int a5, int a6, int a7) {
    const int p0 = a0 + a1 * 256, p1 = a2 + a3 * 256, p2 = a4 + a5 * 256, p3 = a6 + a7 * 256;
    const double lo = __builtin_fma((double)p1, 65536.0, (double)p0);  // exact: < 2^48
    const double hi = __builtin_fma((double)p3, 65536.0, (double)p2);
    return __builtin_fma(hi, 0x1p32, lo);
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// a block of the batch: file f, block b of the file, its first sample; valid = the block exists
struct BlockRef {
    int64_t f, b;
    const int16_t *p;
    bool valid;
};

// an M tile's first block, wave-uniform: block b0 (< max_blocks) of file f0 in the batch's
// [nfiles][max_blocks] grid of blocks (block g = f max_blocks + b); the tile holds g .. g + bpt - 1
struct TilePos {
    int64_t f0, b0;
};

__device__ __forceinline__ TilePos tile_pos(const WelchI8Args &A, int64_t t) {
    const int64_t g0 = uniform_i64(t * A.bpt);
    const int64_t f0 = uniform_i64(g0 / A.max_blocks);
    return TilePos{f0, g0 - f0 * A.max_blocks};
}

// the tile dblocks blocks later: a division only when the step leaves file f0 (once in max_blocks /
// dblocks steps), not two 64-bit divisions per lane and tile
__device__ __forceinline__ TilePos tile_advance(const WelchI8Args &A, TilePos P, int64_t dblocks) {
    P.b0 += dblocks;
    if (P.b0 >= A.max_blocks) {
        const int64_t q = uniform_i64(P.b0 / A.max_blocks);
        P.f0 += q;
        P.b0 -= q * A.max_blocks;
    }
    return P;
}

// the last file a wave looked up (wave-uniform): its sample offset and block count, so that the
// tiles inside one file (all but one in max_blocks / (nslot bpt)) load and divide nothing
struct FileCache {
    int64_t f = -1, o = 0, nb = 0;
};

// block bi (per lane, < span) of the span of blocks starting at P: the files the span touches are
// walked (at most a few, uniform), the lane's block picked from them
__device__ __forceinline__ BlockRef block_at(const int16_t *x, const int64_t *off, const int64_t *len,
                                            const WelchI8Args &A, TilePos P, int bi, FileCache &C, int span) {
    BlockRef r;
    r.f = P.f0;
    r.b = 0;
    r.valid = false;
    r.p = x;
    const int64_t last = P.b0 + span - 1;  // the span's last block, counted from file f0's first
    for (int64_t k = 0, kb = 0; kb <= last && P.f0 + k < A.nfiles; ++k, kb += A.max_blocks) {
        const int64_t f = uniform_i64(P.f0 + k);
        if (f != C.f) {
            int64_t o = off[f], n = len[f];
            asm volatile("" : "+s"(o), "+s"(n));
            C.f = f;
            C.o = o;
            C.nb = uniform_i64(n >= A.block_size ? (n - A.block_size) / A.block_size + 1 : 0);
        }
        const int64_t b = P.b0 + bi - kb;
        if (b >= 0 && b < A.max_blocks && b < C.nb) {
            r.f = f;
            r.b = b;
            r.valid = true;
            r.p = x + C.o + b * (int64_t)A.block_size;
        }
    }
    return r;
}

// psd[(f ld + b) nslots + slot] = the Welch PSD of block (f, b) at the band bins (slot = band bins in
// order), every block of files [0, nfiles) x [0, max_blocks) that exists.  bfrag: [nct][ND][KS][64]
// B fragments; dbl: [nct * 8] the onesided doubling (1 at DC / Nyquist, else 2; 0 past nslots).
// NSEG > 0: the instantiation for nseg = NSEG segments per block and a folded sample scale (the
// live default's shape: the segment loop, the tile's row map and the mean become constants)
template <int KS, int NSEG>
__global__ __launch_bounds__(64 * wi_waves(KS), 1) void welch_i8_kernel(const int16_t *__restrict__ x,
                                                                    const int64_t *__restrict__ off,
                                                                    const int64_t *__restrict__ len, WelchI8Args Ain,
                                                                    const v4i *__restrict__ bfrag,
                                                                    const double *__restrict__ dbl,
                                                                    double *__restrict__ psd) {
    constexpr int NW = wi_waves(KS);
    constexpr bool TR = WI_TRANS && NSEG > 0;  // the transposed tile (WI_MFMA)
    constexpr bool SUPER = WI_SUPER && TR && NSEG == 5;  // 16-block units (below)
    WelchI8Args A = Ain;
    if constexpr (NSEG > 0) {
        A.nseg = NSEG;
        A.bpt = 16 / NSEG;
        A.fold = 1;
        A.rnseg = 1.0 / NSEG;
    }
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int xcd = blockIdx.x & 7, iw = blockIdx.x >> 3;
    const int cgi = iw % A.ngroups, rep = iw / A.ngroups;
    const int ct0 = cgi * A.cg;
    const int nct = min(A.cg, A.nct - ct0);  // column tiles of this workgroup
    if (nct <= 0) return;                    // workgroup-uniform, before any barrier
    v4i *sB = reinterpret_cast<v4i *>(smem);                                        // [cg][ND][KS][64]
    double *sP = reinterpret_cast<double *>(sB + (size_t)A.cg * WI_ND * KS * 64);   // [WAVES][16][PP]
    double *sDbl = sP + NW * 16 * WI_PP;                                      // [cg][8]
    for (int i = threadIdx.x; i < nct * WI_ND * KS * 64; i += 64 * NW) sB[i] = bfrag[(size_t)ct0 * WI_ND * KS * 64 + i];
    // the power scale per slot: the density scale (times xscale^2 when folded) times the onesided
    // doubling, a power of two (exact)
    for (int i = threadIdx.x; i < nct * 8; i += 64 * NW) sDbl[i] = A.pscale * dbl[ct0 * 8 + i];
    __syncthreads();
    const int l = threadIdx.x & 63;
    const int c = l & 15, g = l >> 4;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    double *pw = sP + wv * 16 * WI_PP;
    const int nrow = A.bpt * A.nseg;
    const int64_t nblocks = A.nfiles * A.max_blocks;
    const int64_t ntm = (nblocks + A.bpt - 1) / A.bpt;  // M tiles
    // this XCD's contiguous share of the M tiles; the workgroups of every column group walk it in
    // the same order (stride = the wave slots of one group on this XCD)
    const int64_t t_lo = ntm * xcd / 8, t_hi = ntm * (xcd + 1) / 8;
    const int64_t slot0 = (int64_t)rep * NW + wv, nslot = (int64_t)A.reps * NW;

    // the lane's A row: row c = segment c % nseg of block c / nseg of the tile (rows past nrow and
    // missing blocks read the file start, their results unused)
    const int row_bi = c < nrow ? c / A.nseg : 0;
    const int row_s = c < nrow ? c - row_bi * A.nseg : 0;
    FileCache fc_row, fc_avg;  // the prefetch walks one tile ahead of the averaging
    auto row_ptr = [&](TilePos P) {
        const BlockRef r = block_at(x, off, len, A, P, row_bi, fc_row, A.bpt);
        return r.valid ? r.p + (int64_t)row_s * A.step : x;
    };
    auto fetch = [&](const int16_t *p, int ks, int half) {
        v4u v;
        __builtin_memcpy(&v, p + 64 * ks + 32 * half + 8 * g, 16);
        return v;
    };
    v4u R[2 * KS];
    v4i ah[KS], al[KS];  // the current M tile's sample digits
#if WI_SCHED
    // the B fragments run one K step ahead: digit d of step ks + 1 (or of the next column tile's
    // step 0) is read into bk[d] as soon as step ks's second MFMA on it has issued, 7 MFMAs
    // before its first use, and the MFMA / LDS order is pinned (the scheduler otherwise waits on
    // each fragment right after requesting it)
    v4i bk[WI_ND];
#endif
    auto load_digits = [&](const int16_t *p) __attribute__((always_inline)) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) R[2 * ks] = fetch(p, ks, 0), R[2 * ks + 1] = fetch(p, ks, 1);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            uint32_t w[8];
            __builtin_memcpy(w, &R[2 * ks], 32);
            digits(w, ah[ks], al[ks]);
        }
#if WI_SCHED
#pragma unroll
        for (int d = 0; d < WI_ND; ++d) bk[d] = sB[(size_t)(d * KS) * 64 + l];
#endif
    };
    // one column tile's MFMAs into acc (the B fragments one K step ahead when WI_SCHED)
    auto mm = [&](v4i(&acc)[WI_NW], int j) __attribute__((always_inline)) {
#pragma unroll
        for (int w = 0; w < WI_NW; ++w) acc[w] = v4i{0, 0, 0, 0};
        const v4i *bj = sB + (size_t)j * WI_ND * KS * 64 + l;
#if WI_SCHED
        const v4i *bn = j + 1 < nct ? bj + (size_t)WI_ND * KS * 64 : bj;  // the last tile re-reads its own (unused)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
            for (int d = 0; d < WI_ND; ++d) acc[7 - d] = WI_MFMA(ah[ks], bk[d], acc[7 - d]);
#pragma unroll
            for (int d = 0; d < WI_ND; ++d) {
                acc[6 - d] = WI_MFMA(al[ks], bk[d], acc[6 - d]);
                bk[d] = ks + 1 < KS ? bj[(d * KS + ks + 1) * 64] : bn[(d * KS) * 64];
            }
            __builtin_amdgcn_sched_group_barrier(0x008, 7, 0);  // the 7 h MFMAs
#pragma unroll
            for (int d = 0; d < WI_ND; ++d) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // an l' MFMA, then its fragment's refill
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
        }
#else
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            v4i bk[WI_ND];
#pragma unroll
            for (int d = 0; d < WI_ND; ++d) bk[d] = bj[(d * KS + ks) * 64];
            // h x digit d: weight 256^(7 - d); l' x digit d: 256^(6 - d) (the l' chain second, so
            // the two MFMAs into one accumulator are 7 apart)
#pragma unroll
            for (int d = 0; d < WI_ND; ++d) acc[7 - d] = WI_MFMA(ah[ks], bk[d], acc[7 - d]);
#pragma unroll
            for (int d = 0; d < WI_ND; ++d) acc[6 - d] = WI_MFMA(al[ks], bk[d], acc[6 - d]);
        }
#endif
    };
    // tile j's powers from its accumulators into the wave's scratch pw
    auto epa = [&](const v4i(&acc)[WI_NW], int j) __attribute__((always_inline)) {
        // component c of rows 4 g + i: sum_w 256^w acc_w x 2^-53 x sample scale
        double v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            v[i] = A.pairs ? digit_sum_pairs(acc[0][i], acc[1][i], acc[2][i], acc[3][i], acc[4][i], acc[5][i],
                                             acc[6][i], acc[7][i])
                           : digit_sum(acc[0][i], acc[1][i], acc[2][i], acc[3][i], acc[4][i], acc[5][i], acc[6][i],
                                       acc[7][i]);
            if (!A.fold) v[i] *= A.xscale;
        }
        // processor.py via scipy: conj(X) X = re re + im im, * scale, * 2.  The doubling (a power
        // of two, exact) and, when folded, xscale^2 enter one product with the scale: the same
        // rounding as scipy's three
        if constexpr (TR) {
            // lane (c, g): segment row c of the tile, components 4 g .. 4 g + 3 = bins 2 g, 2 g + 1
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const double p = v[2 * h] * v[2 * h] + v[2 * h + 1] * v[2 * h + 1];
                pw[(2 * g + h) * WI_PT + c] = p * sDbl[j * 8 + 2 * g + h];
            }
        } else {
        // the lane pair (c, c ^ 1) holds a bin's two components; the even lane forms rows 4 g,
        // 4 g + 1, the odd lane rows 4 g + 2, 4 g + 3, each sending the partner the two values it needs
        const bool odd = c & 1;
        const double sj = sDbl[j * 8 + (c >> 1)];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const double mine = odd ? v[2 + h] : v[h];
            const double q = dpp64<0xB1>(odd ? v[h] : v[2 + h]);
            const double p = mine * mine + q * q;  // re re + im im (addition commutes exactly)
            pw[(4 * g + (odd ? 2 : 0) + h) * WI_PP + (c >> 1)] = p * sj;
        }
        }
    };

    if constexpr (SUPER) {
        // The live default's shape (5 segments per block) in units of 16 blocks = 80 segment rows =
        // 5 full M tiles (no idle row: 16 of 16 against 15 of 16).  A block's segments may straddle
        // two tiles of its unit; its running sum is carried in LDS from one tile to the next, in
        // segment order (the same association as summing the 5 rows at once).  Tile m holds the
        // rows of blocks 16 m / 5 .. 16 m / 5 + 3 of the unit.
        double *carry = sDbl + A.cg * 8 + (size_t)wv * A.cg * 8;  // [cg][8] per wave
        if (l < 8) pw[l * WI_PT + 16] = 0.0;                      // the pad column: an exact no-op term
        const int64_t nun = (nblocks + 15) / 16;
        const int64_t u_lo = nun * xcd / 8, u_hi = nun * (xcd + 1) / 8;
        const int ab = l >> 3, bin = l & 7;
        for (int64_t u = u_lo + slot0; u < u_hi; u += nslot) {
            const int64_t g0 = uniform_i64(u * 16);
            const int64_t uf = uniform_i64(g0 / A.max_blocks);
            const TilePos PU{uf, g0 - uf * A.max_blocks};
            for (int m = 0; m < 5; ++m) {
                {
                    const int G = 16 * m + c, bi = G / 5;
                    const BlockRef rr = block_at(x, off, len, A, PU, bi, fc_row, 16);
                    load_digits(rr.valid ? rr.p + (int64_t)(G - 5 * bi) * A.step : x);
                }
                const int bf = (16 * m) / 5;                      // the tile's first block
                const int bi = bf + (ab < 4 ? ab : 0);            // this lane's block (lanes ab < 4)
                const BlockRef blk = block_at(x, off, len, A, PU, bi, fc_avg, 16);
                const int lo = max(5 * bi - 16 * m, 0), hi = min(5 * bi + 5 - 16 * m, 16);
                const bool cin = 5 * bi < 16 * m, cout = 5 * bi + 5 > 16 * m + 16;
                for (int j = 0; j < nct; ++j) {
                    v4i acc[WI_NW];
                    mm(acc, j);
                    epa(acc, j);
                    wave_sync();
                    const int slot = (ct0 + j) * 8 + bin;
                    if (ab < 4 && slot < A.nslots) {
                        // the block's rows of this tile in order (the pad column past them), after
                        // the running sum carried from the previous tile
                        const double *q = pw + bin * WI_PT;
                        double qv[5];
#pragma unroll
                        for (int k = 0; k < 5; ++k) qv[k] = q[lo + k < hi ? lo + k : 16];
                        double s = cin ? carry[j * 8 + bin] : 0.0;
#pragma unroll
                        for (int k = 0; k < 5; ++k) s = s + qv[k];
                        if (cout) {
                            carry[j * 8 + bin] = s;
                        } else if (blk.valid) {
                            const double mn = s * A.rnseg;  // s / nseg correctly rounded (Markstein)
                            psd[(blk.f * A.ld + blk.b) * (int64_t)A.nslots + slot] =
                                __builtin_fma(__builtin_fma(-mn, (double)A.nseg, s), A.rnseg, mn);
                        }
                    }
                    wave_sync();  // pw is rewritten by the next column tile
                }
            }
        }
        return;
    }
    int64_t t = t_lo + slot0;
    if (t >= t_hi) return;  // wave-uniform; no workgroup barrier below
    TilePos P = tile_pos(A, t);
    for (; t < t_hi; t += nslot) {
        load_digits(row_ptr(P));
        // the next tile (the last re-reads itself, unused)
        TilePos Pn = t + nslot < t_hi ? tile_advance(A, P, nslot * A.bpt) : P;
        Pn.f0 = uniform_i64(Pn.f0);
        Pn.b0 = uniform_i64(Pn.b0);
        // the lanes that average a (block, bin): block l >> 3 of the tile, bin l & 7 of a column tile
        const int ab = l >> 3;
        const BlockRef blk = block_at(x, off, len, A, P, ab < A.bpt ? ab : 0, fc_avg, A.bpt);
        const bool avg_lane = ab < A.bpt && blk.valid;
        // tile j's block means from pw to psd
        auto epb = [&](int j) __attribute__((always_inline)) {
            wave_sync();
            if (avg_lane) {  // Pxy.mean(axis=-1): the block's segments in order, / nseg
                const int bin = l & 7;
                const int slot = (ct0 + j) * 8 + bin;
                if (slot < A.nslots) {
                    // the nseg values loaded together (one LDS round trip, not one per segment), then
                    // summed in segment order
                    const double *q = TR ? pw + bin * WI_PT + ab * A.nseg : pw + ab * A.nseg * WI_PP + bin;
                    constexpr int QS = TR ? 1 : WI_PP;
                    constexpr int MS = NSEG > 0 ? NSEG : 16;
                    double qv[MS];
#pragma unroll
                    for (int k = 0; k < MS; ++k) qv[k] = q[min(k, A.nseg - 1) * QS];
                    double s = qv[0];
#pragma unroll
                    for (int k = 1; k < MS; ++k)
                        if (k < A.nseg) s = s + qv[k];
                    // s / nseg correctly rounded: r = RN(1 / nseg), one Newton correction (Markstein)
                    const double m = s * A.rnseg;
                    psd[(blk.f * A.ld + blk.b) * (int64_t)A.nslots + slot] =
                        __builtin_fma(__builtin_fma(-m, (double)A.nseg, s), A.rnseg, m);
                }
            }
            wave_sync();  // pw is rewritten by the next column tile
        };
        for (int j = 0; j < nct; ++j) {
            v4i acc[WI_NW];
            mm(acc, j);
            epa(acc, j);
            epb(j);
        }
        P = Pn;
    }
}

// band_db[(f nbands + j) ld + b] = 10 log10(np.sum(psd[band j])) (-inf when not > 0) of every block
// (f, b) that exists.  A wave takes 8 blocks, 8 lanes each: lane r of a block accumulates numpy's
// interleaved partial r_r = p[r] + p[r + 8] + ... (the pairwise leaf's 8 accumulators, so the 8
// lanes read 64 contiguous bytes per step), three DPP steps combine them as
// ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)), and the block's lane 0 adds the tail in order:
// np.sum's association for a band of 8 <= n <= 128 bins.  Other widths take np_sum on lane 0.
struct BandArgs {
    int64_t nfiles, max_blocks, ld;
    int block_size, nslots, nbands;
    int slot0[MSD_WELCH_MAX_BANDS], width[MSD_WELCH_MAX_BANDS];
};

__global__ __launch_bounds__(256) void welch_i8_bands_kernel(const int64_t *__restrict__ len, BandArgs A,
                                                             const double *__restrict__ psd,
                                                             double *__restrict__ band_db) {
    const int lane = threadIdx.x & 63, r = lane & 7;
    const int64_t gb = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 8 + (lane >> 3);  // this lane's block
    const int64_t nb_all = A.nfiles * A.max_blocks;
    const bool in = gb < nb_all;
    const int64_t f = in ? gb / A.max_blocks : 0, b = in ? gb - f * A.max_blocks : 0;
    bool ok = false;
    if (in) {
        const int64_t n = len[f];
        ok = b < (n >= A.block_size ? (n - A.block_size) / A.block_size + 1 : 0);
    }
    const double *rowp = psd + (f * A.ld + b) * (int64_t)A.nslots;
    const GArrRef row{as_global(rowp)};
    for (int j = 0; j < A.nbands; ++j) {
        const int w = A.width[j], s0 = A.slot0[j];
        double P = 0.0;
        if (w >= 8 && w <= 128) {
#pragma clang fp contract(off)
            // every load first (one memory round trip, not one per step), then the sums in order;
            // the entries past the band are +0.0, an exact no-op on the non-negative powers
            const int lim = w - (w % 8), nq = lim / 8;
            double v[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = ok && q < nq ? row(s0 + r + 8 * q) : 0.0;
            double acc = v[0];
#pragma unroll
            for (int q = 1; q < 16; ++q) acc += v[q];
            acc = acc + dpp64<0xB1>(acc);   // r0 + r1, r2 + r3, ...
            acc = acc + dpp64<0x4E>(acc);   // (r0 + r1) + (r2 + r3), (r4 + r5) + (r6 + r7)
            acc = acc + dpp64<0x141>(acc);  // half-row mirror: lane 0 meets lane 7
            if (r == 0 && ok) {
                double t[7];
#pragma unroll
                for (int k = 0; k < 7; ++k) t[k] = lim + k < w ? row(s0 + lim + k) : 0.0;
#pragma unroll
                for (int k = 0; k < 7; ++k) acc += t[k];
                P = 0.0 + acc;
            }
        } else if (r == 0 && ok && w > 0) {
            P = w < 8 ? np_sum_small(row, s0, w) : np_sum(row, s0, w);
        }
        if (r == 0 && ok) band_db[(f * A.nbands + j) * A.ld + b] = P > 0.0 ? 10.0 * log10(P) : -INFINITY;
    }
}

// one balanced base-256 digit expansion of T: T = sum_b d[b] 256^(6 - b); false if T needs more
bool balanced_digits7(int64_t T, int8_t (&d)[WI_ND]) {
    for (int b = WI_ND - 1; b >= 0; --b) {
        int64_t r = ((T % 256) + 256) % 256;
        if (r >= 128) r -= 256;
        d[b] = (int8_t)r;
        T = (T - r) / 256;
    }
    return T == 0;
}

}  // namespace

// the int8 path applies: int16 samples (checked at launch), nperseg a multiple of 64 up to 512, at
// most 16 segments per block, a window in [-1, 1] (the quantisation and margin.py's bound), >= 1 bin
bool welch_i8_shape(const msd_welch_cfg &c, int nseg, int nslots, const double *window) {
    if (c.nperseg % 64 != 0 || c.nperseg > 64 * WI_MAXKS || nseg < 1 || nseg > 16 || nslots < 1) return false;
    for (int n = 0; n < c.nperseg; ++n)
        if (!std::isfinite(window[n]) || std::fabs(window[n]) > 1.0) return false;
    return true;
}

// T_n = round(v_n 2^53) with sum_n T_n = 0 exactly: floors, then the largest remainders rounded up
// (sum_n v_n = 0 up to long double rounding, so the count to round up lies in [0, L)); |T_n - v_n 2^53| < 1
bool zero_sum_round(const std::vector<long double> &v, std::vector<int64_t> &T) {
    const int L = (int)v.size();
    std::vector<long double> frac(L);
    std::vector<int> idx(L);
    int64_t S = 0;
    for (int n = 0; n < L; ++n) {
        const long double s = v[n] * 0x1p53L, f = floorl(s);
        T[n] = (int64_t)f;
        frac[n] = s - f;
        S += T[n];
        idx[n] = n;
    }
    const int64_t R = -S;
    if (R < 0 || R > L) return false;
    std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return frac[a] > frac[b]; });
    for (int64_t r = 0; r < R; ++r) T[idx[r]] += 1;
    return true;
}

// the plan's B fragments and doubling factors (one device buffer, p->d_i8)
int welch_i8_build(msd_welch_plan *p, const double *window) {
    const msd_welch_cfg &c = p->cfg;
    const int L = c.nperseg, KS = L / 64, nfft = c.nfft;
    std::vector<int> ks_bins;
    std::vector<double> dblv;
    for (int j = 0; j < c.nbands; ++j) {
        if (c.band_hi[j] < c.band_lo[j]) continue;
        for (int k = c.band_lo[j]; k <= c.band_hi[j]; ++k) {
            ks_bins.push_back(k);
            const bool edge = k == 0 || (nfft % 2 == 0 && k == nfft / 2);
            dblv.push_back(edge ? 1.0 : 2.0);
        }
    }
    const int nslots = (int)ks_bins.size();
    const int ncomp = 2 * nslots;
    const int nct = (ncomp + 15) / 16;
    std::vector<int8_t> frag((size_t)nct * WI_ND * KS * 64 * 16, 0);
    std::vector<double> dbl((size_t)nct * 8, 0.0);
    for (int s = 0; s < nslots; ++s) dbl[s] = dblv[s];
    std::vector<int8_t> dig((size_t)WI_ND * L);
    std::vector<long double> cv(L);
    std::vector<int64_t> T(L);
    bool pairs = true;
    for (int cp = 0; cp < ncomp; ++cp) {
        const int64_t k = ks_bins[cp >> 1];
        const bool im = cp & 1;
        // W_k = sum_n w_n e^{-i theta n} in long double; c'_n = w_n e^{-i theta n} - W_k / L
        long double Wre = 0.0L, Wim = 0.0L;
        std::vector<long double> cr(L), ci(L);
        for (int n = 0; n < L; ++n) {
            long double cs, sn;
            unit_root_ld(k * n, nfft, cs, sn);
            cr[n] = (long double)window[n] * cs;
            ci[n] = -(long double)window[n] * sn;
            Wre += cr[n];
            Wim += ci[n];
        }
        const long double Wc = (im ? Wim : Wre) / (long double)L;
        for (int n = 0; n < L; ++n) cv[n] = (im ? ci[n] : cr[n]) - Wc;
        if (!zero_sum_round(cv, T)) return fail(MSD_ERR_INVALID, "welch_i8: coefficient rounding");
        for (int n = 0; n < L; ++n) {
            int8_t d[WI_ND];
            if (!balanced_digits7(T[n], d)) return fail(MSD_ERR_INVALID, "welch_i8: coefficient beyond 7 digits");
            for (int b = 0; b < WI_ND; ++b) dig[(size_t)b * L + n] = d[b];
        }
        // |acc_w| <= 128 (sum_n |d_(7-w)n| + sum_n |d_(6-w)n|) (h x digit 7 - w, l' x digit 6 - w;
        // |h|, |l'| <= 128): the int32 pairs of digit_sum_pairs need |a_w| + 256 |a_(w+1)| < 2^31
        int64_t sad[WI_ND] = {};
        for (int b = 0; b < WI_ND; ++b)
            for (int n = 0; n < L; ++n) sad[b] += std::abs((int)dig[(size_t)b * L + n]);
        int64_t bound[WI_NW] = {};
        for (int w = 0; w < WI_NW; ++w)
            bound[w] = 128 * ((w >= 1 ? sad[7 - w] : 0) + (w <= 6 ? sad[6 - w] : 0));
        for (int w = 0; w < WI_NW; w += 2)
            if (bound[w] + 256 * bound[w + 1] >= (int64_t(1) << 31)) pairs = false;
        const int ct = cp / 16, cc = cp % 16;
        for (int b = 0; b < WI_ND; ++b) {
            for (int ks = 0; ks < KS; ++ks)
                for (int grp = 0; grp < 4; ++grp)
                    for (int jj = 0; jj < 16; ++jj) {
                        const int n = 64 * ks + (jj < 8 ? 8 * grp + jj : 32 + 8 * grp + (jj - 8));
                        const int lane = grp * 16 + cc;
                        frag[((((size_t)ct * WI_ND + b) * KS + ks) * 64 + lane) * 16 + jj] = dig[(size_t)b * L + n];
                    }
        }
    }
    const size_t nb_frag = frag.size(), nb_dbl = sizeof(double) * dbl.size();
    hipError_t e = hipMalloc(&p->d_i8, nb_frag + nb_dbl);
    char *base = static_cast<char *>(p->d_i8);
    if (e == hipSuccess) e = hipMemcpy(base, frag.data(), nb_frag, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(base + nb_frag, dbl.data(), nb_dbl, hipMemcpyHostToDevice);
    if (e != hipSuccess) return hip_fail(e, "welch plan: int8 tables");
    p->i8_nct = nct;
#ifdef WI_FORCE_NOPAIRS
    pairs = false;  // (A/B build)
#endif
    p->i8_pairs = pairs && !std::getenv("MSD_WELCH_I8_NOPAIRS");
    p->i8_special = WI_SPECIAL && !std::getenv("MSD_WELCH_I8_GENERIC");  // (A/B and the identity test)
    return MSD_OK;
}

// the int8 path of msd_welch_bands_dev for int16 samples: the PSD of the band bins per block into
// psd (the caller's, or the context's scratch), then the band dB
int launch_welch_i8(msd_welch_plan *p, const int16_t *x, const int64_t *off, const int64_t *len, int64_t nfiles,
                    int64_t max_blocks, double *band_db, int64_t ld, double *psd) {
    const msd_welch_cfg &c = p->cfg;
    const int KS = c.nperseg / 64;
    const int nct = p->i8_nct;
    if (!psd) {
        const size_t bytes = sizeof(double) * (size_t)nfiles * (size_t)ld * (size_t)p->nslots;
        void *s = nullptr;
        if (int rc = ctx_scratch(p->ctx, 5, bytes, &s)) return rc;
        psd = static_cast<double *>(s);
    }
    WelchI8Args A{};
    A.nfiles = nfiles;
    A.max_blocks = max_blocks;
    A.ld = ld;
    A.block_size = c.block_size;
    A.step = p->step;
    A.nseg = p->nseg;
    A.bpt = 16 / p->nseg;
    A.nct = nct;
    const int nw = wi_waves(KS);
    // per column tile: its B fragments, its 8 power scales, and every wave's 8 carried block sums
    // (the 16-block units of the 5-segment instantiation)
    const size_t per_ct = (size_t)WI_ND * KS * 64 * 16 + sizeof(double) * 8 + sizeof(double) * 8 * nw;
    const size_t scratch = sizeof(double) * nw * 16 * WI_PP;
    A.cg = (int)std::max<size_t>(1, std::min<size_t>((size_t)nct, (WI_LDS - scratch) / per_ct));
    A.ngroups = (nct + A.cg - 1) / A.cg;
    A.cg = (nct + A.ngroups - 1) / A.ngroups;  // balance the groups (39 tiles: 8 groups of 5 / 4)
    const int wg_per_xcd = std::max(1, p->ctx->num_cu / 8);
    A.reps = std::max(1, wg_per_xcd / A.ngroups);
    A.nslots = p->nslots;
    A.xscale = std::ldexp(c.sample_scale, -53);
    int ex = 0;
    const bool pow2 = std::fabs(std::frexp(A.xscale, &ex)) == 0.5;
    const double folded = c.scale * A.xscale * A.xscale;
    A.fold = pow2 && std::isnormal(folded) && std::isnormal(A.xscale * A.xscale);
    A.pscale = A.fold ? folded : c.scale;
    A.pairs = p->i8_pairs;
    A.rnseg = 1.0 / (double)A.nseg;
    const size_t lds = (size_t)A.cg * per_ct + scratch;
    const v4i *frag = static_cast<const v4i *>(p->d_i8);
    const double *dbl = reinterpret_cast<const double *>(static_cast<const char *>(p->d_i8) +
                                                         (size_t)nct * WI_ND * KS * 64 * 16);
    const unsigned grid = (unsigned)(8 * A.ngroups * A.reps);
    hipStream_t st = p->ctx->stream;
    KernelTimer timer(p->ctx, K_WELCH);
    switch (KS) {
#define WI_LAUNCH(K, S)                                                                                        \
    do {                                                                                                       \
        if (int rc = ensure_dyn_lds(reinterpret_cast<const void *>(welch_i8_kernel<K, S>), 160 * 1024)) return rc; \
        hipLaunchKernelGGL((welch_i8_kernel<K, S>), dim3(grid), dim3(64 * nw), lds, st, x, off, len, A, frag, dbl, \
                           psd);                                                                               \
    } while (0)
#define WI_CASE(K)          \
    case K:                 \
        WI_LAUNCH(K, 0);    \
        break;
        WI_CASE(1)
        WI_CASE(2)
        WI_CASE(3)
        case 4:  // the live default (nperseg 256, 5 segments of a 0.2 s block at 4 kHz): its own instantiation
            if (A.nseg == 5 && A.fold && p->i8_special) WI_LAUNCH(4, 5);
            else WI_LAUNCH(4, 0);
            break;
        WI_CASE(8)
#undef WI_CASE
#undef WI_LAUNCH
        default: return fail(MSD_ERR_UNSUPPORTED, "welch_i8: nperseg");
    }
    MSD_HIP(hipGetLastError());
    BandArgs B{};
    B.nfiles = nfiles;
    B.max_blocks = max_blocks;
    B.ld = ld;
    B.block_size = c.block_size;
    B.nslots = p->nslots;
    B.nbands = c.nbands;
    int s0 = 0;
    for (int j = 0; j < c.nbands; ++j) {
        B.slot0[j] = s0;
        B.width[j] = c.band_hi[j] >= c.band_lo[j] ? c.band_hi[j] - c.band_lo[j] + 1 : 0;
        s0 += B.width[j];
    }
    const int64_t nwg = (nfiles * max_blocks + 31) / 32;  // 8 blocks per wave, 4 waves per workgroup
    hipLaunchKernelGGL(welch_i8_bands_kernel, dim3((unsigned)nwg), dim3(256), 0, st, len, B, psd,
                       band_db);
    MSD_HIP(hipGetLastError());
    return MSD_OK;
}

}  // namespace msd
