// The float64 refinement's block step for int16 I/Q on the matrix cores (msd_iq_delta64_dev,
// refine.hip): the DFT of each D = 1024-sample block at the needed bins as an EXACT integer GEMM.
//
// Samples are integers, so the only rounding in sum_n x_n W^{k n} is the twiddles'.  Each real
// twiddle entry (cos, sin of 2 pi k m / N) is stored as T = round(w 2^46), |T| <= 2^46, written in
// six balanced base-256 digits d_0..d_5 in [-128, 127] (T = sum_b d_b 256^(5-b)); each int16 sample
// as x = 256 h + l' + 128 with h = x >> 8 and l' = (x & 255) - 128 both int8.  Then
//   sum_n x_n T_n = sum_b 256^(5-b) (256 sum_n h_n d_bn + sum_n l'_n d_bn + 128 sum_n d_bn)
// and every inner sum is a v_mfma_i32_16x16x64_i8 accumulation, exact in int32.  The only error
// against the true DFT is the twiddles' quantisation, |T 2^-46 - w| <= 2^-47 per real entry: the
// block's bin is off by at most sqrt 2 * 2^-47 * sum (|I| + |Q|) -- 90.5 u (u = 2^-53) against the
// float64 Goertzel's ~3 L / |sin theta| u (~6000 u at C5) -- before the float64 combination.
//
// GEMM shape per 16-row tile = one block of 1024 complex samples: rows = 16 sub-blocks of 64
// samples, K = 128 (the sub-block's I, Q values interleaved as they sit in memory), columns = the
// needed bins' real and imaginary parts times the six digits, packed in NT tiles of 16 columns:
//   tiles 0..5: column c = component c (bin c >> 1, part c & 1) of bins 0..7, digit = tile;
//   tile 6 + e: bin 8 + e, part c >> 3, digit c & 7 (< 6; columns with digit 6, 7 are zero).
// A lane of the result (column c = lane & 15, rows 4 (lane >> 4) + r) thus holds all six digits of
// its component in its own registers (tiles 0..5), and the extra bins' digits spread over 8 lanes.
// The sub-block partials P_s (s = 0..15) combine to the block's bin with float64 twiddles
// W^{64 k s}: each lane multiplies its 4 rows and the four lane groups are summed.  The output is
// refine.hip's bin-major block table, which frame_kernel turns into frames, delta and ed.
//
// One wave per contiguous range of compact blocks, 2 waves per SIMD (~220 VGPRs: the B fragments
// of every tile, 56, stay in registers for the kernel's lifetime; the next block's samples are
// loaded while the current one is reduced).  Bound by HBM (4 KB of samples per block) and the
// float64 reduction; the matrix cores run 28 MFMAs (448 cycles) per block.
#include <cmath>
#include <cstring>
#include <vector>

#include "msd_internal.h"
#include "refine_plan.h"
#include "refine_i8.h"

namespace msd {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int I8_ND = 6;     // twiddle digits
constexpr int I8_SB = 16;    // sub-blocks per block (rows of the tile)
constexpr int I8_SUB = 64;   // complex samples per sub-block

__device__ __forceinline__ int find_range_i8(const int64_t *cs, int nr, int64_t g) {
    int lo = 0, hi = nr - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (cs[mid] <= g) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

template <int CTRL>
__device__ __forceinline__ double dpp64(double x) {
    const long long v = __builtin_bit_cast(long long, x);
    const int lo = __builtin_amdgcn_mov_dpp((int)(v & 0xffffffffll), CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(v >> 32), CTRL, 0xf, 0xf, true);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
typedef unsigned v4u __attribute__((ext_vector_type(4)));
struct Raw {
    v4u a, b, c, d;  // the lane's 64 bytes: int16 values 32 q .. 32 q + 31 of its row
};

__device__ __forceinline__ Raw load_raw(const int16_t *tile, int l) {
    const v4u *p = reinterpret_cast<const v4u *>(tile) + (l & 15) * 16 + (l >> 4) * 4;
    return Raw{__builtin_nontemporal_load(p), __builtin_nontemporal_load(p + 1), __builtin_nontemporal_load(p + 2),
               __builtin_nontemporal_load(p + 3)};
}

// the A fragments of K step ks from the lane's dwords w[8 ks .. 8 ks + 7] (values 16 ks .. 16 ks + 15
// of its chunk): the high bytes (h = x >> 8) and the low bytes minus 128 (l' = (x & 255) ^ 0x80 as int8)
__device__ __forceinline__ void digits(const uint32_t *w, v4i &hi, v4i &lo, uint32_t &habs) {
#pragma unroll
    for (int o = 0; o < 4; ++o) {
        const uint32_t h = __builtin_amdgcn_perm(w[2 * o + 1], w[2 * o], 0x07050301u);
        const uint32_t l = __builtin_amdgcn_perm(w[2 * o + 1], w[2 * o], 0x06040200u) ^ 0x80808080u;
        hi[o] = (int)h;
        lo[o] = (int)l;
        // sum |h| over the 4 bytes: |h| = |(h ^ 0x80) - 0x80| on the offset-binary bytes
        habs = __builtin_amdgcn_sad_u8(h ^ 0x80808080u, 0x80808080u, habs);
    }
}

// f64 sums of lane l and lane l ^ 16 / l ^ 32 (v_permlane16/32_swap: VALU, no LDS round trip)
__device__ __forceinline__ double add_xor16(double x) {
    const long long v = __builtin_bit_cast(long long, x);
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)(v & 0xffffffffll), (unsigned)(v & 0xffffffffll), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(v >> 32), (unsigned)(v >> 32), false, false);
    const double a = __builtin_bit_cast(double, ((unsigned long long)hi[0] << 32) | lo[0]);
    const double b = __builtin_bit_cast(double, ((unsigned long long)hi[1] << 32) | lo[1]);
    return a + b;
}
__device__ __forceinline__ double add_xor32(double x) {
    const long long v = __builtin_bit_cast(long long, x);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)(v & 0xffffffffll), (unsigned)(v & 0xffffffffll), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(v >> 32), (unsigned)(v >> 32), false, false);
    const double a = __builtin_bit_cast(double, ((unsigned long long)hi[0] << 32) | lo[0]);
    const double b = __builtin_bit_cast(double, ((unsigned long long)hi[1] << 32) | lo[1]);
    return a + b;
}
__device__ __forceinline__ int add_xor16_i(int v) {
    const auto r = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
    return (int)(r[0] + r[1]);
}
__device__ __forceinline__ int add_xor32_i(int v) {
    const auto r = __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false);
    return (int)(r[0] + r[1]);
}

template <int NT>
struct Acc {
    v4i h[NT], l[NT];
};

// out (bin-major, refine.hip's block table): out[b * nblocks + g] = B_g[k_b] for b < nk, then the
// block's sample sum (b = nk) and an upper bound of sum (|re| + |im|) (b = nk + 1, .x)
//
// Software-pipelined: while the VALU reduces block g from one accumulator set, the matrix cores
// run block g + 1's 28 MFMAs into the other (the two sets, 112 VGPRs, are why the B fragments
// live in LDS: 14 ds_read_b128 per block); the next block's samples are loaded one block ahead.
template <int NT>
__global__ __launch_bounds__(256, 2) void block_i8_kernel(const int16_t *__restrict__ x, int64_t D,
                                                          const int64_t *__restrict__ bstart,
                                                          const int64_t *__restrict__ bcs, int nr, int64_t nblocks,
                                                          int64_t per_wave, int nk, const v4i *__restrict__ bfrag,
                                                          const int *__restrict__ colinit,
                                                          const double2 *__restrict__ ltw, double2 *__restrict__ out) {
    constexpr int NX = NT - 6;  // extra bins (8 + e), two components each, in tiles 6 ..
    __shared__ v4i sB[NT * 2 * 64];
    for (int i = threadIdx.x; i < NT * 2 * 64; i += 256) sB[i] = bfrag[i];
    __syncthreads();
    const int l = threadIdx.x & 63;
    const int c = l & 15;
    const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t g0 = wave * per_wave;
    const int64_t g1 = g0 + per_wave < nblocks ? g0 + per_wave : nblocks;
    if (g0 >= g1) return;
    int cinit[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) cinit[t] = colinit[t * 16 + c];
    // this lane's sub-block twiddles W^{64 k s} (s = 4 (l >> 4) + r) for its component's bin, the
    // imaginary part signed by the component (re: +, im: -), and the same for its extra bins
    double2 tw[1 + NX][4];
#pragma unroll
    for (int e = 0; e <= NX; ++e)
#pragma unroll
        for (int r = 0; r < 4; ++r) tw[e][r] = ltw[(e * 4 + r) * 64 + l];
    const int ncomp = 2 * (nk < 8 ? nk : 8);
    const int dg = c & 7;  // extra tiles: this lane's digit (6, 7: the sum columns / zero)
    const double xscale = dg < 6 ? __builtin_ldexp(1.0, -6 - 8 * dg) : 0.0;
    auto block_at = [&](int64_t g) {
        const int r = find_range_i8(bcs, nr, g);
        return bstart[r] + (g - bcs[r]);
    };
    // the MFMAs of one block from its raw samples (sum |h| into habs)
    auto matmul = [&](const Raw &raw, Acc<NT> &A, uint32_t &habs) __attribute__((always_inline)) {
        uint32_t w[16];
        __builtin_memcpy(w, &raw, 64);
        v4i ah[2], al[2];
        habs = 0;
        digits(w, ah[0], al[0], habs);
        digits(w + 8, ah[1], al[1], habs);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            A.h[t] = v4i{0, 0, 0, 0};
            A.l[t] = v4i{cinit[t], cinit[t], cinit[t], cinit[t]};
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const v4i b = sB[(t * 2 + ks) * 64 + l];
                A.h[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(ah[ks], b, A.h[t], 0, 0, 0);
                A.l[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(al[ks], b, A.l[t], 0, 0, 0);
            }
    };
    // the float64 reduction of one block and its stores
    auto reduce = [&](const Acc<NT> &A, uint32_t habs, int64_t g) __attribute__((always_inline)) {
        // this lane's component: P_s = 2^-6 sum_d 2^-8d (256 h_d + l_d) by Horner from the lowest digit
        // (its first steps exact), then the twiddled sum over the lane's 4 rows with the partner
        // component (lane ^ 1; the sign rides in tw.y)
        double ym = 0.0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            double p = (double)((A.h[5][r] << 8) + A.l[5][r]);
#pragma unroll
            for (int d = 4; d >= 0; --d) p = __builtin_fma(p, 0x1p-8, (double)((A.h[d][r] << 8) + A.l[d][r]));
            p *= 0x1p-6;
            const double q = dpp64<0xB1>(p);
            ym = __builtin_fma(p, tw[0][r].x, ym);
            ym = __builtin_fma(q, tw[0][r].y, ym);
        }
        ym = add_xor32(add_xor16(ym));  // the four lane groups (rows 0-3, 4-7, 8-11, 12-15)
        // extra bins: each lane one digit of one component; twiddle its rows (partner: lane ^ 8,
        // same digit), scale, then sum the 6 digit lanes of the half-row and the lane groups
        double yx[NX > 0 ? NX : 1];
        int32_t bsum = 0;
#pragma unroll
        for (int e = 0; e < NX; ++e) {
            double acc = 0.0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int32_t tv = (A.h[6 + e][r] << 8) + A.l[6 + e][r];
                if (e == 0) bsum += tv;  // columns 6 / 7 of tile 6: the sub-block sums of I / Q
                const double v = (double)tv;
                const double u = dpp64<0x128>(v);  // row_ror:8 -- the other component, same digit
                acc = __builtin_fma(v, tw[1 + e][r].x, acc);
                acc = __builtin_fma(u, tw[1 + e][r].y, acc);
            }
            acc *= xscale;  // 0 on the lanes without a digit
            acc += dpp64<0xB1>(acc);  // the 8 lanes of the half-row: xor 1, xor 2, mirror
            acc += dpp64<0x4E>(acc);
            acc += dpp64<0x141>(acc);
            yx[e] = add_xor32(add_xor16(acc));
        }
        if constexpr (NX > 0) bsum = add_xor32_i(add_xor16_i(bsum));
        const int hsum = wave_sum_i((int)habs);
        if (l < 16) {
            double *o = reinterpret_cast<double *>(out);
            if (c < ncomp) o[2 * ((int64_t)(c >> 1) * nblocks + g) + (c & 1)] = ym;
#pragma unroll
            for (int e = 0; e < NX; ++e)
                if (dg == 0) o[2 * ((int64_t)(8 + e) * nblocks + g) + (c >> 3)] = yx[e];
            // sum (|I| + |Q|) <= 256 (sum |h| + values): x = 256 h + (x & 255).  frame_kernel bounds the
            // detrended frame's sum |v| by it plus N |mean|, the mean from the block sums (NX > 0:
            // exact; else unknown, the sum row 0 and the bound doubled instead, N |mean| <= sum |x|)
            const double l1 = 256.0 * ((double)hsum + 2.0 * D);
            if constexpr (NX > 0) {
                if (c == 6 || c == 7) o[2 * ((int64_t)nk * nblocks + g) + (c - 6)] = (double)bsum;
                if (l == 0) out[(int64_t)(nk + 1) * nblocks + g] = make_double2(l1, 0.0);
            } else if (l == 0) {
                out[(int64_t)nk * nblocks + g] = make_double2(0.0, 0.0);
                out[(int64_t)(nk + 1) * nblocks + g] = make_double2(2.0 * l1, 0.0);
            }
        }
    };
    Acc<NT> A0, A1;
    uint32_t h0 = 0, h1 = 0;
    Raw raw = load_raw(x + 2 * block_at(g0) * D, l);
    matmul(raw, A0, h0);
    if (g0 + 1 < g1) raw = load_raw(x + 2 * block_at(g0 + 1) * D, l);
    for (int64_t g = g0; g < g1; g += 2) {
        // block g in A0: block g + 1's MFMAs into A1 (its samples loaded), g + 2's samples requested
        if (g + 1 < g1) {
            matmul(raw, A1, h1);
            if (g + 2 < g1) raw = load_raw(x + 2 * block_at(g + 2) * D, l);
        }
        reduce(A0, h0, g);
        if (g + 1 >= g1) break;
        if (g + 2 < g1) {
            matmul(raw, A0, h0);
            if (g + 3 < g1) raw = load_raw(x + 2 * block_at(g + 3) * D, l);
        }
        reduce(A1, h1, g + 1);
    }
}

// one balanced base-256 digit expansion of T (|T| <= 2^46): T = sum_b d[b] 256^(5 - b)
void balanced_digits(int64_t T, int8_t (&d)[I8_ND]) {
    for (int b = I8_ND - 1; b >= 0; --b) {
        int64_t r = ((T % 256) + 256) % 256;  // 0..255
        if (r >= 128) r -= 256;               // -128..127
        d[b] = (int8_t)r;
        T = (T - r) / 256;
    }
}

}  // namespace

bool i8_supported(const RefineGeom &G, const RefineBins &K) {
    return G.D == I8_SB * I8_SUB && K.dc < 0 && K.nk >= 1 && K.nk <= 10;
}

int launch_refine_i8(msd_ctx *ctx, const int16_t *x, const RefineGeom &G, const RefineBins &K, const int64_t *d_bstart,
                     const int64_t *d_bcs, int64_t nblocks, double2 *blk) {
    const int nk = K.nk;
    const int NT = nk <= 8 ? 6 : 6 + (nk - 8);
    const int N = G.N;
    // host tables (B fragments, column starts, lane twiddles), built once per (N, bins) and kept
    uint64_t key = (uint64_t)N * 1000003u + (uint64_t)nk;
    for (int b = 0; b < nk; ++b) key = key * 1000003u + (uint64_t)K.km[b];
    const size_t nb_frag = sizeof(v4i) * (size_t)NT * 2 * 64;
    const size_t nb_init = sizeof(int) * (size_t)NT * 16;
    const size_t nb_tw = sizeof(double2) * (size_t)(1 + (NT - 6)) * 4 * 64;
    const size_t nb_all = nb_frag + nb_init + nb_tw;
    if (ctx->i8_key != key || !ctx->i8_tab) {
        // column (t, c) -> (bin, part, digit), or -1
        auto colmap = [&](int t, int cc, int &bin, int &part, int &dig) {
            if (t < 6) {
                bin = cc >> 1, part = cc & 1, dig = t;
                return bin < nk && bin < 8;
            }
            bin = 8 + (t - 6), part = cc >> 3, dig = cc & 7;
            return bin < nk && dig < I8_ND;
        };
        // tile 6, columns 6 / 7: ones on the I / Q values (the sub-block sums, block_i8_kernel)
        auto sumcol = [&](int t, int cc) { return t == 6 && (cc == 6 || cc == 7); };
        // B[t][v][c] for v = 0..127: value v of a sub-block row = sample v >> 1, I (v even) or Q
        std::vector<int8_t> Bm((size_t)NT * 128 * 16, 0);
        std::vector<int> init((size_t)NT * 16, 0);
        for (int t = 0; t < NT; ++t)
            for (int cc = 0; cc < 16; ++cc) {
                if (sumcol(t, cc)) {
                    for (int v = 0; v < 128; ++v) Bm[((size_t)t * 128 + v) * 16 + cc] = (v & 1) == cc - 6 ? 1 : 0;
                    init[t * 16 + cc] = 128 * 64;
                    continue;
                }
                int bin, part, dig;
                if (!colmap(t, cc, bin, part, dig)) continue;
                const int64_t km = K.km[bin];
                for (int v = 0; v < 128; ++v) {
                    const int64_t m = v >> 1;
                    const double a = 2.0 * M_PI * (double)((km * m) % N) / (double)N;
                    const double C = std::cos(a), S = std::sin(a);
                    // W^{km} = C - i S;  Y = sum (I + i Q)(C - i S): re = I C + Q S, im = Q C - I S
                    const double val = part == 0 ? ((v & 1) ? S : C) : ((v & 1) ? C : -S);
                    int8_t d[I8_ND];
                    balanced_digits((int64_t)std::llround(std::ldexp(val, 46)), d);
                    Bm[((size_t)t * 128 + v) * 16 + cc] = d[dig];
                    init[t * 16 + cc] += 128 * (int)d[dig];
                }
            }
        std::vector<char> tab(nb_all);
        auto *frag = reinterpret_cast<int8_t *>(tab.data());
        for (int t = 0; t < NT; ++t)
            for (int ks = 0; ks < 2; ++ks)
                for (int l = 0; l < 64; ++l)
                    for (int j = 0; j < 16; ++j)  // lane l byte j: k = 16 (l >> 4) + j of step ks
                        frag[(((size_t)t * 2 + ks) * 64 + l) * 16 + j] = Bm[((size_t)t * 128 + 32 * (l >> 4) + 16 * ks + j) * 16 + (l & 15)];
        std::memcpy(tab.data() + nb_frag, init.data(), nb_init);
        auto *ltw = reinterpret_cast<double2 *>(tab.data() + nb_frag + nb_init);
        for (int e = 0; e <= NT - 6; ++e)
            for (int r = 0; r < 4; ++r)
                for (int l = 0; l < 64; ++l) {
                    const int cc = l & 15, s = 4 * (l >> 4) + r;
                    int bin, part;
                    if (e == 0) bin = cc >> 1, part = cc & 1;
                    else bin = 8 + (e - 1), part = cc >> 3;
                    double2 w = make_double2(0.0, 0.0);
                    if (bin < nk && (e > 0 || bin < 8)) {
                        // W^{64 k s} = cos - i sin: own part p, partner q: re = p cos + q sin (own re),
                        // im = p cos - q sin (own im, partner re)
                        const double a = 2.0 * M_PI * (double)(((int64_t)K.km[bin] * 64 * s) % N) / (double)N;
                        w = make_double2(std::cos(a), part == 0 ? std::sin(a) : -std::sin(a));
                    }
                    ltw[(e * 4 + r) * 64 + l] = w;
                }
        DeviceGuard gd(ctx->device);
        MSD_HIP(hipStreamSynchronize(ctx->stream));
        if (ctx->i8_tab) MSD_HIP(hipFree(ctx->i8_tab));
        ctx->i8_tab = nullptr;
        ctx->i8_key = 0;
        MSD_HIP(hipMalloc(&ctx->i8_tab, nb_all));
        MSD_HIP(hipMemcpy(ctx->i8_tab, tab.data(), nb_all, hipMemcpyHostToDevice));
        ctx->i8_key = key;
    }
    const char *tb = static_cast<const char *>(ctx->i8_tab);
    const v4i *d_frag = reinterpret_cast<const v4i *>(tb);
    const int *d_init = reinterpret_cast<const int *>(tb + nb_frag);
    const double2 *d_tw = reinterpret_cast<const double2 *>(tb + nb_frag + nb_init);
    // persistent: 8 waves per CU (2 workgroups of 4), contiguous block ranges per wave
    const int64_t waves_max = (int64_t)ctx->num_cu * 8;
    int64_t per = (nblocks + waves_max - 1) / waves_max;
    if (per < 1) per = 1;
    const int64_t waves = (nblocks + per - 1) / per;
    const unsigned grid = (unsigned)((waves + 3) / 4);
    hipStream_t st = ctx->stream;
    switch (NT) {
        case 6:
            hipLaunchKernelGGL(block_i8_kernel<6>, dim3(grid), dim3(256), 0, st, x, (int64_t)G.D, d_bstart, d_bcs, G.nr,
                               nblocks, per, nk, d_frag, d_init, d_tw, blk);
            break;
        case 7:
            hipLaunchKernelGGL(block_i8_kernel<7>, dim3(grid), dim3(256), 0, st, x, (int64_t)G.D, d_bstart, d_bcs, G.nr,
                               nblocks, per, nk, d_frag, d_init, d_tw, blk);
            break;
        case 8:
            hipLaunchKernelGGL(block_i8_kernel<8>, dim3(grid), dim3(256), 0, st, x, (int64_t)G.D, d_bstart, d_bcs, G.nr,
                               nblocks, per, nk, d_frag, d_init, d_tw, blk);
            break;
        default: return fail(MSD_ERR_UNSUPPORTED, "refine_i8: bins");
    }
    MSD_HIP(hipGetLastError());
    return MSD_OK;
}

// our float64-side rounding chain in units of u = 2^-53 (refine_plan.h's `own`): the twiddles'
// quantisation sqrt 2 * 2^-47 per unit |x| (90.5), the digit Horner sum (6), the 16 sub-block
// products summed with rounded twiddles over two lane levels (16 + 6)
double i8_chain_own() { return 91.0 + 6.0 + 22.0; }

}  // namespace msd
