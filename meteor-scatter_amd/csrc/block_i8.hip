// The block band energies of dsp/src/main.py:352-393 for int16 blocks on the matrix cores:
//     fft_block = np.fft.rfft(block * np.hanning(len(block)), n=Nf); power = |fft_block|^2
// is needed at a few bins only, and for integer samples the windowed DFT at bin k,
//     X_k = sum_n x_n (w_n e^{-2 pi i k n / Nf}),
// is an integer-by-constant dot product.  Each real coefficient w_n cos / w_n sin is stored as
// T = round(c 2^54) (|c| <= 1) in seven balanced base-256 digits d_0..d_6 in [-128, 127], each
// sample as x = 256 h + l' + 128 with h = x >> 8 and l' = (x & 255) - 128, so
//     sum_n x_n T_n = sum_b 256^(6-b) (256 sum_n h_n d_bn + sum_n l'_n d_bn + 128 sum_n d_bn)
// and every inner sum is a v_mfma_i32_16x16x64_i8 accumulation, exact in int32 (K <= 1024:
// |sum| <= 2^24).  The only error against the exact DFT is the coefficients' quantisation,
// 2^-55 sum_n |x_n| (u / 4 per unit |x|, u = 2^-53), plus the float64 digit combination (a few u):
// margin.py's near-tie bound carries it (_i8_chain).  The quantisation is absolute, not relative
// to the window, so it must be far below u: with six digits (2^-47, C5's choice for unwindowed
// blocks) a constant full-scale block's band energy, a Hann sidelobe 30 dB above 1e-12, was
// 4e-9 dB off numpy's.  The replaced float64 Goertzel
// (block_delta2_kernel) is issue-bound on float64 VALU (0.31-0.38 ms for C3's 432 000 blocks);
// here the matrix work is ~12 MFMAs per block and the kernel streams the blocks' 2 KB of samples.
//
// GEMM per 16-row tile = 16 consecutive blocks (row r = block r of the tile), K = L samples in
// K steps of 64 (a lane's A fragment = 16 samples of its row: 8 at 8 g and 8 at 32 + 8 g of the
// step, g = lane >> 4, one 64-B piece per row per load instruction), columns = the components
// (bin j's real part 2 j, imaginary part 2 j + 1; <= 8 bins) in one 16-column tile per digit.  A
// lane of the result (column c = lane & 15, rows 4 (lane >> 4) + i) holds all seven digits of its
// component for 4 blocks: the digits combine by a float64 Horner sum in registers, the real and
// imaginary parts by one DPP swap, and the band sums (numpy's order) run on 16 lanes from LDS.
// The output is block_delta2_kernel's: per block (band energy + 1e-12, noise energy + 1e-12),
// turned into dB and delta by block_db_kernel.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "msd_internal.h"
#include "np_reduce.h"

namespace msd {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

constexpr int BI_ND = 7;       // coefficient digits (= column tiles)
constexpr int BI_ROWS = 16;    // blocks per tile
constexpr int BI_MAXBINS = 8;  // components 2 * bins <= 16 columns
constexpr int BI_PP = 9;       // powers row pitch (doubles): 16 rows on 16 disjoint bank pairs for the band sums
constexpr int BI_WAVES = 8;    // waves per workgroup (2 per SIMD) sharing one copy of the B fragments

template <int CTRL>
__device__ __forceinline__ double dpp64(double x) {
    const long long v = __builtin_bit_cast(long long, x);
    const int lo = __builtin_amdgcn_mov_dpp((int)(v & 0xffffffffll), CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(v >> 32), CTRL, 0xf, 0xf, true);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}

// A fragments of one K step from the lane's 16 samples (w[0..7]: two per dword): high bytes
// h = x >> 8 and low bytes l' = (x & 255) - 128 (offset-binary byte ^ 0x80), both as int8
__device__ __forceinline__ void digits(const uint32_t *w, v4i &hi, v4i &lo) {
#pragma unroll
    for (int o = 0; o < 4; ++o) {
        hi[o] = (int)__builtin_amdgcn_perm(w[2 * o + 1], w[2 * o], 0x07050301u);
        lo[o] = (int)(__builtin_amdgcn_perm(w[2 * o + 1], w[2 * o], 0x06040200u) ^ 0x80808080u);
    }
}

// energy[g] = (sum |X_k|^2 over the band + 1e-12, the same over the noise band) for every block g
// of files [0, nfiles) x [0, blocks_per_file) (blocks past a file's len / B are skipped; energy
// holds nblocks + 1 entries, the last a spare slot for the lanes with nothing to store).  bfrag:
// [BI_ND][KS][64] v4i B fragments, colinit: [BI_ND][16] the 128 sum_n d column constants.
template <int KS>
__global__ __launch_bounds__(64 * BI_WAVES, 1) void block_band_i8_kernel(const int16_t *__restrict__ x,
                                                          const int64_t *__restrict__ off,
                                                          const int64_t *__restrict__ len, int64_t nfiles,
                                                          int64_t blocks_per_file, int64_t B,
                                                          const v4i *__restrict__ bfrag,
                                                          const int *__restrict__ colinit, int nband, int nnoise,
                                                          double2 *__restrict__ energy) {
    __shared__ v4i sB[BI_ND * KS * 64];
    __shared__ int sInit[BI_ND * 16];
    __shared__ double sP[BI_WAVES][BI_ROWS * BI_PP];  // per wave: the tile's powers [row][bin]
    for (int i = threadIdx.x; i < BI_ND * KS * 64; i += 64 * BI_WAVES) sB[i] = bfrag[i];
    for (int i = threadIdx.x; i < BI_ND * 16; i += 64 * BI_WAVES) sInit[i] = colinit[i];
    __syncthreads();
    const int l = threadIdx.x & 63;
    const int c = l & 15, grp = l >> 4, row = l & 15;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t nblocks = nfiles * blocks_per_file;
    const int64_t ntiles = (nblocks + BI_ROWS - 1) / BI_ROWS;
    const int64_t nwaves = (int64_t)gridDim.x * BI_WAVES;
    const int64_t wave = (int64_t)blockIdx.x * BI_WAVES + wv;
    if (wave >= ntiles) return;  // wave-uniform; no workgroup barrier below
    const int nbins = nband + nnoise;
    double *pw = sP[wv];

    // the lane's row of tile t: block g = 16 t + row, its sample pointer (x when the block does not
    // exist: its loads stay in bounds and its energies are not stored).  The files a tile touches
    // are walked with scalar loads (t is wave-uniform): a vector load here would be younger than
    // the prefetched samples in flight, and waiting for it would wait for all of them.
    struct Row {
        const int16_t *p;
        int64_t g;
        bool valid;
    };
    auto row_of = [&](int64_t t) {
        Row r;
        const int64_t g0 = uniform_i64(t * BI_ROWS);
        r.g = g0 + row;
        const int64_t fr = r.g / blocks_per_file;
        const int64_t f0 = uniform_i64(g0 / blocks_per_file);
        const int64_t fl = uniform_i64(std::min((g0 + BI_ROWS - 1) / blocks_per_file, nfiles - 1));
        r.valid = false;
        r.p = x;
        for (int64_t f = f0; f <= fl; ++f) {  // uniform: 1-2 files unless files hold < 16 blocks
            int64_t o = off[f], n = len[f];
            asm volatile("" : "+s"(o), "+s"(n));  // scalar loads before the divergent branch, not vector ones in it
            const int64_t nb = n / B;
            const int64_t b = r.g - f * blocks_per_file;
            if (fr == f && b < nb) {
                r.valid = true;
                r.p = x + o + b * B;
            }
        }
        return r;
    };
    // 16 samples of the row per K step as two 16-B loads.  A row whose start is not on 16 B (a file
    // at an odd sample offset) is read by the same unaligned loads: the HSA target runs with
    // unaligned global access (the compiler itself merges eight 2-B-aligned int16 loads into one
    // dwordx4 here), so no per-row branch sits in the loop.
    auto fetch = [&](const Row &r, int ks, int half) {
        v4u v;
        __builtin_memcpy(&v, r.p + 64 * ks + 32 * half + 8 * grp, 16);
        return v;
    };

    // one tile: its K loop over R (refilled in place with tile `nxt`'s samples as they are used),
    // the digit combination and the energies.  Refills are unconditional (the last tile re-reads
    // itself, unused): a conditional one would join two values in R, and the register copies at the
    // join would wait for the prefetch.
    auto tile = [&](v4u(&R)[2 * KS], const Row &cur, const Row &nxt) __attribute__((always_inline)) {
        v4i Ah[BI_ND], Al[BI_ND];
#pragma unroll
        for (int d = 0; d < BI_ND; ++d) {
            Ah[d] = v4i{0, 0, 0, 0};
            const int ci = sInit[d * 16 + c];
            Al[d] = v4i{ci, ci, ci, ci};
        }
        int boff = l;
        asm volatile("" : "+v"(boff));
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            v4i bk[BI_ND];
#pragma unroll
            for (int d = 0; d < BI_ND; ++d) bk[d] = sB[(d * KS + ks) * 64 + boff];
            uint32_t w[8];
            __builtin_memcpy(w, &R[2 * ks], 32);
            v4i ah, al;
            digits(w, ah, al);
            R[2 * ks] = fetch(nxt, ks, 0);
            R[2 * ks + 1] = fetch(nxt, ks, 1);
#pragma unroll
            for (int d = 0; d < BI_ND; ++d) {
                Ah[d] = __builtin_amdgcn_mfma_i32_16x16x64_i8(ah, bk[d], Ah[d], 0, 0, 0);
                Al[d] = __builtin_amdgcn_mfma_i32_16x16x64_i8(al, bk[d], Al[d], 0, 0, 0);
            }
            // keep each K step's refills in K order: with the prologue store below, every K step
            // then waits for its own two loads only (vmcnt 31-32), a tile of samples in flight
            __builtin_amdgcn_sched_barrier(0);
        }
        // component c of blocks 4 grp + i: sum_b A_b 256^(6 - b) 2^-54 = sum_b A_b 2^(-6 - 8 b),
        // A_b = 256 h_b + l_b (exact in float64)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            double p = __builtin_fma(256.0, (double)Ah[BI_ND - 1][i], (double)Al[BI_ND - 1][i]);
#pragma unroll
            for (int d = BI_ND - 2; d >= 0; --d)
                p = __builtin_fma(p, 0x1p-8, __builtin_fma(256.0, (double)Ah[d][i], (double)Al[d][i]));
            p *= 0x1p-6;
            const double q = dpp64<0xB1>(p);  // the partner component (c ^ 1)
            // |X|^2 = re^2 + im^2: within 2 ulp of np.abs(X)**2 (the bar is 1e-9 dB)
            if (!(c & 1) && (c >> 1) < nbins) pw[(4 * grp + i) * BI_PP + (c >> 1)] = p * p + q * q;
        }
        __builtin_amdgcn_wave_barrier();
        {  // every lane stores (lanes past the tile's 16 rows and missing blocks into the spare slot
           // energy[nblocks]): a store behind a branch would leave the memory counter in two states
           // at the loop head, and the wait for the prefetched samples would become a wait for all
            const double eb = np_sum_small(ArrRef{pw}, row * BI_PP, nband) + 1e-12;
            const double en = np_sum_small(ArrRef{pw}, row * BI_PP + nband, nnoise) + 1e-12;
            energy[l < BI_ROWS && cur.valid ? cur.g : nblocks] = make_double2(eb, en);
        }
        __builtin_amdgcn_wave_barrier();  // pw is rewritten by the next tile
    };
    v4u R[2 * KS];  // the current tile's samples; refilled with the next tile's as they are used
    Row cur = row_of(wave);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        R[2 * ks] = fetch(cur, ks, 0);
        R[2 * ks + 1] = fetch(cur, ks, 1);
    }
    // a store after the first loads, as every tile ends with one: the memory counter enters the loop
    // in the state the loop leaves it, so the first K step waits for its own samples only
    energy[nblocks] = make_double2(0.0, 0.0);
    for (int64_t t = wave; t < ntiles; t += nwaves) {
        // the last tile re-reads itself (unused); a select between two Row values went through
        // scratch at KS = 4, and its loads waited for the prefetched samples
        const Row nxt = row_of(t + nwaves < ntiles ? t + nwaves : t);
        tile(R, cur, nxt);
        cur = nxt;
    }
}

// one balanced base-256 digit expansion of T (|T| <= 2^54): T = sum_b d[b] 256^(6 - b); false if T
// does not fit the seven digits (a carry left over)
bool balanced_digits(int64_t T, int8_t (&d)[BI_ND]) {
    for (int b = BI_ND - 1; b >= 0; --b) {
        int64_t r = ((T % 256) + 256) % 256;
        if (r >= 128) r -= 256;
        d[b] = (int8_t)r;
        T = (T - r) / 256;
    }
    return T == 0;
}

}  // namespace

bool block_i8_shape(int64_t L, int nbins) { return (L == 256 || L == 512 || L == 1024) && nbins >= 1 && nbins <= BI_MAXBINS; }

// the quantisation round(w cos * 2^54) fits seven balanced digits and margin._i8_chain's 2^-55 bound
// holds for |w_n| <= 1 (every window scipy / numpy make); other windows keep the Goertzel kernel
bool block_i8_window(const double *window, int64_t L) {
    for (int64_t n = 0; n < L; ++n)
        if (!std::isfinite(window[n]) || std::fabs(window[n]) > 1.0) return false;
    return true;
}

// the B fragments and column constants of block_band_i8_kernel for the plan's window and bins
int block_i8_build(msd_block_plan *p, const double *window, const int *bins, int nbins) {
    const int L = p->L, KS = L / 64, nfft = p->nfft;
    const int ncomp = 2 * nbins;
    std::vector<int8_t> dig((size_t)BI_ND * 16 * L, 0);  // [digit][component][n]
    std::vector<int> init(BI_ND * 16, 0);
    for (int cp = 0; cp < ncomp; ++cp) {
        const int64_t k = bins[cp >> 1];
        for (int n = 0; n < L; ++n) {
            // w_n cos(2 pi k n / Nf) (re), -w_n sin (im): the argument reduced exactly, long double
            const int64_t m = (k * n) % nfft;
            const long double a = 2.0L * 3.14159265358979323846264338327950288L * (long double)m / (long double)nfft;
            const long double v = (long double)window[n] * ((cp & 1) ? -sinl(a) : cosl(a));
            const int64_t T = llroundl(v * 0x1p54L);
            int8_t d[BI_ND];
            if (!balanced_digits(T, d)) return fail(MSD_ERR_INVALID, "block_i8: coefficient beyond 7 digits");
            for (int b = 0; b < BI_ND; ++b) {
                dig[((size_t)b * 16 + cp) * L + n] = d[b];
                init[b * 16 + cp] += 128 * d[b];
            }
        }
    }
    // fragment [b][ks][lane]: lane (column c = lane & 15, group g = lane >> 4), byte j = sample
    // 64 ks + 8 g + j (j < 8) or 64 ks + 32 + 8 g + (j - 8): the A fragments' order
    std::vector<int8_t> frag((size_t)BI_ND * KS * 64 * 16, 0);
    for (int b = 0; b < BI_ND; ++b)
        for (int ks = 0; ks < KS; ++ks)
            for (int lane = 0; lane < 64; ++lane) {
                const int cc = lane & 15, g = lane >> 4;
                for (int j = 0; j < 16; ++j) {
                    const int n = 64 * ks + (j < 8 ? 8 * g + j : 32 + 8 * g + (j - 8));
                    frag[(((size_t)b * KS + ks) * 64 + lane) * 16 + j] = dig[((size_t)b * 16 + cc) * L + n];
                }
            }
    const size_t nb_frag = frag.size(), nb_init = sizeof(int) * init.size();
    hipError_t e = hipMalloc(&p->d_i8, nb_frag + nb_init);
    if (e == hipSuccess) e = hipMemcpy(p->d_i8, frag.data(), nb_frag, hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = hipMemcpy(static_cast<char *>(p->d_i8) + nb_frag, init.data(), nb_init, hipMemcpyHostToDevice);
    if (e != hipSuccess) return hip_fail(e, "block plan: int8 tables");
    return MSD_OK;
}

int launch_block_i8(msd_block_plan *p, const int16_t *x, const int64_t *off, const int64_t *len, int64_t nfiles,
                    int64_t max_blocks) {
    const int64_t blocks = nfiles * max_blocks;
    const int nband = p->band_hi - p->band_lo + 1 > 0 ? p->band_hi - p->band_lo + 1 : 0;
    const int nnoise = p->noise_hi - p->noise_lo + 1 > 0 ? p->noise_hi - p->noise_lo + 1 : 0;
    const int KS = p->L / 64;
    const v4i *frag = static_cast<const v4i *>(p->d_i8);
    const int *init = reinterpret_cast<const int *>(static_cast<const char *>(p->d_i8) +
                                                    sizeof(v4i) * (size_t)BI_ND * KS * 64);
    // persistent: one 8-wave workgroup per CU (the B fragments fill 28-112 KB of LDS), every wave
    // takes every nwaves-th tile, so the chip sweeps the blocks in order
    const int64_t ntiles = (blocks + BI_ROWS - 1) / BI_ROWS;
    const int64_t grid =
        std::max<int64_t>(1, std::min<int64_t>((ntiles + BI_WAVES - 1) / BI_WAVES, (int64_t)p->ctx->num_cu));
    hipStream_t st = p->ctx->stream;
    switch (KS) {
        case 4:
            hipLaunchKernelGGL(block_band_i8_kernel<4>, dim3((unsigned)grid), dim3(64 * BI_WAVES), 0, st, x, off, len, nfiles, max_blocks,
                               p->block_size, frag, init, nband, nnoise, p->d_energy);
            break;
        case 8:
            hipLaunchKernelGGL(block_band_i8_kernel<8>, dim3((unsigned)grid), dim3(64 * BI_WAVES), 0, st, x, off, len, nfiles, max_blocks,
                               p->block_size, frag, init, nband, nnoise, p->d_energy);
            break;
        case 16:
            hipLaunchKernelGGL(block_band_i8_kernel<16>, dim3((unsigned)grid), dim3(64 * BI_WAVES), 0, st, x, off, len, nfiles,
                               max_blocks, p->block_size, frag, init, nband, nnoise, p->d_energy);
            break;
        default: return fail(MSD_ERR_UNSUPPORTED, "block_i8: L");
    }
    MSD_HIP(hipGetLastError());
    return MSD_OK;
}

}  // namespace msd
