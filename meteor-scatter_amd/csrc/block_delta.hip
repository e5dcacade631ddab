// Block band energies → dB → delta, float64 — the detector front end of the
// reference, dsp/src/main.py:352-393:
//     block = x[i*B:(i+1)*B]
//     fft_block = np.fft.rfft(block * np.hanning(len(block)), n=Nf)   # crops to Nf
//     power = np.abs(fft_block)**2
//     band_dB = 10*log10(sum(power[band]) + 1e-12), noise_dB likewise
//     delta = band_dB - noise_dB
// Only the few in-band bins are ever read, so instead of a full transform each
// block evaluates those bins directly (a float64 DFT over the L = min(B, Nf)
// windowed samples): per bin and lane a rotation recurrence over the lane's
// contiguous samples, then a wave reduction.  One wave = one block; samples are
// read with 16-B loads (2*L bytes per block of B samples).  float64 keeps the
// decision margin |delta - threshold| ≫ the deviation from pocketfft's float64
// result.
#include "msd_internal.h"
#include "np_reduce.h"

namespace msd {
namespace {

constexpr int BD_WAVES = 4;
constexpr int BD_MAXBINS = 4096;  // band + noise bins (dynamic LDS: BD_WAVES * nbins doubles)

template <typename T>
__device__ __forceinline__ double to_d(T v) {
    return static_cast<double>(v);
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// SPL = samples per lane (L <= 64*SPL); samples of lane l: [l*SPL, l*SPL+SPL) ∩ [0, L)
template <typename T, int SPL>
__global__ __launch_bounds__(BD_WAVES * 64) void block_delta_kernel(
    const T *__restrict__ x, const int64_t *__restrict__ off, const int64_t *__restrict__ len, int64_t nfiles,
    int64_t blocks_per_file, int64_t B, int L, int nfft, const double *__restrict__ g_win,
    const double2 *__restrict__ g_tw, const int *__restrict__ bins, int nband, int nnoise, double *__restrict__ band_db,
    double *__restrict__ noise_db, double *__restrict__ delta, int64_t ld) {
    extern __shared__ double pbuf_all[];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int64_t gw = (int64_t)blockIdx.x * BD_WAVES + wave;
    const int64_t f = gw / blocks_per_file;
    const int64_t b = gw - f * blocks_per_file;
    if (f >= nfiles) return;
    const int64_t nb = len[f] / B;
    if (b >= nb) return;  // wave-uniform

    const T *xb = x + off[f] + b * B;
    const int n0 = lane * SPL;
    double v[SPL];
    bool vec = false;
    if constexpr ((SPL * (int)sizeof(T)) % 16 == 0) {
        vec = ((reinterpret_cast<uintptr_t>(xb + n0) & 15) == 0) && (n0 + SPL <= L);
        if (vec) {
            constexpr int PER = 16 / (int)sizeof(T);
            const uint4 *q = reinterpret_cast<const uint4 *>(xb + n0);
#pragma unroll
            for (int i = 0; i < SPL / PER; ++i) {
                const uint4 u = q[i];
                const T *e = reinterpret_cast<const T *>(&u);
#pragma unroll
                for (int j = 0; j < PER; ++j) v[i * PER + j] = to_d(e[j]);
            }
        }
    }
    if (!vec) {
#pragma unroll
        for (int q = 0; q < SPL; ++q) v[q] = (n0 + q < L) ? to_d(xb[n0 + q]) : 0.0;
    }
    // block * np.hanning(B): float64 product, exactly as numpy forms it
#pragma unroll
    for (int q = 0; q < SPL; ++q) v[q] = (n0 + q < L) ? v[q] * g_win[n0 + q] : 0.0;

    const int nbins = nband + nnoise;
    double *pb = pbuf_all + wave * nbins;
    for (int j = 0; j < nbins; ++j) {
        const int k = bins[j];
        // r = exp(-2*pi*i*k*n0/nfft), step = exp(-2*pi*i*k/nfft)
        const double2 r0 = g_tw[(int)(((int64_t)k * n0) % nfft)];
        const double2 st = g_tw[k % nfft];
        double re = 0.0, im = 0.0, cr = r0.x, ci = r0.y;
#pragma unroll
        for (int q = 0; q < SPL; ++q) {
            re += v[q] * cr;
            im += v[q] * ci;
            const double nr = cr * st.x - ci * st.y;
            ci = cr * st.y + ci * st.x;
            cr = nr;
        }
        re = wave_sum_d(re);
        im = wave_sum_d(im);
        if (lane == 0) {
            const double h = hypot(re, im);  // np.abs(complex) then **2
            pb[j] = h * h;
        }
    }
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
        const double be = np_sum(ArrRef{pb}, 0, nband) + 1e-12;
        const double ne = np_sum(ArrRef{pb}, nband, nnoise) + 1e-12;
        const double bd = 10.0 * log10(be);
        const double nd = 10.0 * log10(ne);
        const int64_t o = f * ld + b;
        if (band_db) band_db[o] = bd;
        if (noise_db) noise_db[o] = nd;
        delta[o] = bd - nd;
    }
}

template <typename T, int SPL>
int launch_bd(msd_block_plan *p, const void *x, const int64_t *off, const int64_t *len, int64_t nfiles,
              int64_t max_blocks, double *band_db, double *noise_db, double *delta, int64_t ld) {
    const int64_t waves = nfiles * max_blocks;
    const int64_t grid = (waves + BD_WAVES - 1) / BD_WAVES;
    if (grid > 0x7fffffffLL) return fail(MSD_ERR_UNSUPPORTED, "block_delta: grid too large");
    const size_t lds = sizeof(double) * BD_WAVES * (size_t)(p->nbins > 0 ? p->nbins : 1);
    static bool attr_set = false;
    if (!attr_set) {
        MSD_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(block_delta_kernel<T, SPL>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)(sizeof(double) * BD_WAVES * BD_MAXBINS)));
        attr_set = true;
    }
    hipLaunchKernelGGL((block_delta_kernel<T, SPL>), dim3((unsigned)grid), dim3(BD_WAVES * 64), lds, p->ctx->stream,
                       static_cast<const T *>(x), off, len, nfiles, max_blocks, p->block_size, p->L, p->nfft,
                       p->d_window, p->d_tw, p->d_bins, p->band_hi - p->band_lo + 1 > 0 ? p->band_hi - p->band_lo + 1 : 0,
                       p->noise_hi - p->noise_lo + 1 > 0 ? p->noise_hi - p->noise_lo + 1 : 0, band_db, noise_db,
                       delta, ld);
    MSD_HIP(hipGetLastError());
    return MSD_OK;
}

template <typename T>
int launch_bd_t(msd_block_plan *p, const void *x, const int64_t *off, const int64_t *len, int64_t nfiles,
                int64_t max_blocks, double *band_db, double *noise_db, double *delta, int64_t ld) {
    const int L = p->L;
    if (L <= 64 * 8) return launch_bd<T, 8>(p, x, off, len, nfiles, max_blocks, band_db, noise_db, delta, ld);
    if (L <= 64 * 16) return launch_bd<T, 16>(p, x, off, len, nfiles, max_blocks, band_db, noise_db, delta, ld);
    if (L <= 64 * 32) return launch_bd<T, 32>(p, x, off, len, nfiles, max_blocks, band_db, noise_db, delta, ld);
    if (L <= 64 * 64) return launch_bd<T, 64>(p, x, off, len, nfiles, max_blocks, band_db, noise_db, delta, ld);
    return fail(MSD_ERR_UNSUPPORTED, "block_delta: min(block_size, n_fft) must be <= 4096");
}

}  // namespace

int launch_block_delta(msd_block_plan *p, const void *x, int dtype, const int64_t *off, const int64_t *len,
                       int64_t nfiles, int64_t max_blocks, double *band_db, double *noise_db, double *delta,
                       int64_t ld) {
    if (nfiles == 0 || max_blocks == 0) return MSD_OK;
    const int nband = p->band_hi >= p->band_lo ? p->band_hi - p->band_lo + 1 : 0;
    const int nnoise = p->noise_hi >= p->noise_lo ? p->noise_hi - p->noise_lo + 1 : 0;
    if (nband + nnoise > BD_MAXBINS)
        return fail(MSD_ERR_UNSUPPORTED, "block_delta: at most 4096 FFT bins in the two bands together");
    KernelTimer timer(p->ctx, K_BLOCK);
    switch (dtype) {
        case MSD_U8: return launch_bd_t<uint8_t>(p, x, off, len, nfiles, max_blocks, band_db, noise_db, delta, ld);
        case MSD_I16: return launch_bd_t<int16_t>(p, x, off, len, nfiles, max_blocks, band_db, noise_db, delta, ld);
        case MSD_I32: return launch_bd_t<int32_t>(p, x, off, len, nfiles, max_blocks, band_db, noise_db, delta, ld);
        case MSD_F32: return launch_bd_t<float>(p, x, off, len, nfiles, max_blocks, band_db, noise_db, delta, ld);
        case MSD_F64: return launch_bd_t<double>(p, x, off, len, nfiles, max_blocks, band_db, noise_db, delta, ld);
        default: return fail(MSD_ERR_INVALID, "block_delta: unknown dtype");
    }
}

}  // namespace msd
