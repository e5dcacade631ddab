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

#define BD2_STEP(c, a, b, w) fma((c), (a), (w) - (b))

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

// ---------------------------------------------------------------- fast path
// 16 lanes per block (4 blocks per wave), lane-contiguous segments of SPL samples.  Per
// bin, each lane runs a Goertzel recurrence over its segment (2 float64 ops per sample and
// bin instead of a complex rotation), rotates the partial sum to the block origin, and the
// 16 partials are summed with row-local DPP (no LDS round trip).  The block's window lives
// in LDS.  Bins are carried 8 per sweep over the samples, the remainder in one sized sweep.
constexpr int BD2_GROUPS = 16;  // blocks per 256-thread workgroup
constexpr int BD2_MAXBINS = 64;
constexpr int bd2_pitch(int spl) { return spl | 1; }  // odd window pitch in doubles (see the kernel)

template <int CTRL>
__device__ __forceinline__ double dpp_d(double x) {
    const int2 v = __builtin_bit_cast(int2, x);
    int2 r;
    r.x = __builtin_amdgcn_update_dpp(0, v.x, CTRL, 0xf, 0xf, false);
    r.y = __builtin_amdgcn_update_dpp(0, v.y, CTRL, 0xf, 0xf, false);
    return __builtin_bit_cast(double, r);
}
// every lane of a row of 16 gets the row sum (identical bits in all 16 lanes)
__device__ __forceinline__ double row_sum_d(double v) {
    v += dpp_d<0xB1>(v);   // lane ^ 1
    v += dpp_d<0x4E>(v);   // lane ^ 2
    v += dpp_d<0x141>(v);  // half-row mirror
    v += dpp_d<0x140>(v);  // row mirror
    return v;
}

// One sweep: SW bins (j0 .. j0+SW-1, all < nbins) over the lane's segment, then the rotation to
// the block origin, the 16-lane row sum and |X|^2 into pbuf by the row's lane 0.
template <typename T, int SPL, int SW>
__device__ __forceinline__ void bd2_sweep(const T *__restrict__ xb, const double *__restrict__ win,
                                          const double *__restrict__ bconst, const double2 *__restrict__ rot_tab,
                                          double *__restrict__ pb, int j0, int n0, int L, bool valid, bool vec,
                                          int sub) {
    constexpr int PER = 16 / (int)sizeof(T);                                     // samples per 16-B load
    constexpr int CS = SPL < 64 / (int)sizeof(T) ? SPL : 64 / (int)sizeof(T);  // samples per chunk
    constexpr int NV = (CS * (int)sizeof(T) + 15) / 16;                          // 16-B loads per chunk
    double c2[SW], s1[SW], s2[SW];
#pragma unroll
    for (int t = 0; t < SW; ++t) {
        c2[t] = bconst[3 * (j0 + t)];
        s1[t] = 0.0;
        s2[t] = 0.0;
    }
    if (vec) {  // the common case: whole 16-B-aligned segment inside the block
        for (int m0 = 0; m0 < SPL; m0 += CS) {
            // all loads of the chunk first (one latency per chunk), then the recurrences
            union {
                uint4 u[NV];
                T e[NV * PER];
            } raw;
#pragma unroll
            for (int i = 0; i < NV; ++i) raw.u[i] = reinterpret_cast<const uint4 *>(xb + n0 + m0)[i];
#pragma unroll
            for (int q = 0; q < CS; ++q) {
                const double w = to_d(raw.e[q]) * win[m0 + q];  // block * np.hanning(B)
#pragma unroll
                for (int t = 0; t < SW; ++t) {
                    const double s0 = BD2_STEP(c2[t], s1[t], s2[t], w);
                    s2[t] = s1[t];
                    s1[t] = s0;
                }
                if ((q & 7) == 7) __builtin_amdgcn_sched_barrier(0);
            }
        }
    } else {
        for (int m = 0; m < SPL; ++m) {
            const int n = n0 + m;
            const double w = (valid && n < L) ? to_d(xb[n]) * win[m] : 0.0;
#pragma unroll
            for (int t = 0; t < SW; ++t) {
                const double s0 = BD2_STEP(c2[t], s1[t], s2[t], w);
                s2[t] = s1[t];
                s1[t] = s0;
            }
        }
    }
    // y = s1 - e^{-i th} s2 = sum_m v_m e^{i th (SPL-1-m)}; rotate by e^{-i th (n0+SPL-1)}
#pragma unroll
    for (int t = 0; t < SW; ++t) {
        const double cth = bconst[3 * (j0 + t) + 1], msth = bconst[3 * (j0 + t) + 2];
        const double yr = fma(-cth, s2[t], s1[t]);
        const double yi = -msth * s2[t];
        const double2 rot = rot_tab[(j0 + t) * 16 + sub];
        const double re = row_sum_d(fma(yr, rot.x, -yi * rot.y));
        const double im = row_sum_d(fma(yr, rot.y, yi * rot.x));
        if (sub == 0) {
            // re^2 + im^2: within 2 ulp of np.abs(X)**2 (the bar is 1e-9 dB), without hypot's scaling code
            pb[j0 + t] = re * re + im * im;
        }
    }
}

template <typename T, int SPL>
__global__ __launch_bounds__(256) void block_delta2_kernel(
    const T *__restrict__ x, const int64_t *__restrict__ off, const int64_t *__restrict__ len, int64_t nfiles,
    int64_t blocks_per_file, int64_t B, int L, const double *__restrict__ g_win, const double *__restrict__ bconst,
    int nband, int nnoise, double2 *__restrict__ energy) {
    extern __shared__ double smem_d[];
    // window [16 segments][SPL + 1]: the window reads are ds_read2_b64 (two accesses of 4 x 16
    // lanes, bank = dword mod 32), so with an odd pitch segment s starts at bank 2s mod 32 and the
    // 16 lanes of a block cover the 32 banks once (the 4 blocks of a wave read the same addresses).
    // The rounds 1-2 pitch SPL + 2 put s and s + 8 on one bank: 8 extra LDS cycles per read, the
    // 2.8e7 SQ_LDS_BANK_CONFLICT per C2 launch that tools/lds_bank_model.py reproduces.
    constexpr int WP = bd2_pitch(SPL);
    double *win_all = smem_d;                    // [16][WP]
    double *pbuf = smem_d + 16 * WP;             // [16][nbins]
    const int tid = threadIdx.x;
    const int sub = tid & 15;
    const int grp = tid >> 4;
    const int nbins = nband + nnoise;
    const double2 *rot_tab = reinterpret_cast<const double2 *>(bconst + 3 * nbins);  // [nbins][16]
    for (int i = tid; i < 16 * SPL; i += 256) win_all[(i / SPL) * WP + i % SPL] = i < L ? g_win[i] : 0.0;
    __syncthreads();
    const double *win = win_all + sub * WP;
    const int n0 = sub * SPL;
    constexpr int PER = 16 / (int)sizeof(T);
    constexpr int CS = SPL < 64 / (int)sizeof(T) ? SPL : 64 / (int)sizeof(T);
    double *pb = pbuf + grp * nbins;
    const int64_t nblocks = nfiles * blocks_per_file;

    // persistent: the workgroup walks groups of 16 blocks (window staged once per workgroup)
    for (int64_t gb0 = (int64_t)blockIdx.x * BD2_GROUPS; gb0 < nblocks; gb0 += (int64_t)gridDim.x * BD2_GROUPS) {
        const int64_t gb = gb0 + grp;
        const int64_t f = gb / blocks_per_file;
        const int64_t b = gb - f * blocks_per_file;
        const bool valid = f < nfiles && b < len[f < nfiles ? f : 0] / B;
        const T *xb = valid ? x + off[f] + b * B : x;
        const bool vec = (CS % PER == 0) && valid && ((reinterpret_cast<uintptr_t>(xb + n0) & 15) == 0) &&
                         (n0 + SPL <= L);

        // sweeps of 8 bins, then one sweep sized to the remainder (nbins is uniform: no divergence);
        // every sweep re-reads the segment (L1/L2 hits) and re-applies the window
        int j0 = 0;
        for (; j0 + 8 <= nbins; j0 += 8)
            bd2_sweep<T, SPL, 8>(xb, win, bconst, rot_tab, pb, j0, n0, L, valid, vec, sub);
        switch (nbins - j0) {
            case 1: bd2_sweep<T, SPL, 1>(xb, win, bconst, rot_tab, pb, j0, n0, L, valid, vec, sub); break;
            case 2: bd2_sweep<T, SPL, 2>(xb, win, bconst, rot_tab, pb, j0, n0, L, valid, vec, sub); break;
            case 3: bd2_sweep<T, SPL, 3>(xb, win, bconst, rot_tab, pb, j0, n0, L, valid, vec, sub); break;
            case 4: bd2_sweep<T, SPL, 4>(xb, win, bconst, rot_tab, pb, j0, n0, L, valid, vec, sub); break;
            case 5: bd2_sweep<T, SPL, 5>(xb, win, bconst, rot_tab, pb, j0, n0, L, valid, vec, sub); break;
            case 6: bd2_sweep<T, SPL, 6>(xb, win, bconst, rot_tab, pb, j0, n0, L, valid, vec, sub); break;
            case 7: bd2_sweep<T, SPL, 7>(xb, win, bconst, rot_tab, pb, j0, n0, L, valid, vec, sub); break;
            default: break;
        }
        __builtin_amdgcn_wave_barrier();
        // band energy on the group's lane 0, noise energy on lane 1 (numpy's pairwise order over the
        // powers in LDS); lane 0 takes lane 1's by a shuffle of the whole wave.  The dB values and
        // delta follow in block_db_kernel, 64 blocks per wave: two float64 log10 per block on one
        // lane in sixteen cost a quarter of this kernel's float64 issue
        double e = 0.0;
        if (sub < 2 && valid)
            e = (sub == 0 ? np_sum_small(ArrRef{pb}, 0, nband) : np_sum_small(ArrRef{pb}, nband, nnoise)) + 1e-12;
        const double e_next = __shfl_down(e, 1, 64);
        if (sub == 0 && valid) energy[gb] = make_double2(e, e_next);
        __builtin_amdgcn_wave_barrier();  // pbuf is rewritten by the next group
    }
}

// 10 log10 of the two energies and their difference, one thread per block (main.py:388-393)
__global__ __launch_bounds__(256) void block_db_kernel(const double2 *__restrict__ energy,
                                                       const int64_t *__restrict__ len, int64_t nfiles,
                                                       int64_t blocks_per_file, int64_t B, double *__restrict__ band_db,
                                                       double *__restrict__ noise_db, double *__restrict__ delta,
                                                       int64_t ld) {
    const int64_t gb = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t f = gb / blocks_per_file;
    const int64_t b = gb - f * blocks_per_file;
    if (f >= nfiles || b >= len[f] / B) return;
    const double2 e = energy[gb];
    const double bd = 10.0 * log10(e.x);
    const double nd = 10.0 * log10(e.y);
    const int64_t o = f * ld + b;
    if (band_db) band_db[o] = bd;
    if (noise_db) noise_db[o] = nd;
    delta[o] = bd - nd;
}

template <typename T, int SPL>
int launch_bd2(msd_block_plan *p, const void *x, const int64_t *off, const int64_t *len, int64_t nfiles,
               int64_t max_blocks, double *band_db, double *noise_db, double *delta, int64_t ld) {
    const int64_t blocks = nfiles * max_blocks;
    if ((size_t)blocks + 1 > p->energy_cap) {  // grown once per plan (the stream is drained first);
        MSD_HIP(hipStreamSynchronize(p->ctx->stream));  // + 1: block_i8_kernel's spare slot
        MSD_HIP(hipFree(p->d_energy));
        p->d_energy = nullptr;
        p->energy_cap = 0;
        MSD_HIP(hipMalloc(&p->d_energy, sizeof(double2) * ((size_t)blocks + 1)));
        p->energy_cap = (size_t)blocks + 1;
    }
    // persistent grid: a few workgroups per CU, each walking groups of 16 blocks (4 resident per CU;
    // C3 A/B over two boxes, profiles/r4_bd2_grid_ab.txt: 4 per CU 0.409 ms, 8 0.381-0.393, 16 0.372-0.383,
    // 32 0.382, one per group 0.398)
    const int64_t grid = std::min<int64_t>((blocks + BD2_GROUPS - 1) / BD2_GROUPS, (int64_t)p->ctx->num_cu * 16);
    const size_t lds = sizeof(double) * (16 * bd2_pitch(SPL) + BD2_GROUPS * (size_t)(p->nbins > 0 ? p->nbins : 1));
    bool done = false;
    if constexpr (std::is_same_v<T, int16_t>) {
        if (p->d_i8 && !p->ctx->block_goertzel) {  // the exact integer DFT on the matrix cores
            if (int rc = launch_block_i8(p, static_cast<const int16_t *>(x), off, len, nfiles, max_blocks)) return rc;
            done = true;
        }
    }
    if (!done)
    hipLaunchKernelGGL((block_delta2_kernel<T, SPL>), dim3((unsigned)grid), dim3(256), lds, p->ctx->stream,
                       static_cast<const T *>(x), off, len, nfiles, max_blocks, p->block_size, p->L, p->d_window,
                       p->d_bconst, p->band_hi - p->band_lo + 1 > 0 ? p->band_hi - p->band_lo + 1 : 0,
                       p->noise_hi - p->noise_lo + 1 > 0 ? p->noise_hi - p->noise_lo + 1 : 0, p->d_energy);
    MSD_HIP(hipGetLastError());
    hipLaunchKernelGGL(block_db_kernel, dim3((unsigned)((blocks + 255) / 256)), dim3(256), 0, p->ctx->stream,
                       p->d_energy, len, nfiles, max_blocks, p->block_size, band_db, noise_db, delta, ld);
    MSD_HIP(hipGetLastError());
    return MSD_OK;
}

template <typename T>
int launch_bd2_t(msd_block_plan *p, const void *x, const int64_t *off, const int64_t *len, int64_t nfiles,
                 int64_t max_blocks, double *band_db, double *noise_db, double *delta, int64_t ld) {
    switch (p->spl) {  // must match the rotation table built in msd_block_plan_create
        case 16: return launch_bd2<T, 16>(p, x, off, len, nfiles, max_blocks, band_db, noise_db, delta, ld);
        case 32: return launch_bd2<T, 32>(p, x, off, len, nfiles, max_blocks, band_db, noise_db, delta, ld);
        case 64: return launch_bd2<T, 64>(p, x, off, len, nfiles, max_blocks, band_db, noise_db, delta, ld);
        case 128: return launch_bd2<T, 128>(p, x, off, len, nfiles, max_blocks, band_db, noise_db, delta, ld);
        default: return launch_bd2<T, 256>(p, x, off, len, nfiles, max_blocks, band_db, noise_db, delta, ld);
    }
}

template <typename T, int SPL>
int launch_bd(msd_block_plan *p, const void *x, const int64_t *off, const int64_t *len, int64_t nfiles,
              int64_t max_blocks, double *band_db, double *noise_db, double *delta, int64_t ld) {
    const int64_t waves = nfiles * max_blocks;
    const int64_t grid = (waves + BD_WAVES - 1) / BD_WAVES;
    if (grid > 0x7fffffffLL) return fail(MSD_ERR_UNSUPPORTED, "block_delta: grid too large");
    const size_t lds = sizeof(double) * BD_WAVES * (size_t)(p->nbins > 0 ? p->nbins : 1);
    if (int rc = ensure_dyn_lds(reinterpret_cast<const void *>(block_delta_kernel<T, SPL>),
                                (int)(sizeof(double) * BD_WAVES * BD_MAXBINS)))
        return rc;
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
    if (nband + nnoise <= BD2_MAXBINS && !p->ctx->force_generic) {
        switch (dtype) {
            case MSD_U8: return launch_bd2_t<uint8_t>(p, x, off, len, nfiles, max_blocks, band_db, noise_db, delta, ld);
            case MSD_I16: return launch_bd2_t<int16_t>(p, x, off, len, nfiles, max_blocks, band_db, noise_db, delta, ld);
            case MSD_I32: return launch_bd2_t<int32_t>(p, x, off, len, nfiles, max_blocks, band_db, noise_db, delta, ld);
            case MSD_F32: return launch_bd2_t<float>(p, x, off, len, nfiles, max_blocks, band_db, noise_db, delta, ld);
            case MSD_F64: return launch_bd2_t<double>(p, x, off, len, nfiles, max_blocks, band_db, noise_db, delta, ld);
            default: return fail(MSD_ERR_INVALID, "block_delta: unknown dtype");
        }
    }
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
