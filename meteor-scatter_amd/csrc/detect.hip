// Threshold detectors of the reference, float64, numpy-faithful arithmetic:
//   adaptive: get_detections_adaptive()  dsp/src/main.py:450-522
//   global:   get_detections()           dsp/src/main.py:396-448
// One workgroup per file:
//   1. global mean/std of delta (main.py:399-400 / 464-466) with numpy's pairwise
//      summation: the leaves of numpy's recursion tree are summed in parallel, one
//      thread walks the tree to combine them in numpy's order;
//   2. adaptive only: the "fresh" threshold mean+k*std(delta[max(0,i-W):i]) of every
//      block i is independent of the detector state, so all of them are computed in
//      parallel (one thread per block) — only the choice between fixed / fresh /
//      held threshold depends on the freeze state;
//   3. one thread scans the blocks (state: current threshold, freeze_until, open
//      run) on chunks staged through LDS, emitting runs; the detection dB means are
//      then formed in parallel, one thread per detection.
// FP contraction is off so that mean + k*std rounds like numpy's two operations.
#include "msd_internal.h"
#include "np_reduce.h"

#pragma clang fp contract(off)

namespace msd {
namespace {

constexpr int DT_THREADS = 256;
constexpr int DT_MAXLEAF = 4096;  // numpy leaves of >= 64 elements: nb <= 262144 on the parallel path
constexpr int DT_CHUNK = 1024;    // blocks per LDS-staged scan chunk
// The LDS arrays are sized per launch from ld (>= every file's block count): a 60 s file at
// 0.2 s (300 blocks) needs 4.9 KB instead of the 64 KB of the maximal tables, so the LDS no
// longer caps the kernel at two workgroups per CU (1440 files: 2.8 -> 1.4 resident rounds)

struct DetParams {
    msd_det_cfg cfg;
    int64_t ld, cap, nfiles;
    int32_t has_hist, nbuckets;
    int64_t base_us, bucket_us;
    double block_sec;
    int32_t chunk, leaf_cap;  // LDS: blocks per staged chunk, leaf-table entries
};

// dynamic LDS of a launch: c_delta[chunk] | c_thr[chunk] | leaf_sum[leaf_cap] | leaf_off[leaf_cap + 1]
inline size_t det_lds_bytes(int chunk, int leaf_cap) {
    return sizeof(double) * (2 * (size_t)chunk + leaf_cap) + sizeof(int) * ((size_t)leaf_cap + 1);
}

__device__ __forceinline__ int64_t floordiv(int64_t a, int64_t b) {
    int64_t q = a / b;
    if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
    return q;
}

// numpy np.sum over p[0..n) using the whole workgroup (exact numpy association:
// 8192-element buffer chunks, each a pairwise tree; see np_reduce.h)
template <typename A>
__device__ double wg_np_sum(const A &a, int64_t n, int *leaf_off, double *leaf_sum, int *s_nleaf, int leaf_cap) {
    if (n == 0) return 0.0;
    const int tid = threadIdx.x;
    __shared__ double s_res;
    // a sum of n has at most n / 64 + 1 leaves (every leaf of a chunk above 128 holds >= 64)
    if (n / 64 + 2 > leaf_cap) {  // beyond the leaf table: one thread, global reads
        if (tid == 0) s_res = np_sum(a, 0, n);
        __syncthreads();
        const double r = s_res;
        __syncthreads();
        return r;
    }
    if (tid == 0) {
        int cnt = 0;
        for (int64_t c = 0; c < n; c += NP_BUFSIZE) {
            const int64_t m = n - c < NP_BUFSIZE ? n - c : NP_BUFSIZE;
            np_tree_walk(c, m, [&](int64_t b, int64_t) {
                leaf_off[cnt++] = (int)b;
                return 0.0;
            });
        }
        leaf_off[cnt] = (int)n;
        *s_nleaf = cnt;
    }
    __syncthreads();
    const int nl = *s_nleaf;
    for (int l = tid; l < nl; l += DT_THREADS)
        leaf_sum[l] = np_pairwise_leaf(a, leaf_off[l], leaf_off[l + 1] - leaf_off[l]);
    __syncthreads();
    if (tid == 0) {
        int idx = 0;
        double acc = 0.0;
        for (int64_t c = 0; c < n; c += NP_BUFSIZE) {
            const int64_t m = n - c < NP_BUFSIZE ? n - c : NP_BUFSIZE;
            acc += np_tree_walk(c, m, [&](int64_t, int64_t) { return leaf_sum[idx++]; });
        }
        s_res = acc;
    }
    __syncthreads();
    const double r = s_res;
    __syncthreads();
    return r;
}

// 4 waves per SIMD (<= 128 VGPRs; 132 before, 3 per SIMD): with the per-launch LDS, 4 workgroups per CU
// (A/B on C3's 1440 files: 0.168 -> 0.130 ms; 6 per SIMD, every file resident at once, measured the same)
__global__ __launch_bounds__(DT_THREADS, 4) void detect_kernel(const double *__restrict__ delta,
                                                            const int64_t *__restrict__ nblocks, DetParams P,
                                                            msd_det *__restrict__ dets, int64_t *__restrict__ counts,
                                                            double *__restrict__ thr, double *__restrict__ margin,
                                                            int32_t *__restrict__ status,
                                                            const int64_t *__restrict__ file_start_us,
                                                            int64_t *__restrict__ hist) {
    extern __shared__ double dyn_lds[];
    const int64_t chunk = P.chunk;
    double *c_delta = dyn_lds;
    double *c_thr = c_delta + chunk;
    double *leaf_sum = c_thr + chunk;
    int *leaf_off = reinterpret_cast<int *>(leaf_sum + P.leaf_cap);
    __shared__ int s_nleaf;
    __shared__ int64_t s_count;
    __shared__ int32_t s_status;

    const int tid = threadIdx.x;
    const int64_t f = blockIdx.x;
    const int64_t nb = nblocks[f];
    const double *d = delta + f * P.ld;
    const msd_det_cfg &cfg = P.cfg;

    // a file that fits one LDS chunk (a 60 s file: 300 blocks) is staged once: the global sums,
    // the fresh windows and the scan read it from LDS
    const bool whole = nb <= chunk;
    if (whole) {
        for (int64_t i = tid; i < nb; i += DT_THREADS) c_delta[i] = d[i];
        __syncthreads();
    }

    // ---- 1. global threshold (main.py:399-400, :464-466) ----
    // Instantiated once on the LDS copy and once on global memory, never on a pointer that may be
    // either: a generic pointer is read with flat instructions, which pick LDS or global from the
    // address register alone, and a loop pointer the compiler displaces below an LDS object then
    // leaves the LDS aperture (the round-5 fault; tests/test_build_check.py).
    auto global_thr = [&](const double *src) {
        const double s1 = wg_np_sum(ArrRef{src}, nb, leaf_off, leaf_sum, &s_nleaf, P.leaf_cap);
        const double gmean = s1 / (double)nb;
        const double s2 = wg_np_sum(SqDevRef{src, gmean}, nb, leaf_off, leaf_sum, &s_nleaf, P.leaf_cap);
        const double gstd = sqrt(s2 / (double)nb);
        return gmean + cfg.k_std * gstd;
    };
    const double thr0 = whole ? global_thr(c_delta) : global_thr(d);

    // ---- 2. fresh adaptive thresholds (main.py:475-480), all blocks in parallel ----
    double *tf = thr + f * P.ld;
    if (cfg.adaptive) {
        const int64_t W = cfg.window_blocks;
        // The fixed-init blocks first, then one thread per fresh window from the first one on (a 60 s
        // file: 250 windows on 256 threads, one round).  Every window goes through numpy's tree walked
        // iteratively (np_reduce.h), all lanes in one leaf loop; windows of <= 1928 blocks (depth <= 4;
        // 120 s at 0.1 s is 1200) with four-entry stacks, longer ones through np_sum (seven entries,
        // 8192-block chunks).  The LDS-staged file is its own branch, so that the walk's loads are
        // LDS loads, not flat ones.  (The recursive walk's inlined copy per tree shape, run one shape
        // after another by the lanes of a wave, made this phase 0.08 of the kernel's 0.13 ms on C3.)
        const int64_t f0 = cfg.fixed_init_blocks < nb ? (cfg.fixed_init_blocks > 0 ? cfg.fixed_init_blocks : 0) : nb;
        for (int64_t i = tid; i < f0; i += DT_THREADS) tf[i] = thr0;
        auto fresh = [&](const double *p) {
            for (int64_t i = f0 + tid; i < nb; i += DT_THREADS) {
                const int64_t ws = i - W > 0 ? i - W : 0;
                const int64_t wn = i - ws;
                double m, s;
                if (wn <= NP_ITER_MAX[4]) np_mean_std_iter<4>(p, ws, (int)wn, m, s);
                else np_mean_std(p, ws, wn, m, s);
                tf[i] = m + cfg.k_std * s;
            }
        };
        if (whole) fresh(c_delta);
        else fresh(d);
    }
    __syncthreads();

    // ---- 3. serial scan over LDS-staged chunks ----
    // scan state lives in registers of thread 0 across chunks
    double cur_thr = thr0, min_margin = __builtin_inf();
    int64_t freeze_until = -1, ndet = 0, last_stop = -2;
    int32_t st = 0;
    bool prev_above = false;
    int64_t run_start = -1;
    msd_det *df = dets + f * P.cap;
    if (tid == 0 && !cfg.adaptive && nb == 0) st = 2;  // above_thresh[0] on an empty array
    for (int64_t c0 = 0; c0 < nb; c0 += chunk) {
        const int64_t cn = nb - c0 < chunk ? nb - c0 : chunk;
        for (int64_t i = tid; i < cn; i += DT_THREADS) {
            c_delta[i] = d[c0 + i];
            if (cfg.adaptive) c_thr[i] = tf[c0 + i];
        }
        __syncthreads();
        if (cfg.adaptive && tid < 64) {
            // wave 0: at position k lane l evaluates block k+l under the current state (the
            // threshold is thr0 before the fixed-init end, the fresh one after freeze_until,
            // the held one inside a freeze); the first block above its threshold (ballot) is
            // the only place the state changes, so a span without one is a single step
            const int lane = tid;
            int64_t k = 0;
            while (k < cn) {
                const int64_t j = k + lane;
                const bool valid = j < cn;
                const int64_t jc = valid ? j : cn - 1;
                const int64_t i = c0 + jc;
                const double t = i < cfg.fixed_init_blocks ? thr0 : (i > freeze_until ? c_thr[jc] : cur_thr);
                const double dv = c_delta[jc];
                const uint64_t mask = __ballot(valid && dv > t);
                const int first = mask ? __builtin_ctzll(mask) : 64;
                const bool take = valid && lane <= first;
                if (take) c_thr[j] = t;  // the threshold actually used (thresholds list)
                double mg = take ? fabs(dv - t) : __builtin_inf();
                for (int o = 32; o >= 1; o >>= 1) mg = fmin(mg, __shfl_xor(mg, o, 64));
                if (mg < min_margin) min_margin = mg;
                if (!mask) {  // no event in this span: cur_thr follows the last block's threshold
                    const int last = (int)((cn - k < 64 ? cn - k : 64) - 1);
                    cur_thr = __shfl(t, last);
                    k += 64;
                    continue;
                }
                const int64_t e = c0 + k + first;  // event block
                cur_thr = __shfl(t, first);
                if (ndet == 0 || e > last_stop + 1) {
                    if (lane == 0 && ndet > 0 && ndet - 1 < P.cap) df[ndet - 1].stop = last_stop + 1;
                    ++ndet;
                    if (lane == 0 && ndet - 1 < P.cap) df[ndet - 1].start = e;
                }
                last_stop = e;
                const int64_t fu = e + cfg.freeze_after_blocks;
                const int64_t fs = e - cfg.freeze_before_blocks > 0 ? e - cfg.freeze_before_blocks : 0;
                freeze_until = fu > fs ? fu : fs;
                k += first + 1;
            }
        }
        if (!cfg.adaptive && tid == 0) {
            {
                for (int64_t j = 0; j < cn; ++j) {
                    const int64_t i = c0 + j;
                    const double dv = c_delta[j];
                    const double mg = fabs(dv - thr0);
                    if (mg < min_margin) min_margin = mg;
                    const bool above = dv > thr0;
                    if (above && !prev_above) run_start = i;
                    if (!above && prev_above) {  // burst_stops entry i (diff == -1 at i-1, +1)
                        if (ndet < P.cap) {
                            df[ndet].start = run_start;
                            df[ndet].stop = i;
                        }
                        ++ndet;
                    }
                    prev_above = above;
                }
            }
        }
        __syncthreads();
        if (cfg.adaptive && thr != nullptr) {
            for (int64_t i = tid; i < cn; i += DT_THREADS) tf[c0 + i] = c_thr[i];
        }
        __syncthreads();
    }
    if (tid == 0) {
        if (cfg.adaptive) {
            if (ndet > 0 && ndet - 1 < P.cap) df[ndet - 1].stop = last_stop + 1;
        } else if (nb > 0 && prev_above) {  // open burst at the end: stop = len-1 (main.py:414-415)
            if (ndet < P.cap) {
                df[ndet].start = run_start;
                df[ndet].stop = nb - 1;
            }
            if (nb - 1 - run_start <= 0) st = 1;  // t_dur == 0 → assert (main.py:437)
            ++ndet;
        }
        if (ndet > P.cap) st = 3;
        s_count = ndet;
        s_status = st;
        counts[f] = ndet;
        if (margin) margin[f] = min_margin;
        if (!cfg.adaptive && thr != nullptr && P.ld > 0) tf[0] = thr0;
    }
    __syncthreads();
    // ---- dB means (main.py:422-423, :501-502) and per-hour counts ----
    const int64_t nd = s_count < P.cap ? s_count : P.cap;
    for (int64_t c = tid; c < nd; c += DT_THREADS) {
        const int64_t a = df[c].start, b = df[c].stop;
        const int64_t n = b - a;
        // the staged file (LDS) when it fits one chunk; each branch on its own address space (§1 above)
        const double sum = whole ? np_sum(ArrRef{c_delta}, a, n) : np_sum(ArrRef{d}, a, n);
        df[c].db = sum / (double)n;
        if (P.has_hist) {
            const double t_start = (double)a * P.block_sec;
            const int64_t us = llrint(t_start * 1e6);
            const int64_t bk = floordiv(file_start_us[f] + us - P.base_us, P.bucket_us);
            if (bk >= 0 && bk < P.nbuckets)
                atomicAdd(reinterpret_cast<unsigned long long *>(&hist[bk]), 1ULL);
        }
    }
    if (tid == 0 && status) status[f] = s_status;
}

}  // namespace

int launch_detect(msd_ctx *ctx, const double *delta, const int64_t *nblocks, int64_t nfiles, int64_t ld,
                  const msd_det_cfg *cfg, msd_det *dets, int64_t cap, int64_t *counts, double *thresholds,
                  double *margin, int32_t *status, const msd_hist_cfg *hist) {
    if (nfiles == 0) return MSD_OK;
    if (nfiles > 0x7fffffffLL) return fail(MSD_ERR_UNSUPPORTED, "detect: too many files");
    if (cfg->adaptive && thresholds == nullptr)
        return fail(MSD_ERR_INVALID, "detect: adaptive mode needs a thresholds buffer [nfiles][ld]");
    DetParams P;
    P.cfg = *cfg;
    P.ld = ld;
    P.cap = cap;
    P.nfiles = nfiles;
    P.has_hist = hist != nullptr && hist->counts != nullptr;
    P.nbuckets = hist ? hist->nbuckets : 0;
    P.base_us = hist ? hist->base_us : 0;
    P.bucket_us = hist && hist->bucket_us > 0 ? hist->bucket_us : 1;
    P.block_sec = hist ? hist->block_sec : 0.0;
    const int64_t ldc = ld > 0 ? ld : 1;
    P.chunk = (int32_t)(ldc < DT_CHUNK ? ldc : DT_CHUNK);
    P.leaf_cap = (int32_t)(ldc / 64 + 2 < DT_MAXLEAF ? ldc / 64 + 2 : DT_MAXLEAF);
    KernelTimer timer(ctx, K_DSCAN);
    hipLaunchKernelGGL(detect_kernel, dim3((unsigned)nfiles), dim3(DT_THREADS), det_lds_bytes(P.chunk, P.leaf_cap),
                       ctx->stream, delta, nblocks, P,
                       dets, counts, thresholds, margin, status, hist ? hist->file_start_us : nullptr,
                       hist ? hist->counts : nullptr);
    MSD_HIP(hipGetLastError());
    return MSD_OK;
}

}  // namespace msd
