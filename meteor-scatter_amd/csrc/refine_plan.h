// The host half of msd_iq_delta64_dev (refine.hip), plain C++ (no HIP) so that the CPU sanitizer
// harness (host_check.cpp) can run it: the bins the float64 refinement needs (every band / noise
// bin and its two neighbours, each once, in np.sum's mask order), the block geometry (blocks of
// D = gcd(N, hop) samples, R = N / D per frame), the rounding-chain constant of the error bound, and
// the frame ranges mapped to compact block ranges.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <numeric>
#include <string>
#include <vector>

namespace msd {

constexpr int RF_MAXK = 32;  // needed bins (band and noise bins +- 1)

struct RefineBins {
    int nk;                   // needed bins k' (signed, -N/2 <= k' < N/2 + 1, taken mod N)
    int k[RF_MAXK];
    int km[RF_MAXK];          // k' mod N
    int nb, nn;               // band / noise bins, in np.sum order (ascending FFT index)
    int bidx[RF_MAXK / 2][3]; // per band bin: indices into k[] of k-1, k, k+1
    int nidx[RF_MAXK / 2][3];
    int dc;                   // index into k[] of bin 0, or -1
};

struct RefineGeom {
    int N, D, R, L;           // frame, block, blocks per frame, samples per Goertzel segment
    int rows;                 // 1: block_kernel (D % 64 == 0: 16 lanes x D/16 samples, 16-B aligned quads);
                              // 0: block_small_kernel (one lane per block, any D)
    int64_t hop;
    double scale;             // density: 1 / (fs sum w^2)
    double chain;             // our float64 rounding chain + the reference's, in units of u
    double chain_tail;        // the part of `chain` after the block values (frame combination, taps,
                              // |Y|^2, the reference's chain): chain = own block step + chain_tail
    int nr;                   // frame ranges
};

struct RefinePlan {
    RefineBins K;
    RefineGeom G;
    std::vector<int64_t> fstart, fcs, bstart, bcs;  // per range: first frame, compact frame start;
                                                    // first block, compact block start (+ totals)
    int64_t nblocks = 0, nframes = 0;
};

// 0, or -1 (bad arguments) / -3 (unsupported) with msg set
inline int plan_refine(int nperseg, int64_t hop, double fs, int band_lo, int band_hi, int noise_lo, int noise_hi,
                       const int64_t *ranges, int64_t nranges, int64_t n_samples, RefinePlan &P, std::string &msg) {
    enum { OK = 0, E_INVALID = -1, E_UNSUPPORTED = -3 };
    auto err = [&](int code, const char *m) {
        msg = m;
        return code;
    };
    if (nperseg < 4 || hop <= 0 || !(fs > 0) || nranges < 0 || (nranges && !ranges))
        return err(E_INVALID, "bad arguments");
    // the kernels form twiddle indices k * n (k < N, n <= N) in 32 bits
    if (nperseg > 65536) return err(E_UNSUPPORTED, "nperseg above 65536");
    const int N = nperseg;
    const int h = N / 2;
    auto ok = [&](int lo, int hi) { return hi < lo || (lo >= -h && hi <= N - h - 1); };
    if (!ok(band_lo, band_hi) || !ok(noise_lo, noise_hi))
        return err(E_INVALID, "band outside -N/2 .. N/2-1");
    // needed bins: every band / noise bin and its two neighbours (mod N), each once
    RefineBins &K = P.K;
    K = RefineBins{};
    K.dc = -1;
    auto slot = [&](int kk) -> int {
        const int km = ((kk % N) + N) % N;
        for (int i = 0; i < K.nk; ++i)
            if (((K.k[i] % N) + N) % N == km) return i;
        if (K.nk >= RF_MAXK) return -1;
        K.k[K.nk] = kk;
        return K.nk++;
    };
    // np.sum order over the boolean mask: ascending FFT index (bins >= 0 first, then the negative ones)
    auto fill = [&](int lo, int hi, int (*idx)[3], int &n) -> bool {
        n = 0;
        if (hi < lo) return true;
        std::vector<int> order;
        for (int b = lo; b <= hi; ++b)
            if (b >= 0) order.push_back(b);
        for (int b = lo; b <= hi; ++b)
            if (b < 0) order.push_back(b);
        if ((int)order.size() > RF_MAXK / 2) return false;
        for (int b : order) {
            const int a = slot(b - 1), c = slot(b), e = slot(b + 1);
            if (a < 0 || c < 0 || e < 0) return false;
            idx[n][0] = a;
            idx[n][1] = c;
            idx[n][2] = e;
            ++n;
        }
        return true;
    };
    if (!fill(band_lo, band_hi, K.bidx, K.nb) || !fill(noise_lo, noise_hi, K.nidx, K.nn))
        return err(E_UNSUPPORTED, "bands too wide for the refinement kernel");
    for (int i = 0; i < K.nk; ++i) {
        K.km[i] = ((K.k[i] % N) + N) % N;
        if (K.km[i] == 0) K.dc = i;
    }
    RefineGeom &G = P.G;
    G = RefineGeom{};
    G.N = N;
    G.hop = hop;
    G.D = (int)std::gcd((int64_t)N, hop);
    G.R = N / G.D;
    // block_kernel runs 16 lanes of D/16 samples each and loads them four at a time (16-B quads at
    // m D + n0): D must be a multiple of 64; any other D (e.g. N 1000, hop 500: D 500) takes the
    // one-lane-per-block direct DFT
    G.rows = G.D % 64 == 0 ? 1 : 0;
    G.L = G.rows ? G.D / 16 : G.D;  // samples per Goertzel segment (direct products)
    // periodic Hann: sum w^2 = 3N/8 exactly; scipy's scale 1/(fs * sum(w^2)) from its float64 window
    // (the sum per frame length kept per thread: N cosines cost ~0.1 ms of host time per call,
    // which the C5 step paid between every two steps)
    {
        static thread_local int sw_n = 0;
        static thread_local double sw_v = 0.0;
        if (sw_n != N) {
            double sw = 0.0;
            for (int n = 0; n < N; ++n) {
                const double w = 0.5 - 0.5 * std::cos(2.0 * M_PI * (double)n / (double)N);
                sw += w * w;
            }
            sw_v = sw;
            sw_n = N;
        }
        G.scale = 1.0 / (fs * sw_v);
    }
    // rounding chains in units of u = 2^-53: ours -- the Goertzel recurrence over L samples (3 L
    // Gmax + 8, Gmax = min(1/|sin theta|, L) its error gain), the wave sum (6), the R-block
    // combination (R + 4), the mean, Hann taps and |Y|^2 (8); the reference's pocketfft chain plus
    // detrend and window (4 log2 N + 11)
    double gmax = 1.0;
    for (int i = 0; i < K.nk; ++i) {
        const int km = ((K.k[i] % N) + N) % N;
        if (km == 0) continue;
        const double sn = std::fabs(std::sin(2.0 * M_PI * km / N));
        gmax = std::max(gmax, std::min(sn > 0 ? 1.0 / sn : 1e300, (double)G.L));
    }
    // the one-lane path sums D direct products (D + 4); the Goertzel path 3 L Gmax + 8 and the 16-lane sum
    const double own = G.rows ? 3.0 * G.L * gmax + 8.0 + 4.0 : (double)G.D + 4.0;
    G.chain_tail = (G.R + 4.0) + 8.0 + 4.0 * std::log2((double)N) + 11.0;
    G.chain = own + G.chain_tail;
    if (nranges > (1 << 20)) return err(E_UNSUPPORTED, "too many ranges");
    // frame ranges -> block ranges, compact prefix counts
    std::vector<int64_t> &fstart = P.fstart, &fcs = P.fcs, &bstart = P.bstart, &bcs = P.bcs;
    fstart.assign(nranges, 0);
    fcs.assign(nranges + 1, 0);
    bstart.assign(nranges, 0);
    bcs.assign(nranges + 1, 0);
    fcs[0] = bcs[0] = 0;
    for (int64_t r = 0; r < nranges; ++r) {
        const int64_t a = ranges[2 * r], b = ranges[2 * r + 1];
        if (a < 0 || b <= a || (b - 1) * hop + N > n_samples || (r > 0 && a < ranges[2 * r - 1]))
            return err(E_INVALID, "ranges must be sorted, disjoint, inside the samples");
        fstart[r] = a;
        fcs[r + 1] = fcs[r] + (b - a);
        bstart[r] = a * hop / G.D;
        bcs[r + 1] = bcs[r] + ((b - 1) * hop / G.D + G.R - bstart[r]);
    }
    G.nr = (int)nranges;
    P.nblocks = bcs[nranges];
    P.nframes = fcs[nranges];
    return OK;
}

}  // namespace msd
