// A/B timer for spectrogram kernel variants.  Loads several builds of libmsdsp.so into one process
// (dlopen, RTLD_LOCAL), gives each its own context, and alternates their launches on the same
// device buffers; each launch is timed by the library's own HIP-event timing on its stream.
// After each variant's first launch it compares two output slices with the first variant's.
//   STFT_AB_MODE=c3 (default): msd_stft_psd_dev, 1440 x 60 s 48 kHz int16, 1024 / 512
//                              (STFT_AB_FILES overrides the file count)
//   STFT_AB_MODE=c5:           msd_cstft_psd_dev, one 3 h 192 kHz int16 I/Q stream, 4096 / 1024
//                              (STFT_AB_F32=1: the same samples as float32 I/Q)
//   STFT_AB_ENERGY=0,1,...: per variant, 1 = msd_cstft_psd_energy_dev (c5; the certification's frame
//                  energy partials) instead of msd_cstft_psd_dev -- the same library can be listed twice
//   STFT_AB_FSUMS=0,1,...: per variant, 1 = msd_cstft_psd_fsums_dev with the frames' exact sample
//                  sums (computed here) -- the exact C5 path's detrend input
//   STFT_AB_CLK=1: a variant built with -DXP_CLK leaves block 0's shader-cycle and 100 MHz
//                  realtime counts in the first 16 output bytes; printed per round.
// Build: g++ -O2 -std=c++17 tools/stft_ab.cpp -I include -I /opt/rocm/include -D__HIP_PLATFORM_AMD__
//        -L /opt/rocm/lib -lamdhip64 -ldl -Wl,-rpath,/opt/rocm/lib -o tools/stft_ab
// Usage: tools/stft_ab ROUNDS LIB [LIB ...]
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "msdsp.h"

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(3);                                                                  \
        }                                                                             \
    } while (0)

struct Lib {
    std::string path;
    void *h = nullptr;
    int (*create)(int, msd_ctx **);
    int (*plan_create)(msd_ctx *, int32_t, int32_t, const float *, double, msd_stft_plan **);
    int (*psd_dev)(msd_stft_plan *, const void *, int, const int64_t *, const int64_t *, int64_t, int64_t, float *,
                   int64_t);
    int (*cplan_create)(msd_ctx *, int32_t, int32_t, const float *, double, msd_cstft_plan **);
    int (*cpsd_dev)(msd_cstft_plan *, const void *, int, const int64_t *, const int64_t *, int64_t, int64_t, float *);
    int (*cpsd_en)(msd_cstft_plan *, const void *, int, const int64_t *, const int64_t *, int64_t, int64_t, float *,
                   float *) = nullptr;
    bool energy = false;  // STFT_AB_ENERGY: this variant also writes the frame energy partials
    int (*cpsd_fs)(msd_cstft_plan *, const void *, int, const int64_t *, const int64_t *, int64_t, int64_t, float *,
                   float *, const double *) = nullptr;
    bool fsums = false;   // STFT_AB_FSUMS: this variant gets the frame sums
    int (*sync)(msd_ctx *);
    int (*t_enable)(msd_ctx *, int);
    int (*t_reset)(msd_ctx *);
    int (*t_get)(msd_ctx *, int, double *, int64_t *);
    const char *(*last_error)(void);
    msd_ctx *ctx = nullptr;
    msd_stft_plan *plan = nullptr;
    msd_cstft_plan *cplan = nullptr;
    std::vector<double> ms;
};

template <typename F>
static void sym(Lib &l, F &f, const char *name) {
    f = reinterpret_cast<F>(dlsym(l.h, name));
    if (!f) {
        fprintf(stderr, "%s: missing %s\n", l.path.c_str(), name);
        exit(2);
    }
}

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s ROUNDS LIB...\n", argv[0]);
        return 2;
    }
    const int rounds = atoi(argv[1]);
    const bool c5 = getenv("STFT_AB_MODE") && !strcmp(getenv("STFT_AB_MODE"), "c5");
    // geometry: nfiles streams of n samples (complex samples for c5), N-point frames at hop
    const int64_t nfiles = c5 ? 1 : (getenv("STFT_AB_FILES") ? atoll(getenv("STFT_AB_FILES")) : 1440);
    const int64_t n = c5 ? 192000LL * 3600 * 3 + 3072 : 2880000;
    // STFT_AB_HOP (c5): another hop (C5: 1024, 75 % overlap)
    const int64_t N = c5 ? 4096 : 1024, K = c5 ? 4096 : 513;
    const int64_t hop = c5 ? (getenv("STFT_AB_HOP") ? atoll(getenv("STFT_AB_HOP")) : 1024) : 512;
    const double fs = c5 ? 192000.0 : 48000.0;
    const int64_t T = (n - N) / hop + 1, ld = c5 ? T : (T + 31) / 32 * 32;
    // STFT_AB_F32=1 (c5): float32 I/Q (the int16 samples / 32768) instead of int16
    const bool f32 = c5 && getenv("STFT_AB_F32");
    const int64_t esz = c5 ? (f32 ? 8 : 4) : 2;  // bytes per sample (int16, or I + Q)
    const int kid = c5 ? 6 : 0;      // msd_timing kernel id
    std::vector<Lib> libs;
    for (int i = 2; i < argc; ++i) {
        Lib l;
        l.path = argv[i];
        l.h = dlopen(argv[i], RTLD_NOW | RTLD_LOCAL);
        if (!l.h) {
            fprintf(stderr, "dlopen %s: %s\n", argv[i], dlerror());
            return 2;
        }
        sym(l, l.create, "msd_create");
        sym(l, l.plan_create, "msd_stft_plan_create");
        sym(l, l.psd_dev, "msd_stft_psd_dev");
        sym(l, l.cplan_create, "msd_cstft_plan_create");
        sym(l, l.cpsd_dev, "msd_cstft_psd_dev");
        sym(l, l.sync, "msd_synchronize");
        sym(l, l.t_enable, "msd_timing_enable");
        sym(l, l.t_reset, "msd_timing_reset");
        sym(l, l.t_get, "msd_timing_get");
        sym(l, l.last_error, "msd_last_error");
        l.cpsd_en = reinterpret_cast<decltype(l.cpsd_en)>(dlsym(l.h, "msd_cstft_psd_energy_dev"));
        if (const char *ev = getenv("STFT_AB_ENERGY")) {
            const int idx = (int)libs.size();
            const char *c = ev;
            for (int k = 0; k < idx && c; ++k) {
                c = strchr(c, ',');
                if (c) ++c;
            }
            l.energy = c && *c == '1';
            if (l.energy && !l.cpsd_en) {
                fprintf(stderr, "%s: no msd_cstft_psd_energy_dev\n", argv[i]);
                return 2;
            }
        }
        l.cpsd_fs = reinterpret_cast<decltype(l.cpsd_fs)>(dlsym(l.h, "msd_cstft_psd_fsums_dev"));
        if (const char *ev = getenv("STFT_AB_FSUMS")) {
            const char *c = ev;
            for (int k = 0; k < (int)libs.size() && c; ++k) {
                c = strchr(c, ',');
                if (c) ++c;
            }
            l.fsums = c && *c == '1';
            if (l.fsums && !l.cpsd_fs) {
                fprintf(stderr, "%s: no msd_cstft_psd_fsums_dev\n", argv[i]);
                return 2;
            }
        }
        libs.push_back(l);
    }
    // periodic Hann (float32) and scipy's density scale 1 / (fs * sum w^2)
    std::vector<float> w(N);
    double s2 = 0;
    for (int i = 0; i < N; ++i) {
        w[i] = (float)(0.5 - 0.5 * std::cos(2.0 * M_PI * i / N));
        s2 += (double)w[i] * w[i];
    }
    const double scale = 1.0 / (fs * s2);
    for (auto &l : libs) {
        int rc = l.create(0, &l.ctx) || l.t_enable(l.ctx, 1);
        if (!rc) rc = c5 ? l.cplan_create(l.ctx, N, hop, w.data(), scale, &l.cplan)
                         : l.plan_create(l.ctx, N, hop, w.data(), scale, &l.plan);
        if (rc) {
            fprintf(stderr, "%s: %s\n", l.path.c_str(), l.last_error());
            return 3;
        }
    }
    // input: c3 = 16 distinct seeded noise + tone files replicated over nfiles (the bench's
    // layout); c5 = one stream built from a repeated 2^22-sample seeded block
    const int64_t npad = c5 ? n : (n + 7) / 8 * 8;
    const int64_t blk = c5 ? (1LL << 22) : npad;
    const int nblk = c5 ? 1 : 16;
    std::vector<int16_t> host((size_t)nblk * blk * (c5 ? 2 : 1), 0);
    std::mt19937 rng(1234);
    std::normal_distribution<float> g(0.f, 1000.f);
    auto q16 = [](float v) { return (int16_t)std::max(-32768.f, std::min(32767.f, std::round(v))); };
    for (int f = 0; f < nblk; ++f)
        for (int64_t i = 0; i < blk; ++i) {
            const float ph = 2.0f * (float)M_PI * 1000.f * (float)i / (float)fs + f;
            if (c5) {
                host[2 * i] = q16(g(rng) + 800.f * std::cos(ph));
                host[2 * i + 1] = q16(g(rng) + 800.f * std::sin(ph));
            } else if (i < n) {
                host[f * blk + i] = q16(g(rng) + 800.f * std::sin(ph) + 37.f * f);
            }
        }
    char *dx;
    float *dout;
    int64_t *doff, *dlen;
    CK(hipMalloc(&dx, (size_t)esz * npad * nfiles));
    CK(hipMalloc(&dout, sizeof(float) * K * ld * nfiles));
    std::vector<float> hostf;
    if (f32) {
        hostf.resize(host.size());
        for (size_t i = 0; i < host.size(); ++i) hostf[i] = host[i] / 32768.f;
    }
    const void *src = f32 ? static_cast<const void *>(hostf.data()) : static_cast<const void *>(host.data());
    if (c5) {
        for (int64_t i = 0; i < n; i += blk)
            CK(hipMemcpy(dx + esz * i, src, (size_t)esz * std::min(blk, n - i), hipMemcpyHostToDevice));
    } else {
        for (int64_t f = 0; f < nfiles; ++f)
            CK(hipMemcpy(dx + esz * f * npad, host.data() + (f % 16) * npad, (size_t)esz * npad,
                         hipMemcpyHostToDevice));
    }
    std::vector<int64_t> off(nfiles), len(nfiles, n);
    for (int64_t f = 0; f < nfiles; ++f) off[f] = f * npad;
    CK(hipMalloc(&doff, sizeof(int64_t) * nfiles));
    CK(hipMalloc(&dlen, sizeof(int64_t) * nfiles));
    CK(hipMemcpy(doff, off.data(), sizeof(int64_t) * nfiles, hipMemcpyHostToDevice));
    CK(hipMemcpy(dlen, len.data(), sizeof(int64_t) * nfiles, hipMemcpyHostToDevice));
    const double gbytes = (double)nfiles * ((double)esz * n + 4.0 * K * T) * 1e-9;
    float *detot = nullptr;
    if (c5) CK(hipMalloc(&detot, sizeof(float) * 16 * (T + 4)));
    double *dfs = nullptr;  // STFT_AB_FSUMS: frame t's (sum I, sum Q) of the periodic c5 stream
    if (c5 && getenv("STFT_AB_FSUMS")) {
        std::vector<int64_t> P(2 * (blk + 1), 0);
        for (int64_t i = 0; i < blk; ++i)
            for (int c = 0; c < 2; ++c) P[2 * (i + 1) + c] = P[2 * i + c] + host[2 * i + c];
        auto F = [&](int64_t x, int c) { return (x / blk) * P[2 * blk + c] + P[2 * (x % blk) + c]; };
        std::vector<double> fs(2 * T);
        for (int64_t t = 0; t < T; ++t)
            for (int c = 0; c < 2; ++c) fs[2 * t + c] = (double)(F(t * hop + N, c) - F(t * hop, c));
        CK(hipMalloc(&dfs, sizeof(double) * 2 * T));
        CK(hipMemcpy(dfs, fs.data(), sizeof(double) * 2 * T, hipMemcpyHostToDevice));
    }
    auto launch = [&](Lib &l) {
        if (c5 && l.fsums)
            return l.cpsd_fs(l.cplan, dx, f32 ? MSD_CF32 : MSD_CI16, doff, dlen, nfiles, T, dout, l.energy ? detot : nullptr, dfs);
        if (c5 && l.energy) return l.cpsd_en(l.cplan, dx, f32 ? MSD_CF32 : MSD_CI16, doff, dlen, nfiles, T, dout, detot);
        return c5 ? l.cpsd_dev(l.cplan, dx, f32 ? MSD_CF32 : MSD_CI16, doff, dlen, nfiles, T, dout)
                  : l.psd_dev(l.plan, dx, MSD_I16, doff, dlen, nfiles, T, dout, ld);
    };

    // two output slices compared with the first variant's: c3 the first and last file
    // ([K][ld] each, checked per frame), c5 the first and last 1024 frames ([frame][K])
    const int64_t fsz = c5 ? 1024 * K : K * ld;
    std::vector<float> ref0(fsz), ref1(fsz), cur(fsz);
    for (size_t v = 0; v < libs.size(); ++v) {
        Lib &l = libs[v];
        CK(hipMemset(dout, 0xff, sizeof(float) * fsz));
        if (launch(l) || l.sync(l.ctx)) {
            fprintf(stderr, "%s: %s\n", l.path.c_str(), l.last_error());
            return 4;
        }
        for (int which = 0; which < 2; ++which) {
            const int64_t o = which ? (c5 ? (T - 1024) * K : (nfiles - 1) * fsz) : 0;
            CK(hipMemcpy(v == 0 ? (which ? ref1.data() : ref0.data()) : cur.data(), dout + o, sizeof(float) * fsz,
                         hipMemcpyDeviceToHost));
            if (v == 0) continue;
            const std::vector<float> &r = which ? ref1 : ref0;
            double maxrel = 0;
            int64_t ndiff = 0;
            const int64_t nfr = c5 ? 1024 : T;
            for (int64_t t = 0; t < nfr; ++t) {
                double fm = 0, em = 0;
                for (int64_t k = 0; k < K; ++k) {
                    const int64_t i = c5 ? t * K + k : k * ld + t;
                    fm = std::max(fm, (double)std::fabs(r[i]));
                    em = std::max(em, (double)std::fabs(r[i] - cur[i]));
                    ndiff += r[i] != cur[i];
                }
                maxrel = std::max(maxrel, em / fm);
            }
            printf("variant %zu slice %d vs variant 0: %ld values differ, max per-frame rel err %.3e\n", v, which,
                   (long)ndiff, maxrel);
        }
    }
    // warm-up, then alternate
    for (auto &l : libs)
        for (int i = 0; i < 3; ++i) launch(l);
    for (auto &l : libs) l.sync(l.ctx);
    for (int r = 0; r < rounds; ++r)
        for (auto &l : libs) {
            l.t_reset(l.ctx);
            for (int i = 0; i < 5; ++i) launch(l);
            l.sync(l.ctx);
            double ms = 0;
            int64_t launches = 0;
            l.t_get(l.ctx, kid, &ms, &launches);
            if (c5) {  // + the spectrogram's fix-up kernels where a library has them (round-4 dc_fix, id 11)
                double ms2 = 0;
                int64_t l2 = 0;
                l.t_get(l.ctx, 11, &ms2, &l2);
                if (l2 > 0) ms += ms2;
            }
            l.ms.push_back(ms / launches);
            if (getenv("STFT_AB_CLK")) {
                uint64_t c[2];
                CK(hipMemcpy(c, dout, 16, hipMemcpyDeviceToHost));
                printf("%s: block 0 shader cycles %llu, realtime ticks %llu -> %.0f MHz (at 100 MHz realtime)\n",
                       l.path.c_str(), (unsigned long long)c[0], (unsigned long long)c[1], 100.0 * c[0] / c[1]);
            }
        }
    for (size_t v = 0; v < libs.size(); ++v) {
        auto m = libs[v].ms;
        std::sort(m.begin(), m.end());
        printf("%-60s min %.4f  median %.4f ms  (%.1f GB/s, frac %.4f)\n", libs[v].path.c_str(), m[0],
               m[m.size() / 2], gbytes / m[m.size() / 2] * 1e3, gbytes / m[m.size() / 2] * 1e3 / 8000.0);
    }
    return 0;
}
