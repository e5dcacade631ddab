// A/B timer for STFT kernel variants on the C3 workload (1440 x 60 s 48 kHz int16, 1024 / 512).
// Loads several builds of libmsdsp.so into one process (dlopen, RTLD_LOCAL), gives each its own
// context, and alternates their msd_stft_psd_dev launches on the same device buffers; the time
// of each launch comes from the library's own HIP-event timing on its stream.  After each
// variant's first launch it compares two files' spectrograms with the first variant's.
// Build: g++ -O2 -std=c++17 tools/stft_ab.cpp -I include -I /opt/rocm/include -D__HIP_PLATFORM_AMD__
//        -L /opt/rocm/lib -lamdhip64 -ldl -o tools/stft_ab
// Usage: tools/stft_ab ROUNDS LIB [LIB ...]   (nfiles via STFT_AB_FILES, default 1440)
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>
#include <algorithm>

#include "msdsp.h"

struct Lib {
    std::string path;
    void *h = nullptr;
    int (*create)(int, msd_ctx **);
    int (*plan_create)(msd_ctx *, int32_t, int32_t, const float *, double, msd_stft_plan **);
    int (*psd_dev)(msd_stft_plan *, const void *, int, const int64_t *, const int64_t *, int64_t, int64_t, float *,
                   int64_t);
    int (*sync)(msd_ctx *);
    int (*t_enable)(msd_ctx *, int);
    int (*t_reset)(msd_ctx *);
    int (*t_get)(msd_ctx *, int, double *, int64_t *);
    const char *(*last_error)(void);
    msd_ctx *ctx = nullptr;
    msd_stft_plan *plan = nullptr;
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

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(3);                                                           \
        }                                                                      \
    } while (0)

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s ROUNDS LIB...\n", argv[0]);
        return 2;
    }
    const int rounds = atoi(argv[1]);
    const int64_t nfiles = getenv("STFT_AB_FILES") ? atoll(getenv("STFT_AB_FILES")) : 1440;
    const int64_t n = 2880000, N = 1024, hop = 512, K = 513;
    const int64_t T = (n - N) / hop + 1, ld = (T + 31) / 32 * 32;
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
        sym(l, l.sync, "msd_synchronize");
        sym(l, l.t_enable, "msd_timing_enable");
        sym(l, l.t_reset, "msd_timing_reset");
        sym(l, l.t_get, "msd_timing_get");
        sym(l, l.last_error, "msd_last_error");
        libs.push_back(l);
    }
    // periodic Hann (float32) and scipy's density scale 1 / (fs * sum w^2)
    std::vector<float> w(N);
    double s2 = 0;
    for (int i = 0; i < N; ++i) {
        w[i] = (float)(0.5 - 0.5 * std::cos(2.0 * M_PI * i / N));
        s2 += (double)w[i] * w[i];
    }
    const double scale = 1.0 / (48000.0 * s2);
    for (auto &l : libs) {
        if (l.create(0, &l.ctx) || l.plan_create(l.ctx, N, hop, w.data(), scale, &l.plan) || l.t_enable(l.ctx, 1)) {
            fprintf(stderr, "%s: %s\n", l.path.c_str(), l.last_error());
            return 3;
        }
    }
    // 16 distinct seeded noise + tone files, replicated over nfiles (the bench's layout)
    const int64_t npad = (n + 7) / 8 * 8;
    std::vector<int16_t> host(16 * npad, 0);
    std::mt19937 rng(1234);
    std::normal_distribution<float> g(0.f, 1000.f);
    for (int f = 0; f < 16; ++f)
        for (int64_t i = 0; i < n; ++i) {
            float v = g(rng) + 800.f * std::sin(2.0f * (float)M_PI * 1000.f * (float)i / 48000.f + f) + 37.f * f;
            host[f * npad + i] = (int16_t)std::max(-32768.f, std::min(32767.f, std::round(v)));
        }
    int16_t *dx;
    float *dout;
    int64_t *doff, *dlen;
    CK(hipMalloc(&dx, sizeof(int16_t) * npad * nfiles));
    CK(hipMalloc(&dout, sizeof(float) * K * ld * nfiles));
    for (int64_t f = 0; f < nfiles; ++f)
        CK(hipMemcpy(dx + f * npad, host.data() + (f % 16) * npad, sizeof(int16_t) * npad, hipMemcpyHostToDevice));
    std::vector<int64_t> off(nfiles), len(nfiles, n);
    for (int64_t f = 0; f < nfiles; ++f) off[f] = f * npad;
    CK(hipMalloc(&doff, sizeof(int64_t) * nfiles));
    CK(hipMalloc(&dlen, sizeof(int64_t) * nfiles));
    CK(hipMemcpy(doff, off.data(), sizeof(int64_t) * nfiles, hipMemcpyHostToDevice));
    CK(hipMemcpy(dlen, len.data(), sizeof(int64_t) * nfiles, hipMemcpyHostToDevice));
    const double gbytes = (double)nfiles * (2.0 * n + 4.0 * K * T) * 1e-9;

    // reference output of two files (first and last) from the first variant
    const int64_t fsz = K * ld;
    std::vector<float> ref0(fsz), ref1(fsz), cur(fsz);
    for (size_t v = 0; v < libs.size(); ++v) {
        Lib &l = libs[v];
        CK(hipMemset(dout, 0xff, sizeof(float) * K * ld * 2));
        if (l.psd_dev(l.plan, dx, MSD_I16, doff, dlen, nfiles, T, dout, ld) || l.sync(l.ctx)) {
            fprintf(stderr, "%s: %s\n", l.path.c_str(), l.last_error());
            return 4;
        }
        for (int which = 0; which < 2; ++which) {
            const int64_t f = which ? nfiles - 1 : 0;
            CK(hipMemcpy(v == 0 ? (which ? ref1.data() : ref0.data()) : cur.data(), dout + f * fsz,
                         sizeof(float) * fsz, hipMemcpyDeviceToHost));
            if (v == 0) continue;
            const std::vector<float> &r = which ? ref1 : ref0;
            double maxrel = 0;
            int64_t ndiff = 0;
            for (int64_t t = 0; t < T; ++t) {
                double fm = 0, em = 0;
                for (int64_t k = 0; k < K; ++k) {
                    fm = std::max(fm, (double)std::fabs(r[k * ld + t]));
                    em = std::max(em, (double)std::fabs(r[k * ld + t] - cur[k * ld + t]));
                    ndiff += r[k * ld + t] != cur[k * ld + t];
                }
                maxrel = std::max(maxrel, em / fm);
            }
            printf("variant %zu file %ld vs variant 0: %ld values differ, max per-frame rel err %.3e\n", v, (long)f,
                   (long)ndiff, maxrel);
        }
    }
    // warm-up, then alternate
    for (auto &l : libs)
        for (int i = 0; i < 3; ++i) l.psd_dev(l.plan, dx, MSD_I16, doff, dlen, nfiles, T, dout, ld);
    for (auto &l : libs) l.sync(l.ctx);
    for (int r = 0; r < rounds; ++r)
        for (auto &l : libs) {
            l.t_reset(l.ctx);
            for (int i = 0; i < 5; ++i) l.psd_dev(l.plan, dx, MSD_I16, doff, dlen, nfiles, T, dout, ld);
            l.sync(l.ctx);
            double ms = 0;
            int64_t launches = 0;
            l.t_get(l.ctx, 0, &ms, &launches);
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
        printf("%-60s min %.4f  median %.4f ms  (%.1f GB/s, frac %.4f)\n", libs[v].path.c_str(), m[0], m[m.size() / 2],
               gbytes / m[m.size() / 2] * 1e3, gbytes / m[m.size() / 2] * 1e3 / 8000.0);
    }
    return 0;
}
