// C-ABI of libmsdsp.so (include/msdsp.h): contexts, plans, device memory, the
// host-buffer convenience entry points, per-kernel event timing and the RCCL
// communicator used to reduce per-hour detection counts across GPUs.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <map>
#include <set>
#include <tuple>

#include <vector>

#include "msd_internal.h"

namespace msd {

static thread_local std::string g_last_error;

void set_error(const std::string &msg) { g_last_error = msg; }
int fail(int code, const std::string &msg) {
    set_error(msg);
    return code;
}
int hip_fail(hipError_t e, const char *what) {
    return fail(MSD_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

int ensure_dyn_lds(const void *kernel, int bytes) {
    // the attribute is a per-kernel maximum: only ever raised, so a smaller request after a larger
    // one (plans of different sizes sharing one instantiation) never lowers it under a later launch
    static std::mutex mu;
    static std::map<std::pair<const void *, int>, int> set_to;  // (kernel, device) -> bytes set
    int dev = 0;
    MSD_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lock(mu);
    int &cur = set_to[{kernel, dev}];
    if (bytes <= cur) return MSD_OK;
    MSD_HIP(hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
    cur = bytes;
    return MSD_OK;
}

KernelTimer::KernelTimer(msd_ctx *c, int k) : ctx(c), kernel(k) {
    if (!ctx->timing || !((ctx->timing_mask >> k) & 1u)) return;
    auto take = [&]() {
        hipEvent_t e = nullptr;
        if (!ctx->pool.empty()) {
            e = ctx->pool.back();
            ctx->pool.pop_back();
        } else if (hipEventCreate(&e) != hipSuccess) {
            e = nullptr;
        }
        return e;
    };
    a = take();
    b = take();
    if (a && b) hipEventRecord(a, ctx->stream);
}
KernelTimer::~KernelTimer() {
    if (!ctx->timing || !a || !b) return;
    hipEventRecord(b, ctx->stream);
    ctx->pending.push_back({a, b, kernel});
}

int ctx_scratch(msd_ctx *ctx, int slot, size_t bytes, void **out) {
    if (ctx->scratch_bytes[slot] < bytes) {
        if (ctx->scratch[slot]) {
            MSD_HIP(hipStreamSynchronize(ctx->stream));
            MSD_HIP(hipFree(ctx->scratch[slot]));
            ctx->scratch[slot] = nullptr;
            ctx->scratch_bytes[slot] = 0;
        }
        size_t want = bytes < 4096 ? 4096 : bytes;
        ctx->rf_last_dev = nullptr;  // a new block (perhaps at the old address) holds no uploaded tables
        MSD_HIP(hipMalloc(&ctx->scratch[slot], want));
        ctx->scratch_bytes[slot] = want;
    }
    *out = ctx->scratch[slot];
    return MSD_OK;
}

// ---------------------------------------------------------------- RCCL (dlopen)
struct Rccl {
    void *h = nullptr;
    ncclResult_t (*getUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*commInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*allReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                              hipStream_t) = nullptr;
    ncclResult_t (*allGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
    const char *(*getErrorString)(ncclResult_t) = nullptr;
    bool ok = false;
};

static Rccl *rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        const char *names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
        for (const char *n : names) {
            r.h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
            if (r.h) break;
        }
        if (!r.h) return;
        r.getUniqueId = reinterpret_cast<decltype(r.getUniqueId)>(dlsym(r.h, "ncclGetUniqueId"));
        r.commInitRank = reinterpret_cast<decltype(r.commInitRank)>(dlsym(r.h, "ncclCommInitRank"));
        r.allReduce = reinterpret_cast<decltype(r.allReduce)>(dlsym(r.h, "ncclAllReduce"));
        r.allGather = reinterpret_cast<decltype(r.allGather)>(dlsym(r.h, "ncclAllGather"));
        r.commDestroy = reinterpret_cast<decltype(r.commDestroy)>(dlsym(r.h, "ncclCommDestroy"));
        r.getErrorString = reinterpret_cast<decltype(r.getErrorString)>(dlsym(r.h, "ncclGetErrorString"));
        r.ok = r.getUniqueId && r.commInitRank && r.allReduce && r.allGather && r.commDestroy;
    });
    return r.ok ? &r : nullptr;
}

static int rccl_fail(Rccl *r, ncclResult_t e, const char *what) {
    std::string m = std::string(what) + ": rccl error " + std::to_string((int)e);
    if (r && r->getErrorString) m += std::string(" (") + r->getErrorString(e) + ")";
    return fail(MSD_ERR_RCCL, m);
}

}  // namespace msd

struct msd_comm {
    msd_ctx *ctx = nullptr;
    ncclComm_t comm = nullptr;
};

using namespace msd;

extern "C" {

int msd_abi_version(void) { return MSD_ABI_VERSION; }

const char *msd_last_error(void) { return g_last_error.c_str(); }

int msd_device_count(int *count) {
    if (!count) return fail(MSD_ERR_INVALID, "msd_device_count: null");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *count = 0;
        return hip_fail(e, "hipGetDeviceCount");
    }
    *count = n;
    return MSD_OK;
}

int msd_create(int device, msd_ctx **out) {
    if (!out) return fail(MSD_ERR_INVALID, "msd_create: null out");
    *out = nullptr;
    int n = 0;
    MSD_HIP(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return fail(MSD_ERR_INVALID, "msd_create: no such device");
    MSD_HIP(hipSetDevice(device));
    auto *c = new msd_ctx();
    c->device = device;
    if (hipDeviceGetAttribute(&c->num_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
        c->num_cu <= 0)
        c->num_cu = 256;  // grid sizing only: a wrong count costs balance, not correctness
    c->num_cu_dev = c->num_cu;
    if (const char *e = getenv("MSD_CSTFT_SCHED"))  // A/B runs: static | chunked (MSD_OPT_CSTFT_SCHED)
        c->cstft_sched = !strcmp(e, "static") ? 1 : !strcmp(e, "chunked") ? 2 : 0;
    if (const char *e = getenv("MSD_STFT_SCHED"))  // the same for stft1024_kernel (MSD_OPT_STFT_SCHED)
        c->stft_sched = !strcmp(e, "static") ? 1 : !strcmp(e, "chunked") ? 2 : 0;
    if (const char *e = getenv("MSD_BLOCK_GOERTZEL"))  // A/B runs: MSD_OPT_BLOCK_GOERTZEL
        c->block_goertzel = atoi(e) != 0;
    if (const char *e = getenv("MSD_WELCH_GOERTZEL"))  // A/B runs: MSD_OPT_WELCH_GOERTZEL
        c->welch_goertzel = atoi(e) != 0;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return hip_fail(e, "hipStreamCreate");
    }
    *out = c;
    return MSD_OK;
}

void msd_destroy(msd_ctx *ctx) {
    if (!ctx) return;
    DeviceGuard g(ctx->device);
    hipStreamSynchronize(ctx->stream);
    for (auto &p : ctx->pending) {
        hipEventDestroy(p.a);
        hipEventDestroy(p.b);
    }
    for (auto e : ctx->pool) hipEventDestroy(e);
    for (void *p : ctx->scratch)
        if (p) hipFree(p);
    if (ctx->rf_w) hipFree(ctx->rf_w);
    if (ctx->rf_ev) hipEventSynchronize(ctx->rf_ev), hipEventDestroy(ctx->rf_ev);
    if (ctx->rf_pin) hipHostFree(ctx->rf_pin);
    if (ctx->i8_tab) hipFree(ctx->i8_tab);
    if (ctx->copy_stream) {
        hipStreamSynchronize(ctx->copy_stream);
        hipStreamDestroy(ctx->copy_stream);
    }
    if (ctx->fence_ev) hipEventDestroy(ctx->fence_ev);
    if (ctx->join_ev) hipEventDestroy(ctx->join_ev);
    hipStreamDestroy(ctx->stream);
    delete ctx;
}

int msd_synchronize(msd_ctx *ctx) {
    if (!ctx) return fail(MSD_ERR_INVALID, "null ctx");
    DeviceGuard g(ctx->device);
    MSD_HIP(hipStreamSynchronize(ctx->stream));
    return MSD_OK;
}

int msd_dev_alloc(msd_ctx *ctx, size_t bytes, void **dptr) {
    if (!ctx || !dptr) return fail(MSD_ERR_INVALID, "msd_dev_alloc: null");
    DeviceGuard g(ctx->device);
    *dptr = nullptr;
    MSD_HIP(hipMalloc(dptr, bytes ? bytes : 16));
    return MSD_OK;
}

int msd_dev_free(msd_ctx *ctx, void *dptr) {
    if (!ctx) return fail(MSD_ERR_INVALID, "msd_dev_free: null ctx");
    if (!dptr) return MSD_OK;
    DeviceGuard g(ctx->device);
    MSD_HIP(hipStreamSynchronize(ctx->stream));
    MSD_HIP(hipFree(dptr));
    return MSD_OK;
}

int msd_memcpy_h2d(msd_ctx *ctx, void *dst, const void *src, size_t bytes) {
    if (!ctx || (!dst && bytes) || (!src && bytes)) return fail(MSD_ERR_INVALID, "msd_memcpy_h2d: null");
    if (!bytes) return MSD_OK;
    DeviceGuard g(ctx->device);
    MSD_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
    MSD_HIP(hipStreamSynchronize(ctx->stream));
    return MSD_OK;
}

int msd_memcpy_d2h(msd_ctx *ctx, void *dst, const void *src, size_t bytes) {
    if (!ctx || (!dst && bytes) || (!src && bytes)) return fail(MSD_ERR_INVALID, "msd_memcpy_d2h: null");
    if (!bytes) return MSD_OK;
    DeviceGuard g(ctx->device);
    MSD_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    MSD_HIP(hipStreamSynchronize(ctx->stream));
    return MSD_OK;
}

int msd_memset_dev(msd_ctx *ctx, void *dst, int value, size_t bytes) {
    if (!ctx || (!dst && bytes)) return fail(MSD_ERR_INVALID, "msd_memset_dev: null");
    if (!bytes) return MSD_OK;
    DeviceGuard g(ctx->device);
    MSD_HIP(hipMemsetAsync(dst, value, bytes, ctx->stream));
    return MSD_OK;
}

int msd_set_option(msd_ctx *ctx, int option, int value) {
    if (!ctx) return fail(MSD_ERR_INVALID, "null ctx");
    switch (option) {
        case MSD_OPT_GENERIC_STFT: ctx->force_generic = value != 0; return MSD_OK;
        case MSD_OPT_FRESH_ALL: ctx->fresh_all = value != 0; return MSD_OK;
        case MSD_OPT_REFINE_GOERTZEL: ctx->refine_goertzel = value != 0; return MSD_OK;
        case MSD_OPT_BLOCK_GOERTZEL: ctx->block_goertzel = value != 0; return MSD_OK;
        case MSD_OPT_WELCH_GOERTZEL: ctx->welch_goertzel = value != 0; return MSD_OK;
        case MSD_OPT_CSTFT_RESERVE:
            if (value < 0) return fail(MSD_ERR_INVALID, "msd_set_option: MSD_OPT_CSTFT_RESERVE must be >= 0");
            ctx->cstft_reserve = value;
            return MSD_OK;
        case MSD_OPT_CSTFT_SCHED:
            if (value < 0 || value > 2) return fail(MSD_ERR_INVALID, "msd_set_option: MSD_OPT_CSTFT_SCHED is 0, 1 or 2");
            ctx->cstft_sched = value;
            return MSD_OK;
        case MSD_OPT_STFT_SCHED:
            if (value < 0 || value > 2) return fail(MSD_ERR_INVALID, "msd_set_option: MSD_OPT_STFT_SCHED is 0, 1 or 2");
            ctx->stft_sched = value;
            return MSD_OK;
        case MSD_OPT_STREAM_CUS: {
            // the context's stream re-created on a CU subset: n > 0 the first n CUs of the mask, n < 0
            // all but those |n| (the two are disjoint), 0 every CU; grid sizing follows (num_cu)
            const int total = ctx->num_cu_dev;
            if (value >= total || -value >= total)
                return fail(MSD_ERR_INVALID, "msd_set_option: MSD_OPT_STREAM_CUS out of range");
            DeviceGuard g(ctx->device);
            MSD_HIP(hipStreamSynchronize(ctx->stream));
            hipStream_t st = nullptr;
            if (value == 0) {
                MSD_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
            } else {
                std::vector<uint32_t> mask((size_t)(total + 31) / 32, 0u);
                const int lo = value > 0 ? 0 : -value, hi = value > 0 ? value : total;
                for (int c = lo; c < hi; ++c) mask[(size_t)c / 32] |= 1u << (c % 32);
                MSD_HIP(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()));
            }
            MSD_HIP(hipStreamDestroy(ctx->stream));
            ctx->stream = st;
            ctx->num_cu = value == 0 ? total : value > 0 ? value : total + value;
            ctx->stream_cus = value;
            return MSD_OK;
        }
        default: return fail(MSD_ERR_INVALID, "msd_set_option: unknown option");
    }
}

int msd_timing_enable(msd_ctx *ctx, int enable) {
    if (!ctx) return fail(MSD_ERR_INVALID, "null ctx");
    ctx->timing = enable != 0;
    return MSD_OK;
}

int msd_timing_select(msd_ctx *ctx, uint32_t kernel_mask) {
    if (!ctx) return fail(MSD_ERR_INVALID, "null ctx");
    ctx->timing_mask = kernel_mask;
    return MSD_OK;
}

static int fold_timing(msd_ctx *ctx) {
    if (ctx->pending.empty()) return MSD_OK;
    MSD_HIP(hipStreamSynchronize(ctx->stream));
    for (auto &p : ctx->pending) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            ctx->total_ms[p.kernel] += ms;
            ctx->launches[p.kernel] += 1;
        }
        ctx->pool.push_back(p.a);
        ctx->pool.push_back(p.b);
    }
    ctx->pending.clear();
    return MSD_OK;
}

int msd_timing_reset(msd_ctx *ctx) {
    if (!ctx) return fail(MSD_ERR_INVALID, "null ctx");
    DeviceGuard g(ctx->device);
    int rc = fold_timing(ctx);
    for (int i = 0; i < K_COUNT; ++i) {
        ctx->total_ms[i] = 0;
        ctx->launches[i] = 0;
    }
    return rc;
}

int msd_timing_get(msd_ctx *ctx, int kernel, double *total_ms, int64_t *launches) {
    if (!ctx || kernel < 0 || kernel >= K_COUNT) return fail(MSD_ERR_INVALID, "msd_timing_get: bad args");
    DeviceGuard g(ctx->device);
    int rc = fold_timing(ctx);
    if (rc) return rc;
    if (total_ms) *total_ms = ctx->total_ms[kernel];
    if (launches) *launches = ctx->launches[kernel];
    return MSD_OK;
}

// ------------------------------------------------------------------ STFT plan
}  // extern "C"
namespace {
bool pow2_in(int v, int lo, int hi) { return v >= lo && v <= hi && (v & (v - 1)) == 0; }

// shared by the float32 and float64 plan constructors: window (nperseg values) and the
// twiddles of an nfft-point real FFT, in the plan's precision
int stft_plan_make(msd_ctx *ctx, int32_t nperseg, int32_t nfft, int32_t hop, const float *w32, const double *w64,
                   double scale, int precision, msd_stft_plan **out) {
    *out = nullptr;
    if (nperseg < 1 || !pow2_in(nfft, 16, 16384) || nfft < nperseg)
        return fail(MSD_ERR_UNSUPPORTED, "stft: need 1 <= nperseg <= nfft, nfft a power of two in [16, 16384]");
    if (hop <= 0) return fail(MSD_ERR_INVALID, "stft: need hop = nperseg - noverlap > 0");
    if (precision != MSD_F32 && precision != MSD_F64) return fail(MSD_ERR_INVALID, "stft: precision must be F32 or F64");
    DeviceGuard g(ctx->device);
    auto *p = new msd_stft_plan();
    p->ctx = ctx;
    p->nperseg = nperseg;
    p->nfft = nfft;
    p->hop = hop;
    p->M = nfft / 2;
    p->precision = precision;
    p->scale = scale;
    const int M = p->M;
    std::vector<double2> tw(M), post(M + 1);
    for (int m = 0; m < M; ++m) {
        const double a = -2.0 * M_PI * (double)m / (double)M;
        tw[m] = make_double2(std::cos(a), std::sin(a));
    }
    for (int k = 0; k <= M; ++k) {
        const double a = -M_PI * (double)k / (double)M;
        post[k] = make_double2(std::cos(a), std::sin(a));
    }
    hipError_t e = hipSuccess;
    if (precision == MSD_F32) {
        std::vector<float2> tw32(M), post32(M + 1);
        for (int m = 0; m < M; ++m) tw32[m] = make_float2((float)tw[m].x, (float)tw[m].y);
        for (int k = 0; k <= M; ++k) post32[k] = make_float2((float)post[k].x, (float)post[k].y);
        std::vector<float> win(nperseg);
        for (int i = 0; i < nperseg; ++i) win[i] = w32 ? w32[i] : (float)w64[i];
        if (nperseg == nfft) {  // the window's DFT at bins 0 .. M (stft1024_kernel's mean residual)
            double wmax = 0.0;
            std::vector<long double> cs(nfft), sn(nfft);  // exp(-2 pi i j / N), the argument reduced exactly
            for (int j = 0; j < nfft; ++j) {
                const long double a = -2.0L * 3.141592653589793238462643383279502884L * j / nfft;
                cs[j] = cosl(a);
                sn[j] = sinl(a);
            }
            for (int k = 0; k <= M; ++k) {
                long double re = 0.0L, im = 0.0L;
                for (int i = 0, j = 0; i < nperseg; ++i, j = (j + k) & (nfft - 1)) {
                    re += (long double)win[i] * cs[j];
                    im += (long double)win[i] * sn[j];
                }
                if (k < 2) p->win_dft01[k] = make_double2((double)re, (double)im);
                else wmax = std::max(wmax, (double)std::sqrt(re * re + im * im));
            }
            const double w0 = std::hypot(p->win_dft01[0].x, p->win_dft01[0].y);
            p->win_dft_compact = w0 > 0.0 && wmax <= 1e-6 * w0;
        }
        e = hipMalloc(&p->d_window, sizeof(float) * nperseg);
        if (e == hipSuccess) e = hipMalloc(&p->d_tw, sizeof(float2) * M);
        if (e == hipSuccess) e = hipMalloc(&p->d_post, sizeof(float2) * (M + 1));
        if (e == hipSuccess) e = hipMemcpy(p->d_window, win.data(), sizeof(float) * nperseg, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(p->d_tw, tw32.data(), sizeof(float2) * M, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(p->d_post, post32.data(), sizeof(float2) * (M + 1), hipMemcpyHostToDevice);
    } else {
        std::vector<double> win(nperseg);
        for (int i = 0; i < nperseg; ++i) win[i] = w64 ? w64[i] : (double)w32[i];
        e = hipMalloc(&p->d_window64, sizeof(double) * nperseg);
        if (e == hipSuccess) e = hipMalloc(&p->d_tw64, sizeof(double2) * M);
        if (e == hipSuccess) e = hipMalloc(&p->d_post64, sizeof(double2) * (M + 1));
        if (e == hipSuccess) e = hipMemcpy(p->d_window64, win.data(), sizeof(double) * nperseg, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(p->d_tw64, tw.data(), sizeof(double2) * M, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(p->d_post64, post.data(), sizeof(double2) * (M + 1), hipMemcpyHostToDevice);
    }
    if (e != hipSuccess) {
        msd_stft_plan_destroy(p);
        return hip_fail(e, "stft plan upload");
    }
    *out = p;
    return MSD_OK;
}

// host-buffer convenience path shared by msd_stft_psd / msd_stft_psd_f64: out dense [K][T]
int stft_psd_host(msd_stft_plan *p, const void *x, int dtype, int64_t n, void *out, size_t out_es, int64_t *frames) {
    const size_t es = dtype_size(dtype);
    if (!es) return fail(MSD_ERR_INVALID, "msd_stft_psd: unknown dtype");
    const int64_t T = msd_stft_frames(p, n);
    if (frames) *frames = T;
    if (T == 0) return MSD_OK;
    msd_ctx *ctx = p->ctx;
    DeviceGuard g(ctx->device);
    const int64_t K = p->M + 1;
    const int64_t ld = (T + 31) / 32 * 32;
    const size_t xin = ((size_t)n * es + 255) / 256 * 256;
    void *dx, *dmeta, *dout;
    int rc;
    if ((rc = ctx_scratch(ctx, 0, xin, &dx))) return rc;
    if ((rc = ctx_scratch(ctx, 1, 64, &dmeta))) return rc;
    if ((rc = ctx_scratch(ctx, 2, out_es * K * ld, &dout))) return rc;
    int64_t meta[2] = {0, n};
    MSD_HIP(hipMemcpyAsync(dx, x, (size_t)n * es, hipMemcpyHostToDevice, ctx->stream));
    MSD_HIP(hipMemcpyAsync(dmeta, meta, sizeof(meta), hipMemcpyHostToDevice, ctx->stream));
    const int64_t *doff = static_cast<const int64_t *>(dmeta);
    rc = launch_stft(p, dx, dtype, doff, doff + 1, 1, T, dout, ld);
    if (rc) return rc;
    MSD_HIP(hipMemcpy2DAsync(out, out_es * T, dout, out_es * ld, out_es * T, K, hipMemcpyDeviceToHost, ctx->stream));
    MSD_HIP(hipStreamSynchronize(ctx->stream));
    return MSD_OK;
}
}  // namespace
extern "C" {

int msd_stft_plan_create(msd_ctx *ctx, int32_t nperseg, int32_t hop, const float *window, double scale,
                         msd_stft_plan **out) {
    if (!ctx || !window || !out) return fail(MSD_ERR_INVALID, "msd_stft_plan_create: null");
    *out = nullptr;
    if (!pow2_in(nperseg, 16, 16384))
        return fail(MSD_ERR_UNSUPPORTED, "stft: nperseg must be a power of two in [16, 16384] (nfft = nperseg)");
    if (hop <= 0 || hop > nperseg) return fail(MSD_ERR_INVALID, "stft: need 0 < hop <= nperseg (noverlap < nperseg)");
    return stft_plan_make(ctx, nperseg, nperseg, hop, window, nullptr, scale, MSD_F32, out);
}

int msd_stft_plan_create_ex(msd_ctx *ctx, int32_t nperseg, int32_t nfft, int32_t hop, const double *window,
                            double scale, int precision, msd_stft_plan **out) {
    if (!ctx || !window || !out) return fail(MSD_ERR_INVALID, "msd_stft_plan_create_ex: null");
    return stft_plan_make(ctx, nperseg, nfft, hop, nullptr, window, scale, precision, out);
}

void msd_stft_plan_destroy(msd_stft_plan *p) {
    if (!p) return;
    DeviceGuard g(p->ctx->device);
    hipStreamSynchronize(p->ctx->stream);
    hipFree(p->d_window);
    hipFree(p->d_tw);
    hipFree(p->d_post);
    hipFree(p->d_window64);
    hipFree(p->d_tw64);
    hipFree(p->d_post64);
    if (p->d_sched) hipFree(p->d_sched);
    if (p->d_ticket) hipFree(p->d_ticket);
    delete p;
}

int64_t msd_stft_frames(const msd_stft_plan *p, int64_t n) {
    if (!p || n < p->nperseg) return 0;
    return (n - p->nperseg) / p->hop + 1;
}

int32_t msd_stft_bins(const msd_stft_plan *p) { return p ? p->M + 1 : 0; }

int msd_stft_psd_dev(msd_stft_plan *p, const void *x, int dtype, const int64_t *off, const int64_t *len,
                     int64_t nfiles, int64_t max_frames, float *out, int64_t ld) {
    if (!p || (nfiles > 0 && (!x || !off || !len || !out))) return fail(MSD_ERR_INVALID, "msd_stft_psd_dev: null");
    if (p->precision != MSD_F32) return fail(MSD_ERR_INVALID, "msd_stft_psd_dev: float64 plan (use msd_stft_psd_f64_dev)");
    if (ld % 32 != 0 || ld < max_frames || ld <= 0) return fail(MSD_ERR_INVALID, "stft: ld must be >= max_frames, a positive multiple of 32");
    DeviceGuard g(p->ctx->device);
    return launch_stft(p, x, dtype, off, len, nfiles, max_frames, out, ld);
}

int msd_stft_psd_f64_dev(msd_stft_plan *p, const void *x, int dtype, const int64_t *off, const int64_t *len,
                         int64_t nfiles, int64_t max_frames, double *out, int64_t ld) {
    if (!p || (nfiles > 0 && (!x || !off || !len || !out))) return fail(MSD_ERR_INVALID, "msd_stft_psd_f64_dev: null");
    if (p->precision != MSD_F64) return fail(MSD_ERR_INVALID, "msd_stft_psd_f64_dev: float32 plan (use msd_stft_psd_dev)");
    if (ld % 32 != 0 || ld < max_frames || ld <= 0) return fail(MSD_ERR_INVALID, "stft: ld must be >= max_frames, a positive multiple of 32");
    DeviceGuard g(p->ctx->device);
    return launch_stft(p, x, dtype, off, len, nfiles, max_frames, out, ld);
}

int msd_stft_plan_set_detrend(msd_stft_plan *p, int detrend) {
    if (!p || (detrend != 0 && detrend != 1)) return fail(MSD_ERR_INVALID, "msd_stft_plan_set_detrend: bad args");
    p->detrend = detrend;
    return MSD_OK;
}

int msd_stft_psd(msd_stft_plan *p, const void *x, int dtype, int64_t n, float *out, int64_t *frames) {
    if (!p || !x || !out) return fail(MSD_ERR_INVALID, "msd_stft_psd: null");
    if (p->precision != MSD_F32) return fail(MSD_ERR_INVALID, "msd_stft_psd: float64 plan (use msd_stft_psd_f64)");
    return stft_psd_host(p, x, dtype, n, out, sizeof(float), frames);
}

int msd_stft_psd_f64(msd_stft_plan *p, const void *x, int dtype, int64_t n, double *out, int64_t *frames) {
    if (!p || !x || !out) return fail(MSD_ERR_INVALID, "msd_stft_psd_f64: null");
    if (p->precision != MSD_F64) return fail(MSD_ERR_INVALID, "msd_stft_psd_f64: float32 plan (use msd_stft_psd)");
    return stft_psd_host(p, x, dtype, n, out, sizeof(double), frames);
}

// ------------------------------------------------------------- block-delta plan
int msd_block_plan_create(msd_ctx *ctx, int64_t block_size, int32_t nfft, const double *window, int32_t band_lo,
                          int32_t band_hi, int32_t noise_lo, int32_t noise_hi, msd_block_plan **out) {
    if (!ctx || !out) return fail(MSD_ERR_INVALID, "msd_block_plan_create: null");
    *out = nullptr;
    if (block_size <= 0 || nfft <= 0) return fail(MSD_ERR_INVALID, "block plan: block_size and n_fft must be > 0");
    const int64_t L = block_size < nfft ? block_size : nfft;
    if (L > 4096) return fail(MSD_ERR_UNSUPPORTED, "block plan: min(block_size, n_fft) must be <= 4096");
    if (!window) return fail(MSD_ERR_INVALID, "block plan: null window");
    const int K = nfft / 2 + 1;
    auto clampband = [&](int32_t &lo, int32_t &hi) {
        if (hi < lo) {
            lo = 0;
            hi = -1;
            return true;
        }
        return lo >= 0 && hi < K;
    };
    if (!clampband(band_lo, band_hi) || !clampband(noise_lo, noise_hi))
        return fail(MSD_ERR_INVALID, "block plan: band bins outside [0, n_fft/2]");
    DeviceGuard g(ctx->device);
    auto *p = new msd_block_plan();
    p->ctx = ctx;
    p->block_size = block_size;
    p->nfft = nfft;
    p->L = (int)L;
    p->band_lo = band_lo;
    p->band_hi = band_hi;
    p->noise_lo = noise_lo;
    p->noise_hi = noise_hi;
    std::vector<int> bins;
    for (int k = band_lo; k <= band_hi; ++k) bins.push_back(k);
    for (int k = noise_lo; k <= noise_hi; ++k) bins.push_back(k);
    p->nbins = (int)bins.size();
    std::vector<double2> tw(nfft);
    for (int m = 0; m < nfft; ++m) {
        const double a = -2.0 * M_PI * (double)m / (double)nfft;
        tw[m] = make_double2(std::cos(a), std::sin(a));
    }
    // fast-path constants (block_delta.hip, block_delta2_kernel)
    const int spl = L <= 256 ? 16 : L <= 512 ? 32 : L <= 1024 ? 64 : L <= 2048 ? 128 : 256;
    p->spl = spl;
    std::vector<double> bconst;
    for (int k : bins) {
        const double th = 2.0 * M_PI * (double)(k % nfft) / (double)nfft;
        bconst.push_back(2.0 * std::cos(th));
        bconst.push_back(std::cos(th));
        bconst.push_back(-std::sin(th));
    }
    for (int k : bins) {
        for (int seg = 0; seg < 16; ++seg) {
            const int64_t m = ((int64_t)k * (seg * spl + spl - 1)) % nfft;
            const double a = -2.0 * M_PI * (double)m / (double)nfft;
            bconst.push_back(std::cos(a));
            bconst.push_back(std::sin(a));
        }
    }
    hipError_t e = hipMalloc(&p->d_window, sizeof(double) * L);
    if (e == hipSuccess) e = hipMalloc(&p->d_bconst, sizeof(double) * (bconst.size() + 1));
    if (e == hipSuccess && !bconst.empty())
        e = hipMemcpy(p->d_bconst, bconst.data(), sizeof(double) * bconst.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&p->d_tw, sizeof(double2) * nfft);
    if (e == hipSuccess) e = hipMalloc(&p->d_bins, sizeof(int) * (bins.size() + 1));
    if (e == hipSuccess) e = hipMemcpy(p->d_window, window, sizeof(double) * L, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(p->d_tw, tw.data(), sizeof(double2) * nfft, hipMemcpyHostToDevice);
    if (e == hipSuccess && !bins.empty())
        e = hipMemcpy(p->d_bins, bins.data(), sizeof(int) * bins.size(), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        msd_block_plan_destroy(p);
        return hip_fail(e, "block plan upload");
    }
    if (block_i8_shape(L, p->nbins) && block_i8_window(window, L)) {  // int16 blocks on the matrix cores (block_i8.hip)
        if (int rc = block_i8_build(p, window, bins.data(), p->nbins)) {
            msd_block_plan_destroy(p);
            return rc;
        }
    }
    *out = p;
    return MSD_OK;
}

void msd_block_plan_destroy(msd_block_plan *p) {
    if (!p) return;
    DeviceGuard g(p->ctx->device);
    hipStreamSynchronize(p->ctx->stream);
    hipFree(p->d_window);
    hipFree(p->d_tw);
    hipFree(p->d_bins);
    hipFree(p->d_bconst);
    hipFree(p->d_energy);
    hipFree(p->d_i8);
    delete p;
}

int msd_block_delta_dev(msd_block_plan *p, const void *x, int dtype, const int64_t *off, const int64_t *len,
                        int64_t nfiles, int64_t max_blocks, double *band_db, double *noise_db, double *delta,
                        int64_t ld) {
    if (!p || (nfiles > 0 && (!x || !off || !len || !delta))) return fail(MSD_ERR_INVALID, "msd_block_delta_dev: null");
    if (ld < max_blocks) return fail(MSD_ERR_INVALID, "block_delta: ld < max_blocks");
    DeviceGuard g(p->ctx->device);
    return launch_block_delta(p, x, dtype, off, len, nfiles, max_blocks, band_db, noise_db, delta, ld);
}

int msd_block_delta(msd_block_plan *p, const void *x, int dtype, int64_t n, double *band_db, double *noise_db,
                    double *delta, int64_t *blocks) {
    if (!p || (!x && n) || !delta) return fail(MSD_ERR_INVALID, "msd_block_delta: null");
    const size_t es = dtype_size(dtype);
    if (!es) return fail(MSD_ERR_INVALID, "msd_block_delta: unknown dtype");
    const int64_t nb = n / p->block_size;
    if (blocks) *blocks = nb;
    if (nb == 0) return MSD_OK;
    msd_ctx *ctx = p->ctx;
    DeviceGuard g(ctx->device);
    void *dx, *dmeta, *dout;
    int rc;
    if ((rc = ctx_scratch(ctx, 0, ((size_t)n * es + 255) / 256 * 256, &dx))) return rc;
    if ((rc = ctx_scratch(ctx, 1, 64, &dmeta))) return rc;
    if ((rc = ctx_scratch(ctx, 2, sizeof(double) * 3 * nb, &dout))) return rc;
    int64_t meta[2] = {0, n};
    MSD_HIP(hipMemcpyAsync(dx, x, (size_t)n * es, hipMemcpyHostToDevice, ctx->stream));
    MSD_HIP(hipMemcpyAsync(dmeta, meta, sizeof(meta), hipMemcpyHostToDevice, ctx->stream));
    double *d = static_cast<double *>(dout);
    const int64_t *doff = static_cast<const int64_t *>(dmeta);
    rc = launch_block_delta(p, dx, dtype, doff, doff + 1, 1, nb, d, d + nb, d + 2 * nb, nb);
    if (rc) return rc;
    if (band_db) MSD_HIP(hipMemcpyAsync(band_db, d, sizeof(double) * nb, hipMemcpyDeviceToHost, ctx->stream));
    if (noise_db) MSD_HIP(hipMemcpyAsync(noise_db, d + nb, sizeof(double) * nb, hipMemcpyDeviceToHost, ctx->stream));
    MSD_HIP(hipMemcpyAsync(delta, d + 2 * nb, sizeof(double) * nb, hipMemcpyDeviceToHost, ctx->stream));
    MSD_HIP(hipStreamSynchronize(ctx->stream));
    return MSD_OK;
}

// ------------------------------------------------------------------- detector
static int check_det_cfg(const msd_det_cfg *cfg) {
    if (!cfg) return fail(MSD_ERR_INVALID, "detect: null cfg");
    if (cfg->adaptive != 0 && cfg->adaptive != 1) return fail(MSD_ERR_INVALID, "detect: adaptive must be 0 or 1");
    return MSD_OK;
}

int msd_detect_dev(msd_ctx *ctx, const double *delta, const int64_t *nblocks, int64_t nfiles, int64_t ld,
                   const msd_det_cfg *cfg, msd_det *dets, int64_t cap, int64_t *counts, double *thresholds,
                   double *margin, int32_t *status, const msd_hist_cfg *hist) {
    if (!ctx || (nfiles > 0 && (!delta || !nblocks || !dets || !counts)))
        return fail(MSD_ERR_INVALID, "msd_detect_dev: null");
    int rc = check_det_cfg(cfg);
    if (rc) return rc;
    DeviceGuard g(ctx->device);
    return launch_detect(ctx, delta, nblocks, nfiles, ld, cfg, dets, cap, counts, thresholds, margin, status, hist);
}

int msd_detect(msd_ctx *ctx, const double *delta, int64_t nb, const msd_det_cfg *cfg, msd_det *dets, int64_t cap,
               int64_t *count, double *thresholds, double *margin) {
    if (!ctx || (!delta && nb) || (!dets && cap) || !count) return fail(MSD_ERR_INVALID, "msd_detect: null");
    int rc = check_det_cfg(cfg);
    if (rc) return rc;
    DeviceGuard g(ctx->device);
    const int64_t ld = nb > 0 ? nb : 1;
    const int64_t dcap = cap > 0 ? cap : 1;
    // scratch layout: delta[ld] | thr[ld] | nb | count | margin | status | dets[dcap]
    const size_t bytes = sizeof(double) * 2 * ld + 32 + sizeof(msd_det) * dcap;
    void *s;
    if ((rc = ctx_scratch(ctx, 3, bytes, &s))) return rc;
    char *base = static_cast<char *>(s);
    double *dd = reinterpret_cast<double *>(base);
    double *dthr = dd + ld;
    int64_t *dnb = reinterpret_cast<int64_t *>(dthr + ld);
    int64_t *dcount = dnb + 1;
    double *dmargin = reinterpret_cast<double *>(dcount + 1);
    int32_t *dstatus = reinterpret_cast<int32_t *>(dmargin + 1);
    msd_det *ddets = reinterpret_cast<msd_det *>(base + sizeof(double) * 2 * ld + 32);
    if (nb) MSD_HIP(hipMemcpyAsync(dd, delta, sizeof(double) * nb, hipMemcpyHostToDevice, ctx->stream));
    MSD_HIP(hipMemcpyAsync(dnb, &nb, sizeof(int64_t), hipMemcpyHostToDevice, ctx->stream));
    rc = launch_detect(ctx, dd, dnb, 1, ld, cfg, ddets, dcap, dcount, dthr, dmargin, dstatus, nullptr);
    if (rc) return rc;
    int64_t cnt = 0;
    int32_t st = 0;
    double mg = 0;
    MSD_HIP(hipMemcpyAsync(&cnt, dcount, sizeof(cnt), hipMemcpyDeviceToHost, ctx->stream));
    MSD_HIP(hipMemcpyAsync(&st, dstatus, sizeof(st), hipMemcpyDeviceToHost, ctx->stream));
    MSD_HIP(hipMemcpyAsync(&mg, dmargin, sizeof(mg), hipMemcpyDeviceToHost, ctx->stream));
    MSD_HIP(hipStreamSynchronize(ctx->stream));
    *count = cnt;
    if (margin) *margin = mg;
    const int64_t ncopy = cnt < cap ? cnt : cap;
    if (ncopy > 0) MSD_HIP(hipMemcpyAsync(dets, ddets, sizeof(msd_det) * ncopy, hipMemcpyDeviceToHost, ctx->stream));
    if (thresholds) {
        const int64_t nt = cfg->adaptive ? nb : 1;
        if (nt > 0) MSD_HIP(hipMemcpyAsync(thresholds, dthr, sizeof(double) * nt, hipMemcpyDeviceToHost, ctx->stream));
    }
    MSD_HIP(hipStreamSynchronize(ctx->stream));
    if (st == 2) return fail(MSD_ERR_INDEX, "index 0 is out of bounds for axis 0 with size 0");
    if (st == 1) return fail(MSD_ERR_ASSERT, "Detection duration must be greater than 0");
    if (cnt > cap) return fail(MSD_ERR_CAPACITY, "detect: more detections than capacity");
    return MSD_OK;
}

// ----------------------------------------------------------------------- RCCL
int msd_comm_get_unique_id(char *id) {
    if (!id) return fail(MSD_ERR_INVALID, "msd_comm_get_unique_id: null");
    Rccl *r = rccl();
    if (!r) return fail(MSD_ERR_RCCL, "librccl.so.1 not loadable");
    ncclUniqueId u;
    ncclResult_t e = r->getUniqueId(&u);
    if (e != ncclSuccess) return rccl_fail(r, e, "ncclGetUniqueId");
    std::memcpy(id, u.internal, MSD_COMM_ID_BYTES);
    return MSD_OK;
}

int msd_comm_init(msd_ctx *ctx, int nranks, const char *id, int rank, msd_comm **out) {
    if (!ctx || !id || !out || nranks <= 0 || rank < 0 || rank >= nranks)
        return fail(MSD_ERR_INVALID, "msd_comm_init: bad args");
    *out = nullptr;
    Rccl *r = rccl();
    if (!r) return fail(MSD_ERR_RCCL, "librccl.so.1 not loadable");
    DeviceGuard g(ctx->device);
    hipSetDevice(ctx->device);
    ncclUniqueId u;
    std::memcpy(u.internal, id, MSD_COMM_ID_BYTES);
    auto *c = new msd_comm();
    c->ctx = ctx;
    ncclResult_t e = r->commInitRank(&c->comm, nranks, u, rank);
    if (e != ncclSuccess) {
        delete c;
        return rccl_fail(r, e, "ncclCommInitRank");
    }
    *out = c;
    return MSD_OK;
}

void msd_comm_destroy(msd_comm *c) {
    if (!c) return;
    Rccl *r = rccl();
    if (r && c->comm) {
        DeviceGuard g(c->ctx->device);
        r->commDestroy(c->comm);
    }
    delete c;
}

int msd_comm_allreduce_i64(msd_comm *c, int64_t *dbuf, int64_t n) {
    if (!c || (!dbuf && n)) return fail(MSD_ERR_INVALID, "msd_comm_allreduce_i64: null");
    if (n == 0) return MSD_OK;
    Rccl *r = rccl();
    if (!r) return fail(MSD_ERR_RCCL, "librccl.so.1 not loadable");
    DeviceGuard g(c->ctx->device);
    ncclResult_t e = r->allReduce(dbuf, dbuf, (size_t)n, ncclInt64, ncclSum, c->comm, c->ctx->stream);
    if (e != ncclSuccess) return rccl_fail(r, e, "ncclAllReduce");
    return MSD_OK;
}

int msd_comm_allgather(msd_comm *c, const void *dsend, void *drecv, size_t bytes) {
    if (!c || ((!dsend || !drecv) && bytes)) return fail(MSD_ERR_INVALID, "msd_comm_allgather: null");
    if (bytes == 0) return MSD_OK;
    Rccl *r = rccl();
    if (!r) return fail(MSD_ERR_RCCL, "librccl.so.1 not loadable");
    DeviceGuard g(c->ctx->device);
    ncclResult_t e = r->allGather(dsend, drecv, bytes, ncclChar, c->comm, c->ctx->stream);
    if (e != ncclSuccess) return rccl_fail(r, e, "ncclAllGather");
    return MSD_OK;
}

}  // extern "C"
