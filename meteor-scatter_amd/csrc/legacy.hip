// Legacy spectrogram noise floor (meteor_detect_class/prime_detection.py:65-91):
//   band_power = np.sum(Pxx[noise_band])   — over the band's bins and all frames
// One workgroup per spectrogram; each thread accumulates float64 over rows lo..hi of the
// float32 [K][ld] layout (coalesced along frames), then a wave DPP / LDS reduction.
#include "msd_internal.h"

namespace msd {
namespace {

constexpr int BS_THREADS = 256;

template <typename S>
__global__ __launch_bounds__(BS_THREADS) void spec_band_sum_kernel(const S *__restrict__ spec, int32_t K,
                                                                   int64_t frames, int64_t ld, int32_t lo, int32_t hi,
                                                                   double *__restrict__ out) {
    const int64_t f = blockIdx.x;
    const S *s = spec + f * (int64_t)K * ld;
    double acc = 0.0;
    for (int k = lo; k <= hi; ++k)
        for (int64_t t = threadIdx.x; t < frames; t += BS_THREADS) acc += (double)s[(int64_t)k * ld + t];
    __shared__ double part[BS_THREADS];
    part[threadIdx.x] = acc;
    __syncthreads();
    for (int w = BS_THREADS / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[f] = part[0];
}

}  // namespace
}  // namespace msd

using namespace msd;

namespace {
template <typename S>
int band_sum(msd_ctx *ctx, const S *spec, int64_t nfiles, int32_t K, int64_t frames, int64_t ld, int32_t lo,
             int32_t hi, double *out) {
    if (!ctx || (nfiles > 0 && (!spec || !out))) return fail(MSD_ERR_INVALID, "msd_spec_band_sum_dev: null");
    if (K <= 0 || frames < 0 || ld < frames || lo < 0 || hi >= K)
        return fail(MSD_ERR_INVALID, "msd_spec_band_sum_dev: need 0 <= lo, hi < K, frames <= ld");
    if (nfiles == 0) return MSD_OK;
    if (nfiles > 0x7fffffffLL) return fail(MSD_ERR_UNSUPPORTED, "msd_spec_band_sum_dev: too many spectrograms");
    DeviceGuard g(ctx->device);
    hipLaunchKernelGGL(spec_band_sum_kernel<S>, dim3((unsigned)nfiles), dim3(BS_THREADS), 0, ctx->stream, spec, K,
                       frames, ld, lo, hi, out);
    MSD_HIP(hipGetLastError());
    return MSD_OK;
}
}  // namespace

extern "C" int msd_spec_band_sum_dev(msd_ctx *ctx, const float *spec, int64_t nfiles, int32_t K, int64_t frames,
                                     int64_t ld, int32_t lo, int32_t hi, double *out) {
    return band_sum(ctx, spec, nfiles, K, frames, ld, lo, hi, out);
}

extern "C" int msd_spec_band_sum_f64_dev(msd_ctx *ctx, const double *spec, int64_t nfiles, int32_t K, int64_t frames,
                                         int64_t ld, int32_t lo, int32_t hi, double *out) {
    return band_sum(ctx, spec, nfiles, K, frames, ld, lo, hi, out);
}
