// Minimal reproducer of the round-5 GPU fault.  NOT to be run on a GPU: wave 0's
// load below leaves the LDS aperture and raises HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION.
//
// An out-of-line function sums a generic pointer with numpy's 8-accumulator leaf loop, unrolled by 2.
// The kernel passes it an LDS array at LDS offset 0.  The compiler (ROCm 7.2 clang, gfx950, -O3)
// strength-reduces the loop pointer to `p - 64` and folds +128 .. +240 into the flat loads'
// instruction offsets.  A flat instruction picks its aperture (LDS, scratch or global) from the high
// bits of the address register alone, before the offset is added, so `shared_base - 64` is taken as a
// global address just below the LDS aperture, outside the legal range.
//
// Compile only:  hipcc --offload-arch=gfx950 -O3 -std=c++17 --offload-device-only -S \
//                    tools/repro/flat_lds_offset.hip -o /tmp/flat_lds_offset.s
// and look for `v_lshl_add_u64 v[..], v[..], 0, s[..]` with s = 0xffffffffffffffc0 (-64) feeding
// `flat_load_dwordx4 ... offset:128`.  tools/repro/check_flat_lds_offset.py does this.
#include <hip/hip_runtime.h>
#include <cstdint>

__device__ __forceinline__ double leaf_sum(const double *p, int64_t base, int64_t n) {
    const double *a = p + base;
    double r0 = a[0], r1 = a[1], r2 = a[2], r3 = a[3], r4 = a[4], r5 = a[5], r6 = a[6], r7 = a[7];
    int64_t i = 8;
    const int64_t lim = n - (n % 8);
#pragma unroll 2
    for (; i < lim; i += 8) {
        r0 += a[i + 0];
        r1 += a[i + 1];
        r2 += a[i + 2];
        r3 += a[i + 3];
        r4 += a[i + 4];
        r5 += a[i + 5];
        r6 += a[i + 6];
        r7 += a[i + 7];
    }
    double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
    for (; i < n; ++i) res += a[i];
    return res;
}

// numpy's one split (128 < n <= 256): two leaves, the left one n/2 rounded down to 8 (>= 64, so the
// compiler drops the unrolled loop's trip-count guard there -- the form that displaced the pointer)
__device__ __noinline__ double pair_sum(const double *p, int64_t base, int64_t n) {
    if (n <= 128) return leaf_sum(p, base, n);
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    return leaf_sum(p, base, n2) + leaf_sum(p, base + n2, n - n2);
}

// the callee sees LDS or global memory (as np_sum did: staged segments and band sums), so the pointer
// stays generic
__global__ void repro_kernel(const double *__restrict__ in, int n, int staged, double *__restrict__ out) {
    __shared__ double seg[1024];  // the only LDS object: LDS offset 0
    for (int i = threadIdx.x; i < n; i += blockDim.x) seg[i] = in[i];
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = pair_sum(staged ? seg : in, 0, n);
}
