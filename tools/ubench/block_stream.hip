// Read-bandwidth ceiling of block_band_i8_kernel's sample stream: C3's 1440 files of
// 300 blocks of 9600 int16 samples, of which each block's first 1024 (2 KB) are read -- 0.885 GB
// out of 8.3 GB, 2 KB every 19.2 KB.  Tiles of 16 consecutive blocks, tiles interleaved over the
// waves, WPC waves per CU, the next tile requested while the current one is consumed (one xor per
// dword instead of the arithmetic).
//   PAT 0: the kernel's lane pattern: lane l reads row (l & 15), 16 B at 128 ks + 16 (l >> 4) (+ 64)
//          -- each instruction 16 rows x 64 B;
//   PAT 1: each instruction 1 KB contiguous of one row (lane l at 16 l), rows in turn.
// Build: hipcc --offload-arch=gfx950 -O3 block_stream.hip -o block_stream;  run: ./block_stream
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned v4u __attribute__((ext_vector_type(4)));

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(3);                                                                  \
        }                                                                                  \
    } while (0)

constexpr int64_t B = 9600;   // samples per block
constexpr int KS = 16;        // 64-sample K steps per block row (1024 samples)

template <int PAT, int WPC>
__global__ __launch_bounds__(64 * WPC) void k_stream(const short *__restrict__ x, int64_t nblocks, unsigned *out) {
    const int l = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * WPC + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * WPC;
    const int64_t ntiles = nblocks / 16;
    auto addr = [&](int64_t tile, int i) -> const v4u * {  // i-th of the 32 loads of a tile
        if (PAT == 0) {
            const int ks = i >> 1, h = i & 1;
            const short *row = x + (tile * 16 + (l & 15)) * B;
            return reinterpret_cast<const v4u *>(row + 64 * ks + 32 * h + 8 * (l >> 4));
        }
        const int r = i >> 1, h = i & 1;  // row r, its h-th KB
        const short *row = x + (tile * 16 + r) * B;
        return reinterpret_cast<const v4u *>(row + 512 * h) + l;
    };
    if (wave >= ntiles) return;
    v4u R[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) R[i] = *addr(wave, i);
    unsigned acc = 0;
    for (int64_t t = wave; t < ntiles; t += nwaves) {
        const int64_t nt = t + nwaves < ntiles ? t + nwaves : t;
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            acc ^= R[i].x ^ R[i].y ^ R[i].z ^ R[i].w;
            R[i] = *addr(nt, i);
        }
    }
    out[wave * 64 + l] = acc;
}

template <int PAT, int WPC>
double run(const short *x, int64_t nblocks, unsigned *out, int cus) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int grid = cus;  // one workgroup of WPC waves per CU
    float best = 1e30f;
    for (int rep = 0; rep < 6; ++rep) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((k_stream<PAT, WPC>), dim3(grid), dim3(64 * WPC), 0, 0, x, nblocks, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        if (rep > 0 && ms < best) best = ms;
    }
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return best;
}

int main() {
    const int64_t nblocks = 1440LL * 300;  // 432 000 blocks
    const size_t bytes = (size_t)nblocks * B * sizeof(short);
    short *x = nullptr;
    unsigned *out = nullptr;
    CK(hipMalloc(&x, bytes));
    CK(hipMemset(x, 1, bytes));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    CK(hipMalloc(&out, sizeof(unsigned) * 64 * 16 * cus));
    const double useful = (double)nblocks * 2048.0;
    auto line = [&](const char *name, double ms) {
        std::printf("%-44s %8.4f ms  %7.1f GB/s of the 2 KB per block\n", name, ms, useful / (ms * 1e-3) / 1e9);
    };
    line("kernel lane pattern, 4 waves/CU", run<0, 4>(x, nblocks, out, cus));
    line("kernel lane pattern, 8 waves/CU", run<0, 8>(x, nblocks, out, cus));
    line("1 KB contiguous per instruction, 4 waves/CU", run<1, 4>(x, nblocks, out, cus));
    line("1 KB contiguous per instruction, 8 waves/CU", run<1, 8>(x, nblocks, out, cus));
    CK(hipFree(x));
    CK(hipFree(out));
    return 0;
}
