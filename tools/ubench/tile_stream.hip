// Read-bandwidth ceiling of block_i8_kernel's sample stream: 8.3 GB of int16 I/Q
// read in 16 KB tiles, each lane loading 2 x 16 B per K step from row (l & 15) at byte
// 128 ks + 16 (l >> 4) (+ 64), tiles interleaved over the waves -- the int8 delta kernel's access
// pattern with its arithmetic replaced by one xor per dword -- for DEPTH tiles in flight per wave
// (raw registers: 64 VGPRs per tile) and WPC waves per CU.  Also a plain contiguous read (each
// instruction 1 KB) at the same depth for comparison.
// Build: hipcc --offload-arch=gfx950 -O3 tile_stream.hip -o tile_stream
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned v4u __attribute__((ext_vector_type(4)));

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(3);                                                                  \
        }                                                                                  \
    } while (0)

constexpr int KS = 8;  // K steps per tile, 2 loads each: 16 x 16 B per lane = 16 KB per wave

// PAT 0: the kernel's pattern (row l & 15 of 1 KB rows, 64 B per row per instruction);
// PAT 1: contiguous 1 KB per instruction
// WORK: the int8 kernel's digit extraction per K step (8 v_perm, 4 xor, 4 v_sad_u8) instead of
// the xor; ST: one 1 KB store per tile (the kernel's staged output)
template <int DEPTH, int PAT, int WORK = 0, int ST = 0>
__global__ __launch_bounds__(256) void k_stream(const v4u *__restrict__ x, int64_t ntiles, unsigned *out) {
    const int l = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * 4;
    auto addr = [&](int64_t tile, int ks, int h) -> const v4u * {
        const v4u *t = x + tile * 1024;  // 16 KB tile = 1024 v4u
        if (PAT == 0) return t + (l & 15) * 64 + 8 * ks + 4 * h + (l >> 4);
        return t + (2 * ks + h) * 64 + l;
    };
    v4u raw[DEPTH][2 * KS];
    unsigned acc = 0;
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
        const int64_t t = wave + d * nwaves < ntiles ? wave + d * nwaves : wave;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            raw[d][2 * ks] = *addr(t, ks, 0);
            raw[d][2 * ks + 1] = *addr(t, ks, 1);
        }
    }
    for (int64_t tile = wave; tile < ntiles; tile += DEPTH * nwaves) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            const int64_t tn0 = tile + (d + DEPTH) * nwaves;
            const int64_t tn = tn0 < ntiles ? tn0 : wave;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const v4u a = raw[d][2 * ks], b = raw[d][2 * ks + 1];
                if (WORK) {
                    const unsigned w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
                    for (int o = 0; o < 4; ++o) {
                        const unsigned h = __builtin_amdgcn_perm(w[2 * o + 1], w[2 * o], 0x07050301u);
                        const unsigned lo = __builtin_amdgcn_perm(w[2 * o + 1], w[2 * o], 0x06040200u) ^ 0x80808080u;
                        acc = __builtin_amdgcn_sad_u8(h ^ 0x80808080u, 0x80808080u, acc) ^ lo;
                    }
                } else {
                    acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w;
                }
                raw[d][2 * ks] = *addr(tn, ks, 0);
                raw[d][2 * ks + 1] = *addr(tn, ks, 1);
            }
            // ST 1: 256 B per tile; ST 2: 1 KB (b128 per lane) every 4th tile; ST 3: 256 B per tile
            // but issued as 4 instructions every 4th tile
            if (ST == 1) out[(tile + d * nwaves) % (64 * 1024) * 64 + l] = acc;
            if (ST == 2 && ((tile / nwaves) & 3) == 3) {
                v4u q = {acc, acc + 1, acc + 2, acc + 3};
                reinterpret_cast<v4u *>(out)[(tile + d * nwaves) % (16 * 1024) * 64 + l] = q;
            }
            if (ST == 3 && ((tile / nwaves) & 3) == 3) {
#pragma unroll
                for (int k = 0; k < 4; ++k) out[((tile + d * nwaves) * 4 + k) % (64 * 1024) * 64 + l] = acc + k;
            }
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int DEPTH, int PAT, int WORK = 0, int ST = 0>
float run(const v4u *dx, int64_t ntiles, unsigned *dout, int wpc, int cus) {
    const int grid = cus * wpc / 4;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    hipLaunchKernelGGL((k_stream<DEPTH, PAT, WORK, ST>), dim3(grid), dim3(256), 0, 0, dx, ntiles, dout);
    CK(hipDeviceSynchronize());
    std::vector<float> ms;
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((k_stream<DEPTH, PAT, WORK, ST>), dim3(grid), dim3(256), 0, 0, dx, ntiles, dout);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float t;
        CK(hipEventElapsedTime(&t, a, b));
        ms.push_back(t);
    }
    float best = ms[0];
    for (float t : ms) best = t < best ? t : best;
    return best;
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int64_t bytes = 8294400000LL;  // 3 h of 192 kHz int16 I/Q
    const int64_t ntiles = bytes / 16384;
    v4u *dx;
    unsigned *dout;
    CK(hipMalloc(&dx, ntiles * 16384));
    CK(hipMemset(dx, 1, ntiles * 16384));
    CK(hipMalloc(&dout, sizeof(unsigned) * 64 * 1024 * 64));
    const double gb = ntiles * 16384.0 * 1e-9;
    auto rep = [&](const char *name, int wpc, float ms) {
        std::printf("%-34s waves/CU %2d  %.3f ms  %.2f TB/s\n", name, wpc, ms, gb / ms);
    };
    rep("kernel pattern + digit work", 8, run<1, 0, 1, 0>(dx, ntiles, dout, 8, cus));
    rep("kernel pattern + 1 KB store per tile", 8, run<1, 0, 0, 1>(dx, ntiles, dout, 8, cus));
    rep("kernel pattern + digits + store", 8, run<1, 0, 1, 1>(dx, ntiles, dout, 8, cus));
    rep("kernel pattern + 1 KB store per 4 tiles", 8, run<1, 0, 1, 2>(dx, ntiles, dout, 8, cus));
    rep("kernel pattern + 4 stores per 4 tiles", 8, run<1, 0, 1, 3>(dx, ntiles, dout, 8, cus));
    rep("kernel pattern + store, 2 in flight", 8, run<2, 0, 1, 1>(dx, ntiles, dout, 8, cus));
    for (int wpc : {8, 12, 16}) {
        rep("kernel pattern, 1 tile in flight", wpc, run<1, 0>(dx, ntiles, dout, wpc, cus));
        rep("kernel pattern, 2 tiles in flight", wpc, run<2, 0>(dx, ntiles, dout, wpc, cus));
        rep("contiguous, 1 tile in flight", wpc, run<1, 1>(dx, ntiles, dout, wpc, cus));
        rep("contiguous, 2 tiles in flight", wpc, run<2, 1>(dx, ntiles, dout, wpc, cus));
    }
    rep("kernel pattern, 3 tiles in flight", 8, run<3, 0>(dx, ntiles, dout, 8, cus));
    rep("kernel pattern, 4 tiles in flight", 4, run<4, 0>(dx, ntiles, dout, 4, cus));
    return 0;
}
