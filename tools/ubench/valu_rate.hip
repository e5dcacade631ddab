// Micro-benchmark: VALU issue rate per SIMD on gfx950 as a function of waves per SIMD and of
// the independent chains (ILP) in each wave's stream.  Each wave runs ITER x UNROLL x ILP
// v_fma_f32 (or v_add_f32) in ILP independent dependency chains; one workgroup per CU of
// 4 x W waves (W waves per SIMD).  Cycles come from s_memtime (shader clock) around the loop,
// so the result is in cycles per wave-instruction per SIMD, independent of DVFS.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <map>
#include <algorithm>

// OP: 0 v_fma_f32 (VOP3, 8 B: v = v*a + a), 1 v_add_f32_e32 (VOP2, 4 B), 2 v_fmac_f32_e32 (VOP2:
// v += a*b), 3 v_mul_f32_e32, 4 v_fma_f32 with three distinct sources (v = v*a + b),
// 5 v_sub_f32_e64 (VOP3 encoding of an add), 6 v_pk_add_f32 (two lanes' worth per op)
template <int ILP, int OP>
__global__ void valu(float *out, long long *cyc, int iters, float a) {
    const float b = a * 0.5f;
    float v[ILP];
#pragma unroll
    for (int i = 0; i < ILP; ++i) v[i] = threadIdx.x * 1e-3f + i;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 32; ++u)
#pragma unroll
            for (int i = 0; i < ILP; ++i) {
                if constexpr (OP == 0) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(v[i]) : "v"(a));
                else if constexpr (OP == 1) asm volatile("v_add_f32_e32 %0, %1, %0" : "+v"(v[i]) : "v"(a));
                else if constexpr (OP == 2) asm volatile("v_fmac_f32_e32 %0, %1, %2" : "+v"(v[i]) : "v"(a), "v"(b));
                else if constexpr (OP == 3) asm volatile("v_mul_f32_e32 %0, %1, %0" : "+v"(v[i]) : "v"(a));
                else if constexpr (OP == 4) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(a), "v"(b));
                else if constexpr (OP == 5) asm volatile("v_sub_f32_e64 %0, %0, %1" : "+v"(v[i]) : "v"(a));
                else if constexpr (OP == 6) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(*reinterpret_cast<double *>(&v[i & ~1])) : "v"(*reinterpret_cast<const double *>(&v[0])));
                else if constexpr (OP == 7) asm volatile("v_mul_f32_e32 %0, %0, %0" : "+v"(v[i]));
                else if constexpr (OP == 8) asm volatile("v_fmac_f32_e32 %0, %1, %1" : "+v"(v[i]) : "v"(a));
                else if constexpr (OP == 9) asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(v[i]));
                else if constexpr (OP == 10) asm volatile("v_cvt_f32_i32_sdwa %0, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1" : "+v"(v[i]));
                else if constexpr (OP == 11) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(v[i]) : "v"(a));
                else if constexpr (OP == 12) asm volatile("v_add_f32_dpp %0, %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(v[i]) : "v"(a));
                else if constexpr (OP == 13) asm volatile("v_fma_f32 %0, %1, %1, %0" : "+v"(v[i]) : "v"(a));
                else if constexpr (OP == 14) asm volatile("v_dot2c_i32_i16_e32 %0, %1, %1" : "+v"(v[i]) : "v"(a));
            }
    }
    __syncthreads();
    const long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
#pragma unroll
    for (int i = 0; i < ILP; ++i) s += v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) {
        // per-workgroup start / end and the CU it ran on (HW_ID: CU bits 8-11, SH 12, SE 13-15; XCC_ID)
        const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
        const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11));
        cyc[3 * blockIdx.x] = t0;
        cyc[3 * blockIdx.x + 1] = t1;
        cyc[3 * blockIdx.x + 2] = ((long long)xcc << 32) | ((hw >> 8) & 0xff);
    }
}

template <int ILP, int OP>
void run2(int wgs_per_cu, int waves_per_wg, float *out, long long *cyc, int cus) {
    const int iters = 200;
    const int threads = waves_per_wg * 64;
    const int grid = cus * wgs_per_cu;
    static long long h[3 * 8192];
    double best = 1e30;
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL((valu<ILP, OP>), dim3(grid), dim3(threads), 0, 0, out, cyc, iters, 0.999f);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(h, cyc, sizeof(long long) * 3 * grid, hipMemcpyDeviceToHost);
        // span per CU = last end - first start over the workgroups that ran on it
        std::map<long long, std::pair<long long, long long>> span;
        for (int i = 0; i < grid; ++i) {
            auto it = span.find(h[3 * i + 2]);
            if (it == span.end()) span[h[3 * i + 2]] = {h[3 * i], h[3 * i + 1]};
            else it->second = {std::min(it->second.first, h[3 * i]), std::max(it->second.second, h[3 * i + 1])};
        }
        double m = 0;
        for (auto &kv : span) m += kv.second.second - kv.second.first;
        m /= span.size();
        if (m < best) best = m;
        if (rep == 0 && (int)span.size() != cus) printf("  (%zu distinct CUs seen)\n", span.size());
    }
    const int wps = wgs_per_cu * waves_per_wg / 4;
    const double instr_per_simd = (double)iters * 32 * ILP * wps;
    printf("op %d ILP %d  %d WG/CU x %2d waves (%d waves/SIMD)  %.2f cycles per wave-instruction per SIMD\n", OP, ILP,
           wgs_per_cu, waves_per_wg, wps, best / instr_per_simd);
}

int main() {
    float *out;
    long long *cyc;
    int cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipMalloc(&out, sizeof(float) * cus * 8192);
    hipMalloc(&cyc, sizeof(long long) * cus * 8 * 3);
    const int cfg[][2] = {{1, 16}};
    for (auto &c : cfg) {
        run2<8, 1>(c[0], c[1], out, cyc, cus);
        run2<8, 3>(c[0], c[1], out, cyc, cus);
        run2<8, 4>(c[0], c[1], out, cyc, cus);
        run2<8, 7>(c[0], c[1], out, cyc, cus);
        run2<8, 8>(c[0], c[1], out, cyc, cus);
        run2<8, 9>(c[0], c[1], out, cyc, cus);
        run2<8, 10>(c[0], c[1], out, cyc, cus);
        run2<8, 11>(c[0], c[1], out, cyc, cus);
        run2<8, 12>(c[0], c[1], out, cyc, cus);
        run2<8, 13>(c[0], c[1], out, cyc, cus);
        run2<8, 14>(c[0], c[1], out, cyc, cus);
        run2<4, 1>(c[0], c[1], out, cyc, cus);
        run2<2, 1>(c[0], c[1], out, cyc, cus);
        run2<1, 1>(c[0], c[1], out, cyc, cus);
    }
    // waves per SIMD: fma / add / pk_add at 1, 2, 4, 8
    const int cfg2[][2] = {{1, 4}, {1, 8}, {1, 16}, {2, 16}};
    for (auto &c : cfg2) {
        run2<8, 0>(c[0], c[1], out, cyc, cus);
        run2<8, 1>(c[0], c[1], out, cyc, cus);
        run2<8, 6>(c[0], c[1], out, cyc, cus);
    }
    hipFree(out);
    hipFree(cyc);
    return 0;
}
