// Micro-benchmark: VALU issue cost on gfx950 by operand placement and encoding.  Each wave runs
// ITER x 4 groups of 8 independent instructions on EXPLICIT registers (raw asm, clobbered), so
// the VGPR bank of every operand (register number mod 4) is fixed: v_fma_f32 with its three
// sources in distinct banks / two in one bank / the same register twice, v_add_f32 with both
// sources in one bank, v_cndmask_b32 with a VCC or SGPR-pair mask, DPP, SDWA, v_dot2c, v_perm.
// 16 waves per workgroup, one workgroup per CU (4 waves per SIMD).  Cycles from s_memtime
// (shader clock).  Build: hipcc --offload-arch=gfx950 -O3 operand_rate.hip -o operand_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <algorithm>

#define CLOB "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", \
             "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34",       \
             "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", \
             "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", \
             "v63", "vcc", "s40", "s41"

// 8 chains in bank 0 (v8, v12, ..., v36); sources: bank 1 = v41/v45, bank 2 = v42/v46, bank 3 = v43
#define G8(OP)                                                                                                    \
    OP(v8) OP(v12) OP(v16) OP(v20) OP(v24) OP(v28) OP(v32) OP(v36)

#define FMA_DISTINCT(r) "v_fma_f32 " #r ", v41, v42, " #r "\n"      // banks 0,1,2 (src2 = dst)
#define FMA_SAME01(r) "v_fma_f32 " #r ", v41, v45, " #r "\n"        // src0/src1 both bank 1
#define FMA_SAMEREG(r) "v_fma_f32 " #r ", v41, v41, " #r "\n"       // src0 = src1 register
#define FMA_SRC2BANK(r) "v_fma_f32 " #r ", v44, v41, " #r "\n"      // src0 bank 0 = src2 bank
#define FMAC_DISTINCT(r) "v_fmac_f32_e32 " #r ", v41, v42\n"
#define FMAC_SAME(r) "v_fmac_f32_e32 " #r ", v41, v45\n"
#define ADD_DIFF(r) "v_add_f32_e32 " #r ", v41, " #r "\n"          // banks 1, 0
#define ADD_SAME(r) "v_add_f32_e32 " #r ", v44, " #r "\n"          // banks 0, 0
#define SUB_VOP3(r) "v_sub_f32_e64 " #r ", v41, " #r "\n"
#define MUL_DIFF(r) "v_mul_f32_e32 " #r ", v41, " #r "\n"
#define CND_VCC(r) "v_cndmask_b32_e32 " #r ", v41, " #r ", vcc\n"
#define CND_SGPR(r) "v_cndmask_b32_e64 " #r ", v41, " #r ", s[40:41]\n"
#define DPP_MOV(r) "v_mov_b32_dpp " #r ", v41 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
#define DPP_ADD(r) "v_add_f32_dpp " #r ", v41, " #r " quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
#define SDWA_CVT(r) "v_cvt_f32_i32_sdwa " #r ", v41 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1\n"
#define CVT(r) "v_cvt_f32_i32_e32 " #r ", v41\n"
#define PERM(r) "v_perm_b32 " #r ", v41, v42, v43\n"
#define BFE(r) "v_bfe_i32 " #r ", v41, 16, 16\n"
#define MOV(r) "v_mov_b32_e32 " #r ", v41\n"
// operand sources other than VGPRs: an SGPR, a 32-bit literal, an inline constant
#define FMA_SGPR(r) "v_fma_f32 " #r ", v41, s40, " #r "\n"
#define FMA_NEGSGPR(r) "v_fma_f32 " #r ", v41, s40, -" #r "\n"
#define MUL_LIT(r) "v_mul_f32_e32 " #r ", 0x3f3504f3, " #r "\n"
#define FMAMK_LIT(r) "v_fmamk_f32 " #r ", v41, 0x3f3504f3, " #r "\n"
#define MUL_SGPR(r) "v_mul_f32_e32 " #r ", s40, " #r "\n"
#define ADD_SGPR(r) "v_add_f32_e32 " #r ", s40, " #r "\n"
#define MUL_INL(r) "v_mul_f32_e32 " #r ", 0.5, " #r "\n"
#define FMA_NEGV(r) "v_fma_f32 " #r ", v41, v42, -" #r "\n"
// packed / mixed bodies on the register pairs v[8:9], v[12:13], ... (8 independent chains)
#define G8P(OP) OP(8, 9) OP(12, 13) OP(16, 17) OP(20, 21) OP(24, 25) OP(28, 29) OP(32, 33) OP(36, 37)
#define PKADD(a, b) "v_pk_add_f32 v[" #a ":" #b "], v[42:43], v[" #a ":" #b "]\n"
#define PKFMA(a, b) "v_pk_fma_f32 v[" #a ":" #b "], v[42:43], v[46:47], v[" #a ":" #b "]\n"
#define MIX_ADDFMA(a, b) "v_add_f32_e32 v" #a ", v41, v" #a "\nv_fma_f32 v" #b ", v41, v42, v" #b "\n"

#define I4(a, b, c, d) "v_mov_b32 v" #a ", 1.0\nv_mov_b32 v" #b ", 1.0\nv_mov_b32 v" #c ", 1.0\nv_mov_b32 v" #d ", 1.0\n"
#define INITALL I4(8, 9, 10, 11) I4(12, 13, 14, 15) I4(16, 17, 18, 19) I4(20, 21, 22, 23) I4(24, 25, 26, 27) \
    I4(28, 29, 30, 31) I4(32, 33, 34, 35) I4(36, 37, 38, 39)
#define KERNEL(NAME, BODY)                                                                                    \
    __global__ void NAME(long long *cyc, int iters) {                                                       \
        asm volatile(                                                                                         \
            "v_mov_b32 v41, 1.0\nv_mov_b32 v42, 0.5\nv_mov_b32 v43, 0x03020100\nv_mov_b32 v44, 0.25\n"      \
            "v_mov_b32 v45, 0.75\nv_mov_b32 v46, 0.125\nv_mov_b32 v47, 0.5\nv_mov_b32 v50, 0\n"             \
            "v_mov_b32 v51, 0\n" INITALL "s_mov_b32 vcc_lo, 0x55555555\ns_mov_b32 vcc_hi, 0x55555555\n"                                   \
            "s_mov_b32 s40, 0x33333333\ns_mov_b32 s41, 0x33333333\n" ::                                                     \
                : CLOB);                                                                                      \
        __syncthreads();                                                                                      \
        const long long t0 = __builtin_amdgcn_s_memtime();                                                    \
        for (int it = 0; it < iters; ++it) {                                                                  \
            asm volatile(G8(BODY) G8(BODY) G8(BODY) G8(BODY)::: CLOB);                                        \
        }                                                                                                     \
        __syncthreads();                                                                                      \
        const long long t1 = __builtin_amdgcn_s_memtime();                                                    \
        if (threadIdx.x == 0) {                                                                               \
            const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));                       \
            const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11));                      \
            cyc[3 * blockIdx.x] = t0;                                                                          \
            cyc[3 * blockIdx.x + 1] = t1;                                                                      \
            cyc[3 * blockIdx.x + 2] = ((long long)xcc << 32) | ((hw >> 8) & 0xff);                             \
        }                                                                                                     \
    }

KERNEL(k_fma_distinct, FMA_DISTINCT)
KERNEL(k_fma_same01, FMA_SAME01)
KERNEL(k_fma_samereg, FMA_SAMEREG)
KERNEL(k_fma_src2bank, FMA_SRC2BANK)
KERNEL(k_fmac_distinct, FMAC_DISTINCT)
KERNEL(k_fmac_same, FMAC_SAME)
KERNEL(k_add_diff, ADD_DIFF)
KERNEL(k_add_same, ADD_SAME)
KERNEL(k_sub_vop3, SUB_VOP3)
KERNEL(k_mul_diff, MUL_DIFF)
KERNEL(k_cnd_vcc, CND_VCC)
KERNEL(k_cnd_sgpr, CND_SGPR)
KERNEL(k_dpp_mov, DPP_MOV)
KERNEL(k_dpp_add, DPP_ADD)
KERNEL(k_sdwa_cvt, SDWA_CVT)
KERNEL(k_cvt, CVT)
KERNEL(k_perm, PERM)
KERNEL(k_bfe, BFE)
KERNEL(k_mov, MOV)
KERNEL(k_fma_sgpr, FMA_SGPR)
KERNEL(k_fma_negsgpr, FMA_NEGSGPR)
KERNEL(k_mul_lit, MUL_LIT)
KERNEL(k_fmamk_lit, FMAMK_LIT)
KERNEL(k_mul_sgpr, MUL_SGPR)
KERNEL(k_add_sgpr, ADD_SGPR)
KERNEL(k_mul_inl, MUL_INL)
KERNEL(k_fma_negv, FMA_NEGV)
#define G8 G8P
KERNEL(k_pkadd, PKADD)
KERNEL(k_pkfma, PKFMA)
KERNEL(k_mix_addfma, MIX_ADDFMA)

static void run(void (*kern)(long long *, int), const char *name, int per_iter, long long *cyc, int cus,
                int waves_per_wg) {
    const int iters = 400;
    static long long h[3 * 4096];
    double best = 1e30;
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(kern, dim3(cus), dim3(64 * waves_per_wg), 0, 0, cyc, iters);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(h, cyc, sizeof(long long) * 3 * cus, hipMemcpyDeviceToHost);
        std::map<long long, std::pair<long long, long long>> span;
        for (int i = 0; i < cus; ++i) {
            auto it = span.find(h[3 * i + 2]);
            if (it == span.end()) span[h[3 * i + 2]] = {h[3 * i], h[3 * i + 1]};
            else it->second = {std::min(it->second.first, h[3 * i]), std::max(it->second.second, h[3 * i + 1])};
        }
        double m = 0;
        for (auto &kv : span) m += kv.second.second - kv.second.first;
        m /= span.size();
        best = std::min(best, m);
    }
    const double instr_per_simd = (double)iters * per_iter * (waves_per_wg / 4);
    printf("%-16s %d waves/SIMD  %.2f cycles per wave-instruction per SIMD\n", name, waves_per_wg / 4,
           best / instr_per_simd);
}

int main() {
    long long *cyc;
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    (void)hipMalloc(&cyc, sizeof(long long) * cus * 3);
    for (int w : {16, 8}) {
#define R(k, n) run(k, #k, n, cyc, cus, w);
        R(k_fma_distinct, 32) R(k_fma_same01, 32) R(k_fma_samereg, 32) R(k_fma_src2bank, 32)
        R(k_fmac_distinct, 32) R(k_fmac_same, 32) R(k_add_diff, 32) R(k_add_same, 32) R(k_sub_vop3, 32)
        R(k_mul_diff, 32) R(k_cnd_vcc, 32) R(k_cnd_sgpr, 32) R(k_dpp_mov, 32) R(k_dpp_add, 32)
        R(k_sdwa_cvt, 32) R(k_cvt, 32) R(k_perm, 32) R(k_bfe, 32) R(k_mov, 32) R(k_pkadd, 32) R(k_pkfma, 32)
        R(k_mix_addfma, 64)
        R(k_fma_sgpr, 32) R(k_fma_negsgpr, 32) R(k_mul_lit, 32) R(k_fmamk_lit, 32) R(k_mul_sgpr, 32)
        R(k_add_sgpr, 32) R(k_mul_inl, 32) R(k_fma_negv, 32)
    }
    (void)hipFree(cyc);
    return 0;
}
