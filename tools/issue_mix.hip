// issue_mix.hip -- issue cost of the instruction kinds in the search loop.
// The finest k_search8 loop is 472 VALU instructions per update, most of them
// v_mul/v_add_f32 with VGPR operands; the rest read an SGPR (lane masks of
// v_cndmask, VOPC compares against SGPR bounds), a literal, or carry a DPP
// modifier. DESIGN.md 3 (r03) measured that an SGPR operand halves the VALU
// issue rate of v_mul (38.0 vs 71.2 T lane-ops/s). This times every other
// kind the loop uses, alone and mixed 1:3 with plain v_mul, at 4 and 8 waves
// per SIMD, so each loop change can be priced before it is built.
//   hipcc --offload-arch=gfx950 -O3 tools/issue_mix.hip -o tools/issue_mix
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

// 8 independent chains a0..a7; one "op" = one instruction on one chain
#define V8(OP) OP(0) OP(1) OP(2) OP(3) OP(4) OP(5) OP(6) OP(7)

#define MUL_VV(i) "v_mul_f32 %" #i ", %" #i ", %8\n"
#define MUL_VS(i) "v_mul_f32 %" #i ", %9, %" #i "\n"
#define MUL_VL(i) "v_mul_f32 %" #i ", 0x3f7ff972, %" #i "\n"
#define MUL_DPP(i) "v_mul_f32_dpp %" #i ", %8, %" #i " quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
#define ADD_ROR(i) "v_add_f32_dpp %" #i ", %8, %" #i " row_ror:8 row_mask:0xf bank_mask:0xf\n"
#define MOV_DPP(i) "v_mov_b32_dpp %" #i ", %8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
#define CND_S(i) "v_cndmask_b32_e64 %" #i ", %" #i ", %8, %10\n"
#define CND_VCC(i) "v_cndmask_b32_e32 %" #i ", %" #i ", %8, vcc\n"
#define BFI(i) "v_bfi_b32 %" #i ", %11, %8, %" #i "\n"
#define FMA(i) "v_fma_f32 %" #i ", %" #i ", %8, %12\n"
#define FMAC(i) "v_fmac_f32 %" #i ", %8, %12\n"
#define MAD24(i) "v_mad_i32_i24 %" #i ", %" #i ", %11, %12\n"
#define CMP_S(i) "v_cmp_gt_f32 vcc, %9, %" #i "\n"
#define CMP_V(i) "v_cmp_gt_f32 vcc, %8, %" #i "\n"
#define CMPX(i) "v_cmp_gt_f32_e64 s[20:21], %" #i ", %8\n"
// compare + select pairs, as the compiler emits `c ? a : b` (VCC, or an SGPR pair)
#define CMPSEL_VCC(i) "v_cmp_gt_f32 vcc, %8, %" #i "\nv_cndmask_b32_e32 %" #i ", %" #i ", %8, vcc\n"
#define CMPSEL_S(i) "v_cmp_gt_f32_e64 s[20:21], %8, %" #i "\nv_cndmask_b32_e64 %" #i ", %" #i ", %8, s[20:21]\n"
#define CND_VCC64(i) "v_cndmask_b32_e64 %" #i ", %" #i ", %8, vcc\n"
// 1 op of a kind, then 3 plain v_mul (the mix the loop has at worst)
#define MIX(K) K(0) MUL_VV(1) MUL_VV(2) MUL_VV(3) K(4) MUL_VV(5) MUL_VV(6) MUL_VV(7)

#define KIND(name, body)                                                                                      \
    if (kind == name) {                                                                                        \
        for (int it = 0; it < iters; ++it)                                                                     \
            __asm__ volatile(body                                                                              \
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
                             : "v"(m), "s"(sm), "s"(mask), "v"(vmask), "v"(c)                                  \
                             : "vcc", "s20", "s21");                                                           \
    }

__global__ void __launch_bounds__(256) k_mix(float* out, int kind, int iters, float ms)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    float a0 = 1.0f + (t & 7), a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
          a7 = a0 + 7;
    float m = ms, c = 0.001f;
    __asm__("" : "+v"(m));
    __asm__("" : "+v"(c));
    const float sm = ms;
    const unsigned long long mask = 0x5555555555555555ull;
    int vmask = (t & 1) ? -1 : 0;
    __asm__("" : "+v"(vmask));
    // VCC defined before any kind reads it (as a VALU compare would leave it)
    __asm__ volatile("v_cmp_gt_f32 vcc, %0, %1" ::"v"(m), "v"(c) : "vcc");
    KIND(0, V8(MUL_VV))
    KIND(1, V8(MUL_VS))
    KIND(2, V8(MUL_VL))
    KIND(3, V8(MUL_DPP))
    KIND(4, V8(ADD_ROR))
    KIND(5, V8(MOV_DPP))
    KIND(6, V8(CND_S))
    KIND(7, V8(CND_VCC))
    KIND(8, V8(BFI))
    KIND(9, V8(FMA))
    KIND(10, V8(FMAC))
    KIND(11, V8(MAD24))
    KIND(12, V8(CMP_S))
    KIND(13, V8(CMP_V))
    KIND(14, V8(CMPX))
    KIND(15, MIX(MUL_VS))
    KIND(16, MIX(MUL_VL))
    KIND(17, MIX(MUL_DPP))
    KIND(18, MIX(CND_S))
    KIND(19, MIX(BFI))
    KIND(20, MIX(CMP_S))
    KIND(21, MIX(ADD_ROR))
    KIND(22, MIX(CND_VCC))
    KIND(23, V8(CMPSEL_VCC))
    KIND(24, V8(CMPSEL_S))
    KIND(25, V8(CND_VCC64))
    out[t] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

static const char* kNames[] = {"v_mul v,v",       "v_mul s,v",      "v_mul lit,v",   "v_mul_dpp qperm",
                               "v_add_dpp ror8",  "v_mov_dpp",      "v_cndmask s[]", "v_cndmask vcc",
                               "v_bfi v,v,v",     "v_fma v,v,v",    "v_fmac",        "v_mad_i32_i24",
                               "v_cmp s,v ->vcc", "v_cmp v,v ->vcc", "v_cmp ->s[]",  "mix 1:3 mul s,v",
                               "mix 1:3 mul lit", "mix 1:3 mul_dpp", "mix 1:3 cndmask s", "mix 1:3 bfi",
                               "mix 1:3 cmp s", "mix 1:3 add_dpp ror8", "mix 1:3 cndmask vcc",
                               "cmp->vcc + cndmask vcc", "cmp->s[] + cndmask s[]", "v_cndmask_e64 vcc"};

int main(int argc, char** argv)
{
    const int nk = sizeof(kNames) / sizeof(kNames[0]);
    const int iters = 4000;
    float* out;
    if (hipMalloc(&out, sizeof(float) * 256 * 32 * 256) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    // clock ramp: ~1.5 s of back-to-back launches before anything is timed
    for (int w = 0; w < 300; ++w) hipLaunchKernelGGL(k_mix, dim3(256 * 8), dim3(256), 0, 0, out, 0, iters, 0.999f);
    hipDeviceSynchronize();
    // occupancy sweep: plain v_mul, v_fma and the 1:3 DPP mix at 1..8 waves per SIMD
    printf("occupancy sweep (ns per wave-instruction per SIMD)\n");
    for (int k : {0, 9, 17}) {
        printf("  %-22s", kNames[k]);
        for (int wps = 1; wps <= 8; ++wps) {
            const int blocks = 256 * wps, threads = 256;
            float best = 1e30f;
            for (int rep = 0; rep < 4; ++rep) {
                hipEventRecord(e0, 0);
                hipLaunchKernelGGL(k_mix, dim3(blocks), dim3(threads), 0, 0, out, k, iters * 4, 0.999f);
                hipEventRecord(e1, 0);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                best = ms < best ? ms : best;
            }
            printf(" %d:%.3f", wps, best * 1e6 / ((double)wps * iters * 4 * 8));
        }
        printf("\n");
    }
    for (int wps : {4, 8}) {  // waves per SIMD (256 CUs x 4 SIMDs)
        const int blocks = 256 * wps, threads = 256;  // 4 waves per block, one per SIMD on average
        printf("waves per SIMD %d\n", wps);
        for (int k = 0; k < nk; ++k) {
            hipLaunchKernelGGL(k_mix, dim3(blocks), dim3(threads), 0, 0, out, k, iters, 0.999f);
            hipDeviceSynchronize();
            float best = 1e30f;
            for (int rep = 0; rep < 5; ++rep) {
                hipEventRecord(e0, 0);
                hipLaunchKernelGGL(k_mix, dim3(blocks), dim3(threads), 0, 0, out, k, iters, 0.999f);
                hipEventRecord(e1, 0);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                best = ms < best ? ms : best;
            }
            // instructions per SIMD = waves per SIMD x iters x 8
            const double insts = (double)wps * iters * 8;
            printf("  %-22s %8.3f ms  %6.3f ns per wave-instruction per SIMD\n", kNames[k], best,
                   best * 1e6 / insts);
        }
    }
    if (hipGetLastError() != hipSuccess) return 1;
    hipFree(out);
    return 0;
}
