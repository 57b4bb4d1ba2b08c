// valu_rate.hip -- issue rate of scalar vs packed f32 VALU ops on gfx950:
// every wave runs independent chains of one instruction form; reports
// wave-instructions per SIMD per core cycle (cycles from s_memtime).
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x

template <int K>
__global__ void __launch_bounds__(256) k_rate(float* out, long long* cyc, int n)
{
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const float b = 1.0001f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}, bb = {b, b};
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
        if constexpr (K == 0) {  // v_add_f32
            REP8(asm volatile("v_add_f32 %0, %0, %8\n v_add_f32 %1, %1, %8\n v_add_f32 %2, %2, %8\n v_add_f32 %3, %3, %8\n"
                              "v_add_f32 %4, %4, %8\n v_add_f32 %5, %5, %8\n v_add_f32 %6, %6, %8\n v_add_f32 %7, %7, %8"
                              : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
        } else if constexpr (K == 1) {  // v_mul_f32
            REP8(asm volatile("v_mul_f32 %0, %0, %8\n v_mul_f32 %1, %1, %8\n v_mul_f32 %2, %2, %8\n v_mul_f32 %3, %3, %8\n"
                              "v_mul_f32 %4, %4, %8\n v_mul_f32 %5, %5, %8\n v_mul_f32 %6, %6, %8\n v_mul_f32 %7, %7, %8"
                              : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
        } else if constexpr (K == 2) {  // v_pk_add_f32 (4 pairs = same 8 values)
            REP8(asm volatile("v_pk_add_f32 %0, %0, %4\n v_pk_add_f32 %1, %1, %4\n v_pk_add_f32 %2, %2, %4\n v_pk_add_f32 %3, %3, %4"
                              : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(bb));)
        } else if constexpr (K == 3) {  // v_pk_mul_f32
            REP8(asm volatile("v_pk_mul_f32 %0, %0, %4\n v_pk_mul_f32 %1, %1, %4\n v_pk_mul_f32 %2, %2, %4\n v_pk_mul_f32 %3, %3, %4"
                              : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(bb));)
        } else if constexpr (K == 4) {  // v_pk_mul_f32 with broadcast scalar (op_sel_hi:[1,0])
            REP8(asm volatile("v_pk_mul_f32 %0, %0, %4 op_sel_hi:[1,0]\n v_pk_mul_f32 %1, %1, %4 op_sel_hi:[1,0]\n"
                              "v_pk_mul_f32 %2, %2, %4 op_sel_hi:[1,0]\n v_pk_mul_f32 %3, %3, %4 op_sel_hi:[1,0]"
                              : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(bb));)
        } else if constexpr (K == 5) {  // v_fma_f32
            REP8(asm volatile("v_fma_f32 %0, %0, %8, %8\n v_fma_f32 %1, %1, %8, %8\n v_fma_f32 %2, %2, %8, %8\n v_fma_f32 %3, %3, %8, %8\n"
                              "v_fma_f32 %4, %4, %8, %8\n v_fma_f32 %5, %5, %8, %8\n v_fma_f32 %6, %6, %8, %8\n v_fma_f32 %7, %7, %8, %8"
                              : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
        } else if constexpr (K == 6) {  // DPP add (quad_perm)
            REP8(asm volatile("v_add_f32_dpp %0, %0, %8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
                              "v_add_f32_dpp %1, %1, %8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
                              "v_add_f32_dpp %2, %2, %8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
                              "v_add_f32_dpp %3, %3, %8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
                              "v_add_f32_dpp %4, %4, %8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
                              "v_add_f32_dpp %5, %5, %8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
                              "v_add_f32_dpp %6, %6, %8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
                              "v_add_f32_dpp %7, %7, %8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
                              : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + p0.x + p0.y + p1.x + p1.y + p2.x + p2.y + p3.x + p3.y;
}

template <int K>
void run(const char* name, int waves_per_simd, float* out, long long* cyc)
{
    const int n = 2000, blocks = 256 * waves_per_simd;  // 4 waves per block = 1 per SIMD
    hipLaunchKernelGGL(k_rate<K>, dim3(blocks), dim3(256), 0, 0, out, cyc, 100);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_rate<K>, dim3(blocks), dim3(256), 0, 0, out, cyc, n);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    long long c;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    const double per_wave = (K >= 2 && K <= 4) ? 32.0 * n : 64.0 * n;  // instructions per wave
    const double simd_instr = per_wave * waves_per_simd;                // per SIMD
    printf("%-28s waves/SIMD %d: %.3f ms, %.2f cyc per wave-instr per SIMD (wave0 cycles %lld -> %.2f cyc/instr/wave)\n",
           name, waves_per_simd, ms, ms * 1e-3 * 2.4e9 / simd_instr, c, (double)c / per_wave);
}

int main()
{
    float* out;
    long long* cyc;
    hipMalloc(&out, 256 * 16 * 256 * 4);
    hipMalloc(&cyc, 8);
    for (int w : {1, 2, 4, 8}) {
        run<0>("v_add_f32", w, out, cyc);
        run<1>("v_mul_f32", w, out, cyc);
        run<5>("v_fma_f32", w, out, cyc);
        run<2>("v_pk_add_f32", w, out, cyc);
        run<3>("v_pk_mul_f32", w, out, cyc);
        run<4>("v_pk_mul_f32 bcast", w, out, cyc);
        run<6>("v_add_f32_dpp", w, out, cyc);
    }
    return 0;
}
