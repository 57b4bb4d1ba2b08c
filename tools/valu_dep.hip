// valu_dep.hip -- VALU issue rate vs dependency structure on gfx950, to size
// the ILP the search loop needs: cycles per wave-instruction per SIMD for
// (0) 8 independent chains, (1) one fully dependent chain, (2) 2 and (3) 4
// interleaved chains, (4) the warp's per-pixel mul/add pattern as the
// compiler emits it (every add consumes the product issued just before it),
// (5) the same pattern with two pixels interleaved; at 1..8 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP4(x) x x x x
#define REP8(x) x x x x x x x x

template <int K>
__global__ void __launch_bounds__(256) k_dep(float* out, long long* cyc, int n)
{
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    float t0 = 0, t1 = 0;
    const float b = 1.0001f, w0 = 0.25f, w1 = 0.5f, w2 = 0.125f, w3 = 0.0625f;
    long long c0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
        if constexpr (K == 0) {  // 8 independent chains: 64 instructions
            REP8(asm volatile("v_add_f32 %0, %0, %8\n v_add_f32 %1, %1, %8\n v_add_f32 %2, %2, %8\n v_add_f32 %3, %3, %8\n"
                              "v_add_f32 %4, %4, %8\n v_add_f32 %5, %5, %8\n v_add_f32 %6, %6, %8\n v_add_f32 %7, %7, %8"
                              : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
        } else if constexpr (K == 1) {  // one dependent chain: 64 instructions
            REP8(asm volatile("v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n"
                              "v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1\n v_add_f32 %0, %0, %1"
                              : "+v"(a0) : "v"(b));)
        } else if constexpr (K == 2) {  // 2 interleaved chains
            REP8(asm volatile("v_add_f32 %0, %0, %2\n v_add_f32 %1, %1, %2\n v_add_f32 %0, %0, %2\n v_add_f32 %1, %1, %2\n"
                              "v_add_f32 %0, %0, %2\n v_add_f32 %1, %1, %2\n v_add_f32 %0, %0, %2\n v_add_f32 %1, %1, %2"
                              : "+v"(a0), "+v"(a1) : "v"(b));)
        } else if constexpr (K == 3) {  // 4 interleaved chains
            REP8(asm volatile("v_add_f32 %0, %0, %4\n v_add_f32 %1, %1, %4\n v_add_f32 %2, %2, %4\n v_add_f32 %3, %3, %4\n"
                              "v_add_f32 %0, %0, %4\n v_add_f32 %1, %1, %4\n v_add_f32 %2, %2, %4\n v_add_f32 %3, %3, %4"
                              : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(b));)
        } else if constexpr (K == 4) {  // pixel pattern: mul, mul, add, mul, add, mul, add (7), x9 + 1 pad = 64
            REP8(asm volatile("v_mul_f32 %1, %3, %4\n v_mul_f32 %2, %5, %4\n v_add_f32 %0, %2, %1\n"
                              "v_mul_f32 %2, %6, %4\n v_add_f32 %0, %2, %0\n v_mul_f32 %2, %7, %4\n v_add_f32 %0, %2, %0\n"
                              "v_mul_f32 %1, %3, %0\n"
                              : "+v"(a0), "+v"(t0), "+v"(t1) : "v"(w3), "v"(a1), "v"(w2), "v"(w1), "v"(w0));)
        } else if constexpr (K == 5) {  // two pixels interleaved (same 8 per pixel)
            // A: acc %0, products %2 %3; B: acc %1, products %4 %5
            REP4(asm volatile("v_mul_f32 %2, %6, %7\n v_mul_f32 %4, %6, %7\n v_mul_f32 %3, %8, %7\n v_mul_f32 %5, %8, %7\n"
                              "v_add_f32 %0, %3, %2\n v_add_f32 %1, %5, %4\n v_mul_f32 %3, %9, %7\n v_mul_f32 %5, %9, %7\n"
                              "v_add_f32 %0, %3, %0\n v_add_f32 %1, %5, %1\n v_mul_f32 %3, %10, %7\n v_mul_f32 %5, %10, %7\n"
                              "v_add_f32 %0, %3, %0\n v_add_f32 %1, %5, %1\n v_mul_f32 %2, %6, %0\n v_mul_f32 %4, %6, %1\n"
                              : "+v"(a0), "+v"(a2), "+v"(t0), "+v"(t1), "+v"(a3), "+v"(a4)
                              : "v"(w3), "v"(a1), "v"(w2), "v"(w1), "v"(w0));)
        }
    }
    long long c1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = c1 - c0;
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + t0 + t1;
}

template <int K>
void run(const char* name, int waves_per_simd, float* out, long long* cyc)
{
    const int n = 4000, blocks = 256 * waves_per_simd;  // 4 waves per block = 1 per SIMD
    hipLaunchKernelGGL(k_dep<K>, dim3(blocks), dim3(256), 0, 0, out, cyc, 100);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_dep<K>, dim3(blocks), dim3(256), 0, 0, out, cyc, n);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    long long c;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    const double per_wave = 64.0 * n;
    printf("%-22s waves/SIMD %d: %.3f ms, wave0 %.2f shader cyc/instr -> %.2f cyc per instr per SIMD\n", name,
           waves_per_simd, ms, (double)c / per_wave, (double)c / per_wave / waves_per_simd);
}

int main()
{
    float* out;
    long long* cyc;
    hipMalloc(&out, 256 * 16 * 256 * 4);
    hipMalloc(&cyc, 8);
    for (int w : {1, 2, 3, 4, 5, 6, 8}) {
        run<0>("8 indep chains", w, out, cyc);
        run<1>("1 dep chain", w, out, cyc);
        run<2>("2 chains", w, out, cyc);
        run<3>("4 chains", w, out, cyc);
        run<4>("pixel mul/add", w, out, cyc);
        run<5>("2 pixels interleaved", w, out, cyc);
    }
    return 0;
}
