// pk_power.hip -- does packed f32 arithmetic change the VALU-bound speed of
// a power-capped chip? The same separately rounded mul/add work (16 lane-ops
// per iteration per lane) as 16 scalar v_mul/v_add_f32 or as 8 packed
// v_pk_mul/v_pk_add_f32, on every CU, long enough to reach steady power.
// Prints the time per launch; clocks and power come from amd-smi beside it
// (tools/gpu/pk_power.sh).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize tools/pk_power.hip -o tools/pk_power
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef float f2 __attribute__((ext_vector_type(2)));

template <bool PK>
__global__ void __launch_bounds__(256) k_valu(float* out, int iters, float ms, float cs)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    float r = 0.0f;
    // per-lane (VGPR) operands, as in the search kernel: m, c opaque to the compiler
    float m = ms, c = cs;
    __asm__("" : "+v"(m));
    __asm__("" : "+v"(c));
    if constexpr (PK) {
        f2 a[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = (f2){(float)(t & 7) + i, (float)(t & 3) + 2 * i};
        const f2 mm = {m, m}, cc = {c, c};
        for (int it = 0; it < iters; ++it)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                a[i] = a[i] * mm;
                a[i] = a[i] + cc;
            }
#pragma unroll
        for (int i = 0; i < 4; ++i) r += a[i].x + a[i].y;
    } else {
        float a[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = (float)((t >> (i & 1)) & 7) + i;
        for (int it = 0; it < iters; ++it)
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                a[i] = a[i] * m;
                a[i] = a[i] + c;
            }
#pragma unroll
        for (int i = 0; i < 8; ++i) r += a[i];
    }
    out[t] = r;
}

int main(int argc, char** argv)
{
    const bool pk = argc > 1 && !strcmp(argv[1], "pk");
    const double seconds = argc > 2 ? atof(argv[2]) : 20.0;
    const int blocks = 256 * 16, threads = 256;  // 64 waves per CU: every SIMD full
    const int iters = 20000;
    float* out;
    if (hipMalloc(&out, sizeof(float) * blocks * threads) != hipSuccess) return 1;
    auto launch = [&] {
        if (pk) hipLaunchKernelGGL(k_valu<true>, dim3(blocks), dim3(threads), 0, 0, out, iters, 0.999f, 0.001f);
        else hipLaunchKernelGGL(k_valu<false>, dim3(blocks), dim3(threads), 0, 0, out, iters, 0.999f, 0.001f);
    };
    launch();
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int n = 0;
    float total_ms = 0.0f;
    const auto t0 = std::chrono::steady_clock::now();
    while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < seconds) {
        hipEventRecord(e0, 0);
        for (int k = 0; k < 10; ++k) launch();
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0.0f;
        hipEventElapsedTime(&ms, e0, e1);
        total_ms += ms;
        n += 10;
    }
    const double ops = 16.0 * iters * (double)blocks * threads;  // lane-ops per launch
    printf("%s: %d launches, %.3f ms per launch, %.1f T lane-ops/s\n", pk ? "packed" : "scalar", n, total_ms / n,
           ops / (total_ms / n * 1e-3) / 1e12);
    hipFree(out);
    return 0;
}
