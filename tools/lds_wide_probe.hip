// lds_wide_probe.hip -- can the tolerance-mode search fetch a lane's tap pairs
// with one wide LDS read at a data-dependent (4-mod-8) dword address instead of
// ds_read2_b32? On gfx950, for each form: are the returned
// words right, and what does one read cost per CU (cycles per wave-instruction,
// 4 waves per SIMD), at a conflict-free and at a search-like address pattern.
//
//   A  ds_read2_b32 (two dwords a, a + 1; what the compiler emits)   any a
//   B  ds_read_b64 at a 4-mod-8 byte address (a odd)                  inline asm
//   C  ds_read_b64 at an 8-aligned address (a even)                  reference
//   D  ds_read_b96 at a 4-mod-16 byte address (three dwords)          inline asm
//   E  ds_read2_b32 + ds_read_b32 (the same three dwords)
// Patterns: "linear" lane l reads dwords from 2l + 1 (conflict-free for A),
// "search" lane l reads from row (l / 4) * 72 + (l % 4) * 3 + 1 + 2 (l / 32)
// (the LPP-2 tile: 4 x 4 patches per half-wave, stride 72, grid step 3).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int kWords = 8192;  // 32 KB of LDS per workgroup (reads stay below word 31 * 100 + 480 + 300)
constexpr int kIters = 4096;

template <int MODE, int PAT>
__global__ void __launch_bounds__(256) k_probe(unsigned* out, unsigned* bad, int iters)
{
    __shared__ unsigned lds[kWords];
    for (int i = threadIdx.x; i < kWords; i += 256) lds[i] = i * 2654435761u;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    int a = PAT == 0 ? 2 * lane + 1 : (lane >> 2) * 72 + (lane & 3) * 3 + 1 + 2 * (lane >> 5);
    if (MODE == 2) a &= ~1;                  // aligned reference
    if (MODE == 3) a = (a & ~3) + 1;          // 4-mod-16
    a += 96 * (threadIdx.x >> 6);             // waves apart
    unsigned acc = 0, errs = 0;
    for (int it = 0; it < iters; ++it) {
        const int base = a + ((it * 7) & 31) * 100;  // walk the LDS, same alignment class
        // four independent reads per iteration (offsets 0, 160, 320, 480 dwords), one wait
        unsigned w[4][3] = {};
        if constexpr (MODE == 0 || MODE == 2) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                w[r][0] = lds[base + 160 * r];
                w[r][1] = lds[base + 160 * r + 1];
            }
        } else if constexpr (MODE == 1) {
            unsigned long long v0, v1, v2, v3;
            asm volatile(
                "ds_read_b64 %0, %4\n ds_read_b64 %1, %4 offset:640\n ds_read_b64 %2, %4 offset:1280\n"
                " ds_read_b64 %3, %4 offset:1920\n s_waitcnt lgkmcnt(0)"
                : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3)
                : "v"((unsigned)base * 4)
                : "memory");
            const unsigned long long v[4] = {v0, v1, v2, v3};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                w[r][0] = (unsigned)v[r];
                w[r][1] = (unsigned)(v[r] >> 32);
            }
        } else if constexpr (MODE == 3) {
            typedef unsigned u3 __attribute__((ext_vector_type(3)));
            u3 v0, v1, v2, v3;
            asm volatile(
                "ds_read_b96 %0, %4\n ds_read_b96 %1, %4 offset:640\n ds_read_b96 %2, %4 offset:1280\n"
                " ds_read_b96 %3, %4 offset:1920\n s_waitcnt lgkmcnt(0)"
                : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3)
                : "v"((unsigned)base * 4)
                : "memory");
            const u3 v[4] = {v0, v1, v2, v3};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                w[r][0] = v[r].x;
                w[r][1] = v[r].y;
                w[r][2] = v[r].z;
            }
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                w[r][0] = lds[base + 160 * r];
                w[r][1] = lds[base + 160 * r + 1];
                w[r][2] = lds[base + 160 * r + 2];
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const unsigned e = (unsigned)(base + 160 * r);
            if (MODE != 0 && MODE != 2 && MODE != 4 && it < 64) {
                errs += (w[r][0] != e * 2654435761u) + (w[r][1] != (e + 1) * 2654435761u);
                if (MODE == 3) errs += w[r][2] != (e + 2) * 2654435761u;
            }
            acc ^= w[r][0] + 3 * w[r][1] + 5 * w[r][2];
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
    if (errs) atomicAdd(bad, errs);
}

template <int MODE, int PAT>
static void run(const char* name, const char* pat)
{
    const int blocks = 256 * 4;  // 4 workgroups of 256 per CU: 4 waves per SIMD
    unsigned *out, *bad;
    hipMalloc(&out, sizeof(unsigned) * blocks * 256);
    hipMalloc(&bad, sizeof(unsigned));
    hipMemset(bad, 0, sizeof(unsigned));
    hipLaunchKernelGGL((k_probe<MODE, PAT>), dim3(blocks), dim3(256), 0, 0, out, bad, 64);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((k_probe<MODE, PAT>), dim3(blocks), dim3(256), 0, 0, out, bad, kIters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned nbad = 0;
    hipMemcpy(&nbad, bad, sizeof nbad, hipMemcpyDeviceToHost);
    // per CU: 16 waves x iters iterations, each fetching 4 tap pairs (triples for D / E) per lane
    const double per_cu = 16.0 * kIters * 4;
    std::printf("%-34s %-7s %8.3f ms  %6.2f ns per wave-wide tap-pair (triple) fetch per CU  wrong words: %u\n", name,
                pat, ms, ms * 1e6 / per_cu, nbad);
    hipFree(out);
    hipFree(bad);
}

int main()
{
    run<0, 0>("A ds_read2_b32 (a odd)", "linear");
    run<1, 0>("B ds_read_b64 @4-mod-8", "linear");
    run<2, 0>("C ds_read_b64 aligned (compiler)", "linear");
    run<3, 0>("D ds_read_b96 @4-mod-16", "linear");
    run<4, 0>("E ds_read2_b32 + ds_read_b32", "linear");
    run<0, 1>("A ds_read2_b32 (a odd)", "search");
    run<1, 1>("B ds_read_b64 @4-mod-8", "search");
    run<2, 1>("C ds_read_b64 aligned (compiler)", "search");
    run<3, 1>("D ds_read_b96 @4-mod-16", "search");
    run<4, 1>("E ds_read2_b32 + ds_read_b32", "search");
    std::printf("done\n");
    return 0;
}
