// color_core_check.hip -- are the colour kernel's fast correctly rounded
// operations (dis_device.h div_core, sqrt_core) the IEEE results on their
// fast domains? Their correctness rests on the GPU's v_rcp_f32 / v_sqrt_f32
// seeds (within one ulp, bits unspecified): a CPU model with seeds one ulp off
// fails on divisors with all-ones mantissas, so this checks the real seeds.
//  division: every divisor mantissa b in [1, 2) (2^23) x 64 numerators a in
//    [b 2^-30, b] (the powers of two and hashed mantissas, both edges), plus
//    the same at divisor exponents -60, -31, 30, 59 for every 16th mantissa;
//  sqrt: every x in [1, 4), [2^-96, 2^-94) and [2^94, 2^96) (2^24 each);
//  reciprocal (recip_core, the paper mode's vote weights): every m in
//    [1, 2^30) (30 x 2^23 floats);
// each against the compiler's IEEE a / b and sqrtf. Prints counts; exit 1 on
// a mismatch.  hipcc --offload-arch=gfx950 -O3 -ffp-contract=off
#include <hip/hip_runtime.h>
#include <cstdio>

#include "../optical-flow-using-dense-inverse-search_amd/csrc/dis_device.h"

__device__ unsigned hash32(unsigned x)
{
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    return x ^ (x >> 16);
}

__global__ void k_div(int exp_b, int step, unsigned long long* bad, unsigned int* first)
{
    const unsigned m = (blockIdx.x * blockDim.x + threadIdx.x) * step;
    if (m >= (1u << 23)) return;
    const float b = __uint_as_float(((unsigned)(127 + exp_b) << 23) | m);
    for (int k = 0; k < 64; ++k) {
        float a;
        if (k < 31) {
            a = __uint_as_float((unsigned)(127 + exp_b - k) << 23);  // powers of two in [b 2^-30, b]
        } else if (k < 33) {
            a = k == 31 ? b : b * 0x1p-30f;  // the domain's edges
        } else {
            const unsigned h = hash32(m * 64u + k);
            a = __uint_as_float(((unsigned)(127 + exp_b - (int)(h % 31)) << 23) | (h >> 9));
        }
        if (!dis::div_core_ok(a, b)) continue;
        const float want = a / b, got = dis::div_core(a, b);
        if (__float_as_uint(got) != __float_as_uint(want)) {
            atomicAdd(bad, 1ull);
            atomicMin(first, m);
        }
    }
}

__global__ void k_sqrt(int exp0, unsigned long long* bad, unsigned int* first)
{
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;  // 2^24: two binades
    if (i >= (1u << 24)) return;
    const float x = __uint_as_float((((unsigned)(127 + exp0) << 23) + i));
    if (!dis::sqrt_core_ok(x)) return;
    if (__float_as_uint(dis::sqrt_core(x)) != __float_as_uint(sqrtf(x))) {
        atomicAdd(bad, 1ull);
        atomicMin(first, i);
    }
}

__global__ void k_recip(unsigned long long* bad, unsigned int* first)
{
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;  // 30 binades from 1
    if (i >= 30u << 23) return;
    const float m = __uint_as_float((127u << 23) + i);
    if (__float_as_uint(dis::recip_core(m)) != __float_as_uint(1.0f / m)) {
        atomicAdd(bad, 1ull);
        atomicMin(first, i);
    }
}

int main()
{
    unsigned long long* bad;
    unsigned int* first;
    if (hipMalloc(&bad, 8) != hipSuccess || hipMalloc(&first, 4) != hipSuccess) return 2;
    int rc = 0;
    auto run = [&](const char* what, auto launch) {
        const unsigned big = 0xffffffffu;
        if (hipMemset(bad, 0, 8) != hipSuccess || hipMemcpy(first, &big, 4, hipMemcpyHostToDevice) != hipSuccess) exit(2);
        launch();
        unsigned long long hb = 0;
        unsigned hf = 0;
        if (hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost) != hipSuccess || hipMemcpy(&hf, first, 4, hipMemcpyDeviceToHost) != hipSuccess)
            exit(2);
        printf("color_core_check %-28s mismatches %llu%s", what, hb, hb ? "" : "\n");
        if (hb) printf(" (first index %u)\n", hf), rc = 1;
    };
    run("div b in [1,2)", [&] { hipLaunchKernelGGL(k_div, dim3((1 << 23) / 256), dim3(256), 0, 0, 0, 1, bad, first); });
    for (int e : {-60, -31, 30, 59}) {
        char name[64];
        snprintf(name, sizeof name, "div b in [2^%d, 2^%d)", e, e + 1);
        run(name, [&] { hipLaunchKernelGGL(k_div, dim3((1 << 19) / 256), dim3(256), 0, 0, e, 16, bad, first); });
    }
    for (int e : {0, -96, 94}) {
        char name[64];
        snprintf(name, sizeof name, "sqrt x in [2^%d, 2^%d)", e, e + 2);
        run(name, [&] { hipLaunchKernelGGL(k_sqrt, dim3((1 << 24) / 256), dim3(256), 0, 0, e, bad, first); });
    }
    run("recip m in [1, 2^30)", [&] { hipLaunchKernelGGL(k_recip, dim3((30u << 23) / 256), dim3(256), 0, 0, bad, first); });
    return rc;
}
