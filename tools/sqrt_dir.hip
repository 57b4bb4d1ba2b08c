// sqrt_dir.hip -- which way is the raw v_sqrt_f32 off on the pyramid's inputs?
// For every integer N in [0, 2 * 1020^2] (the exact Sobel sum k1^2 + k2^2 of
// u8 input, see sqrt_check.hip) compares r = v_sqrt_f32(N) with the correctly
// rounded sqrtf(N) and counts r == RN, r == RN + 1 ulp, r == RN - 1 ulp, other;
// then checks the two one-sided corrections (only the "round up" test, only
// the "round down" test) of dis::sqrt_cr for equality with RN on every N. A
// one-sided correction with zero mismatches is exact on the whole domain.
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ float up_only(float x)
{
    const float r = __builtin_amdgcn_sqrtf(x);
    const float rp = __int_as_float(__float_as_int(r) + 1);
    return __builtin_fmaf(-rp, r, x) > 0.0f ? rp : r;
}

__device__ __forceinline__ float down_only(float x)
{
    const float r = __builtin_amdgcn_sqrtf(x);
    const float rm = __int_as_float(__float_as_int(r) - 1);
    return __builtin_fmaf(-rm, r, x) <= 0.0f ? rm : r;
}

__global__ void k_dir(int nmax, unsigned int* cnt)
{
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n > nmax) return;
    const float x = (float)n;
    const int ref = __float_as_int(sqrtf(x));
    const int raw = __float_as_int(__builtin_amdgcn_sqrtf(x));
    const int d = raw - ref;
    atomicAdd(&cnt[d == 0 ? 0 : d == 1 ? 1 : d == -1 ? 2 : 3], 1u);
    if (__float_as_int(up_only(x)) != ref) atomicAdd(&cnt[4], 1u);
    if (__float_as_int(down_only(x)) != ref) atomicAdd(&cnt[5], 1u);
}

int main()
{
    const int nmax = 2 * 1020 * 1020;
    unsigned int* cnt;
    if (hipMalloc(&cnt, 6 * sizeof(unsigned)) != hipSuccess || hipMemset(cnt, 0, 6 * sizeof(unsigned)) != hipSuccess)
        return 2;
    hipLaunchKernelGGL(k_dir, dim3((nmax + 256) / 256), dim3(256), 0, 0, nmax, cnt);
    unsigned h[6];
    if (hipMemcpy(h, cnt, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    printf("sqrt_dir: %d inputs; raw == RN %u, RN+1ulp %u, RN-1ulp %u, other %u; "
           "up-only correction mismatches %u, down-only %u\n",
           nmax + 1, h[0], h[1], h[2], h[3], h[4], h[5]);
    return 0;
}
