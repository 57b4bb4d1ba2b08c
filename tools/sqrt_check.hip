// sqrt_check.hip -- is the raw v_sqrt_f32 correctly rounded on every input the
// pyramid's Sobel magnitude can produce? s = gx^2 + gy^2 with gx, gy multiples
// of 1/8 in [-127.5, 127.5] (u8 input, OpenCV Sobel ksize 3 scale 1/8), so
// s = N / 64 for integer N in [0, 2 * 1020^2]. Compares, for every such N, the
// correctly rounded sqrtf with (a) the raw v_sqrt_f32 and (b) dis::sqrt_cr
// (v_sqrt_f32 + one-ulp correction without the denormal scaling, as the
// pyramid kernel uses it on sqrtf(N) and then scales by 1/8); prints counts.
#include <hip/hip_runtime.h>
#include <cstdio>

#include "../optical-flow-using-dense-inverse-search_amd/csrc/dis_device.h"

__global__ void k_check(int nmax, unsigned int* bad, int* first)
{
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n > nmax) return;
    const float s = (float)n * 0.015625f;  // exact: n < 2^22
    const float ref = sqrtf(s);
    const float a = __builtin_amdgcn_sqrtf(s);
    const float b = dis::sqrt_cr((float)n) * 0.125f;  // the pyramid's form
    if (__float_as_uint(a) != __float_as_uint(ref)) {
        atomicAdd(&bad[0], 1u);
        atomicMin(&first[0], n);
    }
    if (__float_as_uint(b) != __float_as_uint(ref)) {
        atomicAdd(&bad[1], 1u);
        atomicMin(&first[1], n);
    }
}

int main()
{
    const int nmax = 2 * 1020 * 1020;
    unsigned int* bad;
    int* first;
    if (hipMalloc(&bad, 8) != hipSuccess || hipMalloc(&first, 8) != hipSuccess) return 2;
    const int big[2] = {0x7fffffff, 0x7fffffff};
    if (hipMemset(bad, 0, 8) != hipSuccess || hipMemcpy(first, big, 8, hipMemcpyHostToDevice) != hipSuccess) return 2;
    hipLaunchKernelGGL(k_check, dim3((nmax + 256) / 256), dim3(256), 0, 0, nmax, bad, first);
    unsigned int hb[2] = {0, 0};
    int hf[2] = {0, 0};
    if (hipMemcpy(hb, bad, 8, hipMemcpyDeviceToHost) != hipSuccess || hipMemcpy(hf, first, 8, hipMemcpyDeviceToHost) != hipSuccess)
        return 2;
    printf("sqrt_check: %d inputs; raw v_sqrt_f32: %u mismatches (first N = %d); sqrt_cr: %u mismatches (first N = %d)\n",
           nmax + 1, hb[0], hb[0] ? hf[0] : -1, hb[1], hb[1] ? hf[1] : -1);
    return hb[1] ? 1 : 0;
}
