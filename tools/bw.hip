// bw.hip -- achievable HBM bandwidth on this box (calibrates roofline claims):
// float4 streaming read, write and copy over 1 GiB buffers, hipEvent timing,
// best of 5.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4v __attribute__((ext_vector_type(4)));

__global__ void rd(const float4* p, size_t n, float* out)
{
    float s = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        float4 v = p[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1234.5f) out[0] = s;
}
__global__ void wr(float4* p, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}
__global__ void wr_nt(float4* p, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        __builtin_nontemporal_store((f4v){1.f, 2.f, 3.f, (float)i}, reinterpret_cast<f4v*>(p + i));
}
__global__ void wr_const(float4* p, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_float4(2.f, 2.f, 2.f, 2.f);
}
// one contiguous chunk per workgroup (each lane 16 B, the workgroup 4 KB per step)
__global__ void wr_chunk(float4* p, size_t n)
{
    const size_t per = n / gridDim.x;
    float4* q = p + blockIdx.x * per;
    for (size_t i = threadIdx.x; i < per; i += blockDim.x) q[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}
__global__ void wr_chunk_nt(float4* p, size_t n)
{
    const size_t per = n / gridDim.x;
    float4* q = p + blockIdx.x * per;
    for (size_t i = threadIdx.x; i < per; i += blockDim.x)
        __builtin_nontemporal_store((f4v){1.f, 2.f, 3.f, (float)i}, reinterpret_cast<f4v*>(q + i));
}
__global__ void cp(const float4* a, float4* b, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

int main()
{
    const size_t bytes = 1ull << 30, n = bytes / 16;
    float4 *a, *b;
    float* o;
    if (hipMalloc(&a, bytes) || hipMalloc(&b, bytes) || hipMalloc(&o, 64)) return 1;
    hipMemset(a, 0, bytes);
    hipMemset(b, 0, bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* names[8] = {"read", "write", "copy", "write-nt", "write-const", "write-chunk", "write-chunk-nt", "write-2k"};
    for (int k = 0; k < 8; ++k) {
        float best = 1e9f;
        for (int r = 0; r < 6; ++r) {
            hipEventRecord(e0, 0);
            if (k == 0) hipLaunchKernelGGL(rd, dim3(8192), dim3(256), 0, 0, a, n, o);
            if (k == 1) hipLaunchKernelGGL(wr, dim3(8192), dim3(256), 0, 0, b, n);
            if (k == 2) hipLaunchKernelGGL(cp, dim3(8192), dim3(256), 0, 0, a, b, n);
            if (k == 3) hipLaunchKernelGGL(wr_nt, dim3(8192), dim3(256), 0, 0, b, n);
            if (k == 4) hipLaunchKernelGGL(wr_const, dim3(8192), dim3(256), 0, 0, b, n);
            if (k == 5) hipLaunchKernelGGL(wr_chunk, dim3(8192), dim3(256), 0, 0, b, n);
            if (k == 6) hipLaunchKernelGGL(wr_chunk_nt, dim3(8192), dim3(256), 0, 0, b, n);
            if (k == 7) hipLaunchKernelGGL(wr, dim3(2048), dim3(256), 0, 0, b, n);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (r) best = ms < best ? ms : best;
        }
        const double moved = (k == 2 ? 2.0 : 1.0) * bytes;
        std::printf("%-5s %.3f ms  %.2f TB/s\n", names[k], best, moved / best / 1e9);
    }
    return 0;
}
