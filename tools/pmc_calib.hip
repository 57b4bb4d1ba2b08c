// pmc_calib.hip -- calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for
// the access widths the DIS kernels use (MI355X_MICROARCH.md: FETCH_SIZE is
// exact only after calibration for non-16-B loads). Reads a 512 MiB buffer
// (past the 256 MiB Infinity Cache) once per kernel with 1-, 4- and 16-byte
// coalesced loads and writes 512 MiB with 4- and 8-byte stores; prints the
// known byte counts so the PMC rows can be divided by them.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void rd_u8(const unsigned char* p, size_t n, unsigned* out)
{
    unsigned s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += p[i];
    if (s == 0xdeadbeef) out[0] = s;
}
__global__ void rd_u32(const unsigned* p, size_t n, unsigned* out)
{
    unsigned s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += p[i];
    if (s == 0xdeadbeef) out[0] = s;
}
__global__ void rd_u128(const uint4* p, size_t n, unsigned* out)
{
    unsigned s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint4 v = p[i];
        s += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (s == 0xdeadbeef) out[0] = s;
}
__global__ void wr_u32(unsigned* p, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = (unsigned)i;
}
__global__ void wr_f2(float2* p, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = make_float2((float)i, 1.f);
}

int main()
{
    const size_t bytes = 512ull << 20;
    void* buf;
    unsigned* out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    hipMemset(buf, 1, bytes);
    dim3 g(4096), b(256);
    hipLaunchKernelGGL(rd_u8, g, b, 0, 0, (const unsigned char*)buf, bytes, out);
    hipLaunchKernelGGL(rd_u32, g, b, 0, 0, (const unsigned*)buf, bytes / 4, out);
    hipLaunchKernelGGL(rd_u128, g, b, 0, 0, (const uint4*)buf, bytes / 16, out);
    hipLaunchKernelGGL(wr_u32, g, b, 0, 0, (unsigned*)buf, bytes / 4);
    hipLaunchKernelGGL(wr_f2, g, b, 0, 0, (float2*)buf, bytes / 8);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::printf("each kernel moves %zu bytes (%.1f KiB)\n", bytes, bytes / 1024.0);
    hipFree(buf);
    hipFree(out);
    return 0;
}
