// Scalar-load latency probe (experiment): clocks of one dependent s_load from
// the kernarg segment vs from a device buffer, per workgroup, with and without
// a concurrent HBM-streaming kernel.
//   hipcc --offload-arch=gfx950 -O3 tools/karg_probe.hip -o tools/karg_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

struct Args {
    const unsigned* buf;
    unsigned long long* out;
    unsigned pad[60];
};

__global__ void k_probe(Args a)
{
    if (threadIdx.x != 0) return;
    auto kp = __builtin_amdgcn_kernarg_segment_ptr();
    unsigned long long t0, t1, t2, t3;
    unsigned v0, v1, v2;
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t0));
    asm volatile("s_load_dword %0, %1, 0xf0\n s_waitcnt lgkmcnt(0)" : "=s"(v0) : "s"(kp));
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t1));
    asm volatile("s_load_dword %0, %1, 0x0\n s_waitcnt lgkmcnt(0)" : "=s"(v1) : "s"(a.buf + blockIdx.x * 64));
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t2));
    asm volatile("s_load_dword %0, %1, 0xf4\n s_waitcnt lgkmcnt(0)" : "=s"(v2) : "s"(kp));
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t3));
    unsigned long long* o = a.out + blockIdx.x * 4;
    o[0] = t1 - t0;
    o[1] = t2 - t1;
    o[2] = t3 - t2;
    o[3] = v0 + v1 + v2;
}

__global__ void k_stream(const float4* in, float4* out, size_t n)
{
    for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        out[i] = in[i];
}

static void report(const char* tag, std::vector<unsigned long long>& h, int nb)
{
    const char* nm[3] = {"kernarg (first)", "device buffer", "kernarg (again)"};
    for (int k = 0; k < 3; ++k) {
        std::vector<double> d(nb);
        for (int i = 0; i < nb; ++i) d[i] = (double)h[4 * i + k];
        std::sort(d.begin(), d.end());
        printf("%-12s %-16s p10 %6.0f p50 %6.0f p90 %6.0f max %6.0f clk\n", tag, nm[k], d[nb / 10], d[nb / 2],
               d[9 * nb / 10], d[nb - 1]);
    }
}

int main()
{
    const int nb = 4096;
    Args a{};
    unsigned* buf;
    hipMalloc(&buf, nb * 256);
    hipMemset(buf, 0, nb * 256);
    a.buf = buf;
    hipMalloc(&a.out, nb * 4 * sizeof(unsigned long long));
    std::vector<unsigned long long> h(nb * 4);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k_probe, dim3(nb), dim3(64), 0, 0, a);
    hipDeviceSynchronize();
    hipMemcpy(h.data(), a.out, h.size() * 8, hipMemcpyDeviceToHost);
    report("idle", h, nb);
    // under HBM load: a streaming copy on another stream
    const size_t n = (size_t)1 << 26;  // 1 GiB of float4 each way
    float4 *x, *y;
    hipMalloc(&x, n * 16);
    hipMalloc(&y, n * 16);
    hipStream_t s2;
    hipStreamCreate(&s2);
    hipLaunchKernelGGL(k_stream, dim3(4096), dim3(256), 0, s2, x, y, n);
    for (int r = 0; r < 20; ++r) hipLaunchKernelGGL(k_probe, dim3(nb), dim3(64), 0, 0, a);
    hipDeviceSynchronize();
    hipMemcpy(h.data(), a.out, h.size() * 8, hipMemcpyDeviceToHost);
    report("hbm-loaded", h, nb);
    return 0;
}
