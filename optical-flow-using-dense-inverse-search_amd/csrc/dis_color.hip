// dis_color.hip -- Middlebury flow colour coding:
// draw_optical_flow / compute_color, src/color_coding.cpp:13-117.
//
// Two kernels over a batch of n W x H (u,v) fields: k_color_maxrad reduces the
// motion range (maxrad = max(1, max |u| over valid pixels), :88-104, a max is
// order-independent, so the float-bit atomicMax is exact) and k_color_pixels
// maps every pixel to BGR u8 (:106-115; invalid pixels stay black). The float
// expressions are the reference's, in its order, -ffp-contract=off; the one
// library call, atan2f (:52), is restated as a fixed float algorithm (range
// reduction to [0, 1] + the minimax polynomial of ARM's optimized-routines
// atanf, <= 3 ulp) evaluated identically here and in the oracle. (The
// reference's MSVC atan2f is unknown: unpinned.)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>

#include "dis_abi.h"
#include "dis_common.h"

namespace dis {

namespace {

constexpr int kRY = 15, kYG = 6, kGC = 4, kCB = 11, kBM = 13, kMR = 6;
constexpr int kNCols = kRY + kYG + kGC + kCB + kBM + kMR;  // 55 (:23-29)

// the static colour wheel (src/color_coding.cpp:31-56), integer division as
// there, as a constant table: entry k = (r, g, b)
struct Wheel {
    int rgb[kNCols][3];
};

constexpr Wheel make_wheel()
{
    Wheel w{};
    int k = 0;
    for (int i = 0; i < kRY; ++i, ++k) w.rgb[k][0] = 255, w.rgb[k][1] = 255 * i / kRY, w.rgb[k][2] = 0;
    for (int i = 0; i < kYG; ++i, ++k) w.rgb[k][0] = 255 - 255 * i / kYG, w.rgb[k][1] = 255, w.rgb[k][2] = 0;
    for (int i = 0; i < kGC; ++i, ++k) w.rgb[k][0] = 0, w.rgb[k][1] = 255, w.rgb[k][2] = 255 * i / kGC;
    for (int i = 0; i < kCB; ++i, ++k) w.rgb[k][0] = 0, w.rgb[k][1] = 255 - 255 * i / kCB, w.rgb[k][2] = 255;
    for (int i = 0; i < kBM; ++i, ++k) w.rgb[k][0] = 255 * i / kBM, w.rgb[k][1] = 0, w.rgb[k][2] = 255;
    for (int i = 0; i < kMR; ++i, ++k) w.rgb[k][0] = 255, w.rgb[k][1] = 0, w.rgb[k][2] = 255 - 255 * i / kMR;
    return w;
}

__constant__ Wheel c_wheel = make_wheel();  // read-only table: scalar/constant cache loads

// atan2(y, x) for finite y, x: t = min/max in [0, 1], atan(t) = t + t z P(z),
// z = t^2 (ARM optimized-routines atanf coefficients), then the octant fix-up.
__device__ __forceinline__ float atan2_dis(float y, float x)
{
    const float ax = fabsf(x), ay = fabsf(y);
    const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
    const float t = mx > 0.0f ? mn / mx : 0.0f;
    const float z = t * t;
    float p = 0x1.01fd88p-8f;
    p = p * z + -0x1.4c3c60p-6f;
    p = p * z + 0x1.93a2c0p-5f;
    p = p * z + -0x1.491f0ep-4f;
    p = p * z + 0x1.bd7368p-4f;
    p = p * z + -0x1.24051ep-3f;
    p = p * z + 0x1.99935ep-3f;
    p = p * z + -0x1.55555p-2f;
    float r = t + (t * z) * p;
    if (ay > ax) r = 1.57079637f - r;  // pi/2
    if (x < 0.0f || (x == 0.0f && __float_as_int(x) < 0)) r = 3.14159274f - r;  // pi
    return __float_as_int(y) < 0 ? -r : r;
}

// is_flow_correct (src/color_coding.cpp:8-11)
__device__ __forceinline__ bool flow_ok(float x, float y)
{
    return !(x != x) && !(y != y) && fabsf(x) < 1e9f && fabsf(y) < 1e9f;
}

constexpr int kMaxStride = 32;  // maxbits[pair * 32]: one 128-B line per pair (no false sharing)
constexpr int kMaxBlocks = 128;  // reduction workgroups per pair (one atomic each)

// grid (kMaxBlocks, n): per-pair max radius as float bits (all >= 0); each
// workgroup strides over the pair's pixels, reduces in-wave then across its
// 4 waves in LDS, and issues one atomicMax
__global__ void __launch_bounds__(256) k_color_maxrad(const float2* flow, long long npix, unsigned int* maxbits)
{
    __shared__ float red[4];
    const int pair = blockIdx.y;
    const float2* f = flow + (size_t)pair * npix;
    float m = 0.0f;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < npix; i += (long long)gridDim.x * 256) {
        const float2 u = f[i];
        if (flow_ok(u.x, u.y)) m = fmaxf(m, sqrtf(u.x * u.x + u.y * u.y));  // (:101)
    }
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
        atomicMax(&maxbits[pair * kMaxStride], __float_as_uint(m));
    }
}

__global__ void __launch_bounds__(256) k_color_pixels(const float2* flow, long long npix, float maxmotion,
                                                      const unsigned int* maxbits, uint8_t* bgr)
{
    const int pair = blockIdx.y;
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= npix) return;
    // maxrad = maxmotion, or max(1, max radius) when maxmotion <= 0 (:88-104)
    const float maxrad = maxmotion > 0.0f ? maxmotion : fmaxf(1.0f, __uint_as_float(maxbits[pair * kMaxStride]));
    const float2 u = flow[(size_t)pair * npix + i];
    uint8_t* px = bgr + ((size_t)pair * npix + i) * 3;
    if (!flow_ok(u.x, u.y)) {  // dst.setTo(0) (:87)
        px[0] = px[1] = px[2] = 0;
        return;
    }
    // compute_color(u.x / maxrad, u.y / maxrad) (:113, :13-79)
    const float fx = u.x / maxrad, fy = u.y / maxrad;
    const float rad = sqrtf(fx * fx + fy * fy);
    const float a = atan2_dis(-fy, -fx) / 3.14159274f;  // (float)CV_PI
    const float fk = (a + 1.0f) / 2.0f * (float)(kNCols - 1);
    const int k0 = (int)fk;
    const int k1 = (k0 + 1) % kNCols;
    const float f = fk - (float)k0;
    uint8_t o[3];
#pragma unroll
    for (int b = 0; b < 3; ++b) {
        const float col0 = (float)c_wheel.rgb[k0][b] / 255.f;
        const float col1 = (float)c_wheel.rgb[k1][b] / 255.f;
        float col = (1 - f) * col0 + f * col1;
        if (rad <= 1)
            col = 1 - rad * (1 - col);  // increase saturation with radius
        else
            col *= .75f;  // out of range (.75 is exact: same as the double multiply)
        o[2 - b] = (uint8_t)(255.f * col);
    }
    px[0] = o[0];
    px[1] = o[1];
    px[2] = o[2];
}

}  // namespace

hipError_t launch_flow_color(const float* flow, int n, int W, int H, float maxmotion, uint8_t* bgr,
                             unsigned int* maxbits, hipStream_t s)
{
    const long long npix = (long long)W * H;
    hipError_t e = hipMemsetAsync(maxbits, 0, sizeof(unsigned int) * kMaxStride * n, s);
    if (e != hipSuccess) return e;
    if (maxmotion <= 0.0f) {
        const dim3 g((unsigned)std::min<long long>(kMaxBlocks, (npix + 255) / 256), n);
        hipLaunchKernelGGL(k_color_maxrad, g, dim3(256), 0, s, reinterpret_cast<const float2*>(flow), npix, maxbits);
    }
    const dim3 grid((unsigned)((npix + 255) / 256), n);
    hipLaunchKernelGGL(k_color_pixels, grid, dim3(256), 0, s, reinterpret_cast<const float2*>(flow), npix, maxmotion,
                       maxbits, bgr);
    return hipGetLastError();
}

}  // namespace dis
