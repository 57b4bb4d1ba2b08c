// dis_color.hip -- Middlebury flow colour coding:
// draw_optical_flow / compute_color, src/color_coding.cpp:13-117.
//
// Two kernels over a batch of n W x H (u,v) fields: k_color_maxrad reduces the
// motion range (maxrad = max(1, max |u| over valid pixels), :88-104, a max is
// order-independent, so the float-bit atomicMax is exact) and k_color_pixels
// maps every pixel to BGR u8 (:106-115; invalid pixels stay black). The float
// expressions are the reference's, in its order, -ffp-contract=off; the one
// library call, atan2f (:52), is evaluated as the double atan2 rounded to
// float on both sides (kernel and oracle), i.e. correctly rounded in practice.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "dis_abi.h"
#include "dis_common.h"

namespace dis {

namespace {

constexpr int kRY = 15, kYG = 6, kGC = 4, kCB = 11, kBM = 13, kMR = 6;
constexpr int kNCols = kRY + kYG + kGC + kCB + kBM + kMR;  // 55 (:23-29)

struct Wheel {
    int rgb[kNCols][3];
};

// the static colour wheel (src/color_coding.cpp:31-56), integer division as there
Wheel make_wheel()
{
    Wheel w{};
    int k = 0;
    auto set = [&](int r, int g, int b) {
        w.rgb[k][0] = r;
        w.rgb[k][1] = g;
        w.rgb[k][2] = b;
        ++k;
    };
    for (int i = 0; i < kRY; ++i) set(255, 255 * i / kRY, 0);
    for (int i = 0; i < kYG; ++i) set(255 - 255 * i / kYG, 255, 0);
    for (int i = 0; i < kGC; ++i) set(0, 255, 255 * i / kGC);
    for (int i = 0; i < kCB; ++i) set(0, 255 - 255 * i / kCB, 255);
    for (int i = 0; i < kBM; ++i) set(255 * i / kBM, 0, 255);
    for (int i = 0; i < kMR; ++i) set(255, 0, 255 - 255 * i / kMR);
    return w;
}

// is_flow_correct (src/color_coding.cpp:8-11)
__device__ __forceinline__ bool flow_ok(float x, float y)
{
    return !(x != x) && !(y != y) && fabsf(x) < 1e9f && fabsf(y) < 1e9f;
}

// grid (ceil(W*H / 256), n): per-pair max radius as float bits (all >= 0)
__global__ void __launch_bounds__(256) k_color_maxrad(const float2* flow, long long npix, unsigned int* maxbits)
{
    const int pair = blockIdx.y;
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    float m = 0.0f;
    if (i < npix) {
        const float2 u = flow[(size_t)pair * npix + i];
        if (flow_ok(u.x, u.y)) m = sqrtf(u.x * u.x + u.y * u.y);  // (:101)
    }
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) atomicMax(&maxbits[pair], __float_as_uint(m));
}

__global__ void __launch_bounds__(256) k_color_pixels(const float2* flow, long long npix, float maxmotion,
                                                      const unsigned int* maxbits, Wheel w, uint8_t* bgr)
{
    const int pair = blockIdx.y;
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= npix) return;
    // maxrad = maxmotion, or max(1, max radius) when maxmotion <= 0 (:88-104)
    const float maxrad = maxmotion > 0.0f ? maxmotion : fmaxf(1.0f, __uint_as_float(maxbits[pair]));
    const float2 u = flow[(size_t)pair * npix + i];
    uint8_t* px = bgr + ((size_t)pair * npix + i) * 3;
    if (!flow_ok(u.x, u.y)) {  // dst.setTo(0) (:87)
        px[0] = px[1] = px[2] = 0;
        return;
    }
    // compute_color(u.x / maxrad, u.y / maxrad) (:113, :13-79)
    const float fx = u.x / maxrad, fy = u.y / maxrad;
    const float rad = sqrtf(fx * fx + fy * fy);
    const float a = (float)atan2(-(double)fy, -(double)fx) / 3.14159274f;  // (float)CV_PI
    const float fk = (a + 1.0f) / 2.0f * (float)(kNCols - 1);
    const int k0 = (int)fk;
    const int k1 = (k0 + 1) % kNCols;
    const float f = fk - (float)k0;
    for (int b = 0; b < 3; ++b) {
        const float col0 = (float)w.rgb[k0][b] / 255.f;
        const float col1 = (float)w.rgb[k1][b] / 255.f;
        float col = (1 - f) * col0 + f * col1;
        if (rad <= 1)
            col = 1 - rad * (1 - col);  // increase saturation with radius
        else
            col *= .75f;  // out of range (.75 is exact: same as the double multiply)
        px[2 - b] = (uint8_t)(255.f * col);
    }
}

}  // namespace

hipError_t launch_flow_color(const float* flow, int n, int W, int H, float maxmotion, uint8_t* bgr,
                             unsigned int* maxbits, hipStream_t s)
{
    static const Wheel wheel = make_wheel();
    const long long npix = (long long)W * H;
    dim3 grid((unsigned)((npix + 255) / 256), n);
    hipError_t e = hipMemsetAsync(maxbits, 0, sizeof(unsigned int) * n, s);
    if (e != hipSuccess) return e;
    if (maxmotion <= 0.0f)
        hipLaunchKernelGGL(k_color_maxrad, grid, dim3(256), 0, s, reinterpret_cast<const float2*>(flow), npix,
                           maxbits);
    hipLaunchKernelGGL(k_color_pixels, grid, dim3(256), 0, s, reinterpret_cast<const float2*>(flow), npix, maxmotion,
                       maxbits, wheel, bgr);
    return hipGetLastError();
}

}  // namespace dis
