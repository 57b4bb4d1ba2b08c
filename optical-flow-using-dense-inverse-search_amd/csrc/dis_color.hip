// dis_color.hip -- Middlebury flow colour coding:
// draw_optical_flow / compute_color, src/color_coding.cpp:13-117.
//
// Per chunk of fields, two passes over a batch of n W x H (u,v) fields:
// the motion range (maxrad = max(1, max |u| over valid pixels), :88-104; kept
// as the largest squared radius, sqrtf taken once: sqrtf is monotone) and
// then every pixel to BGR u8 (:106-115; invalid pixels stay black), the
// colour pass of one chunk in the same launch as the max pass of the next
// (k_color_step). The float expressions are the reference's, in its order,
// -ffp-contract=off; the divisions and square roots are correctly rounded
// (the field's division through its reciprocal, div_pre; atan2's min/max
// quotient and the radius through the IEEE sequences' cores on the operand
// ranges where those are exact, the IEEE operations elsewhere): the same
// bits. The one library call, atan2f (:52), is restated as a fixed float
// algorithm (range reduction to [0, 1] + the minimax polynomial of ARM's
// optimized-routines atanf, <= 3 ulp) evaluated identically here and in the
// oracle. (The reference's MSVC atan2f is unknown: unpinned.)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>

#include "dis_abi.h"
#include "dis_common.h"
#include "dis_device.h"

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

// a / b and sqrtf(x), correctly rounded on their fast domains, through the
// IEEE sequences' cores (dis_device.h div_core / sqrt_core); kFast: that core,
// clearing `ok` outside its domain (the caller then recomputes the pixel the
// IEEE way); otherwise the IEEE operation
template <bool kFast>
__device__ __forceinline__ float div_rn(float a, float b, bool& ok)
{
    if constexpr (!kFast) return a / b;
    ok = ok && div_core_ok(a, b);
    return div_core(a, b);
}

template <bool kFast>
__device__ __forceinline__ float sqrt_rn(float x, bool& ok)
{
    if constexpr (!kFast) return sqrtf(x);
    ok = ok && sqrt_core_ok(x);
    return sqrt_core(x);
}

// atan2(y, x) for finite y, x: t = min/max in [0, 1], atan(t) = t + t z P(z),
// z = t^2 (ARM optimized-routines atanf coefficients), then the octant fix-up.
template <bool kFast>
__device__ __forceinline__ float atan2_dis(float y, float x, bool& ok)
{
    const float ax = fabsf(x), ay = fabsf(y);
    const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
    bool okd = true;
    const float q = div_rn<kFast>(mn, mx, okd);
    ok = ok && (okd || !(mx > 0.0f));
    const float t = mx > 0.0f ? q : 0.0f;
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
    return fabsf(x) < 1e9f && fabsf(y) < 1e9f;  // a NaN fails the compare: !isnan(x) && ... implied
}

constexpr int kMaxStride = 32;  // per field: [0] max radius bits (one 128-B line per field)
constexpr int kThreads = 256;
constexpr int kBG = 4;               // colour item: kBG groups of 4 consecutive pixels per lane
constexpr int kBpx = kThreads * 4 * kBG;  // pixels per colour item

// u / m correctly rounded for a per-field divisor m given rm = RN(1/m)
// (div_pre, dis_device.h), on the domain where its remainders cannot
// underflow or overflow: m in [2^-60, 2^60] (uniform: checked once per field)
// and |u| >= 2^-60 (or 0); anything else takes the IEEE division.
__device__ __forceinline__ float div_field(float u, float m, float rm, bool fast)
{
    return (fast && (fabsf(u) >= 0x1p-60f || u == 0.0f)) ? div_pre(u, m, rm) : u / m;
}

// One pixel: draw_optical_flow's per-pixel body (src/color_coding.cpp:106-115)
// with compute_color (:13-79) -> packed B | G << 8 | R << 16 (0 when invalid:
// dst.setTo(0), :87). `col` = the wheel as floats (c_wheel / 255.f, the same
// IEEE quotients the reference forms per pixel).
// kFast: the division and sqrt fast paths above, `ok` cleared when an operand
// is outside their domain (the caller then recomputes the pixel with
// kFast = false: the IEEE operations, the same bits either way)
template <bool kFast>
__device__ __forceinline__ unsigned color_px(float2 u, float maxrad, float rmax, bool fast, const float4* col, bool& ok)
{
    if (!flow_ok(u.x, u.y)) return 0u;
    const float fx = div_field(u.x, maxrad, rmax, fast), fy = div_field(u.y, maxrad, rmax, fast);  // (:113)
    const float rad = sqrt_rn<kFast>(fx * fx + fy * fy, ok);
    // atan2(...) / (float)CV_PI, correctly rounded through RN(1 / pi) (div_pre)
    // on its domain, the IEEE division for |t| < 2^-60
    constexpr float kPi = 3.14159274f, kRPi = 1.0f / kPi;
    const float t = atan2_dis<kFast>(-fy, -fx, ok);
    const float a = div_field(t, kPi, kRPi, true);
    const float fk = (a + 1.0f) / 2.0f * (float)(kNCols - 1);
    const int k0 = (int)fk;
    const int k1 = k0 + 1 == kNCols ? 0 : k0 + 1;  // (k0 + 1) % ncols, k0 in [0, ncols - 1]
    const float f = fk - (float)k0;
    unsigned o = 0;
    const float4 w0 = col[k0], w1 = col[k1];  // (r, g, b) of the two wheel entries
#pragma unroll
    for (int b = 0; b < 3; ++b) {
        const float c0 = b == 0 ? w0.x : b == 1 ? w0.y : w0.z, c1 = b == 0 ? w1.x : b == 1 ? w1.y : w1.z;
        float c = (1 - f) * c0 + f * c1;
        if (rad <= 1)
            c = 1 - rad * (1 - c);  // increase saturation with radius
        else
            c *= .75f;  // out of range (.75 is exact: same as the double multiply)
        o |= (unsigned)(uint8_t)(255.f * c) << (8 * (2 - b));  // BGR: channel b (r, g, b) at byte 2 - b
    }
    return o;
}

// Two kernels per chunk of fields, the chunk sized so that its flow stays in
// the 256 MiB Infinity Cache between them (a chunk's fields ~128 MB): the max
// pass reads the flow from HBM, the colour pass re-reads it from the cache, so
// the flow crosses HBM about once. (A single persistent launch with a work
// queue -- max-pass and colour items claimed through an atomic ticket, colour
// items of field f waiting for f's max -- measured 2.1 ms per 32 1080p fields
// against 0.51 ms for the r03 two-kernel form: not kept.)
struct ColorArgs {
    const float2* flow;  // the chunk's first field
    uint8_t* bgr;        // its first image
    unsigned int* ws;    // kMaxStride per field of the chunk: [0] max radius bits
    long long npix;
    float maxmotion;     // > 0: fixed range (ws unused)
    int vec;             // float4 loads / dwordx3 stores (npix % 4 == 0, aligned pointers)
};

// grid (blocks, fields): the valid-pixel max squared radius of each field
// (:88-104; the colour pass takes its sqrtf), reduced per workgroup into one
// float-bit atomicMax (a max is order-independent: exact; squares are >= +0,
// so their bit patterns order like the values)
__device__ __forceinline__ void color_max(const ColorArgs& a, int bx, int nbx, int f)
{
    __shared__ float red[kThreads / 64];
    const float2* fl = a.flow + (size_t)f * a.npix;
    float m = 0.0f;
    const long long step = 2LL * kThreads * nbx;
    for (long long i = 2LL * ((long long)bx * kThreads + threadIdx.x); i < a.npix; i += step) {
        if (a.vec && i + 2 <= a.npix) {
            const float4 u = *reinterpret_cast<const float4*>(fl + i);
            if (flow_ok(u.x, u.y)) m = fmaxf(m, u.x * u.x + u.y * u.y);  // (:101), squared
            if (flow_ok(u.z, u.w)) m = fmaxf(m, u.z * u.z + u.w * u.w);
        } else {
            for (long long q = i; q < i + 2 && q < a.npix; ++q) {
                const float2 u = fl[q];
                if (flow_ok(u.x, u.y)) m = fmaxf(m, u.x * u.x + u.y * u.y);
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0)
        atomicMax(&a.ws[(size_t)kMaxStride * f], __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
}

// grid (ceil(npix / kBpx), fields): each lane colours kBG groups of 4
// consecutive pixels, all its loads in flight before any is consumed
__device__ __forceinline__ void color_pixels(const ColorArgs& a, int bx, int f)
{
    __shared__ float4 col[kNCols];  // the wheel as floats, one 16-byte entry per colour
    for (int i = threadIdx.x; i < kNCols; i += kThreads)
        col[i] = make_float4((float)c_wheel.rgb[i][0] / 255.f, (float)c_wheel.rgb[i][1] / 255.f,
                             (float)c_wheel.rgb[i][2] / 255.f, 0.0f);
    __syncthreads();
    const float2* fl = a.flow + (size_t)f * a.npix;
    // maxrad = maxmotion, or max(1, max radius) when maxmotion <= 0 (:88-104)
    // (the max pass keeps the largest squared radius: sqrtf is monotone, so
    // sqrtf of it is the largest radius, :101, bit for bit)
    const float maxrad =
        a.maxmotion > 0.0f ? a.maxmotion : fmaxf(1.0f, sqrtf(__uint_as_float(a.ws[(size_t)kMaxStride * f])));
    const bool fast = maxrad >= 0x1p-60f && maxrad <= 0x1p60f;
    const float rmax = 1.0f / maxrad;
    const long long pb = (long long)bx * kBpx + 4 * threadIdx.x;
    uint8_t* const out = a.bgr + (size_t)f * a.npix * 3;
    if (a.vec && pb + 4 * kThreads * (kBG - 1) + 4 <= a.npix) {
        float4 v[kBG][2];
#pragma unroll
        for (int g = 0; g < kBG; ++g) {
            const long long p0 = pb + 4 * kThreads * g;
            v[g][0] = *reinterpret_cast<const float4*>(fl + p0);
            v[g][1] = *reinterpret_cast<const float4*>(fl + p0 + 2);
        }
#pragma unroll
        for (int g = 0; g < kBG; ++g) {
            const long long p0 = pb + 4 * kThreads * g;
            bool ok = true;
            unsigned c0 = color_px<true>(make_float2(v[g][0].x, v[g][0].y), maxrad, rmax, fast, col, ok);
            unsigned c1 = color_px<true>(make_float2(v[g][0].z, v[g][0].w), maxrad, rmax, fast, col, ok);
            unsigned c2 = color_px<true>(make_float2(v[g][1].x, v[g][1].y), maxrad, rmax, fast, col, ok);
            unsigned c3 = color_px<true>(make_float2(v[g][1].z, v[g][1].w), maxrad, rmax, fast, col, ok);
            if (__builtin_expect(!ok, 0)) {  // an operand outside the fast domain: the IEEE operations
                c0 = color_px<false>(make_float2(v[g][0].x, v[g][0].y), maxrad, rmax, fast, col, ok);
                c1 = color_px<false>(make_float2(v[g][0].z, v[g][0].w), maxrad, rmax, fast, col, ok);
                c2 = color_px<false>(make_float2(v[g][1].x, v[g][1].y), maxrad, rmax, fast, col, ok);
                c3 = color_px<false>(make_float2(v[g][1].z, v[g][1].w), maxrad, rmax, fast, col, ok);
            }
            // 4 pixels x 3 bytes, little-endian: c0 | c1 << 24, c1 >> 8 | c2 << 16, c2 >> 16 | c3 << 8
            *reinterpret_cast<uint3*>(out + p0 * 3) =
                make_uint3(c0 | (c1 << 24), (c1 >> 8) | (c2 << 16), (c2 >> 16) | (c3 << 8));
        }
    } else {
        for (int g = 0; g < kBG; ++g) {
            const long long p0 = pb + 4 * kThreads * g;
            for (long long q = p0; q < p0 + 4 && q < a.npix; ++q) {
                bool ok = true;
                const unsigned c = color_px<false>(fl[q], maxrad, rmax, fast, col, ok);
                out[q * 3] = (uint8_t)c;
                out[q * 3 + 1] = (uint8_t)(c >> 8);
                out[q * 3 + 2] = (uint8_t)(c >> 16);
            }
        }
    }
}

__global__ void __launch_bounds__(kThreads) k_color_px(ColorArgs a) { color_pixels(a, blockIdx.x, blockIdx.y); }

// One launch per chunk of fields: the colour pass of chunk k (blocks x <
// npx_b, its maxima computed by the previous launch) beside the max pass of
// chunk k + 1 (the other blocks): no dependency inside the launch, so the
// colour pass's arithmetic and the max pass's reads overlap, and chunk k's
// flow, read by the max pass one launch earlier, is re-read from the cache.
struct ColorStep {
    ColorArgs px, mx;
    int npx_b, nmx_b;  // blocks per field of each role
    int npx_f, nmx_f;  // fields of each role (0: role absent)
};

__global__ void __launch_bounds__(kThreads) k_color_step(ColorStep c)
{
    const int x = blockIdx.x, f = blockIdx.y;
    if (x < c.npx_b) {
        if (f < c.npx_f) color_pixels(c.px, x, f);
    } else if (f < c.nmx_f) {
        color_max(c.mx, x - c.npx_b, c.nmx_b, f);
    }
}

}  // namespace

hipError_t launch_flow_color(const float* flow, int n, int W, int H, float maxmotion, uint8_t* bgr,
                             unsigned int* ws, hipStream_t s)
{
    ColorArgs a{};
    a.npix = (long long)W * H;
    a.maxmotion = maxmotion;
    a.vec = a.npix % 4 == 0 && (reinterpret_cast<uintptr_t>(bgr) & 3) == 0 && (reinterpret_cast<uintptr_t>(flow) & 15) == 0;
    const unsigned bx = (unsigned)((a.npix + kBpx - 1) / kBpx);
    if (maxmotion > 0.0f) {  // fixed range: one colour pass over every field
        a.flow = reinterpret_cast<const float2*>(flow);
        a.bgr = bgr;
        a.ws = ws;
        hipLaunchKernelGGL(k_color_px, dim3(bx, n), dim3(kThreads), 0, s, a);
        return hipGetLastError();
    }
    hipError_t e = hipMemsetAsync(ws, 0, sizeof(unsigned int) * kMaxStride * (size_t)n, s);
    if (e != hipSuccess) return e;
    // fields per chunk: ~128 MB of flow, re-read from the Infinity Cache
    const long long fbytes = a.npix * 8;
    // (r04 A/B, 32 x 1080p fields: 32 / 64 / 128 MB chunks 0.41 / 0.36-0.38 / 0.32-0.34 ms)
    constexpr long long kChunkBytes = 128LL << 20;
    const int chunk = (int)std::max<long long>(1, std::min<long long>(n, kChunkBytes / std::max(1LL, fbytes)));
    const unsigned mb = (unsigned)std::min<long long>(256, (a.npix + 2LL * kThreads * 8 - 1) / (2LL * kThreads * 8));
    auto chunk_args = [&](int f0) {
        ColorArgs c = a;
        c.flow = reinterpret_cast<const float2*>(flow) + (size_t)f0 * a.npix;
        c.bgr = bgr + (size_t)f0 * a.npix * 3;
        c.ws = ws + (size_t)kMaxStride * f0;
        return c;
    };
    // launch j: colour pass of chunk j - 1 and max pass of chunk j
    const int nch = (n + chunk - 1) / chunk;
    for (int j = 0; j <= nch; ++j) {
        ColorStep c{};
        if (j > 0) {
            c.px = chunk_args((j - 1) * chunk);
            c.npx_b = (int)bx;
            c.npx_f = std::min(chunk, n - (j - 1) * chunk);
        }
        if (j < nch) {
            c.mx = chunk_args(j * chunk);
            c.nmx_b = (int)mb;
            c.nmx_f = std::min(chunk, n - j * chunk);
        }
        const dim3 grid((unsigned)(c.npx_b + c.nmx_b), (unsigned)std::max(c.npx_f, c.nmx_f));
        hipLaunchKernelGGL(k_color_step, grid, dim3(kThreads), 0, s, c);
    }
    return hipGetLastError();
}

size_t flow_color_ws_words(int n) { return (size_t)kMaxStride * n; }

}  // namespace dis
