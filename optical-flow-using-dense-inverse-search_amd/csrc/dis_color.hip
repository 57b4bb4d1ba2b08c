// dis_color.hip -- Middlebury flow colour coding:
// draw_optical_flow / compute_color, src/color_coding.cpp:13-117.
//
// One persistent kernel over a batch of n W x H (u,v) fields (k_color, below):
// per field the motion range (maxrad = max(1, max |u| over valid pixels),
// :88-104) and then every pixel to BGR u8 (:106-115; invalid pixels stay
// black). The float expressions are the reference's, in its order,
// -ffp-contract=off (the division by maxrad correctly rounded through the
// field's reciprocal, div_pre: the same bits); the one
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

constexpr int kMaxStride = 32;  // per field: [0] max radius bits, [1] finished max-pass items (one 128-B line)
constexpr int kThreads = 256;
constexpr int kApx = kThreads * 64;  // pixels per max-pass item (each lane: 32 float4 = 64 vectors)
constexpr int kBG = 4;               // colour item: kBG groups of 4 consecutive pixels per lane
constexpr int kBpx = kThreads * 4 * kBG;  // pixels per colour item
constexpr int kClaim = 8;            // consecutive items per ticket (one atomic per kClaim items)

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
__device__ __forceinline__ unsigned color_px(float2 u, float maxrad, float rmax, bool fast, const float (*col)[3])
{
    if (!flow_ok(u.x, u.y)) return 0u;
    const float fx = div_field(u.x, maxrad, rmax, fast), fy = div_field(u.y, maxrad, rmax, fast);  // (:113)
    const float rad = sqrtf(fx * fx + fy * fy);
    const float a = atan2_dis(-fy, -fx) / 3.14159274f;  // (float)CV_PI
    const float fk = (a + 1.0f) / 2.0f * (float)(kNCols - 1);
    const int k0 = (int)fk;
    const int k1 = k0 + 1 == kNCols ? 0 : k0 + 1;  // (k0 + 1) % ncols, k0 in [0, ncols - 1]
    const float f = fk - (float)k0;
    unsigned o = 0;
#pragma unroll
    for (int b = 0; b < 3; ++b) {
        float c = (1 - f) * col[k0][b] + f * col[k1][b];
        if (rad <= 1)
            c = 1 - rad * (1 - c);  // increase saturation with radius
        else
            c *= .75f;  // out of range (.75 is exact: same as the double multiply)
        o |= (unsigned)(uint8_t)(255.f * c) << (8 * (2 - b));  // BGR: channel b (r, g, b) at byte 2 - b
    }
    return o;
}

// One persistent launch over a work list of max-pass items A(f) (per field,
// kApx pixels each: the valid-pixel max radius, :88-104, reduced per
// workgroup into one float-bit atomicMax -- a max is order-independent, so the
// result is exact) and colour items B(f) (kBpx pixels each), claimed in order,
// kClaim consecutive items per atomic ticket (one ticket per item was
// measured 10x slower: 97k atomics on one address serialise): A(0), A(1),
// B(0), A(2), B(1), ..., B(n-1). B(f) waits until every A(f) item has
// finished; all of them were claimed before it by running workgroups, which
// work through their claims in order and wait only for lower items, so the
// lowest unfinished item can always proceed. Field
// f's flow is re-read by B(f) one field after A(f) read it, from the L2 / MALL
// (16.6 MB per 1080p field) rather than HBM: the flow crosses HBM about once.
// With maxmotion > 0 there are no A items and no waits. Each colour lane reads
// its 4 pixels as two float4 and writes 12 bytes with one dwordx3 store when
// the field size and pointers allow (vec), else per pixel.
struct ColorArgs {
    const float2* flow;
    uint8_t* bgr;
    unsigned int* ws;  // kMaxStride per field (zeroed), then the ticket at [kMaxStride * n]
    long long npix;
    int n, na, nb;     // fields, A / B items per field (na = 0: fixed maxmotion)
    float maxmotion;
    int vec;
};

// work item t -> (max pass?, field, chunk) in the order A(0) | A(f+1), B(f) ... | B(n-1)
__device__ __forceinline__ void color_item(const ColorArgs& a, long long t, bool& isA, int& f, int& chunk)
{
    if (a.na == 0) {
        isA = false, f = (int)(t / a.nb), chunk = (int)(t % a.nb);
    } else if (t < a.na) {
        isA = true, f = 0, chunk = (int)t;
    } else {
        const long long r = t - a.na, per = a.na + a.nb;
        const int g = (int)(r / per), o = (int)(r % per);  // group g: A(g + 1) then B(g)
        if (g < a.n - 1) {
            isA = o < a.na, f = isA ? g + 1 : g, chunk = isA ? o : o - a.na;
        } else {
            isA = false, f = a.n - 1, chunk = (int)(r - (long long)(a.n - 1) * per);
        }
    }
}

__global__ void __launch_bounds__(kThreads) k_color(ColorArgs a)
{
    __shared__ float col[kNCols][3];
    __shared__ float red[kThreads / 64];
    __shared__ long long claim;
    for (int i = threadIdx.x; i < kNCols * 3; i += kThreads) col[i / 3][i % 3] = (float)c_wheel.rgb[i / 3][i % 3] / 255.f;
    const long long total = (long long)(a.na + a.nb) * a.n;
    unsigned int* const ticket = a.ws + (size_t)kMaxStride * a.n;
    for (;;) {
        __syncthreads();  // the previous claim's LDS use is over (and col is staged)
        // kClaim consecutive items per ticket, processed in order: every item
        // is owned by a running workgroup from the moment it is claimed
        if (threadIdx.x == 0) claim = (long long)atomicAdd(ticket, 1u) * kClaim;
        __syncthreads();
        const long long t0 = claim;
        if (t0 >= total) return;
        for (long long t = t0; t < t0 + kClaim && t < total; ++t) {
            int f, chunk;
            bool isA;
            color_item(a, t, isA, f, chunk);
            const float2* fl = a.flow + (size_t)f * a.npix;
            unsigned int* const fw = a.ws + (size_t)kMaxStride * f;
            if (isA) {
                float m = 0.0f;
                const long long p0 = (long long)chunk * kApx;
#pragma unroll 8
                for (int k = 0; k < kApx / (2 * kThreads); ++k) {
                    const long long i = p0 + 2 * (k * kThreads + threadIdx.x);  // 2 pixels per lane and step
                    if (a.vec && i + 2 <= a.npix) {
                        const float4 u = *reinterpret_cast<const float4*>(fl + i);
                        if (flow_ok(u.x, u.y)) m = fmaxf(m, sqrtf(u.x * u.x + u.y * u.y));  // (:101)
                        if (flow_ok(u.z, u.w)) m = fmaxf(m, sqrtf(u.z * u.z + u.w * u.w));
                    } else {
                        for (long long q = i; q < i + 2 && q < a.npix; ++q) {
                            const float2 u = fl[q];
                            if (flow_ok(u.x, u.y)) m = fmaxf(m, sqrtf(u.x * u.x + u.y * u.y));
                        }
                    }
                }
                for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
                __syncthreads();  // red[] of the previous item read
                if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
                __syncthreads();
                if (threadIdx.x == 0) {
                    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
                    atomicMax(&fw[0], __float_as_uint(m));
                    __hip_atomic_fetch_add(&fw[1], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                }
                continue;
            }
            // maxrad = maxmotion, or max(1, max radius) when maxmotion <= 0 (:88-104)
            float maxrad = a.maxmotion;
            if (a.na) {
                __syncthreads();  // red[] of the previous item read
                if (threadIdx.x == 0) {
                    while (__hip_atomic_load(&fw[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)a.na)
                        __builtin_amdgcn_s_sleep(2);
                    red[0] = fmaxf(1.0f, __uint_as_float(__hip_atomic_load(&fw[0], __ATOMIC_RELAXED,
                                                                           __HIP_MEMORY_SCOPE_AGENT)));
                }
                __syncthreads();
                maxrad = red[0];
            }
            const bool fast = maxrad >= 0x1p-60f && maxrad <= 0x1p60f;
            const float rmax = 1.0f / maxrad;
            const long long pb = (long long)chunk * kBpx + 4 * threadIdx.x;
            if (a.vec && pb + 4 * kThreads * (kBG - 1) + 4 <= a.npix) {
                float4 v[kBG][2];  // all the lane's loads in flight before any is consumed
#pragma unroll
                for (int g = 0; g < kBG; ++g) {
                    const long long p0 = pb + 4 * kThreads * g;
                    v[g][0] = *reinterpret_cast<const float4*>(fl + p0);
                    v[g][1] = *reinterpret_cast<const float4*>(fl + p0 + 2);
                }
#pragma unroll
                for (int g = 0; g < kBG; ++g) {
                    const long long p0 = pb + 4 * kThreads * g;
                    const unsigned c0 = color_px(make_float2(v[g][0].x, v[g][0].y), maxrad, rmax, fast, col);
                    const unsigned c1 = color_px(make_float2(v[g][0].z, v[g][0].w), maxrad, rmax, fast, col);
                    const unsigned c2 = color_px(make_float2(v[g][1].x, v[g][1].y), maxrad, rmax, fast, col);
                    const unsigned c3 = color_px(make_float2(v[g][1].z, v[g][1].w), maxrad, rmax, fast, col);
                    // 4 pixels x 3 bytes, little-endian: c0 | c1 << 24, c1 >> 8 | c2 << 16, c2 >> 16 | c3 << 8
                    *reinterpret_cast<uint3*>(a.bgr + ((size_t)f * a.npix + p0) * 3) =
                        make_uint3(c0 | (c1 << 24), (c1 >> 8) | (c2 << 16), (c2 >> 16) | (c3 << 8));
                }
            } else {
                for (int g = 0; g < kBG; ++g) {
                    const long long p0 = pb + 4 * kThreads * g;
                    for (long long q = p0; q < p0 + 4 && q < a.npix; ++q) {
                        const unsigned c = color_px(fl[q], maxrad, rmax, fast, col);
                        uint8_t* px = a.bgr + ((size_t)f * a.npix + q) * 3;
                        px[0] = (uint8_t)c;
                        px[1] = (uint8_t)(c >> 8);
                        px[2] = (uint8_t)(c >> 16);
                    }
                }
            }
        }
    }
}

}  // namespace

hipError_t launch_flow_color(const float* flow, int n, int W, int H, float maxmotion, uint8_t* bgr,
                             unsigned int* ws, hipStream_t s)
{
    ColorArgs a{};
    a.flow = reinterpret_cast<const float2*>(flow);
    a.bgr = bgr;
    a.ws = ws;
    a.npix = (long long)W * H;
    a.n = n;
    a.na = maxmotion > 0.0f ? 0 : (int)((a.npix + kApx - 1) / kApx);
    a.nb = (int)((a.npix + kBpx - 1) / kBpx);
    a.maxmotion = maxmotion;
    // dwordx3 stores of 4 pixels at byte 12 k of a field, float4 loads of 2 pixels
    a.vec = a.npix % 4 == 0 && (reinterpret_cast<uintptr_t>(bgr) & 3) == 0 && (reinterpret_cast<uintptr_t>(flow) & 15) == 0;
    hipError_t e = hipMemsetAsync(ws, 0, sizeof(unsigned int) * (kMaxStride * (size_t)n + 1), s);
    if (e != hipSuccess) return e;
    const long long items = (long long)(a.na + a.nb) * n;
    if (items >= (1LL << 31)) return hipErrorInvalidValue;
    const unsigned grid = (unsigned)std::min<long long>((items + kClaim - 1) / kClaim, 256 * 8);  // persistent: 8 per CU
    hipLaunchKernelGGL(k_color, dim3(grid), dim3(kThreads), 0, s, a);
    return hipGetLastError();
}

size_t flow_color_ws_words(int n) { return (size_t)kMaxStride * n + 1; }

}  // namespace dis
