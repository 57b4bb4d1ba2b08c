// dis_device.h -- device helpers shared by the DIS kernels (exact float32
// semantics of the reference; compiled with -ffp-contract=off).
#pragma once

#include <hip/hip_runtime.h>

namespace dis {

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// OpenCV BORDER_REFLECT_101 for an offset of at most one pixel outside [0, n).
__device__ __forceinline__ int reflect101(int i, int n)
{
    if (n == 1) return 0;
    i = i < 0 ? -i : i;
    return i >= n ? 2 * n - 2 - i : i;
}

__device__ __forceinline__ int floordiv(int a, int b) { return (a >= 0) ? a / b : -((-a + b - 1) / b); }

// floor(a / b) for a positive integer b given rb = v_rcp_f32(b) (<= 1 ulp):
// (a + 0.5) / b sits >= 0.5 / b away from every integer, and the float error
// of (a + 0.5) * rb is < |a| / b * 2^-22, so the floor is exact for
// |a| < 2^20. Replaces the ~15-instruction integer division sequence.
__device__ __forceinline__ int floordiv_r(int a, float rb)
{
    return (int)floorf(((float)a + 0.5f) * rb);
}

// fminf(fmaxf(v, -1), hi) in one v_med3_f32 (a selection: same value for
// every non-NaN v, which is all the callers pass -- sample positions x + u of
// finite flows; fmaxf's NaN handling cost a canonicalising max besides)
__device__ __forceinline__ float clamp_m1(float v, float hi) { return __builtin_amdgcn_fmed3f(v, -1.0f, hi); }

// I1 sampled at (X, Y): bilinear, replicate border; the position is first
// clamped to [-1, W] x [-1, H] (oracle vr_warp: identical expressions).
__device__ __forceinline__ float bilinear_replicate(const float* __restrict__ I, int W, int H, float X, float Y)
{
    X = clamp_m1(X, (float)W);
    Y = clamp_m1(Y, (float)H);
    const float fx0 = floorf(X), fy0 = floorf(Y);
    const int xa = (int)fx0, ya = (int)fy0;
    const float fx = X - fx0, fy = Y - fy0;
    const int c0 = clampi(xa, 0, W - 1), c1 = clampi(xa + 1, 0, W - 1);
    // 24-bit multiplies (full rate; v_mul_lo_u32 is quarter rate): row < H and
    // W are < 2^24 and the product < 2^31 (a plane < 2^31 floats)
    const unsigned o0 = __umul24((unsigned)clampi(ya, 0, H - 1), (unsigned)W);
    const unsigned o1 = __umul24((unsigned)clampi(ya + 1, 0, H - 1), (unsigned)W);
    const float top = (1.0f - fx) * I[o0 + c0] + fx * I[o0 + c1];
    const float bot = (1.0f - fx) * I[o1 + c0] + fx * I[o1 + c1];
    return (1.0f - fy) * top + fy * bot;
}

// Pre-factored Eigen PartialPivLU of the fixed 2x2 patch Hessian
// (src/patch.cpp:176): pivot on |a10| > |a00| (first index wins ties),
// l = a_q0 / a_p0 (skipped when the pivot is 0), u11 = a_q1 - l * a_p1.
struct LU2 {
    float u00, u01, l10, u11;
    int swap;
};

__device__ __forceinline__ LU2 lu2_factor(float h00, float h01, float h10, float h11)
{
    LU2 f;
    f.swap = fabsf(h10) > fabsf(h00);
    const float a00 = f.swap ? h10 : h00, a01 = f.swap ? h11 : h01;
    const float a10 = f.swap ? h00 : h10, a11 = f.swap ? h01 : h11;
    float l = a10;
    if (a00 != 0.0f) l = a10 / a00;
    f.u00 = a00;
    f.u01 = a01;
    f.l10 = l;
    f.u11 = a11 - l * a01;
    return f;
}

// PartialPivLU::solve: P b, unit-lower forward, upper backward substitution.
__device__ __forceinline__ void lu2_solve(const LU2& f, float b0, float b1, float* x0, float* x1)
{
    float c0 = f.swap ? b1 : b0, c1 = f.swap ? b0 : b1;
    c1 = c1 - f.l10 * c0;
    c1 = c1 / f.u11;
    c0 = c0 - c1 * f.u01;
    c0 = c0 / f.u00;
    *x0 = c0;
    *x1 = c1;
}

// Hessian regularisation (src/patch.cpp:86-90): when the 2x2 determinant is
// exactly zero, add the double literal 1e-10 to the diagonal (float += double).
__device__ __forceinline__ LU2 hessian_lu2(float h00, float h01, float h11)
{
    const float h10 = h01;
    if (h00 * h11 - h10 * h01 == 0.0f) {
        h00 = (float)((double)h00 + 1e-10);
        h11 = (float)((double)h11 + 1e-10);
    }
    return lu2_factor(h00, h01, h10, h11);
}

// Bilinear warp weights and tap base of one sample position
// (src/patch.cpp:207-267): l = floorf(x), k = floorf(y), a = x - l, b = y - k,
// X = ceilf(x + 1e-5f) (Q8: the epsilon is a no-op from 256 on).
struct Warp {
    float w0, w1, w2, w3;
    int X, Y;
};

__device__ __forceinline__ Warp warp_coefs(float x, float y)
{
    Warp w;
    const float l = floorf(x), k = floorf(y);
    const float a = x - l, b = y - k;
    w.w0 = (1 - a) * (1 - b);
    w.w1 = a * (1 - b);
    w.w2 = b * (1 - a);
    w.w3 = a * b;
    w.X = (int)ceilf(x + .00001f);
    w.Y = (int)ceilf(y + .00001f);
    return w;
}

// Densified flow at one level pixel (px, py) (src/patch_grid.cpp:121-182) as a
// gather: every patch whose ps x ps footprint covers the pixel contributes
// 0.5*u in patch-id order (gx outer, gy inner), f starts at +0, the weight is
// the sum of the 0.5s (zero-initialised, Q7), then f /= w if w > 0.
__device__ __forceinline__ float2 dense_at(const float2* __restrict__ u, int npw, int nph, int offw,
                                           int offh, int steps, int hp, int px, int py)
{
    int gx0 = floordiv(px - offw - hp + steps, steps), gx1 = floordiv(px - offw + hp, steps);
    int gy0 = floordiv(py - offh - hp + steps, steps), gy1 = floordiv(py - offh + hp, steps);
    gx0 = gx0 < 0 ? 0 : gx0;
    gy0 = gy0 < 0 ? 0 : gy0;
    gx1 = gx1 > npw - 1 ? npw - 1 : gx1;
    gy1 = gy1 > nph - 1 ? nph - 1 : gy1;
    float fx = 0.0f, fy = 0.0f, w = 0.0f;
    for (int gx = gx0; gx <= gx1; ++gx)
        for (int gy = gy0; gy <= gy1; ++gy) {
            const float2 v = u[gx * nph + gy];
            fx = fx + v.x * 0.5f;
            fy = fy + v.y * 0.5f;
            w = w + 0.5f;
        }
    if (w > 0) {
        fx = fx / w;
        fy = fy / w;
    }
    return make_float2(fx, fy);
}

// Correctly rounded sqrt for x = 0 or a normal float well inside the range
// (no denormal pre-scaling): v_sqrt_f32 is within one ulp; the fma residuals
// of the neighbours r -/+ 1 ulp pick the rounded root. Used by the pyramid on
// x = N, an integer < 2^22 (Sobel magnitude^2 * 64). On that domain the raw
// v_sqrt_f32 of gfx950 is either RN(sqrt N) or one ulp BELOW it (never above:
// tools/sqrt_dir, all 2,080,801 N: 1,744,787 exact, 336,014 one ulp low), so
// only the round-up test is needed (4 VALU instead of 8; k_pyr12 98.7 -> 85.4
// us per 32 1080p pairs). tools/sqrt_check (a -m gpu test) proves the compiled
// form equal to sqrtf on every such N.
__device__ __forceinline__ float sqrt_cr(float x)
{
    const float r = __builtin_amdgcn_sqrtf(x);
    const float rp = __int_as_float(__float_as_int(r) + 1);
    return __builtin_fmaf(-rp, r, x) > 0.0f ? rp : r;
}

// Correctly rounded a / b for a divisor b used many times (the search's
// per-patch LU pivots, the output kernel's densify weights), given r = RN(1 / b)
// (one full division per patch instead of one per update): q0 = a*r is
// within 2 ulp, one fma correction makes it faithful, and Markstein's step
// (exact remainder e = a - b*q1, then RN(q1 + e*r)) rounds it correctly
// (Markstein 1990; Muller et al., Handbook of FP Arithmetic, thm. 4.12),
// given no over/underflow in the remainders -- the patch sums here are
// image-scale. a = +-0 keeps q0 (the fma steps would turn -0 into +0);
// b = 0 gives r = inf and NaN instead of +-inf, which the outlier test
// resets exactly like the reference's inf.
__device__ __forceinline__ float div_pre(float a, float b, float r)
{
    const float q0 = a * r;
    const float q1 = __builtin_fmaf(__builtin_fmaf(-b, q0, a), r, q0);
    const float q2 = __builtin_fmaf(__builtin_fmaf(-b, q1, a), r, q1);
    // the sign of q0 on the magnitude of q2 (one v_bfi_b32 instead of a
    // compare and a VCC select): for a != 0 and finite b the two signs agree
    // (sign(a / b) = sign(a * RN(1 / b)), signed zeros of an underflow
    // included), and for a = +-0 q2 is a zero whose sign the fma steps may
    // have lost while q0's is right -- the bits of `a == 0 ? q0 : q2` for
    // every finite b (the divisors here are finite: patch sums, weights)
    return __int_as_float((__float_as_int(q0) & (int)0x80000000) | (__float_as_int(q2) & 0x7fffffff));
}

// a / b, correctly rounded, for 2^-60 <= b <= 2^60 and a = 0 or
// b 2^-30 <= a <= b (div_core_ok): the core of the IEEE division sequence the
// compiler emits (v_rcp_f32, one Newton step, quotient, two remainder
// corrections) without v_div_scale / v_div_fmas / v_div_fixup, whose scaling
// and special cases these operands never need. The final step's correct
// rounding rests on the refined reciprocal, i.e. on v_rcp_f32's accuracy:
// tools/color_core_check (a -m gpu test) compares it with the IEEE division on
// every divisor mantissa. Used by the colour kernel (atan2's min / max).
__device__ __forceinline__ bool div_core_ok(float a, float b)
{
    return b >= 0x1p-60f && b <= 0x1p60f && (a == 0.0f || (a >= b * 0x1p-30f && a <= b));
}
__device__ __forceinline__ float div_core(float a, float b)
{
    float y = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, y, 1.0f);
    y = __builtin_fmaf(e, y, y);
    float q = a * y;
    float r = __builtin_fmaf(-b, q, a);
    q = __builtin_fmaf(r, y, q);
    r = __builtin_fmaf(-b, q, a);
    return __builtin_fmaf(r, y, q);
}

// RN(1 / m) for 1 <= m < 2^30: v_rcp_f32 and one Newton step (3 instructions
// instead of div_core's 7). Rests on this GPU's v_rcp_f32: alone it is one ulp
// off for 11 % of the domain, with the step exact on all of it --
// tools/color_core_check tries every float m in [1, 2^30) against 1.0f / m.
__device__ __forceinline__ float recip_core(float m)
{
    const float y = __builtin_amdgcn_rcpf(m);
    return __builtin_fmaf(__builtin_fmaf(-m, y, 1.0f), y, y);
}

// 1 / max(1, |d|), correctly rounded (the paper mode's vote weight, Kroeger et
// al. 2016 eq. 4): recip_core for m = max(1, |d|) < 2^30, the IEEE division
// above that (and for NaN-free infinities), behind a wave-uniform test (no
// exec-mask bookkeeping while no lane needs it)
__device__ __forceinline__ float recip_max1(float d)
{
    const float m = fmaxf(1.0f, fabsf(d));
    const float y = recip_core(m);
    if (__builtin_amdgcn_ballot_w64(!(m < 0x1p30f)) == 0) return y;
    return m < 0x1p30f ? y : 1.0f / m;
}

// sqrtf(x), correctly rounded, for x = +0 or 2^-96 <= x <= 2^96 (sqrt_core_ok):
// v_sqrt_f32 (within one ulp) and the residual tests of both neighbours (the
// two-sided form of sqrt_cr above; no denormal scaling in this range);
// tools/color_core_check compares it with sqrtf on whole binades.
__device__ __forceinline__ bool sqrt_core_ok(float x) { return (x >= 0x1p-96f && x <= 0x1p96f) || x == 0.0f; }
__device__ __forceinline__ float sqrt_core(float x)
{
    const float r = __builtin_amdgcn_sqrtf(x);
    const float rm = __int_as_float(__float_as_int(r) - 1);
    const float rp = __int_as_float(__float_as_int(r) + 1);
    float y = __builtin_fmaf(-rm, r, x) <= 0.0f ? rm : r;
    y = __builtin_fmaf(-rp, r, x) > 0.0f ? rp : y;
    return x == 0.0f ? x : y;
}

}  // namespace dis
