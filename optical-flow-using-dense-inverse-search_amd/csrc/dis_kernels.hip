// dis_kernels.hip -- CDNA4 (gfx950) kernels of the DIS hot path.
//
// Compiled with -ffp-contract=off: every float op rounds once in source order,
// matching the reference's non-FMA x64 build. Division and sqrtf are the
// correctly rounded hipcc defaults. Each kernel cites the reference lines it
// implements; layouts are described in DESIGN.md.
//
// Batch: every kernel takes the pair index from blockIdx.z (or .y), so one
// launch covers a whole batch of frame pairs (coarse levels have too few
// patches per pair to fill 256 CUs otherwise).
#include "dis_device.h"
#include "dis_kernels.h"

namespace dis {

// ---------------------------------------------------------------------------
// Small exact-arithmetic helpers
// ---------------------------------------------------------------------------

// Eigen 3.3 vectorized redux (4-wide SSE packets, two accumulators, aligned
// storage) of N products x(0..N-1): src/patch.cpp:82-84, 171-172, 265.
template <int N, typename F>
__device__ __forceinline__ float eigen_sum(F&& x)
{
    if constexpr (N < 4) {
        float r = x(0);
#pragma unroll
        for (int i = 1; i < N; ++i) r = r + x(i);
        return r;
    } else {
        constexpr int A = (N / 4) * 4, A2 = (N / 8) * 8;
        float p0[4], p1[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) p0[j] = x(j);
        if constexpr (A > 4) {
#pragma unroll
            for (int j = 0; j < 4; ++j) p1[j] = x(4 + j);
#pragma unroll
            for (int i = 8; i < A2; i += 8)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    p0[j] = p0[j] + x(i + j);
                    p1[j] = p1[j] + x(i + 4 + j);
                }
#pragma unroll
            for (int j = 0; j < 4; ++j) p0[j] = p0[j] + p1[j];
            if constexpr (A > A2) {
#pragma unroll
                for (int j = 0; j < 4; ++j) p0[j] = p0[j] + x(A2 + j);
            }
        }
        float r = (p0[0] + p0[2]) + (p0[1] + p0[3]);
#pragma unroll
        for (int i = A; i < N; ++i) r = r + x(i);
        return r;
    }
}

// compute_hessian_matrix (src/patch.cpp:75-91) + factorisation.
template <int NP>
__device__ __forceinline__ LU2 hessian_lu(const float* gdx, const float* gdy)
{
    float h00 = eigen_sum<NP>([&](int i) { return gdx[i] * gdx[i]; });
    float h01 = eigen_sum<NP>([&](int i) { return gdx[i] * gdy[i]; });
    float h11 = eigen_sum<NP>([&](int i) { return gdy[i] * gdy[i]; });
    return hessian_lu2(h00, h01, h11);
}

// ---------------------------------------------------------------------------
// K1: level 0 = Sobel magnitude of the padded u8 frame (src/main.cpp:139-160,
// 16-27). Virtual padding: replicate to Wp x Hp (floor/ceil split), then
// OpenCV Sobel (ksize 3, scale 1/8, reflect-101 at the Wp x Hp border).
// grid: (ceil(Wp/64), ceil(Hp/4), 2*batch) ; z = pair*2 + frame
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_level0_mag(const uint8_t* __restrict__ I0,
                                                    const uint8_t* __restrict__ I1, size_t stride,
                                                    size_t pair_stride, int W, int H, int Wp, int Hp,
                                                    int pl, int pt, float* __restrict__ img0,
                                                    float* __restrict__ img1, long long plane_stride)
{
    const int x = blockIdx.x * 64 + threadIdx.x;
    const int y = blockIdx.y * 4 + threadIdx.y;
    const int pair = blockIdx.z >> 1, frame = blockIdx.z & 1;
    if (x >= Wp || y >= Hp) return;
    const uint8_t* src = (frame ? I1 : I0) + (size_t)pair * pair_stride;
    float v[3][3];
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
        const int yy = clampi(reflect101(y + dy - 1, Hp) - pt, 0, H - 1);
        const uint8_t* row = src + (size_t)yy * stride;
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
            const int xx = clampi(reflect101(x + dx - 1, Wp) - pl, 0, W - 1);
            v[dy][dx] = (float)row[xx];
        }
    }
    float R[3], S[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        R[r] = v[r][2] - v[r][0];
        S[r] = v[r][1] * 0.25f + (v[r][0] + v[r][2]) * 0.125f;
    }
    const float gx = R[1] * 0.25f + (R[0] + R[2]) * 0.125f;
    const float gy = S[2] - S[0];
    const float t1 = gx * gx, t2 = gy * gy;
    const float s = t1 + t2;
    float* dst = (frame ? img1 : img0) + (size_t)pair * plane_stride;
    dst[(size_t)y * Wp + x] = sqrtf(s);
}

// ---------------------------------------------------------------------------
// K2a: 2x downsample = OpenCV INTER_LINEAR at exactly 0.5 (fast 2x2 area path):
// ((a + b) + c) + d, times 0.25 (src/main.cpp:29). grid z = pair*2 + frame.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_down2(float* __restrict__ img0, float* __restrict__ img1,
                                               long long plane_stride, long long src_off,
                                               long long dst_off, int Ws, int Wd, int Hd)
{
    const int x = blockIdx.x * 64 + threadIdx.x;
    const int y = blockIdx.y * 4 + threadIdx.y;
    const int pair = blockIdx.z >> 1, frame = blockIdx.z & 1;
    if (x >= Wd || y >= Hd) return;
    float* base = (frame ? img1 : img0) + (size_t)pair * plane_stride;
    const float* a = base + src_off + (size_t)(2 * y) * Ws + 2 * x;
    float s = a[0] + a[1];
    s = s + a[Ws];
    s = s + a[Ws + 1];
    base[dst_off + (size_t)y * Wd + x] = s * 0.25f;
}

// ---------------------------------------------------------------------------
// K2b: Sobel dx, dy of a frame-0 level (src/main.cpp:34-35), reflect-101.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_sobel(const float* __restrict__ img, float* __restrict__ gdx,
                                               float* __restrict__ gdy, long long plane_stride,
                                               long long off, int W, int H)
{
    const int x = blockIdx.x * 64 + threadIdx.x;
    const int y = blockIdx.y * 4 + threadIdx.y;
    const int pair = blockIdx.z;
    if (x >= W || y >= H) return;
    const float* src = img + (size_t)pair * plane_stride + off;
    const int xm = reflect101(x - 1, W), xp = reflect101(x + 1, W);
    float R[3], S[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const float* row = src + (size_t)reflect101(y + r - 1, H) * W;
        const float l = row[xm], c = row[x], rr = row[xp];
        R[r] = rr - l;
        S[r] = c * 0.25f + (l + rr) * 0.125f;
    }
    const size_t o = (size_t)pair * plane_stride + off + (size_t)y * W + x;
    gdx[o] = R[1] * 0.25f + (R[0] + R[2]) * 0.125f;
    gdy[o] = S[2] - S[0];
}

// ---------------------------------------------------------------------------
// Coarse-to-fine initialisation (src/patch_grid.cpp:108-119): nearest (floor)
// lookup of the coarser dense flow at (floor(ref/2)), times 2.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void init_from_coarser(const float2* __restrict__ dense_c, int Wl,
                                                  float refx, float refy, float* ix, float* iy)
{
    const int x = (int)floorf(refx / 2), y = (int)floorf(refy / 2);
    const float2 f = dense_c[(size_t)y * (Wl / 2) + x];
    *ix = f.x * 2;
    *iy = f.y * 2;
}

// ---------------------------------------------------------------------------
// K3 (generic even PS): one lane per patch. Patch::init_patch +
// Patch::inverse_search (src/patch.cpp:31-203) with get_patch_second_image
// (:207-267). Gradients are read from zero-padded dx/dy planes (virtual
// padding), the target image with replicate (clamp) padding.
// grid: (ceil(n/64), 1, batch)
// ---------------------------------------------------------------------------
template <int PS>
__global__ void __launch_bounds__(64) k_search_generic(SearchArgs a)
{
    constexpr int NP = PS * PS, HP = PS / 2;
    const int id = blockIdx.x * 64 + threadIdx.x;
    const int pair = blockIdx.z;
    if (id >= a.n) return;
    const int gx = id / a.nph, gy = id - gx * a.nph;  // x-major ids (src/patch_grid.cpp:39-50)
    const float refx = (float)(gx * a.steps + a.offw), refy = (float)(gy * a.steps + a.offh);
    const int W = a.W, H = a.H;
    const int pad = a.phys_pad;
    const long long rs = W + 2 * pad;          // row stride
    const long long org = pad * rs + pad;      // image origin inside the plane
    const float* dxp = a.dx + (size_t)pair * a.plane_stride + a.plane_off + org;
    const float* dyp = a.dy + (size_t)pair * a.plane_stride + a.plane_off + org;
    const float* I1 = a.img1 + (size_t)pair * a.plane_stride + a.plane_off + org;

    float gdx[NP], gdy[NP], r[NP];
    // get_gradients_on_patch (src/patch.cpp:47-73): rows outer, cols inner
    {
        const int px = (int)refx, py = (int)refy;
#pragma unroll
        for (int j = 0; j < PS; ++j)
#pragma unroll
            for (int i = 0; i < PS; ++i) {
                const int xx = px - HP + i, yy = py - HP + j;
                const bool in = pad > 0 || (xx >= 0 && yy >= 0 && xx < W && yy < H);
                const long long o = in ? (long long)yy * rs + xx : 0;
                gdx[j * PS + i] = in ? dxp[o] : 0.0f;
                gdy[j * PS + i] = in ? dyp[o] : 0.0f;
            }
    }
    const LU2 lu = hessian_lu<NP>(gdx, gdy);
    // paper mode: template part of b = sum(g * (I1n - Tn)),
    // bt = sum(g * Tn), T = frame-0 level image on the patch (replicate border),
    // Tn = T - mean(T) with normalisation (oracle patch_search)
    float bt0 = 0.0f, bt1 = 0.0f;
    if (a.paper) {
        const float* I0 = a.img0 + (size_t)pair * a.plane_stride + a.plane_off + org;
        const int px = (int)refx, py = (int)refy;
        const int lo = pad > 0 ? -pad : 0;
        const int hx = pad > 0 ? W - 1 + pad : W - 1, hy = pad > 0 ? H - 1 + pad : H - 1;
#pragma unroll
        for (int j = 0; j < PS; ++j)
#pragma unroll
            for (int i = 0; i < PS; ++i)
                r[j * PS + i] = I0[(long long)clampi(py - HP + j, lo, hy) * rs + clampi(px - HP + i, lo, hx)];
        if (a.norm) {
            const float mt = eigen_sum<NP>([&](int i) { return r[i]; }) / (float)NP;
#pragma unroll
            for (int i = 0; i < NP; ++i) r[i] = r[i] - mt;
        }
        bt0 = eigen_sum<NP>([&](int i) { return gdx[i] * r[i]; });
        bt1 = eigen_sum<NP>([&](int i) { return gdy[i] * r[i]; });
    }

    float inx = 0.0f, iny = 0.0f;
    if (a.dense_coarse)
        init_from_coarser(a.dense_coarse + (size_t)pair * a.dense_stride, W, refx, refy, &inx, &iny);

    float u0 = inx, u1 = iny;
    const float sx = refx + u0, sy = refy + u1;  // start position (src/patch.cpp:125-128)
    auto oob = [&](float x, float y) {
        return x < a.tmp_lb || y < a.tmp_lb || x > a.tmp_ub_w || y > a.tmp_ub_h;
    };
    auto warp = [&](float x, float y) {  // get_patch_second_image (src/patch.cpp:207-267)
        const float l = floorf(x), k = floorf(y);
        const float fa = x - l, fb = y - k;
        const float w0 = (1 - fa) * (1 - fb), w1 = fa * (1 - fb), w2 = fb * (1 - fa), w3 = fa * fb;
        const int X = (int)ceilf(x + .00001f), Y = (int)ceilf(y + .00001f);  // Q8
        const int lo = pad > 0 ? -pad : 0;
        const int hx = pad > 0 ? W - 1 + pad : W - 1, hy = pad > 0 ? H - 1 + pad : H - 1;
#pragma unroll
        for (int j = 0; j < PS; ++j) {
            const int ya = clampi(Y - HP + j, lo, hy), yc = clampi(Y - HP + j - 1, lo, hy);
            const float* ra = I1 + (long long)ya * rs;
            const float* rc = I1 + (long long)yc * rs;
#pragma unroll
            for (int i = 0; i < PS; ++i) {
                const int xa = clampi(X - HP + i, lo, hx), xb = clampi(X - HP + i - 1, lo, hx);
                float t = w3 * ra[xa];
                t = t + w2 * ra[xb];
                t = t + w1 * rc[xa];
                t = t + w0 * rc[xb];
                r[j * PS + i] = t;
            }
        }
        if (a.norm) {
            const float mean = eigen_sum<NP>([&](int i) { return r[i]; }) / (float)NP;
#pragma unroll
            for (int i = 0; i < NP; ++i) r[i] = r[i] - mean;
        }
    };

    if (!oob(sx, sy)) {  // inverse_search_start (src/patch.cpp:131-153)
        warp(sx, sy);
        for (int counter = 1;; ++counter) {  // src/patch.cpp:165-202
            float b0 = eigen_sum<NP>([&](int i) { return gdx[i] * r[i]; });
            float b1 = eigen_sum<NP>([&](int i) { return gdy[i] * r[i]; });
            if (a.paper) {
                b0 = b0 - bt0;
                b1 = b1 - bt1;
            }
            float d0, d1;
            lu2_solve(lu, b0, b1, &d0, &d1);
            u0 = u0 - d0;
            u1 = u1 - d1;
            const float px = refx + u0, py = refy + u1;
            const float ex = sx - px, ey = sy - py;
            const float nrm = sqrtf(ex * ex + ey * ey);
            if (nrm > a.outlier || oob(px, py) || nrm != nrm) {  // :185-194 (NaN: see oracle)
                u0 = inx;
                u1 = iny;
                break;
            }
            if (counter > a.iters) break;  // :199-201
            warp(px, py);
        }
    }
    float2* out = a.u_out + (size_t)pair * a.u_stride;
    out[id] = make_float2(u0, u1);
}

// ---------------------------------------------------------------------------
// K4: densification (src/patch_grid.cpp:121-182) as a deterministic per-pixel
// gather: contributions in patch-id order (gx outer, gy inner), f starts at
// +0, weights 0.5 each (Q6, Q7: zero-initialised), then f /= w.
// grid: (ceil(W/64), ceil(H/4), batch)
// ---------------------------------------------------------------------------
// RN(1 / (0.5 n)) for n covering patches (compile-time IEEE division: the
// same bits as the division at run time)
struct DensifyRcp {
    float r[257];
};
constexpr DensifyRcp make_densify_rcp()
{
    DensifyRcp t{};
    for (int n = 1; n <= 256; ++n) t.r[n] = 1.0f / (0.5f * (float)n);
    return t;
}
__constant__ DensifyRcp c_densify_rcp = make_densify_rcp();

// block: kDenBX x kDenBY pixels; the patches covering it (at most
// ((kDenBX + 16) / 1 + 1) x ((kDenBY + 16) / 1 + 1) for ps <= 16, step >= 1)
// staged in LDS once, read by every pixel from there (the x-major patch array
// read straight per pixel cost 32 cache lines per wave-load: 344 us per 4K
// level-0 pair of planes, L1/L2-bound)
constexpr int kDenBX = 32, kDenBY = 8;
constexpr int kDenPX = kDenBX + 17, kDenPY = kDenBY + 17;

__global__ void __launch_bounds__(kDenBX * kDenBY) k_densify(DensifyArgs a)
{
    __shared__ float2 su[kDenPX * kDenPY];
    const int x0 = blockIdx.x * kDenBX, y0 = blockIdx.y * kDenBY;
    const int x = x0 + threadIdx.x;
    const int y = y0 + threadIdx.y;
    const int pair = blockIdx.z;
    const int hp = a.ps / 2;
    // patches covering x: ref.x in [x - hp + 1, x + hp] (floor divisions through
    // the reciprocal of the grid step: exact for |a| < 2^20, floordiv_r)
    const float rs = __builtin_amdgcn_rcpf((float)a.steps);
    auto lo = [&](int v, int off) { return max(0, floordiv_r(v - off - hp + 1 + a.steps - 1, rs)); };
    auto hi = [&](int v, int off, int n) { return min(n - 1, floordiv_r(v - off + hp, rs)); };
    const int bx0 = lo(x0, a.offw), by0 = lo(y0, a.offh);
    const int bnx = hi(min(x0 + kDenBX - 1, a.W - 1), a.offw, a.npw) - bx0 + 1;
    const int bny = hi(min(y0 + kDenBY - 1, a.H - 1), a.offh, a.nph) - by0 + 1;
    const float2* u = a.u + (size_t)pair * a.u_stride;
    for (int k = threadIdx.y * kDenBX + threadIdx.x; k < bnx * bny; k += kDenBX * kDenBY) {
        const int cx = k / bny, cy = k - cx * bny;  // consecutive threads: consecutive patch ids
        su[cx * bny + cy] = u[(bx0 + cx) * a.nph + by0 + cy];
    }
    __syncthreads();
    if (x >= a.W || y >= a.H) return;
    const int gx0 = lo(x, a.offw), gx1 = hi(x, a.offw, a.npw);
    const int gy0 = lo(y, a.offh), gy1 = hi(y, a.offh, a.nph);
    float fx = 0.0f, fy = 0.0f, w = 0.0f;
    if (a.paper) {  // SURVEY 8f row 4 (oracle densify_paper)
        const float* I0 = a.img0 + (size_t)pair * a.plane_stride;
        const float* I1 = a.img1 + (size_t)pair * a.plane_stride;
        const float i0 = I0[(size_t)y * a.W + x];
        for (int gx = gx0; gx <= gx1; ++gx)
            for (int gy = gy0; gy <= gy1; ++gy) {
                const float2 v = su[(gx - bx0) * bny + gy - by0];
                const float d = bilinear_replicate(I1, a.W, a.H, (float)x + v.x, (float)y + v.y) - i0;
                const float c = recip_max1(d);  // 1 / max(1, |d|), correctly rounded (dis_device.h)
                fx = fx + c * v.x;
                fy = fy + c * v.y;
                w = w + c;
            }
    } else {
        for (int gx = gx0; gx <= gx1; ++gx)
            for (int gy = gy0; gy <= gy1; ++gy) {
                const float2 v = su[(gx - bx0) * bny + gy - by0];
                fx = fx + v.x * 0.5f;
                fy = fy + v.y * 0.5f;
                w = w + 0.5f;
            }
        // w = 0.5 n exactly: fx / w correctly rounded through the tabulated
        // RN(1 / w) (div_pre); tiny nonzero numerators, whose remainders could
        // underflow, and more than 256 covering patches divide the IEEE way
        const int n = (int)(w * 2.0f);
        const bool tiny = (fx != 0.0f && fabsf(fx) < 0x1p-100f) || (fy != 0.0f && fabsf(fy) < 0x1p-100f);
        if (n > 0 && n <= 256 && !tiny) {
            const float r = c_densify_rcp.r[n];
            fx = div_pre(fx, w, r);
            fy = div_pre(fy, w, r);
            w = 0.0f;  // done
        }
    }
    if (w > 0) {
        fx = fx / w;
        fy = fy / w;
    }
    a.dense[(size_t)pair * a.dense_stride + (size_t)y * a.W + x] = make_float2(fx, fy);
}

// ---------------------------------------------------------------------------
// K5: flow *= 2^F, cv::resize(x2^F, INTER_LINEAR), crop (src/main.cpp:191-198).
// Coefficients: s = (float)((d + .5) * 2^-F - .5) (double), i = floor(s),
// f = s - i, clamped (i < 0 -> 0,0 ; i >= n-1 -> n-1,0); horizontal taps with
// d >= xmax use S[i] alone (HResizeLinear), vertical always S0*b0 + S1*b1.
// grid: (ceil(W/64), ceil(H/4), batch)
// ---------------------------------------------------------------------------
struct Coef {
    int i;
    float f;
};

__device__ __forceinline__ Coef lin_coef(int d, int n_src, double scale)
{
    float fx = (float)((d + 0.5) * scale - 0.5);
    int sx = (int)floorf(fx);
    fx -= (float)sx;
    if (sx < 0) {
        fx = 0;
        sx = 0;
    }
    if (sx >= n_src - 1) {
        fx = 0;
        sx = n_src - 1;
    }
    Coef c;
    c.i = sx;
    c.f = fx;
    return c;
}

__global__ void __launch_bounds__(256) k_upsample_crop(UpsampleArgs a)
{
    const int x = blockIdx.x * 64 + threadIdx.x;
    const int y = blockIdx.y * 4 + threadIdx.y;
    const int pair = blockIdx.z;
    if (x >= a.W || y >= a.H) return;
    const float2* S = a.dense + (size_t)pair * a.dense_stride;
    float2* out = a.flow + (size_t)pair * a.W * a.H;
    const int xx = x + a.pad_left, yy = y + a.pad_top;
    if (a.F == 0) {
        out[(size_t)y * a.W + x] = S[(size_t)yy * a.wF + xx];
        return;
    }
    const float sc = a.sc;
    const Coef cx = lin_coef(xx, a.wF, a.inv_sc);
    const Coef cy = lin_coef(yy, a.hF, a.inv_sc);
    const bool two = xx < a.xmax;
    const int r0 = cy.i, r1 = cy.i + 1 < a.hF ? cy.i + 1 : a.hF - 1;
    float h[2][2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const float2* row = S + (size_t)(k ? r1 : r0) * a.wF;
        const float2 s0 = row[cx.i];
        const float ax = s0.x * sc, ay = s0.y * sc;  // flowout *= sc_fct (:194)
        if (two) {
            const float2 s1 = row[cx.i + 1];
            const float bx = s1.x * sc, by = s1.y * sc;
            h[k][0] = ax * (1.f - cx.f) + bx * cx.f;
            h[k][1] = ay * (1.f - cx.f) + by * cx.f;
        } else {
            h[k][0] = ax;
            h[k][1] = ay;
        }
    }
    const float b0 = 1.f - cy.f, b1 = cy.f;
    out[(size_t)y * a.W + x] = make_float2(h[0][0] * b0 + h[1][0] * b1, h[0][1] * b0 + h[1][1] * b1);
}

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
static inline dim3 grid2d(int W, int H, int z) { return dim3((W + 63) / 64, (H + 3) / 4, z); }

hipError_t launch_level0(const uint8_t* I0, const uint8_t* I1, size_t stride, size_t pair_stride,
                         const Geometry& g, float* img0, float* img1, int batch, hipStream_t s)
{
    hipLaunchKernelGGL(k_level0_mag, grid2d(g.Wp, g.Hp, 2 * batch), dim3(64, 4), 0, s, I0, I1, stride,
                       pair_stride, g.W, g.H, g.Wp, g.Hp, g.pad_left, g.pad_top, img0, img1,
                       (long long)g.plane_stride);
    return hipGetLastError();
}

hipError_t launch_down2(const Geometry& g, int l, float* img0, float* img1, int batch, hipStream_t s)
{
    const LevelGeom& d = g.lv[l];
    const LevelGeom& sl = g.lv[l - 1];
    hipLaunchKernelGGL(k_down2, grid2d(d.W, d.H, 2 * batch), dim3(64, 4), 0, s, img0, img1,
                       (long long)g.plane_stride, sl.plane_off, d.plane_off, sl.W, d.W, d.H);
    return hipGetLastError();
}

hipError_t launch_sobel(const Geometry& g, int l, const float* img0, float* dx, float* dy, int batch,
                        hipStream_t s)
{
    const LevelGeom& d = g.lv[l];
    hipLaunchKernelGGL(k_sobel, grid2d(d.W, d.H, batch), dim3(64, 4), 0, s, img0, dx, dy,
                       (long long)g.plane_stride, d.plane_off, d.W, d.H);
    return hipGetLastError();
}

hipError_t launch_search_generic(const SearchArgs& a, int ps, int batch, hipStream_t s, Timing t)
{
    dim3 grid((a.n + 63) / 64, 1, batch);
    switch (ps) {
#define DIS_CASE(P) \
    case P: DIS_LAUNCH(t, k_search_generic<P>, grid, dim3(64), 0, s, a); break;
        DIS_CASE(2)
        DIS_CASE(4)
        DIS_CASE(6)
        DIS_CASE(8)
        DIS_CASE(10)
        DIS_CASE(12)
        DIS_CASE(14)
        DIS_CASE(16)
#undef DIS_CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_densify(const DensifyArgs& a, int batch, hipStream_t s)
{
    if (a.ps > 16 || a.steps < 1) return hipErrorInvalidValue;  // the staged patch block (kDenPX x kDenPY)
    hipLaunchKernelGGL(k_densify, dim3((a.W + kDenBX - 1) / kDenBX, (a.H + kDenBY - 1) / kDenBY, batch),
                       dim3(kDenBX, kDenBY), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_upsample(const UpsampleArgs& a, int batch, hipStream_t s)
{
    hipLaunchKernelGGL(k_upsample_crop, grid2d(a.W, a.H, batch), dim3(64, 4), 0, s, a);
    return hipGetLastError();
}

}  // namespace dis
