// dis_varref.hip -- variational refinement of a level's dense flow (SURVEY.md
// 8f row 1, BASELINE config 5; absent from the reference: parity unpinned by
// construction, pinned instead to the C restatement dis_oracle_var_refine in
// oracle/dis_oracle.c, which is the specification -- same expressions, same
// order, -ffp-contract=off, so the results are bit-identical).
//
// Per fixed-point iteration (re-warp, linearise, red-black SOR):
//   k_vr_warp   I1w = I1(x + u, y + v)          bilinear, replicate border
//   k_vr_d1     Wx, Wy = 5-tap derivatives of I1w
//   k_vr_d2     Ix, Iy, Iz, Ixx, Ixy, Iyy, Ixz, Iyz
//   k_vr_smooth s = alpha / sqrt(|grad u|^2 + |grad v|^2 + eps^2)
//   k_vr_data   A11, A12, A22, B1, B2 of the normal equations, du = dv = 0
//   k_vr_sor<c> x VR_SOR_ITERS x 2 colours (a colour's pixels are independent)
//   k_vr_apply  flow += (du, dv)
// (k_vr_d0: I0x, I0y once per level.) Planes are per pair, W_l x H_l floats,
// in a context workspace; grid = (pixels / 256, pairs).
#include <hip/hip_runtime.h>

#include "dis_kernels.h"

namespace dis {

namespace {

constexpr float kAlpha = 20.0f, kGamma = 10.0f, kDelta = 5.0f, kZeta = 0.1f, kEps2 = 1e-6f, kOmega = 1.6f;

enum Plane {
    P_I1W, P_I0X, P_I0Y, P_WX, P_WY, P_IX, P_IY, P_IZ, P_IXX, P_IXY, P_IYY, P_IXZ, P_IYZ,
    P_DU, P_DV, P_SW, P_A11, P_A12, P_A22, P_B1, P_B2
};

struct Lvl {
    const float* img0;  // level planes of pair 0 (pre-offset), pair stride plane_stride
    const float* img1;
    long long plane_stride;
    float2* flow;       // dense flow of pair 0 (pre-offset), pair stride flow_stride
    long long flow_stride;
    float* ws;          // workspace of pair 0: kVarRefPlanes planes of ws_plane floats, pair stride ws_stride
    long long ws_plane, ws_stride;
    int W, H;
};

__device__ __forceinline__ int clampi_(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

__device__ __forceinline__ float at(const float* f, int W, int H, int x, int y)
{
    return f[(size_t)clampi_(y, 0, H - 1) * W + clampi_(x, 0, W - 1)];
}

// 5-tap derivative (1, -8, 0, 8, -1) / 12 along (dx, dy), replicate border
__device__ __forceinline__ float deriv(const float* f, int W, int H, int x, int y, int dx, int dy)
{
    const float a = at(f, W, H, x - 2 * dx, y - 2 * dy), b = at(f, W, H, x - dx, y - dy);
    const float c = at(f, W, H, x + dx, y + dy), d = at(f, W, H, x + 2 * dx, y + 2 * dy);
    return (((a - 8.0f * b) + 8.0f * c) - d) / 12.0f;
}

struct Px {
    int x, y, pair;
    size_t i;
    bool ok;
};

__device__ __forceinline__ Px pixel(const Lvl& L)
{
    Px p;
    const long long k = (long long)blockIdx.x * 256 + threadIdx.x;
    p.pair = blockIdx.y;
    p.ok = k < (long long)L.W * L.H;
    p.y = (int)(k / L.W);
    p.x = (int)(k - (long long)p.y * L.W);
    p.i = (size_t)k;
    return p;
}

__device__ __forceinline__ float* plane(const Lvl& L, int pair, int k)
{
    return L.ws + (size_t)pair * L.ws_stride + (size_t)k * L.ws_plane;
}

__global__ void __launch_bounds__(256) k_vr_d0(Lvl L)
{
    const Px p = pixel(L);
    if (!p.ok) return;
    const float* I0 = L.img0 + (size_t)p.pair * L.plane_stride;
    plane(L, p.pair, P_I0X)[p.i] = deriv(I0, L.W, L.H, p.x, p.y, 1, 0);
    plane(L, p.pair, P_I0Y)[p.i] = deriv(I0, L.W, L.H, p.x, p.y, 0, 1);
}

__global__ void __launch_bounds__(256) k_vr_warp(Lvl L)
{
    const Px p = pixel(L);
    if (!p.ok) return;
    const float* I1 = L.img1 + (size_t)p.pair * L.plane_stride;
    const float2 f = L.flow[(size_t)p.pair * L.flow_stride + p.i];
    float X = (float)p.x + f.x, Y = (float)p.y + f.y;
    X = fminf(fmaxf(X, -1.0f), (float)L.W);
    Y = fminf(fmaxf(Y, -1.0f), (float)L.H);
    const float fx0 = floorf(X), fy0 = floorf(Y);
    const int x0 = (int)fx0, y0 = (int)fy0;
    const float fx = X - fx0, fy = Y - fy0;
    const float a = at(I1, L.W, L.H, x0, y0), b = at(I1, L.W, L.H, x0 + 1, y0);
    const float c = at(I1, L.W, L.H, x0, y0 + 1), d = at(I1, L.W, L.H, x0 + 1, y0 + 1);
    const float top = (1.0f - fx) * a + fx * b;
    const float bot = (1.0f - fx) * c + fx * d;
    plane(L, p.pair, P_I1W)[p.i] = (1.0f - fy) * top + fy * bot;
}

__global__ void __launch_bounds__(256) k_vr_d1(Lvl L)
{
    const Px p = pixel(L);
    if (!p.ok) return;
    const float* w = plane(L, p.pair, P_I1W);
    plane(L, p.pair, P_WX)[p.i] = deriv(w, L.W, L.H, p.x, p.y, 1, 0);
    plane(L, p.pair, P_WY)[p.i] = deriv(w, L.W, L.H, p.x, p.y, 0, 1);
}

__global__ void __launch_bounds__(256) k_vr_d2(Lvl L)
{
    const Px p = pixel(L);
    if (!p.ok) return;
    const int W = L.W, H = L.H, x = p.x, y = p.y;
    const size_t i = p.i;
    const float* Wx = plane(L, p.pair, P_WX);
    const float* Wy = plane(L, p.pair, P_WY);
    const float* I0x = plane(L, p.pair, P_I0X);
    const float* I0y = plane(L, p.pair, P_I0Y);
    const float* I0 = L.img0 + (size_t)p.pair * L.plane_stride;
    plane(L, p.pair, P_IX)[i] = 0.5f * (Wx[i] + I0x[i]);
    plane(L, p.pair, P_IY)[i] = 0.5f * (Wy[i] + I0y[i]);
    plane(L, p.pair, P_IZ)[i] = plane(L, p.pair, P_I1W)[i] - I0[i];
    plane(L, p.pair, P_IXX)[i] = 0.5f * (deriv(Wx, W, H, x, y, 1, 0) + deriv(I0x, W, H, x, y, 1, 0));
    plane(L, p.pair, P_IXY)[i] = 0.5f * (deriv(Wx, W, H, x, y, 0, 1) + deriv(I0x, W, H, x, y, 0, 1));
    plane(L, p.pair, P_IYY)[i] = 0.5f * (deriv(Wy, W, H, x, y, 0, 1) + deriv(I0y, W, H, x, y, 0, 1));
    plane(L, p.pair, P_IXZ)[i] = Wx[i] - I0x[i];
    plane(L, p.pair, P_IYZ)[i] = Wy[i] - I0y[i];
}

__global__ void __launch_bounds__(256) k_vr_smooth(Lvl L)
{
    const Px p = pixel(L);
    if (!p.ok) return;
    const int W = L.W;
    const size_t i = p.i;
    const float2* f = L.flow + (size_t)p.pair * L.flow_stride;
    const float uc = f[i].x, vc = f[i].y;
    float gxu = 0.0f, gxv = 0.0f, gyu = 0.0f, gyv = 0.0f;
    if (p.x < W - 1) {
        gxu = f[i + 1].x - uc;
        gxv = f[i + 1].y - vc;
    }
    if (p.y < L.H - 1) {
        gyu = f[i + W].x - uc;
        gyv = f[i + W].y - vc;
    }
    plane(L, p.pair, P_SW)[i] = kAlpha / sqrtf((((gxu * gxu + gyu * gyu) + gxv * gxv) + gyv * gyv) + kEps2);
}

struct Nb {
    float wl, wr, wu, wd;
    size_t il, ir, iu, id;
};

__device__ __forceinline__ Nb neighbours(const float* sw, const Px& p, int W, int H)
{
    const size_t i = p.i;
    Nb n;
    n.wl = p.x > 0 ? sw[i - 1] : 0.0f;
    n.wr = p.x < W - 1 ? sw[i] : 0.0f;
    n.wu = p.y > 0 ? sw[i - W] : 0.0f;
    n.wd = p.y < H - 1 ? sw[i] : 0.0f;
    n.il = p.x > 0 ? i - 1 : i;
    n.ir = p.x < W - 1 ? i + 1 : i;
    n.iu = p.y > 0 ? i - W : i;
    n.id = p.y < H - 1 ? i + W : i;
    return n;
}

__global__ void __launch_bounds__(256) k_vr_data(Lvl L)
{
    const Px p = pixel(L);
    if (!p.ok) return;
    const size_t i = p.i;
    const int pr = p.pair;
    const float Ix = plane(L, pr, P_IX)[i], Iy = plane(L, pr, P_IY)[i], Iz = plane(L, pr, P_IZ)[i];
    const float Ixx = plane(L, pr, P_IXX)[i], Ixy = plane(L, pr, P_IXY)[i], Iyy = plane(L, pr, P_IYY)[i];
    const float Ixz = plane(L, pr, P_IXZ)[i], Iyz = plane(L, pr, P_IYZ)[i];
    const float psiI = kDelta / sqrtf(Iz * Iz + kEps2);
    const float psiG = kGamma / sqrtf((Ixz * Ixz + Iyz * Iyz) + kEps2);
    plane(L, pr, P_A11)[i] = (psiI * (Ix * Ix) + psiG * (Ixx * Ixx + Ixy * Ixy)) + kZeta;
    plane(L, pr, P_A12)[i] = psiI * (Ix * Iy) + psiG * (Ixx * Ixy + Ixy * Iyy);
    plane(L, pr, P_A22)[i] = (psiI * (Iy * Iy) + psiG * (Ixy * Ixy + Iyy * Iyy)) + kZeta;
    const Nb n = neighbours(plane(L, pr, P_SW), p, L.W, L.H);
    const float2* f = L.flow + (size_t)pr * L.flow_stride;
    const float u = f[i].x, v = f[i].y;
    const float su = ((n.wl * (f[n.il].x - u) + n.wr * (f[n.ir].x - u)) + n.wu * (f[n.iu].x - u)) + n.wd * (f[n.id].x - u);
    const float sv = ((n.wl * (f[n.il].y - v) + n.wr * (f[n.ir].y - v)) + n.wu * (f[n.iu].y - v)) + n.wd * (f[n.id].y - v);
    plane(L, pr, P_B1)[i] = su - (psiI * (Iz * Ix) + psiG * (Ixz * Ixx + Iyz * Ixy));
    plane(L, pr, P_B2)[i] = sv - (psiI * (Iz * Iy) + psiG * (Ixz * Ixy + Iyz * Iyy));
    plane(L, pr, P_DU)[i] = 0.0f;
    plane(L, pr, P_DV)[i] = 0.0f;
}

// one colour of a red-black SOR sweep: pixels with (x + y) & 1 == COLOR
template <int COLOR>
__global__ void __launch_bounds__(256) k_vr_sor(Lvl L)
{
    const Px p = pixel(L);
    if (!p.ok || ((p.x + p.y) & 1) != COLOR) return;
    const size_t i = p.i;
    const int pr = p.pair;
    float* du = plane(L, pr, P_DU);
    float* dv = plane(L, pr, P_DV);
    const Nb n = neighbours(plane(L, pr, P_SW), p, L.W, L.H);
    const float A11 = plane(L, pr, P_A11)[i], A12 = plane(L, pr, P_A12)[i], A22 = plane(L, pr, P_A22)[i];
    const float B1 = plane(L, pr, P_B1)[i], B2 = plane(L, pr, P_B2)[i];
    const float sumw = ((n.wl + n.wr) + n.wu) + n.wd;
    const float sdu = ((n.wl * du[n.il] + n.wr * du[n.ir]) + n.wu * du[n.iu]) + n.wd * du[n.id];
    const float nu = (1.0f - kOmega) * du[i] + kOmega * (((B1 + sdu) - A12 * dv[i]) / (A11 + sumw));
    const float sdv = ((n.wl * dv[n.il] + n.wr * dv[n.ir]) + n.wu * dv[n.iu]) + n.wd * dv[n.id];
    const float nv = (1.0f - kOmega) * dv[i] + kOmega * (((B2 + sdv) - A12 * nu) / (A22 + sumw));
    du[i] = nu;
    dv[i] = nv;
}

__global__ void __launch_bounds__(256) k_vr_apply(Lvl L)
{
    const Px p = pixel(L);
    if (!p.ok) return;
    float2* f = L.flow + (size_t)p.pair * L.flow_stride;
    const float2 v = f[p.i];
    f[p.i] = make_float2(v.x + plane(L, p.pair, P_DU)[p.i], v.y + plane(L, p.pair, P_DV)[p.i]);
}

}  // namespace

hipError_t launch_var_refine(const VarRefArgs& a, int n, hipStream_t s)
{
    if (a.iters <= 0) return hipSuccess;
    Lvl L;
    L.img0 = a.img0;
    L.img1 = a.img1;
    L.plane_stride = a.plane_stride;
    L.flow = a.flow;
    L.flow_stride = a.flow_stride;
    L.ws = a.ws;
    L.ws_plane = a.ws_plane;
    L.ws_stride = a.ws_stride;
    L.W = a.W;
    L.H = a.H;
    if ((long long)a.W * a.H > a.ws_plane || a.ws_stride < kVarRefPlanes * a.ws_plane) return hipErrorInvalidValue;
    const dim3 grid((unsigned)(((long long)a.W * a.H + 255) / 256), n), block(256);
    hipLaunchKernelGGL(k_vr_d0, grid, block, 0, s, L);
    for (int it = 0; it < a.iters; ++it) {
        hipLaunchKernelGGL(k_vr_warp, grid, block, 0, s, L);
        hipLaunchKernelGGL(k_vr_d1, grid, block, 0, s, L);
        hipLaunchKernelGGL(k_vr_d2, grid, block, 0, s, L);
        hipLaunchKernelGGL(k_vr_smooth, grid, block, 0, s, L);
        hipLaunchKernelGGL(k_vr_data, grid, block, 0, s, L);
        for (int k = 0; k < kVarRefSor; ++k) {
            hipLaunchKernelGGL(k_vr_sor<0>, grid, block, 0, s, L);
            hipLaunchKernelGGL(k_vr_sor<1>, grid, block, 0, s, L);
        }
        hipLaunchKernelGGL(k_vr_apply, grid, block, 0, s, L);
    }
    return hipGetLastError();
}

}  // namespace dis
