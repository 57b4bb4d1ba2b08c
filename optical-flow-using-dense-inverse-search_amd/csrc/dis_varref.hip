// dis_varref.hip -- variational refinement of a level's dense flow (SURVEY.md
// 8f row 1, BASELINE config 5; absent from the reference: parity unpinned by
// construction, pinned instead to the C restatement dis_oracle_var_refine in
// oracle/dis_oracle.c, which is the specification -- same expressions, same
// order, -ffp-contract=off, so the results are bit-identical).
//
// Two launches per fixed-point iteration (re-warp, linearise, red-black SOR):
//   k_vr_lin  one 32x32 tile of pixels: I1 warped by the current flow over the
//             tile +-4 (bilinear, replicate border), its 5-tap derivatives over
//             the tile +-2, the smoothness weights alpha/sqrt(|grad u|^2 +
//             |grad v|^2 + eps^2) over the tile + its left column / top row --
//             all staged in LDS -- then per pixel the data weights and the
//             normal equations: B1, B2, A12, D1 = A11 + sum w, D2 = A22 + sum w
//             and the pixel's own weight, six planes of the workspace.
//   k_vr_sor  all VR_SOR sweeps x 2 colours of the red-black SOR on a 108x46
//             tile, in LDS, on the tile + a halo of 10 columns / 9 rows: du =
//             dv = 0 everywhere at the first half-sweep, and every later
//             half-sweep can be wrong only one pixel further in from the
//             halo's outer edge, so after the 10th the tile itself is exact
//             (the halo is recomputed by the neighbouring tiles). Then
//             flow += (du, dv) on the tile.
// (k_vr_d0: I0x, I0y once per level.) The planes are per pair, W_l x H_l
// floats, in a context workspace of kVarRefPlanes planes per pair.
#include <hip/hip_runtime.h>

#include "dis_device.h"
#include "dis_kernels.h"

namespace dis {

namespace {

constexpr float kAlpha = 20.0f, kGamma = 10.0f, kDelta = 5.0f, kZeta = 0.1f, kEps2 = 1e-6f, kOmega = 1.6f;

enum Plane { P_I0X, P_I0Y, P_B1, P_B2, P_A12, P_D1, P_D2, P_SW };
static_assert(P_SW + 1 == kVarRefPlanes, "workspace planes");

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

__device__ __forceinline__ float* plane(const Lvl& L, int pair, int k)
{
    return L.ws + (size_t)pair * L.ws_stride + (size_t)k * L.ws_plane;
}

// XCD-aware tile order (as k_pyramid): the dispatcher deals linear block ids
// round-robin to the 8 XCDs; remapped, each XCD walks a contiguous run of
// tiles, so the halos that neighbouring tiles share are fetched into one L2
struct Tile {
    int x, y, z;
};
__device__ __forceinline__ Tile xcd_tile()
{
    const int nbx = gridDim.x, nby = gridDim.y;
    const int nb = nbx * nby * gridDim.z;
    const int lin = blockIdx.x + nbx * (blockIdx.y + nby * blockIdx.z);
    const int per = nb / 8;
    const int t = (lin < per * 8) ? (lin % 8) * per + lin / 8 : lin;
    return Tile{__builtin_amdgcn_readfirstlane(t % nbx), __builtin_amdgcn_readfirstlane((t / nbx) % nby),
                __builtin_amdgcn_readfirstlane(t / (nbx * nby))};
}

// a / b correctly rounded from r = RN(1 / b) (div_pre, dis_device.h);
// numerators below 2^-60 (whose remainders could leave the normal range) take
// IEEE division
__device__ __forceinline__ float sor_div(float a, float b, float r)
{
    if (a != 0.0f && fabsf(a) < 0x1p-60f) return a / b;
    return div_pre(a, b, r);
}

// 5-tap derivative (1, -8, 0, 8, -1) / 12 of the taps a..d at -2, -1, +1, +2;
// the division by 12 from the folded RN(1 / 12) (~6 instructions instead of
// the ~10 of the IEEE sequence; 8.5 of them per pixel in k_vr_lin)
constexpr float kR12 = 1.0f / 12.0f;
__device__ __forceinline__ float d5(float a, float b, float c, float d)
{
    return sor_div(((a - 8.0f * b) + 8.0f * c) - d, 12.0f, kR12);
}

// I0x, I0y of the level (replicate border), once per level; 2-D grid
__global__ void __launch_bounds__(256) k_vr_d0(Lvl L)
{
    const int x = blockIdx.x * 64 + (threadIdx.x & 63), y = blockIdx.y * 4 + (threadIdx.x >> 6), pr = blockIdx.z;
    if (x >= L.W || y >= L.H) return;
    const int W = L.W, H = L.H;
    const float* I0 = L.img0 + (size_t)pr * L.plane_stride;
    const float* r = I0 + (size_t)y * W;
    const float gx = d5(r[clampi_(x - 2, 0, W - 1)], r[clampi_(x - 1, 0, W - 1)], r[clampi_(x + 1, 0, W - 1)],
                        r[clampi_(x + 2, 0, W - 1)]);
    const float gy = d5(I0[(size_t)clampi_(y - 2, 0, H - 1) * W + x], I0[(size_t)clampi_(y - 1, 0, H - 1) * W + x],
                        I0[(size_t)clampi_(y + 1, 0, H - 1) * W + x], I0[(size_t)clampi_(y + 2, 0, H - 1) * W + x]);
    const size_t i = (size_t)y * W + x;
    plane(L, pr, P_I0X)[i] = gx;
    plane(L, pr, P_I0Y)[i] = gy;
}

// ---------------------------------------------------------------------------
// linearisation
// 32 x 32 output tiles and the flow kept only over the tile +-1 (the warp's
// +-4 halo lives in registers until sI is formed): 40.7 KB of LDS, 4
// workgroups per CU (64 x 16 tiles with the flow staged over +-4: 47 KB, 3)
constexpr int kLW = 32, kLH = 32;             // output tile
constexpr int kFW = kLW + 8, kFH = kLH + 8;   // flow loads, warped I1: tile +-4
constexpr int kGW = kLW + 4, kGH = kLH + 4;   // Wx, Wy, I0x, I0y: tile +-2
constexpr int kSW = kLW + 1, kSH = kLH + 1;   // smoothness weight: tile + left column, top row

// Every staged array is indexed by a logical position relative to the tile;
// the entry holds the quantity AT THE CLAMPED position, which is what the
// reference's replicate-border reads of that logical position return. A
// derivative at logical g is evaluated at c = clamp(g) from the entries at
// c +- 1, 2 -- each of which again holds the value at the clamped position.
__global__ void __launch_bounds__(256) k_vr_lin(Lvl L)
{
    __shared__ float2 sF[kLH + 2][kLW + 2];  // the flow over the tile +-1
    __shared__ float sI[kFH][kFW];
    __shared__ float sWx[kGH][kGW], sWy[kGH][kGW], sGx[kGH][kGW], sGy[kGH][kGW];
    __shared__ float sS[kSH][kSW];
    // (plain block order: the XCD-aware order halves this kernel's HBM reads,
    // 904 -> 406 MB per 4K level-0 launch, but measured 3 x 33 us slower per
    // config-5 step)
    const int W = L.W, H = L.H, pr = blockIdx.z, tid = threadIdx.x;
    const int x0 = blockIdx.x * kLW, y0 = blockIdx.y * kLH;
    const float* I0 = L.img0 + (size_t)pr * L.plane_stride;
    const float* I1 = L.img1 + (size_t)pr * L.plane_stride;
    const float2* fl = L.flow + (size_t)pr * L.flow_stride;
    // Every load of a phase is issued before any is consumed (unrolled, fixed
    // trip counts): the flow over the tile +-4, I0x / I0y over the tile +-2 and
    // the tile's I0 in one round, then the warp's bilinear taps (which need the
    // flow) in a second -- two memory latencies per workgroup instead of one
    // per loop iteration.
    constexpr int NF = (kFW * kFH + 255) / 256, NG = (kGW * kGH + 255) / 256, NP = kLW * kLH / 256;
    float2 f[NF];
    float gx0[NG], gy0[NG], i0p[NP];
#pragma unroll
    for (int t = 0; t < NF; ++t) {
        const int k = min(tid + 256 * t, kFW * kFH - 1);
        const int ly = k / kFW, lx = k - ly * kFW;
        f[t] = fl[(size_t)clampi_(y0 - 4 + ly, 0, H - 1) * W + clampi_(x0 - 4 + lx, 0, W - 1)];
    }
#pragma unroll
    for (int t = 0; t < NG; ++t) {
        const int k = min(tid + 256 * t, kGW * kGH - 1);
        const int ly = k / kGW, lx = k - ly * kGW;
        const size_t i = (size_t)clampi_(y0 - 2 + ly, 0, H - 1) * W + clampi_(x0 - 2 + lx, 0, W - 1);
        gx0[t] = plane(L, pr, P_I0X)[i];
        gy0[t] = plane(L, pr, P_I0Y)[i];
    }
#pragma unroll
    for (int t = 0; t < NP; ++t) {
        const int k = tid + 256 * t;
        const int ly = k / kLW, lx = k - ly * kLW;
        i0p[t] = I0[(size_t)min(y0 + ly, H - 1) * W + min(x0 + lx, W - 1)];
    }
    // 1. the warped I1 over the tile +-4 (I1 at the clamped position + its flow)
    float ta[NF], tb[NF], tc[NF], td[NF], wfx[NF], wfy[NF];
#pragma unroll
    for (int t = 0; t < NF; ++t) {
        const int k = min(tid + 256 * t, kFW * kFH - 1);
        const int ly = k / kFW, lx = k - ly * kFW;
        const int gx = clampi_(x0 - 4 + lx, 0, W - 1), gy = clampi_(y0 - 4 + ly, 0, H - 1);
        float X = (float)gx + f[t].x, Y = (float)gy + f[t].y;
        X = fminf(fmaxf(X, -1.0f), (float)W);
        Y = fminf(fmaxf(Y, -1.0f), (float)H);
        const float fx0 = floorf(X), fy0 = floorf(Y);
        const int xa = (int)fx0, ya = (int)fy0;
        wfx[t] = X - fx0;
        wfy[t] = Y - fy0;
        const int c0 = clampi_(xa, 0, W - 1), c1 = clampi_(xa + 1, 0, W - 1);
        const float* r0 = I1 + (size_t)clampi_(ya, 0, H - 1) * W;
        const float* r1 = I1 + (size_t)clampi_(ya + 1, 0, H - 1) * W;
        ta[t] = r0[c0];
        tb[t] = r0[c1];
        tc[t] = r1[c0];
        td[t] = r1[c1];
    }
#pragma unroll
    for (int t = 0; t < NF; ++t) {
        const int k = tid + 256 * t;
        if (k >= kFW * kFH) break;
        const int ly = k / kFW, lx = k - ly * kFW;
        const float fx = wfx[t], fy = wfy[t];
        if (ly >= 3 && ly < kLH + 5 && lx >= 3 && lx < kLW + 5) sF[ly - 3][lx - 3] = f[t];
        const float top = (1.0f - fx) * ta[t] + fx * tb[t];
        const float bot = (1.0f - fx) * tc[t] + fx * td[t];
        sI[ly][lx] = (1.0f - fy) * top + fy * bot;
    }
    // 2. I0x, I0y over the tile +-2
#pragma unroll
    for (int t = 0; t < NG; ++t) {
        const int k = tid + 256 * t;
        if (k >= kGW * kGH) break;
        const int ly = k / kGW, lx = k - ly * kGW;
        sGx[ly][lx] = gx0[t];
        sGy[ly][lx] = gy0[t];
    }
    __syncthreads();
    // 3. Wx, Wy over the tile +-2; smoothness weights (forward differences, 0
    //    at the last column / row) over the tile + left column / top row
    for (int k = tid; k < kGW * kGH; k += 256) {
        const int ly = k / kGW, lx = k - ly * kGW;
        const int ix = clampi_(x0 - 2 + lx, 0, W - 1) - x0 + 4, iy = clampi_(y0 - 2 + ly, 0, H - 1) - y0 + 4;
        sWx[ly][lx] = d5(sI[iy][ix - 2], sI[iy][ix - 1], sI[iy][ix + 1], sI[iy][ix + 2]);
        sWy[ly][lx] = d5(sI[iy - 2][ix], sI[iy - 1][ix], sI[iy + 1][ix], sI[iy + 2][ix]);
    }
    for (int k = tid; k < kSW * kSH; k += 256) {
        const int ly = k / kSW, lx = k - ly * kSW;
        const int x = x0 - 1 + lx, y = y0 - 1 + ly;
        if (x < 0 || y < 0 || x >= W || y >= H) continue;  // never read
        const int fx = lx, fy = ly;  // sF index of (x, y)
        const float uc = sF[fy][fx].x, vc = sF[fy][fx].y;
        float gxu = 0.0f, gxv = 0.0f, gyu = 0.0f, gyv = 0.0f;
        if (x < W - 1) {
            gxu = sF[fy][fx + 1].x - uc;
            gxv = sF[fy][fx + 1].y - vc;
        }
        if (y < H - 1) {
            gyu = sF[fy + 1][fx].x - uc;
            gyv = sF[fy + 1][fx].y - vc;
        }
        sS[ly][lx] = kAlpha / sqrtf((((gxu * gxu + gyu * gyu) + gxv * gxv) + gyv * gyv) + kEps2);
    }
    __syncthreads();
    // 4. per pixel: the data weights at the current flow and the normal
    //    equations of the linearised energy in (du, dv)
#pragma unroll
    for (int t = 0; t < NP; ++t) {
        const int k = tid + 256 * t;
        const int ly = k / kLW, lx = k - ly * kLW;
        const int x = x0 + lx, y = y0 + ly;
        if (x >= W || y >= H) continue;
        const int gx = lx + 2, gy = ly + 2, fx = lx + 1, fy = ly + 1;
        const size_t i = (size_t)y * W + x;
        const float wx = sWx[gy][gx], wy = sWy[gy][gx], i0x = sGx[gy][gx], i0y = sGy[gy][gx];
        const float Ix = 0.5f * (wx + i0x);
        const float Iy = 0.5f * (wy + i0y);
        const float Iz = sI[ly + 4][lx + 4] - i0p[t];
        const float Ixx = 0.5f * (d5(sWx[gy][gx - 2], sWx[gy][gx - 1], sWx[gy][gx + 1], sWx[gy][gx + 2]) +
                                  d5(sGx[gy][gx - 2], sGx[gy][gx - 1], sGx[gy][gx + 1], sGx[gy][gx + 2]));
        const float Ixy = 0.5f * (d5(sWx[gy - 2][gx], sWx[gy - 1][gx], sWx[gy + 1][gx], sWx[gy + 2][gx]) +
                                  d5(sGx[gy - 2][gx], sGx[gy - 1][gx], sGx[gy + 1][gx], sGx[gy + 2][gx]));
        const float Iyy = 0.5f * (d5(sWy[gy - 2][gx], sWy[gy - 1][gx], sWy[gy + 1][gx], sWy[gy + 2][gx]) +
                                  d5(sGy[gy - 2][gx], sGy[gy - 1][gx], sGy[gy + 1][gx], sGy[gy + 2][gx]));
        const float Ixz = wx - i0x;
        const float Iyz = wy - i0y;
        const float psiI = kDelta / sqrtf(Iz * Iz + kEps2);
        const float psiG = kGamma / sqrtf((Ixz * Ixz + Iyz * Iyz) + kEps2);
        const float A11 = (psiI * (Ix * Ix) + psiG * (Ixx * Ixx + Ixy * Ixy)) + kZeta;
        const float A12 = psiI * (Ix * Iy) + psiG * (Ixx * Ixy + Ixy * Iyy);
        const float A22 = (psiI * (Iy * Iy) + psiG * (Ixy * Ixy + Iyy * Iyy)) + kZeta;
        const float s = sS[ly + 1][lx + 1];
        const float wl = x > 0 ? sS[ly + 1][lx] : 0.0f, wr = x < W - 1 ? s : 0.0f;
        const float wu = y > 0 ? sS[ly][lx + 1] : 0.0f, wd = y < H - 1 ? s : 0.0f;
        const float2 fc = sF[fy][fx];
        const float2 fl_ = x > 0 ? sF[fy][fx - 1] : fc, fr = x < W - 1 ? sF[fy][fx + 1] : fc;
        const float2 fu = y > 0 ? sF[fy - 1][fx] : fc, fd = y < H - 1 ? sF[fy + 1][fx] : fc;
        const float u = fc.x, v = fc.y;
        const float su = ((wl * (fl_.x - u) + wr * (fr.x - u)) + wu * (fu.x - u)) + wd * (fd.x - u);
        const float sv = ((wl * (fl_.y - v) + wr * (fr.y - v)) + wu * (fu.y - v)) + wd * (fd.y - v);
        const float sumw = ((wl + wr) + wu) + wd;
        plane(L, pr, P_B1)[i] = su - (psiI * (Iz * Ix) + psiG * (Ixz * Ixx + Iyz * Ixy));
        plane(L, pr, P_B2)[i] = sv - (psiI * (Iz * Iy) + psiG * (Ixz * Ixy + Iyz * Iyy));
        plane(L, pr, P_A12)[i] = A12;
        plane(L, pr, P_D1)[i] = A11 + sumw;
        plane(L, pr, P_D2)[i] = A22 + sumw;
        plane(L, pr, P_SW)[i] = s;
    }
}

// ---------------------------------------------------------------------------
// red-black SOR, all sweeps of one fixed-point iteration per tile
constexpr int kSQ = 64;                  // pixel pairs (even x, odd x) per region row: one wave per row
constexpr int kSRH = 64;                 // region rows
constexpr int kSHX = 10, kSHY = 9;       // halo (even in x: pairs start at even x)
constexpr int kSTW = 2 * kSQ - 2 * kSHX; // 108 output columns
constexpr int kSTH = kSRH - 2 * kSHY;    // 46 output rows
constexpr int kSWaves = 16;
constexpr int kSRows = kSRH / kSWaves;   // region rows per wave
static_assert(kSHY >= 2 * kVarRefSor - 1 && kSHX >= 2 * kVarRefSor - 1, "SOR halo: one pixel per half-sweep after the first");

// one pixel's equation: the SOR update reads its 4 neighbours of the other
// colour; at the image border the neighbour is the pixel itself (weight 0).
// r1, r2 = RN(1 / d1), RN(1 / d2): each of the pixel's 5 updates divides by
// the same d1, d2, so the division is div_pre (correctly rounded from the
// reciprocal, dis_device.h) instead of the IEEE sequence; numerators below
// 2^-60 (whose remainders could leave the normal range) take IEEE division.
// The left smoothness weight is the left pixel's own (its s), which the lane
// holds (odd pixel) or lane q - 1 holds (even pixel), so it is not stored.
struct SorPx {
    float b1, b2, a12, d1, d2, r1, r2, s, su;
};

// lane q - 1's / q + 1's value (DPP wave shifts); 0 past the wave's ends,
// which is the region's zero border
__device__ __forceinline__ float from_left(float v)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xF, 0xF, true));  // wave_shr:1
}
__device__ __forceinline__ float from_right(float v)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xF, 0xF, true));  // wave_shl:1
}

// One wave per region row (rows wv + 16 j), lane q = pixel pair (2q, 2q + 1):
// a pixel's left / right neighbours are in the same wave, so du, dv live in
// registers and reach the neighbours by DPP; only the rows above / below go
// through LDS (sU / sV, written after each update, read after the barrier).
// A region row at distance d from the tile's rows matters for the tile after
// the last half-sweep only while (half-sweep index h, 1-based) + d <= 2 *
// VR_SOR: a row skipped at half-sweep h is wrong afterwards, and that reaches
// the tile at half-sweep h + d. Skipping the rows past that (wave-uniform)
// leaves every value the tile depends on as it was; the rest of the halo is
// wrong either way.
// kInt: every pixel of the region and its 4 neighbours inside the image (no
// border masks; most tiles of a level)
template <bool kInt>
__device__ __forceinline__ void sor_tile(const Lvl& L, float (&sU)[2][kSRH + 2][kSQ + 2],
                                         float (&sV)[2][kSRH + 2][kSQ + 2], int q, int wv, int xs, int ys, int pr)
{
    const int W = L.W, H = L.H;
    SorPx P[kSRows][2];
    float U[kSRows][2], V[kSRows][2];
    const float* B1 = plane(L, pr, P_B1);
    const float* B2 = plane(L, pr, P_B2);
    const float* A12 = plane(L, pr, P_A12);
    const float* D1 = plane(L, pr, P_D1);
    const float* D2 = plane(L, pr, P_D2);
    const float* SW = plane(L, pr, P_SW);
#pragma unroll
    for (int j = 0; j < kSRows; ++j) {
        const int y = ys + wv + kSWaves * j;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            SorPx& p = P[j][c];
            const int x = xs + 2 * q + c;
            const bool in = kInt || (x >= 0 && x < W && y >= 0 && y < H);
            p.b1 = p.b2 = p.a12 = 0.0f;
            p.d1 = p.d2 = 1.0f;
            p.s = p.su = 0.0f;
            U[j][c] = V[j][c] = 0.0f;
            if (in) {
                const size_t i = (size_t)y * W + x;
                p.b1 = B1[i];
                p.b2 = B2[i];
                p.a12 = A12[i];
                p.d1 = D1[i];
                p.d2 = D2[i];
                p.s = SW[i];
                p.su = (kInt || y > 0) ? SW[i - W] : 0.0f;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < kSRows; ++j)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            P[j][c].r1 = 1.0f / P[j][c].d1;
            P[j][c].r2 = 1.0f / P[j][c].d2;
        }
    __syncthreads();  // (the caller's zero fill of sU / sV)
    for (int sweep = 0; sweep < kVarRefSor; ++sweep) {
#pragma unroll
        for (int colour = 0; colour < 2; ++colour) {
            const int h = 2 * sweep + colour + 1;
#pragma unroll
            for (int j = 0; j < kSRows; ++j) {
                const int r = wv + kSWaves * j;  // region row (wave-uniform)
                const int d = max(max(kSHY - r, r - (kSHY + kSTH - 1)), 0);
                if (h + d > 2 * kVarRefSor) continue;
                const int y = ys + r;
                // the pixel of this colour in the pair: x parity = c, (x + y) & 1 == colour
                const int cpar = (colour ^ y) & 1;
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    if (c != cpar) continue;
                    const SorPx& p = P[j][c];
                    const int x = xs + 2 * q + c;
                    const bool in = kInt || (x >= 0 && x < W && y >= 0 && y < H);
                    const bool hl = kInt || x > 0, hr = kInt || x < W - 1, hu = kInt || y > 0, hd = kInt || y < H - 1;
                    const float du = U[j][c], dv = V[j][c];
                    // same row: the pair's other pixel and the neighbouring pair's
                    const float ul0 = c == 0 ? from_left(U[j][1]) : U[j][0];
                    const float ur0 = c == 0 ? U[j][1] : from_right(U[j][0]);
                    const float vl0 = c == 0 ? from_left(V[j][1]) : V[j][0];
                    const float vr0 = c == 0 ? V[j][1] : from_right(V[j][0]);
                    const float sl = c == 0 ? from_left(P[j][1].s) : P[j][0].s;
                    const float wl = hl ? sl : 0.0f, wr = hr ? p.s : 0.0f;
                    const float wu = hu ? p.su : 0.0f, wd = hd ? p.s : 0.0f;
                    const float ul = hl ? ul0 : du, ur = hr ? ur0 : du;
                    const float uu = hu ? sU[c][r][q + 1] : du, ud = hd ? sU[c][r + 2][q + 1] : du;
                    const float vl = hl ? vl0 : dv, vr = hr ? vr0 : dv;
                    const float vu = hu ? sV[c][r][q + 1] : dv, vd = hd ? sV[c][r + 2][q + 1] : dv;
                    const float sdu = ((wl * ul + wr * ur) + wu * uu) + wd * ud;
                    const float nu = (1.0f - kOmega) * du + kOmega * sor_div((p.b1 + sdu) - p.a12 * dv, p.d1, p.r1);
                    const float sdv = ((wl * vl + wr * vr) + wu * vu) + wd * vd;
                    const float nv = (1.0f - kOmega) * dv + kOmega * sor_div((p.b2 + sdv) - p.a12 * nu, p.d2, p.r2);
                    // pixels outside the image keep du = dv = 0 (their cells are never read as
                    // neighbours: the border masks above select the pixel itself)
                    U[j][c] = in ? nu : du;
                    V[j][c] = in ? nv : dv;
                    sU[c][r + 1][q + 1] = U[j][c];
                    sV[c][r + 1][q + 1] = V[j][c];
                }
            }
            __syncthreads();
        }
    }
    // flow += (du, dv) on the tile
    float2* fl = L.flow + (size_t)pr * L.flow_stride;
#pragma unroll
    for (int j = 0; j < kSRows; ++j) {
        const int r = wv + kSWaves * j;
        if (r < kSHY || r >= kSHY + kSTH) continue;
        const int y = ys + r;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const int lx = 2 * q + c - kSHX, x = xs + 2 * q + c;
            if (lx < 0 || lx >= kSTW || (!kInt && !(x >= 0 && x < W && y >= 0 && y < H))) continue;
            float2* f = fl + (size_t)y * W + x;
            const float2 v = *f;
            *f = make_float2(v.x + U[j][c], v.y + V[j][c]);
        }
    }
}

__global__ void __launch_bounds__(1024) k_vr_sor(Lvl L)
{
    // [column parity][region row + 1][pair + 1]; border cells stay 0
    __shared__ float sU[2][kSRH + 2][kSQ + 2], sV[2][kSRH + 2][kSQ + 2];
    const Tile bt = xcd_tile();
    const int W = L.W, H = L.H, pr = bt.z, tid = threadIdx.x;
    const int q = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int x0 = bt.x * kSTW, y0 = bt.y * kSTH;
    const int xs = x0 - kSHX, ys = y0 - kSHY;  // xs even
    for (int k = tid; k < 2 * (kSRH + 2) * (kSQ + 2); k += 1024) {
        (&sU[0][0][0])[k] = 0.0f;
        (&sV[0][0][0])[k] = 0.0f;
    }
    if (xs >= 1 && xs + 2 * kSQ <= W - 1 && ys >= 1 && ys + kSRH <= H - 1)
        sor_tile<true>(L, sU, sV, q, wv, xs, ys, pr);
    else
        sor_tile<false>(L, sU, sV, q, wv, xs, ys, pr);
}

}  // namespace

hipError_t launch_var_refine(const VarRefArgs& a, int n, hipStream_t s, VarRefTiming tfn, void* tctx)
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
    if (a.W <= 0 || a.H <= 0 || (long long)a.W * a.H > a.ws_plane || a.ws_stride < kVarRefPlanes * a.ws_plane)
        return hipErrorInvalidValue;
    const unsigned nn = (unsigned)n;
    hipLaunchKernelGGL(k_vr_d0, dim3((a.W + 63) / 64, (a.H + 3) / 4, nn), dim3(256), 0, s, L);
    const dim3 glin((a.W + kLW - 1) / kLW, (a.H + kLH - 1) / kLH, nn);
    const dim3 gsor((a.W + kSTW - 1) / kSTW, (a.H + kSTH - 1) / kSTH, nn);
    for (int it = 0; it < a.iters; ++it) {
        const Timing tl = tfn ? tfn(tctx, 0) : Timing{};
        DIS_LAUNCH(tl, k_vr_lin, glin, dim3(256), 0, s, L);
        const Timing ts = tfn ? tfn(tctx, 1) : Timing{};
        DIS_LAUNCH(ts, k_vr_sor, gsor, dim3(1024), 0, s, L);
    }
    return hipGetLastError();
}

}  // namespace dis
