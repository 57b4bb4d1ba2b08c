// dis_search_wave.hip -- the north star's mapping of the patch search: one
// wave64 per 8x8 patch, lane = pixel (column c = lane / 8, row j = lane % 8),
// the patch's 21 x 21 target window staged in LDS, the reductions across
// lanes. Same arithmetic as k_search8 (src/patch.cpp:31-267,
// src/patch_grid.cpp:108-119), bit-exact, selected by dis_set_kernel_variant 6.
//
// Eigen's order (A_c = sequential sum down column c, then
// ((A0+A4)+(A2+A6))+((A1+A5)+(A3+A7))) makes each reduction a 7-step dependent
// chain across the column's lanes (DPP row_shr:1) plus 8 readlanes: ~30
// instructions per sum, three sums per update, for ONE patch per wave -- ~150
// wave instructions per patch-update against ~16 at 2 lanes per patch
// (measured 11x slower on the big levels, so the auto choice
// never picks it).
#include "dis_device.h"
#include "dis_kernels.h"

namespace dis {

namespace {

constexpr int kWaveWin = 21;  // window rows / columns: floor(start) -10 .. +10

__device__ __forceinline__ float row_shr1(float v)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x111, 0xF, 0xF, false));  // row_shr:1
}

// Eigen-order sum over the wave's 64 lanes (lane = 8 c + j holds pixel (j, c));
// the result is wave-uniform
__device__ __forceinline__ float wave_patch_sum(float v, int j)
{
    float s = v;
#pragma unroll
    for (int k = 1; k < 8; ++k) {
        const float t = row_shr1(s) + v;  // lane j: S_{j-1} + v_j
        s = j == k ? t : s;
    }
    float A[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) A[c] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(s), 8 * c + 7));
    return ((A[0] + A[4]) + (A[2] + A[6])) + ((A[1] + A[5]) + (A[3] + A[7]));
}

// grid: (ceil(npw * nph / 4), batch), 4 waves (patches) per workgroup, exact
// arithmetic only (the runtime uses it for exact, non-paper, virtual-padding
// levels; the compat and tolerance paths keep their kernels)
__global__ void __launch_bounds__(256) k_search_wave(Search8Args a)
{
    __shared__ float win_all[4][kWaveWin * kWaveWin];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int p = blockIdx.x * 4 + wave;  // patch id, x-major (src/patch_grid.cpp:39-50)
    const int pair = blockIdx.y;
    if (p >= a.npw * a.nph) return;  // whole wave; no workgroup barrier below
    float* const win = win_all[wave];
    const int gx = p / a.nph, gy = p - gx * a.nph;
    const int st = a.steps, W = a.W, H = a.H;
    const int irx = gx * st + a.offw, iry = gy * st + a.offh;
    const float rx = (float)irx, ry = (float)iry;
    const int c = lane >> 3, j = lane & 7;
    const float* I0 = a.img0 + (size_t)pair * a.plane_stride + a.plane_off;
    const float* I1 = a.img1 + (size_t)pair * a.plane_stride + a.plane_off;

    // template gradients at pixel (irx-4+c, iry-4+j): Sobel (ksize 3, 1/8,
    // reflect-101) of the level image, zero outside it (src/main.cpp:34-47)
    const int px = irx - 4 + c, py = iry - 4 + j;
    float R[3], S[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float* row = I0 + (size_t)clampi(reflect101(py - 1 + k, H), 0, H - 1) * W;
        const float l = row[clampi(reflect101(px - 1, W), 0, W - 1)];
        const float m = row[clampi(reflect101(px, W), 0, W - 1)];
        const float r = row[clampi(reflect101(px + 1, W), 0, W - 1)];
        R[k] = r - l;
        S[k] = m * 0.25f + (l + r) * 0.125f;
    }
    const bool in = px >= 0 && px < W && py >= 0 && py < H;
    const float gdx = in ? R[1] * 0.25f + (R[0] + R[2]) * 0.125f : 0.0f;
    const float gdy = in ? S[2] - S[0] : 0.0f;
    const LU2 lu = hessian_lu2(wave_patch_sum(gdx * gdx, j), wave_patch_sum(gdx * gdy, j),
                               wave_patch_sum(gdy * gdy, j));

    // initialisation from the coarser level (src/patch_grid.cpp:108-119)
    float ix = 0.0f, iy = 0.0f;
    if (a.dense_coarse) {
        const float2 d = a.dense_coarse[(size_t)pair * a.dense_stride + (size_t)(iry >> 1) * (W / 2) + (irx >> 1)];
        ix = d.x * 2;
        iy = d.y * 2;
    } else if (a.u_coarse) {
        const float2 d = dense_at(a.u_coarse + (size_t)pair * a.u_stride, a.c_npw, a.c_nph, a.c_offw, a.c_offh, st, 4,
                                  irx >> 1, iry >> 1);
        ix = d.x * 2;
        iy = d.y * 2;
    }
    const float sx = rx + ix, sy = ry + iy;
    float u0 = ix, u1 = iy;
    if (!(sx < a.tmp_lb || sy < a.tmp_lb || sx > a.tmp_ub_w || sy > a.tmp_ub_h)) {
        // the patch's window: every tap lies in floor(start) -9 .. +9 (search_block 4)
        const int tx0 = (int)floorf(sx) - 10, ty0 = (int)floorf(sy) - 10;
        for (int i = lane; i < kWaveWin * kWaveWin; i += 64) {
            const int r = i / kWaveWin, cc = i - r * kWaveWin;
            win[i] = I1[(size_t)clampi(ty0 + r, 0, H - 1) * W + clampi(tx0 + cc, 0, W - 1)];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const float r00 = 1.0f / lu.u00, r11 = 1.0f / lu.u11;
        float pxs = sx, pys = sy;
        for (int counter = 1;; ++counter) {
            const Warp w = warp_coefs(pxs, pys);
            // pixel (j, c): A = (Y-4+j, X-4+c), B = A-1, C = A-row, D = C-1 (src/patch.cpp:247-261)
            const float* b = win + (w.Y - 5 + j - ty0) * kWaveWin + (w.X - 5 + c - tx0);
            float r = w.w3 * b[kWaveWin + 1];
            r = r + w.w2 * b[kWaveWin];
            r = r + w.w1 * b[1];
            r = r + w.w0 * b[0];
            if (a.norm) r = r - wave_patch_sum(r, j) / 64.0f;
            const float b0 = wave_patch_sum(gdx * r, j), b1 = wave_patch_sum(gdy * r, j);
            float c0 = lu.swap ? b1 : b0, c1 = lu.swap ? b0 : b1;
            c1 = c1 - lu.l10 * c0;
            c1 = div_pre(c1, lu.u11, r11);
            c0 = c0 - c1 * lu.u01;
            const float d0 = div_pre(c0, lu.u00, r00), d1 = c1;
            u0 = u0 - d0;
            u1 = u1 - d1;
            pxs = rx + u0;
            pys = ry + u1;
            const float ex = sx - pxs, ey = sy - pys;
            const float s2 = ex * ex + ey * ey;
            if (s2 > a.thr_sq || s2 != s2 || pxs < a.tmp_lb || pys < a.tmp_lb || pxs > a.tmp_ub_w ||
                pys > a.tmp_ub_h) {
                u0 = ix;
                u1 = iy;
                break;
            }
            if (counter > a.iters) break;
        }
    }
    if (lane == 0) a.u_out[(size_t)pair * a.u_stride + p] = make_float2(u0, u1);
}

}  // namespace

hipError_t launch_search_wave(const Search8Args& a, int batch, hipStream_t s, Timing t)
{
    if (a.paper || a.fma || a.gdx_plane) return hipErrorInvalidValue;
    const dim3 grid((unsigned)((a.npw * a.nph + 3) / 4), batch);
    DIS_LAUNCH(t, k_search_wave, grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace dis
