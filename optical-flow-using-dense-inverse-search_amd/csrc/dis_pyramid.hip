// dis_pyramid.hip -- K1+K2 as two streaming kernels (no LDS staging of the
// frames, no workgroup barriers on the bandwidth-heavy part):
//
//   k_pyr12: u8 frame -> (virtual) pad -> level-0 Sobel magnitude -> levels 1
//            and 2, straight from global memory. One lane = one level-2 pixel
//            = a 4x4 block of level-0 magnitudes from its 6x6 u8 window
//            (src/main.cpp:16-30, 139-160); a wave covers 64 consecutive
//            level-2 pixels of one row, so its u8 row loads are one dword per
//            lane (256 contiguous bytes) and the window's halo columns come
//            from the neighbour lanes (DPP wave shifts); its level-1 stores
//            are 8 contiguous bytes per lane (512 B per row), level 2 one
//            float per lane.
//   k_pyr_tail: levels 3..L (L <= 6) from level 2, one wave per 2^(L-2)
//            square of level-2 pixels, intermediate levels in LDS.
//
// Arithmetic is that of k_pyramid (dis_frontback.hip) and of the oracle:
// integer Sobel (exact for u8 input), the magnitude sqrtf(N / 64) as
// sqrt_cr(N) / 8 (correctly rounded), 2x2 means (((a + b) + c) + d) * 0.25
// with a, b the top row -- bit-identical planes.
#include "dis_device.h"
#include "dis_kernels.h"

namespace dis {

namespace {

typedef short short2p __attribute__((ext_vector_type(2)));

// 16-bit lanes (lo, hi) = (byte I, byte J) of the 8 bytes {w1:w0}
template <int I, int J>
__device__ __forceinline__ short2p bytes2(unsigned w0, unsigned w1)
{
    constexpr unsigned sel = 0x0c000c00u | (unsigned)I | ((unsigned)J << 16);
    return __builtin_bit_cast(short2p, __builtin_amdgcn_perm(w1, w0, sel));
}

// DPP wave shifts (gfx9): lane i receives lane i-1 (shr) / i+1 (shl); the
// lanes shifted in from outside the wave keep `old`
__device__ __forceinline__ unsigned wave_shr1(unsigned v, unsigned old)
{
    return (unsigned)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xF, 0xF, false);
}
__device__ __forceinline__ unsigned wave_shl1(unsigned v, unsigned old)
{
    return (unsigned)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x130, 0xF, 0xF, false);
}

// u8 source byte of padded level-0 pixel (x, y): replicate padding to Wp x Hp
// (floor/ceil split, src/main.cpp:139-155) composed with Sobel's reflect-101
// at the Wp x Hp border (src/main.cpp:19-20)
__device__ __forceinline__ int src_row(const PyramidArgs& a, int y)
{
    return clampi(reflect101(y, a.Hp) - a.pt, 0, a.H - 1);
}
__device__ __forceinline__ int src_col(const PyramidArgs& a, int x)
{
    return clampi(reflect101(x, a.Wp) - a.pl, 0, a.W - 1);
}

}  // namespace

// grid: (ceil(W2 / 64), H2, 2 * batch) waves of 64 lanes; z = 2 * pair + frame
__global__ void __launch_bounds__(64) k_pyr12(PyramidArgs a)
{
    const int lane = threadIdx.x;
    const int W2 = a.w[2];
    const int y2 = blockIdx.y;
    const int x2 = blockIdx.x * 64 + lane;
    const int pair = blockIdx.z >> 1, frame = blockIdx.z & 1;
    if (blockIdx.x == 0 && y2 == 0 && blockIdx.z == 0 && lane < a.nzero) a.zero[lane] = 0;
    const uint8_t* in = (frame ? a.I1 : a.I0) + (size_t)pair * a.pair_stride;
    const bool inx = x2 < W2;
    const int xc = inx ? x2 : W2 - 1;  // idle lanes mirror the last column (their loads stay in bounds)
    // window: level-0 columns x0 - 1 .. x0 + 4, rows 4 y2 - 1 .. 4 y2 + 4
    const int x0 = 4 * xc;
    // body dword: the window's columns x0 .. x0 + 3 are source columns
    // x0 - pl .. x0 - pl + 3 (no clamping; dword_ok: aligned); the halo columns
    // are then the neighbour lanes' body bytes (DPP wave shifts), except at the
    // wave's ends, the plane's edges (reflect-101) and the padding (clamping),
    // where the lane loads its halo byte itself
    const bool body = a.dword_ok && x0 >= a.pl && x0 + 3 - a.pl <= a.W - 1;
    const bool nb_l = body && lane > 0 && x0 - 4 >= a.pl;
    const bool nb_r = body && lane < 63 && x0 + 7 - a.pl <= a.W - 1 && x2 + 1 < W2;
    short2p X[6][4];
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        const uint8_t* row = in + (size_t)src_row(a, 4 * y2 - 1 + r) * a.stride;
        unsigned wm;
        if (body) {
            wm = *reinterpret_cast<const unsigned*>(row + x0 - a.pl);
        } else {  // padding columns, unaligned frames: bytes
            wm = (unsigned)row[src_col(a, x0)] | ((unsigned)row[src_col(a, x0 + 1)] << 8) |
                 ((unsigned)row[src_col(a, x0 + 2)] << 16) | ((unsigned)row[src_col(a, x0 + 3)] << 24);
        }
        unsigned wl = wave_shr1(wm, 0u), wr = wave_shl1(wm, 0u);
        if (!nb_l) wl = (unsigned)row[src_col(a, x0 - 1)] << 24;
        if (!nb_r) wr = (unsigned)row[src_col(a, x0 + 4)];
        // window columns 0..5 = byte 3 of wl, bytes 0..3 of wm, byte 0 of wr,
        // each broadcast to both 16-bit lanes
        const short2p B[6] = {bytes2<3, 3>(wl, wm), bytes2<4, 4>(wl, wm), bytes2<5, 5>(wl, wm),
                              bytes2<6, 6>(wl, wm), bytes2<7, 7>(wl, wm), bytes2<4, 4>(wm, wr)};
        // (R, T) = (v[c+2] - v[c], 2 v[c+1] + v[c] + v[c+2]) per column c
        const short2p cm11 = {-1, 1}, c02 = {0, 2};
#pragma unroll
        for (int c = 0; c < 4; ++c) X[r][c] = B[c] * cm11 + (B[c + 1] * c02 + B[c + 2]);
    }
    // level-0 magnitudes x 8: q = (k1, k2) = (2 R1 + R0 + R2, T2 - T0), N = k1^2 + k2^2
    float m[4][4];
    const short2p c20 = {2, 0}, c1m1 = {1, -1};
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const short2p q = X[r + 1][c] * c20 + (X[r][c] * c1m1 + X[r + 2][c]);
            int n;
            __asm__("v_dot2_i32_i16 %0, %1, %1, 0" : "=v"(n) : "v"(q));
            m[r][c] = sqrt_cr((float)n);
        }
    if (!inx) return;
    float* planes = (frame ? a.img1 : a.img0) + (size_t)pair * a.plane_stride;
    if (a.write_l0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float4 v = make_float4(m[r][0] * 0.125f, m[r][1] * 0.125f, m[r][2] * 0.125f, m[r][3] * 0.125f);
            *reinterpret_cast<float4*>(planes + (size_t)(4 * y2 + r) * a.Wp + x0) = v;
        }
    }
    // level 1: ((m00 + m01) + m10) + m11 of the 8x-scaled magnitudes x 2^-5
    // (= the reference's 2x2 mean of the unscaled ones: powers of two commute
    // with the roundings); level 2: the 2x2 mean of level 1
    float l1[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            float s = m[2 * i][2 * j] + m[2 * i][2 * j + 1];
            s = s + m[2 * i + 1][2 * j];
            s = s + m[2 * i + 1][2 * j + 1];
            l1[i][j] = s * 0.03125f;
        }
    float* p1 = planes + a.off[1] + (size_t)(2 * y2) * a.w[1] + 2 * x2;
    *reinterpret_cast<float2*>(p1) = make_float2(l1[0][0], l1[0][1]);
    *reinterpret_cast<float2*>(p1 + a.w[1]) = make_float2(l1[1][0], l1[1][1]);
    float s = l1[0][0] + l1[0][1];
    s = s + l1[1][0];
    s = s + l1[1][1];
    planes[a.off[2] + (size_t)y2 * W2 + x2] = s * 0.25f;
}

// grid: (W2 / T2, H2 / T2, 2 * batch), T2 = 2^(L-2) level-2 pixels per tile
// edge; one wave per tile computes levels 3..L in LDS
template <int L>
__global__ void __launch_bounds__(64) k_pyr_tail(PyramidArgs a)
{
    constexpr int T2 = 1 << (L - 2), N2 = T2 * T2;
    constexpr int PER = (N2 + 63) / 64;
    __shared__ float buf[2][N2 / 4];  // level l at buf[l & 1]
    __shared__ float src[N2];         // the level-2 tile
    const int lane = threadIdx.x;
    const int pair = blockIdx.z >> 1, frame = blockIdx.z & 1;
    float* planes = (frame ? a.img1 : a.img0) + (size_t)pair * a.plane_stride;
    const int tx = blockIdx.x * T2, ty = blockIdx.y * T2;  // level-2 tile origin
    const float* p2 = planes + a.off[2] + (size_t)ty * a.w[2] + tx;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int i = lane + 64 * k;
        if (i < N2) src[i] = p2[(size_t)(i / T2) * a.w[2] + (i % T2)];
    }
    __syncthreads();
    const float* cur = src;
#pragma unroll
    for (int l = 3; l <= L; ++l) {
        const int ns = T2 >> (l - 3), nd = ns / 2;
        float* nxt = buf[l & 1];
        for (int k = lane; k < nd * nd; k += 64) {
            const int y = k / nd, x = k - y * nd;
            const float* p = cur + (2 * y) * ns + 2 * x;
            float s = p[0] + p[1];
            s = s + p[ns];
            s = s + p[ns + 1];
            const float v = s * 0.25f;
            nxt[k] = v;
            planes[a.off[l] + (size_t)((ty >> (l - 2)) + y) * a.w[l] + (tx >> (l - 2)) + x] = v;
        }
        __syncthreads();
        cur = nxt;
    }
}

// Whether the two-kernel pyramid applies: at least levels 1..2 in-kernel and
// a padded size the level-2 grid and the tail tiles divide.
bool pyramid2_fits(const PyramidArgs& a)
{
    return a.levels >= 2 && a.levels <= 6 && a.Wp % (1 << a.levels) == 0 && a.Hp % (1 << a.levels) == 0;
}

hipError_t launch_pyramid2(const PyramidArgs& a, int batch, hipStream_t s, Timing t)
{
    if (!pyramid2_fits(a) || a.nzero > 64) return hipErrorInvalidValue;
    const int W2 = a.Wp >> 2, H2 = a.Hp >> 2;
    if (a.w[2] != W2) return hipErrorInvalidValue;
    DIS_LAUNCH(t, k_pyr12, dim3((W2 + 63) / 64, H2, 2 * batch), dim3(64), 0, s, a);
    if (a.levels >= 3) {
        const int T2 = 1 << (a.levels - 2);
        const dim3 grid(W2 / T2, H2 / T2, 2 * batch);
        switch (a.levels) {
            case 3: hipLaunchKernelGGL(k_pyr_tail<3>, grid, dim3(64), 0, s, a); break;
            case 4: hipLaunchKernelGGL(k_pyr_tail<4>, grid, dim3(64), 0, s, a); break;
            case 5: hipLaunchKernelGGL(k_pyr_tail<5>, grid, dim3(64), 0, s, a); break;
            default: hipLaunchKernelGGL(k_pyr_tail<6>, grid, dim3(64), 0, s, a); break;
        }
    }
    return hipGetLastError();
}

}  // namespace dis
