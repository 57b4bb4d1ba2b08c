// dis_pyramid.hip -- K1+K2 as two streaming kernels (no LDS staging of the
// frames, no workgroup barriers on the bandwidth-heavy part):
//
//   k_pyr12: u8 frame -> (virtual) pad -> level-0 Sobel magnitude -> levels 1
//            and 2, straight from global memory. One lane = four consecutive
//            level-2 pixels = 4x4 blocks of level-0 magnitudes from a 6x18 u8
//            window (src/main.cpp:16-30, 139-160); a wave covers 256
//            consecutive level-2 pixels of one row, so its u8 row loads are
//            one 16-byte load per lane (1 KB contiguous) and the window's halo
//            columns come from the neighbour lanes (DPP wave shifts); its
//            level-1 and level-2 stores are 16-byte stores.
//   k_pyr_tail: levels 3..L (L <= 6) from level 2, one wave per 2^(L-2)
//            square of level-2 pixels, intermediate levels in LDS.
//
// Arithmetic is that of k_pyramid (dis_frontback.hip) and of the oracle:
// integer Sobel (exact for u8 input), the magnitude sqrtf(N / 64) as
// sqrt_cr(N) / 8 (correctly rounded), 2x2 means (((a + b) + c) + d) * 0.25
// with a, b the top row -- bit-identical planes.
#include <type_traits>

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

// Sobel magnitudes (x 8) of the 4x4 level-0 block whose 6x6 u8 window rows
// are the bytes (byte 3 of p, bytes 0..3 of m, byte 0 of n) of dwords p, m, n,
// then its level-1 2x2 block and level-2 pixel. Integer Sobel in packed 16-bit
// lanes (exact: |values| <= 1020): per window row and column c,
// X = (R, T) = (v[c+2] - v[c], 2 v[c+1] + v[c] + v[c+2]); per pixel
// q = (k1, k2) = (2 R1 + R0 + R2, T2 - T0) = X1 (2,0) + X0 (1,-1) + X2 and
// N = k1^2 + k2^2 = dot2(q, q), gx^2 + gy^2 = N / 64 exactly.
struct Block4 {
    float m[4][4];   // 8 x the level-0 magnitudes
    float l1[2][2];  // level 1
    float l2;        // level 2
};

template <int R0, int NR>
__device__ __forceinline__ void block4(const unsigned (&p)[NR], const unsigned (&m)[NR], const unsigned (&n)[NR],
                                       Block4& o)
{
    // rows streamed: X of three window rows live at a time, the magnitudes of
    // one level-1 row (two level-0 rows) at a time (bounded registers)
    const short2p cm11 = {-1, 1}, c02 = {0, 2}, c20 = {2, 0}, c1m1 = {1, -1};
    short2p X[3][4];
    auto xrow = [&](int r, short2p (&x)[4]) {
        const unsigned pr = p[R0 + r], mr = m[R0 + r], nr = n[R0 + r];
        const short2p B[6] = {bytes2<3, 3>(pr, mr), bytes2<4, 4>(pr, mr), bytes2<5, 5>(pr, mr),
                              bytes2<6, 6>(pr, mr), bytes2<7, 7>(pr, mr), bytes2<4, 4>(mr, nr)};
#pragma unroll
        for (int c = 0; c < 4; ++c) x[c] = B[c] * cm11 + (B[c + 1] * c02 + B[c + 2]);
    };
    xrow(0, X[0]);
    xrow(1, X[1]);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        xrow(r + 2, X[(r + 2) % 3]);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const short2p q = X[(r + 1) % 3][c] * c20 + (X[r % 3][c] * c1m1 + X[(r + 2) % 3][c]);
            int nn;
            __asm__("v_dot2_i32_i16 %0, %1, %1, 0" : "=v"(nn) : "v"(q));
            o.m[r][c] = sqrt_cr((float)nn);
        }
        if (r & 1) {
            // level 1: ((m00 + m01) + m10) + m11 of the 8x-scaled magnitudes x
            // 2^-5 (= the reference's 2x2 mean of the unscaled ones: powers of
            // two commute with the roundings)
            const int i = r >> 1;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                float s = o.m[2 * i][2 * j] + o.m[2 * i][2 * j + 1];
                s = s + o.m[2 * i + 1][2 * j];
                s = s + o.m[2 * i + 1][2 * j + 1];
                o.l1[i][j] = s * 0.03125f;
            }
        }
    }
    // level 2: the 2x2 mean of level 1
    float s = o.l1[0][0] + o.l1[0][1];
    s = s + o.l1[1][0];
    s = s + o.l1[1][1];
    o.l2 = s * 0.25f;
}

// grid: (ceil(W2 / 256), H2, 2 * batch) waves; z = 2 * pair + frame. Lane =
// 4 consecutive level-2 pixels of row y = level-0 columns x0 .. x0 + 15
// (x0 = 16 g), window columns x0 - 1 .. x0 + 16, rows 4 y - 1 .. 4 y + 4: the
// 2 halo rows are read once per level-2 row (6 rows per 4, 1.5x the frame
// bytes). Waves in plain order: every order that keeps a wave's vertical
// neighbours on its XCD (XCD remap, chunked remap, 2 / 4 / 8 stacked waves
// per workgroup) or carries the halo rows in registers (2 / 4 rows per wave)
// cut the bytes toward the algorithmic 300 MB per 32 pairs and lost time
// (DRAM locality, not bytes, sets this kernel's rate).
constexpr int kPyrRW = 1;  // level-2 rows per wave
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(5))) k_pyr12(PyramidArgs a)
{
    constexpr int RW = kPyrRW, NR = 4 * RW + 2;
    const int lane = threadIdx.x & 63;
    const int W2 = a.w[2], H2 = a.Hp >> 2;
    const int bx = blockIdx.x, bz = blockIdx.z, yb = blockIdx.y;
    const int y2b = RW * yb;  // first level-2 row of the wave
    const int g = bx * 64 + lane;  // lane's group of 4 level-2 pixels
    const int pair = bz >> 1, frame = bz & 1;
    if (bx == 0 && yb == 0 && bz == 0) {
        for (int i = lane; i < a.nzero; i += 64) a.zero[i] = 0;
    }
    const uint8_t* in = (frame ? a.I1 : a.I0) + (size_t)pair * a.pair_stride;
    const int ng = (W2 + 3) >> 2;                 // groups per row
    const int gc = g < ng ? g : ng - 1;           // idle lanes mirror the last group (loads stay in bounds)
    const int x0 = 16 * gc;
    // body: the window's columns x0 .. x0 + 15 are source columns x0 - pl ..
    // (no clamping; qword_ok: 16-byte aligned rows) -- one 16-byte load per
    // row; the halo columns are then the neighbour lanes' body bytes (DPP wave
    // shifts), except at the wave's ends, the plane's edges (reflect-101) and
    // the padding (clamping), where the lane loads its halo byte itself
    const bool body = a.qword_ok && x0 >= a.pl && x0 + 15 - a.pl <= a.W - 1;
    const bool nb_l = body && lane > 0 && x0 - 16 >= a.pl;
    const bool nb_r = body && lane < 63 && x0 + 31 - a.pl <= a.W - 1 && g + 1 < ng;
    unsigned d[4][NR], wl[NR], wr[NR];
    const uint8_t* rows[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) rows[r] = in + (size_t)src_row(a, 4 * y2b - 1 + r) * a.stride;
    // every row's load in flight before any is consumed (no branch between
    // them): the 16-byte body loads of all lanes (lanes without a body read a
    // harmless in-bounds 16 bytes, W >= 16), then the byte gathers of the
    // lanes that need them (exec-masked, all issued before the wait)
    if (a.qword_ok && a.W >= 16) {
        const int xb = body ? x0 - a.pl : 0;
        uint4 v[NR];
#pragma unroll
        for (int r = 0; r < NR; ++r) v[r] = *reinterpret_cast<const uint4*>(rows[r] + xb);
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            d[0][r] = v[r].x;
            d[1][r] = v[r].y;
            d[2][r] = v[r].z;
            d[3][r] = v[r].w;
        }
    }
    if (!body) {  // padding columns, unaligned frames: bytes
        uint8_t bb[NR][16];
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
            for (int k = 0; k < 16; ++k) bb[r][k] = rows[r][src_col(a, x0 + k)];
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
            for (int k = 0; k < 4; ++k)
                d[k][r] = (unsigned)bb[r][4 * k] | ((unsigned)bb[r][4 * k + 1] << 8) |
                          ((unsigned)bb[r][4 * k + 2] << 16) | ((unsigned)bb[r][4 * k + 3] << 24);
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        wl[r] = wave_shr1(d[3][r], 0u);
        wr[r] = wave_shl1(d[0][r], 0u);
    }
    if (!nb_l || !nb_r) {  // the wave's end lanes, the plane's edges, the padding
        const int cl = src_col(a, x0 - 1), cr = src_col(a, x0 + 16);
        uint8_t hl[NR], hr[NR];
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            hl[r] = rows[r][cl];
            hr[r] = rows[r][cr];
        }
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            if (!nb_l) wl[r] = (unsigned)hl[r] << 24;
            if (!nb_r) wr[r] = (unsigned)hr[r];
        }
    }
    if (g >= ng) return;
    float* planes = (frame ? a.img1 : a.img0) + (size_t)pair * a.plane_stride;
    const int np = min(4, W2 - 4 * g);  // level-2 pixels of this lane (the row's last group may be short)
    auto level_row = [&](auto rr_c) {
        constexpr int rr = decltype(rr_c)::value;  // level-2 row y2b + rr, window rows 4 rr ..
        const int y2 = y2b + rr;
        if (RW > 1 && y2 >= H2) return;
        float l1row[2][8], l2v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            Block4 o;
            block4<4 * rr, NR>(q == 0 ? wl : d[q - 1], d[q], q == 3 ? wr : d[q + 1], o);
            if (a.write_l0 && q < np) {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    *reinterpret_cast<float4*>(planes + (size_t)(4 * y2 + r) * a.Wp + x0 + 4 * q) =
                        make_float4(o.m[r][0] * 0.125f, o.m[r][1] * 0.125f, o.m[r][2] * 0.125f, o.m[r][3] * 0.125f);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                l1row[i][2 * q] = o.l1[i][0];
                l1row[i][2 * q + 1] = o.l1[i][1];
            }
            l2v[q] = o.l2;
        }
        float* p1 = planes + a.off[1] + (size_t)(2 * y2) * a.w[1] + 8 * g;
        float* p2 = planes + a.off[2] + (size_t)y2 * W2 + 4 * g;
        if (np == 4 && a.vec_st) {  // 16-byte stores: level-1 rows and the level-2 plane 16-byte aligned (W_2 % 4 == 0)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                *reinterpret_cast<float4*>(p1 + (size_t)i * a.w[1]) =
                    make_float4(l1row[i][0], l1row[i][1], l1row[i][2], l1row[i][3]);
                *reinterpret_cast<float4*>(p1 + (size_t)i * a.w[1] + 4) =
                    make_float4(l1row[i][4], l1row[i][5], l1row[i][6], l1row[i][7]);
            }
            *reinterpret_cast<float4*>(p2) = make_float4(l2v[0], l2v[1], l2v[2], l2v[3]);
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (q < np) {
                    p1[2 * q] = l1row[0][2 * q];
                    p1[2 * q + 1] = l1row[0][2 * q + 1];
                    p1[a.w[1] + 2 * q] = l1row[1][2 * q];
                    p1[a.w[1] + 2 * q + 1] = l1row[1][2 * q + 1];
                    p2[q] = l2v[q];
                }
        }
    };
    level_row(std::integral_constant<int, 0>{});
    if constexpr (RW > 1) level_row(std::integral_constant<int, 1>{});
    if constexpr (RW > 2) level_row(std::integral_constant<int, 2>{});
    if constexpr (RW > 3) level_row(std::integral_constant<int, 3>{});
}


// k_pyr_tail_reg<L, TPW>: the same levels 3..L without LDS or barriers. One
// wave per TPW horizontally adjacent 16 x 16 level-2 super-tiles; lane
// (qx, qy) = (lane & 7, lane >> 3) loads its 2 x 2 level-2 quad (two 8-byte
// loads) and forms its level-3 pixel in-lane; level 4 / 5 / 6 take the 2 x 2
// of the level below from the lanes 1 / 2 / 4 columns and 8 / 16 / 32 lanes
// away (DPP quad_perm and row_ror:8, ds_bpermute for the rest) -- the same
// ((a + b) + c) + d, a, b the top row, as k_pyr_tail, so bit-identical planes.
// Edge super-tiles (level-2 planes not a multiple of 16 wide / high, L < 6)
// load 0 outside the plane and store only in-plane pixels, whose sources are
// all in-plane (W_l = W_2 / 2^(l-2) exactly: pyramid2_fits).
namespace {
template <int X>
__device__ __forceinline__ float lane_xor(float v)
{
    if constexpr (X == 1) return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));
    else if constexpr (X == 2) return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, true));
    else if constexpr (X == 8) return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xF, 0xF, true));
    else return __shfl_xor(v, X);
}
// 2x2 mean of the level below held at lanes (+0, +DX, +DY, +DX+DY); valid at the top-left lane
template <int DX, int DY>
__device__ __forceinline__ float quad_mean(float v)
{
    const float tr = lane_xor<DX>(v);  // every lane: its x partner's value
    const float bl = lane_xor<DY>(v);
    const float br = lane_xor<DY>(tr);
    float s = v + tr;
    s = s + bl;
    s = s + br;
    return s * 0.25f;
}
}  // namespace

template <int L, int TPW>
__global__ void __launch_bounds__(64) k_pyr_tail_reg(PyramidArgs a)
{
    const int lane = threadIdx.x, qx = lane & 7, qy = lane >> 3;
    const int pair = blockIdx.z >> 1, frame = blockIdx.z & 1;
    float* planes = (frame ? a.img1 : a.img0) + (size_t)pair * a.plane_stride;
    const int W2 = a.w[2], H2 = a.Hp >> 2;
    const int y2 = 16 * blockIdx.y + 2 * qy;  // lane's level-2 rows y2, y2 + 1
    const float* p2 = planes + a.off[2];
    float2 top[TPW], bot[TPW];
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
        const int x2 = 16 * (blockIdx.x * TPW + t) + 2 * qx;
        const bool in = x2 < W2 && y2 < H2;  // W2, H2 even: the whole quad is in or out
        top[t] = in ? *reinterpret_cast<const float2*>(p2 + (size_t)y2 * W2 + x2) : make_float2(0.0f, 0.0f);
        bot[t] = in ? *reinterpret_cast<const float2*>(p2 + (size_t)(y2 + 1) * W2 + x2) : make_float2(0.0f, 0.0f);
    }
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
        const int sx = blockIdx.x * TPW + t;  // super-tile column
        // level 3: in-lane
        float s = top[t].x + top[t].y;
        s = s + bot[t].x;
        s = s + bot[t].y;
        float v = s * 0.25f;
        {
            const int x = 8 * sx + qx, y = 8 * blockIdx.y + qy;
            if (x < a.w[3] && y < (a.Hp >> 3)) planes[a.off[3] + (size_t)y * a.w[3] + x] = v;
        }
        if constexpr (L >= 4) {
            v = quad_mean<1, 8>(v);
            const int x = 4 * sx + (qx >> 1), y = 4 * blockIdx.y + (qy >> 1);
            if (!(qx & 1) && !(qy & 1) && x < a.w[4] && y < (a.Hp >> 4)) planes[a.off[4] + (size_t)y * a.w[4] + x] = v;
        }
        if constexpr (L >= 5) {
            v = quad_mean<2, 16>(v);
            const int x = 2 * sx + (qx >> 2), y = 2 * blockIdx.y + (qy >> 2);
            if (!(qx & 3) && !(qy & 3) && x < a.w[5] && y < (a.Hp >> 5)) planes[a.off[5] + (size_t)y * a.w[5] + x] = v;
        }
        if constexpr (L >= 6) {
            v = quad_mean<4, 32>(v);
            const int x = sx, y = blockIdx.y;
            if (lane == 0 && x < a.w[6] && y < (a.Hp >> 6)) planes[a.off[6] + (size_t)y * a.w[6] + x] = v;
        }
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
    if (!pyramid2_fits(a)) return hipErrorInvalidValue;
    const int W2 = a.Wp >> 2, H2 = a.Hp >> 2;
    if (a.w[2] != W2) return hipErrorInvalidValue;
    const int nrw = (H2 + kPyrRW - 1) / kPyrRW;  // waves per column
    PyramidArgs b = a;
    // level-1 rows start at 2 W_2 y floats, level-2 rows at W_2 y (plane
    // offsets are multiples of 4: Wp, Hp % 4 == 0): 16-byte stores need W_2 % 4 == 0
    // (with C = 2 or 3, Wp is only a multiple of 4 or 8)
    b.vec_st = W2 % 4 == 0;
    DIS_LAUNCH(t, k_pyr12, dim3((W2 + 255) / 256, nrw, 2 * batch), dim3(64), 0, s, b);
    if (a.levels >= 3) {
        constexpr int TPW = 2;  // 16 x 16 level-2 super-tiles per wave, loads in flight together
        const dim3 grid(((W2 + 15) / 16 + TPW - 1) / TPW, (H2 + 15) / 16, 2 * batch);
        switch (a.levels) {
            case 3: hipLaunchKernelGGL((k_pyr_tail_reg<3, TPW>), grid, dim3(64), 0, s, a); break;
            case 4: hipLaunchKernelGGL((k_pyr_tail_reg<4, TPW>), grid, dim3(64), 0, s, a); break;
            case 5: hipLaunchKernelGGL((k_pyr_tail_reg<5, TPW>), grid, dim3(64), 0, s, a); break;
            default: hipLaunchKernelGGL((k_pyr_tail_reg<6, TPW>), grid, dim3(64), 0, s, a); break;
        }
    }
    return hipGetLastError();
}

}  // namespace dis
