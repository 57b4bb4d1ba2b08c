// dis_frontback.hip -- the fused front and back ends of the DIS path.
//
// K1+K2 (k_pyramid): u8 frame -> padded (virtual) -> level-0 Sobel magnitude
// -> every 2x-downsampled level up to min(C, 6), one launch for both frames of
// a batch (src/main.cpp:139-160, 12-31). A workgroup owns a 2^L x 2^L tile of
// level 0; intermediate levels live in LDS, only the levels the search reads
// are written to HBM (level 0 only when F == 0 or in debug mode).
//
// K4+K5 (k_output): densify the finest searched level (src/patch_grid.cpp:
// 121-182) straight from the patch displacements into an LDS tile, then
// flow *= 2^F, cv::resize(INTER_LINEAR) and crop (src/main.cpp:191-198), so
// the finest dense field never round-trips through HBM.
//
// Arithmetic is exactly that of the stand-alone kernels in dis_kernels.hip
// (and of the oracle): same expressions, same order, -ffp-contract=off.
#include "dis_device.h"
#include "dis_kernels.h"

namespace dis {

namespace {

constexpr int kPyrT0Max = 64;                 // level-0 tile edge (2^6)
constexpr int kPyrSS = kPyrT0Max + 2;         // u8 tile row stride (1-px halo)

}  // namespace

// grid: (Wp / T0, Hp / T0, 2 * batch), block 256; z = pair*2 + frame
__global__ void __launch_bounds__(256) k_pyramid(PyramidArgs a)
{
    __shared__ uint8_t src[kPyrSS * kPyrSS];
    __shared__ float buf0[(kPyrT0Max / 2) * (kPyrT0Max / 2)];
    __shared__ float buf1[(kPyrT0Max / 4) * (kPyrT0Max / 4)];

    const int T0 = 1 << a.levels, SS = T0 + 2;
    const int tid = threadIdx.x;
    const int tx = blockIdx.x * T0, ty = blockIdx.y * T0;
    const int pair = blockIdx.z >> 1, frame = blockIdx.z & 1;
    const uint8_t* in = (frame ? a.I1 : a.I0) + (size_t)pair * a.pair_stride;
    float* planes = (frame ? a.img1 : a.img0) + (size_t)pair * a.plane_stride;

    // u8 tile with a 1-pixel halo: replicate padding to Wp x Hp (floor/ceil
    // split) composed with Sobel's reflect-101 at the Wp x Hp border
    for (int i = tid; i < SS * SS; i += 256) {
        const int r = i / SS, c = i - r * SS;
        const int yy = clampi(reflect101(ty - 1 + r, a.Hp) - a.pt, 0, a.H - 1);
        const int xx = clampi(reflect101(tx - 1 + c, a.Wp) - a.pl, 0, a.W - 1);
        src[i] = in[(size_t)yy * a.stride + xx];
    }
    __syncthreads();

    // level 1 (and level 0 when requested)
    const int n1 = T0 / 2;
    for (int k = tid; k < n1 * n1; k += 256) {
        const int y1 = k / n1, x1 = k - y1 * n1;
        float v[4][4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) v[r][c] = (float)src[(2 * y1 + r) * SS + 2 * x1 + c];
        float m[2][2];
#pragma unroll
        for (int dc = 0; dc < 2; ++dc) {
            float R[4], S[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                R[r] = v[r][dc + 2] - v[r][dc];
                S[r] = v[r][dc + 1] * 0.25f + (v[r][dc] + v[r][dc + 2]) * 0.125f;
            }
#pragma unroll
            for (int dr = 0; dr < 2; ++dr) {
                const float gx = R[dr + 1] * 0.25f + (R[dr] + R[dr + 2]) * 0.125f;
                const float gy = S[dr + 2] - S[dr];
                const float t1 = gx * gx, t2 = gy * gy;
                const float s = t1 + t2;
                m[dr][dc] = sqrtf(s);
            }
        }
        if (a.write_l0) {
            float* p0 = planes + (size_t)(ty + 2 * y1) * a.Wp + tx + 2 * x1;
            p0[0] = m[0][0];
            p0[1] = m[0][1];
            p0[a.Wp] = m[1][0];
            p0[a.Wp + 1] = m[1][1];
        }
        float s = m[0][0] + m[0][1];
        s = s + m[1][0];
        s = s + m[1][1];
        const float l1 = s * 0.25f;
        buf0[k] = l1;
        planes[a.off[1] + (size_t)(ty / 2 + y1) * a.w[1] + tx / 2 + x1] = l1;
    }

    // levels 2..levels from LDS, ping-pong buf0 <-> buf1
    float* cur = buf0;
    float* nxt = buf1;
    for (int l = 2; l <= a.levels; ++l) {
        __syncthreads();
        const int ns = T0 >> (l - 1), nd = ns / 2;
        for (int k = tid; k < nd * nd; k += 256) {
            const int y = k / nd, x = k - y * nd;
            const float* p = cur + (2 * y) * ns + 2 * x;
            float s = p[0] + p[1];
            s = s + p[ns];
            s = s + p[ns + 1];
            const float v = s * 0.25f;
            nxt[k] = v;
            planes[a.off[l] + (size_t)((ty >> l) + y) * a.w[l] + (tx >> l) + x] = v;
        }
        float* t = cur;
        cur = nxt;
        nxt = t;
    }
}

hipError_t launch_pyramid(const PyramidArgs& a, int batch, hipStream_t s)
{
    const int T0 = 1 << a.levels;
    if (a.levels < 1 || T0 > kPyrT0Max || a.Wp % T0 || a.Hp % T0) return hipErrorInvalidValue;
    dim3 grid(a.Wp / T0, a.Hp / T0, 2 * batch);
    hipLaunchKernelGGL(k_pyramid, grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// back end
// ---------------------------------------------------------------------------
namespace {

constexpr int kOutTW = 64, kOutTH = 16;  // full-resolution output tile per workgroup
constexpr int kOutSW = kOutTW / 2 + 3;   // level-F source tile bound (F >= 1)
constexpr int kOutSH = kOutTH / 2 + 3;

// cv::resize INTER_LINEAR source index / fraction for destination index d at
// scale 2^F: s = (d + .5) * 2^-F - .5 (exact dyadic in float), clamped.
__device__ __forceinline__ void lin_coef(int d, int n_src, int F, int* i, float* f)
{
    float fx = (float)(2 * d + 1 - (1 << F)) * (1.0f / (float)(2 << F));
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
    *i = sx;
    *f = fx;
}

}  // namespace

// F == 0: crop of the densified level-0 flow. grid (ceil(W/64), ceil(H/4), batch)
__global__ void __launch_bounds__(256) k_output0(OutputArgs a)
{
    const int x = blockIdx.x * 64 + threadIdx.x, y = blockIdx.y * 4 + threadIdx.y;
    const int pair = blockIdx.z;
    if (x >= a.W || y >= a.H) return;
    const float2* u = a.u + (size_t)pair * a.u_stride;
    a.flow[(size_t)pair * a.W * a.H + (size_t)y * a.W + x] =
        dense_at(u, a.npw, a.nph, a.offw, a.offh, a.steps, a.hp, x + a.pad_left, y + a.pad_top);
}

// F >= 1: grid (ceil(W/64), ceil(H/16), batch), block 256 (2x2 pixels per thread)
__global__ void __launch_bounds__(256) k_output(OutputArgs a)
{
    __shared__ float2 dense[kOutSW * kOutSH];
    const int tid = threadIdx.x;
    const int ox = blockIdx.x * kOutTW, oy = blockIdx.y * kOutTH;
    const int pair = blockIdx.z;
    const float2* u = a.u + (size_t)pair * a.u_stride;
    const float sc = a.sc;

    // source window of this tile at level F
    int i0, i1, j0, j1;
    float f;
    lin_coef(ox + a.pad_left, a.wF, a.F, &i0, &f);
    lin_coef(min(ox + kOutTW - 1, a.W - 1) + a.pad_left, a.wF, a.F, &i1, &f);
    lin_coef(oy + a.pad_top, a.hF, a.F, &j0, &f);
    lin_coef(min(oy + kOutTH - 1, a.H - 1) + a.pad_top, a.hF, a.F, &j1, &f);
    i1 = min(i1 + 1, a.wF - 1);
    j1 = min(j1 + 1, a.hF - 1);
    const int rw = i1 - i0 + 1, rh = j1 - j0 + 1;
    for (int k = tid; k < rw * rh; k += 256) {
        const int r = k / rw, c = k - r * rw;
        const float2 d = dense_at(u, a.npw, a.nph, a.offw, a.offh, a.steps, a.hp, i0 + c, j0 + r);
        dense[r * kOutSW + c] = make_float2(d.x * sc, d.y * sc);  // flowout *= sc_fct (:194)
    }
    __syncthreads();

    const int px = ox + (tid & 31) * 2, py = oy + (tid >> 5) * 2;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
        const int y = py + dy;
        if (y >= a.H) continue;
        int yi;
        float yf;
        lin_coef(y + a.pad_top, a.hF, a.F, &yi, &yf);
        const int r0 = yi - j0, r1 = min(yi + 1, a.hF - 1) - j0;
        const float b0 = 1.f - yf, b1 = yf;
        float2 o[2];
#pragma unroll
        for (int dx = 0; dx < 2; ++dx) {
            const int xx = px + dx + a.pad_left;
            int xi;
            float xf;
            lin_coef(xx, a.wF, a.F, &xi, &xf);
            const bool two = xx < a.xmax;
            const int c0 = xi - i0;
            float h[2][2];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const float2* row = dense + (k ? r1 : r0) * kOutSW;
                const float2 s0 = row[c0];
                if (two) {
                    const float2 s1 = row[c0 + 1];
                    h[k][0] = s0.x * (1.f - xf) + s1.x * xf;
                    h[k][1] = s0.y * (1.f - xf) + s1.y * xf;
                } else {
                    h[k][0] = s0.x;
                    h[k][1] = s0.y;
                }
            }
            o[dx] = make_float2(h[0][0] * b0 + h[1][0] * b1, h[0][1] * b0 + h[1][1] * b1);
        }
        float2* dst = a.flow + (size_t)pair * a.W * a.H + (size_t)y * a.W + px;
        if (px + 1 < a.W) {
            if (a.vec_store)
                *reinterpret_cast<float4*>(dst) = make_float4(o[0].x, o[0].y, o[1].x, o[1].y);
            else {
                dst[0] = o[0];
                dst[1] = o[1];
            }
        } else if (px < a.W) {
            dst[0] = o[0];
        }
    }
}

hipError_t launch_output(const OutputArgs& a, int batch, hipStream_t s)
{
    if (a.F == 0) {
        hipLaunchKernelGGL(k_output0, dim3((a.W + 63) / 64, (a.H + 3) / 4, batch), dim3(64, 4), 0, s, a);
    } else {
        // the level-F window of a 64 x 16 output tile must fit the LDS tile
        if ((kOutTW >> a.F) + 3 > kOutSW || (kOutTH >> a.F) + 3 > kOutSH) return hipErrorInvalidValue;
        hipLaunchKernelGGL(k_output, dim3((a.W + kOutTW - 1) / kOutTW, (a.H + kOutTH - 1) / kOutTH, batch),
                           dim3(256), 0, s, a);
    }
    return hipGetLastError();
}

}  // namespace dis
