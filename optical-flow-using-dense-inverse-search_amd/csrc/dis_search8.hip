// dis_search8.hip -- K3 fast path: patch inverse search for patch_size 8.
//
// Implements, for one pyramid level and a batch of pairs, the reference's
//   PatchGrid::patch_init_from_prev_flow   src/patch_grid.cpp:108-119 (fused:
//       densified coarser flow evaluated only at the sampled pixel),
//   Patch::init_patch (template gradients)  src/patch.cpp:31-91 (fused: Sobel
//       of the level image computed on the fly, src/main.cpp:34-35),
//   Patch::inverse_search                   src/patch.cpp:119-203,
//   Patch::get_patch_second_image           src/patch.cpp:207-267.
//
// Mapping (CDNA4, wave64), template LPP = lanes per patch:
//  LPP 4: 16 patches per wave; lane q owns pixel columns q and q+4. Eigen's SSE
//         reduction of a 64-vector (two 4-wide packet accumulators; SURVEY.md
//         A6) is then exact:  A_c = sequential sum down column c (in-lane),
//         C_q = A_q + A_{q+4} (in-lane), sum = (C_0+C_2)+(C_1+C_3) (two DPP
//         quad_perm adds, which also broadcast the sum to the 4 lanes).
//  LPP 2: 32 patches per wave; lane q owns columns 4q..4q+3: A_c in-lane,
//         C_j = A_j + A_{j+4} by one DPP add per j (commutative, so both lanes
//         get C_0..C_3), then (C_0+C_2)+(C_1+C_3) in-lane. Fewer VALU
//         instructions per sample (per-patch work is shared by 2 lanes, not 4)
//         and fewer LDS taps (5 shared tap columns per lane), more registers.
//  LPP 8: 8 patches per wave, one pixel column per lane (lowest latency per
//         patch; chosen for coarse levels, whose few patches leave the chip
//         idle). A patch's lanes are {4h..4h+3} and {4h+8..4h+11} of a 16-lane
//         row (h = 0, 1), holding columns 0..3 and 4..7, so C_q = A_q + A_{q+4}
//         is one DPP row_ror:8 add, followed by the two quad_perm adds.
// A workgroup (LPP waves) owns an 8x8 block of the patch grid and stages the
// target image region every one of its patches can sample (start +-4 px,
// SURVEY.md 7.3 "I1 search window") into one shared LDS tile. When the block's
// start positions are too spread for the tile, the same arithmetic reads the
// level plane through L1/L2 instead (identical results, slower).
#include "dis_device.h"
#include "dis_kernels.h"

#ifndef DIS_SEARCH8_WAVES
#define DIS_SEARCH8_WAVES 5  // min waves per SIMD (caps VGPRs at 96; measured +1% over 4)
#endif

namespace dis {

namespace {

constexpr int kBG = 8;             // patch-grid block per workgroup: kBG x kBG patches
constexpr int kTileMax = 64;       // max staged tile edge (pixels)
constexpr int kTSMax = 96;         // max tile row stride (floats); the host picks it per grid step

// quad_perm DPP controls
constexpr int kQuadXor1 = 0xB1;  // [1,0,3,2]
constexpr int kQuadXor2 = 0x4E;  // [2,3,0,1]
constexpr int kRowRor8 = 0x128;  // row_ror:8 (lane i <-> lane i^8 within a 16-lane row)

template <int CTRL>
__device__ __forceinline__ float quad_perm(float v)
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}

// lane -> (pixel-column slot q, patch-in-block pb) for LPP lanes per patch
template <int LPP>
__device__ __forceinline__ void lane_map(int tid, int& q, int& pb)
{
    if constexpr (LPP == 8) {
        const int w = tid & 15;
        q = (w & 3) | ((w >> 3) << 2);
        pb = ((tid >> 4) << 1) | ((w >> 2) & 1);
    } else {
        q = tid % LPP;
        pb = tid / LPP;
    }
}

// sum of the patch's 4 packet-accumulator lanes: (C0+C2)+(C1+C3), broadcast
template <int LPP>
__device__ __forceinline__ float reduce_cols(float a)
{
    if constexpr (LPP == 8) {
        const float c = a + quad_perm<kRowRor8>(a);  // C_q = A_q + A_{q+4}
        const float t = c + quad_perm<kQuadXor2>(c);
        return t + quad_perm<kQuadXor1>(t);
    } else {
        static_assert(LPP == 4, "reduce_cols: LPP 4 or 8");
        const float t = a + quad_perm<kQuadXor2>(a);  // a = C_q
        return t + quad_perm<kQuadXor1>(t);
    }
}

template <int LPP>
constexpr int kNCol = 8 / LPP;  // pixel columns per lane

// pixel column (0..7) of lane q's ci-th column
template <int LPP>
__device__ __forceinline__ int lane_col(int q, int ci)
{
    return LPP == 8 ? q : LPP == 4 ? q + 4 * ci : 4 * q + ci;
}

// Eigen-order sum of the patch's 64 values; x[ci*8 + row] holds pixel (row,
// lane_col(q, ci)) in lane q of the patch.
template <int LPP>
__device__ __forceinline__ float patch_sum(const float (&x)[8 * kNCol<LPP>])
{
    if constexpr (LPP == 8) {
        float a = x[0];
#pragma unroll
        for (int j = 1; j < 8; ++j) a = a + x[j];
        return reduce_cols<8>(a);
    } else if constexpr (LPP == 4) {
        float a = x[0];
#pragma unroll
        for (int j = 1; j < 8; ++j) a = a + x[j];
        float b = x[8];
#pragma unroll
        for (int j = 9; j < 16; ++j) b = b + x[j];
        return reduce_cols<4>(a + b);  // C_q = A_q + A_{q+4}, then (C0+C2) + (C1+C3)
    } else {
        float C[4];
#pragma unroll
        for (int ci = 0; ci < 4; ++ci) {
            float a = x[8 * ci];
#pragma unroll
            for (int j = 1; j < 8; ++j) a = a + x[8 * ci + j];
            C[ci] = a + quad_perm<kQuadXor1>(a);      // A_ci + A_{ci+4}
        }
        return (C[0] + C[2]) + (C[1] + C[3]);
    }
}

// Eigen order of sum(g .* r): each product rounded, then accumulated in the
// patch_sum order; products are formed inside the chains (no 32-value temp).
template <int LPP, typename Fn>
__device__ __forceinline__ float patch_dot(const float (&g)[8 * kNCol<LPP>], Fn&& r)
{
    if constexpr (LPP == 8) {
        float a = g[0] * r(0);
#pragma unroll
        for (int j = 1; j < 8; ++j) a = a + g[j] * r(j);
        return reduce_cols<8>(a);
    } else if constexpr (LPP == 4) {
        float a = g[0] * r(0);
#pragma unroll
        for (int j = 1; j < 8; ++j) a = a + g[j] * r(j);
        float b = g[8] * r(8);
#pragma unroll
        for (int j = 9; j < 16; ++j) b = b + g[j] * r(j);
        return reduce_cols<4>(a + b);
    } else {
        float C[4];
#pragma unroll
        for (int ci = 0; ci < 4; ++ci) {
            float a = g[8 * ci] * r(8 * ci);
#pragma unroll
            for (int j = 1; j < 8; ++j) a = a + g[8 * ci + j] * r(8 * ci + j);
            C[ci] = a + quad_perm<kQuadXor1>(a);
        }
        return (C[0] + C[2]) + (C[1] + C[3]);
    }
}

// Wave-wide min/max of an int (all 64 lanes participate).
__device__ __forceinline__ int wave_min(int v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ int wave_max(int v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}

// Bilinear warp + mean normalisation (src/patch.cpp:207-267) for one patch
// position; `tap(row, col)` returns the target image at (Y-5+row, X-5+q+col)
// relative rows 0..8 and relative cols {0,1} (set 0) / {4,5} (set 1).
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
    w.X = (int)ceilf(x + .00001f);  // Q8: the epsilon is a no-op from 256 on
    w.Y = (int)ceilf(y + .00001f);
    return w;
}

// `tap(k, c)` returns the target image at row Y-5+k (k = 0..8) and column
// X-5 + (LPP == 2 ? 4q : q) + c.
template <int LPP, typename Tap>
__device__ __forceinline__ void warp_patch(const Warp& w, int norm, Tap&& tap, float (&r)[8 * kNCol<LPP>])
{
    if constexpr (LPP != 2) {
#pragma unroll
        for (int s = 0; s < kNCol<LPP>; ++s) {
            float vb[9], va[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                vb[k] = tap(k, 4 * s);      // column X-5+c  (B / D taps)
                va[k] = tap(k, 4 * s + 1);  // column X-4+c  (A / C taps)
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                // row Y-4+j: A = va[j+1], B = vb[j+1]; row Y-5+j: C = va[j], D = vb[j]
                float t = w.w3 * va[j + 1];
                t = t + w.w2 * vb[j + 1];
                t = t + w.w1 * va[j];
                t = t + w.w0 * vb[j];
                r[8 * s + j] = t;
            }
        }
    } else {
        // 5 shared tap columns, streamed row by row
        float prev[5], cur[5];
#pragma unroll
        for (int c = 0; c < 5; ++c) prev[c] = tap(0, c);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
#pragma unroll
            for (int c = 0; c < 5; ++c) cur[c] = tap(j + 1, c);
#pragma unroll
            for (int ci = 0; ci < 4; ++ci) {
                float t = w.w3 * cur[ci + 1];
                t = t + w.w2 * cur[ci];
                t = t + w.w1 * prev[ci + 1];
                t = t + w.w0 * prev[ci];
                r[8 * ci + j] = t;
            }
#pragma unroll
            for (int c = 0; c < 5; ++c) prev[c] = cur[c];
        }
    }
    if (norm) {
        const float mean = patch_sum<LPP>(r) / 64.0f;  // sum / num_points_patch (:265)
#pragma unroll
        for (int j = 0; j < 8 * kNCol<LPP>; ++j) r[j] = r[j] - mean;
    }
}

// The per-patch iteration (src/patch.cpp:156-203) with a given tap source.
template <int LPP, typename TapAt>
__device__ __forceinline__ void iterate(const Search8Args& a, const LU2& lu, const float (&gx)[8 * kNCol<LPP>],
                                        const float (&gy)[8 * kNCol<LPP>], float rx, float ry, float ix, float iy,
                                        float* pu0, float* pu1, TapAt&& tap_at)
{
    float u0 = ix, u1 = iy;
    const float sx = rx + u0, sy = ry + u1;
    float r[8 * kNCol<LPP>];
    Warp w = warp_coefs(sx, sy);
    warp_patch<LPP>(w, a.norm, tap_at(w), r);
    for (int counter = 1;; ++counter) {
        const float b0 = patch_dot<LPP>(gx, [&](int j) { return r[j]; });
        const float b1 = patch_dot<LPP>(gy, [&](int j) { return r[j]; });
        float d0, d1;
        lu2_solve(lu, b0, b1, &d0, &d1);
        u0 = u0 - d0;
        u1 = u1 - d1;
        const float px = rx + u0, py = ry + u1;
        const float ex = sx - px, ey = sy - py;
        const float s2 = ex * ex + ey * ey;
        // sqrtf(s2) > outlierthresh  <=>  s2 > thr_sq (sqrt is correctly rounded
        // and monotone; thr_sq precomputed on the host); NaN -> reset (see oracle)
        if (s2 > a.thr_sq || s2 != s2 || px < a.tmp_lb || py < a.tmp_lb || px > a.tmp_ub_w ||
            py > a.tmp_ub_h) {
            u0 = ix;
            u1 = iy;
            break;
        }
        if (counter > a.iters) break;
        w = warp_coefs(px, py);
        warp_patch<LPP>(w, a.norm, tap_at(w), r);
    }
    *pu0 = u0;
    *pu1 = u1;
}

}  // namespace

template <int LPP>
constexpr int kWaves = LPP == 2 ? 4 : DIS_SEARCH8_WAVES;  // min waves per SIMD (VGPR cap 512/k)

// grid: (ceil(npw/8), ceil(nph/8), batch); block 64*LPP threads = 8x8 patches
template <int LPP>
__global__ void __launch_bounds__(64 * LPP) __attribute__((amdgpu_waves_per_eu(kWaves<LPP>)))
k_search8(Search8Args a)
{
    constexpr int NT = 64 * LPP, NW = LPP, NC = kNCol<LPP>;
    __shared__ float tile[kTileMax * kTSMax];
    __shared__ float2 cu[192];   // staged coarse patch displacements (<= 12 x 12)
    __shared__ int2 crng[2 * 8];  // per block column/row: covering coarse range
    __shared__ int bnd[4];

    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    int q, pb;  // lane's column slot in its patch, patch in block
    lane_map<LPP>(tid, q, pb);
    const int gx = blockIdx.x * kBG + (pb >> 3);
    const int gy = blockIdx.y * kBG + (pb & 7);
    const int pair = blockIdx.z;
    const bool active = gx < a.npw && gy < a.nph;
    const int W = a.W, H = a.H;
    const float* I0 = a.img0 + (size_t)pair * a.plane_stride + a.plane_off;
    const float* I1 = a.img1 + (size_t)pair * a.plane_stride + a.plane_off;

    if (tid == 0) {
        bnd[0] = 0x7fffffff;
        bnd[1] = 0x7fffffff;
        bnd[2] = -0x7fffffff;
        bnd[3] = -0x7fffffff;
    }

    const int irx = gx * a.steps + a.offw, iry = gy * a.steps + a.offh;
    const float rx = (float)irx, ry = (float)iry;

    // --- template gradients: Sobel (ksize 3, 1/8, reflect-101) of the level
    // image at pixels (rx-4+c, ry-4+j), zero outside the image (zero-padded
    // dx/dy planes, src/main.cpp:45-47). Lane q: columns lane_col(q, ci).
    float gdx[8 * NC], gdy[8 * NC];
    if (active) {
        // NC == 2 owns columns q, q+4 (3 loads each); NC == 4 owns 4 adjacent
        // columns sharing a 6-column window; NC == 1 owns column q (3 loads).
        // All loads are issued before
        // use (a row-streamed variant that holds fewer registers measured 3%
        // slower: less memory-level parallelism in the prologue).
        constexpr int NX = (NC == 1) ? 3 : 6;
        int xs[NX];
#pragma unroll
        for (int m = 0; m < NX; ++m) {
            const int col = (NC == 2)   ? (irx - 4 + q + 4 * (m / 3) + (m % 3) - 1)
                            : (NC == 4) ? (irx - 5 + 4 * q + m)
                                        : (irx - 5 + q + m);
            xs[m] = clampi(reflect101(col, W), 0, W - 1);
        }
        float R[NC][10], S[NC][10];
#pragma unroll
        for (int k = 0; k < 10; ++k) {
            const int yy = clampi(reflect101(iry - 5 + k, H), 0, H - 1);
            const float* row = I0 + (size_t)yy * W;
            float v[NX];
#pragma unroll
            for (int m = 0; m < NX; ++m) v[m] = row[xs[m]];
#pragma unroll
            for (int ci = 0; ci < NC; ++ci) {
                const int m0 = (NC == 2) ? 3 * ci : ci;
                const float l = v[m0], c = v[m0 + 1], rr = v[m0 + 2];
                R[ci][k] = rr - l;
                S[ci][k] = c * 0.25f + (l + rr) * 0.125f;
            }
        }
#pragma unroll
        for (int ci = 0; ci < NC; ++ci) {
            const int px = irx - 4 + lane_col<LPP>(q, ci);
            const bool colin = px >= 0 && px < W;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int py = iry - 4 + j;
                const bool in = colin && py >= 0 && py < H;
                const float dx = R[ci][j + 1] * 0.25f + (R[ci][j] + R[ci][j + 2]) * 0.125f;
                const float dy = S[ci][j + 2] - S[ci][j];
                gdx[8 * ci + j] = in ? dx : 0.0f;
                gdy[8 * ci + j] = in ? dy : 0.0f;
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < 8 * NC; ++j) gdx[j] = gdy[j] = 0.0f;
    }
    LU2 lu;
    {
        const float h00 = patch_dot<LPP>(gdx, [&](int j) { return gdx[j]; });
        const float h01 = patch_dot<LPP>(gdx, [&](int j) { return gdy[j]; });
        const float h11 = patch_dot<LPP>(gdy, [&](int j) { return gdy[j]; });
        lu = hessian_lu2(h00, h01, h11);
    }

    // --- initialisation from the coarser level (src/patch_grid.cpp:108-119):
    // dense_{l+1}(floor(ref/2)) = mean over covering coarse patches (patch-id
    // order, f from +0, weights 0.5: src/patch_grid.cpp:121-182), times 2.
    // The coarse patches any patch of this block needs are staged in LDS first
    // (one load per thread), so the gathers below are LDS reads.
    float ix = 0.0f, iy = 0.0f;
    if (a.u_coarse) {
        const int st = a.steps, hp = 4;
        const int bgx0 = blockIdx.x * kBG, bgx1 = min(bgx0 + kBG - 1, a.npw - 1);
        const int bgy0 = blockIdx.y * kBG, bgy1 = min(bgy0 + kBG - 1, a.nph - 1);
        const int xlo = (bgx0 * st + a.offw) >> 1, xhi = (bgx1 * st + a.offw) >> 1;
        const int ylo = (bgy0 * st + a.offh) >> 1, yhi = (bgy1 * st + a.offh) >> 1;
        const int ga = max(0, floordiv(xlo - a.c_offw - hp + st, st));
        const int gb = min(a.c_npw - 1, floordiv(xhi - a.c_offw + hp, st));
        const int ha = max(0, floordiv(ylo - a.c_offh - hp + st, st));
        const int hb = min(a.c_nph - 1, floordiv(yhi - a.c_offh + hp, st));
        const int PH = hb - ha + 1, PN = (gb - ga + 1) * PH;  // <= 12 x 12 (host-checked)
        const float2* uc = a.u_coarse + (size_t)pair * a.u_stride;
        for (int i = tid; i < PN; i += NT) {
            const int cx = i / PH, cy = i - cx * PH;
            cu[i] = uc[(ga + cx) * a.c_nph + ha + cy];
        }
        if (tid < 2 * kBG) {
            // covering coarse-patch range per block column / row (src/patch_grid.cpp:121-182
            // footprint test), relative to the staged block
            const int t = tid;
            if (t < kBG) {
                const int x = ((bgx0 + t) * st + a.offw) >> 1;  // floor(ref.x / 2)
                crng[t] = make_int2(max(floordiv(x - a.c_offw - hp + st, st), ga) - ga,
                                    min(floordiv(x - a.c_offw + hp, st), gb) - ga);
            } else {
                const int y = ((bgy0 + t - kBG) * st + a.offh) >> 1;
                crng[t] = make_int2(max(floordiv(y - a.c_offh - hp + st, st), ha) - ha,
                                    min(floordiv(y - a.c_offh + hp, st), hb) - ha);
            }
        }
        __syncthreads();
        if (active) {
            const int2 xr = crng[gx - bgx0], yr = crng[kBG + gy - bgy0];
            const int gx0 = xr.x, gx1 = xr.y, gy0 = yr.x, gy1 = yr.y;
            float fx = 0.0f, fy = 0.0f, wt = 0.0f;
            for (int cx = gx0; cx <= gx1; ++cx)
                for (int cy = gy0; cy <= gy1; ++cy) {
                    const float2 v = cu[cx * PH + cy];
                    fx = fx + v.x * 0.5f;
                    fy = fy + v.y * 0.5f;
                    wt = wt + 0.5f;
                }
            if (wt > 0) {
                fx = fx / wt;
                fy = fy / wt;
            }
            ix = fx * 2;
            iy = fy * 2;
        }
    }
    const float sx = rx + ix, sy = ry + iy;
    const bool valid = active && !(sx < a.tmp_lb || sy < a.tmp_lb || sx > a.tmp_ub_w || sy > a.tmp_ub_h);

    // --- shared tile of the target image. Every sample position p of a patch
    // satisfies |p - start| <= 4 (outlier test), so X = ceil(p + 1e-5f) lies in
    // [floor(s)-4, floor(s)+6] (the epsilon is a no-op from |p| >= 256, Q8) and
    // the taps X-5..X+3 in [floor(s)-9, floor(s)+9]; the tile takes one pixel
    // of margin on each side: [floor(s)-10, floor(s)+10] over valid patches.
    {
        const int fxs = valid ? (int)floorf(sx) : 0x7fffffff;
        const int fys = valid ? (int)floorf(sy) : 0x7fffffff;
        const int fxl = valid ? (int)floorf(sx) : -0x7fffffff;
        const int fyl = valid ? (int)floorf(sy) : -0x7fffffff;
        const int m0 = wave_min(fxs), m1 = wave_min(fys), m2 = wave_max(fxl), m3 = wave_max(fyl);
        __syncthreads();  // bnd initialised
        if (lane == 0) {
            atomicMin(&bnd[0], m0);
            atomicMin(&bnd[1], m1);
            atomicMax(&bnd[2], m2);
            atomicMax(&bnd[3], m3);
        }
        __syncthreads();
    }
    const bool any_valid = bnd[0] != 0x7fffffff;
    const int tx0 = bnd[0] - 10, ty0 = bnd[1] - 10;
    const int tw = bnd[2] + 10 - tx0 + 1, th = bnd[3] + 10 - ty0 + 1;
    const bool use_tile = any_valid && tw <= kTileMax && th <= kTileMax;
    const int TS = a.tile_stride;  // rows of vertically adjacent patches on disjoint banks

    float u0 = ix, u1 = iy;
    if (use_tile) {
        // all of this wave's rows in flight at once, then the LDS stores
        float v[kTileMax / NW];
        const int cx = clampi(tx0 + lane, 0, W - 1);
#pragma unroll
        for (int j = 0; j < kTileMax / NW; ++j) {
            const int r = wave + NW * j;
            v[j] = (r < th && lane < tw) ? I1[(size_t)clampi(ty0 + r, 0, H - 1) * W + cx] : 0.0f;
        }
#pragma unroll
        for (int j = 0; j < kTileMax / NW; ++j) {
            const int r = wave + NW * j;
            if (r < th && lane < tw) tile[r * TS + lane] = v[j];
        }
        __syncthreads();
        if (valid) {
            const int qb = LPP == 2 ? 4 * q : q;  // lane's first tap column
            iterate<LPP>(a, lu, gdx, gdy, rx, ry, ix, iy, &u0, &u1, [&](const Warp& w) {
                const float* base = tile + (w.Y - 5 - ty0) * TS + (w.X - 5 + qb - tx0);
                return [base, TS](int k, int c) { return base[k * TS + c]; };
            });
        }
    } else if (valid) {
        const int qb = LPP == 2 ? 4 * q : q;
        iterate<LPP>(a, lu, gdx, gdy, rx, ry, ix, iy, &u0, &u1, [&](const Warp& w) {
            const int y0 = w.Y - 5, x0 = w.X - 5 + qb;
            return [=](int k, int c) {
                return I1[(size_t)clampi(y0 + k, 0, H - 1) * W + clampi(x0 + c, 0, W - 1)];
            };
        });
    }
    if (active && q == 0) a.u_out[(size_t)pair * a.u_stride + gx * a.nph + gy] = make_float2(u0, u1);
}

// LDS tile row stride for grid step `steps`: the 8 vertically adjacent patches
// of a half-wave (4 lanes each) sit steps*S floats apart; pick S in
// [kTileMax+1, kTSMax] minimising the worst bank multiplicity of
// (steps*S*g + q) mod 32, g < 8, q < 4 (ds_read_b32 banking, 32-lane groups).
int search8_tile_stride(int steps)
{
    int best = kTileMax + 1, best_m = 1 << 30;
    for (int S = kTileMax + 1; S <= kTSMax; ++S) {
        int cnt[32] = {0}, m = 0;
        for (int g = 0; g < 8; ++g)
            for (int q = 0; q < 4; ++q) {
                const int b = (int)(((long long)steps * S * g + q) % 32);
                m = ++cnt[b] > m ? cnt[b] : m;
            }
        if (m < best_m) {
            best_m = m;
            best = S;
        }
    }
    return best;
}

hipError_t launch_search8(const Search8Args& a, int batch, hipStream_t s, Timing t)
{
    if (a.tile_stride < kTileMax + 1 || a.tile_stride > kTSMax) return hipErrorInvalidValue;
    dim3 grid((a.npw + kBG - 1) / kBG, (a.nph + kBG - 1) / kBG, batch);
    if (a.lanes_per_patch == 2)
        DIS_LAUNCH(t, k_search8<2>, grid, dim3(128), 0, s, a);
    else if (a.lanes_per_patch == 4)
        DIS_LAUNCH(t, k_search8<4>, grid, dim3(256), 0, s, a);
    else if (a.lanes_per_patch == 8)
        DIS_LAUNCH(t, k_search8<8>, grid, dim3(512), 0, s, a);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace dis
