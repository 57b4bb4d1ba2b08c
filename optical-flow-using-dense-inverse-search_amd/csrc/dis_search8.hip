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
//  LPP 1: 64 patches per wave, the whole patch in one lane (8 columns x 8
//         rows): Eigen's reduction entirely in-lane (no cross-lane traffic),
//         no per-patch scalar work duplicated across lanes, 9 shared tap
//         columns per row; 192 VGPRs of gradients + warp, so 2 waves per SIMD.
//         Workgroup = 2 waves on a 16x8 patch block sharing one wider tile.
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
// A workgroup (LPP waves; 2 for LPP 1) owns a block of the patch grid and stages the
// target image region every one of its patches can sample (start +-4 px,
// SURVEY.md 7.3 "I1 search window") into one shared LDS tile. When the block's
// start positions are too spread for the tile, the same arithmetic reads the
// level plane through L1/L2 instead (identical results, slower).
#include <algorithm>

#include "dis_device.h"
#include "dis_kernels.h"

namespace dis {

namespace {

// patch-grid block per workgroup: kBX<LPP> columns x kBY rows of patches
template <int LPP>
constexpr int kBX = LPP == 1 ? 16 : 8;
constexpr int kBY = 8;
template <int LPP>
constexpr int kThreads = kBX<LPP> * kBY * LPP;
constexpr int kTileH = 64;  // max staged tile rows
template <int LPP>
constexpr int kTileW = LPP == 1 ? 96 : 64;  // max staged tile columns
// max tile row stride (floats); the host picks it per grid step. LPP 2: a
// 64 x 72-float tile (18 KB): 8 two-wave workgroups per CU = 4 waves per SIMD
template <int LPP>
constexpr int kTSMax = LPP == 1 ? 128 : 72;
template <int LPP>
constexpr int kCuMax = LPP == 1 ? 192 : 144;  // staged coarse patches (<= 16 x 12 / 12 x 12 for steps >= 1)
template <int LPP>
constexpr int kCuPer = (kCuMax<LPP> + kThreads<LPP> - 1) / kThreads<LPP>;  // coarse patches per thread
constexpr int kFbWgs = 256;    // persistent k_search8_fb workgroups (grid-stride over the list)
constexpr int kTileGroup = 8;  // tile rows per wave in flight

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
    } else if constexpr (LPP == 1) {
        q = 0;
        pb = tid;
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
    return LPP == 1 ? ci : LPP == 8 ? q : LPP == 4 ? q + 4 * ci : 4 * q + ci;
}

// Eigen-order sum of the patch's 64 values; x[ci*8 + row] holds pixel (row,
// lane_col(q, ci)) in lane q of the patch.
template <int LPP>
__device__ __forceinline__ float patch_sum(const float (&x)[8 * kNCol<LPP>])
{
    if constexpr (LPP == 1) {
        float A[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            A[c] = x[8 * c];
#pragma unroll
            for (int j = 1; j < 8; ++j) A[c] = A[c] + x[8 * c + j];
        }
        return ((A[0] + A[4]) + (A[2] + A[6])) + ((A[1] + A[5]) + (A[3] + A[7]));
    } else if constexpr (LPP == 8) {
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
// kFma (DIS_PRECISION_FMA): a + g*r contracted into one fma per product.
template <int LPP, bool kFma = false, typename Fn>
__device__ __forceinline__ float patch_dot(const float (&g)[8 * kNCol<LPP>], Fn&& r)
{
    auto mac = [](float acc, float x, float y) { return kFma ? __builtin_fmaf(x, y, acc) : acc + x * y; };
    if constexpr (LPP == 1) {
        float A[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            A[c] = g[8 * c] * r(8 * c);
#pragma unroll
            for (int j = 1; j < 8; ++j) A[c] = mac(A[c], g[8 * c + j], r(8 * c + j));
        }
        return ((A[0] + A[4]) + (A[2] + A[6])) + ((A[1] + A[5]) + (A[3] + A[7]));
    } else if constexpr (LPP == 8) {
        float a = g[0] * r(0);
#pragma unroll
        for (int j = 1; j < 8; ++j) a = mac(a, g[j], r(j));
        return reduce_cols<8>(a);
    } else if constexpr (LPP == 4) {
        float a = g[0] * r(0);
#pragma unroll
        for (int j = 1; j < 8; ++j) a = mac(a, g[j], r(j));
        float b = g[8] * r(8);
#pragma unroll
        for (int j = 9; j < 16; ++j) b = mac(b, g[j], r(j));
        return reduce_cols<4>(a + b);
    } else {
        float C[4];
#pragma unroll
        for (int ci = 0; ci < 4; ++ci) {
            float a = g[8 * ci] * r(8 * ci);
#pragma unroll
            for (int j = 1; j < 8; ++j) a = mac(a, g[8 * ci + j], r(8 * ci + j));
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
// position (warp_coefs, dis_device.h). `tap(k, c)` returns the target image at
// row Y-5+k (k = 0..8) and column X-5 + qb + c, qb = the lane's first pixel
// column (LPP 1: 0, LPP 2: 4q, else q).
template <int LPP, bool kFence = false, bool kFma = false, typename Tap>
__device__ __forceinline__ void warp_patch(const Warp& w, int norm, Tap&& tap, float (&r)[8 * kNCol<LPP>])
{
    auto mac = [](float acc, float x, float y) { return kFma ? __builtin_fmaf(x, y, acc) : acc + x * y; };
    if constexpr (LPP == 4 || LPP == 8) {
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
                t = mac(t, w.w2, vb[j + 1]);
                t = mac(t, w.w1, va[j]);
                t = mac(t, w.w0, vb[j]);
                r[8 * s + j] = t;
            }
        }
    } else {
        // NC + 1 shared tap columns (5 for LPP 2, 9 for LPP 1), streamed row by row
        constexpr int NC = kNCol<LPP>, NT = NC + 1;
        float prev[NT], cur[NT];
#pragma unroll
        for (int c = 0; c < NT; ++c) prev[c] = tap(0, c);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
#pragma unroll
            for (int c = 0; c < NT; ++c) cur[c] = tap(j + 1, c);
#pragma unroll
            for (int ci = 0; ci < NC; ++ci) {
                float t = w.w3 * cur[ci + 1];
                t = mac(t, w.w2, cur[ci]);
                t = mac(t, w.w1, prev[ci + 1]);
                t = mac(t, w.w0, prev[ci]);
                r[8 * ci + j] = t;
            }
#pragma unroll
            for (int c = 0; c < NT; ++c) prev[c] = cur[c];
            if constexpr (kFence) __builtin_amdgcn_sched_barrier(0);  // one row of taps in flight
        }
    }
    // (tolerance mode: the mean is folded into centred gradients, search_block)
    if (norm && !kFma) {
        // sum / num_points_patch (:265); x / 64 = x * 2^-6 exactly rounded either
        // way, as v_ldexp (inline exponent) instead of a v_mul with a literal
        const float mean = __builtin_amdgcn_ldexpf(patch_sum<LPP>(r), -6);
#pragma unroll
        for (int j = 0; j < 8 * kNCol<LPP>; ++j) r[j] = r[j] - mean;
    }
}

// The per-patch iteration (src/patch.cpp:156-203) with a given tap source.
// kPaper: b -= (bt0, bt1), the template part of the
// template-subtracted residual (see search_block).
template <int LPP, bool kFence, bool kPaper, bool kFma, typename TapAt>
__device__ __forceinline__ void iterate(const Search8Args& a, const LU2& lu, const float (&gx)[8 * kNCol<LPP>],
                                        const float (&gy)[8 * kNCol<LPP>], float rx, float ry, float ix, float iy,
                                        float bt0, float bt1, float* pu0, float* pu1, TapAt&& tap_at)
{
    float u0 = ix, u1 = iy;
    const float sx = rx + u0, sy = ry + u1;
    float px = sx, py = sy;
    float r[8 * kNCol<LPP>];
    const float r00 = 1.0f / lu.u00, r11 = 1.0f / lu.u11;  // div_pre
    // rotated loop (warp at the top): one copy of the warp code, no peeled
    // first warp holding extra registers
    for (int counter = 1;; ++counter) {
        const Warp w = warp_coefs(px, py);
        warp_patch<LPP, kFence, kFma>(w, a.norm, tap_at(w), r);
        float b0 = patch_dot<LPP, kFma>(gx, [&](int j) { return r[j]; });
        float b1 = patch_dot<LPP, kFma>(gy, [&](int j) { return r[j]; });
        if constexpr (kPaper) {
            b0 = b0 - bt0;
            b1 = b1 - bt1;
        }
        float d0, d1;
        {  // lu2_solve (PartialPivLU::solve, src/patch.cpp:176) with div_pre
            float c0 = lu.swap ? b1 : b0, c1 = lu.swap ? b0 : b1;
            c1 = c1 - lu.l10 * c0;
            if constexpr (kFma) {  // tolerance mode: multiply by the rounded reciprocal
                c1 = c1 * r11;
                c0 = __builtin_fmaf(-c1, lu.u01, c0);
                d0 = c0 * r00;
            } else {
                c1 = div_pre(c1, lu.u11, r11);
                c0 = c0 - c1 * lu.u01;
                d0 = div_pre(c0, lu.u00, r00);
            }
            d1 = c1;
        }
        u0 = u0 - d0;
        u1 = u1 - d1;
        px = rx + u0;
        py = ry + u1;
        const float ex = sx - px, ey = sy - py;
        const float s2 = ex * ex + ey * ey;
        // sqrtf(s2) > outlierthresh  <=>  s2 > thr_sq (sqrt is correctly rounded
        // and monotone; thr_sq precomputed on the host); NaN -> reset (see oracle).
        // One exit test: the reset as selects, then a single divergent break.
        const bool bad = s2 > a.thr_sq || s2 != s2 || px < a.tmp_lb || py < a.tmp_lb || px > a.tmp_ub_w ||
                         py > a.tmp_ub_h;
        u0 = bad ? ix : u0;
        u1 = bad ? iy : u1;
        if (bad || counter > a.iters) break;
    }
    *pu0 = u0;
    *pu1 = u1;
}

[[maybe_unused]] __device__ __forceinline__ float xor1f(float v) { return quad_perm<kQuadXor1>(v); }
constexpr int kQuadEven = 0xA0;  // [0,0,2,2]: lanes 2k, 2k+1 read lane 2k
constexpr int kQuadOdd = 0xF5;   // [1,1,3,3]: lanes 2k, 2k+1 read lane 2k+1
[[maybe_unused]] __device__ __forceinline__ int xor1i(int v) { return __builtin_amdgcn_mov_dpp(v, kQuadXor1, 0xF, 0xF, true); }

// The LPP-2 iteration with the per-patch scalar work split between the
// patch's two lanes (lanes 2k, 2k+1; partner = lane ^ 1): lane q carries
// coordinate q of the patch (0: x, 1: y) -- its reference, start and current
// position, its floor / fraction / ceil in the warp, its part of the tap base,
// its displacement and its bounds test -- so one instruction serves both
// coordinates, and the two right-hand sides come out one per lane from a
// single cross-lane stage. The caller arranged (g1, g2) so that lane 2k's own
// sum is the pivoted c0 and lane 2k+1's c1 (PartialPivLU's row swap folded
// into which gradient each lane carries): C_ci = A_ci(g1) + partner's A_ci(g2).
// Every value is the one iterate() computes: the cross-lane products and sums
// pair the same operands (IEEE mul and add commute), the solve runs on both
// lanes from the same (c0, c1). `tap_at(cv)` gets the lane's own ceil
// coordinate. The outlier reset is applied once, after the loop, on the
// exiting lanes.
template <bool kFence, bool kPaper, bool kFma, typename TapAt>
__device__ __forceinline__ void iterate_split(const Search8Args& a, const LU2& lu, const float (&g1)[32],
                                              const float (&g2)[32], int q, float rv, float iv, float btv,
                                              float* puv, TapAt&& tap_at)
{
    float uv = iv;
    const float sv = rv + uv;
    float pv = sv;
    bool reset = false;  // the exit was an outlier / out-of-bounds reset
    const float ubv = q ? a.tmp_ub_h : a.tmp_ub_w;
    float r[32];
    const float r00 = 1.0f / lu.u00, r11 = 1.0f / lu.u11;  // div_pre
    for (int counter = 1;; ++counter) {
        // warp_coefs, one coordinate per lane: a (b) = frac, 1 - a (1 - b)
        const float fl = floorf(pv), fr = pv - fl, om = 1 - fr;
        const int cv = (int)ceilf(pv + .00001f);
        const float s1 = q ? om : fr, s2w = q ? fr : om;
        Warp w;
        w.w0 = xor1f(om) * om;    // (1 - a)(1 - b)
        w.w1 = xor1f(s1) * s1;    // a (1 - b)
        w.w2 = xor1f(s2w) * s2w;  // b (1 - a)
        w.w3 = xor1f(fr) * fr;    // a b
        float bown;               // lane 2k: the pivoted c0's sum, 2k+1: c1's
        if constexpr (kFma) {
            // tolerance mode with centred gradients (no mean of the warped
            // patch): each warped pixel goes straight into the two dot products,
            // no residual array (fewer VGPRs), per-column accumulators summed
            // in-lane, one cross-lane add per right-hand side; taps streamed
            // row by row (109 VGPRs instead of 128 + a spill)
            auto tap = tap_at(cv);
            float x[4], y[4], prev[5], cur[5];
#pragma unroll
            for (int c = 0; c < 5; ++c) prev[c] = tap(0, c);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
#pragma unroll
                for (int c = 0; c < 5; ++c) cur[c] = tap(j + 1, c);
#pragma unroll
                for (int ci = 0; ci < 4; ++ci) {
                    float t = w.w3 * cur[ci + 1];
                    t = __builtin_fmaf(w.w2, cur[ci], t);
                    t = __builtin_fmaf(w.w1, prev[ci + 1], t);
                    t = __builtin_fmaf(w.w0, prev[ci], t);
                    x[ci] = j ? __builtin_fmaf(g1[8 * ci + j], t, x[ci]) : g1[8 * ci] * t;
                    y[ci] = j ? __builtin_fmaf(g2[8 * ci + j], t, y[ci]) : g2[8 * ci] * t;
                }
#pragma unroll
                for (int c = 0; c < 5; ++c) prev[c] = cur[c];
                __builtin_amdgcn_sched_barrier(0);
            }
            bown = ((x[0] + x[1]) + (x[2] + x[3])) + xor1f((y[0] + y[1]) + (y[2] + y[3]));
        } else {
            warp_patch<2, kFence, false>(w, a.norm, tap_at(cv), r);
            float C[4];
#pragma unroll
            for (int ci = 0; ci < 4; ++ci) {
                float x = g1[8 * ci] * r[8 * ci], y = g2[8 * ci] * r[8 * ci];
#pragma unroll
                for (int j = 1; j < 8; ++j) {
                    x = x + g1[8 * ci + j] * r[8 * ci + j];
                    y = y + g2[8 * ci + j] * r[8 * ci + j];
                }
                C[ci] = x + xor1f(y);
            }
            bown = (C[0] + C[2]) + (C[1] + C[3]);
        }
        if constexpr (kPaper) bown = bown - btv;
        float d0, c1;
        {  // lu2_solve (PartialPivLU::solve, src/patch.cpp:176) with div_pre
            const float c0 = quad_perm<kQuadEven>(bown);  // lane 2k's sum
            c1 = quad_perm<kQuadOdd>(bown) - lu.l10 * c0;  // lane 2k+1's
            if constexpr (kFma) {  // tolerance mode: multiply by the rounded reciprocal
                c1 = c1 * r11;
                d0 = __builtin_fmaf(-c1, lu.u01, c0) * r00;
            } else {
                c1 = div_pre(c1, lu.u11, r11);
                d0 = div_pre(c0 - c1 * lu.u01, lu.u00, r00);
            }
        }
        uv = uv - (q ? c1 : d0);
        pv = rv + uv;
        const float ev = sv - pv, e2 = ev * ev;
        const float n2 = e2 + xor1f(e2);  // ex * ex + ey * ey
        // either coordinate out: the pair's OR, on the scalar unit (one ballot
        // per compare: each v_cmp writes its lane mask straight to SGPRs);
        // !(n2 <= thr_sq): over the threshold or NaN in one compare
        unsigned long long m = __builtin_amdgcn_ballot_w64(!(n2 <= a.thr_sq)) |
                               __builtin_amdgcn_ballot_w64(pv < a.tmp_lb) | __builtin_amdgcn_ballot_w64(pv > ubv);
        m |= ((m >> 1) & 0x5555555555555555ull) | ((m << 1) & 0xAAAAAAAAAAAAAAAAull);
        const bool bad = __builtin_amdgcn_inverse_ballot_w64(m);
        if (bad || counter > a.iters) {
            reset = bad;
            break;
        }
    }
    *puv = reset ? iv : uv;
}

}  // namespace

// min waves per SIMD: LPP 1 holds 192 VGPRs of gradients and warp; the LPP-2
// tile kernel 128 (4 per SIMD, also the LDS tile's limit); its fallback form
// 3; LPP 4 / 8 are capped at 96 VGPRs (5 per SIMD: measured +1 % over 4)
template <int LPP, bool kFallback>
constexpr int kWaves = LPP == 1 ? 2 : LPP == 2 ? (kFallback ? 3 : 4) : 5;

// LDS of one workgroup (block of patches)
template <int LPP>
struct BlockLds {
    float tile[kTileH * kTSMax<LPP>];  // the block's I0 region (gradients), then its I1 tile
    float2 cu[kCuMax<LPP>];            // staged coarse patch displacements
    int2 crng[kBX<LPP> + kBY];         // per block column/row: covering coarse range
    int bnd[4];
};

// One block of patches: (bxi, byi) in units of blocks, pair index `pair`.
// kFallback: blocks whose start positions are too spread for the LDS tile read
// the level plane through L1/L2 (identical results); without it such a block
// is appended to the launch's fallback list (a.fb_count / a.fb_list) for
// k_search8_fb and nothing is written here (keeps this kernel's registers
// low enough for 4 waves per SIMD at LPP 2).
// kPhys (the compat entry dis_flow_from_pyramids, OpticalFlowClass semantics):
// the caller's physically padded planes -- template gradients read from its
// dx/dy planes (whatever their padding holds), I1 taps from its padded I1
// plane clamped to the padded extent -- instead of Sobel of the level image
// and virtual replicate padding.
// TSC: the LDS tile row stride as a compile-time constant (0: a.tile_stride at
// run time). Constant, all 45 taps of an update come from one base address
// plus ds_read immediate offsets (no per-row address arithmetic).
template <int LPP, bool kFallback, bool kPaper, bool kFma = false, bool kPhys = false, int TSC = 0>
__device__ __forceinline__ void search_block(const Search8Args& a, int bxi, int byi, int pair, BlockLds<LPP>& S)
{
    constexpr int NT = kThreads<LPP>, NW = NT / 64, NC = kNCol<LPP>, BX = kBX<LPP>;
    float* const tile = S.tile;
    float2* const cu = S.cu;
    int2* const crng = S.crng;
    int* const bnd = S.bnd;
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;  // wave: scalar row math
    int q, pb;  // lane's column slot in its patch, patch in block
    lane_map<LPP>(tid, q, pb);
    const int st = a.steps;
    const int bgx0 = bxi * BX, bgx1 = min(bgx0 + BX - 1, a.npw - 1);
    const int bgy0 = byi * kBY, bgy1 = min(bgy0 + kBY - 1, a.nph - 1);
    // patch (lx, ly) of the block: column-major 2 x 8 patches per half-wave,
    // or (a.quad, LPP 2) 4 x 4 quadrants -- with tile stride 72 and an odd grid
    // step the 32 lanes of a half-wave then read 32 distinct banks at zero flow
    // (search8_tile_layout)
    const int lx = (LPP == 2 && a.quad) ? 4 * ((pb >> 4) & 1) + (pb & 3) : (pb >> 3);
    const int ly = (LPP == 2 && a.quad) ? 4 * (pb >> 5) + ((pb >> 2) & 3) : (pb & 7);
    const int gx = bgx0 + lx;
    const int gy = bgy0 + ly;
    const bool active = gx < a.npw && gy < a.nph;
    const int W = a.W, H = a.H;
    const float* I0 = a.img0 + (size_t)pair * a.plane_stride + a.plane_off;
    // I1 addressing: row stride ld, origin at image pixel (0, 0), taps clamped
    // to [lo, W-1+pad] x [lo, H-1+pad] (virtual: the level plane, replicate)
    const int pad = kPhys ? a.pad : 0, ld = W + 2 * pad, lo = -pad;
    const float* I1 = a.img1 + (size_t)pair * a.plane_stride + a.plane_off + (kPhys ? pad * ld + pad : 0);
    const int irx = gx * st + a.offw, iry = gy * st + a.offh;
    const float rx = (float)irx, ry = (float)iry;

    // --- 1. global loads, all issued before any is consumed: the coarse patch
    // displacements covering the block (src/patch_grid.cpp:108-119 init) and
    // the block's I0 region for the template gradients (every patch pixel
    // +-1 for the Sobel taps, reflect-101 indices: src/main.cpp:34-35).
    const int hp = 4;
    int ga = 0, ha = 0, PH = 0, PN = 0;
    float2 cuv[kCuPer<LPP>];
    const float2* uc = (a.u_coarse && !a.dense_coarse) ? a.u_coarse + (size_t)pair * a.u_stride : nullptr;
    if (uc) {
        const int xlo = (bgx0 * st + a.offw) >> 1, xhi = (bgx1 * st + a.offw) >> 1;
        const int ylo = (bgy0 * st + a.offh) >> 1, yhi = (bgy1 * st + a.offh) >> 1;
        const float rst = __builtin_amdgcn_rcpf((float)st);
        ga = max(0, floordiv_r(xlo - a.c_offw - hp + st, rst));
        const int gb = min(a.c_npw - 1, floordiv_r(xhi - a.c_offw + hp, rst));
        ha = max(0, floordiv_r(ylo - a.c_offh - hp + st, rst));
        const int hb = min(a.c_nph - 1, floordiv_r(yhi - a.c_offh + hp, rst));
        PH = hb - ha + 1;
        PN = (gb - ga + 1) * PH;  // <= kCuMax (steps >= 1)
        const float rph = __builtin_amdgcn_rcpf((float)PH);
#pragma unroll
        for (int k = 0; k < kCuPer<LPP>; ++k) {
            const int i = tid + k * NT;
            const int cx = floordiv_r(i, rph), cy = i - cx * PH;
            cuv[k] = i < PN ? uc[(ga + cx) * a.c_nph + ha + cy] : make_float2(0.0f, 0.0f);
        }
        if (tid < BX + kBY) {
            // covering coarse-patch range per block column / row (src/patch_grid.cpp:121-182
            // footprint test), relative to the staged block
            const int t = tid;
            if (t < BX) {
                const int x = ((bgx0 + t) * st + a.offw) >> 1;  // floor(ref.x / 2)
                crng[t] = make_int2(max(floordiv_r(x - a.c_offw - hp + st, rst), ga) - ga,
                                    min(floordiv_r(x - a.c_offw + hp, rst), gb) - ga);
            } else {
                const int y = ((bgy0 + t - BX) * st + a.offh) >> 1;
                crng[t] = make_int2(max(floordiv_r(y - a.c_offh - hp + st, rst), ha) - ha,
                                    min(floordiv_r(y - a.c_offh + hp, rst), hb) - ha);
            }
        }
    }
    const int x0 = bgx0 * st + a.offw - 5, y0 = bgy0 * st + a.offh - 5;
    const int RW = (bgx1 - bgx0) * st + 10, RH = (bgy1 - bgy0) * st + 10;
    const int RS = RW | 1;  // odd row stride
    if constexpr (!kPhys) {
        // 64-column strips; rows in groups of 8 per wave: 8 loads in flight
        // per lane, bounded registers (region fits the tile buffer: host-checked)
        for (int cs = 0; cs < RW; cs += 64) {
            const int col = cs + lane;
            const int c0 = clampi(reflect101(x0 + col, W), 0, W - 1);
            for (int r0 = wave; r0 < RH; r0 += 8 * NW) {
                float v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {  // unconditional (clamped) loads; the stores are masked
                    const int r = min(r0 + NW * j, RH - 1);
                    v[j] = I0[(size_t)clampi(reflect101(y0 + r, H), 0, H - 1) * W + c0];
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int r = r0 + NW * j;
                    if (r < RH && col < RW) tile[r * RS + col] = v[j];
                }
            }
        }
    }
    if (uc) {
#pragma unroll
        for (int k = 0; k < kCuPer<LPP>; ++k)
            if (tid + k * NT < PN) cu[tid + k * NT] = cuv[k];
    }
    if (tid == 0) {
        bnd[0] = 0x7fffffff;
        bnd[1] = 0x7fffffff;
        bnd[2] = -0x7fffffff;
        bnd[3] = -0x7fffffff;
    }
    __syncthreads();

    // paper mode (oracle patch_init_paper): the coarse-to-fine
    // initialisation is the coarser level's residual-weighted densification
    // evaluated at the patch's sampled pixel (x, y) = floor(ref / 2): votes of
    // the covering coarse patches (staged above, patch-id order) weighted by
    // 1 / max(1, |I1_{l+1}(x + v) - I0_{l+1}(x)|), I1 bilinear with the
    // replicate border. Before the gradients: fewer registers live.
    float ix = 0.0f, iy = 0.0f;
    if constexpr (kPaper) {
        if (uc && active) {
            const int x = irx >> 1, y = iry >> 1, cW = a.c_W;
            const float* I0c = a.img0 + (size_t)pair * a.plane_stride + a.c_plane_off;
            const float* I1c = a.img1 + (size_t)pair * a.plane_stride + a.c_plane_off;
            const float i0v = I0c[(size_t)y * cW + x];
            const int2 xr = crng[gx - bgx0], yr = crng[BX + gy - bgy0];
            float fx = 0.0f, fy = 0.0f, wt = 0.0f;
            if constexpr (LPP == 2) {
                // the patch's two lanes split the votes (vote t = 2m + q, patch-id
                // order t = (cx - xr.x) * ny + cy - yr.x): each samples and weighs
                // its own, then both add the pair's terms in vote order
                const int ny = yr.y - yr.x + 1, n = max(xr.y - xr.x + 1, 0) * max(ny, 0);
                const float rny = __builtin_amdgcn_rcpf((float)max(ny, 1));
                // up to 2 kPV votes (3 x 3 covering patches): every tap of the
                // lane's votes loaded before the first is used (one memory
                // latency instead of one per vote); a lane past n reloads the
                // last vote and discards it
                constexpr int kPV = 5;
                if (n > 0 && n <= 2 * kPV) {
                    float2 v[kPV];
                    float tp[kPV][4], X[kPV], Y[kPV];
#pragma unroll
                    for (int m = 0; m < kPV; ++m) {
                        const int t = min(2 * m + q, n - 1);
                        const int i = floordiv_r(t, rny);
                        v[m] = cu[(xr.x + i) * PH + yr.x + t - i * ny];
                        // bilinear_replicate (dis_device.h), split at the loads
                        X[m] = clamp_m1((float)x + v[m].x, (float)cW);
                        Y[m] = clamp_m1((float)y + v[m].y, (float)a.c_H);
                        const int xa = (int)floorf(X[m]), ya = (int)floorf(Y[m]);
                        const int c0 = clampi(xa, 0, cW - 1), c1 = clampi(xa + 1, 0, cW - 1);
                        const unsigned o0 = __umul24((unsigned)clampi(ya, 0, a.c_H - 1), (unsigned)cW);
                        const unsigned o1 = __umul24((unsigned)clampi(ya + 1, 0, a.c_H - 1), (unsigned)cW);
                        tp[m][0] = I1c[o0 + c0];
                        tp[m][1] = I1c[o0 + c1];
                        tp[m][2] = I1c[o1 + c0];
                        tp[m][3] = I1c[o1 + c1];
                    }
#pragma unroll
                    for (int m = 0; m < kPV; ++m) {
                        if (2 * m >= n) break;
                        const float fx0 = floorf(X[m]), fy0 = floorf(Y[m]);
                        const float ax = X[m] - fx0, ay = Y[m] - fy0;
                        const float top = (1.0f - ax) * tp[m][0] + ax * tp[m][1];
                        const float bot = (1.0f - ax) * tp[m][2] + ax * tp[m][3];
                        const float d = ((1.0f - ay) * top + ay * bot) - i0v;
                        const float c = recip_max1(d);  // correctly rounded (dis_device.h)
                        const bool own = 2 * m + q < n;
                        const float cvx = own ? c * v[m].x : 0.0f, cvy = own ? c * v[m].y : 0.0f;
                        const float cw = own ? c : 0.0f;
                        fx = fx + quad_perm<kQuadEven>(cvx);
                        fy = fy + quad_perm<kQuadEven>(cvy);
                        wt = wt + quad_perm<kQuadEven>(cw);
                        if (2 * m + 1 < n) {
                            fx = fx + quad_perm<kQuadOdd>(cvx);
                            fy = fy + quad_perm<kQuadOdd>(cvy);
                            wt = wt + quad_perm<kQuadOdd>(cw);
                        }
                    }
                } else {
                    for (int m = 0; 2 * m < n; ++m) {
                        const int t = 2 * m + q;
                        float c = 0.0f, cvx = 0.0f, cvy = 0.0f;
                        if (t < n) {
                            const int i = floordiv_r(t, rny);
                            const float2 v = cu[(xr.x + i) * PH + yr.x + t - i * ny];
                            const float d = bilinear_replicate(I1c, cW, a.c_H, (float)x + v.x, (float)y + v.y) - i0v;
                            c = recip_max1(d);  // correctly rounded (dis_device.h)
                            cvx = c * v.x;
                            cvy = c * v.y;
                        }
                        fx = fx + quad_perm<kQuadEven>(cvx);
                        fy = fy + quad_perm<kQuadEven>(cvy);
                        wt = wt + quad_perm<kQuadEven>(c);
                        if (2 * m + 1 < n) {
                            fx = fx + quad_perm<kQuadOdd>(cvx);
                            fy = fy + quad_perm<kQuadOdd>(cvy);
                            wt = wt + quad_perm<kQuadOdd>(c);
                        }
                    }
                }
            } else {
                for (int cx = xr.x; cx <= xr.y; ++cx)
                    for (int cy = yr.x; cy <= yr.y; ++cy) {
                        const float2 v = cu[cx * PH + cy];
                        const float d = bilinear_replicate(I1c, cW, a.c_H, (float)x + v.x, (float)y + v.y) - i0v;
                        const float c = recip_max1(d);  // correctly rounded (dis_device.h)
                        fx = fx + c * v.x;
                        fy = fy + c * v.y;
                        wt = wt + c;
                    }
            }
            if (wt > 0) {
                fx = fx / wt;
                fy = fy / wt;
            }
            ix = fx * 2;
            iy = fy * 2;
        }
    }

    // --- 2. template gradients: Sobel (ksize 3, 1/8, reflect-101) of the level
    // image at pixels (rx-4+c, ry-4+j), zero outside the image (zero-padded
    // dx/dy planes, src/main.cpp:45-47), from the staged region, rows streamed.
    // Lane q: columns lane_col(q, ci); region column of pixel column c is
    // lx + 1 + c, its Sobel taps lx + c .. lx + c + 2.
    float gdx[8 * NC], gdy[8 * NC];
    if (kPhys && active) {
        // the caller's gradient planes at the patch pixels (padded coordinates)
        const size_t o = (size_t)pair * a.plane_stride + a.plane_off + (size_t)(iry - 4 + pad) * ld + irx - 4 + pad;
#pragma unroll
        for (int ci = 0; ci < NC; ++ci)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                gdx[8 * ci + j] = a.gdx_plane[o + (size_t)j * ld + lane_col<LPP>(q, ci)];
                gdy[8 * ci + j] = a.gdy_plane[o + (size_t)j * ld + lane_col<LPP>(q, ci)];
            }
    } else if (active) {
        constexpr int NX = (NC == 1) ? 3 : (NC == 8) ? 10 : 6;
        const float* reg = tile + ((gy - bgy0) * st) * RS + (gx - bgx0) * st + (NC == 2 ? q : NC == 4 ? 4 * q : q);
        auto xoff = [](int m) { return NC == 2 ? 4 * (m / 3) + (m % 3) : m; };
        float Rw[NC][3], Sw[NC][3];
        auto row = [&](int k) {
            float v[NX];
#pragma unroll
            for (int m = 0; m < NX; ++m) v[m] = reg[k * RS + xoff(m)];
#pragma unroll
            for (int ci = 0; ci < NC; ++ci) {
                const int m0 = (NC == 2) ? 3 * ci : ci;
                const float l = v[m0], c = v[m0 + 1], rr = v[m0 + 2];
                Rw[ci][k % 3] = rr - l;
                Sw[ci][k % 3] = c * 0.25f + (l + rr) * 0.125f;
            }
        };
        row(0);
        row(1);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            row(j + 2);
            __builtin_amdgcn_sched_barrier(0);  // rows streamed: bounded VGPRs
            const int py = iry - 4 + j;
#pragma unroll
            for (int ci = 0; ci < NC; ++ci) {
                const int px = irx - 4 + lane_col<LPP>(q, ci);
                const bool in = px >= 0 && px < W && py >= 0 && py < H;
                const float dx = Rw[ci][(j + 1) % 3] * 0.25f + (Rw[ci][j % 3] + Rw[ci][(j + 2) % 3]) * 0.125f;
                const float dy = Sw[ci][(j + 2) % 3] - Sw[ci][j % 3];
                gdx[8 * ci + j] = in ? dx : 0.0f;
                gdy[8 * ci + j] = in ? dy : 0.0f;
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < 8 * NC; ++j) gdx[j] = gdy[j] = 0.0f;
    }
    // paper mode (oracle patch_search): bt = sum(g * Tn) in the
    // Eigen order, T = the level image on the patch with the replicate border
    // (clamped pixel, which the staged region holds), Tn = T - mean(T) with
    // normalisation
    float bt0 = 0.0f, bt1 = 0.0f;
    if constexpr (kPaper) {
        if (active) {
            float tv[8 * NC];
#pragma unroll
            for (int ci = 0; ci < NC; ++ci) {
                const int cx = clampi(irx - 4 + lane_col<LPP>(q, ci), 0, W - 1) - x0;
#pragma unroll
                for (int j = 0; j < 8; ++j) tv[8 * ci + j] = tile[(clampi(iry - 4 + j, 0, H - 1) - y0) * RS + cx];
            }
            if (a.norm) {
                const float mt = patch_sum<LPP>(tv) / 64.0f;
#pragma unroll
                for (int j = 0; j < 8 * NC; ++j) tv[j] = tv[j] - mt;
            }
            bt0 = patch_dot<LPP>(gdx, [&](int j) { return tv[j]; });
            bt1 = patch_dot<LPP>(gdy, [&](int j) { return tv[j]; });
        }
    }

    // --- 3. initialisation from the coarser level (src/patch_grid.cpp:108-119):
    // dense_{l+1}(floor(ref/2)) = mean over covering coarse patches (patch-id
    // order, f from +0, weights 0.5: src/patch_grid.cpp:121-182), times 2,
    // gathered from the staged coarse displacements (paper mode: above).
    if (kPaper && uc) {
    } else if (a.dense_coarse && active) {
        // from the coarser level's dense flow (refined): src/patch_grid.cpp:108-119
        const float2 d = a.dense_coarse[(size_t)pair * a.dense_stride + (size_t)(iry >> 1) * (W / 2) + (irx >> 1)];
        ix = d.x * 2;
        iy = d.y * 2;
    } else if (uc && active) {
        const int2 xr = crng[gx - bgx0], yr = crng[BX + gy - bgy0];
        float fx = 0.0f, fy = 0.0f, wt = 0.0f;
        for (int cx = xr.x; cx <= xr.y; ++cx)
            for (int cy = yr.x; cy <= yr.y; ++cy) {
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
    LU2 lu;
    {
        const float h00 = patch_dot<LPP, kFma>(gdx, [&](int j) { return gdx[j]; });
        const float h01 = patch_dot<LPP, kFma>(gdx, [&](int j) { return gdy[j]; });
        const float h11 = patch_dot<LPP, kFma>(gdy, [&](int j) { return gdy[j]; });
        lu = hessian_lu2(h00, h01, h11);
    }
    if constexpr (kFma) {
        // tolerance mode (summation order free within the stated tolerance):
        // sum(g (r - mean r)) = sum((g - mean g) r), so the right-hand sides
        // take gradients centred once per patch and the update loop skips the
        // mean of the warped patch (src/patch.cpp:261-266) and its 32
        // subtractions per lane -- the Hessian above keeps the raw gradients
        if (a.norm) {
            const float mx = patch_sum<LPP>(gdx) * (1.0f / 64), my = patch_sum<LPP>(gdy) * (1.0f / 64);
#pragma unroll
            for (int j = 0; j < 8 * NC; ++j) {
                gdx[j] = gdx[j] - mx;
                gdy[j] = gdy[j] - my;
            }
        }
    }
    // LPP 2, split iteration (iterate_split): the lane whose right-hand side is
    // b1 -- the y lane, or the x lane when the LU pivot swapped the rows --
    // keeps (gy, gx)
    constexpr bool kSplit = LPP == 2 && !kPhys;
    [[maybe_unused]] const bool own_y = (lu.swap != 0) != (q != 0);
    if constexpr (kSplit) {
#pragma unroll
        for (int j = 0; j < 8 * NC; ++j) {
            const float x = gdx[j], y = gdy[j];
            gdx[j] = own_y ? y : x;
            gdy[j] = own_y ? x : y;
        }
    }
    const float sx = rx + ix, sy = ry + iy;
    const bool valid = active && !(sx < a.tmp_lb || sy < a.tmp_lb || sx > a.tmp_ub_w || sy > a.tmp_ub_h);

    // --- 4. shared tile of the target image. Every sample position p of a patch
    // satisfies |p - start| <= 4 (outlier test), so X = ceil(p + 1e-5f) lies in
    // [floor(s)-4, floor(s)+6] (the epsilon is a no-op from |p| >= 256, Q8) and
    // the taps X-5..X+3 in [floor(s)-9, floor(s)+9]; the tile takes one pixel
    // of margin on each side: [floor(s)-10, floor(s)+10] over valid patches.
    // (The barrier below also ends every lane's reads of the I0 region.)
    {
        const int fxs = valid ? (int)floorf(sx) : 0x7fffffff;
        const int fys = valid ? (int)floorf(sy) : 0x7fffffff;
        const int fxl = valid ? (int)floorf(sx) : -0x7fffffff;
        const int fyl = valid ? (int)floorf(sy) : -0x7fffffff;
        const int m0 = wave_min(fxs), m1 = wave_min(fys), m2 = wave_max(fxl), m3 = wave_max(fyl);
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
    const int capw = a.tile_cap > 0 ? min(a.tile_cap, kTileW<LPP>) : kTileW<LPP>;
    const int caph = a.tile_cap > 0 ? min(a.tile_cap, kTileH) : kTileH;
    const bool use_tile = any_valid && tw <= capw && th <= caph;
    const int TS = TSC ? TSC : a.tile_stride;  // rows of vertically adjacent patches on disjoint banks
    float u0 = ix, u1 = iy;
    float uv = q ? iy : ix;  // split iteration: the lane's coordinate
    if (use_tile) {
        // 64-column strips; rows in groups of kTileGroup per wave (loads in
        // flight, then the LDS stores)
        for (int cs = 0; cs < tw; cs += 64) {
            const int col = cs + lane;
            const int cx = clampi(tx0 + col, lo, W - 1 + pad);
            for (int r0 = wave; r0 < th; r0 += kTileGroup * NW) {
                float v[kTileGroup];
#pragma unroll
                for (int j = 0; j < kTileGroup; ++j) {  // unconditional (clamped) loads; the stores are masked
                    const int r = min(r0 + NW * j, th - 1);
                    v[j] = I1[(ptrdiff_t)clampi(ty0 + r, lo, H - 1 + pad) * ld + cx];
                }
#pragma unroll
                for (int j = 0; j < kTileGroup; ++j) {
                    const int r = r0 + NW * j;
                    if (r < th && col < tw) tile[r * TS + col] = v[j];
                }
            }
        }
        __syncthreads();
        if constexpr (kSplit) {
            if (valid) {
                // lane's part of the tap base (tile + (Y-5-ty0) TS + (X-5+qb-tx0)):
                // x lane (X - 5 - tx0), y lane (Y - 5 - ty0) TS; summed with the
                // partner's by one DPP add
                const int M = q ? TS : 1, K = q ? -(5 + ty0) * TS : -(5 + tx0);
                // byte offsets: t = cv * 4M + 4K, the pair's sum by one DPP add,
                // then three row-group bases (ds_read2 immediates <= 255 dwords)
                const int M4 = 4 * M, K4 = 4 * K;
                typedef __attribute__((address_space(3))) const char* lds_cp;
                typedef __attribute__((address_space(3))) const float* lds_fp;
                const lds_cp tqb = (lds_cp)(tile + 4 * q);
                // tolerance mode: the three-row step as a loop-invariant VGPR
                // operand (5 address VALU per update instead of 7); the exact
                // kernel is at 128 VGPRs and spilled with it, so it adds the two
                // further bases per update behind opaque copies (a literal each)
                int g3 = 12 * TS;
                if constexpr (kFma) __asm__("" : "+v"(g3));
                iterate_split<false, kPaper, kFma>(a, lu, gdx, gdy, q, q ? ry : rx, q ? iy : ix, own_y ? bt1 : bt0,
                                                   &uv, [&](int cv) {
                                                       const int tb = __mul24(cv, M4) + K4;
                                                       const lds_cp c0 = tqb + (tb + xor1i(tb));
                                                       lds_cp c1 = c0 + g3, c2 = c1 + g3;
                                                       if constexpr (!kFma) {
                                                           c1 = c0 + 12 * TS;
                                                           c2 = c0 + 24 * TS;
                                                           __asm__("" : "+v"(c1));
                                                           __asm__("" : "+v"(c2));
                                                       }
                                                       const lds_fp f0 = (lds_fp)c0, f1 = (lds_fp)c1, f2 = (lds_fp)c2;
                                                       return [=](int k, int c) {
                                                           return k < 3 ? f0[k * TS + c]
                                                                        : k < 6 ? f1[(k - 3) * TS + c] : f2[(k - 6) * TS + c];
                                                       };
                                                   });
            }
        } else if (valid) {
            const int qb = LPP == 2 ? 4 * q : LPP == 1 ? 0 : q;  // lane's first tap column
            iterate<LPP, false, kPaper, kFma>(a, lu, gdx, gdy, rx, ry, ix, iy, bt0, bt1, &u0, &u1, [&](const Warp& w) {
                const float* base = tile + (w.Y - 5 - ty0) * TS + (w.X - 5 + qb - tx0);
                return [=](int k, int c) { return base[k * TS + c]; };
            });
        }
    } else if constexpr (kFallback) {
        // taps read through a buffer descriptor of the (padded) plane: 32-bit
        // byte offsets from its first pixel, the replicate clamping done on
        // the indices -- the same values as I1[clamp(row) * ld + clamp(col)]
        // without 64-bit address arithmetic per tap (fewer VGPRs and VALU)
        const unsigned long long pb = reinterpret_cast<unsigned long long>(I1 + (ptrdiff_t)lo * ld + lo);
        const unsigned long long pu = ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(pb >> 32)) << 32) |
                                      (unsigned)__builtin_amdgcn_readfirstlane((unsigned)pb);
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            reinterpret_cast<void*>(pu), (short)0, (H + 2 * pad) * ld * (int)sizeof(float), 0x00020000);
        const int rmax = H - 1 + pad - lo, cmax = W - 1 + pad - lo;
        auto gtap = [=](int y0, int x0) {
            return [=](int k, int c) {
                const int r = clampi(y0 + k - lo, 0, rmax), cc = clampi(x0 + c - lo, 0, cmax);
                return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (r * ld + cc) * 4, 0, 0));
            };
        };
        if constexpr (kSplit) {
            if (valid) {
                iterate_split<true, kPaper, kFma>(a, lu, gdx, gdy, q, q ? ry : rx, q ? iy : ix, own_y ? bt1 : bt0, &uv,
                                                  [&](int cv) {
                                                      const int cp = xor1i(cv);
                                                      return gtap((q ? cv : cp) - 5, (q ? cp : cv) - 5 + 4 * q);
                                                  });
            }
        } else if (valid) {
            const int qb = LPP == 2 ? 4 * q : LPP == 1 ? 0 : q;
            iterate<LPP, true, kPaper, kFma>(a, lu, gdx, gdy, rx, ry, ix, iy, bt0, bt1, &u0, &u1,
                                             [&](const Warp& w) { return gtap(w.Y - 5, w.X - 5 + qb); });
        }
    } else if (any_valid) {
        // too spread for the tile: k_search8_fb redoes this block
        if (tid == 0) {
            const int slot = atomicAdd(a.fb_count, 1);
            a.fb_list[slot] = (pair * ((a.nph + kBY - 1) / kBY) + byi) * ((a.npw + BX - 1) / BX) + bxi;
        }
        return;
    }
    if constexpr (kSplit) {  // every lane (reconverged): the partner's coordinate
        const float up = xor1f(uv);
        u0 = q ? up : uv;
        u1 = q ? uv : up;
    }
    if (active && q == 0) {
        a.u_out[(size_t)pair * a.u_stride + gx * a.nph + gy] = make_float2(u0, u1);
    }
}

// grid: (ceil(npw/kBX), ceil(nph/kBY), batch); one block of patches per workgroup
template <int LPP, bool kFallback, bool kPaper = false, bool kFma = false, bool kPhys = false, int TSC = 0>
__global__ void __launch_bounds__(kThreads<LPP>) __attribute__((amdgpu_waves_per_eu(kWaves<LPP, kFallback>)))
k_search8(Search8Args a)
{
    __shared__ BlockLds<LPP> S;
    // XCD-aware block order: the dispatcher deals linear workgroup ids
    // round-robin to the 8 XCDs; remap so each XCD walks a contiguous run of
    // blocks and neighbouring blocks' overlapping tiles (halo rows) are
    // fetched once into that XCD's L2 instead of once per XCD
    const int nbx = gridDim.x, nby = gridDim.y, nb = nbx * nby * gridDim.z;
    const int lin = blockIdx.x + nbx * (blockIdx.y + nby * blockIdx.z);
    const int per = nb / 8;
    const int t = lin < per * 8 ? (lin % 8) * per + lin / 8 : lin;
    const int bx = __builtin_amdgcn_readfirstlane(t % nbx);
    const int by = __builtin_amdgcn_readfirstlane((t / nbx) % nby);
    const int bz = __builtin_amdgcn_readfirstlane(t / (nbx * nby));
    search_block<LPP, kFallback, kPaper, kFma, kPhys, TSC>(a, bx, by, bz, S);
}

// The blocks k_search8<LPP, false> listed: persistent workgroups over the list
// (usually empty: every workgroup reads the count and exits).
// Capped at the tile kernel's 128 VGPRs (spilling on this rare path): with more,
// its workgroups cannot take the slots another stream's search kernel frees,
// and the (usually empty) launch waited 70-150 us for that kernel to drain.
template <int LPP, bool kPaper = false, bool kFma = false, bool kPhys = false>
__global__ void __launch_bounds__(kThreads<LPP>) __attribute__((amdgpu_waves_per_eu(kWaves<LPP, false>)))
__attribute__((amdgpu_num_vgpr(128)))
k_search8_fb(Search8Args a)
{
    __shared__ BlockLds<LPP> S;
    const int n = *a.fb_count;
    const int nbx = (a.npw + kBX<LPP> - 1) / kBX<LPP>, nby = (a.nph + kBY - 1) / kBY;
    for (int i = blockIdx.x; i < n; i += gridDim.x) {
        const int e = a.fb_list[i];
        const int bx = e % nbx, t = e / nbx;
        search_block<LPP, true, kPaper, kFma, kPhys>(a, bx, t % nby, t / nby, S);
        __syncthreads();  // LDS reuse by the next listed block
    }
}

// LDS tile row stride and (LPP 2) patch layout for grid step `steps`: the
// patches of one 32-lane LDS group sit at (steps*S*gy + steps*gx + lane column
// offset) floats for zero flow; pick S in [tile width + 1, kTSMax] (and, for
// LPP 2, the 2 x 8 or the 4 x 4 half-wave layout) minimising the worst bank
// multiplicity ((a/4) mod 32, ds_read_b32 banking); ties keep 2 x 8.
static int tile_bank_multiplicity(int steps, int lpp, int quad, int S)
{
    int cnt[32] = {0}, m = 0;
    for (int l = 0; l < 32; ++l) {
        int gx, gy, off;
        if (lpp == 1) {  // lane = patch: gx = l / 8, gy = l % 8
            gx = l >> 3, gy = l & 7, off = 0;
        } else if (lpp == 2) {  // 16 patches x 2 lanes (4 columns apart)
            const int p = l >> 1;
            gx = quad ? (p & 3) : p >> 3, gy = quad ? (p >> 2) & 3 : p & 7, off = 4 * (l & 1);
        } else if (lpp == 4) {  // 8 patches x 4 lanes
            gx = 0, gy = l >> 2, off = l & 3;
        } else {  // lpp 8: 4 patches x 8 lanes
            gx = 0, gy = (l >> 4) * 2 + ((l >> 2) & 1), off = (l & 3) | (((l >> 3) & 1) << 2);
        }
        const int b = (int)(((long long)steps * S * gy + steps * gx + off) % 32);
        m = ++cnt[b] > m ? cnt[b] : m;
    }
    return m;
}

static void tile_layout(int steps, int lpp, int* stride, int* quad)
{
    const int w = lpp == 1 ? kTileW<1> : kTileW<2>, smax = lpp == 1 ? kTSMax<1> : kTSMax<2>;
    int best = w + 1, best_q = 0, best_m = 1 << 30;
    for (int q = 0; q <= (lpp == 2 ? 1 : 0); ++q)
        for (int S = w + 1; S <= smax; ++S) {
            const int m = tile_bank_multiplicity(steps, lpp, q, S);
            if (m < best_m) {
                best_m = m;
                best = S;
                best_q = q;
            }
        }
    *stride = best;
    *quad = best_q;
}

int search8_tile_stride(int steps, int lpp)
{
    int s, q;
    tile_layout(steps, lpp, &s, &q);
    return s;
}

int search8_tile_quad(int steps, int lpp)
{
    int s, q;
    tile_layout(steps, lpp, &s, &q);
    return q;
}

// Whether the LPP-1 layout fits: the 16x8 block's I0 region must fit its tile buffer.
bool search8_lpp1_fits(int steps)
{
    return (15 * steps + 11) * (7 * steps + 10) <= kTileH * kTSMax<1>;
}

// k_search8 with the tile stride the host picked (search8_tile_stride) as a
// template constant: 65, 66, 68 or 72 (every stride tile_layout picks); others
// at run time
template <int LPP, bool kFallback, bool kPaper, bool kFma>
static void launch_ts(const Search8Args& a, dim3 grid, hipStream_t s, Timing t)
{
    const dim3 block(kThreads<LPP>);
    switch (a.tile_stride) {
        case 65: DIS_LAUNCH(t, (k_search8<LPP, kFallback, kPaper, kFma, false, 65>), grid, block, 0, s, a); break;
        case 66: DIS_LAUNCH(t, (k_search8<LPP, kFallback, kPaper, kFma, false, 66>), grid, block, 0, s, a); break;
        case 68: DIS_LAUNCH(t, (k_search8<LPP, kFallback, kPaper, kFma, false, 68>), grid, block, 0, s, a); break;
        case 72: DIS_LAUNCH(t, (k_search8<LPP, kFallback, kPaper, kFma, false, 72>), grid, block, 0, s, a); break;
        default: DIS_LAUNCH(t, (k_search8<LPP, kFallback, kPaper, kFma>), grid, block, 0, s, a); break;
    }
}

template <bool kPaper, bool kFma>
static void launch_search8_t(const Search8Args& a, int L, bool split, dim3 grid, dim3 fb_grid, hipStream_t s,
                             Timing t)
{
    if (L == 1) {
        if (split) {
            DIS_LAUNCH(t, (k_search8<1, false, kPaper, kFma>), grid, dim3(kThreads<1>), 0, s, a);
            hipLaunchKernelGGL((k_search8_fb<1, kPaper, kFma>), fb_grid, dim3(kThreads<1>), 0, s, a);
        } else {
            DIS_LAUNCH(t, (k_search8<1, true, kPaper, kFma>), grid, dim3(kThreads<1>), 0, s, a);
        }
    } else if (L == 2) {
        if (split) {
            launch_ts<2, false, kPaper, kFma>(a, grid, s, t);
            hipLaunchKernelGGL((k_search8_fb<2, kPaper, kFma>), fb_grid, dim3(kThreads<2>), 0, s, a);
        } else {
            DIS_LAUNCH(t, (k_search8<2, true, kPaper, kFma>), grid, dim3(kThreads<2>), 0, s, a);
        }
    } else if (L == 4) {
        DIS_LAUNCH(t, (k_search8<4, true, kPaper, kFma>), grid, dim3(kThreads<4>), 0, s, a);
    } else {
        launch_ts<8, true, kPaper, kFma>(a, grid, s, t);
    }
}

// compat path (physical planes): exact kernels, 2 lanes per patch (tile +
// fallback) or 8 on small levels
static void launch_search8_phys(const Search8Args& a, int L, bool split, dim3 grid, dim3 fb_grid, hipStream_t s)
{
    if (L == 2) {
        if (split) {
            hipLaunchKernelGGL((k_search8<2, false, false, false, true>), grid, dim3(kThreads<2>), 0, s, a);
            hipLaunchKernelGGL((k_search8_fb<2, false, false, true>), fb_grid, dim3(kThreads<2>), 0, s, a);
        } else {
            hipLaunchKernelGGL((k_search8<2, true, false, false, true>), grid, dim3(kThreads<2>), 0, s, a);
        }
    } else {
        hipLaunchKernelGGL((k_search8<8, true, false, false, true>), grid, dim3(kThreads<8>), 0, s, a);
    }
}

hipError_t launch_search8(const Search8Args& a, int batch, hipStream_t s, Timing t)
{
    const int L = a.lanes_per_patch;
    if (L == 64) return launch_search_wave(a, batch, s, t);  // one wave per patch (dis_search_wave.hip)
    if (L != 1 && L != 2 && L != 4 && L != 8) return hipErrorInvalidValue;
    const int w = L == 1 ? kTileW<1> : kTileW<2>, smax = L == 1 ? kTSMax<1> : kTSMax<2>;
    if (a.tile_stride < w + 1 || a.tile_stride > smax) return hipErrorInvalidValue;
    if (L == 1 && !search8_lpp1_fits(a.steps)) return hipErrorInvalidValue;
    if (L != 1 && (7 * a.steps + 11) * (7 * a.steps + 10) > kTileH * kTSMax<2>) return hipErrorInvalidValue;
    const int bx = L == 1 ? kBX<1> : kBX<2>;
    dim3 grid((a.npw + bx - 1) / bx, (a.nph + kBY - 1) / kBY, batch);
    // split: the tile-only kernel (4 waves per SIMD at LPP 2) and a
    // k_search8_fb launch over the blocks it listed. (Searching those blocks
    // in place through a non-inlined call instead made every wave of the tile
    // kernel carry a scratch frame: finest launch 940 -> 1346 us; r03.)
    const bool split = (L == 1 || L == 2) && a.fb_count && a.fb_list;
    // persistent fallback workgroups (grid-stride over the list), one per CU
    const dim3 fb_grid(std::min<long long>(kFbWgs, (long long)grid.x * grid.y * grid.z));
    if (a.gdx_plane) {  // physical planes (compat): exact, non-paper, LPP 2 or 8
        if ((L != 2 && L != 8) || a.paper || a.fma || !a.gdy_plane || a.pad < 0) return hipErrorInvalidValue;
        launch_search8_phys(a, L, split, grid, fb_grid, s);
    } else if (a.paper)  // paper mode has no tolerance variant: always the exact kernels
        launch_search8_t<true, false>(a, L, split, grid, fb_grid, s, t);
    else if (a.fma)
        launch_search8_t<false, true>(a, L, split, grid, fb_grid, s, t);
    else
        launch_search8_t<false, false>(a, L, split, grid, fb_grid, s, t);
    return hipGetLastError();
}

}  // namespace dis
