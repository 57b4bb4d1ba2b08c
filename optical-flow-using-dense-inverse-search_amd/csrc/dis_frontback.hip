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

#include <type_traits>

namespace dis {

namespace {


}  // namespace

// grid: (Wp / T0, Hp / T0, 2 * batch), block 256; z = pair*2 + frame.
// LEVELS (1..6) is a template parameter so every load loop has a compile-time
// trip count and all of a thread's loads are in flight at once.
// frames per pyramid workgroup: 1 (z = 2 * pair + frame); both frames in one
// 256-thread workgroup measured 7 % slower
constexpr int kPyrNF = 1;
constexpr int kPyrT = 128 * kPyrNF;  // threads per pyramid workgroup

typedef short short2v __attribute__((ext_vector_type(2)));

// 16-bit lanes (lo, hi) = (byte i, byte j) of the 8 bytes {w1:w0} (v_perm_b32)
template <int I, int J>
__device__ __forceinline__ short2v byte_pair(unsigned w0, unsigned w1)
{
    constexpr unsigned sel = 0x0c000c00u | (unsigned)I | ((unsigned)J << 16);
    return __builtin_bit_cast(short2v, __builtin_amdgcn_perm(w1, w0, sel));
}


// LDS of one pyramid workgroup. u8 staging: tile column c of row r at byte
// r * SR + CO + c, so the body columns 1..T0 start 4-byte aligned (dword
// stores) and rows are aligned
template <int LEVELS>
struct PyrLds {
    static constexpr int T0 = 1 << LEVELS, SS = T0 + 2, N1 = T0 / 2, CO = 3, SR = (SS + CO + 3) & ~3;
    static constexpr int N2 = N1 / 2 > 0 ? N1 / 2 : 1;
    alignas(16) uint8_t srcs[kPyrNF][SS * SR];
    float bufs0[kPyrNF][N1 * N1];
    float bufs1[kPyrNF][N2 * N2];
};

// Row loads of V bytes (4 or 16) for the tile body (columns 1..T0, aligned
// source columns) + the two halo columns as bytes, for both frames
template <int LEVELS, int V>
struct PyrRows {
    static constexpr int T0 = 1 << LEVELS, SS = T0 + 2;
    static constexpr int Q = T0 / V > 0 ? T0 / V : 1, NBODY = kPyrNF * SS * Q, KB = (NBODY + kPyrT - 1) / kPyrT;
    static constexpr int NH = kPyrNF * SS * 2, KH = (NH + kPyrT - 1) / kPyrT;
    using VT = typename std::conditional<V == 16, uint4, unsigned>::type;
    VT body[KB];
    uint8_t halo[KH];
};

template <int LEVELS, int V>
__device__ __forceinline__ void pyr_load_rows(const PyramidArgs& a, int tx, int ty, int pair, int fsel, int tid,
                                              PyrRows<LEVELS, V>& R)
{
    using P = PyrRows<LEVELS, V>;
    constexpr int SS = P::SS, Q = P::Q, T0 = P::T0;
#pragma unroll
    for (int k = 0; k < P::KB; ++k) {
        const int i = min(tid + kPyrT * k, P::NBODY - 1);
        const int f = i >= SS * Q, rem = i - f * SS * Q, r = rem / Q, j = rem - r * Q;
        const int ys = clampi(reflect101(ty - 1 + r, a.Hp) - a.pt, 0, a.H - 1);
        const uint8_t* in = ((f | fsel) ? a.I1 : a.I0) + (size_t)pair * a.pair_stride;
        R.body[k] = *reinterpret_cast<const typename P::VT*>(in + (size_t)ys * a.stride + (tx - a.pl) + V * j);
    }
#pragma unroll
    for (int k = 0; k < P::KH; ++k) {
        const int i = min(tid + kPyrT * k, P::NH - 1);
        const int f = i >= 2 * SS, rem = i - f * 2 * SS, r = rem >> 1, c = (rem & 1) ? T0 + 1 : 0;
        const int ys = clampi(reflect101(ty - 1 + r, a.Hp) - a.pt, 0, a.H - 1);
        const int xs = clampi(reflect101(tx - 1 + c, a.Wp) - a.pl, 0, a.W - 1);
        const uint8_t* in = ((f | fsel) ? a.I1 : a.I0) + (size_t)pair * a.pair_stride;
        R.halo[k] = in[(size_t)ys * a.stride + xs];
    }
}

// unconditional stores: lanes past the end rewrite the last item (same
// clamped index, same value) -- a conditional store let the compiler sink the
// last load into the branch, after the wait for the others
template <int LEVELS, int V>
__device__ __forceinline__ void pyr_store_rows(PyrLds<LEVELS>& S, int tid, const PyrRows<LEVELS, V>& R)
{
    using P = PyrRows<LEVELS, V>;
    using L = PyrLds<LEVELS>;
    constexpr int SS = P::SS, Q = P::Q, T0 = P::T0;
#pragma unroll
    for (int k = 0; k < P::KB; ++k) {
        const int i = min(tid + kPyrT * k, P::NBODY - 1);
        const int f = i >= SS * Q, rem = i - f * SS * Q, r = rem / Q, j = rem - r * Q;
        unsigned* d = reinterpret_cast<unsigned*>(&S.srcs[f][r * L::SR + L::CO + 1 + V * j]);  // 4-byte aligned
        if constexpr (V == 16) {
            d[0] = R.body[k].x;
            d[1] = R.body[k].y;
            d[2] = R.body[k].z;
            d[3] = R.body[k].w;
        } else {
            d[0] = R.body[k];
        }
    }
#pragma unroll
    for (int k = 0; k < P::KH; ++k) {
        const int i = min(tid + kPyrT * k, P::NH - 1);
        const int f = i >= 2 * SS, rem = i - f * 2 * SS, r = rem >> 1, c = (rem & 1) ? T0 + 1 : 0;
        S.srcs[f][r * L::SR + L::CO + c] = R.halo[k];
    }
}

// whether a tile's body columns map onto aligned source columns (row loads)
__device__ __forceinline__ bool pyr_row_loads(const PyramidArgs& a, int T0, int tx)
{
    return T0 >= 4 && a.dword_ok && tx - a.pl >= 0 && tx - a.pl + T0 <= a.W;
}

// u8 tile with a 1-pixel halo: replicate padding to Wp x Hp (floor/ceil
// split) composed with Sobel's reflect-101 at the Wp x Hp border; tile column
// c of row r at srcs[f][r * SR + CO + c]. Every lane computes its own row /
// column indices (vector unit): with wave-uniform rows the per-row index and
// 64-bit address arithmetic ran on the scalar unit, ~750 scalar instructions
// per wave, which bounded the kernel.
template <int LEVELS>
__device__ __forceinline__ void pyr_stage(const PyramidArgs& a, PyrLds<LEVELS>& S, int tx, int ty, int pair, int fsel, int tid)
{
    using L = PyrLds<LEVELS>;
    constexpr int T0 = L::T0, SS = L::SS, SR = L::SR, CO = L::CO;
    const bool dw = pyr_row_loads(a, T0, tx);
    if (dw && T0 >= 16 && a.qword_ok) {  // 16-byte row loads (3 per lane for a 64 x 64 tile of both frames)
        PyrRows<LEVELS, 16> R;
        pyr_load_rows(a, tx, ty, pair, fsel, tid, R);
        pyr_store_rows(S, tid, R);
    } else if (dw) {
        PyrRows<LEVELS, 4> R;
        pyr_load_rows(a, tx, ty, pair, fsel, tid, R);
        pyr_store_rows(S, tid, R);
    } else {
        // any tile (padding columns, unaligned strides): one byte per item,
        // 8 loads in flight per lane (bounded registers)
        constexpr int NI = kPyrNF * SS * SS, KI = (NI + kPyrT - 1) / kPyrT, G = 8;
#pragma unroll 1
        for (int k0 = 0; k0 < KI; k0 += G) {
            uint8_t v[G];
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const int i = min(tid + kPyrT * (k0 + g), NI - 1);
                const int f = i >= SS * SS, rem = i - f * SS * SS, r = rem / SS, c = rem - r * SS;
                const int ys = clampi(reflect101(ty - 1 + r, a.Hp) - a.pt, 0, a.H - 1);
                const int xs = clampi(reflect101(tx - 1 + c, a.Wp) - a.pl, 0, a.W - 1);
                const uint8_t* in = ((f | fsel) ? a.I1 : a.I0) + (size_t)pair * a.pair_stride;
                v[g] = in[(size_t)ys * a.stride + xs];
            }
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const int i = min(tid + kPyrT * (k0 + g), NI - 1);  // unconditional (see pyr_store_rows)
                const int f = i >= SS * SS, rem = i - f * SS * SS, r = rem / SS, c = rem - r * SS;
                S.srcs[f][r * SR + CO + c] = v[g];
            }
        }
    }
}

// Level 1 (and level 0 when requested) from the staged u8 tile, then levels
// 2..LEVELS from LDS (a barrier per level); the caller has synchronised after
// staging and synchronises before the LDS is reused
template <int LEVELS>
__device__ __forceinline__ void pyr_compute(const PyramidArgs& a, PyrLds<LEVELS>& S, int tx, int ty, int pair, int fsel, int tid)
{
    using L = PyrLds<LEVELS>;
    constexpr int T0 = L::T0, N1 = L::N1, SR = L::SR, CO = L::CO;
#pragma unroll
    for (int f = 0; f < kPyrNF; ++f) {
    const uint8_t* src = S.srcs[f];
    float* buf0 = S.bufs0[f];
    float* planes = ((f | fsel) ? a.img1 : a.img0) + (size_t)pair * a.plane_stride;
    // level 1 (and level 0 when requested). A work item is a 2x2 block of
    // level-1 pixels = a 4x4 block of level-0 magnitudes read from a 6x6 u8
    // window; the separable Sobel row sums R/S are shared by the 16 pixels.
    constexpr int B1 = N1 >= 2 ? 2 : 1;  // level-1 block edge
    constexpr int NB = N1 / B1;          // blocks per tile edge
    constexpr int E0 = 2 * B1;           // level-0 block edge
#pragma unroll
    for (int k0 = 0; k0 < NB * NB; k0 += kPyrT) {
        const int k = k0 + tid;
        if (NB * NB % kPyrT != 0 && k >= NB * NB) break;
        const int by = k / NB, bx = k - by * NB;
        // Sobel in exact integer arithmetic: with u8 input, R = r - l and
        // T = 2c + l + r are integers, gx = (2R1 + R0 + R2) / 8 and
        // gy = (T2 - T0) / 8 exactly (the reference's float expressions have
        // no rounding here), so gx^2 + gy^2 = N / 64 exactly for the integer
        // N = k1^2 + k2^2 < 2^21, and sqrtf(N / 64) = sqrt_cr(N) / 8.
        float m[E0][E0];
        if constexpr (E0 == 4) {
            // packed 16-bit lanes (exact: |values| <= 1020). Per window row and
            // column c: X = (R, T) = (v[c+2] - v[c], 2 v[c+1] + v[c] + v[c+2]);
            // per pixel: q = (k1, k2) = (2 R1 + R0 + R2, T2 - T0) = X1 (2,0) +
            // X0 (1,-1) + X2, and N = k1^2 + k2^2 = dot2(q, q). The 6-byte row
            // comes in as two dwords (4-byte aligned: SR and 4 bx); (v, v)
            // broadcast pairs by v_perm.
            const short2v c02 = {0, 2}, cm11 = {-1, 1}, c20 = {2, 0}, c1m1 = {1, -1};
            short2v X[6][4];
#pragma unroll
            for (int r = 0; r < 6; ++r) {
                // window columns 4 bx .. 4 bx + 5 = bytes CO + 4 bx ..: the last
                // byte of dword 4 bx, dword 4 bx + 4, the first byte of 4 bx + 8
                const unsigned* row = reinterpret_cast<const unsigned*>(src + (E0 * by + r) * SR + E0 * bx);
                const unsigned w0 = row[0], w1 = row[1], w2 = row[2];
                static_assert(CO == 3, "window byte map");
                const short2v B[6] = {byte_pair<3, 3>(w0, w1), byte_pair<4, 4>(w0, w1), byte_pair<5, 5>(w0, w1),
                                      byte_pair<6, 6>(w0, w1), byte_pair<7, 7>(w0, w1), byte_pair<4, 4>(w1, w2)};
#pragma unroll
                for (int c = 0; c < 4; ++c) X[r][c] = B[c] * cm11 + (B[c + 1] * c02 + B[c + 2]);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const short2v q = X[r + 1][c] * c20 + (X[r][c] * c1m1 + X[r + 2][c]);
                    int n;
                    __asm__("v_dot2_i32_i16 %0, %1, %1, 0" : "=v"(n) : "v"(q));
                    m[r][c] = sqrt_cr((float)n);  // 8 x the magnitude (scaled below, exactly)
                }
        } else {
            int R[E0 + 2][E0], T[E0 + 2][E0];
#pragma unroll
            for (int r = 0; r < E0 + 2; ++r) {
                int v[E0 + 2];
#pragma unroll
                for (int c = 0; c < E0 + 2; ++c) v[c] = src[(E0 * by + r) * SR + CO + E0 * bx + c];
#pragma unroll
                for (int c = 0; c < E0; ++c) {
                    R[r][c] = v[c + 2] - v[c];
                    T[r][c] = 2 * v[c + 1] + v[c] + v[c + 2];
                }
            }
#pragma unroll
            for (int r = 0; r < E0; ++r)
#pragma unroll
                for (int c = 0; c < E0; ++c) {
                    const int k1 = 2 * R[r + 1][c] + R[r][c] + R[r + 2][c];
                    const int k2 = T[r + 2][c] - T[r][c];
                    m[r][c] = sqrt_cr((float)(k1 * k1 + k2 * k2));
                }
        }
        // m holds 8 x the level-0 magnitude sqrtf(N / 64) = sqrt_cr(N) / 8:
        // scaling by a power of two commutes with every rounding below (no
        // underflow / overflow), so the level-1 mean ((m00+m01)+m10)+m11)*0.25
        // of the scaled values equals that of the unscaled ones times 2^-5
        if (a.write_l0) {
            float* const p0 = planes + (size_t)ty * a.Wp + tx;  // uniform base, 32-bit lane offsets
#pragma unroll
            for (int r = 0; r < E0; ++r)
#pragma unroll
                for (int c = 0; c < E0; ++c) p0[(E0 * by + r) * a.Wp + E0 * bx + c] = m[r][c] * 0.125f;
        }
        float* const p1 = planes + a.off[1] + (size_t)(ty / 2) * a.w[1] + tx / 2;
#pragma unroll
        for (int i = 0; i < B1; ++i)
#pragma unroll
            for (int j = 0; j < B1; ++j) {
                float s = m[2 * i][2 * j] + m[2 * i][2 * j + 1];
                s = s + m[2 * i + 1][2 * j];
                s = s + m[2 * i + 1][2 * j + 1];
                const float l1 = s * 0.03125f;  // (s / 8) * 0.25, exact
                const int y1 = B1 * by + i, x1 = B1 * bx + j;
                buf0[y1 * N1 + x1] = l1;
                p1[y1 * a.w[1] + x1] = l1;
            }
    }

    }
    // levels 2..LEVELS from LDS for both frames at once (one barrier per
    // level), ping-pong bufs0 <-> bufs1
#pragma unroll
    for (int l = 2; l <= LEVELS; ++l) {
        __syncthreads();
        const int ns = T0 >> (l - 1), nd = ns / 2, nn = nd * nd;
        for (int k = tid; k < kPyrNF * nn; k += kPyrT) {
            const int f = k >= nn, kk = k - f * nn;
            const float* cur = (l & 1) ? S.bufs1[f] : S.bufs0[f];
            float* nxt = (l & 1) ? S.bufs0[f] : S.bufs1[f];
            float* planes = ((f | fsel) ? a.img1 : a.img0) + (size_t)pair * a.plane_stride;
            float* const pl = planes + a.off[l] + (size_t)(ty >> l) * a.w[l] + (tx >> l);
            const int y = kk / nd, x = kk - y * nd;
            const float* p = cur + (2 * y) * ns + 2 * x;
            float s = p[0] + p[1];
            s = s + p[ns];
            s = s + p[ns + 1];
            const float v = s * 0.25f;
            nxt[kk] = v;
            pl[y * a.w[l] + x] = v;
        }
    }
}

template <int LEVELS>
__global__ void __launch_bounds__(kPyrT) __attribute__((amdgpu_waves_per_eu(8))) k_pyramid(PyramidArgs a)
{
    __shared__ PyrLds<LEVELS> S;
    constexpr int T0 = 1 << LEVELS;
    const int tid = threadIdx.x;
    if (blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0) {
        for (int i = tid; i < a.nzero; i += blockDim.x) a.zero[i] = 0;
    }
    // XCD-aware tile order: the dispatcher deals linear block ids round-robin
    // to the 8 XCDs; remap so each XCD gets a contiguous run of tiles along x
    // and horizontally adjacent tiles share their 128-B rows in one L2.
    const int nbx = gridDim.x, nby = gridDim.y;
    const int nb = nbx * nby * gridDim.z;
    const int lin = blockIdx.x + nbx * (blockIdx.y + nby * blockIdx.z);
    const int per = nb / 8;
    const int t = (lin < per * 8) ? (lin % 8) * per + lin / 8 : lin;
    // (divisions run on the vector unit: make the results provably uniform)
    const int bx = __builtin_amdgcn_readfirstlane(t % nbx);
    const int by = __builtin_amdgcn_readfirstlane((t / nbx) % nby);
    const int bz = __builtin_amdgcn_readfirstlane(t / (nbx * nby));
    const int tx = bx * T0, ty = by * T0;
    // both frames of the tile in one workgroup (2x the loads in flight), or
    // (kPyrNF 1) z = 2 * pair + frame
    const int pair = kPyrNF == 2 ? bz : bz >> 1, fsel = kPyrNF == 2 ? 0 : bz & 1;
    pyr_stage(a, S, tx, ty, pair, fsel, tid);
    __syncthreads();
    pyr_compute(a, S, tx, ty, pair, fsel, tid);
}

hipError_t launch_pyramid(const PyramidArgs& a, int batch, hipStream_t s, Timing t)
{
    const int T0 = 1 << a.levels;
    if (a.levels < 1 || a.levels > 6 || a.Wp % T0 || a.Hp % T0) return hipErrorInvalidValue;
    dim3 grid(a.Wp / T0, a.Hp / T0, batch * (2 / kPyrNF));
    switch (a.levels) {
        case 1: DIS_LAUNCH(t, k_pyramid<1>, grid, dim3(kPyrT), 0, s, a); break;
        case 2: DIS_LAUNCH(t, k_pyramid<2>, grid, dim3(kPyrT), 0, s, a); break;
        case 3: DIS_LAUNCH(t, k_pyramid<3>, grid, dim3(kPyrT), 0, s, a); break;
        case 4: DIS_LAUNCH(t, k_pyramid<4>, grid, dim3(kPyrT), 0, s, a); break;
        case 5: DIS_LAUNCH(t, k_pyramid<5>, grid, dim3(kPyrT), 0, s, a); break;
        default: DIS_LAUNCH(t, k_pyramid<6>, grid, dim3(kPyrT), 0, s, a); break;
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// back end
// ---------------------------------------------------------------------------
namespace {

// full-resolution output tile per workgroup (measured: 64 rows beat 16 by
// 2.3 % of the step at F >= 1); at F == 0 32 rows: the level-0 window halves
// the LDS (paper mode 70 -> 39 KB, 2 -> 4 workgroups per CU, -6 % per SLOW
// step; reference mode 44 -> 24 KB, -1 %). Paper mode at F >= 1 with 32 rows
// measured 2 % slower (7 -> 8 workgroups per CU do not pay for the halo).
constexpr int kOutTW = 64, kOutTH = 64;
template <bool UPS>
constexpr int kOutTHf = UPS ? kOutTH : 32;  // rows of an output tile

// LDS shapes per instantiation: level-F window (F == 0 is the widest; F >= 1
// needs half the tile + the interpolation halo) and the staged patch block for
// K = ceil(ps/steps) covering patches per axis (steps >= ceil(8/K), ps = 8).
template <bool UPS, int TH>
struct OutShape {
    static constexpr int SW = UPS ? kOutTW / 2 + 3 : kOutTW + 3;
    static constexpr int SH = UPS ? TH / 2 + 3 : TH + 3;
};
template <bool UPS, int K, int TH>
struct OutPatch {
    static constexpr int st = (8 + K - 1) / K;
    static constexpr int PX = (OutShape<UPS, TH>::SW + 7) / st + 2;
    // odd stride (in float2): the densify's lanes read patches at different
    // column offsets xr.x, which an even stride maps onto the same LDS banks
    static constexpr int PY = ((OutShape<UPS, TH>::SH + 7) / st + 2) | 1;
};

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


// paper mode: I1 of level F over every tap the window's weighted votes can
// reach (floats; F == 0 has the twice wider window), staged when it fits, at a
// fixed row stride (a vote's lower taps at constant LDS offsets). F >= 1:
// 48 x 50 keeps the workgroup at 23 KB of LDS, 7 per CU (56 x 56: 26 KB, 6 per
// CU, measured 6 % slower); a window whose flows spread wider than ~11 level-F
// pixels reads I1 globally instead (same values); F == 0 (32-row tiles):
// 80 x 48 (the box is at least 67 x 35)
template <bool UPS>
constexpr int kPaperStage = UPS ? 48 * 50 : 80 * 48;
template <bool UPS>
constexpr int kPaperSS = UPS ? 48 : 80;

// one float4 (two output pixels) of the flow. (Streaming, non-temporal
// stores made the one-stream kernel trace faster -- the next call's pyramid
// no longer evicted -- but the two-sub-batch step 2-3 % slower: DESIGN.md 3.)
__device__ __forceinline__ void store_flow2(float2* dst, float2 o0, float2 o1)
{
    *reinterpret_cast<float4*>(dst) = make_float4(o0.x, o0.y, o1.x, o1.y);
}

// Output rows of an interior tile at F == 1 (every tap unclamped, every column
// two-tap, the tile inside W x H). lin_coef then reduces to
// i = (d - 1) >> 1, f = 0.75 (d even) / 0.25 (d odd) for a destination index d,
// so with the thread's rows and columns starting at even y / x the taps are
// static given the parities YP = (pad_top - 1) & 1, XP = (pad_left - 1) & 1,
// and each source row's horizontal interpolation -- the same expression as
// the general path, hence the same value -- is formed once and shared by the
// (up to four) output rows that read it.
template <int YP, int XP, int SW, int RPT>
__device__ __forceinline__ void out_rows_f1(const OutputArgs& a, const float2* dense, int i0, int j0, int px, int py,
                                            int pair)
{
    constexpr int LP = XP ^ 1;                               // pad_left & 1 = parity of x = px + pad_left
    constexpr float xf0 = LP ? 0.25f : 0.75f, xf1 = LP ? 0.75f : 0.25f;
    constexpr int o1 = LP ? 0 : 1;                           // source column of pixel 1 - that of pixel 0
    constexpr int NR = (RPT - 1 + YP) / 2 + 2;               // source rows of the thread's RPT output rows
    const int c0 = ((px + a.pad_left - 1) >> 1) - i0;
    const int rs = ((py + a.pad_top - 1) >> 1) - j0;
    float2 h0[NR], h1[NR];
#pragma unroll
    for (int t = 0; t < NR; ++t) {
        const float2* row = dense + (rs + t) * SW + c0;
        const float2 sa = row[0], sb = row[1];
        h0[t] = make_float2(sa.x * (1.f - xf0) + sb.x * xf0, sa.y * (1.f - xf0) + sb.y * xf0);
        if constexpr (o1) {
            const float2 sc = row[2];
            h1[t] = make_float2(sb.x * (1.f - xf1) + sc.x * xf1, sb.y * (1.f - xf1) + sc.y * xf1);
        } else {
            h1[t] = make_float2(sa.x * (1.f - xf1) + sb.x * xf1, sa.y * (1.f - xf1) + sb.y * xf1);
        }
    }
    float2* dst = a.flow + (size_t)pair * a.W * a.H + (size_t)py * a.W + px;
#pragma unroll
    for (int d = 0; d < RPT; ++d) {
        const int t = (d + YP) >> 1;                         // yi - (first source row)
        const float yf = ((d + YP) & 1) ? 0.75f : 0.25f;     // y + pad_top even -> 0.75
        const float b0 = 1.f - yf, b1 = yf;
        const float2 o0 = make_float2(h0[t].x * b0 + h0[t + 1].x * b1, h0[t].y * b0 + h0[t + 1].y * b1);
        const float2 oo = make_float2(h1[t].x * b0 + h1[t + 1].x * b1, h1[t].y * b0 + h1[t + 1].y * b1);
        store_flow2(dst + (size_t)d * a.W, o0, oo);
    }
}

}  // namespace

// grid (ceil(W/64), ceil(H/16), batch), block 256 (2x2 output pixels per thread).
// 1) stage the patch displacements covering this tile's level-F window in LDS
//    (one round of loads), 2) densify the window into LDS (src/patch_grid.cpp:
//    121-182), 3) F == 0: crop; F >= 1: scale by 2^F, resize, crop.
// K = ceil(ps / steps) bounds the covering patches per axis, so the gather is
// an unrolled, predicated K x K loop (no divergent loops).
template <bool UPSAMPLE, int K, bool kPaper = false>
__global__ void __launch_bounds__(256) k_output(OutputArgs a)
{
    constexpr int kTH = kOutTHf<UPSAMPLE>;
    constexpr int kOutSW = OutShape<UPSAMPLE, kTH>::SW, kOutSH = OutShape<UPSAMPLE, kTH>::SH;
    constexpr int kOutPX = OutPatch<UPSAMPLE, K, kTH>::PX, kOutPY = OutPatch<UPSAMPLE, K, kTH>::PY;
    __shared__ float2 pu[(kOutPX + K + 2) * kOutPY];  // + the padding the unmasked taps may read
    __shared__ float rtab[K * K + 1];                  // RN(1 / (0.5 n)), n covering patches
    __shared__ float2 dense[kOutSW * kOutSH];
    __shared__ int2 cr[kOutSW], rr[kOutSH];
    __shared__ float s1[kPaper ? kPaperStage<UPSAMPLE> : 1];  // paper mode: staged I1 (see below)
    __shared__ int pbox[5];
    // paper mode: window columns / rows sorted by their covering-patch count,
    // and per column class v (count v): first pixel index, first sorted
    // column, columns, RCP(columns) bits (see the densify loop)
    __shared__ unsigned char csort[kPaper ? kOutSW : 1], rsort[kPaper ? kOutSH : 1];
    __shared__ int4 ctab[K + 1];
    const int tid = threadIdx.x;
    const int ox = blockIdx.x * kOutTW, oy = blockIdx.y * kTH;
    const int pair = blockIdx.z;
    const float2* u = a.u + (size_t)pair * a.u_stride;
    if (kPaper && tid == 0) {
        pbox[0] = pbox[1] = 0x7fffffff;
        pbox[2] = pbox[3] = -0x7fffffff;
        pbox[4] = 0;
    }

    // level-F window of this tile
    int i0, i1, j0, j1;
    if (UPSAMPLE) {
        float f;
        lin_coef(ox + a.pad_left, a.wF, a.F, &i0, &f);
        lin_coef(min(ox + kOutTW - 1, a.W - 1) + a.pad_left, a.wF, a.F, &i1, &f);
        lin_coef(oy + a.pad_top, a.hF, a.F, &j0, &f);
        lin_coef(min(oy + kTH - 1, a.H - 1) + a.pad_top, a.hF, a.F, &j1, &f);
        i1 = min(i1 + 1, a.wF - 1);
        j1 = min(j1 + 1, a.hF - 1);
    } else {
        i0 = ox + a.pad_left;
        j0 = oy + a.pad_top;
        i1 = min(ox + kOutTW - 1, a.W - 1) + a.pad_left;
        j1 = min(oy + kTH - 1, a.H - 1) + a.pad_top;
    }
    const int rw = i1 - i0 + 1, rh = j1 - j0 + 1;
    // patches whose footprint meets the window
    const int st = a.steps, hp = a.hp;
    const float rst = __builtin_amdgcn_rcpf((float)st);
    const int ga = max(0, floordiv_r(i0 - a.offw - hp + st, rst)), gb = min(a.npw - 1, floordiv_r(i1 - a.offw + hp, rst));
    const int ha = max(0, floordiv_r(j0 - a.offh - hp + st, rst)), hb = min(a.nph - 1, floordiv_r(j1 - a.offh + hp, rst));
    const int PW = gb - ga + 1, PH = hb - ha + 1;  // <= kOutPX x kOutPY (output_fits)
    float umin_x = INFINITY, umin_y = INFINITY, umax_x = -INFINITY, umax_y = -INFINITY;  // paper mode
    bool u_nan = false;  // paper mode: a staged patch with a NaN displacement (see the I1 box below)
    {
        constexpr int NL = (kOutPX * kOutPY + 255) / 256;
        float2 v[NL];
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            const int k = tid + 256 * j;
            const int cx = k / kOutPY, cy = k % kOutPY;
            const bool in = cx < PW && cy < PH;
            v[j] = in ? u[(ga + cx) * a.nph + ha + cy] : make_float2(0.f, 0.f);
            if (kPaper && in) {
                umin_x = fminf(umin_x, v[j].x);
                umax_x = fmaxf(umax_x, v[j].x);
                umin_y = fminf(umin_y, v[j].y);
                umax_y = fmaxf(umax_y, v[j].y);
                u_nan |= v[j].x != v[j].x || v[j].y != v[j].y;
            }
        }
        // new_u = u * 0.5 (src/patch_grid.cpp:156), formed once per patch (paper mode: u itself)
#pragma unroll
        for (int j = 0; j < NL; ++j)
            if (tid + 256 * j < kOutPX * kOutPY)
                pu[tid + 256 * j] = kPaper ? v[j] : make_float2(v[j].x * 0.5f, v[j].y * 0.5f);
    }
    if constexpr (kPaper) {
        // I0 of the window, parked in the .x of each pixel's dense slot (the
        // pixel's densify reads it there before writing the slot), the loads
        // issued together with the patch staging's
        // (lane = column, wave + 4 j = row: no index division; lanes and rows
        // past the window reload its last column / row and store nothing)
        const float* I0 = a.img0 + (size_t)pair * a.plane_stride;
        constexpr int NR = (kOutSH + 3) / 4;
        const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
        for (int cb = 0; cb < kOutSW; cb += 64) {
            const int c = cb + lane;
            const float* col = I0 + (size_t)j0 * a.wF + i0 + min(c, rw - 1);
            float v0[NR];
#pragma unroll
            for (int j = 0; j < NR; ++j) v0[j] = col[(size_t)min(wv + 4 * j, rh - 1) * a.wF];
#pragma unroll
            for (int j = 0; j < NR; ++j)
                if (wv + 4 * j < rh && c < rw) dense[(wv + 4 * j) * kOutSW + c].x = v0[j];
        }
    }
    if (!kPaper && tid >= 64 && tid - 64 <= K * K) {
        const int n = tid - 64;
        rtab[n] = n ? 1.0f / (0.5f * (float)n) : 0.0f;
    }
    // covering patch ranges per window column / row (one floordiv pair each)
    if (tid < rw) {
        const int px = i0 + tid;
        cr[tid] = make_int2(max(floordiv_r(px - a.offw - hp + st, rst), ga) - ga,
                            min(floordiv_r(px - a.offw + hp, rst), gb) - ga);
    }
    if (tid >= 128 && tid - 128 < rh) {
        const int py = j0 + tid - 128;
        rr[tid - 128] = make_int2(max(floordiv_r(py - a.offh - hp + st, rst), ha) - ha,
                                  min(floordiv_r(py - a.offh + hp, rst), hb) - ha);
    }
    __syncthreads();
    // paper mode: sort the window's columns (wave 0) and rows (wave 1) by
    // covering-patch count, a stable counting sort by ballots. The densify
    // below walks the window class by class, so the lanes of a wave share
    // their counts and the K x K vote loop skips the empty slots wave-wide
    // (unsorted, a wave's lanes mix the counts 2 and 3 of steps 3 and every
    // lane issued all 9 slots for 7.1 votes on average).
    if constexpr (kPaper) {
        if (tid < 128) {
            const bool cols = tid < 64;
            const int n = cols ? rw : rh, lane = tid & 63;
            unsigned char* out = cols ? csort : rsort;
            auto cls = [&](int i) {
                if (i >= n) return -1;
                const int2 e = cols ? cr[i] : rr[i];
                return max(e.y - e.x + 1, 0);
            };
            int cnt[K + 1];
#pragma unroll
            for (int v = 0; v <= K; ++v) cnt[v] = 0;
            for (int b = 0; b < n; b += 64) {
                const int v = cls(b + lane);
#pragma unroll
                for (int w = 0; w <= K; ++w) cnt[w] += __popcll(__ballot(v == w));
            }
            int base[K + 1];
            base[0] = 0;
#pragma unroll
            for (int v = 1; v <= K; ++v) base[v] = base[v - 1] + cnt[v - 1];
            if (cols && lane <= K) {
                int b0 = 0, c0 = 0;
#pragma unroll
                for (int v = 0; v <= K; ++v)
                    if (v == lane) {
                        b0 = base[v];
                        c0 = cnt[v];
                    }
                ctab[lane] = make_int4(b0 * rh, b0, c0, __float_as_int(__builtin_amdgcn_rcpf((float)max(c0, 1))));
            }
            for (int b = 0; b < n; b += 64) {
                const int v = cls(b + lane);
#pragma unroll
                for (int w = 0; w <= K; ++w) {
                    const unsigned long long m = __ballot(v == w);
                    if (v == w)
                        out[base[w] + __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u))] =
                            (unsigned char)(b + lane);
                    base[w] += __popcll(m);
                }
            }
        }
    }
    // paper mode: every vote samples I1 (bilinear, replicate border) at
    // X = clamp(RN(x + u.x), -1, W) for a window pixel x and a staged patch's
    // u, so its taps floor(X), floor(X) + 1 lie in [max(i0 + floor(min u.x),
    // -1), min(i1 + floor(max u.x) + 1, W) + 1] (likewise in y). Staged in LDS
    // by logical position, each entry the replicate-clamped pixel the global
    // read would return, when that box fits; else the votes read I1 globally.
    int bx0 = 0, by0 = 0, sws = 0;
    bool staged = false;
    if constexpr (kPaper) {
        auto fl = [](float v) { return (int)fminf(fmaxf(floorf(v), -1048576.0f), 1048576.0f); };
        int m0 = umin_x <= umax_x ? fl(umin_x) : 0x7fffffff, m1 = umin_y <= umax_y ? fl(umin_y) : 0x7fffffff;
        int m2 = umin_x <= umax_x ? fl(umax_x) : -0x7fffffff, m3 = umin_y <= umax_y ? fl(umax_y) : -0x7fffffff;
        // The staged taps' LDS index comes from v_med3 clamps, which do not
        // clamp NaN, and fminf / fmaxf above skip NaN. The search never leaves
        // a NaN displacement (it resets them like outliers), but should one
        // reach this kernel, the whole tile takes the global (replicate-
        // clamped) reads instead of the stage (pbox[4]).
        const bool wave_nan = __ballot(u_nan) != 0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            m0 = min(m0, __shfl_xor(m0, o));
            m1 = min(m1, __shfl_xor(m1, o));
            m2 = max(m2, __shfl_xor(m2, o));
            m3 = max(m3, __shfl_xor(m3, o));
        }
        if ((tid & 63) == 0) {
            if (wave_nan) pbox[4] = 1;
            atomicMin(&pbox[0], m0);
            atomicMin(&pbox[1], m1);
            atomicMax(&pbox[2], m2);
            atomicMax(&pbox[3], m3);
        }
        __syncthreads();
        if (pbox[0] != 0x7fffffff) {
            bx0 = max(i0 + pbox[0], -1);
            by0 = max(j0 + pbox[1], -1);
            const int bx1 = min(i1 + pbox[2] + 1, a.wF) + 1, by1 = min(j1 + pbox[3] + 1, a.hF) + 1;
            sws = bx1 - bx0 + 1;
            const int shs = by1 - by0 + 1;
            staged = !pbox[4] && sws > 0 && shs > 0 && sws <= kPaperSS<UPSAMPLE> && shs * kPaperSS<UPSAMPLE> <= kPaperStage<UPSAMPLE>;
            if (staged) {  // every load issued before the first store: one memory latency
                // lane = column, wave + 4 j = row (as the I0 window above)
                constexpr int SS = kPaperSS<UPSAMPLE>, NR = (kPaperStage<UPSAMPLE> / SS + 3) / 4;
                const float* I1 = a.img1 + (size_t)pair * a.plane_stride;
                const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
                for (int cb = 0; cb < SS; cb += 64) {
                    const int c = cb + lane;
                    const float* col = I1 + clampi(bx0 + min(c, sws - 1), 0, a.wF - 1);
                    float v1[NR];
#pragma unroll
                    for (int j = 0; j < NR; ++j)
                        v1[j] = col[(size_t)clampi(by0 + min(wv + 4 * j, shs - 1), 0, a.hF - 1) * a.wF];
#pragma unroll
                    for (int j = 0; j < NR; ++j)
                        if (wv + 4 * j < shs && c < sws) s1[(wv + 4 * j) * SS + c] = v1[j];
                }
            }
        }
        __syncthreads();
    }
    const float sc = a.sc;
    const float rrw = __builtin_amdgcn_rcpf((float)rw);  // k / rw by floordiv_r (exact, |k| < 2^20)
    int pxc[K + 1];  // paper mode: first pixel index of each column class
#pragma unroll
    for (int v = 0; v <= K; ++v) pxc[v] = kPaper ? ctab[v].x : 0;
    // paper mode, staged: a tap's LDS index fma(floor Y, stride, floor X)
    // (integers below 2^24: exact) from s1b = s1 - (by0 * stride + bx0)
    constexpr int kSS = kPaperSS<UPSAMPLE>;
    const float* s1b = s1 - (by0 * kSS + bx0);
    // the staged / global choice (block-uniform) outside the pixel loop
    auto densify = [&](auto staged_c) {
        constexpr bool kStaged = decltype(staged_c)::value;
        for (int k = tid; k < rw * rh; k += 256) {
            int r, c;
            if constexpr (kPaper) {
                // pixel k of the class-major order: class z (the last whose first
                // index <= k), then sorted row / sorted column within the class
                int z = 0;
#pragma unroll
                for (int v = 1; v <= K; ++v) z += k >= pxc[v] ? 1 : 0;
                const int4 e = ctab[z];
                const int l = k - e.x;
                const int rs = floordiv_r(l, __int_as_float(e.w));
                c = csort[e.y + l - rs * e.z];
                r = rsort[rs];
            } else {
                r = floordiv_r(k, rrw);
                c = k - r * rw;
            }
            // dense value: contributions in patch-id order, f from +0; masked
            // terms add +0, an exact no-op (f is never -0)
            const int2 xr = cr[c], yr = rr[r];
            float fx = 0.0f, fy = 0.0f, w = 0.0f;
            if constexpr (kPaper) {
                // SURVEY 8f row 4 (oracle densify_paper): weight 1/max(1, |I1(x+u) - I0(x)|)
                const int xg = i0 + c, yg = j0 + r;  // level-F pixel
                const float* I1 = a.img1 + (size_t)pair * a.plane_stride;
                const float i0v = dense[r * kOutSW + c].x;  // I0(x), staged above
                const float xf = (float)xg, yf = (float)yg;
#pragma unroll
                for (int i = 0; i < K; ++i)
#pragma unroll
                    for (int j = 0; j < K; ++j) {
                        if ((xr.x + i <= xr.y) && (yr.x + j <= yr.y)) {
                            const float2 t = pu[(xr.x + i) * kOutPY + yr.x + j];
                            float d;
                            if constexpr (kStaged) {  // bilinear_replicate's expressions on the staged taps
                                const float X = clamp_m1(xf + t.x, (float)a.wF);
                                const float Y = clamp_m1(yf + t.y, (float)a.hF);
                                const float fx0 = floorf(X), fy0 = floorf(Y);
                                const float ax = X - fx0, ay = Y - fy0;
                                const float* q = s1b + (int)__builtin_fmaf(fy0, (float)kSS, fx0);
                                const float top = (1.0f - ax) * q[0] + ax * q[1];
                                const float bot = (1.0f - ax) * q[kSS] + ax * q[kSS + 1];
                                d = ((1.0f - ay) * top + ay * bot) - i0v;
                            } else {
                                d = bilinear_replicate(I1, a.wF, a.hF, xf + t.x, yf + t.y) - i0v;
                            }
                            const float cw = recip_max1(d);  // correctly rounded (dis_device.h)
                            fx = fx + cw * t.x;
                            fy = fy + cw * t.y;
                            w = w + cw;
                        }
                    }
            } else {
                // covering patches per axis (<= K), read at constant offsets from the
                // first one (the LDS array is padded for the taps past the range)
                const int nx = max(xr.y - xr.x + 1, 0), ny = max(yr.y - yr.x + 1, 0);
                const float2* pb = pu + xr.x * kOutPY + yr.x;
#pragma unroll
                for (int i = 0; i < K; ++i)
#pragma unroll
                    for (int j = 0; j < K; ++j) {
                        const bool ok = i < nx && j < ny;
                        const float2 t = pb[i * kOutPY + j];
                        fx = fx + (ok ? t.x : 0.0f);
                        fy = fy + (ok ? t.y : 0.0f);
                    }
                // the reference's weight sum of 0.5 per covering patch, exactly
                const int n = nx * ny;
                w = 0.5f * (float)n;
                // fx / w correctly rounded from the tabulated RN(1 / w) (div_pre);
                // tiny nonzero numerators, whose remainders could underflow, take
                // the IEEE division below
                const bool tiny = (fx != 0.0f && fabsf(fx) < 0x1p-100f) || (fy != 0.0f && fabsf(fy) < 0x1p-100f);
                if (n > 0 && !tiny) {
                    const float rcp = rtab[n];
                    fx = div_pre(fx, w, rcp);
                    fy = div_pre(fy, w, rcp);
                    w = 0.0f;  // done
                }
            }
            if (w > 0) {
                fx = fx / w;
                fy = fy / w;
            }
            // flowout *= sc_fct (src/main.cpp:194) before the resize
            dense[r * kOutSW + c] = UPSAMPLE ? make_float2(fx * sc, fy * sc) : make_float2(fx, fy);
        }
    };
    if (kPaper && staged)
        densify(std::true_type{});
    else
        densify(std::false_type{});
    __syncthreads();

    constexpr int RPT = kTH / 8;  // output rows per thread
    const int px = ox + (tid & 31) * 2, py = oy + (tid >> 5) * RPT;
    if constexpr (UPSAMPLE) {
        const int xh = ox + kOutTW - 1 + a.pad_left, yh = oy + kTH - 1 + a.pad_top;
        if (a.F == 1 && a.vec_store && ox + kOutTW <= a.W && oy + kTH <= a.H && ox + a.pad_left >= 1 &&
            oy + a.pad_top >= 1 && ((xh - 1) >> 1) + 1 <= a.wF - 1 && ((yh - 1) >> 1) + 1 <= a.hF - 1 &&
            xh < a.xmax) {  // uniform: an interior tile
            switch (((a.pad_top - 1) & 1) * 2 + ((a.pad_left - 1) & 1)) {
                case 0: out_rows_f1<0, 0, kOutSW, RPT>(a, dense, i0, j0, px, py, pair); break;
                case 1: out_rows_f1<0, 1, kOutSW, RPT>(a, dense, i0, j0, px, py, pair); break;
                case 2: out_rows_f1<1, 0, kOutSW, RPT>(a, dense, i0, j0, px, py, pair); break;
                default: out_rows_f1<1, 1, kOutSW, RPT>(a, dense, i0, j0, px, py, pair); break;
            }
            return;
        }
    }
#pragma unroll
    for (int dy = 0; dy < RPT; ++dy) {
        const int y = py + dy;
        if (y >= a.H) continue;
        float2 o[2];
        if (UPSAMPLE) {
            int yi;
            float yf;
            lin_coef(y + a.pad_top, a.hF, a.F, &yi, &yf);
            const int r0 = yi - j0, r1 = min(yi + 1, a.hF - 1) - j0;
            const float b0 = 1.f - yf, b1 = yf;
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
        } else {
            const float2* row = dense + (y - oy) * kOutSW + (px - ox);
            o[0] = row[0];
            o[1] = row[1];
        }
        float2* dst = a.flow + (size_t)pair * a.W * a.H + (size_t)y * a.W + px;
        if (px + 1 < a.W) {
            if (a.vec_store) {
                store_flow2(dst, o[0], o[1]);
            } else {
                dst[0] = o[0];
                dst[1] = o[1];
            }
        } else if (px < a.W) {
            dst[0] = o[0];
        }
    }
}

bool output_fits(const OutputArgs& a)
{
    // patch size 8 (the fast path), at most 4 covering patches per axis
    // (steps >= 2); the LDS shapes above are derived from exactly that
    return a.hp == 4 && a.steps >= 2;
}

template <int K>
static void launch_output_k(const OutputArgs& a, dim3 grid, hipStream_t s, Timing t)
{
    if (a.paper) {
        if (a.F == 0)
            DIS_LAUNCH(t, (k_output<false, K, true>), grid, dim3(256), 0, s, a);
        else
            DIS_LAUNCH(t, (k_output<true, K, true>), grid, dim3(256), 0, s, a);
    } else if (a.F == 0) {
        DIS_LAUNCH(t, (k_output<false, K>), grid, dim3(256), 0, s, a);
    } else {
        DIS_LAUNCH(t, (k_output<true, K>), grid, dim3(256), 0, s, a);
    }
}

hipError_t launch_output(const OutputArgs& a, int batch, hipStream_t s, Timing t)
{
    if (!output_fits(a)) return hipErrorInvalidValue;
    const int th = a.F == 0 ? kOutTHf<false> : kOutTHf<true>;
    dim3 grid((a.W + kOutTW - 1) / kOutTW, (a.H + th - 1) / th, batch);
    switch ((2 * a.hp + a.steps - 1) / a.steps) {  // K = ceil(ps / steps)
        case 1: launch_output_k<1>(a, grid, s, t); break;
        case 2: launch_output_k<2>(a, grid, s, t); break;
        case 3: launch_output_k<3>(a, grid, s, t); break;
        case 4: launch_output_k<4>(a, grid, s, t); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace dis
