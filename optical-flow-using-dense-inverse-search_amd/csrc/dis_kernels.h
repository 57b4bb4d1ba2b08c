// dis_kernels.h -- kernel argument blocks and host launchers.
#pragma once

#include <hip/hip_ext.h>

#include "dis_common.h"

namespace dis {

// Optional per-launch timing: events attached to the dispatch packet itself
// (hipExtLaunchKernelGGL), so timing adds no extra queue packets.
struct Timing {
    hipEvent_t start = nullptr;
    hipEvent_t stop = nullptr;
};

#define DIS_LAUNCH(T, kernel, grid, block, shmem, stream, ...)                                               \
    do {                                                                                                    \
        if ((T).start)                                                                                      \
            hipExtLaunchKernelGGL(kernel, grid, block, shmem, stream, (T).start, (T).stop, 0, __VA_ARGS__); \
        else                                                                                                \
            hipLaunchKernelGGL(kernel, grid, block, shmem, stream, __VA_ARGS__);                            \
    } while (0)

// One patch-search launch: one level, a batch of pairs.
struct SearchArgs {
    const float* img0;         // frame-0 level planes (stack), for fused gradients
    const float* img1;         // frame-1 level planes (stack)
    const float* dx;           // frame-0 Sobel dx planes (stack)
    const float* dy;           // frame-0 Sobel dy planes (stack)
    const float2* dense_coarse;  // dense flow of level l+1 (nullptr at the coarsest level)
    float2* u_out;             // patch displacements of level l
    long long plane_stride;    // floats per pair
    long long plane_off;       // this level's offset in the plane stack
    long long dense_stride;    // float2 per pair (dense stack), dense_coarse pre-offset
    long long u_stride;        // float2 per pair (patch stack), u_out pre-offset
    int phys_pad;              // 0: virtual padding (clamp image / zero gradients);
                               // >0: planes are physically padded by this many pixels
                               //     (compat path), plane_off points at the padded origin
    int W, H, steps, npw, nph, offw, offh, n;
    float tmp_lb, tmp_ub_w, tmp_ub_h, outlier;
    int iters, norm;
    int paper;                 // template-subtracted residual (dis_params.paper_mode)
};

// Fast patch-size-8 search (dis_search8.hip): gradients fused from the level
// image, init fused from the coarser level's patch displacements.
struct Search8Args {
    const float* img0;        // frame-0 level planes (stack)
    const float* img1;        // frame-1 level planes (stack)
    const float2* u_coarse;   // level l+1 patch u (pre-offset), nullptr at the coarsest level
    float2* u_out;            // level l patch u (pre-offset)
    long long plane_stride, plane_off, u_stride;
    int W, H, steps, npw, nph, offw, offh;
    int c_npw, c_nph, c_offw, c_offh;  // coarser level grid
    float tmp_lb, tmp_ub_w, tmp_ub_h;
    float thr_sq;             // largest float s with sqrtf(s) <= outlierthresh
    int iters, norm;
    int tile_stride;          // LDS tile row stride (search8_tile_stride(steps))
    int quad;                 // LPP 2 patch layout: 0 = 2 x 8, 1 = 4 x 4 patches per half-wave (search8_tile_quad)
    int lanes_per_patch;      // 1, 2, 4 or 8 (k_search8<LPP>)
    const float2* dense_coarse;  // non-null: init from the coarser level's DENSE flow (variational
    long long dense_stride;      //   refinement on) instead of u_coarse; float2 per pair
    int tile_cap;             // > 0: usable tile rows / columns capped at this (variant 9, a parity-test
                              //   switch that sends most blocks through the fallback list); 0 = the full tile
    int* fb_count;            // LPP 1/2: blocks too spread for the LDS tile are listed here
    int* fb_list;             //   (count zeroed before the launch) and redone by k_search8_fb;
                              //   nullptr: one kernel with the global-read path inline
    int paper;                // template-subtracted residual (k_search8<.., kPaper>) and
                              //   the residual-weighted coarse-to-fine initialisation, which reads the
    long long c_plane_off;    //   coarser level's planes (offset in the stack) of size c_W x c_H
    int c_W, c_H;
    int fma;                  // DIS_PRECISION_FMA: contracted warp / dot products, reciprocal solve
    // compat path (dis_flow_from_pyramids): non-null = the caller's physically
    // padded planes (pad pixels on every side, row stride W + 2 pad; plane_off
    // = the padded plane's start): template gradients from gdx/gdy_plane, I1
    // taps from the padded img1 plane
    const float* gdx_plane;
    const float* gdy_plane;
    int pad;
};

struct DensifyArgs {
    const float2* u;       // patch u of the level (pre-offset)
    float2* dense;         // dense flow of the level (pre-offset)
    long long u_stride, dense_stride;
    int W, H, ps, steps, npw, nph, offw, offh;
    // paper mode: votes weighted by 1/max(1, |I1(x+u) - I0(x)|)
    const float* img0;     // level planes of pair 0 (pre-offset), pair stride plane_stride
    const float* img1;
    long long plane_stride;
    int paper;
};

struct UpsampleArgs {
    const float2* dense;   // finest-level dense flow (pre-offset)
    float2* flow;          // W x H output, pair stride W*H
    long long dense_stride;
    int W, H, wF, hF, F, pad_left, pad_top, xmax;
    float sc;
    double inv_sc;
};

// Fused pyramid (dis_frontback.hip): u8 -> levels 1..`levels` (and 0 if write_l0).
struct PyramidArgs {
    const uint8_t* I0;
    const uint8_t* I1;
    size_t stride, pair_stride;
    int W, H, Wp, Hp, pl, pt;
    float* img0;
    float* img1;
    long long plane_stride;
    int levels;    // levels produced in-kernel, 1..6 (tile = 2^levels level-0 pixels)
    int write_l0;  // also store the level-0 magnitude plane
    long long off[kMaxLevels];  // plane offset per level
    int w[kMaxLevels];          // plane width per level
    int* zero;                  // nzero ints set to 0 by workgroup 0 (the searches' fallback counts)
    int nzero;
    int dword_ok;               // I0/I1, stride, pair_stride and pad_left 4-byte aligned: dword row loads
    int qword_ok;               // ... and 16-byte aligned, pad_left a multiple of 16: 16-byte row loads
    int vec_st;                 // k_pyr12: level-1 / level-2 rows 16-byte aligned (W_2 % 4 == 0; set by launch_pyramid2)
};

// Fused densify + upsample + crop (dis_frontback.hip).
struct OutputArgs {
    const float2* u;   // finest-level patch u (pre-offset)
    float2* flow;      // W x H x 2 output, pair stride W*H
    long long u_stride;
    int W, H, wF, hF, F, pad_left, pad_top, xmax;
    int npw, nph, offw, offh, steps, hp;
    int vec_store;     // output base is 16-byte aligned and W even
    float sc;
    // paper mode: votes weighted by 1/max(1, |I1(x+u) - I0(x)|) on level F
    int paper;
    const float* img0;  // level-F planes of pair 0 (pre-offset), pair stride plane_stride
    const float* img1;
    long long plane_stride;
};

hipError_t launch_pyramid(const PyramidArgs& a, int batch, hipStream_t s, Timing t = {});
// the same planes by two streaming kernels (dis_pyramid.hip): levels 1-2 from
// global memory, then levels 3..a.levels; needs a.levels >= 2
bool pyramid2_fits(const PyramidArgs& a);
hipError_t launch_pyramid2(const PyramidArgs& a, int batch, hipStream_t s, Timing t = {});
bool output_fits(const OutputArgs& a);
hipError_t launch_output(const OutputArgs& a, int batch, hipStream_t s, Timing t = {});
hipError_t launch_level0(const uint8_t* I0, const uint8_t* I1, size_t stride, size_t pair_stride,
                         const Geometry& g, float* img0, float* img1, int batch, hipStream_t s);
hipError_t launch_down2(const Geometry& g, int l, float* img0, float* img1, int batch, hipStream_t s);
hipError_t launch_sobel(const Geometry& g, int l, const float* img0, float* dx, float* dy, int batch,
                        hipStream_t s);
hipError_t launch_search_generic(const SearchArgs& a, int ps, int batch, hipStream_t s, Timing t = {});
int search8_tile_stride(int steps, int lanes_per_patch);
int search8_tile_quad(int steps, int lanes_per_patch);  // LPP 2: 4 x 4-patch half-waves (Search8Args.quad)
bool search8_lpp1_fits(int steps);
hipError_t launch_search8(const Search8Args& a, int batch, hipStream_t s, Timing t = {});
// one wave64 per patch (dis_search_wave.hip; lanes_per_patch 64, variant 6)
hipError_t launch_search_wave(const Search8Args& a, int batch, hipStream_t s, Timing t = {});
hipError_t launch_densify(const DensifyArgs& a, int batch, hipStream_t s);
hipError_t launch_upsample(const UpsampleArgs& a, int batch, hipStream_t s);

// Middlebury colour coding of n W x H (u,v) fields into BGR u8 (dis_color.hip);
// maxbits: 32 * n device uints of scratch.
hipError_t launch_flow_color(const float* flow, int n, int W, int H, float maxmotion, uint8_t* bgr,
                             unsigned int* maxbits, hipStream_t s);
// device workspace words launch_flow_color needs for n fields (zeroed by it)
size_t flow_color_ws_words(int n);

// Variational refinement of one level's dense flow (dis_varref.hip).
constexpr int kVarRefPlanes = 8;   // per-pair workspace planes
constexpr int kVarRefSor = 5;      // red-black SOR sweeps per fixed-point iteration
struct VarRefArgs {
    const float* img0;      // level planes of pair 0 (pre-offset), pair stride plane_stride
    const float* img1;
    long long plane_stride;
    float2* flow;           // dense flow of pair 0 (pre-offset), refined in place
    long long flow_stride;  // float2 per pair
    float* ws;              // workspace of pair 0, pair stride ws_stride floats
    long long ws_plane, ws_stride;
    int W, H, iters;
};
// tfn (optional, kernel timing): events for each k_vr_lin (kind 0) and
// k_vr_sor (kind 1) launch
typedef Timing (*VarRefTiming)(void* ctx, int kind);
hipError_t launch_var_refine(const VarRefArgs& a, int n, hipStream_t s, VarRefTiming tfn = nullptr,
                             void* tctx = nullptr);

}  // namespace dis
