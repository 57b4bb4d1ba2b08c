// dis_common.h -- shared host/device definitions of the DIS engine.
//
// Geometry follows the reference exactly (float arithmetic where the reference
// uses float): src/optical_flow.cpp:33-63, src/patch_grid.cpp:17-51.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "dis_abi.h"

namespace dis {

constexpr int kMaxLevels = 16;

// One pyramid level of one pair (image_parameters, include/optical_flow.hpp:14-24,
// plus the PatchGrid geometry, src/patch_grid.cpp:20-23).
struct LevelGeom {
    int W, H;                      // level size (int(W*2^-l), src/optical_flow.cpp:51-53)
    int steps;                     // grid stride
    int npw, nph, offw, offh, n;   // patch grid
    float tmp_lb, tmp_ub_w, tmp_ub_h;  // valid region (src/optical_flow.cpp:55-57)
    long long plane_off;           // float offset of this level in a per-pair plane stack
    long long u_off;               // float2 offset of this level's patch array
    long long dense_off;           // float2 offset of this level's dense flow
};

struct Geometry {
    int W, H;              // input size
    int Wp, Hp;            // padded to a multiple of 2^C (src/main.cpp:139-155)
    int pad_left, pad_top;
    int C, F, ps, iters, norm, steps;
    long long plane_stride;  // floats per pair per plane stack (levels 0..C)
    long long u_stride;      // float2 per pair (patch arrays, levels 0..C)
    long long dense_stride;  // float2 per pair (dense flows, levels 0..C)
    LevelGeom lv[kMaxLevels];
};

// Fills g from validated params; returns false on inconsistent sizes.
bool make_geometry(const dis_params& p, int W, int H, Geometry* g);

}  // namespace dis
