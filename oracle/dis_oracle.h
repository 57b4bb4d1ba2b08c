/*
 * dis_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, single thread) of the reference DIS hot path
 * (nejcgalof/Optical-Flow-using-Dense-Inverse-Search). It is the checker for
 * the HIP engine and the CPU baseline ("port") timed by bench.py. Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it;
 * the product library (libdis_hip.so) never links or calls it.
 *
 * PARITY UNPINNED: the reference ships no tests, fixtures or golden vectors
 *  and cannot be built here (it needs OpenCV 2.4 and
 * Eigen 3, neither present). This restatement follows the
 * reference source line by line (citations in dis_oracle.c); the OpenCV
 * pyramid/resize arithmetic and the Eigen reduction/LU order are restated from
 * the published algorithms of those libraries.
 */
#ifndef DIS_ORACLE_H
#define DIS_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int coarsest_scale;      /* include/optical_flow.hpp:49 */
    int finest_scale;        /* include/optical_flow.hpp:49 */
    int patch_size;          /* include/optical_flow.hpp:51 */
    int iterations;          /* include/optical_flow.hpp:50 */
    float patch_overlap;     /* include/optical_flow.hpp:52, used at src/optical_flow.cpp:38 */
    int patch_normalization; /* include/optical_flow.hpp:53 */
    int var_refine_iters;    /* 0 = the reference (no refinement) */
    int paper_mode;          /* 0 = the reference; 1 = DIS-paper residual + weighted densify */
} dis_oracle_params;

/* Grid geometry of one level (src/optical_flow.cpp:38, src/patch_grid.cpp:20-23). */
int dis_oracle_steps(int patch_size, float patch_overlap);

/* Threads for the per-level patch loop (OpenMP builds; default 1). Returns the
 * count in effect. The patches are independent, so results do not change. */
int dis_oracle_set_threads(int n);
void dis_oracle_grid(int width_l, int height_l, int steps,
                     int* npw, int* nph, int* offw, int* offh);

/* a1: pad to a multiple of 2^C (replicate, floor/ceil split) and convert to
 * float (src/main.cpp:139-160). out has Wp*Hp floats. */
void dis_oracle_padded_size(int W, int H, int coarsest, int* Wp, int* Hp,
                            int* pad_left, int* pad_top);
void dis_oracle_pad_convert(const uint8_t* in, size_t stride, int W, int H,
                            int coarsest, float* out);

/* a2-a4: image pyramid (src/main.cpp:12-38). img is Wp*Hp floats.
 * Outputs are UNPADDED planes of levels 0..C concatenated (level l at offset
 * sum_{k<l} W_k*H_k). dx/dy may be NULL. */
void dis_oracle_pyramid(const float* img, int Wp, int Hp, int coarsest,
                        float* img_levels, float* dx_levels, float* dy_levels);

/* Sobel dx/dy (ksize 3, scale 1/8, reflect-101) of one plane. */
void dis_oracle_sobel(const float* src, int W, int H, float* dx, float* dy);

/* a5-a15: mirror of OpticalFlow::OpticalFlowClass's constructor
 * (src/optical_flow.cpp:19-91). Pyramids are arrays of (coarsest+1) pointers
 * to PADDED planes (row stride W_l + 2*img_padding, pointer at the padded
 * origin). outflow is (width>>F)*(height>>F)*2 floats (u,v interleaved).
 * dbg_patch_u (optional) receives, for levels l=0..C, n_l*2 floats
 * concatenated in level order (levels < F left untouched); dbg_dense likewise
 * receives W_l*H_l*2 floats per level. Returns 0 or a negative error. */
int dis_oracle_flow_from_pyramids(
    float* const* img_first, float* const* img_first_dx, float* const* img_first_dy,
    float* const* img_second, int img_padding, float* outflow,
    int width, int height, int coarsest, int finest, int iterations,
    int patch_size, float patch_overlap, int patch_normalization,
    float* dbg_patch_u, float* dbg_dense);

/* As above, plus `var_refine_iters` fixed-point iterations of variational
 * refinement on each level's dense flow after densification
 * and `paper_mode` (template-subtracted residual and
 * residual-weighted densification, Kroeger et al. 2016 eqs. 3-4). Both are
 * absent from the reference (parity unpinned); 0, 0 = the reference. */
int dis_oracle_flow_from_pyramids_ex(
    float* const* img_first, float* const* img_first_dx, float* const* img_first_dy,
    float* const* img_second, int img_padding, float* outflow,
    int width, int height, int coarsest, int finest, int iterations,
    int patch_size, float patch_overlap, int patch_normalization, int var_refine_iters, int paper_mode,
    float* dbg_patch_u, float* dbg_dense);

/* Variational refinement of one level's dense flow (W*H*2, in place) between
 * level images I0, I1 (row stride `stride`), `fp` fixed-point iterations;
 * and the energy it decreases. Specification in dis_oracle.c. */
void dis_oracle_var_refine(const float* I0, const float* I1, int stride, int W, int H, float* flow, int fp);
double dis_oracle_var_energy(const float* I0, const float* I1, int stride, int W, int H, const float* flow);

/* a16: scale by 2^F, bilinear upsample (OpenCV INTER_LINEAR semantics) and
 * crop the padding (src/main.cpp:191-198). flowF is (Wp>>F)*(Hp>>F)*2. */
void dis_oracle_upsample_crop(const float* flowF, int Wp, int Hp, int finest,
                              int pad_left, int pad_top, int W, int H,
                              float* out);

/* Whole path: u8 frames -> full-resolution W*H*2 flow (src/main.cpp:135-198
 * with construct_pyramide and the OpticalFlowClass constructor). */
int dis_oracle_calc_u8(const dis_oracle_params* p, int W, int H,
                       const uint8_t* I0, const uint8_t* I1, size_t stride,
                       float* flow_out);

/* Middlebury colour coding, draw_optical_flow with
 * compute_color (src/color_coding.cpp:13-117) for one W*H (u,v) field into
 * W*H*3 u8 BGR (OpenCV Vec3b order). maxmotion <= 0: maxrad = max(1, max
 * radius over valid pixels) (:88-104). atan2f (:52) is restated as a fixed
 * float polynomial (the product kernel evaluates the identical one). */
void dis_oracle_flow_color(const float* flow, int W, int H, float maxmotion, uint8_t* bgr);

#ifdef __cplusplus
}
#endif
#endif
