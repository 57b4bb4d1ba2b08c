/*
 * dis_abi.h -- C-ABI of the MI355X-native DIS (Dense Inverse Search) optical
 * flow engine. Plain C types only: pointers, sizes, ints, floats.
 *
 * The reference (nejcgalof/Optical-Flow-using-Dense-Inverse-Search) has no
 * C-ABI or plugin interface; its hot path is reached through
 *   (R1) construct_pyramide()                       src/main.cpp:12-50
 *   (R2) OpticalFlow::OpticalFlowClass::ctor(...)   include/optical_flow.hpp:43-54,
 *                                                   src/optical_flow.cpp:19-91
 *   (R3) the pad / convert / upsample / crop glue   src/main.cpp:135-160, 191-198
 * Each entry point below names the reference interface it replaces. The C++
 * facade in include/dis/dis.hpp (DenseInverseSearch::calc and the
 * OpticalFlow::OpticalFlowClass compatibility class) is built on these.
 *
 * Threading: a dis_ctx is bound to one HIP device; calls on one context must
 * be serialised by the caller. Distinct contexts may run concurrently.
 * Errors: every call returns a dis_status; dis_last_error() returns the
 * calling thread's last error text. No C++ exception crosses this boundary.
 */
#ifndef DIS_ABI_H
#define DIS_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DIS_ABI_VERSION 8

typedef enum dis_status {
    DIS_OK = 0,
    DIS_ERR_INVALID_ARGUMENT = -1, /* bad parameter / pointer / size          */
    DIS_ERR_UNSUPPORTED = -2,      /* valid request this build does not do     */
    DIS_ERR_DEVICE = -3,           /* HIP runtime error or no usable device    */
    DIS_ERR_OUT_OF_MEMORY = -4,    /* device or host allocation failed         */
    DIS_ERR_INTERNAL = -5
} dis_status;

/* Build-defined presets (the reference has none). */
typedef enum dis_preset {
    DIS_PRESET_ULTRAFAST = 0, /* ps 8, overlap 0.5   (steps 4), it 12,  F 2, C auto */
    DIS_PRESET_FAST = 1,      /* ps 8, overlap 0.5   (steps 4), it 16,  F 2, C auto */
    DIS_PRESET_MEDIUM = 2,    /* ps 8, overlap 0.625 (steps 3), it 25,  F 1, C auto */
    DIS_PRESET_SLOW = 3,      /* ps 8, overlap 0.75  (steps 2), it 128, F 0, C auto */
    DIS_PRESET_REFERENCE = 4  /* CLI defaults src/main.cpp:66-71: ps 8, 0.7, it 1000, F 0, C 3 */
} dis_preset;

typedef enum dis_mem {
    DIS_MEM_HOST = 0,  /* pointers are host memory: the call copies and synchronises */
    DIS_MEM_DEVICE = 1 /* pointers are device memory on the context's device: the call
                          is asynchronous on `stream` */
} dis_mem;

/* The reference's scalar knobs (src/optical_flow.cpp:19-31; CLI src/main.cpp:63-92). */
typedef struct dis_params {
    int coarsest_scale;      /* C: coarsest pyramid level, >= finest_scale              */
    int finest_scale;        /* F: finest level searched; output upsampled by 2^F       */
    int patch_size;          /* even, 2..16                                              */
    int iterations;          /* >= 0; each patch does iterations+1 updates (Q3)          */
    float patch_overlap;     /* [0,1); steps = max(1, floor(ps*(1-overlap))) in float    */
    int patch_normalization; /* 0/1: mean-normalise the warped patch (src/patch.cpp:264) */
    int var_refine_iters;    /* 0 = the reference (no refinement, README.md:11); > 0: fixed-point iterations of
                                variational refinement per level (parity unpinned) */
    int paper_mode;          /* 0 = the reference; 1 = the DIS paper's residual and densification (SURVEY 8f
                                row 4, not in the reference, parity unpinned): template-subtracted (and, with
                                normalisation, mean-normalised) residual instead of Q2's warped-patch-only one,
                                and votes weighted by 1/max(1, |I1(x+u) - I0(x)|) instead of Q6's plain mean */
} dis_params;

typedef struct dis_ctx dis_ctx;

/* Work/traffic figures of one frame pair (SURVEY.md 8d formula). */
typedef struct dis_workload {
    int padded_width, padded_height;
    int steps;
    long long patches;          /* sum of n_l over levels F..C                 */
    long long updates;          /* sum of n_l*(iterations+1)                    */
    double algorithmic_bytes;   /* SURVEY.md 8d "B" for one pair                */
    double search_bytes_finest; /* 16*W_F*H_F + 16*n_F: the finest search launch */
    double search_bytes_all;    /* sum over search launches (levels F..C) of
                                   16*W_l*H_l + 16*n_l (+ 8*W_{l+1}*H_{l+1} coarse read) */
    int search_launches;        /* C - F + 1 */
    long long patches_finest;   /* n_F                                          */
    double search_flops_finest; /* algorithmic f32 operations of the finest search
                                   for one pair: n_F * (16N - 3 + 6 + (it+1)(13N + 12))
                                   with normalisation, N = patch_size^2 */
} dis_workload;

int dis_abi_version(void);
const char* dis_last_error(void);
/* "product" (ABI v6; since v7 the sources have no compile-time variants,
 * so every build is the product build) */
const char* dis_build_kind(void);

/* Fill *out with the preset's knobs for a W x H input (C = auto rule). */
dis_status dis_preset_params(dis_preset preset, int width, int height, dis_params* out);

/* Validate knobs for a W x H input (what dis_create checks). */
dis_status dis_validate_params(const dis_params* params, int width, int height);

/* Work and algorithmic bytes per pair for these knobs. */
dis_status dis_workload_info(const dis_params* params, int width, int height, dis_workload* out);

/* Create a context for W x H u8 pairs on HIP device `device`, with device
 * workspace for up to max_batch pairs per call (no allocation in calc). */
dis_status dis_create(dis_ctx** out, const dis_params* params, int width, int height,
                      int max_batch, int device);
dis_status dis_destroy(dis_ctx* ctx);

/* One pair: u8 grayscale frames (row stride `stride` bytes, 0 = width) to a
 * full-resolution W x H x 2 float flow, (u,v) interleaved, row-major.
 * Replaces R3 + R1 + R2 for one pair (src/main.cpp:135-198). */
dis_status dis_calc_u8(dis_ctx* ctx, const uint8_t* I0, const uint8_t* I1, size_t stride,
                       float* flow, dis_mem where, void* stream);

/* n pairs in one call: pair k's frames at I0 + k*pair_stride (bytes), its
 * flow at flow + k*W*H*2 floats. n <= max_batch. */
dis_status dis_calc_batch_u8(dis_ctx* ctx, int n, const uint8_t* I0, const uint8_t* I1,
                             size_t stride, size_t pair_stride, float* flow,
                             dis_mem where, void* stream);

/* Host-frame path (ABI v8): with DIS_MEM_HOST a batch runs in chunks of
 * chunk_pairs pairs (0 = auto, the default: about 64 MB of flow per chunk)
 * through two device slots; chunk j+1's upload, chunk j's computation and
 * chunk j-1's download overlap (the downloads are issued by a thread of the
 * context). The copies go straight between the caller's buffers and the
 * device; page-locked caller buffers (dis_host_alloc, hipHostMalloc /
 * hipHostRegister) make them asynchronous. The results are the device path's,
 * bit for bit, for any chunking. The reference's per-pair loop hands over host
 * frames and gets host flow back (src/main.cpp:102-206). */
dis_status dis_set_host_pipeline(dis_ctx* ctx, int chunk_pairs);
typedef struct dis_host_info {
    int chunk_pairs;     /* pairs per chunk (0 before the first host call)          */
    int last_chunks;     /* chunks of the last host call                            */
    int last_direct_in;  /* 1: the last host call's frames were page-locked         */
    int last_direct_out; /* 1: the last host call's flow buffer was page-locked     */
} dis_host_info;
dis_status dis_host_pipeline_info(dis_ctx* ctx, dis_host_info* out);
/* Page-locked host memory for frames and flows (hipHostMalloc); no context. */
dis_status dis_host_alloc(size_t bytes, void** out);
dis_status dis_host_free(void* p);

/* Compatibility entry with the exact semantics of the reference constructor
 * OpticalFlowClass(...) (include/optical_flow.hpp:43-54): host pyramids of
 * (coarsest+1) PADDED planes (row stride W_l + 2*img_padding, pointer at the
 * padded origin, as built by construct_pyramide, src/main.cpp:41-49), output
 * `outflow` = (width>>F) x (height>>F) x 2 floats at the finest level.
 * width/height must be multiples of 2^coarsest. The *_dx/_dy planes of the
 * second frame are accepted and unused, as in the reference (Q15).
 * Synchronous; runs on HIP device `device`. */
dis_status dis_flow_from_pyramids(const float* const* img_first, const float* const* img_first_dx,
                                  const float* const* img_first_dy, const float* const* img_second,
                                  const float* const* img_second_dx, const float* const* img_second_dy,
                                  int img_padding, float* outflow, int width, int height,
                                  int coarsest_scale, int finest_scale, int iterations,
                                  int patch_size, float patch_overlap, int patch_normalization,
                                  int device);

/* Stage dumps for parity tests: copy one intermediate of pair `pair` from the
 * last calc on this context into host memory `dst` (count floats). Stages:
 * level image frame 0 / frame 1, frame-0 Sobel dx / dy, per-patch u (n_l*2),
 * dense flow (W_l*H_l*2). Requires dis_set_debug(ctx, 1) before the calc.
 * DIS_STAGE_FALLBACK (count 1, no debug mode needed): the number of patch
 * blocks of level `level` whose start positions were too spread for the LDS
 * tile and were searched by the fallback kernel in the last dis_calc_* on this
 * context (graph replays included), summed over the call's sub-batches (`pair`
 * only has to lie in the last batch). dis_flow_from_pyramids has no context
 * and keeps its own counters: a context's count is never changed by it. */
typedef enum dis_stage {
    DIS_STAGE_IMG0 = 0,
    DIS_STAGE_IMG1 = 1,
    DIS_STAGE_DX0 = 2,
    DIS_STAGE_DY0 = 3,
    DIS_STAGE_PATCH_U = 4,
    DIS_STAGE_DENSE = 5,
    DIS_STAGE_FALLBACK = 6
} dis_stage;
dis_status dis_set_debug(dis_ctx* ctx, int enable);

/* Concurrency: a batch call is split into `streams` sub-batches (1..8,
 * default 2) that run on context-owned HIP streams forked from and joined
 * back into the caller's stream. Results do not depend on this setting. */
dis_status dis_set_concurrency(dis_ctx* ctx, int streams);

/* Kernel variant: 0 = auto (specialised kernels where available: the
 * patch_size-8 search with 8 lanes per patch on levels with few patches and 2
 * lanes per patch on the rest), 1 = generic kernels only, 2 / 3 / 4 / 5 = the
 * patch_size-8 search with 4 / 2 / 8 / 1 lanes per patch on every level (5:
 * where the 16x8-patch block fits, grid step <= 7; else 2), 6 = one wave64
 * per patch (lane = pixel) on every exact non-paper level (else 2), 9 = 2
 * lanes per patch on every level with the usable LDS tile
 * capped at 24 rows / columns, so that most patch blocks take the fallback
 * list and kernel (a parity-test switch: natural inputs rarely spread a
 * block's start positions beyond the full tile). All are bit-identical; the
 * switch exists for parity tests and A/B timing. 7 and 8 (ABI v6: one launch
 * per coarse level, the fused coarse head) were removed in v7 -- the head
 * measured slower -- and are refused. */
dis_status dis_set_kernel_variant(dis_ctx* ctx, int variant);

/* Arithmetic of the patch_size-8 search kernels (ABI v4; no reference
 * counterpart -- the reference's own rounding is DIS_PRECISION_EXACT):
 *   DIS_PRECISION_EXACT (default): every float operation separately rounded in
 *     the reference's order -- bit-identical to the oracle;
 *   DIS_PRECISION_FMA: the bilinear warp, the steepest-descent and Hessian dot
 *     products contracted into fma, the LU solve by the pivots' reciprocals --
 *     within the stated tolerance of the reference (mean EPE
 *     <= 3.3e-4 px, p99.9 <= 5.1e-2 px, patch flips <= 0.014 %), faster.
 * Generic kernels (other patch sizes) and paper mode always run exact. */
/* HIP graphs (ABI v4): with graphs on (the default) a batch call is captured
 * once per (n, frame/flow pointers and strides, concurrency, precision,
 * variant) and replayed as one graph -- the fork into the sub-batch streams,
 * every level's launches and the join -- instead of ~25 eager launches; a
 * changed key re-captures (an LRU of four executable graphs per context; an
 * exec is updated only after its previous replay has finished). Kernel timing,
 * debug dumps and variational refinement run eagerly. The
 * capture is thread-local: if another thread synchronises the device or uses
 * the legacy default stream meanwhile, HIP invalidates it and that call runs
 * eagerly instead. Results do not depend on this setting. */
dis_status dis_set_graphs(dis_ctx* ctx, int enable);

/* Stream plans of a batch call (ABI v8; host only, no device needed). Ops are
 * 4 ints each: {kind (0 record, 1 wait, 2 work), stream (0 = the caller's,
 * 1 + k = sub-batch stream k), event (0 = fork, 1 + k = sub-batch k's join),
 * stage}. dis_batch_stream_plan writes the plan a call with `nsub` (2..8)
 * sub-batches and `nstages` stages issues (count ops; ops may be NULL to ask
 * for the count). dis_check_stream_plan applies the rules a plan must keep to
 * be captured into a HIP graph (every waited event recorded in the capture,
 * work only on streams in it, every stream joined back) and
 * returns DIS_ERR_UNSUPPORTED with the broken rule in dis_last_error()
 * otherwise. The runtime checks its plan this way before every capture. */
dis_status dis_batch_stream_plan(int nsub, int nstages, int* ops, int capacity, int* count);
dis_status dis_check_stream_plan(const int* ops, int nops, int nstreams, int nevents);

typedef enum dis_precision { DIS_PRECISION_EXACT = 0, DIS_PRECISION_FMA = 1 } dis_precision;
dis_status dis_set_precision(dis_ctx* ctx, int mode);

/* ABI v6: dis_pipeline_link (v5) is gone -- its linked calls ran eagerly on
 * the device's shared sub-batch streams and lost to two unlinked contexts on
 * two caller streams (DESIGN.md 4 "pipelined"), which needs no API. */
dis_status dis_stage_size(dis_ctx* ctx, int stage, int level, size_t* count);
dis_status dis_debug_dump(dis_ctx* ctx, int stage, int level, int pair, float* dst, size_t count);

/* Per-kernel timing with HIP events recorded on the context's launch stream
 * around every launch of the named kernel class (bench / roofline use).
 * kernel: 0 = fused pyramid, 1 = patch search (all levels), 2 = patch search
 * (finest level only), 3 = fused densify+upsample+crop, 4 / 5 = variational
 * refinement's linearisation / SOR launches at the finest level (ABI v7;
 * timing replaces the refinement's per-level graphs by eager launches).
 * Enabling timing while
 * it is off starts a fresh measurement (accumulated launches and times are
 * cleared); dis_kernel_time returns the totals since then (the event pool
 * grows as needed, so no launch is left out; DIS_ERR_DEVICE if event creation
 * failed and records were lost). */
dis_status dis_set_kernel_timing(dis_ctx* ctx, int enable);
dis_status dis_kernel_time(dis_ctx* ctx, int kernel, int* launches, double* total_ms);

/* Middlebury flow colour coding, src/color_coding.cpp:13-117 (draw_optical_flow
 * with compute_color): n W x H (u,v) float fields (interleaved, row-major,
 * pair stride W*H*2) to n W x H x 3 u8 BGR images (OpenCV Vec3b order).
 * maxmotion > 0 fixes the motion range; <= 0 uses max(1, max |u| over valid
 * pixels) per field, as the reference's default -1. Invalid vectors (NaN or
 * |component| >= 1e9) are black. Host pointers: synchronous; device pointers:
 * asynchronous on `stream`. Runs on HIP device `device`. */
dis_status dis_flow_color(const float* flow, int n, int width, int height, float maxmotion, uint8_t* bgr,
                          dis_mem where, void* stream, int device);

/* Middlebury .flo files (src/IO_flow.cpp:10-98): "PIEH", int32 width,
 * int32 height, width*height*channels float32 row-major interleaved,
 * little-endian; channels 1 (depth), 2 (flow) or 4 (scene flow). Host only
 * (no GPU). Reading validates the tag, the size against the buffer and the
 * exact file length. */
dis_status dis_flo_info(const char* path, int* width, int* height);
dis_status dis_read_flo(const char* path, float* data, int width, int height, int channels);
dis_status dis_write_flo(const char* path, const float* data, int width, int height, int channels);

/* Deterministic synthetic pair (SURVEY.md 8d generator): multi-octave value
 * noise I0 and I1 = I0 warped by a smooth sinusoidal flow; optional
 * ground-truth flow (W*H*2). Host memory, host compute; seed k -> pair k. */
dis_status dis_synth_pair(uint64_t seed, int width, int height, uint8_t* I0, uint8_t* I1,
                          float* gt_flow);

#ifdef __cplusplus
}
#endif
#endif /* DIS_ABI_H */
