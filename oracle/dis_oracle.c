/*
 * dis_oracle.c -- TEST INFRASTRUCTURE ONLY (see dis_oracle.h).
 *
 * CPU restatement of the reference DIS hot path. Every function cites the
 * reference lines (paths relative to the reference checkout) it restates.
 * Built with -O2 -ffp-contract=off so every float operation rounds exactly
 * once, in the order written, as in the reference's MSVC/SSE2 build.
 *
 * PARITY UNPINNED: no reference test, fixture or golden vector exists, and the
 * reference cannot be built here (OpenCV 2.4 + Eigen 3 absent). The arithmetic
 * of those two libraries is restated from their published algorithms:
 *   - OpenCV 2.4 Sobel (separable, scale folded into the smoothing kernel,
 *     BORDER_REFLECT_101), resize 0.5x INTER_LINEAR == fast 2x2 area mean,
 *     resize up INTER_LINEAR (two-tap, clamped at the borders);
 *   - Eigen 3.3 vectorized sum() over a dynamic float vector (SSE2: two 4-wide
 *     packet accumulators, predux = (p0+p2)+(p1+p3)), 2x2 determinant and
 *     PartialPivLU solve (row pivot on |a00| < |a10|, unit-lower then upper
 *     triangular substitution), norm() = sqrt(x*x + y*y).
 */
#include "dis_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* worker threads (1 = the reference's single thread; OpenMP builds only) for
 * the per-level patch loop and the per-pixel stages (rows split among threads;
 * densify split into row bands that each keep the patch-id accumulation
 * order). A test-side speed knob: results are identical for every count. */
static int g_threads = 1;
#ifdef _OPENMP
#define DIS_OMP_ROWS _Pragma("omp parallel for schedule(static) num_threads(g_threads) if (g_threads > 1)")
#else
#define DIS_OMP_ROWS
#endif

/* ------------------------------------------------------------------------- */
/* Eigen-order helpers                                                        */
/* ------------------------------------------------------------------------- */

/* Eigen redux_impl<LinearVectorizedTraversal> over n floats with 4-wide SSE
 * packets and 16-byte aligned storage (alignedStart = 0). Used for every
 * .sum() on the path: src/patch.cpp:82-84, 171-172, 265. */
static float eigen_sum(const float* x, int n)
{
#if defined(DIS_ORACLE_SEQ_SUM)
    /* tolerance calibration only: plain left-to-right order */
    float q = x[0];
    for (int i = 1; i < n; ++i) q = q + x[i];
    return q;
#elif defined(DIS_ORACLE_AVX_SUM)
    /* tolerance calibration only: Eigen with 8-wide AVX packets
     * (two packet accumulators over blocks of 16, predux = lo4 + hi4, then the
     * 4-wide (q0+q2)+(q1+q3)) */
    if (n >= 8) {
        const int a8 = (n / 8) * 8, a16 = (n / 16) * 16;
        float p0[8], p1[8];
        for (int j = 0; j < 8; ++j) p0[j] = x[j];
        if (a8 > 8) {
            for (int j = 0; j < 8; ++j) p1[j] = x[8 + j];
            for (int i = 16; i < a16; i += 16)
                for (int j = 0; j < 8; ++j) {
                    p0[j] = p0[j] + x[i + j];
                    p1[j] = p1[j] + x[i + 8 + j];
                }
            for (int j = 0; j < 8; ++j) p0[j] = p0[j] + p1[j];
            if (a8 > a16)
                for (int j = 0; j < 8; ++j) p0[j] = p0[j] + x[a16 + j];
        }
        float h[4];
        for (int j = 0; j < 4; ++j) h[j] = p0[j] + p0[4 + j];
        float r = (h[0] + h[2]) + (h[1] + h[3]);
        for (int i = a8; i < n; ++i) r = r + x[i];
        return r;
    }
#endif
    if (n < 4) { /* DefaultTraversal */
        float r = x[0];
        for (int i = 1; i < n; ++i) r = r + x[i];
        return r;
    }
    const int aligned = (n / 4) * 4;
    const int aligned2 = (n / 8) * 8;
    float p0[4], p1[4];
    for (int j = 0; j < 4; ++j) p0[j] = x[j];
    if (aligned > 4) {
        for (int j = 0; j < 4; ++j) p1[j] = x[4 + j];
        for (int i = 8; i < aligned2; i += 8)
            for (int j = 0; j < 4; ++j) {
                p0[j] = p0[j] + x[i + j];
                p1[j] = p1[j] + x[i + 4 + j];
            }
        for (int j = 0; j < 4; ++j) p0[j] = p0[j] + p1[j];
        if (aligned > aligned2)
            for (int j = 0; j < 4; ++j) p0[j] = p0[j] + x[aligned2 + j];
    }
    float r = (p0[0] + p0[2]) + (p0[1] + p0[3]);
    for (int i = aligned; i < n; ++i) r = r + x[i];
    return r;
}

/* Eigen PartialPivLU<Matrix2f>::solve (src/patch.cpp:176). h is row-major
 * {h00, h01, h10, h11}. */
static void eigen_lu_solve2(const float h[4], float b0, float b1, float* x0, float* x1)
{
    float a00 = h[0], a01 = h[1], a10 = h[2], a11 = h[3];
    float c0 = b0, c1 = b1;
    /* k = 0: pivot = argmax |col 0| (first index wins ties) */
    if (fabsf(a10) > fabsf(a00)) {
        float t;
        t = a00; a00 = a10; a10 = t;
        t = a01; a01 = a11; a11 = t;
        t = c0; c0 = c1; c1 = t;
    }
    float l10 = a10;
    if (a00 != 0.0f) l10 = a10 / a00;
    a11 = a11 - l10 * a01;
    /* unit-lower forward substitution */
    c1 = c1 - l10 * c0;
    /* upper back substitution */
    c1 = c1 / a11;
    c0 = c0 - c1 * a01;
    c0 = c0 / a00;
    *x0 = c0;
    *x1 = c1;
}

/* ------------------------------------------------------------------------- */
/* a1: pad + convert (src/main.cpp:139-160)                                   */
/* ------------------------------------------------------------------------- */

void dis_oracle_padded_size(int W, int H, int coarsest, int* Wp, int* Hp,
                            int* pad_left, int* pad_top)
{
    int sf = 1 << coarsest;                  /* src/main.cpp:141 */
    int padw = (W % sf) ? sf - W % sf : 0;   /* :142-145 */
    int padh = (H % sf) ? sf - H % sf : 0;   /* :146-149 */
    *Wp = W + padw;
    *Hp = H + padh;
    *pad_left = padw / 2;                    /* floor(padw/2), :152 */
    *pad_top = padh / 2;
}

static int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

void dis_oracle_pad_convert(const uint8_t* in, size_t stride, int W, int H,
                            int coarsest, float* out)
{
    int Wp, Hp, pl, pt;
    dis_oracle_padded_size(W, H, coarsest, &Wp, &Hp, &pl, &pt);
    /* copyMakeBorder BORDER_REPLICATE (:152-153), convertTo(CV_32F) (:159) */
    DIS_OMP_ROWS
    for (int y = 0; y < Hp; ++y) {
        const uint8_t* row = in + (size_t)clampi(y - pt, 0, H - 1) * stride;
        for (int x = 0; x < Wp; ++x)
            out[(size_t)y * Wp + x] = (float)row[clampi(x - pl, 0, W - 1)];
    }
}

/* ------------------------------------------------------------------------- */
/* a2-a4: pyramid (src/main.cpp:12-38)                                        */
/* ------------------------------------------------------------------------- */

/* BORDER_REFLECT_101: -1 -> 1, n -> n-2 (OpenCV borderInterpolate). */
static int reflect101(int i, int n)
{
    if (n == 1) return 0;
    while (i < 0 || i >= n) {
        if (i < 0) i = -i;
        if (i >= n) i = 2 * n - 2 - i;
    }
    return i;
}

/* cv::Sobel(src, dst, CV_32F, 1,0 / 0,1, 3, 1/8.0) (src/main.cpp:19-20,34-35):
 * separable sepFilter2D, row pass then column pass; the 1/8 scale is folded
 * into the smoothing kernel [1 2 1]/8 = {0.125, 0.25, 0.125}.
 *   dx: R(y) = I(x+1)-I(x-1);      dx = R(y)*0.25 + (R(y-1)+R(y+1))*0.125
 *   dy: S(y) = I(x)*0.25 + (I(x-1)+I(x+1))*0.125;   dy = S(y+1) - S(y-1)   */
void dis_oracle_sobel(const float* src, int W, int H, float* dx, float* dy)
{
    float* R = (float*)malloc(sizeof(float) * (size_t)W * H);
    float* S = (float*)malloc(sizeof(float) * (size_t)W * H);
    DIS_OMP_ROWS
    for (int y = 0; y < H; ++y) {
        const float* row = src + (size_t)y * W;
        for (int x = 0; x < W; ++x) {
            float l = row[reflect101(x - 1, W)], c = row[x], r = row[reflect101(x + 1, W)];
            R[(size_t)y * W + x] = r - l;
            S[(size_t)y * W + x] = c * 0.25f + (l + r) * 0.125f;
        }
    }
    DIS_OMP_ROWS
    for (int y = 0; y < H; ++y) {
        const size_t ym = (size_t)reflect101(y - 1, H) * W;
        const size_t yc = (size_t)y * W;
        const size_t yp = (size_t)reflect101(y + 1, H) * W;
        for (int x = 0; x < W; ++x) {
            if (dx) dx[yc + x] = R[yc + x] * 0.25f + (R[ym + x] + R[yp + x]) * 0.125f;
            if (dy) dy[yc + x] = S[yp + x] - S[ym + x];
        }
    }
    free(R);
    free(S);
}

void dis_oracle_pyramid(const float* img, int Wp, int Hp, int coarsest,
                        float* img_levels, float* dx_levels, float* dy_levels)
{
    size_t off = 0, prev_off = 0;
    for (int l = 0; l <= coarsest; ++l) {
        const int W = Wp >> l, H = Hp >> l;
        float* lev = img_levels + off;
        if (l == 0) {
            /* level 0 = Sobel magnitude of the input (src/main.cpp:16-27) */
            float* gx = (float*)malloc(sizeof(float) * (size_t)W * H);
            float* gy = (float*)malloc(sizeof(float) * (size_t)W * H);
            dis_oracle_sobel(img, W, H, gx, gy);
            const long long npx = (long long)W * H;
            DIS_OMP_ROWS
            for (long long i = 0; i < npx; ++i) {
                float t1 = gx[i] * gx[i];   /* dx.mul(dx)  :21 */
                float t2 = gy[i] * gy[i];   /* dy.mul(dy)  :22 */
                float s = t1 + t2;          /* dx2 + dy2   :23 */
                lev[i] = sqrtf(s);          /* cv::sqrt    :24 */
            }
            free(gx);
            free(gy);
        } else {
            /* resize 0.5x INTER_LINEAR == fast area 2x2 (src/main.cpp:29):
             * sum over (sy, sx) in row-major order, times 0.25 */
            const float* p = img_levels + prev_off;
            const int Wq = Wp >> (l - 1);
            DIS_OMP_ROWS
            for (int y = 0; y < H; ++y)
                for (int x = 0; x < W; ++x) {
                    const float* a = p + (size_t)(2 * y) * Wq + 2 * x;
#if defined(DIS_ORACLE_CV_SIMD_DOWN)
                    /* tolerance variant: OpenCV >= 3.0's
                     * ResizeAreaFastVec_SIMD_32f adds the two vertical
                     * pairs first, (tl+bl)+(tr+br), for every column but
                     * the W % 4 tail, which keeps the scalar order */
                    if (x < W - W % 4) {
                        lev[(size_t)y * W + x] = ((a[0] + a[Wq]) + (a[1] + a[Wq + 1])) * 0.25f;
                        continue;
                    }
#endif
                    float s = a[0] + a[1];
                    s = s + a[Wq];
                    s = s + a[Wq + 1];
                    lev[(size_t)y * W + x] = s * 0.25f;
                }
        }
        /* per-level Sobel dx/dy (src/main.cpp:34-37) */
        if (dx_levels || dy_levels)
            dis_oracle_sobel(lev, W, H, dx_levels ? dx_levels + off : NULL,
                             dy_levels ? dy_levels + off : NULL);
        prev_off = off;
        off += (size_t)W * H;
    }
}

/* ------------------------------------------------------------------------- */
/* a6/a7: parameters and grid                                                 */
/* ------------------------------------------------------------------------- */

int dis_oracle_steps(int patch_size, float patch_overlap)
{
    /* src/optical_flow.cpp:38: max(1, (int)floor(ps*(1 - overlap))) in float */
    float f = floorf((float)patch_size * (1.0f - patch_overlap));
    int s = (int)f;
    return s < 1 ? 1 : s;
}

void dis_oracle_grid(int width_l, int height_l, int steps,
                     int* npw, int* nph, int* offw, int* offh)
{
    /* src/patch_grid.cpp:20-23 */
    *npw = (int)ceilf((float)width_l / (float)steps);
    *nph = (int)ceilf((float)height_l / (float)steps);
    *offw = (width_l - (*npw - 1) * steps) / 2;
    *offh = (height_l - (*nph - 1) * steps) / 2;
}

/* ------------------------------------------------------------------------- */
/* a8-a13: one patch (src/patch.cpp)                                           */
/* ------------------------------------------------------------------------- */

typedef struct {
    /* fix_parameters (include/optical_flow.hpp:26-37) */
    int ps, iterations, normalization, npts;
    float outlierthresh;
    /* image_parameters (include/optical_flow.hpp:14-24) */
    int width, height, pad, tmp_w;
    float tmp_lb, tmp_ub_w, tmp_ub_h;
    /* SURVEY 8f row 4 (not in the reference): DIS-paper residual */
    int paper;
} level_ctx;

/* Patch::get_patch_second_image (src/patch.cpp:207-267). */
static void patch_second_image(const level_ctx* c, const float* img_second,
                               float px, float py, float* out)
{
    float l = floorf(px);                  /* :222 */
    float k = floorf(py);                  /* :223 */
    float a = px - l;                      /* :225 */
    float b = py - k;                      /* :226 */
    float w0 = (1 - a) * (1 - b);          /* :227 */
    float w1 = a * (1 - b);                /* :228 */
    float w2 = b * (1 - a);                /* :229 */
    float w3 = a * b;                      /* :230 */
    int X = (int)(ceilf(px + .00001f) + (float)c->pad);   /* :233 */
    int Y = (int)(ceilf(py + .00001f) + (float)c->pad);   /* :234 */
    int lb = -c->ps / 2, ub = c->ps / 2 - 1;               /* :237-238 */
    int ind_e = X - c->ps / 2;                             /* :244 */
    int it = 0;
    for (int ry = Y + lb; ry <= Y + ub; ++ry) {            /* :247 */
        int ia = ind_e + ry * c->tmp_w;                    /* :250 */
        int ic = ind_e + (ry - 1) * c->tmp_w;              /* :251 */
        int ib = ia - 1, id = ic - 1;                      /* :252-253 */
        for (int rx = X + lb; rx <= X + ub; ++rx) {        /* :256 */
            float t = w3 * img_second[ia];                 /* :258 left to right */
            t = t + w2 * img_second[ib];
            t = t + w1 * img_second[ic];
            t = t + w0 * img_second[id];
            out[it++] = t;
            ia++, ib++, ic++, id++;
        }
    }
    if (c->normalization) {                                /* :264-266 */
        float mean = eigen_sum(out, c->npts) / (float)c->npts;
        for (int i = 0; i < c->npts; ++i) out[i] = out[i] - mean;
    }
}

static int out_of_bounds(const level_ctx* c, float x, float y)
{
    /* src/patch.cpp:131-132 and :187-188 */
    return x < c->tmp_lb || y < c->tmp_lb || x > c->tmp_ub_w || y > c->tmp_ub_h;
}

/* Patch::init_patch + Patch::inverse_search for one patch; returns u. */
static void patch_search(const level_ctx* c, const float* imgp, const float* dxp, const float* dyp,
                         const float* img_second, float refx, float refy,
                         float initx, float inity, float* gdx, float* gdy,
                         float* second, float* ux, float* uy)
{
    /* get_gradients_on_patch (src/patch.cpp:47-73): rows j outer, cols i inner */
    int posx = (int)roundf(refx) + c->pad, posy = (int)roundf(refy) + c->pad;
    int lb = -c->ps / 2, ub = c->ps / 2 - 1, q = 0;
    for (int j = lb; j <= ub; ++j)
        for (int i = lb; i <= ub; ++i, ++q) {
            int idx = (posx + i) + (posy + j) * c->tmp_w;
            gdx[q] = dxp[idx];
            gdy[q] = dyp[idx];
        }
    /* compute_hessian_matrix (src/patch.cpp:75-91) */
    float h[4];
    for (int i = 0; i < c->npts; ++i) second[i] = gdx[i] * gdx[i];
    h[0] = eigen_sum(second, c->npts);
    for (int i = 0; i < c->npts; ++i) second[i] = gdx[i] * gdy[i];
    h[1] = eigen_sum(second, c->npts);
    for (int i = 0; i < c->npts; ++i) second[i] = gdy[i] * gdy[i];
    h[3] = eigen_sum(second, c->npts);
    h[2] = h[1];
    if (h[0] * h[3] - h[2] * h[1] == 0.0f) {   /* Eigen 2x2 determinant, :86 */
        h[0] = (float)((double)h[0] + 1e-10);  /* float += double literal, :88 */
        h[3] = (float)((double)h[3] + 1e-10);  /* :89 */
    }
    /* Paper mode (Kroeger et al. 2016 eq. 3, fixes Q2): the
     * residual is template-subtracted, r = (I1w - mean I1w) - (T - mean T)
     * (means only with normalisation), T = the frame-0 level image on the
     * patch (patch_grad, src/patch.cpp:68, which the reference never uses).
     * Since sum(g*(I1n - Tn)) = sum(g*I1n) - sum(g*Tn), the template part is a
     * per-patch constant: b = sum(g*I1n) - bt with bt = sum(g*Tn), both sums
     * in the Eigen order. This split IS the definition the kernels follow. */
    float bt0 = 0.0f, bt1 = 0.0f;
    if (c->paper) {
        float tn[1024], tmp[1024];
        for (int j = lb, q2 = 0; j <= ub; ++j)
            for (int i = lb; i <= ub; ++i, ++q2) tn[q2] = imgp[(posx + i) + (posy + j) * c->tmp_w];
        if (c->normalization) {
            const float mt = eigen_sum(tn, c->npts) / (float)c->npts;
            for (int i = 0; i < c->npts; ++i) tn[i] = tn[i] - mt;
        }
        for (int i = 0; i < c->npts; ++i) tmp[i] = gdx[i] * tn[i];
        bt0 = eigen_sum(tmp, c->npts);
        for (int i = 0; i < c->npts; ++i) tmp[i] = gdy[i] * tn[i];
        bt1 = eigen_sum(tmp, c->npts);
    }

    /* inverse_search_start (src/patch.cpp:119-154), after reset_patch (:102-116) */
    float inx = initx, iny = inity;
    float u0 = initx, u1 = inity;
    float px = refx + u0, py = refy + u1;      /* :125 */
    float sx = px, sy = py;                    /* :128 */
    if (out_of_bounds(c, px, py)) {            /* :131-138 */
        *ux = u0;
        *uy = u1;
        return;
    }
    patch_second_image(c, img_second, px, py, second);   /* :144 */
    int counter = 0;
    if (counter > c->iterations) { *ux = u0; *uy = u1; return; }   /* :147 */

    /* inverse_search loop (src/patch.cpp:165-202) */
    for (;;) {
        counter++;                                              /* :167 */
        float b0, b1;
        {
            float tmp[1024];
            for (int i = 0; i < c->npts; ++i) tmp[i] = gdx[i] * second[i];
            b0 = eigen_sum(tmp, c->npts);                       /* :171 */
            for (int i = 0; i < c->npts; ++i) tmp[i] = gdy[i] * second[i];
            b1 = eigen_sum(tmp, c->npts);                       /* :172 */
        }
        if (c->paper) {                                         /* template part (paper mode) */
            b0 = b0 - bt0;
            b1 = b1 - bt1;
        }
        float d0, d1;
        eigen_lu_solve2(h, b0, b1, &d0, &d1);                   /* :176 */
        u0 = u0 - d0;                                           /* :179 */
        u1 = u1 - d1;
        px = refx + u0;                                         /* :182 */
        py = refy + u1;
        float ex = sx - px, ey = sy - py;
        float nrm = sqrtf(ex * ex + ey * ey);                   /* .norm(), :185 */
        /* A NaN position (only reachable through a singular 2x2 solve) is UB in
         * the reference (cast of NaN to int at :233); it is reset like an
         * outlier here and in the HIP kernels. */
        if (nrm > c->outlierthresh || out_of_bounds(c, px, py) || nrm != nrm) {
            u0 = inx;                                           /* :190 */
            u1 = iny;
            break;                                              /* converged :192 */
        }
        if (counter > c->iterations) break;                     /* :199-201 */
        patch_second_image(c, img_second, px, py, second);      /* :196 */
    }
    *ux = u0;
    *uy = u1;
}

/* ------------------------------------------------------------------------- */
/* a14: densification (src/patch_grid.cpp:121-182)                           */
/* ------------------------------------------------------------------------- */

static float vr_warp(const float* I1, int stride, int W, int H, float X, float Y);

/* Paper mode (Kroeger et al. 2016 eq. 4, fixes Q6): each
 * covering patch's vote is weighted by 1 / max(1, |I1(x + u) - I0(x)|), with
 * I1 bilinear, replicate border (vr_warp), on the level images; contributions
 * in patch-id order, f = ((f + w*u) ...) / (sum of w). */
static void densify_paper(const level_ctx* c, int npw, int nph, int steps, int offw, int offh,
                          const float* patch_u, const float* I0, const float* I1, int stride, float* dense)
{
    const int W = c->width, H = c->height;
    float* weight = (float*)calloc((size_t)W * H, sizeof(float));
    memset(dense, 0, sizeof(float) * 2 * (size_t)W * H);
    int lb = -c->ps / 2, ub = c->ps / 2 - 1;
    for (int gx = 0; gx < npw; ++gx)
        for (int gy = 0; gy < nph; ++gy) {
            const int ip = gx * nph + gy;
            const int rx = gx * steps + offw, ry = gy * steps + offh;
            const float u0 = patch_u[2 * ip], u1 = patch_u[2 * ip + 1];
            for (int y = lb; y <= ub; ++y)
                for (int x = lb; x <= ub; ++x) {
                    int xt = x + rx, yt = y + ry;
                    if (xt >= 0 && yt >= 0 && xt < W && yt < H) {
                        size_t i = (size_t)yt * W + xt;
                        const float d = vr_warp(I1, stride, W, H, (float)xt + u0, (float)yt + u1) -
                                        I0[(size_t)yt * stride + xt];
                        const float w = 1.0f / fmaxf(1.0f, fabsf(d));
                        weight[i] = weight[i] + w;
                        dense[2 * i] = dense[2 * i] + w * u0;
                        dense[2 * i + 1] = dense[2 * i + 1] + w * u1;
                    }
                }
        }
    for (size_t i = 0; i < (size_t)W * H; ++i)
        if (weight[i] > 0) {
            dense[2 * i] = dense[2 * i] / weight[i];
            dense[2 * i + 1] = dense[2 * i + 1] / weight[i];
        }
    free(weight);
}

static void densify(const level_ctx* c, int npw, int nph, int steps, int offw, int offh,
                    const float* patch_u, float* dense)
{
    const int W = c->width, H = c->height;
    float* weight = (float*)calloc((size_t)W * H, sizeof(float)); /* Q7: zeroed */
    memset(dense, 0, sizeof(float) * 2 * (size_t)W * H);          /* :125 */
    const float half = 0.5f;                                      /* :128 */
    int lb = -c->ps / 2, ub = c->ps / 2 - 1;
    /* row bands [y0, y1): each pixel still receives its patches' terms in
     * patch-id order (a band walks every patch in id order, writing only its
     * own rows), so any band count gives the single-threaded result */
    const int nb = g_threads > 1 ? 4 * g_threads : 1;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(g_threads) if (g_threads > 1)
#endif
    for (int b = 0; b < nb; ++b) {
        const int y0 = (int)((long long)H * b / nb), y1 = (int)((long long)H * (b + 1) / nb);
        for (int gx = 0; gx < npw; ++gx)
            for (int gy = 0; gy < nph; ++gy) {                    /* x-major id order */
                const int ip = gx * nph + gy;
                const int rx = gx * steps + offw, ry = gy * steps + offh;
                if (ry + ub < y0 || ry + lb >= y1) continue;
                const float nu0 = patch_u[2 * ip] * half, nu1 = patch_u[2 * ip + 1] * half;
                for (int y = lb; y <= ub; ++y)
                    for (int x = lb; x <= ub; ++x) {
                        int xt = x + rx, yt = y + ry;
                        if (xt >= 0 && yt >= y0 && xt < W && yt < y1) {
                            size_t i = (size_t)yt * W + xt;
                            weight[i] = weight[i] + half;
                            dense[2 * i] = dense[2 * i] + nu0;
                            dense[2 * i + 1] = dense[2 * i + 1] + nu1;
                        }
                    }
            }
    }
    const long long npx = (long long)W * H;
    DIS_OMP_ROWS
    for (long long i = 0; i < npx; ++i)                            /* :138-149 */
        if (weight[i] > 0) {
            dense[2 * i] = dense[2 * i] / weight[i];
            dense[2 * i + 1] = dense[2 * i + 1] / weight[i];
        }
    free(weight);
}

/* ------------------------------------------------------------------------- */
/* variational refinement (absent from the reference,        */
/* README.md:11 -- PARITY UNPINNED by construction). The DIS paper's          */
/* refinement as OpenCV's VariationalRefinement structures it (Kroeger et al.  */
/* 2016, Sec. 2.3; Brox et al. 2004): minimise                                 */
/*   E = delta*Psi(I_z^2) + gamma*Psi(|grad I_z|^2) + alpha*Psi(|grad u|^2 + |grad v|^2), */
/* Psi(s^2) = sqrt(s^2 + eps^2), linearised around the current flow, lagged    */
/* nonlinearity: each of `fp` iterations re-warps I1 by the current flow,      */
/* linearises, solves for the increment with SOR_ITERS red-black SOR sweeps    */
/* and adds it. Every expression and its order below is the spec the HIP       */
/* kernels (dis_varref.hip) follow bit for bit.                                */
/* ------------------------------------------------------------------------- */

#ifndef VR_ALPHA
#define VR_ALPHA 20.0f
#endif
#ifndef VR_GAMMA
#define VR_GAMMA 10.0f
#endif
#ifndef VR_DELTA
#define VR_DELTA 5.0f
#endif
#define VR_ZETA 0.1f
#define VR_EPS2 1e-6f /* eps = 0.001 */
#define VR_OMEGA 1.6f
#define VR_SOR_ITERS 5

static int clampi_(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

/* replicate border */
static float vr_at(const float* f, int stride, int W, int H, int x, int y)
{
    return f[(size_t)clampi_(y, 0, H - 1) * stride + clampi_(x, 0, W - 1)];
}

/* 5-tap derivative (1, -8, 0, 8, -1) / 12 along (dx, dy), replicate border */
static float vr_d(const float* f, int stride, int W, int H, int x, int y, int dx, int dy)
{
    const float a = vr_at(f, stride, W, H, x - 2 * dx, y - 2 * dy), b = vr_at(f, stride, W, H, x - dx, y - dy);
    const float c = vr_at(f, stride, W, H, x + dx, y + dy), d = vr_at(f, stride, W, H, x + 2 * dx, y + 2 * dy);
    return (((a - 8.0f * b) + 8.0f * c) - d) / 12.0f;
}

/* I1 sampled at (x + u, y + v): bilinear, replicate border. The position is
 * first clamped to [-1, W] x [-1, H] (no effect on the value: beyond it both
 * taps clamp to the same edge pixel; keeps the float->int conversion defined). */
static float vr_warp(const float* I1, int stride, int W, int H, float X, float Y)
{
    X = fminf(fmaxf(X, -1.0f), (float)W);
    Y = fminf(fmaxf(Y, -1.0f), (float)H);
    const float fx0 = floorf(X), fy0 = floorf(Y);
    const int x0 = (int)fx0, y0 = (int)fy0;
    const float fx = X - fx0, fy = Y - fy0;
    const float a = vr_at(I1, stride, W, H, x0, y0), b = vr_at(I1, stride, W, H, x0 + 1, y0);
    const float c = vr_at(I1, stride, W, H, x0, y0 + 1), d = vr_at(I1, stride, W, H, x0 + 1, y0 + 1);
    const float top = (1.0f - fx) * a + fx * b;
    const float bot = (1.0f - fx) * c + fx * d;
    return (1.0f - fy) * top + fy * bot;
}

/* flow: dense W*H*2 (u,v interleaved), refined in place. I0/I1 row stride `stride`. */
void dis_oracle_var_refine(const float* I0, const float* I1, int stride, int W, int H, float* flow, int fp)
{
    const size_t n = (size_t)W * H;
    float* P = (float*)calloc(n * 21, sizeof(float));
    float *I1w = P, *I0x = P + n, *I0y = P + 2 * n, *Wx = P + 3 * n, *Wy = P + 4 * n;
    float *Ix = P + 5 * n, *Iy = P + 6 * n, *Iz = P + 7 * n, *Ixx = P + 8 * n, *Ixy = P + 9 * n, *Iyy = P + 10 * n;
    float *Ixz = P + 11 * n, *Iyz = P + 12 * n, *du = P + 13 * n, *dv = P + 14 * n, *sw = P + 15 * n;
    float *A11 = P + 16 * n, *A12 = P + 17 * n, *A22 = P + 18 * n, *B1 = P + 19 * n, *B2 = P + 20 * n;
    int x, y, it, k, color;
    for (y = 0; y < H; ++y)
        for (x = 0; x < W; ++x) {
            const size_t i = (size_t)y * W + x;
            I0x[i] = vr_d(I0, stride, W, H, x, y, 1, 0);
            I0y[i] = vr_d(I0, stride, W, H, x, y, 0, 1);
        }
    for (it = 0; it < fp; ++it) {
        /* 1. warp I1 by the current flow; derivatives of the pair */
        for (y = 0; y < H; ++y)
            for (x = 0; x < W; ++x) {
                const size_t i = (size_t)y * W + x;
                I1w[i] = vr_warp(I1, stride, W, H, (float)x + flow[2 * i], (float)y + flow[2 * i + 1]);
            }
        for (y = 0; y < H; ++y)
            for (x = 0; x < W; ++x) {
                const size_t i = (size_t)y * W + x;
                Wx[i] = vr_d(I1w, W, W, H, x, y, 1, 0);
                Wy[i] = vr_d(I1w, W, W, H, x, y, 0, 1);
            }
        for (y = 0; y < H; ++y)
            for (x = 0; x < W; ++x) {
                const size_t i = (size_t)y * W + x;
                Ix[i] = 0.5f * (Wx[i] + I0x[i]);
                Iy[i] = 0.5f * (Wy[i] + I0y[i]);
                Iz[i] = I1w[i] - vr_at(I0, stride, W, H, x, y);
                Ixx[i] = 0.5f * (vr_d(Wx, W, W, H, x, y, 1, 0) + vr_d(I0x, W, W, H, x, y, 1, 0));
                Ixy[i] = 0.5f * (vr_d(Wx, W, W, H, x, y, 0, 1) + vr_d(I0x, W, W, H, x, y, 0, 1));
                Iyy[i] = 0.5f * (vr_d(Wy, W, W, H, x, y, 0, 1) + vr_d(I0y, W, W, H, x, y, 0, 1));
                Ixz[i] = Wx[i] - I0x[i];
                Iyz[i] = Wy[i] - I0y[i];
            }
        /* 2. smoothness weight per pixel, alpha * Psi'(|grad u|^2 + |grad v|^2),
         * forward differences (0 at the last column / row) */
        for (y = 0; y < H; ++y)
            for (x = 0; x < W; ++x) {
                const size_t i = (size_t)y * W + x;
                const float uc = flow[2 * i], vc = flow[2 * i + 1];
                float gxu = 0.0f, gxv = 0.0f, gyu = 0.0f, gyv = 0.0f;
                if (x < W - 1) {
                    gxu = flow[2 * (i + 1)] - uc;
                    gxv = flow[2 * (i + 1) + 1] - vc;
                }
                if (y < H - 1) {
                    gyu = flow[2 * (i + W)] - uc;
                    gyv = flow[2 * (i + W) + 1] - vc;
                }
                sw[i] = VR_ALPHA / sqrtf((((gxu * gxu + gyu * gyu) + gxv * gxv) + gyv * gyv) + VR_EPS2);
            }
        /* 3. data weights at the current flow (du = dv = 0: Psi' of the residuals)
         * and the normal equations of the linearised energy in (du, dv) */
        for (y = 0; y < H; ++y)
            for (x = 0; x < W; ++x) {
                const size_t i = (size_t)y * W + x;
                const float psiI = VR_DELTA / sqrtf(Iz[i] * Iz[i] + VR_EPS2);
                const float psiG = VR_GAMMA / sqrtf((Ixz[i] * Ixz[i] + Iyz[i] * Iyz[i]) + VR_EPS2);
                A11[i] = (psiI * (Ix[i] * Ix[i]) + psiG * (Ixx[i] * Ixx[i] + Ixy[i] * Ixy[i])) + VR_ZETA;
                A12[i] = psiI * (Ix[i] * Iy[i]) + psiG * (Ixx[i] * Ixy[i] + Ixy[i] * Iyy[i]);
                A22[i] = (psiI * (Iy[i] * Iy[i]) + psiG * (Ixy[i] * Ixy[i] + Iyy[i] * Iyy[i])) + VR_ZETA;
                {
                    const float wl = x > 0 ? sw[i - 1] : 0.0f, wr = x < W - 1 ? sw[i] : 0.0f;
                    const float wu = y > 0 ? sw[i - W] : 0.0f, wd = y < H - 1 ? sw[i] : 0.0f;
                    const size_t il = x > 0 ? i - 1 : i, ir = x < W - 1 ? i + 1 : i;
                    const size_t iu = y > 0 ? i - W : i, id = y < H - 1 ? i + W : i;
                    const float u = flow[2 * i], v = flow[2 * i + 1];
                    const float su = ((wl * (flow[2 * il] - u) + wr * (flow[2 * ir] - u)) + wu * (flow[2 * iu] - u)) +
                                     wd * (flow[2 * id] - u);
                    const float sv = ((wl * (flow[2 * il + 1] - v) + wr * (flow[2 * ir + 1] - v)) +
                                      wu * (flow[2 * iu + 1] - v)) +
                                     wd * (flow[2 * id + 1] - v);
                    B1[i] = su - (psiI * (Iz[i] * Ix[i]) + psiG * (Ixz[i] * Ixx[i] + Iyz[i] * Ixy[i]));
                    B2[i] = sv - (psiI * (Iz[i] * Iy[i]) + psiG * (Ixz[i] * Ixy[i] + Iyz[i] * Iyy[i]));
                }
                du[i] = 0.0f;
                dv[i] = 0.0f;
            }
        /* 4. red-black SOR on (du, dv): colour 0 = (x + y) even first */
        for (k = 0; k < VR_SOR_ITERS; ++k)
            for (color = 0; color < 2; ++color)
                for (y = 0; y < H; ++y)
                    for (x = (y + color) & 1; x < W; x += 2) {
                        const size_t i = (size_t)y * W + x;
                        const float wl = x > 0 ? sw[i - 1] : 0.0f, wr = x < W - 1 ? sw[i] : 0.0f;
                        const float wu = y > 0 ? sw[i - W] : 0.0f, wd = y < H - 1 ? sw[i] : 0.0f;
                        const size_t il = x > 0 ? i - 1 : i, ir = x < W - 1 ? i + 1 : i;
                        const size_t iu = y > 0 ? i - W : i, id = y < H - 1 ? i + W : i;
                        const float sumw = ((wl + wr) + wu) + wd;
                        const float sdu = ((wl * du[il] + wr * du[ir]) + wu * du[iu]) + wd * du[id];
                        const float nu = (1.0f - VR_OMEGA) * du[i] +
                                         VR_OMEGA * (((B1[i] + sdu) - A12[i] * dv[i]) / (A11[i] + sumw));
                        const float sdv = ((wl * dv[il] + wr * dv[ir]) + wu * dv[iu]) + wd * dv[id];
                        const float nv = (1.0f - VR_OMEGA) * dv[i] +
                                         VR_OMEGA * (((B2[i] + sdv) - A12[i] * nu) / (A22[i] + sumw));
                        du[i] = nu;
                        dv[i] = nv;
                    }
        /* 5. flow += (du, dv) */
        for (size_t i = 0; i < n; ++i) {
            flow[2 * i] = flow[2 * i] + du[i];
            flow[2 * i + 1] = flow[2 * i + 1] + dv[i];
        }
    }
    free(P);
}

/* the refinement energy of a flow (for the energy-decrease checks):
 * sum over pixels of delta*Psi(Iz^2) + gamma*Psi(Ixz^2 + Iyz^2) + alpha*Psi(|grad u|^2 + |grad v|^2)
 * with the warp and derivatives of the flow itself (double accumulation). */
double dis_oracle_var_energy(const float* I0, const float* I1, int stride, int W, int H, const float* flow)
{
    const size_t n = (size_t)W * H;
    float* P = (float*)calloc(n * 5, sizeof(float));
    float *I1w = P, *I0x = P + n, *I0y = P + 2 * n, *Wx = P + 3 * n, *Wy = P + 4 * n;
    double e = 0.0;
    int x, y;
    for (y = 0; y < H; ++y)
        for (x = 0; x < W; ++x) {
            const size_t i = (size_t)y * W + x;
            I1w[i] = vr_warp(I1, stride, W, H, (float)x + flow[2 * i], (float)y + flow[2 * i + 1]);
        }
    for (y = 0; y < H; ++y)
        for (x = 0; x < W; ++x) {
            const size_t i = (size_t)y * W + x;
            I0x[i] = vr_d(I0, stride, W, H, x, y, 1, 0);
            I0y[i] = vr_d(I0, stride, W, H, x, y, 0, 1);
            Wx[i] = vr_d(I1w, W, W, H, x, y, 1, 0);
            Wy[i] = vr_d(I1w, W, W, H, x, y, 0, 1);
        }
    for (y = 0; y < H; ++y)
        for (x = 0; x < W; ++x) {
            const size_t i = (size_t)y * W + x;
            const double iz = (double)I1w[i] - vr_at(I0, stride, W, H, x, y);
            const double gx = (double)Wx[i] - I0x[i], gy = (double)Wy[i] - I0y[i];
            const double ux = x < W - 1 ? (double)flow[2 * (i + 1)] - flow[2 * i] : 0.0;
            const double vx = x < W - 1 ? (double)flow[2 * (i + 1) + 1] - flow[2 * i + 1] : 0.0;
            const double uy = y < H - 1 ? (double)flow[2 * (i + W)] - flow[2 * i] : 0.0;
            const double vy = y < H - 1 ? (double)flow[2 * (i + W) + 1] - flow[2 * i + 1] : 0.0;
            e += VR_DELTA * sqrt(iz * iz + 1e-6) + VR_GAMMA * sqrt(gx * gx + gy * gy + 1e-6) +
                 VR_ALPHA * sqrt(ux * ux + uy * uy + vx * vx + vy * vy + 1e-6);
        }
    free(P);
    return e;
}

int dis_oracle_set_threads(int n)
{
#ifdef _OPENMP
    g_threads = n < 1 ? 1 : n;
#else
    (void)n;
    g_threads = 1;
#endif
    return g_threads;
}

/* ------------------------------------------------------------------------- */
/* a15: scale loop (src/optical_flow.cpp:19-91)                                */
/* ------------------------------------------------------------------------- */

int dis_oracle_flow_from_pyramids(
    float* const* img_first, float* const* img_first_dx, float* const* img_first_dy,
    float* const* img_second, int img_padding, float* outflow,
    int width, int height, int coarsest, int finest, int iterations,
    int patch_size, float patch_overlap, int patch_normalization,
    float* dbg_patch_u, float* dbg_dense)
{
    return dis_oracle_flow_from_pyramids_ex(img_first, img_first_dx, img_first_dy, img_second, img_padding, outflow,
                                            width, height, coarsest, finest, iterations, patch_size, patch_overlap,
                                            patch_normalization, 0, 0, dbg_patch_u, dbg_dense);
}

int dis_oracle_flow_from_pyramids_ex(
    float* const* img_first, float* const* img_first_dx, float* const* img_first_dy,
    float* const* img_second, int img_padding, float* outflow,
    int width, int height, int coarsest, int finest, int iterations,
    int patch_size, float patch_overlap, int patch_normalization, int var_refine_iters, int paper_mode,
    float* dbg_patch_u, float* dbg_dense)
{
    if (patch_size < 2 || (patch_size & 1) || patch_size * patch_size > 1024) return -1;
    if (finest < 0 || coarsest < finest) return -1;
    const int steps = dis_oracle_steps(patch_size, patch_overlap);
    const int nlev = coarsest + 1;
    float** flows = (float**)calloc((size_t)nlev, sizeof(float*));
    float** pus = (float**)calloc((size_t)nlev, sizeof(float*));
    size_t dbg_u_off = 0, dbg_d_off = 0;

    for (int scale = coarsest; scale >= finest; --scale) {       /* :67 */
        level_ctx c;
        c.ps = patch_size;
        c.iterations = iterations;
        c.normalization = patch_normalization;
        c.npts = patch_size * patch_size;
        c.outlierthresh = (float)patch_size / 2;                 /* :34 */
        float sf = powf(2.0f, (float)-scale);                    /* :51 */
        c.height = (int)((float)height * sf);                    /* :52 */
        c.width = (int)((float)width * sf);                      /* :53 */
        c.pad = img_padding;
        c.tmp_lb = -(float)patch_size / 2;                       /* :55 */
        c.tmp_ub_w = (float)(c.width + patch_size / 2 - 2);      /* :56 */
        c.tmp_ub_h = (float)(c.height + patch_size / 2 - 2);     /* :57 */
        c.tmp_w = c.width + 2 * img_padding;                     /* :58 */
        c.paper = paper_mode;

        int npw, nph, offw, offh;
        dis_oracle_grid(c.width, c.height, steps, &npw, &nph, &offw, &offh);
        const int n = npw * nph;
        float* pu = (float*)malloc(sizeof(float) * 2 * (size_t)n);
        float* dense = (scale == finest) ? outflow
                                         : (float*)malloc(sizeof(float) * 2 * (size_t)c.width * c.height);
        /* patches are independent (src/patch_grid.cpp:99-106): the optional
         * threads (dis_oracle_set_threads) change nothing but the wall time */
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 64) num_threads(g_threads) if (g_threads > 1)
#endif
        for (int ip = 0; ip < n; ++ip) {
            float gdx[1025], gdy[1025], second[1024];
            const int gx = ip / nph, gy = ip % nph;          /* ip = gx * nph + gy, src/patch_grid.cpp:39-50 */
            const float rx = (float)(gx * steps + offw), ry = (float)(gy * steps + offh);
            float ix = 0.0f, iy = 0.0f;
            if (scale < coarsest) {                          /* src/patch_grid.cpp:108-119 */
                int x = (int)floorf(rx / 2), y = (int)floorf(ry / 2);
                int i = y * (c.width / 2) + x;
                ix = flows[scale + 1][2 * i] * 2;
                iy = flows[scale + 1][2 * i + 1] * 2;
                }
                patch_search(&c, img_first[scale], img_first_dx[scale], img_first_dy[scale], img_second[scale],
                             rx, ry, ix, iy, gdx, gdy, second, &pu[2 * ip], &pu[2 * ip + 1]);
        }
        if (paper_mode)                                          /* SURVEY 8f row 4 */
            densify_paper(&c, npw, nph, steps, offw, offh, pu,
                          img_first[scale] + (size_t)img_padding * c.tmp_w + img_padding,
                          img_second[scale] + (size_t)img_padding * c.tmp_w + img_padding, c.tmp_w, dense);
        else
            densify(&c, npw, nph, steps, offw, offh, pu, dense); /* :86-90 */
        if (var_refine_iters > 0)                                /* SURVEY 8f row 1 (not in the reference) */
            dis_oracle_var_refine(img_first[scale] + (size_t)img_padding * c.tmp_w + img_padding,
                                  img_second[scale] + (size_t)img_padding * c.tmp_w + img_padding, c.tmp_w,
                                  c.width, c.height, dense, var_refine_iters); /* pixel (0,0) of the padded planes */
        flows[scale] = dense;
        pus[scale] = pu;
    }
    /* debug capture, levels 0..C in order */
    for (int l = 0; l <= coarsest; ++l) {
        const int Wl = (int)((float)width * powf(2.0f, (float)-l));
        const int Hl = (int)((float)height * powf(2.0f, (float)-l));
        int npw, nph, offw, offh;
        dis_oracle_grid(Wl, Hl, steps, &npw, &nph, &offw, &offh);
        if (l >= finest) {
            if (dbg_patch_u) memcpy(dbg_patch_u + dbg_u_off, pus[l], sizeof(float) * 2 * (size_t)npw * nph);
            if (dbg_dense) memcpy(dbg_dense + dbg_d_off, flows[l], sizeof(float) * 2 * (size_t)Wl * Hl);
        }
        dbg_u_off += 2 * (size_t)npw * nph;
        dbg_d_off += 2 * (size_t)Wl * Hl;
    }
    for (int l = finest; l <= coarsest; ++l) {
        free(pus[l]);
        if (l != finest) free(flows[l]);
    }
    free(flows);
    free(pus);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* a16: upsample + crop (src/main.cpp:191-198)                                 */
/* ------------------------------------------------------------------------- */

/* cv::resize(..., fx = fy = 2^F, INTER_LINEAR) coefficient table for one
 * axis: s = (float)((d + 0.5) * (1/2^F) - 0.5) in double; i = floor(s);
 * f = s - i; clamp i < 0 -> (0, 0) and i >= n-1 -> (n-1, 0). `full` marks the
 * taps (d < xmax) evaluated as S[i]*(1-f) + S[i+1]*f. */
static void linear_coeffs(int n_src, int n_dst, double scale, int* idx, float* f, int* two_tap)
{
    int xmax = n_dst;
    for (int d = 0; d < n_dst; ++d) {
        float fx = (float)((d + 0.5) * scale - 0.5);
        int sx = (int)floorf(fx);
        fx -= (float)sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx + 1 >= n_src) {
            if (d < xmax) xmax = d;
            if (sx >= n_src - 1) { fx = 0; sx = n_src - 1; }
        }
        idx[d] = sx;
        f[d] = fx;
    }
    for (int d = 0; d < n_dst; ++d) two_tap[d] = d < xmax;
}

void dis_oracle_upsample_crop(const float* flowF, int Wp, int Hp, int finest,
                              int pad_left, int pad_top, int W, int H, float* out)
{
    const int wF = Wp >> finest, hF = Hp >> finest;
    if (finest == 0) {
        for (int y = 0; y < H; ++y)
            memcpy(out + (size_t)y * W * 2, flowF + ((size_t)(y + pad_top) * wF + pad_left) * 2,
                   sizeof(float) * 2 * (size_t)W);
        return;
    }
    const float sc = powf(2.0f, (float)finest);                 /* :181 */
    int* xi = (int*)malloc(sizeof(int) * Wp);
    int* xt = (int*)malloc(sizeof(int) * Wp);
    float* xf = (float*)malloc(sizeof(float) * Wp);
    int* yi = (int*)malloc(sizeof(int) * Hp);
    int* yt = (int*)malloc(sizeof(int) * Hp);
    float* yf = (float*)malloc(sizeof(float) * Hp);
    linear_coeffs(wF, Wp, 1.0 / (double)sc, xi, xf, xt);
    linear_coeffs(hF, Hp, 1.0 / (double)sc, yi, yf, yt);
    /* flowout *= sc_fct (:194) */
    float* s = (float*)malloc(sizeof(float) * 2 * (size_t)wF * hF);
    for (size_t i = 0; i < 2 * (size_t)wF * hF; ++i) s[i] = flowF[i] * sc;
    /* horizontal pass per source row (HResizeLinear), then vertical
     * (VResizeLinear: S0*b0 + S1*b1, row sy+1 clamped) (:195) */
    float* hrow = (float*)malloc(sizeof(float) * 2 * (size_t)Wp * hF);
    DIS_OMP_ROWS
    for (int r = 0; r < hF; ++r)
        for (int x = 0; x < Wp; ++x)
            for (int ch = 0; ch < 2; ++ch) {
                const float* S = s + (size_t)r * wF * 2;
                float v;
                if (xt[x]) v = S[xi[x] * 2 + ch] * (1.f - xf[x]) + S[(xi[x] + 1) * 2 + ch] * xf[x];
                else v = S[xi[x] * 2 + ch];
                hrow[((size_t)r * Wp + x) * 2 + ch] = v;
            }
    DIS_OMP_ROWS
    for (int y = 0; y < H; ++y) {
        const int yy = y + pad_top;
        const int r0 = yi[yy], r1 = (yi[yy] + 1 < hF) ? yi[yy] + 1 : hF - 1;
        const float b1 = yf[yy], b0 = 1.f - yf[yy];
        for (int x = 0; x < W; ++x)
            for (int ch = 0; ch < 2; ++ch) {
                const int xx = x + pad_left;
                float v = hrow[((size_t)r0 * Wp + xx) * 2 + ch] * b0 + hrow[((size_t)r1 * Wp + xx) * 2 + ch] * b1;
                out[((size_t)y * W + x) * 2 + ch] = v;
            }
    }
    free(xi); free(xt); free(xf); free(yi); free(yt); free(yf); free(s); free(hrow);
}

/* ------------------------------------------------------------------------- */
/* whole path (src/main.cpp:135-198)                                           */
/* ------------------------------------------------------------------------- */

static void pad_plane(const float* src, int W, int H, int pad, int replicate, float* dst)
{
    /* copyMakeBorder (src/main.cpp:43-47): replicate for the image, zero for
     * the gradients. */
    const int tw = W + 2 * pad, th = H + 2 * pad;
    DIS_OMP_ROWS
    for (int y = 0; y < th; ++y)
        for (int x = 0; x < tw; ++x) {
            int sx = x - pad, sy = y - pad;
            float v;
            if (replicate) v = src[(size_t)clampi(sy, 0, H - 1) * W + clampi(sx, 0, W - 1)];
            else v = (sx >= 0 && sy >= 0 && sx < W && sy < H) ? src[(size_t)sy * W + sx] : 0.0f;
            dst[(size_t)y * tw + x] = v;
        }
}

int dis_oracle_calc_u8(const dis_oracle_params* p, int W, int H,
                       const uint8_t* I0, const uint8_t* I1, size_t stride,
                       float* flow_out)
{
    const int C = p->coarsest_scale, F = p->finest_scale, ps = p->patch_size;
    if (C < 0 || F < 0 || F > C || ps < 2 || (ps & 1)) return -1;
    int Wp, Hp, pl, pt;
    dis_oracle_padded_size(W, H, C, &Wp, &Hp, &pl, &pt);
    size_t tot = 0;
    for (int l = 0; l <= C; ++l) tot += (size_t)(Wp >> l) * (Hp >> l);
    float* f0 = (float*)malloc(sizeof(float) * (size_t)Wp * Hp);
    float* f1 = (float*)malloc(sizeof(float) * (size_t)Wp * Hp);
    dis_oracle_pad_convert(I0, stride, W, H, C, f0);
    dis_oracle_pad_convert(I1, stride, W, H, C, f1);
    float* img0 = (float*)malloc(sizeof(float) * tot);
    float* dx0 = (float*)malloc(sizeof(float) * tot);
    float* dy0 = (float*)malloc(sizeof(float) * tot);
    float* img1 = (float*)malloc(sizeof(float) * tot);
    dis_oracle_pyramid(f0, Wp, Hp, C, img0, dx0, dy0);
    dis_oracle_pyramid(f1, Wp, Hp, C, img1, NULL, NULL);   /* frame-2 dx/dy never read (Q15) */

    float* P0[32]; float* PX[32]; float* PY[32]; float* P1[32];
    size_t off = 0;
    for (int l = 0; l <= C; ++l) {
        const int w = Wp >> l, h = Hp >> l;
        const size_t psz = (size_t)(w + 2 * ps) * (h + 2 * ps);
        P0[l] = (float*)malloc(sizeof(float) * psz);
        PX[l] = (float*)malloc(sizeof(float) * psz);
        PY[l] = (float*)malloc(sizeof(float) * psz);
        P1[l] = (float*)malloc(sizeof(float) * psz);
        pad_plane(img0 + off, w, h, ps, 1, P0[l]);
        pad_plane(dx0 + off, w, h, ps, 0, PX[l]);
        pad_plane(dy0 + off, w, h, ps, 0, PY[l]);
        pad_plane(img1 + off, w, h, ps, 1, P1[l]);
        /* the reference passes pointers at the padded origin (src/main.cpp:44-48) */
        off += (size_t)w * h;
    }
    float* flowF = (float*)malloc(sizeof(float) * 2 * (size_t)(Wp >> F) * (Hp >> F));
    int rc = dis_oracle_flow_from_pyramids_ex(P0, PX, PY, P1, ps, flowF, Wp, Hp, C, F,
                                           p->iterations, ps, p->patch_overlap,
                                           p->patch_normalization, p->var_refine_iters, p->paper_mode,
                                           NULL, NULL);
    if (rc == 0) dis_oracle_upsample_crop(flowF, Wp, Hp, F, pl, pt, W, H, flow_out);
    for (int l = 0; l <= C; ++l) { free(P0[l]); free(PX[l]); free(PY[l]); free(P1[l]); }
    free(flowF); free(f0); free(f1); free(img0); free(dx0); free(dy0); free(img1);
    return rc;
}

/* ---- colour coding (src/color_coding.cpp) ---------------- */

/* is_flow_correct, src/color_coding.cpp:8-11 */
static int flow_ok(float x, float y)
{
    return !(x != x) && !(y != y) && fabsf(x) < 1e9f && fabsf(y) < 1e9f;
}

/* atan2f (src/color_coding.cpp:52) restated as a fixed float algorithm (the
 * product kernel evaluates the identical one): t = min/max in [0, 1],
 * atan(t) = t + t z P(z), z = t^2, with the minimax coefficients of ARM's
 * optimized-routines atanf (<= 3 ulp), then the octant fix-up. */
static float atan2_dis(float y, float x)
{
    const float ax = fabsf(x), ay = fabsf(y);
    const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
    const float t = mx > 0.0f ? mn / mx : 0.0f;
    const float z = t * t;
    float p = 0x1.01fd88p-8f;
    float r;
    p = p * z + -0x1.4c3c60p-6f;
    p = p * z + 0x1.93a2c0p-5f;
    p = p * z + -0x1.491f0ep-4f;
    p = p * z + 0x1.bd7368p-4f;
    p = p * z + -0x1.24051ep-3f;
    p = p * z + 0x1.99935ep-3f;
    p = p * z + -0x1.55555p-2f;
    r = t + (t * z) * p;
    if (ay > ax) r = 1.57079637f - r;
    if (x < 0.0f || (x == 0.0f && signbit(x))) r = 3.14159274f - r;
    return signbit(y) ? -r : r;
}

/* compute_color, src/color_coding.cpp:13-79: colour wheel (:31-56, integer
 * division), angle, linear interpolation between wheel entries, saturation
 * by radius, BGR store with truncation (:76). */
static void compute_color(float fx, float fy, uint8_t* pix)
{
    enum { RY = 15, YG = 6, GC = 4, CB = 11, BM = 13, MR = 6, NCOLS = RY + YG + GC + CB + BM + MR };
    int wheel[NCOLS][3];
    int k = 0, i, b;
    for (i = 0; i < RY; ++i, ++k) { wheel[k][0] = 255; wheel[k][1] = 255 * i / RY; wheel[k][2] = 0; }
    for (i = 0; i < YG; ++i, ++k) { wheel[k][0] = 255 - 255 * i / YG; wheel[k][1] = 255; wheel[k][2] = 0; }
    for (i = 0; i < GC; ++i, ++k) { wheel[k][0] = 0; wheel[k][1] = 255; wheel[k][2] = 255 * i / GC; }
    for (i = 0; i < CB; ++i, ++k) { wheel[k][0] = 0; wheel[k][1] = 255 - 255 * i / CB; wheel[k][2] = 255; }
    for (i = 0; i < BM; ++i, ++k) { wheel[k][0] = 255 * i / BM; wheel[k][1] = 0; wheel[k][2] = 255; }
    for (i = 0; i < MR; ++i, ++k) { wheel[k][0] = 255; wheel[k][1] = 0; wheel[k][2] = 255 - 255 * i / MR; }
    {
        const float rad = sqrtf(fx * fx + fy * fy);
        const float a = atan2_dis(-fy, -fx) / 3.14159274f; /* / (float)CV_PI */
        const float fk = (a + 1.0f) / 2.0f * (float)(NCOLS - 1);
        const int k0 = (int)fk;
        const int k1 = (k0 + 1) % NCOLS;
        const float f = fk - (float)k0;
        for (b = 0; b < 3; b++) {
            const float col0 = (float)wheel[k0][b] / 255.f;
            const float col1 = (float)wheel[k1][b] / 255.f;
            float col = (1 - f) * col0 + f * col1;
            if (rad <= 1)
                col = 1 - rad * (1 - col);
            else
                col *= .75f;
            pix[2 - b] = (uint8_t)(255.f * col);
        }
    }
}

/* draw_optical_flow, src/color_coding.cpp:81-117 */
void dis_oracle_flow_color(const float* flow, int W, int H, float maxmotion, uint8_t* bgr)
{
    float maxrad = maxmotion;
    long long i, n = (long long)W * H;
    memset(bgr, 0, (size_t)n * 3);
    if (maxmotion <= 0) {
        maxrad = 1;
        for (i = 0; i < n; ++i) {
            const float x = flow[2 * i], y = flow[2 * i + 1];
            if (!flow_ok(x, y)) continue;
            {
                const float r = sqrtf(x * x + y * y);
                maxrad = maxrad > r ? maxrad : r;
            }
        }
    }
    for (i = 0; i < n; ++i) {
        const float x = flow[2 * i], y = flow[2 * i + 1];
        if (flow_ok(x, y)) compute_color(x / maxrad, y / maxrad, bgr + 3 * i);
    }
}
