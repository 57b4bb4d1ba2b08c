# r06 experiment (not kept): I0's second derivatives precomputed once per level
# (k_vr_d1) so k_vr_lin stages no I0x / I0y halo in LDS. Run in the package directory of a /tmp
# copy of the tree, then build there (make ROOT=... BUILD=... LIB=...); argument w5: 5 waves per SIMD.
import sys
p = "csrc/dis_kernels.h"; s = open(p).read()
old = "constexpr int kVarRefPlanes = 8;"; assert old in s
s = s.replace(old, "constexpr int kVarRefPlanes = 11;"); open(p, "w").write(s)
p = "csrc/dis_varref.hip"; s = open(p).read()
old = "enum Plane { P_I0X, P_I0Y, P_B1, P_B2, P_A12, P_D1, P_D2, P_SW };\nstatic_assert(P_SW + 1 == kVarRefPlanes, \"workspace planes\");"
assert old in s
s = s.replace(old, "enum Plane { P_I0X, P_I0Y, P_B1, P_B2, P_A12, P_D1, P_D2, P_SW, P_I0XX, P_I0XY, P_I0YY };\nstatic_assert(P_I0YY + 1 == kVarRefPlanes, \"workspace planes\");")
old = """// ---------------------------------------------------------------------------
// linearisation"""
assert old in s
s = s.replace(old, """// the second derivatives of I0 that k_vr_lin's Ixx, Ixy, Iyy take (the 5-tap
// derivative of I0x along x and y, of I0y along y, replicate border), once per
// level: the same expressions on the same values as the linearisation
// evaluated from its staged I0x / I0y, so the same bits
__global__ void __launch_bounds__(256) k_vr_d1(Lvl L)
{
    const int x = blockIdx.x * 64 + (threadIdx.x & 63), y = blockIdx.y * 4 + (threadIdx.x >> 6), pr = blockIdx.z;
    if (x >= L.W || y >= L.H) return;
    const int W = L.W, H = L.H;
    const float* gx = plane(L, pr, P_I0X);
    const float* gy = plane(L, pr, P_I0Y);
    const float* r = gx + (size_t)y * W;
    const size_t i = (size_t)y * W + x;
    const size_t ym2 = (size_t)clampi_(y - 2, 0, H - 1) * W + x, ym1 = (size_t)clampi_(y - 1, 0, H - 1) * W + x;
    const size_t yp1 = (size_t)clampi_(y + 1, 0, H - 1) * W + x, yp2 = (size_t)clampi_(y + 2, 0, H - 1) * W + x;
    plane(L, pr, P_I0XX)[i] = d5(r[clampi_(x - 2, 0, W - 1)], r[clampi_(x - 1, 0, W - 1)], r[clampi_(x + 1, 0, W - 1)],
                                 r[clampi_(x + 2, 0, W - 1)]);
    plane(L, pr, P_I0XY)[i] = d5(gx[ym2], gx[ym1], gx[yp1], gx[yp2]);
    plane(L, pr, P_I0YY)[i] = d5(gy[ym2], gy[ym1], gy[yp1], gy[yp2]);
}

// ---------------------------------------------------------------------------
// linearisation""", 1)
old = "    __shared__ float sWx[kGH][kGW], sWy[kGH][kGW], sGx[kGH][kGW], sGy[kGH][kGW];"
assert old in s
s = s.replace(old, "    __shared__ float sWx[kGH][kGW], sWy[kGH][kGW];")
old = """    float2 f[NF];
    float gx0[NG], gy0[NG], i0p[NP];"""
assert old in s
s = s.replace(old, """    float2 f[NF];
    float i0p[NP];""")
old = """#pragma unroll
    for (int t = 0; t < NG; ++t) {
        const int k = min(tid + 256 * t, kGW * kGH - 1);
        const int ly = k / kGW, lx = k - ly * kGW;
        const size_t i = (size_t)clampi_(y0 - 2 + ly, 0, H - 1) * W + clampi_(x0 - 2 + lx, 0, W - 1);
        gx0[t] = plane(L, pr, P_I0X)[i];
        gy0[t] = plane(L, pr, P_I0Y)[i];
    }
"""
assert old in s
s = s.replace(old, "")
old = """    // 2. I0x, I0y over the tile +-2
#pragma unroll
    for (int t = 0; t < NG; ++t) {
        const int k = tid + 256 * t;
        if (k >= kGW * kGH) break;
        const int ly = k / kGW, lx = k - ly * kGW;
        sGx[ly][lx] = gx0[t];
        sGy[ly][lx] = gy0[t];
    }
    __syncthreads();"""
assert old in s
s = s.replace(old, """    __syncthreads();
    // 2. I0's first and second derivatives at the thread's pixels (k_vr_d0 / d1),
    //    in flight during step 3
    float pgx[NP], pgy[NP], pxx[NP], pxy[NP], pyy[NP];
#pragma unroll
    for (int t = 0; t < NP; ++t) {
        const int k = tid + 256 * t;
        const int ly = k / kLW, lx = k - ly * kLW;
        const size_t i = (size_t)min(y0 + ly, H - 1) * W + min(x0 + lx, W - 1);
        pgx[t] = plane(L, pr, P_I0X)[i];
        pgy[t] = plane(L, pr, P_I0Y)[i];
        pxx[t] = plane(L, pr, P_I0XX)[i];
        pxy[t] = plane(L, pr, P_I0XY)[i];
        pyy[t] = plane(L, pr, P_I0YY)[i];
    }""")
old = """        const float wx = sWx[gy][gx], wy = sWy[gy][gx], i0x = sGx[gy][gx], i0y = sGy[gy][gx];"""
assert old in s
s = s.replace(old, """        const float wx = sWx[gy][gx], wy = sWy[gy][gx], i0x = pgx[t], i0y = pgy[t];""")
old = """        const float Ixx = 0.5f * (d5(sWx[gy][gx - 2], sWx[gy][gx - 1], sWx[gy][gx + 1], sWx[gy][gx + 2]) +
                                  d5(sGx[gy][gx - 2], sGx[gy][gx - 1], sGx[gy][gx + 1], sGx[gy][gx + 2]));
        const float Ixy = 0.5f * (d5(sWx[gy - 2][gx], sWx[gy - 1][gx], sWx[gy + 1][gx], sWx[gy + 2][gx]) +
                                  d5(sGx[gy - 2][gx], sGx[gy - 1][gx], sGx[gy + 1][gx], sGx[gy + 2][gx]));
        const float Iyy = 0.5f * (d5(sWy[gy - 2][gx], sWy[gy - 1][gx], sWy[gy + 1][gx], sWy[gy + 2][gx]) +
                                  d5(sGy[gy - 2][gx], sGy[gy - 1][gx], sGy[gy + 1][gx], sGy[gy + 2][gx]));"""
assert old in s
s = s.replace(old, """        const float Ixx = 0.5f * (d5(sWx[gy][gx - 2], sWx[gy][gx - 1], sWx[gy][gx + 1], sWx[gy][gx + 2]) + pxx[t]);
        const float Ixy = 0.5f * (d5(sWx[gy - 2][gx], sWx[gy - 1][gx], sWx[gy + 1][gx], sWx[gy + 2][gx]) + pxy[t]);
        const float Iyy = 0.5f * (d5(sWy[gy - 2][gx], sWy[gy - 1][gx], sWy[gy + 1][gx], sWy[gy + 2][gx]) + pyy[t]);""")
old = "    constexpr int NF = (kFW * kFH + 255) / 256, NG = (kGW * kGH + 255) / 256, NP = kLW * kLH / 256;"
assert old in s
s = s.replace(old, "    constexpr int NF = (kFW * kFH + 255) / 256, NP = kLW * kLH / 256;")
old = """    hipLaunchKernelGGL(k_vr_d0, dim3((a.W + 63) / 64, (a.H + 3) / 4, nn), dim3(256), 0, s, L);"""
assert old in s
s = s.replace(old, old + """
    hipLaunchKernelGGL(k_vr_d1, dim3((a.W + 63) / 64, (a.H + 3) / 4, nn), dim3(256), 0, s, L);""")
if len(sys.argv) > 1 and sys.argv[1] == "w5":
    old = "__global__ void __launch_bounds__(256) k_vr_lin(Lvl L)"
    assert old in s
    s = s.replace(old, "__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) k_vr_lin(Lvl L)")
open(p, "w").write(s)
