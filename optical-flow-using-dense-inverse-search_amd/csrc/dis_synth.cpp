// dis_synth.cpp -- deterministic synthetic frame pairs.
//
// Not on the hot path: host-side generator used by bench.py and the tests.
// I0 = multi-octave value noise (periods 4..64 px, smoothstep-interpolated
// lattice values from a splitmix64 hash of (seed, octave, ix, iy)), scaled to
// mean 128 and clamped to u8; the noise has texture at every pyramid level
// after the Sobel magnitude of Q1. I1(x) = I0(x - f(x)) evaluated on the
// continuous noise field, with f = (a + b sin(2 pi y/H + phi),
// c + d cos(2 pi x/W + psi)), a..d in U(-3,3): the flow I0 -> I1 is ~f.
#include <cmath>
#include <cstdint>
#include <vector>

#include "dis_abi.h"

namespace {

inline uint64_t splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

inline double unit(uint64_t h) { return (double)(h >> 11) * (1.0 / 9007199254740992.0); }  // [0,1)

struct Octave {
    int period, x0, y0, nx, ny;
    double amp;
    std::vector<float> lat;  // lattice values in [-1,1)
};

inline double smooth(double t) { return t * t * (3.0 - 2.0 * t); }

struct Noise {
    std::vector<Octave> oct;
    Noise(uint64_t seed, int W, int H)
    {
        static const int periods[5] = {4, 8, 16, 32, 64};
        static const double amps[5] = {1.0, 0.7, 0.5, 0.35, 0.25};
        for (int o = 0; o < 5; ++o) {
            Octave q;
            q.period = periods[o];
            q.amp = amps[o];
            const int margin = 16;  // flow stays within +-6 px
            q.x0 = (int)std::floor((double)-margin / q.period) - 1;
            q.y0 = (int)std::floor((double)-margin / q.period) - 1;
            q.nx = (W + 2 * margin) / q.period + 4;
            q.ny = (H + 2 * margin) / q.period + 4;
            q.lat.resize((size_t)q.nx * q.ny);
            for (int j = 0; j < q.ny; ++j)
                for (int i = 0; i < q.nx; ++i) {
                    uint64_t h = splitmix64(seed * 0x100000001B3ULL ^ splitmix64((uint64_t)o * 0x9E37ULL +
                                                                                  (uint64_t)(i + q.x0) * 0x51ED27ULL +
                                                                                  (uint64_t)(j + q.y0) * 0x3C6EF372FE94F82BULL));
                    q.lat[(size_t)j * q.nx + i] = (float)(2.0 * unit(h) - 1.0);
                }
            oct.push_back(std::move(q));
        }
    }
    double operator()(double x, double y) const
    {
        double s = 0.0;
        for (const Octave& q : oct) {
            const double fx = x / q.period, fy = y / q.period;
            const double ix = std::floor(fx), iy = std::floor(fy);
            const double tx = smooth(fx - ix), ty = smooth(fy - iy);
            int i = (int)ix - q.x0, j = (int)iy - q.y0;
            if (i < 0) i = 0;
            if (j < 0) j = 0;
            if (i > q.nx - 2) i = q.nx - 2;
            if (j > q.ny - 2) j = q.ny - 2;
            const float* r0 = &q.lat[(size_t)j * q.nx + i];
            const float* r1 = r0 + q.nx;
            const double a = r0[0] + (r0[1] - r0[0]) * tx;
            const double b = r1[0] + (r1[1] - r1[0]) * tx;
            s += q.amp * (a + (b - a) * ty);
        }
        return s;
    }
};

inline uint8_t to_u8(double v)
{
    double g = 128.0 + 70.0 * v;  // std ~ 45 for this octave mix
    g = std::floor(g + 0.5);
    return (uint8_t)(g < 0 ? 0 : (g > 255 ? 255 : g));
}

}  // namespace

extern "C" dis_status dis_synth_pair(uint64_t seed, int W, int H, uint8_t* I0, uint8_t* I1, float* gt)
{
    if (W < 1 || H < 1 || !I0 || !I1) return DIS_ERR_INVALID_ARGUMENT;
    Noise nz(seed, W, H);
    const uint64_t hs = splitmix64(seed ^ 0xD1B54A32D192ED03ULL);
    const double a = 6.0 * unit(splitmix64(hs + 1)) - 3.0, b = 6.0 * unit(splitmix64(hs + 2)) - 3.0;
    const double c = 6.0 * unit(splitmix64(hs + 3)) - 3.0, d = 6.0 * unit(splitmix64(hs + 4)) - 3.0;
    const double phi = 6.283185307179586 * unit(splitmix64(hs + 5));
    const double psi = 6.283185307179586 * unit(splitmix64(hs + 6));
    std::vector<double> cu(H), cv(W);
    for (int y = 0; y < H; ++y) cu[y] = a + b * std::sin(6.283185307179586 * y / H + phi);
    for (int x = 0; x < W; ++x) cv[x] = c + d * std::cos(6.283185307179586 * x / W + psi);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const size_t i = (size_t)y * W + x;
            const double u = cu[y], v = cv[x];
            I0[i] = to_u8(nz(x, y));
            I1[i] = to_u8(nz(x - u, y - v));
            if (gt) {
                gt[2 * i] = (float)u;
                gt[2 * i + 1] = (float)v;
            }
        }
    return DIS_OK;
}
