// C++ test of the host facade (include/dis/dis.hpp) -- the way a user of the
// reference would call the engine -- checked bit-exactly against the CPU
// oracle (test infrastructure, oracle/dis_oracle.h). Run on a GPU box by
// tests/test_cpp_facade.py; exits non-zero on any failure.
#include <cstdio>
#include <cmath>
#include <cstring>
#include <vector>

#include "dis/dis.hpp"
#include "dis_oracle.h"

static int failures = 0;
#define EXPECT(cond, msg)                                        \
    do {                                                         \
        if (!(cond)) {                                           \
            std::printf("FAIL: %s (%s:%d)\n", msg, __FILE__, __LINE__); \
            ++failures;                                          \
        }                                                        \
    } while (0)

static bool bitexact(const std::vector<float>& a, const std::vector<float>& b)
{
    return a.size() == b.size() && std::memcmp(a.data(), b.data(), a.size() * sizeof(float)) == 0;
}

// copyMakeBorder(replicate | zero) of one plane (src/main.cpp:43-47)
static std::vector<float> pad(const float* p, int w, int h, int pd, bool replicate)
{
    std::vector<float> o((size_t)(w + 2 * pd) * (h + 2 * pd));
    for (int y = -pd; y < h + pd; ++y)
        for (int x = -pd; x < w + pd; ++x) {
            float v;
            if (replicate) {
                const int xx = x < 0 ? 0 : (x >= w ? w - 1 : x), yy = y < 0 ? 0 : (y >= h ? h - 1 : y);
                v = p[(size_t)yy * w + xx];
            } else {
                v = (x >= 0 && y >= 0 && x < w && y < h) ? p[(size_t)y * w + x] : 0.0f;
            }
            o[(size_t)(y + pd) * (w + 2 * pd) + x + pd] = v;
        }
    return o;
}

int main()
{
    const int W = 200, H = 150;
    std::vector<uint8_t> I0((size_t)W * H), I1((size_t)W * H);
    dis::check(dis_synth_pair(7, W, H, I0.data(), I1.data(), nullptr));

    // 1) calc(I0, I1, flow) with a preset
    {
        dis::DenseInverseSearch eng(dis::Preset::MEDIUM, W, H);
        std::vector<float> flow = eng.calc(I0, I1);
        const dis_params& p = eng.params();
        dis_oracle_params op{p.coarsest_scale, p.finest_scale, p.patch_size, p.iterations, p.patch_overlap,
                             p.patch_normalization};
        std::vector<float> ref(flow.size());
        EXPECT(dis_oracle_calc_u8(&op, W, H, I0.data(), I1.data(), W, ref.data()) == 0, "oracle ran");
        EXPECT(bitexact(flow, ref), "DenseInverseSearch::calc bit-exact vs oracle");
        eng.set_graphs(false);  // eager enqueue: the same bits
        EXPECT(bitexact(eng.calc(I0, I1), ref), "eager calc bit-exact vs oracle");
        eng.set_graphs(true);
        eng.set_precision(DIS_PRECISION_FMA);  // tolerance mode: close, not bit-exact
        std::vector<float> fma = eng.calc(I0, I1);
        double se = 0.0;
        for (size_t i = 0; i < fma.size(); i += 2)
            se += std::sqrt((double)(fma[i] - ref[i]) * (fma[i] - ref[i]) +
                            (double)(fma[i + 1] - ref[i + 1]) * (fma[i + 1] - ref[i + 1]));
        EXPECT(se / (fma.size() / 2) < 1e-2, "FMA mode within a loose mean-EPE bound of the oracle");
        eng.set_precision(DIS_PRECISION_EXACT);
        EXPECT(bitexact(eng.calc(I0, I1), ref), "back to exact");
    }

    // 2) OpticalFlow::OpticalFlowClass over padded pyramids, as src/main.cpp:139-189 builds them
    {
        const int C = 3, F = 1, ps = 8, it = 10;
        const float ov = 0.7f;
        int Wp, Hp, pl, pt;
        dis_oracle_padded_size(W, H, C, &Wp, &Hp, &pl, &pt);
        std::vector<float> f0((size_t)Wp * Hp), f1((size_t)Wp * Hp);
        dis_oracle_pad_convert(I0.data(), W, W, H, C, f0.data());
        dis_oracle_pad_convert(I1.data(), W, W, H, C, f1.data());
        size_t tot = 0;
        for (int l = 0; l <= C; ++l) tot += (size_t)(Wp >> l) * (Hp >> l);
        std::vector<float> l0(tot), dx0(tot), dy0(tot), l1(tot), dx1(tot), dy1(tot);
        dis_oracle_pyramid(f0.data(), Wp, Hp, C, l0.data(), dx0.data(), dy0.data());
        dis_oracle_pyramid(f1.data(), Wp, Hp, C, l1.data(), dx1.data(), dy1.data());
        std::vector<std::vector<float>> P[6];
        float* ptr[6][8];
        size_t off = 0;
        for (int l = 0; l <= C; ++l) {
            const int w = Wp >> l, h = Hp >> l;
            P[0].push_back(pad(&l0[off], w, h, ps, true));
            P[1].push_back(pad(&dx0[off], w, h, ps, false));
            P[2].push_back(pad(&dy0[off], w, h, ps, false));
            P[3].push_back(pad(&l1[off], w, h, ps, true));
            P[4].push_back(pad(&dx1[off], w, h, ps, false));
            P[5].push_back(pad(&dy1[off], w, h, ps, false));
            off += (size_t)w * h;
        }
        for (int k = 0; k < 6; ++k)
            for (int l = 0; l <= C; ++l) ptr[k][l] = P[k][l].data();
        std::vector<float> out((size_t)(Wp >> F) * (Hp >> F) * 2), ref(out.size());
        OpticalFlow::OpticalFlowClass ofc(ptr[0], ptr[1], ptr[2], ptr[3], ptr[4], ptr[5], ps, out.data(), Wp, Hp, C,
                                          F, it, ps, ov, true, false);
        EXPECT(dis_oracle_flow_from_pyramids(ptr[0], ptr[1], ptr[2], ptr[3], ps, ref.data(), Wp, Hp, C, F, it, ps,
                                             ov, 1, nullptr, nullptr) == 0,
               "oracle compat ran");
        EXPECT(bitexact(out, ref), "OpticalFlowClass bit-exact vs oracle");
        bool threw = false;
        try {
            OpticalFlow::OpticalFlowClass bad(ptr[0], ptr[1], ptr[2], ptr[3], ptr[4], ptr[5], ps, out.data(), Wp, Hp,
                                              C, F, it, 7, ov, true, false);
        } catch (const dis::Error& e) {
            threw = e.status() == DIS_ERR_INVALID_ARGUMENT;
        }
        EXPECT(threw, "odd patch size rejected");
        threw = false;
        try {
            OpticalFlow::OpticalFlowClass gui(ptr[0], ptr[1], ptr[2], ptr[3], ptr[4], ptr[5], ps, out.data(), Wp, Hp,
                                              C, F, it, ps, ov, true, true);
        } catch (const dis::Error& e) {
            threw = e.status() == DIS_ERR_UNSUPPORTED;
        }
        EXPECT(threw, "draw_grid rejected");
    }
    std::printf("%s: %d failure(s)\n", failures ? "FAILED" : "OK", failures);
    return failures ? 1 : 0;
}
