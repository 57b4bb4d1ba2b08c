// Pyramid phase probe (experiment, not part of the product): builds
// k_pyramid<6> with DIS_PYR_PROF, runs the 1080p batch-32 launch, and prints
// per-workgroup phase durations (wave 0's shader clocks) and the number of
// workgroups resident per CU over time (wall clock).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -DDIS_PYR_PROF -I include \
//     -I optical-flow-using-dense-inverse-search_amd/csrc tools/pyr_probe.hip -o tools/pyr_probe
#include "../optical-flow-using-dense-inverse-search_amd/csrc/dis_frontback.hip"

#include <algorithm>
#include <cstdio>
#include <map>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                \
        }                                                                            \
    } while (0)

int main(int argc, char** argv)
{
    const int W = 1920, H = 1080, B = argc > 1 ? atoi(argv[1]) : 32, L = 6;
    const int Wp = 1920, Hp = 1088;
    dis::PyramidArgs a{};
    size_t fsz = (size_t)W * H;
    uint8_t *i0, *i1;
    CK(hipMalloc(&i0, fsz * B));
    CK(hipMalloc(&i1, fsz * B));
    std::vector<uint8_t> h(fsz * B);
    for (size_t k = 0; k < h.size(); ++k) h[k] = (uint8_t)((k * 2654435761u) >> 24);
    CK(hipMemcpy(i0, h.data(), h.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(i1, h.data(), h.size(), hipMemcpyHostToDevice));
    long long off = 0;
    for (int l = 0; l <= L; ++l) {
        a.off[l] = off;
        a.w[l] = Wp >> l;
        off += (long long)(Wp >> l) * (Hp >> l);
    }
    float *p0, *p1;
    CK(hipMalloc(&p0, sizeof(float) * off * B));
    CK(hipMalloc(&p1, sizeof(float) * off * B));
    a.I0 = i0;
    a.I1 = i1;
    a.stride = W;
    a.pair_stride = fsz;
    a.W = W;
    a.H = H;
    a.Wp = Wp;
    a.Hp = Hp;
    a.pl = 0;
    a.pt = 4;
    a.img0 = p0;
    a.img1 = p1;
    a.plane_stride = off;
    a.levels = L;
    a.write_l0 = 0;
    a.dword_ok = 1;
    a.qword_ok = argc > 2 ? atoi(argv[2]) : 1;
    const int nb = (Wp / 64) * (Hp / 64) * B;
    unsigned long long* prof;
    CK(hipMalloc(&prof, sizeof(unsigned long long) * 8 * nb));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(dis::g_pyr_prof), &prof, sizeof(prof)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int k = 0; k < 5; ++k) CK(dis::launch_pyramid(a, B, 0, dis::Timing{}));
    CK(hipEventRecord(e0, 0));
    const int R = 20;
    for (int k = 0; k < R; ++k) CK(dis::launch_pyramid(a, B, 0, dis::Timing{}));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("k_pyramid<6> %d pairs: %.1f us per launch (%d workgroups)\n", B, 1e3 * ms / R, nb);
    std::vector<unsigned long long> p(8 * (size_t)nb);
    CK(hipMemcpy(p.data(), prof, sizeof(unsigned long long) * p.size(), hipMemcpyDeviceToHost));
    // phases in shader clocks (wave 0)
    const char* nm[4] = {"load+lds", "barrier", "level1", "levels2+"};
    for (int ph = 0; ph < 4; ++ph) {
        std::vector<double> d(nb);
        for (int i = 0; i < nb; ++i) d[i] = (double)(p[8 * i + ph + 1] - p[8 * i + ph]);
        std::sort(d.begin(), d.end());
        double s = 0;
        for (double v : d) s += v;
        printf("%-10s mean %8.0f  p10 %8.0f  p50 %8.0f  p90 %8.0f clk\n", nm[ph], s / nb, d[nb / 10], d[nb / 2],
               d[9 * nb / 10]);
    }
    {
        std::vector<double> d(nb);
        for (int i = 0; i < nb; ++i) d[i] = (double)(p[8 * i + 4] - p[8 * i + 0]);
        std::sort(d.begin(), d.end());
        double s = 0;
        for (double v : d) s += v;
        printf("%-10s mean %8.0f  p50 %8.0f clk; wall (100 MHz):", "total", s / nb, d[nb / 2]);
        std::vector<double> w(nb);
        unsigned long long t0 = ~0ull, t1 = 0;
        for (int i = 0; i < nb; ++i) {
            w[i] = (double)(p[8 * i + 5] - p[8 * i + 7]) * 10.0;
            t0 = std::min(t0, p[8 * i + 7]);
            t1 = std::max(t1, p[8 * i + 5]);
        }
        std::sort(w.begin(), w.end());
        printf(" wg lifetime p50 %.0f ns, launch span %.1f us\n", w[nb / 2], (t1 - t0) * 1e-2);
        // residency: workgroups per (xcc, se, cu) at the launch midpoint and averaged
        std::map<unsigned long long, int> cus;
        for (int i = 0; i < nb; ++i) {
            const unsigned long long hw = p[8 * i + 6];
            const unsigned long long cu = ((hw >> 32) & 0xf) << 16 | ((hw >> 13) & 7) << 8 | ((hw >> 8) & 0xf) | ((hw >> 12) & 1) << 4;
            cus[cu]++;
        }
        int mn = 1 << 30, mx = 0;
        for (auto& kv : cus) mn = std::min(mn, kv.second), mx = std::max(mx, kv.second);
        printf("CUs used %zu, workgroups per CU min %d max %d\n", cus.size(), mn, mx);
        // average concurrency per CU: sum of lifetimes / (span * CUs)
        double life = 0;
        for (int i = 0; i < nb; ++i) life += (double)(p[8 * i + 5] - p[8 * i + 7]);
        printf("mean resident workgroups per CU %.2f\n", life / ((double)(t1 - t0) * cus.size()));
    }
    return 0;
}
