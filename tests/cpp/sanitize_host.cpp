// Host code under AddressSanitizer + UndefinedBehaviorSanitizer (VERDICT r1
// "host hygiene"): the parts of the repository that run on the CPU and parse
// or produce data -- the C oracle (tests' checker and bench.py's CPU
// baseline), the .flo reader/writer (csrc/dis_io.cpp, src/IO_flow.cpp
// format), the synthetic-pair generator (csrc/dis_synth.cpp) and the CLI's
// PNG decoder (cli/png.hpp), which parses untrusted files. Built by
// `make -C tests/cpp sanitize` with -fsanitize=address,undefined and
// -fno-sanitize-recover, so any finding aborts with a non-zero status.
//
// Corpus: .flo files with a bad tag, truncated header / data, trailing bytes,
// zero / negative / huge sizes; every single-byte corruption and every
// truncation of a valid PNG, plus random garbage, fed to the decoder (which
// must throw or decode, never crash or read out of bounds).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "dis_abi.h"
#include "dis_oracle.h"
#include "png.hpp"

namespace dis {
// dis_io.cpp reports through the runtime's error slot (dis_runtime.hip)
dis_status set_error(dis_status s, const std::string&) { return s; }
}  // namespace dis

static int failures = 0;
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            std::fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #c); \
            ++failures;                                                       \
        }                                                                     \
    } while (0)

static void write_bytes(const std::string& path, const std::vector<uint8_t>& d)
{
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot write " + path);
    if (!d.empty()) std::fwrite(d.data(), 1, d.size(), f);
    std::fclose(f);
}

static std::vector<uint8_t> read_bytes(const std::string& path)
{
    FILE* f = std::fopen(path.c_str(), "rb");
    std::vector<uint8_t> d;
    if (!f) return d;
    int c;
    while ((c = std::fgetc(f)) != EOF) d.push_back((uint8_t)c);
    std::fclose(f);
    return d;
}

static void oracle_paths()
{
    struct Case {
        int W, H, C, F, ps, it;
        float ov;
        int norm, vr, paper;
    } cases[] = {
        {160, 120, 3, 1, 8, 12, 0.625f, 1, 0, 0},  // MEDIUM-like
        {37, 29, 2, 2, 2, 3, 0.0f, 1, 0, 0},       // ragged, ps 2, F == C
        {96, 64, 2, 0, 6, 5, 0.5f, 0, 0, 0},       // ps 6, no normalisation
        {64, 48, 2, 0, 8, 4, 0.75f, 1, 2, 0},      // variational refinement
        {80, 64, 2, 1, 8, 6, 0.5f, 1, 0, 1},       // paper mode
    };
    for (const Case& c : cases) {
        std::vector<uint8_t> I0((size_t)c.W * c.H), I1(I0.size());
        std::vector<float> gt((size_t)c.W * c.H * 2);
        CHECK(dis_synth_pair(7, c.W, c.H, I0.data(), I1.data(), gt.data()) == DIS_OK);
        dis_oracle_params p{c.C, c.F, c.ps, c.it, c.ov, c.norm, c.vr, c.paper};
        std::vector<float> flow((size_t)c.W * c.H * 2, NAN);
        CHECK(dis_oracle_calc_u8(&p, c.W, c.H, I0.data(), I1.data(), (size_t)c.W, flow.data()) == 0);
        for (float v : flow) CHECK(std::isfinite(v));
        std::vector<uint8_t> bgr((size_t)c.W * c.H * 3);
        dis_oracle_flow_color(flow.data(), c.W, c.H, -1.0f, bgr.data());
    }
    // degenerate synthetic sizes
    for (int wh : {1, 2, 3}) {
        std::vector<uint8_t> a((size_t)wh * 5), b(a.size());
        CHECK(dis_synth_pair(1, wh, 5, a.data(), b.data(), nullptr) == DIS_OK);
    }
    CHECK(dis_synth_pair(1, 0, 5, nullptr, nullptr, nullptr) != DIS_OK);
}

static void flo_files(const std::string& dir)
{
    const int W = 13, H = 7;
    std::vector<float> f((size_t)W * H * 2);
    for (size_t i = 0; i < f.size(); ++i) f[i] = (float)i * 0.25f - 3.0f;
    const std::string good = dir + "/good.flo";
    CHECK(dis_write_flo(good.c_str(), f.data(), W, H, 2) == DIS_OK);
    int w = 0, h = 0;
    CHECK(dis_flo_info(good.c_str(), &w, &h) == DIS_OK && w == W && h == H);
    std::vector<float> back(f.size());
    CHECK(dis_read_flo(good.c_str(), back.data(), W, H, 2) == DIS_OK);
    CHECK(std::memcmp(back.data(), f.data(), f.size() * 4) == 0);
    CHECK(dis_read_flo(good.c_str(), back.data(), W + 1, H, 2) != DIS_OK);  // size mismatch
    CHECK(dis_read_flo(good.c_str(), back.data(), W, H, 3) != DIS_OK);      // bad channel count
    const std::vector<uint8_t> d = read_bytes(good);
    auto expect_bad = [&](std::vector<uint8_t> bad, const char* what) {
        const std::string p = dir + "/bad.flo";
        write_bytes(p, bad);
        int bw = 0, bh = 0;
        const dis_status si = dis_flo_info(p.c_str(), &bw, &bh);
        const dis_status sr = dis_read_flo(p.c_str(), back.data(), W, H, 2);
        if (si == DIS_OK && sr == DIS_OK) {
            std::fprintf(stderr, "bad .flo accepted: %s\n", what);
            ++failures;
        }
    };
    expect_bad({}, "empty");
    expect_bad(std::vector<uint8_t>(d.begin(), d.begin() + 3), "short tag");
    expect_bad(std::vector<uint8_t>(d.begin(), d.begin() + 10), "truncated header");
    expect_bad(std::vector<uint8_t>(d.begin(), d.end() - 1), "truncated data");
    std::vector<uint8_t> x = d;
    x.push_back(0);
    expect_bad(x, "trailing byte");
    x = d;
    x[0] ^= 1;
    expect_bad(x, "bad tag");
    for (int32_t bad_w : {0, -1, W + 1, 0x7fffffff}) {
        x = d;
        std::memcpy(&x[4], &bad_w, 4);
        expect_bad(x, "bad width");
    }
    for (int32_t bad_h : {0, -5, 0x40000000}) {
        x = d;
        std::memcpy(&x[8], &bad_h, 4);
        expect_bad(x, "bad height");
    }
    CHECK(dis_read_flo((dir + "/missing.flo").c_str(), back.data(), W, H, 2) != DIS_OK);
    CHECK(dis_write_flo((dir + "/no/such/dir/x.flo").c_str(), f.data(), W, H, 2) != DIS_OK);
}

static int decode_or_throw(const std::vector<uint8_t>& d)
{
    try {
        const png::Gray g = png::decode_gray(d, "fuzz");
        return (int)(g.px.size() == (size_t)g.width * g.height);
    } catch (const std::exception&) {
        return -1;
    }
}

static void png_files()
{
    // a valid 8-bit RGB PNG from the encoder, and a gray one built by hand
    const int w = 11, h = 6;
    std::vector<uint8_t> bgr((size_t)w * h * 3);
    for (size_t i = 0; i < bgr.size(); ++i) bgr[i] = (uint8_t)(i * 37 + 11);
    const std::vector<uint8_t> good = png::encode_bgr(bgr.data(), w, h);
    const png::Gray g = png::decode_gray(good, "good");
    CHECK(g.width == w && g.height == h && g.px.size() == (size_t)w * h);
    long decoded = 0, rejected = 0;
    for (size_t i = 0; i < good.size(); ++i)  // every truncation
        (decode_or_throw(std::vector<uint8_t>(good.begin(), good.begin() + i)) >= 0 ? decoded : rejected)++;
    for (size_t i = 0; i < good.size(); ++i)  // every byte position, three corruptions each
        for (uint8_t m : {(uint8_t)0x01, (uint8_t)0x80, (uint8_t)0xFF}) {
            std::vector<uint8_t> x = good;
            x[i] ^= m;
            (decode_or_throw(x) >= 0 ? decoded : rejected)++;
        }
    // corruptions past the CRC check: mutate one byte of a chunk's type or
    // data and recompute that chunk's CRC (IHDR fields, filter bytes, zlib data)
    for (size_t q = 8; q + 12 <= good.size();) {
        const uint32_t len = png::detail::be32(&good[q]);
        for (size_t i = q + 4; i < q + 8 + len; ++i)
            for (uint8_t m : {(uint8_t)0x01, (uint8_t)0x10, (uint8_t)0xFF}) {
                std::vector<uint8_t> x = good;
                x[i] ^= m;
                const uint32_t c = (uint32_t)crc32(crc32(0L, Z_NULL, 0), &x[q + 4], len + 4);
                x[q + 8 + len] = (uint8_t)(c >> 24);
                x[q + 9 + len] = (uint8_t)(c >> 16);
                x[q + 10 + len] = (uint8_t)(c >> 8);
                x[q + 11 + len] = (uint8_t)c;
                (decode_or_throw(x) >= 0 ? decoded : rejected)++;
            }
        q += 12 + len;
    }
    // well-formed containers around random scanlines: every colour type and
    // bit depth, random sizes, random (also invalid) filter bytes, palettes of
    // random (also short) length -- the filter and sample-unpacking paths
    std::mt19937 gen(11);
    auto chunk = [](std::vector<uint8_t>& o, const char* type, const std::vector<uint8_t>& data) {
        png::detail::put32(o, (uint32_t)data.size());
        const size_t t = o.size();
        o.insert(o.end(), type, type + 4);
        o.insert(o.end(), data.begin(), data.end());
        png::detail::put32(o, (uint32_t)crc32(crc32(0L, Z_NULL, 0), &o[t], (uInt)(data.size() + 4)));
    };
    const int types[][2] = {{0, 1}, {0, 2}, {0, 4}, {0, 8}, {0, 16}, {2, 8}, {2, 16}, {3, 1}, {3, 2},
                            {3, 4}, {3, 8}, {4, 8}, {4, 16}, {6, 8}, {6, 16}, {2, 4}, {5, 8}};
    for (int t = 0; t < 600; ++t) {
        const int ct = types[t % 17][0], dep = types[t % 17][1];
        const int pw = 1 + (int)(gen() % 40), ph = 1 + (int)(gen() % 20);
        const int ch = ct == 2 ? 3 : ct == 4 ? 2 : ct == 6 ? 4 : 1;
        const size_t rowb = ((size_t)pw * ch * dep + 7) / 8;
        std::vector<uint8_t> raw((rowb + 1) * ph);
        for (size_t i = 0; i < raw.size(); ++i) raw[i] = (uint8_t)gen();
        for (int y = 0; y < ph; ++y) raw[y * (rowb + 1)] = (uint8_t)(gen() % (t % 5 ? 5 : 7));
        std::vector<uint8_t> z(compressBound(raw.size()));
        uLongf zl = z.size();
        compress2(z.data(), &zl, raw.data(), raw.size(), 6);
        z.resize(zl);
        std::vector<uint8_t> o = {137, 80, 78, 71, 13, 10, 26, 10};
        std::vector<uint8_t> ihdr;
        png::detail::put32(ihdr, (uint32_t)pw);
        png::detail::put32(ihdr, (uint32_t)ph);
        ihdr.insert(ihdr.end(), {(uint8_t)dep, (uint8_t)ct, 0, 0, 0});
        chunk(o, "IHDR", ihdr);
        if (ct == 3 && t % 3) {
            std::vector<uint8_t> pl(3 * (1 + gen() % 256));
            for (auto& v : pl) v = (uint8_t)gen();
            chunk(o, "PLTE", pl);
        }
        chunk(o, "IDAT", z);
        chunk(o, "IEND", {});
        if (t % 7 == 0) o.resize(o.size() - 1 - gen() % 20);  // truncated
        (decode_or_throw(o) >= 0 ? decoded : rejected)++;
    }
    std::mt19937 rng(5);
    for (int t = 0; t < 2000; ++t) {  // garbage after a valid signature
        std::vector<uint8_t> x(good.begin(), good.begin() + 8);
        const int n = (int)(rng() % 200);
        for (int k = 0; k < n; ++k) x.push_back((uint8_t)rng());
        (decode_or_throw(x) >= 0 ? decoded : rejected)++;
    }
    CHECK(rejected > 0 && decoded > 100);
    std::printf("png corpus: %ld decoded, %ld rejected\n", decoded, rejected);
}

int main(int argc, char** argv)
{
    const std::string dir = argc > 1 ? argv[1] : ".";
    oracle_paths();
    flo_files(dir);
    png_files();
    std::printf("sanitize_host: %d failures\n", failures);
    return failures ? 1 : 0;
}
