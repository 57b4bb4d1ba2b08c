// png.hpp -- minimal PNG codec for the frame-sequence CLI (zlib only; the
// reference reads frames with OpenCV's cv::imread(..., GRAYSCALE) and writes
// the colour-coded flow with cv::imwrite, src/main.cpp:129-130,200).
//
// Decode: 8/16-bit (and 1/2/4-bit gray / palette) non-interlaced PNGs of any
// colour type, to 8-bit gray the way OpenCV's imread does it for GRAYSCALE:
// 16-bit samples keep their high byte, colour goes through cvtColor's fixed
// point Rec.601 luma (R*4899 + G*9617 + B*1868 + 2^13) >> 14, alpha dropped.
// (OpenCV is absent here, so that conversion is unpinned; gray PNGs, the
// usual optical-flow benchmark input after conversion, are exact.)
// Encode: 8-bit RGB, filter 0, zlib level 6.
#pragma once

#include <zlib.h>

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

namespace png {

struct Gray {
    int width = 0, height = 0;
    std::vector<uint8_t> px;  // row-major, width * height
};

namespace detail {

inline uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

inline void put32(std::vector<uint8_t>& v, uint32_t x)
{
    v.push_back((uint8_t)(x >> 24));
    v.push_back((uint8_t)(x >> 16));
    v.push_back((uint8_t)(x >> 8));
    v.push_back((uint8_t)x);
}

inline int paeth(int a, int b, int c)
{
    const int p = a + b - c, pa = p > a ? p - a : a - p, pb = p > b ? p - b : b - p, pc = p > c ? p - c : c - p;
    return (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
}

inline uint8_t luma(int r, int g, int b) { return (uint8_t)((r * 4899 + g * 9617 + b * 1868 + (1 << 13)) >> 14); }

inline std::vector<uint8_t> read_file(const std::string& path)
{
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) throw std::runtime_error("cannot open " + path);
    std::vector<uint8_t> d;
    uint8_t buf[1 << 16];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) d.insert(d.end(), buf, buf + n);
    std::fclose(f);
    return d;
}

}  // namespace detail

inline Gray decode_gray(const std::vector<uint8_t>& d, const std::string& name = "png")
{
    using namespace detail;
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (d.size() < 8 || !std::equal(sig, sig + 8, d.begin())) throw std::runtime_error(name + ": not a PNG");
    int w = 0, h = 0, depth = 0, ctype = -1, interlace = 0;
    std::vector<uint8_t> idat, plte;
    size_t p = 8;
    bool end = false;
    while (!end) {
        if (p + 12 > d.size()) throw std::runtime_error(name + ": truncated");
        const uint32_t len = be32(&d[p]);
        if (len > d.size() - p - 12) throw std::runtime_error(name + ": bad chunk length");
        const uint8_t* type = &d[p + 4];
        const uint8_t* data = &d[p + 8];
        if (crc32(crc32(0L, Z_NULL, 0), type, len + 4) != be32(data + len)) throw std::runtime_error(name + ": CRC");
        const std::string t(reinterpret_cast<const char*>(type), 4);
        if (t == "IHDR") {
            if (len != 13) throw std::runtime_error(name + ": IHDR");
            w = (int)be32(data);
            h = (int)be32(data + 4);
            depth = data[8];
            ctype = data[9];
            interlace = data[12];
            if (data[10] != 0 || data[11] != 0) throw std::runtime_error(name + ": unknown compression/filter");
        } else if (t == "PLTE") {
            plte.assign(data, data + len);
        } else if (t == "IDAT") {
            idat.insert(idat.end(), data, data + len);
        } else if (t == "IEND") {
            end = true;
        }
        p += 12 + len;
    }
    if (w < 1 || h < 1 || w > (1 << 16) || h > (1 << 16) || (long long)w * h > (1LL << 28))
        throw std::runtime_error(name + ": bad size");  // (the engine's frame limit, dis_create)
    if (interlace) throw std::runtime_error(name + ": interlaced PNG not supported");
    int ch;
    switch (ctype) {
        case 0: ch = 1; break;
        case 2: ch = 3; break;
        case 3: ch = 1; break;
        case 4: ch = 2; break;
        case 6: ch = 4; break;
        default: throw std::runtime_error(name + ": bad colour type");
    }
    if (!(depth == 8 || depth == 16 || ((ctype == 0 || ctype == 3) && (depth == 1 || depth == 2 || depth == 4))))
        throw std::runtime_error(name + ": unsupported bit depth");
    if (ctype == 3 && plte.size() < 3) throw std::runtime_error(name + ": missing palette");
    const size_t bits = (size_t)w * ch * depth, rowb = (bits + 7) / 8, bpp = std::max<size_t>(1, ch * depth / 8);
    std::vector<uint8_t> raw((rowb + 1) * h);
    uLongf rawlen = raw.size();
    if (uncompress(raw.data(), &rawlen, idat.data(), idat.size()) != Z_OK || rawlen != raw.size())
        throw std::runtime_error(name + ": bad image data");
    std::vector<uint8_t> img(rowb * h);
    for (int y = 0; y < h; ++y) {
        const uint8_t f = raw[y * (rowb + 1)];
        const uint8_t* s = &raw[y * (rowb + 1) + 1];
        uint8_t* o = &img[y * rowb];
        const uint8_t* up = y ? &img[(y - 1) * rowb] : nullptr;
        for (size_t i = 0; i < rowb; ++i) {
            const int a = i >= bpp ? o[i - bpp] : 0, b = up ? up[i] : 0, c = (up && i >= bpp) ? up[i - bpp] : 0;
            int v;
            switch (f) {
                case 0: v = s[i]; break;
                case 1: v = s[i] + a; break;
                case 2: v = s[i] + b; break;
                case 3: v = s[i] + ((a + b) >> 1); break;
                case 4: v = s[i] + paeth(a, b, c); break;
                default: throw std::runtime_error(name + ": bad filter");
            }
            o[i] = (uint8_t)v;
        }
    }
    Gray g;
    g.width = w;
    g.height = h;
    g.px.resize((size_t)w * h);
    const int bs = depth == 16 ? 2 : 1;  // bytes per sample (>= 8-bit)
    for (int y = 0; y < h; ++y) {
        const uint8_t* r = &img[y * rowb];
        for (int x = 0; x < w; ++x) {
            uint8_t out;
            if (depth < 8) {
                const int per = 8 / depth, sh = 8 - depth * (x % per + 1);
                const int v = (r[x / per] >> sh) & ((1 << depth) - 1);
                if (ctype == 3) {
                    const size_t k = (size_t)v * 3;
                    out = k + 2 < plte.size() ? luma(plte[k], plte[k + 1], plte[k + 2]) : 0;
                } else {
                    out = (uint8_t)(v * 255 / ((1 << depth) - 1));
                }
            } else {
                const uint8_t* s = r + (size_t)x * ch * bs;  // high byte of each sample first
                if (ctype == 0 || ctype == 4) out = s[0];
                else if (ctype == 3) {
                    const size_t k = (size_t)s[0] * 3;
                    out = k + 2 < plte.size() ? luma(plte[k], plte[k + 1], plte[k + 2]) : 0;
                } else {
                    out = luma(s[0], s[bs], s[2 * bs]);
                }
            }
            g.px[(size_t)y * w + x] = out;
        }
    }
    return g;
}

inline Gray read_gray(const std::string& path) { return decode_gray(detail::read_file(path), path); }

// 8-bit RGB PNG from BGR pixels (OpenCV Vec3b order, as cv::imwrite takes them)
inline std::vector<uint8_t> encode_bgr(const uint8_t* bgr, int w, int h)
{
    using namespace detail;
    std::vector<uint8_t> raw((size_t)(3 * w + 1) * h);
    for (int y = 0; y < h; ++y) {
        uint8_t* o = &raw[(size_t)y * (3 * w + 1)];
        o[0] = 0;
        for (int x = 0; x < w; ++x) {
            const uint8_t* s = bgr + ((size_t)y * w + x) * 3;
            o[1 + 3 * x] = s[2];
            o[2 + 3 * x] = s[1];
            o[3 + 3 * x] = s[0];
        }
    }
    uLongf zlen = compressBound(raw.size());
    std::vector<uint8_t> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), raw.size(), 6) != Z_OK) throw std::runtime_error("png: compress");
    z.resize(zlen);
    std::vector<uint8_t> out = {137, 80, 78, 71, 13, 10, 26, 10};
    auto chunk = [&](const char* type, const std::vector<uint8_t>& data) {
        put32(out, (uint32_t)data.size());
        const size_t t0 = out.size();
        out.insert(out.end(), type, type + 4);
        out.insert(out.end(), data.begin(), data.end());
        put32(out, (uint32_t)crc32(crc32(0L, Z_NULL, 0), &out[t0], (uInt)(data.size() + 4)));
    };
    std::vector<uint8_t> ihdr;
    put32(ihdr, (uint32_t)w);
    put32(ihdr, (uint32_t)h);
    ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});
    chunk("IHDR", ihdr);
    chunk("IDAT", z);
    chunk("IEND", {});
    return out;
}

inline void write_bgr(const std::string& path, const uint8_t* bgr, int w, int h)
{
    const std::vector<uint8_t> d = encode_bgr(bgr, w, h);
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot create " + path);
    const bool ok = std::fwrite(d.data(), 1, d.size(), f) == d.size();
    if (std::fclose(f) != 0 || !ok) throw std::runtime_error("write failed: " + path);
}

}  // namespace png
