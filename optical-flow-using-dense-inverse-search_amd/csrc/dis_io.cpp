// dis_io.cpp -- Middlebury .flo I/O: the format of
// ReadFlowFile / SaveFlowFile, src/IO_flow.cpp:10-98 -- the 4 bytes "PIEH"
// (= float 202021.25), int32 width, int32 height, then width*height*channels
// float32, row-major, channels interleaved (1 depth, 2 flow, 4 scene flow),
// little-endian. Unlike the reference (which prints and carries on), every
// malformed file, size mismatch or I/O failure is an error status.
#include <cstdio>
#include <cstring>
#include <string>

#include "dis_abi.h"

namespace dis {
dis_status set_error(dis_status s, const std::string& msg);  // dis_runtime.hip
}

namespace {

constexpr float kTag = 202021.25f;  // "PIEH" read as a little-endian float

struct File {
    FILE* f = nullptr;
    ~File()
    {
        if (f) std::fclose(f);
    }
};

bool channels_ok(int c) { return c == 1 || c == 2 || c == 4; }

}  // namespace

extern "C" {

dis_status dis_flo_info(const char* path, int* width, int* height)
{
    if (!path || !width || !height) return dis::set_error(DIS_ERR_INVALID_ARGUMENT, "null pointer");
    File fh;
    fh.f = std::fopen(path, "rb");
    if (!fh.f) return dis::set_error(DIS_ERR_INVALID_ARGUMENT, std::string("cannot open ") + path);
    float tag = 0.0f;
    int w = 0, h = 0;
    if (std::fread(&tag, 4, 1, fh.f) != 1 || std::fread(&w, 4, 1, fh.f) != 1 || std::fread(&h, 4, 1, fh.f) != 1)
        return dis::set_error(DIS_ERR_INVALID_ARGUMENT, std::string("short .flo header: ") + path);
    if (tag != kTag) return dis::set_error(DIS_ERR_INVALID_ARGUMENT, std::string("not a .flo file (tag): ") + path);
    if (w < 1 || h < 1 || w > (1 << 20) || h > (1 << 20))
        return dis::set_error(DIS_ERR_INVALID_ARGUMENT, std::string("bad .flo dimensions: ") + path);
    *width = w;
    *height = h;
    return DIS_OK;
}

dis_status dis_read_flo(const char* path, float* data, int width, int height, int channels)
{
    if (!data) return dis::set_error(DIS_ERR_INVALID_ARGUMENT, "null pointer");
    if (!channels_ok(channels)) return dis::set_error(DIS_ERR_INVALID_ARGUMENT, "channels must be 1, 2 or 4");
    int w = 0, h = 0;
    const dis_status st = dis_flo_info(path, &w, &h);
    if (st != DIS_OK) return st;
    if (w != width || h != height) return dis::set_error(DIS_ERR_INVALID_ARGUMENT, ".flo size differs from the buffer");
    File fh;
    fh.f = std::fopen(path, "rb");
    if (!fh.f || std::fseek(fh.f, 12, SEEK_SET) != 0) return dis::set_error(DIS_ERR_INVALID_ARGUMENT, "cannot reopen");
    const size_t n = (size_t)w * h * channels;
    if (std::fread(data, sizeof(float), n, fh.f) != n)
        return dis::set_error(DIS_ERR_INVALID_ARGUMENT, std::string(".flo file is too short: ") + path);
    if (std::fgetc(fh.f) != EOF)
        return dis::set_error(DIS_ERR_INVALID_ARGUMENT, std::string(".flo file is too long: ") + path);
    return DIS_OK;
}

dis_status dis_write_flo(const char* path, const float* data, int width, int height, int channels)
{
    if (!path || !data) return dis::set_error(DIS_ERR_INVALID_ARGUMENT, "null pointer");
    if (!channels_ok(channels)) return dis::set_error(DIS_ERR_INVALID_ARGUMENT, "channels must be 1, 2 or 4");
    if (width < 1 || height < 1) return dis::set_error(DIS_ERR_INVALID_ARGUMENT, "width, height must be >= 1");
    File fh;
    fh.f = std::fopen(path, "wb");
    if (!fh.f) return dis::set_error(DIS_ERR_INVALID_ARGUMENT, std::string("cannot create ") + path);
    const size_t n = (size_t)width * height * channels;
    if (std::fwrite("PIEH", 1, 4, fh.f) != 4 || std::fwrite(&width, 4, 1, fh.f) != 1 ||
        std::fwrite(&height, 4, 1, fh.f) != 1 || std::fwrite(data, sizeof(float), n, fh.f) != n)
        return dis::set_error(DIS_ERR_INVALID_ARGUMENT, std::string("write failed: ") + path);
    if (std::fclose(fh.f) != 0) {
        fh.f = nullptr;
        return dis::set_error(DIS_ERR_INVALID_ARGUMENT, std::string("write failed: ") + path);
    }
    fh.f = nullptr;
    return DIS_OK;
}

}  // extern "C"
