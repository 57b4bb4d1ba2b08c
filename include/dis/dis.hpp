// dis.hpp -- C++ host facade of the MI355X DIS engine, header-only over the
// C-ABI (include/dis_abi.h).
//
//   dis::DenseInverseSearch   calc(I0, I1, flow) for u8 frames; presets
//                             (the per-pair body of src/main.cpp:135-198)
//   OpticalFlow::OpticalFlowClass
//                             drop-in for the reference constructor with the
//                             identical signature (include/optical_flow.hpp:43-54,
//                             src/optical_flow.cpp:19-91): padded host pyramids
//                             in, finest-level flow out, computed on the GPU.
//
// Errors surface as dis::Error (status + the ABI's last-error text); the
// reference had no error reporting at all (bad input was UB).
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../dis_abi.h"

namespace dis {

enum class Preset {
    ULTRAFAST = DIS_PRESET_ULTRAFAST,
    FAST = DIS_PRESET_FAST,
    MEDIUM = DIS_PRESET_MEDIUM,
    SLOW = DIS_PRESET_SLOW,
    REFERENCE = DIS_PRESET_REFERENCE,
};

class Error : public std::runtime_error {
public:
    Error(dis_status s, const std::string& what) : std::runtime_error(what), status_(s) {}
    dis_status status() const { return status_; }

private:
    dis_status status_;
};

inline void check(dis_status s)
{
    if (s != DIS_OK) throw Error(s, std::string("dis: ") + dis_last_error());
}

inline dis_params preset_params(Preset p, int width, int height)
{
    dis_params out{};
    check(dis_preset_params(static_cast<dis_preset>(p), width, height, &out));
    return out;
}

class DenseInverseSearch {
public:
    DenseInverseSearch(const dis_params& params, int width, int height, int max_batch = 1, int device = 0)
        : params_(params), width_(width), height_(height)
    {
        check(dis_create(&ctx_, &params_, width, height, max_batch, device));
    }
    DenseInverseSearch(Preset preset, int width, int height, int max_batch = 1, int device = 0)
        : DenseInverseSearch(preset_params(preset, width, height), width, height, max_batch, device)
    {
    }
    static std::unique_ptr<DenseInverseSearch> create(Preset preset, int width, int height, int max_batch = 1,
                                                      int device = 0)
    {
        return std::unique_ptr<DenseInverseSearch>(new DenseInverseSearch(preset, width, height, max_batch, device));
    }
    ~DenseInverseSearch() { dis_destroy(ctx_); }
    DenseInverseSearch(const DenseInverseSearch&) = delete;
    DenseInverseSearch& operator=(const DenseInverseSearch&) = delete;
    DenseInverseSearch(DenseInverseSearch&& o) noexcept
        : ctx_(std::exchange(o.ctx_, nullptr)), params_(o.params_), width_(o.width_), height_(o.height_)
    {
    }

    // Host u8 frames (row stride in bytes, 0 = width) -> host W*H*2 flow (u,v).
    void calc(const uint8_t* I0, const uint8_t* I1, float* flow, size_t stride = 0)
    {
        check(dis_calc_u8(ctx_, I0, I1, stride, flow, DIS_MEM_HOST, nullptr));
    }
    std::vector<float> calc(const std::vector<uint8_t>& I0, const std::vector<uint8_t>& I1)
    {
        if (I0.size() != (size_t)width_ * height_ || I1.size() != I0.size())
            throw Error(DIS_ERR_INVALID_ARGUMENT, "dis: frame size does not match the context");
        std::vector<float> flow((size_t)width_ * height_ * 2);
        calc(I0.data(), I1.data(), flow.data());
        return flow;
    }
    // Device-resident frames/flow; asynchronous on `stream` (hipStream_t).
    void calc_device(const uint8_t* dI0, const uint8_t* dI1, float* dflow, void* stream = nullptr, size_t stride = 0)
    {
        check(dis_calc_u8(ctx_, dI0, dI1, stride, dflow, DIS_MEM_DEVICE, stream));
    }
    // n pairs: frames at I0 + k*pair_stride, flows at flow + k*W*H*2.
    void calc_batch(int n, const uint8_t* I0, const uint8_t* I1, float* flow, dis_mem where = DIS_MEM_HOST,
                    void* stream = nullptr, size_t stride = 0, size_t pair_stride = 0)
    {
        check(dis_calc_batch_u8(ctx_, n, I0, I1, stride, pair_stride, flow, where, stream));
    }
    void set_concurrency(int streams) { check(dis_set_concurrency(ctx_, streams)); }
    // DIS_PRECISION_EXACT (default) or DIS_PRECISION_FMA (dis_abi.h)
    void set_precision(int mode) { check(dis_set_precision(ctx_, mode)); }
    void set_graphs(bool on) { check(dis_set_graphs(ctx_, on ? 1 : 0)); }
    // host-memory batches: pairs per overlapped chunk (0 = auto), ABI v8
    void set_host_pipeline(int chunk_pairs) { check(dis_set_host_pipeline(ctx_, chunk_pairs)); }

    const dis_params& params() const { return params_; }
    int width() const { return width_; }
    int height() const { return height_; }
    dis_ctx* handle() const { return ctx_; }

private:
    dis_ctx* ctx_ = nullptr;
    dis_params params_;
    int width_, height_;
};

// Middlebury colour coding (src/color_coding.cpp draw_optical_flow) of n
// W x H (u,v) fields into BGR u8, on the GPU.
inline void flow_color(const float* flow, int n, int width, int height, uint8_t* bgr, float maxmotion = -1.0f,
                       dis_mem where = DIS_MEM_HOST, void* stream = nullptr, int device = 0)
{
    check(dis_flow_color(flow, n, width, height, maxmotion, bgr, where, stream, device));
}

// Middlebury .flo files (src/IO_flow.cpp ReadFlowFile / SaveFlowFile).
inline void write_flo(const std::string& path, const float* data, int width, int height, int channels = 2)
{
    check(dis_write_flo(path.c_str(), data, width, height, channels));
}
inline std::vector<float> read_flo(const std::string& path, int* width, int* height, int channels = 2)
{
    check(dis_flo_info(path.c_str(), width, height));
    std::vector<float> v((size_t)*width * *height * channels);
    check(dis_read_flo(path.c_str(), v.data(), *width, *height, channels));
    return v;
}

}  // namespace dis

namespace OpticalFlow {

// Same constructor signature and semantics as the reference
// (include/optical_flow.hpp:43-54): the whole coarse-to-fine computation runs
// inside the constructor and writes `outflow` ((width>>F) x (height>>F) x 2).
// draw_grid (an OpenCV GUI debug view) is not supported.
class OpticalFlowClass {
public:
    OpticalFlowClass(float** img_first_in, float** img_first_dx_in, float** img_first_dy_in,
                     float** img_second_in, float** img_second_dx_in, float** img_second_dy_in,
                     int img_padding_in, float* outflow, int width_in, int height_in, int coarsest_scale,
                     int finest_scale, int iterations, int patch_size, float patch_overlap, bool patnorm_in,
                     bool draw_grid, int device = 0)
    {
        if (draw_grid) throw dis::Error(DIS_ERR_UNSUPPORTED, "dis: draw_grid (OpenCV GUI) is not supported");
        dis::check(dis_flow_from_pyramids(img_first_in, img_first_dx_in, img_first_dy_in, img_second_in,
                                          img_second_dx_in, img_second_dy_in, img_padding_in, outflow, width_in,
                                          height_in, coarsest_scale, finest_scale, iterations, patch_size,
                                          patch_overlap, patnorm_in ? 1 : 0, device));
    }
};

}  // namespace OpticalFlow
