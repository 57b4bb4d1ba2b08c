// dis_flow -- frame-sequence CLI over the MI355X engine,
// the reference's main() (src/main.cpp:59-206) with its argument conventions:
//
//   dis_flow                                   alley_1 frames 1..50, defaults
//   dis_flow folder start end
//   dis_flow folder start end iters patch_size coarsest finest overlap norm draw_grid
//
// plus options (after the positionals): --flo (also write OF_<folder>/frame_NNNN.flo,
// the SaveFlowFile format of src/IO_flow.cpp:56-98, which the reference left
// commented out at src/main.cpp:137-146), --batch N (pairs per GPU call,
// default 8; the reference is one pair at a time), --device D, --paper (the DIS
// paper's residual and densification; not the reference's),
// --refine K (K fixed-point iterations of variational refinement, 8f row 1).
//
// For img_i in [start, end): reads <folder>/frame_<img_i>.png and frame_<img_i+1>
// (grayscale, src/main.cpp:118-130), computes the full-resolution flow
// (dis::DenseInverseSearch::calc: src/main.cpp:135-198), colour-codes it
// (dis_flow_color = draw_optical_flow, :200) and writes OF_<folder>/frame_<img_i>.png
// (:201). GUI windows (imshow / draw_grid) are not supported.
#include <sys/stat.h>

#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <stdexcept>
#include <string>
#include <vector>

#include "dis/dis.hpp"
#include "png.hpp"

namespace {

std::string frame_name(const std::string& folder, int i)
{
    char buf[32];
    std::snprintf(buf, sizeof buf, "/frame_%04d", i);
    return folder + buf;
}

void usage()
{
    std::cout << "Not good parameters!\n"
                 "1. Run without parameters with default parameters (alley_1) from 1 to 50\n"
                 "2. Set folder and images with default parameters:\n"
                 "dis_flow folder start_num_image end_num_image\n"
                 "3. Add full settings\n"
                 "dis_flow folder start_num_image end_num_image max_iter patch_size coarsest_scale finest_scale "
                 "patch_overlap patch_norm draw_grid\n"
                 "options: --flo  --batch N  --device D  --paper  --refine K"
              << std::endl;
}

}  // namespace

int main(int argc, char** argv)
{
    // reference defaults, src/main.cpp:63-72
    std::string folder = "alley_1";
    int start = 1, end = 50;
    dis_params p{};
    p.iterations = 1000;
    p.patch_size = 8;
    p.coarsest_scale = 3;
    p.finest_scale = 0;
    p.patch_overlap = 0.7f;
    p.patch_normalization = 1;
    p.var_refine_iters = 0;
    int draw_grid = 0;
    bool write_flo = false;
    int batch = 8, device = 0;

    std::vector<std::string> pos;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        if (a == "--flo") {
            write_flo = true;
        } else if (a == "--batch" && i + 1 < argc) {
            batch = std::atoi(argv[++i]);
        } else if (a == "--device" && i + 1 < argc) {
            device = std::atoi(argv[++i]);
        } else if (a == "--paper") {
            p.paper_mode = 1;
        } else if (a == "--refine" && i + 1 < argc) {
            p.var_refine_iters = std::atoi(argv[++i]);
        } else {
            pos.push_back(a);
        }
    }
    if (pos.size() == 3 || pos.size() == 10) {
        folder = pos[0];
        start = std::atoi(pos[1].c_str());
        end = std::atoi(pos[2].c_str());
    }
    if (pos.size() == 10) {  // argv[4..10] order of src/main.cpp:84-92
        p.iterations = std::atoi(pos[3].c_str());
        p.patch_size = std::atoi(pos[4].c_str());
        p.coarsest_scale = std::atoi(pos[5].c_str());
        p.finest_scale = std::atoi(pos[6].c_str());
        p.patch_overlap = (float)std::atof(pos[7].c_str());
        p.patch_normalization = std::atoi(pos[8].c_str());
        draw_grid = std::atoi(pos[9].c_str());
    } else if (!pos.empty() && pos.size() != 3) {
        usage();
        return 0;  // as the reference
    }
    if (draw_grid) {
        std::cerr << "draw_grid (OpenCV GUI) is not supported" << std::endl;
        return 2;
    }
    if (batch < 1) batch = 1;
    const std::string out_dir = "OF_" + folder;
    ::mkdir(out_dir.c_str(), 0755);  // CreateFolder (src/main.cpp:52-57): existing is fine

    try {
        std::unique_ptr<dis::DenseInverseSearch> eng;
        int W = 0, H = 0;
        for (int i0 = start; i0 < end; i0 += batch) {
            const int n = std::min(batch, end - i0);
            std::vector<png::Gray> frames;
            for (int k = 0; k <= n; ++k) {
                if (k < n) std::cout << "start " << frame_name(folder, i0 + k) << ".png" << std::endl;
                frames.push_back(png::read_gray(frame_name(folder, i0 + k) + ".png"));
            }
            if (!eng || frames[0].width != W || frames[0].height != H) {
                W = frames[0].width;
                H = frames[0].height;
                eng.reset(new dis::DenseInverseSearch(p, W, H, batch, device));
            }
            std::vector<uint8_t> I0((size_t)n * W * H), I1((size_t)n * W * H);
            for (int k = 0; k < n; ++k) {
                if (frames[k].width != W || frames[k].height != H || frames[k + 1].width != W || frames[k + 1].height != H)
                    throw std::runtime_error("frame sizes differ within a batch");
                std::copy(frames[k].px.begin(), frames[k].px.end(), I0.begin() + (size_t)k * W * H);
                std::copy(frames[k + 1].px.begin(), frames[k + 1].px.end(), I1.begin() + (size_t)k * W * H);
            }
            std::vector<float> flow((size_t)n * W * H * 2);
            eng->calc_batch(n, I0.data(), I1.data(), flow.data());
            std::vector<uint8_t> bgr((size_t)n * W * H * 3);
            dis::check(dis_flow_color(flow.data(), n, W, H, -1.0f, bgr.data(), DIS_MEM_HOST, nullptr, device));
            for (int k = 0; k < n; ++k) {
                const std::string base = "OF_" + frame_name(folder, i0 + k);
                png::write_bgr(base + ".png", bgr.data() + (size_t)k * W * H * 3, W, H);
                if (write_flo)
                    dis::check(dis_write_flo((base + ".flo").c_str(), flow.data() + (size_t)k * W * H * 2, W, H, 2));
                std::cout << "finish " << frame_name(folder, i0 + k) << ".png" << std::endl;
            }
        }
    } catch (const std::exception& e) {
        std::cerr << "dis_flow: " << e.what() << std::endl;
        return 1;
    }
    return 0;
}
