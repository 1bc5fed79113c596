// main.cpp — headless equivalent of the reference's main()/Engine::RenderLoop
// (core/main.cpp:4-27, engine.cpp:140-157).  No GLFW/GL context exists in this
// image, so the loop runs a fixed number of frames and
// dumps the last one as a PPM instead of swapping buffers.
//
//   vct_headless <model.obj> [grid=256] [width=800] [height=600] [frames=5] [out.ppm] [devices=1]
//   (devices > 1: one process drives that many GPUs through vct_create_multi)
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>

#include "assets.h"

using namespace vcthost;

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s model.obj [grid] [width] [height] [frames] [out.ppm] [devices]\n", argv[0]);
        return 2;
    }
    ConeTraceSettings s;
    if (argc > 2) s.grid = (uint32_t)std::atoi(argv[2]);
    if (argc > 3) s.width = (uint32_t)std::atoi(argv[3]);
    if (argc > 4) s.height = (uint32_t)std::atoi(argv[4]);
    const int frames = argc > 5 ? std::atoi(argv[5]) : 5;
    const std::string out = argc > 6 ? argv[6] : "vct_frame.ppm";
    if (argc > 7) s.devices = (uint32_t)std::atoi(argv[7]);
    // grid AABB = [-1,1]^3 padded by one voxel (vct.scenes.grid_for_unit_box)
    s.extent = 2.0f * s.grid / (s.grid - 2);
    for (float& a : s.aabb_min) a = -s.extent / 2;

    AssetsManager& A = AssetsManager::Instance();            // assets.cpp:22-45
    A.cameras["FPS"] = std::make_shared<Camera>(0.0f, 0.0f, 3.0f);
    auto model = std::make_shared<Model>();
    std::string err;
    if (!model->LoadObj(argv[1], &err)) {
        std::fprintf(stderr, "ERROR::OBJ:: %s\n", err.c_str());   // model.cpp:25-29
        return 1;
    }
    A.models["test"] = model;
    auto r = std::make_shared<ConeTraceRenderer>("test", s);
    A.renderers["ConeTrace"] = r;
    for (int f = 0; f < frames; ++f) {
        A.renderers["ConeTrace"]->Render();                   // engine.cpp:151
        if (!r->ok()) return 1;
        std::printf("frame %d: K4 %.3f ms, %llu cone steps, %.1f Mcone-steps/s\n", f, r->last_trace_ms(),
                    r->last_cone_steps(), r->last_cone_steps() / (r->last_trace_ms() * 1e3));
    }
    if (!r->WritePPM(out)) return 1;
    std::printf("wrote %s\n", out.c_str());
    return 0;
}
