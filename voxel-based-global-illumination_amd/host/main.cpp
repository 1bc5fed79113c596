// main.cpp — headless equivalent of the reference's main()/Engine::RenderLoop
// (core/main.cpp:4-27, engine.cpp:140-157).  No GLFW/GL context exists in this
// image, so the loop runs a fixed number of frames and
// dumps the last one as a PPM instead of swapping buffers.
//
//   vct_headless <model.obj> [grid=256] [width=800] [height=600] [frames=5] [out.ppm] [devices=1]
//                [--model=reference|identity] [--grid=fit|unit]
//   (devices > 1: one process drives that many GPUs through vct_create_multi)
//   --model: the model matrix of the reference's draw, T(0,-1.75,0) S(0.2)
//            (r_voxelization.cpp:26-29; default), or none;
//   --grid:  the cubic grid around the placed model's bounds with one voxel of
//            padding (default), or [-1,1]^3 padded by one voxel (unit-box scenes).
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

#include "assets.h"

using namespace vcthost;

int main(int argc, char** argv) {
    std::vector<std::string> pos;
    bool ref_model = true, fit_grid = true;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        if (a == "--model=reference") ref_model = true;
        else if (a == "--model=identity") ref_model = false;
        else if (a == "--grid=fit") fit_grid = true;
        else if (a == "--grid=unit") fit_grid = false;
        else if (a.rfind("--", 0) == 0) { std::fprintf(stderr, "unknown option %s\n", a.c_str()); return 2; }
        else pos.push_back(a);
    }
    if (pos.empty()) {
        std::fprintf(stderr, "usage: %s model.obj [grid] [width] [height] [frames] [out.ppm] [devices] "
                             "[--model=reference|identity] [--grid=fit|unit]\n", argv[0]);
        return 2;
    }
    ConeTraceSettings s;
    if (pos.size() > 1) s.grid = (uint32_t)std::atoi(pos[1].c_str());
    if (pos.size() > 2) s.width = (uint32_t)std::atoi(pos[2].c_str());
    if (pos.size() > 3) s.height = (uint32_t)std::atoi(pos[3].c_str());
    const int frames = pos.size() > 4 ? std::atoi(pos[4].c_str()) : 5;
    const std::string out = pos.size() > 5 ? pos[5] : "vct_frame.ppm";
    if (pos.size() > 6) s.devices = (uint32_t)std::atoi(pos[6].c_str());
    if (s.grid < 4) { std::fprintf(stderr, "grid must be >= 4\n"); return 2; }
    if (ref_model) ReferenceModelMatrix(s.model);

    AssetsManager& A = AssetsManager::Instance();            // assets.cpp:22-45
    A.cameras["FPS"] = std::make_shared<Camera>(0.0f, 0.0f, 3.0f);
    auto model = std::make_shared<Model>();
    std::string err;
    if (!model->LoadObj(pos[0], &err)) {
        std::fprintf(stderr, "ERROR::OBJ:: %s\n", err.c_str());   // model.cpp:25-29
        return 1;
    }
    for (const std::string& e : model->texture_errors)            // model.cpp:219-223
        std::printf("Texture failed to load at path: %s\n", e.c_str());
    std::printf("%zu diffuse maps\n", model->textures.size());
    float lo[3], hi[3];
    Model placed = *model;
    placed.Transform(s.model);
    if (fit_grid && placed.Bounds(lo, hi)) {
        GridForBounds(lo, hi, s.grid, s.aabb_min, &s.extent);
    } else {   // [-1,1]^3 padded by one voxel (vct.scenes.grid_for_unit_box)
        s.extent = 2.0f * s.grid / (s.grid - 2);
        for (float& a : s.aabb_min) a = -s.extent / 2;
    }
    std::printf("grid %u: aabb_min %a %a %a extent %a\n", s.grid, (double)s.aabb_min[0], (double)s.aabb_min[1],
                (double)s.aabb_min[2], (double)s.extent);
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
