// renderer.h — the reference's renderer plug-in slot and the VCT implementation.
//
// `Renderer` is assets/code/renderer/renderer.h:3-10 unchanged in shape: one
// argument-less virtual called once per frame (engine.cpp:151).
// `ConeTraceRenderer` is the drop-in that replaces the forward GL draw of
// VoxelizationRenderer::Render (r_voxelization.cpp:4-35) with the C-ABI of
// include/vct.h: on the first frame (or when the scene/light changes) it runs
// K1 voxelize -> K2 inject -> K3 mips, and every frame it builds the G-buffer
// from the active camera and runs K4.  State is pulled from the registry the
// way the reference pulls programs/models/camera from its singletons.
#pragma once
#include <string>
#include <vector>

#include "vct.h"

namespace vcthost {

class Renderer {
public:
    virtual ~Renderer() = default;
    virtual void Render() = 0;
};

struct ConeTraceSettings {
    uint32_t grid = 256;
    uint32_t width = 800, height = 600;   // reference window size, engine.cpp:52
    uint32_t n_diffuse = 9;
    bool specular = true;
    bool aniso = true;
    float light_dir[3] = {0.3f, 1.0f, 0.2f};
    float light_color[3] = {1.0f, 1.0f, 1.0f};
    float roughness = 0.1f;
    float aabb_min[3] = {-1.0f, -1.0f, -1.0f};
    float extent = 2.0f;
    uint32_t devices = 1;                 // > 1: one context over that many GPUs (vct_create_multi)
    // model matrix applied to the model's vertices before K1, column-major; main.cpp
    // sets the reference's T(0,-1.75,0) S(0.2) (r_voxelization.cpp:26-29) by default
    float model[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
};

class ConeTraceRenderer : public Renderer {
public:
    ConeTraceRenderer(const std::string& model_name, const ConeTraceSettings& s);
    ~ConeTraceRenderer() override;
    void Render() override;

    void MarkSceneDirty() { scene_dirty_ = true; }
    bool ok() const { return status_ == VCT_OK; }
    const std::string& error() const { return error_; }
    double last_trace_ms() const { return last_ms_; }
    unsigned long long last_cone_steps() const { return last_steps_; }
    // composite + present (vct_composite_device: direct + albedo * indirect + specular) -> binary PPM
    bool WritePPM(const std::string& path);

private:
    bool check(vct_status s, const char* what);
    bool rebuild_scene();

    std::string model_name_;
    ConeTraceSettings s_;
    vct_ctx* ctx_ = nullptr;
    void* gb_[3] = {nullptr, nullptr, nullptr};
    void* out_[2] = {nullptr, nullptr};
    void* counter_ = nullptr;
    bool scene_dirty_ = true;
    vct_status status_ = VCT_OK;
    std::string error_;
    double last_ms_ = 0.0;
    unsigned long long last_steps_ = 0;
};

}  // namespace vcthost
