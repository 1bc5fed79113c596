// renderer.cpp — ConeTraceRenderer: the reference's Renderer slot driving the VCT C-ABI.
#include "renderer.h"

#include <chrono>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstring>

#include "assets.h"

namespace vcthost {

ConeTraceRenderer::ConeTraceRenderer(const std::string& model_name, const ConeTraceSettings& s)
    : model_name_(model_name), s_(s) {
    vct_config cfg{};
    cfg.n = s.grid;
    for (int k = 0; k < 3; ++k) cfg.aabb_min[k] = s.aabb_min[k];
    cfg.extent = s.extent;
    cfg.aniso = s.aniso ? 1 : 0;
    cfg.n_diffuse = s.n_diffuse;
    cfg.specular = s.specular ? 1 : 0;
    cfg.device = -1;
    if (!check(s.devices > 1 ? vct_create_multi(&cfg, s.devices, &ctx_) : vct_create(&cfg, &ctx_), "vct_create"))
        return;
    const size_t fb = (size_t)s.width * s.height * 16;
    for (auto& p : gb_)
        if (!check(vct_device_alloc(ctx_, fb, &p), "alloc gbuffer")) return;
    for (auto& p : out_)
        if (!check(vct_device_alloc(ctx_, fb, &p), "alloc output")) return;
    check(vct_device_alloc(ctx_, 8, &counter_), "alloc counter");
}

ConeTraceRenderer::~ConeTraceRenderer() {
    if (!ctx_) return;
    for (void* p : gb_) vct_device_free(ctx_, p);
    for (void* p : out_) vct_device_free(ctx_, p);
    vct_device_free(ctx_, counter_);
    vct_destroy(ctx_);
}

bool ConeTraceRenderer::check(vct_status st, const char* what) {
    if (st == VCT_OK) return true;
    status_ = st;
    error_ = std::string(what) + ": " + vct_status_string(st) + " " + (ctx_ ? vct_last_error(ctx_) : "");
    std::fprintf(stderr, "ConeTraceRenderer: %s\n", error_.c_str());   // reference style: print, continue
    return false;
}

bool ConeTraceRenderer::rebuild_scene() {
    auto model = AssetsManager::Instance().models[model_name_];
    if (!model) { error_ = "no model '" + model_name_ + "'"; return false; }
    std::vector<Vertex> v;
    std::vector<unsigned> idx, tri_mat;
    std::vector<float> kd4;
    Model placed = *model;              // the draw's model matrix, as the GL pass applies it (test.vert)
    placed.Transform(s_.model);
    placed.Flatten(v, idx, tri_mat, kd4);
    // the diffuse maps (Model::loadMaterialTextures): albedo = Kd x map in K1 and the G-buffer
    std::vector<vct_texture> tex;
    for (const Texture& t : model->textures) tex.push_back(vct_texture{t.rgba.data(), t.width, t.height});
    if (!check(vct_set_textures(ctx_, tex.data(), (uint32_t)tex.size()), "vct_set_textures")) return false;
    const std::vector<int32_t> map = model->MaterialMap();
    if (!check(vct_voxelize_textured(ctx_, v.data(), sizeof(Vertex), (uint32_t)v.size(), idx.data(),
                                     (uint32_t)idx.size(), tri_mat.data(), kd4.data(), map.data(),
                                     (uint32_t)(kd4.size() / 4), (uint32_t)offsetof(Vertex, TexCoords)),
               "vct_voxelize_textured"))
        return false;
    if (!check(vct_inject_directional(ctx_, s_.light_dir, s_.light_color), "vct_inject_directional")) return false;
    if (!check(vct_build_mips(ctx_), "vct_build_mips")) return false;
    scene_dirty_ = false;
    return true;
}

void ConeTraceRenderer::Render() {
    if (!ctx_ || status_ != VCT_OK) return;
    if (scene_dirty_ && !rebuild_scene()) return;
    auto cam = AssetsManager::Instance().ActiveCamera();
    if (!cam) return;
    const vct_camera vc = cam->ToVct();
    if (!check(vct_gbuffer_raster_device(ctx_, &vc, s_.width, s_.height, s_.roughness, (float*)gb_[0],
                                         (float*)gb_[1], (float*)gb_[2]), "G-buffer"))
        return;
    unsigned long long zero = 0;
    if (!check(vct_memcpy(ctx_, counter_, &zero, 8, 0), "reset counter")) return;
    vct_trace_args a{};
    a.pos4 = (const float*)gb_[0];
    a.nrm4 = (const float*)gb_[1];
    a.alb4 = (const float*)gb_[2];
    a.width = s_.width;
    a.height = s_.height;
    for (int k = 0; k < 3; ++k) a.eye[k] = cam->Position[k];
    a.diffuse4 = (float*)out_[0];
    a.spec4 = (float*)out_[1];
    a.cone_steps = (unsigned long long*)counter_;
    auto t0 = std::chrono::steady_clock::now();
    if (!check(vct_trace_device(ctx_, &a), "vct_trace_device")) return;
    if (!check(vct_synchronize(ctx_), "sync")) return;
    last_ms_ = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    check(vct_memcpy(ctx_, &last_steps_, counter_, 8, 1), "read counter");
}

bool ConeTraceRenderer::WritePPM(const std::string& path) {
    // row f3: composite + present on the device (include/vct.h vct_composite_device), then dump
    if (!ctx_) return false;
    const size_t px = (size_t)s_.width * s_.height;
    void* rgba = nullptr;
    if (!check(vct_device_alloc(ctx_, px * 4, &rgba), "alloc rgba8")) return false;
    std::vector<uint32_t> img(px);
    const bool ok = check(vct_composite_device(ctx_, (const float*)gb_[0], (const float*)gb_[1], (const float*)gb_[2],
                                               (const float*)out_[0], (const float*)out_[1], s_.width, s_.height,
                                               s_.light_dir, s_.light_color, nullptr, (uint32_t*)rgba),
                          "vct_composite_device") &&
                    check(vct_memcpy(ctx_, img.data(), rgba, px * 4, 1), "download rgba8");
    vct_device_free(ctx_, rgba);
    if (!ok) return false;
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    std::fprintf(f, "P6\n%u %u\n255\n", s_.width, s_.height);
    std::vector<unsigned char> row(s_.width * 3);
    for (uint32_t y = 0; y < s_.height; ++y) {
        for (uint32_t x = 0; x < s_.width; ++x) {               // row 0 = top (the G-buffer's ray rule)
            const uint32_t c = img[(size_t)y * s_.width + x];
            row[3 * x] = (unsigned char)(c & 255);
            row[3 * x + 1] = (unsigned char)((c >> 8) & 255);
            row[3 * x + 2] = (unsigned char)((c >> 16) & 255);
        }
        std::fwrite(row.data(), 1, row.size(), f);
    }
    std::fclose(f);
    return true;
}

}  // namespace vcthost
