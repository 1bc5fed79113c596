// r_conetrace.h -- the MI355X voxel-cone-traced GI path as a reference Renderer.
//
// A new file for the reference's assets/code/renderer/ (next to r_voxelization.h).  It
// compiles against the reference's own, unmodified renderer.h, core/assets.h,
// scene/camera.h and include/stdafx.h (tests/test_integration_binding.py) and calls the
// C-ABI of include/vct.h (libvct_hip.so) plus the OBJ loader of include/vct_host.h
// (libvct_host.so), nothing else.  Registered like VoxelizationRenderer
// (assets/code/core/assets.cpp:44) and called once per frame by the engine loop
// (assets/code/core/engine.cpp:151).
#pragma once
#include "renderer.h"

#include <string>
#include <vector>

#include "vct.h"
#include "vct_host.h"

class ConeTraceRenderer : public Renderer
{
public:
	// model_path: the file the registry's Model was built from (assets.cpp:29).  Model keeps
	// its meshes private (scene/model.h), so the renderer loads the same file itself through
	// vct_host.h (assimp 3.3's result under model.cpp:24's flags, bit for bit).
	explicit ConeTraceRenderer(const std::string& model_path, unsigned grid = 256);
	~ConeTraceRenderer();

	virtual void Render();

	// a new directional light: the next frame relights (K2 + K3) without voxelizing again
	void SetLight(const float dir_to_light[3], const float color[3]);

	bool Ok() const { return ok_; }

private:
	bool Check(vct_status st, const char* what);
	bool BuildScene();
	bool Resize(unsigned width, unsigned height);
	void Present();

	std::string path_;
	unsigned grid_;
	vct_ctx* ctx_ = nullptr;
	void* gbuf_[3] = {nullptr, nullptr, nullptr};   // device G-buffer: pos, normal, albedo + roughness
	void* out_[2] = {nullptr, nullptr};              // device diffuse + AO, specular
	void* rgba_ = nullptr;                           // device RGBA8 of the composite
	std::vector<unsigned> pixels_;                   // host copy handed to GL
	unsigned width_ = 0, height_ = 0;
	float light_dir_[3] = {0.3f, 1.0f, 0.2f};        // SURVEY 8d canonical light
	float light_color_[3] = {1.0f, 1.0f, 1.0f};
	bool scene_ready_ = false, light_dirty_ = true, ok_ = true;
	unsigned tex_ = 0, fbo_ = 0;                     // GL objects of the present blit
};
