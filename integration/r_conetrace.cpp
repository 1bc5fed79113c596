// r_conetrace.cpp -- ConeTraceRenderer (r_conetrace.h): the reference's per-frame Renderer
// slot driving the MI355X VCT path through include/vct.h.
//
// Replaces the forward GL draw of VoxelizationRenderer::Render
// (assets/code/renderer/r_voxelization.cpp:4-35) by: K1 voxelize (once per scene) ->
// K2 inject + K3 mips (once per light) -> per frame the G-buffer from the active camera,
// K4 cone trace, composite to RGBA8 on the GPU, and a blit into the default framebuffer.
// State is pulled from the reference's singletons the way r_voxelization.cpp does
// (Engine::Instance()->Window() for the size, Camera::Active() for the view); errors are
// printed and the frame skipped, the reference's only error channel (model.cpp:25-29).
#include "stdafx.h"
#include "r_conetrace.h"

#include <cstddef>

static_assert(sizeof(Vertex) == 56, "vct_voxelize reads the reference's 56-byte Vertex (stdafx.h)");

ConeTraceRenderer::ConeTraceRenderer(const std::string& model_path, unsigned grid)
	: path_(model_path), grid_(grid)
{
}

ConeTraceRenderer::~ConeTraceRenderer()
{
	if (ctx_)
	{
		for (void* p : gbuf_) vct_device_free(ctx_, p);
		for (void* p : out_) vct_device_free(ctx_, p);
		vct_device_free(ctx_, rgba_);
		vct_destroy(ctx_);
	}
	if (fbo_) glDeleteFramebuffers(1, &fbo_);
	if (tex_) glDeleteTextures(1, &tex_);
}

void ConeTraceRenderer::SetLight(const float dir_to_light[3], const float color[3])
{
	for (int k = 0; k < 3; ++k)
	{
		light_dir_[k] = dir_to_light[k];
		light_color_[k] = color[k];
	}
	light_dirty_ = true;
}

bool ConeTraceRenderer::Check(vct_status st, const char* what)
{
	if (st == VCT_OK) return true;
	cout << "ERROR::VCT::" << what << ": " << vct_status_string(st) << " " << (ctx_ ? vct_last_error(ctx_) : "")
	     << endl;
	ok_ = false;
	return false;
}

bool ConeTraceRenderer::BuildScene()
{
	vcth_model* m = nullptr;
	char err[512];
	if (vcth_load_obj(path_.c_str(), &m, err, sizeof err) != 0)
	{
		cout << "ERROR::VCT::LOAD " << err << endl;
		ok_ = false;
		return false;
	}
	// the draw's model matrix (r_voxelization.cpp:26-29), applied to the positions as
	// test.vert applies it to gl_Position
	glm::mat4 modelM = glm::mat4(1.0f);
	modelM = glm::translate(modelM, glm::vec3(0.0f, -1.75f, 0.0f));
	modelM = glm::scale(modelM, glm::vec3(0.2f, 0.2f, 0.2f));
	vcth_transform(m, glm::value_ptr(modelM));
	float lo[3], hi[3];
	if (vcth_bounds(m, lo, hi) != 0)
	{
		cout << "ERROR::VCT::LOAD empty model " << path_ << endl;
		vcth_free(m);
		ok_ = false;
		return false;
	}
	vct_config cfg{};
	cfg.n = grid_;
	vcth_grid_for_bounds(lo, hi, grid_, cfg.aabb_min, &cfg.extent);   // one voxel of padding per side
	cfg.aniso = 1;
	cfg.n_diffuse = 9;
	cfg.specular = 1;
	cfg.device = -1;
	if (!Check(vct_create(&cfg, &ctx_), "vct_create"))
	{
		vcth_free(m);
		return false;
	}
	// Model::loadMeshes' meshes as one vertex / index / per-triangle material list
	vector<Vertex> verts;
	vector<uint32_t> idx, tri_mat;
	for (uint32_t i = 0; i < vcth_num_meshes(m); ++i)
	{
		const void* v = nullptr;
		const uint32_t* ix = nullptr;
		uint32_t nv = 0, ni = 0, mat = 0;
		vcth_mesh(m, i, &v, &nv, &ix, &ni, &mat);
		const uint32_t base = (uint32_t)verts.size();
		const Vertex* vv = static_cast<const Vertex*>(v);
		verts.insert(verts.end(), vv, vv + nv);
		for (uint32_t k = 0; k < ni; ++k) idx.push_back(base + ix[k]);
		tri_mat.insert(tri_mat.end(), ni / 3, mat);
	}
	// Model::loadMaterials: Kd per material, its diffuse map (loadMaterialTextures)
	vector<float> kd;
	vector<int32_t> map;
	for (uint32_t i = 0; i < vcth_num_materials(m); ++i)
	{
		const char* name = nullptr;
		const char* mpath = nullptr;
		float ka[4], kd4[4], ks[4];
		int32_t tex = -1;
		vcth_material(m, i, &name, ka, kd4, ks);
		vcth_material_diffuse_map(m, i, &mpath, &tex);
		kd.insert(kd.end(), kd4, kd4 + 4);
		map.push_back(tex);
	}
	vector<vct_texture> textures;
	for (uint32_t i = 0; i < vcth_num_textures(m); ++i)
	{
		vct_texture t{};
		const char* tpath = nullptr;
		vcth_texture(m, i, &t.rgba8, &t.width, &t.height, &tpath);
		textures.push_back(t);
	}
	for (uint32_t i = 0; i < vcth_num_texture_errors(m); ++i)
		cout << "Texture failed to load at path: " << vcth_texture_error(m, i) << endl;   // model.cpp:221
	const bool ok = Check(vct_set_textures(ctx_, textures.data(), (uint32_t)textures.size()), "vct_set_textures") &&
	                Check(vct_voxelize_textured(ctx_, verts.data(), sizeof(Vertex), (uint32_t)verts.size(), idx.data(),
	                                            (uint32_t)idx.size(), tri_mat.data(), kd.data(), map.data(),
	                                            (uint32_t)map.size(), (uint32_t)offsetof(Vertex, TexCoords)),
	                      "vct_voxelize_textured");
	vcth_free(m);   // both calls are synchronous: the device holds its own copies
	return ok;
}

bool ConeTraceRenderer::Resize(unsigned width, unsigned height)
{
	for (void*& p : gbuf_) { vct_device_free(ctx_, p); p = nullptr; }
	for (void*& p : out_) { vct_device_free(ctx_, p); p = nullptr; }
	vct_device_free(ctx_, rgba_);
	rgba_ = nullptr;
	const size_t px = (size_t)width * height;
	for (void*& p : gbuf_)
		if (!Check(vct_device_alloc(ctx_, px * 16, &p), "alloc G-buffer")) return false;
	for (void*& p : out_)
		if (!Check(vct_device_alloc(ctx_, px * 16, &p), "alloc outputs")) return false;
	if (!Check(vct_device_alloc(ctx_, px * 4, &rgba_), "alloc RGBA8")) return false;
	pixels_.assign(px, 0u);
	if (!tex_) glGenTextures(1, &tex_);
	glBindTexture(GL_TEXTURE_2D, tex_);
	glTexImage2D(GL_TEXTURE_2D, 0, GL_RGBA8, (GLsizei)width, (GLsizei)height, 0, GL_RGBA, GL_UNSIGNED_BYTE, nullptr);
	if (!fbo_) glGenFramebuffers(1, &fbo_);
	glBindFramebuffer(GL_READ_FRAMEBUFFER, fbo_);
	glFramebufferTexture2D(GL_READ_FRAMEBUFFER, GL_COLOR_ATTACHMENT0, GL_TEXTURE_2D, tex_, 0);
	glBindFramebuffer(GL_READ_FRAMEBUFFER, 0);
	width_ = width;
	height_ = height;
	return true;
}

void ConeTraceRenderer::Present()
{
	glBindTexture(GL_TEXTURE_2D, tex_);
	glTexSubImage2D(GL_TEXTURE_2D, 0, 0, 0, (GLsizei)width_, (GLsizei)height_, GL_RGBA, GL_UNSIGNED_BYTE,
	                pixels_.data());
	glBindFramebuffer(GL_READ_FRAMEBUFFER, fbo_);
	glBindFramebuffer(GL_DRAW_FRAMEBUFFER, 0);
	// the composite's row 0 is the top of the image, GL's the bottom: the blit flips
	glBlitFramebuffer(0, 0, (GLint)width_, (GLint)height_, 0, (GLint)height_, (GLint)width_, 0, GL_COLOR_BUFFER_BIT,
	                  GL_NEAREST);
	glBindFramebuffer(GL_READ_FRAMEBUFFER, 0);
}

void ConeTraceRenderer::Render()
{
	// the window size, as r_voxelization.cpp:16-17 takes it for the projection
	GLint width, height;
	glfwGetWindowSize(Engine::Instance()->Window(), &width, &height);
	if (!ok_ || width <= 0 || height <= 0) return;
	if (!scene_ready_ && !(scene_ready_ = BuildScene())) return;
	if (((unsigned)width != width_ || (unsigned)height != height_) && !Resize((unsigned)width, (unsigned)height))
		return;
	if (light_dirty_)
	{
		// a relit frame: K2 + K3 only (a relight build keeps K1's occupancy work)
		if (!Check(vct_inject_directional(ctx_, light_dir_, light_color_), "vct_inject_directional") ||
		    !Check(vct_build_mips(ctx_), "vct_build_mips"))
			return;
		light_dirty_ = false;
	}
	// the active camera in the reference's conventions: lookAt (camera.cpp:24-27),
	// perspective(radians(Zoom), w / h, 0.1, 100) (r_voxelization.cpp:18)
	auto& cam = Camera::Active();
	vct_camera vc{};
	for (int k = 0; k < 3; ++k)
	{
		vc.position[k] = cam->Position[k];
		vc.front[k] = cam->Front[k];
		vc.up[k] = cam->Up[k];
		vc.right[k] = cam->Right[k];
	}
	vc.zoom_deg = cam->Zoom;
	vc.near_plane = 0.1f;
	vc.far_plane = 100.0f;
	if (!Check(vct_gbuffer_raster_device(ctx_, &vc, width_, height_, 0.1f, (float*)gbuf_[0], (float*)gbuf_[1],
	                                     (float*)gbuf_[2]),
	           "vct_gbuffer_raster_device"))
		return;
	vct_trace_args a{};
	a.pos4 = (const float*)gbuf_[0];
	a.nrm4 = (const float*)gbuf_[1];
	a.alb4 = (const float*)gbuf_[2];
	a.width = width_;
	a.height = height_;
	for (int k = 0; k < 3; ++k) a.eye[k] = cam->Position[k];
	a.diffuse4 = (float*)out_[0];
	a.spec4 = (float*)out_[1];
	if (!Check(vct_trace_device(ctx_, &a), "vct_trace_device")) return;
	// direct + albedo x indirect + specular, tone-mapped to RGBA8 on the GPU (background =
	// r_voxelization.cpp:8's clear colour), then one copy to the host for GL
	if (!Check(vct_composite_device(ctx_, a.pos4, a.nrm4, a.alb4, a.diffuse4, a.spec4, width_, height_, light_dir_,
	                                light_color_, nullptr, (uint32_t*)rgba_),
	           "vct_composite_device") ||
	    !Check(vct_memcpy(ctx_, pixels_.data(), rgba_, pixels_.size() * 4, 1), "download RGBA8"))
		return;
	Present();
}
