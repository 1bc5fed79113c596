// scene_capi.cpp — include/vct_host.h over vcthost::Model (CPU only).
#include <cstdlib>
#include <cstring>
#include <exception>
#include <new>
#include <string>

#include "../../include/vct_host.h"
#include "camera.h"
#include "png.h"
#include "scene.h"

struct vcth_model {
    vcthost::Model m;
};

extern "C" {

namespace {
void put_err(char* err, int errlen, const std::string& e) {
    if (err && errlen > 0) {
        std::strncpy(err, e.c_str(), (size_t)errlen - 1);
        err[errlen - 1] = 0;
    }
}
}  // namespace

// No C++ exception crosses the C ABI: an allocation failure (std::bad_alloc /
// std::length_error from a hostile file) becomes -1 with the reason in err.
int vcth_load_obj(const char* path, vcth_model** out, char* err, int errlen) {
    if (!path || !out) return -1;
    *out = nullptr;
    vcth_model* h = nullptr;
    try {
        h = new vcth_model();
        std::string e;
        if (!h->m.LoadObj(path, &e)) {
            put_err(err, errlen, e);
            delete h;
            return -1;
        }
    } catch (const std::exception& ex) {
        put_err(err, errlen, std::string("vcth_load_obj: ") + ex.what());
        delete h;
        return -1;
    }
    *out = h;
    return 0;
}

uint32_t vcth_num_meshes(const vcth_model* m) { return m ? (uint32_t)m->m.meshes.size() : 0u; }
uint32_t vcth_num_materials(const vcth_model* m) { return m ? (uint32_t)m->m.materials.size() : 0u; }

int vcth_mesh(const vcth_model* m, uint32_t i, const void** verts, uint32_t* n_verts, const uint32_t** idx,
              uint32_t* n_idx, uint32_t* material) {
    if (!m || i >= m->m.meshes.size()) return -1;
    const vcthost::Mesh& me = m->m.meshes[i];
    if (verts) *verts = me.vertices.data();
    if (n_verts) *n_verts = (uint32_t)me.vertices.size();
    if (idx) *idx = me.indices.data();
    if (n_idx) *n_idx = (uint32_t)me.indices.size();
    if (material) *material = (uint32_t)me.material;
    return 0;
}

int vcth_material(const vcth_model* m, uint32_t i, const char** name, float ka[4], float kd[4], float ks[4]) {
    if (!m || i >= m->m.materials.size()) return -1;
    const vcthost::Material& mt = m->m.materials[i];
    if (name) *name = mt.name.c_str();
    for (int k = 0; k < 4; ++k) {
        if (ka) ka[k] = mt.Ka[k];
        if (kd) kd[k] = mt.Kd[k];
        if (ks) ks[k] = mt.Ks[k];
    }
    return 0;
}

int vcth_material_diffuse_map(const vcth_model* m, uint32_t i, const char** path, int32_t* texture) {
    if (!m || i >= m->m.materials.size()) return -1;
    const vcthost::Material& mt = m->m.materials[i];
    if (path) *path = mt.diffuse_map.c_str();
    if (texture) *texture = mt.diffuseMaps.empty() ? -1 : mt.diffuseMaps[0];
    return 0;
}

uint32_t vcth_num_textures(const vcth_model* m) { return m ? (uint32_t)m->m.textures.size() : 0u; }

int vcth_texture(const vcth_model* m, uint32_t i, const uint8_t** rgba8, uint32_t* width, uint32_t* height,
                 const char** path) {
    if (!m || i >= m->m.textures.size()) return -1;
    const vcthost::Texture& t = m->m.textures[i];
    if (rgba8) *rgba8 = t.rgba.data();
    if (width) *width = t.width;
    if (height) *height = t.height;
    if (path) *path = t.path.c_str();
    return 0;
}

uint32_t vcth_num_texture_errors(const vcth_model* m) { return m ? (uint32_t)m->m.texture_errors.size() : 0u; }

const char* vcth_texture_error(const vcth_model* m, uint32_t i) {
    return (m && i < m->m.texture_errors.size()) ? m->m.texture_errors[i].c_str() : nullptr;
}

int vcth_decode_png(const uint8_t* file, size_t bytes, uint8_t** data, uint32_t* width, uint32_t* height, int* comp,
                    char* err, int errlen) {
    if (!file || !data || !width || !height || !comp) return -1;
    *data = nullptr;
    vcthost::PngImage img;
    std::string e;
    try {
        if (!vcthost::DecodePng(file, bytes, &img, &e)) {
            put_err(err, errlen, e);
            return -1;
        }
    } catch (const std::exception& ex) {
        put_err(err, errlen, std::string("vcth_decode_png: ") + ex.what());
        return -1;
    }
    uint8_t* out = (uint8_t*)std::malloc(img.data.size() ? img.data.size() : 1);
    if (!out) return -1;
    std::memcpy(out, img.data.data(), img.data.size());
    *data = out;
    *width = img.width;
    *height = img.height;
    *comp = img.comp;
    return 0;
}

void vcth_free_image(uint8_t* data) { std::free(data); }

void vcth_free(vcth_model* m) { delete m; }


void vcth_transform(vcth_model* m, const float mat[16]) {
    if (m && mat) m->m.Transform(mat);
}

int vcth_bounds(const vcth_model* m, float lo[3], float hi[3]) {
    return (m && lo && hi && m->m.Bounds(lo, hi)) ? 0 : -1;
}

void vcth_reference_model_matrix(float mat[16]) {
    if (mat) vcthost::ReferenceModelMatrix(mat);
}

void vcth_grid_for_bounds(const float lo[3], const float hi[3], uint32_t n, float aabb_min[3], float* extent) {
    if (lo && hi && aabb_min && extent && n > 2) vcthost::GridForBounds(lo, hi, n, aabb_min, extent);
}

int vcth_camera_eval(const float init[5], const char* kinds, const float* a, const float* b, int n_ops, float out[15]) {
    if (!init || !out || (n_ops > 0 && (!kinds || !a || !b))) return -1;
    vcthost::Camera c(init[0], init[1], init[2], init[3], init[4]);
    for (int i = 0; i < n_ops; ++i) {
        switch (kinds[i]) {
            case 'm': c.ProcessMouseMovement(a[i], b[i]); break;
            case 's': c.ProcessMouseScroll(a[i]); break;
            case 'f': c.ProcessKeyboard(vcthost::FORWARD, a[i]); break;
            case 'b': c.ProcessKeyboard(vcthost::BACKWARD, a[i]); break;
            case 'l': c.ProcessKeyboard(vcthost::LEFT, a[i]); break;
            case 'r': c.ProcessKeyboard(vcthost::RIGHT, a[i]); break;
            default: return -1;
        }
    }
    for (int k = 0; k < 3; ++k) {
        out[k] = c.Position[k];
        out[3 + k] = c.Front[k];
        out[6 + k] = c.Right[k];
        out[9 + k] = c.Up[k];
    }
    out[12] = c.Yaw;
    out[13] = c.Pitch;
    out[14] = c.Zoom;
    return 0;
}
}  // extern "C"
