// scene_capi.cpp — include/vct_host.h over vcthost::Model (CPU only).
#include <cstring>
#include <new>

#include "../../include/vct_host.h"
#include "scene.h"

struct vcth_model {
    vcthost::Model m;
};

extern "C" {

int vcth_load_obj(const char* path, vcth_model** out, char* err, int errlen) {
    if (!path || !out) return -1;
    *out = nullptr;
    vcth_model* h = new (std::nothrow) vcth_model();
    if (!h) return -1;
    std::string e;
    if (!h->m.LoadObj(path, &e)) {
        if (err && errlen > 0) {
            std::strncpy(err, e.c_str(), (size_t)errlen - 1);
            err[errlen - 1] = 0;
        }
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

void vcth_free(vcth_model* m) { delete m; }

}  // extern "C"
