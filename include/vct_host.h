/* vct_host.h — C entry points of the host scene loader (host/scene.cpp).
 *
 * The reference loads models with assimp inside Model::loadModel
 * (assets/code/scene/model.cpp:21-36: ReadFile with aiProcess_Triangulate |
 * aiProcess_FlipUVs | aiProcess_CalcTangentSpace) and flattens each aiMesh into
 * a vector<Vertex> + vector<GLuint> + Material (model.cpp:38-148).  These
 * functions expose the same result for a Wavefront OBJ/MTL file: per mesh the
 * 56-byte Vertex array (stdafx.h:36-42) and u32 triangle indices, and per
 * material Ka/Kd/Ks as (r, g, b, 1) (model.cpp:48-53).  CPU only; no HIP.
 */
#ifndef VCT_HOST_H
#define VCT_HOST_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct vcth_model vcth_model;

/* Load an OBJ (+ mtllib).  Returns 0, or -1 with a message in err (model.cpp:25-29 prints one). */
int vcth_load_obj(const char* path, vcth_model** out, char* err, int errlen);
uint32_t vcth_num_meshes(const vcth_model* m);
uint32_t vcth_num_materials(const vcth_model* m);
/* Mesh i: verts = n_verts x 56-byte Vertex, idx = n_idx u32 (triangles), material index. */
int vcth_mesh(const vcth_model* m, uint32_t i, const void** verts, uint32_t* n_verts, const uint32_t** idx,
              uint32_t* n_idx, uint32_t* material);
/* Material i: name, Ka/Kd/Ks (r, g, b, 1). */
int vcth_material(const vcth_model* m, uint32_t i, const char** name, float ka[4], float kd[4], float ks[4]);
/* Material i's diffuse map: the map_Kd path of the .mtl ("" = none) and its index in
 * the model's texture list (-1: none, or it failed to load).  The model loads each
 * diffuse map once per path (Model::loadMaterialTextures, model.cpp:150-186). */
int vcth_material_diffuse_map(const vcth_model* m, uint32_t i, const char** path, int32_t* texture);
uint32_t vcth_num_textures(const vcth_model* m);
/* Texture i: RGBA8 texels (row 0 = the image's top row, 1/3-channel images expanded as
 * GL_RED / GL_RGB sample), size, .mtl path: the vct_texture of vct_set_textures. */
int vcth_texture(const vcth_model* m, uint32_t i, const uint8_t** rgba8, uint32_t* width, uint32_t* height,
                 const char** path);
/* Maps that failed to load, "path: reason" (TextureFromFile prints them, model.cpp:219-223). */
uint32_t vcth_num_texture_errors(const vcth_model* m);
const char* vcth_texture_error(const vcth_model* m, uint32_t i);
/* PNG decode as stbi_load(file, &w, &h, &comp, 0) (model.cpp:197): *data = h rows of
 * w * comp bytes (release with vcth_free_image).  Returns 0, or -1 with a message. */
int vcth_decode_png(const uint8_t* file, size_t bytes, uint8_t** data, uint32_t* width, uint32_t* height, int* comp,
                    char* err, int errlen);
void vcth_free_image(uint8_t* data);
void vcth_free(vcth_model* m);
/* Apply a column-major 4x4 model matrix to every vertex position (host Model::Transform). */
void vcth_transform(vcth_model* m, const float mat[16]);
/* Vertex-position bounds; returns 0, or -1 for an empty model. */
int vcth_bounds(const vcth_model* m, float lo[3], float hi[3]);

/* The reference's model matrix, r_voxelization.cpp:26-29 (column-major). */
void vcth_reference_model_matrix(float mat[16]);
/* Cubic grid around [lo, hi], one voxel of padding per side at resolution n. */
void vcth_grid_for_bounds(const float lo[3], const float hi[3], uint32_t n, float aabb_min[3], float* extent);

/* The host FPS camera (host/camera.cpp = the reference Camera, scene/camera.cpp)
 * built from init = (pos x, y, z, yaw, pitch), then n_ops operations: kind[i] in
 * 'm' ProcessMouseMovement(a, b), 's' ProcessMouseScroll(a), 'f' / 'b' / 'l' / 'r'
 * ProcessKeyboard(FORWARD / BACKWARD / LEFT / RIGHT, a).  out[15] = Position,
 * Front, Right, Up, Yaw, Pitch, Zoom. */
int vcth_camera_eval(const float init[5], const char* kinds, const float* a, const float* b, int n_ops, float out[15]);

#ifdef __cplusplus
}
#endif
#endif
