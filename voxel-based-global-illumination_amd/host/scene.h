// scene.h — host-side scene format of the reference, feeding K1 (voxelization).
//
// Mirrors include/stdafx.h:36-42 (`struct Vertex`: Position, Normal,
// TexCoords, Tangent, Bitangent = 56 bytes, attribute offsets as
// mesh.cpp:43-55), scene/material.h:5-18 (`Material` with Ka/Kd/Ks) and the
// Mesh/Model split of scene/mesh.h:7-26, model.h:8-42.  The reference loads
// models with assimp (model.cpp:21-148); assimp is not available on Linux in
// this image (its vendored lib is an MSVC import library), so Model::LoadObj is
// a small Wavefront OBJ/MTL reader covering what the VCT path consumes
// (see scene.cpp for the assimp 3.3 rules it reproduces).
#pragma once
#include <array>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace vcthost {

struct Vertex {                    // 56 bytes, stdafx.h:36-42
    float Position[3];
    float Normal[3];
    float TexCoords[2];
    float Tangent[3];
    float Bitangent[3];
};
static_assert(sizeof(Vertex) == 56, "reference Vertex layout");

struct Texture {                   // stdafx.h:30-34 (GL id -> the decoded texels the C-ABI uploads)
    std::string type;              // "texture_diffuse" (model.cpp:58)
    std::string path;              // as written in the .mtl (the dedup key, model.cpp:160-166)
    uint32_t width = 0, height = 0;
    std::vector<uint8_t> rgba;     // RGBA8, row 0 = the image's top row (vct_texture)
};

struct Material {                  // material.h:5-18
    std::string name;
    std::array<float, 4> Ka{0, 0, 0, 1};
    std::array<float, 4> Kd{1, 1, 1, 1};
    std::array<float, 4> Ks{0, 0, 0, 1};
    std::string diffuse_map;       // map_Kd of the .mtl ("" = none); the only map the VCT path reads
    std::vector<int> diffuseMaps;  // indices into Model::textures (loadMaterialTextures, model.cpp:57)
};

struct Mesh {                      // mesh.h:7-26 CPU copies (vertices, indices, material)
    std::vector<Vertex> vertices;
    std::vector<unsigned> indices;
    int material = 0;
};

class Model {                      // model.h:8-42
public:
    std::vector<Mesh> meshes;
    std::vector<Material> materials;
    std::vector<Texture> textures;   // model.h `textures`: every map loaded once, by path
    std::string directory;           // the model file's directory (model.cpp:30)
    std::vector<std::string> texture_errors;   // maps that failed to load (model.cpp:221 prints them)

    // Wavefront OBJ (+ mtllib).  Returns false and fills `err` on failure.  With
    // load_textures, each material's diffuse map is decoded from `directory` (PNG).
    bool LoadObj(const std::string& path, std::string* err, bool load_textures = true);

    // loadMaterialTextures for the diffuse maps (model.cpp:150-186): a path already in
    // `textures` is shared; a map that fails to decode is reported in texture_errors and
    // the material keeps Kd alone (the reference would sample an incomplete texture).
    void LoadTextures();

    // Apply a 4x4 column-major model matrix (r_voxelization.cpp:26-29 style):
    // p' = (m0 x + m4 y + m8 z + m12, ...), in that float order.
    void Transform(const float m[16]);

    // Axis-aligned bounds of every vertex position (false when the model is empty).
    bool Bounds(float lo[3], float hi[3]) const;

    // Flatten to the C-ABI arrays: vertices, indices, per-triangle material, Kd table.
    void Flatten(std::vector<Vertex>& v, std::vector<unsigned>& idx, std::vector<unsigned>& tri_mat,
                 std::vector<float>& kd4) const;
    // material_map of vct_voxelize_textured: each material's first diffuse map (the one
    // the reference binds as texture_diffuse1) as an index into `textures`, or -1.
    std::vector<int32_t> MaterialMap() const;
};

// The model matrix VoxelizationRenderer::Render draws with:
// glm::scale(glm::translate(mat4(1), (0, -1.75, 0)), (0.2, 0.2, 0.2)), column-major
// (r_voxelization.cpp:26-29; values pinned by tests/golden/ref_camera.json).
void ReferenceModelMatrix(float m[16]);

// Cubic grid around [lo, hi] with one voxel of padding on every side at resolution n:
// edge E = max extent * n / (n - 2), min corner = centre - E / 2.
void GridForBounds(const float lo[3], const float hi[3], uint32_t n, float aabb_min[3], float* extent);

}  // namespace vcthost
