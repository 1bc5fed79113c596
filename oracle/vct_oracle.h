/*
 * vct_oracle.h — CPU restatement of the VCT hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity checker for the HIP path in
 * voxel-based-global-illumination_amd/csrc.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.  The product never links it.
 *
 * Provenance.  The reference repository has no implementation of this path
 * (`VoxelizationProgram` is empty, p_voxelization.h:4-7;
 * `VoxelizationRenderer::Render` is a forward textured draw,
 * r_voxelization.cpp:4-35).  The semantics are SURVEY.md Appendix A as pinned
 * by include/vct_spec.h.  There is no reference output to compare with, so
 * parity is pinned by closed-form known-answer tests (tests/test_oracle_kat.py)
 * and by golden vectors this oracle generated (tests/golden/).  In the strict
 * sense of the task statement this oracle is "parity unpinned" against the
 * reference itself: nothing in the reference computes these numbers.
 *
 * Every array is plain row-major float / integer data:
 *   grid volumes  : [z][y][x][4] floats, linear index x + n*(y + n*z)
 *   mip pyramid   : levels 1..L concatenated; level l holds F(l) volumes of
 *                   n_l^3 texels (F = 6 anisotropic faces +X,-X,+Y,-Y,+Z,-Z, or 1)
 *   G-buffer      : [h][w][4] floats
 */
#ifndef VCT_ORACLE_H
#define VCT_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* floats in the level 1..L part of the pyramid */
size_t vo_pyramid_floats(uint32_t n, int aniso);
/* float offset of level l (1..L) inside the pyramid array */
size_t vo_level_offset(uint32_t n, int aniso, uint32_t level);

/* K1 (A.2): conservative SAT voxelization into fixed-point sums.
 * pos: vertex positions, vertex i at (const char*)verts + i*stride (3 floats).
 * sums6: [n^3][6] int64 (albedo rgb, normal xyz), counts: [n^3] uint32.
 * Arrays are accumulated into (caller zeroes them).  Returns 0 / -1 on bad index. */
int vo_voxelize(uint32_t n, const float g0[3], float extent,
                const void* verts, uint32_t stride, uint32_t n_verts,
                const uint32_t* idx, uint32_t n_idx,
                const uint32_t* tri_mat, const float* kd4, uint32_t n_mat,
                int64_t* sums6, uint32_t* counts);

/* Diffuse maps (include/vct_spec.h "diffuse maps"): RGBA8, row 0 = the image's top row. */
typedef struct vo_texture {
    const uint8_t* rgba8;
    uint32_t width, height;
} vo_texture;

/* T(u, v).rgb: GL_REPEAT, bilinear at the base level, texel centres at +0.5. */
void vo_tex_sample(const vo_texture* t, float u, float v, float rgb[3]);

/* K1's (b1, b2) of voxel centre c projected onto triangle q0 q1 q2 (voxel units),
 * clamped into the triangle. */
void vo_tri_bary(const float q0[3], const float q1[3], const float q2[3], const float c[3], float* b1, float* b2);

/* uv = fmaf(b2, uv2 - uv0, fmaf(b1, uv1 - uv0, uv0)); uv6 = u0 v0 u1 v1 u2 v2 */
void vo_tri_uv(const float uv6[6], float b1, float b2, float* u, float* v);

/* K1 with diffuse maps: material m's triangles (mat_map[m] >= 0) contribute
 * albedo = Kd x T(uv at the voxel centre's projection) per covered voxel; UVs are
 * the two floats at byte uv_offset of each vertex record.  mat_map NULL = vo_voxelize.
 * Returns -1 on a bad vertex / material / texture index. */
int vo_voxelize_tex(uint32_t n, const float g0[3], float extent,
                    const void* verts, uint32_t stride, uint32_t n_verts,
                    const uint32_t* idx, uint32_t n_idx,
                    const uint32_t* tri_mat, const float* kd4, uint32_t n_mat,
                    const int32_t* mat_map, uint32_t uv_offset, const vo_texture* tex, uint32_t n_tex,
                    int64_t* sums6, uint32_t* counts);

/* K1 resolve: albedo/occupancy and normal grids from the sums. */
void vo_resolve(uint32_t n, const int64_t* sums6, const uint32_t* counts,
                float* albedo_occ4, float* normal4);

/* K2 (A.3): directional light injection with a voxel DDA shadow ray. */
void vo_inject(uint32_t n, const float* albedo_occ4, const float* normal4,
               const float dir_to_light[3], const float color[3], float* r0);

/* K3 (A.4): anisotropic (aniso=1) or box-filter (aniso=0) mips of r0. */
void vo_build_mips(uint32_t n, int aniso, const float* r0, float* pyramid);

/* K4 (A.5/A.6): per-pixel diffuse + specular cone trace.
 * Traces rows y with y % row_step == 0 (row_step 1 = full frame); untouched
 * rows of the outputs are left as they are.  steps_px may be NULL.
 * Returns the total number of cone steps taken. */
typedef struct vo_trace_params {
    uint32_t n;
    float g0[3];
    float extent;
    int aniso;
    uint32_t n_diffuse;   /* 0, 1, 9, 16 */
    uint32_t specular;    /* 0 / 1 */
    float eye[3];
} vo_trace_params;

uint64_t vo_trace(const vo_trace_params* p, const float* r0, const float* pyramid,
                  const float* pos4, const float* nrm4, const float* alb4,
                  uint32_t w, uint32_t h, uint32_t row_step,
                  float* diffuse4, float* spec4, uint32_t* steps_px, int n_threads);

/* Composite + present (vct_spec.h): per pixel
 * final = ((albedo*color)*max(n.l,0))*V + albedo*diffuse.rgb + spec.rgb with V
 * the A.3 shadow walk from the cone origin; out_lin4 (a = 1 / 0 background)
 * and out_rgba8 (Reinhard, gamma 1/2.2, background = clear colour).  Either
 * output may be NULL. */
void vo_composite(uint32_t n, const float g0[3], float extent, const float* albedo_occ4,
                  const float* pos4, const float* nrm4, const float* alb4, const float* diffuse4,
                  const float* spec4, uint32_t w, uint32_t h, const float dir_to_light[3],
                  const float color[3], float* out_lin4, uint32_t* out_rgba8);

/* the spec's log2 (exposed for the known-answer tests) */
float vo_log2(float x);

/* Cone set for n_diffuse (1, 9, 16): fills rows (cn, ct, cb, w), returns tau. */
float vo_cone_set(uint32_t n_diffuse, float rows[][4]);

#ifdef __cplusplus
}
#endif
#endif
