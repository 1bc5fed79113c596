/*
 * vct.h — C-ABI drop-in boundary of the MI355X-native voxel-cone-tracing path.
 *
 * What it replaces.  The reference exposes its per-frame hot-path slot as the
 * C++ virtual `Renderer::Render()` (assets/code/renderer/renderer.h:3-10),
 * registered by name in `AssetsManager::renderers`
 * (assets/code/core/assets.h:17-20, assets.cpp:44) and called once per frame at
 * assets/code/core/engine.cpp:151.  Its only implementation,
 * `VoxelizationRenderer::Render` (assets/code/renderer/r_voxelization.cpp:4-35),
 * pulls camera and model state from singletons and issues GL draws; the GI
 * stages its name promises (voxelize, inject, mip, cone-trace) were never
 * written.  This header is the boundary a Renderer
 * subclass calls instead of GL: plain pointers and sizes, no C++ / torch types,
 * status codes instead of exceptions (the reference's only error channel is
 * `throw int` at engine.cpp:55,70 and std::cout prints).
 *
 * Conventions.
 *  - One vct_ctx per host thread, no global state (the reference is
 *    single-threaded: engine.h:7, assets.h:13).  A ctx owns every device buffer.
 *  - Host-pointer entry points are synchronous on return.  *_device entry
 *    points take device pointers and are asynchronous on the ctx stream
 *    (vct_set_stream); vct_synchronize() waits for them.  A host may switch
 *    the ctx stream between vct_trace_device calls so that consecutive frames
 *    run concurrently on different streams (vct.multi.FrameTracer does, for
 *    1.14x at 1080p): the trace's scratch belongs to the stream (4 streams;
 *    a fifth one frees every set after a device synchronize).  The frame
 *    exchanges of a multi-device context (vct_trace_device on a
 *    vct_create_multi ctx) and of vct_comm_trace_frame share one gather
 *    buffer: each such call first waits (on the device, not the host) for the
 *    previous one, whatever stream either ran on, so they stay correct but do
 *    not overlap; vct_comm_synchronize covers the last exchange on any stream.  Grid
 *    updates (voxelize / inject / build_mips / uploads) must be ordered
 *    against traces on other streams by the host (events).
 *  - Data layouts: grids cross the ABI linear-Z RGBA32F, index x + n*(y + n*z)
 *    (the device copy is bricked, see vct_level0_device); the G-buffer and
 *    outputs are [h][w][4] float, row 0 = top of the image.
 *  - Semantics: SURVEY.md Appendix A with the literals of vct_spec.h.
 */
#ifndef VCT_H
#define VCT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VCT_ABI_VERSION 1

typedef struct vct_ctx vct_ctx;

typedef enum vct_status {
    VCT_OK = 0,
    VCT_EINVAL = 1,   /* bad argument                                   */
    VCT_ENOMEM = 2,   /* device allocation failed                       */
    VCT_EDEVICE = 3,  /* HIP runtime / kernel error                     */
    VCT_ECOMM = 4,    /* multi-GPU exchange error                       */
    VCT_ESTATE = 5    /* call out of order (e.g. trace before mips)     */
} vct_status;

/* Grid and cone configuration.  Fields left 0 take the spec default. */
typedef struct vct_config {
    uint32_t n;            /* grid resolution, power of two, 4..1024            */
    float aabb_min[3];     /* world-space min corner of the cubic grid           */
    float extent;          /* cube edge E (> 0); voxel size h = E / n            */
    uint32_t aniso;        /* 1: 6-face anisotropic mips (A.4), 0: box filter    */
    uint32_t n_diffuse;    /* diffuse cones: 0, 1, 9 or 16                        */
    uint32_t specular;     /* 1: trace the specular cone                         */
    int32_t device;        /* HIP device ordinal; -1 = current device            */
} vct_config;

/* Camera in the reference's conventions (scene/camera.h:20-54, camera.cpp:24-27,
 * r_voxelization.cpp:18): RH lookAt, vertical FOV = zoom degrees. */
typedef struct vct_camera {
    float position[3];
    float front[3];        /* unit view direction (camera -z)                    */
    float up[3];           /* unit camera up                                     */
    float right[3];        /* unit camera right                                  */
    float zoom_deg;        /* vertical field of view in degrees                  */
    float near_plane;      /* 0.1 in the reference                               */
    float far_plane;       /* 100 in the reference                               */
} vct_camera;

/* Arguments of the device-resident cone trace (K4).  Float buffers must be
 * 16-byte aligned, the two counters 8-byte aligned (VCT_EINVAL otherwise). */
typedef struct vct_trace_args {
    const float* pos4;     /* device [h][w][4]: world position, w = 1 valid / 0 background */
    const float* nrm4;     /* device [h][w][4]: unit normal                                */
    const float* alb4;     /* device [h][w][4]: albedo rgb, roughness                      */
    uint32_t width, height;
    float eye[3];          /* camera position for the specular cone                        */
    float* diffuse4;       /* device out: (indirect irradiance rgb, ambient occlusion)     */
    float* spec4;          /* device out: (specular rgb, alpha)                            */
    uint32_t* steps_px;    /* device out [h][w] cone steps per pixel, or NULL               */
    unsigned long long* cone_steps; /* device counter, += steps of this call, or NULL      */
    unsigned long long* texel_fetches; /* device counter, += RGBA32F texels the spec reads
                                          (8 per isotropic, 24 per anisotropic level sample), or NULL */
    uint32_t tile_rank;    /* trace only 64x64 tiles t with t % tile_world == tile_rank     */
    uint32_t tile_world;   /* 0 or 1: every tile                                            */
    uint32_t tile_compact; /* 1: outputs in rank-compact tile layout [local tile][64*64][4] */
    uint32_t variant;      /* 0 = default (every form gives identical results; the context picks
                              the fastest per workload, see vct_trace_form).  Public overrides:
                              VCT_VARIANT_FORCE_UNION / _OCCUPANCY (the compiled form),
                              VCT_VARIANT_REORDER / _SCREEN_ORDER (the ray order of a one-rank
                              full frame).  Other bits are A/B experiment switches of the
                              kernel, not part of this interface (csrc/vct_variants.h).      */
} vct_trace_args;

#define VCT_VARIANT_REORDER        0x8000u     /* trace in the Morton order of the cone origins */
#define VCT_VARIANT_FORCE_UNION    0x1000000u  /* four-face-union form (4 waves/SIMD)          */
#define VCT_VARIANT_FORCE_OCCUPANCY 0x2000000u /* occupancy form (5 waves/SIMD)                */
#define VCT_VARIANT_SCREEN_ORDER   0x4000000u  /* trace in screen order                        */

/* ---- lifetime ---------------------------------------------------------- */
vct_status  vct_create(const vct_config* cfg, vct_ctx** out);
void        vct_destroy(vct_ctx* ctx);
const char* vct_last_error(const vct_ctx* ctx);
const char* vct_status_string(vct_status s);
uint32_t    vct_abi_version(void);
vct_status  vct_get_config(const vct_ctx* ctx, vct_config* out);
vct_status  vct_set_stream(vct_ctx* ctx, void* hip_stream); /* NULL = default stream */
vct_status  vct_synchronize(vct_ctx* ctx);

/* ---- one process driving several GPUs (SURVEY.md 8b vct_create_multi) ----------
 * For a host that cannot run one process per GPU (the reference host is one thread
 * with one GL context: engine.h:7, engine.cpp:57).  Device r = (cfg->device + r) mod
 * the device count, r < n_devices (more ranks than devices share devices).  The
 * returned context is device 0's; its calls keep their single-device meaning, except:
 *  - vct_build_mips first copies level 0 to the other devices over xGMI (peer copy,
 *    the replicated grid of SURVEY 8e) when it changed, then builds mips on every device;
 *  - vct_trace / vct_trace_device split the frame into 64x64 tiles (tile t -> device
 *    t % n_devices); every device traces its tiles, the others copy theirs to device 0
 *    (peer copies) and device 0 un-permutes them into the outputs.  Pointers are device
 *    0's; the other devices read the G-buffer through peer access.  tile_world /
 *    tile_compact must be 0.  Outputs and counters are bit-identical to one device.
 *  - vct_synchronize waits for every device; vct_destroy releases every device.
 * K1 and the G-buffer passes run on device 0 only.  In a process per GPU (torch /
 * RCCL) use vct_create per rank instead. */
vct_status  vct_create_multi(const vct_config* cfg, uint32_t n_devices, vct_ctx** out);
uint32_t    vct_num_devices(const vct_ctx* ctx);   /* 1 for a vct_create context */

/* ---- K1 conservative voxelization (A.2) --------------------------------
 * verts: host array of n_verts records of `vertex_stride` bytes whose first 12
 * bytes are the world position (the reference `Vertex`, stdafx.h:36-42, is a
 * 56-byte record with Position at offset 0; mesh.cpp:43-55).  idx: n_idx
 * uint32 indices, 3 per triangle (model.cpp:24 triangulates).  tri_material:
 * per-triangle index into material_kd4 (NULL = material 0).  material_kd4:
 * n_materials x (Kd rgba) as in Material::Kd (material.h:10); NULL = white.
 * Replaces the previous voxel grid; the triangles are kept for
 * vct_gbuffer_raycast_device. */
vct_status vct_voxelize(vct_ctx* ctx, const void* verts, uint32_t vertex_stride, uint32_t n_verts,
                        const uint32_t* idx, uint32_t n_idx, const uint32_t* tri_material,
                        const float* material_kd4, uint32_t n_materials);
/* Same, on geometry already resident on the device (the reference's meshes live
 * in GL buffers after Mesh::setupMesh, mesh.cpp:31-64): every array is a device
 * pointer (verts 4-byte, material_kd4 16-byte aligned).  Returns after K1 has
 * finished (it reads back one candidate count to size its grid). */
vct_status vct_voxelize_device(vct_ctx* ctx, const void* verts, uint32_t vertex_stride, uint32_t n_verts,
                               const uint32_t* idx, uint32_t n_idx, const uint32_t* tri_material,
                               const float* material_kd4, uint32_t n_materials);

/* ---- diffuse maps: albedo = Kd x map (SURVEY.md 8a Model::loadMaterials) -----
 * Replaces what Model::loadMaterialTextures / TextureFromFile (model.cpp:150-226)
 * hand to GL: stbi_load'ed images uploaded with glTexImage2D and sampled with
 * GL_REPEAT / GL_LINEAR (model.cpp:212-216).  A texture is width x height RGBA8
 * texels, row 0 = the image's first row (stbi_load order = GL's t = 0 row); a host
 * loader expands 1- / 3-channel images as GL_RED / GL_RGB sample them, (r,0,0,255) /
 * (r,g,b,255).  Sampling rule, UV of a voxel hit and of a G-buffer hit: vct_spec.h
 * "diffuse maps". */
typedef struct vct_texture {
    const uint8_t* rgba8;  /* host, width * height * 4 bytes                  */
    uint32_t width, height;/* 1 .. VCT_TEX_MAX_DIM                            */
} vct_texture;
/* Uploads the textures to the device, replacing the previous set (n_textures = 0
 * clears it).  Synchronous.  The G-buffer passes sample the set current at their call. */
vct_status vct_set_textures(vct_ctx* ctx, const vct_texture* textures, uint32_t n_textures);
/* K1 with diffuse maps.  As vct_voxelize, plus: material_map[m] = the vct_set_textures
 * index of material m's diffuse map, or -1 (albedo = Kd); uv_offset = byte offset of the
 * two TexCoords floats in a vertex record (24 in the reference Vertex, stdafx.h:36-42,
 * mesh.cpp:49).  A mapped material's triangle contributes albedo = Kd x T(uv) per covered
 * voxel; vct_gbuffer_raycast_device / vct_gbuffer_raster_device then write albedo =
 * Kd x T(uv of the hit).  material_map needs n_materials entries; out-of-range entries
 * are VCT_EINVAL. */
vct_status vct_voxelize_textured(vct_ctx* ctx, const void* verts, uint32_t vertex_stride, uint32_t n_verts,
                                 const uint32_t* idx, uint32_t n_idx, const uint32_t* tri_material,
                                 const float* material_kd4, const int32_t* material_map, uint32_t n_materials,
                                 uint32_t uv_offset);
/* Same on device-resident arrays (material_map 4-byte aligned); see vct_voxelize_device. */
vct_status vct_voxelize_textured_device(vct_ctx* ctx, const void* verts, uint32_t vertex_stride, uint32_t n_verts,
                                        const uint32_t* idx, uint32_t n_idx, const uint32_t* tri_material,
                                        const float* material_kd4, const int32_t* material_map,
                                        uint32_t n_materials, uint32_t uv_offset);

/* ---- K2 direct-light injection (A.3) ----------------------------------- */
vct_status vct_inject_directional(vct_ctx* ctx, const float dir_to_light[3], const float color[3]);

/* ---- K3 mip build (A.4) --------------------------------------------------- */
/* A relight build -- level 0 from vct_inject_directional, and the previous build was one
 * too, with no vct_voxelize* in between -- rebuilds only the blocks that hold geometry
 * and keeps the K4 empty-space maps (after K2, level 0 is nonzero exactly at the
 * occupied voxels).  The result is bit-identical to a full build.  Any dense level-0
 * write (upload_level0, level0_device, set_level0_from_device, the multi-device peer
 * copy) makes the next build a full one. */
vct_status vct_build_mips(vct_ctx* ctx);

/* ---- K4 cone trace (A.5, A.6) ------------------------------------------
 * Host convenience form: uploads the G-buffer, traces every pixel, downloads.
 * out_steps_px / out_cone_steps may be NULL. */
vct_status vct_trace(vct_ctx* ctx, const float* gbuf_pos4, const float* gbuf_nrm4,
                     const float* gbuf_alb_rough4, uint32_t width, uint32_t height,
                     const float eye[3], float* out_diffuse4, float* out_spec4,
                     uint32_t* out_steps_px, uint64_t* out_cone_steps);
/* Device-resident form (asynchronous on the ctx stream). */
vct_status vct_trace_device(vct_ctx* ctx, const vct_trace_args* args);
/* The default variant has two bit-identical compiled forms, the four-face-union form
 * (4 waves/SIMD) and the occupancy form (5 waves/SIMD, three-face bricks), and a one-rank
 * full frame can be traced in screen order or with ray reordering.  The context keeps a
 * choice per workload (frame size, tiling, cone set, grid size; up to four workloads,
 * least recently used replaced): a new workload's first counter-free launches time the
 * candidates (while timing, each launch waits for the previous timed one), then the
 * fastest is kept.  Afterwards launches never block: every 2nd is timed with events
 * that are only polled, and the workload is timed again when its time drifts above
 * 1.35x the settled time three samples in a row (the G-buffer changed), or after a new
 * voxelization once the choice has served 16 launches (doubling, up to 4096, each time
 * the new scene keeps the winner).  While launches alternate streams (overlapped frames;
 * until 64 launches after the last switch) they are not watched, and a timing launch
 * then also waits for the previous launch of any stream.
 * Once the choice is settled, a counter-free launch of at most four generations of waves
 * that does not overlap another frame (a multi-GPU rank's share) records each work unit's
 * (8x8 block x cone part) wave duration, and the next such one dispatches each XCD's units
 * longest first from them (a permutation of the units: outputs unchanged).
 * Returns the kept candidate of the last traced workload -- bit 0 the form (0 union,
 * 1 occupancy), bit 1 ray reordering; a forced candidate when the variant fixes both --
 * or -1 while it is still being timed. */
int32_t    vct_trace_form(const vct_ctx* ctx);
/* Number of 64x64 tiles rank `rank` of `world` traces for a width x height frame. */
uint32_t   vct_tiles_for_rank(uint32_t width, uint32_t height, uint32_t rank, uint32_t world);
/* Scatter all-gathered rank-compact tile buffers ([world][max_tiles][64*64][4],
 * max_tiles = vct_tiles_for_rank(w,h,0,world)) into a [h][w][4] frame. */
vct_status vct_untile_device(vct_ctx* ctx, const float* gathered4, uint32_t width, uint32_t height,
                             uint32_t world, float* frame4);
/* Several planes in one launch: gathered4 = [world][planes][max_tiles][64*64][4],
 * i.e. each rank contributed one [planes][max_tiles*64*64][4] buffer (diffuse
 * and specular side by side, moved by ONE all-gather); plane p is scattered
 * into frames4[p] (a host array of `planes` device pointers, planes <= 4). */
vct_status vct_untile_planes_device(vct_ctx* ctx, const float* gathered4, uint32_t planes, uint32_t width,
                                    uint32_t height, uint32_t world, float* const* frames4);

/* Packed form: rank r contributed exactly its own tiles, [planes][tiles(r)][64*64][4],
 * at tile offset planes * vct_tile_offset(w,h,r,world) of gathered4 (no padding;
 * the gather-to-one-rank layout of vct_comm_trace_frame and vct.multi). */
vct_status vct_untile_planes_packed_device(vct_ctx* ctx, const float* gathered4, uint32_t planes, uint32_t width,
                                           uint32_t height, uint32_t world, float* const* frames4);
/* Tiles of ranks 0..rank-1 (= rank * q + min(rank, T mod world), T tiles, q = T / world). */
uint32_t   vct_tile_offset(uint32_t width, uint32_t height, uint32_t rank, uint32_t world);

/* ---- one process per GPU over RCCL -------------------------
 * For a C/C++ host without torch (the reference engine, engine.cpp:140-157,
 * started once per GPU).  Rank 0 calls vct_comm_get_id and hands the id to the
 * other processes out of band; every rank calls vct_comm_init on its own
 * vct_create context (not a vct_create_multi one).  Calls are collective and
 * queued on the ctx stream. */
typedef struct vct_comm_id { char internal[128]; } vct_comm_id;   /* = ncclUniqueId */
#define VCT_ALL_RANKS (-1)
vct_status vct_comm_get_id(vct_comm_id* out);
vct_status vct_comm_init(vct_ctx* ctx, const vct_comm_id* id, uint32_t nranks, uint32_t rank);
vct_status vct_comm_rank(const vct_ctx* ctx, uint32_t* rank, uint32_t* nranks);
/* ncclBroadcast of the level-0 radiance grid from `root` (after its K2); every
 * rank then runs vct_build_mips itself (the replicated mip pyramid). */
vct_status vct_comm_broadcast_level0(vct_ctx* ctx, uint32_t root);
/* One frame: trace this rank's tiles (tile t -> rank t % nranks; the tile_*
 * fields of args must be 0), then assemble the whole [h][w][4] diffuse / spec
 * frame into args->diffuse4 / spec4 on `root` only (the other ranks send their
 * tiles there: ncclSend / ncclRecv, each rank moves only its own tiles), or on
 * every rank for root = VCT_ALL_RANKS (one ncclAllGather).  Output pointers of
 * non-receiving ranks are not written.  Counters count this rank's tiles. */
vct_status vct_comm_trace_frame(vct_ctx* ctx, const vct_trace_args* args, int32_t root);
/* Releases the communicator (vct_destroy also does). */
vct_status vct_comm_destroy(vct_ctx* ctx);
/* Failure detection.  The communicator is non-blocking: every vct_comm_*
 * call waits for its RCCL calls to be issued for at most the context's deadline
 * (default 300000 ms), polling ncclCommGetAsyncError.  On expiry or an asynchronous
 * error the communicator is aborted (ncclCommAbort) and the call returns VCT_ECOMM
 * (vct_comm_init again to continue), so a dead or absent peer ends the frame loop
 * instead of hanging it. */
vct_status vct_comm_set_timeout(vct_ctx* ctx, uint32_t timeout_ms);
/* Waits until the ctx stream's queued work -- collectives included -- and the last
 * frame exchange (vct_comm_trace_frame on any stream) have finished, polling the
 * stream, that exchange's end event and the communicator with the deadline above. */
vct_status vct_comm_synchronize(vct_ctx* ctx);
/* Where a rank's tiles sit in the exchange buffer of vct_comm_trace_frame (and of the
 * vct.multi driver), in 64x64 tiles: packed for root >= 0 (rank r's [diffuse][spec]
 * planes of tiles(r) at 2 * vct_tile_offset(r); the root receives every block), padded
 * for VCT_ALL_RANKS ([nranks][2][max_tiles], one all-gather).  Pure arithmetic. */
typedef struct vct_comm_layout {
    uint64_t buffer_tiles;   /* tiles of the whole exchange buffer                   */
    uint64_t diffuse_tile;   /* first tile of this rank's diffuse plane              */
    uint64_t spec_tile;      /* first tile of its specular plane                     */
    uint32_t tiles;          /* tiles the rank traces                                */
    uint32_t exchange_tiles; /* tiles it contributes to the exchange (both planes)   */
} vct_comm_layout;
vct_status vct_comm_frame_layout(uint32_t width, uint32_t height, uint32_t nranks, uint32_t rank, int32_t root,
                                 vct_comm_layout* out);

/* ---- G-buffer (input producer) -----------------------
 * Ray-casts the triangles of the last vct_voxelize call through `cam` into a
 * device G-buffer (pos4.w = 1 on hit, 0 on background).  Normals are the face
 * normals turned toward the viewer; albedo = material Kd; alb4.w = roughness. */
vct_status vct_gbuffer_raycast_device(vct_ctx* ctx, const vct_camera* cam, uint32_t width,
                                      uint32_t height, float roughness, float* pos4,
                                      float* nrm4, float* alb4);

/* Same G-buffer as vct_gbuffer_raycast_device, for mesh scenes (SURVEY 8f row
 * f2): the triangles are binned into 16x16-pixel screen tiles through the
 * reference camera (perspective(Zoom, w/h, near, far) + lookAt, r_voxelization.cpp:
 * 16-23), and each pixel's ray is intersected only with its tile's triangles.
 * Ties go to the lower triangle index, so the output equals the brute-force
 * caster's bit for bit.  One small device->host read per call sizes the bins. */
vct_status vct_gbuffer_raster_device(vct_ctx* ctx, const vct_camera* cam, uint32_t width, uint32_t height,
                                     float roughness, float* pos4, float* nrm4, float* alb4);

/* ---- composite + present -------------------------------
 * final = direct + albedo * diffuse.rgb + spec.rgb per pixel, direct = albedo *
 * color * max(n.l, 0) * shadow (the K2 voxel walk from the cone origin), into
 * out_linear4 (float4, a = 1 / 0 background) and/or out_rgba8 (Reinhard, gamma
 * 1/2.2; background = the reference's clear colour, r_voxelization.cpp:8).
 * Device pointers: the G-buffer of the frame and vct_trace_device's outputs.
 * Either output may be NULL, not both.  Needs vct_voxelize. */
vct_status vct_composite_device(vct_ctx* ctx, const float* pos4, const float* nrm4, const float* alb4,
                                const float* diffuse4, const float* spec4, uint32_t width, uint32_t height,
                                const float dir_to_light[3], const float color[3], float* out_linear4,
                                uint32_t* out_rgba8);

/* ---- device memory for hosts without HIP headers (FFI bindings) ----------
 * kind: 0 host->device, 1 device->host, 2 device->device; synchronous. */
vct_status vct_device_alloc(vct_ctx* ctx, size_t bytes, void** dptr);
vct_status vct_device_free(vct_ctx* ctx, void* dptr);
vct_status vct_memcpy(vct_ctx* ctx, void* dst, const void* src, size_t bytes, int kind);

/* ---- grid access (parity, multi-GPU exchange) ---------------------------- */
uint32_t   vct_num_levels(const vct_ctx* ctx);                 /* L + 1 */
vct_status vct_level_dims(const vct_ctx* ctx, uint32_t level, uint32_t* n_l, uint32_t* n_faces);
/* level 0: face must be 0; host_rgba receives n_l^3 x 4 floats */
vct_status vct_download_level(vct_ctx* ctx, uint32_t level, uint32_t face, float* host_rgba);
/* replaces the level-0 radiance grid (n^3 x 4 floats, host); every value must be finite
 * (VCT_EINVAL otherwise: K4's branch-free compositing needs finite samples) */
vct_status vct_upload_level0(vct_ctx* ctx, const float* host_rgba);
/* device pointer + size of the level-0 radiance grid (RCCL broadcast buffer).
 * Device-side level 0 is in the library's internal texel layout (2x2x2 bricks of
 * 8 texels, bricks in linear-Z order; vct_device.h texel_index), not linear-Z:
 * the device pointer and the two device copies below are for moving level 0
 * between contexts of this library (broadcast, replication), not for reading
 * texels; vct_download_level / vct_upload_level0 convert to / from linear-Z. */
vct_status vct_level0_device(vct_ctx* ctx, void** dptr, size_t* bytes);
/* device-to-device copies of the level-0 grid on the ctx stream (host RCCL
 * glue that owns its own communication buffer, e.g. a torch tensor) */
vct_status vct_copy_level0_to_device(vct_ctx* ctx, void* dst);
vct_status vct_set_level0_from_device(vct_ctx* ctx, const void* src);   /* finite values (not checked) */
/* K1 outputs: resolved albedo/occupancy and normal grids (n^3 x 4 floats each) */
vct_status vct_download_voxels(vct_ctx* ctx, float* albedo_occ4, float* normal4);
/* K1 raw accumulators: sums6 [n^3][6] int64 (albedo rgb, normal xyz; 16.16 fixed
 * point), counts [n^3] uint32.  Either pointer may be NULL. */
vct_status vct_download_accum(vct_ctx* ctx, int64_t* sums6, uint32_t* counts);

/* ---- grid dump / load (SURVEY.md 5 "checkpoint / resume") ----------------------
 * The reference persists no state.  A dump is <stem>.json (header: grid config, sections,
 * payload length and sha256) + <stem>.bin (payload, little-endian); the format
 * ("vct-dump/2") is spelled out in csrc/vct_dumpio.h and is the same for every
 * implementation of this header.  Sections:
 *  VCT_DUMP_VOXELS   K1's state: the occupied voxels with their integer sums and counts.
 *                    A context loaded from it is voxelized: vct_inject_directional (any
 *                    light), vct_build_mips, vct_trace and vct_composite_device give what
 *                    they give after the original vct_voxelize, bit for bit.  The
 *                    triangles are not dumped (the G-buffer passes of a loaded context see
 *                    an empty mesh).
 *  VCT_DUMP_LEVEL0   the level-0 radiance (K2's output or an upload); loading it builds
 *                    the mips, so the context can trace at once.
 *  VCT_DUMP_PYRAMID  every face of levels 1..L; on load the rebuilt pyramid is checked
 *                    against it bit for bit (VCT_EINVAL on a difference).
 * Save needs the state a section comes from (VCT_ESTATE otherwise).  Load first checks
 * the payload's length and sha256 and that the dump's grid (n, aabb_min, extent, aniso)
 * is the context's, bit for bit (VCT_EINVAL otherwise, nothing changed); then it
 * replaces the context's grid state.  A failure after that point (a short or corrupt
 * section, an upload or mips error, a rebuilt pyramid that differs) leaves the grid
 * invalid: it reads as never voxelized (VCT_ESTATE for inject / mips / trace) until the
 * next voxelization or successful load.  Synchronous. */
#define VCT_DUMP_VOXELS  0x1u
#define VCT_DUMP_LEVEL0  0x2u
#define VCT_DUMP_PYRAMID 0x4u
vct_status vct_save_grid(vct_ctx* ctx, const char* stem, uint32_t what);
vct_status vct_load_grid(vct_ctx* ctx, const char* stem);
/* A dump's header only: the config it was saved from (device = -1) and its sections,
 * to create a matching context (no context needed; VCT_EINVAL for a missing or malformed
 * header). */
vct_status vct_dump_info(const char* stem, vct_config* cfg, uint32_t* what);

#ifdef __cplusplus
}
#endif
#endif /* VCT_H */
