/*
 * vct_dumpio.h — the file format of vct_save_grid / vct_load_grid (include/vct.h), shared by
 * every implementation of the header (the HIP library and the CPU backend of the tests
 * compile the same vct_dumpio.c), so a dump written by one loads into the other.
 *
 * SURVEY.md section 5 "checkpoint / resume": the reference persists no state; the build
 * dumps the grid for repro cases and to relight a saved scene without its triangles.
 *
 * A dump is two files:
 *   <stem>.json  the header: format "vct-dump/2", kind "grid", the grid config (n,
 *                aabb_min, extent as %.9g -- exact float32 round trips -- aniso, n_diffuse,
 *                specular), the sections present (`what`, VCT_DUMP_*), the occupied-voxel
 *                count, and the payload's byte length and sha256;
 *   <stem>.bin   the payload, little-endian, the sections back to back in this order:
 *     VCT_DUMP_VOXELS   u32 idx[occ] (linear-Z voxel index x + n(y + n z), ascending),
 *                       i64 sums[occ][6] (K1's 16.16 fixed-point albedo rgb, normal xyz),
 *                       u32 counts[occ] (triangles that covered the voxel, > 0);
 *     VCT_DUMP_LEVEL0   f32 [n^3][4] level-0 radiance, linear-Z (vct_download_level);
 *     VCT_DUMP_PYRAMID  f32 levels 1..L, faces 0..F-1 each [n_l^3][4], linear-Z.
 * The reader checks the payload's length and sha256 against the header before any
 * section is handed out.  Plain C (also compiled as HIP C++).
 */
#ifndef VCT_DUMPIO_H
#define VCT_DUMPIO_H

#include <stdint.h>
#include <stdio.h>

#include "../../include/vct.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct vdump_header {
    vct_config cfg;        /* device is not stored (-1 after a read) */
    uint32_t what;         /* VCT_DUMP_* sections present */
    uint64_t occupied;     /* entries of the VCT_DUMP_VOXELS section */
} vdump_header;

typedef struct vdump_sha256 {
    uint32_t h[8];
    uint64_t len;
    uint8_t buf[64];
    uint32_t fill;
} vdump_sha256;

void vdump_sha256_init(vdump_sha256* s);
void vdump_sha256_update(vdump_sha256* s, const void* data, size_t n);
void vdump_sha256_hex(vdump_sha256* s, char out[65]);   /* finalizes */

/* levels and faces of a config (L + 1 levels; 6 faces above level 0 when aniso) */
uint32_t vdump_levels(const vct_config* cfg);
uint32_t vdump_faces(const vct_config* cfg, uint32_t level);
/* byte size of each section and of the whole payload for a header */
uint64_t vdump_voxels_bytes(const vdump_header* h);
uint64_t vdump_level0_bytes(const vdump_header* h);
uint64_t vdump_pyramid_bytes(const vdump_header* h);
uint64_t vdump_payload_bytes(const vdump_header* h);

typedef struct vdump_file {
    FILE* f;
    vdump_sha256 sha;
    uint64_t bytes;        /* written / to read */
    vdump_header h;
    char json[4096], bin[4096];
} vdump_file;

/* 0 on success; otherwise nonzero with a message in err (errlen bytes) */
int vdump_open_write(vdump_file* w, const char* stem, const vdump_header* h, char* err, size_t errlen);
int vdump_write(vdump_file* w, const void* data, size_t n, char* err, size_t errlen);
/* closes the payload and writes the header (with the payload's length and sha256) */
int vdump_close_write(vdump_file* w, char* err, size_t errlen);
/* the header only (vct_dump_config) */
int vdump_read_header(const char* stem, vdump_header* h, char* err, size_t errlen);
/* header + a full pass over the payload checking its length and sha256; then positioned
 * at the payload's first byte */
int vdump_open_read(vdump_file* r, const char* stem, char* err, size_t errlen);
int vdump_read(vdump_file* r, void* data, size_t n, char* err, size_t errlen);
void vdump_close(vdump_file* f);
/* 0 when the dump's grid is the context's: n, aabb_min and extent (bit for bit), aniso */
int vdump_check_config(const vdump_header* h, const vct_config* cfg, char* err, size_t errlen);

#ifdef __cplusplus
}
#endif
#endif /* VCT_DUMPIO_H */
