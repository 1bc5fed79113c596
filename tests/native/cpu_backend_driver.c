/* cpu_backend_driver.c — one call sequence through include/vct.h on the CPU oracle
 * backend (oracle/vct_cpu_backend.c + vct_oracle.c), built with
 * -fsanitize=address,undefined (tests/native/Makefile): random triangles ->
 * voxelize -> inject -> mips -> trace (full frame, ragged tiles, compact + untile,
 * packed untile) -> composite -> downloads, plus the error paths (bad indices,
 * out-of-order calls, bad sizes).  TEST INFRASTRUCTURE (tests/test_sanitizers.py). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "vct.h"

static uint32_t rng = 12345u;
static float frand(void) { rng = rng * 1664525u + 1013904223u; return (float)(rng >> 8) / 16777216.0f; }
#define CHECK(x) do { vct_status s_ = (x); if (s_ != VCT_OK) { fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, s_); return 1; } } while (0)
#define EXPECT(x, st) do { if ((x) != (st)) { fprintf(stderr, "%s:%d %s != %d\n", __FILE__, __LINE__, #x, st); return 1; } } while (0)

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 16, ntri = 40, w = 70, h = 45;
    vct_config cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.n = n; cfg.extent = 2.2f; cfg.aniso = 1; cfg.n_diffuse = 9; cfg.specular = 1;
    for (int k = 0; k < 3; ++k) cfg.aabb_min[k] = -1.1f;
    vct_ctx* c = NULL;
    CHECK(vct_create(&cfg, &c));
    float* v = malloc(sizeof(float) * 14 * 3 * ntri);
    uint32_t* idx = malloc(sizeof(uint32_t) * 3 * ntri);
    uint32_t* mat = malloc(sizeof(uint32_t) * ntri);
    float kd[8] = {0.8f, 0.2f, 0.1f, 1, 0.3f, 0.6f, 0.9f, 1};
    for (uint32_t i = 0; i < 3 * ntri; ++i) {
        for (int k = 0; k < 14; ++k) v[14 * i + k] = k < 3 ? 2.0f * frand() - 1.0f : 0.0f;
        idx[i] = i;
    }
    for (uint32_t t = 0; t < ntri; ++t) mat[t] = t & 1;
    EXPECT(vct_inject_directional(c, (float[]){0, 1, 0}, (float[]){1, 1, 1}), VCT_ESTATE);
    idx[5] = 3 * ntri;                                             /* out of range */
    EXPECT(vct_voxelize(c, v, 56, 3 * ntri, idx, 3 * ntri, mat, kd, 2), VCT_EINVAL);
    EXPECT(vct_inject_directional(c, (float[]){0, 1, 0}, (float[]){1, 1, 1}), VCT_ESTATE);
    idx[5] = 5;
    EXPECT(vct_voxelize(c, v, 56, 3 * ntri, idx, 3 * ntri - 1, mat, kd, 2), VCT_EINVAL);   /* not a multiple of 3 */
    CHECK(vct_voxelize(c, v, 56, 3 * ntri, idx, 3 * ntri, mat, kd, 2));
    EXPECT(vct_build_mips(c), VCT_ESTATE);
    CHECK(vct_inject_directional(c, (float[]){0.3f, 1.0f, 0.2f}, (float[]){1, 1, 1}));
    CHECK(vct_build_mips(c));
    const size_t px = (size_t)w * h;
    float* gb = calloc(px * 12, sizeof(float));
    for (size_t p = 0; p < px; ++p) {
        float* pos = gb + 4 * p; float* nrm = gb + 4 * (px + p); float* alb = gb + 4 * (2 * px + p);
        pos[0] = 2.0f * frand() - 1.0f; pos[1] = 2.0f * frand() - 1.0f; pos[2] = 2.0f * frand() - 1.0f;
        pos[3] = (p % 7) ? 1.0f : 0.0f;
        float nx = frand() - 0.5f, ny = frand() - 0.5f, nz = frand() - 0.5f, l = sqrtf(nx * nx + ny * ny + nz * nz);
        nrm[0] = nx / l; nrm[1] = ny / l; nrm[2] = nz / l;
        alb[0] = alb[1] = alb[2] = 0.5f; alb[3] = 0.02f + 0.5f * frand();
    }
    float* d = calloc(px * 4, sizeof(float));
    float* s = calloc(px * 4, sizeof(float));
    uint32_t* st = calloc(px, sizeof(uint32_t));
    uint64_t tot = 0;
    CHECK(vct_trace(c, gb, gb + 4 * px, gb + 8 * px, w, h, (float[]){0, 0, 3}, d, s, st, &tot));
    /* the frame in ranks: compact tiles, padded untile and packed untile */
    const uint32_t world = 3, maxt = vct_tiles_for_rank(w, h, 0, world), T = vct_tiles_for_rank(w, h, 0, 1);
    float* g = calloc((size_t)world * 2 * maxt * 4096 * 4, sizeof(float));
    float* pk = calloc((size_t)2 * T * 4096 * 4, sizeof(float));
    for (uint32_t r = 0; r < world; ++r) {
        vct_trace_args a;
        memset(&a, 0, sizeof a);
        a.pos4 = gb; a.nrm4 = gb + 4 * px; a.alb4 = gb + 8 * px; a.width = w; a.height = h;
        a.eye[2] = 3.0f; a.tile_rank = r; a.tile_world = world; a.tile_compact = 1;
        a.diffuse4 = g + ((size_t)r * 2) * maxt * 4096 * 4;
        a.spec4 = g + ((size_t)r * 2 + 1) * maxt * 4096 * 4;
        CHECK(vct_trace_device(c, &a));
        const uint32_t nt = vct_tiles_for_rank(w, h, r, world), off = 2 * vct_tile_offset(w, h, r, world);
        memcpy(pk + (size_t)off * 4096 * 4, a.diffuse4, (size_t)nt * 4096 * 16);
        memcpy(pk + ((size_t)off + nt) * 4096 * 4, a.spec4, (size_t)nt * 4096 * 16);
    }
    float* fd = calloc(px * 4, sizeof(float));
    float* fs = calloc(px * 4, sizeof(float));
    float* fr[2] = {fd, fs};
    CHECK(vct_untile_planes_device(c, g, 2, w, h, world, fr));
    if (memcmp(fd, d, px * 16) || memcmp(fs, s, px * 16)) { fprintf(stderr, "untile mismatch\n"); return 1; }
    memset(fd, 0, px * 16);
    CHECK(vct_untile_planes_packed_device(c, pk, 2, w, h, world, fr));
    if (memcmp(fd, d, px * 16) || memcmp(fs, s, px * 16)) { fprintf(stderr, "packed untile mismatch\n"); return 1; }
    float* lin = calloc(px * 4, sizeof(float));
    uint32_t* rgba = calloc(px, sizeof(uint32_t));
    CHECK(vct_composite_device(c, gb, gb + 4 * px, gb + 8 * px, d, s, w, h, (float[]){0.3f, 1, 0.2f}, (float[]){1, 1, 1},
                               lin, rgba));
    for (uint32_t l = 0; l < vct_num_levels(c); ++l) {
        uint32_t nl = 0, nf = 0;
        CHECK(vct_level_dims(c, l, &nl, &nf));
        float* buf = malloc((size_t)nl * nl * nl * 16);
        for (uint32_t f = 0; f < nf; ++f) CHECK(vct_download_level(c, l, f, buf));
        EXPECT(vct_download_level(c, l, nf, buf), VCT_EINVAL);
        free(buf);
    }
    float* vox = malloc((size_t)n * n * n * 32);
    CHECK(vct_download_voxels(c, vox, vox + (size_t)n * n * n * 4));
    int64_t* sums = malloc((size_t)n * n * n * 48);
    uint32_t* cnt = malloc((size_t)n * n * n * 4);
    CHECK(vct_download_accum(c, sums, cnt));
    /* grid dump / load (the shared vct_dumpio.c): a round trip, then damaged headers and
       payloads, each refused with VCT_EINVAL */
    {
        char stem[256], path[300];
        snprintf(stem, sizeof stem, "%s/vct_san_dump_%d_%u", getenv("TMPDIR") ? getenv("TMPDIR") : "/tmp",
                 (int)getpid(), n);
        CHECK(vct_save_grid(c, stem, VCT_DUMP_VOXELS | VCT_DUMP_LEVEL0 | VCT_DUMP_PYRAMID));
        vct_ctx* c2 = NULL;
        CHECK(vct_create(&cfg, &c2));
        CHECK(vct_load_grid(c2, stem));
        float* l0a = malloc((size_t)n * n * n * 16);
        float* l0b = malloc((size_t)n * n * n * 16);
        CHECK(vct_download_level(c, 0, 0, l0a));
        CHECK(vct_download_level(c2, 0, 0, l0b));
        if (memcmp(l0a, l0b, (size_t)n * n * n * 16)) { fprintf(stderr, "dump round trip mismatch\n"); return 1; }
        vct_config got;
        uint32_t what = 0;
        CHECK(vct_dump_info(stem, &got, &what));
        if (got.n != n || what != 7u) { fprintf(stderr, "dump info mismatch\n"); return 1; }
        snprintf(path, sizeof path, "%s.json", stem);
        FILE* f = fopen(path, "rb");
        char hdr[4096];
        const size_t hl = fread(hdr, 1, sizeof hdr - 1, f);
        fclose(f);
        hdr[hl] = 0;
        static const char* cuts[] = {"\"n\"", "\"aabb_min\"", "\"sha256\"", "[", ":", "\"grid\""};
        for (size_t k = 0; k < sizeof cuts / sizeof *cuts; ++k) {   /* truncated at each key */
            const char* at = strstr(hdr, cuts[k]);
            f = fopen(path, "wb");
            fwrite(hdr, 1, at ? (size_t)(at - hdr) + 1 : hl / 2, f);
            fclose(f);
            EXPECT(vct_load_grid(c2, stem), VCT_EINVAL);
            EXPECT(vct_dump_info(stem, &got, &what), VCT_EINVAL);
        }
        f = fopen(path, "wb");
        fwrite(hdr, 1, hl, f);
        fclose(f);
        snprintf(path, sizeof path, "%s.bin", stem);
        f = fopen(path, "r+b");
        fseek(f, 5, SEEK_SET);
        fputc(0x5a, f);
        fclose(f);
        EXPECT(vct_load_grid(c2, stem), VCT_EINVAL);           /* sha256 */
        remove(path);
        EXPECT(vct_load_grid(c2, stem), VCT_EINVAL);           /* no payload */
        snprintf(path, sizeof path, "%s.json", stem);
        remove(path);
        vct_destroy(c2);
        free(l0a); free(l0b);
    }
    vct_comm_id id;
    CHECK(vct_comm_get_id(&id));
    EXPECT(vct_comm_init(c, &id, 2, 0), VCT_ECOMM);
    CHECK(vct_comm_init(c, &id, 1, 0));
    CHECK(vct_comm_destroy(c));
    vct_destroy(c);
    free(v); free(idx); free(mat); free(gb); free(d); free(s); free(st); free(g); free(pk); free(fd); free(fs);
    free(lin); free(rgba); free(vox); free(sums); free(cnt);
    printf("ok %llu cone steps\n", (unsigned long long)tot);
    return 0;
}
