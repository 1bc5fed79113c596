/*
 * vct_oracle.c — CPU restatement of SURVEY.md Appendix A (TEST INFRASTRUCTURE).
 *
 * Written from the published voxel-cone-tracing method (Crassin et al. 2011) and
 * the normative parameters in include/vct_spec.h; the reference repository holds
 * no implementation of this path (p_voxelization.h:4-7,
 * r_voxelization.cpp:4-35).  Scalar, loop-per-voxel / loop-per-pixel code: it is
 * meant to be obviously right, not fast.  Compile with -ffp-contract=off; the
 * only fused operations are the explicit fmaf() calls of the spec.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this file's library.  See vct_oracle.h for layouts.
 */
#include "vct_oracle.h"
#include "../include/vct_spec.h"

#include <math.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct { float x, y, z; } v3;

static v3 v3sub(v3 a, v3 b) { v3 r = {a.x - b.x, a.y - b.y, a.z - b.z}; return r; }
static float v3dot(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static v3 v3cross(v3 a, v3 b) {
    v3 r = {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
    return r;
}
static float fmin3(float a, float b, float c) { return fminf(fminf(a, b), c); }
static float fmax3(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }

static uint32_t ilog2u(uint32_t n) { uint32_t l = 0; while ((1u << (l + 1)) <= n) ++l; return l; }

size_t vo_level_offset(uint32_t n, int aniso, uint32_t level) {
    size_t off = 0;
    const size_t faces = aniso ? VCT_NUM_FACES : 1;
    for (uint32_t l = 1; l < level; ++l) {
        size_t nl = n >> l;
        off += faces * nl * nl * nl * 4;
    }
    return off;
}

size_t vo_pyramid_floats(uint32_t n, int aniso) {
    return vo_level_offset(n, aniso, ilog2u(n) + 1);
}

/* ------------------------------------------------------------------------- */
/* A.2  K1 conservative voxelization                                          */
/* ------------------------------------------------------------------------- */

/* exact 13-axis separating-axis test, box = voxel centre c, half size 0.5 */
static int tri_box_overlap(v3 q0, v3 q1, v3 q2, v3 c) {
    v3 a[3];
    a[0] = v3sub(q0, c); a[1] = v3sub(q1, c); a[2] = v3sub(q2, c);
    /* (1) box face normals */
    if (fmin3(a[0].x, a[1].x, a[2].x) > 0.5f || fmax3(a[0].x, a[1].x, a[2].x) < -0.5f) return 0;
    if (fmin3(a[0].y, a[1].y, a[2].y) > 0.5f || fmax3(a[0].y, a[1].y, a[2].y) < -0.5f) return 0;
    if (fmin3(a[0].z, a[1].z, a[2].z) > 0.5f || fmax3(a[0].z, a[1].z, a[2].z) < -0.5f) return 0;
    v3 e[3];
    e[0] = v3sub(a[1], a[0]); e[1] = v3sub(a[2], a[1]); e[2] = v3sub(a[0], a[2]);
    /* (2) triangle plane */
    {
        v3 nrm = v3cross(e[0], e[1]);
        v3 vmin, vmax;
        if (nrm.x > 0.0f) { vmin.x = -0.5f - a[0].x; vmax.x = 0.5f - a[0].x; }
        else              { vmin.x = 0.5f - a[0].x;  vmax.x = -0.5f - a[0].x; }
        if (nrm.y > 0.0f) { vmin.y = -0.5f - a[0].y; vmax.y = 0.5f - a[0].y; }
        else              { vmin.y = 0.5f - a[0].y;  vmax.y = -0.5f - a[0].y; }
        if (nrm.z > 0.0f) { vmin.z = -0.5f - a[0].z; vmax.z = 0.5f - a[0].z; }
        else              { vmin.z = 0.5f - a[0].z;  vmax.z = -0.5f - a[0].z; }
        if (v3dot(nrm, vmin) > 0.0f) return 0;
        if (!(v3dot(nrm, vmax) >= 0.0f)) return 0;
    }
    /* (3) nine edge x box-axis cross products */
    for (int i = 0; i < 3; ++i) {
        const v3 ed = e[i];
        v3 ax[3];
        ax[0].x = 0.0f;   ax[0].y = -ed.z; ax[0].z = ed.y;   /* X x e */
        ax[1].x = ed.z;   ax[1].y = 0.0f;  ax[1].z = -ed.x;  /* Y x e */
        ax[2].x = -ed.y;  ax[2].y = ed.x;  ax[2].z = 0.0f;   /* Z x e */
        for (int j = 0; j < 3; ++j) {
            const v3 u = ax[j];
            float p0 = v3dot(u, a[0]), p1 = v3dot(u, a[1]), p2 = v3dot(u, a[2]);
            float rad = 0.5f * ((fabsf(u.x) + fabsf(u.y)) + fabsf(u.z));
            if (fmin3(p0, p1, p2) > rad || fmax3(p0, p1, p2) < -rad) return 0;
        }
    }
    return 1;
}

static void cand_range(float mn, float mx, uint32_t n, int* lo, int* hi) {
    int l = (int)ceilf(fmaxf(mn, -1.0f)) - 1;
    int h = (int)floorf(fminf(mx, (float)n + 1.0f));
    if (l < 0) l = 0;
    if (h > (int)n - 1) h = (int)n - 1;
    *lo = l; *hi = h;
}

/* --- diffuse maps (vct_spec.h "diffuse maps"; SURVEY 8a Model::loadMaterials,
 *     model.cpp:150-226: stbi_load -> glTexImage2D, GL_REPEAT / GL_LINEAR :212-216) */
static float tex_lerp(float a, float b, float f) { return fmaf(f, b - a, a); }

void vo_tex_sample(const vo_texture* t, float u, float v, float rgb[3]) {
    if (!isfinite(u)) u = 0.0f;
    if (!isfinite(v)) v = 0.0f;
    const float fu = u - floorf(u), fv = v - floorf(v);
    const float s = fu * (float)t->width - 0.5f, tt = fv * (float)t->height - 0.5f;
    const float sx = floorf(s), sy = floorf(tt);
    const float ax = s - sx, ay = tt - sy;
    int x0 = (int)sx, y0 = (int)sy, x1 = x0 + 1, y1 = y0 + 1;
    const int W = (int)t->width, H = (int)t->height;
    if (x0 < 0) x0 += W;
    if (y0 < 0) y0 += H;
    if (x1 >= W) x1 -= W;
    if (y1 >= H) y1 -= H;
    const uint8_t* p00 = t->rgba8 + 4 * ((size_t)y0 * W + x0);
    const uint8_t* p10 = t->rgba8 + 4 * ((size_t)y0 * W + x1);
    const uint8_t* p01 = t->rgba8 + 4 * ((size_t)y1 * W + x0);
    const uint8_t* p11 = t->rgba8 + 4 * ((size_t)y1 * W + x1);
    for (int c = 0; c < 3; ++c) {
        const float t00 = (float)p00[c] / 255.0f, t10 = (float)p10[c] / 255.0f;
        const float t01 = (float)p01[c] / 255.0f, t11 = (float)p11[c] / 255.0f;
        rgb[c] = tex_lerp(tex_lerp(t00, t10, ax), tex_lerp(t01, t11, ax), ay);
    }
}

void vo_tri_bary(const float q0[3], const float q1[3], const float q2[3], const float c[3], float* b1, float* b2) {
    const v3 e1 = {q1[0] - q0[0], q1[1] - q0[1], q1[2] - q0[2]};
    const v3 e2 = {q2[0] - q0[0], q2[1] - q0[1], q2[2] - q0[2]};
    const v3 w = {c[0] - q0[0], c[1] - q0[1], c[2] - q0[2]};
    const float d11 = v3dot(e1, e1), d12 = v3dot(e1, e2), d22 = v3dot(e2, e2);
    const float w1 = v3dot(w, e1), w2 = v3dot(w, e2);
    const float den = d11 * d22 - d12 * d12;
    float a = 0.0f, b = 0.0f;
    if (den > 0.0f) {
        a = (d22 * w1 - d12 * w2) / den;
        b = (d11 * w2 - d12 * w1) / den;
    }
    a = fmaxf(a, 0.0f);
    b = fmaxf(b, 0.0f);
    const float s = a + b;
    if (s > 1.0f) { a = a / s; b = b / s; }
    *b1 = a;
    *b2 = b;
}

void vo_tri_uv(const float uv6[6], float b1, float b2, float* u, float* v) {
    *u = fmaf(b2, uv6[4] - uv6[0], fmaf(b1, uv6[2] - uv6[0], uv6[0]));
    *v = fmaf(b2, uv6[5] - uv6[1], fmaf(b1, uv6[3] - uv6[1], uv6[1]));
}

int vo_voxelize_tex(uint32_t n, const float g0[3], float extent,
                    const void* verts, uint32_t stride, uint32_t n_verts,
                    const uint32_t* idx, uint32_t n_idx,
                    const uint32_t* tri_mat, const float* kd4, uint32_t n_mat,
                    const int32_t* mat_map, uint32_t uv_offset, const vo_texture* tex, uint32_t n_tex,
                    int64_t* sums6, uint32_t* counts) {
    const float inv_h = (float)n / extent;
    const uint32_t n_tri = n_idx / 3;
    for (uint32_t t = 0; t < n_tri; ++t) {
        uint32_t vi[3] = {idx[3 * t], idx[3 * t + 1], idx[3 * t + 2]};
        if (vi[0] >= n_verts || vi[1] >= n_verts || vi[2] >= n_verts) return -1;
        uint32_t mat = tri_mat ? tri_mat[t] : 0;
        if ((kd4 || mat_map) && mat >= n_mat) return -1;
        const int32_t map = mat_map ? mat_map[mat] : -1;
        if (map < -1 || (map >= 0 && (uint32_t)map >= n_tex)) return -1;
        v3 p[3], q[3];
        float uv[6] = {0, 0, 0, 0, 0, 0};
        for (int k = 0; k < 3; ++k) {
            const char* rec = (const char*)verts + (size_t)vi[k] * stride;
            const float* f = (const float*)rec;
            p[k].x = f[0]; p[k].y = f[1]; p[k].z = f[2];
            q[k].x = (p[k].x - g0[0]) * inv_h;
            q[k].y = (p[k].y - g0[1]) * inv_h;
            q[k].z = (p[k].z - g0[2]) * inv_h;
            if (map >= 0) memcpy(uv + 2 * k, rec + uv_offset, 8);
        }
        /* face normal (world units) and albedo in 16.16 fixed point */
        v3 fn = v3cross(v3sub(p[1], p[0]), v3sub(p[2], p[0]));
        float len = sqrtf(v3dot(fn, fn));
        if (len > 0.0f) { fn.x = fn.x / len; fn.y = fn.y / len; fn.z = fn.z / len; }
        else { fn.x = 0.0f; fn.y = 0.0f; fn.z = 0.0f; }
        int64_t fix[6];
        float kd[3];
        for (int c = 0; c < 3; ++c) {
            kd[c] = kd4 ? kd4[4 * mat + c] : 1.0f;
            fix[c] = (int64_t)roundf(kd[c] * VCT_FIXED_ONE);
        }
        fix[3] = (int64_t)roundf(fn.x * VCT_FIXED_ONE);
        fix[4] = (int64_t)roundf(fn.y * VCT_FIXED_ONE);
        fix[5] = (int64_t)roundf(fn.z * VCT_FIXED_ONE);
        const float q0[3] = {q[0].x, q[0].y, q[0].z}, q1[3] = {q[1].x, q[1].y, q[1].z},
                    q2[3] = {q[2].x, q[2].y, q[2].z};

        int lo[3], hi[3];
        cand_range(fmin3(q[0].x, q[1].x, q[2].x), fmax3(q[0].x, q[1].x, q[2].x), n, &lo[0], &hi[0]);
        cand_range(fmin3(q[0].y, q[1].y, q[2].y), fmax3(q[0].y, q[1].y, q[2].y), n, &lo[1], &hi[1]);
        cand_range(fmin3(q[0].z, q[1].z, q[2].z), fmax3(q[0].z, q[1].z, q[2].z), n, &lo[2], &hi[2]);
        for (int z = lo[2]; z <= hi[2]; ++z)
            for (int y = lo[1]; y <= hi[1]; ++y)
                for (int x = lo[0]; x <= hi[0]; ++x) {
                    v3 c = {(float)x + 0.5f, (float)y + 0.5f, (float)z + 0.5f};
                    if (!tri_box_overlap(q[0], q[1], q[2], c)) continue;
                    size_t v = (size_t)x + (size_t)n * ((size_t)y + (size_t)n * (size_t)z);
                    int64_t fa[3] = {fix[0], fix[1], fix[2]};
                    if (map >= 0) {   /* albedo = Kd x T(uv at the voxel centre's projection) */
                        const float cc[3] = {c.x, c.y, c.z};
                        float b1, b2, u, w, rgb[3];
                        vo_tri_bary(q0, q1, q2, cc, &b1, &b2);
                        vo_tri_uv(uv, b1, b2, &u, &w);
                        vo_tex_sample(&tex[map], u, w, rgb);
                        for (int k = 0; k < 3; ++k) fa[k] = (int64_t)roundf((kd[k] * rgb[k]) * VCT_FIXED_ONE);
                    }
                    for (int k = 0; k < 3; ++k)
                        sums6[6 * v + k] = (int64_t)((uint64_t)sums6[6 * v + k] + (uint64_t)fa[k]);
                    for (int k = 3; k < 6; ++k)
                        sums6[6 * v + k] = (int64_t)((uint64_t)sums6[6 * v + k] + (uint64_t)fix[k]);
                    counts[v] += 1;
                }
    }
    return 0;
}

int vo_voxelize(uint32_t n, const float g0[3], float extent,
                const void* verts, uint32_t stride, uint32_t n_verts,
                const uint32_t* idx, uint32_t n_idx,
                const uint32_t* tri_mat, const float* kd4, uint32_t n_mat,
                int64_t* sums6, uint32_t* counts) {
    return vo_voxelize_tex(n, g0, extent, verts, stride, n_verts, idx, n_idx, tri_mat, kd4, n_mat, NULL, 0, NULL, 0,
                           sums6, counts);
}

void vo_resolve(uint32_t n, const int64_t* sums6, const uint32_t* counts,
                float* albedo_occ4, float* normal4) {
    const size_t nv = (size_t)n * n * n;
    for (size_t v = 0; v < nv; ++v) {
        float* ao = albedo_occ4 + 4 * v;
        float* nm = normal4 + 4 * v;
        uint32_t cnt = counts[v];
        if (cnt == 0) {
            ao[0] = ao[1] = ao[2] = ao[3] = 0.0f;
            nm[0] = nm[1] = nm[2] = nm[3] = 0.0f;
            continue;
        }
        double den = (double)cnt * VCT_FIXED_ONE_D;
        for (int c = 0; c < 3; ++c) ao[c] = (float)((double)sums6[6 * v + c] / den);
        ao[3] = 1.0f;
        double sx = (double)sums6[6 * v + 3], sy = (double)sums6[6 * v + 4], sz = (double)sums6[6 * v + 5];
        double len = sqrt((sx * sx + sy * sy) + sz * sz);
        if (len > 0.0) {
            nm[0] = (float)(sx / len); nm[1] = (float)(sy / len); nm[2] = (float)(sz / len);
        } else {
            nm[0] = nm[1] = nm[2] = 0.0f;
        }
        nm[3] = 0.0f;
    }
}

/* ------------------------------------------------------------------------- */
/* A.3  K2 direct-light injection                                             */
/* ------------------------------------------------------------------------- */

static int occupied(const float* albedo_occ4, uint32_t n, int x, int y, int z) {
    size_t v = (size_t)x + (size_t)n * ((size_t)y + (size_t)n * (size_t)z);
    return albedo_occ4[4 * v + 3] != 0.0f;
}

/* Amanatides-Woo voxel walk from q (voxel units) along l.  1 = reaches outside. */
static float dda_visibility(const float* albedo_occ4, uint32_t n, v3 q, v3 l) {
    int vx = (int)floorf(q.x), vy = (int)floorf(q.y), vz = (int)floorf(q.z);
    const int N = (int)n;
    if (vx < 0 || vy < 0 || vz < 0 || vx >= N || vy >= N || vz >= N) return 1.0f;
    int sx = l.x > 0.0f ? 1 : (l.x < 0.0f ? -1 : 0);
    int sy = l.y > 0.0f ? 1 : (l.y < 0.0f ? -1 : 0);
    int sz = l.z > 0.0f ? 1 : (l.z < 0.0f ? -1 : 0);
    float tdx = sx ? 1.0f / fabsf(l.x) : INFINITY;
    float tdy = sy ? 1.0f / fabsf(l.y) : INFINITY;
    float tdz = sz ? 1.0f / fabsf(l.z) : INFINITY;
    float tmx = sx > 0 ? ((float)(vx + 1) - q.x) * tdx : (sx < 0 ? (q.x - (float)vx) * tdx : INFINITY);
    float tmy = sy > 0 ? ((float)(vy + 1) - q.y) * tdy : (sy < 0 ? (q.y - (float)vy) * tdy : INFINITY);
    float tmz = sz > 0 ? ((float)(vz + 1) - q.z) * tdz : (sz < 0 ? (q.z - (float)vz) * tdz : INFINITY);
    for (;;) {
        if (occupied(albedo_occ4, n, vx, vy, vz)) return 0.0f;
        if (tmx <= tmy && tmx <= tmz) {
            vx += sx; if (vx < 0 || vx >= N) return 1.0f; tmx = tmx + tdx;
        } else if (tmy <= tmz) {
            vy += sy; if (vy < 0 || vy >= N) return 1.0f; tmy = tmy + tdy;
        } else {
            vz += sz; if (vz < 0 || vz >= N) return 1.0f; tmz = tmz + tdz;
        }
    }
}

void vo_inject(uint32_t n, const float* albedo_occ4, const float* normal4,
               const float dir_to_light[3], const float color[3], float* r0) {
    v3 l = {dir_to_light[0], dir_to_light[1], dir_to_light[2]};
    float len = sqrtf(v3dot(l, l));
    if (len > 0.0f) { l.x = l.x / len; l.y = l.y / len; l.z = l.z / len; }
    for (uint32_t z = 0; z < n; ++z)
        for (uint32_t y = 0; y < n; ++y)
            for (uint32_t x = 0; x < n; ++x) {
                size_t v = (size_t)x + (size_t)n * ((size_t)y + (size_t)n * (size_t)z);
                float* out = r0 + 4 * v;
                const float* ao = albedo_occ4 + 4 * v;
                if (ao[3] == 0.0f) { out[0] = out[1] = out[2] = out[3] = 0.0f; continue; }
                v3 nm = {normal4[4 * v], normal4[4 * v + 1], normal4[4 * v + 2]};
                float ndl = v3dot(nm, l);
                float L[3] = {0.0f, 0.0f, 0.0f};
                if (ndl > 0.0f) {
                    v3 q = {((float)x + 0.5f) + nm.x, ((float)y + 0.5f) + nm.y, ((float)z + 0.5f) + nm.z};
                    float vis = dda_visibility(albedo_occ4, n, q, l);
                    for (int c = 0; c < 3; ++c) L[c] = ((ao[c] * color[c]) * ndl) * vis;
                }
                out[0] = L[0]; out[1] = L[1]; out[2] = L[2]; out[3] = 1.0f;
            }
}

/* ------------------------------------------------------------------------- */
/* f3  composite + present (vct_spec.h)                                        */
/* ------------------------------------------------------------------------- */

static uint32_t to8(float v) {
    v = v / (1.0f + v);
    v = powf(v < 0.0f ? 0.0f : v, VCT_INV_GAMMA);
    long q = lroundf(v * 255.0f);
    return (uint32_t)(q < 0 ? 0 : (q > 255 ? 255 : q));
}

void vo_composite(uint32_t n, const float g0[3], float extent, const float* albedo_occ4,
                  const float* pos4, const float* nrm4, const float* alb4, const float* diffuse4,
                  const float* spec4, uint32_t w, uint32_t h, const float dir_to_light[3],
                  const float color[3], float* out_lin4, uint32_t* out_rgba8) {
    v3 l = {dir_to_light[0], dir_to_light[1], dir_to_light[2]};
    float len = sqrtf(v3dot(l, l));
    if (len > 0.0f) { l.x = l.x / len; l.y = l.y / len; l.z = l.z / len; }
    const float inv_h = (float)n / extent;
    for (size_t i = 0; i < (size_t)w * h; ++i) {
        const float *P = pos4 + 4 * i, *N = nrm4 + 4 * i, *A = alb4 + 4 * i;
        const float *D = diffuse4 + 4 * i, *S = spec4 + 4 * i;
        if (P[3] == 0.0f) {
            if (out_lin4) {
                out_lin4[4 * i] = VCT_CLEAR_R; out_lin4[4 * i + 1] = VCT_CLEAR_G;
                out_lin4[4 * i + 2] = VCT_CLEAR_B; out_lin4[4 * i + 3] = 0.0f;
            }
            if (out_rgba8)
                out_rgba8[i] = (uint32_t)lroundf(VCT_CLEAR_R * 255.0f) | ((uint32_t)lroundf(VCT_CLEAR_G * 255.0f) << 8) |
                               ((uint32_t)lroundf(VCT_CLEAR_B * 255.0f) << 16) | (255u << 24);
            continue;
        }
        v3 nm = {N[0], N[1], N[2]};
        float ndl = v3dot(nm, l);
        float d[3] = {0.0f, 0.0f, 0.0f};
        if (ndl > 0.0f) {
            v3 q = {(P[0] - g0[0]) * inv_h + nm.x, (P[1] - g0[1]) * inv_h + nm.y, (P[2] - g0[2]) * inv_h + nm.z};
            float vis = dda_visibility(albedo_occ4, n, q, l);
            for (int c = 0; c < 3; ++c) d[c] = ((A[c] * color[c]) * ndl) * vis;
        }
        float f[3];
        for (int c = 0; c < 3; ++c) f[c] = (d[c] + A[c] * D[c]) + S[c];
        if (out_lin4) {
            out_lin4[4 * i] = f[0]; out_lin4[4 * i + 1] = f[1]; out_lin4[4 * i + 2] = f[2]; out_lin4[4 * i + 3] = 1.0f;
        }
        if (out_rgba8) out_rgba8[i] = to8(f[0]) | (to8(f[1]) << 8) | (to8(f[2]) << 16) | (255u << 24);
    }
}

/* ------------------------------------------------------------------------- */
/* A.4  K3 mips                                                               */
/* ------------------------------------------------------------------------- */

static const float* texel(const float* vol, uint32_t nl, uint32_t x, uint32_t y, uint32_t z) {
    return vol + 4 * ((size_t)x + (size_t)nl * ((size_t)y + (size_t)nl * (size_t)z));
}

/* front-to-back composite of two children: r = f + (1 - f.a) * b */
static void composite(const float* f, const float* b, float* r) {
    float oma = 1.0f - f[3];
    r[0] = f[0] + oma * b[0];
    r[1] = f[1] + oma * b[1];
    r[2] = f[2] + oma * b[2];
    r[3] = f[3] + oma * b[3];
}

void vo_build_mips(uint32_t n, int aniso, const float* r0, float* pyramid) {
    const uint32_t L = ilog2u(n);
    const int faces = aniso ? VCT_NUM_FACES : 1;
    for (uint32_t l = 1; l <= L; ++l) {
        const uint32_t nl = n >> l, nc = nl * 2;
        float* dst = pyramid + vo_level_offset(n, aniso, l);
        const size_t vl = (size_t)nl * nl * nl, vc = (size_t)nc * nc * nc;
        for (int f = 0; f < faces; ++f) {
            const float* src = (l == 1) ? r0 : pyramid + vo_level_offset(n, aniso, l - 1) + (size_t)f * vc * 4;
            float* out = dst + (size_t)f * vl * 4;
            for (uint32_t z = 0; z < nl; ++z)
                for (uint32_t y = 0; y < nl; ++y)
                    for (uint32_t x = 0; x < nl; ++x) {
                        float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
                        const uint32_t cx = 2 * x, cy = 2 * y, cz = 2 * z;
                        if (!aniso) {
                            for (uint32_t dz = 0; dz < 2; ++dz)
                                for (uint32_t dy = 0; dy < 2; ++dy)
                                    for (uint32_t dx = 0; dx < 2; ++dx) {
                                        const float* t = texel(src, nc, cx + dx, cy + dy, cz + dz);
                                        for (int c = 0; c < 4; ++c) acc[c] = acc[c] + t[c];
                                    }
                            for (int c = 0; c < 4; ++c) acc[c] = acc[c] * 0.125f;
                        } else {
                            const int axis = f >> 1;          /* 0 x, 1 y, 2 z */
                            const uint32_t fr = (f & 1) ? 1u : 0u, bk = 1u - fr;
                            for (uint32_t r1 = 0; r1 < 2; ++r1)       /* slower row coordinate */
                                for (uint32_t r0c = 0; r0c < 2; ++r0c) { /* faster row coordinate */
                                    const float *tf, *tb;
                                    if (axis == 0) {        /* rows over (y, z) */
                                        tf = texel(src, nc, cx + fr, cy + r0c, cz + r1);
                                        tb = texel(src, nc, cx + bk, cy + r0c, cz + r1);
                                    } else if (axis == 1) { /* rows over (x, z) */
                                        tf = texel(src, nc, cx + r0c, cy + fr, cz + r1);
                                        tb = texel(src, nc, cx + r0c, cy + bk, cz + r1);
                                    } else {                /* rows over (x, y) */
                                        tf = texel(src, nc, cx + r0c, cy + r1, cz + fr);
                                        tb = texel(src, nc, cx + r0c, cy + r1, cz + bk);
                                    }
                                    float row[4];
                                    composite(tf, tb, row);
                                    for (int c = 0; c < 4; ++c) acc[c] = acc[c] + row[c];
                                }
                            for (int c = 0; c < 4; ++c) acc[c] = acc[c] * 0.25f;
                        }
                        float* o = out + 4 * ((size_t)x + (size_t)nl * ((size_t)y + (size_t)nl * (size_t)z));
                        o[0] = acc[0]; o[1] = acc[1]; o[2] = acc[2]; o[3] = acc[3];
                    }
        }
    }
}

/* ------------------------------------------------------------------------- */
/* A.5 / A.6  K4 cone trace                                                   */
/* ------------------------------------------------------------------------- */

float vo_log2(float x) {
    uint32_t bits;
    memcpy(&bits, &x, 4);
    int e = (int)((bits >> 23) & 0xffu) - 127;
    uint32_t mb = (bits & 0x007fffffu) | 0x3f800000u;
    float f;
    memcpy(&f, &mb, 4);
    if (f > VCT_LOG2_SQRT2) { f = f * 0.5f; e += 1; }
    float s = (f - 1.0f) / (f + 1.0f);
    float z = s * s;
    float p = VCT_LOG2_C9;
    p = fmaf(p, z, VCT_LOG2_C7);
    p = fmaf(p, z, VCT_LOG2_C5);
    p = fmaf(p, z, VCT_LOG2_C3);
    p = fmaf(p, z, 1.0f);
    float ln = (2.0f * s) * p;
    return fmaf(ln, VCT_INV_LN2, (float)e);
}

#define VO_ROW(cn, ct, cb, w) {cn, ct, cb, w},
static const float cones1[1][4] = {VCT_CONES1(VO_ROW)};
static const float cones9[9][4] = {VCT_CONES9(VO_ROW)};
static const float cones16[16][4] = {VCT_CONES16(VO_ROW)};

float vo_cone_set(uint32_t n_diffuse, float rows[][4]) {
    const float(*src)[4] = n_diffuse == 16 ? cones16 : (n_diffuse == 9 ? cones9 : cones1);
    uint32_t k = n_diffuse == 16 ? 16 : (n_diffuse == 9 ? 9 : (n_diffuse == 1 ? 1 : 0));
    for (uint32_t i = 0; i < k; ++i) memcpy(rows[i], src[i], sizeof(float) * 4);
    return n_diffuse == 16 ? VCT_TAN20 : VCT_TAN30;
}

typedef struct {
    uint32_t n, L;
    int aniso;
    const float* r0;
    const float* pyr;
    float tmax;
} tracer;

/* T_l at texel coords c = q * scale - 0.5, zero border */
static void trilinear(const float* vol, uint32_t nl, v3 q, float scale, float out[4]) {
    float cx = q.x * scale - 0.5f, cy = q.y * scale - 0.5f, cz = q.z * scale - 0.5f;
    float fx0 = floorf(cx), fy0 = floorf(cy), fz0 = floorf(cz);
    int ix = (int)fx0, iy = (int)fy0, iz = (int)fz0;
    float fx = cx - fx0, fy = cy - fy0, fz = cz - fz0;
    float wx[2] = {1.0f - fx, fx}, wy[2] = {1.0f - fy, fy}, wz[2] = {1.0f - fz, fz};
    out[0] = out[1] = out[2] = out[3] = 0.0f;
    for (int dz = 0; dz < 2; ++dz)
        for (int dy = 0; dy < 2; ++dy)
            for (int dx = 0; dx < 2; ++dx) {
                int x = ix + dx, y = iy + dy, z = iz + dz;
                if (x < 0 || y < 0 || z < 0 || x >= (int)nl || y >= (int)nl || z >= (int)nl) continue;
                float w = (wx[dx] * wy[dy]) * wz[dz];
                const float* t = texel(vol, nl, (uint32_t)x, (uint32_t)y, (uint32_t)z);
                out[0] = fmaf(w, t[0], out[0]);
                out[1] = fmaf(w, t[1], out[1]);
                out[2] = fmaf(w, t[2], out[2]);
                out[3] = fmaf(w, t[3], out[3]);
            }
}

/* Directional trilinear sample of an anisotropic level (A.5): the three faces
 * selected by the signs of d are combined PER CORNER TEXEL,
 *   v = fmaf(d.z^2, Fz, fmaf(d.y^2, Fy, d.x^2 * Fx)),
 * and the combined texels are trilinearly filtered like T_l.  (Filtering is
 * linear, so this equals sum_f w_f T_l(F_f); fixing the order this way lets
 * a wave whose lanes share one direction combine each texel once.) */
static void trilinear_dir(const float* lvl, size_t vl, uint32_t nl, v3 q, float scale, const int face[3],
                          const float wd[3], float out[4]) {
    float cx = q.x * scale - 0.5f, cy = q.y * scale - 0.5f, cz = q.z * scale - 0.5f;
    float fx0 = floorf(cx), fy0 = floorf(cy), fz0 = floorf(cz);
    int ix = (int)fx0, iy = (int)fy0, iz = (int)fz0;
    float fx = cx - fx0, fy = cy - fy0, fz = cz - fz0;
    float wx[2] = {1.0f - fx, fx}, wy[2] = {1.0f - fy, fy}, wz[2] = {1.0f - fz, fz};
    out[0] = out[1] = out[2] = out[3] = 0.0f;
    for (int dz = 0; dz < 2; ++dz)
        for (int dy = 0; dy < 2; ++dy)
            for (int dx = 0; dx < 2; ++dx) {
                int x = ix + dx, y = iy + dy, z = iz + dz;
                if (x < 0 || y < 0 || z < 0 || x >= (int)nl || y >= (int)nl || z >= (int)nl) continue;
                float w = (wx[dx] * wy[dy]) * wz[dz];
                const float* tX = texel(lvl + (size_t)face[0] * vl, nl, (uint32_t)x, (uint32_t)y, (uint32_t)z);
                const float* tY = texel(lvl + (size_t)face[1] * vl, nl, (uint32_t)x, (uint32_t)y, (uint32_t)z);
                const float* tZ = texel(lvl + (size_t)face[2] * vl, nl, (uint32_t)x, (uint32_t)y, (uint32_t)z);
                for (int c = 0; c < 4; ++c) {
                    float v = wd[0] * tX[c];
                    v = fmaf(wd[1], tY[c], v);
                    v = fmaf(wd[2], tZ[c], v);
                    out[c] = fmaf(w, v, out[c]);
                }
            }
}

/* D_l(q, d): level 0 isotropic; level >= 1 directional (aniso) or isotropic */
static void sample_level(const tracer* tr, uint32_t l, v3 q, const int face[3], const float wd[3],
                         float out[4]) {
    if (l == 0) { trilinear(tr->r0, tr->n, q, 1.0f, out); return; }
    const uint32_t nl = tr->n >> l;
    const float scale = ldexpf(1.0f, -(int)l);
    const float* lvl = tr->pyr + vo_level_offset(tr->n, tr->aniso, l);
    if (!tr->aniso) { trilinear(lvl, nl, q, scale, out); return; }
    trilinear_dir(lvl, (size_t)nl * nl * nl * 4, nl, q, scale, face, wd, out);
}

/* one cone from o along d with half-angle tangent tau; returns step count */
static uint32_t march(const tracer* tr, v3 o, v3 d, float tau, float res[4]) {
    const float tau2 = 2.0f * tau;
    const float nf = (float)tr->n;
    int face[3] = {d.x >= 0.0f ? VCT_FACE_PX : VCT_FACE_NX,
                   d.y >= 0.0f ? VCT_FACE_PY : VCT_FACE_NY,
                   d.z >= 0.0f ? VCT_FACE_PZ : VCT_FACE_NZ};
    float wd[3] = {d.x * d.x, d.y * d.y, d.z * d.z};
    float c[3] = {0.0f, 0.0f, 0.0f}, a = 0.0f, t = 1.0f;
    uint32_t steps = 0;
    for (;;) {
        if (!(a < VCT_ALPHA_STOP)) break;
        if (!(t <= tr->tmax)) break;
        v3 q = {o.x + d.x * t, o.y + d.y * t, o.z + d.z * t};
        if (!(q.x >= 0.0f && q.x <= nf && q.y >= 0.0f && q.y <= nf && q.z >= 0.0f && q.z <= nf)) break;
        float D = fmaxf(1.0f, tau2 * t);
        float m = vo_log2(D);
        if (m > (float)tr->L) m = (float)tr->L;
        uint32_t l0 = (uint32_t)m;
        float fr = m - (float)l0;
        float s[4];
        sample_level(tr, l0, q, face, wd, s);
        if (fr > 0.0f && l0 < tr->L) {
            float s1[4];
            sample_level(tr, l0 + 1, q, face, wd, s1);
            for (int k = 0; k < 4; ++k) s[k] = fmaf(fr, s1[k], (1.0f - fr) * s[k]);
        }
        float oma = 1.0f - a;
        c[0] = fmaf(oma, s[0], c[0]);
        c[1] = fmaf(oma, s[1], c[1]);
        c[2] = fmaf(oma, s[2], c[2]);
        a = fmaf(oma, s[3], a);
        t = t + VCT_STEP_SCALE * D;
        ++steps;
    }
    res[0] = c[0]; res[1] = c[1]; res[2] = c[2]; res[3] = a;
    return steps;
}

uint64_t vo_trace(const vo_trace_params* p, const float* r0, const float* pyramid,
                  const float* pos4, const float* nrm4, const float* alb4,
                  uint32_t w, uint32_t h, uint32_t row_step,
                  float* diffuse4, float* spec4, uint32_t* steps_px, int n_threads) {
    tracer tr;
    tr.n = p->n; tr.L = ilog2u(p->n); tr.aniso = p->aniso; tr.r0 = r0; tr.pyr = pyramid;
    tr.tmax = (float)p->n * VCT_SQRT3;
    float cones[16][4];
    const float tau_d = vo_cone_set(p->n_diffuse, cones);
    const uint32_t nd = p->n_diffuse;
    const float inv_h = (float)p->n / p->extent;
    if (row_step == 0) row_step = 1;
    uint64_t total = 0;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : total)
#endif
    for (int64_t yy = 0; yy < (int64_t)h; yy += row_step) {
        for (uint32_t x = 0; x < w; ++x) {
            const size_t i = (size_t)yy * w + x;
            float* dout = diffuse4 + 4 * i;
            float* sout = spec4 + 4 * i;
            const float* P = pos4 + 4 * i;
            if (P[3] == 0.0f) {
                dout[0] = dout[1] = dout[2] = dout[3] = 0.0f;
                sout[0] = sout[1] = sout[2] = sout[3] = 0.0f;
                if (steps_px) steps_px[i] = 0;
                continue;
            }
            v3 nrm = {nrm4[4 * i], nrm4[4 * i + 1], nrm4[4 * i + 2]};
            v3 o = {(P[0] - p->g0[0]) * inv_h + nrm.x,
                    (P[1] - p->g0[1]) * inv_h + nrm.y,
                    (P[2] - p->g0[2]) * inv_h + nrm.z};
            uint32_t steps = 0;
            /* Duff et al. 2017 branchless orthonormal basis */
            float sgn = copysignf(1.0f, nrm.z);
            float ka = -1.0f / (sgn + nrm.z);
            float kb = (nrm.x * nrm.y) * ka;
            v3 T = {1.0f + ((sgn * nrm.x) * nrm.x) * ka, sgn * kb, -(sgn * nrm.x)};
            v3 B = {kb, sgn + (nrm.y * nrm.y) * ka, -nrm.y};
            float irr[3] = {0.0f, 0.0f, 0.0f}, occ = 0.0f;
            for (uint32_t k = 0; k < nd; ++k) {
                const float cn = cones[k][0], ct = cones[k][1], cb = cones[k][2], wk = cones[k][3];
                v3 d = {(cn * nrm.x + ct * T.x) + cb * B.x,
                        (cn * nrm.y + ct * T.y) + cb * B.y,
                        (cn * nrm.z + ct * T.z) + cb * B.z};
                float res[4];
                steps += march(&tr, o, d, tau_d, res);
                irr[0] = fmaf(wk, res[0], irr[0]);
                irr[1] = fmaf(wk, res[1], irr[1]);
                irr[2] = fmaf(wk, res[2], irr[2]);
                occ = fmaf(wk, res[3], occ);
            }
            dout[0] = irr[0]; dout[1] = irr[1]; dout[2] = irr[2]; dout[3] = 1.0f - occ;
            if (p->specular) {
                v3 v = {p->eye[0] - P[0], p->eye[1] - P[1], p->eye[2] - P[2]};
                float vl = sqrtf(v3dot(v, v));
                v.x = v.x / vl; v.y = v.y / vl; v.z = v.z / vl;
                float ndv = v3dot(nrm, v);
                float k2 = 2.0f * ndv;
                v3 r = {k2 * nrm.x - v.x, k2 * nrm.y - v.y, k2 * nrm.z - v.z};
                float tau = fminf(fmaxf(alb4[4 * i + 3], VCT_SPEC_TAU_MIN), VCT_SPEC_TAU_MAX);
                float res[4];
                steps += march(&tr, o, r, tau, res);
                sout[0] = res[0]; sout[1] = res[1]; sout[2] = res[2]; sout[3] = res[3];
            } else {
                sout[0] = sout[1] = sout[2] = sout[3] = 0.0f;
            }
            if (steps_px) steps_px[i] = steps;
            total += steps;
        }
    }
    return total;
}
