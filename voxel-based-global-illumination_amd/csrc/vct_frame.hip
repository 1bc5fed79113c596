// vct_frame.hip — frame-level kernels around the cone trace:
//  * k_untile: scatters all-gathered rank-compact 64x64 tiles back into the
//    framebuffer (multi-GPU screen tiling);
//  * k_raycast: the G-buffer producer for the synthetic scenes (SURVEY.md 8d
//    G_scene; 8f row f2 replaces it with a rasterizer for mesh scenes).  It
//    follows the reference camera conventions (camera.cpp:24-27,
//    r_voxelization.cpp:18): vertical FOV = Zoom, aspect w/h, near 0.1, far 100.
#include "vct_internal.h"

namespace vct {
namespace {

// [world][planes][max_tiles][64*64] rank-compact tiles -> planes x [h][w] frame
// (blockIdx.z = plane; each rank's planes are contiguous, as one all-gather of
// the rank's [planes][max_tiles*64*64] buffer lays them out)
// packed = 1: rank r's [planes][tiles(r)][64*64] block starts at tile offset
// planes * prefix(r) with no padding (the gather-to-the-presenting-rank layout:
// every rank sends exactly its own tiles); tiles(r) = q + (r < rem), prefix(r) =
// r q + min(r, rem) for T = q world + rem tiles.
struct UntileK {
    const float4* g;
    float4* frame[kMaxUntilePlanes];
    int w, h, world, tiles_x, max_tiles, planes, packed, q, rem;
};

__global__ void __launch_bounds__(256) k_untile(const UntileK k) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15);
    const int y = blockIdx.y * 16 + (threadIdx.x >> 4);
    const int p = blockIdx.z;
    if (x >= k.w || y >= k.h) return;
    const int t = (y / VCT_TILE) * k.tiles_x + (x / VCT_TILE);
    const int rank = t % k.world, lt = t / k.world;
    size_t tile0;   // first tile of (rank, plane) in the gathered buffer
    if (k.packed) {
        const int nt = k.q + (rank < k.rem ? 1 : 0), pre = rank * k.q + min(rank, k.rem);
        tile0 = (size_t)k.planes * pre + (size_t)p * nt;
    } else {
        tile0 = ((size_t)rank * k.planes + p) * k.max_tiles;
    }
    const size_t src = (tile0 + lt) * (VCT_TILE * VCT_TILE) + (size_t)(y % VCT_TILE) * VCT_TILE + (x % VCT_TILE);
    k.frame[p][(size_t)y * k.w + x] = k.g[src];
}

// ---- G-buffer ray caster (input producer for synthetic scenes) -----------
struct RayK {
    const float4* tri;  // [n][4]: v0, e1, e2, (kd, diffuse map as int bits)
    const float4* uv;   // [n][2] TexCoords of textured triangles (NULL: untextured voxelization)
    const uint32_t* texels;   // diffuse maps (vct_set_textures)
    const TexDesc* tdesc;
    uint32_t n_tex;
    uint32_t n_tri;
    int w, h;
    float px, py, pz;
    float fx, fy, fz, ux, uy, uz, rx, ry, rz;
    float tan_half, aspect, near_p, far_p, rough;
    float4* pos;
    float4* nrm;
    float4* alb;
};

constexpr int kRayChunk = 256;

// Moller-Trumbore: ray parameter t of the hit, or -1 (no hit / parallel)
__device__ __forceinline__ float ray_tri(float4 v0, float4 e1, float4 e2, float px, float py, float pz, float dx,
                                         float dy, float dz) {
    const float pvx = dy * e2.z - dz * e2.y, pvy = dz * e2.x - dx * e2.z, pvz = dx * e2.y - dy * e2.x;
    const float det = dot3(e1.x, e1.y, e1.z, pvx, pvy, pvz);
    if (fabsf(det) < 1e-12f) return -1.0f;
    const float inv = 1.0f / det;
    const float tx = px - v0.x, ty = py - v0.y, tz = pz - v0.z;
    const float u = dot3(tx, ty, tz, pvx, pvy, pvz) * inv;
    if (u < 0.0f || u > 1.0f) return -1.0f;
    const float qx = ty * e1.z - tz * e1.y, qy = tz * e1.x - tx * e1.z, qz = tx * e1.y - ty * e1.x;
    const float v = dot3(dx, dy, dz, qx, qy, qz) * inv;
    if (v < 0.0f || u + v > 1.0f) return -1.0f;
    return dot3(e2.x, e2.y, e2.z, qx, qy, qz) * inv;
}

// Moller-Trumbore barycentrics (u, v) of a ray known to hit the triangle (ray_tri's operations)
__device__ __forceinline__ void ray_tri_bary(float4 v0, float4 e1, float4 e2, float px, float py, float pz, float dx,
                                             float dy, float dz, float& u, float& v) {
    const float pvx = dy * e2.z - dz * e2.y, pvy = dz * e2.x - dx * e2.z, pvz = dx * e2.y - dy * e2.x;
    const float det = dot3(e1.x, e1.y, e1.z, pvx, pvy, pvz);
    const float inv = 1.0f / det;
    const float tx = px - v0.x, ty = py - v0.y, tz = pz - v0.z;
    u = dot3(tx, ty, tz, pvx, pvy, pvz) * inv;
    const float qx = ty * e1.z - tz * e1.y, qy = tz * e1.x - tx * e1.z, qz = tx * e1.y - ty * e1.x;
    v = dot3(dx, dy, dz, qx, qy, qz) * inv;
}

// pixel (x, y) -> unit ray direction (row 0 = top; reference camera, r_voxelization.cpp:16-23)
__device__ __forceinline__ void pixel_ray(const RayK& k, int x, int y, float& dx, float& dy, float& dz) {
    const float ndx = (2.0f * ((float)x + 0.5f) / (float)k.w - 1.0f) * k.tan_half * k.aspect;
    const float ndy = (1.0f - 2.0f * ((float)y + 0.5f) / (float)k.h) * k.tan_half;
    dx = k.fx + ndx * k.rx + ndy * k.ux;
    dy = k.fy + ndx * k.ry + ndy * k.uy;
    dz = k.fz + ndx * k.rz + ndy * k.uz;
    const float il = 1.0f / sqrtf(dot3(dx, dy, dz, dx, dy, dz));
    dx *= il; dy *= il; dz *= il;
}

// G-buffer texel of the nearest hit (shared by the brute-force and the binned pass)
__device__ __forceinline__ void write_gbuffer(const RayK& k, int x, int y, float dx, float dy, float dz, float best,
                                              int hit) {
    const size_t p = (size_t)y * k.w + x;
    const float depth = best * dot3(dx, dy, dz, k.fx, k.fy, k.fz);
    if (hit < 0 || depth < k.near_p || depth > k.far_p) {
        k.pos[p] = make_float4(0, 0, 0, 0);
        k.nrm[p] = make_float4(0, 0, 0, 0);
        k.alb[p] = make_float4(0, 0, 0, k.rough);
        return;
    }
    const float4 e1 = k.tri[(size_t)hit * 4 + 1], e2 = k.tri[(size_t)hit * 4 + 2], kd = k.tri[(size_t)hit * 4 + 3];
    float nx = e1.y * e2.z - e1.z * e2.y, ny = e1.z * e2.x - e1.x * e2.z, nz = e1.x * e2.y - e1.y * e2.x;
    const float nl = sqrtf(dot3(nx, ny, nz, nx, ny, nz));
    nx /= nl; ny /= nl; nz /= nl;
    if (dot3(nx, ny, nz, dx, dy, dz) > 0.0f) { nx = -nx; ny = -ny; nz = -nz; }
    k.pos[p] = make_float4(k.px + dx * best, k.py + dy * best, k.pz + dz * best, 1.0f);
    k.nrm[p] = make_float4(nx, ny, nz, 0.0f);
    float ar = kd.x, ag = kd.y, ab = kd.z;
    const int tex = __float_as_int(kd.w);
    if (k.uv && tex >= 0 && (uint32_t)tex < k.n_tex) {   // albedo = Kd x T(uv of the hit)
        float b1, b2, u, v, tr, tg, tb;
        ray_tri_bary(k.tri[(size_t)hit * 4], e1, e2, k.px, k.py, k.pz, dx, dy, dz, b1, b2);
        const float4 a = k.uv[(size_t)hit * 2], b = k.uv[(size_t)hit * 2 + 1];
        const float uv[6] = {a.x, a.y, a.z, a.w, b.x, b.y};
        tri_uv(uv, b1, b2, u, v);
        tex_sample(k.texels, k.tdesc[tex], u, v, tr, tg, tb);
        ar = kd.x * tr; ag = kd.y * tg; ab = kd.z * tb;
    }
    k.alb[p] = make_float4(ar, ag, ab, k.rough);
}

__global__ void __launch_bounds__(256) k_raycast(RayK k) {
    __shared__ float4 sh[kRayChunk * 4];
    const int x = blockIdx.x * 16 + (threadIdx.x & 15);
    const int y = blockIdx.y * 16 + (threadIdx.x >> 4);
    float dx, dy, dz;
    pixel_ray(k, x, y, dx, dy, dz);
    float best = __builtin_inff();
    int hit = -1;
    for (uint32_t base = 0; base < k.n_tri; base += kRayChunk) {
        __syncthreads();
        for (int i = threadIdx.x; i < kRayChunk * 4; i += 256) {
            uint32_t tri = base + i / 4;
            sh[i] = tri < k.n_tri ? k.tri[(size_t)tri * 4 + (i & 3)] : make_float4(0, 0, 0, 0);
        }
        __syncthreads();
        const uint32_t cnt = min((uint32_t)kRayChunk, k.n_tri - base);
        for (uint32_t j = 0; j < cnt; ++j) {
            const float t = ray_tri(sh[4 * j], sh[4 * j + 1], sh[4 * j + 2], k.px, k.py, k.pz, dx, dy, dz);
            if (t > 0.0f && t < best) { best = t; hit = (int)(base + j); }
        }
    }
    if (x >= k.w || y >= k.h) return;
    write_gbuffer(k, x, y, dx, dy, dz, best, hit);
}

// ---- tile-binned G-buffer pass ------------------------
// Screen-space binning of the triangles into 16x16-pixel tiles (projected
// through the reference camera; clipped to cz >= 1e-5 so the bounding boxes are
// conservative), then one workgroup per tile intersects its pixels' rays with
// the tile's triangles only.  Ties in t go to the lower triangle index, so the
// result equals the brute-force caster's bit for bit, at O(px x tris per tile).
constexpr int kGT = 16;

struct BinK {
    RayK r;
    int tiles_x, tiles_y;
    float sxs, sys;                // pixel scale: X = w/2 + (cx/cz) sxs, Y = h/2 - (cy/cz) sys
    int4* rect;                    // per triangle tile rectangle (x0 > x1: culled)
    uint32_t* count;               // per tile: triangles, then the fill cursor
    uint32_t* offset;              // per tile: exclusive prefix of count; [n_tiles] = total
    uint32_t* bins;                // triangle indices grouped by tile
};

__global__ void __launch_bounds__(256) k_bin_rect(BinK k) {
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    if (t >= k.r.n_tri) return;
    const RayK& r = k.r;
    const float4 v0 = r.tri[(size_t)t * 4], e1 = r.tri[(size_t)t * 4 + 1], e2 = r.tri[(size_t)t * 4 + 2];
    float c[3][3];
    const float vx[3] = {v0.x, v0.x + e1.x, v0.x + e2.x}, vy[3] = {v0.y, v0.y + e1.y, v0.y + e2.y},
                vz[3] = {v0.z, v0.z + e1.z, v0.z + e2.z};
    for (int i = 0; i < 3; ++i) {
        const float qx = vx[i] - r.px, qy = vy[i] - r.py, qz = vz[i] - r.pz;
        c[i][0] = dot3(qx, qy, qz, r.rx, r.ry, r.rz);
        c[i][1] = dot3(qx, qy, qz, r.ux, r.uy, r.uz);
        c[i][2] = dot3(qx, qy, qz, r.fx, r.fy, r.fz);
    }
    // clip the triangle to cz >= zc (Sutherland-Hodgman, one plane), project the polygon
    const float zc = 1e-5f;
    float lo_x = __builtin_inff(), lo_y = __builtin_inff(), hi_x = -__builtin_inff(), hi_y = -__builtin_inff();
    bool any = false, beyond = true;
    for (int i = 0; i < 3; ++i) {
        const float* a = c[i];
        const float* b = c[(i + 1) % 3];
        beyond &= a[2] > r.far_p;
        const bool ina = a[2] >= zc, inb = b[2] >= zc;
        float p[2][3];
        int np = 0;
        if (ina) { p[np][0] = a[0]; p[np][1] = a[1]; p[np][2] = a[2]; ++np; }
        if (ina != inb) {
            const float s = (zc - a[2]) / (b[2] - a[2]);
            p[np][0] = a[0] + (b[0] - a[0]) * s; p[np][1] = a[1] + (b[1] - a[1]) * s; p[np][2] = zc; ++np;
        }
        for (int j = 0; j < np; ++j) {
            const float X = 0.5f * (float)r.w + (p[j][0] / p[j][2]) * k.sxs;
            const float Y = 0.5f * (float)r.h - (p[j][1] / p[j][2]) * k.sys;
            lo_x = fminf(lo_x, X); hi_x = fmaxf(hi_x, X); lo_y = fminf(lo_y, Y); hi_y = fmaxf(hi_y, Y);
            any = true;
        }
    }
    int4 rc = make_int4(1, 0, 0, 0);   // culled
    if (any && !beyond) {
        // one pixel of margin, pixel centres at +0.5
        const float x0 = fmaxf(lo_x - 1.5f, 0.0f), x1 = fminf(hi_x + 0.5f, (float)(r.w - 1));
        const float y0 = fmaxf(lo_y - 1.5f, 0.0f), y1 = fminf(hi_y + 0.5f, (float)(r.h - 1));
        if (x0 <= x1 && y0 <= y1)
            rc = make_int4((int)x0 / kGT, (int)y0 / kGT, (int)x1 / kGT, (int)y1 / kGT);
    }
    k.rect[t] = rc;
    for (int ty = rc.y; ty <= rc.w && rc.x <= rc.z; ++ty)
        for (int tx = rc.x; tx <= rc.z; ++tx) atomicAdd(&k.count[ty * k.tiles_x + tx], 1u);
}

// exclusive scan of the tile counts (one workgroup; n_tiles <= 64K at 4K), count -> 0 (fill cursor)
__global__ void __launch_bounds__(1024) k_bin_scan(uint32_t* count, uint32_t* offset, uint32_t n) {
    __shared__ uint32_t part[1024];
    const uint32_t per = (n + 1023) / 1024, lo = threadIdx.x * per, hi = min(lo + per, n);
    uint32_t s = 0;
    for (uint32_t i = lo; i < hi; ++i) s += count[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
        const uint32_t v = threadIdx.x >= d ? part[threadIdx.x - d] : 0u;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = part[threadIdx.x] - s;
    for (uint32_t i = lo; i < hi; ++i) {
        offset[i] = run;
        run += count[i];
        count[i] = 0u;
    }
    if (threadIdx.x == 1023) offset[n] = part[1023];
}

__global__ void __launch_bounds__(256) k_bin_fill(BinK k) {
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    if (t >= k.r.n_tri) return;
    const int4 rc = k.rect[t];
    for (int ty = rc.y; ty <= rc.w && rc.x <= rc.z; ++ty)
        for (int tx = rc.x; tx <= rc.z; ++tx) {
            const int tile = ty * k.tiles_x + tx;
            k.bins[k.offset[tile] + atomicAdd(&k.count[tile], 1u)] = t;
        }
}

__global__ void __launch_bounds__(256) k_bin_raster(BinK k) {
    __shared__ float4 sh[kRayChunk * 3];
    __shared__ uint32_t sid[kRayChunk];
    const RayK& r = k.r;
    const int tile = (int)blockIdx.x;
    const int x = (tile % k.tiles_x) * kGT + (int)(threadIdx.x & 15);
    const int y = (tile / k.tiles_x) * kGT + (int)(threadIdx.x >> 4);
    float dx, dy, dz;
    pixel_ray(r, x, y, dx, dy, dz);
    float best = __builtin_inff();
    int hit = -1;
    const uint32_t beg = k.offset[tile], end = k.offset[tile + 1];
    for (uint32_t base = beg; base < end; base += kRayChunk) {
        __syncthreads();
        const uint32_t cnt = min((uint32_t)kRayChunk, end - base);
        if (threadIdx.x < cnt) {
            const uint32_t t = k.bins[base + threadIdx.x];
            sid[threadIdx.x] = t;
            sh[3 * threadIdx.x] = r.tri[(size_t)t * 4];
            sh[3 * threadIdx.x + 1] = r.tri[(size_t)t * 4 + 1];
            sh[3 * threadIdx.x + 2] = r.tri[(size_t)t * 4 + 2];
        }
        __syncthreads();
        for (uint32_t j = 0; j < cnt; ++j) {
            const float t = ray_tri(sh[3 * j], sh[3 * j + 1], sh[3 * j + 2], r.px, r.py, r.pz, dx, dy, dz);
            const int id = (int)sid[j];
            if (t > 0.0f && (t < best || (t == best && id < hit))) { best = t; hit = id; }
        }
    }
    if (x >= r.w || y >= r.h) return;
    write_gbuffer(r, x, y, dx, dy, dz, best, hit);
}

// ---- composite + present (spec in vct_spec.h) ------------
struct CompK {
    const float4 *pos, *nrm, *alb, *diff, *spec;
    const unsigned long long* bits;
    int n, w, h;
    float g0x, g0y, g0z, inv_h;
    float lx, ly, lz, cr, cg, cb;
    float4* lin;
    uint32_t* rgba8;
};

__device__ __forceinline__ uint32_t to8(float v) {   // Reinhard, gamma 1/2.2, round half away
    v = v / (1.0f + v);
    v = powf(v < 0.0f ? 0.0f : v, VCT_INV_GAMMA);
    const int q = (int)lroundf(v * 255.0f);
    return (uint32_t)(q < 0 ? 0 : (q > 255 ? 255 : q));
}

__global__ void __launch_bounds__(256) k_composite(CompK k) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= (uint32_t)k.w * (uint32_t)k.h) return;
    const float4 P = k.pos[i];
    if (P.w == 0.0f) {   // background: the reference's clear colour
        if (k.lin) k.lin[i] = make_float4(VCT_CLEAR_R, VCT_CLEAR_G, VCT_CLEAR_B, 0.0f);
        if (k.rgba8)
            k.rgba8[i] = (uint32_t)lroundf(VCT_CLEAR_R * 255.0f) | ((uint32_t)lroundf(VCT_CLEAR_G * 255.0f) << 8) |
                         ((uint32_t)lroundf(VCT_CLEAR_B * 255.0f) << 16) | (255u << 24);
        return;
    }
    const float4 N = k.nrm[i], A = k.alb[i], D = k.diff[i], S = k.spec[i];
    const float ndl = dot3(N.x, N.y, N.z, k.lx, k.ly, k.lz);
    float dr = 0.0f, dg = 0.0f, db = 0.0f;
    if (ndl > 0.0f) {
        const float vis = dda_visibility(k.bits, k.n, (P.x - k.g0x) * k.inv_h + N.x, (P.y - k.g0y) * k.inv_h + N.y,
                                         (P.z - k.g0z) * k.inv_h + N.z, k.lx, k.ly, k.lz);
        dr = ((A.x * k.cr) * ndl) * vis;
        dg = ((A.y * k.cg) * ndl) * vis;
        db = ((A.z * k.cb) * ndl) * vis;
    }
    const float fr = (dr + A.x * D.x) + S.x, fg = (dg + A.y * D.y) + S.y, fb = (db + A.z * D.z) + S.z;
    if (k.lin) k.lin[i] = make_float4(fr, fg, fb, 1.0f);
    if (k.rgba8) k.rgba8[i] = to8(fr) | (to8(fg) << 8) | (to8(fb) << 16) | (255u << 24);
}

__global__ void k_add_counters(const unsigned long long* __restrict__ src, uint32_t n, unsigned long long* dst0,
                               unsigned long long* dst1) {
    if (threadIdx.x != 0) return;
    unsigned long long a = 0, b = 0;
    for (uint32_t i = 0; i < n; ++i) {
        a += src[2 * i];
        b += src[2 * i + 1];
    }
    if (dst0) *dst0 += a;
    if (dst1) *dst1 += b;
}

}  // namespace

uint32_t tiles_for_rank(uint32_t w, uint32_t h, uint32_t rank, uint32_t world) {
    if (world == 0) world = 1;
    const uint32_t tx = (w + VCT_TILE - 1) / VCT_TILE, ty = (h + VCT_TILE - 1) / VCT_TILE;
    const uint32_t total = tx * ty;
    if (rank >= world || total <= rank) return 0;
    return (total - rank + world - 1) / world;
}

hipError_t launch_untile(vct_ctx* c, const float4* gathered, uint32_t planes, uint32_t w, uint32_t h,
                         uint32_t world, float4* const* frames, bool packed) {
    if (world == 0) world = 1;
    UntileK k{};
    const uint32_t total = ((w + VCT_TILE - 1) / VCT_TILE) * ((h + VCT_TILE - 1) / VCT_TILE);
    k.packed = packed ? 1 : 0;
    k.q = (int)(total / world);
    k.rem = (int)(total % world);
    k.g = gathered;
    for (uint32_t p = 0; p < planes; ++p) k.frame[p] = frames[p];
    k.w = (int)w; k.h = (int)h; k.world = (int)world; k.planes = (int)planes;
    k.tiles_x = (int)((w + VCT_TILE - 1) / VCT_TILE);
    k.max_tiles = (int)tiles_for_rank(w, h, 0, world);
    dim3 grid((w + 15) / 16, (h + 15) / 16, planes);
    hipLaunchKernelGGL(k_untile, grid, dim3(256), 0, c->stream, k);
    return hipGetLastError();
}

hipError_t launch_add_counters(vct_ctx* c, const unsigned long long* src, uint32_t n, unsigned long long* dst0,
                               unsigned long long* dst1) {
    hipLaunchKernelGGL(k_add_counters, dim3(1), dim3(64), 0, c->stream, src, n, dst0, dst1);
    return hipGetLastError();
}

static RayK ray_params(vct_ctx* c, const vct_camera* cam, uint32_t w, uint32_t h, float rough, float4* pos,
                       float4* nrm, float4* alb) {
    RayK k;
    k.tri = c->mesh.tri; k.n_tri = c->mesh.n_tri;
    k.uv = c->mesh.textured ? c->mesh.uv : nullptr;
    k.texels = c->tex.texels; k.tdesc = c->tex.desc; k.n_tex = c->tex.n;
    k.w = (int)w; k.h = (int)h;
    k.px = cam->position[0]; k.py = cam->position[1]; k.pz = cam->position[2];
    k.fx = cam->front[0]; k.fy = cam->front[1]; k.fz = cam->front[2];
    k.ux = cam->up[0]; k.uy = cam->up[1]; k.uz = cam->up[2];
    k.rx = cam->right[0]; k.ry = cam->right[1]; k.rz = cam->right[2];
    k.tan_half = tanf(cam->zoom_deg * 0.5f * 3.14159265358979f / 180.0f);
    k.aspect = (float)w / (float)h;
    k.near_p = cam->near_plane; k.far_p = cam->far_plane;
    k.rough = rough;
    k.pos = pos; k.nrm = nrm; k.alb = alb;
    return k;
}

hipError_t launch_raycast(vct_ctx* c, const vct_camera* cam, uint32_t w, uint32_t h, float rough,
                          float4* pos, float4* nrm, float4* alb) {
    const RayK k = ray_params(c, cam, w, h, rough, pos, nrm, alb);
    dim3 grid((w + 15) / 16, (h + 15) / 16);
    hipLaunchKernelGGL(k_raycast, grid, dim3(256), 0, c->stream, k);
    return hipGetLastError();
}

hipError_t launch_gbuffer_binned(vct_ctx* c, const vct_camera* cam, uint32_t w, uint32_t h, float rough,
                                 float4* pos, float4* nrm, float4* alb) {
    BinK k;
    k.r = ray_params(c, cam, w, h, rough, pos, nrm, alb);
    k.tiles_x = (int)((w + kGT - 1) / kGT);
    k.tiles_y = (int)((h + kGT - 1) / kGT);
    k.sxs = 0.5f * (float)w / (k.r.tan_half * k.r.aspect);
    k.sys = 0.5f * (float)h / k.r.tan_half;
    const uint32_t n_tiles = (uint32_t)(k.tiles_x * k.tiles_y), n_tri = c->mesh.n_tri;
    const size_t b_rect = ((size_t)n_tri * sizeof(int4) + 255) & ~(size_t)255;
    const size_t b_cnt = ((size_t)n_tiles * 4 + 255) & ~(size_t)255;
    void* sp;
    hipError_t e;
    if ((e = scratch_get(c, 2, b_rect + b_cnt + (size_t)(n_tiles + 1) * 4, &sp)) != hipSuccess) return e;
    k.rect = (int4*)sp;
    k.count = (uint32_t*)((char*)sp + b_rect);
    k.offset = (uint32_t*)((char*)sp + b_rect + b_cnt);
    if ((e = hipMemsetAsync(k.count, 0, (size_t)n_tiles * 4, c->stream)) != hipSuccess) return e;
    const uint32_t tb = (n_tri + 255) / 256;
    if (n_tri) hipLaunchKernelGGL(k_bin_rect, dim3(tb), dim3(256), 0, c->stream, k);
    hipLaunchKernelGGL(k_bin_scan, dim3(1), dim3(1024), 0, c->stream, k.count, k.offset, n_tiles);
    uint32_t total = 0;   // bin storage is sized on the host (one small read back per frame)
    if ((e = hipMemcpyAsync(&total, k.offset + n_tiles, 4, hipMemcpyDeviceToHost, c->stream)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return e;
    if ((e = scratch_get(c, 3, (size_t)(total ? total : 1) * 4, &sp)) != hipSuccess) return e;
    k.bins = (uint32_t*)sp;
    if (n_tri && total) hipLaunchKernelGGL(k_bin_fill, dim3(tb), dim3(256), 0, c->stream, k);
    hipLaunchKernelGGL(k_bin_raster, dim3(n_tiles), dim3(256), 0, c->stream, k);
    return hipGetLastError();
}

hipError_t launch_composite(vct_ctx* c, const float4* pos, const float4* nrm, const float4* alb,
                            const float4* diff, const float4* spec, uint32_t w, uint32_t h, const float l[3],
                            const float color[3], float4* lin, uint32_t* rgba8) {
    const Grid& g = c->grid;
    CompK k;
    k.pos = pos; k.nrm = nrm; k.alb = alb; k.diff = diff; k.spec = spec;
    k.bits = g.occ_bits;
    k.n = (int)g.n; k.w = (int)w; k.h = (int)h;
    k.g0x = g.g0[0]; k.g0y = g.g0[1]; k.g0z = g.g0[2]; k.inv_h = g.inv_h;
    k.lx = l[0]; k.ly = l[1]; k.lz = l[2];
    k.cr = color[0]; k.cg = color[1]; k.cb = color[2];
    k.lin = lin; k.rgba8 = rgba8;
    const uint32_t px = w * h;
    hipLaunchKernelGGL(k_composite, dim3((px + 255) / 256), dim3(256), 0, c->stream, k);
    return hipGetLastError();
}

}  // namespace vct
