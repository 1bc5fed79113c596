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

// [world][max_tiles][64*64] rank-compact tiles -> [h][w] frame
__global__ void __launch_bounds__(256) k_untile(const float4* __restrict__ g, int w, int h, int world,
                                                int tiles_x, int max_tiles, float4* __restrict__ frame) {
    const int x = blockIdx.x * 16 + (threadIdx.x & 15);
    const int y = blockIdx.y * 16 + (threadIdx.x >> 4);
    if (x >= w || y >= h) return;
    const int t = (y / VCT_TILE) * tiles_x + (x / VCT_TILE);
    const int rank = t % world, lt = t / world;
    const size_t src = ((size_t)rank * max_tiles + lt) * (VCT_TILE * VCT_TILE) +
                       (size_t)(y % VCT_TILE) * VCT_TILE + (x % VCT_TILE);
    frame[(size_t)y * w + x] = g[src];
}

// ---- G-buffer ray caster (input producer for synthetic scenes) -----------
struct RayK {
    const float4* tri;  // [n][4]: v0, e1, e2, kd
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

__global__ void __launch_bounds__(256) k_raycast(RayK k) {
    __shared__ float4 sh[kRayChunk * 4];
    const int x = blockIdx.x * 16 + (threadIdx.x & 15);
    const int y = blockIdx.y * 16 + (threadIdx.x >> 4);
    const float ndx = (2.0f * ((float)x + 0.5f) / (float)k.w - 1.0f) * k.tan_half * k.aspect;
    const float ndy = (1.0f - 2.0f * ((float)y + 0.5f) / (float)k.h) * k.tan_half;
    float dx = k.fx + ndx * k.rx + ndy * k.ux;
    float dy = k.fy + ndx * k.ry + ndy * k.uy;
    float dz = k.fz + ndx * k.rz + ndy * k.uz;
    const float il = 1.0f / sqrtf(dot3(dx, dy, dz, dx, dy, dz));
    dx *= il; dy *= il; dz *= il;
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
            const float4 v0 = sh[4 * j], e1 = sh[4 * j + 1], e2 = sh[4 * j + 2];
            const float pvx = dy * e2.z - dz * e2.y, pvy = dz * e2.x - dx * e2.z, pvz = dx * e2.y - dy * e2.x;
            const float det = dot3(e1.x, e1.y, e1.z, pvx, pvy, pvz);
            if (fabsf(det) < 1e-12f) continue;
            const float inv = 1.0f / det;
            const float tx = k.px - v0.x, ty = k.py - v0.y, tz = k.pz - v0.z;
            const float u = dot3(tx, ty, tz, pvx, pvy, pvz) * inv;
            if (u < 0.0f || u > 1.0f) continue;
            const float qx = ty * e1.z - tz * e1.y, qy = tz * e1.x - tx * e1.z, qz = tx * e1.y - ty * e1.x;
            const float v = dot3(dx, dy, dz, qx, qy, qz) * inv;
            if (v < 0.0f || u + v > 1.0f) continue;
            const float t = dot3(e2.x, e2.y, e2.z, qx, qy, qz) * inv;
            if (t > 0.0f && t < best) { best = t; hit = (int)(base + j); }
        }
    }
    if (x >= k.w || y >= k.h) return;
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
    k.alb[p] = make_float4(kd.x, kd.y, kd.z, k.rough);
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

}  // namespace

uint32_t tiles_for_rank(uint32_t w, uint32_t h, uint32_t rank, uint32_t world) {
    if (world == 0) world = 1;
    const uint32_t tx = (w + VCT_TILE - 1) / VCT_TILE, ty = (h + VCT_TILE - 1) / VCT_TILE;
    const uint32_t total = tx * ty;
    if (rank >= world || total <= rank) return 0;
    return (total - rank + world - 1) / world;
}

hipError_t launch_untile(vct_ctx* c, const float4* gathered, uint32_t w, uint32_t h, uint32_t world,
                         float4* frame) {
    if (world == 0) world = 1;
    const int tiles_x = (int)((w + VCT_TILE - 1) / VCT_TILE);
    const int max_tiles = (int)tiles_for_rank(w, h, 0, world);
    dim3 grid((w + 15) / 16, (h + 15) / 16);
    hipLaunchKernelGGL(k_untile, grid, dim3(256), 0, c->stream, gathered, (int)w, (int)h, (int)world,
                       tiles_x, max_tiles, frame);
    return hipGetLastError();
}

hipError_t launch_raycast(vct_ctx* c, const vct_camera* cam, uint32_t w, uint32_t h, float rough,
                          float4* pos, float4* nrm, float4* alb) {
    RayK k;
    k.tri = c->mesh.tri; k.n_tri = c->mesh.n_tri;
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
    dim3 grid((w + 15) / 16, (h + 15) / 16);
    hipLaunchKernelGGL(k_raycast, grid, dim3(256), 0, c->stream, k);
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
