// vct_trace.hip — K4 per-pixel diffuse + specular cone trace (the metric kernel),
// the multi-GPU tile un-permute, and the G-buffer ray caster.
//
// SURVEY.md Appendix A.5 / A.6.  The reference has no cone tracer: its only GPU
// program is the forward textured draw of assets/code/shader/test.{vert,frag},
// invoked by VoxelizationRenderer::Render (assets/code/renderer/r_voxelization.cpp:4-35).
//
// MI355X design of K4 (memory-gather bound, no MFMA):
//  * one lane = one pixel; a 64-lane wave is an 8x8 pixel block and a
//    256-thread workgroup a 16x16 block, so a wave's cones start at nearly the
//    same voxel and march in nearly the same direction: the texel footprint of
//    the 64 lanes overlaps heavily and is served from the CU's L1 / the XCD's L2;
//  * the screen is cut into 64x64 tiles; tile t belongs to rank t % world
//    (SURVEY 8e), and inside a rank the workgroup -> tile map is XCD-aware: the
//    eight round-robin XCD groups each get one contiguous run of tiles, so
//    neighbouring workgroups (which gather the same bricks) share an L2;
//  * diffuse cones have a wave-uniform step sequence (t, D and the mip pair
//    depend only on tau), so the level branch is uniform and the per-lane
//    early-out (a >= 0.95, left the grid) only masks lanes;
//  * texels are 16-byte RGBA32F gathers (global_load_dwordx4), zero border by
//    zeroed weights on clamped addresses (no out-of-bounds access, no branch).
#include "vct_internal.h"

// Debug-build counters (make dbg -> vct/libvct_hip_dbg.so): per wave-step path
// statistics of the LDS variants, read with vct_debug_counters().  Compiled out
// of the product library.
#ifdef VCT_DEBUG_COUNTERS
__device__ unsigned long long vct_dbg_ctr[16];
#define VCT_DBG(i) do { if ((threadIdx.x & 63) == 0) atomicAdd(&vct_dbg_ctr[i], 1ull); } while (0)
#else
#define VCT_DBG(i) do { } while (0)
#endif

extern "C" __device__ int __ockl_wfred_min_i32(int);   // wave-wide reductions over active lanes (ockl)
extern "C" __device__ float __ockl_wfred_min_f32(float);
extern "C" __device__ float __ockl_wfred_max_f32(float);

namespace vct {
namespace {

#define VCT_CROW(cn, ct, cb, w) {cn, ct, cb, w},
__constant__ float c_cones1[1][4] = {VCT_CONES1(VCT_CROW)};
__constant__ float c_cones9[9][4] = {VCT_CONES9(VCT_CROW)};
__constant__ float c_cones16[16][4] = {VCT_CONES16(VCT_CROW)};

struct TraceK {
    const float4* pyr;
    const float4* zero;      // one zero texel (the zero border for LDS-DMA staging)
    uint64_t lvl_off[kMaxLevels + 1];
    int n, L;
    float g0x, g0y, g0z, inv_h, tmax;
    const float4* pos;
    const float4* nrm;
    const float4* alb;
    float4* diff;
    float4* spec;
    uint32_t* steps_px;
    unsigned long long* steps_total;
    unsigned long long* texels_total;
    int w, h;
    float ex, ey, ez;
    int tiles_x, rank, world, n_local_tiles, compact;
    int nd, spec_on, aniso;
    int brick_log2;          // largest staged brick: 2^brick_log2 texels (6..8)
    float tau_d;
};

// trilinear weights + clamped corner indices of one level (GL texel centres)
struct Tri {
    uint32_t i[8];
    float wc[8];
};

__device__ __forceinline__ void tri_setup(int nl, float cx, float cy, float cz, Tri& t) {
    float fx0 = floorf(cx), fy0 = floorf(cy), fz0 = floorf(cz);
    int ix = (int)fx0, iy = (int)fy0, iz = (int)fz0;
    float fx = cx - fx0, fy = cy - fy0, fz = cz - fz0;
    float wx[2] = {1.0f - fx, fx}, wy[2] = {1.0f - fy, fy}, wz[2] = {1.0f - fz, fz};
    int xs[2] = {ix, ix + 1}, ys[2] = {iy, iy + 1}, zs[2] = {iz, iz + 1};
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        if ((unsigned)xs[k] >= (unsigned)nl) { wx[k] = 0.0f; xs[k] = 0; }
        if ((unsigned)ys[k] >= (unsigned)nl) { wy[k] = 0.0f; ys[k] = 0; }
        if ((unsigned)zs[k] >= (unsigned)nl) { wz[k] = 0.0f; zs[k] = 0; }
    }
#pragma unroll
    for (int dz = 0; dz < 2; ++dz)
#pragma unroll
        for (int dy = 0; dy < 2; ++dy)
#pragma unroll
            for (int dx = 0; dx < 2; ++dx) {
                const int c = dz * 4 + dy * 2 + dx;
                t.i[c] = (uint32_t)xs[dx] + (uint32_t)nl * ((uint32_t)ys[dy] + (uint32_t)nl * (uint32_t)zs[dz]);
                t.wc[c] = (wx[dx] * wy[dy]) * wz[dz];
            }
}

__device__ __forceinline__ float4 tri_gather(const float4* __restrict__ vol, const Tri& t) {
    float4 v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = vol[t.i[c]];
    float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        acc.x = fmaf(t.wc[c], v[c].x, acc.x);
        acc.y = fmaf(t.wc[c], v[c].y, acc.y);
        acc.z = fmaf(t.wc[c], v[c].z, acc.z);
        acc.w = fmaf(t.wc[c], v[c].w, acc.w);
    }
    return acc;
}

// D_l(q, d) (A.5): level 0 isotropic, level >= 1 directional over 3 faces.
// s = fmaf(wd_z, T_z, fmaf(wd_y, T_y, wd_x * T_x)) written as a face loop that
// starts from 0 (fmaf(w, t, 0) == w * t); one face's 8 gathers are live at a time.
__device__ __forceinline__ float4 sample_level(const TraceK& k, int l, float qx, float qy, float qz,
                                               int fx, int fy, int fz, float wdx, float wdy, float wdz) {
    const float scale = __uint_as_float((uint32_t)(127 - l) << 23);  // 2^-l, exact
    const int nl = k.n >> l;
    Tri t;
    tri_setup(nl, qx * scale - 0.5f, qy * scale - 0.5f, qz * scale - 0.5f, t);
    const float4* lvl = k.pyr + k.lvl_off[l];
    if (l == 0 || !k.aniso) return tri_gather(lvl, t);
    const size_t vl = (size_t)nl * nl * nl;
    float4 s = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll 1
    for (int f = 0; f < 3; ++f) {
        const int face = f == 0 ? fx : (f == 1 ? fy : fz);
        const float w = f == 0 ? wdx : (f == 1 ? wdy : wdz);
        const float4 tf = tri_gather(lvl + (size_t)face * vl, t);
        s.x = fmaf(w, tf.x, s.x);
        s.y = fmaf(w, tf.y, s.y);
        s.z = fmaf(w, tf.z, s.z);
        s.w = fmaf(w, tf.w, s.w);
    }
    return s;
}

// one cone (A.6); returns steps, accumulates (c, a) into res
__device__ __forceinline__ uint32_t march(const TraceK& k, float ox, float oy, float oz, float dx,
                                          float dy, float dz, float tau, float4& res, uint32_t& texels) {
    const float tau2 = 2.0f * tau;
    const float nf = (float)k.n, Lf = (float)k.L;
    const int fx = dx >= 0.0f ? VCT_FACE_PX : VCT_FACE_NX;
    const int fy = dy >= 0.0f ? VCT_FACE_PY : VCT_FACE_NY;
    const int fz = dz >= 0.0f ? VCT_FACE_PZ : VCT_FACE_NZ;
    const float wdx = dx * dx, wdy = dy * dy, wdz = dz * dz;
    float cr = 0.0f, cg = 0.0f, cb = 0.0f, a = 0.0f, t = 1.0f;
    uint32_t steps = 0;
    for (;;) {
        if (!(a < VCT_ALPHA_STOP)) break;
        if (!(t <= k.tmax)) break;
        const float qx = ox + dx * t, qy = oy + dy * t, qz = oz + dz * t;
        if (!(qx >= 0.0f && qx <= nf && qy >= 0.0f && qy <= nf && qz >= 0.0f && qz <= nf)) break;
        const float D = fmaxf(1.0f, tau2 * t);
        float m = spec_log2(D);
        if (m > Lf) m = Lf;
        const int l0 = (int)m;
        const float fr = m - (float)l0;
        float4 s = sample_level(k, l0, qx, qy, qz, fx, fy, fz, wdx, wdy, wdz);
        texels += (l0 == 0 || !k.aniso) ? 8u : 24u;
        if (fr > 0.0f && l0 < k.L) {
            texels += k.aniso ? 24u : 8u;
            float4 s1 = sample_level(k, l0 + 1, qx, qy, qz, fx, fy, fz, wdx, wdy, wdz);
            const float omf = 1.0f - fr;
            s.x = fmaf(fr, s1.x, omf * s.x);
            s.y = fmaf(fr, s1.y, omf * s.y);
            s.z = fmaf(fr, s1.z, omf * s.z);
            s.w = fmaf(fr, s1.w, omf * s.w);
        }
        const float oma = 1.0f - a;
        cr = fmaf(oma, s.x, cr);
        cg = fmaf(oma, s.y, cg);
        cb = fmaf(oma, s.z, cb);
        a = fmaf(oma, s.w, a);
        t = t + VCT_STEP_SCALE * D;
        ++steps;
    }
    res = make_float4(cr, cg, cb, a);
    return steps;
}

__device__ __forceinline__ const float (*cone_table(int nd))[4] {
    return nd == 16 ? c_cones16 : (nd == 9 ? c_cones9 : c_cones1);
}

__global__ void __launch_bounds__(256) k4_trace(TraceK k) {
    // XCD-aware workgroup -> (local tile, 16x16 block) map (bijective for any grid)
    const uint32_t nb = gridDim.x, b = blockIdx.x;
    const uint32_t xcd = b & 7, q = nb >> 3, r = nb & 7;
    const uint32_t rb = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
    const uint32_t lt = rb >> 4, sub = rb & 15;
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t px = (sub & 3) * 16 + (wave & 1) * 8 + (lane & 7);
    const uint32_t py = (sub >> 2) * 16 + (wave >> 1) * 8 + (lane >> 3);
    const uint32_t tile = lt * (uint32_t)k.world + (uint32_t)k.rank;
    const uint32_t x = (tile % (uint32_t)k.tiles_x) * VCT_TILE + px;
    const uint32_t y = (tile / (uint32_t)k.tiles_x) * VCT_TILE + py;
    const bool in_frame = x < (uint32_t)k.w && y < (uint32_t)k.h;
    const size_t pix = (size_t)y * (size_t)k.w + x;
    const size_t oidx = k.compact ? (size_t)lt * (VCT_TILE * VCT_TILE) + py * VCT_TILE + px : pix;

    float4 dout = make_float4(0.0f, 0.0f, 0.0f, 0.0f), sout = dout;
    uint32_t steps = 0, texels = 0;
    float4 P = in_frame ? k.pos[pix] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (P.w != 0.0f) {
        const float4 N4 = k.nrm[pix];
        const float nx = N4.x, ny = N4.y, nz = N4.z;
        const float ox = (P.x - k.g0x) * k.inv_h + nx;
        const float oy = (P.y - k.g0y) * k.inv_h + ny;
        const float oz = (P.z - k.g0z) * k.inv_h + nz;
        // Duff et al. 2017 branchless orthonormal basis
        const float sgn = copysignf(1.0f, nz);
        const float ka = -1.0f / (sgn + nz);
        const float kb = (nx * ny) * ka;
        const float Tx = 1.0f + ((sgn * nx) * nx) * ka, Ty = sgn * kb, Tz = -(sgn * nx);
        const float Bx = kb, By = sgn + (ny * ny) * ka, Bz = -ny;
        const float(*cones)[4] = cone_table(k.nd);
        float ir = 0.0f, ig = 0.0f, ib = 0.0f, occ = 0.0f;
        for (int c = 0; c < k.nd; ++c) {
            const float cn = cones[c][0], ct = cones[c][1], cb = cones[c][2], wk = cones[c][3];
            const float dx = (cn * nx + ct * Tx) + cb * Bx;
            const float dy = (cn * ny + ct * Ty) + cb * By;
            const float dz = (cn * nz + ct * Tz) + cb * Bz;
            float4 res;
            steps += march(k, ox, oy, oz, dx, dy, dz, k.tau_d, res, texels);
            ir = fmaf(wk, res.x, ir);
            ig = fmaf(wk, res.y, ig);
            ib = fmaf(wk, res.z, ib);
            occ = fmaf(wk, res.w, occ);
        }
        dout = make_float4(ir, ig, ib, 1.0f - occ);
        if (k.spec_on) {
            float vx = k.ex - P.x, vy = k.ey - P.y, vz = k.ez - P.z;
            const float vl = sqrtf(dot3(vx, vy, vz, vx, vy, vz));
            vx = vx / vl; vy = vy / vl; vz = vz / vl;
            const float ndv = dot3(nx, ny, nz, vx, vy, vz);
            const float k2 = 2.0f * ndv;
            const float rx = k2 * nx - vx, ry = k2 * ny - vy, rz = k2 * nz - vz;
            const float tau = fminf(fmaxf(k.alb[pix].w, VCT_SPEC_TAU_MIN), VCT_SPEC_TAU_MAX);
            float4 res;
            steps += march(k, ox, oy, oz, rx, ry, rz, tau, res, texels);
            sout = res;
        }
    }
    if (in_frame || k.compact) {
        k.diff[oidx] = dout;
        k.spec[oidx] = sout;
        if (k.steps_px && in_frame) k.steps_px[pix] = steps;
    }
    if (k.steps_total) {
        uint32_t ws = wave_sum_u32(steps);
        if (lane == 0 && ws) atomicAdd(k.steps_total, (unsigned long long)ws);
    }
    if (k.texels_total) {
        uint32_t wt = wave_sum_u32(texels);
        if (lane == 0 && wt) atomicAdd(k.texels_total, (unsigned long long)wt);
    }
}

// ===========================================================================
// Default variant (0): wave-cooperative 4^3 brick staging in LDS
// ===========================================================================
// The 64 lanes of a wave (an 8x8 pixel block) march the same cone index in
// lock step.  At each step and mip level, if every active lane's 2x2x2
// trilinear footprint lies inside the 4^3 texel brick centred on the first
// active lane (a ballot), the wave loads that brick ONCE -- one texel per
// lane, one 16-B global load per face -- into a wave-private LDS slot and every
// lane reads its 8 corners with ds_read_b128 at immediate offsets
// (+16 B dx, +64 B dy, +256 B dz).  That replaces 8 gathers per lane and face
// (64 address computations, 8 TA-issued 1-KiB wave loads) by one coalesced
// load.  Texels outside the level are staged as zero, which is exactly the
// spec's zero border.  When the footprint does not fit (silhouettes, diverging
// specular lobes) or the lanes disagree on the mip level or face triple, the
// wave falls back to the per-lane gathers of variant 0 for that step.  Both
// paths read the same texels and run the same fmaf chain, so the result is
// bit-identical to variant 0 and to the oracle.
constexpr int kBrickSlots = 6;              // level A: 1 or 3 faces, level B: 3 faces

// component-wise select: `c ? a : b` on two float4 structs lowers to scratch on gfx950
__device__ __forceinline__ float4 sel4(bool c, float4 a, float4 b) {
    return make_float4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
}

// Orders one wave's LDS writes before its (other lanes') LDS reads and vice versa:
// the asm "memory" clobber stops the compiler moving DS ops across it (release /
// acquire fences at wavefront scope do not order a store before a later load of
// a different address), the lgkmcnt(0) makes the hand-off explicit in hardware.
__device__ __forceinline__ void wave_lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ float4 brick_tri(const float4* __restrict__ b, float fx, float fy, float fz) {
    const float wx[2] = {1.0f - fx, fx}, wy[2] = {1.0f - fy, fy}, wz[2] = {1.0f - fz, fz};
    float4 v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = b[(c & 1) + 4 * ((c >> 1) & 1) + 16 * (c >> 2)];
    float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const float w = (wx[c & 1] * wy[(c >> 1) & 1]) * wz[c >> 2];
        acc.x = fmaf(w, v[c].x, acc.x);
        acc.y = fmaf(w, v[c].y, acc.y);
        acc.z = fmaf(w, v[c].z, acc.z);
        acc.w = fmaf(w, v[c].w, acc.w);
    }
    return acc;
}

// Adaptive brick: the wave's footprint at level l is the box spanned by the
// active lanes' positions (per-axis min / max of q, reduced once per step; the
// texel map x -> floor(x * 2^-l - 0.5) is monotonic, so reducing q and mapping
// gives exactly the min / max corner).  The brick is that box rounded up to
// power-of-two dims (2..16 per axis) and staged when it holds <= 256 texels
// (4 texels per lane, 4 KiB per face).  Corners are read at
// base + {0, 1, dx} + {0, dx*dy} (strides are wave-uniform).
constexpr int kSlotTexels = 256;

__device__ __forceinline__ int log2_dim(int e) {
    return e <= 2 ? 1 : (e <= 4 ? 2 : (e <= 8 ? 3 : (e <= 16 ? 4 : 16)));   // 16: never fits
}

__device__ __forceinline__ float4 brick_tri_s(const float4* __restrict__ b, uint32_t sy, uint32_t sz, float fx,
                                              float fy, float fz) {
    const float wx[2] = {1.0f - fx, fx}, wy[2] = {1.0f - fy, fy}, wz[2] = {1.0f - fz, fz};
    float4 v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = b[(c & 1) + sy * ((c >> 1) & 1) + sz * (c >> 2)];
    float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const float w = (wx[c & 1] * wy[(c >> 1) & 1]) * wz[c >> 2];
        acc.x = fmaf(w, v[c].x, acc.x);
        acc.y = fmaf(w, v[c].y, acc.y);
        acc.z = fmaf(w, v[c].z, acc.z);
        acc.w = fmaf(w, v[c].w, acc.w);
    }
    return acc;
}

// D_l for one level.  `mn` / `mx`: wave-uniform min / max of the active lanes'
// q.  `lds` = this wave's 3 x kSlotTexels slots.  Wave-uniform control flow only.
__device__ __forceinline__ float4 level_brick(const TraceK& k, int l, float qx, float qy, float qz, bool active,
                                              const float (&mn)[3], const float (&mx)[3], bool faces_uniform,
                                              int ufaces, int fx, int fy, int fz, float wdx, float wdy, float wdz,
                                              float4* __restrict__ lds) {
    const float scale = __uint_as_float((uint32_t)(127 - l) << 23);
    const int nl = k.n >> l;
    const bool iso = (l == 0 || !k.aniso);
    int o[3], lb[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        o[a] = __builtin_amdgcn_readfirstlane((int)floorf(mn[a] * scale - 0.5f));
        const int hi = __builtin_amdgcn_readfirstlane((int)floorf(mx[a] * scale - 0.5f));
        lb[a] = log2_dim(hi - o[a] + 2);
    }
    const int lxy = lb[0] + lb[1], ltot = lxy + lb[2];
    const bool fits = ltot <= k.brick_log2 && (iso || faces_uniform);
    VCT_DBG(fits ? 2 : 3);
    if (!fits) VCT_DBG(4 + (l < 10 ? l : 10));
    float4 s = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (fits) {
        const float4* lvl = k.pyr + k.lvl_off[l];
        const size_t vl = (size_t)nl * nl * nl;
        const int lane = threadIdx.x & 63;
        const int total = 1 << ltot, mxd = (1 << lb[0]) - 1, myd = (1 << lb[1]) - 1;
        const int nf = iso ? 1 : 3;
        const float4 z4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll 1
        for (int f = 0; f < nf; ++f) {
            // wave-uniform faces: lanes that trace nothing still stage texels
            const int face = iso ? 0 : (f == 0 ? (ufaces & 7) : (f == 1 ? ((ufaces >> 3) & 7) : (ufaces >> 6)));
            const float4* vol = lvl + (size_t)face * vl;
#pragma unroll
            for (int it = 0; it < kSlotTexels / 64; ++it) {
                const int j = lane + 64 * it;
                if (it == 0 || j < total) {
                    const int sx = o[0] + (j & mxd), sy = o[1] + ((j >> lb[0]) & myd), sz = o[2] + (j >> lxy);
                    const bool inb = (unsigned)sx < (unsigned)nl && (unsigned)sy < (unsigned)nl &&
                                     (unsigned)sz < (unsigned)nl && j < total;
                    const uint32_t gi = inb ? (uint32_t)sx + (uint32_t)nl * ((uint32_t)sy + (uint32_t)nl * (uint32_t)sz) : 0u;
                    const float4 v = vol[gi];
                    if (j < total) lds[f * kSlotTexels + j] = sel4(inb, v, z4);
                }
            }
        }
        wave_lds_sync();
        if (active) {
            const float cx = qx * scale - 0.5f, cy = qy * scale - 0.5f, cz = qz * scale - 0.5f;
            const float flx = floorf(cx), fly = floorf(cy), flz = floorf(cz);
            const uint32_t base = (uint32_t)((int)flx - o[0]) + ((uint32_t)((int)fly - o[1]) << lb[0]) +
                                  ((uint32_t)((int)flz - o[2]) << lxy);
            const uint32_t sy = 1u << lb[0], sz = 1u << lxy;
            const float frx = cx - flx, fry = cy - fly, frz = cz - flz;
            if (iso) {
                s = brick_tri_s(lds + base, sy, sz, frx, fry, frz);
            } else {
#pragma unroll 1
                for (int f = 0; f < 3; ++f) {
                    const float w = f == 0 ? wdx : (f == 1 ? wdy : wdz);
                    const float4 tf = brick_tri_s(lds + f * kSlotTexels + base, sy, sz, frx, fry, frz);
                    s.x = fmaf(w, tf.x, s.x);
                    s.y = fmaf(w, tf.y, s.y);
                    s.z = fmaf(w, tf.z, s.z);
                    s.w = fmaf(w, tf.w, s.w);
                }
            }
        }
        wave_lds_sync();
    } else if (active) {
        s = sample_level(k, l, qx, qy, qz, fx, fy, fz, wdx, wdy, wdz);
    }
    return s;
}

// Fixed 4^3 brick (variant 3): D_l for one level; `lds` = this wave's slots (nf x 64 texels).
// Must be called in wave-uniform control flow (all 64 lanes).
__device__ __forceinline__ float4 level_brick4(const TraceK& k, int l, float qx, float qy, float qz, bool active,
                                              int first, bool faces_uniform, int ufaces, int fx, int fy, int fz,
                                              float wdx, float wdy, float wdz, float4* __restrict__ lds) {
    const float scale = __uint_as_float((uint32_t)(127 - l) << 23);
    const int nl = k.n >> l;
    const float cx = qx * scale - 0.5f, cy = qy * scale - 0.5f, cz = qz * scale - 0.5f;
    const float flx = floorf(cx), fly = floorf(cy), flz = floorf(cz);
    const int ix = (int)flx, iy = (int)fly, iz = (int)flz;
    const bool iso = (l == 0 || !k.aniso);
    // brick origin = per-axis minimum corner over the active lanes (wave reduction)
    const int ox = __ockl_wfred_min_i32(active ? ix : INT_MAX);
    const int oy = __ockl_wfred_min_i32(active ? iy : INT_MAX);
    const int oz = __ockl_wfred_min_i32(active ? iz : INT_MAX);
    (void)first;
    const uint32_t lx = (uint32_t)(ix - ox), ly = (uint32_t)(iy - oy), lz = (uint32_t)(iz - oz);
    const bool fits = __all(!active || (lx <= 2u && ly <= 2u && lz <= 2u)) && (iso || faces_uniform);
    float4 s = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    const float4* lvl = k.pyr + k.lvl_off[l];
    const size_t vl = (size_t)nl * nl * nl;
    if (fits) {
        const int lane = threadIdx.x & 63;
        const int sx = ox + (lane & 3), sy = oy + ((lane >> 2) & 3), sz = oz + (lane >> 4);
        const bool inb = (unsigned)sx < (unsigned)nl && (unsigned)sy < (unsigned)nl && (unsigned)sz < (unsigned)nl;
        const uint32_t gi = inb ? (uint32_t)sx + (uint32_t)nl * ((uint32_t)sy + (uint32_t)nl * (uint32_t)sz) : 0u;
        const float4 z4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        auto zsel = [inb, z4](float4 v) { return sel4(inb, v, z4); };
        if (iso) {
            lds[lane] = zsel(lvl[gi]);
        } else {
            // wave-uniform face triple (lanes that trace nothing -- background pixels --
            // still stage texels, so the faces must not come from the lane's own direction)
            const int ux = ufaces & 7, uy = (ufaces >> 3) & 7, uz = ufaces >> 6;
            const float4 a = lvl[(size_t)ux * vl + gi], b = lvl[(size_t)uy * vl + gi], c = lvl[(size_t)uz * vl + gi];
            lds[lane] = zsel(a);
            lds[64 + lane] = zsel(b);
            lds[128 + lane] = zsel(c);
        }
        wave_lds_sync();
        if (active) {
            const uint32_t base = lx + 4u * ly + 16u * lz;
            const float frx = cx - flx, fry = cy - fly, frz = cz - flz;
            if (iso) {
                s = brick_tri(lds + base, frx, fry, frz);
            } else {
#pragma unroll 1
                for (int f = 0; f < 3; ++f) {
                    const float w = f == 0 ? wdx : (f == 1 ? wdy : wdz);
                    const float4 tf = brick_tri(lds + 64 * f + base, frx, fry, frz);
                    s.x = fmaf(w, tf.x, s.x);
                    s.y = fmaf(w, tf.y, s.y);
                    s.z = fmaf(w, tf.z, s.z);
                    s.w = fmaf(w, tf.w, s.w);
                }
            }
        }
        wave_lds_sync();
    } else if (active) {
        s = sample_level(k, l, qx, qy, qz, fx, fy, fz, wdx, wdy, wdz);
    }
    return s;
}

// one cone, wave-synchronous (A.6); same arithmetic as march()
template <bool FIXED>
__device__ __forceinline__ uint32_t march_brick(const TraceK& k, bool valid, float ox, float oy, float oz,
                                                float dx, float dy, float dz, float tau, float4& res,
                                                uint32_t& texels, float4* __restrict__ lds) {
    const float tau2 = 2.0f * tau;
    const float nf = (float)k.n, Lf = (float)k.L;
    const int fx = dx >= 0.0f ? VCT_FACE_PX : VCT_FACE_NX;
    const int fy = dy >= 0.0f ? VCT_FACE_PY : VCT_FACE_NY;
    const int fz = dz >= 0.0f ? VCT_FACE_PZ : VCT_FACE_NZ;
    const float wdx = dx * dx, wdy = dy * dy, wdz = dz * dz;
    float cr = 0.0f, cg = 0.0f, cb = 0.0f, a = 0.0f, t = 1.0f;
    uint32_t steps = 0;
    bool active = valid;
    // face triple uniform over the lanes that trace this cone
    const int fcode = fx | (fy << 3) | (fz << 6);
    unsigned long long vm = __ballot(valid);
    const int f0 = vm ? __builtin_amdgcn_readlane(fcode, __builtin_ctzll(vm)) : fcode;
    const bool faces_uniform = __all(!valid || fcode == f0);
    for (;;) {
        const float qx = ox + dx * t, qy = oy + dy * t, qz = oz + dz * t;
        if (active) {
            if (!(a < VCT_ALPHA_STOP)) active = false;
            else if (!(t <= k.tmax)) active = false;
            else if (!(qx >= 0.0f && qx <= nf && qy >= 0.0f && qy <= nf && qz >= 0.0f && qz <= nf)) active = false;
        }
        const unsigned long long am = __ballot(active);
        if (am == 0ull) break;
        const int first = __builtin_ctzll(am);
        const float D = fmaxf(1.0f, tau2 * t);
        float m = spec_log2(D);
        if (m > Lf) m = Lf;
        const int l0 = (int)m;
        const float fr = m - (float)l0;
        const int l0f = __builtin_amdgcn_readlane(l0, first);
        const bool lvl_uniform = __all(!active || l0 == l0f);
        const bool two = fr > 0.0f && l0 < k.L;
        float4 s;
        if (FIXED && lvl_uniform) {
            s = level_brick4(k, l0f, qx, qy, qz, active, first, faces_uniform, f0, fx, fy, fz, wdx, wdy, wdz, lds);
            if (__any(active && two)) {
                const int l1 = l0f + 1 <= k.L ? l0f + 1 : k.L;
                float4 s1 = level_brick4(k, l1, qx, qy, qz, active && two, first, faces_uniform, f0, fx, fy, fz,
                                         wdx, wdy, wdz, lds + 3 * 64);
                if (active && two) {
                    const float omf = 1.0f - fr;
                    s.x = fmaf(fr, s1.x, omf * s.x);
                    s.y = fmaf(fr, s1.y, omf * s.y);
                    s.z = fmaf(fr, s1.z, omf * s.z);
                    s.w = fmaf(fr, s1.w, omf * s.w);
                }
            }
        } else if (lvl_uniform) {
            // footprint box of the active lanes, shared by both levels of this step
            const float inf = __builtin_inff();
            const float mn[3] = {__ockl_wfred_min_f32(active ? qx : inf), __ockl_wfred_min_f32(active ? qy : inf),
                                 __ockl_wfred_min_f32(active ? qz : inf)};
            const float mx[3] = {__ockl_wfred_max_f32(active ? qx : -inf), __ockl_wfred_max_f32(active ? qy : -inf),
                                 __ockl_wfred_max_f32(active ? qz : -inf)};
            s = level_brick(k, l0f, qx, qy, qz, active, mn, mx, faces_uniform, f0, fx, fy, fz, wdx, wdy, wdz, lds);
            if (__any(active && two)) {
                const int l1 = l0f + 1 <= k.L ? l0f + 1 : k.L;
                float4 s1 = level_brick(k, l1, qx, qy, qz, active && two, mn, mx, faces_uniform, f0, fx, fy, fz,
                                        wdx, wdy, wdz, lds);
                if (active && two) {
                    const float omf = 1.0f - fr;
                    s.x = fmaf(fr, s1.x, omf * s.x);
                    s.y = fmaf(fr, s1.y, omf * s.y);
                    s.z = fmaf(fr, s1.z, omf * s.z);
                    s.w = fmaf(fr, s1.w, omf * s.w);
                }
            }
        } else if (active) {
            s = sample_level(k, l0, qx, qy, qz, fx, fy, fz, wdx, wdy, wdz);
            if (two) {
                float4 s1 = sample_level(k, l0 + 1, qx, qy, qz, fx, fy, fz, wdx, wdy, wdz);
                const float omf = 1.0f - fr;
                s.x = fmaf(fr, s1.x, omf * s.x);
                s.y = fmaf(fr, s1.y, omf * s.y);
                s.z = fmaf(fr, s1.z, omf * s.z);
                s.w = fmaf(fr, s1.w, omf * s.w);
            }
        }
        if (active) {
            texels += (l0 == 0 || !k.aniso) ? 8u : 24u;
            if (two) texels += k.aniso ? 24u : 8u;
            const float oma = 1.0f - a;
            cr = fmaf(oma, s.x, cr);
            cg = fmaf(oma, s.y, cg);
            cb = fmaf(oma, s.z, cb);
            a = fmaf(oma, s.w, a);
            t = t + VCT_STEP_SCALE * D;
            ++steps;
        }
    }
    res = make_float4(cr, cg, cb, a);
    return steps;
}

// ===========================================================================
// Variant 2: brick staging with LDS-DMA prefetch of the NEXT step's bricks
// ===========================================================================
// Variant 0 pays two dependent memory round trips per step (global load ->
// ds_write -> ds_read) and the waves sit in s_waitcnt ~45 % of their cycles.
// Here the bricks of step k+1 are fetched while step k computes: the next t
// (t + D/2) is known before step k samples, so the first active lane's next
// position and mip pair give the next brick origins, and the wave issues
// global_load_lds_dwordx4 (one texel per lane straight into LDS, no VGPRs) into
// the other half of a double-buffered LDS ring.  A step consumes its buffer
// behind a counted s_waitcnt vmcnt(n_next) that leaves the prefetch in flight.
// The DMA is inline asm so the compiler neither waits vmcnt(0) before every
// ds_read (what it does for the builtin) nor reorders around it ("memory").
// The plan is speculative: if the active lanes' levels or footprints do not
// match it, the step falls back to per-lane gathers; results stay bit-exact.
struct Plan {
    int lA, lB;              // levels staged in slots 0..2 / 3..5 (lB = -1: none)
    int ax, ay, az;          // brick origins
    int bx, by, bz;
    int n;                   // LDS-DMA instructions issued for this plan
};

__device__ __forceinline__ void glds16(uint32_t lds_addr, const float4* g) {
    asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(lds_addr), "v"(g) : "memory", "m0");
}

__device__ __forceinline__ void wait_vm(int n) {   // s_waitcnt vmcnt(n), n wave-uniform in 0..6
    switch (n) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    }
}

__device__ __forceinline__ uint32_t lds_u32(const float4* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float4*)p;
}

// stage level l's brick (origin = min corner over the `act` lanes' positions q)
// into `slot0`; returns the number of LDS-DMA instructions issued
__device__ __forceinline__ int stage_dma(const TraceK& k, int l, float qx, float qy, float qz, bool act,
                                         int ufaces, const float4* slot0, int& ox, int& oy, int& oz) {
    const float scale = __uint_as_float((uint32_t)(127 - l) << 23);
    const int nl = k.n >> l;
    // origin = per-axis minimum corner over the lanes expected to sample (act)
    ox = __builtin_amdgcn_readfirstlane(__ockl_wfred_min_i32(act ? (int)floorf(qx * scale - 0.5f) : INT_MAX));
    oy = __builtin_amdgcn_readfirstlane(__ockl_wfred_min_i32(act ? (int)floorf(qy * scale - 0.5f) : INT_MAX));
    oz = __builtin_amdgcn_readfirstlane(__ockl_wfred_min_i32(act ? (int)floorf(qz * scale - 0.5f) : INT_MAX));
    const int lane = threadIdx.x & 63;
    const int sx = ox + (lane & 3), sy = oy + ((lane >> 2) & 3), sz = oz + (lane >> 4);
    const bool inb = (unsigned)sx < (unsigned)nl && (unsigned)sy < (unsigned)nl && (unsigned)sz < (unsigned)nl;
    const uint32_t gi = (uint32_t)sx + (uint32_t)nl * ((uint32_t)sy + (uint32_t)nl * (uint32_t)sz);
    const float4* lvl = k.pyr + k.lvl_off[l];
    const uint32_t base = __builtin_amdgcn_readfirstlane(lds_u32(slot0));
    if (l == 0 || !k.aniso) {
        glds16(base, inb ? lvl + gi : k.zero);
        return 1;
    }
    const size_t vl = (size_t)nl * nl * nl;
    const int ux = ufaces & 7, uy = (ufaces >> 3) & 7, uz = ufaces >> 6;
    glds16(base, inb ? lvl + (size_t)ux * vl + gi : k.zero);
    glds16(base + 1024, inb ? lvl + (size_t)uy * vl + gi : k.zero);
    glds16(base + 2048, inb ? lvl + (size_t)uz * vl + gi : k.zero);
    return 3;
}

// plan + issue the bricks of a step: lanes `act` at positions q, (uniform) cone size D
__device__ __forceinline__ Plan plan_issue(const TraceK& k, float qx, float qy, float qz, bool act, float D,
                                           int ufaces, const float4* buf) {
    Plan p;
    float m = spec_log2(D);
    if (m > (float)k.L) m = (float)k.L;
    const int l0 = (int)m;
    const float fr = m - (float)l0;
    p.lA = __builtin_amdgcn_readfirstlane(l0);
    const bool two = __builtin_amdgcn_readfirstlane((fr > 0.0f && l0 < k.L) ? 1 : 0) != 0;
    p.n = stage_dma(k, p.lA, qx, qy, qz, act, ufaces, buf, p.ax, p.ay, p.az);
    p.lB = -1;
    p.bx = p.by = p.bz = 0;
    if (two) {
        p.lB = p.lA + 1;
        p.n += stage_dma(k, p.lB, qx, qy, qz, act, ufaces, buf + 3 * 64, p.bx, p.by, p.bz);
    }
    return p;
}

// D_l from a staged brick (origin o*) if every lane in `need` fits; `ok` reports it
__device__ __forceinline__ float4 level_from_plan(const TraceK& k, int l, float qx, float qy, float qz, bool need,
                                                  int ox, int oy, int oz, float wdx, float wdy, float wdz,
                                                  const float4* __restrict__ slot0) {
    const float scale = __uint_as_float((uint32_t)(127 - l) << 23);
    const float cx = qx * scale - 0.5f, cy = qy * scale - 0.5f, cz = qz * scale - 0.5f;
    const float flx = floorf(cx), fly = floorf(cy), flz = floorf(cz);
    const uint32_t lx = (uint32_t)((int)flx - ox), ly = (uint32_t)((int)fly - oy), lz = (uint32_t)((int)flz - oz);
    float4 s = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (need) {
        const uint32_t base = lx + 4u * ly + 16u * lz;
        const float frx = cx - flx, fry = cy - fly, frz = cz - flz;
        if (l == 0 || !k.aniso) return brick_tri(slot0 + base, frx, fry, frz);
#pragma unroll 1
        for (int f = 0; f < 3; ++f) {
            const float w = f == 0 ? wdx : (f == 1 ? wdy : wdz);
            const float4 tf = brick_tri(slot0 + 64 * f + base, frx, fry, frz);
            s.x = fmaf(w, tf.x, s.x);
            s.y = fmaf(w, tf.y, s.y);
            s.z = fmaf(w, tf.z, s.z);
            s.w = fmaf(w, tf.w, s.w);
        }
    }
    return s;
}

__device__ __forceinline__ bool fits_plan(int l, float qx, float qy, float qz, bool need, int ox, int oy, int oz) {
    const float scale = __uint_as_float((uint32_t)(127 - l) << 23);
    const uint32_t lx = (uint32_t)((int)floorf(qx * scale - 0.5f) - ox);
    const uint32_t ly = (uint32_t)((int)floorf(qy * scale - 0.5f) - oy);
    const uint32_t lz = (uint32_t)((int)floorf(qz * scale - 0.5f) - oz);
    return __all(!need || (lx <= 2u && ly <= 2u && lz <= 2u));
}

__device__ __forceinline__ uint32_t march_pf(const TraceK& k, bool valid, float ox, float oy, float oz, float dx,
                                             float dy, float dz, float tau, float4& res, uint32_t& texels,
                                             float4* __restrict__ ring) {
    const float tau2 = 2.0f * tau;
    const float nf = (float)k.n, Lf = (float)k.L;
    const int fx = dx >= 0.0f ? VCT_FACE_PX : VCT_FACE_NX;
    const int fy = dy >= 0.0f ? VCT_FACE_PY : VCT_FACE_NY;
    const int fz = dz >= 0.0f ? VCT_FACE_PZ : VCT_FACE_NZ;
    const float wdx = dx * dx, wdy = dy * dy, wdz = dz * dz;
    float cr = 0.0f, cg = 0.0f, cb = 0.0f, a = 0.0f, t = 1.0f;
    uint32_t steps = 0;
    bool active = valid;
    const unsigned long long vm = __ballot(valid);
    if (vm == 0ull) { res = make_float4(0.0f, 0.0f, 0.0f, 0.0f); return 0; }
    const int fcode = fx | (fy << 3) | (fz << 6);
    const int f0 = __builtin_amdgcn_readlane(fcode, __builtin_ctzll(vm));
    const bool faces_uniform = __all(!valid || fcode == f0);
    int buf = 0;
    Plan cur;
    {   // plan of step 0 from the first valid lane
        const int fl = __builtin_ctzll(vm);
        const float D0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(fmaxf(1.0f, tau2 * t)), fl));
        cur = plan_issue(k, ox + dx * t, oy + dy * t, oz + dz * t, valid, D0, f0, ring);
    }
    for (;;) {
        const float qx = ox + dx * t, qy = oy + dy * t, qz = oz + dz * t;
        if (active) {
            if (!(a < VCT_ALPHA_STOP)) active = false;
            else if (!(t <= k.tmax)) active = false;
            else if (!(qx >= 0.0f && qx <= nf && qy >= 0.0f && qy <= nf && qz >= 0.0f && qz <= nf)) active = false;
        }
        const unsigned long long am = __ballot(active);
        if (am == 0ull) break;
        const int first = __builtin_ctzll(am);
        const float D = fmaxf(1.0f, tau2 * t);
        float m = spec_log2(D);
        if (m > Lf) m = Lf;
        const int l0 = (int)m;
        const float fr = m - (float)l0;
        const bool two = fr > 0.0f && l0 < k.L;
        // does the prefetched plan serve every active lane?
        bool ok = faces_uniform && __all(!active || l0 == cur.lA) && (cur.lB >= 0 || !__any(active && two));
        if (ok) ok = fits_plan(cur.lA, qx, qy, qz, active, cur.ax, cur.ay, cur.az);
        if (ok && cur.lB >= 0) ok = fits_plan(cur.lB, qx, qy, qz, active && two, cur.bx, cur.by, cur.bz);
        // prefetch the next step's bricks (speculative, first active lane)
        const float tn = t + VCT_STEP_SCALE * D;
        const float Dn = fmaxf(1.0f, tau2 * tn);
        const float nD = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(Dn), first));
        const float4* cbuf = ring + buf * (kBrickSlots * 64);
        const Plan nxt = plan_issue(k, ox + dx * tn, oy + dy * tn, oz + dz * tn, active, nD, f0,
                                    ring + (buf ^ 1) * (kBrickSlots * 64));
        wait_vm(nxt.n);                 // this step's bricks have landed; the next step's stay in flight
        float4 s = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        VCT_DBG(ok ? 0 : 1);
        if (ok) {
            s = level_from_plan(k, cur.lA, qx, qy, qz, active, cur.ax, cur.ay, cur.az, wdx, wdy, wdz, cbuf);
            if (cur.lB >= 0) {
                const float4 s1 = level_from_plan(k, cur.lB, qx, qy, qz, active && two, cur.bx, cur.by, cur.bz,
                                                  wdx, wdy, wdz, cbuf + 3 * 64);
                if (active && two) {
                    const float omf = 1.0f - fr;
                    s.x = fmaf(fr, s1.x, omf * s.x);
                    s.y = fmaf(fr, s1.y, omf * s.y);
                    s.z = fmaf(fr, s1.z, omf * s.z);
                    s.w = fmaf(fr, s1.w, omf * s.w);
                }
            }
        } else if (active) {
            s = sample_level(k, l0, qx, qy, qz, fx, fy, fz, wdx, wdy, wdz);
            if (two) {
                const float4 s1 = sample_level(k, l0 + 1, qx, qy, qz, fx, fy, fz, wdx, wdy, wdz);
                const float omf = 1.0f - fr;
                s.x = fmaf(fr, s1.x, omf * s.x);
                s.y = fmaf(fr, s1.y, omf * s.y);
                s.z = fmaf(fr, s1.z, omf * s.z);
                s.w = fmaf(fr, s1.w, omf * s.w);
            }
        }
        // every lane's reads of this buffer are done before the next iteration
        // re-targets it (the DMA of step k+2 goes into this buffer)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (active) {
            texels += (l0 == 0 || !k.aniso) ? 8u : 24u;
            if (two) texels += k.aniso ? 24u : 8u;
            const float oma = 1.0f - a;
            cr = fmaf(oma, s.x, cr);
            cg = fmaf(oma, s.y, cg);
            cb = fmaf(oma, s.z, cb);
            a = fmaf(oma, s.w, a);
            t = tn;
            ++steps;
        }
        cur = nxt;
        buf ^= 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // drain the speculative prefetch
    res = make_float4(cr, cg, cb, a);
    return steps;
}

// K4 kernel for the LDS variants: V = 0 brick staging, V = 2 brick staging + DMA prefetch
template <int V>
__global__ void __launch_bounds__(256) k4_trace_lds(TraceK k) {
    __shared__ float4 lds_all[4][V == 2 ? 2 * kBrickSlots * 64 : (V == 3 ? kBrickSlots * 64 : 3 * kSlotTexels)];
    const uint32_t nb = gridDim.x, b = blockIdx.x;
    const uint32_t xcd = b & 7, q = nb >> 3, r = nb & 7;
    const uint32_t rb = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
    const uint32_t lt = rb >> 4, sub = rb & 15;
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float4* lds = lds_all[wave];
    const uint32_t px = (sub & 3) * 16 + (wave & 1) * 8 + (lane & 7);
    const uint32_t py = (sub >> 2) * 16 + (wave >> 1) * 8 + (lane >> 3);
    const uint32_t tile = lt * (uint32_t)k.world + (uint32_t)k.rank;
    const uint32_t x = (tile % (uint32_t)k.tiles_x) * VCT_TILE + px;
    const uint32_t y = (tile / (uint32_t)k.tiles_x) * VCT_TILE + py;
    const bool in_frame = x < (uint32_t)k.w && y < (uint32_t)k.h;
    const size_t pix = in_frame ? (size_t)y * (size_t)k.w + x : 0;
    const size_t oidx = k.compact ? (size_t)lt * (VCT_TILE * VCT_TILE) + py * VCT_TILE + px : pix;

    float4 dout = make_float4(0.0f, 0.0f, 0.0f, 0.0f), sout = dout;
    uint32_t steps = 0, texels = 0;
    float4 P = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (in_frame) P = k.pos[pix];
    const bool valid = P.w != 0.0f;
    if (__any(valid)) {
        float4 N4 = make_float4(0.0f, 1.0f, 0.0f, 0.0f);
        if (valid) N4 = k.nrm[pix];
        const float nx = N4.x, ny = N4.y, nz = N4.z;
        const float ox = (P.x - k.g0x) * k.inv_h + nx;
        const float oy = (P.y - k.g0y) * k.inv_h + ny;
        const float oz = (P.z - k.g0z) * k.inv_h + nz;
        const float sgn = copysignf(1.0f, nz);
        const float ka = -1.0f / (sgn + nz);
        const float kb = (nx * ny) * ka;
        const float Tx = 1.0f + ((sgn * nx) * nx) * ka, Ty = sgn * kb, Tz = -(sgn * nx);
        const float Bx = kb, By = sgn + (ny * ny) * ka, Bz = -ny;
        const float(*cones)[4] = cone_table(k.nd);
        float ir = 0.0f, ig = 0.0f, ib = 0.0f, occ = 0.0f;
        for (int c = 0; c < k.nd; ++c) {
            const float cn = cones[c][0], ct = cones[c][1], cb = cones[c][2], wk = cones[c][3];
            const float dx = (cn * nx + ct * Tx) + cb * Bx;
            const float dy = (cn * ny + ct * Ty) + cb * By;
            const float dz = (cn * nz + ct * Tz) + cb * Bz;
            float4 res;
            if constexpr (V == 2) steps += march_pf(k, valid, ox, oy, oz, dx, dy, dz, k.tau_d, res, texels, lds);
            else steps += march_brick<V == 3>(k, valid, ox, oy, oz, dx, dy, dz, k.tau_d, res, texels, lds);
            ir = fmaf(wk, res.x, ir);
            ig = fmaf(wk, res.y, ig);
            ib = fmaf(wk, res.z, ib);
            occ = fmaf(wk, res.w, occ);
        }
        dout = sel4(valid, make_float4(ir, ig, ib, 1.0f - occ), dout);
        if (k.spec_on) {
            float vx = k.ex - P.x, vy = k.ey - P.y, vz = k.ez - P.z;
            float vl = sqrtf(dot3(vx, vy, vz, vx, vy, vz));
            vl = valid ? vl : 1.0f;
            vx = vx / vl; vy = vy / vl; vz = vz / vl;
            const float ndv = dot3(nx, ny, nz, vx, vy, vz);
            const float k2 = 2.0f * ndv;
            const float rx = k2 * nx - vx, ry = k2 * ny - vy, rz = k2 * nz - vz;
            const float rough = valid ? k.alb[pix].w : 0.1f;
            const float tau = fminf(fmaxf(rough, VCT_SPEC_TAU_MIN), VCT_SPEC_TAU_MAX);
            float4 res;
            if constexpr (V == 2) steps += march_pf(k, valid, ox, oy, oz, rx, ry, rz, tau, res, texels, lds);
            else steps += march_brick<V == 3>(k, valid, ox, oy, oz, rx, ry, rz, tau, res, texels, lds);
            sout = sel4(valid, res, sout);
        }
    }
    if (in_frame || k.compact) {
        k.diff[oidx] = dout;
        k.spec[oidx] = sout;
        if (k.steps_px && in_frame) k.steps_px[pix] = steps;
    }
    if (k.steps_total) {
        uint32_t ws = wave_sum_u32(steps);
        if (lane == 0 && ws) atomicAdd(k.steps_total, (unsigned long long)ws);
    }
    if (k.texels_total) {
        uint32_t wt = wave_sum_u32(texels);
        if (lane == 0 && wt) atomicAdd(k.texels_total, (unsigned long long)wt);
    }
    if constexpr (V == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

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

}  // namespace

uint32_t tiles_for_rank(uint32_t w, uint32_t h, uint32_t rank, uint32_t world) {
    if (world == 0) world = 1;
    const uint32_t tx = (w + VCT_TILE - 1) / VCT_TILE, ty = (h + VCT_TILE - 1) / VCT_TILE;
    const uint32_t total = tx * ty;
    if (rank >= world || total <= rank) return 0;
    return (total - rank + world - 1) / world;
}

hipError_t launch_trace(vct_ctx* c, const vct_trace_args* a) {
    const Grid& g = c->grid;
    TraceK k;
    k.pyr = g.pyr;
    k.zero = g.pyr + g.pyr_texels;
    for (int i = 0; i <= kMaxLevels; ++i) k.lvl_off[i] = g.lvl_off[i];
    k.n = (int)g.n; k.L = (int)g.L;
    k.g0x = g.g0[0]; k.g0y = g.g0[1]; k.g0z = g.g0[2];
    k.inv_h = g.inv_h;
    k.tmax = (float)g.n * VCT_SQRT3;
    k.pos = (const float4*)a->pos4; k.nrm = (const float4*)a->nrm4; k.alb = (const float4*)a->alb4;
    k.diff = (float4*)a->diffuse4; k.spec = (float4*)a->spec4;
    k.steps_px = a->steps_px; k.steps_total = a->cone_steps; k.texels_total = a->texel_fetches;
    k.w = (int)a->width; k.h = (int)a->height;
    k.ex = a->eye[0]; k.ey = a->eye[1]; k.ez = a->eye[2];
    const uint32_t world = a->tile_world ? a->tile_world : 1;
    k.tiles_x = (int)((a->width + VCT_TILE - 1) / VCT_TILE);
    k.rank = (int)(a->tile_world ? a->tile_rank : 0);
    k.world = (int)world;
    const uint32_t nlt = tiles_for_rank(a->width, a->height, (uint32_t)k.rank, world);
    k.n_local_tiles = (int)nlt;
    k.compact = a->tile_compact ? 1 : 0;
    k.nd = (int)c->cfg.n_diffuse;
    k.spec_on = c->cfg.specular ? 1 : 0;
    k.aniso = g.aniso;
    // variant bits 8..11: brick size cap (log2 texels); 0 = default
    const uint32_t cap = (a->variant >> 8) & 0xf;
    k.brick_log2 = cap ? (int)(cap > 8 ? 8 : cap) : 6;
    k.tau_d = c->cfg.n_diffuse == 16 ? VCT_TAN20 : VCT_TAN30;
    if (nlt == 0) return hipSuccess;
    const uint32_t blocks = nlt * 16;
    const uint32_t kv = a->variant & 0xff;
    if (kv == 1)
        hipLaunchKernelGGL(k4_trace, dim3(blocks), dim3(256), 0, c->stream, k);
    else if (kv == 2)
        hipLaunchKernelGGL(k4_trace_lds<2>, dim3(blocks), dim3(256), 0, c->stream, k);
    else if (kv == 3)
        hipLaunchKernelGGL(k4_trace_lds<3>, dim3(blocks), dim3(256), 0, c->stream, k);
    else
        hipLaunchKernelGGL(k4_trace_lds<0>, dim3(blocks), dim3(256), 0, c->stream, k);
    return hipGetLastError();
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

}  // namespace vct

#ifdef VCT_DEBUG_COUNTERS
extern "C" int vct_debug_counters(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(vct_dbg_ctr), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(vct_dbg_ctr), z, sizeof z) != hipSuccess) return -1;
    }
    return 0;
}
#endif
