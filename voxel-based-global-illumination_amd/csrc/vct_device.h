// vct_device.h — device-side spec math shared by the HIP kernels (gfx950).
//
// Every routine here is the device form of a rule of SURVEY.md Appendix A as
// pinned by include/vct_spec.h.  The translation units are compiled with
// -ffp-contract=off, so the operation sequence written here is the one that
// executes; the explicit fmaf() calls are the spec's fused operations.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/vct_spec.h"

namespace vct {

constexpr int kMaxLevels = 11;  // n <= 1024 -> L <= 10

// One step of a cone march with a wave-uniform aperture (A.6): every lane of
// a cone starts at t = 1 and advances by D/2, so (t, D, l0, fr) depend only on
// the step index.  K4 reads them from a per-context table for the diffuse
// cones instead of re-deriving log2 per lane and step.
struct StepRow {
    float t, D, fr;
    int l0;
};
constexpr int kMaxStepRows = 64;   // tan(20 deg) at n = 1024 needs 26 (+1 sentinel)
constexpr int kSpecSlots = 8;
constexpr int kMaxUntilePlanes = 4;   // vct_untile_planes_device      // specular step tables cached per context (distinct roughness values)

// A.6 mip level m = log2(D), D >= 1 (vct_spec.h VCT_LOG2_*).  Host and device:
// the host builds K4's step table with it (vct_trace.hip build_step_table).
__host__ __device__ __forceinline__ float spec_log2(float x) {
    uint32_t bits = __builtin_bit_cast(uint32_t, x);
    int e = (int)((bits >> 23) & 0xffu) - 127;
    float f = __builtin_bit_cast(float, (bits & 0x007fffffu) | 0x3f800000u);
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

// Texel layout of the radiance pyramid in HBM (SURVEY.md A.1 lets the HIP side
// keep a brick-linear internal layout; vct_download_level / vct_upload_level0
// convert to / from linear-Z).  Every face volume of a level is stored as 2x2x2
// bricks of 8 consecutive texels (128 B = one cache line; a trilinear footprint
// touches 1.5^3 = 3.4 lines on average instead of ~4.5 rows of a linear-Z volume;
// round 2: G_rand HBM traffic 302 -> 254 GB per frame), bricks in linear-Z order.

// index of texel (x, y, z) inside one face volume of nl^3 texels (nl a power of two)
__host__ __device__ __forceinline__ uint32_t texel_index(uint32_t x, uint32_t y, uint32_t z, uint32_t nl) {
    const uint32_t nb = nl > 1 ? nl >> 1 : 1u;
    return ((((z >> 1) * nb + (y >> 1)) * nb + (x >> 1)) << 3) | ((z & 1u) << 2) | ((y & 1u) << 1) | (x & 1u);
}

// texel_index for nl = 2^lg from shifts: the same value for every in-range texel
// (x >> 1 < nb); out-of-range coordinates give an unspecified index (never read)
__host__ __device__ __forceinline__ uint32_t texel_index_lg(uint32_t x, uint32_t y, uint32_t z, uint32_t lg) {
    const uint32_t lnb = lg > 0u ? lg - 1u : 0u;
    return (((x >> 1) | ((y >> 1) << lnb) | ((z >> 1) << (2u * lnb))) << 3) | ((z & 1u) << 2) | ((y & 1u) << 1) |
           (x & 1u);
}

// inverse of texel_index: (x, y, z) of index v in a face volume of nl^3 texels
__host__ __device__ __forceinline__ void texel_coords(uint32_t v, uint32_t nl, uint32_t& x, uint32_t& y, uint32_t& z) {
    const uint32_t nb = nl > 1 ? nl >> 1 : 1u, b = v >> 3;
    x = ((b % nb) << 1) | (v & 1u);
    y = (((b / nb) % nb) << 1) | ((v >> 1) & 1u);
    z = ((b / (nb * nb)) << 1) | ((v >> 2) & 1u);
}

// level-0 texel of linear-Z voxel v of an n^3 grid (n a power of two)
__host__ __device__ __forceinline__ uint32_t l0_texel(uint32_t v, uint32_t n) {
    return texel_index(v & (n - 1u), (v / n) & (n - 1u), v / (n * n), n);
}

__device__ __forceinline__ bool occ_at(const unsigned long long* __restrict__ bits, int n, int x, int y, int z) {
    size_t v = (size_t)x + (size_t)n * ((size_t)y + (size_t)n * (size_t)z);
    return (bits[v >> 6] >> (v & 63)) & 1ull;
}

// A.3 shadow walk (Amanatides-Woo) from q (voxel units) toward l over the
// level-0 occupancy bits: 1 = leaves the grid unblocked, 0 = hits a voxel.
__device__ __forceinline__ float dda_visibility(const unsigned long long* __restrict__ bits, int N, float qx, float qy,
                                float qz, float lx, float ly, float lz) {
    int vx = (int)floorf(qx), vy = (int)floorf(qy), vz = (int)floorf(qz);
    if (vx < 0 || vy < 0 || vz < 0 || vx >= N || vy >= N || vz >= N) return 1.0f;
    int sx = lx > 0.0f ? 1 : (lx < 0.0f ? -1 : 0);
    int sy = ly > 0.0f ? 1 : (ly < 0.0f ? -1 : 0);
    int sz = lz > 0.0f ? 1 : (lz < 0.0f ? -1 : 0);
    const float inf = __builtin_inff();
    float tdx = sx ? 1.0f / fabsf(lx) : inf;
    float tdy = sy ? 1.0f / fabsf(ly) : inf;
    float tdz = sz ? 1.0f / fabsf(lz) : inf;
    float tmx = sx > 0 ? ((float)(vx + 1) - qx) * tdx : (sx < 0 ? (qx - (float)vx) * tdx : inf);
    float tmy = sy > 0 ? ((float)(vy + 1) - qy) * tdy : (sy < 0 ? (qy - (float)vy) * tdy : inf);
    float tmz = sz > 0 ? ((float)(vz + 1) - qz) * tdz : (sz < 0 ? (qz - (float)vz) * tdz : inf);
    for (;;) {
        if (occ_at(bits, N, vx, vy, vz)) return 0.0f;
        if (tmx <= tmy && tmx <= tmz) {
            vx += sx; if (vx < 0 || vx >= N) return 1.0f; tmx = tmx + tdx;
        } else if (tmy <= tmz) {
            vy += sy; if (vy < 0 || vy >= N) return 1.0f; tmy = tmy + tdy;
        } else {
            vz += sz; if (vz < 0 || vz >= N) return 1.0f; tmz = tmz + tdz;
        }
    }
}

__device__ __forceinline__ float dot3(float ax, float ay, float az, float bx, float by, float bz) {
    return (ax * bx + ay * by) + az * bz;
}

// ---- diffuse maps (vct_spec.h "diffuse maps") ------------------------------
// Texture t occupies texels [off, off + w*h) of the context's RGBA8 texel array
// (one packed dword per texel: r | g << 8 | b << 16 | a << 24), rows top first.
struct TexDesc {
    uint32_t off, w, h, pad;
};

__device__ __forceinline__ float tex_lerp(float a, float b, float f) { return fmaf(f, b - a, a); }

// T(u, v).rgb: GL_REPEAT wrap, bilinear at the base level, texel centres at +0.5
__device__ __forceinline__ void tex_sample(const uint32_t* __restrict__ texels, TexDesc d, float u, float v,
                                           float& r, float& g, float& b) {
    if (!__builtin_isfinite(u)) u = 0.0f;
    if (!__builtin_isfinite(v)) v = 0.0f;
    const float fu = u - floorf(u), fv = v - floorf(v);
    const float s = fu * (float)d.w - 0.5f, t = fv * (float)d.h - 0.5f;
    const float sx = floorf(s), sy = floorf(t);
    const float ax = s - sx, ay = t - sy;
    int x0 = (int)sx, y0 = (int)sy;          // in [-1, w - 1] / [-1, h - 1]
    int x1 = x0 + 1, y1 = y0 + 1;
    if (x0 < 0) x0 += (int)d.w;
    if (y0 < 0) y0 += (int)d.h;
    if (x1 >= (int)d.w) x1 -= (int)d.w;
    if (y1 >= (int)d.h) y1 -= (int)d.h;
    const uint32_t* base = texels + d.off;
    const uint32_t p00 = base[(size_t)y0 * d.w + x0], p10 = base[(size_t)y0 * d.w + x1];
    const uint32_t p01 = base[(size_t)y1 * d.w + x0], p11 = base[(size_t)y1 * d.w + x1];
    float out[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float t00 = (float)((p00 >> (8 * c)) & 255u) / 255.0f, t10 = (float)((p10 >> (8 * c)) & 255u) / 255.0f;
        const float t01 = (float)((p01 >> (8 * c)) & 255u) / 255.0f, t11 = (float)((p11 >> (8 * c)) & 255u) / 255.0f;
        out[c] = tex_lerp(tex_lerp(t00, t10, ax), tex_lerp(t01, t11, ax), ay);
    }
    r = out[0]; g = out[1]; b = out[2];
}

// K1's (b1, b2): voxel centre (cx, cy, cz) projected onto the plane of q[9], clamped
// into the triangle (vct_spec.h); q in voxel units
__device__ __forceinline__ void tri_bary(const float* __restrict__ q, float cx, float cy, float cz, float& b1,
                                         float& b2) {
    const float e1x = q[3] - q[0], e1y = q[4] - q[1], e1z = q[5] - q[2];
    const float e2x = q[6] - q[0], e2y = q[7] - q[1], e2z = q[8] - q[2];
    const float wx = cx - q[0], wy = cy - q[1], wz = cz - q[2];
    const float d11 = dot3(e1x, e1y, e1z, e1x, e1y, e1z), d12 = dot3(e1x, e1y, e1z, e2x, e2y, e2z);
    const float d22 = dot3(e2x, e2y, e2z, e2x, e2y, e2z);
    const float w1 = dot3(wx, wy, wz, e1x, e1y, e1z), w2 = dot3(wx, wy, wz, e2x, e2y, e2z);
    const float den = d11 * d22 - d12 * d12;
    b1 = 0.0f;
    b2 = 0.0f;
    if (den > 0.0f) {
        b1 = (d22 * w1 - d12 * w2) / den;
        b2 = (d11 * w2 - d12 * w1) / den;
    }
    b1 = fmaxf(b1, 0.0f);
    b2 = fmaxf(b2, 0.0f);
    const float s = b1 + b2;
    if (s > 1.0f) { b1 = b1 / s; b2 = b2 / s; }
}

// uv = fmaf(b2, uv2 - uv0, fmaf(b1, uv1 - uv0, uv0)) per component; uv[6] = u0 v0 u1 v1 u2 v2
__device__ __forceinline__ void tri_uv(const float* __restrict__ uv, float b1, float b2, float& u, float& v) {
    u = fmaf(b2, uv[4] - uv[0], fmaf(b1, uv[2] - uv[0], uv[0]));
    v = fmaf(b2, uv[5] - uv[1], fmaf(b1, uv[3] - uv[1], uv[1]));
}

// 64-lane wave sum (wave64 on CDNA: 6 butterfly steps)
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

}  // namespace vct
