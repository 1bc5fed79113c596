// vct_voxelize.hip — K1 conservative voxelization + resolve, K2 light injection.
//
// SURVEY.md Appendix A.2 / A.3 (the reference has no implementation: its
// VoxelizationProgram is empty, assets/code/program/p_voxelization.h:4-7).
//
// K1 design (MI355X): triangles are flattened into a balanced 1-D work list of
// (triangle, candidate voxel) pairs: a per-triangle candidate count, a device
// exclusive scan, then one lane per candidate running the exact 13-axis SAT
// test.  A few huge triangles (a Cornell wall covers n^2 voxels) therefore
// spread over the whole chip instead of serialising one wave.  Coverage is
// accumulated with 64-bit integer atomics on 16.16 fixed-point values, so the
// result is independent of atomic arrival order: bit-exact and reproducible.
// Per-voxel accumulators are 64-byte records [albedo rgb, normal xyz, count,
// pad] so a voxel's seven atomics land in one half cache line.  The first hit
// of a voxel sets its occupancy bit; resolve and the next call's reset touch
// only the voxels whose bit is set, so a voxelization costs O(candidates +
// occupied voxels) plus a 2 MiB bitmask scan at 256^3, not a 1 GiB stream
// (ctx invariant: records, voxels and bits are zero where no bit is set).
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "vct_internal.h"

#ifdef VCT_DEBUG_WAVES
// per-wave (start, end, HW_ID | XCC_ID << 32) of the last k2_walk launch (timeline build,
// tools/k2_waves.py); compiled out of the product
constexpr int kDbgK2Waves = 1 << 16;
__device__ unsigned long long vct_dbg_k2_wave[kDbgK2Waves][3];
extern "C" int vct_debug_k2_waves(unsigned long long* out, int n) {
    if (n > kDbgK2Waves) n = kDbgK2Waves;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(vct_dbg_k2_wave), sizeof(unsigned long long) * 3 * n) == hipSuccess ? n : -1;
}
extern "C" int vct_debug_k2_waves_clear() {
    static unsigned long long z[kDbgK2Waves][3];
    return hipMemcpyToSymbol(HIP_SYMBOL(vct_dbg_k2_wave), z, sizeof z) == hipSuccess ? 0 : -1;
}
#endif

namespace vct {
namespace {

struct TriGeom {      // 64 B
    float q[9];       // voxel-unit vertex positions
    int lo[3];        // first candidate voxel per axis
    uint32_t ext[3];  // candidate extent per axis (0 = no candidates)
    uint32_t pad;
};
struct TriFix {       // 64 B
    long long fix[6]; // albedo rgb, face normal xyz in 16.16 fixed point
    long long tex;    // diffuse map of the triangle's material (-1: albedo = Kd, fix[0..2])
    long long pad;
};
struct TriUV {        // 48 B, textured triangles only
    float uv[6];      // TexCoords of the three vertices
    float kd[3];      // material Kd (albedo = Kd x T(uv) per hit)
    uint32_t pad[3];
};

__device__ __forceinline__ float fmin3(float a, float b, float c) { return fminf(fminf(a, b), c); }
__device__ __forceinline__ float fmax3(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }

__device__ __forceinline__ void cand_range(float mn, float mx, int n, int& lo, int& hi) {
    int l = (int)ceilf(fmaxf(mn, -1.0f)) - 1;
    int h = (int)floorf(fminf(mx, (float)n + 1.0f));
    lo = l < 0 ? 0 : l;
    hi = h > n - 1 ? n - 1 : h;
}

__global__ void __launch_bounds__(256) k1_tri_setup(
    const char* __restrict__ verts, uint32_t stride, uint32_t n_verts,
    const uint32_t* __restrict__ idx, uint32_t n_tri, const uint32_t* __restrict__ mat,
    const float4* __restrict__ kd, uint32_t n_mat, const int32_t* __restrict__ map, uint32_t uv_offset,
    uint32_t n_tex, int n, float g0x, float g0y, float g0z,
    float inv_h, TriGeom* __restrict__ geom, TriFix* __restrict__ fixo, TriUV* __restrict__ tuv,
    unsigned long long* __restrict__ counts, float4* __restrict__ mesh_tri, float4* __restrict__ mesh_uv,
    int* __restrict__ err, uint32_t* __restrict__ maxabs) {
    uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_tri) return;
    uint32_t vi[3] = {idx[3 * t], idx[3 * t + 1], idx[3 * t + 2]};
    uint32_t m = mat ? mat[t] : 0u;
    TriGeom g;
    TriFix f;
    // the material's diffuse map (material_map, vct_voxelize_textured); out of range -> error
    const int32_t tex = (map && m < n_mat) ? map[m] : -1;
    if (vi[0] >= n_verts || vi[1] >= n_verts || vi[2] >= n_verts || (kd && m >= n_mat) || (map && m >= n_mat) ||
        tex < -1 || (tex >= 0 && (uint32_t)tex >= n_tex)) {
        atomicOr(err, kK1ErrIndex);
        g.ext[0] = g.ext[1] = g.ext[2] = 0;
        counts[t] = 0;
        geom[t] = g;
        return;
    }
    float p[3][3], q[3][3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float* src = (const float*)(verts + (size_t)vi[k] * stride);
        p[k][0] = src[0]; p[k][1] = src[1]; p[k][2] = src[2];
        q[k][0] = (p[k][0] - g0x) * inv_h;
        q[k][1] = (p[k][1] - g0y) * inv_h;
        q[k][2] = (p[k][2] - g0z) * inv_h;
        g.q[3 * k] = q[k][0]; g.q[3 * k + 1] = q[k][1]; g.q[3 * k + 2] = q[k][2];
    }
    float e1[3] = {p[1][0] - p[0][0], p[1][1] - p[0][1], p[1][2] - p[0][2]};
    float e2[3] = {p[2][0] - p[0][0], p[2][1] - p[0][1], p[2][2] - p[0][2]};
    float fn[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2],
                   e1[0] * e2[1] - e1[1] * e2[0]};
    float len = sqrtf(dot3(fn[0], fn[1], fn[2], fn[0], fn[1], fn[2]));
    if (len > 0.0f) { fn[0] = fn[0] / len; fn[1] = fn[1] / len; fn[2] = fn[2] / len; }
    else { fn[0] = 0.0f; fn[1] = 0.0f; fn[2] = 0.0f; }
    float4 alb = kd ? kd[m] : make_float4(1.0f, 1.0f, 1.0f, 1.0f);
    f.fix[0] = (long long)roundf(alb.x * VCT_FIXED_ONE);
    f.fix[1] = (long long)roundf(alb.y * VCT_FIXED_ONE);
    f.fix[2] = (long long)roundf(alb.z * VCT_FIXED_ONE);
    f.fix[3] = (long long)roundf(fn[0] * VCT_FIXED_ONE);
    f.fix[4] = (long long)roundf(fn[1] * VCT_FIXED_ONE);
    f.fix[5] = (long long)roundf(fn[2] * VCT_FIXED_ONE);
    f.tex = tex;
    f.pad = 0;
    {   // the largest |fixed-point value| a hit of this triangle adds (a textured albedo
        // Kd x T with T <= 1 rounds to at most Kd's); clamped at 2^31
        unsigned long long mx = 0;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const unsigned long long a = (unsigned long long)(f.fix[i] < 0 ? -f.fix[i] : f.fix[i]);
            mx = a > mx ? a : mx;
        }
        const uint32_t m32 = mx >= (1ull << 31) ? (1u << 31) : (uint32_t)mx;
        if (m32 > __hip_atomic_load(maxabs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(maxabs, m32);
    }
    if (tex >= 0) {
        TriUV r;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float* src = (const float*)(verts + (size_t)vi[k] * stride + uv_offset);
            r.uv[2 * k] = src[0];
            r.uv[2 * k + 1] = src[1];
        }
        r.kd[0] = alb.x; r.kd[1] = alb.y; r.kd[2] = alb.z;
        r.pad[0] = r.pad[1] = r.pad[2] = 0;
        tuv[t] = r;
        mesh_uv[2 * t + 0] = make_float4(r.uv[0], r.uv[1], r.uv[2], r.uv[3]);
        mesh_uv[2 * t + 1] = make_float4(r.uv[4], r.uv[5], 0.0f, 0.0f);
    }
    unsigned long long cnt = 1;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        int lo, hi;
        cand_range(fmin3(q[0][a], q[1][a], q[2][a]), fmax3(q[0][a], q[1][a], q[2][a]), n, lo, hi);
        g.lo[a] = lo;
        g.ext[a] = hi >= lo ? (uint32_t)(hi - lo + 1) : 0u;
        cnt *= g.ext[a];
    }
    g.pad = 0;
    geom[t] = g;
    fixo[t] = f;
    counts[t] = cnt;
    // keep the triangle for the G-buffer ray caster (world units)
    mesh_tri[4 * t + 0] = make_float4(p[0][0], p[0][1], p[0][2], 0.0f);
    mesh_tri[4 * t + 1] = make_float4(e1[0], e1[1], e1[2], 0.0f);
    mesh_tri[4 * t + 2] = make_float4(e2[0], e2[1], e2[2], 0.0f);
    mesh_tri[4 * t + 3] = make_float4(alb.x, alb.y, alb.z, __int_as_float(tex));
}

// ---- exclusive scan of per-triangle candidate counts (u64) ----------------
constexpr int kScanBlock = 256, kScanItems = 4, kScanTile = kScanBlock * kScanItems;

__device__ __forceinline__ unsigned long long block_excl_scan(unsigned long long v,
                                                             unsigned long long* sh,
                                                             unsigned long long& total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    unsigned long long x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        unsigned long long y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) sh[wid] = x;
    __syncthreads();
    unsigned long long base = 0;
    for (int w = 0; w < wid; ++w) base += sh[w];
    total = sh[0] + sh[1] + sh[2] + sh[3];
    __syncthreads();
    return base + x - v;
}

__global__ void __launch_bounds__(kScanBlock) k_scan_tiles(const unsigned long long* __restrict__ in,
                                                           unsigned long long* __restrict__ out,
                                                           unsigned long long* __restrict__ tile_sums,
                                                           uint32_t count) {
    __shared__ unsigned long long sh[4];
    const size_t base = (size_t)blockIdx.x * kScanTile + (size_t)threadIdx.x * kScanItems;
    unsigned long long v[kScanItems], s = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        v[i] = base + i < count ? in[base + i] : 0ull;
        s += v[i];
    }
    unsigned long long total;
    unsigned long long ex = block_excl_scan(s, sh, total);
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        if (base + i < count) out[base + i] = ex;
        ex += v[i];
    }
    if (threadIdx.x == 0) tile_sums[blockIdx.x] = total;
}

// single-block carry scan over the tile sums (n_tiles small: n_tri / 1024)
__global__ void __launch_bounds__(kScanBlock) k_scan_carry(unsigned long long* __restrict__ tile_sums,
                                                           uint32_t n_tiles,
                                                           unsigned long long* __restrict__ total_out) {
    __shared__ unsigned long long sh[4];
    unsigned long long carry = 0;
    for (uint32_t b = 0; b < n_tiles; b += kScanBlock) {
        uint32_t i = b + threadIdx.x;
        unsigned long long v = i < n_tiles ? tile_sums[i] : 0ull, tot;
        unsigned long long ex = block_excl_scan(v, sh, tot);
        if (i < n_tiles) tile_sums[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) *total_out = carry;
}

__global__ void __launch_bounds__(kScanBlock) k_scan_add(unsigned long long* __restrict__ out,
                                                         const unsigned long long* __restrict__ tile_sums,
                                                         uint32_t count) {
    const size_t base = (size_t)blockIdx.x * kScanTile;
    const unsigned long long add = tile_sums[blockIdx.x];
    for (int i = threadIdx.x; i < kScanTile; i += kScanBlock)
        if (base + i < count) out[base + i] += add;
}

// ---- exact 13-axis triangle/voxel SAT (same rule as oracle/vct_oracle.c) --
__device__ __forceinline__ bool tri_box_overlap(const float* __restrict__ q, float cx, float cy, float cz) {
    float a0x = q[0] - cx, a0y = q[1] - cy, a0z = q[2] - cz;
    float a1x = q[3] - cx, a1y = q[4] - cy, a1z = q[5] - cz;
    float a2x = q[6] - cx, a2y = q[7] - cy, a2z = q[8] - cz;
    if (fmin3(a0x, a1x, a2x) > 0.5f || fmax3(a0x, a1x, a2x) < -0.5f) return false;
    if (fmin3(a0y, a1y, a2y) > 0.5f || fmax3(a0y, a1y, a2y) < -0.5f) return false;
    if (fmin3(a0z, a1z, a2z) > 0.5f || fmax3(a0z, a1z, a2z) < -0.5f) return false;
    float e[3][3] = {{a1x - a0x, a1y - a0y, a1z - a0z},
                     {a2x - a1x, a2y - a1y, a2z - a1z},
                     {a0x - a2x, a0y - a2y, a0z - a2z}};
    {
        float nx = e[0][1] * e[1][2] - e[0][2] * e[1][1];
        float ny = e[0][2] * e[1][0] - e[0][0] * e[1][2];
        float nz = e[0][0] * e[1][1] - e[0][1] * e[1][0];
        float vminx, vmaxx, vminy, vmaxy, vminz, vmaxz;
        if (nx > 0.0f) { vminx = -0.5f - a0x; vmaxx = 0.5f - a0x; } else { vminx = 0.5f - a0x; vmaxx = -0.5f - a0x; }
        if (ny > 0.0f) { vminy = -0.5f - a0y; vmaxy = 0.5f - a0y; } else { vminy = 0.5f - a0y; vmaxy = -0.5f - a0y; }
        if (nz > 0.0f) { vminz = -0.5f - a0z; vmaxz = 0.5f - a0z; } else { vminz = 0.5f - a0z; vmaxz = -0.5f - a0z; }
        if (dot3(nx, ny, nz, vminx, vminy, vminz) > 0.0f) return false;
        if (!(dot3(nx, ny, nz, vmaxx, vmaxy, vmaxz) >= 0.0f)) return false;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float ex = e[i][0], ey = e[i][1], ez = e[i][2];
        const float ax[3][3] = {{0.0f, -ez, ey}, {ez, 0.0f, -ex}, {-ey, ex, 0.0f}};
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const float ux = ax[j][0], uy = ax[j][1], uz = ax[j][2];
            float p0 = dot3(ux, uy, uz, a0x, a0y, a0z);
            float p1 = dot3(ux, uy, uz, a1x, a1y, a1z);
            float p2 = dot3(ux, uy, uz, a2x, a2y, a2z);
            float rad = 0.5f * ((fabsf(ux) + fabsf(uy)) + fabsf(uz));
            if (fmin3(p0, p1, p2) > rad || fmax3(p0, p1, p2) < -rad) return false;
        }
    }
    return true;
}

constexpr int kCandPerThread = 8;
constexpr int kCandBucket = 512;                 // candidates per bucket of the triangle-lookup table

// bucket b -> the triangle holding candidate b * kCandBucket (triangles whose
// candidate range crosses a bucket start write it; a giant triangle writes many)
__global__ void __launch_bounds__(256) k1_bucket_starts(const unsigned long long* __restrict__ offs, uint32_t n_tri,
                                                        const unsigned long long* __restrict__ total_p,
                                                        uint32_t* __restrict__ starts) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_tri) return;
    const unsigned long long lo = offs[t], hi = t + 1 < n_tri ? offs[t + 1] : *total_p;
    if (hi <= lo) return;                        // no candidates
    for (unsigned long long b = (lo + kCandBucket - 1) / kCandBucket; b * kCandBucket < hi; ++b) starts[b] = t;
}

// one lane = kCandPerThread consecutive (triangle, voxel) candidates.  PACKED: a hit adds
// its six 16.16 values as three 64-bit words, r + 2^32 g, b + 2^32 nx, ny + 2^32 nz, plus
// the count (4 atomics instead of 7; K1 is bound by the L2's atomic rate).  The integer
// sums are the same: a word's total is sum(lo) + 2^32 sum(hi) mod 2^64, which gives both
// sums back exactly while |sum| < 2^31 -- k1_resolve checks count x max|value| for that.
template <bool PACKED>
__global__ void __launch_bounds__(256) k1_candidates(const TriGeom* __restrict__ geom,
                                                     const TriFix* __restrict__ fixr,
                                                     const unsigned long long* __restrict__ offs,
                                                     uint32_t n_tri, const unsigned long long* __restrict__ total_p,
                                                     int n, long long* __restrict__ accum,
                                                     unsigned long long* __restrict__ occ_bits,
                                                     const uint32_t* __restrict__ starts,
                                                     const TriUV* __restrict__ tuv,
                                                     const uint32_t* __restrict__ texels,
                                                     const TexDesc* __restrict__ tdesc) {
    const unsigned long long total = *total_p;
    const unsigned long long c0 = ((unsigned long long)blockIdx.x * blockDim.x + threadIdx.x) * kCandPerThread;
    if (c0 >= total) return;
    // upper_bound(offs, c0) - 1, searched between the triangles of this bucket's start
    // and the next bucket's start (a few steps instead of log2(n_tri) dependent loads)
    const unsigned long long bk = c0 / kCandBucket, nbk = (total + kCandBucket - 1) / kCandBucket;
    uint32_t lo = starts[bk], hi = bk + 1 < nbk ? starts[bk + 1] + 1 : n_tri;
    while (hi - lo > 1) {
        uint32_t mid = (lo + hi) >> 1;
        if (offs[mid] <= c0) lo = mid; else hi = mid;
    }
    uint32_t t = lo;
    while (t + 1 < n_tri && offs[t + 1] <= c0) ++t;  // skip zero-count triangles
    unsigned long long next = t + 1 < n_tri ? offs[t + 1] : total;
    for (int k = 0; k < kCandPerThread; ++k) {
        const unsigned long long c = c0 + k;
        if (c >= total) break;
        while (c >= next) { ++t; next = t + 1 < n_tri ? offs[t + 1] : total; }
        const TriGeom& g = geom[t];
        unsigned long long local = c - offs[t];
        uint32_t ex = g.ext[0], ey = g.ext[1];
        uint32_t x = (uint32_t)(local % ex);
        unsigned long long r = local / ex;
        uint32_t y = (uint32_t)(r % ey);
        uint32_t z = (uint32_t)(r / ey);
        int vx = g.lo[0] + (int)x, vy = g.lo[1] + (int)y, vz = g.lo[2] + (int)z;
        float q[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) q[i] = g.q[i];
        if (!tri_box_overlap(q, (float)vx + 0.5f, (float)vy + 0.5f, (float)vz + 0.5f)) continue;
        size_t v = (size_t)vx + (size_t)n * ((size_t)vy + (size_t)n * (size_t)vz);
        unsigned long long* a = (unsigned long long*)(accum + 8 * v);
        const TriFix& f = fixr[t];
        long long fa[3] = {f.fix[0], f.fix[1], f.fix[2]};
        if (f.tex >= 0) {   // albedo = Kd x T(uv at the voxel centre's projection), per hit
            const TriUV r = tuv[t];
            float b1, b2, u, w, tr, tg, tb;
            tri_bary(q, (float)vx + 0.5f, (float)vy + 0.5f, (float)vz + 0.5f, b1, b2);
            tri_uv(r.uv, b1, b2, u, w);
            tex_sample(texels, tdesc[f.tex], u, w, tr, tg, tb);
            fa[0] = (long long)roundf((r.kd[0] * tr) * VCT_FIXED_ONE);
            fa[1] = (long long)roundf((r.kd[1] * tg) * VCT_FIXED_ONE);
            fa[2] = (long long)roundf((r.kd[2] * tb) * VCT_FIXED_ONE);
        }
        if constexpr (PACKED) {
            atomicAdd(a + 0, (unsigned long long)fa[0] + ((unsigned long long)fa[1] << 32));
            atomicAdd(a + 1, (unsigned long long)fa[2] + ((unsigned long long)f.fix[3] << 32));
            atomicAdd(a + 2, (unsigned long long)f.fix[4] + ((unsigned long long)f.fix[5] << 32));
        } else {
#pragma unroll
            for (int i = 0; i < 3; ++i) atomicAdd(a + i, (unsigned long long)fa[i]);
#pragma unroll
            for (int i = 3; i < 6; ++i) atomicAdd(a + i, (unsigned long long)f.fix[i]);
        }
        if (atomicAdd(a + (PACKED ? 3 : 6), 1ull) == 0ull) atomicOr(occ_bits + (v >> 6), 1ull << (v & 63));   // first hit
    }
}

// Sparse reset before a voxelization: the records, voxels and level-0 texels of
// the voxels the previous one occupied (its occupied list; everything else is
// zero by the ctx invariant), so K1 never streams the n^3 x 64-B accumulators.
// One lane per listed voxel (grid-stride, the count is on the device).
__global__ void __launch_bounds__(256) k1_clear(const uint32_t* __restrict__ list, const uint32_t* __restrict__ n_list,
                                                long long* __restrict__ accum, float4* __restrict__ albedo_occ,
                                                float4* __restrict__ normal, float4* __restrict__ level0, uint32_t n) {
    const uint32_t cnt = *n_list;
    const float4 z4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    const longlong2 z = make_longlong2(0, 0);
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < cnt; i += gridDim.x * 256) {
        const size_t v = list[i];
        longlong2* a = (longlong2*)(accum + 8 * v);
        a[0] = z; a[1] = z; a[2] = z; a[3] = z;
        albedo_occ[v] = z4;
        normal[v] = z4;
        level0[l0_texel((uint32_t)v, n)] = z4;   // K2 wrote only occupied voxels
    }
}

// a packed word's two sums (|sum| < 2^31 each)
__host__ __device__ __forceinline__ void unpack_sums(long long w, long long& lo, long long& hi) {
    lo = (long long)(int32_t)(uint32_t)(unsigned long long)w;
    hi = (long long)(((unsigned long long)w - (unsigned long long)lo)) >> 32;
}

// K1 resolve: accumulators -> albedo/occupancy, normal of the voxels K1 hit (the
// occupied list k2_list builds from their bits; the other voxels stay zero).  PACKED: a
// voxel whose count x max|value| could reach 2^31 ORs kK1ErrRedo into *overflow (the pass's
// error word) instead; the host then repeats the voxelization unpacked
template <bool PACKED>
__device__ __forceinline__ void resolve_voxel(const long long* __restrict__ accum, size_t v,
                                              float4* __restrict__ albedo_occ, float4* __restrict__ normal,
                                              uint32_t maxabs, int* __restrict__ overflow);

template <bool PACKED>
__global__ void __launch_bounds__(256) k1_resolve(const long long* __restrict__ accum,
                                                  const uint32_t* __restrict__ list, const uint32_t* __restrict__ n_list,
                                                  float4* __restrict__ albedo_occ, float4* __restrict__ normal,
                                                  const uint32_t* __restrict__ maxabs_p, int* __restrict__ overflow) {
    const uint32_t cnt = *n_list;
    const uint32_t maxabs = PACKED ? *maxabs_p : 0u;
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < cnt; i += gridDim.x * 256)
        resolve_voxel<PACKED>(accum, list[i], albedo_occ, normal, maxabs, overflow);
}

template <bool PACKED>
__device__ __forceinline__ void resolve_voxel(const long long* __restrict__ accum, size_t v,
                                              float4* __restrict__ albedo_occ, float4* __restrict__ normal,
                                              uint32_t maxabs, int* __restrict__ overflow) {
    long long s[7];
    {
        const longlong2* a = (const longlong2*)(accum + 8 * v);
        longlong2 p0 = a[0], p1 = a[1], p2 = a[2], p3 = a[3];
        if constexpr (PACKED) {
            s[6] = p1.y;
            if ((unsigned long long)s[6] * maxabs >= (1ull << 31)) {
                atomicOr(overflow, kK1ErrRedo);
                return;
            }
            unpack_sums(p0.x, s[0], s[1]);
            unpack_sums(p0.y, s[2], s[3]);
            unpack_sums(p1.x, s[4], s[5]);
        } else {
            s[0] = p0.x; s[1] = p0.y; s[2] = p1.x; s[3] = p1.y; s[4] = p2.x; s[5] = p2.y; s[6] = p3.x;
        }
    }
    const unsigned long long cnt = (unsigned long long)s[6];
    double den = (double)cnt * VCT_FIXED_ONE_D;
    float4 ao = make_float4((float)((double)s[0] / den), (float)((double)s[1] / den),
                            (float)((double)s[2] / den), 1.0f);
    double sx = (double)s[3], sy = (double)s[4], sz = (double)s[5];
    double len = sqrt((sx * sx + sy * sy) + sz * sz);
    float4 nm = len > 0.0 ? make_float4((float)(sx / len), (float)(sy / len), (float)(sz / len), 0.0f)
                          : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    albedo_occ[v] = ao;
    normal[v] = nm;
}

// ---- K2 injection ----------------------------------------------------------
// Work-list form (default):
//   k2_list    occupied voxels from the level-0 occupancy bits (a wave takes 64
//              words; per word, lane j owns bit j: ballot + mbcnt give coalesced
//              slots, one atomic per wave);
//   k2_shade   per occupied voxel: n.l <= 0 -> (0,0,0,1) now, else onto the lit list;
//   k2_coarse  one bit per brick of (n/64)^3 voxels (n >= 64; else per voxel), a
//              64-bit row per (y, z) brick row (at most 64^2 rows = 32 KiB);
//   k2_walk    per lit voxel the A.3 shadow walk, with the coarse bits in LDS: a
//              voxel of an empty brick is empty, so its fine word is not read
//              (same cells, same float sequence, same result).
// Level 0 is zeroed first; every voxel's value depends on that voxel alone, so
// the list order (waves append in any order) does not change the output.
// exclusive prefix sum of one value per thread over a 256-thread block, and the
// block total (4 waves: shuffles within the wave, wave totals through LDS)
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t& total) {
    __shared__ uint32_t wt[4];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t incl = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t t = __shfl_up(incl, off, 64);
        if (lane >= (uint32_t)off) incl += t;
    }
    if (lane == 63) wt[wave] = incl;
    __syncthreads();
    uint32_t before = 0;
    for (uint32_t w = 0; w < wave; ++w) before += wt[w];
    total = wt[0] + wt[1] + wt[2] + wt[3];
    __syncthreads();
    return before + incl - v;
}

__device__ __forceinline__ uint32_t lanes_below(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// one block = 256 words; entries in bitmask order; one atomic per block
__global__ void __launch_bounds__(256) k2_list(const unsigned long long* __restrict__ bits, size_t nwords,
                                               uint32_t* __restrict__ list, uint32_t* __restrict__ count) {
    __shared__ uint32_t s_base;
    const size_t w = (size_t)blockIdx.x * 256 + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63;
    const unsigned long long mine = w < nwords ? bits[w] : 0ull;
    uint32_t total;
    const uint32_t excl = block_excl_scan((uint32_t)__popcll(mine), total);
    if (total == 0) return;                                  // block-uniform
    if (threadIdx.x == 0) s_base = atomicAdd(count, total);
    __syncthreads();
    const uint32_t base = s_base;
    const size_t w0 = w - lane;                              // the wave's first word
    for (int i = 0; i < 64; ++i) {
        const unsigned long long m =
            ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(mine >> 32), i) << 32) |
            (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)mine, i);
        if (m == 0ull) continue;
        const uint32_t start = base + (uint32_t)__builtin_amdgcn_readlane((int)excl, i);
        if ((m >> lane) & 1ull) list[start + lanes_below(m)] = (uint32_t)((w0 + i) * 64 + lane);
    }
}

// one block = a chunk of 16 x 256 occupied entries: unlit voxels get (0,0,0,1)
// now, lit ones go onto the lit list in occupied-list order; one atomic per block
constexpr int kShadeJ = 16;
__global__ void __launch_bounds__(256) k2_shade(const uint32_t* __restrict__ occ, const uint32_t* __restrict__ n_occ,
                                                const float4* __restrict__ normal, float lx, float ly, float lz,
                                                uint32_t* __restrict__ lit, uint32_t* __restrict__ n_lit,
                                                float4* __restrict__ r0, uint32_t n) {
    __shared__ uint32_t s_cnt[kShadeJ * 4];
    __shared__ uint32_t s_base;
    const uint32_t cnt = *n_occ;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t c0 = blockIdx.x * (256 * kShadeJ); c0 < cnt; c0 += gridDim.x * (256 * kShadeJ)) {
        uint32_t flags = 0, vs[kShadeJ];
#pragma unroll
        for (int j = 0; j < kShadeJ; ++j) {
            const uint32_t i = c0 + j * 256 + threadIdx.x;
            vs[j] = 0;
            if (i < cnt) {
                const uint32_t v = occ[i];
                const float4 nm = normal[v];
                const float ndl = dot3(nm.x, nm.y, nm.z, lx, ly, lz);
                if (ndl > 0.0f) flags |= 1u << j;
                else r0[l0_texel(v, n)] = make_float4(0.0f, 0.0f, 0.0f, 1.0f);
                vs[j] = v;
            }
            const unsigned long long b = __ballot((flags >> j) & 1u);
            if (lane == 0) s_cnt[j * 4 + wave] = (uint32_t)__popcll(b);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t run = 0;
            for (int q = 0; q < kShadeJ * 4; ++q) {
                const uint32_t t = s_cnt[q];
                s_cnt[q] = run;
                run += t;
            }
            s_base = run ? atomicAdd(n_lit, run) : 0u;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kShadeJ; ++j) {
            const unsigned long long b = __ballot((flags >> j) & 1u);
            if ((flags >> j) & 1u) lit[s_base + s_cnt[j * 4 + wave] + lanes_below(b)] = vs[j];
        }
        __syncthreads();
    }
}

// coarse occupancy: bit bx of 64-bit row (by, bz) (row by + cn bz; brick edge 2^cs, cn =
// n >> cs <= 64 bricks per axis) is set when any voxel of the brick is occupied
__global__ void __launch_bounds__(256) k2_coarse(const unsigned long long* __restrict__ bits, int n, int cs,
                                                 uint32_t* __restrict__ coarse) {
    const int cn = n >> cs;
    const uint32_t c = blockIdx.x * 256 + threadIdx.x;   // bit c = bx + 64 (by + cn bz)
    const uint32_t ncb = 64u * (uint32_t)cn * cn;
    bool any = false;
    if (c < ncb && (int)(c & 63u) < cn) {
        const int bx = (int)(c & 63u), by = (int)((c >> 6) % cn), bz = (int)((c >> 6) / cn);
        const int e = 1 << cs;
        for (int z = bz * e; z < bz * e + e && !any; ++z)
            for (int y = by * e; y < by * e + e && !any; ++y)
                for (int x = bx * e; x < bx * e + e; x += 64 < e ? 64 : e) {
                    const size_t v = (size_t)x + (size_t)n * ((size_t)y + (size_t)n * (size_t)z);
                    const int len = e < 64 ? e : 64;
                    const unsigned long long m = len == 64 ? ~0ull : ((1ull << len) - 1ull) << (v & 63);
                    if (bits[v >> 6] & m) { any = true; break; }
                }
    }
    const unsigned long long b = __ballot(any);
    if (c < ncb && (c & 31) == 0) coarse[c >> 5] = (uint32_t)(b >> (threadIdx.x & 32));
}

constexpr int kCoarseRows = 64 * 64;              // 64-bit rows: 32 KiB of LDS

// A.3 shadow walk with the coarse bits (LDS) in front of the fine word: the
// dda_visibility() sequence, cell for cell.  The light direction is uniform, so the
// step signs and t increments are too.  n = 2^lgn, cn = 2^lgcn coarse cells per axis
// of edge 2^cs; `bits` covers the n^3 / 8 bytes of the occupancy bit mask (a buffer
// resource: an out-of-range offset reads 0).
template <int kB>
__device__ __forceinline__ float dda_coarse(__amdgpu_buffer_rsrc_t bits, const unsigned long long* __restrict__ cb, int lgn,
                                            int cs, int lgcn, float qx, float qy, float qz, float lx, float ly,
                                            float lz) {
    const uint32_t N = 1u << lgn;
    int vx = (int)floorf(qx), vy = (int)floorf(qy), vz = (int)floorf(qz);
    if (max(max((uint32_t)vx, (uint32_t)vy), (uint32_t)vz) >= N) return 1.0f;
    const int sx = lx > 0.0f ? 1 : (lx < 0.0f ? -1 : 0);
    const int sy = ly > 0.0f ? 1 : (ly < 0.0f ? -1 : 0);
    const int sz = lz > 0.0f ? 1 : (lz < 0.0f ? -1 : 0);
    const float inf = __builtin_inff();
    const float tdx = sx ? 1.0f / fabsf(lx) : inf;
    const float tdy = sy ? 1.0f / fabsf(ly) : inf;
    const float tdz = sz ? 1.0f / fabsf(lz) : inf;
    float tmx = sx > 0 ? ((float)(vx + 1) - qx) * tdx : (sx < 0 ? (qx - (float)vx) * tdx : inf);
    float tmy = sy > 0 ? ((float)(vy + 1) - qy) * tdy : (sy < 0 ? (qy - (float)vy) * tdy : inf);
    float tmz = sz > 0 ? ((float)(vz + 1) - qz) * tdz : (sz < 0 ? (qz - (float)vz) * tdz : inf);
    // batches of kB cells: the walk itself (integer cells, the float t sequence)
    // does not depend on the lookups, so a batch's cells are stepped first, branch-free,
    // with their coarse bits, then the fine words of the coarse-occupied ones are looked
    // up together.  The walk is not frozen where it leaves the grid: every axis moves
    // one way, so once outside it stays outside, and a cell counts only while inside.
    for (;;) {
        uint32_t cv[kB], co = 0u;
#pragma unroll
        for (int b = 0; b < kB; ++b) {
            const uint32_t ux = (uint32_t)vx, uy = (uint32_t)vy, uz = (uint32_t)vz;
            const bool in = max(max(ux, uy), uz) < N;
            cv[b] = ux | (uy << lgn) | (uz << (2 * lgn));
            // unconditional LDS read (an outside cell's row wrapped into the table; its bit
            // is dropped): a select on the address becomes an exec-mask branch that waits
            // for every cell's read on its own
            const unsigned long long row = cb[((uy >> cs) | ((uz >> cs) << lgcn)) & (uint32_t)(kCoarseRows - 1)];
            co |= ((uint32_t)(row >> ((ux >> cs) & 63u)) & (uint32_t)in) << b;
            // the spec's choice (x if tmx <= tmy, tmz; else y if tmy <= tmz; else z) from the
            // minimum: no t is NaN
            const float tmin = fminf(fminf(tmx, tmy), tmz);
            const bool bx = tmx == tmin;
            const bool by = !bx && tmy == tmin;
            const bool bz = !bx && !by;
            const float nx = tmx + tdx, ny = tmy + tdy, nz = tmz + tdz;
            vx += bx ? sx : 0;
            vy += by ? sy : 0;
            vz += bz ? sz : 0;
            tmx = bx ? nx : tmx;
            tmy = by ? ny : tmy;
            tmz = bz ? nz : tmz;
        }
        // fine words only when some lane of the wave met a coarse-occupied cell; a cell
        // whose coarse bit is clear reads past the buffer (0)
        if (__builtin_amdgcn_ballot_w64(co != 0u)) {
            uint32_t hit = 0u;
#pragma unroll
            for (int b = 0; b < kB; ++b) {
                const uint32_t off = (co >> b) & 1u ? (cv[b] >> 6) << 3 : 0x80000000u;
                const auto w = __builtin_amdgcn_raw_buffer_load_b64(bits, off, 0, 0);
                const unsigned long long wd = ((unsigned long long)w[1] << 32) | w[0];
                hit |= (uint32_t)(wd >> (cv[b] & 63u));
            }
            if (hit & 1u) return 0.0f;
        }
        if (max(max((uint32_t)vx, (uint32_t)vy), (uint32_t)vz) >= N) return 1.0f;
    }
}

// one lane per lit voxel; BS-thread blocks share one LDS copy of the coarse bits; KB cells
// per lookup batch
template <int KB, int BS>
__global__ void __launch_bounds__(BS) k2_walk(const uint32_t* __restrict__ lit, const uint32_t* __restrict__ n_lit,
                                                const uint32_t* __restrict__ coarse, int cs,
                                                const float4* __restrict__ albedo_occ,
                                                const float4* __restrict__ normal,
                                                const unsigned long long* __restrict__ bits, int n, float lx,
                                                float ly, float lz, float cr, float cg, float cb,
                                                float4* __restrict__ r0) {
    __shared__ unsigned long long cbits[kCoarseRows];
#ifdef VCT_DEBUG_WAVES
    const unsigned long long wave_t0 = __builtin_amdgcn_s_memrealtime();
#endif
    const uint32_t cnt = *n_lit;
    if (blockIdx.x * BS >= cnt) return;           // block-uniform: no lit voxel for this block
    const int cn = n >> cs;
    const int lgn = __builtin_ctz((uint32_t)n), lgcn = lgn - cs;
    const uint32_t nrow = (uint32_t)cn * cn;
    const unsigned long long* crow = reinterpret_cast<const unsigned long long*>(coarse);
    for (uint32_t i = threadIdx.x; i < nrow; i += BS) cbits[i] = crow[i];
    __syncthreads();
    const __amdgpu_buffer_rsrc_t br =
        __builtin_amdgcn_make_buffer_rsrc((void*)bits, (short)0, (int)(((size_t)n * n * n) >> 3), 0x00020000);
    for (uint32_t i = blockIdx.x * BS + threadIdx.x; i < cnt; i += gridDim.x * BS) {
        const uint32_t v = lit[i];
        const float4 ao = albedo_occ[v];
        const float4 nm = normal[v];
        const float ndl = dot3(nm.x, nm.y, nm.z, lx, ly, lz);
        const int x = (int)(v & (uint32_t)(n - 1)), y = (int)((v >> lgn) & (uint32_t)(n - 1)), z = (int)(v >> (2 * lgn));
        const float vis = dda_coarse<KB>(br, cbits, lgn, cs, lgcn, ((float)x + 0.5f) + nm.x, ((float)y + 0.5f) + nm.y,
                                     ((float)z + 0.5f) + nm.z, lx, ly, lz);
        r0[l0_texel(v, (uint32_t)n)] =
            make_float4(((ao.x * cr) * ndl) * vis, ((ao.y * cg) * ndl) * vis, ((ao.z * cb) * ndl) * vis, 1.0f);
    }
#ifdef VCT_DEBUG_WAVES
    {
        const uint32_t wid = blockIdx.x * (BS >> 6) + (threadIdx.x >> 6);
        if ((threadIdx.x & 63) == 0 && wid < (uint32_t)kDbgK2Waves) {
            vct_dbg_k2_wave[wid][0] = wave_t0;
            vct_dbg_k2_wave[wid][1] = __builtin_amdgcn_s_memrealtime();
            const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);      // HW_REG_HW_ID
            const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);    // HW_REG_XCC_ID
            vct_dbg_k2_wave[wid][2] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
        }
    }
#endif
}

// dense form (one lane per voxel), kept for the voxel-parallel A/B (VCT_K2_DENSE)
__global__ void __launch_bounds__(256) k2_inject(const float4* __restrict__ albedo_occ,
                                                 const float4* __restrict__ normal,
                                                 const unsigned long long* __restrict__ bits, int n,
                                                 float lx, float ly, float lz, float cr, float cg,
                                                 float cb, float4* __restrict__ r0) {
    size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    size_t nv = (size_t)n * n * n;
    if (v >= nv) return;
    float4 ao = albedo_occ[v];
    float4* const dst = r0 + l0_texel((uint32_t)v, (uint32_t)n);
    if (ao.w == 0.0f) { *dst = make_float4(0.0f, 0.0f, 0.0f, 0.0f); return; }
    float4 nm = normal[v];
    float ndl = dot3(nm.x, nm.y, nm.z, lx, ly, lz);
    float4 out = make_float4(0.0f, 0.0f, 0.0f, 1.0f);
    if (ndl > 0.0f) {
        int x = (int)(v % n), y = (int)((v / n) % n), z = (int)(v / ((size_t)n * n));
        float vis = dda_visibility(bits, n, ((float)x + 0.5f) + nm.x, ((float)y + 0.5f) + nm.y,
                                   ((float)z + 0.5f) + nm.z, lx, ly, lz);
        out.x = ((ao.x * cr) * ndl) * vis;
        out.y = ((ao.y * cg) * ndl) * vis;
        out.z = ((ao.z * cb) * ndl) * vis;
    }
    *dst = out;
}

// One voxelization pass.  packed: try the packed accumulators (k1_candidates); a voxel
// whose packed sums could have overflowed makes k1_resolve OR kK1ErrRedo into the pass's
// error word, which the caller reads back with the index-range flag (no extra
// synchronisation) and then repeats the pass unpacked.
hipError_t voxelize_pass(vct_ctx* c, const void* d_verts, uint32_t stride, uint32_t n_verts, const uint32_t* d_idx,
                         uint32_t n_tri, const uint32_t* d_mat, const float4* d_kd, uint32_t n_mat,
                         const int32_t* d_map, uint32_t uv_offset, int* d_err, bool packed) {
    Grid& g = c->grid;
    hipStream_t s = c->stream;
    const size_t nv = (size_t)g.n * g.n * g.n;
    hipError_t e;
    // scratch layout: geom | fix | counts | offsets | tile sums | total, max|value| |
    // textured triangles' UVs
    const uint32_t n_tiles = (n_tri + kScanTile - 1) / kScanTile;
    size_t off_geom = 0;
    size_t off_fix = off_geom + sizeof(TriGeom) * (size_t)n_tri;
    size_t off_cnt = off_fix + sizeof(TriFix) * (size_t)n_tri;
    size_t off_offs = off_cnt + 8 * (size_t)n_tri;
    size_t off_tiles = off_offs + 8 * (size_t)n_tri;
    size_t off_total = off_tiles + 8 * (size_t)(n_tiles + 1);
    size_t off_uv = (off_total + 64 + 255) & ~(size_t)255;
    size_t bytes = off_uv + (d_map ? sizeof(TriUV) * (size_t)n_tri : 0);   // (the bucket table: scratch 7)
    void* sp;
    if ((e = scratch_get(c, 1, bytes, &sp)) != hipSuccess) return e;
    char* base = (char*)sp;
    TriGeom* geom = (TriGeom*)(base + off_geom);
    TriFix* fix = (TriFix*)(base + off_fix);
    unsigned long long* cnt = (unsigned long long*)(base + off_cnt);
    unsigned long long* offs = (unsigned long long*)(base + off_offs);
    unsigned long long* tiles = (unsigned long long*)(base + off_tiles);
    unsigned long long* total = (unsigned long long*)(base + off_total);
    uint32_t* maxabs = (uint32_t*)(base + off_total + 8);
    TriUV* tuv = d_map ? (TriUV*)(base + off_uv) : nullptr;

    // sparse reset of the previous voxelization (its occupied list), then the bits
    const size_t nwords = nv / 64;
    const uint32_t lb = (uint32_t)std::min<size_t>((nv + 255) / 256, 4096);
    hipLaunchKernelGGL(k1_clear, dim3(lb), dim3(256), 0, s, g.occ_list, g.occ_count, g.accum, g.albedo_occ,
                       g.normal, g.pyr, g.n);
    if ((e = hipMemsetAsync(g.occ_bits, 0, nwords * 8, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(g.occ_count, 0, 4, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(total, 0, 16, s)) != hipSuccess) return e;   // total, max|value|
    bool use_packed = false;
    if (n_tri > 0) {
        hipLaunchKernelGGL(k1_tri_setup, dim3((n_tri + 255) / 256), dim3(256), 0, s,
                           (const char*)d_verts, stride, n_verts, d_idx, n_tri, d_mat, d_kd, n_mat, d_map,
                           uv_offset, c->tex.n, (int)g.n, g.g0[0], g.g0[1], g.g0[2], g.inv_h, geom, fix, tuv, cnt,
                           c->mesh.tri, c->mesh.uv, d_err, maxabs);
        hipLaunchKernelGGL(k_scan_tiles, dim3(n_tiles), dim3(kScanBlock), 0, s, cnt, offs, tiles, n_tri);
        hipLaunchKernelGGL(k_scan_carry, dim3(1), dim3(kScanBlock), 0, s, tiles, n_tiles, total);
        hipLaunchKernelGGL(k_scan_add, dim3(n_tiles), dim3(kScanBlock), 0, s, offs, tiles, n_tri);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        // the candidate total is only known on the device: read it back to size the grid
        // (with the largest |value| a hit adds)
        unsigned long long h_head[2] = {0, 0};
        if ((e = hipMemcpyAsync(h_head, total, 16, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        const unsigned long long h_total = h_head[0];
        const uint32_t h_maxabs = (uint32_t)h_head[1];
        // a voxel's count never exceeds n_tri: with n_tri x max|value| < 2^31 the resolve's
        // overflow check can never fire; otherwise it may (then the caller repeats the pass
        // unpacked).  When a handful of hits could already overflow: unpacked outright
        const unsigned long long safe = h_maxabs ? ((1ull << 31) - 1) / h_maxabs : ~0ull;
        use_packed = packed && safe >= 256;
        if (h_total > 0) {
            unsigned long long threads = (h_total + kCandPerThread - 1) / kCandPerThread;
            unsigned long long blocks = (threads + 255) / 256;
            if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
            const unsigned long long nbk = (h_total + kCandBucket - 1) / kCandBucket;
            void* bp;
            if ((e = scratch_get(c, 7, (size_t)nbk * 4, &bp)) != hipSuccess) return e;
            uint32_t* starts = (uint32_t*)bp;
            hipLaunchKernelGGL(k1_bucket_starts, dim3((n_tri + 255) / 256), dim3(256), 0, s, offs, n_tri, total,
                               starts);
            if (use_packed)
                hipLaunchKernelGGL(k1_candidates<true>, dim3((uint32_t)blocks), dim3(256), 0, s, geom, fix, offs,
                                   n_tri, total, (int)g.n, g.accum, g.occ_bits, starts, tuv, c->tex.texels,
                                   c->tex.desc);
            else
                hipLaunchKernelGGL(k1_candidates<false>, dim3((uint32_t)blocks), dim3(256), 0, s, geom, fix, offs,
                                   n_tri, total, (int)g.n, g.accum, g.occ_bits, starts, tuv, c->tex.texels,
                                   c->tex.desc);
        }
    }
    // the occupied list (kept for the next reset and for K2), then resolve it
    hipLaunchKernelGGL(k2_list, dim3((uint32_t)((nwords + 255) / 256)), dim3(256), 0, s, g.occ_bits, nwords,
                       g.occ_list, g.occ_count);
    g.accum_packed = use_packed;
    if (use_packed)
        hipLaunchKernelGGL(k1_resolve<true>, dim3(lb), dim3(256), 0, s, g.accum, g.occ_list, g.occ_count,
                           g.albedo_occ, g.normal, maxabs, d_err);
    else
        hipLaunchKernelGGL(k1_resolve<false>, dim3(lb), dim3(256), 0, s, g.accum, g.occ_list, g.occ_count,
                           g.albedo_occ, g.normal, maxabs, d_err);
    return hipGetLastError();
}

}  // namespace

// K1.  Packed accumulators by default (VCT_K1_PACKED=0, read once: the seven-atomic form,
// for A/B).  packed = false forces the seven-atomic form: the caller's repeat of a pass whose
// error word came back with kK1ErrRedo (its occupied list drives the repeat's sparse reset),
// so the result is the same either way.
hipError_t launch_voxelize(vct_ctx* c, const void* d_verts, uint32_t stride,
                           uint32_t n_verts, const uint32_t* d_idx, uint32_t n_tri, const uint32_t* d_mat,
                           const float4* d_kd, uint32_t n_mat, const int32_t* d_map, uint32_t uv_offset,
                           int* d_err, bool packed) {
    static const bool packed_env = [] {
        const char* v = getenv("VCT_K1_PACKED");
        return !(v && strcmp(v, "0") == 0);
    }();
    return voxelize_pass(c, d_verts, stride, n_verts, d_idx, n_tri, d_mat, d_kd, n_mat, d_map, uv_offset, d_err,
                         packed && packed_env);
}

namespace {
// Grid dumps (vct_save_grid / vct_load_grid): K1's state is the occupied voxels' integer
// sums and counts.  k1_gather reads them (unpacking a packed record) as [i][7] int64:
// albedo rgb, normal xyz, count; k1_restore writes such records back into the (cleared)
// seven-atomic layout and sets the voxels' occupancy bits.
__global__ void __launch_bounds__(256) k1_gather(const uint32_t* __restrict__ idx, uint32_t cnt,
                                                 const long long* __restrict__ accum, int packed,
                                                 long long* __restrict__ out) {
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < cnt; i += gridDim.x * 256) {
        const longlong2* a = (const longlong2*)(accum + 8 * (size_t)idx[i]);
        const longlong2 p0 = a[0], p1 = a[1], p2 = a[2], p3 = a[3];
        long long s[7];
        if (packed) {
            unpack_sums(p0.x, s[0], s[1]);
            unpack_sums(p0.y, s[2], s[3]);
            unpack_sums(p1.x, s[4], s[5]);
            s[6] = p1.y;
        } else {
            s[0] = p0.x; s[1] = p0.y; s[2] = p1.x; s[3] = p1.y; s[4] = p2.x; s[5] = p2.y; s[6] = p3.x;
        }
        for (int j = 0; j < 7; ++j) out[7 * (size_t)i + j] = s[j];
    }
}

__global__ void __launch_bounds__(256) k1_restore(const uint32_t* __restrict__ idx, uint32_t cnt,
                                                  const long long* __restrict__ rec, long long* __restrict__ accum,
                                                  unsigned long long* __restrict__ bits) {
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < cnt; i += gridDim.x * 256) {
        const size_t v = idx[i];
        long long* a = accum + 8 * v;
        for (int j = 0; j < 7; ++j) a[j] = rec[7 * (size_t)i + j];
        atomicOr(bits + (v >> 6), 1ull << (v & 63));
    }
}
}  // namespace

hipError_t launch_k1_gather(vct_ctx* c, const uint32_t* d_idx, uint32_t cnt, long long* d_rec) {
    if (cnt == 0) return hipSuccess;
    hipLaunchKernelGGL(k1_gather, dim3(std::min<uint32_t>((cnt + 255) / 256, 4096)), dim3(256), 0, c->stream, d_idx,
                       cnt, (const long long*)c->grid.accum, c->grid.accum_packed ? 1 : 0, d_rec);
    return hipGetLastError();
}

hipError_t launch_k1_restore(vct_ctx* c, const uint32_t* d_idx, uint32_t cnt, const long long* d_rec) {
    Grid& g = c->grid;
    hipStream_t s = c->stream;
    const size_t nv = (size_t)g.n * g.n * g.n, nwords = nv / 64;
    const uint32_t lb = (uint32_t)std::min<size_t>((nv + 255) / 256, 4096);
    // the previous voxelization's sparse reset, as a K1 pass starts (voxelize_pass)
    hipLaunchKernelGGL(k1_clear, dim3(lb), dim3(256), 0, s, g.occ_list, g.occ_count, g.accum, g.albedo_occ,
                       g.normal, g.pyr, g.n);
    hipError_t e;
    if ((e = hipMemsetAsync(g.occ_bits, 0, nwords * 8, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(g.occ_count, 0, 4, s)) != hipSuccess) return e;
    if (cnt)
        hipLaunchKernelGGL(k1_restore, dim3(std::min<uint32_t>((cnt + 255) / 256, 4096)), dim3(256), 0, s, d_idx,
                           cnt, d_rec, g.accum, g.occ_bits);
    hipLaunchKernelGGL(k2_list, dim3((uint32_t)((nwords + 255) / 256)), dim3(256), 0, s, g.occ_bits, nwords,
                       g.occ_list, g.occ_count);
    g.accum_packed = false;
    hipLaunchKernelGGL(k1_resolve<false>, dim3(lb), dim3(256), 0, s, g.accum, g.occ_list, g.occ_count,
                       g.albedo_occ, g.normal, (const uint32_t*)nullptr, (int*)nullptr);
    return hipGetLastError();
}

hipError_t launch_inject(vct_ctx* c, float lx, float ly, float lz, float cr, float cg, float cb) {
    Grid& g = c->grid;
    const size_t nv = (size_t)g.n * g.n * g.n;
    if (getenv("VCT_K2_DENSE")) {
        hipLaunchKernelGGL(k2_inject, dim3((uint32_t)((nv + 255) / 256)), dim3(256), 0, c->stream,
                           g.albedo_occ, g.normal, g.occ_bits, (int)g.n, lx, ly, lz, cr, cg, cb, g.pyr);
        return hipGetLastError();
    }
    // the occupied list is K1's (g.occ_list); the lit list, coarse bits here; then
    // one lane per occupied / lit voxel (n^3 <= 2^30: 32-bit entries)
    int cs = 0;
    while ((g.n >> cs) > 64) ++cs;
    const uint32_t cn = g.n >> cs;                       // coarse bricks per axis (<= 64): 2 cn^2 words
    void* sp = nullptr;
    hipError_t e = scratch_get(c, 4, 256 + nv * 4, &sp);
    if (e != hipSuccess) return e;
    uint32_t* counts = (uint32_t*)sp;            // [0] lit
    uint32_t* lit = (uint32_t*)((char*)sp + 256);
    uint32_t* coarse = g.k2_coarse;              // 64-bit rows, one per (y, z) brick row
    hipStream_t s = c->stream;
    if ((e = hipMemsetAsync(counts, 0, 4, s)) != hipSuccess) return e;
    // level 0 is zero outside the occupied voxels (K1's reset clears what K2 wrote)
    // unless a dense upload replaced it since
    if (g.l0_dense) {
        if ((e = hipMemsetAsync(g.pyr, 0, nv * sizeof(float4), s)) != hipSuccess) return e;
        g.l0_dense = false;
    }
    if (!g.k2_coarse_ok) {                       // the first K2 after K1: the occupancy's coarse bits
        hipLaunchKernelGGL(k2_coarse, dim3((64 * cn * cn + 255) / 256), dim3(256), 0, s, g.occ_bits, (int)g.n, cs,
                           coarse);
        g.k2_coarse_ok = true;
    }
    const uint32_t blocks = (uint32_t)std::min<size_t>((nv / 64 + 255) / 256 + 1, 4096);
    hipLaunchKernelGGL(k2_shade, dim3(blocks), dim3(256), 0, s, g.occ_list, g.occ_count, g.normal, lx, ly, lz, lit,
                       counts, g.pyr, g.n);
    // A/B (VCT_K2_WALK = batch cells * 10000 + block threads, VCT_K2_GRID = blocks): default
    // 16 cells per lookup batch, 256-thread blocks, 2048 of them.  Measured (tools/k2_bench.py,
    // 256^3): atrium 0.186 -> 0.143 ms, courtyard 0.195 -> 0.181 ms against 8 cells x 1024
    // threads: smaller blocks finish their slowest wave sooner and free the CU for the next
    static const int walk = [] {
        const char* v = getenv("VCT_K2_WALK");
        return v ? atoi(v) : 160256;
    }();
    static const uint32_t wgrid = [] {
        const char* v = getenv("VCT_K2_GRID");
        return v ? (uint32_t)atoi(v) : 0u;
    }();
#define VCT_K2_WALK_LAUNCH(KB, BS)                                                                               \
    hipLaunchKernelGGL((k2_walk<KB, BS>), dim3(wgrid ? wgrid : 512u * 1024u / BS), dim3(BS), 0, s, lit, counts,   \
                       coarse, cs, g.albedo_occ, g.normal, g.occ_bits, (int)g.n, lx, ly, lz, cr, cg, cb, g.pyr)
    switch (walk) {
        case 160128: VCT_K2_WALK_LAUNCH(16, 128); break;
        case 160512: VCT_K2_WALK_LAUNCH(16, 512); break;
        case 161024: VCT_K2_WALK_LAUNCH(16, 1024); break;
        case 80256: VCT_K2_WALK_LAUNCH(8, 256); break;
        case 40256: VCT_K2_WALK_LAUNCH(4, 256); break;
        case 41024: VCT_K2_WALK_LAUNCH(4, 1024); break;
        case 81024: VCT_K2_WALK_LAUNCH(8, 1024); break;
        case 320256: VCT_K2_WALK_LAUNCH(32, 256); break;
        case 80128: VCT_K2_WALK_LAUNCH(8, 128); break;
        default: VCT_K2_WALK_LAUNCH(16, 256); break;
    }
#undef VCT_K2_WALK_LAUNCH
    return hipGetLastError();
}

}  // namespace vct
