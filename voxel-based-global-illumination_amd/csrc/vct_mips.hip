// vct_mips.hip — K3: 6-face anisotropic (or box-filter) 3D mip pyramid.
//
// SURVEY.md Appendix A.4.  For each parent texel and each face, the four
// child rows along the face axis are composited front-to-back
// (c = f + (1 - f.a) * b) and averaged.  Level 1 reads the isotropic level-0
// radiance grid; level l >= 2 reads the same face of level l-1.
//
// MI355X design: the pyramid is pure HBM streaming (reads 8 texels and writes
// 1 per face).  In the brick layout (vct_device.h VCT_BRICK2) a parent's eight
// children are one 128-byte brick: every read is a whole cache line.  Levels 1..L are built by one launch per level here; the whole
// pyramid at 256^3 is ~475 MB of traffic (~80 us at the measured 6 TB/s).
// One thread owns one parent texel and produces all six faces from the same
// eight (level 1) or 6 x 8 (level >= 2) children, so each child is read once.
#include "vct_internal.h"

namespace vct {
namespace {

__device__ __forceinline__ float4 comp(float4 f, float4 b) {
    float oma = 1.0f - f.w;
    return make_float4(f.x + oma * b.x, f.y + oma * b.y, f.z + oma * b.z, f.w + oma * b.w);
}
__device__ __forceinline__ float4 add4(float4 a, float4 b) {
    return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float4 scale4(float4 a, float s) {
    return make_float4(a.x * s, a.y * s, a.z * s, a.w * s);
}

// ch[dz][dy][dx] -> six faces, row order identical to the oracle (slow, fast)
__device__ __forceinline__ void aniso_faces(const float4 (&ch)[2][2][2], float4 (&out)[6]) {
#pragma unroll
    for (int f = 0; f < 6; ++f) {
        const int axis = f >> 1;
        const int fr = f & 1, bk = 1 - fr;
        float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
        for (int r1 = 0; r1 < 2; ++r1)
#pragma unroll
            for (int r0 = 0; r0 < 2; ++r0) {
                float4 tf, tb;
                if (axis == 0) { tf = ch[r1][r0][fr]; tb = ch[r1][r0][bk]; }
                else if (axis == 1) { tf = ch[r1][fr][r0]; tb = ch[r1][bk][r0]; }
                else { tf = ch[fr][r1][r0]; tb = ch[bk][r1][r0]; }
                acc = add4(acc, comp(tf, tb));
            }
        out[f] = scale4(acc, 0.25f);
    }
}

// children of parent texel (x, y, z) of a level with nc = 2 nl texels per axis:
// ch[dz][dy][dx] = src[texel of (2x + dx, 2y + dy, 2z + dz)]; in the brick layout
// (VCT_BRICK2) the eight are one 128-byte brick of the child level
__device__ __forceinline__ void load_children(const float4* __restrict__ src, uint32_t x, uint32_t y, uint32_t z,
                                              uint32_t nc, float4 (&ch)[2][2][2]) {
#if VCT_BRICK2
    const float4* b = src + ((size_t)texel_index(2 * x, 2 * y, 2 * z, nc));
#pragma unroll
    for (int dz = 0; dz < 2; ++dz)
#pragma unroll
        for (int dy = 0; dy < 2; ++dy)
#pragma unroll
            for (int dx = 0; dx < 2; ++dx) ch[dz][dy][dx] = b[(dz << 2) | (dy << 1) | dx];
#else
#pragma unroll
    for (int dz = 0; dz < 2; ++dz)
#pragma unroll
        for (int dy = 0; dy < 2; ++dy)
#pragma unroll
            for (int dx = 0; dx < 2; ++dx)
                ch[dz][dy][dx] = src[(size_t)(2 * x + dx) + (size_t)nc * ((size_t)(2 * y + dy) + (size_t)nc * (size_t)(2 * z + dz))];
#endif
}

// level 1 from the isotropic level 0; thread v = output texel v (layout order)
__global__ void __launch_bounds__(256) k3_level1(const float4* __restrict__ src, float4* __restrict__ dst,
                                                 int nl, int aniso) {
    const size_t vl = (size_t)nl * nl * nl;
    size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= vl) return;
    uint32_t x, y, z;
    texel_coords((uint32_t)v, (uint32_t)nl, x, y, z);
    float4 ch[2][2][2];
    load_children(src, x, y, z, 2u * (uint32_t)nl, ch);
    if (!aniso) {
        float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
        for (int dz = 0; dz < 2; ++dz)
#pragma unroll
            for (int dy = 0; dy < 2; ++dy)
#pragma unroll
                for (int dx = 0; dx < 2; ++dx) acc = add4(acc, ch[dz][dy][dx]);
        dst[v] = scale4(acc, 0.125f);
        return;
    }
    float4 out[6];
    aniso_faces(ch, out);
#pragma unroll
    for (int f = 0; f < 6; ++f) dst[(size_t)f * vl + v] = out[f];
}

// level l >= 2 from the same faces of level l-1
__global__ void __launch_bounds__(256) k3_levelN(const float4* __restrict__ src, float4* __restrict__ dst,
                                                 int nl, int aniso) {
    const size_t vl = (size_t)nl * nl * nl;
    size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= vl) return;
    uint32_t x, y, z;
    texel_coords((uint32_t)v, (uint32_t)nl, x, y, z);
    const uint32_t nc = 2u * (uint32_t)nl;
    const size_t vc = (size_t)nc * nc * nc;
    const int faces = aniso ? 6 : 1;
    for (int f = 0; f < faces; ++f) {
        float4 ch[2][2][2];
        load_children(src + (size_t)f * vc, x, y, z, nc, ch);
        float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (!aniso) {
#pragma unroll
            for (int dz = 0; dz < 2; ++dz)
#pragma unroll
                for (int dy = 0; dy < 2; ++dy)
#pragma unroll
                    for (int dx = 0; dx < 2; ++dx) acc = add4(acc, ch[dz][dy][dx]);
            dst[v] = scale4(acc, 0.125f);
            continue;
        }
        const int axis = f >> 1, fr = f & 1, bk = 1 - fr;
#pragma unroll
        for (int r1 = 0; r1 < 2; ++r1)
#pragma unroll
            for (int r0 = 0; r0 < 2; ++r0) {
                float4 tf, tb;
                if (axis == 0) { tf = ch[r1][r0][fr]; tb = ch[r1][r0][bk]; }
                else if (axis == 1) { tf = ch[r1][fr][r0]; tb = ch[r1][bk][r0]; }
                else { tf = ch[fr][r1][r0]; tb = ch[bk][r1][r0]; }
                acc = add4(acc, comp(tf, tb));
            }
        dst[(size_t)f * vl + v] = scale4(acc, 0.25f);
    }
}

// one face volume between the pyramid's layout and linear-Z (download / upload)
__global__ void __launch_bounds__(256) k_relayout(const float4* __restrict__ src, float4* __restrict__ dst, uint32_t nl,
                                                  int to_linear) {
    const size_t vl = (size_t)nl * nl * nl;
    const size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= vl) return;
    const uint32_t x = (uint32_t)(v % nl), y = (uint32_t)((v / nl) % nl), z = (uint32_t)(v / ((size_t)nl * nl));
    const size_t t = texel_index(x, y, z, nl);
    if (to_linear) dst[v] = src[t];
    else dst[t] = src[v];
}

}  // namespace

hipError_t launch_mips(vct_ctx* c) {
    Grid& g = c->grid;
    for (uint32_t l = 1; l <= g.L; ++l) {
        const int nl = (int)(g.n >> l);
        const size_t vl = (size_t)nl * nl * nl;
        const uint32_t blocks = (uint32_t)((vl + 255) / 256);
        float4* dst = g.pyr + g.lvl_off[l];
        const float4* src = g.pyr + g.lvl_off[l - 1];
        if (l == 1)
            hipLaunchKernelGGL(k3_level1, dim3(blocks), dim3(256), 0, c->stream, src, dst, nl, g.aniso);
        else
            hipLaunchKernelGGL(k3_levelN, dim3(blocks), dim3(256), 0, c->stream, src, dst, nl, g.aniso);
    }
    return hipGetLastError();
}

hipError_t launch_relayout(vct_ctx* c, const float4* src, float4* dst, uint32_t nl, bool to_linear) {
    const size_t vl = (size_t)nl * nl * nl;
    hipLaunchKernelGGL(k_relayout, dim3((uint32_t)((vl + 255) / 256)), dim3(256), 0, c->stream, src, dst, nl,
                       to_linear ? 1 : 0);
    return hipGetLastError();
}

}  // namespace vct
