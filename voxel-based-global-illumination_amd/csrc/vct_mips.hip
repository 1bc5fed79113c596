// vct_mips.hip — K3: 6-face anisotropic (or box-filter) 3D mip pyramid.
//
// SURVEY.md Appendix A.4.  For each parent texel and each face, the four
// child rows along the face axis are composited front-to-back
// (c = f + (1 - f.a) * b) and averaged.  Level 1 reads the isotropic level-0
// radiance grid; level l >= 2 reads the same face of level l-1.
//
// MI355X design: the pyramid is pure HBM streaming (reads 8 texels and writes
// 1 per face).  In the brick layout (vct_device.h VCT_BRICK2) a parent's eight
// children are one 128-byte brick: every read is a whole cache line.  At 256^3 the
// pyramid moves ~0.7 GB, 0.46 GB of it in level 1.
//  * level 1 (k3_level1): one thread per parent texel reads its eight isotropic
//    children once and writes all six faces;
//  * levels >= 2 with more than 32^3 parents (k3_levelN_face): one thread per
//    (parent texel, face), one 128-B brick in, one texel out -- six times the
//    threads of a thread-per-parent kernel, so the loads of a level are in flight
//    together instead of six dependent rounds;
//  * the small levels (<= 32^3 parents; 6 of the 8 levels at 256^3) in ONE launch
//    (k3_tail): a workgroup builds an 8^3-parent subtree of one face level by level
//    in LDS, and the last workgroup of each face (an atomic ticket) finishes the
//    levels above the subtrees.  Those levels were one launch each, 4-6 us apiece
//    for a few MB.
// Every texel is computed with the same operations in the same order as the oracle.
#include <cstdlib>

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

// one face of a parent from its children (the k3_levelN operation order)
__device__ __forceinline__ float4 face_of(const float4 (&ch)[2][2][2], int f) {
    const int axis = f >> 1, fr = f & 1, bk = 1 - fr;
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
    return scale4(acc, 0.25f);
}

__device__ __forceinline__ float4 box_of(const float4 (&ch)[2][2][2]) {
    float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
    for (int dz = 0; dz < 2; ++dz)
#pragma unroll
        for (int dy = 0; dy < 2; ++dy)
#pragma unroll
            for (int dx = 0; dx < 2; ++dx) acc = add4(acc, ch[dz][dy][dx]);
    return scale4(acc, 0.125f);
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

// level l >= 2, one thread per (parent texel v, face blockIdx.y); aniso = 0: one face, box filter
__global__ void __launch_bounds__(256) k3_levelN_face(const float4* __restrict__ src, float4* __restrict__ dst,
                                                      int nl, int aniso) {
    const size_t vl = (size_t)nl * nl * nl;
    const size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= vl) return;
    const int f = (int)blockIdx.y;
    uint32_t x, y, z;
    texel_coords((uint32_t)v, (uint32_t)nl, x, y, z);
    const uint32_t nc = 2u * (uint32_t)nl;
    const size_t vc = (size_t)nc * nc * nc;
    float4 ch[2][2][2];
    load_children(src + (size_t)f * vc, x, y, z, nc, ch);
    dst[(size_t)f * vl + v] = aniso ? face_of(ch, f) : box_of(ch);
}

// The small levels ls..L in one launch.  Workgroup (b, f): the B^3 parents of level ls
// in block b of face f (B = min(8, n_ls)), then their subtree up to level ls + log2 B in
// LDS; each level is also written to the pyramid.  The last workgroup of face f to
// finish (ticket == blocks - 1, after a device-scope fence) reads the subtree tops of
// every block of the face and builds the levels above them the same way.
struct TailK {
    float4* pyr;
    uint64_t off[kMaxLevels + 1];   // float4 offset of each level
    int n, ls, L, aniso, B, lgB;
    unsigned* tickets;              // [6] per face, left at 0
};

constexpr int kTailB = 8;

// level `l` (edge nl) of face f from the LDS children cin (edge 2E, linear) into cout
// (edge E, linear) and the pyramid; block origin (ox, oy, oz) in level-l texels
__device__ __forceinline__ void tail_level(const TailK& k, const float4* cin, float4* cout, int E, int l,
                                           uint32_t ox, uint32_t oy, uint32_t oz, int f) {
    const int t = (int)threadIdx.x;
    if (t < E * E * E) {
        const int lx = t % E, ly = (t / E) % E, lz = t / (E * E), C = 2 * E;
        float4 ch[2][2][2];
#pragma unroll
        for (int dz = 0; dz < 2; ++dz)
#pragma unroll
            for (int dy = 0; dy < 2; ++dy)
#pragma unroll
                for (int dx = 0; dx < 2; ++dx)
                    ch[dz][dy][dx] = cin[(2 * lx + dx) + C * ((2 * ly + dy) + C * (2 * lz + dz))];
        const float4 r = k.aniso ? face_of(ch, f) : box_of(ch);
        cout[t] = r;
        const uint32_t nl = (uint32_t)k.n >> l;
        k.pyr[k.off[l] + (size_t)f * nl * nl * nl + texel_index(ox + lx, oy + ly, oz + lz, nl)] = r;
    }
    __syncthreads();
}

__global__ void __launch_bounds__(kTailB * kTailB * kTailB) k3_tail(const TailK k) {
    __shared__ float4 sa[kTailB * kTailB * kTailB], sb[kTailB * kTailB * kTailB];
    __shared__ unsigned s_ticket;
    const int f = (int)blockIdx.y, t = (int)threadIdx.x;
    const uint32_t ns = (uint32_t)k.n >> k.ls;              // parents per axis at level ls
    const uint32_t nbx = ns / (uint32_t)k.B;                 // blocks per axis
    const uint32_t b = blockIdx.x;
    const uint32_t bx = b % nbx, by = (b / nbx) % nbx, bz = b / (nbx * nbx);
    // level ls from level ls - 1 in the pyramid (one brick per parent)
    if (t < k.B * k.B * k.B) {
        const int lx = t % k.B, ly = (t / k.B) % k.B, lz = t / (k.B * k.B);
        const uint32_t x = bx * k.B + lx, y = by * k.B + ly, z = bz * k.B + lz, nc = 2u * ns;
        float4 ch[2][2][2];
        load_children(k.pyr + k.off[k.ls - 1] + (size_t)f * nc * nc * nc, x, y, z, nc, ch);
        const float4 r = k.aniso ? face_of(ch, f) : box_of(ch);
        sa[t] = r;
        k.pyr[k.off[k.ls] + (size_t)f * ns * ns * ns + texel_index(x, y, z, ns)] = r;
    }
    __syncthreads();
    float4 *cin = sa, *cout = sb;
    int l = k.ls;
    for (int E = k.B >> 1; E >= 1; E >>= 1) {               // the block's subtree (edge E at level l)
        ++l;
        tail_level(k, cin, cout, E, l, bx * (uint32_t)E, by * (uint32_t)E, bz * (uint32_t)E, f);
        float4* tmp = cin; cin = cout; cout = tmp;
    }
    if (l == k.L) return;                                    // one block per face reached the top
    // the last block of face f builds the levels above the subtree tops.  One lane fences
    // and takes the ticket: a device-scope fence writes back / invalidates the XCD's L2, so
    // every wave doing its own would serialize thousands of them
    __syncthreads();                                         // every wave's stores have been issued
    if (t == 0) {
        __threadfence();                                     // release the block's writes
        s_ticket = atomicAdd(&k.tickets[f], 1u);
    }
    __syncthreads();
    const uint32_t nblocks = nbx * nbx * nbx;
    if (s_ticket != nblocks - 1u) return;
    if (t == 0) __threadfence();                             // acquire the other blocks' writes
    __syncthreads();
    const uint32_t nt = nbx;                                 // subtree tops per axis (level l)
    if ((uint32_t)t < nt * nt * nt) {
        const uint32_t x = t % nt, y = (t / nt) % nt, z = t / (nt * nt);
        sa[t] = k.pyr[k.off[l] + (size_t)f * nt * nt * nt + texel_index(x, y, z, nt)];
    }
    __syncthreads();
    cin = sa;
    cout = sb;
    for (int E = (int)nt >> 1; E >= 1; E >>= 1) {
        ++l;
        tail_level(k, cin, cout, E, l, 0u, 0u, 0u, f);
        float4* tmp = cin; cin = cout; cout = tmp;
    }
    if (t == 0) k.tickets[f] = 0u;                           // ready for the next build
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
    // A/B (VCT_K3_FUSED=1): thread-per-(parent, face) levels + the fused tail launch.  Measured
    // slower than one thread-per-parent launch per level (256^3: 0.219 vs 0.170 ms; 512^3:
    // 1.51 vs 1.17 ms, tools/k3_bench.py): the per-lane 128-B brick reads are uncoalesced
    // either way and the face split only multiplies them; kept for the record
    const bool old = getenv("VCT_K3_FUSED") == nullptr;
    // the small levels (<= 32^3 parents, level >= 2) go to the fused tail launch
    uint32_t ls = 2;
    while (ls <= g.L && (g.n >> ls) > 32u) ++ls;
    for (uint32_t l = 1; l <= g.L && (old || l < ls); ++l) {
        const int nl = (int)(g.n >> l);
        const size_t vl = (size_t)nl * nl * nl;
        const uint32_t blocks = (uint32_t)((vl + 255) / 256);
        float4* dst = g.pyr + g.lvl_off[l];
        const float4* src = g.pyr + g.lvl_off[l - 1];
        if (l == 1)
            hipLaunchKernelGGL(k3_level1, dim3(blocks), dim3(256), 0, c->stream, src, dst, nl, g.aniso);
        else if (old)
            hipLaunchKernelGGL(k3_levelN, dim3(blocks), dim3(256), 0, c->stream, src, dst, nl, g.aniso);
        else
            hipLaunchKernelGGL(k3_levelN_face, dim3(blocks, g.aniso ? 6 : 1), dim3(256), 0, c->stream, src, dst, nl,
                               g.aniso);
    }
    if (!old && ls <= g.L) {
        if (!c->k3_tickets) {
            hipError_t e = hipMalloc((void**)&c->k3_tickets, 64);
            if (e == hipSuccess) e = hipMemsetAsync(c->k3_tickets, 0, 64, c->stream);
            if (e != hipSuccess) return e;
        }
        TailK k;
        k.pyr = g.pyr;
        for (int i = 0; i <= kMaxLevels; ++i) k.off[i] = g.lvl_off[i];
        k.n = (int)g.n;
        k.ls = (int)ls;
        k.L = (int)g.L;
        k.aniso = g.aniso;
        const uint32_t ns = g.n >> ls;
        k.B = (int)(ns < (uint32_t)kTailB ? ns : (uint32_t)kTailB);
        k.lgB = __builtin_ctz((unsigned)k.B);
        k.tickets = c->k3_tickets;
        const uint32_t nbx = ns / (uint32_t)k.B;
        hipLaunchKernelGGL(k3_tail, dim3(nbx * nbx * nbx, g.aniso ? 6 : 1), dim3(kTailB * kTailB * kTailB), 0,
                           c->stream, k);
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
