// vct_mips.hip — K3: 6-face anisotropic (or box-filter) 3D mip pyramid.
//
// SURVEY.md Appendix A.4.  For each parent texel and each face, the four
// child rows along the face axis are composited front-to-back
// (c = f + (1 - f.a) * b) and averaged.  Level 1 reads the isotropic level-0
// radiance grid; level l >= 2 reads the same face of level l-1.
//
// MI355X design: the pyramid is pure HBM streaming.  In the brick layout (vct_device.h
// texel_index) a parent's eight children are one 128-byte brick, and the bricks of a row of
// parents are contiguous.  k3_block: a workgroup owns an E^3 block of parents of level l
// (E = min(8, n_l)) and builds their whole subtree, levels l .. l + log2 E, in LDS:
//  * its 512 child bricks are staged through LDS with coalesced loads (a wave-instruction
//    reads 1 KB contiguous: eight bricks of a row), so every load instruction touches 8
//    cache lines instead of the 64 of a lane-per-parent brick read (the per-level
//    kernels below ran level 1 at 5.2 TB/s and level 2 at 4.3 TB/s that way);
//  * levels l+1 .. l+log2 E come from LDS, so only level 0 and the subtree tops are ever
//    read from HBM: at 256^3 one launch reads level 0 (268 MB) and writes levels 1-4 of
//    all six faces (230 MB); a second one (6 workgroups) builds levels 5-8.  The
//    per-level plan read every level back (695 MB) in 8 launches.
// Level 1 of an anisotropic pyramid takes the isotropic level 0 and writes all six faces
// (each thread: one parent, six faces); levels >= 2 read the same face (blockIdx.y).
// VCT_K3_PLAN=level selects the per-level kernels (one launch per level) for A/B.
// Every texel is computed with the same operations in the same order as the oracle.
#include <cstdlib>
#include <cstring>

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
// the eight are one 128-byte brick of the child level
__device__ __forceinline__ void load_children(const float4* __restrict__ src, uint32_t x, uint32_t y, uint32_t z,
                                              uint32_t nc, float4 (&ch)[2][2][2]) {
    const float4* b = src + ((size_t)texel_index(2 * x, 2 * y, 2 * z, nc));
#pragma unroll
    for (int dz = 0; dz < 2; ++dz)
#pragma unroll
        for (int dy = 0; dy < 2; ++dy)
#pragma unroll
            for (int dx = 0; dx < 2; ++dx) ch[dz][dy][dx] = b[(dz << 2) | (dy << 1) | dx];
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

// face_of for a face known only at run time: one constant-index body per face (a
// run-time index into ch would put the children in scratch)
__device__ __forceinline__ float4 face_rt(const float4 (&ch)[2][2][2], int f) {
    switch (f) {
        case 0: return face_of(ch, 0);
        case 1: return face_of(ch, 1);
        case 2: return face_of(ch, 2);
        case 3: return face_of(ch, 3);
        case 4: return face_of(ch, 4);
        default: return face_of(ch, 5);
    }
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

// The subtree of an E^3 block of parents of level l (blockIdx.x = block, blockIdx.y = face
// for MODE kFace).  LDS: the staged child bricks (brick c at slots 9c .. 9c + 7: a
// ds_read_b128 lane group of 16 consecutive parents hits 16 distinct bank quads), then,
// in the same array, each level's results (linear, x fastest) for the next one.
enum { kIso6 = 0, kFace = 1, kBox = 2 };
constexpr int kBlk = 8;                       // block edge (parents of level l)

struct BlockK {
    float4* pyr;
    uint64_t off[kMaxLevels + 1];             // float4 offset of each level
    int n, l;                                 // grid edge, first level built
    int brick_writes;                         // level l stored in brick order from LDS (VCT_K3_WRITE)
    uint32_t* b0;                             // level 1 from level 0: the level-0 nonzero bits (Grid::b0), or null
    const uint32_t* live;                     // relight build: workgroup i builds block live[i] (Grid::k3_live_list), or null
};

template <int MODE, int BZ>
__global__ void __launch_bounds__(kBlk * kBlk * BZ) k3_block(const BlockK k) {
    constexpr int kT = kBlk * kBlk * BZ;      // threads: one per parent of a full block
    __shared__ float4 st[kT * 9];

    constexpr int FACES = MODE == kIso6 ? 6 : 1;
    const int t = (int)threadIdx.x;
    const int f0 = MODE == kFace ? (int)blockIdx.y : 0;
    const uint32_t nl = (uint32_t)k.n >> k.l, nc = 2u * nl;
    // block of E x E x Ez parents (E = min(8, n_l), Ez = min(BZ, n_l))
    const int E = nl < (uint32_t)kBlk ? (int)nl : kBlk, Ez = nl < (uint32_t)BZ ? (int)nl : BZ, E3 = E * E * Ez;
    // relight build: only the blocks with an occupied voxel (the others read only +0, and
    // their subtree already holds what this build would write)
    const uint32_t nbk = nl / (uint32_t)E, b = k.live ? k.live[blockIdx.x] : blockIdx.x;
    const uint32_t X0 = (b % nbk) * E, Y0 = ((b / nbk) % nbk) * E, Z0 = (b / (nbk * nbk)) * Ez;
    // children: face f0 of level l-1 (level 0 for kIso6 and level 1 of kBox)
    const float4* src = k.pyr + k.off[k.l - 1] + (MODE == kFace ? (size_t)f0 * nc * nc * nc : 0);
    // staging: float4 u = 8 c + j of the block's child bricks (c linear over the block's
    // parents, x fastest; the child brick of parent (x, y, z) is brick x + nl (y + nl z))
    {
        // (u < E3 * 8 always holds for a full block; a smaller one clamps its spare loads)
        float4 r[8];
        const int lim = E3 * 8 - 1;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int u = min(i * kT + t, lim);
            const int c = u >> 3, j = u & 7;
            const uint32_t cx = (uint32_t)(c % E), cy = (uint32_t)((c / E) % E), cz = (uint32_t)(c / (E * E));
            const size_t brick = (size_t)(X0 + cx) + (size_t)nl * ((size_t)(Y0 + cy) + (size_t)nl * (Z0 + cz));
            r[i] = src[brick * 8 + j];
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int u = i * kT + t;
            if (u <= lim) st[(u >> 3) * 9 + (u & 7)] = r[i];
        }
        if (MODE != kFace && k.b0 && E == kBlk) {
            // the K4 empty-space maps' input: a wave's load i covers the eight child bricks of
            // one x-row of parents, 64 consecutive level-0 texel indices starting at a
            // multiple of 64, so its ballot of "not +0" is one 64-bit word of Grid::b0
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const unsigned long long m = __builtin_amdgcn_ballot_w64(
                    (__float_as_uint(r[i].x) | __float_as_uint(r[i].y) | __float_as_uint(r[i].z) |
                     __float_as_uint(r[i].w)) != 0u);
                const int c = (i * kT + (t & ~63)) >> 3;
                const uint32_t cy = (uint32_t)((c / E) % E), cz = (uint32_t)(c / (E * E));
                const size_t brick = (size_t)X0 + (size_t)nl * ((size_t)(Y0 + cy) + (size_t)nl * (Z0 + cz));
                if ((t & 63) == 0) reinterpret_cast<unsigned long long*>(k.b0)[brick >> 3] = m;
            }
        }
    }
    __syncthreads();
    // level l: thread t = parent t of the block
    float4 out[FACES];
    if (t < E3) {
        float4 ch[2][2][2];
#pragma unroll
        for (int j = 0; j < 8; ++j) ch[j >> 2][(j >> 1) & 1][j & 1] = st[t * 9 + j];
        if constexpr (MODE == kIso6) aniso_faces(ch, out);
        else if constexpr (MODE == kFace) out[0] = face_rt(ch, f0);
        else out[0] = box_of(ch);
    }
    __syncthreads();                          // every staged brick has been read
    const size_t vl = (size_t)nl * nl * nl;
    if (E == kBlk && Ez == BZ && k.brick_writes) {
        // results to LDS first; then thread t writes texel t of the block in brick order
        // (bricks of 2^3 parents, 4 per row: a wave stores two 512-B runs per face)
        if (t < E3) {
#pragma unroll
            for (int f = 0; f < FACES; ++f) st[f * E3 + t] = out[f];
        }
        __syncthreads();
        const int q = t >> 3, j = t & 7;
        const int bx = q & 3, by = (q >> 2) & 3, bz = q >> 4;
        const int lin = (2 * bx + (j & 1)) + kBlk * ((2 * by + ((j >> 1) & 1)) + kBlk * (2 * bz + (j >> 2)));
        const uint32_t nb = nl >> 1;
        const size_t brick = (size_t)((X0 >> 1) + (uint32_t)bx) +
                             (size_t)nb * ((size_t)((Y0 >> 1) + (uint32_t)by) + (size_t)nb * ((Z0 >> 1) + (uint32_t)bz));
#pragma unroll
        for (int f = 0; f < FACES; ++f) k.pyr[k.off[k.l] + (size_t)(f0 + f) * vl + brick * 8 + (size_t)j] = st[f * E3 + lin];
    } else if (t < E3) {
        const uint32_t x = X0 + (uint32_t)(t % E), y = Y0 + (uint32_t)((t / E) % E), z = Z0 + (uint32_t)(t / (E * E));
        const size_t ti = texel_index(x, y, z, nl);
#pragma unroll
        for (int f = 0; f < FACES; ++f) {
            st[f * E3 + t] = out[f];
            k.pyr[k.off[k.l] + (size_t)(f0 + f) * vl + ti] = out[f];
        }
    }
    __syncthreads();
    // levels l+1 ..: from the previous level's results in LDS (face-major, linear), while
    // every block edge still halves (log2 Ez levels)
    int base = 0, Ein = E, Ezin = Ez, l = k.l;
    for (int Eo = E >> 1, Ezo = Ez >> 1; Ezo >= 1; Eo >>= 1, Ezo >>= 1) {
        ++l;
        const int cnt = Eo * Eo * Ezo, nin = Ein * Ein * Ezin, nb = base + FACES * nin;
        const uint32_t no = (uint32_t)k.n >> l;
        if (t < FACES * cnt) {
            const int f = t / cnt, q = t % cnt;
            const int qx = q % Eo, qy = (q / Eo) % Eo, qz = q / (Eo * Eo);
            const float4* cin = st + base + f * nin;
            float4 ch[2][2][2];
#pragma unroll
            for (int dz = 0; dz < 2; ++dz)
#pragma unroll
                for (int dy = 0; dy < 2; ++dy)
#pragma unroll
                    for (int dx = 0; dx < 2; ++dx)
                        ch[dz][dy][dx] = cin[(2 * qx + dx) + Ein * ((2 * qy + dy) + Ein * (2 * qz + dz))];
            const float4 r = MODE == kBox ? box_of(ch) : face_rt(ch, f0 + f);
            st[nb + t] = r;
            const uint32_t ox = X0 >> (l - k.l), oy = Y0 >> (l - k.l), oz = Z0 >> (l - k.l);
            k.pyr[k.off[l] + (size_t)(f0 + f) * no * no * no +
                  texel_index(ox + (uint32_t)qx, oy + (uint32_t)qy, oz + (uint32_t)qz, no)] = r;
        }
        __syncthreads();
        base = nb;
        Ein = Eo;
        Ezin = Ezo;
    }
}

// K4 empty-space maps (Grid::zmap).  occ(m, v): level-m texel v (linear-Z) may be nonzero.
// m = 1 reads the byte of b0 holding the eight level-0 children of v (brick order); m >= 2
// reads the occupancy bytes built from the level below.
__device__ __forceinline__ bool occ_at_level(const uint8_t* __restrict__ b0, const uint8_t* __restrict__ occ,
                                             uint32_t nm, uint32_t x, uint32_t y, uint32_t z) {
    const size_t v = (size_t)x + (size_t)nm * ((size_t)y + (size_t)nm * z);
    return (b0 ? b0[v] : occ[v]) != 0;
}

// level-m occupancy bytes from level m-1 (m = 2: from b0)
__global__ void __launch_bounds__(256) k_occ_down(const uint8_t* __restrict__ b0, const uint8_t* __restrict__ src,
                                                  uint8_t* __restrict__ dst, uint32_t nm) {
    const size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= (size_t)nm * nm * nm) return;
    const uint32_t x = (uint32_t)(v % nm), y = (uint32_t)((v / nm) % nm), z = (uint32_t)(v / ((size_t)nm * nm));
    const uint32_t ns = 2u * nm;
    bool any = false;
#pragma unroll
    for (int a = 0; a < 8; ++a)
        any |= occ_at_level(b0, src, ns, 2u * x + (a & 1), 2u * y + ((a >> 1) & 1), 2u * z + (a >> 2));
    dst[v] = any ? 1u : 0u;
}

// map m: bit of padded position P (p = P - 1 in [-1, nm - 1]^3) = OR of occ over p + {0,1}^3.
// One thread per dword (32 positions of a row): per texel row (y, z) it packs the
// occupancy of texels x0 - 1 .. x0 + 31 (x0 = 32 wx) from nine dword loads of the byte map,
// dilates along x (bit b | bit b + 1) and ORs the four rows p_y + {0,1} x p_z + {0,1}.
__device__ __forceinline__ uint32_t zbits_word(const uint8_t* __restrict__ bytes, uint32_t nm, uint32_t wx,
                                               uint32_t py, uint32_t pz) {
    const int x0 = (int)(wx * 32u);
    uint32_t bits = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int y = (int)py - 1 + (r & 1), z = (int)pz - 1 + (r >> 1);
        if (y < 0 || z < 0 || y >= (int)nm || z >= (int)nm) continue;
        const uint32_t* row = reinterpret_cast<const uint32_t*>(bytes + ((size_t)z * nm + (size_t)y) * nm);
        unsigned long long t = 0;                    // bit b: texel x0 - 1 + b may be nonzero
#pragma unroll
        for (int q = 0; q < 9; ++q) {
            const int o = x0 - 4 + 4 * q;            // texels o .. o + 3 (nm is a multiple of 4)
            if (o < 0 || o >= (int)nm) continue;
            const uint32_t v = row[o >> 2];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int b = o + j - x0 + 1;        // texels x0 - 4 .. x0 - 2 fall outside
                if (b >= 0 && ((v >> (8 * j)) & 0xffu)) t |= 1ull << b;
            }
        }
        bits |= (uint32_t)(t | (t >> 1));
    }
    return bits;
}

__global__ void __launch_bounds__(256) k_zbits(const uint8_t* __restrict__ bytes, uint32_t nm,
                                               uint32_t* __restrict__ dst, uint32_t dim, uint32_t rw) {
    const size_t wi = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (wi >= (size_t)dim * dim * rw) return;
    dst[wi] = zbits_word(bytes, nm, (uint32_t)(wi % rw), (uint32_t)((wi / rw) % dim), (uint32_t)(wi / ((size_t)rw * dim)));
}

struct OccOffsets {
    uint64_t off[Grid::kZLevels + 1];
};
struct ZMapsK {
    int levels;
    uint32_t end[Grid::kZLevels + 1];       // exclusive end dword of map m (maps back to back)
    uint32_t dim[Grid::kZLevels + 1], rw[Grid::kZLevels + 1], occ_off[Grid::kZLevels + 1];
};

// Occupancy bytes of levels 2 .. 5 in one launch: a 256-thread workgroup owns a 16^3
// block of level-1 texels (one 16-byte row segment of b0's bytes per thread), reduces it to
// 8^3 / 4^3 / 2^3 / 1 texels of levels 2 / 3 / 4 / 5 through LDS bit rows and writes
// those levels' bytes (levels above `top` are skipped).  Needs n_1 >= 16.
__global__ void __launch_bounds__(256) k_occ_pyr(const uint8_t* __restrict__ b0, uint8_t* __restrict__ occ,
                                                 OccOffsets o, uint32_t n1, int top) {
    __shared__ uint32_t rows[256];                 // bit rows of the current level, [z][y]
    const uint32_t t = threadIdx.x;
    const uint32_t nb = n1 / 16u, b = blockIdx.x;
    const uint32_t X0 = (b % nb) * 16u, Y0 = ((b / nb) % nb) * 16u, Z0 = (b / (nb * nb)) * 16u;
    {
        const uint32_t y = t & 15u, z = t >> 4;
        const uint4 v = *reinterpret_cast<const uint4*>(b0 + ((size_t)(Z0 + z) * n1 + (Y0 + y)) * n1 + X0);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        uint32_t m = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) m |= ((w[i >> 2] >> (8 * (i & 3))) & 0xffu) ? 1u << i : 0u;
        rows[t] = m;
    }
    __syncthreads();
    // level m (edge e = 16 >> (m - 1) texels of the block): row (y, z) = OR of the four
    // level-(m-1) rows (2y .. 2y+1, 2z .. 2z+1), x pairs merged
    uint32_t e_in = 16u;
    for (int m = 2; m <= 5; ++m) {
        const uint32_t e = e_in >> 1;
        uint32_t r = 0;
        const bool mine = t < e * e;
        if (mine) {
            const uint32_t y = t % e, z = t / e;
            const uint32_t in = rows[(2u * z) * e_in + 2u * y] | rows[(2u * z) * e_in + 2u * y + 1u] |
                                rows[(2u * z + 1u) * e_in + 2u * y] | rows[(2u * z + 1u) * e_in + 2u * y + 1u];
            for (uint32_t x = 0; x < e; ++x) r |= ((in >> (2u * x)) & 3u) ? 1u << x : 0u;
            if (m <= top) {
                const uint32_t nm = n1 >> (m - 1);
                uint8_t* dst = occ + o.off[m] + ((size_t)((Z0 >> (m - 1)) + z) * nm + ((Y0 >> (m - 1)) + y)) * nm +
                               (X0 >> (m - 1));
                for (uint32_t x = 0; x < e; ++x) dst[x] = (uint8_t)((r >> x) & 1u);
            }
        }
        __syncthreads();
        if (mine) rows[t] = r;
        __syncthreads();
        e_in = e;
    }
}

// every map's dwords in one launch (k_zbits per dword, the map found from the offsets)
__global__ void __launch_bounds__(256) k_zbits_all(const uint8_t* __restrict__ b0, const uint8_t* __restrict__ occ,
                                                   ZMapsK z, uint32_t* __restrict__ dst) {
    const uint32_t wi = blockIdx.x * blockDim.x + threadIdx.x;
    int m = 1;
    while (m < z.levels && wi >= z.end[m]) ++m;
    if (wi >= z.end[m]) return;
    const uint32_t first = m == 1 ? 0u : z.end[m - 1];
    const uint8_t* bytes = m == 1 ? b0 : occ + z.occ_off[m];
    const uint32_t dim = z.dim[m], rw = z.rw[m], nm = dim - 1u, li = wi - first;
    const uint32_t wx = li % rw, py = (li / rw) % dim, pz = li / (rw * dim);
    dst[wi] = zbits_word(bytes, nm, wx, py, pz);
}

hipError_t launch_zmaps(vct_ctx* c, hipStream_t st) {
    Grid& g = c->grid;
    const uint32_t n1 = g.n >> 1;
    if (n1 >= 16) {
        OccOffsets o{};
        for (int m = 2; m <= Grid::kZLevels; ++m) o.off[m] = g.occ_off[m];
        const uint32_t nb = n1 / 16u;
        hipLaunchKernelGGL(k_occ_pyr, dim3(nb * nb * nb), dim3(256), 0, st, (const uint8_t*)g.b0, g.occ, o, n1,
                           g.zm_levels);
        ZMapsK z{};
        z.levels = g.zm_levels;
        uint32_t end = 0;
        for (int m = 1; m <= g.zm_levels; ++m) {
            end += g.zm_dim[m] * g.zm_dim[m] * g.zm_rw[m];
            z.end[m] = end;
            z.dim[m] = g.zm_dim[m];
            z.rw[m] = g.zm_rw[m];
            z.occ_off[m] = (uint32_t)g.occ_off[m];
        }
        hipLaunchKernelGGL(k_zbits_all, dim3((end + 255) / 256), dim3(256), 0, st, (const uint8_t*)g.b0,
                           (const uint8_t*)g.occ, z, g.zmap);
        return hipGetLastError();
    }
    for (int m = 2; m <= g.zm_levels; ++m) {
        const uint32_t nm = g.n >> m;
        const size_t cnt = (size_t)nm * nm * nm;
        hipLaunchKernelGGL(k_occ_down, dim3((uint32_t)((cnt + 255) / 256)), dim3(256), 0, st,
                           m == 2 ? (const uint8_t*)g.b0 : nullptr, m == 2 ? nullptr : g.occ + g.occ_off[m - 1],
                           g.occ + g.occ_off[m], nm);
    }
    for (int m = 1; m <= g.zm_levels; ++m) {
        // level 1's occupancy bytes are b0 itself (byte v = the children of texel v)
        const size_t words = (size_t)g.zm_dim[m] * g.zm_dim[m] * g.zm_rw[m];
        hipLaunchKernelGGL(k_zbits, dim3((uint32_t)((words + 255) / 256)), dim3(256), 0, st,
                           m == 1 ? (const uint8_t*)g.b0 : g.occ + g.occ_off[m], g.n >> m, g.zmap + g.zm_off[m],
                           g.zm_dim[m], g.zm_rw[m]);
    }
    return hipGetLastError();
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

// Grid::k3_live for K3's first launch with blocks of 16 x 16 x 2 BZ level-0 voxels (n >= 16):
// one lane per occupied voxel of K1's list; then the list of the live blocks
__global__ void __launch_bounds__(256) k3_live_blocks(const uint32_t* __restrict__ list, const uint32_t* __restrict__ n_list,
                                                      uint32_t lgn, uint32_t zsh, uint8_t* __restrict__ live) {
    const uint32_t cnt = *n_list, mask = (1u << lgn) - 1u, nbk = 1u << (lgn - 4u);
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < cnt; i += gridDim.x * 256u) {
        const uint32_t v = list[i];
        const uint32_t x = v & mask, y = (v >> lgn) & mask, z = v >> (2u * lgn);
        live[(x >> 4) + nbk * ((y >> 4) + nbk * (z >> zsh))] = 1;
    }
}

__global__ void __launch_bounds__(256) k3_live_compact(const uint8_t* __restrict__ live, uint32_t nblocks,
                                                       uint32_t* __restrict__ out, uint32_t* __restrict__ count) {
    const uint32_t b = blockIdx.x * 256u + threadIdx.x;
    const bool on = b < nblocks && live[b] != 0;
    const unsigned long long m = __builtin_amdgcn_ballot_w64(on);
    uint32_t base = 0;
    if ((threadIdx.x & 63u) == 0u && m) base = atomicAdd(count, (uint32_t)__popcll(m));
    base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
    if (on) out[base + (uint32_t)__popcll(m & ((1ull << (threadIdx.x & 63u)) - 1ull))] = b;
}

// K3's block depth: 8 x 8 x 4 parents (256 threads, 36 KB of LDS, subtrees three levels
// deep) beat the 8^3 cube (512 threads, 72 KB, four levels) by 4 % at 256^3 and 9 % at
// 512^3, and 8 x 8 x 2 by 3-4 %: twice the workgroups in flight per CU hide the staging
// loads better than the one saved launch (relight builds too: tools/k3_shapes.sh).
// VCT_K3_BZ = 8 | 2 selects the others (A/B).
// The K3 A/B switches (VCT_K3_BZ, VCT_K3_PLAN, VCT_K3_WRITE, VCT_K3_SPARSE, VCT_ZMAP) are
// all read per call, so a process can flip one between builds and see exactly that one
// change (a getenv per build is nothing beside the build).  They interact in one place:
// VCT_ZMAP=0 leaves the K4 maps invalid, and a relight-sparse build needs the maps of the
// previous build, so it also turns the sparse builds off.
static int env_int(const char* name, int dflt) {
    const char* v = getenv(name);
    return v ? atoi(v) : dflt;
}
static bool env_off(const char* name) {
    const char* v = getenv(name);
    return v && strcmp(v, "0") == 0;
}

static int k3_block_depth() {
    const int b = env_int("VCT_K3_BZ", 4);
    return b == 8 || b == 2 ? b : 4;
}

hipError_t launch_k3_live(vct_ctx* c) {
    Grid& g = c->grid;
    g.k3_live_count = 0;
    if (g.n < 16) return hipSuccess;
    const int bz = k3_block_depth();
    const uint32_t lgn = (uint32_t)__builtin_ctz(g.n), zsh = (uint32_t)__builtin_ctz(2 * bz);
    const uint32_t nblocks = (g.n >> 4) * (g.n >> 4) * (g.n >> zsh);
    uint32_t* cnt = g.k3_live_list + (g.n / 16u) * (g.n / 16u) * (g.n / 4u);   // past the largest list
    hipError_t e = hipMemsetAsync(g.k3_live, 0, nblocks, c->stream);
    if (e == hipSuccess) e = hipMemsetAsync(cnt, 0, sizeof(uint32_t), c->stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k3_live_blocks, dim3(1024), dim3(256), 0, c->stream, (const uint32_t*)g.occ_list,
                       (const uint32_t*)g.occ_count, lgn, zsh, g.k3_live);
    hipLaunchKernelGGL(k3_live_compact, dim3((nblocks + 255) / 256), dim3(256), 0, c->stream,
                       (const uint8_t*)g.k3_live, nblocks, g.k3_live_list, cnt);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    e = hipMemcpyAsync(&g.k3_live_count, cnt, sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream);
    g.k3_live_bz = bz;
    return e;
}

hipError_t launch_mips(vct_ctx* c) {
    Grid& g = c->grid;
    const bool zm_was_valid = g.zm_valid;
    g.zm_valid = false;
    const char* plan = getenv("VCT_K3_PLAN");   // A/B switches: read per call (k3_block_depth)
    const bool zmap_on = !env_off("VCT_ZMAP");
    if (plan && strcmp(plan, "level") == 0) {                            // A/B: one lane-per-parent launch per level (no K4 maps)
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
    BlockK k;
    k.pyr = g.pyr;
    for (int i = 0; i <= kMaxLevels; ++i) k.off[i] = g.lvl_off[i];
    k.n = (int)g.n;
    // level l of a full 8^3 block goes out in brick order from LDS: whole 512-B runs per
    // wave instead of 64-B half bricks (256^3: 0.126 -> 0.122 ms, 512^3: 0.890 -> 0.857 ms);
    // VCT_K3_WRITE=0 writes each parent from its thread (A/B)
    k.brick_writes = env_int("VCT_K3_WRITE", 1);
    k.b0 = nullptr;
    const int bz = k3_block_depth();
    // Relight build (Grid::k3_live): level 0 from K2 (not a dense write) and the last build
    // was one too, for this occupancy -- the non-live blocks of the first launch and the K4
    // maps (built from the same nonzero pattern) are skipped.  VCT_K3_SPARSE=0: A/B without.
    const bool sparse_on = !env_off("VCT_K3_SPARSE");
    const bool k2_level0 = !g.l0_dense;
    const bool sparse = sparse_on && k2_level0 && g.k3_sparse_ok && g.k3_live_bz == bz && g.n >= 16 && zm_was_valid;
    bool built = false;
    for (uint32_t l = 1; l <= g.L;) {
        const uint32_t nl = g.n >> l, E = nl < (uint32_t)kBlk ? nl : (uint32_t)kBlk;
        const uint32_t Ez = nl < (uint32_t)bz ? nl : (uint32_t)bz;
        const uint32_t nbk = nl / E, all = nbk * nbk * (nl / Ez);
        k.l = (int)l;
        k.b0 = (l == 1 && g.zm_levels > 0) ? g.b0 : nullptr;   // the launch that reads level 0
        k.live = (l == 1 && sparse) ? g.k3_live_list : nullptr;
        const uint32_t blocks = k.live ? g.k3_live_count : all;
#define VCT_K3_LAUNCH(BZv)                                                                                      \
    do {                                                                                                        \
        if (blocks == 0) break;                                                                                 \
        constexpr uint32_t thr = (uint32_t)(kBlk * kBlk * BZv);                                                \
        if (!g.aniso) hipLaunchKernelGGL((k3_block<kBox, BZv>), dim3(blocks), dim3(thr), 0, c->stream, k);     \
        else if (l == 1) hipLaunchKernelGGL((k3_block<kIso6, BZv>), dim3(blocks), dim3(thr), 0, c->stream, k); \
        else hipLaunchKernelGGL((k3_block<kFace, BZv>), dim3(blocks, 6), dim3(thr), 0, c->stream, k);          \
    } while (0)
        if (bz == 8) VCT_K3_LAUNCH(8);
        else if (bz == 2) VCT_K3_LAUNCH(2);
        else VCT_K3_LAUNCH(4);
#undef VCT_K3_LAUNCH
        if (k.b0 && !built && !sparse) {
            // level 0's bits are written: the K4 maps (in order on the ctx stream; forked onto a
            // side stream beside K3's top levels it measured slower at 256^3, 0.130 -> 0.139 ms)
            const hipError_t e = launch_zmaps(c, c->stream);
            if (e != hipSuccess) return e;
            built = true;
        }
        l += (uint32_t)__builtin_ctz(Ez) + 1u;
    }
    if (built) {
        g.zm_valid = zmap_on;                  // VCT_ZMAP=0: A/B without (and without sparse builds)
    }
    if (sparse) g.zm_valid = true;            // same level-0 pattern as when they were built
    g.k3_sparse_ok = k2_level0;
    return hipGetLastError();
}

hipError_t launch_relayout(vct_ctx* c, const float4* src, float4* dst, uint32_t nl, bool to_linear) {
    const size_t vl = (size_t)nl * nl * nl;
    hipLaunchKernelGGL(k_relayout, dim3((uint32_t)((vl + 255) / 256)), dim3(256), 0, c->stream, src, dst, nl,
                       to_linear ? 1 : 0);
    return hipGetLastError();
}

}  // namespace vct
