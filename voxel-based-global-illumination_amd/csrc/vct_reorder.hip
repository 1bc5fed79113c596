// vct_reorder.hip — ray reordering for incoherent G-buffers (vct_trace_args.variant 0x8000).
//
// K4 packs an 8x8 pixel block into one wave and stages the 4^3 texel brick that holds
// every lane's footprint in LDS.  That pays when neighbouring pixels are neighbouring
// surface points (a rasterised G-buffer, G_scene).  When they are not (G_rand: every
// pixel an independent random surface point and normal; or any stochastic
// G-buffer), a wave's 64 cones start all over the grid, no brick fits, and the trace
// turns into per-lane gathers that miss L2 (HBM-bound at ~91 % of peak with a 2.3x
// line overfetch).
//
// Reordering: the frame's pixels are grouped by the cell that holds their cone origin
// o = (P - g0) / h + n (the same binary32 sequence as K4), cells in Morton order,
// background pixels after every valid one; K4 then reads lane j of wave w from pixel
// perm[64 w + j] and writes its outputs back to that pixel.  Cones of one wave start in
// a few neighbouring cells, so their footprints share bricks and cache lines.  Every
// pixel runs exactly the arithmetic it runs without the reordering, so outputs and step
// counts are bit-identical whatever the order inside a cell (tested).
//
// Two keys (round 5), one permutation each when the launch traces the specular cone in
// its own part (the parts write different outputs, so each may order the pixels its own
// way):
//   diffuse  sign(n.z) -- the branch of the Duff et al. tangent basis: pixels on either
//            side of it get the ring cones rotated against each other, so a wave mixing them
//            selects five or six faces and gathers -- then the level-lk cell.  Sign major:
//            every wave but the one at the boundary has one sign (G_rand 5.40 -> 4.74 ms
//            against cell major, where each cell's two signs alternate within a wave; the
//            octant major over 8x coarser cells 4.79, sign major over them 4.85);
//   specular the cone's aperture tau = clamp(roughness) in quarter octaves, then a cell 64x
//            coarser than the diffuse one: the pixels of one aperture class are contiguous, so
//            a wave's lanes share one tau (one step table, wave-uniform levels) and lie in
//            Morton-adjacent cells.  A specular cone's mip level is log2(2 tau t): lanes whose tau
//            differ by more than a fraction of an octave disagree on the level at most
//            steps, and such a step is gathered per lane at per-lane levels (64-bit
//            addresses, both levels one after the other).
//
// The grouping is a counting sort, hand-written for the job (round 5; it replaced a
// rocPRIM radix sort of (Morton code, pixel) pairs, four one-sweep passes):
//   k_reorder_count    per pixel its cell (Morton code at level lk: at most 2^21 cells,
//                      level 0 up to 128^3, level 1 at 256^3, level 2 at 512^3) and
//                      its rank in that cell from an atomic on the cell's counter (the
//                      background's counter is bumped once per wave: ballot + mbcnt);
//   k_scan_reduce /    exclusive scan of the counters into cell offsets: tile sums of
//   k_scan_tiles /     4096 counters, a one-block scan of the tile sums, the tiles'
//   k_scan_down        own scans with their carries (in place);
//   k_reorder_scatter  perm[offset(cell) + rank] = pixel.
// One pass over the pixels, two over the counters (8 MB at most), one scatter: no key
// bits are sorted twice.  The order inside a cell follows the atomics (it only moves
// pixels between the waves of that cell, never their results).
#include "vct_internal.h"

namespace vct {
namespace {

// key kinds: cell bits and class bits (at most 2^22 counters = 16 MB)
enum { kKeyDiffuse = 0, kKeySpecular = 1 };
// the diffuse key (A/B): 0 = the cell, then sign(n.z); 1 = sign(n.z), then the cell (default);
// 2 = the normal's octant (signs of x, y, z), then the cell
#ifndef VCT_DIFF_KEY_MODE
#define VCT_DIFF_KEY_MODE 1
#endif
// the specular key's normal bits between the aperture class and the cell (A/B): 0 (default),
// 1 = sign(n.z), 3 = the octant (G_rand 4.74 / 5.09 / 5.85 ms, the latter two over 15-bit cells)
// aperture classes per octave: 2^(VCT_SPEC_TAU_BITS - 3): quarter octaves (G_rand ms under
// super-cells: half octaves over 18-bit cells 4.62-4.64, quarter / eighth octaves over 15-bit
// cells 4.56-4.59 / 4.57, octaves over 18-bit cells 4.77)
#ifndef VCT_SPEC_TAU_BITS
#define VCT_SPEC_TAU_BITS 5
#endif
#ifndef VCT_SPEC_NRM_BITS
#define VCT_SPEC_NRM_BITS 0
#endif
template <int KIND> constexpr uint32_t key_class_bits() {
    return KIND == kKeyDiffuse ? (VCT_DIFF_KEY_MODE == 2 ? 3u : 1u) : (uint32_t)VCT_SPEC_TAU_BITS + VCT_SPEC_NRM_BITS;
}
#ifndef VCT_KEY_DIFF_BITS
#define VCT_KEY_DIFF_BITS 21
#endif
// the specular key: aperture class major, then the level-lk cell (A/B switches; G_rand, ms per
// frame, DESIGN 13.4: cell-major with 18 / 15 / 12 / 9 cell bits 6.46 / 5.96 / 6.08 / 6.91,
// aperture-major with 15 / 18 cell bits 5.54 / 5.42 against cell-major 15 bits 5.54-5.59)
// super-cells of the class-major keys: the top 9 Morton bits (8^3 super-cells) above the class
// (G_rand ms: class fully major 4.74, 3 / 6 / 9 / 12 / 15 bits 4.78-4.80 / 4.83 / 4.62-4.64 /
// 4.70 / 5.0-5.2)
#ifndef VCT_KEY_SUPER_BITS
#define VCT_KEY_SUPER_BITS 9
#endif
#ifndef VCT_SPEC_TAU_MAJOR
#define VCT_SPEC_TAU_MAJOR 1
#endif
#ifndef VCT_KEY_SPEC_BITS
#define VCT_KEY_SPEC_BITS 15
#endif
template <int KIND> constexpr uint32_t key_cell_bits() { return KIND == kKeyDiffuse ? VCT_KEY_DIFF_BITS : VCT_KEY_SPEC_BITS; }
constexpr int kScanPer = 16;                // counters per thread in the scan kernels
constexpr uint32_t kScanTile = 256u * kScanPer;

__device__ __forceinline__ uint32_t spread3(uint32_t v) {   // 10 bits -> every third bit
    v &= 0x3ffu;
    v = (v | (v << 16)) & 0x030000ffu;
    v = (v | (v << 8)) & 0x0300f00fu;
    v = (v | (v << 4)) & 0x030c30c3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}

__device__ __forceinline__ uint32_t lanes_below(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// exclusive prefix sum of one value per thread over a 256-thread block, and the block total
__device__ __forceinline__ uint32_t block_scan256(uint32_t v, uint32_t& total) {
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

// aperture class of a specular cone: tau = clamp(roughness, VCT_SPEC_TAU_MIN, VCT_SPEC_TAU_MAX)
// (as K4 computes it) in 2^(VCT_SPEC_TAU_BITS - 3) classes per octave (quarter octaves by
// default), from its exponent and top mantissa bits
__device__ __forceinline__ uint32_t tau_class(float rough) {
    const float tau = fminf(fmaxf(rough, VCT_SPEC_TAU_MIN), VCT_SPEC_TAU_MAX);
    const int ex = (int)((__float_as_uint(tau) >> 23) & 0xffu) - 127;   // -6 .. 0
    constexpr int sub = VCT_SPEC_TAU_BITS - 3;                          // mantissa bits per octave
    const int hc = (ex + 7) * (1 << sub) + (int)((__float_as_uint(tau) >> (23 - sub)) & ((1u << sub) - 1u));
    return (uint32_t)min(max(hc, 0), (1 << VCT_SPEC_TAU_BITS) - 1);
}

// key of each pixel (cell of its cone origin: level-lk voxels in Morton order, then the
// kind's class bits; background = key ncell) and its rank among the pixels of that key
template <int KIND>
__global__ void __launch_bounds__(256) k_reorder_count(const float4* __restrict__ pos, const float4* __restrict__ nrm,
                                                       const float4* __restrict__ alb, uint32_t npx, float g0x,
                                                       float g0y, float g0z, float inv_h, int n, int lk, uint32_t ncell,
                                                       uint32_t* __restrict__ cnt, uint32_t* __restrict__ cell,
                                                       uint32_t* __restrict__ rank) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    const bool in = i < npx;
    float4 P = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (in) P = pos[i];
    const bool bg = in && P.w == 0.0f;
    uint32_t c = ncell, r = 0;
    if (in && !bg) {
        const float4 N = nrm[i];
        const float ox = (P.x - g0x) * inv_h + N.x;   // the cone origin of K4 (level-0 voxel units)
        const float oy = (P.y - g0y) * inv_h + N.y;
        const float oz = (P.z - g0z) * inv_h + N.z;
        const auto q = [n, lk](float v) {
            const float f = floorf(v);
            return (uint32_t)(f < 0.0f ? 0 : (f > (float)(n - 1) ? n - 1 : (int)f)) >> lk;
        };
        c = spread3(q(ox)) | (spread3(q(oy)) << 1) | (spread3(q(oz)) << 2);
        const uint32_t cbits = 3u * (uint32_t)(__builtin_ctz((uint32_t)n) - lk);
        // class-major keys can keep the top VCT_KEY_SUPER_BITS Morton bits above the class
        // (super-cells: each class is swept once per super-cell instead of once per grid)
        const uint32_t lo = cbits > (uint32_t)VCT_KEY_SUPER_BITS ? cbits - (uint32_t)VCT_KEY_SUPER_BITS : 0u;
        const auto cls = [c, lo](uint32_t k, uint32_t kb) {
            return ((c >> lo) << (lo + kb)) | (k << lo) | (c & ((1u << lo) - 1u));
        };
        if (KIND == kKeyDiffuse) {
            if (VCT_DIFF_KEY_MODE == 0) c = (c << 1) | (N.z < 0.0f ? 1u : 0u);
            else if (VCT_DIFF_KEY_MODE == 1) c = cls(N.z < 0.0f ? 1u : 0u, 1u);
            else c = cls((N.x < 0.0f ? 1u : 0u) | (N.y < 0.0f ? 2u : 0u) | (N.z < 0.0f ? 4u : 0u), 3u);
        }
        else if (VCT_SPEC_TAU_MAJOR) {
            const uint32_t oct = (N.x < 0.0f ? 1u : 0u) | (N.y < 0.0f ? 2u : 0u) | (N.z < 0.0f ? 4u : 0u);
            const uint32_t nb = VCT_SPEC_NRM_BITS == 3 ? oct : (VCT_SPEC_NRM_BITS == 1 ? oct >> 2 : 0u);
            c = cls((tau_class(alb[i].w) << VCT_SPEC_NRM_BITS) | nb, (uint32_t)VCT_SPEC_TAU_BITS + VCT_SPEC_NRM_BITS);
        }
        else c = (c << VCT_SPEC_TAU_BITS) | tau_class(alb[i].w);
        r = atomicAdd(cnt + c, 1u);
    }
    // the background shares one counter: one atomic per wave
    const unsigned long long bm = __builtin_amdgcn_ballot_w64(bg);
    if (bm) {
        const int lead = __builtin_ctzll(bm);
        uint32_t base = 0;
        if ((int)(threadIdx.x & 63) == lead) base = atomicAdd(cnt + ncell, (uint32_t)__builtin_popcountll(bm));
        base = (uint32_t)__builtin_amdgcn_readlane((int)base, lead);
        if (bg) r = base + lanes_below(bm);
    }
    if (in) {
        cell[i] = c;
        rank[i] = r;
    }
}

// counters [t * kScanTile, (t + 1) * kScanTile) -> tile sum t
__global__ void __launch_bounds__(256) k_scan_reduce(const uint32_t* __restrict__ cnt, uint32_t m,
                                                     uint32_t* __restrict__ tiles) {
    const uint32_t base = blockIdx.x * kScanTile + threadIdx.x * kScanPer;
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < kScanPer; ++j) s += base + j < m ? cnt[base + j] : 0u;
    uint32_t total;
    (void)block_scan256(s, total);
    if (threadIdx.x == 0) tiles[blockIdx.x] = total;
}

// exclusive scan of the tile sums in one block (counters <= 2^22 + 1, so ntiles <= 2^22 / 4096
// + 1 = 1025: five rounds of 256)
__global__ void __launch_bounds__(256) k_scan_tiles(uint32_t* __restrict__ tiles, uint32_t ntiles) {
    uint32_t carry = 0;
    for (uint32_t b = 0; b < ntiles; b += 256) {
        const uint32_t i = b + threadIdx.x;
        const uint32_t v = i < ntiles ? tiles[i] : 0u;
        uint32_t total;
        const uint32_t ex = block_scan256(v, total);
        if (i < ntiles) tiles[i] = carry + ex;
        carry += total;
    }
}

// in place: counter -> offset of its cell (tile carry + scan inside the tile)
__global__ void __launch_bounds__(256) k_scan_down(uint32_t* __restrict__ cnt, uint32_t m,
                                                   const uint32_t* __restrict__ tiles) {
    const uint32_t base = blockIdx.x * kScanTile + threadIdx.x * kScanPer;
    uint32_t v[kScanPer], s = 0;
#pragma unroll
    for (int j = 0; j < kScanPer; ++j) {
        v[j] = base + j < m ? cnt[base + j] : 0u;
        s += v[j];
    }
    uint32_t total;
    uint32_t run = tiles[blockIdx.x] + block_scan256(s, total);
#pragma unroll
    for (int j = 0; j < kScanPer; ++j) {
        if (base + j < m) cnt[base + j] = run;
        run += v[j];
    }
}

__global__ void __launch_bounds__(256) k_reorder_scatter(const uint32_t* __restrict__ cell,
                                                         const uint32_t* __restrict__ rank,
                                                         const uint32_t* __restrict__ offs, uint32_t npx,
                                                         uint32_t* __restrict__ perm) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < npx) perm[offs[cell[i]] + rank[i]] = i;
}

}  // namespace

// one counting sort of the frame's pixels by key kind KIND into out (npx entries)
template <int KIND>
static hipError_t sort_pixels(vct_ctx* c, const vct_trace_args* a, uint32_t* kv, uint32_t* cnt, uint32_t* out) {
    const Grid& g = c->grid;
    const uint32_t npx = a->width * a->height;
    const uint32_t lgn = (uint32_t)__builtin_ctz(g.n);
    static_assert(key_cell_bits<KIND>() + key_class_bits<KIND>() <= 22u, "counters: at most 2^22 + 1 (launch_reorder)");
    const uint32_t cb = key_cell_bits<KIND>();
    const uint32_t lk = 3u * lgn > cb ? (3u * lgn - cb + 2u) / 3u : 0u;   // cells: level-lk voxels
    const uint32_t ncell = 1u << (3u * (lgn - lk) + key_class_bits<KIND>());
    const uint32_t m = ncell + 1u;                          // + the background's counter
    const uint32_t ntiles = (m + kScanTile - 1u) / kScanTile;
    uint32_t* cell = kv;
    uint32_t* rank = kv + npx;
    uint32_t* tiles = cnt + m;
    hipStream_t s = c->stream;
    hipError_t e;
    if ((e = hipMemsetAsync(cnt, 0, (size_t)m * sizeof(uint32_t), s)) != hipSuccess) return e;
    const uint32_t pblocks = (npx + 255u) / 256u;
    hipLaunchKernelGGL(k_reorder_count<KIND>, dim3(pblocks), dim3(256), 0, s, (const float4*)a->pos4,
                       (const float4*)a->nrm4, (const float4*)a->alb4, npx, g.g0[0], g.g0[1], g.g0[2], g.inv_h,
                       (int)g.n, (int)lk, ncell, cnt, cell, rank);
    hipLaunchKernelGGL(k_scan_reduce, dim3(ntiles), dim3(256), 0, s, (const uint32_t*)cnt, m, tiles);
    hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(256), 0, s, tiles, ntiles);
    hipLaunchKernelGGL(k_scan_down, dim3(ntiles), dim3(256), 0, s, cnt, m, (const uint32_t*)tiles);
    hipLaunchKernelGGL(k_reorder_scatter, dim3(pblocks), dim3(256), 0, s, (const uint32_t*)cell,
                       (const uint32_t*)rank, (const uint32_t*)cnt, npx, out);
    return hipGetLastError();
}

hipError_t launch_reorder(vct_ctx* c, const vct_trace_args* a, const uint32_t** perm, const uint32_t** perm_spec) {
    const uint32_t npx = a->width * a->height;
    // counters: at most 2^22 + 1, plus the tile sums
    const size_t mmax = (size_t)(1u << 22) + 1u, tmax = (mmax + kScanTile - 1u) / kScanTile;
    void* kv = nullptr;   // [cell | rank | perm | perm_spec] per pixel
    void* sp = nullptr;   // [counters | tile sums]
    hipError_t e;
    if ((e = k4_scratch(c, kScKeys, (size_t)4 * npx * sizeof(uint32_t), &kv, nullptr)) != hipSuccess) return e;
    if ((e = k4_scratch(c, kScSort, (mmax + tmax) * sizeof(uint32_t), &sp, nullptr)) != hipSuccess) return e;
    uint32_t* base = (uint32_t*)kv;
    if ((e = sort_pixels<kKeyDiffuse>(c, a, base, (uint32_t*)sp, base + 2 * (size_t)npx)) != hipSuccess) return e;
    *perm = base + 2 * (size_t)npx;
    if (perm_spec) {
        if ((e = sort_pixels<kKeySpecular>(c, a, base, (uint32_t*)sp, base + 3 * (size_t)npx)) != hipSuccess) return e;
        *perm_spec = base + 3 * (size_t)npx;
    }
    return hipSuccess;
}

}  // namespace vct
