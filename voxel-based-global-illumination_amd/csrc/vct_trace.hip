// vct_trace.hip — K4: per-pixel diffuse + specular cone trace (the metric kernel).
//
// SURVEY.md Appendix A.5 / A.6 with the literals of include/vct_spec.h.  The
// reference has no cone tracer: its only GPU program is the forward textured
// draw of assets/code/shader/test.{vert,frag}, issued by
// VoxelizationRenderer::Render (assets/code/renderer/r_voxelization.cpp:4-35).
//
// MI355X design (memory-gather bound, no MFMA):
//  * one lane = one pixel; a 64-lane wave (one workgroup) is an 8x8 pixel
//    block.  The screen is cut into 64x64 tiles; tile t belongs to rank
//    t % world.  Inside a rank the workgroup -> tile map is
//    XCD-aware: whole tiles are dealt to the eight round-robin XCD groups,
//    so the waves of a tile (which read the same bricks) share an L2.
//  * The lanes of a wave march the same cone index in lock step.  Diffuse
//    cones have a wave-uniform step sequence (t, D and the mip pair depend only
//    on tau), the per-lane early-out (a >= 0.95 / left the grid) just masks the
//    lane, and the wave leaves the loop on a ballot.
//  * Default variant (0): at each step and mip level the wave stages the 4^3
//    texel brick that contains every active lane's 2x2x2 footprint (origin =
//    per-axis minimum corner, a wave reduction; fit checked with one ballot)
//    in a wave-private LDS slot -- one texel per lane, one coalesced 16-B load
//    per face -- and the lanes read their 8 corners with ds_read_b128 at
//    immediate offsets (+16 B dx, +64 B dy, +256 B dz).  When the cone
//    direction is the same for every lane (flat surfaces), the staging lanes
//    also combine the three anisotropic faces of each texel (the spec combines
//    per corner texel), so the lanes read ONE slot instead of three.  Texels
//    outside the level are staged as zero = the spec's zero border.  Waves
//    whose footprint does not fit fall back to per-lane gathers for that step.
//  * Variant 1: per-lane gathers only (global_load_dwordx4, zero border via
//    zeroed weights on clamped addresses).
//  Both variants read the same texels and run the spec's operation order
//  (-ffp-contract=off, explicit fmaf), so they are bit-identical to each other
//  and to the CPU oracle.
#include <climits>

#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "vct_internal.h"

// Debug-build counters (make dbg -> vct/libvct_hip_dbg.so, tools/dbg_counters.py):
// per wave and level sample, which path served it.  Compiled out of the product.
#if defined(VCT_DEBUG_COUNTERS) || defined(VCT_DEBUG_CLOCK)
__device__ unsigned long long vct_dbg_ctr[48];
__device__ unsigned long long vct_dbg_time[8];
#endif
#if defined(VCT_DEBUG_CLOCK) || defined(VCT_DEBUG_WAVES)
// per-wave (start, end) of the real-time counter (100 MHz, chip-wide), indexed by
// blockIdx * waves-per-block + wave; tools/wave_sched.py replays schedules from it
constexpr int kDbgWaves = 1 << 18;
__device__ unsigned long long vct_dbg_wave[kDbgWaves][3];   // start, end, HW_ID | XCC_ID << 32
#endif
#ifdef VCT_DEBUG_COUNTERS
#define VCT_DBG(i) do { if ((threadIdx.x & 63) == 0) atomicAdd(&vct_dbg_ctr[i], 1ull); } while (0)
#define VCT_DBGN(i, v) do { if ((threadIdx.x & 63) == 0) atomicAdd(&vct_dbg_ctr[i], (unsigned long long)(v)); } while (0)
#else
#define VCT_DBG(i) do { } while (0)
#define VCT_DBGN(i, v) do { } while (0)
#endif

// Clock-build (make clk -> vct/libvct_hip_clk.so) per-wave phase clock
// (s_memtime cycles), summed over waves: 0 step head, 1 brick geometry,
// 2 staging (loads -> LDS), 3 LDS sampling, 4 per-lane fallback gathers,
// 5 step tail, 6 kernel total.  Kept apart from the counters, whose global
// atomics would land in the memory waits being timed.
struct PhaseClock {
#ifdef VCT_DEBUG_CLOCK
    unsigned long long acc[7] = {}, last = 0, first = 0;
    unsigned nsteps = 0;
    __device__ void start() { first = last = __builtin_amdgcn_s_memtime(); }
    __device__ void mark(int i) {
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        acc[i] += t - last;
        last = t;
        nsteps += i == 0;
    }
    __device__ void flush() {
        acc[6] = __builtin_amdgcn_s_memtime() - first;
        if ((threadIdx.x & 63) == 0) {
            for (int i = 0; i < 7; ++i) atomicAdd(&vct_dbg_time[i], acc[i]);
            atomicMax(&vct_dbg_time[7], acc[6]);          // longest wave
            const int lg = 63 - __builtin_clzll(acc[6] | 1);   // wave-duration histogram, 2^(10+k) cycles
            atomicAdd(&vct_dbg_ctr[lg < 10 ? 0 : (lg > 31 ? 21 : lg - 10)], 1ull);
            if (lg >= 20) {                                     // phase split of the long waves
                for (int i = 0; i < 7; ++i) atomicAdd(&vct_dbg_ctr[24 + i], acc[i]);
                atomicAdd(&vct_dbg_ctr[22], 1ull);
                atomicAdd(&vct_dbg_ctr[23], (unsigned long long)nsteps);
            } else if (lg >= 18) {
                atomicAdd(&vct_dbg_ctr[31], (unsigned long long)nsteps);
            }
        }
    }
#else
    __device__ void start() {}
    __device__ void mark(int) {}
    __device__ void flush() {}
#endif
};

extern "C" __device__ int __ockl_wfred_min_i32(int);   // wave-wide min over the active lanes

// c = q 2^-l - 1/2 as one fma: the product by a power of two is exact (no overflow,
// and an underflowed product is absorbed by the - 1/2), so the fused form rounds once
// where the spec rounds once: bit-identical
__device__ __forceinline__ float lvl_coord(float q, float scale) {
    return fmaf(q, scale, -0.5f);
}

// the occupancy form of the default cone trace: 96 VGPRs, 7008 B of LDS (no four-face
// union), 5 waves/SIMD; the union form runs kUnionWaves (K4Tuner picks per workload)
constexpr int kOccWaves = 5;   // 6 (80 VGPRs) spills 54-69 VGPRs
constexpr int kUnionWaves = 4;  // __launch_bounds__ minimum waves per SIMD (128 VGPRs, 9984 B of LDS)

namespace vct {
namespace {

#define VCT_CROW(cn, ct, cb, w) {cn, ct, cb, w},
__constant__ float c_cones1[1][4] = {VCT_CONES1(VCT_CROW)};
__constant__ float c_cones9[9][4] = {VCT_CONES9(VCT_CROW)};
__constant__ float c_cones16[16][4] = {VCT_CONES16(VCT_CROW)};

// level l's buffer range as the O32 kernels bind it (one 16-B scalar load per level view)
struct alignas(16) LevelRange {
    const float4* base;          // pyr + lvl_off[l]
    uint32_t bytes;              // the level's size (every face; num_records is unsigned), 0 above 32 bits
    uint32_t pad;
};

// one empty-space map of Grid::zmap (positions p in [-1, n_m - 1]^3 at p + 1, rows of rw dwords)
struct ZLevel {
    uint32_t off, dim, rw, pad;
};

struct TraceK {
    const float4* pyr;
    uint64_t lvl_off[kMaxLevels + 1];
    LevelRange lvl[kMaxLevels + 1];
    int n, L;
    int lgn;                     // log2 n
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
    int tiles_x, rank, world, compact;
    int nd, spec_on, aniso;
    float tau_d;
    const StepRow* steps_tab;    // diffuse-cone step table (tau_d), sentinel-terminated
    unsigned* spec_keys;         // [kSpecSlots] tau bit patterns of the specular step tables (~0u = free)
    unsigned* spec_state;        // [kSpecSlots] 0 building, 1 ready, 2 needs more than 64 rows
    StepRow* spec_rows;          // [kSpecSlots][64]
    int spec_tabs;               // 0: specular cones always derive their steps per lane (variant bit 0x100)
    int split;                   // 0: one workgroup per 16x16 block traces every cone; 1: two (diffuse | specular);
                                 // 2: ndp diffuse parts (cones [g * nd_chunk, ...)) | specular
    int nd_chunk;                // split 2: diffuse cones per part (part g: [g * nd_chunk, (g + 1) * nd_chunk) & nd)
    int ndp;                     // split 2: diffuse parts (>= 2), each followed in blockIdx order by the next
    int spec_first;              // split 2: the specular part comes first in blockIdx order (variant 0x2000)
    int xcd_g;                   // units per XCD chunk of the workgroup map (0 = one contiguous run per XCD)
    float4* sc_part;             // split 2: [px] diffuse sum after cones [0, nd_chunk)  (per output index)
    float4* sc_cone;             // split 2: [cone - nd_chunk][px] results of cones [nd_chunk, nd)
    size_t sc_px;                // pixels per scratch plane
    unsigned* sc_flag;           // split 2: [block][wave] hand-over counter (0 between launches)
    const uint32_t* perm;        // ray reordering (variant 0x8000): lane j of wave u traces pixel perm[64 u + j]
    const uint32_t* perm_spec;   // the specular part's order (null: perm)
    uint32_t npx;                // its length (w * h)
    const uint32_t* order;       // dispatch order: workgroup i traces unit order[i] (null: unit i)
    uint32_t* dur;               // per unit: its wave's duration in s_memrealtime ticks (null: not recorded)
    const uint32_t* zmap;        // Grid::zmap (empty-space maps 1..zm_levels; zm_levels = 0: no test)
    uint32_t zmap_bytes;
    int zm_levels;
    ZLevel zm[Grid::kZLevels + 1];
};

__device__ __forceinline__ const float (*cone_table(int nd))[4] {
    return nd == 16 ? c_cones16 : (nd == 9 ? c_cones9 : c_cones1);
}

// Wave votes on lane masks (SGPR pairs).  HIP's __any/__all/__ballot take an
// int and round-trip every predicate through a VGPR (v_cndmask + v_cmp); so
// does a ballot of an ANDed predicate.  Vote on the bare compare and AND the
// lane set in as a scalar mask: ballot(c) & m.
__device__ __forceinline__ unsigned long long wballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ bool wany(bool p) { return wballot(p) != 0ull; }
__device__ __forceinline__ bool wall(bool p) { return wballot(!p) == 0ull; }
// every lane of mask m satisfies c
__device__ __forceinline__ bool wall_in(unsigned long long m, bool c) { return (wballot(!c) & m) == 0ull; }

__device__ __forceinline__ float4 sel4(bool c, float4 a, float4 b) {   // a float4 `?:` lowers to scratch
    return make_float4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
}

__device__ __forceinline__ void acc_fma(float4& acc, float w, float4 v) {
    acc.x = fmaf(w, v.x, acc.x);
    acc.y = fmaf(w, v.y, acc.y);
    acc.z = fmaf(w, v.z, acc.z);
    acc.w = fmaf(w, v.w, acc.w);
}

// v = fmaf(wz, Z, fmaf(wy, Y, wx * X)): the spec's per-texel face combination
__device__ __forceinline__ float4 combine3(float wx, float wy, float wz, float4 X, float4 Y, float4 Z) {
    return make_float4(fmaf(wz, Z.x, fmaf(wy, Y.x, wx * X.x)), fmaf(wz, Z.y, fmaf(wy, Y.y, wx * X.y)),
                       fmaf(wz, Z.z, fmaf(wy, Y.z, wx * X.z)), fmaf(wz, Z.w, fmaf(wy, Y.w, wx * X.w)));
}

// corners whose three anisotropic faces are in registers at once (VGPR budget)
constexpr int kCh = 4;
// the occupancy form (5 waves/SIMD, 96 VGPRs) keeps 2 corners x 3 faces in flight
#ifndef VCT_K4_CHOCC
#define VCT_K4_CHOCC 2
#endif
constexpr int kChOcc = VCT_K4_CHOCC;
// the union form stages five-face cones too (4 x 4 x 3 bricks)
#ifndef VCT_K4_FIVE
#define VCT_K4_FIVE 1
#endif
// ... and six-face cones (4 x 4 x 3 bricks in the kBz6 layout, a march of their own)
#ifndef VCT_K4_SIX
#define VCT_K4_SIX 1
#endif
template <bool UNION> constexpr int gather_chunk() { return UNION ? kCh : kChOcc; }

// trilinear corner weights (x fastest), w_c = (wx * wy) * wz
__device__ __forceinline__ void corner_weights(float fx, float fy, float fz, float (&wc)[8]) {
    const float wx[2] = {1.0f - fx, fx}, wy[2] = {1.0f - fy, fy}, wz[2] = {1.0f - fz, fz};
#pragma unroll
    for (int c = 0; c < 8; ++c) wc[c] = (wx[c & 1] * wy[(c >> 1) & 1]) * wz[c >> 2];
}

// One level of the pyramid as the kernels read it.  O32 (every level below
// 2 GiB, n <= 512): a buffer resource over the level (wave-uniform, SGPRs),
// 32-bit byte offsets, and the spec's zero border from the hardware range
// check -- a texel outside the level is fetched at an out-of-range offset and
// reads as 0, so no select waits on the load.  Else: 64-bit addresses and an
// explicit select.
template <bool O32>
struct LevelView;

template <>
struct LevelView<true> {
    __amdgpu_buffer_rsrc_t r;
    __device__ float4 fetch(uint32_t i, bool in) const {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, in ? i << 4 : 0xfffffff0u, 0, 0);
        return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
    }
};

template <>
struct LevelView<false> {
    const float4* p;
    __device__ float4 fetch(uint32_t i, bool in) const {
        const float4 v = p[in ? i : 0u];
        return sel4(in, v, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    }
};

// level l (wave-uniform): O32 takes the level's base and size from the host's per-level
// table in the kernel arguments (launch_trace; one scalar load per level view, measured
// faster than deriving them on the scalar unit, which also held ~34 more SGPRs)
template <bool O32>
__device__ __forceinline__ LevelView<O32> level_view(const TraceK& k, int l) {
    if constexpr (O32) {
        const LevelRange r = k.lvl[l];
        return LevelView<true>{__builtin_amdgcn_make_buffer_rsrc((void*)r.base, (short)0, (int)r.bytes, 0x00020000)};
    } else {
        return LevelView<false>{k.pyr + k.lvl_off[l]};
    }
}

// level l differing per lane (per-pixel roughness): 64-bit per-lane base, so no
// buffer resource (a scalar operand) has to be built from a per-lane value
__device__ __forceinline__ LevelView<false> level_view_lane(const TraceK& k, int l) {
    const uint64_t n = (uint64_t)k.n, n3 = n * n * n, F = k.aniso ? 6u : 1u;
    const uint64_t m = n >> (l > 0 ? l - 1 : 0);
    const uint64_t off = l == 0 ? 0u : n3 + F * ((n3 - m * m * m) / 7u);
    return LevelView<false>{k.pyr + off};
}

// ===========================================================================
// per-lane gathers (variant 1, and the fallback of variant 0)
// ===========================================================================
// Brick layout byte offsets as OR-able bit fields (n a power of two): inside a face
// volume of nl^3 texels, coordinate x contributes (x >> 1) << 7 | (x & 1) << 4, y
// (y >> 1) << (lnb + 7) | (y & 1) << 5 and z (z >> 1) << (2 lnb + 7) | (z & 1) << 6
// (nb = nl / 2 = 2^lnb bricks per axis); face f adds f << (3 lg nl + 4).  The fields
// are disjoint, so a texel's byte offset is the OR of its three axis terms (and its
// face), and an axis term of kOut = 0xfffffff0 for a coordinate outside the level
// makes the OR kOut: past the buffer resource's range, which reads as 0 (the spec's
// zero border).  One v_or3 per corner instead of adds, range checks and selects.
constexpr uint32_t kOut = 0xfffffff0u;
struct AxisTerms { uint32_t t0, t1; };     // coordinates c and c + 1
__device__ __forceinline__ AxisTerms axis_terms(int c, uint32_t nl, uint32_t sh, uint32_t bit) {
    const uint32_t u = (uint32_t)c, odd = u & 1u;
    const uint32_t t0 = ((u >> 1) << sh) | (odd << bit);
    // c + 1: the same 2-brick when c is even (+ 1 << bit), else the next one (wraps to 0 for c = -1)
    const uint32_t t1 = odd ? t0 + ((1u << sh) - (1u << bit)) : t0 + (1u << bit);
    return AxisTerms{u < nl ? t0 : kOut, u + 1u < nl ? t1 : kOut};
}

struct LevelBits { uint32_t nl, shy, shz, shf; };   // per level l (wave-uniform)
__device__ __forceinline__ LevelBits level_bits(const TraceK& k, int l) {
    const uint32_t lg = (uint32_t)(k.lgn - l), lnb = lg > 0u ? lg - 1u : 0u;
    return LevelBits{1u << lg, lnb + 7u, 2u * lnb + 7u, 3u * lg + 4u};
}

// D_l for a wave-uniform level through its buffer resource (O32, brick layout):
// same texels, weights and fmaf order as sample_level
template <int KC>
__device__ __forceinline__ float4 sample_level_bits(const TraceK& k, int l, float qx, float qy, float qz, int fx,
                                                    int fy, int fz, float wdx, float wdy, float wdz) {
    const float scale = __uint_as_float((uint32_t)(127 - l) << 23);  // 2^-l, exact
    const float cx = lvl_coord(qx, scale), cy = lvl_coord(qy, scale), cz = lvl_coord(qz, scale);
    const float flx = floorf(cx), fly = floorf(cy), flz = floorf(cz);
    float wc[8];
    corner_weights(cx - flx, cy - fly, cz - flz, wc);
    const LevelBits lb = level_bits(k, l);
    const AxisTerms X = axis_terms((int)flx, lb.nl, 7u, 4u), Y = axis_terms((int)fly, lb.nl, lb.shy, 5u),
                    Z = axis_terms((int)flz, lb.nl, lb.shz, 6u);
    uint32_t off[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) off[c] = (c & 1 ? X.t1 : X.t0) | ((c >> 1) & 1 ? Y.t1 : Y.t0) | (c >> 2 ? Z.t1 : Z.t0);
    const LevelView<true> lv = level_view<true>(k, l);
    const auto ld = [&](uint32_t o) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(lv.r, o, 0, 0);
        return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
    };
    float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (l == 0 || !k.aniso) {
        float4 v[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) v[c] = ld(off[c]);
#pragma unroll
        for (int c = 0; c < 8; ++c) acc_fma(acc, wc[c], v[c]);
        return acc;
    }
    const uint32_t FX = (uint32_t)fx << lb.shf, FY = (uint32_t)fy << lb.shf, FZ = (uint32_t)fz << lb.shf;
#pragma unroll
    for (int h = 0; h < 8; h += KC) {          // KC corners x 3 faces in flight
        float4 vx[KC], vy[KC], vz[KC];
#pragma unroll
        for (int c = 0; c < KC; ++c) {
            vx[c] = ld(off[h + c] | FX);
            vy[c] = ld(off[h + c] | FY);
            vz[c] = ld(off[h + c] | FZ);
        }
#pragma unroll
        for (int c = 0; c < KC; ++c) acc_fma(acc, wc[h + c], combine3(wdx, wdy, wdz, vx[c], vy[c], vz[c]));
        __builtin_amdgcn_sched_barrier(0);     // keep the next chunk's loads below (VGPR budget)
    }
    return acc;
}

// D_l(q, d) (A.5): level 0 / isotropic = T_l; anisotropic = faces combined per
// corner texel, then trilinear.  Zero border: out-of-range corners read as 0
// (LevelView); fmaf(w, 0, acc) == acc, the spec's zero-border sum.
template <bool O32, bool UNIF = false, int KC = kCh>   // UNIF: l wave-uniform (buffer resource); else per lane
__device__ __forceinline__ float4 sample_level(const TraceK& k, int l, float qx, float qy, float qz,
                                               int fx, int fy, int fz, float wdx, float wdy, float wdz) {
    if constexpr (O32 && UNIF) return sample_level_bits<KC>(k, l, qx, qy, qz, fx, fy, fz, wdx, wdy, wdz);
    const float scale = __uint_as_float((uint32_t)(127 - l) << 23);  // 2^-l, exact
    const int nl = k.n >> l;
    const float cx = lvl_coord(qx, scale), cy = lvl_coord(qy, scale), cz = lvl_coord(qz, scale);
    const float flx = floorf(cx), fly = floorf(cy), flz = floorf(cz);
    const int ix = (int)flx, iy = (int)fly, iz = (int)flz;
    float wc[8];
    corner_weights(cx - flx, cy - fly, cz - flz, wc);
    uint32_t idx[8];
    bool in[8];
    const int xs[2] = {ix, ix + 1}, ys[2] = {iy, iy + 1}, zs[2] = {iz, iz + 1};
    // brick layout (vct_device.h texel_index), per-axis terms: corner index = X + Y + Z.
    // 24-bit multiplies (v_mul_lo_u32 is quarter rate) where every in-range term fits
    // (n <= 512: (z >> 1) nb^2 < 2^24); an out-of-range corner's index is never read
    const uint32_t nb = nl > 1 ? (uint32_t)nl >> 1 : 1u, nb2 = nb * nb;
    uint32_t tx[2], ty[2], tz[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const uint32_t x = (uint32_t)xs[j], y = (uint32_t)ys[j], z = (uint32_t)zs[j];
        tx[j] = ((x >> 1) << 3) | (x & 1u);
        ty[j] = ((O32 ? __umul24(y >> 1, nb) : (y >> 1) * nb) << 3) | ((y & 1u) << 1);
        tz[j] = ((O32 ? __umul24(z >> 1, nb2) : (z >> 1) * nb2) << 3) | ((z & 1u) << 2);
    }
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const int x = xs[c & 1], y = ys[(c >> 1) & 1], z = zs[c >> 2];
        in[c] = (unsigned)x < (unsigned)nl && (unsigned)y < (unsigned)nl && (unsigned)z < (unsigned)nl;
        idx[c] = tx[c & 1] + ty[(c >> 1) & 1] + tz[c >> 2];
    }
    const auto lv = [&] {
        if constexpr (UNIF) return level_view<O32>(k, l);
        else return level_view_lane(k, l);
    }();
    float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (l == 0 || !k.aniso) {
        float4 v[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) v[c] = lv.fetch(idx[c], in[c]);
#pragma unroll
        for (int c = 0; c < 8; ++c) acc_fma(acc, wc[c], v[c]);
        return acc;
    }
    const uint32_t vl = (uint32_t)nl * (uint32_t)nl * (uint32_t)nl;
    const uint32_t X = (uint32_t)fx * vl, Y = (uint32_t)fy * vl, Z = (uint32_t)fz * vl;
#pragma unroll
    for (int h = 0; h < 8; h += KC) {          // KC corners x 3 faces in flight
        float4 vx[KC], vy[KC], vz[KC];
#pragma unroll
        for (int c = 0; c < KC; ++c) {
            vx[c] = lv.fetch(X + idx[h + c], in[h + c]);
            vy[c] = lv.fetch(Y + idx[h + c], in[h + c]);
            vz[c] = lv.fetch(Z + idx[h + c], in[h + c]);
        }
#pragma unroll
        for (int c = 0; c < KC; ++c) acc_fma(acc, wc[h + c], combine3(wdx, wdy, wdz, vx[c], vy[c], vz[c]));
        __builtin_amdgcn_sched_barrier(0);     // keep the next chunk's loads below (VGPR budget)
    }
    return acc;
}

__device__ __forceinline__ float4 blend(float4 s, float4 s1, float fr) {   // (1 - fr) s + fr s1
    const float omf = 1.0f - fr;
    return make_float4(fmaf(fr, s1.x, omf * s.x), fmaf(fr, s1.y, omf * s.y), fmaf(fr, s1.z, omf * s.z),
                       fmaf(fr, s1.w, omf * s.w));
}

// one cone (A.6), per lane; returns steps, (c, a) in res
template <bool O32>
__device__ __forceinline__ uint32_t march(const TraceK& k, float ox, float oy, float oz, float dx, float dy,
                                          float dz, float tau, float4& res, uint32_t& texels) {
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
        float4 s = sample_level<O32>(k, l0, qx, qy, qz, fx, fy, fz, wdx, wdy, wdz);
        texels += (l0 == 0 || !k.aniso) ? 8u : 24u;
        if (fr > 0.0f && l0 < k.L) {
            texels += k.aniso ? 24u : 8u;
            s = blend(s, sample_level<O32>(k, l0 + 1, qx, qy, qz, fx, fy, fz, wdx, wdy, wdz), fr);
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

// ===========================================================================
// wave-cooperative 4^3 LDS bricks with a two-entry brick cache (variant 0)
// ===========================================================================
// A brick is the 4^3 texel block of one level whose origin is the per-axis
// minimum corner of the active lanes' 2x2x2 footprints.  Lane j stages texel
// (j & 3, (j >> 2) & 3, j >> 4): one coalesced 16-B load per face.  Modes:
//   iso   level 0 / isotropic grid: one slot block (64 texels)
//   comb  anisotropic, the cone direction is the same for every lane: the
//         staging lanes combine the three faces (the spec combines per corner
//         texel), one slot block
//   faces anisotropic otherwise: one slot block per face any lane selects
//         (3, or 4 when one axis has lanes on both sides)
// A staged brick stays in LDS for the following steps of the same cone: level
// l lives in entry l & 1 (a step's two levels never collide), and a step
// reuses the entry when it holds level l and every active lane's footprint
// still lies inside it.  Consecutive steps move ~0.25-1 texel, so a brick
// typically serves two to four steps.
// Brick layout in LDS (float4 slots): texel (x, y, z) at x + 4y + kBz z.  A
// ds_read_b128 serves 16 lanes per LDS cycle, conflict-free when their slots
// differ mod 16; kBz = 19 (= 3 mod 16) keeps the 3x3 corner offsets a wave
// spans in any two axes (floors, walls) distinct mod 16, where 16 would alias
// every z step onto the same banks.
constexpr int kBz = 19;
constexpr int kBlk = 3 * kBz + 16;              // one face block: 73 slots
// 4 x 4 x 3 bricks: a face block of 2 BZ + 16 slots.  Four-face cones in the occupancy
// form: four 54-slot blocks (216 slots) in the 219-slot entry.  Six-face cones in the
// union form: six blocks in the BZ = kBz6 layout (6 x 52 = 312 slots; six 54-slot blocks,
// 324, would not let 16 waves' two entries fit the 160 KB).  18 = 2 mod 16 keeps the
// x / y spans distinct mod 16 and costs a two-way conflict where a 16-lane group spans
// three corners in x and two in z.
template <int BZ> constexpr int blk3() { return 2 * BZ + 16; }
constexpr int kBlk3 = blk3<kBz>();
constexpr int kBz6 = 18;
constexpr int kBlk6 = blk3<kBz6>();
// float4 slots per cache entry: up to 4 face blocks (3 without the four-face union), or
// six 4 x 4 x 3 blocks.  The two cache entries live in LDS regions 0 and 1 (entry a in
// region `flip`): 9984 B per wave with the six-face union (4 waves/SIMD fit the 160 KB),
// 7008 B without the union (5 waves/SIMD).
template <bool UNION> constexpr int entry_slots() {
    return UNION ? (VCT_K4_SIX && 6 * kBlk6 > 4 * kBlk ? 6 * kBlk6 : 4 * kBlk) : 3 * kBlk;
}
template <bool UNION> constexpr int lds_slots() { return 2 * entry_slots<UNION>(); }

// One wave's LDS hand-off (writes -> other lanes' reads, and reads -> next
// writes): the asm "memory" clobber keeps the compiler from moving DS ops
// across it, lgkmcnt(0) makes it explicit in hardware.
__device__ __forceinline__ void wave_lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

struct ConeCtl {                 // wave-uniform facts about one cone
    int funion;                  // faces (bit per VCT_FACE_*) any valid lane selects
    int nfaces;                  // popcount(funion)
    int f0, f1, f2, f3, f4, f5;  // the faces of funion in increasing order (first nfaces valid)
    bool dir_uniform;            // every valid lane has the same wd = d^2 (bitwise) and the same faces
    int neg;                     // bit a: every valid lane moves toward -axis a (brick slack goes there)
    float uwx, uwy, uwz;         // that wd
    int z3;                      // 1: faces-mode bricks are 4 x 4 x 3 (a four-face cone in the occupancy form,
                                 // a five- or six-face cone in the union form)
    int bstr;                    // faces-mode block stride (kBlk, kBlk3 with z3, kBlk6 for six faces)
};

struct BrickEntry {
    int lvl;                     // staged level (-1 = empty)
    int ox, oy, oz;              // its origin
    int zero;                    // every staged texel is +0: any sample from it is exactly (+0, +0, +0, +0)
};
// The cache holds the bricks of the step's two levels: `a` for level l0, `b`
// for l0 + 1.  A cone's mip level never decreases, so when l0 advances by one
// the old `b` becomes the new `a` (b moves in, the LDS regions trade roles) and
// `b` restages; no per-step indexing (a runtime-indexed pair would cost
// scalar selects on every access).
struct BrickCache {              // wave-uniform
    BrickEntry a, b;
    int flip;                    // 0: a in LDS region 0, b in region 1; 1: swapped
};

struct Corner {                  // one lane's trilinear footprint at one level
    float fx, fy, fz;
    int ix, iy, iz;
};

__device__ __forceinline__ Corner level_corner(int l, float qx, float qy, float qz) {
    const float scale = __uint_as_float((uint32_t)(127 - l) << 23);   // 2^-l, exact
    const float cx = lvl_coord(qx, scale), cy = lvl_coord(qy, scale), cz = lvl_coord(qz, scale);
    const float flx = floorf(cx), fly = floorf(cy), flz = floorf(cz);
    Corner c;
    c.fx = cx - flx; c.fy = cy - fly; c.fz = cz - flz;
    c.ix = (int)flx; c.iy = (int)fly; c.iz = (int)flz;
    return c;
}

// z3 = 1: a 4 x 4 x 3 brick (iz - oz <= 1; the shift keeps a negative offset out of range)
__device__ __forceinline__ bool in_brick(const Corner& c, const BrickEntry& b, int z3) {
    return max(max((uint32_t)(c.ix - b.ox), (uint32_t)(c.iy - b.oy)), (uint32_t)(c.iz - b.oz) << z3) <= 2u;
}

// Empty-space test of one lane's level-l trilinear footprint (corner c): its texels lie
// under the level-(l+1) texels (c >> 1) + {0,1}^3, so bit (c >> 1) of map l+1 clear means
// every one of them, in every face, is +0 -- the sample is exactly +0 (the trilinear
// fmaf chain of zeros), the same value the texels would give.  1 when there is no map.
__device__ __forceinline__ uint32_t zbit(const TraceK& k, int l, const Corner& c) {
    const int m = l + 1;
    if (m > k.zm_levels) return 1u;
    const ZLevel z = k.zm[m];
    const uint32_t X = (uint32_t)((c.ix >> 1) + 1), Y = (uint32_t)((c.iy >> 1) + 1), Z = (uint32_t)((c.iz >> 1) + 1);
    // an inactive lane's corner may be garbage: its offset reads 0 past the range (and
    // its bit is masked off by the caller)
    const uint32_t w = z.off + __umul24(__umul24(Z, z.dim) + Y, z.rw) + (X >> 5);
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc((void*)k.zmap, (short)0, (int)k.zmap_bytes, 0x00020000);
    return (__builtin_amdgcn_raw_buffer_load_b32(r, w << 2, 0, 0) >> (X & 31u)) & 1u;
}

// Brick origin on one axis without a 64-lane reduction: relative to the first
// active lane's corner b, the wave fits only if every active lane is within
// [b-2, b+2]; two ballots then give the minimum (or maximum) exactly.  The
// brick's slack (3 - span corners) is put ahead of the march: origin = min
// when the cone moves toward +axis, max - 2 when it moves toward -axis (neg),
// so the following steps stay inside longer.
// negb = 0 or 1 (the cone moves toward -axis): integer arithmetic on wave-uniform values
// only, so the origin stays on the scalar unit (a `neg ? :` on a bool is lowered as a
// lane mask and drags the origin into VGPRs)
__device__ __forceinline__ int wave_origin(int v, unsigned long long am, int fl, int negb, int back = 2) {
    const int b = __builtin_amdgcn_readlane(v, fl);
    const int sg = 1 - 2 * negb;                       // +1 / -1
    const int sv = __mul24(v, sg), sb = b * sg;        // mirrored toward -axis
    // cnt = (m1 & am != 0) + (m2 & am != 0) from the SCC that s_and_b64 sets (4 scalar
    // instructions instead of two masks, two compare / select pairs and an add)
    unsigned long long m2 = wballot(sv < sb - 1), m1 = wballot(sv < sb);   // m2 within m1
    int cnt;
    asm("s_and_b64 %1, %1, %3\n\ts_cselect_b32 %0, 1, 0\n\ts_and_b64 %2, %2, %3\n\ts_addc_u32 %0, %0, 0"
        : "=&s"(cnt), "+s"(m1), "+s"(m2) : "s"(am) : "scc");
    return b - sg * cnt - back * negb;      // back = brick depth - 2
}

// a brick origin over the lanes of am (neg: bit a = the cone moves toward -axis a),
// if every footprint fits the brick there
__device__ __forceinline__ bool brick_origin(const Corner& c, unsigned long long am, int neg, BrickEntry& b, int z3) {
    const int fl = am ? __builtin_ctzll(am) : 0;
    b.ox = wave_origin(c.ix, am, fl, neg & 1);
    b.oy = wave_origin(c.iy, am, fl, (neg >> 1) & 1);
    b.oz = wave_origin(c.iz, am, fl, (neg >> 2) & 1, 2 - z3);
    return wall_in(am, in_brick(c, b, z3));
}

enum { kIso = 0, kComb = 1, kFaces = 2 };

// the lane id, re-derived where it is used: the staging offsets built from it would
// otherwise be hoisted out of the march and held in VGPRs for its whole length
__device__ __forceinline__ int lane_id_opaque() {
    int lane = (int)threadIdx.x;
    asm volatile("" : "+v"(lane));
    return lane & 63;
}

struct Tex4 { float4 a, b, c, d; };

// this lane's staging texel: iso -> a; comb / faces -> faces f0..f3 of the union in a..d
template <bool O32, int AM = -1>   // AM: see step_bricks
__device__ __forceinline__ Tex4 stage_load(const TraceK& k, int l, const BrickEntry& be, int mode,
                                           const ConeCtl& cc) {
    const int nl = k.n >> l;
    const int lane = lane_id_opaque();
    const int sx = be.ox + (lane & 3), sy = be.oy + ((lane >> 2) & 3), sz = be.oz + (lane >> 4);
    const bool inb = (unsigned)sx < (unsigned)nl && (unsigned)sy < (unsigned)nl && (unsigned)sz < (unsigned)nl;
    const uint32_t gi = texel_index_lg((uint32_t)sx, (uint32_t)sy, (uint32_t)sz, (uint32_t)(k.lgn - l));
    const float4 z4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    const LevelView<O32> lv = level_view<O32>(k, l);
    Tex4 t;
    t.b = t.c = t.d = z4;
    if (mode == kIso) {
        t.a = lv.fetch(gi, inb);
    } else {
        const uint32_t sh = 3u * (uint32_t)(k.lgn - l);   // face volume nl^3 = 1 << sh
        t.a = lv.fetch(((uint32_t)cc.f0 << sh) + gi, inb);
        t.b = lv.fetch(((uint32_t)cc.f1 << sh) + gi, inb);
        t.c = lv.fetch(((uint32_t)cc.f2 << sh) + gi, inb);
        if (AM != kComb && cc.nfaces > 3) t.d = lv.fetch(((uint32_t)cc.f3 << sh) + gi, inb);
    }
    return t;
}

__device__ __forceinline__ uint32_t bits4(float4 v) {
    return __float_as_uint(v.x) | __float_as_uint(v.y) | __float_as_uint(v.z) | __float_as_uint(v.w);
}

// stores this lane's staging texel(s); returns true when every value it stored is +0
template <int AM = -1, int BZ = kBz>
__device__ __forceinline__ bool stage_store(int mode, const ConeCtl& cc, const Tex4& t, float4* __restrict__ lds) {
    constexpr int B3 = blk3<BZ>();
    const int lane = lane_id_opaque();
    float4* p = lds + ((lane & 15) + BZ * (lane >> 4));
    uint32_t nz;
    if (mode == kIso) {
        p[0] = t.a;
        nz = bits4(t.a);
    } else if (AM == kComb || mode == kComb) {     // f0, f1, f2 = the x, y, z faces
        const float4 v = combine3(cc.uwx, cc.uwy, cc.uwz, t.a, t.b, t.c);
        p[0] = v;
        nz = bits4(v);
    } else if (cc.z3) {             // 4 x 4 x 3: the lanes of z = 3 store nothing
        nz = 0u;
        if (lane < 48) {
            p[0] = t.a;
            p[B3] = t.b;
            p[2 * B3] = t.c;
            p[3 * B3] = t.d;
            nz = bits4(t.a) | bits4(t.b) | bits4(t.c) | bits4(t.d);
        }
    } else {
        p[0] = t.a;
        p[kBlk] = t.b;
        p[2 * kBlk] = t.c;
        nz = bits4(t.a) | bits4(t.b) | bits4(t.c);
        if (cc.nfaces > 3) {
            p[3 * kBlk] = t.d;
            nz |= bits4(t.d);
        }
    }
    return nz == 0u;
}

// the fifth (sixth) face block of a five- (six-) face brick (union form, 4 x 4 x 3): face
// `face` at block `blk`, staged after the other four (its texel is not held with them: the
// union form has no VGPRs to spare); true when the lane stored +0 only
template <bool O32, int BZ = kBz>
__device__ __forceinline__ bool stage_face(const TraceK& k, int l, const BrickEntry& be, int face, int blk,
                                           float4* __restrict__ lds) {
    const int nl = k.n >> l;
    const int lane = lane_id_opaque();
    const int sx = be.ox + (lane & 3), sy = be.oy + ((lane >> 2) & 3), sz = be.oz + (lane >> 4);
    const bool inb = (unsigned)sx < (unsigned)nl && (unsigned)sy < (unsigned)nl && (unsigned)sz < (unsigned)nl;
    const uint32_t gi = texel_index_lg((uint32_t)sx, (uint32_t)sy, (uint32_t)sz, (uint32_t)(k.lgn - l));
    const LevelView<O32> lv = level_view<O32>(k, l);
    const uint32_t sh = 3u * (uint32_t)(k.lgn - l);
    const float4 v = lv.fetch(((uint32_t)face << sh) + gi, inb);
    uint32_t nz = 0u;
    if (lane < 48) {
        lds[(lane & 15) + BZ * (lane >> 4) + blk * blk3<BZ>()] = v;
        nz = bits4(v);
    }
    return nz == 0u;
}

// slot of the lane's corner 0 in a staged entry
template <int BZ = kBz>
__device__ __forceinline__ int brick_slot(const Corner& c, const BrickEntry& be) {
    return (c.ix - be.ox) + 4 * (c.iy - be.oy) + __mul24(BZ, c.iz - be.oz);
}

// D_l from a staged brick: corner 0 at slot `off`; faces mode reads the lane's own
// face blocks at float4 offsets bx, by, bz
template <int KL, int BZ = kBz>   // KL: corners x 3 faces per LDS burst in faces mode
__device__ __forceinline__ float4 brick_sample(const Corner& c, int off, bool one_slot, int bx,
                                               int by, int bz, float wdx, float wdy, float wdz,
                                               const float4* __restrict__ lds) {
    float wc[8];
    corner_weights(c.fx, c.fy, c.fz, wc);
    const float4* b = lds + off;
    float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (one_slot) {
        float4 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = b[(i & 1) + 4 * ((i >> 1) & 1) + BZ * (i >> 2)];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc_fma(acc, wc[i], v[i]);
    } else {
        const float4 *X = b + bx, *Y = b + by, *Z = b + bz;
#pragma unroll
        for (int h = 0; h < 8; h += KL) {
            float4 vx[KL], vy[KL], vz[KL];
#pragma unroll
            for (int i = 0; i < KL; ++i) {
                const int o = ((h + i) & 1) + 4 * (((h + i) >> 1) & 1) + BZ * ((h + i) >> 2);
                vx[i] = X[o]; vy[i] = Y[o]; vz[i] = Z[o];
            }
#pragma unroll
            for (int i = 0; i < KL; ++i) acc_fma(acc, wc[h + i], combine3(wdx, wdy, wdz, vx[i], vy[i], vz[i]));
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    return acc;
}

// debug counters 16..: why a level sample fell back to gathers (too many
// faces; else the footprint span max-min over the active lanes)
__device__ __forceinline__ void dbg_fallback_reason(const Corner& c, bool active, bool faces_ok, int l,
                                                    bool one_slot = false) {
#ifdef VCT_DEBUG_COUNTERS
    if (!faces_ok) { VCT_DBG(16); return; }
    const int sx = -__ockl_wfred_min_i32(active ? -c.ix : INT_MIN + 1) - __ockl_wfred_min_i32(active ? c.ix : INT_MAX);
    const int sy = -__ockl_wfred_min_i32(active ? -c.iy : INT_MIN + 1) - __ockl_wfred_min_i32(active ? c.iy : INT_MAX);
    const int sz = -__ockl_wfred_min_i32(active ? -c.iz : INT_MIN + 1) - __ockl_wfred_min_i32(active ? c.iz : INT_MAX);
    const int sp = max(sx, max(sy, sz));
    const int bin = sp <= 3 ? 0 : (sp <= 5 ? 1 : (sp <= 9 ? 2 : 3));
    VCT_DBG((l == 0 ? 18 : 22) + bin);
    if (one_slot) {             // iso / combined-face gathers: which larger brick would hold them
        VCT_DBG(45);
        if (sp <= 3) VCT_DBG(43);                               // 5^3
        if (sp <= 4) VCT_DBG(44);                               // 6^3
        const int mn = min(sx, min(sy, sz)), md = sx + sy + sz - sp - mn;
        if (sp <= 6 && md <= 6 && mn <= 1) VCT_DBG(46);         // 8 x 8 x 3 in some orientation
        if ((sp + 2) * (md + 2) * (mn + 2) <= 216) VCT_DBG(47); // a box of <= 216 texels
    }
#endif
}

// A lane's cone direction as the step code reads it: the faces it selects (signs of
// d), their weights d^2 and its face blocks in a faces-mode brick.  Derived on use from
// d and a 6-bit block code rather than held in 9 VGPRs over the march: march_brick
// passes d and the code through an empty asm at every step, so LLVM cannot hoist the
// derivations back out of the loop (a few VALU in the faces-mode / gather paths only).
struct LaneDir {
    float dx, dy, dz;
    uint32_t blk;                // bits 0-2 / 3-5 / 6-8: the x / y / z face's block index in the union
    __device__ int fx() const { return dx >= 0.0f ? VCT_FACE_PX : VCT_FACE_NX; }
    __device__ int fy() const { return dy >= 0.0f ? VCT_FACE_PY : VCT_FACE_NY; }
    __device__ int fz() const { return dz >= 0.0f ? VCT_FACE_PZ : VCT_FACE_NZ; }
    __device__ float wx() const { return dx * dx; }
    __device__ float wy() const { return dy * dy; }
    __device__ float wz() const { return dz * dz; }
    __device__ int bx(int str) const { return __mul24(str, (int)(blk & 7u)); }
    __device__ int by(int str) const { return __mul24(str, (int)((blk >> 3) & 7u)); }
    __device__ int bz(int str) const { return __mul24(str, (int)(blk >> 6)); }
};

// One step's blended sample (1 - fr) D_{l0} + fr D_{l0+1} for a wave-uniform l0.
// Each level is served from the cache, restaged (both levels' loads in one
// batch) or, when the wave's footprint does not fit, gathered per lane.
// AM: the cone's anisotropic staging mode when march_brick specialised the march on it
// (kComb for dir_uniform cones, kFaces otherwise; -1 = read cc.dir_uniform per step).
// BZ = kBz6: the march of a six-face cone (union form), every brick in that layout.
template <bool O32, bool UNION, int KL, int AM = -1, int BZ = kBz>
__device__ __forceinline__ float4 step_bricks(const TraceK& k, int l0, float qx, float qy, float qz,
                                              unsigned long long amA, unsigned long long amB, float fr, const ConeCtl& cc, const LaneDir& ld,
                                              float4* __restrict__ lds, BrickCache& bc, PhaseClock& pc) {
    const float4 z4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    // lane masks in SGPRs; the per-lane bools are their inverse ballots (no VGPR round trip)
    const bool active = __builtin_amdgcn_inverse_ballot_w64(amA);
    const bool activeB = __builtin_amdgcn_inverse_ballot_w64(amB);
    const bool needB = amB != 0ull;
    const int l1 = l0 + 1;                     // needB implies l0 < L
    const int aniso_mode = AM >= 0 ? AM : (cc.dir_uniform ? kComb : kFaces);
    const int modeA = (l0 == 0 || !k.aniso) ? kIso : aniso_mode;
    const int modeB = k.aniso ? aniso_mode : kIso;
    constexpr int kMaxFaces = UNION && VCT_K4_FIVE ? (VCT_K4_SIX && BZ == kBz6 ? 6 : 5) : 4;
    const bool faces_ok = AM == kComb || cc.nfaces <= kMaxFaces;
    // faces-mode levels of a four-face cone in the occupancy form: 4 x 4 x 3 bricks
    // (a dir_uniform cone has three faces: never z3)
    const int z3A = AM != kComb && modeA == kFaces ? cc.z3 : 0, z3B = AM != kComb && modeB == kFaces ? cc.z3 : 0;
    if (bc.a.lvl != l0 && bc.b.lvl == l0) {       // the level advanced by one: b becomes a
        // a cone's level never decreases, so the old a (level l0 - 1) is dead: b moves into
        // a's place, b is emptied and the LDS regions trade roles (no three-way swap)
        bc.a = bc.b;
        bc.b.lvl = -1;
        bc.flip ^= 1;
    }
    float4* ldsA = lds + bc.flip * entry_slots<UNION>();
    float4* ldsB = lds + (bc.flip ^ 1) * entry_slots<UNION>();
    const bool faces_okA = faces_ok, faces_okB = faces_ok;
    // level A: cached, empty, restaged, or gathered
    const Corner cA = level_corner(l0, qx, qy, qz);
    BrickEntry bA = bc.a;
    bool useA = bA.lvl == l0 && wall_in(amA, in_brick(cA, bA, z3A));
    Corner cB;                                 // read only where needB (no copies of cA per step)
    BrickEntry bB = bc.b;
    bool useB = false;
    if (needB) {
        cB = level_corner(l1, qx, qy, qz);
        useB = bB.lvl == l1 && wall_in(amB, in_brick(cB, bB, z3B));
    }
    // a level-A miss first tests for empty space (Grid::zmap): nzA = the active lanes whose
    // footprint may hold a nonzero texel; none -> the sample is exactly +0 and neither a
    // staging nor a gather happens.  Measured (atrium / courtyard, A/B in one box): -2.6 % /
    // -4.5 %.  Not kept: the same test for level B (its misses are mostly nonempty
    // stagings, which then wait for two round trips: +2 % / +1 %), before level B's gathers
    // only (+3 %), only on level A's gather path (+1 %), only for levels <= 1 or <= 2 (the
    // gain shrinks), maps up to level 5 instead of 4 (+0.5 %), and the bit of the next
    // step's level A loaded one step ahead (its position and corner VALU: +7 %).
    // level B restages first: its loads go out before level A's empty-space test waits, so
    // the two round trips overlap (A/B: atrium -1.0 %, courtyard -0.3 %)
    bool stB = false;
    if (needB && !useB && (modeB != kFaces || faces_okB)) {
        BrickEntry nb{};
        nb.lvl = l1;
        if (brick_origin(cB, amB, cc.neg, nb, z3B)) {
            bB = nb;
            bc.b = nb;
            useB = stB = true;
        }
    }
    Tex4 tB;
    if (stB) tB = stage_load<O32, AM>(k, l1, bB, modeB, cc);
    if (stB) VCT_DBG(AM == kComb ? 33 : (modeB == kFaces ? 34 : 42));   // level-B stagings by mode
    if (stB && useA) VCT_DBG(35);                                       // ... while level A hit the cache
    const unsigned long long nzA = useA ? amA : wballot(zbit(k, l0, cA) != 0u) & amA;
    const bool emptyA = nzA == 0ull;                  // the sample is exactly +0
    if (!useA && emptyA) VCT_DBG(32);
    // a brick whose texels are all +0 (empty space) is marked: its samples are exactly
    // zero (fmaf(w, +0, +0) = +0 through the whole trilinear chain), so hits on it skip
    // the LDS reads and the FMAs
    if (stB) {
        bool zB = stage_store<AM, BZ>(modeB, cc, tB, ldsB);
        if (UNION && VCT_K4_FIVE && AM != kComb && modeB == kFaces && cc.nfaces > 4) zB = stage_face<O32, BZ>(k, l1, bB, cc.f4, 4, ldsB) && zB;
        if (kMaxFaces > 5 && modeB == kFaces) zB = stage_face<O32, BZ>(k, l1, bB, cc.f5, 5, ldsB) && zB;
        bB.zero = bc.b.zero = wall(zB);
    }
    bool stA = false;
    if (!useA && !emptyA && (modeA != kFaces || faces_okA)) {
        BrickEntry nb{};
        nb.lvl = l0;
        if (brick_origin(cA, amA, cc.neg, nb, z3A)) {
            bA = nb;
            bc.a = nb;
            useA = stA = true;
        }
    }
    VCT_DBG(useA ? (stA ? 2 : 3) : 1);
    VCT_DBG(needB ? (useB ? (stB ? 27 : 26) : 28) : 31);   // level B: hit / staged / gathered / not sampled
    if (useA && modeA == kFaces) VCT_DBG(29);               // brick samples read three faces per corner
    if (useB && modeB == kFaces) VCT_DBG(30);
    pc.mark(1);
    if (stA) {
        bool zA = stage_store<AM, BZ>(modeA, cc, stage_load<O32, AM>(k, l0, bA, modeA, cc), ldsA);
        if (UNION && VCT_K4_FIVE && AM != kComb && modeA == kFaces && cc.nfaces > 4) zA = stage_face<O32, BZ>(k, l0, bA, cc.f4, 4, ldsA) && zA;
        if (kMaxFaces > 5 && modeA == kFaces) zA = stage_face<O32, BZ>(k, l0, bA, cc.f5, 5, ldsA) && zA;
        bA.zero = bc.a.zero = wall(zA);
    }
    if (stA || stB) wave_lds_sync();
    pc.mark(2);
    const bool readA = useA && !bA.zero, readB = useB && !bB.zero;
    if (useA) VCT_DBG(bA.zero ? 17 : 15);          // level-A samples from zero / nonzero bricks
    // every lane samples (no exec-mask branches): an inactive lane reads the brick's
    // corner-0 texels instead of its own (staged, finite), and its march adds nothing
    // (march_brick scales the sample by 0).  The +0 of an unread level is assigned on its
    // own branch (an initial value would be materialised on every path of the step)
    float4 sA, sB;
    if (readA)
        sA = brick_sample<KL, BZ>(cA, active ? brick_slot<BZ>(cA, bA) : 0, AM == kComb || modeA != kFaces, ld.bx(cc.bstr), ld.by(cc.bstr), ld.bz(cc.bstr),
                              ld.wx(), ld.wy(), ld.wz(), ldsA);
    else
        sA = z4;
    if (readB)
        sB = brick_sample<KL, BZ>(cB, activeB ? brick_slot<BZ>(cB, bB) : 0, AM == kComb || modeB != kFaces, ld.bx(cc.bstr), ld.by(cc.bstr),
                              ld.bz(cc.bstr), ld.wx(), ld.wy(), ld.wz(), ldsB);
    else
        sB = z4;
    if (readA || readB) wave_lds_sync();
    pc.mark(3);
    // per-lane gathers (level A: only the lanes whose footprint may be nonzero load; the
    // others' sample is exactly +0 already)
    if (!useA && !emptyA) {
        VCT_DBG(4 + (l0 < 10 ? l0 : 10));
        dbg_fallback_reason(cA, active, modeA != kFaces || faces_okA, l0, AM == kComb || modeA != kFaces);
        if (__builtin_amdgcn_inverse_ballot_w64(nzA))
            sA = sample_level<O32, true, gather_chunk<UNION>()>(k, l0, qx, qy, qz, ld.fx(), ld.fy(), ld.fz(), ld.wx(), ld.wy(), ld.wz());
    }
    if (needB && !useB) {
        VCT_DBG(4 + (l1 < 10 ? l1 : 10));
        dbg_fallback_reason(cB, activeB, modeB != kFaces || faces_okB, l1, AM == kComb || modeB != kFaces);
        if (activeB)
            sB = sample_level<O32, true, gather_chunk<UNION>()>(k, l1, qx, qy, qz, ld.fx(), ld.fy(), ld.fz(), ld.wx(), ld.wy(), ld.wz());
    }
    pc.mark(4);
    return activeB ? blend(sA, sB, fr) : sA;
}

// The step table held in registers: lane j keeps row j; row i is read with
// v_readlane (no memory round trip at the head of every step).
struct StepRegs {
    float t, D, fr;
    int l0;
};

// ---------------------------------------------------------------------------
// specular step tables: the specular aperture is per pixel (roughness), but a
// wave whose pixels share one tau can march from a table too.  Tables live in
// a per-context cache keyed by tau's bit pattern (they depend only on tau, n
// and L): the first wave that meets a new tau claims a slot, builds the rows
// (the march() recurrence, lane i keeping row i) and publishes them; later
// waves, frames and G-buffers only look them up.  A wave that finds the slot
// still being built, or no free slot, derives (t, D, l0, fr) per lane.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool spec_table(const TraceK& k, float tau, unsigned long long vm, StepRegs& tab) {
    if (!k.spec_tabs) return false;
    const int lane = threadIdx.x & 63;
    const int fl = vm ? __builtin_ctzll(vm) : 0;
    const float tau0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tau), fl));
    if (!wall_in(vm, tau == tau0)) return false;
    const unsigned key = __float_as_uint(tau0);
    for (int j = 0; j < kSpecSlots; ++j) {
        unsigned kj = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(&k.spec_keys[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if (kj == ~0u) {                                        // free: try to claim it for this tau
            unsigned old = 0;
            if (lane == 0) old = atomicCAS(&k.spec_keys[j], ~0u, key);
            old = __builtin_amdgcn_readfirstlane(old);
            if (old == ~0u) {
                const float tau2 = 2.0f * tau0, Lf = (float)k.L;
                float t = 1.0f;
                StepRow mine{__builtin_inff(), 1.0f, 0.0f, 0};
                bool fits = false;
                for (int i = 0; i < 64; ++i) {
                    if (!(t <= k.tmax)) { fits = true; break; }   // row i stays the sentinel
                    const float D = fmaxf(1.0f, tau2 * t);
                    float m = spec_log2(D);
                    if (m > Lf) m = Lf;
                    const int l0 = (int)m;
                    if (lane == i) mine = StepRow{t, D, m - (float)l0, l0};
                    t = t + VCT_STEP_SCALE * D;
                }
                k.spec_rows[j * 64 + lane] = mine;
                __threadfence();
                if (lane == 0) __hip_atomic_store(&k.spec_state[j], fits ? 1u : 2u, __ATOMIC_RELEASE,
                                                  __HIP_MEMORY_SCOPE_AGENT);
                if (!fits) return false;
                tab = StepRegs{mine.t, mine.D, mine.fr, mine.l0};
                return true;
            }
            kj = old;
        }
        if (kj == key) {
            const unsigned st = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(&k.spec_state[j], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT));
            if (st != 1u) return false;
            const StepRow r = k.spec_rows[j * 64 + lane];
            tab = StepRegs{r.t, r.D, r.fr, r.l0};
            return true;
        }
    }
    return false;
}

// one cone, wave-synchronous (A.6); same arithmetic as march().  TAB: (t, D,
// l0, fr) come from a step table (the diffuse one, or a specular one).  CNT:
// count steps and texel fetches (the launches that report them); else both stay 0.
template <bool O32, bool UNION, bool TAB, int KL, bool CNT = true>
__device__ __forceinline__ uint32_t march_brick(const TraceK& k, bool valid, float ox, float oy, float oz,
                                                float dx, float dy, float dz, float tau, float4& res,
                                                uint32_t& texels, float4* __restrict__ lds, const StepRegs& tab,
                                                PhaseClock& pc) {
    const float tau2 = 2.0f * tau;
    const float nf = (float)k.n, Lf = (float)k.L;
    const int fx = dx >= 0.0f ? VCT_FACE_PX : VCT_FACE_NX;
    const int fy = dy >= 0.0f ? VCT_FACE_PY : VCT_FACE_NY;
    const int fz = dz >= 0.0f ? VCT_FACE_PZ : VCT_FACE_NZ;
    const float wdx = dx * dx, wdy = dy * dy, wdz = dz * dz;
    float cr = 0.0f, cg = 0.0f, cb = 0.0f, a = 0.0f, t = 1.0f;
    uint32_t steps = 0;
    unsigned long long am = wballot(valid);      // lanes still marching (an SGPR lane mask)
    ConeCtl cc;
    LaneDir ld;
    {
        const unsigned long long vm = wballot(valid);
        const int fl = vm ? __builtin_ctzll(vm) : 0;
        int u = 0;
#pragma unroll
        for (int f = 0; f < 6; ++f) u |= (wballot((fx == f) | (fy == f) | (fz == f)) & vm) ? 1 << f : 0;
        cc.funion = u;
        cc.neg = ((u & 3) == 2 ? 1 : 0) | ((u & 12) == 8 ? 2 : 0) | ((u & 48) == 32 ? 4 : 0);
        cc.nfaces = __builtin_popcount(u);
        cc.f0 = __builtin_ctz(u | 64);
        u &= u - 1;
        cc.f1 = __builtin_ctz(u | 64);
        u &= u - 1;
        cc.f2 = __builtin_ctz(u | 64);
        u &= u - 1;
        cc.f3 = __builtin_ctz(u | 64);
        u &= u - 1;
        cc.f4 = __builtin_ctz(u | 64);
        u &= u - 1;
        cc.f5 = __builtin_ctz(u | 64);
        // a background lane's faces may lie outside the union (which only the valid lanes
        // define): it gets block 0, so its (discarded) brick samples read staged texels
        ld.blk = valid ? (uint32_t)__builtin_popcount(cc.funion & ((1 << fx) - 1)) |
                             (uint32_t)__builtin_popcount(cc.funion & ((1 << fy) - 1)) << 3 |
                             (uint32_t)__builtin_popcount(cc.funion & ((1 << fz) - 1)) << 6
                       : 0u;
        cc.uwx = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wdx), fl));
        cc.uwy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wdy), fl));
        cc.uwz = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wdz), fl));
        // same d^2 everywhere AND one face per axis (d and -d share d^2)
        cc.dir_uniform = wall_in(vm, (wdx == cc.uwx) & (wdy == cc.uwy) & (wdz == cc.uwz)) && cc.nfaces == 3;
        // the union form's entries hold five 4 x 4 x 3 face blocks (270 slots) or six in
        // the kBz6 layout (312)
        cc.z3 = (!UNION && cc.nfaces == 4) || (UNION && VCT_K4_FIVE && cc.nfaces >= 5) ? 1 : 0;
        cc.bstr = UNION && VCT_K4_SIX && cc.nfaces == 6 ? kBlk6 : (cc.z3 ? kBlk3 : kBlk);
    }
    BrickCache bc;
    bc.a = bc.b = BrickEntry{-1, 0, 0, 0, 0};
    bc.flip = 0;
    // The table marches are compiled once per anisotropic staging mode: a dir_uniform
    // cone (flat surfaces) stages combined faces at every anisotropic level, any other
    // cone stages face blocks, so the per-step mode selects, the four-face / z3 tests
    // and the faces-mode sampling fold away in the combined-face copy.  (Specialising
    // the per-lane specular march too measured slower: -1.0 % instead of -1.6 %.)
    auto march_loop = [&](auto am_tag, auto bz_tag) __attribute__((always_inline)) {
    constexpr int AM = decltype(am_tag)::value;
    constexpr int BZ = decltype(bz_tag)::value;
    for (int i = 0;; ++i) {
        asm volatile("" : "+v"(dx), "+v"(dy), "+v"(dz), "+v"(ld.blk));   // see LaneDir
        ld.dx = dx; ld.dy = dy; ld.dz = dz;
        float D, fr;
        int l0, frb = 0;
        if constexpr (TAB) {                    // wave-uniform row i
            t = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tab.t), i));
            D = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(tab.D), i));
            frb = __builtin_amdgcn_readlane(__float_as_int(tab.fr), i);
            fr = __int_as_float(frb);
            l0 = __builtin_amdgcn_readlane(tab.l0, i);
        }
        const float qx = ox + dx * t, qy = oy + dy * t, qz = oz + dz * t;
        // a >= 0.95, t > tmax or outside the grid ends the lane's march (no short-circuit
        // branches).  Table rows end with t = +inf: q then has an infinite component (|d| = 1
        // leaves at most two zero ones, whose NaN min3 / max3 skip), so `inside` already
        // ends the march there and the t test is only needed for per-lane steps
        const float qmin = fminf(fminf(qx, qy), qz), qmax = fmaxf(fmaxf(qx, qy), qz);
        // one ballot per bare compare, ANDed as scalar masks (a ballot of an ANDed i1 goes
        // through a VGPR)
        am &= wballot(qmin >= 0.0f) & wballot(qmax <= nf) & wballot(a < VCT_ALPHA_STOP);
        if constexpr (!TAB) am &= wballot(t <= k.tmax);
        if (am == 0ull) break;
        const bool active = __builtin_amdgcn_inverse_ballot_w64(am);
        VCT_DBG(TAB ? 36 : 38);                               // wave-steps (table / per-lane steps)
        VCT_DBGN(37, __builtin_popcountll(am));               // active lanes over those wave-steps
        VCT_DBGN(39, __builtin_popcountll(wballot(valid)));   // lanes holding a valid pixel
        if constexpr (!TAB) {
            D = fmaxf(1.0f, tau2 * t);
            float m = spec_log2(D);
            if (m > Lf) m = Lf;
            l0 = (int)m;
            fr = m - (float)l0;
        }
        // both levels sampled: fr > 0 (fr >= +0 here, so a nonzero bit pattern) and l0 < L;
        // for table rows both are wave-uniform: a scalar test, no VALU compare and ballot
        unsigned long long two_m;
        // on the scalar unit from fr's bits (LLVM otherwise turns the bit test into a VALU class test)
        if constexpr (TAB)
            asm("s_cmp_lg_u32 %1, 0\n\ts_cselect_b64 %0, -1, 0\n\ts_cmp_lt_i32 %2, %3\n\ts_cselect_b64 %0, %0, 0"
                : "=&s"(two_m) : "s"(frb), "s"(l0), "s"(k.L) : "scc");
        else two_m = wballot(fr > 0.0f) & wballot(l0 < k.L);
        const bool two = __builtin_amdgcn_inverse_ballot_w64(two_m);
        const int l0f = TAB ? l0 : __builtin_amdgcn_readlane(l0, __builtin_ctzll(am));
        float4 s = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (TAB || wall_in(am, l0 == l0f)) {     // wave-uniform mip pair: brick path
            pc.mark(0);
            s = step_bricks<O32, UNION, KL, AM, BZ>(k, l0f, qx, qy, qz, am, am & two_m, fr, cc, ld, lds, bc, pc);
        } else if (active) {                    // lanes disagree on the level (per-lane roughness)
            s = sample_level<O32, false, gather_chunk<UNION>()>(k, l0, qx, qy, qz, ld.fx(), ld.fy(), ld.fz(), ld.wx(),
                                                                  ld.wy(), ld.wz());
            if (two)
                s = blend(s, sample_level<O32, false, gather_chunk<UNION>()>(k, l0 + 1, qx, qy, qz, ld.fx(), ld.fy(), ld.fz(), ld.wx(), ld.wy(), ld.wz()),
                          fr);
        }
        // no exec-mask branch: an inactive lane's sample is finite, and with oma = +0 the
        // fmaf leaves its (c, a) as they are (fmaf(+0, s, c) = c for c >= +0)
        {
            if constexpr (CNT) {
                if (active) {
                    texels += (l0 == 0 || !k.aniso) ? 8u : 24u;
                    if (two) texels += k.aniso ? 24u : 8u;
                    ++steps;
                }
            }
            const float oma = active ? 1.0f - a : 0.0f;
            cr = fmaf(oma, s.x, cr);
            cg = fmaf(oma, s.y, cg);
            cb = fmaf(oma, s.z, cb);
            a = fmaf(oma, s.w, a);
            if constexpr (!TAB) t = t + VCT_STEP_SCALE * D;   // t of a finished lane is never read again
        }
        pc.mark(5);
    }
    };
    using BzStd = std::integral_constant<int, kBz>;
    if (TAB && cc.dir_uniform) march_loop(std::integral_constant<int, kComb>{}, BzStd{});
    else if (UNION && VCT_K4_SIX && TAB && cc.nfaces == 6) march_loop(std::integral_constant<int, kFaces>{}, std::integral_constant<int, kBz6>{});
    else if (TAB) march_loop(std::integral_constant<int, kFaces>{}, BzStd{});
    else march_loop(std::integral_constant<int, -1>{}, BzStd{});
    res = make_float4(cr, cg, cb, a);
    return steps;
}

// Hand-over data between the two diffuse parts of split 2: relaxed agent-scope
// atomic stores / loads (device-coherent sc1 accesses, no L2 write-back or
// invalidate as a release / acquire fence would issue per wave); the writer
// waits for its stores before it counts in on the pair's flag.
__device__ __forceinline__ void st_coherent(float4* p, float4 v) {
    uint32_t* q = reinterpret_cast<uint32_t*>(p);
    __hip_atomic_store(q + 0, __float_as_uint(v.x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 1, __float_as_uint(v.y), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 2, __float_as_uint(v.z), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 3, __float_as_uint(v.w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float4 ld_coherent(float4* p) {
    uint32_t* q = reinterpret_cast<uint32_t*>(p);
    return make_float4(__uint_as_float(__hip_atomic_load(q + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)),
                       __uint_as_float(__hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)),
                       __uint_as_float(__hip_atomic_load(q + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)),
                       __uint_as_float(__hip_atomic_load(q + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
}

// ===========================================================================
// the kernel: pixel setup, cone loop, outputs (BRICK = variant 0, else 1)
// ===========================================================================
// One wave per workgroup (an 8x8 block): a wave's LDS is released when that wave
// ends (measured: four waves per workgroup held it until the slowest of four ended).
// S3: the split-2 instantiation.  CNT: the launch reports step / texel counts
// (steps_px, cone_steps, texel_fetches); the timed frame loop passes none and runs
// the form without the counting VALU.
constexpr int kKL = 2;    // corners x 3 faces per LDS burst in faces mode (1 / 4 measured slower)
template <bool BRICK, int MINW, bool UNION, bool O32, bool S3 = false, bool CNT = true>
__global__ void __launch_bounds__(64, MINW) k4_trace(TraceK k) {
    __shared__ float4 lds[BRICK ? lds_slots<UNION>() : 1];
    // split: the grid is 2 or 3 parts over the same pixels, dispatched in
    // blockIdx order: split 1 = diffuse cones | specular cone; split 2 = diffuse
    // cones [0, c) | [c, 2c) | ... | specular (ndp diffuse parts of c = nd_chunk cones;
    // two by default).  The parts are multiples of
    // 8 blocks, so a block's parts run on the same XCD (same L2).  Shorter waves:
    // the last waves of a launch (the tail when a rank traces few tiles) end
    // sooner.  In split 2 the diffuse parts hand over through global scratch:
    // each leaves its data, the last to finish completes the spec's cone-order
    // sum (the same fmaf chain) and writes the output.
    const uint32_t nb = S3 ? gridDim.x / (uint32_t)(k.ndp + 1) : (k.split ? gridDim.x >> 1 : gridDim.x);
    // the unit this workgroup traces: blockIdx, or its entry of a dispatch order (a
    // permutation of the units, e.g. longest first)
    const uint32_t vb = k.order ? k.order[blockIdx.x] : blockIdx.x;
    const unsigned long long t_start = k.dur ? __builtin_amdgcn_s_memrealtime() : 0ull;
    const uint32_t rpart = S3 ? vb / nb : (vb >= nb ? 1u : 0u);   // in unit order
    const uint32_t b = vb - rpart * nb;
    // its role: S3 parts 0..ndp-1 diffuse, ndp specular (spec_first: the specular part first)
    const uint32_t part = (S3 && k.spec_first) ? (rpart == 0 ? (uint32_t)k.ndp : rpart - 1u) : rpart;
    // XCD-aware workgroup -> (local tile, 8x8 block) map, bijective for any grid.
    // The hardware hands workgroup b to XCD b & 7.  Units (waves) are dealt to the
    // XCDs in chunks of G consecutive units (the
    // pixels of a chunk share that XCD's L2), chunk c to XCD c & 7, so every XCD
    // gets a screen-wide sample of the frame: cost varies strongly across the
    // image (the atrium's middle rows cost ~2x its top and bottom rows), and
    // with one contiguous run of tiles per XCD the slowest XCD set the launch.
    // Units past the last full round of 8 chunks go round-robin.  k.xcd_g = 0:
    // one contiguous run per XCD (the earlier map, kept for A/B).
    const uint32_t xcd = b & 7;
    uint32_t rbw;
    if (k.xcd_g == 0) {
        const uint32_t q = nb >> 3, r = nb & 7;
        rbw = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
    } else {
        const uint32_t G = (uint32_t)k.xcd_g, full = (nb / (8u * G)) * (8u * G);
        const uint32_t kk = b >> 3;
        rbw = b < full ? G * (xcd + 8u * (kk / G)) + kk % G : b;
    }
    const uint32_t rb = rbw >> 2;                 // the 16x16 block
    const uint32_t wave = rbw & 3u;               // its 8x8 quarter
    const uint32_t lt = rb >> 4, sub = rb & 15;
    int c_lo = 0, c_hi = k.nd, grp = 0;        // diffuse cones [c_lo, c_hi); grp g >= 1: diffuse part g - 1 of split 2
    bool do_spec = k.spec_on != 0, wr_diff = true, wr_spec = true;
    if (k.split == 1) {
        if (part == 0) { do_spec = false; wr_spec = false; }
        else { c_hi = 0; wr_diff = false; }
    } else if (S3) {
        if (part == (uint32_t)k.ndp) { c_hi = 0; wr_diff = false; }
        else { do_spec = false; wr_spec = false; wr_diff = false; grp = (int)part + 1;
               c_lo = (int)part * k.nd_chunk; c_hi = min(k.nd, c_lo + k.nd_chunk); }
    }
    const bool do_diff = c_hi > c_lo;
    const uint32_t lane = threadIdx.x & 63;
    PhaseClock pc;
    pc.start();
#if defined(VCT_DEBUG_CLOCK) || defined(VCT_DEBUG_WAVES)
    const unsigned long long wave_t0 = __builtin_amdgcn_s_memrealtime();
#endif
    // lane -> pixel of the wave's 8x8 block in Morton order: the lanes of each
    // ds_read_b128 / load group are then a compact 2x2 / 4x4 pixel block (measured
    // against row-major lanes: 2.07 -> 1.92 ms in round 1)
    const uint32_t mx = (lane & 1) | ((lane >> 1) & 2) | ((lane >> 2) & 4);
    const uint32_t my = ((lane >> 1) & 1) | ((lane >> 2) & 2) | ((lane >> 3) & 4);
    const uint32_t px = (sub & 3) * 16 + (wave & 1) * 8 + mx;
    const uint32_t py = (sub >> 2) * 16 + (wave >> 1) * 8 + my;
    bool in_frame;
    uint32_t pix, oidx;                          // w * h < 2^32 (vct_trace_device)
    if (k.perm) {                                // reordered rays: whole frame, outputs at the pixel
        const uint32_t si = (rb * 4u + wave) * 64u + lane;
        const uint32_t* perm = (k.perm_spec && !do_diff) ? k.perm_spec : k.perm;
        in_frame = si < k.npx;
        pix = oidx = in_frame ? perm[si] : 0u;
    } else {
        const uint32_t tile = lt * (uint32_t)k.world + (uint32_t)k.rank;
        const uint32_t x = (tile % (uint32_t)k.tiles_x) * VCT_TILE + px;
        const uint32_t y = (tile / (uint32_t)k.tiles_x) * VCT_TILE + py;
        in_frame = x < (uint32_t)k.w && y < (uint32_t)k.h;
        pix = in_frame ? y * (uint32_t)k.w + x : 0u;
        oidx = k.compact ? lt * (VCT_TILE * VCT_TILE) + py * VCT_TILE + px : pix;
    }

    float4 dout = make_float4(0.0f, 0.0f, 0.0f, 0.0f), sout = dout;
    uint32_t steps = 0, texels = 0;
    float4 P = dout;
    if (in_frame) P = k.pos[pix];
    const bool valid = P.w != 0.0f;
    // BRICK: every lane of a wave with any valid pixel stays in the wave-uniform
    // loops (background lanes stage texels); variant 1: only valid lanes trace
    const bool run = BRICK ? wany(valid) : valid;
    StepRegs tab{};
    if (BRICK && run && do_diff && lane < (uint32_t)kMaxStepRows) {
        const StepRow r = k.steps_tab[lane];
        tab = StepRegs{r.t, r.D, r.fr, r.l0};
    }
    float ir = 0.0f, ig = 0.0f, ib = 0.0f, occ = 0.0f;   // diffuse sum in cone order
    if (run) {
        float4 N4 = make_float4(0.0f, 1.0f, 0.0f, 0.0f);
        if (valid) N4 = k.nrm[pix];
        float nx = N4.x, ny = N4.y, nz = N4.z;
        const float ox = (P.x - k.g0x) * k.inv_h + nx;
        const float oy = (P.y - k.g0y) * k.inv_h + ny;
        const float oz = (P.z - k.g0z) * k.inv_h + nz;
        const float(*cones)[4] = cone_table(k.nd);
        for (int c = S3 ? c_lo : 0; c < c_hi; ++c) {
            // the tangent frame is rebuilt per cone (a few VALU per ~12 steps) instead of
            // holding 6 VGPRs over the march; the empty asm keeps LLVM from hoisting it
            asm volatile("" : "+v"(nx), "+v"(ny), "+v"(nz));
            // Duff et al. 2017 branchless orthonormal basis
            const float sgn = copysignf(1.0f, nz);
            const float ka = -1.0f / (sgn + nz);
            const float kb = (nx * ny) * ka;
            const float Tx = 1.0f + ((sgn * nx) * nx) * ka, Ty = sgn * kb, Tz = -(sgn * nx);
            const float Bx = kb, By = sgn + (ny * ny) * ka, Bz = -ny;
            const float cn = cones[c][0], ct = cones[c][1], cb = cones[c][2], wk = cones[c][3];
            const float dx = (cn * nx + ct * Tx) + cb * Bx;
            const float dy = (cn * ny + ct * Ty) + cb * By;
            const float dz = (cn * nz + ct * Tz) + cb * Bz;
            float4 res;
            if constexpr (BRICK) steps += march_brick<O32, UNION, true, kKL, CNT>(k, valid, ox, oy, oz, dx, dy, dz, k.tau_d, res, texels, lds, tab, pc);
            else steps += march<O32>(k, ox, oy, oz, dx, dy, dz, k.tau_d, res, texels);
            if (S3 && grp >= 2) {                // later parts: results go to the hand-over scratch
                if (in_frame || k.compact) st_coherent(&k.sc_cone[(size_t)(c - k.nd_chunk) * k.sc_px + oidx], res);
            } else {
                ir = fmaf(wk, res.x, ir);
                ig = fmaf(wk, res.y, ig);
                ib = fmaf(wk, res.z, ib);
                occ = fmaf(wk, res.w, occ);
            }
        }
        dout = sel4(valid, make_float4(ir, ig, ib, 1.0f - occ), dout);
        if (do_spec) {
            // position and normal are read again rather than held over the diffuse march
            // (the compiler fence keeps the loads from being merged with the first ones)
            asm volatile("" ::: "memory");
            if (in_frame) P = k.pos[pix];
            if (valid) N4 = k.nrm[pix];
            nx = N4.x; ny = N4.y; nz = N4.z;
            float vx = k.ex - P.x, vy = k.ey - P.y, vz = k.ez - P.z;
            float vl = sqrtf(dot3(vx, vy, vz, vx, vy, vz));
            vl = valid ? vl : 1.0f;
            vx = vx / vl; vy = vy / vl; vz = vz / vl;
            const float ndv = dot3(nx, ny, nz, vx, vy, vz);
            const float k2 = 2.0f * ndv;
            const float rx = k2 * nx - vx, ry = k2 * ny - vy, rz = k2 * nz - vz;
            float rough = 0.1f;
            if (valid) rough = k.alb[pix].w;
            const float tau = fminf(fmaxf(rough, VCT_SPEC_TAU_MIN), VCT_SPEC_TAU_MAX);
            float4 res;
            if constexpr (BRICK) {
                if (spec_table(k, tau, wballot(valid), tab))
                    steps += march_brick<O32, UNION, true, kKL, CNT>(k, valid, ox, oy, oz, rx, ry, rz, tau, res, texels, lds, tab, pc);
                else
                    steps += march_brick<O32, UNION, false, kKL, CNT>(k, valid, ox, oy, oz, rx, ry, rz, tau, res, texels, lds, tab, pc);
            } else {
                steps += march<O32>(k, ox, oy, oz, rx, ry, rz, tau, res, texels);
            }
            sout = sel4(valid, res, sout);
        }
    }
    if (S3 && grp != 0) {
        // split 2 hand-over: leave this part's data, count in; the last of the ndp
        // waves (same block, same wave slot) finishes the cone-order sum
        const bool px_ok = in_frame || k.compact;
        if (grp == 1 && px_ok) st_coherent(&k.sc_part[oidx], make_float4(ir, ig, ib, occ));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the device-coherent stores have landed
        const uint32_t wid = rb * 4u + wave;
        uint32_t prev = 0;
        if (lane == 0) prev = atomicAdd(&k.sc_flag[wid], 1u);
        prev = (uint32_t)__builtin_amdgcn_readfirstlane((int)prev);
        if (prev == (uint32_t)k.ndp - 1u) {      // every other part has counted in: its data is there
            float4 acc = make_float4(ir, ig, ib, occ);
            if (grp != 1 && px_ok) acc = ld_coherent(&k.sc_part[oidx]);
            const float(*cones)[4] = cone_table(k.nd);
            for (int c = k.nd_chunk; c < k.nd; ++c) {
                const float wk = cones[c][3];
                float4 res = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                if (px_ok) res = ld_coherent(&k.sc_cone[(size_t)(c - k.nd_chunk) * k.sc_px + oidx]);
                acc.x = fmaf(wk, res.x, acc.x);
                acc.y = fmaf(wk, res.y, acc.y);
                acc.z = fmaf(wk, res.z, acc.z);
                acc.w = fmaf(wk, res.w, acc.w);
            }
            dout = sel4(valid, make_float4(acc.x, acc.y, acc.z, 1.0f - acc.w), dout);
            wr_diff = true;
            if (lane == 0) k.sc_flag[wid] = 0u;   // ready for the next launch
        }
    }
    if (in_frame || k.compact) {
        if (wr_diff) k.diff[oidx] = dout;
        if (wr_spec) k.spec[oidx] = sout;
        if (CNT && k.steps_px && in_frame) k.steps_px[pix] = steps;
    }
    if (CNT && k.steps_total) {
        const uint32_t ws = wave_sum_u32(steps);
        if (lane == 0 && ws) atomicAdd(k.steps_total, (unsigned long long)ws);
    }
    if (CNT && k.texels_total) {
        const uint32_t wt = wave_sum_u32(texels);
        if (lane == 0 && wt) atomicAdd(k.texels_total, (unsigned long long)wt);
    }
    if (k.dur && lane == 0) k.dur[vb] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_start);
    pc.flush();
#if defined(VCT_DEBUG_CLOCK) || defined(VCT_DEBUG_WAVES)
    {
        const uint32_t wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        if (lane == 0 && wid < (uint32_t)kDbgWaves) {
            vct_dbg_wave[wid][0] = wave_t0;
            vct_dbg_wave[wid][1] = __builtin_amdgcn_s_memrealtime();
            const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);      // HW_REG_HW_ID
            const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);    // HW_REG_XCC_ID
            vct_dbg_wave[wid][2] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
        }
    }
#endif
}

// Longest-first dispatch (LPT) of a K4 launch.  A unit (workgroup = one 8x8 block of one
// cone part) runs on XCD unit % 8 (round-robin placement; the XCD map inside k4_trace keeps a
// tile's units on one XCD), so the order is built per residue class: class x's units
// {x, x + 8, ...} are bucketed by their last recorded duration (log2 with four steps per
// octave, longest bucket first) and dealt to the class's workgroups x + 8 i in that order.
// Each unit's duration is read once (a concurrent frame may be rewriting it: any values
// give a permutation), so the result is always a permutation of the units and the frame's
// outputs are those of blockIdx order (every unit runs the same arithmetic wherever it is
// dispatched).  Emulated (tools/lpt_emul.py, same-frame durations): one rank of 8 at 1080p
// 0.234 -> 0.201 ms, one of 4 0.392 -> 0.364 ms, the full C3 frame 1.109 -> 1.073 ms; on the
// device the full frame lost (the order kernel and the scattered tiles cost more than its
// tail), hence launch_trace's size and overlap rule.
constexpr uint32_t kLptMaxGenerations = 4;       // LPT for launches of <= 4 x (CUs x 20) waves
constexpr uint32_t kLptBuckets = 128;
constexpr uint32_t kLptMaxPerClass = 48u * 1024u;   // key bytes per class in LDS
__global__ void __launch_bounds__(1024) k4_lpt_order(const uint32_t* __restrict__ dur, uint32_t units,
                                                     uint32_t* __restrict__ order) {
    extern __shared__ uint8_t key[];              // per unit of this class
    __shared__ uint32_t off[kLptBuckets];
    const uint32_t x = blockIdx.x, tid = threadIdx.x;
    const uint32_t nc = units > x ? (units - x + 7u) / 8u : 0u;
    for (uint32_t i = tid; i < kLptBuckets; i += 1024u) off[i] = 0u;
    __syncthreads();
    for (uint32_t j = tid; j < nc; j += 1024u) {
        const uint32_t d = dur[x + 8u * j] | 1u;
        const uint32_t lg = 31u - (uint32_t)__builtin_clz(d);
        const uint32_t sub = lg >= 2u ? (d >> (lg - 2u)) & 3u : 0u;
        const uint32_t bk = min(4u * lg + sub, kLptBuckets - 1u);
        const uint8_t kk = (uint8_t)(kLptBuckets - 1u - bk);   // the longest first
        key[j] = kk;
        atomicAdd(&off[kk], 1u);
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t run = 0;
        for (uint32_t i = 0; i < kLptBuckets; ++i) {
            const uint32_t t = off[i];
            off[i] = run;
            run += t;
        }
    }
    __syncthreads();
    for (uint32_t j = tid; j < nc; j += 1024u) {
        const uint32_t pos = atomicAdd(&off[key[j]], 1u);
        order[x + 8u * pos] = x + 8u * j;
    }
}

// Longest-first with locality: a STABLE partition of each class into kLptParts duration
// bands below the class's longest unit (>= max / 2, >= max / 4, >= max / 8, the rest),
// longest band first, each band in blockIdx order.  The plain bucket sort above scatters a
// tile's units over the whole launch (its L2 locality: the courtyard +2 %, the pipelined
// C3 frame +3 %); inside a band the units keep the XCD map's tile order.
constexpr int kLptParts = 4;
constexpr int kLptRounds = 32;                   // units per class <= 32 x 1024 (a 4K frame: 32 640)
__device__ __forceinline__ uint32_t lpt_band(uint32_t d, uint32_t dmax) {
    // floor(log2(dmax / d)) clamped to the bands, from the leading-bit positions (+1 when
    // d's mantissa exceeds dmax's shifted down: exact for the band edges dmax / 2^k)
    const uint32_t dd = d | 1u;
    int k = (int)__builtin_clz(dd) - (int)__builtin_clz(dmax | 1u);
    if (k >= 0 && ((dmax | 1u) >> k) > dd) ++k;   // d below dmax >> k: one band further
    return (uint32_t)min(max(k, 0), kLptParts - 1);
}

__global__ void __launch_bounds__(1024) k4_lpt_bands(const uint32_t* __restrict__ dur, uint32_t units,
                                                     uint32_t* __restrict__ order) {
    __shared__ uint32_t wmax[16], wc[16][kLptParts], base[kLptParts], run[kLptParts], rt[kLptParts];
    const uint32_t x = blockIdx.x, tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t nc = units > x ? (units - x + 7u) / 8u : 0u;
    uint32_t m = 0;
    for (uint32_t j = tid; j < nc; j += 1024u) m = max(m, dur[x + 8u * j]);
    for (int o = 32; o >= 1; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
    if (lane == 0) wmax[wave] = m;
    if (tid < kLptParts) base[tid] = run[tid] = 0u;
    __syncthreads();
    uint32_t dmax = 0;
    for (int w = 0; w < 16; ++w) dmax = max(dmax, wmax[w]);
    // each unit's band from ONE read of its duration (a concurrent frame may be rewriting
    // it: the bands counted and the bands placed must be the same), kept in registers; the
    // band sizes first, then the units placed round by round (1024 consecutive units a round)
    __shared__ uint8_t keys[kLptRounds * 1024];
    const uint32_t rounds = (nc + 1023u) / 1024u;   // <= kLptRounds (launch_trace)
    for (uint32_t j = tid; j < nc; j += 1024u) {
        const uint32_t k = lpt_band(dur[x + 8u * j], dmax);
        keys[j] = (uint8_t)k;
        atomicAdd(&run[k], 1u);
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t acc = 0;
        for (int k = 0; k < kLptParts; ++k) {
            base[k] = acc;
            acc += run[k];
            run[k] = 0u;
        }
    }
    __syncthreads();
    for (uint32_t r = 0; r < rounds; ++r) {
        const uint32_t j = r * 1024u + tid;
        const uint32_t key = j < nc ? (uint32_t)keys[j] : (uint32_t)kLptParts;
        unsigned long long mine = 0ull;
#pragma unroll
        for (int k = 0; k < kLptParts; ++k) {
            const unsigned long long b = __builtin_amdgcn_ballot_w64(key == (uint32_t)k);
            if (lane == 0) wc[wave][k] = (uint32_t)__builtin_popcountll(b);
            if (key == (uint32_t)k) mine = b;
        }
        __syncthreads();
        if (tid < kLptParts) {
            uint32_t acc = 0;
            for (int w = 0; w < 16; ++w) {
                const uint32_t t = wc[w][tid];
                wc[w][tid] = acc;
                acc += t;
            }
            rt[tid] = acc;
        }
        __syncthreads();
        if (j < nc) {
            const uint32_t pos = base[key] + run[key] + wc[wave][key] +
                                 __builtin_amdgcn_mbcnt_hi((uint32_t)(mine >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mine, 0u));
            order[x + 8u * pos] = x + 8u * j;
        }
        __syncthreads();
        if (tid < kLptParts) run[tid] += rt[tid];
        __syncthreads();
    }
}

}  // namespace

int build_step_table(float tau, uint32_t n, uint32_t L, StepRow* rows) {
    // the march() recurrence of the kernels, on the host (same binary32 operation sequence)
    const float tau2 = 2.0f * tau, tmax = (float)n * VCT_SQRT3, Lf = (float)L;
    float t = 1.0f;
    for (int i = 0; i < kMaxStepRows; ++i) {
        if (!(t <= tmax)) {
            rows[i] = StepRow{__builtin_huge_valf(), 1.0f, 0.0f, 0};
            return i + 1;
        }
        const float D = fmaxf(1.0f, tau2 * t);
        float m = spec_log2(D);
        if (m > Lf) m = Lf;
        const int l0 = (int)m;
        rows[i] = StepRow{t, D, m - (float)l0, l0};
        t = t + VCT_STEP_SCALE * D;
    }
    return -1;
}

// launches of at most this many 16x16 blocks split the diffuse cones into two
// parts (three parts with the specular cone): few blocks per CU, so the tail of
// the longest waves dominates (a rank of an 8-GPU frame traces 1/8)
constexpr uint32_t kSplit3MaxBlocks = 1024;   // measured: 3 parts pay off at 1080p / 8 ranks only

// The candidate of a default-variant launch (K4Tuner in vct_internal.h): bit 0 the
// form (0 union, 1 occupancy), bit 1 ray reordering.  cands lists the candidates the
// variant leaves open (n of them, 1, 2 or 4).  While an entry is timing, timed
// (counter-free) launches cycle through the candidates until each has kSamples
// completed samples after its first (cold) one, then the fastest is kept; counting
// launches take the choice (cands[0] while timing) and are never timed.  Once chosen,
// every kWatchEvery-th timed launch is watched without blocking (drift check).
// *evp: the event pair to record around the launch, or null.
static bool tune_log() {
    static const bool on = getenv("VCT_TUNE_LOG") != nullptr;
    return on;
}

static void k4_retime(K4Tuner::Entry& t, bool by_epoch) {
    for (int f = 0; f < 4; ++f) {
        t.seen[f] = 1;                           // warm code: no cold sample to drop
        t.best[f] = 0.0f;
        for (bool& b : t.busy[f]) b = false;     // watch samples in flight: not timing samples
    }
    t.prev = t.chosen;
    t.by_epoch = by_epoch;
    t.chosen = -1;
    t.drift = 0;
    t.since = t.launches = 0;
    t.last = nullptr;
    ++t.retimes;
}

static int k4_form(vct_ctx* c, uint64_t key, const int* cands_in, int n_in, bool timed, hipEvent_t** evp) {
    K4Tuner& T = c->k4tune;
    *evp = nullptr;
    int ix = -1;
    for (int i = 0; i < K4Tuner::kEntries; ++i)
        if (T.e[i].key == key) ix = i;
    if (ix < 0) {                                // a new workload: the least recently used entry
        ix = 0;
        for (int i = 1; i < K4Tuner::kEntries; ++i)
            if (T.e[i].used < T.e[ix].used) ix = i;
        K4Tuner::Entry& e = T.e[ix];
        e.key = key;
        e.chosen = -1;
        k4_retime(e, false);
        for (int f = 0; f < 4; ++f) e.seen[f] = 0;   // first timing: drop each candidate's cold sample
        e.retimes = 0;
        e.epoch = c->grid_epoch;
        e.epoch_wait = K4Tuner::kEpochMin;
        e.hist_ok = false;                       // another workload's durations
        e.hist_cand = -1;
    }
    K4Tuner::Entry& t = T.e[ix];
    t.used = ++T.clock;
    T.cur = ix;
    if (n_in == 1) {                             // the variant forces the candidate
        t.chosen = cands_in[0];
        return cands_in[0];
    }
    bool overlapped = false;                     // the previous launch (another stream) still runs
    if (timed) {
        if (T.prev_set && T.prev_stream != c->stream) T.multi_until = T.clock + K4Tuner::kMultiLaunches;
        T.prev_stream = c->stream;
        T.prev_set = true;
        T.multi = T.clock < T.multi_until;
        if (T.multi && T.prev_end) overlapped = hipEventQuery(T.prev_end) == hipErrorNotReady;
    }
    if (t.chosen < 0 && timed && t.last) {       // while timing: this entry's previous timed launch first
        (void)hipEventSynchronize(t.last);
        t.last = nullptr;
    }
    if (t.chosen < 0 && timed && overlapped) {   // ... and the previous launch of any stream
        (void)hipEventSynchronize(T.prev_end);
        overlapped = false;
    }
    for (int f = 0; f < 4; ++f)                  // harvest completed samples (non-blocking)
        for (int sl = 0; sl < K4Tuner::kSlots; ++sl) {
            if (!t.busy[f][sl] || hipEventQuery(t.ev[f][sl][1]) != hipSuccess) continue;
            t.busy[f][sl] = false;
            float ms = 0.0f;
            if (hipEventElapsedTime(&ms, t.ev[f][sl][0], t.ev[f][sl][1]) != hipSuccess) continue;
            if (t.chosen >= 0) {                 // a watch sample of the chosen candidate
                if (f != t.chosen) continue;
                if (t.settled <= 0.0f) t.settled = ms;   // chosen without timing: the first sample settles it
                else t.drift = ms > K4Tuner::kDrift * t.settled ? t.drift + 1 : 0;
                continue;
            }
            if (t.seen[f]++ == 0) continue;      // the first launch of a candidate pays its code load
            t.best[f] = t.best[f] == 0.0f ? ms : fminf(t.best[f], ms);
        }
    if (t.chosen < 0) {                          // a candidate clearly slower than the best so far: done
        float lo = 0.0f;
        for (int f = 0; f < 4; ++f)
            if (t.best[f] > 0.0f && (lo == 0.0f || t.best[f] < lo)) lo = t.best[f];
        for (int f = 0; f < 4; ++f)
            if (t.best[f] > K4Tuner::kCompetitive * lo && t.seen[f] <= K4Tuner::kSamples) t.seen[f] = K4Tuner::kSamples + 1;
    }
    if (t.chosen >= 0 && timed) {
        if (t.drift >= K4Tuner::kDriftRuns) {
            if (tune_log())
                fprintf(stderr, "[vct tune] key %016llx: drift of %d (settled %.4f ms): time again\n",
                        (unsigned long long)t.key, t.chosen, t.settled);
            k4_retime(t, false);                 // the workload changed under the key: every candidate
            t.epoch = c->grid_epoch;
        } else if (t.epoch != c->grid_epoch && t.since >= t.epoch_wait) {
            if (tune_log())
                fprintf(stderr, "[vct tune] key %016llx: new scene (after %u launches): time again\n",
                        (unsigned long long)t.key, t.since);
            k4_retime(t, true);
            t.epoch = c->grid_epoch;
        }
    }
    const int* cands = cands_in;
    const int n = n_in;
    if (t.chosen >= 0) {
        // a host overlapping frames on two streams gets no watch: a launch's event time then
        // depends on how much of it the neighbouring frames shared (measured: false drifts)
        if (!timed || ++t.since % K4Tuner::kWatchEvery != 0 || T.multi) return t.chosen;
        const int f = t.chosen, sl = t.head[f];
        if (t.busy[f][sl]) return f;
        for (hipEvent_t& ev : t.ev[f][sl])
            if (!ev && hipEventCreate(&ev) != hipSuccess) return f;
        t.busy[f][sl] = true;
        t.head[f] = (sl + 1) % K4Tuner::kSlots;
        *evp = t.ev[f][sl];
        return f;
    }
    bool done = true;
    for (int i = 0; i < n; ++i) done = done && t.seen[cands[i]] > K4Tuner::kSamples;
    if (done) {
        int b = cands[0];
        for (int i = 1; i < n; ++i)
            if (t.best[cands[i]] < t.best[b]) b = cands[i];
        t.chosen = b;
        t.settled = t.best[b];
        t.since = 0;
        if (t.by_epoch)                          // a scene change that kept the winner: wait longer next time
            t.epoch_wait = b == t.prev ? (t.epoch_wait * 2u > K4Tuner::kEpochMax ? K4Tuner::kEpochMax : t.epoch_wait * 2u)
                                       : K4Tuner::kEpochMin;
        if (tune_log())
            fprintf(stderr, "[vct tune] key %016llx chose %d (%.4f ms) of %d candidates; best ms %.4f %.4f %.4f %.4f; "
                            "retime %u%s\n",
                    (unsigned long long)t.key, b, t.best[b], n, t.best[0], t.best[1], t.best[2], t.best[3], t.retimes,
                    t.by_epoch ? " (new scene)" : "");
        for (int f = 0; f < 4; ++f)              // samples still in flight belong to the timing
            for (bool& bz : t.busy[f]) bz = false;
        return t.chosen;
    }
    if (!timed) return cands[0];
    const int f = cands[t.launches++ % (uint32_t)n];
    const int sl = t.head[f];
    if (t.busy[f][sl]) return f;                 // every slot of this candidate in flight: run untimed
    for (hipEvent_t& e : t.ev[f][sl])
        if (!e && hipEventCreate(&e) != hipSuccess) return f;
    t.busy[f][sl] = true;
    t.head[f] = (sl + 1) % K4Tuner::kSlots;
    *evp = t.ev[f][sl];
    t.last = t.ev[f][sl][1];
    return f;
}

hipError_t launch_trace(vct_ctx* c, const vct_trace_args* a) {
    const Grid& g = c->grid;
    TraceK k;
    k.pyr = g.pyr;
    for (int i = 0; i <= kMaxLevels; ++i) {
        k.lvl_off[i] = g.lvl_off[i];
        // level i's bytes (all faces): n_i^3 texels x 16 B, x 6 faces above level 0 when anisotropic
        const uint64_t ni = i <= (int)g.L ? (uint64_t)(g.n >> i) : 0u;
        const uint64_t by = ni * ni * ni * 16u * (i > 0 && g.aniso ? 6u : 1u);
        k.lvl[i] = LevelRange{g.pyr + g.lvl_off[i], by <= 0xffffffffull ? (uint32_t)by : 0u, 0u};   // 2 GiB at 512^3
    }
    k.n = (int)g.n; k.L = (int)g.L;
    k.lgn = __builtin_ctz(g.n);
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
    k.compact = a->tile_compact ? 1 : 0;
    k.nd = (int)c->cfg.n_diffuse;
    k.spec_on = c->cfg.specular ? 1 : 0;
    k.aniso = g.aniso;
    k.tau_d = c->cfg.n_diffuse == 16 ? VCT_TAN20 : VCT_TAN30;
    k.steps_tab = c->step_tab;
    k.spec_keys = c->spec_keys;
    k.spec_state = c->spec_keys + kSpecSlots;
    k.spec_rows = c->spec_rows;
    k.spec_tabs = (a->variant & 0x100) ? 0 : 1;
    // cone groups in separate workgroups (variant bits: 0x200 off, 0x400 three parts,
    // 0x800 two parts; default by launch size); per-pixel step counts need every
    // cone of a pixel in one lane, so steps_px keeps one part
    k.split = (k.spec_on && k.nd > 0 && !a->steps_px && !(a->variant & 0x200)) ? 1 : 0;
    k.nd_chunk = (k.nd + 1) / 2;
    k.ndp = 2;
    k.spec_first = (a->variant & kVarSpecFirst) ? 1 : 0;
    {   // variant bits 16-19: XCD map (0 default; 1 contiguous runs; 2..6: chunks of 1, 4, 16, 64, 256 units)
        static const int g_of[7] = {0, 0, 1, 4, 16, 64, 256};
        const uint32_t m = (a->variant >> 16) & 0xf;
        k.xcd_g = g_of[m < 7 ? m : 0];
    }
    k.sc_part = k.sc_cone = nullptr; k.sc_flag = nullptr; k.sc_px = 0;
    k.perm = k.perm_spec = nullptr;
    k.order = c->k4_dbg_order;
    k.dur = c->k4_dbg_dur;
    k.npx = a->width * a->height;
    k.zmap = g.zm_valid ? g.zmap : nullptr;
    k.zm_levels = g.zm_valid ? g.zm_levels : 0;
    k.zmap_bytes = 0;
    for (int m = 0; m <= Grid::kZLevels; ++m) {
        k.zm[m] = ZLevel{g.zm_off[m], g.zm_dim[m], g.zm_rw[m], 0u};
        if (m >= 1 && m <= k.zm_levels) k.zmap_bytes = 4u * (g.zm_off[m] + g.zm_dim[m] * g.zm_dim[m] * g.zm_rw[m]);
    }
    // low byte: 0 default, 1 per-lane gathers; the other variant bits of vct_variants.h
    if ((a->variant & 0xfe) != 0 || (a->variant & kVarRetired) != 0) return hipErrorInvalidValue;
    uint32_t nlt = tiles_for_rank(a->width, a->height, (uint32_t)k.rank, world);
    if (nlt == 0) return hipSuccess;
    const bool counting = k.steps_px || k.steps_total || k.texels_total;
    // Default variant: the form (bits 0x1000000 / 0x2000000 force union / occupancy) and,
    // for a one-rank full frame, the ray order (0x8000 forces reordering, 0x4000000 screen
    // order) that the bits leave open are chosen by the tuner (k4_form).  Other variants:
    // reordering only when 0x8000 asks for it.
    const bool deflt = (a->variant & 0xff) == 0;
    const bool can_reorder = world == 1 && !k.compact;
    const bool cnt_form = counting || (a->variant & kVarCountingForm);
    int cand = 0;
    hipEvent_t* ev = nullptr;
    {
        int forms[2], nf = 0, orders[2], no = 0;
        if (a->variant & VCT_VARIANT_FORCE_UNION) forms[nf++] = 0;
        else if (a->variant & VCT_VARIANT_FORCE_OCCUPANCY) forms[nf++] = 1;
        else { forms[nf++] = 0; forms[nf++] = 1; }
        if (!can_reorder || (a->variant & VCT_VARIANT_SCREEN_ORDER)) orders[no++] = 0;
        else if ((a->variant & VCT_VARIANT_REORDER) || !deflt) orders[no++] = (a->variant & VCT_VARIANT_REORDER) ? 1 : 0;
        else { orders[no++] = 0; orders[no++] = 1; }
        if (deflt) {
            int cands[4], n = 0;
            for (int o = 0; o < no; ++o)
                for (int f = 0; f < nf; ++f) cands[n++] = forms[f] | orders[o] << 1;
            // FNV-1a over the workload: not the buffers, the scene or the counters (a changed
            // scene or G-buffer under the same key is caught by the drift watch)
            uint64_t key = 1469598103934665603ull;
            for (uint64_t v : {(uint64_t)a->width, (uint64_t)a->height, (uint64_t)k.rank, (uint64_t)k.world,
                               (uint64_t)k.compact, (uint64_t)c->cfg.n_diffuse, (uint64_t)k.spec_on, (uint64_t)g.n,
                               (uint64_t)(a->variant & 0x7ffff00u)})
                key = (key ^ v) * 1099511628211ull;
            cand = k4_form(c, key, cands, n, !cnt_form, &ev);
        } else {
            cand = orders[0] << 1;
        }
    }
    if (ev && hipEventRecord(ev[0], c->stream) != hipSuccess) ev = nullptr;
    if (cand & 2) {
        // ray reordering (full frame, one rank): waves take 64 consecutive entries of the
        // sorted pixel list; nlt counts 64-wave units of it instead of 64x64 tiles
        // the specular part (split launches) gets its own order by cell and cone aperture
        hipError_t e = launch_reorder(c, a, &k.perm, (k.split && k.spec_on && !(a->variant & kVarOnePerm)) ? &k.perm_spec : nullptr);
        if (e != hipSuccess) return e;
        nlt = (k.npx + 64u * 64u - 1u) / (64u * 64u);
    }
    uint32_t blocks = nlt * 16;
    if (k.split && k.nd > 1 && ((a->variant & 0x400) || (!(a->variant & 0x800) && blocks <= kSplit3MaxBlocks))) {
        // ndp diffuse parts + the specular part (ndp = 2 unless variant bits 20-23 ask for
        // more); hand-over scratch [part | cones nd_chunk..nd-1] per output pixel + flags
        uint32_t ndp = (a->variant >> 20) & 0xfu;
        ndp = ndp < 2u ? 2u : (ndp > (uint32_t)k.nd ? (uint32_t)k.nd : ndp);
        const uint32_t chunk = ((uint32_t)k.nd + ndp - 1u) / ndp;
        k.nd_chunk = (int)chunk;
        k.ndp = (int)(((uint32_t)k.nd + chunk - 1u) / chunk);   // no empty part
        const size_t npx = k.compact ? (size_t)nlt * VCT_TILE * VCT_TILE : (size_t)a->width * a->height;
        const size_t fbytes = (size_t)blocks * 4 * sizeof(unsigned);
        bool fresh = false;                                  // flags: zeroed when allocated, then
        void* fp = nullptr;                                  // reset by the kernel after each hand-over
        void* sp = nullptr;
        hipError_t e = k4_scratch(c, kScFlags, fbytes, &fp, &fresh);
        if (e != hipSuccess) return e;
        if (fresh && (e = hipMemsetAsync(fp, 0, fbytes, c->stream)) != hipSuccess) return e;
        if ((e = k4_scratch(c, kScHand, (size_t)(1 + k.nd - k.nd_chunk) * npx * sizeof(float4), &sp, nullptr)) !=
            hipSuccess)
            return e;
        k.split = 2;
        k.sc_flag = (unsigned*)fp;
        k.sc_part = (float4*)sp;
        k.sc_cone = k.sc_part + npx;
        k.sc_px = npx;
    }
    const uint32_t nparts = k.split == 2 ? (uint32_t)k.ndp + 1u : 1u + (uint32_t)k.split;
    blocks *= nparts * 4u;                       // one wave (8x8 block) per workgroup
    if (((a->variant >> 16) & 0xf) == 0) {
        // default XCD chunk: whole 64x64 tiles (64 waves) for full frames; 64x16 strips
        // for the small launches of a multi-GPU rank (measured: 1080p 1.60 -> 1.44 ms,
        // 4K 6.91 -> 6.15 ms, one rank of 8: 0.288 -> 0.265 ms)
        k.xcd_g = blocks / nparts >= 16384u ? 64 : 16;
    }
    // longest-first dispatch for the timed launches of a settled default workload (not
    // while its candidates are being timed), from the durations its previous launch recorded;
    // only for launches of at most kLptMaxGenerations generations of waves (a multi-GPU
    // rank's share) that do not overlap another frame: a large launch balances its own tail
    // and a concurrent frame fills it (measured: C3 frame +2 %, pipelined +2 %, one rank of 4
    // -6 %, of 8 -3 %)
    if (!c->n_cu && hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess)
        c->n_cu = 0;
    const bool lpt_size = c->n_cu > 0 && blocks <= (uint32_t)c->n_cu * 4u * kOccWaves * kLptMaxGenerations;
    const uint32_t per_class = (blocks + 7u) / 8u;   // units of residue class 0, the largest
    if (deflt && !cnt_form && !(a->variant & kVarNoLpt) && c->k4tune.cur >= 0 && !c->k4_dbg_order && !c->k4_dbg_dur &&
        per_class <= kLptMaxPerClass && !c->k4tune.multi && (lpt_size || (a->variant & kVarLptAll))) {
        K4Tuner::Entry& te = c->k4tune.e[c->k4tune.cur];
        if (te.chosen >= 0) {
            if (te.hist_cap < blocks) {
                if (te.hist) {
                    // a launch on any stream may still write it (the durations are shared by the
                    // streams; only an entry taken over by a larger workload gets here): retired,
                    // freed with the context -- no device-wide wait in the launch path
                    c->k4tune.retired.push_back(te.hist);
                    te.hist = nullptr;
                    te.hist_cap = 0;
                }
                // the first buffer covers every launch the default rule dispatches longest first
                const uint32_t cap = blocks > (uint32_t)c->n_cu * 4u * kOccWaves * kLptMaxGenerations
                                         ? blocks : (uint32_t)c->n_cu * 4u * kOccWaves * kLptMaxGenerations;
                hipError_t e = hipMalloc((void**)&te.hist, (size_t)cap * sizeof(uint32_t));
                if (e != hipSuccess) return e;
                te.hist_cap = cap;
                te.hist_ok = false;
            }
            if (te.hist_units != blocks || te.hist_cand != cand) te.hist_ok = false;
            if (te.hist_ok) {
                void* op = nullptr;
                hipError_t e = k4_scratch(c, kScOrder, (size_t)blocks * sizeof(uint32_t), &op, nullptr);
                if (e != hipSuccess) return e;
                if ((a->variant & kVarLptSort) || per_class > (uint32_t)kLptRounds * 1024u)
                    hipLaunchKernelGGL(k4_lpt_order, dim3(8), dim3(1024), per_class, c->stream,
                                       (const uint32_t*)te.hist, blocks, (uint32_t*)op);
                else
                    hipLaunchKernelGGL(k4_lpt_bands, dim3(8), dim3(1024), 0, c->stream, (const uint32_t*)te.hist,
                                       blocks, (uint32_t*)op);
                k.order = (const uint32_t*)op;
                ++c->k4_lpt_launches;
            }
            k.dur = te.hist;
            te.hist_units = blocks;
            te.hist_cand = cand;
            te.hist_ok = true;
        }
    }
    // O32 instantiations need every level below 4 GiB: n <= 512
    const bool o32 = g.n <= 512;
#define VCT_K4(BRICK, MINW, UNION, CNT)                                                                 \
    do {                                                                                               \
        if (k.split == 2) {                                                                            \
            if (o32) hipLaunchKernelGGL((k4_trace<BRICK, MINW, UNION, true, true, CNT>), dim3(blocks), dim3(64), 0, c->stream, k); \
            else hipLaunchKernelGGL((k4_trace<BRICK, MINW, UNION, false, true, CNT>), dim3(blocks), dim3(64), 0, c->stream, k);   \
        } else if (o32) hipLaunchKernelGGL((k4_trace<BRICK, MINW, UNION, true, false, CNT>), dim3(blocks), dim3(64), 0, c->stream, k); \
        else hipLaunchKernelGGL((k4_trace<BRICK, MINW, UNION, false, false, CNT>), dim3(blocks), dim3(64), 0, c->stream, k);    \
    } while (0)
    switch (a->variant & 0xff) {   // 0 default; 1 per-lane gathers
        case 1: VCT_K4(false, 1, true, true); break;
        default: {
            // 0x4000: the counting form without counters; the form is the candidate's bit 0
            const int form = cand & 1;
            if (cnt_form) {
                if (form) VCT_K4(true, kOccWaves, false, true);
                else VCT_K4(true, kUnionWaves, true, true);
            } else {
                if (form) VCT_K4(true, kOccWaves, false, false);
                else VCT_K4(true, kUnionWaves, true, false);
            }
            if (ev) (void)hipEventRecord(ev[1], c->stream);
            K4Tuner& T = c->k4tune;
            if (deflt && !cnt_form && T.multi && (T.prev_end || hipEventCreateWithFlags(&T.prev_end,
                                                                          hipEventDisableTiming) == hipSuccess))
                (void)hipEventRecord(T.prev_end, c->stream);
        }
    }
#undef VCT_K4
    return hipGetLastError();
}

}  // namespace vct

// Test / tool hook (not part of include/vct.h): the following launches trace unit order[i]
// in workgroup i and record each unit's duration into dur (device pointers, null = off).
extern "C" int vct_debug_k4_sched(vct_ctx* c, const uint32_t* order, uint32_t* dur) {
    if (!c) return -1;
    c->k4_dbg_order = order;
    c->k4_dbg_dur = dur;
    return 0;
}

// Test hook: the number of K4 launches of this context dispatched in a longest-first order.
extern "C" long long vct_debug_k4_lpt_launches(const vct_ctx* c) { return c ? (long long)c->k4_lpt_launches : -1; }

#if defined(VCT_DEBUG_CLOCK) || defined(VCT_DEBUG_WAVES)
extern "C" int vct_debug_waves(unsigned long long* out, int n) {   // out[n][3]; n <= 1 << 18
    if (n > kDbgWaves) n = kDbgWaves;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(vct_dbg_wave), sizeof(unsigned long long) * 3 * n) == hipSuccess ? n : -1;
}
#endif
#if defined(VCT_DEBUG_COUNTERS) || defined(VCT_DEBUG_CLOCK)
extern "C" int vct_debug_counters(unsigned long long* out, int reset) {   // out[56]: 32 counters, 8 clocks, 16 more counters
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(vct_dbg_ctr), sizeof(unsigned long long) * 32) != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out + 40, HIP_SYMBOL(vct_dbg_ctr), sizeof(unsigned long long) * 16,
                            sizeof(unsigned long long) * 32) != hipSuccess)
        return -1;
    if (hipMemcpyFromSymbol(out + 32, HIP_SYMBOL(vct_dbg_time), sizeof(unsigned long long) * 8) != hipSuccess)
        return -1;
    if (reset) {
        unsigned long long z[48] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(vct_dbg_ctr), z, sizeof z) != hipSuccess) return -1;
        if (hipMemcpyToSymbol(HIP_SYMBOL(vct_dbg_time), z, sizeof(unsigned long long) * 8) != hipSuccess) return -1;
    }
    return 0;
}
#endif
