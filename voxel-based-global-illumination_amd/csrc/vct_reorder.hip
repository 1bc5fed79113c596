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
// Reordering: a key per pixel = the Morton code of the level-0 voxel holding its cone
// origin o = (P - g0) / h + n (the same binary32 sequence as K4), background pixels
// after every valid one; a device radix sort (rocPRIM) of (key, pixel) pairs; K4 then
// reads lane j of wave w from pixel perm[64 w + j] and writes its outputs back to that
// pixel.  Cones of one wave start in a few neighbouring voxels, so their footprints
// share bricks and cache lines.  Every pixel runs exactly the arithmetic it runs
// without the reordering, so outputs and step counts are bit-identical (tested).
#include <rocprim/device/device_radix_sort.hpp>

#include "vct_internal.h"

namespace vct {
namespace {

__device__ __forceinline__ uint32_t spread3(uint32_t v) {   // 10 bits -> every third bit
    v &= 0x3ffu;
    v = (v | (v << 16)) & 0x030000ffu;
    v = (v | (v << 8)) & 0x0300f00fu;
    v = (v | (v << 4)) & 0x030c30c3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}

__global__ void __launch_bounds__(256) k_reorder_keys(const float4* __restrict__ pos, const float4* __restrict__ nrm,
                                                      uint32_t npx, float g0x, float g0y, float g0z, float inv_h,
                                                      int n, uint32_t* __restrict__ keys,
                                                      uint32_t* __restrict__ vals) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= npx) return;
    const float4 P = pos[i];
    uint32_t key = 1u << 30;                 // background: after every valid pixel
    if (P.w != 0.0f) {
        const float4 N = nrm[i];
        const float ox = (P.x - g0x) * inv_h + N.x;   // the cone origin of K4 (level-0 voxel units)
        const float oy = (P.y - g0y) * inv_h + N.y;
        const float oz = (P.z - g0z) * inv_h + N.z;
        const auto cell = [n](float q) {
            const float f = floorf(q);
            return (uint32_t)(f < 0.0f ? 0 : (f > (float)(n - 1) ? n - 1 : (int)f));
        };
        key = spread3(cell(ox)) | (spread3(cell(oy)) << 1) | (spread3(cell(oz)) << 2);
    }
    keys[i] = key;
    vals[i] = i;
}

}  // namespace

hipError_t launch_reorder(vct_ctx* c, const vct_trace_args* a, const uint32_t** perm) {
    const Grid& g = c->grid;
    const uint32_t npx = a->width * a->height;
    const size_t pairs = (size_t)npx * sizeof(uint32_t);
    size_t tmp_bytes = 0;
    hipError_t e = rocprim::radix_sort_pairs(nullptr, tmp_bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                             (const uint32_t*)nullptr, (uint32_t*)nullptr, npx, 0, 31, c->stream);
    if (e != hipSuccess) return e;
    void* kv = nullptr;   // [keys in | keys out | values in | values out]
    void* tmp = nullptr;
    if ((e = k4_scratch(c, kScKeys, 4 * pairs, &kv, nullptr)) != hipSuccess) return e;
    if ((e = k4_scratch(c, kScSort, tmp_bytes ? tmp_bytes : 1, &tmp, nullptr)) != hipSuccess) return e;
    uint32_t* keys_in = (uint32_t*)kv;
    uint32_t* keys_out = keys_in + npx;
    uint32_t* vals_in = keys_out + npx;
    uint32_t* vals_out = vals_in + npx;
    hipLaunchKernelGGL(k_reorder_keys, dim3((npx + 255) / 256), dim3(256), 0, c->stream,
                       (const float4*)a->pos4, (const float4*)a->nrm4, npx, g.g0[0], g.g0[1], g.g0[2], g.inv_h,
                       (int)g.n, keys_in, vals_in);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // bits 0..29: the Morton code (n <= 1024), bit 30: background
    e = rocprim::radix_sort_pairs(tmp, tmp_bytes, keys_in, keys_out, vals_in, vals_out, npx, 0, 31, c->stream);
    if (e != hipSuccess) return e;
    *perm = vals_out;
    return hipSuccess;
}

}  // namespace vct
