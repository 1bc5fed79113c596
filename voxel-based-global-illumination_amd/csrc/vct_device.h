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

__device__ __forceinline__ float dot3(float ax, float ay, float az, float bx, float by, float bz) {
    return (ax * bx + ay * by) + az * bz;
}

// 64-lane wave sum (wave64 on CDNA: 6 butterfly steps)
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

}  // namespace vct
