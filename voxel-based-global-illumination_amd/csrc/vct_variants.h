// vct_variants.h — A/B experiment switches of the K4 launch (vct_trace_args.variant).
//
// NOT part of the include/vct.h interface: the public bits are VCT_VARIANT_REORDER,
// VCT_VARIANT_FORCE_UNION / _OCCUPANCY and VCT_VARIANT_SCREEN_ORDER.  Every switch
// below gives bit-identical outputs and step counts (tests/test_parity_gpu.py
// test_trace_variants_bitexact); they exist for the measurements in DESIGN.md §5.
//
//   low byte   0 LDS bricks (default), 1 per-lane gathers, 2 bricks without the
//              four-face union, 3 row-major lanes
//   0x100      no specular step tables
//   0x200      all cones in one workgroup (no cone split)
//   0x400      three cone parts (two diffuse + specular), 0x800 two parts
//   0x1000     four waves per workgroup
//   0x2000     specular part dispatched first
//   0x4000     the counting form without counters
//   bits 16-19 XCD map: 0 default, 1 contiguous runs, 2..6 chunks of 1/4/16/64/256 units
//   bits 20-23 diffuse parts of the three-part split (2 default)
#pragma once
#include "../../include/vct.h"

namespace vct {
constexpr uint32_t kVarGathers = 0x01u, kVarNoUnion = 0x02u, kVarRowMajor = 0x03u;
constexpr uint32_t kVarNoSpecTables = 0x100u, kVarNoSplit = 0x200u, kVarThreeParts = 0x400u, kVarTwoParts = 0x800u;
constexpr uint32_t kVarWg4 = 0x1000u, kVarSpecFirst = 0x2000u, kVarCountingForm = 0x4000u;
static_assert(VCT_VARIANT_REORDER == 0x8000u && VCT_VARIANT_FORCE_UNION == 0x1000000u &&
                  VCT_VARIANT_FORCE_OCCUPANCY == 0x2000000u && VCT_VARIANT_SCREEN_ORDER == 0x4000000u,
              "public variant bits");
}  // namespace vct
