// vct_variants.h — A/B switches of the K4 launch (vct_trace_args.variant).
//
// NOT part of the include/vct.h interface: the public bits are VCT_VARIANT_REORDER,
// VCT_VARIANT_FORCE_UNION / _OCCUPANCY and VCT_VARIANT_SCREEN_ORDER.  Every switch
// below gives bit-identical outputs and step counts (tests/test_parity_gpu.py
// test_trace_variants_bitexact); they exist for the measurements in DESIGN.md §5.
// None of them adds a compiled kernel beyond variant 1's per-lane gathers.
//
//   low byte   0 LDS bricks (default), 1 per-lane gathers
//   0x100      no specular step tables
//   0x200      all cones in one workgroup (no cone split)
//   0x400      three cone parts (two diffuse + specular), 0x800 two parts
//   0x2000     split into parts (0x400 / small launches): the specular part first in
//              blockIdx order (longest waves dispatched first; round 5 re-measures it with
//              finer diffuse parts, bits 20-23)
//   0x4000     the counting form without counters
//   bits 16-19 XCD map: 0 default, 1 contiguous runs, 2..6 chunks of 1/4/16/64/256 units
//   bits 20-23 diffuse parts of the three-part split (2 default)
//   0x10000000 longest-first dispatch for settled launches of any size (default: launches
//              of at most four generations of waves); never for launches that overlap
//              another frame on a second stream (the order scratch is shared by the streams)
//   0x20000000 no longest-first dispatch (units in blockIdx order)
//   0x40000000 ray reordering: one order for every cone part (no specular order)
//   0x80000000 longest-first dispatch as a full bucket sort (default: four stable bands)
//
// Retired in round 4 (measured and not kept; the launch returns an
// error for them): low byte 2 (bricks without the four-face union, superseded by the
// occupancy form), 3 (row-major lanes), 0x1000 (four waves per workgroup).
#pragma once
#include "../../include/vct.h"

namespace vct {
constexpr uint32_t kVarGathers = 0x01u;
constexpr uint32_t kVarNoSpecTables = 0x100u, kVarNoSplit = 0x200u, kVarThreeParts = 0x400u, kVarTwoParts = 0x800u;
constexpr uint32_t kVarCountingForm = 0x4000u;
constexpr uint32_t kVarSpecFirst = 0x2000u;
constexpr uint32_t kVarLptAll = 0x10000000u;
constexpr uint32_t kVarNoLpt = 0x20000000u;
constexpr uint32_t kVarOnePerm = 0x40000000u;
constexpr uint32_t kVarLptSort = 0x80000000u;
constexpr uint32_t kVarRetired = 0x1000u;
static_assert(VCT_VARIANT_REORDER == 0x8000u && VCT_VARIANT_FORCE_UNION == 0x1000000u &&
                  VCT_VARIANT_FORCE_OCCUPANCY == 0x2000000u && VCT_VARIANT_SCREEN_ORDER == 0x4000000u,
              "public variant bits");
}  // namespace vct
