// Dispatch slot -> vcache work unit (row block b, column part h) under XCD-
// aware placement (MAP 1), shared by k_vcache (csrc/vcache.hip) and its CPU
// replay (tools/vc_sim.cpp); constexpr, so callable from host and device.
//
// Workgroups are placed round-robin over the 8 XCDs (slot i -> XCD i % 8).
//   MAP 0 (product, inline in k_vcache; restated here as vc_unit_map0 for
//          the replay): the parts of one block are 8 slots apart -- one XCD.
//   MAP 1, SPLIT 2: XCDs 0-3 take column half 0, XCDs 4-7 half 1.
//   MAP 1, SPLIT 4: XCDs 2h and 2h+1 take column part h, so each XCD's L2
//                   serves one quarter of x (2 MiB on C3).
// Each is a bijection of [0, nblocks * SPLIT) onto the units; MAP 1 applies
// only when nblocks divides evenly (vc_map1_applies), else MAP 0 runs.
#pragma once

#include <algorithm>
#include <cstdint>

namespace hipspmv {

template <int SPLIT>
constexpr bool vc_map1_applies(uint32_t nblocks) {
  return (SPLIT == 2 && nblocks % 4 == 0) || (SPLIT == 4 && nblocks % 2 == 0);
}

template <int SPLIT>
constexpr void vc_unit_map1(uint32_t slot, uint32_t& b, uint32_t& h) {
  const uint32_t grp = slot % 8;
  h = grp / (8 / SPLIT);
  b = (slot / 8) * (8 / SPLIT) + grp % (8 / SPLIT);
}

template <int SPLIT>
constexpr void vc_unit_map0(uint32_t slot, uint32_t nblocks, uint32_t& b, uint32_t& h) {
  if (SPLIT == 1) {
    b = slot;
    h = 0;
    return;
  }
  const uint32_t g = slot / (8 * SPLIT), rem = slot % (8 * SPLIT);
  const uint32_t nbg = std::min(8u, nblocks - g * 8);
  h = rem / nbg;
  b = g * 8 + rem % nbg;
}

}  // namespace hipspmv
