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

// MAP 2 (any SPLIT > 1, any grid G = nblocks * SPLIT <= 256): the units in
// part-major order (u = h * nblocks + b) are dealt to the XCDs in contiguous
// runs -- XCD k (the slots s with s mod 8 == k) takes units [off_k, off_k +
// c_k), c_k = its slot count -- so each XCD's L2 serves one column part of x
// (C3, 3 parts of 85 blocks: six XCDs hold one part, two hold two) instead of
// all of x.  The parts of a block then sit on different XCDs (the combine
// hand-off is placement-independent, csrc/combine.h).
constexpr void vc_unit_map2(uint32_t slot, uint32_t G, uint32_t nblocks, uint32_t& b, uint32_t& h) {
  const uint32_t k = slot % 8, j = slot / 8;
  uint32_t off = 0;
  for (uint32_t q = 0; q < k; ++q) off += (G - q + 7) / 8;  // slots on XCD q: ceil((G - q) / 8)
  const uint32_t u = off + j;
  h = u / nblocks;
  b = u % nblocks;
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
