// The column-part combine of the split vector-cache kernels (k_vcache with
// SPLIT 3/4, k_vquad): every unit (b, h) of row block b holds the partial y of
// its column part h in LDS; y = p0 + p1 + ... in part order (deterministic).
//
// Owner combines.  The block's row pairs are cut into SPLIT
// shares; unit h owns share h.  It publishes its partials of the other shares
// with write-through (sc1) 16-byte stores, drains, counts each one (one
// agent-scope add per share word), then waits for the SPLIT - 1 publishers of
// its own share, reads their partials (sc1) and writes those y rows
// (MI355X_MICROARCH.md, Valid forms, table row 1).  The parts of a block run
// at once, so every CU moves (SPLIT-1)/SPLIT of its partial out and as much
// in; the last-arriver form (one CU reads every other partial) cost 11.5 us
// of 118 at C3 four parts.
//
// No deadlock without co-residency: the owner's wait is bounded; an owner
// that gives up publishes its own share too and counts it, and the add that
// finds the count at SPLIT - 1 (all SPLIT in) belongs to the unit that
// combines the share -- it has nothing left to wait for.  Every word returns
// to 0 in the launch (the combining unit stores it once all adds are in), and
// no path reads a partial that was not counted.
#ifndef SPMV_AMD_COMBINE_H_
#define SPMV_AMD_COMBINE_H_

#include <hip/hip_runtime.h>

#include "device_common.h"

namespace hipspmv {

// published: the block's SPLIT share words; partial: part o of block b at
// partial + (o * nblocks + b) * VRP; scratch: SPLIT + 2 LDS words no lane
// reads any more; y: the block's first row.  Call from every lane of the
// workgroup after the last write of ylds and a barrier; NOWAIT (test hook)
// makes every owner give up at once.  fallbacks (optional): counts the owners
// that gave up waiting and published their own share (results are exact either
// way; the count only says which path ran).
template <typename T, int SPLIT, int VT, uint32_t VRP, bool NOWAIT = false>
__device__ __forceinline__ void owner_combine(const T* ylds, uint32_t* scratch, T* partial, uint32_t* published,
                                              uint32_t b, uint32_t h, uint32_t nblocks, uint32_t nr, T* y, int t,
                                              uint32_t* fallbacks = nullptr) {
  constexpr uint32_t PAIRS = VRP / 2;
  constexpr uint32_t QP = (PAIRS + SPLIT - 1) / SPLIT;  // row pairs per share
  constexpr int NQ = (QP + VT - 1) / VT;                // per lane
  static_assert(VRP % 2 == 0, "row pairs");
  const u64x2* const yl2 = reinterpret_cast<const u64x2*>(ylds);
  const uint32_t npairs = (nr + 1) / 2;
  const __amdgpu_buffer_rsrc_t mine = buf_rsrc(partial + ((size_t)h * nblocks + b) * VRP, 8 * VRP);
  // y written through (sc1) like the partials: the launch then ends with no dirty y lines in L2, so
  // the next eager launch does not wait for their write-back at the kernel boundary
  const __amdgpu_buffer_rsrc_t yr = buf_rsrc(y, 8 * nr);
  auto pair_of = [&](uint32_t q, int j) { return q * QP + (uint32_t)t + (uint32_t)j * VT; };
  auto in_share = [&](uint32_t q, int j) {
    return (QP % VT == 0 || (uint32_t)t + (uint32_t)j * VT < QP) && pair_of(q, j) < PAIRS;
  };
  auto publish = [&](uint32_t q) {
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      const uint32_t p = pair_of(q, j);
      if (in_share(q, j) && p < npairs) st_128_sc1(mine, 16 * p, yl2[p]);
    }
  };
  auto combine = [&](uint32_t q) {  // y rows of share q = p0 + p1 + ... in part order, own part from LDS
    u64x2 v[SPLIT][NQ];
#pragma unroll
    for (int o = 0; o < SPLIT; ++o) {
      const __amdgpu_buffer_rsrc_t src = buf_rsrc(partial + ((size_t)o * nblocks + b) * VRP, 8 * VRP);
#pragma unroll
      for (int j = 0; j < NQ; ++j) {
        const uint32_t p = min(pair_of(q, j), PAIRS - 1);
        v[o][j] = (uint32_t)o == h ? yl2[p] : ld_128_sc1(src, 16 * p);
      }
    }
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      T a0 = __builtin_bit_cast(T, (uint64_t)v[0][j].x), a1 = __builtin_bit_cast(T, (uint64_t)v[0][j].y);
#pragma unroll
      for (int o = 1; o < SPLIT; ++o) {
        a0 = a0 + __builtin_bit_cast(T, (uint64_t)v[o][j].x);
        a1 = a1 + __builtin_bit_cast(T, (uint64_t)v[o][j].y);
      }
      const uint32_t p = pair_of(q, j);
      if (in_share(q, j)) {  // rows past nr fall outside the descriptor: no store
        typedef unsigned int u32x2c __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2c, a0), yr, (int)(16 * p), 0, 16);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2c, a1), yr, (int)(16 * p + 8), 0, 16);
      }
    }
  };
  auto reset = [&](uint32_t q) {
    if (t == 0) __hip_atomic_store(published + q, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
#pragma unroll
  for (int k = 1; k < SPLIT; ++k) publish((h + k) % SPLIT);  // the other owners' shares
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // lane q != h counts share q; an add that finds SPLIT - 1 is the last of
  // all SPLIT (that share's owner gave up and published too): we combine it
  if ((uint32_t)t < (uint32_t)SPLIT && (uint32_t)t != h)
    scratch[t] = __hip_atomic_fetch_add(published + t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t == 0) {  // the owner's wait for the publishers of share h, bounded (~0.5 ms)
    uint32_t ok = 0;
    for (uint32_t spin = 0; spin < (NOWAIT ? 0u : 1u << 10) && !ok; ++spin) {
      ok = __hip_atomic_load(published + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)SPLIT - 1;
      if (!ok) __builtin_amdgcn_s_sleep(2);
    }
    scratch[SPLIT] = ok;
  }
  __syncthreads();
  uint32_t todo = 0;  // bit q: this unit writes the y rows of share q (workgroup-uniform: LDS words)
#pragma unroll
  for (uint32_t q = 0; q < (uint32_t)SPLIT; ++q)
    if (q != h && scratch[q] == (uint32_t)SPLIT - 1) todo |= 1u << q;
  if (scratch[SPLIT]) {
    todo |= 1u << h;
    reset(h);  // its SPLIT - 1 adds are all in
  } else {
    // a publisher of share h is not running yet (the grid is not all
    // resident): publish our part as well and count it; nobody waits
    publish(h);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
      scratch[SPLIT + 1] = __hip_atomic_fetch_add(published + h, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (fallbacks) __hip_atomic_fetch_add(fallbacks, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (scratch[SPLIT + 1] == (uint32_t)SPLIT - 1) todo |= 1u << h;
  }
#pragma unroll
  for (uint32_t q = 0; q < (uint32_t)SPLIT; ++q) {
    if (!(todo & (1u << q))) continue;
    if (q != h || !scratch[SPLIT]) reset(q);  // all SPLIT adds in
    combine(q);
  }
}

}  // namespace hipspmv

#endif
