// k_wgather: windowed-gather SpMV for wide x.
//
// When x is too wide for the LDS vector cache to pay (C4/C5: 16M columns,
// x = 128 MB; every row block would have to stream all of it), x stays in
// global memory and is gathered per nonzero -- but in column WINDOWS: the
// entries of row block b that fall into window w (2^CB columns, 512 KiB of x)
// form segment (b, w) of the vcache layout (csrc/plan.cpp build_vcache with
// kWgWindow; row runs sorted by x line, sort_segments_by_line, so the lanes
// of a gather that hit one line are neighbours), and every workgroup walks
// the windows in the same order, so the whole chip gathers from one
// L2-resident window at a time instead of from all 128 MB.  The row block's y accumulators live in LDS as in k_vcache;
// within a window each row is one run processed by one lane in column order,
// windows are separated by a barrier, so every row is summed in ascending
// column order from y_in or +0.0: ORDERED, bit-identical to SoftwareSpMV.
//
// Bytes per launch: 12 per nonzero (entries) + 8 per distinct (block, column)
// gather line touched + 8 per row of y (+8 for beta 1).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "combine.h"
#include "device_common.h"
#include "hipspmv_internal.h"
#include "kernels.h"

namespace hipspmv {

// MSK: entry loads masked past each step's segment (a buffer descriptor over
// the block's entries; an out-of-range lane issues no request), so a register
// window wider than the mean segment costs no over-read -- the launcher sizes
// EPT to the layout's longest segment and no step takes the slow path.
//
// PARTS 2 (kWgSplit, FAST): work unit (b, h) walks the windows of column part
// h only, from +0.0 (part 1) or y_in (part 0), and the two partials of block b
// are combined p0 + p1 by owner_combine.  Workgroup w runs on XCD w mod 8:
// units are numbered so that part 0 fills XCDs 0-3 and part 1 XCDs 4-7 (a
// grid tail of fewer than 8 units alternates the parts), so each XCD's L2
// fetches only its half of x.
// (The body is shared by the kernels k_wgather, PARTS 1, and k_wgather_split,
// PARTS 2, so each form has its own symbol in a profile.)
template <typename T, int CB, int DE, int EPT, bool NTE, bool MSK, int PARTS>
__device__ __forceinline__ void wgather_body(const uint32_t* __restrict__ seg, const uint32_t* __restrict__ ecode,
                                             const T* __restrict__ evals, const T* __restrict__ x,
                                             const T* __restrict__ y_in, T* __restrict__ y_out, uint32_t rows,
                                             uint32_t rows_per_block, uint32_t npanels, uint32_t npad, uint32_t last,
                                             int beta, uint32_t b0, T* __restrict__ partial,
                                             uint32_t* __restrict__ tickets, uint32_t nblocks, uint32_t nt_from,
                                             int xmap) {
#pragma clang fp contract(off)
  static_assert(PARTS == 1 || PARTS == 2, "one or two column parts");
  constexpr int VT = kVcThreads;
  constexpr uint32_t W = 1u << CB, CMASK = W - 1, RMASK = (1u << (30 - CB)) - 1;
  constexpr int VR = 1 << (30 - CB);
  __shared__ T ylds[VR];
  __shared__ uint32_t segl[kWgWindow.segmax];
  const int t = threadIdx.x;
  uint32_t b = b0 + blockIdx.x, h = 0;  // this launch's blocks start at b0 (launch chunks, kWgChunk)
  if constexpr (PARTS == 2) {
    // xmap 1 (option wgather_map, diagnostic): the halves alternate, h = u mod 2, so every XCD runs
    // units of both halves -- the A/B of the XCD placement
    const uint32_t u = blockIdx.x, full = xmap ? 0u : gridDim.x & ~7u;
    if (u < full) {
      h = (u & 7u) >> 2;
      b = b0 + (u >> 3) * 4 + (u & 3u);
    } else {
      h = (u - full) & 1u;
      b = b0 + full / 2 + (u - full) / 2;
    }
  }
  const uint32_t r0 = b * rows_per_block;
  if (r0 >= rows) return;  // never with a vcache_grid_ok geometry
  const uint32_t nr = min(rows_per_block, rows - r0);
  const uint32_t* sp = seg + ((size_t)b * PARTS + h) * (npad + 1);
  // this unit's windows: [pf, pf + nloc) (PARTS 1: all of them)
  const uint32_t pf = vc_part_first(h, npanels, PARTS), nloc = vc_part_first(h + 1, npanels, PARTS) - pf;
  if ((uint32_t)t <= npad) segl[t] = sp[t];
  for (uint32_t i = t; i < nr; i += VT) ylds[i] = beta && h == 0 ? y_in[r0 + i] : T(0);
  __syncthreads();

  const uint32_t e0 = __builtin_amdgcn_readfirstlane(segl[0]);
  const uint32_t ne = __builtin_amdgcn_readfirstlane(segl[npad]) - e0;
  const __amdgpu_buffer_rsrc_t dcode = buf_rsrc(ecode + e0, 4 * ne), dvals = buf_rsrc(evals + e0, 8 * ne);
  auto load_e = [&](uint32_t s, uint32_t* c, T* v) {
    const uint32_t beg = segl[min(s, npad)];
    if constexpr (MSK) {
      const uint32_t end = segl[min(s + 1, npad)] - e0;
      auto ld = [&](auto aux_c) {
        constexpr int aux = decltype(aux_c)::value;
#pragma unroll
        for (int j = 0; j < EPT; ++j) {
          const uint32_t q = beg - e0 + t + j * VT;
          const bool in = q < end;
          c[j] = __builtin_amdgcn_raw_buffer_load_b32(dcode, in ? (int)(4 * q) : (int)0x80000000, 0, aux);
          v[j] = __builtin_bit_cast(
              T, __builtin_amdgcn_raw_buffer_load_b64(dvals, in ? (int)(8 * q) : (int)0x80000000, 0, aux));
        }
      };
      // PARTS 2: row blocks b < nt_from keep their entries with the default policy (Infinity-Cache
      // resident across launches), the others non-temporal (wave-uniform branch)
      if (PARTS == 2 && NTE && b < nt_from)
        ld(std::integral_constant<int, 0>{});
      else
        ld(std::integral_constant<int, NTE ? 2 : 0>{});  // nt
      return;
    }
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const uint32_t i = min(beg + t + j * VT, last);  // clamped, validity checked at use
      if (NTE) {  // streamed once: non-temporal, so the gathered x window keeps L2
        c[j] = __builtin_nontemporal_load(ecode + i);
        v[j] = __builtin_nontemporal_load(evals + i);
      } else {
        c[j] = ecode[i];
        v[j] = evals[i];
      }
    }
  };
  auto run = [&](uint32_t i, uint32_t code, T v, T xv, const T* xs) {
    const uint32_t row = (code >> CB) & RMASK;
    T acc = madd(ylds[row], v, xv);
    while (code & kVcMore) {  // several entries of one row in this window (rare)
      ++i;
      code = ecode[i];
      acc = madd(acc, evals[i], xs[code & CMASK]);
    }
    ylds[row] = acc;
  };
  auto apply = [&](uint32_t s, const uint32_t* c, const T* v) {
    const T* xs = x + (size_t)(pf + s) * W;
    const uint32_t beg = segl[s], end = segl[s + 1];
    T xv[EPT];
#pragma unroll
    for (int j = 0; j < EPT; ++j) {  // all gathers first, then the LDS updates
      const bool act = beg + t + j * VT < end && !(c[j] & kVcCont);
      xv[j] = act ? xs[c[j] & CMASK] : T(0);
    }
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const uint32_t q = beg + t + j * VT;
      if (q < end && !(c[j] & kVcCont)) run(q, c[j], v[j], xv[j], xs);
    }
    if (!MSK)  // (masked: the launcher sized EPT to the longest segment)
      for (uint32_t q = beg + EPT * VT + t; q < end; q += VT) {  // beyond the register window
        const uint32_t code = ecode[q];
        if (!(code & kVcCont)) run(q, code, evals[q], xs[code & CMASK], xs);
      }
  };

  uint32_t EC[DE][EPT];
  T EV[DE][EPT];
#pragma unroll
  for (int i = 0; i < DE; ++i) load_e(i, EC[i], EV[i]);
  for (uint32_t base = 0; base < nloc; base += DE) {
#pragma unroll
    for (int i = 0; i < DE; ++i) {
      const uint32_t s = base + i;
      if (s >= nloc) break;
      apply(s, EC[i], EV[i]);
      load_e(s + DE, EC[i], EV[i]);
      __syncthreads();  // window s's y updates before window s+1's
    }
  }
  if constexpr (PARTS == 1) {
    for (uint32_t i = t; i < nr; i += VT) y_out[r0 + i] = ylds[i];
  } else {  // (segl is free now: its first words are the combine's LDS scratch)
    owner_combine<T, PARTS, VT, (uint32_t)VR>(ylds, segl, partial, tickets + 4 * (size_t)b, b, h, nblocks, nr,
                                              y_out + r0, t);
  }
}

template <typename T, int CB, int DE, int EPT, bool NTE = false, bool MSK = false>
__global__ __launch_bounds__(kVcThreads) void k_wgather(const uint32_t* __restrict__ seg,
                                                         const uint32_t* __restrict__ ecode,
                                                         const T* __restrict__ evals, const T* __restrict__ x,
                                                         const T* __restrict__ y_in, T* __restrict__ y_out,
                                                         uint32_t rows, uint32_t rows_per_block, uint32_t npanels,
                                                         uint32_t npad, uint32_t last, int beta, uint32_t b0) {
  wgather_body<T, CB, DE, EPT, NTE, MSK, 1>(seg, ecode, evals, x, y_in, y_out, rows, rows_per_block, npanels, npad,
                                            last, beta, b0, nullptr, nullptr, 0, 0, 0);
}

template <typename T, int CB, int DE, int EPT, bool NTE = false, bool MSK = false>
__global__ __launch_bounds__(kVcThreads) void k_wgather_split(
    const uint32_t* __restrict__ seg, const uint32_t* __restrict__ ecode, const T* __restrict__ evals,
    const T* __restrict__ x, const T* __restrict__ y_in, T* __restrict__ y_out, uint32_t rows,
    uint32_t rows_per_block, uint32_t npanels, uint32_t npad, uint32_t last, int beta, uint32_t b0,
    T* __restrict__ partial, uint32_t* __restrict__ tickets, uint32_t nblocks, uint32_t nt_from, int xmap) {
  wgather_body<T, CB, DE, EPT, NTE, MSK, 2>(seg, ecode, evals, x, y_in, y_out, rows, rows_per_block, npanels, npad,
                                            last, beta, b0, partial, tickets, nblocks, nt_from, xmap);
}

// Pipelined form (option vcache_xlane 2; every segment must fit the register
// window, EPT*1024 entries): the entry ring and the x gathers are inline-asm
// loads with exact vmcnt waits (device_common.h), so nothing drains the ring:
// step s issues the gathers of step s+1 (their codes landed DE-1 steps
// earlier) and then the entries of step s+DE, and consumes the gathers issued
// one step before.  Per step, in issue order: G(s+1) [EPT], E(s+DE) [2 EPT].
//   wait E(s+1): younger = steps s+2-DE .. s-1 = (DE-2) * 3 EPT
//   wait G(s)  : younger = E(s-1+DE) + G(s+1) = 3 EPT   (s == 0: G(1) only, EPT)
// Run continuations come from the next lanes of the wave (products formed by
// every lane), or, past the wave, from scalar loads (lgkmcnt).
template <typename T, int CB, int DE, int EPT>
__global__ __launch_bounds__(kVcThreads) void k_wgather_pipe(const uint32_t* __restrict__ seg,
                                                              const uint32_t* __restrict__ ecode,
                                                              const T* __restrict__ evals, const T* __restrict__ x,
                                                              const T* __restrict__ y_in, T* __restrict__ y_out,
                                                              uint32_t rows, uint32_t rows_per_block,
                                                              uint32_t npanels, uint32_t npad, uint32_t last,
                                                              int beta, uint32_t b0) {
#pragma clang fp contract(off)
  constexpr int VT = kVcThreads;
  constexpr uint32_t W = 1u << CB, CMASK = W - 1, RMASK = (1u << (30 - CB)) - 1;
  constexpr int VR = 1 << (30 - CB);
  static_assert(DE >= 2 && DE % 2 == 0, "ring depth: even, the gather buffer alternates");
  __shared__ T ylds[VR];
  __shared__ uint32_t segl[kWgWindow.segmax];
  const int t = threadIdx.x;
  const uint32_t lw = t & 63;
  const uint32_t b = b0 + blockIdx.x;
  const uint32_t r0 = b * rows_per_block;
  if (r0 >= rows) return;  // never with a vcache_grid_ok geometry
  const uint32_t nr = min(rows_per_block, rows - r0);
  const uint32_t* sp = seg + (size_t)b * (npad + 1);
  if ((uint32_t)t <= npad) segl[t] = sp[t];
  for (uint32_t i = t; i < nr; i += VT) ylds[i] = beta ? y_in[r0 + i] : T(0);
  __syncthreads();

  auto load_e = [&](uint32_t s, uint32_t* c, T* v) {  // 2*EPT loads, always issued
    const uint32_t beg = segl[min(s, npad)];
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const uint32_t i = min(beg + t + j * VT, last);
      c[j] = ald_u32(ecode + i);
      v[j] = ald_64(evals + i);
    }
  };
  auto gather = [&](uint32_t s, const uint32_t* c, T* g) {  // EPT loads, always issued (x[0] when idle)
    const uint32_t beg = segl[min(s, npad)], end = segl[min(s + 1, npad)];
    const T* xs = x + (size_t)min(s, npanels - 1) * W;
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const bool ok = s < npanels && beg + t + j * VT < end;
      g[j] = ald_64(ok ? xs + (c[j] & CMASK) : x);
    }
  };
  auto apply = [&](uint32_t s, const uint32_t* c, const T* v, const T* g) {
    const T* xs = x + (size_t)s * W;
    const uint32_t beg = segl[s], end = segl[s + 1];
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const uint32_t q = beg + t + j * VT;
      const uint32_t code = c[j];
      const bool valid = q < end;
      const T p = valid ? v[j] * g[j] : T(0);
      const bool own = valid && !(code & kVcCont);
      const uint32_t row = (code >> CB) & RMASK;
      T acc = own ? ylds[row] + p : T(0);
      bool more = own && (code & kVcMore);
      bool fb = false;
      uint32_t fbi = 0;
      for (uint32_t k = 1; __builtin_amdgcn_ballot_w64(more) != 0; ++k) {
        const T pk = __shfl_down(p, k);
        const uint32_t ck = __shfl_down(code, k);
        if (more) {
          if (lw + k < 64) {
            acc = acc + pk;
            more = (ck & kVcMore) != 0;
          } else {
            fb = true;
            fbi = q + k;
            more = false;
          }
        }
      }
      for (uint64_t m = __builtin_amdgcn_ballot_w64(fb); m; m &= m - 1) {  // rare
        const uint32_t l = (uint32_t)__builtin_ctzll(m);
        uint32_t i = __builtin_amdgcn_readlane(fbi, l);
        const uint64_t ab = __builtin_bit_cast(uint64_t, acc);
        T a = __builtin_bit_cast(T, (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)ab, l) |
                                        ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(ab >> 32), l) << 32));
        uint32_t cd;
        do {
          cd = sld_32(ecode + i);
          const T pv = __builtin_bit_cast(T, sld_64(evals + i)) * __builtin_bit_cast(T, sld_64(xs + (cd & CMASK)));
          a = a + pv;
          ++i;
        } while (cd & kVcMore);
        if (lw == l) acc = a;
      }
      if (own) ylds[row] = acc;
    }
  };

  uint32_t EC[DE][EPT];
  T EV[DE][EPT];
  T G[2][EPT];
#pragma unroll
  for (int i = 0; i < DE; ++i) load_e(i, EC[i], EV[i]);
  vm_wait<0>();
  gather(0, EC[0], G[0]);
  // step 0, peeled: G(0) has only G(1) younger than it
  gather(1, EC[1], G[1]);
  vm_wait<EPT>();
  apply(0, EC[0], EV[0], G[0]);
  load_e(DE, EC[0], EV[0]);
  __syncthreads();
  // steps 1 .. nsteps-1, padded to whole unrolled groups (extra steps do no
  // work but keep their loads), so the loop has no early exit: every path
  // through it issues the same loads, which is what the waits count on
  const uint32_t nsteps = 1 + (npanels - 1 + DE - 1) / DE * DE;
  for (uint32_t base = 1; base < nsteps; base += DE) {
#pragma unroll
    for (int i = 0; i < DE; ++i) {
      const uint32_t s = base + i;  // ring slot (i + 1) % DE, gather buffer (i + 1) & 1
      vm_wait<(DE - 2) * 3 * EPT>();  // E(s+1) landed
      gather(s + 1, EC[(i + 2) % DE], G[i & 1]);
      vm_wait<3 * EPT>();  // G(s) landed
      if (s < npanels) apply(s, EC[(i + 1) % DE], EV[(i + 1) % DE], G[(i + 1) & 1]);
      load_e(s + DE, EC[(i + 1) % DE], EV[(i + 1) % DE]);
      __syncthreads();  // window s's y updates before window s+1's
    }
  }
  vm_wait<0>();
  for (uint32_t i = t; i < nr; i += VT) y_out[r0 + i] = ylds[i];
}

template <typename T, int DE, int EPT, bool NTE, bool MSK, int PARTS>
static void launch_one(const VcacheArgs& a, uint32_t n, uint32_t b0, hipStream_t s) {
  constexpr int CB = kWgWindow.colbits;
  if constexpr (PARTS == 1)
    hipLaunchKernelGGL((k_wgather<T, CB, DE, EPT, NTE, MSK>), dim3(n), dim3(kVcThreads), 0, s, a.seg, a.code,
                       (const T*)a.vals, (const T*)a.x, (const T*)a.y_in, (T*)a.y_out, a.rows, a.rows_per_block,
                       a.npanels, a.npad, a.last, a.beta, b0);
  else
    hipLaunchKernelGGL((k_wgather_split<T, CB, DE, EPT, NTE, MSK>), dim3(2 * n), dim3(kVcThreads), 0, s, a.seg,
                       a.code, (const T*)a.vals, (const T*)a.x, (const T*)a.y_in, (T*)a.y_out, a.rows,
                       a.rows_per_block, a.npanels, a.npad, a.last, a.beta, b0, (T*)a.partial, a.tickets, a.nblocks,
                       a.nt_from, a.map);
}

template <typename T, int PARTS>
static hipError_t launch_wgather_t(const VcacheArgs& a, hipStream_t s) {
  // blocks [b0, b0 + n) per launch: a chunk the chip holds at once walks the x
  // windows together (kWgChunk units); the launches run in stream order
  const uint32_t chunk = a.chunk ? (a.chunk + PARTS - 1) / PARTS : a.nblocks;
  // non-temporal entry loads: PARTS 1 all or none (nt_from 0: all); PARTS 2 the blocks b >= nt_from,
  // chosen at run time inside the NTE forms (nt_from >= nblocks: every block resident)
  const bool nt = PARTS == 1 ? a.nt_from == 0 : true;
  for (uint32_t b0 = 0; b0 < a.nblocks; b0 += chunk) {
    const uint32_t n = a.nblocks - b0 < chunk ? a.nblocks - b0 : chunk;
    if (PARTS == 1 && a.xlane >= 2 && a.max_seg <= 2u * kVcThreads)
      hipLaunchKernelGGL((k_wgather_pipe<T, kWgWindow.colbits, 4, 2>), dim3(n), dim3(kVcThreads), 0, s, a.seg, a.code,
                         (const T*)a.vals, (const T*)a.x, (const T*)a.y_in, (T*)a.y_out, a.rows, a.rows_per_block,
                         a.npanels, a.npad, a.last, a.beta, b0);
    else if (PARTS == 1 && a.xlane >= 2 && a.max_seg <= 4u * kVcThreads)
      hipLaunchKernelGGL((k_wgather_pipe<T, kWgWindow.colbits, 4, 4>), dim3(n), dim3(kVcThreads), 0, s, a.seg, a.code,
                         (const T*)a.vals, (const T*)a.x, (const T*)a.y_in, (T*)a.y_out, a.rows, a.rows_per_block,
                         a.npanels, a.npad, a.last, a.beta, b0);
    else if (nt && a.max_seg <= 2u * kVcThreads)
      launch_one<T, 4, 2, true, true, PARTS>(a, n, b0, s);
    else if (nt && a.max_seg <= 3u * kVcThreads)
      launch_one<T, 4, 3, true, true, PARTS>(a, n, b0, s);
    else if (nt && a.max_seg <= 6u * kVcThreads)
      launch_one<T, 2, 6, true, true, PARTS>(a, n, b0, s);
    else if (nt && a.max_seg <= 9u * kVcThreads)
      launch_one<T, 2, 9, true, true, PARTS>(a, n, b0, s);
    else if (nt)
      launch_one<T, 4, 2, true, false, PARTS>(a, n, b0, s);
    else if constexpr (PARTS == 1)  // (PARTS 2 always takes an NTE form: residency per block at run time)
      launch_one<T, 4, 2, false, false, 1>(a, n, b0, s);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_wgather(int dtype, const VcacheArgs& a, hipStream_t s) {
  // the layout must be kWgWindow's (window width, row-block bound, one part)
  // or kWgSplit's (two parts, with the combine scratch)
  static_assert(kWgSplit.colbits == kWgWindow.colbits && kWgSplit.rows == 1 << (30 - kWgSplit.colbits) &&
                    kWgSplit.panel == kWgWindow.panel,
                "the two-part layout uses the kernel's window and y block");
  const VcGeom& g = a.split == 2 ? kWgSplit : kWgWindow;
  if (!vcache_grid_ok(a.rows, a.cols, a.rows_per_block, a.nblocks, a.npanels, a.part_panels, a.npad, a.panel,
                      a.split, g) ||
      (a.split == 1 && a.part_panels != a.npanels) || (a.split == 2 && (!a.partial || !a.tickets)))
    return hipErrorInvalidValue;
  if (a.split == 2)
    return dtype ? launch_wgather_t<uint64_t, 2>(a, s) : launch_wgather_t<double, 2>(a, s);
  return dtype ? launch_wgather_t<uint64_t, 1>(a, s) : launch_wgather_t<double, 1>(a, s);
}

}  // namespace hipspmv
