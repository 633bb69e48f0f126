// Device helpers shared by the HIPSpMV kernels (internal).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace hipspmv {

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

// acc + a*b with the product rounded (f64) / truncated mod 2^64 (u64) before
// the add -- never fused -- as SoftwareSpMV.cpp:62 computes it on x86.
template <typename T>
__device__ __forceinline__ T madd(T acc, T a, T b) {
#pragma clang fp contract(off)
  const T p = a * b;
  return acc + p;
}

// Loads the compiler's waitcnt pass does not see (CX == 2 / LD == 2 rings):
// hipcc (ROCm 7.2) merges the pending-load state pessimistically at a loop
// header and emits s_waitcnt vmcnt(0) there -- draining a DE-deep register
// ring once per unrolled group (tools probe: a 4-slot ring gets vmcnt(0) at
// the header and vmcnt(3) elsewhere).  Loads issued by inline asm are
// invisible to that pass; the kernel then waits with explicit, exact counts
// (vmcnt is in order for loads on gfx9).  Only the ring's own loads may be in
// flight between a load and its wait for the counts to hold.
__device__ __forceinline__ uint32_t ald_u32(const uint32_t* p) {
  uint32_t r;
  asm volatile("global_load_dword %0, %1, off" : "=v"(r) : "v"(p) : "memory");
  return r;
}
template <typename T>
__device__ __forceinline__ T ald_64(const T* p) {
  uint64_t r;
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
  return __builtin_bit_cast(T, r);
}
__device__ __forceinline__ u64x2 ald_128(const void* p) {
  u64x2 r;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
  return r;
}
// Write-through (sc1) 16-byte store / load through a buffer descriptor: the
// hand-off accesses of the column-part combine (MI355X_MICROARCH.md, Valid
// forms, table row 1: every handed-off byte stored and loaded sc1; aux 16 =
// sc1, cdna_hip_programming.md Guideline 16 R1).  Builtins, not inline asm:
// the compiler counts them in its waits and keeps their data registers until
// the store has read them.  `base` must be wave-uniform; offsets in bytes.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void st_128_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off, u64x2 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, (int)off, 0, 16);
}
__device__ __forceinline__ u64x2 ld_128_sc1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(u64x2, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 16));
}
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt field");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ uint64_t sld_64(const void* p) {  // scalar (SMEM, lgkmcnt) load of a uniform address
  uint64_t r;
  asm volatile("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r) : "s"(p) : "memory");
  return r;
}
__device__ __forceinline__ uint32_t sld_32(const void* p) {
  uint32_t r;
  asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r) : "s"(p) : "memory");
  return r;
}

}  // namespace hipspmv
