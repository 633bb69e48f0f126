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

}  // namespace hipspmv
