// mck_common.hpp -- small wave-level helpers shared by the CRC and XXH3
// drivers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mck {

// v_readlane returns int: widen through uint32_t, never sign-extend.
__device__ __forceinline__ uint32_t readlane_u32(uint32_t v, uint32_t k) {
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), static_cast<int>(k)));
}
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, uint32_t k) {
  return ((uint64_t)readlane_u32((uint32_t)(v >> 32), k) << 32) | (uint64_t)readlane_u32((uint32_t)v, k);
}

// Span tickets: lane 0 takes the next ticket from a workgroup-local LDS
// counter; the value is spread with ds_bpermute, so the compiler treats it
// as per-lane and loads the span's descriptor with VECTOR loads (counted in
// vmcnt, in order with the data loads) rather than scalar loads, whose
// lgkmcnt the next LDS access would drain.  Spans then go to whichever wave
// of the workgroup frees up first: ragged batches stay balanced inside a CU.
template <class P>
__device__ __forceinline__ uint32_t lds_ticket(P ctr) {
  uint32_t t = 0;
  if ((threadIdx.x & 63) == 0) t = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return (uint32_t)__builtin_amdgcn_ds_bpermute(0, (int)t);
}

}  // namespace mck
