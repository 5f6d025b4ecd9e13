// mck_common.hpp -- small wave-level helpers shared by the CRC and XXH3
// drivers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mck {

typedef unsigned int span_u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const span_u32x4 span_gbl_u32x4_t;
// 16-byte load through a global (address_space(1)) pointer: a global_load
// (vmcnt-ordered), not a flat_load; any byte address (the hardware splits
// misaligned accesses).
//
// NT = non-temporal ("nt" bit): every span byte is read exactly once.  It
// pays only when each load INSTRUCTION reads contiguous bytes (the XXH3 row
// layout: +3-4 % at 4 KiB, same-process A/B); the CRC layout, where one
// instruction touches 16 B of every 64 B and the next three instructions
// the rest of the same lines, drops from 5.66 to 3.77 TB/s with nt (the
// lines are not kept for the sibling loads), so CRC loads use the default
// policy.
template <bool NT>
__device__ __forceinline__ uint4 span_load16(uint64_t addr) {
  span_u32x4 v;
  if (NT)
    v = __builtin_nontemporal_load(reinterpret_cast<span_gbl_u32x4_t*>(addr));
  else
    v = *reinterpret_cast<span_gbl_u32x4_t*>(addr);
  return make_uint4(v.x, v.y, v.z, v.w);
}

// 16 bytes at ANY byte address through a vector load, also when the address
// is wave-uniform: for a uniform address the compiler may pick s_load, and
// scalar loads are dword-granular (they drop the low two address bits) --
// a misaligned uniform 16-byte load then reads the wrong bytes.  The empty
// asm makes the address a VGPR value.
// A value every lane holds, as the scalar the compiler can branch on.
__device__ __forceinline__ uint32_t rfl_u32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

__device__ __forceinline__ uint4 vload16_any(uint64_t addr) {
  asm volatile("" : "+v"(addr));
  return span_load16<false>(addr);
}

// a ^ b ^ c in one gfx950 v_bitop3_b32 (truth table 0x96): the checksum
// kernels are VALU-bound, and XOR trees are a large part of their VALU.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint64_t xor3_64(uint64_t a, uint64_t b, uint64_t c) {
  return ((uint64_t)xor3((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32)) << 32) |
         xor3((uint32_t)a, (uint32_t)b, (uint32_t)c);
}

// v_readlane returns int: widen through uint32_t, never sign-extend.
__device__ __forceinline__ uint32_t readlane_u32(uint32_t v, uint32_t k) {
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), static_cast<int>(k)));
}
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, uint32_t k) {
  return ((uint64_t)readlane_u32((uint32_t)(v >> 32), k) << 32) | (uint64_t)readlane_u32((uint32_t)v, k);
}

__device__ __forceinline__ uint64_t readfirstlane_u64(uint64_t v) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32)) << 32) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
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
