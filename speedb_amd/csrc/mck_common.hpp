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

// Byte-balanced contiguous shares of a ragged batch [first, first + count)
// over the grid.  Workgroup b's boundary is the first span whose offset
// reaches b/G of the batch's offset range, searched over S = min(count, 8192)
// evenly spaced samples of the offsets (span k * count / S, one load per
// thread per 1024 samples); "the first sample at or past a target" is
// monotone in the target for ANY offsets, so the shares always partition the
// batch, and they are balanced to ~count/S spans when the offsets grow with
// the bytes (an SST or blob file image).  Each boundary is clamped to within
// `slack` spans of the count-balanced one (the row drivers' descriptor cache
// bounds a share's spans).  Count-balanced shares hand the SST verify mix's
// workgroups up to 1.2x the mean bytes (their end times spread 165-209 us
// over a 1 GiB image).  scratch: 2 x u32 in LDS.  Workgroup-uniform; has
// barriers.
template <class F>
__device__ __forceinline__ uint32_t k_or_count(uint32_t k, uint32_t S, uint32_t count, const F& idx) {
  return k >= S ? count : idx(k);
}
template <class Op, class P>
__device__ __forceinline__ void share_by_bytes(const Op& op, uint32_t first, uint32_t count, uint32_t slack,
                                               P scratch, uint32_t* lo, uint32_t* hi) {
  const uint32_t G = gridDim.x, b = blockIdx.x;
  const uint32_t clo = (uint32_t)((uint64_t)count * b / G), chi = (uint32_t)((uint64_t)count * (b + 1) / G);
  constexpr uint32_t kS = 8192;  // 2^13
  const uint32_t S = count < kS ? count : kS;
  if (S == 0 || G == 1) {
    *lo = clo;
    *hi = chi;
    return;
  }
  if (threadIdx.x < 2) scratch[threadIdx.x] = S;
  __syncthreads();
  const uint64_t o0 = op.off(first), oL = op.off(first + count - 1);
  const uint64_t range = oL > o0 ? oL - o0 : 0;
  const uint64_t tb = o0 + range * b / G, te = o0 + range * (b + 1) / G;
  uint32_t kb = S, ke = S;
  // sample k is span k * count / S: k itself when S = count, else (S = 2^13)
  // a shift (no 64-bit division per sample)
  for (uint32_t k = threadIdx.x; k < S; k += blockDim.x) {
    const uint32_t i = S == count ? k : (uint32_t)(((uint64_t)k * count) >> 13);
    const uint64_t o = op.off(first + i);
    kb = (o >= tb && k < kb) ? k : kb;
    ke = (o >= te && k < ke) ? k : ke;
  }
  if (kb < S) __hip_atomic_fetch_min(&scratch[0], kb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  if (ke < S) __hip_atomic_fetch_min(&scratch[1], ke, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __syncthreads();
  kb = scratch[0];
  ke = scratch[1];
  __syncthreads();  // the scratch may be reused
  const auto clampb = [&](uint32_t x, uint32_t c) {
    const uint32_t a = c > slack ? c - slack : 0u;
    const uint64_t z = (uint64_t)c + slack < count ? (uint64_t)c + slack : count;
    return x < a ? a : x > z ? (uint32_t)z : x;
  };
  const auto idx = [&](uint32_t k) { return S == count ? k : (uint32_t)(((uint64_t)k * count) >> 13); };
  *lo = b == 0 ? 0u : clampb(k_or_count(kb, S, count, idx), clo);
  *hi = b + 1 == G ? count : clampb(k_or_count(ke, S, count, idx), chi);
}

}  // namespace mck
