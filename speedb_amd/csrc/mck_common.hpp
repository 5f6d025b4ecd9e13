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

// Byte-balanced contiguous shares of a ragged batch of `count` spans.  A
// share of spans b, b + G, ... (or of count / G consecutive spans) holds a
// random number of the big spans: in a compaction-shaped 4/16/64 KiB mix of
// 1 GiB the fullest of 256 shares carries 1.23x the mean bytes, and the
// launch lasts as long as its workgroup.  Here every workgroup reads all the
// lengths (a few hundred KiB at most, L2-resident after the first workgroup
// of an XCD) and takes [lo, hi): span i belongs to workgroup b when the
// batch offset of its first byte (the sum of the lengths before it) lies in
// [total b / G, total (b + 1) / G) (the last workgroup also takes trailing
// empty spans).  Each boundary is then clamped to within `slack` spans of
// the boundary by count (count b / G), which bounds a share at count / G +
// 1 + 2 slack spans for drivers with a fixed descriptor cache.  All
// workgroups compute the same prefix and the same clamps, so the ranges
// partition [0, count) exactly.  lds: blockDim / 64 u64.  Ends with a
// barrier.
#ifndef MCK_BALANCE_MAX_SPANS
#define MCK_BALANCE_MAX_SPANS (1u << 18)
#endif
constexpr uint32_t kBalanceMaxSpans = MCK_BALANCE_MAX_SPANS;  // beyond: shares by count (their bytes average out)
// (The lengths are read as 16-byte vectors, eight vectors -- 32 lengths --
// in flight per thread, with clamped addresses so every load of a batch is
// issued at once; a first version read one length per load and waited for
// each, ~80 us of serial L2 round trips per launch.)
constexpr uint32_t kLenVecs = 8;
// sum of lens[c0, c1) (c0 a multiple of 4, lens 16-byte aligned)
__device__ __forceinline__ uint64_t lens_sum(const uint32_t* lens, uint32_t c0, uint32_t c1) {
  uint64_t sum = 0;
  for (uint32_t i = c0; i < c1; i += 4 * kLenVecs) {
    uint4 v[kLenVecs];
#pragma unroll
    for (uint32_t k = 0; k < kLenVecs; k++) {
      const uint32_t j = i + 4 * k < c1 ? i + 4 * k : c0;
      v[k] = *reinterpret_cast<const uint4*>(lens + j);
    }
#pragma unroll
    for (uint32_t k = 0; k < kLenVecs; k++) {
      const uint32_t j = i + 4 * k;
      sum += (j < c1 ? v[k].x : 0u) + (j + 1 < c1 ? v[k].y : 0u);
      sum += (j + 2 < c1 ? v[k].z : 0u) + (j + 3 < c1 ? v[k].w : 0u);
    }
  }
  return sum;
}
// spans of [c0, c1) whose first byte (p0 + the lengths before them) lies
// below t
__device__ __forceinline__ uint32_t lens_below(const uint32_t* lens, uint32_t c0, uint32_t c1, uint64_t p0,
                                               uint64_t t) {
  uint32_t n = 0;
  uint64_t p = p0;
  for (uint32_t i = c0; i < c1; i += 4 * kLenVecs) {
    uint4 v[kLenVecs];
#pragma unroll
    for (uint32_t k = 0; k < kLenVecs; k++) {
      const uint32_t j = i + 4 * k < c1 ? i + 4 * k : c0;
      v[k] = *reinterpret_cast<const uint4*>(lens + j);
    }
#pragma unroll
    for (uint32_t k = 0; k < kLenVecs; k++) {
      const uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
      for (uint32_t q = 0; q < 4; q++) {
        const bool in = i + 4 * k + q < c1;
        n += in && p < t ? 1u : 0u;
        p += in ? w[q] : 0u;
      }
    }
  }
  return n;
}
// lens: the batch's length array (nullptr: every span the same length --
// the shares by count are balanced already)
__device__ __forceinline__ void balanced_range(const uint32_t* lens, uint32_t count, uint32_t slack, uint64_t* lds,
                                               uint32_t* lo, uint32_t* hi) {
  const uint64_t G = gridDim.x, b = blockIdx.x;
  if (lens == nullptr || (reinterpret_cast<uint64_t>(lens) & 15)) {  // grid-uniform
    // (an unaligned length array -- a sliced view -- keeps the shares by count)
    *lo = (uint32_t)((uint64_t)count * b / G);
    *hi = (uint32_t)((uint64_t)count * (b + 1) / G);
    return;
  }
  const uint32_t nt = blockDim.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, nw = nt >> 6;
  const uint32_t per = ((count + nt - 1) / nt + 3) & ~3u;
  const uint32_t c0 = min(tid * per, count), c1 = min(c0 + per, count);
  const uint64_t sum = lens_sum(lens, c0, c1);
  uint64_t x = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(x, d, 64);
    x += lane >= (uint32_t)d ? y : 0ull;
  }
  if (lane == 63) lds[wid] = x;
  __syncthreads();
  uint64_t below = 0, total = 0;
  for (uint32_t w = 0; w < nw; w++) {
    const uint64_t v = lds[w];
    below += w < wid ? v : 0ull;
    total += v;
  }
  __syncthreads();
  const uint64_t tlo = total * b / G, thi = total * (b + 1) / G;
  // spans whose first byte lies below tlo / thi (the prefix never
  // decreases): a chunk that ends below the target counts whole, one that
  // starts at or above it not at all; only the chunk holding the target
  // walks its lengths
  const uint64_t e = below + x - sum;  // the chunk's first byte
  const auto cnt = [&](uint64_t t) -> uint32_t {
    if (e + sum < t) return c1 - c0;
    if (e >= t) return 0u;
    return lens_below(lens, c0, c1, e, t);
  };
  uint64_t r = ((uint64_t)cnt(thi) << 32) | cnt(tlo);
  for (int m = 32; m >= 1; m >>= 1) r += __shfl_xor(r, m, 64);
  if (lane == 0) lds[wid] = r;
  __syncthreads();
  uint64_t tot = 0;
  for (uint32_t w = 0; w < nw; w++) tot += lds[w];
  const auto clampb = [&](uint32_t v, uint64_t bb) {
    const uint32_t c = (uint32_t)((uint64_t)count * bb / G);
    const uint32_t a = c > slack ? c - slack : 0u, z = count - c > slack ? c + slack : count;
    return v < a ? a : v > z ? z : v;
  };
  *lo = clampb((uint32_t)tot, b);
  *hi = b + 1 == G ? count : clampb((uint32_t)(tot >> 32), b + 1);
  __syncthreads();
}

}  // namespace mck
