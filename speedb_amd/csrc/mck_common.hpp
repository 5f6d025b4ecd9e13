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
// over the grid.  Workgroup b's boundary j (j = b for its first span, b + 1
// for its end) is the first span whose offset reaches o0 + range * j / G
// (o0, o0 + range: the first and last span's offsets), found by a sampled
// search: each level samples the current index range at 512 evenly spaced
// points (one load per thread, half the workgroup per boundary), the first
// sample at or past the target narrows the range to the gap before it, and a
// range of <= 512 spans is scanned whole -- two levels (two load round
// trips) up to 262,144 spans, three up to 2^27.  "The first sample at or past
// a target" is monotone in the target for ANY offsets, level by level, so the
// shares always partition the batch; they are exact byte balance when the
// offsets grow with the bytes (an SST or blob file image).  Each boundary is
// clamped to within `slack` spans of the count-balanced one.  (Round 4 took
// 8192 samples per workgroup, eight dependent loads per thread: 13.5 us
// before the first unit of a 1 GiB SST image, round-5 stamps; count-balanced
// CRC shares of that image hold 3.0-4.9 MiB and their end times track the
// bytes, correlation 0.98.)  scratch: 12 x u32 in LDS.  Workgroup-uniform;
// has barriers; blockDim.x = 1024.
// prefetch(i): a load of span i's descriptors whose value is discarded --
// issued for the count-balanced share's first spans with the first level's
// samples, so the window staging that follows finds them in the cache (the
// SST images' staging waited 6-9 us on them, round-5 stamps).
// overlap(): the caller's own prologue work (its loads ride along with the
// first level's round trip); called exactly once on every path.
struct NoOverlap {
  __device__ void operator()() const {}
};
template <class Op, class P, class F, class O = NoOverlap>
__device__ __forceinline__ void share_by_bytes(const Op& op, uint32_t first, uint32_t count, uint32_t slack,
                                               P scratch, uint32_t* lo, uint32_t* hi, const F& prefetch,
                                               const O& overlap = O{}) {
  const uint32_t G = gridDim.x, b = blockIdx.x;
  const uint32_t clo = (uint32_t)((uint64_t)count * b / G), chi = (uint32_t)((uint64_t)count * (b + 1) / G);
  if (count <= 1 || G == 1) {
    *lo = clo;
    *hi = chi;
    overlap();
    return;
  }
  constexpr uint32_t kS = 512;  // samples per boundary and level
  uint32_t nlev = 1;
  for (uint32_t c = count; c > kS; c = c / kS + 1) nlev++;
  const uint32_t tgt = threadIdx.x >= kS ? 1u : 0u, t = threadIdx.x & (kS - 1);
  if (threadIdx.x < 2 * nlev) scratch[threadIdx.x] = 0xFFFFFFFFu;
  // (a barrier waits for every load in flight: the scratch is set up before
  // the first loads, so the range ends, the first level's samples -- their
  // positions do not depend on the target -- and the prefetch share one
  // round trip)
  __syncthreads();
  const uint64_t o0 = op.off(first), oL = op.off(first + count - 1);
  const uint32_t p0 = count > kS ? (uint32_t)((uint64_t)count * t / kS) : t;  // level 0's sample
  const uint64_t s0 = count > kS || t < count ? op.off(first + p0) : 0ull;
  const uint32_t pf = clo + threadIdx.x < count ? prefetch(first + clo + threadIdx.x) : 0u;
  overlap();
  const uint64_t range = oL > o0 ? oL - o0 : 0;
  const uint32_t j = b + tgt;
  // o0 + range * j / G without a 128-bit product
  const uint64_t T = o0 + (range / G) * j + (range % G) * j / G;
  uint32_t L = 0, R = count, res = j == 0 ? 0u : count;
  bool done = j == 0 || j == G;
  for (uint32_t lev = 0; lev < nlev; lev++) {
    const uint32_t n = R - L;
    const bool whole = n <= kS;
    const uint32_t p = whole ? L + t : L + (uint32_t)((uint64_t)n * t / kS);
    const bool flag = !done && (!whole || t < n) && (lev == 0 ? s0 : op.off(first + p)) >= T;
    const uint64_t m = __ballot(flag);
    if ((threadIdx.x & 63) == 0 && m)
      __hip_atomic_fetch_min(&scratch[2 * lev + tgt], (t & ~63u) + (uint32_t)__builtin_ctzll(m), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
    __syncthreads();
    if (done) continue;
    const uint32_t tf = scratch[2 * lev + tgt];  // first sample at or past T (~0: none)
    if (whole) {
      res = tf < n ? L + tf : R;
      done = true;
    } else if (tf == 0) {
      res = L;
      done = true;
    } else {
      const uint32_t tl = tf > kS ? kS : tf;  // none: the gap after the last sample
      const uint32_t nL = L + (uint32_t)((uint64_t)n * (tl - 1) / kS) + 1;
      const uint32_t nR = tf > kS ? R : L + (uint32_t)((uint64_t)n * tf / kS);
      L = nL;
      R = nR;
      if (L >= R) {
        res = R;
        done = true;
      }
    }
  }
  const uint32_t cc = tgt ? chi : clo;
  const uint32_t a = cc > slack ? cc - slack : 0u;
  const uint64_t z = (uint64_t)cc + slack < count ? (uint64_t)cc + slack : count;
  res = res < a ? a : res > z ? (uint32_t)z : res;
  if (t == 0) scratch[2 * nlev + tgt] = res;
  asm volatile("" ::"v"(pf));  // (the prefetch's value, never used)
  __syncthreads();
  *lo = scratch[2 * nlev];
  *hi = scratch[2 * nlev + 1];
  __syncthreads();  // the scratch may be reused
}

}  // namespace mck
