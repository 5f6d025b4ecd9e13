// mck_crc.hpp -- device side of the batched CRC32C engine (gfx950).
//
// One wavefront owns one span at a time.  A span is cut into 4 KiB "rounds"
// anchored at its 16-byte-aligned END; in every round lane l owns the 64-byte
// chunk [round_base + 64*l, +64), loaded as 4 x 16-byte coalesced loads (the
// wave's 64 lanes read 4 KiB contiguous).  Each lane runs a table-driven
// 4-byte CRC step over its chunk; the lanes' partial "pure" states are then
// shifted into place with per-lane tables and XOR-reduced across the wave.
//
// Why it is exact (the algebra of util/crc32c.cc:1221-1266):
//   * pure CRC (init 0, no inversion) is linear, and leading zero bytes do
//     not change it, so bytes before the span are loaded as zeros;
//   * Value/Extend's init (~init_crc) is XORed into the first 4 span bytes;
//   * bytes after the span (up to the aligned end) are zeros appended: the
//     result is un-shifted by those k < 16 bytes with an inverse table;
//   * between a lane's chunks in consecutive rounds lie 4032 bytes owned by
//     other lanes: the lane's state is advanced by zshift(., 4032).
//
// LDS image (105 KiB per workgroup, filled once per persistent workgroup):
//   [0, 64K)       4-byte-step byte tables, 16 interleaved copies: entry
//                  (table t, byte v, copy c) at v<<8 | t<<6 | c<<2, lane l
//                  reads copy l%16 => the address is ONE v_perm_b32 of the
//                  state and a per-lane constant, and lanes l, l+16 are the
//                  only possible bank sharers (<=2-way);
//   [64K, 96K)     per-lane final shift, nibble tables [8][16][64 lanes];
//   [96K, +512)    gap shift (4032 B), nibble tables [8][16];
//   [+512, +512)   1-byte extend, nibble tables;
//   [+1K, +9K)     un-shift by k bytes, nibble tables [16][8][16].
// Nibble tables have 16 entries in 16 distinct banks, so they never conflict.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mck_tables.hpp"

namespace mck {

constexpr uint32_t kLdsStep = 0;
constexpr uint32_t kLdsFinal = 65536;
constexpr uint32_t kLdsGap = kLdsFinal + 32768;
constexpr uint32_t kLdsExt1 = kLdsGap + 512;
constexpr uint32_t kLdsUnshift = kLdsExt1 + 512;
constexpr uint32_t kCrcLdsBytes = kLdsUnshift + kMaxUnshift * 512;  // 107520

struct alignas(16) Chunk {
  uint4 v[4];
};

__device__ __forceinline__ uint32_t lds_u32(const uint8_t* lds, uint32_t off) {
  return *reinterpret_cast<const uint32_t*>(lds + off);
}

// Fill the LDS image from the device-global tables.  All threads call it,
// followed by __syncthreads().
__device__ __forceinline__ void crc_fill_lds(uint8_t* lds, const CrcTables* __restrict__ g) {
  uint4* l4 = reinterpret_cast<uint4*>(lds);
  for (int i = threadIdx.x; i < 4096; i += blockDim.x) {
    // 16-byte slot i covers word indices 4i..4i+3 = copies c..c+3 of
    // (t = (i >> 2) & 3, v = i >> 4)
    uint32_t x = g->step[(i >> 2) & 3][i >> 4];
    l4[i] = make_uint4(x, x, x, x);
  }
  const uint4* src = reinterpret_cast<const uint4*>(&g->lane_final[0][0][0]);
  uint4* dst = reinterpret_cast<uint4*>(lds + kLdsFinal);
  constexpr int n16 = (kCrcLdsBytes - kLdsFinal) / 16;
  static_assert(sizeof(CrcTables) - sizeof(CrcTables::step) == kCrcLdsBytes - kLdsFinal, "layout");
  for (int i = threadIdx.x; i < n16; i += blockDim.x) dst[i] = src[i];
}

// Per-lane constants for the v_perm address formation.
struct CrcLane {
  uint32_t pc[4];
  uint32_t lane4;  // lane * 4
  int lane;
};
__device__ __forceinline__ CrcLane crc_lane() {
  CrcLane L;
  L.lane = threadIdx.x & 63;
  const uint32_t c = (uint32_t)(L.lane & 15);
#pragma unroll
  for (int t = 0; t < 4; t++) L.pc[t] = ((uint32_t)t << 6) | (c << 2);
  L.lane4 = (uint32_t)L.lane << 2;
  return L;
}

// s' = zshift(s, 4): 4 byte-table lookups; address byte1 = state byte t,
// byte0 = per-lane (table, copy) slot.
__device__ __forceinline__ uint32_t crc_step4(const uint8_t* lds, uint32_t s, const CrcLane& L) {
  const uint32_t a0 = __builtin_amdgcn_perm(s, L.pc[0], 0x0C0C0400u);
  const uint32_t a1 = __builtin_amdgcn_perm(s, L.pc[1], 0x0C0C0500u);
  const uint32_t a2 = __builtin_amdgcn_perm(s, L.pc[2], 0x0C0C0600u);
  const uint32_t a3 = __builtin_amdgcn_perm(s, L.pc[3], 0x0C0C0700u);
  return lds_u32(lds, a0) ^ lds_u32(lds, a1) ^ lds_u32(lds, a2) ^ lds_u32(lds, a3);
}

// A linear map given as 8 nibble tables [8][16] at LDS offset `off`.
__device__ __forceinline__ uint32_t crc_nibmap(const uint8_t* lds, uint32_t off, uint32_t s) {
  uint32_t r = 0;
#pragma unroll
  for (int n = 0; n < 8; n++) r ^= lds_u32(lds, off + n * 64 + (((s >> (4 * n)) & 15u) << 2));
  return r;
}

// zshift(s, 64*(63-lane)) with the per-lane tables.
__device__ __forceinline__ uint32_t crc_lane_final(const uint8_t* lds, uint32_t s, const CrcLane& L) {
  uint32_t r = 0;
#pragma unroll
  for (int n = 0; n < 8; n++)
    r ^= lds_u32(lds, kLdsFinal + n * 4096 + ((((s >> (4 * n)) & 15u) << 8) | L.lane4));
  return r;
}

__device__ __forceinline__ uint32_t wave_xor32(uint32_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v ^= __shfl_xor(v, o, 64);
  return v;
}

// Geometry of one span under the end-anchored round grid.
struct CrcSpan {
  uint64_t ptr;   // first byte
  uint64_t end;   // one past last byte
  uint64_t a0;    // ptr rounded down to 16
  uint64_t a1;    // end rounded up to 16
  int32_t rounds; // number of 4 KiB rounds covering [a0, a1)
  uint32_t init;  // ~init_crc: XORed into the first 4 bytes
  bool tiny;      // n < 4: computed bitwise by lane 0
};

__device__ __forceinline__ CrcSpan crc_span(const uint8_t* p, uint64_t n, uint32_t init_crc) {
  CrcSpan s;
  s.ptr = reinterpret_cast<uint64_t>(p);
  s.end = s.ptr + n;
  s.a0 = s.ptr & ~15ull;
  s.a1 = (s.end + 15) & ~15ull;
  s.tiny = n < 4;
  s.rounds = s.tiny ? 1 : (int32_t)((s.a1 - s.a0 + kRoundBytes - 1) / kRoundBytes);
  s.init = ~init_crc;
  return s;
}

__device__ __forceinline__ Chunk crc_load_chunk(const CrcSpan& sp, int r, const CrcLane& L) {
  Chunk c;
  const uint64_t cb = sp.a1 - (uint64_t)kRoundBytes * (r + 1) + (uint64_t)L.lane * kChunkBytes;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const uint64_t pa = cb + 16 * j;
    // pieces wholly before the span (or any piece of a tiny span) read as 0
    if (!sp.tiny && pa >= sp.a0)
      c.v[j] = *reinterpret_cast<const uint4*>(pa);
    else
      c.v[j] = make_uint4(0, 0, 0, 0);
  }
  return c;
}

// Zero bytes outside [ptr, end) and XOR the init into [ptr, ptr+4).
__device__ __forceinline__ uint32_t crc_mask_word(uint32_t w, uint64_t aw, const CrcSpan& sp) {
  const int64_t lo = (int64_t)(sp.ptr - aw);  // invalid bytes at the low end
  const int64_t hi = (int64_t)(sp.end - aw);  // valid bytes end here
  uint64_t m = 0xFFFFFFFFull;
  if (lo > 0) m = lo >= 4 ? 0 : (m << (8 * lo)) & 0xFFFFFFFFull;
  if (hi < 4) m = hi <= 0 ? 0 : m & (0xFFFFFFFFull >> (8 * (4 - hi)));
  w &= (uint32_t)m;
  if (lo > -4 && lo < 4) {
    const uint32_t x = lo >= 0 ? (uint32_t)((uint64_t)sp.init << (8 * lo))
                               : (uint32_t)(sp.init >> (8 * -lo));
    w ^= x;
  }
  return w;
}

__device__ __forceinline__ void crc_mask_chunk(Chunk& c, uint64_t cb, const CrcSpan& sp) {
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const uint64_t pa = cb + 16 * j;
    c.v[j].x = crc_mask_word(c.v[j].x, pa, sp);
    c.v[j].y = crc_mask_word(c.v[j].y, pa + 4, sp);
    c.v[j].z = crc_mask_word(c.v[j].z, pa + 8, sp);
    c.v[j].w = crc_mask_word(c.v[j].w, pa + 12, sp);
  }
}

// Advance one lane over its chunk of round r.
__device__ __forceinline__ uint32_t crc_round(const uint8_t* lds, uint32_t s, Chunk c, const CrcSpan& sp, int r,
                                              const CrcLane& L) {
  if (r != sp.rounds - 1) s = crc_nibmap(lds, kLdsGap, s);  // wave-uniform
  const uint64_t cb = sp.a1 - (uint64_t)kRoundBytes * (r + 1) + (uint64_t)L.lane * kChunkBytes;
  if (cb < sp.ptr + 4 || cb + kChunkBytes > sp.end) crc_mask_chunk(c, cb, sp);  // edge lanes only
#pragma unroll
  for (int j = 0; j < 4; j++) {
    s ^= c.v[j].x;
    s = crc_step4(lds, s, L);
    s ^= c.v[j].y;
    s = crc_step4(lds, s, L);
    s ^= c.v[j].z;
    s = crc_step4(lds, s, L);
    s ^= c.v[j].w;
    s = crc_step4(lds, s, L);
  }
  return s;
}

// Bitwise CRC-32C Extend for tiny spans (n < 4), one lane.
__device__ __forceinline__ uint32_t crc_tiny(const CrcSpan& sp) {
  uint32_t s = sp.init;
  for (uint64_t a = sp.ptr; a < sp.end; a++) {
    s ^= *reinterpret_cast<const uint8_t*>(a);
#pragma unroll
    for (int k = 0; k < 8; k++) s = (s >> 1) ^ ((s & 1u) ? kCrc32cPoly : 0u);
  }
  return ~s;
}

// Combine the lanes' states into the span's CRC (Extend semantics).  Every
// lane returns the same value.
__device__ __forceinline__ uint32_t crc_finish(const uint8_t* lds, uint32_t s, const CrcSpan& sp,
                                               const CrcLane& L) {
  uint32_t p = wave_xor32(crc_lane_final(lds, s, L));
  const uint32_t k = (uint32_t)(sp.a1 - sp.end);
  if (k) p = crc_nibmap(lds, kLdsUnshift + k * 512, p);
  uint32_t crc = ~p;
  if (sp.tiny) crc = __shfl(crc_tiny(sp), 0, 64);
  return crc;
}

// CRC Extend by one byte on a finished CRC value (all lanes identical).
__device__ __forceinline__ uint32_t crc_extend_byte(const uint8_t* lds, uint32_t crc, uint8_t b) {
  return ~crc_nibmap(lds, kLdsExt1, ~crc ^ (uint32_t)b);
}

__device__ __forceinline__ uint32_t crc_mask(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }

// Persistent, software-pipelined driver: each wave walks (span, round) pairs
// of spans wave_id, wave_id + nwaves, ...; the next pair's chunk is loaded
// before the current one is hashed.  Op supplies the spans and consumes the
// results:
//   const uint8_t* Op::ptr(i), uint64_t Op::len(i), uint32_t Op::init_crc(i),
//   void Op::finish(i, crc, lds)   (all lanes call it; lane 0 writes)
template <class Op>
__device__ __forceinline__ void crc_spans_driver(const Op& op, uint32_t count, uint8_t* lds,
                                                 const CrcTables* __restrict__ g) {
  crc_fill_lds(lds, g);
  __syncthreads();
  const CrcLane L = crc_lane();
  const uint32_t wpb = blockDim.x >> 6;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * wpb + (threadIdx.x >> 6));
  const uint32_t nwaves = gridDim.x * wpb;
  uint32_t i = wave;
  if (i >= count) return;
  CrcSpan sp = crc_span(op.ptr(i), op.len(i), op.init_crc(i));
  int r = sp.rounds - 1;
  Chunk cur = crc_load_chunk(sp, r, L);
  uint32_t s = 0;
  for (;;) {
    uint32_t ni = i;
    int nr = r - 1;
    CrcSpan nsp = sp;
    bool more = true;
    if (nr < 0) {
      ni = i + nwaves;
      more = ni < count;
      if (more) {
        nsp = crc_span(op.ptr(ni), op.len(ni), op.init_crc(ni));
        nr = nsp.rounds - 1;
      }
    }
    Chunk nxt;
    if (more) nxt = crc_load_chunk(nsp, nr, L);
    s = crc_round(lds, s, cur, sp, r, L);
    if (r == 0) {
      op.finish(i, crc_finish(lds, s, sp, L), lds);
      s = 0;
    }
    if (!more) break;
    i = ni;
    r = nr;
    sp = nsp;
    cur = nxt;
  }
}

}  // namespace mck
