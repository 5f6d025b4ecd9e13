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
//   * Value/Extend's init state (~init_crc) sits at the span's first byte;
//     it is injected into the owning lane's state at the enclosing 16-byte
//     piece boundary, pre-un-shifted by the (ptr mod 16) bytes in between;
//   * bytes after the span (up to the aligned end) are zeros appended: the
//     result is un-shifted by those k < 16 bytes with an inverse table;
//   * between a lane's chunks in consecutive rounds lie 4032 bytes owned by
//     other lanes: the lane's state is advanced by zshift(., 4032).
// A 16-byte-aligned span therefore runs with no masking and no divergence.
//
// LDS image (128 KiB per workgroup, filled once per persistent workgroup):
//   [0, 32K)       per-lane final shift, nibble tables [8][16][64 lanes];
//   [32K, +512)    gap shift (4032 B), nibble tables [8][16];
//   [+512, +512)   1-byte extend, nibble tables;
//   [33K, 41K)     un-shift by k bytes, nibble tables [16][8][16];
//   [64K, 128K)    4-byte-step byte tables, 16 interleaved copies: entry
//                  (table t, byte v, copy c) at 64K | v<<8 | t<<6 | c<<2;
//                  lane l reads copy l%16, so the address is ONE v_perm_b32
//                  of the state and a per-lane constant, and lanes l, l+16
//                  are the only possible bank sharers (<=2-way).
// Nibble tables sit below 64 KiB so their offsets fold into ds_read
// immediates; 16 entries in 16 distinct banks never conflict.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mck_tables.hpp"

namespace mck {

constexpr uint32_t kLdsFinal = 0;
constexpr uint32_t kLdsGap = kLdsFinal + 32768;
constexpr uint32_t kLdsExt1 = kLdsGap + 512;
constexpr uint32_t kLdsUnshift = kLdsExt1 + 512;
constexpr uint32_t kLdsNibEnd = kLdsUnshift + kMaxUnshift * 512;  // 41984
constexpr uint32_t kLdsStep = 65536;
constexpr uint32_t kCrcLdsBytes = kLdsStep + 65536;  // 131072

struct alignas(16) Chunk {
  uint4 v[4];
};

// The kernels declare no static __shared__, so the dynamic LDS image starts
// at LDS address 0 and table addresses are absolute: reading through an
// address_space(3) pointer built from the integer avoids re-adding the base.
typedef __attribute__((address_space(3))) const uint32_t lds_word_t;
__device__ __forceinline__ uint32_t lds_u32(const uint8_t*, uint32_t off) {
  return *reinterpret_cast<lds_word_t*>(static_cast<size_t>(off));
}

// 16-byte load through a global (address_space(1)) pointer: keeps the load a
// global_load (vmcnt-ordered) rather than a flat_load.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gbl_u32x4_t;
__device__ __forceinline__ uint4 gload16(uint64_t addr) {
  const u32x4 v = *reinterpret_cast<gbl_u32x4_t*>(addr);
  return make_uint4(v.x, v.y, v.z, v.w);
}

// Fill the LDS image from the device-global tables.  All threads call it,
// followed by __syncthreads().
__device__ __forceinline__ void crc_fill_lds(uint8_t* lds, const CrcTables* __restrict__ g) {
  uint4* l4 = reinterpret_cast<uint4*>(lds + kLdsStep);
  for (int i = threadIdx.x; i < 4096; i += blockDim.x) {
    // 16-byte slot i covers word indices 4i..4i+3 = copies c..c+3 of
    // (t = (i >> 2) & 3, v = i >> 4)
    uint32_t x = g->step[(i >> 2) & 3][i >> 4];
    l4[i] = make_uint4(x, x, x, x);
  }
  const uint4* src = reinterpret_cast<const uint4*>(&g->lane_final[0][0][0]);
  uint4* dst = reinterpret_cast<uint4*>(lds + kLdsFinal);
  constexpr int n16 = (kLdsNibEnd - kLdsFinal) / 16;
  static_assert(sizeof(CrcTables) - sizeof(CrcTables::step) == kLdsNibEnd - kLdsFinal, "layout");
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
  for (int t = 0; t < 4; t++) L.pc[t] = kLdsStep | ((uint32_t)t << 6) | (c << 2);
  L.lane4 = (uint32_t)L.lane << 2;
  return L;
}

// s' = zshift(s, 4): 4 byte-table lookups; address byte1 = state byte t,
// byte0 = per-lane (table, copy) slot, byte2 = 1 (the 64 KiB region).
__device__ __forceinline__ uint32_t crc_step4(const uint8_t* lds, uint32_t s, const CrcLane& L) {
  const uint32_t a0 = __builtin_amdgcn_perm(s, L.pc[0], 0x0C020400u);
  const uint32_t a1 = __builtin_amdgcn_perm(s, L.pc[1], 0x0C020500u);
  const uint32_t a2 = __builtin_amdgcn_perm(s, L.pc[2], 0x0C020600u);
  const uint32_t a3 = __builtin_amdgcn_perm(s, L.pc[3], 0x0C020700u);
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

// Un-shift by a wave-uniform k in [0, 16) bytes.
__device__ __forceinline__ uint32_t crc_unshift(const uint8_t* lds, uint32_t k, uint32_t s) {
  return crc_nibmap(lds, kLdsUnshift + k * 512, s);
}

// Geometry of one span under the end-anchored round grid.
struct CrcSpan {
  uint64_t ptr;    // first byte
  uint64_t end;    // one past last byte
  uint64_t a0;     // ptr rounded down to 16
  uint64_t a1;     // end rounded up to 16
  int32_t rounds;  // number of 4 KiB rounds covering [a0, a1)
  uint32_t head;   // ptr - a0: leading bytes of the first piece to zero
  uint32_t kt;     // a1 - end: trailing zero bytes to un-shift
  uint32_t inj;    // init state, un-shifted to the piece boundary a0
  uint32_t init_crc;
  bool empty;      // n == 0: Extend(init, "") = init
};

__device__ __forceinline__ CrcSpan crc_span(const uint8_t* lds, const uint8_t* p, uint64_t n, uint32_t init_crc) {
  CrcSpan s;
  s.ptr = reinterpret_cast<uint64_t>(p);
  s.end = s.ptr + n;
  s.a0 = s.ptr & ~15ull;
  s.a1 = (s.end + 15) & ~15ull;
  s.empty = n == 0;
  s.rounds = s.empty ? 1 : (int32_t)((s.a1 - s.a0 + kRoundBytes - 1) / kRoundBytes);
  s.head = (uint32_t)(s.ptr - s.a0);
  s.kt = (uint32_t)(s.a1 - s.end);
  s.init_crc = init_crc;
  s.inj = ~init_crc;
  if (s.head) s.inj = crc_unshift(lds, s.head, s.inj);  // wave-uniform branch
  return s;
}

__device__ __forceinline__ uint64_t crc_chunk_base(const CrcSpan& sp, int r, const CrcLane& L) {
  return sp.a1 - (uint64_t)kRoundBytes * (r + 1) + (uint64_t)L.lane * kChunkBytes;
}

// Branch-free so the compiler can count outstanding loads (a load under an
// exec-masked branch makes every later wait a vmcnt(0) and kills the
// prefetch): pieces wholly before the span load from a0 instead and are
// zeroed by a select.
__device__ __forceinline__ Chunk crc_load_chunk(const CrcSpan& sp, int r, const CrcLane& L) {
  Chunk c;
  const uint64_t cb = crc_chunk_base(sp, r, L);
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const uint64_t pa = cb + 16 * j;
    const bool ok = !sp.empty && pa >= sp.a0;
    const uint4 v = gload16(ok ? pa : sp.a0);
    c.v[j] = ok ? v : make_uint4(0, 0, 0, 0);
  }
  return c;
}

// keep bytes [lo, hi) of a 16-byte piece, zero the rest
__device__ __forceinline__ uint32_t keep_bytes(uint32_t w, int k, int lo, int hi) {
  const int a = lo - 4 * k, b = hi - 4 * k;  // keep [a, b) of this word
  uint64_t m = 0xFFFFFFFFull;
  if (a > 0) m = a >= 4 ? 0 : (m << (8 * a)) & 0xFFFFFFFFull;
  if (b < 4) m = b <= 0 ? 0 : m & (0xFFFFFFFFull >> (8 * (4 - b)));
  return w & (uint32_t)m;
}
__device__ __forceinline__ void keep_piece(uint4& v, int lo, int hi) {
  v.x = keep_bytes(v.x, 0, lo, hi);
  v.y = keep_bytes(v.y, 1, lo, hi);
  v.z = keep_bytes(v.z, 2, lo, hi);
  v.w = keep_bytes(v.w, 3, lo, hi);
}

__device__ __forceinline__ uint32_t crc_piece(const uint8_t* lds, uint32_t s, const uint4& v, const CrcLane& L) {
  s ^= v.x;
  s = crc_step4(lds, s, L);
  s ^= v.y;
  s = crc_step4(lds, s, L);
  s ^= v.z;
  s = crc_step4(lds, s, L);
  s ^= v.w;
  s = crc_step4(lds, s, L);
  return s;
}

// Advance one lane over its chunk of round r.
__device__ __forceinline__ uint32_t crc_round(const uint8_t* lds, uint32_t s, Chunk c, const CrcSpan& sp, int r,
                                              const CrcLane& L) {
  if (r != sp.rounds - 1) s = crc_nibmap(lds, kLdsGap, s);  // wave-uniform
  const uint64_t cb = crc_chunk_base(sp, r, L);
  // piece (0..3) of this chunk that starts at a0, or out of range
  const int64_t jh = (int64_t)(sp.a0 - cb) >> 4;
  if (sp.head && jh >= 0 && jh < 4) {  // unaligned start: one lane, once
#pragma unroll
    for (int j = 0; j < 4; j++)
      if (j == jh) keep_piece(c.v[j], (int)sp.head, 16);
  }
  if (sp.kt && r == 0 && L.lane == 63) keep_piece(c.v[3], 0, 16 - (int)sp.kt);  // unaligned end
  const uint32_t inj = sp.empty ? 0u : sp.inj;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    s ^= jh == j ? inj : 0u;
    s = crc_piece(lds, s, c.v[j], L);
  }
  return s;
}

// Combine the lanes' states into the span's CRC (Extend semantics).  Every
// lane returns the same value.
__device__ __forceinline__ uint32_t crc_finish(const uint8_t* lds, uint32_t s, const CrcSpan& sp,
                                               const CrcLane& L) {
  uint32_t p = wave_xor32(crc_lane_final(lds, s, L));
  if (sp.kt) p = crc_unshift(lds, sp.kt, p);
  return sp.empty ? sp.init_crc : ~p;
}

// CRC Extend by one byte on a finished CRC value (all lanes identical).
__device__ __forceinline__ uint32_t crc_extend_byte(const uint8_t* lds, uint32_t crc, uint8_t b) {
  return ~crc_nibmap(lds, kLdsExt1, ~crc ^ (uint32_t)b);
}

__device__ __forceinline__ uint32_t crc_mask(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }

// Persistent, software-pipelined driver: each wave walks (span, round) pairs
// of spans wave_id, wave_id + nwaves, ...; the next pair's chunk is loaded
// before the current one is hashed.  Span descriptors are fetched 64 spans at
// a time (lane l loads the descriptor of the wave's l-th next span) and read
// back with v_readlane, so a descriptor costs no memory latency per span.
// Op supplies the spans and consumes the results:
//   const uint8_t* Op::base(), uint64_t Op::off(i), uint64_t Op::len(i),
//   uint32_t Op::init_crc(i)                    (per lane, i < count)
//   void Op::finish(i, crc, lds)   (all lanes call it; lane 0 writes)
struct SpanDesc {
  uint64_t off;
  uint64_t len;
  uint32_t init;
};

template <class Op>
__device__ __forceinline__ SpanDesc crc_desc_fetch(const Op& op, uint32_t first, uint32_t nwaves, uint32_t count,
                                                   const CrcLane& L) {
  SpanDesc d{0, 0, 0};
  const uint64_t i = (uint64_t)first + (uint64_t)L.lane * nwaves;
  if (i < count) {
    d.off = op.off((uint32_t)i);
    d.len = op.len((uint32_t)i);
    d.init = op.init_crc((uint32_t)i);
  }
  return d;
}
// v_readlane returns int: widen through uint32_t, never sign-extend.
__device__ __forceinline__ uint32_t readlane_u32(uint32_t v, uint32_t k) {
  return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), static_cast<int>(k)));
}
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, uint32_t k) {
  return ((uint64_t)readlane_u32((uint32_t)(v >> 32), k) << 32) | (uint64_t)readlane_u32((uint32_t)v, k);
}
__device__ __forceinline__ SpanDesc crc_desc_pick(const SpanDesc& d, uint32_t k) {
  SpanDesc r;
  r.off = readlane_u64(d.off, k);
  r.len = readlane_u64(d.len, k);
  r.init = readlane_u32(d.init, k);
  return r;
}

template <class Op>
__device__ __forceinline__ void crc_spans_driver(const Op& op, uint32_t count, uint8_t* lds,
                                                 const CrcTables* __restrict__ g) {
  crc_fill_lds(lds, g);
  __syncthreads();
  const CrcLane L = crc_lane();
  const uint32_t wpb = blockDim.x >> 6;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * wpb + (threadIdx.x >> 6));
  const uint32_t nwaves = gridDim.x * wpb;
  if (wave >= count) return;
  const uint64_t base = reinterpret_cast<uint64_t>(op.base());
  uint32_t i = wave;  // current span
  uint32_t k = 0;     // its slot in the descriptor batch
  SpanDesc db = crc_desc_fetch(op, i, nwaves, count, L);
  SpanDesc d = crc_desc_pick(db, 0);
  CrcSpan sp = crc_span(lds, reinterpret_cast<const uint8_t*>(base + d.off), d.len, d.init);
  int r = sp.rounds - 1;
  Chunk cur = crc_load_chunk(sp, r, L);
  uint32_t s = 0;
  for (;;) {
    uint32_t ni = i, nk = k;
    int nr = r - 1;
    CrcSpan nsp = sp;
    bool more = true;
    if (nr < 0) {
      ni = i + nwaves;
      more = ni < count;
      if (more) {
        nk = k + 1;
        if (nk == 64) {
          db = crc_desc_fetch(op, ni, nwaves, count, L);
          nk = 0;
        }
        const SpanDesc nd = crc_desc_pick(db, nk);
        nsp = crc_span(lds, reinterpret_cast<const uint8_t*>(base + nd.off), nd.len, nd.init);
        nr = nsp.rounds - 1;
      }
    }
    // unconditional (see crc_load_chunk); after the last round it re-reads
    // the current chunk, which is never used
    const Chunk nxt = crc_load_chunk(more ? nsp : sp, more ? nr : r, L);
    s = crc_round(lds, s, cur, sp, r, L);
    if (r == 0) {
      op.finish(i, crc_finish(lds, s, sp, L), lds);
      s = 0;
    }
    if (!more) break;
    i = ni;
    k = nk;
    r = nr;
    sp = nsp;
    cur = nxt;
  }
}

}  // namespace mck
