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
//     not change it;
//   * Value/Extend's init state (~init_crc) sits at the span's first byte;
//     it is injected into the "owner" lane's state at the start of its
//     first-round chunk, pre-un-shifted by the hb < 64 bytes in between,
//     which that lane zeroes; lanes whose first chunk lies wholly before the
//     span drop their state after the first round;
//   * bytes after the span (up to the aligned end) are zeros appended: the
//     result is un-shifted by those kt < 16 bytes;
//   * between a lane's chunks in consecutive rounds lie 4032 bytes owned by
//     other lanes: the lane's state is advanced by zshift(., 4032).
// A span whose start is on the 64-byte grid and whose end is 16-aligned runs
// with no masking and no divergence.
//
// LDS image (160 KiB per workgroup, filled once per persistent workgroup):
//   [0, 32K)       per-lane final shift, nibble tables [8][16][64 lanes];
//   [32K, +512)    gap shift (4032 B), nibble tables [8][16];
//   [+512, +512)   1-byte extend, nibble tables;
//   [+512, +512)   32-byte shift, nibble tables (joins a lane's chains);
//   [+512, +512)   16-byte shift, nibble tables;
//   [64K, 128K)    4-byte-step byte tables, 16 interleaved copies: entry
//                  (table t, byte v, copy c) at 64K | v<<8 | t<<6 | c<<2;
//                  lane l reads copy l%16, so the address is ONE v_perm_b32
//                  of the state and per-lane constants; with the per-lane
//                  table rotation (crc_lane) every lookup is conflict-free;
//   [128K, 160K)   un-shift by k < 64 bytes, nibble tables [64][8][16]
//                  (k is wave-uniform: the base goes in an SGPR).
// Fixed-offset nibble tables sit below 64 KiB so their offsets fold into
// ds_read immediates; 16 entries in 16 distinct banks never conflict.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <type_traits>

#include "mck_common.hpp"
#include "mck_tables.hpp"

namespace mck {

constexpr uint32_t kLdsFinal = 0;
constexpr uint32_t kLdsGap = kLdsFinal + 32768;
constexpr uint32_t kLdsExt1 = kLdsGap + 512;
constexpr uint32_t kLdsHalf = kLdsExt1 + 512;
constexpr uint32_t kLdsQuarter = kLdsHalf + 512;
constexpr uint32_t kLdsLowEnd = kLdsQuarter + 512;  // 34816

// Independent lookup chains per lane and round (1, 2 or 4); see crc_round.
// One chain since the row-transposed loads made the kernels VALU-bound:
// the join of two chains (a 32-byte nibble map per round) costs more than
// the latency it hides (headline 0.786 vs 0.774, SST 0.657 vs 0.648, WAL
// 0.711 vs 0.700; four chains: 73.1 vs 76.5 %).
constexpr int kCrcChains = 1;
static_assert(kCrcChains == 1 || kCrcChains == 2 || kCrcChains == 4, "chains");
constexpr uint32_t kLdsStep = 65536;
constexpr uint32_t kLdsUnshift = 131072;
constexpr uint32_t kCrcLdsBytes = kLdsUnshift + kMaxUnshift * 512;  // 163840

static_assert(offsetof(CrcTables, gap) - offsetof(CrcTables, lane_final) == kLdsGap - kLdsFinal, "layout");
static_assert(offsetof(CrcTables, unshift) - offsetof(CrcTables, lane_final) == kLdsLowEnd - kLdsFinal, "layout");

// A lane's chunk of P 16-byte pieces (the wave driver and the row driver
// use P = 4; the one-pass WAL writer's rows P = 5).
template <int P = 4>
struct alignas(16) ChunkN {
  uint4 v[P];
};
using Chunk = ChunkN<4>;

// The kernels declare no static __shared__, so the dynamic LDS image starts
// at LDS address 0 and table addresses are absolute: reading through an
// address_space(3) pointer built from the integer avoids re-adding the base.
typedef __attribute__((address_space(3))) const uint32_t lds_word_t;
__device__ __forceinline__ uint32_t lds_u32(uint32_t off) {
  return *reinterpret_cast<lds_word_t*>(static_cast<size_t>(off));
}

__device__ __forceinline__ uint4 gload16(uint64_t addr) { return span_load16<false>(addr); }

// Fill the LDS image from the device-global tables, in two halves so that
// the table loads of all threads are in flight together (one memory round
// trip instead of one per loop trip) and the caller can issue its first
// span loads in between: crc_fill_load(), [span loads], crc_fill_store(),
// __syncthreads().  Every CRC kernel runs kCrcBlock threads per workgroup.
// UNSHIFT = false skips the un-shift tables (uniform FULL batches never
// un-shift).
constexpr int kCrcBlock = 1024;
constexpr int kFillLow = (int)(kLdsLowEnd - kLdsFinal) / 16;  // 2176 slots
constexpr int kFillUnshift = kMaxUnshift * 512 / 16;          // 2048 slots
struct CrcFill {
  uint32_t step[4096 / kCrcBlock];
  uint4 low[(kFillLow + kCrcBlock - 1) / kCrcBlock];
  uint4 un[kFillUnshift / kCrcBlock];
};
template <bool UNSHIFT>
__device__ __forceinline__ void crc_fill_load(CrcFill& f, const CrcTables* __restrict__ g) {
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 4096 / kCrcBlock; k++) {
    // 16-byte slot i covers word indices 4i..4i+3 = copies c..c+3 of
    // (t = (i >> 2) & 3, v = i >> 4)
    const int i = t + kCrcBlock * k;
    f.step[k] = g->step[(i >> 2) & 3][i >> 4];
  }
  const uint4* lo = reinterpret_cast<const uint4*>(&g->lane_final[0][0][0]);
#pragma unroll
  for (int k = 0; k < (kFillLow + kCrcBlock - 1) / kCrcBlock; k++) {
    const int i = t + kCrcBlock * k;
    f.low[k] = lo[i < kFillLow ? i : 0];
  }
  if (UNSHIFT) {
    const uint4* us = reinterpret_cast<const uint4*>(&g->unshift[0][0][0]);
#pragma unroll
    for (int k = 0; k < kFillUnshift / kCrcBlock; k++) f.un[k] = us[t + kCrcBlock * k];
  }
}
template <bool UNSHIFT>
__device__ __forceinline__ void crc_fill_store(const CrcFill& f, uint8_t* lds) {
  const int t = threadIdx.x;
  uint4* l4 = reinterpret_cast<uint4*>(lds + kLdsStep);
#pragma unroll
  for (int k = 0; k < 4096 / kCrcBlock; k++) {
    const uint32_t x = f.step[k];
    l4[t + kCrcBlock * k] = make_uint4(x, x, x, x);
  }
  uint4* dlo = reinterpret_cast<uint4*>(lds + kLdsFinal);
#pragma unroll
  for (int k = 0; k < (kFillLow + kCrcBlock - 1) / kCrcBlock; k++) {
    const int i = t + kCrcBlock * k;
    if (i < kFillLow) dlo[i] = f.low[k];
  }
  if (UNSHIFT) {
    uint4* dus = reinterpret_cast<uint4*>(lds + kLdsUnshift);
#pragma unroll
    for (int k = 0; k < kFillUnshift / kCrcBlock; k++) dus[t + kCrcBlock * k] = f.un[k];
  }
}
__device__ __forceinline__ void crc_fill_lds(uint8_t* lds, const CrcTables* __restrict__ g) {
  CrcFill f;
  crc_fill_load<true>(f, g);
  crc_fill_store<true>(f, lds);
}

// Per-lane constants for the v_perm address formation.  Lookup k of a step
// reads table t = (k + h) & 3 with h = bit 4 of the lane id: within each
// 32-lane LDS group, lanes 0-15 and 16-31 then always hit opposite halves
// of the 32 banks (bank = (t & 1) * 16 + lane % 16), so all 32 lanes of the
// group are on distinct banks -- conflict-free with only 16 table copies.
// The v_perm selector (byte1 <- state byte t) is therefore per lane.
struct CrcLane {
  uint32_t pc[4];   // 64K | t << 6 | copy << 2
  uint32_t sel[4];  // v_perm selector for table t
  uint32_t lane4;   // lane * 4
  int lane;         // chunk position (the virtual lane under transposed loads)
  int plane;        // physical lane (16-byte mini-round pieces, descriptor slots)
};
__device__ __forceinline__ CrcLane crc_lane() {
  CrcLane L;
  L.lane = threadIdx.x & 63;
  const uint32_t c = (uint32_t)(L.lane & 15), h = (uint32_t)(L.lane >> 4) & 1u;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t t = ((uint32_t)k + h) & 3u;
    L.pc[k] = kLdsStep | (t << 6) | (c << 2);
    // byte0 <- pc.b0, byte1 <- state byte t, byte2 <- pc.b2 (=1), byte3 <- 0
    L.sel[k] = 0x0C020000u | ((4u + t) << 8);
  }
  L.lane4 = (uint32_t)L.lane << 2;
  L.plane = L.lane;
  return L;
}

// zshift(s, 4) ^ w: 4 byte-table lookups, one v_perm_b32 address each; w is
// the next data word, folded in by the same two bitop3 that join the
// lookups (a step costs 4 perm + 2 bitop3 instead of 4 perm + 4 xor).
__device__ __forceinline__ uint32_t crc_step4x(uint32_t s, const CrcLane& L, uint32_t w) {
  const uint32_t a0 = __builtin_amdgcn_perm(s, L.pc[0], L.sel[0]);
  const uint32_t a1 = __builtin_amdgcn_perm(s, L.pc[1], L.sel[1]);
  const uint32_t a2 = __builtin_amdgcn_perm(s, L.pc[2], L.sel[2]);
  const uint32_t a3 = __builtin_amdgcn_perm(s, L.pc[3], L.sel[3]);
  return xor3(xor3(lds_u32(a0), lds_u32(a1), lds_u32(a2)), lds_u32(a3), w);
}
// s' = zshift(s, 4)
__device__ __forceinline__ uint32_t crc_step4(uint32_t s, const CrcLane& L) { return crc_step4x(s, L, 0u); }

// A linear map given as 8 nibble tables [8][16] at LDS offset `off`.
__device__ __forceinline__ uint32_t crc_nibmap(uint32_t off, uint32_t s) {
  uint32_t x[8];
#pragma unroll
  for (int n = 0; n < 8; n++) x[n] = lds_u32(off + n * 64 + (((s >> (4 * n)) & 15u) << 2));
  return xor3(xor3(x[0], x[1], x[2]), xor3(x[3], x[4], x[5]), x[6] ^ x[7]);
}

// zshift(s, 64*(63-lane)) with the per-lane tables.
__device__ __forceinline__ uint32_t crc_lane_final(uint32_t s, const CrcLane& L) {
  uint32_t x[8];
#pragma unroll
  for (int n = 0; n < 8; n++) x[n] = lds_u32(kLdsFinal + n * 4096 + ((((s >> (4 * n)) & 15u) << 8) | L.lane4));
  return xor3(xor3(x[0], x[1], x[2]), xor3(x[3], x[4], x[5]), x[6] ^ x[7]);
}

// XOR over the 64 lanes, returned wave-uniform: DPP butterfly inside each
// 16-lane row (xor 1, xor 2, half-mirror, mirror), then the 4 row totals are
// read out with v_readlane.  No LDS traffic.
__device__ __forceinline__ uint32_t wave_xor32(uint32_t v) {
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);   // quad_perm [1,0,3,2]
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true);   // quad_perm [2,3,0,1]
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, true);  // row_half_mirror
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, true);  // row_mirror
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) ^ (uint32_t)__builtin_amdgcn_readlane((int)v, 16) ^
         (uint32_t)__builtin_amdgcn_readlane((int)v, 32) ^ (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}

// Un-shift by a wave-uniform k in [0, 64) bytes.
__device__ __forceinline__ uint32_t crc_unshift(uint32_t k, uint32_t s) {
  return crc_nibmap(kLdsUnshift + k * 512, s);
}

// Geometry of one span under the end-anchored round grid.
struct CrcSpan {
  uint64_t ptr;    // first byte
  uint64_t end;    // one past last byte
  uint64_t a0;     // ptr rounded down to 16 (lowest address ever loaded)
  uint64_t a1;     // end rounded up to 16
  int32_t rounds;  // 4 KiB rounds covering [ptr, a1)
  int32_t owner;   // lane whose first-round chunk holds ptr
  uint32_t hb;     // ptr - owner's chunk start: bytes the owner zeroes
  uint32_t kt;     // a1 - end: trailing zero bytes to un-shift
  uint32_t inj;    // init state, un-shifted by hb bytes
  uint32_t init_crc;
  bool empty;      // n == 0: Extend(init, "") = init
  // Head mini-round (mini = 1): the first <= 1 KiB of the span, when that is
  // all a first 4 KiB round would hold, is hashed with 16-byte chunks per
  // lane instead (a quarter of the step work) and reduced to one state that
  // the first full round injects at lane 0.  The mini round is round
  // rounds-1; full rounds are rounds-1-mini .. 0.
  int32_t mini;
  int32_t owner_m;  // lane whose 16-byte mini chunk holds ptr
  uint32_t hb_m;    // ptr - that chunk's start (< 16)
  uint32_t inj_m;   // init state, un-shifted by hb_m bytes
};

constexpr uint32_t kMiniBytes = 1024;  // 64 lanes x 16 bytes

// INJ = false leaves the init state un-un-shifted (no LDS read: the
// geometry, and so the first loads, before the table fill); crc_span_inj
// completes it.
template <bool INJ = true>
__device__ __forceinline__ CrcSpan crc_span(const uint8_t* p, uint64_t n, uint32_t init_crc) {
  CrcSpan s;
  s.ptr = reinterpret_cast<uint64_t>(p);
  s.end = s.ptr + n;
  s.a0 = s.ptr & ~15ull;
  s.a1 = (s.end + 15) & ~15ull;
  s.empty = n == 0;
  s.kt = (uint32_t)(s.a1 - s.end);
  s.init_crc = init_crc;
  const uint64_t cover = s.a1 - s.ptr;  // > 0 unless empty
  const uint32_t head = (uint32_t)(cover % kRoundBytes);
  s.mini = !s.empty && head != 0 && head <= kMiniBytes;
  if (s.mini) {
    const int32_t full = (int32_t)(cover / kRoundBytes);
    s.rounds = full + 1;
    const uint32_t lead = kMiniBytes - head;  // mini base .. ptr
    s.owner_m = (int32_t)(lead >> 4);
    s.hb_m = lead & 15u;
    s.inj_m = ~init_crc;
    if (INJ && s.hb_m) s.inj_m = crc_unshift(s.hb_m, s.inj_m);  // wave-uniform branch
    // the first full round starts exactly at the mini round's end
    s.owner = 0;
    s.hb = 0;
    s.inj = 0;
    return s;
  }
  s.owner_m = 64;
  s.hb_m = 0;
  s.inj_m = 0;
  s.rounds = s.empty ? 1 : (int32_t)((cover + kRoundBytes - 1) / kRoundBytes);
  const uint32_t lead = (uint32_t)((uint64_t)kRoundBytes * s.rounds - cover);  // base0 .. ptr
  s.owner = s.empty ? 64 : (int32_t)(lead >> 6);
  s.hb = lead & 63u;
  s.inj = ~init_crc;
  if (INJ && s.hb) s.inj = crc_unshift(s.hb, s.inj);  // wave-uniform branch
  return s;
}
__device__ __forceinline__ void crc_span_inj(CrcSpan& s) {
  if (s.mini && s.hb_m) s.inj_m = crc_unshift(s.hb_m, s.inj_m);  // wave-uniform branches
  if (!s.mini && s.hb) s.inj = crc_unshift(s.hb, s.inj);
}

// ---- transposed loads -------------------------------------------------------
// The chunk layout makes every load instruction touch 16 B of each of the
// 64 chunks (64 lines); a streaming probe (microbench/layout_probe.hip,
// 4 GiB, 16 waves/CU, one round prefetched) reads 6.05 TB/s that way,
// 6.13 TB/s when each instruction reads 1 KiB contiguous, and 6.90 TB/s
// contiguous with non-temporal loads (the chunk layout with nt: 3.82).  So
// every 16-byte load instruction reads one whole contiguous KiB of the round
// (non-temporal), and a transpose inside the wave hands each lane its chunk.
// (Round 5 dropped the lane-quad variant with virtual lanes -- crc_lane_t,
// quad_transpose -- which only the retired uniform-batch kernel could select.)
// Lane l = 16 k + c loads the 16 B at 1024 j + 64 c + 16 k -- each
// instruction reads the round's 1 KiB j whole, in a permuted lane order --
// and a 4 x 4 transpose over (row k, register j) made of two
// v_permlane16_swap and two v_permlane32_swap per 32-bit component (4
// instructions, each moving two registers, instead of 16 DPP moves and
// selects) leaves lane l holding the 64-byte chunk l: the chunk layout
// itself, no virtual lanes.
__device__ __forceinline__ Chunk crc_load_chunk_rt(const CrcSpan& sp, int r, int plane) {
  const uint64_t b = sp.a1 - (uint64_t)kRoundBytes * (r + 1) + 64ull * (plane & 15) + 16ull * (plane >> 4);
  Chunk c;
#pragma unroll
  for (int j = 0; j < 4; j++) c.v[j] = span_load16<true>(b + 1024ull * j);
  return c;
}
__device__ __forceinline__ void row_transpose(Chunk& c) {
#pragma unroll
  for (int d = 0; d < 4; d++) {
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; j++) w[j] = reinterpret_cast<const uint32_t*>(&c.v[j])[d];
    // row bit 0 <-> register bit 0: a's odd rows swap with b's even rows
    auto p = __builtin_amdgcn_permlane16_swap(w[0], w[1], false, false);
    w[0] = p[0];
    w[1] = p[1];
    p = __builtin_amdgcn_permlane16_swap(w[2], w[3], false, false);
    w[2] = p[0];
    w[3] = p[1];
    // row bit 1 <-> register bit 1: a's rows 2-3 swap with b's rows 0-1
    p = __builtin_amdgcn_permlane32_swap(w[0], w[2], false, false);
    w[0] = p[0];
    w[2] = p[1];
    p = __builtin_amdgcn_permlane32_swap(w[1], w[3], false, false);
    w[1] = p[0];
    w[3] = p[1];
#pragma unroll
    for (int j = 0; j < 4; j++) reinterpret_cast<uint32_t*>(&c.v[j])[d] = w[j];
  }
}
__device__ __forceinline__ uint64_t crc_chunk_base(const CrcSpan& sp, int r, const CrcLane& L) {
  return sp.a1 - (uint64_t)kRoundBytes * (r + 1) + (uint64_t)L.lane * kChunkBytes;
}

// Loads stay outside branches so the compiler can count them (a load under
// an exec-masked branch turns later waits into vmcnt(0) and kills the
// prefetch).  In the first round, pieces below a0 read a0 instead (their
// data is discarded); only the address computation is branched, uniformly.
// T = transposed loads (see crc_load_chunk_rt): full rounds read 1 KiB
// contiguous per instruction, non-temporal; row_transpose() before
// crc_round turns them into chunks.
template <bool T = false>
__device__ __forceinline__ Chunk crc_load_chunk(const CrcSpan& sp, int r, const CrcLane& L) {
  uint64_t pa[4];
  if (T) {  // the row-transpose layout (crc_load_chunk_rt; row_transpose before crc_round)
    const uint64_t b = sp.a1 - (uint64_t)kRoundBytes * (r + 1) + 64ull * (L.plane & 15) + 16ull * (L.plane >> 4);
#pragma unroll
    for (int j = 0; j < 4; j++) pa[j] = b + 1024ull * j;
  } else {
    const uint64_t cb = crc_chunk_base(sp, r, L);
#pragma unroll
    for (int j = 0; j < 4; j++) pa[j] = cb + 16 * j;
  }
  if (sp.mini && r == sp.rounds - 1) {
    // mini round: lane l's 16 bytes at a1 - 4 KiB * (rounds-1) - 1 KiB + 16 l
    // (all four loads read it: the load count stays fixed for vmcnt)
    uint64_t a = sp.a1 - (uint64_t)kRoundBytes * (sp.rounds - 1) - kMiniBytes + 16ull * L.plane;
    a = a < sp.a0 ? sp.a0 : a;
#pragma unroll
    for (int j = 0; j < 4; j++) pa[j] = a;
  } else if (r == sp.rounds - 1 && (sp.owner > 0 || sp.hb >= 16 || sp.empty)) {
#pragma unroll
    for (int j = 0; j < 4; j++) pa[j] = pa[j] < sp.a0 ? sp.a0 : pa[j];
  }
  Chunk c;
#pragma unroll
  for (int j = 0; j < 4; j++) c.v[j] = span_load16<T>(pa[j]);
  return c;
}

// zero bytes [0, hb) of a chunk (hb < 64): the owner lane's bytes before ptr
__device__ __forceinline__ void crc_zero_head(Chunk& c, uint32_t hb) {
#pragma unroll
  for (int j = 0; j < 4; j++) {
    uint32_t* w = reinterpret_cast<uint32_t*>(&c.v[j]);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int b = 16 * j + 4 * q;  // first byte of this word
      const int z = (int)hb - b;     // bytes of this word to zero
      w[q] = z <= 0 ? w[q] : z >= 4 ? 0u : w[q] & (0xFFFFFFFFu << (8 * z));
    }
  }
}
// keep the first `keep` (1..15) bytes of a 16-byte piece
__device__ __forceinline__ void crc_keep_head_bytes(uint4& v, uint32_t keep) {
  uint32_t* w = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int k = (int)keep - 4 * q;
    w[q] = k >= 4 ? w[q] : k <= 0 ? 0u : w[q] & (0xFFFFFFFFu >> (8 * (4 - k)));
  }
}

// Advance one lane over its chunk of round r.  The chunk is hashed as
// kCrcChains interleaved chains over consecutive 64/kCrcChains-byte parts,
// so each lane keeps that many independent LDS lookup chains in flight (the
// per-lane work is latency-bound on the chain), joined at the end of the
// round by zshift(part state, bytes after the part) and XOR.
// zshift(s, 16 * (63 - lane)): 64-byte part by the final-shift tables of
// lane 63 - (63 - lane) / 4, the remaining 0..48 bytes by the 16/32-byte maps.
__device__ __forceinline__ uint32_t crc_lane_final16(uint32_t s, const CrcLane& L) {
  const uint32_t d = 63u - (uint32_t)L.plane;  // (mini rounds: physical pieces)
  const uint32_t l4 = (63u - (d >> 2)) << 2;
  uint32_t x[8];
#pragma unroll
  for (int n = 0; n < 8; n++) x[n] = lds_u32(kLdsFinal + n * 4096 + ((((s >> (4 * n)) & 15u) << 8) | l4));
  s = xor3(xor3(x[0], x[1], x[2]), xor3(x[3], x[4], x[5]), x[6] ^ x[7]);
  const uint32_t q = crc_nibmap(kLdsQuarter, s);
  s = (d & 1u) ? q : s;
  const uint32_t h = crc_nibmap(kLdsHalf, s);
  return (d & 2u) ? h : s;
}

// The head mini-round: every lane folds its 16-byte chunk (the first word of
// c); returns the pure state at the mini round's end, wave-uniform.
__device__ __forceinline__ uint32_t crc_mini_round(Chunk c, const CrcSpan& sp, const CrcLane& L) {
  uint32_t* w = reinterpret_cast<uint32_t*>(&c.v[0]);
  if (sp.hb_m && L.plane == sp.owner_m) {  // zero the owner's bytes before ptr
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int z = (int)sp.hb_m - 4 * q;
      w[q] = z <= 0 ? w[q] : z >= 4 ? 0u : w[q] & (0xFFFFFFFFu << (8 * z));
    }
  }
  if (sp.rounds == 1 && sp.kt && L.plane == 63) crc_keep_head_bytes(c.v[0], 16 - sp.kt);  // span ends here
  uint32_t x = L.plane == sp.owner_m ? sp.inj_m : 0u;
  x ^= w[0];
#pragma unroll
  for (int q = 0; q < 4; q++) x = crc_step4x(x, L, q < 3 ? w[q + 1] : 0u);
  x = L.plane < sp.owner_m ? 0u : x;
  if (sp.owner_m == 63) return readlane_u32(x, 63);  // one chunk: already at the end
  return wave_xor32(crc_lane_final16(x, L));
}

__device__ __forceinline__ uint32_t crc_round(uint32_t s, Chunk c, const CrcSpan& sp, int r, const CrcLane& L) {
  if (sp.mini && r == sp.rounds - 1) return crc_mini_round(c, sp, L);  // wave-uniform
  const bool first = r == sp.rounds - 1 - sp.mini;                       // wave-uniform
  uint32_t x[kCrcChains];
  if (first && sp.mini) {
    x[0] = L.lane == 0 ? s : 0u;  // the mini round's state, at lane 0's chunk start
  } else if (first) {
    x[0] = L.lane == sp.owner ? sp.inj : 0u;
    if (sp.hb && L.lane == sp.owner) crc_zero_head(c, sp.hb);  // one lane, unaligned starts
  } else {
    x[0] = crc_nibmap(kLdsGap, s);
  }
  if (sp.kt && r == 0 && L.lane == 63) crc_keep_head_bytes(c.v[3], 16 - sp.kt);  // unaligned end
#pragma unroll
  for (int q = 1; q < kCrcChains; q++) x[q] = 0;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&c.v[0]);
  constexpr int kWords = 16 / kCrcChains;  // words per chain
#pragma unroll
  for (int q = 0; q < kCrcChains; q++) x[q] ^= w[q * kWords];
#pragma unroll
  for (int i = 0; i < kWords; i++) {
#pragma unroll
    for (int q = 0; q < kCrcChains; q++) x[q] = crc_step4x(x[q], L, i + 1 < kWords ? w[q * kWords + i + 1] : 0u);
  }
  if (kCrcChains == 1) {
    s = x[0];
  } else if (kCrcChains == 2) {
    s = crc_nibmap(kLdsHalf, x[0]) ^ x[1];
  } else {
    const uint32_t t0 = crc_nibmap(kLdsQuarter, x[0]) ^ x[1];
    const uint32_t t1 = crc_nibmap(kLdsQuarter, x[2]) ^ x[3];
    s = crc_nibmap(kLdsHalf, t0) ^ t1;
  }
  if (first && !sp.mini) s = L.lane < sp.owner ? 0u : s;  // chunks wholly before the span
  return s;
}

// Combine the lanes' states into the span's CRC (Extend semantics).  Every
// lane returns the same value.
__device__ __forceinline__ uint32_t crc_finish(uint32_t s, const CrcSpan& sp, const CrcLane& L) {
  // a span that was only a mini round is already reduced
  uint32_t p = (sp.mini && sp.rounds == 1) ? s : wave_xor32(crc_lane_final(s, L));
  if (sp.kt) p = crc_unshift(sp.kt, p);
  return sp.empty ? sp.init_crc : ~p;
}

// CRC Extend by one byte on a finished CRC value (all lanes identical):
// eight shift-and-reduce steps, no table, so it works under every driver's
// LDS image (the unit driver's has no ext1 map).
__device__ __forceinline__ uint32_t crc_extend_byte(uint32_t crc, uint8_t b) {
  uint32_t c = ~crc ^ (uint32_t)b;
#pragma unroll
  for (int k = 0; k < 8; k++) c = (c >> 1) ^ (kCrc32cPoly & (0u - (c & 1u)));
  return ~c;
}

__device__ __forceinline__ uint32_t crc_mask(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }


typedef __attribute__((address_space(3))) uint32_t lds_u32_t;
typedef __attribute__((address_space(3))) uint64_t lds_u64_t;
__device__ __forceinline__ lds_u32_t* lds_p32(uint32_t off) { return reinterpret_cast<lds_u32_t*>(static_cast<size_t>(off)); }
__device__ __forceinline__ lds_u64_t* lds_p64(uint32_t off) { return reinterpret_cast<lds_u64_t*>(static_cast<size_t>(off)); }

// (Round 5 retired the uniform-batch driver, crc_uniform_driver /
// k_crc_uniform: uniform batches run on k_crc_ragged like any other, whose
// body/head and row drivers measured faster at every length -- 4 KiB
// blocks 0.784 -> 0.805 of peak, whole-file 64 KiB pieces 0.787 -> 0.815,
// 512 B 0.157 -> 0.596; profiles/r5/uniform_retired/.)

// ---------------------------------------------------------------------------
// Row driver: one 16-lane ROW per span, four spans per wave.
//
// The wave driver above reduces every span across the whole wave (lane-final
// shift, wave XOR, epilogue): for spans of a few hundred bytes that per-span
// chain, not bandwidth, sets the rate (a flat ~2.2 G spans/s per GPU,
// DESIGN.md §10).  Here each row of 16 lanes owns a span and walks it in
// 1 KiB rounds anchored at the span's 16-byte-aligned end (lane c of the row
// owns the 64-byte chunk at round_base + 64 c, the same 4-byte table step as
// the wave driver), so four spans are reduced side by side by one
// instruction stream: the lane-final shift zshift(s, 64 (15 - c)) is the
// wave table's lane 48 + c, the row XOR is a 4-step DPP butterfly, and the
// head/tail/init handling of crc_round runs per row (vector values instead
// of wave-uniform ones).  Rows take spans from an LDS ticket of their
// workgroup's share -- see row_desc_stage for the LDS-staged descriptor feed --
// and every data load is issued unconditionally (exec-masked loads would
// force vmcnt(0) waits, see crc_load_chunk).
// LDS: the wave driver's image plus the 960-byte row gap map, the init
// tables and the descriptor cache, all below the step tables.
constexpr uint32_t kLdsRowGap = kLdsLowEnd;  // 3 x 512 B (W = 4, 8, 16), below the step tables
template <int W, int P = 4>
constexpr uint32_t row_gap_off() {
  // P = 5 (80-byte chunks, W = 16 only): the kernel overwrites the W = 4 map
  // with CrcTables::gap80 (wal_write_rows)
  return P == 5 ? kLdsRowGap : kLdsRowGap + 512u * (W == 4 ? 0 : W == 8 ? 1 : 2);
}
// How the row driver gets a span's CRC init (Extend's init_crc):
//   kInitZero  -- always 0 (Value): ~init is injected from a 64-entry LDS
//                 table of unshift(~0, hb) instead of an 8-lookup map;
//   kInitTyped -- init = type_crc[key & 15] (WAL records: key = the record
//                 type byte), from a [16][64] LDS table built at kernel start;
//   kInitArray -- arbitrary per-span init (key = the init itself).
// init_key(i) is the only load; the table lookup happens when the span is
// set up, one iteration later, so no load depends on another in flight.
enum RowInit : int { kInitZero = 0, kInitTyped = 1, kInitArray = 2 };
constexpr uint32_t kLdsRowInj = kLdsRowGap + 1536;    // [16][64] u32: unshift(~init_t, k)
constexpr uint32_t kLdsRowInit = kLdsRowInj + 4096;   // [16] u32: init_t
static_assert(kLdsRowInit + 64 <= kLdsStep, "row tables must fit below the step tables");
// descriptor cache of the row feed (row_desc_stage) and its ticket
constexpr uint32_t kRowDescCache = 1528;
constexpr uint32_t kLdsRowDesc = kLdsRowInit + 64;                   // 16 B x 1536
constexpr uint32_t kLdsRowTicket = kLdsRowDesc + 16 * kRowDescCache;  // u32
// byte masks of one 16-byte piece: head[h] keeps bytes >= h, tail[k] keeps
// the first 16 - k bytes (h, k < 16), as 4 words
constexpr uint32_t kLdsRowMaskHead = kLdsRowTicket + 64;
constexpr uint32_t kLdsRowMaskTail = kLdsRowMaskHead + 256;
static_assert(kLdsRowMaskTail + 256 <= kLdsStep, "row tables must fit below the step tables");
static_assert(kLdsRowTicket + 32 <= kLdsRowMaskHead, "ticket + totals");
static_assert(offsetof(CrcTables, gap_row) - offsetof(CrcTables, unshift) == kMaxUnshift * 512, "layout");
static_assert(sizeof(((CrcTables*)nullptr)->gap_row[0]) == 512, "one row gap map = 32 slots");

__device__ __forceinline__ bool wave_any(bool p) { return __ballot(p) != 0ull; }

// The wave driver's image plus the row gap maps of every width.
__device__ __forceinline__ void crc_fill_rows(uint8_t* lds, const CrcTables* __restrict__ g) {
  CrcFill f;
  crc_fill_load<true>(f, g);
  const int t = threadIdx.x;
  const uint4* rg = reinterpret_cast<const uint4*>(&g->gap_row[0][0][0]);
  const uint4 x = rg[t < 96 ? t : 0];
  crc_fill_store<true>(f, lds);
  if (t < 96) reinterpret_cast<uint4*>(lds + kLdsRowGap)[t] = x;
}

struct RowSpan {
  uint64_t ptr;    // first byte
  uint64_t a0;     // ptr rounded down to 16
  uint64_t a1;     // end rounded up to 16
  uint32_t n;      // bytes
  int32_t rounds;  // 64 W-byte row rounds covering [ptr, a1)
  int32_t owner;   // row lane whose first-round chunk holds ptr (W: none)
  uint32_t hb;     // ptr - owner's chunk start (< 64)
  uint32_t kt;     // a1 - end (< 16)
  uint32_t inj;    // ~init un-shifted by hb bytes
  uint32_t init;
};

// Per-workgroup init tables (after the LDS fill): inj[t][k] =
// unshift(~init_t, k) and init_t, with init_t = the op's typed init for
// kInitTyped ops and 0 otherwise (row t = 0 then serves kInitZero).
template <class Op>
__device__ __forceinline__ void row_init_tables(const Op& op) {
  const uint32_t t = threadIdx.x;  // kCrcBlock = 1024 = 16 x 64 entries
  const uint32_t init = Op::kTypedInit ? op.typed_init(t >> 6) : 0u;
  *lds_p32(kLdsRowInj + 4 * t) = crc_unshift(t & 63, ~init);
  if ((t & 63) == 0) *lds_p32(kLdsRowInit + 4 * (t >> 6)) = init;
  if (t < 128) {
    const int h = (int)(t >> 2) & 15, k = (int)(t & 3);
    uint32_t m;
    if (t < 64) {  // keep bytes >= h of the piece
      const int d = h - 4 * k;
      m = d <= 0 ? 0xFFFFFFFFu : d >= 4 ? 0u : 0xFFFFFFFFu << (8 * d);
      *lds_p32(kLdsRowMaskHead + 4 * (t & 63)) = m;
    } else {  // keep the first 16 - h bytes
      const int keep = 16 - h - 4 * k;
      m = keep >= 4 ? 0xFFFFFFFFu : keep <= 0 ? 0u : 0xFFFFFFFFu >> (8 * (4 - keep));
      *lds_p32(kLdsRowMaskTail + 4 * (t & 63)) = m;
    }
  }
}

// P pieces per lane chunk: Q = 16 P bytes per lane, rounds of Q W bytes.
// P = 4: inj = unshift(~init, hb), injected at the chunk's start.  P = 5: hb
// can reach 79, past the 64-entry init table, so inj = unshift(~init,
// hb & 15) and row_round injects it at piece hb >> 4 instead (the owner's
// pieces before it are zero, so the two are the same state).
template <int W, int P = 4>
__device__ __forceinline__ RowSpan row_span(uint64_t ptr, uint32_t n, uint32_t key, int kind) {
  static_assert(P == 4 || (P == 5 && W == 16), "chunk pieces");
  constexpr uint32_t Q = 16u * P, R = Q * W;
  RowSpan s;
  s.ptr = ptr;
  s.n = n;
  s.a0 = ptr & ~15ull;
  s.a1 = (ptr + n + 15) & ~15ull;
  s.kt = (uint32_t)(s.a1 - (ptr + n));
  const uint32_t cover = (uint32_t)(s.a1 - ptr);
  s.rounds = n == 0 ? 1 : (int32_t)((cover + R - 1) / R);
  const uint32_t lead = R * (uint32_t)s.rounds - cover;
  s.owner = n == 0 ? W : (int32_t)(lead / Q);
  s.hb = lead % Q;
  const uint32_t hk = P == 4 ? s.hb : (s.hb & 15u);
  if (kind == kInitArray) {  // wave-uniform
    s.init = key;
    s.inj = crc_unshift(hk, ~key);  // unshift by 0 is the identity
  } else {
    const uint32_t t = kind == kInitTyped ? (key & 15u) : 0u;
    s.inj = *lds_p32(kLdsRowInj + 4 * (t * 64 + hk));
    s.init = *lds_p32(kLdsRowInit + 4 * t);
  }
  return s;
}

__device__ __forceinline__ RowSpan row_span_sel(bool a, const RowSpan& x, const RowSpan& y) {
  RowSpan s;
  s.ptr = a ? x.ptr : y.ptr;
  s.a0 = a ? x.a0 : y.a0;
  s.a1 = a ? x.a1 : y.a1;
  s.n = a ? x.n : y.n;
  s.rounds = a ? x.rounds : y.rounds;
  s.owner = a ? x.owner : y.owner;
  s.hb = a ? x.hb : y.hb;
  s.kt = a ? x.kt : y.kt;
  s.inj = a ? x.inj : y.inj;
  s.init = a ? x.init : y.init;
  return s;
}

// Row round r of a span: lane c's 64-byte chunk.  In the first round the
// pieces wholly before a0 read the zero piece `zp` instead, so they need no
// masking (and lanes before the owner hash zeros); only the piece at a0
// keeps ptr - a0 < 16 bytes of another span to mask (row_round).
template <int W, int P = 4>
__device__ __forceinline__ ChunkN<P> row_load_chunk(const RowSpan& sp, int r, uint32_t c, uint64_t zp) {
  constexpr uint64_t Q = 16u * P;
  const uint64_t b = sp.a1 - Q * W * (uint32_t)(r + 1) + Q * c;
  const bool first = r == sp.rounds - 1;
  // first round: b >= a0 - Q W, so the low words give the exact offset
  const int32_t rel = first ? (int32_t)((uint32_t)b - (uint32_t)sp.a0) : 0;
  ChunkN<P> ch;
#pragma unroll
  for (int j = 0; j < P; j++) {
    const uint64_t a = rel < -16 * j ? zp : b + 16ull * j;
    ch.v[j] = span_load16<false>(a);
  }
  return ch;
}

__device__ __forceinline__ uint4 lds_u32x4(uint32_t off) {
  const span_u32x4 v = *reinterpret_cast<__attribute__((address_space(3))) const span_u32x4*>(static_cast<size_t>(off));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void and4(uint4& v, const uint4& m) {
  v.x &= m.x;
  v.y &= m.y;
  v.z &= m.z;
  v.w &= m.w;
}

template <int W, int P = 4>
__device__ __forceinline__ uint32_t row_round(uint32_t s, ChunkN<P> ch, const RowSpan& sp, int r, uint32_t c,
                                              const CrcLane& L) {
  const bool first = r == sp.rounds - 1;
  const bool own = (int32_t)c == sp.owner;
  // Unconditional (no branch, so no phi copies of the chunk): the owner's
  // a0 piece -- its piece hb >> 4, the ones before it are zero -- keeps the
  // bytes from ptr on, w & (m | ~sel) with sel = all-ones on that piece (one
  // bitop3 per word); lane 15's last piece keeps the bytes before the end.
  const uint32_t h0 = (uint32_t)sp.ptr & 15u;  // bytes of the a0 piece before ptr
  const uint4 mh = lds_u32x4(kLdsRowMaskHead + 16 * h0);
  const uint4 mt = lds_u32x4(kLdsRowMaskTail + 16 * ((r == 0 && c == W - 1) ? sp.kt : 0u));
  const uint32_t pa = (first && own) ? sp.hb >> 4 : (uint32_t)P;
  uint32_t sels[P];
#pragma unroll
  for (int j = 0; j < P; j++) {
    const uint32_t sel = (uint32_t)j == pa ? ~0u : 0u;
    sels[j] = sel;
    ch.v[j].x = __builtin_amdgcn_bitop3_b32(ch.v[j].x, mh.x, sel, 0xD0);
    ch.v[j].y = __builtin_amdgcn_bitop3_b32(ch.v[j].y, mh.y, sel, 0xD0);
    ch.v[j].z = __builtin_amdgcn_bitop3_b32(ch.v[j].z, mh.z, sel, 0xD0);
    ch.v[j].w = __builtin_amdgcn_bitop3_b32(ch.v[j].w, mh.w, sel, 0xD0);
  }
  and4(ch.v[P - 1], mt);
  uint32_t gap = s;  // W = 1: a lane's rounds are adjacent (no gap to shift over)
  if constexpr (W > 1) {
    gap = 0;
    if (wave_any(!first)) gap = crc_nibmap(row_gap_off<W, P>(), s);
  }
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&ch.v[0]);
  if constexpr (P == 4) {
    uint32_t x = first ? (own ? sp.inj : 0u) : gap;
    x ^= w[0];
#pragma unroll
    for (int k = 0; k < 16; k++) x = crc_step4x(x, L, k < 15 ? w[k + 1] : 0u);
    return x;
  } else {
    // P = 5: the init enters at the owner's piece pa (sels[pa] is all-ones)
    const uint32_t inj = sp.inj;
    uint32_t x = (first ? 0u : gap) ^ w[0] ^ (sels[0] & inj);
#pragma unroll
    for (int k = 0; k < 4 * P; k++) {
      uint32_t nw = 0u;
      if (k + 1 < 4 * P) nw = ((k + 1) & 3) ? w[k + 1] : (w[k + 1] ^ (sels[(k + 1) >> 2] & inj));
      x = crc_step4x(x, L, nw);
    }
    return x;
  }
}

// XOR over the W lanes of each row, in every lane of the row (DPP).
template <int W>
__device__ __forceinline__ uint32_t row_xor32(uint32_t v) {
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);  // quad_perm [1,0,3,2]
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true);  // quad_perm [2,3,0,1]
  if (W >= 8) v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, true);  // row_half_mirror
  if (W >= 16) v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, true);  // row_mirror
  return v;
}

// zshift(s, 64*(63-lane)) with the per-lane tables, column lane4 = lane * 4.
__device__ __forceinline__ uint32_t crc_lane_final4(uint32_t s, uint32_t lane4) {
  uint32_t x[8];
#pragma unroll
  for (int n = 0; n < 8; n++) x[n] = lds_u32(kLdsFinal + n * 4096 + ((((s >> (4 * n)) & 15u) << 8) | lane4));
  return xor3(xor3(x[0], x[1], x[2]), xor3(x[3], x[4], x[5]), x[6] ^ x[7]);
}
template <int W>
__device__ __forceinline__ uint32_t row_finish4(uint32_t s, const RowSpan& sp, uint32_t lf4) {
  uint32_t p = row_xor32<W>(crc_lane_final4(s, lf4));
  if (wave_any(sp.kt != 0)) p = crc_unshift(sp.kt, p);
  return sp.n == 0 ? sp.init : ~p;
}

// The span's CRC (Extend semantics) in every lane of its row; Lf = the lane
// constants with lane4 = (64 - W + c) * 4 (shift by 64 (W - 1 - c)).
// 4- and 8-lane rows: the shift and the un-shift as one map
// (CrcTables::rowfin4 / rowfin8, copied by crc_rows_windows_w): 8 lookups
// per finish instead of 16, and no un-shift branch.  rowfin4 (32 KiB) goes
// over the lane-final tables, which no row mode but 16-lane rows reads;
// rowfin8 (64 KiB) over those and the un-shift tables, so only for ops
// that never un-shift an init at run time (no per-span init array: the init
// injection tables are built before the copy).
constexpr uint32_t kLdsRowFin4 = kLdsFinal;
template <class Op, class = void>
struct op_array_init : std::false_type {};
template <class Op>
struct op_array_init<Op, std::void_t<decltype(Op::kArrayInit)>> : std::bool_constant<Op::kArrayInit> {};
template <class Op>
constexpr bool kRowFin8 = !op_array_init<Op>::value;
// The combined map of (lane c, kt) applied to s: 8 nibble lookups in the
// lane-minor layout [kt][n][v][c]; W = 8 splits it by kt over the two 32 KiB
// halves (kt < 8: the lane-final area, else the un-shift area).
template <int W>
__device__ __forceinline__ uint32_t row_finmap(uint32_t s, uint32_t c, uint32_t kt) {
  constexpr uint32_t kMap = 8 * 16 * W * 4;  // bytes per kt
  const uint32_t base = W == 4 ? kLdsFinal + kt * kMap
                               : (kt < 8 ? kLdsFinal : kLdsUnshift) + (kt & 7u) * kMap;
  uint32_t x[8];
#pragma unroll
  for (int n = 0; n < 8; n++) x[n] = lds_u32(base + ((uint32_t)n * 16u + ((s >> (4 * n)) & 15u)) * (W * 4) + 4 * c);
  return xor3(xor3(x[0], x[1], x[2]), xor3(x[3], x[4], x[5]), x[6] ^ x[7]);
}
template <int W, bool FIN8 = false>
__device__ __forceinline__ uint32_t row_finish(uint32_t s, const RowSpan& sp, const CrcLane& Lf) {
  if constexpr (W == 4) {
    const uint32_t c = (Lf.lane4 >> 2) - 60u;  // Lf.lane4 = (64 - W + c) * 4
    const uint32_t p = row_xor32<4>(row_finmap<4>(s, c, sp.kt));
    return sp.n == 0 ? sp.init : ~p;
  }
  if constexpr (W == 8 && FIN8) {
    const uint32_t c = (Lf.lane4 >> 2) - 56u;
    const uint32_t p = row_xor32<8>(row_finmap<8>(s, c, sp.kt));
    return sp.n == 0 ? sp.init : ~p;
  }
  uint32_t p = s;  // W = 1: the lane's state is the span's (no shift, no row XOR)
  if constexpr (W > 1) p = row_xor32<W>(crc_lane_final(s, Lf));
  if (wave_any(sp.kt != 0)) p = crc_unshift(sp.kt, p);
  return sp.n == 0 ? sp.init : ~p;
}

// Descriptor feed of the row driver: a workgroup's share is staged in LDS,
// a window of at most kRowDescCache spans at a time, as 16-byte records
// {off, len, key}; a row takes the next one with an LDS ticket when its span
// ends, one span ahead, so the chunk loads of a new span never wait for a
// descriptor load (every load in the loop is a data load).
// The staging also sums the window's span bytes into the u64 at
// kLdsRowTotal (zeroed here; valid after the next __syncthreads + the
// atomics): the row width is chosen from its mean.
constexpr uint32_t kLdsRowTotal = kLdsRowTicket + 8;  // u64
// A workgroup's share of spans [first, first + count): span first + b + G t
// (interleaved: the grid sweeps the batch front to back together) or, BLK,
// the contiguous range [count b / G, count (b + 1) / G) (neighbouring spans
// on one CU, so the cache lines two spans share stay in one XCD's L2).
struct RowShare {
  uint32_t start, stride, n;
  __device__ uint32_t idx(uint32_t t) const { return start + stride * t; }
};
template <bool BLK>
__device__ __forceinline__ RowShare row_share(uint32_t first, uint32_t count) {
  const uint32_t G = gridDim.x, b = blockIdx.x;
  if (BLK) {
    const uint32_t lo = (uint32_t)((uint64_t)count * b / G), hi = (uint32_t)((uint64_t)count * (b + 1) / G);
    return {first + lo, 1u, hi - lo};
  }
  return {first + b, G, (count - b + G - 1) / G};
}

template <class Op>
__device__ __forceinline__ void row_desc_stage(const Op& op, const RowShare& sh, bool total) {
  const uint32_t n = sh.n;
  uint64_t sum = 0;
  for (uint32_t t = threadIdx.x; t < n; t += blockDim.x) {
    const uint32_t i = sh.idx(t);
    const uint64_t off = op.off(i);
    const uint32_t len = (uint32_t)op.len(i);
    sum += len;
    const span_u32x4 d = {(uint32_t)off, (uint32_t)(off >> 32), len, op.init_key(i)};
    *reinterpret_cast<__attribute__((address_space(3))) span_u32x4*>(static_cast<size_t>(kLdsRowDesc + 16 * t)) = d;
  }
  if (threadIdx.x == 0) *lds_p32(kLdsRowTicket) = 0;
  if (total) {
    // wave sums, then one LDS atomic per wave (after a barrier zeroes them)
    for (int m = 32; m >= 1; m >>= 1) sum += __shfl_xor(sum, m, 64);
    if (threadIdx.x == 0) *lds_p64(kLdsRowTotal) = 0;
    __syncthreads();
    if ((threadIdx.x & 63) == 0)
      __hip_atomic_fetch_add(lds_p64(kLdsRowTotal), sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

// Next ticket for every row that asks (take, row-uniform): lane 0 of the row
// takes it, the row reads it.
template <int W>
__device__ __forceinline__ uint32_t row_ticket(bool take) {
  uint32_t t = 0;
  if ((threadIdx.x & (W - 1)) == 0 && take)
    t = __hip_atomic_fetch_add(lds_p32(kLdsRowTicket), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)((threadIdx.x & (63u & ~(uint32_t)(W - 1))) << 2), (int)t);
}

// Descriptor of ticket t; t >= share (no span left) reads slot 0, a valid
// span of the share (slots past the share hold no descriptor).
__device__ __forceinline__ uint4 row_desc(uint32_t t, uint32_t share) {
  const span_u32x4 v = *reinterpret_cast<__attribute__((address_space(3))) const span_u32x4*>(
      static_cast<size_t>(kLdsRowDesc + 16 * (t < share ? t : 0)));
  return make_uint4(v.x, v.y, v.z, v.w);
}

// LDS prologue of the row (and auto) kernels: tables, descriptors, init
// tables; ends with a barrier.
template <class Op>
__device__ __forceinline__ void crc_rows_prologue(const Op& op, const RowShare& sh, uint8_t* lds,
                                                  const CrcTables* __restrict__ g, bool total) {
  crc_fill_rows(lds, g);
  row_desc_stage<Op>(op, sh, total);
  __syncthreads();
  row_init_tables(op);
  __syncthreads();
}

// A row's place in its share: span ticket t (slot i), its descriptor-derived
// geometry sp, round r; the next ticket nt (descriptor nd, prefetched).
struct RowState {
  RowSpan sp;
  uint4 nd;
  uint32_t i, nt;
  int32_t r;
  uint32_t live;
};
template <class Op>
struct RowCtx {
  const Op& op;
  const RowShare& sh;
  uint64_t base, zp;
  uint32_t share, c;
  int kind;
  const CrcLane &L, &Lf;
};
// One iteration of the row loop: round A.r of A's span (chunk ca, loaded)
// is folded while B -- the row's next round, or its next span's first --
// is set up and its chunk cb loaded.  Returns whether any row goes on.
template <class Op, int W>
__device__ __forceinline__ bool crc_rows_step(const RowCtx<Op>& x, const RowState& A, const Chunk& ca,
                                              const typename Op::Pre& pa, RowState& B, Chunk& cb,
                                              typename Op::Pre& pb, uint32_t& s) {
  const bool live = A.live != 0;
  const bool last = A.r == 0;  // this round ends the row's span
  const bool go = live && (!last || A.nt < x.share);
  // set up unconditionally (rows that are not switching discard it): a
  // branch would merge the span's registers through copies every round
  const RowSpan nsp = row_span<W>(x.base + (((uint64_t)A.nd.y << 32) | A.nd.x), A.nd.z, A.nd.w, x.kind);
  const bool sw = go && last;  // the row moves to its next span
  B.sp = row_span_sel(sw, nsp, A.sp);
  B.r = go ? (last ? nsp.rounds - 1 : A.r - 1) : A.r;
  B.i = sw ? x.sh.idx(A.nt) : A.i;
  // unconditional: the next unit's chunk and epilogue inputs
  cb = row_load_chunk<W>(B.sp, B.r, x.c, x.zp);
  pb = x.op.pre(B.i, B.sp.ptr, B.sp.n);
  // rows that moved on take the ticket after (LDS only)
  B.nt = A.nt;
  B.nd = A.nd;
  if (wave_any(sw)) {
    const uint32_t tk = row_ticket<W>(sw);
    if (sw) {
      B.nt = tk;
      B.nd = row_desc(tk, x.share);
    }
  }
  B.live = go ? 1u : 0u;
  s = row_round<W>(s, ca, A.sp, A.r, x.c, x.L);
  if (wave_any(live && last))
    x.op.finish(A.i, row_finish<W, kRowFin8<Op>>(s, A.sp, x.Lf), pa, live && last && x.c == 0);
  return wave_any(go);
}

template <class Op, int W>
__device__ __forceinline__ void crc_rows_loop(const Op& op, const RowShare& sh, const CrcTables* __restrict__ g) {
  static_assert(W == 1 || W == 4 || W == 8 || W == 16, "row width");
  const CrcLane L = crc_lane();
  CrcLane Lf = L;
  const uint32_t c = threadIdx.x & (W - 1);
  Lf.lane4 = (64u - W + c) << 2;
  const uint32_t share = sh.n;  // this workgroup's spans
  if (share == 0) return;        // (slot 0 would be read unstaged)
  const RowCtx<Op> x{op, sh, reinterpret_cast<uint64_t>(op.base()), reinterpret_cast<uint64_t>(&g->zero16[0]),
                     share, c, op.init_kind(), L, Lf};
  // the row's current span (ticket t) and the next one (ticket nt, prefetched)
  RowState A;
  const uint32_t t = row_ticket<W>(true);
  A.live = t < share ? 1u : 0u;
  const uint4 d = row_desc(t, share);
  A.i = sh.idx(A.live ? t : 0);
  A.sp = row_span<W>(x.base + (((uint64_t)d.y << 32) | d.x), d.z, d.w, x.kind);
  A.r = A.sp.rounds - 1;
  Chunk ca = row_load_chunk<W>(A.sp, A.r, c, x.zp);
  typename Op::Pre pa = op.pre(A.i, A.sp.ptr, A.sp.n);
  A.nt = row_ticket<W>(true);
  A.nd = row_desc(A.nt, share);
  uint32_t s = 0;
  // unrolled twice: the two iterations' chunks, spans and epilogue inputs
  // swap register names instead of being copied every round (the body/head
  // driver's body loop measured +7 % for the same change).  The loop's
  // breaks merge at its header, where the compiler then drains every load in
  // flight once per iteration (vmcnt(0)): that drain turned out to pace the
  // loads well -- with none, 16-lane rows of 1 KiB spans measured 0.649 ->
  // 0.559 of peak, one per step 0.616; 8-lane rows gain 1-2 % with one per
  // four steps (200-500-B spans 0.538 -> 0.549), 16-lane rows lose 5-8 %
  // (profiles/r5/rows_pace/).
  RowState B;
  Chunk cb;
  typename Op::Pre pb;
  for (;;) {
    if (!crc_rows_step<Op, W>(x, A, ca, pa, B, cb, pb, s)) break;
    if (!crc_rows_step<Op, W>(x, B, cb, pb, A, ca, pa, s)) break;
    if constexpr (W == 8) {
      if (!crc_rows_step<Op, W>(x, A, ca, pa, B, cb, pb, s)) break;
      if (!crc_rows_step<Op, W>(x, B, cb, pb, A, ca, pa, s)) break;
    }
  }
}

// ---------------------------------------------------------------------------
// Ragged batches: one kernel over the whole batch (k_crc_ragged), contiguous
// shares, and every workgroup runs its share on the row drivers (below) when
// the share's spans average less than kAutoLongMin bytes, else on the
// body/head driver (mck_crc_bh.hpp).  The choice is made from a fixed sample
// of the share's lengths (crc_share_long).  (The host cannot choose: ragged
// lengths live on the device.)  4096: below one whole 4 KiB round a span is
// all head to the body/head driver, whose heads run on 4-lane rows -- spans
// of 2000-4000 B measured 0.44-0.45 there against 0.59-0.64 on 16-lane rows,
// while from 4 KiB + jitter on the body/head driver wins (4100-4400 B 0.739
// vs 0.576, 4096 B 0.819 vs 0.642; microbench/rows_width.py,
// profiles/r5/rows_width/sweep3.txt, sweep4.txt; round 4's bound was 2560).
constexpr uint32_t kAutoLongMin = 4096;    // mean span bytes
constexpr uint32_t kAutoRows1Max = 80;     // one lane per span below ~80 B
constexpr uint32_t kAutoRows4Max = 240;    // 4-lane rows up to 240 B
constexpr uint32_t kAutoRows8Max = 640;    // 8-lane rows up to 640 B, 16-lane rows above
template <class Op>
__device__ __forceinline__ bool crc_share_long(const Op& op, const RowShare& sh) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t m = sh.n < 64 ? sh.n : 64u;  // spans k n / m, k < m
  uint64_t len = 0;
  if (lane < m) len = op.len(sh.idx((uint32_t)((uint64_t)lane * sh.n / m)));
  for (int d = 32; d >= 1; d >>= 1) len += __shfl_xor(len, d, 64);
  return len >= (uint64_t)kAutoLongMin * m;
}

// The row drivers over a share, in windows of at most kRowDescCache spans
// (one launch per batch; the table image is filled once).  The width is
// chosen once per share, from its first window's mean span: one lane per
// span below ~80 B (20-100 B: 0.16-0.19 vs 0.09 of peak on 8-lane rows,
// whose 512-B rounds are mostly padding there), 4-lane rows up to 240 B,
// 8-lane rows up to 640 B, 16-lane rows above.  Round 5's sweep with every
// width forced (microbench/rows_width.py, profiles/r5/rows_width/): 4-lane
// rows win at a 200-B mean (100-300 B: 0.421 vs 0.386) but 8-lane rows from
// ~275 B on (150-400 B 0.489 vs 0.450, 250-350 B 0.511 vs 0.454, 200-500 B
// 0.555 vs 0.458: round 4's 384-B bound was too high); 8 vs 16 lanes
// depends on the spread around a 600-700-B mean (400-800 B: 16 lanes 0.534
// vs 0.519; 100-1100 B WAL records: 8 lanes 0.511 vs 0.492).  (The window loop sits inside each width's branch: a
// loop around all four widths kept every width's lane constants live and
// spilled 76-132 B per lane.)  force: 0 = by length, 2 = rows16, 3 = rows8,
// 5 = rows4, 6 = one lane per span (test hook).
template <class Op, int W>
__device__ __forceinline__ void crc_rows_windows_w(const Op& op, const RowShare& share, uint32_t nwin,
                                                   const CrcTables* __restrict__ g) {
  const uint32_t n = share.n;
  if constexpr (W == 4 || (W == 8 && kRowFin8<Op>)) {  // the combined finish maps (row_finish)
    static_assert(sizeof(g->rowfin4) == 32768 && kLdsRowFin4 + 32768 <= kLdsGap, "rowfin4 fits the lane-final area");
    static_assert(sizeof(g->rowfin8) == 65536 && kLdsUnshift + 32768 <= kCrcLdsBytes, "rowfin8 halves fit");
    const uint4* src = reinterpret_cast<const uint4*>(W == 4 ? &g->rowfin4[0][0][0][0] : &g->rowfin8[0][0][0][0]);
    constexpr int kPer = W == 4 ? 2 : 4;  // 16-byte slots per thread
    uint4 v[kPer];
#pragma unroll
    for (int k = 0; k < kPer; k++) v[k] = src[threadIdx.x + kCrcBlock * k];
    __syncthreads();  // every reader of the tables overwritten here is done (the init tables are built)
#pragma unroll
    for (int k = 0; k < kPer; k++) {
      const uint32_t slot = threadIdx.x + kCrcBlock * k;  // 2048 slots = 32 KiB per half
      const uint32_t off = slot < 2048 ? kLdsFinal + 16 * slot : kLdsUnshift + 16 * (slot - 2048);
      *reinterpret_cast<__attribute__((address_space(3))) span_u32x4*>(static_cast<size_t>(off)) =
          span_u32x4{v[k].x, v[k].y, v[k].z, v[k].w};
    }
    __syncthreads();
  }
  for (uint32_t wi = 0; wi < nwin; wi++) {
    const uint32_t w0 = (uint32_t)((uint64_t)n * wi / nwin), w1 = (uint32_t)((uint64_t)n * (wi + 1) / nwin);
    const RowShare sh{share.start + share.stride * w0, share.stride, w1 - w0};
    if (wi) {  // window 0 was staged by the caller
      __syncthreads();  // every row is done with the previous window's slots
      row_desc_stage<Op>(op, sh, false);
      __syncthreads();
    }
    crc_rows_loop<Op, W>(op, sh, g);
  }
}
template <class Op>
__device__ __forceinline__ void crc_rows_windows(const Op& op, const RowShare& share, uint8_t* lds,
                                                 const CrcTables* __restrict__ g, int force) {
  const uint32_t n = share.n;
  const uint32_t nwin = (n + kRowDescCache - 1) / kRowDescCache;
  const RowShare sh0{share.start, share.stride, (uint32_t)((uint64_t)n / nwin)};
  crc_rows_prologue<Op>(op, sh0, lds, g, true);
  const uint64_t mean = *lds_p64(kLdsRowTotal) / sh0.n;
  const int mode = force ? force
                         : mean <= kAutoRows1Max ? 6
                         : mean <= kAutoRows4Max ? 5
                         : mean <= kAutoRows8Max ? 3
                                                 : 2;
  if (mode == 6)
    crc_rows_windows_w<Op, 1>(op, share, nwin, g);
  else if (mode == 5)
    crc_rows_windows_w<Op, 4>(op, share, nwin, g);
  else if (mode == 3)
    crc_rows_windows_w<Op, 8>(op, share, nwin, g);
  else
    crc_rows_windows_w<Op, 16>(op, share, nwin, g);
}

}  // namespace mck
