// mck_block.hpp -- per-KV protection of uncompressed block entries
// (SURVEY.md 8f row 4): table/block_based/block.cc:1091-1222
// Block::Initialize{Data,Index,MetaIndex}BlockProtectionInfo.
//
// A block is prefix-compressed: an entry's key is the previous key's first
// `shared` bytes plus its own `non_shared` bytes, and only restart points
// (every block_restart_interval-th entry, shared == 0) start from nothing.
// One THREAD per block walks it in order, as the reference's
// SeekToFirst/Next loop does (64 blocks per wave keep every lane busy and
// the dependent header reads of thousands of blocks in flight), in passes:
//
//   k_block_layout_t  entry count, reassembled key bytes, restart interval
//                     and status per block; the exclusive scans
//                     (k_blk_scan_*) give each block its key index base and
//                     key-arena base
//   k_block_kv_t      walks again, reassembling every key in a per-thread
//                     LDS buffer: ProtectKV(key, value).Encode(prot_bytes)
//                     for every entry, values over 240 B left to
//   k_block_long_rows the long-value list in key order, XXPH3 on the XXH3
//                     row loop (16-lane rows, 16-byte loads)
//
// Entry k of a block lands at key index key_base[block] + k, in the order the
// reference's SeekToFirst/Next loop generates them (:1116-1123).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mck {

enum { kBlkData = 0, kBlkIndex = 1, kBlkIndexDelta = 2, kBlkIndexDeltaFk = 3, kBlkMeta = 4 };
enum { kBlkOk = 0, kBlkBadContents = 1, kBlkBadEntry = 2, kBlkBadRestarts = 3 };

typedef __attribute__((address_space(1))) const uint32_t gbl_u32u_t;

__device__ __forceinline__ uint32_t blk_u8(const uint8_t* p) {
  return *reinterpret_cast<gbl_u8_t*>(reinterpret_cast<uint64_t>(p));
}
// LE32 at any byte address (unaligned global load)
__device__ __forceinline__ uint32_t blk_u32(const uint8_t* p) {
  return *reinterpret_cast<gbl_u32u_t*>(reinterpret_cast<uint64_t>(p));
}

// block.cc:994-1083 NumRestarts / IndexType / Block::Block: restart array
// offset `ro` and restart count `nr`; ok = false is the constructor's error
// marker (size_ = 0) or NewDataIterator's "bad block contents" (rd_header).
struct BlkHdr {
  uint32_t ro, nr;
  bool ok;
};
// ---- byte readers: a block (or key area) staged in LDS, or in global memory
// Offsets are relative to the block's first byte.  The LDS slot holds the
// 16-byte-aligned global chunks covering the block; `head` = the block's
// offset in its first chunk.  Unaligned dword/qword reads are assembled from
// aligned LDS dwords with v_alignbyte (the slot is padded past its end).
struct LdsRd {
  const uint32_t* w;
  uint32_t head;
  __device__ __forceinline__ uint32_t u8(uint32_t o) const {
    const uint32_t i = head + o;
    return (w[i >> 2] >> (8 * (i & 3))) & 255u;
  }
  __device__ __forceinline__ uint32_t u32(uint32_t o) const {
    const uint32_t i = head + o, s = 8 * (i & 3), k = i >> 2;
    return (uint32_t)((((uint64_t)w[k + 1] << 32) | w[k]) >> s);
  }
  __device__ __forceinline__ uint64_t u64(uint32_t o) const {
    const uint32_t i = head + o, s = 8 * (i & 3), k = i >> 2;
    const uint32_t w0 = w[k], w1 = w[k + 1], w2 = w[k + 2];
    const uint32_t lo = (uint32_t)((((uint64_t)w1 << 32) | w0) >> s);
    const uint32_t hi = (uint32_t)((((uint64_t)w2 << 32) | w1) >> s);
    return ((uint64_t)hi << 32) | lo;
  }
};
struct GblRd {
  const uint8_t* p;
  __device__ __forceinline__ uint32_t u8(uint32_t o) const { return blk_u8(p + o); }
  __device__ __forceinline__ uint32_t u32(uint32_t o) const { return blk_u32(p + o); }
  __device__ __forceinline__ uint64_t u64(uint32_t o) const {
    return *reinterpret_cast<gbl_u64u_t*>(reinterpret_cast<uint64_t>(p + o));
  }
  // 16 bytes at any alignment in one load instruction (a per-lane walk's
  // loads each touch up to 64 lines: fewer, wider instructions)
  __device__ __forceinline__ void u64x2(uint32_t o, uint64_t& lo, uint64_t& hi) const {
    const span_u32x4 v = *reinterpret_cast<__attribute__((address_space(1))) const span_u32x4*>(
        reinterpret_cast<uint64_t>(p + o));
    lo = (uint64_t)v.y << 32 | v.x;
    hi = (uint64_t)v.w << 32 | v.z;
  }
};

template <class R>
__device__ __forceinline__ uint64_t rd_varint(const R& r, uint32_t& p, uint32_t lim, int max_shift, bool& ok) {
  uint64_t x = 0;
  for (int shift = 0; shift <= max_shift; shift += 7) {
    if (p >= lim) break;
    const uint64_t b = r.u8(p++);
    x |= (b & 127) << shift;
    if (!(b & 128)) return x;
  }
  ok = false;
  return 0;
}

// One entry at offset p (offsets relative to the block): DecodeEntry
// (:37-64) / CheckAndDecodeEntry (:68-97) with the bounds CheckAndDecodeEntry
// checks; index blocks with delta-encoded values: DecodeEntryV4 (:110-139) and
// the value's encoded length from IndexValue::DecodeFrom (table/format.cc
// :137-162: delta size when shared != 0, else a BlockHandle; then the
// length-prefixed first key).  Returns false for "bad entry in block";
// q = key delta, v = value.
template <int KIND, class R>
__device__ __forceinline__ bool rd_entry(const R& r, uint32_t p, uint32_t lim, uint32_t* sh, uint32_t* ns,
                                         uint32_t* q, uint32_t* v, uint32_t* vl) {
  if (p > lim || lim - p < 3) return false;
  bool ok = true;
  const uint64_t s = rd_varint(r, p, lim, 28, ok);
  const uint64_t k = ok ? rd_varint(r, p, lim, 28, ok) : 0;
  if (!ok) return false;
  if (KIND == kBlkIndexDelta || KIND == kBlkIndexDeltaFk) {
    if ((uint64_t)(lim - p) < k) return false;
    const uint32_t v0 = p + (uint32_t)k;
    uint32_t c = v0;
    (void)rd_varint(r, c, lim, 63, ok);             // delta size, or the handle's offset
    if (ok && s == 0) (void)rd_varint(r, c, lim, 63, ok);  // the handle's size
    if (KIND == kBlkIndexDeltaFk && ok) {
      const uint64_t fk = rd_varint(r, c, lim, 28, ok);
      ok = ok && (uint64_t)(lim - c) >= fk;
      c += ok ? (uint32_t)fk : 0u;
    }
    if (!ok) return false;
    *v = v0;
    *vl = c - v0;
  } else {
    const uint64_t x = rd_varint(r, p, lim, 28, ok);
    if (!ok || (uint64_t)(lim - p) < k + x) return false;
    *v = p + (uint32_t)k;
    *vl = (uint32_t)x;
  }
  *sh = (uint32_t)s;
  *ns = (uint32_t)k;
  *q = p;
  return true;
}

// DecodeEntry's fast path (block.cc:45-50): shared, non_shared and
// value_length each one byte (< 128) -- one dword read instead of three
// varint walks; anything else goes through rd_entry.  The dword may reach
// one byte past the entry area: the restart array follows it.
template <int KIND, class R>
__device__ __forceinline__ bool rd_entry_fast(const R& r, uint32_t p, uint32_t lim, uint32_t* sh, uint32_t* ns,
                                              uint32_t* q, uint32_t* v, uint32_t* vl) {
  if (p > lim || lim - p < 3) return false;
  const uint32_t u = r.u32(p);
  if (KIND != kBlkIndexDelta && KIND != kBlkIndexDeltaFk && (u & 0x808080u) == 0) {
    const uint32_t k = (u >> 8) & 255u, x = (u >> 16) & 255u;
    if (lim - (p + 3) < k + x) return false;
    *sh = u & 255u;
    *ns = k;
    *q = p + 3;
    *v = p + 3 + k;
    *vl = x;
    return true;
  }
  return rd_entry<KIND>(r, p, lim, sh, ns, q, v, vl);
}

// rd_entry_fast with the entry's first dword already loaded (prefetched by
// the caller right after the previous entry was decoded).
template <int KIND, class R>
__device__ __forceinline__ bool rd_entry_pre(const R& r, uint32_t p, uint32_t lim, uint32_t u, uint32_t* sh,
                                             uint32_t* ns, uint32_t* q, uint32_t* v, uint32_t* vl) {
  if (p > lim || lim - p < 3) return false;
  if (KIND != kBlkIndexDelta && KIND != kBlkIndexDeltaFk && (u & 0x808080u) == 0) {
    const uint32_t k = (u >> 8) & 255u, x = (u >> 16) & 255u;
    if (lim - (p + 3) < k + x) return false;
    *sh = u & 255u;
    *ns = k;
    *q = p + 3;
    *v = p + 3 + k;
    *vl = x;
    return true;
  }
  return rd_entry<KIND>(r, p, lim, sh, ns, q, v, vl);
}

// inclusive scan across the wave
__device__ __forceinline__ uint64_t wave_incl_scan_u64(uint64_t v, uint32_t lane) {
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t u = __shfl_up(v, o, 64);
    if (lane >= (uint32_t)o) v += u;
  }
  return v;
}

// the wave's LDS writes visible to its other lanes
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// A wave's LDS slot for a staged span (k_dbg_xp: the wave-cooperative long
// loop over an LDS copy).
constexpr uint32_t kBlkSlot = 6144;                           // bytes staged
constexpr uint32_t kBlkSlotWords = (kBlkSlot + 16 + 16 + 16) / 4;  // + head, tail chunk, pad

// Copy the block into the wave's slot; returns the LdsRd over it.
__device__ __forceinline__ LdsRd blk_stage(const uint8_t* g, uint32_t n, uint32_t* slot, uint32_t lane) {
  const uint64_t a = reinterpret_cast<uint64_t>(g);
  const uint32_t head = (uint32_t)(a & 15), nch = (head + n + 15) >> 4;
  const uint64_t g0 = a - head;
  for (uint32_t i = lane; i < nch; i += 64) {
    const uint4 v = span_load16<false>(g0 + 16ull * i);
    slot[4 * i] = v.x;
    slot[4 * i + 1] = v.y;
    slot[4 * i + 2] = v.z;
    slot[4 * i + 3] = v.w;
  }
  wave_lds_sync();
  return LdsRd{slot, head};
}

// block.cc:994-1083 NumRestarts / IndexType / the Block constructor;
// data_block_hash_index.cc:76-84 (NUM_BUCK u16 before the footer)
template <class R>
__device__ __forceinline__ BlkHdr rd_header(const R& r, uint64_t n64) {
  BlkHdr h{0, 0, false};
  if (n64 < 4 || n64 > 0xFFFFFFFFull) return h;
  const uint32_t size = (uint32_t)n64;
  const uint32_t footer = r.u32(size - 4);
  bool hash = false;
  uint32_t nr = footer;
  if (size <= (1u << 16)) {
    hash = footer >> 31;
    nr = footer & 0x7FFFFFFFu;
  }
  h.nr = nr;
  if (!hash) {
    const uint32_t ro = size - (1 + nr) * 4u;
    if (ro > size - 4u) return h;
    h.ro = ro;
  } else {
    if (size < 6) return h;
    const uint16_t sz16 = (uint16_t)(size - 4);
    const uint16_t nb = (uint16_t)(r.u8(sz16 - 2) | (r.u8(sz16 - 1) << 8));
    const uint16_t map_offset = (uint16_t)(sz16 - 2 - nb);
    const uint32_t ro = (uint32_t)map_offset - nr * 4u;
    if (ro > map_offset) return h;
    h.ro = ro;
  }
  h.ok = nr == 0 || size >= 8;
  return h;
}

// ---- XXPH3 over a reader (util/xxph3.h; see xxph3_short / xxph3_long_lane) --
template <class R>
__device__ __forceinline__ uint64_t xp_mix16(const R& r, uint32_t o, int s, uint64_t seed) {
  return mul128_fold64(r.u64(o) ^ (sec64(s) + seed), r.u64(o + 8) ^ (sec64(s + 8) - seed));
}
template <class R>
__device__ __forceinline__ uint64_t xp_short(const R& r, uint32_t o, uint32_t len, uint64_t seed) {
  if (len <= 16) {
    if (len > 8) {
      const uint64_t lo = r.u64(o) ^ (sec64(0) + seed), hi = r.u64(o + len - 8) ^ (sec64(8) - seed);
      return xxph3_avalanche(len + (lo + hi) + mul128_fold64(lo, hi));
    }
    if (len >= 4) return xxph3_4to8(r.u32(o), r.u32(o + len - 4), len, seed);
    if (len) return xxph3_1to3(r.u8(o), r.u8(o + (len >> 1)), r.u8(o + len - 1), len, seed);
    return mul128_fold64(seed + sec64(0), P64_2);
  }
  uint64_t acc = (uint64_t)len * P64_1;
  if (len <= 128) {
    if (len > 32) {
      if (len > 64) {
        if (len > 96) {
          acc += xp_mix16(r, o + 48, 96, seed);
          acc += xp_mix16(r, o + len - 64, 112, seed);
        }
        acc += xp_mix16(r, o + 32, 64, seed);
        acc += xp_mix16(r, o + len - 48, 80, seed);
      }
      acc += xp_mix16(r, o + 16, 32, seed);
      acc += xp_mix16(r, o + len - 32, 48, seed);
    }
    acc += xp_mix16(r, o, 0, seed);
    acc += xp_mix16(r, o + len - 16, 16, seed);
    return xxph3_avalanche(acc);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) acc += xp_mix16(r, o + 16 * i, 16 * i, seed);
  acc = xxph3_avalanche(acc);
  const int rounds = (int)len / 16;
#pragma unroll
  for (int i = 8; i < 15; i++)
    if (i < rounds) acc += xp_mix16(r, o + 16 * i, 16 * (i - 8) + 3, seed);
  acc += xp_mix16(r, o + len - 16, 136 - 17, seed);
  return xxph3_avalanche(acc);
}
// xp_short for 17..128 bytes with the loads batched: xp_mid_load issues
// all eight 16-byte pieces at once (xp_short's nested length tests each wait
// for their own loads: up to four memory round trips per value on a
// scattered per-lane walk), xp_mid_fold hashes them.  Piece t is pair t >> 1:
// the front piece at 16 i (t even) or the back one at len - 16 (i + 1) (t
// odd), secret offset 16 t either way; offsets are clamped into the span
// (pieces a length does not use are loaded and dropped).  129..240 bytes
// stay on xp_short: a second batch for the part after the first 128 bytes
// measured slower (200-byte values 6.09 vs 5.90 ms per step).
template <class R>
__device__ __forceinline__ void xp_mid_load(const R& r, uint32_t o, uint32_t len, uint64_t (&d)[16]) {
  const int last = (int)len - 16;
#pragma unroll
  for (int t = 0; t < 8; t++) {
    int off = (t & 1) ? last - 16 * (t >> 1) : 16 * (t >> 1);
    off = off < 0 ? 0 : off > last ? last : off;
    r.u64x2(o + (uint32_t)off, d[2 * t], d[2 * t + 1]);
  }
}
__device__ __forceinline__ uint64_t xp_mid_fold(const uint64_t (&d)[16], uint32_t len, uint64_t seed) {
  uint64_t acc = (uint64_t)len * P64_1;
  const uint32_t pairs = (len + 31) / 32;
#pragma unroll
  for (int t = 0; t < 8; t++) {
    const uint64_t m = mul128_fold64(d[2 * t] ^ (sec64(16 * t) + seed), d[2 * t + 1] ^ (sec64(16 * t + 8) - seed));
    acc += (uint32_t)(t >> 1) < pairs ? m : 0ull;
  }
  return xxph3_avalanche(acc);
}

// 17..128-byte values of a wave's lanes hashed by lane octets (all 64 lanes
// call it; `mine`: this lane has such a value, at global address va).  In
// step j octet g hashes the value of lane 8 g + j, its lane 8 g + t loading
// piece t (xp_mid_load's order and clamping): each load instruction reads
// eight contiguous <= 128-byte windows, where a per-lane hash's reads 64
// scattered pieces -- the per-lane walk is bound by the texture addresser
// (TA busy ~95 % of the protect kernel, ~64 lanes' worth of cycles per
// divergent load).  The octet sums its terms with DPP (reduce-scatter: lane
// 8 g + j ends with the sum for its own value).  klo / khi: sec64(16 t) + seed, sec64(16 t + 8) - seed.
__device__ __forceinline__ uint64_t xp_mid_octets(uint64_t va, uint32_t vl, bool mine, uint64_t klo, uint64_t khi,
                                                  uint32_t lane) {
  const uint32_t t = lane & 7, gb = lane & ~7u;
  const uint64_t zp = reinterpret_cast<uint64_t>(&g_zero16[0]);
  const uint32_t lm_own = mine ? vl : 0u;
  span_u32x4 d[8];
  uint32_t lens[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int src = (int)gb + j;
    const uint64_t a = __shfl(va, src, 64);
    const uint32_t lm = (uint32_t)__shfl((int)lm_own, src, 64);  // 0: no value there
    const int last = (int)lm - 16;
    int off = (t & 1) ? last - 16 * (int)(t >> 1) : 16 * (int)(t >> 1);
    off = off < 0 ? 0 : off > last ? last : off;
    const uint64_t addr = lm ? a + (uint32_t)off : zp;
    d[j] = *reinterpret_cast<__attribute__((address_space(1))) const span_u32x4*>(addr);
    lens[j] = lm;
  }
  uint64_t m[8];  // this lane's term for value j (piece t of it)
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const uint64_t lo = (uint64_t)d[j].y << 32 | d[j].x, hi = (uint64_t)d[j].w << 32 | d[j].z;
    const uint64_t mm = mul128_fold64(lo ^ klo, hi ^ khi);
    const uint32_t pairs = (lens[j] + 31) / 32;
    m[j] = (t >> 1) < pairs ? mm : 0ull;
  }
  // Reduce-scatter over the octet: lane t ends with the sum over the octet
  // of value t's terms (its own value), in three exchange steps -- bit 2 of
  // the value index with the half-row mirror partner (7 - t), then bit 1
  // (lane ^ 2) and bit 0 (lane ^ 1) -- 7 exchanged values instead of eight
  // 3-step octet sums, and one avalanche per lane instead of eight.
  uint64_t r1[4], r2[2];
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const uint64_t keep = (t & 4) ? m[4 + q] : m[q], send = (t & 4) ? m[q] : m[4 + q];
    r1[q] = keep + dpp64<0x141>(send);  // row_half_mirror
  }
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const uint64_t keep = (t & 2) ? r1[2 + q] : r1[q], send = (t & 2) ? r1[q] : r1[2 + q];
    r2[q] = keep + dpp64<0x4E>(send);  // quad_perm [2,3,0,1]: lane ^ 2
  }
  const uint64_t keep = (t & 1) ? r2[1] : r2[0], send = (t & 1) ? r2[0] : r2[1];
  const uint64_t sum = keep + dpp64<0xB1>(send);  // quad_perm [1,0,3,2]: lane ^ 1
  return xxph3_avalanche((uint64_t)lm_own * P64_1 + sum);
}

// one lane, any length (keys)
template <class R>
__device__ __noinline__ uint64_t xp_lane(const R& r, uint32_t o, uint32_t len, uint64_t seed) {
  if (len <= 240) return xp_short(r, o, len, seed);
  uint64_t acc[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
  const uint32_t nb = len / 1024;
  auto stripe = [&](uint32_t p, int soff) {
    for (int l = 0; l < 8; l++) {
      const uint64_t d = r.u64(p + 8 * l), k = d ^ csec64(soff + 8 * l, seed);
      acc[l] += d + mul32to64(k);
    }
  };
  for (uint32_t b = 0; b < nb; b++) {
    for (int s2 = 0; s2 < 16; s2++) stripe(o + 1024 * b + 64 * s2, 8 * s2);
    for (int l = 0; l < 8; l++) {
      uint64_t a = acc[l];
      a ^= a >> 47;
      a ^= csec64(128 + 8 * l, seed);
      acc[l] = a * P32_1;
    }
  }
  const int nst = (int)((len - 1024 * nb) / 64);
  for (int s2 = 0; s2 < nst; s2++) stripe(o + 1024 * nb + 64 * s2, 8 * s2);
  if (len & 63) stripe(o + len - 64, 121);
  uint64_t res = (uint64_t)len * P64_1;
  for (int l = 0; l < 4; l++)
    res += mul128_fold64(acc[2 * l] ^ csec64(11 + 16 * l, seed), acc[2 * l + 1] ^ csec64(19 + 16 * l, seed));
  return xxph3_avalanche(res);
}

// Per-lane secret words of the wave-cooperative long loop (seed fixed):
// lane = 8 g + l (accumulator l, stripe group g = stripes g and g + 8).
struct XpWaveSec {
  uint64_t s0, s1, scr, last, m;
};
__device__ __forceinline__ XpWaveSec xp_wave_sec(uint32_t lane, uint64_t seed) {
  const int l = lane & 7, g = lane >> 3;
  XpWaveSec k;
  k.s0 = csec64(8 * g + 8 * l, seed);
  k.s1 = csec64(8 * (g + 8) + 8 * l, seed);
  k.scr = csec64(128 + 8 * l, seed);
  k.last = csec64(121 + 8 * l, seed);
  k.m = csec64((l & 1) ? 19 + 16 * (l >> 1) : 11 + 16 * (l >> 1), seed);
  return k;
}
// sum over the 8 lanes with the same (lane & 7)
__device__ __forceinline__ uint64_t xp_sum_groups(uint64_t v) {
  v += __shfl_xor(v, 8, 64);
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}
// XXPH3 long loop (len > 240) of ONE span by the whole wave: within a 1 KiB
// segment the 128 (stripe, accumulator) terms are independent sums, so lane
// (g, l) folds stripes g and g + 8 for accumulator l and the 8 groups are
// summed before the (sequential) scramble.  Result valid on every lane.
template <class R>
__device__ __forceinline__ uint64_t xp_wave_long(const R& r, uint32_t o, uint32_t len, const XpWaveSec& k,
                                                 uint32_t lane) {
  const uint32_t l = lane & 7, g = lane >> 3;
  uint64_t acc = l < 4 ? (l < 2 ? (l ? P64_1 : (uint64_t)P32_3) : (l == 2 ? P64_2 : P64_3))
                      : (l < 6 ? (l == 4 ? P64_4 : (uint64_t)P32_2) : (l == 6 ? P64_5 : (uint64_t)P32_1));
  const uint32_t nb = len / 1024;
  for (uint32_t b = 0; b < nb; b++) {
    const uint32_t p = o + 1024 * b + 64 * g + 8 * l;
    const uint64_t d0 = r.u64(p), d1 = r.u64(p + 512);
    acc += xp_sum_groups(d0 + mul32to64(d0 ^ k.s0) + d1 + mul32to64(d1 ^ k.s1));
    acc ^= acc >> 47;
    acc ^= k.scr;
    acc *= P32_1;
  }
  const uint32_t nst = (len - 1024 * nb) / 64;
  uint64_t part = 0;
  const uint32_t p = o + 1024 * nb + 64 * g + 8 * l;
  if (g < nst) {
    const uint64_t d = r.u64(p);
    part += d + mul32to64(d ^ k.s0);
  }
  if (g + 8 < nst) {
    const uint64_t d = r.u64(p + 512);
    part += d + mul32to64(d ^ k.s1);
  }
  acc += xp_sum_groups(part);
  if (len & 63) {
    const uint64_t d = r.u64(o + len - 64 + 8 * l);
    acc += d + mul32to64(d ^ k.last);
  }
  // merge: lanes l = 2j, 2j + 1 pair up
  // (shuffles outside the ?: -- clang lowers a ?: with call operands to a
  // branch, and a shuffle there reads masked lanes: found by the
  // mck_internal_xp_wave test)
  const uint64_t other = __shfl_xor(acc, 1, 64), mo = __shfl_xor(k.m, 1, 64);
  const uint64_t f = mul128_fold64(acc ^ k.m, other ^ mo);
  uint64_t t = (l & 1) ? 0 : f;
  t += __shfl_xor(t, 2, 64);
  t += __shfl_xor(t, 4, 64);
  return xxph3_avalanche((uint64_t)len * P64_1 + readlane_u64(t, 0));
}

// XXPH3 long loop (len > 240) of FOUR spans at once, one per 16-lane row:
// lane = 16 row + 8 g + l folds accumulator l over the stripes s = g, g + 2,
// ..., g + 14 of each 1 KiB segment (8 loads per segment, all issued
// together), the two stripe groups are summed with one DPP-free shuffle and
// the scramble / last stripe / merge follow the wave version.  `sec` is the
// seeded secret in LDS as 24 u64 words (word w = bytes 8w of
// XXPH3_initCustomSecret); klast / km: this lane's last-stripe and merge
// secret words.  Result valid on every lane of the row.
template <class R>
__device__ __forceinline__ uint64_t xp_row_long(const R& r, uint32_t o, uint32_t len, const uint64_t* sec,
                                                uint64_t klast, uint64_t km, uint32_t lane) {
  const uint32_t l = lane & 7, g = (lane >> 3) & 1;
  uint64_t acc = l < 4 ? (l < 2 ? (l ? P64_1 : (uint64_t)P32_3) : (l == 2 ? P64_2 : P64_3))
                       : (l < 6 ? (l == 4 ? P64_4 : (uint64_t)P32_2) : (l == 6 ? P64_5 : (uint64_t)P32_1));
  const uint32_t nb = len / 1024, nst = (len - 1024 * nb) / 64;
  for (uint32_t b = 0; b <= nb; b++) {
    const uint32_t base = o + 1024 * b + 64 * g + 8 * l;
    uint64_t part = 0;
#pragma unroll
    for (uint32_t m = 0; m < 8; m++) {
      const uint32_t st = g + 2 * m;
      if (b < nb || st < nst) {
        const uint64_t d = r.u64(base + 128 * m);
        part += d + mul32to64(d ^ sec[st + l]);
      }
    }
    const uint64_t other = __shfl_xor(part, 8, 64);
    acc += part + other;
    if (b < nb) {
      acc ^= acc >> 47;
      acc ^= sec[16 + l];
      acc *= P32_1;
    }
  }
  if (len & 63) {
    const uint64_t d = r.u64(o + len - 64 + 8 * l);
    acc += d + mul32to64(d ^ klast);
  }
  const uint64_t other = __shfl_xor(acc, 1, 64), mo = __shfl_xor(km, 1, 64);
  const uint64_t f = mul128_fold64(acc ^ km, other ^ mo);
  uint64_t t = (l & 1) ? 0 : f;
  t += __shfl_xor(t, 2, 64);
  t += __shfl_xor(t, 4, 64);
  const uint64_t t0 = __shfl(t, (int)(lane & ~15u), 64);
  return xxph3_avalanche((uint64_t)len * P64_1 + t0);
}

// ---- one THREAD per block ----------------------------------------------------
// Each lane owns a whole
// block and walks it in order, exactly as the reference's SeekToFirst/Next
// loop does; 64 blocks per wave keep every lane busy and the
// dependent header reads of thousands of blocks in flight hide the memory
// latency.  (Round 2 measured one wave per block, one lane per restart
// interval: ~1000 (layout) / ~3500 (kv) VALU instructions per block issued
// for a few lanes -- removed.)

// Sequential walk of one block (block.cc:1091-1132 with the restart checks
// of the layout pass); on_entry(idx, key_len, shared, delta_off, value_off,
// value_len) per entry.  Returns the status; *nk, *kb, *ri.
template <int KIND, class R, class F>
__device__ __forceinline__ int blk_seq_walk(const R& rd, uint64_t n, uint32_t* nk, uint64_t* kb, uint32_t* ri_out,
                                            F&& on_entry) {
  *nk = 0;
  *kb = 0;
  *ri_out = 0;
  const BlkHdr h = rd_header(rd, n);
  if (!h.ok) return kBlkBadContents;
  if (h.nr == 0) return kBlkOk;
  for (uint32_t r = 0; r < h.nr; r++) {
    const uint32_t x = rd.u32(h.ro + 4 * r);
    if (r == 0 ? (h.ro != 0 && x != 0) : (x <= rd.u32(h.ro + 4 * (r - 1)) || x >= h.ro)) return kBlkBadRestarts;
  }
  if (h.ro == 0) return h.nr == 1 ? kBlkOk : kBlkBadRestarts;
  uint32_t idx = 0, interval = 0, in_cur = 0, r = 0, kl = 0;
  uint32_t next = rd.u32(h.ro);  // restart point r
  uint64_t kbytes = 0;
  uint32_t p = 0;
  while (p < h.ro) {
    if (r < h.nr && p > next) return kBlkBadRestarts;  // a restart point inside an entry
    const bool at_restart = r < h.nr && p == next;
    if (at_restart) {
      if (r == 1)
        interval = in_cur;
      else if (r > 1 && in_cur != interval)
        return kBlkBadRestarts;
      in_cur = 0;
      r++;
      next = r < h.nr ? rd.u32(h.ro + 4 * r) : 0xFFFFFFFFu;
    }
    uint32_t sh, ns, q, v, vl;
    if (!rd_entry_fast<KIND>(rd, p, h.ro, &sh, &ns, &q, &v, &vl)) return kBlkBadEntry;
    if (at_restart && sh != 0) return r == 1 ? kBlkBadEntry : kBlkBadRestarts;
    if (kl < sh) return kBlkBadEntry;
    on_entry(idx, sh + ns, sh, q, v, vl);
    kl = sh + ns;
    kbytes += kl;
    idx++;
    in_cur++;
    p = v + vl;
  }
  if (r != h.nr) return kBlkBadRestarts;
  *nk = idx;
  *kb = kbytes;
  *ri_out = h.nr > 1 ? interval : 0;
  return kBlkOk;
}

template <int KIND>
__global__ __launch_bounds__(256) void k_block_layout_t(SpanSrc blocks, uint32_t count, uint64_t* key_cnt,
                                                        uint64_t* key_bytes, uint32_t* interval_out,
                                                        int32_t* status) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= count) return;
  uint32_t nk, ri;
  uint64_t kb;
  const int st = blk_seq_walk<KIND>(GblRd{blocks.ptr(b)}, blocks.len(b), &nk, &kb, &ri,
                                    [](uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t) {});
  key_cnt[b] = st == kBlkOk ? nk : 0;
  key_bytes[b] = st == kBlkOk ? kb : 0;
  interval_out[b] = st == kBlkOk ? ri : 0;
  status[b] = st;
}

// Pass 2, one thread per block.  The current key lives in a per-thread LDS
// buffer and is updated in place as IterKey::TrimAppend does
// (block.cc:641-651): entry e only writes its non_shared bytes at [shared,
// shared + non_shared) -- the prefix is already there -- and is hashed from
// the buffer; the value is hashed in place.  A key longer than the buffer
// moves the thread to its block's arena share (global, same in-place rule).
constexpr uint32_t kBlkKeyBuf = 128;  // bytes of LDS key buffer per thread
// Values of more than 240 bytes (XXPH3's long loop) are not hashed by the
// walk (round 3): a lane's long value would be read with 8-byte loads from
// 64 different blocks per instruction, or, four at a time by 16-lane rows
// (round 2), serialise the bandwidth-bound hashing behind the latency-bound
// walk in one wave.  (Round 3 swept the list with a wave per 64 keys and 8-byte
// loads per lane, k_block_long: 1000-B values 0.335 of peak; the row loop
// below, 0.362.)  The walk writes the entry's hash WITHOUT the value's
// (ProtectKV XORs the per-field hashes, and the Encode truncation commutes
// with XOR) and records the value in a LONG-VALUE LIST indexed by the key
// index k -- so the list is in memory order (keys follow blocks, entries
// follow each other) and needs no scan: long_len[k] = value length (0: no
// long value; the host zeroes the array), long_off[k] = value address,
// and, to verify, long_part[k] = the partial hash.  k_block_long_rows then
// sweeps the key range front to back with the XXPH3 row driver (one value
// per 16-lane row, 16-byte loads), XORs the value hash into enc[k] (protect)
// or compares partial ^ value hash with the stored bytes (verify).
constexpr uint32_t kBlkLong = 241;
// Encode(n) bytes of key k in a kv_checksum array: one load of n bytes when
// the array is aligned to n, byte loads otherwise.
__device__ __forceinline__ uint64_t blk_load_prot(const uint8_t* a, uint64_t k, uint32_t n) {
  const uint64_t at = reinterpret_cast<uint64_t>(a) + k * n;
  if ((at & (n - 1)) == 0) {  // n = 1, 2, 4, 8
    if (n == 8) return *reinterpret_cast<gbl_u64u_t*>(at);
    if (n == 4) return *reinterpret_cast<gbl_u32u_t*>(at);
    if (n == 2) return *reinterpret_cast<__attribute__((address_space(1))) const uint16_t*>(at);
    return *reinterpret_cast<gbl_u8_t*>(at);
  }
  uint64_t s = 0;
  for (uint32_t c = 0; c < n; c++) s |= (uint64_t)*reinterpret_cast<gbl_u8_t*>(at + c) << (8 * c);
  return s;
}
// 17..128-byte values are hashed by lane octets (xp_mid_octets)
template <int KIND, bool VERIFY>
__global__ __launch_bounds__(256) void k_block_kv_t(SpanSrc blocks, uint32_t count, const uint64_t* key_base,
                                                    const uint64_t* arena_base, uint8_t* arena, uint64_t* long_off,
                                                    uint32_t* long_len, uint64_t K_total, uint64_t* long_part,
                                                    uint32_t prot_bytes,
                                                    uint8_t* enc, const uint8_t* stored, uint8_t* mismatch,
                                                    uint32_t* mismatch_count) {
  // + 20 B: dword reads and the 16-byte delta write past the key end; an odd
  // stride in dwords keeps the 64 lanes' buffers on distinct banks
  __shared__ uint32_t s_key[256][kBlkKeyBuf / 4 + 5];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t k0 = 0, cnt = 0, aslice = 0;
  bool active = false;
  if (b < count) {
    k0 = ldg_u64(key_base, b);
    cnt = ldg_u64(key_base, b + 1) - k0;
    active = cnt != 0 && k0 <= K_total && cnt <= K_total - k0;  // no keys (or a bad block): idle
  }
  uint8_t* const lkey = reinterpret_cast<uint8_t*>(s_key[threadIdx.x]);
  uint8_t* const gkey = active ? arena + ldg_u64(arena_base, b) : arena;
  if (active) aslice = ldg_u64(arena_base, b + 1) - ldg_u64(arena_base, b);
  bool global_key = false;
  const GblRd rd{active ? blocks.ptr(b) : nullptr};
  const uint64_t n64 = active ? blocks.len(b) : 0;
  const uint32_t n = (uint32_t)n64;
  // Protect: the layout pass validated the block.  Verify: the block may
  // have changed since it was protected, so the walk trusts nothing -- a bad
  // header or entry, more or fewer entries than key_base gives the block, a
  // shared prefix longer than the previous key or a key longer than the
  // block's arena slice makes the block BAD: every one of its protect-time
  // keys is flagged and nothing outside [k0, k0 + cnt) is touched (the
  // iterator's CorruptionError, block.h:559-565).
  bool bad = false;
  uint32_t nbad = 0, kprev = 0;
  uint32_t ro = 0;
  if (active) {
    const BlkHdr h = rd_header(rd, n64);
    ro = h.ro;
    if constexpr (VERIFY) {
      if (!h.ok || h.ro == 0) {
        bad = true;
        active = false;
      }
    }
  }
  const uint64_t oklo = sec64(16 * (int)(lane & 7)) + kSeedV, okhi = sec64(16 * (int)(lane & 7) + 8) - kSeedV;
  // 8-byte protection into an aligned array: entries are stored in pairs
  const bool p8 = !VERIFY && prot_bytes == 8 && (reinterpret_cast<uint64_t>(enc) & 7) == 0;
  uint64_t pend = 0;  // p8: the lane's even entry, stored with the odd one after it
  uint32_t p = 0, idx = 0;
  // The next entry's first 16 bytes, one entry ahead: its header and, on
  // DecodeEntry's fast path, its key delta's first 13 bytes -- ONE divergent
  // load per entry where the header dword and two key-delta loads were three
  // (a load whose 64 lanes read 64 blocks is what bounds this kernel: the
  // texture addresser).  uok = false: the 16 bytes would
  // leave the block, the entry is read field by field.
  uint4 U = make_uint4(0, 0, 0, 0);
  bool uok = false;
  bool any_long = false;  // this lane recorded a long value
  if (active) {
    uok = n >= 16;
    if (uok) U = vload16_any(reinterpret_cast<uint64_t>(rd.p));
  }
  while (__any(active)) {
    uint32_t sh = 0, ns = 0, q = 0, v = 0, vl = 0;
    uint64_t hv = 0;
    uint32_t kw[4];
    bool vmid = false;
    if (active) {
      const uint4 Uc = U;
      bool fast = false;
      if (KIND != kBlkIndexDelta && KIND != kBlkIndexDeltaFk && uok && (Uc.x & 0x808080u) == 0) {
        // block.cc:45-50: shared, non_shared, value length one byte each
        const uint32_t kk = (Uc.x >> 8) & 255u, xx = (Uc.x >> 16) & 255u;
        if (p <= ro && ro - p >= 3 && ro - (p + 3) >= kk + xx) {
          sh = Uc.x & 255u;
          ns = kk;
          q = p + 3;
          v = q + kk;
          vl = xx;
          fast = true;
        }
      }
      const bool dec = fast || rd_entry<KIND>(rd, p, ro, &sh, &ns, &q, &v, &vl);
      if constexpr (VERIFY) {
        if (!dec || idx >= cnt || sh > kprev ||
            (sh + ns > kBlkKeyBuf && (uint64_t)sh + ns > aslice)) {
          bad = true;
          active = false;
          sh = ns = q = v = vl = 0;
        }
      }
      const uint32_t pn = v + vl;
      if (active && pn < ro) {
        uok = pn + 16 <= n;
        if (uok) U = vload16_any(reinterpret_cast<uint64_t>(rd.p + pn));
      }
      // the key delta's first 16 bytes: bytes 3..18 of the entry on the fast
      // path (the dword at p + 16 only when non_shared > 13: then it lies
      // before the value); otherwise two 8-byte loads at q (8 bytes at q are
      // always inside the block: the restart array + footer follow)
      if (fast) {
        const uint32_t e = ns > 13 ? rd.u32(p + 16) : 0u;
        kw[0] = __builtin_amdgcn_alignbyte(Uc.y, Uc.x, 3);
        kw[1] = __builtin_amdgcn_alignbyte(Uc.z, Uc.y, 3);
        kw[2] = __builtin_amdgcn_alignbyte(Uc.w, Uc.z, 3);
        kw[3] = __builtin_amdgcn_alignbyte(e, Uc.w, 3);
      } else {
        const uint64_t k01 = rd.u64(q), k23 = rd.u64(ns > 8 ? q + 8 : q);
        kw[0] = (uint32_t)k01;
        kw[1] = (uint32_t)(k01 >> 32);
        kw[2] = (uint32_t)k23;
        kw[3] = (uint32_t)(k23 >> 32);
      }
      vmid = vl > 16 && vl <= 128;
    }
    {
      const uint64_t hm = xp_mid_octets(reinterpret_cast<uint64_t>(rd.p) + v, vl, vmid, oklo, okhi, lane);
      hv = vmid ? hm : 0ull;
    }
    const bool lng = active && vl >= kBlkLong;
    if (active) {
      const uint32_t kl = sh + ns;
      if (!global_key && kl > kBlkKeyBuf) {  // rare: move the prefix to the arena
        for (uint32_t i = 0; i < sh; i++) gkey[i] = lkey[i];
        global_key = true;
      }
      // IterKey::TrimAppend: only the non-shared bytes change
      if (!global_key) {
        // the delta's first 16 bytes from kw (written whole: bytes past the
        // key are never read as key) as five aligned dwords, the first merged
        // with the shared prefix bytes below sh (16 byte stores were 16 LDS
        // instructions per entry); the rest (rare) in dword loads
        {
          uint32_t* kd = s_key[threadIdx.x] + (sh >> 2);
          const uint32_t s4 = sh & 3u, sb = 4u - s4;  // alignbyte uses sb & 3: s4 = 0 is the plain copy
          const uint32_t prev = s4 ? kd[0] << (8 * sb) : 0u;  // the prefix bytes, at the top
          kd[0] = s4 ? __builtin_amdgcn_alignbyte(kw[0], prev, sb) : kw[0];
          kd[1] = s4 ? __builtin_amdgcn_alignbyte(kw[1], kw[0], sb) : kw[1];
          kd[2] = s4 ? __builtin_amdgcn_alignbyte(kw[2], kw[1], sb) : kw[2];
          kd[3] = s4 ? __builtin_amdgcn_alignbyte(kw[3], kw[2], sb) : kw[3];
          kd[4] = __builtin_amdgcn_alignbyte(0u, kw[3], sb);  // (s4 = 0: past the 16 bytes, never read)
        }
        for (uint32_t i = sh + 16; i < kl; i += 4) {
          const uint32_t w = rd.u32(q + i - sh);
          for (uint32_t c = 0; c < 4 && i + c < kl; c++) lkey[i + c] = (uint8_t)(w >> (8 * c));
        }
        const LdsRd kr{s_key[threadIdx.x], 0};
        hv ^= xp_short(kr, 0, kl, kSeedK);
      } else {
        for (uint32_t i = sh; i < kl; i++) gkey[i] = (uint8_t)rd.u8(q + i - sh);
        __threadfence_block();
        hv ^= xp_lane(GblRd{gkey}, 0, kl, kSeedK);
      }
      if (!vmid && !lng) hv ^= xp_short(rd, v, vl, kSeedV);  // <= 16 or 129..240 bytes
    }
    any_long |= lng;
    if (active) {
      const uint64_t k = k0 + idx;
      if (lng) {  // to the long-value list; k_block_long_rows completes the entry
        long_off[k] = reinterpret_cast<uint64_t>(rd.p) + v;
        long_len[k] = vl;
        if constexpr (VERIFY) long_part[k] = hv;
      }
      if constexpr (!VERIFY) {
        if (p8) {
          // entries idx - 1, idx as one 16-byte store when idx is odd (half
          // the divergent stores); a block's last even entry alone
          if (idx & 1) {
            *reinterpret_cast<__attribute__((address_space(1))) span_u32x4*>(
                reinterpret_cast<uint64_t>(enc) + 8 * (k - 1)) =
                span_u32x4{(uint32_t)pend, (uint32_t)(pend >> 32), (uint32_t)hv, (uint32_t)(hv >> 32)};
          } else if (v + vl >= ro) {
            reinterpret_cast<uint64_t*>(enc)[k] = hv;
          }
          pend = hv;
        } else {
          for (uint32_t c = 0; c < prot_bytes; c++) enc[k * prot_bytes + c] = (uint8_t)(hv >> (8 * c));
        }
      } else if (!lng) {
        const uint64_t sv = blk_load_prot(stored, k, prot_bytes);
        const uint64_t keep = prot_bytes >= 8 ? ~0ull : ((1ull << (8 * prot_bytes)) - 1);
        const bool miss = sv != (hv & keep);
        mismatch[k] = miss;
        nbad += miss;
        if (miss && mismatch_count) atomicAdd(mismatch_count, 1u);
      }
      idx++;
      kprev = sh + ns;
      p = v + vl;
      active = p < ro;
    }
  }
  if constexpr (VERIFY) {
    if (b < count && cnt != 0 && !bad && idx != cnt && k0 <= K_total && cnt <= K_total - k0) bad = true;
    if (bad) {  // rare: flag the whole block, drop its long values from the sweep
      for (uint64_t k = k0; k < k0 + cnt; k++) {
        mismatch[k] = 1;
        long_len[k] = 0;
      }
      if (mismatch_count && cnt > nbad) atomicAdd(mismatch_count, (uint32_t)(cnt - nbad));
    }
  }
  // one flag store per wave (every writer stores 1; an atomic per step on
  // one address serialised the walk: 1000-B values 0.363 -> 0.274): the
  // long-value sweep exits at once when no value was recorded
  if (__ballot(any_long) && lane == 0) long_len[K_total] = 1u;
}

// ---- one pass (round 4): layout and protection in the same walk ------------
// The two-pass pair above reads every block twice: k_block_layout_t's walk
// touches every 128-byte line (one entry header per ~line at 100-byte
// values) only to count entries for the key index, then k_block_kv_t walks
// again -- 100-B values: 4.2 + 8.3 GB of HBM reads for a 4.3 GB image, the
// layout pass a third of the step.  k_block_kv_walk does the layout checks
// and the hashing in ONE walk and parks every entry's hash (without a long
// value's) in a per-block SLOT (slot_cap entries per block, rounded up to
// even: 8 bytes each, stored in 16-byte pairs as k_block_kv_t's output) and
// a long value's offset/length beside it; the scan of the counts gives the
// key index, and k_block_kv_flush moves the slots to the kv_checksum array
// (coalesced: a thread per slot pair).  A block with more than slot_cap
// entries, or a key longer than the LDS buffer and arena_cap, gets
// MCK_BLOCK_SLOT_OVERFLOW and no keys; the caller protects it with the
// two-pass pair.
constexpr int kBlkSlotOverflow = 4;

// Entry e of block b: slot_h[b * stride + e] = the hash without the long
// value's; slot_m[...] = (value offset in block << 32 | length), written for
// long values only; bit e of the block's long mask (blk_long, stride / 32
// words per block, rounded up) marks them.
__host__ __device__ __forceinline__ uint32_t blk_slot_stride(uint32_t slot_cap) { return (slot_cap + 1) & ~1u; }
__host__ __device__ __forceinline__ uint32_t blk_long_words(uint32_t slot_cap) {
  return (blk_slot_stride(slot_cap) + 31) / 32;
}
// Where entry e of block b's slot lives.  MCK_BLK_SLOT_T (round 6): the 64
// blocks of a wave (b >> 6; the walk's lane is b & 63) keep entry e side by
// side, so the walk's per-entry store -- every active lane is at the same
// entry index -- is one coalesced 512-byte row per wave; block-major slots
// (b * stride + e) were 16-byte pair stores, 64 lines per instruction, each
// line completed over ~16 entries: 0.62 GB written for 0.28 GB of slots at
// 100-B values and a partly written line per lane in L2 beside the window
// lines the walk re-reads.  The slot area holds count rounded up to 64.
#ifndef MCK_BLK_SLOT_T
#define MCK_BLK_SLOT_T 1
#endif
__host__ __device__ __forceinline__ uint64_t blk_slot_at(uint32_t b, uint32_t e, uint32_t stride) {
  if (MCK_BLK_SLOT_T) return ((uint64_t)(b >> 6) * stride + e) * 64 + (b & 63);
  return (uint64_t)b * stride + e;
}
__host__ __device__ __forceinline__ uint64_t blk_slot_count(uint32_t count) {
  return MCK_BLK_SLOT_T ? ((uint64_t)count + 63) & ~63ull : count;
}

// ---- entry windows (round 5) ----------------------------------------------
// The walk's divergent loads -- each entry's 16-byte head (U), its key's
// fifth dword and eight octet value loads per 64 entries -- are what bound it
// (the texture addresser, TA_BUSY 91 %).  Since an entry's
// start p is known one entry ahead, the octet loads fetch the whole ENTRY
// window [p, p + 128) instead: in step j lane 8 g + t loads bytes [16 t,
// 16 t + 16) of lane 8 g + j's window (one load instruction: eight
// contiguous 128-byte windows), the pieces are parked in the lanes' LDS rows
// at the next iteration's start, and each lane then reads its head, key and
// (17..128-byte) value pieces from its own row -- no per-lane global load
// for an entry that fits the window and the block.  Rows are 36 dwords
// (144 B: 16-byte aligned, conflict-free b128 stores; 16 B of pad for the
// unaligned reads at the row end).
constexpr uint32_t kBlkWin = 128, kBlkWinRow = 36;
// MCK_BLK_SLOT_NT: the walk's slot stores non-temporal (A/B knob: a lane's
// partly written slot line otherwise sits in L2 for ~16 entries beside the
// window lines the next entry re-reads)
#ifndef MCK_BLK_SLOT_NT
#define MCK_BLK_SLOT_NT 0
#endif
#ifndef MCK_BLK_RS_CACHE
#define MCK_BLK_RS_CACHE 1
#endif
__device__ __forceinline__ uint4 lds_row_u4(const uint32_t* w, uint32_t o) {  // 16 bytes at byte o
  const uint32_t i = o >> 2, sb = o & 3u;
  const uint32_t d0 = w[i], d1 = w[i + 1], d2 = w[i + 2], d3 = w[i + 3], d4 = w[i + 4];
  return make_uint4(__builtin_amdgcn_alignbyte(d1, d0, sb), __builtin_amdgcn_alignbyte(d2, d1, sb),
                    __builtin_amdgcn_alignbyte(d3, d2, sb), __builtin_amdgcn_alignbyte(d4, d3, sb));
}
// Octet step loads: W[j] = piece (lane & 7) of the window at address a of
// lane (lane & ~7) + j, or the zero page where that lane has none.
__device__ __forceinline__ void blk_win_load(uint4 (&W)[8], uint64_t a, bool have, uint32_t lane, uint64_t zp) {
  const uint32_t t = lane & 7, gb = lane & ~7u;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const uint64_t aj = __shfl(a, (int)gb + j, 64);
    const bool hj = __shfl((int)have, (int)gb + j, 64) != 0;
    W[j] = span_load16<false>(hj ? aj + 16u * t : zp);
  }
}
// ... parked in the rows: piece t of lane (gb + j)'s window -> row gb + j.
__device__ __forceinline__ void blk_win_store(uint32_t (*rows)[kBlkWinRow], const uint4 (&W)[8], uint32_t tid) {
  const uint32_t t = tid & 7, g0 = tid & ~7u;
#pragma unroll
  for (int j = 0; j < 8; j++)
    *reinterpret_cast<uint4*>(&rows[g0 + j][4 * t]) = W[j];
}
// xp_mid_octets over the lanes' windows: value j = bytes [vo, vo + vl) of
// lane (gb + j)'s row (17 <= vl <= 128, vo + vl <= 128).
__device__ __forceinline__ uint64_t xp_mid_octets_win(const uint32_t (*rows)[kBlkWinRow], uint32_t vo, uint32_t vl,
                                                      bool mine, uint64_t klo, uint64_t khi, uint32_t tid) {
  const uint32_t lane = tid & 63, t = lane & 7, g0 = tid & ~7u, gb = lane & ~7u;
  const uint32_t lm_own = mine ? vl : 0u;
  uint64_t m[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int src = (int)gb + j;
    const uint32_t o = (uint32_t)__shfl((int)vo, src, 64);
    const uint32_t lm = (uint32_t)__shfl((int)lm_own, src, 64);
    const int last = (int)lm - 16;
    int off = (t & 1) ? last - 16 * (int)(t >> 1) : 16 * (int)(t >> 1);
    off = off < 0 ? 0 : off > last ? last : off;
    const uint4 d = lds_row_u4(rows[g0 + j], lm ? o + (uint32_t)off : 0u);
    const uint64_t lo = (uint64_t)d.y << 32 | d.x, hi = (uint64_t)d.w << 32 | d.z;
    const uint64_t mm = mul128_fold64(lo ^ klo, hi ^ khi);
    m[j] = (t >> 1) < (lm + 31) / 32 ? mm : 0ull;
  }
  uint64_t r1[4], r2[2];
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const uint64_t keep = (t & 4) ? m[4 + q] : m[q], send = (t & 4) ? m[q] : m[4 + q];
    r1[q] = keep + dpp64<0x141>(send);
  }
#pragma unroll
  for (int q = 0; q < 2; q++) {
    const uint64_t keep = (t & 2) ? r1[2 + q] : r1[q], send = (t & 2) ? r1[q] : r1[2 + q];
    r2[q] = keep + dpp64<0x4E>(send);
  }
  const uint64_t keep = (t & 1) ? r2[1] : r2[0], send = (t & 1) ? r2[0] : r2[1];
  const uint64_t sum = keep + dpp64<0xB1>(send);
  return xxph3_avalanche((uint64_t)lm_own * P64_1 + sum);
}

template <int KIND>
__global__ __launch_bounds__(256) void k_block_kv_walk(SpanSrc blocks, uint32_t count, uint32_t slot_cap,
                                                       uint8_t* arena, uint32_t arena_cap, uint64_t* slot_h,
                                                       uint64_t* slot_m, uint32_t* blk_long, uint64_t* key_cnt,
                                                       uint64_t* key_bytes, uint32_t* interval_out,
                                                       int32_t* status, uint32_t* long_flag) {
  __shared__ uint32_t s_key[256][kBlkKeyBuf / 4 + 5];  // as k_block_kv_t
  __shared__ __attribute__((aligned(16))) uint32_t s_win[256][kBlkWinRow];  // the entry windows
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  uint8_t* const lkey = reinterpret_cast<uint8_t*>(s_key[threadIdx.x]);
  const bool in = b < count;
  const GblRd rd{in ? blocks.ptr(b) : nullptr};
  const LdsRd wr{s_win[threadIdx.x], 0};  // this lane's window (entry-relative offsets)
  const uint64_t zp = reinterpret_cast<uint64_t>(&g_zero16[0]);
  const uint64_t n64 = in ? blocks.len(b) : 0;
  // ---- the block's header and restart array: blk_seq_walk's checks
  int st = kBlkOk;
  BlkHdr h{0, 0, false};
  bool active = false;
  uint32_t rs1 = 0, rs2 = 0, rs3 = 0;  // restart points 1..3 (MCK_BLK_RS_CACHE)
  if (in) {
    h = rd_header(rd, n64);
    if (!h.ok) {
      st = kBlkBadContents;
    } else if (h.nr != 0) {
      // four restart words per round trip (a loop of dependent-exit loads
      // was one round trip per restart point)
      uint32_t prev = 0;
      for (uint32_t r0 = 0; r0 < h.nr && st == kBlkOk; r0 += 4) {
        uint32_t x[4];
#pragma unroll
        for (int j = 0; j < 4; j++) x[j] = r0 + j < h.nr ? rd.u32(h.ro + 4 * (r0 + j)) : 0u;
        if (MCK_BLK_RS_CACHE && r0 == 0) {
          rs1 = x[1];
          rs2 = x[2];
          rs3 = x[3];
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const uint32_t r = r0 + j;
          if (r < h.nr && st == kBlkOk && (r == 0 ? (h.ro != 0 && x[j] != 0) : (x[j] <= prev || x[j] >= h.ro)))
            st = kBlkBadRestarts;
          prev = x[j];
        }
      }
      if (st == kBlkOk && h.ro == 0 && h.nr != 1) st = kBlkBadRestarts;
      active = st == kBlkOk && h.ro != 0;
    }
  }
  const uint32_t n = (uint32_t)n64, ro = h.ro, nr = h.nr;
  uint8_t* const gkey = arena + (uint64_t)(in ? b : 0) * arena_cap;
  bool global_key = false;
  const uint64_t oklo = sec64(16 * (int)(lane & 7)) + kSeedV, okhi = sec64(16 * (int)(lane & 7) + 8) - kSeedV;
  const uint32_t sstride = blk_slot_stride(slot_cap);
  const uint64_t sbase = (uint64_t)(in ? b : 0) * sstride;
  uint64_t pend = 0;  // the lane's even entry, stored with the odd one after it
  uint32_t lmask = 0;  // long entries of the current 32
  uint32_t* const lwords = blk_long + (uint64_t)(in ? b : 0) * blk_long_words(slot_cap);
  uint32_t p = 0, idx = 0, interval = 0, in_cur = 0, r = 0, kl = 0;
  // restart point r and, loaded one restart ahead, r + 1
  uint32_t next = active ? rd.u32(ro) : 0u;
  uint32_t nextn = active && nr > 1 ? (MCK_BLK_RS_CACHE ? rs1 : rd.u32(ro + 4)) : 0xFFFFFFFFu;
  uint64_t kbytes = 0;
  // the next entry, one entry ahead: its window (octet loads, wnx) when
  // [p, p + 128) lies in the block, else its first 16 bytes (U, uok)
  uint4 U = make_uint4(0, 0, 0, 0);
  uint4 Wn[8];
  bool uok = false, wnx = false;
  bool any_long = false;
  if (active) {
    wnx = n >= kBlkWin;
    uok = !wnx && n >= 16;
    if (uok) U = vload16_any(reinterpret_cast<uint64_t>(rd.p));
  }
  blk_win_load(Wn, reinterpret_cast<uint64_t>(rd.p), wnx, lane, zp);
  while (__any(active)) {
    uint32_t sh = 0, ns = 0, q = 0, v = 0, vl = 0;
    uint32_t kw[4] = {0, 0, 0, 0};
    bool vmid = false;
    // this iteration's windows into the rows (their loads were issued one
    // entry ago)
    const bool wok = wnx;
    if (__any(wok)) {
      blk_win_store(s_win, Wn, threadIdx.x);
      wave_lds_sync();
    }
    wnx = false;
    uint32_t pn = 0;  // the next entry (wnx)
    if (active) {
      // block.cc:1091-1132 with the restart checks of blk_seq_walk
      int err = kBlkOk;
      if (r < nr && p > next) err = kBlkBadRestarts;  // a restart point inside an entry
      const bool at_restart = r < nr && p == next;
      if (err == kBlkOk && at_restart) {
        if (r == 1)
          interval = in_cur;
        else if (r > 1 && in_cur != interval)
          err = kBlkBadRestarts;
        in_cur = 0;
        r++;
        next = nextn;
        // (the restart array's line is long gone from L2 by now: points 1..3
        // come from the header pass's registers)
        nextn = r + 1 < nr ? (MCK_BLK_RS_CACHE && r + 1 <= 3 ? (r == 1 ? rs2 : rs3) : rd.u32(ro + 4 * (r + 1)))
                           : 0xFFFFFFFFu;
      }
      const uint4 Uc = wok ? lds_row_u4(s_win[threadIdx.x], 0) : U;
      bool fast = false;
      if (err == kBlkOk) {
        if (KIND != kBlkIndexDelta && KIND != kBlkIndexDeltaFk && (uok || wok) && (Uc.x & 0x808080u) == 0) {
          const uint32_t kk = (Uc.x >> 8) & 255u, xx = (Uc.x >> 16) & 255u;
          if (p <= ro && ro - p >= 3 && ro - (p + 3) >= kk + xx) {
            sh = Uc.x & 255u;
            ns = kk;
            q = p + 3;
            v = q + kk;
            vl = xx;
            fast = true;
          }
        }
        if (!fast && !rd_entry<KIND>(rd, p, ro, &sh, &ns, &q, &v, &vl)) err = kBlkBadEntry;
      }
      if (err == kBlkOk && at_restart && sh != 0) err = r == 1 ? kBlkBadEntry : kBlkBadRestarts;
      if (err == kBlkOk && kl < sh) err = kBlkBadEntry;
      if (err == kBlkOk && idx >= slot_cap) err = kBlkSlotOverflow;
      if (err == kBlkOk && !global_key && sh + ns > kBlkKeyBuf && sh + ns > arena_cap) err = kBlkSlotOverflow;
      if (err == kBlkOk && global_key && sh + ns > arena_cap) err = kBlkSlotOverflow;
      if (err != kBlkOk) {
        st = err;
        active = false;
      } else {
        pn = v + vl;
        uok = false;
        if (pn < ro) {
          // a window only while entries fit one (the next is likely the
          // size of this one): a 1000-byte value's entry would fetch 112
          // bytes it never uses, where its 16-byte head is all the walk needs
          wnx = pn + kBlkWin <= n && pn - p <= kBlkWin;
          uok = !wnx && pn + 16 <= n;
          if (uok) U = vload16_any(reinterpret_cast<uint64_t>(rd.p + pn));
        }
        if (fast) {
          const uint32_t e = ns > 13 ? (wok ? s_win[threadIdx.x][4] : rd.u32(p + 16)) : 0u;
          kw[0] = __builtin_amdgcn_alignbyte(Uc.y, Uc.x, 3);
          kw[1] = __builtin_amdgcn_alignbyte(Uc.z, Uc.y, 3);
          kw[2] = __builtin_amdgcn_alignbyte(Uc.w, Uc.z, 3);
          kw[3] = __builtin_amdgcn_alignbyte(e, Uc.w, 3);
        } else {
          const uint64_t k01 = rd.u64(q), k23 = rd.u64(ns > 8 ? q + 8 : q);
          kw[0] = (uint32_t)k01;
          kw[1] = (uint32_t)(k01 >> 32);
          kw[2] = (uint32_t)k23;
          kw[3] = (uint32_t)(k23 >> 32);
        }
        vmid = vl > 16 && vl <= 128;
      }
    }
    // the next entries' windows: in flight while this entry is hashed
    if (__any(wnx)) blk_win_load(Wn, reinterpret_cast<uint64_t>(rd.p) + pn, wnx, lane, zp);
    // the entry lies in its window: key and value bytes from the row
    const bool inwin = active && wok && v + vl <= p + kBlkWin;
    uint64_t hv = 0;
    if (__any(vmid && inwin)) {
      const uint64_t hm = xp_mid_octets_win(s_win, v - p, vl, vmid && inwin, oklo, okhi, threadIdx.x);
      hv = vmid && inwin ? hm : hv;
    }
    if (__any(vmid && !inwin)) {
      const uint64_t hm = xp_mid_octets(reinterpret_cast<uint64_t>(rd.p) + v, vl, vmid && !inwin, oklo, okhi, lane);
      hv = vmid && !inwin ? hm : hv;
    }
    const bool lng = active && vl >= kBlkLong;
    if (active) {
      const uint32_t kn = sh + ns;
      if (!global_key && kn > kBlkKeyBuf) {  // rare: move the prefix to the block's arena slot
        for (uint32_t i = 0; i < sh; i++) gkey[i] = lkey[i];
        global_key = true;
      }
      if (!global_key) {  // IterKey::TrimAppend in the LDS buffer (k_block_kv_t)
        {
          uint32_t* kd = s_key[threadIdx.x] + (sh >> 2);
          const uint32_t s4 = sh & 3u, sb = 4u - s4;
          const uint32_t prev = s4 ? kd[0] << (8 * sb) : 0u;
          kd[0] = s4 ? __builtin_amdgcn_alignbyte(kw[0], prev, sb) : kw[0];
          kd[1] = s4 ? __builtin_amdgcn_alignbyte(kw[1], kw[0], sb) : kw[1];
          kd[2] = s4 ? __builtin_amdgcn_alignbyte(kw[2], kw[1], sb) : kw[2];
          kd[3] = s4 ? __builtin_amdgcn_alignbyte(kw[3], kw[2], sb) : kw[3];
          kd[4] = __builtin_amdgcn_alignbyte(0u, kw[3], sb);
        }
        for (uint32_t i = sh + 16; i < kn; i += 4) {
          const uint32_t w = inwin ? wr.u32(q - p + i - sh) : rd.u32(q + i - sh);
          for (uint32_t c = 0; c < 4 && i + c < kn; c++) lkey[i + c] = (uint8_t)(w >> (8 * c));
        }
        const LdsRd kr{s_key[threadIdx.x], 0};
        hv ^= xp_short(kr, 0, kn, kSeedK);
      } else {
        for (uint32_t i = sh; i < kn; i++) gkey[i] = (uint8_t)rd.u8(q + i - sh);
        __threadfence_block();
        hv ^= xp_lane(GblRd{gkey}, 0, kn, kSeedK);
      }
      if (!vmid && !lng) {  // <= 16 or 129..240 bytes
        if (inwin)
          hv ^= xp_short(wr, v - p, vl, kSeedV);
        else
          hv ^= xp_short(rd, v, vl, kSeedV);
      }
      if (MCK_BLK_SLOT_T) {
        if constexpr (MCK_BLK_SLOT_NT)  // (whole rows: streamed out, not parked in L2)
          __builtin_nontemporal_store(hv, &slot_h[blk_slot_at(b, idx, sstride)]);
        else
          slot_h[blk_slot_at(b, idx, sstride)] = hv;
      } else if (idx & 1) {  // entries idx - 1, idx as one 16-byte store (half the divergent stores)
        const span_u32x4 pr{(uint32_t)pend, (uint32_t)(pend >> 32), (uint32_t)hv, (uint32_t)(hv >> 32)};
        auto* dst = reinterpret_cast<__attribute__((address_space(1))) span_u32x4*>(
            reinterpret_cast<uint64_t>(slot_h + sbase + idx - 1));
        if constexpr (MCK_BLK_SLOT_NT)
          __builtin_nontemporal_store(pr, dst);
        else
          *dst = pr;
      } else if (v + vl >= ro) {  // the block's last entry, even
        slot_h[sbase + idx] = hv;
      }
      pend = hv;
      if (lng) {
        slot_m[MCK_BLK_SLOT_T ? blk_slot_at(b, idx, sstride) : sbase + idx] = (uint64_t)v << 32 | vl;
        lmask |= 1u << (idx & 31);
      }
      if ((idx & 31) == 31 || v + vl >= ro) {
        lwords[idx >> 5] = lmask;
        lmask = 0;
      }
      kl = kn;
      kbytes += kn;
      idx++;
      in_cur++;
      p = v + vl;
      active = p < ro;
    }
    any_long |= lng;
  }
  if (in) {
    if (st == kBlkOk && nr != 0 && ro != 0 && r != nr) st = kBlkBadRestarts;
    const bool ok = st == kBlkOk;
    key_cnt[b] = ok ? idx : 0;
    key_bytes[b] = ok ? kbytes : 0;
    interval_out[b] = ok && nr > 1 ? interval : 0;
    status[b] = st;
  }
  if (__ballot(any_long) && lane == 0) *long_flag = 1u;
}

// Slots -> the kv_checksum array (protect) or the mismatch flags (verify),
// and the long-value list k_block_long_rows sweeps (long_len[k] for every
// key): thread t moves slot pair t of the flattened slot array, 4 pairs per
// thread (a wave per block ran into the dispatcher: 0.27 ms at 1M blocks).
template <bool VERIFY>
__device__ __forceinline__ void blk_flush_one(SpanSrc blocks, uint32_t stride, uint32_t b, uint32_t i,
                                              const uint64_t* slot_h,
                                              const uint64_t* slot_m, const uint32_t* blk_long,
                                              const uint64_t* key_base, const uint64_t* prot_base, uint64_t kcap,
                                              uint32_t prot_bytes, bool p8, uint8_t* enc,
                                              const uint8_t* stored, uint8_t* mismatch, uint32_t* mismatch_count,
                                              uint64_t* long_off, uint32_t* long_len, uint64_t* long_part,
                                              bool batch_long) {
  uint64_t k0 = ldg_u64(key_base, b);
  const uint64_t cnt = ldg_u64(key_base, b + 1) - k0;
  if (i >= cnt) return;
  if constexpr (VERIFY) {
    // keys are the PROTECT-time ones (block.h:623: kv_checksum_ + n *
    // cur_entry_idx_ within the block's own array); a block whose entry
    // count changed is k_block_kv_verify_bad's
    k0 = ldg_u64(prot_base, b);
    if (ldg_u64(prot_base, b + 1) - k0 != cnt || k0 > kcap || cnt > kcap - k0) return;
  }
  const uint64_t s0 = blk_slot_at(b, i, stride);
  const uint64_t s1 = blk_slot_at(b, i + 1, stride);
  const bool two = i + 1 < cnt;
  uint64_t h[2];
  if (MCK_BLK_SLOT_T) {
    h[0] = slot_h[s0];
    h[1] = two ? slot_h[s1] : 0;
  } else if (two) {
    const span_u32x4 v = *reinterpret_cast<__attribute__((address_space(1))) const span_u32x4*>(
        reinterpret_cast<uint64_t>(slot_h + s0));
    h[0] = (uint64_t)v.y << 32 | v.x;
    h[1] = (uint64_t)v.w << 32 | v.z;
  } else {
    h[0] = slot_h[s0];
    h[1] = 0;
  }
  // i is even: entries i, i + 1 share a mask word
  const uint32_t lm = (ldg_u32(blk_long, b * blk_long_words(stride) + (i >> 5)) >> (i & 31)) & 3u;
  const uint64_t base = lm ? reinterpret_cast<uint64_t>(blocks.ptr(b)) : 0;
#pragma unroll
  for (int e = 0; e < 2; e++) {
    if (e == 1 && !two) break;
    const uint64_t k = k0 + i + e;
    const uint64_t m = (lm >> e) & 1u ? slot_m[e ? s1 : s0] : 0ull;  // (unwritten for short values)
    const uint32_t vl = (uint32_t)m;
    if (batch_long) long_len[k] = vl;  // (no long value in the batch: the sweep exits on the flag)
    if (vl) {
      long_off[k] = base + (m >> 32);
      if constexpr (VERIFY) long_part[k] = h[e];
    }
    if constexpr (!VERIFY) {
      if (p8)
        reinterpret_cast<uint64_t*>(enc)[k] = h[e];
      else
        for (uint32_t c = 0; c < prot_bytes; c++) enc[k * prot_bytes + c] = (uint8_t)(h[e] >> (8 * c));
    } else if (!vl) {
      const uint64_t sv = blk_load_prot(stored, k, prot_bytes);
      const uint64_t keep = prot_bytes >= 8 ? ~0ull : ((1ull << (8 * prot_bytes)) - 1);
      const bool bad = sv != (h[e] & keep);
      mismatch[k] = bad;
      if (bad && mismatch_count) atomicAdd(mismatch_count, 1u);
    }
  }
}
template <bool VERIFY>
__global__ __launch_bounds__(256) void k_block_kv_flush(SpanSrc blocks, uint32_t npairs, uint32_t stride,
                                                        const uint64_t* slot_h, const uint64_t* slot_m,
                                                        const uint32_t* blk_long, const uint64_t* key_base,
                                                        const uint64_t* prot_base, uint64_t kcap,
                                                        uint32_t prot_bytes, uint8_t* enc, const uint8_t* stored,
                                                        uint8_t* mismatch, uint32_t* mismatch_count,
                                                        uint64_t* long_off, uint32_t* long_len,
                                                        uint64_t* long_part, const uint32_t* long_flag) {
  const bool p8 = prot_bytes == 8 && (reinterpret_cast<uint64_t>(enc) & 7) == 0;
  const bool batch_long = *long_flag != 0;
  const uint32_t hs = stride >> 1;
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (MCK_BLK_SLOT_T) {
    // wave-interleaved slots: workgroup c flushes the 64-block chunk c, its
    // threads striding over the chunk's pairs block-major (consecutive
    // threads, consecutive pairs of one block: coalesced output writes);
    // every slot line (16 blocks' entry e) is read by this workgroup alone,
    // so once from HBM (a pair per thread across workgroups split the lines
    // over XCDs: 0.59 GB fetched for 0.28; lane-per-block writes scattered
    // 16-byte pieces: 1.43 GB written for 0.28)
    const uint32_t nb = npairs / hs, per = 64 * hs;
    for (uint32_t c = blockIdx.x; (uint64_t)c * 64 < nb; c += gridDim.x)
      for (uint32_t jl = threadIdx.x; jl < per; jl += blockDim.x) {
        const uint32_t b = c * 64 + jl / hs;
        if (b >= nb) break;
        blk_flush_one<VERIFY>(blocks, stride, b, 2 * (jl % hs), slot_h, slot_m, blk_long, key_base, prot_base, kcap,
                              prot_bytes, p8, enc, stored, mismatch, mismatch_count, long_off, long_len, long_part,
                              batch_long);
      }
    return;
  }
  const uint32_t g = gridDim.x * blockDim.x;
#pragma unroll
  for (uint32_t u = 0; u < 4; u++) {
    const uint64_t j = t + (uint64_t)u * g;
    if (j < npairs) {
      const uint32_t b = (uint32_t)(j / hs), i = 2 * (uint32_t)(j - (uint64_t)b * hs);
      blk_flush_one<VERIFY>(blocks, stride, b, i, slot_h, slot_m, blk_long, key_base, prot_base, kcap, prot_bytes,
                            p8, enc, stored, mismatch, mismatch_count, long_off, long_len, long_part, batch_long);
    }
  }
}

// One-pass verify, blocks whose walk now gives another entry count than
// protect did (a corrupt header, entry or restart array; walk failures count
// 0): every protect-time key of the block is flagged and leaves the long-value
// sweep, no other block's keys move.  A block the walk could not park
// (kBlkSlotOverflow) is not verified: its keys stay unflagged and the caller
// re-verifies the batch with the two-pass pair (status says which).
__global__ __launch_bounds__(256) void k_block_kv_verify_bad(uint32_t count, const uint64_t* walk_base,
                                                             const uint64_t* prot_base, const int32_t* status,
                                                             uint64_t kcap, uint8_t* mismatch,
                                                             uint32_t* mismatch_count, uint32_t* long_len,
                                                             const uint32_t* long_flag) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= count) return;
  const uint64_t k0 = ldg_u64(prot_base, b), cp = ldg_u64(prot_base, b + 1) - k0;
  const uint64_t cw = ldg_u64(walk_base, b + 1) - ldg_u64(walk_base, b);
  if (cp == cw || k0 >= kcap) return;
  const uint64_t k1 = cp > kcap - k0 ? kcap : k0 + cp;
  const bool flag = status[b] != kBlkSlotOverflow;
  const bool batch_long = *long_flag != 0;
  for (uint64_t k = k0; k < k1; k++) {
    mismatch[k] = flag;
    if (batch_long) long_len[k] = 0;
  }
  if (flag && mismatch_count) atomicAdd(mismatch_count, (uint32_t)(k1 - k0));
}

__global__ __launch_bounds__(64) void k_dbg_xp(const uint8_t* d, uint32_t len, uint64_t seed, uint64_t* out) {
  __shared__ uint32_t slot[kBlkSlotWords];
  const uint32_t lane = threadIdx.x & 63;
  const XpWaveSec ws = xp_wave_sec(lane, seed);
  const uint64_t a = xp_wave_long(GblRd{d}, 0, len, ws, lane);
  const uint64_t b = xp_lane(GblRd{d}, 0, len, seed);
  uint64_t c = 0;
  if (len <= kBlkSlot) c = xp_wave_long(blk_stage(d, len, slot, lane), 0, len, ws, lane);
  // row k of the wave hashes the span's first len - 61 k bytes
  __shared__ uint64_t sec[24];
  if (lane < 24) sec[lane] = csec64(8 * (int)lane, seed);
  __syncthreads();
  const uint32_t l8 = lane & 7;
  const uint64_t klast = csec64(121 + 8 * (int)l8, seed);
  const uint64_t km = csec64((l8 & 1) ? 19 + 16 * (int)(l8 >> 1) : 11 + 16 * (int)(l8 >> 1), seed);
  const uint64_t r = xp_row_long(GblRd{d}, 0, len - 61 * (lane >> 4), sec, klast, km, lane);
  if (lane == 0) {
    out[0] = a;
    out[1] = b;
    out[2] = c;
  }
  if ((lane & 15) == 0) out[3 + (lane >> 4)] = r;
}

// The long-value list on the XXH3 row driver (round 4): each 16-lane row
// walks key chunks [16 c, 16 c + 16), c = its row id, + rows in the grid,
// ... (one coalesced read of 16 lengths per row; a chunk without long
// values costs nothing more) and hashes the chunk's long values one after
// another with xxh3_rows_loop (XXPH3 preview rules, seed kSeedV): 16-byte
// dword-aligned loads, one KiB per row per iteration, one scramble per
// segment and row -- where k_block_long's wave-wide sweep read 8 bytes per
// lane per load.  op.finish XORs the value's hash into enc[k] (protect) or
// compares partial ^ hash with the stored bytes (verify).
template <bool VERIFY>
struct OpBlkLongRows {
  const uint64_t* long_off;
  const uint32_t* long_len;  // [K]
  const uint64_t* long_part;
  uint32_t prot_bytes;
  uint8_t* enc;
  const uint8_t* stored;
  uint8_t* mismatch;
  uint32_t* mismatch_count;
  const uint32_t* any_long;  // nonzero: the walk recorded a long value
  __device__ void finish(uint32_t k, uint64_t hv) const {
    if constexpr (!VERIFY) {  // enc[k] holds Encode(partial): XOR the value's hash in
      if (prot_bytes == 8 && ((reinterpret_cast<uint64_t>(enc) & 7) == 0)) {
        reinterpret_cast<uint64_t*>(enc)[k] ^= hv;
      } else {
        for (uint32_t b = 0; b < prot_bytes; b++) enc[(uint64_t)k * prot_bytes + b] ^= (uint8_t)(hv >> (8 * b));
      }
    } else {
      const uint64_t keep = prot_bytes >= 8 ? ~0ull : ((1ull << (8 * prot_bytes)) - 1);
      const uint64_t sv = blk_load_prot(stored, k, prot_bytes);
      const bool bad = sv != ((long_part[k] ^ hv) & keep);
      mismatch[k] = bad;
      if (bad && mismatch_count) atomicAdd(mismatch_count, 1u);
    }
  }
};
template <bool VERIFY>
__global__ __launch_bounds__(256) void k_block_long_rows(OpBlkLongRows<VERIFY> op, const uint64_t* key_base,
                                                         uint32_t nblocks, uint64_t kcap) {
  // keys of the batch (< 2^32: the host checks), never past the list's room
  const uint64_t K = min(ldg_u64(key_base, nblocks), kcap);
  if (*op.any_long == 0) return;  // no long value in the batch
  const X3Row X = x3_row(kSeedV);
  const uint32_t wpb = blockDim.x >> 6;
  const uint64_t rows = (uint64_t)gridDim.x * wpb * 4;
  uint64_t c = ((uint64_t)blockIdx.x * wpb + (threadIdx.x >> 6)) * 4 + X.row;  // the row's chunk
  uint32_t mask = 0, mylen = 0;  // the chunk's long values (row bits) / this lane's key's length
  uint64_t myoff = 0;
  bool have = false;
  // idle rows load from a valid address (the list itself)
  X3Span rs{reinterpret_cast<uint64_t>(op.long_off), 0, 0, 0, 0, 0, false};
  auto next = [&](X3Span& r) -> bool {
    for (;;) {
      if (mask) {  // row-uniform
        const uint32_t b = (uint32_t)__builtin_ctz(mask);
        mask &= mask - 1;
        const int src = (int)(((uint32_t)X.lane & ~15u) + b);
        r.ptr = (uint64_t)__shfl((long long)myoff, src, 64);
        r.len = (uint32_t)__shfl((int)mylen, src, 64);
        // XXPH3 util/xxph3.h:1516-1543 (len > 240)
        r.nb = (uint32_t)(r.len / 1024);
        r.nst = (uint32_t)((r.len - 1024ull * r.nb) / 64);
        r.tail = (r.len & 63) != 0;
        r.g = 0;
        r.i = (uint32_t)(16 * c + b);
        return true;
      }
      if (have) c += rows;
      have = true;
      if (16 * c >= K) return false;
      const uint64_t k = 16 * c + (uint32_t)X.j;
      mylen = k < K ? op.long_len[k] : 0u;
      myoff = mylen ? op.long_off[k] : 0ull;
      mask = (uint32_t)(__ballot(mylen != 0) >> (16 * X.row)) & 0xFFFFu;
    }
  };
  const bool act = next(rs);
  xxh3_rows_loop<OpBlkLongRows<VERIFY>, true>(op, X, rs, act, next);
}

// ---- exclusive scan of two u64 arrays (key counts, key bytes) --------------
constexpr uint32_t kBlkScanThreads = 256, kBlkScanPer = 8, kBlkScanTile = kBlkScanThreads * kBlkScanPer;

// workgroup-wide exclusive scan of one u64 per thread; returns the total
__device__ __forceinline__ uint64_t wg_excl_scan_u64(uint64_t v, uint64_t* lds, uint64_t* excl) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t incl = wave_incl_scan_u64(v, lane);
  if (lane == 63) lds[w] = incl;
  __syncthreads();
  uint64_t base = 0, tot = 0;
  for (uint32_t i = 0; i < kBlkScanThreads / 64; i++) {
    if (i < w) base += lds[i];
    tot += lds[i];
  }
  __syncthreads();
  *excl = base + incl - v;
  return tot;
}

__global__ __launch_bounds__(256) void k_blk_scan_tiles(const uint64_t* a, const uint64_t* b, uint32_t n,
                                                        uint64_t* tsum) {
  __shared__ uint64_t lds[2][4];
  const uint64_t t0 = (uint64_t)blockIdx.x * kBlkScanTile + threadIdx.x * kBlkScanPer;
  uint64_t sa = 0, sb = 0;
  for (uint32_t k = 0; k < kBlkScanPer; k++)
    if (t0 + k < n) {
      sa += a[t0 + k];
      sb += b[t0 + k];
    }
  uint64_t ea, eb;
  const uint64_t ta = wg_excl_scan_u64(sa, lds[0], &ea);
  const uint64_t tb = wg_excl_scan_u64(sb, lds[1], &eb);
  if (threadIdx.x == 0) {
    tsum[2 * blockIdx.x] = ta;
    tsum[2 * blockIdx.x + 1] = tb;
  }
}

// one workgroup: tile sums -> exclusive tile offsets; totals to a[n], b[n]
__global__ __launch_bounds__(256) void k_blk_scan_top(uint64_t* tsum, uint32_t ntiles, uint64_t* a, uint64_t* b,
                                                      uint32_t n) {
  __shared__ uint64_t lds[2][4];
  uint64_t ca = 0, cb = 0;
  for (uint32_t t0 = 0; t0 < ntiles; t0 += kBlkScanThreads) {
    const uint32_t t = t0 + threadIdx.x;
    const uint64_t va = t < ntiles ? tsum[2 * t] : 0, vb = t < ntiles ? tsum[2 * t + 1] : 0;
    uint64_t ea, eb;
    const uint64_t ta = wg_excl_scan_u64(va, lds[0], &ea);
    const uint64_t tb = wg_excl_scan_u64(vb, lds[1], &eb);
    if (t < ntiles) {
      tsum[2 * t] = ca + ea;
      tsum[2 * t + 1] = cb + eb;
    }
    ca += ta;
    cb += tb;
  }
  if (threadIdx.x == 0) {
    a[n] = ca;
    b[n] = cb;
  }
}

__global__ __launch_bounds__(256) void k_blk_scan_apply(uint64_t* a, uint64_t* b, uint32_t n, const uint64_t* tsum) {
  __shared__ uint64_t lds[2][4];
  const uint64_t t0 = (uint64_t)blockIdx.x * kBlkScanTile + threadIdx.x * kBlkScanPer;
  uint64_t va[kBlkScanPer], vb[kBlkScanPer], sa = 0, sb = 0;
  for (uint32_t k = 0; k < kBlkScanPer; k++) {
    va[k] = t0 + k < n ? a[t0 + k] : 0;
    vb[k] = t0 + k < n ? b[t0 + k] : 0;
    sa += va[k];
    sb += vb[k];
  }
  uint64_t ea, eb;
  (void)wg_excl_scan_u64(sa, lds[0], &ea);
  (void)wg_excl_scan_u64(sb, lds[1], &eb);
  ea += tsum[2 * blockIdx.x];
  eb += tsum[2 * blockIdx.x + 1];
  for (uint32_t k = 0; k < kBlkScanPer; k++)
    if (t0 + k < n) {
      a[t0 + k] = ea;
      b[t0 + k] = eb;
      ea += va[k];
      eb += vb[k];
    }
}

}  // namespace mck
