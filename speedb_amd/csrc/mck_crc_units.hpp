// mck_crc_units.hpp -- the unit-stream CRC32C driver for ragged batches of
// spans of a few KiB and more (SST data blocks of 4096 + 0..255 B + the type
// byte, 4/16/64 KiB compaction mixes, blob records).
//
// Why another driver.  The wave driver (mck_crc.hpp crc_drive) walks a span
// in 4 KiB rounds of 64-byte lane chunks anchored at the span's end; a 4300-B
// block is then one full round plus a head round holding 208 bytes, and the
// loop iteration of that head round keeps only 1 KiB in flight for the wave
// (4300-B blocks ran at 0.50-0.63 of the HBM roofline against 0.78 for
// aligned 4 KiB).  A long span is one wave's sequential rounds, so the last
// 64 KiB span of a launch leaves the rest of the GPU idle (~25 us per launch
// of the SST mix).
//
// Layout.  A span [ptr, ptr + n) is cut into 1 KiB UNITS anchored at its
// 16-aligned end a1: unit k covers [a1 - 1024 (k + 1), a1 - 1024 k).  In
// every unit lane l holds the 16-byte piece at 16 l, so ONE load instruction
// reads the unit's 1 KiB contiguous (non-temporal) and no transpose is
// needed.  A lane's pieces in consecutive units are 1008 bytes apart: after
// a piece the lane's state is "pending" (its last word xored, not yet
// stepped), and the next piece starts with zshift(., 4 + 1008) ^ w0 -- one
// 4-lookup byte-table step (gap1012) instead of the regular 4-byte step, so
// a unit costs every lane exactly four table steps.  At the end the lane's
// state is moved to the unit end by zshift(., 4 + 16 (63 - l)) (per-lane
// nibble tables, ulane_final) and XOR-reduced over the wave.  Head: the
// lanes whose piece lies wholly before the span load a zero piece; the piece
// holding ptr is masked below ptr and receives ~init un-shifted by those
// bytes.  Tail: the last piece is masked past the end and the result
// un-shifted by the < 16 bytes appended.  (The algebra of Crc32cCombine,
// util/crc32c.cc:1221-1266, as in mck_crc.hpp.)
//
// Streams.  A window of the workgroup's spans (up to kUDescCache) is laid
// out as one sequence of units -- spans in window order, each span's units
// in address order -- and cut into W equal STREAMS, one per wave: wave w
// folds units [T w / W, T (w + 1) / W), four per loop iteration (4 KiB in
// flight, the next iteration's loads issued before the current one is
// folded), across span boundaries: a 4300-B block is 5 units, and an
// iteration may hold the last unit of one block and the first three of the
// next.  The slots of an iteration are worked out lane-parallel from the
// units' prefix in LDS (unit_slots).  A span cut by a stream boundary (at
// most W - 1 per window, and every span longer than a stream) is shared:
// each stream's portion is reduced, moved to the span end by zshift(1024 m)
// (pow1k, m = units after the portion) and XORed into the span's LDS
// accumulator, and the stream that completes the last portion (an LDS
// counter) runs the epilogue.  No tickets, no per-span scheduling: every
// wave does the same number of units.
//
// LDS image (160 KiB, filled once per persistent workgroup):
//   [0, 64K)    gap1012 byte tables, 8 copies: entry (t, v, c) at
//               v << 8 | (t & 1) << 6 | (t >> 1) << 5 | c << 2 (bit 7 clear);
//               lane l of octet o reads copy l & 7 of table (k + o) & 3 in
//               lookup k, so the 32 lanes of an LDS group hit 32 banks;
//               in the bit-7 holes the per-lane final shift: entry
//               (n, nib, l) at n << 13 | nib << 9 | (l >> 5) << 8 | 128 |
//               (l & 31) << 2 (bank = l & 31: conflict-free)
//   [64K, 128K) the 4-byte step tables (kLdsStep layout, CrcLane)
//   [128K, ..)  un-shift by k < 16, byte masks, the staging scan's wave
//               sums, the window's descriptors, the shared spans'
//               accumulators and the units' prefix.
#pragma once
#include "mck_crc.hpp"

namespace mck {

constexpr uint32_t kUnitBytes = 1024;
constexpr uint32_t kULdsUnshift = 131072;                        // [16][8][16]
constexpr uint32_t kULdsMaskHead = kULdsUnshift + 16 * 512;      // [16] x 16 B: keep bytes >= h
constexpr uint32_t kULdsMaskTail = kULdsMaskHead + 256;          // [16] x 16 B: keep the first 16 - k
constexpr uint32_t kULdsWaveSum = kULdsMaskTail + 256;           // u32 per wave (staging scan)
constexpr uint32_t kUDescCache = 832;                            // descriptors per window
constexpr uint32_t kULdsDesc = kULdsWaveSum + 64;                // 16 B {off lo, off hi, len, inj}
constexpr uint32_t kULdsAcc = kULdsDesc + 16 * kUDescCache;      // {xor, count} per slot
constexpr uint32_t kULdsUpre = kULdsAcc + 8 * kUDescCache;       // u32 per slot + 65 (lookahead pad)
constexpr uint32_t kULdsEnd = kULdsUpre + 4 * (kUDescCache + 65);
static_assert(kULdsEnd <= kCrcLdsBytes, "unit driver LDS image must fit");

// ---- LDS fill -----------------------------------------------------------
__device__ __forceinline__ void crc_units_fill(const CrcTables* __restrict__ g) {
  const uint32_t t = threadIdx.x;  // kCrcBlock threads
  // [0, 64K): 16384 words, 16 per thread
  uint32_t lo[16];
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const uint32_t w = t + kCrcBlock * k;
    const uint32_t v = w >> 6, slot = w & 31;
    if (((w >> 5) & 1) == 0) {
      const uint32_t tt = ((slot >> 4) & 1) | (((slot >> 3) & 1) << 1);
      lo[k] = g->gap1012[tt][v];
    } else {
      lo[k] = g->ulane_final[v >> 5][(v >> 1) & 15][((v & 1) << 5) | slot];
    }
  }
  CrcFill f;
#pragma unroll
  for (int k = 0; k < 4096 / kCrcBlock; k++) {
    const int i = (int)t + kCrcBlock * k;
    f.step[k] = g->step[(i >> 2) & 3][i >> 4];
  }
  const uint4* us = reinterpret_cast<const uint4*>(&g->unshift[0][0][0]);
  const uint4 u = us[t < 512 ? t : 0];  // k < 16: 8 KiB
#pragma unroll
  for (int k = 0; k < 16; k++) *lds_p32(4 * (t + kCrcBlock * k)) = lo[k];
  uint4* l4 = reinterpret_cast<uint4*>(static_cast<size_t>(kLdsStep));
#pragma unroll
  for (int k = 0; k < 4096 / kCrcBlock; k++) {
    const uint32_t x = f.step[k];
    *reinterpret_cast<__attribute__((address_space(3))) span_u32x4*>(static_cast<size_t>(kLdsStep + 16 * (t + kCrcBlock * k))) =
        span_u32x4{x, x, x, x};
  }
  (void)l4;
  if (t < 512)
    *reinterpret_cast<__attribute__((address_space(3))) span_u32x4*>(static_cast<size_t>(kULdsUnshift + 16 * t)) =
        span_u32x4{u.x, u.y, u.z, u.w};
  if (t < 128) {
    const int h = (int)(t >> 2) & 15, k = (int)(t & 3);
    uint32_t m;
    if (t < 64) {  // keep bytes >= h of the piece
      const int d = h - 4 * k;
      m = d <= 0 ? 0xFFFFFFFFu : d >= 4 ? 0u : 0xFFFFFFFFu << (8 * d);
      *lds_p32(kULdsMaskHead + 4 * (t & 63)) = m;
    } else {  // keep the first 16 - h bytes
      const int keep = 16 - h - 4 * k;
      m = keep >= 4 ? 0xFFFFFFFFu : keep <= 0 ? 0u : 0xFFFFFFFFu >> (8 * (4 - keep));
      *lds_p32(kULdsMaskTail + 4 * (t & 63)) = m;
    }
  }
}

// ---- per-lane constants -----------------------------------------------------
struct UnitLane {
  CrcLane S;        // the 4-byte step (mck_crc.hpp)
  uint32_t gpc[4];  // gap step: byte 0 of entry (t, ., c) per lookup
  uint32_t gsel[4];
  uint32_t fl;      // ulane_final column
  uint32_t lane;
};
__device__ __forceinline__ UnitLane unit_lane() {
  UnitLane U;
  U.S = crc_lane();
  const uint32_t l = threadIdx.x & 63, c = l & 7, o = (l >> 3) & 3;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t t = ((uint32_t)k + o) & 3u;
    U.gpc[k] = ((t & 1u) << 6) | ((t >> 1) << 5) | (c << 2);
    // byte0 <- gpc.b0, byte1 <- state byte t, bytes 2, 3 <- 0 (tables at 0)
    U.gsel[k] = 0x0C0C0000u | ((4u + t) << 8);
  }
  U.fl = ((l >> 5) << 8) | 128u | ((l & 31) << 2);
  U.lane = l;
  return U;
}

// zshift(s, 1012) ^ w: the pending step of a piece's last word plus the
// 1008 bytes to the lane's piece in the next unit.
__device__ __forceinline__ uint32_t crc_gap4x(uint32_t s, const UnitLane& U, uint32_t w) {
  const uint32_t a0 = __builtin_amdgcn_perm(s, U.gpc[0], U.gsel[0]);
  const uint32_t a1 = __builtin_amdgcn_perm(s, U.gpc[1], U.gsel[1]);
  const uint32_t a2 = __builtin_amdgcn_perm(s, U.gpc[2], U.gsel[2]);
  const uint32_t a3 = __builtin_amdgcn_perm(s, U.gpc[3], U.gsel[3]);
  return xor3(xor3(lds_u32(a0), lds_u32(a1), lds_u32(a2)), lds_u32(a3), w);
}

// zshift(s, 4 + 16 (63 - l)): a lane's pending state to the unit's end.
__device__ __forceinline__ uint32_t unit_lane_final(uint32_t s, uint32_t fl) {
  uint32_t x[8];
#pragma unroll
  for (int n = 0; n < 8; n++) x[n] = lds_u32((uint32_t)n * 8192u + (((s >> (4 * n)) & 15u) << 9) + fl);
  return xor3(xor3(x[0], x[1], x[2]), xor3(x[3], x[4], x[5]), x[6] ^ x[7]);
}

__device__ __forceinline__ uint32_t unit_unshift(uint32_t k, uint32_t s) {
  return crc_nibmap(kULdsUnshift + k * 512, s);
}

// A linear map given as 8 nibble tables in global memory (wave-uniform s).
__device__ __forceinline__ uint32_t gmem_nibmap(const uint32_t (*tab)[16], uint32_t s) {
  uint32_t r = 0;
#pragma unroll
  for (int n = 0; n < 8; n++) r ^= tab[n][(s >> (4 * n)) & 15u];
  return r;
}

// ---- spans and units ---------------------------------------------------------
__device__ __forceinline__ uint32_t unit_count(uint64_t ptr, uint32_t n) {
  const uint64_t a0 = ptr & ~15ull, a1 = (ptr + n + 15) & ~15ull;
  return n ? (uint32_t)(((a1 - a0) >> 4) + 63) >> 6 : 0u;
}

// staged descriptor: {off lo, off hi, len, inj}
__device__ __forceinline__ uint4 unit_desc(uint32_t t) {
  const span_u32x4 v = *reinterpret_cast<__attribute__((address_space(3))) const span_u32x4*>(
      static_cast<size_t>(kULdsDesc + 16 * t));
  return make_uint4(v.x, v.y, v.z, v.w);
}
// exclusive prefix of the window's units: upre(t) = first unit of span t
__device__ __forceinline__ uint32_t upre(uint32_t t) { return *lds_p32(kULdsUpre + 4 * t); }

template <class Op>
__device__ __forceinline__ uint32_t unit_init(const Op& op, int kind, uint32_t key) {
  return kind == kInitArray ? key : kind == kInitTyped ? op.typed_init(key & 15u) : 0u;
}

// Epilogue inputs through VECTOR loads: i and ptr are wave-uniform here, and
// the compiler would turn loads at uniform addresses into scalar loads,
// whose lgkmcnt every LDS wait of the table steps then drains.
template <class Op>
__device__ __forceinline__ typename Op::Pre unit_pre(const Op& op, uint32_t i, uint64_t ptr, uint64_t n) {
  asm volatile("" : "+v"(i), "+v"(ptr));
  return op.pre(i, ptr, n);
}

// Share window: slots [0, wn) are spans idx(slot).
struct UShare {
  uint32_t start, stride;
  __device__ uint32_t idx(uint32_t t) const { return start + stride * t; }
};

__device__ __forceinline__ uint32_t rfl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

// One iteration's NU unit slots, worked out lane-parallel (lane j mod NU
// computes slot j): the load addresses come back as scalars (v_readlane),
// the flags as ballots; the rest stays in the lanes and is read (v_readlane,
// in wave-uniform branches) only by a head, tail or end slot.  Slot j is
// window unit g0 + j of the wave's stream.
// NU = 8 for ops without epilogue inputs (OpCrcValue: two iterations' 16
// pieces and plans fit 128 VGPRs), 4 for the block / WAL / blob ops, whose
// two prefetched epilogue inputs per plan would spill at 8 (A/B: 4300-B
// Value blocks 0.599 at 8 vs 0.585 at 4; the SST verify mix spilled 80 B
// per lane at 8 and lost 20 %).
template <class Op>
constexpr uint32_t unit_slots_of() {
  return sizeof(typename Op::Pre) <= 4 ? 8u : 4u;
}
// flags: 8 bits each, bit j = slot j
constexpr uint32_t kUFirst = 1u, kUHead = 1u << 8, kUTail = 1u << 16, kUEnd = 1u << 24;
template <uint32_t NU>
struct USlots {
  uint64_t base[NU];   // slot j's unit: [base, base + 1 KiB)
  uint32_t below[NU];  // lanes below this load the zero piece (64: no unit)
  uint32_t flags;           // kUFirst << j: the lane state restarts (span head or stream
                            // start); kUHead << j: the span's head unit; kUTail << j: its
                            // last unit, with bytes past the end; kUEnd << j: the stream's
                            // portion of the span ends
  uint32_t g0;
  // per lane (slot lane & (NU - 1)): own | hb << 8 | kt << 16, the injected
  // init state, the window slot
  uint32_t h, inj, t;
};

// Plan the slots of units g0 .. g0 + NU - 1 of stream [gs, ge); tc = a span
// at or before the span of unit g0 (advanced here).
template <uint32_t NU>
__device__ __forceinline__ USlots<NU> unit_slots(uint32_t g0, uint32_t gs, uint32_t ge, uint32_t wn, uint32_t& tc,
                                                 uint64_t base, uint32_t lane) {
  static_assert(NU == 4 || NU == 8, "unit slots per iteration");
  USlots<NU> P;
  P.g0 = g0;
  // spans tc + 1 + lane: the spans that start at or before unit g are
  // counted by a ballot over the window's unit prefix (empty spans included,
  // the prefix padded with ~0); tc stays at or before the span of g0
  uint32_t v = upre(tc + 1 + lane);
  uint32_t c0 = (uint32_t)__popcll(__ballot(v <= g0));
  while (c0 == 64) {  // 64 or more spans start in (tc, g0]: skip ahead
    tc += 64;
    v = upre(tc + 1 + lane);
    c0 = (uint32_t)__popcll(__ballot(v <= g0));
  }
  // the later slots from the same lookahead; a full count (64 spans starting
  // in (tc, g0 + j]: runs of empty spans) walks on from tc + 64.  Slots past
  // the window's last unit (the last stream's final plans) count upre(wn) =
  // T too: they are clamped to the last span, so every descriptor and
  // epilogue load such a slot issues is a real span's.
  const uint32_t tl = wn - 1;
  const uint32_t j = lane & (NU - 1);
  uint32_t t = min(tc + c0, tl), tlast = t;
#pragma unroll
  for (uint32_t q = 1; q < NU; q++) {
    const uint32_t gq = g0 + q;
    uint32_t c = (uint32_t)__popcll(__ballot(v <= gq));
    uint32_t tb = tc;
    while (c == 64) {
      tb += 64;
      c = (uint32_t)__popcll(__ballot(upre(tb + 1 + lane) <= gq));
    }
    const uint32_t tq = min(tb + c, tl);
    t = j == q ? tq : t;
    tlast = tq;
  }
  tc = tlast;
  const uint32_t g = g0 + j;
  const bool live = g < ge;
  const uint4 d = unit_desc(t);
  const uint32_t u0 = upre(t), u1 = upre(t + 1);
  const uint64_t ptr = base + (((uint64_t)d.y << 32) | d.x);
  const uint64_t a1 = (ptr + d.z + 15) & ~15ull;
  const uint32_t kt = (uint32_t)(a1 - (ptr + d.z));
  const uint32_t U = u1 - u0, kk = u1 - 1 - g;  // unit kk from the span's end
  const bool head = live && kk == U - 1;
  const uint32_t own = 64u * U - (uint32_t)((a1 - (ptr & ~15ull)) >> 4);
  const uint64_t ub = a1 - (uint64_t)kUnitBytes * (kk + 1);
  const uint32_t below = live ? (head ? own : 0u) : 64u;
  const bool tail = live && kk == 0 && kt != 0;
  const bool first = live && (g == gs || head);
  const bool end = live && (g + 1 == ge || kk == 0);
  constexpr uint32_t m = (1u << NU) - 1u;
  P.flags = ((uint32_t)__ballot(first) & m) * kUFirst | ((uint32_t)__ballot(head) & m) * kUHead |
            ((uint32_t)__ballot(tail) & m) * kUTail | ((uint32_t)__ballot(end) & m) * kUEnd;
#pragma unroll
  for (uint32_t q = 0; q < NU; q++) {
    P.base[q] = readlane_u64(ub, q);
    P.below[q] = readlane_u32(below, q);
  }
  P.h = own | (((uint32_t)ptr & 15u) << 8) | (kt << 16);
  P.inj = d.w;
  P.t = t;
  return P;
}

// The plan's loads: lane l's piece of every slot's unit (the zero piece for
// lanes before a span's head and for empty slots).  Straight-line, so every
// load is unconditional and the waits exact.
template <uint32_t NU>
__device__ __forceinline__ ChunkN<NU> unit_load(const USlots<NU>& P, uint32_t lane16, uint32_t lane, uint64_t zp) {
  ChunkN<NU> c;
#pragma unroll
  for (uint32_t j = 0; j < NU; j++) c.v[j] = span_load16<true>(lane < P.below[j] ? zp : P.base[j] + lane16);
  return c;
}

// keep bytes >= h of a 16-byte piece (h < 16)
__device__ __forceinline__ void unit_mask_head(uint4& v, uint32_t h) {
  uint32_t* w = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int z = (int)h - 4 * q;
    w[q] &= z <= 0 ? 0xFFFFFFFFu : z >= 4 ? 0u : 0xFFFFFFFFu << (8 * z);
  }
}
// keep the first 16 - k bytes (k < 16)
__device__ __forceinline__ void unit_mask_tail(uint4& v, uint32_t k) {
  uint32_t* w = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int keep = 16 - (int)k - 4 * q;
    w[q] &= keep >= 4 ? 0xFFFFFFFFu : keep <= 0 ? 0u : 0xFFFFFFFFu >> (8 * (4 - keep));
  }
}

// The stream's portion of span t ends with unit g (lane state s): reduce it
// to the state at the unit's end.  A span inside the stream [gs, ge) is
// finished at once; a span cut by stream boundaries has its portion moved to
// the span end by zshift(1024 kk) (kk = units after g: pow1k) and XORed into
// the span's LDS accumulator, whose counter sums the portions' units: the
// stream whose portion completes the span's U units runs the epilogue.
template <class Op>
__device__ __forceinline__ void unit_flush(const Op& op, const UShare& sh, uint64_t base, uint32_t t, uint32_t g,
                                           uint32_t s, const typename Op::Pre& pre, uint32_t gs, uint32_t ge,
                                           const UnitLane& UL, const CrcTables* __restrict__ gt) {
  uint32_t p = wave_xor32(unit_lane_final(s, UL.fl));  // pure state at the end of unit g
  const uint4 d = unit_desc(t);
  const uint64_t ptr = base + (((uint64_t)d.y << 32) | d.x);
  const uint32_t n = d.z;
  const uint32_t kt = (uint32_t)(((ptr + n + 15) & ~15ull) - (ptr + n));
  const uint32_t u0 = upre(t), u1 = upre(t + 1);
  const uint32_t i = sh.idx(t);
  if (u0 < gs || u1 > ge) {  // wave-uniform: a shared span
    const uint32_t pu = g + 1 - (u0 > gs ? u0 : gs);  // this portion's units
    for (uint32_t kk = u1 - 1 - g, b = 0; kk; kk >>= 1, b++)
      if (kk & 1) p = gmem_nibmap(gt->pow1k[b], p);
    uint32_t c = 0;
    if (UL.lane == 0) {
      __hip_atomic_fetch_xor(lds_p32(kULdsAcc + 8 * t), p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      c = __hip_atomic_fetch_add(lds_p32(kULdsAcc + 8 * t + 4), pu, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (c + pu == u1 - u0)
        p = __hip_atomic_load(lds_p32(kULdsAcc + 8 * t), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    c = rfl(c);
    if (c + pu != u1 - u0) return;
    p = rfl(p);
    if (kt) p = unit_unshift(kt, p);
    op.finish(i, ~p, unit_pre(op, i, ptr, n), UL.lane == 0);
    return;
  }
  if (kt) p = unit_unshift(kt, p);
  op.finish(i, ~p, pre, UL.lane == 0);
}

// The wave's stream over one share window: units [gs, ge) of the window's
// unit sequence (spans in window order, each span's units in address order),
// NU per iteration, the next iteration's loads and the epilogue inputs of its
// first two span ends issued before the current one is folded.
template <class Op>
__device__ __forceinline__ void crc_units_window(const Op& op, const UShare& sh, uint32_t wn,
                                                 const CrcTables* __restrict__ g) {
  const UnitLane UL = unit_lane();
  const uint32_t lane = UL.lane, lane16 = 16u * lane;
  const uint64_t base = reinterpret_cast<uint64_t>(op.base());
  const uint64_t zp = reinterpret_cast<uint64_t>(&g->zero16[0]);
  typedef typename Op::Pre Pre;
  constexpr uint32_t NU = unit_slots_of<Op>();
  typedef USlots<NU> Slots;
  const uint32_t T = rfl(upre(wn));  // the window's units
  const uint32_t W = blockDim.x >> 6, w = threadIdx.x >> 6;
  const uint32_t gs = rfl((uint32_t)((uint64_t)T * w / W)), ge = rfl((uint32_t)((uint64_t)T * (w + 1) / W));
  if (gs >= ge) return;
  uint32_t tc = 0;
  // epilogue inputs of span end number e of a plan (its first two: a fixed
  // number of loads per iteration keeps vmcnt exact; fewer ends repeat one)
  const auto end_slot = [](const Slots& X, uint32_t e) {
    uint32_t m = X.flags / kUEnd;
    if (e) m &= m - 1;
    return m ? (uint32_t)__builtin_ctz(m) : 0u;
  };
  const auto pre_of = [&](const Slots& X, uint32_t j) {
    const uint32_t t = readlane_u32(X.t, j);
    const uint4 d = unit_desc(t);
    return unit_pre(op, sh.idx(t), base + (((uint64_t)d.y << 32) | d.x), d.z);
  };
  Slots P = unit_slots<NU>(gs, gs, ge, wn, tc, base, lane);
  ChunkN<NU> cur = unit_load(P, lane16, lane, zp);
  Pre pre0 = pre_of(P, end_slot(P, 0)), pre1 = pre_of(P, end_slot(P, 1));
  uint32_t s = 0;
  for (uint32_t g0 = gs; g0 < ge; g0 += NU) {
    const Slots Q = unit_slots<NU>(g0 + NU, gs, ge, wn, tc, base, lane);
    const ChunkN<NU> nxt = unit_load(Q, lane16, lane, zp);
    const Pre pn0 = pre_of(Q, end_slot(Q, 0)), pn1 = pre_of(Q, end_slot(Q, 1));
    const uint32_t f = P.flags;
    uint32_t se[NU];  // the lane state after each slot (the span ends' states)
#pragma unroll
    for (uint32_t j = 0; j < NU; j++) {
      uint4 v = cur.v[j];
      uint32_t extra = 0;
      if (f & (kUHead << j)) {  // wave-uniform: the head unit of a span
        const uint32_t h = readlane_u32(P.h, j);
        if (lane == (h & 255u)) {
          unit_mask_head(v, (h >> 8) & 15u);
          extra = readlane_u32(P.inj, j);
        }
      }
      if (f & (kUTail << j)) {
        const uint32_t h = readlane_u32(P.h, j);
        if (lane == 63) unit_mask_tail(v, h >> 16);
      }
      // a unit's first piece: zshift(state, 1012) ^ w0 -- from state 0 (and
      // the init injected at the head piece) when a portion starts here
      uint32_t x = crc_gap4x((f & (kUFirst << j)) ? 0u : s, UL, v.x ^ extra);
      x = crc_step4x(x, UL.S, v.y);
      x = crc_step4x(x, UL.S, v.z);
      s = crc_step4x(x, UL.S, v.w);
      se[j] = s;
    }
    // the portions that end in this iteration (one code copy for all)
    uint32_t nend = 0;
    for (uint32_t m = f / kUEnd; m; m &= m - 1, nend++) {
      const uint32_t j = (uint32_t)__builtin_ctz(m);
      uint32_t sj = se[0];
#pragma unroll
      for (uint32_t q = 1; q < NU; q++) sj = j == q ? se[q] : sj;
      const Pre pr = nend == 0 ? pre0 : nend == 1 ? pre1 : pre_of(P, j);
      unit_flush(op, sh, base, readlane_u32(P.t, j), P.g0 + j, sj, pr, gs, ge, UL, g);
    }
    P = Q;
    cur = nxt;
    pre0 = pn0;
    pre1 = pn1;
  }
}

// Ragged batch [first, first + count): workgroup b owns the contiguous
// range [count b / G, count (b + 1) / G) (BLK) or spans b, b + G, ...;
// processed in windows of kUDescCache descriptors.  A window's units are
// cut into W equal streams, one per wave: every wave gets the same number of
// units (no tickets), and a span longer than a stream is simply shared by
// the neighbouring streams.
template <class Op>
__device__ __forceinline__ void crc_units_driver(const Op& op, const RowShare& share, const CrcTables* __restrict__ g) {
  crc_units_fill(g);
  const uint32_t start = share.start, stride = share.stride, n = share.n;
  const uint64_t base = reinterpret_cast<uint64_t>(op.base());
  const int kind = op.init_kind();
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6, wpb = blockDim.x >> 6;
  __syncthreads();  // the un-shift tables are read by the staging
  for (uint32_t w0 = 0; w0 < n; w0 += kUDescCache) {
    const uint32_t wn = n - w0 < kUDescCache ? n - w0 : kUDescCache;
    const UShare sh{start + stride * w0, stride};
    if (w0) __syncthreads();  // the previous window's waves are done with its slots
    // descriptors, accumulators, and the units' exclusive prefix (a chunk of
    // blockDim spans at a time); padded with ~0 for the streams' lookahead
    uint32_t carry = 0;
    for (uint32_t c0 = 0; c0 < wn; c0 += blockDim.x) {
      const uint32_t t = c0 + threadIdx.x;
      uint32_t u = 0;
      if (t < wn) {
        const uint32_t i = sh.idx(t);
        const uint64_t off = op.off(i);
        const uint32_t len = (uint32_t)op.len(i);
        const uint32_t init = unit_init(op, kind, op.init_key(i));
        const uint32_t hb = (uint32_t)(base + off) & 15u;
        const uint32_t inj = hb ? unit_unshift(hb, ~init) : ~init;
        const span_u32x4 d = {(uint32_t)off, (uint32_t)(off >> 32), len, inj};
        *reinterpret_cast<__attribute__((address_space(3))) span_u32x4*>(static_cast<size_t>(kULdsDesc + 16 * t)) = d;
        *lds_p64(kULdsAcc + 8 * t) = 0;
        u = unit_count(base + off, len);
        // Extend(init, "") = init: empty spans (no units) finish here
        if (len == 0) op.finish(i, init, op.pre(i, base + off, 0), true);
      }
      uint32_t x = u;
#pragma unroll
      for (int dd = 1; dd < 64; dd <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, dd, 64);
        x += lane >= (uint32_t)dd ? y : 0u;
      }
      if (lane == 63) *lds_p32(kULdsWaveSum + 4 * wid) = x;
      __syncthreads();
      uint32_t below = 0, tot = 0;
      for (uint32_t q = 0; q < wpb; q++) {
        const uint32_t ws = *lds_p32(kULdsWaveSum + 4 * q);
        below += q < wid ? ws : 0u;
        tot += ws;
      }
      if (t < wn) *lds_p32(kULdsUpre + 4 * t) = carry + below + x - u;
      carry += tot;
      __syncthreads();
    }
    if (threadIdx.x <= 64) *lds_p32(kULdsUpre + 4 * (wn + threadIdx.x)) = threadIdx.x ? 0xFFFFFFFFu : carry;
    __syncthreads();
    crc_units_window(op, sh, wn, g);
  }
}

// Ragged batches: the driver is chosen per workgroup from its share's mean
// span length (the host cannot see device-resident lengths): 8-lane rows up
// to 640 B, 16-lane rows up to 2.5 KiB, the unit stream up to 8 KiB when the
// spans would leave the wave driver's 4 KiB rounds > 20 % empty, else the
// wave driver.
// force: 0 = by length, 1 = the 4 KiB-round wave driver, 2 = rows16,
// 3 = rows8, 4 = unit stream, 5 = rows4, 6 = one lane per span.
constexpr uint32_t kAutoUnitsMin = 2560, kAutoUnitsMax = 8192;  // mean span bytes
constexpr uint32_t kAutoRows1Max = 80;
template <class Op, bool T, bool BLK>
__device__ __forceinline__ void crc_auto_units_driver(const Op& op, uint32_t first, uint32_t count, uint8_t* lds,
                                                      const CrcTables* __restrict__ g, int force) {
  // the workgroup's share (contiguous ranges: neighbouring spans on one CU;
  // interleaved under the test hook) -- every driver works on the same one
  const RowShare sh = row_share<BLK>(first, count);
  if (sh.n == 0) return;  // workgroup-uniform (the row feed would read an unstaged slot 0)
  int mode = force;
  bool lpt = force == 1;
  if (!mode) {
    // Stage the share for the row drivers first (LDS tables, descriptors,
    // init tables) and choose from the staging's totals: the share's bytes
    // and the bytes the wave driver's 4 KiB rounds would cover.  Row-driver
    // shares (short spans, many launches per batch) then read their lengths
    // once instead of twice; the wave driver restages longest first and the
    // unit stream stages its own.
    crc_rows_prologue<Op>(op, sh, lds, g, true, false);
    const uint64_t total = *lds_p64(kLdsRowTotal), wtotal = *lds_p64(kLdsRowWaveTotal);
    const bool longs = *lds_p32(kLdsRowLongs) != 0;
    const uint64_t mean = total / (sh.n ? sh.n : 1);
    // one lane per span below ~80 B (20-100 B: 0.16-0.19 vs 0.09 of peak on
    // 8-lane rows, whose 512-B rounds are mostly padding there; 50-150 B:
    // 0.14 vs 0.15, 100-300 B: 0.17 vs 0.25 -- a lane's span switch every
    // few rounds costs the whole wave);
    // the unit stream for spans of a few KiB that waste the wave driver's
    // rounds (4100-4400 B: 0.60 vs 0.54 of peak); aligned 4 KiB multiples
    // and the long spans of the SST mix stay on the wave driver (4096 B: 0.74
    // vs 0.69; 4/16/64 KiB mix: 0.67 vs 0.57)
    // Ops with epilogue inputs run 4 unit slots (unit_slots_of) and lose
    // there: blob records of 16 + 4096 B at 16-byte-misaligned offsets read
    // 0.42 of peak on the unit stream, 0.55 on 16-lane rows.
    const bool waste = 4 * wtotal > 5 * total;
    const int few = unit_slots_of<Op>() == 8 ? 4 : 2;
    mode = mean <= kAutoRows1Max            ? 6
           : mean <= kAutoRows8Max          ? 3
           : mean <= kAutoUnitsMin          ? 2
           : mean <= kAutoUnitsMax && waste ? few
                                            : 1;
    __syncthreads();  // every wave has read the totals (the unit stream refills the LDS)
    if (mode == 1 && longs) {  // longest first for the wave driver (with spans of >= 8 KiB)
      row_desc_stage<Op>(op, sh, false, true);
      __syncthreads();
    }
    lpt = mode == 1 && longs;
  } else if (force != 4 && force != 7) {
    crc_rows_prologue<Op>(op, sh, lds, g, true, force == 1);
  }
  if (mode == 4)
    crc_units_driver<Op>(op, sh, g);
  else
    crc_auto_dispatch<Op, T>(op, sh, g, mode, lpt);
}

}  // namespace mck
