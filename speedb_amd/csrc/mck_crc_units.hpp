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
// Stream.  Each wave consumes UNITS, four per loop iteration (4 KiB in
// flight, the next iteration's loads issued before the current one is
// folded), from a queue of ITEMS that crosses span boundaries: a 4300-B
// block is 5 units, and an iteration holds the last unit of one block and
// the first three of the next.  Items come from an LDS ticket shared by the
// workgroup's 16 waves.  Spans of more than 24 units are split into 16 KiB
// PIECES (items of their own, end-anchored, the head piece 9..24 units):
// a piece's partial state is moved to the span end by zshift(16384 m)
// (pow16k), XORed into the span's LDS accumulator, and the wave that
// completes the span's last piece (an LDS counter) runs the epilogue -- no
// span keeps one wave busy for more than 24 units.
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
//   [128K, ..)  un-shift by k < 16, byte masks, ticket, the share's
//               descriptors and the split spans' accumulators.
#pragma once
#include "mck_crc.hpp"

namespace mck {

constexpr uint32_t kUnitBytes = 1024;
constexpr uint32_t kPieceUnits = 16;    // units per piece of a split span
constexpr uint32_t kSplitUnits = 24;    // spans of more units are split
constexpr uint32_t kULdsUnshift = 131072;                        // [16][8][16]
constexpr uint32_t kULdsMaskHead = kULdsUnshift + 16 * 512;      // [16] x 16 B: keep bytes >= h
constexpr uint32_t kULdsMaskTail = kULdsMaskHead + 256;          // [16] x 16 B: keep the first 16 - k
constexpr uint32_t kULdsTicket = kULdsMaskTail + 256;            // u64 {slot, piece}
constexpr uint32_t kUDescCache = 960;                            // descriptors per window
constexpr uint32_t kULdsDesc = kULdsTicket + 64;                 // 16 B {off lo, off hi, len, key}
constexpr uint32_t kULdsAcc = kULdsDesc + 16 * kUDescCache;      // {xor, count} per slot
constexpr uint32_t kULdsEnd = kULdsAcc + 8 * kUDescCache;
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

// ---- items ----------------------------------------------------------------
// One item = one span (<= 24 units) or one 16 KiB piece of a longer span.
// Wave-uniform (SGPRs).  Units are processed from khi down to klo (address
// order).
struct UItem {
  uint64_t ptr;   // span start (device address)
  uint64_t a1;    // span end rounded up to 16
  uint32_t t;     // slot in the share window
  uint32_t U;     // units of the span
  uint32_t M, m;  // pieces of the span, this piece (0 = last)
  uint32_t kt;    // a1 - end
  uint32_t inj;   // unshift(~init, ptr & 15): Extend's init state at the piece holding ptr
  __device__ uint32_t klo() const { return kPieceUnits * m; }
  __device__ uint32_t khi() const { return m == M - 1 ? U - 1 : kPieceUnits * m + kPieceUnits - 1; }
  // head unit: lanes below own load zeros, lane own holds ptr
  __device__ uint32_t own() const { return 64u * U - (uint32_t)((a1 - (ptr & ~15ull)) >> 4); }
  __device__ uint32_t hb() const { return (uint32_t)ptr & 15u; }
  __device__ uint64_t n() const { return a1 - kt - ptr; }
};

__device__ __forceinline__ uint32_t unit_count(uint64_t ptr, uint32_t n) {
  const uint64_t a0 = ptr & ~15ull, a1 = (ptr + n + 15) & ~15ull;
  return n ? (uint32_t)(((a1 - a0) >> 4) + 63) >> 6 : 0u;
}
// items of a span: 0 for an empty span (finished when the window is staged)
__device__ __forceinline__ uint32_t unit_pieces(uint32_t U) {
  return U == 0 ? 0u : U <= kSplitUnits ? 1u : (U - 9u) / kPieceUnits + 1u;
}

// staged descriptor: {off lo, off hi, len, inj}
__device__ __forceinline__ uint4 unit_desc(uint32_t t) {
  const span_u32x4 v = *reinterpret_cast<__attribute__((address_space(3))) const span_u32x4*>(
      static_cast<size_t>(kULdsDesc + 16 * t));
  return make_uint4(v.x, v.y, v.z, v.w);
}

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

// Take the next item of the window: lane 0 advances the {slot, piece}
// ticket with a CAS (empty spans, finished at staging, are skipped); the
// item is wave-uniform.  Only LDS traffic (no memory op: the caller's
// in-flight loads are not waited for).  False when the window is exhausted.
__device__ __forceinline__ bool unit_take(uint32_t wn, uint64_t base, UItem* it) {
  uint32_t t = 0xFFFFFFFFu, q = 0;
  uint4 d = make_uint4(0, 0, 0, 0);
  if ((threadIdx.x & 63) == 0) {
    uint64_t old = __hip_atomic_load(lds_p64(kULdsTicket), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    for (;;) {
      const uint32_t ot = (uint32_t)old, oq = (uint32_t)(old >> 32);
      if (ot >= wn) break;
      const uint4 x = unit_desc(ot);
      const uint32_t M = unit_pieces(unit_count(base + (((uint64_t)x.y << 32) | x.x), x.z));
      const uint64_t nw = oq + 1 < M ? old + (1ull << 32) : (uint64_t)(ot + 1);
      if (__hip_atomic_compare_exchange_strong(lds_p64(kULdsTicket), &old, nw, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP)) {
        if (M == 0) {  // an empty span: nothing to hash
          old = nw;
          continue;
        }
        t = ot;
        q = oq;
        d = x;
        break;
      }
    }
  }
  t = rfl(t);
  if (t >= wn) return false;
  q = rfl(q);
  const uint64_t ptr = base + (((uint64_t)rfl(d.y) << 32) | rfl(d.x));
  const uint32_t n = rfl(d.z);
  it->ptr = ptr;
  it->t = t;
  it->a1 = (ptr + n + 15) & ~15ull;
  it->U = unit_count(ptr, n);
  it->M = unit_pieces(it->U);
  it->m = it->M - 1 - q;
  it->kt = (uint32_t)(it->a1 - (ptr + n));
  it->inj = rfl(d.w);
  return true;
}

// One iteration's four unit slots, precomputed when the iteration is planned
// (wave-uniform, SGPRs): slots [0, na) are units of item A (the cursor's
// item), slots [na, na + nb) the first units of item B (the prefetched
// next item); the rest are empty.  A plan ends at most one item (A): B is
// taken only if it continues past the plan, so one set of epilogue inputs
// per iteration suffices.
constexpr uint32_t kUFirst = 1u, kUHead = 16u, kUTail = 256u, kUAEnd = 4096u;  // << slot
struct UPlan {
  uint64_t base[4];   // slot j's unit: [base, base + 1 KiB)
  uint32_t below[4];  // lanes below this load the zero piece (64: empty slot)
  uint32_t flags;     // kUFirst << j: an item starts at slot j; kUHead << j: ... at its span's
                      // head unit; kUTail << j: slot j is its span's last unit; kUAEnd: A ends
  uint32_t na;
  uint32_t hA, hB;    // own | hb << 8 | kt << 16 of A's and B's spans
  uint32_t injA, injB;
  uint32_t At, Am;    // A's window slot and piece (the flush re-reads the rest)
};

struct UnitCursor {
  UItem C, N;  // current item (units kc, kc - 1, ... not yet loaded), prefetched next item
  uint32_t kc;
  bool cv, nv;  // valid
};

__device__ __forceinline__ uint32_t unit_hpack(const UItem& I) { return I.own() | (I.hb() << 8) | (I.kt << 16); }

// Plan the next iteration from the cursor; sets *consumed when N was used
// (the caller takes a new N after issuing the loads).
__device__ __forceinline__ UPlan unit_plan(UnitCursor& q, bool* consumed) {
  UPlan P;
  *consumed = false;
  if (!q.cv && q.nv) {  // the previous item ended on the iteration boundary
    q.C = q.N;
    q.kc = q.C.khi();
    q.cv = true;
    q.nv = false;
    *consumed = true;
  }
#pragma unroll
  for (int j = 0; j < 4; j++) {
    P.base[j] = 0;
    P.below[j] = 64;
  }
  P.flags = 0;
  P.na = 0;
  P.hA = P.hB = P.injA = P.injB = 0;
  P.At = q.C.t;
  P.Am = q.C.m;
  if (!q.cv) return P;
  const UItem& C = q.C;
  const uint32_t avail = q.kc - C.klo() + 1;
  const uint32_t na = avail < 4 ? avail : 4;
  P.na = na;
  P.hA = unit_hpack(C);
  P.injA = C.inj;
  const uint32_t ownA = C.own();
#pragma unroll
  for (uint32_t j = 0; j < 4; j++) {
    if (j < na) {
      const uint32_t k = q.kc - j;
      P.base[j] = C.a1 - (uint64_t)kUnitBytes * (k + 1);
      P.below[j] = k == C.U - 1 ? ownA : 0u;
      P.flags |= (k == C.U - 1 ? kUHead << j : 0u) | (k == 0 && C.kt ? kUTail << j : 0u);
    }
  }
  if (q.kc == C.khi()) P.flags |= kUFirst;
  if (avail > 4) {
    q.kc -= 4;
    return P;
  }
  P.flags |= kUAEnd;
  q.cv = false;
  if (na < 4 && q.nv) {
    const UItem& N = q.N;
    const uint32_t bu = N.khi() - N.klo() + 1;
    if (bu > 4 - na) {  // B continues past this plan (so none of its slots is its last unit)
      const uint32_t kh = N.khi(), ownB = N.own();
#pragma unroll
      for (uint32_t j = 1; j < 4; j++) {
        if (j >= na) {
          const uint32_t k = kh - (j - na);
          P.base[j] = N.a1 - (uint64_t)kUnitBytes * (k + 1);
          P.below[j] = k == N.U - 1 ? ownB : 0u;
          P.flags |= (k == N.U - 1 ? kUHead << j : 0u) | (j == na ? kUFirst << j : 0u);
        }
      }
      P.hB = unit_hpack(N);
      P.injB = N.inj;
      q.nv = false;
      *consumed = true;
      q.C = N;
      q.kc = kh - (4 - na);
      q.cv = true;
    }
  }
  return P;
}

// The four loads of plan P: lane l's piece of every slot's unit (the zero
// piece for lanes before a span's head and for empty slots).  Straight-line,
// so every load is unconditional and the waits exact.
__device__ __forceinline__ Chunk unit_load(const UPlan& P, uint32_t lane16, uint32_t lane, uint64_t zp) {
  Chunk c;
#pragma unroll
  for (int j = 0; j < 4; j++) c.v[j] = span_load16<true>(lane < P.below[j] ? zp : P.base[j] + lane16);
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

// Item (window slot t, piece m) has its last unit folded (lane state s):
// reduce, and either run the epilogue or (piece of a split span) add the
// partial to the span's accumulator; the wave completing the span's last
// piece runs the epilogue.
template <class Op>
__device__ __forceinline__ void unit_flush(const Op& op, const UShare& sh, uint64_t base, uint32_t t, uint32_t m,
                                           uint32_t s, const typename Op::Pre& pre, const UnitLane& UL,
                                           const CrcTables* __restrict__ g) {
  uint32_t p = wave_xor32(unit_lane_final(s, UL.fl));  // pure state at a1 - 1024 klo
  const uint4 d = unit_desc(t);
  const uint64_t ptr = base + (((uint64_t)d.y << 32) | d.x);
  const uint32_t n = d.z;
  const uint32_t kt = (uint32_t)(((ptr + n + 15) & ~15ull) - (ptr + n));
  const uint32_t M = unit_pieces(unit_count(ptr, n));
  const uint32_t i = sh.idx(t);
  if (M > 1) {
    for (uint32_t mm = m, b = 0; mm; mm >>= 1, b++)
      if (mm & 1) p = gmem_nibmap(g->pow16k[b], p);
    uint32_t c = 0;
    if (UL.lane == 0) {
      __hip_atomic_fetch_xor(lds_p32(kULdsAcc + 8 * t), p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      c = __hip_atomic_fetch_add(lds_p32(kULdsAcc + 8 * t + 4), 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (c == M - 1) p = __hip_atomic_load(lds_p32(kULdsAcc + 8 * t), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    c = rfl(c);
    if (c != M - 1) return;
    p = rfl(p);
    if (kt) p = unit_unshift(kt, p);
    op.finish(i, ~p, unit_pre(op, i, ptr, n), UL.lane == 0);
    return;
  }
  if (kt) p = unit_unshift(kt, p);
  op.finish(i, ~p, pre, UL.lane == 0);
}

// The wave loop over one share window.
template <class Op>
__device__ __forceinline__ void crc_units_window(const Op& op, const UShare& sh, uint32_t wn,
                                                 const CrcTables* __restrict__ g) {
  const UnitLane UL = unit_lane();
  const uint32_t lane16 = 16u * UL.lane;
  const uint64_t base = reinterpret_cast<uint64_t>(op.base());
  const uint64_t zp = reinterpret_cast<uint64_t>(&g->zero16[0]);
  typedef typename Op::Pre Pre;
  UnitCursor q;
  q.cv = false;
  q.kc = 0;
  q.nv = unit_take(wn, base, &q.N);
  if (!q.nv) return;
  q.C = q.N;
  bool consumed;
  UPlan P = unit_plan(q, &consumed);
  Chunk cur = unit_load(P, lane16, UL.lane, zp);
  // epilogue inputs of the item the plan ends, issued after its chunks in
  // every iteration (a fixed number of loads per iteration keeps vmcnt exact)
  const auto pre_of = [&](const UPlan& X) {
    const uint4 d = unit_desc(X.At);
    return unit_pre(op, sh.idx(X.At), base + (((uint64_t)d.y << 32) | d.x), d.z);
  };
  Pre pre = pre_of(P);
  if (consumed) q.nv = unit_take(wn, base, &q.N);
  uint32_t s = 0;
  while (P.na) {
    bool cn;
    const UPlan Q = unit_plan(q, &cn);
    const Chunk nxt = unit_load(Q, lane16, UL.lane, zp);
    const Pre pn = pre_of(Q);
    if (cn) q.nv = unit_take(wn, base, &q.N);
    uint32_t sA = s;
    const uint32_t f = P.flags;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
      uint4 v = cur.v[j];
      uint32_t extra = 0;
      if (f & (kUHead << j)) {  // wave-uniform: the head unit of a span
        const uint32_t h = j < P.na ? P.hA : P.hB;
        if (UL.lane == (h & 255u)) {
          unit_mask_head(v, (h >> 8) & 15u);
          extra = j < P.na ? P.injA : P.injB;
        }
      }
      if ((f & (kUTail << j)) && UL.lane == 63) unit_mask_tail(v, P.hA >> 16);
      // a unit's first piece: zshift(state, 1012) ^ w0 -- from state 0 (and
      // the init injected at the head piece) when an item starts here
      uint32_t x = crc_gap4x((f & (kUFirst << j)) ? 0u : s, UL, v.x ^ extra);
      x = crc_step4x(x, UL.S, v.y);
      x = crc_step4x(x, UL.S, v.z);
      s = crc_step4x(x, UL.S, v.w);
      if (j + 1 == P.na) sA = s;  // A's last unit in this plan
    }
    if (f & kUAEnd) unit_flush(op, sh, base, P.At, P.Am, sA, pre, UL, g);
    P = Q;
    cur = nxt;
    pre = pn;
  }
}

// Ragged batch [first, first + count): workgroup b owns the contiguous
// range [count b / G, count (b + 1) / G) (BLK) or spans b, b + G, ...;
// processed in windows of kUDescCache descriptors.
template <class Op, bool BLK>
__device__ __forceinline__ void crc_units_driver(const Op& op, uint32_t first, uint32_t count,
                                                 const CrcTables* __restrict__ g) {
  crc_units_fill(g);
  const uint32_t G = gridDim.x, b = blockIdx.x;
  uint32_t start, stride, n;
  if (BLK) {
    const uint32_t lo = (uint32_t)((uint64_t)count * b / G), hi = (uint32_t)((uint64_t)count * (b + 1) / G);
    start = first + lo;
    stride = 1;
    n = hi - lo;
  } else {
    start = first + b;
    stride = G;
    n = count > b ? (count - b + G - 1) / G : 0;
  }
  const uint64_t base = reinterpret_cast<uint64_t>(op.base());
  const int kind = op.init_kind();
  __syncthreads();  // the un-shift tables are read by the staging
  for (uint32_t w0 = 0; w0 < n; w0 += kUDescCache) {
    const uint32_t wn = n - w0 < kUDescCache ? n - w0 : kUDescCache;
    const UShare sh{start + stride * w0, stride};
    if (w0) __syncthreads();  // the previous window's waves are done with its slots
    for (uint32_t t = threadIdx.x; t < wn; t += blockDim.x) {
      const uint32_t i = sh.idx(t);
      const uint64_t off = op.off(i);
      const uint32_t len = (uint32_t)op.len(i);
      const uint32_t init = unit_init(op, kind, op.init_key(i));
      const uint32_t hb = (uint32_t)(base + off) & 15u;
      const uint32_t inj = hb ? unit_unshift(hb, ~init) : ~init;
      const span_u32x4 d = {(uint32_t)off, (uint32_t)(off >> 32), len, inj};
      *reinterpret_cast<__attribute__((address_space(3))) span_u32x4*>(static_cast<size_t>(kULdsDesc + 16 * t)) = d;
      *lds_p64(kULdsAcc + 8 * t) = 0;
      // Extend(init, "") = init: empty spans finish here (the ticket skips them)
      if (len == 0) op.finish(i, init, op.pre(i, base + off, 0), true);
    }
    if (threadIdx.x == 0) *lds_p64(kULdsTicket) = 0;
    __syncthreads();
    crc_units_window(op, sh, wn, g);
  }
}

// Ragged batches: the driver is chosen per workgroup from its share's mean
// span length (the host cannot see device-resident lengths): 8-lane rows up
// to 640 B, 16-lane rows up to 2.5 KiB, the unit stream above.
// force: 0 = by length, 1 = the 4 KiB-round wave driver, 2 = rows16,
// 3 = rows8, 4 = unit stream, 5 = rows4.
constexpr uint32_t kAutoUnitsMin = 2560;  // mean span bytes
template <class Op, bool T, bool BLK>
__device__ __forceinline__ void crc_auto_units_driver(const Op& op, uint32_t first, uint32_t count, uint8_t* lds,
                                                      const CrcTables* __restrict__ g, int force) {
  int mode = force;
  if (!mode) {
    const RowShare sh = row_share<BLK>(first, count);
    uint64_t sum = 0;
    for (uint32_t t = threadIdx.x; t < sh.n; t += blockDim.x) sum += op.len(sh.idx(t));
    for (int m = 32; m >= 1; m >>= 1) sum += __shfl_xor(sum, m, 64);
    if ((threadIdx.x & 63) == 0) *lds_p64(kULdsDesc + 8 * (threadIdx.x >> 6)) = sum;
    __syncthreads();
    uint64_t total = 0;
    for (uint32_t w = 0; w < blockDim.x / 64; w++) total += *lds_p64(kULdsDesc + 8 * w);
    __syncthreads();  // the scratch is overwritten by the drivers' fills
    const uint64_t mean = total / (sh.n ? sh.n : 1);
    mode = mean <= kAutoRows8Max ? 3 : mean <= kAutoUnitsMin ? 2 : 4;
  }
  if (mode == 4)
    crc_units_driver<Op, BLK>(op, first, count, g);
  else
    crc_auto_driver<Op, T, BLK>(op, first, count, lds, g, mode);
}

}  // namespace mck
