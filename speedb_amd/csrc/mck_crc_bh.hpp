// mck_crc_bh.hpp -- the body/head CRC32C driver for ragged batches of spans
// of a few KiB and more (SST data blocks of 4096 + 0..255 B + the type byte,
// the 4/16/64 KiB compaction mix, blob records).
//
// Why.  The wave driver (mck_crc.hpp crc_drive) walks a span in 4 KiB
// rounds anchored at its 16-aligned end.  A 4300-B block is one full round
// plus a head "mini round" of ~200 bytes, and the loop iteration that loads
// that mini round keeps 1 KiB in flight for the wave instead of 4 KiB: the
// rate of a wave is set by the bytes it has in flight per memory latency, so
// a 4 KiB + jitter block costs almost two full rounds (0.54 of the HBM peak
// against 0.74 for aligned 4 KiB).  A 64 KiB span is 16 dependent rounds on
// one wave: the last ones of a launch run while the rest of the GPU drains.
//
// Decomposition.  Span [ptr, ptr + n), a1 = its end rounded up to 16,
// cover = a1 - ptr: BODY = the F = cover / 4096 whole 4 KiB rounds ending at
// a1, HEAD = the h = cover % 4096 bytes before them (the whole span when
// F = 0).  CRC-32C is linear (util/crc32c.cc:1221-1266, Crc32cCombine): the
// span's pure state at a1 is
//     zshift(head state, 4096 F)  ^  XOR_j zshift(piece j state, 4096 R j)
// where the body is cut into PIECES of at most R = kBhPieceRounds rounds
// anchored at a1 (piece j = rounds R j .. R j + R - 1 counted from the end).  ~init is injected
// at ptr (in the head; in the body's first round when h = 0) and the < 16
// bytes past the end are masked and un-shifted at the end, as in crc_drive.
//   * pieces run on the wave driver's round (row-transposed non-temporal
//     loads, 4 KiB in flight per wave, the 4032-byte gap map between rounds,
//     the per-lane final shift and the wave XOR at the piece end);
//   * heads run 16 or 64 AT A TIME, one per 4-lane row or per lane, on the
//     row driver's round (256- or 64-byte rounds of 64-byte lane chunks
//     anchored at the head's end, lanes before the head load the zero
//     piece): one iteration per 16 heads of <= 256 bytes instead of one per
//     head;
//   * each part XORs its state, moved to a1 by zshift(4096 m) (nibble maps
//     of 4096 * 2^b in LDS, one per set bit of m), into the span's LDS
//     accumulator and decrements its part counter; the part that brings it
//     to zero un-shifts the tail and runs the epilogue.  A span of ONE part
//     (a head-only span; a span whose cover is a multiple of 4 KiB and at
//     most 16 KiB) finishes at once.
//
// Scheduling.  A workgroup walks its share in WINDOWS of kBNC spans staged
// in LDS (descriptors, accumulators, the exclusive prefix of the pieces, the
// list of spans with a head).  Its waves take TICKETS from one LDS counter:
// tickets [0, HB) are head batches (8 consecutive heads of the list), the
// rest body pieces in address order (a wave finds a piece's span by a ballot
// over the prefix, searching forward from its previous one).  Heads first:
// a piece -- the span end above all, which holds the epilogue inputs -- is
// then normally the last part of its span.  Every wave keeps one unit (a
// 4 KiB body round or an 8-head round) loaded ahead of the one it folds.
//
// LDS image (160 KiB):
//   [0, 32K)        per-lane final shift (kLdsFinal, as the wave driver)
//   [32K, +512)     gap map 4032 (kLdsGap)
//   then            row gap maps (W = 4, 8, 16), head / tail byte masks,
//                   init injection tables, control words, zshift(4096 * 2^b)
//                   maps, un-shift maps k < 16, the window's head list
//   [64K, 128K)     the 4-byte step tables (kLdsStep, CrcLane)
//   [128K, 160K)    the window's descriptors, accumulators, piece prefix
#pragma once
#include "mck_crc.hpp"

namespace mck {

// A window of a share: slot t is span start + stride t.
struct UShare {
  uint32_t start, stride;
  __device__ uint32_t idx(uint32_t t) const { return start + stride * t; }
};
__device__ __forceinline__ uint32_t rfl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

constexpr uint32_t kBNC = 1024;                          // spans per window (<= kCrcBlock)
constexpr uint32_t kBhPieceRounds = 4;                   // 4 KiB rounds per body piece
constexpr uint32_t kBLdsRowGap = kLdsGap + 512;          // [3] zshift(., 64 (W - 1)): W = 4, 8, 16-lane rows
constexpr uint32_t kBLdsMaskHead = kBLdsRowGap + 1536;   // [16] x 16 B: keep bytes >= h
constexpr uint32_t kBLdsMaskTail = kBLdsMaskHead + 256;  // [16] x 16 B: keep the first 16 - k
constexpr uint32_t kBLdsInj = kBLdsMaskTail + 256;       // [16 types][16 k]: unshift(~init_t, k)
constexpr uint32_t kBLdsInit = kBLdsInj + 1024;          // [16] init_t
constexpr uint32_t kBLdsCtl = kBLdsInit + 64;            // ticket, nheads, npieces, head row width
constexpr uint32_t kBLdsWsum = kBLdsCtl + 16;            // u64 x 16 waves: the scans' wave totals
constexpr uint32_t kBLdsWsum2 = kBLdsWsum + 128;         // u64 x 16 waves: head bytes / heads
constexpr uint32_t kBPowBits = 21;                       // 4096 * 2^b, b <= 20 (spans < 4 GiB)
constexpr uint32_t kBLdsPow = kBLdsCtl + 512;            // [21][8][16]
constexpr uint32_t kBLdsUnshift = kBLdsPow + kBPowBits * 512;  // [16][8][16]
constexpr uint32_t kBLdsHlist = kBLdsUnshift + 16 * 512;       // u32 x kBNC
static_assert(kBLdsHlist + 4 * kBNC <= kLdsStep, "BH low image overlaps the step tables");
constexpr uint32_t kBLdsDesc = kLdsStep + 65536;               // 16 B x kBNC {off lo, off hi, len, key}
constexpr uint32_t kBLdsAcc = kBLdsDesc + 16 * kBNC;           // {xor, parts left} x kBNC
constexpr uint32_t kBLdsBpre = kBLdsAcc + 8 * kBNC;            // u32 x (kBNC + 65)
static_assert(kBLdsBpre + 4 * (kBNC + 65) <= kCrcLdsBytes, "BH image must fit the LDS");
static_assert(kPowBits >= (int)kBPowBits + 2, "pow1k holds zshift(4096 * 2^b) as entry b + 2");
static_assert(kBNC <= (uint32_t)kCrcBlock, "one staging slot per thread");

__device__ __forceinline__ uint32_t bh_init_of(int kind, uint32_t key, uint32_t typed) {
  return kind == kInitArray ? key : kind == kInitTyped ? typed : 0u;
}

// ---- LDS fill: tables from the device copy, then the computed ones -------------
// Split in two: the loads (bh_fill_load, registers) and the stores + the
// computed tables (bh_fill_store), so a caller can issue the loads with its
// own first memory round trip (k_crc_ragged: the byte-share search).
struct BhFill {
  uint32_t st[4];
  uint4 l[3];
  uint4 rg, pw, us;
};
constexpr int kBhFillLow = (int)(kLdsGap + 512) / 16;  // lane_final + gap: 2080 slots
__device__ __forceinline__ void bh_fill_load(BhFill& f, const CrcTables* __restrict__ g) {
  const uint32_t t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t i = t + kCrcBlock * k;
    f.st[k] = g->step[(i >> 2) & 3][i >> 4];
  }
  const uint4* lo = reinterpret_cast<const uint4*>(&g->lane_final[0][0][0]);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const int i = (int)t + kCrcBlock * k;
    f.l[k] = lo[i < kBhFillLow ? i : 0];
  }
  // row gaps (96 slots), pow maps (b + 2 of pow1k: 672 slots), un-shift k < 16 (512)
  f.rg = reinterpret_cast<const uint4*>(&g->gap_row[0][0][0])[t < 96 ? t : 0];
  f.pw = reinterpret_cast<const uint4*>(&g->pow1k[2][0][0])[t < kBPowBits * 32 ? t : 0];
  f.us = reinterpret_cast<const uint4*>(&g->unshift[0][0][0])[t < 512 ? t : 0];
}
template <class Op>
__device__ __forceinline__ void bh_fill_store(const Op& op, const BhFill& f) {
  const uint32_t t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint32_t x = f.st[k];
    *reinterpret_cast<__attribute__((address_space(3))) span_u32x4*>(
        static_cast<size_t>(kLdsStep + 16 * (t + kCrcBlock * k))) = span_u32x4{x, x, x, x};
  }
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const int i = (int)t + kCrcBlock * k;
    if (i < kBhFillLow)
      *reinterpret_cast<__attribute__((address_space(3))) span_u32x4*>(static_cast<size_t>(16 * i)) =
          span_u32x4{f.l[k].x, f.l[k].y, f.l[k].z, f.l[k].w};
  }
  typedef __attribute__((address_space(3))) span_u32x4 lds_u32x4_t;
  if (t < 96) *reinterpret_cast<lds_u32x4_t*>(static_cast<size_t>(kBLdsRowGap + 16 * t)) = span_u32x4{f.rg.x, f.rg.y, f.rg.z, f.rg.w};
  if (t < kBPowBits * 32)
    *reinterpret_cast<lds_u32x4_t*>(static_cast<size_t>(kBLdsPow + 16 * t)) = span_u32x4{f.pw.x, f.pw.y, f.pw.z, f.pw.w};
  if (t < 512) *reinterpret_cast<lds_u32x4_t*>(static_cast<size_t>(kBLdsUnshift + 16 * t)) = span_u32x4{f.us.x, f.us.y, f.us.z, f.us.w};
  if (t < 128) {  // byte masks of a 16-byte piece
    const int h = (int)(t >> 2) & 15, k = (int)(t & 3);
    if (t < 64) {  // keep bytes >= h
      const int d = h - 4 * k;
      *lds_p32(kBLdsMaskHead + 4 * (t & 63)) = d <= 0 ? 0xFFFFFFFFu : d >= 4 ? 0u : 0xFFFFFFFFu << (8 * d);
    } else {  // keep the first 16 - h bytes
      const int keep = 16 - h - 4 * k;
      *lds_p32(kBLdsMaskTail + 4 * (t & 63)) = keep >= 4 ? 0xFFFFFFFFu : keep <= 0 ? 0u : 0xFFFFFFFFu >> (8 * (4 - keep));
    }
  }
  __syncthreads();
  // init injection: inj[ty][k] = unshift(~init_ty, k) (ty = 0 serves init 0)
  if (t < 256) {
    const uint32_t init = Op::kTypedInit ? op.typed_init(t >> 4) : 0u;
    *lds_p32(kBLdsInj + 4 * t) = crc_nibmap(kBLdsUnshift + (t & 15) * 512, ~init);
    if ((t & 15) == 0) *lds_p32(kBLdsInit + 4 * (t >> 4)) = init;
  }
}

// ---- window staging -----------------------------------------------------------
__device__ __forceinline__ uint4 bh_desc(uint32_t t) {
  const span_u32x4 v = *reinterpret_cast<__attribute__((address_space(3))) const span_u32x4*>(
      static_cast<size_t>(kBLdsDesc + 16 * t));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint32_t bh_bpre(uint32_t t) { return *lds_p32(kBLdsBpre + 4 * t); }

// Geometry of a span from its descriptor.
struct BhGeo {
  uint64_t ptr, a1;
  uint32_t n, F, h, kt;
};
__device__ __forceinline__ BhGeo bh_geo(uint64_t base, const uint4& d) {
  BhGeo x;
  x.ptr = base + (((uint64_t)d.y << 32) | d.x);
  x.n = d.z;
  x.a1 = (x.ptr + x.n + 15) & ~15ull;
  const uint64_t cover = x.a1 - x.ptr;
  x.F = (uint32_t)(cover >> 12);
  x.h = (uint32_t)cover & 4095u;
  x.kt = (uint32_t)(x.a1 - (x.ptr + x.n));
  return x;
}

// Head rows: W lanes per head, 64 W-byte rounds, 64 / W heads per batch
// round.  A window takes one lane per head (64 heads a round) when 1.25x its
// mean head fits 64 bytes -- blob records' 16-31-byte heads -- and 4-lane
// rows (256-byte rounds, 16 heads) otherwise -- SST blocks' 0-272-byte
// heads.  The head list puts the heads that fit one round before the
// longer ones, so a batch of short heads is one round.  (8- and 16-lane
// variants as well made the kernel spill: each width is a copy of the head
// loop.)
__device__ __forceinline__ uint32_t bh_head_w(uint32_t hbytes, uint32_t nheads) {
  return 5ull * hbytes <= 256ull * nheads ? 1u : 4u;  // 1.25 x mean <= 64  <=>  5 sum <= 256 n
}

// Stage window slots [0, wn) = spans sh.idx(t): descriptors, accumulators
// {0, parts}, the head list (heads of one W-row round first) and the
// pieces' exclusive prefix (padded for the ballot search); empty spans
// finish here (Extend(init, "") = init).  Ends with a barrier; the totals
// and W are at kBLdsCtl + 4 / + 8 / + 12.
template <class Op>
__device__ __forceinline__ void crc_bh_stage(const Op& op, const UShare& sh, uint32_t wn, uint64_t base, int kind) {
  const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6, nw = blockDim.x >> 6;
  uint32_t hh = 0, P = 0, hc = 0;
  if (t < wn) {
    const uint32_t i = sh.idx(t);
    const uint64_t off = op.off(i);
    const uint32_t len = (uint32_t)op.len(i);
    const uint32_t key = op.init_key(i);
    const uint4 d = make_uint4((uint32_t)off, (uint32_t)(off >> 32), len, key);
    *reinterpret_cast<__attribute__((address_space(3))) span_u32x4*>(static_cast<size_t>(kBLdsDesc + 16 * t)) =
        span_u32x4{d.x, d.y, d.z, d.w};
    const BhGeo x = bh_geo(base, d);
    if (len == 0) {
      const uint32_t init = bh_init_of(kind, key, *lds_p32(kBLdsInit + 4 * (key & 15u)));
      op.finish(i, init, op.pre(i, x.ptr, 0), true);
    } else {
      hh = (x.F == 0 || x.h != 0) ? 1u : 0u;
      hc = x.F ? x.h : (uint32_t)(x.a1 - x.ptr);  // the head's cover (when hh)
      P = (x.F + kBhPieceRounds - 1) / kBhPieceRounds;
    }
    *lds_p64(kBLdsAcc + 8 * t) = (uint64_t)(P + hh) << 32;
  }
  // the window's head bytes and heads -> W
  uint64_t hs = hh ? ((uint64_t)hc << 16) | 1u : 0ull;  // heads < 2^16, bytes < 2^40
#pragma unroll
  for (int dd = 32; dd >= 1; dd >>= 1)
    hs += ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(hs >> 32), dd, 64) << 32) |
          (uint32_t)__shfl_xor((int)(uint32_t)hs, dd, 64);
  if (lane == 0) *lds_p64(kBLdsWsum2 + 8 * w) = hs;
  __syncthreads();
  uint64_t htot = 0;
  for (uint32_t q = 0; q < nw; q++) htot += *lds_p64(kBLdsWsum2 + 8 * q);
  const uint32_t W = bh_head_w((uint32_t)(htot >> 16), (uint32_t)(htot & 0xFFFFu));
  const uint32_t one = hh && hc <= 64u * W ? 1u : 0u;  // the head fits one round
  // exclusive scans of (pieces, long heads, one-round heads), packed:
  // heads < 2^16 per window, pieces < 2^32
  const uint64_t v = ((uint64_t)P << 32) | ((uint64_t)(hh - one) << 16) | one;
  uint64_t x = v;
#pragma unroll
  for (int dd = 1; dd < 64; dd <<= 1) {
    const uint64_t y = ((uint64_t)(uint32_t)__shfl_up((int)(uint32_t)(x >> 32), dd, 64) << 32) |
                       (uint32_t)__shfl_up((int)(uint32_t)x, dd, 64);
    x += lane >= (uint32_t)dd ? y : 0ull;
  }
  if (lane == 63) *lds_p64(kBLdsWsum + 8 * w) = x;
  __syncthreads();
  uint64_t below = 0, tot = 0;
  for (uint32_t q = 0; q < nw; q++) {
    const uint64_t ws = *lds_p64(kBLdsWsum + 8 * q);
    below += q < w ? ws : 0ull;
    tot += ws;
  }
  const uint64_t ex = below + x - v;
  const uint32_t n1 = (uint32_t)(tot & 0xFFFFu), nl = (uint32_t)((tot >> 16) & 0xFFFFu);
  if (t < wn) {
    *lds_p32(kBLdsBpre + 4 * t) = (uint32_t)(ex >> 32);
    if (hh) *lds_p32(kBLdsHlist + 4 * (one ? (uint32_t)(ex & 0xFFFFu) : n1 + (uint32_t)((ex >> 16) & 0xFFFFu))) = t;
  }
  const uint32_t nheads = n1 + nl, npieces = (uint32_t)(tot >> 32);
  if (t <= 64) *lds_p32(kBLdsBpre + 4 * (wn + t)) = t ? 0xFFFFFFFFu : npieces;
  if (t == 0) {
    *lds_p32(kBLdsCtl) = 0;  // ticket
    *lds_p32(kBLdsCtl + 4) = nheads;
    *lds_p32(kBLdsCtl + 8) = npieces;
    *lds_p32(kBLdsCtl + 12) = W;
  }
  __syncthreads();
}

// ---- units of work --------------------------------------------------------------
// Tickets [0, HB) are head batches, the rest body pieces.  A wave runs two
// loops, each with one unit loaded ahead of the one it folds: its head
// batches, then -- from the first body ticket it draws, whose loads the head
// loop's last iteration already issued -- its body pieces.  (One loop over
// both kinds kept both kinds' state and branches live in every iteration:
// ~60 more VALU and ~200 SALU per unit, SQ counters profiles/r4/prof1.)

// A head batch round: head (64 / W) k + row of the list on W-lane row
// `lane / W` (row values).
struct BhHeadU {
  uint64_t hptr;    // the span's first byte
  uint32_t ht;      // window slot
  uint32_t hlive;   // the row has a head in this batch
  uint32_t hn;      // the SPAN's bytes
  uint32_t hinj;    // ~init, un-shifted by (hptr & 15): injected at the piece holding hptr
  int32_t hrounds;  // 64 W-byte rounds of the head
  int32_t q, R;     // the batch's round / rounds (wave-uniform)
};
// A body piece: rounds rhi down to rlo of span slot bt (wave-uniform).
struct BhBodyU {
  uint64_t ba1;     // the span's 16-aligned end
  uint32_t bt;
  int32_t r, rlo, rhi;
  uint32_t bkt;
  uint32_t binj;    // ~init at lane 0 of round rhi (h = 0, the span's first piece), else 0
  uint32_t bparts;  // the span's parts (1: finish at once)
  uint32_t live;    // 0: no piece left
};

// A head's geometry: [ptr, a1 - kt) with a1 16-aligned -- the whole span
// (F = 0) or the h bytes before its body -- in 64 W-byte rounds anchored at
// a1; `owner` = the row lane whose first-round chunk holds ptr, hb = ptr -
// that chunk's start.
struct BhHead {
  uint64_t a0, a1;
  uint32_t F, kt, cover;
  int32_t owner;
  uint32_t hb;
};
template <int W>
__device__ __forceinline__ BhHead bh_hgeo(uint64_t ptr, uint32_t n, int32_t rounds) {
  BhHead x;
  x.a0 = ptr & ~15ull;
  const uint64_t a1 = (ptr + n + 15) & ~15ull;
  x.F = (uint32_t)((a1 - ptr) >> 12);
  x.a1 = a1 - ((uint64_t)x.F << 12);
  x.kt = x.F ? 0u : (uint32_t)(a1 - (ptr + n));
  x.cover = (uint32_t)(x.a1 - ptr);
  const uint32_t lead = 64u * W * (uint32_t)rounds - x.cover;
  x.owner = (int32_t)(lead >> 6);
  x.hb = lead & 63u;
  return x;
}

// Head batch k (< HB): head (64 / W) k + row of the list on W-lane row
// `lane / W`.
template <int W>
__device__ __forceinline__ BhHeadU bh_head_of(uint32_t k, uint64_t base, int kind, uint32_t nheads, uint32_t lane) {
  BhHeadU u;
  constexpr uint32_t NB = 64 / W;
  const uint32_t e = NB * k + lane / W;
  u.hlive = e < nheads ? 1u : 0u;
  u.ht = *lds_p32(kBLdsHlist + 4 * (u.hlive ? e : NB * k));
  const uint4 d = bh_desc(u.ht);
  const BhGeo x = bh_geo(base, d);
  u.hptr = x.ptr;
  u.hn = x.n;
  // the head: the whole span (F = 0) or the h bytes before the body
  const uint32_t cover = x.F ? x.h : (uint32_t)(x.a1 - x.ptr);  // > 0
  u.hrounds = (int32_t)((cover + 64 * W - 1) / (64 * W));
  const uint32_t hk = (uint32_t)x.ptr & 15u;  // = the owner's hb % 16 (chunks are 16-aligned)
  u.hinj = kind == kInitArray ? crc_nibmap(kBLdsUnshift + hk * 512, ~d.w)
                              : *lds_p32(kBLdsInj + 4 * ((kind == kInitTyped ? (d.w & 15u) * 16 : 0u) + hk));
  uint32_t R = u.hlive ? (uint32_t)u.hrounds : 0u;  // the batch's rounds: the wave max
#pragma unroll
  for (int dd = 32; dd >= 1; dd >>= 1) R = max(R, (uint32_t)__shfl_xor((int)R, dd, 64));
  u.R = (int32_t)rfl(R);
  u.q = 0;
  return u;
}

// Body piece q (q >= npieces: none); tc = the wave's search cursor (pieces
// are drawn in increasing order, so the search only moves forward).
__device__ __forceinline__ BhBodyU bh_body_of(uint32_t q, uint32_t npieces, uint64_t base, int kind, uint32_t& tc,
                                              uint32_t lane) {
  BhBodyU u;
  u.live = q < npieces ? 1u : 0u;
  u.bt = 0;
  u.r = u.rlo = u.rhi = 0;
  u.ba1 = 0;
  u.bkt = 0;
  u.binj = 0;
  u.bparts = 1;
  if (!u.live) return u;
  uint32_t v = bh_bpre(tc + 1 + lane);
  uint32_t c0 = (uint32_t)__popcll(__ballot(v <= q));
  while (c0 == 64) {
    tc += 64;
    v = bh_bpre(tc + 1 + lane);
    c0 = (uint32_t)__popcll(__ballot(v <= q));
  }
  tc += c0;
  u.bt = tc;
  const uint4 d = bh_desc(tc);
  const uint4 ds = make_uint4(rfl(d.x), rfl(d.y), rfl(d.z), rfl(d.w));
  const BhGeo x = bh_geo(base, ds);
  const uint32_t P = (x.F + kBhPieceRounds - 1) / kBhPieceRounds;
  const uint32_t j = P - 1 - (q - rfl(bh_bpre(tc)));  // pieces in address order
  u.rlo = (int32_t)(kBhPieceRounds * j);
  u.rhi = (int32_t)min(kBhPieceRounds * j + kBhPieceRounds - 1, x.F - 1);
  u.r = u.rhi;
  u.ba1 = x.a1;
  u.bkt = x.kt;
  const bool first = j == P - 1 && x.h == 0;  // the span starts at this piece's first round
  u.binj = first ? ~bh_init_of(kind, ds.w, *lds_p32(kBLdsInit + 4 * (ds.w & 15u))) : 0u;
  u.bparts = P + (x.h != 0 ? 1u : 0u);
  return u;
}

// Round r of a body piece: the row-transposed layout (crc_load_chunk_rt),
// non-temporal; no piece left: the zero piece.
__device__ __forceinline__ Chunk bh_load_body(const BhBodyU& u, uint32_t lane, uint64_t zp) {
  Chunk ch;
  const uint64_t b = u.ba1 - (uint64_t)kRoundBytes * (uint32_t)(u.r + 1) + 64ull * (lane & 15) + 16ull * (lane >> 4);
#pragma unroll
  for (int j = 0; j < 4; j++) ch.v[j] = span_load16<true>(u.live ? b + 1024ull * j : zp);
  return ch;
}
// Round q of a head batch: lane c of a row the 64-byte chunk c of its
// round (the pieces wholly before the head and idle rows read the zero
// piece).
template <int W>
__device__ __forceinline__ Chunk bh_load_head(const BhHeadU& u, uint32_t lane, uint64_t zp) {
  Chunk ch;
  const uint32_t c = lane & (W - 1);
  const BhHead x = bh_hgeo<W>(u.hptr, u.hn, u.hrounds);
  const int32_t rr = u.hrounds - 1 - u.q;
  const bool act = u.hlive && rr >= 0;
  const uint64_t b = x.a1 - 64ull * W * (uint32_t)(rr + 1) + 64ull * c;
  const int32_t rel = rr == u.hrounds - 1 ? (int32_t)((uint32_t)b - (uint32_t)x.a0) : 0;
#pragma unroll
  for (int j = 0; j < 4; j++) ch.v[j] = span_load16<false>((!act || rel < -16 * j) ? zp : b + 16ull * j);
  return ch;
}

// Epilogue inputs of a span: every part loads its span's own (Op::pre
// depends on the span only), so whichever part finishes it has them.
// Vector loads: a body's arguments are wave-uniform, and uniform loads
// compile to scalar ones, which drop the low address bits.
template <class Op>
__device__ __forceinline__ typename Op::Pre bh_pre_body(const Op& op, const BhBodyU& u, const UShare& sh,
                                                        uint64_t base) {
  const uint4 d = bh_desc(u.bt);
  uint64_t ptr = base + (((uint64_t)d.y << 32) | d.x);
  uint32_t i = sh.idx(u.bt);
  asm volatile("" : "+v"(i), "+v"(ptr));
  return op.pre(i, ptr, d.z);
}
template <class Op>
__device__ __forceinline__ typename Op::Pre bh_pre_head(const Op& op, const BhHeadU& u, const UShare& sh) {
  return op.pre(sh.idx(u.ht), u.hptr, u.hn);
}

__device__ __forceinline__ uint32_t bh_unshift(uint32_t k, uint32_t s) { return crc_nibmap(kBLdsUnshift + k * 512, s); }

// zshift(p, 4096 m), one nibble map per set bit of m (m wave-uniform).
__device__ __forceinline__ uint32_t bh_pow_u(uint32_t p, uint32_t m) {
  for (; m; m &= m - 1) p = crc_nibmap(kBLdsPow + (uint32_t)__builtin_ctz(m) * 512, p);
  return p;
}
// The same with m per lane.
__device__ __forceinline__ uint32_t bh_pow_v(uint32_t p, uint32_t m) {
  while (wave_any(m != 0)) {
    const uint32_t b = (uint32_t)__builtin_ctz(m | 0x80000000u) & 31u;
    const uint32_t x = crc_nibmap(kBLdsPow + (b < kBPowBits ? b : 0u) * 512, p);
    p = m ? x : p;
    m &= m - 1;
  }
  return p;
}

// A body piece ends: p = its pure state at the piece end (wave-uniform).
template <class Op>
__device__ __forceinline__ void bh_body_end(const Op& op, const BhBodyU& u, uint32_t p, const typename Op::Pre& pre,
                                            const UShare& sh, uint32_t lane) {
  p = bh_pow_u(p, (uint32_t)u.rlo);  // the piece end is 4096 rlo bytes before a1
  if (u.bparts != 1) {
    uint32_t left = 0;
    if (lane == 0) {
      __hip_atomic_fetch_xor(lds_p32(kBLdsAcc + 8 * u.bt), p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      left = __hip_atomic_fetch_add(lds_p32(kBLdsAcc + 8 * u.bt + 4), 0xFFFFFFFFu, __ATOMIC_ACQ_REL,
                                    __HIP_MEMORY_SCOPE_WORKGROUP);
      if (left == 1) p = __hip_atomic_load(lds_p32(kBLdsAcc + 8 * u.bt), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (rfl(left) != 1) return;
    p = rfl(p);
  }
  if (u.bkt) p = bh_unshift(u.bkt, p);
  op.finish(sh.idx(u.bt), ~p, pre, lane == 0);
}

// Head rows end (fin: the row's head ends in this round): p = the pure state
// at the head end, in every lane of the row.
template <int W, class Op>
__device__ __forceinline__ void bh_head_end(const Op& op, const BhHeadU& u, uint32_t p, bool fin, const UShare& sh,
                                            uint32_t lane) {
  const bool lead = (lane & (W - 1)) == 0;
  const uint32_t F = (uint32_t)((((u.hptr + u.hn + 15) & ~15ull) - u.hptr) >> 12);
  const bool direct = F == 0;  // the head is the whole span
  bool done = fin && direct;
  if (wave_any(fin && !direct)) {
    const bool part = fin && !direct;
    const uint32_t q = bh_pow_v(p, part ? F : 0u);  // the head end is 4096 F bytes before a1
    p = part ? q : p;
    uint32_t left = 0;
    if (part && lead) {
      __hip_atomic_fetch_xor(lds_p32(kBLdsAcc + 8 * u.ht), p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      left = __hip_atomic_fetch_add(lds_p32(kBLdsAcc + 8 * u.ht + 4), 0xFFFFFFFFu, __ATOMIC_ACQ_REL,
                                    __HIP_MEMORY_SCOPE_WORKGROUP);
      if (left == 1) p = __hip_atomic_load(lds_p32(kBLdsAcc + 8 * u.ht), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if constexpr (W > 1) {  // the row leader's values to its row
      const int src = (int)((lane & ~(uint32_t)(W - 1)) << 2);
      left = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)left);
      const uint32_t pl = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)p);
      p = part ? pl : p;
    }
    done = done || (part && left == 1);
  }
  if (!wave_any(done)) return;
  const uint32_t kt = (uint32_t)(0u - (uint32_t)(u.hptr + u.hn)) & 15u;
  const uint32_t x = bh_unshift(kt, p);
  p = kt ? x : p;
  // the epilogue inputs only now: heads run before the bodies, so a head
  // finishes its span mostly when it IS the span (no prefetch registers
  // through the head loop)
  op.finish(sh.idx(u.ht), ~p, bh_pre_head(op, u, sh), done && lead);
}

// One 64 W-byte round of the head batch (row values; q wave-uniform).
template <int W>
__device__ __forceinline__ uint32_t bh_head_round(uint32_t s, Chunk ch, const BhHeadU& u, uint32_t c, const CrcLane& L) {
  const BhHead hg = bh_hgeo<W>(u.hptr, u.hn, u.hrounds);
  const int32_t rr = u.hrounds - 1 - u.q;
  const bool first = u.q == 0;  // every live row starts its head in the batch's first round
  const bool own = (int32_t)c == hg.owner;
  const uint32_t h0 = (uint32_t)u.hptr & 15u;
  const uint4 mh = lds_u32x4(kBLdsMaskHead + 16 * h0);
  const uint4 mt = lds_u32x4(kBLdsMaskTail + 16 * ((rr == 0 && c == W - 1) ? hg.kt : 0u));
  const uint32_t pa = (first && own) ? hg.hb >> 4 : 4u;
  uint32_t sels[4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const uint32_t sel = (uint32_t)j == pa ? ~0u : 0u;
    sels[j] = sel;
    ch.v[j].x = __builtin_amdgcn_bitop3_b32(ch.v[j].x, mh.x, sel, 0xD0);
    ch.v[j].y = __builtin_amdgcn_bitop3_b32(ch.v[j].y, mh.y, sel, 0xD0);
    ch.v[j].z = __builtin_amdgcn_bitop3_b32(ch.v[j].z, mh.z, sel, 0xD0);
    ch.v[j].w = __builtin_amdgcn_bitop3_b32(ch.v[j].w, mh.w, sel, 0xD0);
  }
  and4(ch.v[3], mt);
  // a lane's next chunk is 64 W bytes on: zshift(., 64 (W - 1)) after its
  // own 64 (W = 1: adjacent, the state carries over)
  uint32_t gap = s;
  if constexpr (W > 1) gap = crc_nibmap(kBLdsRowGap + 512u * (W == 4 ? 0u : W == 8 ? 1u : 2u), s);
  gap = first ? 0u : gap;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&ch.v[0]);
  const uint32_t inj = u.hinj;
  uint32_t x = gap ^ w[0] ^ (sels[0] & inj);
#pragma unroll
  for (int k = 0; k < 16; k++) {
    uint32_t nw = 0u;
    if (k + 1 < 16) nw = ((k + 1) & 3) ? w[k + 1] : (w[k + 1] ^ (sels[(k + 1) >> 2] & inj));
    x = crc_step4x(x, L, nw);
  }
  return x;
}

// One 4 KiB round of a body piece (chunk already row-transposed).
__device__ __forceinline__ uint32_t bh_body_round(uint32_t s, Chunk ch, const BhBodyU& u, uint32_t lane,
                                                  const CrcLane& L) {
  const bool first = u.r == u.rhi;
  uint32_t x = first ? (lane == 0 ? u.binj : 0u) : crc_nibmap(kLdsGap, s);
  if (u.r == 0 && u.bkt && lane == 63) crc_keep_head_bytes(ch.v[3], 16 - u.bkt);  // bytes past the end
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&ch.v[0]);
  x ^= w[0];
#pragma unroll
  for (int k = 0; k < 16; k++) x = crc_step4x(x, L, k < 15 ? w[k + 1] : 0u);
  return x;
}

// ---- the body loop ----------------------------------------------------------------
template <class Op>
struct BhCtx {
  const Op& op;
  const UShare& sh;
  uint64_t base, zp;
  uint32_t HB, npieces;
  int kind;
  uint32_t lane;
  const CrcLane& L;
};
// The unit after b: its next round, or the next piece drawn (none after none).
template <class Op>
__device__ __forceinline__ BhBodyU bh_next_body(const BhCtx<Op>& x, uint32_t& tc, const BhBodyU& b) {
  BhBodyU n = b;
  if (!b.live) return n;  // wave-uniform
  if (b.r > b.rlo) {
    n.r = b.r - 1;
    return n;
  }
  const uint32_t k = rfl(lds_ticket(lds_p32(kBLdsCtl)));
  return bh_body_of(k - x.HB, x.npieces, x.base, x.kind, tc, x.lane);
}
// n's epilogue inputs: b's when n is b's next round
template <class Op>
__device__ __forceinline__ typename Op::Pre bh_pre_next(const BhCtx<Op>& x, const BhBodyU& b, const BhBodyU& n,
                                                        const typename Op::Pre& pb) {
  if (b.live && b.r > b.rlo) return pb;  // wave-uniform
  return bh_pre_body(x.op, n, x.sh, x.base);
}
// Fold round A (loaded); issue B = next(A).  Returns B.live.
template <class Op, bool T>
__device__ __forceinline__ bool bh_body_step(const BhCtx<Op>& x, uint32_t& tc, const BhBodyU& bA, BhBodyU& bB,
                                             const Chunk& cA, Chunk& cB, const typename Op::Pre& pA,
                                             typename Op::Pre& pB, uint32_t& s) {
  bB = bh_next_body(x, tc, bA);
  cB = bh_load_body(bB, x.lane, x.zp);
  pB = bh_pre_next(x, bA, bB, pA);
  Chunk cur = cA;
  if (T) row_transpose(cur);
  s = bh_body_round(s, cur, bA, x.lane, x.L);
  if (bA.r == bA.rlo) bh_body_end(x.op, bA, wave_xor32(crc_lane_final(s, x.L)), pA, x.sh, x.lane);
  return bB.live != 0;
}
// The wave's head batches, from its first ticket k (< HB); returns the first
// ticket past them.
template <int W, class Op>
__device__ __forceinline__ uint32_t crc_bh_heads(const Op& op, const UShare& sh, uint64_t base, uint64_t zp, uint32_t k,
                                                 uint32_t HB, uint32_t nheads, const CrcLane& L) {
  const int kind = op.init_kind();
  const uint32_t lane = threadIdx.x & 63, c = lane & (W - 1);
  const uint32_t lf4 = (64u - W + c) << 2;  // lane-final column 64 - W + c: zshift(., 64 (W - 1 - c))
  BhHeadU u = bh_head_of<W>(k, base, kind, nheads, lane);
  Chunk cur = bh_load_head<W>(u, lane, zp);
  uint32_t hs = 0;  // the rows' states (a head's state carries over its rounds)
  for (;;) {
    BhHeadU nu = u;
    bool nh = true;
    if (u.q + 1 < u.R) {
      nu.q = u.q + 1;
    } else {
      k = rfl(lds_ticket(lds_p32(kBLdsCtl)));
      nh = k < HB;
      if (nh) nu = bh_head_of<W>(k, base, kind, nheads, lane);
      nu.hlive = nh ? nu.hlive : 0u;  // the last iteration loads the zero piece
    }
    const Chunk nxt = bh_load_head<W>(nu, lane, zp);
    hs = bh_head_round<W>(hs, cur, u, c, L);
    const bool fin = u.hlive && u.hrounds - 1 - u.q == 0;
    if (wave_any(fin)) {
      uint32_t p = hs;  // W = 1: the lane's state is its head's
      if constexpr (W > 1) p = row_xor32<W>(crc_lane_final4(hs, lf4));
      bh_head_end<W>(op, u, p, fin, sh, lane);
    }
    if (!nh) return k;
    u = nu;
    cur = nxt;
  }
}

template <class Op, bool T>
__device__ __forceinline__ void crc_bh_window(const Op& op, const UShare& sh, uint64_t base, const CrcTables* __restrict__ g) {
  const int kind = op.init_kind();
  const CrcLane L = crc_lane();
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t zp = reinterpret_cast<uint64_t>(&g->zero16[0]);
  const uint32_t nheads = *lds_p32(kBLdsCtl + 4), npieces = *lds_p32(kBLdsCtl + 8), W = *lds_p32(kBLdsCtl + 12);
  const uint32_t HB = (nheads + 64 / W - 1) / (64 / W);
  typedef typename Op::Pre Pre;
  uint32_t tc = 0;
  uint32_t k = rfl(lds_ticket(lds_p32(kBLdsCtl)));
  if (k < HB) {  // head batches (W wave-uniform)
    if (W == 1)
      k = crc_bh_heads<1>(op, sh, base, zp, k, HB, nheads, L);
    else
      k = crc_bh_heads<4>(op, sh, base, zp, k, HB, nheads, L);
  }
  // ---- body pieces ----
  // (ticket k >= HB: the wave's first body piece; its loads were not issued
  // ahead -- one round trip per wave and window)
  const BhCtx<Op> x{op, sh, base, zp, HB, npieces, kind, lane, L};
  BhBodyU b0 = bh_body_of(k - HB, npieces, base, kind, tc, lane);
  if (!b0.live) return;
  Chunk c0 = bh_load_body(b0, lane, zp);
  Pre p0 = bh_pre_body(op, b0, sh, base);
  uint32_t s = 0;
  // the loop unrolled twice: the loaded round and the one in flight swap
  // register names instead of 16 v_mov per round (ragged 4096-B spans 0.775
  // -> 0.828, 4100-4400 B 0.679 -> 0.715, same box; two rounds in flight per
  // wave, unrolled three times, measured the same: 0.828 / 0.719)
  BhBodyU b1;
  Chunk c1;
  Pre p1;
  for (;;) {
    if (!bh_body_step<Op, T>(x, tc, b0, b1, c0, c1, p0, p1, s)) break;
    if (!bh_body_step<Op, T>(x, tc, b1, b0, c1, c0, p1, p0, s)) break;
  }
}

// A workgroup's share [start, start + n) (contiguous), in windows of at most
// kBNC spans, as even as the share allows.
template <class Op, bool T>
__device__ __forceinline__ void crc_bh_driver(const Op& op, const RowShare& share, const CrcTables* __restrict__ g,
                                              bool filled = false) {
  if (!filled) {  // (k_crc_ragged fills the image itself when it searched byte shares)
    BhFill f;
    bh_fill_load(f, g);
    bh_fill_store(op, f);
  }
  const uint64_t base = reinterpret_cast<uint64_t>(op.base());
  const int kind = op.init_kind();
  const uint32_t n = share.n;
  const uint32_t nwin = (n + kBNC - 1) / kBNC;
  __syncthreads();  // the init tables (read by the staging of empty spans)
  for (uint32_t wi = 0; wi < nwin; wi++) {
    const uint32_t w0 = (uint32_t)((uint64_t)n * wi / nwin), w1 = (uint32_t)((uint64_t)n * (wi + 1) / nwin);
    const UShare sh{share.start + share.stride * w0, share.stride};
    if (wi) __syncthreads();  // the previous window's waves are done with its slots
    crc_bh_stage(op, sh, w1 - w0, base, kind);
    crc_bh_window<Op, T>(op, sh, base, g);
  }
}

}  // namespace mck
