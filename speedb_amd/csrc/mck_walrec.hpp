// mck_walrec.hpp -- WAL recovery in one device pass (round 6): every physical
// record's CRC32C (ReadPhysicalRecord, db/log_reader.cc:512-525) and, from
// the SAME registers, the XXH3_64bits record_checksum of every
// single-fragment record (ReadRecord's kFullType case, :95-116: the logical
// record IS the fragment, :107-110).
//
// Input: the host plan of the log (mck_wal_recover's walk, mck_walk.h): one
// 16-byte descriptor per physical record -- payload offset, type, length,
// the header's stored CRC.  The header walk is the host's (it reads the
// headers anyway to hand the records out), so the device only hashes.
//
// Layout: the CRC row driver's (16-lane rows, one record per row, records
// taken from an LDS ticket), but with the round grid anchored at the
// payload START (a0 = payload & ~3): row round k covers [a0 + 1024 k, +1024),
// lane c the 64-byte chunk a0 + 1024 k + 64 c.  That grid is XXH3's: round k
// is segment k (1 KiB = 16 stripes of 64 B, util/xxhash.h:5141-5171) and
// lane c's chunk holds stripe c shifted by b = payload & 3 bytes, so the
// stripe is the chunk funnel-shifted with one more dword (the next chunk's
// first, loaded beside the chunk).  Per round a lane folds its chunk into the
// CRC (the 4-byte table step) and its stripe into XXH3's 8 accumulator
// terms; a reduce-scatter over the row leaves accumulator a's segment sum in
// lanes a and a + 8, which keep accumulator a and scramble it after every
// full segment.  One read of the log, no second pass, no record copies.
//
// The CRC covers [type][log number if recyclable][payload] as
// EmitPhysicalRecord does (db/log_writer.cc:281-298): the type (and log
// number) bytes are the row's init state (type_crc, as the writer's), the
// payload is the span.  With the start-anchored grid the last round ends
// past the record: lanes past its last byte keep their previous state and
// shift it by one more row round, and the sum is un-shifted by the < 64
// bytes after the end (the lane-final tables shift by any 64 j, j < 64).
#pragma once
#include "mck_kernels.hpp"

namespace mck {

// == mck_wal_rec_desc (mck.h)
struct WalRecDesc {
  uint32_t off_lo;  // payload offset in the image, bits 0-31
  uint32_t hi;      // bits 0-15: payload offset bits 32-47; 16-23: record type; 24: hash the record
  uint32_t len;     // payload bytes
  uint32_t stored;  // the header's masked CRC (LE32)
};
static_assert(sizeof(WalRecDesc) == 16, "descriptor");

// LDS: the row drivers' image (crc_fill_rows: wave image + row gap maps),
// then this kernel's init tables (every type byte 0-255: a corrupt record's
// type byte is CRC'd as it is, "unknown record type" comes after the CRC),
// descriptor cache, ticket and the XXH3 secret words.
constexpr uint32_t kLdsWrInj = kLdsRowInj;                   // [256][4] u32: unshift(~init_t, b)
constexpr uint32_t kLdsWrInit = kLdsWrInj + 4096;            // [256] u32: init_t
constexpr uint32_t kWrDescCache = 1300;
constexpr uint32_t kLdsWrDesc = kLdsWrInit + 1024;
constexpr uint32_t kLdsWrTicket = kLdsWrDesc + 16 * kWrDescCache;
constexpr uint32_t kLdsWrSecret = kLdsWrTicket + 64;  // 25 u64 words of XXH3_kSecret
static_assert(kLdsWrSecret + 8 * 25 <= kLdsStep, "below the step tables");

// The CRC init of a record of type t: type_crc[t] (+ the log number for the
// recyclable types, db/log_writer.cc:48-51, 281-289) for the 16 codes the
// host table holds, Value(&t, 1) beyond; and the same un-shifted by b < 4
// bytes (the lane-0 injection).  After crc_fill_rows' barrier.
__device__ __forceinline__ void wr_init_tables(const WalTypeCrcs& tc) {
  const uint32_t t = threadIdx.x >> 2, b = threadIdx.x & 3u;  // 1024 threads = 256 x 4
  const uint32_t init = t < 16 ? tc.v[t] : crc_extend_byte(0u, (uint8_t)t);
  *lds_p32(kLdsWrInj + 4 * threadIdx.x) = crc_unshift(b, ~init);
  if (b == 0) *lds_p32(kLdsWrInit + 4 * t) = init;
}

// A row's record and round (the derived geometry is recomputed where it is
// used: the row state stays at 7 VGPRs, three copies of it are live).
struct WrRow {
  uint64_t P;        // payload address
  uint32_t len;      // payload bytes
  uint32_t k;        // current round
  uint32_t i;        // record index
  uint32_t stored;   // the header's masked CRC
  uint32_t th;       // type | hash << 8 (hash 1: XXH3 by stripes, len > 240; 2: short XXH3; 0: none)
  __device__ uint64_t a0() const { return P & ~3ull; }  // the grid
  __device__ uint32_t b() const { return (uint32_t)P & 3u; }
  __device__ uint32_t type() const { return th & 0xFFu; }
  __device__ uint32_t hash() const { return th >> 8; }
  __device__ uint32_t R() const {  // rounds
    const uint32_t cover = len + b();
    return cover ? (cover + 1023) >> 10 : 1u;
  }
  // XXH3 long loop (util/xxhash.h:5141-5171; len > 240 here): full
  // segments, stripes of the partial one
  __device__ uint32_t nb() const { return (len - 1) >> 10; }
  __device__ uint32_t nst() const { return ((len - 1) & 1023u) >> 6; }
};
__device__ __forceinline__ WrRow wr_row(const uint4& d, uint32_t i, uint64_t base) {
  WrRow r;
  r.P = base + ((uint64_t)d.x | ((uint64_t)(d.y & 0xFFFFu) << 32));
  r.len = d.z;
  r.stored = d.w;
  const uint32_t h = (d.y >> 24) & 1u;
  r.th = ((d.y >> 16) & 0xFFu) | ((h ? (r.len > 240 ? 1u : 2u) : 0u) << 8);
  r.k = 0;
  r.i = i;
  return r;
}
__device__ __forceinline__ WrRow wr_sel(bool a, const WrRow& x, const WrRow& y) {
  WrRow r;
  r.P = a ? x.P : y.P;
  r.len = a ? x.len : y.len;
  r.k = a ? x.k : y.k;
  r.i = a ? x.i : y.i;
  r.stored = a ? x.stored : y.stored;
  r.th = a ? x.th : y.th;
  return r;
}

// A row round's loads: lane c's chunk, the dword after it (the stripe's
// last b bytes), and -- when the round is the record's XXH3 merge round
// (segment nb) -- lanes 0-7's 8-byte word of the last stripe (at len - 64,
// util/xxhash.h:5160-5165), as three dwords covering it.  Every piece past
// the record reads the zero piece instead (a piece at x < end ends at most
// 15 bytes past it: the image is readable 16 bytes past nbytes).
struct WrLoads {
  Chunk ch;
  uint32_t e;
  uint32_t l0, l1, l2;
};
__device__ __forceinline__ WrLoads wr_load(const WrRow& r, uint32_t c) {
  WrLoads L;
  // offsets from the grid base a0; a piece past the record reads the
  // record's last dword instead (clamped: one v_min per address, no 64-bit
  // compare-and-select), whose data the rounds mask out
  const uint64_t a0 = r.a0();
  const uint32_t cover = r.len + r.b();
  const uint32_t lim = cover ? (cover - 1) & ~3u : 0u;  // the last dword of the record (or its start)
  const uint32_t cb = 1024u * r.k + 64u * c;
#pragma unroll
  for (int j = 0; j < 4; j++) L.ch.v[j] = span_load16<false>(a0 + min(cb + 16u * j, lim));
  L.e = gload4(a0 + min(cb + 64u, lim));
  // the last stripe's word c (lanes 0-7), as the three dwords covering it;
  // other lanes and rounds read the round's first dword -- one address per
  // row, in the line lane 0's chunk load fetches (round 6: the record's
  // first dword, long evicted after round 0, cost a line per row round,
  // FETCH 1.109 x at 32 KiB records; each lane's own chunk instead put 16
  // lines per row on the texture addresser for each of the three loads:
  // 0.667 -> 0.470 of peak)
  const bool ls = r.hash() == 1u && r.k == r.nb() && c < 8;
  const uint32_t w4 = ls ? (cover - 64 + 8 * c) & ~3u : min(1024u * r.k, lim);
  L.l0 = gload4(a0 + w4);
  L.l1 = gload4(a0 + min(w4 + 4, lim));
  L.l2 = gload4(a0 + min(w4 + 8, lim));
  return L;
}

__device__ __forceinline__ uint32_t abyte(uint32_t hi, uint32_t lo, uint32_t s) {
  return __builtin_amdgcn_alignbyte(hi, lo, s);
}
template <int CTRL>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) {
  return ((uint64_t)dpp32<CTRL>((uint32_t)(v >> 32)) << 32) | dpp32<CTRL>((uint32_t)v);
}
constexpr int kDppHalfMirror = 0x141, kDppQuadXor1 = 0xB1, kDppQuadXor2 = 0x4E, kDppRowRor8 = 0x128,
              kDppRowRor4 = 0x124;
__device__ __forceinline__ uint64_t sel64(bool a, uint64_t x, uint64_t y) { return a ? x : y; }

// Sum of A[lane & 7] over the 16 lanes of each row (a reduce-scatter: A[0..7]
// are this lane's terms of the 8 accumulators).  Partners c ^ 7 (half
// mirror), c ^ 2, c ^ 1 split the accumulator index bit by bit, then the two
// halves add (c ^ 8).
__device__ __forceinline__ uint64_t wr_row_reduce(const uint64_t (&A)[8], uint32_t c) {
  const bool b2 = (c & 4u) != 0, b1 = (c & 2u) != 0, b0 = (c & 1u) != 0;
  uint64_t B[4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const uint64_t send = sel64(b2, A[j], A[4 + j]);
    const uint64_t keep = sel64(b2, A[4 + j], A[j]);
    B[j] = keep + dpp_u64<kDppHalfMirror>(send);
  }
  uint64_t C[2];
#pragma unroll
  for (int j = 0; j < 2; j++) {
    const uint64_t send = sel64(b1, B[j], B[2 + j]);
    const uint64_t keep = sel64(b1, B[2 + j], B[j]);
    C[j] = keep + dpp_u64<kDppQuadXor2>(send);
  }
  const uint64_t send = sel64(b0, C[0], C[1]);
  const uint64_t keep = sel64(b0, C[1], C[0]);
  uint64_t D = keep + dpp_u64<kDppQuadXor1>(send);
  return D + dpp_u64<kDppRowRor8>(D);
}

__device__ __forceinline__ uint64_t lds_sec(uint32_t w) { return *lds_p64(kLdsWrSecret + 8 * w); }

// Per-lane XXH3 constants: lane c keeps accumulator a = c & 7.  Only the
// scramble secret stays in registers; XXH3_INIT_ACC and the last-stripe /
// merge secrets (once per record) are read from LDS where they are used.
constexpr uint32_t kLdsWrInitAcc = kLdsWrSecret + 8 * 25;  // [8] u64 XXH3_INIT_ACC
static_assert(kLdsWrInitAcc + 64 <= kLdsStep, "below the step tables");
struct WrX3 {
  uint64_t ks;  // scramble secret (offset 128 + 8 a)
  __device__ uint64_t init(uint32_t c) const { return *lds_p64(kLdsWrInitAcc + 8 * (c & 7u)); }
};
__device__ __forceinline__ WrX3 wr_x3(uint32_t c) {
  WrX3 X;
  X.ks = sec64(128 + 8 * (int)(c & 7u));
  return X;
}
// 8 secret bytes at byte offset 8 w + B, 0 < B < 8 (the merge secrets at
// 11 + 8 a = 8 (1 + a) + 3, the last stripe's at 121 + 8 a = 8 (15 + a) + 1)
template <int B>
__device__ __forceinline__ uint64_t lds_sec_at(uint32_t w) {
  const uint64_t lo = *lds_p64(kLdsWrSecret + 8 * w), hi = *lds_p64(kLdsWrSecret + 8 * w + 8);
  return (lo >> (8 * B)) | (hi << (64 - 8 * B));
}

// One row round of XXH3: stripe c of segment k (lane c's chunk shifted by b,
// the extra dword e) into acc.  Returns the record's hash in lane 0 of the
// row at its merge round (valid where `merge`).
__device__ __forceinline__ uint64_t wr_x3_round(const WrRow& r, const WrLoads& L, uint32_t c, const WrX3& X,
                                                uint64_t& acc, bool act, bool& merge) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&L.ch.v[0]);
  const uint32_t nb = r.nb(), b = r.b();
  uint64_t W[8];
#pragma unroll
  for (int q = 0; q < 8; q++) {
    const uint32_t lo = abyte(w[2 * q + 1], w[2 * q], b);
    const uint32_t hi = abyte(2 * q + 2 < 16 ? w[2 * q + 2] : L.e, w[2 * q + 1], b);
    W[q] = ((uint64_t)hi << 32) | lo;
  }
  uint64_t A[8];
#pragma unroll
  for (int q = 0; q < 8; q++) {
    // v0.8.1: acc[q] += lo32(d ^ s) * hi32(d ^ s); acc[q ^ 1] += d
    A[q] = mul32to64(W[q] ^ lds_sec(c + q)) + W[q ^ 1];
  }
  // only the partial segment's stripes past nst drop out (a row that does
  // not hash this round reduces garbage into its own sum, unused)
  if (wave_any(act && r.k == nb)) {
    const bool valid = r.k < nb || c < r.nst();
#pragma unroll
    for (int q = 0; q < 8; q++) A[q] = valid ? A[q] : 0ull;
  }
  const uint64_t S = wr_row_reduce(A, c);
  acc += act ? S : 0ull;
  const bool full = act && r.k < nb;
  acc = full ? xxh3_scramble(acc, X.ks) : acc;
  merge = act && r.k == nb;
  uint64_t h = 0;
  if (wave_any(merge)) {
    // the last stripe (util/xxhash.h:5160-5165): lane a < 8 holds its word a
    const uint32_t s = (uint32_t)(r.P + r.len - 64 + 8 * (c & 7u)) & 3u;
    const uint64_t lw = ((uint64_t)abyte(L.l2, L.l1, s) << 32) | abyte(L.l1, L.l0, s);
    const uint64_t lx = dpp_u64<kDppQuadXor1>(lw);  // word a ^ 1
    const uint64_t tl = mul32to64(lw ^ lds_sec_at<1>(15 + (c & 7u))) + lx;  // offset 121 + 8 a
    // lanes 0-7 hold accumulator a = c; lanes 8-15 the same sums (copies).
    // (the DPP result taken before the ?: -- inside it clang branches, and
    // the move would read the masked-off lanes 0-7 as zeros)
    const uint64_t tl8 = dpp_u64<kDppRowRor8>(tl);
    const uint64_t am = acc + (c < 8 ? tl : tl8);
    // merge (util/xxhash.h:5182-5206): pairs (2i, 2i + 1) in lanes 2i, 2i + 1
    const uint64_t mine = am ^ lds_sec_at<3>(1 + (c & 7u));  // offset 11 + 8 a
    const uint64_t odd = dpp_u64<kDppQuadXor1>(mine);
    uint64_t m = (c & 1u) ? 0ull : mul128_fold64(mine, odd);
    m += dpp_u64<kDppQuadXor2>(m);  // lanes 0 + 2, 4 + 6
    m += dpp_u64<kDppRowRor4>(m);   // (0 + 2) + (4 + 6) in lane 0
    h = xxh3_avalanche((uint64_t)r.len * P64_1 + m);
  }
  return h;
}

// One row round of the CRC: lane c's chunk into the lane's state (the row
// driver's 4-byte table step), the record's init injected at lane 0 of
// round 0, the bytes before the payload zeroed; in the record's last round
// the lanes past its last byte keep their state.  Returns the state.
__device__ __forceinline__ uint32_t wr_crc_round(uint32_t s, const WrRow& r, Chunk ch, uint32_t c,
                                                 const CrcLane& L, bool act) {
  const bool first = r.k == 0, last = r.k + 1 == r.R();
  const uint32_t b = r.b();
  uint32_t* w = reinterpret_cast<uint32_t*>(&ch.v[0]);
  // first round, lane 0: the b bytes before the payload are zeros
  if (first && c == 0) w[0] &= 0xFFFFFFFFu << (8 * b);
  // last round: lane e keeps the first kb bytes of its chunk
  const uint32_t E = r.len + b - 1024 * r.k;  // bytes of the round in the record (1..1024)
  const uint32_t e = (E - 1) >> 6, kb = E - 64 * e;
  if (last && c == e) {
#pragma unroll
    for (int q = 0; q < 16; q++) {
      const int kq = (int)kb - 4 * q;
      w[q] = kq >= 4 ? w[q] : kq <= 0 ? 0u : w[q] & (0xFFFFFFFFu >> (8 * (4 - kq)));
    }
  }
  uint32_t x = 0;
  if (wave_any(!first)) x = crc_nibmap(row_gap_off<16>(), s);
  x = first ? (c == 0 ? *lds_p32(kLdsWrInj + 4 * (r.type() * 4 + b)) : 0u) : x;
  x ^= w[0];
#pragma unroll
  for (int k = 0; k < 16; k++) x = crc_step4x(x, L, k < 15 ? w[k + 1] : 0u);
  return (act && !(last && c > e)) ? x : s;
}

// The record's CRC (Extend(type_crc, payload)) from the last round's states.
__device__ __forceinline__ uint32_t wr_crc_finish(uint32_t s, const WrRow& r, uint32_t c) {
  const uint32_t E = r.len + r.b() - 1024 * (r.R() - 1);
  const uint32_t e = (E - 1) >> 6, kb = E - 64 * e;
  // to the end of chunk e: lanes c <= e (this round) by 64 (e - c), lanes
  // past e (the previous round) by 64 (16 + e - c)
  const uint32_t j = c <= e ? e - c : 16 + e - c;
  uint32_t p = row_xor32<16>(crc_lane_final4(s, (63u - j) << 2));
  if (wave_any(kb != 64)) p = crc_unshift(64 - kb, p);
  return r.len == 0 ? *lds_p32(kLdsWrInit + 4 * r.type()) : ~p;
}

__device__ __forceinline__ uint4 wr_desc(uint32_t t, uint32_t share) {
  const span_u32x4 v = *reinterpret_cast<__attribute__((address_space(3))) const span_u32x4*>(
      static_cast<size_t>(kLdsWrDesc + 16 * (t < share ? t : 0)));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint32_t wr_ticket(bool take) {
  uint32_t t = 0;
  if ((threadIdx.x & 15) == 0 && take)
    t = __hip_atomic_fetch_add(lds_p32(kLdsWrTicket), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)((threadIdx.x & 48u) << 2), (int)t);
}

struct WrArgs {
  const uint8_t* wal;
  const WalRecDesc* recs;
  uint32_t count;
  uint8_t* ok;       // per record: 1 = the CRC holds
  uint64_t* x3;      // per record: XXH3_64bits of its payload (hashed records)
};

// A window of the workgroup's records [w0, w0 + n): staged, then the rows loop.
struct WrCtx {
  const WrArgs& a;
  uint32_t w0, n, c;
  uint64_t base;
  const CrcLane& L;
  const WrX3& X;
};
// One iteration: round A.k of A's record (loads LA) is hashed while B -- the
// row's next round or its next record's first -- is set up and loaded.
// Returns whether any row goes on.
__device__ __forceinline__ bool wr_step(const WrCtx& x, const WrRow& A, const WrLoads& LA, bool live, WrRow& B,
                                        WrLoads& LB, bool& blive, uint32_t& nt, uint4& nd, uint32_t& s,
                                        uint64_t& acc) {
  const uint32_t c = x.c;
  const bool last = A.k + 1 == A.R();
  const bool go = live && (!last || nt < x.n);
  const bool sw = go && last;
  B = A;
  B.k = A.k + 1;
  const WrRow N = wr_row(nd, x.w0 + (nt < x.n ? nt : 0), x.base);
  B = wr_sel(sw, N, B);
  LB = wr_load(B, c);
  if (wave_any(sw)) {
    const uint32_t tk = wr_ticket(sw);
    if (sw) {
      nt = tk;
      nd = wr_desc(tk, x.n);
    }
  }
  // this round: CRC, then XXH3 from the same registers
  s = wr_crc_round(s, A, LA.ch, c, x.L, live);
  bool merge = false;
  const bool xa = live && A.hash() == 1u && A.k <= A.nb();
  uint64_t h = 0;
  if (wave_any(xa)) h = wr_x3_round(A, LA, c, x.X, acc, xa, merge);
  if (wave_any(live && last)) {
    const uint32_t crc = wr_crc_finish(s, A, c);
    if (live && last && c == 0) x.a.ok[A.i] = crc_mask(crc) == A.stored ? 1 : 0;
    // a record of <= 240 bytes: its XXH3 on the row, one window per lane
    // (x3s_row_hash; the small classes on lane 0)
    const bool sh = live && last && A.hash() == 2u;
    if (wave_any(sh)) {
      const uint64_t h2 = x3s_hash_row<false>(A.P, sh ? A.len : 0u, 0);  // (other rows: an empty span)
      if (sh && c == 0) x.a.x3[A.i] = h2;
    }
    s = (live && last) ? 0u : s;
  }
  if (merge && c == 0) x.a.x3[A.i] = h;
  if (merge || (live && last)) acc = x.X.init(c);
  blive = go;
  return wave_any(go);
}

// A window of the workgroup's records [w0, w0 + n) (staged), the rows loop
// unrolled twice so the two iterations' rows and loads swap register names
// instead of being copied every round.
template <bool U2>
__device__ __forceinline__ void wr_rows_loop(const WrArgs& a, uint32_t w0, uint32_t n, const CrcLane& L,
                                             const WrX3& X) {
  const uint32_t c = threadIdx.x & 15u;
  const WrCtx x{a, w0, n, c, reinterpret_cast<uint64_t>(a.wal), L, X};
  uint32_t t = wr_ticket(true);
  bool la = t < n, lb = false;
  WrRow A = wr_row(wr_desc(t, n), w0 + (la ? t : 0), x.base), B;
  WrLoads LA = wr_load(A, c), LB;
  uint32_t nt = wr_ticket(true);
  uint4 nd = wr_desc(nt, n);
  uint32_t s = 0;
  uint64_t acc = X.init(c);
  if (!wave_any(la)) return;
  if constexpr (U2) {
    for (;;) {
      if (!wr_step(x, A, LA, la, B, LB, lb, nt, nd, s, acc)) break;
      if (!wr_step(x, B, LB, lb, A, LA, la, nt, nd, s, acc)) break;
    }
  } else {
    while (wr_step(x, A, LA, la, B, LB, lb, nt, nd, s, acc)) {
      A = B;
      LA = LB;
      la = lb;
    }
  }
}

// Workgroup b: a byte-balanced contiguous share of the records, in windows
// of kWrDescCache staged in LDS.
struct WrOffs {
  const WalRecDesc* recs;
  __device__ uint64_t off(uint32_t i) const {
    const uint4 d = reinterpret_cast<const uint4*>(recs)[i];
    return (uint64_t)d.x | ((uint64_t)(d.y & 0xFFFFu) << 32);
  }
};
template <bool U2>
__global__ __launch_bounds__(1024) void k_wal_recover(WrArgs a, WalTypeCrcs tc) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  asm volatile("" ::"v"((uint32_t)(size_t)lds));
  uint32_t lo, hi;
  share_by_bytes(WrOffs{a.recs}, 0u, a.count, a.count / gridDim.x + 1, lds_p32(kLdsWrTicket + 8), &lo, &hi,
                 [&](uint32_t i) { return a.recs[i].len; });
  crc_fill_rows(lds, &g_crc_tables);
  if (threadIdx.x < 25) *lds_p64(kLdsWrSecret + 8 * threadIdx.x) = kXxh3SecretW.w[threadIdx.x];
  if (threadIdx.x >= 32 && threadIdx.x < 40) {  // XXH3_INIT_ACC (util/xxhash.h:5208-5209)
    const uint32_t q = threadIdx.x - 32;
    const uint64_t ia = q == 0 ? (uint64_t)P32_3 : q == 1 ? P64_1 : q == 2 ? P64_2 : q == 3 ? P64_3
                      : q == 4 ? P64_4 : q == 5 ? (uint64_t)P32_2 : q == 6 ? P64_5 : (uint64_t)P32_1;
    *lds_p64(kLdsWrInitAcc + 8 * q) = ia;
  }
  __syncthreads();
  wr_init_tables(tc);
  const CrcLane L = crc_lane();
  const WrX3 X = wr_x3(threadIdx.x & 15u);
  const uint32_t n = hi - lo;
  for (uint32_t w0 = 0; w0 < n; w0 += kWrDescCache) {
    const uint32_t wn = n - w0 < kWrDescCache ? n - w0 : kWrDescCache;
    __syncthreads();  // (the init tables are built / every row is done with the previous window)
    for (uint32_t t = threadIdx.x; t < wn; t += blockDim.x) {
      const uint4 d = reinterpret_cast<const uint4*>(a.recs)[lo + w0 + t];
      *reinterpret_cast<__attribute__((address_space(3))) span_u32x4*>(static_cast<size_t>(kLdsWrDesc + 16 * t)) =
          span_u32x4{d.x, d.y, d.z, d.w};
    }
    if (threadIdx.x == 0) *lds_p32(kLdsWrTicket) = 0;
    __syncthreads();
    wr_rows_loop<U2>(a, lo + w0, wn, L, X);
  }
}

}  // namespace mck
