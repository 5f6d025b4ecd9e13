// mck_walrec.hpp -- WAL recovery in one device pass (round 6): every physical
// record's CRC32C (ReadPhysicalRecord, db/log_reader.cc:450-584) and, from
// the same read of the image, the XXH3_64bits record checksum of every
// single-fragment record (ReadRecord's kFullType case, :95-116 -- the
// logical record IS the fragment, hashed in place, :107-110).
//
// The walk is k_wal_verify's (one wave per 32 KiB block, a wave's blocks
// form one record pipeline, the next block's first round loaded with the
// last one of a record that ends its block).  A kFullType /
// kRecyclableFullType record of more than 240 bytes is also hashed by the
// XXH3 wave layout (x3w_*, mck_xxh.hpp) in lockstep with its CRC rounds, one
// iteration behind: iteration m runs CRC round m (4 KiB, end-anchored) and
// XXH3 unit m - 1 (4 KiB, start-anchored).  Unit m - 1 lies in CRC windows
// m - 1 and m, whose loads were issued before it, so its loads are L2 hits on
// lines the CRC loads brought in (no second HBM read), and they are issued
// before the CRC prefetch of window m + 1, so waiting for them never waits
// for the prefetch (vmcnt retires in order).  Shorter full records take the
// short classes (xxh3_short) on one lane after the CRC, from L2.
//
// Output per block: mck_wal_block_result (as k_wal_verify), and the hashes
// of the block's full-type records, in walk order: record k of block b at
// x3[base_b + k] for k < cap_b, with base_b = slot_base[b] and cap_b =
// slot_base[b + 1] - base_b (a dense array: the host's plan counted the full
// records of every block, mck_wal_recover) or, without slot_base, base_b =
// b * nslots and cap_b = nslots.  The host walk (mck_wal.cc) counts the full
// records it reads per block to find a record's slot; multi-fragment records
// are hashed by a gather + XXH3 batch.
#pragma once
#include "mck_kernels.hpp"

namespace mck {

// per-wave 1 KiB XXH3 exchange buffer (x3w_fold's tx), in the LDS bytes the
// wave-driver CRC image leaves free below the step tables
constexpr uint32_t kLdsWalX3 = kLdsLowEnd;
static_assert(kLdsWalX3 + 16 * 1024 <= kLdsStep, "16 waves x 1 KiB below the step tables");

// the XXH3 wave layout's per-lane constants (X3Row, ~50 VGPRs if kept in
// registers beside the CRC pipeline's): one copy per lane index in LDS,
// written once per workgroup, read inside each fold (only the fields the
// fold uses are loaded); the loads' address math needs only the lane's
// indices (x3_row_idx)
constexpr uint32_t kLdsWalX3Row = kLdsWalX3 + 16 * 1024;
static_assert(kLdsWalX3Row + 64 * sizeof(X3Row) <= kLdsStep, "X3Row per lane below the step tables");
static_assert(sizeof(X3Row) % 8 == 0, "X3Row as u64 words");
__device__ __forceinline__ X3Row x3_row_lds() {
  X3Row X;
  uint64_t* d = reinterpret_cast<uint64_t*>(&X);
  const uint32_t off = kLdsWalX3Row + (uint32_t)sizeof(X3Row) * (threadIdx.x & 63);
#pragma unroll
  for (uint32_t i = 0; i < sizeof(X3Row) / 8; i++) d[i] = *lds_p64(off + 8 * i);
  return X;
}
__device__ __forceinline__ void x3_row_lds_store() {
  if (threadIdx.x < 64) {
    const X3Row X = x3_row(0);
    const uint64_t* s = reinterpret_cast<const uint64_t*>(&X);
#pragma unroll
    for (uint32_t i = 0; i < sizeof(X3Row) / 8; i++)
      *lds_p64(kLdsWalX3Row + (uint32_t)sizeof(X3Row) * threadIdx.x + 8 * i) = s[i];
  }
}
__device__ __forceinline__ X3Row x3_row_idx() {
  X3Row X{};
  X.lane = threadIdx.x & 63;
  X.row = X.lane >> 4;
  X.j = X.lane & 15;
  X.q = X.j & 3;
  X.st4 = X.j >> 2;
  X.role = X.lane >> 5;
  return X;
}

// CRC image fill for any workgroup size (crc_fill_lds assumes kCrcBlock
// threads): once per persistent workgroup
__device__ __forceinline__ void crc_fill_lds_any(uint8_t* lds, const CrcTables* __restrict__ g) {
  uint4* l4 = reinterpret_cast<uint4*>(lds + kLdsStep);
  for (uint32_t i = threadIdx.x; i < 4096; i += blockDim.x) {
    const uint32_t x = g->step[(i >> 2) & 3][i >> 4];
    l4[i] = make_uint4(x, x, x, x);
  }
  const uint4* lo = reinterpret_cast<const uint4*>(&g->lane_final[0][0][0]);
  uint4* dlo = reinterpret_cast<uint4*>(lds + kLdsFinal);
  for (uint32_t i = threadIdx.x; i < (uint32_t)kFillLow; i += blockDim.x) dlo[i] = lo[i];
  const uint4* us = reinterpret_cast<const uint4*>(&g->unshift[0][0][0]);
  uint4* dus = reinterpret_cast<uint4*>(lds + kLdsUnshift);
  for (uint32_t i = threadIdx.x; i < (uint32_t)kFillUnshift; i += blockDim.x) dus[i] = us[i];
}

// finish() target of the XXH3 wave fold: slot k of the current block
struct OpWalX3 {
  uint64_t* out;  // x3 + block * nslots
  typedef NoPre Pre;
  __device__ void finish(uint32_t k, uint64_t h, const Pre& = Pre{}) const { out[k] = h; }
};

// An interior unit k (k + 1 < units: four full segments, loads x3w_round_load)
// folded into the lane's accumulator: x3w_fold's round part with every
// segment scrambled.
__device__ __forceinline__ void x3w_interior(const X3WSpan& sp, X3RoundLoads R, uint64_t& a, uint64_t* tx) {
  const X3Row X = x3_row_lds();
  uint64_t c0, c1;
  x3w_round_sums<false>(sp, R, X, c0, c1);
  if (X.st4 == 0) {
    tx[4 * X.q + X.row] = c0;
    tx[64 + 4 * X.q + X.row] = c1;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
  const ulonglong2* tr = reinterpret_cast<const ulonglong2*>(tx + 64 * X.role + 4 * X.q);
  const ulonglong2 t01 = tr[0], t23 = tr[1];
  a = xxh3_scramble(a + t01.x, X.ksw);
  a = xxh3_scramble(a + t01.y, X.ksw);
  a = xxh3_scramble(a + t23.x, X.ksw);
  a = xxh3_scramble(a + t23.y, X.ksw);
}

// x3: NULL = CRC only (k_wal_verify's output).
// T: transposed CRC loads (non-temporal) as k_wal_verify<true>; the XXH3
// re-reads use the default policy.
constexpr int kWalRecThreads = 512;  // 8 waves per CU: 256 VGPRs each
template <bool T>
__global__ __launch_bounds__(kWalRecThreads) void k_wal_recover(const uint8_t* wal, uint64_t nbytes, uint32_t log_number,
                                                      WalResult* res, uint32_t nblocks, uint64_t* x3,
                                                      const uint64_t* slot_base, uint32_t nslots) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  crc_fill_lds_any(lds, &g_crc_tables);
  x3_row_lds_store();
  __syncthreads();
  const CrcLane L = crc_lane();
  const X3Row XI = x3_row_idx();
  uint64_t* tx = reinterpret_cast<uint64_t*>(lds + kLdsWalX3 + 1024u * (threadIdx.x >> 6));
  const uint32_t wpb = blockDim.x >> 6;
  const uint32_t nw = gridDim.x * wpb;
  // block k's slots (wave-uniform: the loads go through the scalar cache)
  auto slots_of = [&](uint32_t k, uint64_t& base, uint32_t& cap) {
    if (!x3) {
      base = 0;
      cap = 0;
    } else if (slot_base) {
      base = slot_base[k];
      cap = (uint32_t)(slot_base[k + 1] - base);
    } else {
      base = (uint64_t)k * nslots;
      cap = nslots;
    }
  };
  uint32_t cb = __builtin_amdgcn_readfirstlane(blockIdx.x * wpb + (threadIdx.x >> 6));
  if (cb >= nblocks) return;
  auto block_size = [&](uint32_t k) {
    const uint64_t rem = nbytes - (uint64_t)k * 32768;
    return rem < 32768 ? (uint32_t)rem : 32768u;
  };
  auto last_block = [&](uint32_t k) { return nbytes - (uint64_t)k * 32768 <= 32768; };
  auto emit = [&](uint32_t k, uint32_t ok, int32_t status, uint32_t pos) {
    if ((threadIdx.x & 63) == 0) {
      WalResult o;
      o.records_ok = ok;
      o.status = status;
      o.stop_offset = status ? pos : block_size(k);
      o.bytes_ok = pos;
      res[k] = o;
    }
  };
  // a block's first record from the 16-byte vector load h of its start
  // (w1: header bytes 4-7 -- length, type, first log-number byte)
  auto parse_first = [&](uint32_t k, const uint4& h) {
    const uint32_t w1 = rfl_u32(h.y);
    return wal_parse(block_size(k), last_block(k), log_number, w1,
                     [&] { return (w1 >> 24) | (rfl_u32(h.z) << 8); });
  };
  uint32_t cpos = 0, cok = 0, kf = 0;  // record offset, records verified before it, full records before it
  uint64_t xbase;
  uint32_t xcap;
  slots_of(cb, xbase, xcap);
  uint4 hb = wal_hdr16(wal, cb);
  bool seek = true;
  WalRec rec{};
  uint32_t stored = 0, type = 0;
  CrcSpan sp = crc_span(wal, 0, 0u);
  Chunk cur{};
  for (;;) {
    if (seek) {
      for (;;) {  // finish blocks until a record to hash
        const uint32_t left = block_size(cb) - cpos;
        const uint8_t* h = wal + (uint64_t)cb * 32768 + cpos;
        uint32_t w1 = 0;
        if (cpos == 0) {
          w1 = rfl_u32(hb.y);
          rec = parse_first(cb, hb);
          stored = rfl_u32(hb.x);
        } else {
          if (left >= 7) {
            stored = rfl_u32(rd32_bytes(h));
            w1 = rfl_u32((uint32_t)h[4] | ((uint32_t)h[5] << 8) | ((uint32_t)h[6] << 16));
          }
          rec = wal_parse(left, last_block(cb), log_number, w1, [&] { return rfl_u32(rd32_bytes(h + 7)); });
        }
        type = (w1 >> 16) & 0xFFu;
        if (rec.go) break;
        emit(cb, cok, rec.status, cpos);
        cb += nw;
        if (cb >= nblocks) return;
        cpos = 0;
        cok = 0;
        kf = 0;
        slots_of(cb, xbase, xcap);
        hb = wal_hdr16(wal, cb);
      }
      sp = crc_span(wal + (uint64_t)cb * 32768 + cpos + 6, rec.length + rec.hsize - 6, 0u);
      cur = crc_load_chunk<T>(sp, sp.rounds - 1, L);
    }
    const uint32_t size = block_size(cb);
    const uint32_t e = cpos + rec.hsize + rec.length;
    const uint32_t nb = cb + nw;
    const bool spec = size - e < 7 && nb < nblocks;
    const uint4 hn = wal_hdr16(wal, spec ? nb : cb);
    WalRec nrec = rec;
    auto next_span = [&] {
      return nrec.go ? crc_span(wal + (uint64_t)nb * 32768 + 6, nrec.length + nrec.hsize - 6, 0u)
                     : crc_span(wal + (uint64_t)nb * 32768, 0, 0u);
    };
    // the record's XXH3 (ReadRecord's record_checksum of a one-fragment record)
    const bool full = type == 1u || type == 5u;
    const bool slot = full && kf < xcap;
    const OpWalX3 xop{x3 + xbase};
    const uint64_t xptr = sp.ptr + rec.hsize - 6;  // the payload
    const uint32_t xlen = rec.length;
    const X3WSpan xs = x3w_span<false>(xptr, xlen, kf);
    const uint32_t units = (slot && xlen > 240) ? xs.units : 0u;
    const uint32_t iters = (uint32_t)sp.rounds > units ? (uint32_t)sp.rounds : units + 1;
    uint64_t a = x3_row_lds().iw;
    uint32_t s = 0;
    for (uint32_t m = 0; m < iters; m++) {  // wave-uniform
      const int r = sp.rounds - 1 - (int)m;    // CRC round (< 0: XXH3 only)
      const bool xu = m >= 1 && m <= units;     // XXH3 unit m - 1
      const bool xl = xu && m == units;         // ... the last one
      // XXH3 loads first (L2), then the CRC load of the next window (or of
      // the next block's first round with this record's last iteration)
      X3RoundLoads R{};
      X3WLoads XL{};
      if (xu && !xl) R = x3w_round_load<false>(xs, m - 1, XI);
      if (xl) XL = x3w_load<false>(xs, m - 1, XI);
      Chunk nxt;
      if (r > 0) {
        nxt = crc_load_chunk<T>(sp, r - 1, L);
      } else if (m + 1 == iters && spec) {
        nrec = parse_first(nb, hn);
        const CrcSpan nsp = next_span();
        nxt = crc_load_chunk<T>(nsp, nsp.rounds - 1, L);
      }
      if (r >= 0) {
        if (T && !(sp.mini && r == sp.rounds - 1)) row_transpose(cur);  // wave-uniform
        s = crc_round(s, cur, sp, r, L);
      }
      if (r > 0 || (m + 1 == iters && spec)) cur = nxt;
      if (xu && !xl) x3w_interior(xs, R, a, tx);
      if (xl) x3w_fold<OpWalX3, false>(xop, xs, m - 1, XL, x3_row_lds(), a, NoPre{}, tx);
    }
    const bool pass = crc_mask(rfl_u32(crc_finish(s, sp, L))) == stored;
    if (pass && slot && xlen <= 240 && (threadIdx.x & 63) == 0)
      xop.finish(kf, xxh3_short(reinterpret_cast<const uint8_t*>(xptr), xlen));
    if (!pass) {
      emit(cb, cok, 1, cpos);  // kBadRecordChecksum
    } else if (size - e < 7) {
      emit(cb, cok + 1, last_block(cb) && size > e ? 5 : 0, e);
    } else {  // the next record of the same block
      cok++;
      kf += full ? 1u : 0u;
      cpos = e;
      seek = true;
      continue;
    }
    if (nb >= nblocks) return;
    cb = nb;
    cpos = 0;
    cok = 0;
    kf = 0;
    slots_of(cb, xbase, xcap);
    hb = spec ? hn : wal_hdr16(wal, cb);
    seek = !(spec && nrec.go);
    if (!seek) {  // pipelined: the record's first round is in cur
      rec = nrec;
      sp = next_span();
      stored = rfl_u32(hn.x);
      type = (rfl_u32(hn.y) >> 16) & 0xFFu;
    }
  }
}

}  // namespace mck
