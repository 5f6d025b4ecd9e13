// mck_tables.hpp -- GF(2) constant tables for the CRC32C kernels.
//
// CRC-32C is linear over GF(2): the "pure" state (init 0, no final
// inversion -- the algebra of util/crc32c.cc:1221-1266) after appending d
// zero bytes is zshift(s, d) = s * x^(8d) mod P, P the reflected Castagnoli
// polynomial 0x82f63b78 (util/crc32c.cc:1193).  Every table here is a byte-
// or nibble-wise decomposition of one such linear map, so a map costs 4 byte
// lookups or 8 nibble lookups.  Tables are generated on the host once per
// process and uploaded to each device (mck_engine.cpp).
#pragma once
#include <stdint.h>

namespace mck {

constexpr uint32_t kCrc32cPoly = 0x82f63b78u;  // reflected

// Lanes cover 64-byte chunks; a wave covers one 4 KiB "round" of a span.
constexpr int kChunkBytes = 64;
constexpr int kRoundBytes = 64 * kChunkBytes;                   // 4096
constexpr int kGapBytes = kRoundBytes - kChunkBytes;            // 4032
constexpr int kMaxUnshift = 64;                                 // k in [0,64)
// Row driver (mck_crc.hpp crc_rows_driver): a row of W = 4, 8 or 16 lanes
// covers one 64 W-byte round of a span; its lanes' chunks are 64 (W - 1)
// bytes apart between rounds.
constexpr int kRowWidths = 3;  // W = 4 << k
constexpr int row_gap_bytes(int k) { return (4 << k) * kChunkBytes - kChunkBytes; }
// Body/head driver: a span's head and body pieces are moved to its end by
// zshift(4096 m), m <= 2^20 (spans < 4 GiB): pow1k entries 2..22.
constexpr int kPowBits = 23;

struct alignas(16) CrcTables {
  uint32_t step[4][256];          // zshift(v << 8t, 4): the 4-byte step
  uint32_t lane_final[8][16][64]; // zshift(v << 4n, 64*(63-lane))
  uint32_t gap[8][16];            // zshift(v << 4n, kGapBytes)
  uint32_t ext1[8][16];           // zshift(v << 4n, 1)
  uint32_t half[8][16];           // zshift(v << 4n, 32): joins a lane's chains
  uint32_t quarter[8][16];        // zshift(v << 4n, 16)
  uint32_t unshift[kMaxUnshift][8][16];  // zshift^-1(v << 4n, k)
  uint32_t gap_row[kRowWidths][8][16];  // zshift(v << 4n, 64 (W - 1)): row driver
  uint32_t zero16[4];             // a zero piece: the row driver's loads before a span
  // 80-byte lane chunks in 16-lane rows (the one-pass WAL writer: a 1280-byte
  // round holds a whole ~1 KB record fragment)
  uint32_t lane_final80[8][16][16];  // zshift(v << 4n, 80 (15 - c))
  uint32_t gap80[8][16];             // zshift(v << 4n, 80 * 15)
  // interleaved pieces in 16-lane rows (the one-pass WAL writer's default:
  // lane c holds pieces c + 16 j of a 1280-byte round, j = 0..4)
  uint32_t lane_final16[8][16][16];  // zshift(v << 4n, 4 + 16 (15 - c))
  uint32_t gap244[4][256];           // zshift(v << 8t, 244): piece to piece
  // body/head driver (mck_crc_bh.hpp): a span's parts moved to its end
  uint32_t pow1k[kPowBits][8][16];    // zshift(v << 4n, 1024 * 2^b)
  // 4- / 8-lane rows' finish (round 4): lane c's shift to the row's end and
  // the un-shift of the kt trailing zero bytes as ONE map, a shift by
  // 64 (W - 1 - c) - kt bytes (an un-shift for c = W - 1); lane-minor, as
  // lane_final, so the lanes of a row read neighbouring LDS banks
  uint32_t rowfin4[16][8][16][4];  // [kt][n][v][c]
  uint32_t rowfin8[16][8][16][8];
};

// ---- host-side GF(2) helpers (also used by the host shims) ----------------
inline uint32_t gf_mulx(uint32_t a) { return (a >> 1) ^ ((a & 1u) ? kCrc32cPoly : 0u); }
// inverse of gf_mulx: bit 31 of P is set, so bit 31 of mulx(a) = a & 1.
inline uint32_t gf_unmulx(uint32_t b) {
  uint32_t lo = b >> 31;
  return ((b ^ (lo ? kCrc32cPoly : 0u)) << 1) | lo;
}
inline uint32_t gf_mul(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (int j = 0; j < 32; j++) {
    if (b & (0x80000000u >> j)) p ^= a;
    a = gf_mulx(a);
  }
  return p;
}
inline uint32_t gf_xpow8n(uint64_t nbytes) {
  uint32_t r = 0x80000000u, sq = 0x00800000u;  // x^0, x^8
  while (nbytes) {
    if (nbytes & 1) r = gf_mul(r, sq);
    sq = gf_mul(sq, sq);
    nbytes >>= 1;
  }
  return r;
}
inline uint32_t gf_zshift(uint32_t s, uint64_t nbytes) { return gf_mul(s, gf_xpow8n(nbytes)); }

inline void build_crc_tables(CrcTables* t) {
  const uint32_t k4 = gf_xpow8n(4);
  for (int b = 0; b < 4; b++)
    for (int v = 0; v < 256; v++) t->step[b][v] = gf_mul((uint32_t)v << (8 * b), k4);
  for (int l = 0; l < 64; l++) {
    const uint32_t k = gf_xpow8n((uint64_t)kChunkBytes * (63 - l));
    for (int n = 0; n < 8; n++)
      for (int v = 0; v < 16; v++) t->lane_final[n][v][l] = gf_mul((uint32_t)v << (4 * n), k);
  }
  const uint32_t kg = gf_xpow8n(kGapBytes), k1 = gf_xpow8n(1), k32 = gf_xpow8n(kChunkBytes / 2),
                 k16 = gf_xpow8n(kChunkBytes / 4);
  for (int n = 0; n < 8; n++)
    for (int v = 0; v < 16; v++) {
      t->gap[n][v] = gf_mul((uint32_t)v << (4 * n), kg);
      t->ext1[n][v] = gf_mul((uint32_t)v << (4 * n), k1);
      t->half[n][v] = gf_mul((uint32_t)v << (4 * n), k32);
      t->quarter[n][v] = gf_mul((uint32_t)v << (4 * n), k16);
    }
  for (int k = 0; k < 4; k++) t->zero16[k] = 0;
  for (int k = 0; k < kRowWidths; k++) {
    const uint32_t kr = gf_xpow8n(row_gap_bytes(k));
    for (int n = 0; n < 8; n++)
      for (int v = 0; v < 16; v++) t->gap_row[k][n][v] = gf_mul((uint32_t)v << (4 * n), kr);
  }
  for (int c = 0; c < 16; c++) {
    const uint32_t k = gf_xpow8n(80u * (15 - c));
    for (int n = 0; n < 8; n++)
      for (int v = 0; v < 16; v++) t->lane_final80[n][v][c] = gf_mul((uint32_t)v << (4 * n), k);
  }
  {
    const uint32_t k = gf_xpow8n(80u * 15);
    for (int n = 0; n < 8; n++)
      for (int v = 0; v < 16; v++) t->gap80[n][v] = gf_mul((uint32_t)v << (4 * n), k);
  }
  for (int c = 0; c < 16; c++) {
    const uint32_t k = gf_xpow8n(4u + 16u * (15 - c));
    for (int n = 0; n < 8; n++)
      for (int v = 0; v < 16; v++) t->lane_final16[n][v][c] = gf_mul((uint32_t)v << (4 * n), k);
  }
  {
    const uint32_t k = gf_xpow8n(244);
    for (int b = 0; b < 4; b++)
      for (int v = 0; v < 256; v++) t->gap244[b][v] = gf_mul((uint32_t)v << (8 * b), k);
  }
  for (int b = 0; b < kPowBits; b++) {
    const uint32_t k = gf_xpow8n(1024ull << b);
    for (int n = 0; n < 8; n++)
      for (int v = 0; v < 16; v++) t->pow1k[b][n][v] = gf_mul((uint32_t)v << (4 * n), k);
  }
  for (int k = 0; k < kMaxUnshift; k++)
    for (int n = 0; n < 8; n++)
      for (int v = 0; v < 16; v++) {
        uint32_t x = (uint32_t)v << (4 * n);
        for (int i = 0; i < 8 * k; i++) x = gf_unmulx(x);
        t->unshift[k][n][v] = x;
      }
  // rowfin4 / rowfin8: lane c of a W-lane row, kt trailing bytes: a shift
  // by 64 (W - 1 - c) - kt bytes (< 0, an un-shift, only for c = W - 1)
  auto rowfin = [&](int W, int c, int kt, int n, int v) {
    const int d = kChunkBytes * (W - 1 - c) - kt;
    uint32_t x = (uint32_t)v << (4 * n);
    if (d >= 0) return gf_mul(x, gf_xpow8n((uint64_t)d));
    for (int i = 0; i < -8 * d; i++) x = gf_unmulx(x);
    return x;
  };
  for (int c = 0; c < 8; c++)
    for (int kt = 0; kt < 16; kt++)
      for (int n = 0; n < 8; n++)
        for (int v = 0; v < 16; v++) {
          if (c < 4) t->rowfin4[kt][n][v][c] = rowfin(4, c, kt, n, v);
          t->rowfin8[kt][n][v][c] = rowfin(8, c, kt, n, v);
        }
}

}  // namespace mck
