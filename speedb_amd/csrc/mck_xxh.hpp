// mck_xxh.hpp -- device XXH3-64 (16-lane row per span) and legacy XXH32/XXH64
// (lane per span), xxHash v0.8.1 as vendored at util/xxhash.h; and XXPH3,
// the XXH3 preview (v0.7.2, util/xxph3.h) behind Hash64 / NPHash64, which
// runs on the same row driver (template flag PREVIEW).
//
// XXH3 long inputs (n > 240, util/xxhash.h:5141-5227): 8 u64 accumulators;
// each 1 KiB segment = 16 stripes x 64 B, and within a segment the 128
// (stripe, accumulator-lane) terms are independent sums mod 2^64; only the
// scramble between segments is sequential.
//
// Layout: every 16-lane row of a wave owns one span.  Lane j of a row owns
// accumulator pair q = j & 3 (accumulators 2q, 2q+1) and the four stripes
// st4, st4+4, st4+8, st4+12 (st4 = j >> 2): per segment it issues four
// 16-byte loads (the row's 16 lanes read 256 contiguous bytes per load) and
// folds its four stripes locally, so the per-segment reduction is only 2
// in-row DPP steps (over st4) and the scramble chain never leaves the row.
// Rows walk their own spans (statically strided), so ragged batches keep all
// rows busy; the wave loops while any row has work.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mck_common.hpp"

namespace mck {

constexpr uint64_t P64_1 = 0x9E3779B185EBCA87ull, P64_2 = 0xC2B2AE3D27D4EB4Full,
                   P64_3 = 0x165667B19E3779F9ull, P64_4 = 0x85EBCA77C2B2AE63ull,
                   P64_5 = 0x27D4EB2F165667C5ull;
constexpr uint32_t P32_1 = 0x9E3779B1u, P32_2 = 0x85EBCA77u, P32_3 = 0xC2B2AE3Du,
                   P32_4 = 0x27D4EB2Fu, P32_5 = 0x165667B1u;

// XXH3_kSecret, util/xxhash.h:3661-3674 (192 bytes)
constexpr uint8_t kXxh3SecretBytes[192] = {
    0xb8, 0xfe, 0x6c, 0x39, 0x23, 0xa4, 0x4b, 0xbe, 0x7c, 0x01, 0x81, 0x2c, 0xf7, 0x21, 0xad, 0x1c,
    0xde, 0xd4, 0x6d, 0xe9, 0x83, 0x90, 0x97, 0xdb, 0x72, 0x40, 0xa4, 0xa4, 0xb7, 0xb3, 0x67, 0x1f,
    0xcb, 0x79, 0xe6, 0x4e, 0xcc, 0xc0, 0xe5, 0x78, 0x82, 0x5a, 0xd0, 0x7d, 0xcc, 0xff, 0x72, 0x21,
    0xb8, 0x08, 0x46, 0x74, 0xf7, 0x43, 0x24, 0x8e, 0xe0, 0x35, 0x90, 0xe6, 0x81, 0x3a, 0x26, 0x4c,
    0x3c, 0x28, 0x52, 0xbb, 0x91, 0xc3, 0x00, 0xcb, 0x88, 0xd0, 0x65, 0x8b, 0x1b, 0x53, 0x2e, 0xa3,
    0x71, 0x64, 0x48, 0x97, 0xa2, 0x0d, 0xf9, 0x4e, 0x38, 0x19, 0xef, 0x46, 0xa9, 0xde, 0xac, 0xd8,
    0xa8, 0xfa, 0x76, 0x3f, 0xe3, 0x9c, 0x34, 0x3f, 0xf9, 0xdc, 0xbb, 0xc7, 0xc7, 0x0b, 0x4f, 0x1d,
    0x8a, 0x51, 0xe0, 0x4b, 0xcd, 0xb4, 0x59, 0x31, 0xc8, 0x9f, 0x7e, 0xc9, 0xd9, 0x78, 0x73, 0x64,
    0xea, 0xc5, 0xac, 0x83, 0x34, 0xd3, 0xeb, 0xc3, 0xc5, 0x81, 0xa0, 0xff, 0xfa, 0x13, 0x63, 0xeb,
    0x17, 0x0d, 0xdd, 0x51, 0xb7, 0xf0, 0xda, 0x49, 0xd3, 0x16, 0x55, 0x26, 0x29, 0xd4, 0x68, 0x9e,
    0x2b, 0x16, 0xbe, 0x58, 0x7d, 0x47, 0xa1, 0xfc, 0x8f, 0xf8, 0xb8, 0xd1, 0x7a, 0xd0, 0x31, 0xce,
    0x45, 0xcb, 0x3a, 0x8f, 0x95, 0x16, 0x04, 0x28, 0xaf, 0xd7, 0xfb, 0xca, 0xbb, 0x4b, 0x40, 0x7e,
};
// ... as 24 little-endian 8-byte words (+ one zero word): a secret word at a
// per-lane byte offset is two aligned 8-byte loads and a funnel shift (the
// byte-wise read was up to 16 byte loads per word: the XXH3 wave driver's
// per-lane constants alone were ~100 loads per lane in its prologue)
struct X3SecretWords {
  uint64_t w[25];
};
constexpr X3SecretWords x3_secret_words() {
  X3SecretWords r{};
  for (int i = 0; i < 24; i++) {
    uint64_t v = 0;
    for (int b = 7; b >= 0; b--) v = (v << 8) | kXxh3SecretBytes[8 * i + b];
    r.w[i] = v;
  }
  r.w[24] = 0;
  return r;
}
__constant__ const X3SecretWords kXxh3SecretW = x3_secret_words();

__device__ __forceinline__ uint64_t sec64(int off) {
  const int w = off >> 3, sh = (off & 7) * 8;
  const uint64_t lo = kXxh3SecretW.w[w];
  if (sh == 0) return lo;
  return (lo >> sh) | (kXxh3SecretW.w[w + 1] << (64 - sh));
}
__device__ __forceinline__ uint32_t sec32(int off) { return (uint32_t)sec64(off); }
// 8 bytes at byte offset `off` of the seeded secret of
// XXPH3_initCustomSecret (util/xxph3.h:1613-1624): 8-byte word w of the
// default secret gets +seed (w even) or -seed (w odd).  seed 0 = the default
// secret, so XXH3 v0.8.1 uses the same accessor.
__device__ __forceinline__ uint64_t csec64(int off, uint64_t seed) {
  const int w = off >> 3, sh = (off & 7) * 8;
  const uint64_t lo = kXxh3SecretW.w[w] + ((w & 1) ? 0 - seed : seed);
  if (sh == 0) return lo;
  const uint64_t hi = kXxh3SecretW.w[w + 1] + (((w + 1) & 1) ? 0 - seed : seed);
  return (lo >> sh) | (hi << (64 - sh));
}

// unaligned little-endian reads from device memory
__device__ __forceinline__ uint64_t rd64(const uint8_t* p) {
  uint64_t v;
  __builtin_memcpy(&v, p, 8);
  return v;
}
__device__ __forceinline__ uint32_t rd32(const uint8_t* p) {
  uint32_t v;
  __builtin_memcpy(&v, p, 4);
  return v;
}

__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __forceinline__ uint64_t mul32to64(uint64_t x) {
  return (uint64_t)(uint32_t)x * (uint64_t)(uint32_t)(x >> 32);
}
__device__ __forceinline__ uint64_t mul128_fold64(uint64_t a, uint64_t b) {
  return (a * b) ^ __umul64hi(a, b);
}
__device__ __forceinline__ uint64_t xxh64_avalanche(uint64_t h) {
  h ^= h >> 33;
  h *= P64_2;
  h ^= h >> 29;
  h *= P64_3;
  h ^= h >> 32;
  return h;
}
__device__ __forceinline__ uint64_t xxh3_avalanche(uint64_t h) {
  h ^= h >> 37;
  h *= 0x165667919E3779F9ull;
  return h ^ (h >> 32);
}
__device__ __forceinline__ uint64_t xxh3_rrmxmx(uint64_t h, uint64_t len) {
  h ^= rotl64(h, 49) ^ rotl64(h, 24);
  h *= 0x9FB21C651E98DF25ull;
  h ^= (h >> 35) + len;
  h *= 0x9FB21C651E98DF25ull;
  return h ^ (h >> 28);
}
__device__ __forceinline__ uint64_t xxh3_mix16(const uint8_t* in, int s) {
  return mul128_fold64(rd64(in) ^ sec64(s), rd64(in + 8) ^ sec64(s + 8));
}

// XXH3_64bits for n <= 240 (util/xxhash.h:3990, 4060, 4100), one lane.
__device__ __noinline__ uint64_t xxh3_short(const uint8_t* in, uint64_t len) {
  if (len <= 16) {
    if (len > 8) {
      const uint64_t bf1 = sec64(24) ^ sec64(32), bf2 = sec64(40) ^ sec64(48);
      const uint64_t lo = rd64(in) ^ bf1, hi = rd64(in + len - 8) ^ bf2;
      return xxh3_avalanche(len + __builtin_bswap64(lo) + hi + mul128_fold64(lo, hi));
    }
    if (len >= 4) {
      const uint64_t in1 = rd32(in), in2 = rd32(in + len - 4);
      const uint64_t bf = sec64(8) ^ sec64(16);
      return xxh3_rrmxmx((in2 + (in1 << 32)) ^ bf, len);
    }
    if (len) {
      const uint32_t c1 = in[0], c2 = in[len >> 1], c3 = in[len - 1];
      const uint32_t comb = (c1 << 16) | (c2 << 24) | c3 | ((uint32_t)len << 8);
      return xxh64_avalanche((uint64_t)comb ^ (uint64_t)(sec32(0) ^ sec32(4)));
    }
    return xxh64_avalanche(sec64(56) ^ sec64(64));
  }
  uint64_t acc = len * P64_1, acc_end;
  if (len <= 128) {
    acc += xxh3_mix16(in, 0);
    acc_end = xxh3_mix16(in + len - 16, 16);
    if (len > 32) {
      acc += xxh3_mix16(in + 16, 32);
      acc_end += xxh3_mix16(in + len - 32, 48);
      if (len > 64) {
        acc += xxh3_mix16(in + 32, 64);
        acc_end += xxh3_mix16(in + len - 48, 80);
        if (len > 96) {
          acc += xxh3_mix16(in + 48, 96);
          acc_end += xxh3_mix16(in + len - 64, 112);
        }
      }
    }
    return xxh3_avalanche(acc + acc_end);
  }
  for (int i = 0; i < 8; i++) acc += xxh3_mix16(in + 16 * i, 16 * i);
  acc_end = xxh3_mix16(in + len - 16, 136 - 17);
  acc = xxh3_avalanche(acc);
  const int rounds = (int)len / 16;
  for (int i = 8; i < rounds; i++) acc_end += xxh3_mix16(in + 16 * i, 16 * (i - 8) + 3);
  return xxh3_avalanche(acc + acc_end);
}

// ---- XXPH3 (the XXH3 preview v0.7.2 behind Hash64/NPHash64) ---------------
// util/xxph3.h; util/hash.cc:81-88.  Differs from v0.8.1 in the short
// length classes, the avalanche constant (PRIME64_3), the non-swapping
// accumulate and the block/last-stripe rules of the long loop.
__device__ __forceinline__ uint64_t xxph3_avalanche(uint64_t h) {  // :1073
  h ^= h >> 37;
  h *= P64_3;
  return h ^ (h >> 32);
}
__device__ __forceinline__ uint64_t xxph3_mix16(const uint8_t* in, int s, uint64_t seed) {  // :1644
  return mul128_fold64(rd64(in) ^ (sec64(s) + seed), rd64(in + 8) ^ (sec64(s + 8) - seed));
}
// :1102 len 4..8 on the two (possibly overlapping) 4-byte words
__device__ __forceinline__ uint64_t xxph3_4to8(uint32_t lo, uint32_t hi, uint64_t len, uint64_t seed) {
  const uint64_t keyed = ((uint64_t)lo | ((uint64_t)hi << 32)) ^ (sec64(0) + seed);
  const uint64_t mix = len + ((keyed ^ (keyed >> 51)) * P32_1);
  return xxph3_avalanche((mix ^ (mix >> 47)) * P64_2);
}
// :1086 len 1..3
__device__ __forceinline__ uint64_t xxph3_1to3(uint32_t c1, uint32_t c2, uint32_t c3, uint64_t len,
                                               uint64_t seed) {
  const uint32_t comb = c1 | (c2 << 8) | (c3 << 16) | ((uint32_t)len << 24);
  return xxph3_avalanche(((uint64_t)comb ^ ((uint64_t)sec32(0) + seed)) * P64_1);
}
// Hash64 of a register value: 1-byte op type, 4-byte CF id, 8-byte seqno
// (db/kv_checksum.h hashes them through their in-memory LE bytes)
__device__ __forceinline__ uint64_t xxph3_u8(uint32_t b, uint64_t seed) { return xxph3_1to3(b, b, b, 1, seed); }
__device__ __forceinline__ uint64_t xxph3_u32(uint32_t x, uint64_t seed) { return xxph3_4to8(x, x, 4, seed); }
__device__ __forceinline__ uint64_t xxph3_u64(uint64_t x, uint64_t seed) {
  return xxph3_4to8((uint32_t)x, (uint32_t)(x >> 32), 8, seed);
}

// XXPH3_64bits_withSeed for n <= 240 (:1086-1147 incl. the RocksDB len-0
// rule, :1655, :1685), one lane.
__device__ __noinline__ uint64_t xxph3_short(const uint8_t* in, uint64_t len, uint64_t seed) {
  if (len <= 16) {
    if (len > 8) {
      const uint64_t lo = rd64(in) ^ (sec64(0) + seed), hi = rd64(in + len - 8) ^ (sec64(8) - seed);
      return xxph3_avalanche(len + (lo + hi) + mul128_fold64(lo, hi));
    }
    if (len >= 4) return xxph3_4to8(rd32(in), rd32(in + len - 4), len, seed);
    if (len) return xxph3_1to3(in[0], in[len >> 1], in[len - 1], len, seed);
    return mul128_fold64(seed + sec64(0), P64_2);
  }
  uint64_t acc = len * P64_1;
  if (len <= 128) {
    if (len > 32) {
      if (len > 64) {
        if (len > 96) {
          acc += xxph3_mix16(in + 48, 96, seed);
          acc += xxph3_mix16(in + len - 64, 112, seed);
        }
        acc += xxph3_mix16(in + 32, 64, seed);
        acc += xxph3_mix16(in + len - 48, 80, seed);
      }
      acc += xxph3_mix16(in + 16, 32, seed);
      acc += xxph3_mix16(in + len - 32, 48, seed);
    }
    acc += xxph3_mix16(in, 0, seed);
    acc += xxph3_mix16(in + len - 16, 16, seed);
    return xxph3_avalanche(acc);
  }
  for (int i = 0; i < 8; i++) acc += xxph3_mix16(in + 16 * i, 16 * i, seed);
  acc = xxph3_avalanche(acc);
  const int rounds = (int)len / 16;
  for (int i = 8; i < rounds; i++) acc += xxph3_mix16(in + 16 * i, 16 * (i - 8) + 3, seed);
  acc += xxph3_mix16(in + len - 16, 136 - 17, seed);
  return xxph3_avalanche(acc);
}

// XXPH3 long loop on ONE lane (:1516-1587 with the seeded secret), for the
// rare long key; values go through the row driver.
__device__ __noinline__ uint64_t xxph3_long_lane(const uint8_t* in, uint64_t len, uint64_t seed) {
  uint64_t acc[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
  const uint64_t nb = len / 1024;
  auto stripe = [&](const uint8_t* p, int soff) {
    for (int l = 0; l < 8; l++) {
      const uint64_t d = rd64(p + 8 * l), k = d ^ csec64(soff + 8 * l, seed);
      acc[l] += d + mul32to64(k);
    }
  };
  for (uint64_t b = 0; b < nb; b++) {
    for (int s2 = 0; s2 < 16; s2++) stripe(in + 1024 * b + 64 * s2, 8 * s2);
    for (int l = 0; l < 8; l++) {
      uint64_t a = acc[l];
      a ^= a >> 47;
      a ^= csec64(128 + 8 * l, seed);
      acc[l] = a * P32_1;
    }
  }
  const int nst = (int)((len - 1024 * nb) / 64);
  for (int s2 = 0; s2 < nst; s2++) stripe(in + 1024 * nb + 64 * s2, 8 * s2);
  if (len & 63) stripe(in + len - 64, 121);
  uint64_t r = len * P64_1;
  for (int l = 0; l < 4; l++)
    r += mul128_fold64(acc[2 * l] ^ csec64(11 + 16 * l, seed), acc[2 * l + 1] ^ csec64(19 + 16 * l, seed));
  return xxph3_avalanche(r);
}

__device__ __forceinline__ uint64_t xxph3_any(const uint8_t* in, uint64_t len, uint64_t seed) {
  return len <= 240 ? xxph3_short(in, len, seed) : xxph3_long_lane(in, len, seed);
}

// 64-bit DPP move (both halves with the same control)
template <int CTRL>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)v, CTRL, 0xF, 0xF, true);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(v >> 32), CTRL, 0xF, 0xF, true);
  return ((uint64_t)hi << 32) | lo;
}
// sum over the 4 lanes of a row with the same (lane & 3): row_ror 4, 8
__device__ __forceinline__ uint64_t row_sum_st4(uint64_t v) {
  v += dpp64<0x124>(v);
  v += dpp64<0x128>(v);
  return v;
}
// sum over the 4 lanes of a quad: quad_perm [1,0,3,2], [2,3,0,1]
__device__ __forceinline__ uint64_t quad_sum(uint64_t v) {
  v += dpp64<0xB1>(v);
  v += dpp64<0x4E>(v);
  return v;
}
__device__ __forceinline__ uint64_t xxh3_scramble(uint64_t a, uint64_t k) {
  a ^= a >> 47;
  a ^= k;
  return a * P32_1;
}

// 16-byte global load at any byte address (full rate at 4-byte alignment)
__device__ __forceinline__ uint4 gload16u(uint64_t addr) { return span_load16<true>(addr); }

// ---- byte-misaligned spans -------------------------------------------------
// A 16-byte load at a byte-misaligned address runs far below rate (SST-shaped
// mix, XXH3: 4.27 TB/s with block starts at any byte, 5.24 at 4-byte-aligned
// starts; uniform 4097-byte stride 3.92 vs 4112-byte 5.13).  So every lane
// loads DWORD-aligned: for the window [a, a + 16) with s = a & 3 (s = 4 when
// a is dword-aligned), U = the 16 bytes at a - s + 4 and D0 = the dword at
// a - s, which is the previous window's U.w -- the neighbouring lane's, taken
// with DPP -- or, at the start of a contiguous run, one extra dword load.
// Then window dword d = bytes s..s+3 of (U[d] : U[d-1]) (v_perm_b32).  Every
// address read lies in the dwords that hold the window's bytes.
typedef __attribute__((address_space(1))) const uint32_t gbl_u32c_t;
__device__ __forceinline__ uint32_t gload4(uint64_t addr) { return *reinterpret_cast<gbl_u32c_t*>(addr); }
__device__ __forceinline__ uint32_t rd_shift(uint64_t ptr) {
  const uint32_t b = (uint32_t)ptr & 3u;
  return b ? b : 4u;
}
__device__ __forceinline__ uint32_t rd_sel(uint32_t s) { return 0x03020100u + s * 0x01010101u; }
__device__ __forceinline__ uint64_t floor4(uint64_t a) { return a & ~3ull; }
__device__ __forceinline__ uint4 rd_fix(const uint4& u, uint32_t d0, uint32_t sel) {
  return make_uint4(__builtin_amdgcn_perm(u.x, d0, sel), __builtin_amdgcn_perm(u.y, u.x, sel),
                    __builtin_amdgcn_perm(u.z, u.y, sel), __builtin_amdgcn_perm(u.w, u.z, sel));
}
// (take DPP results into a variable before any ?: -- clang lowers ?: with
// call operands to branches, and the move would then read masked lanes)
template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
constexpr int kDppRowRor1 = 0x121;   // lane j of a row <- lane j - 1 (mod 16)
constexpr int kDppWaveShr1 = 0x138;  // lane l <- lane l - 1
constexpr int kDppQuadShr1 = 0x90;   // quad_perm [0,0,1,2]: lane q <- lane q - 1

// The row layout (lane j of a 16-lane row reads bytes 16 j of each 256-byte
// chunk k = 0..3 of a 1 KiB segment): previous dword of window (k, j) is
// the U.w of (k, j - 1), of (k - 1, 15) for j = 0, and e0 (the dword before
// the segment) for (0, 0).
__device__ __forceinline__ void rd_fix_row(uint4 (&d)[4], uint32_t e0, int j, uint32_t sel) {
  uint32_t r[4];
#pragma unroll
  for (int k = 0; k < 4; k++) r[k] = dpp32<kDppRowRor1>(d[k].w);
#pragma unroll
  for (int k = 0; k < 4; k++) d[k] = rd_fix(d[k], j ? r[k] : k ? r[k - 1] : e0, sel);
}

// Per-lane constants of the row layout.
struct X3Row {
  uint64_t k0[4], k1[4];  // stripe secrets for accumulators 2q, 2q+1 of stripe st4+4k
  uint64_t ks0, ks1;      // scramble secret (offset 128)
  uint64_t kl0, kl1;      // last-stripe secret (offset 121)
  uint64_t km0, km1;      // merge secret (offset 11)
  uint64_t i0, i1;        // XXH3_INIT_ACC
  uint64_t ko0, ko1;      // wave layout, lone partial segment: stripe lane>>2, pair q
  uint64_t seed;          // XXPH3 seed (0 for XXH3)
  // wave layout: rows 0-1 carry accumulator 2q of the chain, rows 2-3
  // accumulator 2q + 1 (role = lane >> 5), so a scramble instruction
  // advances both accumulators of a pair at once
  uint64_t ksw, iw;       // the role's scramble secret and initial value
  int lane, row, j, q, st4, role;
};
__device__ __forceinline__ X3Row x3_row(uint64_t seed) {
  X3Row X;
  X.lane = threadIdx.x & 63;
  X.row = X.lane >> 4;
  X.j = X.lane & 15;
  X.q = X.j & 3;
  X.st4 = X.j >> 2;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int st = X.st4 + 4 * k;
    X.k0[k] = csec64(8 * st + 16 * X.q, seed);
    X.k1[k] = csec64(8 * st + 16 * X.q + 8, seed);
  }
  X.ks0 = csec64(128 + 16 * X.q, seed);
  X.ks1 = csec64(136 + 16 * X.q, seed);
  X.kl0 = csec64(121 + 16 * X.q, seed);
  X.kl1 = csec64(129 + 16 * X.q, seed);
  X.km0 = csec64(11 + 16 * X.q, seed);
  X.km1 = csec64(19 + 16 * X.q, seed);
  X.ko0 = csec64(8 * (X.lane >> 2) + 16 * X.q, seed);
  X.ko1 = csec64(8 * (X.lane >> 2) + 16 * X.q + 8, seed);
  X.seed = seed;
  // INIT_ACC = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1}
  X.i0 = X.q == 0 ? (uint64_t)P32_3 : X.q == 1 ? P64_2 : X.q == 2 ? P64_4 : P64_5;
  X.i1 = X.q == 0 ? P64_1 : X.q == 1 ? P64_3 : X.q == 2 ? (uint64_t)P32_2 : (uint64_t)P32_1;
  X.role = X.lane >> 5;
  X.ksw = X.role ? X.ks1 : X.ks0;
  X.iw = X.role ? X.i1 : X.i0;
  return X;
}

// ---- short spans (n <= 240) on 16-lane rows (round 6) ---------------------
// XXH3_64bits and XXPH3 for 17 <= n <= 240 (util/xxhash.h:4060-4130,
// util/xxph3.h:1112-1147) are sums of independent mix16 terms -- a 16-byte
// window of the input against a 16-byte secret window -- under one or two
// avalanches.  Lane j of a row takes one window:
//   n <= 128: m = ceil(n / 32) pairs; lanes j < m the front windows 16 j
//     (secret 32 j), lanes 8 <= j < 8 + m the back windows n - 16 (j - 7)
//     (secret 32 (j - 8) + 16); h = avalanche(n P1 + sum of all)
//   n > 128: lanes j < 8 the windows 16 j (secret 16 j): S0; lanes
//     8 <= j < n / 16 the windows 16 j (secret 16 (j - 8) + 3) and lane 15
//     the last window n - 16 (secret 119): S1;
//     h = avalanche(avalanche(n P1 + S0) + S1)
// S0 and S1 sit in the two half-rows in both classes, so one 3-step half-row
// sum and one row_ror 8 give both.  A row hashes a short span with one
// coalesced 16-byte load per lane where one lane used to walk up to 15
// windows alone while its wave waited.  n <= 16 (one or two loads, the
// small classes): lane 0 of the row, as before.
struct X3Short {
  uint64_t a0, a1;  // lane j's secret words for n <= 128
  uint64_t b0, b1;  // ... for n > 128
};
// (the short classes key mix16 with secret + seed / secret - seed,
// util/xxph3.h:1644 -- not the custom secret of the long loop; seed 0 for XXH3)
__device__ __forceinline__ X3Short x3s_keys(uint32_t j, uint64_t seed) {
  const int sa = 32 * (int)(j & 3u) + (j < 8 ? 0 : 16);
  const int sb = j < 8 ? 16 * (int)j : j < 15 ? 16 * (int)(j - 8) + 3 : 119;
  X3Short K;
  K.a0 = sec64(sa) + seed;
  K.a1 = sec64(sa + 8) - seed;
  K.b0 = sec64(sb) + seed;
  K.b1 = sec64(sb + 8) - seed;
  return K;
}
// The 16 bytes at any byte address from dword-aligned loads (a 16-byte
// load at a byte-misaligned address runs far below rate): the dwords at
// a & ~3 and the next one, funnel-shifted.  Reads at most 3 bytes past
// a + 16, inside the dword holding byte a + 15 (s = 0: the last dword of the
// window again).
__device__ __forceinline__ uint4 load16_realign(uint64_t a) {
  const uint64_t a4 = a & ~3ull;
  const uint32_t s = (uint32_t)a & 3u;
  const uint4 u = span_load16<false>(a4);
  const uint32_t e = gload4(a4 + (s ? 16u : 12u));
  return make_uint4(__builtin_amdgcn_alignbyte(u.y, u.x, s), __builtin_amdgcn_alignbyte(u.z, u.y, s),
                    __builtin_amdgcn_alignbyte(u.w, u.z, s), __builtin_amdgcn_alignbyte(e, u.w, s));
}
// lane j's window offset in a span of 17 <= n <= 240 bytes, and whether the
// lane has one
__device__ __forceinline__ uint32_t x3s_off(uint32_t n, uint32_t j, bool& has) {
  if (n <= 128) {
    has = (j & 7u) < ((n + 31) >> 5);
    return j < 8 ? 16 * j : n - 16 * (j - 7);
  }
  has = j < 8 || j < (n >> 4) || j == 15;
  return j == 15 ? n - 16 : 16 * j;
}
// the small classes (n <= 16) of XXH3 / XXPH3, one lane
template <bool PREVIEW>
__device__ __forceinline__ uint64_t x3_small(const uint8_t* in, uint64_t len, uint64_t seed) {
  if constexpr (PREVIEW) {
    if (len > 8) {
      const uint64_t lo = rd64(in) ^ (sec64(0) + seed), hi = rd64(in + len - 8) ^ (sec64(8) - seed);
      return xxph3_avalanche(len + (lo + hi) + mul128_fold64(lo, hi));
    }
    if (len >= 4) return xxph3_4to8(rd32(in), rd32(in + len - 4), len, seed);
    if (len) return xxph3_1to3(in[0], in[len >> 1], in[len - 1], len, seed);
    return mul128_fold64(seed + sec64(0), P64_2);
  } else {
    if (len > 8) {
      const uint64_t bf1 = sec64(24) ^ sec64(32), bf2 = sec64(40) ^ sec64(48);
      const uint64_t lo = rd64(in) ^ bf1, hi = rd64(in + len - 8) ^ bf2;
      return xxh3_avalanche(len + __builtin_bswap64(lo) + hi + mul128_fold64(lo, hi));
    }
    if (len >= 4) {
      const uint64_t in1 = rd32(in), in2 = rd32(in + len - 4);
      const uint64_t bf = sec64(8) ^ sec64(16);
      return xxh3_rrmxmx((in2 + (in1 << 32)) ^ bf, len);
    }
    if (len) {
      const uint32_t c1 = in[0], c2 = in[len >> 1], c3 = in[len - 1];
      const uint32_t comb = (c1 << 16) | (c2 << 24) | c3 | ((uint32_t)len << 8);
      return xxh64_avalanche((uint64_t)comb ^ (uint64_t)(sec32(0) ^ sec32(4)));
    }
    return xxh64_avalanche(sec64(56) ^ sec64(64));
  }
}
// The row's hash of a 17..240-byte span from lane j's window d (has: the
// lane holds one); valid in lanes 0-7 of the row.  Every lane of the row
// must be active (DPP).
template <bool PREVIEW>
__device__ __forceinline__ uint64_t x3s_row_hash(uint32_t n, const uint4& d, bool has, const X3Short& K) {
  const bool mid = n <= 128;
  const uint64_t lo = ((uint64_t)d.y << 32) | d.x, hi = ((uint64_t)d.w << 32) | d.z;
  const uint64_t v = has ? mul128_fold64(lo ^ (mid ? K.a0 : K.b0), hi ^ (mid ? K.a1 : K.b1)) : 0ull;
  uint64_t t = quad_sum(v);
  t += dpp64<0x141>(t);                      // half mirror: the half-row's sum
  const uint64_t u = dpp64<0x128>(t);        // row_ror 8: the other half's
  const uint64_t a = (uint64_t)n * P64_1 + t;
  if constexpr (PREVIEW) return mid ? xxph3_avalanche(a + u) : xxph3_avalanche(xxph3_avalanche(a) + u);
  else return mid ? xxh3_avalanche(a + u) : xxh3_avalanche(xxh3_avalanche(a) + u);
}

// A row's span of n <= 240 bytes at ptr, called by the row's 16 lanes
// together: its hash in lane 0 (out of line: the row loops that meet an
// occasional short span keep their registers -- inlined, per-KV protection's
// verify kernel went from 128 to 144 VGPRs)
template <bool PREVIEW>
__device__ __noinline__ uint64_t x3s_hash_row(uint64_t ptr, uint64_t n, uint64_t seed) {
  const uint32_t j = threadIdx.x & 15u;
  bool has;
  const uint32_t o = x3s_off((uint32_t)n, j, has);
  has = has && n > 16;
  const uint4 d = load16_realign(has ? ptr + o : ptr & ~15ull);
  const uint64_t h = x3s_row_hash<PREVIEW>((uint32_t)n, d, has, x3s_keys(j, seed));
  return n <= 16 && j == 0 ? x3_small<PREVIEW>(reinterpret_cast<const uint8_t*>(ptr), n, seed) : h;
}

// Every short span (n <= 240) among slots t0, t0 + rows, ... < n of a row,
// U spans per row in flight, the next group's descriptors loaded while the
// current one is hashed.  slot(t, &len, &off) -> span index.  Lane u of the
// row finishes span u of a group (U <= 8).  Wave-uniform: every lane calls
// it with the same n and rows.
// (kl: the 16 lanes' keys in LDS, read where they are used -- the caller's
// row-loop constants stay live across this pass; nullptr: in registers)
// (KLDS is a template flag, not a null test: a runtime choice between the
// LDS keys and a register copy had the compiler take the copy's address --
// a scratch store of 32 bytes per lane per iteration, WRITE 4.6 x the
// outputs at 100-300 B)
template <class Op, bool PREVIEW, int U, bool KLDS = false, class Slot>
__device__ __forceinline__ void x3_short_rows(const Op& op, uint32_t t0, uint32_t n, uint32_t rows, uint64_t seed,
                                              Slot&& slot, const X3Short* kl = nullptr) {
  static_assert(U <= 8, "lanes 0-7 hold the hashes");
  if (n == 0) return;
  const uint32_t j = threadIdx.x & 15u;
  X3Short Kr{};
  if constexpr (!KLDS) Kr = x3s_keys(j, seed);
  const uint64_t base = reinterpret_cast<uint64_t>(op.base());
  uint32_t len[U], idx[U];
  uint64_t off[U];
  auto fetch = [&](uint32_t t) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t tt = t + rows * (uint32_t)u;
      idx[u] = slot(tt < n ? tt : n - 1, len[u], off[u]);
      len[u] = tt < n ? len[u] : 0xFFFFFFFFu;  // past the slots: not short
    }
  };
  fetch(t0);
  for (uint32_t t = t0; __any(t < n); t += rows * U) {
    bool sh[U], has[U];
    uint4 d[U];
    uint32_t ln[U], ix[U];
    uint64_t ptr[U];
    bool any = false;
#pragma unroll
    for (int u = 0; u < U; u++) {
      ln[u] = len[u];
      ix[u] = idx[u];
      ptr[u] = base + off[u];
      sh[u] = ln[u] <= 240u;
      any |= sh[u];
    }
    if (__any(any)) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t o = x3s_off(ln[u], j, has[u]);
        has[u] = has[u] && sh[u] && ln[u] > 16u;
        d[u] = load16_realign(has[u] ? ptr[u] + o : ptr[u] & ~15ull);  // (idle: the span's 16-byte line)
      }
    }
    fetch(t + rows * U);  // (past n: clamped slots, flagged not short)
    if (__any(any)) {
      X3Short K;
      if constexpr (KLDS)
        K = kl[j];
      else
        K = Kr;
#pragma unroll
      for (int u = 0; u < U; u++) {
        uint64_t h = x3s_row_hash<PREVIEW>(ln[u], d[u], has[u], K);
        if (sh[u] && ln[u] <= 16u && j == (uint32_t)u)
          h = x3_small<PREVIEW>(reinterpret_cast<const uint8_t*>(ptr[u]), ln[u], seed);
        if (sh[u] && j == (uint32_t)u) op.finish(ix[u], h);
      }
    }
  }
}

// One row's span in progress.
struct X3Span {
  uint64_t ptr, len;
  uint32_t nb;   // full segments: (len - 1) / 1024 (XXPH3: len / 1024)
  uint32_t nst;  // stripes in the last, partial segment
  uint32_t g;    // segment being processed
  uint32_t i;    // span index
  bool tail;     // last stripe at len - 64 (XXPH3: only if len % 64)
  // XXH3: the descriptor of span pi (hlen, off), loaded when span i started
  // (x3_next_long)
  uint64_t pl = 0, po = 0;
  uint32_t pi = ~0u;
};

// A row's long span (n > 240) from its start.
template <bool PREVIEW>
__device__ __forceinline__ void x3_span_start(X3Span& rs, uint64_t ptr, uint64_t len, uint32_t i) {
  rs.ptr = ptr;
  rs.len = len;
  // XXH3 util/xxhash.h:5141-5171; XXPH3 util/xxph3.h:1516-1543
  const uint64_t body = PREVIEW ? len : len - 1;
  rs.nb = (uint32_t)(body / 1024);
  rs.nst = (uint32_t)((body - 1024ull * rs.nb) / 64);
  rs.tail = PREVIEW ? (len & 63) != 0 : true;
  rs.g = 0;
  rs.i = i;
}

// Advance the row to its next long span (hashing short ones -- n <= 240 --
// on the row's first lane on the way).  Op: base(), off(i), hlen(i),
// finish(i, h) (called by lane j == 0 of the row).  Returns false when the
// row has no spans left.
// (SKIP_SHORT: the caller already hashed the short spans, one per lane)
template <class Op, bool PREVIEW, bool SKIP_SHORT = false>
__device__ __forceinline__ bool x3_next_long(const Op& op, uint32_t i, uint32_t count, uint32_t stride,
                                             const X3Row& X, X3Span& rs) {
  const uint64_t base = reinterpret_cast<uint64_t>(op.base());
  for (; i < count; i += stride) {
    // XXH3 (ragged batches: a descriptor is two dependent loads before the
    // span's data loads): the next span's descriptor was loaded when this
    // one started, so it arrives while the span is hashed.  (Not for XXPH3:
    // per-KV protection's verify op sits at 128 VGPRs, 4 waves per SIMD.)
    const bool pf = !PREVIEW && i == rs.pi;
    const uint64_t len = pf ? rs.pl : op.hlen(i);
    const uint64_t ptr = base + (pf ? rs.po : op.off(i));
    if (len > 240) {
      if constexpr (!PREVIEW) {
        const uint32_t ni = i + stride, pj = ni < count ? ni : i;  // (unconditional loads)
        rs.pi = ni;
        rs.pl = op.hlen(pj);
        rs.po = op.off(pj);
      }
      x3_span_start<PREVIEW>(rs, ptr, len, i);
      return true;
    }
    if constexpr (!SKIP_SHORT) {
      if constexpr (PREVIEW) {
        // XXPH3 (k_xph3): lane 0 of the row -- short values are rare there,
        // and the row call cost per-KV protection's verify kernel its fourth
        // wave per SIMD (128 -> 130 VGPRs)
        if (X.j == 0) op.finish(i, xxph3_short(reinterpret_cast<const uint8_t*>(ptr), len, X.seed));
      } else {  // the whole row: one window per lane
        const uint64_t h = x3s_hash_row<false>(ptr, len, 0);
        if (X.j == 0) op.finish(i, h);
      }
    }
  }
  return false;
}

// PREVIEW = XXPH3 (Hash64 with `seed`), else XXH3_64bits v0.8.1 (seed 0).
//
// Epilogues are batched: a row's finished span
// parks (index, hash) in lane `slot` of the row, and every 16 spans the 16
// lanes run op.finish together -- its epilogue loads (op.pre) included --
// instead of lane 0 running one finish (and every iteration carrying the
// span's epilogue inputs in registers) per span.  For the per-KV protection
// epilogue (key, op type and seqno hashes) that is most of a ~1 KiB span's
// non-data VALU work.
// The row loop: each row walks its span segment by segment; next_span(rs)
// moves a row whose span ended to its next long one (false: none left).
template <class Op, bool PREVIEW, bool NT, class Next>
__device__ __forceinline__ void xxh3_rows_loop_p(const Op& op, const X3Row& X, X3Span& rs, bool act,
                                                 Next&& next_span) {
  uint64_t a0 = X.i0, a1 = X.i1;
  uint32_t slot = 0, si = 0;
  uint64_t shv = 0;
  bool sv = false;
  // the raw last dword (d[3].w) of each lane's previous segment: lane 15's is
  // the dword before the row's next segment (e0 below)
  uint32_t pw = 0;
  while (__any(act)) {
    // loads first and unconditional (clamped when a stripe is not part of
    // the segment, or the row is idle), so they are counted and in flight
    const uint64_t seg = rs.ptr + 1024ull * rs.g;
    const bool full = rs.g < rs.nb;
    // dword-aligned loads (see rd_fix); lanes without work read the span's
    // first dwords
    const uint32_t sh = rd_shift(rs.ptr), sel = rd_sel(sh);
    const uint64_t idle = floor4(rs.ptr);
    uint4 d[4];
    bool ok[4];
#pragma unroll
    for (int k = 0; k < 4; k++) ok[k] = act && (full || (uint32_t)(X.st4 + 4 * k) < rs.nst);
    const uint64_t sb = seg + 64 * X.st4 + 16 * X.q - sh + 4;  // + 256 k
    const uint64_t lst = rs.ptr + rs.len - 64;  // last stripe: its own byte offset
    const uint32_t shl = rd_shift(lst);
    // the last stripe is used only in the span's last segment: before that
    // the load (unconditional, for the vmcnt count) reads the segment's own
    // first stripe, whose line this iteration fetches anyway -- re-reading
    // the span's last 64 bytes in every segment cost ~6 % extra HBM reads
    // at 4 KiB (PMC traffic 1.09x, non-temporal loads do not keep the line)
    // a last segment holding no stripe (len just past a segment multiple)
    // is finished in the iteration of the full segment before it: the last
    // stripe is loaded here and merged after the scramble (one iteration
    // per span instead of two at 1025-1088 bytes)
    const bool fin = full && rs.g + 1 == rs.nb && rs.nst == 0;
    const bool lastseg = !full || fin;
    const uint64_t lsa = act ? (lastseg ? lst + 16 * X.q - shl + 4 : seg + 16 * X.q - sh + 4) : idle;
#pragma unroll
    for (int k = 0; k < 4; k++) d[k] = span_load16<NT>(ok[k] ? sb + 256 * k : idle);
    uint4 dl = span_load16<NT>(lsa);
    // the dword before the segment: loaded only at the span's first segment;
    // later it is the previous segment's last dword, already in lane 15's
    // registers -- re-reading it fetched that line again (non-temporal loads
    // do not keep it): PMC traffic 1.107x at 4 KiB
    // (XXH3 only: the XXPH3 users -- per-KV protection, ~1 KiB spans of one
    // segment -- would pay the register for nothing: OpKvProtect<true> went
    // from 128 to 130 VGPRs, 4 -> 3 waves per SIMD, -6 %)
    uint32_t e0p = 0;
    if constexpr (!PREVIEW) {
      e0p = dpp32<kDppRowRor1>(pw);  // lane 0 of the row (the one user) <- lane 15
      pw = d[3].w;
    }
    // Realignment only while some active row's span (or its last stripe)
    // is not dword-aligned (wave-uniform branch): for an aligned one rd_fix
    // is the identity, and its two dword loads, 20 v_perm and 5 DPP moves
    // per iteration are skipped (profiles/r5/x3_align/).
    if (__any(act && (((uint32_t)rs.ptr | (uint32_t)rs.len) & 3u) != 0)) {
      uint32_t e0;
      if constexpr (!PREVIEW) {
        const uint32_t e0l = gload4(act && rs.g == 0 && seg - sh >= idle ? seg - sh : act ? seg - sh + 4 : idle);
        e0 = rs.g ? e0p : e0l;
      } else {
        e0 = gload4(act && seg - sh >= idle ? seg - sh : idle);
      }
      const uint32_t el = gload4(act ? (lastseg ? lst - shl : seg - sh + 4) : idle);
      rd_fix_row(d, e0, X.j, sel);
      const uint32_t pl = dpp32<kDppQuadShr1>(dl.w);  // unconditional in the branch: see x3w_fold
      dl = rd_fix(dl, X.q ? pl : el, rd_sel(shl));
    }
    uint64_t c0 = 0, c1 = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint64_t d0 = ((uint64_t)d[k].y << 32) | d[k].x, d1 = ((uint64_t)d[k].w << 32) | d[k].z;
      // v0.8.1 adds the data word to the neighbouring accumulator
      // (acc[l ^ 1]); the preview adds it to its own (acc_64bits)
      c0 += ok[k] ? (PREVIEW ? d0 : d1) + mul32to64(d0 ^ X.k0[k]) : 0;
      c1 += ok[k] ? (PREVIEW ? d1 : d0) + mul32to64(d1 ^ X.k1[k]) : 0;
    }
    a0 += row_sum_st4(c0);
    a1 += row_sum_st4(c1);
    if (full) {
      a0 = xxh3_scramble(a0, X.ks0);
      a1 = xxh3_scramble(a1, X.ks1);
      rs.g++;
    }
    if (act && lastseg) {  // last (partial) segment done: last stripe, merge, next span
      const uint64_t l0 = ((uint64_t)dl.y << 32) | dl.x, l1 = ((uint64_t)dl.w << 32) | dl.z;
      if (rs.tail) {
        a0 += (PREVIEW ? l0 : l1) + mul32to64(l0 ^ X.kl0);
        a1 += (PREVIEW ? l1 : l0) + mul32to64(l1 ^ X.kl1);
      }
      const uint64_t m = quad_sum(mul128_fold64(a0 ^ X.km0, a1 ^ X.km1));
      const uint64_t h = PREVIEW ? xxph3_avalanche(rs.len * P64_1 + m) : xxh3_avalanche(rs.len * P64_1 + m);
      if ((uint32_t)X.j == slot) {
        si = rs.i;
        shv = h;
        sv = true;
      }
      if (++slot == 16) {
        if (sv) op.finish(si, shv);
        sv = false;
        slot = 0;
      }
      act = next_span(rs);
      a0 = X.i0;
      a1 = X.i1;
    }
  }
  if (sv) op.finish(si, shv);
}
// Non-temporal loads only for waves whose first spans are all 16-byte
// aligned: a misaligned segment's 256-byte chunks share their boundary lines
// with the next chunk's load instruction, which non-temporal loads do not
// keep (1000-byte spans at 8-byte alignment: 0.621 of peak with
// non-temporal loads, 0.705 without; aligned 1 KiB spans 0.760 with, 0.712
// without -- profiles/r5/x3_align/).  Chosen once per wave from the rows'
// first spans (a per-iteration choice would need both load sets in the
// loop, and the compiler merges them into one without the policy).
template <class Op, bool PREVIEW, class Next>
__device__ __forceinline__ void xxh3_rows_loop(const Op& op, const X3Row& X, X3Span& rs, bool act,
                                               Next&& next_span) {
  if (!__any(act && ((uint32_t)rs.ptr & 15u) != 0))  // wave-uniform
    xxh3_rows_loop_p<Op, PREVIEW, true>(op, X, rs, act, next_span);
  else
    xxh3_rows_loop_p<Op, PREVIEW, false>(op, X, rs, act, next_span);
}

template <class Op, bool PREVIEW = false>
__device__ __forceinline__ void xxh3_rows_driver(const Op& op, uint32_t count, uint64_t seed = 0) {
  const X3Row X = x3_row(seed);
  const uint32_t wpb = blockDim.x >> 6;
  const uint32_t stride = gridDim.x * wpb * 4;  // rows in the grid
  const uint32_t first = (blockIdx.x * wpb + (threadIdx.x >> 6)) * 4 + X.row;
  // idle rows keep loading from a valid address: the batch's base
  X3Span rs{reinterpret_cast<uint64_t>(op.base()), 0, 0, 0, 0, 0, false};
  const bool act = x3_next_long<Op, PREVIEW>(op, first, count, stride, X, rs);
  xxh3_rows_loop<Op, PREVIEW>(op, X, rs, act, [&](X3Span& r) {
    return x3_next_long<Op, PREVIEW>(op, r.i + stride, count, stride, X, r);
  });
}


// ---- XXH3 / XXPH3, one WAVE per span ---------------------------------------
// For batches of KiB-sized blocks (SST): spans are dealt to waves like the
// CRC engine, so a long span is not serialised on one 16-lane row and a
// ragged batch balances over 4x fewer, 4x faster workers.
// Round k: row r folds segment g = 4k + r (4 x 16-byte loads per lane: the
// wave reads 4 KiB contiguous).  A segment's stripe sums C_g do not depend
// on the accumulators -- only the scramble between segments is sequential --
// so after the in-row reduction row 0 gathers the four rows' C_g for its
// accumulator pair q (v_permlane16/32_swap) and runs acc = scramble(acc +
// C_g) over the round's segments; segment nb is the partial one (no
// scramble).  When it would be alone in a round it is spread over all 64
// lanes (stripe = lane / 4) instead.  Then the last stripe and the merge.
// value of lane ^ 16 / lane ^ 32 (gfx950 v_permlane16/32_swap: with both
// operands = v, one result is v itself and the other the partner row's value)
__device__ __forceinline__ uint32_t xl16(uint32_t v) {
  const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  return xor3(r[0], r[1], v);
}
__device__ __forceinline__ uint32_t xl32(uint32_t v) {
  const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return xor3(r[0], r[1], v);
}
__device__ __forceinline__ uint64_t xl16_64(uint64_t v) {
  return ((uint64_t)xl16((uint32_t)(v >> 32)) << 32) | xl16((uint32_t)v);
}
__device__ __forceinline__ uint64_t xl32_64(uint64_t v) {
  return ((uint64_t)xl32((uint32_t)(v >> 32)) << 32) | xl32((uint32_t)v);
}

// Workgroup b (1024 threads) owns spans b, b + G, ... (interleaved over the
// batch).  When its share fits, the descriptors are staged in LDS and each
// wave takes the next span with an LDS ticket as it frees up (balanced
// inside the CU); otherwise the waves walk the share round-robin.
constexpr uint32_t kX3DescCache = 1024;

// One span on the wave, cut into "units": unit k < rounds is round k (four
// segments, one per row); the last unit (k = units - 1) also carries the
// lone partial segment (spread over the wave) and the last stripe.  Every
// unit issues the same loads per lane -- six dword-aligned 16-byte loads and
// three dwords for the realignment (rd_fix), clamped to the span's first
// dwords where a load has no work -- all before any is used, so a unit costs
// one HBM round trip (the next unit is not prefetched).
struct X3WSpan {
  uint64_t ptr, len;
  uint32_t i;       // span index
  uint32_t nb;      // full segments
  uint32_t nst;     // stripes in the partial segment nb
  uint32_t rounds;  // four-segment rounds
  uint32_t units;   // max(rounds, 1)
  bool lone;        // segment nb is folded by the whole wave in the last unit
  bool tail;        // last stripe at len - 64
};
template <bool PREVIEW>
__device__ __forceinline__ X3WSpan x3w_span(uint64_t ptr, uint64_t len, uint32_t i) {
  X3WSpan sp;
  sp.ptr = ptr;
  sp.len = len;
  sp.i = i;
  // XXH3 util/xxhash.h:5141-5171; XXPH3 util/xxph3.h:1516-1543
  const uint64_t body = PREVIEW ? len : len - 1;
  sp.nb = (uint32_t)(body / 1024);
  sp.nst = (uint32_t)((body - 1024ull * sp.nb) / 64);
  sp.tail = PREVIEW ? (len & 63) != 0 : true;
  // when the last round would hold only the partial segment nb, it is
  // spread over the whole wave instead
  sp.lone = (sp.nb & 3) == 0;
  sp.rounds = sp.nb / 4 + (sp.lone ? 0 : 1);
  sp.units = sp.rounds ? sp.rounds : 1;
  return sp;
}
struct X3WLoads {
  uint4 d[4];  // round part: stripes st4 + 4m of segment 4k + row, pair q
  uint4 v;     // lone partial segment: stripe lane / 4, pair q
  uint4 dl;    // last stripe (len - 64), pair q
  uint32_t e0, ev, el;  // the dwords before the row's segment, the lone segment, the last stripe
};
__device__ __forceinline__ bool x3w_ok(const X3WSpan& sp, uint32_t k, uint32_t g, uint32_t st) {
  return k < sp.rounds && (g < sp.nb || (g == sp.nb && st < sp.nst));
}
// (dword-aligned loads, realigned in x3w_fold: see rd_fix; loads without
// work read the span's first dwords)
// (NT = false: the default cache policy, for a fused kernel that re-reads
// bytes another load of the same wave just brought into L2)
template <bool NT = true>
__device__ __forceinline__ X3WLoads x3w_load(const X3WSpan& sp, uint32_t k, const X3Row& X) {
  X3WLoads L;
  const uint32_t g = 4 * k + X.row;
  const uint64_t seg = sp.ptr + 1024ull * g;
  const uint32_t sh = rd_shift(sp.ptr);
  const uint64_t idle = floor4(sp.ptr);
#pragma unroll
  for (int m = 0; m < 4; m++) {
    const uint32_t st = (uint32_t)(X.st4 + 4 * m);
    L.d[m] = span_load16<NT>(x3w_ok(sp, k, g, st) ? seg + 64 * st + 16 * X.q - sh + 4 : idle);
  }
  const bool last = k + 1 == sp.units;
  const bool okl = last && sp.lone && (uint32_t)(X.lane >> 2) < sp.nst;
  const uint64_t lone = sp.ptr + 1024ull * sp.nb, lst = sp.ptr + sp.len - 64;
  L.v = span_load16<NT>(okl ? lone + 16 * X.lane - sh + 4 : idle);
  const uint32_t shl = rd_shift(lst);  // the last stripe's own byte offset
  L.dl = span_load16<NT>(last ? lst + 16 * X.q - shl + 4 : idle);
  // the realignment dwords only for a span that needs them (x3w_fold skips
  // rd_fix for dword-aligned spans and last stripes; wave-uniform branch)
  L.e0 = L.ev = L.el = 0;
  if (((uint32_t)sp.ptr | (uint32_t)sp.len) & 3u) {
    L.e0 = gload4(x3w_ok(sp, k, g, 0) && g ? seg - sh : idle);
    L.ev = gload4(okl && sp.nb ? lone - sh : idle);
    L.el = gload4(last ? lst - shl : idle);
  }
  return L;
}

// Fold unit k of the span into the lane's accumulator a (accumulator 2q in
// rows 0-1, 2q + 1 in rows 2-3: X.role); after the last unit, merge, finish
// and reset it.  tx: the wave's 1 KiB LDS buffer (free: the parked sums are
// chained).
template <class Op, bool PREVIEW>
__device__ __forceinline__ void x3w_fold(const Op& op, const X3WSpan& sp, uint32_t k, X3WLoads L,
                                         const X3Row& X, uint64_t& a, const typename Op::Pre& e, uint64_t* tx) {
  const uint32_t sel = rd_sel(rd_shift(sp.ptr));
  const bool r1 = X.role != 0;
  if (k < sp.rounds) {  // wave-uniform
    const uint32_t g = 4 * k + X.row;
    if (sp.ptr & 3) rd_fix_row(L.d, L.e0, X.j, sel);  // wave-uniform: dword-aligned spans need no fix
    uint64_t c0 = 0, c1 = 0;
#pragma unroll
    for (int m = 0; m < 4; m++) {
      const bool ok = x3w_ok(sp, k, g, (uint32_t)(X.st4 + 4 * m));
      const uint64_t d0 = ((uint64_t)L.d[m].y << 32) | L.d[m].x, d1 = ((uint64_t)L.d[m].w << 32) | L.d[m].z;
      // v0.8.1 adds the data word to the neighbouring accumulator
      // (acc[l ^ 1]); the preview adds it to its own (acc_64bits)
      c0 += ok ? (PREVIEW ? d0 : d1) + mul32to64(d0 ^ X.k0[m]) : 0;
      c1 += ok ? (PREVIEW ? d1 : d0) + mul32to64(d1 ^ X.k1[m]) : 0;
    }
    c0 = row_sum_st4(c0);
    c1 = row_sum_st4(c1);
    // Rows 0 (role 0) and 2 (role 1) gather the four rows' sums of their
    // accumulator in segment order, through LDS (tx[role][q][row]: one
    // 8-byte store per row and accumulator, two 16-byte reads -- the
    // v_permlane16/32 transposes cost ~30 VALU a unit); rows 1 and 3 compute
    // an unused chain.
    if (X.st4 == 0) {
      tx[4 * X.q + X.row] = c0;
      tx[64 + 4 * X.q + X.row] = c1;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    const ulonglong2* tr = reinterpret_cast<const ulonglong2*>(tx + 64 * X.role + 4 * X.q);
    const ulonglong2 t01 = tr[0], t23 = tr[1];
    const uint64_t T[4] = {t01.x, t01.y, t23.x, t23.y};
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const uint32_t gr = 4 * k + r;
      if (gr > sp.nb) break;  // wave-uniform
      a += T[r];
      if (gr < sp.nb) a = xxh3_scramble(a, X.ksw);
    }
  }
  if (k + 1 < sp.units) return;  // wave-uniform
  if (sp.lone) {  // segment nb alone: lane = stripe * 4 + pair
    const bool okl = (uint32_t)(X.lane >> 2) < sp.nst;
    uint4 v = L.v;
    if (sp.ptr & 3) {  // wave-uniform
      // (DPP result taken before the ?: -- inside it the move would run
      // with the source lanes masked off)
      const uint32_t pv = dpp32<kDppWaveShr1>(L.v.w);
      v = rd_fix(L.v, X.lane ? pv : L.ev, sel);
    }
    const uint64_t d0 = ((uint64_t)v.y << 32) | v.x, d1 = ((uint64_t)v.w << 32) | v.z;
    uint64_t c0 = okl ? (PREVIEW ? d0 : d1) + mul32to64(d0 ^ X.ko0) : 0;
    uint64_t c1 = okl ? (PREVIEW ? d1 : d0) + mul32to64(d1 ^ X.ko1) : 0;
    c0 = row_sum_st4(c0);
    c1 = row_sum_st4(c1);
    c0 += xl16_64(c0);
    c1 += xl16_64(c1);
    c0 += xl32_64(c0);  // the wave's sum, in every lane
    c1 += xl32_64(c1);
    a += r1 ? c1 : c0;
  }
  uint4 dl = L.dl;
  if ((sp.ptr + sp.len) & 3) {  // wave-uniform: the last stripe's own alignment
    const uint32_t pl = dpp32<kDppQuadShr1>(L.dl.w);
    dl = rd_fix(L.dl, X.q ? pl : L.el, rd_sel(rd_shift(sp.ptr + sp.len - 64)));
  }
  const uint64_t l0 = ((uint64_t)dl.y << 32) | dl.x, l1 = ((uint64_t)dl.w << 32) | dl.z;
  if (sp.tail) {  // the role's word and secret
    const uint64_t lw = r1 ? l1 : l0, lo = r1 ? l0 : l1;
    a += (PREVIEW ? lw : lo) + mul32to64(lw ^ (r1 ? X.kl1 : X.kl0));
  }
  // row 0's lanes take accumulator 2q + 1 from row 2 (lane ^ 32)
  const uint64_t b = xl32_64(a);
  const uint64_t m = quad_sum(mul128_fold64(a ^ X.km0, b ^ X.km1));
  const uint64_t h = PREVIEW ? xxph3_avalanche(sp.len * P64_1 + m) : xxh3_avalanche(sp.len * P64_1 + m);
  if (X.lane == 0) op.finish(sp.i, h, e);
  a = X.iw;
}

// Every unit issues all its loads -- the four round loads, the lone partial
// segment, the last stripe and the epilogue inputs -- before any is used, so
// a span of up to 4 KiB + 1 segment costs ONE memory round trip (the
// unpipelined loads of round, lone segment, last stripe and the epilogue's
// dependent descriptor/trailer reads were four).  Latency across units is
// hidden by the other waves (16 per CU); prefetching the next unit in
// registers as well needs ~150 VGPRs, and at 3 waves per SIMD measured
// slower (4.07 vs 4.91 TB/s on the SST-shaped mix).
// An interior unit (k + 1 < units) is always a full round -- segments 4k ..
// 4k + 3 all full (k < rounds - 1 <= nb / 4 - 1) -- so it needs no clamped
// addresses, no per-stripe masks, no lone-segment / last-stripe / epilogue
// loads: four 16-byte loads at one base + 256 B immediates (+ the dword
// before the row's segment when the span is byte-misaligned) and the fold.
// x3w_round_sums: the round's segment sums (row r's lanes: segment 4k + r,
// their accumulator pair q).
struct X3RoundLoads {
  uint4 d[4];
  uint32_t e0;  // the dword before the row's segment (byte-misaligned spans)
};
template <bool NT = true>
__device__ __forceinline__ X3RoundLoads x3w_round_load(const X3WSpan& sp, uint32_t k, const X3Row& X) {
  X3RoundLoads R;
  const uint32_t sh = rd_shift(sp.ptr);
  const uint64_t seg = sp.ptr + 1024ull * (4 * k + X.row);
  const uint64_t a = seg + 64 * X.st4 + 16 * X.q - sh + 4;
#pragma unroll
  for (int m = 0; m < 4; m++) R.d[m] = span_load16<NT>(a + 256 * m);
  // (rd_shift is 4, not 0, for a dword-aligned span: seg - 4 could lie
  // before the buffer)
  R.e0 = (sp.ptr & 3) ? gload4(seg - sh) : 0u;  // wave-uniform
  return R;
}
template <bool PREVIEW>
__device__ __forceinline__ void x3w_round_sums(const X3WSpan& sp, X3RoundLoads R, const X3Row& X, uint64_t& c0,
                                               uint64_t& c1) {
  uint4(&d)[4] = R.d;
  if (sp.ptr & 3) rd_fix_row(d, R.e0, X.j, rd_sel(rd_shift(sp.ptr)));  // wave-uniform
  c0 = 0;
  c1 = 0;
#pragma unroll
  for (int m = 0; m < 4; m++) {
    const uint64_t d0 = ((uint64_t)d[m].y << 32) | d[m].x, d1 = ((uint64_t)d[m].w << 32) | d[m].z;
    c0 += (PREVIEW ? d0 : d1) + mul32to64(d0 ^ X.k0[m]);
    c1 += (PREVIEW ? d1 : d0) + mul32to64(d1 ^ X.k1[m]);
  }
  c0 = row_sum_st4(c0);  // segment 4k + row's sums, in every lane of the row
  c1 = row_sum_st4(c1);
}

// ---- long spans in pieces (round 3) -----------------------------------------
// A span of more than kX3PieceRounds rounds (16 KiB) no longer runs on one
// wave, round after dependent round -- at the end of a launch the last 64 KiB
// spans' 16 sequential round trips were the whole GPU's tail (~25 us per
// launch).  Its rounds are dealt out in pieces of
// kX3PieceRounds, like single spans, to whichever waves of the workgroup
// free up.  The segment sums C_g do not depend on the accumulators, so every
// piece computes its C_g in parallel and parks them in its wave's LDS
// buffer; only the chain acc = scramble(acc + C_g) is sequential (8 x u64,
// a few VALU per segment).  Piece p waits for piece p - 1's accumulators
// (LDS, per span), chains its own segments and publishes them; the last
// piece issues the final unit's loads (partial segment, last stripe,
// epilogue inputs) before it waits, then folds and finishes the span.
// Pieces are handed out in order, so the piece a wave waits for is held by
// a wave that started earlier and never waits on a later one: the oldest
// unfinished piece always runs, and every wave of the workgroup is resident.
constexpr uint32_t kX3PieceRounds = 4;
constexpr uint32_t kX3MaxWaves = 16;

template <bool PREVIEW>
__device__ __forceinline__ uint32_t x3w_pieces(uint64_t len) {
  if (len <= 240) return 0;  // the short classes, done per lane before the loop
  return (x3w_span<PREVIEW>(0, len, 0).units + kX3PieceRounds - 1) / kX3PieceRounds;
}

// Workgroup LDS of the piece feed.
struct X3Lds {
  uint64_t off[kX3DescCache];
  uint32_t len[kX3DescCache];
  uint32_t pre[kX3DescCache + 1];  // exclusive prefix of pieces per span; [n] = total
  uint32_t done[kX3DescCache];     // pieces of span t chained so far
  uint32_t wsum[kX3MaxWaves];
  uint32_t ctr;
  uint32_t lists[2][4];  // rows share, by window parity: short count, long count, long ticket
  X3Short skeys[16];     // rows share: x3_short_rows' keys of row lane j
  uint64_t sec[24];      // rows share: XXH3_kSecret as words (x3_mid_quads)
  ulonglong2 acc[kX3DescCache][4];                       // span t's accumulators, pair q
  ulonglong2 csum[kX3MaxWaves][4 * kX3PieceRounds][4];  // a wave's parked C_g, pair q
};

struct X3Piece {
  X3WSpan sp;
  uint32_t t, p, np;
};
// Tickets count pieces; a wave's tickets increase, so it finds its span by
// a forward search from the last one (one LDS read per lane per 64 spans).
struct X3FeedPieces {
  X3Lds* s;
  uint32_t n, b, G, tc;
  uint64_t base;
  template <bool PREVIEW>
  __device__ __forceinline__ bool next(X3Piece& pc) {
    const uint32_t item = __builtin_amdgcn_readfirstlane(lds_ticket(&s->ctr));
    if (item >= s->pre[n]) return false;
    const uint32_t lane = threadIdx.x & 63;
    for (;;) {  // first span t >= tc with pre[t + 1] > item (exists: item < pre[n])
      const uint32_t tt = tc + lane;
      const uint32_t c = (uint32_t)__popcll(__ballot(tt < n && s->pre[tt + 1] <= item));
      tc += c;
      if (c < 64) break;
    }
    const uint32_t t = tc;
    const uint32_t p0 = __builtin_amdgcn_readfirstlane(s->pre[t]);
    pc.t = t;
    pc.p = item - p0;
    pc.np = __builtin_amdgcn_readfirstlane(s->pre[t + 1]) - p0;
    pc.sp = x3w_span<PREVIEW>(readfirstlane_u64(base + s->off[t]), readfirstlane_u64((uint64_t)s->len[t]),
                              b + G * t);
    return true;
  }
};

// Park the piece's segment sums (rounds k0 .. ke - 1) in the wave's buffer.
// (Round 4 measured round k + 1's loads issued before round k is summed --
// two rounds in flight per wave, 127 VGPRs: SST XXH3 image 0.682 -> 0.600,
// same box; the other waves of the CU already cover the round trip.)
template <bool PREVIEW>
__device__ __forceinline__ void x3p_park(const X3WSpan& sp, uint32_t k0, uint32_t ke, const X3Row& X,
                                         ulonglong2 (*cs)[4]) {
  for (uint32_t k = k0; k < ke; k++) {
    uint64_t c0, c1;
    x3w_round_sums<PREVIEW>(sp, x3w_round_load(sp, k, X), X, c0, c1);
    // each row parks its own segment's sums (lanes st4 = 0 of the row)
    if (X.st4 == 0) cs[4 * (k - k0) + X.row][X.q] = make_ulonglong2(c0, c1);
  }
}
// Wait for piece p - 1 of span t, then chain the parked segments.
__device__ __forceinline__ void x3p_chain(X3Lds* s, uint32_t t, uint32_t p, uint32_t segs, const X3Row& X,
                                          ulonglong2 (*cs)[4], uint64_t& a) {
  if (p) {
    while (__builtin_amdgcn_readfirstlane(
               __hip_atomic_load(&s->done[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) != p)
      __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    const ulonglong2 v = s->acc[t][X.q];
    a = X.role ? v.y : v.x;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");  // the parked sums to the other lanes
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
  for (uint32_t g = 0; g < segs; g++) {
    const ulonglong2 c = cs[g][X.q];
    a = xxh3_scramble(a + (X.role ? c.y : c.x), X.ksw);
  }
}
__device__ __forceinline__ void x3p_publish(X3Lds* s, uint32_t t, uint32_t p, const X3Row& X, uint64_t a) {
  // accumulator 2q from row 0 (lanes 0-3), 2q + 1 from row 2 (lanes 32-35)
  if (X.lane < 4) s->acc[t][X.q].x = a;
  if (X.lane >= 32 && X.lane < 36) s->acc[t][X.q].y = a;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  if (X.lane == 0) __hip_atomic_store(&s->done[t], p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <class Op, bool PREVIEW>
__device__ __forceinline__ void xxh3_piece_loop(const Op& op, X3FeedPieces& f, const X3Row& X) {
  ulonglong2(*const cs)[4] = f.s->csum[threadIdx.x >> 6];
  X3Piece pc;
  while (f.template next<PREVIEW>(pc)) {
    const X3WSpan& cur = pc.sp;
    uint64_t a = X.iw;
    // a whole span (np = 1) is its own last piece: the same code
    const uint32_t kl = cur.units - 1;  // the last unit
    const uint32_t k0 = pc.p * kX3PieceRounds;
    const bool last = pc.p + 1 == pc.np;
    const uint32_t ke = last ? kl : k0 + kX3PieceRounds;
    x3p_park<PREVIEW>(cur, k0, ke, X, cs);
    if (!last) {
      x3p_chain(f.s, pc.t, pc.p, 4 * kX3PieceRounds, X, cs, a);
      x3p_publish(f.s, pc.t, pc.p, X, a);
      continue;
    }
    const X3WLoads L = x3w_load(cur, kl, X);
    const typename Op::Pre e = op.pre(cur.i, cur.ptr, cur.len);
    x3p_chain(f.s, pc.t, pc.p, 4 * (kl - k0), X, cs, a);
    x3w_fold<Op, PREVIEW>(op, cur, kl, L, X, a, e, reinterpret_cast<uint64_t*>(cs));
  }
}

// Shares of spans that average 256 B - 2.5 KiB run on 16-lane rows inside
// the wave kernel (xxh3_rows_loop, as k_xxh3): the wave units' 4 KiB rounds
// are mostly padding there -- ragged 300-700 B 0.407 vs 0.153 of peak,
// 500-1500 B 0.456 vs 0.275, 1000-3000 B 0.554 vs 0.464; from ~3 KiB the
// wave units win (2000-4000 B 0.636 vs 0.590, SST-sized 4 KiB + jitter
// 0.733 vs 0.628; microbench/x3_width.py, profiles/r5/x3_width/).  Chosen
// per workgroup from a sample of its share's lengths, as crc_share_long.
// (round 6: no lower bound -- below 256 B the wave units padded every
// 241-600-byte span to a 4 KiB round: ragged 100-300 B ran at 0.136; the
// rows share with short spans on lane quads (x3_short_quads) and 241..512-
// byte spans on lane quads (x3_mid_quads) runs 100-300 B at 0.41 and
// 16-240 B at 0.445, against 0.243 on the wave units' one-span-per-lane
// short loop; profiles/r6/x3short/)
#ifndef X3_ROWS_MIN
#define X3_ROWS_MIN 0u
#endif
constexpr uint32_t kX3RowsMin = X3_ROWS_MIN, kX3RowsMax = 2560;  // mean span bytes
template <class Op>
__device__ __forceinline__ bool x3_share_rows(const Op& op, uint32_t lo, uint32_t hi) {
  const uint32_t n = hi - lo, lane = threadIdx.x & 63;
  const uint32_t m = n < 64 ? n : 64u;
  uint64_t len = 0;
  if (lane < m) len = op.hlen(lo + (uint32_t)((uint64_t)lane * n / m));
  for (int d = 32; d >= 1; d >>= 1) len += __shfl_xor(len, d, 64);
  return m != 0 && len >= (uint64_t)kX3RowsMin * m && len < (uint64_t)kX3RowsMax * m;
}

// Short spans (<= 240 B) on lane quads: lane q of a quad takes windows q,
// q + 4, q + 8, q + 12 of x3s_off's sixteen (four loads), the quad sums
// S0 (windows < 8) and S1 with two quad_sum -- four spans per row per
// iteration where x3_short_rows hashed one per row slot.  Keys from LDS.
template <class Op, class Slot>
__device__ __forceinline__ void x3_short_quads(const Op& op, uint32_t n, const X3Short* kl, Slot&& slot) {
  if (n == 0) return;
  const uint32_t qd = threadIdx.x >> 2, nq = blockDim.x >> 2, q = threadIdx.x & 3u;
  const uint64_t base = reinterpret_cast<uint64_t>(op.base());
  for (uint32_t t = qd; __any(t < n); t += nq) {
    const bool act = t < n;
    uint32_t len;
    uint64_t off;
    const uint32_t idx = slot(act ? t : n - 1, len, off);
    const uint64_t ptr = base + off;
    uint4 d[4];
    bool has[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t o = x3s_off(len, q + 4 * (uint32_t)k, has[k]);
      has[k] = has[k] && act && len > 16;
      d[k] = load16_realign(has[k] ? ptr + o : ptr & ~15ull);
    }
    const bool mid = len <= 128;
    uint64_t s0 = 0, s1 = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const X3Short K = kl[q + 4 * k];
      const uint64_t lo = ((uint64_t)d[k].y << 32) | d[k].x, hi = ((uint64_t)d[k].w << 32) | d[k].z;
      const uint64_t v = has[k] ? mul128_fold64(lo ^ (mid ? K.a0 : K.b0), hi ^ (mid ? K.a1 : K.b1)) : 0ull;
      if (k < 2)
        s0 += v;
      else
        s1 += v;
    }
    s0 = quad_sum(s0);
    s1 = quad_sum(s1);
    const uint64_t a = (uint64_t)len * P64_1 + s0;
    uint64_t h = mid ? xxh3_avalanche(a + s1) : xxh3_avalanche(xxh3_avalanche(a) + s1);
    if (act && q == 0) {
      if (len <= 16) h = x3_small<false>(reinterpret_cast<const uint8_t*>(ptr), len, 0);
      op.finish(idx, h);
    }
  }
}

// ---- spans of 241..1024 bytes on lane quads (round 6) ----------------------
// XXH3_64bits of 240 < n <= 1024 (util/xxhash.h:5141-5227 with no full
// block: nbStripes = (n - 1) / 64 stripes of the one partial segment, the
// last stripe at n - 64, the merge) needs no scramble, so a span is FOUR
// lanes: lane q of the quad keeps accumulators 2q, 2q + 1 and reads bytes
// [16 q, 16 q + 16) of every stripe (the quad reads each 64-byte stripe
// whole), four stripes per iteration.  The 16-lane row loop spent a whole
// 1 KiB iteration on such a span (a 280-byte span filled 27 % of it); four
// spans per row now share one.  Stripe secrets from the LDS copy (word
// s + 2 q of stripe s).
template <class Op, class Slot>
__device__ __forceinline__ void x3_mid_quads(const Op& op, uint32_t n, const X3Row& X, const uint64_t* lsec,
                                             Slot&& slot) {
  if (n == 0) return;
  const uint32_t qd = threadIdx.x >> 2, nq = blockDim.x >> 2, q = threadIdx.x & 3u;
  const uint64_t base = reinterpret_cast<uint64_t>(op.base());
  for (uint32_t t = qd; __any(t < n); t += nq) {
    const bool act = t < n;
    uint32_t len;
    uint64_t off;
    const uint32_t idx = slot(act ? t : n - 1, len, off);
    const uint64_t ptr = base + off;
    const uint32_t nst = act ? (len - 1) >> 6 : 0u;  // 240 < len <= 1024: no full segment
    uint64_t a0 = X.i0, a1 = X.i1;
    for (uint32_t g = 0; __any(4 * g < nst); g++) {
      uint4 d[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t st = 4 * g + (uint32_t)k;
        d[k] = load16_realign(st < nst ? ptr + 64 * st + 16 * q : ptr & ~15ull);
      }
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t st = 4 * g + (uint32_t)k;
        if (st < nst) {  // v0.8.1: acc[i] += data[i ^ 1] + lo32(d ^ s) * hi32(d ^ s)
          const uint64_t d0 = ((uint64_t)d[k].y << 32) | d[k].x, d1 = ((uint64_t)d[k].w << 32) | d[k].z;
          a0 += d1 + mul32to64(d0 ^ lsec[st + 2 * q]);
          a1 += d0 + mul32to64(d1 ^ lsec[st + 2 * q + 1]);
        }
      }
    }
    // the last stripe (secret 121 + 16 q) and the merge (secret 11 + 16 q)
    const uint4 dl = load16_realign(act ? ptr + len - 64 + 16 * q : ptr & ~15ull);
    const uint64_t l0 = ((uint64_t)dl.y << 32) | dl.x, l1 = ((uint64_t)dl.w << 32) | dl.z;
    a0 += l1 + mul32to64(l0 ^ X.kl0);
    a1 += l0 + mul32to64(l1 ^ X.kl1);
    const uint64_t m = quad_sum(mul128_fold64(a0 ^ X.km0, a1 ^ X.km1));
    const uint64_t h = xxh3_avalanche((uint64_t)len * P64_1 + m);
    if (act && q == 0) op.finish(idx, h);
  }
}

#ifndef X3S_U
#define X3S_U 2
#endif
#ifndef X3S_MIDMAX
#define X3S_MIDMAX 512u
#endif
#ifndef X3S_QUADS
#define X3S_QUADS 1
#endif
#ifndef X3S_WIN
#define X3S_WIN 1024
#endif
// The rows share (spans averaging < 2.5 KiB, round 6): windows of
// blockDim spans, staged in LDS and split into a short list (<= 240 B,
// hashed first by x3_short_rows, four per row in flight) and a long list the
// rows draw from by LDS ticket -- balanced inside the workgroup, where the
// static row stride left a row that drew short or small spans idle.  Each
// thread loads the next window's descriptor while the current window runs.
// (Round 6 first ran the short spans as a separate pass over the share's
// global descriptors: ragged 241-600 B fell from 0.363 to 0.316, every
// slot costing the rows a dependent descriptor load.)
// The rows share's hashes park in LDS (slot of the window) and thread t
// finishes window slot t after both passes: one coalesced output write per
// window instead of an 8-byte store per span from whichever row finished it
// (XXH3 100-300 B: WRITE_SIZE 0.215 x the algorithmic bytes, six times the
// 8-byte outputs, before).
template <class Op>
struct X3ParkOp {
  const Op& op;
  uint64_t* hv;
  uint32_t wb;
  __device__ const uint8_t* base() const { return op.base(); }
  __device__ uint64_t off(uint32_t i) const { return op.off(i); }
  __device__ uint64_t hlen(uint32_t i) const { return op.hlen(i); }
  __device__ void finish(uint32_t i, uint64_t h) const { hv[i - wb] = h; }
};
template <class Op, bool PREVIEW>
__device__ __forceinline__ void x3_rows_share(const Op& op, X3Lds& s, uint32_t lo, uint32_t hi, const X3Row& X,
                                              uint64_t seed) {
  // window W spans (<= blockDim.x; threads t >= W stage nothing)
  const uint32_t n = hi - lo, W = X3S_WIN < blockDim.x ? X3S_WIN : blockDim.x, t = threadIdx.x;
  const uint32_t rows = blockDim.x >> 4, row = t >> 4, j = t & 15u;
  const uint64_t base = reinterpret_cast<uint64_t>(op.base());
  uint32_t nlen = 0;
  uint64_t noff = 0;
  if (t < W && t < n) {
    nlen = (uint32_t)op.hlen(lo + t);
    noff = op.off(lo + t);
  }
  if (t < 8) (&s.lists[0][0])[t] = 0;
  if (t < 16) s.skeys[t] = x3s_keys(t, seed);
  if (t < 24) s.sec[t] = sec64(8 * (int)t);
  // the mid list lives past the parked hashes in the piece path's accumulators
  uint32_t* const mlist = reinterpret_cast<uint32_t*>(&s.acc[0][0]) + 2 * kX3DescCache;
  uint32_t par = 0;
  for (uint32_t w0 = 0; w0 < n; w0 += W, par ^= 1u) {
    const uint32_t wn = n - w0 < W ? n - w0 : W;
    uint32_t* L = &s.lists[par][0];
    __syncthreads();  // (the previous window's rows are done with its lists; the counters are zero)
    if (t < W) {
      s.off[t] = noff;
      s.len[t] = nlen;
    }
    // short (<= 240), mid (<= 1024: x3_mid_quads), long (the row loop)
    const bool in = t < wn, sh = in && nlen <= 240u, md = in && nlen > 240u && nlen <= X3S_MIDMAX,
               lg = in && nlen > X3S_MIDMAX;
    const uint64_t ms = __ballot(sh), mm = __ballot(md), ml = __ballot(lg);
    const uint32_t lane = t & 63u;
    uint32_t bs = 0, bm = 0, bl = 0;
    if (lane == 0) {
      if (ms) bs = atomicAdd(&L[0], (uint32_t)__popcll(ms));
      if (ml) bl = atomicAdd(&L[1], (uint32_t)__popcll(ml));
      if (mm) bm = atomicAdd(&L[3], (uint32_t)__popcll(mm));
    }
    bs = __shfl(bs, 0, 64);
    bm = __shfl(bm, 0, 64);
    bl = __shfl(bl, 0, 64);
    const uint64_t below = (1ull << lane) - 1;
    if (sh) s.pre[bs + (uint32_t)__popcll(ms & below)] = t;
    if (md) mlist[bm + (uint32_t)__popcll(mm & below)] = t;
    if (lg) s.done[bl + (uint32_t)__popcll(ml & below)] = t;
    if (t < 4) s.lists[par ^ 1u][t] = 0;  // the next window's counters
    __syncthreads();
    // the next window's descriptors, in flight while this one runs
    {
      const uint32_t k = w0 + W + t;
      if (t < W && k < n) {
        nlen = (uint32_t)op.hlen(lo + k);
        noff = op.off(lo + k);
      }
    }
    const uint32_t wb = lo + w0, nshort = L[0], nlong = L[1];
    uint64_t* hv = reinterpret_cast<uint64_t*>(&s.acc[0][0]);  // (the piece path's accumulators, unused here)
    const X3ParkOp<Op> pop{op, hv, wb};
    auto sslot = [&](uint32_t q, uint32_t& len, uint64_t& off) {
      const uint32_t k = s.pre[q];
      len = s.len[k];
      off = s.off[k];
      return wb + k;
    };
    if constexpr (X3S_QUADS && !PREVIEW)
      x3_short_quads(pop, nshort, s.skeys, sslot);
    else
      x3_short_rows<X3ParkOp<Op>, PREVIEW, X3S_U, true>(pop, row, nshort, rows, seed, sslot, s.skeys);
    x3_mid_quads(pop, L[3], X, s.sec, [&](uint32_t q, uint32_t& len, uint64_t& off) {
      const uint32_t k = mlist[q];
      len = s.len[k];
      off = s.off[k];
      return wb + k;
    });
    auto next = [&](X3Span& r) {
      uint32_t tk = 0;
      if (j == 0) tk = atomicAdd(&L[2], 1u);
      tk = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((t & 0x30u) << 2), (int)tk);
      if (tk >= nlong) return false;
      const uint32_t k = s.done[tk];
      x3_span_start<PREVIEW>(r, base + s.off[k], s.len[k], wb + k);
      return true;
    };
    // idle rows keep loading from a valid address: the batch's base
    X3Span rs{base, 0, 0, 0, 0, 0, false};
    const bool act = next(rs);
    // (round 6 measured the row loop's constants re-read from LDS after the
    // short pass, so that more short spans per row fit in flight: slower at
    // every shape, and 4 or 8 spans per row slower than 2 -- 16-240 B 0.240
    // with 2, 0.203 with 4, 0.097 with 8)
    xxh3_rows_loop<X3ParkOp<Op>, PREVIEW>(pop, X, rs, act, next);
    __syncthreads();
    if (t < wn) op.finish(wb + t, hv[t]);
  }
}

// Workgroup b's share: a byte-balanced contiguous range (share_by_bytes),
// staged in windows of kX3DescCache spans, long spans in pieces.
template <class Op, bool PREVIEW>
__device__ __forceinline__ void xxh3_wave_driver(const Op& op, uint32_t count, uint64_t seed) {
  __shared__ X3Lds s;
  const uint32_t lane = threadIdx.x & 63, wpb = blockDim.x >> 6, wid = threadIdx.x >> 6;
  uint32_t lo, hi;
  // the per-lane constants' loads ride along with the search's first round
  // trip (their ~1.2 us came after the 5 us search: round-5 LDS stamps,
  // microbench/r5_stamps_x3.py)
  X3Row X;
  share_by_bytes(op, 0u, count, 0xFFFFFFFFu, &s.wsum[0], &lo, &hi,
                 [&](uint32_t i) { return (uint32_t)op.off(i) ^ (uint32_t)op.hlen(i); },
                 [&] { X = x3_row(seed); });
  if (x3_share_rows(op, lo, hi)) {  // workgroup-uniform
    x3_rows_share<Op, PREVIEW>(op, s, lo, hi, X, seed);
    return;
  }
  const uint32_t start = lo, stride = 1, n = hi - lo;
  for (uint32_t w0 = 0; w0 < n; w0 += kX3DescCache) {
    const uint32_t wn = n - w0 < kX3DescCache ? n - w0 : kX3DescCache;
    const uint32_t wb = start + stride * w0;  // span of window slot t: wb + stride t
    if (w0) __syncthreads();  // the previous window's waves are done with its slots
    for (uint32_t t = threadIdx.x; t < wn; t += blockDim.x) {
      s.off[t] = op.off(wb + stride * t);
      s.len[t] = (uint32_t)op.hlen(wb + stride * t);
      s.done[t] = 0;
    }
    if (threadIdx.x == 0) s.ctr = 0;
    // pieces per span, exclusive prefix (a chunk of blockDim spans at a time)
    uint32_t carry = 0;
    for (uint32_t c0 = 0; c0 < wn; c0 += blockDim.x) {
      const uint32_t t = c0 + threadIdx.x;
      // (the length this thread staged above: no second global read)
      const uint32_t v = t < wn ? x3w_pieces<PREVIEW>(s.len[t]) : 0;
      uint32_t x = v;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
        x += lane >= (uint32_t)d ? y : 0u;
      }
      if (lane == 63) s.wsum[wid] = x;
      __syncthreads();
      uint32_t below = 0, tot = 0;
      for (uint32_t w = 0; w < wpb; w++) {
        const uint32_t ws = s.wsum[w];
        below += w < wid ? ws : 0u;
        tot += ws;
      }
      if (t < wn) s.pre[t] = carry + below + x - v;
      carry += tot;
      __syncthreads();
    }
    if (threadIdx.x == 0) s.pre[wn] = carry;
    __syncthreads();
    // short spans (<= 240 bytes: the three small-input classes) first, one
    // per lane -- outside the pipelined loop (spans of KiBs: few are short)
    const uint64_t base = reinterpret_cast<uint64_t>(op.base());
    for (uint32_t t = threadIdx.x; t < wn; t += blockDim.x) {
      const uint64_t len = s.len[t];
      if (len <= 240) {
        const uint8_t* p = reinterpret_cast<const uint8_t*>(base + s.off[t]);
        op.finish(wb + stride * t, PREVIEW ? xxph3_short(p, len, seed) : xxh3_short(p, len));
      }
    }
    // (Round 4 measured spans of one piece -- <= 4 rounds, the SST mix's 4
    // and 16 KiB blocks -- on 16-lane rows first, segment by segment as
    // xxh3_rows_driver, one scramble per segment and row: SST XXH3 image
    // 0.613 vs 0.666 on the wave units, same box; not kept.)
    X3FeedPieces f{&s, wn, wb, stride, 0, base};
    xxh3_piece_loop<Op, PREVIEW>(op, f, X);
  }
}

// ---- legacy XXH32 / XXH64, one lane per span ----------------------------
// The span may be followed by one virtual byte (the block type byte of
// ComputeBuiltinChecksumWithLastByte, table/format.cc:604-645).
struct VBytes {
  const uint8_t* p;
  uint64_t n;       // bytes in memory
  bool has_extra;   // one more virtual byte
  uint8_t extra;
  __device__ uint64_t size() const { return n + (has_extra ? 1 : 0); }
  __device__ uint8_t at(uint64_t i) const { return i < n ? p[i] : extra; }
  __device__ uint32_t r32(uint64_t i) const {
    if (i + 4 <= n) return rd32(p + i);
    return (uint32_t)at(i) | ((uint32_t)at(i + 1) << 8) | ((uint32_t)at(i + 2) << 16) | ((uint32_t)at(i + 3) << 24);
  }
  __device__ uint64_t r64(uint64_t i) const {
    if (i + 8 <= n) return rd64(p + i);
    return (uint64_t)r32(i) | ((uint64_t)r32(i + 4) << 32);
  }
};

__device__ __forceinline__ uint32_t xxh32_round(uint32_t acc, uint32_t in) {
  return rotl32(acc + in * P32_2, 13) * P32_1;
}
__device__ __noinline__ uint32_t xxh32_lane(const VBytes& b, uint32_t seed) {
  const uint64_t len = b.size();
  uint64_t i = 0;
  uint32_t h;
  if (len >= 16) {
    uint32_t v1 = seed + P32_1 + P32_2, v2 = seed + P32_2, v3 = seed, v4 = seed - P32_1;
    const uint64_t limit = len - 16;
    for (; i + 16 <= b.n && i <= limit; i += 16) {
      const uint4 w = *reinterpret_cast<const uint4*>(b.p + i);
      v1 = xxh32_round(v1, w.x);
      v2 = xxh32_round(v2, w.y);
      v3 = xxh32_round(v3, w.z);
      v4 = xxh32_round(v4, w.w);
    }
    for (; i <= limit; i += 16) {
      v1 = xxh32_round(v1, b.r32(i));
      v2 = xxh32_round(v2, b.r32(i + 4));
      v3 = xxh32_round(v3, b.r32(i + 8));
      v4 = xxh32_round(v4, b.r32(i + 12));
    }
    h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18);
  } else {
    h = seed + P32_5;
  }
  h += (uint32_t)len;
  for (; i + 4 <= len; i += 4) h = rotl32(h + b.r32(i) * P32_3, 17) * P32_4;
  for (; i < len; i++) h = rotl32(h + b.at(i) * P32_5, 11) * P32_1;
  h ^= h >> 15;
  h *= P32_2;
  h ^= h >> 13;
  h *= P32_3;
  h ^= h >> 16;
  return h;
}

__device__ __forceinline__ uint64_t xxh64_round(uint64_t acc, uint64_t in) {
  return rotl64(acc + in * P64_2, 31) * P64_1;
}
__device__ __forceinline__ uint64_t xxh64_merge(uint64_t acc, uint64_t v) {
  acc ^= xxh64_round(0, v);
  return acc * P64_1 + P64_4;
}
__device__ __noinline__ uint64_t xxh64_lane(const VBytes& b, uint64_t seed) {
  const uint64_t len = b.size();
  uint64_t i = 0;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + P64_1 + P64_2, v2 = seed + P64_2, v3 = seed, v4 = seed - P64_1;
    const uint64_t limit = len - 32;
    for (; i + 32 <= b.n && i <= limit; i += 32) {
      const uint4 w0 = *reinterpret_cast<const uint4*>(b.p + i);
      const uint4 w1 = *reinterpret_cast<const uint4*>(b.p + i + 16);
      v1 = xxh64_round(v1, ((uint64_t)w0.y << 32) | w0.x);
      v2 = xxh64_round(v2, ((uint64_t)w0.w << 32) | w0.z);
      v3 = xxh64_round(v3, ((uint64_t)w1.y << 32) | w1.x);
      v4 = xxh64_round(v4, ((uint64_t)w1.w << 32) | w1.z);
    }
    for (; i <= limit; i += 32) {
      v1 = xxh64_round(v1, b.r64(i));
      v2 = xxh64_round(v2, b.r64(i + 8));
      v3 = xxh64_round(v3, b.r64(i + 16));
      v4 = xxh64_round(v4, b.r64(i + 24));
    }
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = xxh64_merge(h, v1);
    h = xxh64_merge(h, v2);
    h = xxh64_merge(h, v3);
    h = xxh64_merge(h, v4);
  } else {
    h = seed + P64_5;
  }
  h += len;
  for (; i + 8 <= len; i += 8) h = rotl64(h ^ xxh64_round(0, b.r64(i)), 27) * P64_1 + P64_4;
  if (i + 4 <= len) {
    h = rotl64(h ^ ((uint64_t)b.r32(i) * P64_1), 23) * P64_2 + P64_3;
    i += 4;
  }
  for (; i < len; i++) h = rotl64(h ^ (b.at(i) * P64_5), 11) * P64_1;
  return xxh64_avalanche(h);
}

}  // namespace mck
