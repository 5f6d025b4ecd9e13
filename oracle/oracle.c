/*
 * oracle.c -- plain-C restatement of the reference checksum path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Written from the published
 * algorithms (CRC-32C / Castagnoli, RFC 3720 B.4; xxHash v0.8.1 XXH32, XXH64,
 * XXH3-64) and the reference's call-site semantics; each function cites the
 * reference line it follows.  Speed is not a goal here: the CRC is a plain
 * slice-by-8 table walk and XXH3 is the scalar accumulate loop.
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* CRC-32C                                                             */
/* ------------------------------------------------------------------ */

/* Reflected Castagnoli polynomial (util/crc32c.cc:1193 crc32c_m). */
#define ORC_CRC32C_POLY 0x82f63b78u

static uint32_t crc_tab[8][256];
static int crc_tab_ready = 0;

static void crc_tab_init(void) {
  if (crc_tab_ready) return;
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c >> 1) ^ ((c & 1u) ? ORC_CRC32C_POLY : 0u);
    crc_tab[0][i] = c;
  }
  for (int t = 1; t < 8; t++)
    for (uint32_t i = 0; i < 256; i++)
      crc_tab[t][i] = (crc_tab[t - 1][i] >> 8) ^ crc_tab[0][crc_tab[t - 1][i] & 0xff];
  crc_tab_ready = 1;
}

static inline uint32_t rd32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
         ((uint32_t)p[3] << 24);
}
static inline uint64_t rd64(const uint8_t* p) {
  return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32);
}

/* "Pure" (init 0, no final inversion) table update; the state algebra the
 * reference describes at util/crc32c.cc:1221-1266. */
static uint32_t crc_pure_update(uint32_t s, const uint8_t* p, size_t n) {
  crc_tab_init();
  while (n >= 8) {
    uint32_t lo = rd32(p) ^ s, hi = rd32(p + 4);
    s = crc_tab[7][lo & 0xff] ^ crc_tab[6][(lo >> 8) & 0xff] ^
        crc_tab[5][(lo >> 16) & 0xff] ^ crc_tab[4][lo >> 24] ^
        crc_tab[3][hi & 0xff] ^ crc_tab[2][(hi >> 8) & 0xff] ^
        crc_tab[1][(hi >> 16) & 0xff] ^ crc_tab[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) s = (s >> 8) ^ crc_tab[0][(s ^ *p++) & 0xff];
  return s;
}

/* util/crc32c.cc:275-316 ExtendImpl: l = crc ^ ~0 ... return l ^ ~0. */
uint32_t orc_crc32c_extend(uint32_t init_crc, const void* data, size_t n) {
  return ~crc_pure_update(~init_crc, (const uint8_t*)data, n);
}

/* util/crc32c.h:35 Value = Extend(0, data, n). */
uint32_t orc_crc32c_value(const void* data, size_t n) {
  return orc_crc32c_extend(0, data, n);
}

/* util/crc32c.h:37-45: rotate right by 15, add kMaskDelta. */
uint32_t orc_crc32c_mask(uint32_t crc) {
  return ((crc >> 15) | (crc << 17)) + 0xa282ead8u;
}

/* util/crc32c.h:48-51. */
uint32_t orc_crc32c_unmask(uint32_t masked) {
  uint32_t rot = masked - 0xa282ead8u;
  return (rot >> 17) | (rot << 15);
}

/* Multiply two reflected GF(2)[x] residues mod P (bit 31 = x^0).
 * Same algebra as util/crc32c.cc:1138 gf_multiply_sw. */
static uint32_t gf_mul(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (int j = 0; j < 32; j++) {
    if (b & (0x80000000u >> j)) p ^= a;
    a = (a >> 1) ^ ((a & 1u) ? ORC_CRC32C_POLY : 0u); /* a *= x */
  }
  return p;
}

/* x^(8*nbytes) mod P, reflected. */
static uint32_t x_pow_8n(uint64_t nbytes) {
  uint32_t result = 0x80000000u; /* x^0 */
  uint32_t sq = 0x00800000u;     /* x^8 */
  while (nbytes) {
    if (nbytes & 1) result = gf_mul(result, sq);
    sq = gf_mul(sq, sq);
    nbytes >>= 1;
  }
  return result;
}

uint32_t orc_crc32c_zshift(uint32_t state, uint64_t nbytes) {
  return gf_mul(state, x_pow_8n(nbytes));
}

/* util/crc32c.cc:1274-1289 Crc32cCombine.  With the inverted-in/inverted-out
 * convention the algebra of 1221-1266 reduces to
 *   Value(A||B) = zshift(Value(A), |B|) ^ Value(B). */
uint32_t orc_crc32c_combine(uint32_t crc1, uint32_t crc2, size_t crc2len) {
  return orc_crc32c_zshift(crc1, crc2len) ^ crc2;
}

/* ------------------------------------------------------------------ */
/* xxHash v0.8.1 (util/xxhash.h, namespaced ROCKSDB_ in the reference)   */
/* ------------------------------------------------------------------ */

#define P32_1 0x9E3779B1u
#define P32_2 0x85EBCA77u
#define P32_3 0xC2B2AE3Du
#define P32_4 0x27D4EB2Fu
#define P32_5 0x165667B1u
#define P64_1 0x9E3779B185EBCA87ull
#define P64_2 0xC2B2AE3D27D4EB4Full
#define P64_3 0x165667B19E3779F9ull
#define P64_4 0x85EBCA77C2B2AE63ull
#define P64_5 0x27D4EB2F165667C5ull

static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

/* XXH32 (util/xxhash.h XXH32_round / XXH32_avalanche / XXH32_finalize). */
static inline uint32_t xxh32_round(uint32_t acc, uint32_t in) {
  acc += in * P32_2;
  acc = rotl32(acc, 13);
  return acc * P32_1;
}

uint32_t orc_xxh32(const void* data, size_t n, uint32_t seed) {
  const uint8_t* p = (const uint8_t*)data;
  const uint8_t* end = p + n;
  uint32_t h;
  if (n >= 16) {
    uint32_t v1 = seed + P32_1 + P32_2, v2 = seed + P32_2, v3 = seed,
             v4 = seed - P32_1;
    const uint8_t* limit = end - 15;
    do {
      v1 = xxh32_round(v1, rd32(p));
      v2 = xxh32_round(v2, rd32(p + 4));
      v3 = xxh32_round(v3, rd32(p + 8));
      v4 = xxh32_round(v4, rd32(p + 12));
      p += 16;
    } while (p < limit);
    h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18);
  } else {
    h = seed + P32_5;
  }
  h += (uint32_t)n;
  size_t rem = (size_t)(end - p);
  while (rem >= 4) {
    h += rd32(p) * P32_3;
    h = rotl32(h, 17) * P32_4;
    p += 4;
    rem -= 4;
  }
  while (rem--) {
    h += (*p++) * P32_5;
    h = rotl32(h, 11) * P32_1;
  }
  h ^= h >> 15;
  h *= P32_2;
  h ^= h >> 13;
  h *= P32_3;
  h ^= h >> 16;
  return h;
}

/* XXH64 (util/xxhash.h XXH64_round / XXH64_mergeRound / XXH64_finalize). */
static inline uint64_t xxh64_round(uint64_t acc, uint64_t in) {
  acc += in * P64_2;
  acc = rotl64(acc, 31);
  return acc * P64_1;
}
static inline uint64_t xxh64_merge(uint64_t acc, uint64_t v) {
  acc ^= xxh64_round(0, v);
  return acc * P64_1 + P64_4;
}
static inline uint64_t xxh64_avalanche(uint64_t h) {
  h ^= h >> 33;
  h *= P64_2;
  h ^= h >> 29;
  h *= P64_3;
  h ^= h >> 32;
  return h;
}

uint64_t orc_xxh64(const void* data, size_t n, uint64_t seed) {
  const uint8_t* p = (const uint8_t*)data;
  const uint8_t* end = p + n;
  uint64_t h;
  if (n >= 32) {
    uint64_t v1 = seed + P64_1 + P64_2, v2 = seed + P64_2, v3 = seed,
             v4 = seed - P64_1;
    const uint8_t* limit = end - 31;
    do {
      v1 = xxh64_round(v1, rd64(p));
      v2 = xxh64_round(v2, rd64(p + 8));
      v3 = xxh64_round(v3, rd64(p + 16));
      v4 = xxh64_round(v4, rd64(p + 24));
      p += 32;
    } while (p < limit);
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = xxh64_merge(h, v1);
    h = xxh64_merge(h, v2);
    h = xxh64_merge(h, v3);
    h = xxh64_merge(h, v4);
  } else {
    h = seed + P64_5;
  }
  h += (uint64_t)n;
  size_t rem = (size_t)(end - p);
  while (rem >= 8) {
    h ^= xxh64_round(0, rd64(p));
    h = rotl64(h, 27) * P64_1 + P64_4;
    p += 8;
    rem -= 8;
  }
  if (rem >= 4) {
    h ^= (uint64_t)rd32(p) * P64_1;
    h = rotl64(h, 23) * P64_2 + P64_3;
    p += 4;
    rem -= 4;
  }
  while (rem--) {
    h ^= (*p++) * P64_5;
    h = rotl64(h, 11) * P64_1;
  }
  return xxh64_avalanche(h);
}

/* XXH3_kSecret (util/xxhash.h:3661-3674), 192 bytes. */
static const uint8_t kSecret[192] = {
    0xb8, 0xfe, 0x6c, 0x39, 0x23, 0xa4, 0x4b, 0xbe, 0x7c, 0x01, 0x81, 0x2c,
    0xf7, 0x21, 0xad, 0x1c, 0xde, 0xd4, 0x6d, 0xe9, 0x83, 0x90, 0x97, 0xdb,
    0x72, 0x40, 0xa4, 0xa4, 0xb7, 0xb3, 0x67, 0x1f, 0xcb, 0x79, 0xe6, 0x4e,
    0xcc, 0xc0, 0xe5, 0x78, 0x82, 0x5a, 0xd0, 0x7d, 0xcc, 0xff, 0x72, 0x21,
    0xb8, 0x08, 0x46, 0x74, 0xf7, 0x43, 0x24, 0x8e, 0xe0, 0x35, 0x90, 0xe6,
    0x81, 0x3a, 0x26, 0x4c, 0x3c, 0x28, 0x52, 0xbb, 0x91, 0xc3, 0x00, 0xcb,
    0x88, 0xd0, 0x65, 0x8b, 0x1b, 0x53, 0x2e, 0xa3, 0x71, 0x64, 0x48, 0x97,
    0xa2, 0x0d, 0xf9, 0x4e, 0x38, 0x19, 0xef, 0x46, 0xa9, 0xde, 0xac, 0xd8,
    0xa8, 0xfa, 0x76, 0x3f, 0xe3, 0x9c, 0x34, 0x3f, 0xf9, 0xdc, 0xbb, 0xc7,
    0xc7, 0x0b, 0x4f, 0x1d, 0x8a, 0x51, 0xe0, 0x4b, 0xcd, 0xb4, 0x59, 0x31,
    0xc8, 0x9f, 0x7e, 0xc9, 0xd9, 0x78, 0x73, 0x64, 0xea, 0xc5, 0xac, 0x83,
    0x34, 0xd3, 0xeb, 0xc3, 0xc5, 0x81, 0xa0, 0xff, 0xfa, 0x13, 0x63, 0xeb,
    0x17, 0x0d, 0xdd, 0x51, 0xb7, 0xf0, 0xda, 0x49, 0xd3, 0x16, 0x55, 0x26,
    0x29, 0xd4, 0x68, 0x9e, 0x2b, 0x16, 0xbe, 0x58, 0x7d, 0x47, 0xa1, 0xfc,
    0x8f, 0xf8, 0xb8, 0xd1, 0x7a, 0xd0, 0x31, 0xce, 0x45, 0xcb, 0x3a, 0x8f,
    0x95, 0x16, 0x04, 0x28, 0xaf, 0xd7, 0xfb, 0xca, 0xbb, 0x4b, 0x40, 0x7e,
};

static inline uint64_t mul128_fold64(uint64_t a, uint64_t b) {
  unsigned __int128 r = (unsigned __int128)a * b;
  return (uint64_t)r ^ (uint64_t)(r >> 64);
}
static inline uint64_t xorshift64(uint64_t v, int s) { return v ^ (v >> s); }
static inline uint64_t swap64(uint64_t x) { return __builtin_bswap64(x); }
static inline uint32_t swap32(uint32_t x) { return __builtin_bswap32(x); }

/* util/xxhash.h:3877 XXH3_avalanche */
static uint64_t xxh3_avalanche(uint64_t h) {
  h = xorshift64(h, 37);
  h *= 0x165667919E3779F9ull;
  return xorshift64(h, 32);
}
/* util/xxhash.h XXH3_rrmxmx */
static uint64_t xxh3_rrmxmx(uint64_t h, uint64_t len) {
  h ^= rotl64(h, 49) ^ rotl64(h, 24);
  h *= 0x9FB21C651E98DF25ull;
  h ^= (h >> 35) + len;
  h *= 0x9FB21C651E98DF25ull;
  return xorshift64(h, 28);
}

/* util/xxhash.h XXH3_mix16B (seed 0) */
static uint64_t mix16(const uint8_t* in, const uint8_t* sec) {
  return mul128_fold64(rd64(in) ^ rd64(sec), rd64(in + 8) ^ rd64(sec + 8));
}

/* util/xxhash.h:3990 XXH3_len_0to16_64b and its 1to3 / 4to8 / 9to16 parts. */
static uint64_t xxh3_0to16(const uint8_t* in, size_t len) {
  if (len > 8) {
    uint64_t bf1 = rd64(kSecret + 24) ^ rd64(kSecret + 32);
    uint64_t bf2 = rd64(kSecret + 40) ^ rd64(kSecret + 48);
    uint64_t lo = rd64(in) ^ bf1;
    uint64_t hi = rd64(in + len - 8) ^ bf2;
    uint64_t acc = len + swap64(lo) + hi + mul128_fold64(lo, hi);
    return xxh3_avalanche(acc);
  }
  if (len >= 4) {
    uint32_t in1 = rd32(in), in2 = rd32(in + len - 4);
    uint64_t bf = rd64(kSecret + 8) ^ rd64(kSecret + 16);
    uint64_t in64 = in2 + ((uint64_t)in1 << 32);
    return xxh3_rrmxmx(in64 ^ bf, len);
  }
  if (len) {
    uint8_t c1 = in[0], c2 = in[len >> 1], c3 = in[len - 1];
    uint32_t comb = ((uint32_t)c1 << 16) | ((uint32_t)c2 << 24) |
                    ((uint32_t)c3 << 0) | ((uint32_t)len << 8);
    uint64_t bf = (uint64_t)(rd32(kSecret) ^ rd32(kSecret + 4));
    return xxh64_avalanche((uint64_t)comb ^ bf);
  }
  return xxh64_avalanche(rd64(kSecret + 56) ^ rd64(kSecret + 64));
}

/* util/xxhash.h:4060 XXH3_len_17to128_64b */
static uint64_t xxh3_17to128(const uint8_t* in, size_t len) {
  uint64_t acc = len * P64_1, acc_end;
  acc += mix16(in, kSecret);
  acc_end = mix16(in + len - 16, kSecret + 16);
  if (len > 32) {
    acc += mix16(in + 16, kSecret + 32);
    acc_end += mix16(in + len - 32, kSecret + 48);
    if (len > 64) {
      acc += mix16(in + 32, kSecret + 64);
      acc_end += mix16(in + len - 48, kSecret + 80);
      if (len > 96) {
        acc += mix16(in + 48, kSecret + 96);
        acc_end += mix16(in + len - 64, kSecret + 112);
      }
    }
  }
  return xxh3_avalanche(acc + acc_end);
}

/* util/xxhash.h:4100 XXH3_len_129to240_64b */
static uint64_t xxh3_129to240(const uint8_t* in, size_t len) {
  uint64_t acc = len * P64_1, acc_end;
  unsigned rounds = (unsigned)len / 16;
  for (unsigned i = 0; i < 8; i++) acc += mix16(in + 16 * i, kSecret + 16 * i);
  acc_end = mix16(in + len - 16, kSecret + 136 - 17);
  acc = xxh3_avalanche(acc);
  for (unsigned i = 8; i < rounds; i++)
    acc_end += mix16(in + 16 * i, kSecret + 16 * (i - 8) + 3);
  return xxh3_avalanche(acc + acc_end);
}

/* util/xxhash.h:4953 XXH3_accumulate_512_scalar (one 64-byte stripe). */
static void acc512(uint64_t acc[8], const uint8_t* in, const uint8_t* sec) {
  for (int l = 0; l < 8; l++) {
    uint64_t dv = rd64(in + 8 * l);
    uint64_t dk = dv ^ rd64(sec + 8 * l);
    acc[l ^ 1] += dv;
    acc[l] += (uint64_t)(uint32_t)dk * (dk >> 32);
  }
}
/* util/xxhash.h:4979 XXH3_scalarScrambleRound */
static void scramble(uint64_t acc[8], const uint8_t* sec) {
  for (int l = 0; l < 8; l++) {
    uint64_t a = acc[l];
    a = xorshift64(a, 47);
    a ^= rd64(sec + 8 * l);
    a *= P32_1;
    acc[l] = a;
  }
}

/* util/xxhash.h:5141-5227 hashLong_internal_loop + hashLong_64b_internal. */
static uint64_t xxh3_long(const uint8_t* in, size_t len) {
  uint64_t acc[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
  const size_t stripes_per_block = (192 - 64) / 8; /* 16 */
  const size_t block_len = 64 * stripes_per_block; /* 1024 */
  const size_t nb_blocks = (len - 1) / block_len;
  for (size_t n = 0; n < nb_blocks; n++) {
    for (size_t s = 0; s < stripes_per_block; s++)
      acc512(acc, in + n * block_len + s * 64, kSecret + s * 8);
    scramble(acc, kSecret + 192 - 64);
  }
  size_t nb_stripes = ((len - 1) - block_len * nb_blocks) / 64;
  for (size_t s = 0; s < nb_stripes; s++)
    acc512(acc, in + nb_blocks * block_len + s * 64, kSecret + s * 8);
  acc512(acc, in + len - 64, kSecret + 192 - 64 - 7);
  uint64_t r = len * P64_1;
  for (int i = 0; i < 4; i++)
    r += mul128_fold64(acc[2 * i] ^ rd64(kSecret + 11 + 16 * i),
                       acc[2 * i + 1] ^ rd64(kSecret + 11 + 16 * i + 8));
  return xxh3_avalanche(r);
}

/* util/xxhash.h:5304 XXH3_64bits_internal dispatch by length. */
uint64_t orc_xxh3_64(const void* data, size_t n) {
  const uint8_t* in = (const uint8_t*)data;
  if (n <= 16) return xxh3_0to16(in, n);
  if (n <= 128) return xxh3_17to128(in, n);
  if (n <= 240) return xxh3_129to240(in, n);
  return xxh3_long(in, n);
}

/* ------------------------------------------------------------------ */
/* XXPH3 -- the XXH3 *preview* (v0.7.2) behind Hash64 / NPHash64        */
/* (util/xxph3.h, util/hash.cc:81-88).  Same default secret as XXH3     */
/* (util/xxph3.h:924), but its own length classes, avalanche constant, */
/* non-swapping accumulate and block/last-stripe rules.                */
/* ------------------------------------------------------------------ */

/* primes P32_* / P64_* as above (util/xxph3.h:568-650, same values) */

/* util/xxph3.h:1073 XXPH3_avalanche */
static uint64_t xxph3_avalanche(uint64_t h) {
  h ^= h >> 37;
  h *= P64_3;
  return h ^ (h >> 32);
}

/* util/xxph3.h:1086-1147 XXPH3_len_0to16_64b (incl. the RocksDB change for
 * len 0 at 1139-1142) */
static uint64_t xxph3_0to16(const uint8_t* in, size_t len, const uint8_t* sec, uint64_t seed) {
  if (len > 8) {
    uint64_t lo = rd64(in) ^ (rd64(sec) + seed);
    uint64_t hi = rd64(in + len - 8) ^ (rd64(sec + 8) - seed);
    return xxph3_avalanche(len + (lo + hi) + mul128_fold64(lo, hi));
  }
  if (len >= 4) {
    uint64_t in64 = (uint64_t)rd32(in) | ((uint64_t)rd32(in + len - 4) << 32);
    uint64_t keyed = in64 ^ (rd64(sec) + seed);
    uint64_t mix = len + ((keyed ^ (keyed >> 51)) * P32_1);
    return xxph3_avalanche((mix ^ (mix >> 47)) * P64_2);
  }
  if (len) {
    uint32_t comb = (uint32_t)in[0] | ((uint32_t)in[len >> 1] << 8) | ((uint32_t)in[len - 1] << 16) |
                    ((uint32_t)len << 24);
    uint64_t keyed = (uint64_t)comb ^ ((uint64_t)rd32(sec) + seed);
    return xxph3_avalanche(keyed * P64_1);
  }
  return mul128_fold64(seed + rd64(sec), P64_2);
}

/* util/xxph3.h:1644 XXPH3_mix16B */
static uint64_t xxph3_mix16(const uint8_t* in, const uint8_t* sec, uint64_t seed) {
  return mul128_fold64(rd64(in) ^ (rd64(sec) + seed), rd64(in + 8) ^ (rd64(sec + 8) - seed));
}

/* util/xxph3.h:1655 XXPH3_len_17to128_64b */
static uint64_t xxph3_17to128(const uint8_t* in, size_t len, uint64_t seed) {
  uint64_t acc = len * P64_1;
  if (len > 32) {
    if (len > 64) {
      if (len > 96) {
        acc += xxph3_mix16(in + 48, kSecret + 96, seed);
        acc += xxph3_mix16(in + len - 64, kSecret + 112, seed);
      }
      acc += xxph3_mix16(in + 32, kSecret + 64, seed);
      acc += xxph3_mix16(in + len - 48, kSecret + 80, seed);
    }
    acc += xxph3_mix16(in + 16, kSecret + 32, seed);
    acc += xxph3_mix16(in + len - 32, kSecret + 48, seed);
  }
  acc += xxph3_mix16(in, kSecret, seed);
  acc += xxph3_mix16(in + len - 16, kSecret + 16, seed);
  return xxph3_avalanche(acc);
}

/* util/xxph3.h:1685 XXPH3_len_129to240_64b */
static uint64_t xxph3_129to240(const uint8_t* in, size_t len, uint64_t seed) {
  uint64_t acc = len * P64_1;
  int rounds = (int)len / 16, i;
  for (i = 0; i < 8; i++) acc += xxph3_mix16(in + 16 * i, kSecret + 16 * i, seed);
  acc = xxph3_avalanche(acc);
  for (i = 8; i < rounds; i++) acc += xxph3_mix16(in + 16 * i, kSecret + 16 * (i - 8) + 3, seed);
  acc += xxph3_mix16(in + len - 16, kSecret + 136 - 17, seed);
  return xxph3_avalanche(acc);
}

/* util/xxph3.h:1330-1344 scalar accumulate_512, XXPH3_acc_64bits (no lane
 * swap) */
static void xxph3_acc512(uint64_t acc[8], const uint8_t* in, const uint8_t* sec) {
  for (int i = 0; i < 8; i++) {
    uint64_t d = rd64(in + 8 * i), k = d ^ rd64(sec + 8 * i);
    acc[i] += d;
    acc[i] += (k & 0xFFFFFFFFu) * (k >> 32);
  }
}

/* util/xxph3.h:1516-1543 hashLong_internal_loop + 1574-1587 merge, over a
 * 192-byte secret */
static uint64_t xxph3_long(const uint8_t* in, size_t len, const uint8_t* sec) {
  uint64_t acc[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
  const size_t block = 1024, nb = len / block;
  size_t n, s;
  for (n = 0; n < nb; n++) {
    for (s = 0; s < 16; s++) xxph3_acc512(acc, in + n * block + 64 * s, sec + 8 * s);
    scramble(acc, sec + 128);
  }
  size_t stripes = (len - nb * block) / 64;
  for (s = 0; s < stripes; s++) xxph3_acc512(acc, in + nb * block + 64 * s, sec + 8 * s);
  if (len & 63) xxph3_acc512(acc, in + len - 64, sec + 192 - 64 - 7);
  uint64_t r = len * P64_1;
  for (int i = 0; i < 4; i++) r += mul128_fold64(acc[2 * i] ^ rd64(sec + 11 + 16 * i),
                                                 acc[2 * i + 1] ^ rd64(sec + 19 + 16 * i));
  return xxph3_avalanche(r);
}

/* util/xxph3.h:1737-1744 XXPH3_64bits_withSeed (long inputs with a seed use
 * the custom secret of XXPH3_initCustomSecret, 1613-1624) */
uint64_t orc_hash64(const void* data, size_t n, uint64_t seed) {
  const uint8_t* in = (const uint8_t*)data;
  if (n <= 16) return xxph3_0to16(in, n, kSecret, seed);
  if (n <= 128) return xxph3_17to128(in, n, seed);
  if (n <= 240) return xxph3_129to240(in, n, seed);
  if (seed == 0) return xxph3_long(in, n, kSecret);
  uint8_t sec[192];
  for (int i = 0; i < 12; i++) {
    uint64_t a = rd64(kSecret + 16 * i) + seed, b = rd64(kSecret + 16 * i + 8) - seed;
    memcpy(sec + 16 * i, &a, 8);
    memcpy(sec + 16 * i + 8, &b, 8);
  }
  return xxph3_long(in, n, sec);
}

/* db/kv_checksum.h:84-88 seeds; ProtectKV 324-331, ProtectKVO 296-306,
 * ProtectS 456-462, ProtectC 432-438.  Fields hashed with NPHash64 and
 * XORed; op type is 1 byte, the seqno 8 bytes LE, the CF id 4 bytes LE. */
uint64_t orc_kv_protect(int mode, const void* key, size_t kn, const void* value, size_t vn,
                        uint8_t op, uint64_t extra) {
  uint64_t v = orc_hash64(key, kn, 0) ^ orc_hash64(value, vn, 0xD28AAD72F49BD50BULL);
  if (mode >= 1) v ^= orc_hash64(&op, 1, 0xA5155AE5E937AA16ULL);
  if (mode == 2) {
    uint8_t b[8];
    memcpy(b, &extra, 8);
    v ^= orc_hash64(b, 8, 0x77A00858DDD37F21ULL);
  } else if (mode == 3) {
    uint32_t cf = (uint32_t)extra;
    v ^= orc_hash64(&cf, 4, 0x4A2AB5CBD26F542CULL);
  }
  return v;
}

/* ------------------------------------------------------------------ */
/* Block trailer / WAL record semantics                                */
/* ------------------------------------------------------------------ */

/* table/format.cc:569-575 ModifyChecksumForLastByte. */
static inline uint32_t modify_last_byte(uint32_t v, uint8_t b) {
  return v ^ (uint32_t)b * 0x6b9083d9u;
}

/* table/format.cc:578-602 ComputeBuiltinChecksum. */
uint32_t orc_builtin_checksum(int type, const void* data, size_t n) {
  const uint8_t* p = (const uint8_t*)data;
  switch (type) {
    case ORC_kCRC32c:
      return orc_crc32c_mask(orc_crc32c_value(p, n));
    case ORC_kxxHash:
      return orc_xxh32(p, n, 0);
    case ORC_kxxHash64:
      return (uint32_t)orc_xxh64(p, n, 0);
    case ORC_kXXH3:
      if (n == 0) return 0;
      return modify_last_byte((uint32_t)orc_xxh3_64(p, n - 1), p[n - 1]);
    default:
      return 0;
  }
}

/* table/format.cc:604-645 ComputeBuiltinChecksumWithLastByte: equal to the
 * plain function over data||last_byte (table/table_test.cc:2297-2300). */
uint32_t orc_builtin_checksum_with_last_byte(int type, const void* data,
                                             size_t n, uint8_t last_byte) {
  const uint8_t* p = (const uint8_t*)data;
  switch (type) {
    case ORC_kCRC32c:
      return orc_crc32c_mask(
          orc_crc32c_extend(orc_crc32c_value(p, n), &last_byte, 1));
    case ORC_kXXH3:
      return modify_last_byte((uint32_t)orc_xxh3_64(p, n), last_byte);
    case ORC_kxxHash:
    case ORC_kxxHash64: {
      /* streaming over data||last_byte; restated as one contiguous pass */
      uint8_t stackbuf[4096];
      uint8_t* tmp = stackbuf;
      uint8_t* heap = 0;
      if (n + 1 > sizeof(stackbuf)) {
        heap = (uint8_t*)malloc(n + 1);
        tmp = heap;
      }
      memcpy(tmp, p, n);
      tmp[n] = last_byte;
      uint32_t v = type == ORC_kxxHash ? orc_xxh32(tmp, n + 1, 0)
                                       : (uint32_t)orc_xxh64(tmp, n + 1, 0);
      if (heap) {
        free(heap);
      }
      return v;
    }
    default:
      return 0;
  }
}

/* table/format.h:119-146 ChecksumModifierForContext. */
uint32_t orc_context_modifier(uint32_t base, uint64_t offset) {
  uint32_t all_or_nothing = 0u - (uint32_t)(base != 0);
  uint32_t m = base ^ ((uint32_t)offset + (uint32_t)(offset >> 32));
  return m & all_or_nothing;
}

/* table/block_based/reader_common.cc:26-63 VerifyBlockChecksum. */
int orc_verify_block(int type, const void* block, size_t payload_len,
                     uint32_t base, uint64_t offset, uint32_t* stored_out,
                     uint32_t* computed_out) {
  const uint8_t* p = (const uint8_t*)block;
  size_t len = payload_len + 1;
  uint32_t stored = rd32(p + len);
  uint32_t computed = orc_builtin_checksum(type, p, len);
  stored -= orc_context_modifier(base, offset);
  if (stored_out) *stored_out = stored;
  if (computed_out) *computed_out = computed;
  return stored == computed;
}

/* db/log_writer.cc:263-311 EmitPhysicalRecord + type_crc_ (48-51):
 * crc = Value(&type, 1); recyclable: Extend(crc, LE32(log_number), 4);
 * crc = Crc32cCombine(crc, Value(payload, n), n); Mask(crc). */
uint32_t orc_wal_record_crc(uint8_t type, const void* payload, size_t n,
                            int recyclable, uint32_t log_number) {
  uint32_t crc = orc_crc32c_value(&type, 1);
  if (recyclable) {
    uint8_t ln[4] = {(uint8_t)log_number, (uint8_t)(log_number >> 8),
                     (uint8_t)(log_number >> 16), (uint8_t)(log_number >> 24)};
    crc = orc_crc32c_extend(crc, ln, 4);
  }
  crc = orc_crc32c_combine(crc, orc_crc32c_value(payload, n), n);
  return orc_crc32c_mask(crc);
}

/* util/file_checksum_helper.h:22-46 FileChecksumGenCrc32c */
void orc_file_checksum_crc32c(const void* data, size_t n, uint8_t out[4]) {
  const uint32_t c = orc_crc32c_extend(0, data, n);
  out[0] = (uint8_t)(c >> 24);
  out[1] = (uint8_t)(c >> 16);
  out[2] = (uint8_t)(c >> 8);
  out[3] = (uint8_t)c;
}

/* ------------------------------------------------------------------ */
/* Per-KV protection of an uncompressed block's entries                */
/* ------------------------------------------------------------------ */

/* util/coding.h GetVarint32Ptr / GetVarint64Ptr: NULL when the varint runs
 * past limit or past 5 / 10 bytes. */
static const uint8_t* orc_varint(const uint8_t* p, const uint8_t* limit, int max_shift, uint64_t* v) {
  uint64_t r = 0;
  for (int shift = 0; shift <= max_shift && p < limit; shift += 7) {
    uint64_t b = *p++;
    if (b & 128) {
      r |= (b & 127) << shift;
    } else {
      *v = r | (b << shift);
      return p;
    }
  }
  return 0;
}

/* table/block_based/block.cc:994-1027 NumRestarts / IndexType and the Block
 * constructor (:1036-1083): the restart array offset, or -1 for the
 * constructor's error marker (size_ = 0).  Hash-index footers (bit 31) only
 * for blocks <= kMaxBlockSizeSupportedByHashIndex (64 KiB). */
static int64_t orc_block_restarts(const uint8_t* d, uint32_t size, uint32_t* num_restarts) {
  *num_restarts = 0;
  if (size < 4) return -1;
  uint32_t footer = rd32(d + size - 4);
  int hash = 0;
  uint32_t n = footer;
  if (size <= (1u << 16)) {
    hash = (footer >> 31) & 1;
    n = footer & 0x7FFFFFFFu;
  }
  *num_restarts = n;
  if (!hash) {
    uint32_t ro = size - (1 + n) * 4u;
    if (ro > size - 4u) return -1;
    return ro;
  }
  if (size < 6) return -1;
  /* data_block_hash_index.cc:76-84 Initialize (NUM_BUCK u16 before the footer) */
  uint16_t sz16 = (uint16_t)(size - 4);
  uint16_t nb = (uint16_t)(d[sz16 - 2] | (d[sz16 - 1] << 8));
  uint16_t map_offset = (uint16_t)(sz16 - 2 - nb);
  uint32_t ro = (uint32_t)map_offset - n * 4u;
  if (ro > map_offset) return -1;
  return ro;
}

/* One entry at p (table/block_based/block.cc:37-64 DecodeEntry, :68-97
 * CheckAndDecodeEntry, :110-139 DecodeEntryV4 + :719-727 DecodeCurrentValue /
 * table/format.cc:137-162 IndexValue::DecodeFrom for delta-encoded index
 * values).  Returns the key delta's start, or NULL ("bad entry in block"). */
static const uint8_t* orc_block_entry(int kind, const uint8_t* p, const uint8_t* limit, uint32_t* shared,
                                      uint32_t* non_shared, const uint8_t** val, uint32_t* vlen) {
  uint64_t s, ns, vl = 0;
  if (limit - p < 3) return 0;
  if (kind == ORC_BLOCK_INDEX_DELTA || kind == ORC_BLOCK_INDEX_DELTA_FIRST_KEY) {
    if ((p = orc_varint(p, limit, 28, &s)) == 0) return 0;
    if ((p = orc_varint(p, limit, 28, &ns)) == 0) return 0;
    if ((uint64_t)(limit - p) < ns) return 0;
    const uint8_t* v = p + ns;
    const uint8_t* q = v;
    uint64_t x;
    if (s != 0) { /* delta-encoded size (GetVarsignedint64) */
      if ((q = orc_varint(q, limit, 63, &x)) == 0) return 0;
    } else { /* BlockHandle::DecodeFrom: offset, size */
      if ((q = orc_varint(q, limit, 63, &x)) == 0) return 0;
      if ((q = orc_varint(q, limit, 63, &x)) == 0) return 0;
    }
    if (kind == ORC_BLOCK_INDEX_DELTA_FIRST_KEY) { /* GetLengthPrefixedSlice */
      if ((q = orc_varint(q, limit, 28, &x)) == 0) return 0;
      if ((uint64_t)(limit - q) < x) return 0;
      q += x;
    }
    *shared = (uint32_t)s;
    *non_shared = (uint32_t)ns;
    *val = v;
    *vlen = (uint32_t)(q - v);
    return p;
  }
  if ((p = orc_varint(p, limit, 28, &s)) == 0) return 0;
  if ((p = orc_varint(p, limit, 28, &ns)) == 0) return 0;
  if ((p = orc_varint(p, limit, 28, &vl)) == 0) return 0;
  if ((uint64_t)(limit - p) < ns + vl) return 0;
  *shared = (uint32_t)s;
  *non_shared = (uint32_t)ns;
  *val = p + ns;
  *vlen = (uint32_t)vl;
  return p;
}

/* table/block_based/block.cc:1091-1132 Block::InitializeDataBlockProtectionInfo
 * (:1134-1181 Index, :1183-1222 MetaIndex): walk the entries in order,
 * reassembling every key from the previous one (ParseNextKey :617-665), and
 * write ProtectionInfo64().ProtectKV(key, value).Encode(prot_bytes)
 * (block.h:271-274) per entry.  GetRestartInterval (block.h:484-497) and
 * NumberOfKeys (:500-512) size the output.  The reference only asserts what
 * BlockBuilder guarantees (block_builder.cc:188-252: restart array sorted and
 * on entry starts, shared == 0 at every restart point, every interval but the
 * last holding exactly block_restart_interval entries); this restatement, like
 * the engine, reports a block breaking it as ORC_BLOCK_BAD_RESTARTS. */
int orc_block_kv_protect(int kind, const void* block, size_t n, uint32_t prot_bytes, uint8_t* out,
                         size_t out_cap, uint32_t* nkeys_out, uint32_t* interval_out) {
  const uint8_t* d = (const uint8_t*)block;
  *nkeys_out = 0;
  if (interval_out) *interval_out = 0;
  if (n > 0xFFFFFFFFu) return ORC_BLOCK_BAD_CONTENTS;
  uint32_t nr;
  int64_t ro = orc_block_restarts(d, (uint32_t)n, &nr);
  if (ro < 0) return ORC_BLOCK_BAD_CONTENTS;
  if (nr == 0) return ORC_BLOCK_OK; /* protection_bytes_per_key_ stays 0 */
  if (n < 8) return ORC_BLOCK_BAD_CONTENTS; /* NewDataIterator: "bad block contents" */
  const uint8_t* limit = d + ro;
  const uint8_t* ra = d + ro;
  /* restart array as BlockBuilder writes it */
  if (ro != 0 && rd32(ra) != 0) return ORC_BLOCK_BAD_RESTARTS;
  for (uint32_t r = 1; r < nr; r++)
    if (rd32(ra + 4 * r) <= rd32(ra + 4 * (r - 1)) || rd32(ra + 4 * r) >= ro) return ORC_BLOCK_BAD_RESTARTS;
  if (ro == 0) return nr == 1 ? ORC_BLOCK_OK : ORC_BLOCK_BAD_RESTARTS; /* no entries */
  uint8_t* key = 0;
  size_t kcap = 0, klen = 0;
  uint32_t idx = 0, interval = 0, in_cur = 0, r = 0;
  const uint8_t* p = d;
  int st = ORC_BLOCK_OK;
  while (p < limit) {
    const uint32_t off = (uint32_t)(p - d);
    const int at_restart = r < nr && off == rd32(ra + 4 * r);
    if (r < nr && off > rd32(ra + 4 * r)) { st = ORC_BLOCK_BAD_RESTARTS; break; } /* restart inside an entry */
    if (at_restart) {
      if (r == 1) interval = in_cur;
      else if (r > 1 && in_cur != interval) { st = ORC_BLOCK_BAD_RESTARTS; break; }
      in_cur = 0;
      r++;
    }
    uint32_t sh, ns, vl;
    const uint8_t* v;
    const uint8_t* q = orc_block_entry(kind, p, limit, &sh, &ns, &v, &vl);
    if (!q) { st = ORC_BLOCK_BAD_ENTRY; break; }
    /* shared != 0 at a restart point: the first entry of the block has no key
     * to share with (ParseNextKey's raw_key_.Size() < shared); later ones
     * would reuse the previous interval's key (not a BlockBuilder layout) */
    if (at_restart && sh != 0) { st = r == 1 ? ORC_BLOCK_BAD_ENTRY : ORC_BLOCK_BAD_RESTARTS; break; }
    if (klen < sh) { st = ORC_BLOCK_BAD_ENTRY; break; }
    if (sh + (size_t)ns > kcap) {
      kcap = 2 * (sh + (size_t)ns) + 64;
      key = (uint8_t*)realloc(key, kcap);
    }
    memcpy(key + sh, q, ns); /* TrimAppend(shared, p, non_shared) */
    klen = sh + (size_t)ns;
    const uint64_t h = orc_kv_protect(0, key, klen, v, vl, 0, 0);
    if ((size_t)(idx + 1) * prot_bytes <= out_cap)
      for (uint32_t b = 0; b < prot_bytes; b++) out[(size_t)idx * prot_bytes + b] = (uint8_t)(h >> (8 * b));
    idx++;
    in_cur++;
    p = v + vl;
  }
  free(key);
  if (st == ORC_BLOCK_OK && r != nr) st = ORC_BLOCK_BAD_RESTARTS; /* restarts past the last entry */
  if (st != ORC_BLOCK_OK) return st;
  if (nr == 1) interval = 0; /* GetRestartInterval: 0 for a single restart */
  *nkeys_out = idx;
  if (interval_out) *interval_out = interval;
  return ORC_BLOCK_OK;
}
