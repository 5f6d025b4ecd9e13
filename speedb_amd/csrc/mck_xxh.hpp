// mck_xxh.hpp -- device XXH3-64 (wave per span) and legacy XXH32/XXH64
// (lane per span), xxHash v0.8.1 as vendored at util/xxhash.h.
//
// XXH3 long inputs (n > 240, util/xxhash.h:5141-5227): 8 u64 accumulators;
// each 1 KiB segment = 16 stripes x 64 B; within a segment the 128
// (stripe, accumulator-lane) terms are independent sums mod 2^64, so the
// wave computes them in parallel: lane l owns stripe l>>2 and accumulator
// pair q = l&3 (16 contiguous bytes per lane => one coalesced 1 KiB load per
// segment).  The per-segment sums are reduced across the 16 stripe lanes and
// then applied in order with the (nonlinear, sequential) scramble.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mck {

constexpr uint64_t P64_1 = 0x9E3779B185EBCA87ull, P64_2 = 0xC2B2AE3D27D4EB4Full,
                   P64_3 = 0x165667B19E3779F9ull, P64_4 = 0x85EBCA77C2B2AE63ull,
                   P64_5 = 0x27D4EB2F165667C5ull;
constexpr uint32_t P32_1 = 0x9E3779B1u, P32_2 = 0x85EBCA77u, P32_3 = 0xC2B2AE3Du,
                   P32_4 = 0x27D4EB2Fu, P32_5 = 0x165667B1u;

// XXH3_kSecret, util/xxhash.h:3661-3674 (192 bytes)
__constant__ const uint8_t kXxh3Secret[192] = {
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

__device__ __forceinline__ uint64_t sec64(int off) {
  uint64_t v = 0;
#pragma unroll
  for (int b = 7; b >= 0; b--) v = (v << 8) | kXxh3Secret[off + b];
  return v;
}
__device__ __forceinline__ uint32_t sec32(int off) {
  uint32_t v = 0;
#pragma unroll
  for (int b = 3; b >= 0; b--) v = (v << 8) | kXxh3Secret[off + b];
  return v;
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

// Per-lane secret words for the long path.
struct XxhLane {
  uint64_t k0, k1;    // stripe secret for accumulators 2q, 2q+1 of stripe st
  uint64_t ks0, ks1;  // scramble secret (offset 128)
  uint64_t kl0, kl1;  // last-stripe secret (offset 121)
  uint64_t km0, km1;  // merge secret (offset 11)
  uint64_t i0, i1;    // XXH3_INIT_ACC for 2q, 2q+1
  int lane, st, q;
};
__device__ __forceinline__ XxhLane xxh_lane() {
  XxhLane X;
  X.lane = threadIdx.x & 63;
  X.st = X.lane >> 2;
  X.q = X.lane & 3;
  X.k0 = sec64(8 * X.st + 16 * X.q);
  X.k1 = sec64(8 * X.st + 16 * X.q + 8);
  X.ks0 = sec64(128 + 16 * X.q);
  X.ks1 = sec64(136 + 16 * X.q);
  X.kl0 = sec64(121 + 16 * X.q);
  X.kl1 = sec64(129 + 16 * X.q);
  X.km0 = sec64(11 + 16 * X.q);
  X.km1 = sec64(19 + 16 * X.q);
  // INIT_ACC = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1}
  const uint64_t init[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
  X.i0 = X.q == 0 ? init[0] : X.q == 1 ? init[2] : X.q == 2 ? init[4] : init[6];
  X.i1 = X.q == 0 ? init[1] : X.q == 1 ? init[3] : X.q == 2 ? init[5] : init[7];
  return X;
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int o) {
  const uint32_t lo = __shfl_xor((uint32_t)v, o, 64), hi = __shfl_xor((uint32_t)(v >> 32), o, 64);
  return ((uint64_t)hi << 32) | lo;
}
// sum over the 16 stripe lanes sharing q (lane bits 2..5)
__device__ __forceinline__ uint64_t sum_stripes(uint64_t v) {
  v += shfl_xor64(v, 4);
  v += shfl_xor64(v, 8);
  v += shfl_xor64(v, 16);
  v += shfl_xor64(v, 32);
  return v;
}
__device__ __forceinline__ uint64_t xxh3_scramble(uint64_t a, uint64_t k) {
  a ^= a >> 47;
  a ^= k;
  return a * P32_1;
}

// XXH3_64bits of [in, in+len), len > 240; all lanes of the wave call it and
// all return the hash.
__device__ __forceinline__ uint64_t xxh3_long_wave(const uint8_t* in, uint64_t len, const XxhLane& X) {
  uint64_t a0 = X.i0, a1 = X.i1;
  const uint64_t nb = (len - 1) / 1024;                          // full segments
  const int nstripes = (int)(((len - 1) - 1024 * nb) / 64);      // in the last one
  for (uint64_t g0 = 0; g0 <= nb; g0 += 4) {
    uint4 d[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint64_t g = g0 + j;
      const bool act = g < nb || (g == nb && X.st < nstripes);
      d[j] = act ? *reinterpret_cast<const uint4*>(in + 1024 * g + 16 * X.lane) : make_uint4(0, 0, 0, 0);
    }
    uint64_t c0[4], c1[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint64_t g = g0 + j;
      const bool act = g < nb || (g == nb && X.st < nstripes);
      const uint64_t d0 = ((uint64_t)d[j].y << 32) | d[j].x, d1 = ((uint64_t)d[j].w << 32) | d[j].z;
      c0[j] = act ? d1 + mul32to64(d0 ^ X.k0) : 0;
      c1[j] = act ? d0 + mul32to64(d1 ^ X.k1) : 0;
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
      c0[j] = sum_stripes(c0[j]);
      c1[j] = sum_stripes(c1[j]);
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint64_t g = g0 + j;
      if (g <= nb) {
        a0 += c0[j];
        a1 += c1[j];
        if (g < nb) {
          a0 = xxh3_scramble(a0, X.ks0);
          a1 = xxh3_scramble(a1, X.ks1);
        }
      }
    }
  }
  {  // last stripe at in + len - 64, secret + 121
    const uint8_t* p = in + len - 64 + 16 * X.q;
    const uint64_t d0 = rd64(p), d1 = rd64(p + 8);
    a0 += d1 + mul32to64(d0 ^ X.kl0);
    a1 += d0 + mul32to64(d1 ^ X.kl1);
  }
  uint64_t m = mul128_fold64(a0 ^ X.km0, a1 ^ X.km1);
  m += shfl_xor64(m, 1);
  m += shfl_xor64(m, 2);
  return xxh3_avalanche(len * P64_1 + m);
}

__device__ __forceinline__ uint64_t xxh3_wave(const uint8_t* in, uint64_t len, const XxhLane& X) {
  if (len <= 240) return __shfl(X.lane == 0 ? xxh3_short(in, len) : 0ull, 0, 64);
  return xxh3_long_wave(in, len, X);
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
