// mck_kernels.hpp -- kernel templates and the per-call "ops" that bind the
// generic CRC32C / XXH3 / XXH32 / XXH64 span engines to the reference's
// call-site semantics (table/format.cc:578-645, block_based_table_builder.cc
// :1333-1348, reader_common.cc:26-63, log_writer.cc:263-311).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mck_crc.hpp"
#include "mck_crc_bh.hpp"
#include "mck_xxh.hpp"

namespace mck {

extern __device__ CrcTables g_crc_tables;
constexpr uint32_t kRandomPrime = 0x6b9083d9u;  // table/format.cc:573

// ---- span source: the mck_spans descriptor --------------------------------
// Descriptor loads go through global (address_space(1)) pointers: written
// as `lengths ? lengths[i] : length` the compiler may select between the
// array and the kernel argument's own address and issue a FLAT load, which
// also counts in lgkmcnt -- every LDS wait of the table steps then waits for
// that memory load too.
typedef __attribute__((address_space(1))) const uint32_t gdesc_u32_t;
typedef __attribute__((address_space(1))) const uint64_t gdesc_u64_t;
typedef __attribute__((address_space(1))) const uint8_t gdesc_u8_t;
__device__ __forceinline__ uint32_t ldg_u32(const uint32_t* p, uint32_t i) {
  return *reinterpret_cast<gdesc_u32_t*>(reinterpret_cast<uint64_t>(p + i));
}
__device__ __forceinline__ uint64_t ldg_u64(const uint64_t* p, uint32_t i) {
  return *reinterpret_cast<gdesc_u64_t*>(reinterpret_cast<uint64_t>(p + i));
}
__device__ __forceinline__ uint8_t ldg_u8(const uint8_t* p, uint32_t i) {
  return *reinterpret_cast<gdesc_u8_t*>(reinterpret_cast<uint64_t>(p + i));
}

struct SpanSrc {
  const uint8_t* base;
  const uint64_t* offsets;
  const uint32_t* lengths;
  uint64_t stride;
  uint32_t length;
  __device__ __forceinline__ uint64_t off(uint32_t i) const {
    return offsets ? ldg_u64(offsets, i) : (uint64_t)i * stride;
  }
  __device__ __forceinline__ uint64_t len(uint32_t i) const { return lengths ? ldg_u32(lengths, i) : length; }
  __device__ __forceinline__ const uint8_t* ptr(uint32_t i) const { return base + off(i); }
};



// table/format.h:119-146 ChecksumModifierForContext
__device__ __forceinline__ uint32_t context_modifier(uint32_t base, uint64_t offset) {
  const uint32_t all_or_nothing = 0u - (uint32_t)(base != 0);
  return (base ^ ((uint32_t)offset + (uint32_t)(offset >> 32))) & all_or_nothing;
}

__device__ __forceinline__ uint32_t rd32_bytes(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// What a block op does with a block's builtin checksum.
enum BlockMode : int {
  kModeBuiltin = 0,  // out[i] = builtin(span, last?)
  kModeTrailer = 1,  // out[i] = builtin(span, comp[i]) + modifier(file offset)
  kModeVerify = 2,   // span+type byte vs stored LE32 (context removed)
};

struct BlockArgs {
  SpanSrc s;
  const uint8_t* last;     // builtin: optional last bytes; trailer: comp types
  const uint64_t* foff;    // trailer/verify: file offsets (NULL = s.off)
  uint32_t base_ctx;       // base_context_checksum
  uint32_t* out;           // builtin/trailer result; verify: computed (opt)
  uint8_t* mismatch;       // verify
  uint32_t* stored;        // verify (opt)
  uint32_t* mismatch_count;  // verify (opt)
  unsigned long long* stats_mismatch = nullptr;  // verify: the engine's per-device BLOCK_CHECKSUM_MISMATCH_COUNT (64-bit)
};

// Epilogue inputs of a block op, loaded by the driver together with the
// span's data (software-pipelined drivers issue them before folding the
// current unit), so the epilogue never issues a dependent load that would
// wait behind the next unit's prefetch (vmcnt retires in order):
//   at = address of the byte after the hashed span (verify: type byte, then
//        the stored LE32; XXH3 builtin: the last checksummed byte)
//   two aligned dwords around it, the file offset, last[i].
struct BlockPre {
  uint32_t w0, w1;
  uint32_t sh;  // (at & 3) * 8
  uint32_t last;
  uint64_t foff;
  __device__ __forceinline__ uint64_t bytes() const { return (((uint64_t)w1 << 32) | w0) >> sh; }
};
typedef __attribute__((address_space(1))) const uint32_t gbl_u32_t;
typedef __attribute__((address_space(1))) const uint64_t gbl_u64_t;
typedef __attribute__((address_space(1))) const uint8_t gbl_u8_t;
// at: device address; off = the span's offset from the batch base.  Verify
// reads the 8 bytes at floor4(at) (type byte + stored LE32 lie inside them:
// never past the 4-byte word holding the trailer's last byte); the other
// modes read only the dword holding byte `at` where they need it.
template <int MODE>
__device__ __forceinline__ BlockPre block_pre(const BlockArgs& a, uint32_t i, uint64_t at, uint64_t off,
                                              bool need_at) {
  BlockPre e;
  const uint64_t a4 = at & ~3ull;
  e.sh = (uint32_t)(at & 3) * 8;
  e.w0 = need_at ? *reinterpret_cast<gbl_u32_t*>(a4) : 0u;
  e.w1 = MODE == kModeVerify ? *reinterpret_cast<gbl_u32_t*>(a4 + 4) : 0u;
  e.last = (MODE == kModeTrailer || (MODE == kModeBuiltin && a.last)) ? *reinterpret_cast<gbl_u8_t*>(reinterpret_cast<uint64_t>(a.last + i)) : 0u;
  e.foff = MODE == kModeBuiltin ? 0 : a.foff ? *reinterpret_cast<gbl_u64_t*>(reinterpret_cast<uint64_t>(a.foff + i)) : off;
  return e;
}

// Verify / trailer epilogue shared by every hash kind.  `v` = builtin value.
template <int MODE>
__device__ __forceinline__ void block_epilogue(const BlockArgs& a, uint32_t i, uint32_t v, const BlockPre& e) {
  if (MODE == kModeBuiltin) {
    a.out[i] = v;
  } else if (MODE == kModeTrailer) {
    a.out[i] = v + context_modifier(a.base_ctx, e.foff);
  } else {
    const uint32_t stored = (uint32_t)(e.bytes() >> 8) - context_modifier(a.base_ctx, e.foff);
    const bool bad = stored != v;
    a.mismatch[i] = bad;
    if (a.out) a.out[i] = v;
    if (a.stored) a.stored[i] = stored;
    if (bad && a.mismatch_count) atomicAdd(a.mismatch_count, 1u);
    if (bad && a.stats_mismatch) atomicAdd(a.stats_mismatch, 1ull);
  }
}
// Same, with the inputs loaded here (drivers without epilogue prefetch).
template <int MODE>
__device__ __forceinline__ void block_epilogue(const BlockArgs& a, uint32_t i, uint32_t v) {
  const uint64_t off = a.s.off(i);
  block_epilogue<MODE>(a, i, v,
                       block_pre<MODE>(a, i, reinterpret_cast<uint64_t>(a.s.base) + off + a.s.len(i), off,
                                       MODE == kModeVerify));
}

struct NoPre {};

// ============================ CRC32C ======================================
// CRC ops: the generic driver calls pre(i, ptr, len) with the span's
// last-round loads and finish(i, crc, pre) after its last round.
struct OpCrcValue {
  SpanSrc s;
  const uint32_t* init;
  uint32_t flags;
  uint32_t* out;
  typedef NoPre Pre;
  static constexpr bool kArrayInit = true;  // per-span inits: the row loop un-shifts them (no rowfin8)
  __device__ const uint8_t* base() const { return s.base; }
  __device__ uint64_t off(uint32_t i) const { return s.off(i); }
  __device__ uint64_t len(uint32_t i) const { return s.len(i); }
  __device__ uint32_t init_crc(uint32_t i) const { return init ? init[i] : 0u; }
  static constexpr bool kTypedInit = false;
  __device__ int init_kind() const { return init ? kInitArray : kInitZero; }
  __device__ uint32_t init_key(uint32_t i) const { return init ? ldg_u32(init, i) : 0u; }
  __device__ uint32_t typed_init(uint32_t) const { return 0u; }
  __device__ Pre pre(uint32_t, uint64_t, uint64_t) const { return Pre{}; }
  __device__ void finish(uint32_t i, uint32_t crc, const Pre&, bool writer) const {
    if (writer) out[i] = (flags & 1u) ? crc_mask(crc) : crc;
  }
};

// OpCrcValue without per-span inits (Value, init 0): the 8-lane rows'
// combined finish maps apply (kRowFin8: no init un-shift at run time)
struct OpCrcValueZ : OpCrcValue {
  static constexpr bool kArrayInit = false;
  __device__ int init_kind() const { return kInitZero; }
  __device__ uint32_t init_key(uint32_t) const { return 0u; }
  __device__ uint32_t init_crc(uint32_t) const { return 0u; }
};

// WAL write side: init = Value(type byte [+ LE32 log number])
struct WalTypeCrcs {
  uint32_t v[16];
};
struct OpCrcWal {
  SpanSrc s;
  const uint8_t* types;
  WalTypeCrcs tc;
  uint32_t* out;
  typedef NoPre Pre;
  __device__ const uint8_t* base() const { return s.base; }
  __device__ uint64_t off(uint32_t i) const { return s.off(i); }
  __device__ uint64_t len(uint32_t i) const { return s.len(i); }
  __device__ uint32_t init_crc(uint32_t i) const { return tc.v[types[i] & 15]; }
  static constexpr bool kTypedInit = true;
  __device__ int init_kind() const { return kInitTyped; }
  __device__ uint32_t init_key(uint32_t i) const { return ldg_u8(types, i); }
  __device__ uint32_t typed_init(uint32_t t) const { return tc.v[t & 15]; }
  __device__ Pre pre(uint32_t, uint64_t, uint64_t) const { return Pre{}; }
  __device__ void finish(uint32_t i, uint32_t crc, const Pre&, bool writer) const {
    if (writer) out[i] = crc_mask(crc);
  }
};

// verify: the CRC span is payload || type byte (len = payload + 1); the
// stored LE32 follows it
template <int MODE>
struct OpCrcBlock {
  static constexpr bool kByteShares = true;  // blocks of a file image, in file order
  BlockArgs a;
  typedef BlockPre Pre;
  __device__ const uint8_t* base() const { return a.s.base; }
  __device__ uint64_t off(uint32_t i) const { return a.s.off(i); }
  __device__ uint64_t len(uint32_t i) const { return a.s.len(i) + (MODE == kModeVerify ? 1 : 0); }
  __device__ uint32_t init_crc(uint32_t) const { return 0u; }
  static constexpr bool kTypedInit = false;
  __device__ int init_kind() const { return kInitZero; }
  __device__ uint32_t init_key(uint32_t) const { return 0u; }
  __device__ uint32_t typed_init(uint32_t) const { return 0u; }
  __device__ Pre pre(uint32_t i, uint64_t ptr, uint64_t len) const {
    // verify: bytes from the type byte (ptr + len - 1) on
    return block_pre<MODE>(a, i, ptr + len - (MODE == kModeVerify ? 1 : 0),
                           ptr - reinterpret_cast<uint64_t>(a.s.base), MODE == kModeVerify);
  }
  __device__ void finish(uint32_t i, uint32_t crc, const Pre& e, bool writer) const {
    if (MODE == kModeTrailer || (MODE == kModeBuiltin && a.last)) crc = crc_extend_byte(crc, (uint8_t)e.last);
    if (writer) block_epilogue<MODE>(a, i, crc_mask(crc), e);
  }
};


// ---- small batches: one wave per span --------------------------------------
// A batch of a few short spans (a MultiGet's <= 32 blocks,
// RetrieveMultipleBlocks) is latency, not bandwidth: the row and body/head
// drivers' descriptor staging, init tables, span scans and barriers are a
// chain of dependent round trips before the first data load.  For at most
// kSmallBatch spans of at most kSmallSpanMax bytes each workgroup instead
// gives every span of its share (<= 16 here) a wave: descriptor and epilogue
// loads issued with the table fill, the first round's loads before its
// stores, then the wave driver's rounds (crc_round), the finish.  Its own instance of k_crc_ragged
// (SMALL): one more path in the bandwidth instance spilled the blob and
// index-block ops' registers.
constexpr uint32_t kSmallBatch = 64, kSmallSpanMax = 16384;
template <class Op>
__device__ __forceinline__ bool crc_share_small(const Op& op, const RowShare& sh) {
  if (sh.n > 16) return false;  // workgroup-uniform
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t len = lane < sh.n ? op.len(sh.idx(lane)) : 0;
  return !wave_any(len > kSmallSpanMax);  // (every wave reads the same lengths)
}
template <class Op>
__device__ __forceinline__ void crc_small_share(const Op& op, const RowShare& sh, uint8_t* lds,
                                                const CrcTables* __restrict__ g) {
  const uint32_t w = threadIdx.x >> 6;
  // table loads and the span's descriptor in flight together; the first
  // round's loads (they need the descriptor) before the table stores (the
  // init state's un-shift reads the tables: after them)
  CrcFill f;
  crc_fill_load<true>(f, g);
  const uint32_t i = sh.idx(w < sh.n ? w : 0);
  const uint64_t ptr = reinterpret_cast<uint64_t>(op.base()) + op.off(i);
  const uint64_t n = op.len(i);
  const typename Op::Pre e = op.pre(i, ptr, n);
  const CrcLane L = crc_lane();
  CrcSpan sp = crc_span<false>(reinterpret_cast<const uint8_t*>(ptr), n, op.init_crc(i));
  Chunk cur = crc_load_chunk<false>(sp, sp.rounds - 1, L);
  crc_fill_store<true>(f, lds);
  __syncthreads();
  if (w >= sh.n) return;  // wave-uniform
  crc_span_inj(sp);
  uint32_t s = 0;
  for (int r = sp.rounds - 1; r >= 0; r--) {  // next round's loads issued first
    const Chunk nxt = crc_load_chunk<false>(sp, r > 0 ? r - 1 : 0, L);
    s = crc_round(s, cur, sp, r, L);
    cur = nxt;
  }
  op.finish(i, crc_finish(s, sp, L), e, (threadIdx.x & 63) == 0);
}

// Ragged batches in ONE launch: each workgroup runs its share on the
// body/head driver or the row drivers (crc_share_long), or, in a small batch,
// a wave per span (crc_share_small).  force: 0 = by length, 7 = body/head for
// every share, 2/3/5/6 = that row width for every share, 8 = row drivers,
// width by length (the interleaved test order), 9 = a wave per span wherever
// crc_share_small allows it (SMALL instances).
// Ops over the spans of one file image in file order (SST blocks, blob
// records) take byte-balanced shares (share_by_bytes) in large batches:
// count-balanced shares of the SST mix differ by up to 1.6x in bytes, and the
// launch ends with the fullest one.
template <class Op, class = void>
struct ByteShares : std::false_type {};
template <class Op>
struct ByteShares<Op, std::void_t<decltype(Op::kByteShares)>> : std::integral_constant<bool, Op::kByteShares> {};
constexpr uint32_t kByteSharesMin = 64;  // spans per workgroup (a small batch keeps count shares: latency)

template <class Op, bool T, bool BLK = true, bool SMALL = false>
__global__ __launch_bounds__(1024) void k_crc_ragged(Op op, uint32_t first, uint32_t count, int force) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  asm volatile("" ::"v"((uint32_t)(size_t)lds));
  RowShare sh = row_share<BLK>(first, count);
  bool filled = false;  // the body/head image is in LDS
  if constexpr (BLK && ByteShares<Op>::value) {
    if (count >= kByteSharesMin * gridDim.x) {  // workgroup-uniform
      // the body/head table loads ride along with the search's first round
      // trip and are stored right after it (the row drivers, should a share
      // take them, fill their own image over it)
      BhFill fill;
      uint32_t lo, hi;
      share_by_bytes(op, first, count, count / gridDim.x, lds_p32(kBLdsWsum), &lo, &hi,
                     [&](uint32_t i) { return (uint32_t)op.off(i) ^ (uint32_t)op.len(i); },
                     [&] { bh_fill_load(fill, &g_crc_tables); });
      bh_fill_store(op, fill);
      // every wave's image stores (the injection tables, which read the
      // un-shift tables) land before anything reuses those LDS bytes: the
      // row drivers' prologue writes its row-gap maps and descriptors there
      __syncthreads();
      sh = RowShare{first + lo, 1u, hi - lo};
      filled = true;
    }
  }
  if (sh.n == 0) return;  // workgroup-uniform
  if constexpr (SMALL) {
    if ((force == 0 || force == 9) && crc_share_small(op, sh)) {
      crc_small_share(op, sh, lds, &g_crc_tables);
      return;
    }
  }
  const bool bh = force == 7 || (force == 0 && BLK && crc_share_long(op, sh));
  if (bh)
    crc_bh_driver<Op, T>(op, sh, &g_crc_tables, filled);
  else
    crc_rows_windows<Op>(op, sh, lds, &g_crc_tables, force == 8 || force == 9 ? 0 : force);
}


// ============================ XXH3 ========================================
// one span per 16-lane row (xxh3_rows_driver) or per wave (xxh3_wave_driver)
template <class Op>
__global__ __launch_bounds__(256) void k_xxh3(Op op, uint32_t count) {
  xxh3_rows_driver(op, count);
}
// Wave driver workgroup: 16 waves, one workgroup per CU.
constexpr int kX3WaveThreads = 1024;
static_assert(kX3WaveThreads / 64 <= kX3MaxWaves, "X3Lds holds a parked-sum buffer per wave");
template <class Op>
__global__ __launch_bounds__(kX3WaveThreads) void k_xxh3_wave(Op op, uint32_t count) {
  xxh3_wave_driver<Op, false>(op, count, 0);
}

// XXH3 ops.  Both drivers call pre(i, ptr, hlen) with the span's loads (the
// wave driver with every unit, the row driver with every segment) and
// finish(i, h, pre); spans <= 240 bytes (hashed on one lane) call
// finish(i, h).
struct OpX3Value {
  SpanSrc s;
  uint64_t* out;
  typedef NoPre Pre;
  __device__ const uint8_t* base() const { return s.base; }
  __device__ uint64_t off(uint32_t i) const { return s.off(i); }
  __device__ uint64_t hlen(uint32_t i) const { return s.len(i); }
  __device__ Pre pre(uint32_t, uint64_t, uint64_t) const { return Pre{}; }
  __device__ void finish(uint32_t i, uint64_t h, const Pre& = Pre{}) const { out[i] = h; }
};

// kXXH3 block checksum (table/format.cc:569-597): lo32(XXH3 of all but the
// last checksummed byte) ^ last byte * kRandomPrime; 0 for empty input.
template <int MODE>
struct OpX3Block {
  BlockArgs a;
  typedef BlockPre Pre;
  __device__ const uint8_t* base() const { return a.s.base; }
  __device__ uint64_t off(uint32_t i) const { return a.s.off(i); }
  __device__ uint64_t hlen(uint32_t i) const {
    const uint64_t n = a.s.len(i);
    // verify: payload || type byte -> hash the payload; trailer / explicit
    // last byte: hash the span; builtin: all but the span's last byte
    if (MODE == kModeVerify || MODE == kModeTrailer || a.last) return n;
    return n ? n - 1 : 0;
  }
  // the byte after the hashed part: verify -- the type byte (then the
  // stored LE32); builtin without last bytes -- the span's last byte
  __device__ Pre pre(uint32_t i, uint64_t ptr, uint64_t hlen) const {
    const bool need = MODE == kModeVerify || (MODE == kModeBuiltin && !a.last);
    return block_pre<MODE>(a, i, ptr + hlen, ptr - reinterpret_cast<uint64_t>(a.s.base), need);
  }
  // (the wave driver hashes only spans > 240 bytes here, never empty ones)
  __device__ void finish(uint32_t i, uint64_t h, const Pre& e) const {
    uint32_t v;
    if (MODE == kModeVerify || (MODE == kModeBuiltin && !a.last))
      v = (uint32_t)h ^ (uint32_t)(e.bytes() & 0xFF) * kRandomPrime;
    else
      v = (uint32_t)h ^ e.last * kRandomPrime;
    block_epilogue<MODE>(a, i, v, e);
  }
  // row driver and short spans: inputs loaded here; an empty builtin span
  // is 0 (table/format.cc:588) and reads nothing
  __device__ void finish(uint32_t i, uint64_t h) const {
    const uint64_t ptr = reinterpret_cast<uint64_t>(a.s.ptr(i));
    if (MODE == kModeBuiltin && !a.last && a.s.len(i) == 0) {
      block_epilogue<MODE>(a, i, 0u, block_pre<MODE>(a, i, ptr, 0, false));
      return;
    }
    finish(i, h, pre(i, ptr, hlen(i)));
  }
};

// ===================== XXPH3: Hash64 / per-KV protection =================
// Same row driver as XXH3, preview rules (util/xxph3.h), seeded.
template <class Op>
__global__ __launch_bounds__(256) void k_xph3(Op op, uint32_t count, uint64_t seed) {
  xxh3_rows_driver<Op, true>(op, count, seed);
}

// Uniform batches of <= 240-byte spans (round 6): one span per lane QUAD
// (the short classes' windows as x3_short_quads: lane q takes windows q,
// q + 4, q + 8, q + 12, keys secret +/- seed, util/xxph3.h:1112-1147), 16
// spans per wave at a time -- the row driver hashed a short span on one
// lane of its row (a uniform batch of 100-byte values: one value per row per
// round trip).  The quad's lane 0 runs the op's epilogue (finish(i, h)).
template <class Op>
__global__ __launch_bounds__(256) void k_xph3_quads(Op op, uint32_t count, uint64_t seed) {
  const uint32_t q = threadIdx.x & 3u;
  const uint32_t nq = gridDim.x * (blockDim.x >> 2);
  X3Short K[4];
#pragma unroll
  for (int k = 0; k < 4; k++) K[k] = x3s_keys(q + 4 * (uint32_t)k, seed);
  const uint64_t base = reinterpret_cast<uint64_t>(op.base());
  for (uint32_t t = blockIdx.x * (blockDim.x >> 2) + (threadIdx.x >> 2); __any(t < count); t += nq) {
    const bool act = t < count;
    const uint32_t i = act ? t : count - 1;
    const uint64_t len = op.hlen(i);
    const uint64_t ptr = base + op.off(i);
    const uint32_t n = (uint32_t)len;  // <= 240: launch_xph3 sends only such batches here
    uint4 d[4];
    bool has[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t o = x3s_off(n, q + 4 * (uint32_t)k, has[k]);
      has[k] = has[k] && act && n > 16;
      d[k] = load16_realign(has[k] ? ptr + o : ptr & ~15ull);
    }
    const bool mid = n <= 128;
    uint64_t s0 = 0, s1 = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint64_t lo = ((uint64_t)d[k].y << 32) | d[k].x, hi = ((uint64_t)d[k].w << 32) | d[k].z;
      const uint64_t v = has[k] ? mul128_fold64(lo ^ (mid ? K[k].a0 : K[k].b0), hi ^ (mid ? K[k].a1 : K[k].b1)) : 0ull;
      if (k < 2)
        s0 += v;
      else
        s1 += v;
    }
    s0 = quad_sum(s0);
    s1 = quad_sum(s1);
    const uint64_t a = (uint64_t)n * P64_1 + s0;
    uint64_t h = mid ? xxph3_avalanche(a + s1) : xxph3_avalanche(xxph3_avalanche(a) + s1);
    if (act && q == 0) {
      if (len <= 16) h = x3_small<true>(reinterpret_cast<const uint8_t*>(ptr), len, seed);
      op.finish(i, h);
    }
  }
}

// util/hash.h:45 NPHash64(data, n, seed) == util/hash.cc:81 Hash64
struct OpXpValue {
  SpanSrc s;
  uint64_t* out;
  typedef NoPre Pre;
  __device__ const uint8_t* base() const { return s.base; }
  __device__ uint64_t off(uint32_t i) const { return s.off(i); }
  __device__ uint64_t hlen(uint32_t i) const { return s.len(i); }
  __device__ Pre pre(uint32_t, uint64_t, uint64_t) const { return Pre{}; }
  __device__ void finish(uint32_t i, uint64_t h, const Pre& = Pre{}) const { out[i] = h; }
};

// db/kv_checksum.h:84-88 field seeds
constexpr uint64_t kSeedK = 0, kSeedV = 0xD28AAD72F49BD50Bull, kSeedO = 0xA5155AE5E937AA16ull,
                   kSeedS = 0x77A00858DDD37F21ull, kSeedC = 0x4A2AB5CBD26F542Cull;

// ProtectionInfo64 of one KV (db/kv_checksum.h): the row driver hashes the
// VALUE (seed kSeedV); finish() XORs in the key (seed 0), and per kind the op
// type (1 byte), seqno (8 bytes LE) or CF id (4 bytes LE).
//   kind 0 ProtectKV (:324), 1 ProtectKVO (:296), 2 ProtectKVO.ProtectS
//   (:456), 3 ProtectKVO.ProtectC (:432)
// VERIFY: ProtectionInfo::Verify(len, stored) (:103-121): the low
// `prot_bytes` bytes of the value against stored[i*prot_bytes ..].
// The row driver issues pre() with the value's loads, so the key bytes (up
// to 16: the first and last 8), op type, seqno / CF id and stored bytes are
// in registers when the value's hash completes (no dependent loads behind
// the next segment's); keys longer than 16 bytes are read in finish().
__device__ const uint64_t g_zero16[2] = {0, 0};
struct KvPre {
  // len >= 8: key bytes [0, 8) and [len - 8, len); len 1..7: the aligned
  // qwords holding the first and the last key byte (no read leaves the
  // pages the key occupies), joined in finish()
  uint64_t k0, k1;
  uint64_t klen;
  uint32_t sh;  // len 1..7: key start & 7
  uint64_t extra;
  uint64_t stored;  // verify: the stored protection bytes, LE
  uint32_t op;
};
// XXPH3 of a key of len <= 16 from its first and last 8 bytes
// (xxph3_short's 0 / 1-3 / 4-8 / 9-16 classes, util/xxph3.h:1390-1445)
__device__ __forceinline__ uint64_t xxph3_le16(uint64_t a, uint64_t b, uint64_t len, uint64_t seed) {
  if (len > 8) {
    const uint64_t lo = a ^ (sec64(0) + seed), hi = b ^ (sec64(8) - seed);
    return xxph3_avalanche(len + (lo + hi) + mul128_fold64(lo, hi));
  }
  if (len >= 4) return xxph3_4to8((uint32_t)a, (uint32_t)(a >> (8 * (len - 4))), len, seed);
  if (len) {
    return xxph3_1to3((uint32_t)(a & 0xFF), (uint32_t)((a >> (8 * (len >> 1))) & 0xFF),
                      (uint32_t)((a >> (8 * (len - 1))) & 0xFF), len, seed);
  }
  return mul128_fold64(seed + sec64(0), P64_2);
}
typedef __attribute__((address_space(1))) const uint64_t gbl_u64u_t;
template <bool VERIFY>
struct OpKvProtect {
  SpanSrc keys, values;
  const uint8_t* ops;
  const uint64_t* extras;
  int kind;
  uint64_t* out;
  const uint8_t* stored;
  uint32_t prot_bytes;
  uint8_t* mismatch;
  uint32_t* mismatch_count;
  // compute mode: also (or instead of out) the Encode(prot_bytes) form,
  // prot_bytes little-endian bytes per KV (db/kv_checksum.h:97-121)
  uint8_t* enc = nullptr;
  typedef KvPre Pre;
  __device__ const uint8_t* base() const { return values.base; }
  __device__ uint64_t off(uint32_t i) const { return values.off(i); }
  __device__ uint64_t hlen(uint32_t i) const { return values.len(i); }
  __device__ Pre pre(uint32_t i, uint64_t, uint64_t) const {
    KvPre e;
    e.klen = keys.len(i);
    const uint64_t kp = reinterpret_cast<uint64_t>(keys.ptr(i));
    // an empty key reads nothing of its own: a zero word instead
    const uint64_t z = reinterpret_cast<uint64_t>(&g_zero16[0]);
    const bool wide = e.klen >= 8;
    const uint64_t a0 = wide ? kp : e.klen ? kp & ~7ull : z;
    const uint64_t a1 = wide ? kp + e.klen - 8 : e.klen ? (kp + e.klen - 1) & ~7ull : z;
    e.k0 = *reinterpret_cast<gbl_u64u_t*>(a0);  // any byte alignment (unaligned global loads)
    e.k1 = *reinterpret_cast<gbl_u64u_t*>(a1);
    e.sh = (uint32_t)(kp & 7);
    e.op = ops ? *reinterpret_cast<gbl_u8_t*>(reinterpret_cast<uint64_t>(ops + i)) : 0u;
    e.extra = kind >= 2 ? *reinterpret_cast<gbl_u64_t*>(reinterpret_cast<uint64_t>(extras + i)) : 0;
    e.stored = 0;
    if (VERIFY) {
      const uint64_t st = reinterpret_cast<uint64_t>(stored) + (uint64_t)i * prot_bytes;
      for (uint32_t b = 0; b < prot_bytes; b++) e.stored |= (uint64_t)*reinterpret_cast<gbl_u8_t*>(st + b) << (8 * b);
    }
    return e;
  }
  __device__ void finish(uint32_t i, uint64_t hv, const Pre& e) const {
    const uint64_t k0 = e.klen >= 8 || e.sh == 0 ? e.k0 : (e.k0 >> (8 * e.sh)) | (e.k1 << (64 - 8 * e.sh));
    uint64_t v = hv ^ (e.klen <= 16 ? xxph3_le16(k0, e.k1, e.klen, kSeedK)
                                    : xxph3_any(keys.ptr(i), e.klen, kSeedK));
    if (kind >= 1) v ^= xxph3_u8(e.op, kSeedO);
    if (kind == 2) v ^= xxph3_u64(e.extra, kSeedS);
    if (kind == 3) v ^= xxph3_u32((uint32_t)e.extra, kSeedC);
    if (!VERIFY) {
      if (out) out[i] = v;
      if (enc)
        for (uint32_t b = 0; b < prot_bytes; b++) enc[(uint64_t)i * prot_bytes + b] = (uint8_t)(v >> (8 * b));
      return;
    }
    const uint64_t sv = e.stored;
    const uint64_t keep = prot_bytes >= 8 ? ~0ull : ((1ull << (8 * prot_bytes)) - 1);
    const bool bad = sv != (v & keep);
    mismatch[i] = bad;
    if (out) out[i] = v;
    if (bad && mismatch_count) atomicAdd(mismatch_count, 1u);
  }
  __device__ void finish(uint32_t i, uint64_t hv) const { finish(i, hv, pre(i, 0, 0)); }
};

// ===================== legacy XXH32 / XXH64 ===============================
template <class Op>
__global__ __launch_bounds__(256) void k_legacy(Op op, uint32_t count) {
  const uint32_t nt = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < count; i += nt) op.run(i);
}

template <bool IS64>
struct OpLegacyValue {
  SpanSrc s;
  uint64_t seed;
  void* out;
  __device__ void run(uint32_t i) const {
    const VBytes b{s.ptr(i), s.len(i), false, 0};
    if (IS64)
      static_cast<uint64_t*>(out)[i] = xxh64_lane(b, seed);
    else
      static_cast<uint32_t*>(out)[i] = xxh32_lane(b, (uint32_t)seed);
  }
};

template <bool IS64, int MODE>
struct OpLegacyBlock {
  BlockArgs a;
  __device__ void run(uint32_t i) const {
    const uint8_t* p = a.s.ptr(i);
    const uint64_t n = a.s.len(i);
    VBytes b{p, n, false, 0};
    if (MODE == kModeVerify) b.n = n + 1;
    if (MODE == kModeTrailer || (MODE == kModeBuiltin && a.last)) {
      b.has_extra = true;
      b.extra = a.last[i];
    }
    const uint32_t v = IS64 ? (uint32_t)xxh64_lane(b, 0) : xxh32_lane(b, 0);
    block_epilogue<MODE>(a, i, v);
  }
};

// kNoChecksum: builtin value 0 (table/format.cc:599-601)
template <int MODE>
struct OpNoneBlock {
  BlockArgs a;
  __device__ void run(uint32_t i) const { block_epilogue<MODE>(a, i, 0u); }
};

// ===================== device WAL writer ==================================
// A planned physical record (mck_wal_plan): the fragment's payload in the
// source, its header's offset in the output, the trailer padding before it.
struct WalFrag {  // = mck_wal_fragment
  uint64_t src_off, dst_off;
  uint32_t length;
  uint8_t type, pad;
  uint16_t reserved;
};

// ===================== one-pass WAL writer ==================================
// mck_wal_write_batch in ONE kernel: the row driver (crc_rows_loop's
// structure, 16-lane rows) CRCs each fragment and, in the same iteration,
// writes what log::Writer appends for it (db/log_writer.cc:263-311):
//   * the payload's 16-byte-aligned OUTPUT pieces of the round's source
//     window [S, S + 64 W): piece q starts at source x = S + e + 16 q
//     (e = -delta mod 16, delta = output - source); lane c takes q = c + W j,
//     so every load / store instruction covers 16 W contiguous bytes (with
//     q = 4 c + j, 64-byte strided 16-byte stores, walwrite took 3.75 ms
//     instead of 0.92 without the pieces); it loads them dword-aligned (16 B +
//     the next dword, re-read from L1/L2: the CRC loads of the same bytes
//     came in one iteration earlier), realigns with v_alignbyte and stores
//     them;
//   * at the span's last round: the < 16 payload bytes before the first and
//     after the last full output piece, byte by byte, and the trailer padding
//     + header ([masked CRC][len][type][log number]) -- the CRC is known then.
// Stores with nothing to write are exec-masked (round 2 measured sinks for
// them: slower).  The
// payload is read from HBM once.
// LDS: the row image; fragments' dst_off at kLdsWalAux, over the un-shift
// tables k >= 16, which this kernel never reads (typed init: no per-span
// un-shift; the tail un-shift is < 16).
constexpr uint32_t kLdsWalAux = kLdsUnshift + 16 * 512;
static_assert(kLdsWalAux + 8 * kRowDescCache <= kCrcLdsBytes, "WAL aux table must fit");

struct OpWalWrite {
  const uint8_t* src;
  const WalFrag* frags;
  WalTypeCrcs tc;
  uint32_t log_number;
  uint32_t* crcs;  // masked fragment CRCs (the API's crc_scratch)
  uint8_t* out;
  __device__ const uint8_t* base() const { return src; }
  __device__ uint64_t off(uint32_t i) const { return frags[i].src_off; }
  __device__ uint64_t len(uint32_t i) const { return frags[i].length; }
  static constexpr bool kTypedInit = true;
  __device__ int init_kind() const { return kInitTyped; }
  // key = type | pad << 8 (init_kind kInitTyped uses key & 15)
  __device__ uint32_t init_key(uint32_t i) const {
    return (uint32_t)ldg_u8(&frags[i].type, 0) | ((uint32_t)ldg_u8(&frags[i].pad, 0) << 8);
  }
  __device__ uint32_t typed_init(uint32_t t) const { return tc.v[t & 15]; }
};

__device__ __forceinline__ uint32_t wal_hdr_byte(uint32_t h, uint32_t crc, uint32_t len, uint32_t type,
                                                 uint32_t log_number) {
  // h < header size: [crc LE32][len LE16][type][log number LE32]
  return h < 4 ? (crc >> (8 * h)) & 0xFF : h < 6 ? (len >> (8 * (h - 4))) & 0xFF : h == 6 ? type
                                                                                    : (log_number >> (8 * (h - 7))) & 0xFF;
}

typedef __attribute__((address_space(1))) uint8_t gbl_st_u8_t;
typedef __attribute__((address_space(1))) uint32_t gbl_st_u32_t;
typedef __attribute__((address_space(1))) span_u32x4 gbl_st_u32x4_t;
__device__ __forceinline__ void st_u8(uint64_t a, uint32_t v) { *reinterpret_cast<gbl_st_u8_t*>(a) = (uint8_t)v; }
__device__ __forceinline__ void st_u32(uint64_t a, uint32_t v) { *reinterpret_cast<gbl_st_u32_t*>(a) = v; }
// 16 bytes at an aligned output address (plain stores: non-temporal ones
// measured slower for the WAL writer, 1.527 vs 1.480 ms per step)
__device__ __forceinline__ void st16(uint64_t a, uint4 o) {
  *reinterpret_cast<gbl_st_u32x4_t*>(a) = span_u32x4{o.x, o.y, o.z, o.w};
}

// ---- one-pass WAL writer: interleaved pieces -------------------------------
// Lane c of a 16-lane row loads pieces c + 16 j (j = 0..4) of the fragment's
// 1280-byte round: every load instruction reads 256 contiguous bytes per
// row, and -- the point -- the row already holds the round in the layout the
// output wants (store j of lane c is output piece c + 16 j), so the copy
// needs no second read of the payload: output piece k is bytes e.. of source
// pieces k and k + 1 (lane c + 1's piece j, via DPP; lane 15 takes lane 0's
// piece j + 1), realigned by the fragment's (dst - src) mod 16.  The piece
// straddling two rounds (lane 15, j = 4) is stored by lane 0 in the next
// round from a one-register carry.  The CRC algebra: a lane's pieces are
// 240 bytes apart, so its state moves piece to piece by zshift(., 244) (the
// pending 4-byte step + the gap; a 4 KiB byte table), and the lane-final
// shift is zshift(., 4 + 16 (15 - c)) (CrcTables::lane_final16).
constexpr uint32_t kLdsWalGap244 = kLdsWalAux + 8 * kRowDescCache + 64;  // [4][256] u32
constexpr uint32_t kLdsWalCarry = kLdsWalGap244 + 4096;  // 16 B per row
static_assert(kLdsWalGap244 % 16 == 0 && kLdsWalCarry + 16 * 64 <= kCrcLdsBytes, "gap table must fit");

__device__ __forceinline__ uint32_t il_gap(uint32_t x, uint32_t w) {
  uint32_t l[4];
#pragma unroll
  for (int b = 0; b < 4; b++) l[b] = lds_u32(kLdsWalGap244 + 1024u * b + (((x >> (8 * b)) & 255u) << 2));
  return xor3(xor3(l[0], l[1], l[2]), l[3], w);
}

// Round r of a span: lane c's pieces c + 16 j; pieces before the span read
// the zero piece (only in its first round).
__device__ __forceinline__ ChunkN<5> il_load(const RowSpan& sp, int r, uint32_t c, uint64_t zp) {
  const uint64_t b = sp.a1 - 1280ull * (uint32_t)(r + 1) + 16ull * c;
  ChunkN<5> ch;
#pragma unroll
  for (int j = 0; j < 5; j++) {
    const uint64_t a = b + 256ull * j;
    ch.v[j] = span_load16<false>(a < sp.a0 ? zp : a);
  }
  return ch;
}

// Round r's foreign bytes zeroed in place: the piece holding ptr (piece k0 =
// (ptr - first round start) / 16 of the first round) keeps the bytes from
// ptr on, lane 15's last piece in the last round those before the end.  The
// copy only stores whole payload pieces, so it can share the masked chunk.
__device__ __forceinline__ uint32_t il_owner_piece(const RowSpan& sp, int r, uint32_t c) {
  const uint32_t k0 = 5u * (uint32_t)sp.owner + (sp.hb >> 4);
  const bool own = r == sp.rounds - 1 && sp.owner < 16 && c == (k0 & 15u);
  return own ? k0 >> 4 : 5u;
}
__device__ __forceinline__ void il_mask(ChunkN<5>& ch, const RowSpan& sp, int r, uint32_t c) {
  const uint32_t pa = il_owner_piece(sp, r, c);
  const uint4 mh = lds_u32x4(kLdsRowMaskHead + 16 * ((uint32_t)sp.ptr & 15u));
  const uint4 mt = lds_u32x4(kLdsRowMaskTail + 16 * ((r == 0 && c == 15) ? sp.kt : 0u));
#pragma unroll
  for (int j = 0; j < 5; j++) {
    const uint32_t sel = (uint32_t)j == pa ? ~0u : 0u;
    ch.v[j].x = __builtin_amdgcn_bitop3_b32(ch.v[j].x, mh.x, sel, 0xD0);
    ch.v[j].y = __builtin_amdgcn_bitop3_b32(ch.v[j].y, mh.y, sel, 0xD0);
    ch.v[j].z = __builtin_amdgcn_bitop3_b32(ch.v[j].z, mh.z, sel, 0xD0);
    ch.v[j].w = __builtin_amdgcn_bitop3_b32(ch.v[j].w, mh.w, sel, 0xD0);
  }
  and4(ch.v[4], mt);
}

// The lane's state after its five (masked) pieces, the last 4-byte step
// pending; x = the state at its first piece (0 in a span's first round).
__device__ __forceinline__ uint32_t il_round(uint32_t x, const ChunkN<5>& ch, const RowSpan& sp, int r, uint32_t c,
                                             const CrcLane& L) {
  const uint32_t pa = il_owner_piece(sp, r, c);
  const uint32_t inj = sp.inj;
  x ^= ch.v[0].x ^ (pa == 0 ? inj : 0u);
#pragma unroll
  for (int j = 0; j < 5; j++) {
    x = crc_step4x(x, L, ch.v[j].y);
    x = crc_step4x(x, L, ch.v[j].z);
    x = crc_step4x(x, L, ch.v[j].w);
    if (j < 4) x = il_gap(x, ch.v[j + 1].x ^ (pa == (uint32_t)(j + 1) ? inj : 0u));
  }
  return x;
}

// 16 bytes at byte e (q2 = e & 8, q1 = e & 4, be = e & 3) of lo || hi.
__device__ __forceinline__ uint4 il_align(const uint4& lo, const uint4& hi, uint32_t q2, uint32_t q1, uint32_t be) {
  const uint32_t X[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  uint32_t Y[6], Z[5];
#pragma unroll
  for (int m = 0; m < 6; m++) Y[m] = q2 ? X[m + 2] : X[m];
#pragma unroll
  for (int t = 0; t < 5; t++) Z[t] = q1 ? Y[t + 1] : Y[t];
  uint4 o;
  o.x = __builtin_amdgcn_alignbyte(Z[1], Z[0], be);
  o.y = __builtin_amdgcn_alignbyte(Z[2], Z[1], be);
  o.z = __builtin_amdgcn_alignbyte(Z[3], Z[2], be);
  o.w = __builtin_amdgcn_alignbyte(Z[4], Z[3], be);
  return o;
}

template <int CTRL>
__device__ __forceinline__ uint4 dpp_u32x4(const uint4& v) {
  uint4 r;
  r.x = (uint32_t)__builtin_amdgcn_mov_dpp((int)v.x, CTRL, 0xF, 0xF, true);
  r.y = (uint32_t)__builtin_amdgcn_mov_dpp((int)v.y, CTRL, 0xF, 0xF, true);
  r.z = (uint32_t)__builtin_amdgcn_mov_dpp((int)v.z, CTRL, 0xF, 0xF, true);
  r.w = (uint32_t)__builtin_amdgcn_mov_dpp((int)v.w, CTRL, 0xF, 0xF, true);
  return r;
}
constexpr int kDppRowRor15 = 0x12F;  // lane j of a row <- lane j + 1 (mod 16)
constexpr int kDppRowRor1x = 0x121;  // lane j of a row <- lane j - 1 (mod 16)

// A row's place in the writer's share: fragment slot i, its geometry sp
// (record type / trailer padding in key, header offset in the output dst),
// round r; the next ticket nt (descriptor nd, header offset ndst).
struct WalIlState {
  RowSpan sp;
  uint4 nd;
  uint64_t dst, ndst;
  uint32_t key, i, nt, live;
  int32_t r;
};
struct WalIlCtx {
  const OpWalWrite& op;
  const RowShare& sh;
  uint64_t base, obase, zp;
  uint32_t share, c, lf4, carry_slot;
  const CrcLane& L;
};
constexpr int kWalW = 16, kWalNP = 5;
constexpr int kWalHdr = 2;  // padding + header bytes per lane (pad + hs <= 21)

// One iteration: the output of (A's fragment, round A.r) from the round's own
// registers (ca, masked in place), its CRC round, and B -- the row's next
// round or its next fragment's first -- set up and loaded into cb.  x = the
// lane's CRC state at its next piece.  Returns whether any row goes on.
__device__ __forceinline__ bool wal_il_step(const WalIlCtx& X, const WalIlState& A, ChunkN<kWalNP>& ca,
                                            WalIlState& B, ChunkN<kWalNP>& cb, uint32_t& x) {
  constexpr int W = kWalW, NP = kWalNP;
  const uint32_t c = X.c;
  const bool live = A.live != 0;
  const RowSpan& sp = A.sp;
  const int r = A.r;
  const bool last = r == 0;
  const bool firstr = r == sp.rounds - 1;
  const bool fin = live && last;

  const uint32_t type = A.key & 0xFF, pad = (A.key >> 8) & 0xFF;
  il_mask(ca, sp, r, c);

  // ---- next unit (as crc_rows_step), its load in flight over the CRC round ----
  const bool go = live && (!last || A.nt < X.share);
  const RowSpan nsp = row_span<W, NP>(X.base + (((uint64_t)A.nd.y << 32) | A.nd.x), A.nd.z, A.nd.w, kInitTyped);
  const bool sw = go && last;
  B.sp = row_span_sel(sw, nsp, sp);
  B.r = go ? (last ? nsp.rounds - 1 : r - 1) : r;
  B.i = sw ? X.sh.idx(A.nt) : A.i;
  cb = il_load(B.sp, B.r, c, X.zp);

  x = il_round(firstr ? 0u : x, ca, sp, r, c, X.L);
  uint32_t crc = 0;
  if (wave_any(fin)) crc = crc_mask(row_finish4<W>(x, sp, X.lf4));
  if (wave_any(live && !last)) x = il_gap(x, 0u);  // to the lane's piece in the next round
  __builtin_amdgcn_sched_barrier(0);

  // ---- the output of this (span, round), from the round's own registers ----
  // Every store of the round -- payload pieces, the edge bytes, the header
  // once the CRC is known -- issues here, back to back: a 128-B line the
  // round writes in parts is then complete before L2 writes it back (stores
  // split around the CRC round measured 1.09-1.15x the stream's bytes).
  const uint32_t hs = ((type >= 5 && type <= 8) || type == 11) ? 11u : 7u;
  const uint64_t P = X.obase + A.dst + hs;  // payload in the output
  // the < 16 payload bytes before the first and after the last full output
  // piece (lane c: head byte c, tail byte c), loaded first (L2 hits: the
  // round just read them), stored after the pieces
  uint32_t bh = 0, bt = 0, ebt = 0;  // head byte c, tail byte c, the tail byte's offset
  bool okh = false, okt = false;
  if (wave_any(fin)) {
    const uint32_t Pl = (uint32_t)P;  // payload start mod 2^32
    const uint32_t hb = (16u - (Pl & 15u)) & 15u;  // bytes before the first aligned piece
    const uint32_t hb_end = hb < sp.n ? hb : sp.n;
    const uint32_t tb = (Pl + sp.n) & 15u;
    // (sp.n < tb: a payload inside one 16-byte granule -- its head bytes
    // cover it, no tail bytes; no unsigned wraparound)
    const uint32_t tb_beg = (sp.n >= tb && sp.n - tb > hb_end) ? sp.n - tb : hb_end;
    okh = fin && c < hb_end;
    ebt = tb_beg + c;
    okt = fin && ebt < sp.n;
    bh = *reinterpret_cast<gbl_u8_t*>(okh ? sp.ptr + c : X.zp);
    bt = *reinterpret_cast<gbl_u8_t*>(okt ? sp.ptr + ebt : X.zp);
  }

  const uint64_t ps = sp.ptr;               // payload in the source
  const uint64_t delta = P - ps;            // (mod 2^64)
  const uint32_t e = (uint32_t)(0ull - delta) & 15u;
  const uint32_t q2 = e & 8u, q1 = e & 4u, be = e & 3u;
  // output piece c + 16 j takes source bytes [x0 + 256 j, + 16), x0 = the
  // round's window start + e + 16 c; whole pieces of the payload only
  // (rel = offset in the payload, 32-bit: fragments are < 4 GiB)
  const uint32_t win = (uint32_t)(sp.a1 - ps) - 1280u * (uint32_t)(r + 1);  // window start - ps
  const int32_t rel0 = (int32_t)(win + e + 16u * c);
  const int32_t lim = (int32_t)sp.n - 16;
  const uint64_t oa0 = P + (uint64_t)(int64_t)rel0;  // output address of piece c
  {  // the piece that straddles the previous round and this one: lane 15's
     // piece 4 of that round waits in the row's LDS slot
    const int32_t relm = (int32_t)(win + e) - 16;
    const bool okm = live && !firstr && e != 0 && c == 0 && relm >= 0 && relm <= lim;
    if (wave_any(okm)) {
      const uint4 cm = lds_u32x4(X.carry_slot);
      const uint4 o = il_align(cm, ca.v[0], q2, q1, be);
      if (okm) st16(P + (uint64_t)(int64_t)relm, o);
    }
  }
  uint4 rj = dpp_u32x4<kDppRowRor15>(ca.v[0]);  // lane c + 1's piece j
#pragma unroll
  for (int j = 0; j < NP; j++) {
    const uint4 rn = j + 1 < NP ? dpp_u32x4<kDppRowRor15>(ca.v[j + 1]) : rj;
    const int32_t rel = rel0 + 256 * j;
    const bool ok = live && rel >= 0 && rel <= lim && !(j == NP - 1 && c == 15 && e != 0);
    const uint4 nb = (j < NP - 1 && c == 15) ? rn : rj;
    const uint4 o = il_align(ca.v[j], nb, q2, q1, be);
    if (ok) st16(oa0 + 256ull * j, o);
    rj = rn;
    // one piece at a time (the scheduler would otherwise hoist every
    // piece's DPP moves and selects and spill)
    __builtin_amdgcn_sched_barrier(0);
  }
  if (c == 15) {
    const span_u32x4 cv = {ca.v[NP - 1].x, ca.v[NP - 1].y, ca.v[NP - 1].z, ca.v[NP - 1].w};
    *reinterpret_cast<__attribute__((address_space(3))) span_u32x4*>(static_cast<size_t>(X.carry_slot)) = cv;
  }
  {  // the < 16 payload bytes before the first and after the last full output piece
    const uint64_t oh = P + c, ot = P + ebt;
    if (okh) st_u8(oh, bh);
    if (okt) st_u8(ot, bt);
  }
  if (fin && c == 0) st_u32(reinterpret_cast<uint64_t>(X.op.crcs + A.i), crc);
  // trailer padding + header: bytes c + 16 m of [dst - pad, dst + hs)
  const uint64_t hstart = X.obase + A.dst - pad;
#pragma unroll
  for (int m = 0; m < kWalHdr; m++) {
    const uint32_t b = c + (uint32_t)W * m;
    const bool okb = fin && b < pad + hs;
    const uint32_t val = b < pad ? 0u : wal_hdr_byte(b - pad, crc, sp.n, type, X.op.log_number);
    if (okb) st_u8(hstart + b, val);
  }

  // ---- advance ----
  B.nt = A.nt;
  B.nd = A.nd;
  B.ndst = A.ndst;
  if (wave_any(sw)) {
    const uint32_t tk = row_ticket<W>(sw);
    if (sw) {
      B.nt = tk;
      B.nd = row_desc(tk, X.share);
      B.ndst = *lds_p64(kLdsWalAux + 8 * (tk < X.share ? tk : 0));
    }
  }
  B.key = sw ? A.nd.w : A.key;
  B.dst = sw ? A.ndst : A.dst;
  B.live = go ? 1u : 0u;
  return wave_any(go);
}

// fragments' dst_off, staged like the descriptors (row_desc_stage order)
__device__ __forceinline__ void wal_stage_dst(const OpWalWrite& op, const RowShare& sh) {
  for (uint32_t t = threadIdx.x; t < sh.n; t += blockDim.x) *lds_p64(kLdsWalAux + 8 * t) = op.frags[sh.idx(t)].dst_off;
}

// The row loop over one window of <= kRowDescCache fragments (staged).
__device__ __forceinline__ void wal_write_window(const OpWalWrite& op, const RowShare& sh, const CrcLane& L,
                                                 const CrcTables* __restrict__ g) {
  constexpr int W = kWalW, NP = kWalNP;
  const uint32_t c = threadIdx.x & (W - 1);
  const uint32_t share = sh.n;
  // the row's LDS slot for the previous round's straddling piece
  const WalIlCtx X{op, sh, reinterpret_cast<uint64_t>(op.src), reinterpret_cast<uint64_t>(op.out),
                   reinterpret_cast<uint64_t>(&g->zero16[0]), share, c, c << 2, kLdsWalCarry + 16u * (threadIdx.x >> 4), L};
  WalIlState A;
  const uint32_t t = row_ticket<W>(true);
  A.live = t < share ? 1u : 0u;
  const uint4 d = row_desc(t, share);
  A.dst = *lds_p64(kLdsWalAux + 8 * (t < share ? t : 0));
  A.i = sh.idx(A.live ? t : 0);
  A.sp = row_span<W, NP>(X.base + (((uint64_t)d.y << 32) | d.x), d.z, d.w, kInitTyped);
  A.key = d.w;
  A.r = A.sp.rounds - 1;
  ChunkN<NP> ca = il_load(A.sp, A.r, c, X.zp);
  A.nt = row_ticket<W>(true);
  A.nd = row_desc(A.nt, share);
  A.ndst = *lds_p64(kLdsWalAux + 8 * (A.nt < share ? A.nt : 0));
  uint32_t x = 0;  // the lane's CRC state at its next piece
  // unrolled twice: the rounds' chunks and states swap register names
  // instead of 20 v_mov per round
  WalIlState B;
  ChunkN<NP> cb;
  for (;;) {
    if (!wal_il_step(X, A, ca, B, cb, x)) break;
    if (!wal_il_step(X, B, cb, A, ca, x)) break;
  }
}

// A workgroup's contiguous fragment range in windows of <= kRowDescCache
// (its LDS descriptor and dst_off tables): one launch serves any group
// commit (round 4; launches of <= ncu * kRowDescCache fragments each paid
// the launch's ramp and drain, 6 per 2M-record step).
__device__ __forceinline__ void wal_write_il(const OpWalWrite& op, uint32_t first, uint32_t count, uint8_t* lds,
                                             const CrcTables* __restrict__ g) {
  constexpr bool BLK = true;  // contiguous fragment ranges per workgroup
  const RowShare share = row_share<BLK>(first, count);
  const uint32_t nwin = (share.n + kRowDescCache - 1) / kRowDescCache;
  if (nwin == 0) return;  // workgroup-uniform
  auto win = [&](uint32_t wi) {
    const uint32_t w0 = (uint32_t)((uint64_t)share.n * wi / nwin), w1 = (uint32_t)((uint64_t)share.n * (wi + 1) / nwin);
    return RowShare{share.start + share.stride * w0, share.stride, w1 - w0};
  };
  const RowShare sh0 = win(0);
  crc_rows_prologue<OpWalWrite>(op, sh0, lds, g, false);
  wal_stage_dst(op, sh0);
  {  // lane-final map over lane-final columns 0-15, the piece-to-piece byte table
    const uint32_t t = threadIdx.x;
    if (t < 512) {
      const uint4 x = reinterpret_cast<const uint4*>(&g->lane_final16[0][0][0])[t];
      *reinterpret_cast<uint4*>(lds + kLdsFinal + 256 * (t >> 2) + 16 * (t & 3)) = x;
    } else if (t < 768) {
      const uint4 x = reinterpret_cast<const uint4*>(&g->gap244[0][0])[t - 512];
      *reinterpret_cast<uint4*>(lds + kLdsWalGap244 + 16 * (t - 512)) = x;
    }
  }
  __syncthreads();
  const CrcLane L = crc_lane();
  for (uint32_t wi = 0; wi < nwin; wi++) {
    const RowShare sh = win(wi);
    if (wi) {
      __syncthreads();  // every row is done with the previous window's slots
      row_desc_stage<OpWalWrite>(op, sh, false);
      wal_stage_dst(op, sh);
      __syncthreads();
    }
    wal_write_window(op, sh, L, g);
  }
}

__global__ __launch_bounds__(1024) void k_wal_write_il(OpWalWrite op, uint32_t first, uint32_t count) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  wal_write_il(op, first, count, lds, &g_crc_tables);
}

// ---- WAL recovery: reassemble logical records (mck_wal_gather_batch) -----
// Copy each fragment's payload to out + dst_off: one wave per fragment, the
// body as aligned 16-byte stores assembled from dword-aligned source loads
// (v_alignbyte), the < 16-byte head and tail byte-wise.  Every load of a
// fragment's first KiB is issued before any of its stores and the next
// fragment's descriptor before them -- one memory round trip per typical
// (1 KB) fragment (1.038 vs 1.143 ms per 2.16M fragments, round 1).
struct WalCopyPass {
  uint64_t pay, body0, body1, end, head_end;
  uint64_t ha, ca, ta;  // this lane's head byte, body chunk, tail byte (output offsets)
  bool hv, cv, tv;
  uint8_t hb, tb;
  uint4 v;
};

// 16 output bytes at payload-relative source offset s: one 16-byte load at
// the dword below s (dword-aligned: a byte-misaligned 16-byte load runs far
// below rate) plus the next dword when s is not dword-aligned.
__device__ __forceinline__ uint4 wal_chunk_load(const uint8_t* src, uint64_t s) {
  const uint64_t s4 = s & ~3ull;
  const uint32_t sh = (uint32_t)(s & 3);
  const uint4 a = span_load16<false>(reinterpret_cast<uint64_t>(src + s4));
  // with sh == 0 the fifth dword is not needed (and could lie past the
  // payload's last dword): re-read the fourth
  const uint32_t e = reinterpret_cast<const uint32_t*>(src + s4)[sh ? 4 : 3];
  uint4 v;
  v.x = __builtin_amdgcn_alignbyte(a.y, a.x, sh);
  v.y = __builtin_amdgcn_alignbyte(a.z, a.y, sh);
  v.z = __builtin_amdgcn_alignbyte(a.w, a.z, sh);
  v.w = __builtin_amdgcn_alignbyte(e, a.w, sh);
  return v;
}

__device__ __forceinline__ void wal_gather_issue(WalCopyPass& p, const WalFrag& f, const uint8_t* __restrict__ src,
                                                 uint32_t lane) {
  p.end = f.dst_off + f.length;
  p.pay = f.dst_off;                     // output offset of payload byte 0
  p.body0 = (p.pay + 15) & ~15ull;       // first 16-aligned chunk of payload
  p.body1 = p.end & ~15ull;              // end of the last full chunk
  const bool body = p.body0 < p.body1;
  // head: [pay, body0) byte-wise -- or the whole fragment when it has no
  // full 16-byte chunk; tail: [body1, end) byte-wise (< 16 bytes)
  p.head_end = body ? p.body0 : p.end;
  p.ha = p.pay + lane;
  p.hv = p.ha < p.head_end;
  p.ca = p.body0 + 16ull * lane;
  p.cv = body && p.ca < p.body1;
  p.ta = p.body1 + lane;
  p.tv = body && p.ta < p.end;
  p.hb = p.tb = 0;
  if (p.hv) p.hb = src[f.src_off + (p.ha - p.pay)];
  if (p.tv) p.tb = src[f.src_off + (p.ta - p.pay)];
  if (p.cv) p.v = wal_chunk_load(src, f.src_off + (p.ca - p.pay));
}

__global__ __launch_bounds__(256) void k_wal_gather(const uint8_t* __restrict__ src, const WalFrag* __restrict__ frags,
                                                    uint32_t nfrags, uint8_t* __restrict__ out) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wpb = blockDim.x >> 6;
  const uint32_t nw = gridDim.x * wpb;
  uint32_t fi = __builtin_amdgcn_readfirstlane(blockIdx.x * wpb + (threadIdx.x >> 6));
  if (fi >= nfrags) return;
  WalFrag f = frags[fi];
  for (;;) {
    WalCopyPass p;
    wal_gather_issue(p, f, src, lane);
    const uint32_t fn = fi + nw;
    const bool more = fn < nfrags;
    const WalFrag f2 = frags[more ? fn : fi];
    if (p.hv) out[p.ha] = p.hb;
    if (p.cv) *reinterpret_cast<uint4*>(out + p.ca) = p.v;
    if (p.tv) out[p.ta] = p.tb;
    // the rest of a long fragment (beyond the first 64 x 16 bytes)
    for (uint64_t c = p.ca + 16ull * 64; c < p.body1; c += 16ull * 64)
      *reinterpret_cast<uint4*>(out + c) = wal_chunk_load(src, f.src_off + (c - p.pay));
    if (!more) break;
    fi = fn;
    f = f2;
  }
}

// ===================== blob log records ===================================
// db/blob/blob_log_format.cc:97-135 BlobLogRecord: a 32-byte header
// [key_size u64][value_size u64][expiration u64][header_crc u32][blob_crc
// u32], then key and value.  header_crc = Mask(Value(header[0..24))),
// blob_crc = Mask(Extend(Value(key), value)) = Mask(Value(key || value)).
// The CRC span is key || value; the header travels as the epilogue input.
struct BlobPre {
  uint4 h0, h1;  // header bytes [0, 16), [16, 32)
};
// crc32c::Value of the 24 header bytes on every lane (6 table steps).
__device__ __forceinline__ uint32_t blob_header_crc(const BlobPre& e) {
  const CrcLane L = crc_lane();
  const uint32_t w[6] = {e.h0.x, e.h0.y, e.h0.z, e.h0.w, e.h1.x, e.h1.y};
  uint32_t s = 0xFFFFFFFFu ^ w[0];
#pragma unroll
  for (int k = 0; k < 6; k++) s = crc_step4x(s, L, k < 5 ? w[k + 1] : 0u);
  return ~s;
}
template <bool WRITE>
struct OpBlobRecord {
  static constexpr bool kByteShares = true;  // records in file order
  const uint8_t* file;
  const uint64_t* rec_off;   // record header offsets in the file
  const uint32_t* blob_len;  // key_size + value_size
  uint8_t* status;           // verify: bit 0 header CRC bad, bit 1 blob CRC bad
  uint32_t* mismatch_count;  // verify (opt): records with any bad CRC
  typedef BlobPre Pre;
  __device__ const uint8_t* base() const { return file; }
  __device__ uint64_t off(uint32_t i) const { return rec_off[i] + 32; }
  __device__ uint64_t len(uint32_t i) const { return blob_len[i]; }
  __device__ uint32_t init_crc(uint32_t) const { return 0u; }
  static constexpr bool kTypedInit = false;
  __device__ int init_kind() const { return kInitZero; }
  __device__ uint32_t init_key(uint32_t) const { return 0u; }
  __device__ uint32_t typed_init(uint32_t) const { return 0u; }
  __device__ Pre pre(uint32_t, uint64_t ptr, uint64_t) const {
    // (record headers sit at any byte offset: vload16_any, never s_load)
    return Pre{vload16_any(ptr - 32), vload16_any(ptr - 16)};
  }
  __device__ void finish(uint32_t i, uint32_t crc, const Pre& e, bool writer) const {
    const uint32_t hcrc = crc_mask(blob_header_crc(e));
    const uint32_t bcrc = crc_mask(crc);
    if (!writer) return;
    if (WRITE) {  // BlobLogRecord::EncodeHeaderTo: the two CRC fields, LE
      uint8_t* h = const_cast<uint8_t*>(file) + rec_off[i] + 24;
#pragma unroll
      for (int b = 0; b < 4; b++) {
        h[b] = (uint8_t)(hcrc >> (8 * b));
        h[4 + b] = (uint8_t)(bcrc >> (8 * b));
      }
    } else {  // DecodeHeaderFrom + CheckBlobCRC
      const uint8_t st = (uint8_t)((hcrc != e.h1.z ? 1u : 0u) | (bcrc != e.h1.w ? 2u : 0u));
      status[i] = st;
      if (st && mismatch_count) atomicAdd(mismatch_count, 1u);
    }
  }
};

// ===================== long spans: pieces + combine =======================
// util/crc32c.cc:1221-1289 Crc32cCombine, applied to every piece of a long
// span at once.  Pieces i were hashed by the batch kernels (v[i] = Value of
// piece i); with pure(.) the init-0, no-inversion CRC,
//   Extend(init, span) = ~( zshift(~init, n) ^ XOR_i zshift(pure_i, after_i) )
//   pure_i = ~v[i] ^ zshift(~0, len_i)      (Value's init state, removed)
// after_i = bytes of the span behind piece i.  The caller seeds *out with
// ~zshift(~init, n); every wave XORs in its pieces' terms atomically (XOR
// commutes: the result does not depend on the order).
__device__ __forceinline__ uint32_t gf_mul_dev(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#pragma unroll 8
  for (int j = 0; j < 32; j++) {
    p ^= (b & (0x80000000u >> j)) ? a : 0u;
    a = (a >> 1) ^ ((a & 1u) ? kCrc32cPoly : 0u);
  }
  return p;
}

struct CrcPowers {
  uint32_t x8[64];  // x^(8 * 2^k) mod P, k < 64 (util/crc32c.cc crc32c_powers)
};

__device__ __forceinline__ uint32_t gf_zshift_dev(uint32_t s, uint64_t nbytes, const CrcPowers& pw) {
  for (int k = 0; nbytes; k++, nbytes >>= 1)
    if (nbytes & 1) s = gf_mul_dev(s, pw.x8[k]);
  return s;
}

__global__ __launch_bounds__(256) void k_crc_combine(const uint32_t* __restrict__ v, uint32_t npieces,
                                                     uint64_t piece, uint64_t n, uint32_t c_full,
                                                     uint32_t c_tail, CrcPowers pw, uint32_t* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t term = 0;
  if (i < npieces) {
    const uint64_t start = (uint64_t)i * piece;
    const uint64_t len = n - start < piece ? n - start : piece;
    const uint32_t pure = ~v[i] ^ (len == piece ? c_full : c_tail);
    term = gf_zshift_dev(pure, n - start - len, pw);
  }
  term = wave_xor32(term);
  if ((threadIdx.x & 63) == 0 && term) atomicXor(out, term);
}

// Read (and with reset, clear) the per-device mismatch ticker in ONE atomic
// step: a verify kernel running concurrently loses no count between the read
// and the clear (mck_statistics_get).
__global__ void k_stats_take(unsigned long long* ctr, unsigned long long* out, int reset) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *out = reset ? atomicExch(ctr, 0ull) : atomicAdd(ctr, 0ull);
}

// ============================ WAL verify ==================================
// db/log_reader.cc:450-584 ReadPhysicalRecord with checksum_ = true, applied
// to every 32 KiB block independently; one wave per block.
struct WalResult {
  uint32_t records_ok;
  int32_t status;
  uint32_t stop_offset;
  uint32_t bytes_ok;
};


// The block's first header comes from a 16-byte vector load issued while
// the previous block is hashed (one memory round trip per 32 KiB block
// saved: configs[3] blocks hold one record each, whose ~8 CRC rounds the
// header read used to precede); later records of a block read theirs on
// demand.  A 16-byte load at a block start stays in the 16-byte granule
// holding the block's first byte, so it never leaves the image's pages.
__device__ __forceinline__ uint4 wal_hdr16(const uint8_t* wal, uint32_t b) {
  return vload16_any(reinterpret_cast<uint64_t>(wal) + (uint64_t)b * 32768);
}

// ReadPhysicalRecord's header checks (db/log_reader.cc:450-560) for the
// record at a block offset with `left` bytes to the block's end: go = 1 when
// the record is to be hashed, else status says why the block stops there (0:
// a < 7-byte trailer, skipped).  w0/w1 are the header's first 7 bytes (CRC,
// length, type); lognum() reads the recyclable header's log number.
struct WalRec {
  uint32_t go;
  int32_t status;
  uint32_t hsize;
  uint32_t length;
};
template <class LogNum>
__device__ __forceinline__ WalRec wal_parse(uint32_t left, bool last_block, uint32_t log_number, uint32_t w1,
                                            LogNum lognum) {
  WalRec r{0u, 0, 7u, 0u};
  if (left < 7) {
    // fewer than kHeaderSize bytes: block trailer (skip), or at EOF a
    // truncated header (db/log_reader.cc:432-440)
    if (last_block && left > 0) r.status = 5;  // MCK_WAL_BAD_HEADER
    return r;
  }
  r.length = w1 & 0xFFFFu;
  const uint32_t type = (w1 >> 16) & 0xFFu;
  if ((type >= 5 && type <= 8) || type == 11) {
    r.hsize = 11;
    if (left < 11) {
      if (last_block) r.status = 5;
      return r;
    }
    if (lognum() != log_number) {
      r.status = 4;  // kOldRecord
      return r;
    }
  }
  if (r.hsize + r.length > left) {
    r.status = 2;  // kBadRecordLen
    return r;
  }
  if (type == 0 && r.length == 0) {
    r.status = 3;  // kZeroType, length 0: buffer cleared
    return r;
  }
  r.go = 1;
  return r;
}

// One wave per block; a wave's records form one software pipeline: each
// record is hashed round by round with the next round's chunk in flight,
// and when a record ends its block (configs[3]: one record per block) its
// last round already loads the first round of the wave's NEXT block, whose
// header was read at the record's start, so the wave never waits a memory
// trip between blocks.  A record followed by another in the same block
// hands over without that overlap (its header is read on demand, byte by
// byte, as ReadPhysicalRecord reads the buffer), and so does one whose
// checksum fails or whose successor header does not parse.
template <bool T>
__global__ __launch_bounds__(1024) void k_wal_verify(const uint8_t* wal, uint64_t nbytes, uint32_t log_number,
                                                     WalResult* res, uint32_t nblocks) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  crc_fill_lds(lds, &g_crc_tables);
  __syncthreads();
  const CrcLane L = crc_lane();
  const uint32_t wpb = blockDim.x >> 6;
  const uint32_t nw = gridDim.x * wpb;
  uint32_t cb = __builtin_amdgcn_readfirstlane(blockIdx.x * wpb + (threadIdx.x >> 6));
  if (cb >= nblocks) return;
  auto block_size = [&](uint32_t k) {
    const uint64_t rem = nbytes - (uint64_t)k * 32768;
    return rem < 32768 ? (uint32_t)rem : 32768u;
  };
  auto last_block = [&](uint32_t k) { return nbytes - (uint64_t)k * 32768 <= 32768; };  // EOF inside it
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
  auto parse_first = [&](uint32_t k, const uint4& h) {
    const uint32_t w1 = rfl_u32(h.y);
    return wal_parse(block_size(k), last_block(k), log_number, w1,
                     [&] { return (w1 >> 24) | (rfl_u32(h.z) << 8); });
  };
  uint32_t cpos = 0, cok = 0;          // current record: block offset, records verified before it
  uint4 hb = wal_hdr16(wal, cb);       // the current block's first header (cpos == 0)
  bool seek = true;                    // the current record still has to be parsed and loaded
  WalRec rec{};
  uint32_t stored = 0;
  CrcSpan sp = crc_span(wal, 0, 0u);
  Chunk cur{};
  for (;;) {
    if (seek) {
      for (;;) {  // finish blocks until a record to hash
        const uint32_t left = block_size(cb) - cpos;
        const uint8_t* h = wal + (uint64_t)cb * 32768 + cpos;
        if (cpos == 0) {
          rec = parse_first(cb, hb);
          stored = rfl_u32(hb.x);
        } else {
          uint32_t w1 = 0;
          if (left >= 7) {  // (rfl: the header words are wave-uniform, so is the control flow)
            stored = rfl_u32(rd32_bytes(h));
            w1 = rfl_u32((uint32_t)h[4] | ((uint32_t)h[5] << 8) | ((uint32_t)h[6] << 16));
          }
          rec = wal_parse(left, last_block(cb), log_number, w1, [&] { return rfl_u32(rd32_bytes(h + 7)); });
        }
        if (rec.go) break;
        emit(cb, cok, rec.status, cpos);
        cb += nw;
        if (cb >= nblocks) return;
        cpos = 0;
        cok = 0;
        hb = wal_hdr16(wal, cb);
      }
      sp = crc_span(wal + (uint64_t)cb * 32768 + cpos + 6, rec.length + rec.hsize - 6, 0u);
      cur = crc_load_chunk<T>(sp, sp.rounds - 1, L);
    }
    // does the block end with this record (if it passes)?  Then the next
    // record is the first of the wave's next block: its header now, its
    // first round with this record's last.
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
    uint32_t s = 0;
    for (int r = sp.rounds - 1; r >= 0; r--) {
      Chunk nxt;
      // unconditional loads (see crc_load_chunk); without a next block,
      // round 0 of this record is read again and never used.  The next
      // span's geometry lives only for its load (SGPRs are the limit here)
      if (r > 0 || !spec) {
        nxt = crc_load_chunk<T>(sp, r > 0 ? r - 1 : 0, L);
      } else {
        nrec = parse_first(nb, hn);
        const CrcSpan nsp = next_span();
        nxt = crc_load_chunk<T>(nsp, nsp.rounds - 1, L);
      }
      if (T && !(sp.mini && r == sp.rounds - 1)) row_transpose(cur);  // wave-uniform
      s = crc_round(s, cur, sp, r, L);
      cur = nxt;
    }
    // Unmask(stored) == actual  <=>  stored == Mask(actual).  (Every lane
    // holds the CRC; rfl tells the compiler, so the record stream's state
    // stays in SGPRs and its control flow scalar.)
    const bool pass = crc_mask(rfl_u32(crc_finish(s, sp, L))) == stored;
    if (!pass) {
      emit(cb, cok, 1, cpos);  // kBadRecordChecksum
    } else if (size - e < 7) {
      // the block's trailer (skipped), or at EOF a truncated header
      emit(cb, cok + 1, last_block(cb) && size > e ? 5 : 0, e);
    } else {  // the next record of the same block
      cok++;
      cpos = e;
      seek = true;
      continue;
    }
    if (nb >= nblocks) return;
    cb = nb;
    cpos = 0;
    cok = 0;
    hb = spec ? hn : wal_hdr16(wal, cb);
    seek = !(spec && nrec.go);
    if (!seek) {  // pipelined: the record's first round is in cur
      rec = nrec;
      sp = next_span();
      stored = rfl_u32(hn.x);
    }
  }
}

}  // namespace mck
