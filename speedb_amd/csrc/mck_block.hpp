// mck_block.hpp -- per-KV protection of uncompressed block entries
// (SURVEY.md 8f row 4): table/block_based/block.cc:1091-1222
// Block::Initialize{Data,Index,MetaIndex}BlockProtectionInfo.
//
// A block is prefix-compressed: an entry's key is the previous key's first
// `shared` bytes plus its own `non_shared` bytes, and only restart points
// (every block_restart_interval-th entry, shared == 0) start from nothing.
// The restart array therefore cuts a block into independent intervals, and
// the device walks them in parallel: one wave per block, lane r per restart
// interval r (r += 64 for blocks with more intervals).  Three passes:
//
//   k_block_layout       walk every interval: entry count, reassembled key
//                        bytes, first error; per block the key count and
//                        key bytes (-> exclusive scans, k_blk_scan_*)
//   k_block_materialize  walk again, reassembling each key into a key arena
//                        and writing per-entry key/value spans
//   k_xph3<OpKvProtect>  ProtectKV(key, value).Encode(prot_bytes) per entry
//                        on the XXPH3 row driver (the batched KV kernel)
//
// Entry k of a block lands at key index key_base[block] + k, in the order the
// reference's SeekToFirst/Next loop generates them (:1116-1123).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mck {

enum { kBlkData = 0, kBlkIndex = 1, kBlkIndexDelta = 2, kBlkIndexDeltaFk = 3, kBlkMeta = 4 };
enum { kBlkOk = 0, kBlkBadContents = 1, kBlkBadEntry = 2, kBlkBadRestarts = 3 };

typedef __attribute__((address_space(1))) const uint32_t gbl_u32u_t;

__device__ __forceinline__ uint32_t blk_u8(const uint8_t* p) {
  return *reinterpret_cast<gbl_u8_t*>(reinterpret_cast<uint64_t>(p));
}
// LE32 at any byte address (unaligned global load)
__device__ __forceinline__ uint32_t blk_u32(const uint8_t* p) {
  return *reinterpret_cast<gbl_u32u_t*>(reinterpret_cast<uint64_t>(p));
}

// util/coding.h GetVarint32Ptr (max_shift 28) / GetVarint64Ptr (63): nullptr
// when the varint runs past lim or past its length.
__device__ __forceinline__ const uint8_t* blk_varint(const uint8_t* p, const uint8_t* lim, int max_shift,
                                                     uint64_t* v) {
  uint64_t r = 0;
  for (int shift = 0; shift <= max_shift && p < lim; shift += 7) {
    const uint64_t b = blk_u8(p++);
    r |= (b & 127) << shift;
    if (!(b & 128)) {
      *v = r;
      return p;
    }
  }
  return nullptr;
}

// block.cc:994-1083 NumRestarts / IndexType / Block::Block: restart array
// offset `ro` and restart count `nr`; ok = false is the constructor's error
// marker (size_ = 0) or NewDataIterator's "bad block contents".
struct BlkHdr {
  uint32_t ro, nr;
  bool ok;
};
__device__ __forceinline__ BlkHdr blk_header(const uint8_t* d, uint64_t n64) {
  BlkHdr h{0, 0, false};
  if (n64 < 4 || n64 > 0xFFFFFFFFull) return h;
  const uint32_t size = (uint32_t)n64;
  const uint32_t footer = blk_u32(d + size - 4);
  bool hash = false;
  uint32_t nr = footer;
  if (size <= (1u << 16)) {  // kMaxBlockSizeSupportedByHashIndex
    hash = footer >> 31;
    nr = footer & 0x7FFFFFFFu;
  }
  h.nr = nr;
  if (!hash) {
    const uint32_t ro = size - (1 + nr) * 4u;
    if (ro > size - 4u) return h;
    h.ro = ro;
  } else {
    if (size < 6) return h;
    // data_block_hash_index.cc:76-84: NUM_BUCK (u16) before the footer
    const uint16_t sz16 = (uint16_t)(size - 4);
    const uint16_t nb = (uint16_t)(blk_u8(d + sz16 - 2) | (blk_u8(d + sz16 - 1) << 8));
    const uint16_t map_offset = (uint16_t)(sz16 - 2 - nb);
    const uint32_t ro = (uint32_t)map_offset - nr * 4u;
    if (ro > map_offset) return h;
    h.ro = ro;
  }
  // NewDataIterator (:1244): a block shorter than 8 bytes with restarts
  h.ok = nr == 0 || size >= 8;
  return h;
}

// One entry at p: DecodeEntry (:37-64) / CheckAndDecodeEntry (:68-97) with
// the bounds CheckAndDecodeEntry checks; index blocks with delta-encoded
// values: DecodeEntryV4 (:110-139) and the value's encoded length from
// IndexValue::DecodeFrom (table/format.cc:137-162: delta size when shared != 0,
// else a BlockHandle; then the length-prefixed first key).  Returns the key
// delta's start or nullptr ("bad entry in block").
template <int KIND>
__device__ __forceinline__ const uint8_t* blk_entry(const uint8_t* p, const uint8_t* lim, uint32_t* sh,
                                                    uint32_t* ns, const uint8_t** val, uint32_t* vl) {
  if (lim - p < 3) return nullptr;
  uint64_t s, k, x;
  if ((p = blk_varint(p, lim, 28, &s)) == nullptr) return nullptr;
  if ((p = blk_varint(p, lim, 28, &k)) == nullptr) return nullptr;
  if (KIND == kBlkIndexDelta || KIND == kBlkIndexDeltaFk) {
    if ((uint64_t)(lim - p) < k) return nullptr;
    const uint8_t* v = p + k;
    const uint8_t* q = blk_varint(v, lim, 63, &x);
    if (q && s == 0) q = blk_varint(q, lim, 63, &x);
    if (KIND == kBlkIndexDeltaFk && q) {
      q = blk_varint(q, lim, 28, &x);
      if (q && (uint64_t)(lim - q) < x) q = nullptr;
      if (q) q += x;
    }
    if (!q) return nullptr;
    *val = v;
    *vl = (uint32_t)(q - v);
  } else {
    if ((p = blk_varint(p, lim, 28, &x)) == nullptr) return nullptr;
    if ((uint64_t)(lim - p) < k + x) return nullptr;
    *val = p + k;
    *vl = (uint32_t)x;
  }
  *sh = (uint32_t)s;
  *ns = (uint32_t)k;
  return p;
}

// Walk of one restart interval [start, end): entry count, reassembled key
// bytes and the first error, as code (r << 2 | stage): stage 0 bad entry,
// 1 shared != 0 at a restart point past the first (the reference would reuse
// the previous interval's key; BlockBuilder never writes it), 2 an entry
// running over the next restart point.  ~0 = no error.
struct BlkWalk {
  uint32_t cnt;
  uint64_t kbytes;
  uint64_t err;
};
template <int KIND>
__device__ __forceinline__ BlkWalk blk_walk(const uint8_t* d, uint32_t ro, uint32_t r, uint32_t start,
                                            uint32_t end) {
  BlkWalk w{0, 0, ~0ull};
  const uint8_t* lim = d + ro;
  const uint8_t* p = d + start;
  const uint8_t* e = d + end;
  uint32_t kl = 0;
  while (p < e) {
    uint32_t sh, ns, vl;
    const uint8_t* v;
    const uint8_t* q = blk_entry<KIND>(p, lim, &sh, &ns, &v, &vl);
    if (!q) {
      w.err = (uint64_t)r << 2;
      return w;
    }
    if (w.cnt == 0 && sh != 0) {
      w.err = ((uint64_t)r << 2) | (r ? 1u : 0u);
      return w;
    }
    if (kl < sh) {
      w.err = (uint64_t)r << 2;
      return w;
    }
    kl = sh + ns;
    w.kbytes += kl;
    w.cnt++;
    p = v + vl;
  }
  if (p != e) w.err = ((uint64_t)r << 2) | 2u;
  return w;
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
  for (int o = 32; o >= 1; o >>= 1) {
    const uint64_t u = __shfl_xor(v, o, 64);
    v = u < v ? u : v;
  }
  return v;
}
// inclusive scan across the wave
__device__ __forceinline__ uint64_t wave_incl_scan_u64(uint64_t v, uint32_t lane) {
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t u = __shfl_up(v, o, 64);
    if (lane >= (uint32_t)o) v += u;
  }
  return v;
}

// Restart array as BlockBuilder writes it: restart[0] == 0 (when there are
// entries), strictly increasing, inside the entry area.  Wave-uniform result.
__device__ __forceinline__ bool blk_restarts_ok(const uint8_t* d, const BlkHdr& h, uint32_t lane) {
  bool bad = false;
  const uint8_t* ra = d + h.ro;
  for (uint32_t r = lane; r < h.nr; r += 64) {
    const uint32_t x = blk_u32(ra + 4 * r);
    if (r == 0)
      bad |= h.ro != 0 && x != 0;
    else
      bad |= x <= blk_u32(ra + 4 * (r - 1)) || x >= h.ro;
  }
  return !__any(bad);
}

// Pass 1: per block key count / key bytes / status (+ restart interval).
// key_cnt and key_bytes receive the per-block values in place; the scan
// kernels turn them into exclusive offsets.
template <int KIND>
__global__ __launch_bounds__(256) void k_block_layout(SpanSrc blocks, uint32_t count, uint64_t* key_cnt,
                                                      uint64_t* key_bytes, uint32_t* interval_out,
                                                      int32_t* status) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  for (uint32_t b = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); b < count; b += nw) {
    const uint8_t* d = blocks.ptr(b);
    const BlkHdr h = blk_header(d, blocks.len(b));
    int st = kBlkOk;
    uint64_t keys = 0, kb = 0;
    uint32_t ri = 0;
    if (!h.ok) {
      st = kBlkBadContents;
    } else if (h.nr == 0) {
      // empty block: protection stays off, no keys
    } else if (!blk_restarts_ok(d, h, lane)) {
      st = kBlkBadRestarts;
    } else if (h.ro == 0) {
      st = h.nr == 1 ? kBlkOk : kBlkBadRestarts;
    } else {
      const uint8_t* ra = d + h.ro;
      uint64_t err = ~0ull;
      uint32_t first_cnt = 0;
      for (uint32_t r0 = 0; r0 < h.nr; r0 += 64) {
        const uint32_t r = r0 + lane;
        BlkWalk w{0, 0, ~0ull};
        if (r < h.nr) w = blk_walk<KIND>(d, h.ro, r, blk_u32(ra + 4 * r), r + 1 < h.nr ? blk_u32(ra + 4 * (r + 1)) : h.ro);
        if (r0 == 0) first_cnt = readlane_u32(w.cnt, 0);
        // every interval but the last holds interval-0's count (GetRestartInterval)
        if (r < h.nr && w.err == ~0ull && r + 1 < h.nr && w.cnt != first_cnt) w.err = ((uint64_t)r << 2) | 2u;
        err = err < w.err ? err : w.err;
        keys += w.cnt;
        kb += w.kbytes;
      }
      err = wave_min_u64(err);
      keys = wave_sum_u64(keys);
      kb = wave_sum_u64(kb);
      if (err != ~0ull) {
        st = (err & 3) == 0 ? kBlkBadEntry : kBlkBadRestarts;
      } else {
        ri = h.nr > 1 ? first_cnt : 0;
      }
    }
    if (st != kBlkOk) keys = kb = ri = 0;
    if (lane == 0) {
      key_cnt[b] = keys;
      key_bytes[b] = kb;
      if (interval_out) interval_out[b] = ri;
      status[b] = st;
    }
  }
}

// Pass 2: reassemble keys into the arena, write per-entry spans.
// key_base/arena_base: exclusive scans [count + 1].
template <int KIND>
__global__ __launch_bounds__(256) void k_block_materialize(SpanSrc blocks, uint32_t count,
                                                           const uint64_t* key_base, const uint64_t* arena_base,
                                                           uint8_t* arena, uint64_t* koff, uint32_t* klen,
                                                           uint64_t* voff, uint32_t* vlen) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  for (uint32_t b = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); b < count; b += nw) {
    const uint64_t k0 = ldg_u64(key_base, b);
    if (ldg_u64(key_base, b + 1) == k0) continue;  // no keys (or a bad block)
    const uint8_t* d = blocks.ptr(b);
    const uint64_t boff = blocks.off(b);
    const BlkHdr h = blk_header(d, blocks.len(b));
    const uint8_t* ra = d + h.ro;
    const uint8_t* lim = d + h.ro;
    uint64_t acarry = ldg_u64(arena_base, b);
    uint32_t ri = 0;
    for (uint32_t r0 = 0; r0 < h.nr; r0 += 64) {
      const uint32_t r = r0 + lane;
      const bool own = r < h.nr;
      const uint32_t start = own ? blk_u32(ra + 4 * r) : 0;
      const uint32_t end = own ? (r + 1 < h.nr ? blk_u32(ra + 4 * (r + 1)) : h.ro) : 0;
      BlkWalk w{0, 0, ~0ull};
      if (own) w = blk_walk<KIND>(d, h.ro, r, start, end);
      if (r0 == 0) ri = readlane_u32(w.cnt, 0);
      const uint64_t incl = wave_incl_scan_u64(w.kbytes, lane);
      uint64_t a = acarry + incl - w.kbytes;
      acarry += readlane_u64(incl, 63);
      if (!own) continue;
      uint64_t idx = k0 + (uint64_t)r * ri;
      const uint8_t* p = d + start;
      const uint8_t* e = d + end;
      uint64_t prev = a;
      while (p < e) {
        uint32_t sh, ns, vl;
        const uint8_t* v;
        const uint8_t* q = blk_entry<KIND>(p, lim, &sh, &ns, &v, &vl);
        // shared prefix from the previous key (this lane wrote it), then the delta
        for (uint32_t i = 0; i < sh; i++) arena[a + i] = arena[prev + i];
        for (uint32_t i = 0; i < ns; i++) arena[a + sh + i] = (uint8_t)blk_u8(q + i);
        koff[idx] = a;
        klen[idx] = sh + ns;
        voff[idx] = boff + (uint64_t)(v - d);
        vlen[idx] = vl;
        idx++;
        prev = a;
        a += sh + ns;
        p = v + vl;
      }
    }
  }
}

// ---- exclusive scan of two u64 arrays (key counts, key bytes) --------------
constexpr uint32_t kBlkScanThreads = 256, kBlkScanPer = 8, kBlkScanTile = kBlkScanThreads * kBlkScanPer;

// workgroup-wide exclusive scan of one u64 per thread; returns the total
__device__ __forceinline__ uint64_t wg_excl_scan_u64(uint64_t v, uint64_t* lds, uint64_t* excl) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t incl = wave_incl_scan_u64(v, lane);
  if (lane == 63) lds[w] = incl;
  __syncthreads();
  uint64_t base = 0, tot = 0;
  for (uint32_t i = 0; i < kBlkScanThreads / 64; i++) {
    if (i < w) base += lds[i];
    tot += lds[i];
  }
  __syncthreads();
  *excl = base + incl - v;
  return tot;
}

__global__ __launch_bounds__(256) void k_blk_scan_tiles(const uint64_t* a, const uint64_t* b, uint32_t n,
                                                        uint64_t* tsum) {
  __shared__ uint64_t lds[2][4];
  const uint64_t t0 = (uint64_t)blockIdx.x * kBlkScanTile + threadIdx.x * kBlkScanPer;
  uint64_t sa = 0, sb = 0;
  for (uint32_t k = 0; k < kBlkScanPer; k++)
    if (t0 + k < n) {
      sa += a[t0 + k];
      sb += b[t0 + k];
    }
  uint64_t ea, eb;
  const uint64_t ta = wg_excl_scan_u64(sa, lds[0], &ea);
  const uint64_t tb = wg_excl_scan_u64(sb, lds[1], &eb);
  if (threadIdx.x == 0) {
    tsum[2 * blockIdx.x] = ta;
    tsum[2 * blockIdx.x + 1] = tb;
  }
}

// one workgroup: tile sums -> exclusive tile offsets; totals to a[n], b[n]
__global__ __launch_bounds__(256) void k_blk_scan_top(uint64_t* tsum, uint32_t ntiles, uint64_t* a, uint64_t* b,
                                                      uint32_t n) {
  __shared__ uint64_t lds[2][4];
  uint64_t ca = 0, cb = 0;
  for (uint32_t t0 = 0; t0 < ntiles; t0 += kBlkScanThreads) {
    const uint32_t t = t0 + threadIdx.x;
    const uint64_t va = t < ntiles ? tsum[2 * t] : 0, vb = t < ntiles ? tsum[2 * t + 1] : 0;
    uint64_t ea, eb;
    const uint64_t ta = wg_excl_scan_u64(va, lds[0], &ea);
    const uint64_t tb = wg_excl_scan_u64(vb, lds[1], &eb);
    if (t < ntiles) {
      tsum[2 * t] = ca + ea;
      tsum[2 * t + 1] = cb + eb;
    }
    ca += ta;
    cb += tb;
  }
  if (threadIdx.x == 0) {
    a[n] = ca;
    b[n] = cb;
  }
}

__global__ __launch_bounds__(256) void k_blk_scan_apply(uint64_t* a, uint64_t* b, uint32_t n, const uint64_t* tsum) {
  __shared__ uint64_t lds[2][4];
  const uint64_t t0 = (uint64_t)blockIdx.x * kBlkScanTile + threadIdx.x * kBlkScanPer;
  uint64_t va[kBlkScanPer], vb[kBlkScanPer], sa = 0, sb = 0;
  for (uint32_t k = 0; k < kBlkScanPer; k++) {
    va[k] = t0 + k < n ? a[t0 + k] : 0;
    vb[k] = t0 + k < n ? b[t0 + k] : 0;
    sa += va[k];
    sb += vb[k];
  }
  uint64_t ea, eb;
  (void)wg_excl_scan_u64(sa, lds[0], &ea);
  (void)wg_excl_scan_u64(sb, lds[1], &eb);
  ea += tsum[2 * blockIdx.x];
  eb += tsum[2 * blockIdx.x + 1];
  for (uint32_t k = 0; k < kBlkScanPer; k++)
    if (t0 + k < n) {
      a[t0 + k] = ea;
      b[t0 + k] = eb;
      ea += va[k];
      eb += vb[k];
    }
}

}  // namespace mck
