// mck_engine.hip -- C ABI of the MI355X block-checksum engine: per-device
// context, launch geometry, the batched device entry points, the scalar
// shims and the host-resident multi-GPU pipeline.  See include/speedb_amd/
// mck.h for the contract of every function.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "../../include/speedb_amd/mck.h"
#include "mck_internal.h"
#include "mck_kernels.hpp"
#include "mck_block.hpp"
#include "mck_walrec.hpp"

namespace mck {

__device__ CrcTables g_crc_tables;

namespace {

thread_local char t_err[512] = "";

void set_err(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(t_err, sizeof t_err, fmt, ap);
  va_end(ap);
}

#define MCK_HIP(call)                                                                \
  do {                                                                               \
    hipError_t e_ = (call);                                                          \
    if (e_ != hipSuccess) {                                                          \
      set_err("%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), __FILE__, __LINE__); \
      return MCK_EHIP;                                                               \
    }                                                                                \
  } while (0)

constexpr int kMaxDev = 64;

struct DevCtx {
  std::once_flag once;
  int status = MCK_ENODEV;
  int ncu = 0;
  unsigned long long* d_stats = nullptr;  // device counters: [0] block checksum mismatches, [1] read-out slot
};
DevCtx g_dev[kMaxDev];

const CrcTables& host_tables() {
  static CrcTables* t = [] {
    CrcTables* x = new CrcTables;
    build_crc_tables(x);
    return x;
  }();
  return *t;
}

// Set the dynamic-LDS limit of a CRC kernel instantiation (once per device).
template <class K>
int ensure_lds(K kern, int dev) {
  static std::atomic<uint64_t> done{0};
  const uint64_t bit = 1ull << dev;
  if (done.load(std::memory_order_acquire) & bit) return MCK_OK;
  // the LDS images are addressed from 0: a kernel with static LDS (the
  // compiler promoting private arrays) would read shifted tables
  hipFuncAttributes fa;
  MCK_HIP(hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(kern)));
  if (fa.sharedSizeBytes != 0) {
    set_err("a CRC kernel has %zu B of static LDS; its image must start at 0", (size_t)fa.sharedSizeBytes);
    return MCK_EHIP;
  }
  MCK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)kCrcLdsBytes));
  done.fetch_or(bit, std::memory_order_acq_rel);
  return MCK_OK;
}

// Initialise the current device: check it is gfx950 and upload the tables.
int current_device(int* dev_out, int* ncu_out) {
  int dev = 0;
  MCK_HIP(hipGetDevice(&dev));
  if (dev < 0 || dev >= kMaxDev) {
    set_err("device index %d out of range", dev);
    return MCK_ENODEV;
  }
  DevCtx& d = g_dev[dev];
  std::call_once(d.once, [&] {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) {
      d.status = MCK_EHIP;
      return;
    }
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
      set_err("device %d is %s; this engine is built for gfx950 only", dev, prop.gcnArchName);
      d.status = MCK_ENODEV;
      return;
    }
    d.ncu = prop.multiProcessorCount;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_crc_tables), &host_tables(), sizeof(CrcTables)) != hipSuccess ||
        hipMalloc(&d.d_stats, 64) != hipSuccess || hipMemset(d.d_stats, 0, 64) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess) {
      d.status = MCK_EHIP;
      return;
    }
    d.status = MCK_OK;
  });
  if (d.status != MCK_OK) {
    if (!t_err[0]) set_err("device %d initialisation failed", dev);
    return d.status;
  }
  if (dev_out) *dev_out = dev;
  if (ncu_out) *ncu_out = d.ncu;
  return MCK_OK;
}

// Engine statistics (mck_statistics_get): host-side counters of the batched
// calls; the mismatch ticker is counted on each device (DevCtx::d_stats).
struct HostStats {
  std::atomic<uint64_t> compute{0}, batches{0}, spans{0}, bytes{0};
};
HostStats g_stats;

// engine-internal batched calls (host pipeline chunks, long-span pieces,
// scalar shims) are not counted again
thread_local int t_nostat = 0;
struct NoStat {
  NoStat() { t_nostat++; }
  ~NoStat() { t_nostat--; }
};

void stat_batch(uint64_t spans, uint64_t known_bytes) {
  if (t_nostat) return;
  g_stats.batches.fetch_add(1, std::memory_order_relaxed);
  g_stats.spans.fetch_add(spans, std::memory_order_relaxed);
  if (known_bytes) g_stats.bytes.fetch_add(known_bytes, std::memory_order_relaxed);
}
// bytes of a batch when the host knows them (uniform lengths)
uint64_t known_bytes(const mck_spans* s) { return s->lengths ? 0 : (uint64_t)s->length * s->count; }

unsigned long long* dev_stats(int dev) { return g_dev[dev].d_stats; }

// PerfContext::block_checksum_time (mck_perf_context_get): per thread, the
// device time of the verify batches this thread issued at a timing level,
// measured by an event pair on each batch's stream and read when asked for.
struct PerfPending {
  hipEvent_t a, b;
  int dev;
};
struct PerfCtx {
  int level = MCK_PERF_kEnableCount;  // the reference's default PerfLevel
  uint64_t time_ns = 0, count = 0, batches = 0;
  std::vector<PerfPending> pending;
  std::vector<std::pair<int, hipEvent_t>> pool;  // (device, event) for reuse
  // (events are not destroyed at thread exit: the runtime may be gone)
};
thread_local PerfCtx t_perf;

hipEvent_t perf_event(int dev) {
  for (size_t k = t_perf.pool.size(); k-- > 0;)
    if (t_perf.pool[k].first == dev) {
      hipEvent_t e = t_perf.pool[k].second;
      t_perf.pool.erase(t_perf.pool.begin() + k);
      return e;
    }
  hipEvent_t e = nullptr;
  return hipEventCreate(&e) == hipSuccess ? e : nullptr;
}

// Brackets one verify batch: begin() before its launches, end() after.
struct PerfScope {
  hipStream_t st;
  int dev = -1;
  hipEvent_t a = nullptr;
  PerfScope(hipStream_t s, uint64_t blocks) : st(s) {
    if (t_perf.level < MCK_PERF_kEnableCount) return;
    t_perf.count += blocks;
    t_perf.batches++;
    if (t_perf.level < MCK_PERF_kEnableTimeExceptForMutex || !blocks || hipGetDevice(&dev) != hipSuccess) return;
    a = perf_event(dev);
    if (a && hipEventRecord(a, st) != hipSuccess) {
      t_perf.pool.push_back({dev, a});
      a = nullptr;
    }
  }
  void end(bool ok) {
    if (!a) return;
    hipEvent_t b = ok ? perf_event(dev) : nullptr;
    if (b && hipEventRecord(b, st) == hipSuccess) {
      t_perf.pending.push_back(PerfPending{a, b, dev});
    } else {
      t_perf.pool.push_back({dev, a});
      if (b) t_perf.pool.push_back({dev, b});
    }
    a = nullptr;
  }
  ~PerfScope() { end(false); }
};

int check_spans(const mck_spans* s) {
  if (!s) {
    set_err("spans is NULL");
    return MCK_EINVAL;
  }
  if (s->count && !s->base) {
    set_err("spans->base is NULL");
    return MCK_EINVAL;
  }
  return MCK_OK;
}

SpanSrc to_src(const mck_spans* s) {
  return SpanSrc{static_cast<const uint8_t*>(s->base), s->offsets, s->lengths, s->stride, s->length};
}

// Generic CRC driver load layout: row-transposed, non-temporal loads
// (crc_drive<Op, true>: SST mix 63.0 -> 66.4 %, ragged 4 KiB 65.0 -> 69.3 %,
// 64 KiB 74.7 -> 83.4 %).
constexpr bool kCrcGenericT = true;

// Ragged batches: one launch of k_crc_ragged over the whole batch; each
// workgroup runs its contiguous share on the row drivers or the body/head
// driver, chosen on the device from a sample of the share's lengths
// (crc_share_long: the host cannot see device-resident lengths).  Both walk
// their shares in LDS windows, so one launch serves any batch size.  (Round
// 4 first launched the two drivers as two kernels over the same shares: the
// one with nothing to do still cost ~5 us per batch, 2.5 % of a 1 GiB SST
// image.)  Tests force one driver / the interleaved order through
// mck_test_set_crc_driver; production code never calls it.
std::atomic<int> g_crc_force{0}, g_crc_interleaved{0};
int crc_auto_force() { return g_crc_force.load(std::memory_order_relaxed); }
bool crc_auto_blocked() { return g_crc_interleaved.load(std::memory_order_relaxed) == 0; }

// A launch whose error comes back from hipLaunchKernel itself: no separate
// hipGetLastError call per batch (the latency path's host cost, tests/cpp/
// latency_verify.hip: the API enqueued in 3.6 us against 1.4 us for an
// empty kernel).
template <class... P, class... A>
hipError_t launch_k(void (*k)(P...), dim3 grid, dim3 block, size_t shm, hipStream_t st, A&&... args) {
  std::tuple<P...> vals{std::forward<A>(args)...};
  void* ptrs[sizeof...(P)];
  std::apply([&](auto&... v) {
    size_t i = 0;
    ((ptrs[i++] = static_cast<void*>(&v)), ...);
  }, vals);
  return hipLaunchKernel(reinterpret_cast<const void*>(k), grid, block, ptrs, shm, st);
}

template <class Op>
int launch_crc(const Op& op, uint32_t count, hipStream_t st, int dev = -1, int ncu = 0) {
  if (!count) return MCK_OK;
  int rc = 0;
  if (dev < 0 && (rc = current_device(&dev, &ncu))) return rc;
  constexpr bool T = kCrcGenericT;
  const int force = crc_auto_force();
  const bool blk = crc_auto_blocked();
  // (>= 4 spans per workgroup: a batch of a few thousand large spans -- one
  // 64 MiB SST file -- still fills every CU)
  const uint32_t grid = std::min<uint32_t>((uint32_t)ncu, (count + 3) / 4);
  if (blk && ((count <= kSmallBatch && force == 0) || force == 9)) {  // a wave per span (latency)
    if ((rc = ensure_lds(k_crc_ragged<Op, T, true, true>, dev))) return rc;
    MCK_HIP(launch_k(k_crc_ragged<Op, T, true, true>, dim3(grid), dim3(1024), kCrcLdsBytes, st, op, 0u, count,
                     force));
    return MCK_OK;
  } else if (blk) {
    if ((rc = ensure_lds(k_crc_ragged<Op, T, true>, dev))) return rc;
    hipLaunchKernelGGL((k_crc_ragged<Op, T, true>), dim3(grid), dim3(1024), kCrcLdsBytes, st, op, 0u, count,
                       force == 9 ? 0 : force);
  } else {  // the interleaved order (test hook): row drivers only
    if ((rc = ensure_lds(k_crc_ragged<Op, T, false>, dev))) return rc;
    hipLaunchKernelGGL((k_crc_ragged<Op, T, false>), dim3(grid), dim3(1024), kCrcLdsBytes, st, op, 0u, count,
                       force == 7 ? 7 : (force ? force : 8));
  }
  MCK_HIP(hipGetLastError());
  return MCK_OK;
}


// XXH3 driver choice: one 16-lane row per span for uniform batches of short
// spans (every row gets the same work; round 1 measured 5495 vs 4849 GiB/s
// at 1M x 4 KiB, before the wave kernel's byte-balanced shares and prologue
// overlap -- it now wins from ~3 KiB, below), one wave per span for ragged
// batches (a long span is not serialised on one row and waves balance
// better: SST verify mix 3287 vs 2752 GiB/s; the wave kernel itself runs
// rows for shares of 256 B - 2.5 KiB spans).
// (test hook: mck_test_set_xxh3_driver -- 1 = the wave driver, 2 = rows,
// for any batch; production code never calls it)
std::atomic<int> g_x3_force{0};
// Uniform batches of spans of >= kX3UniformWaveMin bytes go to the wave
// kernel too (round 5, microbench/x3_width.py u:<len>, profiles/r5/x3_width/
// uniform.txt: 4 KiB 0.827 vs 0.761 on rows, 16 KiB 0.801 vs 0.685; 1-2 KiB
// stay on rows, 0.774-0.815 vs 0.721-0.768).
constexpr uint32_t kX3UniformWaveMin = 3072;
#ifndef X3_UNIFORM_QUAD_MAX
#define X3_UNIFORM_QUAD_MAX 512u
#endif
template <class Op>
int launch_xxh3(const Op& op, uint32_t count, hipStream_t st, bool uniform, uint32_t uniform_len = 0) {
  if (!count) return MCK_OK;
  int ncu;
  int rc = current_device(nullptr, &ncu);
  if (rc) return rc;
  // (small batches keep the rows kernel: no share search in their latency)
  if (uniform && uniform_len >= kX3UniformWaveMin && count >= 16u * (uint32_t)ncu) uniform = false;
  // uniform spans of <= 512 bytes too: the wave kernel's rows share hashes
  // them four per row on lane quads (x3_short_quads / x3_mid_quads), the
  // rows kernel one per row
  if (uniform && uniform_len <= X3_UNIFORM_QUAD_MAX && count >= 16u * (uint32_t)ncu) uniform = false;
  const int force = g_x3_force.load(std::memory_order_relaxed);
  if (force) uniform = force == 2;
  if (!uniform) {
    // one workgroup per CU, spans dealt by LDS tickets
    const uint32_t grid = std::min<uint32_t>((uint32_t)ncu, (count + 3) / 4);
    hipLaunchKernelGGL((k_xxh3_wave<Op>), dim3(grid), dim3(kX3WaveThreads), 0, st, op, count);
  } else {
    // 16 rows (spans) per 256-thread workgroup
    const uint32_t grid = std::min<uint32_t>((uint32_t)ncu * 8, (count + 15) / 16);
    hipLaunchKernelGGL((k_xxh3<Op>), dim3(grid), dim3(256), 0, st, op, count);
  }
  MCK_HIP(hipGetLastError());
  return MCK_OK;
}

// (test hook: mck_test_set_xph3_quads(0) sends uniform short batches to the
// row driver, for the A/B and the parity of both)
#ifndef XPH3_QUADS_DEFAULT
#define XPH3_QUADS_DEFAULT 1
#endif
std::atomic<int> g_xph3_quads{XPH3_QUADS_DEFAULT};
template <class Op>
int launch_xph3(const Op& op, uint32_t count, uint64_t seed, hipStream_t st, bool uniform_short = false) {
  if (!count) return MCK_OK;
  int ncu;
  int rc = current_device(nullptr, &ncu);
  if (rc) return rc;
  if (uniform_short && g_xph3_quads.load(std::memory_order_relaxed)) {  // every span <= 240 bytes
    const uint32_t grid = std::min<uint32_t>((uint32_t)ncu * 8, (count + 63) / 64);
    hipLaunchKernelGGL(k_xph3_quads<Op>, dim3(grid), dim3(256), 0, st, op, count, seed);
    MCK_HIP(hipGetLastError());
    return MCK_OK;
  }
  const uint32_t grid = std::min<uint32_t>((uint32_t)ncu * 8, (count + 15) / 16);
  hipLaunchKernelGGL(k_xph3<Op>, dim3(grid), dim3(256), 0, st, op, count, seed);
  MCK_HIP(hipGetLastError());
  return MCK_OK;
}

template <class Op>
int launch_legacy(const Op& op, uint32_t count, hipStream_t st) {
  if (!count) return MCK_OK;
  int ncu;
  int rc = current_device(nullptr, &ncu);
  if (rc) return rc;
  const uint32_t grid = std::min<uint32_t>((uint32_t)ncu * 8, (count + 255) / 256);
  hipLaunchKernelGGL(k_legacy<Op>, dim3(grid), dim3(256), 0, st, op, count);
  MCK_HIP(hipGetLastError());
  return MCK_OK;
}

template <int MODE>
int launch_block(int type, const BlockArgs& a, uint32_t count, hipStream_t st, int dev = -1, int ncu = 0) {
  switch (type) {
    case MCK_kCRC32c:
      return launch_crc(OpCrcBlock<MODE>{a}, count, st, dev, ncu);
    case MCK_kXXH3:
      return launch_xxh3(OpX3Block<MODE>{a}, count, st, a.s.lengths == nullptr, a.s.length);
    case MCK_kxxHash:
      return launch_legacy(OpLegacyBlock<false, MODE>{a}, count, st);
    case MCK_kxxHash64:
      return launch_legacy(OpLegacyBlock<true, MODE>{a}, count, st);
    case MCK_kNoChecksum:
      return launch_legacy(OpNoneBlock<MODE>{a}, count, st);
    default:
      set_err("unknown checksum type %d", type);
      return MCK_EINVAL;
  }
}

// Value(type byte [+ LE32 log number]) for every record type, db/log_writer.cc
// :48-51 (type_crc_) and :281-291 (recyclable log number).
WalTypeCrcs wal_type_crcs(uint32_t log_number) {
  WalTypeCrcs t;
  for (int ty = 0; ty < 16; ty++) {
    uint32_t s = ~0u;
    auto feed = [&](uint8_t b) {
      s ^= b;
      for (int k = 0; k < 8; k++) s = gf_mulx(s);
    };
    feed((uint8_t)ty);
    const bool recyclable = (ty >= 5 && ty <= 8) || ty == 11;
    if (recyclable)
      for (int k = 0; k < 4; k++) feed((uint8_t)(log_number >> (8 * k)));
    t.v[ty] = ~s;
  }
  return t;
}

// ---- per-thread staging for the synchronous scalar shims ------------------
struct Staging {
  int dev = -1;
  void* d_buf = nullptr;
  size_t cap = 0;
  ~Staging() {
    if (d_buf) (void)hipFree(d_buf);
  }
};
thread_local Staging t_stage;

// d_buf = [64 B of results][data, n bytes][scratch, `extra` bytes]
int stage_in(const void* data, size_t n, uint8_t** d_data, void** d_out, size_t extra = 0,
             uint32_t** d_scratch = nullptr) {
  int dev;
  int rc = current_device(&dev, nullptr);
  if (rc) return rc;
  const size_t data_sz = (n + 64 + 255) & ~size_t(255);
  const size_t need = 64 + data_sz + extra;
  if (t_stage.dev != dev || t_stage.cap < need) {
    if (t_stage.d_buf) (void)hipFree(t_stage.d_buf);
    t_stage.d_buf = nullptr;
    t_stage.cap = 0;
    const size_t cap = std::max<size_t>(need, 1 << 20);
    MCK_HIP(hipMalloc(&t_stage.d_buf, cap));
    t_stage.cap = cap;
    t_stage.dev = dev;
  }
  *d_out = t_stage.d_buf;  // 64 bytes of results
  *d_data = static_cast<uint8_t*>(t_stage.d_buf) + 64;
  if (d_scratch) *d_scratch = reinterpret_cast<uint32_t*>(*d_data + data_sz);
  if (n) MCK_HIP(hipMemcpy(*d_data, data, n, hipMemcpyHostToDevice));
  return MCK_OK;
}

// ---- per-KV protection of block entries: launch helpers ------------------
template <template <int> class K, class... A>
int launch_blk(int kind, uint32_t count, hipStream_t st, A... args);

// Dynamic LDS that caps the walks at two workgroups (8 waves) per CU:
// fewer blocks in flight per CU keep each walk's lines in L2 between its
// header, key and value reads (100-B values, round 4: the kv walk fetched
// 2.7x its image at 4 workgroups per CU, 1.9x at 2, and ran 15 % faster;
// the layout walk 1.2x -> 1.0x, 9 % faster).
constexpr size_t kBlkLayoutLdsPad = 56 * 1024;
constexpr size_t kBlkWalkLdsPad = 17 * 1024;  // + the walks' 37 KiB key buffers
template <int KIND>
struct BlkLayoutT {
  static void go(dim3, hipStream_t st, SpanSrc s, uint32_t n, uint64_t* a, uint64_t* b, uint32_t* ri, int32_t* stt) {
    hipLaunchKernelGGL(k_block_layout_t<KIND>, dim3((n + 255) / 256), dim3(256), kBlkLayoutLdsPad, st, s, n, a, b, ri, stt);
  }
};
template <int KIND>
struct BlkKvT {
  template <class... A>
  static void go(dim3, hipStream_t st, bool verify, SpanSrc s, uint32_t n, const uint64_t* kb, const uint64_t* ab,
                 uint8_t* arena, uint64_t* long_off, uint32_t* long_len, uint64_t nkeys, uint64_t* long_part,
                 A... rest) {
    if (verify)
      hipLaunchKernelGGL((k_block_kv_t<KIND, true>), dim3((n + 255) / 256), dim3(256), kBlkWalkLdsPad, st, s, n, kb, ab, arena,
                         long_off, long_len, nkeys, long_part, rest...);
    else
      hipLaunchKernelGGL((k_block_kv_t<KIND, false>), dim3((n + 255) / 256), dim3(256), kBlkWalkLdsPad, st, s, n, kb, ab, arena,
                         long_off, long_len, nkeys, long_part, rest...);
  }
};
template <template <int> class K, class... A>
int launch_blk(int kind, uint32_t count, hipStream_t st, A... args) {
  int ncu;
  if (int rc = current_device(nullptr, &ncu)) return rc;
  const dim3 g(std::min<uint32_t>((uint32_t)ncu * 16, (count + 3) / 4));
  switch (kind) {
    case MCK_BLOCK_DATA: K<kBlkData>::go(g, st, args...); break;
    case MCK_BLOCK_INDEX: K<kBlkIndex>::go(g, st, args...); break;
    case MCK_BLOCK_INDEX_DELTA: K<kBlkIndexDelta>::go(g, st, args...); break;
    case MCK_BLOCK_INDEX_DELTA_FIRST_KEY: K<kBlkIndexDeltaFk>::go(g, st, args...); break;
    case MCK_BLOCK_META: K<kBlkMeta>::go(g, st, args...); break;
    default:
      set_err("unknown block kind %d", kind);
      return MCK_EINVAL;
  }
  MCK_HIP(hipGetLastError());
  return MCK_OK;
}

uint64_t blk_tiles(uint32_t count) { return ((uint64_t)count + kBlkScanTile - 1) / kBlkScanTile; }

// work area: [long_off u64 K][long_part u64 K][long_len u32 K][u32: long values recorded][spare] [key arena]
// (the long-value list of k_block_kv_t / k_block_long_rows, indexed by key)
struct BlkWork {
  uint64_t *long_off, *long_part;
  uint32_t* long_len;
  uint8_t* arena;
};
uint64_t blk_work_head(uint64_t keys) { return (keys * 24 + 255) & ~255ull; }
BlkWork blk_work(void* work, uint64_t keys) {
  uint8_t* w = static_cast<uint8_t*>(work);
  return BlkWork{reinterpret_cast<uint64_t*>(w), reinterpret_cast<uint64_t*>(w + 8 * keys),
                 reinterpret_cast<uint32_t*>(w + 16 * keys), w + blk_work_head(keys)};
}

int blk_kv(int kind, const mck_spans* blocks, uint32_t prot_bytes, const uint64_t* key_base,
           const uint64_t* arena_base, const uint32_t* restart_interval, uint64_t total_keys, void* work,
           uint8_t* enc, const uint8_t* stored, uint8_t* mismatch, uint32_t* mismatch_count, hipStream_t st) {
  if (int rc = check_spans(blocks)) return rc;
  if (kind < MCK_BLOCK_DATA || kind > MCK_BLOCK_META) {
    set_err("unknown block kind %d", kind);
    return MCK_EINVAL;
  }
  if (prot_bytes != 1 && prot_bytes != 2 && prot_bytes != 4 && prot_bytes != 8) {
    set_err("protection_bytes_per_key must be 1, 2, 4 or 8 (got %u)", prot_bytes);
    return MCK_EINVAL;
  }
  if (blocks->count && (!key_base || !arena_base || !restart_interval)) {
    set_err("key_base/arena_base/restart_interval is NULL");
    return MCK_EINVAL;
  }
  if (total_keys && !work) {
    set_err("work is NULL");
    return MCK_EINVAL;
  }
  if (!total_keys || !blocks->count) return MCK_OK;
  if (total_keys > 0xFFFFFFFFull) {
    set_err("more than 2^32 - 1 keys in one batch (%llu)", (unsigned long long)total_keys);
    return MCK_EINVAL;
  }
  const BlkWork w = blk_work(work, total_keys);
  const bool verify = stored != nullptr;
  // no long value unless the walk records one; [total_keys] counts them
  MCK_HIP(hipMemsetAsync(w.long_len, 0, 4 * total_keys + 4, st));
  if (int rc = launch_blk<BlkKvT>(kind, blocks->count, st, verify, to_src(blocks), blocks->count, key_base,
                                  arena_base, w.arena, w.long_off, w.long_len, total_keys, w.long_part, prot_bytes,
                                  enc, stored,
                                  mismatch, mismatch_count))
    return rc;
  int ncu;
  if (int rc = current_device(nullptr, &ncu)) return rc;
  // 16 keys per row chunk; rows = 16 per workgroup of 256
  const uint32_t grid = (uint32_t)std::min<uint64_t>((uint64_t)ncu * 8, (total_keys + 255) / 256);
  if (verify)
    hipLaunchKernelGGL(k_block_long_rows<true>, dim3(grid), dim3(256), 0, st,
                       OpBlkLongRows<true>{w.long_off, w.long_len, w.long_part, prot_bytes, enc, stored, mismatch,
                                           mismatch_count, w.long_len + total_keys},
                       key_base, blocks->count, total_keys);
  else
    hipLaunchKernelGGL(k_block_long_rows<false>, dim3(grid), dim3(256), 0, st,
                       OpBlkLongRows<false>{w.long_off, w.long_len, w.long_part, prot_bytes, enc, stored, mismatch,
                                            mismatch_count, w.long_len + total_keys},
                       key_base, blocks->count, total_keys);
  MCK_HIP(hipGetLastError());
  return MCK_OK;
}

// ---- one pass: k_block_kv_walk + scan + k_block_kv_flush + long values -----
// (MCK_BLK_WALK_PAD: dynamic LDS added to the walk's launch, an occupancy
// A/B knob for variant builds; the product build adds none)
#ifndef MCK_BLK_WALK_PAD
#define MCK_BLK_WALK_PAD 0
#endif
template <int KIND>
struct BlkWalkT {
  template <class... A>
  static void go(dim3, hipStream_t st, uint32_t n, size_t lds_pad, A... args) {
    hipLaunchKernelGGL(k_block_kv_walk<KIND>, dim3((n + 255) / 256), dim3(256), lds_pad, st, args...);
  }
};
static_assert(kBlkSlotOverflow == MCK_BLOCK_SLOT_OVERFLOW, "status codes");

// work: [scan tiles][flag u32, pad to 256][slot_h, slot_m: u64 x count x stride][long masks]
//       [long_off u64 x K][long_part u64 x K][long_len u32 x K][arena count x arena_cap]
//       [walk key_base, walk arena_base: u64 x (count + 1) each; verify only], K = count x slot_cap
struct BlkBlocksWork {
  uint64_t* tsum;
  uint32_t* flag;
  uint64_t *slot_h, *slot_m;
  uint32_t* blk_long;
  uint64_t *long_off, *long_part;
  uint32_t* long_len;
  uint8_t* arena;
  uint64_t *walk_kb, *walk_ab;
  uint64_t bytes;
};
BlkBlocksWork blk_blocks_work(void* work, uint32_t count, uint32_t slot_cap, uint32_t arena_cap) {
  auto up = [](uint64_t x) { return (x + 255) & ~255ull; };
  const uint64_t K = (uint64_t)count * slot_cap;
  uint8_t* w = static_cast<uint8_t*>(work);
  BlkBlocksWork r{};
  uint64_t o = 0;
  r.tsum = reinterpret_cast<uint64_t*>(w + o);
  o += up(16 * blk_tiles(count) + 64);
  r.flag = reinterpret_cast<uint32_t*>(w + o);
  o += 256;
  const uint64_t S = blk_slot_count(count) * blk_slot_stride(slot_cap);
  r.slot_h = reinterpret_cast<uint64_t*>(w + o);
  o += up(8 * S);
  r.slot_m = reinterpret_cast<uint64_t*>(w + o);
  o += up(8 * S);
  r.blk_long = reinterpret_cast<uint32_t*>(w + o);
  o += up(4ull * count * blk_long_words(slot_cap));
  r.long_off = reinterpret_cast<uint64_t*>(w + o);
  o += up(8 * K);
  r.long_part = reinterpret_cast<uint64_t*>(w + o);
  o += up(8 * K);
  r.long_len = reinterpret_cast<uint32_t*>(w + o);
  o += up(4 * K + 4);
  r.arena = w + o;
  o += up((uint64_t)count * arena_cap + 16);
  r.walk_kb = reinterpret_cast<uint64_t*>(w + o);
  o += up(8ull * (count + 1));
  r.walk_ab = reinterpret_cast<uint64_t*>(w + o);
  o += up(8ull * (count + 1));
  r.bytes = o;
  return r;
}

// Protect (prot_base == nullptr): key_base / arena_base are the caller's
// outputs.  Verify: prot_base / total_keys are the protect-time key index
// (what `stored` and `mismatch` are laid out by); the walk's own index goes
// to the work area and only decides which blocks still match it.
int blk_kv_blocks(int kind, const mck_spans* blocks, uint32_t prot_bytes, uint32_t slot_cap, uint32_t arena_cap,
                  uint64_t* key_base, uint64_t* arena_base, const uint64_t* prot_base, uint64_t total_keys,
                  uint32_t* restart_interval, int32_t* status, void* work, uint8_t* enc, const uint8_t* stored,
                  uint8_t* mismatch, uint32_t* mismatch_count, hipStream_t st) {
  if (int rc = check_spans(blocks)) return rc;
  if (kind < MCK_BLOCK_DATA || kind > MCK_BLOCK_META) {
    set_err("unknown block kind %d", kind);
    return MCK_EINVAL;
  }
  if (prot_bytes != 1 && prot_bytes != 2 && prot_bytes != 4 && prot_bytes != 8) {
    set_err("protection_bytes_per_key must be 1, 2, 4 or 8 (got %u)", prot_bytes);
    return MCK_EINVAL;
  }
  stat_batch(blocks->count, known_bytes(blocks));
  const bool verify = stored != nullptr;
  if (verify ? !prot_base : (!key_base || !arena_base)) {
    set_err(verify ? "key_base (protect-time) is NULL" : "key_base/arena_base is NULL");
    return MCK_EINVAL;
  }
  const uint32_t n = blocks->count;
  if (!n) {
    if (!verify) {
      MCK_HIP(hipMemsetAsync(key_base, 0, 8, st));
      MCK_HIP(hipMemsetAsync(arena_base, 0, 8, st));
    }
    return MCK_OK;
  }
  if (!restart_interval || !status || !work || (!enc && !stored) || (verify && total_keys && !mismatch)) {
    set_err("restart_interval/status/work/out is NULL");
    return MCK_EINVAL;
  }
  if (slot_cap == 0 || blk_slot_count(n) * blk_slot_stride(slot_cap) > 0xFFFFFFFFull) {
    set_err("slot_cap must be >= 1 with count * slot_cap < 2^32 (got %u x %u)", n, slot_cap);
    return MCK_EINVAL;
  }
  const uint64_t K = (uint64_t)n * slot_cap;  // room of the long-value list
  if (verify && total_keys > K) {
    set_err("total_keys %llu exceeds count * slot_cap = %llu: verify this batch with "
            "mck_block_kv_verify_batch", (unsigned long long)total_keys, (unsigned long long)K);
    return MCK_EINVAL;
  }
  const BlkBlocksWork w = blk_blocks_work(work, n, slot_cap, arena_cap);
  uint64_t* const kb = verify ? w.walk_kb : key_base;
  uint64_t* const ab = verify ? w.walk_ab : arena_base;
  MCK_HIP(hipMemsetAsync(w.flag, 0, 4, st));
  // (the walk's key buffers + entry windows, 73 KiB static, already hold it
  // at two workgroups per CU: no pad)
  if (int rc = launch_blk<BlkWalkT>(kind, n, st, n, (size_t)MCK_BLK_WALK_PAD, to_src(blocks), n, slot_cap, w.arena, arena_cap,
                                    w.slot_h, w.slot_m, w.blk_long, kb, ab, restart_interval, status, w.flag))
    return rc;
  const uint32_t tiles = (uint32_t)blk_tiles(n);
  hipLaunchKernelGGL(k_blk_scan_tiles, dim3(tiles), dim3(kBlkScanThreads), 0, st, kb, ab, n, w.tsum);
  hipLaunchKernelGGL(k_blk_scan_top, dim3(1), dim3(kBlkScanThreads), 0, st, w.tsum, tiles, kb, ab, n);
  hipLaunchKernelGGL(k_blk_scan_apply, dim3(tiles), dim3(kBlkScanThreads), 0, st, kb, ab, n, w.tsum);
  int ncu;
  if (int rc = current_device(nullptr, &ncu)) return rc;
  const uint32_t stride = blk_slot_stride(slot_cap);
  const uint32_t npairs = n * (stride / 2);
  // 4 pairs per thread (wave-interleaved slots: a workgroup per 64-block
  // chunk)
  const uint32_t fgrid = MCK_BLK_SLOT_T ? (uint32_t)((n + 63) / 64) : (uint32_t)(((uint64_t)npairs + 1023) / 1024);
  const uint64_t kcap = verify ? total_keys : K;
  const uint64_t* const kidx = verify ? prot_base : kb;  // the index the outputs are laid out by
  if (verify) {
    hipLaunchKernelGGL(k_block_kv_verify_bad, dim3((n + 255) / 256), dim3(256), 0, st, n, kb, prot_base, status,
                       kcap, mismatch, mismatch_count, w.long_len, w.flag);
    hipLaunchKernelGGL(k_block_kv_flush<true>, dim3(fgrid), dim3(256), 0, st, to_src(blocks), npairs, stride,
                       w.slot_h, w.slot_m, w.blk_long, kb, prot_base, kcap, prot_bytes, enc, stored, mismatch,
                       mismatch_count, w.long_off, w.long_len, w.long_part, w.flag);
  } else {
    hipLaunchKernelGGL(k_block_kv_flush<false>, dim3(fgrid), dim3(256), 0, st, to_src(blocks), npairs, stride,
                       w.slot_h, w.slot_m, w.blk_long, kb, kb, kcap, prot_bytes, enc, stored, mismatch,
                       mismatch_count, w.long_off, w.long_len, w.long_part, w.flag);
  }
  const uint32_t grid = (uint32_t)std::min<uint64_t>((uint64_t)ncu * 8, (K + 255) / 256);
  if (verify)
    hipLaunchKernelGGL(k_block_long_rows<true>, dim3(grid), dim3(256), 0, st,
                       OpBlkLongRows<true>{w.long_off, w.long_len, w.long_part, prot_bytes, enc, stored, mismatch,
                                           mismatch_count, w.flag},
                       kidx, n, kcap);
  else
    hipLaunchKernelGGL(k_block_long_rows<false>, dim3(grid), dim3(256), 0, st,
                       OpBlkLongRows<false>{w.long_off, w.long_len, w.long_part, prot_bytes, enc, stored, mismatch,
                                            mismatch_count, w.flag},
                       kidx, n, kcap);
  MCK_HIP(hipGetLastError());
  return MCK_OK;
}
}  // namespace
}  // namespace mck

using namespace mck;

// ============================================================================
extern "C" {

const char* mck_last_error(void) { return t_err; }
void mck_internal_set_error(const char* msg) { snprintf(t_err, sizeof t_err, "%s", msg); }
const char* mck_version(void) { return "speedb_amd mck 0.1 (gfx950)"; }

int mck_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  int good = 0;
  for (int i = 0; i < n; i++) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, i) == hipSuccess && strncmp(p.gcnArchName, "gfx950", 6) == 0) good++;
  }
  return good;
}

// ---- scalar u32 algebra (host) ------------------------------------------
uint32_t mck_crc32c_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + 0xa282ead8u; }
uint32_t mck_crc32c_unmask(uint32_t m) {
  const uint32_t rot = m - 0xa282ead8u;
  return (rot >> 17) | (rot << 15);
}
// Value(A||B) = zshift(Value(A), |B|) ^ Value(B): util/crc32c.cc:1221-1289
uint32_t mck_crc32c_combine(uint32_t crc1, uint32_t crc2, size_t crc2len) {
  return gf_zshift(crc1, crc2len) ^ crc2;
}
uint32_t mck_context_modifier(uint32_t base, uint64_t offset) {
  const uint32_t all_or_nothing = 0u - (uint32_t)(base != 0);
  return (base ^ ((uint32_t)offset + (uint32_t)(offset >> 32))) & all_or_nothing;
}

// ---- batched device API ----------------------------------------------------
int mck_crc32c_batch(const mck_spans* spans, const uint32_t* init_crcs, uint32_t flags, uint32_t* out,
                     mck_stream_t stream) {
  t_err[0] = 0;
  if (int rc = check_spans(spans)) return rc;
  stat_batch(spans->count, known_bytes(spans));
  if (spans->count && !out) {
    set_err("out is NULL");
    return MCK_EINVAL;
  }
  const OpCrcValue op{to_src(spans), init_crcs, flags & MCK_F_MASK, out};
  // uniform batches too: k_crc_ragged reads off(i) = i * stride (round 5
  // retired the uniform-batch kernel, slower at every length)
  if (!init_crcs)  // (no init array: OpCrcValueZ takes the rows' combined finish maps)
    return launch_crc(OpCrcValueZ{op}, spans->count, reinterpret_cast<hipStream_t>(stream));
  return launch_crc(op, spans->count, reinterpret_cast<hipStream_t>(stream));
}

// file/writable_file_writer.cc:743-747: EncodeFixed32(Extend(0, piece)) --
// the batched CRC with init 0, unmasked (the LE32 bytes are the u32 itself).
int mck_handoff_checksum_batch(const mck_spans* pieces, uint32_t* out, mck_stream_t stream) {
  return mck_crc32c_batch(pieces, nullptr, 0u, out, stream);
}

int mck_xxh3_64_batch(const mck_spans* spans, uint64_t* out, mck_stream_t stream) {
  t_err[0] = 0;
  if (int rc = check_spans(spans)) return rc;
  stat_batch(spans->count, known_bytes(spans));
  if (spans->count && !out) {
    set_err("out is NULL");
    return MCK_EINVAL;
  }
  return launch_xxh3(OpX3Value{to_src(spans), out}, spans->count, reinterpret_cast<hipStream_t>(stream),
                     spans->lengths == nullptr, spans->length);
}

int mck_xxh32_batch(const mck_spans* spans, uint32_t seed, uint32_t* out, mck_stream_t stream) {
  t_err[0] = 0;
  if (int rc = check_spans(spans)) return rc;
  stat_batch(spans->count, known_bytes(spans));
  if (spans->count && !out) {
    set_err("out is NULL");
    return MCK_EINVAL;
  }
  return launch_legacy(OpLegacyValue<false>{to_src(spans), seed, out}, spans->count,
                       reinterpret_cast<hipStream_t>(stream));
}

int mck_xxh64_batch(const mck_spans* spans, uint64_t seed, uint64_t* out, mck_stream_t stream) {
  t_err[0] = 0;
  if (int rc = check_spans(spans)) return rc;
  stat_batch(spans->count, known_bytes(spans));
  if (spans->count && !out) {
    set_err("out is NULL");
    return MCK_EINVAL;
  }
  return launch_legacy(OpLegacyValue<true>{to_src(spans), seed, out}, spans->count,
                       reinterpret_cast<hipStream_t>(stream));
}

int mck_builtin_checksum_batch(int type, const mck_spans* spans, const uint8_t* last_bytes, uint32_t* out,
                               mck_stream_t stream) {
  t_err[0] = 0;
  if (int rc = check_spans(spans)) return rc;
  stat_batch(spans->count, known_bytes(spans));
  if (spans->count && !out) {
    set_err("out is NULL");
    return MCK_EINVAL;
  }
  BlockArgs a{to_src(spans), last_bytes, nullptr, 0, out, nullptr, nullptr, nullptr};
  return launch_block<kModeBuiltin>(type, a, spans->count, reinterpret_cast<hipStream_t>(stream));
}

int mck_sst_trailer_batch(int type, const mck_spans* payloads, const uint8_t* comp_types,
                          const uint64_t* file_offsets, uint32_t base_context_checksum, uint32_t* out,
                          mck_stream_t stream) {
  t_err[0] = 0;
  if (int rc = check_spans(payloads)) return rc;
  stat_batch(payloads->count, known_bytes(payloads));
  if (payloads->count && (!out || !comp_types)) {
    set_err("out / comp_types is NULL");
    return MCK_EINVAL;
  }
  BlockArgs a{to_src(payloads), comp_types, file_offsets, base_context_checksum, out, nullptr, nullptr, nullptr};
  return launch_block<kModeTrailer>(type, a, payloads->count, reinterpret_cast<hipStream_t>(stream));
}

int mck_sst_verify_batch(int type, const mck_spans* payloads, const uint64_t* file_offsets,
                         uint32_t base_context_checksum, uint8_t* mismatch, uint32_t* computed, uint32_t* stored,
                         uint32_t* mismatch_count, mck_stream_t stream) {
  t_err[0] = 0;
  if (int rc = check_spans(payloads)) return rc;
  stat_batch(payloads->count, known_bytes(payloads));
  if (payloads->count && !mismatch) {
    set_err("mismatch is NULL");
    return MCK_EINVAL;
  }
  BlockArgs a{to_src(payloads), nullptr, file_offsets, base_context_checksum, computed, mismatch, stored,
              mismatch_count};
  // BLOCK_CHECKSUM_COMPUTE_COUNT (include/rocksdb/statistics.h:451): one
  // per VerifyBlockChecksum; mismatches are counted on the device
  g_stats.compute.fetch_add(payloads->count, std::memory_order_relaxed);
  int dev = -1, ncu = 0;  // one device lookup for the whole call
  if (payloads->count) {
    if (int rc = current_device(&dev, &ncu)) return rc;
    a.stats_mismatch = dev_stats(dev);
  }
  PerfScope perf(reinterpret_cast<hipStream_t>(stream), payloads->count);
  const int rc = launch_block<kModeVerify>(type, a, payloads->count, reinterpret_cast<hipStream_t>(stream), dev, ncu);
  perf.end(rc == MCK_OK);
  return rc;
}

int mck_wal_record_crc_batch(const mck_spans* payloads, const uint8_t* types, uint32_t log_number, uint32_t* out,
                             mck_stream_t stream) {
  t_err[0] = 0;
  if (int rc = check_spans(payloads)) return rc;
  stat_batch(payloads->count, known_bytes(payloads));
  if (payloads->count && (!out || !types)) {
    set_err("out / types is NULL");
    return MCK_EINVAL;
  }
  return launch_crc(OpCrcWal{to_src(payloads), types, wal_type_crcs(log_number), out}, payloads->count,
                    reinterpret_cast<hipStream_t>(stream));
}

int mck_wal_verify_batch(const void* wal, uint64_t nbytes, uint32_t log_number, mck_wal_block_result* results,
                         mck_stream_t stream) {
  t_err[0] = 0;
  static_assert(sizeof(mck_wal_block_result) == sizeof(WalResult), "layout");
  if (!nbytes) return MCK_OK;
  if (!wal || !results) {
    set_err("wal / results is NULL");
    return MCK_EINVAL;
  }
  const uint64_t nb64 = (nbytes + 32767) / 32768;
  if (nb64 > 0xFFFFFFFFull) {
    set_err("WAL image too large");
    return MCK_EINVAL;
  }
  int dev, ncu;
  if (int rc = current_device(&dev, &ncu)) return rc;
  if (int rc = ensure_lds(k_wal_verify<true>, dev)) return rc;
  const uint32_t nblocks = (uint32_t)nb64;
  const uint32_t grid = std::min<uint32_t>(ncu, (nblocks + 15) / 16);
  hipLaunchKernelGGL(k_wal_verify<true>, dim3(grid), dim3(1024), kCrcLdsBytes,
                     reinterpret_cast<hipStream_t>(stream), static_cast<const uint8_t*>(wal), nbytes, log_number,
                     reinterpret_cast<WalResult*>(results), nblocks);
  MCK_HIP(hipGetLastError());
  return MCK_OK;
}

// One device pass of WAL recovery (mck_walrec.hpp): the CRC verdict of every
// physical record of a host plan and, from the same registers, the XXH3
// record checksum of the one-fragment records.
int mck_wal_recover_batch(const void* wal, const mck_wal_rec_desc* recs, uint32_t count, uint32_t log_number,
                          uint8_t* crc_ok, uint64_t* record_hashes, mck_stream_t stream) {
  t_err[0] = 0;
  static_assert(sizeof(mck_wal_rec_desc) == sizeof(WalRecDesc), "layout");
  if (!count) return MCK_OK;
  if (!wal || !recs || !crc_ok || !record_hashes) {
    set_err("wal / recs / crc_ok / record_hashes is NULL");
    return MCK_EINVAL;
  }
  int dev, ncu;
  if (int rc = current_device(&dev, &ncu)) return rc;
  const uint32_t grid = std::min<uint32_t>(ncu, (count + 63) / 64);
  const WrArgs a{static_cast<const uint8_t*>(wal), reinterpret_cast<const WalRecDesc*>(recs), count, crc_ok,
                 record_hashes};
  // (round 6 A/B: the rows loop unrolled twice, its rows and loads swapping
  // register names, 0.640 / 0.317 of peak on the 32 KiB / 100 B - 4 KiB logs
  // against 0.629 / 0.313 copying them every round; profiles/r6/walrec_ab/)
  if (int rc = ensure_lds(k_wal_recover<true>, dev)) return rc;
  hipLaunchKernelGGL(k_wal_recover<true>, dim3(grid), dim3(1024), kCrcLdsBytes, reinterpret_cast<hipStream_t>(stream),
                     a, wal_type_crcs(log_number));
  MCK_HIP(hipGetLastError());
  return MCK_OK;
}

// ---- device WAL writer -------------------------------------------------------
// ONE kernel, k_wal_write_il (mck_kernels.hpp): the row
// driver's loop (16-lane rows, 80-byte lane chunks of interleaved 16-byte
// pieces, one ~1 KB fragment per 1280-byte round) CRCs every fragment and,
// from the same registers, writes the log stream; contiguous fragment ranges
// per workgroup, in LDS windows of kRowDescCache (one launch per batch).
// (Round 2 measured the alternatives --
// two kernels overlapped in pieces on a side stream, 8-lane rows, 64-byte
// chunks, re-reading copies, interleaved order -- and kept this one; they
// were removed from the library in round 3.)
int mck_wal_write_batch(const void* src, const mck_wal_fragment* frags, uint32_t nfrags, uint32_t log_number,
                        uint32_t* crc_scratch, void* out, mck_stream_t stream) {
  t_err[0] = 0;
  static_assert(sizeof(mck_wal_fragment) == sizeof(WalFrag), "layout");
  if (!nfrags) return MCK_OK;
  if (!src || !frags || !crc_scratch || !out) {
    set_err("src / frags / crc_scratch / out is NULL");
    return MCK_EINVAL;
  }
  if (reinterpret_cast<uintptr_t>(out) & 15u) {
    set_err("out must be 16-byte aligned");
    return MCK_EINVAL;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const WalFrag* f = reinterpret_cast<const WalFrag*>(frags);
  const OpWalWrite op{static_cast<const uint8_t*>(src), f, wal_type_crcs(log_number), log_number, crc_scratch,
                      static_cast<uint8_t*>(out)};
  int dev, ncu;
  if (int rc = current_device(&dev, &ncu)) return rc;
  if (int rc = ensure_lds(k_wal_write_il, dev)) return rc;
  // one launch: each workgroup walks its range in LDS windows (wal_write_il)
  const uint32_t grid = std::min<uint32_t>(ncu, (nfrags + 63) / 64);
  hipLaunchKernelGGL(k_wal_write_il, dim3(grid), dim3(1024), kCrcLdsBytes, st, op, 0u, nfrags);
  MCK_HIP(hipGetLastError());
  return MCK_OK;
}

int mck_wal_gather_batch(const void* wal, const mck_wal_fragment* frags, uint32_t nfrags, void* out,
                         mck_stream_t stream) {
  t_err[0] = 0;
  if (!nfrags) return MCK_OK;
  if (!wal || !frags || !out) {
    set_err("wal / frags / out is NULL");
    return MCK_EINVAL;
  }
  if (reinterpret_cast<uintptr_t>(out) & 15u) {
    set_err("out must be 16-byte aligned");
    return MCK_EINVAL;
  }
  int ncu;
  if (int rc = current_device(nullptr, &ncu)) return rc;
  const uint32_t grid = std::min<uint32_t>((uint32_t)ncu * 8, (nfrags + 3) / 4);
  hipLaunchKernelGGL(k_wal_gather, dim3(grid), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     static_cast<const uint8_t*>(wal), reinterpret_cast<const WalFrag*>(frags), nfrags,
                     static_cast<uint8_t*>(out));
  MCK_HIP(hipGetLastError());
  return MCK_OK;
}

// ---- blob log records --------------------------------------------------------
int mck_blob_record_batch(int write, void* file, const uint64_t* record_offsets, const uint32_t* blob_lengths,
                          uint32_t count, uint8_t* status, uint32_t* mismatch_count, mck_stream_t stream) {
  t_err[0] = 0;
  if (count && (!file || !record_offsets || !blob_lengths || (!write && !status))) {
    set_err("file / record_offsets / blob_lengths / status is NULL");
    return MCK_EINVAL;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (write)
    return launch_crc(OpBlobRecord<true>{static_cast<const uint8_t*>(file), record_offsets, blob_lengths, nullptr,
                                         nullptr},
                      count, st);
  return launch_crc(OpBlobRecord<false>{static_cast<const uint8_t*>(file), record_offsets, blob_lengths, status,
                                        mismatch_count},
                    count, st);
}

// ---- long spans ------------------------------------------------------------
uint64_t mck_crc32c_long_scratch_words(uint64_t n) {
  return (n + MCK_LONG_PIECE_BYTES - 1) / MCK_LONG_PIECE_BYTES;
}

int mck_crc32c_long(const void* data, uint64_t n, uint32_t init_crc, uint32_t* scratch, uint32_t* out,
                    mck_stream_t stream) {
  t_err[0] = 0;
  if (!out || (n && (!data || !scratch))) {
    set_err("data / scratch / out is NULL");
    return MCK_EINVAL;
  }
  const uint64_t P = MCK_LONG_PIECE_BYTES;
  const uint64_t full = n / P, tail = n % P, npieces = full + (tail ? 1 : 0);
  if (npieces > 0xFFFFFFFFull) {
    set_err("span too long (%llu pieces)", (unsigned long long)npieces);
    return MCK_EINVAL;
  }
  int dev, ncu;
  if (int rc = current_device(&dev, &ncu)) return rc;
  stat_batch(1, n);
  NoStat nostat;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // seed: ~zshift(~init, n); n == 0 leaves init_crc (Extend(c, "") = c)
  MCK_HIP(hipMemsetD32Async(out, (int)~gf_zshift(~init_crc, n), 1, st));
  if (!n) return MCK_OK;
  if (full) {
    const mck_spans s{data, nullptr, nullptr, P, (uint32_t)P, (uint32_t)full};
    if (int rc = mck_crc32c_batch(&s, nullptr, 0, scratch, stream)) return rc;
  }
  if (tail) {
    const mck_spans s{static_cast<const uint8_t*>(data) + full * P, nullptr, nullptr, 0, (uint32_t)tail, 1};
    if (int rc = mck_crc32c_batch(&s, nullptr, 0, scratch + full, stream)) return rc;
  }
  static const CrcPowers pw = [] {
    CrcPowers p;
    for (int k = 0; k < 64; k++) p.x8[k] = gf_xpow8n(1ull << k);
    return p;
  }();
  static const uint32_t c_full = gf_zshift(0xFFFFFFFFu, P);
  const uint32_t c_tail = gf_zshift(0xFFFFFFFFu, tail);
  const uint32_t grid = (uint32_t)((npieces + 255) / 256);
  hipLaunchKernelGGL(k_crc_combine, dim3(grid), dim3(256), 0, st, scratch, (uint32_t)npieces, P, n, c_full, c_tail,
                     pw, out);
  MCK_HIP(hipGetLastError());
  return MCK_OK;
}

// ---- scalar data shims (GPU, synchronous) ----------------------------------
// Extend over more than this many bytes goes through the long-span path
// (pieces hashed in parallel + device combine) instead of one span.
constexpr size_t kShimLongBytes = 1u << 20;

// kind 0: Extend(init, data); kind 1: ComputeBuiltinChecksum[WithLastByte].
static int scalar_u32(int kind, uint32_t init, const void* data, size_t n, int type, int has_last, char last,
                      uint32_t* res) {
  t_err[0] = 0;
  NoStat nostat;
  if (!res) {
    set_err("out is NULL");
    return MCK_EINVAL;
  }
  *res = 0;
  if (!data && n) {
    set_err("data is NULL");
    return MCK_EINVAL;
  }
  uint8_t* d_data;
  void* d_out;
  int rc;
  if (kind == 0 && n > kShimLongBytes) {
    uint32_t* d_scratch;
    if ((rc = stage_in(data, n, &d_data, &d_out, 4 * mck_crc32c_long_scratch_words(n), &d_scratch))) return rc;
    if ((rc = mck_crc32c_long(d_data, n, init, d_scratch, static_cast<uint32_t*>(d_out), nullptr))) return rc;
    MCK_HIP(hipMemcpy(res, d_out, 4, hipMemcpyDeviceToHost));
    return MCK_OK;
  }
  if (n > 0xFFFFFFFFull) {
    set_err("span too long for the scalar shim");
    return MCK_EINVAL;
  }
  if ((rc = stage_in(data, n, &d_data, &d_out))) return rc;
  uint8_t* d_last = static_cast<uint8_t*>(d_out) + 32;
  if (has_last) MCK_HIP(hipMemcpy(d_last, &last, 1, hipMemcpyHostToDevice));
  const mck_spans s{d_data, nullptr, nullptr, 0, (uint32_t)n, 1};
  uint32_t* d_init = static_cast<uint32_t*>(d_out) + 4;
  if (kind == 0) {
    MCK_HIP(hipMemcpy(d_init, &init, 4, hipMemcpyHostToDevice));
    rc = mck_crc32c_batch(&s, d_init, 0, static_cast<uint32_t*>(d_out), nullptr);
  } else {
    rc = mck_builtin_checksum_batch(type, &s, has_last ? d_last : nullptr, static_cast<uint32_t*>(d_out), nullptr);
  }
  if (rc) return rc;
  MCK_HIP(hipMemcpy(res, d_out, 4, hipMemcpyDeviceToHost));
  return MCK_OK;
}

// kind 0: XXH3_64bits; kind 1: NPHash64(seed).
static int scalar_u64(int kind, const void* data, size_t n, uint64_t seed, uint64_t* res) {
  t_err[0] = 0;
  NoStat nostat;
  if (!res) {
    set_err("out is NULL");
    return MCK_EINVAL;
  }
  *res = 0;
  if (!data && n) {
    set_err("data is NULL");
    return MCK_EINVAL;
  }
  if (n > 0xFFFFFFFFull) {
    set_err("span too long for the scalar shim");
    return MCK_EINVAL;
  }
  uint8_t* d_data;
  void* d_out;
  int rc;
  if ((rc = stage_in(data, n, &d_data, &d_out))) return rc;
  const mck_spans s{d_data, nullptr, nullptr, 0, (uint32_t)n, 1};
  rc = kind == 0 ? mck_xxh3_64_batch(&s, static_cast<uint64_t*>(d_out), nullptr)
                 : mck_np_hash64_batch(&s, seed, static_cast<uint64_t*>(d_out), nullptr);
  if (rc) return rc;
  MCK_HIP(hipMemcpy(res, d_out, 8, hipMemcpyDeviceToHost));
  return MCK_OK;
}

int mck_crc32c_extend_r(uint32_t init_crc, const void* data, size_t n, uint32_t* out) {
  return scalar_u32(0, init_crc, data, n, 0, 0, 0, out);
}
int mck_crc32c_value_r(const void* data, size_t n, uint32_t* out) { return scalar_u32(0, 0, data, n, 0, 0, 0, out); }
int mck_builtin_checksum_r(int type, const void* data, size_t n, uint32_t* out) {
  return scalar_u32(1, 0, data, n, type, 0, 0, out);
}
int mck_builtin_checksum_with_last_byte_r(int type, const void* data, size_t n, char last_byte, uint32_t* out) {
  return scalar_u32(1, 0, data, n, type, 1, last_byte, out);
}
int mck_xxh3_64_r(const void* data, size_t n, uint64_t* out) { return scalar_u64(0, data, n, 0, out); }
int mck_np_hash64_r(const void* data, size_t n, uint64_t seed, uint64_t* out) {
  return scalar_u64(1, data, n, seed, out);
}

// The signature-compatible shims.  The reference functions cannot fail, so
// an error is either fatal (default: a re-pointed call site must not store
// a wrong checksum) or 0 with mck_last_error() set (MCK_SHIM_ERRORS_ZERO,
// or SPEEDB_AMD_SHIM_ERRORS=zero).
namespace {
std::atomic<int> g_shim_policy{-1};  // -1: not read from the environment yet
std::atomic<mck_shim_error_handler> g_shim_handler{nullptr};
std::atomic<void*> g_shim_arg{nullptr};
int shim_policy() {
  int p = g_shim_policy.load(std::memory_order_acquire);
  if (p < 0) {
    const char* e = getenv("SPEEDB_AMD_SHIM_ERRORS");
    const int env = (e && (strcmp(e, "zero") == 0 || strcmp(e, "0") == 0)) ? MCK_SHIM_ERRORS_ZERO : MCK_SHIM_ERRORS_ABORT;
    int expected = -1;
    g_shim_policy.compare_exchange_strong(expected, env, std::memory_order_acq_rel);
    p = g_shim_policy.load(std::memory_order_acquire);
  }
  return p;
}
// the failure path of a plain shim: the handler, then abort or 0
void shim_error(int rc, const char* fn) {
  char msg[512];
  snprintf(msg, sizeof msg, "speedb_amd: %s failed (%d): %s", fn, rc, mck_last_error());
  if (mck_shim_error_handler h = g_shim_handler.load(std::memory_order_acquire))
    h(msg, g_shim_arg.load(std::memory_order_acquire));
  if (shim_policy() == MCK_SHIM_ERRORS_ABORT) {
    fprintf(stderr, "%s\n(the reference function has no error channel; use the *_r variant or "
                    "SPEEDB_AMD_SHIM_ERRORS=zero)\n", msg);
    fflush(stderr);
    abort();
  }
}
uint32_t shim_u32(int rc, uint32_t v, const char* fn) {
  if (rc == MCK_OK) return v;
  shim_error(rc, fn);
  return 0;
}
uint64_t shim_u64(int rc, uint64_t v, const char* fn) {
  if (rc == MCK_OK) return v;
  shim_error(rc, fn);
  return 0;
}
}  // namespace

int mck_set_shim_error_policy(int policy, mck_shim_error_handler handler, void* arg) {
  if (policy != MCK_SHIM_ERRORS_ABORT && policy != MCK_SHIM_ERRORS_ZERO) {
    set_err("unknown shim error policy %d", policy);
    return MCK_EINVAL;
  }
  const int prev = shim_policy();
  g_shim_arg.store(arg, std::memory_order_release);
  g_shim_handler.store(handler, std::memory_order_release);
  g_shim_policy.store(policy, std::memory_order_release);
  return prev;
}
uint32_t mck_crc32c_extend(uint32_t init_crc, const void* data, size_t n) {
  uint32_t v = 0;
  return shim_u32(mck_crc32c_extend_r(init_crc, data, n, &v), v, "mck_crc32c_extend");
}
uint32_t mck_crc32c_value(const void* data, size_t n) {
  uint32_t v = 0;
  return shim_u32(mck_crc32c_value_r(data, n, &v), v, "mck_crc32c_value");
}
uint32_t mck_builtin_checksum(int type, const void* data, size_t n) {
  uint32_t v = 0;
  return shim_u32(mck_builtin_checksum_r(type, data, n, &v), v, "mck_builtin_checksum");
}
uint32_t mck_builtin_checksum_with_last_byte(int type, const void* data, size_t n, char last_byte) {
  uint32_t v = 0;
  return shim_u32(mck_builtin_checksum_with_last_byte_r(type, data, n, last_byte, &v), v,
                     "mck_builtin_checksum_with_last_byte");
}
uint64_t mck_xxh3_64(const void* data, size_t n) {
  uint64_t v = 0;
  return shim_u64(mck_xxh3_64_r(data, n, &v), v, "mck_xxh3_64");
}
uint64_t mck_np_hash64(const void* data, size_t n, uint64_t seed) {
  uint64_t v = 0;
  return shim_u64(mck_np_hash64_r(data, n, seed, &v), v, "mck_np_hash64");
}
int mck_np_hash64_batch(const mck_spans* spans, uint64_t seed, uint64_t* out, mck_stream_t stream) {
  t_err[0] = 0;
  if (int rc = check_spans(spans)) return rc;
  stat_batch(spans->count, known_bytes(spans));
  if (spans->count && !out) {
    set_err("out is NULL");
    return MCK_EINVAL;
  }
  return launch_xph3(OpXpValue{to_src(spans), out}, spans->count, seed, reinterpret_cast<hipStream_t>(stream),
                     spans->lengths == nullptr && spans->length <= 240);
}

static int check_kv(int kind, const mck_spans* keys, const mck_spans* values, const uint64_t* extras) {
  if (int rc = check_spans(keys)) return rc;
  if (int rc = check_spans(values)) return rc;
  if (keys->count != values->count) {
    set_err("keys->count != values->count");
    return MCK_EINVAL;
  }
  if (kind < MCK_KV_PROTECT_KV || kind > MCK_KV_PROTECT_KVOC) {
    set_err("unknown protection kind %d", kind);
    return MCK_EINVAL;
  }
  if ((kind == MCK_KV_PROTECT_KVOS || kind == MCK_KV_PROTECT_KVOC) && values->count && !extras) {
    set_err("extras (seqnos / CF ids) are NULL");
    return MCK_EINVAL;
  }
  return MCK_OK;
}

int mck_kv_protect_batch(int kind, const mck_spans* keys, const mck_spans* values, const uint8_t* op_types,
                         const uint64_t* extras, uint64_t* out, mck_stream_t stream) {
  t_err[0] = 0;
  if (int rc = check_kv(kind, keys, values, extras)) return rc;
  if (values->count && !out) {
    set_err("out is NULL");
    return MCK_EINVAL;
  }
  const OpKvProtect<false> op{to_src(keys), to_src(values), op_types, extras, kind, out, nullptr, 0, nullptr, nullptr};
  return launch_xph3(op, values->count, kSeedV, reinterpret_cast<hipStream_t>(stream),
                     values->lengths == nullptr && values->length <= 240);
}

int mck_kv_protect_verify_batch(int kind, const mck_spans* keys, const mck_spans* values, const uint8_t* op_types,
                                const uint64_t* extras, const uint8_t* stored, uint32_t prot_bytes,
                                uint8_t* mismatch, uint32_t* mismatch_count, uint64_t* computed,
                                mck_stream_t stream) {
  t_err[0] = 0;
  if (int rc = check_kv(kind, keys, values, extras)) return rc;
  if (prot_bytes != 1 && prot_bytes != 2 && prot_bytes != 4 && prot_bytes != 8) {
    set_err("prot_bytes must be 1, 2, 4 or 8 (got %u)", prot_bytes);
    return MCK_EINVAL;
  }
  if (values->count && (!stored || !mismatch)) {
    set_err("stored/mismatch is NULL");
    return MCK_EINVAL;
  }
  const OpKvProtect<true> op{to_src(keys), to_src(values), op_types, extras, kind, computed, stored, prot_bytes,
                             mismatch, mismatch_count};
  return launch_xph3(op, values->count, kSeedV, reinterpret_cast<hipStream_t>(stream),
                     values->lengths == nullptr && values->length <= 240);
}

// ---- per-KV protection of block entries (block.cc:1091-1222) ---------------

uint64_t mck_block_kv_scratch_bytes(uint32_t count) { return 16 * blk_tiles(count) + 64; }

uint64_t mck_block_kv_work_bytes(uint64_t total_keys, uint64_t total_key_bytes) {
  return blk_work_head(total_keys) + total_key_bytes + 16;
}

int mck_block_kv_layout_batch(int kind, const mck_spans* blocks, uint64_t* key_base, uint64_t* arena_base,
                              uint32_t* restart_interval, int32_t* status, void* scratch, mck_stream_t stream) {
  t_err[0] = 0;
  if (int rc = check_spans(blocks)) return rc;
  if (!key_base || !arena_base || (blocks->count && (!status || !scratch || !restart_interval))) {
    set_err("key_base/arena_base/status/restart_interval/scratch is NULL");
    return MCK_EINVAL;
  }
  stat_batch(blocks->count, known_bytes(blocks));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const uint32_t n = blocks->count;
  if (!n) {
    MCK_HIP(hipMemsetAsync(key_base, 0, 8, st));
    MCK_HIP(hipMemsetAsync(arena_base, 0, 8, st));
    return MCK_OK;
  }
  if (int rc = launch_blk<BlkLayoutT>(kind, n, st, to_src(blocks), n, key_base, arena_base, restart_interval, status))
    return rc;
  const uint32_t tiles = (uint32_t)blk_tiles(n);
  uint64_t* tsum = static_cast<uint64_t*>(scratch);
  hipLaunchKernelGGL(k_blk_scan_tiles, dim3(tiles), dim3(kBlkScanThreads), 0, st, key_base, arena_base, n, tsum);
  hipLaunchKernelGGL(k_blk_scan_top, dim3(1), dim3(kBlkScanThreads), 0, st, tsum, tiles, key_base, arena_base, n);
  hipLaunchKernelGGL(k_blk_scan_apply, dim3(tiles), dim3(kBlkScanThreads), 0, st, key_base, arena_base, n, tsum);
  MCK_HIP(hipGetLastError());
  return MCK_OK;
}

int mck_block_kv_protect_batch(int kind, const mck_spans* blocks, uint32_t prot_bytes, const uint64_t* key_base,
                               const uint64_t* arena_base, const uint32_t* restart_interval, uint64_t total_keys,
                               void* work, uint8_t* out, mck_stream_t stream) {
  t_err[0] = 0;
  if (total_keys && !out) {
    set_err("out is NULL");
    return MCK_EINVAL;
  }
  return blk_kv(kind, blocks, prot_bytes, key_base, arena_base, restart_interval, total_keys, work, out, nullptr,
                nullptr, nullptr, reinterpret_cast<hipStream_t>(stream));
}

int mck_block_kv_verify_batch(int kind, const mck_spans* blocks, uint32_t prot_bytes, const uint64_t* key_base,
                              const uint64_t* arena_base, const uint32_t* restart_interval, uint64_t total_keys,
                              void* work, const uint8_t* stored, uint8_t* mismatch, uint32_t* mismatch_count,
                              mck_stream_t stream) {
  t_err[0] = 0;
  if (total_keys && (!stored || !mismatch)) {
    set_err("stored/mismatch is NULL");
    return MCK_EINVAL;
  }
  return blk_kv(kind, blocks, prot_bytes, key_base, arena_base, restart_interval, total_keys, work, nullptr, stored,
                mismatch, mismatch_count, reinterpret_cast<hipStream_t>(stream));
}

uint64_t mck_block_kv_blocks_work_bytes(uint32_t count, uint32_t slot_cap, uint32_t arena_cap) {
  return blk_blocks_work(nullptr, count, slot_cap, arena_cap).bytes;
}

int mck_block_kv_protect_blocks_batch(int kind, const mck_spans* blocks, uint32_t prot_bytes, uint32_t slot_cap,
                                      uint32_t arena_cap, uint64_t* key_base, uint64_t* arena_base,
                                      uint32_t* restart_interval, int32_t* status, void* work, uint8_t* out,
                                      mck_stream_t stream) {
  t_err[0] = 0;
  return blk_kv_blocks(kind, blocks, prot_bytes, slot_cap, arena_cap, key_base, arena_base, nullptr, 0,
                       restart_interval, status, work, out, nullptr, nullptr, nullptr,
                       reinterpret_cast<hipStream_t>(stream));
}

int mck_block_kv_verify_blocks_batch(int kind, const mck_spans* blocks, uint32_t prot_bytes, uint32_t slot_cap,
                                     uint32_t arena_cap, const uint64_t* key_base, uint64_t total_keys,
                                     uint32_t* restart_interval, int32_t* status, void* work, const uint8_t* stored,
                                     uint8_t* mismatch, uint32_t* mismatch_count, mck_stream_t stream) {
  t_err[0] = 0;
  if (!stored) {
    set_err("stored is NULL");
    return MCK_EINVAL;
  }
  return blk_kv_blocks(kind, blocks, prot_bytes, slot_cap, arena_cap, nullptr, nullptr, key_base, total_keys,
                       restart_interval, status, work, nullptr, stored, mismatch, mismatch_count,
                       reinterpret_cast<hipStream_t>(stream));
}

// Internal test hook (not part of mck.h): XXPH3 of one device span by the
// block kernels' wave-cooperative long loop, the per-lane loop, and the wave
// loop over an LDS-staged copy: out[0..2]; out[3 + k] = the row-cooperative
// loop (xp_row_long) over the first len - 61 k bytes, k = 0..3.
int mck_internal_xp_wave(const void* data, uint32_t len, uint64_t seed, uint64_t* out, mck_stream_t stream) {
  if (int rc = current_device(nullptr, nullptr)) return rc;
  hipLaunchKernelGGL(k_dbg_xp, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
                     static_cast<const uint8_t*>(data), len, seed, out);
  MCK_HIP(hipGetLastError());
  return MCK_OK;
}

// ---- partitioning + host-resident multi-GPU pipeline -----------------------
int mck_partition_spans(const uint32_t* host_lengths, uint32_t count, uint32_t length, int parts, uint32_t* first) {
  t_err[0] = 0;
  if (parts <= 0 || !first) {
    set_err("bad parts/first");
    return MCK_EINVAL;
  }
  uint64_t total = 0;
  for (uint32_t i = 0; i < count; i++) total += host_lengths ? host_lengths[i] : length;
  first[0] = 0;
  uint64_t acc = 0;
  uint32_t i = 0;
  for (int p = 1; p < parts; p++) {
    const uint64_t target = (total * (uint64_t)p + parts / 2) / (uint64_t)parts;
    while (i < count && acc + (host_lengths ? host_lengths[i] : length) / 2 < target) {
      acc += host_lengths ? host_lengths[i] : length;
      i++;
    }
    first[p] = i;
  }
  first[parts] = count;
  return MCK_OK;
}

namespace {

struct HostJob {
  int kind;
  const uint8_t* base;
  const uint64_t* offs;
  const uint32_t* lens;
  uint64_t stride;
  uint32_t length;
  uint32_t flags;
  size_t chunk_bytes;
  uint32_t* out32;
  uint64_t* out64;
  uint64_t off(uint32_t i) const { return offs ? offs[i] : (uint64_t)i * stride; }
  uint32_t len(uint32_t i) const { return lens ? lens[i] : length; }
};

// Per-device staging of the host-resident pipeline, allocated on first use
// and reused by every later call (grown when a call needs more): kHostSlots
// slots, each a stream + device chunk/descriptor/result buffers + pinned
// descriptor/result buffers.  One call at a time per device (the mutex);
// mck_host_pipeline_release() frees it.
constexpr int kHostSlots = 2;
struct HostSlot {
  hipStream_t st = nullptr;
  uint8_t* d_data = nullptr;
  uint64_t* d_off = nullptr;
  uint32_t* d_len = nullptr;
  uint64_t* d_res = nullptr;
  uint64_t* h_off = nullptr;
  uint32_t* h_len = nullptr;
  uint64_t* h_res = nullptr;
  uint32_t first = 0, n = 0;  // spans of the chunk in flight
};
struct HostPipe {
  std::mutex mu;
  size_t cap = 0;          // chunk bytes per slot
  uint32_t max_spans = 0;  // descriptor/result entries per slot
  int dev = -1;            // device the buffers and streams were built on
  HostSlot slot[kHostSlots];
};
static HostPipe g_host[kMaxDev];

// Free every buffer of a pipeline (caller holds its mutex, device is current).
static void host_pipe_free(HostPipe& p) {
  for (HostSlot& s : p.slot) {
    if (s.st) (void)hipStreamSynchronize(s.st);
    if (s.st) (void)hipStreamDestroy(s.st);
    if (s.d_data) (void)hipFree(s.d_data);
    if (s.d_off) (void)hipFree(s.d_off);
    if (s.d_len) (void)hipFree(s.d_len);
    if (s.d_res) (void)hipFree(s.d_res);
    if (s.h_off) (void)hipHostFree(s.h_off);
    if (s.h_len) (void)hipHostFree(s.h_len);
    if (s.h_res) (void)hipHostFree(s.h_res);
    s = HostSlot{};
  }
  p.cap = 0;
  p.max_spans = 0;
  p.dev = -1;
}

// Make the pipeline hold at least cap chunk bytes and max_spans entries per
// slot.  On failure everything is freed (no partial state survives).
static int host_pipe_reserve(HostPipe& p, int dev, size_t cap, uint32_t max_spans) {
  if (p.dev == dev && p.cap >= cap && p.max_spans >= max_spans && p.slot[0].st) return MCK_OK;
  cap = std::max(cap, p.cap);
  max_spans = std::max(max_spans, p.max_spans);
  if (p.dev >= 0 && p.dev != dev) {
    // a pipe built on another device (the virtual-devices hook maps pipe
    // indices to device 0) is freed on that device, then rebuilt on dev
    (void)hipSetDevice(p.dev);
    host_pipe_free(p);
    (void)hipSetDevice(dev);
  }
  host_pipe_free(p);
  p.dev = dev;
  hipError_t e = hipSuccess;
  const char* what = "";
  auto ok = [&](hipError_t r, const char* w) {
    if (r != hipSuccess && e == hipSuccess) {
      e = r;
      what = w;
    }
    return e == hipSuccess;
  };
  for (HostSlot& s : p.slot) {
    if (!ok(hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking), "hipStreamCreate") ||
        !ok(hipMalloc(&s.d_data, cap + 64), "hipMalloc(chunk)") ||
        !ok(hipMalloc(&s.d_off, (size_t)max_spans * 8), "hipMalloc(offsets)") ||
        !ok(hipMalloc(&s.d_len, (size_t)max_spans * 4), "hipMalloc(lengths)") ||
        !ok(hipMalloc(&s.d_res, (size_t)max_spans * 8), "hipMalloc(results)") ||
        !ok(hipHostMalloc(&s.h_off, (size_t)max_spans * 8, hipHostMallocDefault), "hipHostMalloc(offsets)") ||
        !ok(hipHostMalloc(&s.h_len, (size_t)max_spans * 4, hipHostMallocDefault), "hipHostMalloc(lengths)") ||
        !ok(hipHostMalloc(&s.h_res, (size_t)max_spans * 8, hipHostMallocDefault), "hipHostMalloc(results)"))
      break;
  }
  if (e != hipSuccess) {
    host_pipe_free(p);
    set_err("%s failed: %s (chunk %zu B, %u spans per slot)", what, hipGetErrorString(e), cap, max_spans);
    return e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation ? MCK_ENOMEM : MCK_EHIP;
  }
  p.cap = cap;
  p.max_spans = max_spans;
  return MCK_OK;
}

// One device's share [lo, hi) of a host batch (spans sorted by offset):
// chunks of spans are staged through the slots round-robin, each on its own
// stream, so the H2D copy of one chunk overlaps the kernel of the previous
// one; results come back D2H into pinned memory and are copied out when the
// slot is reused.  Every exit path leaves no copy in flight.
// `pipe` picks the staging (g_host[pipe]); it is the device itself, except
// under mck_test_set_virtual_devices, where pipes 0..k-1 all run on device 0.
static int run_device_share(int dev, int pipe, const HostJob& J, uint32_t lo, uint32_t hi) {
  NoStat nostat;
  MCK_HIP(hipSetDevice(dev));
  if (lo >= hi) return MCK_OK;
  int rc = current_device(nullptr, nullptr);
  if (rc) return rc;
  // the longest span bounds the chunk
  size_t cap = J.chunk_bytes;
  for (uint32_t i = lo; i < hi; i++) cap = std::max<size_t>(cap, (size_t)J.len(i) + 32);
  const uint32_t max_spans = (uint32_t)std::min<uint64_t>(hi - lo, 1u << 20);
  HostPipe& P = g_host[pipe];
  std::lock_guard<std::mutex> lock(P.mu);
  if ((rc = host_pipe_reserve(P, dev, cap, max_spans))) return rc;
  const size_t res_sz = J.kind == MCK_kXXH3 ? 8 : 4;
  auto drain = [&](HostSlot& s) -> int {
    if (!s.n) return MCK_OK;
    const hipError_t e = hipStreamSynchronize(s.st);
    const uint32_t first = s.first, n = s.n;
    s.n = 0;
    if (e != hipSuccess) {
      set_err("hipStreamSynchronize failed: %s", hipGetErrorString(e));
      return MCK_EHIP;
    }
    if (J.kind == MCK_kXXH3)
      memcpy(J.out64 + first, s.h_res, (size_t)n * 8);
    else
      memcpy(J.out32 + first, s.h_res, (size_t)n * 4);
    return MCK_OK;
  };
  auto quiesce = [&] {  // error exit: wait for every slot, keep the first error
    for (HostSlot& s : P.slot) {
      if (s.st) (void)hipStreamSynchronize(s.st);
      s.n = 0;
    }
  };
  auto issue = [&](HostSlot& s, uint32_t i, uint32_t j, uint64_t start, uint64_t endb) -> int {
    MCK_HIP(hipMemcpyAsync(s.d_data, J.base + start, endb - start, hipMemcpyHostToDevice, s.st));
    MCK_HIP(hipMemcpyAsync(s.d_off, s.h_off, (size_t)(j - i) * 8, hipMemcpyHostToDevice, s.st));
    MCK_HIP(hipMemcpyAsync(s.d_len, s.h_len, (size_t)(j - i) * 4, hipMemcpyHostToDevice, s.st));
    const mck_spans sp{s.d_data, s.d_off, s.d_len, 0, 0, j - i};
    const int r = J.kind == MCK_kXXH3
                      ? mck_xxh3_64_batch(&sp, s.d_res, reinterpret_cast<mck_stream_t>(s.st))
                      : mck_crc32c_batch(&sp, nullptr, J.flags, reinterpret_cast<uint32_t*>(s.d_res),
                                         reinterpret_cast<mck_stream_t>(s.st));
    if (r) return r;
    MCK_HIP(hipMemcpyAsync(s.h_res, s.d_res, (size_t)(j - i) * res_sz, hipMemcpyDeviceToHost, s.st));
    return MCK_OK;
  };
  uint32_t i = lo;
  for (int k = 0; i < hi; k++) {
    HostSlot& s = P.slot[k % kHostSlots];
    if ((rc = drain(s))) break;
    // spans [i, j) whose covering byte range fits the chunk
    const uint64_t start = J.off(i);
    uint32_t j = i;
    uint64_t endb = start;
    while (j < hi && j - i < P.max_spans) {
      const uint64_t e = J.off(j) + J.len(j);
      if (j > i && std::max(endb, e) - start > P.cap) break;
      endb = std::max(endb, e);
      s.h_off[j - i] = J.off(j) - start;
      s.h_len[j - i] = J.len(j);
      j++;
    }
    s.first = i;
    s.n = j - i;
    if ((rc = issue(s, i, j, start, endb))) break;
    i = j;
  }
  if (rc) {
    quiesce();
    return rc;
  }
  for (HostSlot& s : P.slot)
    if ((rc = drain(s))) {
      quiesce();
      return rc;
    }
  return MCK_OK;
}

// Test hook (mck_test_set_virtual_devices): k > 0 makes mck_host_batch_checksum
// see k devices, all of them device 0, each with its own staging, streams and
// host thread -- the ndev > 1 branch on a one-GPU box.
std::atomic<int> g_virtual_devs{0};

}  // namespace

int mck_host_batch_checksum(int kind, const void* host_base, const uint64_t* host_offsets,
                            const uint32_t* host_lengths, uint64_t stride, uint32_t length, uint32_t count,
                            uint32_t flags, int ndev, size_t chunk_bytes, uint32_t* out32, uint64_t* out64,
                            double* seconds) {
  t_err[0] = 0;
  const auto t0 = std::chrono::steady_clock::now();
  if (kind != MCK_kCRC32c && kind != MCK_kXXH3) {
    set_err("kind must be MCK_kCRC32c or MCK_kXXH3");
    return MCK_EINVAL;
  }
  if (count && (!host_base || (kind == MCK_kCRC32c ? !out32 : !out64))) {
    set_err("NULL base/out");
    return MCK_EINVAL;
  }
  int have = 0;
  if (hipGetDeviceCount(&have) != hipSuccess || have <= 0) {
    set_err("no HIP device");
    return MCK_ENODEV;
  }
  const int virt = g_virtual_devs.load(std::memory_order_relaxed);
  if (virt > 0) have = virt;
  int prev = 0;
  (void)hipGetDevice(&prev);
  // ndev <= 0: only the calling thread's current device (one process per
  // GPU); otherwise devices [0, ndev)
  std::vector<int> devs;
  if (ndev <= 0) {
    devs.push_back(prev);
  } else {
    // asking for more devices than the process sees is an error, never a
    // silent clamp (a caller that believes it spreads over 8 GPUs must not
    // time 1)
    if (ndev > have || ndev > kMaxDev) {
      set_err("ndev = %d devices asked for, %d present", ndev, have);
      return MCK_ENODEV;
    }
    for (int d = 0; d < ndev; d++) devs.push_back(d);
  }
  ndev = (int)devs.size();
  if (!chunk_bytes) chunk_bytes = 256u << 20;
  for (uint32_t i = 1; host_offsets && i < count; i++)
    if (host_offsets[i] < host_offsets[i - 1]) {
      set_err("host_offsets must be non-decreasing");
      return MCK_EINVAL;
    }
  std::vector<uint32_t> first(ndev + 1);
  mck_partition_spans(host_lengths, count, length, ndev, first.data());
  HostJob J{kind, static_cast<const uint8_t*>(host_base), host_offsets, host_lengths, stride, length,
            flags & MCK_F_MASK, chunk_bytes, out32, out64};
  std::vector<int> rcs(ndev, 0);
  std::vector<std::string> errs(ndev);
  // (virtual devices: pipe d on device 0; ndev <= 0 keeps the caller's device)
  const auto phys = [&](int d) { return virt > 0 && ndev > 1 ? 0 : devs[d]; };
  const auto pipe = [&](int d) { return virt > 0 && ndev > 1 ? d : devs[d]; };
  if (ndev == 1) {
    rcs[0] = run_device_share(phys(0), pipe(0), J, first[0], first[1]);
    if (rcs[0]) errs[0] = t_err;
  } else {
    std::vector<std::thread> th;
    for (int d = 0; d < ndev; d++)
      th.emplace_back([&, d] {
        rcs[d] = run_device_share(phys(d), pipe(d), J, first[d], first[d + 1]);
        if (rcs[d]) errs[d] = t_err;
      });
    for (auto& t : th) t.join();
  }
  (void)hipSetDevice(prev);
  for (int d = 0; d < ndev; d++)
    if (rcs[d]) {
      set_err("device %d: %s", devs[d], errs[d].c_str());
      return rcs[d];
    }
  uint64_t bytes = 0;
  for (uint32_t i = 0; i < count; i++) bytes += host_lengths ? host_lengths[i] : length;
  stat_batch(count, bytes);
  if (seconds) *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return MCK_OK;
}

int mck_statistics_get(mck_statistics* out, int reset) {
  t_err[0] = 0;
  if (!out) {
    set_err("out is NULL");
    return MCK_EINVAL;
  }
  memset(out, 0, sizeof *out);
  const auto take = [&](std::atomic<uint64_t>& c) { return reset ? c.exchange(0) : c.load(); };
  out->block_checksum_compute_count = take(g_stats.compute);
  out->batches = take(g_stats.batches);
  out->spans = take(g_stats.spans);
  out->bytes_known = take(g_stats.bytes);
  int prev = 0;
  (void)hipGetDevice(&prev);
  int rc = MCK_OK;
  for (int d = 0; d < kMaxDev; d++) {
    if (!g_dev[d].d_stats) continue;
    unsigned long long c = 0;
    bool ok = hipSetDevice(d) == hipSuccess;
    if (ok) {
      hipLaunchKernelGGL(k_stats_take, dim3(1), dim3(64), 0, 0, g_dev[d].d_stats, g_dev[d].d_stats + 1, reset);
      ok = hipGetLastError() == hipSuccess &&
           hipMemcpy(&c, g_dev[d].d_stats + 1, sizeof c, hipMemcpyDeviceToHost) == hipSuccess;
    }
    if (!ok) {
      set_err("reading the device counters of device %d failed", d);
      rc = MCK_EHIP;
      continue;
    }
    out->block_checksum_mismatch_count += c;
  }
  (void)hipSetDevice(prev);
  return rc;
}

int mck_set_perf_level(int level) {
  t_err[0] = 0;
  if (level < MCK_PERF_kDisable || level > MCK_PERF_kEnableTime) {
    set_err("perf level must be %d..%d", MCK_PERF_kDisable, MCK_PERF_kEnableTime);
    return MCK_EINVAL;
  }
  t_perf.level = level;
  return MCK_OK;
}

int mck_get_perf_level(void) { return t_perf.level; }

int mck_perf_context_get(mck_perf_context* out, int reset) {
  t_err[0] = 0;
  if (!out) {
    set_err("out is NULL");
    return MCK_EINVAL;
  }
  int rc = MCK_OK;
  for (const PerfPending& p : t_perf.pending) {
    float ms = 0.f;
    if (hipEventSynchronize(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
      t_perf.time_ns += (uint64_t)((double)ms * 1e6);
    } else if (rc == MCK_OK) {
      set_err("timing a verify batch failed");
      rc = MCK_EHIP;
    }
    t_perf.pool.push_back({p.dev, p.a});
    t_perf.pool.push_back({p.dev, p.b});
  }
  t_perf.pending.clear();
  out->block_checksum_time = t_perf.time_ns;
  out->block_checksum_count = t_perf.count;
  out->block_checksum_batches = t_perf.batches;
  if (reset) t_perf.time_ns = t_perf.count = t_perf.batches = 0;
  return rc;
}

int mck_test_set_xxh3_driver(int driver) {
  t_err[0] = 0;
  if (driver < 0 || driver > 2) {
    set_err("driver must be 0 (by batch shape), 1 (wave per span) or 2 (16-lane rows)");
    return MCK_EINVAL;
  }
  g_x3_force.store(driver, std::memory_order_relaxed);
  return MCK_OK;
}

int mck_test_set_crc_driver(int driver, int interleaved) {
  t_err[0] = 0;
  // 1 (the 4 KiB-round wave driver) and 4 (the unit stream) were retired
  // in round 4 by the body/head driver (7); 9 = the small-batch wave-per-span
  // path wherever it applies
  if (driver < 0 || driver > 9 || driver == 1 || driver == 4 || driver == 8) {
    set_err("driver must be 0, 2, 3, 5, 6, 7 or 9");
    return MCK_EINVAL;
  }
  g_crc_force.store(driver, std::memory_order_relaxed);
  g_crc_interleaved.store(interleaved ? 1 : 0, std::memory_order_relaxed);
  return MCK_OK;
}

void mck_host_pipeline_release(void) {
  int prev = 0;
  (void)hipGetDevice(&prev);
  for (int d = 0; d < kMaxDev; d++) {
    HostPipe& P = g_host[d];
    std::lock_guard<std::mutex> lock(P.mu);
    if (!P.slot[0].st && !P.cap) continue;
    // each pipe is freed on the device it was built on (pipes of virtual
    // devices live on device 0, a caller's own device's pipe on that device)
    if (P.dev < 0 || hipSetDevice(P.dev) != hipSuccess) continue;
    host_pipe_free(P);
  }
  (void)hipSetDevice(prev);
}

int mck_test_set_xph3_quads(int on) {
  g_xph3_quads.store(on ? 1 : 0, std::memory_order_relaxed);
  return MCK_OK;
}

int mck_test_set_virtual_devices(int k) {
  t_err[0] = 0;
  if (k < 0 || k > kMaxDev) {
    set_err("virtual devices must be 0..%d", kMaxDev);
    return MCK_EINVAL;
  }
  // pipes built for real devices must not be reused under the other mapping
  mck_host_pipeline_release();
  g_virtual_devs.store(k, std::memory_order_relaxed);
  return MCK_OK;
}

}  // extern "C"
