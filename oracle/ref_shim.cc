// ref_shim.cc -- C-ABI wrapper over the REFERENCE's own checksum primitives.
//
// TEST INFRASTRUCTURE ONLY.  oracle/Makefile compiles this file together with
// the reference's util/crc32c.cc, util/xxhash.cc and util/hash.cc (and the
// header-only db/kv_checksum.h), read in place from
// /root/reference, into oracle/_ref/libspdb_ref.so (git-ignored).  Nothing is
// copied into this repository.  It is used (a) to pin oracle.c, (b) to make
// the golden fixtures under tests/golden/, and (c) as bench.py's
// "reference" cpu_baseline on the GPU box's host cores.
//
// ChecksumModifierForContext is called from the reference's own header
// (table/format.h, inline; its includes compile header-only).
// The block-checksum dispatch (table/format.cc:578-645) lives in a file that
// drags in the whole table layer, so it is restated here over the reference's
// own crc32c:: and XXH* primitives; the WAL record CRC likewise restates
// db/log_writer.cc:263-311 over crc32c::Value/Extend/Crc32cCombine/Mask.
#include <pthread.h>
#include <stdint.h>
#include <string.h>
#include <time.h>

#include <string>
#include <vector>

#include "db/kv_checksum.h"
#include "table/format.h"
#include "util/crc32c.h"
#include "util/hash.h"
#include "util/xxhash.h"

namespace c = ROCKSDB_NAMESPACE::crc32c;

extern "C" {

uint32_t ref_crc32c_extend(uint32_t init, const void* p, size_t n) {
  return c::Extend(init, static_cast<const char*>(p), n);
}
uint32_t ref_crc32c_value(const void* p, size_t n) {
  return c::Value(static_cast<const char*>(p), n);
}
uint32_t ref_crc32c_mask(uint32_t v) { return c::Mask(v); }
uint32_t ref_crc32c_unmask(uint32_t v) { return c::Unmask(v); }
uint32_t ref_crc32c_combine(uint32_t a, uint32_t b, size_t blen) {
  return c::Crc32cCombine(a, b, blen);
}
uint64_t ref_xxh3_64(const void* p, size_t n) { return XXH3_64bits(p, n); }
uint32_t ref_xxh32(const void* p, size_t n, uint32_t seed) {
  return XXH32(p, n, seed);
}
uint64_t ref_xxh64(const void* p, size_t n, uint64_t seed) {
  return XXH64(p, n, seed);
}

// util/hash.cc:81-88 Hash64 (= NPHash64, util/hash.h:45-64) -> XXPH3.
uint64_t ref_hash64(const void* p, size_t n, uint64_t seed) {
  return ROCKSDB_NAMESPACE::Hash64(static_cast<const char*>(p), n, seed);
}

// db/kv_checksum.h, the reference's own templates, read back through the
// public Encode(8, ...):  mode 0 ProtectKV(key, value); 1 ProtectKVO(key,
// value, op); 2 ProtectKVO(...).ProtectS(seq = extra); 3 ProtectKVO(...)
// .ProtectC(cf = (uint32)extra).
uint64_t ref_kv_protect(int mode, const void* key, size_t kn, const void* value,
                        size_t vn, uint8_t op, uint64_t extra) {
  namespace R = ROCKSDB_NAMESPACE;
  const R::Slice k(static_cast<const char*>(key), kn);
  const R::Slice v(static_cast<const char*>(value), vn);
  const R::ValueType t = static_cast<R::ValueType>(op);
  char buf[8];
  switch (mode) {
    case 0:
      R::ProtectionInfo64().ProtectKV(k, v).Encode(8, buf);
      break;
    case 1:
      R::ProtectionInfo64().ProtectKVO(k, v, t).Encode(8, buf);
      break;
    case 2:
      R::ProtectionInfo64().ProtectKVO(k, v, t).ProtectS(extra).Encode(8, buf);
      break;
    default:
      R::ProtectionInfo64()
          .ProtectKVO(k, v, t)
          .ProtectC(static_cast<uint32_t>(extra))
          .Encode(8, buf);
      break;
  }
  uint64_t r;
  memcpy(&r, buf, 8);  // EncodeFixed64 is little-endian
  return r;
}

// table/format.h:119-146, the reference's own inline function.
uint32_t ref_context_modifier(uint32_t base_context_checksum, uint64_t offset) {
  return ROCKSDB_NAMESPACE::ChecksumModifierForContext(base_context_checksum, offset);
}

// table/format.cc:578-602 over the reference primitives.
uint32_t ref_builtin_checksum(int type, const void* data, size_t n) {
  const char* p = static_cast<const char*>(data);
  switch (type) {
    case 1:
      return c::Mask(c::Value(p, n));
    case 2:
      return XXH32(p, n, 0);
    case 3:
      return static_cast<uint32_t>(XXH64(p, n, 0));
    case 4:
      if (n == 0) return 0;
      return static_cast<uint32_t>(XXH3_64bits(p, n - 1)) ^
             static_cast<uint8_t>(p[n - 1]) * 0x6b9083d9u;
    default:
      return 0;
  }
}

// db/log_writer.cc:263-311 over the reference primitives.
uint32_t ref_wal_record_crc(uint8_t type, const void* payload, size_t n,
                            int recyclable, uint32_t log_number) {
  char t = static_cast<char>(type);
  uint32_t crc = c::Value(&t, 1);
  if (recyclable) {
    char ln[4];
    memcpy(ln, &log_number, 4);  // little-endian host (x86)
    crc = c::Extend(crc, ln, 4);
  }
  crc = c::Crc32cCombine(crc, c::Value(static_cast<const char*>(payload), n), n);
  return c::Mask(crc);
}

// ---------------------------------------------------------------------------
// CPU baseline harness.  Mirrors tools/db_bench_tool.cc:4392-4412
// (ChecksumBenchmark): every thread hashes one block at a time, one call per
// block, `kind` 0 = crc32c::Value, 1 = XXH3_64bits.
//   mode 0 ("db_bench", cache-hot): the same std::string(block,'x') buffer
//          over and over until bytes_per_thread;
//   mode 1 (DRAM-resident): distinct blocks of `buf` (caller-filled, len
//          nblocks*block), statically strided across threads, for
//          `passes` passes.
// Returns total bytes hashed; *seconds gets the wall time of the parallel
// region (all threads started before the clock).
// ---------------------------------------------------------------------------
struct BenchArg {
  int kind, mode;
  size_t block;
  uint64_t bytes_per_thread;
  const char* buf;
  uint64_t nblocks, tid, nthreads, passes;
  uint64_t bytes;
  uint32_t sink;
  pthread_barrier_t* bar;
};

static void* bench_thread(void* p) {
  BenchArg* a = static_cast<BenchArg*>(p);
  uint32_t val = 0;
  uint64_t bytes = 0;
  pthread_barrier_wait(a->bar);
  if (a->mode == 0) {
    std::string data(a->block, 'x');
    while (bytes < a->bytes_per_thread) {
      val += a->kind == 0 ? c::Value(data.data(), a->block)
                          : static_cast<uint32_t>(XXH3_64bits(data.data(), a->block));
      bytes += a->block;
    }
  } else {
    for (uint64_t pass = 0; pass < a->passes; pass++)
      for (uint64_t b = a->tid; b < a->nblocks; b += a->nthreads) {
        const char* blk = a->buf + b * a->block;
        val += a->kind == 0 ? c::Value(blk, a->block)
                            : static_cast<uint32_t>(XXH3_64bits(blk, a->block));
        bytes += a->block;
      }
  }
  a->bytes = bytes;
  a->sink = val;
  pthread_barrier_wait(a->bar);
  return nullptr;
}

uint64_t ref_bench(int kind, int mode, int nthreads, size_t block,
                   uint64_t bytes_per_thread, const void* buf,
                   uint64_t nblocks, uint64_t passes, double* seconds,
                   uint32_t* sink) {
  std::vector<pthread_t> th(nthreads);
  std::vector<BenchArg> args(nthreads);
  pthread_barrier_t bar;
  pthread_barrier_init(&bar, nullptr, nthreads + 1);
  for (int i = 0; i < nthreads; i++) {
    args[i] = BenchArg{kind, mode, block, bytes_per_thread,
                       static_cast<const char*>(buf), nblocks,
                       static_cast<uint64_t>(i), static_cast<uint64_t>(nthreads),
                       passes, 0, 0, &bar};
    pthread_create(&th[i], nullptr, bench_thread, &args[i]);
  }
  timespec t0, t1;
  pthread_barrier_wait(&bar);
  clock_gettime(CLOCK_MONOTONIC, &t0);
  pthread_barrier_wait(&bar);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  uint64_t total = 0;
  uint32_t s = 0;
  for (int i = 0; i < nthreads; i++) {
    pthread_join(th[i], nullptr);
    total += args[i].bytes;
    s += args[i].sink;
  }
  pthread_barrier_destroy(&bar);
  *seconds = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
  if (sink) *sink = s;
  return total;
}

}  // extern "C"
