// mck_walrec.cc -- mck_wal_recover: WAL recovery with the record checksums,
// the checksum work in ONE device pass (mck_wal_recover_batch,
// mck_walrec.hpp), the reader's walk on the host (mck_walk.h).
#include <hip/hip_runtime_api.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <memory>
#include <new>
#include <thread>
#include <vector>

#include "../../include/speedb_amd/mck.h"
#include "mck_internal.h"
#include "mck_walk.h"

using namespace mck_walk;

// ---------------------------------------------------------------------------
// WAL recovery with the record checksums (db/db_impl/db_impl_open.cc:1204-1221:
// ReadRecord(&record, &scratch, mode, &record_checksum) until false), the
// checksum work in ONE device pass over the image:
//   1. plan: the host walk trusting every CRC, counting the full-type records
//      of every block -> dense slots (prefix sum) and the multi-fragment
//      records;
//   2. device: mck_wal_recover_batch (every physical record's CRC32C + the
//      XXH3 of every full-type record in place, into its slot) and, on the same
//      stream, mck_wal_gather_batch + mck_xxh3_64_batch for the multi-fragment
//      records only; one readback;
//   3. if a CRC failed (a block stopped with MCK_WAL_BAD_CHECKSUM), the walk
//      again over the verdicts (records, drops and reports as the reference's
//      reader sees them), and its multi-fragment records hashed again.
// Without a failure the plan IS the reader's walk: the verdicts only change
// the walk where a checksum fails.
// ---------------------------------------------------------------------------
struct mck_wal_recovery {
  WalWalk W;
  std::vector<uint64_t> checksums;
  std::vector<mck_wal_block_result> blocks;  // the device's per-block verdicts
  mck_wal_recovery_info info{};
};

namespace {
double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Device scratch of one recover call (one allocation, freed in order on the
// stream).
struct DevArena {
  hipStream_t st;
  char* base = nullptr;
  size_t used = 0, cap = 0;
  ~DevArena() {
    if (base) (void)hipFreeAsync(base, st);
  }
  int reserve(size_t bytes) {
    cap = bytes ? bytes : 16;
    if (hipMallocAsync(reinterpret_cast<void**>(&base), cap, st) != hipSuccess) {
      base = nullptr;
      mck_internal_set_error("hipMallocAsync failed (recover scratch)");
      return MCK_ENOMEM;
    }
    return MCK_OK;
  }
  template <class T>
  T* take(size_t n) {  // 256-byte aligned pieces (the gather output needs 16)
    T* p = reinterpret_cast<T*>(base + used);
    used += (n * sizeof(T) + 255) & ~size_t(255);
    return p;
  }
  static size_t need(size_t n, size_t sz) { return (n * sz + 255) & ~size_t(255); }
};

// The multi-fragment records of a walk: their fragments re-based into one
// contiguous gather buffer, and each record's (offset, length) in it.
struct MultiPlan {
  std::vector<size_t> recs;  // record indices in the walk
  std::vector<mck_wal_fragment> frags;
  std::vector<uint64_t> offs;
  std::vector<uint32_t> lens;
  uint64_t bytes = 0;
};
MultiPlan multi_plan(const WalWalk& W) {
  MultiPlan M;
  for (size_t r = 0; r < W.roff.size(); r++) {
    if (W.rhoff[r] != ~0ull) continue;  // one fragment: hashed in place
    M.recs.push_back(r);
    M.offs.push_back(M.bytes);
    M.lens.push_back(W.rlen[r]);
    for (uint64_t j = W.rfrag[r]; j < W.rfrag[r + 1]; j++) {
      mck_wal_fragment f = W.fr[j];
      f.dst_off = M.bytes + (f.dst_off - W.roff[r]);
      M.frags.push_back(f);
    }
    M.bytes += (W.rlen[r] + 15) & ~uint64_t(15);  // 16-aligned records
  }
  return M;
}

// Launch the gather + XXH3 of a multi plan on the stream (results at d_out).
int launch_multi(const void* wal_dev, const MultiPlan& M, DevArena& A, uint64_t** d_out, hipStream_t st) {
  *d_out = nullptr;
  if (M.recs.empty()) return MCK_OK;
  mck_wal_fragment* d_fr = A.take<mck_wal_fragment>(M.frags.size());
  uint64_t* d_offs = A.take<uint64_t>(M.offs.size());
  uint32_t* d_lens = A.take<uint32_t>(M.lens.size());
  uint8_t* d_buf = A.take<uint8_t>(M.bytes + 64);
  *d_out = A.take<uint64_t>(M.recs.size());
  if (hipMemcpyAsync(d_fr, M.frags.data(), M.frags.size() * sizeof(mck_wal_fragment), hipMemcpyHostToDevice, st) ||
      hipMemcpyAsync(d_offs, M.offs.data(), M.offs.size() * 8, hipMemcpyHostToDevice, st) ||
      hipMemcpyAsync(d_lens, M.lens.data(), M.lens.size() * 4, hipMemcpyHostToDevice, st)) {
    mck_internal_set_error("hipMemcpyAsync failed (multi-fragment plan)");
    return MCK_EHIP;
  }
  mck_stream_t s = reinterpret_cast<mck_stream_t>(st);
  if (!M.frags.empty())
    if (int rc = mck_wal_gather_batch(wal_dev, d_fr, (uint32_t)M.frags.size(), d_buf, s)) return rc;
  const mck_spans sp{d_buf, d_offs, d_lens, 0, 0, (uint32_t)M.recs.size()};
  return mck_xxh3_64_batch(&sp, *d_out, s);
}
size_t multi_bytes(const MultiPlan& M) {
  if (M.recs.empty()) return 0;
  return DevArena::need(M.frags.size(), sizeof(mck_wal_fragment)) + DevArena::need(M.offs.size(), 8) +
         DevArena::need(M.lens.size(), 4) + DevArena::need(M.bytes + 64, 1) + DevArena::need(M.recs.size(), 8);
}
}  // namespace

// The per-block results (mck_wal_verify_batch's) the walk over verdicts
// consumes, from the block walk and the device's per-record verdicts: a
// block stops at its first record whose CRC fails, else where its walk did.
static void block_results(const std::vector<PhysRec>& phys, const std::vector<BlockStop>& stops,
                          const std::vector<uint8_t>& ok, uint64_t nbytes, std::vector<mck_wal_block_result>& res) {
  res.resize(stops.size());
  for (size_t b = 0; b < stops.size(); b++) {
    const BlockStop& st = stops[b];
    const uint64_t base = b * (uint64_t)MCK_WAL_kBlockSize;
    const uint32_t size = (uint32_t)std::min<uint64_t>(MCK_WAL_kBlockSize, nbytes - base);
    mck_wal_block_result r{st.count, st.status, st.status ? st.pos : size, st.pos};
    for (uint32_t j = 0; j < st.count; j++) {
      if (!ok[st.first + j]) {
        const uint32_t h = (uint32_t)(phys[st.first + j].hoff - base);
        r = mck_wal_block_result{j, MCK_WAL_BAD_CHECKSUM, h, h};
        break;
      }
    }
    res[b] = r;
  }
}

extern "C" int mck_wal_recover(const void* wal_host, const void* wal_dev, uint64_t nbytes, uint32_t log_number,
                               int recovery_mode, mck_stream_t stream, mck_wal_recovery** out) {
  mck_internal_set_error("");
  if (!out || (nbytes && (!wal_host || !wal_dev))) {
    mck_internal_set_error("wal_host / wal_dev / out is NULL");
    return MCK_EINVAL;
  }
  *out = nullptr;
  if (recovery_mode < MCK_WAL_kTolerateCorruptedTailRecords || recovery_mode > MCK_WAL_kSkipAnyCorruptedRecords) {
    mck_internal_set_error("unknown WALRecoveryMode");
    return MCK_EINVAL;
  }
  if (nbytes >> 48) {
    mck_internal_set_error("WAL image too large (payload offsets are 48-bit)");
    return MCK_EINVAL;
  }
  mck_wal_recovery* R = new (std::nothrow) mck_wal_recovery();
  if (!R) {
    mck_internal_set_error("out of memory");
    return MCK_ENOMEM;
  }
  const uint8_t* d = static_cast<const uint8_t*>(wal_host);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  double t0 = now_s();
  // 1. the plan: every physical record (the block walk) and the reader's
  //    walk with every CRC trusted
  std::vector<PhysRec> phys;
  std::vector<BlockStop> stops;
  wal_block_walk(d, nbytes, log_number, phys, stops);
  if (phys.size() > 0xFFFFFFFFull) {
    delete R;
    mck_internal_set_error("more than 2^32 physical records");
    return MCK_EINVAL;
  }
  const uint32_t np = (uint32_t)phys.size();
  WalWalk plan;
  if (!wal_walk_fast(nbytes, phys, stops, plan)) {  // (the list walk declines: the reader's walk)
    if (int rc = wal_walk(d, nbytes, log_number, recovery_mode, nullptr, plan, &phys)) {
      delete R;
      return rc;
    }
  }
  // the device plan, one descriptor per physical record (ranges over
  // threads: the array's first-touch page faults dominate its build)
  std::unique_ptr<mck_wal_rec_desc[]> desc(new (std::nothrow) mck_wal_rec_desc[np ? np : 1]);  // (no zeroing pass)
  if (!desc) {
    delete R;
    mck_internal_set_error("out of memory");
    return MCK_ENOMEM;
  }
  {
    const uint32_t hw = std::max(1u, std::thread::hardware_concurrency());
    const uint32_t T = std::min<uint32_t>(std::min<uint32_t>(hw, 16), np / 65536 + 1);
    auto fill = [&](uint32_t lo, uint32_t hi) {
      for (uint32_t i = lo; i < hi; i++) {
        const PhysRec& p = phys[i];
        const uint64_t po = p.hoff + p.hsize;
        const bool full = p.type == 1 || p.type == 5;
        desc[i] = mck_wal_rec_desc{(uint32_t)po,
                                   (uint32_t)(po >> 32) | ((uint32_t)p.type << 16) | (full ? MCK_WAL_REC_HASH : 0u),
                                   p.length, p.stored};
      }
    };
    if (T <= 1) {
      fill(0, np);
    } else {
      std::vector<std::thread> th;
      for (uint32_t k = 0; k < T; k++)
        th.emplace_back(fill, (uint32_t)((uint64_t)np * k / T), (uint32_t)((uint64_t)np * (k + 1) / T));
      for (auto& x : th) x.join();
    }
  }
  const MultiPlan M = plan.compression ? MultiPlan{} : multi_plan(plan);
  R->info.walk_seconds = now_s() - t0;
  R->info.host_walks = 1;
  // 2. the device pass (+ the multi-fragment records), one readback
  t0 = now_s();
  std::vector<uint8_t> ok(np);
  std::vector<uint64_t> hashes(np), mhash(M.recs.size());
  int rc = MCK_OK;
  {
    DevArena A{st};
    const size_t need = DevArena::need(np, sizeof(mck_wal_rec_desc)) + DevArena::need(np, 1) +
                        DevArena::need(np, 8) + multi_bytes(M);
    if (np && !(rc = A.reserve(need))) {
      auto* d_desc = A.take<mck_wal_rec_desc>(np);
      auto* d_ok = A.take<uint8_t>(np);
      auto* d_hash = A.take<uint64_t>(np);
      uint64_t* d_mh = nullptr;
      if (hipMemcpyAsync(d_desc, desc.get(), (size_t)np * sizeof(mck_wal_rec_desc), hipMemcpyHostToDevice, st)) {
        mck_internal_set_error("hipMemcpyAsync failed (record plan)");
        rc = MCK_EHIP;
      }
      if (!rc) rc = mck_wal_recover_batch(wal_dev, d_desc, np, log_number, d_ok, d_hash, stream);
      if (!rc) rc = launch_multi(wal_dev, M, A, &d_mh, st);
      if (!rc && (hipMemcpyAsync(ok.data(), d_ok, np, hipMemcpyDeviceToHost, st) ||
                  hipMemcpyAsync(hashes.data(), d_hash, (size_t)np * 8, hipMemcpyDeviceToHost, st) ||
                  (d_mh && hipMemcpyAsync(mhash.data(), d_mh, mhash.size() * 8, hipMemcpyDeviceToHost, st)))) {
        mck_internal_set_error("hipMemcpyAsync failed (recover results)");
        rc = MCK_EHIP;
      }
    }
    if (!rc && hipStreamSynchronize(st)) {
      mck_internal_set_error("hipStreamSynchronize failed (recover)");
      rc = MCK_EHIP;
    }
  }
  R->info.device_seconds = now_s() - t0;
  if (rc) {
    delete R;
    return rc;
  }
  block_results(phys, stops, ok, nbytes, R->blocks);
  // 3. a failed checksum changes the walk: walk again over the verdicts
  bool bad = false;
  for (uint32_t i = 0; i < np && !bad; i++) bad = !ok[i];
  WalWalk& W = R->W;
  const MultiPlan* MP = &M;
  MultiPlan M2;
  std::vector<uint64_t> mhash2;
  if (!bad) {
    W = std::move(plan);
  } else {
    t0 = now_s();
    rc = wal_walk(d, nbytes, log_number, recovery_mode, R->blocks.data(), W, &phys);
    R->info.walk_seconds += now_s() - t0;
    R->info.host_walks = 2;
    if (rc) {
      mck_internal_set_error("recover: the walk over the verdicts reached a record the block walk did not");
      delete R;
      return rc;
    }
    if (!W.compression) {
      M2 = multi_plan(W);
      mhash2.resize(M2.recs.size());
      t0 = now_s();
      if (!M2.recs.empty()) {
        DevArena A{st};
        uint64_t* d_mh = nullptr;
        if (!(rc = A.reserve(multi_bytes(M2)))) rc = launch_multi(wal_dev, M2, A, &d_mh, st);
        if (!rc && (hipMemcpyAsync(mhash2.data(), d_mh, mhash2.size() * 8, hipMemcpyDeviceToHost, st) ||
                    hipStreamSynchronize(st))) {
          mck_internal_set_error("recover: multi-fragment readback failed");
          rc = MCK_EHIP;
        }
      }
      R->info.device_seconds += now_s() - t0;
      if (rc) {
        delete R;
        return rc;
      }
      MP = &M2;
    }
  }
  const std::vector<uint64_t>& mh = bad ? mhash2 : mhash;
  // 4. every record's checksum: a one-fragment record's from its physical
  //    record (records come in file order: one forward cursor)
  const size_t nr = W.roff.size();
  R->info.nrecords = nr;
  R->info.has_checksums = W.compression ? 0u : 1u;
  if (!W.compression) {
    R->checksums.assign(nr, 0);
    uint32_t cur = 0;
    for (size_t r = 0; r < nr; r++) {
      if (W.rhoff[r] == ~0ull) continue;
      while (cur < np && phys[cur].hoff < W.rhoff[r]) cur++;
      if (cur >= np || phys[cur].hoff != W.rhoff[r]) {  // cannot happen: the block walk lists every record
        mck_internal_set_error("recover: a record outside the block walk");
        delete R;
        return MCK_EINVAL;
      }
      R->checksums[r] = hashes[cur];
      R->info.in_place++;
    }
    for (size_t j = 0; j < MP->recs.size(); j++) R->checksums[MP->recs[j]] = mh[j];
    R->info.gathered = MP->recs.size();
    R->info.gathered_bytes = 0;
    for (uint32_t n : MP->lens) R->info.gathered_bytes += n;
  }
  *out = R;
  return MCK_OK;
}

extern "C" int mck_wal_recovery_read_out(const mck_wal_recovery* r, mck_wal_read_out* out) {
  mck_internal_set_error("");
  if (!r) {
    mck_internal_set_error("recovery is NULL");
    return MCK_EINVAL;
  }
  if (int rc = check_read_args(nullptr, 0, MCK_WAL_kTolerateCorruptedTailRecords, out)) return rc;
  return wal_copy_out(r->W, out);
}

extern "C" int mck_wal_recovery_checksums(const mck_wal_recovery* r, uint64_t* checksums, uint64_t cap) {
  mck_internal_set_error("");
  if (!r) {
    mck_internal_set_error("recovery is NULL");
    return MCK_EINVAL;
  }
  if (!r->info.has_checksums) {
    mck_internal_set_error("compressed WAL: the record checksums are over the decompressed records (the caller's)");
    return MCK_ENOTSUP;
  }
  if (r->checksums.empty()) return MCK_OK;
  if (!checksums || cap < r->checksums.size()) {
    mck_internal_set_error("checksums capacity too small");
    return MCK_EINVAL;
  }
  memcpy(checksums, r->checksums.data(), r->checksums.size() * 8);
  return MCK_OK;
}

extern "C" int mck_wal_recovery_get_info(const mck_wal_recovery* r, mck_wal_recovery_info* info) {
  if (!r || !info) return MCK_EINVAL;
  *info = r->info;
  return MCK_OK;
}

extern "C" int mck_wal_recovery_block_results(const mck_wal_recovery* r, mck_wal_block_result* results,
                                              uint64_t cap) {
  mck_internal_set_error("");
  if (!r || (!results && !r->blocks.empty()) || cap < r->blocks.size()) {
    mck_internal_set_error("recovery / results is NULL or the capacity is too small");
    return MCK_EINVAL;
  }
  if (!r->blocks.empty()) memcpy(results, r->blocks.data(), r->blocks.size() * sizeof(mck_wal_block_result));
  return MCK_OK;
}

extern "C" int mck_wal_recovery_report_positions(const mck_wal_recovery* r, uint64_t* positions, uint64_t cap) {
  mck_internal_set_error("");
  if (!r || (!positions && !r->W.report_pos.empty()) || cap < r->W.report_pos.size()) {
    mck_internal_set_error("recovery / positions is NULL or the capacity is too small");
    return MCK_EINVAL;
  }
  if (!r->W.report_pos.empty()) memcpy(positions, r->W.report_pos.data(), r->W.report_pos.size() * 8);
  return MCK_OK;
}

extern "C" void mck_wal_recovery_free(mck_wal_recovery* r) { delete r; }

