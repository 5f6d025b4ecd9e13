// Reference-side adapters: what a maintainer adds to the Speedb tree to bind
// its checksum call sites to the engine.  This
// header is compiled against the reference's own headers by
// tests/test_integration_compile.py (-fsyntax-only, skipped when the
// reference tree is absent), so a signature drift on either side -- the
// reference's interfaces or include/speedb_amd/checksum.hpp -- fails a test
// instead of surfacing in a maintainer's build.
//
// Include it from a translation unit of the reference tree (include paths
// <ref>/include and <ref>, the HIP runtime headers, and this repo's include/).
#pragma once

#include <array>
#include <memory>
#include <string>
#include <type_traits>
#include <vector>

#include "db/log_format.h"
#include "db/log_reader.h"
#include "rocksdb/file_checksum.h"
#include "rocksdb/options.h"
#include "speedb_amd/checksum.hpp"
#include "speedb_amd/mck.h"
#include "table/block_based/block_based_table_reader.h"
#include "table/block_based/reader_common.h"
#include "table/format.h"
#include "util/coding.h"
#include "util/compression.h"

namespace speedb_amd_rocksdb {
namespace rdb = ROCKSDB_NAMESPACE;

// ---- the reference interfaces these adapters stand in for ----------------
// table/format.h:307-311
static_assert(std::is_same<decltype(&rdb::ComputeBuiltinChecksum),
                           uint32_t (*)(rdb::ChecksumType, const char*, size_t)>::value,
              "rocksdb::ComputeBuiltinChecksum signature drifted (table/format.h)");
static_assert(std::is_same<decltype(&rdb::ComputeBuiltinChecksumWithLastByte),
                           uint32_t (*)(rdb::ChecksumType, const char*, size_t, char)>::value,
              "rocksdb::ComputeBuiltinChecksumWithLastByte signature drifted (table/format.h)");
// table/format.h:119
static_assert(std::is_same<decltype(&rdb::ChecksumModifierForContext), uint32_t (*)(uint32_t, uint64_t)>::value,
              "rocksdb::ChecksumModifierForContext signature drifted (table/format.h)");
// table/block_based/reader_common.h:33-36
static_assert(std::is_same<decltype(&rdb::VerifyBlockChecksum),
                           rdb::Status (*)(const rdb::Footer&, const char*, size_t, const std::string&,
                                           uint64_t)>::value,
              "rocksdb::VerifyBlockChecksum signature drifted (reader_common.h)");
// include/rocksdb/table.h:69-75: the same on-disk enum values
static_assert((int)rdb::kNoChecksum == (int)speedb_amd::kNoChecksum && (int)rdb::kCRC32c == (int)speedb_amd::kCRC32c &&
                  (int)rdb::kxxHash == (int)speedb_amd::kxxHash &&
                  (int)rdb::kxxHash64 == (int)speedb_amd::kxxHash64 && (int)rdb::kXXH3 == (int)speedb_amd::kXXH3,
              "ChecksumType values differ");
static_assert(std::string_view(rdb::kStandardDbFileChecksumFuncName) ==
                  std::string_view(speedb_amd::kStandardDbFileChecksumFuncName),
              "file checksum function name differs");

inline rdb::Status ToRocks(const speedb_amd::Status& s) {
  if (s.ok()) return rdb::Status::OK();
  if (s.IsCorruption()) return rdb::Status::Corruption(s.message());
  if (s.IsInvalidArgument()) return rdb::Status::InvalidArgument(s.message());
  if (s.IsNotSupported()) return rdb::Status::NotSupported(s.message());
  return rdb::Status::IOError(s.message());
}

inline speedb_amd::Footer FromRocks(const rdb::Footer& footer) {
  return speedb_amd::Footer{static_cast<speedb_amd::ChecksumType>(footer.checksum_type()),
                            footer.base_context_checksum()};
}

// ---- 2.1: reader_common.cc:26-63 VerifyBlockChecksum, re-pointed ---------
// Same signature and Corruption message as the reference; a device error is
// an IOError (the reference function cannot fail any other way).
inline rdb::Status VerifyBlockChecksum(const rdb::Footer& footer, const char* data, size_t block_size,
                                       const std::string& file_name, uint64_t offset) {
  try {
    return ToRocks(speedb_amd::VerifyBlockChecksum(FromRocks(footer), data, block_size, file_name, offset));
  } catch (const speedb_amd::DeviceError& e) {
    return rdb::Status::IOError(e.what());
  }
}
static_assert(std::is_same<decltype(&VerifyBlockChecksum), decltype(&rdb::VerifyBlockChecksum)>::value,
              "the shim must keep the reference's signature");

// MultiGet / RetrieveMultipleBlocks (block_based_table_reader_sync_and_async.h
// :217-228): every block of one MultiRead buffer already in device memory,
// one batch; per_block[i] is what VerifyBlockChecksum would return.
inline rdb::Status VerifyBlockChecksums(const rdb::Footer& footer, const void* dev_image, uint64_t file_base,
                                        const std::vector<rdb::BlockHandle>& handles,
                                        const std::string& file_name, std::vector<rdb::Status>* per_block,
                                        mck_stream_t stream = nullptr) {
  std::vector<speedb_amd::BlockHandle> hs;
  hs.reserve(handles.size());
  for (const rdb::BlockHandle& h : handles) hs.push_back({h.offset(), h.size()});
  std::vector<speedb_amd::Status> st;
  const speedb_amd::Status s =
      speedb_amd::VerifyBlockChecksums(FromRocks(footer), dev_image, file_base, hs, file_name, &st, stream);
  if (per_block) {
    per_block->clear();
    for (const speedb_amd::Status& x : st) per_block->push_back(ToRocks(x));
  }
  return ToRocks(s);
}

// ---- 2.2: whole-SST listing with compressed index blocks ------------------
// enable_index_compression defaults to true (include/rocksdb/table.h:541):
// mck_sst_list_blocks_uncompress hands each compressed index / meta block to
// this callback, which runs the reference's own UncompressBlockData
// (table/format.h:412) with the table's dictionary and keeps the result alive
// until the listing returns.
static_assert(std::is_same<decltype(&rdb::UncompressBlockData),
                           rdb::Status (*)(const rdb::UncompressionInfo&, const char*, size_t, rdb::BlockContents*,
                                           uint32_t, const rdb::ImmutableOptions&, rdb::MemoryAllocator*)>::value,
              "rocksdb::UncompressBlockData signature drifted (table/format.h)");
struct UncompressCtx {
  const rdb::ImmutableOptions* ioptions;
  uint32_t format_version;
  const rdb::UncompressionDict* dict = &rdb::UncompressionDict::GetEmptyDict();
  std::vector<rdb::BlockContents> held;  // the uncompressed blocks (their buffers do not move)
  rdb::Status status;                    // the first failure, for the caller
};
inline int UncompressWithReference(void* c, uint8_t type, uint64_t /*block_offset*/, const void* raw,
                                   uint64_t raw_size, const void** out, uint64_t* out_size) {
  auto* ctx = static_cast<UncompressCtx*>(c);
  const auto ct = static_cast<rdb::CompressionType>(type);
  rdb::UncompressionContext uctx(ct);
  rdb::UncompressionInfo info(uctx, *ctx->dict, ct);
  rdb::BlockContents contents;
  rdb::Status s = rdb::UncompressBlockData(info, static_cast<const char*>(raw), static_cast<size_t>(raw_size),
                                           &contents, ctx->format_version, *ctx->ioptions);
  if (!s.ok()) {
    if (ctx->status.ok()) ctx->status = s;
    return s.IsNotSupported() ? MCK_ENOTSUP : MCK_ECORRUPT;
  }
  *out = contents.data.data();
  *out_size = contents.data.size();
  ctx->held.push_back(std::move(contents));
  return MCK_OK;
}
static_assert(std::is_same<decltype(&UncompressWithReference), mck_sst_uncompress_fn>::value,
              "the callback must keep mck_sst_uncompress_fn's signature");

// ---- 2.3 / 2.4: the WAL -----------------------------------------------------
// include/rocksdb/options.h:383-420 WALRecoveryMode: the engine's mode codes
// are the enum's values (mck_wal_read_records / mck_wal_recover take them)
static_assert((int)rdb::WALRecoveryMode::kTolerateCorruptedTailRecords == MCK_WAL_kTolerateCorruptedTailRecords &&
                  (int)rdb::WALRecoveryMode::kAbsoluteConsistency == MCK_WAL_kAbsoluteConsistency &&
                  (int)rdb::WALRecoveryMode::kPointInTimeRecovery == MCK_WAL_kPointInTimeRecovery &&
                  (int)rdb::WALRecoveryMode::kSkipAnyCorruptedRecords == MCK_WAL_kSkipAnyCorruptedRecords,
              "WALRecoveryMode values differ (include/rocksdb/options.h)");
static_assert((int)rdb::WALRecoveryMode::kTolerateCorruptedTailRecords ==
                      (int)speedb_amd::log::WALRecoveryMode::kTolerateCorruptedTailRecords &&
                  (int)rdb::WALRecoveryMode::kSkipAnyCorruptedRecords ==
                      (int)speedb_amd::log::WALRecoveryMode::kSkipAnyCorruptedRecords,
              "the mirror's WALRecoveryMode differs");
// db/log_format.h:20-52: block and header sizes, every record type
static_assert(rdb::log::kBlockSize == MCK_WAL_kBlockSize && rdb::log::kHeaderSize == MCK_WAL_kHeaderSize &&
                  rdb::log::kRecyclableHeaderSize == MCK_WAL_kRecyclableHeaderSize,
              "WAL block / header sizes differ (db/log_format.h)");
static_assert((int)rdb::log::kZeroType == speedb_amd::log::kZeroType &&
                  (int)rdb::log::kFullType == speedb_amd::log::kFullType &&
                  (int)rdb::log::kFirstType == speedb_amd::log::kFirstType &&
                  (int)rdb::log::kMiddleType == speedb_amd::log::kMiddleType &&
                  (int)rdb::log::kLastType == speedb_amd::log::kLastType &&
                  (int)rdb::log::kRecyclableFullType == speedb_amd::log::kRecyclableFullType &&
                  (int)rdb::log::kRecyclableFirstType == speedb_amd::log::kRecyclableFirstType &&
                  (int)rdb::log::kRecyclableMiddleType == speedb_amd::log::kRecyclableMiddleType &&
                  (int)rdb::log::kRecyclableLastType == speedb_amd::log::kRecyclableLastType &&
                  (int)rdb::log::kSetCompressionType == speedb_amd::log::kSetCompressionType &&
                  (int)rdb::log::kUserDefinedTimestampSizeType == speedb_amd::log::kUserDefinedTimestampSizeType &&
                  (int)rdb::log::kRecyclableUserDefinedTimestampSizeType ==
                      speedb_amd::log::kRecyclableUserDefinedTimestampSizeType &&
                  rdb::log::kMaxRecordType == speedb_amd::log::kRecyclableUserDefinedTimestampSizeType,
              "WAL record types differ (db/log_format.h)");

// The reference's reader interfaces the adapters stand in for
// (db/log_reader.h:41-48 Reporter::Corruption, :76-79 ReadRecord).
template <class T>
struct MemberFn;
template <class C, class R, class... A>
struct MemberFn<R (C::*)(A...)> {
  using type = R(A...);
};
static_assert(std::is_same<MemberFn<decltype(&rdb::log::Reader::Reporter::Corruption)>::type,
                           void(size_t, const rdb::Status&)>::value,
              "log::Reader::Reporter::Corruption signature drifted (db/log_reader.h)");
static_assert(std::is_same<MemberFn<decltype(&rdb::log::Reader::ReadRecord)>::type,
                           bool(rdb::Slice*, std::string*, rdb::WALRecoveryMode, uint64_t*)>::value,
              "log::Reader::ReadRecord signature drifted (db/log_reader.h)");

// Reporter adapter: the engine's reports, replayed into the reference's
// Reporter in its own order (each inside the ReadRecord call that makes it,
// mck_wal_recovery_report_positions), as Reader::ReportCorruption does
// (db/log_reader.cc:399-407: Corruption(bytes, Status::Corruption(reason))).
class ReporterBridge : public speedb_amd::log::RecoveryReader::Reporter {
 public:
  explicit ReporterBridge(rdb::log::Reader::Reporter* r) : r_(r) {}
  void Corruption(size_t bytes, const speedb_amd::Status& s) override {
    if (r_) r_->Corruption(bytes, rdb::Status::Corruption(s.message()));
  }

 private:
  rdb::log::Reader::Reporter* r_;
};

// DBImpl::RecoverLogFiles' reader (db/db_impl/db_impl_open.cc:1204-1221):
// constructed like log::Reader (reporter, log number), fed the whole log once
// (Recover: the file's bytes and their device copy), then ReadRecord with the
// reference's signature -- records, record_checksum (XXH3_64bits) and the
// reporter's calls as log::Reader yields them, the CRCs and XXH3 of the
// whole log computed in one device pass (mck_wal_recover).
class GpuLogRecoveryReader {
 public:
  GpuLogRecoveryReader(rdb::log::Reader::Reporter* reporter, uint64_t log_num)
      : bridge_(reporter), reader_(&bridge_, log_num) {}
  rdb::Status Recover(const char* file_bytes, const void* dev_bytes, uint64_t n, rdb::WALRecoveryMode mode,
                      mck_stream_t stream = nullptr) {
    return ToRocks(reader_.Recover(file_bytes, dev_bytes, n,
                                   static_cast<speedb_amd::log::WALRecoveryMode>(mode), stream));
  }
  bool ReadRecord(rdb::Slice* record, std::string* scratch,
                  rdb::WALRecoveryMode wal_recovery_mode = rdb::WALRecoveryMode::kTolerateCorruptedTailRecords,
                  uint64_t* record_checksum = nullptr) {
    std::string_view v;
    const bool got = reader_.ReadRecord(&v, scratch, static_cast<speedb_amd::log::WALRecoveryMode>(wal_recovery_mode),
                                        record_checksum);
    *record = rdb::Slice(v.data(), v.size());
    return got;
  }
  uint64_t LastRecordOffset() const { return reader_.LastRecordOffset(); }

 private:
  ReporterBridge bridge_;
  speedb_amd::log::RecoveryReader reader_;
};
static_assert(std::is_same<MemberFn<decltype(&GpuLogRecoveryReader::ReadRecord)>::type,
                           MemberFn<decltype(&rdb::log::Reader::ReadRecord)>::type>::value,
              "the recovery reader must keep log::Reader::ReadRecord's signature");

// ---- 2.5: SST block trailers, a run of blocks at once -----------------------
// BlockBasedTableBuilder::WriteMaybeCompressedBlock
// (table/block_based/block_based_table_builder.cc:1304-1358) appends
// [compression type][LE32 checksum + ChecksumModifierForContext(base, offset)]
// behind each block; the builder (or a compaction output job holding many
// blocks in device memory) seals a run of them in one batch: the block
// contents as the builder's Slice / CompressionType / BlockHandle, the
// trailers written the way the builder writes them (EncodeFixed32).
static_assert(rdb::BlockBasedTable::kBlockTrailerSize == 5, "block trailer is [type][LE32] (block_based_table_reader.h)");
static_assert(sizeof(rdb::CompressionType) == 1, "the trailer's type byte is the CompressionType value");
inline rdb::Status ComputeBlockTrailers(rdb::ChecksumType checksum_type, uint32_t base_context_checksum,
                                        const void* dev_image, uint64_t file_base,
                                        const std::vector<rdb::BlockHandle>& handles,
                                        const std::vector<rdb::CompressionType>& comp_types,
                                        std::vector<std::array<char, rdb::BlockBasedTable::kBlockTrailerSize>>* trailers,
                                        mck_stream_t stream = nullptr) {
  const size_t n = handles.size();
  trailers->assign(n, {});
  if (n != comp_types.size()) return rdb::Status::InvalidArgument("one compression type per block");
  if (!n) return rdb::Status::OK();
  std::vector<uint64_t> offs(n), foffs(n);
  std::vector<uint32_t> lens(n), out(n);
  std::vector<uint8_t> ct(n);
  for (size_t i = 0; i < n; i++) {
    offs[i] = handles[i].offset() - file_base;
    foffs[i] = handles[i].offset();
    lens[i] = static_cast<uint32_t>(handles[i].size());
    ct[i] = static_cast<uint8_t>(comp_types[i]);
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  void* d = nullptr;
  const size_t bytes = n * (8 + 8 + 4 + 4 + 1);
  if (hipMalloc(&d, bytes) != hipSuccess) return rdb::Status::IOError("hipMalloc failed");
  char* p = static_cast<char*>(d);
  uint64_t* d_off = reinterpret_cast<uint64_t*>(p);
  uint64_t* d_foff = reinterpret_cast<uint64_t*>(p + 8 * n);
  uint32_t* d_len = reinterpret_cast<uint32_t*>(p + 16 * n);
  uint32_t* d_out = reinterpret_cast<uint32_t*>(p + 20 * n);
  uint8_t* d_ct = reinterpret_cast<uint8_t*>(p + 24 * n);
  (void)hipMemcpyAsync(d_off, offs.data(), 8 * n, hipMemcpyHostToDevice, st);
  (void)hipMemcpyAsync(d_foff, foffs.data(), 8 * n, hipMemcpyHostToDevice, st);
  (void)hipMemcpyAsync(d_len, lens.data(), 4 * n, hipMemcpyHostToDevice, st);
  (void)hipMemcpyAsync(d_ct, ct.data(), n, hipMemcpyHostToDevice, st);
  const mck_spans sp{dev_image, d_off, d_len, 0, 0, static_cast<uint32_t>(n)};
  const int rc = mck_sst_trailer_batch(static_cast<int>(checksum_type), &sp, d_ct, d_foff, base_context_checksum,
                                       d_out, stream);
  if (!rc) (void)hipMemcpyAsync(out.data(), d_out, 4 * n, hipMemcpyDeviceToHost, st);
  const bool synced = hipStreamSynchronize(st) == hipSuccess;
  (void)hipFree(d);
  if (rc) return ToRocks(speedb_amd::FromRc(rc, "mck_sst_trailer_batch"));
  if (!synced) return rdb::Status::IOError("hipStreamSynchronize failed");
  for (size_t i = 0; i < n; i++) {
    (*trailers)[i][0] = static_cast<char>(comp_types[i]);
    rdb::EncodeFixed32((*trailers)[i].data() + 1, out[i]);
  }
  return rdb::Status::OK();
}

// ---- 2.6: include/rocksdb/file_checksum.h:50-90 ---------------------------
class GpuFileChecksumGenCrc32c : public rdb::FileChecksumGenerator {
 public:
  explicit GpuFileChecksumGenCrc32c(const rdb::FileChecksumGenContext& c)
      : impl_(speedb_amd::FileChecksumGenContext{c.file_name, c.requested_checksum_func_name}) {}
  void Update(const char* data, size_t n) override { impl_.Update(data, n); }
  // bytes already in HBM (a device-built SST): no host copy
  bool UpdateDevice(const void* dev_data, uint64_t n, mck_stream_t stream = nullptr) {
    return impl_.UpdateDevice(dev_data, n, stream);
  }
  void Finalize() override { impl_.Finalize(); }
  std::string GetChecksum() const override { return impl_.GetChecksum(); }
  const char* Name() const override { return impl_.Name(); }

 private:
  speedb_amd::FileChecksumGenCrc32c impl_;
};

class GpuFileChecksumGenFactory : public rdb::FileChecksumGenFactory {
 public:
  std::unique_ptr<rdb::FileChecksumGenerator> CreateFileChecksumGenerator(
      const rdb::FileChecksumGenContext& context) override {
    if (context.requested_checksum_func_name.empty() ||
        context.requested_checksum_func_name == rdb::kStandardDbFileChecksumFuncName)
      return std::unique_ptr<rdb::FileChecksumGenerator>(new GpuFileChecksumGenCrc32c(context));
    return nullptr;
  }
  static const char* kClassName() { return "FileChecksumGenCrc32cFactory"; }
  const char* Name() const override { return kClassName(); }
};

}  // namespace speedb_amd_rocksdb
