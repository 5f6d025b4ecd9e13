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

#include <memory>
#include <string>
#include <type_traits>
#include <vector>

#include "rocksdb/file_checksum.h"
#include "speedb_amd/checksum.hpp"
#include "speedb_amd/mck.h"
#include "table/block_based/reader_common.h"
#include "table/format.h"
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
