// checksum.hpp -- C++ host-side mirror of the reference's block-checksum
// interface, implemented over the engine's C ABI (mck.h).
//
// A Speedb/RocksDB build re-points its call sites at these names (see
// INTEGRATION.md); signatures, argument meaning and error behaviour follow
// the reference:
//   crc32c::Value / Extend / Mask / Unmask / Crc32cCombine  util/crc32c.h:21-53
//   XXH3_64bits                                             util/xxhash.h:5329
//   ChecksumType                                            include/rocksdb/table.h:69-75
//   ComputeBuiltinChecksum[WithLastByte]                    table/format.cc:578-645
//   ChecksumModifierForContext                              table/format.h:119-146
//   VerifyBlockChecksum                                     table/block_based/reader_common.cc:26-63
//   log::EmitPhysicalRecord's header CRC                    db/log_writer.cc:263-311
// plus the batched entry points the reference lacks (VerifyBlockChecksums
// for RetrieveMultipleBlocks / VerifyChecksumInBlocks, block trailer
// generation for a run of blocks, whole-WAL verification).
//
// Header-only; link against speedb_amd/libspeedb_amd.so.
#pragma once
#include <stdint.h>

#include <memory>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

#include "mck.h"

namespace speedb_amd {

// include/rocksdb/table.h:69-75
enum ChecksumType : char {
  kNoChecksum = 0x0,
  kCRC32c = 0x1,
  kxxHash = 0x2,
  kxxHash64 = 0x3,
  kXXH3 = 0x4,
};

// The slice of rocksdb::Status this path produces.
class Status {
 public:
  Status() = default;
  static Status OK() { return Status(); }
  static Status Corruption(const std::string& msg) { return Status(kCorruption, msg); }
  static Status InvalidArgument(const std::string& msg) { return Status(kInvalidArgument, msg); }
  static Status IOError(const std::string& msg) { return Status(kIOError, msg); }
  static Status NotSupported(const std::string& msg) { return Status(kNotSupported, msg); }
  bool ok() const { return code_ == kOk; }
  bool IsCorruption() const { return code_ == kCorruption; }
  bool IsInvalidArgument() const { return code_ == kInvalidArgument; }
  bool IsNotSupported() const { return code_ == kNotSupported; }
  bool IsIOError() const { return code_ == kIOError; }
  const std::string& message() const { return msg_; }
  std::string ToString() const {
    switch (code_) {
      case kOk:
        return "OK";
      case kCorruption:
        return "Corruption: " + msg_;
      case kInvalidArgument:
        return "Invalid argument: " + msg_;
      case kNotSupported:
        return "Not implemented: " + msg_;
      default:
        return "IO error: " + msg_;
    }
  }

 private:
  enum Code { kOk, kCorruption, kInvalidArgument, kIOError, kNotSupported };
  Status(Code c, const std::string& m) : code_(c), msg_(m) {}
  Code code_ = kOk;
  std::string msg_;
};

inline Status FromRc(int rc, const char* what) {
  if (rc == MCK_OK) return Status::OK();
  if (rc == MCK_ECORRUPT) return Status::Corruption(mck_last_error());
  if (rc == MCK_ENOTSUP) return Status::NotSupported(mck_last_error());
  std::string m = std::string(what) + ": " + mck_last_error();
  return rc == MCK_EINVAL ? Status::InvalidArgument(m) : Status::IOError(m);
}

// The reference's checksum functions return a bare value and cannot fail.
// Here the data-reading ones run on the GPU and CAN (no device, a HIP
// error): a re-pointed call site must never receive a made-up checksum (a
// trailer writer would store it, a verifier would compare against it), so
// the mirror's reference-named functions go through the error-reporting
// *_r entry points and throw DeviceError on failure -- never the plain
// mck_* shims, which return 0.  Callers that cannot take an exception use
// the *_r functions of mck.h directly.
class DeviceError : public std::runtime_error {
 public:
  DeviceError(const char* what, int rc)
      : std::runtime_error(std::string(what) + " failed (rc=" + std::to_string(rc) + "): " + mck_last_error()),
        rc_(rc) {}
  int rc() const { return rc_; }

 private:
  int rc_;
};

inline uint32_t CheckedU32(int rc, uint32_t v, const char* what) {
  if (rc != MCK_OK) throw DeviceError(what, rc);
  return v;
}
inline uint64_t CheckedU64(int rc, uint64_t v, const char* what) {
  if (rc != MCK_OK) throw DeviceError(what, rc);
  return v;
}

namespace crc32c {
static const uint32_t kMaskDelta = 0xa282ead8ul;
inline uint32_t Extend(uint32_t init_crc, const char* data, size_t n) {
  uint32_t v = 0;
  const int rc = mck_crc32c_extend_r(init_crc, data, n, &v);
  return CheckedU32(rc, v, "crc32c::Extend");
}
inline uint32_t Value(const char* data, size_t n) {
  uint32_t v = 0;
  const int rc = mck_crc32c_value_r(data, n, &v);
  return CheckedU32(rc, v, "crc32c::Value");
}
inline uint32_t Mask(uint32_t crc) { return mck_crc32c_mask(crc); }
inline uint32_t Unmask(uint32_t masked_crc) { return mck_crc32c_unmask(masked_crc); }
inline uint32_t Crc32cCombine(uint32_t crc1, uint32_t crc2, size_t crc2len) {
  return mck_crc32c_combine(crc1, crc2, crc2len);
}
}  // namespace crc32c

inline uint64_t XXH3_64bits(const void* data, size_t n) {
  uint64_t v = 0;
  const int rc = mck_xxh3_64_r(data, n, &v);
  return CheckedU64(rc, v, "XXH3_64bits");
}

inline uint32_t ComputeBuiltinChecksum(ChecksumType type, const char* data, size_t data_size) {
  uint32_t v = 0;
  const int rc = mck_builtin_checksum_r(type, data, data_size, &v);
  return CheckedU32(rc, v, "ComputeBuiltinChecksum");
}
inline uint32_t ComputeBuiltinChecksumWithLastByte(ChecksumType type, const char* data, size_t data_size,
                                                   char last_byte) {
  uint32_t v = 0;
  const int rc = mck_builtin_checksum_with_last_byte_r(type, data, data_size, last_byte, &v);
  return CheckedU32(rc, v, "ComputeBuiltinChecksumWithLastByte");
}
inline uint32_t ChecksumModifierForContext(uint32_t base_context_checksum, uint64_t offset) {
  return mck_context_modifier(base_context_checksum, offset);
}

inline uint32_t DecodeFixed32(const char* p) {
  const unsigned char* u = reinterpret_cast<const unsigned char*>(p);
  return (uint32_t)u[0] | ((uint32_t)u[1] << 8) | ((uint32_t)u[2] << 16) | ((uint32_t)u[3] << 24);
}

// The two footer fields VerifyBlockChecksum reads (table/format.h Footer).
struct Footer {
  ChecksumType checksum_type = kXXH3;
  uint32_t base_context_checksum = 0;
};

inline Status BlockChecksumMismatch(ChecksumType type, uint32_t stored, uint32_t computed, bool context,
                                    const std::string& file_name, uint64_t offset, size_t block_size) {
  if (type == kCRC32c) {  // reader_common.cc:51-55: unmask for people
    stored = crc32c::Unmask(stored);
    computed = crc32c::Unmask(computed);
  }
  return Status::Corruption("block checksum mismatch: stored" + std::string(context ? "(context removed)" : "") +
                            " = " + std::to_string(stored) + ", computed = " + std::to_string(computed) +
                            ", type = " + std::to_string((int)type) + "  in " + file_name + " offset " +
                            std::to_string(offset) + " size " + std::to_string(block_size));
}

// table/block_based/reader_common.cc:26-63.  data = block payload followed by
// its 5-byte trailer, host memory.
inline Status VerifyBlockChecksum(const Footer& footer, const char* data, size_t block_size,
                                  const std::string& file_name, uint64_t offset) {
  const ChecksumType type = footer.checksum_type;
  const size_t len = block_size + 1;
  uint32_t stored = DecodeFixed32(data + len);
  const uint32_t computed = ComputeBuiltinChecksum(type, data, len);
  const uint32_t modifier = ChecksumModifierForContext(footer.base_context_checksum, offset);
  stored -= modifier;
  if (stored == computed) return Status::OK();
  return BlockChecksumMismatch(type, stored, computed, modifier != 0, file_name, offset, block_size);
}

// PerfLevel / PerfContext::block_checksum_time (include/rocksdb/perf_level.h,
// include/rocksdb/perf_context.h:97), per thread: at a timing level every
// verify batch's DEVICE time is accumulated (mck_perf_context_get).
enum PerfLevel : unsigned char {
  kUninitialized = 0,
  kDisable = 1,
  kEnableCount = 2,
  kEnableTimeExceptForMutex = 3,
  kEnableTimeAndCPUTimeExceptForMutex = 4,
  kEnableTime = 5,
};
inline void SetPerfLevel(PerfLevel level) { (void)mck_set_perf_level(level); }
inline PerfLevel GetPerfLevel() { return static_cast<PerfLevel>(mck_get_perf_level()); }
struct PerfContext {
  uint64_t block_checksum_time = 0;   // ns of device time
  uint64_t block_checksum_count = 0;  // blocks verified
  void Reset() {
    mck_perf_context c;
    (void)mck_perf_context_get(&c, 1);
    block_checksum_time = block_checksum_count = 0;
  }
};
// This thread's context, brought up to date (waits for its timed batches).
inline PerfContext* get_perf_context() {
  static thread_local PerfContext ctx;
  mck_perf_context c;
  if (mck_perf_context_get(&c, 0) == MCK_OK) {
    ctx.block_checksum_time = c.block_checksum_time;
    ctx.block_checksum_count = c.block_checksum_count;
  }
  return &ctx;
}

// A block handle (table/format.h BlockHandle): payload offset and size.
struct BlockHandle {
  uint64_t offset;
  uint64_t size;
};

// Batched read-side verify: the caller has the blocks' bytes (payload +
// trailer, at handle.offset - file_base) in device memory, e.g. the buffer a
// MultiRead filled (table/block_based/block_based_table_reader_sync_and_async.h
// :217-228 verifies these one by one).  Writes one Status per block; returns
// the first non-OK status (or OK).
inline Status VerifyBlockChecksums(const Footer& footer, const void* dev_image, uint64_t file_base,
                                   const std::vector<BlockHandle>& handles, const std::string& file_name,
                                   std::vector<Status>* per_block, mck_stream_t stream = nullptr);

// table/block_based/block_based_table_reader.cc:2336-2500
// BlockBasedTable::VerifyChecksum of a whole SST image in host memory: the
// footer / metaindex / properties / index are read on the host
// (mck_sst_list_blocks), the format_version 6 footer checksum is checked, and
// every block is verified on the GPU in one batch.  Returns the first
// failure (Footer::DecodeFrom's or VerifyBlockChecksum's message).
inline Status VerifySstFile(const std::string& file_name, const char* image, uint64_t size,
                            std::vector<mck_sst_block>* blocks_out = nullptr, mck_stream_t stream = nullptr);

namespace log {
// db/log_format.h:22-45
enum RecordType {
  kZeroType = 0,
  kFullType = 1,
  kFirstType = 2,
  kMiddleType = 3,
  kLastType = 4,
  kRecyclableFullType = 5,
  kRecyclableFirstType = 6,
  kRecyclableMiddleType = 7,
  kRecyclableLastType = 8,
  kSetCompressionType = 9,
  kUserDefinedTimestampSizeType = 10,
  kRecyclableUserDefinedTimestampSizeType = 11,
};
constexpr unsigned int kBlockSize = MCK_WAL_kBlockSize;
constexpr int kHeaderSize = MCK_WAL_kHeaderSize;
constexpr int kRecyclableHeaderSize = MCK_WAL_kRecyclableHeaderSize;

inline bool IsRecyclable(unsigned t) {
  return (t >= kRecyclableFullType && t <= kRecyclableLastType) || t == kRecyclableUserDefinedTimestampSizeType;
}

// db/log_writer.cc:281-298: the masked header CRC of one physical record.
inline uint32_t PhysicalRecordCrc(RecordType t, const char* payload, size_t n, uint64_t log_number) {
  const char type_byte = static_cast<char>(t);
  uint32_t crc = crc32c::Value(&type_byte, 1);
  if (IsRecyclable(t)) {
    char buf[4];
    const uint32_t ln = static_cast<uint32_t>(log_number);
    for (int i = 0; i < 4; i++) buf[i] = static_cast<char>(ln >> (8 * i));
    crc = crc32c::Extend(crc, buf, 4);
  }
  const uint32_t payload_crc = crc32c::Value(payload, n);
  crc = crc32c::Crc32cCombine(crc, payload_crc, n);
  return crc32c::Mask(crc);
}

// include/rocksdb/options.h:383-420
enum class WALRecoveryMode : char {
  kTolerateCorruptedTailRecords = MCK_WAL_kTolerateCorruptedTailRecords,
  kAbsoluteConsistency = MCK_WAL_kAbsoluteConsistency,
  kPointInTimeRecovery = MCK_WAL_kPointInTimeRecovery,
  kSkipAnyCorruptedRecords = MCK_WAL_kSkipAnyCorruptedRecords,
};

// log::Reader::ReadRecord (db/log_reader.cc:69-321) as DBImpl::RecoverLogFiles
// drives it (db/db_impl/db_impl_open.cc:1204-1221: records until false, each
// with its XXH3 record_checksum), over the engine's one-pass recovery
// (mck_wal_recover): Recover() runs the device pass and the reader's walk for
// the whole log once; ReadRecord() then hands out the records in order, with
// the reporter's Corruption(bytes, status) calls made inside the ReadRecord
// call where the reference makes them (mck_wal_recovery_report_positions).
// A record is a view into the caller's host image (one fragment) or
// reassembled into *scratch (fragmented), as the reference returns it.
class RecoveryReader {
 public:
  class Reporter {  // log::Reader::Reporter (db/log_reader.h:41-48)
   public:
    virtual ~Reporter() {}
    virtual void Corruption(size_t bytes, const Status& status) = 0;
  };
  RecoveryReader(Reporter* reporter, uint64_t log_num) : reporter_(reporter), log_num_(log_num) {}
  ~RecoveryReader() { mck_wal_recovery_free(rec_); }
  RecoveryReader(const RecoveryReader&) = delete;
  void operator=(const RecoveryReader&) = delete;

  // The whole log: wal_host (the file's bytes) and the same nbytes at
  // wal_dev (device memory, readable 16 bytes past nbytes).
  Status Recover(const char* wal_host, const void* wal_dev, uint64_t nbytes, WALRecoveryMode mode,
                 mck_stream_t stream = nullptr) {
    mck_wal_recovery_free(rec_);
    rec_ = nullptr;
    host_ = wal_host;
    mode_ = mode;
    next_ = next_report_ = 0;
    int rc = mck_wal_recover(wal_host, wal_dev, nbytes, static_cast<uint32_t>(log_num_), static_cast<int>(mode),
                             stream, &rec_);
    if (rc) return FromRc(rc, "mck_wal_recover");
    mck_wal_read_out o{};
    o.struct_size = sizeof(o);
    if ((rc = mck_wal_recovery_read_out(rec_, &o))) return FromRc(rc, "mck_wal_recovery_read_out");
    frags_.resize(o.nfrags);
    roff_.resize(o.nrecords);
    rlen_.resize(o.nrecords);
    rfile_.resize(o.nrecords);
    reports_.resize(o.nreports);
    report_pos_.resize(o.nreports);
    o.frags = frags_.data();
    o.frag_cap = frags_.size();
    o.rec_offsets = roff_.data();
    o.rec_lengths = rlen_.data();
    o.rec_file_offsets = rfile_.data();
    o.rec_cap = roff_.size();
    o.reports = reports_.data();
    o.report_cap = reports_.size();
    if ((rc = mck_wal_recovery_read_out(rec_, &o))) return FromRc(rc, "mck_wal_recovery_read_out");
    if ((rc = mck_wal_recovery_report_positions(rec_, report_pos_.data(), report_pos_.size())))
      return FromRc(rc, "mck_wal_recovery_report_positions");
    if ((rc = mck_wal_recovery_get_info(rec_, &info_))) return FromRc(rc, "mck_wal_recovery_get_info");
    checksums_.assign(roff_.size(), 0);
    if (info_.has_checksums && (rc = mck_wal_recovery_checksums(rec_, checksums_.data(), checksums_.size())))
      return FromRc(rc, "mck_wal_recovery_checksums");
    return Status::OK();
  }

  // record_checksum: XXH3_64bits of the record (compressed logs: unset, the
  // reference hashes the decompressed record).  mode must be Recover()'s.
  bool ReadRecord(std::string_view* record, std::string* scratch,
                  WALRecoveryMode mode = WALRecoveryMode::kTolerateCorruptedTailRecords,
                  uint64_t* record_checksum = nullptr) {
    scratch->clear();
    *record = std::string_view();
    if (mode != mode_) throw std::invalid_argument("RecoveryReader: the recovery mode of Recover() is fixed");
    ForwardReports(next_);
    if (next_ >= roff_.size()) return false;
    const size_t r = next_++;
    size_t f = frag_idx_;
    while (f < frags_.size() && frags_[f].dst_off < roff_[r]) f++;
    size_t e = f;
    while (e < frags_.size() && (frags_[e].dst_off < roff_[r] + rlen_[r] || (e == f && rlen_[r] == 0))) e++;
    frag_idx_ = e;
    if (e - f == 1) {  // one fragment: a view of the image
      *record = std::string_view(host_ + frags_[f].src_off, frags_[f].length);
    } else {
      for (size_t k = f; k < e; k++) scratch->append(host_ + frags_[k].src_off, frags_[k].length);
      *record = std::string_view(*scratch);
    }
    last_record_offset_ = rfile_[r];
    if (record_checksum && info_.has_checksums) *record_checksum = checksums_[r];
    return true;
  }
  uint64_t LastRecordOffset() const { return last_record_offset_; }
  const mck_wal_recovery_info& info() const { return info_; }

 private:
  void ForwardReports(size_t upto) {
    for (; next_report_ < reports_.size() && report_pos_[next_report_] <= upto; next_report_++)
      if (reporter_)
        reporter_->Corruption(static_cast<size_t>(reports_[next_report_].bytes),
                              Status::Corruption(mck_wal_reason_string(reports_[next_report_].reason)));
  }
  Reporter* reporter_;
  uint64_t log_num_;
  const char* host_ = nullptr;
  WALRecoveryMode mode_ = WALRecoveryMode::kTolerateCorruptedTailRecords;
  mck_wal_recovery* rec_ = nullptr;
  mck_wal_recovery_info info_{};
  std::vector<mck_wal_fragment> frags_;
  std::vector<uint64_t> roff_, rfile_, checksums_, report_pos_;
  std::vector<uint32_t> rlen_;
  std::vector<mck_wal_report> reports_;
  size_t next_ = 0, next_report_ = 0, frag_idx_ = 0;
  uint64_t last_record_offset_ = 0;
};
}  // namespace log

// util/hash.h:45 NPHash64 / util/hash.cc:81 Hash64 -- XXPH3 on the GPU
// (DeviceError on failure, as above).
inline uint64_t NPHash64(const char* data, size_t n, uint64_t seed = 0) {
  uint64_t v = 0;
  const int rc = mck_np_hash64_r(data, n, seed, &v);
  return CheckedU64(rc, v, "NPHash64");
}
inline uint64_t Hash64(const char* data, size_t n, uint64_t seed = 0) { return NPHash64(data, n, seed); }

// db/kv_checksum.h ProtectionInfo64, flattened: one value type whose Protect*
// / Strip* / Update* steps XOR in the NPHash64 of a field with that field's
// seed (:84-88), exactly as the reference's template chain does.
class ProtectionInfo64 {
 public:
  static constexpr uint64_t kSeedK = 0, kSeedV = 0xD28AAD72F49BD50Bull, kSeedO = 0xA5155AE5E937AA16ull,
                            kSeedS = 0x77A00858DDD37F21ull, kSeedC = 0x4A2AB5CBD26F542Cull;
  ProtectionInfo64() = default;
  explicit ProtectionInfo64(uint64_t v) : val_(v) {}
  uint64_t GetVal() const { return val_; }
  // ProtectKV (:324) / ProtectKVO (:296) / StripKVO (:400)
  ProtectionInfo64 ProtectKV(const std::string& key, const std::string& value) const {
    return ProtectionInfo64(val_ ^ NPHash64(key.data(), key.size(), kSeedK) ^
                            NPHash64(value.data(), value.size(), kSeedV));
  }
  ProtectionInfo64 ProtectKVO(const std::string& key, const std::string& value, uint8_t op_type) const {
    const char t = static_cast<char>(op_type);
    return ProtectionInfo64(ProtectKV(key, value).val_ ^ NPHash64(&t, 1, kSeedO));
  }
  ProtectionInfo64 StripKVO(const std::string& key, const std::string& value, uint8_t op_type) const {
    return ProtectKVO(key, value, op_type);  // XOR is its own inverse
  }
  // ProtectS (:456) / StripS (:466), ProtectC (:432) / StripC (:442)
  ProtectionInfo64 ProtectS(uint64_t seqno) const {
    char b[8];
    for (int i = 0; i < 8; i++) b[i] = static_cast<char>(seqno >> (8 * i));
    return ProtectionInfo64(val_ ^ NPHash64(b, 8, kSeedS));
  }
  ProtectionInfo64 StripS(uint64_t seqno) const { return ProtectS(seqno); }
  ProtectionInfo64 ProtectC(uint32_t cf) const {
    char b[4];
    for (int i = 0; i < 4; i++) b[i] = static_cast<char>(cf >> (8 * i));
    return ProtectionInfo64(val_ ^ NPHash64(b, 4, kSeedC));
  }
  ProtectionInfo64 StripC(uint32_t cf) const { return ProtectC(cf); }
  // Encode / Verify (:80-121): the low `len` bytes, little-endian
  void Encode(uint8_t len, char* dst) const {
    for (int i = 0; i < len; i++) dst[i] = static_cast<char>(val_ >> (8 * i));
  }
  bool Verify(uint8_t len, const char* p) const {
    for (int i = 0; i < len; i++)
      if (static_cast<uint8_t>(p[i]) != static_cast<uint8_t>(val_ >> (8 * i))) return false;
    return true;
  }
  // GetStatus (:286-292)
  Status GetStatus() const { return val_ ? Status::Corruption("ProtectionInfo mismatch") : Status::OK(); }

 private:
  uint64_t val_ = 0;
};

// ---------------------------------------------------------------------------
// Whole-file checksums: include/rocksdb/file_checksum.h:23-90,
// util/file_checksum_helper.h:22-72.
constexpr char kUnknownFileChecksum[] = "";
constexpr char kUnknownFileChecksumFuncName[] = "Unknown";
constexpr char kStandardDbFileChecksumFuncName[] = "FileChecksumCrc32c";

struct FileChecksumGenContext {
  std::string file_name;
  std::string requested_checksum_func_name;
};

class FileChecksumGenerator {
 public:
  virtual ~FileChecksumGenerator() {}
  virtual void Update(const char* data, size_t n) = 0;
  virtual void Finalize() = 0;
  virtual std::string GetChecksum() const = 0;
  virtual const char* Name() const = 0;
};

// checksum_ = crc32c::Extend over every Update, from 0; Finalize stores it as
// 4 big-endian bytes.  Update() takes host bytes (inputs over 1 MiB go
// through the engine's long-span path); UpdateDevice() takes bytes already
// in device memory (mck_crc32c_long, no host copy).  Exceptions never escape
// (include/rocksdb/file_checksum.h:47-49) and a generator has no error
// channel: after a device error the generator is failed() and Finalize
// gives kUnknownFileChecksum (the file's checksum is then unknown, never
// wrong).
class FileChecksumGenCrc32c : public FileChecksumGenerator {
 public:
  explicit FileChecksumGenCrc32c(const FileChecksumGenContext& /*context*/) {}
  ~FileChecksumGenCrc32c() override;
  void Update(const char* data, size_t n) override {
    uint32_t v = 0;
    if (failed_ || mck_crc32c_extend_r(checksum_, data, n, &v) != MCK_OK) {
      failed_ = true;
      return;
    }
    checksum_ = v;
  }
  // Returns false (the generator failed, mck_last_error() set) on a HIP error.
  bool UpdateDevice(const void* dev_data, uint64_t n, mck_stream_t stream = nullptr);
  void Finalize() override {
    if (failed_) {
      checksum_str_ = kUnknownFileChecksum;
      return;
    }
    char b[4];
    for (int i = 0; i < 4; i++) b[i] = static_cast<char>(checksum_ >> (24 - 8 * i));
    checksum_str_.assign(b, 4);
  }
  bool failed() const { return failed_; }
  std::string GetChecksum() const override { return checksum_str_; }
  const char* Name() const override { return "FileChecksumCrc32c"; }

 private:
  uint32_t checksum_ = 0;
  bool failed_ = false;
  std::string checksum_str_;
  uint32_t* d_scratch_ = nullptr;  // device: long-span piece CRCs + result
  uint64_t scratch_words_ = 0;
};

class FileChecksumGenCrc32cFactory {
 public:
  std::unique_ptr<FileChecksumGenerator> CreateFileChecksumGenerator(const FileChecksumGenContext& context) {
    if (context.requested_checksum_func_name.empty() ||
        context.requested_checksum_func_name == "FileChecksumCrc32c")
      return std::unique_ptr<FileChecksumGenerator>(new FileChecksumGenCrc32c(context));
    return nullptr;
  }
  static const char* kClassName() { return "FileChecksumGenCrc32cFactory"; }
  const char* Name() const { return kClassName(); }
};

// ---------------------------------------------------------------------------
// Per-KV protection of block entries: table/block_based/block.cc:1091-1222
// Block::Initialize{Data,Index,MetaIndex}BlockProtectionInfo for a batch of
// uncompressed block contents (host bytes; staged to the device here).
// kind: MCK_BLOCK_DATA / _INDEX / _INDEX_DELTA / _INDEX_DELTA_FIRST_KEY /
// _META.  Per block: kv_checksum_ (num_keys * protection_bytes_per_key bytes,
// ProtectionInfo64().ProtectKV(key, value).Encode(n) per entry, block.h
// :271-274), the block's status ("bad block contents", "bad entry in block")
// and GetRestartInterval.
struct BlockKvChecksums {
  std::vector<std::string> kv_checksum;
  std::vector<Status> status;
  std::vector<uint32_t> restart_interval;
};
inline Status InitializeBlockProtectionInfo(int kind, const std::vector<std::string>& blocks,
                                            uint8_t protection_bytes_per_key, BlockKvChecksums* out,
                                            mck_stream_t stream = nullptr);

// ---------------------------------------------------------------------------
// inline definitions of the batched helpers (need HIP for device buffers)
// ---------------------------------------------------------------------------
}  // namespace speedb_amd

#include <hip/hip_runtime_api.h>

namespace speedb_amd {

inline Status VerifyBlockChecksums(const Footer& footer, const void* dev_image, uint64_t file_base,
                                   const std::vector<BlockHandle>& handles, const std::string& file_name,
                                   std::vector<Status>* per_block, mck_stream_t stream) {
  const uint32_t n = static_cast<uint32_t>(handles.size());
  if (per_block) per_block->assign(n, Status::OK());
  if (!n) return Status::OK();
  std::vector<uint64_t> offs(n), foffs(n);
  std::vector<uint32_t> lens(n);
  for (uint32_t i = 0; i < n; i++) {
    offs[i] = handles[i].offset - file_base;
    foffs[i] = handles[i].offset;
    lens[i] = static_cast<uint32_t>(handles[i].size);
  }
  uint64_t *d_off = nullptr, *d_foff = nullptr;
  uint32_t *d_len = nullptr, *d_comp = nullptr, *d_stored = nullptr, *d_cnt = nullptr;
  uint8_t* d_mm = nullptr;
  auto cleanup = [&] {
    (void)hipFree(d_off);
    (void)hipFree(d_foff);
    (void)hipFree(d_len);
    (void)hipFree(d_comp);
    (void)hipFree(d_stored);
    (void)hipFree(d_cnt);
    (void)hipFree(d_mm);
  };
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (hipMalloc(&d_off, n * 8) != hipSuccess || hipMalloc(&d_foff, n * 8) != hipSuccess ||
      hipMalloc(&d_len, n * 4) != hipSuccess || hipMalloc(&d_comp, n * 4) != hipSuccess ||
      hipMalloc(&d_stored, n * 4) != hipSuccess || hipMalloc(&d_cnt, 4) != hipSuccess ||
      hipMalloc(&d_mm, n) != hipSuccess) {
    cleanup();
    return Status::IOError("hipMalloc failed");
  }
  (void)hipMemcpyAsync(d_off, offs.data(), n * 8, hipMemcpyHostToDevice, st);
  (void)hipMemcpyAsync(d_foff, foffs.data(), n * 8, hipMemcpyHostToDevice, st);
  (void)hipMemcpyAsync(d_len, lens.data(), n * 4, hipMemcpyHostToDevice, st);
  (void)hipMemsetAsync(d_cnt, 0, 4, st);
  const mck_spans sp{dev_image, d_off, d_len, 0, 0, n};
  int rc = mck_sst_verify_batch(footer.checksum_type, &sp, d_foff, footer.base_context_checksum, d_mm, d_comp,
                                d_stored, d_cnt, stream);
  if (rc) {
    cleanup();
    return FromRc(rc, "mck_sst_verify_batch");
  }
  std::vector<uint8_t> mm(n);
  std::vector<uint32_t> comp(n), stored(n);
  (void)hipMemcpyAsync(mm.data(), d_mm, n, hipMemcpyDeviceToHost, st);
  (void)hipMemcpyAsync(comp.data(), d_comp, n * 4, hipMemcpyDeviceToHost, st);
  (void)hipMemcpyAsync(stored.data(), d_stored, n * 4, hipMemcpyDeviceToHost, st);
  const hipError_t e = hipStreamSynchronize(st);
  cleanup();
  if (e != hipSuccess) return Status::IOError(hipGetErrorString(e));
  Status first;
  for (uint32_t i = 0; i < n; i++) {
    if (!mm[i]) continue;
    const bool ctx = ChecksumModifierForContext(footer.base_context_checksum, handles[i].offset) != 0;
    Status s = BlockChecksumMismatch(footer.checksum_type, stored[i], comp[i], ctx, file_name, handles[i].offset,
                                     handles[i].size);
    if (first.ok()) first = s;
    if (per_block) (*per_block)[i] = s;
  }
  return first;
}

inline FileChecksumGenCrc32c::~FileChecksumGenCrc32c() {
  if (d_scratch_) (void)hipFree(d_scratch_);
}

inline bool FileChecksumGenCrc32c::UpdateDevice(const void* dev_data, uint64_t n, mck_stream_t stream) {
  if (failed_) return false;
  failed_ = true;  // until this update has completed
  const uint64_t need = mck_crc32c_long_scratch_words(n) + 1;  // + result word
  if (need > scratch_words_) {
    if (d_scratch_) (void)hipFree(d_scratch_);
    d_scratch_ = nullptr;
    scratch_words_ = 0;
    if (hipMalloc(&d_scratch_, need * 4) != hipSuccess) return false;
    scratch_words_ = need;
  }
  if (mck_crc32c_long(dev_data, n, checksum_, d_scratch_ + 1, d_scratch_, stream) != MCK_OK) return false;
  uint32_t v = 0;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (hipMemcpyAsync(&v, d_scratch_, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return false;
  checksum_ = v;
  failed_ = false;
  return true;
}

inline Status InitializeBlockProtectionInfo(int kind, const std::vector<std::string>& blocks,
                                            uint8_t protection_bytes_per_key, BlockKvChecksums* out,
                                            mck_stream_t stream) {
  const uint32_t n = static_cast<uint32_t>(blocks.size());
  out->kv_checksum.assign(n, std::string());
  out->status.assign(n, Status::OK());
  out->restart_interval.assign(n, 0);
  if (!n) return Status::OK();
  std::vector<uint64_t> offs(n);
  std::vector<uint32_t> lens(n);
  uint64_t total = 0;
  for (uint32_t i = 0; i < n; i++) {
    offs[i] = total;
    lens[i] = static_cast<uint32_t>(blocks[i].size());
    total += (blocks[i].size() + 15) & ~uint64_t(15);
  }
  std::string image(total + 64, '\0');
  for (uint32_t i = 0; i < n; i++) image.replace(offs[i], blocks[i].size(), blocks[i]);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  std::vector<void*> bufs;
  auto cleanup = [&] {
    for (void* b : bufs) (void)hipFree(b);
  };
  auto alloc = [&](size_t bytes) -> void* {
    void* p = nullptr;
    if (hipMalloc(&p, bytes ? bytes : 1) != hipSuccess) return nullptr;
    bufs.push_back(p);
    return p;
  };
  uint8_t* d_img = static_cast<uint8_t*>(alloc(image.size()));
  uint64_t* d_off = static_cast<uint64_t*>(alloc(n * 8));
  uint32_t* d_len = static_cast<uint32_t*>(alloc(n * 4));
  uint64_t* d_kb = static_cast<uint64_t*>(alloc((n + 1) * 8));
  uint64_t* d_ab = static_cast<uint64_t*>(alloc((n + 1) * 8));
  uint32_t* d_ri = static_cast<uint32_t*>(alloc(n * 4));
  int32_t* d_st = static_cast<int32_t*>(alloc(n * 4));
  void* d_scratch = alloc(mck_block_kv_scratch_bytes(n));
  if (!d_img || !d_off || !d_len || !d_kb || !d_ab || !d_ri || !d_st || !d_scratch) {
    cleanup();
    return Status::IOError("hipMalloc failed");
  }
  (void)hipMemcpyAsync(d_img, image.data(), image.size(), hipMemcpyHostToDevice, st);
  (void)hipMemcpyAsync(d_off, offs.data(), n * 8, hipMemcpyHostToDevice, st);
  (void)hipMemcpyAsync(d_len, lens.data(), n * 4, hipMemcpyHostToDevice, st);
  const mck_spans sp{d_img, d_off, d_len, 0, 0, n};
  int rc = mck_block_kv_layout_batch(kind, &sp, d_kb, d_ab, d_ri, d_st, d_scratch, stream);
  std::vector<uint64_t> kb(n + 1), ab(n + 1);
  std::vector<int32_t> sts(n);
  if (!rc) {
    (void)hipMemcpyAsync(kb.data(), d_kb, (n + 1) * 8, hipMemcpyDeviceToHost, st);
    (void)hipMemcpyAsync(ab.data(), d_ab, (n + 1) * 8, hipMemcpyDeviceToHost, st);
    (void)hipMemcpyAsync(sts.data(), d_st, n * 4, hipMemcpyDeviceToHost, st);
    (void)hipMemcpyAsync(out->restart_interval.data(), d_ri, n * 4, hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) rc = MCK_EHIP;
  }
  if (rc) {
    cleanup();
    return FromRc(rc, "mck_block_kv_layout_batch");
  }
  const uint64_t keys = kb[n], pb = protection_bytes_per_key;
  void* d_work = alloc(mck_block_kv_work_bytes(keys, ab[n]));
  uint8_t* d_out = static_cast<uint8_t*>(alloc(keys * pb));
  if (!d_work || !d_out) {
    cleanup();
    return Status::IOError("hipMalloc failed");
  }
  rc = mck_block_kv_protect_batch(kind, &sp, protection_bytes_per_key, d_kb, d_ab, d_ri, keys, d_work, d_out, stream);
  std::string all(keys * pb, '\0');
  if (!rc && keys) {
    (void)hipMemcpyAsync(&all[0], d_out, keys * pb, hipMemcpyDeviceToHost, st);
    if (hipStreamSynchronize(st) != hipSuccess) rc = MCK_EHIP;
  }
  cleanup();
  if (rc) return FromRc(rc, "mck_block_kv_protect_batch");
  Status first;
  for (uint32_t i = 0; i < n; i++) {
    out->kv_checksum[i] = all.substr(kb[i] * pb, (kb[i + 1] - kb[i]) * pb);
    if (sts[i] != MCK_BLOCK_OK) {
      out->status[i] = Status::Corruption(sts[i] == MCK_BLOCK_BAD_CONTENTS ? "bad block contents"
                                          : sts[i] == MCK_BLOCK_BAD_ENTRY  ? "bad entry in block"
                                                                           : "block restart layout not as written by BlockBuilder");
      if (first.ok()) first = out->status[i];
    }
  }
  return first;
}

inline Status VerifySstFile(const std::string& file_name, const char* image, uint64_t size,
                            std::vector<mck_sst_block>* blocks_out, mck_stream_t stream) {
  mck_sst_footer f;
  uint64_t n = 0;
  int rc = mck_sst_list_blocks(image, size, &f, nullptr, 0, &n);
  if (rc) return FromRc(rc, "mck_sst_list_blocks");
  std::vector<mck_sst_block> blocks(n);
  rc = mck_sst_list_blocks(image, size, &f, blocks.data(), n, &n);
  if (rc) return FromRc(rc, "mck_sst_list_blocks");
  rc = mck_sst_verify_footer(image + f.footer_offset, &f);
  if (rc) return FromRc(rc, "mck_sst_verify_footer");
  if (blocks_out) *blocks_out = blocks;
  void* d = nullptr;
  if (hipMalloc(&d, size + 64) != hipSuccess) return Status::IOError("hipMalloc failed");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (hipMemcpyAsync(d, image, size, hipMemcpyHostToDevice, st) != hipSuccess) {
    (void)hipFree(d);
    return Status::IOError("hipMemcpyAsync failed");
  }
  std::vector<BlockHandle> handles(n);
  for (uint64_t i = 0; i < n; i++) handles[i] = BlockHandle{blocks[i].offset, blocks[i].size};
  Footer footer;
  footer.checksum_type = static_cast<ChecksumType>(f.checksum_type);
  footer.base_context_checksum = f.base_context_checksum;
  Status s = VerifyBlockChecksums(footer, d, 0, handles, file_name, nullptr, stream);
  (void)hipFree(d);
  return s;
}

}  // namespace speedb_amd
