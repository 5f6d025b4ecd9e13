// mck_wal.cc -- host-side write plan of the device WAL writer: the
// fragmentation log::Writer::AddRecord performs (db/log_writer.cc:79-175),
// on sizes only.  The bytes are written on the device by
// mck_wal_write_batch (mck_engine.hip).
#include <stddef.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <thread>
#include <vector>

#include "../../include/speedb_amd/mck.h"
#include "mck_internal.h"
#include "mck_walk.h"

namespace {
// db/log_format.h:22-45
constexpr uint8_t kFullType = 1, kFirstType = 2, kMiddleType = 3, kLastType = 4;
constexpr uint8_t kRecyclableFullType = 5, kRecyclableFirstType = 6, kRecyclableMiddleType = 7,
                  kRecyclableLastType = 8;
}  // namespace

extern "C" int mck_wal_plan(const uint64_t* src_offsets, const uint32_t* lengths, uint32_t count,
                            uint32_t block_offset, int recycle, mck_wal_fragment* frags, uint64_t cap,
                            uint64_t* nfrags, uint64_t* out_bytes, uint32_t* new_block_offset) {
  mck_internal_set_error("");
  if ((count && (!src_offsets || !lengths)) || !nfrags) {
    mck_internal_set_error("NULL argument");
    return MCK_EINVAL;
  }
  const uint32_t kBlock = MCK_WAL_kBlockSize;
  const uint32_t hs = recycle ? MCK_WAL_kRecyclableHeaderSize : MCK_WAL_kHeaderSize;
  if (block_offset > kBlock) {
    mck_internal_set_error("block_offset > kBlockSize");
    return MCK_EINVAL;
  }
  uint64_t pos = 0, n = 0;  // output bytes written, fragments
  uint32_t boff = block_offset;
  for (uint32_t r = 0; r < count; r++) {
    uint64_t left = lengths[r], ptr = src_offsets[r];
    bool begin = true;
    do {  // an empty record still emits one zero-length physical record
      uint32_t pad = 0;
      const uint32_t leftover = kBlock - boff;
      if (leftover < hs) {  // switch to a new block; fill the trailer
        pad = leftover;
        pos += leftover;
        boff = 0;
      }
      const uint64_t avail = kBlock - boff - hs;
      const uint64_t frag = left < avail ? left : avail;
      const bool end = left == frag;
      uint8_t type;
      if (begin && end)
        type = recycle ? kRecyclableFullType : kFullType;
      else if (begin)
        type = recycle ? kRecyclableFirstType : kFirstType;
      else if (end)
        type = recycle ? kRecyclableLastType : kLastType;
      else
        type = recycle ? kRecyclableMiddleType : kMiddleType;
      if (frags) {
        if (n >= cap) {
          mck_internal_set_error("frags capacity too small");
          return MCK_EINVAL;
        }
        frags[n] = mck_wal_fragment{ptr, pos, (uint32_t)frag, type, (uint8_t)pad, 0};
      }
      n++;
      pos += hs + frag;
      boff += hs + (uint32_t)frag;
      ptr += frag;
      left -= frag;
      begin = false;
    } while (left > 0);
  }
  *nfrags = n;
  if (out_bytes) *out_bytes = pos;
  if (new_block_offset) *new_block_offset = boff;
  return MCK_OK;
}

// ---------------------------------------------------------------------------
// log::Reader (db/log_reader.cc) over a host WAL image, checksums supplied by
// the device: ReadRecord (:69-321) called until it returns false, on top of
// ReadPhysicalRecord (:450-584) and ReadMore (:400-448).  The reader reads the
// file in kBlockSize pieces from offset 0, so "the buffer" is the unread rest
// of the current 32 KiB block; a short last block sets eof_.  Every
// Reporter::Corruption call is recorded as (offset, bytes, reason).
// ---------------------------------------------------------------------------
namespace {

constexpr uint32_t kZeroType = 0, kSetCompressionType = 9, kUserDefinedTimestampSizeType = 10,
                   kRecyclableUserDefinedTimestampSizeType = 11;
// ReadPhysicalRecord's extra results (db/log_reader.h:136-156)
constexpr int kEof = 12, kBadRecord = 13, kBadHeader = 14, kOldRecord = 15, kBadRecordLen = 16,
              kBadRecordChecksum = 17;

// header[6] as the reference reads it: `const unsigned int type = header[6]`
// with a (signed) char header, so bytes >= 128 sign-extend.
inline uint32_t header_type(const uint8_t* h) { return (uint32_t)(int32_t)(int8_t)h[6]; }
inline int unknown_type_reason(uint32_t type) { return MCK_WAL_R_UNKNOWN_TYPE_BASE + (int)(type & 255); }

// Reader::UpdateRecordedTimestampSize (db/log_reader.cc:594-616) over a
// decoded UserDefinedTimestampSizeRecord (util/udt_util.h:46-65: [cf LE32,
// ts size LE16] pairs): the first entry with a zero size, or for a column
// family already recorded in this log, is the corruption reported.
struct TsRecorder {
  std::vector<uint32_t> cfs;
  // 0 = OK, else the MCK_WAL_R_* reason
  int update(const uint8_t* p, uint32_t n) {
    for (uint32_t o = 0; o + 6 <= n; o += 6) {
      const uint32_t cf = (uint32_t)p[o] | ((uint32_t)p[o + 1] << 8) | ((uint32_t)p[o + 2] << 16) |
                          ((uint32_t)p[o + 3] << 24);
      const uint32_t ts = (uint32_t)p[o + 4] | ((uint32_t)p[o + 5] << 8);
      if (ts == 0) return MCK_WAL_R_TS_ZERO_SIZE;
      if (std::find(cfs.begin(), cfs.end(), cf) != cfs.end()) return MCK_WAL_R_TS_CF_UPDATE;
      cfs.push_back(cf);
    }
    return 0;
  }
};

struct WalReader {
  const uint8_t* d;
  uint64_t nbytes;
  uint32_t log_number;
  int mode;
  const mck_wal_block_result* verified;
  // buffer_ = [buf_off, buf_off + buf_size) of the file
  uint64_t buf_off = 0, buf_size = 0, end_of_buffer_offset = 0;
  bool eof = false, recycled = false, first_record_read = false;
  int err = MCK_OK;
  std::vector<mck_wal_report> reports;
  uint64_t dropped = 0;

  void report(uint64_t off, uint64_t bytes, int reason) {
    reports.push_back(mck_wal_report{off, bytes, reason, 0});
    if (records_so_far) report_pos.push_back(records_so_far->size());
    dropped += bytes;
  }
  // per report: the records returned before it (the ReadRecord call that
  // reported it returns record report_pos[i], or false at the end)
  const std::vector<uint64_t>* records_so_far = nullptr;
  std::vector<uint64_t> report_pos;
  bool strict() const {  // kAbsoluteConsistency / kPointInTimeRecovery
    return mode == MCK_WAL_kAbsoluteConsistency || mode == MCK_WAL_kPointInTimeRecovery;
  }

  // :400-448 ReadMore
  bool read_more(uint64_t* drop_size, int* error) {
    if (!eof) {
      const uint64_t n = std::min<uint64_t>(MCK_WAL_kBlockSize, nbytes - end_of_buffer_offset);
      buf_off = end_of_buffer_offset;
      buf_size = n;
      end_of_buffer_offset += n;
      if (n < MCK_WAL_kBlockSize) eof = true;
      return true;
    }
    if (buf_size) {  // a truncated header at the end of the file
      *drop_size = buf_size;
      buf_size = 0;
      *error = kBadHeader;
      return false;
    }
    *error = kEof;
    return false;
  }

  // the device's verdict on the record whose header is at file offset h
  bool crc_ok(uint64_t h) {
    if (!verified) return true;
    const mck_wal_block_result& r = verified[h / MCK_WAL_kBlockSize];
    const uint32_t o = (uint32_t)(h % MCK_WAL_kBlockSize);
    if (o < r.stop_offset) return true;
    if (o == r.stop_offset && r.status == MCK_WAL_BAD_CHECKSUM) return false;
    err = MCK_EINVAL;  // the results are not this image's
    return false;
  }

  // :450-584 ReadPhysicalRecord; *frag = (file offset, length) of the payload
  int read_physical(uint64_t* frag_off, uint32_t* frag_len, uint64_t* drop_size) {
    for (;;) {
      if (buf_size < MCK_WAL_kHeaderSize) {
        int r = kEof;
        if (!read_more(drop_size, &r)) return r;
        continue;
      }
      if (phys && !phys->empty()) {  // the headers ahead are known: fetch them while this one is parsed
        while (pcur + 1 < phys->size() && (*phys)[pcur].hoff < buf_off) pcur++;
        __builtin_prefetch(d + (*phys)[std::min<size_t>(pcur + 16, phys->size() - 1)].hoff);
      }
      const uint8_t* h = d + buf_off;
      const uint32_t length = (uint32_t)h[4] | ((uint32_t)h[5] << 8);
      const uint32_t type = header_type(h);
      uint32_t hs = MCK_WAL_kHeaderSize;
      if ((type >= 5 && type <= 8) || type == kRecyclableUserDefinedTimestampSizeType) {
        if (end_of_buffer_offset - buf_size == 0) recycled = true;
        hs = MCK_WAL_kRecyclableHeaderSize;
        if (buf_size < hs) {
          int r = kEof;
          if (!read_more(drop_size, &r)) return r;
          continue;
        }
        const uint32_t ln = (uint32_t)h[7] | ((uint32_t)h[8] << 8) | ((uint32_t)h[9] << 16) | ((uint32_t)h[10] << 24);
        if (ln != log_number) return kOldRecord;
      }
      if (hs + (uint64_t)length > buf_size) {
        *drop_size = buf_size;
        buf_size = 0;
        return kBadRecordLen;
      }
      if (type == kZeroType && length == 0) {
        buf_size = 0;
        return kBadRecord;
      }
      if (!crc_ok(buf_off)) {
        *drop_size = buf_size;
        buf_size = 0;
        return kBadRecordChecksum;
      }
      last_hoff = buf_off;  // (mck_wal_recover: the record's physical record)
      *frag_off = buf_off + hs;
      *frag_len = length;
      buf_off += hs + length;
      buf_size -= hs + length;
      read_ok = true;  // (a type byte may equal one of the error codes above)
      return (int)type;
    }
  }
  bool read_ok = false;  // the last read_physical returned a record
  uint64_t last_hoff = 0;  // header offset of the last record read_physical returned
  // the block walk's records (optional): their headers are prefetched ahead
  const std::vector<mck_walk::PhysRec>* phys = nullptr;
  size_t pcur = 0;
};

}  // namespace

extern "C" const char* mck_wal_reason_string(int reason) {
  switch (reason) {
    case MCK_WAL_R_CHECKSUM_MISMATCH: return "checksum mismatch";
    case MCK_WAL_R_BAD_RECORD_LENGTH: return "bad record length";
    case MCK_WAL_R_TRUNCATED_HEADER: return "truncated header";
    case MCK_WAL_R_TRUNCATED_BODY: return "truncated record body";
    case MCK_WAL_R_ERROR_IN_MIDDLE: return "error in middle of record";
    case MCK_WAL_R_MISSING_START_1: return "missing start of fragmented record(1)";
    case MCK_WAL_R_MISSING_START_2: return "missing start of fragmented record(2)";
    case MCK_WAL_R_PARTIAL_WITHOUT_END_1: return "partial record without end(1)";
    case MCK_WAL_R_PARTIAL_WITHOUT_END_2: return "partial record without end(2)";
    case MCK_WAL_R_TRAILING_DATA: return "error reading trailing data";
    case MCK_WAL_R_TS_INTERSPERSED: return "user-defined timestamp size record interspersed partial record";
    case MCK_WAL_R_TS_DECODE: return "could not decode user-defined timestamp size record";
    case MCK_WAL_R_TS_ZERO_SIZE: return "User-defined timestamp size record contains zero timestamp size.";
    case MCK_WAL_R_TS_CF_UPDATE:
      return "User-defined timestamp size record contains update to recorded column family.";
    case MCK_WAL_R_COMPRESSION_MULTIPLE: return "read multiple SetCompressionType records";
    case MCK_WAL_R_COMPRESSION_NOT_FIRST: return "SetCompressionType not the first record";
    case MCK_WAL_R_COMPRESSION_DECODE: return "could not decode SetCompressionType record";
    default:
      if (reason >= MCK_WAL_R_UNKNOWN_TYPE_BASE && reason < MCK_WAL_R_UNKNOWN_TYPE_BASE + 256) {
        static thread_local char buf[40];
        const uint8_t b = (uint8_t)(reason - MCK_WAL_R_UNKNOWN_TYPE_BASE);
        snprintf(buf, sizeof buf, "unknown record type %u", (unsigned)(int)(int8_t)b);
        return buf;
      }
      return "";
  }
}

namespace mck_walk {
// log::Reader (checksum = true) reading the whole image: ReadRecord until it
// returns false, over the device's verdicts (NULL = trust every CRC).
int wal_walk(const uint8_t* d, uint64_t nbytes, uint32_t log_number, int recovery_mode,
             const mck_wal_block_result* verified, WalWalk& W, const std::vector<PhysRec>* phys) {
  WalReader R{d, nbytes, log_number, recovery_mode, verified};
  R.records_so_far = &W.roff;
  R.phys = phys;
  if (phys) {  // about one record per physical record
    W.fr.reserve(phys->size());
    W.roff.reserve(phys->size());
    W.rlen.reserve(phys->size());
    W.rfile.reserve(phys->size());
    W.rhoff.reserve(phys->size());
    W.rfrag.reserve(phys->size() + 1);
  }
  TsRecorder ts;
  std::vector<mck_wal_fragment>& fr = W.fr;
  std::vector<uint64_t>& roff = W.roff;
  std::vector<uint64_t>& rfile = W.rfile;
  std::vector<uint32_t>& rlen = W.rlen;
  uint64_t dst = 0;             // end of the reassembled buffer
  uint64_t cur_start = 0;       // dst offset of scratch (the record being assembled)
  uint64_t cur_file = 0;        // file offset of its first physical record
  size_t cur_first_frag = 0;    // its first fragment in fr
  bool in_fragmented_record = false;
  // WAL compression: the chunks fed to StreamingUncompress, in order, and per
  // fragment of fr the stream entry it came from
  uint32_t compression = 0;
  bool compression_read = false;
  std::vector<mck_wal_fragment>& stream = W.stream;
  std::vector<uint64_t> fr_sidx;
  auto feed = [&](uint64_t off, uint32_t len, uint32_t type) {
    if (compression) stream.push_back(mck_wal_fragment{off, ~0ull, len, (uint8_t)type, 0, 0});
  };
  auto scratch_size = [&] { return dst - cur_start; };
  auto scratch_clear = [&] {  // scratch->clear(): its fragments are dropped
    fr.resize(cur_first_frag);
    fr_sidx.resize(cur_first_frag);
    dst = cur_start;
  };
  auto scratch_append = [&](uint64_t off, uint32_t len, uint8_t type) {
    fr.push_back(mck_wal_fragment{off, dst, len, type, 0, 0});
    fr_sidx.push_back(compression ? stream.size() - 1 : ~0ull);  // the chunk just fed
    dst += len;
  };
  auto scratch_assign = [&](uint64_t off, uint32_t len, uint8_t type, uint64_t file_off) {
    scratch_clear();
    cur_first_frag = fr.size();
    cur_file = file_off;
    scratch_append(off, len, type);
  };
  auto emit = [&](uint64_t hoff) {  // ReadRecord returns *record = scratch
    for (size_t j = cur_first_frag; j < fr.size(); j++)
      if (fr_sidx[j] != ~0ull) stream[fr_sidx[j]].dst_off = j;
    roff.push_back(cur_start);
    rlen.push_back((uint32_t)(dst - cur_start));
    rfile.push_back(cur_file);
    W.rhoff.push_back(hoff);
    W.rfrag.push_back(cur_first_frag);
    cur_start = dst;
    cur_first_frag = fr.size();
    R.first_record_read = true;
  };
  // ReadRecord, called until it returns false (the whole log)
  bool more = true;
  while (more && R.err == MCK_OK) {
    in_fragmented_record = false;
    scratch_clear();
    for (;;) {
      const uint64_t phys = R.end_of_buffer_offset - R.buf_size;
      uint64_t drop_size = 0, foff = 0;
      uint32_t flen = 0;
      R.read_ok = false;
      const int t = R.read_physical(&foff, &flen, &drop_size);
      if (R.err) break;
      // ReadPhysicalRecord feeds every record it returns (but the
      // compression and timestamp-size records) to the uncompressor
      if (R.read_ok && t != (int)kSetCompressionType && t != (int)kUserDefinedTimestampSizeType &&
          t != (int)kRecyclableUserDefinedTimestampSizeType)
        feed(foff, flen, (uint32_t)t);
      if (t == 1 || t == 5) {  // kFullType
        if (in_fragmented_record && scratch_size()) R.report(phys, scratch_size(), MCK_WAL_R_PARTIAL_WITHOUT_END_1);
        scratch_assign(foff, flen, (uint8_t)t, phys);
        emit(R.last_hoff);
        break;
      } else if (t == 2 || t == 6) {  // kFirstType
        if (in_fragmented_record && scratch_size()) R.report(phys, scratch_size(), MCK_WAL_R_PARTIAL_WITHOUT_END_2);
        scratch_assign(foff, flen, (uint8_t)t, phys);
        in_fragmented_record = true;
      } else if (t == 3 || t == 7) {  // kMiddleType
        if (!in_fragmented_record)
          R.report(phys, flen, MCK_WAL_R_MISSING_START_1);
        else
          scratch_append(foff, flen, (uint8_t)t);
      } else if (t == 4 || t == 8) {  // kLastType
        if (!in_fragmented_record) {
          R.report(phys, flen, MCK_WAL_R_MISSING_START_2);
        } else {
          scratch_append(foff, flen, (uint8_t)t);
          emit(~0ull);
          break;
        }
      } else if (t == (int)kSetCompressionType) {  // :167-188
        if (compression_read) R.report(phys, flen, MCK_WAL_R_COMPRESSION_MULTIPLE);
        if (R.first_record_read) R.report(phys, flen, MCK_WAL_R_COMPRESSION_NOT_FIRST);
        cur_file = phys;
        scratch_clear();
        // CompressionTypeRecord::DecodeFrom (util/compression.h:1710-1725):
        // LE32, a streaming-capable type (kNoCompression or kZSTD)
        const uint8_t* p = R.d + foff;
        const uint32_t ct = flen >= 4 ? (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
                                            ((uint32_t)p[3] << 24)
                                      : 0xFFFFFFFFu;
        if (ct != 0 && ct != 7) {
          R.report(phys, flen, MCK_WAL_R_COMPRESSION_DECODE);
        } else {
          compression_read = true;   // InitCompression (:590-600)
          compression = ct;          // kNoCompression: no uncompressor
        }
      } else if (t == (int)kUserDefinedTimestampSizeType || t == (int)kRecyclableUserDefinedTimestampSizeType) {
        if (in_fragmented_record && scratch_size()) R.report(phys, scratch_size(), MCK_WAL_R_TS_INTERSPERSED);
        // prospective_record_offset = last_record_offset_ = this record's
        // offset: a record it interrupted and that then completes reports it
        cur_file = phys;
        scratch_clear();
        if (flen % 6) {
          R.report(phys, flen, MCK_WAL_R_TS_DECODE);  // util/udt_util.h:46-64
        } else if (const int why = ts.update(R.d + foff, flen)) {
          R.report(phys, flen, why);
        }
      } else if (t == kBadHeader || t == kEof) {
        if (t == kBadHeader && R.strict()) R.report(phys, drop_size, MCK_WAL_R_TRUNCATED_HEADER);
        if (in_fragmented_record) {
          if (R.strict()) R.report(phys, scratch_size(), MCK_WAL_R_TRAILING_DATA);
          scratch_clear();
        }
        more = false;
        break;
      } else if (t == kOldRecord && R.mode != MCK_WAL_kSkipAnyCorruptedRecords) {
        if (in_fragmented_record) {
          if (R.strict()) R.report(phys, scratch_size(), MCK_WAL_R_TRAILING_DATA);
          scratch_clear();
        }
        more = false;
        break;
      } else if (t == kOldRecord || t == kBadRecord) {
        // kSkipAnyCorruptedRecords: an old record is skipped like a bad one.
        // (The reference then re-parses the same header forever: its buffer
        // is not advanced on kOldRecord; the walk ends here instead.)
        if (in_fragmented_record) {
          R.report(phys, scratch_size(), MCK_WAL_R_ERROR_IN_MIDDLE);
          in_fragmented_record = false;
          scratch_clear();
        }
        if (t == kOldRecord) {
          more = false;
          break;
        }
      } else if (t == kBadRecordLen && R.eof) {
        if (R.strict()) R.report(phys, drop_size, MCK_WAL_R_TRUNCATED_BODY);
        more = false;
        break;
      } else if (t == kBadRecordLen || t == kBadRecordChecksum) {
        if (R.recycled && R.mode == MCK_WAL_kTolerateCorruptedTailRecords) {
          scratch_clear();
          more = false;
          break;
        }
        R.report(phys, drop_size, t == kBadRecordLen ? MCK_WAL_R_BAD_RECORD_LENGTH : MCK_WAL_R_CHECKSUM_MISMATCH);
        if (in_fragmented_record) {
          R.report(phys, scratch_size(), MCK_WAL_R_ERROR_IN_MIDDLE);
          in_fragmented_record = false;
          scratch_clear();
        }
      } else {  // unknown record type
        R.report(phys, flen + (in_fragmented_record ? scratch_size() : 0), unknown_type_reason((uint32_t)t));
        in_fragmented_record = false;
        scratch_clear();
      }
    }
  }
  if (R.err) return R.err;
  scratch_clear();
  W.rfrag.push_back(fr.size());
  W.records_bytes = dst;
  W.reports = std::move(R.reports);
  W.report_pos = std::move(R.report_pos);
  W.dropped = R.dropped;
  W.end_offset = R.end_of_buffer_offset - R.buf_size;
  W.compression = compression;
  return MCK_OK;
}

// ReadRecord over a log the block walk fully describes (mck_walk.h): the
// reader then visits exactly the listed physical records, in order -- a
// block's rest under 7 bytes (or a recyclable header's 11) is the trailer
// ReadMore skips, and every block ended there -- so the state machine of
// wal_walk runs over the list: kFullType returns its fragment, kFirstType ..
// kLastType reassemble.  Anything that would make the reader report, drop or
// stop early (a block stopped for a bad length, an old or zero record, a
// truncated header at the end of the file; a middle or last fragment without
// a first, a full or first one inside a fragmented record, a record left
// open at the end; compression, timestamp-size or unknown types) declines.
// (The reader's walk re-read every header from the image, one cache miss
// per record: 172-209 ns per record on 2M 100-4096-byte records, against
// the list's sequential read; microbench/walk_time.cc.)
bool wal_walk_fast(uint64_t nbytes, const std::vector<PhysRec>& phys, const std::vector<BlockStop>& stops,
                   WalWalk& W) {
  for (const BlockStop& b : stops)
    if (b.status != MCK_WAL_OK) return false;
  bool infrag = false;
  for (const PhysRec& p : phys) {  // the order check first: W is left untouched on a decline
    const uint32_t t = p.type;
    if (t == 1 || t == 5 || t == 2 || t == 6) {
      if (infrag) return false;
      infrag = t == 2 || t == 6;
    } else if (t == 3 || t == 7) {
      if (!infrag) return false;
    } else if (t == 4 || t == 8) {
      if (!infrag) return false;
      infrag = false;
    } else {
      return false;
    }
  }
  if (infrag) return false;
  // the fill runs in parallel over ranges of the list that start at a full
  // or first fragment (its page faults and stores spread over threads):
  // pass 1 counts each range's records and bytes, pass 2 writes at the
  // prefix sums
  const size_t np = phys.size();
  const uint64_t hw = std::max<unsigned>(1u, std::thread::hardware_concurrency());
  const size_t T = (size_t)std::min<uint64_t>(std::min<uint64_t>(hw, 16), np / 65536 + 1);
  std::vector<size_t> cut(T + 1, np);
  cut[0] = 0;
  for (size_t k = 1; k < T; k++) {
    size_t j = std::max(cut[k - 1], np * k / T);
    while (j < np && !(phys[j].type == 1 || phys[j].type == 5 || phys[j].type == 2 || phys[j].type == 6)) j++;
    cut[k] = j;
  }
  std::vector<size_t> rbase(T + 1, 0);
  std::vector<uint64_t> bbase(T + 1, 0);
  auto par = [&](auto&& fn) {
    if (T == 1) return fn(0);
    std::vector<std::thread> th;
    for (size_t k = 0; k < T; k++) th.emplace_back([&, k] { fn(k); });
    for (auto& x : th) x.join();
  };
  par([&](size_t k) {
    size_t n = 0;
    uint64_t by = 0;
    for (size_t j = cut[k]; j < cut[k + 1]; j++) {
      const uint32_t t = phys[j].type;
      n += t == 1 || t == 5 || t == 4 || t == 8;
      by += phys[j].length;
    }
    rbase[k + 1] = n;
    bbase[k + 1] = by;
  });
  for (size_t k = 0; k < T; k++) {
    rbase[k + 1] += rbase[k];
    bbase[k + 1] += bbase[k];
  }
  const size_t nrec = rbase[T];
  W = WalWalk{};
  W.fr.resize(np);
  W.roff.resize(nrec);
  W.rlen.resize(nrec);
  W.rfile.resize(nrec);
  W.rhoff.resize(nrec);
  W.rfrag.resize(nrec + 1);
  par([&](size_t k) {
    uint64_t dst = bbase[k], cur_start = dst, cur_file = 0;
    size_t first = cut[k], r = rbase[k];
    // the reader's record offset is where the buffer stood before the
    // record's first fragment was read: the previous record's end, which
    // precedes a block's trailer (db/log_reader.cc:98 physical_record_offset)
    uint64_t prev_end = cut[k] ? phys[cut[k] - 1].hoff + phys[cut[k] - 1].hsize + phys[cut[k] - 1].length : 0;
    for (size_t j = cut[k]; j < cut[k + 1]; j++) {
      const PhysRec& p = phys[j];
      const uint32_t t = p.type;
      W.fr[j] = mck_wal_fragment{p.hoff + p.hsize, dst, p.length, (uint8_t)t, 0, 0};
      if (t == 1 || t == 5 || t == 2 || t == 6) {
        cur_start = dst;
        cur_file = prev_end;
        first = j;
      }
      prev_end = p.hoff + p.hsize + p.length;
      dst += p.length;
      if (t == 1 || t == 5 || t == 4 || t == 8) {
        W.roff[r] = cur_start;
        W.rlen[r] = (uint32_t)(dst - cur_start);
        W.rfile[r] = cur_file;
        W.rhoff[r] = (t == 1 || t == 5) ? p.hoff : ~0ull;
        W.rfrag[r] = first;
        r++;
      }
    }
  });
  const uint64_t dst = bbase[T];
  W.rfrag[nrec] = phys.size();
  W.records_bytes = dst;
  W.end_offset = nbytes;
  return true;
}

// mck_wal_read_out (caller arrays, *_cap sizes) from a walk
int wal_copy_out(const WalWalk& W, mck_wal_read_out* out) {
  const bool has_stream = out->struct_size >= sizeof(mck_wal_read_out);
  if (W.compression && !has_stream) {
    mck_internal_set_error("compressed WAL: mck_wal_read_out.struct_size has no room for the compression fields");
    return MCK_ENOTSUP;
  }
  out->nfrags = W.fr.size();
  out->nrecords = W.roff.size();
  out->records_bytes = W.records_bytes;
  out->nreports = W.reports.size();
  out->dropped_bytes = W.dropped;
  out->end_offset = W.end_offset;
  if (out->frags) {
    if (out->frag_cap < W.fr.size()) {
      mck_internal_set_error("frags capacity too small");
      return MCK_EINVAL;
    }
    if (!W.fr.empty()) memcpy(out->frags, W.fr.data(), W.fr.size() * sizeof(mck_wal_fragment));
  }
  if (out->rec_offsets || out->rec_lengths || out->rec_file_offsets) {
    if (out->rec_cap < W.roff.size()) {
      mck_internal_set_error("records capacity too small");
      return MCK_EINVAL;
    }
    if (!W.roff.empty()) {
      if (out->rec_offsets) memcpy(out->rec_offsets, W.roff.data(), W.roff.size() * 8);
      if (out->rec_lengths) memcpy(out->rec_lengths, W.rlen.data(), W.rlen.size() * 4);
      if (out->rec_file_offsets) memcpy(out->rec_file_offsets, W.rfile.data(), W.rfile.size() * 8);
    }
  }
  if (out->reports) {
    const size_t n = std::min<size_t>(out->report_cap, W.reports.size());
    if (n) memcpy(out->reports, W.reports.data(), n * sizeof(mck_wal_report));
  }
  if (!has_stream) return MCK_OK;
  out->compression_type = W.compression;
  out->nstream = W.stream.size();
  if (out->stream) {
    if (out->stream_cap < W.stream.size()) {
      mck_internal_set_error("stream capacity too small");
      return MCK_EINVAL;
    }
    if (!W.stream.empty()) memcpy(out->stream, W.stream.data(), W.stream.size() * sizeof(mck_wal_fragment));
  }
  return MCK_OK;
}

int check_read_args(const void* wal, uint64_t nbytes, int recovery_mode, const mck_wal_read_out* out) {
  if ((!wal && nbytes) || !out) {
    mck_internal_set_error("wal / out is NULL");
    return MCK_EINVAL;
  }
  static_assert(offsetof(mck_wal_read_out, compression_type) == MCK_WAL_READ_OUT_V1_SIZE, "v1 layout");
  if (out->struct_size != MCK_WAL_READ_OUT_V1_SIZE && out->struct_size != sizeof(mck_wal_read_out)) {
    // a struct of another (older or unknown) layout -- e.g. one built before
    // struct_size became the first field -- is refused, never written
    mck_internal_set_error("mck_wal_read_out.struct_size is neither MCK_WAL_READ_OUT_V1_SIZE nor sizeof(mck_wal_read_out)");
    return MCK_EINVAL;
  }
  if (recovery_mode < MCK_WAL_kTolerateCorruptedTailRecords || recovery_mode > MCK_WAL_kSkipAnyCorruptedRecords) {
    mck_internal_set_error("unknown WALRecoveryMode");
    return MCK_EINVAL;
  }
  return MCK_OK;
}
// k_wal_verify's per-block walk (mck_kernels.hpp wal_parse) on the host,
// without the CRCs: a < 7-byte rest is the block trailer (at the end of the
// file: a truncated header), a recyclable header needs 11 bytes, a record of
// another log, a length past the block and a zero-length kZeroType stop it.
namespace {
// Blocks [b0, b1) of the walk into phys / stops[b0 .. b1) (stops[b].first
// relative to this range's first record).
void block_walk_range(const uint8_t* d, uint64_t nbytes, uint32_t log_number, uint64_t b0, uint64_t b1,
                      std::vector<PhysRec>& phys, BlockStop* stops) {
  phys.reserve(phys.size() + (b1 - b0));
  for (uint64_t b = b0; b < b1; b++) {
    const uint64_t base = b * MCK_WAL_kBlockSize;
    const uint32_t size = (uint32_t)std::min<uint64_t>(MCK_WAL_kBlockSize, nbytes - base);
    const bool last = nbytes - base <= MCK_WAL_kBlockSize;
    BlockStop& st = stops[b];
    st.first = phys.size();
    st.status = MCK_WAL_OK;
    uint32_t pos = 0;
    for (;;) {
      const uint32_t left = size - pos;
      const uint8_t* h = d + base + pos;
      if (left < MCK_WAL_kHeaderSize) {
        if (last && left > 0) st.status = MCK_WAL_BAD_HEADER;
        break;
      }
      const uint32_t length = (uint32_t)h[4] | ((uint32_t)h[5] << 8);
      const uint32_t type = h[6];
      uint32_t hs = MCK_WAL_kHeaderSize;
      if ((type >= 5 && type <= 8) || type == 11) {
        hs = MCK_WAL_kRecyclableHeaderSize;
        if (left < hs) {
          if (last) st.status = MCK_WAL_BAD_HEADER;
          break;
        }
        const uint32_t ln = (uint32_t)h[7] | ((uint32_t)h[8] << 8) | ((uint32_t)h[9] << 16) | ((uint32_t)h[10] << 24);
        if (ln != log_number) {
          st.status = MCK_WAL_OLD_RECORD;
          break;
        }
      }
      if (hs + length > left) {
        st.status = MCK_WAL_BAD_LENGTH;
        break;
      }
      if (type == 0 && length == 0) {
        st.status = MCK_WAL_ZERO_RECORD;
        break;
      }
      const uint32_t stored = (uint32_t)h[0] | ((uint32_t)h[1] << 8) | ((uint32_t)h[2] << 16) | ((uint32_t)h[3] << 24);
      phys.push_back(PhysRec{base + pos, length, (uint8_t)hs, (uint8_t)type, stored});
      pos += hs + length;
    }
    st.count = (uint32_t)(phys.size() - st.first);
    st.pos = pos;
  }
}
}  // namespace

// k_wal_verify's per-block walk (mck_kernels.hpp wal_parse) on the host,
// without the CRCs: a < 7-byte rest is the block trailer (at the end of the
// file: a truncated header), a recyclable header needs 11 bytes, a record of
// another log, a length past the block and a zero-length kZeroType stop it.
// Blocks are independent: a large log is walked by several threads (each
// header is a cache miss one hop after the last -- the walk is memory-latency
// bound, not compute bound), their lists concatenated in file order.
void wal_block_walk(const uint8_t* d, uint64_t nbytes, uint32_t log_number, std::vector<PhysRec>& phys,
                    std::vector<BlockStop>& stops) {
  const uint64_t nb = (nbytes + MCK_WAL_kBlockSize - 1) / MCK_WAL_kBlockSize;
  stops.resize(nb);
  const uint64_t hw = std::max<unsigned>(1u, std::thread::hardware_concurrency());
  const uint64_t T = std::min<uint64_t>(std::min<uint64_t>(hw, 16), nb / 256 + 1);
  if (T <= 1) {
    phys.clear();
    block_walk_range(d, nbytes, log_number, 0, nb, phys, stops.data());
    return;
  }
  std::vector<std::vector<PhysRec>> part(T);
  std::vector<std::thread> th;
  for (uint64_t t = 0; t < T; t++)
    th.emplace_back([&, t] { block_walk_range(d, nbytes, log_number, nb * t / T, nb * (t + 1) / T, part[t], stops.data()); });
  for (auto& x : th) x.join();
  uint64_t total = 0;
  for (const auto& p : part) total += p.size();
  phys.clear();
  phys.reserve(total);
  for (uint64_t t = 0; t < T; t++) {
    const uint64_t off = phys.size();
    for (uint64_t b = nb * t / T; b < nb * (t + 1) / T; b++) stops[b].first += off;
    phys.insert(phys.end(), part[t].begin(), part[t].end());
  }
}

}  // namespace mck_walk

using namespace mck_walk;

extern "C" int mck_wal_plan_records(const void* wal, uint64_t nbytes, uint32_t log_number, mck_wal_rec_desc* out,
                                    uint64_t cap, uint64_t* count) {
  mck_internal_set_error("");
  if ((!wal && nbytes) || !count) {
    mck_internal_set_error("wal / count is NULL");
    return MCK_EINVAL;
  }
  if (nbytes >> 48) {
    mck_internal_set_error("WAL image too large (payload offsets are 48-bit)");
    return MCK_EINVAL;
  }
  std::vector<PhysRec> phys;
  std::vector<BlockStop> stops;
  wal_block_walk(static_cast<const uint8_t*>(wal), nbytes, log_number, phys, stops);
  *count = phys.size();
  if (!out) return MCK_OK;
  if (cap < phys.size()) {
    mck_internal_set_error("out capacity too small");
    return MCK_EINVAL;
  }
  for (size_t i = 0; i < phys.size(); i++) {
    const PhysRec& p = phys[i];
    const uint64_t po = p.hoff + p.hsize;
    const bool full = p.type == 1 || p.type == 5;
    out[i] = mck_wal_rec_desc{(uint32_t)po, (uint32_t)(po >> 32) | ((uint32_t)p.type << 16) | (full ? MCK_WAL_REC_HASH : 0u),
                              p.length, p.stored};
  }
  return MCK_OK;
}

extern "C" int mck_test_wal_walk_fast(const void* wal, uint64_t nbytes, uint32_t log_number) {
  const uint8_t* d = static_cast<const uint8_t*>(wal);
  std::vector<PhysRec> phys;
  std::vector<BlockStop> stops;
  wal_block_walk(d, nbytes, log_number, phys, stops);
  WalWalk F, S;
  if (!wal_walk_fast(nbytes, phys, stops, F)) return 0;
  if (wal_walk(d, nbytes, log_number, MCK_WAL_kTolerateCorruptedTailRecords, nullptr, S, &phys)) return -1;
  auto same_fr = [](const std::vector<mck_wal_fragment>& a, const std::vector<mck_wal_fragment>& b) {
    if (a.size() != b.size()) return false;
    for (size_t i = 0; i < a.size(); i++)
      if (a[i].src_off != b[i].src_off || a[i].dst_off != b[i].dst_off || a[i].length != b[i].length ||
          a[i].type != b[i].type || a[i].pad != b[i].pad)
        return false;
    return true;
  };
  const bool eq = same_fr(F.fr, S.fr) && F.roff == S.roff && F.rfile == S.rfile && F.rlen == S.rlen &&
                  F.rhoff == S.rhoff && F.rfrag == S.rfrag && S.reports.empty() && F.reports.empty() &&
                  F.report_pos == S.report_pos && F.dropped == S.dropped && F.end_offset == S.end_offset &&
                  F.records_bytes == S.records_bytes && F.compression == S.compression && S.stream.empty();
  return eq ? 1 : -1;
}

extern "C" int mck_wal_read_records(const void* wal, uint64_t nbytes, uint32_t log_number, int recovery_mode,
                                    const mck_wal_block_result* verified, mck_wal_read_out* out) {
  mck_internal_set_error("");
  if (int rc = check_read_args(wal, nbytes, recovery_mode, out)) return rc;
  WalWalk W;
  if (int rc = wal_walk(static_cast<const uint8_t*>(wal), nbytes, log_number, recovery_mode, verified, W)) {
    mck_internal_set_error("verify results do not match the WAL image (a record the device did not reach)");
    return rc;
  }
  return wal_copy_out(W, out);
}

// The reassembly plan alone: mck_wal_read_records without CRCs, in the
// default kTolerateCorruptedTailRecords mode.
extern "C" int mck_wal_list_records(const void* wal, uint64_t nbytes, uint32_t log_number, mck_wal_fragment* frags,
                                    uint64_t frag_cap, uint64_t* nfrags, uint64_t* rec_offsets,
                                    uint32_t* rec_lengths, uint64_t rec_cap, uint64_t* nrecords,
                                    uint64_t* records_bytes) {
  mck_wal_read_out o;
  memset(&o, 0, sizeof o);
  o.struct_size = sizeof o;
  o.frags = frags;
  o.frag_cap = frag_cap;
  o.rec_offsets = rec_offsets;
  o.rec_lengths = rec_lengths;
  o.rec_cap = rec_cap;
  const int rc = mck_wal_read_records(wal, nbytes, log_number, MCK_WAL_kTolerateCorruptedTailRecords, nullptr, &o);
  if (rc) return rc;
  if (nfrags) *nfrags = o.nfrags;
  if (nrecords) *nrecords = o.nrecords;
  if (records_bytes) *records_bytes = o.records_bytes;
  return MCK_OK;
}

// ---------------------------------------------------------------------------
// log::FragmentBufferedReader (db/log_reader.cc:618-931) over a growing host
// image: the reader of secondary instances / WAL tailing.  The "file" is
// [0, avail); a read returns what is written so far.  Restated over file
// offsets: buffer_ = [buf_off, buf_off + buf_size), fragments_ = the payload
// fragments of the record being assembled (kept across ReadRecord calls).
// ---------------------------------------------------------------------------
struct mck_wal_tail {
  uint32_t log_number = 0;
  const uint8_t* d = nullptr;
  uint64_t avail = 0;
  const mck_wal_block_result* verified = nullptr;
  uint64_t buf_off = 0, buf_size = 0, end_of_buffer_offset = 0;
  uint64_t eof_offset = 0;
  // the header of a record of an older log instance the reader stopped at
  // (~0: none); see mck_wal_tail_old_record
  uint64_t old_record_offset = ~0ull;
  bool eof = false, recycled = false, first_record_read = false, in_fragmented_record = false;
  uint64_t last_record_offset = 0;
  std::vector<mck_wal_fragment> fragments;  // fragments_ (dst_off within the record)
  uint64_t fragments_size = 0;
  std::vector<mck_wal_fragment> record;     // the last record returned
  uint64_t record_bytes = 0;
  std::vector<mck_wal_report> reports;
  uint64_t dropped = 0;
  TsRecorder ts;
  int err = MCK_OK;

  void report(uint64_t off, uint64_t bytes, int reason) {
    reports.push_back(mck_wal_report{off, bytes, reason, 0});
    dropped += bytes;
  }
  uint64_t file_read(uint64_t n) {  // SequentialFileReader::Read of n bytes
    const uint64_t got = std::min<uint64_t>(n, avail > end_of_buffer_offset ? avail - end_of_buffer_offset : 0);
    end_of_buffer_offset += got;
    return got;
  }
  // Reader::UnmarkEOFInternal (:340-397): read the rest of the block the EOF
  // was in, behind what is left of the buffer
  void unmark_eof_internal() {
    const uint64_t remaining = MCK_WAL_kBlockSize - eof_offset;
    const uint64_t added = file_read(remaining);
    buf_size += added;  // buffer_ = [consumed, eof_offset + added) of the block
    if (added < remaining) {
      eof = true;
      eof_offset += added;
    } else {
      eof_offset = 0;
    }
  }
  // FragmentBufferedReader::UnmarkEOF (:777-783)
  void unmark_eof() {
    eof = false;
    unmark_eof_internal();
  }
  // :785-823 TryReadMore (no read errors on a memory image)
  bool try_read_more() {
    if (!eof) {  // the last read was a full block: what is left is a trailer
      buf_off = end_of_buffer_offset;
      buf_size = file_read(MCK_WAL_kBlockSize);
      if (buf_size < MCK_WAL_kBlockSize) {
        eof = true;
        eof_offset = buf_size;
      }
      return true;
    }
    unmark_eof();
    return true;
  }
  // Verdicts of records after a checksum failure inside a block: only the
  // tailing reader reaches them (the failure dropped a buffer that ended at
  // the file's end, the block grew, and UnmarkEOF reads on behind it), and a
  // block's verdict stops at its first failure.  The caller verifies the
  // block from the first such record on (mck_wal_tail_pending_verify /
  // mck_wal_tail_add_verdict); those verdicts are kept here.
  struct SubVerdict {
    uint64_t from;  // file offset the verification started at
    mck_wal_block_result r;
  };
  std::vector<SubVerdict> sub;
  uint64_t need_from = ~0ull;  // a verdict is needed from this offset on
  // 1 = the CRC holds, 0 = it does not, -1 = no verdict covers h yet
  int crc_ok(uint64_t h) {
    if (!verified) return 1;
    const uint64_t blk = h / MCK_WAL_kBlockSize;
    for (size_t k = sub.size(); k-- > 0;) {  // the latest verification of h's block from at or before h
      const SubVerdict& v = sub[k];
      if (v.from / MCK_WAL_kBlockSize != blk || v.from > h) continue;
      const uint64_t o = h - v.from;
      if (o < v.r.stop_offset) return 1;
      if (o == v.r.stop_offset && v.r.status == MCK_WAL_BAD_CHECKSUM) return 0;
      break;
    }
    const mck_wal_block_result& r = verified[blk];
    const uint32_t o = (uint32_t)(h % MCK_WAL_kBlockSize);
    if (o < r.stop_offset) return 1;
    if (o == r.stop_offset && r.status == MCK_WAL_BAD_CHECKSUM) return 0;
    if (r.status == MCK_WAL_BAD_CHECKSUM) {  // past the block's first failure
      need_from = h;
      return -1;
    }
    err = MCK_EINVAL;  // stale or foreign verdicts (a block verified before it grew)
    return 0;
  }
  // :826-931 TryReadFragment; true = the caller processes *type_or_err
  bool try_read_fragment(uint64_t* frag_off, uint32_t* frag_len, uint64_t* drop_size, uint32_t* type_or_err) {
    while (buf_size < MCK_WAL_kHeaderSize) {
      const uint64_t old = buf_size;
      try_read_more();
      if (old == buf_size) return false;
    }
    const uint8_t* h = d + buf_off;
    const uint32_t type = header_type(h);
    const uint32_t length = (uint32_t)h[4] | ((uint32_t)h[5] << 8);
    uint32_t hs = MCK_WAL_kHeaderSize;
    if ((type >= 5 && type <= 8) || type == kRecyclableUserDefinedTimestampSizeType) {
      if (end_of_buffer_offset - buf_size == 0) recycled = true;
      hs = MCK_WAL_kRecyclableHeaderSize;
      while (buf_size < MCK_WAL_kRecyclableHeaderSize) {
        const uint64_t old = buf_size;
        try_read_more();
        if (old == buf_size) return false;
      }
      const uint8_t* g = d + buf_off;
      const uint32_t ln = (uint32_t)g[7] | ((uint32_t)g[8] << 8) | ((uint32_t)g[9] << 16) | ((uint32_t)g[10] << 24);
      if (ln != log_number) {
        old_record_offset = buf_off;
        *type_or_err = kOldRecord;
        return true;
      }
    }
    while ((uint64_t)hs + length > buf_size) {
      const uint64_t old = buf_size;
      try_read_more();
      if (old == buf_size) return false;
    }
    // buffer_.clear() (:880, :889-891): the window moves past what it held,
    // so buf_off + buf_size stays end_of_buffer_offset and a later
    // UnmarkEOFInternal appends the NEW bytes behind it
    if (type == kZeroType && length == 0) {
      buf_off += buf_size;
      buf_size = 0;
      *type_or_err = kBadRecord;
      return true;
    }
    const int ok = crc_ok(buf_off);
    if (ok < 0) return false;  // nothing consumed: ReadRecord returns MCK_EAGAIN
    if (!ok) {
      *drop_size = buf_size;
      buf_off += buf_size;
      buf_size = 0;
      *type_or_err = kBadRecordChecksum;
      return true;
    }
    *frag_off = buf_off + hs;
    *frag_len = length;
    buf_off += hs + length;
    buf_size -= hs + length;
    *type_or_err = type;
    return true;
  }
  void fragments_clear() {
    fragments.clear();
    fragments_size = 0;
  }
  void fragments_append(uint64_t off, uint32_t len, uint32_t type) {
    fragments.push_back(mck_wal_fragment{off, fragments_size, len, (uint8_t)type, 0, 0});
    fragments_size += len;
  }
  // :618-775 ReadRecord; 1 = a record, 0 = none (yet)
  int read_record() {
    uint64_t prospective_record_offset = 0;
    const uint64_t physical_record_offset = end_of_buffer_offset - buf_size;
    uint64_t drop_size = 0, foff = 0;
    uint32_t flen = 0, t = 0;
    old_record_offset = ~0ull;
    need_from = ~0ull;
    while (try_read_fragment(&foff, &flen, &drop_size, &t)) {
      if (err) return err;
      if (t == 1 || t == 5) {  // kFullType
        if (in_fragmented_record && fragments_size) report(physical_record_offset, fragments_size, MCK_WAL_R_PARTIAL_WITHOUT_END_1);
        fragments_clear();
        record.assign(1, mck_wal_fragment{foff, 0, flen, (uint8_t)t, 0, 0});
        record_bytes = flen;
        prospective_record_offset = physical_record_offset;
        last_record_offset = prospective_record_offset;
        first_record_read = true;
        in_fragmented_record = false;
        return 1;
      } else if (t == 2 || t == 6) {  // kFirstType
        if (in_fragmented_record || fragments_size) report(physical_record_offset, fragments_size, MCK_WAL_R_PARTIAL_WITHOUT_END_2);
        prospective_record_offset = physical_record_offset;
        fragments_clear();
        fragments_append(foff, flen, t);
        in_fragmented_record = true;
      } else if (t == 3 || t == 7) {  // kMiddleType
        if (!in_fragmented_record)
          report(physical_record_offset, flen, MCK_WAL_R_MISSING_START_1);
        else
          fragments_append(foff, flen, t);
      } else if (t == 4 || t == 8) {  // kLastType
        if (!in_fragmented_record) {
          report(physical_record_offset, flen, MCK_WAL_R_MISSING_START_2);
        } else {
          fragments_append(foff, flen, t);
          record = fragments;
          record_bytes = fragments_size;
          fragments_clear();
          last_record_offset = prospective_record_offset;
          first_record_read = true;
          in_fragmented_record = false;
          return 1;
        }
      } else if (t == kSetCompressionType) {
        mck_internal_set_error("WAL compression (kSetCompressionType record) is not supported");
        return MCK_ENOTSUP;
      } else if (t == kUserDefinedTimestampSizeType || t == kRecyclableUserDefinedTimestampSizeType) {
        // (:712 tests scratch, which ReadRecord cleared: never reported)
        fragments_clear();
        prospective_record_offset = physical_record_offset;
        last_record_offset = prospective_record_offset;
        in_fragmented_record = false;
        if (flen % 6) {
          report(physical_record_offset, flen, MCK_WAL_R_TS_DECODE);
        } else if (const int why = ts.update(d + foff, flen)) {
          report(physical_record_offset, flen, why);
        }
      } else if (t == (uint32_t)kBadHeader || t == (uint32_t)kBadRecord || t == (uint32_t)kEof ||
                 t == (uint32_t)kOldRecord) {
        if (in_fragmented_record) {
          report(physical_record_offset, fragments_size, MCK_WAL_R_ERROR_IN_MIDDLE);
          in_fragmented_record = false;
          fragments_clear();
        }
        // kOldRecord does not advance the buffer: the reference's loop would
        // parse the same header again forever; report "no record" instead
        if (t == (uint32_t)kOldRecord) return 0;
      } else if (t == (uint32_t)kBadRecordChecksum) {
        if (recycled) {
          fragments_clear();
          return 0;
        }
        report(physical_record_offset, drop_size, MCK_WAL_R_CHECKSUM_MISMATCH);
        if (in_fragmented_record) {
          report(physical_record_offset, fragments_size, MCK_WAL_R_ERROR_IN_MIDDLE);
          in_fragmented_record = false;
          fragments_clear();
        }
      } else {
        report(physical_record_offset, flen + (in_fragmented_record ? fragments_size : 0), unknown_type_reason(t));
        in_fragmented_record = false;
        fragments_clear();
      }
    }
    if (err) return err;
    return need_from != ~0ull ? MCK_EAGAIN : 0;
  }
};

extern "C" int mck_wal_tail_create(uint32_t log_number, mck_wal_tail** out) {
  mck_internal_set_error("");
  if (!out) {
    mck_internal_set_error("out is NULL");
    return MCK_EINVAL;
  }
  *out = new (std::nothrow) mck_wal_tail();
  if (!*out) {
    mck_internal_set_error("out of memory");
    return MCK_ENOMEM;
  }
  (*out)->log_number = log_number;
  return MCK_OK;
}

extern "C" void mck_wal_tail_destroy(mck_wal_tail* r) { delete r; }

extern "C" int mck_wal_tail_set_image(mck_wal_tail* r, const void* wal, uint64_t nbytes,
                                      const mck_wal_block_result* verified) {
  mck_internal_set_error("");
  if (!r || (!wal && nbytes)) {
    mck_internal_set_error("reader / wal is NULL");
    return MCK_EINVAL;
  }
  if (nbytes < r->end_of_buffer_offset) {
    mck_internal_set_error("the WAL image shrank below what the reader has read");
    return MCK_EINVAL;
  }
  r->d = static_cast<const uint8_t*>(wal);
  r->avail = nbytes;
  r->verified = verified;
  return MCK_OK;
}

extern "C" int mck_wal_tail_read_record(mck_wal_tail* r, uint64_t* nfrags, uint64_t* record_bytes,
                                        uint64_t* last_record_offset) {
  mck_internal_set_error("");
  if (!r) {
    mck_internal_set_error("reader is NULL");
    return MCK_EINVAL;
  }
  if (r->err) return r->err;
  const int rc = r->read_record();
  if (rc < 0) {
    if (rc == MCK_EINVAL) mck_internal_set_error("verify results do not match the WAL image (stale verdicts?)");
    return rc;
  }
  if (rc == 1) {
    if (nfrags) *nfrags = r->record.size();
    if (record_bytes) *record_bytes = r->record_bytes;
    if (last_record_offset) *last_record_offset = r->last_record_offset;
  }
  return rc;
}

extern "C" int mck_wal_tail_record_fragments(const mck_wal_tail* r, mck_wal_fragment* frags, uint64_t cap) {
  mck_internal_set_error("");
  if (!r || (!frags && !r->record.empty())) {
    mck_internal_set_error("reader / frags is NULL");
    return MCK_EINVAL;
  }
  if (cap < r->record.size()) {
    mck_internal_set_error("frags capacity too small");
    return MCK_EINVAL;
  }
  if (!r->record.empty()) memcpy(frags, r->record.data(), r->record.size() * sizeof(mck_wal_fragment));
  return MCK_OK;
}

extern "C" int mck_wal_tail_unmark_eof(mck_wal_tail* r) {
  if (!r) return MCK_EINVAL;
  r->unmark_eof();
  return MCK_OK;
}

extern "C" int mck_wal_tail_is_eof(const mck_wal_tail* r) { return r && r->eof ? 1 : 0; }

extern "C" int mck_wal_tail_pending_verify(const mck_wal_tail* r, uint64_t* file_offset, uint64_t* nbytes) {
  if (!r || r->need_from == ~0ull) return 0;
  const uint64_t end = std::min<uint64_t>((r->need_from / MCK_WAL_kBlockSize + 1) * MCK_WAL_kBlockSize, r->avail);
  if (file_offset) *file_offset = r->need_from;
  if (nbytes) *nbytes = end - r->need_from;
  return 1;
}

extern "C" int mck_wal_tail_add_verdict(mck_wal_tail* r, uint64_t file_offset, const mck_wal_block_result* res) {
  mck_internal_set_error("");
  if (!r || !res) {
    mck_internal_set_error("reader / result is NULL");
    return MCK_EINVAL;
  }
  if (file_offset >= r->avail) {
    mck_internal_set_error("verdict offset past the image");
    return MCK_EINVAL;
  }
  // only the verdict mck_wal_tail_pending_verify asked for, and only one that
  // decides the pending record (its CRC holds past it, or fails AT it): any
  // other would leave the reader asking for the same verdict forever
  char msg[160];
  if (r->need_from == ~0ull || file_offset != r->need_from) {
    snprintf(msg, sizeof msg, "no verdict pending at offset %llu", (unsigned long long)file_offset);
    mck_internal_set_error(msg);
    return MCK_EINVAL;
  }
  if (res->stop_offset == 0 && res->status != MCK_WAL_BAD_CHECKSUM) {
    snprintf(msg, sizeof msg, "verdict at %llu makes no progress (stop_offset 0, status %d)",
             (unsigned long long)file_offset, (int)res->status);
    mck_internal_set_error(msg);
    return MCK_EINVAL;
  }
  r->sub.push_back(mck_wal_tail::SubVerdict{file_offset, *res});
  r->need_from = ~0ull;
  return MCK_OK;
}

extern "C" int mck_wal_tail_old_record(const mck_wal_tail* r, uint64_t* header_offset) {
  if (!r || r->old_record_offset == ~0ull) return 0;
  if (header_offset) *header_offset = r->old_record_offset;
  return 1;
}

extern "C" int mck_wal_tail_reports(const mck_wal_tail* r, mck_wal_report* reports, uint64_t cap, uint64_t* n,
                                    uint64_t* dropped_bytes) {
  if (!r) return MCK_EINVAL;
  const uint64_t k = std::min<uint64_t>(cap, r->reports.size());
  if (reports && k) memcpy(reports, r->reports.data(), k * sizeof(mck_wal_report));
  if (n) *n = r->reports.size();
  if (dropped_bytes) *dropped_bytes = r->dropped;
  return MCK_OK;
}
