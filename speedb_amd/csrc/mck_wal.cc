// mck_wal.cc -- host-side write plan of the device WAL writer: the
// fragmentation log::Writer::AddRecord performs (db/log_writer.cc:79-175),
// on sizes only.  The bytes are written on the device by
// mck_wal_write_batch (mck_engine.hip).
#include <string.h>

#include <vector>

#include "../../include/speedb_amd/mck.h"
#include "mck_internal.h"

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

// log::Reader::ReadRecord (db/log_reader.cc:69-321) + ReadPhysicalRecord
// (:450-584) without the CRC check, on a host image.
extern "C" int mck_wal_list_records(const void* wal, uint64_t nbytes, uint32_t log_number, mck_wal_fragment* frags,
                                    uint64_t frag_cap, uint64_t* nfrags, uint64_t* rec_offsets,
                                    uint32_t* rec_lengths, uint64_t rec_cap, uint64_t* nrecords,
                                    uint64_t* records_bytes) {
  mck_internal_set_error("");
  if (!wal && nbytes) {
    mck_internal_set_error("wal is NULL");
    return MCK_EINVAL;
  }
  const uint8_t* d = static_cast<const uint8_t*>(wal);
  const uint64_t kBlock = MCK_WAL_kBlockSize;
  std::vector<mck_wal_fragment> fr;
  std::vector<uint64_t> roff;
  std::vector<uint32_t> rlen;
  uint64_t dst = 0;           // end of the reassembled buffer
  uint64_t cur_start = 0;     // dst offset of the record being assembled
  size_t cur_first_frag = 0;  // its first fragment in fr
  bool in_frag = false;
  auto drop_partial = [&] {
    if (in_frag) {
      fr.resize(cur_first_frag);
      dst = cur_start;
      in_frag = false;
    }
  };
  auto add_frag = [&](uint64_t src, uint32_t len, uint8_t type) {
    fr.push_back(mck_wal_fragment{src, dst, len, type, 0, 0});
    dst += len;
  };
  auto emit = [&] {
    roff.push_back(cur_start);
    rlen.push_back((uint32_t)(dst - cur_start));
    in_frag = false;
  };
  uint64_t pos = 0;
  while (pos < nbytes) {
    const uint64_t block_end = (pos / kBlock + 1) * kBlock;
    const uint64_t avail = (block_end < nbytes ? block_end : nbytes) - pos;  // buffer_.size()
    if (avail < MCK_WAL_kHeaderSize) {  // block trailer, or a truncated header at EOF
      if (block_end >= nbytes) break;
      pos = block_end;
      continue;
    }
    const uint8_t* h = d + pos;
    const uint32_t length = (uint32_t)h[4] | ((uint32_t)h[5] << 8);
    const uint8_t type = h[6];
    uint32_t hs = MCK_WAL_kHeaderSize;
    if ((type >= 5 && type <= 8) || type == 11) {
      hs = MCK_WAL_kRecyclableHeaderSize;
      if (avail < hs) break;  // truncated header at EOF
      const uint32_t ln = (uint32_t)h[7] | ((uint32_t)h[8] << 8) | ((uint32_t)h[9] << 16) | ((uint32_t)h[10] << 24);
      if (ln != log_number) break;  // kOldRecord: end of this log's records
    }
    if (hs + (uint64_t)length > avail) {  // kBadRecordLen: drop the rest of the block
      if (block_end >= nbytes) break;     // at EOF: truncated record body
      drop_partial();
      pos = block_end;
      continue;
    }
    if (type == 0 && length == 0) {  // kZeroType padding: the buffer is cleared
      if (block_end >= nbytes) break;
      pos = block_end;
      continue;
    }
    const uint64_t payload = pos + hs;
    switch (type) {
      case 1:
      case 5:  // kFullType
        drop_partial();
        cur_start = dst;
        cur_first_frag = fr.size();
        add_frag(payload, length, type);
        emit();
        break;
      case 2:
      case 6:  // kFirstType
        drop_partial();
        cur_start = dst;
        cur_first_frag = fr.size();
        add_frag(payload, length, type);
        in_frag = true;
        break;
      case 3:
      case 7:  // kMiddleType
        if (in_frag) add_frag(payload, length, type);
        break;
      case 4:
      case 8:  // kLastType
        if (in_frag) {
          add_frag(payload, length, type);
          emit();
        }
        break;
      default:  // kSetCompressionType / timestamp-size records / unknown
        drop_partial();
        break;
    }
    pos = payload + length;
  }
  drop_partial();  // EOF inside a fragmented record: ignored
  if (nfrags) *nfrags = fr.size();
  if (nrecords) *nrecords = roff.size();
  if (records_bytes) *records_bytes = dst;
  if (frags) {
    if (frag_cap < fr.size()) {
      mck_internal_set_error("frags capacity too small");
      return MCK_EINVAL;
    }
    memcpy(frags, fr.data(), fr.size() * sizeof(mck_wal_fragment));
  }
  if (rec_offsets || rec_lengths) {
    if (rec_cap < roff.size()) {
      mck_internal_set_error("records capacity too small");
      return MCK_EINVAL;
    }
    if (rec_offsets) memcpy(rec_offsets, roff.data(), roff.size() * 8);
    if (rec_lengths) memcpy(rec_lengths, rlen.data(), rlen.size() * 4);
  }
  return MCK_OK;
}
