// mck_blob.cc -- host-side walk of a blob file (db/blob/blob_log_format.h):
// the 30-byte BlobLogHeader, the records (32-byte header + key + value) in
// file order, and the 32-byte BlobLogFooter.  The records' header and blob
// CRCs are then checked on the GPU in one mck_blob_record_batch call.
//
// Restated (speedb-io/speedb):
//   BlobLogHeader::DecodeFrom        db/blob/blob_log_format.cc:27-55
//   BlobLogFooter::DecodeFrom        db/blob/blob_log_format.cc:70-95
//   record sizes / record_size()     db/blob/blob_log_format.h:118-160
//   BlobLogSequentialReader          db/blob/blob_log_sequential_reader.cc:64-135
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#include "../../include/speedb_amd/mck.h"
#include "mck_internal.h"

namespace {

int fail(int rc, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  mck_internal_set_error(buf);
  return rc;
}
uint32_t fixed32(const uint8_t* p) {
  return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}
uint64_t fixed64(const uint8_t* p) { return (uint64_t)fixed32(p) | (uint64_t)fixed32(p + 4) << 32; }

}  // namespace

extern "C" int mck_blob_list_records(const void* file, uint64_t size, mck_blob_file_info* info,
                                     mck_blob_record* records, uint64_t cap, uint64_t* nrecords) {
  mck_internal_set_error("");
  if (!file || !info || !nrecords) return fail(MCK_EINVAL, "NULL argument");
  const uint8_t* d = static_cast<const uint8_t*>(file);
  memset(info, 0, sizeof *info);
  const char* hdr_err = "Error while decoding blob log header";
  if (size < MCK_BLOB_kHeaderSize) return fail(MCK_ECORRUPT, "%s: Unexpected blob file header size", hdr_err);
  if (fixed32(d) != MCK_BLOB_kMagicNumber) return fail(MCK_ECORRUPT, "%s: Magic number mismatch", hdr_err);
  info->version = fixed32(d + 4);
  if (info->version != 1) return fail(MCK_ECORRUPT, "%s: Unknown header version", hdr_err);
  info->column_family_id = fixed32(d + 8);
  info->has_ttl = (d[12] & 1) == 1;
  info->compression = d[13];
  info->expiration_first = fixed64(d + 14);
  info->expiration_second = fixed64(d + 22);
  // a footer is the last 32 bytes when they start with the magic number;
  // its CRC (BlobLogFooter::DecodeFrom) is checked on the device by the
  // caller (footer_crc = the stored value)
  uint64_t end = size;
  if (size >= MCK_BLOB_kHeaderSize + MCK_BLOB_kFooterSize) {
    const uint8_t* f = d + size - MCK_BLOB_kFooterSize;
    if (fixed32(f) == MCK_BLOB_kMagicNumber) {
      info->has_footer = 1;
      info->footer_blob_count = fixed64(f + 4);
      info->footer_crc = fixed32(f + 28);
      end = size - MCK_BLOB_kFooterSize;
    }
  }
  std::vector<mck_blob_record> out;
  uint64_t pos = MCK_BLOB_kHeaderSize;
  while (pos < end) {
    if (end - pos < MCK_BLOB_kRecordHeaderSize)
      return fail(MCK_ECORRUPT, "Error while decoding blob record: Unexpected blob record header size");
    const uint64_t ks = fixed64(d + pos), vs = fixed64(d + pos + 8);
    const uint64_t room = end - pos - MCK_BLOB_kRecordHeaderSize;
    if (ks > room || vs > room - ks)
      return fail(MCK_ECORRUPT, "Error while reading blob record at %llu: key/value size past the end of the file",
                  (unsigned long long)pos);
    if (ks + vs > 0xFFFFFFFFull) return fail(MCK_ENOTSUP, "blob record larger than 4 GiB at %llu",
                                             (unsigned long long)pos);
    out.push_back(mck_blob_record{pos, ks, vs});
    pos += MCK_BLOB_kRecordHeaderSize + ks + vs;
  }
  if (info->has_footer && info->footer_blob_count != out.size())
    return fail(MCK_ECORRUPT, "blob count mismatch: footer says %llu, file holds %llu records",
                (unsigned long long)info->footer_blob_count, (unsigned long long)out.size());
  *nrecords = out.size();
  if (records) {
    if (cap < out.size()) return fail(MCK_EINVAL, "records capacity too small");
    if (!out.empty()) memcpy(records, out.data(), out.size() * sizeof(mck_blob_record));
  }
  return MCK_OK;
}
