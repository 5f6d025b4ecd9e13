// mck_sst.cc -- host-side reader of the block-based table (SST) layout, as
// far as whole-file checksum verification needs it (SURVEY.md 8f row 1:
// DB::VerifyChecksum / BlockBasedTable::VerifyChecksum as one batched device
// scan).  It lists every checksummed block of an SST image held in host
// memory; the blocks' bytes are then verified on the GPU in ONE
// mck_sst_verify_batch call over the listed handles, and the format_version
// 6 footer checksum with the builtin-checksum shim (mck_sst_verify_footer).
//
// What is restated (paths in the speedb-io/speedb tree):
//   Footer::DecodeFrom                        table/format.cc:348-470
//   BlockHandle::DecodeFrom, IndexValue       table/format.cc:82-160
//   block entry decoding (DecodeEntry/V4)     table/block_based/block.cc:31-139
//   restart array / num_restarts              table/block_based/block.cc
//   index value delta encoding                table/block_based/block.cc:715-725
//   properties block (varint64 integer props) table/meta_blocks.cc:60-130
//   index type property (fixed32)             table/block_based/block_based_table_builder.cc:239
//   meta block names                          table/meta_blocks.cc:29-35,
//                                             block_based_table_builder.cc:2096-2100,
//                                             block_based_table_factory.cc:1141-1143
//   VerifyChecksum / VerifyChecksumInBlocks / VerifyChecksumInMetaBlocks
//                                             table/block_based/block_based_table_reader.cc:2336-2500
// Compressed index / meta blocks are not decompressed here (the codecs are
// the reference's): mck_sst_list_blocks reports them as MCK_ENOTSUP, and
// mck_sst_list_blocks_uncompress hands each to the caller's callback (the
// reference's UncompressBlockData) and parses what it returns.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <string>
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

constexpr uint64_t kBlockBasedTableMagicNumber = 0x88e241b785f4cff7ull;
constexpr uint64_t kLegacyBlockBasedTableMagicNumber = 0xdb4775248b80fb57ull;
constexpr uint32_t kBlockTrailerSize = 5;
constexpr uint32_t kMaxVarint64Length = 10;
constexpr uint32_t kHandleMax = 2 * kMaxVarint64Length;                 // 20
constexpr uint32_t kVersion0EncodedLength = 2 * kHandleMax + 8;         // 48
constexpr uint32_t kNewVersionsEncodedLength = 1 + 2 * kHandleMax + 4 + 8;  // 53
constexpr uint32_t kLatestFormatVersion = 6;

uint32_t fixed32(const uint8_t* p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }
uint64_t fixed64(const uint8_t* p) { return (uint64_t)fixed32(p) | (uint64_t)fixed32(p + 4) << 32; }

struct Slice {
  const uint8_t* p;
  uint64_t n;
};

bool varint64(Slice* s, uint64_t* v) {
  uint64_t r = 0;
  for (uint32_t shift = 0; shift <= 63 && s->n; shift += 7) {
    const uint8_t b = *s->p++;
    s->n--;
    r |= (uint64_t)(b & 127) << shift;
    if (!(b & 128)) {
      *v = r;
      return true;
    }
  }
  return false;
}
bool varint32(Slice* s, uint32_t* v) {
  uint64_t x;
  if (!varint64(s, &x) || x > 0xFFFFFFFFull) return false;
  *v = (uint32_t)x;
  return true;
}
// util/coding.h GetVarsignedint64: zigzag
bool varsigned64(Slice* s, int64_t* v) {
  uint64_t u;
  if (!varint64(s, &u)) return false;
  *v = (int64_t)(u >> 1) ^ -(int64_t)(u & 1);
  return true;
}

struct Handle {
  uint64_t offset = 0, size = 0;
};
bool decode_handle(Slice* s, Handle* h) { return varint64(s, &h->offset) && varint64(s, &h->size); }

// One parsed block: entries (key, value) in order; keys fully materialised
// (shared prefixes applied).
struct Entry {
  std::string key;
  Slice value;
};

class File {
 public:
  File(const uint8_t* d, uint64_t n, mck_sst_uncompress_fn fn = nullptr, void* ctx = nullptr)
      : d_(d), n_(n), fn_(fn), ctx_(ctx) {}

  // The contents of block `h` (trailer follows): the stored payload, or for
  // a compressed block what the caller's uncompress callback returns.
  int payload(const Handle& h, const char* what, Slice* out) const {
    if (h.offset > n_ || h.size > n_ - h.offset || n_ - h.offset - h.size < kBlockTrailerSize)
      return fail(MCK_ECORRUPT, "%s block handle (offset %llu, size %llu) is past the end of the file (%llu bytes)",
                  what, (unsigned long long)h.offset, (unsigned long long)h.size, (unsigned long long)n_);
    const uint8_t type = d_[h.offset + h.size];
    if (type != 0) {
      if (!fn_)
        return fail(MCK_ENOTSUP, "%s block at offset %llu is compressed (type %u): cannot be parsed on the host", what,
                    (unsigned long long)h.offset, type);
      const void* u = nullptr;
      uint64_t un = 0;
      const int rc = fn_(ctx_, type, h.offset, d_ + h.offset, h.size, &u, &un);
      if (rc != MCK_OK)
        return fail(rc, "%s block at offset %llu: uncompress callback failed (type %u, rc %d)", what,
                    (unsigned long long)h.offset, type, rc);
      if (!u && un) return fail(MCK_EINVAL, "%s block at offset %llu: uncompress callback returned NULL", what,
                                (unsigned long long)h.offset);
      *out = Slice{static_cast<const uint8_t*>(u), un};
      return MCK_OK;
    }
    *out = Slice{d_ + h.offset, h.size};
    return MCK_OK;
  }

  // Block entries (DecodeEntry): [shared v32][non_shared v32]
  // [value_length v32][key delta][value], then the restart array and
  // num_restarts (bit 31 = the data-block hash-index flag).
  static int entries(Slice b, const char* what, std::vector<Entry>* out) {
    if (b.n < 4) return fail(MCK_ECORRUPT, "%s block too small (%llu bytes)", what, (unsigned long long)b.n);
    const uint32_t num_restarts = fixed32(b.p + b.n - 4) & 0x7FFFFFFFu;
    if ((uint64_t)num_restarts * 4 + 4 > b.n)
      return fail(MCK_ECORRUPT, "%s block: bad restart array (%u restarts in %llu bytes)", what, num_restarts,
                  (unsigned long long)b.n);
    Slice s{b.p, b.n - 4 - (uint64_t)num_restarts * 4};
    std::string key;
    out->clear();
    while (s.n) {
      uint32_t shared, non_shared, vlen;
      if (!varint32(&s, &shared) || !varint32(&s, &non_shared) || !varint32(&s, &vlen))
        return fail(MCK_ECORRUPT, "%s block: bad entry header", what);
      if (shared > key.size() || non_shared > s.n || vlen > s.n - non_shared)
        return fail(MCK_ECORRUPT, "%s block: bad entry lengths", what);
      key.resize(shared);
      key.append(reinterpret_cast<const char*>(s.p), non_shared);
      s.p += non_shared;
      s.n -= non_shared;
      Entry e;
      e.key = key;
      e.value = Slice{s.p, vlen};
      s.p += vlen;
      s.n -= vlen;
      out->push_back(e);
    }
    return MCK_OK;
  }

  // Index block (table/block_based/block.cc IndexBlockIter): every entry's
  // value is an IndexValue -- a full BlockHandle, or with delta encoding and
  // shared != 0 the varsigned size delta, offset = prev.offset + prev.size +
  // kBlockTrailerSize -- optionally followed by a length-prefixed first key.
  static int index_handles(Slice b, bool delta, bool first_key, const char* what, std::vector<Handle>* out) {
    if (b.n < 4) return fail(MCK_ECORRUPT, "%s block too small", what);
    const uint32_t num_restarts = fixed32(b.p + b.n - 4) & 0x7FFFFFFFu;
    if ((uint64_t)num_restarts * 4 + 4 > b.n) return fail(MCK_ECORRUPT, "%s block: bad restart array", what);
    Slice s{b.p, b.n - 4 - (uint64_t)num_restarts * 4};
    uint64_t key_len = 0;
    Handle prev;
    bool have_prev = false;
    while (s.n) {
      uint32_t shared, non_shared, vlen = 0;
      if (!varint32(&s, &shared) || !varint32(&s, &non_shared) || (!delta && !varint32(&s, &vlen)))
        return fail(MCK_ECORRUPT, "%s block: bad entry header", what);
      if (shared > key_len || non_shared > s.n) return fail(MCK_ECORRUPT, "%s block: bad entry lengths", what);
      key_len = (uint64_t)shared + non_shared;
      s.p += non_shared;
      s.n -= non_shared;
      Slice v = delta ? s : Slice{s.p, vlen};
      if (!delta && vlen > s.n) return fail(MCK_ECORRUPT, "%s block: bad value length", what);
      const uint64_t vstart = v.n;
      Handle h;
      if (delta && shared != 0) {
        int64_t d;
        if (!have_prev || !varsigned64(&v, &d)) return fail(MCK_ECORRUPT, "bad delta-encoded index value");
        h.offset = prev.offset + prev.size + kBlockTrailerSize;
        h.size = prev.size + (uint64_t)d;
      } else if (!decode_handle(&v, &h)) {
        return fail(MCK_ECORRUPT, "bad block handle");
      }
      if (first_key) {
        uint32_t fk;
        if (!varint32(&v, &fk) || fk > v.n) return fail(MCK_ECORRUPT, "bad first key in block info");
        v.p += fk;
        v.n -= fk;
      }
      const uint64_t used = vstart - v.n;
      if (delta) {
        s.p += used;
        s.n -= used;
      } else {
        s.p += vlen;
        s.n -= vlen;
      }
      out->push_back(h);
      prev = h;
      have_prev = true;
    }
    return MCK_OK;
  }

  const uint8_t* d_;
  uint64_t n_;
  mck_sst_uncompress_fn fn_;
  void* ctx_;
};

bool starts_with(const std::string& s, const char* p) { return s.compare(0, strlen(p), p) == 0; }

int meta_kind(const std::string& name) {
  if (starts_with(name, "fullfilter.")) return MCK_SST_BLOCK_FILTER;
  if (starts_with(name, "partitionedfilter.")) return MCK_SST_BLOCK_FILTER_PARTITION_INDEX;
  if (name == "rocksdb.properties") return MCK_SST_BLOCK_PROPERTIES;
  if (name == "rocksdb.compression_dict") return MCK_SST_BLOCK_COMPRESSION_DICT;
  if (name == "rocksdb.range_del") return MCK_SST_BLOCK_RANGE_DEL;
  if (name == "rocksdb.index") return MCK_SST_BLOCK_INDEX;
  return MCK_SST_BLOCK_OTHER_META;  // hash-index prefixes/metadata, obsolete filter.*
}

}  // namespace

extern "C" {

int mck_sst_decode_footer(const void* tail, uint64_t tail_len, uint64_t tail_offset, mck_sst_footer* f) {
  mck_internal_set_error("");
  if (!tail || !f) return fail(MCK_EINVAL, "NULL argument");
  if (tail_len < kVersion0EncodedLength) return fail(MCK_ECORRUPT, "file is too short (%llu bytes) to be an sstable",
                                                     (unsigned long long)tail_len);
  const uint8_t* in = static_cast<const uint8_t*>(tail);
  memset(f, 0, sizeof *f);
  const uint8_t* magic_ptr = in + tail_len - 8;
  uint64_t magic = fixed64(magic_ptr);
  const bool legacy = magic == kLegacyBlockBasedTableMagicNumber;
  if (legacy) magic = kBlockBasedTableMagicNumber;
  if (magic != kBlockBasedTableMagicNumber)
    return fail(MCK_ECORRUPT, "Bad table magic number: expected %llu, found %llu",
                (unsigned long long)kBlockBasedTableMagicNumber, (unsigned long long)magic);
  f->magic = magic;
  f->block_trailer_size = kBlockTrailerSize;
  Slice s;
  if (legacy) {
    f->format_version = 0;
    f->checksum_type = MCK_kCRC32c;
    f->footer_offset = tail_offset + tail_len - kVersion0EncodedLength;
    s = Slice{in + tail_len - kVersion0EncodedLength, 2 * kHandleMax};
  } else {
    f->format_version = fixed32(magic_ptr - 4);
    if (f->format_version > kLatestFormatVersion)
      return fail(MCK_ECORRUPT, "Corrupt or unsupported format_version: %u", f->format_version);
    if (tail_len < kNewVersionsEncodedLength) return fail(MCK_ECORRUPT, "Input is too short to be an SST file");
    const uint8_t* foot = in + tail_len - kNewVersionsEncodedLength;
    f->footer_offset = tail_offset + tail_len - kNewVersionsEncodedLength;
    f->checksum_type = foot[0];
    if (f->checksum_type > MCK_kXXH3)
      return fail(MCK_ECORRUPT, "Corrupt or unsupported checksum type: %u", (unsigned)foot[0]);
    s = Slice{foot + 1, 2 * kHandleMax};
  }
  if (f->format_version >= 6) {
    static const uint8_t kExtendedMagic[4] = {0x3e, 0x00, 0x7a, 0x00};
    if (memcmp(s.p, kExtendedMagic, 4) != 0) return fail(MCK_ECORRUPT, "Bad extended magic number");
    f->footer_checksum = fixed32(s.p + 4);
    f->base_context_checksum = fixed32(s.p + 8);
    if (f->base_context_checksum == 0) return fail(MCK_ECORRUPT, "Invalid base context checksum");
    const uint32_t metaindex_size = fixed32(s.p + 12);
    if (fixed64(s.p + 32) != 0) return fail(MCK_ENOTSUP, "File uses a future feature not supported in this version");
    const uint64_t metaindex_end = f->footer_offset - kBlockTrailerSize;
    if (metaindex_size > metaindex_end) return fail(MCK_ECORRUPT, "bad metaindex size");
    f->metaindex_offset = metaindex_end - metaindex_size;
    f->metaindex_size = metaindex_size;
    f->has_index_handle = 0;  // in the metaindex ("rocksdb.index")
  } else {
    Handle m, x;
    if (!decode_handle(&s, &m) || !decode_handle(&s, &x)) return fail(MCK_ECORRUPT, "bad block handle");
    f->metaindex_offset = m.offset;
    f->metaindex_size = m.size;
    f->index_offset = x.offset;
    f->index_size = x.size;
    f->has_index_handle = 1;
  }
  return MCK_OK;
}

int mck_sst_list_blocks(const void* file, uint64_t file_size, mck_sst_footer* footer, mck_sst_block* blocks,
                        uint64_t cap, uint64_t* nblocks) {
  return mck_sst_list_blocks_uncompress(file, file_size, nullptr, nullptr, footer, blocks, cap, nblocks);
}

int mck_sst_index_handles(const void* contents, uint64_t size, int value_delta_encoded, uint32_t index_type, int kind,
                          mck_sst_block* out, uint64_t cap, uint64_t* n) {
  mck_internal_set_error("");
  if ((!contents && size) || !n) return fail(MCK_EINVAL, "NULL argument");
  if (index_type > 3) return fail(MCK_EINVAL, "index_type %u is not a block-based table index type", index_type);
  std::vector<Handle> hs;
  if (int rc = File::index_handles(Slice{static_cast<const uint8_t*>(contents), size}, value_delta_encoded != 0,
                                   index_type == 3, "index", &hs))
    return rc;
  *n = hs.size();
  if (out) {
    if (cap < hs.size())
      return fail(MCK_EINVAL, "capacity %llu < %llu", (unsigned long long)cap, (unsigned long long)hs.size());
    for (size_t i = 0; i < hs.size(); i++) out[i] = mck_sst_block{hs[i].offset, hs[i].size, kind, 0};
  }
  return MCK_OK;
}

int mck_sst_list_blocks_uncompress(const void* file, uint64_t file_size, mck_sst_uncompress_fn uncompress, void* ctx,
                                   mck_sst_footer* footer, mck_sst_block* blocks, uint64_t cap, uint64_t* nblocks) {
  mck_internal_set_error("");
  if (!file || !footer || !nblocks) return fail(MCK_EINVAL, "NULL argument");
  const uint8_t* d = static_cast<const uint8_t*>(file);
  const uint64_t tail = file_size < kNewVersionsEncodedLength ? file_size : kNewVersionsEncodedLength;
  if (int rc = mck_sst_decode_footer(d + file_size - tail, tail, file_size - tail, footer)) return rc;
  File F(d, file_size, uncompress, ctx);
  std::vector<mck_sst_block> out;
  auto add = [&](uint64_t off, uint64_t size, int kind) { out.push_back(mck_sst_block{off, size, kind, 0}); };

  // metaindex: name -> handle (VerifyChecksumInMetaBlocks)
  Handle mh{footer->metaindex_offset, footer->metaindex_size};
  Slice mb;
  if (int rc = F.payload(mh, "metaindex", &mb)) return rc;
  add(mh.offset, mh.size, MCK_SST_BLOCK_METAINDEX);
  std::vector<Entry> meta;
  if (int rc = File::entries(mb, "metaindex", &meta)) return rc;
  Handle props;
  bool have_props = false;
  std::vector<std::pair<Handle, int>> filter_partition_indexes;
  for (const Entry& e : meta) {
    Slice v = e.value;
    Handle h;
    if (!decode_handle(&v, &h)) return fail(MCK_ECORRUPT, "bad block handle");
    const int kind = meta_kind(e.key);
    if (kind == MCK_SST_BLOCK_INDEX) {  // format_version >= 6
      footer->index_offset = h.offset;
      footer->index_size = h.size;
      footer->has_index_handle = 1;
      continue;  // listed with the index below
    }
    if (kind == MCK_SST_BLOCK_PROPERTIES) {
      props = h;
      have_props = true;
    }
    if (kind == MCK_SST_BLOCK_FILTER_PARTITION_INDEX) filter_partition_indexes.push_back({h, kind});
    add(h.offset, h.size, kind);
  }
  if (!footer->has_index_handle) return fail(MCK_ECORRUPT, "Cannot find the index block handle in the metaindex");

  // properties: index type (fixed32 user property), value delta encoding
  // (varint64 integer property); absent = kBinarySearch, full values
  uint32_t index_type = 0;
  uint64_t delta = 0;
  if (have_props) {
    Slice pb;
    if (int rc = F.payload(props, "properties", &pb)) return rc;
    std::vector<Entry> pe;
    if (int rc = File::entries(pb, "properties", &pe)) return rc;
    for (const Entry& e : pe) {
      Slice v = e.value;
      if (e.key == "rocksdb.block.based.table.index.type" && v.n >= 4) index_type = fixed32(v.p);
      if (e.key == "rocksdb.index.value.is.delta.encoded" && !varint64(&v, &delta))
        return fail(MCK_ECORRUPT, "bad integer table property");
    }
  }
  footer->index_type = index_type;
  footer->index_value_is_delta_encoded = delta != 0;
  const bool first_key = index_type == 3;  // kBinarySearchWithFirstKey

  // index (+ partitions for kTwoLevelIndexSearch) -> data blocks
  // (VerifyChecksumInBlocks walks the same handles)
  Handle ih{footer->index_offset, footer->index_size};
  Slice ib;
  if (int rc = F.payload(ih, "index", &ib)) return rc;
  add(ih.offset, ih.size, MCK_SST_BLOCK_INDEX);
  std::vector<Handle> level;
  if (int rc = File::index_handles(ib, delta != 0, first_key, "index", &level)) return rc;
  if (index_type == 2) {  // kTwoLevelIndexSearch: the top level lists partitions
    std::vector<Handle> parts = level, data;
    for (const Handle& p : parts) {
      Slice pb;
      if (int rc = F.payload(p, "index partition", &pb)) return rc;
      add(p.offset, p.size, MCK_SST_BLOCK_INDEX_PARTITION);
      if (int rc = File::index_handles(pb, delta != 0, false, "index partition", &data)) return rc;
    }
    level.swap(data);
  }
  for (const Handle& h : level) add(h.offset, h.size, MCK_SST_BLOCK_DATA);
  // partitioned filters: the partition index lists the filter partitions
  for (auto& fp : filter_partition_indexes) {
    Slice fb;
    if (int rc = F.payload(fp.first, "filter partition index", &fb)) return rc;
    std::vector<Handle> fparts;
    if (int rc = File::index_handles(fb, delta != 0, false, "filter partition index", &fparts)) return rc;
    for (const Handle& h : fparts) add(h.offset, h.size, MCK_SST_BLOCK_FILTER_PARTITION);
  }
  for (const mck_sst_block& b : out)
    if (b.offset > file_size || b.size > file_size - b.offset || file_size - b.offset - b.size < kBlockTrailerSize)
      return fail(MCK_ECORRUPT, "block handle (offset %llu, size %llu) is past the end of the file",
                  (unsigned long long)b.offset, (unsigned long long)b.size);
  *nblocks = out.size();
  if (blocks) {
    if (cap < out.size()) return fail(MCK_EINVAL, "blocks capacity %llu < %llu", (unsigned long long)cap,
                                      (unsigned long long)out.size());
    if (!out.empty()) memcpy(blocks, out.data(), out.size() * sizeof(mck_sst_block));
  }
  return MCK_OK;
}

// table/format.cc:405-440: the format_version 6 footer checksum = the
// builtin checksum of the 53-byte footer with its checksum field zeroed,
// plus the context modifier of the footer's offset.  Computed with the
// engine's builtin-checksum shim (on the GPU).
int mck_sst_verify_footer(const void* footer53, const mck_sst_footer* f) {
  mck_internal_set_error("");
  if (!footer53 || !f) return fail(MCK_EINVAL, "NULL argument");
  if (f->format_version < 6 || f->checksum_type == MCK_kNoChecksum) return MCK_OK;
  uint8_t copy[kNewVersionsEncodedLength];
  memcpy(copy, footer53, sizeof copy);
  memset(copy + 5, 0, 4);
  const uint32_t c = mck_builtin_checksum(f->checksum_type, copy, sizeof copy);
  if (mck_last_error()[0]) return MCK_EHIP;
  const uint32_t computed = c + mck_context_modifier(f->base_context_checksum, f->footer_offset);
  if (computed != f->footer_checksum)
    return fail(MCK_ECORRUPT, "Footer at %llu checksum mismatch", (unsigned long long)f->footer_offset);
  return MCK_OK;
}

}  // extern "C"
