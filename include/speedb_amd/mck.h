/*
 * mck.h -- C ABI of the MI355X block-checksum engine ("mck" = MI355X
 * checksum kernels).
 *
 * This is the drop-in boundary for Speedb's per-block checksum path.  The
 * reference has no plugin slot for block checksums (ChecksumType is a closed
 * enum, include/rocksdb/table.h:69-75); its boundary is a set of internal C++
 * functions, each of which is replaced below by an extern "C" entry point with
 * plain pointers and sizes.  INTEGRATION.md shows the reference-side binding.
 *
 * Two families:
 *   1. Scalar, signature-compatible shims (host pointers, synchronous).  The
 *      u32 algebra (Mask/Unmask/Combine/context modifier) runs on the host;
 *      every function that reads data bytes runs on the GPU.
 *   2. Batched device API: many independent spans per call, device-resident
 *      data, asynchronous on a HIP stream.  This is the hot path.
 *
 * Conventions (mirroring the reference):
 *   - return 0 on success, a negative MCK_E* code on argument/HIP errors; a
 *     checksum mismatch is data (an output), never an error;
 *   - the caller owns every buffer; nothing is allocated per call on the
 *     batched path;
 *   - reentrant and thread-safe; one engine context per device, created
 *     lazily on first use of that device;
 *   - data spans may start at any byte address; device buffers must be
 *     readable up to the next 16-byte boundary past each span (true of any
 *     hipMalloc allocation).
 */
#ifndef SPEEDB_AMD_MCK_H_
#define SPEEDB_AMD_MCK_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* A HIP stream (hipStream_t); NULL = the device's default stream. */
typedef struct ihipStream_t* mck_stream_t;

/* ---- error codes --------------------------------------------------------- */
#define MCK_OK 0
#define MCK_EINVAL (-1)   /* bad argument (NULL pointer, bad type, ...)     */
#define MCK_EHIP (-2)     /* a HIP runtime call failed; see mck_last_error */
#define MCK_ENODEV (-3)   /* no usable gfx950 device / device index       */
#define MCK_ENOMEM (-4)   /* staging allocation failed                    */
#define MCK_ECORRUPT (-5) /* corrupt SST structure (footer, handles ...)  */
#define MCK_ENOTSUP (-6)  /* valid but unsupported here (e.g. compressed index) */
#define MCK_EAGAIN (-7)   /* call again after supplying what the call asked for */

/* ---- checksum types: include/rocksdb/table.h:69-75 ChecksumType ---------- */
#define MCK_kNoChecksum 0
#define MCK_kCRC32c 1
#define MCK_kxxHash 2
#define MCK_kxxHash64 3
#define MCK_kXXH3 4

/* ---- WAL record types: db/log_format.h:22-45 ----------------------------- */
#define MCK_WAL_kBlockSize 32768
#define MCK_WAL_kHeaderSize 7
#define MCK_WAL_kRecyclableHeaderSize 11

/* Message of the last error on this thread ("" if none). */
const char* mck_last_error(void);
/* Engine version string. */
const char* mck_version(void);
/* Number of usable gfx950 devices (0 if none). */
int mck_device_count(void);

/* ========================================================================= */
/* 1. Scalar shims                                                          */
/* ========================================================================= */

/* util/crc32c.h:44 Mask / :50 Unmask (host, pure u32 algebra) */
uint32_t mck_crc32c_mask(uint32_t crc);
uint32_t mck_crc32c_unmask(uint32_t masked_crc);
/* util/crc32c.h:31 / util/crc32c.cc:1274 Crc32cCombine (host, O(log n)) */
uint32_t mck_crc32c_combine(uint32_t crc1, uint32_t crc2, size_t crc2len);
/* table/format.h:119 ChecksumModifierForContext (host) */
uint32_t mck_context_modifier(uint32_t base_context_checksum, uint64_t offset);

/* Data-reading shims.  Host pointers, synchronous; the bytes are staged to
 * the calling thread's current device and hashed there (one H2D copy, one
 * launch, one D2H copy per call: tens of microseconds -- see DESIGN.md
 * "Scalar shims" for the measured latency).  They exist so that a reference
 * call site CAN be re-pointed without a batching rewrite; they are not the
 * fast path.  INTEGRATION.md keeps the reference's CPU crc32c::Extend for
 * small synchronous calls and routes only batch-shaped callers to family 2.
 *
 * Error behaviour: the reference functions have no failure channel
 * (util/crc32c.h:26, include/rocksdb/file_checksum.h:47-49), so a plain
 * shim cannot return an error.  By default it FAILS LOUDLY: on any error --
 * in particular when mck_device_count() == 0 or a HIP call fails -- it
 * prints mck_last_error() to stderr and aborts, so a call site re-pointed at
 * a shim never stores a wrong checksum.  mck_set_shim_error_policy (or the
 * environment variable SPEEDB_AMD_SHIM_ERRORS=zero, read once) selects the
 * round-5 behaviour instead: return 0 with mck_last_error() set.  A caller
 * that must handle errors uses the *_r variants, which return 0 / MCK_E*
 * and write the result through `out`. */
#define MCK_SHIM_ERRORS_ABORT 0 /* default: message to stderr, abort()      */
#define MCK_SHIM_ERRORS_ZERO 1  /* return 0, mck_last_error() set            */
/* Called (when set) with the error message before the policy applies --
 * e.g. a maintainer's logger. */
typedef void (*mck_shim_error_handler)(const char* message, void* arg);
/* Process-wide; returns the previous policy, or MCK_EINVAL for an unknown
 * one. */
int mck_set_shim_error_policy(int policy, mck_shim_error_handler handler, void* arg);
/* util/crc32c.h:26 Extend, :35 Value */
uint32_t mck_crc32c_extend(uint32_t init_crc, const void* data, size_t n);
uint32_t mck_crc32c_value(const void* data, size_t n);
/* util/xxhash.h:5329 XXH3_64bits */
uint64_t mck_xxh3_64(const void* data, size_t n);
/* table/format.cc:578 ComputeBuiltinChecksum */
uint32_t mck_builtin_checksum(int type, const void* data, size_t n);
/* util/hash.h:45 NPHash64 / util/hash.cc:81 Hash64 (XXPH3, seeded) */
uint64_t mck_np_hash64(const void* data, size_t n, uint64_t seed);
/* table/format.cc:604 ComputeBuiltinChecksumWithLastByte */
uint32_t mck_builtin_checksum_with_last_byte(int type, const void* data,
                                             size_t n, char last_byte);

/* Error-returning variants of the shims above: 0 on success with the result
 * in *out, MCK_EINVAL / MCK_EHIP / MCK_ENODEV / MCK_ENOMEM otherwise (*out
 * = 0 then). */
int mck_crc32c_extend_r(uint32_t init_crc, const void* data, size_t n,
                        uint32_t* out);
int mck_crc32c_value_r(const void* data, size_t n, uint32_t* out);
int mck_xxh3_64_r(const void* data, size_t n, uint64_t* out);
int mck_builtin_checksum_r(int type, const void* data, size_t n,
                           uint32_t* out);
int mck_builtin_checksum_with_last_byte_r(int type, const void* data,
                                          size_t n, char last_byte,
                                          uint32_t* out);
int mck_np_hash64_r(const void* data, size_t n, uint64_t seed,
                    uint64_t* out);

/* ========================================================================= */
/* 2. Batched device API                                                    */
/* ========================================================================= */

/* A batch of independent byte spans in device memory.
 *   span i = [base + off_i, base + off_i + len_i)
 *   off_i  = offsets ? offsets[i] : i * stride
 *   len_i  = lengths ? lengths[i] : length
 * offsets/lengths, when given, are device arrays of `count` entries. */
typedef struct mck_spans {
  const void* base;
  const uint64_t* offsets;
  const uint32_t* lengths;
  uint64_t stride;
  uint32_t length;
  uint32_t count;
} mck_spans;

/* flags for mck_crc32c_batch */
#define MCK_F_MASK 1u /* store crc32c::Mask(crc) instead of crc */

/* out[i] = Extend(init_crcs ? init_crcs[i] : 0, span i)   (util/crc32c.h:26)
 * optionally masked.  out: device array [count]. */
int mck_crc32c_batch(const mck_spans* spans, const uint32_t* init_crcs,
                     uint32_t flags, uint32_t* out, mck_stream_t stream);

/* out[i] = XXH3_64bits(span i)   (util/xxhash.h:5329) */
int mck_xxh3_64_batch(const mck_spans* spans, uint64_t* out,
                      mck_stream_t stream);

/* out[i] = XXH32(span i, seed) / XXH64(span i, seed)  (legacy kxxHash /
 * kxxHash64 block checksums) */
int mck_xxh32_batch(const mck_spans* spans, uint32_t seed, uint32_t* out,
                    mck_stream_t stream);
int mck_xxh64_batch(const mck_spans* spans, uint64_t seed, uint64_t* out,
                    mck_stream_t stream);

/* out[i] = ComputeBuiltinChecksum(type, span i)                 if !last_bytes
 *        = ComputeBuiltinChecksumWithLastByte(type, span i, last_bytes[i])
 * (table/format.cc:578-645).  last_bytes: device array [count] or NULL. */
int mck_builtin_checksum_batch(int type, const mck_spans* spans,
                               const uint8_t* last_bytes, uint32_t* out,
                               mck_stream_t stream);

/* Write side of the SST trailer (table/block_based/block_based_table_builder.cc
 * :1333-1348): for every block payload span,
 *   out[i] = ComputeBuiltinChecksumWithLastByte(type, payload_i, comp_types[i])
 *            + ChecksumModifierForContext(base_context_checksum, file_off_i)
 * file_off_i = file_offsets ? file_offsets[i] : spans->offsets[i] (or
 * i*stride).  The caller writes [comp_type][LE32 out[i]] after the payload. */
int mck_sst_trailer_batch(int type, const mck_spans* payloads,
                          const uint8_t* comp_types,
                          const uint64_t* file_offsets,
                          uint32_t base_context_checksum, uint32_t* out,
                          mck_stream_t stream);

/* Read side (table/block_based/reader_common.cc:26 VerifyBlockChecksum):
 * every span is a block payload of len_i bytes followed in memory by its
 * 5-byte trailer [type][LE32 stored].  For block i:
 *   computed = ComputeBuiltinChecksum(type, payload_i || type_byte)
 *   stored   = LE32 - ChecksumModifierForContext(base, file_off_i)
 *   mismatch[i] = stored != computed
 * Outputs (device arrays, each optional except mismatch):
 *   mismatch[count] (uint8 0/1), computed[count], stored[count],
 *   mismatch_count (one uint32, atomically incremented per mismatch; the
 *   caller zeroes it). */
int mck_sst_verify_batch(int type, const mck_spans* payloads,
                         const uint64_t* file_offsets,
                         uint32_t base_context_checksum, uint8_t* mismatch,
                         uint32_t* computed, uint32_t* stored,
                         uint32_t* mismatch_count, mck_stream_t stream);

/* WAL record CRC, write side (db/log_writer.cc:263-311 EmitPhysicalRecord):
 * out[i] = Mask(crc of [type_i][LE32 log_number if recyclable][payload_i]).
 * types: device array [count].  recyclable = record type is 5..8 or 11. */
int mck_wal_record_crc_batch(const mck_spans* payloads, const uint8_t* types,
                             uint32_t log_number, uint32_t* out,
                             mck_stream_t stream);

/* ---- device WAL writer ------------------------------ */

/* One physical record of the write plan. */
typedef struct mck_wal_fragment {
  uint64_t src_off;  /* payload offset in the source buffer                */
  uint64_t dst_off;  /* header offset in the output stream                 */
  uint32_t length;   /* payload bytes (<= kBlockSize - header size)         */
  uint8_t type;      /* record type (db/log_format.h)                       */
  uint8_t pad;       /* zero bytes written just before the header (the
                        previous block's trailer, < header size)           */
  uint16_t reserved;
} mck_wal_fragment;

/* Host: log::Writer::AddRecord's fragmentation (db/log_writer.cc:79-175, no
 * WAL compression) of `count` logical records of host_lengths[r] bytes at
 * source offsets host_src_offsets[r], appended to a log whose current block
 * holds block_offset bytes.  Writes the fragments (frags = NULL queries the
 * count), the number of bytes the records add to the log (*out_bytes, incl.
 * block-trailer padding) and the writer's block_offset_ afterwards. */
int mck_wal_plan(const uint64_t* host_src_offsets, const uint32_t* host_lengths,
                 uint32_t count, uint32_t block_offset, int recycle,
                 mck_wal_fragment* frags, uint64_t cap, uint64_t* nfrags,
                 uint64_t* out_bytes, uint32_t* new_block_offset);

/* Device: write the planned physical records into `out` (device; byte
 * offsets of the plan relative to out) exactly as log::Writer appends them
 * (db/log_writer.cc:263-311 EmitPhysicalRecord): trailer zero padding,
 * [masked CRC LE32][length LE16][type][log number LE32 if recyclable],
 * payload.  frags: device array [nfrags]; crc_scratch: device u32 [nfrags]
 * (the masked fragment CRCs); out must be 16-byte aligned (any hipMalloc
 * allocation is).  One kernel computes every fragment's CRC and writes the
 * stream from the same registers (the payload is read once). */
int mck_wal_write_batch(const void* src, const mck_wal_fragment* frags,
                        uint32_t nfrags, uint32_t log_number,
                        uint32_t* crc_scratch, void* out, mck_stream_t stream);

/* ---- WAL recovery: logical records ----------------- */

/* Host: log::Reader::ReadRecord's reassembly (db/log_reader.cc:69-321) over a
 * WAL image in host memory: every logical record as the list of its
 * fragments' payloads (src_off = offset in the WAL image, dst_off = offset in
 * one contiguous record buffer, length, type) and the records themselves as
 * (rec_offsets[r], rec_lengths[r]) in that buffer.  Physical records are
 * walked as ReadPhysicalRecord does (32 KiB blocks, trailers, legacy and
 * recyclable headers, kZeroType padding); a bad length drops the rest of its
 * block, a record of another log (recycled file) or a truncated header ends
 * the walk; partial records are dropped as ReadRecord drops them.  CRCs are
 * NOT checked here (mck_wal_verify_batch does that on the device).  Any
 * output pointer may be NULL to query counts; *records_bytes = size of the
 * contiguous buffer. */
int mck_wal_list_records(const void* wal, uint64_t nbytes, uint32_t log_number,
                         mck_wal_fragment* frags, uint64_t frag_cap,
                         uint64_t* nfrags, uint64_t* rec_offsets,
                         uint32_t* rec_lengths, uint64_t rec_cap,
                         uint64_t* nrecords, uint64_t* records_bytes);

/* Device: copy every fragment's payload (wal + src_off, length bytes) to
 * out + dst_off -- reassembles the logical records of mck_wal_list_records
 * into one buffer, whose records' XXH3_64bits (ReadRecord's record_checksum,
 * db/log_reader.cc:107-158) are then one mck_xxh3_64_batch.  out: 16-byte
 * aligned device buffer. */
int mck_wal_gather_batch(const void* wal, const mck_wal_fragment* frags,
                         uint32_t nfrags, void* out, mck_stream_t stream);

/* Per-32KiB-block result of a WAL verify scan (db/log_reader.cc:450-584
 * ReadPhysicalRecord, checksum on).  Records of block b are walked in order;
 * the walk stops at the first record that the reference would not return. */
typedef struct mck_wal_block_result {
  uint32_t records_ok;   /* physical records that verified before the stop */
  int32_t status;        /* MCK_WAL_OK or the MCK_WAL_* reason for the stop */
  uint32_t stop_offset;  /* byte offset within the block of the stopping
                            record's header (block size if none)           */
  uint32_t bytes_ok;     /* header+payload bytes of the verified records   */
} mck_wal_block_result;

#define MCK_WAL_OK 0
#define MCK_WAL_BAD_CHECKSUM 1   /* kBadRecordChecksum: drop rest of block */
#define MCK_WAL_BAD_LENGTH 2     /* kBadRecordLen: header+length > block   */
#define MCK_WAL_ZERO_RECORD 3    /* kZeroType with length 0 (kBadRecord)  */
#define MCK_WAL_OLD_RECORD 4     /* recyclable record of another log      */
#define MCK_WAL_BAD_HEADER 5     /* truncated header at end of input      */

/* Verify every physical record of a WAL image of `nbytes` bytes (device
 * memory, starting at a 32 KiB block boundary; the last block may be
 * short).  results: device array [ceil(nbytes / 32768)]. */
int mck_wal_verify_batch(const void* wal, uint64_t nbytes,
                         uint32_t log_number, mck_wal_block_result* results,
                         mck_stream_t stream);

/* WAL recovery's device pass (DBImpl::RecoverLogFiles reads every record with
 * a record_checksum, db/db_impl/db_impl_open.cc:1217-1221): for every
 * physical record of a host plan of the log, its CRC32C verdict
 * (ReadPhysicalRecord, db/log_reader.cc:512-525) and -- from the SAME read of
 * its bytes -- the XXH3_64bits of its payload when asked (ReadRecord's
 * record_checksum of a one-fragment record is the fragment's XXH3,
 * :107-110).  The plan is what the reader's header walk yields
 * (mck_wal_recover builds it): per record the payload offset in the image,
 * its type, its length and the header's stored (masked) CRC. */
typedef struct mck_wal_rec_desc {
  uint32_t payload_off_lo; /* payload offset in the image, bits 0-31        */
  uint32_t hi;             /* bits 0-15: payload offset bits 32-47;
                              bits 16-23: record type (db/log_format.h);
                              bit 24: hash the payload (XXH3_64bits)      */
  uint32_t length;         /* payload bytes                               */
  uint32_t stored_crc;     /* the header's masked CRC (LE32 at the header) */
} mck_wal_rec_desc;
#define MCK_WAL_REC_HASH (1u << 24)
/* wal: the image in device memory (readable 16 bytes past its end);
 * recs: device array [count], in file order; crc_ok[i] = 1 when
 * Mask(Extend(type_crc[+log number], payload)) equals the stored CRC, else
 * 0; record_hashes[i] = XXH3_64bits(payload) of every record flagged
 * MCK_WAL_REC_HASH (others untouched).  Device arrays [count]. */
int mck_wal_recover_batch(const void* wal, const mck_wal_rec_desc* recs, uint32_t count,
                          uint32_t log_number, uint8_t* crc_ok, uint64_t* record_hashes,
                          mck_stream_t stream);
/* Host: the plan of a WAL image in host memory -- every physical record of
 * every 32 KiB block, each block walked from offset 0 as ReadPhysicalRecord
 * parses it (the records any reader of the log can reach), in file order,
 * MCK_WAL_REC_HASH set on the full-type ones (kFullType /
 * kRecyclableFullType).  out NULL: *count only. */
int mck_wal_plan_records(const void* wal, uint64_t nbytes, uint32_t log_number,
                         mck_wal_rec_desc* out, uint64_t cap, uint64_t* count);

/* ---- log::Reader, the whole log (db/log_reader.cc:69-584) ----------------- */

/* WALRecoveryMode (include/rocksdb/options.h) */
#define MCK_WAL_kTolerateCorruptedTailRecords 0
#define MCK_WAL_kAbsoluteConsistency 1
#define MCK_WAL_kPointInTimeRecovery 2
#define MCK_WAL_kSkipAnyCorruptedRecords 3

/* Reporter::Corruption reasons (the Status::Corruption messages of
 * db/log_reader.cc; mck_wal_reason_string gives the text) */
#define MCK_WAL_R_CHECKSUM_MISMATCH 1
#define MCK_WAL_R_BAD_RECORD_LENGTH 2
#define MCK_WAL_R_TRUNCATED_HEADER 3
#define MCK_WAL_R_TRUNCATED_BODY 4
#define MCK_WAL_R_ERROR_IN_MIDDLE 5
#define MCK_WAL_R_MISSING_START_1 6
#define MCK_WAL_R_MISSING_START_2 7
#define MCK_WAL_R_PARTIAL_WITHOUT_END_1 8
#define MCK_WAL_R_PARTIAL_WITHOUT_END_2 9
#define MCK_WAL_R_TRAILING_DATA 10
#define MCK_WAL_R_TS_INTERSPERSED 11
#define MCK_WAL_R_TS_DECODE 12
/* Reader::UpdateRecordedTimestampSize (db/log_reader.cc:594-616) */
#define MCK_WAL_R_TS_ZERO_SIZE 13
#define MCK_WAL_R_TS_CF_UPDATE 14
/* ReadRecord's kSetCompressionType case (db/log_reader.cc:167-188) */
#define MCK_WAL_R_COMPRESSION_MULTIPLE 15
#define MCK_WAL_R_COMPRESSION_NOT_FIRST 16
#define MCK_WAL_R_COMPRESSION_DECODE 17
/* "unknown record type %u" of header[6] read as a (signed) char: types
 * >= 128 print as 4294967xxx, as in the reference */
#define MCK_WAL_R_UNKNOWN_TYPE_BASE 256 /* + the record type byte */

/* One Reporter::Corruption(bytes, reason) call. */
typedef struct mck_wal_report {
  uint64_t offset; /* file offset of the physical record being read      */
  uint64_t bytes;  /* the dropped bytes the reader reports              */
  int32_t reason;  /* MCK_WAL_R_*                                        */
  uint32_t reserved;
} mck_wal_report;

/* Outputs of mck_wal_read_records.  Every array pointer may be NULL (counts
 * only); the *_cap fields give the array sizes.  Zero-initialise the struct
 * and set struct_size = sizeof(mck_wal_read_out): the library writes no field
 * past struct_size, and a caller whose struct ends before the compression
 * fields (MCK_WAL_READ_OUT_V1_SIZE) gets MCK_ENOTSUP for a compressed WAL
 * instead of a write past its struct.  Any other struct_size (e.g. a caller
 * built before struct_size became the first field, whose frags pointer sits
 * there) is refused with MCK_EINVAL, nothing written. */
typedef struct mck_wal_read_out {
  uint64_t struct_size;       /* sizeof(mck_wal_read_out) of the caller    */
  mck_wal_fragment* frags;    /* payload fragments of the returned records */
  uint64_t frag_cap;
  uint64_t nfrags;
  uint64_t* rec_offsets;      /* record r = [rec_offsets[r], +rec_lengths[r])
                                 of the contiguous record buffer           */
  uint32_t* rec_lengths;
  uint64_t* rec_file_offsets; /* file offset of the record's first physical
                                 record (LastRecordOffset)                */
  uint64_t rec_cap;
  uint64_t nrecords;
  uint64_t records_bytes;     /* size of the contiguous record buffer      */
  mck_wal_report* reports;    /* in order; up to report_cap are stored     */
  uint64_t report_cap;
  uint64_t nreports;
  uint64_t dropped_bytes;     /* sum of the reported bytes                 */
  uint64_t end_offset;        /* where ReadRecord returned false           */
  /* WAL compression (a kSetCompressionType record, db/log_writer.cc
   * AddCompressionTypeRecord): 0 = none, else the record's CompressionType
   * (kZSTD = 7).  From that record on, every physical record's payload is a
   * chunk of ONE streaming-compressed stream: `frags` then hold the
   * compressed chunks of each returned record, and the reader's
   * StreamingUncompress is fed every chunk in `stream` order (also chunks of
   * records later dropped, as ReadPhysicalRecord does, :534-571): stream[k]
   * .dst_off = the index in `frags` of that chunk, or ~0 when its record was
   * not returned.  Decompression, its errors (kBadRecord) and the XXH3
   * record checksum over the decompressed bytes are the caller's. */
  uint32_t compression_type;
  uint32_t reserved;
  mck_wal_fragment* stream;
  uint64_t stream_cap;
  uint64_t nstream;
} mck_wal_read_out;
/* struct_size of the layout without the compression fields */
#define MCK_WAL_READ_OUT_V1_SIZE 120

/* log::Reader (checksum = true, no WAL compression) reading a whole WAL
 * image in HOST memory: ReadRecord (db/log_reader.cc:69-321) called until it
 * returns false, over ReadPhysicalRecord (:450-584) and ReadMore, in the
 * given WALRecoveryMode.  The record CRCs are NOT computed here: `verified`
 * is the host copy of mck_wal_verify_batch's per-block results for the same
 * image (the device's verdict on every physical record); NULL trusts every
 * CRC.  Returns the logical records (as fragments of one contiguous buffer,
 * for mck_wal_gather_batch) and every corruption the reader would report,
 * with the bytes it drops.  A compressed WAL (kSetCompressionType record) is
 * walked and CRC-verified the same way; its records come back as compressed
 * chunks (see mck_wal_read_out.compression_type).  Results that do not
 * belong to the image: MCK_EINVAL. */
int mck_wal_read_records(const void* wal, uint64_t nbytes, uint32_t log_number,
                         int recovery_mode,
                         const mck_wal_block_result* verified,
                         mck_wal_read_out* out);

/* ---- WAL recovery with record checksums, one device pass ------------------ */
/* DBImpl::RecoverLogFiles' read loop (db/db_impl/db_impl_open.cc:1204-1221):
 * log::Reader::ReadRecord(&record, &scratch, mode, &record_checksum) until it
 * returns false, over a whole WAL image, with every CRC32C (ReadPhysicalRecord,
 * db/log_reader.cc:512-525) and every record's XXH3_64bits record_checksum
 * (:107-110 one fragment, :128-158 streamed over fragments) computed on the
 * device in ONE read of the image (mck_wal_recover_batch); multi-fragment
 * records are gathered and hashed in the same stream.  wal_host: the image in
 * host memory (the reader's header walk, as the reference reads it from the
 * file); wal_dev: the same nbytes in device memory (readable 16 bytes past
 * nbytes).  Synchronous: returns after the results are on the host.  The
 * result holds what mck_wal_read_records returns for the same image and mode
 * (records, fragments, reports, drops) plus the checksums.
 * *out: free with mck_wal_recovery_free. */
typedef struct mck_wal_recovery mck_wal_recovery;
int mck_wal_recover(const void* wal_host, const void* wal_dev, uint64_t nbytes,
                    uint32_t log_number, int recovery_mode, mck_stream_t stream,
                    mck_wal_recovery** out);
/* The walk's records, fragments and reports, exactly as mck_wal_read_records
 * fills `out` (same capacity rules: call with NULL arrays for the counts). */
int mck_wal_recovery_read_out(const mck_wal_recovery* r, mck_wal_read_out* out);
/* record_checksum (XXH3_64bits) of every returned record, in order
 * (cap >= nrecords).  MCK_ENOTSUP for a compressed WAL: there the reference
 * hashes the DECOMPRESSED record (db/log_reader.cc:537-571), the caller's. */
int mck_wal_recovery_checksums(const mck_wal_recovery* r, uint64_t* checksums,
                               uint64_t cap);
typedef struct mck_wal_recovery_info {
  uint64_t nrecords;
  uint64_t in_place;        /* one-fragment records hashed by the recover pass  */
  uint64_t gathered;        /* multi-fragment records (gather + XXH3 batch)     */
  uint64_t gathered_bytes;  /* their bytes                                      */
  uint32_t host_walks;      /* 1, or 2 when a CRC failed (walk over verdicts)    */
  uint32_t has_checksums;   /* 0: compressed WAL                                 */
  double walk_seconds;      /* host header walks                                 */
  double device_seconds;    /* device pass(es): launch to results on the host    */
} mck_wal_recovery_info;
int mck_wal_recovery_get_info(const mck_wal_recovery* r, mck_wal_recovery_info* info);
/* The device pass's per-block results (as mck_wal_verify_batch's), host copy;
 * cap >= ceil(nbytes / 32768). */
int mck_wal_recovery_block_results(const mck_wal_recovery* r, mck_wal_block_result* results,
                                   uint64_t cap);
/* Where each report of mck_wal_recovery_read_out falls in the record stream:
 * positions[i] = the records returned before report i, i.e. the reader's
 * Reporter::Corruption call for it happens inside the ReadRecord call that
 * returns record positions[i] (== nrecords: the final call, which returns
 * false).  cap >= nreports.  What a log::Reader::Reporter adapter needs to
 * replay the reports in the reference's order (integration/rocksdb_adapters.h). */
int mck_wal_recovery_report_positions(const mck_wal_recovery* r, uint64_t* positions, uint64_t cap);
void mck_wal_recovery_free(mck_wal_recovery* r);

/* Text of a MCK_WAL_R_* reason ("checksum mismatch", "unknown record type
 * 101", ...); Status::Corruption(reason).ToString() is "Corruption: " + it. */
const char* mck_wal_reason_string(int reason);

/* ---- log::FragmentBufferedReader: tailing a WAL that is being written ----
 * db/log_reader.cc:618-931 (ReadRecord, TryReadMore, TryReadFragment,
 * UnmarkEOF), the reader of secondary instances and WAL tailing
 * (allow_retry_read).  Unlike log::Reader it never treats a short read as
 * the end of the log: a record whose header or body is not yet written is
 * kept (its fragments across calls) and ReadRecord returns "no record yet";
 * the caller lets the file grow and calls again.  The file is a host image
 * that only grows (bytes already handed out must not change); its CRC
 * verdicts come from mck_wal_verify_batch over the same image, as for
 * mck_wal_read_records (a block verified while partially written must be
 * verified again once it grew).  No WAL compression (kSetCompressionType:
 * MCK_ENOTSUP), no I/O errors (a memory image cannot fail a read). */
typedef struct mck_wal_tail mck_wal_tail;

/* A reader of log `log_number` (checksum on).  *out = the reader. */
int mck_wal_tail_create(uint32_t log_number, mck_wal_tail** out);
void mck_wal_tail_destroy(mck_wal_tail* r);

/* The file as written so far: [wal, wal + nbytes) and the per-block verdicts
 * for it (NULL = trust every CRC).  Call before ReadRecord whenever the file
 * grew; the pointers must stay valid until the next call. */
int mck_wal_tail_set_image(mck_wal_tail* r, const void* wal, uint64_t nbytes,
                           const mck_wal_block_result* verified);

/* FragmentBufferedReader::ReadRecord.  Returns 1 with a record (*nfrags
 * payload fragments, *record_bytes, *last_record_offset = LastRecordOffset;
 * the fragments via mck_wal_tail_record_fragments), 0 when no complete
 * record is available yet, MCK_EAGAIN when it needs CRC verdicts no block
 * result holds (see mck_wal_tail_pending_verify), another negative MCK_E*
 * code on error. */
int mck_wal_tail_read_record(mck_wal_tail* r, uint64_t* nfrags, uint64_t* record_bytes,
                             uint64_t* last_record_offset);

/* The fragments of the record the last successful read returned (src_off in
 * the file, dst_off within the record); cap >= its nfrags. */
int mck_wal_tail_record_fragments(const mck_wal_tail* r, mck_wal_fragment* frags, uint64_t cap);

/* Reader::UnmarkEOF / IsEOF. */
int mck_wal_tail_unmark_eof(mck_wal_tail* r);
int mck_wal_tail_is_eof(const mck_wal_tail* r);

/* After MCK_EAGAIN: the reader passed a checksum failure inside a block that
 * was partly written when it was verified (the failure dropped a buffer that
 * ended at the file's end; the block then grew and UnmarkEOF reads on behind
 * it, db/log_reader.cc:340-397), and a block result stops at its block's
 * first failure.  Returns 1 with [*file_offset, +*nbytes) = the rest of that
 * block as written so far: verify it as one block (mck_wal_verify_batch over
 * wal + *file_offset, *nbytes bytes -> one result), hand the result to
 * mck_wal_tail_add_verdict and call ReadRecord again (nothing was consumed).
 * 0 when no verdict is pending. */
int mck_wal_tail_pending_verify(const mck_wal_tail* r, uint64_t* file_offset, uint64_t* nbytes);
int mck_wal_tail_add_verdict(mck_wal_tail* r, uint64_t file_offset, const mck_wal_block_result* result);

/* 1 when the last ReadRecord stopped at a recyclable record of an OLDER log
 * instance (its log number is not this reader's): *header_offset = that
 * header's file offset.  The reference's FragmentBufferedReader re-parses the
 * same header forever there (db/log_reader.cc:736-747 + :864-867); this
 * reader returns "no record" without consuming it, so every later call stops
 * at the same header whatever is appended -- a caller tells that stall apart
 * from "waiting for data" here.  0 otherwise. */
int mck_wal_tail_old_record(const mck_wal_tail* r, uint64_t* header_offset);

/* Reporter::Corruption calls so far: *n reports (up to cap stored) and the
 * total dropped bytes. */
int mck_wal_tail_reports(const mck_wal_tail* r, mck_wal_report* reports, uint64_t cap,
                         uint64_t* n, uint64_t* dropped_bytes);


/* ---- long spans / whole files ----------------------- */

/* Piece size of mck_crc32c_long (a multiple of the 4 KiB kernel round). */
#define MCK_LONG_PIECE_BYTES 65536u

/* uint32 scratch words mck_crc32c_long needs for an n-byte span. */
uint64_t mck_crc32c_long_scratch_words(uint64_t n);

/* *out = crc32c::Extend(init_crc, data, n) for ONE long device-resident span,
 * e.g. a whole SST/blob file image: util/file_checksum_helper.h:22-60
 * FileChecksumGenCrc32c (Extend over every Update, checksum_ starting at 0),
 * file/writable_file_writer.cc:100-131 (buffer CRC handoff).  The span is cut
 * into MCK_LONG_PIECE_BYTES pieces hashed in parallel by the batch kernel and
 * joined on the device with the Crc32cCombine algebra (util/crc32c.cc
 * :1221-1289).  data: any alignment; scratch: device array of
 * mck_crc32c_long_scratch_words(n) uint32; out: device pointer to one uint32.
 * Asynchronous on `stream`. */
int mck_crc32c_long(const void* data, uint64_t n, uint32_t init_crc,
                    uint32_t* scratch, uint32_t* out, mck_stream_t stream);

/* ---- per-KV protection ----------------------------- */

/* util/hash.h:45 NPHash64 == util/hash.cc:81 Hash64 == XXPH3_64bits_withSeed
 * (util/xxph3.h:1737), the XXH3 *preview* -- not XXH3_64bits.
 * out[i] = NPHash64(span i, seed). */
int mck_np_hash64_batch(const mck_spans* spans, uint64_t seed, uint64_t* out,
                        mck_stream_t stream);

/* db/kv_checksum.h ProtectionInfo64 of a batch of KVs (key span i, value
 * span i, same count):
 *   MCK_KV_PROTECT_KV    ProtectKV(key, value)                (:324)
 *   MCK_KV_PROTECT_KVO   ProtectKVO(key, value, op_types[i])  (:296)
 *   MCK_KV_PROTECT_KVOS  ProtectKVO(...).ProtectS(extras[i])  (:456; seqno)
 *   MCK_KV_PROTECT_KVOC  ProtectKVO(...).ProtectC(extras[i])  (:432; CF id)
 * out[i] = the u64 protection value; its Encode(len) form
 * (db/kv_checksum.h:80-98) is the low `len` bytes, little-endian.
 * op_types: device [count] (NULL = 0); extras: device [count] u64. */
#define MCK_KV_PROTECT_KV 0
#define MCK_KV_PROTECT_KVO 1
#define MCK_KV_PROTECT_KVOS 2
#define MCK_KV_PROTECT_KVOC 3
int mck_kv_protect_batch(int kind, const mck_spans* keys,
                         const mck_spans* values, const uint8_t* op_types,
                         const uint64_t* extras, uint64_t* out,
                         mck_stream_t stream);

/* ProtectionInfo::Verify(prot_bytes, stored + i*prot_bytes) (db/kv_checksum.h
 * :100-121) for every KV: mismatch[i] = 0/1; mismatch_count (optional,
 * caller-zeroed) counts mismatches; computed (optional) gets the u64 values.
 * prot_bytes: 1, 2, 4 or 8. */
int mck_kv_protect_verify_batch(int kind, const mck_spans* keys,
                                const mck_spans* values,
                                const uint8_t* op_types,
                                const uint64_t* extras, const uint8_t* stored,
                                uint32_t prot_bytes, uint8_t* mismatch,
                                uint32_t* mismatch_count, uint64_t* computed,
                                mck_stream_t stream);

/* ---- WritableFileWriter checksum handoff ------------ */

/* file/writable_file_writer.cc:743-747 Crc32cHandoffChecksumCalculation for
 * a batch of pieces about to be handed to FSWritableFile::Append:
 * out[i] = crc32c::Extend(0, piece i); its little-endian bytes are the
 * EncodeFixed32 checksum_buf of DataVerificationInfo (the device is
 * little-endian, so out viewed as bytes is [count][4] checksum_bufs).  The
 * writer's bookkeeping (buffered_data_crc32c_checksum_ via Crc32cCombine /
 * Extend, :99-165, :638-720) is host algebra over these values:
 * speedb_amd.handoff.WritableFileWriter. */
int mck_handoff_checksum_batch(const mck_spans* pieces, uint32_t* out,
                               mck_stream_t stream);

/* ---- per-KV protection of block entries ------------ */

/* table/block_based/block.cc:1091 Block::InitializeDataBlockProtectionInfo,
 * :1134 InitializeIndexBlockProtectionInfo, :1183
 * InitializeMetaIndexBlockProtectionInfo for a batch of uncompressed block
 * contents (the span of each block = its BlockContents, without the 5-byte
 * trailer).  For every entry k of block i, in iteration order:
 *   out[(key_base[i] + k) * prot_bytes ...] =
 *       ProtectionInfo64().ProtectKV(key, value).Encode(prot_bytes)
 * (block.h:271-274 GenerateKVChecksum) -- the block's kv_checksum_ array.
 * The key is the full reassembled key (iter->key()); the value is
 * iter->value() (data, metaindex) or iter->raw_value() (index: the encoded
 * IndexValue bytes).  `kind` names the iterator that parses the entries: */
#define MCK_BLOCK_DATA 0                  /* DataBlockIter (DecodeEntry)      */
#define MCK_BLOCK_INDEX 1                 /* IndexBlockIter, value_is_full    */
#define MCK_BLOCK_INDEX_DELTA 2           /* IndexBlockIter, delta-encoded
                                             values (format_version >= 4)     */
#define MCK_BLOCK_INDEX_DELTA_FIRST_KEY 3 /* ... + first key in the value
                                             (kBinarySearchWithFirstKey)      */
#define MCK_BLOCK_META 4                  /* MetaBlockIter (metaindex)        */

/* Per-block status.  A block that is not OK gets no keys -- the reference
 * sets its error marker (size_ = 0) and builds no protection. */
#define MCK_BLOCK_OK 0
#define MCK_BLOCK_BAD_CONTENTS 1 /* Block ctor error marker / NewDataIterator
                                    "bad block contents"                       */
#define MCK_BLOCK_BAD_ENTRY 2    /* "bad entry in block" (BlockIter::
                                    CorruptionError, block.h:559)             */
#define MCK_BLOCK_BAD_RESTARTS 3 /* restart array / intervals not as
                                    BlockBuilder writes them (restart[0] != 0,
                                    not increasing, shared != 0 at a restart,
                                    an interval other than the last holding
                                    fewer or more than block_restart_interval
                                    entries): the reference only asserts these
                                    and its output is undefined there          */
#define MCK_BLOCK_SLOT_OVERFLOW 4 /* one-pass entry points only: more than
                                     slot_cap entries, or a key longer than
                                     128 bytes and arena_cap; protect the
                                     block with the two-pass pair instead     */

/* Scratch for mck_block_kv_layout_batch (device bytes). */
uint64_t mck_block_kv_scratch_bytes(uint32_t count);

/* Pass 1 (device): every block's entry count and reassembled key bytes,
 * as exclusive scans: key_base[count + 1] (key_base[count] = total keys),
 * arena_base[count + 1] (total key bytes at [count]); status[count];
 * restart_interval[count] (GetRestartInterval, block.h:484; pass 2 reads it).
 * The caller reads key_base[count] and arena_base[count] back to size the
 * work area and the output. */
int mck_block_kv_layout_batch(int kind, const mck_spans* blocks,
                              uint64_t* key_base, uint64_t* arena_base,
                              uint32_t* restart_interval, int32_t* status,
                              void* scratch, mck_stream_t stream);

/* Device bytes of the work area of pass 2 (per-entry spans + key arena). */
uint64_t mck_block_kv_work_bytes(uint64_t total_keys, uint64_t total_key_bytes);

/* Pass 2: out = total_keys * prot_bytes bytes (device).  prot_bytes 1/2/4/8
 * (block_protection_bytes_per_key). */
int mck_block_kv_protect_batch(int kind, const mck_spans* blocks,
                               uint32_t prot_bytes, const uint64_t* key_base,
                               const uint64_t* arena_base,
                               const uint32_t* restart_interval,
                               uint64_t total_keys, void* work, uint8_t* out,
                               mck_stream_t stream);

/* Read side: the per-entry check DataBlockIter / IndexBlockIter /
 * MetaBlockIter run on every key they parse (block.h:567-574
 * PerKVChecksumCorruptionError) for all entries at once:
 * mismatch[key] = 0/1 against stored (the kv_checksum_ arrays, laid out as
 * `out` above); mismatch_count (optional, caller-zeroed) counts them. */
int mck_block_kv_verify_batch(int kind, const mck_spans* blocks,
                              uint32_t prot_bytes, const uint64_t* key_base,
                              const uint64_t* arena_base,
                              const uint32_t* restart_interval,
                              uint64_t total_keys, void* work,
                              const uint8_t* stored,
                              uint8_t* mismatch, uint32_t* mismatch_count,
                              mck_stream_t stream);

/* One pass (layout + protection in one walk of every block, no host
 * round trip): the outputs of mck_block_kv_layout_batch (key_base,
 * arena_base, restart_interval, status) and of mck_block_kv_protect_batch
 * (out, laid out by key_base) from one call.  Every block's entries are
 * parked in `slot_cap` 16-byte slots of the work area until the key index is
 * known; keys over 128 bytes use an `arena_cap`-byte slice per block.  A
 * block that does not fit gets MCK_BLOCK_SLOT_OVERFLOW and no keys.
 * out: count * slot_cap * prot_bytes bytes (room for any outcome; the
 * first key_base[count] * prot_bytes are written). */
uint64_t mck_block_kv_blocks_work_bytes(uint32_t count, uint32_t slot_cap,
                                        uint32_t arena_cap);
int mck_block_kv_protect_blocks_batch(int kind, const mck_spans* blocks,
                                      uint32_t prot_bytes, uint32_t slot_cap,
                                      uint32_t arena_cap, uint64_t* key_base,
                                      uint64_t* arena_base,
                                      uint32_t* restart_interval,
                                      int32_t* status, void* work,
                                      uint8_t* out, mck_stream_t stream);
/* ... and the read-side check in one pass.  key_base / total_keys are the
 * PROTECT-time key index (key_base[count + 1], device; total_keys =
 * key_base[count], at most count * slot_cap): `stored` and `mismatch` are laid
 * out by it, as the iterators index kv_checksum_ by the entry's position in
 * its own block (block.h:623).  mismatch: total_keys bytes.  status / restart
 * interval: the walk's.  A block whose walk now fails, or gives another entry
 * count than key_base, has every one of its keys flagged (the iterator's
 * CorruptionError, block.h:559-565) and no other block's keys move.  A block
 * with status MCK_BLOCK_SLOT_OVERFLOW is not verified (its keys are left
 * unflagged): re-verify the batch with mck_block_kv_verify_batch. */
int mck_block_kv_verify_blocks_batch(int kind, const mck_spans* blocks,
                                     uint32_t prot_bytes, uint32_t slot_cap,
                                     uint32_t arena_cap,
                                     const uint64_t* key_base,
                                     uint64_t total_keys,
                                     uint32_t* restart_interval,
                                     int32_t* status, void* work,
                                     const uint8_t* stored, uint8_t* mismatch,
                                     uint32_t* mismatch_count,
                                     mck_stream_t stream);

/* ---- SST files: whole-file verification ------------- */

/* Footer of a block-based table (table/format.h Footer). */
typedef struct mck_sst_footer {
  uint64_t magic;                  /* table magic (legacy magic upconverted) */
  uint32_t format_version;
  int32_t checksum_type;           /* MCK_k* */
  uint32_t base_context_checksum;  /* format_version >= 6, else 0          */
  uint32_t footer_checksum;        /* format_version >= 6: stored value    */
  uint32_t block_trailer_size;     /* 5                                     */
  uint32_t has_index_handle;       /* 0 until the metaindex supplied it (v6) */
  uint64_t footer_offset;
  uint64_t metaindex_offset, metaindex_size;
  uint64_t index_offset, index_size;
  uint32_t index_type;             /* BlockBasedTableOptions::IndexType     */
  uint32_t index_value_is_delta_encoded;
} mck_sst_footer;

/* Block kinds (table/block_based/block_type.h, meta block names of
 * table/meta_blocks.cc:29-35, block_based_table_builder.cc:2096-2100). */
#define MCK_SST_BLOCK_DATA 0
#define MCK_SST_BLOCK_INDEX 1
#define MCK_SST_BLOCK_INDEX_PARTITION 2
#define MCK_SST_BLOCK_METAINDEX 3
#define MCK_SST_BLOCK_PROPERTIES 4
#define MCK_SST_BLOCK_FILTER 5
#define MCK_SST_BLOCK_FILTER_PARTITION_INDEX 6
#define MCK_SST_BLOCK_FILTER_PARTITION 7
#define MCK_SST_BLOCK_RANGE_DEL 8
#define MCK_SST_BLOCK_COMPRESSION_DICT 9
#define MCK_SST_BLOCK_OTHER_META 10

/* One checksummed block: payload [offset, offset + size), then its 5-byte
 * trailer [compression type][LE32 checksum + context modifier]. */
typedef struct mck_sst_block {
  uint64_t offset;
  uint64_t size;
  int32_t kind;
  uint32_t reserved;
} mck_sst_block;

/* table/format.cc:348-470 Footer::DecodeFrom on the last tail_len bytes of a
 * file (tail_offset = their file offset; tail_len >= 48, normally 53).
 * Host memory, no device work; the v6 footer checksum is checked by
 * mck_sst_verify_footer.  MCK_ECORRUPT / MCK_ENOTSUP with the reference's
 * message in mck_last_error(). */
int mck_sst_decode_footer(const void* tail, uint64_t tail_len,
                          uint64_t tail_offset, mck_sst_footer* footer);

/* Every checksummed block of an SST image held in HOST memory, in the order
 * BlockBasedTable::VerifyChecksum visits them (table/block_based/
 * block_based_table_reader.cc:2336-2500): metaindex, meta blocks, index (and
 * its partitions for kTwoLevelIndexSearch), data blocks, filter partitions.
 * Reads the footer, metaindex, properties (index type, value delta
 * encoding) and index blocks on the host.  blocks = NULL queries the count
 * (*nblocks).  Compressed index/meta blocks: MCK_ENOTSUP. */
int mck_sst_list_blocks(const void* file, uint64_t file_size,
                        mck_sst_footer* footer, mck_sst_block* blocks,
                        uint64_t cap, uint64_t* nblocks);

/* A compressed block's contents, supplied by the caller: called by
 * mck_sst_list_blocks_uncompress for every block the lister must read (index,
 * index partitions, filter partition index, metaindex, properties) whose
 * trailer names a compression type -- enable_index_compression is on by
 * default (include/rocksdb/table.h:541).  raw / raw_size = the stored payload
 * (the 5-byte trailer excluded), block_offset = its handle offset.  On MCK_OK
 * *out / *out_size are the uncompressed contents, valid until the listing call
 * returns (the callback's owner keeps them).  The reference-side callback is
 * UncompressBlockData (table/format.h:412) with the table's dictionary
 * (integration/rocksdb_adapters.h UncompressWithReference).  Any other return
 * value fails the listing with that code. */
typedef int (*mck_sst_uncompress_fn)(void* ctx, uint8_t compression_type,
                                     uint64_t block_offset, const void* raw,
                                     uint64_t raw_size, const void** out,
                                     uint64_t* out_size);

/* mck_sst_list_blocks for tables with compressed index / meta blocks: each is
 * uncompressed by `uncompress` (NULL = MCK_ENOTSUP, as mck_sst_list_blocks)
 * and then parsed as usual (table/block_based/block_based_table_reader.cc:
 * 2336-2412 reads the index through the block cache, i.e. uncompressed).
 * The listed handles, sizes and kinds are those of the stored blocks, which
 * is what mck_sst_verify_batch checks. */
int mck_sst_list_blocks_uncompress(const void* file, uint64_t file_size,
                                   mck_sst_uncompress_fn uncompress, void* ctx,
                                   mck_sst_footer* footer, mck_sst_block* blocks,
                                   uint64_t cap, uint64_t* nblocks);

/* The block handles ONE uncompressed index block lists, for a reader that
 * already holds the index contents (IndexBlockIter, table/block_based/
 * block.cc: every entry's value is an IndexValue -- a full BlockHandle, or
 * with value_delta_encoded and shared != 0 the varsigned size delta after the
 * previous handle -- followed, for index_type 3 (kBinarySearchWithFirstKey),
 * by the length-prefixed first key).  Every output handle gets `kind`
 * (MCK_SST_BLOCK_DATA for a single-level index or a partition,
 * MCK_SST_BLOCK_INDEX_PARTITION for a two-level index's top level).  out =
 * NULL queries the count (*n). */
int mck_sst_index_handles(const void* contents, uint64_t size,
                          int value_delta_encoded, uint32_t index_type,
                          int kind, mck_sst_block* out, uint64_t cap,
                          uint64_t* n);

/* table/format.cc:405-440: check the format_version 6 footer checksum of the
 * 53 footer bytes (host memory); 0 for older formats / kNoChecksum.  The
 * blocks themselves are verified with ONE mck_sst_verify_batch over the
 * listed handles (file image in device memory, offsets = handle offsets). */
int mck_sst_verify_footer(const void* footer53, const mck_sst_footer* footer);

/* ---- blob files: db/blob/blob_log_format.{h,cc} ------ */

#define MCK_BLOB_kHeaderSize 30        /* BlobLogHeader::kSize        */
#define MCK_BLOB_kFooterSize 32        /* BlobLogFooter::kSize        */
#define MCK_BLOB_kRecordHeaderSize 32  /* BlobLogRecord::kHeaderSize  */
#define MCK_BLOB_kMagicNumber 2395959u

/* Blob file header/footer fields (BlobLogHeader / BlobLogFooter). */
typedef struct mck_blob_file_info {
  uint32_t version;
  uint32_t column_family_id;
  uint8_t has_ttl;
  uint8_t compression;
  uint8_t has_footer;   /* the last 32 bytes start with the magic number */
  uint8_t reserved;
  uint64_t expiration_first, expiration_second;
  uint64_t footer_blob_count;
  uint32_t footer_crc;  /* stored; = Mask(Value(footer[0..28))) if intact */
  uint32_t reserved2;
} mck_blob_file_info;

/* One record: header at `offset`, then key_size + value_size blob bytes. */
typedef struct mck_blob_record {
  uint64_t offset;
  uint64_t key_size;
  uint64_t value_size;
} mck_blob_record;

/* Walk a blob file image in HOST memory (BlobLogSequentialReader order):
 * decode the header (BlobLogHeader::DecodeFrom), list every record by its
 * header's sizes, and decode the footer when the last 32 bytes start with
 * the magic number (its CRC -- footer_crc -- is for the caller to check on
 * the device, BlobLogFooter::DecodeFrom).  Host only, no device work.
 * records = NULL queries the count.  MCK_ECORRUPT with the
 * reference's message (e.g. "Error while decoding blob log header: Magic
 * number mismatch") on a structural error. */
int mck_blob_list_records(const void* file, uint64_t file_size,
                          mck_blob_file_info* info, mck_blob_record* records,
                          uint64_t cap, uint64_t* nrecords);

/* Every record of a device-resident blob file image in one batch
 * (BlobLogRecord::DecodeHeaderFrom + CheckBlobCRC, blob_log_format.cc
 * :103-135):
 *   write == 0: status[i] = (header CRC mismatch) | (blob CRC mismatch) << 1,
 *               mismatch_count (optional, caller-zeroed) += records with any;
 *   write != 0: BlobLogRecord::EncodeHeaderTo's CRC fields -- header_crc and
 *               blob_crc are computed and stored into each record header.
 * record_offsets: device u64 [count] (header offsets), blob_lengths: device
 * u32 [count] (key_size + value_size). */
int mck_blob_record_batch(int write, void* file, const uint64_t* record_offsets,
                          const uint32_t* blob_lengths, uint32_t count,
                          uint8_t* status, uint32_t* mismatch_count,
                          mck_stream_t stream);

/* ========================================================================= */
/* 3. Multi-GPU / host-resident input                                       */
/* ========================================================================= */

/* Split `count` spans with the given host-side lengths into `parts`
 * contiguous ranges of near-equal byte totals: range p = [first[p],
 * first[p+1]).  first: host array [parts + 1]. */
int mck_partition_spans(const uint32_t* host_lengths, uint32_t count,
                        uint32_t length, int parts, uint32_t* first);

/* Host-resident batch: spans live in host memory (pinned or pageable; pinned
 * gives full PCIe rate), sorted by offset.  The batch is partitioned by bytes
 * across devices [0, ndev) -- or, with ndev <= 0, runs on the calling
 * thread's current device only (one process per GPU); ndev above the
 * devices the process sees is MCK_ENODEV, not a clamp -- and streamed
 * through each device in double-buffered chunks of
 * `chunk_bytes` (H2D copy of chunk k+1 overlaps the kernel on chunk k); the
 * per-span results come back to host memory.
 * kind: MCK_kCRC32c (out32 = Value, masked if flags & MCK_F_MASK) or
 *       MCK_kXXH3 (out64 = XXH3_64bits).
 * host_offsets / host_lengths: host arrays (NULL => uniform as in mck_spans).
 * The per-device staging (two slots, each a stream, a device chunk buffer
 * of max(chunk_bytes, longest span + 32) bytes, and device + pinned
 * descriptor/result arrays) is allocated on a device's first call and reused
 * by later ones (grown when a call needs more); calls on one device are
 * serialised.  On any error every copy already queued has completed before
 * the call returns, and a failed allocation leaves nothing allocated.
 * Returns 0 on success.  *seconds (optional) = wall time of the call. */
int mck_host_batch_checksum(int kind, const void* host_base,
                            const uint64_t* host_offsets,
                            const uint32_t* host_lengths, uint64_t stride,
                            uint32_t length, uint32_t count, uint32_t flags,
                            int ndev, size_t chunk_bytes, uint32_t* out32,
                            uint64_t* out64, double* seconds);
/* Free the host pipeline's cached staging on every device. */
void mck_host_pipeline_release(void);

/* ========================================================================= */
/* 4. Statistics                                                            */
/* ========================================================================= */

/* Engine counters since load (or the last reset), process-wide:
 *   block_checksum_compute_count  BLOCK_CHECKSUM_COMPUTE_COUNT
 *                                 (include/rocksdb/statistics.h:451): blocks
 *                                 submitted to mck_sst_verify_batch (one per
 *                                 VerifyBlockChecksum)
 *   block_checksum_mismatch_count BLOCK_CHECKSUM_MISMATCH_COUNT (:455):
 *                                 blocks those verifies flagged, counted on
 *                                 each device (completed work only: sync the
 *                                 streams first)
 *   batches / spans               batched device calls and their spans
 *   bytes_known                   span bytes of the batches whose lengths the
 *                                 host knows (uniform batches, host batches);
 *                                 ragged device batches keep their lengths on
 *                                 the device and are not included */
typedef struct mck_statistics {
  uint64_t block_checksum_compute_count;
  uint64_t block_checksum_mismatch_count;
  uint64_t batches;
  uint64_t spans;
  uint64_t bytes_known;
} mck_statistics;

/* Fill *out (reads each initialised device's counters: synchronous);
 * reset != 0 zeroes them: each device's mismatch ticker (64-bit) is read and
 * cleared in one atomic exchange, so no count of a verify kernel running
 * concurrently is lost. */
int mck_statistics_get(mck_statistics* out, int reset);

/* PerfContext (include/rocksdb/perf_context.h:97 block_checksum_time; the
 * reference times every VerifyBlockChecksum with PERF_TIMER_GUARD,
 * table/block_based/reader_common.cc:29).  Per calling thread, as the
 * reference's thread-local perf context.  level: the reference's PerfLevel
 * values (include/rocksdb/perf_level.h: 1 kDisable, 2 kEnableCount -- the
 * default --, 3..5 also time).  At a timing level every
 * mck_sst_verify_batch call brackets its kernel(s) with two HIP events on
 * its stream; block_checksum_time is the DEVICE time of those batches in
 * nanoseconds, available once they completed: mck_perf_context_get waits
 * for this thread's outstanding batches.  block_checksum_count = blocks
 * verified (kEnableCount and up), batches = verify calls. */
#define MCK_PERF_kDisable 1
#define MCK_PERF_kEnableCount 2
#define MCK_PERF_kEnableTimeExceptForMutex 3
#define MCK_PERF_kEnableTime 5
typedef struct mck_perf_context {
  uint64_t block_checksum_time;   /* ns of device time, timed levels only */
  uint64_t block_checksum_count;  /* blocks verified */
  uint64_t block_checksum_batches;
} mck_perf_context;
int mck_set_perf_level(int level);
int mck_get_perf_level(void);
/* Fill *out for the calling thread (synchronous on this thread's timed
 * batches); reset != 0 zeroes it (PerfContext::Reset). */
int mck_perf_context_get(mck_perf_context* out, int reset);

/* Test hook: k > 0 makes mck_host_batch_checksum see k "devices" that are all
 * device 0, each with its own staging, streams and host thread, so the
 * ndev > 1 branch (per-device threads, concurrent first use, result
 * concatenation) runs on a one-GPU box; 0 restores the real devices.  Frees
 * the cached host pipelines.  Never used by production code. */
int mck_test_set_virtual_devices(int k);

/* TEST HOOK (parity tests only; never needed in production): a ragged CRC
 * batch runs each workgroup's share on the row drivers or the body/head
 * driver, chosen from a sample of its lengths, so a mixed parity batch may
 * exercise only one.  driver: 0 = by length (the default), 2 = 16-lane rows,
 * 3 = 8-lane rows, 5 = 4-lane rows, 6 = one lane per span, 7 = the
 * body/head driver, 9 = a wave per span wherever a workgroup's share allows
 * it (<= 16 spans of <= 16 KiB; by default only batches of <= 64 spans take
 * it) (1 and 4, the retired wave driver and unit stream, and 8 are
 * refused); interleaved != 0 deals spans to workgroups round-robin (row
 * drivers only) instead of in contiguous ranges.  Process-wide. */
int mck_test_set_crc_driver(int driver, int interleaved);
/* Test hook: the XXH3 driver for every batch -- 0 = by batch shape (rows for
 * uniform batches, a wave per span for ragged ones), 1 = a wave per span,
 * 2 = 16-lane rows.  Production code never calls it. */
int mck_test_set_xxh3_driver(int driver);
/* Test hook (host only): mck_wal_recover's plan walk from the block walk's
 * list (wal_walk_fast) against the reader's walk over the image, both with
 * every CRC trusted.  1 = the list walk ran and every output (fragments,
 * records, offsets, reports, end offset) equals the reader's; 0 = it
 * declined (the reader's walk is then the plan); -1 = they differ.
 * Production code never calls it. */
int mck_test_wal_walk_fast(const void* wal, uint64_t nbytes, uint32_t log_number);
/* Test hook: 0 sends uniform batches of <= 240-byte spans of the XXPH3
 * entry points (mck_np_hash64_batch, mck_kv_protect*_batch) to the row
 * driver instead of the lane-quad kernel (1, the default).  Process-wide;
 * production code never calls it. */
int mck_test_set_xph3_quads(int on);

#ifdef __cplusplus
}
#endif
#endif /* SPEEDB_AMD_MCK_H_ */
