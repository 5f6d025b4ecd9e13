/*
 * oracle.h -- CPU restatement of the reference's block-checksum path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in speedb_amd/ links, loads or calls
 * this code.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may use it, and only as the checker.
 *
 * Every function names the reference file:line whose behaviour it restates
 * (paths relative to the speedb-io/speedb tree).  The restatement is pinned
 * against the reference's own known-answer vectors (util/crc32c_test.cc,
 * table/table_test.cc BuiltinChecksumTest) and against oracle/_ref, a build
 * of the reference's util/crc32c.cc + util/xxhash.cc made by oracle/Makefile.
 */
#ifndef SPEEDB_AMD_ORACLE_H_
#define SPEEDB_AMD_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* util/crc32c.h:26 Extend, :35 Value */
uint32_t orc_crc32c_extend(uint32_t init_crc, const void* data, size_t n);
uint32_t orc_crc32c_value(const void* data, size_t n);
/* util/crc32c.h:44 Mask, :50 Unmask */
uint32_t orc_crc32c_mask(uint32_t crc);
uint32_t orc_crc32c_unmask(uint32_t masked);
/* util/crc32c.cc:1274 Crc32cCombine */
uint32_t orc_crc32c_combine(uint32_t crc1, uint32_t crc2, size_t crc2len);
/* "pure" state after appending n zero bytes (the zero-extension operator
 * behind util/crc32c.cc:1199 Crc32AppendZeroes) */
uint32_t orc_crc32c_zshift(uint32_t state, uint64_t nbytes);

/* util/file_checksum_helper.h:22-46 FileChecksumGenCrc32c: Update() =
 * crc32c::Extend from checksum_ = 0, Finalize() = PutFixed32 of
 * EndianSwapValue(checksum_), i.e. the 4 big-endian bytes of Value(file). */
void orc_file_checksum_crc32c(const void* data, size_t n, uint8_t out[4]);

/* util/xxhash.h:5329 XXH3_64bits (seed 0, default secret) */
uint64_t orc_xxh3_64(const void* data, size_t n);
/* util/xxhash.h XXH32 / XXH64 with a seed (kxxHash / kxxHash64) */
uint32_t orc_xxh32(const void* data, size_t n, uint32_t seed);
uint64_t orc_xxh64(const void* data, size_t n, uint64_t seed);

/* include/rocksdb/table.h:69-75 ChecksumType */
enum { ORC_kNoChecksum = 0, ORC_kCRC32c = 1, ORC_kxxHash = 2,
       ORC_kxxHash64 = 3, ORC_kXXH3 = 4 };

/* table/format.cc:578 ComputeBuiltinChecksum */
uint32_t orc_builtin_checksum(int type, const void* data, size_t n);
/* table/format.cc:604 ComputeBuiltinChecksumWithLastByte */
uint32_t orc_builtin_checksum_with_last_byte(int type, const void* data,
                                             size_t n, uint8_t last_byte);
/* table/format.h:119 ChecksumModifierForContext */
uint32_t orc_context_modifier(uint32_t base_context_checksum, uint64_t offset);
/* table/block_based/reader_common.cc:26 VerifyBlockChecksum: returns 1 if
 * the block [payload n][type][LE32 stored] verifies, 0 otherwise; writes the
 * (un-context-modified) stored value and the computed value. */
int orc_verify_block(int type, const void* block, size_t payload_len,
                     uint32_t base_context_checksum, uint64_t offset,
                     uint32_t* stored_out, uint32_t* computed_out);

/* db/log_writer.cc:263 EmitPhysicalRecord -- masked header CRC of one
 * physical record.  recyclable != 0 mixes the low 32 bits of log_number. */
uint32_t orc_wal_record_crc(uint8_t type, const void* payload, size_t n,
                            int recyclable, uint32_t log_number);

/* util/hash.cc:81 Hash64 == util/hash.h:45 NPHash64 == XXPH3_64bits_withSeed
 * (util/xxph3.h:1737), the preview XXH3 -- NOT XXH3_64bits. */
uint64_t orc_hash64(const void* data, size_t n, uint64_t seed);

/* db/kv_checksum.h per-KV protection (ProtectionInfo64), value as the
 * Encode(8) bytes read LE.  mode 0 ProtectKV; 1 ProtectKVO(op); 2 KVO then
 * ProtectS(seqno = extra); 3 KVO then ProtectC(cf = (uint32)extra). */
uint64_t orc_kv_protect(int mode, const void* key, size_t kn, const void* value,
                        size_t vn, uint8_t op, uint64_t extra);

/* Per-KV protection of one uncompressed block's entries
 * (table/block_based/block.cc:1091 InitializeDataBlockProtectionInfo, :1134
 * Index, :1183 MetaIndex).  kind: which iterator parses the entries. */
enum { ORC_BLOCK_DATA = 0, ORC_BLOCK_INDEX = 1, ORC_BLOCK_INDEX_DELTA = 2,
       ORC_BLOCK_INDEX_DELTA_FIRST_KEY = 3, ORC_BLOCK_META = 4 };
enum { ORC_BLOCK_OK = 0, ORC_BLOCK_BAD_CONTENTS = 1, ORC_BLOCK_BAD_ENTRY = 2,
       ORC_BLOCK_BAD_RESTARTS = 3 };
/* Writes nkeys * prot_bytes checksum bytes (as far as out_cap allows),
 * *nkeys_out and the restart interval; returns an ORC_BLOCK_* status. */
int orc_block_kv_protect(int kind, const void* block, size_t n, uint32_t prot_bytes, uint8_t* out,
                         size_t out_cap, uint32_t* nkeys_out, uint32_t* interval_out);

#ifdef __cplusplus
}
#endif
#endif /* SPEEDB_AMD_ORACLE_H_ */
