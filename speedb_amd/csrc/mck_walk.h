// mck_walk.h -- the host log::Reader walk shared by mck_wal_read_records
// (mck_wal.cc, plain C++: the parsers' sanitizer build compiles it with g++)
// and mck_wal_recover (mck_walrec.cc, HIP runtime).
#pragma once
#include <stdint.h>

#include <vector>

#include "../../include/speedb_amd/mck.h"

namespace mck_walk {

// What one whole-log ReadRecord walk produced (mck_wal_read_records'
// outputs, plus per record the (block, k) slot of a one-fragment record).
struct WalWalk {
  std::vector<mck_wal_fragment> fr;
  std::vector<uint64_t> roff, rfile;
  std::vector<uint32_t> rlen;
  std::vector<uint64_t> rhoff;  // one-fragment record: its physical record's header offset; ~0 = fragmented
  std::vector<uint64_t> rfrag;  // record r's fragments: fr[rfrag[r] .. rfrag[r + 1])
  std::vector<mck_wal_report> reports;
  std::vector<uint64_t> report_pos;  // per report: records returned before it
  uint64_t dropped = 0, end_offset = 0, records_bytes = 0;
  uint32_t compression = 0;
  std::vector<mck_wal_fragment> stream;
};

// Every physical record of every 32 KiB block, each block walked on its own
// from offset 0 as ReadPhysicalRecord parses it (db/log_reader.cc:450-584;
// k_wal_verify's walk): the records a reader can reach, whatever it drops.
struct PhysRec {
  uint64_t hoff;    // header offset
  uint32_t length;  // payload bytes
  uint8_t hsize;    // 7 or 11
  uint8_t type;
  uint32_t stored;  // the header's masked CRC
};
struct BlockStop {  // where the block's walk stopped, and why (MCK_WAL_* status)
  uint64_t first;   // its first record in the list
  uint32_t count;   // its records
  uint32_t pos;     // stop position in the block
  int32_t status;
};
void wal_block_walk(const uint8_t* d, uint64_t nbytes, uint32_t log_number, std::vector<PhysRec>& phys,
                    std::vector<BlockStop>& stops);
// log::Reader (checksum = true) reading the whole image: ReadRecord until it
// returns false, over the device's verdicts (NULL = trust every CRC).
// phys (optional): the block walk's records of the same image (their headers
// are prefetched ahead of the walk).
int wal_walk(const uint8_t* d, uint64_t nbytes, uint32_t log_number, int recovery_mode,
             const mck_wal_block_result* verified, WalWalk& W, const std::vector<PhysRec>* phys = nullptr);

// The same walk (verified = NULL) from the block walk's list alone, without
// reading the image again, when the log holds nothing the list does not
// describe: every block walked to its end (MCK_WAL_OK), only the full /
// first / middle / last types in a well-formed order.  Returns false (W
// untouched) otherwise; the caller then runs wal_walk.
bool wal_walk_fast(uint64_t nbytes, const std::vector<PhysRec>& phys, const std::vector<BlockStop>& stops,
                   WalWalk& W);

// mck_wal_read_out (caller arrays, *_cap sizes) from a walk
int wal_copy_out(const WalWalk& W, mck_wal_read_out* out);
// argument checks of the read-out entry points (struct_size, mode)
int check_read_args(const void* wal, uint64_t nbytes, int recovery_mode, const mck_wal_read_out* out);

}  // namespace mck_walk
