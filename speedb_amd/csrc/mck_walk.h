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
  std::vector<uint64_t> rblk;  // full-type record: its physical record's block; ~0 = multi-fragment
  std::vector<uint32_t> rk;    // ... and its index among the block's full-type records
  std::vector<uint64_t> rfrag;  // record r's fragments: fr[rfrag[r] .. rfrag[r + 1])
  std::vector<uint32_t> full_counts;  // per block (count_full)
  std::vector<mck_wal_report> reports;
  std::vector<uint64_t> report_pos;  // per report: records returned before it
  uint64_t dropped = 0, end_offset = 0, records_bytes = 0;
  uint32_t compression = 0;
  std::vector<mck_wal_fragment> stream;
};

// log::Reader (checksum = true) reading the whole image: ReadRecord until it
// returns false, over the device's verdicts (NULL = trust every CRC);
// count_full fills full_counts (full-type records per block).
int wal_walk(const uint8_t* d, uint64_t nbytes, uint32_t log_number, int recovery_mode,
             const mck_wal_block_result* verified, bool count_full, WalWalk& W);
// mck_wal_read_out (caller arrays, *_cap sizes) from a walk
int wal_copy_out(const WalWalk& W, mck_wal_read_out* out);
// argument checks of the read-out entry points (struct_size, mode)
int check_read_args(const void* wal, uint64_t nbytes, int recovery_mode, const mck_wal_read_out* out);

}  // namespace mck_walk
