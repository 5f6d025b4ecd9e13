// Host-side timing of mck_wal_recover's walks (no GPU): a synthetic log of
// logical records of [lo, hi] bytes written in the log format (7-byte
// headers, 32 KiB blocks, zero trailers; CRCs not computed -- the plan walk
// trusts them), then the block walk, the reader's walk over it and the
// descriptor build, each timed.
//   g++ -O2 -std=c++17 -pthread microbench/walk_time.cc speedb_amd/csrc/mck_wal.cc -o /tmp/walk_time
//   /tmp/walk_time <log MiB> <lo> <hi>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../speedb_amd/csrc/mck_walk.h"

using namespace mck_walk;

extern "C" void mck_internal_set_error(const char*) {}

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const uint64_t target = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 1024) << 20;
  const uint32_t lo = argc > 2 ? atoi(argv[2]) : 100, hi = argc > 3 ? atoi(argv[3]) : 4096;
  std::vector<uint8_t> img;
  img.reserve(target + (1 << 20));
  std::mt19937_64 rng(7);
  uint64_t nrec = 0;
  while (img.size() < target) {
    uint32_t left = lo + (uint32_t)(rng() % (hi - lo + 1));
    bool first = true;
    while (true) {
      uint32_t boff = (uint32_t)(img.size() % 32768), room = 32768 - boff;
      if (room < 7) {
        img.resize(img.size() + room, 0);
        continue;
      }
      const uint32_t n = std::min(left, room - 7);
      const bool end = n == left;
      const uint8_t type = first && end ? 1 : first ? 2 : end ? 4 : 3;
      const uint8_t h[7] = {1, 2, 3, 4, (uint8_t)n, (uint8_t)(n >> 8), type};
      img.insert(img.end(), h, h + 7);
      img.resize(img.size() + n, (uint8_t)nrec);
      left -= n;
      first = false;
      if (end) break;
    }
    nrec++;
  }
  printf("log %.1f MiB, %lu records of %u-%u B\n", img.size() / 1048576.0, (unsigned long)nrec, lo, hi);
  for (int rep = 0; rep < 3; rep++) {
    double t0 = now();
    std::vector<PhysRec> phys;
    std::vector<BlockStop> stops;
    wal_block_walk(img.data(), img.size(), 0, phys, stops);
    double t1 = now();
    WalWalk W;
    int rc = wal_walk(img.data(), img.size(), 0, MCK_WAL_kTolerateCorruptedTailRecords, nullptr, W, &phys);
    double t2 = now();
    std::vector<mck_wal_rec_desc> desc(phys.size());
    for (size_t i = 0; i < phys.size(); i++) {
      const PhysRec& p = phys[i];
      const uint64_t po = p.hoff + p.hsize;
      desc[i] = mck_wal_rec_desc{(uint32_t)po, (uint32_t)(po >> 32) | ((uint32_t)p.type << 16), p.length, p.stored};
    }
    double t3 = now();
    WalWalk F;
    const bool fast = wal_walk_fast(img.size(), phys, stops, F);
    double t4 = now();
    printf("fast walk %s %.1f ms (%.1f ns/record), same records %d\n", fast ? "ran" : "declined", (t4 - t3) * 1e3,
           (t4 - t3) * 1e9 / W.roff.size(), (int)(F.roff == W.roff && F.rfrag == W.rfrag && F.rhoff == W.rhoff));
    printf("rc %d phys %zu records %zu: block walk %.1f ms, reader walk %.1f ms (%.1f ns/record), desc %.1f ms\n", rc,
           phys.size(), W.roff.size(), (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t2 - t1) * 1e9 / W.roff.size(),
           (t3 - t2) * 1e3);
  }
  return 0;
}
