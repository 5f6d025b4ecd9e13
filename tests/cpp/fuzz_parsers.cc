// fuzz_parsers.cc -- TEST INFRASTRUCTURE: drives the engine's host-side
// parsers of untrusted file bytes (csrc/mck_sst.cc, mck_wal.cc, mck_blob.cc)
// over a corpus of damaged images, built together with them under
// -fsanitize=address,undefined (tests/test_parsers_sanitized.py).  Only the
// host code is built: the device entry points the parsers call are stubbed
// below (their values do not matter to memory safety).
//
// usage: fuzz_parsers <sst|wal|blob> file...
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/speedb_amd/mck.h"

static thread_local char g_err[512];
extern "C" void mck_internal_set_error(const char* msg) { snprintf(g_err, sizeof g_err, "%s", msg); }
extern "C" const char* mck_last_error(void) { return g_err; }
extern "C" uint32_t mck_context_modifier(uint32_t base, uint64_t offset) {
  const uint32_t all_or_nothing = 0u - (uint32_t)(base != 0);
  return (base ^ ((uint32_t)offset + (uint32_t)(offset >> 32))) & all_or_nothing;
}
extern "C" uint32_t mck_builtin_checksum(int type, const void* data, size_t n) {
  // touch every byte so an out-of-range span is caught by ASan
  uint32_t h = (uint32_t)type;
  const uint8_t* p = static_cast<const uint8_t*>(data);
  for (size_t i = 0; i < n; i++) h = h * 31 + p[i];
  return h;
}

static std::vector<uint8_t> slurp(const char* path) {
  std::vector<uint8_t> v;
  FILE* f = fopen(path, "rb");
  if (!f) return v;
  uint8_t buf[65536];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) v.insert(v.end(), buf, buf + n);
  fclose(f);
  return v;
}

// Copy into an exactly-sized heap buffer so any read past the image is an
// ASan report (a vector's capacity could hide it).
static uint8_t* exact(const std::vector<uint8_t>& v) {
  uint8_t* p = static_cast<uint8_t*>(malloc(v.size() ? v.size() : 1));
  if (v.size()) memcpy(p, v.data(), v.size());
  return p;
}

static void run_sst(const uint8_t* d, uint64_t n) {
  mck_sst_footer f;
  if (n >= 48) {
    const uint64_t tl = n < 53 ? n : 53;
    (void)mck_sst_decode_footer(d + n - tl, tl, n - tl, &f);
  }
  uint64_t cnt = 0;
  if (mck_sst_list_blocks(d, n, &f, nullptr, 0, &cnt) == MCK_OK && cnt < (1u << 22)) {
    std::vector<mck_sst_block> b(cnt ? cnt : 1);
    (void)mck_sst_list_blocks(d, n, &f, b.data(), cnt, &cnt);
    if (n >= 53 && f.footer_offset + 53 <= n) (void)mck_sst_verify_footer(d + f.footer_offset, &f);
  }
}

static void run_wal(const uint8_t* d, uint64_t n) {
  const uint64_t nb = (n + 32767) / 32768;
  std::vector<mck_wal_block_result> ok(nb ? nb : 1);
  for (auto& r : ok) r = mck_wal_block_result{0, MCK_WAL_OK, 32768, 0};
  for (int mode = 0; mode < 4; mode++)
    for (int v = 0; v < 2; v++)
      for (uint32_t ln : {0u, 123u}) {
        mck_wal_read_out o;
        memset(&o, 0, sizeof o);
        o.struct_size = sizeof o;
        if (mck_wal_read_records(d, n, ln, mode, v ? ok.data() : nullptr, &o) != MCK_OK) continue;
        std::vector<mck_wal_fragment> fr(o.nfrags ? o.nfrags : 1);
        std::vector<uint64_t> ro(o.nrecords ? o.nrecords : 1), rf(ro.size());
        std::vector<uint32_t> rl(ro.size());
        std::vector<mck_wal_report> rep(o.nreports ? o.nreports : 1);
        mck_wal_read_out o2 = o;
        o2.frags = fr.data();
        o2.frag_cap = o.nfrags;
        o2.rec_offsets = ro.data();
        o2.rec_lengths = rl.data();
        o2.rec_file_offsets = rf.data();
        o2.rec_cap = o.nrecords;
        o2.reports = rep.data();
        o2.report_cap = o.nreports;
        if (mck_wal_read_records(d, n, ln, mode, v ? ok.data() : nullptr, &o2) != MCK_OK) abort();
        // every fragment lies inside the image and the record buffer
        for (uint64_t i = 0; i < o2.nfrags; i++)
          if (fr[i].src_off + fr[i].length > n || fr[i].dst_off + fr[i].length > o2.records_bytes) abort();
        for (uint64_t r = 0; r < o2.nreports; r++) (void)strlen(mck_wal_reason_string(rep[r].reason));
      }
  uint64_t nf = 0;
  (void)mck_wal_list_records(d, n, 0, nullptr, 0, &nf, nullptr, nullptr, 0, nullptr, nullptr);
  // the write plan over record sizes taken from the bytes
  std::vector<uint64_t> so;
  std::vector<uint32_t> ln;
  uint64_t pos = 0;
  for (uint64_t i = 0; i + 2 <= n && so.size() < 4096; i += 2) {
    const uint32_t len = (uint32_t)d[i] | ((uint32_t)d[i + 1] << 8);
    so.push_back(pos);
    ln.push_back(len * (1 + (d[i] & 3)));
    pos += ln.back();
  }
  uint64_t cnt = 0, ob = 0;
  uint32_t nbo = 0;
  const uint32_t bo = n ? (uint32_t)(d[0] * 131u) % 32769u : 0;
  if (mck_wal_plan(so.data(), ln.data(), (uint32_t)so.size(), bo, n & 1, nullptr, 0, &cnt, &ob, &nbo) == MCK_OK) {
    std::vector<mck_wal_fragment> fr(cnt ? cnt : 1);
    (void)mck_wal_plan(so.data(), ln.data(), (uint32_t)so.size(), bo, n & 1, fr.data(), cnt, &cnt, &ob, &nbo);
  }
}

static void run_blob(const uint8_t* d, uint64_t n) {
  mck_blob_file_info info;
  uint64_t cnt = 0;
  if (mck_blob_list_records(d, n, &info, nullptr, 0, &cnt) == MCK_OK && cnt < (1u << 22)) {
    std::vector<mck_blob_record> r(cnt ? cnt : 1);
    (void)mck_blob_list_records(d, n, &info, r.data(), cnt, &cnt);
    for (uint64_t i = 0; i < cnt; i++)
      if (r[i].offset + 32 + r[i].key_size + r[i].value_size > n) abort();
  }
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s <sst|wal|blob> file...\n", argv[0]);
    return 2;
  }
  const std::string kind = argv[1];
  for (int i = 2; i < argc; i++) {
    const std::vector<uint8_t> v = slurp(argv[i]);
    uint8_t* d = exact(v);
    if (kind == "sst")
      run_sst(d, v.size());
    else if (kind == "wal")
      run_wal(d, v.size());
    else
      run_blob(d, v.size());
    free(d);
  }
  printf("ok %d\n", argc - 2);
  return 0;
}
