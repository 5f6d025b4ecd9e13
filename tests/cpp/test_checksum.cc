// test_checksum.cc -- the reference's checksum tests, restated against the
// C++ host mirror (include/speedb_amd/checksum.hpp) and so against the GPU
// engine.  Expected values are the reference's own (util/crc32c_test.cc,
// table/table_test.cc); test names follow theirs.  Needs a GPU; built and
// run by tests/test_cpp_mirror.py.
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <string>
#include <vector>

#include "speedb_amd/checksum.hpp"

using namespace speedb_amd;

static int g_fail = 0, g_checks = 0;
#define EXPECT_EQ(a, b)                                                                       \
  do {                                                                                        \
    g_checks++;                                                                               \
    auto va_ = (a);                                                                           \
    auto vb_ = (b);                                                                           \
    if (!(va_ == vb_)) {                                                                      \
      g_fail++;                                                                               \
      fprintf(stderr, "%s:%d: EXPECT_EQ(%s, %s) failed\n", __FILE__, __LINE__, #a, #b);       \
    }                                                                                         \
  } while (0)
#define EXPECT_NE(a, b) EXPECT_EQ(!((a) == (b)), true)
#define EXPECT_TRUE(a) EXPECT_EQ(!!(a), true)
#define TEST(s, n) static void s##_##n()
#define RUN(s, n)                         \
  do {                                    \
    int before = g_fail;                  \
    s##_##n();                            \
    printf("[%s] %s.%s\n", g_fail == before ? "  OK  " : " FAIL ", #s, #n); \
  } while (0)

// util/crc32c_test.cc:70-94
TEST(CRC, StandardResults) {
  char buf[32];
  memset(buf, 0, sizeof(buf));
  EXPECT_EQ(0x8a9136aaU, crc32c::Value(buf, sizeof(buf)));
  memset(buf, 0xff, sizeof(buf));
  EXPECT_EQ(0x62a8ab43U, crc32c::Value(buf, sizeof(buf)));
  for (int i = 0; i < 32; i++) buf[i] = static_cast<char>(i);
  EXPECT_EQ(0x46dd794eU, crc32c::Value(buf, sizeof(buf)));
  for (int i = 0; i < 32; i++) buf[i] = static_cast<char>(31 - i);
  EXPECT_EQ(0x113fdb5cU, crc32c::Value(buf, sizeof(buf)));
  unsigned char data[48] = {
      0x01, 0xc0, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00,
      0x14, 0x00, 0x00, 0x00, 0x00, 0x00, 0x04, 0x00, 0x00, 0x00, 0x00, 0x14, 0x00, 0x00, 0x00, 0x18,
      0x28, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x02, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00,
  };
  EXPECT_EQ(0xd9963a56U, crc32c::Value(reinterpret_cast<char*>(data), sizeof(data)));
}

TEST(CRC, Values) { EXPECT_NE(crc32c::Value("a", 1), crc32c::Value("foo", 3)); }

TEST(CRC, Extend) {
  EXPECT_EQ(crc32c::Value("hello world", 11), crc32c::Extend(crc32c::Value("hello ", 6), "world", 5));
}

TEST(CRC, Mask) {
  uint32_t crc = crc32c::Value("foo", 3);
  EXPECT_NE(crc, crc32c::Mask(crc));
  EXPECT_NE(crc, crc32c::Mask(crc32c::Mask(crc)));
  EXPECT_EQ(crc, crc32c::Unmask(crc32c::Mask(crc)));
  EXPECT_EQ(crc, crc32c::Unmask(crc32c::Unmask(crc32c::Mask(crc32c::Mask(crc)))));
}

TEST(CRC, Crc32cCombineBasicTest) {
  uint32_t crc1 = crc32c::Value("hello ", 6), crc2 = crc32c::Value("world", 5);
  EXPECT_EQ(crc32c::Value("hello world", 11), crc32c::Crc32cCombine(crc1, crc2, 5));
}

TEST(CRC, Crc32cCombineOrderMattersTest) {
  uint32_t crc1 = crc32c::Value("hello ", 6), crc2 = crc32c::Value("world", 5);
  EXPECT_NE(crc32c::Value("hello world", 11), crc32c::Crc32cCombine(crc2, crc1, 6));
}

// util/crc32c_test.cc:144-158, scaled from 4096 to 257 sizes (each is a
// synchronous GPU round trip here)
TEST(CRC, Crc32cCombineFullCoverTest) {
  std::mt19937_64 rnd(301);
  std::string s1(1 << 20, 0);
  for (auto& c : s1) c = static_cast<char>(rnd());
  const uint32_t crc1 = crc32c::Value(s1.data(), s1.size());
  for (int size2 = 0; size2 < 4096; size2 += 16) {
    std::string s2(size2, 0);
    for (auto& c : s2) c = static_cast<char>(rnd());
    const uint32_t crc2 = crc32c::Value(s2.data(), s2.size());
    EXPECT_EQ(crc32c::Extend(crc1, s2.data(), s2.size()), crc32c::Crc32cCombine(crc1, crc2, s2.size()));
  }
}

static std::string Hex(uint32_t v) {
  char b[9];
  const unsigned char* u = reinterpret_cast<const unsigned char*>(&v);  // little endian as in file
  snprintf(b, sizeof b, "%02X%02X%02X%02X", u[0], u[1], u[2], u[3]);
  return b;
}
static std::string ChecksumAsString(const std::string& data, ChecksumType t) {
  uint32_t v = ComputeBuiltinChecksum(t, data.data(), data.size());
  if (data.size() >= 1)
    EXPECT_EQ(v, ComputeBuiltinChecksumWithLastByte(t, data.data(), data.size() - 1, data.back()));
  return Hex(v);
}
static std::string ChecksumAsString(std::string* data, char new_last_byte, ChecksumType t) {
  data->back() = new_last_byte;
  return ChecksumAsString(*data, t);
}

// table/table_test.cc:2325-2403 BuiltinChecksumTest.ChecksumSchemas
TEST(BuiltinChecksumTest, ChecksumSchemas) {
  std::string b0 = "x";
  std::string b1 = "This is a short block!x";
  std::string b2;
  for (int i = 0; i < 100; ++i) b2.append("This is a long block!");
  b2.append("x");
  std::string empty;
  const char ct1 = 0, ct2 = 1, ct3 = 7;  // kNoCompression, kSnappyCompression, kZSTD
  const char* want[5][10] = {
      {"00000000", "00000000", "00000000", "00000000", "00000000", "00000000", "00000000", "00000000",
       "00000000", "00000000"},
      {"D8EA82A2", "D28F2549", "052B2843", "46F8F711", "583F0355", "2F9B0A57", "ECE7DA1D", "943EF0AB",
       "43A2EDB1", "00E53D63"},
      {"055DCC02", "3EB065CF", "31F79238", "320D2E00", "4A2E5FB0", "0BD9F652", "B4107E50", "20F4D4BA",
       "8F1A1F99", "A191A338"},
      {"99E9D851", "682705DB", "30E7211B", "B7BB58E8", "B74655EF", "B6C8BBBE", "AED9E3B4", "0D4999FE",
       "F5932423", "6B31BAB1"},
      {"00000000", "C294D338", "1B174353", "2D0E20C8", "B37FB5E6", "6AFC258D", "5CE54616", "FA2D482E",
       "23AED845", "15B7BBDE"},
  };
  for (int t = 0; t < 5; t++) {
    const ChecksumType ct = static_cast<ChecksumType>(t);
    EXPECT_EQ(ChecksumAsString(empty, ct), std::string(want[t][0]));
    EXPECT_EQ(ChecksumAsString(&b0, ct1, ct), std::string(want[t][1]));
    EXPECT_EQ(ChecksumAsString(&b0, ct2, ct), std::string(want[t][2]));
    EXPECT_EQ(ChecksumAsString(&b0, ct3, ct), std::string(want[t][3]));
    EXPECT_EQ(ChecksumAsString(&b1, ct1, ct), std::string(want[t][4]));
    EXPECT_EQ(ChecksumAsString(&b1, ct2, ct), std::string(want[t][5]));
    EXPECT_EQ(ChecksumAsString(&b1, ct3, ct), std::string(want[t][6]));
    EXPECT_EQ(ChecksumAsString(&b2, ct1, ct), std::string(want[t][7]));
    EXPECT_EQ(ChecksumAsString(&b2, ct2, ct), std::string(want[t][8]));
    EXPECT_EQ(ChecksumAsString(&b2, ct3, ct), std::string(want[t][9]));
  }
}

// reader_common.cc:26-63 through the scalar mirror, and the batched verify
// over a run of blocks with one corrupted byte in some of them.
TEST(BlockChecksum, VerifyScalarAndBatched) {
  std::mt19937_64 rnd(7);
  for (ChecksumType t : {kCRC32c, kXXH3, kxxHash, kxxHash64}) {
    for (uint32_t base : {0u, 0x9e3779b9u}) {
      // build a run of blocks [payload][type][LE32 checksum + modifier]
      std::string img;
      std::vector<BlockHandle> handles;
      const uint64_t file_base = 1ull << 32;
      for (int b = 0; b < 64; b++) {
        const size_t n = (b % 3 == 0 ? 4096 : b % 3 == 1 ? 16384 : 65536) + rnd() % 256;
        std::string payload(n, 0);
        for (auto& c : payload) c = static_cast<char>(rnd());
        const char comp = static_cast<char>(b % 2 ? 1 : 0);
        const uint64_t off = file_base + img.size();
        uint32_t ck = ComputeBuiltinChecksumWithLastByte(t, payload.data(), n, comp);
        ck += ChecksumModifierForContext(base, off);
        handles.push_back({off, n});
        img += payload;
        img.push_back(comp);
        for (int i = 0; i < 4; i++) img.push_back(static_cast<char>(ck >> (8 * i)));
      }
      Footer f{t, base};
      // scalar
      EXPECT_TRUE(VerifyBlockChecksum(f, img.data() + (handles[3].offset - file_base), handles[3].size, "x.sst",
                                      handles[3].offset).ok());
      // batched, clean then corrupted
      std::string bad = img;
      const int corrupt[3] = {5, 17, 40};
      for (int b : corrupt) bad[handles[b].offset - file_base + 100] ^= 0x04;
      for (int pass = 0; pass < 2; pass++) {
        const std::string& src = pass ? bad : img;
        void* d = nullptr;
        if (hipMalloc(&d, src.size() + 64) != hipSuccess) {
          g_fail++;
          return;
        }
        (void)hipMemcpy(d, src.data(), src.size(), hipMemcpyHostToDevice);
        std::vector<Status> per;
        Status s = VerifyBlockChecksums(f, d, file_base, handles, "000042.sst", &per);
        (void)hipFree(d);
        EXPECT_EQ(s.ok(), pass == 0);
        int nbad = 0;
        for (size_t i = 0; i < per.size(); i++) nbad += !per[i].ok();
        EXPECT_EQ(nbad, pass ? 3 : 0);
        if (pass) {
          EXPECT_TRUE(per[5].IsCorruption() && per[17].IsCorruption() && per[40].IsCorruption());
          // the batched message equals the scalar VerifyBlockChecksum message
          const Status one = VerifyBlockChecksum(f, bad.data() + (handles[17].offset - file_base),
                                                 handles[17].size, "000042.sst", handles[17].offset);
          EXPECT_EQ(one.ToString(), per[17].ToString());
          EXPECT_EQ(per[17].ToString().rfind("Corruption: block checksum mismatch: stored", 0), 0u);
        }
      }
    }
  }
}

// db/log_writer.cc:48-51 type_crc_ and the record CRC algebra
TEST(Log, PhysicalRecordCrc) {
  const uint32_t type_crc[5] = {0xa016d052u, 0xb34623a6u, 0x412da0a5u, 0x95e7c44eu, 0x678c474du};
  for (int t = 1; t <= 5; t++) {
    const char c = static_cast<char>(t);
    EXPECT_EQ(crc32c::Value(&c, 1), type_crc[t - 1]);
  }
  std::string payload = "a physical record payload";
  for (int t = 1; t <= 8; t++) {
    std::string hdr_and_payload(1, static_cast<char>(t));
    if (log::IsRecyclable(t)) hdr_and_payload += std::string("\x7b\x00\x00\x00", 4);  // log 123
    hdr_and_payload += payload;
    const uint32_t direct = crc32c::Mask(crc32c::Value(hdr_and_payload.data(), hdr_and_payload.size()));
    EXPECT_EQ(log::PhysicalRecordCrc(static_cast<log::RecordType>(t), payload.data(), payload.size(), 123),
              direct);
  }
}

// log::Writer restated on the host (db/log_writer.cc:79-175, 263-311; legacy
// headers), CRCs from the mirror's PhysicalRecordCrc.
static void LogWrite(std::string* log, uint32_t* block_offset, const std::string& rec) {
  size_t left = rec.size(), ptr = 0;
  bool begin = true;
  do {
    const uint32_t leftover = log::kBlockSize - *block_offset;
    if (leftover < (uint32_t)log::kHeaderSize) {
      log->append(leftover, '\0');
      *block_offset = 0;
    }
    const size_t avail = log::kBlockSize - *block_offset - log::kHeaderSize;
    const size_t frag = left < avail ? left : avail;
    const bool end = left == frag;
    const log::RecordType t = begin && end ? log::kFullType : begin ? log::kFirstType
                              : end ? log::kLastType : log::kMiddleType;
    const uint32_t crc = log::PhysicalRecordCrc(t, rec.data() + ptr, frag, 0);
    char h[7] = {(char)crc, (char)(crc >> 8), (char)(crc >> 16), (char)(crc >> 24), (char)(frag & 0xff),
                 (char)(frag >> 8), (char)t};
    log->append(h, 7);
    log->append(rec.data() + ptr, frag);
    *block_offset += 7 + (uint32_t)frag;
    ptr += frag;
    left -= frag;
    begin = false;
  } while (left > 0);
}
struct CountingReporter : log::RecoveryReader::Reporter {
  size_t dropped = 0;
  std::string message;
  void Corruption(size_t bytes, const Status& s) override {
    dropped += bytes;
    message += s.ToString();
  }
};
static std::string BigString(const std::string& part, size_t n) {  // db/log_test.cc:23-33
  std::string r;
  while (r.size() < n) r += part;
  r.resize(n);
  return r;
}
// db/log_test.cc:342-350 Fragmentation and :513-521 ChecksumMismatch through
// the one-pass recovery reader, each record with its XXH3 record_checksum.
TEST(Log, RecoveryReader) {
  auto run = [](const std::string& img, CountingReporter* rep, std::vector<std::string>* out,
                std::vector<uint64_t>* sums) {
    void* d = nullptr;
    EXPECT_EQ(hipMalloc(&d, img.size() + 64), hipSuccess);
    EXPECT_EQ(hipMemcpy(d, img.data(), img.size(), hipMemcpyHostToDevice), hipSuccess);
    log::RecoveryReader reader(rep, 0);
    EXPECT_TRUE(reader.Recover(img.data(), d, img.size(), log::WALRecoveryMode::kTolerateCorruptedTailRecords).ok());
    std::string_view rec;
    std::string scratch;
    uint64_t sum = 0;
    while (reader.ReadRecord(&rec, &scratch, log::WALRecoveryMode::kTolerateCorruptedTailRecords, &sum)) {
      out->emplace_back(rec);
      sums->push_back(sum);
    }
    (void)hipFree(d);
  };
  {
    std::string img;
    uint32_t bo = 0;
    const std::vector<std::string> want = {"small", BigString("medium", 50000), BigString("large", 100000)};
    for (const auto& r : want) LogWrite(&img, &bo, r);
    CountingReporter rep;
    std::vector<std::string> got;
    std::vector<uint64_t> sums;
    run(img, &rep, &got, &sums);
    EXPECT_TRUE(got == want);
    EXPECT_EQ(rep.dropped, 0u);
    for (size_t i = 0; i < got.size() && i < sums.size(); i++) EXPECT_EQ(sums[i], XXH3_64bits(want[i].data(), want[i].size()));
  }
  {
    std::string img;
    uint32_t bo = 0;
    LogWrite(&img, &bo, "foooooo");
    img[0] = static_cast<char>(img[0] + 14);  // IncrementByte(0, 14)
    CountingReporter rep;
    std::vector<std::string> got;
    std::vector<uint64_t> sums;
    run(img, &rep, &got, &sums);
    EXPECT_TRUE(got.empty());
    EXPECT_EQ(rep.dropped, 14u);
    EXPECT_TRUE(rep.message.find("checksum mismatch") != std::string::npos);
  }
}

// util/hash_test.cc:162-228 (a sample of Hash64SmallValueSchema)
TEST(HashTest, Hash64SmallValueSchema) {
  EXPECT_EQ(Hash64("", 0, 0), uint64_t{5999572062939766020u});
  EXPECT_EQ(Hash64("\x08", 1, 0), uint64_t{583283813901344696u});
  EXPECT_EQ(Hash64("\x4d\x76", 2, 0), uint64_t{6859542833406258115u});
  EXPECT_EQ(Hash64("\x67\x53\x81\x1c", 4, 0), uint64_t{9010661983527562386u});
  EXPECT_EQ(Hash64("\x31\x1b\x98\x75\x96\x22\xd3\x9a", 8, 0), uint64_t{9844314944338447628u});
  EXPECT_EQ(Hash64("\xbd\x2c\x63\x38\xbf\xe9\x78\xb7\xbf\x15", 10, 0), uint64_t{10551812464348219044u});
}

// db/kv_checksum.h: the scalar template chain == the batched kernel, and
// Protect/Strip round trips to 0 (GetStatus OK)
TEST(KvChecksum, ScalarChainEqualsBatch) {
  std::mt19937_64 rnd(11);
  const int n = 64;
  std::vector<std::string> keys(n), vals(n);
  std::vector<uint8_t> ops(n);
  std::vector<uint64_t> seqs(n);
  std::string kimg, vimg;
  std::vector<uint64_t> koff(n), voff(n);
  std::vector<uint32_t> klen(n), vlen(n);
  for (int i = 0; i < n; i++) {
    keys[i].resize(i % 5 == 0 ? 300 : 8 + rnd() % 40);
    vals[i].resize(i % 7 == 0 ? 0 : rnd() % 3000);
    for (auto& c : keys[i]) c = static_cast<char>(rnd());
    for (auto& c : vals[i]) c = static_cast<char>(rnd());
    ops[i] = static_cast<uint8_t>(rnd());
    seqs[i] = rnd();
    koff[i] = kimg.size();
    klen[i] = static_cast<uint32_t>(keys[i].size());
    kimg += keys[i];
    voff[i] = vimg.size();
    vlen[i] = static_cast<uint32_t>(vals[i].size());
    vimg += vals[i];
  }
  void *dk, *dv, *dko, *dvo, *dkl, *dvl, *dops, *dseq, *dout;
  if (hipMalloc(&dk, kimg.size() + 64) || hipMalloc(&dv, vimg.size() + 64) || hipMalloc(&dko, 8 * n) ||
      hipMalloc(&dvo, 8 * n) || hipMalloc(&dkl, 4 * n) || hipMalloc(&dvl, 4 * n) || hipMalloc(&dops, n) ||
      hipMalloc(&dseq, 8 * n) || hipMalloc(&dout, 8 * n)) {
    g_fail++;
    return;
  }
  (void)hipMemcpy(dk, kimg.data(), kimg.size(), hipMemcpyHostToDevice);
  (void)hipMemcpy(dv, vimg.data(), vimg.size(), hipMemcpyHostToDevice);
  (void)hipMemcpy(dko, koff.data(), 8 * n, hipMemcpyHostToDevice);
  (void)hipMemcpy(dvo, voff.data(), 8 * n, hipMemcpyHostToDevice);
  (void)hipMemcpy(dkl, klen.data(), 4 * n, hipMemcpyHostToDevice);
  (void)hipMemcpy(dvl, vlen.data(), 4 * n, hipMemcpyHostToDevice);
  (void)hipMemcpy(dops, ops.data(), n, hipMemcpyHostToDevice);
  (void)hipMemcpy(dseq, seqs.data(), 8 * n, hipMemcpyHostToDevice);
  const mck_spans ks{dk, static_cast<uint64_t*>(dko), static_cast<uint32_t*>(dkl), 0, 0, (uint32_t)n};
  const mck_spans vs{dv, static_cast<uint64_t*>(dvo), static_cast<uint32_t*>(dvl), 0, 0, (uint32_t)n};
  EXPECT_EQ(mck_kv_protect_batch(MCK_KV_PROTECT_KVOS, &ks, &vs, static_cast<uint8_t*>(dops),
                                 static_cast<uint64_t*>(dseq), static_cast<uint64_t*>(dout), nullptr),
            0);
  std::vector<uint64_t> out(n);
  (void)hipMemcpy(out.data(), dout, 8 * n, hipMemcpyDeviceToHost);
  for (void* p : {dk, dv, dko, dvo, dkl, dvl, dops, dseq, dout}) (void)hipFree(p);
  for (int i = 0; i < n; i++) {
    const ProtectionInfo64 kvos = ProtectionInfo64().ProtectKVO(keys[i], vals[i], ops[i]).ProtectS(seqs[i]);
    EXPECT_EQ(kvos.GetVal(), out[i]);
    EXPECT_TRUE(kvos.StripS(seqs[i]).StripKVO(keys[i], vals[i], ops[i]).GetStatus().ok());
    char enc[8];
    kvos.Encode(4, enc);
    EXPECT_TRUE(kvos.Verify(4, enc));
  }
}

// util/file_checksum_helper.h:22-72: FileChecksumCrc32c = big-endian
// crc32c::Value of the whole file, however the Updates are cut; host Update
// (incl. the > 1 MiB long-span path), device UpdateDevice and the factory's
// name matching.
TEST(FileChecksum, Crc32cGenerator) {
  FileChecksumGenCrc32cFactory factory;
  FileChecksumGenContext ctx;
  EXPECT_TRUE(factory.CreateFileChecksumGenerator(ctx) != nullptr);
  ctx.requested_checksum_func_name = "FileChecksumCrc32c";
  auto g0 = factory.CreateFileChecksumGenerator(ctx);
  EXPECT_TRUE(g0 != nullptr);
  ctx.requested_checksum_func_name = "SomethingElse";
  EXPECT_TRUE(factory.CreateFileChecksumGenerator(ctx) == nullptr);
  EXPECT_EQ(std::string(g0->Name()), std::string(kStandardDbFileChecksumFuncName));
  g0->Update("1234", 4);
  g0->Update("56789", 5);
  g0->Finalize();
  EXPECT_EQ(g0->GetChecksum(), std::string("\xe3\x06\x92\x83", 4));  // crc32c_test.cc:81 "123456789"

  std::mt19937_64 rng(4546);
  std::string file((3u << 20) + 17, '\0');
  for (auto& c : file) c = static_cast<char>(rng());
  FileChecksumGenCrc32c whole(ctx), pieces(ctx), dev(ctx);
  whole.Update(file.data(), file.size());
  size_t pos = 0, step = 1;
  while (pos < file.size()) {
    const size_t n = std::min(step, file.size() - pos);
    pieces.Update(file.data() + pos, n);
    pos += n;
    step = step * 7 + 3;
  }
  void* d = nullptr;
  EXPECT_EQ(hipMalloc(&d, file.size() + 64), hipSuccess);
  EXPECT_EQ(hipMemcpy(d, file.data(), file.size(), hipMemcpyHostToDevice), hipSuccess);
  // device Updates at odd offsets: 5 bytes, then (1 MiB + 3), then the rest
  EXPECT_TRUE(dev.UpdateDevice(d, 5));
  EXPECT_TRUE(dev.UpdateDevice(static_cast<char*>(d) + 5, (1u << 20) + 3));
  EXPECT_TRUE(dev.UpdateDevice(static_cast<char*>(d) + (1u << 20) + 8, file.size() - (1u << 20) - 8));
  (void)hipFree(d);
  for (auto* g : {&whole, &pieces, &dev}) g->Finalize();
  EXPECT_EQ(pieces.GetChecksum(), whole.GetChecksum());
  EXPECT_EQ(dev.GetChecksum(), whole.GetChecksum());
  const uint32_t v = crc32c::Value(file.data(), file.size());
  const std::string& w = whole.GetChecksum();
  EXPECT_EQ(((uint32_t)(uint8_t)w[0] << 24) | ((uint32_t)(uint8_t)w[1] << 16) | ((uint32_t)(uint8_t)w[2] << 8) |
                (uint32_t)(uint8_t)w[3],
            v);
}

// BlockBasedTable::VerifyChecksum of an SST image written by the test-side
// writer (tests/sst_format.py): clean -> OK; with one payload byte flipped at
// `bad_off` -> Corruption naming the block.
static int VerifySstFileCase(const char* path, long bad_off) {
  FILE* fp = fopen(path, "rb");
  if (!fp) return 2;
  std::string img;
  char buf[1 << 16];
  size_t k;
  while ((k = fread(buf, 1, sizeof buf, fp)) > 0) img.append(buf, k);
  fclose(fp);
  std::vector<mck_sst_block> blocks;
  Status s = VerifySstFile("000042.sst", img.data(), img.size(), &blocks);
  printf("clean: %s (%zu blocks)\n", s.ToString().c_str(), blocks.size());
  EXPECT_TRUE(s.ok());
  EXPECT_TRUE(blocks.size() > 3);
  img[bad_off] ^= 0x08;
  s = VerifySstFile("000042.sst", img.data(), img.size());
  printf("corrupt: %s\n", s.ToString().c_str());
  EXPECT_TRUE(s.IsCorruption());
  EXPECT_TRUE(s.ToString().find("block checksum mismatch") != std::string::npos);
  EXPECT_TRUE(s.ToString().find("in 000042.sst offset") != std::string::npos);
  img[bad_off] ^= 0x08;
  img[img.size() - 1] ^= 0x01;  // magic
  s = VerifySstFile("000042.sst", img.data(), img.size());
  EXPECT_TRUE(s.IsCorruption());
  EXPECT_TRUE(s.ToString().find("Bad table magic number") != std::string::npos);
  printf("%d checks, %d failures\n", g_checks, g_fail);
  return g_fail ? 1 : 0;
}

// table/block_based/block_test.cc builds blocks with BlockBuilder and checks
// the per-KV checksums through the iterators; here: a BlockBuilder-layout
// data block (prefix-compressed keys, restart interval 4), the batched
// InitializeBlockProtectionInfo against ProtectionInfo64().ProtectKV per
// entry, and a damaged block's status.
static std::string Varint32(uint32_t v) {
  std::string o;
  while (v >= 128) {
    o.push_back(static_cast<char>((v & 127) | 128));
    v >>= 7;
  }
  o.push_back(static_cast<char>(v));
  return o;
}
static std::string BuildBlock(const std::vector<std::pair<std::string, std::string>>& kvs, uint32_t ri) {
  std::string buf, last;
  std::vector<uint32_t> restarts;
  for (size_t i = 0; i < kvs.size(); i++) {
    const std::string& k = kvs[i].first;
    size_t shared = 0;
    if (i % ri == 0) {
      restarts.push_back(static_cast<uint32_t>(buf.size()));
    } else {
      while (shared < k.size() && shared < last.size() && k[shared] == last[shared]) shared++;
    }
    buf += Varint32(static_cast<uint32_t>(shared)) + Varint32(static_cast<uint32_t>(k.size() - shared)) +
           Varint32(static_cast<uint32_t>(kvs[i].second.size())) + k.substr(shared) + kvs[i].second;
    last = k;
  }
  if (restarts.empty()) restarts.push_back(0);
  auto fixed32 = [&](uint32_t v) {
    for (int b = 0; b < 4; b++) buf.push_back(static_cast<char>(v >> (8 * b)));
  };
  for (uint32_t r : restarts) fixed32(r);
  fixed32(static_cast<uint32_t>(restarts.size()));
  return buf;
}

TEST(BlockProtection, DataBlockMatchesProtectKV) {
  std::vector<std::pair<std::string, std::string>> kvs;
  for (int i = 0; i < 37; i++) {
    char k[32];
    snprintf(k, sizeof k, "user_key_%06d", i * 7);
    std::string key(k);
    key += std::string("\x01\x02\x03\x04\x05\x06\x07\x08", 8);  // seqno/type footer
    kvs.emplace_back(key, std::string(static_cast<size_t>((i * 53) % 400), static_cast<char>('a' + i % 26)));
  }
  std::vector<std::string> blocks{BuildBlock(kvs, 4), BuildBlock(kvs, 1), std::string("\x01\x00", 2)};
  BlockKvChecksums out;
  Status s = InitializeBlockProtectionInfo(MCK_BLOCK_DATA, blocks, 8, &out);
  EXPECT_TRUE(s.IsCorruption());  // the third block
  EXPECT_TRUE(out.status[0].ok());
  EXPECT_TRUE(out.status[1].ok());
  EXPECT_TRUE(out.status[2].IsCorruption());
  EXPECT_EQ(out.restart_interval[0], 4u);
  EXPECT_EQ(out.kv_checksum[2].size(), 0u);
  for (int b = 0; b < 2; b++) {
    EXPECT_EQ(out.kv_checksum[b].size(), kvs.size() * 8);
    for (size_t i = 0; i < kvs.size() && out.kv_checksum[b].size() == kvs.size() * 8; i++) {
      char want[8];
      ProtectionInfo64().ProtectKV(kvs[i].first, kvs[i].second).Encode(8, want);
      EXPECT_EQ(out.kv_checksum[b].substr(i * 8, 8), std::string(want, 8));
    }
  }
}

// No device: every reference-named function of the mirror that reads data
// must refuse loudly (DeviceError), never hand back a checksum of 0; the file
// checksum generator (no exceptions, no error channel) ends unknown.
static int NoDeviceCases() {
  const char d[] = "123456789";
  int thrown = 0, n = 0;
  auto expect_throw = [&](const char* name, auto fn) {
    n++;
    try {
      (void)fn();
      fprintf(stderr, "%s returned a value without a device\n", name);
    } catch (const DeviceError& e) {
      thrown++;
      printf("[  OK  ] %s: %s\n", name, e.what());
    }
  };
  expect_throw("crc32c::Value", [&] { return crc32c::Value(d, 9); });
  expect_throw("crc32c::Extend", [&] { return crc32c::Extend(0, d, 9); });
  expect_throw("XXH3_64bits", [&] { return XXH3_64bits(d, 9); });
  expect_throw("ComputeBuiltinChecksum", [&] { return ComputeBuiltinChecksum(kCRC32c, d, 9); });
  expect_throw("ComputeBuiltinChecksumWithLastByte",
               [&] { return ComputeBuiltinChecksumWithLastByte(kXXH3, d, 9, 'x'); });
  expect_throw("NPHash64", [&] { return NPHash64(d, 9, 0); });
  expect_throw("log::PhysicalRecordCrc", [&] { return log::PhysicalRecordCrc(log::kFullType, d, 9, 7); });
  expect_throw("VerifyBlockChecksum", [&] {
    Footer f;
    f.checksum_type = kCRC32c;
    char blk[16] = {0};
    return VerifyBlockChecksum(f, blk, 8, "x.sst", 0).ok();
  });
  // host algebra needs no device
  n++;
  if (crc32c::Unmask(crc32c::Mask(0xE3069283u)) == 0xE3069283u) thrown++;
  FileChecksumGenCrc32c gen(FileChecksumGenContext{});
  gen.Update(d, 9);
  gen.Finalize();
  n++;
  if (gen.failed() && gen.GetChecksum() == kUnknownFileChecksum) thrown++;
  // PerfContext needs no device to be read
  n++;
  SetPerfLevel(kEnableTime);
  get_perf_context()->Reset();
  if (GetPerfLevel() == kEnableTime && get_perf_context()->block_checksum_time == 0) thrown++;
  SetPerfLevel(kEnableCount);
  printf("%d checks, %d failures\n", n, n - thrown);
  return thrown == n ? 0 : 1;
}

// PERF_TIMER_GUARD(block_checksum_time) (reader_common.cc:29): the batched
// verify's device time lands in this thread's perf context at a timing level.
TEST(Perf, BlockChecksumTime) {
  std::vector<uint8_t> img(64 * 4101 + 64, 0);
  std::vector<BlockHandle> h;
  for (int i = 0; i < 64; i++) {
    char* p = reinterpret_cast<char*>(img.data()) + i * 4101;
    for (int k = 0; k < 4096; k++) p[k] = static_cast<char>(k * 7 + i);
    p[4096] = 0;
    const uint32_t c = crc32c::Mask(crc32c::Value(p, 4097));
    for (int k = 0; k < 4; k++) p[4097 + k] = static_cast<char>(c >> (8 * k));
    h.push_back(BlockHandle{static_cast<uint64_t>(i) * 4101, 4096});
  }
  void* d = nullptr;
  EXPECT_EQ(hipMalloc(&d, img.size()), hipSuccess);
  EXPECT_EQ(hipMemcpy(d, img.data(), img.size(), hipMemcpyHostToDevice), hipSuccess);
  Footer f;
  f.checksum_type = kCRC32c;
  SetPerfLevel(kEnableTimeExceptForMutex);
  get_perf_context()->Reset();
  std::vector<Status> per;
  EXPECT_TRUE(VerifyBlockChecksums(f, d, 0, h, "perf.sst", &per).ok());
  EXPECT_EQ(get_perf_context()->block_checksum_count, 64u);
  EXPECT_TRUE(get_perf_context()->block_checksum_time > 0);
  SetPerfLevel(kEnableCount);
  (void)hipFree(d);
}

int main(int argc, char** argv) {
  if (argc == 2 && !strcmp(argv[1], "--nodevice")) return NoDeviceCases();
  if (mck_device_count() < 1) {
    fprintf(stderr, "no gfx950 device\n");
    return 2;
  }
  if (argc == 4 && !strcmp(argv[1], "--sst")) return VerifySstFileCase(argv[2], atol(argv[3]));
  RUN(CRC, StandardResults);
  RUN(CRC, Values);
  RUN(CRC, Extend);
  RUN(CRC, Mask);
  RUN(CRC, Crc32cCombineBasicTest);
  RUN(CRC, Crc32cCombineOrderMattersTest);
  RUN(CRC, Crc32cCombineFullCoverTest);
  RUN(BuiltinChecksumTest, ChecksumSchemas);
  RUN(BlockChecksum, VerifyScalarAndBatched);
  RUN(Log, PhysicalRecordCrc);
  RUN(Log, RecoveryReader);
  RUN(HashTest, Hash64SmallValueSchema);
  RUN(KvChecksum, ScalarChainEqualsBatch);
  RUN(FileChecksum, Crc32cGenerator);
  RUN(BlockProtection, DataBlockMatchesProtectKV);
  RUN(Perf, BlockChecksumTime);
  printf("%d checks, %d failures\n", g_checks, g_fail);
  return g_fail ? 1 : 0;
}
