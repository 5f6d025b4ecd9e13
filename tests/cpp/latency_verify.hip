// C++-timed latency of one small VerifyBlockChecksum batch (VERDICT r4 item
// 3): mck_sst_verify_batch + hipStreamSynchronize called directly, no Python,
// no torch -- the call a re-pointed RetrieveMultipleBlocks would make
// (table/block_based/block_based_table_reader_sync_and_async.h:217-228: at
// most MultiGetContext::MAX_BATCH_SIZE = 32 blocks, table/multiget_context.h
// :103).  Blocks: 4096 + 0..255 B payload + 5-byte trailer, kCRC32c, sealed by
// the engine's own write side (mck_sst_trailer_batch), device-resident.
//
// Per batch size n: median / p10 / p90 of 2000 calls, each = verify + sync;
// floor_us = an empty kernel launch + sync on the same stream (what any
// device call costs); kernel_us = the verify's device time (hipEvents).  The
// flags are checked: all clear, then exactly one flagged block after a
// flipped payload byte.  Prints one JSON object.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <chrono>
#include <random>
#include <string>
#include <vector>

#include "speedb_amd/mck.h"

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 2;                                                                   \
    }                                                                             \
  } while (0)
#define MK(x)                                                                     \
  do {                                                                            \
    int r_ = (x);                                                                 \
    if (r_ != MCK_OK) {                                                           \
      fprintf(stderr, "%s:%d %s: rc %d %s\n", __FILE__, __LINE__, #x, r_, mck_last_error()); \
      return 2;                                                                   \
    }                                                                             \
  } while (0)

__global__ void k_empty() {}

struct Stat {
  double p10, p50, p90;
};
static Stat stat(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  auto at = [&](double q) { return v[(size_t)(q * (v.size() - 1))]; };
  return {at(0.1), at(0.5), at(0.9)};
}
template <class F>
static std::vector<double> timed(F f, int reps) {
  for (int i = 0; i < 100; i++) f();
  std::vector<double> t(reps);
  for (int i = 0; i < reps; i++) {
    const auto a = std::chrono::steady_clock::now();
    f();
    t[i] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count();
  }
  return t;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 2000;
  // "spin": the host spins in hipStreamSynchronize instead of sleeping
  // (hipDeviceScheduleSpin, set before the context exists)
  const bool spin = argc > 2 && std::string(argv[2]) == "spin";
  if (spin) CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const mck_stream_t ms = reinterpret_cast<mck_stream_t>(st);
  // floor: an empty launch + sync
  hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st);
  CK(hipStreamSynchronize(st));
  bool bad = false;
  const Stat fl = stat(timed([&] {
                             hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st);
                             if (hipStreamSynchronize(st) != hipSuccess) bad = true;
                           },
                           reps));
  // the same empty launch, device time between two events
  hipEvent_t f0, f1;
  CK(hipEventCreate(&f0));
  CK(hipEventCreate(&f1));
  std::vector<double> ft(200);
  for (auto& x : ft) {
    CK(hipEventRecord(f0, st));
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st);
    CK(hipEventRecord(f1, st));
    CK(hipEventSynchronize(f1));
    float m = 0;
    CK(hipEventElapsedTime(&m, f0, f1));
    x = m * 1e3;
  }
  printf("{\"harness\": \"tests/cpp/latency_verify.hip\", \"sync\": \"%s\", \"reps\": %d, \"floor_us\": %.2f, "
         "\"floor_kernel_us\": %.2f, \"rows\": [", spin ? "spin" : "default", reps, fl.p50, stat(ft).p50);
  std::mt19937_64 rng(1);
  const int sizes[] = {1, 8, 32, 64, 256};
  for (int si = 0; si < 5; si++) {
    const uint32_t n = (uint32_t)sizes[si];
    std::vector<uint64_t> offs(n);
    std::vector<uint32_t> lens(n);
    uint64_t pos = 0;
    for (uint32_t i = 0; i < n; i++) {
      lens[i] = 4096 + (uint32_t)(rng() % 256);
      offs[i] = pos;
      pos += lens[i] + 5;
    }
    std::vector<uint8_t> img(pos + 64);
    for (auto& b : img) b = (uint8_t)rng();
    uint8_t* d_img;
    uint64_t* d_off;
    uint32_t *d_len, *d_ck, *d_cnt;
    uint8_t *d_mm, *d_type;
    CK(hipMalloc(&d_img, img.size()));
    CK(hipMalloc(&d_off, 8 * n));
    CK(hipMalloc(&d_len, 4 * n));
    CK(hipMalloc(&d_ck, 4 * n));
    CK(hipMalloc(&d_cnt, 4));
    CK(hipMalloc(&d_mm, n));
    CK(hipMalloc(&d_type, n));
    CK(hipMemcpy(d_img, img.data(), img.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_off, offs.data(), 8 * n, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_len, lens.data(), 4 * n, hipMemcpyHostToDevice));
    CK(hipMemset(d_type, 0, n));
    // seal: [type 0][LE32 trailer] after every payload
    const mck_spans sp{d_img, d_off, d_len, 0, 0, n};
    MK(mck_sst_trailer_batch(MCK_kCRC32c, &sp, d_type, nullptr, 0, d_ck, ms));
    std::vector<uint32_t> ck(n);
    CK(hipMemcpyAsync(ck.data(), d_ck, 4 * n, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    for (uint32_t i = 0; i < n; i++) {
      img[offs[i] + lens[i]] = 0;
      for (int k = 0; k < 4; k++) img[offs[i] + lens[i] + 1 + k] = (uint8_t)(ck[i] >> (8 * k));
    }
    CK(hipMemcpy(d_img, img.data(), img.size(), hipMemcpyHostToDevice));
    int rc = 0;
    const auto call = [&] {
      if (mck_sst_verify_batch(MCK_kCRC32c, &sp, nullptr, 0, d_mm, nullptr, nullptr, nullptr, ms) != MCK_OK) rc = 1;
      if (hipStreamSynchronize(st) != hipSuccess) rc = 1;
    };
    const Stat s = stat(timed(call, reps));
    // host time to ENQUEUE one call (no sync; 64 calls, then one sync):
    // the API's own CPU cost, next to an empty kernel's launch
    const auto enq = [&](auto one) {
      std::vector<double> v(50);
      for (auto& x : v) {
        (void)hipStreamSynchronize(st);
        const auto a = std::chrono::steady_clock::now();
        for (int r = 0; r < 64; r++) one();
        x = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count() / 64;
      }
      (void)hipStreamSynchronize(st);
      return stat(v).p50;
    };
    double enq_us = 0, enq_empty_us = 0;
    {
      const auto r = enq([&] { (void)mck_sst_verify_batch(MCK_kCRC32c, &sp, nullptr, 0, d_mm, nullptr, nullptr, nullptr, ms); });
      enq_us = r;
      const auto r2 = enq([&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st); });
      enq_empty_us = r2;
    }
    // device time of the verify alone
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<double> kt(200);
    for (auto& x : kt) {
      CK(hipEventRecord(e0, st));
      MK(mck_sst_verify_batch(MCK_kCRC32c, &sp, nullptr, 0, d_mm, nullptr, nullptr, nullptr, ms));
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms_ = 0;
      CK(hipEventElapsedTime(&ms_, e0, e1));
      x = ms_ * 1e3;
    }
    const Stat k = stat(kt);
    // flags: none, then exactly the corrupted block
    std::vector<uint8_t> mm(n);
    CK(hipMemcpy(mm.data(), d_mm, n, hipMemcpyDeviceToHost));
    bool ok = rc == 0 && std::all_of(mm.begin(), mm.end(), [](uint8_t v) { return v == 0; });
    const uint32_t victim = n / 2;
    uint8_t b;
    CK(hipMemcpy(&b, d_img + offs[victim] + 7, 1, hipMemcpyDeviceToHost));
    b ^= 0x10;
    CK(hipMemcpy(d_img + offs[victim] + 7, &b, 1, hipMemcpyHostToDevice));
    CK(hipMemset(d_cnt, 0, 4));
    MK(mck_sst_verify_batch(MCK_kCRC32c, &sp, nullptr, 0, d_mm, nullptr, nullptr, d_cnt, ms));
    CK(hipStreamSynchronize(st));
    uint32_t cnt = 0;
    CK(hipMemcpy(mm.data(), d_mm, n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&cnt, d_cnt, 4, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n; i++) ok = ok && mm[i] == (i == victim ? 1 : 0);
    ok = ok && cnt == 1;
    printf("%s{\"blocks\": %u, \"bytes\": %llu, \"device_us\": %.2f, \"p10_us\": %.2f, \"p90_us\": %.2f, "
           "\"kernel_us\": %.2f, \"enqueue_us\": %.2f, \"enqueue_empty_us\": %.2f, \"ok\": %s}",
           si ? ", " : "", n, (unsigned long long)(pos - 5ull * n), s.p50, s.p10, s.p90, k.p50, enq_us, enq_empty_us,
           ok ? "true" : "false");
    bad = bad || !ok;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(d_img);
    (void)hipFree(d_off);
    (void)hipFree(d_len);
    (void)hipFree(d_ck);
    (void)hipFree(d_cnt);
    (void)hipFree(d_mm);
    (void)hipFree(d_type);
  }
  printf("]}\n");
  return bad ? 1 : 0;
}
