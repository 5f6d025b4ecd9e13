// mb_engine.hip -- the round-2 microbenchmark kernel (uniform aligned 4 KiB
// blocks only) behind the engine's mck_crc32c_batch ABI, for same-process
// A/B against the product kernel (design tool, not product code).
#include "mb_crc2.hip"

struct SpansAbi {
  const void* base;
  const uint64_t* offsets;
  const uint32_t* lengths;
  uint64_t stride;
  uint32_t length;
  uint32_t count;
};

extern "C" int mck_crc32c_batch(const SpansAbi* s, const uint32_t*, uint32_t, uint32_t* out, hipStream_t st) {
  static uint32_t *d_byte = nullptr, *d_fin = nullptr;
  static int ncu = 0;
  if (!d_byte) {
    std::vector<uint32_t> h_byte(1024), h_fin(8192);
    byte_tables(4, h_byte.data());
    lane_final_tables(64, h_fin.data());
    hipMalloc(&d_byte, 4096);
    hipMalloc(&d_fin, 32768);
    hipMemcpy(d_byte, h_byte.data(), 4096, hipMemcpyHostToDevice);
    hipMemcpy(d_fin, h_fin.data(), 32768, hipMemcpyHostToDevice);
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    ncu = p.multiProcessorCount;
    hipFuncSetAttribute((const void*)k_crc_v4<16, 1, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        tab_bytes<16>() + 32768);
  }
  if (s->offsets || s->lengths || s->stride != 4096 || s->length != 4096) return -1;
  k_crc_v4<16, 1, true><<<ncu, 1024, tab_bytes<16>() + 32768, st>>>((const uint8_t*)s->base, s->count, d_byte,
                                                                      d_fin, out);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
extern "C" int mck_xxh3_64_batch(const SpansAbi*, uint64_t*, hipStream_t) { return -1; }
