// FETCH_SIZE / WRITE_SIZE calibration on a known byte count (VERDICT r2
// item 4): MI355X_MICROARCH.md says FETCH_SIZE reports exactly half the
// bytes of a wide coalesced DEFAULT-policy read; the engine's XXH3 and WAL
// verify kernels read with non-temporal loads and their traffic read 1.09-
// 1.10x the algorithmic bytes after that doubling.  Each kernel below reads
// (or writes) exactly `bytes` once, from a 4 GiB buffer (16x the 256 MiB
// Infinity Cache, so nothing is served from a previous launch), 16 waves per
// CU, one 4 KiB round per wave in flight (the engine's shape):
//   rd_contig<0>   lane l loads 16 B at 16 l + 1024 j (default policy)
//   rd_contig<1>   the same, non-temporal
//   rd_dword<1>    non-temporal 16-B loads + one dword load at the start of
//                  every 1 KiB (the XXH3 realignment dword, rd_fix)
//   rd_chunk<0/1>  lane l loads 16 B at 64 l + 16 j (the CRC chunk layout)
//   wr_contig<0/1> 16-B stores, default / non-temporal
// Run: ./nt_calib (timing) or under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
// (one launch of each kernel after one warmup launch of each).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g4;
typedef __attribute__((address_space(1))) const unsigned g1;
typedef __attribute__((address_space(1))) u32x4 gw4;

template <bool NT>
__device__ __forceinline__ u32x4 ld16(const unsigned char* p) {
  const g4* q = reinterpret_cast<const g4*>(reinterpret_cast<size_t>(p));
  return NT ? __builtin_nontemporal_load(q) : *q;
}

template <int LAYOUT, bool NT, bool DWORD>
__device__ __forceinline__ void rd_body(const unsigned char* data, size_t rounds, unsigned* out) {
  const unsigned lane = threadIdx.x & 63;
  const size_t w = blockIdx.x * 16 + (threadIdx.x >> 6), nw = gridDim.x * 16;
  u32x4 acc = {0, 0, 0, 0};
  unsigned dacc = 0;
  for (size_t r = w; r < rounds; r += nw) {
    const unsigned char* b = data + 4096 * r;
    u32x4 c[4];
#pragma unroll
    for (int j = 0; j < 4; j++) c[j] = ld16<NT>(b + (LAYOUT == 0 ? 16 * lane + 1024 * j : 64 * lane + 16 * j));
    if (DWORD) {
      // lanes 0, 16, 32, 48: the dword before each 256-B row of the round
      const unsigned k = lane & 15 ? 0u : lane * 16;
      dacc ^= *reinterpret_cast<const g1*>(reinterpret_cast<size_t>(b + k * 4));
    }
#pragma unroll
    for (int j = 0; j < 4; j++) acc ^= c[j];
  }
  out[blockIdx.x * 1024 + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w ^ dacc;
}
template <bool NT>
__global__ __launch_bounds__(1024) void rd_contig(const unsigned char* d, size_t rounds, unsigned* o) {
  rd_body<0, NT, false>(d, rounds, o);
}
template <bool NT>
__global__ __launch_bounds__(1024) void rd_dword(const unsigned char* d, size_t rounds, unsigned* o) {
  rd_body<0, NT, true>(d, rounds, o);
}
template <bool NT>
__global__ __launch_bounds__(1024) void rd_chunk(const unsigned char* d, size_t rounds, unsigned* o) {
  rd_body<1, NT, false>(d, rounds, o);
}
template <bool NT>
__global__ __launch_bounds__(1024) void wr_contig(unsigned char* d, size_t rounds) {
  const unsigned lane = threadIdx.x & 63;
  const size_t w = blockIdx.x * 16 + (threadIdx.x >> 6), nw = gridDim.x * 16;
  const u32x4 v = {lane, (unsigned)w, 7u, 9u};
  for (size_t r = w; r < rounds; r += nw) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
      gw4* q = reinterpret_cast<gw4*>(reinterpret_cast<size_t>(d + 4096 * r + 16 * lane + 1024 * j));
      if (NT)
        __builtin_nontemporal_store(v, q);
      else
        *q = v;
    }
  }
}

#define CHECK(x)                                                     \
  do {                                                               \
    hipError_t e_ = (x);                                             \
    if (e_ != hipSuccess) {                                          \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
      return 1;                                                      \
    }                                                                \
  } while (0)

template <class F>
static float timed(F f) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  f();  // warmup
  (void)hipEventRecord(a, 0);
  f();
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  const size_t bytes = 4ull << 30, rounds = bytes / 4096;
  int ncu = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) == hipSuccess) ncu = prop.multiProcessorCount;
  unsigned char* d;
  unsigned* o;
  CHECK(hipMalloc(&d, bytes));
  CHECK(hipMalloc(&o, (size_t)ncu * 1024 * 4));
  CHECK(hipMemset(d, 1, bytes));
  CHECK(hipDeviceSynchronize());
  const dim3 g(ncu), b(1024);
  struct R {
    const char* name;
    float ms;
  } rs[7] = {
      {"rd_contig<default>", timed([&] { hipLaunchKernelGGL(rd_contig<false>, g, b, 0, 0, d, rounds, o); })},
      {"rd_contig<nt>", timed([&] { hipLaunchKernelGGL(rd_contig<true>, g, b, 0, 0, d, rounds, o); })},
      {"rd_dword<nt>", timed([&] { hipLaunchKernelGGL(rd_dword<true>, g, b, 0, 0, d, rounds, o); })},
      {"rd_chunk<default>", timed([&] { hipLaunchKernelGGL(rd_chunk<false>, g, b, 0, 0, d, rounds, o); })},
      {"rd_chunk<nt>", timed([&] { hipLaunchKernelGGL(rd_chunk<true>, g, b, 0, 0, d, rounds, o); })},
      {"wr_contig<default>", timed([&] { hipLaunchKernelGGL(wr_contig<false>, g, b, 0, 0, d, rounds); })},
      {"wr_contig<nt>", timed([&] { hipLaunchKernelGGL(wr_contig<true>, g, b, 0, 0, d, rounds); })},
  };
  CHECK(hipDeviceSynchronize());
  for (const R& r : rs) printf("%-20s %8.4f ms %7.3f TB/s  bytes %zu\n", r.name, r.ms, bytes / r.ms / 1e9, bytes);
  return 0;
}
