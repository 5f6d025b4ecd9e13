// Load-layout probe (design tool): stream 4 GiB through 256 x 1024-thread
// persistent workgroups, 4 KiB per wave per round, one round prefetched,
// XOR-reduce; layout 0 = CRC chunks (lane l: 16 B at 64 l + 16 j), layout
// 1 = contiguous per instruction (lane l: 16 B at 16 l + 1024 j); nt = 0/1.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g4;
template <int LAYOUT, bool NT>
__device__ __forceinline__ u32x4 ld(const unsigned char* base, unsigned lane, int j) {
  const size_t off = LAYOUT == 0 ? 64 * lane + 16 * j : 16 * lane + 1024 * j;
  const g4* p = reinterpret_cast<g4*>(reinterpret_cast<size_t>(base + off));
  return NT ? __builtin_nontemporal_load(p) : *p;
}
template <int LAYOUT, bool NT>
__global__ __launch_bounds__(1024) void k(const unsigned char* data, size_t rounds, unsigned* out) {
  const unsigned lane = threadIdx.x & 63;
  const size_t w = blockIdx.x * 16 + (threadIdx.x >> 6), nw = gridDim.x * 16;
  u32x4 acc = {0, 0, 0, 0};
  size_t r = w;
  if (r >= rounds) return;
  u32x4 c[4];
  for (int j = 0; j < 4; j++) c[j] = ld<LAYOUT, NT>(data + 4096 * r, lane, j);
  for (;;) {
    const size_t nr = r + nw;
    const bool more = nr < rounds;
    u32x4 n[4];
    for (int j = 0; j < 4; j++) n[j] = ld<LAYOUT, NT>(data + 4096 * (more ? nr : r), lane, j);
    for (int j = 0; j < 4; j++) acc ^= c[j];
    if (!more) break;
    r = nr;
    for (int j = 0; j < 4; j++) c[j] = n[j];
  }
  out[blockIdx.x * 1024 + threadIdx.x] = acc.x ^ acc.y ^ acc.z ^ acc.w;
}
template <int L, bool NT>
float run(const unsigned char* d, size_t rounds, unsigned* o) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 100; i++) hipLaunchKernelGGL((k<L, NT>), dim3(256), dim3(1024), 0, 0, d, rounds, o);
  hipEventRecord(a, 0);
  for (int i = 0; i < 50; i++) hipLaunchKernelGGL((k<L, NT>), dim3(256), dim3(1024), 0, 0, d, rounds, o);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / 50;
}
int main() {
  const size_t bytes = 4ull << 30, rounds = bytes / 4096;
  unsigned char* d;
  unsigned* o;
  if (hipMalloc(&d, bytes) || hipMalloc(&o, 256 * 1024 * 4)) return 1;
  hipMemset(d, 1, bytes);
  float t[4] = {run<0, false>(d, rounds, o), run<1, false>(d, rounds, o), run<0, true>(d, rounds, o),
                run<1, true>(d, rounds, o)};
  const char* nm[4] = {"crc-chunks", "contiguous", "crc-chunks nt", "contiguous nt"};
  for (int i = 0; i < 4; i++) printf("%-16s %.4f ms  %.3f TB/s\n", nm[i], t[i], bytes / t[i] / 1e9);
  return 0;
}
