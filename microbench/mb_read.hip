// mb_read.hip -- design microbenchmark (not product code): streaming-read
// throughput of the CRC kernel's access pattern (lane owns a contiguous 64-B
// chunk: 4 x dwordx4 at 64*lane + 16*j) vs a contiguous-per-instruction
// pattern (16*lane + 1024*j), with a tunable amount of per-round VALU work
// and one round prefetched, 16 waves per CU, persistent grid.
#include "mb_common.h"

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gu32x4;

template <int PATTERN, int WORK>
__global__ __launch_bounds__(1024) void k_read(const uint8_t* base, uint32_t nblk, uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 16 + (threadIdx.x >> 6));
  const uint32_t nw = gridDim.x * 16;
  auto addr = [&](uint32_t b, int j) -> uint64_t {
    const uint64_t blk = reinterpret_cast<uint64_t>(base) + (uint64_t)b * 4096;
    return PATTERN == 0 ? blk + 64 * lane + 16 * j : blk + 16 * lane + 1024 * j;
  };
  uint32_t acc = lane;
  uint32_t b = wave;
  if (b >= nblk) return;
  u32x4 cur[4], nxt[4];
#pragma unroll
  for (int j = 0; j < 4; j++) cur[j] = *reinterpret_cast<gu32x4*>(addr(b, j));
  for (;;) {
    const uint32_t nb = b + nw;
    const bool more = nb < nblk;
#pragma unroll
    for (int j = 0; j < 4; j++) nxt[j] = *reinterpret_cast<gu32x4*>(addr(more ? nb : b, j));
    uint32_t v = cur[0].x ^ cur[1].y ^ cur[2].z ^ cur[3].w ^ cur[0].w ^ cur[1].z ^ cur[2].y ^ cur[3].x;
#pragma unroll
    for (int w = 0; w < WORK; w++) v = __builtin_amdgcn_perm(v, v ^ 0x9e3779b9u, 0x05040302u) + 0x7f4a7c15u;
    acc ^= v;
    if (!more) break;
    b = nb;
#pragma unroll
    for (int j = 0; j < 4; j++) cur[j] = nxt[j];
  }
  out[blockIdx.x * 1024 + threadIdx.x] = acc;
}

template <int P, int W>
static void run(const uint8_t* d, uint32_t nblk, uint32_t* out, int ncu) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int it = 0; it < 3; it++) hipLaunchKernelGGL((k_read<P, W>), dim3(ncu), dim3(1024), 0, 0, d, nblk, out);
  CK(hipEventRecord(e0));
  const int iters = 10;
  for (int it = 0; it < iters; it++) hipLaunchKernelGGL((k_read<P, W>), dim3(ncu), dim3(1024), 0, 0, d, nblk, out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= iters;
  printf("pattern=%s work=%3d  %.3f ms  %.3f TB/s\n", P == 0 ? "lane64B " : "contig1K", W, ms,
         (double)nblk * 4096 / (ms * 1e-3) / 1e12);
}

int main() {
  int ncu;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const uint32_t nblk = 1u << 20;
  uint8_t* d;
  uint32_t* out;
  CK(hipMalloc(&d, (size_t)nblk * 4096 + 4096));
  CK(hipMalloc(&out, (size_t)ncu * 1024 * 4));
  CK(hipMemset(d, 0x5a, (size_t)nblk * 4096 + 4096));
  run<0, 0>(d, nblk, out, ncu);
  run<1, 0>(d, nblk, out, ncu);
  run<0, 64>(d, nblk, out, ncu);
  run<1, 64>(d, nblk, out, ncu);
  run<0, 128>(d, nblk, out, ncu);
  run<1, 128>(d, nblk, out, ncu);
  run<0, 256>(d, nblk, out, ncu);
  run<1, 256>(d, nblk, out, ncu);
  run<0, 512>(d, nblk, out, ncu);
  run<1, 512>(d, nblk, out, ncu);
  return 0;
}
