// Read+write ceiling probe: a 16-lane row copies 1280-B rounds (five
// 16-B loads per lane, then five stores), rounds grid-strided, 2.2 GB
// source -> destination, the WAL writer's geometry without the CRC.
// Variants: plain, non-temporal loads, non-temporal stores, both; grid
// sizes.  Prints (read + write bytes) / best time as a fraction of 8 TB/s.
//   hipcc --offload-arch=gfx950 -O3 -o copy_probe copy_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int NTL, int NTS, int WG>
__global__ __launch_bounds__(WG) void k_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, uint64_t rounds) {
  const uint32_t c = threadIdx.x & 15;
  const uint64_t rows = (uint64_t)gridDim.x * (WG / 16);
  for (uint64_t g = (uint64_t)blockIdx.x * (WG / 16) + (threadIdx.x >> 4); g < rounds; g += rows) {
    const uint64_t b = 80ull * g + c;
    uint4 v[5];
#pragma unroll
    for (int j = 0; j < 5; j++) {
      if (NTL) {
        v[j].x = __builtin_nontemporal_load(&src[b + 16 * j].x);
        v[j].y = __builtin_nontemporal_load(&src[b + 16 * j].y);
        v[j].z = __builtin_nontemporal_load(&src[b + 16 * j].z);
        v[j].w = __builtin_nontemporal_load(&src[b + 16 * j].w);
      } else {
        v[j] = src[b + 16 * j];
      }
    }
#pragma unroll
    for (int j = 0; j < 5; j++) {
      if (NTS) {
        __builtin_nontemporal_store(v[j].x, &dst[b + 16 * j].x);
        __builtin_nontemporal_store(v[j].y, &dst[b + 16 * j].y);
        __builtin_nontemporal_store(v[j].z, &dst[b + 16 * j].z);
        __builtin_nontemporal_store(v[j].w, &dst[b + 16 * j].w);
      } else {
        dst[b + 16 * j] = v[j];
      }
    }
  }
}

template <int NTL, int NTS, int WG>
static void run(const char* name, uint4* s, uint4* d, uint64_t rounds, int grid) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float best = 1e9;
  for (int rep = 0; rep < 8; rep++) {
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL((k_copy<NTL, NTS, WG>), dim3(grid), dim3(WG), 0, 0, s, d, rounds);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    if (rep > 1 && ms < best) best = ms;
  }
  printf("%-10s wg %4d grid %6d: %.4f ms  frac %.4f\n", name, WG, grid, best, 2.0 * 1280.0 * rounds / (best * 1e-3) / 8e12);
}

int main() {
  const uint64_t bytes = 2217106570ull / 1280 * 1280;
  const uint64_t rounds = bytes / 1280;
  uint4 *s, *d;
  if (hipMalloc(&s, bytes) != hipSuccess || hipMalloc(&d, bytes) != hipSuccess) return 2;
  (void)hipMemset(s, 1, bytes);
  for (int grid : {1024, 2048, 4096, 8192}) {
    run<0, 0, 1024>("plain", s, d, rounds, grid / 4);
    run<0, 0, 256>("plain", s, d, rounds, grid);
  }
  run<1, 0, 256>("nt-load", s, d, rounds, 4096);
  run<0, 1, 256>("nt-store", s, d, rounds, 4096);
  run<1, 1, 256>("nt-both", s, d, rounds, 4096);
  run<0, 1, 1024>("nt-store", s, d, rounds, 1024);
  return 0;
}
