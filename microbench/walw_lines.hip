// Write-traffic probe for the WAL writer's store pattern.
// A 16-lane row stores one 1280-B round as five 256-B store instructions
// (lane c: bytes 16 c + 256 j), rounds back to back, the stream shifted by
// `off` bytes from a 128-B line.  mode 0 = the writer's order (instruction j
// covers [256 j, 256 j + 256) of the round); mode 1 = lane rotation: lane c
// stores in instruction t its piece t + (c < k0), k0 chosen so every
// instruction covers whole 128-B lines (six instructions, the first and last
// partial).  Run under rocprofv3 --pmc WRITE_SIZE; prints kernel ms per mode.
//   hipcc --offload-arch=gfx950 -O3 -o walw_lines walw_lines.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint4 g_u4;

template <int MODE>
__global__ __launch_bounds__(256) void k_rounds(uint8_t* out, uint64_t rounds, uint32_t off) {
  const uint32_t c = threadIdx.x & 15;
  const uint64_t rows = (uint64_t)gridDim.x * 16;
  for (uint64_t g = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 4); g < rounds; g += rows) {
    const uint64_t rb = (uint64_t)out + off + 1280ull * g;
    uint4 v[5];
#pragma unroll
    for (int j = 0; j < 5; j++) v[j] = make_uint4((uint32_t)g, c, j, 7);
    if (MODE == 0) {
#pragma unroll
      for (int j = 0; j < 5; j++) *reinterpret_cast<g_u4*>(rb + 256ull * j + 16ull * c) = v[j];
    } else {
      // pieces k = c + 16 j at rb + 16 k; lines start at k = k0 mod 8
      const uint32_t k0 = ((128u - (uint32_t)(rb & 127u)) & 127u) >> 4;
      const bool lo = c < k0;
#pragma unroll
      for (int t = -1; t < 5; t++) {
        const int j = lo ? t + 1 : t;
        if (j >= 0 && j < 5) {
          const uint4 x = j == 0 ? v[0] : j == 1 ? v[1] : j == 2 ? v[2] : j == 3 ? v[3] : v[4];
          *reinterpret_cast<g_u4*>(rb + 256ull * j + 16ull * c) = x;
        }
      }
    }
  }
}

int main(int argc, char** argv) {
  const uint64_t bytes = 2ull << 30;
  const uint64_t rounds = (bytes - 256) / 1280;
  uint8_t* d;
  if (hipMalloc(&d, bytes) != hipSuccess) return 2;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const uint32_t offs[] = {0, 16, 64, 112};
  for (int mode = 0; mode < 2; mode++)
    for (uint32_t off : offs) {
      float best = 1e9;
      for (int rep = 0; rep < 6; rep++) {
        (void)hipEventRecord(a, 0);
        if (mode == 0)
          hipLaunchKernelGGL(k_rounds<0>, dim3(4096), dim3(256), 0, 0, d, rounds, off);
        else
          hipLaunchKernelGGL(k_rounds<1>, dim3(4096), dim3(256), 0, 0, d, rounds, off);
        (void)hipEventRecord(b, 0);
        if (hipEventSynchronize(b) != hipSuccess) return 3;
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (rep && ms < best) best = ms;
      }
      printf("mode %d off %3u: %.4f ms  %.1f GB/s (stream %llu B)\n", mode, off, best, 1280.0 * rounds / best / 1e6,
             (unsigned long long)(1280ull * rounds));
    }
  (void)hipFree(d);
  return 0;
}
