// mb_lds.hip -- calibrate ds_read_b32 bank conflicts for the CRC table
// layouts (design experiment, not product code).  Each kernel runs 4
// independent lookup chains per lane; run under rocprofv3 with
// SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS to get conflict cycles per lookup.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef __attribute__((address_space(3))) const unsigned lds_word_t;
__device__ __forceinline__ unsigned ld(unsigned off) { return *reinterpret_cast<lds_word_t*>((size_t)off); }

// MODE 0: R16 interleave [v][t][c16], table t = k           (product v1)
// MODE 1: R16 interleave, table t = (k + bit4(lane)) & 3    (product v2)
// MODE 2: R32 interleave [t][v][c32], bank = lane % 32
// MODE 3: R16 with copy = lane % 16, t = k, but word = v*64 + c*4 + t (t innermost)
// MODE 4: every lane reads word lane (no randomness) -- baseline
// MODE 5: R1 (no replication) [t][v]
template <int MODE>
__global__ __launch_bounds__(1024) void k_lds(unsigned* out, int iters) {
  extern __shared__ unsigned smem[];
  for (int i = threadIdx.x; i < 32768; i += blockDim.x) smem[i] = i * 2654435761u;
  __syncthreads();
  const unsigned lane = threadIdx.x & 63, c16 = lane & 15, h = (lane >> 4) & 1, c32 = lane & 31;
  unsigned s[4] = {lane * 7919u, lane * 104729u + 1, lane * 1299709u + 2, lane * 15485863u + 3};
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const unsigned v = (s[q] >> (8 * k)) & 255u;
        unsigned a;
        if (MODE == 0) a = (v * 64 + k * 16 + c16) * 4;
        if (MODE == 1) a = (v * 64 + ((k + h) & 3) * 16 + c16) * 4;
        if (MODE == 2) a = ((k * 256 + v) * 32 + c32) * 4;
        if (MODE == 3) a = (v * 64 + c16 * 4 + k) * 4;
        if (MODE == 4) a = lane * 4 + k * 256;
        if (MODE == 5) a = (k * 256 + v) * 4;
        s[q] = s[q] * 5u + ld(a) + 1u;
      }
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s[0] ^ s[1] ^ s[2] ^ s[3];
}

template <int MODE>
void run(unsigned* d, int ncu, const char* name) {
  auto kern = k_lds<MODE>;
  hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  kern<<<ncu, 1024, 131072>>>(d, 10);
  hipEventRecord(a);
  kern<<<ncu, 1024, 131072>>>(d, 2000);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  double lookups = (double)ncu * 1024 * 2000 * 16;
  printf("%-28s %8.3f ms  %7.2f lookups/clk/CU @2.4GHz\n", name, ms, lookups / (ms * 1e-3) / ncu / 2.4e9);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  unsigned* d;
  hipMalloc(&d, p.multiProcessorCount * 1024 * 4);
  run<0>(d, p.multiProcessorCount, "R16 t=k");
  run<1>(d, p.multiProcessorCount, "R16 t=(k+bit4)&3");
  run<2>(d, p.multiProcessorCount, "R32 bank=lane%32");
  run<3>(d, p.multiProcessorCount, "R16 t innermost");
  run<4>(d, p.multiProcessorCount, "word=lane (no conflicts)");
  run<5>(d, p.multiProcessorCount, "R1 random");
  return 0;
}
