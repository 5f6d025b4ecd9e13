// mb_crc2.hip -- round-2 design experiments (not product code):
//   * v_perm-formed LDS addresses (1 VALU per table lookup) with R=16/32
//     interleaved table copies,
//   * ILP (several blocks per wave iteration) and register prefetch of the
//     next iteration's blocks,
//   * unaligned 16-B global loads (correctness + bandwidth).
#include "mb_common.h"

// LDS table image for the 4-byte CRC step, interleaved so that lane c's copy
// sits in bank c:
//   R=32: addr = (t>>1)<<16 | v<<8 | (t&1)<<7 | c<<2       (128 KiB)
//   R=16: addr =              v<<8 |      t<<6 | c<<2       ( 64 KiB)
template <int R>
__device__ __forceinline__ uint32_t tab_addr(int t, uint32_t v, uint32_t c) {
  if (R == 32) return ((uint32_t)(t >> 1) << 16) | (v << 8) | ((uint32_t)(t & 1) << 7) | (c << 2);
  return (v << 8) | ((uint32_t)t << 6) | (c << 2);
}
template <int R>
constexpr int tab_bytes() { return R == 32 ? 131072 : 65536; }

template <int R>
__device__ __forceinline__ void fill_tab(uint8_t* lds, const uint32_t* __restrict__ g_byte) {
  // g_byte: [4][256]
  for (int i = threadIdx.x; i < 4 * 256 * R; i += blockDim.x) {
    int c = i % R, tv = i / R, t = tv >> 8, v = tv & 255;
    *(uint32_t*)(lds + tab_addr<R>(t, v, c)) = g_byte[t * 256 + v];
  }
}

struct PermC {
  uint32_t c[4];
};
template <int R>
__device__ __forceinline__ PermC make_permc(uint32_t c) {
  PermC p;
  for (int t = 0; t < 4; t++) p.c[t] = tab_addr<R>(t, 0, c);
  return p;
}

// one pure 4-byte CRC step: s' = zshift(s, 4) via 4 byte lookups
template <int R>
__device__ __forceinline__ uint32_t step4p(const uint8_t* lds, uint32_t s, const PermC& pc) {
  // selector: byte0 <- C.b0, byte1 <- s.b_k, byte2 <- C.b2, byte3 <- 0
  uint32_t a0 = __builtin_amdgcn_perm(s, pc.c[0], 0x0C020400u);
  uint32_t a1 = __builtin_amdgcn_perm(s, pc.c[1], 0x0C020500u);
  uint32_t a2 = __builtin_amdgcn_perm(s, pc.c[2], 0x0C020600u);
  uint32_t a3 = __builtin_amdgcn_perm(s, pc.c[3], 0x0C020700u);
  uint32_t x0 = *(const uint32_t*)(lds + a0);
  uint32_t x1 = *(const uint32_t*)(lds + a1);
  uint32_t x2 = *(const uint32_t*)(lds + a2);
  uint32_t x3 = *(const uint32_t*)(lds + a3);
  return x0 ^ x1 ^ x2 ^ x3;
}

__device__ __forceinline__ uint32_t lane_final(const uint32_t* __restrict__ ft, uint32_t s, int lane) {
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) r ^= ft[((k * 16 + ((s >> (4 * k)) & 15u)) << 6) + lane];
  return r;
}
__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v ^= __shfl_xor(v, o, 64);
  return v;
}

struct Chunk {
  uint4 v[4];
};
__device__ __forceinline__ Chunk load_chunk(const uint8_t* p) {
  const uint4* q = (const uint4*)p;
  Chunk c;
  c.v[0] = q[0];
  c.v[1] = q[1];
  c.v[2] = q[2];
  c.v[3] = q[3];
  return c;
}

template <int R>
__device__ __forceinline__ uint32_t chunk_crc(const uint8_t* lds, const Chunk& ch, uint32_t s, const PermC& pc) {
#pragma unroll
  for (int j = 0; j < 4; j++) {
    s ^= ch.v[j].x;
    s = step4p<R>(lds, s, pc);
    s ^= ch.v[j].y;
    s = step4p<R>(lds, s, pc);
    s ^= ch.v[j].z;
    s = step4p<R>(lds, s, pc);
    s ^= ch.v[j].w;
    s = step4p<R>(lds, s, pc);
  }
  return s;
}

// wave per 4 KiB block, 64 B per lane, ILP blocks per iteration, optional
// register prefetch of the next iteration.
template <int R, int ILP, bool PF>
__global__ __launch_bounds__(1024) void k_crc_v4(const uint8_t* __restrict__ p, size_t nblk,
                                                 const uint32_t* __restrict__ g_byte,
                                                 const uint32_t* __restrict__ g_final,
                                                 uint32_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  fill_tab<R>(smem, g_byte);
  uint32_t* fin = (uint32_t*)(smem + tab_bytes<R>());
  for (int i = threadIdx.x; i < 8 * 16 * 64; i += blockDim.x) fin[i] = g_final[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const PermC pc = make_permc<R>(lane & (R - 1));
  const uint32_t init = lane == 0 ? ~0u : 0u;
  size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
  size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  size_t b = wave * ILP;
  const size_t step = nw * ILP;
  Chunk cur[ILP];
  if (PF) {
#pragma unroll
    for (int i = 0; i < ILP; i++)
      if (b + i < nblk) cur[i] = load_chunk(p + (b + i) * BLK + lane * 64);
  }
  for (; b < nblk; b += step) {
    Chunk nxt[ILP];
    if (PF) {
#pragma unroll
      for (int i = 0; i < ILP; i++)
        if (b + step + i < nblk) nxt[i] = load_chunk(p + (b + step + i) * BLK + lane * 64);
    } else {
#pragma unroll
      for (int i = 0; i < ILP; i++)
        if (b + i < nblk) cur[i] = load_chunk(p + (b + i) * BLK + lane * 64);
    }
    uint32_t s[ILP];
#pragma unroll
    for (int i = 0; i < ILP; i++) s[i] = init;
#pragma unroll
    for (int j = 0; j < 4; j++) {
#pragma unroll
      for (int i = 0; i < ILP; i++) {
        s[i] ^= cur[i].v[j].x;
        s[i] = step4p<R>(smem, s[i], pc);
      }
#pragma unroll
      for (int i = 0; i < ILP; i++) {
        s[i] ^= cur[i].v[j].y;
        s[i] = step4p<R>(smem, s[i], pc);
      }
#pragma unroll
      for (int i = 0; i < ILP; i++) {
        s[i] ^= cur[i].v[j].z;
        s[i] = step4p<R>(smem, s[i], pc);
      }
#pragma unroll
      for (int i = 0; i < ILP; i++) {
        s[i] ^= cur[i].v[j].w;
        s[i] = step4p<R>(smem, s[i], pc);
      }
    }
#pragma unroll
    for (int i = 0; i < ILP; i++) {
      uint32_t f = wave_xor(lane_final(fin, s[i], lane));
      if (lane == 0 && b + i < nblk) out[b + i] = ~f;
    }
    if (PF) {
#pragma unroll
      for (int i = 0; i < ILP; i++) cur[i] = nxt[i];
    }
  }
}

// ---------------- unaligned loads ----------------
__global__ void k_read_unaligned(const uint8_t* __restrict__ p, size_t n16, size_t off, uint32_t* out) {
  uint32_t acc = 0;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  const uint8_t* q = p + off;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += stride) {
    uint4 a = *(const uint4*)(q + 16 * i);
    acc ^= a.x ^ a.y ^ a.z ^ a.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}
__global__ void k_copy_unaligned(const uint8_t* __restrict__ p, size_t n16, size_t off, uint4* dst) {
  size_t stride = (size_t)gridDim.x * blockDim.x;
  const uint8_t* q = p + off;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += stride)
    dst[i] = *(const uint4*)(q + 16 * i);
}

template <typename F>
static double time_ms(F launch, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  launch();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; i++) launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipGetLastError());
  return ms / reps;
}
static void report(const char* name, double ms, size_t bytes) {
  double gibs = bytes / (ms * 1e-3) / (1024.0 * 1024 * 1024);
  double tbs = bytes / (ms * 1e-3) / 1e12;
  printf("%-44s %8.3f ms %8.1f GiB/s %6.3f TB/s %5.1f%%\n", name, ms, gibs, tbs, 100 * tbs / 8.0);
  fflush(stdout);
}

#ifndef MB_NO_MAIN
int main(int argc, char** argv) {
  size_t nblk = argc > 1 ? strtoull(argv[1], 0, 10) : (1u << 20);
  int reps = argc > 2 ? atoi(argv[2]) : 10;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  size_t bytes = nblk * BLK;
  uint8_t* d_data;
  uint32_t* d_out;
  CK(hipMalloc(&d_data, bytes + 64));
  CK(hipMalloc(&d_out, nblk * 4));
  k_fill<<<4096, 256>>>((uint64_t*)d_data, (bytes + 64) / 8, 42);
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> h_byte(1024), h_fin(8192);
  byte_tables(4, h_byte.data());
  lane_final_tables(64, h_fin.data());
  uint32_t *d_byte, *d_fin;
  CK(hipMalloc(&d_byte, 4096));
  CK(hipMalloc(&d_fin, 32768));
  CK(hipMemcpy(d_byte, h_byte.data(), 4096, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_fin, h_fin.data(), 32768, hipMemcpyHostToDevice));

  std::vector<size_t> sidx;
  std::vector<uint32_t> ref;
  for (size_t i = 0; i < nblk; i += 997) sidx.push_back(i);
  sidx.push_back(nblk - 1);
  std::vector<uint8_t> blk(BLK);
  for (size_t i : sidx) {
    CK(hipMemcpy(blk.data(), d_data + i * BLK, BLK, hipMemcpyDeviceToHost));
    ref.push_back(cpu_crc(blk.data(), BLK));
  }
  int fails = 0;
  auto check = [&](const char* nm) {
    std::vector<uint32_t> got(nblk);
    CK(hipMemcpy(got.data(), d_out, nblk * 4, hipMemcpyDeviceToHost));
    int bad = 0;
    for (size_t i = 0; i < sidx.size(); i++) bad += got[sidx[i]] != ref[i];
    if (bad) printf("  %s: FAIL %d/%zu\n", nm, bad, sidx.size());
    fails += bad;
    CK(hipMemset(d_out, 0, nblk * 4));
  };

  // unaligned loads
  {
    size_t n16 = bytes / 16;
    int grid = ncu * 2;
    uint4* d_copy;
    CK(hipMalloc(&d_copy, 1 << 20));
    std::vector<uint8_t> h_src((1 << 20) + 64), h_cp(1 << 20);
    CK(hipMemcpy(h_src.data(), d_data, h_src.size(), hipMemcpyDeviceToHost));
    for (size_t off : {0, 1, 3, 4, 8, 12}) {
      k_copy_unaligned<<<256, 256>>>(d_data, (1 << 20) / 16, off, d_copy);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(h_cp.data(), d_copy, 1 << 20, hipMemcpyDeviceToHost));
      bool ok = memcmp(h_cp.data(), h_src.data() + off, 1 << 20) == 0;
      char nm[64];
      snprintf(nm, sizeof nm, "unaligned uint4 read off=%zu (%s)", off, ok ? "copy ok" : "COPY WRONG");
      report(nm, time_ms([&] { k_read_unaligned<<<grid, 1024>>>(d_data, n16, off, d_out); }, reps), bytes);
    }
    CK(hipFree(d_copy));
  }

#define RUN4(R, ILP, PF, WGS)                                                                         \
  do {                                                                                                \
    auto kern = k_crc_v4<R, ILP, PF>;                                                                 \
    size_t lds = tab_bytes<R>() + 32768;                                                              \
    CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
    char nm[96];                                                                                      \
    snprintf(nm, sizeof nm, "v4 perm R%d ILP%d PF%d [%dx1024, %zuKiB]", R, ILP, (int)PF, WGS,         \
             lds / 1024);                                                                             \
    report(nm, time_ms([&] { kern<<<ncu * WGS, 1024, lds>>>(d_data, nblk, d_byte, d_fin, d_out); }, reps), bytes); \
    check(nm);                                                                                        \
  } while (0)

  RUN4(32, 1, false, 1);
  RUN4(32, 1, true, 1);
  RUN4(32, 2, false, 1);
  RUN4(32, 2, true, 1);
  RUN4(32, 4, false, 1);
  RUN4(16, 1, true, 1);
  RUN4(16, 2, true, 1);
  RUN4(16, 2, false, 1);
  RUN4(16, 4, false, 1);
  printf("fails=%d\n", fails);
  return fails ? 1 : 0;
}
#endif
