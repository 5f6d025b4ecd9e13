// mb_crc.hip -- design experiments for the batched CRC32C kernel (not product
// code).  Measures, on 1M x 4 KiB device-resident blocks:
//   * raw read bandwidth for the candidate per-wave access patterns, and
//   * full CRC32C kernels for the candidate work decompositions / LDS table
//     layouts,
// each checked against a CPU CRC on a sample of blocks.
//
// Build: hipcc -O3 --offload-arch=gfx950 -o mb_crc mb_crc.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, \
              __LINE__);                                                   \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

static constexpr uint32_t POLY = 0x82f63b78u;
static constexpr size_t BLK = 4096;

// ---------------- host GF(2) helpers ----------------
static uint32_t gf_mul(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (int j = 0; j < 32; j++) {
    if (b & (0x80000000u >> j)) p ^= a;
    a = (a >> 1) ^ ((a & 1u) ? POLY : 0u);
  }
  return p;
}
static uint32_t xpow8n(uint64_t n) {
  uint32_t r = 0x80000000u, sq = 0x00800000u;
  while (n) {
    if (n & 1) r = gf_mul(r, sq);
    sq = gf_mul(sq, sq);
    n >>= 1;
  }
  return r;
}
static uint32_t zshift(uint32_t s, uint64_t n) { return gf_mul(s, xpow8n(n)); }
static uint32_t cpu_crc(const uint8_t* p, size_t n) {
  uint32_t s = ~0u;
  for (size_t i = 0; i < n; i++) {
    s ^= p[i];
    for (int k = 0; k < 8; k++) s = (s >> 1) ^ ((s & 1u) ? POLY : 0u);
  }
  return ~s;
}
// byte tables for zshift(., d): tab[k][v] = zshift(v << 8k, d)
static void byte_tables(uint64_t d, uint32_t* out /*4*256*/) {
  uint32_t K = xpow8n(d);
  for (int k = 0; k < 4; k++)
    for (int v = 0; v < 256; v++) out[k * 256 + v] = gf_mul((uint32_t)v << (8 * k), K);
}
static void nib_tables(uint64_t d, uint32_t* out /*8*16*/) {
  uint32_t K = xpow8n(d);
  for (int k = 0; k < 8; k++)
    for (int v = 0; v < 16; v++) out[k * 16 + v] = gf_mul((uint32_t)v << (4 * k), K);
}
// per-lane final tables, layout [n][v][lane]: zshift(v<<4n, piece*(63-lane))
static void lane_final_tables(uint64_t piece, uint32_t* out /*8*16*64*/) {
  for (int l = 0; l < 64; l++) {
    uint32_t K = xpow8n(piece * (63 - l));
    for (int k = 0; k < 8; k++)
      for (int v = 0; v < 16; v++) out[(k * 16 + v) * 64 + l] = gf_mul((uint32_t)v << (4 * k), K);
  }
}

// ---------------- data generation ----------------
__global__ void k_fill(uint64_t* p, size_t n, uint64_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = z ^ (z >> 31);
  }
}

// ---------------- raw read patterns ----------------
__global__ void k_read_coalesced(const uint4* __restrict__ p, size_t n16, uint32_t* out) {
  uint32_t acc = 0;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    uint4 a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
    acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w;
  }
  for (; i < n16; i += stride) {
    uint4 a = p[i];
    acc ^= a.x ^ a.y ^ a.z ^ a.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// wave per 4 KiB block; lane reads 64 contiguous bytes.
__global__ void k_read_lane64(const uint8_t* __restrict__ p, size_t nblk, uint32_t* out) {
  const int lane = threadIdx.x & 63;
  size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
  size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  uint32_t acc = 0;
  for (size_t b = wave; b < nblk; b += nw) {
    const uint4* q = (const uint4*)(p + b * BLK + lane * 64);
    uint4 a = q[0], bb = q[1], c = q[2], d = q[3];
    acc ^= a.x ^ a.y ^ a.z ^ a.w ^ bb.x ^ bb.y ^ bb.z ^ bb.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// wave per 4 KiB block; lane reads 16B at k*1024 + 16*lane.
__global__ void k_read_wave_coal(const uint8_t* __restrict__ p, size_t nblk, uint32_t* out) {
  const int lane = threadIdx.x & 63;
  size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
  size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  uint32_t acc = 0;
  for (size_t b = wave; b < nblk; b += nw) {
    const uint4* q = (const uint4*)(p + b * BLK + lane * 16);
    uint4 a = q[0], bb = q[64], c = q[128], d = q[192];
    acc ^= a.x ^ a.y ^ a.z ^ a.w ^ bb.x ^ bb.y ^ bb.z ^ bb.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// lane per 4 KiB block; lane walks its block in 64-B (or 128-B) steps.
template <int STEP>
__global__ void k_read_lanepb(const uint8_t* __restrict__ p, size_t nblk, uint32_t* out) {
  const int lane = threadIdx.x & 63;
  size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
  size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  uint32_t acc = 0;
  for (size_t g = wave; g * 64 < nblk; g += nw) {
    const uint4* q = (const uint4*)(p + (g * 64 + lane) * BLK);
    for (int o = 0; o < (int)(BLK / 16); o += STEP / 16) {
      uint4 v[STEP / 16];
#pragma unroll
      for (int j = 0; j < STEP / 16; j++) v[j] = q[o + j];
#pragma unroll
      for (int j = 0; j < STEP / 16; j++) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// ---------------- CRC kernels ----------------
// LDS byte tables replicated R times: addr = ((t*256+v)*R + c)*4, c = lane % R.
template <int R>
struct ByteTab {
  static constexpr int LOG2R = R == 1 ? 0 : R == 2 ? 1 : R == 4 ? 2 : R == 8 ? 3 : R == 16 ? 4 : 5;
  static constexpr int BYTES = 4 * 256 * R * 4;
};

template <int R>
__device__ __forceinline__ uint32_t step4(const uint32_t* __restrict__ tab, uint32_t s, uint32_t c) {
  // tab: [4][256][R] replicated pure 4-byte-step tables; index k = byte k of s
  constexpr int SH = ByteTab<R>::LOG2R;
  uint32_t i0 = ((s & 0xffu) << SH) | c;
  uint32_t i1 = (((s >> 8) & 0xffu) << SH) | c;
  uint32_t i2 = (((s >> 16) & 0xffu) << SH) | c;
  uint32_t i3 = ((s >> 24) << SH) | c;
  return tab[i0] ^ tab[(256 << SH) + i1] ^ tab[(512 << SH) + i2] ^ tab[(768 << SH) + i3];
}

__device__ __forceinline__ uint32_t nib_shift(const uint32_t* __restrict__ nt, uint32_t s) {
  // nt: [8][16] nibble tables of a zshift
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) r ^= nt[k * 16 + ((s >> (4 * k)) & 15u)];
  return r;
}

__device__ __forceinline__ uint32_t lane_final(const uint32_t* __restrict__ ft, uint32_t s, int lane) {
  // ft: [8][16][64] per-lane nibble tables
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

// V2: wave per block, lane handles 64 contiguous bytes; main loop byte tables
// (replicated R) or nibble tables (NIB); per-lane final nibble table.
template <int R, bool NIB, bool FINAL_LDS>
__global__ __launch_bounds__(1024) void k_crc_v2(const uint8_t* __restrict__ p, size_t nblk,
                                                 const uint32_t* __restrict__ g_byte,
                                                 const uint32_t* __restrict__ g_nib4,
                                                 const uint32_t* __restrict__ g_final,
                                                 uint32_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  constexpr int TAB_WORDS = NIB ? 128 : 1024 * R;
  uint32_t* tab = smem;
  uint32_t* fin = smem + TAB_WORDS;
  for (int i = threadIdx.x; i < TAB_WORDS; i += blockDim.x)
    tab[i] = NIB ? g_nib4[i] : g_byte[i / R];
  if (FINAL_LDS)
    for (int i = threadIdx.x; i < 8 * 16 * 64; i += blockDim.x) fin[i] = g_final[i];
  __syncthreads();
  const uint32_t* ft = FINAL_LDS ? fin : g_final;
  const int lane = threadIdx.x & 63;
  const uint32_t c = lane & (R - 1);
  size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
  size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t b = wave; b < nblk; b += nw) {
    const uint4* q = (const uint4*)(p + b * BLK + lane * 64);
    uint4 v0 = q[0], v1 = q[1], v2 = q[2], v3 = q[3];
    uint32_t w[16] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w,
                      v2.x, v2.y, v2.z, v2.w, v3.x, v3.y, v3.z, v3.w};
    uint32_t s = lane == 0 ? ~0u : 0u;
#pragma unroll
    for (int j = 0; j < 16; j++) {
      s ^= w[j];
      s = NIB ? nib_shift(tab, s) : step4<R>(tab, s, c);
    }
    s = lane_final(ft, s, lane);
    s = wave_xor(s);
    if (lane == 0) out[b] = ~s;
  }
}

// V1: wave per block, coalesced 16 B pieces at k*1024+16*lane; gap shift
// (1008 B) via nibble tables; per-lane final for 16-B pieces.
template <int R>
__global__ __launch_bounds__(1024) void k_crc_v1(const uint8_t* __restrict__ p, size_t nblk,
                                                 const uint32_t* __restrict__ g_byte,
                                                 const uint32_t* __restrict__ g_gap,
                                                 const uint32_t* __restrict__ g_final16,
                                                 uint32_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  constexpr int TAB_WORDS = 1024 * R;
  uint32_t* tab = smem;
  uint32_t* gap = smem + TAB_WORDS;
  uint32_t* fin = gap + 128;
  for (int i = threadIdx.x; i < TAB_WORDS; i += blockDim.x) tab[i] = g_byte[i / R];
  for (int i = threadIdx.x; i < 128; i += blockDim.x) gap[i] = g_gap[i];
  for (int i = threadIdx.x; i < 8 * 16 * 64; i += blockDim.x) fin[i] = g_final16[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const uint32_t c = lane & (R - 1);
  size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
  size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t b = wave; b < nblk; b += nw) {
    const uint4* q = (const uint4*)(p + b * BLK + lane * 16);
    uint4 v[4] = {q[0], q[64], q[128], q[192]};
    uint32_t s = lane == 0 ? ~0u : 0u;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (k) s = nib_shift(gap, s);
      s ^= v[k].x; s = step4<R>(tab, s, c);
      s ^= v[k].y; s = step4<R>(tab, s, c);
      s ^= v[k].z; s = step4<R>(tab, s, c);
      s ^= v[k].w; s = step4<R>(tab, s, c);
    }
    s = lane_final(fin, s, lane);
    s = wave_xor(s);
    if (lane == 0) out[b] = ~s;
  }
}

// V3: lane per block.
template <int R>
__global__ __launch_bounds__(1024) void k_crc_v3(const uint8_t* __restrict__ p, size_t nblk,
                                                 const uint32_t* __restrict__ g_byte,
                                                 uint32_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  constexpr int TAB_WORDS = 1024 * R;
  uint32_t* tab = smem;
  for (int i = threadIdx.x; i < TAB_WORDS; i += blockDim.x) tab[i] = g_byte[i / R];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const uint32_t c = lane & (R - 1);
  size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
  size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t g = wave; g * 64 < nblk; g += nw) {
    size_t b = g * 64 + lane;
    const uint4* q = (const uint4*)(p + b * BLK);
    uint32_t s = ~0u;
    for (int o = 0; o < (int)(BLK / 16); o += 4) {
      uint4 v[4] = {q[o], q[o + 1], q[o + 2], q[o + 3]};
#pragma unroll
      for (int j = 0; j < 4; j++) {
        s ^= v[j].x; s = step4<R>(tab, s, c);
        s ^= v[j].y; s = step4<R>(tab, s, c);
        s ^= v[j].z; s = step4<R>(tab, s, c);
        s ^= v[j].w; s = step4<R>(tab, s, c);
      }
    }
    out[b] = ~s;
  }
}

// ---------------- driver ----------------
struct Ctx {
  uint8_t* d_data;
  size_t nblk;
  uint32_t* d_out;
  uint32_t* d_byte;
  uint32_t* d_nib4;
  uint32_t* d_gap;
  uint32_t* d_fin64;
  uint32_t* d_fin16;
  std::vector<uint8_t> h_sample;  // first blocks copied back
  std::vector<uint32_t> ref;      // CPU CRCs of sampled blocks
  std::vector<size_t> sample_idx;
  int ncu;
};

template <typename F>
static double time_ms(F launch, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  launch();  // warm
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
  printf("%-36s %9.3f ms  %8.1f GiB/s  %6.3f TB/s  %5.1f%% of 8 TB/s\n", name, ms, gibs, tbs,
         100 * tbs / 8.0);
  fflush(stdout);
}

static int check(Ctx& C, const char* name) {
  std::vector<uint32_t> got(C.nblk);
  CK(hipMemcpy(got.data(), C.d_out, C.nblk * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  for (size_t i = 0; i < C.sample_idx.size(); i++)
    if (got[C.sample_idx[i]] != C.ref[i]) {
      if (bad < 3)
        printf("  %s MISMATCH blk %zu got %08x want %08x\n", name, C.sample_idx[i], got[C.sample_idx[i]],
               C.ref[i]);
      bad++;
    }
  printf("  %s: %s (%zu sampled)\n", name, bad ? "FAIL" : "ok", C.sample_idx.size());
  CK(hipMemset(C.d_out, 0, C.nblk * 4));
  return bad;
}

int main(int argc, char** argv) {
  size_t nblk = argc > 1 ? strtoull(argv[1], 0, 10) : (1u << 20);
  int reps = argc > 2 ? atoi(argv[2]) : 10;
  Ctx C;
  C.nblk = nblk;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  C.ncu = prop.multiProcessorCount;
  printf("device %s  CUs %d  LDS/block %zu  clock %d kHz\n", prop.gcnArchName, C.ncu,
         prop.sharedMemPerBlock, prop.clockRate);
  size_t bytes = nblk * BLK;
  CK(hipMalloc(&C.d_data, bytes));
  CK(hipMalloc(&C.d_out, nblk * 4));
  CK(hipMemset(C.d_out, 0, nblk * 4));
  k_fill<<<4096, 256>>>((uint64_t*)C.d_data, bytes / 8, 42);
  CK(hipDeviceSynchronize());

  std::vector<uint32_t> h_byte(1024), h_nib4(128), h_gap(128), h_fin64(8192), h_fin16(8192);
  byte_tables(4, h_byte.data());
  nib_tables(4, h_nib4.data());
  nib_tables(1008, h_gap.data());
  lane_final_tables(64, h_fin64.data());
  lane_final_tables(16, h_fin16.data());
  auto up = [](std::vector<uint32_t>& h, uint32_t** d) {
    CK(hipMalloc(d, h.size() * 4));
    CK(hipMemcpy(*d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  };
  up(h_byte, &C.d_byte);
  up(h_nib4, &C.d_nib4);
  up(h_gap, &C.d_gap);
  up(h_fin64, &C.d_fin64);
  up(h_fin16, &C.d_fin16);

  // reference sample
  for (size_t i = 0; i < nblk; i += 997) C.sample_idx.push_back(i);
  C.sample_idx.push_back(nblk - 1);
  std::vector<uint8_t> blk(BLK);
  for (size_t i : C.sample_idx) {
    CK(hipMemcpy(blk.data(), C.d_data + i * BLK, BLK, hipMemcpyDeviceToHost));
    C.ref.push_back(cpu_crc(blk.data(), BLK));
  }

  const int ncu = C.ncu;
  // raw read patterns
  {
    size_t n16 = bytes / 16;
    for (int wpc : {8, 16, 32}) {
      int grid = ncu * wpc / 4;
      char nm[64];
      snprintf(nm, sizeof nm, "read coalesced (%d w/CU)", wpc);
      report(nm, time_ms([&] { k_read_coalesced<<<grid, 256>>>((const uint4*)C.d_data, n16, C.d_out); }, reps),
             bytes);
    }
    for (int wpc : {8, 16, 32}) {
      int grid = ncu * wpc / 4;
      char nm[64];
      snprintf(nm, sizeof nm, "read wave-coal 4K (%d w/CU)", wpc);
      report(nm, time_ms([&] { k_read_wave_coal<<<grid, 256>>>(C.d_data, nblk, C.d_out); }, reps), bytes);
      snprintf(nm, sizeof nm, "read lane64 4K (%d w/CU)", wpc);
      report(nm, time_ms([&] { k_read_lane64<<<grid, 256>>>(C.d_data, nblk, C.d_out); }, reps), bytes);
      snprintf(nm, sizeof nm, "read lane/blk 64B (%d w/CU)", wpc);
      report(nm, time_ms([&] { k_read_lanepb<64><<<grid, 256>>>(C.d_data, nblk, C.d_out); }, reps), bytes);
      snprintf(nm, sizeof nm, "read lane/blk 128B (%d w/CU)", wpc);
      report(nm, time_ms([&] { k_read_lanepb<128><<<grid, 256>>>(C.d_data, nblk, C.d_out); }, reps), bytes);
    }
  }
  int fails = 0;
  // CRC kernels
  auto run_v2 = [&](auto kern, int tab_words, bool fin_lds, const char* nm, int threads, int wg_per_cu) {
    size_t lds = (size_t)tab_words * 4 + (fin_lds ? 8192 * 4 : 0);
    CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int grid = ncu * wg_per_cu;
    char full[96];
    snprintf(full, sizeof full, "%s [%dx%d thr, %zuKiB]", nm, wg_per_cu, threads, lds / 1024);
    report(full, time_ms([&] { kern<<<grid, threads, lds>>>(C.d_data, nblk, C.d_byte, C.d_nib4, C.d_fin64, C.d_out); }, reps),
           bytes);
    fails += check(C, full);
  };
  run_v2(k_crc_v2<1, true, true>, 128, true, "v2 nib main, fin lds", 1024, 1);
  run_v2(k_crc_v2<1, true, true>, 128, true, "v2 nib main, fin lds", 512, 4);
  run_v2(k_crc_v2<1, false, true>, 1024, true, "v2 byte R1, fin lds", 1024, 1);
  run_v2(k_crc_v2<8, false, true>, 8192, true, "v2 byte R8, fin lds", 1024, 1);
  run_v2(k_crc_v2<8, false, true>, 8192, true, "v2 byte R8, fin lds", 512, 2);
  run_v2(k_crc_v2<16, false, true>, 16384, true, "v2 byte R16, fin lds", 1024, 1);
  run_v2(k_crc_v2<16, false, false>, 16384, false, "v2 byte R16, fin glob", 1024, 1);
  run_v2(k_crc_v2<32, false, false>, 32768, false, "v2 byte R32, fin glob", 1024, 1);
  run_v2(k_crc_v2<32, false, true>, 32768, true, "v2 byte R32, fin lds", 1024, 1);

  auto run_v1 = [&](auto kern, int R, const char* nm, int threads, int wg_per_cu) {
    size_t lds = (size_t)1024 * R * 4 + 128 * 4 + 8192 * 4;
    CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int grid = ncu * wg_per_cu;
    char full[96];
    snprintf(full, sizeof full, "%s [%dx%d thr, %zuKiB]", nm, wg_per_cu, threads, lds / 1024);
    report(full, time_ms([&] { kern<<<grid, threads, lds>>>(C.d_data, nblk, C.d_byte, C.d_gap, C.d_fin16, C.d_out); }, reps),
           bytes);
    fails += check(C, full);
  };
  run_v1(k_crc_v1<8>, 8, "v1 coal+gap R8", 1024, 1);
  run_v1(k_crc_v1<16>, 16, "v1 coal+gap R16", 1024, 1);

  auto run_v3 = [&](auto kern, int R, const char* nm, int threads, int wg_per_cu) {
    size_t lds = (size_t)1024 * R * 4;
    CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int grid = ncu * wg_per_cu;
    char full[96];
    snprintf(full, sizeof full, "%s [%dx%d thr, %zuKiB]", nm, wg_per_cu, threads, lds / 1024);
    report(full, time_ms([&] { kern<<<grid, threads, lds>>>(C.d_data, nblk, C.d_byte, C.d_out); }, reps), bytes);
    fails += check(C, full);
  };
  run_v3(k_crc_v3<16>, 16, "v3 lane/blk R16", 1024, 1);
  run_v3(k_crc_v3<32>, 32, "v3 lane/blk R32", 1024, 1);
  run_v3(k_crc_v3<8>, 8, "v3 lane/blk R8", 1024, 2);
  printf("fails=%d\n", fails);
  return fails ? 1 : 0;
}
