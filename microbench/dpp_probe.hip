// DPP / v_perm semantics probe (design tool): prints what lane l receives.
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int CTRL>
__device__ unsigned dpp(unsigned v) { return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false); }
__global__ void k(unsigned* out) {
  const unsigned l = threadIdx.x;
  out[l] = dpp<0x121>(l + 100);
  out[64 + l] = dpp<0x138>(l + 100);
  out[128 + l] = dpp<0x90>(l + 100);
  out[192 + l] = __builtin_amdgcn_perm(0x77665544u, 0x33221100u, 0x03020100u + (l & 7) * 0x01010101u);
}
int main() {
  unsigned* d;
  unsigned h[256];
  if (hipMalloc(&d, sizeof h)) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost)) return 2;
  const char* nm[3] = {"row_ror:1", "wave_shr:1", "quad_perm[0,0,1,2]"};
  for (int t = 0; t < 3; t++) {
    printf("%-20s", nm[t]);
    for (int l = 0; l < 20; l++) printf(" %u", h[64 * t + l] ? h[64 * t + l] - 100 : 999);
    printf("\n");
  }
  for (int s = 0; s < 8; s++) printf("perm s=%d -> %08x\n", s, h[192 + s]);
  return 0;
}
