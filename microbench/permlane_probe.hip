// v_permlane16_swap / v_permlane32_swap semantics probe (design tool)
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned* out) {
  const unsigned l = threadIdx.x;
  const auto a = __builtin_amdgcn_permlane16_swap(100 + l, 200 + l, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(100 + l, 200 + l, false, false);
  out[l] = a[0];
  out[64 + l] = a[1];
  out[128 + l] = b[0];
  out[192 + l] = b[1];
}
int main() {
  unsigned* d;
  unsigned h[256];
  if (hipMalloc(&d, sizeof h)) return 1;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost)) return 2;
  const char* nm[4] = {"p16 a(100+l)", "p16 b(200+l)", "p32 a(100+l)", "p32 b(200+l)"};
  for (int t = 0; t < 4; t++) {
    printf("%-14s", nm[t]);
    for (int l = 0; l < 64; l += 8) printf(" [%2d]%u", l, h[64 * t + l]);
    printf("\n");
  }
  return 0;
}
