// Probe of the lane-butterfly primitives used by selscan_bwd_sg_k (permlane32/16 swap, DPP rotations)
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void probe(unsigned* o) {
  const int l = threadIdx.x;
  unsigned x = 1000 + l, y = 2000 + l;
  auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
  o[l] = r[0]; o[64 + l] = r[1];
  auto s = __builtin_amdgcn_permlane16_swap(x, y, false, false);
  o[128 + l] = s[0]; o[192 + l] = s[1];
  o[256 + l] = __builtin_amdgcn_update_dpp(0, (int)x, 0x128, 0xF, 0xF, false);  // row_ror:8
  o[320 + l] = __builtin_amdgcn_update_dpp(0, (int)x, 0x124, 0xF, 0xF, false);  // row_ror:4
  o[384 + l] = __builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, false);  // row_half_mirror
}
int main() {
  unsigned* d; hipMalloc(&d, 448 * 4);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  unsigned h[448]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* nm[7] = {"p32 r0", "p32 r1", "p16 r0", "p16 r1", "ror8", "ror4", "hmirror"};
  for (int k = 0; k < 7; ++k) {
    printf("%-8s", nm[k]);
    for (int l = 0; l < 64; ++l) printf(" %u", h[64 * k + l]);
    printf("\n");
  }
  return 0;
}
