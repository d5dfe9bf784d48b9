// lane_sum8 as in selective_scan.hip vs a host reduction
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
template <int CTRL>
__device__ __forceinline__ float dppf(float old, float src) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old), __builtin_bit_cast(int, src),
                                                               CTRL, 0xF, 0xF, false));
}
// v_permlane32_swap / v_permlane16_swap: x <- [x_lo, y_lo], y <- [x_hi, y_hi] (32-lane halves), and
// x <- [x_r0, y_r0, x_r2, y_r2], y <- [x_r1, y_r1, x_r3, y_r3] (16-lane rows).  Inline asm: the compiler's
// builtins for these return the first result twice (ROCm 7.2 clang: `v_add x, x` after the swap).
__device__ __forceinline__ void permlane32_swap(float& x, float& y) {
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(x), "+v"(y));
}
__device__ __forceinline__ void permlane16_swap(float& x, float& y) {
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 1" : "+v"(x), "+v"(y));
}
__device__ float* dbg;
__device__ __forceinline__ float lane_sum8(const float (&v)[8]) {
  const int lane = threadIdx.x & 63;
  float w4[4], w2[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float x = v[i], y = v[i + 4];
    permlane32_swap(x, y);
    w4[i] = x + y;
    dbg[i * 64 + lane] = w4[i];
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    float x = w4[i], y = w4[i + 2];
    permlane16_swap(x, y);
    w2[i] = x + y;
    dbg[(4 + i) * 64 + lane] = w2[i];
  }
  const float p = w2[0] + dppf<0x128>(0.f, w2[0]);
  const float q = w2[1] + dppf<0x128>(0.f, w2[1]);
  float z = (lane & 8) ? q : p;
  dbg[6 * 64 + lane] = z;
  z += dppf<0x141>(0.f, z);
  z += dppf<0xB1>(0.f, z);
  z += dppf<0x4E>(0.f, z);
  return z;
}
__global__ void k(const float* in, float* out) {
  float v[8];
  for (int i = 0; i < 8; ++i) v[i] = in[i * 64 + threadIdx.x];
  out[threadIdx.x] = lane_sum8(v);
}
int main() {
  float h[512], r[64];
  for (int i = 0; i < 512; ++i) h[i] = (float)((i * 7919) % 1000) / 100.f;
  float *di, *dout; hipMalloc(&di, sizeof(h)); hipMalloc(&dout, sizeof(r));
  hipMemcpy(di, h, sizeof(h), hipMemcpyHostToDevice);
  float* dd; hipMalloc(&dd, 7 * 64 * 4);
  hipMemcpyToSymbol(HIP_SYMBOL(dbg), &dd, sizeof(dd));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, di, dout);
  float hd[7 * 64]; hipMemcpy(hd, dd, sizeof(hd), hipMemcpyDeviceToHost);
  // expected stage values
  for (int st = 0; st < 7; ++st) {
    int bad = 0;
    for (int l = 0; l < 64; ++l) {
      float e = 0; int nlanes = 0;
      for (int m = 0; m < 64; ++m) {
        int vi; bool in;
        if (st < 4) { vi = st + 4 * ((l >> 5) & 1); in = ((m ^ l) & ~32) == 0; }
        else if (st < 6) { vi = (st - 4) + 2 * ((l >> 4) & 1) + 4 * ((l >> 5) & 1); in = ((m ^ l) & ~48) == 0; }
        else { vi = ((l >> 3) & 7); in = ((m ^ l) & ~56) == 0; }
        if (in) { e += h[vi * 64 + m]; ++nlanes; }
      }
      if (fabsf(hd[st * 64 + l] - e) > 1e-3f * fabsf(e)) { if (bad < 3) printf("stage %d lane %d got %f want %f\n", st, l, hd[st*64+l], e); ++bad; }
    }
    printf("stage %d bad %d\n", st, bad);
  }
  hipMemcpy(r, dout, sizeof(r), hipMemcpyDeviceToHost);
  float ex[8] = {0};
  for (int i = 0; i < 8; ++i) for (int l = 0; l < 64; ++l) ex[i] += h[i * 64 + l];
  int bad = 0;
  for (int l = 0; l < 64; ++l) {
    const float e = ex[(l >> 3) & 7];
    if (fabsf(r[l] - e) > 1e-3f * fabsf(e)) { ++bad; if (bad < 10) printf("lane %d got %f want %f\n", l, r[l], e); }
  }
  printf("expected:"); for (int i = 0; i < 8; ++i) printf(" %f", ex[i]); printf("\n");
  printf("got lanes 0,8,..:"); for (int l = 0; l < 64; l += 8) printf(" %f", r[l]); printf("\nbad=%d\n", bad);
  return 0;
}
