// probe: do unaligned dword loads / stores from global and LDS return the bytes at the address?
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
typedef uint32_t __attribute__((aligned(1))) u32u;
__global__ void k(const uint8_t *g, uint32_t *out, uint8_t *gs) {
  __shared__ uint8_t l[256];
  const int t = threadIdx.x;
  for (int i = t; i < 256; i += 64) l[i] = g[i];
  __syncthreads();
  uint8_t *volatile lp = l;  // generic pointer into LDS
  out[t] = *(const u32u *)(g + t);
  out[64 + t] = *(const u32u *)(lp + t);
  if (t < 16) *(u32u *)(gs + 4 * t + 1) = 0x04030201u * (t + 1);
}
int main() {
  uint8_t h[256], *g, *gs;
  for (int i = 0; i < 256; i++) h[i] = (uint8_t)i;
  uint32_t *o, ho[128];
  hipMalloc(&g, 256); hipMalloc(&o, 512); hipMalloc(&gs, 128);
  hipMemcpy(g, h, 256, hipMemcpyHostToDevice);
  hipMemset(gs, 0, 128);
  k<<<1, 64>>>(g, o, gs);
  hipMemcpy(ho, o, 512, hipMemcpyDeviceToHost);
  uint8_t hs[128];
  hipMemcpy(hs, gs, 128, hipMemcpyDeviceToHost);
  int bad_g = 0, bad_l = 0, bad_s = 0;
  for (int t = 0; t < 64; t++) {
    uint32_t want = t | (t + 1) << 8 | (t + 2) << 16 | (uint32_t)(t + 3) << 24;
    bad_g += ho[t] != want;
    bad_l += ho[64 + t] != want;
  }
  for (int t = 0; t < 16; t++)
    for (int b = 0; b < 4; b++) bad_s += hs[4 * t + 1 + b] != (uint8_t)((b + 1) * (t + 1));
  printf("unaligned global load mismatches %d, LDS load mismatches %d, global store mismatches %d\n", bad_g, bad_l, bad_s);
  printf("g[1]=%08x l[1]=%08x\n", ho[1], ho[65]);
  return 0;
}
