// Probe: VOP3P v_dot4_i32_i8 with the destination register tied to src0
// (v_dot4_i32_i8 vX, vX, s, vY), directly after the VALU op that wrote vX, and
// the same with s_nop padding, vs the builtin.  Prints mismatch counts.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
__global__ void k(const int *x, int *o, int n, int s0, int s1) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  const int a = x[2 * i], c = x[2 * i + 1];
  const int want = __builtin_amdgcn_sdot4(a ^ s1, s0, c, false);
  int r1, r2, r3;
  asm volatile("v_xor_b32 %0, %1, %2\n\tv_dot4_i32_i8 %0, %0, %3, %4" : "=&v"(r1) : "v"(a), "s"(s1), "s"(s0), "v"(c));
  asm volatile("v_xor_b32 %0, %1, %2\n\ts_nop 1\n\tv_dot4_i32_i8 %0, %0, %3, %4" : "=&v"(r2) : "v"(a), "s"(s1), "s"(s0), "v"(c));
  int t;
  asm volatile("v_xor_b32 %1, %2, %3\n\tv_dot4_i32_i8 %0, %1, %4, %5" : "=&v"(r3), "=&v"(t) : "v"(a), "s"(s1), "s"(s0), "v"(c));
  o[3 * i + 0] = r1 != want;
  o[3 * i + 1] = r2 != want;
  o[3 * i + 2] = r3 != want;
}
int main() {
  const int n = 1 << 16;
  int *h = (int *)malloc(2 * n * 4), *o = (int *)malloc(3 * n * 4);
  srand(1);
  for (int i = 0; i < 2 * n; i++) h[i] = (rand() << 16) ^ rand();
  int *d, *od;
  (void)hipMalloc(&d, 2 * n * 4);
  (void)hipMalloc(&od, 3 * n * 4);
  (void)hipMemcpy(d, h, 2 * n * 4, hipMemcpyHostToDevice);
  k<<<n / 64, 64>>>(d, od, n, 0x05f9c301, 0x80808080);
  (void)hipMemcpy(o, od, 3 * n * 4, hipMemcpyDeviceToHost);
  int bad[3] = {0};
  for (int i = 0; i < n; i++)
    for (int j = 0; j < 3; j++) bad[j] += o[3 * i + j];
  printf("dst==src0 right after its write: %d, with s_nop 1: %d, separate dst: %d mismatches\n", bad[0], bad[1], bad[2]);
  return 0;
}
