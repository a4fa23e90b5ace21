// Probe: chains of VOP3P v_dot4_i32_i8 / v_dot2_i32_i16 written as inline asm
// (each result the next one's accumulator, back to back) vs the builtins, and
// the same chains with s_nop padding.  Prints mismatch counts.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int a4(int a, int s, int c) { int r; asm("v_dot4_i32_i8 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(s), "v"(c)); return r; }
__device__ __forceinline__ int a4n(int a, int s, int c) { int r; asm("v_dot4_i32_i8 %0, %1, %2, %3\n\ts_nop 4" : "=v"(r) : "v"(a), "s"(s), "v"(c)); return r; }
__device__ __forceinline__ int a2(int a, int s, int c) { int r; asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(s), "v"(c)); return r; }
__device__ __forceinline__ int a2n(int a, int s, int c) { int r; asm("v_dot2_i32_i16 %0, %1, %2, %3\n\ts_nop 4" : "=v"(r) : "v"(a), "s"(s), "v"(c)); return r; }
__device__ __forceinline__ int b4(int a, int s, int c) { return __builtin_amdgcn_sdot4(a, s, c, false); }
__device__ __forceinline__ int b2(int a, int s, int c) { return __builtin_amdgcn_sdot2(__builtin_bit_cast(s16x2, a), __builtin_bit_cast(s16x2, s), c, false); }
__global__ void k(const int *x, int *o, int n, int s0, int s1, int s2) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  const int a = x[3 * i], b = x[3 * i + 1], c = x[3 * i + 2];
  const int r0 = b4(a, s0, b4(b, s1, b4(c, s2, 8224)));
  const int r1 = a4(a, s0, a4(b, s1, a4(c, s2, 8224)));
  const int r2 = a4n(a, s0, a4n(b, s1, a4n(c, s2, 8224)));
  const int q0 = b2(a, s0, b2(b, s1, b2(c, s2, 0)));
  const int q1 = a2(a, s0, a2(b, s1, a2(c, s2, 0)));
  const int q2 = a2n(a, s0, a2n(b, s1, a2n(c, s2, 0)));
  o[4 * i + 0] = r0 != r1;
  o[4 * i + 1] = r0 != r2;
  o[4 * i + 2] = q0 != q1;
  o[4 * i + 3] = q0 != q2;
}
int main() {
  const int n = 1 << 16;
  int *h = (int *)malloc(3 * n * 4), *o = (int *)malloc(4 * n * 4);
  srand(1);
  for (int i = 0; i < 3 * n; i++) h[i] = (rand() << 16) ^ rand();
  int *d, *od;
  (void)hipMalloc(&d, 3 * n * 4);
  (void)hipMalloc(&od, 4 * n * 4);
  (void)hipMemcpy(d, h, 3 * n * 4, hipMemcpyHostToDevice);
  k<<<n / 64, 64>>>(d, od, n, 0x05f9c301, 0x7f80017f, 0x0013fff9);
  (void)hipMemcpy(o, od, 4 * n * 4, hipMemcpyDeviceToHost);
  int bad[4] = {0};
  for (int i = 0; i < n; i++)
    for (int j = 0; j < 4; j++) bad[j] += o[4 * i + j];
  printf("chain mismatches: dot4 asm %d, dot4 asm+nop %d, dot2 asm %d, dot2 asm+nop %d\n", bad[0], bad[1], bad[2], bad[3]);
  return 0;
}
