// Probe: the VOP3P v_dot4_i32_i8 / v_dot2_i32_i16 forms written as inline asm
// vs the compiler builtins (v_dot*c), on random operands.  Prints mismatches.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef short s16x2 __attribute__((ext_vector_type(2)));
__global__ void k(const int *a, const int *b, const int *c, int *o, int n, int su, int sv) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  int r0 = __builtin_amdgcn_sdot4(a[i], b[i], c[i], false), r1, r2, r3, r4, r5;
  asm("v_dot4_i32_i8 %0, %1, %2, %3" : "=v"(r1) : "v"(a[i]), "v"(b[i]), "v"(c[i]));
  asm("v_dot4_i32_i8 %0, %1, %2, %3" : "=v"(r2) : "v"(a[i]), "s"(su), "v"(c[i]));
  const int q0 = __builtin_amdgcn_sdot2(__builtin_bit_cast(s16x2, a[i]), __builtin_bit_cast(s16x2, b[i]), c[i], false);
  asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r3) : "v"(a[i]), "v"(b[i]), "v"(c[i]));
  const int q1 = __builtin_amdgcn_sdot2(__builtin_bit_cast(s16x2, a[i]), __builtin_bit_cast(s16x2, sv), c[i], false);
  asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r4) : "v"(a[i]), "s"(sv), "v"(c[i]));
  const int q2 = __builtin_amdgcn_sdot4(a[i], su, 0, false);
  asm("v_dot4_i32_i8 %0, %1, %2, 0" : "=v"(r5) : "v"(a[i]), "s"(su));
  const int s0 = __builtin_amdgcn_sdot4(a[i], su, c[i], false);
  o[8 * i + 0] = r0 != r1;
  o[8 * i + 1] = s0 != r2;
  o[8 * i + 2] = q0 != r3;
  o[8 * i + 3] = q1 != r4;
  o[8 * i + 4] = q2 != r5;
  o[8 * i + 5] = r0;
  o[8 * i + 6] = r1;
  o[8 * i + 7] = 0;
}
int main() {
  const int n = 1 << 16;
  int *h = (int *)malloc(3 * n * 4), *o = (int *)malloc(8 * n * 4);
  srand(1);
  for (int i = 0; i < 3 * n; i++) h[i] = (rand() << 16) ^ rand();
  for (int i = 2 * n; i < 3 * n; i++) h[i] = (rand() % 2000000) - 1000000;
  int *d, *od;
  hipMalloc(&d, 3 * n * 4);
  hipMalloc(&od, 8 * n * 4);
  hipMemcpy(d, h, 3 * n * 4, hipMemcpyHostToDevice);
  k<<<n / 64, 64>>>(d, d + n, d + 2 * n, od, n, 0x05f9c301, 0x0013fff9);
  hipMemcpy(o, od, 8 * n * 4, hipMemcpyDeviceToHost);
  int bad[5] = {0};
  for (int i = 0; i < n; i++)
    for (int j = 0; j < 5; j++) bad[j] += o[8 * i + j];
  printf("mismatches: dot4 vv %d, dot4 vs %d, dot2 vv %d, dot2 vs %d, dot4 z %d  (example %d vs %d)\n", bad[0], bad[1],
         bad[2], bad[3], bad[4], o[5], o[6]);
  return 0;
}
