// VALU throughput probe (gfx950): cycles per wave-instruction of the integer
// ops k_recon's filters use, with every SIMD holding W waves.  Timing only.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef short s16x2 __attribute__((ext_vector_type(2)));
template <int OP>
__global__ __launch_bounds__(64) void k(unsigned *out, int iters, unsigned seed) {
  unsigned a[8];
  for (int j = 0; j < 8; j++) a[j] = seed * (threadIdx.x + 17 * j + 1);
  const unsigned b = seed ^ 0x01fe03fdu, c = seed * 3u;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if (OP == 0) a[j] = a[j] + b;
      if (OP == 1) a[j] = (unsigned)__builtin_amdgcn_sdot4((int)c, (int)b, (int)a[j], false);
      if (OP == 2) a[j] = (unsigned)__builtin_amdgcn_sdot2(__builtin_bit_cast(s16x2, c), __builtin_bit_cast(s16x2, b), (int)a[j], false);
      if (OP == 3) a[j] = __builtin_amdgcn_perm(a[j], b, 0x05040100u);
      if (OP == 4) a[j] = __builtin_amdgcn_alignbyte(a[j], b, 3);
      if (OP == 5) a[j] = (unsigned)__builtin_amdgcn_udot4(c, b, a[j], false);
    }
  }
  unsigned s = 0;
  for (int j = 0; j < 8; j++) s ^= a[j];
  if (s == 0x12345678u) out[threadIdx.x] = s;
}
int main() {
  unsigned *o;
  hipMalloc(&o, 4096);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char *names[] = {"v_add_u32", "v_dot4_i32_i8", "v_dot2_i32_i16", "v_perm_b32", "v_alignbyte", "v_dot4_u32_u8"};
  const int iters = 4096;
  for (int W = 1; W <= 8; W *= 2) {
    const int grid = 256 * 4 * W;
    for (int op = 0; op < 6; op++) {
      auto run = [&] {
        switch (op) {
          case 0: k<0><<<grid, 64>>>(o, iters, 7); break;
          case 1: k<1><<<grid, 64>>>(o, iters, 7); break;
          case 2: k<2><<<grid, 64>>>(o, iters, 7); break;
          case 3: k<3><<<grid, 64>>>(o, iters, 7); break;
          case 4: k<4><<<grid, 64>>>(o, iters, 7); break;
          default: k<5><<<grid, 64>>>(o, iters, 7); break;
        }
      };
      run();
      hipEventRecord(e0);
      for (int r = 0; r < 5; r++) run();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double instr_per_simd = (double)W * iters * 8;  // wave-instructions per SIMD per launch
      printf("waves/SIMD %d  %-16s %.3f ns per wave-instruction per SIMD (%.2f cycles at 2.4 GHz)\n", W, names[op],
             ms * 1e6 / 5 / instr_per_simd, ms * 1e6 / 5 / instr_per_simd * 2.4);
    }
  }
  return 0;
}
