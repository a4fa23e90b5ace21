#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
__global__ void k(const uint8_t* buf, uint32_t* out) {
  int t = threadIdx.x;  // t = byte offset 0..7
  const uint8_t* p = buf + 16 + t;
  uintptr_t a = (uintptr_t)p;
  const uint32_t* w = (const uint32_t*)(a & ~(uintptr_t)3);
  uint32_t sh = (uint32_t)(a & 3);
  uint32_t d0 = w[0], d1 = w[1], d2 = w[2];
  out[t*3+0] = __builtin_amdgcn_alignbyte(d1, d0, sh);
  out[t*3+1] = __builtin_amdgcn_alignbyte(d2, d1, sh);
  out[t*3+2] = sh;
}
int main() {
  uint8_t h[64]; for (int i=0;i<64;i++) h[i]=i;
  uint8_t* d; uint32_t* o; hipMalloc(&d,64); hipMalloc(&o,8*3*4);
  hipMemcpy(d,h,64,hipMemcpyHostToDevice);
  k<<<1,8>>>(d,o);
  uint32_t r[24]; hipMemcpy(r,o,sizeof(r),hipMemcpyDeviceToHost);
  for (int t=0;t<8;t++) printf("off %d sh %u e0 %08x e1 %08x\n", t, r[t*3+2], r[t*3], r[t*3+1]);
  return 0;
}
