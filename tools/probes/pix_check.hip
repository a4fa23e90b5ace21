// probe: the encoder's pixel primitives (enc_pix.h / enc_rd.h) on the GPU vs
// the same source built for the host (TE_HOST).  Writes pix_<dev|host>.out;
// compare the two files.  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o pix_dev pix_check.hip
//   g++ -x c++ -O2 -std=c++17 -DTE_HOST -o pix_host pix_check.hip
#if !defined(TE_HOST)
#include <hip/hip_runtime.h>
#endif
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include "../../thor_amd/csrc/enc_rd.h"

#define RS 256
#define NC 512
struct Case {
  int kind, w, h, mvx, mvy, sign, bipred, oa, ob;
};
TE_FN void run_case(const Case &c, const uint8_t *ref, uint8_t *dst, uint32_t *res) {
  const uint8_t *a = ref + 100 * RS + 100 + c.oa, *b = ref + 120 * RS + 90 + c.ob;
  TeMv mv;
  mv.x = (int16_t)c.mvx;
  mv.y = (int16_t)c.mvy;
  int x = 0, y = 0;
  switch (c.kind) {
    case 0: te_mc_luma(dst, c.w, a, RS, c.w, c.h, mv, c.sign, c.bipred); break;
    case 1: te_mc_chroma(dst, c.w, a, RS, c.w, c.h, mv, c.sign); break;
    case 2: res[0] = te_sad(a, RS, b, RS, c.w, c.h); break;
    case 3: res[0] = te_ssd(a, RS, b, RS, c.w, c.h); break;
    case 4: res[0] = te_widesad(a, RS, b, RS, c.w, c.h, &x); res[1] = (uint32_t)x; break;
    case 5: te_avg_rect(dst, c.w, a, RS, b, RS, c.w, c.h); break;
    case 6: te_copy_rect(dst, c.w, a, RS, c.w, c.h); break;
    case 7: res[0] = te_fasthalf(a, RS, b, RS, c.w, c.h, &x, &y); res[1] = (uint32_t)x; res[2] = (uint32_t)y; break;
  }
  te_sync();
}
#if !defined(TE_HOST)
__global__ void k(const Case *cs, const uint8_t *ref, uint8_t *dst, uint32_t *res) {
  run_case(cs[blockIdx.x], ref, dst + blockIdx.x * 4096, res + blockIdx.x * 4);
}
#endif
int main() {
  std::vector<uint8_t> ref(RS * RS);
  uint32_t s = 12345;
  for (auto &v : ref) {
    s = s * 1103515245u + 12345u;
    v = (uint8_t)(s >> 16);
  }
  std::vector<Case> cs(NC);
  const int ws[] = {4, 8, 16, 32, 64, 2};
  for (int i = 0; i < NC; i++) {
    s = s * 1103515245u + 12345u;
    Case &c = cs[i];
    c.kind = i % 8;
    c.w = ws[(i / 8) % 6];
    c.h = ws[(i / 48) % 5];
    if (c.kind != 0 && c.kind != 1 && c.w == 2) c.w = 4;
    c.mvx = (int)((s >> 8) % 61) - 30;
    c.mvy = (int)((s >> 16) % 61) - 30;
    c.sign = (s >> 3) & 1;
    c.bipred = (s >> 4) & 1;
    c.oa = (int)((s >> 5) % 7);
    c.ob = (int)((s >> 11) % 5);
  }
  std::vector<uint8_t> dst(NC * 4096, 0);
  std::vector<uint32_t> res(NC * 4, 0);
#if defined(TE_HOST)
  for (int i = 0; i < NC; i++) run_case(cs[i], ref.data(), dst.data() + i * 4096, res.data() + i * 4);
  FILE *f = fopen("pix_host.out", "wb");
#else
  Case *dc;
  uint8_t *dref, *ddst;
  uint32_t *dres;
  (void)hipMalloc(&dc, NC * sizeof(Case));
  (void)hipMalloc(&dref, RS * RS);
  (void)hipMalloc(&ddst, NC * 4096);
  (void)hipMalloc(&dres, NC * 16);
  (void)hipMemcpy(dc, cs.data(), NC * sizeof(Case), hipMemcpyHostToDevice);
  (void)hipMemcpy(dref, ref.data(), RS * RS, hipMemcpyHostToDevice);
  (void)hipMemset(ddst, 0, NC * 4096);
  (void)hipMemset(dres, 0, NC * 16);
  k<<<NC, 64>>>(dc, dref, ddst, dres);
  (void)hipMemcpy(dst.data(), ddst, NC * 4096, hipMemcpyDeviceToHost);
  (void)hipMemcpy(res.data(), dres, NC * 16, hipMemcpyDeviceToHost);
  FILE *f = fopen("pix_dev.out", "wb");
#endif
  fwrite(dst.data(), 1, dst.size(), f);
  fwrite(res.data(), 4, res.size(), f);
  fclose(f);
  return 0;
}
