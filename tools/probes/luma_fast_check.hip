// Probe: k_recon's fast-path luma / chroma filters (luma8_fast, chroma4_fast)
// against the round-2 forms (luma_rows, chroma_rows) on the same random LDS
// window, for every (bipred, fx, fy, sh).  Prints mismatch counts per case.
#include "../../thor_amd/csrc/recon.hip"
#include "../../thor_amd/csrc/inter.hip"
#include <stdio.h>
__global__ void kk(const uint8_t *src, int *bad) {
  __shared__ RefWin w;
  const int lane = threadIdx.x, cc = lane & 15, gr = lane >> 4;
  for (int i = lane; i < (int)sizeof(RefWin); i += 64) ((uint8_t *)&w)[i] = src[blockIdx.x * 7 + i];
  wave_lds_sync();
  const int bip = blockIdx.y & 1, fx = (blockIdx.y >> 1) & 3, fy = (blockIdx.y >> 3) & 3, sh = blockIdx.z;
  if (fx == 2 && fy == 2) return;
  const int lwb = 4 * cc + sh;
  int v01, v23, v45;
  tap_pairs6(g_taps.luma[bip][fy][0], g_taps.luma[bip][fy][1], v01, v23, v45);
  uint32_t a[8], b[8];
  const LdsLuma l{w.y + 8 * gr * WL_P + (lwb & ~3)};
  luma_rows<0, 8>(l, (uint32_t)(lwb & 3), g_taps.luma[bip][fx][0], g_taps.luma[bip][fx][1], v01, v23, v45, a, false);
  const unsigned long long th48 = (unsigned long long)(uint32_t)g_taps.luma[bip][fx][0] |
                                  ((unsigned long long)(uint32_t)(g_taps.luma[bip][fx][1] & 0xffff) << 32);
  luma8_fast(w.y + 8 * gr * WL_P + (lwb & ~3), lwb & 3, th48, v01, v23, v45, b, false);
  int n = 0;
  for (int i = 0; i < 8; i++) n += a[i] != b[i];
  if (n) atomicAdd(&bad[blockIdx.y * 4 + blockIdx.z], n);
  if (blockIdx.x == 0 && blockIdx.y == 2 && blockIdx.z == 0 && lane < 2)
    for (int i = 0; i < 8; i++) printf("lane %d row %d old %08x new %08x\n", lane, i, a[i], b[i]);
  // chroma with the same fractions (x2 for eighths)
  const int cfx = 2 * fx + bip, cfy = 2 * fy, cwb = 2 * cc + sh;
  const int cvt = g_taps.chroma[cfy];
  const int c01 = (tap8(cvt, 0) & 0xffff) | (tap8(cvt, 1) << 16), c23 = (tap8(cvt, 2) & 0xffff) | (tap8(cvt, 3) << 16);
  uint32_t ca[4], cb[4];
  const LdsChroma c{w.u + 4 * gr * WC_P + (cwb & ~3), w.v + 4 * gr * WC_P + (cwb & ~3)};
  chroma_rows<0, 4>(c, (uint32_t)(cwb & 3), g_taps.chroma[cfx], c01, c23, ca, false);
  chroma4_fast(w.u + 4 * gr * WC_P + (cwb & ~3), w.v + 4 * gr * WC_P + (cwb & ~3), cwb & 3,
               (unsigned long long)(uint32_t)g_taps.chroma[cfx], c01, c23, cb, false);
  n = 0;
  for (int i = 0; i < 4; i++) n += ca[i] != cb[i];
  if (n) atomicAdd(&bad[64 + blockIdx.y * 4 + blockIdx.z], n);
}
int main() {
  const int N = 64 * 7 + 8192;
  uint8_t *h = (uint8_t *)malloc(N);
  srand(3);
  for (int i = 0; i < N; i++) h[i] = rand() & 255;
  uint8_t *d;
  int *bad, hb[128];
  (void)hipMalloc(&d, N);
  (void)hipMalloc(&bad, sizeof(hb));
  (void)hipMemcpy(d, h, N, hipMemcpyHostToDevice);
  (void)hipMemset(bad, 0, sizeof(hb));
  kk<<<dim3(64, 16, 4), 64>>>(d, bad);
  (void)hipMemcpy(hb, bad, sizeof(hb), hipMemcpyDeviceToHost);
  int tot = 0;
  for (int y = 0; y < 16; y++)
    for (int z = 0; z < 4; z++) {
      if (hb[y * 4 + z] || hb[64 + y * 4 + z])
        printf("bip %d fx %d fy %d sh %d: luma %d chroma %d words differ\n", y & 1, (y >> 1) & 3, (y >> 3) & 3, z,
               hb[y * 4 + z], hb[64 + y * 4 + z]);
      tot += hb[y * 4 + z] + hb[64 + y * 4 + z];
    }
  printf("total differing words: %d\n", tot);
  return 0;
}
