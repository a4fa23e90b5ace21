// Residuals of every coded transform block of a frame (gfx950), computed in k_prep_resid.
//
// Restates the residual half of decode_and_reconstruct_block_inter / _intra
// (dec/decode_block.c:48-120): dequantize (common/common_block.c:132-146),
// then the 2-D inverse transform (common/transform.c:432-518: pass 1 over the
// coded columns with clip16((s + 64) >> 7) between passes, pass 2 with
// clip16((s + 2048) >> 12); 64x64 = 32-point transform + 2x2 replication,
// :496-517).  The residual does not depend on any neighbour, so it runs for
// the whole frame before prediction: one 64-lane workgroup per (CU,
// component); the result goes to the frame's int16 residual planes (Y W x H,
// then U and V W/2 x H/2), where k_recon adds it to inter predictions and
// k_intra to intra ones.
//
// Only the low-frequency q x q corner (q = min(N,16)) can be coded
// (common/transform.c:309-327), so pass 1 runs over q columns and pass 2 over
// q terms: the coded tile is the whole input.
#include "common.h"

// 32-point basis (g*mat_hevc, common/transform.c:41-245) as a constant table.
struct Dct32Table {
  int8_t v[1024];
  constexpr Dct32Table() : v() {
    const int c[33] = {64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67, 64,
                       61, 57, 54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9,  4,  0};
    for (int k = 0; k < 32; k++)
      for (int n = 0; n < 32; n++) {
        int e = 0;
        if (k == 0) e = 64;
        else {
          int t = (k * (2 * n + 1)) & 127;
          e = t <= 32 ? c[t] : (t <= 64 ? -c[64 - t] : (t <= 96 ? -c[t - 64] : c[128 - t]));
        }
        v[k * 32 + n] = (int8_t)e;
      }
  }
};
__constant__ Dct32Table g_dct32 = Dct32Table();

struct ResidLds {
  int16_t D[256];      // dequantised q x q tile, transposed: D[k][m]
  int16_t T[16 * 32];  // pass-1 output, transposed: T[y][k]
};

__device__ __forceinline__ int sx8(int w, int i) { return __builtin_amdgcn_sbfe(w, 8 * i, 8); }

// Basis columns as int16 pairs for the inverse passes: for an n-point TU (n =
// 4, 8, 16, 32), column p holds (M[2j*step][p], M[(2j+1)*step][p]) for the q =
// min(n,16) coefficient rows, step = 32/n.  4 KB; each lane loads its 8 words.
struct MColTable {
  uint32_t v[4][32][8];
  constexpr MColTable() : v() {
    const int c[33] = {64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67, 64,
                       61, 57, 54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9,  4,  0};
    for (int s = 0; s < 4; s++) {
      const int n = 4 << s, step = 32 / n, q = n < 16 ? n : 16;
      for (int p = 0; p < n; p++)
        for (int j = 0; j < 8; j++) {
          int e[2] = {0, 0};
          for (int h = 0; h < 2; h++) {
            const int k = (2 * j + h) * step;
            if (2 * j + h >= q) continue;
            if (k == 0) e[h] = 64;
            else {
              const int t = (k * (2 * p + 1)) & 127;
              e[h] = t <= 32 ? c[t] : (t <= 64 ? -c[64 - t] : (t <= 96 ? -c[t - 64] : c[128 - t]));
            }
          }
          v[s][p][j] = ((uint32_t)e[0] & 0xffffu) | ((uint32_t)e[1] << 16);
        }
    }
  }
};
__constant__ MColTable g_mcol = MColTable();

typedef short s16x2_r __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int rdot2(uint32_t a, uint32_t b, int c) {  // a.lo*b.lo + a.hi*b.hi + c (int16 pairs)
  return __builtin_amdgcn_sdot2(__builtin_bit_cast(s16x2_r, a), __builtin_bit_cast(s16x2_r, b), c, false);
}

// One TU across the wave; writes the n x n (x2 replicated for 64) residual
// at `out` (row stride `ostride` int16).  Lane p = lane % n owns basis column
// p (q basis rows as int16 pairs in registers); the dequantised coefficients
// (transposed) and the pass-1 output (transposed) are read as int16 pairs
// broadcast to every lane of a group, so each pass is q/2 v_dot2 per output.
__device__ void tu_inverse(ResidLds &L, const int16_t *__restrict__ coef, int ntu, int qp, int16_t *__restrict__ out,
                           int ostride) {
  const int lane = threadIdx.x & 63;
  const int rep = ntu == 64, n = rep ? 32 : ntu, q = n < 16 ? n : 16;
  const int step = 32 / n;
  const int lshift = qp / 6, scale = dequant_scale(qp % 6);
  const int rshift = ilog2i(ntu) - 1, add = 1 << (rshift - 1);
  for (int e = lane; e < q * q; e += 64) {  // dequantize (int16 store, common_block.c:143), transposed
    const int m = e / q, k = e - m * q;
    L.D[k * q + m] = (int16_t)wrap16(((coef[e] * scale) * (1 << lshift) + add) >> rshift);
  }
  const int p = lane & (n - 1), grp = lane / n, ngrp = 64 / n;
  const uint4 *mp = (const uint4 *)g_mcol.v[ilog2i(n) - 2][p];
  const uint4 m0 = mp[0], m1 = mp[1];
  const uint32_t mc[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
  (void)step;
  wave_lds_sync();
  for (int k = grp; k < q; k += ngrp) {  // pass 1, transform.c:455-463: T[k][p]
    const uint32_t *dk = (const uint32_t *)&L.D[k * q];
    int s = 64;
#pragma unroll
    for (int j = 0; j < 8; j++)
      if (2 * j < q) s = rdot2(mc[j], dk[j], s);
    L.T[p * q + k] = (int16_t)clip16(s >> 7);
  }
  wave_lds_sync();
  for (int y = grp; y < n; y += ngrp) {  // pass 2, :466-484: out[y][p]
    const uint32_t *ty = (const uint32_t *)&L.T[y * q];
    int s = 2048;
#pragma unroll
    for (int j = 0; j < 8; j++)
      if (2 * j < q) s = rdot2(mc[j], ty[j], s);
    const int r = clip16(s >> 12);
    if (rep) {  // 2x2 replication
      const uint32_t w = (uint32_t)(r & 0xffff) * 0x10001u;
      *(uint32_t *)(out + (long long)(2 * y) * ostride + 2 * p) = w;
      *(uint32_t *)(out + (long long)(2 * y + 1) * ostride + 2 * p) = w;
    } else {
      out[(long long)y * ostride + p] = (int16_t)r;
    }
  }
  wave_lds_sync();  // the next TU rewrites D and T
}

// resid_tu: one wavefront per coded transform block, from the frame's TU list
// (thor_build_tu_list: coefficient offset, position, size, component, qp).
// Every TU is independent, so the launch is as wide as the frame's coded
// residual and a skip-dominated P frame launches only a handful of waves.
__device__ __forceinline__ void resid_tu(ResidLds &L, int idx, const thor_tu_t *__restrict__ tus, int ntus,
                                         const int16_t *__restrict__ coeffs, int16_t *__restrict__ resid, int W, int H) {
  if (idx >= ntus) return;
  const thor_tu_t T = tus[idx];
  const int c = T.comp, ntu = T.size;
  const int pw = c ? W >> 1 : W;
  int16_t *plane = resid + (c == 0 ? 0 : (long long)W * H + (c == 2 ? (long long)(W >> 1) * (H >> 1) : 0));
  wave_lds_sync();
  tu_inverse(L, coeffs + T.coeff_off, ntu, T.qp, plane + (long long)T.y * pw + T.x, pw);
}
