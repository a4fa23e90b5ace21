// Host-side work lists of the batched decoder C-ABI (thor_build_clpf_list /
// _tu_list / _intra_list, include/thor_amd.h): plain C++, no HIP, so the
// fuzz harness (tools/fuzz/host_fuzz.cpp) builds it for the CPU under
// ASan + UBSan.  Included once, by capi.hip.
#pragma once
#include <stdint.h>

#include <vector>

#include "../../include/thor_amd.h"

// chroma_qp, common/common_block.c:78-83 (clamped index)
static int chroma_qp_host(int q) {
  static const int t[52] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17,
                            18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 29, 30, 31, 32, 33, 33,
                            34, 34, 35, 35, 36, 36, 37, 37, 38, 39, 40, 41, 42, 43, 44, 45};
  return t[q < 0 ? 0 : (q > 51 ? 51 : q)];
}

int thor_build_clpf_list(const uint8_t *host_flags, int nsb, uint32_t *out) {
  if (nsb < 0 || (nsb > 0 && !host_flags)) return THOR_ERR_ARG;
  int n = 0;
  for (int i = 0; i < nsb; i++)
    if (host_flags[i]) {
      if (out) out[n] = (uint32_t)i;
      n++;
    }
  return n;
}

int thor_build_tu_list(const thor_block_t *host_blocks, int nblocks, thor_tu_t *out) {
  if (nblocks < 0 || (nblocks > 0 && !host_blocks)) return THOR_ERR_ARG;
  int n = 0;
  for (int b = 0; b < nblocks; b++) {
    const thor_block_t &B = host_blocks[b];
    if (B.mode == 0 /* M_SKIP */) continue;  // SKIP carries no residual (dec/decode_block.c:213-242)
    for (int c = 0; c < 3; c++) {
      if (!((B.coeff_mask >> c) & 1)) continue;
      // tb-split gives 4 quarters; chroma of an 8x8 CU is not split (dec/decode_block.c:449-450)
      const int split = B.tb_split && (c == 0 || B.size > 8);
      const int size = c ? B.size >> 1 : B.size, ntu = split ? size >> 1 : size;
      const int nt = ntu == 64 ? 32 : ntu, q = nt < 16 ? nt : 16;
      const int py = c ? B.ypos >> 1 : B.ypos, px = c ? B.xpos >> 1 : B.xpos;
      for (int t = 0; t < (split ? 4 : 1); t++) {  // quarters in raster order, :101-102
        if (out) {
          thor_tu_t &T = out[n];
          T.coeff_off = B.coeff_off[c] + (uint32_t)(t * q * q);
          T.y = (uint16_t)(py + (t >> 1) * ntu);
          T.x = (uint16_t)(px + (t & 1) * ntu);
          T.size = (uint8_t)ntu;
          T.comp = (uint8_t)c;
          T.qp = (uint8_t)(c ? chroma_qp_host(B.qp) : (B.qp > 51 ? 51 : B.qp));  // a corrupt qp clamps as chroma_qp_host does
          T.rsv = 0;
        }
        n++;
      }
    }
  }
  return n;
}

int thor_build_intra_list(const thor_block_t *host_blocks, int nblocks, uint32_t *out) {
  if (nblocks < 0 || (nblocks > 0 && !host_blocks)) return THOR_ERR_ARG;
  int n = 0;
  for (int b = 0; b < nblocks; b++)
    if (host_blocks[b].mode == 1 /* M_INTRA */) {
      if (out) out[n] = (uint32_t)b;
      n++;
    }
  return n;
}

// The multi-key k_recon units of a frame (include/thor_amd.h).  Restates the
// classification k_frame_prep applies when it writes the half-SB plans
// (prep_body, recon.hip): a half SB is planned when one 64x64 inter CU covers it
// with one (MV, reference) key per prediction pass, and multi-key when it holds
// a smaller inter CU or a 64x64 INTER / BIPRED CU whose two quarters there differ
// (mv_arr per quarter, dec/decode_block.c:381-392).  Units in ascending order.
int thor_build_slow_list(const thor_block_t *host_blocks, int nblocks, int width, int height, uint32_t *out) {
  if (nblocks < 0 || (nblocks > 0 && !host_blocks) || width <= 0 || height <= 0) return THOR_ERR_ARG;
  const int sbw = (width + 63) >> 6, sbh = (height + 63) >> 6, np = (sbw + 1) >> 1;
  std::vector<uint8_t> slow((size_t)2 * sbw * sbh, 0);  // per half SB (FrameCtx::hplan order)
  for (int b = 0; b < nblocks; b++) {
    const thor_block_t &B = host_blocks[b];
    if (B.mode == 1 /* M_INTRA */) continue;
    const int sbx = B.xpos >> 6, sby = B.ypos >> 6;
    if (sbx >= sbw || sby >= sbh) continue;  // outside the frame: k_frame_prep marks nothing either
    const int hs = 2 * (sby * sbw + sbx);
    if (B.size < 64) {
      slow[hs + ((B.ypos & 63) >= 32)] = 1;
      continue;
    }
    const bool quarters = B.mode == 2 || B.mode == 3;  // M_INTER, M_BIPRED
    const bool bi = B.mode == 3 || ((B.mode == 0 || B.mode == 4) && B.dir == 2);
    for (int h = 0; h < 2; h++) {
      const int q0 = quarters ? 2 * h : 0, q1 = quarters ? 2 * h + 1 : 0;
      const bool same = B.mv0[2 * q0] == B.mv0[2 * q1] && B.mv0[2 * q0 + 1] == B.mv0[2 * q1 + 1] &&
                        (!bi || (B.mv1[2 * q0] == B.mv1[2 * q1] && B.mv1[2 * q0 + 1] == B.mv1[2 * q1 + 1]));
      if (!same && B.ypos + 32 * h < height) slow[hs + h] = 1;
    }
  }
  int n = 0;
  for (int sby = 0; sby < sbh; sby++)
    for (int q = 0; q < 4; q++)  // slice row 4 x sby + q: half q >> 1
      for (int p = 0; p < np; p++) {
        const int h = q >> 1, l = 2 * (sby * sbw + 2 * p) + h;
        if (!slow[l] && !(2 * p + 1 < sbw && slow[l + 2])) continue;
        if (out) out[n] = (uint32_t)((4 * sby + q) * np + p);
        n++;
      }
  return n;
}
