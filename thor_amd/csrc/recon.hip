// Per-frame reconstruction kernels for gfx950 (MI355X): cell side-info,
// inter MC + dequant + inverse transform + reconstruction, intra.
//
// Layout: frames live in a ring of padded slots in HBM (pad 96 luma / 48
// chroma, create_yuv_frame, common/common_frame.c:324-351).  The current
// frame is reconstructed in place into its slot; deblock / CLPF / pad then
// run in place (loopfilter.hip), after which the slot is a reference.
#include "common.h"

// ---------------------------------------------------------------------------
// prep_body (k_frame_prep, intra.hip): one wavefront per CU.  Writes the per-4x4 cell map (CU index) and
// the packed side-info that copy_deblock_data (dec/decode_block.c:122-156)
// stores for deblocking/CLPF.
// ---------------------------------------------------------------------------
// A half with several (MV, reference) keys: tag its plan record as multi-key
// (common.h), so the planned-order workgroup of each of its two k_recon units
// leaves them to the slow-list workgroups (thor_build_slow_list lists the same
// units).  Every CU of the half stores the same record: no atomics.
__device__ __forceinline__ void slow_mark(const FrameCtx &f, int sbx, int sby, int h) {
  const int sbw = (f.W + 63) >> 6;
  if (sbx >= sbw || sby >= ((f.H + 63) >> 6)) return;
  f.hplan[2 * (sby * sbw + sbx) + h] = make_uint4(0u, PLAN_SLOW, 0u, (unsigned)f.gen);
}

// PREP_CPW CUs per wave, 64 / PREP_CPW lanes each (round 6: 4 -- a 4K P frame is ~2 000 64x64 SKIP CUs
// whose waves spent their short lives waiting on one descriptor load; a quarter as many waves, the four
// descriptor loads of a wave in flight together)
#ifndef PREP_CPW
#define PREP_CPW 4
#endif
#define PREP_LPC (64 / PREP_CPW)
__device__ __forceinline__ void prep_body(int bx, const FrameCtx &f) {
  const int b = (bx * 4 + (threadIdx.x >> 6)) * PREP_CPW + ((threadIdx.x & 63) / PREP_LPC);
  const int lane = threadIdx.x & (PREP_LPC - 1);  // lane within the CU's group
  if (b >= f.nblocks) return;
  const int cstride = f.W >> 2;
  const thor_block_t &B = f.blk[b];
  int S = B.size;
  int mode = B.mode;
  // Band-local loop filters (row sharding, pb1 > 0): the cells of luma rows
  // [pb0 - 8, pb1 + 8) are all anyone here reads -- the band's deblocking with
  // its 8-row halo groups, its CLPF, its k_recon units -- so CUs wholly outside
  // them write nothing (each rank preps ~1/N of the frame, not all of it).
  if (f.pb1 > 0 && (B.ypos + S <= f.pb0 - 8 || B.ypos >= f.pb1 + 8)) return;
  int bw = B.bwidth >> 2, bh = B.bheight >> 2;
  int pb = mode == M_INTER ? B.pb_part : 0;
  int tb = B.tb_split > 0;
  int lsz = ilog2i(S);
  int lqv = lsz - (((tb || pb == 2 || pb == 3) && S > 8) ? 1 : 0);  // PART_VER / PART_QUAD, :90
  int lqh = lsz - (((tb || pb == 1 || pb == 3) && S > 8) ? 1 : 0);  // PART_HOR / PART_QUAD, :183
  uint16_t base = (uint16_t)((mode & 7) | ((B.cbp_y != 0) << 3) | ((B.cbp_u != 0) << 4) | ((B.cbp_v != 0) << 5) |
                             (lqv << 8) | (lqh << 11) | ((lsz - 3) << 14));
  // the MC words k_recon reads (dec/decode_block.c:213-451): bi-pred for BIPRED
  // and bi-directional SKIP / MERGE; `sign` = reference after the current frame
  // (uni-pred: >, each bi-pred leg: >=, :259-260, :291, :328-329, :358, :377,
  // :416-417); reference slot by frame number
  const bool bi = mode == M_BIPRED || ((mode == M_SKIP || mode == M_MERGE) && B.dir == 2);
  // the temporal-interpolated reference (-2) carries the current frame's
  // number (dec/decode_frame.c:108) and lives in its own slot
  const int ref0 = B.ref0 == -2 ? f.frame_num : B.ref0, ref1 = B.ref1 == -2 ? f.frame_num : B.ref1;
  const int sg0 = bi ? (ref0 >= f.frame_num) : (ref0 > f.frame_num);
  const int sg1 = ref1 >= f.frame_num;
  const int8_t *lut = (const int8_t *)f.slot_lut;
  const int s0 = B.ref0 == -2 ? f.islot : lut[ref0 & 127];
  const int s1 = bi ? (B.ref1 == -2 ? f.islot : lut[ref1 & 127]) : 0;
  // an inter CU naming a reference that is not resident: flag it (ctl[2] ->
  // THOR_ERR_REF from thor_dec_sync / thor_dec_read_frame) instead of leaving
  // stale slot pixels behind silently
  if (lane == 0 && mode != M_INTRA && (s0 < 0 || (bi && s1 < 0))) atomicOr(&f.ctl[2], 1u);
  const unsigned resbits = mode == M_SKIP ? 0u : ((unsigned)(B.coeff_mask & 7) << 18);
  const bool quarters = mode == M_INTER || mode == M_BIPRED;  // four size/2 quarters with mv_arr[i], :381-392
  // Per-cell MC words are read only by k_recon's per-cell path.  With a slow
  // list that path runs only for the listed (multi-key) halves, masking every
  // other half's cells, so the words are written only for CUs that can lie in
  // one: inter CUs under 64x64 (they make their half multi-key), 64x64 INTER /
  // BIPRED CUs with differing quarters, and -- when the frame lists any unit --
  // intra CUs under 64x64 (inactive words for a multi-key half's intra cells).
  // A planned 64x64 CU's or an intra SB's words are never read: 4K P frames
  // wrote 8 B per 4x4 cell (33 MB per 8-frame launch) for nothing.  Without a
  // list every unit that is not planned on both halves takes the per-cell path,
  // so every CU writes them.
  bool need_mc = !f.slow;
  if (!need_mc) {
    if (S < 64) need_mc = mode != M_INTRA || f.nslow > 0;
    else if (quarters)
      need_mc = B.mv0[0] != B.mv0[2] || B.mv0[1] != B.mv0[3] || B.mv0[4] != B.mv0[6] || B.mv0[5] != B.mv0[7] ||
                (mode == M_BIPRED && (B.mv1[0] != B.mv1[2] || B.mv1[1] != B.mv1[3] || B.mv1[4] != B.mv1[6] ||
                                      B.mv1[5] != B.mv1[7]));
  }
  int div = S >> 3;
  int y4 = B.ypos >> 2, x4 = B.xpos >> 2;
  for (int c = lane; c < bw * bh; c += PREP_LPC) {
    int m = c / bw, n = c - m * bw;
    int q = 2 * (m / div) + (n / div);
    int a0 = B.mv0[2 * q], a1 = B.mv0[2 * q + 1], a2 = B.mv1[2 * q], a3 = B.mv1[2 * q + 1];
    int big = (abs(a0) >= 4) | (abs(a1) >= 4) | (abs(a2) >= 4) | (abs(a3) >= 4);
    int idx = (y4 + m) * cstride + x4 + n;
    f.cellinfo[idx] = base | (uint16_t)(big << 6);
    if (!need_mc) continue;
    // MC word (the SKIP rectangle is already clipped to the frame: bwidth / bheight)
    const int qq = quarters ? q : 0;
    int m0x = B.mv0[2 * qq], m0y = B.mv0[2 * qq + 1], m1x = B.mv1[2 * qq], m1y = B.mv1[2 * qq + 1];
    if (sg0) { m0x = -m0x; m0y = -m0y; }
    if (sg1) { m1x = -m1x; m1y = -m1y; }
    const bool act = mode != M_INTRA && s0 >= 0 && (!bi || s1 >= 0);
    const unsigned meta =
        act ? ((unsigned)s0 | ((unsigned)(bi ? s1 : 0) << 8) | CELL_ACT | (bi ? CELL_BI : 0u) | resbits) : 0u;
    f.cellmc[idx] = make_uint2((uint32_t)((m0x & 0xffff) | (m0y << 16)), meta);
    if (act && bi) f.cellmv1[idx] = (m1x & 0xffff) | (m1y << 16);
  }
  // Half-SB plans (FrameCtx::hplan): lane h of a 64x64 inter CU whose half h
  // has rows inside the frame writes half h's record when quarters 2h and 2h+1 share their MVs
  // (always so for SKIP / MERGE, which use mv_arr[0]; INTER / BIPRED halves of
  // a horizontal split too).
  // Every other half with inter work (smaller inter CUs, or a 64x64 INTER / BIPRED
  // half whose two quarters differ) is multi-key: with a slow list its record is
  // tagged so (slow_mark), the list's workgroups reconstruct its units first.
  if (f.hplan && f.slow && S < 64 && lane == 0 && mode != M_INTRA)
    slow_mark(f, B.xpos >> 6, B.ypos >> 6, (B.ypos & 63) >= 32);
  if (f.hplan && S == 64 && lane < 2 && mode != M_INTRA) {
    const int h = lane, q0 = quarters ? 2 * h : 0, q1 = quarters ? 2 * h + 1 : 0;
    const bool same = B.mv0[2 * q0] == B.mv0[2 * q1] && B.mv0[2 * q0 + 1] == B.mv0[2 * q1 + 1] &&
                      (!bi || (B.mv1[2 * q0] == B.mv1[2 * q1] && B.mv1[2 * q0 + 1] == B.mv1[2 * q1 + 1]));
    const bool inside = B.ypos + 32 * h < f.H;  // rows / columns past the frame edge are not stored (k_recon)
    if (!same && inside && f.slow) slow_mark(f, B.xpos >> 6, B.ypos >> 6, h);
    if (same && inside && s0 >= 0 && (!bi || s1 >= 0)) {
      int m0x = B.mv0[2 * q0], m0y = B.mv0[2 * q0 + 1], m1x = B.mv1[2 * q0], m1y = B.mv1[2 * q0 + 1];
      if (sg0) { m0x = -m0x; m0y = -m0y; }
      if (sg1) { m1x = -m1x; m1y = -m1y; }
      const unsigned meta = (unsigned)s0 | ((unsigned)(bi ? s1 : 0) << 8) | CELL_ACT | (bi ? CELL_BI : 0u) | resbits;
      const int sbw = (f.W + 63) >> 6;
      const int hsb = 2 * ((B.ypos >> 6) * sbw + (B.xpos >> 6)) + h;
      f.hplan[hsb] = make_uint4((uint32_t)((m0x & 0xffff) | (m0y << 16)), meta,
                                bi ? (uint32_t)((m1x & 0xffff) | (m1y << 16)) : 0u, (unsigned)f.gen);
    }
  }
}

// ---------------------------------------------------------------------------
// Motion compensation helpers (get_inter_prediction_luma/chroma,
// common/inter_prediction.c:72-180).  Reads are dword-aligned and realigned
// with v_alignbyte; the padded ring guarantees every tap is addressable.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void load_bytes12(const uint8_t *p, uint32_t &e0, uint32_t &e1, uint32_t &e2) {
  uintptr_t a = (uintptr_t)p;
  const uint32_t *w = (const uint32_t *)(a & ~(uintptr_t)3);
  uint32_t sh = (uint32_t)(a & 3);
  uint32_t d0 = w[0], d1 = w[1], d2 = w[2], d3 = w[3];
  e0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
  e1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
  e2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
}
__device__ __forceinline__ void load_bytes8(const uint8_t *p, uint32_t &e0, uint32_t &e1) {
  uintptr_t a = (uintptr_t)p;
  const uint32_t *w = (const uint32_t *)(a & ~(uintptr_t)3);
  uint32_t sh = (uint32_t)(a & 3);
  uint32_t d0 = w[0], d1 = w[1], d2 = w[2];
  e0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
  e1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
}
__device__ __forceinline__ int byte_of(uint32_t w, int i) { return (w >> (8 * i)) & 255; }

// Pack an already-clipped byte into lane-byte j.  The empty asm keeps hipcc
// (ROCm 7.2, gfx950) from fusing pairs of clip255(x >> n) into
// v_ashr_pk_u8_i32, which leaves the upper half of its destination register
// unchanged while the compiler assumes it zero: byte 2 came out corrupted
// (found by tests/test_gpu_kernels.py).
__device__ __forceinline__ uint32_t put_byte(int v, int j) {
  asm volatile("" : "+v"(v));
  return (uint32_t)v << (8 * j);
}

// Keep every MC tap inside the padded slot.  Conformant streams stay within
// +-80 px of the frame (the encoder clamps, enc/encode_block.c:816-828), so
// these clamps never bind for them; they only make malformed input safe.
__device__ __forceinline__ int ry_clamp(int v, int H) { return v < -(THOR_PAD_Y - 8) ? -(THOR_PAD_Y - 8) : (v > H + THOR_PAD_Y - 12 ? H + THOR_PAD_Y - 12 : v); }
__device__ __forceinline__ int rx_clamp(int v, int W) { return v < -(THOR_PAD_Y - 8) ? -(THOR_PAD_Y - 8) : (v > W + THOR_PAD_Y - 16 ? W + THOR_PAD_Y - 16 : v); }
__device__ __forceinline__ int ry_clamp_c(int v, int H) { return v < -(THOR_PAD_C - 4) ? -(THOR_PAD_C - 4) : (v > H + THOR_PAD_C - 6 ? H + THOR_PAD_C - 6 : v); }
__device__ __forceinline__ int rx_clamp_c(int v, int W) { return v < -(THOR_PAD_C - 4) ? -(THOR_PAD_C - 4) : (v > W + THOR_PAD_C - 8 ? W + THOR_PAD_C - 8 : v); }

// 6-tap luma filters, common/inter_prediction.c:47-59
__device__ __forceinline__ void luma_taps(int frac, int bipred, int t[6]) {
  if (bipred) {
    if (frac == 1) { t[0] = 2; t[1] = -10; t[2] = 59; t[3] = 17; t[4] = -5; t[5] = 1; }
    else if (frac == 2) { t[0] = 1; t[1] = -8; t[2] = 39; t[3] = 39; t[4] = -8; t[5] = 1; }
    else if (frac == 3) { t[0] = 1; t[1] = -5; t[2] = 17; t[3] = 59; t[4] = -10; t[5] = 2; }
    else { t[0] = 0; t[1] = 0; t[2] = 64; t[3] = 0; t[4] = 0; t[5] = 0; }
  } else {
    if (frac == 1) { t[0] = 1; t[1] = -7; t[2] = 55; t[3] = 19; t[4] = -5; t[5] = 1; }
    else if (frac == 2) { t[0] = 1; t[1] = -7; t[2] = 38; t[3] = 38; t[4] = -7; t[5] = 1; }
    else if (frac == 3) { t[0] = 1; t[1] = -5; t[2] = 19; t[3] = 55; t[4] = -7; t[5] = 1; }
    else { t[0] = 0; t[1] = 0; t[2] = 64; t[3] = 0; t[4] = 0; t[5] = 0; }
  }
}
// 4-tap 1/8-pel chroma filters, common/inter_prediction.c:61-70
__device__ __forceinline__ void chroma_taps(int frac, int t[4]) {
  const int c[8][4] = {{0, 64, 0, 0},    {-2, 58, 10, -2}, {-4, 54, 16, -2}, {-4, 44, 28, -4},
                       {-4, 36, 36, -4}, {-4, 28, 44, -4}, {-2, 16, 54, -4}, {-2, 10, 58, -2}};
  t[0] = c[frac][0]; t[1] = c[frac][1]; t[2] = c[frac][2]; t[3] = c[frac][3];
}

// Four horizontally adjacent luma predictions starting at `src` (the
// MV-displaced position of the first pixel).  Returns 4 packed bytes.
__device__ uint32_t mc_luma4(const uint8_t *src, int stride, int fx, int fy, int bipred) {
  if (fx == 0 && fy == 0) {  // integer MV: copy (inter_prediction.c:133-140)
    uint32_t e0, e1;
    load_bytes8(src, e0, e1);
    return e0;
  }
  if (fx == 2 && fy == 2) {  // (2,2) 4x4 low-pass (inter_prediction.c:145-157)
    int r[4][7];
    for (int a = 0; a < 4; a++) {
      uint32_t e0, e1;
      load_bytes8(src + (a - 1) * stride - 1, e0, e1);
      for (int i = 0; i < 4; i++) r[a][i] = byte_of(e0, i);
      for (int i = 0; i < 3; i++) r[a][4 + i] = byte_of(e1, i);
    }
    uint32_t out = 0;
    for (int j = 0; j < 4; j++) {
      int s = r[0][j + 1] + r[0][j + 2] + r[1][j] + 2 * r[1][j + 1] + 2 * r[1][j + 2] + r[1][j + 3] + r[2][j] +
              2 * r[2][j + 1] + 2 * r[2][j + 2] + r[2][j + 3] + r[3][j + 1] + r[3][j + 2];
      out |= put_byte(clip255((s + 8) >> 4), j);
    }
    return out;
  }
  int fv[6], fh[6];
  luma_taps(fy, bipred, fv);
  luma_taps(fx, bipred, fh);
  int v[9];
  for (int c = 0; c < 9; c++) v[c] = 0;
  // vertical 6-tap into int32 over columns -2..+6 (inter_prediction.c:160-168)
  for (int n = 0; n < 6; n++) {
    uint32_t e0, e1, e2;
    load_bytes12(src + (n - 2) * stride - 2, e0, e1, e2);
    int f = fv[n];
    for (int c = 0; c < 4; c++) v[c] += f * byte_of(e0, c);
    for (int c = 0; c < 4; c++) v[4 + c] += f * byte_of(e1, c);
    v[8] += f * byte_of(e2, 0);
  }
  uint32_t out = 0;
  for (int j = 0; j < 4; j++) {  // horizontal (inter_prediction.c:170-178)
    int s = fh[0] * v[j] + fh[1] * v[j + 1] + fh[2] * v[j + 2] + fh[3] * v[j + 3] + fh[4] * v[j + 4] + fh[5] * v[j + 5];
    out |= put_byte(clip255((s + 2048) >> 12), j);
  }
  return out;
}

// One chroma prediction at `src` (MV-displaced).  inter_prediction.c:86-117
__device__ int mc_chroma1(const uint8_t *src, int stride, int fx, int fy) {
  if (fx == 0 && fy == 0) return src[0];
  int th[4], tv[4];
  chroma_taps(fx, th);
  chroma_taps(fy, tv);
  int s = 0;
  for (int m = 0; m < 4; m++) {
    uint32_t e0, e1;
    load_bytes8(src + (m - 1) * stride - 1, e0, e1);
    int t = th[0] * byte_of(e0, 0) + th[1] * byte_of(e0, 1) + th[2] * byte_of(e0, 2) + th[3] * byte_of(e0, 3);
    s += tv[m] * t;
  }
  return clip255((s + 2048) >> 12);
}
