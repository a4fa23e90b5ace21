// Device-resident Thor encoder, part 3: the RD loop of one superblock --
// encode_block, cost_calc, motion estimation, intra mode search, early skip,
// mode_decision_rdo and the quadtree process_block (enc/encode_block.c), and
// the per-SB entry encode_frame runs (enc/encode_frame.c:112-147).
#pragma once
#include "enc_pix.h"

// Per-wave working memory (global memory on the device; one per SB-row worker).
#define TE_BLK (64 * 64 * 3 / 2)
#define TE_BEST_WORDS 1024
struct TeLevel {             // one quadtree level (64, 32, 16, 8)
  uint8_t rbuf[2][TE_BLK];   // rec_block / rec_block_best (roles swap, see te_copy_best)
  int16_t cbuf[3][3 * TE_COEF_COMP];  // coefficient sets: best, tmp, spare
  uint32_t bbits[TE_BEST_WORDS];      // the best candidate's syntax bits (TeBlockInfo::best_bits)
};
// The 32 / 16 / 8 levels' reconstruction buffers and the 16 / 8 levels'
// coefficient sets and kept syntax bits (80 of an SB's 85 CUs): global
// memory (TeScratchMem::sl), L2-resident -- in LDS they would hold
// k_enc_rows to one worker per SIMD.  Capacity of the
// kept bits: overflow falls back to running write_block again
// (te_keep_best_bits).
struct TeSmallLv {
  uint8_t rec1[2][32 * 32 * 3 / 2], rec2[2][16 * 16 * 3 / 2], rec3[2][8 * 8 * 3 / 2];
  int16_t cf2[2][3 * 256], cf3[2][3 * 64];
  uint32_t bb2[128], bb3[64];
};
struct TeScratchMem {         // global memory, one per worker wave
  TeLevel lv[4];
  TeSmallLv sl;
  TeBlockInfo bi[4];                 // (host build: the per-level block state; LDS on the device)
  TeParam tmp;                       // (host build: the candidate parameters; LDS on the device)
  uint8_t pb0[TE_BLK], pb1[TE_BLK];  // bi-pred legs (Y | U | V, compact)
  uint8_t org8[64 * 64];             // bi-pred search target (search_bipred_prediction_params)
  uint8_t rf[64 * 64];               // exact sub-pel ME prediction
  TeTx tx;                           // (host build: the LDS-resident buffers live here)
  TeNbr nb;
  uint8_t pb[TE_BLK];
};
// The worker's buffers, passed by value: on the device the hot ones (the
// transform chain, intra neighbours, the current prediction) point into LDS.
struct TeScratch {
  TeLevel *lv;
  uint8_t *pb, *pb0, *pb1, *org8, *rf;
  TeTx *tx;
  TeNbr *nb;
  TeBlockInfo *bi;  // [4], one per quadtree level (the recursion's block_info)
  TeParam *tmp;     // the candidate of mode_decision / search_early_skip (never live at once)
  TeSmallLv *sl;
};
TE_FN TeScratch te_scratch(TeScratchMem &M, TeTx *tx, TeNbr *nb, uint8_t *pb, TeBlockInfo *bi, TeParam *tmp,
                           TeSmallLv *sl) {
  TeScratch S;
  S.lv = M.lv;
  S.pb = pb;
  S.pb0 = M.pb0;
  S.pb1 = M.pb1;
  S.org8 = M.org8;
  S.rf = M.rf;
  S.tx = tx;
  S.nb = nb;
  S.bi = bi;
  S.tmp = tmp;
  S.sl = sl;
  return S;
}
// a callee's view of the scratch: the LDS members re-declared as LDS
TE_FN TeScratch te_local(TeScratch S) {
  S.pb = te_lds(S.pb);
  S.tx = te_lds(S.tx);
  S.nb = te_lds(S.nb);
  S.bi = te_lds(S.bi);
  S.tmp = te_lds(S.tmp);
  S.sl = te_glb(S.sl);  // global: the LDS budget of two workers per SIMD (k_enc_rows)
  return S;
}
// The worker's buffer table, rebuilt where it is needed instead of passed
// down the call tree (a table passed by value was copied to the scratch stack
// at every call, one through LDS had to be held in registers): on the device
// the LDS members sit at fixed addresses and the global ones at fixed offsets
// from the worker's TeScratchMem, whose address k_enc_rows leaves in LDS.
#if defined(TE_HOST)
static TeScratch g_te_scratch;  // the harness's buffers
static inline void te_set_scratch(const TeScratch &S) { g_te_scratch = S; }
static inline TeScratch te_here() { return g_te_scratch; }
#else
__shared__ TeTx g_te_tx;
__shared__ TeNbr g_te_nb;
__shared__ TeBlockInfo g_te_bi[4];
__shared__ TeParam g_te_tmp;
__shared__ TeScratchMem *g_te_mem;
__shared__ uint8_t g_te_pb[TE_BLK];
__device__ __forceinline__ TeScratch te_here() {
  TeScratchMem &M = *g_te_mem;
  return te_local(te_scratch(M, &g_te_tx, &g_te_nb, g_te_pb, g_te_bi, &g_te_tmp, &M.sl));
}
#endif
// State of the superblock being encoded (frame_info mvcand / best_ref are
// reset per SB, enc/encode_frame.c:117-121) and its bit stream.
struct TeSB {
  TeBits bits;
  TeMvCand mc;
  int best_ref;
};

TE_FN uint8_t *te_pu(uint8_t *b, int size) { return b + size * size; }
TE_FN uint8_t *te_pv(uint8_t *b, int size) { return b + size * size + (size / 2) * (size / 2); }

TE_FN void te_copy_bytes(uint8_t *d, const uint8_t *s, int n) {
  if ((n & 3) == 0)
    for (int e = 4 * TE_LANE; e < n; e += 4 * TE_NL) te_st4(d + e, te_ld4(s + e));
  else
    for (int e = TE_LANE; e < n; e += TE_NL) d[e] = s[e];
  te_sync();
}
// d[y * ds + x] = (a[y * as + x] + b[y * bs + x]) >> 1 over a w x h block
TE_FN void te_avg_rect(uint8_t *d, int ds, const uint8_t *a, int as, const uint8_t *b, int bs, int w, int h) {
  if ((w & 3) == 0) {
    const int w4 = w >> 2, n4 = w4 * h;
    for (int g = TE_LANE; g < n4; g += TE_NL) {
      const int i = te_dv(g, w4), j = (g - i * w4) * 4;
      te_st4(d + i * ds + j, te_avg4(te_ld4(a + i * as + j), te_ld4(b + i * bs + j)));
    }
  } else {
    for (int e = TE_LANE; e < w * h; e += TE_NL) {
      const int i = te_dv(e, w), j = e - te_dv(e, w) * w;
      d[i * ds + j] = (uint8_t)(((int)a[i * as + j] + (int)b[i * bs + j]) >> 1);
    }
  }
}
// d[y * ds + x] = s[y * ss + x] over a w x h block
TE_FN void te_copy_rect(uint8_t *d, int ds, const uint8_t *s, int ss, int w, int h) {
  if ((w & 3) == 0) {
    const int w4 = w >> 2, n4 = w4 * h;
    for (int g = TE_LANE; g < n4; g += TE_NL) {
      const int i = te_dv(g, w4), j = (g - i * w4) * 4;
      te_st4(d + i * ds + j, te_ld4(s + i * ss + j));
    }
  } else {
    for (int e = TE_LANE; e < w * h; e += TE_NL) {
      const int i = te_dv(e, w), j = e - te_dv(e, w) * w;
      d[i * ds + j] = s[i * ss + j];
    }
  }
}
// four int16 at an 8-byte aligned address
TE_FN void te_st4x16(int16_t *p, int a, int b, int c, int d) {
  const uint32_t lo = ((uint32_t)a & 0xffffu) | (uint32_t)b << 16, hi = ((uint32_t)c & 0xffffu) | (uint32_t)d << 16;
#if !defined(TE_HOST)
  *(uint2 *)p = make_uint2(lo, hi);
#else
  memcpy(p, &lo, 4);
  memcpy(p + 2, &hi, 4);
#endif
}
// R[y * n + x] = o[y * os + x] - p[y * ps + x] (n x n, int16)
TE_FN void te_residual(int16_t *R, const uint8_t *o, int os, const uint8_t *p, int ps, int n) {
  if ((n & 3) == 0) {
    const int w4 = n >> 2, n4 = w4 * n;
    for (int g = TE_LANE; g < n4; g += TE_NL) {
      const int i = te_dv(g, w4), j = (g - i * w4) * 4;
      const uint32_t a = te_ld4(o + i * os + j), b = te_ld4(p + i * ps + j);
      te_st4x16(R + i * n + j, te_b(a, 0) - te_b(b, 0), te_b(a, 1) - te_b(b, 1), te_b(a, 2) - te_b(b, 2),
                te_b(a, 3) - te_b(b, 3));
    }
  } else {
    for (int e = TE_LANE; e < n * n; e += TE_NL) {
      const int y = te_dv(e, n), x = e - te_dv(e, n) * n;
      R[e] = (int16_t)((int)o[y * os + x] - (int)p[y * ps + x]);
    }
  }
  te_sync();
}

// A 64 x 64 residual straight into the pre-summed input of its transform
// (te_fwd_tx's 64 path, common/transform.c:273-307): X.A = f x f sums of
// o - p, f = 4 (fast: 16 x 16) or 2 (32 x 32), int16 wrap.  The sums are
// exact, so this equals summing a materialised residual; X.R then only ever
// holds up to 32 x 32.
TE_FN void te_residual64(TeTx &X, const uint8_t *o, int os, const uint8_t *p, int ps, int fast) {
  if (fast) {
    for (int e = TE_LANE; e < 256; e += TE_NL) {
      const int i = e >> 4, j = (e & 15) * 4;
      int s = 0;
      for (int a = 0; a < 4; a++) {
        const uint32_t x = te_ld4(o + (4 * i + a) * os + j), y = te_ld4(p + (4 * i + a) * ps + j);
        s += te_b(x, 0) + te_b(x, 1) + te_b(x, 2) + te_b(x, 3) - te_b(y, 0) - te_b(y, 1) - te_b(y, 2) - te_b(y, 3);
      }
      X.A[e] = (int16_t)te_wrap16(s);
    }
  } else {
    for (int g = TE_LANE; g < 512; g += TE_NL) {  // two outputs per lane: 4 columns x 2 rows
      const int i = g >> 4, j = (g & 15) * 4;
      const uint32_t o0 = te_ld4(o + (2 * i) * os + j), o1 = te_ld4(o + (2 * i + 1) * os + j);
      const uint32_t p0 = te_ld4(p + (2 * i) * ps + j), p1 = te_ld4(p + (2 * i + 1) * ps + j);
      for (int k = 0; k < 2; k++) {
        const int s = te_b(o0, 2 * k) + te_b(o0, 2 * k + 1) + te_b(o1, 2 * k) + te_b(o1, 2 * k + 1) - te_b(p0, 2 * k) -
                      te_b(p0, 2 * k + 1) - te_b(p1, 2 * k) - te_b(p1, 2 * k + 1);
        X.A[i * 32 + (j >> 1) + k] = (int16_t)te_wrap16(s);
      }
    }
  }
  te_sync();
}
// the residual of an N x N transform block into its transform's input
TE_FN void te_residual_tx(TeTx &X, const uint8_t *o, int os, const uint8_t *p, int ps, int n, int fast) {
  if (n == 64) te_residual64(X, o, os, p, ps, fast);
  else te_residual(X.R, o, os, p, ps, n);
}

// clip_mv, enc/encode_block.c:816-828 (C division by 4; the right-edge test
// omits `size`, the clamp includes it, as there)
TE_FN TeMv te_clip_mv(TeMv m, int ypos, int xpos, int fw, int fh, int size, int sign) {
  const int ext = 96 - 16;
  int mvy = sign ? -m.y : m.y, mvx = sign ? -m.x : m.x;
  if (ypos + mvy / 4 < -ext) mvy = 4 * (-ext - ypos);
  if (ypos + mvy / 4 + size > fh + ext) mvy = 4 * (fh + ext - ypos - size);
  if (xpos + mvx / 4 < -ext) mvx = 4 * (-ext - xpos);
  if (xpos + mvx / 4 > fw + ext) mvx = 4 * (fw + ext - xpos - size);
  TeMv r;
  r.y = (int16_t)(sign ? -mvy : mvy);
  r.x = (int16_t)(sign ? -mvx : mvx);
  return r;
}

// get_inter_prediction_yuv, enc/encode_block.c:1534-1567: `split` predicts the
// four size/2 quarters with mv[0..3].  Writes a compact Y|U|V block (stride size).
TE_FN void te_pred_yuv(const TeFrame &F, int r, uint8_t *pb, const TeBlockInfo &bi, const TeMv *mv, int sign, int bipred,
                       int split) {
  const int div = split + 1, bw = bi.bwidth / div, bh = bi.bheight / div, size = bi.size;
  const int ypos = bi.ypos, xpos = bi.xpos;
#if defined(THOR_ENC_TRACE) && !defined(TE_HOST)
  if (size == 8 && split) {
    const uint64_t ex = __builtin_amdgcn_read_exec();
    TE_TR(F.frame_num, 13, ypos, xpos, (uint32_t)ex, (uint32_t)(ex >> 32), r, 0);
  }
#endif
  for (int index = 0; index < div * div; index++) {
    const int idx = index & 1, idy = (index >> 1) & 1;
    const TeMv m = te_clip_mv(mv[index], ypos, xpos, F.W, F.H, size, sign);
    te_mc_luma(pb + idy * bh * size + idx * bw, size, F.refy[r] + (ypos + idy * bh) * F.rsy + xpos + idx * bw, F.rsy, bw, bh,
               m, sign, bipred);
#if defined(THOR_ENC_TRACE)
    if (size == 8 && split)
      TE_TR(F.frame_num, 12, ypos, xpos, r | index << 4 | sign << 8 | bipred << 9 | bw << 12 | bh << 20,
            (m.x & 0xffff) | (int)m.y << 16, (mv[index].x & 0xffff) | (int)mv[index].y << 16,
            te_ld4(pb + idy * bh * size + idx * bw));
#endif
    const int oc = idy * (bh / 2) * (size / 2) + idx * (bw / 2);
    const int orc = (ypos / 2 + idy * (bh / 2)) * F.rsc + xpos / 2 + idx * (bw / 2);
    te_mc_chroma(te_pu(pb, size) + oc, size / 2, F.refu[r] + orc, F.rsc, bw / 2, bh / 2, m, sign);
    te_mc_chroma(te_pv(pb, size) + oc, size / 2, F.refv[r] + orc, F.rsc, bw / 2, bh / 2, m, sign);
  }
}
// average_blocks_all, enc/encode_block.c:1569-1588: truncating (p0 + p1) >> 1
// over bwidth x bheight (chroma halves)
TE_FN void te_avg_yuv(uint8_t *d, const uint8_t *a, const uint8_t *b, const TeBlockInfo &bi) {
  const int size = bi.size, bw = bi.bwidth, bh = bi.bheight;
  te_avg_rect(d, size, a, size, b, size, bw, bh);
  const int cw = bw / 2, ch = bh / 2, cs = size / 2, co = size * size, cq = cs * cs;
  te_avg_rect(d + co, cs, a + co, cs, b + co, cs, cw, ch);
  te_avg_rect(d + co + cq, cs, a + co + cq, cs, b + co + cq, cs, cw, ch);
  te_sync();
}

TE_FN int te_sign_of(const TeFrame &F, int ref_idx, int bi) {
  // uni-pred: ref->frame_num > rec->frame_num; bi-pred legs: >= (encode_block.c:1694, :1707)
  return bi ? F.ref_fnum[ref_idx] >= F.frame_num : F.ref_fnum[ref_idx] > F.frame_num;
}

// rec[y * rs + x] = bit ? clip255(residual(y, x) + pb[y * ps + x]) : pb[..] (n x n)
TE_FN void te_recon(uint8_t *rec, int rs, const uint8_t *pb, int ps, const TeTx &X, int n, int bit) {
  if ((n & 3) == 0) {
    const int w4 = n >> 2, n4 = w4 * n;
    for (int g = TE_LANE; g < n4; g += TE_NL) {
      const int i = te_dv(g, w4), j = (g - i * w4) * 4;
      uint32_t v = te_ld4(pb + i * ps + j);
      if (bit)
        v = te_pack4(te_clip255(te_res_at(X, n, i, j) + te_b(v, 0)), te_clip255(te_res_at(X, n, i, j + 1) + te_b(v, 1)),
                     te_clip255(te_res_at(X, n, i, j + 2) + te_b(v, 2)), te_clip255(te_res_at(X, n, i, j + 3) + te_b(v, 3)));
      te_st4(rec + i * rs + j, v);
    }
  } else {
    for (int e = TE_LANE; e < n * n; e += TE_NL) {
      const int y = te_dv(e, n), x = e - te_dv(e, n) * n;
      const int p = pb[y * ps + x];
      rec[y * rs + x] = (uint8_t)(bit ? te_clip255(te_res_at(X, n, y, x) + p) : p);
    }
  }
  te_sync();
}

// ---- transform-block chains -------------------------------------------------
// encode_and_reconstruct_block_inter, enc/encode_block.c:1469-1532, one
// component: orig (frame, stride os) - pred -> levels (tiles of `coef`) ->
// rec (compact, stride size).  Returns cbp (4-bit mask when tb-split).
TE_NOINL int te_enc_inter_comp(const TeFrame &F_, const uint8_t *org, int os, int size, int qp,
                               const uint8_t *pb_, int16_t *coef, uint8_t *rec, int type, int tb_split, int ts) {
  const TeFrame &F = *te_lds(&F_);
  const TeScratch S = te_here();
  const uint8_t *pb = te_lds(pb_);
  TE_P(TP_INTER_COMP);
  TeTx &X = *S.tx;
  int cbp = 0;
  if (tb_split) {
    const int s2 = size / 2, fast = size == 64 || F.speed > 1;
    // rblock: the reconstructed residual of every quarter, kept in rec as a
    // running copy of pred + residual (reconstruct_block after the loop, :1510)
    for (int t = 0; t < 4; t++) {
      const int i = (t >> 1) * s2, j = (t & 1) * s2;
      te_residual_tx(X, org + i * os + j, os, pb + i * size + j, size, s2, fast);
      te_fwd_tx(X, s2, fast);
      const int bit = te_quant_chain(X, qp, s2, type, coef + t * ts);
      if (bit) te_inv_tx(X, s2);
      te_recon(rec + i * size + j, size, pb + i * size + j, size, X, s2, bit);
      cbp = (cbp << 1) + bit;
    }
    return cbp;
  }
  const int fast = (size == 64 && F.speed > 0) || F.speed > 1;
  te_residual_tx(X, org, os, pb, size, size, fast);
  te_fwd_tx(X, size, fast);
  cbp = te_quant_chain(X, qp, size, type, coef);
  if (cbp) te_inv_tx(X, size);
  te_recon(rec, size, pb, size, X, size, cbp);
  return cbp;
}

#if !defined(TE_HOST)
// The search's predictions without a prediction buffer: pixel (i, j) of
// `mode` straight from the neighbour arrays (the same formulas as
// te_intra_pred, enc_pix.h).  lF / tF hold the 2n-long 1-2-1 filtered edges
// (what the up-right and down-left-left modes read); the n-long filter of the
// up-left modes differs from them only at index n - 1 (lFe / tFe).  T / L:
// the planar edge sums.
struct TeIpc {
  int dc, TL, tlF, tFe, lFe;
};
TE_FN int te_ipx(const TeNbr &nb, const TeIpc &c, int n, int mode, int i, int j) {
  switch (mode) {
    case TE_PLANAR:
      return te_clip255((nb.L[i] + nb.T[j] - c.TL + 4) / 8);
    case TE_HOR:
      return nb.left[i];
    case TE_VER:
      return nb.top[j];
    case TE_UPLEFT: {
      const int d = i - j;
      if (d > 0) return d - 1 == n - 1 ? c.lFe : nb.lF[d - 1];
      return d == 0 ? c.tlF : (-d - 1 == n - 1 ? c.tFe : nb.tF[-d - 1]);
    }
    case TE_UPUPLEFT: {
      const int d = i - 2 * j;
      if (d > 1) return d - 2 == n - 1 ? c.lFe : nb.lF[d - 2];
      if (d == 1) return c.tlF;
      const int t0 = nb.tF[0];
      if (d == 0) return (c.tlF + t0) >> 1;
      const int h = (-d) / 2, th = h == n - 1 ? c.tFe : nb.tF[h];
      if (d & 1) return th;
      return (th + (h - 1 == n - 1 ? c.tFe : nb.tF[h - 1])) >> 1;
    }
    case TE_UPLEFTLEFT: {
      const int d = 2 * i - j;
      if (d < -1) return -d - 2 == n - 1 ? c.tFe : nb.tF[-d - 2];
      if (d == -1) return c.tlF;
      const int l0 = nb.lF[0];
      if (d == 0) return (c.tlF + l0) >> 1;
      const int h = d / 2, lh = h == n - 1 ? c.lFe : nb.lF[h];
      if (d & 1) return lh;
      return (lh + (h - 1 == n - 1 ? c.lFe : nb.lF[h - 1])) >> 1;
    }
    case TE_UPRIGHT:
      return nb.tF[i + j + 1];
    case TE_UPUPRIGHT: {
      const int d = i + 2 * j;
      return (d & 1) ? (int)nb.tF[(d + 1) / 2] : (nb.tF[d / 2] + nb.tF[d / 2 + 1]) >> 1;
    }
    case TE_DOWNLEFTLEFT: {
      const int d = 2 * i + j;
      return (d & 1) ? (int)nb.lF[(d + 1) / 2] : (nb.lF[d / 2] + nb.lF[d / 2 + 1]) >> 1;
    }
    default:  // DC (the search's: (left, top) always)
      return c.dc;
  }
}
TE_FN uint32_t te_ipx4(const TeNbr &nb, const TeIpc &c, int n, int mode, int i, int j) {
  return te_pack4(te_ipx(nb, c, n, mode, i, j), te_ipx(nb, c, n, mode, i, j + 1), te_ipx(nb, c, n, mode, i, j + 2),
                  te_ipx(nb, c, n, mode, i, j + 3));
}
// the arrays and constants te_ipx reads, for the n x n block whose edges are in nb
TE_FN TeIpc te_ipx_consts(const TeNbr &nb, int n) {  // (reads only)
  uint32_t sum = 0;
  for (int k = TE_LANE; k < n; k += TE_NL) sum += nb.left[k] + nb.top[k];
  sum = te_sum(sum);
  TeIpc c;
  c.dc = ((int)sum + n) / (2 * n);
  c.TL = nb.left[1] + 2 * nb.left[0] + 2 * nb.tl + 2 * nb.top[0] + nb.top[1];
  c.tlF = (2 * nb.tl + nb.left[0] + nb.top[0] + 2) >> 2;
  c.tFe = (nb.top[n - 2] + 3 * nb.top[n - 1] + 2) >> 2;
  c.lFe = (nb.left[n - 2] + 3 * nb.left[n - 1] + 2) >> 2;
  return c;
}
TE_FN TeIpc te_ipx_setup(TeNbr &nb, int n) {
  for (int k = TE_LANE; k < 2 * n; k += TE_NL) {
    // 1-2-1 filters of both edges over 2n (filter_121, common/intra_prediction.c:39-48)
    const int e = k == 2 * n - 1;
    nb.tF[k] = (uint8_t)(k == 0 ? (3 * nb.top[0] + nb.top[1] + 2) >> 2
                                : (e ? (nb.top[k - 1] + 3 * nb.top[k] + 2) >> 2
                                     : (nb.top[k - 1] + 2 * nb.top[k] + nb.top[k + 1] + 2) >> 2));
    nb.lF[k] = (uint8_t)(k == 0 ? (3 * nb.left[0] + nb.left[1] + 2) >> 2
                                : (e ? (nb.left[k - 1] + 3 * nb.left[k] + 2) >> 2
                                     : (nb.left[k - 1] + 2 * nb.left[k] + nb.left[k + 1] + 2) >> 2));
    // planar edge sums (:182-214)
    const int s = k >= n, jj = k - s * n;
    const uint8_t *a = s ? nb.left : nb.top;
    int v;
    if (jj == 0) v = 3 * a[0] + 2 * a[0] + 2 * a[1] + a[2];
    else if (jj == 1) v = a[0] + 2 * a[0] + 2 * a[1] + 2 * a[2] + a[3];
    else if (jj == n - 2) v = a[n - 4] + 2 * a[n - 3] + 2 * a[n - 2] + 2 * a[n - 1] + a[n - 1];
    else if (jj == n - 1) v = a[n - 3] + 2 * a[n - 2] + 2 * a[n - 1] + 3 * a[n - 1];
    else v = a[jj - 2] + 2 * a[jj - 1] + 2 * a[jj] + 2 * a[jj + 1] + a[jj + 2];
    (s ? nb.L : nb.T)[jj] = v;
  }
  te_sync();
  return te_ipx_consts(nb, n);
}
#endif

#ifndef TE_C4
#if defined(TE_HOST)
#define TE_C4 0
#else
#define TE_C4 1
#endif
#endif
// encode_and_reconstruct_block_intra, enc/encode_block.c:1398-1467, one
// component.  rf / fs: the frame being reconstructed at the CU origin.
TE_FN int te_enc_intra_comp(const TeFrame &F_, const uint8_t *org, int os, const uint8_t *rf, int fs,
                               int ypos, int xpos, int size, int qp, uint8_t *pb_, int16_t *coef, uint8_t *rec, int type,
                               int tb_split, int mode, int ur, int dl, int ts) {
  const TeFrame &F = *te_lds(&F_);
  const TeScratch S = te_here();
  uint8_t *pb = te_lds(pb_);
  TE_P(TP_INTRA_COMP);
  TeTx &X = *S.tx;
  const int fast = F.speed > 1;
  if (tb_split) {
    const int s2 = size / 2;
    int cbp = 0;
    for (int t = 0; t < 4; t++) {
      const int i = (t >> 1) * s2, j = (t & 1) * s2;
      te_make_top_and_left(*S.nb, rf, fs, rec + i * size + j, size, i, j, ypos, xpos, s2, ur, dl, 1);
      te_intra_pred(*S.nb, ypos + i, xpos + j, s2, pb, mode, 0);
      te_residual_tx(X, org + i * os + j, os, pb, s2, s2, fast);
      te_fwd_tx(X, s2, fast);
      const int bit = te_quant_chain(X, qp, s2, type, coef + t * ts);
      if (bit) te_inv_tx(X, s2);
      te_recon(rec + i * size + j, size, pb, s2, X, s2, bit);
      cbp = (cbp << 1) + bit;
    }
    return cbp;
  }
  te_make_top_and_left(*S.nb, rf, fs, nullptr, 0, 0, 0, ypos, xpos, size, ur, dl, 0);
  te_intra_pred(*S.nb, ypos, xpos, size, pb, mode, 0);
  te_residual_tx(X, org, os, pb, size, size, fast);
  te_fwd_tx(X, size, fast);
  const int cbp = te_quant_chain(X, qp, size, type, coef);
  if (cbp) te_inv_tx(X, size);
  te_recon(rec, size, pb, size, X, size, cbp);
  return cbp;
}

#if !defined(TE_HOST)
// te_enc_intra_comp for a 4 x 4 block (the chroma of an 8 x 8 CU: 2 of the 3
// chains of the commonest CU) with every step in registers: lane r < 16 holds
// pixel / coefficient r (raster) of the block; the transforms' row and column
// passes gather their four inputs with ds_bpermute (no LDS round trip, no
// barrier); quantize's last position and the RDOQ-light masks are wave
// reductions, its candidate loop scalar.  The same arithmetic as the generic
// chain: te_fwd_gen<4>, te_quant_t, te_inv_gen<4>, te_recon (enc_pix.h).
TE_FN int te_d4(uint32_t w, int k) { return __builtin_amdgcn_sbfe((int)w, 8 * k, 8); }
TE_FN uint32_t te_or16(uint32_t v) {  // OR over lanes 0..15 (lanes >= 16 contribute 0), uniform
  v |= (uint32_t)TE_DPP(v, 0xB1);
  v |= (uint32_t)TE_DPP(v, 0x4E);
  v |= (uint32_t)TE_DPP(v, 0x141);
  v |= (uint32_t)TE_DPP(v, 0x140);
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
}
// residual -> levels (into coef) -> reconstruction (into rec, stride 4) of the
// 4 x 4 block whose prediction lane r < 16 holds in p; returns cbp
TE_FN int te_c4_code(int p, const uint8_t *org, int os, int qp, int16_t *coef, uint8_t *rec, int type) {
  const int lane = TE_LANE, r = lane & 15, i = r >> 2, j = r & 3, base = lane & ~15;
  const bool act = lane < 16;
  // HEVC 4-point basis rows (D[i][k]) and columns (D[k][j]) as packed int8
  const uint32_t rowD = i == 0 ? 0x40404040u : (i == 1 ? 0xADDC2453u : (i == 2 ? 0x40C0C040u : 0xDC53AD24u));
  const uint32_t colD = j == 0 ? 0x24405340u : (j == 1 ? 0xADC02440u : (j == 2 ? 0x53C0DC40u : 0xDC40AD40u));
  const int R = (int)org[i * os + j] - p;
  // transform (common/transform.c:309-327): T = D R^T, C = D T^T, 16-bit wraps; N = 4: shifts 2, 7
  int t = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) t += te_d4(rowD, k) * __shfl(R, base + 4 * j + k);
  t = te_wrap16((t + 2) >> 2);
  int C = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) C += te_d4(rowD, k) * __shfl(t, base + 4 * j + k);
  C = te_wrap16((C + 64) >> 7);
  // quantize (enc/encode_block.c:75-172, rdoq 0), q = 4
  const int intra = (type >> 1) & 1, chroma = type & 1;
  const int scale = te_gquant[qp % 6], shift2 = 21 - 2 + qp / 6;
  const int offset = (intra ? 38 : -26) * (1 << (shift2 - 8));
  const int pos = (int)((0xfea9db83c7426510ull >> (4 * r)) & 15);  // te_zz(4, r)
  const int lp = (act && (te_abs(te_abs(C) * scale + offset) >> shift2) != 0) ? pos : -1;
  const int last_pos = te_maxi(lp);
  const int off0 = (intra ? 102 : 51) * (1 << (shift2 - 8)), off1 = (intra ? 115 : 90) * (1 << (shift2 - 8));
  int lev = 0;
  if (act && pos <= last_pos) {
    const int ac = scale * te_abs(C);
    const int l0 = ac >> shift2;
    const int l = (ac + ((l0 == 0 || chroma) ? off0 : off1)) >> shift2;
    lev = C < 0 ? -l : l;
  }
  const int cbp = te_any(lev != 0);
  if (cbp) {  // RDOQ light (:134-168) on the scan-order masks, as te_quant_t
    const int n = chroma ? last_pos + 1 : 16;
    const int thr = (73 * te_gdequant[qp % 6] << (qp / 6)) >> (4 + 2);
    uint32_t big = te_or16(act && te_abs(lev) > 1 ? 1u << pos : 0u);
    uint32_t nzm = te_or16(act && lev != 0 ? 1u << pos : 0u);
    uint32_t chg = 0, neg = 0;
    uint32_t m = big & (n >= 16 ? 0xffffu : ((1u << n) - 1)) & ~3u;
    while (m) {
      const int q = __builtin_ctz(m);
      m &= m - 1;
      int flag = 1;
      if (q > 2 && ((big >> (q - 3)) & 1)) flag = 0;
      if (q > 3 && ((big >> (q - 4)) & 1) && ((nzm >> (q - 3)) & 1)) flag = 0;
      if (q == 2 && (chroma == 0 || last_pos >= 6)) flag = 0;
      if (flag && !((nzm >> (q - 2)) & 1) && !((nzm >> (q - 1)) & 1) && ((big >> q) & 1)) {
        // coefficients at scan positions q, q - 1, q - 2: their raster lanes (te_izz(4, .))
        const int c1 = __builtin_amdgcn_readlane(C, (int)((0xfeb7adc963258410ull >> (4 * q)) & 15));
        const int c2 = __builtin_amdgcn_readlane(C, (int)((0xfeb7adc963258410ull >> (4 * (q - 1))) & 15));
        const int c3 = __builtin_amdgcn_readlane(C, (int)((0xfeb7adc963258410ull >> (4 * (q - 2))) & 15));
        const int K1 = te_abs(c1), K2 = te_abs(c2), K3 = te_abs(c3), K4 = TE_MAX(K2, K3);
        int at, v;
        if (K1 + K4 < thr) {
          at = q;
          v = c1 < 0 ? -1 : 1;
        } else if (K2 > K3) {
          at = q - 1;
          v = c2 < 0 ? -1 : 1;
        } else {
          at = q - 2;
          v = c3 < 0 ? -1 : 1;
        }
        chg |= 1u << at;
        neg = v < 0 ? neg | (1u << at) : neg & ~(1u << at);
        big &= ~(1u << at);
        nzm |= 1u << at;
      }
    }
    if ((chg >> pos) & 1) lev = ((neg >> pos) & 1) ? -1 : 1;
  }
  if (act) coef[r] = (int16_t)lev;
  int v = p;
  if (cbp) {
    // dequantize (common/common_block.c:132-146): rshift 1, add 1
    const int d = te_wrap16(((lev * te_gdequant[qp % 6]) * (1 << (qp / 6)) + 1) >> 1);
    // inverse transform (common/transform.c:432-518): T'[k][y] = D^T C ..., R = D^T C D, clips
    int t2 = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) t2 += te_d4(colD, k) * __shfl(d, base + 4 * k + i);
    t2 = te_clip16((t2 + 64) >> 7);
    int res = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) res += te_d4(colD, k) * __shfl(t2, base + 4 * k + i);
    res = te_clip16((res + 2048) >> 12);
    v = te_clip255(res + p);
  }
  if (act) rec[r] = (uint8_t)v;
  te_sync();
  return cbp;
}
// The same for an 8 x 8 block: lane r holds pixel / coefficient r (raster).
// The forward passes are the reference SIMD transform8 (te_fwd8: 16-bit
// wrapping butterflies), output (k, row) in lane 8k + row, its input row
// gathered with eight ds_bpermute; the inverse passes take the 8-point basis
// column from the worker's LDS copy (X.M).
TE_FN uint32_t te_or_wave(uint32_t v) {  // OR over the wave, uniform
  v |= (uint32_t)TE_DPP(v, 0xB1);
  v |= (uint32_t)TE_DPP(v, 0x4E);
  v |= (uint32_t)TE_DPP(v, 0x141);
  v |= (uint32_t)TE_DPP(v, 0x140);
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) | (uint32_t)__builtin_amdgcn_readlane((int)v, 16) |
         (uint32_t)__builtin_amdgcn_readlane((int)v, 32) | (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}
TE_FN int te_fwd8r(const int *s, int k, int shift) {  // te_fwd8 (enc_pix.h) on a register row
  int E[4], O[4];
#pragma unroll
  for (int m = 0; m < 4; m++) {
    E[m] = te_wrap16(s[m] + s[7 - m]);
    O[m] = te_wrap16(s[m] - s[7 - m]);
  }
  const int EO0 = te_wrap16(E[0] - E[3]), EO1 = te_wrap16(E[1] - E[2]);
  int v;
  switch (k) {
    case 0: v = 64 * E[0] + 64 * E[1] + 64 * E[2] + 64 * E[3]; break;
    case 4: v = 64 * E[0] - 64 * E[1] - 64 * E[2] + 64 * E[3]; break;
    case 2: v = 83 * EO0 + 36 * EO1; break;
    case 6: v = 36 * EO0 - 83 * EO1; break;
    case 1: v = 89 * O[0] + 75 * O[1] + 50 * O[2] + 18 * O[3]; break;
    case 3: v = 75 * O[0] - 18 * O[1] - 89 * O[2] - 50 * O[3]; break;
    case 5: v = 50 * O[0] - 89 * O[1] + 18 * O[2] + 75 * O[3]; break;
    default: v = 18 * O[0] - 50 * O[1] + 75 * O[2] - 89 * O[3]; break;
  }
  return te_wrap16((v + (1 << (shift - 1))) >> shift);
}
TE_FN int te_c8_code(int p, const uint8_t *org, int os, int qp, int16_t *coef, uint8_t *rec, int type) {
  const TeScratch S = te_here();
  const TeTx &X = *S.tx;
  const int L = TE_LANE, hi = L >> 3, lo = L & 7;
  const int R = (int)org[hi * os + lo] - p;
  // transform8 (common/common_kernels.c:1887-1967): T[k][row] from row `row` of R, then C[k][row] from row `row` of T
  int x[8];
#pragma unroll
  for (int m = 0; m < 8; m++) x[m] = __shfl(R, 8 * lo + m);
  const int t = te_fwd8r(x, hi, 3);
#pragma unroll
  for (int m = 0; m < 8; m++) x[m] = __shfl(t, 8 * lo + m);
  const int C = te_fwd8r(x, hi, 8);
  // quantize (enc/encode_block.c:75-172, rdoq 0), q = 8
  const int intra = (type >> 1) & 1, chroma = type & 1;
  const int scale = te_gquant[qp % 6], shift2 = 21 - 3 + qp / 6;
  const int offset = (intra ? 38 : -26) * (1 << (shift2 - 8));
  const int pos = te_zz(8, L);
  const int lp = (te_abs(te_abs(C) * scale + offset) >> shift2) != 0 ? pos : -1;
  const int last_pos = te_maxi(lp);
  const int off0 = (intra ? 102 : 51) * (1 << (shift2 - 8)), off1 = (intra ? 115 : 90) * (1 << (shift2 - 8));
  int lev = 0;
  if (pos <= last_pos) {
    const int ac = scale * te_abs(C);
    const int l0 = ac >> shift2;
    const int l = (ac + ((l0 == 0 || chroma) ? off0 : off1)) >> shift2;
    lev = C < 0 ? -l : l;
  }
  const int cbp = te_any(lev != 0);
  if (cbp) {  // RDOQ light (:134-168) on the scan-order masks, as te_quant_t
    const int n = chroma ? last_pos + 1 : 64;
    const int thr = (73 * te_gdequant[qp % 6] << (qp / 6)) >> (4 + 3);
    const bool b1 = te_abs(lev) > 1, b0 = lev != 0;
    uint64_t big = (uint64_t)te_or_wave(b1 && pos < 32 ? 1u << pos : 0u) |
                   (uint64_t)te_or_wave(b1 && pos >= 32 ? 1u << (pos - 32) : 0u) << 32;
    uint64_t nzm = (uint64_t)te_or_wave(b0 && pos < 32 ? 1u << pos : 0u) |
                   (uint64_t)te_or_wave(b0 && pos >= 32 ? 1u << (pos - 32) : 0u) << 32;
    uint64_t chg = 0, neg = 0;
    uint64_t m = big & (n >= 64 ? ~0ull : ((1ull << n) - 1)) & ~3ull;
    while (m) {
      const int q = __builtin_ctzll(m);
      m &= m - 1;
      int flag = 1;
      if (q > 2 && ((big >> (q - 3)) & 1)) flag = 0;
      if (q > 3 && ((big >> (q - 4)) & 1) && ((nzm >> (q - 3)) & 1)) flag = 0;
      if (q == 2 && (chroma == 0 || last_pos >= 6)) flag = 0;
      if (flag && !((nzm >> (q - 2)) & 1) && !((nzm >> (q - 1)) & 1) && ((big >> q) & 1)) {
        const int c1 = __builtin_amdgcn_readlane(C, te_izz(8, q));
        const int c2 = __builtin_amdgcn_readlane(C, te_izz(8, q - 1));
        const int c3 = __builtin_amdgcn_readlane(C, te_izz(8, q - 2));
        const int K1 = te_abs(c1), K2 = te_abs(c2), K3 = te_abs(c3), K4 = TE_MAX(K2, K3);
        int at, v;
        if (K1 + K4 < thr) {
          at = q;
          v = c1 < 0 ? -1 : 1;
        } else if (K2 > K3) {
          at = q - 1;
          v = c2 < 0 ? -1 : 1;
        } else {
          at = q - 2;
          v = c3 < 0 ? -1 : 1;
        }
        chg |= 1ull << at;
        neg = v < 0 ? neg | (1ull << at) : neg & ~(1ull << at);
        big &= ~(1ull << at);
        nzm |= 1ull << at;
      }
    }
    if ((chg >> pos) & 1) lev = ((neg >> pos) & 1) ? -1 : 1;
  }
  coef[L] = (int16_t)lev;
  int v = p;
  if (cbp) {
    // dequantize (common/common_block.c:132-146): rshift 2, add 2
    const int d = te_wrap16(((lev * te_gdequant[qp % 6]) * (1 << (qp / 6)) + 2) >> 2);
    // inverse transform (common/transform.c:432-518), te_inv_gen<8>: basis column `lo` from X.M
    int dc[8];
#pragma unroll
    for (int k = 0; k < 8; k++) dc[k] = TE_DCT(X, 8, k, lo);
    int t2 = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) t2 += dc[k] * __shfl(d, 8 * k + hi);
    t2 = te_clip16((t2 + 64) >> 7);
    int res = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) res += dc[k] * __shfl(t2, 8 * k + hi);
    res = te_clip16((res + 2048) >> 12);
    v = te_clip255(res + p);
  }
  rec[L] = (uint8_t)v;
  te_sync();
  return cbp;
}
TE_FN int te_enc_intra_c8(const uint8_t *org, int os, const uint8_t *rf, int fs, int ypos, int xpos, int qp,
                          int16_t *coef, uint8_t *rec, int type, int mode, int ur, int dl, int key) {
  TE_P(TP_INTRA_COMP);
  const TeScratch S = te_here();
  TeNbr &nbw = *S.nb;
  TeIpc c;
  if (key && __builtin_amdgcn_readfirstlane(g_te_nb_key) == key) {  // the search just built them for this block
    c = te_ipx_consts(nbw, 8);
  } else {
    te_make_top_and_left(nbw, rf, fs, nullptr, 0, 0, 0, ypos, xpos, 8, ur, dl, 0);
    c = te_ipx_setup(nbw, 8);
  }
  const TeNbr &nb = nbw;
  {  // DC of get_intra_prediction (position-aware, common/intra_prediction.c:145-160)
    int sl = 0, st = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      sl += nb.left[k];
      st += nb.top[k];
    }
    c.dc = ((xpos != 0 ? sl : st) + (ypos != 0 ? st : sl) + 8) / 16;
  }
  const int L = TE_LANE;
  return te_c8_code(te_ipx(nb, c, 8, mode, L >> 3, L & 7), org, os, qp, coef, rec, type);
}
TE_FN int te_enc_inter_c8(const uint8_t *org, int os, int qp, const uint8_t *pb, int16_t *coef, uint8_t *rec, int type) {
  TE_P(TP_INTER_COMP);
  return te_c8_code(te_lds(pb)[TE_LANE], org, os, qp, coef, rec, type);
}
TE_FN int te_enc_intra_c4(const TeFrame &F, const uint8_t *org, int os, const uint8_t *rf, int fs, int ypos, int xpos,
                          int qp, int16_t *coef, uint8_t *rec, int type, int mode, int ur, int dl) {
  TE_P(TP_INTRA_COMP);
  (void)F;
  const TeScratch S = te_here();
  TeNbr &nbw = *S.nb;
  te_make_top_and_left(nbw, rf, fs, nullptr, 0, 0, 0, ypos, xpos, 4, ur, dl, 0);
  TeIpc c = te_ipx_setup(nbw, 4);
  const TeNbr &nb = nbw;
  {  // DC of get_intra_prediction (position-aware, common/intra_prediction.c:145-160)
    const int sl = nb.left[0] + nb.left[1] + nb.left[2] + nb.left[3], st = nb.top[0] + nb.top[1] + nb.top[2] + nb.top[3];
    c.dc = ((xpos != 0 ? sl : st) + (ypos != 0 ? st : sl) + 4) / 8;
  }
  const int r = TE_LANE & 15;
  return te_c4_code(te_ipx(nb, c, 4, mode, r >> 2, r & 3), org, os, qp, coef, rec, type);
}
// te_enc_inter_comp for a 4 x 4 block: the prediction from the compact buffer (stride 4)
TE_FN int te_enc_inter_c4(const uint8_t *org, int os, int qp, const uint8_t *pb, int16_t *coef, uint8_t *rec, int type) {
  TE_P(TP_INTER_COMP);
  return te_c4_code(te_lds(pb)[TE_LANE & 15], org, os, qp, coef, rec, type);
}
#else
TE_FN int te_enc_inter_c8(const uint8_t *, int, int, const uint8_t *, int16_t *, uint8_t *, int) { return 0; }
TE_FN int te_enc_intra_c8(const uint8_t *, int, const uint8_t *, int, int, int, int, int16_t *, uint8_t *, int, int, int,
                          int, int) {
  return 0;
}
TE_FN int te_enc_inter_c4(const uint8_t *, int, int, const uint8_t *, int16_t *, uint8_t *, int) { return 0; }
TE_FN int te_enc_intra_c4(const TeFrame &, const uint8_t *, int, const uint8_t *, int, int, int, int, int16_t *, uint8_t *,
                          int, int, int, int) {
  return 0;  // (TE_C4 is 0 on the host: the generic chain runs)
}
#endif

// The candidate just written (its nbits end at b.pos) became the best: keep
// its syntax bits, so that the final encode of the block (re-use, the same
// parameters and contexts) copies them instead of running write_block again.
TE_FN void te_keep_best_bits(TeBits &b, TeBlockInfo &bi, int nbits) {
  if (nbits > bi.best_cap * 32 || b.pos > b.cap) {
    bi.best_nbits = -1;
    return;
  }
  if ((b.pos & 31) && TE_LANE == 0) b.w[b.pos >> 5] = b.cur;  // the register word (stored again when complete)
  te_sync();
  const int start = b.pos - nbits, nw = (nbits + 31) >> 5, cw = b.cap >> 5;
  for (int i = TE_LANE; i < nw; i += TE_NL) {
    const int p = start + 32 * i, wi = p >> 5, sh = p & 31;
    uint32_t v = b.w[wi] << sh;
    if (sh && wi + 1 < cw) v |= b.w[wi + 1] >> (32 - sh);
    bi.best_bits[i] = v;
  }
  te_sync();
  bi.best_nbits = nbits;
}
// put nbits kept by te_keep_best_bits
TE_FN void te_put_kept(TeBits &b, const uint32_t *w, int nbits) {
#if !defined(TE_HOST)
  for (int base = 0; base * 32 < nbits; base += 64) {
    const int nw = TE_MIN(64, ((nbits + 31) >> 5) - base);
    const uint32_t wl = TE_LANE < nw ? w[base + TE_LANE] : 0u;
    for (int i = 0; i < nw; i++) {
      const int n = TE_MIN(32, nbits - 32 * (base + i));
      const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)wl, i);
      te_put(b, n, n == 32 ? v : v >> (32 - n));
    }
  }
#else
  for (int i = 0; 32 * i < nbits; i++) {
    const int n = TE_MIN(32, nbits - 32 * i);
    te_put(b, n, n == 32 ? w[i] : w[i] >> (32 - n));
  }
#endif
}

// encode_block, enc/encode_block.c:1590-1800: predict, code the residual into
// bi.rec, write the block's syntax.  Returns the bit count.
// One out-of-line copy of the intra chain for the P / B frames' copy of
// te_encode_block below.
TE_NOINL int te_enc_intra_comp_nc(const TeFrame &F_, const uint8_t *org, int os, const uint8_t *rf, int fs, int ypos,
                                  int xpos, int size, int qp, uint8_t *pb_, int16_t *coef, uint8_t *rec, int type,
                                  int tb_split, int mode, int ur, int dl, int ts) {
  return te_enc_intra_comp(F_, org, os, rf, fs, ypos, xpos, size, qp, pb_, coef, rec, type, tb_split, mode, ur, dl, ts);
}
// IFR: the I-frame copy, with the intra chains inlined (no call per
// component); P / B frames use the other, whose body stays small for the
// inter candidates that dominate them.
template <bool IFR>
TE_FN int te_encode_block_t(const TeFrame &F_, TeBits &b_, TeBlockInfo &bi_, TeParam &p_) {
  const TeFrame &F = *te_lds(&F_);
  const TeScratch S = te_here();
  TeBlockInfo &bi = *te_lds(&bi_);
  TeBits &b = *te_lds(&b_);
  TeParam &p = *te_lds(&p_);
  TE_P(TP_ENC_BLOCK);
  const int size = bi.size, ypos = bi.ypos, xpos = bi.xpos, yC = ypos / 2, xC = xpos / 2, sC = size / 2;
  const int mode = p.mode;
  const int qpY = F.qp + bi.delta_qp, qpC = te_chroma_qp(qpY);
  uint8_t *recY = bi.rec, *recU = te_pu(bi.rec, size), *recV = te_pv(bi.rec, size);
  const int tb_split = TE_MAX(0, p.tb_param), zero_block = p.tb_param == -1;
  p.tb_split = tb_split;
  const uint8_t *oY = F.oy + ypos * F.osy + xpos, *oU = F.ou + yC * F.osc + xC, *oV = F.ov + yC * F.osc + xC;
  int cy = 0, cu = 0, cv = 0;
  const int itype = (F.frame_type == TE_I) << 1;  // quantisation type follows the frame type (:1764)
  if (mode == TE_INTRA) {
    const int ur = te_upright_avail(ypos, xpos, size, F.W), dl = te_downleft_avail(ypos, xpos, size, F.H);
#define TE_INTRA_CHAINS(fn)                                                                                        \
  if (TE_C4 && size == 8 && !tb_split)                                                                             \
    cy = te_enc_intra_c8(oY, F.osy, F.ry + ypos * F.rsy + xpos, F.rsy, ypos, xpos, qpY, p.coeff, recY, itype | 0,   \
                         p.intra_mode, ur, dl, te_nb_key(ypos, xpos, 8));                                          \
  else                                                                                                             \
    cy = fn(F, oY, F.osy, F.ry + ypos * F.rsy + xpos, F.rsy, ypos, xpos, size, qpY, S.pb, p.coeff, recY, itype | 0,  \
            tb_split, p.intra_mode, ur, dl, p.ts);                                                                 \
  if (TE_C4 && sC == 8 && !(tb_split && size > 8)) {                                                              \
    cu = te_enc_intra_c8(oU, F.osc, F.ru + yC * F.rsc + xC, F.rsc, yC, xC, qpC, p.coeff + p.cs, recU, itype | 1,     \
                         p.intra_mode, ur, dl, 0);                                                                 \
    cv = te_enc_intra_c8(oV, F.osc, F.rv + yC * F.rsc + xC, F.rsc, yC, xC, qpC, p.coeff + 2 * p.cs, recV, itype | 1, \
                         p.intra_mode, ur, dl, 0);                                                                 \
  } else if (TE_C4 && sC == 4) {                                                                                  \
    cu = te_enc_intra_c4(F, oU, F.osc, F.ru + yC * F.rsc + xC, F.rsc, yC, xC, qpC, p.coeff + p.cs, recU, itype | 1,  \
                         p.intra_mode, ur, dl);                                                                    \
    cv = te_enc_intra_c4(F, oV, F.osc, F.rv + yC * F.rsc + xC, F.rsc, yC, xC, qpC, p.coeff + 2 * p.cs, recV,        \
                         itype | 1, p.intra_mode, ur, dl);                                                         \
  } else {                                                                                                         \
    cu = fn(F, oU, F.osc, F.ru + yC * F.rsc + xC, F.rsc, yC, xC, sC, qpC, S.pb, p.coeff + p.cs, recU, itype | 1,   \
            tb_split && size > 8, p.intra_mode, ur, dl, p.ts);                                                     \
    cv = fn(F, oV, F.osc, F.rv + yC * F.rsc + xC, F.rsc, yC, xC, sC, qpC, S.pb, p.coeff + 2 * p.cs, recV,          \
            itype | 1, tb_split && size > 8, p.intra_mode, ur, dl, p.ts);                                          \
  }
    if constexpr (IFR) {
      TE_INTRA_CHAINS(te_enc_intra_comp)
    } else {
      TE_INTRA_CHAINS(te_enc_intra_comp_nc)
    }
#undef TE_INTRA_CHAINS
  } else {
    const int bip = F.enable_bipred;
    if (mode == TE_SKIP) {
      if (p.dir == 2) {
        te_pred_yuv(F, p.ref_idx0, S.pb0, bi, p.mv0, te_sign_of(F, p.ref_idx0, 1), bip, 0);
        te_pred_yuv(F, p.ref_idx1, S.pb1, bi, p.mv1, te_sign_of(F, p.ref_idx1, 1), bip, 0);
        te_avg_yuv(bi.rec, S.pb0, S.pb1, bi);
      } else {
        te_pred_yuv(F, p.ref_idx0, bi.rec, bi, p.mv0, te_sign_of(F, p.ref_idx0, 0), bip, 0);
      }
    } else if (mode == TE_MERGE) {
      if (p.dir == 2) {
        te_pred_yuv(F, p.ref_idx0, S.pb0, bi, p.mv0, te_sign_of(F, p.ref_idx0, 1), bip, 0);
        te_pred_yuv(F, p.ref_idx1, S.pb1, bi, p.mv1, te_sign_of(F, p.ref_idx1, 1), bip, 0);
        te_avg_yuv(S.pb, S.pb0, S.pb1, bi);
      } else {
        te_pred_yuv(F, p.ref_idx0, S.pb, bi, p.mv0, te_sign_of(F, p.ref_idx0, 0), bip, 0);
      }
    } else if (mode == TE_INTER) {
      te_pred_yuv(F, p.ref_idx0, S.pb, bi, p.mv0, te_sign_of(F, p.ref_idx0, 0), bip, F.enable_pb_split);
    } else if (mode == TE_BIPRED) {
      te_pred_yuv(F, p.ref_idx0, S.pb0, bi, p.mv0, te_sign_of(F, p.ref_idx0, 1), bip, F.enable_pb_split);
      te_pred_yuv(F, p.ref_idx1, S.pb1, bi, p.mv1, te_sign_of(F, p.ref_idx1, 1), bip, F.enable_pb_split);
      te_avg_yuv(S.pb, S.pb0, S.pb1, bi);
    }
    if (mode != TE_SKIP) {
      if (zero_block) {
        te_copy_bytes(bi.rec, S.pb, size * size + 2 * sC * sC);
      } else {
        if (TE_C4 && size == 8 && !tb_split)
          cy = te_enc_inter_c8(oY, F.osy, qpY, S.pb, p.coeff, recY, itype | 0);
        else
          cy = te_enc_inter_comp(F, oY, F.osy, size, qpY, S.pb, p.coeff, recY, itype | 0, tb_split, p.ts);
        if (TE_C4 && sC == 8 && !(tb_split && size > 8)) {
          cu = te_enc_inter_c8(oU, F.osc, qpC, te_pu(S.pb, size), p.coeff + p.cs, recU, itype | 1);
          cv = te_enc_inter_c8(oV, F.osc, qpC, te_pv(S.pb, size), p.coeff + 2 * p.cs, recV, itype | 1);
        } else if (TE_C4 && sC == 4) {
          cu = te_enc_inter_c4(oU, F.osc, qpC, te_pu(S.pb, size), p.coeff + p.cs, recU, itype | 1);
          cv = te_enc_inter_c4(oV, F.osc, qpC, te_pv(S.pb, size), p.coeff + 2 * p.cs, recV, itype | 1);
        } else {
          cu = te_enc_inter_comp(F, oU, F.osc, sC, qpC, te_pu(S.pb, size), p.coeff + p.cs, recU, itype | 1,
                                 tb_split && size > 8, p.ts);
          cv = te_enc_inter_comp(F, oV, F.osc, sC, qpC, te_pv(S.pb, size), p.coeff + 2 * p.cs, recV,
                                 itype | 1, tb_split && size > 8, p.ts);
        }
      }
    }
  }
  p.cbp_y = cy;
  p.cbp_u = cu;
  p.cbp_v = cv;
  const int nbits = te_write_block(b, F, bi, p, S.tx->scan);
  TE_TR(F.frame_num, 2, bi.ypos, bi.xpos, bi.size | p.mode << 8 | (p.tb_param + 1) << 12 | p.skip_idx << 16,
        p.ref_idx0 | p.ref_idx1 << 4 | p.pb_part << 8 | p.intra_mode << 12, nbits, cy | cu << 1 | cv << 2);
  if (tb_split) p.cbp_y = p.cbp_u = p.cbp_v = 1;  // deblocking only (:1781-1784)
  return nbits;
}
// The two out-of-line copies (one call frame each; the I-frame copy may also be
// inlined where it has a single call site, TE_EB1_INLINE)
TE_NOINL int te_encode_block_i(const TeFrame &F, TeBits &b, TeBlockInfo &bi, TeParam &p) {
  return te_encode_block_t<true>(F, b, bi, p);
}
TE_NOINL int te_encode_block_p(const TeFrame &F, TeBits &b, TeBlockInfo &bi, TeParam &p) {
  return te_encode_block_t<false>(F, b, bi, p);
}
TE_FN int te_encode_block(const TeFrame &F, TeBits &b, TeBlockInfo &bi, TeParam &p) {
  return te_lds(&F)->frame_type == TE_I ? te_encode_block_i(F, b, bi, p) : te_encode_block_p(F, b, bi, p);
}
#ifdef TE_EB1_INLINE
#define TE_ENCODE_I te_encode_block_t<true>
#else
#define TE_ENCODE_I te_encode_block_i
#endif
// The final encode of a block with its best parameters bi.bp (process_block,
// enc/encode_block.c:2953-2962 / 3012-3018).  Without tb-split the best
// candidate's reconstruction is in rec_best and (usually) its syntax bits in
// best_bits: copy them here, inline, so this common case makes no call -- a
// call of te_encode_block_t saves and restores ~100 callee-saved VGPRs through
// scratch.  Otherwise it is a full encode.
TE_FN int te_encode_final(const TeFrame &F_, TeBits &b_, TeBlockInfo &bi_) {
  const TeFrame &F = *te_lds(&F_);
  TeBlockInfo &bi = *te_lds(&bi_);
  TeBits &b = *te_lds(&b_);
  if (!F.enable_tb_split) {  // re_use: the best candidate's reconstruction becomes rec (a swap, as copy_best does)
    uint8_t *t = bi.rec;
    bi.rec = bi.rec_best;
    bi.rec_best = t;
    if (bi.best_nbits >= 0) {  // the best candidate's own syntax bits
      te_put_kept(b, bi.best_bits, bi.best_nbits);
      return bi.best_nbits;
    }
    return te_write_block(b, F, bi, bi.bp, te_here().tx->scan);
  }
  return te_encode_block(F, b, bi, bi.bp);
}

// cost_calc, enc/encode_block.c:1218-1228
TE_FN uint32_t te_cost(const TeFrame &F, const TeBlockInfo &bi, const uint8_t *rec, int w, int h, int nbits) {
  TE_P(TP_COST);
  const int size = bi.size, sC = size / 2;
  const int ypos = bi.ypos, xpos = bi.xpos;
  const uint32_t sy = te_ssd(F.oy + ypos * F.osy + xpos, F.osy, rec, size, w, h);
  const uint32_t su = te_ssd(F.ou + (ypos / 2) * F.osc + xpos / 2, F.osc, te_pu((uint8_t *)rec, size), sC, w / 2, h / 2);
  const uint32_t sv = te_ssd(F.ov + (ypos / 2) * F.osc + xpos / 2, F.osc, te_pv((uint8_t *)rec, size), sC, w / 2, h / 2);
  const double prod = F.lambda * (double)nbits;
  uint32_t cost = sy + su + sv + (uint32_t)(int32_t)(prod + 0.5);
  if (cost > (1u << 30)) cost = 1u << 30;
  TE_TR(F.frame_num, 3, ypos, xpos, size, sy, su + sv, cost);
  return cost;
}

// search orders (constant memory: local arrays indexed at run time would be
// built on the stack on every call)
TE_CONST int8_t te_intra_order[10] = {TE_DC,      TE_HOR,       TE_VER,       TE_PLANAR,     TE_UPLEFT,
                                      TE_UPRIGHT, TE_UPUPRIGHT, TE_UPUPLEFT, TE_UPLEFTLEFT, TE_DOWNLEFTLEFT};
TE_CONST int8_t te_hex_dy[6] = {1, 2, 1, -1, -2, -1}, te_hex_dx[6] = {-1, 0, 1, 1, 0, -1};  // enc/encode_block.c:908-909
TE_CONST int8_t te_hp_m[9] = {0, 0, -2, 2, 0, -2, -2, 2, 2}, te_hp_n[9] = {0, -2, 0, 0, 2, -2, 2, -2, 2};  // :942-943
TE_CONST int8_t te_qp_m[9] = {0, 0, -1, 1, 0, -1, -1, 1, 1}, te_qp_n[9] = {0, -1, 0, 0, 1, -1, 1, -1, 1};


#if !defined(TE_HOST)
// blocks of 16 x 16 and up: T 4-pixel chunks per lane, the original in registers, one mode after the other
template <int T>
TE_FN void te_isearch(const TeNbr &nb, const TeIpc &c, const uint8_t *o, int os, int size, const int8_t *order, int n,
                      int &min_sad, int &best) {
  const int w4 = size >> 2;
  uint32_t org[T];
  int ci[T], cj[T];
#pragma unroll
  for (int t = 0; t < T; t++) {
    const int g = TE_LANE + 64 * t;
    ci[t] = te_dv(g, w4);
    cj[t] = (g - ci[t] * w4) * 4;
    org[t] = te_ld4(o + ci[t] * os + cj[t]);
  }
#pragma unroll 1
  for (int k = 0; k < n; k++) {
    const int mode = order[k];
    uint32_t a = 0;
#pragma unroll
    for (int t = 0; t < T; t++) a = te_sad4(org[t], te_ipx4(nb, c, size, mode, ci[t], cj[t]), a);
    const int sad = (int)te_sum(a);
    if (sad < min_sad) {
      best = mode;
      min_sad = sad;
    }
  }
}
#endif

// search_intra_prediction_params, enc/encode_block.c:1230-1329: SAD over the
// first `num_modes` modes in the order DC, HOR, VER, PLANAR, [UPLEFT ...].
// Device: every mode's prediction computed in registers against the original
// (no prediction buffer, no barrier per mode) -- 8x8: four modes at a time,
// one per 16-lane row (a row's sum is one DPP reduction); larger blocks: the
// modes one after the other over the whole wave, their sums reduced together.
// The first strictly smaller SAD wins, in the search order, as the reference.
TE_NOINL int te_search_intra(const TeFrame &F_, const TeBlockInfo &bi_, int num_modes, int *mode_out) {
  const TeFrame &F = *te_lds(&F_);
  const TeScratch S = te_here();
  const TeBlockInfo &bi = *te_lds(&bi_);
  TE_P(TP_SEARCH_INTRA);
  const int size = bi.size, ypos = bi.ypos, xpos = bi.xpos;
  const int ur = te_upright_avail(ypos, xpos, size, F.W), dl = te_downleft_avail(ypos, xpos, size, F.H);
  te_make_top_and_left(*S.nb, F.ry + ypos * F.rsy + xpos, F.rsy, nullptr, 0, 0, 0, ypos, xpos, size, ur, dl, 0);
  const int8_t *order = te_intra_order;
  int min_sad = 1 << 30, best = TE_DC;
  const int n = num_modes == 4 ? 4 : 10;
  const uint8_t *o = F.oy + ypos * F.osy + xpos;
#if !defined(TE_HOST)
  const TeNbr &nb = *S.nb;
  const TeIpc c = te_ipx_setup(*S.nb, size);
  if (TE_LANE == 0) g_te_nb_key = te_nb_key(ypos, xpos, size);  // (te_intra_pred below forgets it, sizes 32 / 64)
  te_sync();
  if (size == 8) {
    const int ch = TE_LANE & 15, row = TE_LANE >> 4, i = ch >> 1, j = (ch & 1) * 4;
    const uint32_t org = te_ld4(o + i * F.osy + j);
#pragma unroll
    for (int pass = 0; pass < 3; pass++) {
      if (4 * pass >= n) break;
      const int k = 4 * pass + row;
      uint32_t a = 0;
      if (k < n) a = te_sad4(org, te_ipx4(nb, c, 8, order[k], i, j), 0);
      a += (uint32_t)TE_DPP(a, 0xB1);
      a += (uint32_t)TE_DPP(a, 0x4E);
      a += (uint32_t)TE_DPP(a, 0x141);
      a += (uint32_t)TE_DPP(a, 0x140);
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int kk = 4 * pass + r;
        const int sad = __builtin_amdgcn_readlane((int)a, 16 * r);
        if (kk < n && sad < min_sad) {
          best = order[kk];
          min_sad = sad;
        }
      }
    }
  } else if (size == 16) {
    te_isearch<1>(nb, c, o, F.osy, size, order, n, min_sad, best);
  } else {  // 32, 64: few calls, many chunks per lane -- the prediction buffer keeps the code small
    const int w4 = size >> 2, n4 = w4 * size;
    uint32_t org[16];
#pragma unroll
    for (int t = 0; t < 16; t++) {
      const int g = TE_LANE + 64 * t;
      org[t] = 0;
      if (g < n4) {
        const int i = te_dv(g, w4), j = (g - i * w4) * 4;
        org[t] = te_ld4(o + i * F.osy + j);
      }
    }
    for (int k = 0; k < n; k++) {
      te_intra_pred(*S.nb, ypos, xpos, size, S.pb, order[k], 1);
      uint32_t a = 0;
#pragma unroll
      for (int t = 0; t < 16; t++) {
        const int g = TE_LANE + 64 * t;
        if (g < n4) a = te_sad4(org[t], te_ld4(S.pb + 4 * g), a);
      }
      const int sad = (int)te_sum(a);
      if (sad < min_sad) {
        best = order[k];
        min_sad = sad;
      }
    }
  }
#else
  for (int k = 0; k < n; k++) {
    te_intra_pred(*S.nb, ypos, xpos, size, S.pb, order[k], 1);
    const int sad = (int)te_sad(o, F.osy, S.pb, size, size, size);
    if (sad < min_sad) {
      best = order[k];
      min_sad = sad;
    }
  }
#endif
  *mode_out = best;
  return min_sad;
}

TE_FN uint32_t te_lambda_bits(double lam, int bits) { return (uint32_t)(lam * (double)bits + 0.5); }

#if !defined(TE_HOST)
// ---- candidate-parallel motion search (device) ------------------------------
// motion_estimate tries its candidates one at a time: each SAD a full-wave pass
// that ends in a reduction and a scalar compare after a memory round trip, most
// lanes idle for the small blocks.  The candidates of one search step are
// independent -- only the choice among them is ordered -- so here a step's
// candidates are evaluated together: the block's 4x4 units spread over the
// lanes (nu = w/4 x h/4 units, a power of two: nu <= 64 gives 64 / nu
// candidates per pass, one unit per lane; nu > 64, nu / 64 units per lane and
// two candidates per pass), the original held in registers in the same layout,
// one segmented DPP reduction per pass, then the reference's ordered scan over
// the step's costs (strictly below the running minimum): the same argmin, ties
// to the earlier candidate, as the one-at-a-time loop.
struct TeMeBlk {
  int w4, lw4, nu, lnu;  // units per row and its log2; units in the block and its log2
  uint32_t o[4][4];      // original unit rows: o[t][y] = row y of the lane's unit t
};
TE_FN int te_me_unit(const TeMeBlk &B, int t) { return B.nu <= 64 ? (TE_LANE & (B.nu - 1)) : TE_LANE + 64 * t; }
TE_FN void te_me_blk(TeMeBlk &B, const uint8_t *org, int os, int w, int h) {
  B.w4 = w >> 2;
  B.lw4 = __builtin_ctz(B.w4);
  B.nu = B.w4 * (h >> 2);
  B.lnu = __builtin_ctz(B.nu);
  const int nt = B.nu > 64 ? B.nu >> 6 : 1;
#pragma unroll
  for (int t = 0; t < 4; t++) {
#pragma unroll
    for (int y = 0; y < 4; y++) B.o[t][y] = 0;
    if (t < nt) {
      const int u = te_me_unit(B, t), i0 = (u >> B.lw4) * 4, j = (u & (B.w4 - 1)) * 4;
#pragma unroll
      for (int y = 0; y < 4; y++) B.o[t][y] = te_ld4(org + (i0 + y) * os + j);
    }
  }
}
// the lane's part of the SAD of the block at p (full-pel)
TE_FN uint32_t te_me_sad_lane(const TeMeBlk &B, const uint8_t *p, int rs) {
  const int nt = B.nu > 64 ? B.nu >> 6 : 1;
  uint32_t s = 0;
#pragma unroll
  for (int t = 0; t < 4; t++)
    if (t < nt) {
      const int u = te_me_unit(B, t), i0 = (u >> B.lw4) * 4, j = (u & (B.w4 - 1)) * 4;
      const uint8_t *q = p + i0 * rs + j;
      uint32_t d[4];
#pragma unroll
      for (int y = 0; y < 4; y++) d[y] = te_ld4(q + y * rs);
#pragma unroll
      for (int y = 0; y < 4; y++) s = te_sad4(B.o[t][y], d[y], s);
    }
  return s;
}
// the lane's part of the SAD of the sub-pel prediction at mv (te_mc_luma's
// 4x4-unit form, common/inter_prediction.c:120-180, fused: no prediction buffer)
TE_FN uint32_t te_me_mcsad_lane(const TeMeBlk &B, const uint8_t *ref, int rs, TeMv mv, int sign, int bipred) {
  const int mx = sign ? -mv.x : mv.x, my = sign ? -mv.y : mv.y;
  const int fy = my & 3, fx = mx & 3;
  const uint8_t *r = ref + (my >> 2) * rs + (mx >> 2);
  const int nt = B.nu > 64 ? B.nu >> 6 : 1;
  uint32_t s = 0;
#pragma unroll
  for (int t = 0; t < 4; t++) {
    if (t >= nt) continue;
    const int u = te_me_unit(B, t), i0 = (u >> B.lw4) * 4, j = (u & (B.w4 - 1)) * 4;
    int o[4][4];
    if (fx == 2 && fy == 2) {  // rows -1..5, columns -1..6, :145-157
      uint32_t lo[7], hi[7];
#pragma unroll
      for (int q = 0; q < 7; q++) {
        const uint8_t *p = r + (i0 - 1 + q) * rs + j - 1;
        lo[q] = te_ld4(p);
        hi[q] = te_ld4(p + 4);
      }
      int c[7][8];
#pragma unroll
      for (int q = 0; q < 7; q++)
#pragma unroll
        for (int k = 0; k < 4; k++) {
          c[q][k] = te_b(lo[q], k);
          c[q][k + 4] = te_b(hi[q], k);
        }
#pragma unroll
      for (int y = 0; y < 4; y++)
#pragma unroll
        for (int x = 0; x < 4; x++) {
          const int k = x + 1;
          const int *a = c[y], *b = c[y + 1], *d = c[y + 2], *e = c[y + 3];
          const int v = a[k] + a[k + 1] + b[k - 1] + 2 * b[k] + 2 * b[k + 1] + b[k + 2] + d[k - 1] + 2 * d[k] +
                        2 * d[k + 1] + d[k + 2] + e[k] + e[k + 1];
          o[y][x] = te_clip255((v + 8) >> 4);
        }
    } else {  // separable 6-tap (fraction 0: the identity taps {0, 0, 64, 0, 0, 0}, exact), :160-178
      const int8_t *fv = (bipred ? te_luma_bi : te_luma_uni)[fy];
      const int8_t *fh = (bipred ? te_luma_bi : te_luma_uni)[fx];
      uint32_t d[9][3];
#pragma unroll
      for (int q = 0; q < 9; q++) {
        const uint8_t *p = r + (i0 - 2 + q) * rs + j - 2;
        d[q][0] = te_ld4(p);
        d[q][1] = te_ld4(p + 4);
        d[q][2] = te_ld4(p + 8);
      }
      int hk[9][4];
#pragma unroll
      for (int q = 0; q < 9; q++) {
        int c[12];
#pragma unroll
        for (int b = 0; b < 4; b++) {
          c[b] = te_b(d[q][0], b);
          c[b + 4] = te_b(d[q][1], b);
          c[b + 8] = te_b(d[q][2], b);
        }
#pragma unroll
        for (int x = 0; x < 4; x++) {
          int a = 0;
#pragma unroll
          for (int m = 0; m < 6; m++) a += fh[m] * c[x + m];
          hk[q][x] = a;
        }
      }
#pragma unroll
      for (int y = 0; y < 4; y++)
#pragma unroll
        for (int x = 0; x < 4; x++) {
          int a = 0;
#pragma unroll
          for (int k = 0; k < 6; k++) a += fv[k] * hk[y + k][x];
          o[y][x] = te_clip255((a + 2048) >> 12);
        }
    }
#pragma unroll
    for (int y = 0; y < 4; y++) s = te_sad4(B.o[t][y], te_pack4(o[y][0], o[y][1], o[y][2], o[y][3]), s);
  }
  return s;
}
// v summed over every segment of 2^l lanes: l <= 4 in every lane of the segment
// (DPP inside 16-lane rows), l = 5, 6 per row (te_seg_get adds the rows)
TE_FN uint32_t te_seg_sum(uint32_t v, int l) {
  if (l >= 1) v += (uint32_t)TE_DPP(v, 0xB1);   // lane ^ 1
  if (l >= 2) v += (uint32_t)TE_DPP(v, 0x4E);   // lane ^ 2
  if (l >= 3) v += (uint32_t)TE_DPP(v, 0x141);  // row half mirror: the two quads of 8 lanes
  if (l >= 4) v += (uint32_t)TE_DPP(v, 0x140);  // row mirror: the two halves of a row
  return v;
}
TE_FN uint32_t te_seg_get(uint32_t v, int l, int sl) {
  if (l <= 4) return (uint32_t)__builtin_amdgcn_readlane((int)v, sl << l);
  if (l == 5) return (uint32_t)__builtin_amdgcn_readlane((int)v, 32 * sl) + (uint32_t)__builtin_amdgcn_readlane((int)v, 32 * sl + 16);
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) + (uint32_t)__builtin_amdgcn_readlane((int)v, 16) +
         (uint32_t)__builtin_amdgcn_readlane((int)v, 32) + (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}
// The costs of candidates 0 .. n-1 (cand(k): the candidate vector, a pure
// function of k evaluated per lane; SUBPEL: through the MC filters) plus
// mvcost(c), scanned in order: a cost strictly below min_sad becomes the best.
// Returns the index of the last improvement, -1 if none.
template <bool SUBPEL, class Cand, class MvCost>
TE_FN int te_me_scan(const TeMeBlk &B, const uint8_t *ref, int rs, int sign, int bipred, int n, Cand cand,
                     MvCost mvcost, uint32_t &min_sad, TeMv &mv_opt) {
  const int s = sign ? -1 : 1;
  auto lane_sad = [&](TeMv c) -> uint32_t {
    if constexpr (SUBPEL) return te_me_mcsad_lane(B, ref, rs, c, sign, bipred);
    else return te_me_sad_lane(B, ref + s * (c.x >> 2) + s * (c.y >> 2) * rs, rs);
  };
  int best = -1;
  auto take = [&](int k, uint32_t sad) {
    const TeMv c = cand(k);
    const uint32_t cost = sad + mvcost(c);
    if (cost < min_sad) {
      min_sad = cost;
      mv_opt = c;
      best = k;
    }
  };
  if (B.nu <= 64) {  // 64 / nu candidates per pass, one unit per lane
    const int G = 64 >> B.lnu, slot = TE_LANE >> B.lnu;
    for (int base = 0; base < n; base += G) {
      const int k = base + slot;
      uint32_t v = 0;
      if (k < n) v = lane_sad(cand(k));
      v = te_seg_sum(v, B.lnu);
      for (int sl = 0; sl < G && base + sl < n; sl++) take(base + sl, te_seg_get(v, B.lnu, sl));
    }
  } else {  // whole-wave blocks: two candidates per pass (both in flight before either reduction)
    for (int base = 0; base < n; base += 2) {
      const bool two = base + 1 < n;
      const uint32_t v0 = lane_sad(cand(base));
      const uint32_t v1 = two ? lane_sad(cand(base + 1)) : 0u;
      const uint32_t s0 = te_sum(v0), s1 = te_sum(v1);
      take(base, s0);
      if (two) take(base + 1, s1);
    }
  }
  return best;
}
#endif

// motion_estimate, enc/encode_block.c:830-1016 (params->sync = 0).  `org` /
// `os`: the block (or partition) of the original; `ref`: the reference at the
// block (partition) origin; size: the CU size (clip_mv, the size-16 rules).
TE_NOINL uint32_t te_motion_estimate(const TeFrame &F_, TeSB &sb_, int r, const uint8_t *org, int os,
                                     const uint8_t *ref, int size, int width, int height, TeMv *mv, TeMv mvc, TeMv mvp,
                                     int sign, int xpos, int ypos, int enable_bipred) {
  const TeFrame &F = *te_lds(&F_);
  const TeScratch S = te_here();
  TeSB &sb = *te_lds(&sb_);
  TE_P(TP_ME);
  const int rs = F.rsy, s = sign ? -1 : 1;
  const double lam = F.sqrt_lambda;
  uint32_t min_sad = TE_MAX_UINT32;
  TeMv mv_opt, mv_ref, c;
  mv_opt.x = mv_opt.y = 0;
  mv_ref.y = (int16_t)((((int)mvc.y + 2) >> 2) << 2);
  mv_ref.x = (int16_t)((((int)mvc.x + 2) >> 2) << 2);
#if !defined(TE_HOST) && !defined(TE_ME_SEQ)
  TeMeBlk B;
  te_me_blk(B, org, os, width, height);
  auto mvcost = [&](TeMv c) -> uint32_t { return te_lambda_bits(lam, te_mv_bits(c.y - mvp.y, c.x - mvp.x)); };
  const int wide32 = size == 16 && F.speed < 2 && F.speed > 0;  // speed 1: the step-32 pass takes widesad
#endif
  if ((size == 16 && enable_bipred) || F.speed == 0) {  // telescope search
    int step = 32;
#if !defined(TE_HOST) && !defined(TE_ME_SEQ)
    // the 5 x 5 grid of a step, row-major, the centre skipped after the first step
    for (; step >= 4 && !(step == 32 && wide32); step >>= 1) {
      const TeMv ref0 = mv_ref;
      const int st = step, skipc = step < 32;
      auto cand = [&](int idx) -> TeMv {
        const int q = idx + (skipc && idx >= 12 ? 1 : 0);
        TeMv c;
        c.y = (int16_t)(ref0.y + (q / 5 - 2) * st);
        c.x = (int16_t)(ref0.x + (q % 5 - 2) * st);
        return te_clip_mv(c, ypos, xpos, F.W, F.H, size, sign);
      };
      te_me_scan<false>(B, ref, rs, sign, enable_bipred, 25 - skipc, cand, mvcost, min_sad, mv_opt);
      mv_ref = mv_opt;
    }
#endif
    while (step >= 4) {
      const int range = 2 * step;
      for (int k = -range; k <= range; k += step)
        for (int l = -range; l <= range; l += step) {
          if (step < 32 && !k && !l) continue;
          c.y = (int16_t)(mv_ref.y + k);
          c.x = (int16_t)(mv_ref.x + l);
          c = te_clip_mv(c, ypos, xpos, F.W, F.H, size, sign);
          uint32_t sad;
          const uint8_t *rp = ref + s * (c.x >> 2) + s * (c.y >> 2) * rs;
          if (step == 32 && size == 16 && F.speed < 2 && F.speed > 0) {
            int x = 0;
            sad = te_widesad(org, os, rp, rs, width, height, &x);
            c.x = (int16_t)(c.x + (s * x << 2));
          } else {
            sad = te_sad(org, os, rp, rs, width, height);
          }
          sad += te_lambda_bits(lam, te_mv_bits(c.y - mvp.y, c.x - mvp.x));
          if (sad < min_sad) {
            min_sad = sad;
            mv_opt = c;
          }
        }
      mv_ref = mv_opt;
      step >>= 1;
    }
  }
#if !defined(TE_HOST) && !defined(TE_ME_SEQ)
  if (size != 16) {  // candidate search (the size-16 candidates take widesad: one at a time below)
    const TeMv *cl = sb.mc.mv[r];
    auto cand = [&](int idx) -> TeMv {
      const TeMv cm = cl[idx];
      TeMv c;
      c.y = (int16_t)(cm.y << 2);
      c.x = (int16_t)(cm.x << 2);
      return te_clip_mv(c, ypos, xpos, F.W, F.H, size, sign);
    };
    te_me_scan<false>(B, ref, rs, sign, enable_bipred, sb.mc.num[r], cand, mvcost, min_sad, mv_opt);
  } else
#endif
  for (int idx = 0; idx < sb.mc.num[r]; idx++) {  // candidate search
    int x = 0;
    const TeMv cm = sb.mc.mv[r][idx];
    c.y = (int16_t)(cm.y << 2);
    c.x = (int16_t)(cm.x << 2);
    c = te_clip_mv(c, ypos, xpos, F.W, F.H, size, sign);
    const uint8_t *rp = ref + s * (c.x >> 2) + s * (c.y >> 2) * rs;
    uint32_t sad = size == 16 ? te_widesad(org, os, rp, rs, width, height, &x) : te_sad(org, os, rp, rs, width, height);
    c.x = (int16_t)(c.x + (s * x << 2));
    sad += te_lambda_bits(lam, te_mv_bits(c.y - mvp.y, c.x - mvp.x));
    if (sad < min_sad) {
      min_sad = sad;
      mv_opt = c;
    }
  }
  mv_ref = mv_opt;
  const int maxsteps = size <= 16 || F.speed == 0 ? 6 : 0;
  int start = 0, end = 5;
  for (int step = 1; step < maxsteps; step++) {  // full-pel hexagon search
    const int8_t *diy = te_hex_dy, *dix = te_hex_dx;
    int dir = start - 1, best_dir = -1;
#if !defined(TE_HOST) && !defined(TE_ME_SEQ)
    {  // directions start .. end (cyclic), in order
      const int nd = (end - start + 6) % 6 + 1, st0 = start;
      const TeMv ref0 = mv_ref;
      auto cand = [&](int idx) -> TeMv {
        const int d = (st0 + idx) % 6;
        TeMv c;
        c.y = (int16_t)(ref0.y + dix[d] * 4);
        c.x = (int16_t)(ref0.x + diy[d] * 4);
        return te_clip_mv(c, ypos, xpos, F.W, F.H, size, sign);
      };
      const int bk = te_me_scan<false>(B, ref, rs, sign, enable_bipred, nd, cand, mvcost, min_sad, mv_opt);
      best_dir = bk < 0 ? -1 : (st0 + bk) % 6;
    }
    if (0)
#endif
    do {
      dir++;
      dir = dir == 6 ? 0 : dir;
      c.y = (int16_t)(mv_ref.y + dix[dir] * 4);
      c.x = (int16_t)(mv_ref.x + diy[dir] * 4);
      c = te_clip_mv(c, ypos, xpos, F.W, F.H, size, sign);
      uint32_t sad = te_sad(org, os, ref + s * (c.x >> 2) + s * (c.y >> 2) * rs, rs, width, height);
      sad += te_lambda_bits(lam, te_mv_bits(c.y - mvp.y, c.x - mvp.x));
      if (sad < min_sad) {
        min_sad = sad;
        mv_opt = c;
        best_dir = dir;
      }
    } while (dir != end);
    mv_ref = mv_opt;
    start = best_dir ? best_dir - 1 : 5;
    end = start + 2;
    end -= (end >= 6) * 6;
    if (best_dir < 0) break;
  }
  TE_TR(F.frame_num, 9, ypos, xpos, size | width << 8 | height << 16, r, min_sad,
        (mv_ref.x & 0xffff) | (int)mv_ref.y << 16);
  int ydelta_hp = 0, xdelta_hp = 0, ydelta_qp = 0, xdelta_qp = 0;
  uint32_t cmin = min_sad;
  if (F.speed == 0) {  // exact half- and quarter-pel search through the MC filters
    const int8_t *hm = te_hp_m, *hn = te_hp_n;
#if !defined(TE_HOST) && !defined(TE_ME_SEQ)
    {
      const TeMv ref0 = mv_ref;
      auto hcand = [&](int idx) -> TeMv {
        TeMv c;
        c.y = (int16_t)(ref0.y + hm[idx + 1]);
        c.x = (int16_t)(ref0.x + hn[idx + 1]);
        return c;
      };
      TeMv dummy;
      const int hb = te_me_scan<true>(B, ref, rs, sign, enable_bipred, 8, hcand, mvcost, cmin, dummy);
      if (hb >= 0) {
        ydelta_hp = hm[hb + 1];
        xdelta_hp = hn[hb + 1];
      }
      mv_opt.x = (int16_t)(mv_opt.x + xdelta_hp);
      mv_opt.y = (int16_t)(mv_opt.y + ydelta_hp);
      const int8_t *qm = te_qp_m, *qn = te_qp_n;
      const TeMv opt0 = mv_opt;
      auto qcand = [&](int idx) -> TeMv {
        TeMv c;
        c.y = (int16_t)(opt0.y + qm[idx + 1]);
        c.x = (int16_t)(opt0.x + qn[idx + 1]);
        return c;
      };
      auto qcost = [&](TeMv c) -> uint32_t {
        return (uint32_t)(int)(lam * (double)te_mv_bits(c.y - mvp.y, c.x - mvp.x) + 0.5);
      };
      const int qb = te_me_scan<true>(B, ref, rs, sign, enable_bipred, 8, qcand, qcost, cmin, dummy);
      if (qb >= 0) {
        ydelta_qp = qm[qb + 1];
        xdelta_qp = qn[qb + 1];
      }
    }
    if (0) {
#endif
    for (int i = 1; i <= 8; i++) {
      c.y = (int16_t)(mv_ref.y + hm[i]);
      c.x = (int16_t)(mv_ref.x + hn[i]);
      te_mc_luma(S.rf, width, ref, rs, width, height, c, sign, enable_bipred);
      uint32_t sad = te_sad(org, os, S.rf, width, width, height);
      sad += te_lambda_bits(lam, te_mv_bits(c.y - mvp.y, c.x - mvp.x));
      if (sad < cmin) {
        cmin = sad;
        ydelta_hp = hm[i];
        xdelta_hp = hn[i];
      }
    }
    mv_opt.x = (int16_t)(mv_opt.x + xdelta_hp);
    mv_opt.y = (int16_t)(mv_opt.y + ydelta_hp);
    const int8_t *qm = te_qp_m, *qn = te_qp_n;
    for (int i = 1; i <= 8; i++) {
      c.y = (int16_t)(mv_opt.y + qm[i]);
      c.x = (int16_t)(mv_opt.x + qn[i]);
      te_mc_luma(S.rf, width, ref, rs, width, height, c, sign, enable_bipred);
      uint32_t sad = te_sad(org, os, S.rf, width, width, height);
      sad += (uint32_t)(int)(lam * (double)te_mv_bits(c.y - mvp.y, c.x - mvp.x) + 0.5);
      if (sad < cmin) {
        cmin = sad;
        ydelta_qp = qm[i];
        xdelta_qp = qn[i];
      }
    }
#if !defined(TE_HOST) && !defined(TE_ME_SEQ)
    }
#endif
  } else {  // fast bilinear approximation
    mv_ref.x = (int16_t)(mv_ref.x * s);
    mv_ref.y = (int16_t)(mv_ref.y * s);
    int spx, spy;
    uint32_t sad = te_fasthalf(org, os, ref + (mv_ref.x >> 2) + (mv_ref.y >> 2) * rs, rs, width, height, &spx, &spy);
    sad += te_lambda_bits(lam, te_mv_bits(mv_ref.y + s * spy - mvp.y, mv_ref.x + s * spx - mvp.x));
    if (sad < cmin) {
      cmin = sad;
      xdelta_hp = s * spx;
      ydelta_hp = s * spy;
    }
    spx = xdelta_hp;
    spy = ydelta_hp;
    mv_ref.x = (int16_t)(mv_opt.x + s * spx);
    mv_ref.y = (int16_t)(mv_opt.y + s * spy);
    mv_opt.x = (int16_t)(mv_opt.x + xdelta_hp);
    mv_opt.y = (int16_t)(mv_opt.y + ydelta_hp);
    sad = te_fastquarter(org, os, ref + s * (mv_ref.x >> 2) + s * (mv_ref.y >> 2) * rs, rs, width, height, &spx, &spy);
    sad += (uint32_t)(int)(lam * (double)te_mv_bits(mv_ref.y + s * spy - mvp.y, mv_ref.x + s * spx - mvp.x) + 0.5);
    if (sad < cmin) {
      cmin = sad;
      xdelta_qp = s * spx;
      ydelta_qp = s * spy;
    }
  }
  mv_opt.x = (int16_t)(mv_opt.x + xdelta_qp);
  mv_opt.y = (int16_t)(mv_opt.y + ydelta_qp);
  *mv = mv_opt;
  TE_TR(F.frame_num, 1, ypos, xpos, size | width << 8 | height << 16, r | sb.mc.num[r] << 8, TE_MIN(cmin, min_sad),
        (mv_opt.x & 0xffff) | (int)mv_opt.y << 16);
  return TE_MIN(cmin, min_sad);
}

// search_inter_prediction_params, enc/encode_block.c:1331-1396
TE_FN uint32_t te_search_inter(const TeFrame &F, TeSB &sb, int r, const uint8_t *org, int os,
                               const TeBlockInfo &bi, TeMv mvc, TeMv mvp, TeMv *mv_arr, int part, int sign,
                               int enable_bipred) {
  const int size = bi.size, ypos = bi.ypos, xpos = bi.xpos, rs = F.rsy;
  const uint8_t *ref_y = F.refy[r] + ypos * rs + xpos;
  TeMv mv, mvp2 = mvp;
  uint32_t sad = 0;
  if (part == 0) {
    sad += te_motion_estimate(F, sb, r, org, os, ref_y, size, size, size, &mv, mvc, mvp2, sign, xpos, ypos,
                              enable_bipred);
    mv_arr[0] = mv_arr[1] = mv_arr[2] = mv_arr[3] = mv;
  } else if (part == 1) {  // PART_HOR
    for (int index = 0; index < 4; index += 2) {
      const int py = index >> 1;
      sad += te_motion_estimate(F, sb, r, org + py * (size / 2) * os, os, ref_y + py * (size / 2) * rs, size, size,
                                size / 2, &mv, mvc, mvp2, sign, xpos, ypos, enable_bipred);
      mv_arr[index] = mv_arr[index + 1] = mv;
      mvp2 = mv_arr[0];
    }
  } else if (part == 2) {  // PART_VER
    for (int index = 0; index < 2; index++) {
      sad += te_motion_estimate(F, sb, r, org + index * (size / 2), os, ref_y + index * (size / 2), size, size / 2,
                                size, &mv, mvc, mvp2, sign, xpos, ypos, enable_bipred);
      mv_arr[index] = mv_arr[index + 2] = mv;
      mvp2 = mv_arr[0];
    }
  } else {  // PART_QUAD
    for (int index = 0; index < 4; index++) {
      const int px = index & 1, py = (index & 2) >> 1;
      sad += te_motion_estimate(F, sb, r, org + py * (size / 2) * os + px * (size / 2), os,
                                ref_y + py * (size / 2) * rs + px * (size / 2), size, size / 2, size / 2, &mv, mvc,
                                mvp2, sign, xpos, ypos, enable_bipred);
      mv_arr[index] = mv;
      mvp2 = mv_arr[0];
    }
  }
  return sad;
}

// copy_best_parameters, enc/encode_block.c:1983-2045.  The reconstructed
// block and the coefficient set of the candidate become the best by swapping
// buffer roles instead of copying (only components with cbp are ever read).
TE_FN void te_copy_best(TeBlockInfo &bi, TeParam &tmp) {
  TeParam &b = bi.bp;
  uint8_t *t = bi.rec_best;
  bi.rec_best = bi.rec;
  bi.rec = t;
  int16_t *c = b.coeff;
  b.coeff = tmp.coeff;
  tmp.coeff = c;
  b.pb_part = tmp.pb_part;
  b.skip_idx = tmp.skip_idx;
  b.mode = tmp.mode;
  b.cbp_y = tmp.cbp_y;
  b.cbp_u = tmp.cbp_u;
  b.cbp_v = tmp.cbp_v;
  b.tb_param = tmp.tb_param;
  b.tb_split = tmp.tb_split;
  if (tmp.mode == TE_SKIP || tmp.mode == TE_MERGE) {
    const TeInterPred &cp = tmp.mode == TE_SKIP ? bi.skip_c[tmp.skip_idx] : bi.merge_c[tmp.skip_idx];
    b.ref_idx0 = cp.ref_idx0;
    b.ref_idx1 = cp.ref_idx1;
    for (int i = 0; i < 4; i++) {
      b.mv0[i] = cp.mv0;
      b.mv1[i] = cp.mv1;
    }
    b.dir = cp.bipred_flag;
  } else if (tmp.mode == TE_INTRA) {
    b.ref_idx0 = b.ref_idx1 = 0;
    for (int i = 0; i < 4; i++) b.mv0[i].x = b.mv0[i].y = b.mv1[i].x = b.mv1[i].y = 0;
    b.dir = -1;
    b.intra_mode = tmp.intra_mode;
  } else {  // INTER / BIPRED
    b.ref_idx0 = tmp.ref_idx0;
    b.ref_idx1 = tmp.ref_idx1;
    for (int i = 0; i < 4; i++) {
      b.mv0[i] = tmp.mv0[i];
      b.mv1[i] = tmp.mv1[i];
    }
    b.dir = tmp.mode == TE_INTER ? 0 : 2;
  }
}

// copy_block_to_frame (:1802-1819) + copy_deblock_data (:1947-1981)
TE_FN void te_commit_block(const TeFrame &F, const TeBlockInfo &bi) {
  TE_P(TP_COMMIT);
  const int size = bi.size, bw = bi.bwidth, bh = bi.bheight, sC = size / 2;
  uint8_t *r = bi.rec;
  te_copy_rect(F.ry + bi.ypos * F.rsy + bi.xpos, F.rsy, r, size, bw, bh);
  const int cw = bw / 2, ch = bh / 2, oc = (bi.ypos / 2) * F.rsc + bi.xpos / 2;
  te_copy_rect(F.ru + oc, F.rsc, te_pu(r, size), sC, cw, ch);
  te_copy_rect(F.rv + oc, F.rsc, te_pv(r, size), sC, cw, ch);
  const TeParam &p = bi.bp;
  const int div = size / 8, bs = F.W / 4;
  const int nw = bw / 4, nh = bh / 4;
  for (int e = TE_LANE; e < nw * nh; e += TE_NL) {
    const int m = te_dv(e, nw), n = e - te_dv(e, nw) * nw;
    const int m0 = div > 0 ? m / div : 0, n0 = div > 0 ? n / div : 0, index = 2 * m0 + n0;
    TeCell c;
    c.ip.mv0 = p.mv0[index];
    c.ip.mv1 = p.mv1[index];
    c.ip.ref_idx0 = p.ref_idx0;
    c.ip.ref_idx1 = p.ref_idx1;
    c.ip.bipred_flag = p.dir;
    c.mode = (uint8_t)p.mode;
    c.size = (uint8_t)size;
    c.tb_split = (uint8_t)TE_MAX(0, p.tb_param);
    c.pb_part = (uint8_t)(p.mode == TE_INTER ? p.pb_part : 0);
    c.cbp_y = (uint8_t)p.cbp_y;
    c.cbp_u = (uint8_t)p.cbp_u;
    c.cbp_v = (uint8_t)p.cbp_v;
    c.rsv = 0;
    F.cells[(bi.ypos / 4 + m) * bs + bi.xpos / 4 + n] = c;
  }
  te_sync();
}

// search_bipred_prediction_params, enc/encode_block.c:2047-2202, me_mode 0
// (the iterative uni-pred search on the modified target org8)
TE_NOINL uint32_t te_search_bipred(const TeFrame &F_, TeSB &sb_, TeBlockInfo &bi_, int part,
                                   TeMv *mv_center, TeMv mvp, int *ref_idx0, int *ref_idx1, TeMv *mv_arr0,
                                   TeMv *mv_arr1) {
  const TeFrame &F = *te_lds(&F_);
  const TeScratch S = te_here();
  TeSB &sb = *te_lds(&sb_);
  TeBlockInfo &bi = *te_lds(&bi_);
  const int size = bi.size;
  const int num_iter = F.speed == 0 ? 2 : 1;
  int ref_idx = (F.frame_type == TE_B && F.interp_ref == 1) ? 1 : 0;
  int min_ref_idx0 = ref_idx, min_ref_idx1 = 0;
  TeMv m0[4], m1[4], mv_all[4];
  for (int i = 0; i < 4; i++) m0[i] = m1[i] = mvp;
  int min_sad = 1 << 30;
  const uint8_t *org = F.oy + bi.ypos * F.osy + bi.xpos;
  for (int n = 0; n < num_iter; n++) {
    const int stop = part == 0 ? 0 : 1;
    for (int list = 1; list >= stop; list--) {
      const TeMv mv = list ? m0[0] : m1[0];
      ref_idx = list ? min_ref_idx0 : min_ref_idx1;
      const int sign = F.ref_fnum[ref_idx] > F.frame_num;
      // the leg's vectors copied by value: a pointer select between the two
      // private arrays (list ? m0 : m1) is miscompiled by this hipcc for gfx950
      // (the m1 array is read for list 1 in the second iteration)
      TeMv leg[4];
      for (int i = 0; i < 4; i++) leg[i] = list ? m0[i] : m1[i];
      te_pred_yuv(F, ref_idx, S.pb, bi, leg, sign, 1, 1);
      for (int e = TE_LANE; e < size * size; e += TE_NL) {
        const int y = te_dv(e, size), x = e - te_dv(e, size) * size;
        S.org8[e] = (uint8_t)te_clip255(2 * (int)org[y * F.osy + x] - (int)S.pb[e]);
      }
      te_sync();
#if defined(THOR_ENC_TRACE)
      {
        uint32_t sp = 0, so = 0, sc = 0;
        for (int e = TE_LANE; e < size * size; e += TE_NL) {
          sp += S.pb[e] * (e + 1);
          so += S.org8[e] * (e + 1);
        }
        for (int e = TE_LANE; e < size * size / 2; e += TE_NL) sc += S.pb[size * size + e] * (e + 1);
        TE_TR(F.frame_num, 7, bi.ypos, bi.xpos, ref_idx | list << 4, te_sum(sp), te_sum(so),
              (m0[0].x & 0xffff) | (int)m0[0].y << 16);
        TE_TR(F.frame_num, 8, bi.ypos, bi.xpos, (m0[1].x & 0xffff) | (int)m0[1].y << 16,
              (m0[2].x & 0xffff) | (int)m0[2].y << 16, (m0[3].x & 0xffff) | (int)m0[3].y << 16, te_sum(sc));
        if (size == 8)
          for (int q = 0; q < 64; q += 16) {
            int w[4];
            for (int k = 0; k < 4; k++)
              w[k] = S.pb[q + 4 * k] | S.pb[q + 4 * k + 1] << 8 | S.pb[q + 4 * k + 2] << 16 | S.pb[q + 4 * k + 3] << 24;
            TE_TR(F.frame_num, 10, bi.ypos, bi.xpos, w[0], w[1], w[2], w[3]);
          }
        {
          const uint8_t *rp = F.refy[ref_idx] + bi.ypos * F.rsy + bi.xpos - 8;
          for (int q = 0; q < 2; q++) {
            int w[4];
            for (int k = 0; k < 4; k++)
              w[k] = rp[q * F.rsy + 4 * k] | rp[q * F.rsy + 4 * k + 1] << 8 | rp[q * F.rsy + 4 * k + 2] << 16 |
                     rp[q * F.rsy + 4 * k + 3] << 24;
            TE_TR(F.frame_num, 11, bi.ypos, bi.xpos, w[0], w[1], w[2], w[3]);
          }
        }
      }
#endif
      int ref_start, ref_end;
      if (F.frame_type == TE_P) {
        ref_start = 0;
        ref_end = F.num_ref - 1;
      } else {
        ref_start = ref_end = list ? 1 : 0;
        if (F.interp_ref) {
          ref_start += 1;
          ref_end += 1;
        }
      }
      for (int r = ref_start; r <= ref_end; r++) {
        const int sg = F.ref_fnum[r] > F.frame_num;
        const TeMv mvp2 = (F.frame_type == TE_B && list == 1) ? mv : mvp;
        const int sad = (int)te_search_inter(F, sb, r, S.org8, size, bi, mv_center[r], mvp2, mv_all, part, sg, 1);
        for (int i = 0; i < 4; i++) te_add_mvcand(sb.mc, r, mv_all[i]);
        if (sad < min_sad) {
          min_sad = sad;
          if (list) {
            min_ref_idx1 = r;
            for (int i = 0; i < 4; i++) m1[i] = mv_all[i];
          } else {
            min_ref_idx0 = r;
            for (int i = 0; i < 4; i++) m0[i] = mv_all[i];
          }
        }
      }
    }
  }
  TE_TR(F.frame_num, 4, bi.ypos, bi.xpos, size, min_ref_idx0 | min_ref_idx1 << 4, min_sad,
        (m0[0].x & 0xffff) | (int)m1[0].x << 16);
  *ref_idx0 = min_ref_idx0;
  *ref_idx1 = min_ref_idx1;
  for (int i = 0; i < 4; i++) {
    mv_arr0[i] = m0[i];
    mv_arr1[i] = m1[i];
  }
  return (uint32_t)(min_sad / 2);
}

// One candidate of motion_estimate_bi (enc/encode_block.c:1141-1160): the
// vector clipped for ref0's leg (sign 0), that clipped vector clipped again for
// ref1's negated leg; the truncating average of the two bi-table predictions
// against the original; *c returns the doubly clipped vector, which is what
// the MV cost and the result use.
TE_FN uint32_t te_bi_joint_sad(const TeFrame &F, const uint8_t *org, const uint8_t *p0, const uint8_t *p1,
                               int size, int ypos, int xpos, TeMv *c, TeMv mvp) {
  const TeScratch S = te_here();
  const TeMv c0 = te_clip_mv(*c, ypos, xpos, F.W, F.H, size, 0);
  te_mc_luma(S.pb0, size, p0, F.rsy, size, size, c0, 0, 2);
  const TeMv c1 = te_clip_mv(c0, ypos, xpos, F.W, F.H, size, 1);
  te_mc_luma(S.pb1, size, p1, F.rsy, size, size, c1, 1, 2);
  te_avg_rect(S.rf, size, S.pb0, size, S.pb1, size, size, size);
  te_sync();
  *c = c1;
  return te_sad(org, F.osy, S.rf, size, size, size) + te_lambda_bits(F.sqrt_lambda, te_mv_bits(c1.y - mvp.y, c1.x - mvp.x));
}

// search_bipred_prediction_params with me_mode 1 (enc/encode_block.c:2079-2111,
// B frames at speed 0): one vector for both legs, mv on ref_idx 0 (1 with an
// interpolated reference) and -mv on the next index, found by
// motion_estimate_bi (:1102-1216): a telescope from a 32-pel grid down to
// quarter pel around the rounded centre, then the candidate list.  That list
// is read as stored -- integer-rounded vectors used as quarter-pel ones -- and
// is first rewritten in place (slots num..3 zeroed, slot 4 = mvp, slot 5 = 0,
// :1171-1179), which later searches of the superblock see too.
TE_NOINL void te_search_bipred_joint(const TeFrame &F_, TeSB &sb_, const TeBlockInfo &bi_,
                                     const TeMv *mv_center, TeMv mvp, int *ref_idx0, int *ref_idx1, TeMv *mv_out) {
  const TeFrame &F = *te_lds(&F_);
  TeSB &sb = *te_lds(&sb_);
  const TeBlockInfo &bi = *te_lds(&bi_);
  const int size = bi.size, ypos = bi.ypos, xpos = bi.xpos;
  const int r0 = F.interp_ref ? 1 : 0, r1 = F.interp_ref ? 2 : 1;
  const uint8_t *org = F.oy + ypos * F.osy + xpos;
  const uint8_t *p0 = F.refy[r0] + ypos * F.rsy + xpos, *p1 = F.refy[r1] + ypos * F.rsy + xpos;
  uint32_t min_sad = TE_MAX_UINT32;
  TeMv mv_opt, mv_ref;
  mv_opt.x = mv_opt.y = 0;
  mv_ref.y = (int16_t)((((int)mv_center[r0].y + 2) >> 2) << 2);
  mv_ref.x = (int16_t)((((int)mv_center[r0].x + 2) >> 2) << 2);
  for (int step = 32; step > 0; step >>= 1) {
    for (int k = -step; k <= step; k += step)
      for (int l = -step; l <= step; l += step) {
        if (step < 32 && !k && !l) continue;
        if (step == 1) {
          const int vf = mv_ref.y & 3, hf = mv_ref.x & 3;
          const int ak = k < 0 ? -k : k, al = l < 0 ? -l : l;
          if (!vf && !hf) {
            if (ak != al) continue;  // integer pel: diagonal neighbours only
          } else if (vf == 2 && hf == 2) {
            continue;
          } else if (ak == al) {
            continue;
          }
        }
        TeMv c;
        c.y = (int16_t)(mv_ref.y + k);
        c.x = (int16_t)(mv_ref.x + l);
        const uint32_t sad = te_bi_joint_sad(F, org, p0, p1, size, ypos, xpos, &c, mvp);
        if (sad < min_sad) {
          min_sad = sad;
          mv_opt = c;
        }
      }
    mv_ref = mv_opt;
  }
  {  // the candidate list rewritten in place (every lane stores the same values)
    TeMv z;
    z.x = z.y = 0;
    for (int idx = sb.mc.num[r0]; idx < 4; idx++) sb.mc.mv[r0][idx] = z;
    sb.mc.mv[r0][4] = mvp;
    sb.mc.mv[r0][5] = z;
    te_sync();
  }
  for (int idx = 0; idx < 6; idx++) {  // ME_CANDIDATES, common/global.h:70
    TeMv c = sb.mc.mv[r0][idx];
    const uint32_t sad = te_bi_joint_sad(F, org, p0, p1, size, ypos, xpos, &c, mvp);
    if (sad < min_sad) {
      min_sad = sad;
      mv_opt = c;
    }
  }
  TE_TR(F.frame_num, 14, ypos, xpos, size, r0 | r1 << 4, min_sad, (mv_opt.x & 0xffff) | (int)mv_opt.y << 16);
  *ref_idx0 = r0;
  *ref_idx1 = r1;
  for (int i = 0; i < 4; i++) mv_out[i] = mv_opt;
}

// mode_decision_rdo, enc/encode_block.c:2204-2479
TE_NOINL uint32_t te_mode_decision(const TeFrame &F_, TeSB &sb_, TeBlockInfo &bi_, int16_t *tmp_coef) {
  const TeFrame &F = *te_lds(&F_);
  const TeScratch S = te_here();
  TeSB &sb = *te_lds(&sb_);
  TeBlockInfo &bi = *te_lds(&bi_);
  TE_P(TP_MODE);
  const int size = bi.size, ypos = bi.ypos, xpos = bi.xpos;
  TeBits &b = sb.bits;
  const int frame_type = F.frame_type;
  const int rectangular = bi.bwidth != size || bi.bheight != size;
  const int intra_inter_sad = F.speed > 0 && !F.sync;
  uint32_t min_cost = TE_MAX_UINT32, sad_intra = TE_MAX_UINT32, sad_inter = TE_MAX_UINT32, cost;
  int do_inter = 1, do_intra = 1;
  int intra_mode = TE_DC;
  const int pos_ref = b.pos;
  TeParam &tmp = *S.tmp;
  te_zero_words(&tmp, sizeof(TeParam));
  te_sync();
  tmp.coeff = tmp_coef;
  tmp.cs = bi.bp.cs;
  tmp.ts = bi.bp.ts;
  if (frame_type != TE_I) {  // skip candidates
    tmp.tb_param = 0;
    tmp.pb_part = 0;
    for (int k = 0; k < bi.num_skip; k++) {
      tmp.skip_idx = k;
      tmp.ref_idx0 = bi.skip_c[k].ref_idx0;
      tmp.ref_idx1 = bi.skip_c[k].ref_idx1;
      tmp.mv0[0] = bi.skip_c[k].mv0;
      tmp.mv1[0] = bi.skip_c[k].mv1;
      tmp.dir = bi.skip_c[k].bipred_flag;
      tmp.mode = TE_SKIP;
      const int nbits = te_encode_block(F, b, bi, tmp);
      cost = te_cost(F, bi, bi.rec, bi.bwidth, bi.bheight, nbits);
      if (cost < min_cost) {
        min_cost = cost;
        te_copy_best(bi, tmp);
        te_keep_best_bits(b, bi, nbits);
      }
    }
  }
  if (!rectangular && size <= 64) {
    if (frame_type != TE_I) {
      tmp.tb_param = 0;
      for (int k = 0; k < bi.num_merge; k++) {  // merge candidates
        tmp.skip_idx = k;
        tmp.ref_idx0 = bi.merge_c[k].ref_idx0;
        tmp.ref_idx1 = bi.merge_c[k].ref_idx1;
        tmp.mv0[0] = bi.merge_c[k].mv0;
        tmp.mv1[0] = bi.merge_c[k].mv1;
        tmp.dir = bi.merge_c[k].bipred_flag;
        tmp.mode = TE_MERGE;
        const int nbits = te_encode_block(F, b, bi, tmp);
        cost = te_cost(F, bi, bi.rec, size, size, nbits);
        if (cost < min_cost) {
          min_cost = cost;
          te_copy_best(bi, tmp);
          te_keep_best_bits(b, bi, nbits);
        }
      }
      if (intra_inter_sad) {
        sad_intra = (uint32_t)te_search_intra(F, bi, F.num_intra_modes, &intra_mode);
        sad_intra += (uint32_t)(int)(F.sqrt_lambda * (double)2 + 0.5);
      }
      // inter: ME per reference
      TeMv mv_all[4][4], mv_center[TE_MAX_REF], mvp;
      int min_idx, max_idx;
      if (sb.best_ref < 0 || F.speed < 2 || F.enable_bipred || F.sync) {
        min_idx = 0;
        max_idx = F.num_ref - 1;
      } else {
        min_idx = max_idx = sb.best_ref;
      }
      int32_t worst_cost = 0, best_cost = (int32_t)TE_MAX_UINT32;
      for (int r = min_idx; r <= max_idx; r++) {
        tmp.ref_idx0 = r;
        tmp.ref_idx1 = r;
        mvp = te_mv_pred(ypos, xpos, F.W, F.H, size, F.cells);
        te_add_mvcand(sb.mc, r, mvp);
        te_sync();
        bi.mvp = mvp;
        const int sign = F.ref_fnum[r] >= F.frame_num;
        mv_center[r] = mvp;
        sad_inter = TE_MAX_UINT32;
        for (int part = 0; part < bi.max_num_pb_part; part++) {
          const uint32_t sad = te_search_inter(F, sb, r, F.oy + ypos * F.osy + xpos, F.osy, bi, mv_center[r], mvp,
                                               mv_all[part], part, sign, F.enable_bipred);
          for (int i = 0; i < 4; i++) te_add_mvcand(sb.mc, r, mv_all[part][i]);
          te_sync();
          mv_center[r] = mv_all[0][0];
          sad_inter = TE_MIN(sad_inter, sad);
        }
        if (intra_inter_sad) {
          do_inter = sad_inter < sad_intra;
          if (sad_inter < sad_intra) do_intra = 0;
        }
        if (do_inter) {
          for (int part = 0; part < bi.max_num_pb_part; part++) {
            tmp.pb_part = part;
            for (int i = 0; i < 4; i++) tmp.mv0[i] = tmp.mv1[i] = mv_all[part][i];
            const int min_tb = F.speed < 1 ? -1 : 0, max_tb = bi.max_num_tb_part - 1;
            tmp.mode = TE_INTER;
            for (int tbp = min_tb; tbp <= max_tb; tbp++) {
              tmp.tb_param = tbp;
              const int nbits = te_encode_block(F, b, bi, tmp);
              cost = te_cost(F, bi, bi.rec, size, size, nbits);
              // worst_cost = max(worst_cost, cost), best_cost = min(best_cost, cost): int vs uint32 compares
              worst_cost = (uint32_t)worst_cost > cost ? worst_cost : (int32_t)cost;
              best_cost = (uint32_t)best_cost < cost ? best_cost : (int32_t)cost;
              if (cost < min_cost) {
                min_cost = cost;
                te_copy_best(bi, tmp);
                te_keep_best_bits(b, bi, nbits);
              }
            }
          }
        }
      }
      // one reference convincingly better: remember it (best_ref_idx is always 0, :2237, :2376-2377)
      if (worst_cost && (int32_t)((uint32_t)worst_cost * 3u) > (int32_t)((uint32_t)best_cost * 4u)) sb.best_ref = 0;
      if (F.num_ref > 1 && F.enable_bipred && do_inter) {  // bi-pred (BIPRED_PART 0: one partition)
        int r0, r1;
        TeMv a0[4], a1[4];
        const int part = 0;
        te_search_bipred(F, sb, bi, part, mv_center, mvp, &r0, &r1, a0, a1);
        tmp.pb_part = part;
        tmp.ref_idx0 = r0;
        tmp.ref_idx1 = r1;
        for (int i = 0; i < 4; i++) {
          tmp.mv0[i] = a0[i];
          tmp.mv1[i] = a1[i];
        }
        tmp.mode = TE_BIPRED;
        tmp.tb_param = 0;
        const int nbits = te_encode_block(F, b, bi, tmp);
        cost = te_cost(F, bi, bi.rec, size, size, nbits);
        if (cost < min_cost) {
          min_cost = cost;
          te_copy_best(bi, tmp);
          te_keep_best_bits(b, bi, nbits);
        }
        if (frame_type == TE_B && F.speed == 0) {  // joint mv0 = -mv1 search (me_mode 1, :2410-2426)
          TeMv aj[4];
          te_search_bipred_joint(F, sb, bi, mv_center, mvp, &r0, &r1, aj);
          tmp.pb_part = 0;
          tmp.ref_idx0 = r0;
          tmp.ref_idx1 = r1;
          for (int i = 0; i < 4; i++) tmp.mv0[i] = tmp.mv1[i] = aj[i];
          tmp.mode = TE_BIPRED;
          tmp.tb_param = 0;
          const int nbj = te_encode_block(F, b, bi, tmp);
          cost = te_cost(F, bi, bi.rec, size, size, nbj);
          if (cost < min_cost) {
            min_cost = cost;
            te_copy_best(bi, tmp);
            te_keep_best_bits(b, bi, nbj);
          }
        }
      }
    }
    if (do_intra) {
      const int max_tb = bi.max_num_tb_part - 1;
      if (F.intra_rdo) {
        uint32_t min_icost = TE_MAX_UINT32;
        int best_mode = TE_DC;
        for (int im = TE_DC; im < F.num_intra_modes; im++) {
          tmp.intra_mode = im;
          for (int tbp = 0; tbp <= max_tb; tbp++) {
            tmp.tb_param = tbp;
            tmp.mode = TE_INTRA;
            const int nbits = te_encode_block(F, b, bi, tmp);
            cost = te_cost(F, bi, bi.rec, size, size, nbits);
            if (cost < min_icost) {
              min_icost = cost;
              best_mode = im;
            }
          }
        }
        intra_mode = best_mode;
      } else {
        te_search_intra(F, bi, F.num_intra_modes, &intra_mode);
      }
      tmp.intra_mode = intra_mode;
      for (int tbp = 0; tbp <= max_tb; tbp++) {
        tmp.tb_param = tbp;
        tmp.mode = TE_INTRA;
        const int nbits = te_encode_block(F, b, bi, tmp);
        cost = te_cost(F, bi, bi.rec, size, size, nbits);
        if (cost < min_cost) {
          min_cost = cost;
          te_copy_best(bi, tmp);
          te_keep_best_bits(b, bi, nbits);
        }
      }
    }
  }
  te_rewind(b, pos_ref);  // rewind (:2476)
  TE_TR(F.frame_num, 5, ypos, xpos, size, min_cost, bi.bp.mode, sad_intra);
  return min_cost;
}

// mode_decision_rdo of an I frame (enc/encode_block.c:2204-2479 with only the
// intra branch live: an I-frame CU is never rectangular, encode_this).  Inlined
// into process_block: te_mode_decision's body, sized for the P / B candidates,
// saves ~110 callee-saved VGPRs through scratch per call.
TE_FN uint32_t te_mode_decision_intra(const TeFrame &F_, TeBlockInfo &bi_, TeBits &b_, int16_t *tmp_coef) {
  const TeFrame &F = *te_lds(&F_);
  const TeScratch S = te_here();
  TeBlockInfo &bi = *te_lds(&bi_);
  TeBits &b = *te_lds(&b_);
  TE_P(TP_MODE);
  const int size = bi.size;
  uint32_t min_cost = TE_MAX_UINT32, cost;
  int intra_mode = TE_DC;
  const int pos_ref = b.pos;
  TeParam &tmp = *S.tmp;
  te_zero_words(&tmp, sizeof(TeParam));
  te_sync();
  tmp.coeff = tmp_coef;
  tmp.cs = bi.bp.cs;
  tmp.ts = bi.bp.ts;
  // intra_rdo: every (mode, tb split) candidate for the mode (:2446-2462), then the
  // chosen mode's tb splits against the block's best (:2463-2474) -- one loop,
  // so the encode has a single call site
  const int ntb = bi.max_num_tb_part, nrdo = F.intra_rdo ? F.num_intra_modes * ntb : 0;
  uint32_t min_icost = TE_MAX_UINT32;
  int best_mode = TE_DC;
#ifdef TE_MDI_TWO
  if (F.intra_rdo) {
    for (int im = TE_DC; im < F.num_intra_modes; im++) {
      tmp.intra_mode = im;
      for (int tbp = 0; tbp < ntb; tbp++) {
        tmp.tb_param = tbp;
        tmp.mode = TE_INTRA;
        const int nbits = TE_ENCODE_I(F, b, bi, tmp);
        cost = te_cost(F, bi, bi.rec, size, size, nbits);
        if (cost < min_icost) {
          min_icost = cost;
          best_mode = im;
        }
      }
    }
    intra_mode = best_mode;
  } else {
    te_search_intra(F, bi, F.num_intra_modes, &intra_mode);
  }
  tmp.intra_mode = intra_mode;
  for (int tbp = 0; tbp < ntb; tbp++) {
    tmp.tb_param = tbp;
    tmp.mode = TE_INTRA;
    const int nbits = TE_ENCODE_I(F, b, bi, tmp);
    cost = te_cost(F, bi, bi.rec, size, size, nbits);
    if (cost < min_cost) {
      min_cost = cost;
      te_copy_best(bi, tmp);
      te_keep_best_bits(b, bi, nbits);
    }
  }
  (void)nrdo;
#else
  if (!F.intra_rdo) te_search_intra(F, bi, F.num_intra_modes, &intra_mode);
  for (int st = 0; st < nrdo + ntb; st++) {
    const bool rdo = st < nrdo;
    if (st == nrdo && F.intra_rdo) intra_mode = best_mode;
    const int im = rdo ? TE_DC + st / ntb : intra_mode;
    tmp.intra_mode = im;
    tmp.tb_param = rdo ? st - (st / ntb) * ntb : st - nrdo;
    tmp.mode = TE_INTRA;
    const int nbits = TE_ENCODE_I(F, b, bi, tmp);
    cost = te_cost(F, bi, bi.rec, size, size, nbits);
    if (rdo) {
      if (cost < min_icost) {
        min_icost = cost;
        best_mode = im;
      }
    } else if (cost < min_cost) {
      min_cost = cost;
      te_copy_best(bi, tmp);
      te_keep_best_bits(b, bi, nbits);
    }
  }
#endif
  te_rewind(b, pos_ref);  // rewind (:2476)
  TE_TR(F.frame_num, 5, bi.ypos, bi.xpos, size, min_cost, bi.bp.mode, TE_MAX_UINT32);
  return min_cost;
}

// ---- early skip (enc/encode_block.c:2481-2783) -------------------------------
// check_early_skip_sub_block (luma, :2505-2538): 2x2-average + (N/2)-point
// transform against half the threshold (N = 4: plain 4-point transform).
TE_FN int te_es_luma(const uint8_t *org, int os, int size, const uint8_t *pb, int thr) {
  const TeScratch S = te_here();
  TeTx &X = *S.tx;
  int n = size;
  if (size > 4) {
    const int s2 = size / 2, h2 = s2 / 2;  // two outputs per lane: 4 columns x 2 rows
    for (int g = TE_LANE; g < s2 * h2; g += TE_NL) {
      const int i = te_dv(g, h2), j = (g - i * h2) * 2;
      const int i2 = 2 * i, j2 = 2 * j;
      const uint32_t o0 = te_ld4(org + i2 * os + j2), o1 = te_ld4(org + (i2 + 1) * os + j2);
      const uint32_t p0 = te_ld4(pb + i2 * size + j2), p1 = te_ld4(pb + (i2 + 1) * size + j2);
      for (int k = 0; k < 2; k++) {
        const int a = te_b(o0, 2 * k) - te_b(p0, 2 * k), b = te_b(o0, 2 * k + 1) - te_b(p0, 2 * k + 1);
        const int c = te_b(o1, 2 * k) - te_b(p1, 2 * k), d = te_b(o1, 2 * k + 1) - te_b(p1, 2 * k + 1);
        X.R[i * s2 + j + k] = (int16_t)((a + b + c + d + 2) >> 2);
      }
    }
    n = s2;
  } else {
    for (int e = TE_LANE; e < 16; e += TE_NL) {
      const int i = e >> 2, j = e & 3;
      X.R[e] = (int16_t)((int)org[i * os + j] - pb[i * 4 + j]);
    }
  }
  te_sync();
  te_fwd_tx(X, n, 0);
  int flag = 0;
  for (int e = TE_LANE; e < n * n; e += TE_NL) flag |= te_abs(X.C[e]) > thr;
  return te_any(flag);
}
#if !defined(TE_HOST)
// The early-skip checks fused with their uni-pred prediction (device): the
// prediction is never stored.  Each lane computes 4x4 MC outputs (te_mc_luma's
// / te_mc_chroma's unit form, common/inter_prediction.c:72-180) with the
// original's rows loaded in the same round trip, and reduces them straight to
// what the check reads -- the 2x2-averaged residual (luma) or the column sums
// (chroma) -- so one memory round trip and no prediction-buffer LDS round trip
// per check.
TE_FN void te_mc_luma_unit(const uint8_t *r, int rs, int i0, int j, int fx, int fy, int bipred, int o[4][4]) {
  if (fx == 2 && fy == 2) {  // rows -1..5, columns -1..6, :145-157
    uint32_t lo[7], hi[7];
#pragma unroll
    for (int q = 0; q < 7; q++) {
      const uint8_t *p = r + (i0 - 1 + q) * rs + j - 1;
      lo[q] = te_ld4(p);
      hi[q] = te_ld4(p + 4);
    }
    int c[7][8];
#pragma unroll
    for (int q = 0; q < 7; q++)
#pragma unroll
      for (int k = 0; k < 4; k++) {
        c[q][k] = te_b(lo[q], k);
        c[q][k + 4] = te_b(hi[q], k);
      }
#pragma unroll
    for (int y = 0; y < 4; y++)
#pragma unroll
      for (int x = 0; x < 4; x++) {
        const int k = x + 1;
        const int *a = c[y], *b = c[y + 1], *d = c[y + 2], *e = c[y + 3];
        const int v = a[k] + a[k + 1] + b[k - 1] + 2 * b[k] + 2 * b[k + 1] + b[k + 2] + d[k - 1] + 2 * d[k] +
                      2 * d[k + 1] + d[k + 2] + e[k] + e[k + 1];
        o[y][x] = te_clip255((v + 8) >> 4);
      }
    return;
  }
  if (!fx && !fy) {  // integer vector: a copy
#pragma unroll
    for (int y = 0; y < 4; y++) {
      const uint32_t v = te_ld4(r + (i0 + y) * rs + j);
#pragma unroll
      for (int x = 0; x < 4; x++) o[y][x] = te_b(v, x);
    }
    return;
  }
  // separable 6-tap (fraction 0: the identity taps {0, 0, 64, 0, 0, 0}, exact), :160-178
  const int8_t *fv = (bipred ? te_luma_bi : te_luma_uni)[fy];
  const int8_t *fh = (bipred ? te_luma_bi : te_luma_uni)[fx];
  uint32_t d[9][3];
#pragma unroll
  for (int q = 0; q < 9; q++) {
    const uint8_t *p = r + (i0 - 2 + q) * rs + j - 2;
    d[q][0] = te_ld4(p);
    d[q][1] = te_ld4(p + 4);
    d[q][2] = te_ld4(p + 8);
  }
  int hk[9][4];
#pragma unroll
  for (int q = 0; q < 9; q++) {
    int c[12];
#pragma unroll
    for (int b = 0; b < 4; b++) {
      c[b] = te_b(d[q][0], b);
      c[b + 4] = te_b(d[q][1], b);
      c[b + 8] = te_b(d[q][2], b);
    }
#pragma unroll
    for (int x = 0; x < 4; x++) {
      int a = 0;
#pragma unroll
      for (int m = 0; m < 6; m++) a += fh[m] * c[x + m];
      hk[q][x] = a;
    }
  }
#pragma unroll
  for (int y = 0; y < 4; y++)
#pragma unroll
    for (int x = 0; x < 4; x++) {
      int a = 0;
#pragma unroll
      for (int k = 0; k < 6; k++) a += fv[k] * hk[y + k][x];
      o[y][x] = te_clip255((a + 2048) >> 12);
    }
}
// te_mc_chroma's 4x4 unit (fraction 0 included: the identity taps {0, 64, 0, 0} are exact)
TE_FN void te_mc_chroma_unit(const uint8_t *r, int rs, int i0, int j, int fx, int fy, int o[4][4]) {
  const int8_t *fh = te_chroma_f[fx], *fv = te_chroma_f[fy];
  uint32_t lo[7], hi[7];
#pragma unroll
  for (int q = 0; q < 7; q++) {
    const uint8_t *p = r + (i0 - 1 + q) * rs + j - 1;
    lo[q] = te_ld4(p);
    hi[q] = te_ld4(p + 4);
  }
  int hk[7][4];
#pragma unroll
  for (int q = 0; q < 7; q++) {
    int c[8];
#pragma unroll
    for (int b = 0; b < 4; b++) {
      c[b] = te_b(lo[q], b);
      c[b + 4] = te_b(hi[q], b);
    }
#pragma unroll
    for (int x = 0; x < 4; x++) {
      int a = 0;
#pragma unroll
      for (int k = 0; k < 4; k++) a += fh[k] * c[x + k];
      hk[q][x] = a;
    }
  }
#pragma unroll
  for (int y = 0; y < 4; y++)
#pragma unroll
    for (int x = 0; x < 4; x++) {
      int a = 0;
#pragma unroll
      for (int m = 0; m < 4; m++) a += fv[m] * hk[y + m][x];
      o[y][x] = te_clip255((a + 2048) >> 12);
    }
}
// te_mc_luma (sub-block origin `ref`, vector mv / sign) + te_es_luma, size 8..32
TE_FN int te_es_luma_mc(const uint8_t *ref, int rs, TeMv mv, int sign, int bipred, const uint8_t *org, int os,
                        int size, int thr) {
  const TeScratch S = te_here();
  TeTx &X = *S.tx;
  const int mx = sign ? -mv.x : mv.x, my = sign ? -mv.y : mv.y;
  const int fy = my & 3, fx = mx & 3;
  const uint8_t *r = ref + (my >> 2) * rs + (mx >> 2);
  const int w4 = size >> 2, s2 = size >> 1;
  if (TE_LANE < w4 * w4) {
    const int u = TE_LANE, i0 = te_dv(u, w4) * 4, j = (u - te_dv(u, w4) * w4) * 4;
    uint32_t ov[4];
#pragma unroll
    for (int y = 0; y < 4; y++) ov[y] = te_ld4(org + (i0 + y) * os + j);
    int o[4][4];
    te_mc_luma_unit(r, rs, i0, j, fx, fy, bipred, o);
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
      for (int b = 0; b < 2; b++) {
        const int y = 2 * a, x = 2 * b;
        const int s = te_b(ov[y], x) - o[y][x] + te_b(ov[y], x + 1) - o[y][x + 1] + te_b(ov[y + 1], x) - o[y + 1][x] +
                      te_b(ov[y + 1], x + 1) - o[y + 1][x + 1];
        X.R[(i0 / 2 + a) * s2 + j / 2 + b] = (int16_t)((s + 2) >> 2);
      }
  }
  te_sync();
  te_fwd_tx(X, s2, 0);
  int flag = 0;
  for (int e = TE_LANE; e < s2 * s2; e += TE_NL) flag |= te_abs(X.C[e]) > thr;
  return te_any(flag);
}
// te_mc_chroma + te_es_chroma (size 4, 8 or 16; only the pixels the check reads)
TE_FN int te_es_chroma_mc(const uint8_t *ref, int rs, TeMv mv, int sign, const uint8_t *org, int os, int size,
                          int thr) {
  const int mx = sign ? -mv.x : mv.x, my = sign ? -mv.y : mv.y;
  const int fy = my & 7, fx = mx & 7;
  const uint8_t *r = ref + (my >> 3) * rs + (mx >> 3);
  int flag = 0;
  const int nu = size == 8 ? 4 : 1;  // 8x8: every column over 8 rows; else the top-left 4x4, column pairs
  int cs[4] = {0, 0, 0, 0};          // the lane's unit: column sums of org - pred over its 4 rows
  if (TE_LANE < nu) {
    const int i0 = (TE_LANE >> 1) * 4, j = (TE_LANE & 1) * 4;
    uint32_t ov[4];
#pragma unroll
    for (int y = 0; y < 4; y++) ov[y] = te_ld4(org + (i0 + y) * os + j);
    int o[4][4];
    te_mc_chroma_unit(r, rs, i0, j, fx, fy, o);
#pragma unroll
    for (int x = 0; x < 4; x++)
#pragma unroll
      for (int y = 0; y < 4; y++) cs[x] += te_b(ov[y], x) - o[y][x];
  }
  if (size == 8) {  // the bottom units' sums join the top ones' (lane ^ 2 within a quad)
#pragma unroll
    for (int x = 0; x < 4; x++) {
      const int tot = cs[x] + TE_DPP(cs[x], 0x4E);
      if (TE_LANE < 2) flag |= te_wrap16(tot) > (int)(int16_t)thr;
    }
  } else if (TE_LANE == 0) {
    flag = (cs[0] + cs[1] > thr) | (cs[2] + cs[3] > thr);
  }
  return te_any(flag);
}
#endif

// check_early_skip_sub_blockC (:2540-2611): column sums of the residual
// (8x8: all 8 columns over 8 rows; other sizes: the top-left 4x4 only, column
// pairs) against the threshold
TE_FN int te_es_chroma(const uint8_t *org, int os, int size, const uint8_t *pb, int thr) {
  int flag = 0;
  if (size == 8) {
    for (int j = TE_LANE; j < 8; j += TE_NL) {
      int s = 0;
      for (int i = 0; i < 8; i++) s += (int)org[i * os + j] - pb[i * 8 + j];
      flag |= te_wrap16(s) > (int)(int16_t)thr;
    }
  } else {
    for (int jp = TE_LANE; jp < 2; jp += TE_NL) {
      int s = 0;
      for (int i = 0; i < 4; i++)
        for (int k = 0; k < 2; k++) s += (int)org[i * os + 2 * jp + k] - pb[i * size + 2 * jp + k];
      flag |= s > thr;
    }
  }
  return te_any(flag);
}

// check_early_skip_block, :2613-2741.  Returns 1 when every sub-block is insignificant.
#ifdef TE_ES_INLINE
TE_FN
#else
TE_NOINL
#endif
int te_check_early_skip(const TeFrame &F_, const TeBlockInfo &bi_, const TeParam &p_) {
  const TeFrame &F = *te_lds(&F_);
  const TeScratch S = te_here();
  const TeBlockInfo &bi = *te_lds(&bi_);
  const TeParam &p = *te_lds(&p_);
  TE_P(TP_ES_CHECK);
  const int size = bi.size, ypos = bi.ypos, xpos = bi.xpos, size0 = TE_MIN(size, 32);
  const int qpY = F.qp + bi.delta_qp, qpC = te_chroma_qp(qpY);
  const int *T = F.es_thr + ((F.speed > 1 && size == 64) ? 52 * 4 : 0);  // 1.3x threshold for 64x64 at speed 2
  const int thr_y = T[qpY * 4 + (size0 == 8 ? 0 : (size0 == 16 ? 1 : 2))], thr_c = T[qpC * 4 + 3];
  const int bip = F.enable_bipred, s0c = size0 / 2;
  uint8_t *pb = S.pb, *pb0 = S.pb0, *pb1 = S.pb1;
  for (int i = 0; i < size; i += size0)
    for (int j = 0; j < size; j += size0) {
      const uint8_t *oY = F.oy + (ypos + i) * F.osy + xpos + j;
      const uint8_t *oU = F.ou + ((ypos + i) / 2) * F.osc + (xpos + j) / 2;
      const uint8_t *oV = F.ov + ((ypos + i) / 2) * F.osc + (xpos + j) / 2;
      const int ry = (ypos + i) * F.rsy + xpos + j, rc = ((ypos + i) / 2) * F.rsc + (xpos + j) / 2;
      if (p.dir == 2) {
        const int sg0 = F.ref_fnum[p.ref_idx0] >= F.frame_num, sg1 = F.ref_fnum[p.ref_idx1] >= F.frame_num;
        TeMv m0 = te_clip_mv(p.mv0[0], ypos, xpos, F.W, F.H, size0, sg0);
        TeMv m1 = te_clip_mv(p.mv1[0], ypos, xpos, F.W, F.H, size0, sg1);
        te_mc_luma(pb0, size0, F.refy[p.ref_idx0] + ry, F.rsy, size0, size0, m0, sg0, bip);
        te_mc_luma(pb1, size0, F.refy[p.ref_idx1] + ry, F.rsy, size0, size0, m1, sg1, bip);
        te_avg_rect(pb, size0, pb0, size0, pb1, size0, size0, size0);
        te_sync();
        if (te_es_luma(oY, F.osy, size0, pb, thr_y)) return 0;
        // chroma legs use the unclipped vectors (:2680-2702)
        for (int c = 0; c < 2; c++) {
          te_mc_chroma(pb0, s0c, (c ? F.refv : F.refu)[p.ref_idx0] + rc, F.rsc, s0c, s0c, p.mv0[0], sg0);
          te_mc_chroma(pb1, s0c, (c ? F.refv : F.refu)[p.ref_idx1] + rc, F.rsc, s0c, s0c, p.mv1[0], sg1);
          te_avg_rect(pb, s0c, pb0, s0c, pb1, s0c, s0c, s0c);
          te_sync();
          if (te_es_chroma(c ? oV : oU, F.osc, s0c, pb, thr_c)) return 0;
        }
      } else {
        const int sign = F.ref_fnum[p.ref_idx0] > F.frame_num;
        // the vector is clipped in place for every sub-block (:2722), and the clipped one serves chroma
        TeMv mv = te_clip_mv(p.mv0[0], ypos, xpos, F.W, F.H, size0, sign);
#if !defined(TE_HOST)
        if (te_es_luma_mc(F.refy[p.ref_idx0] + ry, F.rsy, mv, sign, bip, oY, F.osy, size0, thr_y)) return 0;
        if (te_es_chroma_mc(F.refu[p.ref_idx0] + rc, F.rsc, mv, sign, oU, F.osc, s0c, thr_c)) return 0;
        if (te_es_chroma_mc(F.refv[p.ref_idx0] + rc, F.rsc, mv, sign, oV, F.osc, s0c, thr_c)) return 0;
        continue;
#endif
        te_mc_luma(pb, size0, F.refy[p.ref_idx0] + ry, F.rsy, size0, size0, mv, sign, bip);
        if (te_es_luma(oY, F.osy, size0, pb, thr_y)) return 0;
        te_mc_chroma(pb, s0c, F.refu[p.ref_idx0] + rc, F.rsc, s0c, s0c, mv, sign);
        if (te_es_chroma(oU, F.osc, s0c, pb, thr_c)) return 0;
        te_mc_chroma(pb, s0c, F.refv[p.ref_idx0] + rc, F.rsc, s0c, s0c, mv, sign);
        if (te_es_chroma(oV, F.osc, s0c, pb, thr_c)) return 0;
      }
    }
  return 1;
}

// search_early_skip_candidates, :2743-2783
TE_NOINL int te_search_early_skip(const TeFrame &F_, TeSB &sb_, TeBlockInfo &bi_, int16_t *tmp_coef,
                                  uint32_t *best_cost) {
  const TeFrame &F = *te_lds(&F_);
  const TeScratch S = te_here();
  TeSB &sb = *te_lds(&sb_);
  TeBlockInfo &bi = *te_lds(&bi_);
  TE_P(TP_ES_SEARCH);
  uint32_t min_cost = TE_MAX_UINT32;
  int early = 0;
  TeParam &tmp = *S.tmp;
  te_zero_words(&tmp, sizeof(TeParam));
  te_sync();
  tmp.coeff = tmp_coef;
  tmp.cs = bi.bp.cs;
  tmp.ts = bi.bp.ts;
  for (int k = 0; k < bi.num_skip; k++) {
    tmp.tb_param = 0;
    tmp.skip_idx = k;
    tmp.ref_idx0 = bi.skip_c[k].ref_idx0;
    tmp.ref_idx1 = bi.skip_c[k].ref_idx1;
    tmp.mv0[0] = bi.skip_c[k].mv0;
    tmp.mv1[0] = bi.skip_c[k].mv1;
    tmp.dir = bi.skip_c[k].bipred_flag;
    if (te_check_early_skip(F, bi, tmp)) {
      early = 1;
      tmp.mode = TE_SKIP;
      const int nbits = te_encode_block(F, sb.bits, bi, tmp);
      const uint32_t cost = te_cost(F, bi, bi.rec, bi.size, bi.size, nbits);
      if (cost < min_cost) {
        min_cost = cost;
        te_copy_best(bi, tmp);
        te_keep_best_bits(sb.bits, bi, nbits);
      }
    }
  }
  *best_cost = min_cost;
  return early;
}

// ---- process_block, enc/encode_block.c:2787-3033 ----------------------------
// Template over the CU size: the quadtree recursion unrolls at compile time
// (64 -> 32 -> 16 -> 8); level L = log2(64 / SIZE) owns TeScratch::lv[L].
template <int SIZE>
TE_NOINL uint32_t te_process_block(const TeFrame &F_, TeSB &sb_, int ypos, int xpos, int qp);
template <int SIZE>
TE_FN uint32_t te_process_block_b(const TeFrame &F_, TeSB &sb_, int ypos, int xpos, int qp);
// A quadrant of the recursion: the 8x8 and 16x16 levels (80 of an SB's 85
// CUs) inlined into the 32x32 one -- two call frames fewer per small CU
// (-3 % and -2.6 % of a 4K I frame at 240 streams); the 32 and
// 64 levels stay calls.
template <int NS>
TE_FN uint32_t te_process_quad(const TeFrame &F, TeSB &sb, int ypos, int xpos, int qp) {
  if constexpr (NS == 8 || NS == 16) return te_process_block_b<NS>(F, sb, ypos, xpos, qp);
  return te_process_block<NS>(F, sb, ypos, xpos, qp);
}
template <int SIZE>
TE_NOINL uint32_t te_process_block(const TeFrame &F_, TeSB &sb_, int ypos, int xpos, int qp) {
  return te_process_block_b<SIZE>(F_, sb_, ypos, xpos, qp);
}
template <int SIZE>
TE_FN uint32_t te_process_block_b(const TeFrame &F_, TeSB &sb_, int ypos, int xpos, int qp) {
  const TeFrame &F = *te_lds(&F_);
  const TeScratch S = te_here();
  TeSB &sb = *te_lds(&sb_);
  constexpr int L = SIZE == 64 ? 0 : (SIZE == 32 ? 1 : (SIZE == 16 ? 2 : 3));
  const int W = F.W, H = F.H, ft = F.frame_type;
  if (ypos >= H || xpos >= W) return 0;
  const int encode_this = ypos + SIZE <= H && xpos + SIZE <= W;
  const int encode_smaller = SIZE > 8 * (encode_this && ft != TE_I && !F.sync && F.speed > 0 ? 2 : 1);
  const int top_down = !encode_smaller && SIZE > 8;
  const int encode_rect = !encode_this && ft != TE_I;
  if (!encode_this && !encode_smaller) return 0;
  uint32_t cost_small = 1u << 28, cost = 1u << 28;
  TeBits &b = sb.bits;
  const int pos_ref = b.pos;
  TeLevel &lv = S.lv[L];
  TeBlockInfo &bi = S.bi[L];
  te_zero_words(&bi, sizeof(TeBlockInfo));
  te_sync();
  bi.ctx = te_block_ctx(ypos, xpos, H, W, SIZE, F.cells, F.use_block_contexts);
  bi.size = SIZE;
  bi.bwidth = TE_MIN(SIZE, W - xpos);
  bi.bheight = TE_MIN(SIZE, H - ypos);
  bi.ypos = ypos;
  bi.xpos = xpos;
  bi.max_num_tb_part = F.enable_tb_split == 1 ? 2 : 1;
  bi.max_num_pb_part = F.enable_pb_split ? 4 : 1;
  bi.delta_qp = qp - F.qp;
  // this level's buffers: LDS for the small levels (TeSmallLv), the worker's global scratch otherwise
  TeSmallLv &sl = *S.sl;
  int16_t *const cb0 = SIZE == 16 ? sl.cf2[0] : (SIZE == 8 ? sl.cf3[0] : lv.cbuf[0]);
  int16_t *const cb1 = SIZE == 16 ? sl.cf2[1] : (SIZE == 8 ? sl.cf3[1] : lv.cbuf[1]);
  bi.rec = SIZE == 32 ? sl.rec1[0] : (SIZE == 16 ? sl.rec2[0] : (SIZE == 8 ? sl.rec3[0] : lv.rbuf[0]));
  bi.rec_best = SIZE == 32 ? sl.rec1[1] : (SIZE == 16 ? sl.rec2[1] : (SIZE == 8 ? sl.rec3[1] : lv.rbuf[1]));
  bi.best_bits = SIZE == 16 ? sl.bb2 : (SIZE == 8 ? sl.bb3 : lv.bbits);
  bi.best_cap = SIZE == 16 ? 128 : (SIZE == 8 ? 64 : TE_BEST_WORDS);
  bi.best_nbits = -1;
  bi.bp.coeff = cb0;
  bi.bp.cs = TE_CS(SIZE);
  bi.bp.ts = TE_TS(SIZE);
  int16_t *tmp_coef = cb1;
  if (ft != TE_I) {
    bi.num_skip = te_mv_skip(ypos, xpos, W, H, SIZE, F.cells, bi.skip_c);
    bi.num_merge = te_mv_skip(ypos, xpos, W, H, SIZE, F.cells, bi.merge_c);
  }
  if (encode_this && ft != TE_I && F.early_skip_thr > 0.0f) {
    bi.final_encode = 2;
    uint32_t es_cost = 0;
    const int early = te_search_early_skip(F, sb, bi, tmp_coef, &es_cost);
    te_rewind(b, pos_ref);
    if (early) {
      bi.final_encode = 3;
      // the best candidate (a SKIP, tb_param 0) is re-used as it was costed: its reconstruction and bits,
      // hence its cost_calc (:2966-2967) -- recomputed only if the parameters had to change
      const int same = bi.bp.mode == TE_SKIP && bi.bp.tb_param == 0 && !F.enable_tb_split;
      if (!same) bi.best_nbits = -1;
      bi.bp.mode = TE_SKIP;
      bi.bp.tb_param = 0;
      const int nbit = te_encode_final(F, b, bi);
      cost = same ? es_cost : te_cost(F, bi, bi.rec, SIZE, SIZE, nbit);
      te_commit_block(F, bi);
      return cost;
    }
  }
  if constexpr (SIZE > 8) {
    if (encode_smaller) {
      constexpr int NS = SIZE / 2;
      if (encode_this) te_write_super_mode(b, F, bi, 0, 0, 1);
      else if (ft != TE_I) te_put(b, 1, 0);
      if (SIZE == 64 && F.max_delta_qp) te_write_delta_qp(b, bi.delta_qp);
      cost_small = 0;
      for (int q = 0; q < 4; q++)  // (0,0) (NS,0) (0,NS) (NS,NS): the reference's order
        cost_small += te_process_quad<NS>(F, sb, ypos + (q & 1) * NS, xpos + (q >> 1) * NS, qp);
    }
  }
  if (encode_this) {
    bi.final_encode = 0;
    // the tmp coefficient set: whichever of cbuf[0..1] the best does not hold
    int16_t *const tc = bi.bp.coeff == cb0 ? cb1 : cb0;
    cost = ft == TE_I ? te_mode_decision_intra(F, bi, b, tc) : te_mode_decision(F, sb, bi, tc);
    const int me_threshold = SIZE * SIZE * te_iq8[qp] / 8;
    if constexpr (SIZE > 8) {
      if (top_down && cost > (uint32_t)me_threshold) {
        constexpr int NS = SIZE / 2;
        te_write_super_mode(b, F, bi, 0, 0, 1);
        cost_small = 0;
        for (int q = 0; q < 4; q++)
          cost_small += te_process_quad<NS>(F, sb, ypos + (q & 1) * NS, xpos + (q >> 1) * NS, qp);
      }
    }
    if (cost <= cost_small) {
      te_rewind(b, pos_ref);
      bi.final_encode = 1;
      te_encode_final(F, b, bi);
      te_commit_block(F, bi);
    }
  } else if (encode_rect) {
    bi.final_encode = 0;
    cost = te_mode_decision(F, sb, bi, bi.bp.coeff == cb0 ? cb1 : cb0);
    if (cost <= cost_small) {
      te_rewind(b, pos_ref);
      bi.final_encode = 1;
      if (bi.bp.mode != TE_SKIP || bi.bp.tb_param != 0) bi.best_nbits = -1;
      bi.bp.mode = TE_SKIP;
      bi.bp.tb_param = 0;
      te_encode_final(F, b, bi);
      te_commit_block(F, bi);
    }
  }
  return TE_MIN(cost, cost_small);
}

// One superblock as encode_frame runs it (enc/encode_frame.c:114-146): reset
// the ME candidate lists, then process_block(64) -- with the delta-qp RD
// search when max_delta_qp is set (trials leave their candidates behind, as
// there).  Returns the SB's bit count in sb.bits.
// costs (optional, nullptr: off): the returned cost of each top-level
// process_block call of the SB -- every delta-QP trial in order, then the final
// encode (enc/encode_frame.c:133-145) -- for the per-SB RD-cost parity check
// (thor_enc_sb_costs, tests/golden/rd_costs.npz).
TE_FN void te_encode_sb(const TeFrame &F, TeSB &sb, int k, int l, int32_t *costs = nullptr) {
  TE_P(TP_SB);
  const int ypos = k * 64, xpos = l * 64;
  for (int r = 0; r < F.num_ref; r++) {
    sb.mc.num[r] = 0;
    sb.mc.mask[r] = 0;
  }
  sb.best_ref = -1;
  te_bits_start(sb.bits);
  if (F.max_delta_qp) {
    int min_cost = 1 << 30, best_qp = F.qp;
    int t = 0;
    for (int q = F.qp - F.max_delta_qp; q <= F.qp + F.max_delta_qp; q += F.delta_qp_step, t++) {
      const int cost = (int)te_process_block<64>(F, sb, ypos, xpos, q);
      TE_TR(F.frame_num, 6, ypos, xpos, q, cost, 0, 0);
      if (costs && TE_LANE == 0) costs[t] = cost;
      if (cost < min_cost) {
        min_cost = cost;
        best_qp = q;
      }
    }
    te_rewind(sb.bits, 0);
    const int cost = (int)te_process_block<64>(F, sb, ypos, xpos, best_qp);
    if (costs && TE_LANE == 0) costs[t] = cost;
  } else {
    const int cost = (int)te_process_block<64>(F, sb, ypos, xpos, F.qp);
    if (costs && TE_LANE == 0) costs[0] = cost;
  }
  te_bits_flush(sb.bits);
}

// clpf_decision + the CLPF candidate test of clpf_frame, enc/encode_frame.c:50-63,
// common/common_frame.c:499-513 (detect_clpf_simd == detect_clpf on full SBs,
// enc/encode_block.c:3036-3057): for SB (k, l) of the deblocked frame,
// returns -1 when no 8x8 block is a candidate (no bit), else the flag bit.
TE_FN int te_clpf_decide(const TeFrame &F, int k, int l) {
  const int bs = F.W / 4;
  int cand = 0;
  uint32_t s0 = 0, s1 = 0;
  for (int e = TE_LANE; e < 64 * 64; e += TE_NL) {
    const int y = e >> 6, x = e & 63;
    const int ypos = k * 64 + y, xpos = l * 64 + x;
    const TeCell &c = F.cells[(ypos / 4) * bs + xpos / 4];
    const int blk = (y & 7) == 0 && (x & 7) == 0;
    if (blk) cand |= c.mode != TE_BIPRED && (c.cbp_y || c.cbp_u || c.cbp_v);
    const TeCell &c8 = F.cells[((ypos & ~7) / 4) * bs + (xpos & ~7) / 4];
    if (c8.cbp_y && c8.mode != TE_BIPRED) {
      const uint8_t *r = F.ry;
      const int rs = F.rsy;
      const int X = r[ypos * rs + xpos];
      const int A = y == 0 ? X : r[(ypos - 1) * rs + xpos];
      const int B = x == 0 ? X : r[ypos * rs + xpos - 1];
      const int C = x == 63 ? X : r[ypos * rs + xpos + 1];
      const int D = y == 63 ? X : r[(ypos + 1) * rs + xpos];
      const int delta = ((A > X) + (B > X) + (C > X) + (D > X) > 2) - ((A < X) + (B < X) + (C < X) + (D < X) > 2);
      const int O = F.oy[ypos * F.osy + xpos];
      s0 += (uint32_t)((O - X) * (O - X));
      s1 += (uint32_t)((O - X - delta) * (O - X - delta));
    }
  }
  cand = te_any(cand);
  s0 = te_sum(s0);
  s1 = te_sum(s1);
  if (!cand) return -1;
  return (int)s1 < (int)s0;
}
