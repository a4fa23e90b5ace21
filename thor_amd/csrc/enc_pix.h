// Device-resident Thor encoder, part 2: SPMD pixel kernels (motion
// compensation, SAD / SSD and the fast sub-pel searches, intra prediction,
// residual, forward / inverse transform, quantisation).  Lane-parallel loops
// over the block, wave reductions for the sums; every producer ends with
// te_sync() so any lane may read its output.  See enc_core.h for the model.
#pragma once
#include "enc_core.h"

// HEVC integer DCT basis (g*mat_hevc, common/transform.c:41-245): row k of the
// N-point matrix is row k*32/N of the 32-point matrix.
struct TeDct {
  int8_t m[32][32];
  constexpr TeDct() : m() {
    const int c[33] = {64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67, 64,
                       61, 57, 54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9,  4,  0};
    for (int k = 0; k < 32; k++)
      for (int n = 0; n < 32; n++) {
        int v = 64;
        if (k == 0) v = 64;
        else {
          const int t = (k * (2 * n + 1)) % 128;
          v = t <= 32 ? c[t] : (t <= 64 ? -c[64 - t] : (t <= 96 ? -c[t - 64] : c[128 - t]));
        }
        m[k][n] = (int8_t)v;
      }
  }
};
TE_CONST TeDct te_dct = TeDct();
TE_FN int te_dctN(int N, int k, int n) { return te_dct.m[k * (32 / N)][n]; }

// 6-tap luma (uni-pred / enable_bipred tables) and 4-tap chroma filters,
// common/inter_prediction.c:47-70
TE_CONST int8_t te_luma_uni[4][6] = {{0, 0, 64, 0, 0, 0}, {1, -7, 55, 19, -5, 1}, {1, -7, 38, 38, -7, 1}, {1, -5, 19, 55, -7, 1}};
TE_CONST int8_t te_luma_bi[4][6] = {{0, 0, 64, 0, 0, 0}, {2, -10, 59, 17, -5, 1}, {1, -8, 39, 39, -8, 1}, {1, -5, 17, 59, -10, 2}};
TE_CONST int8_t te_chroma_f[8][4] = {{0, 64, 0, 0},    {-2, 58, 10, -2}, {-4, 54, 16, -2}, {-4, 44, 28, -4},
                                     {-4, 36, 36, -4}, {-4, 28, 44, -4}, {-2, 16, 54, -4}, {-2, 10, 58, -2}};

// get_inter_prediction_luma, common/inter_prediction.c:120-180 (its SIMD
// dispatch, common/common_kernels.c:165-784, computes the same values):
// `ref` points at the block's co-located position in the padded reference.
TE_FN void te_mc_luma(uint8_t *dst, int ds, const uint8_t *ref, int rs, int w, int h, TeMv mv, int sign, int bipred) {
  TE_P(TP_MC_Y);
  const int mx = sign ? -mv.x : mv.x, my = sign ? -mv.y : mv.y;
  const int fy = my & 3, fx = mx & 3;
  const uint8_t *r = ref + (my >> 2) * rs + (mx >> 2);
  if ((w & 3) == 0 && (h & 3) == 0) {
    // 4 x 4 outputs per lane: every source row the unit needs is loaded up
    // front (dwords, all in flight at once) and filtered horizontally once,
    // then the vertical taps run from registers
    const int w4 = w >> 2, nu = w4 * (h >> 2);
    for (int u = TE_LANE; u < nu; u += TE_NL) {
      const int rg = te_dv(u, w4), j = (u - rg * w4) * 4, i0 = rg * 4;
      int o[4][4];
      if (!fx && !fy) {
        for (int y = 0; y < 4; y++) te_st4(dst + (i0 + y) * ds + j, te_ld4(r + (i0 + y) * rs + j));
        continue;
      } else if (fx == 2 && fy == 2) {  // rows -1..5, columns -1..6
        uint32_t lo[7], hi[7];
#pragma unroll
        for (int t = 0; t < 7; t++) {
          const uint8_t *p = r + (i0 - 1 + t) * rs + j - 1;
          lo[t] = te_ld4(p);
          hi[t] = te_ld4(p + 4);
        }
        int c[7][8];
#pragma unroll
        for (int t = 0; t < 7; t++)
          for (int k = 0; k < 4; k++) {
            c[t][k] = te_b(lo[t], k);
            c[t][k + 4] = te_b(hi[t], k);
          }
#pragma unroll
        for (int y = 0; y < 4; y++)
          for (int x = 0; x < 4; x++) {  // c[y + dy + 1][x + dx + 1]
            const int k = x + 1;
            const int *a = c[y], *b = c[y + 1], *d = c[y + 2], *e = c[y + 3];
            const int v = a[k] + a[k + 1] + b[k - 1] + 2 * b[k] + 2 * b[k + 1] + b[k + 2] + d[k - 1] + 2 * d[k] +
                          2 * d[k + 1] + d[k + 2] + e[k] + e[k + 1];
            o[y][x] = te_clip255((v + 8) >> 4);
          }
      } else {
        const int8_t *fv = (bipred ? te_luma_bi : te_luma_uni)[fy];
        const int8_t *fh = (bipred ? te_luma_bi : te_luma_uni)[fx];
        int hk[9][4];  // horizontally filtered rows -2..6 (fy == 0: rows 0..3 at index 2..5)
        if (fx) {
          uint32_t d[9][3];
          const int t0 = fy ? 0 : 2, t1 = fy ? 9 : 6;
#pragma unroll
          for (int t = 0; t < 9; t++)
            if (t >= t0 && t < t1) {
              const uint8_t *p = r + (i0 - 2 + t) * rs + j - 2;
              d[t][0] = te_ld4(p);
              d[t][1] = te_ld4(p + 4);
              d[t][2] = te_ld4(p + 8);
            }
#pragma unroll
          for (int t = 0; t < 9; t++)
            if (t >= t0 && t < t1) {
              int c[12];
              for (int b = 0; b < 4; b++) {
                c[b] = te_b(d[t][0], b);
                c[b + 4] = te_b(d[t][1], b);
                c[b + 8] = te_b(d[t][2], b);
              }
              for (int x = 0; x < 4; x++) {
                int a = 0;
                for (int m = 0; m < 6; m++) a += fh[m] * c[x + m];
                hk[t][x] = a;
              }
            }
        } else {  // horizontal taps (0, 0, 64, 0, 0, 0); fy != 0 here
          uint32_t d[9];
#pragma unroll
          for (int t = 0; t < 9; t++) d[t] = te_ld4(r + (i0 - 2 + t) * rs + j);
#pragma unroll
          for (int t = 0; t < 9; t++)
            for (int x = 0; x < 4; x++) hk[t][x] = 64 * te_b(d[t], x);
        }
#pragma unroll
        for (int y = 0; y < 4; y++)
          for (int x = 0; x < 4; x++) {
            int a;
            if (fy) {
              a = 0;
              for (int k = 0; k < 6; k++) a += fv[k] * hk[y + k][x];
            } else {
              a = 64 * hk[y + 2][x];
            }
            o[y][x] = te_clip255((a + 2048) >> 12);
          }
      }
      for (int y = 0; y < 4; y++) te_st4(dst + (i0 + y) * ds + j, te_pack4(o[y][0], o[y][1], o[y][2], o[y][3]));
    }
    te_sync();
    return;
  }
  const int n = w * h;
  if (!fx && !fy) {
    for (int e = TE_LANE; e < n; e += TE_NL) {
      const int i = te_dv(e, w), j = e - te_dv(e, w) * w;
      dst[i * ds + j] = r[i * rs + j];
    }
  } else if (fx == 2 && fy == 2) {  // (2,2): 4x4 low-pass centre, :145-157
    for (int e = TE_LANE; e < n; e += TE_NL) {
      const int i = te_dv(e, w), j = e - te_dv(e, w) * w;
      const uint8_t *p = r + i * rs + j;
      int s = p[-rs] + p[-rs + 1] + p[-1] + 2 * p[0] + 2 * p[1] + p[2] + p[rs - 1] + 2 * p[rs] + 2 * p[rs + 1] + p[rs + 2] +
              p[2 * rs] + p[2 * rs + 1];
      dst[i * ds + j] = (uint8_t)te_clip255((s + 8) >> 4);
    }
  } else {  // separable 6-tap, exact 32-bit sums, clip255((s + 2048) >> 12)
    const int8_t *fv = (bipred ? te_luma_bi : te_luma_uni)[fy];
    const int8_t *fh = (bipred ? te_luma_bi : te_luma_uni)[fx];
    for (int e = TE_LANE; e < n; e += TE_NL) {
      const int i = te_dv(e, w), j = e - te_dv(e, w) * w;
      const uint8_t *p = r + (i - 2) * rs + j - 2;
      int s = 0;
      for (int m = 0; m < 6; m++) {
        int t = 0;
        for (int k = 0; k < 6; k++) t += fv[k] * p[k * rs + m];
        s += fh[m] * t;
      }
      dst[i * ds + j] = (uint8_t)te_clip255((s + 2048) >> 12);
    }
  }
  te_sync();
}

// get_inter_prediction_chroma, common/inter_prediction.c:72-118: the luma MV
// read as 1/8-pel on the chroma plane.
TE_FN void te_mc_chroma(uint8_t *dst, int ds, const uint8_t *ref, int rs, int w, int h, TeMv mv, int sign) {
  TE_P(TP_MC_C);
  const int mx = sign ? -mv.x : mv.x, my = sign ? -mv.y : mv.y;
  const int fy = my & 7, fx = mx & 7;
  const uint8_t *r = ref + (my >> 3) * rs + (mx >> 3);
  if ((w & 3) == 0 && (h & 3) == 0) {  // 4 x 4 outputs per lane, rows -1..4 loaded up front
    const int w4 = w >> 2, nu = w4 * (h >> 2);
    const int8_t *fh = te_chroma_f[fx], *fv = te_chroma_f[fy];
    for (int u = TE_LANE; u < nu; u += TE_NL) {
      const int rg = te_dv(u, w4), j = (u - rg * w4) * 4, i0 = rg * 4;
      if (!fx && !fy) {
        for (int y = 0; y < 4; y++) te_st4(dst + (i0 + y) * ds + j, te_ld4(r + (i0 + y) * rs + j));
        continue;
      }
      uint32_t lo[7], hi[7];
#pragma unroll
      for (int t = 0; t < 7; t++) {
        const uint8_t *p = r + (i0 - 1 + t) * rs + j - 1;
        lo[t] = te_ld4(p);
        hi[t] = te_ld4(p + 4);
      }
      int hk[7][4];
#pragma unroll
      for (int t = 0; t < 7; t++) {
        int c[8];
        for (int b = 0; b < 4; b++) {
          c[b] = te_b(lo[t], b);
          c[b + 4] = te_b(hi[t], b);
        }
        for (int x = 0; x < 4; x++) {
          int a = 0;
          for (int k = 0; k < 4; k++) a += fh[k] * c[x + k];
          hk[t][x] = a;
        }
      }
#pragma unroll
      for (int y = 0; y < 4; y++) {
        int o[4];
        for (int x = 0; x < 4; x++) {
          int a = 0;
          for (int m = 0; m < 4; m++) a += fv[m] * hk[y + m][x];
          o[x] = te_clip255((a + 2048) >> 12);
        }
        te_st4(dst + (i0 + y) * ds + j, te_pack4(o[0], o[1], o[2], o[3]));
      }
    }
    te_sync();
    return;
  }
  if ((w & 3) == 0) {  // four outputs per lane
    const int w4 = w >> 2, n4 = w4 * h;
    if (!fx && !fy) {
      for (int g = TE_LANE; g < n4; g += TE_NL) {
        const int i = te_dv(g, w4), j = (g - i * w4) * 4;
        te_st4(dst + i * ds + j, te_ld4(r + i * rs + j));
      }
    } else {
      const int8_t *fh = te_chroma_f[fx], *fv = te_chroma_f[fy];
      for (int g = TE_LANE; g < n4; g += TE_NL) {
        const int i = te_dv(g, w4), j = (g - i * w4) * 4;
        int s[4] = {0, 0, 0, 0};
        for (int m = 0; m < 4; m++) {  // rows -1..2, columns -1..6
          const uint8_t *p = r + (i - 1 + m) * rs + j - 1;
          const uint32_t lo = te_ld4(p), hi = te_ld4(p + 4);
          int c[8];
          for (int b = 0; b < 4; b++) {
            c[b] = te_b(lo, b);
            c[b + 4] = te_b(hi, b);
          }
          for (int x = 0; x < 4; x++) {
            int t = 0;
            for (int k = 0; k < 4; k++) t += fh[k] * c[x + k];
            s[x] += fv[m] * t;
          }
        }
        te_st4(dst + i * ds + j, te_pack4(te_clip255((s[0] + 2048) >> 12), te_clip255((s[1] + 2048) >> 12),
                                          te_clip255((s[2] + 2048) >> 12), te_clip255((s[3] + 2048) >> 12)));
      }
    }
    te_sync();
    return;
  }
  const int n = w * h;
  if (!fx && !fy) {
    for (int e = TE_LANE; e < n; e += TE_NL) {
      const int i = te_dv(e, w), j = e - te_dv(e, w) * w;
      dst[i * ds + j] = r[i * rs + j];
    }
  } else {
    const int8_t *fh = te_chroma_f[fx], *fv = te_chroma_f[fy];
    for (int e = TE_LANE; e < n; e += TE_NL) {
      const int i = te_dv(e, w), j = e - te_dv(e, w) * w;
      const uint8_t *p = r + (i - 1) * rs + j - 1;
      int s = 0;
      for (int m = 0; m < 4; m++) {
        int t = 0;
        for (int k = 0; k < 4; k++) t += fh[k] * p[m * rs + k];
        s += fv[m] * t;
      }
      dst[i * ds + j] = (uint8_t)te_clip255((s + 2048) >> 12);
    }
  }
  te_sync();
}

// sad_calc (enc/encode_block.c:740-755) / ssd_calc (:782-797): exact sums
TE_FN uint32_t te_sad(const uint8_t *a, int as, const uint8_t *b, int bs, int w, int h) {
  TE_P(TP_SAD);
  uint32_t s = 0;
  if ((w & 3) == 0) {
    const int w4 = w >> 2, n4 = w4 * h;
    for (int g = TE_LANE; g < n4; g += TE_NL) {
      const int i = te_dv(g, w4), j = (g - i * w4) * 4;
      s = te_sad4(te_ld4(a + i * as + j), te_ld4(b + i * bs + j), s);
    }
    return te_sum(s);
  }
  for (int e = TE_LANE; e < w * h; e += TE_NL) {
    const int i = te_dv(e, w), j = e - te_dv(e, w) * w;
    s += (uint32_t)te_abs((int)a[i * as + j] - (int)b[i * bs + j]);
  }
  return te_sum(s);
}
TE_FN uint32_t te_ssd(const uint8_t *a, int as, const uint8_t *b, int bs, int w, int h) {
  uint32_t s = 0;
  if ((w & 3) == 0) {  // sum (a - b)^2 = sum a^2 + sum b^2 - 2 sum ab, exact modulo 2^32
    const int w4 = w >> 2, n4 = w4 * h;
    uint32_t ab = 0;
    for (int g = TE_LANE; g < n4; g += TE_NL) {
      const int i = te_dv(g, w4), j = (g - i * w4) * 4;
      const uint32_t x = te_ld4(a + i * as + j), y = te_ld4(b + i * bs + j);
      s = te_dot4(y, y, te_dot4(x, x, s));
      ab = te_dot4(x, y, ab);
    }
    return te_sum(s - 2u * ab);
  }
  for (int e = TE_LANE; e < w * h; e += TE_NL) {
    const int i = te_dv(e, w), j = e - te_dv(e, w) * w;
    const int d = (int)a[i * as + j] - (int)b[i * bs + j];
    s += (uint32_t)(d * d);
  }
  return te_sum(s);
}

TE_CONST int8_t te_wide_off[5] = {-3, -1, 0, 1, 3};
// widesad_calc, enc/encode_block.c:757-780 (its SIMD form widesad_calc_simd,
// enc/enc_kernels.c:71-98, keeps the first minimum too): SAD at horizontal
// offsets -3, -1, 0, 1, 3; returns the best, *x = its offset.
TE_FN uint32_t te_widesad(const uint8_t *a, int as, const uint8_t *b, int bs, int w, int h, int *x) {
  const int8_t *off = te_wide_off;
  uint32_t s[5] = {0, 0, 0, 0, 0};
  if ((w & 3) == 0) {  // b columns j-4..j+7 as three dwords, the five offsets by byte alignment
    const int w4 = w >> 2, n4 = w4 * h;
    for (int g = TE_LANE; g < n4; g += TE_NL) {
      const int i = te_dv(g, w4), j = (g - i * w4) * 4;
      const uint32_t av = te_ld4(a + i * as + j);
      const uint8_t *q = b + i * bs + j;
      const uint32_t d0 = te_ld4(q - 4), d1 = te_ld4(q), d2 = te_ld4(q + 4);
      s[0] = te_sad4(av, te_align4(d1, d0, 1), s[0]);
      s[1] = te_sad4(av, te_align4(d1, d0, 3), s[1]);
      s[2] = te_sad4(av, d1, s[2]);
      s[3] = te_sad4(av, te_align4(d2, d1, 1), s[3]);
      s[4] = te_sad4(av, te_align4(d2, d1, 3), s[4]);
    }
  } else
  for (int e = TE_LANE; e < w * h; e += TE_NL) {
    const int i = te_dv(e, w), j = e - te_dv(e, w) * w;
    const int av = a[i * as + j];
    for (int k = 0; k < 5; k++) s[k] += (uint32_t)te_abs(av - (int)b[i * bs + j + off[k]]);
  }
  uint32_t best = 0;
  int bx = 0;
  for (int k = 0; k < 5; k++) {
    const uint32_t v = te_sum(s[k]);
    if (k == 0 || v < best) {
      best = v;
      bx = off[k];
    }
  }
  *x = bx;
  return best;
}

// sad_calc_fasthalf, enc/encode_block.c:497-605 (== sad_calc_fasthalf_simd):
// eight approximate half-pel positions from rounding averages around `b`.
TE_FN uint32_t te_fasthalf(const uint8_t *a, int as, const uint8_t *b, int bs, int width, int height, int *x, int *y) {
  uint32_t tl = 0, tr = 0, br = 0, bl = 0, top = 0, right = 0, down = 0, left = 0;
  for (int e = TE_LANE; e < width * height; e += TE_NL) {
    const int i = te_dv(e, width), j = e - te_dv(e, width) * width;
    const uint8_t *q = b + i * bs;
    const int A = a[i * as + j];
    int t1, t2, t3, t4, t5, t6, t7, t8, ptl, ptr, pbr, pbl;
    t1 = (q[-bs + j - 1] + q[-bs + j] + 1) >> 1;
    t2 = (q[j - 1] + q[j] + 1) >> 1;
    t1 = (t1 + t2) >> 1;
    t3 = (q[-2 * bs + j - 1] + q[bs + j - 1] + 1) >> 1;
    t4 = (q[-2 * bs + j] + q[bs + j] + 1) >> 1;
    t3 = (t3 + t4) >> 1;
    t5 = (q[-bs + j - 2] + q[-bs + j + 1] + 1) >> 1;
    t6 = (q[j - 2] + q[j + 1] + 1) >> 1;
    t5 = (t5 + t6) >> 1;
    t5 = (t3 + t5) >> 1;
    ptl = (t5 + t1) >> 1;
    left += (uint32_t)te_abs(A - t2);

    t1 = (q[-bs + j] + q[-bs + j + 1] + 1) >> 1;
    t8 = (q[j] + q[j + 1] + 1) >> 1;
    t1 = (t1 + t8) >> 1;
    t5 = (q[-2 * bs + j + 1] + q[bs + j + 1] + 1) >> 1;
    t3 = (t4 + t5) >> 1;
    t4 = (q[-bs + j - 1] + q[-bs + j + 2] + 1) >> 1;
    t7 = (q[j - 1] + q[j + 2] + 1) >> 1;
    t5 = (t7 + t4) >> 1;
    t5 = (t3 + t5) >> 1;
    ptr = (t5 + t1) >> 1;
    right += (uint32_t)te_abs(A - t8);

    t1 = (q[bs + j - 1] + q[bs + j] + 1) >> 1;
    t3 = (t1 + t2) >> 1;
    t2 = (q[-bs + j - 1] + q[2 * bs + j - 1] + 1) >> 1;
    t4 = (q[-bs + j] + q[2 * bs + j] + 1) >> 1;
    t5 = (t4 + t2) >> 1;
    t1 = (q[bs + j - 2] + q[bs + j + 1] + 1) >> 1;
    t2 = (t6 + t1) >> 1;
    t2 = (t5 + t2) >> 1;
    pbl = (t2 + t3) >> 1;

    t2 = (q[bs + j] + q[bs + j + 1] + 1) >> 1;
    t3 = (t8 + t2) >> 1;
    t5 = (q[-bs + j + 1] + q[2 * bs + j + 1] + 1) >> 1;
    t6 = (t4 + t5) >> 1;
    t8 = (q[bs + j - 1] + q[bs + j + 2] + 1) >> 1;
    t1 = (t7 + t8) >> 1;
    t2 = (t6 + t1) >> 1;
    pbr = (t2 + t3) >> 1;

    down += (uint32_t)te_abs(A - ((q[j] + q[j + bs] + 1) >> 1));
    top += (uint32_t)te_abs(A - ((q[j] + q[j - bs] + 1) >> 1));
    tl += (uint32_t)te_abs(A - ptl);
    tr += (uint32_t)te_abs(A - ptr);
    br += (uint32_t)te_abs(A - pbr);
    bl += (uint32_t)te_abs(A - pbl);
  }
  tl = te_sum(tl); tr = te_sum(tr); br = te_sum(br); bl = te_sum(bl);
  top = te_sum(top); right = te_sum(right); down = te_sum(down); left = te_sum(left);
  int bestx = 0, besty = -2;
  if (down < top) { besty = 2; top = down; }
  if (right < top) { bestx = 2; besty = 0; top = right; }
  if (left < top) { bestx = -2; besty = 0; top = left; }
  if (tl < top) { bestx = -2; besty = -2; top = tl; }
  if (tr < top) { bestx = 2; besty = -2; top = tr; }
  if (br < top) { bestx = 2; besty = 2; top = br; }
  if (bl < top) { bestx = -2; besty = 2; top = bl; }
  *x = bestx;
  *y = besty;
  return top;
}

// sad_calc_fastquarter, enc/encode_block.c:609-738 (== the SIMD form): eight
// approximate quarter-pel positions around the half-pel position (*x, *y) in,
// the best offset out.
TE_FN uint32_t te_fastquarter(const uint8_t *o, int os, const uint8_t *r, int rs, int width, int height, int *x, int *y) {
  uint32_t tl = 0, tr = 0, br = 0, bl = 0, top = 0, right = 0, down = 0, left = 0;
  const int X = *x, Y = *y;
  for (int e = TE_LANE; e < width * height; e += TE_NL) {
    const int i = te_dv(e, width), j = e - te_dv(e, width) * width;
    const uint8_t *q = r + i * rs;
    const int O = o[i * os + j];
    if (X & Y) {
      const int a = q[j], d = q[j + 1], ee = q[j + rs + 1], f = q[j + rs];
      const int ad = (a + d + 1) >> 1, de = (d + ee + 1) >> 1, af = (a + f + 1) >> 1, fe = (f + ee + 1) >> 1;
      tl += te_abs(O - ((ad + af) >> 1));
      top += te_abs(O - ((de + a) >> 1));
      tr += te_abs(O - ((ad + de) >> 1));
      left += te_abs(O - ((ad + f) >> 1));
      right += te_abs(O - ((ad + ee) >> 1));
      bl += te_abs(O - ((af + fe) >> 1));
      down += te_abs(O - ((de + f) >> 1));
      br += te_abs(O - ((de + fe) >> 1));
    } else if (X) {
      const int a = q[j], b = q[j - rs], c = q[j - rs + 1], d = q[j + 1], ee = q[j + rs + 1], f = q[j + rs];
      const int ad = (a + d + 1) >> 1, de = (d + ee + 1) >> 1, dc = (d + c + 1) >> 1, af = (a + f + 1) >> 1,
                ab = (a + b + 1) >> 1;
      tl += te_abs(O - ((ad + ab) >> 1));
      top += te_abs(O - ((dc + a) >> 1));
      tr += te_abs(O - ((ad + dc) >> 1));
      left += te_abs(O - ((ad + a) >> 1));
      right += te_abs(O - ((ad + d) >> 1));
      bl += te_abs(O - ((ad + af) >> 1));
      down += te_abs(O - ((af + d) >> 1));
      br += te_abs(O - ((ad + de) >> 1));
    } else if (Y) {
      const int a = q[j], d = q[j + 1], ee = q[j + rs + 1], f = q[j + rs], g = q[j + rs - 1], h = q[j - 1];
      const int ad = (a + d + 1) >> 1, af = (a + f + 1) >> 1, fe = (f + ee + 1) >> 1, ah = (a + h + 1) >> 1,
                gf = (g + f + 1) >> 1;
      tl += te_abs(O - ((ah + af) >> 1));
      top += te_abs(O - ((af + a) >> 1));
      tr += te_abs(O - ((ad + af) >> 1));
      left += te_abs(O - ((gf + a) >> 1));
      right += te_abs(O - ((ad + f) >> 1));
      bl += te_abs(O - ((af + gf) >> 1));
      down += te_abs(O - ((af + f) >> 1));
      br += te_abs(O - ((af + fe) >> 1));
    } else {
      const int a = q[j], b = q[j - rs], d = q[j + 1], f = q[j + rs], h = q[j - 1];
      const int ad = (a + d + 1) >> 1, af = (a + f + 1) >> 1, ah = (a + h + 1) >> 1, ab = (a + b + 1) >> 1;
      tl += te_abs(O - ((ah + ab) >> 1));
      top += te_abs(O - ((ab + a) >> 1));
      tr += te_abs(O - ((ad + ab) >> 1));
      left += te_abs(O - ((ah + a) >> 1));
      right += te_abs(O - ((ad + a) >> 1));
      bl += te_abs(O - ((ah + af) >> 1));
      down += te_abs(O - ((af + a) >> 1));
      br += te_abs(O - ((af + ad) >> 1));
    }
  }
  tl = te_sum(tl); tr = te_sum(tr); br = te_sum(br); bl = te_sum(bl);
  top = te_sum(top); right = te_sum(right); down = te_sum(down); left = te_sum(left);
  int bestx = 0, besty = -1;
  if (tl < top) { bestx = -1; top = tl; }
  if (tr < top) { bestx = 1; top = tr; }
  if (left < top) { bestx = -1; besty = 0; top = left; }
  if (right < top) { bestx = 1; besty = 0; top = right; }
  if (bl < top) { bestx = -1; besty = 1; top = bl; }
  if (down < top) { bestx = 0; besty = 1; top = down; }
  if (br < top) { bestx = 1; besty = 1; top = br; }
  *x = bestx;
  *y = besty;
  return top;
}

// ---- intra prediction (common/intra_prediction.c) ---------------------------
// Neighbour arrays: left[0..2n), top[0..2n), *tl.  Built by make_top_and_left
// (:57-143): `rf` = frame pixel at the CU origin (stride fs), `rb` = compact
// reconstructed block at the sub-TU origin (stride rbs) for tb-split TUs.
struct TeNbr {
  uint8_t left[2 * 64 + 2], top[2 * 64 + 2];
  uint8_t lF[2 * 64 + 2], tF[2 * 64 + 2];  // 1-2-1 filtered copies
  int T[64], L[64];                        // planar edge sums
  int tl, tlF, TL;
};
#if !defined(TE_HOST)
// The luma block whose neighbour arrays and search setup the worker's TeNbr
// holds (set by te_search_intra after te_ipx_setup, 0: none): the block's
// 8 x 8 register chain then skips rebuilding them.  Every writer of the
// arrays forgets it first.
__shared__ int g_te_nb_key;
#define TE_NB_FORGET()                 \
  do {                                 \
    if (TE_LANE == 0) g_te_nb_key = 0; \
  } while (0)
#else
#define TE_NB_FORGET() \
  do {                 \
  } while (0)
#endif
TE_FN int te_nb_key(int ypos, int xpos, int size) { return ((ypos << 16) | (xpos << 3) | te_log2(size)) + 1; }
TE_FN void te_make_top_and_left(TeNbr &nb, const uint8_t *rf, int fs, const uint8_t *rb, int rbs, int i, int j, int ypos,
                                int xpos, int size, int cb_ur, int cb_dl, int tb_split) {
  TE_P(TP_TOPLEFT);
  TE_NB_FORGET();
  int dl, ur;
  if (!tb_split) {
    dl = cb_dl;
    ur = cb_ur;
  } else {
    dl = (j == 0 && (i == 0 || cb_dl)) ? 1 : 0;
    ur = (j == 0 || (i == 0 && cb_ur)) ? 1 : 0;
  }
  const int leftlen = dl ? size + 1 : size, toplen = ur ? size + 1 : size;
  // top row source
  const int top128 = tb_split ? (ypos + i == 0) : (ypos == 0);
  const uint8_t *tsrc = (!tb_split || i == 0) ? rf - fs + (tb_split ? j : 0) : rb - rbs;
  const int left128 = tb_split ? (xpos + j == 0) : (xpos == 0);
  const uint8_t *lsrc;  // left column pointer, stride ls
  int ls;
  if (!tb_split || j == 0) {
    lsrc = rf + (tb_split ? i * fs : 0) - 1;
    ls = fs;
  } else {
    lsrc = rb - 1;
    ls = rbs;
  }
  for (int k = TE_LANE; k < 2 * size; k += TE_NL) {
    nb.top[k] = top128 ? 128 : tsrc[k < toplen ? k : toplen - 1];
    nb.left[k] = left128 ? 128 : lsrc[(k < leftlen ? k : leftlen - 1) * ls];
  }
  // top-left
  int tl;
  if (top128) tl = 128;
  else if (!tb_split || i == 0) tl = xpos > 0 ? rf[-fs + (tb_split ? j : 0) - 1] : tsrc[0];
  else tl = xpos > 0 ? (j > 0 ? rb[-rbs - 1] : rf[(i - 1) * fs - 1]) : tsrc[0];
  if (top128) tl = left128 ? 128 : lsrc[0];  // `if (ypos[+i]==0) *top_left = left[0]`
  nb.tl = tl;
  te_sync();
}

// filter_121 (:39-48) of in[0..len) into out
TE_FN void te_f121(const uint8_t *in, uint8_t *out, int len) {
  for (int j = TE_LANE; j < len; j += TE_NL) {
    int v;
    if (j == 0) v = (3 * in[0] + in[1] + 2) >> 2;
    else if (j == len - 1) v = (in[len - 2] + 3 * in[len - 1] + 2) >> 2;
    else v = (in[j - 1] + 2 * in[j] + in[j + 1] + 2) >> 2;
    out[j] = (uint8_t)v;
  }
}

// get_intra_prediction (:363-388) and the mode functions (:145-361) into a
// compact n x n block.  search_dc: search_intra_prediction_params' DC
// (enc/encode_block.c:1250, always (left, top)) instead of the position-aware one.
TE_FN void te_intra_pred(TeNbr &nb, int ypos, int xpos, int n, uint8_t *pb, int mode, int search_dc) {
  TE_P(TP_IPRED);
  TE_NB_FORGET();
  // four horizontally adjacent pixels per lane and step (n >= 4), one dword store
  const int n4 = (n * n) >> 2;
  auto quad = [&](auto px) {
    for (int g = TE_LANE; g < n4; g += TE_NL) {
      const int e = 4 * g, i = te_dv(e, n), j = e - i * n;
      te_st4(pb + e, te_pack4(px(i, j), px(i, j + 1), px(i, j + 2), px(i, j + 3)));
    }
  };
  switch (mode) {
    case TE_PLANAR: {  // :182-214, C division truncating toward zero
      for (int k = TE_LANE; k < 2 * n; k += TE_NL) {
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
      const int TL = nb.left[1] + 2 * nb.left[0] + 2 * nb.tl + 2 * nb.top[0] + nb.top[1];
      quad([&](int i, int j) { return te_clip255((nb.L[i] + nb.T[j] - TL + 4) / 8); });
      break;
    }
    case TE_HOR:
      quad([&](int i, int j) { return (int)nb.left[i]; });
      break;
    case TE_VER:
      quad([&](int i, int j) { return (int)nb.top[j]; });
      break;
    case TE_UPLEFT:
    case TE_UPUPLEFT:
    case TE_UPLEFTLEFT: {
      te_f121(nb.left, nb.lF, n);
      te_f121(nb.top, nb.tF, n);
      const int tlF = (2 * nb.tl + nb.left[0] + nb.top[0] + 2) >> 2;
      te_sync();
      if (mode == TE_UPLEFT) {  // :216-240
        quad([&](int i, int j) {
          const int d = i - j;
          return (int)(d > 0 ? nb.lF[d - 1] : (d == 0 ? tlF : nb.tF[-d - 1]));
        });
      } else if (mode == TE_UPUPLEFT) {  // :279-307
        quad([&](int i, int j) {
          const int d = i - 2 * j;
          if (d > 1) return (int)nb.lF[d - 2];
          if (d == 1) return tlF;
          if (d == 0) return (tlF + nb.tF[0]) >> 1;
          if (d & 1) return (int)nb.tF[(-d) / 2];
          return (nb.tF[(-d) / 2] + nb.tF[(-d) / 2 - 1]) >> 1;
        });
      } else {  // :309-337
        quad([&](int i, int j) {
          const int d = 2 * i - j;
          if (d < -1) return (int)nb.tF[-d - 2];
          if (d == -1) return tlF;
          if (d == 0) return (tlF + nb.lF[0]) >> 1;
          if (d & 1) return (int)nb.lF[d / 2];
          return (nb.lF[d / 2] + nb.lF[d / 2 - 1]) >> 1;
        });
      }
      break;
    }
    case TE_UPRIGHT:
    case TE_UPUPRIGHT: {
      te_f121(nb.top, nb.tF, 2 * n);
      te_sync();
      if (mode == TE_UPRIGHT) {  // :242-256
        quad([&](int i, int j) { return (int)nb.tF[i + j + 1]; });
      } else {  // :258-277
        quad([&](int i, int j) {
          const int d = i + 2 * j;
          return (d & 1) ? (int)nb.tF[(d + 1) / 2] : (nb.tF[d / 2] + nb.tF[d / 2 + 1]) >> 1;
        });
      }
      break;
    }
    case TE_DOWNLEFTLEFT: {  // :339-361
      te_f121(nb.left, nb.lF, 2 * n);
      te_sync();
      quad([&](int i, int j) {
        const int d = 2 * i + j;
        return (d & 1) ? (int)nb.lF[(d + 1) / 2] : (nb.lF[d / 2] + nb.lF[d / 2 + 1]) >> 1;
      });
      break;
    }
    default: {  // DC, :145-160 (and out-of-range modes, :386-387)
      const uint8_t *a = (search_dc || xpos != 0) ? nb.left : nb.top;
      const uint8_t *b = (search_dc || ypos != 0) ? nb.top : nb.left;
      uint32_t s = 0;
      for (int k = TE_LANE; k < n; k += TE_NL) s += a[k] + b[k];
      s = te_sum(s);
      const int dc = ((int)s + n) / (2 * n);
      quad([&](int, int) { return dc; });
      break;
    }
  }
  te_sync();
}

// ---- transform chain -----------------------------------------------------------
// Scratch of one transform block (compact, q = min(N, 16)).
struct TeTx {
  int16_t R[32 * 32];  // residual (N x N, N <= 32), reconstructed residual (64: the 32-point output)
  int16_t A[32 * 32];  // pre-summed input of the 32 / 64 paths
  int16_t T[32 * 32];  // pass-1 output
  int16_t C[256];      // q x q coefficients / levels (raster; every value fits 16 bits)
  int16_t S[256];      // levels in scan order
  int16_t O[256];      // coefficients in scan order (RDOQ light)
  int16_t scan[256];   // write_coeff scratch
  int8_t M[32 * 32];   // 32-point DCT basis (te_dct), loaded once per worker
};
TE_FN void te_load_basis(TeTx &X) {
  for (int e = TE_LANE; e < 1024; e += TE_NL) X.M[e] = te_dct.m[e >> 5][e & 31];
  te_sync();
}
// row k of the N-point basis = row k * 32 / N of the 32-point one
#define TE_DCT(X, N, k, n) ((int)(X).M[((k) * (32 / (N))) * 32 + (n)])

// One output of the reference SIMD 8-point forward pass (transform8,
// common/common_kernels.c:1887-1967): 16-bit wrapping butterflies.
TE_FN int te_fwd8(const int16_t *s, int k, int shift) {
  int E[4], O[4];
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

// The two matrix passes of transform (common/transform.c:309-327) for an
// N-point basis, N a compile-time constant so the inner products unroll and
// their LDS reads issue back to back: in (N x N) -> X.T (q x N) -> X.C (q x q).
template <int N>
TE_FN void te_fwd_gen(TeTx &X, const int16_t *in, int sh1, int sh2) {
  constexpr int q = N < 16 ? N : 16;
  const int add1 = 1 << (sh1 - 1), add2 = 1 << (sh2 - 1);
  for (int e = TE_LANE; e < q * N; e += TE_NL) {  // :309-316, int16 store
    const int i = e / N, j = e % N;
    const int16_t *x = &in[j * N];
    int s = 0;
#pragma unroll
    for (int k = 0; k < N; k++) s += TE_DCT(X, N, i, k) * (int)x[k];
    X.T[i * N + j] = (int16_t)te_wrap16((s + add1) >> sh1);
  }
  te_sync();
  for (int e = TE_LANE; e < q * q; e += TE_NL) {  // :319-327
    const int i = e / q, j = e % q;
    const int16_t *t = &X.T[j * N];
    int s = 0;
#pragma unroll
    for (int k = 0; k < N; k++) s += TE_DCT(X, N, i, k) * (int)t[k];
    X.C[i * q + j] = (int16_t)te_wrap16((s + add2) >> sh2);
  }
  te_sync();
}

// transform, common/transform.c:249-330 (SIMD transform_simd for the 8x8
// butterfly wrap): X.R (size x size, stride size; 64: X.A, te_residual64) -> X.C (q x q raster).
TE_FN void te_fwd_tx(TeTx &X, int size, int fast) {
  TE_P(TP_FWD);
  const int lg = te_log2(size);
  int N = size, sh1 = lg, sh2 = lg + 5;
  const int16_t *in = X.R;
  if (size == 8) {
    for (int e = TE_LANE; e < 64; e += TE_NL) {
      const int row = e >> 3, k = e & 7;
      X.T[k * 8 + row] = (int16_t)te_fwd8(&X.R[row * 8], k, sh1);
    }
    te_sync();
    for (int e = TE_LANE; e < 64; e += TE_NL) {
      const int row = e >> 3, k = e & 7;
      X.C[k * 8 + row] = (int16_t)te_fwd8(&X.T[row * 8], k, sh2);
    }
    te_sync();
    return;
  }
  // size 64: X.A already holds the pre-summed residual (te_residual64)
  if (size > 16 && fast) {  // 2x2 / 4x4 pre-sum into a 16-point transform, :273-293
    N = 16;
    sh1 += 1 + (size == 64);
    sh2 = 9;
    if (size == 32)
      for (int e = TE_LANE; e < 256; e += TE_NL) {
        const int i = e >> 4, j = e & 15;
        const int16_t *r = &X.R[(2 * i) * 32 + 2 * j];
        X.A[e] = (int16_t)te_wrap16(r[0] + r[1] + r[32] + r[33]);
      }
    in = X.A;
  } else if (size == 64) {  // 2x2 pre-sum into a 32-point transform, :294-307
    N = 32;
    sh1 = 7;
    sh2 = 10;
    in = X.A;
  }
  te_sync();
  if (N == 4) te_fwd_gen<4>(X, in, sh1, sh2);
  else if (N == 16) te_fwd_gen<16>(X, in, sh1, sh2);
  else te_fwd_gen<32>(X, in, sh1, sh2);
}

// quantize, enc/encode_block.c:75-172 (rdoq = 0): X.C -> levels (q x q
// raster) in X.C.  Returns cbp.  With `coef`: the levels go there (raster)
// and X.C holds them dequantized instead -- the chains' quantize, level copy
// and dequantize in one pass (X.C is only read when cbp != 0).
TE_FN int te_quant_t(TeTx &X, int qp, int size, int type, int16_t *coef) {
  TE_P(TP_QUANT);
  const int intra = (type >> 1) & 1, chroma = type & 1;
  const int lg = te_log2(size), q = TE_MIN(size, 16), nq = q * q;
  const int scale = te_gquant[qp % 6], shift2 = 21 - lg + qp / 6;
  const int offset = (intra ? 38 : -26) * (1 << (shift2 - 8));
  // each lane's coefficients and scan positions stay in registers across the passes
  constexpr int NS = (256 + TE_NL - 1) / TE_NL;
  int posv[NS], cv[NS];
  int lp = -1;
#pragma unroll
  for (int t = 0; t < NS; t++) {
    const int r = TE_LANE + TE_NL * t;
    posv[t] = r < nq ? te_zz(q, r) : 256;
    cv[t] = r < nq ? X.C[r] : 0;
    if (r < nq && (te_abs(te_abs(cv[t]) * scale + offset) >> shift2) != 0) lp = TE_MAX(lp, posv[t]);
  }
  const int last_pos = te_maxi(lp);  // -1: no level (the reference loop ends at pos = -1)
  const int off0 = (intra ? 102 : 51) * (1 << (shift2 - 8)), off1 = (intra ? 115 : 90) * (1 << (shift2 - 8));
  int any = 0;
#pragma unroll
  for (int t = 0; t < NS; t++) {
    const int r = TE_LANE + TE_NL * t;
    if (r >= nq) continue;
    const int pos = posv[t];
    int lev = 0;
    if (pos <= last_pos) {
      const int c = cv[t];
      const int ac = scale * te_abs(c);
      const int l0 = ac >> shift2;
      const int l = (ac + ((l0 == 0 || chroma) ? off0 : off1)) >> shift2;
      lev = c < 0 ? -l : l;
      any |= l != 0;
    }
    X.S[pos] = (int16_t)lev;
    X.O[pos] = (int16_t)cv[t];
  }
  const int cbp = te_any(any);
  te_sync();
  if (cbp) {  // "RDOQ light" (:134-168), serial over the scan.  Only positions whose
    // initial level exceeds 1 can trigger: earlier iterations modify indices
    // below the one they visit, so S[pos] is still its initial value when pos
    // is visited.  Visit just those, in order.  Every test the loop makes on
    // the current levels is |S| > 1 or S != 0, so it runs on two scan-order
    // bit masks (uniform registers) that each change updates -- no LDS round
    // trip or barrier per candidate; the changed levels go to X.S for the
    // raster pass below.
    const int n = chroma ? last_pos + 1 : nq;
    const int thr = (73 * te_gdequant[qp % 6] << (qp / 6)) >> (4 + lg);
    uint64_t big[4], nzm[4];
#if defined(TE_HOST)
    for (int k = 0; k < 4; k++) big[k] = nzm[k] = 0;
    for (int pos = 0; pos < nq; pos++) {
      if (te_abs(X.S[pos]) > 1) big[pos >> 6] |= 1ULL << (pos & 63);
      if (X.S[pos] != 0) nzm[pos >> 6] |= 1ULL << (pos & 63);
    }
#else
    for (int k = 0; k < 4; k++) {
      const int pos = TE_LANE + 64 * k;
      const int sv = pos < nq ? X.S[pos] : 0;
      big[k] = __ballot(te_abs(sv) > 1);
      nzm[k] = __ballot(sv != 0);
    }
#endif
#define TE_BIG(p) ((big[(p) >> 6] >> ((p) & 63)) & 1)
#define TE_NZ(p) ((nzm[(p) >> 6] >> ((p) & 63)) & 1)
    for (int k = 0; k < 4; k++) {
      const int lo = TE_MAX(2, 64 * k), hi = TE_MIN(n, 64 * k + 64);
      if (lo >= hi) continue;
      uint64_t m = big[k] & (hi - 64 * k >= 64 ? ~0ULL : ((1ULL << (hi - 64 * k)) - 1)) & (~0ULL << (lo - 64 * k));
      while (m) {
        const int pos = k * 64 + __builtin_ctzll(m);
        m &= m - 1;
        int flag = 1;
        if (pos > 2 && TE_BIG(pos - 3)) flag = 0;
        if (pos > 3 && TE_BIG(pos - 4) && TE_NZ(pos - 3)) flag = 0;
        if (pos == 2 && (chroma == 0 || last_pos >= 6)) flag = 0;
        if (flag && !TE_NZ(pos - 2) && !TE_NZ(pos - 1) && TE_BIG(pos)) {
          const int c1 = X.O[pos], c2 = X.O[pos - 1], c3 = X.O[pos - 2];
          const int K1 = te_abs(c1), K2 = te_abs(c2), K3 = te_abs(c3), K4 = TE_MAX(K2, K3);
          int at, v;
          if (K1 + K4 < thr) {
            at = pos;
            v = c1 < 0 ? -1 : 1;
          } else if (K2 > K3) {
            at = pos - 1;
            v = c2 < 0 ? -1 : 1;
          } else {
            at = pos - 2;
            v = c3 < 0 ? -1 : 1;
          }
          if (TE_LANE == 0) X.S[at] = (int16_t)v;
          big[at >> 6] &= ~(1ULL << (at & 63));  // |v| == 1
          nzm[at >> 6] |= 1ULL << (at & 63);
        }
      }
    }
#undef TE_BIG
#undef TE_NZ
  }
  te_sync();
  if (coef) {  // the levels to the candidate's coefficient tile, X.C dequantized (common_block.c:132-146)
    const int rshift = lg - 1, add = 1 << (rshift - 1), lshift = qp / 6, dscale = te_gdequant[qp % 6];
#pragma unroll
    for (int t = 0; t < NS; t++) {
      const int r = TE_LANE + TE_NL * t;
      if (r < nq) {
        const int lev = X.S[posv[t]];
        coef[r] = (int16_t)lev;
        X.C[r] = (int16_t)te_wrap16(((lev * dscale) * (1 << lshift) + add) >> rshift);
      }
    }
  } else {
#pragma unroll
    for (int t = 0; t < NS; t++) {  // back to raster (:170-174)
      const int r = TE_LANE + TE_NL * t;
      if (r < nq) X.C[r] = X.S[posv[t]];
    }
  }
  te_sync();
  return cbp;
}
TE_FN int te_quant(TeTx &X, int qp, int size, int type) { return te_quant_t(X, qp, size, type, nullptr); }

// dequantize (common/common_block.c:132-146), int16 truncating store, in place
TE_FN void te_dequant(TeTx &X, int qp, int size) {
  const int q = TE_MIN(size, 16);
  const int rshift = te_log2(size) - 1, add = 1 << (rshift - 1);
  const int lshift = qp / 6, scale = te_gdequant[qp % 6];
  for (int e = TE_LANE; e < q * q; e += TE_NL) X.C[e] = (int16_t)te_wrap16(((X.C[e] * scale) * (1 << lshift) + add) >> rshift);
  te_sync();
}
#ifndef TE_QUANT_FUSE
#define TE_QUANT_FUSE 1
#endif
// quantize -> the levels into the candidate's tile -> X.C dequantized (when cbp)
TE_FN int te_quant_chain(TeTx &X, int qp, int size, int type, int16_t *coef) {
#if TE_QUANT_FUSE
  return te_quant_t(X, qp, size, type, coef);
#else
  const int cbp = te_quant(X, qp, size, type);
  const int q = TE_MIN(size, 16);
  for (int e = TE_LANE; e < q * q; e += TE_NL) coef[e] = (int16_t)X.C[e];
  if (cbp) te_dequant(X, qp, size);
  return cbp;
#endif
}

// inverse_transform (common/transform.c:432-518): X.C (q x q) -> X.R
// (n x n, n = min(size, 32); 64 = the 32-point output, replicated 2x2 by the reader).
template <int n>
TE_FN void te_inv_gen(TeTx &X) {
  constexpr int q = n < 16 ? n : 16;
  for (int e = TE_LANE; e < q * n; e += TE_NL) {
    const int k = e / n, yp = e % n;  // coefficient column k
    int s = 0;
#pragma unroll
    for (int m = 0; m < q; m++) s += TE_DCT(X, n, m, yp) * X.C[m * q + k];
    X.T[k * n + yp] = (int16_t)te_clip16((s + 64) >> 7);
  }
  te_sync();
  for (int e = TE_LANE; e < n * n; e += TE_NL) {
    const int yp = e / n, xp = e % n;
    int s = 0;
#pragma unroll
    for (int k = 0; k < q; k++) s += TE_DCT(X, n, k, xp) * (int)X.T[k * n + yp];
    X.R[yp * n + xp] = (int16_t)te_clip16((s + 2048) >> 12);
  }
  te_sync();
}
TE_FN void te_inv_tx(TeTx &X, int size) {
  TE_P(TP_INV);
  switch (size) {
    case 4: te_inv_gen<4>(X); break;
    case 8: te_inv_gen<8>(X); break;
    case 16: te_inv_gen<16>(X); break;
    default: te_inv_gen<32>(X); break;  // 32, and 64 (the 32-point output, replicated 2x2 by the reader)
  }
}
// residual value at (y, x) of an inverse-transformed N x N block in X.R
TE_FN int te_res_at(const TeTx &X, int size, int y, int x) {
  return size == 64 ? X.R[(y >> 1) * 32 + (x >> 1)] : X.R[y * size + x];
}
