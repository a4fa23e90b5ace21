/*
 * TEST INFRASTRUCTURE ONLY -- the checker, never the thing measured or shipped.
 * Clean-room CPU restatement of Thor's per-block reconstruction hot path.
 * See thor_oracle.h for the contract; each function cites the reference
 * file:line (under /root/reference) whose behaviour it restates.
 * Arithmetic right shifts of negative ints are relied on (gcc semantics, as
 * in the reference, which is compiled by gcc -std=c99).
 */
#include "thor_oracle.h"

#include <stdlib.h>
#include <string.h>

#define CLIP255(x) ((x) < 0 ? 0 : ((x) > 255 ? 255 : (x)))
#define CLIP16(x) ((x) < -32768 ? -32768 : ((x) > 32767 ? 32767 : (x)))
#define MIN(a, b) ((a) < (b) ? (a) : (b))
#define MAX(a, b) ((a) > (b) ? (a) : (b))

static int ilog2(int x) {
  int r = 0;
  while (x > 1) { x >>= 1; r++; }
  return r;
}
static inline int16_t wrap16(int v) { return (int16_t)(uint16_t)(v & 0xffff); }

/* ------------------------------------------------------------------------ *
 * Motion compensation
 * ------------------------------------------------------------------------ */

/* 6-tap luma filters, common/inter_prediction.c:47-59.  Table selected by the
 * sequence-level bipred flag (dec/decode_block.c:174). */
static const int luma_uni[4][6] = {
    {0, 0, 64, 0, 0, 0}, {1, -7, 55, 19, -5, 1}, {1, -7, 38, 38, -7, 1}, {1, -5, 19, 55, -7, 1}};
static const int luma_bi[4][6] = {
    {0, 0, 64, 0, 0, 0}, {2, -10, 59, 17, -5, 1}, {1, -8, 39, 39, -8, 1}, {1, -5, 17, 59, -10, 2}};
/* 4-tap 1/8-pel chroma filters, common/inter_prediction.c:61-70 */
static const int chroma_f[8][4] = {{0, 64, 0, 0},    {-2, 58, 10, -2}, {-4, 54, 16, -2}, {-4, 44, 28, -4},
                                   {-4, 36, 36, -4}, {-4, 28, 44, -4}, {-2, 16, 54, -4}, {-2, 10, 58, -2}};

/* get_inter_prediction_luma, common/inter_prediction.c:120-180 */
void or_mc_luma(uint8_t *pb, int ps, const uint8_t *ref, int rs, int w, int h, int mvx, int mvy, int sign,
                int bipred) {
  if (sign) { mvx = -mvx; mvy = -mvy; }
  int fy = mvy & 3, fx = mvx & 3;
  const uint8_t *r = ref + (mvy >> 2) * rs + (mvx >> 2);
  if (!fx && !fy) {
    for (int i = 0; i < h; i++) memcpy(pb + i * ps, r + i * rs, w);
    return;
  }
  if (fx == 2 && fy == 2) { /* (2,2) low-pass centre, :145-157 */
    static const int k[4][4] = {{0, 1, 1, 0}, {1, 2, 2, 1}, {1, 2, 2, 1}, {0, 1, 1, 0}};
    for (int i = 0; i < h; i++)
      for (int j = 0; j < w; j++) {
        int s = 0;
        for (int a = 0; a < 4; a++)
          for (int b = 0; b < 4; b++) s += k[a][b] * r[(i + a - 1) * rs + j + b - 1];
        pb[i * ps + j] = (uint8_t)CLIP255((s + 8) >> 4);
      }
    return;
  }
  const int *fv = (bipred ? luma_bi : luma_uni)[fy];
  const int *fh = (bipred ? luma_bi : luma_uni)[fx];
  /* vertical into an int32 temporary over columns -2..w+2, then horizontal */
  for (int i = 0; i < h; i++)
    for (int j = 0; j < w; j++) {
      int s = 0;
      for (int m = 0; m < 6; m++) {
        int t = 0;
        for (int n = 0; n < 6; n++) t += fv[n] * r[(i + n - 2) * rs + j + m - 2];
        s += fh[m] * t;
      }
      pb[i * ps + j] = (uint8_t)CLIP255((s + 2048) >> 12);
    }
}

/* get_inter_prediction_chroma, common/inter_prediction.c:72-118: the luma MV
 * read as 1/8-pel on the chroma plane. */
void or_mc_chroma(uint8_t *pb, int ps, const uint8_t *ref, int rs, int w, int h, int mvx, int mvy, int sign) {
  if (sign) { mvx = -mvx; mvy = -mvy; }
  int fy = mvy & 7, fx = mvx & 7;
  const uint8_t *r = ref + (mvy >> 3) * rs + (mvx >> 3);
  if (!fx && !fy) {
    for (int i = 0; i < h; i++) memcpy(pb + i * ps, r + i * rs, w);
    return;
  }
  for (int i = 0; i < h; i++)
    for (int j = 0; j < w; j++) {
      int s = 0;
      for (int m = 0; m < 4; m++) {
        int t = 0;
        for (int n = 0; n < 4; n++) t += chroma_f[fx][n] * r[(i + m - 1) * rs + j + n - 1];
        s += chroma_f[fy][m] * t;
      }
      pb[i * ps + j] = (uint8_t)CLIP255((s + 2048) >> 12);
    }
}

/* ------------------------------------------------------------------------ *
 * Quantisation / transforms
 * ------------------------------------------------------------------------ */
static const int dequant_scale[6] = {40, 45, 51, 57, 64, 72}; /* gdequant_table, common/common_block.c:98 */
static const int quant_scale[6] = {26214, 23302, 20560, 18396, 16384, 14564}; /* gquant_table :97 */

/* dequantize, common/common_block.c:132-146 (int16 truncating store) */
void or_dequantize(const int16_t *coeff, int16_t *rcoeff, int qp, int size) {
  int rshift = ilog2(size) - 1;
  int lshift = qp / 6;
  int scale = dequant_scale[qp % 6];
  int add = 1 << (rshift - 1);
  for (int i = 0; i < size * size; i++) rcoeff[i] = wrap16(((coeff[i] * scale) * (1 << lshift) + add) >> rshift);
}

/* HEVC integer DCT basis (the g*mat_hevc tables, common/transform.c:41-245):
 * row k of the N-point matrix is row k*32/N of the 32-point matrix, whose
 * entries are the published H.265 constants for cos(theta*pi/64). */
static const int cos64[33] = {64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67, 64,
                              61, 57, 54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9,  4,  0};
static int dct32(int k, int n) {
  if (k == 0) return 64;
  int t = (k * (2 * n + 1)) % 128;
  if (t <= 32) return cos64[t];
  if (t <= 64) return -cos64[64 - t];
  if (t <= 96) return -cos64[t - 64];
  return cos64[128 - t];
}
static int dctN(int N, int k, int n) { return dct32(k * (32 / N), n); }

/* inverse_transform_non_simd, common/transform.c:432-486, and the size-64
 * path of inverse_transform :488-518 (32-point on the top-left 32x32
 * coefficients, then 2x2 pixel replication).  Only the first min(N,16)
 * coefficient rows/columns take part (the partial butterflies :332-430 are
 * exactly this sum). */
void or_inverse_transform(const int16_t *coeff, int16_t *block, int size) {
  int N = size == 64 ? 32 : size;
  int cs = size; /* coefficient stride */
  int q = MIN(N, 16);
  int tmp[16][32];
  for (int i = 0; i < q; i++) /* coefficient column i */
    for (int j = 0; j < N; j++) {
      int s = 0;
      for (int k = 0; k < q; k++) s += dctN(N, k, j) * coeff[k * cs + i];
      tmp[i][j] = CLIP16((s + 64) >> 7);
    }
  int16_t out[32 * 32];
  for (int i = 0; i < N; i++)
    for (int j = 0; j < N; j++) {
      int s = 0;
      for (int k = 0; k < q; k++) s += dctN(N, k, j) * tmp[k][i];
      out[i * N + j] = (int16_t)CLIP16((s + 2048) >> 12);
    }
  if (size == 64) {
    for (int i = 0; i < 64; i++)
      for (int j = 0; j < 64; j++) block[i * 64 + j] = out[(i >> 1) * 32 + (j >> 1)];
  } else {
    memcpy(block, out, sizeof(int16_t) * N * N);
  }
}

/* One forward 8-point pass as the reference's SIMD kernel computes it
 * (transform8, common/common_kernels.c:1887-1967): the even/odd butterfly sums
 * E, O and EO are formed in 16-bit lanes (v128_add_16 / v128_sub_16) and wrap;
 * products and the final sums are 32-bit; results are stored as the low 16
 * bits (v128_unziplo_16).  Output is transposed (dst[k*8 + row]). */
static void fwd8_simd_pass(const int16_t *src, int16_t *dst, int shift) {
  int rnd = 1 << (shift - 1);
  for (int row = 0; row < 8; row++) {
    const int16_t *s = src + row * 8;
    int16_t E[4], O[4];
    for (int k = 0; k < 4; k++) {
      E[k] = wrap16(s[k] + s[7 - k]);
      O[k] = wrap16(s[k] - s[7 - k]);
    }
    int16_t EO0 = wrap16(E[0] - E[3]), EO1 = wrap16(E[1] - E[2]);
    int v[8];
    v[0] = 64 * E[0] + 64 * E[1] + 64 * E[2] + 64 * E[3];
    v[4] = 64 * E[0] - 64 * E[1] - 64 * E[2] + 64 * E[3];
    v[2] = 83 * EO0 + 36 * EO1;
    v[6] = 36 * EO0 - 83 * EO1;
    v[1] = 89 * O[0] + 75 * O[1] + 50 * O[2] + 18 * O[3];
    v[3] = 75 * O[0] - 18 * O[1] - 89 * O[2] - 50 * O[3];
    v[5] = 50 * O[0] - 89 * O[1] + 18 * O[2] + 75 * O[3];
    v[7] = 18 * O[0] - 50 * O[1] + 75 * O[2] - 89 * O[3];
    for (int k = 0; k < 8; k++) dst[k * 8 + row] = wrap16((v[k] + rnd) >> shift);
  }
}

/* transform, common/transform.c:249-330 (low-frequency min(N,16)^2 only; the
 * rest of coeff is left untouched).  The reference build runs the SIMD path
 * (transform_simd, common/common_kernels.c:2176-2250), which equals this C
 * restatement for every size except 8x8, where the SIMD 16-bit butterfly is
 * restated by fwd8_simd_pass. */
void or_transform(const int16_t *block, int16_t *coeff, int size, int fast) {
  int dsize = size;
  int lg = ilog2(size);
  int shift1 = lg, shift2 = lg + 5;
  int qsize = MIN(size, 16);
  int N = size;
  static int16_t tmp2[32 * 32];
  const int16_t *in = block;
  if (size == 8) {
    int16_t t[64], c[64];
    fwd8_simd_pass(block, t, shift1);
    fwd8_simd_pass(t, c, shift2);
    memcpy(coeff, c, sizeof(c));
    return;
  }
  if (size > 16 && fast) {
    N = 16;
    shift1 += 1 + (size == 64);
    shift2 = 9;
    int f = size / 16;
    for (int i = 0; i < 16; i++)
      for (int j = 0; j < 16; j++) {
        int s = 0;
        for (int a = 0; a < f; a++)
          for (int b = 0; b < f; b++) s += block[(i * f + a) * size + j * f + b];
        tmp2[i * 16 + j] = wrap16(s);
      }
    in = tmp2;
  } else if (size == 64) {
    N = 32;
    shift1 = 7;
    shift2 = 10;
    for (int i = 0; i < 32; i++)
      for (int j = 0; j < 32; j++)
        tmp2[i * 32 + j] = wrap16(block[(2 * i) * 64 + 2 * j] + block[(2 * i + 1) * 64 + 2 * j] +
                                  block[(2 * i) * 64 + 2 * j + 1] + block[(2 * i + 1) * 64 + 2 * j + 1]);
    in = tmp2;
  }
  int add1 = 1 << (shift1 - 1), add2 = 1 << (shift2 - 1);
  static int16_t tmp[64][64];
  for (int i = 0; i < qsize; i++)
    for (int j = 0; j < N; j++) {
      int s = 0;
      for (int k = 0; k < N; k++) s += dctN(N, i, k) * in[j * N + k];
      tmp[i][j] = wrap16((s + add1) >> shift1);
    }
  for (int i = 0; i < qsize; i++)
    for (int j = 0; j < qsize; j++) {
      int s = 0;
      for (int k = 0; k < N; k++) s += dctN(N, i, k) * tmp[j][k];
      coeff[i * dsize + j] = wrap16((s + add2) >> shift2);
    }
}

static const int zz16[16] = {0, 1, 5, 6, 2, 4, 7, 12, 3, 8, 11, 13, 9, 10, 14, 15};
/* zigzag64/zigzag256 of common/common_block.c:45-73 are the same diagonal
 * scan; generated here: anti-diagonals alternating direction. */
static void make_zigzag(int n, int *zz) {
  int idx = 0;
  for (int d = 0; d < 2 * n - 1; d++) {
    if (d % 2 == 0) { /* up-right: from bottom-left to top-right */
      for (int i = MIN(d, n - 1); i >= 0 && d - i < n; i--) zz[i * n + (d - i)] = idx++;
    } else {
      for (int i = MAX(0, d - n + 1); i <= d && i < n; i++) zz[i * n + (d - i)] = idx++;
    }
  }
}

/* quantize, enc/encode_block.c:75-172 (rdoq = 0, the default of every
 * configuration used here, enc/strings.c:331).  Writes the low-frequency
 * qsize^2 corner of coeffq; returns cbp. */
int or_quantize(const int16_t *coeff, int16_t *coeffq, int qp, int size, int coeff_block_type) {
  int intra_block = (coeff_block_type >> 1) & 1;
  int chroma_flag = coeff_block_type & 1;
  int lg = ilog2(size);
  int qsize = MIN(16, size);
  int scale = quant_scale[qp % 6];
  int shift2 = 21 - lg + qp / 6;
  int zz[256];
  if (qsize == 4) memcpy(zz, zz16, sizeof(zz16));
  else make_zigzag(qsize, zz);
  int sc[256], sq[256];
  memset(sq, 0, sizeof(sq));
  for (int i = 0; i < qsize; i++)
    for (int j = 0; j < qsize; j++) sc[zz[i * qsize + j]] = coeff[i * size + j];
  int offset = (intra_block ? 38 : -26) * (1 << (shift2 - 8));
  int level = 0, pos = qsize * qsize - 1;
  while (level == 0 && pos >= 0) {
    level = abs(abs(sc[pos]) * scale + offset) >> shift2;
    pos--;
  }
  int last_pos = level ? pos + 1 : pos;
  int cbp = 0;
  int off0 = intra_block ? 102 : 51, off1 = intra_block ? 115 : 90;
  for (pos = 0; pos <= last_pos; pos++) {
    int c = sc[pos];
    int sgn = c < 0 ? -1 : 1;
    int ac = scale * abs(c);
    int l0 = ac >> shift2;
    int off = ((l0 == 0 || chroma_flag) ? off0 : off1) * (1 << (shift2 - 8));
    int l = (ac + off) >> shift2;
    sq[pos] = sgn * l;
    cbp = cbp || (l != 0);
  }
  if (cbp) { /* "RDOQ light", :134-168 */
    int N = chroma_flag ? last_pos + 1 : qsize * qsize;
    for (pos = 2; pos < N; pos++) {
      int flag = 1;
      if (pos > 2 && abs(sq[pos - 3]) > 1) flag = 0;
      if (pos > 3 && abs(sq[pos - 4]) > 1 && abs(sq[pos - 3]) > 0) flag = 0;
      if (pos == 2 && (chroma_flag == 0 || last_pos >= 6)) flag = 0;
      if (flag && sq[pos - 2] == 0 && sq[pos - 1] == 0 && abs(sq[pos]) > 1) {
        int K1 = abs(sc[pos]), K2 = abs(sc[pos - 1]), K3 = abs(sc[pos - 2]);
        int K4 = MAX(K2, K3);
        int thr = (73 * dequant_scale[qp % 6] << (qp / 6)) >> (4 + lg);
        if (K1 + K4 < thr) sq[pos] = sc[pos] < 0 ? -1 : 1;
        else if (K2 > K3) sq[pos - 1] = sc[pos - 1] < 0 ? -1 : 1;
        else sq[pos - 2] = sc[pos - 2] < 0 ? -1 : 1;
      }
    }
  }
  for (int i = 0; i < qsize; i++)
    for (int j = 0; j < qsize; j++) coeffq[i * size + j] = (int16_t)sq[zz[i * qsize + j]];
  return cbp != 0;
}

/* reconstruct_block, common/common_block.c:148-156 */
void or_reconstruct_block(const int16_t *block, const uint8_t *pblock, uint8_t *rec, int size, int stride) {
  for (int i = 0; i < size; i++)
    for (int j = 0; j < size; j++) rec[i * stride + j] = (uint8_t)CLIP255(block[i * size + j] + pblock[i * size + j]);
}

uint32_t or_sad(const uint8_t *a, const uint8_t *b, int as, int bs, int w, int h) {
  uint32_t s = 0; /* sad_calc, enc/encode_block.c:497-509 */
  for (int i = 0; i < h; i++)
    for (int j = 0; j < w; j++) s += abs(a[i * as + j] - b[i * bs + j]);
  return s;
}
uint32_t or_ssd(const uint8_t *a, const uint8_t *b, int as, int bs, int w, int h) {
  uint32_t s = 0; /* ssd_calc, enc/encode_block.c:783-797 */
  for (int i = 0; i < h; i++)
    for (int j = 0; j < w; j++) {
      int d = a[i * as + j] - b[i * bs + j];
      s += (uint32_t)(d * d);
    }
  return s;
}

/* ------------------------------------------------------------------------ *
 * Intra prediction
 * ------------------------------------------------------------------------ */

/* get_upright_available / get_downleft_available, common/common_block.c:110-129 */
int or_upright_available(int ypos, int xpos, int size, int width) {
  int a = (ypos > 0) && (xpos + size < width);
  if (size == 32 && (ypos % 64) == 32) a = 0;
  if (size == 16 && ((ypos % 32) == 16 || ((ypos % 64) == 32 && (xpos % 32) == 16))) a = 0;
  if (size == 8 && ((ypos % 16) == 8 || ((ypos % 32) == 16 && (xpos % 16) == 8) || ((ypos % 64) == 32 && (xpos % 32) == 24)))
    a = 0;
  return a;
}
int or_downleft_available(int ypos, int xpos, int size, int height) {
  int a = (xpos > 0) && (ypos + size < height);
  if (size == 64) a = 0;
  if (size == 32 && (ypos % 64) == 32) a = 0;
  if (size == 16 && ((ypos % 64) == 48 || ((ypos % 64) == 16 && (xpos % 32) == 16))) a = 0;
  if (size == 8 && ((ypos % 64) == 56 || ((ypos % 16) == 8 && (xpos % 16) == 8) || ((ypos % 64) == 24 && (xpos % 32) == 16)))
    a = 0;
  return a;
}

/* make_top_and_left, common/intra_prediction.c:57-143.  rec_frame points at
 * the CU origin; rblock at the sub-TU origin (tb_split). */
void or_make_top_and_left(uint8_t *left, uint8_t *top, uint8_t *top_left, const uint8_t *rf, int fs,
                          const uint8_t *rb, int rbs, int i, int j, int ypos, int xpos, int size, int cb_ur, int cb_dl,
                          int tb_split) {
  int len = 2 * size;
  int dl, ur;
  if (!tb_split) {
    dl = cb_dl;
    ur = cb_ur;
    int leftlen = dl ? size + 1 : size, toplen = ur ? size + 1 : size;
    if (ypos == 0) {
      memset(top, 128, len);
      *top_left = 128;
    } else {
      memcpy(top, rf - fs, toplen);
      memset(top + size, top[toplen - 1], size);
      *top_left = xpos > 0 ? rf[-fs - 1] : top[0];
    }
    if (xpos == 0) memset(left, 128, len);
    else {
      for (int k = 0; k < leftlen; k++) left[k] = rf[k * fs - 1];
      memset(left + size, left[leftlen - 1], size);
    }
    if (ypos == 0) *top_left = left[0];
  } else {
    dl = (j == 0 && (i == 0 || cb_dl)) ? 1 : 0;
    ur = (j == 0 || (i == 0 && cb_ur)) ? 1 : 0;
    int leftlen = dl ? size + 1 : size, toplen = ur ? size + 1 : size;
    if (ypos + i == 0) {
      memset(top, 128, len);
      *top_left = 128;
    } else if (i == 0) {
      memcpy(top, rf - fs + j, toplen);
      memset(top + size, top[toplen - 1], size);
      *top_left = xpos > 0 ? rf[-fs + j - 1] : top[0];
    } else {
      memcpy(top, rb - rbs, toplen);
      memset(top + size, top[toplen - 1], size);
      *top_left = xpos > 0 ? (j > 0 ? rb[-rbs - 1] : rf[(i - 1) * fs - 1]) : top[0];
    }
    if (xpos + j == 0) memset(left, 128, len);
    else if (j == 0) {
      for (int k = 0; k < leftlen; k++) left[k] = rf[(i + k) * fs - 1];
      memset(left + size, left[leftlen - 1], size);
    } else {
      for (int k = 0; k < leftlen; k++) left[k] = rb[k * rbs - 1];
      memset(left + size, left[leftlen - 1], size);
    }
    if (ypos + i == 0) *top_left = left[0];
  }
}

/* filter_121, common/intra_prediction.c:39-48 */
static void f121(const uint8_t *in, uint8_t *out, int len) {
  out[0] = (uint8_t)((3 * in[0] + in[1] + 2) >> 2);
  for (int j = 1; j < len - 1; j++) out[j] = (uint8_t)((in[j - 1] + 2 * in[j] + in[j + 1] + 2) >> 2);
  out[len - 1] = (uint8_t)((in[len - 2] + 3 * in[len - 1] + 2) >> 2);
}

/* get_intra_prediction and the ten mode functions, common/intra_prediction.c:145-388 */
void or_intra_pred(const uint8_t *left, const uint8_t *top, uint8_t tl, int ypos, int xpos, int n, uint8_t *pb,
                   int mode) {
  uint8_t lF[128], tF[128], tlF;
  switch (mode) {
    case 1: { /* planar, :182-214 -- C division truncates toward zero */
      int T[64], L[64];
      for (int s = 0; s < 2; s++) {
        const uint8_t *a = s ? left : top;
        int *F = s ? L : T;
        F[0] = 3 * a[0] + 2 * a[0] + 2 * a[1] + a[2];
        F[1] = a[0] + 2 * a[0] + 2 * a[1] + 2 * a[2] + a[3];
        for (int j = 2; j < n - 2; j++) F[j] = a[j - 2] + 2 * a[j - 1] + 2 * a[j] + 2 * a[j + 1] + a[j + 2];
        F[n - 2] = a[n - 4] + 2 * a[n - 3] + 2 * a[n - 2] + 2 * a[n - 1] + a[n - 1];
        F[n - 1] = a[n - 3] + 2 * a[n - 2] + 2 * a[n - 1] + 3 * a[n - 1];
      }
      int TL = left[1] + 2 * left[0] + 2 * tl + 2 * top[0] + top[1];
      for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
          int v = (L[i] + T[j] - TL + 4) / 8;
          pb[i * n + j] = (uint8_t)CLIP255(v);
        }
      return;
    }
    case 2: /* horizontal */
      for (int i = 0; i < n; i++) memset(pb + i * n, left[i], n);
      return;
    case 3: /* vertical */
      for (int i = 0; i < n; i++) memcpy(pb + i * n, top, n);
      return;
    case 4: /* up-left, :216-240 */
      f121(left, lF, n);
      f121(top, tF, n);
      tlF = (uint8_t)((2 * tl + left[0] + top[0] + 2) >> 2);
      for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
          int d = i - j;
          pb[i * n + j] = d > 0 ? lF[d - 1] : (d == 0 ? tlF : tF[-d - 1]);
        }
      return;
    case 5: /* up-right, :242-256 */
      f121(top, tF, 2 * n);
      for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) pb[i * n + j] = tF[i + j + 1];
      return;
    case 6: /* up-up-right, :258-277 */
      f121(top, tF, 2 * n);
      for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
          int d = i + 2 * j;
          pb[i * n + j] = (d & 1) ? tF[(d + 1) / 2] : (uint8_t)((tF[d / 2] + tF[d / 2 + 1]) >> 1);
        }
      return;
    case 7: /* up-up-left, :279-307 */
      f121(left, lF, n);
      f121(top, tF, n);
      tlF = (uint8_t)((2 * tl + left[0] + top[0] + 2) >> 2);
      for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
          int d = i - 2 * j;
          uint8_t v;
          if (d > 1) v = lF[d - 2];
          else if (d == 1) v = tlF;
          else if (d == 0) v = (uint8_t)((tlF + tF[0]) >> 1);
          else if (d & 1) v = tF[(-d) / 2];
          else v = (uint8_t)((tF[(-d) / 2] + tF[(-d) / 2 - 1]) >> 1);
          pb[i * n + j] = v;
        }
      return;
    case 8: /* up-left-left, :309-337 */
      f121(left, lF, n);
      f121(top, tF, n);
      tlF = (uint8_t)((2 * tl + left[0] + top[0] + 2) >> 2);
      for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
          int d = 2 * i - j;
          uint8_t v;
          if (d < -1) v = tF[-d - 2];
          else if (d == -1) v = tlF;
          else if (d == 0) v = (uint8_t)((tlF + lF[0]) >> 1);
          else if (d & 1) v = lF[d / 2];
          else v = (uint8_t)((lF[d / 2] + lF[d / 2 - 1]) >> 1);
          pb[i * n + j] = v;
        }
      return;
    case 9: /* down-left-left, :339-361 */
      f121(left, lF, 2 * n);
      for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
          int d = 2 * i + j;
          pb[i * n + j] = (d & 1) ? lF[(d + 1) / 2] : (uint8_t)((lF[d / 2] + lF[d / 2 + 1]) >> 1);
        }
      return;
    default: { /* DC (mode 0 and out-of-range), :145-160, :363-388 */
      const uint8_t *a = xpos != 0 ? left : top;
      const uint8_t *b = ypos != 0 ? top : left;
      int s = 0;
      for (int j = 0; j < n; j++) s += a[j] + b[j];
      int dc = (s + n) / (2 * n);
      memset(pb, dc, n * n);
      return;
    }
  }
}

/* clpf_block, common/common_block.c:180-197 */
void or_clpf_block(const uint8_t *src, uint8_t *dst, int ss, int ds, int x0, int y0, int size, int width, int height) {
  int left = x0 & ~(ds - 1), top = y0 & ~(ds - 1);
  int right = MIN(width - 1, left + ds - 1), bottom = MIN(height - 1, top + ds - 1);
  for (int y = y0; y < y0 + size; y++)
    for (int x = x0; x < x0 + size; x++) {
      int X = src[y * ss + x];
      int A = y == top ? X : src[(y - 1) * ss + x];
      int B = x == left ? X : src[y * ss + x - 1];
      int C = x == right ? X : src[y * ss + x + 1];
      int D = y == bottom ? X : src[(y + 1) * ss + x];
      int delta = ((A > X) + (B > X) + (C > X) + (D > X) > 2) - ((A < X) + (B < X) + (C < X) + (D < X) > 2);
      dst[(y - top) * ds + x - left] = (uint8_t)(X + delta);
    }
}

/* ------------------------------------------------------------------------ *
 * Frame level
 * ------------------------------------------------------------------------ */
static const int chroma_qp_tab[52] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17,
                                      18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 29, 30, 31, 32, 33, 33,
                                      34, 34, 35, 35, 36, 36, 37, 37, 38, 39, 40, 41, 42, 43, 44, 45};
static const int beta_tab[52] = {0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  6,  7,
                                 8,  9,  10, 11, 12, 13, 14, 15, 16, 17, 18, 20, 22, 24, 26, 28, 30, 32,
                                 34, 36, 38, 40, 42, 44, 46, 48, 50, 52, 54, 56, 58, 60, 62, 64};
static const int tc_tab[56] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1,  1,  1,  1,  1,  1,  1,  1,  1, 2,
                               2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 5, 5, 6, 6, 7, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13, 14, 14};

/* per-4x4 side info as copy_deblock_data (dec/decode_block.c:122-156) stores it */
typedef or_cell_t dbinfo_t;

static void fill_dbinfo(dbinfo_t *db, int bstride, const thor_block_t *b) {
  int size = b->size;
  int div = size / 8;
  int pb_part = b->mode == 2 ? b->pb_part : 0;
  for (int m = 0; m < b->bheight / 4; m++)
    for (int n = 0; n < b->bwidth / 4; n++) {
      int m0 = div > 0 ? m / div : 0, n0 = div > 0 ? n / div : 0;
      int idx = 2 * m0 + n0;
      dbinfo_t *d = &db[(b->ypos / 4 + m) * bstride + b->xpos / 4 + n];
      d->mode = b->mode;
      d->cbp_y = b->cbp_y;
      d->cbp_u = b->cbp_u;
      d->cbp_v = b->cbp_v;
      d->size = (uint8_t)size;
      d->tb_split = b->tb_split > 0;
      d->pb_part = (uint8_t)pb_part;
      d->mv0x = b->mv0[2 * idx];
      d->mv0y = b->mv0[2 * idx + 1];
      d->mv1x = b->mv1[2 * idx];
      d->mv1y = b->mv1[2 * idx + 1];
    }
}

/* deblock_frame_y, common/common_frame.c:46-241 (NEW_DEBLOCK_TEST,
 * NEW_MV_TEST, NEW_DEBLOCK_FILTER all 1: common/global.h:88-90) */
static void deblock_y(uint8_t *Y, int s, const dbinfo_t *db, int width, int height, int qp) {
  int beta = beta_tab[qp], tc = tc_tab[qp];
  int bs = width / 4;
  for (int pass = 0; pass < 2; pass++) {
    int i0 = pass ? 8 : 0, j0 = pass ? 0 : 8;
    for (int i = i0; i < height; i += 8)
      for (int j = j0; j < width; j += 8) {
        /* sample pointer p(a, t): pixel at distance a across the edge (a<0: p side), t along it */
#define PX(a, t) (*(pass ? &Y[(i + (a)) * s + j + (t)] : &Y[(i + (t)) * s + j + (a)]))
        int d = abs(PX(-2, 2) - PX(-1, 2)) + abs(PX(1, 2) - PX(0, 2)) + abs(PX(-2, 5) - PX(-1, 5)) +
                abs(PX(1, 5) - PX(0, 5));
        for (int m = 0; m < 8; m += 4) {
          int qi = pass ? (i / 4) * bs + (j + m) / 4 : ((i + m) / 4) * bs + j / 4;
          int pi = pass ? qi - bs : qi - 1;
          const dbinfo_t *P = &db[pi], *Q = &db[qi];
          int qsize = Q->size;
          int part_split = pass ? (Q->pb_part == 1 || Q->pb_part == 3) : (Q->pb_part == 2 || Q->pb_part == 3);
          if ((Q->tb_split || part_split) && qsize > 8) qsize /= 2;
          int mv = abs(P->mv0y) >= 4 || abs(Q->mv0y) >= 4 || abs(P->mv0x) >= 4 || abs(Q->mv0x) >= 4 ||
                   abs(P->mv1y) >= 4 || abs(Q->mv1y) >= 4 || abs(P->mv1x) >= 4 || abs(Q->mv1x) >= 4;
          int cbp = P->cbp_y || Q->cbp_y;
          int intra = P->mode == 1 || Q->mode == 1;
          int interior = (pass ? i : j) % qsize > 0;
          if (d < beta && !interior && (mv || cbp || intra)) {
            for (int t = m; t < m + 4; t++) {
              int p1 = PX(-2, t), p0 = PX(-1, t), q0 = PX(0, t), q1 = PX(1, t);
              int delta = (18 * (q0 - p0) - 6 * (q1 - p1) + 16) >> 5;
              delta = delta < -tc ? -tc : (delta > tc ? tc : delta);
              PX(-2, t) = (uint8_t)CLIP255(p1 + delta / 2);
              PX(-1, t) = (uint8_t)CLIP255(p0 + delta);
              PX(0, t) = (uint8_t)CLIP255(q0 - delta);
              PX(1, t) = (uint8_t)CLIP255(q1 - delta / 2);
            }
          }
        }
#undef PX
      }
  }
}

/* deblock_frame_uv, common/common_frame.c:243-321 */
static void deblock_uv(uint8_t *C, int s, const dbinfo_t *db, int width, int height, int qp) {
  int tc = tc_tab[qp];
  int bs = width / 4;
  for (int pass = 0; pass < 2; pass++) {
    int i0 = pass ? 8 : 0, j0 = pass ? 0 : 8;
    for (int i = i0; i < height; i += 8)
      for (int j = j0; j < width; j += 8) {
        int i2 = i / 2, j2 = j / 2;
        int qi = (i / 4) * bs + j / 4;
        int pi = pass ? qi - bs : qi - 1;
        int intra = db[pi].mode == 1 || db[qi].mode == 1;
        int interior = (pass ? i : j) % db[qi].size > 0;
        if (!interior && intra) {
          for (int t = 0; t < 4; t++) {
#define PC(a) (*(pass ? &C[(i2 + (a)) * s + j2 + t] : &C[(i2 + t) * s + j2 + (a)]))
            int p1 = PC(-2), p0 = PC(-1), q0 = PC(0), q1 = PC(1);
            int delta = (4 * (q0 - p0) + (p1 - q1) + 4) >> 3;
            delta = delta < -tc ? -tc : (delta > tc ? tc : delta);
            PC(-1) = (uint8_t)CLIP255(p0 + delta);
            PC(0) = (uint8_t)CLIP255(q0 - delta);
#undef PC
          }
        }
      }
  }
}

/* clpf_frame, common/common_frame.c:485-557 (floor SB counts, :496-497) */
static void clpf_frame(or_frame_t *f, const dbinfo_t *db, int width, int height, const uint8_t *flags) {
  int nh = width / 64, nv = height / 64;
  int bs = width / 4;
  uint8_t tmp[64 * 64 * 3 / 2];
  for (int k = 0; k < nv; k++)
    for (int l = 0; l < nh; l++) {
      int cand = 0;
      for (int m = 0; m < 8; m++)
        for (int n = 0; n < 8; n++) {
          const dbinfo_t *d = &db[((k * 64 + m * 8) / 4) * bs + (l * 64 + n * 8) / 4];
          cand |= d->mode != 3 && (d->cbp_y || d->cbp_u || d->cbp_v);
        }
      if (!(cand && flags[k * nh + l])) continue;
      for (int m = 0; m < 64; m++) memcpy(tmp + m * 64, f->y + (k * 64 + m) * f->stride_y + l * 64, 64);
      for (int m = 0; m < 32; m++) {
        memcpy(tmp + 4096 + m * 32, f->u + (k * 32 + m) * f->stride_c + l * 32, 32);
        memcpy(tmp + 5120 + m * 32, f->v + (k * 32 + m) * f->stride_c + l * 32, 32);
      }
      for (int m = 0; m < 8; m++)
        for (int n = 0; n < 8; n++) {
          int xpos = l * 64 + n * 8, ypos = k * 64 + m * 8;
          const dbinfo_t *d = &db[(ypos / 4) * bs + xpos / 4];
          if (d->mode == 3) continue;
          if (d->cbp_y) or_clpf_block(f->y, tmp, f->stride_y, 64, xpos, ypos, 8, width, height);
          if (d->cbp_u) or_clpf_block(f->u, tmp + 4096, f->stride_c, 32, xpos / 2, ypos / 2, 4, width / 2, height / 2);
          if (d->cbp_v) or_clpf_block(f->v, tmp + 5120, f->stride_c, 32, xpos / 2, ypos / 2, 4, width / 2, height / 2);
        }
      for (int m = 0; m < 64; m++) memcpy(f->y + (k * 64 + m) * f->stride_y + l * 64, tmp + m * 64, 64);
      for (int m = 0; m < 32; m++) {
        memcpy(f->u + (k * 32 + m) * f->stride_c + l * 32, tmp + 4096 + m * 32, 32);
        memcpy(f->v + (k * 32 + m) * f->stride_c + l * 32, tmp + 5120 + m * 32, 32);
      }
    }
}

/* pad_yuv_frame, common/common_frame.c:405-462 */
void or_pad_frame(or_frame_t *f, int w, int h, int py, int pc) {
  for (int c = 0; c < 3; c++) {
    uint8_t *p = c == 0 ? f->y : (c == 1 ? f->u : f->v);
    int s = c == 0 ? f->stride_y : f->stride_c;
    int pw = c == 0 ? w : w / 2, ph = c == 0 ? h : h / 2, pad = c == 0 ? py : pc;
    for (int i = 0; i < ph; i++) {
      memset(p + i * s - pad, p[i * s], pad);
      memset(p + i * s + pw, p[i * s + pw - 1], pad);
    }
    for (int i = -pad; i < 0; i++) memcpy(p + i * s - pad, p - pad, pw + 2 * pad);
    for (int i = ph; i < ph + pad; i++) memcpy(p + i * s - pad, p + (ph - 1) * s - pad, pw + 2 * pad);
  }
}

static const or_frame_t *find_ref(const or_frame_t *refs, int nrefs, int frame_num) {
  for (int r = 0; r < nrefs; r++)
    if (refs[r].frame_num == frame_num) return &refs[r];
  return NULL;
}

/* compact coefficient slots of one component -> N x N TU(s) as read_block leaves them */
static void expand_tu(const int16_t *pool, int16_t *tu, int n, int q) {
  memset(tu, 0, sizeof(int16_t) * n * n);
  for (int r = 0; r < q; r++) memcpy(tu + r * n, pool + r * q, sizeof(int16_t) * q);
}

/* dequantize + inverse_transform of one N x N TU from compact slots */
static void residual_tu(const int16_t *pool, int n, int qp, int16_t *res) {
  int16_t c[64 * 64], rc[64 * 64];
  expand_tu(pool, c, n, MIN(n, 16));
  or_dequantize(c, rc, qp, n);
  or_inverse_transform(rc, res, n);
}

/* decode_and_reconstruct_block_inter, dec/decode_block.c:90-120 */
static void recon_inter_comp(uint8_t *rec, int stride, int size, int qp, const uint8_t *pb, const int16_t *pool,
                             int has_coeff, int tb_split) {
  int16_t res[64 * 64];
  if (!has_coeff) memset(res, 0, sizeof(int16_t) * size * size);
  else if (tb_split) {
    int h = size / 2, q = MIN(h, 16);
    int16_t r2[32 * 32];
    for (int t = 0; t < 4; t++) {
      residual_tu(pool + t * q * q, h, qp, r2);
      int oi = (t >> 1) * h, oj = (t & 1) * h;
      for (int k = 0; k < h; k++) memcpy(res + (oi + k) * size + oj, r2 + k * h, sizeof(int16_t) * h);
    }
  } else {
    residual_tu(pool, size, qp, res);
  }
  or_reconstruct_block(res, pb, rec, size, stride);
}

/* decode_and_reconstruct_block_intra, dec/decode_block.c:48-88 */
static void recon_intra_comp(uint8_t *rec, int stride, int size, int qp, const int16_t *pool, int has_coeff,
                             int tb_split, int ur, int dl, int mode, int ypos, int xpos) {
  uint8_t leftb[130], topb[130], tl;
  uint8_t *left = leftb + 1, *top = topb + 1;
  uint8_t pb[64 * 64];
  int16_t res[64 * 64];
  if (tb_split) {
    int h = size / 2, q = MIN(h, 16);
    for (int i = 0; i < size; i += h)
      for (int j = 0; j < size; j += h) {
        or_make_top_and_left(left, top, &tl, rec, stride, rec + i * stride + j, stride, i, j, ypos, xpos, h, ur, dl, 1);
        or_intra_pred(left, top, tl, ypos + i, xpos + j, h, pb, mode);
        int t = 2 * (i / h) + j / h;
        if (has_coeff) residual_tu(pool + t * q * q, h, qp, res);
        else memset(res, 0, sizeof(int16_t) * h * h);
        or_reconstruct_block(res, pb, rec + i * stride + j, h, stride);
      }
  } else {
    or_make_top_and_left(left, top, &tl, rec, stride, NULL, 0, 0, 0, ypos, xpos, size, ur, dl, 0);
    or_intra_pred(left, top, tl, ypos, xpos, size, pb, mode);
    if (has_coeff) residual_tu(pool, size, qp, res);
    else memset(res, 0, sizeof(int16_t) * size * size);
    or_reconstruct_block(res, pb, rec, size, stride);
  }
}

int or_decode_frame(const thor_seq_t *seq, const thor_frame_hdr_t *hdr, or_frame_t *cur, const or_frame_t *refs,
                    int nrefs, const thor_block_t *blocks, int nblocks, const int16_t *coeffs,
                    const uint8_t *clpf_flags, int stop_stage) {
  int W = seq->width, H = seq->height;
  int bstride = W / 4;
  dbinfo_t *db = calloc((size_t)(H / 4) * bstride, sizeof(dbinfo_t));
  if (!db) return THOR_ERR_NOMEM;
  uint8_t *p0 = malloc(3 * 64 * 64), *p1 = malloc(3 * 64 * 64), *pb = malloc(3 * 64 * 64);
  int err = 0;
  for (int bi = 0; bi < nblocks && !err; bi++) {
    const thor_block_t *b = &blocks[bi];
    int S = b->size, C = S / 2;
    int x = b->xpos, y = b->ypos;
    uint8_t *ry = cur->y + y * cur->stride_y + x;
    uint8_t *ru = cur->u + (y / 2) * cur->stride_c + x / 2;
    uint8_t *rv = cur->v + (y / 2) * cur->stride_c + x / 2;
    int qpy = b->qp, qpc = chroma_qp_tab[b->qp];
    if (b->mode == 1) { /* MODE_INTRA */
      int ur = or_upright_available(y, x, S, W), dl = or_downleft_available(y, x, S, H);
      int tbc = b->tb_split && S > 8;
      recon_intra_comp(ry, cur->stride_y, S, qpy, coeffs + b->coeff_off[0], b->coeff_mask & 1, b->tb_split, ur, dl,
                       b->intra_mode, y, x);
      recon_intra_comp(ru, cur->stride_c, C, qpc, coeffs + b->coeff_off[1], b->coeff_mask & 2, tbc, ur, dl,
                       b->intra_mode, y / 2, x / 2);
      recon_intra_comp(rv, cur->stride_c, C, qpc, coeffs + b->coeff_off[2], b->coeff_mask & 4, tbc, ur, dl,
                       b->intra_mode, y / 2, x / 2);
    } else {
      const or_frame_t *r0 = find_ref(refs, nrefs, b->ref0);
      int bi_dir = (b->mode == 3) || ((b->mode == 0 || b->mode == 4) && b->dir == 2);
      const or_frame_t *r1 = bi_dir ? find_ref(refs, nrefs, b->ref1) : NULL;
      if (!r0 || (bi_dir && !r1)) { err = THOR_ERR_REF; break; }
      /* the interpolated reference (-2) carries the current frame's number
       * (dec/decode_frame.c:108), so its `sign` compares equal */
      const int fn0 = b->ref0 == -2 ? hdr->frame_num : b->ref0, fn1 = b->ref1 == -2 ? hdr->frame_num : b->ref1;
      int sign0 = bi_dir ? (fn0 >= hdr->frame_num) : (fn0 > hdr->frame_num);
      int sign1 = bi_dir ? (fn1 >= hdr->frame_num) : 0;
      int quarters = (b->mode == 2 || b->mode == 3);
      int pw = b->mode == 0 ? b->bwidth : S, ph = b->mode == 0 ? b->bheight : S;
      for (int leg = 0; leg < (bi_dir ? 2 : 1); leg++) {
        const or_frame_t *rf = leg ? r1 : r0;
        const int16_t *mv = leg ? b->mv1 : b->mv0;
        int sg = leg ? sign1 : sign0;
        uint8_t *dy = (bi_dir ? (leg ? p1 : p0) : pb), *du = dy + 4096, *dv = dy + 4096 + 1024;
        const uint8_t *fy = rf->y + y * rf->stride_y + x;
        const uint8_t *fu = rf->u + (y / 2) * rf->stride_c + x / 2;
        const uint8_t *fv = rf->v + (y / 2) * rf->stride_c + x / 2;
        if (quarters) { /* dec/decode_block.c:362-392, :419-434 */
          int hs = S / 2, hc = C / 2;
          for (int q = 0; q < 4; q++) {
            int qx = q & 1, qy = q >> 1;
            int mx = mv[2 * q], my = mv[2 * q + 1];
            or_mc_luma(dy + qy * hs * S + qx * hs, S, fy + qy * hs * rf->stride_y + qx * hs, rf->stride_y, hs, hs, mx,
                       my, sg, seq->bipred);
            or_mc_chroma(du + qy * hc * C + qx * hc, C, fu + qy * hc * rf->stride_c + qx * hc, rf->stride_c, hc, hc, mx,
                         my, sg);
            or_mc_chroma(dv + qy * hc * C + qx * hc, C, fv + qy * hc * rf->stride_c + qx * hc, rf->stride_c, hc, hc, mx,
                         my, sg);
          }
        } else {
          or_mc_luma(dy, S, fy, rf->stride_y, pw, ph, mv[0], mv[1], sg, seq->bipred);
          or_mc_chroma(du, C, fu, rf->stride_c, pw / 2, ph / 2, mv[0], mv[1], sg);
          or_mc_chroma(dv, C, fv, rf->stride_c, pw / 2, ph / 2, mv[0], mv[1], sg);
        }
      }
      if (bi_dir) { /* truncating average, dec/decode_block.c:272-283 */
        for (int i = 0; i < 3 * 4096; i++) pb[i] = (uint8_t)((p0[i] + p1[i]) >> 1);
      }
      if (b->mode == 0) { /* SKIP: copy bwidth x bheight, no residual */
        for (int i = 0; i < b->bheight; i++) memcpy(ry + i * cur->stride_y, pb + i * S, b->bwidth);
        for (int i = 0; i < b->bheight / 2; i++) {
          memcpy(ru + i * cur->stride_c, pb + 4096 + i * C, b->bwidth / 2);
          memcpy(rv + i * cur->stride_c, pb + 5120 + i * C, b->bwidth / 2);
        }
      } else {
        int tbc = b->tb_split && S > 8;
        recon_inter_comp(ry, cur->stride_y, S, qpy, pb, coeffs + b->coeff_off[0], b->coeff_mask & 1, b->tb_split);
        recon_inter_comp(ru, cur->stride_c, C, qpc, pb + 4096, coeffs + b->coeff_off[1], b->coeff_mask & 2, tbc);
        recon_inter_comp(rv, cur->stride_c, C, qpc, pb + 5120, coeffs + b->coeff_off[2], b->coeff_mask & 4, tbc);
      }
    }
    fill_dbinfo(db, bstride, b);
  }
  if (!err && stop_stage >= 1 && seq->deblocking) {
    deblock_y(cur->y, cur->stride_y, db, W, H, hdr->qp);
    int qpc = chroma_qp_tab[hdr->qp];
    deblock_uv(cur->u, cur->stride_c, db, W, H, qpc);
    deblock_uv(cur->v, cur->stride_c, db, W, H, qpc);
  }
  if (!err && stop_stage >= 2 && seq->clpf && hdr->clpf_on && clpf_flags) clpf_frame(cur, db, W, H, clpf_flags);
  free(db);
  free(p0);
  free(p1);
  free(pb);
  return err;
}

/* One transform block of an RD candidate, as encode_and_reconstruct_block_inter
 * / _intra run it per TU (enc/encode_block.c:1434-1518): get_residual
 * (:484-493), transform, quantize (rdoq 0), then dequantize + inverse_transform
 * + reconstruct_block if cbp, else rec = pred (:1512-1517).  Writes the q x q
 * levels compact (q = min(size,16)) and returns cbp; *ssd = SSD(orig, rec)
 * (ssd_calc, :783-797). */
int or_encode_tu(const uint8_t *orig, int os, const uint8_t *pred, int ps, uint8_t *rec, int rs, int size, int qp,
                 int type, int fast, int16_t *levels, uint32_t *ssd) {
  int16_t res[64 * 64], coeff[64 * 64], coeffq[64 * 64], rco[64 * 64], rblk[64 * 64];
  uint8_t pb[64 * 64];
  int q = MIN(size, 16);
  for (int i = 0; i < size; i++)
    for (int j = 0; j < size; j++) {
      res[i * size + j] = (int16_t)(orig[i * os + j] - pred[i * ps + j]);
      pb[i * size + j] = pred[i * ps + j];
    }
  memset(coeff, 0, sizeof(coeff));
  memset(coeffq, 0, sizeof(coeffq));
  or_transform(res, coeff, size, fast);
  int cbp = or_quantize(coeff, coeffq, qp, size, type);
  for (int i = 0; i < q; i++)
    for (int j = 0; j < q; j++) levels[i * q + j] = coeffq[i * size + j];
  uint8_t out[64 * 64];
  if (cbp) {
    or_dequantize(coeffq, rco, qp, size);
    or_inverse_transform(rco, rblk, size);
    or_reconstruct_block(rblk, pb, out, size, size);
  } else {
    memcpy(out, pb, (size_t)size * size);
  }
  for (int i = 0; i < size; i++)
    for (int j = 0; j < size; j++) rec[i * rs + j] = out[i * size + j];
  *ssd = or_ssd(orig, out, os, size, size, size);
  return cbp;
}

/* scale_frame_down2x2 luma loop (common/temporal_interp.c:161-168; the SIMD
 * variant :196-210 computes the same bytes) on one plane, no padding. */
void or_scale_down2x2(const uint8_t *in, int si, uint8_t *out, int so, int wo, int ho) {
  for (int i = 0; i < ho; i++)
    for (int j = 0; j < wo; j++) {
      const int a = (in[(2 * i) * si + 2 * j] + in[(2 * i + 1) * si + 2 * j] + 1) >> 1;
      const int b = (in[(2 * i) * si + 2 * j + 1] + in[(2 * i + 1) * si + 2 * j + 1] + 1) >> 1;
      out[i * so + j] = (uint8_t)((a + b) >> 1);
    }
}

/* pad_yuv_frame's luma part (common/common_frame.c:414-430) on one plane */
void or_pad_plane(uint8_t *p, int s, int w, int h, int pad) {
  for (int i = 0; i < h; i++) {
    memset(p + i * s - pad, p[i * s], pad);
    memset(p + i * s + w, p[i * s + w - 1], pad);
  }
  for (int i = -pad; i < 0; i++) memcpy(p + i * s - pad, p - pad, w + 2 * pad);
  for (int i = h; i < h + pad; i++) memcpy(p + i * s - pad, p + (h - 1) * s - pad, w + 2 * pad);
}

/* scale_val / scale_mv (common/temporal_interp.c:66-91) */
static int or_scale_val(int v, int numer, int denom) {
  if (denom == 0) return 0;
  int prod = v * numer;
  if (denom < 0) {
    denom = -denom;
    prod = -prod;
  }
  return prod >= 0 ? (prod + denom / 2) / denom : -((-prod + denom / 2) / denom);
}

/* interpolate_comp (common/temporal_interp.c:920-944) with mot_comp_avg
 * (:387-441) inlined; mv arrays are (x, y) int16 pairs, 1/8 pel. */
void or_interp_comp(const uint8_t *p0, int s0, const uint8_t *p1, int s1, uint8_t *out, int so, const int16_t *mv0,
                    const int16_t *mv1, int bw, int bh, int bs, int wP, int hP, int pad, int chroma, int wt0, int wt1) {
  for (int yp = 0; yp < bh; yp++)
    for (int xp = 0; xp < bw; xp++) {
      const int b = yp * bw + xp;
      int16_t m0x = mv0[2 * b], m0y = mv0[2 * b + 1], m1x = mv1[2 * b], m1y = mv1[2 * b + 1];
      if (chroma) {
        m1x >>= 1;
        m1y >>= 1;
        if (-wt1 == wt0) {
          m0x = m1x;
          m0y = m1y;
        } else if (-wt1 == -wt0) {
          m0x = (int16_t)-m1x;
          m0y = (int16_t)-m1y;
        } else {
          m0x = (int16_t)or_scale_val(m1x, -wt1, wt0);
          m0y = (int16_t)or_scale_val(m1y, -wt1, wt0);
        }
      }
      const int xs0 = xp * bs + ((m0x + 4) >> 3), xs1 = xp * bs + ((m1x + 4) >> 3);
      const int ys0 = yp * bs + ((m0y + 4) >> 3), ys1 = yp * bs + ((m1y + 4) >> 3);
      const int in0 = xs0 >= -pad && xs0 + bs <= wP && ys0 >= -pad && ys0 + bs <= hP;
      const int in1 = xs1 >= -pad && xs1 + bs <= wP && ys1 >= -pad && ys1 + bs <= hP;
      uint8_t *p = out + (yp * bs) * so + xp * bs;
      for (int i = 0; i < bs; i++)
        for (int j = 0; j < bs; j++) {
          int v;
          if (in0 && in1) v = (p0[(ys0 + i) * s0 + xs0 + j] + p1[(ys1 + i) * s1 + xs1 + j] + 1) / 2;
          else if (in1) v = p1[(ys1 + i) * s1 + xs1 + j];
          else if (in0) v = p0[ys0 * s0 + xs0 + i * s1 + j];
          else {
            const int x0 = MIN(wP - 1, MAX(-pad, j + xs0)), x1 = MIN(wP - 1, MAX(-pad, j + xs1));
            const int y0 = MIN(hP - 1, MAX(-pad, i + ys0)), y1 = MIN(hP - 1, MAX(-pad, i + ys1));
            v = (p0[y0 * s0 + x0] + p1[y1 * s1 + x1] + 1) / 2;
          }
          p[i * so + j] = (uint8_t)v;
        }
    }
}

/* The frame loop filters over caller-supplied per-4x4 side info (the
 * encoder-side checker, tools/enc_host): deblock_frame_y / _uv
 * (common/common_frame.c:46-321, chroma at chroma_qp[qp]) and clpf_frame with
 * per-SB flags (:485-557). */
void or_deblock_cells(or_frame_t *f, const or_cell_t *cells, int W, int H, int qp) {
  deblock_y(f->y, f->stride_y, cells, W, H, qp);
  int qpc = chroma_qp_tab[qp];
  deblock_uv(f->u, f->stride_c, cells, W, H, qpc);
  deblock_uv(f->v, f->stride_c, cells, W, H, qpc);
}
void or_clpf_cells(or_frame_t *f, const or_cell_t *cells, int W, int H, const uint8_t *flags) {
  clpf_frame(f, cells, W, H, flags);
}
