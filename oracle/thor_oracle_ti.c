/*
 * TEST INFRASTRUCTURE ONLY -- the checker, never the thing measured or shipped.
 * Clean-room CPU restatement of Thor's temporal-interpolated reference frame
 * (interpolate_frames, common/temporal_interp.c:972-1053): the luma pyramid,
 * the hierarchical bi-directional block motion search (motion_estimate_bi,
 * :852-918, with its skip test, candidate search and merge pass) and the
 * motion-compensated average of the two references.  Each helper cites the
 * lines it restates.  Pinned by tests/golden/interp_frames.npz (the reference's
 * own interpolate_frames run through oracle/_ref/libthor_ref.so,
 * tools/make_interp_goldens.py) and by the reference decoder's per-frame md5s
 * of the interp_ref streams.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "thor_oracle.h"

#define TI_MIN(a, b) ((a) < (b) ? (a) : (b))
#define TI_MAX(a, b) ((a) > (b) ? (a) : (b))
#define TI_ABS(a) ((a) < 0 ? -(a) : (a))

/* constants of common/temporal_interp.c:12-37 */
enum { TI_BBS = 16, TI_BS = 8, TI_COST_MAX = 0x3fffffff, TI_LAMBDA = 3000, TI_SHIFT = 4, TI_ACC = 3, TI_SKIP_THR = 8 };

typedef struct {
  int16_t x, y;
} ti_mv;

/* scale_val / scale_mv (:66-91) */
static int ti_scale_val(int v, int numer, int denom) {
  if (denom == 0) return 0;
  int prod = v * numer;
  if (denom < 0) {
    denom = -denom;
    prod = -prod;
  }
  return prod >= 0 ? (prod + denom / 2) / denom : -((-prod + denom / 2) / denom);
}
static ti_mv ti_scale(ti_mv m, int numer, int denom) {
  ti_mv o;
  if (numer == denom) return m;
  if (numer == -denom) {
    o.x = (int16_t)-m.x;
    o.y = (int16_t)-m.y;
    return o;
  }
  o.x = (int16_t)ti_scale_val(m.x, numer, denom);
  o.y = (int16_t)ti_scale_val(m.y, numer, denom);
  return o;
}

/* One pyramid level's luma pair (pic[0], pic[1] after the `reversed` swap,
 * :870-872) and its block-vector fields. */
typedef struct {
  const uint8_t *p[2];
  int s[2];
  int w, h, pad;     /* plane size and padding (pad_hor_y == pad_ver_y here) */
  int bw, bh, step;  /* alloc_mv_data (:93-139): 8-px blocks, searched in 16-px steps */
  int wt0, wt1;
  ti_mv *m[2];       /* mv_data->mv[0], mv[1] (the search field) */
  uint8_t *bg;       /* bgmap */
} ti_level;

static uint8_t ti_px(const ti_level *L, int k, int y, int x) { return L->p[k][y * L->s[k] + x]; }

/* sad_cost (:443-523), luma only (USE_CHROMA 0): the vectors are rounded to
 * whole pixels; a pair of blocks inside [-pad, w+pad) x [-pad, h+pad) is a
 * plain SAD, else every tap is clamped into that range. */
static uint32_t ti_sad(const ti_level *L, int x0, int y0, ti_mv a, ti_mv b, int size, uint32_t start) {
  const int xa = x0 + ((a.x + 4) >> TI_ACC), ya = y0 + ((a.y + 4) >> TI_ACC);
  const int xb = x0 + ((b.x + 4) >> TI_ACC), yb = y0 + ((b.y + 4) >> TI_ACC);
  const int wP = L->w + L->pad, hP = L->h + L->pad, pad = L->pad;
  uint32_t c = start;
  const int inside = xa >= -pad && xa + size <= wP && ya >= -pad && ya + size <= hP && xb >= -pad &&
                     xb + size <= wP && yb >= -pad && yb + size <= hP;
  for (int i = 0; i < size; i++)
    for (int j = 0; j < size; j++) {
      int v0, v1;
      if (inside) {
        v0 = ti_px(L, 0, ya + i, xa + j);
        v1 = ti_px(L, 1, yb + i, xb + j);
      } else {
        v0 = ti_px(L, 0, TI_MIN(hP - 1, TI_MAX(-pad, i + ya)), TI_MIN(wP - 1, TI_MAX(-pad, j + xa)));
        v1 = ti_px(L, 1, TI_MIN(hP - 1, TI_MAX(-pad, i + yb)), TI_MIN(wP - 1, TI_MAX(-pad, j + xb)));
      }
      c += (uint32_t)TI_ABS(v1 - v0);
    }
  return c;
}

/* get_mv_cost (:366-385): lambda-weighted distance to the already searched
 * neighbours (above-right, above, above-left, left; first row: left only; first
 * column: above-right and above; last column of later rows: none). */
static int ti_mv_cost(const ti_level *L, ti_mv mv, int xp, int yp, int lambda) {
  const ti_mv *a = L->m[1];
  const int bw = L->bw, st = L->step;
  int d = 0;
#define TI_D(p) (TI_ABS(mv.x - a[p].x) + TI_ABS(mv.y - a[p].y))
  if (xp == 0 && yp == 0) d = 0;
  else if (yp > 0 && xp > 0 && xp < bw - st)
    d = TI_D((yp - st) * bw + xp + st) + TI_D((yp - st) * bw + xp) + TI_D((yp - st) * bw + xp - st) +
        TI_D(yp * bw + xp - st);
  else if (yp == 0) d = TI_D(xp - st);
  else if (xp == 0) d = TI_D((yp - st) * bw + xp + st) + TI_D((yp - st) * bw + xp);
#undef TI_D
  return (d * lambda) >> (TI_SHIFT + TI_ACC);
}

/* add_cand (:273-286): append unless full or already listed */
static int ti_add(ti_mv *list, int len, ti_mv c) {
  if (len >= 20) return len;
  for (int i = 0; i < len; i++)
    if (list[i].x == c.x && list[i].y == c.y) return len;
  list[len] = c;
  return len + 1;
}

/* mv_absdist_filter (:761-782): the entry with the least L1 distance to the
 * others, the last such on ties (<=) */
static ti_mv ti_median(const ti_mv *l, int n) {
  int best = 0, bc = TI_COST_MAX;
  for (int j = 0; j < n; j++) {
    int c = 0;
    for (int i = 0; i < n; i++) c += TI_ABS(l[i].x - l[j].x) + TI_ABS(l[i].y - l[j].y);
    if (c <= bc) {
      best = j;
      bc = c;
    }
  }
  return l[best];
}

/* One search position of the first pass of motion_estimate_bi (:876-895):
 * make_skip_vector (:820-832), skip_test (:525-647), get_cands (:303-351) and
 * adaptive_search_v2 (:650-725), then the 2x2 propagation.  `guide` is the
 * up-scaled vector field of the coarser level (NULL at the top level). */
static void ti_search(ti_level *L, const ti_mv *guide, int xp, int yp) {
  const int bw = L->bw, st = L->step, pos = yp * bw + xp;
  ti_mv *m0 = L->m[0], *m1 = L->m[1];
  const int x0 = xp * TI_BS, y0 = yp * TI_BS;
  /* skip vector: median of the above-right, left and above vectors */
  ti_mv nb[3], skip = {0, 0};
  int n = 0;
  if (yp > 0 && xp < bw - st) nb[n++] = m1[(yp - st) * bw + xp + st];
  if (xp > 0) nb[n++] = m1[yp * bw + xp - st];
  if (yp > 0) nb[n++] = m1[(yp - st) * bw + xp];
  if (n) skip = ti_median(nb, n);
  const ti_mv skip0 = ti_scale(skip, -L->wt1, L->wt0);
  /* skip test: every 8x8 of the 16x16 within SKIP_THRESHOLD * 64 at the skip
   * vectors, all inside the padded frame */
  int is_skip = 1;
  for (int p = 0; p < TI_BBS && is_skip; p += 8)
    for (int q = 0; q < TI_BBS && is_skip; q += 8) {
      const int xa = x0 + q + ((skip0.x + 4) >> TI_ACC), ya = y0 + p + ((skip0.y + 4) >> TI_ACC);
      const int xb = x0 + q + ((skip.x + 4) >> TI_ACC), yb = y0 + p + ((skip.y + 4) >> TI_ACC);
      const int wP = L->w + L->pad, hP = L->h + L->pad, pad = L->pad;
      if (!(xa >= -pad && xa + 8 <= wP && ya >= -pad && ya + 8 <= hP && xb >= -pad && xb + 8 <= wP && yb >= -pad &&
            yb + 8 <= hP)) {
        is_skip = 0;
        break;
      }
      int sum = 0;
      for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) sum += TI_ABS(ti_px(L, 0, ya + i, xa + j) - ti_px(L, 1, yb + i, xb + j));
      if (sum > TI_SKIP_THR * 64) is_skip = 0;
    }
  ti_mv r0, r1;
  if (is_skip) {
    L->bg[pos] = 1;
    r1 = skip;
    r0 = skip0;
  } else {
    /* candidates: zero, the guide, above-right, left, above */
    ti_mv cand[20];
    int nc = 0;
    const ti_mv zero = {0, 0};
    nc = ti_add(cand, nc, zero);
    if (guide) nc = ti_add(cand, nc, ti_scale(guide[pos], L->wt0, L->wt0));
    if (yp > 0 && xp < bw - st) nc = ti_add(cand, nc, m1[(yp - st) * bw + xp + st]);
    if (xp > 0) nc = ti_add(cand, nc, m1[yp * bw + xp - st]);
    if (yp > 0) nc = ti_add(cand, nc, m1[(yp - st) * bw + xp]);
    /* adaptive_search_v2: each candidate costed, promising ones refined by a
     * shrinking cross (guided: one 1-px step size, at most 2 rounds) */
    const int lambda = guide ? TI_LAMBDA / 4 : TI_LAMBDA;
    ti_mv best = cand[0];
    ti_mv best0 = ti_scale(best, -L->wt1, L->wt0);
    uint32_t best_cost = TI_COST_MAX;
    for (int c = 0; c < nc; c++) {
      ti_mv cm = cand[c], cm0 = ti_scale(cm, -L->wt1, L->wt0);
      uint32_t cc = (uint32_t)ti_mv_cost(L, cm, xp, yp, lambda);
      cc = ti_sad(L, x0, y0, cm0, cm, TI_BBS, cc);
      if (((uint32_t)(4 + c) * cc) / 8 < best_cost) {
        int shift = guide ? TI_ACC : 3 + TI_ACC, count = guide ? 8 : 64;
        while (shift >= TI_ACC && count > 0) {
          const int o = 1 << shift;
          const ti_mv ctr = cm;
          ti_mv cross[4];
          cross[0].x = (int16_t)(ctr.x - o), cross[0].y = ctr.y;
          cross[1].x = (int16_t)(ctr.x + o), cross[1].y = ctr.y;
          cross[2].x = ctr.x, cross[2].y = (int16_t)(ctr.y - o);
          cross[3].x = ctr.x, cross[3].y = (int16_t)(ctr.y + o);
          int better = 0;
          for (int i = 0; i < 4; i++) {
            const ti_mv q0 = ti_scale(cross[i], -L->wt1, L->wt0);
            uint32_t bc = (uint32_t)ti_mv_cost(L, cross[i], xp, yp, lambda);
            bc = ti_sad(L, x0, y0, q0, cross[i], TI_BBS, bc);
            if (bc < cc) {
              cc = bc;
              cm = cross[i];
              cm0 = q0;
              better = 1;
            }
          }
          if (!better) shift--;
          count -= 4;
        }
      }
      if (cc < best_cost) {
        best = cm;
        best0 = cm0;
        best_cost = cc;
      }
    }
    r1 = best;
    r0 = best0;
  }
  for (int q = 0; q < st; q++)
    for (int p = 0; p < st; p++) {
      m0[pos + q * bw + p] = r0;
      m1[pos + q * bw + p] = r1;
      L->bg[pos + q * bw + p] = L->bg[pos];
    }
}

/* motion_estimate_bi (:852-918): the raster-order search pass over 16x16
 * steps, then the merge pass over every 8x8 block (get_merge_cands :288-301,
 * merge_candidate_search :727-759) writing the final fields f0 / f1. */
static void ti_motion_estimate(ti_level *L, const ti_mv *guide, ti_mv *f0, ti_mv *f1) {
  const int bw = L->bw, bh = L->bh, st = L->step;
  memset(L->bg, 0, (size_t)bw * bh);
  if (!guide) {
    memset(L->m[0], 0, sizeof(ti_mv) * bw * bh);
    memset(L->m[1], 0, sizeof(ti_mv) * bw * bh);
  }
  for (int i = 0; i < bh; i += st)
    for (int j = 0; j < bw; j += st) ti_search(L, guide, j, i);
  const ti_mv *m1 = L->m[1];
  for (int i = 0; i < bh; i++)
    for (int j = 0; j < bw; j++) {
      const int off = (i & 1) ? 2 : 1; /* the reference keys both offsets on the row parity */
      ti_mv cand[20];
      int nc = 0;
      nc = ti_add(cand, nc, m1[i * bw + j]);
      if (i - off >= 0) nc = ti_add(cand, nc, m1[(i - off) * bw + j]);
      if (i + off < bh) nc = ti_add(cand, nc, m1[(i + off) * bw + j]);
      if (j - off >= 0) nc = ti_add(cand, nc, m1[i * bw + j - off]);
      if (j + off < bw) nc = ti_add(cand, nc, m1[i * bw + j + off]);
      if (nc > 1) {
        uint32_t bc = TI_COST_MAX;
        ti_mv b1 = {0, 0}, b0 = {0, 0};
        for (int c = 0; c < nc; c++) {
          const ti_mv q0 = ti_scale(cand[c], -L->wt1, L->wt0);
          const uint32_t cost = ti_sad(L, j * TI_BS, i * TI_BS, q0, cand[c], TI_BS, 0);
          if (cost < bc) {
            bc = cost;
            b1 = cand[c];
            b0 = q0;
          }
        }
        f0[i * bw + j] = b0;
        f1[i * bw + j] = b1;
      } else {
        f0[i * bw + j] = L->m[0][i * bw + j];
        f1[i * bw + j] = L->m[1][i * bw + j];
      }
    }
}

int or_ti_levels(int width, int height) {
  /* max_levels = min(MAX_LEVELS, (int)(log10(min(w, h)) / log10(2.0) - 4.0)) (:977), in the
   * reference's double arithmetic */
  const int l = (int)(log10((double)TI_MIN(width, height)) / log10(2.0) - 4.0);
  return TI_MIN(4, l);
}

void or_ti_weights(int ratio, int pos, int *wt0, int *wt1, int *reversed) {
  /* alloc_mv_data, interpolating (:120-126) */
  *reversed = pos > ratio / 2;
  *wt0 = *reversed ? pos : ratio - pos;
  *wt1 = ratio - *wt0;
}

int or_interpolate_frames(const or_frame_t *ref0, const or_frame_t *ref1, int pad_y, or_frame_t *out, int width,
                          int height, int ratio, int pos, int16_t *const *lv_mv0, int16_t *const *lv_mv1) {
  const int nl = or_ti_levels(width, height);
  if (nl < 1) return -1;
  int wt0, wt1, rev;
  or_ti_weights(ratio, pos, &wt0, &wt1, &rev);
  /* luma pyramid of both references (:1000-1019): levels 1.. with a 32-px margin */
  uint8_t *lvbuf[4][2] = {{0}};
  const uint8_t *lp[4][2];
  int ls[4], lpad[4];
  lp[0][0] = ref0->y;
  lp[0][1] = ref1->y;
  ls[0] = ref0->stride_y;
  lpad[0] = pad_y;
  for (int l = 1; l < nl; l++) {
    const int w = width >> l, h = height >> l;
    ls[l] = (w + 64 + 15) & ~15;
    lpad[l] = 32;
    for (int k = 0; k < 2; k++) {
      lvbuf[l][k] = (uint8_t *)calloc((size_t)(h + 64) * ls[l], 1);
      uint8_t *o = lvbuf[l][k] + 32 * ls[l] + 32;
      or_scale_down2x2(lp[l - 1][k], ls[l - 1], o, ls[l], w, h);
      or_pad_plane(o, ls[l], w, h, 32);
      lp[l][k] = o;
    }
  }
  ti_mv *guide = NULL, *f0 = NULL, *f1 = NULL;
  int gbw = 0;
  for (int l = nl - 1; l >= 0; l--) {
    const int w = width >> l, h = height >> l;
    ti_level L;
    L.step = TI_BBS / TI_BS;
    L.bw = L.step * ((w + TI_BBS - 1) / TI_BBS);
    L.bh = L.step * ((h + TI_BBS - 1) / TI_BBS);
    L.w = w;
    L.h = h;
    L.pad = lpad[l];
    L.wt0 = wt0;
    L.wt1 = wt1;
    for (int k = 0; k < 2; k++) { /* pic[0] / pic[1], swapped when reversed */
      L.p[k] = lp[l][rev ? 1 - k : k];
      L.s[k] = ls[l];
    }
    const size_t area = (size_t)L.bw * L.bh;
    L.m[0] = (ti_mv *)calloc(area, sizeof(ti_mv));
    L.m[1] = (ti_mv *)calloc(area, sizeof(ti_mv));
    L.bg = (uint8_t *)calloc(area, 1);
    ti_mv *g = NULL;
    if (guide) { /* upscale_mv_data_2x2 (:247-271) of the coarser level's final field; only mv[1] is read */
      g = (ti_mv *)calloc(area, sizeof(ti_mv));
      for (int i = 0; i < L.bh; i++)
        for (int j = 0; j < L.bw; j++) {
          const ti_mv v = f1[(i / 2) * gbw + j / 2];
          g[i * L.bw + j].x = (int16_t)(v.x << 1);
          g[i * L.bw + j].y = (int16_t)(v.y << 1);
        }
    }
    ti_mv *n0 = (ti_mv *)calloc(area, sizeof(ti_mv)), *n1 = (ti_mv *)calloc(area, sizeof(ti_mv));
    ti_motion_estimate(&L, g, n0, n1);
    if (lv_mv0 && lv_mv0[l]) memcpy(lv_mv0[l], n0, area * sizeof(ti_mv));
    if (lv_mv1 && lv_mv1[l]) memcpy(lv_mv1[l], n1, area * sizeof(ti_mv));
    free(g);
    free(guide);
    free(f0);
    free(L.m[0]);
    free(L.m[1]);
    free(L.bg);
    f0 = n0;
    f1 = n1;
    guide = f1;
    gbw = L.bw;
    if (l == 0) {
      /* interpolate_frame (:946-970): Y in 8x8 blocks (pad 4), U / V in 4x4 (pad 2) */
      const or_frame_t *pa = rev ? ref1 : ref0, *pb = rev ? ref0 : ref1;
      or_interp_comp(pa->y, pa->stride_y, pb->y, pb->stride_y, out->y, out->stride_y, (const int16_t *)f0,
                     (const int16_t *)f1, L.bw, L.bh, 8, width + 4, height + 4, 4, 0, wt0, wt1);
      or_interp_comp(pa->u, pa->stride_c, pb->u, pb->stride_c, out->u, out->stride_c, (const int16_t *)f0,
                     (const int16_t *)f1, L.bw, L.bh, 4, (width + 4) / 2, (height + 4) / 2, 2, 1, wt0, wt1);
      or_interp_comp(pa->v, pa->stride_c, pb->v, pb->stride_c, out->v, out->stride_c, (const int16_t *)f0,
                     (const int16_t *)f1, L.bw, L.bh, 4, (width + 4) / 2, (height + 4) / 2, 2, 1, wt0, wt1);
    }
  }
  free(f0);
  free(f1);
  for (int l = 1; l < nl; l++)
    for (int k = 0; k < 2; k++) free(lvbuf[l][k]);
  return 0;
}
