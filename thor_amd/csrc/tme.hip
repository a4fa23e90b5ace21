// Temporal-interpolated reference frame on the GPU:
// interpolate_frames (common/temporal_interp.c:972-1053) = luma pyramid of both
// references (pyramid.hip), then per level, coarsest first, motion_estimate_bi
// (:852-918), then interpolate_frame at level 0 (interp.hip).
//
// motion_estimate_bi has two passes over the level's 8x8-block vector field:
//
//  * the search pass visits 16x16 steps in raster order; a step reads the
//    vectors of its above-right, above, above-left and left steps (skip vector
//    :820-832, candidates :303-351, vector cost :366-385), so rows of steps
//    form a wavefront (WPP): step (r, c) may run once row r-1 has finished step
//    c+1.  k_ti_search runs one wave64 per step row, rows handed out by ticket
//    (a row only ever waits on a row whose wave already runs: no deadlock),
//    progress words polled relaxed and acquired once per observed advance (the
//    encoder's protocol, enc.hip).  Inside a step the 64 lanes split the 16x16
//    block (4 px per lane: dword loads realigned by v_alignbyte, v_sad_u8);
//    the candidates' SADs, and the four points of each cross-search round, run
//    side by side and reduce two at a time (a 16x16 SAD fits in 16 bits);
//  * the merge pass (:900-911) reads only the finished search field: every 8x8
//    block independent, k_ti_merge gives each 16 lanes.
//
// All arithmetic is the reference's integer arithmetic (1/8-pel vectors rounded
// to whole pixels, scale_val's rounded division, uint32 costs), so the field
// and the interpolated frame are bit-exact (tests/test_gpu_interp_frames.py).

#define TI_MAXL 4  // MAX_LEVELS (:20)

struct TiLevel {
  const uint8_t *p0, *p1;  // pic[0], pic[1] luma (0,0), after the `reversed` swap (:870-872)
  int s0, s1;
  int w, h, pad;           // level size; padding (pad_hor_y == pad_ver_y)
  int bw, bh;              // 8x8-block grid (alloc_mv_data :97-99)
  int wt0, wt1;
  uint32_t *m0, *m1;       // search field (mv_data->mv[0], mv[1]): int16 x | y << 16
  uint32_t *f0, *f1;       // final field after the merge pass
  const uint32_t *guide;   // final f1 of the coarser level (up-scaled on read), nullptr at the top
  int gbw;
  unsigned long long *pub; // per step: (generation << 32) | mv1, the wavefront's ready flags
  unsigned *ticket;
  unsigned gen;            // this launch's generation tag
  unsigned *err;
  unsigned long long *dbg; // optional (diagnostics): per step (ready, done) s_memrealtime stamps
};

__device__ __forceinline__ int ti_x(uint32_t v) { return (int)(int16_t)(v & 0xffff); }
__device__ __forceinline__ int ti_y(uint32_t v) { return (int)(int16_t)(v >> 16); }
__device__ __forceinline__ uint32_t ti_mv(int x, int y) { return (uint32_t)(x & 0xffff) | ((uint32_t)(y & 0xffff) << 16); }

// scale_val / scale_mv (:66-91), results stored as int16 (mv_t)
__device__ __forceinline__ int ti_scale_val(int v, int numer, int denom) {
  if (denom == 0) return 0;
  int prod = v * numer;
  if (denom < 0) {
    denom = -denom;
    prod = -prod;
  }
  return prod >= 0 ? (prod + denom / 2) / denom : -((-prod + denom / 2) / denom);
}
__device__ __forceinline__ uint32_t ti_scale(uint32_t m, int numer, int denom) {
  if (numer == denom) return m;
  if (numer == -denom) return ti_mv(-ti_x(m), -ti_y(m));
  return ti_mv(ti_scale_val(ti_x(m), numer, denom), ti_scale_val(ti_y(m), numer, denom));
}
__device__ __forceinline__ int ti_round(int v) { return (v + 4) >> 3; }  // ACC_BITS 3, :392-395

__device__ __forceinline__ uint32_t ti_ld_relaxed(const unsigned *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// uniform field value written by another wave (after the acquire): a vector
// load, kept out of the scalar cache
__device__ __forceinline__ uint32_t ti_ld_field(const uint32_t *p) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// 4 bytes at an arbitrary address: two aligned dwords + v_alignbyte
__device__ __forceinline__ uint32_t ti_load4(const uint8_t *p) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t *w = (const uint32_t *)(a & ~(uintptr_t)3);
  return __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(a & 3));
}

// This lane's share (row `r`, columns 4q..4q+3) of sad_cost (:443-523) for a
// size x size block at (x0, y0) with vectors (a: pic[0], b: pic[1]).  The
// inside test is uniform; outside, every tap is clamped into the padded plane.
__device__ __forceinline__ uint32_t ti_sad_part(const TiLevel &L, int x0, int y0, uint32_t a, uint32_t b, int size,
                                                int r, int q) {
  const int xa = x0 + ti_round(ti_x(a)), ya = y0 + ti_round(ti_y(a));
  const int xb = x0 + ti_round(ti_x(b)), yb = y0 + ti_round(ti_y(b));
  const int pad = L.pad, wP = L.w + pad, hP = L.h + pad;
  const bool inside = xa >= -pad && xa + size <= wP && ya >= -pad && ya + size <= hP && xb >= -pad &&
                      xb + size <= wP && yb >= -pad && yb + size <= hP;
  if (inside) {
    const uint32_t va = ti_load4(L.p0 + (long long)(ya + r) * L.s0 + xa + 4 * q);
    const uint32_t vb = ti_load4(L.p1 + (long long)(yb + r) * L.s1 + xb + 4 * q);
    return __builtin_amdgcn_sad_u8(va, vb, 0u);
  }
  uint32_t s = 0;
  const int y0c = min(hP - 1, max(-pad, r + ya)), y1c = min(hP - 1, max(-pad, r + yb));
  for (int j = 0; j < 4; j++) {
    const int c = 4 * q + j;
    const int xac = min(wP - 1, max(-pad, c + xa)), xbc = min(wP - 1, max(-pad, c + xb));
    const int va = L.p0[(long long)y0c * L.s0 + xac], vb = L.p1[(long long)y1c * L.s1 + xbc];
    s += (uint32_t)abs(vb - va);
  }
  return s;
}

// Sum over each 16-lane DPP row, in every lane of the row: quad butterflies,
// then the half-row and row mirrors (4 VALU ops, no LDS-pipe permutes).
__device__ __forceinline__ uint32_t ti_row_sum(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xb1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4e, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xf, 0xf, false);  // row_half_mirror
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xf, 0xf, false);  // row_mirror
  return v;
}
// Wave total, uniform: the four row sums read out and added on the scalar unit.
__device__ __forceinline__ uint32_t ti_wave_sum(uint32_t v) {
  const uint32_t r = ti_row_sum(v);
  return __builtin_amdgcn_readlane(r, 0) + __builtin_amdgcn_readlane(r, 16) + __builtin_amdgcn_readlane(r, 32) +
         __builtin_amdgcn_readlane(r, 48);
}

// get_mv_cost (:366-385) from the step's neighbour vectors (already loaded)
__device__ __forceinline__ int ti_mv_cost(uint32_t mv, int xp, int yp, int bw, uint32_t tr, uint32_t t, uint32_t tl,
                                          uint32_t l, int lambda) {
  const int x = ti_x(mv), y = ti_y(mv);
#define TI_D(n) (abs(x - ti_x(n)) + abs(y - ti_y(n)))
  int d = 0;
  if (xp == 0 && yp == 0) d = 0;
  else if (yp > 0 && xp > 0 && xp < bw - 2) d = TI_D(tr) + TI_D(t) + TI_D(tl) + TI_D(l);
  else if (yp == 0) d = TI_D(l);
  else if (xp == 0) d = TI_D(tr) + TI_D(t);
#undef TI_D
  return (d * lambda) >> 7;  // LAMBDA_SHIFT + ACC_BITS
}

__device__ __forceinline__ int ti_add(uint32_t *list, int n, uint32_t c) {
  for (int i = 0; i < n; i++)
    if (list[i] == c) return n;
  list[n] = c;
  return n + 1;
}

// mv_absdist_filter (:761-782): last minimum (<=)
__device__ __forceinline__ uint32_t ti_median(const uint32_t *l, int n) {
  int best = 0, bc = 0x3fffffff;
  for (int j = 0; j < n; j++) {
    int c = 0;
    for (int i = 0; i < n; i++) c += abs(ti_x(l[i]) - ti_x(l[j])) + abs(ti_y(l[i]) - ti_y(l[j]));
    if (c <= bc) {
      best = j;
      bc = c;
    }
  }
  return l[best];
}

// Sliding LDS window of both pictures around the current step: a ring of
// 16-px column tiles (T_k covers x in [16k, 16k + 16)), TI_WH rows from y0 -
// TI_WR.  Step c reads T_{c-2} .. T_{c+2} while T_{c+3} is being loaded.
#define TI_WR 32
#define TI_WH (16 + 2 * TI_WR)
#define TI_TILES 6
struct TiWin {
  uint8_t t[2][TI_TILES][TI_WH][16];
};

__device__ __forceinline__ int ti_slot(int k) { return (k + 6 * TI_TILES) % TI_TILES; }  // k >= -2

// Stage tile T_k (rows y0 - TI_WR ..) of both pictures: 2 x TI_WH 16-byte rows,
// row coordinates clamped into the plane's allocation (clamped rows lie outside
// [-pad, h + pad), so no in-frame SAD ever reads them).
// Every lane issues its three loads unconditionally (surplus lanes re-load the
// last row): a load skipped under an exec mask would leave its register
// "pending" across the loop back-edge and cost a vmcnt(0) every step.
struct TiTile {
  uint4 v0, v1, v2;  // this lane's rows idx = lane, lane + 64, lane + 128 (named: kept in registers)
};
__device__ __forceinline__ uint4 ti_tile_row(const TiLevel &L, int k, int y0, int idx) {
  idx = min(idx, 2 * TI_WH - 1);
  const int pic = idx >= TI_WH, r = idx - pic * TI_WH;
  const int y = min(L.h + L.pad - 1, max(-L.pad, y0 - TI_WR + r));
  const uint8_t *p = pic ? L.p1 : L.p0;
  const int s = pic ? L.s1 : L.s0;
  return *(const uint4 *)(p + (long long)y * s + 16 * k);
}
__device__ __forceinline__ TiTile ti_tile_load(const TiLevel &L, int k, int y0) {
  const int lane = threadIdx.x;
  return TiTile{ti_tile_row(L, k, y0, lane), ti_tile_row(L, k, y0, lane + 64), ti_tile_row(L, k, y0, lane + 128)};
}
__device__ __forceinline__ void ti_tile_put(TiWin &W, int sl, int idx, uint4 v) {
  if (idx < 2 * TI_WH) {
    const int pic = idx >= TI_WH, r = idx - pic * TI_WH;
    *(uint4 *)&W.t[pic][sl][r][0] = v;
  }
}
__device__ __forceinline__ void ti_tile_store(TiWin &W, int k, const TiTile &t) {
  const int lane = threadIdx.x, sl = ti_slot(k);
  ti_tile_put(W, sl, lane, t.v0);
  ti_tile_put(W, sl, lane + 64, t.v1);
  ti_tile_put(W, sl, lane + 128, t.v2);
}

// 4 pixels of picture `pic` at window row wr, level column x = u + 4q + sh
// (u: uniform, dword aligned; sh: uniform byte shift)
__device__ __forceinline__ uint32_t ti_win4(const TiWin &W, int pic, int u, int sh, int q, int wr) {
  const int ta = (u & 15) + 4 * q, tb = ta + 4;
  const int k0 = u >> 4;
  const uint32_t A = *(const uint32_t *)&W.t[pic][ti_slot(k0 + (ta >> 4))][wr][ta & 15];
  const uint32_t B = *(const uint32_t *)&W.t[pic][ti_slot(k0 + (tb >> 4))][wr][tb & 15];
  return __builtin_amdgcn_alignbyte(B, A, (uint32_t)sh);
}

// Spin (uniformly) until the published word of a step of the row above carries
// this launch's generation.  A wedged wavefront (60 s) is reported once and the
// wave stops waiting for the rest of its row (`dead`), so the launch drains in
// bounded time whatever the number of steps.
__device__ __forceinline__ unsigned long long ti_spin(const unsigned long long *p, unsigned gen, unsigned *err,
                                                      bool &dead) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long w;
  while (__builtin_amdgcn_readfirstlane(
             (uint32_t)((w = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 32)) != gen) {
    if (dead) break;
    __builtin_amdgcn_s_sleep(1);
    if (__builtin_amdgcn_s_memrealtime() - t0 > 6000000000ULL) {  // 60 s: report, never hang the GPU
      if (threadIdx.x == 0) atomicOr(err, 1u);
      dead = true;
      break;
    }
  }
  return w;
}

// This lane's share of a 16x16 sad_cost at step origin (x0, y0): from the LDS
// window when both displaced blocks lie in it (and in the padded frame), else
// from the planes (ti_sad_part).
// Vectors and the path choice are made explicitly uniform (SGPRs, scalar
// branch): a VALU-computed condition would be treated as divergent, the
// if / else linearised, and the window path would then wait (vmcnt(0)) on the
// fallback path's loads -- and with them on the tile prefetch -- every step.
__device__ __forceinline__ uint32_t ti_sad16(const TiLevel &L, const TiWin &W, int x0, int y0, uint32_t a, uint32_t b,
                                             int r, int q) {
  a = __builtin_amdgcn_readfirstlane(a);
  b = __builtin_amdgcn_readfirstlane(b);
  const int dxa = ti_round(ti_x(a)), dya = ti_round(ti_y(a)), dxb = ti_round(ti_x(b)), dyb = ti_round(ti_y(b));
  const int xa = x0 + dxa, ya = y0 + dya, xb = x0 + dxb, yb = y0 + dyb;
  const int pad = L.pad, wP = L.w + pad, hP = L.h + pad;
  const bool inside = xa >= -pad && xa + 16 <= wP && ya >= -pad && ya + 16 <= hP && xb >= -pad && xb + 16 <= wP &&
                      yb >= -pad && yb + 16 <= hP;
  const bool inwin = abs(dxa) <= TI_WR && abs(dya) <= TI_WR && abs(dxb) <= TI_WR && abs(dyb) <= TI_WR;
  if (__builtin_amdgcn_readfirstlane((int)(inside && inwin))) {
    const uint32_t va = ti_win4(W, 0, xa & ~3, xa & 3, q, dya + TI_WR + r);
    const uint32_t vb = ti_win4(W, 1, xb & ~3, xb & 3, q, dyb + TI_WR + r);
    return __builtin_amdgcn_sad_u8(va, vb, 0u);
  }
  return ti_sad_part(L, x0, y0, a, b, 16, r, q);
}

__device__ __forceinline__ unsigned long long ti_ld64(const unsigned long long *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The search pass of motion_estimate_bi (:874-896): one wave per step row.
// A step publishes its vector as a 64-bit (generation, mv1) word; the row
// below spins on exactly the word it needs (its above-right step), so the
// wavefront needs no progress counters and no fences: the vector travels with
// its own ready flag.
__global__ __launch_bounds__(64) void k_ti_search(const TiLevel L) {
  __shared__ TiWin W;
  const int lane = threadIdx.x, r16 = lane >> 2, q = lane & 3;
  const int nrows = L.bh >> 1, ncols = L.bw >> 1, bw = L.bw;
  unsigned t = 0;
  if (lane == 0) t = atomicAdd(L.ticket, 1u);
  const int row = (int)__builtin_amdgcn_readfirstlane(t);
  if (row >= nrows) return;
  const int yp = 2 * row, y0 = yp * 8;
  const bool guided = L.guide != nullptr;
  const int lambda = guided ? 3000 / 4 : 3000;
  const int wt0 = L.wt0, wt1 = L.wt1;
  const unsigned long long tag = (unsigned long long)L.gen << 32;
  const unsigned long long *above = L.pub + (long long)(row - 1) * ncols;
  unsigned long long *mine = L.pub + (long long)row * ncols;
  // the window for step 0: tiles -2 .. 2
  for (int k = -2; k <= 2; k++) ti_tile_store(W, k, ti_tile_load(L, k, y0));
  uint32_t left = 0;          // this row's previous step (written by this wave)
  uint32_t up_l = 0, up = 0;  // row above: steps c-1 and c (rolled forward)
  uint32_t up_r = 0;
  unsigned long long next = 0;  // prefetched published word of the row above
  bool dead = false;            // a wait of this wave gave up: wait no more
  if (row > 0) next = ti_ld64(above + (ncols > 1 ? 1 : 0));
  for (int c = 0; c < ncols; c++) {
    const int xp = 2 * c, x0 = xp * 8;
    const TiTile pf = ti_tile_load(L, c + 3, y0);  // next step's new tile, in flight during this step
    if (row > 0) {
      // above-right (or, at the last column, nothing new: its vectors are already held)
      if (c == 0) {
        up = __builtin_amdgcn_readfirstlane((uint32_t)ti_spin(above, L.gen, L.err, dead));
        up_l = 0;
      } else {
        up_l = up;
        up = up_r;
      }
      if (c + 1 < ncols) {
        unsigned long long w = next;
        if (__builtin_amdgcn_readfirstlane((uint32_t)(w >> 32)) != L.gen) w = ti_spin(above + c + 1, L.gen, L.err, dead);
        up_r = __builtin_amdgcn_readfirstlane((uint32_t)w);
        if (c + 2 < ncols) next = ti_ld64(above + c + 2);  // the next step's, early
      }
    }
    unsigned long long t_ready = 0;
    if (L.dbg) t_ready = __builtin_amdgcn_s_memrealtime();
    // skip vector (:820-832) and its pic[0] companion
    uint32_t nb[3];
    int n = 0;
    if (yp > 0 && xp < bw - 2) nb[n++] = up_r;
    if (xp > 0) nb[n++] = left;
    if (yp > 0) nb[n++] = up;
    const uint32_t skip1 = n ? ti_median(nb, n) : 0u;
    const uint32_t skip0 = ti_scale(skip1, -wt1, wt0);
    // skip_test (:525-647): each 8x8 quarter of the 16x16 within 8 * 64 and inside the padded frame
    bool skip;
    {
      const int xa = x0 + ti_round(ti_x(skip0)), ya = y0 + ti_round(ti_y(skip0));
      const int xb = x0 + ti_round(ti_x(skip1)), yb = y0 + ti_round(ti_y(skip1));
      const int pad = L.pad, wP = L.w + pad, hP = L.h + pad;
      skip = xa >= -pad && xa + 16 <= wP && ya >= -pad && ya + 16 <= hP && xb >= -pad && xb + 16 <= wP &&
             yb >= -pad && yb + 16 <= hP;
      if (skip) {
        const uint32_t s = ti_sad16(L, W, x0, y0, skip0, skip1, r16, q);
        // quarter sums: left / right column half packed (16 bits each), rows of 16 lanes =
        // 4 image rows, rows 0-1 the top quarters, 2-3 the bottom ones
        const uint32_t r = ti_row_sum(q < 2 ? s : s << 16);
        const uint32_t top = __builtin_amdgcn_readlane(r, 0) + __builtin_amdgcn_readlane(r, 16);
        const uint32_t bot = __builtin_amdgcn_readlane(r, 32) + __builtin_amdgcn_readlane(r, 48);
        const uint32_t thr = 8u * 64u;
        skip = (top & 0xffff) <= thr && (top >> 16) <= thr && (bot & 0xffff) <= thr && (bot >> 16) <= thr;
      }
    }
    uint32_t r0, r1;
    if (skip) {
      r1 = skip1;
      r0 = skip0;
    } else {
      // get_cands (:303-351): zero, the guide, above-right, left, above
      uint32_t cand[5];
      int nc = 0;
      cand[nc++] = 0u;
      if (guided) {
        const uint32_t g = L.guide[(long long)(yp >> 1) * L.gbw + (xp >> 1)];
        nc = ti_add(cand, nc, ti_mv(ti_x(g) << 1, ti_y(g) << 1));  // upscale_mv_data_2x2 (:266-267); scale by wt0/wt0 = identity
      }
      if (yp > 0 && xp < bw - 2) nc = ti_add(cand, nc, up_r);
      if (xp > 0) nc = ti_add(cand, nc, left);
      if (yp > 0) nc = ti_add(cand, nc, up);
      // every candidate's cost at once (adaptive_search_v2 :674-683), two SADs per reduction
      uint32_t cost[5];
      for (int k = 0; k < nc; k += 2) {
        uint32_t s = ti_sad16(L, W, x0, y0, ti_scale(cand[k], -wt1, wt0), cand[k], r16, q);
        if (k + 1 < nc) s |= ti_sad16(L, W, x0, y0, ti_scale(cand[k + 1], -wt1, wt0), cand[k + 1], r16, q) << 16;
        s = ti_wave_sum(s);
        cost[k] = (s & 0xffff) + (uint32_t)ti_mv_cost(cand[k], xp, yp, bw, up_r, up, up_l, left, lambda);
        if (k + 1 < nc) cost[k + 1] = (s >> 16) + (uint32_t)ti_mv_cost(cand[k + 1], xp, yp, bw, up_r, up, up_l, left, lambda);
      }
      uint32_t best = cand[0], best_cost = 0x3fffffffu;
      for (int k = 0; k < nc; k++) {
        uint32_t cm = cand[k], cc = cost[k];
        if (((uint32_t)(4 + k) * cc) / 8 < best_cost) {
          // cross refinement (:685-712): guided one 1-px step size (<= 2 rounds), else 8..1 px (<= 16 rounds)
          int shift = guided ? 3 : 6, count = guided ? 8 : 64;
          while (shift >= 3 && count > 0) {
            const int o = 1 << shift, cx = ti_x(cm), cy = ti_y(cm);
            const uint32_t p[4] = {ti_mv(cx - o, cy), ti_mv(cx + o, cy), ti_mv(cx, cy - o), ti_mv(cx, cy + o)};
            uint32_t s01 = ti_sad16(L, W, x0, y0, ti_scale(p[0], -wt1, wt0), p[0], r16, q) |
                           (ti_sad16(L, W, x0, y0, ti_scale(p[1], -wt1, wt0), p[1], r16, q) << 16);
            uint32_t s23 = ti_sad16(L, W, x0, y0, ti_scale(p[2], -wt1, wt0), p[2], r16, q) |
                           (ti_sad16(L, W, x0, y0, ti_scale(p[3], -wt1, wt0), p[3], r16, q) << 16);
            s01 = ti_wave_sum(s01);
            s23 = ti_wave_sum(s23);
            const uint32_t sads[4] = {s01 & 0xffff, s01 >> 16, s23 & 0xffff, s23 >> 16};
            bool better = false;
            for (int i = 0; i < 4; i++) {
              const uint32_t bc = sads[i] + (uint32_t)ti_mv_cost(p[i], xp, yp, bw, up_r, up, up_l, left, lambda);
              if (bc < cc) {
                cc = bc;
                cm = p[i];
                better = true;
              }
            }
            if (!better) shift--;
            count -= 4;
          }
        }
        if (cc < best_cost) {
          best = cm;
          best_cost = cc;
        }
      }
      r1 = best;
      r0 = ti_scale(best, -wt1, wt0);
    }
    // publish (the row below waits on exactly this word), then the 2x2 blocks of the step (:884-894)
    if (lane == 0) __hip_atomic_store(mine + c, tag | r1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (L.dbg && lane == 0) {
      L.dbg[2 * ((long long)row * ncols + c)] = t_ready;
      L.dbg[2 * ((long long)row * ncols + c) + 1] = __builtin_amdgcn_s_memrealtime();
    }
    if (lane < 4) {
      const long long o = (long long)(yp + (lane >> 1)) * bw + xp + (lane & 1);
      L.m0[o] = r0;
      L.m1[o] = r1;
    }
    left = r1;
    // slide the window: T_{c+3} replaces T_{c-3} (no longer read)
    wave_lds_sync();
    ti_tile_store(W, c + 3, pf);
    wave_lds_sync();
  }
}

// The merge pass (:900-911, get_merge_cands :288-301, merge_candidate_search
// :727-759): 16 lanes per 8x8 block (row r, columns 4q..4q+3), 4 blocks per wave.
__global__ __launch_bounds__(256) void k_ti_merge(const TiLevel L) {
  const int g = (blockIdx.x * 256 + threadIdx.x) >> 4, l16 = threadIdx.x & 15;
  const int bw = L.bw, bh = L.bh;
  const bool live = g < bw * bh;
  const int i = live ? g / bw : 0, j = live ? g - i * bw : 0;
  const int off = (i & 1) ? 2 : 1;  // the reference keys both offsets on the row parity
  const uint32_t *m1 = L.m1;
  uint32_t cand[5];
  int nc = 0;
  cand[nc++] = m1[(long long)i * bw + j];
  if (i - off >= 0) nc = ti_add(cand, nc, m1[(long long)(i - off) * bw + j]);
  if (i + off < bh) nc = ti_add(cand, nc, m1[(long long)(i + off) * bw + j]);
  if (j - off >= 0) nc = ti_add(cand, nc, m1[(long long)i * bw + j - off]);
  if (j + off < bw) nc = ti_add(cand, nc, m1[(long long)i * bw + j + off]);
  uint32_t b0 = L.m0[(long long)i * bw + j], b1 = cand[0];
  if (nc > 1) {
    uint32_t bc = 0x3fffffffu;
    b0 = b1 = 0;
    for (int k = 0; k < nc; k++) {
      const uint32_t q0 = ti_scale(cand[k], -L.wt1, L.wt0);
      const uint32_t s = ti_row_sum(ti_sad_part(L, j * 8, i * 8, q0, cand[k], 8, l16 >> 1, l16 & 1));
      if (s < bc) {
        bc = s;
        b1 = cand[k];
        b0 = q0;
      }
    }
  }
  if (live && l16 == 0) {
    L.f0[(long long)i * bw + j] = b0;
    L.f1[(long long)i * bw + j] = b1;
  }
}

// ---- host: the interpolation context and interpolate_frames ---------------
struct thor_ti {
  int width, height, device, nl;  // nl = max_levels (search levels); pyramid levels nl - 1
  uint8_t *pyr;                   // both references' down-sampled levels (32-px margin)
  uint8_t *lv[2][THOR_PYR_MAX];
  int ls[THOR_PYR_MAX];
  uint32_t *fields;               // per level: m0, m1, f0, f1
  long long foff[TI_MAXL];
  int bw[TI_MAXL], bh[TI_MAXL];
  unsigned long long *pub;        // per level: published step vectors (k_ti_search)
  long long poff[TI_MAXL];
  unsigned *tickets;              // one per level
  unsigned gen;                   // last generation tag used
  unsigned long long *dbg;        // diagnostics: level-0 step stamps (thor_ti_debug)
  unsigned *err;
};

static int ti_levels_host(int w, int h) {  // max_levels (:977)
  const int m = w < h ? w : h;
  if (m <= 0) return 0;
  const int l = (int)(log10((double)m) / log10(2.0) - 4.0);
  return l < TI_MAXL ? l : TI_MAXL;
}

extern "C" {

thor_ti_t *thor_ti_create(int width, int height, int device) {
  create_begin();
  const int nl = width <= 0 || height <= 0 || (width & 7) || (height & 7) ? 0 : ti_levels_host(width, height);
  if (nl < 1) {
    create_fail(THOR_ERR_ARG, 0, "thor_ti_create: unsupported frame size %dx%d", width, height);
    return nullptr;
  }
  if (hipSetDevice(device) != hipSuccess) {
    (void)hipGetLastError();
    create_fail(THOR_ERR_ARG, 0, "thor_ti_create: no HIP device %d", device);
    return nullptr;
  }
  thor_ti *t = new thor_ti();  // value-initialised: every pointer null
  t->width = width;
  t->height = height;
  t->device = device;
  t->nl = nl;
  size_t pbytes = 0;
  for (int l = 1; l < nl; l++) {
    const int w = width >> l, h = height >> l;
    t->ls[l - 1] = (w + 2 * THOR_PYR_PAD + 15) & ~15;
    pbytes += 2 * (((size_t)(h + 2 * THOR_PYR_PAD) * t->ls[l - 1] + 255) & ~(size_t)255);
  }
  size_t fwords = 0, pwords = 0;
  for (int l = 0; l < nl; l++) {
    const int w = width >> l, h = height >> l;
    t->bw[l] = 2 * ((w + 15) / 16);
    t->bh[l] = 2 * ((h + 15) / 16);
    t->foff[l] = (long long)fwords;
    fwords += 4 * (size_t)t->bw[l] * t->bh[l];
    t->poff[l] = (long long)pwords;
    pwords += (size_t)(t->bh[l] / 2) * (t->bw[l] / 2);
  }
  bool ok = true;
  // + 256: the search window's last 16-byte tile of a row may run past the last plane's end
  if (pbytes) ok = dev_alloc(&t->pyr, pbytes + 256, "thor_ti_create: pyramids");
  ok = ok && dev_alloc(&t->fields, fwords * 4, "thor_ti_create: vector fields");
  ok = ok && dev_alloc(&t->pub, pwords * 8, "thor_ti_create: publication words") &&
       hipMemset(t->pub, 0, pwords * 8) == hipSuccess;
  ok = ok && dev_alloc(&t->tickets, 64, "thor_ti_create: tickets");
  ok = ok && dev_alloc(&t->err, 64, "thor_ti_create: error word") && hipMemset(t->err, 0, 64) == hipSuccess;
  if (!ok) {
    create_fail(THOR_ERR_HIP, 0, "thor_ti_create: HIP call failed");
    (void)hipGetLastError();
    thor_ti_destroy(t);
    return nullptr;
  }
  size_t o = 0;
  for (int l = 1; l < nl; l++) {
    const int h = height >> l;
    const size_t b = ((size_t)(h + 2 * THOR_PYR_PAD) * t->ls[l - 1] + 255) & ~(size_t)255;
    for (int k = 0; k < 2; k++) {
      t->lv[k][l - 1] = t->pyr + o + (size_t)THOR_PYR_PAD * t->ls[l - 1] + THOR_PYR_PAD;
      o += b;
    }
  }
  return t;
}

void thor_ti_destroy(thor_ti_t *t) {
  if (!t) return;
  (void)hipSetDevice(t->device);
  if (t->pyr) (void)hipFree(t->pyr);
  if (t->fields) (void)hipFree(t->fields);
  if (t->pub) (void)hipFree(t->pub);
  if (t->tickets) (void)hipFree(t->tickets);
  if (t->err) (void)hipFree(t->err);
  delete t;
}

int thor_interpolate_frames(thor_ti_t *t, const thor_yuv_planes_t *ref0, const thor_yuv_planes_t *ref1, int pad_y,
                            const thor_yuv_planes_t *out, int ratio, int pos, void *stream) {
  if (!t || !ref0 || !ref1 || !out || ratio <= 0 || pos < 0 || pad_y < 16) return THOR_ERR_ARG;
  if (ref0->stride_y != ref1->stride_y || ref0->stride_c != ref1->stride_c) return THOR_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  const int W = t->width, H = t->height, nl = t->nl;
  // alloc_mv_data weights, interpolating (:120-126)
  const int rev = pos > ratio / 2;
  const int wt0 = rev ? pos : ratio - pos, wt1 = ratio - wt0;
  if (nl > 1) {
    const int rc = thor_scale_pyramid2(ref0->y, ref1->y, ref0->stride_y, W, H, t->lv[0], t->lv[1], t->ls, nl - 1, stream);
    if (rc != THOR_OK) return rc;
  }
  if (hipMemsetAsync(t->tickets, 0, 4 * TI_MAXL, st) != hipSuccess) return THOR_ERR_HIP;
  for (int l = nl - 1; l >= 0; l--) {
    TiLevel L;
    const uint8_t *a = l ? t->lv[0][l - 1] : ref0->y, *b = l ? t->lv[1][l - 1] : ref1->y;
    L.p0 = rev ? b : a;
    L.p1 = rev ? a : b;
    L.s0 = L.s1 = l ? t->ls[l - 1] : ref0->stride_y;
    L.w = W >> l;
    L.h = H >> l;
    L.pad = l ? THOR_PYR_PAD : pad_y;
    L.bw = t->bw[l];
    L.bh = t->bh[l];
    L.wt0 = wt0;
    L.wt1 = wt1;
    const size_t area = (size_t)L.bw * L.bh;
    uint32_t *F = t->fields + t->foff[l];
    L.m0 = F;
    L.m1 = F + area;
    L.f0 = F + 2 * area;
    L.f1 = F + 3 * area;
    L.guide = l + 1 < nl ? t->fields + t->foff[l + 1] + 3 * (size_t)t->bw[l + 1] * t->bh[l + 1] : nullptr;
    L.gbw = l + 1 < nl ? t->bw[l + 1] : 0;
    L.pub = t->pub + t->poff[l];
    L.ticket = t->tickets + l;
    L.gen = ++t->gen;  // a fresh tag: words of earlier launches never read as ready
    if (L.gen == 0) L.gen = ++t->gen;
    L.err = t->err;
    L.dbg = l == 0 ? t->dbg : nullptr;
    k_ti_search<<<L.bh / 2, 64, 0, st>>>(L);
    if (hipGetLastError() != hipSuccess) return THOR_ERR_HIP;
    k_ti_merge<<<(unsigned)((area * 16 + 255) / 256), 256, 0, st>>>(L);
    if (hipGetLastError() != hipSuccess) return THOR_ERR_HIP;
  }
  // interpolate_frame (:946-970) with the level-0 final field
  const size_t area0 = (size_t)t->bw[0] * t->bh[0];
  const uint32_t *F0 = t->fields + t->foff[0];
  thor_interp_plane_t pl[3];
  const thor_yuv_planes_t *pa = rev ? ref1 : ref0, *pb = rev ? ref0 : ref1;
  pl[0] = {pa->y, pb->y, out->y, pa->stride_y, pb->stride_y, out->stride_y};
  pl[1] = {pa->u, pb->u, out->u, pa->stride_c, pb->stride_c, out->stride_c};
  pl[2] = {pa->v, pb->v, out->v, pa->stride_c, pb->stride_c, out->stride_c};
  return thor_interp_frame(pl, (const int16_t *)(F0 + 2 * area0), (const int16_t *)(F0 + 3 * area0), t->bw[0],
                           t->bh[0], W, H, wt0, wt1, stream);
}

int thor_ti_read_fields(thor_ti_t *t, int level, int16_t *mv0, int16_t *mv1) {
  if (!t || level < 0 || level >= t->nl) return THOR_ERR_ARG;
  if (hipSetDevice(t->device) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return THOR_ERR_HIP;
  unsigned e = 0;
  if (hipMemcpy(&e, t->err, 4, hipMemcpyDeviceToHost) != hipSuccess) return THOR_ERR_HIP;
  if (e) return THOR_ERR_HIP;
  const size_t area = (size_t)t->bw[level] * t->bh[level];
  const uint32_t *F = t->fields + t->foff[level];
  if (mv0 && hipMemcpy(mv0, F + 2 * area, area * 4, hipMemcpyDeviceToHost) != hipSuccess) return THOR_ERR_HIP;
  if (mv1 && hipMemcpy(mv1, F + 3 * area, area * 4, hipMemcpyDeviceToHost) != hipSuccess) return THOR_ERR_HIP;
  return THOR_OK;
}

// Diagnostics (not in the public header): record (ready, done) s_memrealtime
// stamps of every level-0 search step into dev_buf (2 x u64 per step).
int thor_ti_debug(thor_ti_t *t, void *dev_buf) {
  if (!t) return THOR_ERR_ARG;
  t->dbg = (unsigned long long *)dev_buf;
  return THOR_OK;
}

int thor_ti_status(thor_ti_t *t) {
  if (!t) return THOR_ERR_ARG;
  unsigned e = 0;
  if (hipMemcpy(&e, t->err, 4, hipMemcpyDeviceToHost) != hipSuccess) return THOR_ERR_HIP;
  if (e) {
    const unsigned z = 0;
    (void)hipMemcpy(t->err, &z, 4, hipMemcpyHostToDevice);
    return THOR_ERR_HIP;
  }
  return THOR_OK;
}

}  // extern "C"
