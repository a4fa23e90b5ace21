// In-loop filters and reference padding for gfx950: deblock_frame_y/uv
// (common/common_frame.c:46-321), clpf_frame (:485-557), pad_yuv_frame
// (:405-462).  All in place on the current slot.
#include "common.h"

// beta_table / tc_table, common/common_frame.c:36-44
__device__ __forceinline__ int beta_of(int qp) {
  const int t[52] = {0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  6,  7,
                     8,  9,  10, 11, 12, 13, 14, 15, 16, 17, 18, 20, 22, 24, 26, 28, 30, 32,
                     34, 36, 38, 40, 42, 44, 46, 48, 50, 52, 54, 56, 58, 60, 62, 64};
  return t[qp];
}
__device__ __forceinline__ int tc_of(int qp) {
  const int t[56] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1,  1,  1,  1,  1,  1,  1,  1,  1, 2,
                     2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 5, 5, 6, 6, 7, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13, 14, 14};
  return t[qp];
}

// Luma edge decision for one 4-pixel segment (common/common_frame.c:80-115,
// NEW_DEBLOCK_TEST / NEW_MV_TEST): pos = j (vertical) or i (horizontal).
__device__ __forceinline__ bool luma_edge_on(uint16_t P, uint16_t Q, int pos, bool vertical) {
  int lq = vertical ? CI_LQV(Q) : CI_LQH(Q);
  bool interior = (pos & ((1 << lq) - 1)) != 0;
  bool mv = CI_MVBIG(P) | CI_MVBIG(Q);
  bool cbp = CI_CBPY(P) | CI_CBPY(Q);
  bool intra = CI_MODE(P) == 1 || CI_MODE(Q) == 1;
  return !interior && (mv || cbp || intra);
}

__device__ __forceinline__ void filt4(int &p1, int &p0, int &q0, int &q1, int tc) {
  // NEW_DEBLOCK_FILTER (common/common_frame.c:133-147); delta/2 truncates toward 0
  int delta = (18 * (q0 - p0) - 6 * (q1 - p1) + 16) >> 5;
  delta = delta < -tc ? -tc : (delta > tc ? tc : delta);
  int h = delta / 2;
  int np1 = clip255(p1 + h), np0 = clip255(p0 + delta), nq0 = clip255(q0 - delta), nq1 = clip255(q1 - h);
  p1 = np1; p0 = np0; q0 = nq0; q1 = nq1;
}

// R luma edge segments per lane in three phases, so every phase's global
// loads are in flight together: (1) the side-info decisions of all items,
// (2) the pixels of the items that are on, (3) activity test, filter, store.
template <int R>
__device__ __forceinline__ void luma_v_items(int t0, int tstep, uint8_t *Y, int sy, int W, int H,
                                             const uint16_t *cell, int qp, int g0 = 0, int g1 = 1 << 30) {
  const int ne = (W >> 3) - 1, cs = W >> 2;
  const int beta = beta_of(qp), tc = tc_of(qp);
  int ii[R], jj[R];
  uint16_t cq[R][4];
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int t = t0 + r * tstep, g = t / ne, e = t - g * ne + 1;
    ii[r] = g * 8;
    jj[r] = e * 8;
    cq[r][0] = cq[r][1] = cq[r][2] = cq[r][3] = 0;
    if (g < (H >> 3) && g >= g0 && g < g1) {  // [g0, g1): 8-row groups of a row band (phase_b_rows)
      const int qa = (ii[r] >> 2) * cs + (jj[r] >> 2);
      cq[r][0] = cell[qa - 1];
      cq[r][1] = cell[qa];
      cq[r][2] = cell[qa + cs - 1];
      cq[r][3] = cell[qa + cs];
    }
  }
  bool on0[R], on1[R];
  uint32_t A[R][8], Bv[R][8];
#pragma unroll
  for (int r = 0; r < R; r++) {
    on0[r] = cq[r][1] && luma_edge_on(cq[r][0], cq[r][1], jj[r], true);  // cq 0: past the frame
    on1[r] = cq[r][3] && luma_edge_on(cq[r][2], cq[r][3], jj[r], true);
    if (on0[r] || on1[r]) {
      const uint8_t *base = Y + (long long)ii[r] * sy + jj[r] - 4;
#pragma unroll
      for (int k = 0; k < 8; k++) {  // rows 2 and 5 feed the activity test; the rest only where filtered
        A[r][k] = Bv[r][k] = 0;
        if (k == 2 || k == 5 || (k < 4 ? on0[r] : on1[r])) {
          A[r][k] = *(const uint32_t *)(base + (long long)k * sy);
          Bv[r][k] = *(const uint32_t *)(base + (long long)k * sy + 4);
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; r++) {
    if (!(on0[r] || on1[r])) continue;
    // p1 = A byte2, p0 = A byte3, q0 = B byte0, q1 = B byte1
#define P1(k) ((int)((A[r][k] >> 16) & 255))
#define P0(k) ((int)(A[r][k] >> 24))
#define Q0(k) ((int)(Bv[r][k] & 255))
#define Q1(k) ((int)((Bv[r][k] >> 8) & 255))
    const int d = abs(P1(2) - P0(2)) + abs(Q1(2) - Q0(2)) + abs(P1(5) - P0(5)) + abs(Q1(5) - Q0(5));
    if (d >= beta) continue;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      if (!(k < 4 ? on0[r] : on1[r])) continue;
      int p1 = P1(k), p0 = P0(k), q0 = Q0(k), q1 = Q1(k);
      filt4(p1, p0, q0, q1, tc);
      A[r][k] = (A[r][k] & 0xffffu) | ((uint32_t)p1 << 16) | ((uint32_t)p0 << 24);
      Bv[r][k] = (Bv[r][k] & 0xffff0000u) | (uint32_t)q0 | ((uint32_t)q1 << 8);
    }
#undef P1
#undef P0
#undef Q0
#undef Q1
    uint8_t *base = Y + (long long)ii[r] * sy + jj[r] - 4;
#pragma unroll
    for (int k = 0; k < 8; k++) {  // only the filtered half's rows go back
      if (!(k < 4 ? on0[r] : on1[r])) continue;
      *(uint32_t *)(base + (long long)k * sy) = A[r][k];
      *(uint32_t *)(base + (long long)k * sy + 4) = Bv[r][k];
    }
  }
}

template <int R>
__device__ __forceinline__ void luma_h_items(int t0, int tstep, uint8_t *Y, int sy, int W, int H,
                                             const uint16_t *cell, int qp, int i0 = 0, int i1 = 1 << 30) {
  const int ng = W >> 3, cs = W >> 2;
  const int beta = beta_of(qp), tc = tc_of(qp);
  int ii[R], jj[R];
  uint16_t cq[R][4];
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int t = t0 + r * tstep, k = t / ng, gcol = t - k * ng;
    ii[r] = (k + 1) * 8;
    jj[r] = gcol * 8;
    cq[r][0] = cq[r][1] = cq[r][2] = cq[r][3] = 0;
    if (ii[r] < H && ii[r] >= i0 && ii[r] <= i1) {  // [i0, i1]: edges of a row band (phase_b_rows)
      const int qa = (ii[r] >> 2) * cs + (jj[r] >> 2);
      cq[r][0] = cell[qa - cs];
      cq[r][1] = cell[qa];
      cq[r][2] = cell[qa + 1 - cs];
      cq[r][3] = cell[qa + 1];
    }
  }
  bool on0[R], on1[R];
  uint2 rows[R][4];  // rows i-2 .. i+1 (p1, p0, q0, q1)
#pragma unroll
  for (int r = 0; r < R; r++) {
    on0[r] = cq[r][1] && luma_edge_on(cq[r][0], cq[r][1], ii[r], false);
    on1[r] = cq[r][3] && luma_edge_on(cq[r][2], cq[r][3], ii[r], false);
    if (on0[r] || on1[r]) {
      const uint8_t *base = Y + (long long)(ii[r] - 2) * sy + jj[r];
#pragma unroll
      for (int k = 0; k < 4; k++) rows[r][k] = *(const uint2 *)(base + (long long)k * sy);
    }
  }
#pragma unroll
  for (int r = 0; r < R; r++) {
    if (!(on0[r] || on1[r])) continue;
    auto px = [&](int k, int c) -> int { return (int)(((c < 4 ? rows[r][k].x : rows[r][k].y) >> (8 * (c & 3))) & 255); };
    const int d =
        abs(px(0, 2) - px(1, 2)) + abs(px(3, 2) - px(2, 2)) + abs(px(0, 5) - px(1, 5)) + abs(px(3, 5) - px(2, 5));
    if (d >= beta) continue;
    uint32_t out[4][2] = {{rows[r][0].x, rows[r][0].y}, {rows[r][1].x, rows[r][1].y}, {rows[r][2].x, rows[r][2].y},
                          {rows[r][3].x, rows[r][3].y}};
#pragma unroll
    for (int n = 0; n < 8; n += 4) {
      if (!(n ? on1[r] : on0[r])) continue;
      const int w = n >> 2;
      uint32_t o0 = 0, o1 = 0, o2 = 0, o3 = 0;
#pragma unroll
      for (int c = 0; c < 4; c++) {
        int p1 = px(0, n + c), p0 = px(1, n + c), q0 = px(2, n + c), q1 = px(3, n + c);
        filt4(p1, p0, q0, q1, tc);
        o0 |= (uint32_t)p1 << (8 * c);
        o1 |= (uint32_t)p0 << (8 * c);
        o2 |= (uint32_t)q0 << (8 * c);
        o3 |= (uint32_t)q1 << (8 * c);
      }
      out[0][w] = o0; out[1][w] = o1; out[2][w] = o2; out[3][w] = o3;
    }
    uint8_t *base = Y + (long long)(ii[r] - 2) * sy + jj[r];
#pragma unroll
    for (int k = 0; k < 4; k++) *(uint2 *)(base + (long long)k * sy) = make_uint2(out[k][0], out[k][1]);
  }
}

// Chroma (deblock_frame_uv): intra-only edges, p0/q0 modified.  One thread
// per (edge, 8-luma-row/column group) per plane (blockIdx.y = plane).
__device__ __forceinline__ void k_deblock_chroma_v_body(int t, int by, uint8_t *U, uint8_t *V, int sc, int W, int H,
                                                          const uint16_t *cell, int qpc, int g0 = 0, int g1 = 1 << 30) {
  uint8_t *C = by ? V : U;
  int ne = (W >> 3) - 1;
  int g = t / ne, e = t - g * ne + 1;
  if (g >= (H >> 3) || g < g0 || g >= g1) return;
  int i = g * 8, j = e * 8;
  int cs = W >> 2;
  int qi = (i >> 2) * cs + (j >> 2);
  uint16_t P = cell[qi - 1], Q = cell[qi];
  bool intra = CI_MODE(P) == 1 || CI_MODE(Q) == 1;
  bool interior = (j & ((1 << CI_LSZ(Q)) - 1)) != 0;
  if (!intra || interior) return;
  int tc = tc_of(qpc);
  int i2 = i >> 1, j2 = j >> 1;
  for (int k = 0; k < 4; k++) {
    uint8_t *p = C + (long long)(i2 + k) * sc + j2;
    int p1 = p[-2], p0 = p[-1], q0 = p[0], q1 = p[1];
    int delta = (4 * (q0 - p0) + (p1 - q1) + 4) >> 3;
    delta = delta < -tc ? -tc : (delta > tc ? tc : delta);
    p[-1] = (uint8_t)clip255(p0 + delta);
    p[0] = (uint8_t)clip255(q0 - delta);
  }
}

__device__ __forceinline__ void k_deblock_chroma_h_body(int t, int by, uint8_t *U, uint8_t *V, int sc, int W, int H,
                                                          const uint16_t *cell, int qpc, int i0 = 0, int i1 = 1 << 30) {
  uint8_t *C = by ? V : U;
  int ng = W >> 3;
  int k = t / ng, gcol = t - k * ng;
  int i = (k + 1) * 8, j = gcol * 8;
  if (i >= H || i < i0 || i > i1) return;
  int cs = W >> 2;
  int qi = (i >> 2) * cs + (j >> 2);
  uint16_t P = cell[qi - cs], Q = cell[qi];
  bool intra = CI_MODE(P) == 1 || CI_MODE(Q) == 1;
  bool interior = (i & ((1 << CI_LSZ(Q)) - 1)) != 0;
  if (!intra || interior) return;
  int tc = tc_of(qpc);
  int i2 = i >> 1, j2 = j >> 1;
  for (int l = 0; l < 4; l++) {
    uint8_t *p = C + (long long)i2 * sc + j2 + l;
    int p1 = p[-2 * sc], p0 = p[-sc], q0 = p[0], q1 = p[sc];
    int delta = (4 * (q0 - p0) + (p1 - q1) + 4) >> 3;
    delta = delta < -tc ? -tc : (delta > tc ? tc : delta);
    p[-sc] = (uint8_t)clip255(p0 + delta);
    p[0] = (uint8_t)clip255(q0 - delta);
  }
}

// CLPF, one workgroup per whole 64x64 SB (the SB count is floor'd,
// common/common_frame.c:496-497).  The SB is filtered when some 8x8 block is
// a candidate (not BIPRED, any cbp) and the stream's decision flag is set.
// Every 8x8 block that is not BIPRED is filtered per plane with coded
// residual (clpf_block, common/common_block.c:180-197), reading the
// unfiltered SB (LDS copy) with clamping at the SB border.
// One launch per edge direction for every frame of a batch (grid y = frame):
// luma blocks first, then U, then V (the chroma filters read only the cell
// side info, never luma pixels, so the planes are independent within a pass;
// vertical edges of all planes before horizontal ones, deblock_frame_y /
// deblock_frame_uv, common/common_frame.c:46-321).
// Chroma edges filter only where P or Q is intra (deblock_frame_uv,
// common/common_frame.c:243-321), so they are enumerated from the frame's
// intra CU list: one wave per (intra CU, plane), one lane per 8-luma-pixel
// segment of its left / right (vertical pass) or top / bottom (horizontal
// pass) boundary.  An edge between two intra CUs is filtered once, by the CU
// on its Q side.
// Row band of a band-local phase B (row sharding, FrameCtx.pb0/pb1 luma rows;
// pb1 = 0: the whole frame).  For every pixel of rows [y0, y1) to come out
// final: horizontal edges at rows i in [y0, y1] (the edge at y1 writes rows
// y1 - 2, y1 - 1) and vertical edges on the 8-row groups covering rows
// [y0 - 2, y1 + 2) that those read, i.e. groups [y0/8 - 1, y1/8 + 1).
struct DbRows {
  int g0, g1, i0, i1;
  __device__ __forceinline__ explicit DbRows(const FrameCtx &f) {
    if (f.pb1 > 0) {
      g0 = (f.pb0 >> 3) - 1;
      g1 = (f.pb1 >> 3) + 1;
      i0 = f.pb0;
      i1 = f.pb1;
    } else {
      g0 = 0;
      g1 = i1 = 1 << 30;
      i0 = 0;
    }
  }
};
__device__ __forceinline__ void chroma_intra_edges(const FrameCtx &f, int item, bool vertical) {
  const int lane = threadIdx.x & 63;
  if (item >= 2 * f.nintra) return;
  const int plane = item & 1;
  const thor_block_t &B = f.blk[f.ilist[item >> 1]];
  const int S = B.size, x = B.xpos, y = B.ypos, nseg = S >> 3;
  if (lane >= 2 * nseg) return;
  const int side = lane >= nseg, k = lane - side * nseg;  // side 0: this CU is Q, 1: this CU is P
  const int cs = f.W >> 2;
  const int i = vertical ? y + 8 * k : (side ? y + S : y);
  const int j = vertical ? (side ? x + S : x) : x + 8 * k;
  if (i >= f.H || j >= f.W || (vertical ? j : i) < 8) return;
  if (side && CI_MODE(f.cellinfo[(i >> 2) * cs + (j >> 2)]) == M_INTRA) return;  // the intra Q CU owns it
  const DbRows rb(f);
  if (vertical)
    k_deblock_chroma_v_body((i >> 3) * ((f.W >> 3) - 1) + (j >> 3) - 1, plane, f.cu, f.cv, f.sc, f.W, f.H,
                            f.cellinfo, f.qpc, rb.g0, rb.g1);
  else
    k_deblock_chroma_h_body(((i >> 3) - 1) * (f.W >> 3) + (j >> 3), plane, f.cu, f.cv, f.sc, f.W, f.H, f.cellinfo,
                            f.qpc, rb.i0, rb.i1);
}

// DB_ITEMS luma edge segments per lane (grid-stride): a quarter as many
// waves, and most segments of a skip-dominated frame end after two side-info
// reads.  Blocks [0, nbl): luma; [nbl, ...): chroma of the intra CUs (four
// (CU, plane) items per workgroup).
#define DB_ITEMS 4
__global__ __launch_bounds__(256) void k_deblock_v(const FrameBatch fb_, int nbl, int clist) {
  const FrameCtx *__restrict__ F = FRAME_BATCH_CTX();
  const FrameCtx &f = F[blockIdx.y];
  if (!f.deblock) return;
  const int b = blockIdx.x;
  if (b >= nbl) {
    if (clist) {  // few intra CUs: enumerate their boundaries
      chroma_intra_edges(f, (b - nbl) * 4 + (threadIdx.x >> 6), true);
      return;
    }
    const int c = (b - nbl) >= nbl, bb = b - nbl - c * nbl;  // every chroma edge segment, per plane
    for (int r = 0; r < DB_ITEMS; r++)
      k_deblock_chroma_v_body(bb * 256 + (int)threadIdx.x + r * nbl * 256, c, f.cu, f.cv, f.sc, f.W, f.H, f.cellinfo, f.qpc,
                              DbRows(f).g0, DbRows(f).g1);
    return;
  }
  const DbRows rb(f);
  luma_v_items<DB_ITEMS>(b * 256 + (int)threadIdx.x, nbl * 256, f.cy, f.sy, f.W, f.H, f.cellinfo, f.qp, rb.g0, rb.g1);
}
__global__ __launch_bounds__(256) void k_deblock_h(const FrameBatch fb_, int nbl, int clist) {
  const FrameCtx *__restrict__ F = FRAME_BATCH_CTX();
  const FrameCtx &f = F[blockIdx.y];
  if (!f.deblock) return;
  const int b = blockIdx.x;
  if (b >= nbl) {
    if (clist) {  // few intra CUs: enumerate their boundaries
      chroma_intra_edges(f, (b - nbl) * 4 + (threadIdx.x >> 6), false);
      return;
    }
    const int c = (b - nbl) >= nbl, bb = b - nbl - c * nbl;  // every chroma edge segment, per plane
    for (int r = 0; r < DB_ITEMS; r++)
      k_deblock_chroma_h_body(bb * 256 + (int)threadIdx.x + r * nbl * 256, c, f.cu, f.cv, f.sc, f.W, f.H, f.cellinfo, f.qpc,
                              DbRows(f).i0, DbRows(f).i1);
    return;
  }
  const DbRows rb(f);
  luma_h_items<DB_ITEMS>(b * 256 + (int)threadIdx.x, nbl * 256, f.cy, f.sy, f.W, f.H, f.cellinfo, f.qp, rb.i0, rb.i1);
}

// One flagged SB per workgroup.  The SB's pixels and its 64 8x8-block side
// info words are loaded speculatively together with the flag (one round
// trip), then staged in LDS; each lane filters 16 consecutive pixels of a row
// and writes them back as one 16-byte store.
__device__ __forceinline__ int clpf_px(const uint8_t *s, int pitch, int n, int r, int c) {
  const int X = s[r * pitch + c];
  const int A = r == 0 ? X : s[(r - 1) * pitch + c];
  const int Bv = c == 0 ? X : s[r * pitch + c - 1];
  const int Cv = c == n - 1 ? X : s[r * pitch + c + 1];
  const int D = r == n - 1 ? X : s[(r + 1) * pitch + c];
  const int delta = ((A > X) + (Bv > X) + (Cv > X) + (D > X) > 2) - ((A < X) + (Bv < X) + (Cv < X) + (D < X) > 2);
  return (X + delta) & 255;
}
__device__ __forceinline__ void k_clpf_body(int bx, uint8_t *Y, uint8_t *U, uint8_t *V, int sy, int sc, int W, int H,
                                            const uint16_t *cell, const uint8_t *flags, uint8_t *sY, uint8_t *sU,
                                            uint8_t *sV, uint16_t *sC) {
  const int nh = W >> 6;
  const int k = bx / nh, l = bx - (bx / nh) * nh;
  const int tid = threadIdx.x;
  const int cs = W >> 2;
  uint8_t *y0 = Y + (long long)(k * 64) * sy + l * 64;
  uint8_t *u0 = U + (long long)(k * 32) * sc + l * 32;
  uint8_t *v0 = V + (long long)(k * 32) * sc + l * 32;
  // speculative loads: flag, the lane's 16 luma bytes, 4 U + 4 V bytes, one side-info word
  const int fl = flags[bx];
  const int ry = tid >> 2, cy = (tid & 3) * 16;
  const uint4 py = *(const uint4 *)(y0 + (long long)ry * sy + cy);
  const int rc = tid >> 3, cc = (tid & 7) * 4;
  const uint32_t pu = *(const uint32_t *)(u0 + (long long)rc * sc + cc);
  const uint32_t pv = *(const uint32_t *)(v0 + (long long)rc * sc + cc);
  uint16_t ci = 0;
  if (tid < 64) ci = cell[((k * 64 + (tid >> 3) * 8) >> 2) * cs + ((l * 64 + (tid & 7) * 8) >> 2)];
  if (!fl) return;  // uniform
  *(uint4 *)&sY[ry * 64 + cy] = py;
  *(uint32_t *)&sU[rc * 32 + cc] = pu;
  *(uint32_t *)&sV[rc * 32 + cc] = pv;
  if (tid < 64) sC[tid] = ci;
  __syncthreads();
  // candidate SB: some 8x8 block not BIPRED with any cbp (clpf_frame, common/common_frame.c:498-508)
  int cand = 0;
  for (int b = 0; b < 64; b++) {
    const uint16_t c = sC[b];
    cand |= CI_MODE(c) != 3 && (CI_CBPY(c) | CI_CBPU(c) | CI_CBPV(c));
  }
  if (!cand) return;  // uniform (every lane read the same 64 words)
  // luma: 16 pixels of row ry from column cy (two 8x8 blocks)
  {
    uint32_t o[4];
    const uint16_t c0 = sC[(ry >> 3) * 8 + (cy >> 3)], c1 = sC[(ry >> 3) * 8 + (cy >> 3) + 1];
    const bool f0 = CI_MODE(c0) != 3 && CI_CBPY(c0), f1 = CI_MODE(c1) != 3 && CI_CBPY(c1);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      uint32_t w = 0;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int c = cy + 4 * q + j;
        const bool f = (4 * q + j) < 8 ? f0 : f1;
        const int v = f ? clpf_px(sY, 64, 64, ry, c) : sY[ry * 64 + c];
        w |= (uint32_t)v << (8 * j);
      }
      o[q] = w;
    }
    if (f0 || f1) *(uint4 *)(y0 + (long long)ry * sy + cy) = make_uint4(o[0], o[1], o[2], o[3]);
  }
  // chroma: lanes 0-63 U, 64-127 V; 16 pixels of row r from column c0 (four 4x4 blocks)
  if (tid < 128) {
    const int pl = tid >> 6, t = tid & 63;
    const int r = t >> 1, c0 = (t & 1) * 16;
    const uint8_t *s = pl ? sV : sU;
    uint32_t o[4];
    bool any = false;
#pragma unroll
    for (int q = 0; q < 4; q++) {  // 4x4 chroma block q of the 16 columns = 8x8 luma block (r/4, c0/4 + q)
      const uint16_t c = sC[(r >> 2) * 8 + (c0 >> 2) + q];
      const bool f = CI_MODE(c) != 3 && (pl ? CI_CBPV(c) : CI_CBPU(c));
      any |= f;
      uint32_t w = 0;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int cc2 = c0 + 4 * q + j;
        const int v = f ? clpf_px(s, 32, 32, r, cc2) : s[r * 32 + cc2];
        w |= (uint32_t)v << (8 * j);
      }
      o[q] = w;
    }
    if (any) *(uint4 *)((pl ? v0 : u0) + (long long)r * sc + c0) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}
__global__ __launch_bounds__(256) void k_clpf(const FrameBatch fb_) {
  const FrameCtx *__restrict__ F = FRAME_BATCH_CTX();
  __shared__ uint8_t sY[64 * 64], sU[32 * 32], sV[32 * 32];
  __shared__ uint16_t sC[64];
  const FrameCtx &f = F[blockIdx.y];
  if (!f.clpf_on) return;
  // one workgroup per flagged SB (the host's list), or per SB without a list
  const int nwork = f.n_clpf >= 0 ? f.n_clpf : (f.W >> 6) * (f.H >> 6);
  if ((int)blockIdx.x >= nwork) return;
  const int sb = f.n_clpf >= 0 ? (int)f.clpf_list[blockIdx.x] : (int)blockIdx.x;
  if (sb >= (f.W >> 6) * (f.H >> 6)) return;
  if (f.pb1 > 0) {  // band-local phase B: the band's SB rows only (CLPF reads nothing outside its SB)
    const int r = sb / (f.W >> 6);
    if (r < (f.pb0 >> 6) || r >= ((f.pb1 + 63) >> 6)) return;
  }
  k_clpf_body(sb, f.cy, f.cu, f.cv, f.sy, f.sc, f.W, f.H, f.cellinfo, f.clpf_flags, sY, sU, sV, sC);
}


// pad_yuv_frame (common/common_frame.c:405-462): every padding byte equals
// the nearest interior pixel (rows clamp, then columns clamp).  Work unit = one
// 16-byte chunk of padding: per plane, the side margins of every interior row
// (left [-pad, 0), right [w & ~15, w + pad) -- a chunk straddling the right
// edge keeps its interior bytes), then the top / bottom pad rows over
// [-pad, w + pad) rounded up to 16 (still inside the stride).  Rows start
// 16-byte aligned at x = -pad (create_yuv_frame's strides and pads).
// Row sharding pads only the rows a rank holds final: interior rows [r0, r1),
// the top pad rows when r0 == 0 and the bottom ones when r1 == h (the whole
// plane: r0 = 0, r1 = h).
struct PadPlane {
  uint8_t *P;
  int s, w, h, pad, nl, nr, rc, r0, ntop, sides, total;
  __device__ __forceinline__ PadPlane(uint8_t *P_, int s_, int w_, int h_, int pad_, int r0_, int r1_)
      : P(P_), s(s_), w(w_), h(h_), pad(pad_), r0(r0_) {
    nl = pad >> 4;
    nr = (w + pad - (w & ~15) + 15) >> 4;
    rc = (w + 2 * pad + 15) >> 4;
    sides = (r1_ - r0_) * (nl + nr);
    ntop = r0_ == 0 ? pad : 0;
    total = sides + (ntop + (r1_ == h ? pad : 0)) * rc;
  }
  __device__ __forceinline__ void chunk(int e) const {
    int row, x0;
    const uint8_t *src;
    if (e < sides) {
      row = e / (nl + nr);
      const int k = e - row * (nl + nr);
      row += r0;
      src = P + (long long)row * s;
      x0 = k < nl ? -pad + 16 * k : (w & ~15) + 16 * (k - nl);
    } else {
      const int e2 = e - sides, r = e2 / rc;
      x0 = -pad + 16 * (e2 - r * rc);
      row = r < ntop ? r - pad : h + (r - ntop);
      src = P + (long long)(r < ntop ? 0 : h - 1) * s;
    }
    uint8_t *dst = P + (long long)row * s + x0;
    uint4 v;
    if (x0 >= 0 && x0 + 16 <= w) {
      v = *(const uint4 *)(src + x0);
    } else if (x0 + 16 <= 0 || x0 >= w) {
      const uint32_t b = (uint32_t)src[x0 < 0 ? 0 : w - 1] * 0x01010101u;
      v = make_uint4(b, b, b, b);
    } else {
      uint32_t wd[4];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        uint32_t acc = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
          int x = x0 + 4 * q + j;
          x = x < 0 ? 0 : (x > w - 1 ? w - 1 : x);
          acc |= (uint32_t)src[x] << (8 * j);
        }
        wd[q] = acc;
      }
      v = make_uint4(wd[0], wd[1], wd[2], wd[3]);
    }
    *(uint4 *)dst = v;
  }
};
__device__ __forceinline__ void k_pad_body(int e, uint8_t *Y, uint8_t *U, uint8_t *V, int sy, int sc, int W, int H,
                                           int r0, int r1) {
  const PadPlane py(Y, sy, W, H, THOR_PAD_Y, r0, r1);
  if (e < py.total) {
    py.chunk(e);
    return;
  }
  e -= py.total;
  const PadPlane pu(U, sc, W >> 1, H >> 1, THOR_PAD_C, r0 >> 1, r1 >> 1);
  if (e < pu.total) {
    pu.chunk(e);
    return;
  }
  e -= pu.total;
  const PadPlane pv(V, sc, W >> 1, H >> 1, THOR_PAD_C, r0 >> 1, r1 >> 1);
  if (e < pv.total) pv.chunk(e);
}
// every frame of a batch (grid z); also used on one frame by thor_dec_write_frame.
// Luma rows [r0, r1) of each frame (even; r1 <= 0: the whole frame).
__global__ __launch_bounds__(256) void k_pad(const FrameBatch fb_, int r0, int r1) {
  const FrameCtx *__restrict__ F = FRAME_BATCH_CTX();
  const FrameCtx &f = F[blockIdx.y];
  if (r1 <= 0) r0 = 0, r1 = f.H;
  k_pad_body(blockIdx.x * 256 + threadIdx.x, f.cy, f.cu, f.cv, f.sy, f.sc, f.W, f.H, r0, r1);
}
// 16-byte chunks of padding of one frame (host-side copy of PadPlane's count),
// luma rows [r0, r1) (r1 <= 0: all)
static inline int pad_chunks(int W, int H, int r0 = 0, int r1 = 0) {
  if (r1 <= 0) r0 = 0, r1 = H;
  auto plane = [](int w, int h, int pad, int a, int b) {
    const int nl = pad >> 4, nr = (w + pad - (w & ~15) + 15) >> 4, rc = (w + 2 * pad + 15) >> 4;
    return (b - a) * (nl + nr) + ((a == 0 ? pad : 0) + (b == h ? pad : 0)) * rc;
  };
  return plane(W, H, THOR_PAD_Y, r0, r1) + 2 * plane(W >> 1, H >> 1, THOR_PAD_C, r0 >> 1, r1 >> 1);
}
