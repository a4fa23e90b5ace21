// Intra reconstruction for gfx950: decode_and_reconstruct_block_intra
// (dec/decode_block.c:48-88) over a frame's intra CUs.
//
// Intra CUs read the pre-deblock reconstruction of their left / top / top-left
// / top-right / bottom-left neighbours (make_top_and_left,
// common/intra_prediction.c:57-143), so they form a dependency chain in
// decode order.  Y, U and V never read each other, so a frame's intra work is
// 3 x (SB rows) independent chains.  Each chain is ONE wave: it owns one
// component of one 64x64 SB row and reconstructs that row's intra CUs in
// decode order, one transform block at a time.  A chain is a latency chain,
// not a throughput problem, so a single wave is the fast shape: its LDS
// operations complete in order (no barriers between building a block's
// neighbour arrays and predicting from them), its uniform block parameters
// are computed once (not once per wave of a workgroup, on the CU's one scalar
// unit), and the DC sum is a DPP reduction.  The rows of a component form a
// wavefront (WPP pattern): row k may work on SB l once row k-1 of the same
// component has completed SBs 0..l+1 (the top-right neighbour is the furthest
// pixel read, common/common_block.c:110-118; the bottom-left is never read
// across an SB row, :120-129).
//
// Transform blocks reconstruct into the SB's LDS image only.  When a chain
// leaves an SB it stores the SB's bottom pixel row -- the only pixels the
// next chain reads -- to an edge-row buffer, then the whole image to the
// frame.  Hand-off without agent-scope fences (cdna_hip_programming.md
// Guideline 16, form R1): the edge store is write-through (sc1) and waited for
// alone, then one lane publishes the progress word with a relaxed agent-scope
// atomic; the consumer polls that word relaxed and reads the edge row with
// sc1 loads (which bypass its L1), so no acquire is needed.  Everything else
// a chain reads comes from earlier launches (residual, k_recon's pixels, the
// CU descriptors) and is issued before the poll, so its latency hides behind
// the wait.  Tasks (row, component) are dequeued in row order (atomic head):
// every awaited chain is held by a running workgroup, so the grid drains.
#include "common.h"

#define IMG_X0 4  // image column -4 at byte 0: rows are dword aligned
#define SC1 16    // buffer instruction aux: sc1 (write-through store / L1-bypassing load)

template <int C>
struct CompGeom {
  static constexpr int SZ = C ? 32 : 64;  // SB size in this plane
  static constexpr int IW = SZ + 8;       // image row: cols -4 .. SZ+3
  static constexpr int IH = SZ + 1;       // image rows -1 .. SZ-1
  static constexpr int DW = IW / 4;       // dwords per image row
};

struct IntraChain {
  int16_t res[64 * 64];  // k_prep_resid's residual over the SB (16-B aligned rows)
  int16_t p5[128];       // planar 5-tap filtered edges: top at 0, left at 64
  uint8_t flt[256];      // directional edge array of the current TU (U_OFF layout below)
  uint8_t img[65 * 72];  // SB image of this component
};
// Dynamic LDS: two words per intra CU of the chain's row (cu_words).
extern __shared__ uint2 g_cuw[];

__device__ __forceinline__ int upright_available(int ypos, int xpos, int size, int width) {
  int a = (ypos > 0) && (xpos + size < width);  // common/common_block.c:110-118
  if (size == 32 && (ypos % 64) == 32) a = 0;
  if (size == 16 && ((ypos % 32) == 16 || ((ypos % 64) == 32 && (xpos % 32) == 16))) a = 0;
  if (size == 8 && ((ypos % 16) == 8 || ((ypos % 32) == 16 && (xpos % 16) == 8) || ((ypos % 64) == 32 && (xpos % 32) == 24))) a = 0;
  return a;
}
__device__ __forceinline__ int downleft_available(int ypos, int xpos, int size, int height) {
  int a = (xpos > 0) && (ypos + size < height);  // common/common_block.c:120-129
  if (size == 64) a = 0;
  if (size == 32 && (ypos % 64) == 32) a = 0;
  if (size == 16 && ((ypos % 64) == 48 || ((ypos % 64) == 16 && (xpos % 32) == 16))) a = 0;
  if (size == 8 && ((ypos % 64) == 56 || ((ypos % 16) == 8 && (xpos % 16) == 8) || ((ypos % 64) == 24 && (xpos % 32) == 16))) a = 0;
  return a;
}

// An intra CU as two words (built lane-parallel once per chain, read back
// uniformly): w0 = ypos | xpos << 16; w1 = size | mode << 8 | tb_split << 12 |
// coeff_mask << 13 | up-right available << 16 | down-left available << 17.
// Modes past the last intra mode predict DC (get_intra_prediction's default).
__device__ __forceinline__ uint2 cu_words(const thor_block_t &D, int W, int H) {
  const int y = D.ypos, x = D.xpos, S = D.size;
  const int m = D.intra_mode > 9 ? 0 : D.intra_mode;
  const uint32_t w1 = (uint32_t)S | (uint32_t)m << 8 | (uint32_t)(D.tb_split != 0) << 12 |
                      (uint32_t)(D.coeff_mask & 7) << 13 | (uint32_t)upright_available(y, x, S, W) << 16 |
                      (uint32_t)downleft_available(y, x, S, H) << 17;
  return make_uint2((uint32_t)y | (uint32_t)x << 16, w1);
}

// Parameters of one transform block (uniform: scalar registers).
struct TuP {
  int n, lg, has, mode;
  int iy, ix;  // TU origin inside the SB image
  int toplen, leftlen, top_none, left_none;
  int xnz, ynz;  // xnz bit0: TU x != 0 (DC selector, :366); bit1: CU x > 0 (top_left, :79/:96)
};

// Component C's transform block of TU step t (intra_prediction.c:57-143 +
// dec/decode_block.c:48-88: tb_split gives 4 raster sub-TUs; chroma of an
// 8x8 CU is not split).
__device__ __forceinline__ TuP make_tup(int comp, int S, int tbc, int y, int x, int mode, int cmask, int t, int ur_cb,
                                        int dl_cb) {
  TuP p;
  const int ch = comp != 0;
  const int size = S >> ch;
  const int n = tbc ? size >> 1 : size;
  const int i0_ = tbc ? (t >> 1) * n : 0, j0_ = tbc ? (t & 1) * n : 0;
  const int yp = y >> ch, xp = x >> ch;
  const int sbm = (64 >> ch) - 1;
  p.n = n;
  p.lg = ilog2i(n);
  p.has = (cmask >> comp) & 1;
  p.mode = mode;
  p.iy = (yp & sbm) + i0_;
  p.ix = (xp & sbm) + j0_;
  int dl, ur;  // make_top_and_left availability (intra_prediction.c:70-76, :100-104)
  if (!tbc) { dl = dl_cb; ur = ur_cb; }
  else {
    dl = (j0_ == 0 && (i0_ == 0 || dl_cb)) ? 1 : 0;
    ur = (j0_ == 0 || (i0_ == 0 && ur_cb)) ? 1 : 0;
  }
  p.toplen = ur ? n + 1 : n;
  p.leftlen = dl ? n + 1 : n;
  p.top_none = (yp + i0_) == 0;
  p.left_none = (xp + j0_) == 0;
  p.xnz = ((xp + j0_) != 0) | ((xp > 0) << 1);
  p.ynz = (yp + i0_) != 0;
  return p;
}

__device__ __forceinline__ unsigned ld_progress(const unsigned *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Sum over the wave (every lane active): DPP within rows of 16, then the four
// row sums through readlane.  Uniform result.
__device__ __forceinline__ int wave_sum(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xf, 0xf, true);   // quad_perm [1,0,3,2]
  v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xf, 0xf, true);   // quad_perm [2,3,0,1]
  v += __builtin_amdgcn_update_dpp(0, v, 0x141, 0xf, 0xf, true);  // row_half_mirror
  v += __builtin_amdgcn_update_dpp(0, v, 0x140, 0xf, 0xf, true);  // row_mirror
  return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
         __builtin_amdgcn_readlane(v, 48);
}

// Residual of SB (k, l), 8 int16 per item, plain loads (written by k_prep_resid in
// an earlier launch; rows past the plane read as 0).
template <int C>
struct ResLoad {
  static constexpr int SZ = CompGeom<C>::SZ, PER = SZ / 8, NR = SZ * PER, RR = NR / 64;
  uint4 v[RR];
  __device__ __forceinline__ void issue(__amdgpu_buffer_rsrc_t rr, int pw, int k, int l) {
#pragma unroll
    for (int r = 0; r < RR; r++) {
      const int q = threadIdx.x + 64 * r;
      const int row = q / PER, x = l * SZ + 8 * (q - row * PER), y = k * SZ + row;
      v[r] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rr, 2 * (y * pw + x), 0, 0));
    }
  }
  __device__ __forceinline__ void commit(IntraChain &L) const {
#pragma unroll
    for (int r = 0; r < RR; r++) {
      const int q = threadIdx.x + 64 * r;
      const int row = q / PER, col = 8 * (q - row * PER);
      *(uint4 *)&L.res[row * SZ + col] = v[r];
    }
  }
};

// The pixel image of SB (k, l) of component C in LDS: image row -1 (cols
// -4..SZ+3) is the edge row of SB row k-1 (written by chain k-1, or by
// k_recon for inter pixels): sc1 loads issued after the poll.  With FULL (P
// frames: k_recon reconstructed the inter CUs) rows 0..SZ-1 come from the
// frame, issued before the poll (nothing this launch writes them).  The left
// column is the previous SB's last image column when the chain just left that
// SB, else the frame's (k_recon's pixels; without FULL every CU is intra, so
// the chain visits every SB and only SB 0 lacks a previous one -- its left
// column is outside the frame and never read).  Bytes past the frame's right
// / bottom edge are never used as neighbours (availability,
// common_block.c:100-129).
template <int C, bool FULL>
struct ImgLoad {
  using G = CompGeom<C>;
  static constexpr int PER = G::SZ / 16;                  // 16-B pieces per interior row
  static constexpr int RI = FULL ? G::SZ * PER / 64 : 0;  // per lane
  uint4 iv[RI > 0 ? RI : 1];
  uint32_t ev, lv;
  __device__ __forceinline__ void issue_interior(__amdgpu_buffer_rsrc_t fr, int pofs, int stride, int k, int l,
                                                 bool from_prev) {
    const int lane = threadIdx.x;
#pragma unroll
    for (int r = 0; r < RI; r++) {
      const int q = lane + 64 * r;
      const int row = q / PER, col = 16 * (q - row * PER);
      iv[r] = __builtin_bit_cast(
          uint4, __builtin_amdgcn_raw_buffer_load_b128(fr, pofs + (k * G::SZ + row) * stride + l * G::SZ + col, 0, 0));
    }
    lv = 0;
    if (FULL && !from_prev && lane < G::SZ)
      lv = __builtin_amdgcn_raw_buffer_load_b8(fr, pofs + (k * G::SZ + lane) * stride + l * G::SZ - 1, 0, 0);
  }
  __device__ __forceinline__ void issue_edge(__amdgpu_buffer_rsrc_t eb, int ew, int k, int l) {
    const int lane = threadIdx.x;
    ev = 0;
    if (lane < G::DW)
      ev = __builtin_amdgcn_raw_buffer_load_b32(eb, (k - 1) * ew + EDGE_MARGIN + l * G::SZ - IMG_X0 + 4 * lane, 0, SC1);
  }
  // LDS operations of one wave complete in order: the left column of the
  // SB left behind is read before the new image overwrites it.
  __device__ __forceinline__ void commit(IntraChain &L, bool from_prev) const {
    const int lane = threadIdx.x;
    uint8_t *img = L.img + G::IW + IMG_X0;  // image (0,0)
    const uint8_t keep = (from_prev && lane < G::SZ) ? img[lane * G::IW + G::SZ - 1] : 0;
#pragma unroll
    for (int r = 0; r < RI; r++) {
      const int q = lane + 64 * r;
      const int row = q / PER, col = 16 * (q - row * PER);
      uint32_t *d = (uint32_t *)(img + row * G::IW + col);
      d[0] = iv[r].x;
      d[1] = iv[r].y;
      d[2] = iv[r].z;
      d[3] = iv[r].w;
    }
    if (lane < G::DW) *(uint32_t *)(img - G::IW - IMG_X0 + 4 * lane) = ev;
    if (lane < G::SZ) {
      if (from_prev) img[lane * G::IW - 1] = keep;
      else if (FULL) img[lane * G::IW - 1] = (uint8_t)lv;
    }
  }
};

// The chain leaves SB (k, l): its edge row goes out write-through (sc1) and is
// waited for (nothing else of the wave's is in flight then), then one lane
// publishes "SBs < next are done" (form R1).
template <int C>
__device__ __forceinline__ void publish_sb(IntraChain &L, __amdgpu_buffer_rsrc_t eb, int ew, int k, int l, unsigned *my,
                                           unsigned next) {
  using G = CompGeom<C>;
  const int lane = threadIdx.x;
  const uint8_t *img = L.img + G::IW + IMG_X0;
  if (lane < G::SZ / 4)
    __builtin_amdgcn_raw_buffer_store_b32(*(const uint32_t *)(img + (G::SZ - 1) * G::IW + 4 * lane), eb,
                                          k * ew + EDGE_MARGIN + l * G::SZ + 4 * lane, 0, SC1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_store(my, next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// ... then the whole SB image goes to the frame (plain stores: only later
// launches read it).  Rows / columns past the frame edge land in the slot's
// padding, which k_pad rewrites.
template <int C>
__device__ __forceinline__ void store_sb(const IntraChain &L, __amdgpu_buffer_rsrc_t fr, int pofs, int stride, int k,
                                         int l) {
  using G = CompGeom<C>;
  constexpr int PER = G::SZ / 16, NR = G::SZ * PER;
  const uint8_t *img = L.img + G::IW + IMG_X0;
#pragma unroll
  for (int r = 0; r < NR / 64; r++) {
    const int q = threadIdx.x + 64 * r;
    const int row = q / PER, col = 16 * (q - row * PER);
    const uint32_t *s = (const uint32_t *)(img + row * G::IW + col);
    __builtin_amdgcn_raw_buffer_store_b128(
        __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, make_uint4(s[0], s[1], s[2], s[3])), fr,
        pofs + (k * G::SZ + row) * stride + l * G::SZ + col, 0, 0);
  }
}

// filter_121 of one edge sample over len (:39-48); a, b, c = samples k-1, k, k+1
__device__ __forceinline__ int f121(int k, int len, int a, int b, int c) {
  return k == 0 ? (3 * b + c + 2) >> 2 : (k == len - 1 ? (a + 3 * b + 2) >> 2 : (a + 2 * b + c + 2) >> 2);
}
// planar 5-tap (:190-204); v0..v4 = samples k-2..k+2
__device__ __forceinline__ int p5f(int k, int n, int v0, int v1, int v2, int v3, int v4) {
  if (k == 0) return 5 * v2 + 2 * v3 + v4;
  if (k == 1) return 3 * v1 + 2 * v2 + 2 * v3 + v4;
  if (k == n - 2) return v0 + 2 * v1 + 2 * v2 + 3 * v3;
  if (k == n - 1) return v0 + 2 * v1 + 5 * v2;
  return v0 + 2 * v1 + 2 * v2 + 2 * v3 + v4;
}

// Probe-only phase timers (built with -DINTRA_PROBE_TIMERS by tools/intra_probe.py).
struct ProbeAcc {
  unsigned long long sb, a, c, ntu;
};
#ifdef INTRA_PROBE_TIMERS
#define PROBE_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define PROBE_ADD(field, from) (pa.field += __builtin_amdgcn_s_memtime() - (from))
#else
#define PROBE_T(v)
#define PROBE_ADD(field, from)
#endif

// The neighbour samples of one transform block, read from the SB image with
// make_top_and_left's rules (intra_prediction.c:57-143): 128 outside the
// frame, the last available sample repeated past the up-right / down-left
// availability (toplen / leftlen), indices clamped to the 2n edge.
struct Edges {
  int iw;            // image row bytes of the component
  int tbase, lbase;  // byte offsets in L.img of image row -1 at the TU's x / column -1 at its y
  int cnt;           // 2n
  const TuP *p;
  __device__ __forceinline__ int top(const IntraChain &L, int m) const {
    m = m < 0 ? 0 : (m > cnt - 1 ? cnt - 1 : m);
    m = m < p->toplen ? m : p->toplen - 1;
    const int x = L.img[tbase + m];
    return p->top_none ? 128 : x;
  }
  __device__ __forceinline__ int left(const IntraChain &L, int m) const {
    m = m < 0 ? 0 : (m > cnt - 1 ? cnt - 1 : m);
    m = m < p->leftlen ? m : p->leftlen - 1;
    const int x = L.img[lbase + m * iw];
    return p->left_none ? 128 : x;
  }
  __device__ __forceinline__ int side(const IntraChain &L, bool is_left, int m) const {
    return is_left ? left(L, m) : top(L, m);
  }
};

// Edge arrays of the directional modes in L.flt (one byte per sample):
//   4 / 7 / 8: U[U_OFF+1+k] = left filtered over n, U[U_OFF-1-k] = top
//              filtered over n, U[U_OFF] = the filtered top-left corner;
//   5 / 6:     U[k] = top filtered over 2n;   9: U[k] = left filtered over 2n.
// Planar keeps its 5-tap sums in L.p5 (top at 0, left at 64); H, V and DC
// read the image directly / reduce to one value.
#define U_OFF 64

// Phase A of mode M: the mode's edge array, R samples per lane (2n <= 64R);
// the DC sum of get_dc_pred(xpos!=0 ? left:top, ypos!=0 ? top:left)
// (:145-160, :366) by DPP.  Returns DC.
template <int M, int R>
__device__ __forceinline__ int tu_edges(IntraChain &L, const TuP &p, const Edges &E) {
  const int n = p.n, cnt = 2 * n;
  int dcacc = 0;
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int q = threadIdx.x + 64 * r;
    if (M == 5 || M == 6 || M == 9) {  // one side over 2n (:216-361's pre-filter over 2n)
      const bool lft = M == 9;
      const int a = E.side(L, lft, q - 1), b = E.side(L, lft, q), c = E.side(L, lft, q + 1);
      if (q < cnt) L.flt[q] = (uint8_t)f121(q, cnt, a, b, c);
    } else {  // both sides over n: q < n the top edge, n <= q < 2n the left
      const bool lft = q >= n;
      const int k = lft ? q - n : q;
      if (M == 0) {
        const int xs = p.xnz & 1;
        const int w = lft ? xs + (!p.ynz) : (!xs) + p.ynz;
        const int v = E.side(L, lft, k);
        dcacc += q < cnt ? v * w : 0;
      } else if (M == 1) {
        const int v0 = E.side(L, lft, k - 2), v1 = E.side(L, lft, k - 1), v2 = E.side(L, lft, k);
        const int v3 = E.side(L, lft, k + 1), v4 = E.side(L, lft, k + 2);
        if (q < cnt) L.p5[lft ? 64 + k : k] = (int16_t)p5f(k, n, v0, v1, v2, v3, v4);
      } else {  // 4, 7, 8
        const int a = E.side(L, lft, k - 1), b = E.side(L, lft, k), c = E.side(L, lft, k + 1);
        if (q < cnt) L.flt[lft ? U_OFF + 1 + k : U_OFF - 1 - k] = (uint8_t)f121(k, n, a, b, c);
      }
    }
  }
  return M == 0 ? (wave_sum(dcacc) + n) / (2 * n) : 0;
}

// Prediction of 4 horizontally adjacent pixels (i, j..j+3) of mode M
// (get_intra_prediction, intra_prediction.c:363-388; directional modes
// :216-361 as index pairs into the edge array: value (U[a] + U[b]) >> 1, a == b
// where the mode takes one sample).
template <int M>
__device__ __forceinline__ void pred4(const IntraChain &L, const TuP &p, int iw, const uint8_t *trow,
                                      const uint8_t *lcol, int pTL, int dc, int i, int j, int pv[4]) {
  const uint8_t *U = L.flt;
  if (M == 0) {
#pragma unroll
    for (int e = 0; e < 4; e++) pv[e] = dc;
  } else if (M == 1) {  // planar, C division (:186-214)
    const uint2 t = *(const uint2 *)&L.p5[j];
    const int li = L.p5[64 + i] - pTL + 4;
    pv[0] = clip255((li + (int)(int16_t)(t.x & 0xffff)) / 8);
    pv[1] = clip255((li + (int)(int16_t)(t.x >> 16)) / 8);
    pv[2] = clip255((li + (int)(int16_t)(t.y & 0xffff)) / 8);
    pv[3] = clip255((li + (int)(int16_t)(t.y >> 16)) / 8);
  } else if (M == 2) {  // horizontal: left[i]
    const int x = lcol[i * iw];
    const int v = p.left_none ? 128 : x;
#pragma unroll
    for (int e = 0; e < 4; e++) pv[e] = v;
  } else if (M == 3) {  // vertical: top[j]
    const uint32_t x = *(const uint32_t *)(trow + j);
    const uint32_t w = p.top_none ? 0x80808080u : x;
#pragma unroll
    for (int e = 0; e < 4; e++) pv[e] = (w >> (8 * e)) & 255;
  } else {
#pragma unroll
    for (int e = 0; e < 4; e++) {
      int a, b;
      if (M == 4) {
        a = b = U_OFF + i - j - e;
      } else if (M == 5) {
        a = b = i + j + e + 1;
      } else if (M == 6 || M == 9) {
        const int d = M == 6 ? i + 2 * (j + e) : 2 * i + j + e;
        a = (d + 1) >> 1;
        b = (d >> 1) + 1;
      } else if (M == 7) {
        const int d = i - 2 * (j + e);
        const int t = -d;
        a = d >= 1 ? U_OFF + d - 1 : U_OFF - ((t + 1) >> 1);
        b = d >= 1 ? U_OFF + d - 1 : U_OFF - (t >> 1) - 1;
      } else {  // 8
        const int d = 2 * i - (j + e);
        a = d <= -1 ? U_OFF + d + 1 : U_OFF + ((d + 1) >> 1);
        b = d <= -1 ? U_OFF + d + 1 : U_OFF + (d >> 1) + 1;
      }
      pv[e] = (M == 4 || M == 5) ? (int)U[a] : ((int)U[a] + (int)U[b]) >> 1;
    }
  }
}

// Phase C: 4 horizontally adjacent pixels per lane and step (prediction +
// residual, one dword into the image).
template <int M>
__device__ __forceinline__ void tu_pred(IntraChain &L, const TuP &p, int iw, int sz, const uint8_t *trow,
                                        const uint8_t *lcol, int pTL, int dc) {
  const int n = p.n, lgq = p.lg - 2, ng = (n * n) >> 2;
  uint8_t *img = L.img + iw + IMG_X0;
  for (int g = threadIdx.x; g < ng; g += 64) {
    const int i = g >> lgq, j = (g & ((n >> 2) - 1)) << 2;
    uint2 rw = make_uint2(0, 0);
    if (p.has) rw = *(const uint2 *)&L.res[(p.iy + i) * sz + p.ix + j];
    int pv[4];
    pred4<M>(L, p, iw, trow, lcol, pTL, dc, i, j, pv);
    *(uint32_t *)(img + (p.iy + i) * iw + p.ix + j) = put_byte(clip255(pv[0] + (int)(int16_t)(rw.x & 0xffff)), 0) |
                                                      put_byte(clip255(pv[1] + (int)(int16_t)(rw.x >> 16)), 1) |
                                                      put_byte(clip255(pv[2] + (int)(int16_t)(rw.y & 0xffff)), 2) |
                                                      put_byte(clip255(pv[3] + (int)(int16_t)(rw.y >> 16)), 3);
  }
}

// One transform block of mode M: phase A (the mode's edge array, corner
// terms), phase C (every pixel).  LDS operations of the wave complete in
// order, so the phases only need compiler ordering.
template <int M>
__device__ __forceinline__ void tu_mode(IntraChain &L, const TuP &p, int iw, int sz, ProbeAcc &pa) {
  PROBE_T(ta0);
  const uint8_t *img = L.img + iw + IMG_X0;
  const uint8_t *trow = img + (p.iy - 1) * iw + p.ix, *lcol = img + p.iy * iw + p.ix - 1;
  Edges E;
  E.iw = iw;
  E.tbase = (int)(trow - L.img);
  E.lbase = (int)(lcol - L.img);
  E.cnt = 2 * p.n;
  E.p = &p;
  int dc = 0, pTL = 0;
  if (M != 2 && M != 3) dc = p.n == 64 ? tu_edges<M, 2>(L, p, E) : tu_edges<M, 1>(L, p, E);
  if (M == 1 || M == 4 || M == 7 || M == 8) {  // corner terms (:77-99, :186-189), uniform
    int tl = p.top_none ? 128 : ((p.xnz & 2) ? trow[-1] : trow[0]);
    if (p.top_none) tl = p.left_none ? 128 : lcol[0];  // ypos+i==0: top_left = left[0]
    const int t0 = E.top(L, 0), l0 = E.left(L, 0);
    if (M == 1) pTL = __builtin_amdgcn_readfirstlane(E.left(L, 1) + 2 * l0 + 2 * tl + 2 * t0 + E.top(L, 1));
    else if (threadIdx.x == 0) L.flt[U_OFF] = (uint8_t)((2 * tl + l0 + t0 + 2) >> 2);
  }
  wave_lds_sync();
  PROBE_ADD(a, ta0);
  PROBE_T(tc0);
  tu_pred<M>(L, p, iw, sz, trow, lcol, pTL, dc);
  wave_lds_sync();  // the next TU reads these pixels (and rewrites the edge arrays)
  PROBE_ADD(c, tc0);
  (void)pa;
}

__device__ __forceinline__ void intra_tu(IntraChain &L, const TuP &p, int iw, int sz, ProbeAcc &pa) {
  switch (p.mode) {  // uniform
    case 1: tu_mode<1>(L, p, iw, sz, pa); break;
    case 2: tu_mode<2>(L, p, iw, sz, pa); break;
    case 3: tu_mode<3>(L, p, iw, sz, pa); break;
    case 4: tu_mode<4>(L, p, iw, sz, pa); break;
    case 5: tu_mode<5>(L, p, iw, sz, pa); break;
    case 6: tu_mode<6>(L, p, iw, sz, pa); break;
    case 7: tu_mode<7>(L, p, iw, sz, pa); break;
    case 8: tu_mode<8>(L, p, iw, sz, pa); break;
    case 9: tu_mode<9>(L, p, iw, sz, pa); break;
    default: tu_mode<0>(L, p, iw, sz, pa); break;
  }
}

// What a chain needs to move between SBs (uniform).
struct ChainCtx {
  __amdgpu_buffer_rsrc_t fr, rr, eb;  // current frame slot, residual plane, edge rows
  int pofs, stride, pw, ew, row, nsbw, full, dbg_flags;
  unsigned *my, *ctl;
  const unsigned *above;
};

// The chain enters SB l (component class CH: 0 luma, 1 chroma): flush +
// publish the SB left behind, issue the loads with no dependency (residual,
// FULL interior), store the old image, wait for the row above, then the
// edge row.
template <int CH>
__device__ __forceinline__ void sb_enter(IntraChain &L, const ChainCtx &k, int l, int &cur_sb, int &seen,
                                         unsigned long long &tw) {
  const bool from_prev = cur_sb == l - 1;
  if (cur_sb >= 0) publish_sb<CH>(L, k.eb, k.ew, k.row, cur_sb, k.my, (unsigned)l);
  ResLoad<CH> res;
  res.issue(k.rr, k.pw, k.row, l);
  ImgLoad<CH, true> imf;
  ImgLoad<CH, false> imn;
  if (k.full) imf.issue_interior(k.fr, k.pofs, k.stride, k.row, l, from_prev);
  if (cur_sb >= 0) store_sb<CH>(L, k.fr, k.pofs, k.stride, k.row, cur_sb);
  int need = l + 2 < k.nsbw ? l + 2 : k.nsbw;
  if (k.dbg_flags & 1) need = 0;  // debug: ignore the wavefront dependency (wrong pixels)
  if (seen < need) {
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    int v = (int)__builtin_amdgcn_readfirstlane(ld_progress(k.above));
    unsigned spins = 0;
    while (v < need) {
      __builtin_amdgcn_s_sleep(1);
      v = (int)__builtin_amdgcn_readfirstlane(ld_progress(k.above));
      if (++spins > (1u << 27)) {
        if (threadIdx.x == 0) atomicOr(&k.ctl[1], 1u);
        break;
      }
    }
    seen = v;
    tw += __builtin_amdgcn_s_memtime() - t0;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the sc1 edge loads below the poll
  if (k.full) {
    imf.issue_edge(k.eb, k.ew, k.row, l);
    imf.commit(L, from_prev);
  } else {
    imn.issue_edge(k.eb, k.ew, k.row, l);
    imn.commit(L, from_prev);
  }
  res.commit(L);
  wave_lds_sync();
  cur_sb = l;
}
template <int CH>
__device__ __forceinline__ void sb_leave(IntraChain &L, const ChainCtx &k, int cur_sb) {
  publish_sb<CH>(L, k.eb, k.ew, k.row, cur_sb, k.my, 0x7fffffffu);
  store_sb<CH>(L, k.fr, k.pofs, k.stride, k.row, cur_sb);
}

// One chain: component comp of SB row `row`; its ncu intra CUs' words are
// staged in g_cuw[0 .. ncu).  The transform-block code is shared by the
// three components (one copy in the instruction cache).
__device__ __forceinline__ unsigned long long intra_chain(IntraChain &L, const FrameCtx &f, int comp, int ncu,
                                                          unsigned *ctl, unsigned *progress, int row, int full,
                                                          const int16_t *__restrict__ resid, int dbg_flags,
                                                          ProbeAcc &pa) {
  unsigned long long tw = 0;  // ticks spent waiting on the row above (debug)
  const int ch = comp != 0;
  uint8_t *const plane = comp == 0 ? f.cy : (comp == 1 ? f.cu : f.cv);
  const int pw = f.W >> ch, ph = f.H >> ch;
  const int16_t *rplane = resid + (comp == 0 ? 0 : (long long)f.W * f.H + (comp == 2 ? (long long)pw * ph : 0));
  const uint8_t *slot = f.cy - f.offy;  // the current frame's ring slot
  ChainCtx k;
  k.fr = __builtin_amdgcn_make_buffer_rsrc((void *)slot, 0, (int)f.slot_bytes, 0x00020000);
  k.rr = __builtin_amdgcn_make_buffer_rsrc((void *)rplane, 0, 2 * pw * ph, 0x00020000);
  k.pofs = (int)(plane - slot);
  k.stride = ch ? f.sc : f.sy;
  k.pw = pw;
  k.ew = ch ? f.ewc : f.ewy;
  const uint8_t *ebase =
      f.edge + (comp == 0 ? 0 : (long long)f.nsbrows * f.ewy + (comp == 2 ? (long long)f.nsbrows * f.ewc : 0));
  k.eb = __builtin_amdgcn_make_buffer_rsrc((void *)ebase, 0, f.nsbrows * k.ew, 0x00020000);
  k.row = row;
  k.nsbw = (f.W + 63) >> 6;
  k.full = full;
  k.dbg_flags = dbg_flags;
  k.my = progress + 3 * row + comp;
  k.ctl = ctl;
  k.above = progress + 3 * (row - 1) + comp;
  const int iw = ch ? CompGeom<1>::IW : CompGeom<0>::IW, sz = 64 >> ch;
  int seen = row == f.ir0 ? 0x7fffffff : 0, cur_sb = -2;  // the first row (of the frame / band) waits on nothing
  uint2 wn = ncu > 0 ? g_cuw[0] : make_uint2(0, 0);
  for (int it = 0; it < ncu; it++) {
    const uint32_t w0 = __builtin_amdgcn_readfirstlane(wn.x), w1 = __builtin_amdgcn_readfirstlane(wn.y);
    if (it + 1 < ncu) wn = g_cuw[it + 1];  // next CU's words in flight during this one
    const int y = w0 & 0xffff, x = w0 >> 16, S = w1 & 0xff, mode = (w1 >> 8) & 15, tb = (w1 >> 12) & 1;
    const int cmask = (w1 >> 13) & 7, ur_cb = (w1 >> 16) & 1, dl_cb = (w1 >> 17) & 1;
    const int l = x >> 6;
    if (l != cur_sb) {
      PROBE_T(ts0);
      if (ch) sb_enter<1>(L, k, l, cur_sb, seen, tw);
      else sb_enter<0>(L, k, l, cur_sb, seen, tw);
      PROBE_ADD(sb, ts0);
    }
    const int tbc = ch ? (tb && S > 8) : tb;
    const int nsteps = tbc ? 4 : 1;
    for (int t = 0; t < nsteps; t++)
      intra_tu(L, make_tup(comp, S, tbc, y, x, mode, cmask, t, ur_cb, dl_cb), iw, sz, pa);
#ifdef INTRA_PROBE_TIMERS
    pa.ntu += nsteps;
#endif
  }
  if (cur_sb >= 0) {
    if (ch) sb_leave<1>(L, k, cur_sb);
    else sb_leave<0>(L, k, cur_sb);
  } else if (threadIdx.x == 0) {
    __hip_atomic_store(k.my, 0x7fffffffu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return tw;
}

// Per-frame setup before k_intra: each SB row's segment of the intra list
// (decode order is raster SB order) into rowstart[0..nrows]; progress words
// and the task head cleared.
// Row segments of the intra list (decode order is SB-row major, so each SB
// row's CUs are contiguous): rowstart[r] = first list index in SB row >= r.
// With few intra CUs, element-parallel (every element's row and its
// predecessor's: one round of independent loads); with many, a binary search
// per row (rows in parallel).
__device__ __forceinline__ void intra_setup_body(const thor_block_t *__restrict__ blk,
                                                 const uint32_t *__restrict__ list, int n_intra, unsigned *ctl,
                                                 unsigned *progress, int *rowstart, int nrows) {
  const int t = threadIdx.x, nt = blockDim.x;
  if (n_intra < nt) {  // few intra CUs (P frames): one round of independent loads
    const int i = t;
    if (i <= n_intra) {
      const int ri = i < n_intra ? (blk[list[i]].ypos >> 6) : nrows;  // nrows: sentinel past the last element
      const int rp = i > 0 ? (blk[list[i - 1]].ypos >> 6) : -1;
      for (int r = rp + 1; r <= ri && r <= nrows; r++) rowstart[r] = i;
    }
  } else {  // many (I frames): a binary search per row, rows in parallel
    for (int r = t; r <= nrows; r += nt) {
      int lo = 0, hi = n_intra;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((blk[list[mid]].ypos >> 6) < r) lo = mid + 1;
        else hi = mid;
      }
      rowstart[r] = lo;
    }
  }
  for (int q = t; q < 3 * nrows; q += nt) progress[q] = 0;
  if (t == 0) ctl[0] = 0;
}

// k_frame_prep: everything a frame needs before reconstruction, in one launch
// of 256-lane workgroups: [0, nprep) the per-4x4 side info (prep_body,
// 4 x PREP_CPW CUs per workgroup), [nprep, nprep + nres) the residuals of the coded
// transform blocks (resid_tu, four per workgroup), and one last workgroup that
// sets up the intra chains (row segments of the intra list, progress words).
// All three only read the frame's parse output.
__global__ __launch_bounds__(256) void k_frame_prep(const FrameBatch fb_) {
  const FrameCtx *__restrict__ F = FRAME_BATCH_CTX();
  __shared__ ResidLds RL[4];
  const FrameCtx &f = F[blockIdx.y];
  const int b = blockIdx.x;
  if (f.nblocks <= 0) return;
  if (b < f.nprep) prep_body(b, f);
  else if (b < f.nprep + f.nres) {
    const int w = threadIdx.x >> 6, idx = (b - f.nprep) * 4 + w;
    if (f.ir1 > 0 && idx < f.ntus) {  // band-local intra (row sharding): only the band's rows are reconstructed here
      const thor_tu_t T = f.tus[idx];
      const int y = T.comp ? 2 * T.y : T.y, n = T.comp ? 2 * T.size : T.size;
      if (y + n <= 64 * f.ir0 || y >= 64 * f.ir1) return;
    }
    resid_tu(RL[w], idx, f.tus, f.ntus, f.coeffs, f.resid, f.W, f.H);
  } else if (b == f.nprep + f.nres && f.nintra > 0) {
    intra_setup_body(f.blk, f.ilist, f.nintra, f.ctl, f.progress, f.rowstart, f.nsbrows);
  }
}

__global__ __launch_bounds__(64) void k_intra(const FrameBatch fb_, unsigned long long *dbg, int dbg_flags) {
  const FrameCtx *__restrict__ F = FRAME_BATCH_CTX();
  __shared__ IntraChain L;
  const FrameCtx &f = F[blockIdx.y];
  if (f.nintra <= 0) return;
  if (blockIdx.y) dbg = nullptr;
  const thor_block_t *__restrict__ blk = f.blk;
  const uint32_t *__restrict__ list = f.ilist;
  const int *__restrict__ rowstart = f.rowstart;
  unsigned *ctl = f.ctl, *progress = f.progress;
  const int nrows = f.nsbrows, full_sb = f.full_sb;
  const int16_t *__restrict__ resid = f.resid;
  const int lane = threadIdx.x;
  // SB rows [ir0, ir1): the whole frame, or (band-local intra, row sharding) the
  // band's rows, whose first chain reads the row above from the edge buffer
  // (the rank above hands it over) instead of waiting for it
  const int ir0 = f.ir0, ir1 = f.ir1 > 0 ? f.ir1 : nrows;
  for (;;) {
    const int task = (int)__builtin_amdgcn_readfirstlane(lane == 0 ? atomicAdd(&ctl[0], 1u) : 0u);
    if (task >= 3 * (ir1 - ir0)) return;
    const int row = ir0 + task / 3, c = task - 3 * (row - ir0);
    const int i0 = rowstart[row], ncu = rowstart[row + 1] - i0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    // stage the row's CU words (lane-parallel, four batches of loads in flight)
    for (int b = 0; b < ncu; b += 256) {
      uint32_t id[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int q = b + 64 * u + lane;
        id[u] = q < ncu ? list[i0 + q] : 0u;
      }
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int q = b + 64 * u + lane;
        if (q < ncu) g_cuw[q] = cu_words(blk[id[u]], f.W, f.H);
      }
    }
    wave_lds_sync();
    unsigned long long tw;
    ProbeAcc pa = {0, 0, 0, 0};
    tw = intra_chain(L, f, c, ncu, ctl, progress, row, full_sb, resid, dbg_flags, pa);
    if (dbg && lane == 0) {
      unsigned long long *o = dbg + 16 * task;
      o[0] = t0;
      o[1] = __builtin_amdgcn_s_memtime();
      o[2] = tw;
      o[3] = (unsigned long long)ncu;
      o[4] = pa.sb;
      o[5] = pa.a;
      o[6] = pa.c;
      o[7] = pa.ntu;
    }
    wave_lds_sync();  // the next task restages g_cuw
  }
}
