// Intra reconstruction for gfx950: decode_and_reconstruct_block_intra
// (dec/decode_block.c:48-88) over a frame's intra CUs.
//
// Intra CUs read the pre-deblock reconstruction of their left / top / top-left
// / top-right / bottom-left neighbours (make_top_and_left,
// common/intra_prediction.c:57-143), so they form a dependency chain in
// decode order.  Y, U and V never read each other, so a frame's intra work is
// 3 x (SB rows) independent chains.  Each chain is one 256-lane workgroup: it
// owns one component of one 64x64 SB row and reconstructs that row's intra
// CUs in decode order, one transform block at a time: the lanes build the
// neighbour arrays the mode needs (one edge sample per lane), then predict one
// pixel each (1024 lanes = 16 waves, so LDS latency hides).  The rows of a
// component form a wavefront (WPP pattern): row k may work on SB l once row
// k-1 of the same component has completed SBs 0..l+1 (the top-right neighbour
// is the furthest pixel read, common/common_block.c:110-118; the bottom-left
// is never read across an SB row, :120-129).
//
// Transform blocks reconstruct into the SB's LDS image only.  When a chain
// leaves an SB it stores the SB's bottom pixel row -- the only pixels the
// next chain reads -- to an edge-row buffer, then the whole image to the
// frame.  Hand-off without agent-scope fences (cdna_hip_programming.md
// Guideline 16, form R1): the edge store is write-through (sc1) and waited for
// alone, the workgroup meets at a barrier and one lane publishes the progress
// word with a relaxed agent-scope atomic; the consumer polls that word relaxed
// and reads the edge row with sc1 loads (which bypass its L1), so no acquire
// is needed.  Everything else a chain reads comes from earlier launches
// (residual, k_recon's pixels) and is issued before the poll, so its latency
// hides behind the wait.  Tasks (row,
// component) are dequeued in row order (atomic head): every awaited chain is
// held by a running workgroup, so the grid always drains.
#include "common.h"

#define DESC_WIN 128  // CU descriptors staged in LDS per window load
#define IMG_X0 4      // image column -4 at byte 0: rows are dword aligned
#ifndef INTRA_THREADS
#define INTRA_THREADS 1024
#endif
#define SC1 16        // buffer instruction aux: sc1 (write-through store / L1-bypassing load)

template <int C>
struct CompGeom {
  static constexpr int SZ = C ? 32 : 64;      // SB size in this plane
  static constexpr int IW = SZ + 8;           // image row: cols -4 .. SZ+3
  static constexpr int IH = SZ + 1;           // image rows -1 .. SZ-1
  static constexpr int DW = IW / 4;           // dwords per image row
};

struct IntraChain {
  uint8_t img[65 * 72];          // SB image of this component
  int16_t res[64 * 64];          // k_resid's residual over the SB
  thor_block_t desc[DESC_WIN];   // intra CUs [dbase, dbase + DESC_WIN) of the row
  uint8_t raw[256];              // neighbours of the current TU: top at 0, left at 128 (make_top_and_left)
  uint8_t flt[256];              // 1-2-1 filtered top / left, over n or 2n by mode
  int16_t p5[128];               // planar 5-tap filtered edges: top at 0, left at 64
  int dcsum[2], tlF, pTL;      // DC sums double-buffered by TU parity
  int task, seen;
};

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

// Parameters of one transform block (uniform: scalar registers).
struct TuP {
  int active, n, lg, has, mode;
  int iy, ix;           // TU origin inside the SB image
  int toplen, leftlen, top_none, left_none;
  int xnz, ynz;         // xnz bit0: TU x != 0 (DC selector, :366); bit1: CU x > 0 (top_left, :79/:96)
  long long gofs;       // plane offset of the TU origin
};

// Component C's transform block of TU step t (intra_prediction.c:57-143 +
// dec/decode_block.c:48-88: tb_split gives 4 raster sub-TUs; chroma of an
// 8x8 CU is not split).
template <int C>
__device__ __forceinline__ TuP make_tup(int S, int tb, int y, int x, int mode, int cmask, int t, int ur_cb, int dl_cb,
                                        int stride) {
  TuP p;
  int size = C ? S >> 1 : S;
  int tbc = C ? (tb && S > 8) : tb;
  p.active = t < (tbc ? 4 : 1);
  int n = tbc ? size >> 1 : size;
  int i0_ = tbc ? (t >> 1) * n : 0, j0_ = tbc ? (t & 1) * n : 0;
  int yp = C ? y >> 1 : y, xp = C ? x >> 1 : x;
  constexpr int sbm = CompGeom<C>::SZ - 1;
  p.n = n;
  p.lg = ilog2i(n);
  p.has = (cmask >> C) & 1;
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
  p.gofs = (long long)(yp + i0_) * stride + xp + j0_;
  return p;
}

__device__ __forceinline__ unsigned ld_progress(const unsigned *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Residual of SB (k, l), 4 int16 per item, plain loads (written by k_resid in
// an earlier launch; rows past the plane read as 0).
template <int C>
struct ResLoad {
  static constexpr int SZ = CompGeom<C>::SZ, PER = SZ / 4, NR = SZ * PER;
  static constexpr int RR = (NR + INTRA_THREADS - 1) / INTRA_THREADS;
  uint2 v[RR];
  __device__ __forceinline__ void issue(__amdgpu_buffer_rsrc_t rr, int pw, int k, int l) {
#pragma unroll
    for (int r = 0; r < RR; r++) {
      const int q = threadIdx.x + INTRA_THREADS * r;
      const int row = q / PER, x = l * SZ + 4 * (q - row * PER), y = k * SZ + row;
      v[r] = q < NR ? __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rr, 2 * (y * pw + x), 0, 0))
                    : make_uint2(0, 0);
    }
  }
  __device__ __forceinline__ void commit(IntraChain &L) const {
#pragma unroll
    for (int r = 0; r < RR; r++) {
      const int q = threadIdx.x + INTRA_THREADS * r;
      const int row = q / PER, col = 4 * (q - row * PER);
      if (q < NR) *(uint2 *)&L.res[row * SZ + col] = v[r];
    }
  }
};

// The pixel image of SB (k, l) of component C in LDS: image row -1 (cols
// -4..SZ+3) is the edge row of SB row k-1 (written by chain k-1, or by
// k_recon for inter pixels): sc1 loads issued after the poll.  With FULL (P
// frames: k_recon reconstructed the inter CUs) rows 0..SZ-1 come from the
// frame, issued before the poll (nothing this launch writes them).  The left
// column is the previous SB's last image column when the chain just left that
// SB, else the frame's (k_recon's pixels, or outside the frame).  Bytes past
// the frame's right / bottom edge are never used as neighbours
// (availability, common_block.c:100-129).
template <int C, bool FULL>
struct ImgLoad {
  using G = CompGeom<C>;
  static constexpr int NIMG = FULL ? G::SZ * G::DW : 0;
  static constexpr int RI = (NIMG + INTRA_THREADS - 1) / INTRA_THREADS;
  uint32_t iv[RI > 0 ? RI : 1];
  uint32_t ev, lv;
  __device__ __forceinline__ void issue_interior(__amdgpu_buffer_rsrc_t fr, int pofs, int stride, int k, int l,
                                                 bool from_prev) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int r = 0; r < RI; r++) {
      const int q = tid + INTRA_THREADS * r;
      const int row = q / G::DW, col = q - row * G::DW;
      iv[r] = q < NIMG ? __builtin_amdgcn_raw_buffer_load_b32(
                             fr, pofs + (k * G::SZ + row) * stride + l * G::SZ - IMG_X0 + 4 * col, 0, 0)
                       : 0u;
    }
    lv = 0;
    if (!FULL && !from_prev && tid < G::SZ)
      lv = __builtin_amdgcn_raw_buffer_load_b8(fr, pofs + (k * G::SZ + tid) * stride + l * G::SZ - 1, 0, 0);
  }
  __device__ __forceinline__ void issue_edge(__amdgpu_buffer_rsrc_t eb, int ew, int k, int l) {
    const int tid = threadIdx.x;
    ev = 0;
    if (tid < G::DW)
      ev = __builtin_amdgcn_raw_buffer_load_b32(eb, (k - 1) * ew + EDGE_MARGIN + l * G::SZ - IMG_X0 + 4 * tid, 0, SC1);
  }
  __device__ __forceinline__ void commit(IntraChain &L, bool from_prev) const {
    const int tid = threadIdx.x;
    uint8_t *img = L.img + G::IW + IMG_X0;  // image (0,0)
    const uint8_t keep = (from_prev && tid < G::SZ) ? img[tid * G::IW + G::SZ - 1] : 0;
    __syncthreads();  // `keep` read everywhere before the image is overwritten
#pragma unroll
    for (int r = 0; r < RI; r++) {
      const int q = tid + INTRA_THREADS * r;
      const int row = q / G::DW, col = q - row * G::DW;
      if (q < NIMG) *(uint32_t *)(img + row * G::IW - IMG_X0 + 4 * col) = iv[r];
    }
    if (tid < G::DW) *(uint32_t *)(img - G::IW - IMG_X0 + 4 * tid) = ev;
    if (tid < G::SZ) {
      if (from_prev) img[tid * G::IW - 1] = keep;
      else if (!FULL) img[tid * G::IW - 1] = (uint8_t)lv;
    }
  }
};

// The chain leaves SB (k, l): its edge row goes out write-through (sc1) and is
// waited for (nothing else of this wave's is in flight then), the workgroup
// meets, one lane publishes "SBs < next are done" (form R1).
template <int C>
__device__ __forceinline__ void publish_sb(IntraChain &L, __amdgpu_buffer_rsrc_t eb, int ew, int k, int l, unsigned *my,
                                           unsigned next) {
  using G = CompGeom<C>;
  const int tid = threadIdx.x;
  const uint8_t *img = L.img + G::IW + IMG_X0;
  if (tid < G::SZ / 4)
    __builtin_amdgcn_raw_buffer_store_b32(*(const uint32_t *)(img + (G::SZ - 1) * G::IW + 4 * tid), eb,
                                          k * ew + EDGE_MARGIN + l * G::SZ + 4 * tid, 0, SC1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) __hip_atomic_store(my, next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// ... then the whole SB image goes to the frame (plain stores: only later
// launches read it).  Rows / columns past the frame edge land in the slot's
// padding, which k_pad rewrites.
template <int C>
__device__ __forceinline__ void store_sb(const IntraChain &L, __amdgpu_buffer_rsrc_t fr, int pofs, int stride, int k,
                                         int l) {
  using G = CompGeom<C>;
  const int tid = threadIdx.x;
  const uint8_t *img = L.img + G::IW + IMG_X0;
  if (tid >= 256) return;
  if (C == 0) {  // 64 rows x 64 B: 16 B per lane
    const int row = tid >> 2, col = (tid & 3) * 16;
    const uint32_t *q = (const uint32_t *)(img + row * G::IW + col);
    __builtin_amdgcn_raw_buffer_store_b128(
        __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, make_uint4(q[0], q[1], q[2], q[3])), fr,
        pofs + (k * G::SZ + row) * stride + l * G::SZ + col, 0, 0);
  } else {  // 32 rows x 32 B: 4 B per lane
    const int row = tid >> 3, col = (tid & 7) * 4;
    __builtin_amdgcn_raw_buffer_store_b32(*(const uint32_t *)(img + row * G::IW + col), fr,
                                          pofs + (k * G::SZ + row) * stride + l * G::SZ + col, 0, 0);
  }
}

// Neighbours of one transform block inside the SB image, with
// make_top_and_left's rules (intra_prediction.c:57-143): 128 outside the
// frame, the last available sample repeated past the up-right / down-left
// availability (toplen / leftlen), indices clamped to the 2n edge.
template <int C>
struct Nb {
  const uint8_t *trow, *lcol;  // image row -1 at the TU's x, image column -1 at its y
  int cnt, toplen, leftlen, top_none, left_none;
  __device__ __forceinline__ int T(int m) const {
    m = m < 0 ? 0 : (m > cnt - 1 ? cnt - 1 : m);
    return top_none ? 128 : trow[m < toplen ? m : toplen - 1];
  }
  __device__ __forceinline__ int Lf(int m) const {
    m = m < 0 ? 0 : (m > cnt - 1 ? cnt - 1 : m);
    return left_none ? 128 : lcol[(m < leftlen ? m : leftlen - 1) * CompGeom<C>::IW];
  }
};

// filter_121 of one edge sample over len (:39-48); v[] = samples k-1, k, k+1
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

// Pixel (i, j) of mode M from the edge arrays (get_intra_prediction,
// intra_prediction.c:363-388; directional modes :216-361 with their 1-2-1
// pre-filters over n for 4 / 7 / 8 and over 2n for 5 / 6 and 9).
template <int M>
__device__ __forceinline__ int intra_px(const IntraChain &L, int tlF, int pTL, int dc, int i, int j) {
  const uint8_t *ft = L.flt, *fl = L.flt + 128;
  if (M == 1) return clip255((L.p5[64 + i] + L.p5[j] - pTL + 4) / 8);  // planar, C division
  if (M == 2) return L.raw[128 + i];
  if (M == 3) return L.raw[j];
  if (M == 4) {
    const int d = i - j;
    return d > 0 ? fl[d - 1] : (d == 0 ? tlF : ft[-d - 1]);
  }
  if (M == 5) return ft[i + j + 1];
  if (M == 6) {
    const int d = i + 2 * j;
    return (d & 1) ? ft[(d + 1) >> 1] : (ft[d >> 1] + ft[(d >> 1) + 1]) >> 1;
  }
  if (M == 7) {
    const int d = i - 2 * j;
    if (d > 1) return fl[d - 2];
    if (d == 1) return tlF;
    if (d == 0) return (tlF + ft[0]) >> 1;
    const int h = (-d) >> 1;
    return (d & 1) ? ft[h] : (ft[h] + ft[h - 1]) >> 1;
  }
  if (M == 8) {
    const int d = 2 * i - j;
    if (d < -1) return ft[-d - 2];
    if (d == -1) return tlF;
    if (d == 0) return (tlF + fl[0]) >> 1;
    const int h = d >> 1;
    return (d & 1) ? fl[h] : (fl[h] + fl[h - 1]) >> 1;
  }
  if (M == 9) {
    const int d = 2 * i + j;
    return (d & 1) ? fl[(d + 1) >> 1] : (fl[d >> 1] + fl[(d >> 1) + 1]) >> 1;
  }
  return dc;
}

// Phase C: one pixel per lane (4 for 64x64 blocks): prediction + residual.
template <int M, int C>
__device__ __forceinline__ void intra_pred_px(IntraChain &L, const TuP &p, int par) {
  using G = CompGeom<C>;
  uint8_t *img = L.img + G::IW + IMG_X0;
  const int n = p.n;
  const int tlF = L.tlF, pTL = L.pTL, dc = M == 0 ? (L.dcsum[par] + n) / (2 * n) : 0;
  for (int q = threadIdx.x; q < n * n; q += INTRA_THREADS) {
    const int i = q >> p.lg, j = q & (n - 1);
    const int r = p.has ? (int)L.res[(p.iy + i) * G::SZ + p.ix + j] : 0;
    img[(p.iy + i) * G::IW + p.ix + j] = (uint8_t)clip255(intra_px<M>(L, tlF, pTL, dc, i, j) + r);
  }
}

// One transform block: phase A builds the neighbour arrays the mode needs,
// one sample per lane (lanes 0..2n-1 the top edge, 2n..4n-1 the left edge)
// and the DC sum by LDS atomics; phase C predicts every pixel.  Two barriers.
// The SB reaches the frame once, when the chain leaves it.
template <int C>
__device__ __forceinline__ void intra_tu(IntraChain &L, const TuP &p, int par) {
  using G = CompGeom<C>;
  const int tid = threadIdx.x;
  uint8_t *img = L.img + G::IW + IMG_X0;
  Nb<C> b;
  b.trow = img + (p.iy - 1) * G::IW + p.ix;
  b.lcol = img + p.iy * G::IW + p.ix - 1;
  b.cnt = 2 * p.n;
  b.toplen = p.toplen;
  b.leftlen = p.leftlen;
  b.top_none = p.top_none;
  b.left_none = p.left_none;
  const int n = p.n, cnt = 2 * n, mode = p.mode;
#ifndef INTRA_PROBE_SKIP_A
  if (tid < 2 * cnt) {  // ---- phase A: lanes 0..2n-1 the top edge, 2n..4n-1 the left edge, selects only ----
    const int side = tid >= cnt;
    const int k = tid - side * cnt;
    const int len = side ? p.leftlen : p.toplen, none = side ? p.left_none : p.top_none;
    const int step = side ? G::IW : 1;
    const int base = (int)((side ? b.lcol : b.trow) - L.img);
    int v[5];
#pragma unroll
    for (int o = 0; o < 5; o++) {
      int m = k - 2 + o;
      m = m < 0 ? 0 : (m > cnt - 1 ? cnt - 1 : m);
      m = m < len ? m : len - 1;
      const int x = L.img[base + m * step];
      v[o] = none ? 128 : x;
    }
    L.raw[128 * side + k] = (uint8_t)v[2];
    // the one pre-filter this mode reads: 1-2-1 over n (4, 7, 8), over 2n of
    // the top (5, 6) or of the left (9); planar 5-tap; DC sum
    const int flen = (mode == 5 || mode == 6 || mode == 9) ? cnt : n;
    const bool want_f = (mode == 4 || mode == 7 || mode == 8) ? k < n
                        : ((mode == 5 || mode == 6) ? !side : (mode == 9 ? (bool)side : false));
    if (want_f) L.flt[128 * side + k] = (uint8_t)f121(k, flen, v[1], v[2], v[3]);
    if (mode == 1 && k < n) L.p5[64 * side + k] = (int16_t)p5f(k, n, v[0], v[1], v[2], v[3], v[4]);
    if ((mode == 0 || mode > 9) && k < n) {
      // DC sum of get_dc_pred(xpos!=0 ? left:top, ypos!=0 ? top:left), :145-160, :366
      const int xs = p.xnz & 1;
      const int w = side ? xs + (!p.ynz) : (!xs) + p.ynz;
      if (w) atomicAdd(&L.dcsum[par], v[2] * w);
    }
    if (tid == 0) {  // corner terms (:77-99, :186-189)
      int tl = p.top_none ? 128 : ((p.xnz & 2) ? b.trow[-1] : b.trow[0]);
      if (p.top_none) tl = p.left_none ? 128 : b.lcol[0];  // ypos+i==0: top_left = left[0]
      const int t0 = b.T(0), l0 = b.Lf(0);
      L.tlF = (2 * tl + l0 + t0 + 2) >> 2;
      L.pTL = b.Lf(1) + 2 * l0 + 2 * tl + 2 * t0 + b.T(1);
    }
  }
#endif
  __syncthreads();
  if (tid == 0) L.dcsum[par ^ 1] = 0;  // the next TU's sum (last read before this TU's first barrier)
#if defined(INTRA_PROBE_SKIP_C)
  if (0)
#elif defined(INTRA_PROBE_ONE_MODE)
  intra_pred_px<0, C>(L, p, par);
  if (0)
#endif
  switch (mode) {  // uniform
    case 1: intra_pred_px<1, C>(L, p, par); break;
    case 2: intra_pred_px<2, C>(L, p, par); break;
    case 3: intra_pred_px<3, C>(L, p, par); break;
    case 4: intra_pred_px<4, C>(L, p, par); break;
    case 5: intra_pred_px<5, C>(L, p, par); break;
    case 6: intra_pred_px<6, C>(L, p, par); break;
    case 7: intra_pred_px<7, C>(L, p, par); break;
    case 8: intra_pred_px<8, C>(L, p, par); break;
    case 9: intra_pred_px<9, C>(L, p, par); break;
    default: intra_pred_px<0, C>(L, p, par); break;
  }
  __syncthreads();  // the next TU reads these pixels (and rewrites the edge arrays)
}

// One chain: component C of SB row `row`.
template <int C>
__device__ unsigned long long intra_chain(IntraChain &L, const FrameCtx &f, const thor_block_t *__restrict__ blk,
                                          const uint32_t *__restrict__ list, int i0, int i1, unsigned *ctl,
                                          unsigned *progress, int row, int full, const int16_t *__restrict__ resid,
                                          int dbg_flags, bool timed, unsigned long long *tsb) {
  unsigned long long tw = 0;  // ticks spent waiting on the row above (debug)
  unsigned long long t_sb = 0, t_tu = 0, n_sb = 0, n_tu = 0;  // debug: SB transitions / TUs
  const int tid = threadIdx.x;
  uint8_t *const plane = C == 0 ? f.cy : (C == 1 ? f.cu : f.cv);
  const int stride = C ? f.sc : f.sy;
  const int pw = C ? f.W >> 1 : f.W, ph = C ? f.H >> 1 : f.H;
  const int16_t *rplane = resid + (C == 0 ? 0 : (long long)f.W * f.H + (C == 2 ? (long long)pw * ph : 0));
  const uint8_t *slot = f.cy - f.offy;  // the current frame's ring slot
  const __amdgpu_buffer_rsrc_t fr = __builtin_amdgcn_make_buffer_rsrc((void *)slot, 0, (int)f.slot_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc((void *)rplane, 0, 2 * pw * ph, 0x00020000);
  const int pofs = (int)(plane - slot);
  const int ew = C ? f.ewc : f.ewy;
  const uint8_t *ebase = f.edge + (C == 0 ? 0 : (long long)f.nsbrows * f.ewy + (C == 2 ? (long long)f.nsbrows * f.ewc : 0));
  const __amdgpu_buffer_rsrc_t eb = __builtin_amdgcn_make_buffer_rsrc((void *)ebase, 0, f.nsbrows * ew, 0x00020000);
  const int nsbw = (f.W + 63) >> 6;
  unsigned *my = progress + 3 * row + C;
  const unsigned *above = progress + 3 * (row - 1) + C;
  int seen = row == 0 ? 0x7fffffff : 0, cur_sb = -2, ntu = 0;
  int dbase = i0 - DESC_WIN;
  for (int it = i0; it < i1; it++) {
    if (it - dbase >= DESC_WIN) {  // stage the next window of CU descriptors
      dbase = it;
      __syncthreads();
      for (int q = tid; q < DESC_WIN && it + q < i1; q += INTRA_THREADS) L.desc[q] = blk[list[it + q]];
      __syncthreads();
    }
    // descriptor fields are uniform: scalar registers
    const thor_block_t &D = L.desc[it - dbase];
    const int y = __builtin_amdgcn_readfirstlane(D.ypos), x = __builtin_amdgcn_readfirstlane(D.xpos);
    const int S = __builtin_amdgcn_readfirstlane(D.size), tb = __builtin_amdgcn_readfirstlane(D.tb_split) != 0;
    const int mode = __builtin_amdgcn_readfirstlane(D.intra_mode), cmask = __builtin_amdgcn_readfirstlane(D.coeff_mask);
    const int l = x >> 6;
    if (l != cur_sb) {
      const unsigned long long ts0 = timed ? __builtin_amdgcn_s_memtime() : 0;
      // SB transition: loads with no dependency first (residual, FULL interior),
      // flush + publish the SB left behind, wait for the row above, edge row
      const bool from_prev = cur_sb == l - 1;
      if (cur_sb >= 0) publish_sb<C>(L, eb, ew, row, cur_sb, my, (unsigned)l);
      ResLoad<C> res;
      res.issue(rr, pw, row, l);
      ImgLoad<C, true> imf;
      ImgLoad<C, false> imn;
      if (full) imf.issue_interior(fr, pofs, stride, row, l, from_prev);
      else imn.issue_interior(fr, pofs, stride, row, l, from_prev);
      if (cur_sb >= 0) store_sb<C>(L, fr, pofs, stride, row, cur_sb);
      int need = l + 2 < nsbw ? l + 2 : nsbw;
      if (dbg_flags & 1) need = 0;  // debug: ignore the wavefront dependency (wrong pixels)
      if (seen < need) {
        if (tid == 0) {
          const unsigned long long t0 = timed ? __builtin_amdgcn_s_memtime() : 0;
          unsigned v = ld_progress(above);
          unsigned spins = 0;
          while ((int)v < need) {
            __builtin_amdgcn_s_sleep(1);
            v = ld_progress(above);
            if (++spins > (1u << 27)) { atomicOr(&ctl[1], 1u); break; }
          }
          L.seen = (int)v;
          if (timed) tw += __builtin_amdgcn_s_memtime() - t0;
        }
        __syncthreads();
        seen = L.seen;
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the sc1 edge loads below the poll
      if (full) {
        imf.issue_edge(eb, ew, row, l);
        imf.commit(L, from_prev);
      } else {
        imn.issue_edge(eb, ew, row, l);
        imn.commit(L, from_prev);
      }
      res.commit(L);
      __syncthreads();
      cur_sb = l;
      if (timed) { t_sb += __builtin_amdgcn_s_memtime() - ts0; n_sb++; }
    }
    const int ur_cb = upright_available(y, x, S, f.W), dl_cb = downleft_available(y, x, S, f.H);
    const int nsteps = (C == 0 ? tb : (tb && S > 8)) ? 4 : 1;
    const unsigned long long tt0 = timed ? __builtin_amdgcn_s_memtime() : 0;
    for (int t = 0; t < nsteps; t++) {
      const TuP p = make_tup<C>(S, tb, y, x, mode, cmask, t, ur_cb, dl_cb, stride);
      if (dbg_flags & 4) {  // debug: barriers only (measures the TU loop overhead)
        __syncthreads();
        __syncthreads();
      } else {
        intra_tu<C>(L, p, ntu++ & 1);
      }
    }
    if (timed) { t_tu += __builtin_amdgcn_s_memtime() - tt0; n_tu += nsteps; }
  }
  if (cur_sb >= 0) {
    publish_sb<C>(L, eb, ew, row, cur_sb, my, 0x7fffffffu);
    store_sb<C>(L, fr, pofs, stride, row, cur_sb);
  } else if (tid == 0) {
    __hip_atomic_store(my, 0x7fffffffu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (timed && tid == 0) {
    tsb[0] = t_sb; tsb[1] = t_tu; tsb[2] = n_sb; tsb[3] = n_tu;
  }
  return tw;
}

__global__ __launch_bounds__(INTRA_THREADS) void k_intra(FrameCtx f, const thor_block_t *__restrict__ blk,
                                                         const uint32_t *__restrict__ list, int n_intra, unsigned *ctl,
                                                         unsigned *progress, int nrows, unsigned long long *dbg,
                                                         int dbg_flags, int full_sb, const int16_t *__restrict__ resid) {
  __shared__ IntraChain L;
  const int tid = threadIdx.x;
  for (;;) {
    if (tid == 0) {
      L.task = (int)atomicAdd(&ctl[0], 1u);
      L.dcsum[0] = 0;
    }
    __syncthreads();
    const int task = L.task;
    __syncthreads();
    if (task >= 3 * nrows) return;
    const int row = task / 3, c = task - 3 * row;
    // decode order is raster SB order: binary-search this row's segment
    int lo = 0, hi = n_intra;
    while (lo < hi) { int mid = (lo + hi) >> 1; if ((blk[list[mid]].ypos >> 6) < row) lo = mid + 1; else hi = mid; }
    const int i0 = lo;
    hi = n_intra;
    while (lo < hi) { int mid = (lo + hi) >> 1; if ((blk[list[mid]].ypos >> 6) <= row) lo = mid + 1; else hi = mid; }
    const int i1 = lo;
    const unsigned long long t0 = dbg ? __builtin_amdgcn_s_memtime() : 0;
    unsigned long long tw;
    const bool timed = dbg != nullptr;
    if (c == 0) tw = intra_chain<0>(L, f, blk, list, i0, i1, ctl, progress, row, full_sb, resid, dbg_flags, timed,
                                      dbg ? dbg + 16 * task + 4 : nullptr);
    else if (c == 1) tw = intra_chain<1>(L, f, blk, list, i0, i1, ctl, progress, row, full_sb, resid, dbg_flags, timed,
                                      dbg ? dbg + 16 * task + 4 : nullptr);
    else tw = intra_chain<2>(L, f, blk, list, i0, i1, ctl, progress, row, full_sb, resid, dbg_flags, timed,
                                      dbg ? dbg + 16 * task + 4 : nullptr);
    if (dbg && tid == 0) {
      unsigned long long *o = dbg + 16 * task;
      o[0] = t0;
      o[1] = __builtin_amdgcn_s_memtime();
      o[2] = tw;
      o[3] = (unsigned long long)(i1 - i0);
    }
  }
}
