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
  int16_t res[64 * 64];  // k_resid's residual over the SB (16-B aligned rows)
  uint8_t img[65 * 72];  // SB image of this component
  uint8_t raw[256];      // neighbours of the current TU: top at 0, left at 128 (make_top_and_left)
  uint8_t flt[256];      // 1-2-1 filtered top / left, over n or 2n by mode
  int16_t p5[128];       // planar 5-tap filtered edges: top at 0, left at 64
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
template <int C>
__device__ __forceinline__ TuP make_tup(int S, int tbc, int y, int x, int mode, int cmask, int t, int ur_cb, int dl_cb) {
  TuP p;
  const int size = C ? S >> 1 : S;
  const int n = tbc ? size >> 1 : size;
  const int i0_ = tbc ? (t >> 1) * n : 0, j0_ = tbc ? (t & 1) * n : 0;
  const int yp = C ? y >> 1 : y, xp = C ? x >> 1 : x;
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

// Residual of SB (k, l), 8 int16 per item, plain loads (written by k_resid in
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

// Phase C: four horizontally adjacent pixels per lane and step: prediction +
// residual, one dword into the image.
template <int M, int C>
__device__ __forceinline__ void intra_pred(IntraChain &L, const TuP &p, int tlF, int pTL, int dc) {
  using G = CompGeom<C>;
  uint8_t *img = L.img + G::IW + IMG_X0;
  const int n = p.n, lgq = p.lg - 2, ng = (n * n) >> 2;
  for (int g = threadIdx.x; g < ng; g += 64) {
    const int i = g >> lgq, j = (g & ((n >> 2) - 1)) << 2;
    uint2 rw = make_uint2(0, 0);
    if (p.has) rw = *(const uint2 *)&L.res[(p.iy + i) * G::SZ + p.ix + j];
    const int r[4] = {(int)(int16_t)(rw.x & 0xffff), (int)(int16_t)(rw.x >> 16), (int)(int16_t)(rw.y & 0xffff),
                      (int)(int16_t)(rw.y >> 16)};
    uint32_t o = 0;
#pragma unroll
    for (int e = 0; e < 4; e++) o |= put_byte(clip255(intra_px<M>(L, tlF, pTL, dc, i, j + e) + r[e]), e);
    *(uint32_t *)(img + (p.iy + i) * G::IW + p.ix + j) = o;
  }
}

// One transform block.  Phase A builds the neighbour arrays the mode needs,
// one edge sample per lane and step (samples 0..2n-1 the top edge, 2n..4n-1
// the left edge, make_top_and_left's rules: 128 outside the frame, the last
// available sample repeated past the up-right / down-left availability,
// indices clamped to the 2n edge), the corner terms uniformly and the DC sum
// by DPP; phase C predicts every pixel.  The SB reaches the frame once, when
// the chain leaves it.
template <int C>
__device__ __forceinline__ void intra_tu(IntraChain &L, const TuP &p) {
  using G = CompGeom<C>;
  const int lane = threadIdx.x;
  const uint8_t *img = L.img + G::IW + IMG_X0;
  const uint8_t *trow = img + (p.iy - 1) * G::IW + p.ix, *lcol = img + p.iy * G::IW + p.ix - 1;
  const int n = p.n, cnt = 2 * n, mode = p.mode;
  const bool is_dc = mode == 0;
  const int flen = (mode == 5 || mode == 6 || mode == 9) ? cnt : n;
  const int tbase = (int)(trow - L.img), lbase = (int)(lcol - L.img);
  int dcacc = 0;
  for (int q = lane; q < 2 * cnt; q += 64) {
    const int side = q >= cnt;
    const int k = q - side * cnt;
    const int len = side ? p.leftlen : p.toplen, none = side ? p.left_none : p.top_none;
    const int step = side ? G::IW : 1;
    const int base = side ? lbase : tbase;
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
    const bool want_f = (mode == 4 || mode == 7 || mode == 8) ? k < n
                        : ((mode == 5 || mode == 6) ? !side : (mode == 9 ? (bool)side : false));
    if (want_f) L.flt[128 * side + k] = (uint8_t)f121(k, flen, v[1], v[2], v[3]);
    if (mode == 1 && k < n) L.p5[64 * side + k] = (int16_t)p5f(k, n, v[0], v[1], v[2], v[3], v[4]);
    if (is_dc && k < n) {
      // DC sum of get_dc_pred(xpos!=0 ? left:top, ypos!=0 ? top:left), :145-160, :366
      const int xs = p.xnz & 1;
      const int w = side ? xs + (!p.ynz) : (!xs) + p.ynz;
      dcacc += v[2] * w;
    }
  }
  int tlF = 0, pTL = 0, dc = 0;
  if (mode == 1 || mode == 4 || mode == 7 || mode == 8) {  // corner terms (:77-99, :186-189), uniform
    auto T = [&](int m) { return p.top_none ? 128 : (int)trow[m < p.toplen ? m : p.toplen - 1]; };
    auto Lf = [&](int m) { return p.left_none ? 128 : (int)lcol[(m < p.leftlen ? m : p.leftlen - 1) * G::IW]; };
    int tl = p.top_none ? 128 : ((p.xnz & 2) ? trow[-1] : trow[0]);
    if (p.top_none) tl = p.left_none ? 128 : lcol[0];  // ypos+i==0: top_left = left[0]
    const int t0 = T(0), l0 = Lf(0);
    tlF = __builtin_amdgcn_readfirstlane((2 * tl + l0 + t0 + 2) >> 2);
    pTL = __builtin_amdgcn_readfirstlane(Lf(1) + 2 * l0 + 2 * tl + 2 * t0 + T(1));
  }
  if (is_dc) dc = (wave_sum(dcacc) + n) / (2 * n);
  wave_lds_sync();
  switch (mode) {  // uniform
    case 1: intra_pred<1, C>(L, p, tlF, pTL, dc); break;
    case 2: intra_pred<2, C>(L, p, tlF, pTL, dc); break;
    case 3: intra_pred<3, C>(L, p, tlF, pTL, dc); break;
    case 4: intra_pred<4, C>(L, p, tlF, pTL, dc); break;
    case 5: intra_pred<5, C>(L, p, tlF, pTL, dc); break;
    case 6: intra_pred<6, C>(L, p, tlF, pTL, dc); break;
    case 7: intra_pred<7, C>(L, p, tlF, pTL, dc); break;
    case 8: intra_pred<8, C>(L, p, tlF, pTL, dc); break;
    case 9: intra_pred<9, C>(L, p, tlF, pTL, dc); break;
    default: intra_pred<0, C>(L, p, tlF, pTL, dc); break;
  }
  wave_lds_sync();  // the next TU reads these pixels (and rewrites the edge arrays)
}

// One chain: component C of SB row `row`; its ncu intra CUs' words are staged
// in g_cuw[0 .. ncu).
template <int C>
__device__ unsigned long long intra_chain(IntraChain &L, const FrameCtx &f, int ncu, unsigned *ctl, unsigned *progress,
                                          int row, int full, const int16_t *__restrict__ resid, int dbg_flags) {
  unsigned long long tw = 0;  // ticks spent waiting on the row above (debug)
  const int lane = threadIdx.x;
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
  int seen = row == 0 ? 0x7fffffff : 0, cur_sb = -2;
  uint2 wn = ncu > 0 ? g_cuw[0] : make_uint2(0, 0);
  for (int it = 0; it < ncu; it++) {
    const uint32_t w0 = __builtin_amdgcn_readfirstlane(wn.x), w1 = __builtin_amdgcn_readfirstlane(wn.y);
    if (it + 1 < ncu) wn = g_cuw[it + 1];  // next CU's words in flight during this one
    const int y = w0 & 0xffff, x = w0 >> 16, S = w1 & 0xff, mode = (w1 >> 8) & 15, tb = (w1 >> 12) & 1;
    const int cmask = (w1 >> 13) & 7, ur_cb = (w1 >> 16) & 1, dl_cb = (w1 >> 17) & 1;
    const int l = x >> 6;
    if (l != cur_sb) {
      // SB transition: flush + publish the SB left behind, loads with no
      // dependency (residual, FULL interior), wait for the row above, edge row
      const bool from_prev = cur_sb == l - 1;
      if (cur_sb >= 0) publish_sb<C>(L, eb, ew, row, cur_sb, my, (unsigned)l);
      ResLoad<C> res;
      res.issue(rr, pw, row, l);
      ImgLoad<C, true> imf;
      ImgLoad<C, false> imn;
      if (full) imf.issue_interior(fr, pofs, stride, row, l, from_prev);
      if (cur_sb >= 0) store_sb<C>(L, fr, pofs, stride, row, cur_sb);
      int need = l + 2 < nsbw ? l + 2 : nsbw;
      if (dbg_flags & 1) need = 0;  // debug: ignore the wavefront dependency (wrong pixels)
      if (seen < need) {
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
        int v = (int)__builtin_amdgcn_readfirstlane(ld_progress(above));
        unsigned spins = 0;
        while (v < need) {
          __builtin_amdgcn_s_sleep(1);
          v = (int)__builtin_amdgcn_readfirstlane(ld_progress(above));
          if (++spins > (1u << 27)) {
            if (lane == 0) atomicOr(&ctl[1], 1u);
            break;
          }
        }
        seen = v;
        tw += __builtin_amdgcn_s_memtime() - t0;
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
      wave_lds_sync();
      cur_sb = l;
    }
    const int tbc = C == 0 ? tb : (tb && S > 8);
    const int nsteps = tbc ? 4 : 1;
    for (int t = 0; t < nsteps; t++) intra_tu<C>(L, make_tup<C>(S, tbc, y, x, mode, cmask, t, ur_cb, dl_cb));
  }
  if (cur_sb >= 0) {
    publish_sb<C>(L, eb, ew, row, cur_sb, my, 0x7fffffffu);
    store_sb<C>(L, fr, pofs, stride, row, cur_sb);
  } else if (lane == 0) {
    __hip_atomic_store(my, 0x7fffffffu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return tw;
}

// Per-frame setup before k_intra: each SB row's segment of the intra list
// (decode order is raster SB order) into rowstart[0..nrows]; progress words
// and the task head cleared.
__global__ __launch_bounds__(64) void k_intra_setup(const thor_block_t *__restrict__ blk,
                                                    const uint32_t *__restrict__ list, int n_intra, unsigned *ctl,
                                                    unsigned *progress, int *rowstart, int nrows) {
  for (int r = threadIdx.x; r <= nrows; r += 64) {
    int lo = 0, hi = n_intra;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if ((blk[list[mid]].ypos >> 6) < r) lo = mid + 1;
      else hi = mid;
    }
    rowstart[r] = lo;
  }
  for (int q = threadIdx.x; q < 3 * nrows; q += 64) progress[q] = 0;
  if (threadIdx.x == 0) ctl[0] = 0;
}

__global__ __launch_bounds__(64) void k_intra(FrameCtx f, const thor_block_t *__restrict__ blk,
                                              const uint32_t *__restrict__ list, const int *__restrict__ rowstart,
                                              unsigned *ctl, unsigned *progress, int nrows, unsigned long long *dbg,
                                              int dbg_flags, int full_sb, const int16_t *__restrict__ resid) {
  __shared__ IntraChain L;
  const int lane = threadIdx.x;
  for (;;) {
    const int task = (int)__builtin_amdgcn_readfirstlane(lane == 0 ? atomicAdd(&ctl[0], 1u) : 0u);
    if (task >= 3 * nrows) return;
    const int row = task / 3, c = task - 3 * row;
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
    if (c == 0) tw = intra_chain<0>(L, f, ncu, ctl, progress, row, full_sb, resid, dbg_flags);
    else if (c == 1) tw = intra_chain<1>(L, f, ncu, ctl, progress, row, full_sb, resid, dbg_flags);
    else tw = intra_chain<2>(L, f, ncu, ctl, progress, row, full_sb, resid, dbg_flags);
    if (dbg && lane == 0) {
      unsigned long long *o = dbg + 16 * task;
      o[0] = t0;
      o[1] = __builtin_amdgcn_s_memtime();
      o[2] = tw;
      o[3] = (unsigned long long)ncu;
    }
    wave_lds_sync();  // the next task restages g_cuw
  }
}
