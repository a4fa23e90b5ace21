// Intra reconstruction for gfx950: decode_and_reconstruct_block_intra
// (dec/decode_block.c:48-88) over a frame's intra CUs.
//
// Intra CUs read the pre-deblock reconstruction of their left / top / top-left
// / top-right / bottom-left neighbours (make_top_and_left,
// common/intra_prediction.c:57-143), so they form a dependency chain in
// decode order.  Y, U and V never read each other, so a frame's intra work is
// 3 x (SB rows) independent chains.  Each chain is one 256-lane workgroup: it
// owns one component of one 64x64 SB row and reconstructs that row's intra
// CUs in decode order, one transform block at a time: wave 0 gathers the
// neighbours and the edge filters the mode needs (phase A), then all four
// waves predict, add the residual and store (phase C).  The rows of a
// component form a wavefront (WPP pattern): row k may work on SB l once row
// k-1 of the same component has completed SBs 0..l+1 (the top-right neighbour
// is the furthest pixel read, common/common_block.c:110-118; the bottom-left
// is never read across an SB row, :120-129).
//
// Hand-off between chains without agent-scope fences (cdna_hip_programming.md
// Guideline 16, form R1): every frame store of a chain is a write-through
// (sc1) buffer store; at an SB boundary every wave drains (vmcnt(0)), the
// workgroup meets at a barrier and one lane publishes the progress word with a
// relaxed agent-scope atomic; the consumer polls that word relaxed and reads
// every frame byte with sc1 buffer loads (which bypass its L1), so no acquire
// is needed.  The residual (k_resid, an earlier launch) is loaded plainly and
// issued before the poll, so its latency hides behind the wait.  Tasks (row,
// component) are dequeued in row order (atomic head): every awaited chain is
// held by a running workgroup, so the grid always drains.
#include "common.h"

#define DESC_WIN 128  // CU descriptors staged in LDS per window load
#define IMG_X0 4      // image column -4 at byte 0: rows are dword aligned
#define INTRA_THREADS 256
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
  uint8_t top[136], left[136];   // raw neighbours (make_top_and_left)
  uint8_t ft[136], fl[136];      // 1-2-1 filtered top / left (over n or 2n, by mode)
  int16_t p5t[64], p5l[64];      // planar 5-tap filtered edges
  int dc, tlF, pTL;              // phase A results for phase C
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

// Prediction of pixel (i, j) from the per-TU edge arrays phase A prepared:
// the ten modes of intra_prediction.c:145-388 with every filter_121 /
// 5-tap term looked up instead of recomputed.  ft/fl hold filter_121 over n
// (modes 4, 7, 8) or over 2n (modes 5, 6 / 9), as get_intra_prediction
// filters them (:250-388).
__device__ __forceinline__ int intra_px2(const uint8_t *top, const uint8_t *left, const uint8_t *ft,
                                         const uint8_t *fl, const int16_t *p5t, const int16_t *p5l, int tlF,
                                         int pTL, int dc, int mode, int i, int j) {
  switch (mode) {
    case 1: return clip255((p5l[i] + p5t[j] - pTL + 4) / 8);  // planar, C division
    case 2: return left[i];
    case 3: return top[j];
    case 4: {
      int d = i - j;
      return d > 0 ? fl[d - 1] : (d == 0 ? tlF : ft[-d - 1]);
    }
    case 5: return ft[i + j + 1];
    case 6: {
      int d = i + 2 * j;
      return (d & 1) ? ft[(d + 1) >> 1] : (ft[d >> 1] + ft[(d >> 1) + 1]) >> 1;
    }
    case 7: {
      int d = i - 2 * j;
      if (d > 1) return fl[d - 2];
      if (d == 1) return tlF;
      if (d == 0) return (tlF + ft[0]) >> 1;
      int h = (-d) >> 1;
      return (d & 1) ? ft[h] : (ft[h] + ft[h - 1]) >> 1;
    }
    case 8: {
      int d = 2 * i - j;
      if (d < -1) return ft[-d - 2];
      if (d == -1) return tlF;
      if (d == 0) return (tlF + fl[0]) >> 1;
      int h = d >> 1;
      return (d & 1) ? fl[h] : (fl[h] + fl[h - 1]) >> 1;
    }
    case 9: {
      int d = 2 * i + j;
      return (d & 1) ? fl[(d + 1) >> 1] : (fl[d >> 1] + fl[(d >> 1) + 1]) >> 1;
    }
    default: return dc;
  }
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
// Every wave drains its sc1 frame stores, the workgroup meets, one lane
// publishes (form R1: write-through payload stores need no release fence).
__device__ __forceinline__ void publish_progress(unsigned *p, unsigned v) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
      v[r] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rr, 2 * (y * pw + x), 0, 0));
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

// Stage the pixel image of SB (k, l) of component C: the row above (cols
// -4..SZ+3) always from the frame (written by row k-1); with FULL (P frames:
// k_recon reconstructed the inter CUs) the SB interior and its left column
// from the frame too; otherwise (every CU of the row is intra) the left
// column is the previous SB's last image column when that SB was this one's
// left neighbour, else the frame's.  Frame reads may fall in the slot's
// padding (row -1, columns past the right edge, rows past the bottom): those
// bytes are never used as neighbours (availability, common_block.c:100-129).
// Every frame load is sc1 (handed-off bytes, see the header).
template <int C, bool FULL>
__device__ __forceinline__ void load_img(IntraChain &L, __amdgpu_buffer_rsrc_t fr, int pofs, int stride, int k, int l,
                                         bool from_prev) {
  using G = CompGeom<C>;
  const int tid = threadIdx.x;
  uint8_t *img = L.img + G::IW + IMG_X0;  // image (0,0)
  constexpr int NIMG = (FULL ? G::IH : 1) * G::DW;
  constexpr int RI = (NIMG + INTRA_THREADS - 1) / INTRA_THREADS;
  uint32_t iv[RI];
#pragma unroll
  for (int r = 0; r < RI; r++) {
    const int q = tid + INTRA_THREADS * r;
    const int row = q / G::DW, col = q - row * G::DW;
    const int off = pofs + (k * G::SZ - 1 + row) * stride + l * G::SZ - IMG_X0 + 4 * col;
    iv[r] = __builtin_amdgcn_raw_buffer_load_b32(fr, off, 0, SC1);
  }
  uint32_t lv = 0;
  if (!FULL && !from_prev && tid < G::SZ)
    lv = __builtin_amdgcn_raw_buffer_load_b8(fr, pofs + (k * G::SZ + tid) * stride + l * G::SZ - 1, 0, SC1);
  const uint8_t keep = (!FULL && from_prev && tid < G::SZ) ? img[tid * G::IW + G::SZ - 1] : 0;
  __syncthreads();  // `keep` read everywhere before the image is overwritten
#pragma unroll
  for (int r = 0; r < RI; r++) {
    const int q = tid + INTRA_THREADS * r;
    const int row = q / G::DW, col = q - row * G::DW;
    if (q < NIMG) *(uint32_t *)(img + (row - 1) * G::IW - IMG_X0 + 4 * col) = iv[r];
  }
  if (!FULL && tid < G::SZ) img[tid * G::IW - 1] = from_prev ? keep : (uint8_t)lv;
}

// One transform block: wave 0 gathers the neighbours (make_top_and_left,
// intra_prediction.c:57-143) and the edge filters the mode needs (phase A);
// all waves predict, add the residual and store to the LDS image and, sc1,
// to the frame (phase C).
template <int C>
__device__ void intra_tu(IntraChain &L, const TuP &p, __amdgpu_buffer_rsrc_t fr, int pofs, int stride) {
  using G = CompGeom<C>;
  const int tid = threadIdx.x;
  uint8_t *img = L.img + G::IW + IMG_X0;
  const int n = p.n, cnt = 2 * n, mode = p.mode;
  const uint8_t *trow = img + (p.iy - 1) * G::IW + p.ix;
  const uint8_t *lcol = img + p.iy * G::IW + p.ix - 1;
  if (tid < 64) {  // ---- phase A (wave 0) ----
    const bool dcm = mode == 0 || mode > 9;
    int dcpart = 0;
    for (int k = tid; k < cnt; k += 64) {
      int T[5], Lf[5];
#pragma unroll
      for (int o = 0; o < 5; o++) {
        int m = k - 2 + o;
        m = m < 0 ? 0 : (m > cnt - 1 ? cnt - 1 : m);
        T[o] = p.top_none ? 128 : trow[m < p.toplen ? m : p.toplen - 1];
        Lf[o] = p.left_none ? 128 : lcol[(m < p.leftlen ? m : p.leftlen - 1) * G::IW];
      }
      L.top[k] = (uint8_t)T[2];
      L.left[k] = (uint8_t)Lf[2];
      if (mode == 4 || mode == 7 || mode == 8) {  // filter_121 over n (:39-48)
        if (k < n) {
          L.ft[k] = (uint8_t)(k == 0 ? (3 * T[2] + T[3] + 2) >> 2
                                     : (k == n - 1 ? (T[1] + 3 * T[2] + 2) >> 2 : (T[1] + 2 * T[2] + T[3] + 2) >> 2));
          L.fl[k] = (uint8_t)(k == 0 ? (3 * Lf[2] + Lf[3] + 2) >> 2
                                     : (k == n - 1 ? (Lf[1] + 3 * Lf[2] + 2) >> 2 : (Lf[1] + 2 * Lf[2] + Lf[3] + 2) >> 2));
        }
      } else if (mode == 5 || mode == 6) {  // filter_121 of top over 2n
        L.ft[k] = (uint8_t)(k == 0 ? (3 * T[2] + T[3] + 2) >> 2
                                   : (k == cnt - 1 ? (T[1] + 3 * T[2] + 2) >> 2 : (T[1] + 2 * T[2] + T[3] + 2) >> 2));
      } else if (mode == 9) {  // filter_121 of left over 2n
        L.fl[k] = (uint8_t)(k == 0 ? (3 * Lf[2] + Lf[3] + 2) >> 2
                                   : (k == cnt - 1 ? (Lf[1] + 3 * Lf[2] + 2) >> 2 : (Lf[1] + 2 * Lf[2] + Lf[3] + 2) >> 2));
      } else if (mode == 1) {  // planar 5-tap (:190-204)
        if (k < n) {
          int t5, l5;
          if (k == 0) { t5 = 5 * T[2] + 2 * T[3] + T[4]; l5 = 5 * Lf[2] + 2 * Lf[3] + Lf[4]; }
          else if (k == 1) { t5 = 3 * T[1] + 2 * T[2] + 2 * T[3] + T[4]; l5 = 3 * Lf[1] + 2 * Lf[2] + 2 * Lf[3] + Lf[4]; }
          else if (k == n - 2) { t5 = T[0] + 2 * T[1] + 2 * T[2] + 3 * T[3]; l5 = Lf[0] + 2 * Lf[1] + 2 * Lf[2] + 3 * Lf[3]; }
          else if (k == n - 1) { t5 = T[0] + 2 * T[1] + 5 * T[2]; l5 = Lf[0] + 2 * Lf[1] + 5 * Lf[2]; }
          else { t5 = T[0] + 2 * T[1] + 2 * T[2] + 2 * T[3] + T[4]; l5 = Lf[0] + 2 * Lf[1] + 2 * Lf[2] + 2 * Lf[3] + Lf[4]; }
          L.p5t[k] = (int16_t)t5;
          L.p5l[k] = (int16_t)l5;
        }
      } else if (dcm && k < n) {
        // DC sum of get_dc_pred(xpos!=0 ? left:top, ypos!=0 ? top:left), :145-160, :366
        const int xs = p.xnz & 1;
        dcpart += T[2] * ((!xs) + p.ynz) + Lf[2] * (xs + (!p.ynz));
      }
    }
    if (dcm) {  // wave reduction of the DC sum
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) dcpart += __shfl_xor(dcpart, o);
    }
    if (tid == 0) {  // corner terms
      int tl = p.top_none ? 128 : ((p.xnz & 2) ? trow[-1] : trow[0]);
      if (p.top_none) tl = p.left_none ? 128 : lcol[0];  // ypos+i==0: top_left = left[0]
      const int t0 = p.top_none ? 128 : trow[0], t1 = p.top_none ? 128 : trow[1 < p.toplen ? 1 : p.toplen - 1];
      const int l0 = p.left_none ? 128 : lcol[0];
      const int l1 = p.left_none ? 128 : lcol[(1 < p.leftlen ? 1 : p.leftlen - 1) * G::IW];
      L.tlF = (2 * tl + l0 + t0 + 2) >> 2;
      L.pTL = l1 + 2 * l0 + 2 * tl + 2 * t0 + t1;
      L.dc = dcm ? (dcpart + n) / (2 * n) : 0;
    }
  }
  __syncthreads();
  // ---- phase C: 1x4 strips over every lane ----
  const int tlF = L.tlF, pTL = L.pTL, dc = L.dc;
  const int strips = (n * n) >> 2;
  for (int s = tid; s < strips; s += INTRA_THREADS) {
    const int i = (s << 2) >> p.lg, j = (s << 2) & (n - 1);
    uint2 cur = make_uint2(0, 0);
    if (p.has) cur = *(const uint2 *)&L.res[(p.iy + i) * G::SZ + p.ix + j];
    const int rr[4] = {(int)(int16_t)(cur.x & 0xffff), (int)(int16_t)(cur.x >> 16), (int)(int16_t)(cur.y & 0xffff),
                       (int)(int16_t)(cur.y >> 16)};
    uint32_t w = 0;
#pragma unroll
    for (int u = 0; u < 4; u++)
      w |= put_byte(clip255(intra_px2(L.top, L.left, L.ft, L.fl, L.p5t, L.p5l, tlF, pTL, dc, mode, i, j + u) + rr[u]), u);
    *(uint32_t *)(img + (p.iy + i) * G::IW + p.ix + j) = w;
    __builtin_amdgcn_raw_buffer_store_b32(w, fr, pofs + (int)p.gofs + i * stride + j, 0, SC1);
  }
  __syncthreads();  // the next TU reads these pixels (and rewrites the edge arrays)
}

// One chain: component C of SB row `row`.
template <int C>
__device__ unsigned long long intra_chain(IntraChain &L, const FrameCtx &f, const thor_block_t *__restrict__ blk,
                                          const uint32_t *__restrict__ list, int i0, int i1, unsigned *ctl,
                                          unsigned *progress, int row, int full, const int16_t *__restrict__ resid,
                                          int dbg_flags, bool timed) {
  unsigned long long tw = 0;  // ticks spent waiting on the row above (debug)
  const int tid = threadIdx.x;
  uint8_t *const plane = C == 0 ? f.cy : (C == 1 ? f.cu : f.cv);
  const int stride = C ? f.sc : f.sy;
  const int pw = C ? f.W >> 1 : f.W, ph = C ? f.H >> 1 : f.H;
  const int16_t *rplane = resid + (C == 0 ? 0 : (long long)f.W * f.H + (C == 2 ? (long long)pw * ph : 0));
  const uint8_t *slot = f.cy - f.offy;  // the current frame's ring slot
  const __amdgpu_buffer_rsrc_t fr = __builtin_amdgcn_make_buffer_rsrc((void *)slot, 0, (int)f.slot_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc((void *)rplane, 0, 2 * pw * ph, 0x00020000);
  const int pofs = (int)(plane - slot);
  const int nsbw = (f.W + 63) >> 6;
  unsigned *my = progress + 3 * row + C;
  const unsigned *above = progress + 3 * (row - 1) + C;
  int seen = row == 0 ? 0x7fffffff : 0, pub = 0, cur_sb = -2;
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
      // SB transition: publish this chain's progress, issue the residual (no
      // dependency), wait for the row above, stage the image
      if (l > pub) {  // every SB of this row left of l is complete
        publish_progress(my, (unsigned)l);
        pub = l;
      }
      ResLoad<C> res;
      res.issue(rr, pw, row, l);
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
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the sc1 loads below the poll
      const bool from_prev = !full && cur_sb == l - 1;
      if (full) load_img<C, true>(L, fr, pofs, stride, row, l, false);
      else load_img<C, false>(L, fr, pofs, stride, row, l, from_prev);
      res.commit(L);
      __syncthreads();
      cur_sb = l;
    }
    const int ur_cb = upright_available(y, x, S, f.W), dl_cb = downleft_available(y, x, S, f.H);
    const int nsteps = (C == 0 ? tb : (tb && S > 8)) ? 4 : 1;
    for (int t = 0; t < nsteps; t++) {
      const TuP p = make_tup<C>(S, tb, y, x, mode, cmask, t, ur_cb, dl_cb, stride);
      intra_tu<C>(L, p, fr, pofs, stride);
    }
  }
  publish_progress(my, 0x7fffffffu);
  return tw;
}

__global__ __launch_bounds__(INTRA_THREADS) void k_intra(FrameCtx f, const thor_block_t *__restrict__ blk,
                                                         const uint32_t *__restrict__ list, int n_intra, unsigned *ctl,
                                                         unsigned *progress, int nrows, unsigned long long *dbg,
                                                         int dbg_flags, int full_sb, const int16_t *__restrict__ resid) {
  __shared__ IntraChain L;
  const int tid = threadIdx.x;
  for (;;) {
    if (tid == 0) L.task = (int)atomicAdd(&ctl[0], 1u);
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
    if (c == 0) tw = intra_chain<0>(L, f, blk, list, i0, i1, ctl, progress, row, full_sb, resid, dbg_flags, timed);
    else if (c == 1) tw = intra_chain<1>(L, f, blk, list, i0, i1, ctl, progress, row, full_sb, resid, dbg_flags, timed);
    else tw = intra_chain<2>(L, f, blk, list, i0, i1, ctl, progress, row, full_sb, resid, dbg_flags, timed);
    if (dbg && tid == 0) {
      unsigned long long *o = dbg + 4 * task;
      o[0] = t0;
      o[1] = __builtin_amdgcn_s_memtime();
      o[2] = tw;
      o[3] = (unsigned long long)(i1 - i0);
    }
  }
}
