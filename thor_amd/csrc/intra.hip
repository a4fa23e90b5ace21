// Intra reconstruction for gfx950: decode_and_reconstruct_block_intra
// (dec/decode_block.c:48-88) over a frame's intra CUs.
//
// Intra CUs read the pre-deblock reconstruction of their left / top / top-left
// / top-right / bottom-left neighbours (make_top_and_left,
// common/intra_prediction.c:57-143), so they form a dependency chain in
// decode order.  The chain is walked as a wavefront over 64x64 SB rows (the
// WPP pattern): one workgroup owns one SB row and reconstructs that row's
// intra CUs in decode order; row k may work on SB l once row k-1 has
// completed SBs 0..l+1 (the top-right neighbour is the furthest pixel read,
// common/common_block.c:110-118; the bottom-left is never read across an SB
// row, :120-129).  Row progress is published with an agent-scope release and
// read with one relaxed poll + one agent-scope acquire per SB, never per CU.
//
// Inside a row the workgroup keeps the SB being reconstructed in LDS as a
// padded image (the SB plus its left column and the row above), so every
// neighbour read after the SB is loaded is an LDS read, global stores are
// fire-and-forget, and the per-TU barriers wait on LDS only.  Rows are
// dequeued in order (atomic head): every awaited row is held by a running
// workgroup, so the grid always drains.
#include "common.h"

#define SBY_W 68  // luma SB image: rows -1..63, cols -1..64 (+pad), stride 68
#define SBY_H 65
#define SBC_W 36  // chroma: rows -1..31, cols -1..32 (+pad)
#define SBC_H 33

struct IntraLds {
  uint8_t img[SBY_H * SBY_W + 2 * SBC_H * SBC_W + 16];
  uint8_t top[136], left[136], tF[136], lF[136];
  int pT[64], pL[64];
  int8_t M[32 * 32];
  int16_t D[3][4 * 256];  // dequantised coefficients of the CU, per component (compact slots)
  int16_t T[16][64];      // inverse transform pass 1
  int tl, tlF, pTL, dc;
  int row, i0, i1, seen, pub, cur_sb;
};

__device__ __forceinline__ uint8_t *sb_img(IntraLds &L, int comp) {
  return comp == 0 ? L.img : L.img + SBY_H * SBY_W + (comp - 1) * SBC_H * SBC_W;
}

// Barrier for LDS traffic only: global stores stay in flight.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

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

__device__ __forceinline__ int f121(const uint8_t *a, int k, int len) {  // filter_121, intra_prediction.c:39-48
  if (k == 0) return (3 * a[0] + a[1] + 2) >> 2;
  if (k == len - 1) return (a[len - 2] + 3 * a[len - 1] + 2) >> 2;
  return (a[k - 1] + 2 * a[k] + a[k + 1] + 2) >> 2;
}

// One transform block.  (ypos, xpos): CU origin in plane coordinates;
// (sy0, sx0): CU origin inside the SB image; (i0, j0): TU offset in the CU.
// All 256 threads call it; three LDS-only barriers.
__device__ void intra_tu(IntraLds &L, int comp, uint8_t *plane, int stride, int mode, int ypos, int xpos, int sy0,
                         int sx0, int size, int i0, int j0, int tb, int ur_cb, int dl_cb, const int16_t *D,
                         int has_coef) {
  int tid = threadIdx.x;
  int n = tb ? size >> 1 : size;
  int len = 2 * n;
  int iw = comp ? SBC_W : SBY_W;
  uint8_t *img = sb_img(L, comp) + iw + 1;  // SB (0,0)
  // ---- phase 1: make_top_and_left (intra_prediction.c:57-143) from the SB image ----
  int dl, ur;
  if (!tb) { dl = dl_cb; ur = ur_cb; }
  else {
    dl = (j0 == 0 && (i0 == 0 || dl_cb)) ? 1 : 0;
    ur = (j0 == 0 || (i0 == 0 && ur_cb)) ? 1 : 0;
  }
  int toplen = ur ? n + 1 : n, leftlen = dl ? n + 1 : n;
  bool top_none = (ypos + i0) == 0, left_none = (xpos + j0) == 0;
  const uint8_t *trow = img + (sy0 + i0 - 1) * iw + sx0 + j0;
  const uint8_t *lcol = img + (sy0 + i0) * iw + sx0 + j0 - 1;
  if (tid < len) {
    int k = tid;
    L.top[k] = top_none ? 128 : trow[k < toplen ? k : toplen - 1];
    L.left[k] = left_none ? 128 : lcol[(k < leftlen ? k : leftlen - 1) * iw];
  }
  if (tid == 255) {
    int tl = top_none ? 128 : (xpos > 0 ? trow[-1] : trow[0]);
    if (top_none) tl = left_none ? 128 : lcol[0];  // ypos+i==0: top_left = left[0]
    L.tl = tl;
  }
  lds_barrier();
  // ---- phase 2: edge filters / DC sum / inverse transform pass 1 ----
  if (mode == 4 || mode == 7 || mode == 8) {
    if (tid < n) {
      L.tF[tid] = (uint8_t)f121(L.top, tid, n);
      L.lF[tid] = (uint8_t)f121(L.left, tid, n);
    }
    if (tid == 64) L.tlF = (2 * L.tl + L.left[0] + L.top[0] + 2) >> 2;
  } else if (mode == 5 || mode == 6) {
    if (tid < 2 * n) L.tF[tid] = (uint8_t)f121(L.top, tid, 2 * n);
  } else if (mode == 9) {
    if (tid < 2 * n) L.lF[tid] = (uint8_t)f121(L.left, tid, 2 * n);
  } else if (mode == 1) {  // planar 5-tap edges (intra_prediction.c:182-214)
    if (tid < 2 * n) {
      const uint8_t *a = tid < n ? L.top : L.left;
      int j = tid < n ? tid : tid - n;
      int v;
      if (j == 0) v = 5 * a[0] + 2 * a[1] + a[2];
      else if (j == 1) v = 3 * a[0] + 2 * a[1] + 2 * a[2] + a[3];
      else if (j == n - 2) v = a[n - 4] + 2 * a[n - 3] + 2 * a[n - 2] + 3 * a[n - 1];
      else if (j == n - 1) v = a[n - 3] + 2 * a[n - 2] + 5 * a[n - 1];
      else v = a[j - 2] + 2 * a[j - 1] + 2 * a[j] + 2 * a[j + 1] + a[j + 2];
      if (tid < n) L.pT[j] = v;
      else L.pL[j] = v;
    }
    if (tid == 255) L.pTL = L.left[1] + 2 * L.left[0] + 2 * L.tl + 2 * L.top[0] + L.top[1];
  } else if (mode == 0 || mode > 9) {
    // DC: get_dc_pred(xpos!=0 ? left:top, ypos!=0 ? top:left), :145-160, :366
    if (tid < 64) {
      const uint8_t *a = (xpos + j0) != 0 ? L.left : L.top;
      const uint8_t *c = (ypos + i0) != 0 ? L.top : L.left;
      int s = tid < n ? a[tid] + c[tid] : 0;
      for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
      if (tid == 0) L.dc = (s + n) / (2 * n);
    }
  }
  int q = n < 16 ? n : 16;
  int nt = n == 64 ? 32 : n, rep = n == 64;
  if (has_coef) {
    int step = 32 / nt;
    for (int it = tid; it < q * nt; it += 256) {
      int k = it / nt, yp = it - k * nt;
      int s = 0;
      for (int m = 0; m < q; m++) s += (int)L.M[(m * step) * 32 + yp] * (int)D[m * q + k];
      L.T[k][yp] = (int16_t)clip16((s + 64) >> 7);
    }
  }
  lds_barrier();
  // ---- phase 3: prediction + residual + reconstruction ----
  uint8_t *dst = plane + (long long)(ypos + i0) * stride + xpos + j0;
  uint8_t *idst = img + (sy0 + i0) * iw + sx0 + j0;
  int step = 32 / nt;
  int lg = ilog2i(n);
  for (int p = tid; p < n * n; p += 256) {
    int i = p >> lg, j = p & (n - 1);
    int v;
    switch (mode) {
      case 1: v = clip255((L.pL[i] + L.pT[j] - L.pTL + 4) / 8); break;
      case 2: v = L.left[i]; break;
      case 3: v = L.top[j]; break;
      case 4: { int d = i - j; v = d > 0 ? L.lF[d - 1] : (d == 0 ? L.tlF : L.tF[-d - 1]); } break;
      case 5: v = L.tF[i + j + 1]; break;
      case 6: { int d = i + 2 * j; v = (d & 1) ? L.tF[(d + 1) / 2] : (L.tF[d / 2] + L.tF[d / 2 + 1]) >> 1; } break;
      case 7: {
        int d = i - 2 * j;
        if (d > 1) v = L.lF[d - 2];
        else if (d == 1) v = L.tlF;
        else if (d == 0) v = (L.tlF + L.tF[0]) >> 1;
        else if (d & 1) v = L.tF[(-d) / 2];
        else v = (L.tF[(-d) / 2] + L.tF[(-d) / 2 - 1]) >> 1;
      } break;
      case 8: {
        int d = 2 * i - j;
        if (d < -1) v = L.tF[-d - 2];
        else if (d == -1) v = L.tlF;
        else if (d == 0) v = (L.tlF + L.lF[0]) >> 1;
        else if (d & 1) v = L.lF[d / 2];
        else v = (L.lF[d / 2] + L.lF[d / 2 - 1]) >> 1;
      } break;
      case 9: { int d = 2 * i + j; v = (d & 1) ? L.lF[(d + 1) / 2] : (L.lF[d / 2] + L.lF[d / 2 + 1]) >> 1; } break;
      default: v = L.dc; break;
    }
    if (has_coef) {
      int xp = j >> rep, yp = i >> rep;
      int s = 0;
      for (int k = 0; k < q; k++) s += (int)L.M[(k * step) * 32 + xp] * (int)L.T[k][yp];
      v = clip255(clip16((s + 2048) >> 12) + v);
    }
    idst[i * iw + j] = (uint8_t)v;
    dst[(long long)i * stride + j] = (uint8_t)v;
  }
  lds_barrier();  // the next TU (tb-split raster order) / next CU reads these pixels from LDS
}

__device__ __forceinline__ unsigned ld_progress(const unsigned *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Caller: every storing wave has passed a full __syncthreads() (vmcnt drained).
__device__ __forceinline__ void publish_progress(unsigned *p, unsigned v) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Load SB (k, l) with its left column and the row above (cols -1..64) from
// the frame into the LDS image.
__device__ void load_sb_image(IntraLds &L, const FrameCtx &f, int k, int l) {
  int tid = threadIdx.x;
  for (int comp = 0; comp < 3; comp++) {
    int sz = comp ? 32 : 64, iw = comp ? SBC_W : SBY_W;
    int W = comp ? f.W >> 1 : f.W, H = comp ? f.H >> 1 : f.H;
    int stride = comp ? f.sc : f.sy;
    const uint8_t *pl = comp == 0 ? f.cy : (comp == 1 ? f.cu : f.cv);
    int y0 = k * sz, x0 = l * sz;
    uint8_t *img = sb_img(L, comp);
    int cols = sz + 2;
    for (int p = tid; p < (sz + 1) * cols; p += 256) {
      int r = p / cols, c = p - r * cols;  // image row r = frame row y0-1+r
      int y = y0 - 1 + r, x = x0 - 1 + c;
      uint8_t v = 0;
      if (y >= 0 && y < H && x >= 0 && x < W + 64) v = pl[(long long)y * stride + x];  // padded slot: x<W+pad ok
      img[r * iw + c] = v;
    }
  }
}

__global__ __launch_bounds__(256) void k_intra(FrameCtx f, const thor_block_t *__restrict__ blk,
                                               const int16_t *__restrict__ coeffs, const uint32_t *__restrict__ list,
                                               int n_intra, unsigned *ctl, unsigned *progress, int nrows) {
  __shared__ IntraLds L;
  int tid = threadIdx.x;
  for (int i = tid; i < 1024; i += 256) L.M[i] = (int8_t)dct32_entry(i >> 5, i & 31);
  int nsbw = (f.W + 63) >> 6;
  for (;;) {
    __syncthreads();
    if (tid == 0) {
      int row = (int)atomicAdd(&ctl[0], 1u);
      L.row = row;
      if (row < nrows) {
        // decode order is raster SB order: binary-search this row's segment
        int lo = 0, hi = n_intra;
        while (lo < hi) { int mid = (lo + hi) >> 1; if ((blk[list[mid]].ypos >> 6) < row) lo = mid + 1; else hi = mid; }
        L.i0 = lo;
        hi = n_intra;
        while (lo < hi) { int mid = (lo + hi) >> 1; if ((blk[list[mid]].ypos >> 6) <= row) lo = mid + 1; else hi = mid; }
        L.i1 = lo;
        L.seen = row == 0 ? 0x7fffffff : 0;
        L.pub = 0;
        L.cur_sb = -1;
      }
    }
    __syncthreads();
    int row = L.row;
    if (row >= nrows) return;
    int i0 = L.i0, i1 = L.i1;
    for (int it = i0; it < i1; it++) {
      int b = (int)list[it];
      thor_block_t B = blk[b];
      int S = B.size, x = B.xpos, y = B.ypos;
      int l = x >> 6;
      if (l != L.cur_sb) {
        // SB transition: drain this workgroup's stores, publish, acquire above row, load the new SB image
        __syncthreads();
        if (tid == 0) {
          if (l > L.pub) {  // every SB of this row left of l is complete
            publish_progress(&progress[row], (unsigned)l);
            L.pub = l;
          }
          int need = l + 2 < nsbw ? l + 2 : nsbw;
          if (L.seen < need) {
            unsigned v = ld_progress(&progress[row - 1]);
            unsigned spins = 0;
            while ((int)v < need) {
              __builtin_amdgcn_s_sleep(1);
              v = ld_progress(&progress[row - 1]);
              if (++spins > (1u << 27)) { atomicOr(&ctl[1], 1u); break; }
            }
            L.seen = (int)v;
          }
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          L.cur_sb = l;
        }
        __syncthreads();
        load_sb_image(L, f, row, l);
        __syncthreads();
      }
      // stage this CU's dequantised coefficients (dequantize, common/common_block.c:132-146)
      int tb = B.tb_split != 0;
      for (int comp = 0; comp < 3; comp++) {
        if (!((B.coeff_mask >> comp) & 1)) continue;
        int size = comp ? S >> 1 : S;
        int tbc = comp ? (tb && S > 8) : tb;
        int n = tbc ? size >> 1 : size, q = n < 16 ? n : 16, ntu = tbc ? 4 : 1;
        int qp = comp ? chroma_qp(B.qp) : B.qp;
        int lshift = qp / 6, scale = dequant_scale(qp % 6);
        int rshift = ilog2i(n) - 1, add = 1 << (rshift - 1);
        const int16_t *cp = coeffs + B.coeff_off[comp];
        for (int p = tid; p < ntu * q * q; p += 256)
          L.D[comp][p] = (int16_t)wrap16(((cp[p] * scale) * (1 << lshift) + add) >> rshift);
      }
      lds_barrier();
      int ur = upright_available(y, x, S, f.W), dl = downleft_available(y, x, S, f.H);
      int mode = B.intra_mode;
      for (int comp = 0; comp < 3; comp++) {
        int size = comp ? S >> 1 : S;
        int tbc = comp ? (tb && S > 8) : tb;
        uint8_t *plane = comp == 0 ? f.cy : (comp == 1 ? f.cu : f.cv);
        int stride = comp ? f.sc : f.sy;
        int yp = comp ? y >> 1 : y, xp = comp ? x >> 1 : x;
        int sbm = comp ? 31 : 63;
        int has = (B.coeff_mask >> comp) & 1;
        if (!tbc) {
          intra_tu(L, comp, plane, stride, mode, yp, xp, yp & sbm, xp & sbm, size, 0, 0, 0, ur, dl, L.D[comp], has);
        } else {
          int h = size >> 1, qq = h < 16 ? h : 16;
          for (int t = 0; t < 4; t++)
            intra_tu(L, comp, plane, stride, mode, yp, xp, yp & sbm, xp & sbm, size, (t >> 1) * h, (t & 1) * h, 1, ur,
                     dl, L.D[comp] + t * qq * qq, has);
        }
      }
    }
    __syncthreads();
    if (tid == 0) publish_progress(&progress[row], 0x7fffffffu);
  }
}
