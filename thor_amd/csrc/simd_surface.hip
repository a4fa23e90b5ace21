// The reference's SIMD kernel surface (common/common_kernels.h:31-41,
// enc/enc_kernels.h:32-37), same names and signatures, executed on the GPU.
//
// These per-block entry points exist so the reference Thorenc/Thordec host C
// links this library unchanged in place of common_kernels.c/enc_kernels.c
// (oracle/Makefile: thordec_amd).  Each call stages the block's exact input
// footprint through device memory, runs one small kernel built from the same
// device functions as the batched frame path, and copies the result back.
// They are correct but launch-latency bound (~tens of us per call); the
// batched API (include/thor_amd.h) is the fast path.
#include <mutex>

#include "../../include/thor_kernels.h"

namespace {

struct Staging {
  uint8_t *in = nullptr, *out = nullptr;
  size_t in_cap = 0, out_cap = 0;
  hipStream_t stream = nullptr;
  std::mutex mu;
  bool ensure(size_t in_bytes, size_t out_bytes) {
    if (!stream && hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return false;
    if (in_bytes > in_cap) {
      if (in) (void)hipFree(in);
      in_cap = in_bytes + 4096;
      if (hipMalloc(&in, in_cap) != hipSuccess) return false;
    }
    if (out_bytes > out_cap) {
      if (out) (void)hipFree(out);
      out_cap = out_bytes + 4096;
      if (hipMalloc(&out, out_cap) != hipSuccess) return false;
    }
    return true;
  }
};
Staging g_stage;

[[noreturn]] void die(const char *what) {
  // The reference surface has no error channel (void functions, abort on
  // fatal errors: common/global.h:38-44); a failed GPU call must not return
  // silently wrong pixels.
  fprintf(stderr, "thor_amd: %s failed (no GPU?)\n", what);
  abort();
}
#define SCHK(x) \
  do {          \
    if ((x) != hipSuccess) die(#x); \
  } while (0)

// Window geometry for MC: rows [-3, h+4), columns [-4, w+12) around the
// block origin; only the reference footprint (rows -2..h+2, cols -2..w+2
// luma; -1..h+1, -1..w+1 chroma) is filled from the host.
struct Win {
  int ws, rows;
  long long org;  // offset of (0,0)
};
Win mc_window(int w, int h) {
  Win W;
  W.ws = (w + 16 + 15) & ~15;
  W.rows = h + 7;
  W.org = 3LL * W.ws + 4;
  return W;
}

}  // namespace

__global__ void k_mc_block(int comp, const uint8_t *src, int ss, uint8_t *dst, int ds, int w, int h, int fx,
                           int fy, int bipred) {
  for (int idx = threadIdx.x; idx < ((comp == 0) ? (w * h + 3) / 4 : w * h); idx += blockDim.x) {
    if (comp == 0) {
      int per_row = (w + 3) / 4;
      int r = idx / per_row, c = (idx - r * per_row) * 4;
      uint32_t v = mc_luma4(src + (long long)r * ss + c, ss, fx, fy, bipred);
      for (int j = 0; j < 4 && c + j < w; j++) dst[(long long)r * ds + c + j] = (uint8_t)(v >> (8 * j));
    } else {
      int r = idx / w, c = idx - r * w;
      dst[(long long)r * ds + c] = (uint8_t)mc_chroma1(src + (long long)r * ss + c, ss, fx, fy);
    }
  }
}

static void mc_call(int comp, int width, int height, int xoff, int yoff, unsigned char *qp, int qstride,
                    const unsigned char *ip, int istride, int bipred) {
  std::lock_guard<std::mutex> lk(g_stage.mu);
  Win W = mc_window(width, height);
  int lo = comp == 0 ? 2 : 1, hi = comp == 0 ? 3 : 2;  // footprint margins
  if (!g_stage.ensure((size_t)W.ws * W.rows, (size_t)width * height)) die("staging alloc");
  SCHK(hipMemsetAsync(g_stage.in, 0, (size_t)W.ws * W.rows, g_stage.stream));
  SCHK(hipMemcpy2DAsync(g_stage.in + W.org - lo * W.ws - lo, W.ws, ip - (long long)lo * istride - lo, istride,
                        width + lo + hi, height + lo + hi, hipMemcpyHostToDevice, g_stage.stream));
  k_mc_block<<<1, 256, 0, g_stage.stream>>>(comp, g_stage.in + W.org, W.ws, g_stage.out, width, width, height, xoff,
                                            yoff, bipred);
  SCHK(hipGetLastError());
  SCHK(hipMemcpy2DAsync(qp, qstride, g_stage.out, width, width, height, hipMemcpyDeviceToHost, g_stage.stream));
  SCHK(hipStreamSynchronize(g_stage.stream));
}

extern "C" {

// common/common_kernels.c:762-784 (dispatcher over centre / edge / inner x uni / bi)
void get_inter_prediction_luma_simd(int width, int height, int xoff, int yoff, unsigned char *qp, int qstride,
                                    const unsigned char *ip, int istride, int bipred) {
  mc_call(0, width, height, xoff, yoff, qp, qstride, ip, istride, bipred);
}

// common/common_kernels.c:786-878
void get_inter_prediction_chroma_simd(int width, int height, int xoff, int yoff, unsigned char *qp, int qstride,
                                      const unsigned char *ip, int istride) {
  mc_call(1, width, height, xoff, yoff, qp, qstride, ip, istride, 0);
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Distortion / averaging / CLPF kernels of the surface.  One workgroup of 256
// lanes per call; sums reduce through wave shuffles and LDS.
// ---------------------------------------------------------------------------
enum { D_SAD = 0, D_SSD, D_SADU, D_WIDE, D_HALF, D_QUARTER, D_CLPFDET };

template <int K>
__device__ __forceinline__ void block_reduce(unsigned (&v)[K], unsigned *out) {
  __shared__ unsigned part[4][8];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < K; k++) {
    unsigned s = v[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) part[w][k] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < K; k++) out[k] = part[0][k] + part[1][k] + part[2][k] + part[3][k];
  }
}

// Sum-type distortions over a w x h block.  a/b point at (0,0) of staged
// copies that hold every byte the reference kernel reads.
__global__ __launch_bounds__(256) void k_dist_call(int mode, const uint8_t *a, int as, const uint8_t *b, int bs,
                                                   int w, int h, int px, int py, unsigned *out) {
  if (mode == D_SAD || mode == D_SSD || mode == D_SADU) {
    unsigned s[1] = {0};
    for (int e = threadIdx.x; e < w * h; e += 256) {
      int i = e / w, j = e - i * w;
      if (mode == D_SADU && w > 8) {
        // sad_calc_simd_unaligned's default case (common/common_kernels.c:108-120)
        // advances both pointers by four rows after EVERY 16-column step:
        // logical (i, j) reads row 4*((i/4)*(w/16) + j/16) + i%4, column j.
        i = 4 * ((i >> 2) * (w >> 4) + (j >> 4)) + (i & 3);
      }
      const int d = (int)a[i * as + j] - (int)b[i * bs + j];
      s[0] += mode == D_SSD ? (unsigned)(d * d) : (unsigned)abs(d);
    }
    block_reduce<1>(s, out);
  } else if (mode == D_WIDE) {  // widesad_calc_simd, enc/enc_kernels.c:71-98: x offsets -3,-1,0,1,3
    unsigned s[5] = {0, 0, 0, 0, 0};
    const int off[5] = {-3, -1, 0, 1, 3};
    for (int e = threadIdx.x; e < w * h; e += 256) {
      const int i = e / w, j = e - i * w;
      const int av = a[i * as + j];
#pragma unroll
      for (int k = 0; k < 5; k++) s[k] += (unsigned)abs(av - (int)b[i * bs + j + off[k]]);
    }
    unsigned r[5];
    block_reduce<5>(s, r);
    if (threadIdx.x == 0) {
      const unsigned code[5] = {0, 2, 3, 4, 6};  // (sad << 3) | (offset + 3), minimum wins
      unsigned best = 0xffffffffu;
      for (int k = 0; k < 5; k++) best = min(best, (r[k] << 3) | code[k]);
      out[0] = best >> 3;
      out[1] = (unsigned)((int)(best & 7) - 3);
    }
  } else if (mode == D_HALF) {  // sad_calc_fasthalf, enc/encode_block.c:497-605
    // order: tl tr br bl top right down left
    unsigned s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int e = threadIdx.x; e < w * h; e += 256) {
      const int i = e / w, j = e - i * w;
      const uint8_t *B = b + i * bs;
      const int S = bs;
      const int A = a[i * as + j];
      int t1, t2, t3, t4, t5, t6, t7, t8, ptl, ptr, pbr, pbl;
      t1 = (B[-S + j - 1] + B[-S + j] + 1) >> 1;
      t2 = (B[j - 1] + B[j] + 1) >> 1;
      t1 = (t1 + t2) >> 1;
      t3 = (B[-2 * S + j - 1] + B[S + j - 1] + 1) >> 1;
      t4 = (B[-2 * S + j] + B[S + j] + 1) >> 1;
      t3 = (t3 + t4) >> 1;
      t5 = (B[-S + j - 2] + B[-S + j + 1] + 1) >> 1;
      t6 = (B[j - 2] + B[j + 1] + 1) >> 1;
      t5 = (t5 + t6) >> 1;
      t5 = (t3 + t5) >> 1;
      ptl = (t5 + t1) >> 1;
      s[7] += abs(A - t2);
      t1 = (B[-S + j] + B[-S + j + 1] + 1) >> 1;
      t8 = (B[j] + B[j + 1] + 1) >> 1;
      t1 = (t1 + t8) >> 1;
      t5 = (B[-2 * S + j + 1] + B[S + j + 1] + 1) >> 1;
      t3 = (t4 + t5) >> 1;
      t4 = (B[-S + j - 1] + B[-S + j + 2] + 1) >> 1;
      t7 = (B[j - 1] + B[j + 2] + 1) >> 1;
      t5 = (t7 + t4) >> 1;
      t5 = (t3 + t5) >> 1;
      ptr = (t5 + t1) >> 1;
      s[5] += abs(A - t8);
      t1 = (B[S + j - 1] + B[S + j] + 1) >> 1;
      t3 = (t1 + t2) >> 1;
      t2 = (B[-S + j - 1] + B[2 * S + j - 1] + 1) >> 1;
      t4 = (B[-S + j] + B[2 * S + j] + 1) >> 1;
      t5 = (t4 + t2) >> 1;
      t1 = (B[S + j - 2] + B[S + j + 1] + 1) >> 1;
      t2 = (t6 + t1) >> 1;
      t2 = (t5 + t2) >> 1;
      pbl = (t2 + t3) >> 1;
      t2 = (B[S + j] + B[S + j + 1] + 1) >> 1;
      t3 = (t8 + t2) >> 1;
      t5 = (B[-S + j + 1] + B[2 * S + j + 1] + 1) >> 1;
      t6 = (t4 + t5) >> 1;
      t8 = (B[S + j - 1] + B[S + j + 2] + 1) >> 1;
      t1 = (t7 + t8) >> 1;
      t2 = (t6 + t1) >> 1;
      pbr = (t2 + t3) >> 1;
      s[6] += abs(A - ((B[j] + B[j + S] + 1) >> 1));
      s[4] += abs(A - ((B[j] + B[j - S] + 1) >> 1));
      s[0] += abs(A - ptl);
      s[1] += abs(A - ptr);
      s[2] += abs(A - pbr);
      s[3] += abs(A - pbl);
    }
    unsigned r[8];
    block_reduce<8>(s, r);
    if (threadIdx.x == 0) {  // :578-605, strict-less updates in this order
      unsigned top = r[4];
      int bx = 0, by = -2;
      if (r[6] < top) { by = 2; top = r[6]; }
      if (r[5] < top) { bx = 2; by = 0; top = r[5]; }
      if (r[7] < top) { bx = -2; by = 0; top = r[7]; }
      if (r[0] < top) { bx = -2; by = -2; top = r[0]; }
      if (r[1] < top) { bx = 2; by = -2; top = r[1]; }
      if (r[2] < top) { bx = 2; by = 2; top = r[2]; }
      if (r[3] < top) { bx = -2; by = 2; top = r[3]; }
      out[0] = top;
      out[1] = (unsigned)bx;
      out[2] = (unsigned)by;
    }
  } else if (mode == D_QUARTER) {  // sad_calc_fastquarter, enc/encode_block.c:609-735; (px, py) = *x, *y in
    // order: tl top tr left right bl down br
    unsigned s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int e = threadIdx.x; e < w * h; e += 256) {
      const int i = e / w, j = e - i * w;
      const uint8_t *r = b + i * bs;
      const int rs = bs;
      const int O = a[i * as + j];
      int p[8];
      if (px & py) {
        const int A = r[j], D = r[j + 1], E = r[j + rs + 1], F = r[j + rs];
        const int ad = (A + D + 1) >> 1, de = (D + E + 1) >> 1, af = (A + F + 1) >> 1, fe = (F + E + 1) >> 1;
        p[0] = (ad + af) >> 1; p[1] = (de + A) >> 1; p[2] = (ad + de) >> 1; p[3] = (ad + F) >> 1;
        p[4] = (ad + E) >> 1; p[5] = (af + fe) >> 1; p[6] = (de + F) >> 1; p[7] = (de + fe) >> 1;
      } else if (px) {
        const int A = r[j], Bv = r[j - rs], Cv = r[j - rs + 1], D = r[j + 1], E = r[j + rs + 1], F = r[j + rs];
        const int ad = (A + D + 1) >> 1, de = (D + E + 1) >> 1, dc = (D + Cv + 1) >> 1, af = (A + F + 1) >> 1,
                  ab = (A + Bv + 1) >> 1;
        p[0] = (ad + ab) >> 1; p[1] = (dc + A) >> 1; p[2] = (ad + dc) >> 1; p[3] = (ad + A) >> 1;
        p[4] = (ad + D) >> 1; p[5] = (ad + af) >> 1; p[6] = (af + D) >> 1; p[7] = (ad + de) >> 1;
      } else if (py) {
        const int A = r[j], D = r[j + 1], E = r[j + rs + 1], F = r[j + rs], G = r[j + rs - 1], Hh = r[j - 1];
        const int ad = (A + D + 1) >> 1, af = (A + F + 1) >> 1, fe = (F + E + 1) >> 1, ah = (A + Hh + 1) >> 1,
                  gf = (G + F + 1) >> 1;
        p[0] = (ah + af) >> 1; p[1] = (af + A) >> 1; p[2] = (ad + af) >> 1; p[3] = (gf + A) >> 1;
        p[4] = (ad + F) >> 1; p[5] = (af + gf) >> 1; p[6] = (af + F) >> 1; p[7] = (af + fe) >> 1;
      } else {
        const int A = r[j], Bv = r[j - rs], D = r[j + 1], F = r[j + rs], Hh = r[j - 1];
        const int ad = (A + D + 1) >> 1, af = (A + F + 1) >> 1, ah = (A + Hh + 1) >> 1, ab = (A + Bv + 1) >> 1;
        p[0] = (ah + ab) >> 1; p[1] = (ab + A) >> 1; p[2] = (ad + ab) >> 1; p[3] = (ah + A) >> 1;
        p[4] = (ad + A) >> 1; p[5] = (ah + af) >> 1; p[6] = (af + A) >> 1; p[7] = (af + ad) >> 1;
      }
#pragma unroll
      for (int k = 0; k < 8; k++) s[k] += (unsigned)abs(O - p[k]);
    }
    unsigned rr[8];
    block_reduce<8>(s, rr);
    if (threadIdx.x == 0) {  // :704-735
      unsigned top = rr[1];
      int bx = 0, by = -1;
      if (rr[0] < top) { bx = -1; top = rr[0]; }
      if (rr[2] < top) { bx = 1; top = rr[2]; }
      if (rr[3] < top) { bx = -1; by = 0; top = rr[3]; }
      if (rr[4] < top) { bx = 1; by = 0; top = rr[4]; }
      if (rr[5] < top) { bx = -1; by = 1; top = rr[5]; }
      if (rr[6] < top) { bx = 0; by = 1; top = rr[6]; }
      if (rr[7] < top) { bx = 1; by = 1; top = rr[7]; }
      out[0] = top;
      out[1] = (unsigned)bx;
      out[2] = (unsigned)by;
    }
  } else {  // D_CLPFDET: detect_clpf_simd, enc/enc_kernels.c:124-159; a = org, b = rec at (x0, y0)
    // (px, py) = SB-relative flags: bit0 left edge, bit1 right edge, bit2 top edge, bit3 bottom edge
    unsigned s[2] = {0, 0};
    const int e = threadIdx.x;
    if (e < 64) {
      const int y = e >> 3, x = e & 7;
      const int X = b[y * bs + x];
      const int A = (y == 0 && (px & 4)) ? X : b[(y - 1) * bs + x];
      const int Bv = (x == 0 && (px & 1)) ? X : b[y * bs + x - 1];
      const int Cv = (x == 7 && (px & 2)) ? X : b[y * bs + x + 1];
      const int D = (y == 7 && (px & 8)) ? X : b[(y + 1) * bs + x];
      const int delta = ((A > X) + (Bv > X) + (Cv > X) + (D > X) > 2) - ((A < X) + (Bv < X) + (Cv < X) + (D < X) > 2);
      const int O = a[y * as + x];
      const int F = (X + delta) & 255;
      s[0] = (unsigned)((O - X) * (O - X));
      s[1] = (unsigned)((O - F) * (O - F));
    }
    block_reduce<2>(s, out);
  }
}

// block_avg_simd, common/common_kernels.c:34-74: rounding average (a + b + 1) >> 1.
__global__ void k_avg_call(uint8_t *p, const uint8_t *r0, const uint8_t *r1, int w, int h) {
  for (int e = threadIdx.x; e < w * h; e += blockDim.x) p[e] = (uint8_t)((r0[e] + r1[e] + 1) >> 1);
}

// clpf_block4 / clpf_block8, common/common_kernels.c:2277-2356: n x n block at
// `src` (staged with a one-pixel ring), edge flags as in D_CLPFDET.
__global__ void k_clpf_call(const uint8_t *src, int ss, uint8_t *dst, int n, int flags) {
  const int e = threadIdx.x;
  if (e >= n * n) return;
  const int y = e / n, x = e - y * n;
  const int X = src[y * ss + x];
  const int A = (y == 0 && (flags & 4)) ? X : src[(y - 1) * ss + x];
  const int Bv = (x == 0 && (flags & 1)) ? X : src[y * ss + x - 1];
  const int Cv = (x == n - 1 && (flags & 2)) ? X : src[y * ss + x + 1];
  const int D = (y == n - 1 && (flags & 8)) ? X : src[(y + 1) * ss + x];
  const int delta = ((A > X) + (Bv > X) + (Cv > X) + (D > X) > 2) - ((A < X) + (Bv < X) + (Cv < X) + (D < X) > 2);
  dst[e] = (uint8_t)(X + delta);
}

namespace {

// A rectangle [x0, x0+w) x [y0, y0+h) around a host pointer, staged at byte
// `off` of the input staging buffer; returns the device address of (0,0).
struct Rect {
  int x0, y0, w, h;
};
const uint8_t *stage_rect(size_t &off, const uint8_t *host, int stride, Rect r) {
  const int pitch = (r.w + 15) & ~15;
  uint8_t *dev = g_stage.in + off;
  SCHK(hipMemcpy2DAsync(dev, pitch, host + (long long)r.y0 * stride + r.x0, stride, r.w, r.h, hipMemcpyHostToDevice,
                        g_stage.stream));
  off += (size_t)pitch * r.h + 256;
  return dev - (long long)r.y0 * pitch - r.x0;
}
int rect_pitch(Rect r) { return (r.w + 15) & ~15; }
size_t rect_bytes(Rect r) { return (size_t)rect_pitch(r) * r.h + 256; }

// One distortion call: stage a (rect ra) and b (rect rb), run, return out[0..2].
void dist_call(int mode, const uint8_t *a, int as, Rect ra, const uint8_t *b, int bs, Rect rb, int w, int h, int px,
               int py, unsigned out[3]) {
  std::lock_guard<std::mutex> lk(g_stage.mu);
  if (!g_stage.ensure(rect_bytes(ra) + rect_bytes(rb), 64)) die("staging alloc");
  size_t off = 0;
  const uint8_t *da = stage_rect(off, a, as, ra);
  const uint8_t *db = stage_rect(off, b, bs, rb);
  k_dist_call<<<1, 256, 0, g_stage.stream>>>(mode, da, rect_pitch(ra), db, rect_pitch(rb), w, h, px, py,
                                             (unsigned *)g_stage.out);
  SCHK(hipGetLastError());
  SCHK(hipMemcpyAsync(out, g_stage.out, 3 * sizeof(unsigned), hipMemcpyDeviceToHost, g_stage.stream));
  SCHK(hipStreamSynchronize(g_stage.stream));
}

// SIMD-literal edge flags of the CLPF kernels: left/top are SB-relative offsets
// (<= 0), right/bottom = min(frame extent - 1, left/top + SB - 1).
int clpf_flags(int x0, int y0, int width, int height, int sb, int n) {
  const int left = (x0 & ~(sb - 1)) - x0, top = (y0 & ~(sb - 1)) - y0;
  const int right = min(width - 1, left + sb - 1), bottom = min(height - 1, top + sb - 1);
  return (left == 0 ? 1 : 0) | (right == n - 1 ? 2 : 0) | (top == 0 ? 4 : 0) | (bottom == n - 1 ? 8 : 0);
}

void clpf_call(const uint8_t *src, uint8_t *dst, int sstride, int dstride, int x0, int y0, int width, int height,
               int n, int sb) {
  std::lock_guard<std::mutex> lk(g_stage.mu);
  const Rect r = {x0 - 1, y0 - 1, n + 2, n + 2};
  if (!g_stage.ensure(rect_bytes(r), 64)) die("staging alloc");
  const int flags = clpf_flags(x0, y0, width, height, sb, n);
  // the reference reads a neighbour only where the flag does not replace it
  // by the centre; stage the ring anyway but only from rows / columns it may read
  Rect rr = r;
  if (flags & 4) { rr.y0 += 1; rr.h -= 1; }
  if (flags & 8) rr.h -= 1;
  if (flags & 1) { rr.x0 += 1; rr.w -= 1; }
  if (flags & 2) rr.w -= 1;
  size_t off = 0;
  const uint8_t *ds = stage_rect(off, src, sstride, rr);
  k_clpf_call<<<1, 64, 0, g_stage.stream>>>(ds + (long long)y0 * rect_pitch(rr) + x0, rect_pitch(rr), g_stage.out, n,
                                           flags);
  SCHK(hipGetLastError());
  // dst is the SB-local buffer: the block lands at its SB-relative position
  uint8_t *d = dst + (long long)(y0 & (sb - 1)) * dstride + (x0 & (sb - 1));
  SCHK(hipMemcpy2DAsync(d, dstride, g_stage.out, n, n, n, hipMemcpyDeviceToHost, g_stage.stream));
  SCHK(hipStreamSynchronize(g_stage.stream));
}

}  // namespace

extern "C" {

// transform_simd, common/common_kernels.c:2176-2250.  Writes exactly the
// region the reference writes: N x N for N <= 16, the 16 x 16 corner for 32
// and fast 64, the 32 x 32 corner for non-fast 64 (whose rows / columns 16..31
// the reference fills from uninitialised scratch; zeros here).
void transform_simd(const int16_t *block, int16_t *coeff, int size, int fast) {
  if (size != 4 && size != 8 && size != 16 && size != 32 && size != 64) die("transform_simd size");
  std::lock_guard<std::mutex> lk(g_stage.mu);
  const size_t nb = (size_t)size * size * sizeof(int16_t);
  if (!g_stage.ensure(nb, 32 * 32 * sizeof(int16_t))) die("staging alloc");
  SCHK(hipMemcpyAsync(g_stage.in, block, nb, hipMemcpyHostToDevice, g_stage.stream));
  SCHK(hipMemsetAsync(g_stage.out, 0, 32 * 32 * sizeof(int16_t), g_stage.stream));
  k_ftx_call<<<1, 64, 0, g_stage.stream>>>((const int16_t *)g_stage.in, (int16_t *)g_stage.out, size, fast);
  SCHK(hipGetLastError());
  const int q = size < 16 ? size : 16;
  const int wr = (size == 64 && !fast) ? 32 : q;  // written region
  SCHK(hipMemcpy2DAsync(coeff, size * sizeof(int16_t), g_stage.out, q * sizeof(int16_t), q * sizeof(int16_t), q,
                        hipMemcpyDeviceToHost, g_stage.stream));
  SCHK(hipStreamSynchronize(g_stage.stream));
  if (wr > q)
    for (int i = 0; i < wr; i++)
      for (int j = (i < q ? q : 0); j < wr; j++) coeff[i * size + j] = 0;
}

// inverse_transform_simd, common/common_kernels.c:2252-2275
void inverse_transform_simd(const int16_t *coeff, int16_t *block, int size) {
  if (size != 4 && size != 8 && size != 16 && size != 32 && size != 64) die("inverse_transform_simd size");
  std::lock_guard<std::mutex> lk(g_stage.mu);
  const size_t nb = (size_t)size * size * sizeof(int16_t);
  if (!g_stage.ensure(nb, nb)) die("staging alloc");
  const int q = size < 16 ? size : 16;  // the only coefficients the partial butterflies read
  SCHK(hipMemcpy2DAsync(g_stage.in, size * sizeof(int16_t), coeff, size * sizeof(int16_t), q * sizeof(int16_t), q,
                        hipMemcpyHostToDevice, g_stage.stream));
  k_itx_call<<<1, 64, 0, g_stage.stream>>>((const int16_t *)g_stage.in, (int16_t *)g_stage.out, size);
  SCHK(hipGetLastError());
  SCHK(hipMemcpyAsync(block, g_stage.out, nb, hipMemcpyDeviceToHost, g_stage.stream));
  SCHK(hipStreamSynchronize(g_stage.stream));
}

// block_avg_simd, common/common_kernels.c:34-74
void block_avg_simd(uint8_t *p, uint8_t *r0, uint8_t *r1, int sp, int s0, int s1, int width, int height) {
  std::lock_guard<std::mutex> lk(g_stage.mu);
  const size_t nb = (size_t)width * height;
  if (!g_stage.ensure(2 * nb + 256, nb)) die("staging alloc");
  SCHK(hipMemcpy2DAsync(g_stage.in, width, r0, s0, width, height, hipMemcpyHostToDevice, g_stage.stream));
  SCHK(hipMemcpy2DAsync(g_stage.in + nb + 256, width, r1, s1, width, height, hipMemcpyHostToDevice, g_stage.stream));
  k_avg_call<<<1, 256, 0, g_stage.stream>>>(g_stage.out, g_stage.in, g_stage.in + nb + 256, width, height);
  SCHK(hipGetLastError());
  SCHK(hipMemcpy2DAsync(p, sp, g_stage.out, width, width, height, hipMemcpyDeviceToHost, g_stage.stream));
  SCHK(hipStreamSynchronize(g_stage.stream));
}

// sad_calc_simd_unaligned, common/common_kernels.c:76-123 (including the
// default case's row advance per 16-column step)
int sad_calc_simd_unaligned(uint8_t *a, uint8_t *b, int astride, int bstride, int width, int height) {
  const int rows = width > 8 ? height * (width / 16) : height;
  const int cols = width > 8 ? (width / 16) * 16 : width;
  unsigned out[3];
  dist_call(D_SADU, a, astride, Rect{0, 0, cols, rows}, b, bstride, Rect{0, 0, cols, rows}, width, height, 0, 0, out);
  return (int)out[0];
}

// sad_calc_simd, enc/enc_kernels.c:32-69
int sad_calc_simd(uint8_t *a, uint8_t *b, int astride, int bstride, int width, int height) {
  unsigned out[3];
  dist_call(D_SAD, a, astride, Rect{0, 0, width, height}, b, bstride, Rect{0, 0, width, height}, width, height, 0, 0,
            out);
  return (int)out[0];
}

// ssd_calc_simd, enc/enc_kernels.c:100-122 (size x size)
int ssd_calc_simd(uint8_t *a, uint8_t *b, int astride, int bstride, int size) {
  unsigned out[3];
  dist_call(D_SSD, a, astride, Rect{0, 0, size, size}, b, bstride, Rect{0, 0, size, size}, size, size, 0, 0, out);
  return (int)out[0];
}

// widesad_calc_simd, enc/enc_kernels.c:71-98
unsigned int widesad_calc_simd(uint8_t *a, uint8_t *b, int astride, int bstride, int width, int height, int *x) {
  unsigned out[3];
  dist_call(D_WIDE, a, astride, Rect{0, 0, width, height}, b, bstride, Rect{-3, 0, width + 6, height}, width, height,
            0, 0, out);
  *x = (int)out[1];
  return out[0];
}

// sad_calc_fasthalf_simd, enc/enc_kernels.c:162-344 (== sad_calc_fasthalf,
// enc/encode_block.c:497-605); reads b rows -2..h+1, columns -2..w+1
unsigned int sad_calc_fasthalf_simd(const uint8_t *a, const uint8_t *b, int astride, int bstride, int width,
                                    int height, int *x, int *y) {
  unsigned out[3];
  dist_call(D_HALF, a, astride, Rect{0, 0, width, height}, b, bstride, Rect{-2, -2, width + 4, height + 4}, width,
            height, 0, 0, out);
  *x = (int)out[1];
  *y = (int)out[2];
  return out[0];
}

// sad_calc_fastquarter_simd, enc/enc_kernels.c:348-648 (== sad_calc_fastquarter,
// enc/encode_block.c:609-735); reads r rows -1..h, columns -1..w
unsigned int sad_calc_fastquarter_simd(const uint8_t *o, const uint8_t *r, int os, int rs, int width, int height,
                                       int *x, int *y) {
  unsigned out[3];
  dist_call(D_QUARTER, o, os, Rect{0, 0, width, height}, r, rs, Rect{-1, -1, width + 2, height + 2}, width, height,
            *x, *y, out);
  *x = (int)out[1];
  *y = (int)out[2];
  return out[0];
}

// detect_clpf_simd, enc/enc_kernels.c:124-159 (accumulates into *sum0, *sum1)
void detect_clpf_simd(const uint8_t *rec, const uint8_t *org, int x0, int y0, int width, int height, int so,
                      int stride, int *sum0, int *sum1) {
  const int flags = clpf_flags(x0, y0, width, height, 64, 8);
  Rect rr = {-1, -1, 10, 10};  // around the block origin
  if (flags & 4) { rr.y0 += 1; rr.h -= 1; }
  if (flags & 8) rr.h -= 1;
  if (flags & 1) { rr.x0 += 1; rr.w -= 1; }
  if (flags & 2) rr.w -= 1;
  unsigned out[3];
  dist_call(D_CLPFDET, org + (long long)y0 * so + x0, so, Rect{0, 0, 8, 8}, rec + (long long)y0 * stride + x0, stride,
            rr, 8, 8, flags, 0, out);
  *sum0 += (int)out[0];
  *sum1 += (int)out[1];
}

// clpf_block4 / clpf_block8, common/common_kernels.c:2277-2356
void clpf_block4(const uint8_t *src, uint8_t *dst, int sstride, int dstride, int x0, int y0, int width, int height) {
  clpf_call(src, dst, sstride, dstride, x0, y0, width, height, 4, 32);
}
void clpf_block8(const uint8_t *src, uint8_t *dst, int sstride, int dstride, int x0, int y0, int width, int height) {
  clpf_call(src, dst, sstride, dstride, x0, y0, width, height, 8, 64);
}

}  // extern "C"
