// The reference's block- and frame-level reconstruction entry points
// (include/thor_l2.h; SURVEY.md sec. 8(b) "L2 entry points"), same names and
// signatures, executed on the GPU.  The frame-level deblocking converts the
// caller's deblock_data_t array into the decoder's 16-bit cell words and runs
// the decoder's own deblocking bodies (loopfilter.hip); the block-level calls
// run the device encoder's SPMD primitives (enc_pix.h) in one wave.  Inputs
// are staged through device memory and results copied back, as the SIMD
// surface does (simd_surface.hip: same staging, same abort-on-failure rule).
#include "../../include/thor_l2.h"

namespace {

struct L2Stage {
  std::mutex mu;
  hipStream_t stream = nullptr;
  uint8_t *buf = nullptr;
  size_t cap = 0;
  uint8_t *host = nullptr;  // pinned bounce buffer for strided planes
  size_t hcap = 0;
  bool ensure(size_t bytes, size_t hbytes = 0) {
    if (!stream && hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return false;
    if (bytes > cap) {
      if (buf) (void)hipFree(buf);
      cap = bytes + 65536;
      if (hipMalloc(&buf, cap) != hipSuccess) return false;
    }
    if (hbytes > hcap) {
      if (host) (void)hipHostFree(host);
      hcap = hbytes + 65536;
      if (hipHostMalloc(&host, hcap, 0) != hipSuccess) return false;
    }
    return true;
  }
};
L2Stage g_l2;

[[noreturn]] void l2_die(const char *what) {
  fprintf(stderr, "thor_amd: %s\n", what);
  abort();
}
#define L2CHK(x) \
  do {           \
    if ((x) != hipSuccess) l2_die(#x " failed (no GPU?)"); \
  } while (0)

}  // namespace

// deblock_data_t (44 B) -> the decoder's cell word (common.h CI_*), per the
// decisions deblock_frame_y/uv take from it (common/common_frame.c:107-115,
// :268-276): mode, cbp, NEW_MV_TEST |mv| >= 4, the edge-size halving for
// tb_split / PART_VER / PART_QUAD (vertical) and PART_HOR / PART_QUAD
// (horizontal) when size > 8.
__global__ __launch_bounds__(256) void k_l2_cells(const thor_ref_deblock_data_t *__restrict__ dd, int n,
                                                  uint16_t *__restrict__ cell) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const thor_ref_deblock_data_t D = dd[i];
  const int S = D.size ? D.size : 8;
  const int lsz = ilog2i(S);
  const int split = S > 8;
  const int lqv = lsz - ((D.tb_split || D.pb_part == 2 || D.pb_part == 3) && split ? 1 : 0);
  const int lqh = lsz - ((D.tb_split || D.pb_part == 1 || D.pb_part == 3) && split ? 1 : 0);
  const thor_ref_inter_pred_t &P = D.inter_pred;
  const int big = abs(P.mv0.x) >= 4 || abs(P.mv0.y) >= 4 || abs(P.mv1.x) >= 4 || abs(P.mv1.y) >= 4;
  cell[i] = (uint16_t)((D.mode & 7) | ((D.cbp_y != 0) << 3) | ((D.cbp_u != 0) << 4) | ((D.cbp_v != 0) << 5) |
                       (big << 6) | (lqv << 8) | (lqh << 11) | (((lsz - 3) & 3) << 14));
}

__global__ __launch_bounds__(256) void k_l2_deblock_y(int vertical, uint8_t *Y, int sy, int W, int H,
                                                      const uint16_t *__restrict__ cell, int qp, int nbl) {
  if (vertical) luma_v_items<DB_ITEMS>(blockIdx.x * 256 + (int)threadIdx.x, nbl * 256, Y, sy, W, H, cell, qp);
  else luma_h_items<DB_ITEMS>(blockIdx.x * 256 + (int)threadIdx.x, nbl * 256, Y, sy, W, H, cell, qp);
}
__global__ __launch_bounds__(256) void k_l2_deblock_uv(int vertical, uint8_t *U, uint8_t *V, int sc, int W, int H,
                                                       const uint16_t *__restrict__ cell, int qpc, int n) {
  const int plane = blockIdx.y;
  for (int t = blockIdx.x * 256 + threadIdx.x; t < n; t += gridDim.x * 256) {
    if (vertical) k_deblock_chroma_v_body(t, plane, U, V, sc, W, H, cell, qpc);
    else k_deblock_chroma_h_body(t, plane, U, V, sc, W, H, cell, qpc);
  }
}

// The block-level primitives, one wave each.
__global__ __launch_bounds__(64) void k_l2_dequant(const int16_t *__restrict__ c, int16_t *__restrict__ r, int qp,
                                                   int size) {
  // dequantize, common/common_block.c:132-146 (int16 store truncates)
  const int rshift = ilog2i(size) - 1, add = 1 << (rshift - 1), lshift = qp / 6, scale = dequant_scale(qp % 6);
  for (int e = threadIdx.x; e < size * size; e += 64) r[e] = (int16_t)((((int)c[e] * scale << lshift) + add) >> rshift);
}
__global__ __launch_bounds__(64) void k_l2_recon(const int16_t *__restrict__ b, const uint8_t *__restrict__ p,
                                                 uint8_t *__restrict__ o, int size) {
  // reconstruct_block, common/common_block.c:148-156
  for (int e = threadIdx.x; e < size * size; e += 64) o[e] = (uint8_t)clip255((int)b[e] + (int)p[e]);
}
__global__ __launch_bounds__(64) void k_l2_intra(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, int ypos,
                                                 int xpos, int size, int mode) {
  // get_intra_prediction (common/intra_prediction.c:363-388): in = left[2 size] | top[2 size] | top_left
  __shared__ TeNbr nb;
  __shared__ uint8_t pb[64 * 64];
  for (int k = threadIdx.x; k < 2 * size; k += 64) {
    nb.left[k] = in[k];
    nb.top[k] = in[2 * size + k];
  }
  if (threadIdx.x == 0) nb.tl = in[4 * size];
  te_sync();
  te_intra_pred(nb, ypos, xpos, size, pb, mode, 0);
  for (int e = threadIdx.x; e < size * size; e += 64) out[e] = pb[e];
}
__global__ __launch_bounds__(64) void k_l2_top_left(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, int size,
                                                    int toplen, int leftlen, int top128, int left128, int tl_mode) {
  // make_top_and_left (common/intra_prediction.c:57-143): in = the bytes the
  // reference reads (top run | left run | top-left source); 128 fills and the
  // replication of the last available sample past toplen / leftlen.
  for (int k = threadIdx.x; k < 2 * size; k += 64) {
    out[k] = left128 ? 128 : in[2 * size + 1 + (k < leftlen ? k : leftlen - 1)];
    out[2 * size + k] = top128 ? 128 : in[k < toplen ? k : toplen - 1];
  }
  if (threadIdx.x == 0) {
    int tl;
    if (top128) tl = left128 ? 128 : in[2 * size + 1];  // `if (ypos[+i] == 0) *top_left = left[0]`
    else tl = tl_mode ? in[2 * size] : in[0];           // rec / rblock corner, or top[0] at xpos == 0
    out[4 * size] = (uint8_t)tl;
  }
}
__global__ __launch_bounds__(64) void k_l2_quant(const int16_t *__restrict__ in, int16_t *__restrict__ out, int qp,
                                                 int size, int type, int *cbp_out) {
  // quantize, enc/encode_block.c:75-172 (rdoq 0, RDOQ light): in / out q x q raster
  __shared__ TeTx X;
  te_load_zig();
  const int q = size < 16 ? size : 16;
  for (int e = threadIdx.x; e < q * q; e += 64) X.C[e] = in[e];
  te_sync();
  const int cbp = te_quant(X, qp, size, type);
  for (int e = threadIdx.x; e < q * q; e += 64) out[e] = X.C[e];
  if (threadIdx.x == 0) *cbp_out = cbp;
}

extern "C" {

static void l2_deblock(thor_ref_yuv_frame_t *rec, thor_ref_deblock_data_t *dd, int W, int H, int qp, int chroma) {
  if (!rec || !dd || W <= 0 || H <= 0 || (W & 7) || (H & 7) || qp < 0 || qp > 51) l2_die("deblock: bad arguments");
  std::lock_guard<std::mutex> lk(g_l2.mu);
  const int ncell = (W / 4) * (H / 4);
  const size_t ddb = (size_t)ncell * sizeof(thor_ref_deblock_data_t), cb = ((size_t)ncell * 2 + 255) & ~(size_t)255;
  // planes with the ring-slot geometry the kernels are written for (16-byte rows)
  const int sy = (W + 15) & ~15, sc = (W / 2 + 15) & ~15;
  const size_t yb = (size_t)sy * H, ub = (size_t)sc * (H / 2);
  const size_t pix = chroma ? 2 * ub : yb;
  if (!g_l2.ensure(((ddb + 255) & ~(size_t)255) + cb + pix)) l2_die("deblock: staging alloc failed");
  uint8_t *d_dd = g_l2.buf, *d_cell = d_dd + ((ddb + 255) & ~(size_t)255), *d_pix = d_cell + cb;
  hipStream_t st = g_l2.stream;
  L2CHK(hipMemcpyAsync(d_dd, dd, ddb, hipMemcpyHostToDevice, st));
  k_l2_cells<<<(ncell + 255) / 256, 256, 0, st>>>((const thor_ref_deblock_data_t *)d_dd, ncell, (uint16_t *)d_cell);
  L2CHK(hipGetLastError());
  if (!chroma) {
    L2CHK(hipMemcpy2DAsync(d_pix, sy, rec->y, rec->stride_y, W, H, hipMemcpyHostToDevice, st));
    const int nv = ((W >> 3) - 1) * (H >> 3), nh = (W >> 3) * ((H >> 3) - 1);
    const int bv = (nv + 256 * DB_ITEMS - 1) / (256 * DB_ITEMS), bh = (nh + 256 * DB_ITEMS - 1) / (256 * DB_ITEMS);
    if (bv) k_l2_deblock_y<<<bv, 256, 0, st>>>(1, d_pix, sy, W, H, (const uint16_t *)d_cell, qp, bv);
    if (bh) k_l2_deblock_y<<<bh, 256, 0, st>>>(0, d_pix, sy, W, H, (const uint16_t *)d_cell, qp, bh);
    L2CHK(hipGetLastError());
    L2CHK(hipMemcpy2DAsync(rec->y, rec->stride_y, d_pix, sy, W, H, hipMemcpyDeviceToHost, st));
  } else {
    uint8_t *dU = d_pix, *dV = d_pix + ub;
    L2CHK(hipMemcpy2DAsync(dU, sc, rec->u, rec->stride_c, W / 2, H / 2, hipMemcpyHostToDevice, st));
    L2CHK(hipMemcpy2DAsync(dV, sc, rec->v, rec->stride_c, W / 2, H / 2, hipMemcpyHostToDevice, st));
    const int nv = ((W >> 3) - 1) * (H >> 3), nh = (W >> 3) * ((H >> 3) - 1);
    if (nv) k_l2_deblock_uv<<<dim3((nv + 255) / 256, 2), 256, 0, st>>>(1, dU, dV, sc, W, H, (const uint16_t *)d_cell, qp, nv);
    if (nh) k_l2_deblock_uv<<<dim3((nh + 255) / 256, 2), 256, 0, st>>>(0, dU, dV, sc, W, H, (const uint16_t *)d_cell, qp, nh);
    L2CHK(hipGetLastError());
    L2CHK(hipMemcpy2DAsync(rec->u, rec->stride_c, dU, sc, W / 2, H / 2, hipMemcpyDeviceToHost, st));
    L2CHK(hipMemcpy2DAsync(rec->v, rec->stride_c, dV, sc, W / 2, H / 2, hipMemcpyDeviceToHost, st));
  }
  L2CHK(hipStreamSynchronize(st));
}

// common/common_frame.c:46-241
void deblock_frame_y(thor_ref_yuv_frame_t *rec, thor_ref_deblock_data_t *deblock_data, int width, int height,
                     uint8_t qp) {
  l2_deblock(rec, deblock_data, width, height, qp, 0);
}
// common/common_frame.c:243-321
void deblock_frame_uv(thor_ref_yuv_frame_t *rec, thor_ref_deblock_data_t *deblock_data, int width, int height,
                      uint8_t qp) {
  l2_deblock(rec, deblock_data, width, height, qp, 1);
}

// common/common_block.c:132-146
void dequantize(int16_t *coeff, int16_t *rcoeff, int quant, int size) {
  if (size < 4 || size > 64 || (size & (size - 1)) || quant < 0 || quant > 51) l2_die("dequantize: bad arguments");
  std::lock_guard<std::mutex> lk(g_l2.mu);
  const size_t n = (size_t)size * size * 2;
  if (!g_l2.ensure(2 * n)) l2_die("dequantize: staging alloc failed");
  hipStream_t st = g_l2.stream;
  L2CHK(hipMemcpyAsync(g_l2.buf, coeff, n, hipMemcpyHostToDevice, st));
  k_l2_dequant<<<1, 64, 0, st>>>((const int16_t *)g_l2.buf, (int16_t *)(g_l2.buf + n), quant, size);
  L2CHK(hipGetLastError());
  L2CHK(hipMemcpyAsync(rcoeff, g_l2.buf + n, n, hipMemcpyDeviceToHost, st));
  L2CHK(hipStreamSynchronize(st));
}

// common/common_block.c:148-156
void reconstruct_block(int16_t *block, uint8_t *pblock, uint8_t *rec, int size, int stride) {
  if (size < 2 || size > 64) l2_die("reconstruct_block: bad arguments");
  std::lock_guard<std::mutex> lk(g_l2.mu);
  const size_t n = (size_t)size * size;
  if (!g_l2.ensure(4 * n)) l2_die("reconstruct_block: staging alloc failed");
  hipStream_t st = g_l2.stream;
  uint8_t *db = g_l2.buf, *dp = db + 2 * n, *dout = dp + n;
  L2CHK(hipMemcpyAsync(db, block, 2 * n, hipMemcpyHostToDevice, st));
  L2CHK(hipMemcpyAsync(dp, pblock, n, hipMemcpyHostToDevice, st));
  k_l2_recon<<<1, 64, 0, st>>>((const int16_t *)db, dp, dout, size);
  L2CHK(hipGetLastError());
  L2CHK(hipMemcpy2DAsync(rec, stride, dout, size, size, size, hipMemcpyDeviceToHost, st));
  L2CHK(hipStreamSynchronize(st));
}

// common/intra_prediction.c:363-388
void get_intra_prediction(uint8_t *left, uint8_t *top, uint8_t top_left, int ypos, int xpos, int size,
                          uint8_t *pblock, int intra_mode) {
  if (size < 4 || size > 64) l2_die("get_intra_prediction: bad arguments");
  std::lock_guard<std::mutex> lk(g_l2.mu);
  const size_t nin = 4 * (size_t)size + 1, nout = (size_t)size * size;
  if (!g_l2.ensure(nin + nout + 64, nin)) l2_die("get_intra_prediction: staging alloc failed");
  memcpy(g_l2.host, left, 2 * size);
  memcpy(g_l2.host + 2 * size, top, 2 * size);
  g_l2.host[4 * size] = top_left;
  hipStream_t st = g_l2.stream;
  uint8_t *din = g_l2.buf, *dout = g_l2.buf + ((nin + 63) & ~(size_t)63);
  L2CHK(hipMemcpyAsync(din, g_l2.host, nin, hipMemcpyHostToDevice, st));
  k_l2_intra<<<1, 64, 0, st>>>(din, dout, ypos, xpos, size, intra_mode);
  L2CHK(hipGetLastError());
  L2CHK(hipMemcpyAsync(pblock, dout, nout, hipMemcpyDeviceToHost, st));
  L2CHK(hipStreamSynchronize(st));
}

// common/intra_prediction.c:57-143.  The host stages exactly the bytes the
// reference reads (which depend only on the positions and flags); the device
// builds the two neighbour arrays from them.
void make_top_and_left(uint8_t *left, uint8_t *top, uint8_t *top_left, uint8_t *rec_frame, int fstride,
                       uint8_t *rblock, int rbstride, int i, int j, int ypos, int xpos, int size,
                       int upright_available, int downleft_available, int tb_split) {
  if (size < 2 || size > 64) l2_die("make_top_and_left: bad arguments");
  int dl, ur;
  if (!tb_split) {
    dl = downleft_available;
    ur = upright_available;
  } else {
    dl = (j == 0 && (i == 0 || downleft_available)) ? 1 : 0;
    ur = (j == 0 || (i == 0 && upright_available)) ? 1 : 0;
  }
  const int leftlen = dl ? size + 1 : size, toplen = ur ? size + 1 : size;
  const int top128 = tb_split ? (ypos + i == 0) : (ypos == 0);
  const int left128 = tb_split ? (xpos + j == 0) : (xpos == 0);
  const uint8_t *tsrc = (!tb_split || i == 0) ? rec_frame - fstride + (tb_split ? j : 0) : rblock - rbstride;
  const uint8_t *lsrc = (!tb_split || j == 0) ? rec_frame + (tb_split ? i * fstride : 0) - 1 : rblock - 1;
  const int ls = (!tb_split || j == 0) ? fstride : rbstride;
  std::lock_guard<std::mutex> lk(g_l2.mu);
  const size_t nin = 4 * (size_t)size + 2, nout = 4 * (size_t)size + 1;
  if (!g_l2.ensure(nin + nout + 64, nin)) l2_die("make_top_and_left: staging alloc failed");
  uint8_t *h = g_l2.host;
  memset(h, 0, nin);
  int tl_mode = 0;
  if (!top128) {
    memcpy(h, tsrc, toplen);  // the top run (memcpy of toplen bytes, :78 / :113 / :118)
    if (xpos > 0) {           // the corner (:81 / :116 / :121)
      tl_mode = 1;
      if (!tb_split || i == 0) h[2 * size] = rec_frame[-fstride + (tb_split ? j : 0) - 1];
      else h[2 * size] = j > 0 ? rblock[-rbstride - 1] : rec_frame[(i - 1) * fstride - 1];
    }
  }
  if (!left128)
    for (int k = 0; k < leftlen; k++) h[2 * size + 1 + k] = lsrc[(long long)k * ls];  // :88-90 / :126-128 / :133-135
  hipStream_t st = g_l2.stream;
  uint8_t *din = g_l2.buf, *dout = g_l2.buf + ((nin + 63) & ~(size_t)63);
  L2CHK(hipMemcpyAsync(din, h, nin, hipMemcpyHostToDevice, st));
  k_l2_top_left<<<1, 64, 0, st>>>(din, dout, size, toplen, leftlen, top128, left128, tl_mode);
  L2CHK(hipGetLastError());
  L2CHK(hipMemcpyAsync(h, dout, nout, hipMemcpyDeviceToHost, st));
  L2CHK(hipStreamSynchronize(st));
  memcpy(left, h, 2 * size);
  memcpy(top, h + 2 * size, 2 * size);
  *top_left = h[4 * size];
}

// enc/encode_block.c:75-172
int quantize(int16_t *coeff, int16_t *coeffq, int qp, int size, int coeff_block_type, int rdoq) {
  if (rdoq) l2_die("quantize: rdoq 1 (full RDOQ) is not implemented by this build");
  if (size < 4 || size > 64 || (size & (size - 1)) || qp < 0 || qp > 51) l2_die("quantize: bad arguments");
  std::lock_guard<std::mutex> lk(g_l2.mu);
  const int q = size < 16 ? size : 16;
  const size_t n = (size_t)q * q * 2;
  if (!g_l2.ensure(2 * n + 64)) l2_die("quantize: staging alloc failed");
  hipStream_t st = g_l2.stream;
  uint8_t *din = g_l2.buf, *dout = din + n;
  int *dcbp = (int *)(dout + n);
  L2CHK(hipMemcpy2DAsync(din, 2 * q, coeff, 2 * (size_t)size, 2 * q, q, hipMemcpyHostToDevice, st));
  k_l2_quant<<<1, 64, 0, st>>>((const int16_t *)din, (int16_t *)dout, qp, size, coeff_block_type, dcbp);
  L2CHK(hipGetLastError());
  int cbp = 0;
  L2CHK(hipMemcpy2DAsync(coeffq, 2 * (size_t)size, dout, 2 * q, 2 * q, q, hipMemcpyDeviceToHost, st));
  L2CHK(hipMemcpyAsync(&cbp, dcbp, sizeof(int), hipMemcpyDeviceToHost, st));
  L2CHK(hipStreamSynchronize(st));
  return cbp;
}

}  // extern "C"
