// Per-frame reconstruction kernels for gfx950 (MI355X): cell side-info,
// inter MC + dequant + inverse transform + reconstruction, intra.
//
// Layout: frames live in a ring of padded slots in HBM (pad 96 luma / 48
// chroma, create_yuv_frame, common/common_frame.c:324-351).  The current
// frame is reconstructed in place into its slot; deblock / CLPF / pad then
// run in place (loopfilter.hip), after which the slot is a reference.
#include "common.h"

// ---------------------------------------------------------------------------
// k_prep: one wavefront per CU.  Writes the per-4x4 cell map (CU index) and
// the packed side-info that copy_deblock_data (dec/decode_block.c:122-156)
// stores for deblocking/CLPF.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_prep(const thor_block_t *__restrict__ blk, int nblocks,
                                              uint16_t *__restrict__ cellinfo, int32_t *__restrict__ cellmap,
                                              int cstride) {
  int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  int lane = threadIdx.x & 63;
  if (b >= nblocks) return;
  const thor_block_t &B = blk[b];
  int S = B.size;
  int mode = B.mode;
  int bw = B.bwidth >> 2, bh = B.bheight >> 2;
  int pb = mode == M_INTER ? B.pb_part : 0;
  int tb = B.tb_split > 0;
  int lsz = ilog2i(S);
  int lqv = lsz - (((tb || pb == 2 || pb == 3) && S > 8) ? 1 : 0);  // PART_VER / PART_QUAD, :90
  int lqh = lsz - (((tb || pb == 1 || pb == 3) && S > 8) ? 1 : 0);  // PART_HOR / PART_QUAD, :183
  uint16_t base = (uint16_t)((mode & 7) | ((B.cbp_y != 0) << 3) | ((B.cbp_u != 0) << 4) | ((B.cbp_v != 0) << 5) |
                             (lqv << 8) | (lqh << 11) | ((lsz - 3) << 14));
  int div = S >> 3;
  int y4 = B.ypos >> 2, x4 = B.xpos >> 2;
  for (int c = lane; c < bw * bh; c += 64) {
    int m = c / bw, n = c - m * bw;
    int q = 2 * (m / div) + (n / div);
    int a0 = B.mv0[2 * q], a1 = B.mv0[2 * q + 1], a2 = B.mv1[2 * q], a3 = B.mv1[2 * q + 1];
    int big = (abs(a0) >= 4) | (abs(a1) >= 4) | (abs(a2) >= 4) | (abs(a3) >= 4);
    int idx = (y4 + m) * cstride + x4 + n;
    cellinfo[idx] = base | (uint16_t)(big << 6);
    cellmap[idx] = b;
  }
}

// ---------------------------------------------------------------------------
// Motion compensation helpers (get_inter_prediction_luma/chroma,
// common/inter_prediction.c:72-180).  Reads are dword-aligned and realigned
// with v_alignbyte; the padded ring guarantees every tap is addressable.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void load_bytes12(const uint8_t *p, uint32_t &e0, uint32_t &e1, uint32_t &e2) {
  uintptr_t a = (uintptr_t)p;
  const uint32_t *w = (const uint32_t *)(a & ~(uintptr_t)3);
  uint32_t sh = (uint32_t)(a & 3);
  uint32_t d0 = w[0], d1 = w[1], d2 = w[2], d3 = w[3];
  e0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
  e1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
  e2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
}
__device__ __forceinline__ void load_bytes8(const uint8_t *p, uint32_t &e0, uint32_t &e1) {
  uintptr_t a = (uintptr_t)p;
  const uint32_t *w = (const uint32_t *)(a & ~(uintptr_t)3);
  uint32_t sh = (uint32_t)(a & 3);
  uint32_t d0 = w[0], d1 = w[1], d2 = w[2];
  e0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
  e1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
}
__device__ __forceinline__ int byte_of(uint32_t w, int i) { return (w >> (8 * i)) & 255; }

// Pack an already-clipped byte into lane-byte j.  The empty asm keeps hipcc
// (ROCm 7.2, gfx950) from fusing pairs of clip255(x >> n) into
// v_ashr_pk_u8_i32, which leaves the upper half of its destination register
// unchanged while the compiler assumes it zero: byte 2 came out corrupted
// (found by tests/test_gpu_kernels.py).
__device__ __forceinline__ uint32_t put_byte(int v, int j) {
  asm volatile("" : "+v"(v));
  return (uint32_t)v << (8 * j);
}

// Keep every MC tap inside the padded slot.  Conformant streams stay within
// +-80 px of the frame (the encoder clamps, enc/encode_block.c:816-828), so
// these clamps never bind for them; they only make malformed input safe.
__device__ __forceinline__ int ry_clamp(int v, int H) { return v < -(THOR_PAD_Y - 8) ? -(THOR_PAD_Y - 8) : (v > H + THOR_PAD_Y - 12 ? H + THOR_PAD_Y - 12 : v); }
__device__ __forceinline__ int rx_clamp(int v, int W) { return v < -(THOR_PAD_Y - 8) ? -(THOR_PAD_Y - 8) : (v > W + THOR_PAD_Y - 16 ? W + THOR_PAD_Y - 16 : v); }
__device__ __forceinline__ int ry_clamp_c(int v, int H) { return v < -(THOR_PAD_C - 4) ? -(THOR_PAD_C - 4) : (v > H + THOR_PAD_C - 6 ? H + THOR_PAD_C - 6 : v); }
__device__ __forceinline__ int rx_clamp_c(int v, int W) { return v < -(THOR_PAD_C - 4) ? -(THOR_PAD_C - 4) : (v > W + THOR_PAD_C - 8 ? W + THOR_PAD_C - 8 : v); }

// 6-tap luma filters, common/inter_prediction.c:47-59
__device__ __forceinline__ void luma_taps(int frac, int bipred, int t[6]) {
  if (bipred) {
    if (frac == 1) { t[0] = 2; t[1] = -10; t[2] = 59; t[3] = 17; t[4] = -5; t[5] = 1; }
    else if (frac == 2) { t[0] = 1; t[1] = -8; t[2] = 39; t[3] = 39; t[4] = -8; t[5] = 1; }
    else if (frac == 3) { t[0] = 1; t[1] = -5; t[2] = 17; t[3] = 59; t[4] = -10; t[5] = 2; }
    else { t[0] = 0; t[1] = 0; t[2] = 64; t[3] = 0; t[4] = 0; t[5] = 0; }
  } else {
    if (frac == 1) { t[0] = 1; t[1] = -7; t[2] = 55; t[3] = 19; t[4] = -5; t[5] = 1; }
    else if (frac == 2) { t[0] = 1; t[1] = -7; t[2] = 38; t[3] = 38; t[4] = -7; t[5] = 1; }
    else if (frac == 3) { t[0] = 1; t[1] = -5; t[2] = 19; t[3] = 55; t[4] = -7; t[5] = 1; }
    else { t[0] = 0; t[1] = 0; t[2] = 64; t[3] = 0; t[4] = 0; t[5] = 0; }
  }
}
// 4-tap 1/8-pel chroma filters, common/inter_prediction.c:61-70
__device__ __forceinline__ void chroma_taps(int frac, int t[4]) {
  const int c[8][4] = {{0, 64, 0, 0},    {-2, 58, 10, -2}, {-4, 54, 16, -2}, {-4, 44, 28, -4},
                       {-4, 36, 36, -4}, {-4, 28, 44, -4}, {-2, 16, 54, -4}, {-2, 10, 58, -2}};
  t[0] = c[frac][0]; t[1] = c[frac][1]; t[2] = c[frac][2]; t[3] = c[frac][3];
}

// Four horizontally adjacent luma predictions starting at `src` (the
// MV-displaced position of the first pixel).  Returns 4 packed bytes.
__device__ uint32_t mc_luma4(const uint8_t *src, int stride, int fx, int fy, int bipred) {
  if (fx == 0 && fy == 0) {  // integer MV: copy (inter_prediction.c:133-140)
    uint32_t e0, e1;
    load_bytes8(src, e0, e1);
    return e0;
  }
  if (fx == 2 && fy == 2) {  // (2,2) 4x4 low-pass (inter_prediction.c:145-157)
    int r[4][7];
    for (int a = 0; a < 4; a++) {
      uint32_t e0, e1;
      load_bytes8(src + (a - 1) * stride - 1, e0, e1);
      for (int i = 0; i < 4; i++) r[a][i] = byte_of(e0, i);
      for (int i = 0; i < 3; i++) r[a][4 + i] = byte_of(e1, i);
    }
    uint32_t out = 0;
    for (int j = 0; j < 4; j++) {
      int s = r[0][j + 1] + r[0][j + 2] + r[1][j] + 2 * r[1][j + 1] + 2 * r[1][j + 2] + r[1][j + 3] + r[2][j] +
              2 * r[2][j + 1] + 2 * r[2][j + 2] + r[2][j + 3] + r[3][j + 1] + r[3][j + 2];
      out |= put_byte(clip255((s + 8) >> 4), j);
    }
    return out;
  }
  int fv[6], fh[6];
  luma_taps(fy, bipred, fv);
  luma_taps(fx, bipred, fh);
  int v[9];
  for (int c = 0; c < 9; c++) v[c] = 0;
  // vertical 6-tap into int32 over columns -2..+6 (inter_prediction.c:160-168)
  for (int n = 0; n < 6; n++) {
    uint32_t e0, e1, e2;
    load_bytes12(src + (n - 2) * stride - 2, e0, e1, e2);
    int f = fv[n];
    for (int c = 0; c < 4; c++) v[c] += f * byte_of(e0, c);
    for (int c = 0; c < 4; c++) v[4 + c] += f * byte_of(e1, c);
    v[8] += f * byte_of(e2, 0);
  }
  uint32_t out = 0;
  for (int j = 0; j < 4; j++) {  // horizontal (inter_prediction.c:170-178)
    int s = fh[0] * v[j] + fh[1] * v[j + 1] + fh[2] * v[j + 2] + fh[3] * v[j + 3] + fh[4] * v[j + 4] + fh[5] * v[j + 5];
    out |= put_byte(clip255((s + 2048) >> 12), j);
  }
  return out;
}

// One chroma prediction at `src` (MV-displaced).  inter_prediction.c:86-117
__device__ int mc_chroma1(const uint8_t *src, int stride, int fx, int fy) {
  if (fx == 0 && fy == 0) return src[0];
  int th[4], tv[4];
  chroma_taps(fx, th);
  chroma_taps(fy, tv);
  int s = 0;
  for (int m = 0; m < 4; m++) {
    uint32_t e0, e1;
    load_bytes8(src + (m - 1) * stride - 1, e0, e1);
    int t = th[0] * byte_of(e0, 0) + th[1] * byte_of(e0, 1) + th[2] * byte_of(e0, 2) + th[3] * byte_of(e0, 3);
    s += tv[m] * t;
  }
  return clip255((s + 2048) >> 12);
}

// ---------------------------------------------------------------------------
// Residual: dequantize (common/common_block.c:132-146) + inverse transform
// (common/transform.c:432-518) restricted to the pixels a lane owns.
//   T[k][y'] = clip16((sum_m M[m][y'] * D[m][k] + 64) >> 7)     pass 1
//   r[y][x]  = clip16((sum_k M[k][x'] * T[k][y'] + 2048) >> 12) pass 2
// with m, k < q = min(N,16) (only the low-frequency corner is coded), M the
// N-point basis (N = 32 and x' = x/2, y' = y/2 for 64x64 TUs: 32-point IT
// then 2x2 replication, transform.c:496-517).  Pass 1 is shared by the `g`
// lanes that own the same TU row: lane `member` computes k = member, member+g..
// ---------------------------------------------------------------------------
struct TuRef {
  const int16_t *coef;  // compact q x q slots
  int ntu;              // TU size as coded (4..64): dequant shift
  int n;                // transform size (ntu, or 32 for 64)
  int q;                // min(n, 16)
  int qp;
  int rep;              // 1 for 64x64 TUs
};

__device__ __forceinline__ int dq(int c, int scale, int lshift, int add, int rshift) {
  return wrap16(((c * scale) * (1 << lshift) + add) >> rshift);
}

// pass 1 for IT row yp: this lane's share of T[k], written to lds[k]
__device__ __forceinline__ void it_pass1(const TuRef &t, const int8_t *M, int yp, int member, int g, int16_t *lds) {
  int lshift = t.qp / 6, scale = dequant_scale(t.qp % 6);
  int rshift = ilog2i(t.ntu) - 1, add = 1 << (rshift - 1);
  int step = 32 / t.n;
  for (int k = member; k < t.q; k += g) {
    int s = 0;
    for (int m = 0; m < t.q; m++) s += (int)M[(m * step) * 32 + yp] * dq(t.coef[m * t.q + k], scale, lshift, add, rshift);
    lds[k] = (int16_t)clip16((s + 64) >> 7);
  }
}
__device__ __forceinline__ int it_pass2(const TuRef &t, const int8_t *M, int xp, const int16_t *T) {
  int step = 32 / t.n;
  int s = 0;
  for (int k = 0; k < t.q; k++) s += (int)M[(k * step) * 32 + xp] * (int)T[k];
  return clip16((s + 2048) >> 12);
}

// ---------------------------------------------------------------------------
// k_inter: one wavefront per 16x16 luma tile (+ its 8x8 U and V tiles).
// Each lane owns a 1x4 luma strip and one pixel of each chroma plane; the CU
// covering a lane comes from the cell map, so a tile may hold one CU (>= 16)
// or four 8x8 CUs.  Restates decode_block for SKIP / MERGE / INTER / BIPRED
// (dec/decode_block.c:213-451): MC per quarter MV (INTER/BIPRED predict four
// size/2 quarters, :381-392), truncating bi-pred average (:272-283), then
// decode_and_reconstruct_block_inter (:90-120).  For intra CUs only the
// residual (dequant + inverse transform, dec/decode_block.c:67-69,80-81) is
// computed here -- it does not depend on neighbours -- and stored as int16
// into `resid` for k_intra, which adds it to the prediction.
// ---------------------------------------------------------------------------
#define TILE_WAVES 4
__global__ __launch_bounds__(256) void k_inter(FrameCtx f, const thor_block_t *__restrict__ blk,
                                               const int16_t *__restrict__ coeffs,
                                               const int32_t *__restrict__ cellmap, int tiles_w, int ntiles,
                                               int16_t *__restrict__ resid) {
  __shared__ int8_t Ms[32 * 32];
  __shared__ int16_t Tl[TILE_WAVES][64][16];
  for (int i = threadIdx.x; i < 1024; i += 256) Ms[i] = (int8_t)dct32_entry(i >> 5, i & 31);
  __syncthreads();
  int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  int tile = blockIdx.x * TILE_WAVES + wave;
  if (tile >= ntiles) return;
  int ty = tile / tiles_w, tx = tile - ty * tiles_w;
  int cs = f.W >> 2;
  int16_t(*T)[16] = Tl[wave];

  // ---------------- luma: lane -> row r, columns c0..c0+3 ----------------
  {
    int r = lane >> 2, c0 = (lane & 3) * 4;
    int y = ty * 16 + r, x = tx * 16 + c0;
    bool act = y < f.H;
    int b = act ? cellmap[(y >> 2) * cs + (x >> 2)] : 0;
    const thor_block_t &B = blk[b];
    int mode = B.mode;
    bool intra = act && mode == M_INTRA;
    act = act && mode != M_INTRA;
    if (mode == M_SKIP) act = act && (x < B.xpos + B.bwidth) && (y < B.ypos + B.bheight);
    int S = B.size;
    int xc = x - B.xpos, yc = y - B.ypos;
    uint32_t pred = 0;
    if (act) {
      int q = (mode == M_INTER || mode == M_BIPRED) ? (2 * (yc >= (S >> 1)) + (xc >= (S >> 1))) : 0;
      bool bi = mode == M_BIPRED || ((mode == M_SKIP || mode == M_MERGE) && B.dir == 2);
      int mvx = B.mv0[2 * q], mvy = B.mv0[2 * q + 1];
      int sg = bi ? (B.ref0 >= f.frame_num) : (B.ref0 > f.frame_num);
      if (sg) { mvx = -mvx; mvy = -mvy; }
      int sl = find_slot(f, B.ref0);
      const uint8_t *rp = slot_plane(f, sl < 0 ? 0 : sl, 0) + (long long)ry_clamp(y + (mvy >> 2), f.H) * f.sy +
                          rx_clamp(x + (mvx >> 2), f.W);
      pred = mc_luma4(rp, f.sy, mvx & 3, mvy & 3, f.bipred);
      if (bi) {
        int ux = B.mv1[2 * q], uy = B.mv1[2 * q + 1];
        if (B.ref1 >= f.frame_num) { ux = -ux; uy = -uy; }
        int s1 = find_slot(f, B.ref1);
        const uint8_t *rp1 = slot_plane(f, s1 < 0 ? 0 : s1, 0) + (long long)ry_clamp(y + (uy >> 2), f.H) * f.sy +
                             rx_clamp(x + (ux >> 2), f.W);
        uint32_t p1 = mc_luma4(rp1, f.sy, ux & 3, uy & 3, f.bipred);
        pred = (pred & p1) + (((pred ^ p1) >> 1) & 0x7f7f7f7fu);  // (p0+p1)>>1 per byte
      }
    }
    bool res = (act || intra) && mode != M_SKIP && (B.coeff_mask & 1);
    uint32_t outv = pred;
    // residual (cooperative pass 1 over lanes sharing a TU row)
    TuRef t;
    int xin = 0, yin = 0, g = 1;
    if (res) {
      int tb = B.tb_split != 0;
      t.ntu = tb ? S >> 1 : S;
      t.rep = t.ntu == 64;
      t.n = t.rep ? 32 : t.ntu;
      t.q = t.n < 16 ? t.n : 16;
      t.qp = B.qp;
      int ti = tb ? (2 * (yc >= t.ntu) + (xc >= t.ntu)) : 0;
      t.coef = coeffs + B.coeff_off[0] + ti * t.q * t.q;
      xin = xc - (tb ? (xc >= t.ntu) * t.ntu : 0);
      yin = yc - (tb ? (yc >= t.ntu) * t.ntu : 0);
      g = t.ntu >= 16 ? 4 : (t.ntu >> 2);
    }
    if (res) it_pass1(t, Ms, yin >> t.rep, lane % g, g, T[lane - lane % g]);
    wave_lds_sync();
    if (res) {
      outv = 0;
      int rr[4];
      for (int j = 0; j < 4; j++) {
        rr[j] = it_pass2(t, Ms, (xin + j) >> t.rep, T[lane - lane % g]);
        outv |= put_byte(clip255(rr[j] + (int)byte_of(pred, j)), j);
      }
      if (intra) {
        uint2 w;
        w.x = (uint32_t)(rr[0] & 0xffff) | ((uint32_t)rr[1] << 16);
        w.y = (uint32_t)(rr[2] & 0xffff) | ((uint32_t)rr[3] << 16);
        *(uint2 *)(resid + (long long)y * f.W + x) = w;
      }
    }
    if (act) *(uint32_t *)(f.cy + (long long)y * f.sy + x) = outv;
  }
  wave_lds_sync();

  // ---------------- chroma: lane -> one pixel of each plane ----------------
  {
    int r = lane >> 3, c = lane & 7;
    int y = ty * 8 + r, x = tx * 8 + c;  // chroma coordinates
    bool act = y < (f.H >> 1);
    int b = act ? cellmap[((2 * y) >> 2) * cs + ((2 * x) >> 2)] : 0;
    const thor_block_t &B = blk[b];
    int mode = B.mode;
    bool intra = act && mode == M_INTRA;
    act = act && mode != M_INTRA;
    if (mode == M_SKIP) act = act && (2 * x < B.xpos + B.bwidth) && (2 * y < B.ypos + B.bheight);
    int S = B.size, SC = S >> 1;
    int xc = x - (B.xpos >> 1), yc = y - (B.ypos >> 1);
    int q = (mode == M_INTER || mode == M_BIPRED) ? (2 * (yc >= (SC >> 1)) + (xc >= (SC >> 1))) : 0;
    bool bi = mode == M_BIPRED || ((mode == M_SKIP || mode == M_MERGE) && B.dir == 2);
    int mvx = B.mv0[2 * q], mvy = B.mv0[2 * q + 1];
    if (bi ? (B.ref0 >= f.frame_num) : (B.ref0 > f.frame_num)) { mvx = -mvx; mvy = -mvy; }
    int ux = B.mv1[2 * q], uy = B.mv1[2 * q + 1];
    if (B.ref1 >= f.frame_num) { ux = -ux; uy = -uy; }
    int sl0 = act ? find_slot(f, B.ref0) : 0, sl1 = (act && bi) ? find_slot(f, B.ref1) : 0;
    sl0 = sl0 < 0 ? 0 : sl0;
    sl1 = sl1 < 0 ? 0 : sl1;
    int tbc = B.tb_split && S > 8;  // dec/decode_block.c:449-450
    TuRef t;
    int xin = 0, yin = 0, g = 1;
    t.ntu = tbc ? SC >> 1 : SC;
    t.rep = 0;
    t.n = t.ntu;
    t.q = t.n < 16 ? t.n : 16;
    t.qp = chroma_qp(B.qp);
    int ti = tbc ? (2 * (yc >= t.ntu) + (xc >= t.ntu)) : 0;
    xin = xc - (tbc ? (xc >= t.ntu) * t.ntu : 0);
    yin = yc - (tbc ? (yc >= t.ntu) * t.ntu : 0);
    g = t.ntu >= 8 ? 8 : t.ntu;
    for (int comp = 1; comp <= 2; comp++) {
      int pred = 0;
      if (act) {
        const uint8_t *rp = slot_plane(f, sl0, comp) + (long long)ry_clamp_c(y + (mvy >> 3), f.H >> 1) * f.sc +
                            rx_clamp_c(x + (mvx >> 3), f.W >> 1);
        pred = mc_chroma1(rp, f.sc, mvx & 7, mvy & 7);
        if (bi) {
          const uint8_t *rp1 = slot_plane(f, sl1, comp) + (long long)ry_clamp_c(y + (uy >> 3), f.H >> 1) * f.sc +
                               rx_clamp_c(x + (ux >> 3), f.W >> 1);
          pred = (pred + mc_chroma1(rp1, f.sc, ux & 7, uy & 7)) >> 1;
        }
      }
      bool res = (act || intra) && mode != M_SKIP && (B.coeff_mask & (1 << comp));
      if (res) {
        t.coef = coeffs + B.coeff_off[comp] + ti * t.q * t.q;
        it_pass1(t, Ms, yin, lane % g, g, T[lane - lane % g]);
      }
      wave_lds_sync();
      int outv = pred;
      if (res) {
        int rr = it_pass2(t, Ms, xin, T[lane - lane % g]);
        outv = clip255(rr + pred);
        if (intra) {
          long long cplane = (long long)f.W * f.H + (long long)(comp - 1) * (f.W >> 1) * (f.H >> 1);
          resid[cplane + (long long)y * (f.W >> 1) + x] = (int16_t)rr;
        }
      }
      wave_lds_sync();
      if (act) (comp == 1 ? f.cu : f.cv)[(long long)y * f.sc + x] = (uint8_t)outv;
    }
  }
}

