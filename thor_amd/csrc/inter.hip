// k_recon: inter reconstruction, one wavefront per half (64x32) superblock (gfx950).
//
// Restates, for every non-intra CU of a frame, decode_block's prediction
// (dec/decode_block.c:213-451: SKIP / MERGE / INTER / BIPRED; INTER and BIPRED
// predict four size/2 quarters with mv_arr[i], :381-392; truncating bi-pred
// average, :272-283) through get_inter_prediction_luma/chroma
// (common/inter_prediction.c:72-180), then reconstruct_block
// (common/common_block.c:148-156) with the residual k_prep_resid (resid.hip) left in
// the int16 residual planes (dequantize + inverse_transform, :90-120).
//
// One wave per half SB (rows 0-31 or 32-63), mapped XCD-major (a band of
// consecutive half SBs per XCD, so neighbours share their reference rows in
// that XCD's L2).
//  P0  lane = one 4-row half of an 8x8 unit: resolve its 4x4 cells' MC parameters -- quarter MV
//      with the `sign` negation (inter_prediction.c:78-79, :125-126),
//      reference slot, bi-pred, coded residual per component -- into LDS.
//  P1  one pass (two with bi-pred: mv1 / slot1 of the bi-pred cells).
//      Work item = (lane, segment): lane = 4-px luma column x 8 rows + 2-px
//      chroma column x 4 rows per plane; segment = one 4x4 cell row (the MV may
//      change every 4 luma rows: 8x8 INTER quarters).  A job takes the distinct
//      (mv, slot) keys of its items one at a time (one key per job in the
//      common case): that key's displaced reference window (37 x 96 B luma,
//      2 x 19 x 64 B chroma) is staged HBM -> LDS with 16-byte loads, all in
//      flight at once, biased (^0x80) on the way.
//      Horizontal taps: v_dot4_i32_i8 on the (p - 128) bytes (the bias folds
//      into the rounding constant); vertical taps: v_dot2_i32_i16 on pairs of
//      rows of the int16 horizontal sums.  Taps are uniform per key.  The (2,2)
//      centre filter (inter_prediction.c:145-157) is u_i + u_j, u = [0 1 1 0]:
//      a 4-tap and a 2-tap horizontal sum per row, packed, four v_dot2 down.
//  P2  residual add where the cell's CU carries coefficients, then
//      the lane's rows go to the frame (64 contiguous bytes per 16 lanes/row).
//
// Separable order: the reference computes the vertical taps first into int32
// and the horizontal second; the sum is the same exact integer either way.
#include <stddef.h>

#include <type_traits>

#include "common.h"

#ifndef RECON_PROBE
#define RECON_PROBE 0  // timing-only probe builds (tools/gpu_var.sh); 0 in the product
#endif

#define SB_CELLS 256

// The work unit (common.h): 128 x 16 luma + 2 x 64 x 8 chroma, two SBs side by
// side.  Lane geometry: LCC = 4-px luma / 2-px chroma column (0..31), LGR = row
// group (8 luma / 4 chroma rows, 0..1).
#define LCC(lane) ((lane) & 31)
#define LGR(lane) ((lane) >> 5)

// reference window for one (mv, slot) key and one unit
#define WL_P 160  // luma pitch: 128 + 5 taps + 15 alignment -> 160 B (10 chunks)
#define WL_R 21   // 16 rows + 5
#define WC_P 96   // chroma pitch: 64 + 3 + 15 -> 96 B (6 chunks)
#define WC_R 11   // 8 rows + 3
#define WL_CH (WL_R * WL_P / 16)  // 16-byte chunks: 210
#define WC_CH (WC_R * WC_P / 16)  // 66 per plane
#define WIN_LOADS 6               // ceil((210 + 2 * 66) / 64)
struct alignas(16) RefWin {  // 16-B aligned: window chunks and the store transposes move as ds_*_b128
  uint8_t y[WL_R * WL_P];
  uint8_t u[WC_R * WC_P];
  uint8_t v[WC_R * WC_P];
};

#define UNIT_CELLS 128  // 4 cell rows x 32 cells
struct ReconLds {
  RefWin win;
  int mv0[UNIT_CELLS];        // per 4x4 cell: (mvx, mvy) int16 pair, sign applied
  int mv1[UNIT_CELLS];
  unsigned meta[UNIT_CELLS];  // slot0 | slot1 << 8 | ACT | BI | RES(c)
  int8_t lut[128];            // display frame number & 127 -> ring slot
};

__device__ __forceinline__ int tap8(int w, int i) { return __builtin_amdgcn_sbfe(w, 8 * i, 8); }

// Filter tables (common/inter_prediction.c:47-70) as packed int8 words:
// luma word0 = taps 0..3, word1 = taps 4,5 (uni table, then the sequence-level
// bipred table); chroma = 4 taps.  Indexed by uniform fractions: scalar loads.
struct TapTables {
  int luma[2][4][2];
  int chroma[8];
  constexpr TapTables() : luma(), chroma() {
    const int t[2][4][6] = {{{0, 0, 64, 0, 0, 0}, {1, -7, 55, 19, -5, 1}, {1, -7, 38, 38, -7, 1}, {1, -5, 19, 55, -7, 1}},
                            {{0, 0, 64, 0, 0, 0}, {2, -10, 59, 17, -5, 1}, {1, -8, 39, 39, -8, 1}, {1, -5, 17, 59, -10, 2}}};
    const int c[8][4] = {{0, 64, 0, 0},    {-2, 58, 10, -2}, {-4, 54, 16, -2}, {-4, 44, 28, -4},
                         {-4, 36, 36, -4}, {-4, 28, 44, -4}, {-2, 16, 54, -4}, {-2, 10, 58, -2}};
    for (int b = 0; b < 2; b++)
      for (int f = 0; f < 4; f++) {
        luma[b][f][0] = (t[b][f][0] & 255) | ((t[b][f][1] & 255) << 8) | ((t[b][f][2] & 255) << 16) |
                        (int)((unsigned)(t[b][f][3] & 255) << 24);
        luma[b][f][1] = (t[b][f][4] & 255) | ((t[b][f][5] & 255) << 8);
      }
    for (int f = 0; f < 8; f++)
      chroma[f] = (c[f][0] & 255) | ((c[f][1] & 255) << 8) | ((c[f][2] & 255) << 16) | (int)((unsigned)(c[f][3] & 255) << 24);
  }
};
__constant__ TapTables g_taps = TapTables();
// The host copy of the same words: capi.hip puts it into k_recon's ReconGeo.
constexpr TapTables k_taps = TapTables();

// Rounding constant of the 2-D filters with the (p - 128) bias folded in:
// 2048 + 128 * 64 * 64 (every tap set sums to 64).
#define MC_RND (2048 + 524288)

// Horizontal sums H' = sum t_k (p_k - 128) fit int16 (|H'| <= 128 * 94 for
// every luma table, 128 * 64 for the scaled centre terms, 128 * 72 chroma), so
// the vertical pass runs on pairs of rows packed as int16x2 with
// v_dot2_i32_i16: P(r) = (H'[r], H'[r+1]) per pixel, three dot2 per luma
// pixel (taps (t0,t1) (t2,t3) (t4,t5)), two per chroma pixel.
typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int dot2(uint32_t pair, int taps, int acc) {
  return __builtin_amdgcn_sdot2(__builtin_bit_cast(s16x2, pair), __builtin_bit_cast(s16x2, taps), acc, false);
}
__device__ __forceinline__ int dot4(uint32_t a, int taps, int acc) {
  return __builtin_amdgcn_sdot4((int)a, taps, acc, false);
}
__device__ __forceinline__ int dot4z(uint32_t a, int taps) { return dot4(a, taps, 0); }
__device__ __forceinline__ uint32_t pack_lo16(int lo, int hi) {  // (lo & 0xffff) | hi << 16
  return __builtin_amdgcn_perm((uint32_t)hi, (uint32_t)lo, 0x05040100u);
}
// packed int16 pairs of a 6-tap word (t0,t1), (t2,t3), (t4,t5)
// (the fast path scales them: m = 16, |tap| x 16 <= 944 stays an int16)
__device__ __forceinline__ int tap_pair(int a, int b, int m) { return ((a * m) & 0xffff) | ((b * m) << 16); }
__device__ __forceinline__ void tap_pairs6(int w0, int w1, int &p01, int &p23, int &p45, int m = 1) {
  p01 = tap_pair(tap8(w0, 0), tap8(w0, 1), m);
  p23 = tap_pair(tap8(w0, 2), tap8(w0, 3), m);
  p45 = tap_pair(tap8(w1, 0), tap8(w1, 1), m);
}

// Four horizontal 6-tap sums from the 12 bytes d0..d2 (window bytes are stored ^ 0x80),
// starting `sh` bytes in (the byte 2 left of the lane's first pixel).
__device__ __forceinline__ void luma_h4(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t sh, int tw0, int tw1,
                                        int h[4]) {
  const uint32_t e0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
  const uint32_t e1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
  const uint32_t e2 = __builtin_amdgcn_alignbyte(d2, d2, sh);  // byte 0 = byte 8 of the window
  h[0] = dot4(e1, tw1, dot4z(e0, tw0));
#pragma unroll
  for (int j = 1; j < 4; j++) {
    const uint32_t lo = __builtin_amdgcn_alignbyte(e1, e0, j), hi = __builtin_amdgcn_alignbyte(e2, e1, j);
    h[j] = dot4(hi, tw1, dot4z(lo, tw0));
  }
}

// clip255 of four ints packed as bytes a | b << 8 | c << 16 | d << 24:
// saturate to int16 pairs (v_cvt_pk_i16_i32), then to u8 (v_sat_pk_u8_i16),
// then one byte permute -- 5 instructions instead of 4 x (clamp, shift, or).
__device__ __forceinline__ uint32_t sat_u8x2(int a, int b) {
  const s16x2 p = __builtin_amdgcn_cvt_pk_i16(a, b);
  uint32_t r;
  asm("v_sat_pk_u8_i16 %0, %1" : "=v"(r) : "v"(p));
  return r;  // bytes 0, 1 (the upper half is not relied upon)
}
__device__ __forceinline__ uint32_t pack4_u8(int a, int b, int c, int d) {
  return __builtin_amdgcn_perm(sat_u8x2(c, d), sat_u8x2(a, b), 0x05040100u);
}
// clip255(s >> 16) of four sums packed as bytes: the high halves of (a, b)
// and (c, d) as int16 pairs (one byte permute each), then v_sat_pk_u8_i16.
// The fast path scales its vertical taps by 16 so that the >> 12 of the 2-D
// filters is this >> 16 (5 instructions per 4 px instead of 9).
__device__ __forceinline__ uint32_t sat_u8x2_pk(uint32_t p) {
  uint32_t r;
  asm("v_sat_pk_u8_i16 %0, %1" : "=v"(r) : "v"(p));
  return r;
}
__device__ __forceinline__ uint32_t pack4_hi16_u8(int a, int b, int c, int d) {
  const uint32_t ab = __builtin_amdgcn_perm((uint32_t)b, (uint32_t)a, 0x07060302u);
  const uint32_t cd = __builtin_amdgcn_perm((uint32_t)d, (uint32_t)c, 0x07060302u);
  return __builtin_amdgcn_perm(sat_u8x2_pk(cd), sat_u8x2_pk(ab), 0x05040100u);
}
__device__ __forceinline__ uint32_t avg_bytes(uint32_t a, uint32_t b) {  // (p0 + p1) >> 1 per byte
  return (a & b) + (((a ^ b) >> 1) & 0x7f7f7f7fu);
}


// The uniform filter of one key.
struct Key {
  int mv, slot;
  int fx, fy, cfx, cfy;  // luma quarter / chroma eighth fractions
  int dx, dy, cdx, cdy;  // integer displacements
};
// Row sources.  A staged LDS window (bytes already biased ^0x80), or the
// reference ring directly (waves whose items need more than one window): the
// direct source prefetches every row of a call before any arithmetic.
struct LdsLuma {
  static constexpr bool PF = false;
  const uint8_t *base;  // window byte of strip row -2, column -2 (dword aligned)
  __device__ __forceinline__ void get(int r, uint32_t d[3]) const {
    const uint32_t *p = (const uint32_t *)(base + (r + 2) * WL_P);
    d[0] = p[0]; d[1] = p[1]; d[2] = p[2];
  }
};
struct GlobLuma {
  static constexpr bool PF = false;
  __amdgpu_buffer_rsrc_t ring;
  int o, stride;  // ring offset of strip row 0, column -2 (dword aligned)
  __device__ __forceinline__ void get(int r, uint32_t d[3]) const {
    const auto v = __builtin_amdgcn_raw_buffer_load_b96(ring, o + r * stride, 0, 0);
    d[0] = v[0] ^ 0x80808080u; d[1] = v[1] ^ 0x80808080u; d[2] = v[2] ^ 0x80808080u;
  }
};
struct LdsChroma {
  static constexpr bool PF = false;
  const uint8_t *u, *v;  // window byte of strip row -1, column -1 (dword aligned)
  __device__ __forceinline__ void get(int r, uint32_t du[2], uint32_t dv[2]) const {
    const uint32_t *pu = (const uint32_t *)(u + (r + 1) * WC_P), *pv = (const uint32_t *)(v + (r + 1) * WC_P);
    du[0] = pu[0]; du[1] = pu[1]; dv[0] = pv[0]; dv[1] = pv[1];
  }
};
struct GlobChroma {
  static constexpr bool PF = false;
  __amdgpu_buffer_rsrc_t ring;
  int o, uvd, stride;  // ring offset (U) of strip row 0, column -1 (dword aligned)
  __device__ __forceinline__ void get(int r, uint32_t du[2], uint32_t dv[2]) const {
    const auto a = __builtin_amdgcn_raw_buffer_load_b64(ring, o + r * stride, 0, 0);
    const auto b = __builtin_amdgcn_raw_buffer_load_b64(ring, o + uvd + r * stride, 0, 0);
    du[0] = a[0] ^ 0x80808080u; du[1] = a[1] ^ 0x80808080u; dv[0] = b[0] ^ 0x80808080u; dv[1] = b[1] ^ 0x80808080u;
  }
};

// Luma rows R0 .. R0+N-1 of the lane's 8-row strip; `sh` = byte offset of
// column -2 inside the fetched dwords.  Vertical taps as int16 pairs.
template <int R0, int N, class Src>
__device__ __forceinline__ void luma_rows(const Src &src, uint32_t sh, int tw0, int tw1, int v01, int v23, int v45,
                                          uint32_t out[8], bool acc) {
  constexpr int NR = N + 5;
  uint32_t pre[Src::PF ? NR : 1][3];
  if (Src::PF) {
#pragma unroll
    for (int k = 0; k < NR; k++) src.get(R0 - 2 + k, pre[Src::PF ? k : 0]);
  }
  int hp[4];                // H' of the previous row
  uint32_t pa[6][4];        // P(r) = (H'[r], H'[r+1]), ring by strip row
  auto hrow = [&](int r) {  // strip row r -> P(r-1)
    uint32_t d[3];
    if (Src::PF) { d[0] = pre[Src::PF ? r - R0 + 2 : 0][0]; d[1] = pre[Src::PF ? r - R0 + 2 : 0][1]; d[2] = pre[Src::PF ? r - R0 + 2 : 0][2]; }
    else src.get(r, d);
    int hc[4];
    luma_h4(d[0], d[1], d[2], sh, tw0, tw1, hc);
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (r > R0 - 2) pa[(r + 5) % 6][j] = pack_lo16(hp[j], hc[j]);
      hp[j] = hc[j];
    }
  };
#pragma unroll
  for (int r = R0 - 2; r <= R0 + 2; r++) hrow(r);
#pragma unroll
  for (int i = R0; i < R0 + N; i++) {
    hrow(i + 3);
    int v[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      int a = dot2(pa[(i - 2 + 6) % 6][j], v01, MC_RND);
      a = dot2(pa[(i + 6) % 6][j], v23, a);
      a = dot2(pa[(i + 2 + 6) % 6][j], v45, a);
      v[j] = a >> 12;
    }
    const uint32_t o = pack4_u8(v[0], v[1], v[2], v[3]);
    out[i] = acc ? avg_bytes(out[i], o) : o;  // bi-pred: truncating average with pass 0
  }
}

// The (2,2) centre position (inter_prediction.c:145-157): kernel
// K[i][j] = u_i + u_j over rows / columns -1..2, u = [0 1 1 0], so per output
// row o: S = Hv(o) + Hv(o+1) + Hu(o-1) + Hu(o) + Hu(o+1) + Hu(o+2) with Hv the
// 4-tap [1 1 1 1] and Hu the 2-tap [1 1] horizontal sums.  Q(r) = (Hv, Hu)
// packed int16 -> four v_dot2 per pixel; (S + 8) >> 4 with the bias
// 128 * 16 = 2048 folded in.
template <int R0, int N, class Src>
__device__ __forceinline__ void luma_rows_ctr(const Src &src, uint32_t sh, uint32_t out[8], bool acc) {
  constexpr int NR = N + 3;
  uint32_t pre[Src::PF ? NR : 1][3];
  if (Src::PF) {
#pragma unroll
    for (int k = 0; k < NR; k++) src.get(R0 - 1 + k, pre[Src::PF ? k : 0]);
  }
  uint32_t q[6][4];
  auto hrow = [&](int r) {
    uint32_t d[3];
    if (Src::PF) { d[0] = pre[Src::PF ? r - R0 + 1 : 0][0]; d[1] = pre[Src::PF ? r - R0 + 1 : 0][1]; d[2] = pre[Src::PF ? r - R0 + 1 : 0][2]; }
    else src.get(r, d);
    const uint32_t e0 = __builtin_amdgcn_alignbyte(d[1], d[0], sh), e1 = __builtin_amdgcn_alignbyte(d[2], d[1], sh);
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t lo = j ? __builtin_amdgcn_alignbyte(e1, e0, j) : e0;  // bytes at offsets -2..1
      const uint32_t hi = j ? __builtin_amdgcn_alignbyte(e1, e1, j) : e1;  // byte 0 at offset 2
      const int hv = dot4(hi, 0x00000001, dot4z(lo, 0x01010100));
      const int hu = dot4z(lo, 0x01010000);
      q[(r + 6) % 6][j] = pack_lo16(hv, hu);
    }
  };
#pragma unroll
  for (int r = R0 - 1; r <= R0 + 2; r++) hrow(r);
#pragma unroll
  for (int i = R0; i < R0 + N; i++) {
    if (i > R0) hrow(i + 2);
    int v[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      int a = dot2(q[(i - 1 + 6) % 6][j], 0x00010000, 2048 + 8);
      a = dot2(q[(i + 6) % 6][j], 0x00010001, a);
      a = dot2(q[(i + 1 + 6) % 6][j], 0x00010001, a);
      a = dot2(q[(i + 2 + 6) % 6][j], 0x00010000, a);
      v[j] = a >> 4;
    }
    const uint32_t o = pack4_u8(v[0], v[1], v[2], v[3]);
    out[i] = acc ? avg_bytes(out[i], o) : o;  // bi-pred: truncating average with pass 0
  }
}

// Chroma rows R0 .. R0+N-1 (of 4) of the lane's 2-px column, U and V.
template <int R0, int N, class Src>
__device__ __forceinline__ void chroma_rows(const Src &src, uint32_t sh, int tw, int v01, int v23, uint32_t out[4],
                                            bool acc) {
  constexpr int NR = N + 3;
  uint32_t preu[Src::PF ? NR : 1][2], prev_[Src::PF ? NR : 1][2];
  if (Src::PF) {
#pragma unroll
    for (int k = 0; k < NR; k++) src.get(R0 - 1 + k, preu[Src::PF ? k : 0], prev_[Src::PF ? k : 0]);
  }
  int pu_prev[2], pv_prev[2];
  uint32_t pu[4][2], pv[4][2];  // P(r) = (H'[r], H'[r+1]) per plane
  auto h2 = [&](const uint32_t d[2], int h[2]) {
    const uint32_t e0 = __builtin_amdgcn_alignbyte(d[1], d[0], sh);
    const uint32_t e1 = sh == 3 ? d[1] : __builtin_amdgcn_alignbyte(d[1], d[0], sh + 1);
    h[0] = dot4z(e0, tw);
    h[1] = dot4z(e1, tw);
  };
  auto hrow = [&](int r) {
    uint32_t du[2], dv[2];
    if (Src::PF) {
      const int k = Src::PF ? r - R0 + 1 : 0;
      du[0] = preu[k][0]; du[1] = preu[k][1]; dv[0] = prev_[k][0]; dv[1] = prev_[k][1];
    } else src.get(r, du, dv);
    int hu[2], hv[2];
    h2(du, hu);
    h2(dv, hv);
#pragma unroll
    for (int j = 0; j < 2; j++) {
      if (r > R0 - 1) {
        pu[(r + 3) % 4][j] = pack_lo16(pu_prev[j], hu[j]);
        pv[(r + 3) % 4][j] = pack_lo16(pv_prev[j], hv[j]);
      }
      pu_prev[j] = hu[j];
      pv_prev[j] = hv[j];
    }
  };
#pragma unroll
  for (int r = R0 - 1; r <= R0 + 1; r++) hrow(r);
#pragma unroll
  for (int i = R0; i < R0 + N; i++) {
    hrow(i + 2);
    int au[2], av[2];
#pragma unroll
    for (int j = 0; j < 2; j++) {
      au[j] = dot2(pu[(i + 1) % 4][j], v23, dot2(pu[(i + 3) % 4][j], v01, MC_RND)) >> 12;
      av[j] = dot2(pv[(i + 1) % 4][j], v23, dot2(pv[(i + 3) % 4][j], v01, MC_RND)) >> 12;
    }
    const uint32_t uv = pack4_u8(au[0], au[1], av[0], av[1]);  // U in the low half, V in the high half
    out[i] = acc ? avg_bytes(out[i], uv) : uv;
  }
}

// The luma / chroma calls of one segment set: both segments (rows 0-7 / 0-3)
// when they share the key, else each on its own.
template <class LSrc, class CSrc>
__device__ __forceinline__ void filter_items(bool m0, bool m1, const LSrc &l0, const LSrc &l1, uint32_t lsh0, uint32_t lsh1,
                                             const CSrc &c0, const CSrc &c1, uint32_t csh0, uint32_t csh1,
                                             const Key &K0, const Key &K1, bool same, int bipred, uint32_t ty[8],
                                             uint32_t tc[4], bool acc) {
  auto luma = [&](auto r0c, auto nc, const LSrc &src, uint32_t sh, const Key &K) {
    constexpr int R0 = decltype(r0c)::value, N = decltype(nc)::value;
    if (K.fx == 2 && K.fy == 2) luma_rows_ctr<R0, N>(src, sh, ty, acc);
    else {
      int v01, v23, v45;
      tap_pairs6(g_taps.luma[bipred][K.fy][0], g_taps.luma[bipred][K.fy][1], v01, v23, v45);
      luma_rows<R0, N>(src, sh, g_taps.luma[bipred][K.fx][0], g_taps.luma[bipred][K.fx][1], v01, v23, v45, ty, acc);
    }
  };
  auto chroma = [&](auto r0c, auto nc, const CSrc &src, uint32_t sh, const Key &K) {
    constexpr int R0 = decltype(r0c)::value, N = decltype(nc)::value;
    const int cvt = g_taps.chroma[K.cfy];
    chroma_rows<R0, N>(src, sh, g_taps.chroma[K.cfx], (tap8(cvt, 0) & 0xffff) | (tap8(cvt, 1) << 16),
                       (tap8(cvt, 2) & 0xffff) | (tap8(cvt, 3) << 16), tc, acc);
  };
  using I0 = std::integral_constant<int, 0>;
  using I2 = std::integral_constant<int, 2>;
  using I4 = std::integral_constant<int, 4>;
  using I8 = std::integral_constant<int, 8>;
  if (m0 && m1 && same) {
    luma(I0{}, I8{}, l0, lsh0, K0);
    chroma(I0{}, I4{}, c0, csh0, K0);
  } else {
    if (m0) { luma(I0{}, I4{}, l0, lsh0, K0); chroma(I0{}, I2{}, c0, csh0, K0); }
    if (m1) { luma(I4{}, I4{}, l1, lsh1, K1); chroma(I2{}, I2{}, c1, csh1, K1); }
  }
}

__device__ __forceinline__ Key make_key(int mv, int slot) {
  Key K;
  K.mv = mv;
  K.slot = slot;
  const int mvx = (int)(int16_t)(mv & 0xffff), mvy = mv >> 16;
  K.fx = mvx & 3; K.fy = mvy & 3; K.dx = mvx >> 2; K.dy = mvy >> 2;      // quarter-pel luma
  K.cfx = mvx & 7; K.cfy = mvy & 7; K.cdx = mvx >> 3; K.cdy = mvy >> 3;  // the same value as 1/8-pel chroma, :80-83
  return K;
}

// Window loads of key K for the half SB whose luma origin is (x0, y0): every
// byte a matching item reads lies inside.  Rows / columns outside the slot's
// padding only occur for non-conformant MVs and then read other ring memory
// or (past the ring) zeros through the buffer descriptor -- never out of bounds.
struct WinLoad {
  uint4 v[WIN_LOADS];
};
// Chunk q (16 bytes) of the window is LDS bytes [16q, 16q + 16): RefWin is
// contiguous, luma rows of WL_P = 10 chunks, then U and V rows of WC_P = 6.
// Its ring offset is its row's start + 16 x its column, i.e. 16q plus
// (row x (stride - pitch)): per load a reciprocal multiply for the row and one
// multiply-add; loads 0-2 are all luma, 4-5 all chroma.
__device__ __forceinline__ void win_issue(WinLoad &W, const FrameCtx &f, __amdgpu_buffer_rsrc_t ring, const Key &K,
                                          int x0, int y0) {
  const int lane = threadIdx.x;
  const long long sbase = (long long)K.slot * f.slot_bytes;
  const int cx0 = x0 >> 1, cy0 = y0 >> 1;
  const int ly = (int)(sbase + f.offy + (long long)(y0 - 2 + K.dy) * f.sy + ((x0 - 2 + K.dx) & ~15));
  const int cu = (int)(sbase + f.offu + (long long)(cy0 - 1 + K.cdy) * f.sc + ((cx0 - 1 + K.cdx) & ~15));
  const int uvd = (int)(f.offv - f.offu) - WC_R * WC_P;  // V rows follow U's in the window
  const int syd = f.sy - WL_P, scd = f.sc - WC_P;
#pragma unroll
  for (int i = 0; i < WIN_LOADS; i++) {
    const int q = lane + 64 * i;
    int offl = 0, offc = 0;
    if (64 * i < WL_CH) offl = ly + 16 * q + __mul24((q * 205) >> 11, syd);  // q / 10, exact for q < 1029 (24-bit mad)
    if (64 * i + 63 >= WL_CH) {
      const int q2 = q - WL_CH;  // chroma chunk: U 0..65, V 66..131
      const bool pv = q2 >= WC_CH;
      const int q3 = pv ? q2 - WC_CH : q2;
      offc = cu + 16 * q2 + (pv ? uvd : 0) + __mul24((q3 * 171) >> 10, scd);  // q3 / 6, exact for q3 < 256
    }
    int off = 64 * i + 63 < WL_CH ? offl : (64 * i >= WL_CH ? offc : (q < WL_CH ? offl : offc));
#if RECON_PROBE == 1  // timing probe: the same bytes as whole 128-B lines, 8 rows per load (wrong output)
    off = (int)((ly & ~127) + (q >> 3) * f.sy + (q & 7) * 16);
#elif RECON_PROBE == 2  // timing probe: no chroma window loads (wrong output)
    if (64 * i >= WL_CH) continue;
#elif RECON_PROBE == 4  // timing probe: every wave loads the same 6 KB (wrong output)
    off = (int)(f.offy + 16 * q);
#endif
    if (64 * i + 63 >= WL_CH + 2 * WC_CH && q >= WL_CH + 2 * WC_CH) continue;  // past the window
    W.v[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(ring, off, 0, 0));
  }
}
__device__ __forceinline__ void win_commit(const WinLoad &W, RefWin &w) {
  static_assert(sizeof(RefWin) == 16 * (WL_CH + 2 * WC_CH), "window chunks are contiguous");
  const int lane = threadIdx.x;
#pragma unroll
  for (int i = 0; i < WIN_LOADS; i++)
    if (64 * i + 63 < WL_CH + 2 * WC_CH || lane + 64 * i < WL_CH + 2 * WC_CH) {
      uint4 v = W.v[i];
      v.x ^= 0x80808080u; v.y ^= 0x80808080u; v.z ^= 0x80808080u; v.w ^= 0x80808080u;
      *(uint4 *)(w.y + 16 * (lane + 64 * i)) = v;
    }
}

// A pass's items of this lane: segment s (cell row 2 LGR + s of the unit).
struct Items {
  unsigned pend;
  int mv[2], slot[2];
};
__device__ __forceinline__ Items job_items(const ReconLds &L, int pass) {
  const int lane = threadIdx.x, cc = LCC(lane), gr = LGR(lane);
  Items it;
  it.pend = 0;
#pragma unroll
  for (int s = 0; s < 2; s++) {
    const int cell = (2 * gr + s) * 32 + cc;
    const unsigned meta = L.meta[cell];
    const bool act = (meta & CELL_ACT) && (pass == 0 || (meta & CELL_BI));
    it.mv[s] = pass ? L.mv1[cell] : L.mv0[cell];
    it.slot[s] = pass ? (int)((meta >> 8) & 255) : (int)(meta & 255);
    it.pend |= act ? (1u << s) : 0u;
  }
  return it;
}
// The first pending key of a job (uniform); false if the job has no items.
__device__ __forceinline__ bool first_key(const Items &it, Key &K) {
  const unsigned long long bal = __ballot(it.pend != 0);
  if (!bal) return false;
  const int ln = __builtin_ctzll(bal);
  const int s1 = (it.pend & 1) ? 0 : 1;
  K = make_key(__builtin_amdgcn_readlane(s1 ? it.mv[1] : it.mv[0], ln),
               __builtin_amdgcn_readlane(s1 ? it.slot[1] : it.slot[0], ln));
  return true;
}

// Filter every pending item whose key is K from the staged window; clears them.
__device__ __forceinline__ void filter_key(const RefWin &w, const Key &K, int bipred, int x0, Items &it, uint32_t ty[8],
                                           uint32_t tc[4], bool acc) {
  const int lane = threadIdx.x, cc = LCC(lane), gr = LGR(lane);
  const bool m0 = (it.pend & 1) && it.mv[0] == K.mv && it.slot[0] == K.slot;
  const bool m1 = (it.pend & 2) && it.mv[1] == K.mv && it.slot[1] == K.slot;
  const int lwb = 4 * cc + ((x0 - 2 + K.dx) & 15);
  const int cwb = 2 * cc + (((x0 >> 1) - 1 + K.cdx) & 15);
  const LdsLuma l{w.y + 8 * gr * WL_P + (lwb & ~3)};
  const LdsChroma c{w.u + 4 * gr * WC_P + (cwb & ~3), w.v + 4 * gr * WC_P + (cwb & ~3)};
  // The key is uniform, so every lane filters its whole strip (8 luma, 4
  // chroma rows) with ONE instantiation per filter shape, and each segment
  // keeps the result only where it matches: a small code footprint for the
  // common path (k_recon's code otherwise overflows the instruction cache).
  uint32_t ny[8], nc[4];
  if (K.fx == 2 && K.fy == 2) {
    luma_rows_ctr<0, 8>(l, (uint32_t)(lwb & 3), ny, false);
  } else {
    int v01, v23, v45;
    tap_pairs6(g_taps.luma[bipred][K.fy][0], g_taps.luma[bipred][K.fy][1], v01, v23, v45);
    luma_rows<0, 8>(l, (uint32_t)(lwb & 3), g_taps.luma[bipred][K.fx][0], g_taps.luma[bipred][K.fx][1], v01, v23, v45,
                    ny, false);
  }
  {
    const int cvt = g_taps.chroma[K.cfy];
    chroma_rows<0, 4>(c, (uint32_t)(cwb & 3), g_taps.chroma[K.cfx], (tap8(cvt, 0) & 0xffff) | (tap8(cvt, 1) << 16),
                      (tap8(cvt, 2) & 0xffff) | (tap8(cvt, 3) << 16), nc, false);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const bool m = i < 4 ? m0 : m1;
    ty[i] = m ? (acc ? avg_bytes(ty[i], ny[i]) : ny[i]) : ty[i];  // bi-pred: truncating average with pass 0
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const bool m = i < 2 ? m0 : m1;
    tc[i] = m ? (acc ? avg_bytes(tc[i], nc[i]) : nc[i]) : tc[i];
  }
  it.pend &= ~((m0 ? 1u : 0u) | (m1 ? 2u : 0u));
}

// ---- fast-path filters (the half's plan: one key for every cell) ----
// The fast path's dot products: the builtins (v_dot4c / v_dot2c, each chain
// seeded by one v_mov).  The VOP3P forms written as inline asm were tried:
// v_dot4_i32_i8 so written gave wrong, run-to-run varying sums in this kernel
// (tools/probes/luma_fast_check.hip) and the v_dot2 form measured no faster.
__device__ __forceinline__ int vdot4(uint32_t a, int taps, int acc) { return dot4(a, taps, acc); }
__device__ __forceinline__ int vdot2(uint32_t a, int taps, int acc) { return dot2(a, taps, acc); }
__device__ __forceinline__ int vdot2_0(uint32_t a, int taps) { return dot2(a, taps, 0); }

// The rounding constant of the 2-D filters folded into the horizontal sums:
// every tap set sums to 64, so adding HB to each H' adds 64 * HB = MC_RND to
// every vertical sum, and H' + HB stays inside int16 for every table (luma
// [-12017, 11953] + 8224, chroma [-10232, 10168] + 8224).
#define HB 8224

// Tap words of a k-tap filter (int8 taps packed from byte 0) placed at byte
// offset o of a 12-byte window: word w holds the taps that land on bytes
// 4w .. 4w + 3 (zeros elsewhere).  Uniform: scalar arithmetic.
__device__ __forceinline__ void shifted_taps(unsigned long long t48, int o, int &w0, int &w1, int &w2) {
  const unsigned long long lo = t48 << (8 * o);
  w0 = (int)(uint32_t)lo;
  w1 = (int)(uint32_t)(lo >> 32);
  w2 = o > 2 ? (int)(uint32_t)(t48 >> (64 - 8 * o)) : 0;
}

// clip255(x >> 6) of four sums packed as bytes (|x| < 2^15): int16 pairs, a
// packed shift, saturation to u8 -- the one-dimensional filters' output (the
// rounding 32 is in the sums' seed).
typedef short i16x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack4_sh6_u8(int a, int b, int c, int d) {
  const i16x2v sh = {6, 6};
  const i16x2v ab = __builtin_amdgcn_cvt_pk_i16(a, b) >> sh, cd = __builtin_amdgcn_cvt_pk_i16(c, d) >> sh;
  return __builtin_amdgcn_perm(sat_u8x2_pk(__builtin_bit_cast(uint32_t, cd)),
                               sat_u8x2_pk(__builtin_bit_cast(uint32_t, ab)), 0x05040100u);
}

// Eight luma rows of the lane's 4-px column, 6x6 taps.  `base` = the window
// byte of strip row -2, column -2 rounded down to a dword; SH = the byte offset
// of column -2 in it (uniform: the dispatcher switches on it).  Horizontal: dot4
// per pixel on the unshifted dwords with per-pixel shifted tap words (no
// v_alignbyte); pixel j's taps cover window bytes SH + j .. SH + j + 5, so d0 is
// read only for SH + j <= 3 and d2 only for SH + j >= 3 -- 9 dot4 per row of 4 px
// instead of 12.  Vertical: three dot2 per pixel on (H'[r], H'[r+1]) pairs.
// FX0 / FY0: the horizontal / vertical fraction is 0, i.e. the taps are
// {0, 0, 64, 0, 0, 0} (common/inter_prediction.c:47-59): one dot4 per pixel for
// the horizontal pass / no vertical pass at all ((64 x 64 x p + 2048) >> 12 =
// (64 x H + 2048) >> 12 = (H + 32) >> 6 exactly, so the one-dimensional forms
// are the same integers as the two-dimensional filter).
template <int SH, bool FX0, bool FY0>
__device__ __forceinline__ void luma8_fast(const uint8_t *base, unsigned long long th48, int v01, int v23,
                                           int v45, uint32_t out[8], bool acc, bool k0 = true, bool k1 = true) {
  int T[4][3];
#pragma unroll
  for (int j = 0; j < 4; j++) shifted_taps(th48, SH + j, T[j][0], T[j][1], T[j][2]);
  const int hb = HB;  // in a VGPR: the chains' seed (one scalar operand per instruction)
  auto hsum = [&](int r, int hc[4]) {  // strip row r: H' + HB of the lane's 4 pixels
    const uint32_t *q = (const uint32_t *)(base + (r + 2) * WL_P);
    const uint32_t d0 = q[0], d1 = q[1], d2 = q[2];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (FX0) {  // the one non-zero tap (64) sits on window byte SH + j + 2
        const int w = (SH + j + 2) >> 2;
        hc[j] = vdot4(w == 0 ? d0 : (w == 1 ? d1 : d2), T[j][w], hb);
      } else {
        int a = hb;
        if (SH + j >= 3) a = vdot4(d2, T[j][2], a);
        a = vdot4(d1, T[j][1], a);
        if (SH + j <= 3) a = vdot4(d0, T[j][0], a);
        hc[j] = a;
      }
    }
  };
  if (FY0) {  // horizontal only: rows 0..7
#pragma unroll
    for (int i = 0; i < 8; i++) {
      int hc[4];
      hsum(i, hc);
      const uint32_t o = pack4_sh6_u8(hc[0], hc[1], hc[2], hc[3]);
      if (i < 4 ? k0 : k1) out[i] = acc ? avg_bytes(out[i], o) : o;
    }
    return;
  }
  int hp[4];
  uint32_t pa[6][4];
  auto hrow = [&](int r) {  // strip row r (-2 .. 10) -> P(r - 1)
    int hc[4];
    hsum(r, hc);
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (r > -2) pa[(r + 5) % 6][j] = pack_lo16(hp[j], hc[j]);
      hp[j] = hc[j];
    }
  };
#pragma unroll
  for (int r = -2; r <= 2; r++) hrow(r);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    hrow(i + 3);
    int v[4];
#pragma unroll
    for (int j = 0; j < 4; j++)
      v[j] = vdot2(pa[(i + 2 + 6) % 6][j], v45, vdot2(pa[(i + 6) % 6][j], v23, vdot2_0(pa[(i - 2 + 6) % 6][j], v01)));
    const uint32_t o = pack4_hi16_u8(v[0], v[1], v[2], v[3]);  // vertical taps x 16
    if (i < 4 ? k0 : k1) out[i] = acc ? avg_bytes(out[i], o) : o;  // k0 / k1: the segment's key matches
  }
}

// The (2,2) position (common/inter_prediction.c:145-157), fast form: the
// kernel K[i][j] = u_i + u_j (rows / columns -1..2, u = [0 1 1 0]) is
//   S(o) = H2(o-1) + H4(o) + H4(o+1) + H2(o+2),
// H4 = the [1 2 2 1] and H2 = the [0 1 1 0] horizontal sums over columns -1..2
// (dot4 with compile-time shifted tap words on the biased bytes: H4' = H4 - 768,
// H2' = H2 - 256, and H2's seed 1028 carries the bias and the rounding:
// 2 x (256 + 1028) + 2 x 768 ... = S + 8 exactly).  Output (S + 8) >> 4 with
// the rows as int16 pairs of pixels: packed adds and shifts (|S| < 2^13).
template <int SH>
__device__ __forceinline__ void luma8_ctr(const uint8_t *base, uint32_t out[8], bool acc, bool k0 = true,
                                          bool k1 = true) {
  constexpr unsigned long long t4 = 0x0000010202010000ull >> 8;  // {0, 1, 2, 2, 1, 0} at window bytes 0..5
  constexpr unsigned long long t2 = 0x0000000101000000ull >> 8;  // {0, 0, 1, 1, 0, 0}
  auto word = [](unsigned long long t, int o, int w) -> int {
    const unsigned long long lo = t << (8 * o);
    return w == 0 ? (int)(uint32_t)lo : (w == 1 ? (int)(uint32_t)(lo >> 32) : (o > 2 ? (int)(uint32_t)(t >> (64 - 8 * o)) : 0));
  };
  i16x2v p4[4][2], p2[4][2];  // rows as (pixel 0, 1), (pixel 2, 3) pairs, ring by strip row
  auto hrow = [&](int r) {  // strip row r (-1 .. 9)
    const uint32_t *q = (const uint32_t *)(base + (r + 2) * WL_P);
    const uint32_t d[3] = {q[0], q[1], q[2]};
    int h4[4], h2[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      int a = 0, c = 1028;
#pragma unroll
      for (int w = (SH + j + 1) >> 2; w <= (SH + j + 4) >> 2; w++) a = vdot4(d[w], word(t4, SH + j, w), a);
#pragma unroll
      for (int w = (SH + j + 2) >> 2; w <= (SH + j + 3) >> 2; w++) c = vdot4(d[w], word(t2, SH + j, w), c);
      h4[j] = a;
      h2[j] = c;
    }
    const int k = (r + 4) & 3;
    p4[k][0] = __builtin_amdgcn_cvt_pk_i16(h4[0], h4[1]);
    p4[k][1] = __builtin_amdgcn_cvt_pk_i16(h4[2], h4[3]);
    p2[k][0] = __builtin_amdgcn_cvt_pk_i16(h2[0], h2[1]);
    p2[k][1] = __builtin_amdgcn_cvt_pk_i16(h2[2], h2[3]);
  };
#pragma unroll
  for (int r = -1; r <= 1; r++) hrow(r);
  const i16x2v sh = {4, 4};
#pragma unroll
  for (int o = 0; o < 8; o++) {
    hrow(o + 2);
    uint32_t hv[2];
#pragma unroll
    for (int e = 0; e < 2; e++) {
      const i16x2v s = (p2[(o + 3) & 3][e] + p4[(o + 4) & 3][e]) + (p4[(o + 5) & 3][e] + p2[(o + 6) & 3][e]);
      hv[e] = sat_u8x2_pk(__builtin_bit_cast(uint32_t, s >> sh));
    }
    const uint32_t v = __builtin_amdgcn_perm(hv[1], hv[0], 0x05040100u);
    if (o < 4 ? k0 : k1) out[o] = acc ? avg_bytes(out[o], v) : v;
  }
}

// Four chroma rows of the lane's 2-px column, U and V (4x4 taps).  sh = byte
// offset of column -1 in the first dword (uniform).
// CY0: the vertical fraction is 0 ({0, 64, 0, 0}): rows 0..3 only, no vertical
// pass ((H + 32) >> 6, the same integers, as for luma).
template <bool CY0>
__device__ __forceinline__ void chroma4_fast(const uint8_t *bu, const uint8_t *bv, int sh, unsigned long long tc32,
                                             int v01, int v23, uint32_t out[4], bool acc, bool k0 = true,
                                             bool k1 = true) {
  int T[2][2];
#pragma unroll
  for (int j = 0; j < 2; j++) {
    const unsigned long long x = tc32 << (8 * (sh + j));
    T[j][0] = (int)(uint32_t)x;
    T[j][1] = (int)(uint32_t)(x >> 32);
  }
  const int hb = HB;
  auto hsum = [&](int r, int hu[2], int hv[2]) {  // strip row r: H' + HB of the lane's 2 U and 2 V pixels
    const uint32_t *qu = (const uint32_t *)(bu + (r + 1) * WC_P), *qv = (const uint32_t *)(bv + (r + 1) * WC_P);
    const uint32_t u0 = qu[0], u1 = qu[1], w0 = qv[0], w1 = qv[1];
#pragma unroll
    for (int j = 0; j < 2; j++) {
      hu[j] = vdot4(u0, T[j][0], vdot4(u1, T[j][1], hb));
      hv[j] = vdot4(w0, T[j][0], vdot4(w1, T[j][1], hb));
    }
  };
  if (CY0) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
      int hu[2], hv[2];
      hsum(i, hu, hv);
      const uint32_t uv = pack4_sh6_u8(hu[0], hu[1], hv[0], hv[1]);
      if (i < 2 ? k0 : k1) out[i] = acc ? avg_bytes(out[i], uv) : uv;
    }
    return;
  }
  int pu_prev[2], pv_prev[2];
  uint32_t pu[4][2], pv[4][2];
  auto hrow = [&](int r) {  // strip row r (-1 .. 5)
    int hu[2], hv[2];
    hsum(r, hu, hv);
#pragma unroll
    for (int j = 0; j < 2; j++) {
      if (r > -1) {
        pu[(r + 3) % 4][j] = pack_lo16(pu_prev[j], hu[j]);
        pv[(r + 3) % 4][j] = pack_lo16(pv_prev[j], hv[j]);
      }
      pu_prev[j] = hu[j];
      pv_prev[j] = hv[j];
    }
  };
#pragma unroll
  for (int r = -1; r <= 1; r++) hrow(r);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    hrow(i + 2);
    int au[2], av[2];
#pragma unroll
    for (int j = 0; j < 2; j++) {
      au[j] = vdot2(pu[(i + 1) % 4][j], v23, vdot2_0(pu[(i + 3) % 4][j], v01));
      av[j] = vdot2(pv[(i + 1) % 4][j], v23, vdot2_0(pv[(i + 3) % 4][j], v01));
    }
    const uint32_t uv = pack4_hi16_u8(au[0], au[1], av[0], av[1]);  // vertical taps x 16
    if (i < 2 ? k0 : k1) out[i] = acc ? avg_bytes(out[i], uv) : uv;
  }
}

// The half's plan says every cell has key K in this pass: filter straight
// into the prediction registers (no per-segment key match).
__device__ __forceinline__ void filter_all(const RefWin &w, const Key &K, int bipred, int x0, uint32_t ty[8],
                                           uint32_t tc[4], bool acc, bool k0 = true, bool k1 = true) {
  const ReconGeo *G = RECON_GEO();
  auto luma_word = [&](int b, int f, int wd) { return G->tl[b][f][wd]; };
  auto chroma_word = [&](int f) { return G->tc[f]; };
  const int lane = threadIdx.x, cc = LCC(lane), gr = LGR(lane);
  const int lwb = 4 * cc + ((x0 - 2 + K.dx) & 15);
  const int cwb = 2 * cc + (((x0 >> 1) - 1 + K.cdx) & 15);
  const LdsLuma l{w.y + 8 * gr * WL_P + (lwb & ~3)};
  const LdsChroma c{w.u + 4 * gr * WC_P + (cwb & ~3), w.v + 4 * gr * WC_P + (cwb & ~3)};
  const uint8_t *lb = w.y + 8 * gr * WL_P + (lwb & ~3);
  const int lsh = lwb & 3;  // uniform
  if (K.fx == 2 && K.fy == 2) {
    switch (lsh) {
      case 0: luma8_ctr<0>(lb, ty, acc, k0, k1); break;
      case 1: luma8_ctr<1>(lb, ty, acc, k0, k1); break;
      case 2: luma8_ctr<2>(lb, ty, acc, k0, k1); break;
      default: luma8_ctr<3>(lb, ty, acc, k0, k1); break;
    }
  } else {
    int v01, v23, v45;
    tap_pairs6(luma_word(bipred, K.fy, 0), luma_word(bipred, K.fy, 1), v01, v23, v45, 16);
    const unsigned long long th48 = (unsigned long long)(uint32_t)luma_word(bipred, K.fx, 0) |
                                    ((unsigned long long)(uint32_t)(luma_word(bipred, K.fx, 1) & 0xffff) << 32);
#define LUMA8(SHv, X0, Y0) luma8_fast<SHv, X0, Y0>(lb, th48, v01, v23, v45, ty, acc, k0, k1)
#define LUMA8_SH(X0, Y0)            \
  switch (lsh) {                    \
    case 0: LUMA8(0, X0, Y0); break; \
    case 1: LUMA8(1, X0, Y0); break; \
    case 2: LUMA8(2, X0, Y0); break; \
    default: LUMA8(3, X0, Y0); break; \
  }
    if (K.fy == 0) {
      if (K.fx == 0) {
        LUMA8_SH(true, true)
      } else {
        LUMA8_SH(false, true)
      }
    } else if (K.fx == 0) {
      LUMA8_SH(true, false)
    } else {
      LUMA8_SH(false, false)
    }
#undef LUMA8_SH
#undef LUMA8
  }
  const int cvt = chroma_word(K.cfy);
  const uint8_t *cu = w.u + 4 * gr * WC_P + (cwb & ~3), *cv = w.v + 4 * gr * WC_P + (cwb & ~3);
  const unsigned long long tc32 = (unsigned long long)(uint32_t)chroma_word(K.cfx);
  const int c01 = tap_pair(tap8(cvt, 0), tap8(cvt, 1), 16), c23 = tap_pair(tap8(cvt, 2), tap8(cvt, 3), 16);
  if (K.cfy == 0) chroma4_fast<true>(cu, cv, cwb & 3, tc32, c01, c23, tc, acc, k0, k1);
  else chroma4_fast<false>(cu, cv, cwb & 3, tc32, c01, c23, tc, acc, k0, k1);  // vertical taps x 16
  (void)l;
  (void)c;
}

// Waves whose items need several keys: every item straight from the ring,
// per-lane keys (one pass, no per-key staging round trips).
__device__ __forceinline__ void filter_direct(const FrameCtx &f, __amdgpu_buffer_rsrc_t ring, int bipred, int x0,
                                              int y0, Items &it, uint32_t ty[8], uint32_t tc[4], bool acc) {
  const int lane = threadIdx.x, cc = LCC(lane), gr = LGR(lane);
  const Key K0 = make_key(it.mv[0], it.slot[0]), K1 = make_key(it.mv[1], it.slot[1]);
  const bool m0 = it.pend & 1, m1 = (it.pend >> 1) & 1;
  const bool same = it.mv[0] == it.mv[1] && it.slot[0] == it.slot[1];
  const int uvd = (int)(f.offv - f.offu);
  auto lo = [&](const Key &K) {
    return (int)((long long)K.slot * f.slot_bytes + f.offy + (long long)(y0 + 8 * gr + K.dy) * f.sy + x0 + 4 * cc - 2 + K.dx);
  };
  auto co = [&](const Key &K) {
    return (int)((long long)K.slot * f.slot_bytes + f.offu + (long long)((y0 >> 1) + 4 * gr + K.cdy) * f.sc +
                 (x0 >> 1) + 2 * cc - 1 + K.cdx);
  };
  const int l0 = lo(K0), l1 = lo(K1), c0 = co(K0), c1 = co(K1);
  const GlobLuma g0{ring, l0 & ~3, f.sy}, g1{ring, l1 & ~3, f.sy};
  const GlobChroma h0{ring, c0 & ~3, uvd, f.sc}, h1{ring, c1 & ~3, uvd, f.sc};
  filter_items(m0, m1, g0, g1, (uint32_t)(l0 & 3), (uint32_t)(l1 & 3), h0, h1, (uint32_t)(c0 & 3), (uint32_t)(c1 & 3), K0,
               K1, same, bipred, ty, tc, acc);
  it.pend = 0;
}

// clip255(pixel + residual) of four pixels (bytes of p) and their int16
// residuals (a.x = r0 | r1 << 16, a.y = r2 | r3 << 16): the pixels widened to
// int16 pairs (one byte permute per pair), a saturating packed add, then
// v_sat_pk_u8_i16 -- 7 instructions instead of 4 x (extract, add, clamp,
// insert).  Exact: a sum outside int16 saturates to a bound, which clips to
// the same 0 / 255.
__device__ __forceinline__ uint32_t add_res4v(uint32_t p, uint2 a) {
  const uint32_t pl = __builtin_amdgcn_perm(0u, p, 0x0c010c00u), ph = __builtin_amdgcn_perm(0u, p, 0x0c030c02u);
  uint32_t sl, sh;
  asm("v_pk_add_i16 %0, %1, %2 clamp" : "=v"(sl) : "v"(pl), "v"(a.x));
  asm("v_pk_add_i16 %0, %1, %2 clamp" : "=v"(sh) : "v"(ph), "v"(a.y));
  return __builtin_amdgcn_perm(sat_u8x2_pk(sh), sat_u8x2_pk(sl), 0x05040100u);
}
__device__ __forceinline__ uint32_t add_res4(uint32_t p, const int16_t *__restrict__ r) {
  return add_res4v(p, *(const uint2 *)r);
}
__device__ __forceinline__ uint32_t add_res2(uint32_t p, const int16_t *__restrict__ r) {
  const uint32_t a = *(const uint32_t *)r;
  return put_byte(clip255((int)(p & 255) + (int)(int16_t)(a & 0xffff)), 0) |
         put_byte(clip255((int)((p >> 8) & 255) + (int)(int16_t)(a >> 16)), 1);
}

// Stage key K's window and filter it into (ty, tc): every lane filters, lanes
// with `mine` keep the result (bi-pred pass 1: truncating average with pass 0).
__device__ __forceinline__ void plan_pass(ReconLds &L, const FrameCtx &f, __amdgpu_buffer_rsrc_t ring, const Key &K,
                                          int x0, int y0, uint32_t ty[8], uint32_t tc[4], bool acc, bool mine) {
  WinLoad W;
  win_issue(W, f, ring, K, x0, y0);
  wave_lds_sync();  // the previous pass's reads of the window are done
  win_commit(W, L.win);
  wave_lds_sync();
  filter_all(L.win, K, f.bipred, x0, ty, tc, acc, mine, mine);
}

#ifndef RECON_RES_PREFETCH
#define RECON_RES_PREFETCH 1
#endif
#ifndef RECON_WPE
#define RECON_WPE 1
#endif
__global__ __launch_bounds__(64, RECON_WPE) void k_recon(const FrameBatch fb_, const ReconGeo g,
                                                           unsigned long long *__restrict__ dbg) {
  const FrameCtx *__restrict__ F = FRAME_BATCH_CTX();
  __shared__ ReconLds L;
  const int lane = threadIdx.x;
  // Flat grid (capi.hip): blocks [0, nfr x maxslow) take the frames' slow-list
  // entries (frame-interleaved, so every frame's multi-key units start first);
  // then each frame's NU blocks walk its units in XCD-major order --
  // workgroup b runs on XCD b % 8 (round-robin dispatch), so each XCD gets a
  // contiguous band of slice rows and vertical neighbours share their reference
  // rows in that XCD's L2.  Speed only, never correctness.
  const int W0 = F[0].W;
  const int sbw = (W0 + 63) >> 6, np = g.np, nu = g.nu, NU = g.NU;
  const int nslow = g.nfr * g.maxslow;
  int fi, u;
  bool listed = false;
  if ((int)blockIdx.x < nslow) {
    const int idx = recon_div(blockIdx.x, g.mnfr);
    fi = blockIdx.x - idx * g.nfr;
    const FrameCtx &f = F[fi];
    if (!f.slow || f.nblocks <= 0 || idx >= f.nslow) return;
    u = (int)f.slow[idx];
    if (u >= nu) return;  // (the host builder never lists one)
    listed = true;
  } else {
    const int b = blockIdx.x - nslow;
    fi = recon_div(b, g.mNU);
    const int loc = b - fi * NU, per = NU >> 3;
    u = (loc & 7) * per + (loc >> 3);
    if (u >= nu) return;
  }
  u = __builtin_amdgcn_readfirstlane(u);  // uniform (the scalar loads below need it in SGPRs)
  fi = __builtin_amdgcn_readfirstlane(fi);
  const FrameCtx &f = F[fi];
  {  // every frame-context word the kernel reads, fetched together: one scalar-load round trip
     // instead of a chain of them spread over the branches below (the empty asm needs them all)
    const uint8_t *a0 = f.slots, *a1 = f.cy, *a2 = f.edge;
    const uint4 *a3 = f.hplan;
    const int16_t *a4 = f.resid;
    const long long b0 = f.slot_bytes, b1 = f.ring_bytes, b2 = f.offy, b3 = f.offu, b4 = f.offv;
    const int c0 = f.nblocks, c1 = f.band0, c2 = f.band1, c3 = f.gen, c4 = f.sy, c5 = f.sc, c6 = f.bipred, c7 = f.W,
              c8 = f.H, c9 = f.ewy, c10 = f.ewc, c11 = f.nsbrows;
    asm volatile("" ::"s"(a0), "s"(a1), "s"(a2), "s"(a3), "s"(a4), "s"(b0), "s"(b1), "s"(b2), "s"(b3), "s"(b4), "s"(c0),
                 "s"(c1), "s"(c2), "s"(c3), "s"(c4), "s"(c5), "s"(c6), "s"(c7), "s"(c8), "s"(c9), "s"(c10), "s"(c11),
                 "s"(dbg));
  }
  if (f.nblocks <= 0) return;
  if (fi) dbg = nullptr;
  int16_t *__restrict__ resid = f.resid;
  // debug only (null in the product path): s_memrealtime stamps, 8 u64 per unit of frame 0
  unsigned long long *stamp = dbg ? dbg + u * 8 : nullptr;
#define STAMP(i) \
  if (stamp && lane == 0) stamp[i] = __builtin_amdgcn_s_memrealtime();
  STAMP(0);
  if (stamp && lane == 0) {  // placement: HW_ID (wave, simd, cu, sh, se) | XCC_ID << 32
    const unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
    const unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));
    stamp[7] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
  }
  const int srow = recon_div(u, g.mnp), pr = u - srow * np;  // slice row (4 per SB row), SB pair
  const int sby = srow >> 2, qtr = srow & 3, h = qtr >> 1;
  if (sby < f.band0 || sby >= f.band1) return;  // another shard's rows (row-band sharding)
  const int cs = f.W >> 2;
  const int x0 = 128 * pr, y0 = 16 * srow, cc = LCC(lane), gr = LGR(lane);
  const bool bex = 2 * pr + 1 < sbw;  // the pair's right SB exists
  const bool last = qtr == 3;         // the unit holds SB row 63: the edge rows k_intra reads

  // ---- fast path: the unit's planned halves (k_frame_prep: one 64x64 inter
  // CU, one key per pass) -- no per-cell resolution (P0): scalar loads, then
  // straight to the window staging ----
  // The halves' plan records: current (tag == gen) and planned, current and
  // tagged multi-key (PLAN_SLOW), or not current -- with a slow list, a half
  // with no inter pixels (intra only, or below the frame).  With a list, the
  // planned-order workgroup reconstructs the unit's planned halves (a multi-key
  // or empty neighbour half is masked) and the list's workgroup the multi-key
  // halves on the per-cell path (the planned neighbour masked); without one,
  // a unit whose two halves are not both planned takes the per-cell path whole.
  bool keep_a = true, keep_b = true;  // per-cell path: the halves whose cells it reconstructs
  if (f.hplan) {
    typedef unsigned u32x16 __attribute__((ext_vector_type(16)));
    u32x16 pv;  // plans of halves hsb and hsb + 2 (scalar, uniform loads through the constant cache)
    const int hsb = 2 * (sby * sbw + 2 * pr) + h;
    asm volatile("s_load_dwordx16 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(pv) : "s"(f.hplan + hsb) : "memory");
    STAMP(1);
    const uint4 pa = make_uint4(pv[0], pv[1], pv[2], pv[3]);
    const uint4 pb = bex ? make_uint4(pv[8], pv[9], pv[10], pv[11]) : pa;
    const bool cura = (int)pa.w == f.gen, curb = bex && (int)pb.w == f.gen;
    const bool sla = cura && (pa.y & PLAN_SLOW), slb = curb && (pb.y & PLAN_SLOW);
    bool doa, dob;  // halves this workgroup reconstructs on the planned path
    if (f.slow) {
      if (listed) {
        keep_a = sla;
        keep_b = slb;
        doa = dob = false;
      } else {
        doa = cura && !sla;
        dob = curb && !slb;
        if (!doa && !dob) return;  // nothing planned: empty, or the list's workgroup has it
      }
    } else {
      doa = cura && (curb || !bex);
      dob = doa && bex;
    }
    if (doa || dob) {
      const __amdgpu_buffer_rsrc_t ring =
          __builtin_amdgcn_make_buffer_rsrc((void *)f.slots, 0, (int)f.ring_bytes, 0x00020000);
      const unsigned ma = doa ? pa.y : 0u, mb = dob ? pb.y : 0u;
#if RECON_RES_PREFETCH
      if ((ma | mb) & (CELL_RES(0) | CELL_RES(1) | CELL_RES(2))) {
        // The unit's residual lines into L2 now, so the reads after the filter
        // hit there instead of waiting on HBM: one dword per 128-B line (luma
        // rows are 2 lines, chroma rows 1), written to LDS the fast path does
        // not use (buffer_load ... lds holds no register); out-of-range
        // offsets read nothing (buffer bounds).  Lanes 0-31 luma, 32-47 U/V.
        typedef __attribute__((address_space(3))) void lds_void;
        const int npx = f.W * f.H;
        const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc((void *)resid, 0, 3 * npx, 0x00020000);
        unsigned off = 0xffffffffu;
        if (lane < 32) {
          off = 2u * (unsigned)((y0 + (lane >> 1)) * f.W + x0 + 64 * (lane & 1));
        } else if (lane < 48) {
          const int wc = f.W >> 1;
          off = 2u * (unsigned)(npx + ((lane >> 3) & 1) * (npx >> 2) + ((y0 >> 1) + (lane & 7)) * wc + (x0 >> 1));
        }
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rr, (lds_void *)(void *)L.mv0, 4, off, 0, 0, 0);
      }
#endif
      const bool mine_a = cc < 16;  // filter lanes: columns of the left SB
      uint32_t ly[8], lc[4];
      {  // pass 0: mv0 (one window when both SBs share the key, else one per SB)
        const Key KA = make_key((int)pa.x, (int)(ma & 255)), KB = make_key((int)pb.x, (int)(mb & 255));
        STAMP(2);
        if (doa && dob && KA.mv == KB.mv && KA.slot == KB.slot) {
          plan_pass(L, f, ring, KA, x0, y0, ly, lc, false, true);
        } else {
          if (doa) plan_pass(L, f, ring, KA, x0, y0, ly, lc, false, mine_a);
          if (dob) plan_pass(L, f, ring, KB, x0, y0, ly, lc, false, !mine_a);
        }
        STAMP(4);
      }
      const bool bia = ma & CELL_BI, bib = mb & CELL_BI;
      if (bia || bib) {  // pass 1: mv1 of the bi-pred SB(s), truncating average with pass 0
        const Key KA = make_key((int)pa.z, (int)((ma >> 8) & 255)), KB = make_key((int)pb.z, (int)((mb >> 8) & 255));
        if (bia && bib && KA.mv == KB.mv && KA.slot == KB.slot) {
          plan_pass(L, f, ring, KA, x0, y0, ly, lc, true, true);
        } else {
          if (bia) plan_pass(L, f, ring, KA, x0, y0, ly, lc, true, mine_a);
          if (bib) plan_pass(L, f, ring, KB, x0, y0, ly, lc, true, !mine_a);
        }
      }
      STAMP(3);
      // ---- residual + stores: the prediction goes through LDS (the window is
      // free now) so each lane holds 16 contiguous bytes of one row -- three
      // 16-byte stores per lane: the luma rows as whole 128-B lines (row pixel 0
      // is line-aligned, capi.hip), the chroma rows as 64-B segments.  The
      // store tail is bound by store instructions and the lines they touch ----
      wave_lds_sync();
      uint8_t *const ty = L.win.y, *const tc = L.win.y + 2048;  // 16 x 128 B luma; 8 x 64 B U, then V
#pragma unroll
      for (int i = 0; i < 8; i++) *(uint32_t *)(ty + (8 * gr + i) * 128 + 4 * cc) = ly[i];
#pragma unroll
      for (int i = 0; i < 4; i++) {
        *(uint16_t *)(tc + (4 * gr + i) * 64 + 2 * cc) = (uint16_t)lc[i];
        *(uint16_t *)(tc + 512 + (4 * gr + i) * 64 + 2 * cc) = (uint16_t)(lc[i] >> 16);
      }
      wave_lds_sync();
      uint4 py0 = *(const uint4 *)(ty + 16 * lane), py1 = *(const uint4 *)(ty + 1024 + 16 * lane);
      uint4 pc = *(const uint4 *)(tc + 16 * lane);
      const int r = lane >> 3, xl = x0 + 16 * (lane & 7);  // luma: rows r and r + 8 of the unit
      const int pl1 = lane >> 5, rc = (lane & 31) >> 2;     // chroma: plane U / V, row rc
      const int xcl = (x0 >> 1) + 16 * (lane & 3), yc = (y0 >> 1) + rc;
      const unsigned mly = (lane & 4) ? mb : ma, mlc = (lane & 2) ? mb : ma;  // the SB of the lane's chunk
      if (mly & CELL_RES(0)) {
        const int16_t *rY = resid;
#pragma unroll
        for (int k = 0; k < 2; k++) {
          const int y = y0 + r + 8 * k;
          if (y >= f.H) continue;
          uint4 &p = k ? py1 : py0;
          const int16_t *q = rY + (long long)y * f.W + xl;  // 16-B aligned: W % 8 == 0, xl % 16 == 0
          if (xl < f.W) {  // (then xl + 8 <= W: all of the first 8 pixels)
            const uint4 a = *(const uint4 *)q;
            p.x = add_res4v(p.x, make_uint2(a.x, a.y));
            p.y = add_res4v(p.y, make_uint2(a.z, a.w));
          }
          if (xl + 8 < f.W) {
            const uint4 a = *(const uint4 *)(q + 8);
            p.z = add_res4v(p.z, make_uint2(a.x, a.y));
            p.w = add_res4v(p.w, make_uint2(a.z, a.w));
          }
        }
      }
      if ((mlc & CELL_RES(1 + pl1)) && yc < (f.H >> 1)) {
        const int wc = f.W >> 1;
        const int16_t *q = resid + (long long)f.W * f.H + (long long)pl1 * wc * (f.H >> 1) + (long long)yc * wc + xcl;
        if (xcl < wc) pc.x = add_res4(pc.x, q);
        if (xcl + 4 < wc) pc.y = add_res4(pc.y, q + 4);
        if (xcl + 8 < wc) pc.z = add_res4(pc.z, q + 8);
        if (xcl + 12 < wc) pc.w = add_res4(pc.w, q + 12);
      }
      // Stores through a descriptor over the current slot: one lane offset per
      // plane, the second luma row set in the scalar offset.  A unit at the
      // frame's bottom / right edge stores its rows / columns past the edge into
      // the slot's padding, which k_pad rewrites (W, H multiples of 8; padding
      // >= 48); the columns of a right SB past the last one are not stored.
      const __amdgpu_buffer_rsrc_t cur =
          __builtin_amdgcn_make_buffer_rsrc((void *)(f.cy - f.offy), 0, (int)f.slot_bytes, 0x00020000);
      const int oy = (int)f.offy + (y0 + r) * f.sy + xl;
      const int offu = __builtin_amdgcn_readfirstlane((int)f.offu), offv = __builtin_amdgcn_readfirstlane((int)f.offv);
      const int oc = (pl1 ? offv : offu) + yc * f.sc + xcl;  // (a select of scalars, not a per-lane load of the field)
      typedef unsigned v4u __attribute__((ext_vector_type(4)));
#if RECON_PROBE == 3  // timing probe: no pixel stores (wrong output)
      if (f.W > 0) return;
#endif
      const bool sty = (lane & 4) ? dob : doa, stc = (lane & 2) ? dob : doa;  // the lane's chunks' halves are ours
      if (sty) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, py0), cur, oy, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, py1), cur, oy, 8 * f.sy, 0);
      }
      if (stc) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, pc), cur, oc, 0, 0);
      if (last) {  // SB row 63 / chroma SB row 31: the edge rows k_intra's next SB row reads
        if (sty && r == 7 && y0 + 15 < f.H && xl < f.W)
          *(uint4 *)(f.edge + (long long)sby * f.ewy + EDGE_MARGIN + xl) = py1;
        if (stc && rc == 7 && yc < (f.H >> 1) && xcl < (f.W >> 1))
          *(uint4 *)(f.edge + (long long)f.nsbrows * f.ewy + (long long)(pl1 * f.nsbrows + sby) * f.ewc + EDGE_MARGIN +
                     xcl) = pc;
      }
      STAMP(5);
      return;
    }
  }

#ifdef RECON_PLAN_ONLY
  if (f.W > 0) return;
#endif
  // reference lookup table (packed by the host)
  if (lane < 32) *(int *)&L.lut[4 * lane] = f.slot_lut[lane];
  if (stamp) {  // debug: the frame context's scalar loads have returned
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    STAMP(1);
  }

  // ---- P0: lane = cell row cr of 8x8 unit uu of the work unit: the two cells'
  // MC words that k_frame_prep resolved (quarter MV with the `sign` negation,
  // inter_prediction.c:78-79 / :125-126, reference slots, bi-pred, coded
  // residual per component), one 16-byte load ----
  const int uu = lane >> 1, cr = lane & 1;
  const int ur = uu >> 4, uc = uu & 15;
  const int uy = y0 + 8 * ur, ux = x0 + 8 * uc;
  const int lrow = 2 * ur + cr;  // cell row inside the unit
  uint4 mc = make_uint4(0, 0, 0, 0);
  const int cidx = ((uy >> 2) + cr) * cs + (ux >> 2);
  if (uy < f.H && ux < f.W && (uc < 8 ? keep_a : keep_b)) mc = *(const uint4 *)&f.cellmc[cidx];
  bool inter = false, bi_any = false;
#pragma unroll
  for (int c = 0; c < 2; c++) {
    const unsigned meta = c ? mc.w : mc.y;
    const int cell = lrow * 32 + 2 * uc + c;
    L.mv0[cell] = (int)(c ? mc.z : mc.x);
    L.mv1[cell] = (meta & CELL_BI) ? f.cellmv1[cidx + c] : 0;
    L.meta[cell] = meta;
    inter |= (meta & CELL_ACT) != 0;
    bi_any |= (meta & CELL_BI) != 0;
  }
  const bool any_inter = __ballot(inter) != 0, any_bi = __ballot(bi_any) != 0;
  wave_lds_sync();
  STAMP(2);
  if (!any_inter) {
    STAMP(5);
    return;
  }

  // ---- P1: prediction (pass 0: mv0; pass 1: mv1 of the bi-pred cells) ----
  const __amdgpu_buffer_rsrc_t ring =  // one descriptor over the whole ring (< 2 GiB: 32-bit offsets)
      __builtin_amdgcn_make_buffer_rsrc((void *)f.slots, 0, (int)f.ring_bytes, 0x00020000);
  uint32_t ly[8], lc[4];  // the lane's prediction: 8 luma rows x 4 px, 4 chroma rows x 2 px x (U, V)
  for (int pass = 0; pass <= (int)any_bi; pass++) {
    Items it = job_items(L, pass);
    Key K;
    if (first_key(it, K)) {
      const bool m0 = (it.pend & 1) && it.mv[0] == K.mv && it.slot[0] == K.slot;
      const bool m1 = (it.pend & 2) && it.mv[1] == K.mv && it.slot[1] == K.slot;
      if (__ballot(it.pend != ((m0 ? 1u : 0u) | (m1 ? 2u : 0u))) == 0) {  // one key: one staged window
        WinLoad W;
        win_issue(W, f, ring, K, x0, y0);
        win_commit(W, L.win);
        wave_lds_sync();
        if (pass == 0) STAMP(4);
        filter_key(L.win, K, f.bipred, x0, it, ly, lc, pass != 0);
      } else {
        if (pass == 0) STAMP(4);
        filter_direct(f, ring, f.bipred, x0, y0, it, ly, lc, pass != 0);
      }
    }
    wave_lds_sync();
  }
  STAMP(3);

  // ---- P2: residual + store ----
  const int16_t *rY = resid, *rU = resid + (long long)f.W * f.H, *rV = rU + (long long)(f.W >> 1) * (f.H >> 1);
  const int x = x0 + 4 * cc, yb = y0 + 8 * gr;
  const int xc = (x0 >> 1) + 2 * cc, ycb = (y0 >> 1) + 4 * gr;
#pragma unroll
  for (int s = 0; s < 2; s++) {
    const unsigned meta = L.meta[(2 * gr + s) * 32 + cc];
    if (!(meta & CELL_ACT)) continue;
#pragma unroll
    for (int i = 4 * s; i < 4 * s + 4; i++) {
      const int y = yb + i;
      uint32_t v = ly[i];
      if (meta & CELL_RES(0)) v = add_res4(v, rY + (long long)y * f.W + x);
      *(uint32_t *)(f.cy + (long long)y * f.sy + x) = v;
      if (i == 7 && last && gr == 1)  // SB row 63: the edge row k_intra's next SB row reads
        *(uint32_t *)(f.edge + (long long)sby * f.ewy + EDGE_MARGIN + x) = v;
    }
#pragma unroll
    for (int i = 2 * s; i < 2 * s + 2; i++) {
      const int y = ycb + i;
      uint32_t vu = lc[i] & 0xffff, vv = lc[i] >> 16;
      if (meta & CELL_RES(1)) vu = add_res2(vu, rU + (long long)y * (f.W >> 1) + xc);
      if (meta & CELL_RES(2)) vv = add_res2(vv, rV + (long long)y * (f.W >> 1) + xc);
      *(uint16_t *)(f.cu + (long long)y * f.sc + xc) = (uint16_t)vu;
      *(uint16_t *)(f.cv + (long long)y * f.sc + xc) = (uint16_t)vv;
      if (i == 3 && last && gr == 1) {  // chroma SB row 31
        uint8_t *e = f.edge + (long long)f.nsbrows * f.ewy + (long long)sby * f.ewc + EDGE_MARGIN + xc;
        *(uint16_t *)e = (uint16_t)vu;
        *(uint16_t *)(e + (long long)f.nsbrows * f.ewc) = (uint16_t)vv;
      }
    }
  }
  STAMP(5);
#undef STAMP
}
