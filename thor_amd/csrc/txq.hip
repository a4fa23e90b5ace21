// Encoder-side transform-block chain for gfx950: residual, forward transform,
// quantize, dequantize, inverse transform, reconstruction and SSD of one
// transform block per wavefront.
//
// Restates encode_and_reconstruct_block_inter / _intra's per-TU body
// (enc/encode_block.c:1434-1518): get_residual (:484-493) -> transform
// (common/transform.c:249-330, SIMD transform_simd common/common_kernels.c:
// 2176-2250) -> quantize (enc/encode_block.c:75-172, rdoq = 0) -> if cbp:
// dequantize (common/common_block.c:132-146) -> inverse_transform
// (common/transform.c:432-518) -> reconstruct_block (common/common_block.c:
// 148-156), else rec = pred; then the SSD that cost_calc sums
// (enc/encode_block.c:1218-1228).
//
// The same device functions back the per-call SIMD surface entries
// transform_simd / inverse_transform_simd (simd_surface.hip).
//
// Everything here is integer; the only floating point is cost_calc's
// (int32)(lambda * nbits + 0.5) in k_enc_cost, built with
// -ffp-contract=off so the multiply and add round separately as on x86 SSE2.
#include "common.h"

// Zigzag scans of the low-frequency corner (zigzag16 / zigzag64 / zigzag256,
// common/common_block.c:38-73): zz[raster] = scan position, iz = inverse.
struct ZigzagTables {
  uint8_t zz4[16], iz4[16], zz8[64], iz8[64], zz16[256], iz16[256];
  static constexpr void diag(int n, uint8_t *zz) {
    // anti-diagonals, alternating direction (even d: bottom-left to top-right)
    int idx = 0;
    for (int d = 0; d < 2 * n - 1; d++) {
      if (d % 2 == 0) {
        for (int i = (d < n - 1 ? d : n - 1); i >= 0 && d - i < n; i--) zz[i * n + (d - i)] = (uint8_t)idx++;
      } else {
        for (int i = (d - n + 1 > 0 ? d - n + 1 : 0); i <= d && i < n; i++) zz[i * n + (d - i)] = (uint8_t)idx++;
      }
    }
  }
  constexpr ZigzagTables() : zz4(), iz4(), zz8(), iz8(), zz16(), iz16() {
    const uint8_t z4[16] = {0, 1, 5, 6, 2, 4, 7, 12, 3, 8, 11, 13, 9, 10, 14, 15};
    for (int i = 0; i < 16; i++) zz4[i] = z4[i];
    diag(8, zz8);
    diag(16, zz16);
    for (int i = 0; i < 16; i++) iz4[zz4[i]] = (uint8_t)i;
    for (int i = 0; i < 64; i++) iz8[zz8[i]] = (uint8_t)i;
    for (int i = 0; i < 256; i++) iz16[zz16[i]] = (uint8_t)i;
  }
};
__constant__ ZigzagTables g_zz = ZigzagTables();

// gquant_table, common/common_block.c:97
__device__ __forceinline__ int quant_scale(int r) {
  return r == 0 ? 26214 : r == 1 ? 23302 : r == 2 ? 20560 : r == 3 ? 18396 : r == 4 ? 16384 : 14564;
}

// Working set of one transform block (one wavefront, ~14 KB of LDS).
struct TxLds {
  int16_t R[32 * 32];  // residual in / reconstructed residual out (row-major, stride = min(size, 32);
                       // a 64x64 TU's input is pre-summed straight into A, its output is the
                       // 32x32 inverse before the 2x2 replication)
  int16_t A[32 * 32];  // 2x2 / 4x4 pre-summed input of the 32/64 paths
  int16_t T[16 * 32];  // forward pass-1 output / inverse pass-1 output
  int C[256];          // q x q coefficients (raster), then quantised levels (raster)
  int S[256];          // scan-order levels during quantisation
  int8_t M[1024];      // 32-point DCT basis
};

__device__ __forceinline__ void tx_load_basis(TxLds &L) {
  const int lane = threadIdx.x & 63;
  *(uint4 *)&L.M[16 * lane] = *(const uint4 *)&g_dct32.v[16 * lane];
}

__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ unsigned wave_sum_u(unsigned v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// One output of the reference SIMD 8-point forward pass (transform8,
// common/common_kernels.c:1887-1967): E/O/EO butterflies in 16-bit lanes
// (wrapping), products and sums in 32 bits, stored as the low 16 bits.
__device__ __forceinline__ int fwd8_simd(const int16_t *s, int k, int shift) {
  int E[4], O[4];
#pragma unroll
  for (int m = 0; m < 4; m++) {
    E[m] = wrap16(s[m] + s[7 - m]);
    O[m] = wrap16(s[m] - s[7 - m]);
  }
  const int EO0 = wrap16(E[0] - E[3]), EO1 = wrap16(E[1] - E[2]);
  int v;
  switch (k) {
    case 0: v = 64 * E[0] + 64 * E[1] + 64 * E[2] + 64 * E[3]; break;
    case 4: v = 64 * E[0] - 64 * E[1] - 64 * E[2] + 64 * E[3]; break;
    case 2: v = 83 * EO0 + 36 * EO1; break;
    case 6: v = 36 * EO0 - 83 * EO1; break;
    case 1: v = 89 * O[0] + 75 * O[1] + 50 * O[2] + 18 * O[3]; break;
    case 3: v = 75 * O[0] - 18 * O[1] - 89 * O[2] - 50 * O[3]; break;
    case 5: v = 50 * O[0] - 89 * O[1] + 18 * O[2] + 75 * O[3]; break;
    default: v = 18 * O[0] - 50 * O[1] + 75 * O[2] - 89 * O[3]; break;
  }
  return wrap16((v + (1 << (shift - 1))) >> shift);
}

// Pre-summed input of a 64x64 TU into L.A from element accessor v(y, x):
// 4x4 sums -> 16x16 (fast) or 2x2 sums -> 32x32 (transform.c:273-307), int16 stores.
template <class V>
__device__ __forceinline__ void presum64(TxLds &L, int fast, V v) {
  const int lane = threadIdx.x & 63;
  const int f = fast ? 4 : 2, n = 64 / f;
  for (int e = lane; e < n * n; e += 64) {
    const int i = e / n, j = e - i * n;
    int s = 0;
    for (int a = 0; a < f; a++)
      for (int b = 0; b < f; b++) s += v(i * f + a, j * f + b);
    L.A[e] = (int16_t)wrap16(s);
  }
}

// Forward transform of L.R (size x size, stride size; size 64: L.A pre-summed) into L.C (q x q raster,
// q = min(size, 16)), the low-frequency corner transform / transform_simd
// compute (common/transform.c:249-330; 32/64 `fast` pre-sum 2x2 / 4x4 into a
// 16-point transform, :273-293; 64 non-fast pre-sums 2x2 into a 32-point
// transform, :294-307; stage-1 results stored as int16, :315).
__device__ void fwd_tx(TxLds &L, int size, int fast) {
  const int lane = threadIdx.x & 63;
  const int lg = ilog2i(size);
  int N = size, sh1 = lg, sh2 = lg + 5;
  const int16_t *in = L.R;
  if (size > 16 && fast) {
    N = 16;
    sh1 += 1 + (size == 64);
    sh2 = 9;
    if (size == 32) {  // 2x2 pre-sum (a 64x64 TU arrives pre-summed 4x4 in A)
      for (int e = lane; e < 256; e += 64) {
        const int i = e >> 4, j = e & 15;
        const int16_t *r = &L.R[(2 * i) * 32 + 2 * j];
        L.A[e] = (int16_t)wrap16(r[0] + r[1] + r[32] + r[33]);
      }
    }
    in = L.A;
  } else if (size == 64) {  // pre-summed 2x2 into A by the caller
    N = 32;
    sh1 = 7;
    sh2 = 10;
    in = L.A;
  }
  wave_lds_sync();
  const int q = size < 16 ? size : 16;
  if (N == 8) {  // reference SIMD butterflies (transposing passes)
    {
      const int row = lane >> 3, k = lane & 7;
      L.T[k * 8 + row] = (int16_t)fwd8_simd(&in[row * 8], k, sh1);
    }
    wave_lds_sync();
    {
      const int row = lane >> 3, k = lane & 7;
      L.C[k * 8 + row] = fwd8_simd(&L.T[row * 8], k, sh2);
    }
    wave_lds_sync();
    return;
  }
  const int step = 32 / N;
  const int add1 = 1 << (sh1 - 1), add2 = 1 << (sh2 - 1);
  for (int e = lane; e < q * N; e += 64) {  // 1st dimension, transform.c:309-316
    const int i = e / N, j = e - i * N;
    const int8_t *m = &L.M[(i * step) * 32];
    const int16_t *x = &in[j * N];
    int s = 0;
    for (int k = 0; k < N; k++) s += (int)m[k] * (int)x[k];
    L.T[i * N + j] = (int16_t)wrap16((s + add1) >> sh1);
  }
  wave_lds_sync();
  for (int e = lane; e < q * q; e += 64) {  // 2nd dimension, :319-327
    const int i = e / q, j = e - i * q;
    const int8_t *m = &L.M[(i * step) * 32];
    const int16_t *t = &L.T[j * N];
    int s = 0;
    for (int k = 0; k < N; k++) s += (int)m[k] * (int)t[k];
    L.C[i * q + j] = wrap16((s + add2) >> sh2);
  }
  wave_lds_sync();
}

// quantize, enc/encode_block.c:75-172 (rdoq = 0, the default of every
// configuration, enc/strings.c:331): L.C (q x q raster) -> quantised levels in
// L.C (raster).  Returns cbp.
__device__ int quant_tu(TxLds &L, int qp, int size, int type) {
  const int lane = threadIdx.x & 63;
  const int intra = (type >> 1) & 1, chroma = type & 1;
  const int lg = ilog2i(size), q = size < 16 ? size : 16, nq = q * q;
  const int scale = quant_scale(qp % 6), shift2 = 21 - lg + qp / 6;
  const uint8_t *iz = q == 4 ? g_zz.iz4 : (q == 8 ? g_zz.iz8 : g_zz.iz16);
  const uint8_t *zz = q == 4 ? g_zz.zz4 : (q == 8 ? g_zz.zz8 : g_zz.zz16);
  // last_pos: the highest scan position whose dead-zone level is non-zero (:104-113)
  const int offset = (intra ? 38 : -26) * (1 << (shift2 - 8));
  int lp = -1;
  for (int pos = lane; pos < nq; pos += 64) {
    const int c = L.C[iz[pos]];
    if ((abs(abs(c) * scale + offset) >> shift2) != 0) lp = pos;
  }
  const int last_pos = wave_max(lp);
  // forward scan up to last_pos (:115-131)
  const int off0 = (intra ? 102 : 51) * (1 << (shift2 - 8)), off1 = (intra ? 115 : 90) * (1 << (shift2 - 8));
  int any = 0;
  for (int pos = lane; pos < nq; pos += 64) {
    int lev = 0;
    if (pos <= last_pos) {
      const int c = L.C[iz[pos]];
      const int ac = scale * abs(c);
      const int l0 = ac >> shift2;
      const int l = (ac + ((l0 == 0 || chroma) ? off0 : off1)) >> shift2;
      lev = c < 0 ? -l : l;
      any |= l != 0;
    }
    L.S[pos] = lev;
  }
  const int cbp = __any(any) ? 1 : 0;
  wave_lds_sync();
  if (cbp && lane == 0) {  // "RDOQ light" (:134-168): sequential over the scan
    const int n = chroma ? last_pos + 1 : nq;
    const int thr = (73 * dequant_scale(qp % 6) << (qp / 6)) >> (4 + lg);
    for (int pos = 2; pos < n; pos++) {
      int flag = 1;
      if (pos > 2 && abs(L.S[pos - 3]) > 1) flag = 0;
      if (pos > 3 && abs(L.S[pos - 4]) > 1 && abs(L.S[pos - 3]) > 0) flag = 0;
      if (pos == 2 && (chroma == 0 || last_pos >= 6)) flag = 0;
      if (flag && L.S[pos - 2] == 0 && L.S[pos - 1] == 0 && abs(L.S[pos]) > 1) {
        const int c1 = L.C[iz[pos]], c2 = L.C[iz[pos - 1]], c3 = L.C[iz[pos - 2]];
        const int K1 = abs(c1), K2 = abs(c2), K3 = abs(c3), K4 = max(K2, K3);
        if (K1 + K4 < thr) L.S[pos] = c1 < 0 ? -1 : 1;
        else if (K2 > K3) L.S[pos - 1] = c2 < 0 ? -1 : 1;
        else L.S[pos - 2] = c3 < 0 ? -1 : 1;
      }
    }
  }
  wave_lds_sync();
  for (int e = lane; e < nq; e += 64) L.C[e] = L.S[zz[e]];  // back to raster (:170-174)
  wave_lds_sync();
  return cbp;
}

// dequantize (common/common_block.c:132-146) of the q x q levels in L.C into
// L.C, int16 truncating store.
__device__ void dequant_tu(TxLds &L, int qp, int size) {
  const int lane = threadIdx.x & 63;
  const int q = size < 16 ? size : 16;
  const int rshift = ilog2i(size) - 1, add = 1 << (rshift - 1);
  const int lshift = qp / 6, scale = dequant_scale(qp % 6);
  for (int e = lane; e < q * q; e += 64) L.C[e] = wrap16(((L.C[e] * scale) * (1 << lshift) + add) >> rshift);
  wave_lds_sync();
}

// Inverse transform (common/transform.c:432-518) of the q x q coefficients in
// L.C into L.R (n x n, n = min(size, 32)): pass 1 clip16((s + 64) >> 7), pass 2
// clip16((s + 2048) >> 12); 64 = 32-point, the caller replicates 2x2.
__device__ void inv_tx(TxLds &L, int size) {
  const int lane = threadIdx.x & 63;
  const int rep = size == 64, n = rep ? 32 : size, q = n < 16 ? n : 16, step = 32 / n;
  for (int e = lane; e < q * n; e += 64) {  // T[k][y'] over coefficient column k
    const int k = e / n, yp = e - k * n;
    int s = 0;
    for (int m = 0; m < q; m++) s += (int)L.M[(m * step) * 32 + yp] * L.C[m * q + k];
    L.T[k * n + yp] = (int16_t)clip16((s + 64) >> 7);
  }
  wave_lds_sync();
  for (int e = lane; e < n * n; e += 64) {
    const int yp = e / n, xp = e - yp * n;
    int s = 0;
    for (int k = 0; k < q; k++) s += (int)L.M[(k * step) * 32 + xp] * (int)L.T[k * n + yp];
    L.R[yp * n + xp] = (int16_t)clip16((s + 2048) >> 12);  // 64: before the 2x2 replication
  }
  wave_lds_sync();
}

// ---------------------------------------------------------------------------
// Batched encoder transform-block chain: one wavefront per thor_enc_tu_t.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_enc_tu(const thor_enc_tu_t *__restrict__ tus, int n,
                                               const uint8_t *__restrict__ orig, const uint8_t *__restrict__ pred,
                                               uint8_t *__restrict__ rec, int16_t *__restrict__ coeffq,
                                               uint8_t *__restrict__ cbp_out, uint32_t *__restrict__ ssd_out) {
  __shared__ TxLds L;
  const int t = blockIdx.x;
  if (t >= n) return;
  const int lane = threadIdx.x;
  const thor_enc_tu_t U = tus[t];
  const int size = U.size, q = size < 16 ? size : 16;
  if ((size != 4 && size != 8 && size != 16 && size != 32 && size != 64) || U.qp > 51) {
    if (lane == 0) cbp_out[t] = 255;  // invalid descriptor: nothing read or written
    return;
  }
  tx_load_basis(L);
  const uint8_t *po = orig + U.orig_off, *pp = pred + U.pred_off;
  auto res = [&](int y, int x) {  // get_residual, enc/encode_block.c:484-493
    return (int)(int16_t)((int)po[(long long)y * U.orig_stride + x] - (int)pp[(long long)y * U.pred_stride + x]);
  };
  if (size == 64) presum64(L, U.fast, res);
  else
    for (int e = lane; e < size * size; e += 64) {
      const int y = e / size, x = e - y * size;
      L.R[e] = (int16_t)res(y, x);
    }
  wave_lds_sync();
  fwd_tx(L, size, U.fast);
  const int cbp = quant_tu(L, U.qp, size, U.type);
  for (int e = lane; e < q * q; e += 64) coeffq[U.coeff_off + e] = (int16_t)L.C[e];
  if (cbp) {
    dequant_tu(L, U.qp, size);
    inv_tx(L, size);
  }
  uint8_t *pr = rec + U.rec_off;
  unsigned ssd = 0;
  for (int e = lane; e < size * size; e += 64) {  // reconstruct_block / memcpy(rec, pblock), :1512-1517
    const int y = e / size, x = e - y * size;
    const int p = pp[(long long)y * U.pred_stride + x];
    const int rv = size == 64 ? L.R[(y >> 1) * 32 + (x >> 1)] : L.R[e];  // 64: 2x2 replication
    const int r = cbp ? clip255(rv + p) : p;
    pr[(long long)y * U.rec_stride + x] = (uint8_t)r;
    const int d = (int)po[(long long)y * U.orig_stride + x] - r;
    ssd += (unsigned)(d * d);
  }
  ssd = wave_sum_u(ssd);
  if (lane == 0) {
    cbp_out[t] = (uint8_t)cbp;
    ssd_out[t] = ssd;
  }
}

// cost_calc, enc/encode_block.c:1218-1228: SSD_Y + SSD_U + SSD_V +
// (int32)(lambda * nbits + 0.5), clamped to 2^30.  The per-component SSDs are
// sums of k_enc_tu's per-TU SSDs over the CU (exact integers).
__global__ void k_enc_cost(const uint32_t *__restrict__ ssd, const int32_t *__restrict__ tu_first,
                           const int32_t *__restrict__ tu_count, const int32_t *__restrict__ nbits, double lambda,
                           uint32_t *__restrict__ cost, int ncu) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncu) return;
  unsigned s = 0;
  for (int i = 0; i < tu_count[c]; i++) s += ssd[tu_first[c] + i];
  const double prod = lambda * (double)nbits[c];
  unsigned v = s + (unsigned)(int)(prod + 0.5);
  if (v > (1u << 30)) v = 1u << 30;
  cost[c] = v;
}

// ---------------------------------------------------------------------------
// Per-call kernels behind the SIMD surface (simd_surface.hip)
// ---------------------------------------------------------------------------
// transform_simd: block (size x size int16) -> the q x q corner of coeff,
// written compact (the host copies it into the caller's stride-`size` array).
__global__ __launch_bounds__(64) void k_ftx_call(const int16_t *__restrict__ block, int16_t *__restrict__ out,
                                                 int size, int fast) {
  __shared__ TxLds L;
  const int lane = threadIdx.x;
  tx_load_basis(L);
  if (size == 64) presum64(L, fast, [&](int y, int x) { return (int)block[y * 64 + x]; });
  else
    for (int e = lane; e < size * size; e += 64) L.R[e] = block[e];
  wave_lds_sync();
  fwd_tx(L, size, fast);
  const int q = size < 16 ? size : 16;
  for (int e = lane; e < q * q; e += 64) out[e] = (int16_t)L.C[e];
}

// inverse_transform_simd: the q x q corner of coeff (stride size; the
// reference's partial butterflies read no other coefficient) -> block.
__global__ __launch_bounds__(64) void k_itx_call(const int16_t *__restrict__ coeff, int16_t *__restrict__ block,
                                                 int size) {
  __shared__ TxLds L;
  const int lane = threadIdx.x;
  tx_load_basis(L);
  const int n = size == 64 ? 32 : size, q = n < 16 ? n : 16;
  for (int e = lane; e < q * q; e += 64) L.C[e] = coeff[(e / q) * size + (e % q)];
  wave_lds_sync();
  inv_tx(L, size);
  for (int e = lane; e < size * size; e += 64) {
    const int y = e / size, x = e - y * size;
    block[e] = size == 64 ? L.R[(y >> 1) * 32 + (x >> 1)] : L.R[e];
  }
}

extern "C" {

int thor_enc_tu_batch(const thor_enc_tu_t *tus, int n, const uint8_t *orig, const uint8_t *pred, uint8_t *rec,
                      int16_t *coeffq, uint8_t *cbp, uint32_t *ssd, void *stream) {
  if (n < 0 || (n > 0 && (!tus || !orig || !pred || !rec || !coeffq || !cbp || !ssd))) return THOR_ERR_ARG;
  if (n == 0) return THOR_OK;
  k_enc_tu<<<n, 64, 0, (hipStream_t)stream>>>(tus, n, orig, pred, rec, coeffq, cbp, ssd);
  return hipGetLastError() == hipSuccess ? THOR_OK : THOR_ERR_HIP;
}

int thor_enc_cost_batch(const uint32_t *ssd, const int32_t *tu_first, const int32_t *tu_count, const int32_t *nbits,
                        double lambda, uint32_t *cost, int ncu, void *stream) {
  if (ncu < 0 || (ncu > 0 && (!ssd || !tu_first || !tu_count || !nbits || !cost))) return THOR_ERR_ARG;
  if (ncu == 0) return THOR_OK;
  k_enc_cost<<<(ncu + 255) / 256, 256, 0, (hipStream_t)stream>>>(ssd, tu_first, tu_count, nbits, lambda, cost, ncu);
  return hipGetLastError() == hipSuccess ? THOR_OK : THOR_ERR_HIP;
}

}  // extern "C"
