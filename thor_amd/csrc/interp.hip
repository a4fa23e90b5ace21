// Temporal interpolation: motion-compensated average of two references over a
// block MV field -- interpolate_comp
// (common/temporal_interp.c:920-944) calling mot_comp_avg (:387-441) per
// bs x bs block, for one plane.  The MV field is the output of the
// (raster-serial, host) hierarchical search motion_estimate_bi (:852); this is
// the pixel-parallel stage after it.  One lane per output pixel; the block's
// case (both references inside the padded area / only ref1 / only ref0 /
// clamped) is block-uniform, as in the reference.

__device__ __forceinline__ int interp_scale_val(int v, int numer, int denom) {
  // scale_val, temporal_interp.c:66-75
  if (denom == 0) return 0;
  int prod = v * numer;
  if (denom < 0) {
    denom = -denom;
    prod = -prod;
  }
  return prod >= 0 ? (prod + denom / 2) / denom : -((-prod + denom / 2) / denom);
}

__global__ __launch_bounds__(256) void k_interp_comp(const uint8_t *__restrict__ p0, int s0,
                                                     const uint8_t *__restrict__ p1, int s1, uint8_t *__restrict__ out,
                                                     int so, const int16_t *__restrict__ mv0,
                                                     const int16_t *__restrict__ mv1, int bw, int bh, int bs, int wP,
                                                     int hP, int pad, int chroma, int wt0, int wt1) {
  const int x = blockIdx.x * 64 + (threadIdx.x & 63), y = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (x >= bw * bs || y >= bh * bs) return;
  const int xp = x / bs, yp = y / bs, j = x - xp * bs, i = y - yp * bs;
  const int b = yp * bw + xp;
  int m0x = mv0[2 * b], m0y = mv0[2 * b + 1];
  int m1x = mv1[2 * b], m1y = mv1[2 * b + 1];
  if (chroma) {  // :934-938 (int16 mv_t: the shift is arithmetic)
    m1x = (int16_t)(m1x >> 1);
    m1y = (int16_t)(m1y >> 1);
    const int numer = -wt1, denom = wt0;  // scale_mv, :77-91
    if (numer == denom) {
      m0x = m1x;
      m0y = m1y;
    } else if (numer == -denom) {
      m0x = (int16_t)-m1x;
      m0y = (int16_t)-m1y;
    } else {
      m0x = (int16_t)interp_scale_val(m1x, numer, denom);
      m0y = (int16_t)interp_scale_val(m1y, numer, denom);
    }
  }
  // integer rounding of the 1/8-pel vectors (ACC_BITS 3, :35-37,392-395)
  const int xs0 = xp * bs + ((m0x + 4) >> 3), xs1 = xp * bs + ((m1x + 4) >> 3);
  const int ys0 = yp * bs + ((m0y + 4) >> 3), ys1 = yp * bs + ((m1y + 4) >> 3);
  const bool in0 = xs0 >= -pad && xs0 + bs <= wP && ys0 >= -pad && ys0 + bs <= hP;
  const bool in1 = xs1 >= -pad && xs1 + bs <= wP && ys1 >= -pad && ys1 + bs <= hP;
  uint32_t v;
  if (in0 && in1) {
    v = ((uint32_t)p0[(long long)(ys0 + i) * s0 + xs0 + j] + p1[(long long)(ys1 + i) * s1 + xs1 + j] + 1) >> 1;
  } else if (in1) {
    v = p1[(long long)(ys1 + i) * s1 + xs1 + j];
  } else if (in0) {
    // :420-422 reads ref0's rows with ref1's stride
    v = p0[(long long)ys0 * s0 + xs0 + (long long)i * s1 + j];
  } else {
    const int x0 = min(wP - 1, max(-pad, j + xs0)), x1 = min(wP - 1, max(-pad, j + xs1));
    const int y0 = min(hP - 1, max(-pad, i + ys0)), y1 = min(hP - 1, max(-pad, i + ys1));
    v = ((uint32_t)p0[(long long)y0 * s0 + x0] + p1[(long long)y1 * s1 + x1] + 1) >> 1;
  }
  out[(long long)y * so + x] = (uint8_t)v;
}

// Fast path for the reference's block sizes (bs = 8 luma / 4 chroma,
// BLOCK_STEP/2, temporal_interp.c:12,994): one lane per block row.  Consecutive
// lanes are consecutive blocks of a pixel row, so the 4/8-byte stores are
// contiguous across the wave; each displaced reference row segment is read as
// 2-3 aligned dwords and realigned with v_alignbyte (every dword read holds at
// least one byte of the segment, so it lies inside the plane's allocation).
template <int BS>
struct InterpRow;
template <>
struct InterpRow<8> {
  typedef uint2 T;
  static __device__ __forceinline__ uint2 load(const uint8_t *p) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t *q = (const uint32_t *)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    const uint32_t d0 = q[0], d1 = q[1], d2 = sh ? q[2] : 0u;
    return make_uint2(__builtin_amdgcn_alignbyte(d1, d0, sh), __builtin_amdgcn_alignbyte(d2, d1, sh));
  }
  static __device__ __forceinline__ uint2 avg(uint2 a, uint2 b) {
    return make_uint2((a.x | b.x) - (((a.x ^ b.x) >> 1) & 0x7f7f7f7fu), (a.y | b.y) - (((a.y ^ b.y) >> 1) & 0x7f7f7f7fu));
  }
  static __device__ __forceinline__ void put(uint8_t *o, uint2 v) { *(uint2 *)o = v; }
  static __device__ __forceinline__ void set(uint2 &v, int j, uint32_t b) {
    if (j < 4) v.x |= b << (8 * j);
    else v.y |= b << (8 * (j - 4));
  }
};
template <>
struct InterpRow<4> {
  typedef uint32_t T;
  static __device__ __forceinline__ uint32_t load(const uint8_t *p) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t *q = (const uint32_t *)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    const uint32_t d0 = q[0], d1 = sh ? q[1] : 0u;
    return __builtin_amdgcn_alignbyte(d1, d0, sh);
  }
  static __device__ __forceinline__ uint32_t avg(uint32_t a, uint32_t b) {
    return (a | b) - (((a ^ b) >> 1) & 0x7f7f7f7fu);
  }
  static __device__ __forceinline__ void put(uint8_t *o, uint32_t v) { *(uint32_t *)o = v; }
  static __device__ __forceinline__ void set(uint32_t &v, int j, uint32_t b) { v |= b << (8 * j); }
};

template <int BS>
__device__ __forceinline__ void interp_row(const uint8_t *__restrict__ p0, int s0, const uint8_t *__restrict__ p1, int s1,
                                           uint8_t *__restrict__ out, int so, const int16_t *__restrict__ mv0,
                                           const int16_t *__restrict__ mv1, int bw, int bh, int wP, int hP, int pad,
                                           int chroma, int wt0, int wt1, int xp, int y) {
  typedef InterpRow<BS> R;
  if (xp >= bw || y >= bh * BS) return;
  const int yp = y / BS, i = y - yp * BS;
  const int b = yp * bw + xp;
  const uint32_t w1 = ((const uint32_t *)mv1)[b];
  int m1x = (int16_t)(w1 & 0xffffu), m1y = (int16_t)(w1 >> 16);
  int m0x, m0y;
  if (chroma) {  // :934-938
    m1x = (int16_t)(m1x >> 1);
    m1y = (int16_t)(m1y >> 1);
    const int numer = -wt1, denom = wt0;
    if (numer == denom) {
      m0x = m1x;
      m0y = m1y;
    } else if (numer == -denom) {
      m0x = (int16_t)-m1x;
      m0y = (int16_t)-m1y;
    } else {
      m0x = (int16_t)interp_scale_val(m1x, numer, denom);
      m0y = (int16_t)interp_scale_val(m1y, numer, denom);
    }
  } else {
    const uint32_t w0 = ((const uint32_t *)mv0)[b];
    m0x = (int16_t)(w0 & 0xffffu);
    m0y = (int16_t)(w0 >> 16);
  }
  const int xs0 = xp * BS + ((m0x + 4) >> 3), xs1 = xp * BS + ((m1x + 4) >> 3);
  const int ys0 = yp * BS + ((m0y + 4) >> 3), ys1 = yp * BS + ((m1y + 4) >> 3);
  const bool in0 = xs0 >= -pad && xs0 + BS <= wP && ys0 >= -pad && ys0 + BS <= hP;
  const bool in1 = xs1 >= -pad && xs1 + BS <= wP && ys1 >= -pad && ys1 + BS <= hP;
  typename R::T v;
  if (in0 && in1) {
    v = R::avg(R::load(p0 + (long long)(ys0 + i) * s0 + xs0), R::load(p1 + (long long)(ys1 + i) * s1 + xs1));
  } else if (in1) {
    v = R::load(p1 + (long long)(ys1 + i) * s1 + xs1);
  } else if (in0) {
    v = R::load(p0 + (long long)ys0 * s0 + xs0 + (long long)i * s1);  // ref1's stride, :420-422
  } else {
    v = typename R::T{};
    const int y0 = min(hP - 1, max(-pad, i + ys0)), y1 = min(hP - 1, max(-pad, i + ys1));
#pragma unroll
    for (int j = 0; j < BS; j++) {
      const int x0 = min(wP - 1, max(-pad, j + xs0)), x1 = min(wP - 1, max(-pad, j + xs1));
      R::set(v, j, ((uint32_t)p0[(long long)y0 * s0 + x0] + p1[(long long)y1 * s1 + x1] + 1) >> 1);
    }
  }
  R::put(out + (long long)y * so + xp * BS, v);
}

template <int BS>
__global__ __launch_bounds__(256) void k_interp_rows(const uint8_t *__restrict__ p0, int s0,
                                                     const uint8_t *__restrict__ p1, int s1, uint8_t *__restrict__ out,
                                                     int so, const int16_t *__restrict__ mv0,
                                                     const int16_t *__restrict__ mv1, int bw, int bh, int wP, int hP,
                                                     int pad, int chroma, int wt0, int wt1) {
  interp_row<BS>(p0, s0, p1, s1, out, so, mv0, mv1, bw, bh, wP, hP, pad, chroma, wt0, wt1,
                 blockIdx.x * 64 + (threadIdx.x & 63), blockIdx.y * 4 + (threadIdx.x >> 6));
}

// interpolate_frame (:946-970) in one launch: grid z = plane (Y with 8-px
// blocks, U and V with 4-px blocks and the derived chroma vectors).
struct InterpFrame {
  thor_interp_plane_t pl[3];
};
__global__ __launch_bounds__(256) void k_interp_frame(const InterpFrame F, const int16_t *__restrict__ mv0,
                                                      const int16_t *__restrict__ mv1, int bw, int bh, int w, int h,
                                                      int wt0, int wt1) {
  const int xp = blockIdx.x * 64 + (threadIdx.x & 63), y = blockIdx.y * 4 + (threadIdx.x >> 6);
  const thor_interp_plane_t &P = F.pl[blockIdx.z];
  if (blockIdx.z == 0)
    interp_row<8>(P.p0, P.s0, P.p1, P.s1, P.out, P.so, mv0, mv1, bw, bh, w + 4, h + 4, 4, 0, wt0, wt1, xp, y);
  else
    interp_row<4>(P.p0, P.s0, P.p1, P.s1, P.out, P.so, mv0, mv1, bw, bh, (w + 4) / 2, (h + 4) / 2, 2, 1, wt0, wt1, xp,
                  y);
}

extern "C" {

int thor_interp_comp(const uint8_t *p0, int s0, const uint8_t *p1, int s1, uint8_t *out, int so, const int16_t *mv0,
                     const int16_t *mv1, int bw, int bh, int bs, int wP, int hP, int pad, int chroma, int wt0, int wt1,
                     void *stream) {
  if (bw == 0 || bh == 0) return THOR_OK;
  if (!p0 || !p1 || !out || !mv0 || !mv1 || bw < 0 || bh < 0 || bs < 1 || bs > 64 || pad < 0) return THOR_ERR_ARG;
  const bool mv_ok = !(((uintptr_t)mv1 | (chroma ? 0 : (uintptr_t)mv0)) & 3);
  if ((bs == 8 || bs == 4) && mv_ok && !(((uintptr_t)out | (uintptr_t)so) & (bs - 1))) {
    const dim3 grid((bw + 63) / 64, (bh * bs + 3) / 4);
    if (bs == 8)
      k_interp_rows<8><<<grid, 256, 0, (hipStream_t)stream>>>(p0, s0, p1, s1, out, so, mv0, mv1, bw, bh, wP, hP, pad,
                                                                chroma, wt0, wt1);
    else
      k_interp_rows<4><<<grid, 256, 0, (hipStream_t)stream>>>(p0, s0, p1, s1, out, so, mv0, mv1, bw, bh, wP, hP, pad,
                                                                chroma, wt0, wt1);
    return hipGetLastError() == hipSuccess ? THOR_OK : THOR_ERR_HIP;
  }
  const dim3 grid((bw * bs + 63) / 64, (bh * bs + 3) / 4);
  k_interp_comp<<<grid, 256, 0, (hipStream_t)stream>>>(p0, s0, p1, s1, out, so, mv0, mv1, bw, bh, bs, wP, hP, pad,
                                                       chroma, wt0, wt1);
  return hipGetLastError() == hipSuccess ? THOR_OK : THOR_ERR_HIP;
}

int thor_interp_frame(const thor_interp_plane_t *planes, const int16_t *mv0, const int16_t *mv1, int bw, int bh,
                      int width, int height, int wt0, int wt1, void *stream) {
  if (bw == 0 || bh == 0) return THOR_OK;
  if (!planes || !mv0 || !mv1 || bw < 0 || bh < 0 || width <= 0 || height <= 0) return THOR_ERR_ARG;
  InterpFrame F;
  bool fast = !(((uintptr_t)mv0 | (uintptr_t)mv1) & 3);
  for (int c = 0; c < 3; c++) {
    F.pl[c] = planes[c];
    if (!F.pl[c].p0 || !F.pl[c].p1 || !F.pl[c].out) return THOR_ERR_ARG;
    if (((uintptr_t)F.pl[c].out | (uintptr_t)F.pl[c].so) & (c ? 3 : 7)) fast = false;
  }
  if (!fast) {  // per-plane launches on the general kernel
    for (int c = 0; c < 3; c++) {
      const thor_interp_plane_t &P = F.pl[c];
      const int rc = c == 0 ? thor_interp_comp(P.p0, P.s0, P.p1, P.s1, P.out, P.so, mv0, mv1, bw, bh, 8, width + 4,
                                               height + 4, 4, 0, wt0, wt1, stream)
                            : thor_interp_comp(P.p0, P.s0, P.p1, P.s1, P.out, P.so, mv0, mv1, bw, bh, 4,
                                               (width + 4) / 2, (height + 4) / 2, 2, 1, wt0, wt1, stream);
      if (rc) return rc;
    }
    return THOR_OK;
  }
  const dim3 grid((bw + 63) / 64, (bh * 8 + 3) / 4, 3);
  k_interp_frame<<<grid, 256, 0, (hipStream_t)stream>>>(F, mv0, mv1, bw, bh, width, height, wt0, wt1);
  return hipGetLastError() == hipSuccess ? THOR_OK : THOR_ERR_HIP;
}

}  // extern "C"
