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

extern "C" {

int thor_interp_comp(const uint8_t *p0, int s0, const uint8_t *p1, int s1, uint8_t *out, int so, const int16_t *mv0,
                     const int16_t *mv1, int bw, int bh, int bs, int wP, int hP, int pad, int chroma, int wt0, int wt1,
                     void *stream) {
  if (bw == 0 || bh == 0) return THOR_OK;
  if (!p0 || !p1 || !out || !mv0 || !mv1 || bw < 0 || bh < 0 || bs < 1 || bs > 64 || pad < 0) return THOR_ERR_ARG;
  const dim3 grid((bw * bs + 63) / 64, (bh * bs + 3) / 4);
  k_interp_comp<<<grid, 256, 0, (hipStream_t)stream>>>(p0, s0, p1, s1, out, so, mv0, mv1, bw, bh, bs, wP, hP, pad,
                                                       chroma, wt0, wt1);
  return hipGetLastError() == hipSuccess ? THOR_OK : THOR_ERR_HIP;
}

}  // extern "C"
