// Temporal-interpolation down-sampling pyramid.
//
// interpolate_frames (common/temporal_interp.c:972-1019) builds, per reference
// frame, max_levels-1 luma levels by chaining scale_frame_down2x2[_simd]
// (:151-245): out[i][j] = (avg(in[2i][2j], in[2i+1][2j]) +
// avg(in[2i][2j+1], in[2i+1][2j+1])) >> 1 with avg(p,q) = (p+q+1)>>1, then
// pad_yuv_frame (common/common_frame.c:405-462) on the 32-pixel luma margin of
// the level (create_yuv_frame(.., 32, 32, 16, 16), temporal_interp.c:1004).
// USE_CHROMA is 0 (temporal_interp.c:19): the SIMD path -- the reference
// default -- down-samples luma only, and nothing downstream reads level chroma.
//
// One launch writes every level: a thread owns an 8x8 tile of level 0 and
// computes its 4x4 level-1, 2x2 level-2 and 1x1 level-3 pixels in registers
// (level l+1 pixel (i,j) depends only on level-l pixels (2i..2i+1, 2j..2j+1),
// so the tiles nest without halo).  Level 0 is read once; the levels are
// written once (1 + 1/4 + 1/16 + 1/64 B per level-0 pixel of traffic).  A
// second launch pads every level (PadPlane, loopfilter.hip).

#define THOR_PYR_PAD 32
#define THOR_PYR_MAX 3

struct PyrLevels {
  uint8_t *y[THOR_PYR_MAX];
  int s[THOR_PYR_MAX], w[THOR_PYR_MAX], h[THOR_PYR_MAX];
  int n;
};

__device__ __forceinline__ uint32_t pyr_px(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  // a,b: column 2j rows 2i,2i+1; c,d: column 2j+1
  return (((a + b + 1) >> 1) + ((c + d + 1) >> 1)) >> 1;
}

// grid z = frame (interpolate_frames down-samples ref0 and ref1, :1011-1019)
struct PyrJob {
  const uint8_t *src[2];
  PyrLevels L[2];
};
__global__ __launch_bounds__(256) void k_down_pyramid(const int ss, int W, int H, const PyrJob J) {
  const uint8_t *__restrict__ src = J.src[blockIdx.z];
  const PyrLevels &L = J.L[blockIdx.z];
  const int tx = blockIdx.x * 64 + threadIdx.x, ty = blockIdx.y * 4 + threadIdx.y;
  if (4 * tx >= L.w[0] || 4 * ty >= L.h[0]) return;
  const int x0 = 8 * tx, y0 = 8 * ty;
  uint32_t a[8][8];
  if (x0 + 8 <= W && y0 + 8 <= H) {
#pragma unroll
    for (int r = 0; r < 8; r++) {
      const uint2 v = *(const uint2 *)(src + (long long)(y0 + r) * ss + x0);
#pragma unroll
      for (int k = 0; k < 4; k++) {
        a[r][k] = (v.x >> (8 * k)) & 255u;
        a[r][4 + k] = (v.y >> (8 * k)) & 255u;
      }
    }
  } else {
    // frame edge: clamp (clamped samples only feed pixels outside the level)
#pragma unroll
    for (int r = 0; r < 8; r++) {
      const int y = min(y0 + r, H - 1);
#pragma unroll
      for (int k = 0; k < 8; k++) a[r][k] = src[(long long)y * ss + min(x0 + k, W - 1)];
    }
  }
  // level 1: 4x4
  uint32_t b[4][4];
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) b[i][j] = pyr_px(a[2 * i][2 * j], a[2 * i + 1][2 * j], a[2 * i][2 * j + 1], a[2 * i + 1][2 * j + 1]);
  {
    const int ox = 4 * tx, oy = 4 * ty;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      if (oy + i >= L.h[0]) break;
      uint8_t *o = L.y[0] + (long long)(oy + i) * L.s[0] + ox;
      if (ox + 4 <= L.w[0]) {
        *(uint32_t *)o = b[i][0] | (b[i][1] << 8) | (b[i][2] << 16) | (b[i][3] << 24);
      } else {
        for (int j = 0; ox + j < L.w[0]; j++) o[j] = (uint8_t)b[i][j];
      }
    }
  }
  if (L.n < 2) return;
  uint32_t c[2][2];
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int j = 0; j < 2; j++) c[i][j] = pyr_px(b[2 * i][2 * j], b[2 * i + 1][2 * j], b[2 * i][2 * j + 1], b[2 * i + 1][2 * j + 1]);
  {
    const int ox = 2 * tx, oy = 2 * ty;
#pragma unroll
    for (int i = 0; i < 2; i++) {
      if (oy + i >= L.h[1]) break;
      uint8_t *o = L.y[1] + (long long)(oy + i) * L.s[1] + ox;
      if (ox + 2 <= L.w[1]) {
        *(uint16_t *)o = (uint16_t)(c[i][0] | (c[i][1] << 8));
      } else if (ox < L.w[1]) {
        o[0] = (uint8_t)c[i][0];
      }
    }
  }
  if (L.n < 3) return;
  if (tx < L.w[2] && ty < L.h[2])
    L.y[2][(long long)ty * L.s[2] + tx] = (uint8_t)pyr_px(c[0][0], c[1][0], c[0][1], c[1][1]);
}

// pad every level (grid y = level)
__global__ __launch_bounds__(256) void k_pad_pyramid(const PyrJob J) {
  const PyrLevels &L = J.L[blockIdx.z];
  const int l = blockIdx.y;
  const PadPlane p(L.y[l], L.s[l], L.w[l], L.h[l], THOR_PYR_PAD, 0, L.h[l]);
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e < p.total) p.chunk(e);
}

static inline int pyr_pad_chunks(int w, int h) {
  const int pad = THOR_PYR_PAD;
  const int nl = pad >> 4, nr = (w + pad - (w & ~15) + 15) >> 4, rc = (w + 2 * pad + 15) >> 4;
  return h * (nl + nr) + 2 * pad * rc;
}

extern "C" {

int thor_pyramid_levels(int width, int height) {
  // interpolate_frames: max_levels = min(MAX_LEVELS=4, (int)(log10(min(w,h))/log10(2.0)-4.0))
  // (temporal_interp.c:20,977); levels 1 .. max_levels-1 are down-sampled.
  const int m = width < height ? width : height;
  if (m <= 0) return 0;
  int ml = (int)(log10((double)m) / log10(2.0) - 4.0);
  if (ml > THOR_PYR_MAX + 1) ml = THOR_PYR_MAX + 1;
  return ml > 1 ? ml - 1 : 0;
}

static int pyramid_launch(const uint8_t *const *srcs, int nframes, int src_stride, int width, int height,
                          uint8_t *const *const *levels, const int *level_strides, int nlevels, void *stream) {
  if (nlevels == 0) return THOR_OK;
  if (!levels || !level_strides || nlevels < 0 || nlevels > THOR_PYR_MAX) return THOR_ERR_ARG;
  if (width <= 0 || height <= 0 || (width >> nlevels) < 1 || (height >> nlevels) < 1) return THOR_ERR_ARG;
  if ((src_stride & 7) || src_stride < width) return THOR_ERR_ARG;
  PyrJob J{};
  int chunks = 0;
  for (int f = 0; f < nframes; f++) {
    if (!srcs[f] || ((uintptr_t)srcs[f] & 7) || !levels[f]) return THOR_ERR_ARG;
    J.src[f] = srcs[f];
    PyrLevels &L = J.L[f];
    L.n = nlevels;
    for (int l = 0; l < nlevels; l++) {
      L.y[l] = levels[f][l];
      L.s[l] = level_strides[l];
      L.w[l] = width >> (l + 1);
      L.h[l] = height >> (l + 1);
      // create_yuv_frame layout: 16-byte aligned rows at x = -pad, stride % 16 == 0
      if (!L.y[l] || ((uintptr_t)L.y[l] & 15) || (L.s[l] & 15) || L.s[l] < L.w[l] + 2 * THOR_PYR_PAD) return THOR_ERR_ARG;
      const int c = pyr_pad_chunks(L.w[l], L.h[l]);
      chunks = c > chunks ? c : chunks;
    }
  }
  hipStream_t st = (hipStream_t)stream;
  const PyrLevels &L = J.L[0];
  const dim3 grid((L.w[0] + 4 * 64 - 1) / (4 * 64), (L.h[0] + 4 * 4 - 1) / (4 * 4), nframes);
  k_down_pyramid<<<grid, dim3(64, 4), 0, st>>>(src_stride, width, height, J);
  if (hipGetLastError() != hipSuccess) return THOR_ERR_HIP;
  k_pad_pyramid<<<dim3((chunks + 255) / 256, nlevels, nframes), 256, 0, st>>>(J);
  return hipGetLastError() == hipSuccess ? THOR_OK : THOR_ERR_HIP;
}

int thor_scale_pyramid(const uint8_t *src, int src_stride, int width, int height, uint8_t *const *levels,
                       const int *level_strides, int nlevels, void *stream) {
  if (nlevels != 0 && !src) return THOR_ERR_ARG;
  return pyramid_launch(&src, 1, src_stride, width, height, &levels, level_strides, nlevels, stream);
}

int thor_scale_pyramid2(const uint8_t *src0, const uint8_t *src1, int src_stride, int width, int height,
                        uint8_t *const *levels0, uint8_t *const *levels1, const int *level_strides, int nlevels,
                        void *stream) {
  const uint8_t *srcs[2] = {src0, src1};
  uint8_t *const *lv[2] = {levels0, levels1};
  return pyramid_launch(srcs, 2, src_stride, width, height, lv, level_strides, nlevels, stream);
}

}  // extern "C"
