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
