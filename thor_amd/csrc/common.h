// Shared device-side definitions for the thor_amd HIP kernels (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/thor_amd.h"

#include <stdarg.h>
#include <stdio.h>

#define THOR_MAX_SLOTS 40
#define THOR_PAD_Y 96
#define THOR_PAD_C 48

// Why the last create call (thor_dec_create / thor_enc_create / thor_ti_create)
// of the calling thread returned NULL: thor_last_create_error.
struct ThorCreateErr {
  int code;
  size_t bytes;  // THOR_ERR_NOMEM: the allocation that failed
  char msg[192];
};
static thread_local ThorCreateErr g_create_err = {THOR_OK, 0, {0}};
static inline void create_fail(int code, size_t bytes, const char *fmt, ...) {
  if (g_create_err.code != THOR_OK) return;  // keep the first (root) cause of this create call
  g_create_err.code = code;
  g_create_err.bytes = bytes;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_create_err.msg, sizeof(g_create_err.msg), fmt, ap);
  va_end(ap);
}
static inline void create_begin() {
  g_create_err.code = THOR_OK;
  g_create_err.bytes = 0;
  g_create_err.msg[0] = 0;
}
// hipMalloc that records the failure (out of memory -> THOR_ERR_NOMEM with the
// bytes asked for) and clears HIP's sticky last error so later launches do not
// report it.
template <class T>
static inline bool dev_alloc(T **p, size_t bytes, const char *what) {
  void *q = nullptr;
  const hipError_t e = hipMalloc(&q, bytes);
  if (e == hipSuccess) {
    *p = (T *)q;
    return true;
  }
  *p = nullptr;
  (void)hipGetLastError();
  create_fail(e == hipErrorOutOfMemory ? THOR_ERR_NOMEM : THOR_ERR_HIP, bytes, "%s: hipMalloc(%zu bytes): %s", what,
              bytes, hipGetErrorString(e));
  return false;
}

// block_mode_t, common/types.h:83-90
enum { M_SKIP = 0, M_INTRA = 1, M_INTER = 2, M_BIPRED = 3, M_MERGE = 4 };

// Everything a per-frame kernel needs to address the current frame, the
// resident references and the frame's parse output.  One per frame of a
// batch (FrameBatch below).
struct FrameCtx {
  uint8_t *cy, *cu, *cv;  // current frame, interior (0,0)
  const uint8_t *slots;   // base of the reference ring
  long long slot_bytes;   // bytes per slot
  long long ring_bytes;   // bytes of the whole ring (slot_bytes x slots, < 2 GiB)
  long long offy, offu, offv;  // interior (0,0) offsets inside a slot
  int sy, sc;             // luma / chroma stride (create_yuv_frame, common/common_frame.c:331-332)
  int W, H;
  int frame_num;
  int bipred;             // sequence-level luma filter table select (dec/maindec.c:147)
  int nref;
  int slot_lut[32];       // frame_num & 127 -> slot (int8, -1 none), 4 per word
  // Edge rows: the bottom pixel row of every SB row, per component (the only
  // pixels one intra chain hands to the next).  Y rows of ewy bytes, then U
  // and V rows of ewc bytes; column x at byte EDGE_MARGIN + x.
  uint8_t *edge;
  int ewy, ewc, nsbrows;
  // The frame's job (parse output, DEVICE pointers) and its context's work
  // buffers.  Batched launches read one FrameCtx per frame from device memory
  // (grid y / z = frame of the batch).
  const thor_block_t *blk;
  const int16_t *coeffs;
  const thor_tu_t *tus;
  const uint32_t *ilist;
  const uint8_t *clpf_flags;
  const uint32_t *clpf_list;  // flagged SBs (n_clpf >= 0) or every SB (n_clpf < 0)
  int n_clpf;
  uint16_t *cellinfo;
  uint2 *cellmc;    // per 4x4 cell: (mv0 with `sign` applied, MC meta word) -- k_recon's P0 input
  int32_t *cellmv1; // per 4x4 cell: mv1 (written for bi-pred cells only)
  int16_t *resid;
  unsigned *ctl, *progress;
  int *rowstart;
  int nblocks, ntus, nintra, nprep, nres, full_sb;
  int qp, qpc, deblock, clpf_on;
  int band0, band1;  // SB rows k_recon reconstructs (row-band sharding); all by default
  int islot;         // slot of the frame's temporal-interpolated reference (blocks' ref -2), -1 none
  int pb0, pb1;      // band-local phase B: luma rows [pb0, pb1) deblocked / CLPF'd here; pb1 = 0: whole frame
  int ir0, ir1;      // SB rows whose intra chains run here (band-local intra); ir1 = 0: every row
  // Per half SB (64x32 luma) prediction plan, written by k_frame_prep for the
  // halves one 64x64 inter CU covers with a single (MV, reference) key per
  // prediction pass: (mv0, MC meta word, mv1, tag).  A record is this frame's
  // iff tag == gen (no clearing between frames); k_recon then skips the
  // per-cell resolution.  Null: no plans (every half takes the per-cell path).
  uint4 *hplan;
  int gen;
  const uint32_t *slow;  // the frame's multi-key units (null: none listed, every unit in planned order)
  int nslow;
};
// A batch of frames travels in the kernel argument segment (8 x 384 B, under
// the 4 KB kernarg limit): the host fills it per call, no upload copy.  Every
// batched kernel takes it as its FIRST argument and reads the per-frame
// contexts straight from the kernarg segment (scalar loads, dynamic index).
#define THOR_MAX_BATCH 8

// MC meta word of a 4x4 cell (cellmc.y): reference slots and flags
#define CELL_ACT 0x10000u
#define CELL_BI 0x20000u
#define CELL_RES(c) (0x40000u << (c))  // inter cell with a coded residual in component c
struct FrameBatch {
  FrameCtx f[THOR_MAX_BATCH];
};
static_assert(sizeof(FrameBatch) + 16 <= 4096, "the batch travels in the kernarg segment");
#define FRAME_BATCH_CTX() ((const FrameCtx *)__builtin_amdgcn_kernarg_segment_ptr())
#define EDGE_MARGIN 32

// k_recon's work unit: 128 x 16 luma pixels (a quarter-SB row of two
// horizontally adjacent SBs) + 2 x 64 x 8 chroma; unit u = slice row x pairs +
// pair, slice row = 4 x SB row + quarter (inter.hip).
__host__ __device__ __forceinline__ int half_count(int W, int H) { return 2 * ((W + 63) >> 6) * ((H + 63) >> 6); }
__host__ __device__ __forceinline__ int unit_pairs(int W) { return (((W + 63) >> 6) + 1) >> 1; }
__host__ __device__ __forceinline__ int unit_count(int W, int H) { return unit_pairs(W) * 4 * ((H + 63) >> 6); }

// The slow list of a frame (thor_frame_in_t::slow_list, built on the host by
// thor_build_slow_list): the units with several (MV, reference) keys in a half.
// k_recon dispatches them ahead of the planned units so their long per-cell
// path overlaps the rest of the launch instead of forming its tail.  With a
// list, k_frame_prep tags each multi-key half's plan record {.y = PLAN_SLOW,
// .w = gen} (plain stores of one value, no atomics), and a planned-order
// workgroup whose unit holds such a half leaves it to the list.
#define PLAN_SLOW 0x80000000u

// k_recon's launch geometry, from the host: every index division of the flat
// grid as one multiply-high by a host-computed reciprocal (a runtime scalar
// division is ~35 SALU + a VALU reciprocal round trip per wave).
struct ReconGeo {
  int nfr, maxslow;   // frames in the batch; slow-list slots per frame
  int nu, NU, np;     // units per frame, NU = nu rounded up to 8, SB pairs per slice row
  unsigned mnfr, mNU, mnp;  // reciprocals (recon_recip) of nfr, NU, np
  // MC filter words (common/inter_prediction.c:47-70, packed int8 as inter.hip's
  // TapTables): luma [bipred table][fraction][taps 0-3, taps 4-5], chroma [fraction].
  // Read by uniform index with one scalar load each (a select chain over
  // compile-time constants became table-address arithmetic, ~40 SALU a word).
  int tl[2][4][2];
  int tc[8];
};
static_assert(sizeof(FrameBatch) % 8 == 0, "ReconGeo follows the batch in k_recon's kernarg segment");
// k_recon's ReconGeo argument, read in place in the kernarg segment (dynamic
// indices: scalar loads, no private copy)
#define RECON_GEO() ((const ReconGeo *)((const char *)__builtin_amdgcn_kernarg_segment_ptr() + sizeof(FrameBatch)))
// q = x / d for x < 2^32 / d: m = floor((2^32 - 1) / d) + 1 (d > 1; d = 1: m = 0, q = x)
__host__ __device__ __forceinline__ unsigned recon_recip(unsigned d) { return d > 1 ? 0xffffffffu / d + 1u : 0u; }
__device__ __forceinline__ int recon_div(unsigned x, unsigned m) { return m ? (int)__umulhi(x, m) : (int)x; }
__host__ __device__ __forceinline__ size_t hplan_entries(int W, int H) { return (size_t)half_count(W, H); }

// Per-4x4-cell side information for deblocking / CLPF, packed into 16 bits
// (replaces the 44-byte deblock_data_t, common/types.h:127-135):
//   [2:0] mode  [3] cbp.y  [4] cbp.u  [5] cbp.v  [6] |mv| >= 4 (NEW_MV_TEST,
//   common/common_frame.c:101-102)  [10:8] log2 q_size for vertical edges
//   [13:11] log2 q_size for horizontal edges  [15:14] log2(size) - 3
#define CI_MODE(c) ((c)&7)
#define CI_CBPY(c) (((c) >> 3) & 1)
#define CI_CBPU(c) (((c) >> 4) & 1)
#define CI_CBPV(c) (((c) >> 5) & 1)
#define CI_MVBIG(c) (((c) >> 6) & 1)
#define CI_LQV(c) (((c) >> 8) & 7)
#define CI_LQH(c) (((c) >> 11) & 7)
#define CI_LSZ(c) ((((c) >> 14) & 3) + 3)

__device__ __forceinline__ int clip255(int x) { return x < 0 ? 0 : (x > 255 ? 255 : x); }
__device__ __forceinline__ int clip16(int x) { return x < -32768 ? -32768 : (x > 32767 ? 32767 : x); }
__device__ __forceinline__ int wrap16(int x) { return (int)(int16_t)(uint16_t)(x & 0xffff); }
__device__ __forceinline__ int ilog2i(int x) { return 31 - __clz(x); }

// Ordering of LDS traffic inside one wavefront (no workgroup barrier needed:
// each wave owns its LDS slice).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// HEVC integer DCT basis used by Thor (g*mat_hevc, common/transform.c:41-245):
// row k of the N-point matrix is row k*32/N of the 32-point one.
__device__ __forceinline__ int dct32_entry(int k, int n) {
  const int c[33] = {64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67, 64,
                     61, 57, 54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9,  4,  0};
  if (k == 0) return 64;
  int t = (k * (2 * n + 1)) & 127;
  if (t <= 32) return c[t];
  if (t <= 64) return -c[64 - t];
  if (t <= 96) return -c[t - 64];
  return c[128 - t];
}

__device__ __forceinline__ const uint8_t *slot_plane(const FrameCtx &f, int slot, int comp) {
  const uint8_t *s = f.slots + (long long)slot * f.slot_bytes;
  return s + (comp == 0 ? f.offy : (comp == 1 ? f.offu : f.offv));
}

// gdequant_table, common/common_block.c:98
__device__ __forceinline__ int dequant_scale(int r) {
  return r == 0 ? 40 : r == 1 ? 45 : r == 2 ? 51 : r == 3 ? 57 : r == 4 ? 64 : 72;
}
// chroma_qp, common/common_block.c:78-83
__device__ __forceinline__ int chroma_qp(int q) {
  if (q < 30) return q;
  const int t[22] = {29, 30, 31, 32, 33, 33, 34, 34, 35, 35, 36, 36, 37, 37, 38, 39, 40, 41, 42, 43, 44, 45};
  return t[q - 30];
}
