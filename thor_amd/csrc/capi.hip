// Host side of libthor_amd.so: the batched per-frame C-ABI (include/thor_amd.h).
// Restates the frame-level control of dec/decode_frame.c:45-148 around the
// GPU stages: a ring of padded reference slots standing in for the
// decoder's sliding window (decode_frame.c:138-147, MAX_REF_FRAMES = 33,
// common/global.h:69), then per frame: side-info -> inter -> intra ->
// deblock -> CLPF -> pad, all enqueued on one HIP stream.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "common.h"

// kernels (recon.hip, intra.hip, loopfilter.hip)
__global__ void k_frame_prep(const thor_block_t *, int, uint16_t *, int32_t *, const uint32_t *, int, const int16_t *,
                             int16_t *, const uint32_t *, int, unsigned *, unsigned *, int *, int, int, int, int, int);
__global__ void k_recon(FrameCtx, const thor_block_t *, const int16_t *, const int32_t *, int16_t *,
                        unsigned long long *);
__global__ void k_intra(FrameCtx, const thor_block_t *, const uint32_t *, const int *, unsigned *, unsigned *, int,
                        unsigned long long *, int, int, const int16_t *);
__global__ void k_deblock_v(uint8_t *, uint8_t *, uint8_t *, int, int, int, int, const uint16_t *, int, int, int, int);
__global__ void k_deblock_h(uint8_t *, uint8_t *, uint8_t *, int, int, int, int, const uint16_t *, int, int, int, int);
__global__ void k_clpf(uint8_t *, uint8_t *, uint8_t *, int, int, int, int, const uint16_t *, const uint8_t *);
__global__ void k_pad(uint8_t *, uint8_t *, uint8_t *, int, int, int, int);

#define HIPCHK(x)                                                                               \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      fprintf(stderr, "thor_amd: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, \
              __LINE__);                                                                        \
      return THOR_ERR_HIP;                                                                      \
    }                                                                                           \
  } while (0)

static int chroma_qp_host(int q) {
  static const int t[52] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17,
                            18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 29, 30, 31, 32, 33, 33,
                            34, 34, 35, 35, 36, 36, 37, 37, 38, 39, 40, 41, 42, 43, 44, 45};
  return t[q < 0 ? 0 : (q > 51 ? 51 : q)];
}

struct thor_dec {
  thor_seq_t seq;
  int device;
  hipStream_t own_stream, stream;
  int sy, sc;
  long long offy, offu, offv, slot_bytes;
  int nslots;
  uint8_t *slots;
  std::vector<int> slot_fnum;   // -1 = empty
  std::vector<long long> slot_age;
  long long decode_count;
  uint16_t *cellinfo;
  int32_t *cellmap;
  unsigned *ctl;       // [0] intra row head, [1] timeout flag
  unsigned *progress;  // intra wavefront progress per (SB row, component)
  int16_t *resid;      // residual planes (Y, U, V; int16), written by k_prep_resid, read by k_recon / k_intra
  uint8_t *edge;       // SB-row edge rows (FrameCtx::edge)
  int ewy, ewc;
  unsigned long long *dbg;  // optional per-row intra timing (debug)
  unsigned long long *dbg_recon;  // optional k_recon phase stamps (debug)
  int dbg_flags;
  int stop_stage;
  // optional per-stage timing (hipEvents on the decode stream)
  int timing;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used;
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> ev_marks;
};

enum { ST_PREP = 0, ST_INTER, ST_INTRA, ST_DEBLOCK, ST_CLPF, ST_PAD, ST_COUNT };

static hipEvent_t ev_next(thor_dec *d) {
  if (d->ev_used == d->ev_pool.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    d->ev_pool.push_back(e);
  }
  return d->ev_pool[d->ev_used++];
}
struct StageMark {
  thor_dec *d;
  int stage;
  hipEvent_t a;
  StageMark(thor_dec *d_, int s) : d(d_), stage(s), a(nullptr) {
    if (d->timing && (a = ev_next(d))) (void)hipEventRecord(a, d->stream);
  }
  ~StageMark() {
    if (!a) return;
    hipEvent_t b = ev_next(d);
    if (!b) return;
    (void)hipEventRecord(b, d->stream);
    d->ev_marks.push_back({stage, {a, b}});
  }
};

extern "C" {

const char *thor_version(void) { return "thor_amd 0.1 (gfx950)"; }

int thor_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

void *thor_dev_alloc(size_t bytes) {
  void *p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
  return p;
}
int thor_dev_free(void *p) {
  HIPCHK(hipFree(p));
  return THOR_OK;
}
int thor_h2d(void *dst, const void *src, size_t bytes) {
  HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
  return THOR_OK;
}
int thor_d2h(void *dst, const void *src, size_t bytes) {
  HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
  return THOR_OK;
}

thor_dec_t *thor_dec_create(const thor_seq_t *seq, int device, int num_slots) {
  if (!seq || seq->width <= 0 || seq->height <= 0 || (seq->width & 15) || (seq->height & 7)) return nullptr;
  if (num_slots <= 1) num_slots = 34;  // 33 references + the frame being decoded
  if (num_slots > THOR_MAX_SLOTS) num_slots = THOR_MAX_SLOTS;
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  thor_dec *d = new thor_dec();
  d->seq = *seq;
  d->device = device;
  int W = seq->width, H = seq->height;
  d->sy = (W + 2 * THOR_PAD_Y + 15) & ~15;       // common/common_frame.c:331
  d->sc = (W / 2 + 2 * THOR_PAD_C + 15) & ~15;   // :332
  long long ybytes = (long long)(H + 2 * THOR_PAD_Y) * d->sy;
  long long cbytes = (long long)(H / 2 + 2 * THOR_PAD_C) * d->sc;
  ybytes = (ybytes + 255) & ~255LL;
  cbytes = (cbytes + 255) & ~255LL;
  d->offy = (long long)THOR_PAD_Y * d->sy + THOR_PAD_Y;
  d->offu = ybytes + (long long)THOR_PAD_C * d->sc + THOR_PAD_C;
  d->offv = ybytes + cbytes + (long long)THOR_PAD_C * d->sc + THOR_PAD_C;
  d->slot_bytes = ybytes + 2 * cbytes + 256;
  if (d->slot_bytes * num_slots >= (1LL << 31)) {  // k_recon addresses the ring with 32-bit buffer offsets
    delete d;
    return nullptr;
  }
  d->nslots = num_slots;
  d->slot_fnum.assign(num_slots, -1);
  d->slot_age.assign(num_slots, -1);
  d->decode_count = 0;
  d->stop_stage = 2;
  d->progress = nullptr;
  d->resid = nullptr;
  d->edge = nullptr;
  d->dbg = nullptr;
  d->dbg_recon = nullptr;
  d->dbg_flags = 0;
  d->timing = 0;
  d->ev_used = 0;
  bool ok = hipStreamCreateWithFlags(&d->own_stream, hipStreamNonBlocking) == hipSuccess;
  d->stream = d->own_stream;
  ok = ok && hipMalloc(&d->slots, d->slot_bytes * num_slots) == hipSuccess;
  ok = ok && hipMemset(d->slots, 0, d->slot_bytes * num_slots) == hipSuccess;
  size_t ncell = (size_t)(W / 4) * (H / 4);
  ok = ok && hipMalloc(&d->cellinfo, ncell * sizeof(uint16_t)) == hipSuccess;
  ok = ok && hipMalloc(&d->cellmap, ncell * sizeof(int32_t)) == hipSuccess;
  ok = ok && hipMemset(d->cellmap, 0, ncell * sizeof(int32_t)) == hipSuccess;
  ok = ok && hipMemset(d->cellinfo, 0, ncell * sizeof(uint16_t)) == hipSuccess;
  ok = ok && hipMalloc(&d->ctl, 64) == hipSuccess;
  ok = ok && hipMalloc(&d->resid, (size_t)W * H * 3) == hipSuccess;  // 1.5 px/luma px x 2 B
  // intra progress words (3 per SB row), then the rows' intra-list segments (nrows + 1)
  ok = ok && hipMalloc(&d->progress, (size_t)4 * ((H + 63) / 64 + 2) * sizeof(unsigned)) == hipSuccess;
  d->ewy = (W + 2 * EDGE_MARGIN + 15) & ~15;
  d->ewc = (W / 2 + 2 * EDGE_MARGIN + 15) & ~15;
  ok = ok && hipMalloc(&d->edge, (size_t)((H + 63) / 64) * (d->ewy + 2 * d->ewc)) == hipSuccess;
  ok = ok && hipMemset(d->ctl, 0, 64) == hipSuccess;
  {  // k_intra stages a row's CU words in LDS (up to (W/8) x 8 CUs)
    size_t lds = (size_t)((W + 7) / 8) * 8 * sizeof(uint2);
    if (lds > 48 * 1024)
      ok = ok && hipFuncSetAttribute((const void *)k_intra, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) ==
                     hipSuccess;
  }
  if (!ok) {
    thor_dec_destroy(d);
    return nullptr;
  }
  return d;
}

void thor_dec_destroy(thor_dec_t *d) {
  if (!d) return;
  (void)hipSetDevice(d->device);
  if (d->own_stream) (void)hipStreamSynchronize(d->own_stream);
  if (d->slots) (void)hipFree(d->slots);
  if (d->cellinfo) (void)hipFree(d->cellinfo);
  if (d->cellmap) (void)hipFree(d->cellmap);
  if (d->ctl) (void)hipFree(d->ctl);
  if (d->progress) (void)hipFree(d->progress);
  if (d->resid) (void)hipFree(d->resid);
  if (d->edge) (void)hipFree(d->edge);
  for (auto e : d->ev_pool) (void)hipEventDestroy(e);
  if (d->own_stream) (void)hipStreamDestroy(d->own_stream);
  delete d;
}

void *thor_dec_stream(thor_dec_t *d) { return d ? (void *)d->stream : nullptr; }
int thor_dec_set_stream(thor_dec_t *d, void *stream) {
  if (!d) return THOR_ERR_ARG;
  d->stream = stream ? (hipStream_t)stream : d->own_stream;
  return THOR_OK;
}
int thor_dec_set_stop_stage(thor_dec_t *d, int stage) {
  if (!d || stage < 0 || stage > 2) return THOR_ERR_ARG;
  d->stop_stage = stage;
  return THOR_OK;
}
int thor_dec_sync(thor_dec_t *d) {
  if (!d) return THOR_ERR_ARG;
  HIPCHK(hipStreamSynchronize(d->stream));
  unsigned to = 0;
  HIPCHK(hipMemcpy(&to, d->ctl + 1, sizeof(unsigned), hipMemcpyDeviceToHost));
  if (to) {
    fprintf(stderr, "thor_amd: intra dependency wait timed out\n");
    return THOR_ERR_HIP;
  }
  return THOR_OK;
}

static int find_slot_host(const thor_dec *d, int fnum) {
  for (int s = 0; s < d->nslots; s++)
    if (d->slot_fnum[s] == fnum) return s;
  return -1;
}

// Slot for the frame about to be decoded: a free slot, else the one decoded
// longest ago (sliding window: the reference shifted out, decode_frame.c:138-147).
static int pick_slot(const thor_dec *d, int frame_num) {
  for (int s = 0; s < d->nslots; s++)  // re-decoding a frame reuses its slot
    if (d->slot_fnum[s] == frame_num) return s;
  int best = 0;
  for (int s = 0; s < d->nslots; s++) {
    if (d->slot_fnum[s] < 0) return s;
    if (d->slot_age[s] < d->slot_age[best]) best = s;
  }
  return best;
}

static FrameCtx make_ctx(const thor_dec *d, int cur_slot, int frame_num) {
  FrameCtx f;
  memset(&f, 0, sizeof(f));
  uint8_t *cur = d->slots + (long long)cur_slot * d->slot_bytes;
  f.cy = cur + d->offy;
  f.cu = cur + d->offu;
  f.cv = cur + d->offv;
  f.slots = d->slots;
  f.slot_bytes = d->slot_bytes;
  f.ring_bytes = d->slot_bytes * d->nslots;
  f.offy = d->offy;
  f.offu = d->offu;
  f.offv = d->offv;
  f.sy = d->sy;
  f.sc = d->sc;
  f.W = d->seq.width;
  f.H = d->seq.height;
  f.frame_num = frame_num;
  f.bipred = d->seq.bipred;
  f.nref = 0;
  for (int s = 0; s < d->nslots; s++) {
    if (s == cur_slot || d->slot_fnum[s] < 0) continue;
    f.ref_fnum[f.nref] = d->slot_fnum[s];
    f.ref_slot[f.nref] = s;
    f.nref++;
  }
  f.edge = d->edge;
  f.ewy = d->ewy;
  f.ewc = d->ewc;
  f.nsbrows = (d->seq.height + 63) / 64;
  int8_t lut[128];
  memset(lut, -1, sizeof(lut));
  for (int r = 0; r < f.nref; r++) lut[f.ref_fnum[r] & 127] = (int8_t)f.ref_slot[r];
  memcpy(f.slot_lut, lut, sizeof(lut));
  return f;
}

int thor_dec_frame(thor_dec_t *d, const thor_frame_hdr_t *hdr, const thor_block_t *blocks, int nblocks,
                   const int16_t *coeffs, const uint8_t *clpf_flags, const uint32_t *intra_list, int n_intra,
                   const uint32_t *tu_list, int n_tu) {
  if (!d || !hdr || nblocks < 0 || (nblocks > 0 && !blocks)) return THOR_ERR_ARG;
  if (n_intra > 0 && !intra_list) return THOR_ERR_ARG;
  if (n_tu < 0 || (n_tu > 0 && (!tu_list || !coeffs))) return THOR_ERR_ARG;
  HIPCHK(hipSetDevice(d->device));
  int W = d->seq.width, H = d->seq.height;
  int cur = pick_slot(d, hdr->frame_num);
  FrameCtx f = make_ctx(d, cur, hdr->frame_num);
  // k_recon resolves references through a 128-entry table keyed by
  // frame_num & 127: resident frame numbers must be distinct modulo 128
  for (int a = 0; a < f.nref; a++)
    for (int b = a + 1; b < f.nref; b++)
      if (((f.ref_fnum[a] ^ f.ref_fnum[b]) & 127) == 0) return THOR_ERR_REF;
  hipStream_t st = d->stream;
  if (nblocks > 0) {
    {
      // side info + residuals of every coded transform block + intra chain setup
      StageMark m(d, ST_PREP);
      const int nrows = (H + 63) / 64;
      int *rowstart = (int *)(d->progress + 3 * (nrows + 1));
      const int nprep = (nblocks + 3) / 4, nres = (n_tu + 3) / 4;
      k_frame_prep<<<nprep + nres + 1, 256, 0, st>>>(blocks, nblocks, d->cellinfo, d->cellmap, tu_list, n_tu, coeffs,
                                                     d->resid, intra_list, n_intra, d->ctl, d->progress, rowstart,
                                                     nrows, W, H, nprep, nres);
      HIPCHK(hipGetLastError());
    }
    int nsb = ((W + 63) / 64) * ((H + 63) / 64);
    StageMark m(d, ST_INTER);  // k_recon alone: the inter-reconstruction roofline kernel
    k_recon<<<8 * ((2 * nsb + 7) / 8), 64, 0, st>>>(f, blocks, coeffs, d->cellmap, d->resid, d->dbg_recon);
    HIPCHK(hipGetLastError());
  }
  if (n_intra > 0) {
    int nrows = (H + 63) / 64;
    StageMark m(d, ST_INTRA);
    int *rowstart = (int *)(d->progress + 3 * (nrows + 1));  // set up by k_frame_prep
    // full SB images only when inter CUs were reconstructed (their pixels are intra neighbours)
    int full_sb = n_intra < nblocks;
    // one single-wave chain per (SB row, component); LDS holds the row's CU words
    size_t lds = (size_t)((W + 7) / 8) * 8 * sizeof(uint2);
    k_intra<<<3 * nrows, 64, lds, st>>>(f, blocks, intra_list, rowstart, d->ctl, d->progress, nrows, d->dbg,
                                        d->dbg_flags, full_sb, d->resid);
    HIPCHK(hipGetLastError());
  }
  if (d->stop_stage >= 1 && d->seq.deblocking) {
    StageMark m(d, ST_DEBLOCK);
    int nv = ((W >> 3) - 1) * (H >> 3);
    int nh = (W >> 3) * ((H >> 3) - 1);
    int qpc = chroma_qp_host(hdr->qp);
    // luma and both chroma planes of one edge direction per launch
    const int bv = (nv + 255) / 256, bh = (nh + 255) / 256;
    k_deblock_v<<<3 * bv, 256, 0, st>>>(f.cy, f.cu, f.cv, d->sy, d->sc, W, H, d->cellinfo, hdr->qp, qpc, bv, bv);
    k_deblock_h<<<3 * bh, 256, 0, st>>>(f.cy, f.cu, f.cv, d->sy, d->sc, W, H, d->cellinfo, hdr->qp, qpc, bh, bh);
    HIPCHK(hipGetLastError());
  }
  if (d->stop_stage >= 2 && d->seq.clpf && hdr->clpf_on && clpf_flags) {
    int nsb = (W / 64) * (H / 64);
    if (nsb > 0) {
      StageMark m(d, ST_CLPF);
      k_clpf<<<nsb, 256, 0, st>>>(f.cy, f.cu, f.cv, d->sy, d->sc, W, H, d->cellinfo, clpf_flags);
      HIPCHK(hipGetLastError());
    }
  }
  {
    StageMark m(d, ST_PAD);
    k_pad<<<dim3(H + 2 * THOR_PAD_Y, 3), 256, 0, st>>>(f.cy, f.cu, f.cv, d->sy, d->sc, W, H);
    HIPCHK(hipGetLastError());
  }
  d->slot_fnum[cur] = hdr->frame_num;
  d->slot_age[cur] = d->decode_count++;
  return THOR_OK;
}

// Debug hook (not in the public header): per-row intra timing into a device
// buffer of 4 u64 per SB row; flags bit0 ignores the wavefront waits.
extern "C" int thor_dec_debug_intra(thor_dec_t *d, void *dev_buf, int flags) {
  if (!d) return THOR_ERR_ARG;
  d->dbg = (unsigned long long *)dev_buf;
  d->dbg_flags = flags;
  return THOR_OK;
}

// Debug hook (not in the public header): k_recon phase stamps, 8 u64 per wave.
extern "C" int thor_dec_debug_recon(thor_dec_t *d, void *dev_buf) {
  if (!d) return THOR_ERR_ARG;
  d->dbg_recon = (unsigned long long *)dev_buf;
  return THOR_OK;
}

int thor_dec_set_timing(thor_dec_t *d, int on) {
  if (!d) return THOR_ERR_ARG;
  d->timing = on;
  return THOR_OK;
}

int thor_dec_stage_ms(thor_dec_t *d, double *ms, int nstages) {
  if (!d || !ms || nstages <= 0) return THOR_ERR_ARG;
  HIPCHK(hipStreamSynchronize(d->stream));
  for (int i = 0; i < nstages; i++) ms[i] = 0.0;
  for (auto &m : d->ev_marks) {
    float t = 0.f;
    HIPCHK(hipEventElapsedTime(&t, m.second.first, m.second.second));
    if (m.first < nstages) ms[m.first] += t;
  }
  d->ev_marks.clear();
  d->ev_used = 0;
  return THOR_OK;
}

int thor_dec_stage_marks(thor_dec_t *d, int *stage, double *ms, int cap) {
  if (!d || cap < 0 || (cap > 0 && (!stage || !ms))) return THOR_ERR_ARG;
  HIPCHK(hipStreamSynchronize(d->stream));
  int n = 0;
  for (auto &m : d->ev_marks) {
    if (n >= cap) break;
    float t = 0.f;
    HIPCHK(hipEventElapsedTime(&t, m.second.first, m.second.second));
    stage[n] = m.first;
    ms[n] = t;
    n++;
  }
  d->ev_marks.clear();
  d->ev_used = 0;
  return n;
}

int thor_build_tu_list(const thor_block_t *host_blocks, int nblocks, uint32_t *out) {
  if (nblocks < 0 || (nblocks > 0 && !host_blocks)) return THOR_ERR_ARG;
  if (nblocks >= (1 << 27)) return THOR_ERR_ARG;
  int n = 0;
  for (int b = 0; b < nblocks; b++) {
    const thor_block_t &B = host_blocks[b];
    if (B.mode == M_SKIP) continue;  // SKIP carries no residual (dec/decode_block.c:213-242)
    for (int c = 0; c < 3; c++) {
      if (!((B.coeff_mask >> c) & 1)) continue;
      // tb-split gives 4 quarters; chroma of an 8x8 CU is not split (dec/decode_block.c:449-450)
      const int split = B.tb_split && (c == 0 || B.size > 8);
      for (int t = 0; t < (split ? 4 : 1); t++) {
        if (out) out[n] = ((uint32_t)b << 4) | ((uint32_t)c << 2) | (uint32_t)t;
        n++;
      }
    }
  }
  return n;
}

int thor_build_intra_list(const thor_block_t *host_blocks, int nblocks, uint32_t *out) {
  if (nblocks < 0 || (nblocks > 0 && !host_blocks)) return THOR_ERR_ARG;
  int n = 0;
  for (int b = 0; b < nblocks; b++)
    if (host_blocks[b].mode == M_INTRA) {
      if (out) out[n] = (uint32_t)b;
      n++;
    }
  return n;
}

int thor_dec_read_frame(thor_dec_t *d, int frame_num, uint8_t *y, uint8_t *u, uint8_t *v) {
  if (!d) return THOR_ERR_ARG;
  int s = find_slot_host(d, frame_num);
  if (s < 0) return THOR_ERR_REF;
  HIPCHK(hipSetDevice(d->device));
  HIPCHK(hipStreamSynchronize(d->stream));
  int W = d->seq.width, H = d->seq.height;
  const uint8_t *base = d->slots + (long long)s * d->slot_bytes;
  if (y) HIPCHK(hipMemcpy2D(y, W, base + d->offy, d->sy, W, H, hipMemcpyDeviceToHost));
  if (u) HIPCHK(hipMemcpy2D(u, W / 2, base + d->offu, d->sc, W / 2, H / 2, hipMemcpyDeviceToHost));
  if (v) HIPCHK(hipMemcpy2D(v, W / 2, base + d->offv, d->sc, W / 2, H / 2, hipMemcpyDeviceToHost));
  return THOR_OK;
}

int thor_dec_write_frame(thor_dec_t *d, int frame_num, const uint8_t *y, const uint8_t *u, const uint8_t *v) {
  if (!d || !y || !u || !v) return THOR_ERR_ARG;
  HIPCHK(hipSetDevice(d->device));
  int s = find_slot_host(d, frame_num);
  if (s < 0) s = pick_slot(d, frame_num);
  int W = d->seq.width, H = d->seq.height;
  uint8_t *base = d->slots + (long long)s * d->slot_bytes;
  HIPCHK(hipMemcpy2D(base + d->offy, d->sy, y, W, W, H, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy2D(base + d->offu, d->sc, u, W / 2, W / 2, H / 2, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy2D(base + d->offv, d->sc, v, W / 2, W / 2, H / 2, hipMemcpyHostToDevice));
  k_pad<<<dim3(H + 2 * THOR_PAD_Y, 3), 256, 0, d->stream>>>(base + d->offy, base + d->offu, base + d->offv, d->sy,
                                                            d->sc, W, H);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(d->stream));
  d->slot_fnum[s] = frame_num;
  d->slot_age[s] = d->decode_count++;
  return THOR_OK;
}

}  // extern "C"
