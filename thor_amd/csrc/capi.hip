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

// kernels (intra.hip, inter.hip, loopfilter.hip): the frame batch by value, first argument
__global__ void k_frame_prep(const FrameBatch);
__global__ void k_recon(const FrameBatch, const ReconGeo, unsigned long long *);
__global__ void k_intra(const FrameBatch, unsigned long long *, int);
__global__ void k_deblock_v(const FrameBatch, int, int);
__global__ void k_deblock_h(const FrameBatch, int, int);
__global__ void k_clpf(const FrameBatch);
__global__ void k_pad(const FrameBatch, int, int);

#define HIPCHK(x)                                                                               \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      fprintf(stderr, "thor_amd: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, \
              __LINE__);                                                                        \
      return THOR_ERR_HIP;                                                                      \
    }                                                                                           \
  } while (0)

#include "host_lists.h"

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
  uint2 *cellmc;
  int32_t *cellmv1;
  unsigned *ctl;       // [0] intra row head, [1] timeout flag
  unsigned *progress;  // intra wavefront progress per (SB row, component)
  int16_t *resid;      // residual planes (Y, U, V; int16), written by k_prep_resid, read by k_recon / k_intra
  uint8_t *edge;       // SB-row edge rows (FrameCtx::edge)
  uint4 *hplan;        // per half SB prediction plans (FrameCtx::hplan)
  unsigned plan_gen;   // tag of the latest frame's plans
  int ewy, ewc;
  unsigned long long *dbg;  // optional per-row intra timing (debug)
  unsigned long long *dbg_recon;  // optional k_recon phase stamps (debug)
  int dbg_flags;
  int stop_stage;
  hipEvent_t xev[2];  // cross-stream ordering when a batch mixes contexts on different streams
  int band0, band1;    // SB rows k_recon reconstructs (row sharding); band1 0 = all
  int band_intra;      // row sharding: the intra chains of the band's rows only (thor_dec_set_band_intra)
  int band_local;      // phase B filters only the band's rows (thor_dec_set_band_local)
  int band_pad;        // band-local: thor_dec_frame_finish pads only the band's rows (thor_dec_set_band_pad)
  void *pending;       // Batch of a thor_dec_frame_begin awaiting its _end (or, band-local, its _finish)
  int pending_ended;   // band-local: _end done, _finish (pad + commit) due
  // temporal-interpolated references (seq.interp_ref): slot `islot` after the
  // ring holds the current frame's interpolated reference; `ti` its scratch
  int islot;
  thor_ti_t *ti;
  // optional per-stage timing (hipEvents on the decode stream)
  int timing;
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used;
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> ev_marks;
};

enum { ST_PREP = 0, ST_INTER, ST_INTRA, ST_DEBLOCK, ST_CLPF, ST_PAD, ST_INTERP, ST_COUNT };

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

int thor_last_create_error(size_t *bytes, char *msg, size_t cap) {
  if (bytes) *bytes = g_create_err.bytes;
  if (msg && cap) snprintf(msg, cap, "%s", g_create_err.msg);
  return g_create_err.code;
}

thor_dec_t *thor_dec_create(const thor_seq_t *seq, int device, int num_slots) {
  create_begin();
  if (!seq || seq->width <= 0 || seq->height <= 0 || (seq->width & 7) || (seq->height & 7)) {  // multiples of 8 (enc/strings.c:437)
    create_fail(THOR_ERR_ARG, 0, "thor_dec_create: frame size must be positive multiples of 8");
    return nullptr;
  }
  if (num_slots <= 1) num_slots = 34;  // 33 references + the frame being decoded
  if (num_slots > THOR_MAX_SLOTS) num_slots = THOR_MAX_SLOTS;
  if (hipSetDevice(device) != hipSuccess) {
    (void)hipGetLastError();
    create_fail(THOR_ERR_ARG, 0, "thor_dec_create: no HIP device %d", device);
    return nullptr;
  }
  thor_dec *d = new thor_dec();
  d->seq = *seq;
  d->device = device;
  int W = seq->width, H = seq->height;
  // The padding of create_yuv_frame (common/common_frame.c:324-351: 96 luma / 48
  // chroma on every side), laid out so that every row's pixel 0 sits on a 128-byte
  // line boundary: strides are multiples of 128 and each plane starts 32 / 80
  // bytes into its 256-aligned block.  k_recon's 128-pixel units then store whole
  // luma lines (inter.hip).
  d->sy = (W + 2 * THOR_PAD_Y + 127) & ~127;
  d->sc = (W / 2 + 2 * THOR_PAD_C + 127) & ~127;
  const int ylead = (128 - THOR_PAD_Y % 128) % 128, clead = (128 - THOR_PAD_C % 128) % 128;
  long long ybytes = ylead + (long long)(H + 2 * THOR_PAD_Y) * d->sy;
  long long cbytes = clead + (long long)(H / 2 + 2 * THOR_PAD_C) * d->sc;
  ybytes = (ybytes + 255) & ~255LL;
  cbytes = (cbytes + 255) & ~255LL;
  d->offy = ylead + (long long)THOR_PAD_Y * d->sy + THOR_PAD_Y;
  d->offu = ybytes + clead + (long long)THOR_PAD_C * d->sc + THOR_PAD_C;
  d->offv = ybytes + cbytes + clead + (long long)THOR_PAD_C * d->sc + THOR_PAD_C;
  d->slot_bytes = ybytes + 2 * cbytes + 256;
  if (d->slot_bytes * (num_slots + (seq->interp_ref ? 1 : 0)) >= (1LL << 31)) {  // k_recon addresses the ring with 32-bit buffer offsets
    create_fail(THOR_ERR_ARG, (size_t)(d->slot_bytes * (num_slots + (seq->interp_ref ? 1 : 0))),
                "thor_dec_create: a ring of %d slots of %lld bytes exceeds the 2 GiB a buffer descriptor addresses",
                num_slots, d->slot_bytes);
    delete d;
    return nullptr;
  }
  d->nslots = num_slots;
  d->islot = seq->interp_ref ? num_slots : -1;
  d->ti = nullptr;
  const int alloc_slots = num_slots + (seq->interp_ref ? 1 : 0);
  d->slot_fnum.assign(num_slots, -1);
  d->slot_age.assign(num_slots, -1);
  d->decode_count = 0;
  d->stop_stage = 2;
  d->progress = nullptr;
  d->resid = nullptr;
  d->edge = nullptr;
  d->hplan = nullptr;
  d->plan_gen = 0;
  d->dbg = nullptr;
  d->dbg_recon = nullptr;
  d->dbg_flags = 0;
  d->timing = 0;
  d->xev[0] = d->xev[1] = nullptr;
  d->band0 = d->band1 = 0;
  d->band_local = 0;
  d->band_pad = 0;
  d->band_intra = 0;
  d->pending_ended = 0;
  d->pending = nullptr;
  d->ev_used = 0;
  bool ok = hipStreamCreateWithFlags(&d->own_stream, hipStreamNonBlocking) == hipSuccess;
  if (!ok) create_fail(THOR_ERR_HIP, 0, "thor_dec_create: hipStreamCreate failed");
  d->stream = d->own_stream;
  ok = ok && dev_alloc(&d->slots, d->slot_bytes * alloc_slots, "thor_dec_create: reference ring");
  ok = ok && hipMemset(d->slots, 0, d->slot_bytes * alloc_slots) == hipSuccess;
  if (ok && seq->interp_ref) ok = (d->ti = thor_ti_create(W, H, device)) != nullptr;
  size_t ncell = (size_t)(W / 4) * (H / 4);
  ok = ok && dev_alloc(&d->cellinfo, ncell * sizeof(uint16_t), "thor_dec_create: cell side info");
  ok = ok && dev_alloc(&d->cellmc, ncell * sizeof(uint2), "thor_dec_create: cell MC words");
  ok = ok && hipMemset(d->cellmc, 0, ncell * sizeof(uint2)) == hipSuccess;
  ok = ok && dev_alloc(&d->cellmv1, ncell * sizeof(int32_t), "thor_dec_create: cell mv1");
  ok = ok && hipMemset(d->cellmv1, 0, ncell * sizeof(int32_t)) == hipSuccess;
  ok = ok && hipMemset(d->cellinfo, 0, ncell * sizeof(uint16_t)) == hipSuccess;
  ok = ok && dev_alloc(&d->ctl, 64, "thor_dec_create: control words");
  ok = ok && dev_alloc(&d->resid, (size_t)W * H * 3, "thor_dec_create: residual planes");  // 1.5 px/luma px x 2 B
  // intra progress words (3 per SB row), then the rows' intra-list segments (nrows + 1)
  ok = ok && dev_alloc(&d->progress, (size_t)4 * ((H + 63) / 64 + 2) * sizeof(unsigned), "thor_dec_create: progress");
  d->ewy = (W + 2 * EDGE_MARGIN + 15) & ~15;
  d->ewc = (W / 2 + 2 * EDGE_MARGIN + 15) & ~15;
  ok = ok && dev_alloc(&d->edge, (size_t)((H + 63) / 64) * (d->ewy + 2 * d->ewc), "thor_dec_create: edge rows");
  const size_t nplan = hplan_entries(W, H);  // per half-SB plans (common.h)
  ok = ok && dev_alloc(&d->hplan, nplan * sizeof(uint4), "thor_dec_create: half-SB plans");
  ok = ok && hipMemset(d->hplan, 0, nplan * sizeof(uint4)) == hipSuccess;  // tag 0: no plan (gen starts at 1)
  ok = ok && hipMemset(d->ctl, 0, 64) == hipSuccess;
  for (int i = 0; ok && i < 2; i++) ok = hipEventCreateWithFlags(&d->xev[i], hipEventDisableTiming) == hipSuccess;
  {  // k_intra stages a row's CU words in LDS (up to (W/8) x 8 CUs)
    size_t lds = (size_t)((W + 7) / 8) * 8 * sizeof(uint2);
    if (lds > 48 * 1024)
      ok = ok && hipFuncSetAttribute((const void *)k_intra, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) ==
                     hipSuccess;
  }
  if (!ok) {
    create_fail(THOR_ERR_HIP, 0, "thor_dec_create: HIP call failed");  // no-op when an allocation said why
    (void)hipGetLastError();
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
  if (d->cellmc) (void)hipFree(d->cellmc);
  if (d->cellmv1) (void)hipFree(d->cellmv1);
  if (d->ctl) (void)hipFree(d->ctl);
  if (d->progress) (void)hipFree(d->progress);
  if (d->resid) (void)hipFree(d->resid);
  if (d->edge) (void)hipFree(d->edge);
  if (d->hplan) (void)hipFree(d->hplan);
  if (d->ti) thor_ti_destroy(d->ti);
  for (int i = 0; i < 2; i++)
    if (d->xev[i]) (void)hipEventDestroy(d->xev[i]);
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
// Reads and clears the intra-chain timeout flag (ctl[1], set by k_intra when a
// wavefront wait gives up): each call reports only the timeouts since the last.
// Also reads and clears the missing-reference flag (ctl[2], set by k_frame_prep
// when an inter CU names a frame that is not resident in the ring).
static int check_timeout(thor_dec *d) {
  unsigned fl[2] = {0, 0};
  HIPCHK(hipMemcpy(fl, d->ctl + 1, sizeof(fl), hipMemcpyDeviceToHost));
  if (fl[0] | fl[1]) {
    const unsigned zero[2] = {0, 0};
    HIPCHK(hipMemcpy(d->ctl + 1, zero, sizeof(zero), hipMemcpyHostToDevice));
  }
  if (fl[1]) {
    fprintf(stderr, "thor_amd: a block references a frame that is not resident\n");
    return THOR_ERR_REF;
  }
  if (fl[0]) {
    fprintf(stderr, "thor_amd: intra dependency wait timed out\n");
    return THOR_ERR_HIP;
  }
  if (d->ti && thor_ti_status(d->ti) != THOR_OK) {
    fprintf(stderr, "thor_amd: interpolation search wait timed out\n");
    return THOR_ERR_HIP;
  }
  return THOR_OK;
}

int thor_dec_sync(thor_dec_t *d) {
  if (!d) return THOR_ERR_ARG;
  HIPCHK(hipStreamSynchronize(d->stream));
  return check_timeout(d);
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

// FrameCtx of the frame about to be decoded into slot `cur_slot`; the resident
// references are every other occupied slot.  Returns false if two resident
// frame numbers collide modulo 128 (k_recon's lookup table key).
static bool make_ctx(const thor_dec *d, int cur_slot, int frame_num, FrameCtx &f) {
  memset(&f, 0, sizeof(f));
  uint8_t *cur = d->slots + (long long)cur_slot * d->slot_bytes;
  f.cy = cur + d->offy;
  f.cu = cur + d->offu;
  f.cv = cur + d->offv;
  f.slots = d->slots;
  f.slot_bytes = d->slot_bytes;
  f.ring_bytes = d->slot_bytes * (d->nslots + (d->islot >= 0 ? 1 : 0));
  f.islot = -1;
  f.offy = d->offy;
  f.offu = d->offu;
  f.offv = d->offv;
  f.sy = d->sy;
  f.sc = d->sc;
  f.W = d->seq.width;
  f.H = d->seq.height;
  f.frame_num = frame_num;
  f.bipred = d->seq.bipred;
  f.edge = d->edge;
  f.ewy = d->ewy;
  f.ewc = d->ewc;
  f.nsbrows = (d->seq.height + 63) / 64;
  f.cellinfo = d->cellinfo;
  f.cellmc = d->cellmc;
  f.cellmv1 = d->cellmv1;
  f.resid = d->resid;
  f.ctl = d->ctl;
  f.progress = d->progress;
  f.rowstart = (int *)(d->progress + 3 * (f.nsbrows + 1));
  int8_t lut[128];
  memset(lut, -1, sizeof(lut));
  f.nref = 0;
  for (int s = 0; s < d->nslots; s++) {
    if (s == cur_slot || d->slot_fnum[s] < 0) continue;
    const int k = d->slot_fnum[s] & 127;
    if (lut[k] >= 0) return false;
    lut[k] = (int8_t)s;
    f.nref++;
  }
  memcpy(f.slot_lut, lut, sizeof(lut));
  return true;
}

static int dec_frames_chunk(thor_dec_t *const *ds, int n, const thor_frame_hdr_t *hdrs, const thor_frame_in_t *ins);

int thor_dec_frames(thor_dec_t *const *ds, int n, const thor_frame_hdr_t *hdrs, const thor_frame_in_t *ins) {
  if (!ds || !hdrs || !ins || n <= 0) return THOR_ERR_ARG;
  for (int i = 0; i < n; i++) {
    if (!ds[i]) return THOR_ERR_ARG;
    // a band-local context decodes through thor_dec_frame_begin / _end / _finish only; rejected here,
    // before any chunk is enqueued, so a refused call leaves no frame half decoded
    if (ds[i]->band_local && ds[i]->band1 > 0) return THOR_ERR_ARG;
    for (int j = 0; j < i; j++)
      if (ds[i] == ds[j]) return THOR_ERR_ARG;  // one frame per context per call (a stream's frames are serial)
  }
  for (int o = 0; o < n; o += THOR_MAX_BATCH) {  // THOR_MAX_BATCH frames per launch
    const int rc = dec_frames_chunk(ds + o, n - o < THOR_MAX_BATCH ? n - o : THOR_MAX_BATCH, hdrs + o, ins + o);
    if (rc != THOR_OK) return rc;
  }
  return THOR_OK;
}

// A prepared batch: FrameCtx per frame + launch geometry.
struct Batch {
  FrameBatch fb;
  int n, cur[THOR_MAX_BATCH], frame_num[THOR_MAX_BATCH];
  // interpolated reference per frame: source slots (-1: none) and interpolate_frames' (ratio, pos)
  int ia[THOR_MAX_BATCH], ib[THOR_MAX_BATCH], iratio[THOR_MAX_BATCH], ipos[THOR_MAX_BATCH];
  int max_prep, any_intra, any_clpf, any_deblock, clpf_grid, max_intra, max_slow;
  int intra_done;  // thor_dec_frame_intra ran the intra stage already
};

static int batch_prepare(thor_dec_t *const *ds, int n, const thor_frame_hdr_t *hdrs, const thor_frame_in_t *ins,
                         Batch &b) {
  thor_dec *lead = ds[0];
  if (!lead) return THOR_ERR_ARG;
  const int W = lead->seq.width, H = lead->seq.height;
  for (int i = 0; i < n; i++) {
    const thor_dec *d = ds[i];
    const thor_frame_in_t &in = ins[i];
    if (!d || d->device != lead->device || d->seq.width != W || d->seq.height != H) return THOR_ERR_ARG;
    if (d->pending) return THOR_ERR_ARG;  // a thor_dec_frame_begin without its _end
    if (in.nblocks < 0 || (in.nblocks > 0 && !in.blocks)) return THOR_ERR_ARG;
    if (in.n_intra < 0 || (in.n_intra > 0 && !in.intra_list)) return THOR_ERR_ARG;
    if (in.n_tu < 0 || (in.n_tu > 0 && (!in.tu_list || !in.coeffs))) return THOR_ERR_ARG;
    if (in.slow_list && (in.n_slow < 0 || in.n_slow > unit_count(W, H))) return THOR_ERR_ARG;
  }
  memset(&b.fb, 0, sizeof(b.fb));
  b.n = n;
  b.intra_done = 0;
  b.max_prep = 1;
  b.any_intra = b.any_clpf = b.any_deblock = 0;
  b.clpf_grid = 0;
  b.max_intra = 0;
  b.max_slow = 0;
  for (int i = 0; i < n; i++) {
    thor_dec *d = ds[i];
    const thor_frame_in_t &in = ins[i];
    b.cur[i] = pick_slot(d, hdrs[i].frame_num);
    b.frame_num[i] = hdrs[i].frame_num;
    FrameCtx &f = b.fb.f[i];
    if (!make_ctx(d, b.cur[i], hdrs[i].frame_num, f)) return THOR_ERR_REF;
    b.ia[i] = b.ib[i] = -1;
    b.iratio[i] = b.ipos[i] = 0;
    if (hdrs[i].interp_ratio > 0) {  // dec/decode_frame.c:91-109
      if (!d->ti || hdrs[i].interp_pos < 0) return THOR_ERR_ARG;
      b.ia[i] = find_slot_host(d, hdrs[i].interp_ref[0]);
      b.ib[i] = find_slot_host(d, hdrs[i].interp_ref[1]);
      if (b.ia[i] < 0 || b.ib[i] < 0 || b.ia[i] == b.cur[i] || b.ib[i] == b.cur[i]) return THOR_ERR_REF;
      b.iratio[i] = hdrs[i].interp_ratio;
      b.ipos[i] = hdrs[i].interp_pos;
      f.islot = d->islot;
    }
    f.hplan = d->hplan;
    if (++d->plan_gen == 0) d->plan_gen = 1;  // tag 0 marks "no plan"
    f.gen = (int)d->plan_gen;
    f.slow = in.slow_list;
    f.nslow = in.slow_list ? in.n_slow : 0;
    b.max_slow = b.max_slow > f.nslow ? b.max_slow : f.nslow;
    f.blk = in.blocks;
    f.coeffs = in.coeffs;
    f.tus = in.tu_list;
    f.ilist = in.intra_list;
    f.clpf_flags = in.clpf_flags;
    f.clpf_list = in.clpf_list;
    f.n_clpf = in.clpf_list ? in.n_clpf : -1;
    f.nblocks = in.nblocks;
    f.ntus = in.n_tu;
    f.nintra = in.n_intra;
    f.nprep = (in.nblocks + 4 * PREP_CPW - 1) / (4 * PREP_CPW);  // workgroups of 4 waves x PREP_CPW CUs (prep_body)
    f.nres = (in.n_tu + 3) / 4;
    f.full_sb = in.n_intra < in.nblocks;  // full SB images only when inter CUs were reconstructed
    f.qp = hdrs[i].qp;
    f.qpc = chroma_qp_host(hdrs[i].qp);
    f.deblock = d->stop_stage >= 1 && d->seq.deblocking;
    f.clpf_on = d->stop_stage >= 2 && d->seq.clpf && hdrs[i].clpf_on && in.clpf_flags;
    f.band0 = d->band0;
    f.band1 = d->band1 > 0 ? d->band1 : f.nsbrows;
    f.pb0 = f.pb1 = 0;
    f.ir0 = 0;
    f.ir1 = 0;
    if (d->band_intra && d->band1 > 0) {
      f.ir0 = d->band0;
      f.ir1 = d->band1 > d->band0 ? d->band1 : d->band0;
      if (f.ir1 == f.ir0) f.nintra = 0;  // an empty band: no chains
    }
    if (d->band_local && d->band1 > 0) {
      f.pb0 = d->band0 * 64;
      f.pb1 = d->band1 * 64 < H ? d->band1 * 64 : H;
      if (f.pb1 <= f.pb0) f.pb0 = f.pb1 = H;  // an empty band: nothing to filter (pb1 > 0 keeps it band-local)
    }
    b.max_prep = b.max_prep > f.nprep + f.nres + 1 ? b.max_prep : f.nprep + f.nres + 1;
    b.any_intra |= in.n_intra > 0;
    b.max_intra = b.max_intra > in.n_intra ? b.max_intra : in.n_intra;
    if (f.clpf_on) {
      const int w = f.n_clpf >= 0 ? f.n_clpf : (W / 64) * (H / 64);
      b.clpf_grid = b.clpf_grid > w ? b.clpf_grid : w;
    }
    b.any_clpf |= f.clpf_on;
    b.any_deblock |= f.deblock;
  }
  return THOR_OK;
}

// Diagnostic: extra dynamic LDS per k_recon workgroup (bytes) to cap its
// occupancy (THOR_RECON_LDS_PAD; 0 in the product path).
static int recon_lds_pad() {
  static int v = [] {
    const char *e = getenv("THOR_RECON_LDS_PAD");
    return e ? atoi(e) : 0;
  }();
  return v;
}

static thor_yuv_planes_t slot_planes(const thor_dec *d, int s) {
  uint8_t *base = d->slots + (long long)s * d->slot_bytes;
  return thor_yuv_planes_t{base + d->offy, base + d->offu, base + d->offv, d->sy, d->sc};
}

// The frames' temporal-interpolated references (interpolate_frames + pad_yuv_frame,
// dec/decode_frame.c:106-107) into their contexts' interpolation slots.
static int batch_interp(thor_dec_t *const *ds, const Batch &b) {
  hipStream_t st = ds[0]->stream;
  for (int i = 0; i < b.n; i++) {
    if (b.iratio[i] <= 0) continue;
    thor_dec *d = ds[i];
    StageMark m(ds[0], ST_INTERP);
    const thor_yuv_planes_t ra = slot_planes(d, b.ia[i]), rb = slot_planes(d, b.ib[i]), o = slot_planes(d, d->islot);
    const int rc = thor_interpolate_frames(d->ti, &ra, &rb, THOR_PAD_Y, &o, b.iratio[i], b.ipos[i], st);
    if (rc != THOR_OK) return rc;
    FrameBatch fb;
    memset(&fb, 0, sizeof(fb));
    fb.f[0].cy = o.y;
    fb.f[0].cu = o.u;
    fb.f[0].cv = o.v;
    fb.f[0].sy = d->sy;
    fb.f[0].sc = d->sc;
    fb.f[0].W = d->seq.width;
    fb.f[0].H = d->seq.height;
    k_pad<<<dim3((pad_chunks(d->seq.width, d->seq.height) + 255) / 256, 1), 256, 0, st>>>(fb, 0, 0);
    HIPCHK(hipGetLastError());
  }
  return THOR_OK;
}

// Phase A: side info, residuals, intra setup, inter reconstruction (the SB
// rows of each context's band).
static int batch_phase_a(thor_dec *lead, const Batch &b) {
  const int W = lead->seq.width, H = lead->seq.height, n = b.n;
  hipStream_t st = lead->stream;
  {
    // side info + residuals of every coded transform block + intra chain setup
    StageMark m(lead, ST_PREP);
    k_frame_prep<<<dim3(b.max_prep, n), 256, 0, st>>>(b.fb);
    HIPCHK(hipGetLastError());
  }
  {
    StageMark m(lead, ST_INTER);  // k_recon alone: the inter-reconstruction roofline kernel
    // one flat grid: every frame's slow-list units first (frame-interleaved, as
    // many slots as the longest list), then each frame's units in XCD-major order
    // (inter.hip)
    ReconGeo g;
    g.nfr = n;
    g.maxslow = b.max_slow;
    g.nu = unit_count(W, H);
    g.NU = 8 * ((g.nu + 7) / 8);
    g.np = unit_pairs(W);
    g.mnfr = recon_recip((unsigned)g.nfr);
    g.mNU = recon_recip((unsigned)g.NU);
    g.mnp = recon_recip((unsigned)g.np);
    memcpy(g.tl, k_taps.luma, sizeof(g.tl));
    memcpy(g.tc, k_taps.chroma, sizeof(g.tc));
    k_recon<<<dim3(n * (b.max_slow + g.NU), 1), 64, recon_lds_pad(), st>>>(b.fb, g, lead->dbg_recon);
    HIPCHK(hipGetLastError());
  }
  return THOR_OK;
}

// Phase B: intra, deblock, CLPF, reference padding (pad = 0: the band-local
// form, padded by thor_dec_frame_finish after the final-rows exchange).
static int batch_intra(thor_dec *lead, const Batch &b) {
  const int W = lead->seq.width, H = lead->seq.height, n = b.n;
  const int nrows = (H + 63) / 64;
  if (b.any_intra && !b.intra_done) {
    StageMark m(lead, ST_INTRA);
    // one single-wave chain per (SB row, component); LDS holds the row's CU words
    size_t lds = (size_t)((W + 7) / 8) * 8 * sizeof(uint2);
    k_intra<<<dim3(3 * nrows, n), 64, lds, lead->stream>>>(b.fb, lead->dbg, lead->dbg_flags);
    HIPCHK(hipGetLastError());
  }
  return THOR_OK;
}

static int batch_phase_b(thor_dec *lead, const Batch &b, int pad = 1) {
  const int W = lead->seq.width, H = lead->seq.height, n = b.n;
  hipStream_t st = lead->stream;
  const int rc = batch_intra(lead, b);
  if (rc != THOR_OK) return rc;
  if (b.any_deblock) {
    StageMark m(lead, ST_DEBLOCK);
    int nv = ((W >> 3) - 1) * (H >> 3);
    int nh = (W >> 3) * ((H >> 3) - 1);
    // luma and both chroma planes of one edge direction per launch
    const int bv = (nv + 256 * DB_ITEMS - 1) / (256 * DB_ITEMS), bh = (nh + 256 * DB_ITEMS - 1) / (256 * DB_ITEMS);
    // chroma: with few intra CUs (P frames) one (intra CU, plane) item per wave,
    // else every chroma edge segment like luma
    const int clist = b.max_intra <= 1024;
    const int bc = clist ? (2 * b.max_intra + 3) / 4 : 0;
    k_deblock_v<<<dim3(clist ? bv + bc : 3 * bv, n), 256, 0, st>>>(b.fb, bv, clist);
    k_deblock_h<<<dim3(clist ? bh + bc : 3 * bh, n), 256, 0, st>>>(b.fb, bh, clist);
    HIPCHK(hipGetLastError());
  }
  if (b.any_clpf && b.clpf_grid > 0) {
    StageMark m(lead, ST_CLPF);
    k_clpf<<<dim3(b.clpf_grid, n), 256, 0, st>>>(b.fb);
    HIPCHK(hipGetLastError());
  }
  if (pad) {
    StageMark m(lead, ST_PAD);
    k_pad<<<dim3((pad_chunks(W, H) + 255) / 256, n), 256, 0, st>>>(b.fb, 0, 0);
    HIPCHK(hipGetLastError());
  }
  return THOR_OK;
}

static void batch_commit(thor_dec_t *const *ds, const Batch &b) {
  for (int i = 0; i < b.n; i++) {
    ds[i]->slot_fnum[b.cur[i]] = b.frame_num[i];
    ds[i]->slot_age[b.cur[i]] = ds[i]->decode_count++;
  }
}

static int dec_frames_chunk(thor_dec_t *const *ds, int n, const thor_frame_hdr_t *hdrs, const thor_frame_in_t *ins) {
  thor_dec *lead = ds[0];
  for (int i = 0; i < n; i++)  // band-local phase B needs the begin / end / finish protocol
    if (ds[i]->band_local && ds[i]->band1 > 0) return THOR_ERR_ARG;
  Batch b;
  int rc = batch_prepare(ds, n, hdrs, ins, b);
  if (rc != THOR_OK) return rc;
  HIPCHK(hipSetDevice(lead->device));
  hipStream_t st = lead->stream;
  // order the batch after each member context's earlier work on other streams
  for (int i = 1; i < n; i++)
    if (ds[i]->stream != st) {
      HIPCHK(hipEventRecord(lead->xev[0], ds[i]->stream));
      HIPCHK(hipStreamWaitEvent(st, lead->xev[0], 0));
    }
  if ((rc = batch_interp(ds, b)) != THOR_OK) return rc;
  if ((rc = batch_phase_a(lead, b)) != THOR_OK) return rc;
  if ((rc = batch_phase_b(lead, b)) != THOR_OK) return rc;
  // later work a member context enqueues on its own stream follows this batch
  bool rec = false;
  for (int i = 1; i < n; i++)
    if (ds[i]->stream != st) {
      if (!rec) HIPCHK(hipEventRecord(lead->xev[1], st));
      rec = true;
      HIPCHK(hipStreamWaitEvent(ds[i]->stream, lead->xev[1], 0));
    }
  batch_commit(ds, b);
  return THOR_OK;
}

// ---- row-band sharding ------------------------------
int thor_dec_set_band(thor_dec_t *d, int sb_row0, int sb_row1) {
  if (!d) return THOR_ERR_ARG;
  const int nrows = (d->seq.height + 63) / 64;
  if (sb_row0 < 0 || sb_row1 < sb_row0 || sb_row1 > nrows) return THOR_ERR_ARG;
  d->band0 = sb_row0;
  d->band1 = sb_row1 == 0 && sb_row0 == 0 ? 0 : sb_row1;
  return THOR_OK;
}

int thor_dec_set_band_local(thor_dec_t *d, int on) {
  if (!d || d->pending) return THOR_ERR_ARG;
  d->band_local = on != 0;
  return THOR_OK;
}

int thor_dec_set_band_pad(thor_dec_t *d, int on) {
  if (!d || d->pending) return THOR_ERR_ARG;
  d->band_pad = on != 0;
  return THOR_OK;
}

int thor_dec_set_band_intra(thor_dec_t *d, int on) {
  if (!d || d->pending) return THOR_ERR_ARG;
  d->band_intra = on != 0;
  return THOR_OK;
}

int thor_dec_frame_intra(thor_dec_t *d) {
  if (!d || !d->pending || d->pending_ended) return THOR_ERR_ARG;
  Batch *b = (Batch *)d->pending;
  HIPCHK(hipSetDevice(d->device));
  const int rc = batch_intra(d, *b);
  if (rc == THOR_OK) b->intra_done = 1;
  return rc;
}

int thor_dec_frame_begin(thor_dec_t *d, const thor_frame_hdr_t *hdr, const thor_frame_in_t *in) {
  if (!d || !hdr || !in || d->pending) return THOR_ERR_ARG;
  Batch *b = new Batch();
  thor_dec_t *ds[1] = {d};
  int rc = batch_prepare(ds, 1, hdr, in, *b);
  if (rc == THOR_OK) {
    if (hipSetDevice(d->device) != hipSuccess) rc = THOR_ERR_HIP;
    else if ((rc = batch_interp(ds, *b)) == THOR_OK) rc = batch_phase_a(d, *b);
  }
  if (rc != THOR_OK) {
    delete b;
    return rc;
  }
  d->pending = b;
  return THOR_OK;
}

int thor_dec_frame_end(thor_dec_t *d) {
  if (!d || !d->pending || d->pending_ended) return THOR_ERR_ARG;
  Batch *b = (Batch *)d->pending;
  HIPCHK(hipSetDevice(d->device));
  const int local = b->fb.f[0].pb1 > 0;
  int rc = batch_phase_b(d, *b, !local);
  if (rc == THOR_OK && local) {  // the final-rows exchange, then thor_dec_frame_finish
    d->pending_ended = 1;
    return THOR_OK;
  }
  thor_dec_t *ds[1] = {d};
  if (rc == THOR_OK) batch_commit(ds, *b);
  d->pending = nullptr;
  delete b;
  return rc;
}

int thor_dec_frame_finish(thor_dec_t *d) {
  if (!d || !d->pending || !d->pending_ended) return THOR_ERR_ARG;
  Batch *b = (Batch *)d->pending;
  HIPCHK(hipSetDevice(d->device));
  const int W = d->seq.width, H = d->seq.height;
  int rc = THOR_OK;
  // the whole frame, or (thor_dec_set_band_pad) only the band's rows -- the only ones final here
  const FrameCtx &f = b->fb.f[0];
  const int r0 = d->band_pad ? f.pb0 : 0, r1 = d->band_pad ? f.pb1 : 0;
  if (!d->band_pad || r1 > r0) {
    StageMark m(d, ST_PAD);
    k_pad<<<dim3((pad_chunks(W, H, r0, r1) + 255) / 256, 1), 256, 0, d->stream>>>(b->fb, r0, r1);
    if (hipGetLastError() != hipSuccess) rc = THOR_ERR_HIP;
  }
  thor_dec_t *ds[1] = {d};
  if (rc == THOR_OK) batch_commit(ds, *b);
  d->pending = nullptr;
  d->pending_ended = 0;
  delete b;
  return rc;
}

// Rows [y0, y0 + nrows) of luma (and the matching chroma rows) of the frame in
// `frame_num`'s slot, or of the frame begun and not yet ended, packed as
// Y (nrows x W) | U (nrows/2 x W/2) | V; rows past the frame are skipped.
static int band_slot(thor_dec *d, int frame_num) {
  if (d->pending) {
    Batch *b = (Batch *)d->pending;
    if (b->frame_num[0] == frame_num) return b->cur[0];
  }
  return find_slot_host(d, frame_num);
}

int thor_dec_get_rows(thor_dec_t *d, int frame_num, int y0, int nrows, void *dst) {
  if (!d || !dst || y0 < 0 || nrows <= 0 || (y0 & 1) || (nrows & 1)) return THOR_ERR_ARG;
  const int s = band_slot(d, frame_num);
  if (s < 0) return THOR_ERR_REF;
  const int W = d->seq.width, H = d->seq.height;
  const int n = y0 + nrows > H ? H - y0 : nrows;
  if (n <= 0) return THOR_OK;
  const uint8_t *base = d->slots + (long long)s * d->slot_bytes;
  uint8_t *o = (uint8_t *)dst;
  HIPCHK(hipSetDevice(d->device));
  HIPCHK(hipMemcpy2DAsync(o, W, base + d->offy + (long long)y0 * d->sy, d->sy, W, n, hipMemcpyDeviceToDevice, d->stream));
  o += (long long)nrows * W;
  for (int c = 0; c < 2; c++) {
    const long long off = (c ? d->offv : d->offu) + (long long)(y0 / 2) * d->sc;
    HIPCHK(hipMemcpy2DAsync(o, W / 2, base + off, d->sc, W / 2, n / 2, hipMemcpyDeviceToDevice, d->stream));
    o += (long long)(nrows / 2) * (W / 2);
  }
  return THOR_OK;
}

int thor_dec_put_rows(thor_dec_t *d, int frame_num, int y0, int nrows, const void *src) {
  if (!d || !src || y0 < 0 || nrows <= 0 || (y0 & 1) || (nrows & 1)) return THOR_ERR_ARG;
  const int s = band_slot(d, frame_num);
  if (s < 0) return THOR_ERR_REF;
  const int W = d->seq.width, H = d->seq.height;
  const int n = y0 + nrows > H ? H - y0 : nrows;
  if (n <= 0) return THOR_OK;
  uint8_t *base = d->slots + (long long)s * d->slot_bytes;
  const uint8_t *i = (const uint8_t *)src;
  HIPCHK(hipSetDevice(d->device));
  HIPCHK(hipMemcpy2DAsync(base + d->offy + (long long)y0 * d->sy, d->sy, i, W, W, n, hipMemcpyDeviceToDevice, d->stream));
  // the intra chains read SB-row bottom rows from the edge buffer (k_recon
  // writes the inter pixels there for its own band): refresh every SB row
  // whose bottom row this band carries
  const int sb0 = y0 / 64, sb1 = (y0 + n) / 64;  // SB rows whose row 63 lies inside [y0, y0 + n)
  const long long r63 = 64LL * sb0 + 63 - y0;     // that row of SB row sb0, in the source
  if (sb1 > sb0)
    HIPCHK(hipMemcpy2DAsync(d->edge + (long long)sb0 * d->ewy + EDGE_MARGIN, d->ewy, i + r63 * W, 64LL * W, W,
                            sb1 - sb0, hipMemcpyDeviceToDevice, d->stream));
  i += (long long)nrows * W;
  const int nsbrows = (H + 63) / 64;
  for (int c = 0; c < 2; c++) {
    const long long off = (c ? d->offv : d->offu) + (long long)(y0 / 2) * d->sc;
    HIPCHK(hipMemcpy2DAsync(base + off, d->sc, i, W / 2, W / 2, n / 2, hipMemcpyDeviceToDevice, d->stream));
    if (sb1 > sb0)
      HIPCHK(hipMemcpy2DAsync(d->edge + (long long)nsbrows * d->ewy + (long long)c * nsbrows * d->ewc +
                                  (long long)sb0 * d->ewc + EDGE_MARGIN,
                              d->ewc, i + (r63 / 2) * (W / 2), 32LL * (W / 2), W / 2, sb1 - sb0, hipMemcpyDeviceToDevice,
                              d->stream));
    i += (long long)(nrows / 2) * (W / 2);
  }
  return THOR_OK;
}

int thor_dec_frame(thor_dec_t *d, const thor_frame_hdr_t *hdr, const thor_block_t *blocks, int nblocks,
                   const int16_t *coeffs, const uint8_t *clpf_flags, const uint32_t *intra_list, int n_intra,
                   const thor_tu_t *tu_list, int n_tu) {
  if (!d || !hdr) return THOR_ERR_ARG;
  thor_frame_in_t in = {blocks, nblocks, coeffs, clpf_flags, intra_list, n_intra, tu_list, n_tu, nullptr, -1, nullptr, 0};
  return thor_dec_frames(&d, 1, hdr, &in);
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

int thor_dec_read_frame(thor_dec_t *d, int frame_num, uint8_t *y, uint8_t *u, uint8_t *v) {
  if (!d) return THOR_ERR_ARG;
  int s = find_slot_host(d, frame_num);
  if (s < 0) return THOR_ERR_REF;
  HIPCHK(hipSetDevice(d->device));
  HIPCHK(hipStreamSynchronize(d->stream));
  {
    const int rc = check_timeout(d);  // a frame whose intra chains timed out is not returned as valid
    if (rc != THOR_OK) return rc;
  }
  int W = d->seq.width, H = d->seq.height;
  const uint8_t *base = d->slots + (long long)s * d->slot_bytes;
  if (y) HIPCHK(hipMemcpy2D(y, W, base + d->offy, d->sy, W, H, hipMemcpyDeviceToHost));
  if (u) HIPCHK(hipMemcpy2D(u, W / 2, base + d->offu, d->sc, W / 2, H / 2, hipMemcpyDeviceToHost));
  if (v) HIPCHK(hipMemcpy2D(v, W / 2, base + d->offv, d->sc, W / 2, H / 2, hipMemcpyDeviceToHost));
  return THOR_OK;
}

int thor_dec_put_ref_rows(thor_dec_t *d, int frame_num, int y0, int nrows, const void *src) {
  if (!d || !src || y0 < 0 || nrows <= 0 || (y0 & 1) || (nrows & 1)) return THOR_ERR_ARG;
  const int s = find_slot_host(d, frame_num);  // a resident reference, not the frame being decoded
  if (s < 0) return THOR_ERR_REF;
  const int W = d->seq.width, H = d->seq.height;
  const int n = y0 + nrows > H ? H - y0 : nrows;
  if (n <= 0) return THOR_OK;
  uint8_t *base = d->slots + (long long)s * d->slot_bytes;
  const uint8_t *i = (const uint8_t *)src;
  HIPCHK(hipSetDevice(d->device));
  HIPCHK(hipMemcpy2DAsync(base + d->offy + (long long)y0 * d->sy, d->sy, i, W, W, n, hipMemcpyDeviceToDevice, d->stream));
  i += (long long)nrows * W;
  for (int c = 0; c < 2; c++) {
    const long long off = (c ? d->offv : d->offu) + (long long)(y0 / 2) * d->sc;
    HIPCHK(hipMemcpy2DAsync(base + off, d->sc, i, W / 2, W / 2, n / 2, hipMemcpyDeviceToDevice, d->stream));
    i += (long long)(nrows / 2) * (W / 2);
  }
  return THOR_OK;
}

int thor_dec_pad_frame(thor_dec_t *d, int frame_num) {
  if (!d) return THOR_ERR_ARG;
  const int s = find_slot_host(d, frame_num);
  if (s < 0) return THOR_ERR_REF;
  const int W = d->seq.width, H = d->seq.height;
  uint8_t *base = d->slots + (long long)s * d->slot_bytes;
  FrameBatch fb;
  memset(&fb, 0, sizeof(fb));
  FrameCtx *hp = fb.f;
  hp->cy = base + d->offy;
  hp->cu = base + d->offu;
  hp->cv = base + d->offv;
  hp->sy = d->sy;
  hp->sc = d->sc;
  hp->W = W;
  hp->H = H;
  HIPCHK(hipSetDevice(d->device));
  k_pad<<<dim3((pad_chunks(W, H) + 255) / 256, 1), 256, 0, d->stream>>>(fb, 0, 0);
  HIPCHK(hipGetLastError());
  return THOR_OK;
}

int thor_dec_write_frame(thor_dec_t *d, int frame_num, const uint8_t *y, const uint8_t *u, const uint8_t *v) {
  if (!d || !y || !u || !v || d->pending) return THOR_ERR_ARG;
  HIPCHK(hipSetDevice(d->device));
  HIPCHK(hipStreamSynchronize(d->stream));  // in-flight kernels may still read the slot being replaced
  int s = find_slot_host(d, frame_num);
  if (s < 0) s = pick_slot(d, frame_num);
  int W = d->seq.width, H = d->seq.height;
  uint8_t *base = d->slots + (long long)s * d->slot_bytes;
  HIPCHK(hipMemcpy2D(base + d->offy, d->sy, y, W, W, H, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy2D(base + d->offu, d->sc, u, W / 2, W / 2, H / 2, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy2D(base + d->offv, d->sc, v, W / 2, W / 2, H / 2, hipMemcpyHostToDevice));
  {
    FrameBatch fb;
    memset(&fb, 0, sizeof(fb));
    FrameCtx *hp = fb.f;
    hp->cy = base + d->offy;
    hp->cu = base + d->offu;
    hp->cv = base + d->offv;
    hp->sy = d->sy;
    hp->sc = d->sc;
    hp->W = W;
    hp->H = H;
    k_pad<<<dim3((pad_chunks(W, H) + 255) / 256, 1), 256, 0, d->stream>>>(fb, 0, 0);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipStreamSynchronize(d->stream));
  d->slot_fnum[s] = frame_num;
  d->slot_age[s] = d->decode_count++;
  return THOR_OK;
}

}  // extern "C"
