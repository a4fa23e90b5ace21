/*
 * TEST INFRASTRUCTURE ONLY -- never linked into the product library.
 *
 * Link-time hooks (-Wl,--wrap=...) that turn the *unmodified* reference
 * decoder (dec/*.c + common/*.c compiled from /root/reference by
 * oracle/Makefile) into a trace recorder.  No reference source is edited or
 * copied; every hook calls straight through to the reference function
 * (__real_*) and only observes arguments / results.
 *
 * Hooked cross-TU calls:
 *   decode_frame            dec/decode_frame.c:45   (called from dec/maindec.c:169)
 *   read_block              dec/read_bits.c:221     (called from dec/decode_block.c:231)
 *   deblock_frame_y         common/common_frame.c:46 (called from dec/decode_frame.c:125)
 *   clpf_frame              common/common_frame.c:485 (called from dec/decode_frame.c:131)
 *   create_reference_frame  common/common_frame.c:464 (called from dec/decode_frame.c:147)
 *
 * Output (env THOR_TRACE=<file>): the per-frame block-descriptor trace that the
 * GPU batched path replays (format: thor_amd/trace.py).
 * Optional (env THOR_TRACE_DUMP=<dir>): raw I420 dumps of every frame at three
 * stages -- pre-deblock, post-deblock (pre-CLPF), final -- used to pin the
 * oracle stage by stage.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>

#include "global.h"
#include "types.h"
#include "maindec.h"
#include "common_frame.h"
#include "read_bits.h"

void __real_decode_frame(decoder_info_t *decoder_info, yuv_frame_t *rec_buffer);
int __real_read_block(decoder_info_t *decoder_info, stream_t *stream, block_info_dec_t *block_info, frame_type_t frame_type);
void __real_deblock_frame_y(yuv_frame_t *rec, deblock_data_t *deblock_data, int width, int height, uint8_t qp);
void __real_clpf_frame(yuv_frame_t *rec, yuv_frame_t *org, const deblock_data_t *deblock_data, void *stream,
                       int (*decision)(int, int, yuv_frame_t *, yuv_frame_t *, const deblock_data_t *, int, void *));
void __real_create_reference_frame(yuv_frame_t *ref, yuv_frame_t *rec);

static FILE *g_trace = NULL;
static const char *g_dump = NULL;
static int g_init = 0;
static int g_decode_order = 0;

/* growable per-frame buffers */
static uint8_t *g_blk = NULL;
static size_t g_blk_len = 0, g_blk_cap = 0;
static uint32_t g_nblocks = 0;
static uint8_t g_clpf[4096];
static int g_clpf_on = 0;
static int g_nsb = 0;
static int g_stage_post_deblock_done = 0;
static decoder_info_t *g_dec = NULL;

static void buf_put(const void *p, size_t n) {
  if (g_blk_len + n > g_blk_cap) {
    g_blk_cap = (g_blk_len + n) * 2 + 65536;
    g_blk = realloc(g_blk, g_blk_cap);
  }
  memcpy(g_blk + g_blk_len, p, n);
  g_blk_len += n;
}

static void put_u32(FILE *f, uint32_t v) { fwrite(&v, 4, 1, f); }

static void dump_frame(yuv_frame_t *fr, const char *stage) {
  if (!g_dump) return;
  char path[1024];
  snprintf(path, sizeof(path), "%s/f%03d_%s.yuv", g_dump, g_decode_order, stage);
  FILE *f = fopen(path, "wb");
  if (!f) return;
  int w = fr->width, h = fr->height;
  for (int i = 0; i < h; i++) fwrite(fr->y + i * fr->stride_y, 1, w, f);
  for (int i = 0; i < h / 2; i++) fwrite(fr->u + i * fr->stride_c, 1, w / 2, f);
  for (int i = 0; i < h / 2; i++) fwrite(fr->v + i * fr->stride_c, 1, w / 2, f);
  fclose(f);
}

static void init_once(decoder_info_t *d) {
  if (g_init) return;
  g_init = 1;
  const char *p = getenv("THOR_TRACE");
  g_dump = getenv("THOR_TRACE_DUMP");
  if (p) g_trace = fopen(p, "wb");
  if (g_trace) {
    fwrite("THTR", 1, 4, g_trace);
    put_u32(g_trace, 1);
    uint16_t wh[2] = {(uint16_t)d->width, (uint16_t)d->height};
    fwrite(wh, 2, 2, g_trace);
    uint8_t seq[12] = {(uint8_t)d->pb_split, (uint8_t)d->tb_split_enable, (uint8_t)d->max_num_ref,
                       (uint8_t)d->interp_ref, (uint8_t)d->max_delta_qp, (uint8_t)d->deblocking,
                       (uint8_t)d->clpf, (uint8_t)d->use_block_contexts, (uint8_t)d->bipred, 0, 0, 0};
    fwrite(seq, 1, 12, g_trace);
  }
}

static int ref_frame_num(decoder_info_t *d, int ref_idx) {
  if (ref_idx < 0 || ref_idx >= d->frame_info.num_ref) return -1;
  int r = d->frame_info.ref_array[ref_idx];
  if (r < 0) return -2; /* interpolated reference (config 5 only) */
  return d->ref[r]->frame_num;
}

static int any_nonzero(const int16_t *c, int n) {
  for (int i = 0; i < n; i++) if (c[i]) return 1;
  return 0;
}

int __wrap_read_block(decoder_info_t *d, stream_t *stream, block_info_dec_t *bi, frame_type_t frame_type) {
  int ret = __real_read_block(d, stream, bi, frame_type);
  if (!g_trace) return ret;
  block_param_t *bp = &bi->block_param;
  int size = bi->block_pos.size;
  int sizeC = size / 2;
  uint8_t mask = 0;
  int coded = bp->mode != MODE_SKIP;
  if (coded && any_nonzero(bi->coeffq_y, size * size)) mask |= 1;
  if (coded && any_nonzero(bi->coeffq_u, sizeC * sizeC)) mask |= 2;
  if (coded && any_nonzero(bi->coeffq_v, sizeC * sizeC)) mask |= 4;
  uint8_t hdr[20];
  uint16_t ypos = bi->block_pos.ypos, xpos = bi->block_pos.xpos;
  memcpy(hdr + 0, &ypos, 2);
  memcpy(hdr + 2, &xpos, 2);
  hdr[4] = (uint8_t)size;
  hdr[5] = bi->block_pos.bwidth;
  hdr[6] = bi->block_pos.bheight;
  hdr[7] = (uint8_t)bp->mode;
  hdr[8] = (uint8_t)bp->intra_mode;
  hdr[9] = (uint8_t)bp->tb_split;
  hdr[10] = (uint8_t)bp->pb_part;
  hdr[11] = (uint8_t)bp->dir;
  hdr[12] = (uint8_t)d->frame_info.qpb;
  hdr[13] = (uint8_t)bi->cbp.y;
  hdr[14] = (uint8_t)bi->cbp.u;
  hdr[15] = (uint8_t)bi->cbp.v;
  hdr[16] = mask;
  hdr[17] = hdr[18] = hdr[19] = 0;
  buf_put(hdr, 20);
  int16_t mv[16];
  for (int i = 0; i < 4; i++) {
    mv[2 * i + 0] = bp->mv_arr0[i].x;
    mv[2 * i + 1] = bp->mv_arr0[i].y;
    mv[8 + 2 * i + 0] = bp->mv_arr1[i].x;
    mv[8 + 2 * i + 1] = bp->mv_arr1[i].y;
  }
  buf_put(mv, sizeof(mv));
  int32_t rf[2];
  rf[0] = bp->mode == MODE_INTRA ? -1 : ref_frame_num(d, bp->ref_idx0);
  rf[1] = bp->mode == MODE_INTRA ? -1 : ref_frame_num(d, bp->ref_idx1);
  buf_put(rf, sizeof(rf));
  if (mask & 1) buf_put(bi->coeffq_y, 2 * size * size);
  if (mask & 2) buf_put(bi->coeffq_u, 2 * sizeC * sizeC);
  if (mask & 4) buf_put(bi->coeffq_v, 2 * sizeC * sizeC);
  g_nblocks++;
  return ret;
}

void __wrap_deblock_frame_y(yuv_frame_t *rec, deblock_data_t *dd, int width, int height, uint8_t qp) {
  dump_frame(rec, "pre_deblock");
  __real_deblock_frame_y(rec, dd, width, height, qp);
}

static int (*g_real_decision)(int, int, yuv_frame_t *, yuv_frame_t *, const deblock_data_t *, int, void *);

static int logging_decision(int k, int l, yuv_frame_t *r, yuv_frame_t *o, const deblock_data_t *dd, int s, void *stream) {
  int v = g_real_decision(k, l, r, o, dd, s, stream);
  int nsb_hor = r->width / MAX_BLOCK_SIZE;
  int idx = k * nsb_hor + l;
  if (idx >= 0 && idx < (int)sizeof(g_clpf)) g_clpf[idx] = (uint8_t)(v ? 1 : 0);
  return v;
}

void __wrap_clpf_frame(yuv_frame_t *rec, yuv_frame_t *org, const deblock_data_t *dd, void *stream,
                       int (*decision)(int, int, yuv_frame_t *, yuv_frame_t *, const deblock_data_t *, int, void *)) {
  dump_frame(rec, "post_deblock");
  g_stage_post_deblock_done = 1;
  g_clpf_on = 1;
  g_real_decision = decision;
  __real_clpf_frame(rec, org, dd, stream, logging_decision);
}

void __wrap_create_reference_frame(yuv_frame_t *ref, yuv_frame_t *rec) {
  if (!g_stage_post_deblock_done) dump_frame(rec, "post_deblock");
  dump_frame(rec, "final");
  __real_create_reference_frame(ref, rec);
}

void __wrap_decode_frame(decoder_info_t *d, yuv_frame_t *rec_buffer) {
  init_once(d);
  g_dec = d;
  g_blk_len = 0;
  g_nblocks = 0;
  g_clpf_on = 0;
  g_stage_post_deblock_done = 0;
  g_nsb = (d->width / MAX_BLOCK_SIZE) * (d->height / MAX_BLOCK_SIZE);
  memset(g_clpf, 0, sizeof(g_clpf));
  /* reference frame numbers must be read before the sliding window moves */
  __real_decode_frame(d, rec_buffer);
  if (g_trace) {
    fwrite("FRME", 1, 4, g_trace);
    int32_t hdr[4] = {g_decode_order, d->frame_info.display_frame_num, 0, 0};
    uint8_t fb[4] = {(uint8_t)d->frame_info.frame_type, d->frame_info.qp, (uint8_t)d->frame_info.num_ref,
                     (uint8_t)g_clpf_on};
    fwrite(hdr, 4, 2, g_trace);
    fwrite(fb, 1, 4, g_trace);
    put_u32(g_trace, g_nblocks);
    put_u32(g_trace, (uint32_t)g_blk_len);
    put_u32(g_trace, (uint32_t)(g_clpf_on ? g_nsb : 0));
    fwrite(g_blk, 1, g_blk_len, g_trace);
    if (g_clpf_on) fwrite(g_clpf, 1, g_nsb, g_trace);
    fflush(g_trace);
  }
  g_decode_order++;
}
