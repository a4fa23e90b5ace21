/*
 * TEST INFRASTRUCTURE ONLY -- never linked into the product library.
 *
 * A link-time hook (-Wl,--wrap=process_block) that turns the *unmodified*
 * reference encoder (enc/*.c + common/*.c compiled from /root/reference by
 * oracle/Makefile, target _ref/thorenc_rd) into a recorder of its per-superblock
 * RD costs.  Only the cross-TU calls are wrapped: encode_frame's calls of
 * process_block for each 64x64 superblock (enc/encode_frame.c:133-144) -- every
 * delta-QP trial (qp - max_delta_qp .. qp + max_delta_qp in delta_qp_step
 * steps, :133-139) and the final encode with the best QP (:142), or the single
 * call without delta QP (:145); process_block's recursive calls for the
 * quadtree (enc/encode_block.c:2942-2984) stay inside their TU, unwrapped.
 * The hook calls straight through (__real_process_block) and only records
 * arguments and the returned cost.
 *
 * Output (env THOR_RD_LOG=<file>): little-endian int32 records
 *   frame_num, size, ypos, xpos, qp, cost
 * one per top-level call, in call order, flushed per record (a run may be cut
 * short once the frames of interest are logged).
 */
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

#include "global.h"
#include "mainenc.h"

int __real_process_block(encoder_info_t *encoder_info, int size, int ypos, int xpos, int qp);

static FILE *rd_log(void) {
  static FILE *f = NULL;
  static int tried = 0;
  if (!tried) {
    const char *p = getenv("THOR_RD_LOG");
    tried = 1;
    if (p) f = fopen(p, "wb");
  }
  return f;
}

int __wrap_process_block(encoder_info_t *encoder_info, int size, int ypos, int xpos, int qp) {
  const int cost = __real_process_block(encoder_info, size, ypos, xpos, qp);
  FILE *f = rd_log();
  if (f) {
    const int32_t r[6] = {encoder_info->frame_info.frame_num, size, ypos, xpos, qp, cost};
    fwrite(r, sizeof(r), 1, f);
    fflush(f);
  }
  return cost;
}
