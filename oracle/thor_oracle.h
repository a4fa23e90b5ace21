/*
 * TEST INFRASTRUCTURE ONLY -- the checker, never the thing measured or shipped.
 *
 * Clean-room CPU restatement of the Thor per-block reconstruction hot path
 * (SURVEY.md sec. 8(a)).  Every function cites the reference file:line whose
 * behaviour it restates.  Parity of this restatement is pinned against the
 * reference itself: kernel-level vectors generated from the reference build
 * (tests/golden/ kernel vectors, tools/make_goldens.py) and per-stage frame digests of the
 * reference decoder on committed streams (tests/golden/streams.json).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load liboracle.so.
 */
#ifndef THOR_ORACLE_H
#define THOR_ORACLE_H
#include <stdint.h>
#include "../include/thor_amd.h"
#ifdef __cplusplus
extern "C" {
#endif

/* ---- block kernels ------------------------------------------------------ */
void or_mc_luma(uint8_t *pblock, int pstride, const uint8_t *ref, int rstride, int width, int height, int mvx,
                int mvy, int sign, int bipred);
void or_mc_chroma(uint8_t *pblock, int pstride, const uint8_t *ref, int rstride, int width, int height, int mvx,
                  int mvy, int sign);
void or_dequantize(const int16_t *coeff, int16_t *rcoeff, int qp, int size);
void or_inverse_transform(const int16_t *coeff, int16_t *block, int size);
void or_transform(const int16_t *block, int16_t *coeff, int size, int fast);
int or_quantize(const int16_t *coeff, int16_t *coeffq, int qp, int size, int coeff_block_type);
void or_reconstruct_block(const int16_t *block, const uint8_t *pblock, uint8_t *rec, int size, int stride);
void or_make_top_and_left(uint8_t *left, uint8_t *top, uint8_t *top_left, const uint8_t *rec_frame, int fstride,
                          const uint8_t *rblock, int rbstride, int i, int j, int ypos, int xpos, int size,
                          int upright_available, int downleft_available, int tb_split);
void or_intra_pred(const uint8_t *left, const uint8_t *top, uint8_t top_left, int ypos, int xpos, int size,
                   uint8_t *pblock, int mode);
int or_upright_available(int ypos, int xpos, int size, int width);
int or_downleft_available(int ypos, int xpos, int size, int height);
void or_clpf_block(const uint8_t *src, uint8_t *dst, int sstride, int dstride, int x0, int y0, int size, int width,
                   int height);
uint32_t or_sad(const uint8_t *a, const uint8_t *b, int astride, int bstride, int width, int height);
uint32_t or_ssd(const uint8_t *a, const uint8_t *b, int astride, int bstride, int width, int height);

int or_encode_tu(const uint8_t *orig, int os, const uint8_t *pred, int ps, uint8_t *rec, int rs, int size, int qp,
                 int type, int fast, int16_t *levels, uint32_t *ssd);

/* ---- frames ------------------------------------------------------------- */
/* per-4x4 side info as copy_deblock_data stores it (dec/decode_block.c:122-156,
 * enc/encode_block.c:1947-1981) */
typedef struct {
  uint8_t mode, cbp_y, cbp_u, cbp_v, size, tb_split, pb_part;
  int16_t mv0x, mv0y, mv1x, mv1y;
} or_cell_t;

typedef struct or_frame {
  uint8_t *y, *u, *v; /* interior (0,0) pointers of padded planes */
  int stride_y, stride_c;
  int frame_num;
} or_frame_t;

/* Restates decode_block (dec/decode_block.c:158-471) over a frame's
 * descriptors, then deblock_frame_y/uv (common/common_frame.c:46-321) and
 * clpf_frame (common/common_frame.c:485-557).  stop_stage: 0 recon only,
 * 1 + deblock, 2 + CLPF.  Returns 0 or a negative error. */
int or_decode_frame(const thor_seq_t *seq, const thor_frame_hdr_t *hdr, or_frame_t *cur, const or_frame_t *refs,
                    int nrefs, const thor_block_t *blocks, int nblocks, const int16_t *coeffs,
                    const uint8_t *clpf_flags, int stop_stage);
/* pad_yuv_frame (common/common_frame.c:405-462), pad 96 luma / 48 chroma */
void or_pad_frame(or_frame_t *f, int width, int height, int pad_y, int pad_c);
/* temporal interpolation pyramid: scale_frame_down2x2 luma (common/temporal_interp.c:151-168)
 * and pad_yuv_frame's luma part (common/common_frame.c:414-430) */
void or_scale_down2x2(const uint8_t *in, int si, uint8_t *out, int so, int wo, int ho);
void or_pad_plane(uint8_t *p, int s, int w, int h, int pad);

/* temporal interpolation: interpolate_comp + mot_comp_avg (common/temporal_interp.c:387-441,920-944) */
void or_interp_comp(const uint8_t *p0, int s0, const uint8_t *p1, int s1, uint8_t *out, int so, const int16_t *mv0,
                    const int16_t *mv1, int bw, int bh, int bs, int wP, int hP, int pad, int chroma, int wt0, int wt1);

/* temporal-interpolated reference frame: interpolate_frames (common/temporal_interp.c:972-1053),
 * thor_oracle_ti.c.  ref0/ref1: padded frames (luma pad pad_y); out: the interpolated frame's
 * planes (written over 16*ceil(w/16) x 16*ceil(h/16), i.e. into out's padding).  lv_mv0/lv_mv1:
 * optional per-level outputs of the final block-vector fields (bw*bh int16 pairs, level 0 first). */
int or_ti_levels(int width, int height);
void or_ti_weights(int ratio, int pos, int *wt0, int *wt1, int *reversed);
int or_interpolate_frames(const or_frame_t *ref0, const or_frame_t *ref1, int pad_y, or_frame_t *out, int width,
                          int height, int ratio, int pos, int16_t *const *lv_mv0, int16_t *const *lv_mv1);

struct or_frame;
void or_deblock_cells(struct or_frame *f, const or_cell_t *cells, int W, int H, int qp);
void or_clpf_cells(struct or_frame *f, const or_cell_t *cells, int W, int H, const uint8_t *flags);

#ifdef __cplusplus
}
#endif
#endif
