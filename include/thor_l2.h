/*
 * thor_amd -- the reference's block- and frame-level reconstruction entry
 * points ("L2 entry points"), exported by libthor_amd.so
 * with the reference's own names, signatures and struct layouts, so the
 * reference decoder / encoder host C calls them instead of its CPU versions:
 *
 *   deblock_frame_y / _uv     common/common_frame.h:30-31
 *   get_intra_prediction      common/intra_prediction.h:45-46
 *   make_top_and_left         common/intra_prediction.h:31-32
 *   dequantize                common/common_block.h:38
 *   reconstruct_block         common/common_block.h:39
 *   quantize                  enc/encode_block.c:75 (rdoq = 0)
 *
 * Each runs on the GPU: the call's inputs are staged to device memory, one
 * launch (two per deblocking direction) computes, the result is copied back.
 * The frame-level deblocking is the batched decoder's own kernels over the
 * caller's deblock_data; the block-level calls are launch-latency bound and
 * exist for drop-in completeness (the batched API, thor_amd.h, is the fast
 * path).  Like the reference these return no status; a GPU failure, or a
 * request this build does not implement (quantize with rdoq = 1), aborts with
 * a message instead of returning wrong data.
 */
#ifndef THOR_L2_H
#define THOR_L2_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* yuv_frame_t, common/types.h:41-59 (same layout) */
typedef struct thor_ref_yuv_frame {
  uint8_t *y, *u, *v;
  int width, height, stride_y, stride_c, offset_y, offset_c, pad_hor_y, pad_hor_c, pad_ver_y, pad_ver_c, area_y,
      area_c, frame_num;
} thor_ref_yuv_frame_t;

/* mv_t / inter_pred_t / deblock_data_t, common/types.h:105-135 (same layout, 44 bytes) */
typedef struct thor_ref_mv {
  int16_t x, y;
} thor_ref_mv_t;
typedef struct thor_ref_inter_pred {
  thor_ref_mv_t mv0, mv1;
  uint32_t ref_idx0, ref_idx1, bipred_flag;
} thor_ref_inter_pred_t;
typedef struct thor_ref_deblock_data {
  int32_t mode;                /* block_mode_t */
  int32_t cbp_y, cbp_u, cbp_v; /* cbp_t */
  uint8_t size, tb_split;
  int32_t pb_part;             /* part_t */
  thor_ref_inter_pred_t inter_pred;
} thor_ref_deblock_data_t;

/* common/common_frame.h:30 -- in place on rec's Y plane; deblock_data holds
 * (height/4) x (width/4) entries (MIN_PB_SIZE 4) */
void deblock_frame_y(thor_ref_yuv_frame_t *rec, thor_ref_deblock_data_t *deblock_data, int width, int height,
                     uint8_t qp);
/* common/common_frame.h:31 -- qp is the chroma qp (the caller passes chroma_qp[qp]) */
void deblock_frame_uv(thor_ref_yuv_frame_t *rec, thor_ref_deblock_data_t *deblock_data, int width, int height,
                      uint8_t qp);
/* common/intra_prediction.h:31-32 -- left[0..2*size), top[0..2*size), *top_left */
void make_top_and_left(uint8_t *left, uint8_t *top, uint8_t *top_left, uint8_t *rec_frame, int fstride,
                       uint8_t *rblock, int rbstride, int i, int j, int ypos, int xpos, int size,
                       int upright_available, int downleft_available, int tb_split);
/* common/intra_prediction.h:45-46 -- intra_mode: intra_mode_t (common/types.h:137-149); pblock size x size */
void get_intra_prediction(uint8_t *left, uint8_t *top, uint8_t top_left, int ypos, int xpos, int size,
                          uint8_t *pblock, int intra_mode);
/* common/common_block.h:38 */
void dequantize(int16_t *coeff, int16_t *rcoeff, int quant, int size);
/* common/common_block.h:39 */
void reconstruct_block(int16_t *block, uint8_t *pblock, uint8_t *rec, int size, int stride);
/* enc/encode_block.c:75 -- writes the top-left min(size,16)^2 of coeffq
 * (size x size layout), returns cbp; rdoq must be 0 */
int quantize(int16_t *coeff, int16_t *coeffq, int qp, int size, int coeff_block_type, int rdoq);

#ifdef __cplusplus
}
#endif
#endif
