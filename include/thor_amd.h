/*
 * thor_amd -- MI355X-native per-block reconstruction for the Thor video codec.
 *
 * Public C-ABI of libthor_amd.so (thor_amd/csrc).  Two surfaces:
 *
 *  1. The reference's SIMD kernel surface, same names and signatures, so the
 *     reference Thorenc/Thordec host C links this library in place of
 *     common/common_kernels.c and enc/enc_kernels.c (see thor_kernels.h).
 *
 *  2. A batched per-frame surface (this header): block-descriptor arrays in,
 *     one launch per stage, frames resident in HBM.  This is what a restated
 *     decode_frame (dec/decode_frame.c:45-148) calls; the per-block symbols
 *     alone would be launch-latency bound.
 *
 * No torch types cross this boundary: plain pointers, sizes and int status
 * codes (0 = ok, <0 = error; the reference has no error convention and aborts,
 * common/global.h:38-44 -- this library never aborts).
 */
#ifndef THOR_AMD_H
#define THOR_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------ */
#define THOR_OK 0
#define THOR_ERR_ARG (-1)
#define THOR_ERR_HIP (-2)
#define THOR_ERR_NOMEM (-3)
#define THOR_ERR_REF (-4) /* a block names a reference frame that is not resident */

/* ---- block descriptor ------------------------------------------------- *
 * One decoded CU as the parser leaves it (dec/maindec.h:47-57, block_param_t
 * common/types.h:153-170).  72 bytes, naturally aligned.                     */
typedef struct thor_block {
  uint16_t ypos, xpos;      /* luma position of the CU                        */
  uint8_t size;             /* 8..64                                           */
  uint8_t bwidth, bheight;  /* clipped to the frame (rectangular edge SKIP,
                               dec/decode_block.c:222-226)                     */
  uint8_t mode;             /* block_mode_t: 0 SKIP 1 INTRA 2 INTER 3 BIPRED 4 MERGE */
  uint8_t intra_mode;       /* intra_mode_t (common/types.h:137-149)           */
  uint8_t tb_split;         /* 4 transform blocks                              */
  uint8_t pb_part;          /* part_t, deblocking only                         */
  uint8_t dir;              /* 2 = bi-directional SKIP/MERGE                   */
  uint8_t qp;               /* block qp (frame qp + delta qp)                  */
  uint8_t cbp_y, cbp_u, cbp_v; /* cbp as stored in deblock_data             */
  uint8_t coeff_mask;       /* bit c: component c (Y,U,V) has coefficients     */
  uint8_t rsv[3];
  int16_t mv0[8];           /* mv_arr0[4] as (x, y) pairs, quarter-pel luma    */
  int16_t mv1[8];           /* mv_arr1[4]                                      */
  int32_t ref0, ref1;       /* display frame_num of the reference (-1 none, -2 the
                               frame's temporal-interpolated reference,
                               dec/decode_block.c:249: interp_frames[0])     */
  uint32_t coeff_off[3];    /* int16 offset of each component in the frame's
                               compact coefficient pool                        */
} thor_block_t;

/* Compact coefficient pool: per component of a CU, one qsize x qsize int16
 * tile per transform block (qsize = min(N,16): only the low-frequency corner
 * can be non-zero, common/transform.c:309-327), tb-split quarters consecutive
 * in raster order, row-major inside a tile. */

/* ---- sequence / frame parameters -------------------------------------- */
typedef struct thor_seq {
  int32_t width, height;
  int32_t bipred;      /* sequence-level enable_bipred: selects the luma MC table
                          for every luma call (dec/maindec.c:147)            */
  int32_t deblocking;  /* dec/maindec.c:144 */
  int32_t clpf;        /* dec/maindec.c:145 */
  int32_t tb_split_enable;
  int32_t interp_ref;  /* sequence may use temporal-interpolated references
                          (dec/maindec.c:140): the decoder then keeps an
                          interpolation slot and its motion-search scratch  */
} thor_seq_t;

typedef struct thor_frame_hdr {
  int32_t frame_num;   /* display frame number */
  int32_t frame_type;  /* 0 I, 1 P, 2 B */
  int32_t qp;          /* frame qp: drives deblocking (dec/decode_frame.c:124-128) */
  int32_t clpf_on;     /* CLPF signalled on for this frame (dec/decode_frame.c:130) */
  /* temporal-interpolated reference (dec/decode_frame.c:91-109): when
   * interp_ratio > 0 the frame's ref index 0 is interpolate_frames(ref_a,
   * ref_b, interp_ratio, interp_pos) of the resident frames numbered
   * interp_ref[0] (ref_array[1]) and interp_ref[1] (ref_array[2]); blocks name
   * it as reference -2.  interp_ratio 0: no interpolated reference. */
  int32_t interp_ref[2];
  int32_t interp_ratio, interp_pos;
} thor_frame_hdr_t;

/* One coded transform block of a frame (thor_build_tu_list): everything the
 * residual kernel needs, so it reads no block descriptor.  12 bytes. */
typedef struct thor_tu {
  uint32_t coeff_off; /* int16 offset of the TU's q x q tile in the coefficient pool */
  uint16_t y, x;      /* TU origin in its plane (chroma planes: chroma pixels)     */
  uint8_t size;       /* 4..64                                                     */
  uint8_t comp;       /* 0 Y, 1 U, 2 V                                             */
  uint8_t qp;         /* component qp (chroma: chroma_qp[qp])                      */
  uint8_t rsv;
} thor_tu_t;

/* ---- batched decoder context ------------------------------------------ */
typedef struct thor_dec thor_dec_t;

/* Create a device-resident decoder: a ring of padded reference frames (pad 96
 * luma / 48 chroma, stride as create_yuv_frame, common/common_frame.c:324-351)
 * on HIP device `device`.  Returns NULL on failure; thor_last_create_error
 * says why.  num_slots <= 1: 34 (the reference's 33-frame window + the frame
 * being decoded); a reference evicted from a smaller ring is reported as
 * THOR_ERR_REF by the decode call that names it, never decoded wrongly. */
thor_dec_t *thor_dec_create(const thor_seq_t *seq, int device, int num_slots);

/* Why the last thor_dec_create / thor_enc_create / thor_ti_create of the
 * calling thread returned NULL: THOR_ERR_ARG (unsupported parameters, e.g. a
 * ring over the 2 GiB one buffer descriptor addresses), THOR_ERR_NOMEM (HBM
 * exhausted; *bytes = the size of the allocation that failed) or THOR_ERR_HIP;
 * THOR_OK after a successful create.  `msg` (may be NULL) receives a one-line
 * reason naming the buffer. */
int thor_last_create_error(size_t *bytes, char *msg, size_t cap);
void thor_dec_destroy(thor_dec_t *d);

/* Decode (reconstruct) one frame.  `blocks`, `coeffs`, `clpf_flags` and
 * `intra_list` are DEVICE pointers (inputs resident in HBM); `nblocks`
 * descriptors in decode order.  `intra_list` holds the indices of the intra
 * CUs in decode order (thor_build_intra_list) and `tu_list` the coded
 * transform blocks (thor_build_tu_list): the only planning data the parser
 * hands over besides the descriptors.  Enqueues every stage on the
 * context's stream and returns without waiting: per-4x4 side info, inter MC +
 * dequant + inverse transform + reconstruction, intra, deblock Y/UV, CLPF,
 * padding.  The reconstructed frame becomes reference `frame_num`. */
int thor_dec_frame(thor_dec_t *d, const thor_frame_hdr_t *hdr, const thor_block_t *blocks, int nblocks,
                   const int16_t *coeffs, const uint8_t *clpf_flags, const uint32_t *intra_list, int n_intra,
                   const thor_tu_t *tu_list, int n_tu);


/* One frame's parse output (DEVICE pointers), as thor_dec_frame takes it. */
typedef struct thor_frame_in {
  const thor_block_t *blocks;
  int32_t nblocks;
  const int16_t *coeffs;
  const uint8_t *clpf_flags;
  const uint32_t *intra_list;
  int32_t n_intra;
  const thor_tu_t *tu_list;
  int32_t n_tu;
  const uint32_t *clpf_list; /* indices of the SBs whose CLPF flag is set (thor_build_clpf_list) */
  int32_t n_clpf;            /* -1: no list, scan every SB's flag */
  /* k_recon units (128x16 luma) that hold several (MV, reference) keys in a
   * half SB (thor_build_slow_list): dispatched first, so their long per-cell
   * path overlaps the planned units instead of forming the launch's tail.
   * When given, it must be exactly thor_build_slow_list's output for THIS
   * frame's blocks: k_frame_prep then writes per-cell MC words only for the
   * listed halves, and a multi-key half that is not listed is not
   * reconstructed.  NULL: no list (every unit in planned order, same output). */
  const uint32_t *slow_list;
  int32_t n_slow;
} thor_frame_in_t;

/* Decode one frame in each of `n` DIFFERENT contexts with one launch per stage
 * (grid dimension = frame, up to 8 frames per launch): a server decoding many
 * streams batches their next frames.  All contexts must share the device and frame size.
 * Work is enqueued on ds[0]'s stream, ordered after each member context's
 * earlier work on its own stream and before its later work.  n = 1 is
 * thor_dec_frame. */
int thor_dec_frames(thor_dec_t *const *ds, int n, const thor_frame_hdr_t *hdrs, const thor_frame_in_t *ins);

/* ---- row-band sharding of one stream across GPUs ---
 * thor_dec_set_band: k_recon reconstructs only SB rows [sb_row0, sb_row1) of
 * this context's frames (0, 0 = all).  thor_dec_frame_begin enqueues side info,
 * residuals and the band's inter reconstruction; the caller then exchanges
 * bands (thor_dec_get_rows / thor_dec_put_rows on DEVICE buffers, e.g. an RCCL
 * all-gather on the same stream); thor_dec_frame_end enqueues intra, deblock,
 * CLPF and padding of the whole frame.  Rows are packed Y (nrows x W) | U |
 * V (nrows/2 x W/2 each); put_rows (y0, nrows even) also refreshes the
 * SB-row edge rows the intra chains read for every SB row whose bottom row it
 * carries.  Rows past the frame are skipped. */
int thor_dec_set_band(thor_dec_t *d, int sb_row0, int sb_row1);
int thor_dec_frame_begin(thor_dec_t *d, const thor_frame_hdr_t *hdr, const thor_frame_in_t *in);
int thor_dec_frame_end(thor_dec_t *d);
int thor_dec_get_rows(thor_dec_t *d, int frame_num, int y0, int nrows, void *dst);
int thor_dec_put_rows(thor_dec_t *d, int frame_num, int y0, int nrows, const void *src);
/* Band-local phase B (on = 1, with a band set): thor_dec_frame_end then
 * enqueues intra for the whole frame (its chains cross bands) but deblocking
 * and CLPF only for the band's rows (the deblocking reads a 2-row halo the
 * first exchange already carries), and no padding; the caller exchanges the
 * bands' final rows (get_rows / put_rows again, same packing) and calls
 * thor_dec_frame_finish, which pads the frame and makes it a reference.  Each
 * rank's loop filters then cover 1/N of the frame instead of all of it. */
int thor_dec_set_band_local(thor_dec_t *d, int on);
int thor_dec_frame_finish(thor_dec_t *d);
/* Band-local contexts whose frames are never whole on this rank (the halo and
 * boundary exchanges of thor_amd/shard.py): thor_dec_frame_finish pads only
 * the band's rows (the top / bottom pad rows only on the first / last band);
 * a reference row fetched later is re-padded by thor_dec_pad_frame. */
int thor_dec_set_band_pad(thor_dec_t *d, int on);
/* Band-local intra (on = 1, with a band set; the boundary exchange of
 * thor_amd/shard.py, which replaces the pre-deblock all-gather): the intra
 * chains of the band's SB rows only, the first of them reading the row above
 * from the edge rows (thor_dec_put_rows of the two luma rows ending the SB row
 * above, from the rank that owns it) instead of waiting for it.
 * thor_dec_frame_intra enqueues that intra stage between thor_dec_frame_begin
 * and thor_dec_frame_end (which then skips it), so the caller can hand the
 * band's bottom edge rows to the rank below and exchange the deblocking halo
 * rows (8 above, 8 below the band) after it. */
int thor_dec_set_band_intra(thor_dec_t *d, int on);
int thor_dec_frame_intra(thor_dec_t *d);
/* MV-reach halo exchange (band-local contexts, thor_amd/shard.py halo mode):
 * instead of all-gathering every band's final rows, each rank fetches, before
 * a frame's thor_dec_frame_begin, only the rows of its references that the
 * frame's vectors in its band can reach.  put_ref_rows writes rows
 * [y0, y0 + nrows) (y0, nrows even; same packing as get_rows) into the
 * resident frame `frame_num` without touching the intra edge rows;
 * pad_frame then redoes that frame's border padding from its edge pixels (the
 * rows a rank holds final are padded correctly; a vector reaching past the
 * frame edge makes its rank fetch the edge row). */
int thor_dec_put_ref_rows(thor_dec_t *d, int frame_num, int y0, int nrows, const void *src);
int thor_dec_pad_frame(thor_dec_t *d, int frame_num);

/* Host helper: write the decode-order indices of the intra CUs of a frame
 * (host descriptors) to `out` (may be NULL to count); returns the count. */
int thor_build_intra_list(const thor_block_t *host_blocks, int nblocks, uint32_t *out);
/* Host helper: indices of the SBs whose CLPF decision flag is set (the CLPF
 * launch is as wide as this list; `out` may be NULL to count). */
int thor_build_clpf_list(const uint8_t *host_flags, int nsb, uint32_t *out);
/* Host helper: the frame's coded transform blocks (the residual work list the
 * parser knows from the cbp flags, dec/decode_block.c:90-120), tb-split
 * quarters in raster order, chroma of 8x8 CUs unsplit.  `out` may be NULL to
 * count; returns the count. */
int thor_build_tu_list(const thor_block_t *host_blocks, int nblocks, thor_tu_t *out);
/* Host helper: the frame's multi-key reconstruction units (thor_frame_in_t
 * slow_list), ascending.  A half SB (64x32 luma) is multi-key when it holds an
 * inter CU smaller than 64x64, or is a half inside the frame of a 64x64 INTER /
 * BIPRED CU whose two quarters there differ in a motion vector; a unit (128x16
 * luma: SB pair p, slice row 4 x SB row + quarter) is listed when the half of
 * either of its SBs is.  `out` may be NULL to count; returns the count. */
int thor_build_slow_list(const thor_block_t *host_blocks, int nblocks, int width, int height, uint32_t *out);

/* Stage control for parity debugging: 0 recon only, 1 +deblock, 2 +CLPF (default 2). */
int thor_dec_set_stop_stage(thor_dec_t *d, int stage);

/* Copy frame `frame_num` (unpadded I420, tightly packed) to host memory. */
int thor_dec_read_frame(thor_dec_t *d, int frame_num, uint8_t *y, uint8_t *u, uint8_t *v);
/* Upload a frame (e.g. an externally decoded reference) into a slot. */
int thor_dec_write_frame(thor_dec_t *d, int frame_num, const uint8_t *y, const uint8_t *u, const uint8_t *v);
int thor_dec_sync(thor_dec_t *d);

/* Per-stage GPU timing with hipEvents on the context's stream.  When on,
 * thor_dec_frame brackets each stage; thor_dec_stage_ms waits for the stream
 * and returns the milliseconds accumulated per stage since the last call:
 * [0] side info + residuals (k_prep, k_resid), [1] inter recon (k_recon), [2] intra,
 * [3] deblock, [4] CLPF, [5] pad, [6] temporal-interpolated reference. */
int thor_dec_set_timing(thor_dec_t *d, int on);
int thor_dec_stage_ms(thor_dec_t *d, double *ms, int nstages);
/* The same marks one by one in enqueue order (stage index, milliseconds), so
 * a caller can attribute them to frames; returns the count (<= cap) and
 * clears the marks. */
int thor_dec_stage_marks(thor_dec_t *d, int *stage, double *ms, int cap);

/* The HIP stream the context enqueues on (hipStream_t as void*), so callers
 * can record events / capture graphs around thor_dec_frame. */
void *thor_dec_stream(thor_dec_t *d);
/* Set the stream (e.g. torch's current stream); NULL = the context's own. */
int thor_dec_set_stream(thor_dec_t *d, void *stream);

/* ---- batched encoder transform-block chain ----------------------------- *
 * One descriptor per transform block (TU) of an RD candidate.  The chain is
 * encode_and_reconstruct_block_inter / _intra's per-TU body
 * (enc/encode_block.c:1434-1518): get_residual (:484-493) -> transform
 * (common/transform.c:249-330) -> quantize (enc/encode_block.c:75-172,
 * rdoq 0) -> [cbp] dequantize + inverse_transform (common/common_block.c:
 * 132-146, common/transform.c:432-518) -> reconstruct_block
 * (common/common_block.c:148-156) or rec = pred -> SSD(orig, rec).
 * 32 bytes, naturally aligned. */
typedef struct thor_enc_tu {
  int32_t orig_off;    /* byte offset of the TU's (0,0) in `orig`             */
  int32_t pred_off;    /* byte offset of the TU's (0,0) in `pred`             */
  int32_t rec_off;     /* byte offset of the TU's (0,0) in `rec`              */
  int32_t coeff_off;   /* int16 offset of the TU's q x q level tile in `coeffq`
                          (q = min(size,16), the compact pool layout above)   */
  int32_t orig_stride, pred_stride, rec_stride;
  uint8_t size;        /* 4, 8, 16, 32 or 64                                   */
  uint8_t qp;          /* component qp (chroma: chroma_qp[qp], common/common_block.c:78-83) */
  uint8_t type;        /* coeff_block_type: bit1 intra, bit0 chroma (enc/encode_block.c:77-78) */
  uint8_t fast;        /* transform `fast` flag       */
} thor_enc_tu_t;

/* Run the chain for `n` TUs (all pointers DEVICE pointers).  Per TU: the q x q
 * quantised levels into coeffq, cbp (0/1; 255 = invalid descriptor) and the
 * TU's SSD(orig, rec).  Enqueued on `stream` (hipStream_t, NULL = default). */
int thor_enc_tu_batch(const thor_enc_tu_t *tus, int n, const uint8_t *orig, const uint8_t *pred, uint8_t *rec,
                      int16_t *coeffq, uint8_t *cbp, uint32_t *ssd, void *stream);

/* cost_calc (enc/encode_block.c:1218-1228) for `ncu` candidates: the SSDs of
 * TUs tu_first[c] .. tu_first[c]+tu_count[c]-1 (Y, U and V TUs of the CU)
 * plus (int32)(lambda * nbits[c] + 0.5), clamped to 2^30.  DEVICE pointers. */
int thor_enc_cost_batch(const uint32_t *ssd, const int32_t *tu_first, const int32_t *tu_count, const int32_t *nbits,
                        double lambda, uint32_t *cost, int ncu, void *stream);

/* ---- the .bit parser (host) that feeds the batched decoder -------------- *
 * Restates the reference's serial syntax layer (dec/getbits.c, dec/getvlc.c,
 * dec/read_bits.c, decode_frame / process_block_dec): one frame payload (the
 * bytes after a chunk's 4-byte length, dec/getbits.c:48-69) in, the frame's
 * descriptors, compact coefficient pool and CLPF flags out -- thor_dec_frame's
 * inputs (copy them to device memory).  The first payload carries the sequence
 * header.  Output pointers stay valid until the next call. */
typedef struct thor_parser thor_parser_t;
typedef struct thor_parsed_frame {
  thor_seq_t seq;
  thor_frame_hdr_t hdr;
  int32_t decode_order, num_ref;
  const thor_block_t *blocks;
  int32_t nblocks;
  const int16_t *coeffs;
  int32_t ncoeffs;
  const uint8_t *clpf_flags; /* per full SB, raster (W/64 x H/64) */
  int32_t nclpf;
} thor_parsed_frame_t;
thor_parser_t *thor_parser_create(void);
void thor_parser_destroy(thor_parser_t *p);
int thor_parser_seq(const thor_parser_t *p, thor_seq_t *seq);
int thor_parse_frame(thor_parser_t *p, const uint8_t *payload, size_t nbytes, thor_parsed_frame_t *out);
/* One host image of a parsed frame's decoder input, for ONE host-to-device copy:
 * descriptors | coefficient pool | CLPF flags | intra list | TU list | CLPF list
 * | slow list, each part 256-byte aligned (the thor_build_* lists built here).
 * Returns THOR_OK with the image written, or THOR_ERR_NOMEM when `cap` is below
 * lay->bytes (`img` may be NULL to size it); lay gets the parts' offsets and
 * counts either way (n_flags = 0 and n_clpf = -1 when the frame signals no CLPF). */
typedef struct thor_frame_image {
  uint64_t bytes;
  uint64_t off_blocks, off_coeffs, off_flags, off_intra, off_tus, off_clpf, off_slow;
  int32_t nblocks, ncoeffs, n_flags, n_intra, n_tu, n_clpf, n_slow;
} thor_frame_image_t;
int thor_frame_image(const thor_parsed_frame_t *pf, uint8_t *img, size_t cap, thor_frame_image_t *lay);

/* ---- device-resident encoder (the full RD loop) ---- *
 * Encoder parameters: enc_params (enc/mainenc.h:34-88), the flags of the
 * reference's configuration files / command line (enc/strings.c:286-338),
 * same names and types (float where the reference parses ARG_FLOAT).      */
typedef struct thor_enc_params {
  int32_t width, height, qp, num_frames, skip;
  float frame_rate;
  float lambda_coeffI, lambda_coeffP, lambda_coeffB, lambda_coeffB0, lambda_coeffB1, lambda_coeffB2, lambda_coeffB3;
  float early_skip_thr;
  int32_t enable_tb_split, enable_pb_split, max_num_ref, HQperiod, num_reorder_pics, dyadic_coding, interp_ref;
  int32_t dqpP, dqpB, dqpB0, dqpB1, dqpB2, dqpB3;
  float mqpP, mqpB, mqpB0, mqpB1, mqpB2, mqpB3;
  int32_t dqpI, intra_period, intra_rdo, rdoq, max_delta_qp, delta_qp_step, encoder_speed, sync, deblocking, clpf,
      snrcalc, use_block_contexts, enable_bipred;
} thor_enc_params_t;

/* The reference defaults (enc/strings.c:286-338). */
void thor_enc_default_params(thor_enc_params_t *p);
/* 0 if the parameters are supported by the device encoder, else THOR_ERR_ARG
 * (check_parameters, enc/strings.c:431-479, plus this build's limits:
 * rdoq 0, sync 0). */
int thor_enc_check_params(const thor_enc_params_t *p);

/* A device-resident encoder context: the reference's frame loop
 * (enc/mainenc.c:222-591) planned on the host, every frame's RD loop, loop
 * filters and bit packing on the GPU (wavefront-parallel superblock rows).
 * The output is the reference Thorenc's .bit, byte for byte. */
typedef struct thor_enc thor_enc_t;
thor_enc_t *thor_enc_create(const thor_enc_params_t *p, int device);
void thor_enc_destroy(thor_enc_t *e);
/* frames the context will code (params.num_frames after -skip) */
int thor_enc_num_frames(const thor_enc_t *e);
/* input frame (display order, 0 = first after -skip) the next call codes;
 * -1 when every frame is coded */
int thor_enc_next_input(const thor_enc_t *e);
void *thor_enc_stream(thor_enc_t *e);
/* Re-create the context's stream restricted to the CUs whose bits are set in
 * mask[0..nwords) (bit c % 32 of word c / 32 = CU c; hipExtStreamCreateWithCUMask).
 * A scheduling knob: CUs left out stay free for concurrent decode launches.
 * The masked stream is a BLOCKING stream (it orders against the null stream).
 * The old stream is destroyed: a handle thor_enc_stream returned before is
 * invalid afterwards.  Must not overlap a thor_enc_frames call on the context
 * (nothing here guards against it).  On THOR_ERR_HIP the old stream is kept. */
int thor_enc_set_cu_mask(thor_enc_t *e, const uint32_t *mask, int nwords);
/* Code the next frame of each of `n` DIFFERENT contexts (same device and
 * size, n <= 512) with one launch per stage.  Thread-safe: calls on the same
 * device are serialised (they share that device's work pool; begin and end of
 * one call run under one hold of its lock); a context must not be used by two
 * calls at once.  On THOR_ERR_HIP (a device error flag,
 * e.g. a WPP wait that gave up) no context advances: the frame can be coded
 * again.  orig[i]: DEVICE pointer to the
 * context's input frame thor_enc_next_input(es[i]), planar I420, luma stride
 * orig_stride[i] (NULL: width), chroma stride half of it.  Synchronous. */
int thor_enc_frames(thor_enc_t *const *es, int n, const uint8_t *const *orig, const int *orig_stride);
/* thor_enc_frames in two halves, so the device codes the next frame while the
 * host collects the last one: _begin enqueues every stage of the batch and
 * advances the contexts (the next frame may be begun at once: up to two
 * batches in flight per device, a context's frames on one stream; a frame with
 * an interpolated reference waits for the batches in flight before its
 * interpolation); _end waits for the oldest batch begun with exactly these
 * contexts (the same es / n), reads its coded words back and makes them the
 * contexts' chunks (thor_enc_frame_bytes).  On a device error _end drops every
 * batch in flight and returns every dropped batch's contexts to their state
 * before the oldest of them (those frames can be coded again).
 * thor_enc_reset refuses a context with a batch in flight; thor_enc_destroy
 * drops its batches and returns their other contexts to their state before
 * them. */
int thor_enc_frames_begin(thor_enc_t *const *es, int n, const uint8_t *const *orig, const int *orig_stride);
int thor_enc_frames_end(thor_enc_t *const *es, int n);
int thor_enc_frame(thor_enc_t *e, const uint8_t *orig, int orig_stride);
/* The last coded frame's .bit chunk (4-byte big-endian length + payload,
 * enc/putbits.c:57-95; the first chunk carries the sequence header):
 * returns its size, copies min(size, cap) bytes to dst when non-NULL. */
long long thor_enc_frame_bytes(const thor_enc_t *e, uint8_t *dst, size_t cap);
/* Sequence launch (enc_seq.hip): the next `nframes` frames (coding order) of
 * each of n contexts in ONE persistent launch.  Frame f + 1 of a context starts
 * as soon as its frame f is a finished reference (RD loop, loop filters, CLPF,
 * padding), independently of the other contexts, and each frame's bits go to
 * page-locked host memory as soon as they are packed.  in[i * nframes + f]:
 * context i's f-th input frame (I420, luma stride = width): a device pointer
 * (fetch = 0), or a host pointer to page-locked, device-accessible memory
 * (fetch = 1: the launch copies it to dev[i * nframes + f], W*H*3/2 bytes of
 * device memory, one frame ahead of the RD loop).  arena_bytes: host space for
 * the coded frames (<= 0: W*H/32 bytes per frame + 16 KB).  Contexts with
 * interpolated references or SB-cost recording are refused (THOR_ERR_ARG:
 * thor_enc_frames codes them), and so is a second launch, or a batch, while
 * one is in flight on the device.  Returns at once with the launch in flight.
 * thor_enc_seq_ready: out[i * nframes + f] = chunk size of that frame if it is
 * final, else -1 (non-blocking); returns how many are final.
 * thor_enc_seq_chunk: the chunk (4-byte big-endian length + payload) of
 * context i's f-th frame, min(size, cap) bytes copied; returns its size.  Both
 * read the launch in flight or, after thor_enc_seq_end, the last one ended,
 * until the next thor_enc_seq_begin on the device (one caller at a time).
 * THOR_SEQ_CLASSES / THOR_SEQ_CLAIM / THOR_SEQ_PRIO / THOR_SEQ_RETIRE in the
 * environment select the scheduling variants measured in DESIGN.md §3b.
 * thor_enc_seq_end: waits; on a device error every context returns to its
 * state before the launch (THOR_ERR_HIP, THOR_ERR_NOMEM when a frame outgrew
 * the output buffer or the arena); else each context's last frame is also its
 * thor_enc_frame_bytes chunk.  stats (optional, 4 values): workers launched,
 * workers retired early (after the I frames, to free CU slots), tasks run,
 * arena words used. */
/* input frame index (display order) of the frame `ahead` frames after the next
 * one in coding order (ahead = 0: thor_enc_next_input); -1 past the end */
int thor_enc_plan_input(const thor_enc_t *e, int ahead);
int thor_enc_seq_begin(thor_enc_t *const *es, int n, int nframes, const uint8_t *const *in, uint8_t *const *dev,
                       int fetch, long long arena_bytes);
int thor_enc_seq_ready(thor_enc_t *e0, long long *out, int count);
long long thor_enc_seq_chunk(thor_enc_t *e0, int i, int f, uint8_t *dst, size_t cap);
int thor_enc_seq_end(thor_enc_t *e0, long long *stats);
/* The last ended sequence launch's profile, summed over its workers (100 MHz
 * ticks): per task type (RD, FETCH, DBV, DBH, FIN, PACK) the time in tasks,
 * then the task counts, then idle time, time waiting for a claimed queue slot
 * and failed claims.  Returns 15; copies min(15, n) values. */
int thor_enc_seq_profile(thor_enc_t *e0, long long *out, int n);
/* The per-frame batch RD kernel's profile since the last call on `device`,
 * summed over its workers (100 MHz ticks): time coding superblocks, time
 * waiting for a queue slot, superblocks coded; cleared.  Returns 3. */
int thor_enc_rows_profile(int device, long long *out);
/* The last coded frame's reconstruction (deblocked, CLPF'd), host planes. */
int thor_enc_read_recon(thor_enc_t *e, uint8_t *y, uint8_t *u, uint8_t *v);
/* Per-superblock RD costs (parity instrumentation, tests/golden/rd_costs.npz):
 * with on = 1 the context records, for every 64x64 superblock of each frame it
 * codes from then on, the cost each top-level process_block call returns
 * (enc/encode_frame.c:133-145) -- every delta-QP trial (qp - max_delta_qp ..
 * qp + max_delta_qp in delta_qp_step steps), then the final encode; without
 * delta QP the one call.  thor_enc_sb_costs copies the last ended frame's
 * records (raster SB order, *per_sb int32 per SB) to dst (min(count, cap))
 * and returns their count; call it before a later frame of the context is
 * begun.  THOR_ERR_ARG when recording is off. */
int thor_enc_record_sb_costs(thor_enc_t *e, int on);
long long thor_enc_sb_costs(thor_enc_t *e, int32_t *dst, size_t cap, int *per_sb);
/* Restart the context at the first frame of its sequence (the reference
 * window emptied, the sequence header due again): a server re-using a
 * context for the next clip of the same parameters. */
int thor_enc_reset(thor_enc_t *e);
/* Diagnostics only: superblock row `row` of every stream never releases the
 * row below it (-1: off) -- its SBs are coded, the next row's never become
 * ready -- and a worker's wait for its next superblock gives up after
 * `spin_ms` milliseconds (<= 0: the 5-minute default).  Each worker gives up
 * at most once and then exits, so the launch drains in bounded time and the
 * call returns THOR_ERR_HIP (the SBs never coded pack as nothing). */
int thor_enc_debug_stall(int row, int spin_ms);

/* ---- temporal interpolation: luma down-sampling pyramid ----------------- */

/* Number of down-sampled levels interpolate_frames builds for a width x height
 * reference: max_levels - 1 with max_levels = min(MAX_LEVELS = 4,
 * (int)(log10(min(w, h)) / log10(2) - 4)) (common/temporal_interp.c:20,977). */
int thor_pyramid_levels(int width, int height);

/* Replaces the chain of scale_frame_down2x2_simd calls on one reference frame
 * (common/temporal_interp.c:1011-1019, kernel :187-245): level l (1-based,
 * l <= nlevels <= 3) is (width >> l) x (height >> l) luma, each pixel
 * (avg(v0,v1) + avg(h0,h1)) >> 1 of the 2x2 block below it, then padded by
 * edge replication over a 32-pixel margin (pad_yuv_frame,
 * common/common_frame.c:405-462).  Chroma is not produced: USE_CHROMA is 0
 * (temporal_interp.c:19), so the SIMD path leaves level chroma unwritten and
 * nothing reads it.  `levels` / `level_strides` are HOST arrays of DEVICE
 * pointers / strides; `src` is level 0's (0,0) (8-byte
 * aligned, stride % 8 == 0); levels[l-1] is level l's (0,0) in a
 * create_yuv_frame(.., 32, 32, ..) plane (16-byte aligned, stride % 16 == 0,
 * stride >= w + 64, 32 rows above and below).  One launch computes every
 * level, a second pads them.  Enqueued on `stream`. */
int thor_scale_pyramid(const uint8_t *src, int src_stride, int width, int height, uint8_t *const *levels,
                       const int *level_strides, int nlevels, void *stream);

/* Both references of interpolate_frames (:1011-1019) in the same two launches
 * (grid z = frame); same frame size and strides for the two, as
 * interpolate_frames allocates them. */
int thor_scale_pyramid2(const uint8_t *src0, const uint8_t *src1, int src_stride, int width, int height,
                        uint8_t *const *levels0, uint8_t *const *levels1, const int *level_strides, int nlevels,
                        void *stream);

/* Replaces interpolate_comp (common/temporal_interp.c:920-944) on one plane:
 * for each of the bw x bh blocks of bs x bs pixels, mot_comp_avg (:387-441)
 * with the block's vectors (1/8 pel, rounded to integer: ACC_BITS 3) --
 * (ref0 + ref1 + 1) / 2 when both displaced blocks lie inside
 * [-pad, wP) x [-pad, hP), else a copy of the one that does (ref1 first;
 * ref0 rows read with s1, as :420-422 does), else the clamped average.
 * chroma != 0: mv1 is halved and mv0 = scale_mv(mv1, -wt1, wt0) (:934-938),
 * the mv0 array is then not read.  mv0/mv1: bw*bh (x, y) int16 pairs
 * (mv_data->mv[0], mv[1]).  p0/p1 are the (0,0) of pic[0]/pic[1] (already
 * swapped by mv_data->reversed, :950-951).  All DEVICE pointers; enqueued on
 * `stream`. */
int thor_interp_comp(const uint8_t *p0, int s0, const uint8_t *p1, int s1, uint8_t *out, int so, const int16_t *mv0,
                     const int16_t *mv1, int bw, int bh, int bs, int wP, int hP, int pad, int chroma, int wt0, int wt1,
                     void *stream);

/* interpolate_frame (common/temporal_interp.c:946-970) in one launch: Y with
 * the reference's 8x8 blocks (bs = BLOCK_STEP/2, pad 4, wP = width + 4), U and
 * V with 4x4 blocks (pad 2, wP = (width + 4) / 2) -- the thor_interp_comp
 * semantics above per plane.  planes[0..2] = Y, U, V: (0,0) DEVICE pointers of
 * pic[0], pic[1] (already swapped by mv_data->reversed) and the output. */
typedef struct thor_interp_plane {
  const uint8_t *p0, *p1;
  uint8_t *out;
  int32_t s0, s1, so;
} thor_interp_plane_t;
int thor_interp_frame(const thor_interp_plane_t *planes, const int16_t *mv0, const int16_t *mv1, int bw, int bh,
                      int width, int height, int wt0, int wt1, void *stream);

/* ---- temporal-interpolated reference frame (interpolate_frames) ----------- *
 * The whole of interpolate_frames (common/temporal_interp.c:972-1053) on the
 * GPU: both references' luma pyramids, motion_estimate_bi per level (:852-918;
 * its raster-order search pass as a wavefront of step rows, then the merge
 * pass) and interpolate_frame (:946-970).  A context holds the scratch for one
 * frame size (pyramid levels, per-level vector fields).                       */
typedef struct thor_ti thor_ti_t;
typedef struct thor_yuv_planes {
  uint8_t *y, *u, *v; /* interior (0,0) of each plane, DEVICE pointers */
  int32_t stride_y, stride_c;
} thor_yuv_planes_t;
thor_ti_t *thor_ti_create(int width, int height, int device);
void thor_ti_destroy(thor_ti_t *t);
/* interpolate_frames(out, ref0, ref1, ratio, pos): ref0 / ref1 padded frames
 * (luma padding pad_y >= 16, edge-replicated, as create_reference_frame leaves
 * them; same strides); out's interior is written (and up to 15 columns / rows
 * past the right and bottom edges), not padded.  Enqueued on `stream`. */
int thor_interpolate_frames(thor_ti_t *t, const thor_yuv_planes_t *ref0, const thor_yuv_planes_t *ref1, int pad_y,
                            const thor_yuv_planes_t *out, int ratio, int pos, void *stream);
/* Host copies of the last call's final vector field of `level` (0 = full
 * size): bw x bh (x, y) int16 pairs each, bw = 2 * ceil((W >> level) / 16),
 * bh likewise (alloc_mv_data, :97-99).  Synchronises the device. */
int thor_ti_read_fields(thor_ti_t *t, int level, int16_t *mv0, int16_t *mv1);
/* THOR_OK, or THOR_ERR_HIP if a search wavefront wait gave up (then cleared). */
int thor_ti_status(thor_ti_t *t);

/* ---- device memory helpers (so the C-ABI is usable without torch) ------ */
void *thor_dev_alloc(size_t bytes);
int thor_dev_free(void *p);
int thor_h2d(void *dst, const void *src, size_t bytes);
int thor_d2h(void *dst, const void *src, size_t bytes);
int thor_device_count(void);
const char *thor_version(void);

#ifdef __cplusplus
}
#endif
#endif
