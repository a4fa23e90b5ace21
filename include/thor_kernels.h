/*
 * thor_amd -- the reference's SIMD kernel surface, exported by libthor_amd.so
 * with the reference's own names and signatures so that Thor's host C links
 * it in place of common/common_kernels.c (+ enc/enc_kernels.c).
 *
 * Every entry point runs on the GPU (one small kernel per call, inputs staged
 * through device memory).  Semantics are the reference SIMD build's, which is
 * the reference; each declaration cites the reference
 * declaration it replaces.  Like the reference, these return no status; a
 * GPU failure aborts rather than return wrong pixels.
 */
#ifndef THOR_KERNELS_H
#define THOR_KERNELS_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* common/common_kernels.h:32 */
void block_avg_simd(uint8_t *p, uint8_t *r0, uint8_t *r1, int sp, int s0, int s1, int width, int height);
/* common/common_kernels.h:33 */
int sad_calc_simd_unaligned(uint8_t *a, uint8_t *b, int astride, int bstride, int width, int height);
/* common/common_kernels.h:34 -- xoff/yoff: quarter-pel fractions; ip: integer-displaced reference */
void get_inter_prediction_luma_simd(int width, int height, int xoff, int yoff, unsigned char *qp, int qstride,
                                    const unsigned char *ip, int istride, int bipred);
/* common/common_kernels.h:35 -- xoff/yoff: eighth-pel fractions */
void get_inter_prediction_chroma_simd(int width, int height, int xoff, int yoff, unsigned char *qp, int qstride,
                                      const unsigned char *ip, int istride);
/* common/common_kernels.h:36 */
void transform_simd(const int16_t *block, int16_t *coeff, int size, int fast);
/* common/common_kernels.h:37 */
void inverse_transform_simd(const int16_t *coeff, int16_t *block, int size);
/* common/common_kernels.h:38-39 */
void clpf_block4(const uint8_t *src, uint8_t *dst, int sstride, int dstride, int x0, int y0, int width, int height);
void clpf_block8(const uint8_t *src, uint8_t *dst, int sstride, int dstride, int x0, int y0, int width, int height);

/* enc/enc_kernels.h:32-37 */
int sad_calc_simd(uint8_t *a, uint8_t *b, int astride, int bstride, int width, int height);
int ssd_calc_simd(uint8_t *a, uint8_t *b, int astride, int bstride, int size);
void detect_clpf_simd(const uint8_t *rec, const uint8_t *org, int x0, int y0, int width, int height, int so,
                      int stride, int *sum0, int *sum1);
unsigned int sad_calc_fasthalf_simd(const uint8_t *a, const uint8_t *b, int astride, int bstride, int width,
                                    int height, int *x, int *y);
unsigned int sad_calc_fastquarter_simd(const uint8_t *o, const uint8_t *r, int os, int rs, int width, int height,
                                       int *x, int *y);
unsigned int widesad_calc_simd(uint8_t *a, uint8_t *b, int astride, int bstride, int width, int height, int *x);

#ifdef __cplusplus
}
#endif
#endif
