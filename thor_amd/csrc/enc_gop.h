// Host side of the Thor encoder: encoder parameters, frame-level control
// (coding order, frame type, QP, lambda, reference selection, the sliding
// reference window) and the stream framing.  Restates enc/mainenc.c:73-660,
// enc/encode_frame.c:65-110 and enc/putbits.c:57-95.  Plain C++ (host only).
#pragma once
#include <math.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../../include/thor_amd.h"

#define TE_GOP_MAX_REF 8

// squared_lambda_QP, enc/encode_frame.c:37-44
static const double te_sq_lambda[52] = {
    0.0382,    0.0485,    0.0615,    0.0781,    0.0990,    0.1257,    0.1595,    0.2023,    0.2567,    0.3257,    0.4132,
    0.5243,    0.6652,    0.8440,    1.0709,    1.3588,    1.7240,    2.1874,    2.7754,    3.5214,    4.4679,    5.6688,
    7.1926,    9.1259,    11.5789,   14.6912,   18.6402,   23.6505,   30.0076,   38.0735,   48.3075,   61.2922,   77.7672,
    98.6706,   125.1926,  158.8437,  201.5399,  255.7126,  324.4467,  411.6560,  522.3067,  662.6996,  840.8294,  1066.8393,
    1353.5994, 1717.4389, 2179.0763, 2764.7991, 3507.9607, 4450.8797, 5647.2498, 7165.1970};

static inline int te_log2i_host(unsigned x) {
  int r = 0;
  while (x > 1) {
    x >>= 1;
    r++;
  }
  return r;
}

// Coding order <-> display order of a dyadic sub-GOP, enc/mainenc.c:47-71
static inline int te_reorder_offset(int idx, int sub_gop, int dyadic) {
  static const int cd1[1] = {0}, cd2[2] = {1, 0}, cd4[4] = {3, 1, 0, 2}, cd8[8] = {7, 3, 1, 5, 0, 2, 4, 6},
                   cd16[16] = {15, 7, 3, 11, 1, 5, 9, 13, 0, 2, 4, 6, 8, 10, 12, 14};
  static const int *c2d[5] = {cd1, cd2, cd4, cd8, cd16};
  if (dyadic && sub_gop > 1) return c2d[te_log2i_host(sub_gop)][idx] - sub_gop + 1;
  return idx == 0 ? 0 : idx - sub_gop;
}
static inline int te_display_to_code(int sub_gop, int i) {
  static const int dc1[2] = {-1, 0}, dc2[3] = {-2, 1, 0}, dc4[5] = {-4, 2, 1, 3, 0}, dc8[9] = {-8, 4, 2, 5, 1, 6, 3, 7, 0},
                   dc16[17] = {-16, 8, 4, 9, 2, 10, 5, 11, 1, 12, 6, 13, 3, 14, 7, 15, 0};
  static const int *d2c[5] = {dc1, dc2, dc4, dc8, dc16};
  return d2c[te_log2i_host(sub_gop)][i];
}

// One frame's plan: what encode_frame needs from main().
struct TeFramePlan {
  int input_index;  // frame of the input sequence (display order, after -skip)
  int frame_num;    // frame_info.frame_num
  int frame_type, qp, b_level, num_ref, interp_ref, num_intra_modes;
  int ref_array[TE_GOP_MAX_REF];  // indices into the sliding window (ref[0] = most recently coded)
  int ref_fnum[TE_GOP_MAX_REF];   // frame numbers of those references when this frame is coded
  // interp_ref: ref index 0 is interpolate_frames(window[interp_a], window[interp_b],
  // interp_ratio, interp_pos), numbered frame_num (enc/mainenc.c:324-330, :381-387)
  int interp_a, interp_b, interp_ratio, interp_pos;
  double lambda;
};

// The per-frame decisions of main()'s frame loop (enc/mainenc.c:222-491),
// driven frame by frame; `window_fnum` mirrors encoder_info.ref[]'s frame
// numbers (garbage-free: slots never written hold INT32_MIN and are never
// referenced by conformant plans).
struct TeGop {
  thor_enc_params_t p;
  int sub_gop, min_interp_depth, last_PorI_frame, last_intra_frame_num, num_encoded;
  int frame_num0, k;  // position in the coding-order loop
  std::vector<int> window_fnum;
  std::vector<TeFramePlan> plans;  // every frame, coding order

  explicit TeGop(const thor_enc_params_t &prm) : p(prm) {
    sub_gop = p.num_reorder_pics + 1 > 1 ? p.num_reorder_pics + 1 : 1;
    min_interp_depth = te_log2i_host(p.num_reorder_pics + 1) - 2;
    if (p.frame_rate > 30) min_interp_depth--;
    last_PorI_frame = -1;
    last_intra_frame_num = 0;
    num_encoded = 0;
    window_fnum.assign(33, (int)0x80000000);
    plan_all();
  }

  void plan_frame(int frame_num_in, TeFramePlan &f) {
    thor_enc_params_t &P = p;
    f.input_index = frame_num_in;
    f.frame_num = frame_num_in - P.skip;
    if (P.num_reorder_pics == 0) {
      f.frame_type = P.intra_period > 0 ? ((num_encoded % P.intra_period) == 0 ? 0 : 1) : (num_encoded == 0 ? 0 : 1);
    } else {
      if (P.intra_period > 0)
        f.frame_type = (f.frame_num % P.intra_period) == 0 ? 0 : ((f.frame_num % sub_gop) == 0 ? 1 : 2);
      else
        f.frame_type = f.frame_num == 0 ? 0 : ((f.frame_num % sub_gop) == 0 ? 1 : 2);
    }
    const int coded_phase = (num_encoded + sub_gop - 2) % sub_gop + 1;
    const int b_level = te_log2i_host(coded_phase);
    f.b_level = b_level;
    int qp;
    if (f.frame_type == 0) {
      qp = P.qp + P.dqpI;
      last_intra_frame_num = f.frame_num;
    } else if (P.num_reorder_pics == 0) {
      qp = (num_encoded % P.HQperiod) ? (int)(P.mqpP * (float)P.qp) + P.dqpP : P.qp;
    } else if (f.frame_num % sub_gop) {
      const float m[5] = {P.mqpB0, P.mqpB1, P.mqpB2, P.mqpB3, P.mqpB};
      const int d[5] = {P.dqpB0, P.dqpB1, P.dqpB2, P.dqpB3, P.dqpB};
      const int lv = P.dyadic_coding ? (b_level < 4 ? b_level : 4) : 4;
      qp = (int)(m[lv] * (float)P.qp) + d[lv];
    } else {
      qp = (f.frame_num % P.HQperiod) ? (int)(P.mqpP * (float)P.qp) + P.dqpP : P.qp;
    }
    f.qp = qp < 0 ? 0 : (qp > 51 ? 51 : qp);
    f.num_ref = f.frame_type == 0 ? 0 : (num_encoded < P.max_num_ref ? num_encoded : P.max_num_ref);
    f.interp_ref = 0;
    f.interp_a = f.interp_b = -1;
    f.interp_ratio = f.interp_pos = 0;
    int *ra = f.ref_array;
    for (int r = 0; r < TE_GOP_MAX_REF; r++) ra[r] = 0;
    if (f.num_ref > 0) {
      if (P.num_reorder_pics > 0) {
        if (P.dyadic_coding) {
          if ((num_encoded - 1) % sub_gop == 0) {
            ra[0] = num_encoded == 1 ? 0 : sub_gop - 1;
            if (f.num_ref > 1) ra[1] = mini(32, mini(num_encoded - 1, 2 * sub_gop - 1));
            for (int r = 2; r < f.num_ref; r++) ra[r] = r - 2;
          } else {
            const int display_phase = (f.frame_num - 1) % sub_gop;
            const int ref_offset = sub_gop >> (b_level + 1);
            if (b_level >= min_interp_depth && P.interp_ref) {
              if (f.num_ref == 2) f.num_ref++;
              f.interp_ref = 1;
              ra[1] = mini(num_encoded - 1, coded_phase - te_display_to_code(sub_gop, display_phase - ref_offset + 1) - 1);
              ra[2] = mini(num_encoded - 1, coded_phase - te_display_to_code(sub_gop, display_phase + ref_offset + 1) - 1);
              ra[0] = -1;
              f.interp_a = ra[1];
              f.interp_b = ra[2];
              f.interp_ratio = 2;
              f.interp_pos = 1;
              for (int r = 3; r < f.num_ref; r++) ra[r] = r - 3;
            } else {
              ra[0] = mini(num_encoded - 1, coded_phase - te_display_to_code(sub_gop, display_phase - ref_offset + 1) - 1);
              ra[1] = mini(num_encoded - 1, coded_phase - te_display_to_code(sub_gop, display_phase + ref_offset + 1) - 1);
              for (int r = 2; r < f.num_ref; r++) ra[r] = r - 2;
            }
          }
        } else {
          if ((num_encoded - 1) % sub_gop == 0) {
            ra[0] = num_encoded == 1 ? 0 : sub_gop - 1;
            if (f.num_ref > 1) ra[1] = mini(32, mini(num_encoded - 1, 2 * sub_gop - 1));
            for (int r = 2; r < f.num_ref; r++) ra[r] = r - 1;
          } else {
            const int phase = (num_encoded + sub_gop - 2) % sub_gop;
            if (P.interp_ref && f.num_ref > 0) {
              if (f.num_ref == 2) f.num_ref++;
              f.interp_ref = 1;
              ra[1] = 0;
              if (f.num_ref > 1) ra[2] = phase == 0 ? mini(sub_gop, num_encoded - 1) : mini(phase, num_encoded - 1);
              ra[0] = -1;
              f.interp_a = ra[1];
              f.interp_b = ra[2];
              f.interp_ratio = sub_gop - phase;
              f.interp_pos = phase != 0 ? 1 : sub_gop - phase - 1;
              if (f.num_ref > 2) ra[3] = mini(phase ? phase + sub_gop : 2 * sub_gop, num_encoded - 1);
              for (int r = 4; r < f.num_ref; r++) ra[r] = r - 4 + 1;
            } else {
              ra[0] = 0;
              if (f.num_ref > 1) ra[1] = phase == 0 ? mini(sub_gop, num_encoded - 1) : mini(phase, num_encoded - 1);
              if (f.num_ref > 2) ra[2] = mini(phase ? phase + sub_gop : 2 * sub_gop, num_encoded - 1);
              for (int r = 3; r < f.num_ref; r++) ra[r] = r - 3 + 1;
            }
          }
        }
      } else {
        ra[0] = last_PorI_frame;
        if (f.num_ref == 2) {
          ra[1] = ((num_encoded + P.HQperiod - 2) % P.HQperiod) + 1;
        } else if (f.num_ref == 3) {
          const int r1 = ((num_encoded + P.HQperiod - 2) % P.HQperiod) + 1;
          ra[1] = r1;
          ra[2] = r1 == 1 ? 2 : 1;
        } else if (f.num_ref == 4) {
          const int r1 = ((num_encoded + P.HQperiod - 2) % P.HQperiod) + 1, r2 = r1 == 1 ? 2 : 1;
          int r3 = r2 + 1;
          if (r3 == r1) r3 += 1;
          ra[1] = r1;
          ra[2] = r2;
          ra[3] = r3;
        } else {
          for (int r = 1; r < f.num_ref; r++) ra[r] = r;
        }
      }
    }
    // remove duplicate references (:457-470)
    for (int r = f.num_ref - 1; r > 0; --r)
      for (int k2 = r - 1; k2 >= 0; --k2)
        if (ra[k2] == ra[r]) {
          for (int s = r; s < f.num_ref - 1; ++s) ra[s] = ra[s + 1];
          f.num_ref--;
          break;
        }
    // remove references that break random access (:472-486)
    if (f.frame_num > last_intra_frame_num)
      for (int r = f.num_ref - 1; r >= 0; --r)
        if (ra[r] >= 0 && window_fnum[ra[r]] < last_intra_frame_num) {
          for (int s = r; s < f.num_ref - 1; ++s) ra[s] = ra[s + 1];
          f.num_ref--;
        }
    for (int r = 0; r < TE_GOP_MAX_REF; r++)
      f.ref_fnum[r] = r >= f.num_ref ? -1 : (ra[r] < 0 ? f.frame_num : (ra[r] < 33 ? window_fnum[ra[r]] : -1));
    f.num_intra_modes = (P.intra_rdo == 0 || (f.frame_type != 0 && P.encoder_speed > 0)) ? 4 : 10;
    // lambda (enc/encode_frame.c:77-94): float coefficients promoted to double
    float lc;
    if (f.frame_type == 0) lc = P.lambda_coeffI;
    else if (f.frame_type == 1) lc = P.lambda_coeffP;
    else {
      const float c[5] = {P.lambda_coeffB0, P.lambda_coeffB1, P.lambda_coeffB2, P.lambda_coeffB3, P.lambda_coeffB};
      lc = c[f.b_level < 4 ? f.b_level : 4];
    }
    f.lambda = lc * te_sq_lambda[f.qp];
  }

  // after a frame is coded: slide the window (enc/encode_frame.c:165-177) and
  // main()'s bookkeeping (:517-579)
  void commit(const TeFramePlan &f) {
    for (int r = 32; r > 0; r--) window_fnum[r] = window_fnum[r - 1];
    window_fnum[0] = f.frame_num;
    num_encoded++;
    last_PorI_frame = f.frame_type != 2 ? 0 : last_PorI_frame + 1;
  }

  // The whole coding-order plan for p.num_frames input frames (main()'s two
  // loops, :222-591, including the revert to PPP coding at the tail).
  void plan_all() {
    plans.clear();
    const int nin = p.skip + p.num_frames;
    for (int f0 = p.skip; f0 < p.skip + p.num_frames && f0 < nin; f0 += sub_gop) {
      for (int kk = 0; kk < sub_gop; kk++) {
        const int fn = f0 + te_reorder_offset(kk, sub_gop, p.dyadic_coding);
        if (fn < p.skip) continue;
        TeFramePlan f;
        plan_frame(fn, f);
        plans.push_back(f);
        commit(f);
      }
      if ((f0 + sub_gop + 1 > nin || f0 + sub_gop >= p.skip + p.num_frames) && sub_gop >= 2) {
        p.HQperiod = sub_gop;
        sub_gop = 1;
        p.num_reorder_pics = 0;
      }
    }
  }
  static int mini(int a, int b) { return a < b ? a : b; }
};

// Early-skip thresholds (check_early_skip_transform_coeff / _sub_blockC,
// enc/encode_block.c:2481-2611 with the thresholds of check_early_skip_block
// :2632-2636), [scaled][qp][kind]: kind 0..2 luma (N/2 = 4, 8, 16), 3 chroma.
static inline void te_es_thresholds(float early_skip_thr, int *out /* 2*52*4 */) {
  for (int sc = 0; sc < 2; sc++) {
    float t = early_skip_thr;
    if (sc) t = (float)(1.3 * t);
    for (int qp = 0; qp < 52; qp++) {
      static const int gq[6] = {26214, 23302, 20560, 18396, 16384, 14564};
      const int scale = gq[qp % 6];
      for (int k = 0; k < 3; k++) {
        const int size2 = 4 << k, lg = te_log2i_host(size2);
        const int shift2 = 21 - lg + qp / 6;
        const double fql = (double)(1 << shift2) / (double)scale;
        const double rel = 0.5 * t;
        out[(sc * 52 + qp) * 4 + k] = (int)(rel * fql);
      }
      const int shift2 = 21 - 5 + qp / 6;
      const double fql = (double)(1 << shift2) / (double)scale;
      out[(sc * 52 + qp) * 4 + 3] = (int)(t * fql);
    }
  }
}

// Bit string builder for headers (putbits, enc/putbits.c:112-129)
struct TeHostBits {
  std::vector<uint8_t> bytes;
  uint64_t nbits = 0;
  void put(int n, uint32_t v) {
    for (int i = n - 1; i >= 0; i--) {
      const int bit = (v >> i) & 1;
      if ((nbits & 7) == 0) bytes.push_back(0);
      if (bit) bytes.back() |= (uint8_t)(0x80 >> (nbits & 7));
      nbits++;
    }
  }
  // append `n` bits from an MSB-first word buffer
  void append_words(const uint32_t *w, int n) {
    for (int i = 0; i < n; i++) put(1, (w[i >> 5] >> (31 - (i & 31))) & 1);
  }
};

// Sequence header, enc/mainenc.c:196-207
static inline void te_seq_header(TeHostBits &b, const thor_enc_params_t &p) {
  b.put(16, p.width);
  b.put(16, p.height);
  b.put(1, p.enable_pb_split);
  b.put(1, p.enable_tb_split);
  b.put(2, p.max_num_ref - 1);
  b.put(1, p.interp_ref);
  b.put(3, p.max_delta_qp);
  b.put(1, p.deblocking);
  b.put(1, p.clpf);
  b.put(1, p.use_block_contexts);
  b.put(1, p.enable_bipred);
}
// Frame header, enc/encode_frame.c:96-110
static inline void te_frame_header(TeHostBits &b, const TeFramePlan &f) {
  b.put(1, f.frame_type != 0);
  b.put(8, f.qp);
  b.put(4, f.num_intra_modes);
  if (f.frame_type != 0) b.put(2, f.num_ref - 1);
  for (int r = 0; r < f.num_ref; r++) b.put(6, f.ref_array[r] + 1);
  b.put(16, f.frame_num);
}

// enc/strings.c:286-338 defaults
static inline void te_default_params(thor_enc_params_t *p) {
  memset(p, 0, sizeof(*p));
  p->num_frames = 600;
  p->width = 1920;
  p->height = 1080;
  p->qp = 32;
  p->frame_rate = 60;
  p->lambda_coeffI = p->lambda_coeffP = p->lambda_coeffB = 1.0f;
  p->lambda_coeffB0 = p->lambda_coeffB1 = p->lambda_coeffB2 = p->lambda_coeffB3 = 1.0f;
  p->early_skip_thr = 0.0f;
  p->max_num_ref = 1;
  p->HQperiod = 1;
  p->dyadic_coding = 1;
  p->mqpP = p->mqpB = p->mqpB0 = p->mqpB1 = p->mqpB2 = p->mqpB3 = 1.0f;
  p->delta_qp_step = 1;
  p->deblocking = 1;
  p->clpf = 1;
  p->snrcalc = 1;
}

// Set one parameter by its command-line name ("-qp" etc.): 0 ok, -1 unknown.
static inline int te_set_param(thor_enc_params_t *p, const char *k, const char *v) {
#define TE_I(n)                      \
  if (!strcmp(k, "-" #n)) {          \
    p->n = (int32_t)atoi(v);         \
    return 0;                        \
  }
#define TE_F(n)                      \
  if (!strcmp(k, "-" #n)) {          \
    p->n = (float)atof(v);           \
    return 0;                        \
  }
  TE_I(width) TE_I(height) TE_I(qp) TE_I(skip) TE_F(frame_rate)
  TE_F(lambda_coeffI) TE_F(lambda_coeffP) TE_F(lambda_coeffB) TE_F(lambda_coeffB0) TE_F(lambda_coeffB1)
  TE_F(lambda_coeffB2) TE_F(lambda_coeffB3) TE_F(early_skip_thr) TE_I(enable_tb_split) TE_I(enable_pb_split)
  TE_I(max_num_ref) TE_I(HQperiod) TE_I(num_reorder_pics) TE_I(dyadic_coding) TE_I(interp_ref) TE_I(dqpP)
  TE_I(dqpB) TE_I(dqpB0) TE_I(dqpB1) TE_I(dqpB2) TE_I(dqpB3) TE_F(mqpP) TE_F(mqpB) TE_F(mqpB0) TE_F(mqpB1)
  TE_F(mqpB2) TE_F(mqpB3) TE_I(dqpI) TE_I(intra_period) TE_I(intra_rdo) TE_I(rdoq) TE_I(max_delta_qp)
  TE_I(delta_qp_step) TE_I(encoder_speed) TE_I(sync) TE_I(deblocking) TE_I(clpf) TE_I(snrcalc)
  TE_I(use_block_contexts) TE_I(enable_bipred)
  if (!strcmp(k, "-n")) {
    p->num_frames = atoi(v);
    return 0;
  }
  if (!strcmp(k, "-f")) {
    p->frame_rate = (float)atof(v);
    return 0;
  }
#undef TE_I
#undef TE_F
  return -1;
}

// What this device encoder supports (and check_parameters, enc/strings.c:431-479)
static inline int te_check_params(const thor_enc_params_t *p) {
  // check_parameters (enc/strings.c:431-479); its fatalerror() is THOR_ERR_ARG here
  if (p->num_frames <= 0) return THOR_ERR_ARG;
  if (p->width <= 0 || p->height <= 0 || (p->width & 7) || (p->height & 7)) return THOR_ERR_ARG;
  if (p->max_num_ref < 1 || p->max_num_ref > 4) return THOR_ERR_ARG;
  if (p->max_delta_qp >= 8) return THOR_ERR_ARG;
  if (p->HQperiod >= 33) return THOR_ERR_ARG;  // MAX_REF_FRAMES, common/global.h:67
  const int nrp1 = p->num_reorder_pics + 1;
  if (p->num_reorder_pics > 0 && p->HQperiod > 1 && p->HQperiod % nrp1) return THOR_ERR_ARG;
  if (p->dyadic_coding && (nrp1 < 1 || (nrp1 & (nrp1 - 1)))) return THOR_ERR_ARG;
  if (p->num_reorder_pics > 0 && p->max_num_ref < 2) return THOR_ERR_ARG;
  if (nrp1 != 0 && p->intra_period % nrp1) return THOR_ERR_ARG;
  // what the reference leaves to the user but this encoder needs: the header
  // field widths (16-bit sizes, 3-bit max_delta_qp), a sub-GOP of at most 16
  // (the coding-order tables), a QP trial loop that ends, a window of one
  // HQ period at least
  if (p->width > 65535 || p->height > 65535 || p->qp < 0 || p->qp > 51 || p->HQperiod < 1) return THOR_ERR_ARG;
  if (p->num_reorder_pics < 0 || nrp1 > 16 || p->max_delta_qp < 0) return THOR_ERR_ARG;
  if (p->max_delta_qp > 0 && p->delta_qp_step < 1) return THOR_ERR_ARG;
  if (p->skip < 0) return THOR_ERR_ARG;
  if (p->rdoq) return THOR_ERR_ARG;  // full RDOQ is not implemented
  if (p->sync) return THOR_ERR_ARG;  // WPP row sync (requires encoder_speed 2 in the reference) is not implemented
  return THOR_OK;
}
