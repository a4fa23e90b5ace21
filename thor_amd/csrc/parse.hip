// Host side: the .bit parser that feeds the batched GPU decoder.
//
// Restates the reference decoder's serial syntax layer -- the bit reader
// (dec/getbits.c:48-162), the VLC tables (dec/getvlc.c:33-207), the frame
// header and CLPF signalling (dec/decode_frame.c:45-133), the quadtree walk
// (process_block_dec / decode_super_mode, dec/decode_block.c:474-669) and the
// block syntax (read_block / read_coeff / read_mv, dec/read_bits.c:46-820) --
// and emits, per frame, exactly what the GPU path consumes: thor_block_t
// descriptors in decode order, the compact coefficient pool and the per-SB
// CLPF flags (include/thor_amd.h).  MV prediction and skip / merge candidates
// come from the same neighbour logic the device encoder uses (enc_core.h).
// Serial bit parsing is host work by design.
#include <string.h>

#include <vector>

#include "common.h"
#include "enc_core.h"

namespace {

// getbits / getbits1 / showbits / flushbits over one frame's payload; bits
// past the end read as zero (fillbfr, dec/getbits.c:71-106).  The payload is
// copied once into a zero-padded buffer, so a read of up to 32 bits is one
// unaligned big-endian 64-bit load and two shifts.
struct TpBits {
  std::vector<uint8_t> buf;
  size_t nbits = 0, pos = 0;
  bool err = false;  // a malformed code word (corrupt input): the frame is rejected
  void set(const uint8_t *p, size_t nbytes) {
    buf.assign(nbytes + 16, 0);
    if (nbytes) memcpy(buf.data(), p, nbytes);
    nbits = nbytes * 8;
    pos = 0;
    err = false;
  }
  uint32_t show(int n) const {  // n <= 32
    if (n <= 0) return 0;
    const size_t byte = pos >> 3;
    if (byte + 8 > buf.size()) return 0;  // far past the end (corrupt input): zeros
    uint64_t w;
    memcpy(&w, buf.data() + byte, 8);
    w = __builtin_bswap64(w) << (pos & 7);
    return (uint32_t)(w >> (64 - n));
  }
  uint32_t get(int n) {
    const uint32_t v = show(n);
    pos += n;
    return v;
  }
  uint32_t get1() {
    const uint32_t v = show(1);
    pos++;
    return v;
  }
  void flush(int n) { pos += n; }
};

// get_vlc0_limit, dec/getvlc.c:33-43
int vlc0_limit(TpBits &b, int maxbit) {
  int tmp = 0, nbit = 0;
  while (tmp == 0 && nbit < maxbit) {
    tmp = (int)b.get1();
    nbit++;
  }
  return tmp == 0 ? maxbit : nbit - 1;
}

// get_vlc, dec/getvlc.c:45-207 (tables 0-5 and 10: the ones the syntax uses)
int get_vlc(TpBits &b, int n) {
  if (n < 6) {
    int zeroes = 0, cw = 0, done = 0;
    while (!done && zeroes < 6) {
      if (b.get1()) {
        cw = (int)b.get(n);
        done = 1;
      } else {
        zeroes++;
      }
    }
    if (done) return (zeroes << n) + cw;
    int lead = n;
    for (;;) {
      if (!b.show(1)) {
        lead++;
        b.flush(1);
        if (lead > 30) {  // no valid code word is this long (corrupt or truncated input)
          b.err = true;
          return 0;
        }
      } else {
        const int tmp = (int)b.get(lead + 1);
        return 6 * (1 << n) + tmp - (1 << n);
      }
    }
  }
  // n == 10
  int lead = 0;
  for (;;) {
    if (!b.show(1)) {
      lead++;
      b.flush(1);
      if (lead > 30) {  // corrupt stream: stop consuming
        b.err = true;
        return 0;
      }
    } else {
      return (int)b.get(lead + 1) - 1;
    }
  }
}

// read_mv, dec/read_bits.c:46-58
TeMv read_mv(TpBits &b, TeMv mvp) {
  TeMv m;
  int code = get_vlc(b, 10);
  m.x = (int16_t)(mvp.x + ((code & 1) ? -((code + 1) / 2) : code / 2));
  code = get_vlc(b, 10);
  m.y = (int16_t)(mvp.y + ((code & 1) ? -((code + 1) / 2) : code / 2));
  return m;
}

// find_index, dec/read_bits.c:63-99
int find_index(int code, int maxrun, int type) {
  const int maxrun2 = maxrun > 4 ? maxrun : 4;
  if (type) {
    if (code == 0) return -1;
    if (code <= 5) return code - 1;
    if (code == 6) return maxrun2 + 1;
    if (code == 7) return maxrun2 + 2;
    if (code <= maxrun2 + 3) return code - 3;
    return code - 1;
  }
  if (code <= 1) return code;
  if (code == 2) return -1;
  if (code <= 5) return code - 1;
  if (code == 6) return maxrun2 + 1;
  if (code == 7) return maxrun2 + 2;
  if (code <= maxrun2 + 3) return code - 3;
  return code - 1;
}

// read_coeff, dec/read_bits.c:101-210, into a q x q tile (q = min(size, 16),
// raster); returns non-zero if any level is non-zero
int read_coeff(TpBits &b, int16_t *tile, int size, int type) {
  const int q = size < 16 ? size : 16, N = q * q;
  const int chroma = type & 1, intra = (type >> 1) & 1;
  int vlc_adaptive = intra && !chroma;
  int16_t sc[256];
  memset(sc, 0, sizeof(sc));
  int pos = 0;
  if (chroma) {
    if (b.get1()) {
      sc[0] = b.get1() ? -1 : 1;
      pos = N;
    }
  }
  int level_mode = 1, level = 1;
  while (pos < N) {
    if (level_mode) {
      while (pos < N && level > 0) {
        level = get_vlc(b, vlc_adaptive);
        const int sign = level ? (int)b.get1() : 1;
        sc[pos] = (int16_t)(sign ? -level : level);
        if (chroma == 0) vlc_adaptive = level > 3;
        pos++;
      }
    }
    if (pos >= N) break;
    const int maxrun = N - pos - 1;
    int code;
    if (chroma && size <= 8) {
      code = get_vlc(b, 10);
    } else {
      if (b.show(2) == 2) code = (int)b.get(2) - 2;
      else code = get_vlc(b, 2) - 1;
    }
    if (code < 0) {  // only a malformed (all-zero) code word decodes below 0
      b.err = true;
      break;
    }
    const int index = find_index(code, maxrun, chroma);
    if (index == -1) break;
    const int maxrun2 = maxrun > 4 ? maxrun : 4;
    const int level_flag = index / (maxrun2 + 1), run = index % (maxrun2 + 1);
    pos += run;
    int sign;
    if (level_flag) {
      const int tmp = get_vlc(b, 0);
      sign = tmp & 1;
      level = (tmp >> 1) + 2;
    } else {
      level = 1;
      sign = (int)b.get1();
    }
    if (pos < 256) sc[pos] = (int16_t)(sign ? -level : level);
    level_mode = level > 1;
    pos++;
  }
  int any = 0;
  for (int r = 0; r < N; r++) {
    tile[r] = sc[te_zz(q, r)];
    any |= tile[r] != 0;
  }
  return any;
}

}  // namespace

struct thor_parser {
  int have_seq = 0;
  thor_seq_t seq;
  int pb_split = 0, max_num_ref = 0, interp_ref = 0, max_delta_qp = 0, use_block_contexts = 0;
  int decode_order = 0;
  std::vector<int> window;  // frame numbers of the sliding window (decode_frame.c:135-147)
  std::vector<TeCell> cells;
  // current frame
  TpBits b;
  int frame_type = 0, qp = 0, qpb = 0, num_ref = 0, num_intra_modes = 0, fr_interp = 0, frame_num = 0;
  int ref_array[8];
  std::vector<thor_block_t> blocks;
  std::vector<int16_t> coeffs;
  std::vector<uint8_t> clpf, clpf_cand;
  int clpf_on = 0;
  int error = 0;
};

namespace {

int ref_frame_num(const thor_parser *P, int ref_idx) {
  if (ref_idx < 0 || ref_idx >= P->num_ref) return -1;
  const int r = P->ref_array[ref_idx];
  if (r < 0) return -2;
  return P->window[r];
}

// decode_super_mode, dec/decode_block.c:474-622.  Returns split_flag; *mode / *ref_idx.
int super_mode(thor_parser *P, int size, int decode_this, const TeCtx &ctx, int *mode, int *ref_idx) {
  TpBits &b = P->b;
  *mode = TE_SKIP;
  if (P->frame_type == TE_I) {
    *mode = TE_INTRA;
    if (size > 8 && decode_this) return (int)b.get(1);
    return !decode_this;
  }
  if (!decode_this) return !b.get(1);
  if (size > 64) {
    const int split = !b.get(1);
    return split;
  }
  const int num_ref = P->num_ref;
  const int bipred_possible = num_ref > 1 && P->seq.bipred;
  const int split_possible = size > 8;
  const int maxbit = 2 + num_ref + split_possible + bipred_possible;
  int code = vlc0_limit(b, maxbit);
  if (P->fr_interp) {
    if ((ctx.index == 2 || ctx.index > 3) && size > 8)
      if (code < 3) code = (code + 1) % 3;
    if (split_possible && code == 1) return 1;
    if (!split_possible && code > 0) code += 1;
    if (!bipred_possible && code >= 3) code += 1;
    if (code == 0) *mode = TE_SKIP;
    else if (code == 2) *mode = TE_MERGE;
    else if (code == 3) *mode = TE_BIPRED;
    else if (code == 4) *mode = TE_INTRA;
    else if (code == 4 + num_ref) {
      *mode = TE_INTER;
      *ref_idx = 0;
    } else {
      *mode = TE_INTER;
      *ref_idx = code - 4;
    }
    return 0;
  }
  if ((ctx.index == 2 || ctx.index > 3) && size > 8)
    if (code < 4) code = (code + 1) % 4;
  if (split_possible && code == 1) return 1;
  if (!split_possible && code > 0) code += 1;
  if (!bipred_possible && code >= 4) code += 1;
  if (code == 0) *mode = TE_SKIP;
  else if (code == 2) {
    *mode = TE_INTER;
    *ref_idx = 0;
  } else if (code == 3) *mode = TE_MERGE;
  else if (code == 4) *mode = TE_BIPRED;
  else if (code == 5) *mode = TE_INTRA;
  else {
    *mode = TE_INTER;
    *ref_idx = code - 5;
  }
  return 0;
}

// read_block, dec/read_bits.c:221-820, + copy_deblock_data (dec/decode_block.c:122-156)
void read_block(thor_parser *P, int size, int ypos, int xpos, int mode, int ref_idx_in, const TeCtx &ctx) {
  TpBits &b = P->b;
  const int W = P->seq.width, H = P->seq.height;
  thor_block_t B;
  memset(&B, 0, sizeof(B));
  B.ypos = (uint16_t)ypos;
  B.xpos = (uint16_t)xpos;
  B.size = (uint8_t)size;
  B.bwidth = (uint8_t)(size < W - xpos ? size : W - xpos);
  B.bheight = (uint8_t)(size < H - ypos ? size : H - ypos);
  B.mode = (uint8_t)mode;
  B.qp = (uint8_t)P->qpb;
  TeMv m0[4], m1[4];
  memset(m0, 0, sizeof(m0));
  memset(m1, 0, sizeof(m1));
  int ref_idx0 = 0, ref_idx1 = 0, dir = 0, pb_part = 0, intra_mode = 0, tb_split = 0;
  int cbp_y = 0, cbp_u = 0, cbp_v = 0;
  const int coeff_type = (mode == TE_INTRA) << 1;
  if (mode == TE_SKIP || mode == TE_MERGE) {
    TeInterPred cand[2];
    const int n = te_mv_skip(ypos, xpos, W, H, size, P->cells.data(), cand);
    int idx = 0;
    if (n == 2) idx = (int)b.get(1);
    ref_idx0 = cand[idx].ref_idx0;
    ref_idx1 = cand[idx].ref_idx1;
    for (int i = 0; i < 4; i++) {
      m0[i] = cand[idx].mv0;
      m1[i] = cand[idx].mv1;
    }
    dir = cand[idx].bipred_flag;
  } else if (mode == TE_INTER) {
    if (P->pb_split) {
      if (b.get(1)) pb_part = 0;
      else if (b.get(1)) pb_part = 1;
      else pb_part = 3 - (int)b.get(1);
    }
    const int ref_idx = P->num_ref > 1 ? ref_idx_in : 0;
    const TeMv mvp = te_mv_pred(ypos, xpos, W, H, size, P->cells.data());
    TeMv mvp2 = mvp;
    if (pb_part == 0) {
      m0[0] = read_mv(b, mvp2);
      m0[1] = m0[2] = m0[3] = m0[0];
    } else if (pb_part == 1) {
      m0[0] = read_mv(b, mvp2);
      mvp2 = m0[0];
      m0[2] = read_mv(b, mvp2);
      m0[1] = m0[0];
      m0[3] = m0[2];
    } else if (pb_part == 2) {
      m0[0] = read_mv(b, mvp2);
      mvp2 = m0[0];
      m0[1] = read_mv(b, mvp2);
      m0[2] = m0[0];
      m0[3] = m0[1];
    } else {
      m0[0] = read_mv(b, mvp2);
      mvp2 = m0[0];
      m0[1] = read_mv(b, mvp2);
      m0[2] = read_mv(b, mvp2);
      m0[3] = read_mv(b, mvp2);
    }
    for (int i = 0; i < 4; i++) m1[i] = m0[i];
    ref_idx0 = ref_idx1 = ref_idx;
    dir = 0;
  } else if (mode == TE_BIPRED) {
    const TeMv mvp = te_mv_pred(ypos, xpos, W, H, size, P->cells.data());
    TeMv mvp2 = mvp;
    m0[0] = read_mv(b, mvp2);
    m0[1] = m0[2] = m0[3] = m0[0];
    // stat_frame_type: a frame with a future reference counts as B (decode_frame.c:79-85)
    int is_b = P->frame_type == TE_B;
    for (int r = 0; r < P->num_ref; r++)
      if (P->ref_array[r] != -1 && P->window[P->ref_array[r]] > P->frame_num) is_b = 1;
    if (is_b) mvp2 = m0[0];
    m1[0] = read_mv(b, mvp2);
    m1[1] = m1[2] = m1[3] = m1[0];
    if (is_b) {
      ref_idx0 = 0;
      ref_idx1 = 1;
      if (P->fr_interp == 1) {
        ref_idx0++;
        ref_idx1++;
      }
    } else if (P->num_ref == 2) {
      const int code = vlc0_limit(b, 3);
      ref_idx0 = (code >> 1) & 1;
      ref_idx1 = code & 1;
    } else {
      const int code = get_vlc(b, 10);
      ref_idx0 = (code >> 2) & 3;
      ref_idx1 = code & 3;
    }
    dir = 2;
  } else {  // INTRA
    if (P->num_intra_modes <= 4) {
      intra_mode = (int)b.get(2);
    } else if (P->num_intra_modes <= 8) {
      const int inv[10] = {3, 2, 0, 9, 8, 4, 7, 6, 1, 5};
      int code, tmp = (int)b.get(2);
      if (tmp < 3) code = tmp;
      else {
        tmp = (int)b.get(2);
        code = tmp < 3 ? 3 + tmp : 6 + (int)b.get(1);
      }
      intra_mode = inv[code];
    } else {
      const int inv[10] = {3, 2, 0, 1, 9, 8, 4, 7, 6, 5};
      int code;
      if (b.get(1)) code = (int)b.get(1);
      else if (b.get(1)) code = 2 + (int)b.get(1);
      else if (b.get(1)) code = 4 + (int)b.get(1);
      else code = 6 + (int)b.get(2);
      intra_mode = inv[code];
    }
    ref_idx0 = ref_idx1 = 0;
    dir = -1;
  }
  // coefficients: compact q x q tiles appended to the pool
  int16_t tile[256];
  uint32_t off[3] = {0, 0, 0};
  int mask = 0;
  if (mode != TE_SKIP) {
    const int cbp_table[8] = {1, 0, 5, 2, 6, 3, 7, 4};
    int code = get_vlc(b, 0);
    if (P->seq.tb_split_enable && (mode == TE_INTRA || mode == TE_INTER)) {
      tb_split = code == 2;
      if (code > 2) code -= 1;
    }
    const int sizeC = size / 2;
    if (!tb_split) {
      int tmp = 0;
      if (mode == TE_MERGE) {
        if (code == 7) code = 1;
        else if (code > 0) code = code + 1;
      }
      while (tmp < 8 && code != cbp_table[tmp]) tmp++;
      if (mode != TE_MERGE && ctx.cbp == 0 && tmp < 2) tmp = 1 - tmp;
      cbp_y = tmp & 1;
      cbp_u = (tmp >> 1) & 1;
      cbp_v = (tmp >> 2) & 1;
      const int cb[3] = {cbp_y, cbp_u, cbp_v};
      for (int c = 0; c < 3; c++) {
        if (!cb[c]) continue;
        const int n = c ? sizeC : size, q = n < 16 ? n : 16;
        if (read_coeff(b, tile, n, coeff_type | (c ? 1 : 0))) {
          mask |= 1 << c;
          off[c] = (uint32_t)P->coeffs.size();
          P->coeffs.insert(P->coeffs.end(), tile, tile + q * q);
        }
      }
    } else {
      // four transform blocks; every component's tiles are consecutive in the pool
      std::vector<int16_t> comp[3];
      int any[3] = {0, 0, 0};
      if (size > 8) {
        for (int index = 0; index < 4; index++) {
          int c2 = get_vlc(b, 0), tmp = 0;
          while (tmp < 8 && c2 != cbp_table[tmp]) tmp++;
          if (ctx.cbp == 0 && tmp < 2) tmp = 1 - tmp;
          const int cb[3] = {tmp & 1, (tmp >> 1) & 1, (tmp >> 2) & 1};
          for (int c = 0; c < 3; c++) {
            const int n = c ? sizeC / 2 : size / 2, q = n < 16 ? n : 16;
            if (cb[c]) any[c] |= read_coeff(b, tile, n, coeff_type | (c ? 1 : 0));
            else memset(tile, 0, sizeof(int16_t) * q * q);
            comp[c].insert(comp[c].end(), tile, tile + q * q);
          }
        }
      } else {
        for (int index = 0; index < 4; index++) {
          const int cy = (int)b.get(1);
          const int n = size / 2, q = n;
          if (cy) any[0] |= read_coeff(b, tile, n, coeff_type);
          else memset(tile, 0, sizeof(int16_t) * q * q);
          comp[0].insert(comp[0].end(), tile, tile + q * q);
        }
        int cu = 0, cv = 0;
        if (b.get(1)) {
          cu = cv = 0;
        } else if (b.get(1)) {
          cu = 1;
        } else if (b.get(1)) {
          cv = 1;
        } else {
          cu = cv = 1;
        }
        const int cb[3] = {0, cu, cv};
        for (int c = 1; c < 3; c++) {
          const int n = sizeC, q = n < 16 ? n : 16;
          if (cb[c]) any[c] |= read_coeff(b, tile, n, coeff_type | 1);
          else memset(tile, 0, sizeof(int16_t) * q * q);
          comp[c].insert(comp[c].end(), tile, tile + q * q);
        }
      }
      for (int c = 0; c < 3; c++)
        if (any[c]) {
          mask |= 1 << c;
          off[c] = (uint32_t)P->coeffs.size();
          P->coeffs.insert(P->coeffs.end(), comp[c].begin(), comp[c].end());
        }
      cbp_y = cbp_u = cbp_v = 1;  // deblocking only (read_bits.c:713-715, :779-781)
    }
  }
  B.intra_mode = (uint8_t)intra_mode;
  B.tb_split = (uint8_t)tb_split;
  B.pb_part = (uint8_t)pb_part;
  B.dir = (uint8_t)dir;
  B.cbp_y = (uint8_t)cbp_y;
  B.cbp_u = (uint8_t)cbp_u;
  B.cbp_v = (uint8_t)cbp_v;
  B.coeff_mask = (uint8_t)mask;
  for (int i = 0; i < 4; i++) {
    B.mv0[2 * i] = m0[i].x;
    B.mv0[2 * i + 1] = m0[i].y;
    B.mv1[2 * i] = m1[i].x;
    B.mv1[2 * i + 1] = m1[i].y;
  }
  B.ref0 = mode == TE_INTRA ? -1 : ref_frame_num(P, ref_idx0);
  B.ref1 = mode == TE_INTRA ? -1 : ref_frame_num(P, ref_idx1);
  for (int c = 0; c < 3; c++) B.coeff_off[c] = off[c];
  P->blocks.push_back(B);
  // copy_deblock_data (dec/decode_block.c:122-156), boundary cells only: later
  // CUs read a neighbour's cells only along its bottom row and right column
  // (te_mv_pred / te_mv_skip / te_block_ctx), so the interior is never read and
  // the per-frame memset of the reference (decode_frame.c:53) is not needed
  // either -- every cell read in a frame was written earlier in that frame.
  const int bs = W / 4, div = size / 8, bh4 = B.bheight / 4, bw4 = B.bwidth / 4;
  for (int e = 0; e < bh4 + bw4 - 1; e++) {
    const int m = e < bw4 ? bh4 - 1 : e - bw4, n = e < bw4 ? e : bw4 - 1;
    {
      const int m0i = div > 0 ? m / div : 0, n0i = div > 0 ? n / div : 0, index = 2 * m0i + n0i;
      TeCell &c = P->cells[(ypos / 4 + m) * bs + xpos / 4 + n];
      c.cbp_y = (uint8_t)cbp_y;
      c.cbp_u = (uint8_t)cbp_u;
      c.cbp_v = (uint8_t)cbp_v;
      c.tb_split = (uint8_t)tb_split;
      c.pb_part = (uint8_t)(mode == TE_INTER ? pb_part : 0);
      c.size = (uint8_t)size;
      c.mode = (uint8_t)mode;
      c.ip.mv0 = m0[index];
      c.ip.mv1 = m1[index];
      c.ip.ref_idx0 = ref_idx0;
      c.ip.ref_idx1 = ref_idx1;
      c.ip.bipred_flag = dir;
    }
  }
}

// process_block_dec, dec/decode_block.c:625-669
void process_block(thor_parser *P, int size, int ypos, int xpos) {
  const int W = P->seq.width, H = P->seq.height;
  if (ypos >= H || xpos >= W || P->error) return;
  const int decode_this = ypos + size <= H && xpos + size <= W;
  const int decode_rect = !decode_this && P->frame_type != TE_I;
  const TeCtx ctx = te_block_ctx(ypos, xpos, H, W, size, P->cells.data(), P->use_block_contexts);
  int mode = TE_SKIP, ref_idx = 0;
  const int split = super_mode(P, size, decode_this, ctx, &mode, &ref_idx);
  if (size == 64 && (split || mode != TE_SKIP) && P->max_delta_qp > 0) {
    // read_delta_qp, dec/read_bits.c:212-220
    const int a = get_vlc(P->b, 0);
    const int s = a > 0 ? (int)P->b.get(1) : 0;
    P->qpb = P->qp + (s ? -a : a);
    if (P->qpb < 0 || P->qpb > 51) P->error = 1;  // corrupt input: the tables are indexed by qp
  }
  if (split) {
    if (size <= 8) {
      P->error = 1;
      return;
    }
    const int ns = size / 2;
    process_block(P, ns, ypos, xpos);
    process_block(P, ns, ypos + ns, xpos);
    process_block(P, ns, ypos, xpos + ns);
    process_block(P, ns, ypos + ns, xpos + ns);
  } else if (decode_this || decode_rect) {
    read_block(P, size, ypos, xpos, mode, ref_idx, ctx);
  }
}

}  // namespace

extern "C" {

thor_parser_t *thor_parser_create(void) {
  thor_parser *P = new thor_parser();
  memset(&P->seq, 0, sizeof(P->seq));
  P->window.assign(33, -1);
  return P;
}
void thor_parser_destroy(thor_parser_t *P) { delete P; }

int thor_parser_seq(const thor_parser_t *P, thor_seq_t *seq) {
  if (!P || !seq || !P->have_seq) return THOR_ERR_ARG;
  *seq = P->seq;
  return THOR_OK;
}

int thor_parse_frame(thor_parser_t *P, const uint8_t *payload, size_t nbytes, thor_parsed_frame_t *out) {
  if (!P || !payload || !out) return THOR_ERR_ARG;
  TpBits &b = P->b;
  b.set(payload, nbytes);
  if (!P->have_seq) {  // sequence header, dec/maindec.c:124-147
    P->seq.width = (int)b.get(16);
    P->seq.height = (int)b.get(16);
    P->pb_split = (int)b.get(1);
    P->seq.tb_split_enable = (int)b.get(1);
    P->max_num_ref = (int)b.get(2) + 1;
    P->interp_ref = (int)b.get(1);
    P->seq.interp_ref = P->interp_ref;
    P->max_delta_qp = (int)b.get(3);
    P->seq.deblocking = (int)b.get(1);
    P->seq.clpf = (int)b.get(1);
    P->use_block_contexts = (int)b.get(1);
    P->seq.bipred = (int)b.get(1);
    // 16-bit sizes; this build also caps the area at 16384^2 pixels (a corrupt header must not size
    // GBs of side info) -- not each side: the encoder codes frames up to 65 535 px wide (te_check_params)
    if (P->seq.width <= 0 || P->seq.height <= 0 || (P->seq.width & 7) || (P->seq.height & 7) ||
        (long long)P->seq.width * P->seq.height > 16384LL * 16384)
      return THOR_ERR_ARG;
    P->have_seq = 1;
    P->cells.assign((size_t)(P->seq.width / 4) * (P->seq.height / 4), TeCell());
  }
  const int W = P->seq.width, H = P->seq.height;
  // frame header, dec/decode_frame.c:58-78
  P->frame_type = (int)b.get(1);
  P->qp = (int)b.get(8);
  P->num_intra_modes = (int)b.get(4);
  P->fr_interp = 0;
  if (P->frame_type != TE_I) {
    P->num_ref = (int)b.get(2) + 1;
    for (int r = 0; r < P->num_ref; r++) {
      P->ref_array[r] = (int)b.get(6) - 1;
      if (P->ref_array[r] == -1) P->fr_interp = 1;
    }
    if (P->num_ref == 2 && P->ref_array[0] == -1) P->ref_array[P->num_ref++] = (int)b.get(5) - 1;
  } else {
    P->num_ref = 0;
  }
  P->frame_num = (int)b.get(16);
  if (P->qp > 51) return THOR_ERR_ARG;  // corrupt header: qp indexes the dequantisation / loop-filter tables
  for (int r = 0; r < P->num_ref; r++) {
    if (P->ref_array[r] == -1) continue;  // the interpolated reference
    if (P->ref_array[r] < 0 || P->ref_array[r] > 32 || P->window[P->ref_array[r]] < 0) return THOR_ERR_REF;
  }
  // the interpolated reference is built only for num_ref > 2 with ref_array[0] == -1
  // (decode_frame.c:91-109); any other use of index -1 would read a stale frame
  int interp_a = -1, interp_b = -1, interp_ratio = 0, interp_pos = 0;
  if (P->fr_interp) {
    if (!(P->num_ref > 2 && P->ref_array[0] == -1) || P->ref_array[1] < 0 || P->ref_array[2] < 0) return THOR_ERR_REF;
    for (int r = 1; r < P->num_ref; r++)
      if (P->ref_array[r] == -1) return THOR_ERR_REF;
    interp_a = P->window[P->ref_array[1]];
    interp_b = P->window[P->ref_array[2]];
    int off1 = interp_b - P->frame_num, off2 = P->frame_num - interp_a;
    if (off1 < 0 && off2 < 0) {
      off1 = -off1;
      off2 = -off2;
    }
    if (off1 == off2) off1 = off2 = 1;
    interp_ratio = off1 + off2;
    interp_pos = off2;
    if (interp_ratio <= 0) return THOR_ERR_REF;  // the one-sided case the reference leaves unhandled (:105)
  }
  P->qpb = P->qp;
  P->blocks.clear();
  P->coeffs.clear();
  P->error = 0;
  const int nsbh = (W + 63) / 64, nsbv = (H + 63) / 64;
  for (int k = 0; k < nsbv; k++)
    for (int l = 0; l < nsbh; l++) process_block(P, 64, k * 64, l * 64);
  if (P->error) return THOR_ERR_ARG;
  // CLPF signalling (decode_frame.c:130-133, clpf_frame common/common_frame.c:485-513)
  const int nh = W / 64, nv = H / 64;
  P->clpf.assign((size_t)nh * nv, 0);
  P->clpf_on = 0;
  if (P->seq.clpf && b.get(1)) {
    P->clpf_on = 1;
    const int all = (int)b.get(1);
    // an SB is a candidate when a cell on its 8x8 grid belongs to a non-BIPRED CU
    // with coded residual; every CU of a full SB covers a grid cell, so this is
    // the OR over the SB's CUs
    std::vector<uint8_t> &cand = P->clpf_cand;
    cand.assign((size_t)nh * nv, 0);
    for (const thor_block_t &B : P->blocks) {
      const int k = B.ypos / 64, l = B.xpos / 64;
      if (k < nv && l < nh && B.mode != TE_BIPRED && (B.cbp_y || B.cbp_u || B.cbp_v)) cand[k * nh + l] = 1;
    }
    for (int k = 0; k < nv; k++)
      for (int l = 0; l < nh; l++)
        if (cand[k * nh + l]) P->clpf[k * nh + l] = all ? 1 : (uint8_t)b.get(1);
  }
  if (b.pos > b.nbits || b.err) return THOR_ERR_ARG;  // read past the payload / malformed: truncated or corrupt
  // slide the window (decode_frame.c:135-147)
  for (int r = 32; r > 0; r--) P->window[r] = P->window[r - 1];
  P->window[0] = P->frame_num;
  memset(out, 0, sizeof(*out));
  out->seq = P->seq;
  out->hdr.frame_num = P->frame_num;
  out->hdr.frame_type = P->frame_type;
  out->hdr.qp = P->qp;
  out->hdr.clpf_on = P->clpf_on;
  out->hdr.interp_ref[0] = interp_a;
  out->hdr.interp_ref[1] = interp_b;
  out->hdr.interp_ratio = interp_ratio;
  out->hdr.interp_pos = interp_pos;
  out->num_ref = P->num_ref;
  out->decode_order = P->decode_order++;
  out->blocks = P->blocks.data();
  out->nblocks = (int32_t)P->blocks.size();
  out->coeffs = P->coeffs.data();
  out->ncoeffs = (int32_t)P->coeffs.size();
  out->clpf_flags = P->clpf.data();
  out->nclpf = (int32_t)P->clpf.size();
  return THOR_OK;
}

int thor_frame_image(const thor_parsed_frame_t *pf, uint8_t *img, size_t cap, thor_frame_image_t *lay) {
  if (!pf || !lay || pf->nblocks < 0 || pf->ncoeffs < 0 || pf->nclpf < 0 || (pf->nblocks > 0 && !pf->blocks) ||
      (pf->ncoeffs > 0 && !pf->coeffs) || (pf->nclpf > 0 && !pf->clpf_flags))
    return THOR_ERR_ARG;
  const thor_block_t *bl = pf->blocks;
  const int nb = pf->nblocks, W = pf->seq.width, H = pf->seq.height;
  const int nflags = pf->hdr.clpf_on ? pf->nclpf : 0;
  memset(lay, 0, sizeof(*lay));
  lay->nblocks = nb;
  lay->ncoeffs = pf->ncoeffs;
  lay->n_flags = nflags;
  lay->n_intra = thor_build_intra_list(bl, nb, nullptr);
  lay->n_tu = thor_build_tu_list(bl, nb, nullptr);
  lay->n_clpf = nflags ? thor_build_clpf_list(pf->clpf_flags, nflags, nullptr) : -1;
  lay->n_slow = thor_build_slow_list(bl, nb, W, H, nullptr);
  if (lay->n_intra < 0 || lay->n_tu < 0 || lay->n_slow < 0) return THOR_ERR_ARG;
  uint64_t o = 0;
  auto part = [&](uint64_t &off, uint64_t n) {
    off = o;
    o += (n + 255) & ~(uint64_t)255;
  };
  part(lay->off_blocks, (uint64_t)nb * sizeof(thor_block_t));
  part(lay->off_coeffs, (uint64_t)pf->ncoeffs * sizeof(int16_t));
  part(lay->off_flags, (uint64_t)nflags);
  part(lay->off_intra, (uint64_t)lay->n_intra * 4);
  part(lay->off_tus, (uint64_t)lay->n_tu * sizeof(thor_tu_t));
  part(lay->off_clpf, (uint64_t)(lay->n_clpf > 0 ? lay->n_clpf : 0) * 4);
  part(lay->off_slow, (uint64_t)lay->n_slow * 4);
  lay->bytes = o > 256 ? o : 256;
  if (!img || cap < lay->bytes) return THOR_ERR_NOMEM;
  if (nb) memcpy(img + lay->off_blocks, bl, (size_t)nb * sizeof(thor_block_t));
  if (pf->ncoeffs) memcpy(img + lay->off_coeffs, pf->coeffs, (size_t)pf->ncoeffs * sizeof(int16_t));
  if (nflags) memcpy(img + lay->off_flags, pf->clpf_flags, (size_t)nflags);
  thor_build_intra_list(bl, nb, (uint32_t *)(img + lay->off_intra));
  thor_build_tu_list(bl, nb, (thor_tu_t *)(img + lay->off_tus));
  if (nflags) thor_build_clpf_list(pf->clpf_flags, nflags, (uint32_t *)(img + lay->off_clpf));
  thor_build_slow_list(bl, nb, W, H, (uint32_t *)(img + lay->off_slow));
  return THOR_OK;
}

}  // extern "C"
