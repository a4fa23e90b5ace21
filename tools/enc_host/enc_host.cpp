// TEST / DEBUG HARNESS ONLY -- never part of libthor_amd.so.
//
// Runs the device encoder's RD source (thor_amd/csrc/enc_*.h) as plain host
// C++ (TE_HOST: one "lane", serial loops) over a .yuv file, so the RD logic can
// be checked bit for bit against the reference encoder's .bit on a CPU-only
// box.  Frame loop filters come from the CPU oracle (oracle/thor_oracle.c).
//
//   enc_host -if in.yuv -of out.bit [-rf rec.yuv] [-rdlog costs.bin] -width W -height H -n N [-qp ..] ...
//
// -rdlog: every superblock's top-level process_block costs (te_encode_sb's
// cost record: delta-QP trials, then the final encode) as int32 records
// (frame_num, 64, ypos, xpos, qp or -1 for the final encode, cost) -- the
// layout of tests/golden/rd_costs.npz, whose reference records carry the
// final encode's QP instead of -1.
#define TE_HOST 1
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "../../oracle/thor_oracle.h"
#include "../../thor_amd/csrc/enc_gop.h"
#include "../../thor_amd/csrc/enc_rd.h"

struct HostFrame {
  std::vector<uint8_t> buf;
  or_frame_t f;
  HostFrame(int W, int H) {
    const int sy = (W + 192 + 15) & ~15, sc = (W / 2 + 96 + 15) & ~15;
    const size_t ys = (size_t)(H + 192) * sy, cs = (size_t)(H / 2 + 96) * sc;
    buf.assign(ys + 2 * cs + 64, 0);
    f.stride_y = sy;
    f.stride_c = sc;
    f.y = buf.data() + 96 * sy + 96;
    f.u = buf.data() + ys + 48 * sc + 48;
    f.v = buf.data() + ys + cs + 48 * sc + 48;
    f.frame_num = -1;
  }
};

int main(int argc, char **argv) {
  thor_enc_params_t P;
  te_default_params(&P);
  const char *in = nullptr, *out = nullptr, *recf = nullptr, *rdlog = nullptr;
  const char *trace_out = nullptr;
  (void)trace_out;
  int verbose = 0;
  for (int i = 1; i + 1 < argc; i += 2) {
    if (!strcmp(argv[i], "-if")) in = argv[i + 1];
    else if (!strcmp(argv[i], "-of")) out = argv[i + 1];
    else if (!strcmp(argv[i], "-rf")) recf = argv[i + 1];
    else if (!strcmp(argv[i], "-rdlog")) rdlog = argv[i + 1];
    else if (!strcmp(argv[i], "-v")) verbose = atoi(argv[i + 1]);
#if defined(THOR_ENC_TRACE)
    else if (!strcmp(argv[i], "-trace_frame")) te_trace_frame = atoi(argv[i + 1]);
    else if (!strcmp(argv[i], "-trace_out")) trace_out = argv[i + 1];
#endif
    else if (te_set_param(&P, argv[i], argv[i + 1])) {
      fprintf(stderr, "unknown parameter %s\n", argv[i]);
      return 2;
    }
  }
  if (!in || !out || te_check_params(&P)) {
    fprintf(stderr, "usage / unsupported parameters\n");
    return 2;
  }
  const int W = P.width, H = P.height;
#if defined(THOR_ENC_TRACE)
  if (trace_out) {
    te_trace_cap = 1u << 24;
    te_trace_buf = (int *)calloc(8 + 8 * (size_t)te_trace_cap, sizeof(int));
  }
#endif
  FILE *fi = fopen(in, "rb"), *fo = fopen(out, "wb"), *fr = recf ? fopen(recf, "wb") : nullptr;
  FILE *frd = rdlog ? fopen(rdlog, "wb") : nullptr;
  if (!fi || !fo || (rdlog && !frd)) return 3;
  const int ntrial = P.max_delta_qp ? (2 * P.max_delta_qp) / (P.delta_qp_step > 0 ? P.delta_qp_step : 1) + 1 : 0;
  std::vector<int32_t> costs(ntrial + 1);
  const size_t fsz = (size_t)W * H * 3 / 2;
  std::vector<uint8_t> orig(fsz);
  TeGop gop(P);
  std::vector<HostFrame *> window(33, nullptr);
  for (auto &w : window) w = new HostFrame(W, H);
  HostFrame cur(W, H), interp(W, H);
  std::vector<TeCell> cells((size_t)(W / 4) * (H / 4));
  std::vector<or_cell_t> ocells(cells.size());
  TeScratchMem *SM = (TeScratchMem *)calloc(1, sizeof(TeScratchMem));
  te_set_scratch(te_scratch(*SM, &SM->tx, &SM->nb, SM->pb, SM->bi, &SM->tmp, &SM->sl));
  te_load_basis(SM->tx);
  TeSB sb;
  std::vector<uint32_t> sbw(1 << 17);
  sb.bits.w = sbw.data();
  sb.bits.cap = (int)sbw.size() * 32;
  std::vector<int> es(2 * 52 * 4);
  te_es_thresholds(P.early_skip_thr, es.data());
  const int nsbh = (W + 63) / 64, nsbv = (H + 63) / 64;
  bool first = true;
  for (const TeFramePlan &pl : gop.plans) {
    fseek(fi, (long)(pl.input_index * fsz), SEEK_SET);
    if (fread(orig.data(), 1, fsz, fi) != fsz) return 4;
    TeFrame F;
    memset(&F, 0, sizeof(F));
    F.oy = orig.data();
    F.ou = orig.data() + W * H;
    F.ov = F.ou + W * H / 4;
    F.osy = W;
    F.osc = W / 2;
    F.ry = cur.f.y;
    F.ru = cur.f.u;
    F.rv = cur.f.v;
    F.rsy = cur.f.stride_y;
    F.rsc = cur.f.stride_c;
    if (pl.interp_ref) {  // the interpolated reference (enc/mainenc.c:324-330, :381-387)
      or_interpolate_frames(&window[pl.interp_a]->f, &window[pl.interp_b]->f, 96, &interp.f, W, H, pl.interp_ratio,
                            pl.interp_pos, nullptr, nullptr);
      or_pad_frame(&interp.f, W, H, 96, 48);
      interp.f.frame_num = pl.frame_num;
    }
    for (int r = 0; r < pl.num_ref; r++) {
      const HostFrame *rf = pl.ref_array[r] < 0 ? &interp : window[pl.ref_array[r]];
      F.refy[r] = rf->f.y;
      F.refu[r] = rf->f.u;
      F.refv[r] = rf->f.v;
      F.ref_fnum[r] = rf->f.frame_num;
    }
    memset(cells.data(), 0, cells.size() * sizeof(TeCell));
    F.cells = cells.data();
    F.W = W;
    F.H = H;
    F.frame_num = pl.frame_num;
    F.frame_type = pl.frame_type;
    F.qp = pl.qp;
    F.num_ref = pl.num_ref;
    F.num_intra_modes = pl.num_intra_modes;
    F.interp_ref = pl.interp_ref;
    F.lambda = pl.lambda;
    F.sqrt_lambda = sqrt(pl.lambda);
    F.speed = P.encoder_speed;
    F.enable_tb_split = P.enable_tb_split;
    F.enable_pb_split = P.enable_pb_split;
    F.enable_bipred = P.enable_bipred;
    F.max_delta_qp = P.max_delta_qp;
    F.delta_qp_step = P.delta_qp_step;
    F.intra_rdo = P.intra_rdo;
    F.use_block_contexts = P.use_block_contexts;
    F.rdoq = P.rdoq;
    F.sync = P.sync;
    F.early_skip_thr = P.early_skip_thr;
    F.es_thr = es.data();
    TeHostBits fb;
    if (first) te_seq_header(fb, P);
    first = false;
    te_frame_header(fb, pl);
    for (int k = 0; k < nsbv; k++)
      for (int l = 0; l < nsbh; l++) {
        te_encode_sb(F, sb, k, l, frd ? costs.data() : nullptr);
        fb.append_words(sb.bits.w, sb.bits.pos);
        for (int t = 0; frd && t <= ntrial; t++) {
          const int32_t r[6] = {pl.frame_num, 64, 64 * k, 64 * l,
                                t < ntrial ? pl.qp - P.max_delta_qp + t * P.delta_qp_step : -1, costs[t]};
          fwrite(r, sizeof(r), 1, frd);
        }
        if (verbose > 1) fprintf(stderr, "frame %d sb %d,%d bits %d\n", pl.frame_num, k, l, sb.bits.pos);
      }
    for (size_t i = 0; i < cells.size(); i++) {
      const TeCell &c = cells[i];
      or_cell_t &o = ocells[i];
      o.mode = c.mode;
      o.cbp_y = c.cbp_y;
      o.cbp_u = c.cbp_u;
      o.cbp_v = c.cbp_v;
      o.size = c.size;
      o.tb_split = c.tb_split;
      o.pb_part = c.pb_part;
      o.mv0x = c.ip.mv0.x;
      o.mv0y = c.ip.mv0.y;
      o.mv1x = c.ip.mv1.x;
      o.mv1y = c.ip.mv1.y;
    }
    if (P.deblocking) or_deblock_cells(&cur.f, ocells.data(), W, H, pl.qp);
    if (P.clpf) {
      fb.put(1, 1);
      fb.put(1, 0);  // sb_signal = 1 (enc/encode_frame.c:156-160)
      std::vector<uint8_t> flags((size_t)(W / 64) * (H / 64) + 1, 0);
      for (int k = 0; k < H / 64; k++)
        for (int l = 0; l < W / 64; l++) {
          const int d = te_clpf_decide(F, k, l);
          if (d >= 0) {
            fb.put(1, d);
            flags[k * (W / 64) + l] = (uint8_t)d;
          }
        }
      or_clpf_cells(&cur.f, ocells.data(), W, H, flags.data());
    }
    // frame chunk: 4-byte big-endian length + bytes (flush_all_bits, enc/putbits.c:57-95)
    const uint32_t nb = (uint32_t)fb.bytes.size();
    const uint8_t hdr[4] = {(uint8_t)(nb >> 24), (uint8_t)(nb >> 16), (uint8_t)(nb >> 8), (uint8_t)nb};
    fwrite(hdr, 1, 4, fo);
    fwrite(fb.bytes.data(), 1, nb, fo);
    if (verbose) fprintf(stderr, "frame %d type %d qp %d bytes %u\n", pl.frame_num, pl.frame_type, pl.qp, nb);
    if (fr) {  // coding order == display order for the low-delay configurations this harness checks
      for (int i = 0; i < H; i++) fwrite(cur.f.y + i * cur.f.stride_y, 1, W, fr);
      for (int i = 0; i < H / 2; i++) fwrite(cur.f.u + i * cur.f.stride_c, 1, W / 2, fr);
      for (int i = 0; i < H / 2; i++) fwrite(cur.f.v + i * cur.f.stride_c, 1, W / 2, fr);
    }
    // slide the reference window: the frame shifted out takes the new picture
    HostFrame *tmp = window[32];
    for (int r = 32; r > 0; r--) window[r] = window[r - 1];
    window[0] = tmp;
    memcpy(tmp->buf.data(), cur.buf.data(), cur.buf.size());
    tmp->f.frame_num = pl.frame_num;
    or_pad_frame(&tmp->f, W, H, 96, 48);
  }
#if defined(THOR_ENC_TRACE)
  if (trace_out && te_trace_buf) {
    FILE *ft = fopen(trace_out, "wb");
    const unsigned n = (unsigned)te_trace_buf[0] < te_trace_cap ? (unsigned)te_trace_buf[0] : te_trace_cap;
    fwrite(te_trace_buf + 8, 32, n, ft);
    fclose(ft);
  }
#endif
  fclose(fi);
  fclose(fo);
  if (fr) fclose(fr);
  if (frd) fclose(frd);
  free(SM);
  return 0;
}
