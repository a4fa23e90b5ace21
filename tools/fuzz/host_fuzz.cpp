// TEST HARNESS ONLY: the encoder's host control (thor_amd/csrc/enc_gop.h:
// te_set_param, te_check_params, the GOP planner TeGop, the header writers,
// the early-skip thresholds) and the decoder's host work lists
// (thor_amd/csrc/host_lists.h) built for the CPU with AddressSanitizer +
// UndefinedBehaviorSanitizer and driven by a seeded parameter / block fuzz.
//
//   host_fuzz ITER SEED
//
// Parameters: each iteration starts from the defaults and sets 1..8 fields to
// values drawn around their legal ranges (and well outside them).  Every set
// the checker accepts is planned for a bounded number of frames and every plan
// must satisfy what the device encoder relies on: QP in 0..51, at most 4
// references, reference indices inside the 33-frame window (or -1 = the
// interpolated reference), reference frame numbers already coded, interpolated
// sources inside the window, frame numbers covering the input exactly once.
// Lists: random block arrays (legal and corrupt descriptors) go through the
// count-then-fill calling convention into buffers of exactly the counted size.
#include <stdio.h>
#include <stdlib.h>

#include <set>
#include <vector>

#include "../../thor_amd/csrc/enc_gop.h"
#include "../../thor_amd/csrc/host_lists.h"

static uint64_t rng = 1;
static uint32_t rnd() {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return (uint32_t)rng;
}
static int pick(const int *v, int n) { return v[rnd() % n]; }

static int fails = 0;
#define CHECK(c, ...)                                 \
  do {                                                \
    if (!(c)) {                                       \
      if (fails++ < 20) {                             \
        fprintf(stderr, "host_fuzz: %s: ", #c);       \
        fprintf(stderr, __VA_ARGS__);                 \
        fprintf(stderr, "\n");                        \
      }                                               \
    }                                                 \
  } while (0)

static int fuzz_params(int it) {
  thor_enc_params_t p;
  te_default_params(&p);
  p.num_frames = 1 + (int)(rnd() % 40);
  static const char *keys[] = {"-width", "-height", "-qp", "-skip", "-max_num_ref", "-HQperiod", "-num_reorder_pics",
                               "-dyadic_coding", "-interp_ref", "-intra_period", "-max_delta_qp", "-delta_qp_step",
                               "-dqpI", "-dqpP", "-dqpB", "-mqpP", "-mqpB0", "-n", "-f", "-encoder_speed",
                               "-intra_rdo", "-rdoq", "-sync", "-enable_bipred", "-lambda_coeffB2", "-bogus"};
  static const int vals[] = {-7, -1, 0, 1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 31, 32, 33, 51, 52, 64, 100, 1080, 1920,
                             65535, 65536, 100000};
  const int nset = 1 + (int)(rnd() % 8);
  for (int s = 0; s < nset; s++) {
    const char *k = keys[rnd() % (sizeof(keys) / sizeof(keys[0]))];
    char v[32];
    snprintf(v, sizeof(v), "%d", pick(vals, sizeof(vals) / sizeof(vals[0])));
    const int rc = te_set_param(&p, k, v);
    CHECK(rc == 0 || !strcmp(k, "-bogus"), "te_set_param(%s) = %d", k, rc);
  }
  if (rnd() % 3 == 0) {  // legal GOP shapes more often than chance gives them
    static const int nr[] = {0, 1, 3, 7, 15};
    p.num_reorder_pics = pick(nr, 5);
    p.HQperiod = p.num_reorder_pics ? p.num_reorder_pics + 1 : 1 + (int)(rnd() % 8);
    p.max_num_ref = 2 + (int)(rnd() % 3);
    p.intra_period = (int)(rnd() % 3) * (p.num_reorder_pics + 1) * 2;
    p.interp_ref = (int)(rnd() % 2);
    p.skip = (int)(rnd() % 3);
  }
  if (p.num_frames > 64) p.num_frames = 64;  // bound the planning work, not the checker's input
  if (te_check_params(&p) != THOR_OK) return 0;
  // what the checker let through must plan cleanly
  TeGop g(p);
  const int nplans = (int)g.plans.size();
  CHECK(nplans == p.num_frames, "it %d: %d plans for %d frames", it, nplans, p.num_frames);
  std::set<int> coded;
  for (const TeFramePlan &f : g.plans) {
    CHECK(f.qp >= 0 && f.qp <= 51, "it %d: qp %d", it, f.qp);
    CHECK(f.num_ref >= 0 && f.num_ref <= 4, "it %d: num_ref %d", it, f.num_ref);
    CHECK(f.frame_num >= 0 && f.frame_num < p.num_frames && !coded.count(f.frame_num), "it %d: frame_num %d", it,
          f.frame_num);
    CHECK((f.frame_type == 0) == (f.num_ref == 0) || f.frame_type != 0, "it %d: I frame with references", it);
    for (int r = 0; r < f.num_ref; r++) {
      CHECK(f.ref_array[r] >= -1 && f.ref_array[r] < 33, "it %d: ref_array[%d] = %d", it, r, f.ref_array[r]);
      CHECK(f.ref_array[r] >= 0 || (f.interp_ref && r == 0), "it %d: ref -1 without interp_ref", it);
      if (f.ref_array[r] >= 0)
        CHECK(coded.count(f.ref_fnum[r]), "it %d: frame %d refers to %d, not coded yet", it, f.frame_num, f.ref_fnum[r]);
    }
    if (f.interp_ref) {
      CHECK(f.interp_a >= 0 && f.interp_a < 33 && f.interp_b >= 0 && f.interp_b < 33, "it %d: interp sources %d %d",
            it, f.interp_a, f.interp_b);
      CHECK(f.interp_ratio > 0, "it %d: interp_ratio %d", it, f.interp_ratio);
    }
    TeHostBits b;
    te_frame_header(b, f);
    CHECK(b.nbits > 0, "it %d: empty frame header", it);
    coded.insert(f.frame_num);
  }
  TeHostBits sh;
  te_seq_header(sh, g.p);
  CHECK(sh.nbits == 44, "it %d: sequence header %llu bits", it, (unsigned long long)sh.nbits);
  std::vector<int> thr(2 * 52 * 4);
  te_es_thresholds(p.early_skip_thr, thr.data());
  return 1;
}

static void fuzz_lists(int it) {
  const int nb = (int)(rnd() % 300);
  std::vector<thor_block_t> blk(nb);
  const bool corrupt = rnd() % 4 == 0;
  for (thor_block_t &B : blk) {
    memset(&B, 0, sizeof(B));
    static const int sz[] = {8, 16, 32, 64};
    B.size = (uint8_t)(corrupt ? rnd() : pick(sz, 4));
    B.xpos = (uint16_t)(corrupt ? rnd() : 8 * (rnd() % 480));
    B.ypos = (uint16_t)(corrupt ? rnd() : 8 * (rnd() % 270));
    B.mode = (uint8_t)(corrupt ? rnd() : rnd() % 5);
    B.tb_split = (uint8_t)(corrupt ? rnd() : rnd() % 2);
    B.coeff_mask = (uint8_t)(corrupt ? rnd() : rnd() % 8);
    B.qp = (uint8_t)(corrupt ? rnd() : rnd() % 52);
    for (int c = 0; c < 3; c++) B.coeff_off[c] = rnd();
  }
  const thor_block_t *bp = nb ? blk.data() : nullptr;
  const int ntu = thor_build_tu_list(bp, nb, nullptr);
  CHECK(ntu >= 0 && ntu <= 12 * nb, "it %d: %d TUs from %d blocks", it, ntu, nb);
  std::vector<thor_tu_t> tus(ntu > 0 ? ntu : 0);
  CHECK(thor_build_tu_list(bp, nb, tus.data()) == ntu, "it %d: TU count changed between passes", it);
  for (const thor_tu_t &T : tus) CHECK(T.comp < 3 && T.qp <= 51, "it %d: TU comp %d qp %d", it, T.comp, T.qp);
  const int ni = thor_build_intra_list(bp, nb, nullptr);
  std::vector<uint32_t> il(ni > 0 ? ni : 0);
  CHECK(thor_build_intra_list(bp, nb, il.data()) == ni, "it %d: intra count changed", it);
  for (uint32_t i : il) CHECK(i < (uint32_t)nb && blk[i].mode == 1, "it %d: intra list entry %u", it, i);
  std::vector<uint8_t> fl(nb);
  for (uint8_t &x : fl) x = (uint8_t)(rnd() % 2 ? rnd() : 0);
  const int nc = thor_build_clpf_list(nb ? fl.data() : nullptr, nb, nullptr);
  std::vector<uint32_t> cl(nc > 0 ? nc : 0);
  CHECK(thor_build_clpf_list(nb ? fl.data() : nullptr, nb, cl.data()) == nc, "it %d: CLPF count changed", it);
  for (size_t j = 1; j < cl.size(); j++) CHECK(cl[j] > cl[j - 1], "it %d: CLPF list not increasing", it);
  for (thor_block_t &B : blk)
    for (int k = 0; k < 8; k++) {
      B.mv0[k] = (int16_t)(rnd() % 3 ? 0 : rnd());
      B.mv1[k] = (int16_t)(rnd() % 3 ? 0 : rnd());
    }
  const int nu = 4 * 34 * 30;  // units of a 4K frame (unit_count, common.h)
  const int ns = thor_build_slow_list(bp, nb, 3840, 2160, nullptr);
  CHECK(ns >= 0 && ns <= nu, "it %d: %d slow units", it, ns);
  std::vector<uint32_t> sl(ns > 0 ? ns : 0);
  CHECK(thor_build_slow_list(bp, nb, 3840, 2160, sl.data()) == ns, "it %d: slow count changed", it);
  for (size_t j = 0; j < sl.size(); j++)
    CHECK(sl[j] < (uint32_t)nu && (j == 0 || sl[j] > sl[j - 1]), "it %d: slow list entry %u", it, sl[j]);
  // the argument errors
  CHECK(thor_build_slow_list(nullptr, 3, 64, 64, nullptr) == THOR_ERR_ARG, "slow list null");
  CHECK(thor_build_slow_list(bp, nb, 0, 64, nullptr) == THOR_ERR_ARG, "slow list width");
  CHECK(thor_build_tu_list(nullptr, 3, nullptr) == THOR_ERR_ARG, "tu list null");
  CHECK(thor_build_intra_list(bp, -1, nullptr) == THOR_ERR_ARG, "intra list negative");
  CHECK(thor_build_clpf_list(nullptr, 5, nullptr) == THOR_ERR_ARG, "clpf list null");
}

int main(int argc, char **argv) {
  if (argc < 3) return 2;
  const int iters = atoi(argv[1]);
  rng = 0x9E3779B97F4A7C15ull ^ (uint64_t)atoll(argv[2]);
  int accepted = 0;
  for (int it = 0; it < iters; it++) {
    accepted += fuzz_params(it);
    fuzz_lists(it);
  }
  // the shipped configurations must pass the checker (configs.py mirrors them)
  {
    thor_enc_params_t p;
    te_default_params(&p);
    p.num_reorder_pics = 15;
    p.HQperiod = 16;
    p.max_num_ref = 4;
    p.intra_period = 0;
    p.interp_ref = 1;
    CHECK(te_check_params(&p) == THOR_OK, "HDB16-shaped parameters rejected");
  }
  printf("host_fuzz: %d iterations, %d parameter sets accepted and planned, %d failures\n", iters, accepted, fails);
  return fails ? 5 : 0;
}
