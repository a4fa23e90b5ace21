// TEST HARNESS ONLY: the host .bit parser (thor_amd/csrc/parse.hip) built for
// the CPU with AddressSanitizer + UndefinedBehaviorSanitizer, fed every golden
// .bit intact and then seeded corruptions of it: truncated frame payloads, bit
// flips, overwritten byte runs, dropped / repeated / reordered frames and a
// corrupt sequence header.  Every call must return THOR_OK or a THOR_ERR_*
// code; the sanitizers abort the run on any out-of-bounds access, use of
// uninitialised memory they can see, or undefined behaviour.
//
//   parse_fuzz ITER SEED file.bit [file.bit ...]
#include <stdio.h>
#include <stdlib.h>

#include <string>
#include <vector>

#include "../../thor_amd/csrc/host_lists.h"
#include "../../thor_amd/csrc/parse.hip"

typedef std::vector<uint8_t> Bytes;

static std::vector<Bytes> chunks(const Bytes &f) {  // 4-byte big-endian length + payload (dec/getbits.c:48-69)
  std::vector<Bytes> out;
  size_t o = 0;
  while (o + 4 <= f.size()) {
    const size_t n = (size_t)f[o] << 24 | (size_t)f[o + 1] << 16 | (size_t)f[o + 2] << 8 | f[o + 3];
    if (o + 4 + n > f.size()) break;
    out.emplace_back(f.begin() + o + 4, f.begin() + o + 4 + n);
    o += 4 + n;
  }
  return out;
}

static uint64_t rng = 1;
static uint32_t rnd() {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return (uint32_t)rng;
}

static int parse_all(const std::vector<Bytes> &fr, int *bad) {
  thor_parser_t *p = thor_parser_create();
  int ok = 0;
  for (const Bytes &c : fr) {
    thor_parsed_frame_t out;
    const uint8_t dummy = 0;
    const int rc = thor_parse_frame(p, c.empty() ? &dummy : c.data(), c.size(), &out);
    if (rc == THOR_OK) {
      ok++;
      // touch what the decoder would read
      volatile long long s = 0;
      for (int i = 0; i < out.nblocks; i++) s += out.blocks[i].coeff_off[0] + out.blocks[i].size + out.blocks[i].qp;
      for (int i = 0; i < out.ncoeffs; i++) s += out.coeffs[i];
      for (int i = 0; i < out.nclpf; i++) s += out.clpf_flags[i];
      // the decoder's upload image (thor_frame_image): sized, then written
      thor_frame_image_t lay;
      if (thor_frame_image(&out, nullptr, 0, &lay) != THOR_ERR_NOMEM) (*bad)++;
      std::vector<uint8_t> img(lay.bytes);
      if (thor_frame_image(&out, img.data(), img.size(), &lay) != THOR_OK) (*bad)++;
    } else if (rc > 0 || rc < -16) {
      (*bad)++;
    }
  }
  thor_parser_destroy(p);
  return ok;
}

int main(int argc, char **argv) {
  if (argc < 4) return 2;
  const int iters = atoi(argv[1]);
  rng = 0x9E3779B97F4A7C15ull ^ (uint64_t)atoll(argv[2]);
  long long calls = 0, oks = 0;
  int bad = 0;
  for (int a = 3; a < argc; a++) {
    FILE *f = fopen(argv[a], "rb");
    if (!f) return 3;
    Bytes data;
    int ch;
    while ((ch = fgetc(f)) != EOF) data.push_back((uint8_t)ch);
    fclose(f);
    const std::vector<Bytes> fr = chunks(data);
    if ((size_t)parse_all(fr, &bad) != fr.size()) {
      fprintf(stderr, "%s: intact stream did not parse\n", argv[a]);
      return 4;
    }
    for (int it = 0; it < iters; it++) {
      std::vector<Bytes> m = fr;
      const int kind = (int)(rnd() % 7);
      const size_t k = rnd() % m.size();
      Bytes &c = m[k];
      switch (kind) {
        case 0:  // truncate one frame
          c.resize(c.empty() ? 0 : rnd() % c.size());
          break;
        case 1: {  // flip 1..16 bits of one frame
          const int n = 1 + (int)(rnd() % 16);
          for (int j = 0; j < n && !c.empty(); j++) c[rnd() % c.size()] ^= (uint8_t)(1u << (rnd() % 8));
          break;
        }
        case 2: {  // overwrite a run of bytes with noise
          if (c.empty()) break;
          const size_t o = rnd() % c.size(), n = 1 + rnd() % 64;
          for (size_t j = o; j < o + n && j < c.size(); j++) c[j] = (uint8_t)rnd();
          break;
        }
        case 3:  // drop a frame
          m.erase(m.begin() + k);
          break;
        case 4:  // repeat a frame
          m.insert(m.begin() + k, m[k]);
          break;
        case 5:  // swap two frames
          std::swap(m[k], m[rnd() % m.size()]);
          break;
        case 6: {  // corrupt the sequence header (first 4 bytes: width / height) and the frame header after it
          Bytes &h = m[0];
          for (int j = 0; j < 8 && j < (int)h.size(); j++)
            if (rnd() % 3 == 0) h[j] = (uint8_t)rnd();
          break;
        }
      }
      if (m.empty()) continue;
      oks += parse_all(m, &bad);
      calls += (long long)m.size();
    }
  }
  printf("parse_fuzz: %lld parse calls, %lld ok, %d unexpected return codes\n", calls, oks, bad);
  return bad ? 5 : 0;
}
