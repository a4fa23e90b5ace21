// Device-resident Thor encoder, part 1: portability layer, tables, the bit
// writer, VLC tables, block syntax (write_block) and the neighbour logic (MV
// predictor, skip / merge candidates, block contexts, availability).
//
// SPMD single source.  The encoder runs as ONE wavefront per superblock row
// (WPP, enc.hip): control flow is wave-uniform, pixel work is spread over the
// 64 lanes with `for (e = TE_LANE; e < n; e += TE_NL)` loops and wave
// reductions.  The same source also compiles as plain host C++ with
// TE_NL = 1 (TE_HOST, tools/enc_host/): that build exists ONLY as a debugging
// harness for the RD logic against the reference bitstream on a CPU-only box;
// libthor_amd.so never contains it.
//
// Every function restates the reference behaviour it cites (file:line under
// the reference tree; enc/ and common/ of awakecoding/thor).  Integer and
// float semantics follow the reference's gcc -std=c99 x86-64 build exactly:
// arithmetic right shifts, C division truncating toward zero, float params
// promoted to double, no FMA contraction (-ffp-contract=off).
#pragma once
#include <stdint.h>
#include <string.h>

#include <stdlib.h>
#if defined(TE_HOST)
#define TE_FN static inline
#define TE_NOINL static
#define TE_LANE 0
#define TE_NL 1
#define TE_CONST static const
#define TE_HD static inline
#define TE_MFN inline
#else
#define TE_FN __device__ __forceinline__
#define TE_NOINL __device__ __noinline__
#define TE_LANE ((int)threadIdx.x)
#define TE_NL 64
#define TE_CONST __constant__ static const
#define TE_HD __host__ __device__ inline
#define TE_MFN __device__ __forceinline__
#endif

// ---- wave helpers -----------------------------------------------------------
// te_sync: every lane's earlier global / LDS writes are visible to every lane
// of the wave afterwards.  One wave per worker: the memory operations of a
// wavefront are performed in order, so a wavefront-scope fence (no
// instruction, it only stops the compiler from moving memory operations
// across it) plus a wave barrier is all that is needed -- no s_waitcnt drain.
TE_FN void te_sync() {
#if !defined(TE_HOST)
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#endif
}
// Wave reductions (every call site is wave-uniform control flow, all 64
// lanes active): DPP within each 16-lane row -- quad_perm [1,0,3,2], [2,3,0,1],
// row_half_mirror, row_mirror, each lane then holds its row's result -- and the
// four rows combined through readlane in SGPRs.  Four VALU ops and four
// readlanes, no LDS round trip (the __shfl_xor butterfly was six
// ds_bpermute_b32 round trips per reduction).  Returns a uniform value.
#if !defined(TE_HOST)
#define TE_DPP(v, ctrl) __builtin_amdgcn_update_dpp((int)(v), (int)(v), (ctrl), 0xF, 0xF, false)
#endif
TE_FN uint32_t te_sum(uint32_t v) {
#if !defined(TE_HOST)
  v += (uint32_t)TE_DPP(v, 0xB1);
  v += (uint32_t)TE_DPP(v, 0x4E);
  v += (uint32_t)TE_DPP(v, 0x141);
  v += (uint32_t)TE_DPP(v, 0x140);
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) + (uint32_t)__builtin_amdgcn_readlane((int)v, 16) +
         (uint32_t)__builtin_amdgcn_readlane((int)v, 32) + (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
#else
  return v;
#endif
}
TE_FN int te_maxi(int v) {
#if !defined(TE_HOST)
  v = max(v, TE_DPP(v, 0xB1));
  v = max(v, TE_DPP(v, 0x4E));
  v = max(v, TE_DPP(v, 0x141));
  v = max(v, TE_DPP(v, 0x140));
  return max(max(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
             max(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
#else
  return v;
#endif
}
TE_FN int te_any(int v) {
#if !defined(TE_HOST)
  return __any(v) ? 1 : 0;
#else
  return v != 0;
#endif
}

// e / w for the lane-strided 2-D loops: a shift for the (usual) power-of-two
// widths, a division otherwise (rectangular edge blocks)
TE_FN int te_dv(int e, int w) {
#if !defined(TE_HOST)
  return (w & (w - 1)) == 0 ? e >> __builtin_ctz(w) : e / w;
#else
  return e / w;
#endif
}

// te_lds(p): on the device, p is known to point into LDS (a worker's
// __shared__ state handed down through a generic pointer or reference).  The
// cast lets the compiler emit ds_* instead of flat_* accesses for it in the
// (non-inlined) callee -- flat accesses wait on both memory counters and take
// the vector-memory path.  Identity on the host.
#if !defined(TE_HOST)
template <typename T>
__device__ __forceinline__ T *te_lds(T *p) {
  return (T *)(__attribute__((address_space(3))) T *)p;
}
// te_glb(p): p points into global memory (the worker's TeScratchMem)
template <typename T>
__device__ __forceinline__ T *te_glb(T *p) {
  return (T *)(__attribute__((address_space(1))) T *)p;
}
#else
template <typename T>
static inline T *te_lds(T *p) {
  return p;
}
template <typename T>
static inline T *te_glb(T *p) {
  return p;
}
#endif
// zero n bytes (n % 4 == 0, 4-byte aligned) with every lane
TE_FN void te_zero_words(void *p, int n) {
  uint32_t *w = (uint32_t *)p;
  for (int e = TE_LANE; e < (n >> 2); e += TE_NL) w[e] = 0u;
}

// ---- 4-pixel (dword) helpers ----------------------------------------------------
// Pixel loops that can take four horizontally adjacent pixels per lane do so:
// one (possibly unaligned) dword load / store instead of four byte accesses,
// and the byte-SIMD ALU ops of CDNA (v_sad_u8, v_dot4_u32_u8).  The host build
// computes the same values byte by byte.
typedef uint32_t __attribute__((aligned(1))) te_u32u;
#if !defined(TE_HOST)
TE_FN uint32_t te_ld4(const uint8_t *p) { return *(const te_u32u *)p; }
TE_FN void te_st4(uint8_t *p, uint32_t v) { *(te_u32u *)p = v; }
#else
TE_FN uint32_t te_ld4(const uint8_t *p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
TE_FN void te_st4(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }
#endif
TE_FN int te_b(uint32_t v, int k) { return (int)((v >> (8 * k)) & 255u); }
// sum |a_k - b_k| + acc
TE_FN uint32_t te_sad4(uint32_t a, uint32_t b, uint32_t acc) {
#if !defined(TE_HOST)
  return __builtin_amdgcn_sad_u8(a, b, acc);
#else
  for (int k = 0; k < 4; k++) acc += (uint32_t)abs(te_b(a, k) - te_b(b, k));
  return acc;
#endif
}
// sum a_k * b_k + acc (unsigned bytes)
TE_FN uint32_t te_dot4(uint32_t a, uint32_t b, uint32_t acc) {
#if !defined(TE_HOST)
  return __builtin_amdgcn_udot4(a, b, acc, false);
#else
  for (int k = 0; k < 4; k++) acc += (uint32_t)(te_b(a, k) * te_b(b, k));
  return acc;
#endif
}
// bytes (lo | hi << 32) >> (8 * s), s in 0..3
TE_FN uint32_t te_align4(uint32_t hi, uint32_t lo, int s) {
#if !defined(TE_HOST)
  return __builtin_amdgcn_alignbyte(hi, lo, s);
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * s));
#endif
}
// per byte: (a + b) >> 1 (truncating) and (a + b + 1) >> 1 (rounding), exact
TE_FN uint32_t te_avg4(uint32_t a, uint32_t b) { return (a & b) + (((a ^ b) >> 1) & 0x7f7f7f7fu); }
TE_FN uint32_t te_ravg4(uint32_t a, uint32_t b) { return (a | b) - (((a ^ b) >> 1) & 0x7f7f7f7fu); }
// four values in 0..255 -> bytes.  The empty asm keeps the compiler from
// fusing a clamp-and-pack into gfx950's v_ashr_pk_u8_i32, whose result this
// hipcc (ROCm 7.2) ORs with the stale upper half of the destination register
// (byte 2 of the packed word comes out corrupted; tools/probes/pix_check.hip).
TE_FN uint32_t te_pack4(int a, int b, int c, int d) {
#if !defined(TE_HOST)
  asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
#endif
  return (uint32_t)a | (uint32_t)b << 8 | (uint32_t)c << 16 | (uint32_t)d << 24;
}

// Optional per-function cycle accounting (built only with -DTHOR_ENC_PROFILE,
// tools/enc_profile.py): s_memtime deltas and call counts per category.
#if defined(THOR_ENC_PROFILE) && !defined(TE_HOST)
__device__ unsigned long long *te_prof_buf;
struct TeProf {
  int c;
  unsigned long long t;
  __device__ __forceinline__ TeProf(int c_) : c(c_), t(__builtin_amdgcn_s_memtime()) {}
  __device__ __forceinline__ ~TeProf() {
    if (threadIdx.x == 0 && te_prof_buf) {
      atomicAdd(&te_prof_buf[2 * c], __builtin_amdgcn_s_memtime() - t);
      atomicAdd(&te_prof_buf[2 * c + 1], 1ULL);
    }
  }
};
#define TE_P(c) TeProf te_prof_scope_(c)
#else
#define TE_P(c)
#endif
// Optional decision trace (built only with -DTHOR_ENC_TRACE: tools/enc_trace.py
// on the device, tools/enc_host on the host): 8 ints per record -- frame,
// kind, ypos, xpos, a, b, c, d -- for the frame number te_trace_frame, so the
// RD decisions of the device and host builds can be compared record by record
// (per superblock; WPP interleaves superblocks on the device).
#if defined(THOR_ENC_TRACE)
#if defined(TE_HOST)
static int *te_trace_buf;  // [0]: record count, records from [8]
static unsigned te_trace_cap;
static int te_trace_frame = -1;
static inline void te_trace_put(int fr, int k, int y, int x, int a, int b, int c, int d) {
  if (!te_trace_buf || fr != te_trace_frame) return;
  const unsigned i = (unsigned)te_trace_buf[0]++;
  if (i >= te_trace_cap) return;
  int *r = te_trace_buf + 8 + 8 * (size_t)i;
  r[0] = fr, r[1] = k, r[2] = y, r[3] = x, r[4] = a, r[5] = b, r[6] = c, r[7] = d;
}
#else
__device__ int *te_trace_buf;
__device__ unsigned te_trace_cap;
__device__ int te_trace_frame;
__device__ __forceinline__ void te_trace_put(int fr, int k, int y, int x, int a, int b, int c, int d) {
  if (!te_trace_buf || fr != te_trace_frame) return;
  if ((int)threadIdx.x == __builtin_ctzll(__builtin_amdgcn_read_exec())) {  // first active lane
    const unsigned i = atomicAdd((unsigned *)te_trace_buf, 1u);
    if (i < te_trace_cap) {
      int *r = te_trace_buf + 8 + 8 * (size_t)i;
      r[0] = fr, r[1] = k, r[2] = y, r[3] = x, r[4] = a, r[5] = b, r[6] = c, r[7] = d;
    }
  }
}
#endif
#define TE_TR(fr, k, y, x, a, b, c, d) te_trace_put(fr, k, y, x, (int)(a), (int)(b), (int)(c), (int)(d))
#else
#define TE_TR(fr, k, y, x, a, b, c, d)
#endif

enum { TP_WCOEF, TP_WBLOCK, TP_INTER_COMP, TP_INTRA_COMP, TP_ENC_BLOCK, TP_COST, TP_SEARCH_INTRA, TP_ME, TP_MODE,
       TP_ES_CHECK, TP_ES_SEARCH, TP_COMMIT, TP_MC_Y, TP_MC_C, TP_FWD, TP_QUANT, TP_INV, TP_IPRED, TP_TOPLEFT, TP_SAD,
       TP_SB, TP_WAIT, TP_N };

#define TE_MIN(a, b) ((a) < (b) ? (a) : (b))
#define TE_MAX(a, b) ((a) > (b) ? (a) : (b))
TE_FN int te_clip255(int x) { return x < 0 ? 0 : (x > 255 ? 255 : x); }
TE_FN int te_clip16(int x) { return x < -32768 ? -32768 : (x > 32767 ? 32767 : x); }
TE_FN int te_wrap16(int x) { return (int)(int16_t)(uint16_t)(x & 0xffff); }
TE_FN int te_abs(int x) { return x < 0 ? -x : x; }
TE_FN int te_log2(int x) {  // log2i of a power of two
  int r = 0;
  while (x > 1) {
    x >>= 1;
    r++;
  }
  return r;
}
TE_FN int te_log2u(unsigned x) {  // floor(log2) (common/simd.h log2i), x >= 1
  int r = 0;
  while (x > 1) {
    x >>= 1;
    r++;
  }
  return r;
}

// ---- constants (common/global.h:57-88, common/types.h) ---------------------
enum { TE_SKIP = 0, TE_INTRA = 1, TE_INTER = 2, TE_BIPRED = 3, TE_MERGE = 4 };
enum { TE_I = 0, TE_P = 1, TE_B = 2 };
enum { TE_DC = 0, TE_PLANAR, TE_HOR, TE_VER, TE_UPLEFT, TE_UPRIGHT, TE_UPUPRIGHT, TE_UPUPLEFT, TE_UPLEFTLEFT,
       TE_DOWNLEFTLEFT, TE_NUM_INTRA };
#define TE_MAX_UINT32 2147483648u  // MAX_UINT32 is `1<<31` (global.h:65), i.e. 2^31 as uint32_t
#define TE_MAX_REF 4               // references an encoder frame can use (max_num_ref <= 4, 2-bit header field)
#define TE_MVCAND 64               // frame_info_t.mvcand[..][64] (enc/mainenc.h:126)

struct TeMv {
  int16_t x, y;
};
// inter_pred_t (common/types.h:111-118); uint32 ref_idx / bipred_flag kept as
// int32 (bipred_flag is -1 for intra neighbours: dir = -1, encode_block.c:2028)
struct TeInterPred {
  TeMv mv0, mv1;
  int32_t ref_idx0, ref_idx1, bipred_flag;
};
// deblock_data_t per 4x4 cell (common/types.h:127-135), filled by copy_deblock_data
// (enc/encode_block.c:1947-1981), zeroed per frame (enc/encode_frame.c:74)
struct TeCell {
  TeInterPred ip;
  uint8_t mode, size, tb_split, pb_part;
  uint8_t cbp_y, cbp_u, cbp_v, rsv;
};
struct TeCtx {  // block_context_t (common/types.h:181-188)
  int split, cbp, index;
};

// Frame-level inputs of one encoder frame (encoder_info_t / frame_info_t /
// enc_params, enc/mainenc.h): everything the RD loop reads besides the pixels.
struct TeFrame {
  const uint8_t *oy, *ou, *ov;  // original frame (orig), interior (0,0)
  int osy, osc;
  uint8_t *ry, *ru, *rv;        // frame being reconstructed (rec), interior (0,0)
  int rsy, rsc;                 // strides of rec AND of every reference (one ring)
  const uint8_t *refy[TE_MAX_REF], *refu[TE_MAX_REF], *refv[TE_MAX_REF];  // ref[ref_array[r]] (padded 96/48)
  int ref_fnum[TE_MAX_REF];
  TeCell *cells;
  int W, H;
  int frame_num, frame_type, qp, num_ref, num_intra_modes, interp_ref;
  double lambda, sqrt_lambda;   // frame_info->lambda and sqrt(lambda), computed on the host
  // enc_params (enc/strings.c:286-338)
  int speed, enable_tb_split, enable_pb_split, enable_bipred, max_delta_qp, delta_qp_step;
  int intra_rdo, use_block_contexts, rdoq, sync;
  float early_skip_thr;
  const int *es_thr;  // early-skip thresholds [2][52][4], te_es_thresholds (host)
};

// ---- tables -------------------------------------------------------------------
TE_CONST int te_chroma_qp_t[52] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17,
                                   18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 29, 30, 31, 32, 33, 33,
                                   34, 34, 35, 35, 36, 36, 37, 37, 38, 39, 40, 41, 42, 43, 44, 45};
TE_FN int te_chroma_qp(int q) { return te_chroma_qp_t[q < 0 ? 0 : (q > 51 ? 51 : q)]; }
TE_CONST int te_gquant[6] = {26214, 23302, 20560, 18396, 16384, 14564};  // common/common_block.c:97
TE_CONST int te_gdequant[6] = {40, 45, 51, 57, 64, 72};                  // :98
// iq_8x8, enc/encode_block.c:2967-2971
TE_CONST uint16_t te_iq8[52] = {6,   7,   8,   8,   10,  11,  12,  13,  15,  17,  19,   21,   24,   27,
                                30,  34,  38,  43,  48,  54,  60,  68,  76,  86,  96,   108,  121,  136,
                                152, 171, 192, 216, 242, 272, 305, 342, 384, 431, 484,  543,  610,  684,
                                768, 862, 968, 1086, 1219, 1368, 1536, 1724, 1935, 2172};

// zigzag scans (common/common_block.c:38-73; zigzag16 / 64 / 256 all follow
// this rule): anti-diagonals, alternating direction.  te_zz(q, raster) = scan
// position, te_izz(q, pos) = raster index, from tables built at compile time.
struct TeZigzag {
  uint8_t zz[3][256], iz[3][256];  // q = 4, 8, 16
  constexpr TeZigzag() : zz(), iz() {
    for (int t = 0; t < 3; t++) {
      const int q = 4 << t;
      for (int r = 0; r < q * q; r++) {
        const int i = r / q, j = r % q, d = i + j;
        int before = 0;
        if (d < q) before = d * (d + 1) / 2;
        else {
          const int e = 2 * q - 1 - d;
          before = q * q - e * (e + 1) / 2;
        }
        const int lo = d < q ? 0 : d - q + 1, hi = d < q ? d : q - 1;
        const int z = (d & 1) ? before + (i - lo) : before + (hi - i);
        zz[t][r] = (uint8_t)z;
        iz[t][z] = (uint8_t)r;
      }
    }
  }
};
TE_CONST TeZigzag te_zig = TeZigzag();
#if defined(TE_HOST)
static const TeZigzag &te_zig_h = te_zig;
#else
static const TeZigzag te_zig_h = TeZigzag();  // host copy (the parser)
#endif
#if !defined(TE_HOST)
// LDS copy for the encoder worker (k_enc_rows loads it once: te_load_zig); the
// per-lane lookups of quantize / write_coeff then cost an LDS read, not a
// divergent global load
__shared__ uint8_t te_zig_lds[1][3][256];  // te_zz only: te_izz (write_coeff's scan) reads the constant table
__device__ __forceinline__ void te_load_zig() {
  for (int e = threadIdx.x; e < 768; e += 64) {
    te_zig_lds[0][e >> 8][e & 255] = te_zig.zz[e >> 8][e & 255];
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
#endif
TE_HD int te_zz(int q, int r) {
#if defined(__HIP_DEVICE_COMPILE__)
  return te_zig_lds[0][q == 4 ? 0 : (q == 8 ? 1 : 2)][r];
#else
  return te_zig_h.zz[q == 4 ? 0 : (q == 8 ? 1 : 2)][r];
#endif
}
TE_FN int te_izz(int q, int pos) {
  return te_zig.iz[q == 4 ? 0 : (q == 8 ? 1 : 2)][pos];
}

// ---- bit writer (enc/putbits.c:112-146) -------------------------------------
// One stream per superblock: MSB-first bits into 32-bit words.  The word being
// filled lives in a register (`cur`, zeros past `pos`); a completed word is
// stored once (lane 0).  Rewinding (write_stream_pos) restores the partial
// word at the old position; later writes overwrite what followed.
struct TeBits {
  uint32_t *w;
  int pos, cap;  // bits
  uint32_t cur;
};
TE_FN void te_bits_start(TeBits &b) {
  b.pos = 0;
  b.cur = 0;
}
TE_FN void te_put(TeBits &b, int n, uint32_t val) {
  if (n <= 0) return;
  if (n < 32) val &= (1u << n) - 1;
  const int room = 32 - (b.pos & 31);
  if (n < room) {
    b.cur |= val << (room - n);
  } else {
    const int n1 = n - room;  // bits that spill into the next word
    const uint32_t full = b.cur | (n1 ? val >> n1 : val);
    if (TE_LANE == 0 && b.pos + room <= b.cap) b.w[b.pos >> 5] = full;
    b.cur = n1 ? (val & ((1u << n1) - 1)) << (32 - n1) : 0u;
  }
  b.pos += n;
}
TE_FN void te_rewind(TeBits &b, int p) {
  const int off = p & 31;
  const uint32_t keep = off ? ~(0xffffffffu >> off) : 0u;
  if ((p >> 5) != (b.pos >> 5)) {
    // the word at p was completed and stored: reload it (lane 0 wrote it, and
    // a wave's memory operations are performed in order)
    b.cur = off ? (b.w[p >> 5] & keep) : 0u;
  } else {
    b.cur &= keep;
  }
  b.pos = p;
}
// A register copy of a writer whose state is wave-uniform: the serial syntax
// writers work on it (SGPRs, scalar branches) instead of going through the
// caller's TeBits in memory on every put, and store it back once at the end.
TE_FN int te_uni(int v) {
#if !defined(TE_HOST)
  return __builtin_amdgcn_readfirstlane(v);
#else
  return v;
#endif
}
TE_FN TeBits te_bits_local(const TeBits &b) {
  TeBits l;
#if !defined(TE_HOST)
  const uint64_t a = (uint64_t)b.w;
  l.w = (uint32_t *)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(a >> 32)) << 32) |
                     (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a));
  l.cur = (uint32_t)__builtin_amdgcn_readfirstlane((int)b.cur);
#else
  l.w = b.w;
  l.cur = b.cur;
#endif
  l.pos = te_uni(b.pos);
  l.cap = te_uni(b.cap);
  return l;
}

// store the partial last word (end of a superblock)
TE_FN void te_bits_flush(TeBits &b) {
  if ((b.pos & 31) && TE_LANE == 0 && b.pos <= b.cap) b.w[b.pos >> 5] = b.cur;
}

// quote_vlc / put_vlc, enc/putvlc.c:34-229 (tables 0-5, 10, 11; the others
// are unused by the encoder): code length, and the code word in *code.
TE_FN int te_vlc(unsigned n, unsigned cn, unsigned *code) {
  unsigned len, c;
  if (n <= 5) {
    if ((int)cn < (6 * (1 << n))) {
      const unsigned t = 1u << n;
      c = t + (cn & (t - 1));
      len = 1 + n + (cn >> n);
    } else {
      c = cn - (6 * (1 << n)) + (1 << n);
      len = (6 - n) + 1 + 2 * te_log2u(c);
    }
  } else if (n == 10) {
    c = cn + 1;
    len = 1 + 2 * te_log2u(c);
  } else {  // n == 11
    len = cn < 2 ? cn + 1 : cn / 2 + 3;
    c = cn < 2 ? 1 : 2 + (cn & 1);
  }
  if (code) *code = c;
  return (int)len;
}
TE_FN int te_quote_vlc(unsigned n, unsigned cn) { return te_vlc(n, cn, nullptr); }
TE_FN int te_put_vlc(TeBits &b, unsigned n, unsigned cn) {
  unsigned c;
  const int len = te_vlc(n, cn, &c);
  // putbits(len, code): len can exceed 32 only for absurd code numbers
  if (len > 32) {
    te_put(b, len - 32, 0);
    te_put(b, 32, c);
  } else {
    te_put(b, len, c);
  }
  return len;
}

// quote_mv_bits, enc/encode_block.c:799-814
TE_FN int te_mv_bits(int dy, int dx) {
  int bits = te_quote_vlc(10, 2 * te_abs(dx) - (dx < 0 ? 1 : 0));
  bits += te_quote_vlc(10, 2 * te_abs(dy) - (dy < 0 ? 1 : 0));
  return bits;
}
// write_mv, enc/write_bits.c:50-69
TE_FN void te_write_mv(TeBits &b, TeMv mv, TeMv mvp) {
  const int dx = mv.x - mvp.x, dy = mv.y - mvp.y;
  te_put_vlc(b, 10, 2 * (uint16_t)te_abs(dx) - (dx < 0 ? 1 : 0));
  te_put_vlc(b, 10, 2 * (uint16_t)te_abs(dy) - (dy < 0 ? 1 : 0));
}

// ---- availability (common/common_block.c:100-129) ----------------------------
TE_HD int te_up_avail(int ypos) { return ypos > 0; }
TE_HD int te_left_avail(int xpos) { return xpos > 0; }
TE_HD int te_upright_avail(int ypos, int xpos, int size, int width) {
  int a = (ypos > 0) && (xpos + size < width);
  if (size == 32 && (ypos % 64) == 32) a = 0;
  if (size == 16 && ((ypos % 32) == 16 || ((ypos % 64) == 32 && (xpos % 32) == 16))) a = 0;
  if (size == 8 && ((ypos % 16) == 8 || ((ypos % 32) == 16 && (xpos % 16) == 8) || ((ypos % 64) == 32 && (xpos % 32) == 24)))
    a = 0;
  return a;
}
TE_HD int te_downleft_avail(int ypos, int xpos, int size, int height) {
  int a = (xpos > 0) && (ypos + size < height);
  if (size == 64) a = 0;
  if (size == 32 && (ypos % 64) == 32) a = 0;
  if (size == 16 && ((ypos % 64) == 48 || ((ypos % 64) == 16 && (xpos % 32) == 16))) a = 0;
  if (size == 8 && ((ypos % 64) == 56 || ((ypos % 16) == 8 && (xpos % 16) == 8) || ((ypos % 64) == 24 && (xpos % 32) == 16)))
    a = 0;
  return a;
}

TE_HD TeInterPred te_zero_pred() {
  TeInterPred z;
  z.mv0.x = z.mv0.y = z.mv1.x = z.mv1.y = 0;
  z.ref_idx0 = z.ref_idx1 = z.bipred_flag = 0;
  return z;
}

// get_mv_pred, common/inter_prediction.c:182-294: median of three neighbours
// chosen by the availability pattern.
TE_HD TeMv te_mv_pred(int ypos, int xpos, int width, int height, int size, const TeCell *db) {
  const int bsz = size / 4, bs = width / 4, bi = (ypos / 4) * bs + xpos / 4;
  const int up0 = bi - bs, up1 = bi - bs + (bsz - 1) / 2, up2 = bi - bs + bsz - 1;
  const int l0 = bi - 1, l1 = bi + bs * ((bsz - 1) / 2) - 1, l2 = bi + bs * (bsz - 1) - 1;
  const int dl = bi + bs * bsz - 1, ur = bi - bs + bsz, ul = bi - bs - 1;
  const int U = te_up_avail(ypos), UR = te_upright_avail(ypos, xpos, size, width), L = te_left_avail(xpos),
            DL = te_downleft_avail(ypos, xpos, size, height);
  TeMv z;
  z.x = z.y = 0;
  TeMv a = z, b = z, c = z;
  if (U == 0 && UR == 0 && L == 0 && DL == 0) {
  } else if (U == 1 && UR == 0 && L == 0 && DL == 0) {
    a = db[up0].ip.mv0; b = db[up1].ip.mv0; c = db[up2].ip.mv0;
  } else if (U == 1 && UR == 1 && L == 0 && DL == 0) {
    a = db[up0].ip.mv0; b = db[up2].ip.mv0; c = db[ur].ip.mv0;
  } else if (U == 0 && UR == 0 && L == 1 && DL == 0) {
    a = db[l0].ip.mv0; b = db[l1].ip.mv0; c = db[l2].ip.mv0;
  } else if (U == 1 && UR == 0 && L == 1 && DL == 0) {
    a = db[ul].ip.mv0; b = db[up2].ip.mv0; c = db[l2].ip.mv0;
  } else if (U == 1 && UR == 1 && L == 1 && DL == 0) {
    a = db[up0].ip.mv0; b = db[ur].ip.mv0; c = db[l2].ip.mv0;
  } else if (U == 0 && UR == 0 && L == 1 && DL == 1) {
    a = db[l0].ip.mv0; b = db[l2].ip.mv0; c = db[dl].ip.mv0;
  } else if (U == 1 && UR == 0 && L == 1 && DL == 1) {
    a = db[up2].ip.mv0; b = db[l0].ip.mv0; c = db[dl].ip.mv0;
  } else if (U == 1 && UR == 1 && L == 1 && DL == 1) {
    a = db[up0].ip.mv0; b = db[ur].ip.mv0; c = db[l0].ip.mv0;
  }
  TeMv p;
  if (a.x < b.x) p.x = TE_MIN(b.x, TE_MAX(a.x, c.x));
  else p.x = TE_MIN(a.x, TE_MAX(b.x, c.x));
  if (a.y < b.y) p.y = TE_MIN(b.y, TE_MAX(a.y, c.y));
  else p.y = TE_MIN(a.y, TE_MAX(b.y, c.y));
  return p;
}

TE_HD int te_pred_equal(const TeInterPred &t, const TeInterPred &c) {
  // duplicate test of get_mv_skip / get_mv_merge (inter_prediction.c:434-438, :587-591)
  return t.mv0.x == c.mv0.x && t.mv0.y == c.mv0.y && t.ref_idx0 == c.ref_idx0 && t.mv1.x == c.mv1.x &&
         t.mv1.y == c.mv1.y && t.ref_idx1 == c.ref_idx1 && (t.bipred_flag == c.bipred_flag || t.bipred_flag == -1);
}

// get_mv_skip / get_mv_merge with LIMITED_SKIP (common/global.h:81),
// common/inter_prediction.c:449-501 / :296-348: left (bottom-most) and
// up-right (else up, right-most) neighbours, duplicates removed.  The merge
// list is the same derivation (both functions are identical under
// LIMITED_SKIP; bipred_copy is unused there).
TE_HD int te_mv_skip(int ypos, int xpos, int width, int height, int size, const TeCell *db, TeInterPred *out) {
  const int bsz = size / 4, bs = width / 4, bi = (ypos / 4) * bs + xpos / 4;
  int up0 = bi - bs, up2 = bi - bs + bsz - 1, l0 = bi - 1, l2 = bi + bs * (bsz - 1) - 1, ur = bi - bs + bsz;
  const int U = te_up_avail(ypos), L = te_left_avail(xpos), UR = te_upright_avail(ypos, xpos, size, width);
  if (ypos + size > height) l2 = l0;
  if (xpos + size > width) up2 = up0;
  TeInterPred t0 = L ? db[l2].ip : te_zero_pred();
  TeInterPred t1 = UR ? db[ur].ip : (U ? db[up2].ip : te_zero_pred());
  out[0] = t0;
  int n = 1;
  if (!te_pred_equal(t1, out[0])) out[n++] = t1;
  return n;
}

// find_block_contexts, common/common_block.c:158-178
TE_HD TeCtx te_block_ctx(int ypos, int xpos, int height, int width, int size, const TeCell *db, int enable) {
  TeCtx c;
  if (ypos >= 8 && xpos >= 8 && ypos + size < height && xpos + size < width && enable && size <= 64) {
    const int bs = width / 4, bi = (ypos / 4) * bs + xpos / 4;
    const TeCell &u = db[bi - bs], &l = db[bi - 1];
    c.split = (u.size < size) + (l.size < size);
    c.cbp = (u.cbp_y > 0) + (l.cbp_y > 0);
    const int cbp2 = (u.cbp_y > 0 || u.cbp_u > 0 || u.cbp_v > 0) + (l.cbp_y > 0 || l.cbp_u > 0 || l.cbp_v > 0);
    c.index = 3 * c.split + cbp2;
  } else {
    c.split = c.cbp = c.index = -1;
  }
  return c;
}

// add_mvcandidate, enc/encode_block.c:60-73: integer-rounded MV, deduplicated
// by a 64-bit hash mask (hash collisions drop the candidate, as there).
struct TeMvCand {
  TeMv mv[TE_MAX_REF][TE_MVCAND];
  int num[TE_MAX_REF];
  uint64_t mask[TE_MAX_REF];
};
TE_FN void te_add_mvcand(TeMvCand &mc, int r, TeMv mv) {
  TeMv im;
  im.x = (int16_t)((mv.x + 2) >> 2);
  im.y = (int16_t)((mv.y + 2) >> 2);
  const uint64_t m = (uint64_t)1 << ((((int)im.y << 3) ^ (int)im.x) & 63);
  if (!(m & mc.mask[r])) {
    // every lane stores the same value: each lane later reads its own write,
    // so no cross-lane ordering is needed
    mc.mv[r][mc.num[r]] = im;
    mc.num[r] += 1;
  }
  mc.mask[r] |= m;
}

// ---- block parameters (block_param_t, common/types.h:153-170) ---------------
// Coefficients are stored compactly: per component four q x q tiles
// (q = min(N, 16)), one per transform block (tb-split quarters in raster
// order), row-major.  Only that low-frequency corner can be non-zero
// (common/transform.c:309-327; quantize writes nothing else, enc/encode_block.c:170-174).
#define TE_COEF_COMP 1024
// Per-level strides of that layout: component stride cs (the 64 / 32 levels'
// 1024, the 16 / 8 levels' own size^2) and tb-split tile stride ts
// (min(N/2, 16)^2), so the small levels' coefficient sets are small enough for LDS.
#define TE_CS(S) ((S) <= 16 ? (S) * (S) : TE_COEF_COMP)
#define TE_TS(S) ((S) <= 32 ? ((S) / 2) * ((S) / 2) : 256)
struct TeParam {
  int mode, intra_mode, skip_idx, pb_part;
  TeMv mv0[4], mv1[4];
  int ref_idx0, ref_idx1, dir;
  int cbp_y, cbp_u, cbp_v;
  int tb_param, tb_split;
  int16_t *coeff;  // 3 components (Y, U, V) at stride cs, tb-split tiles at stride ts
  int cs, ts;
};

struct TeBlockInfo {  // block_info_t, enc/mainenc.h:97-116
  int size, ypos, xpos, bwidth, bheight;
  TeParam bp;  // block_info.block_param (the best so far)
  TeInterPred skip_c[2], merge_c[2];
  int num_skip, num_merge;
  TeMv mvp;
  int max_num_pb_part, max_num_tb_part, delta_qp, final_encode;
  TeCtx ctx;
  uint8_t *rec, *rec_best;  // compact Y (size^2) | U | V ((size/2)^2 each)
  uint32_t *best_bits;      // the syntax bits the best candidate wrote (MSB first), or
  int best_nbits;           // -1: not kept (the final write_block runs again)
  int best_cap;             // capacity of best_bits in words
};

// ---- block syntax (enc/write_bits.c) --------------------------------------
// find_code, write_bits.c:71-108
TE_FN int te_find_code(int run, int level, int maxrun, int chroma, int eob) {
  const int maxrun2 = TE_MAX(4, maxrun);
  const int index = run + (level > 1) * (maxrun2 + 1);
  if (chroma) {
    if (eob) return 0;
    if (index <= 4) return index + 1;
    if (index <= maxrun2) return index + 3;
    if (index == maxrun2 + 1) return 6;
    if (index == maxrun2 + 2) return 7;
    return index + 1;
  }
  if (eob) return 2;
  if (index < 2) return index;
  if (index <= 4) return index + 1;
  if (index <= maxrun2) return index + 3;
  if (index == maxrun2 + 1) return 6;
  if (index == maxrun2 + 2) return 7;
  return index + 1;
}

// write_coeff, write_bits.c:110-253: run-level VLC of one transform block's
// q x q tile `c` (raster) of an N x N block.  The scan-order levels sit in
// registers (device: lane l holds positions l, l+64, l+128, l+192, read back
// with readlane) with a non-zero bitmap, so the serial coder steps only over
// coded events: runs of zeros are skipped with bit scans.
struct TeScanRegs {
#if defined(TE_HOST)
  int v[256];
  uint64_t nz[4];
  TE_MFN int at(int pos) const { return v[pos]; }
#else
  int v0, v1, v2, v3;
  uint64_t nz[4];
  __device__ __forceinline__ int at(int pos) const {
    const int k = pos >> 6;
    const int r = k == 0 ? v0 : (k == 1 ? v1 : (k == 2 ? v2 : v3));
    return __builtin_amdgcn_readlane(r, pos & 63);
  }
#endif
  // first non-zero position >= pos (pos < 256), or 256
  TE_MFN int next_nz(int pos) const {
    for (int k = pos >> 6; k < 4; k++) {
      const uint64_t m = nz[k] & (k == (pos >> 6) ? (~0ULL << (pos & 63)) : ~0ULL);
      if (m) return k * 64 + __builtin_ctzll(m);
    }
    return 256;
  }
  TE_MFN int last_nz() const {
    for (int k = 3; k >= 0; k--)
      if (nz[k]) return k * 64 + 63 - __builtin_clzll(nz[k]);
    return -1;
  }
};
TE_FN void te_load_scan(TeScanRegs &R, const int16_t *c, int q) {
  const int N = q * q;
#if defined(TE_HOST)
  for (int k = 0; k < 4; k++) R.nz[k] = 0;
  for (int pos = 0; pos < 256; pos++) {
    R.v[pos] = pos < N ? c[te_izz(q, pos)] : 0;
    if (R.v[pos]) R.nz[pos >> 6] |= 1ULL << (pos & 63);
  }
#else
  const int l = TE_LANE;
  R.v0 = l < N ? c[te_izz(q, l)] : 0;
  R.v1 = l + 64 < N ? c[te_izz(q, l + 64)] : 0;
  R.v2 = l + 128 < N ? c[te_izz(q, l + 128)] : 0;
  R.v3 = l + 192 < N ? c[te_izz(q, l + 192)] : 0;
  R.nz[0] = __ballot(R.v0 != 0);
  R.nz[1] = __ballot(R.v1 != 0);
  R.nz[2] = __ballot(R.v2 != 0);
  R.nz[3] = __ballot(R.v3 != 0);
#endif
}
#if !defined(TE_HOST)
// write_coeff's events from pos 0 with every lane coding its own positions
// (device).  The coder's mode before position p is a two-state recurrence --
// level mode continues over non-zero levels and ends after a coded zero; run
// mode returns to level mode after a level > 1 -- i.e. L[p+1] = big[p] |
// (nz[p] & L[p]), L[0] = 1, which is the carry chain of nz + big + 1 over the
// 256 scan positions (scalar adds).  Each lane then codes its position's event
// -- level mode: the level VLC (table 1 after a previous level-mode level > 3,
// or at the start of an intra luma block; table 0 otherwise) and the sign;
// run mode, at a non-zero: the run/level code from the position after the
// previous event, then the level / sign -- as one code word of <= 58 bits
// (|level| <= 32768), and the words go into the writer in scan order.  Then
// the tail: the extra level-mode zero and EOB, as the serial coder.
TE_FN int te_prev_bit(uint64_t w, int base) { return w ? base + 63 - __builtin_clzll(w) : -1; }
TE_FN void te_coeff_events(TeBits &b, const TeScanRegs &R, int N, int size, int chroma, int intra, int last_pos) {
  const int l = TE_LANE;
  uint64_t big[4], g3[4], Lm[4];
  big[0] = __ballot(te_abs(R.v0) > 1);
  big[1] = __ballot(te_abs(R.v1) > 1);
  big[2] = __ballot(te_abs(R.v2) > 1);
  big[3] = __ballot(te_abs(R.v3) > 1);
  g3[0] = __ballot(te_abs(R.v0) > 3);
  g3[1] = __ballot(te_abs(R.v1) > 3);
  g3[2] = __ballot(te_abs(R.v2) > 3);
  g3[3] = __ballot(te_abs(R.v3) > 3);
  uint64_t cin = 1;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint64_t a = R.nz[k], t = a + big[k], s = t + cin;
    Lm[k] = s ^ a ^ big[k];
    cin = (t < a) | (s < t);
  }
  const uint64_t below = (1ull << l) - 1;  // lanes' lower positions within a word (l < 64)
  int pl_lo = -1, pe_lo = -1;             // highest level-mode / event position in the words already done
  const int kmax = last_pos >> 6;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (k > kmax) break;
    const int v = k == 0 ? R.v0 : (k == 1 ? R.v1 : (k == 2 ? R.v2 : R.v3));
    const int p = 64 * k + l;
    const uint64_t upto = kmax > k ? ~0ull : (last_pos == 64 * k + 63 ? ~0ull : ((2ull << (last_pos & 63)) - 1));
    const uint64_t lw = Lm[k] & upto, ew = (Lm[k] | R.nz[k]) & upto;
    int len = 0;
    uint64_t code = 0;
    const int level = te_abs(v), sign = v < 0 ? 1 : 0;
    if ((lw >> l) & 1) {  // level mode
      int pl = te_prev_bit(lw & below, 64 * k);
      if (pl < 0) pl = pl_lo;
      int adapt = 0;
      if (!chroma) {
        if (pl < 0) {
          adapt = intra;
        } else {
          const int kw = pl >> 6;
          const uint64_t gw = kw == k ? g3[k] : (kw == 0 ? g3[0] : (kw == 1 ? g3[1] : g3[2]));
          adapt = (int)((gw >> (pl & 63)) & 1);
        }
      }
      unsigned c;
      len = te_vlc((unsigned)adapt, (unsigned)level, &c);
      code = c;
      if (level) {
        code = (code << 1) | (uint64_t)sign;
        len++;
      }
    } else if ((ew >> l) & 1) {  // run mode, a non-zero level
      int pe = te_prev_bit(ew & below, 64 * k);
      if (pe < 0) pe = pe_lo;
      const int ps = pe + 1, run = p - ps;
      const int cn = te_find_code(run, level, N - ps - 1, chroma, 0);
      unsigned c1, c2;
      int n1, n2;
      if (chroma && size <= 8) {
        n1 = te_vlc(10, (unsigned)cn, &c1);
      } else if (cn == 0) {
        n1 = 2;
        c1 = 2;
      } else {
        n1 = te_vlc(2, (unsigned)(cn + 1), &c1);
      }
      if (level > 1) {
        n2 = te_vlc(0, (unsigned)(2 * (level - 2) + sign), &c2);
      } else {
        n2 = 1;
        c2 = (unsigned)sign;
      }
      code = ((uint64_t)c1 << n2) | c2;
      len = n1 + n2;
    }
    // the words in scan order (the writer is uniform: scalar puts)
    uint64_t em = __ballot(len > 0);
    const uint32_t chi = (uint32_t)(code >> 32), clo = (uint32_t)code;
    while (em) {
      const int s = __builtin_ctzll(em);
      em &= em - 1;
      const int n = __builtin_amdgcn_readlane(len, s);
      const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)clo, s);
      if (n > 32) {
        te_put(b, n - 32, (uint32_t)__builtin_amdgcn_readlane((int)chi, s));
        te_put(b, 32, lo);
      } else {
        te_put(b, n, lo);
      }
    }
    const int plw = te_prev_bit(lw, 64 * k), pew = te_prev_bit(ew, 64 * k);
    if (plw >= 0) pl_lo = plw;
    if (pew >= 0) pe_lo = pew;
  }
  // tail (write_bits.c:223-252): after the last non-zero, still in level mode
  // -> one more zero level; then EOB unless the block is full
  int pos = last_pos + 1;
  if (pos < N) {
    const int kl = last_pos >> 6;
    const uint64_t nzw = R.nz[0] * (kl == 0) | R.nz[1] * (kl == 1) | R.nz[2] * (kl == 2) | R.nz[3] * (kl == 3);
    const uint64_t bw = big[0] * (kl == 0) | big[1] * (kl == 1) | big[2] * (kl == 2) | big[3] * (kl == 3);
    const uint64_t lmw = Lm[0] * (kl == 0) | Lm[1] * (kl == 1) | Lm[2] * (kl == 2) | Lm[3] * (kl == 3);
    const int bl = last_pos & 63;
    const bool fin = ((nzw >> bl) & 1) ? (((bw | lmw) >> bl) & 1) != 0 : true;  // (no non-zero: cbp says never)
    if (fin) {
      int adapt = 0;
      if (!chroma) {
        if (pl_lo < 0) {
          adapt = intra;
        } else {
          const int kw = pl_lo >> 6;
          const uint64_t gw = g3[0] * (kw == 0) | g3[1] * (kw == 1) | g3[2] * (kw == 2) | g3[3] * (kw == 3);
          adapt = (int)((gw >> (pl_lo & 63)) & 1);
        }
      }
      te_put_vlc(b, (unsigned)adapt, 0);
      pos++;
    }
  }
  if (pos < N) {
    const int cn = te_find_code(0, 0, 0, chroma, 1);
    if (chroma && size <= 8) {
      te_put_vlc(b, 0, cn);
    } else {
      if (cn == 0) te_put(b, 2, 2);
      else te_put_vlc(b, 2, cn + 1);
    }
  }
}
#endif

// The writer state travels by value (in registers) in and out: a reference
// would pin the caller's register copy to the stack.  Inlined into
// write_block (its only caller): no call frame per coded TU.
TE_FN TeBits te_write_coeff(TeBits b_in, const int16_t *c, int size, int type) {
  TE_P(TP_WCOEF);
  TeBits b = te_bits_local(b_in);
  size = te_uni(size);
  type = te_uni(type);
  const int q = TE_MIN(16, size), N = q * q;
  const int chroma = type & 1, intra = (type >> 1) & 1;
  int vlc_adaptive = intra && !chroma;
  TeScanRegs R;
  te_load_scan(R, c, q);
  int last_pos = R.last_nz();
  if (last_pos < 0) last_pos = 0;  // cbp != 0 guarantees a non-zero level (fatalerror otherwise, :142-143)
  int pos = 0;
  if (chroma) {
    const int s0 = R.at(0);
    if (last_pos == 0 && te_abs(s0) == 1) {
      te_put(b, 1, 1);
      te_put(b, 1, s0 < 0 ? 1 : 0);
      pos = N;
    } else {
      te_put(b, 1, 0);
    }
  }
#if !defined(TE_HOST) && !defined(TE_WCOEF_SERIAL)
  if (pos == 0) {  // (not the chroma single +-1 DC)
    te_coeff_events(b, R, N, size, chroma, intra, last_pos);
    return b;
  }
#endif
  int level_mode = 1, level = 1;
  while (pos <= last_pos) {
    if (level_mode) {
      while (pos <= last_pos && level > 0) {
        const int cc = R.at(pos);
        level = te_abs(cc);
        te_put_vlc(b, vlc_adaptive, level);
        if (level > 0) te_put(b, 1, cc < 0 ? 1 : 0);
        if (chroma == 0) vlc_adaptive = level > 3;
        pos++;
      }
    }
    if (pos <= last_pos) {  // run mode: the next non-zero lies at or before last_pos
      const int maxrun = N - pos - 1;
      const int np = R.next_nz(pos);
      const int run = np - pos;
      const int cc = R.at(np);
      level = te_abs(cc);
      const int sign = cc < 0 ? 1 : 0;
      const int cn = te_find_code(run, level, maxrun, chroma, 0);
      if (chroma && size <= 8) {
        te_put_vlc(b, 10, cn);
      } else {
        if (cn == 0) te_put(b, 2, 2);
        else te_put_vlc(b, 2, cn + 1);
      }
      if (level > 1) te_put_vlc(b, 0, 2 * (level - 2) + sign);
      else te_put(b, 1, sign);
      pos = np + 1;
      level_mode = level > 1;
    }
  }
  if (pos < N) {
    if (level_mode) {  // terminated in level mode: one extra zero before EOB (:223-236)
      te_put_vlc(b, vlc_adaptive, 0);
      pos++;
    }
  }
  if (pos < N) {  // EOB (:238-252)
    const int cn = te_find_code(0, 0, 0, chroma, 1);
    if (chroma && size <= 8) {
      te_put_vlc(b, 0, cn);
    } else {
      if (cn == 0) te_put(b, 2, 2);
      else te_put_vlc(b, 2, cn + 1);
    }
  }
  return b;
}

// write_block's code tables (enc/write_bits.c:385 cbp codes, :401-413 intra mode codes),
// constant memory: a local array indexed at run time would be built on the
// stack on every call
TE_CONST int8_t te_wb_cbp[8] = {1, 0, 5, 2, 6, 3, 7, 4};
TE_CONST int8_t te_wb_map8[10] = {2, 8, 1, 0, 5, 9, 7, 6, 4, 3};
TE_CONST int8_t te_wb_len8[8] = {2, 2, 2, 4, 4, 4, 5, 5};
TE_CONST int8_t te_wb_cw8[8] = {0, 1, 2, 12, 13, 14, 30, 31};
TE_CONST int8_t te_wb_map10[10] = {2, 3, 1, 0, 6, 9, 8, 7, 5, 4};
TE_CONST int8_t te_wb_len10[10] = {2, 2, 3, 3, 4, 4, 5, 5, 5, 5};
TE_CONST int8_t te_wb_cw10[10] = {2, 3, 2, 3, 2, 3, 0, 1, 2, 3};

// write_delta_qp, write_bits.c:255-265
TE_FN void te_write_delta_qp(TeBits &b, int dqp) {
  te_put_vlc(b, 0, te_abs(dqp));
  if (dqp != 0) te_put(b, 1, dqp < 0 ? 1 : 0);
}

// write_super_mode, write_bits.c:268-362
TE_FN void te_write_super_mode(TeBits &b, const TeFrame &F, const TeBlockInfo &bi, int mode, int ref_idx0,
                               int split_flag) {
  const int size = bi.size;
  if (F.frame_type != TE_I) {
    if (split_flag == 1) {
      if (size > 64) {
        te_put(b, 1, 0);
      } else {
        int code = 1;
        if (bi.ctx.index == 2 || bi.ctx.index > 3) code = (code + 3) % 4;
        te_put(b, code + 1, 1);
      }
      return;
    }
    int code = 0;
    const int bipred_possible = F.num_ref > 1 && F.enable_bipred;
    const int split_possible = size > 8;
    const int maxbit = 2 + F.num_ref + split_possible + bipred_possible;
    if (F.interp_ref) {
      if (mode == TE_SKIP) code = 0;
      else if (mode == TE_MERGE) code = 2;
      else if (mode == TE_BIPRED) code = 3;
      else if (mode == TE_INTRA) code = 4;
      else if (mode == TE_INTER && ref_idx0 > 0) code = 4 + ref_idx0;
      else code = 4 + F.num_ref;
      if (!bipred_possible && code > 3) code = code - 1;
      if (!split_possible && code > 1) code = code - 1;
      if ((bi.ctx.index == 2 || bi.ctx.index > 3) && size > 8) {
        if (code < 3) code = (code + 2) % 3;
      }
    } else {
      if (mode == TE_SKIP) code = 0;
      else if (mode == TE_INTER && ref_idx0 == 0) code = 2;
      else if (mode == TE_MERGE) code = 3;
      else if (mode == TE_BIPRED) code = 4;
      else if (mode == TE_INTRA) code = 5;
      else if (mode == TE_INTER && ref_idx0 > 0) code = 5 + ref_idx0;
      if (!bipred_possible && code > 4) code = code - 1;
      if (!split_possible && code > 1) code = code - 1;
      if ((bi.ctx.index == 2 || bi.ctx.index > 3) && size > 8) {
        if (code < 4) code = (code + 3) % 4;
      }
    }
    if (code == maxbit) te_put(b, maxbit, 0);
    else te_put(b, code + 1, 1);
  } else {
    if (size > 8 || split_flag == 1) te_put(b, 1, split_flag);
  }
}

TE_FN const int16_t *te_tile(const TeParam &p, int comp, int idx) { return p.coeff + comp * p.cs + idx * p.ts; }

// write_block, write_bits.c:364-650.  Returns the number of bits written.
TE_NOINL int te_write_block(TeBits &bo_, const TeFrame &F_, const TeBlockInfo &bi_, const TeParam &p_, int16_t *scan_) {
  const TeFrame &F = *te_lds(&F_);
  const TeBlockInfo &bi = *te_lds(&bi_);
  TeBits &bo = *te_lds(&bo_);
  const TeParam &p = *te_lds(&p_);
  (void)scan_;  // (unused: the coefficient coder keeps its scan in registers)
  TE_P(TP_WBLOCK);
  TeBits b = te_bits_local(bo);
  const int start = b.pos;
  const int size = bi.size, mode = p.mode, tb_split = p.tb_split;
  const int coeff_type = (mode == TE_INTRA) << 1;
  const int8_t *cbp_table = te_wb_cbp;
  te_write_super_mode(b, F, bi, mode, p.ref_idx0, 0);
  if (size == 64 && mode != TE_SKIP && F.max_delta_qp) te_write_delta_qp(b, bi.delta_qp);
  if (mode == TE_INTRA) {
    const int im = p.intra_mode;
    if (F.num_intra_modes <= 4) {
      te_put(b, 2, im);
    } else if (F.num_intra_modes <= 8) {
      const int code = te_wb_map8[im];
      te_put(b, te_wb_len8[code], te_wb_cw8[code]);
    } else {
      const int code = te_wb_map10[im];
      te_put(b, te_wb_len10[code], te_wb_cw10[code]);
    }
  } else if (mode == TE_INTER) {
    if (bi.max_num_pb_part > 1) {
      if (p.pb_part == 0) te_put(b, 1, 1);
      else if (p.pb_part == 1) te_put(b, 2, 1);
      else if (p.pb_part == 2) te_put(b, 3, 1);
      else te_put(b, 3, 0);
    }
    TeMv mvp2 = bi.mvp;
    if (p.pb_part == 0) {
      te_write_mv(b, p.mv0[0], mvp2);
    } else if (p.pb_part == 1) {
      te_write_mv(b, p.mv0[0], mvp2);
      mvp2 = p.mv0[0];
      te_write_mv(b, p.mv0[2], mvp2);
    } else if (p.pb_part == 2) {
      te_write_mv(b, p.mv0[0], mvp2);
      mvp2 = p.mv0[0];
      te_write_mv(b, p.mv0[1], mvp2);
    } else {
      te_write_mv(b, p.mv0[0], mvp2);
      mvp2 = p.mv0[0];
      te_write_mv(b, p.mv0[1], mvp2);
      te_write_mv(b, p.mv0[2], mvp2);
      te_write_mv(b, p.mv0[3], mvp2);
    }
  } else if (mode == TE_BIPRED) {  // BIPRED_PART 0 (common/global.h:76)
    TeMv mvp2 = bi.mvp;
    if (p.pb_part == 0) te_write_mv(b, p.mv0[0], mvp2);
    if (F.frame_type == TE_B) mvp2 = p.mv0[0];
    if (p.pb_part == 0) {
      te_write_mv(b, p.mv1[0], mvp2);
    } else if (p.pb_part == 1) {
      te_write_mv(b, p.mv1[0], mvp2);
      mvp2 = p.mv1[0];
      te_write_mv(b, p.mv1[2], mvp2);
    } else if (p.pb_part == 2) {
      te_write_mv(b, p.mv1[0], mvp2);
      mvp2 = p.mv1[0];
      te_write_mv(b, p.mv1[1], mvp2);
    } else {
      te_write_mv(b, p.mv1[0], mvp2);
      mvp2 = p.mv1[0];
      te_write_mv(b, p.mv1[1], mvp2);
      te_write_mv(b, p.mv1[2], mvp2);
      te_write_mv(b, p.mv1[3], mvp2);
    }
    if (F.frame_type == TE_P) {
      if (F.num_ref == 2) {
        const int code = 2 * p.ref_idx0 + p.ref_idx1;
        if (code == 3) te_put(b, 3, 0);
        else te_put(b, code + 1, 1);
      } else {
        te_put_vlc(b, 10, 4 * p.ref_idx0 + p.ref_idx1);
      }
    }
  } else if (mode == TE_SKIP) {
    if (bi.num_skip == 4) {
      te_put(b, 2, p.skip_idx);
    } else if (bi.num_skip == 3) {
      if (p.skip_idx == 0) te_put(b, 1, 1);
      else if (p.skip_idx == 1) te_put(b, 2, 0);
      else te_put(b, 2, 1);
    } else if (bi.num_skip == 2) {
      te_put(b, 1, p.skip_idx);
    }
  } else if (mode == TE_MERGE) {
    if (bi.num_merge == 4) {
      te_put(b, 2, p.skip_idx);
    } else if (bi.num_merge == 3) {
      if (p.skip_idx == 0) te_put(b, 1, 1);
      else if (p.skip_idx == 1) te_put(b, 2, 0);
      else te_put(b, 2, 1);
    } else if (bi.num_merge == 2) {
      te_put(b, 1, p.skip_idx);
    }
  }
  if (mode != TE_SKIP) {
    int max_tb = 1, code;
    if (mode == TE_MERGE || mode == TE_BIPRED) max_tb = 1;
    else if (mode == TE_INTER) max_tb = bi.max_num_tb_part > 1 ? 2 : 1;
    else if (mode == TE_INTRA) max_tb = bi.max_num_tb_part;
    if (max_tb > 1) {
      if (tb_split) {
        code = 2;
      } else {
        const int cbp = p.cbp_y + (p.cbp_u << 1) + (p.cbp_v << 2);
        code = cbp_table[cbp];
        if (bi.ctx.cbp == 0 && code < 2) code = 1 - code;
        if (code > 1) code++;
      }
    } else {
      const int cbp = p.cbp_y + (p.cbp_u << 1) + (p.cbp_v << 2);
      code = cbp_table[cbp];
      if (mode == TE_MERGE) {
        if (code == 1) code = 7;
        else if (code > 1) code = code - 1;
      } else {
        if (bi.ctx.cbp == 0 && code < 2) code = 1 - code;
      }
    }
    te_put_vlc(b, 0, code);
    // The coded tiles in syntax order, with the split CBP codes between them,
    // as one loop: a single coefficient-coder call site (its device body is
    // large; eight inlined copies doubled write_block's code).
    //   no split:   Y, U, V
    //   split > 8:  per quarter: CBP code, Y, U, V
    //   split 8x8:  per quarter: cbp_y bit, Y; then the chroma CBP, U, V
    const int nstep = tb_split == 0 ? 3 : (size > 8 ? 16 : 11);
#pragma clang loop unroll(disable)
    for (int s = 0; s < nstep; s++) {
      int comp = 0, index = 0, tsz = 0, on = 0;
      if (tb_split == 0) {
        comp = s;
        tsz = s ? size / 2 : size;
        on = s == 0 ? p.cbp_y : (s == 1 ? p.cbp_u : p.cbp_v);
      } else if (size > 8) {
        index = s >> 2;
        const int cy = (p.cbp_y >> (3 - index)) & 1, cu = (p.cbp_u >> (3 - index)) & 1, cv = (p.cbp_v >> (3 - index)) & 1;
        if ((s & 3) == 0) {
          code = cbp_table[cy + (cu << 1) + (cv << 2)];
          if (bi.ctx.cbp == 0 && code < 2) code = 1 - code;
          te_put_vlc(b, 0, code);
          continue;
        }
        comp = (s & 3) - 1;
        tsz = comp ? size / 4 : size / 2;
        on = comp == 0 ? cy : (comp == 1 ? cu : cv);
      } else if (s < 8) {
        index = s >> 1;
        const int cy = (p.cbp_y >> (3 - index)) & 1;
        if ((s & 1) == 0) {
          te_put(b, 1, cy);
          continue;
        }
        tsz = size / 2;
        on = cy;
      } else if (s == 8) {
        // chroma of an 8x8 CU is not split: cbp_u / cbp_v are the block values here
        const int cbp = p.cbp_u + 2 * p.cbp_v;
        if (cbp == 0) te_put(b, 1, 1);
        else if (cbp == 1) te_put(b, 2, 1);
        else if (cbp == 2) te_put(b, 3, 1);
        else te_put(b, 3, 0);
        continue;
      } else {
        comp = s - 8;
        tsz = size / 2;
        on = comp == 1 ? p.cbp_u : p.cbp_v;
      }
      if (on) b = te_write_coeff(b, te_tile(p, comp, index), tsz, coeff_type | (comp ? 1 : 0));
    }
  }
  bo = b;
  return b.pos - start;
}
