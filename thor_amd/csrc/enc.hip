// Device-resident Thor encoder for gfx950: kernels and the host C-ABI
// (include/thor_amd.h, "device-resident encoder").
//
// Per frame (and per batch of up to THOR_ENC_MAX_BATCH streams, one launch
// per stage for all of them):
//   k_enc_rows      the RD loop: persistent wave64 workers take the batch's
//                   superblocks from one queue in readiness order; SB (k, l) is
//                   queued when SB (k, l-1) and SB (k-1, l+1) are done (the
//                   up-right neighbour is the furthest one the RD loop reads,
//                   enc/encode_block.c:2819-2879).  The RD loop of
//                   the SB (enc_rd.h) writes the reconstruction into the ring
//                   slot, the 4x4 side info and the SB's bit string.
//                   Each SB's cells also become the loop filters' 16-bit words there.
//   k_enc_db_v/h    deblocking of every job's frame (the decoder's bodies, loopfilter.hip)
//   k_enc_clpf      CLPF decision per full SB (clpf_decision, enc/encode_frame.c:50-63)
//                   and CLPF of the flagged ones, one 8x8 block per lane
//   k_enc_pad       padding (the decoder's body)
//   k_enc_pack      frame header + SB bit strings + CLPF bits -> the frame's
//                   bytes (putbits / flush_all_bits, enc/putbits.c:57-129),
//                   written straight into page-locked host memory
#include <atomic>

#include "common.h"
#include "enc_gop.h"
#include "enc_rd.h"

#include <deque>
#include <map>
#include <mutex>

#define THOR_ENC_MAX_BATCH 512  // te_q_item codes the job in 9 bits
#define TE_MAX_WORKERS 4096  // k_enc_rows workgroups per launch (4 x 1 024 SIMDs)
#define THOR_ENC_SB_WORDS 4096  // 131072 bits of one SB's stream (trial writes included)

__global__ void k_deblock_v(const FrameBatch, int, int);
__global__ void k_deblock_h(const FrameBatch, int, int);
__global__ void k_clpf(const FrameBatch);
__global__ void k_pad(const FrameBatch, int, int);

// One stream's frame job (device memory, one per stream of a launch).
struct TeJob {
  TeFrame F;
  uint32_t *sb_words;   // [nsb][THOR_ENC_SB_WORDS]
  int *sb_nbits;        // [nsb]
  unsigned *deps;       // [nsb] finished dependencies per SB (left, up-right), k_enc_rows' scheduler
  int qbase;            // this job's range of the scheduler queue k_enc_clear marks empty
  int8_t *clpf_bits;    // [nsb_full]: -1 no bit, else the flag
  uint8_t *clpf_flags;  // [nsb_full]: CLPF applied (k_clpf input)
  uint16_t *cellinfo;
  const uint32_t *hdr_words;  // frame header (+ sequence header) bits, MSB first
  int hdr_bits;
  uint32_t *out_words;  // packed frame
  int *out_bits;
  int nsbh, nsbv, clpf, deblock;
  int32_t *sb_costs;    // optional [nsb][cost_stride]: each SB's delta-QP trial costs, then its final cost
  int cost_stride;
};

// Poll with a relaxed device-coherent load; the acquire fence follows once,
// after the condition holds (an acquire load per poll would invalidate the
// L2 on every iteration of every waiting wave).
__device__ __forceinline__ unsigned te_ld_relaxed(const unsigned *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Superblock scheduler.  An SB (k, l) may be coded once its left neighbour
// (k, l - 1) and its up-right one (k - 1, min(l + 1, nsbh - 1)) are done -- the
// WPP order of the reference's neighbour reads (enc/encode_block.c:2819-2879).
// Workers are persistent single-wave workgroups that take the batch's SBs from
// one queue in readiness order: the worker that completes an SB counts it
// into its dependants' counters (`deps`) and queues each one it completes.
// A worker that took slot h waits until slot h is filled; every SB is queued
// exactly once, so every slot below the batch's SB count fills (the slots a
// waiting worker holds are past every queued SB, and a queued SB is always
// held by a running worker).  Unlike one worker per SB row, a worker never
// idles while its row waits for the row above: it codes whatever SB of any
// stream is ready.  No state travels between a worker's SBs (the SB's syntax
// state is reset per SB, te_encode_sb; neighbours come from the cells and the
// reconstruction in global memory).
// Two workers per SIMD: the RD loop is a latency-bound chain of small
// dependent steps (LDS round trips, VALU -> SALU hand-offs), so a second wave
// hides part of it -- 15 % off the 4K I frame at 240 streams.
// That needs <= 20 KB of LDS per worker (the small levels live in global
// memory, TeSmallLv) and <= 256 registers.  THOR_ENC_WPE overrides (experiments).
#if !defined(THOR_ENC_WPE)
#define THOR_ENC_WPE 2
#endif
#define TE_WPE __attribute__((amdgpu_waves_per_eu(THOR_ENC_WPE)))
#define TE_Q_EMPTY 0xffffffffu
// Priority levels of the SB queue (TE_QLEVELS > 1, an experiment): an SB of row k goes to level
// k * TE_QLEVELS / nsbv, a worker takes the oldest ready SB of the lowest non-empty level -- the upper
// rows of every stream gate its whole frame, so the streams that are behind get the workers first.
// Measured SLOWER (240 x 4K x 8 frames, 4 levels: 1.73-1.76 s vs 1.54-1.57 s; the P-frame SBs cost
// 24 % more summed RD time -- leaving readiness order costs the neighbouring SBs' shared L2 lines,
// profiles/r07/queue_levels_*.txt), so the product keeps one FIFO.
// Level v's head / tail at q[64 v] / q[64 v + 32] (separate 128-byte lines), its items at off[v].
#ifndef TE_QLEVELS
#define TE_QLEVELS 1
#endif
struct TeQLevels {
  unsigned off[8], cap[8];
};
#define TE_QHEAD(v) ((v)*64)
#define TE_QTAIL(v) ((v)*64 + 32)
#define TE_QDONE (8 * 64)
// Continuation (TE_CONT, single queue): the worker that makes its right neighbour (k, l + 1) ready
// codes it next itself instead of queueing it -- the row's chain skips a queue round trip and the SB
// runs where its left neighbour's data and the overlapping search window are warm.  The queue then
// fills fewer slots than there are SBs: q[TE_QTOTAL] counts the slots that will fill (decremented per
// kept SB); a ticket at or past it will never fill and its worker leaves.  Measured SLOWER (240 x 4K x 8
// frames: 1.64-1.67 s vs 1.54-1.57 s, queue waits of the I frame doubled, P-frame RD time +3 %;
// profiles/r07/continuation_*.txt): off.
#ifndef TE_CONT
#define TE_CONT 0
#endif
#define TE_QTOTAL (8 * 64 + 32)
// A queue item: job s (< THOR_ENC_MAX_BATCH = 512: 9 bits), SB row k and column l
// (11 bits each: frames up to 65 535 px, te_check_params' limit, have <= 1 024
// SB rows / columns).  The top bit stays clear, so no item equals TE_Q_EMPTY.
__device__ __forceinline__ unsigned te_q_item(int s, int k, int l) { return (unsigned)s << 22 | (unsigned)k << 11 | (unsigned)l; }
// (lane 0) one more finished dependency of SB (k, l) of job s; queue it when that was its last.
// Relaxed atomics: the worker's release fence after its SB already wrote its
// results back to device scope (every dependency's did, before its count), and
// the worker that takes the SB acquires once -- an acquire / release per
// atomic here would write back and invalidate the XCD's L2 several times per SB.
__device__ __forceinline__ void te_dep_done(const TeJob &J, int s, int k, int l, unsigned *q, unsigned *items,
                                            const TeQLevels &QL) {
  const unsigned need = (unsigned)((l > 0) + (k > 0));
  const unsigned old = __hip_atomic_fetch_add(&J.deps[k * J.nsbh + l], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (old + 1 == need) {
#if TE_QLEVELS > 1
    const int v = k * TE_QLEVELS / J.nsbv;
    const unsigned slot = __hip_atomic_fetch_add(&q[TE_QTAIL(v)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&items[QL.off[v] + slot], te_q_item(s, k, l), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
    (void)QL;
    const unsigned slot = __hip_atomic_fetch_add(&q[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&items[slot], te_q_item(s, k, l), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
  }
}
// the 16-bit loop-filter word of a cell (the decoder's packing, prep_body in recon.hip)
__device__ __forceinline__ uint16_t te_cellinfo_word(const TeCell &c) {
  const int size = c.size < 8 ? 8 : c.size;
  const int lsz = size >= 64 ? 6 : (size >= 32 ? 5 : (size >= 16 ? 4 : 3));
  const int tb = c.tb_split > 0, pb = c.pb_part;
  const int lqv = lsz - (((tb || pb == 2 || pb == 3) && size > 8) ? 1 : 0);
  const int lqh = lsz - (((tb || pb == 1 || pb == 3) && size > 8) ? 1 : 0);
  const int big = (abs(c.ip.mv0.x) >= 4) | (abs(c.ip.mv0.y) >= 4) | (abs(c.ip.mv1.x) >= 4) | (abs(c.ip.mv1.y) >= 4);
  return (uint16_t)((c.mode & 7) | ((c.cbp_y != 0) << 3) | ((c.cbp_u != 0) << 4) | ((c.cbp_v != 0) << 5) | (big << 6) |
                    (lqv << 8) | (lqh << 11) | ((lsz - 3) << 14));
}
// the loop-filter words of SB (k, l)'s cells, once the SB is coded (its cells are final then)
__device__ __forceinline__ void te_sb_cellinfo(const TeJob &J, int k, int l) {
  const int cs = J.F.W >> 2, r0 = k * 16, c0 = l * 16;
  for (int e = threadIdx.x; e < 256; e += 64) {
    const int r = r0 + (e >> 4), c = c0 + (e & 15);
    if (r < (J.F.H >> 2) && c < cs) J.cellinfo[r * cs + c] = te_cellinfo_word(J.F.cells[r * cs + c]);
  }
}

// k_enc_rows' profile, summed over its workers across launches (100 MHz ticks): time coding SBs,
// time waiting for a queue slot, SBs coded (thor_enc_rows_profile reads and clears it)
__device__ unsigned long long g_te_rows_prof[4];
__global__ __launch_bounds__(64) TE_WPE void k_enc_rows(const TeJob *__restrict__ jobs, unsigned total, unsigned *q,
                                                 unsigned *items, TeScratchMem *scratch, unsigned *err,
                                                 unsigned long long spin_limit, int stall_row, const TeQLevels QL) {
  __shared__ TeFrame s_F;  // the job's frame parameters, read all through the RD loop
  __shared__ TeSB s_sb;    // the superblock's bit writer and ME candidate lists
  // the worker's buffers (te_here): LDS at fixed addresses (g_te_*), global at
  // fixed offsets from its TeScratchMem
  g_te_mem = &scratch[blockIdx.x];
  te_load_basis(g_te_tx);
  te_load_zig();
  TeSB &sb = s_sb;
  const int lane = threadIdx.x;
  int cur = -1;  // the job whose frame parameters s_F holds
  unsigned long long t_work = 0, t_wait = 0, n_sb = 0;  // (lane 0) this worker's profile
#if TE_CONT
  unsigned keep = TE_Q_EMPTY;  // (lane 0) the SB this worker codes next, without the queue
#endif
  for (;;) {
    unsigned h = 0;
    const unsigned long long tw0 = __builtin_amdgcn_s_memrealtime();
#if TE_QLEVELS > 1
    // the lowest level with a ready SB: a ticket there when it looks non-empty (a ticket past its
    // items so far waits for its slot: every slot below the level's SB count fills); every level's
    // tickets all handed out: leave; nothing ready anywhere for spin_limit with no SB finished: give up
    unsigned item = 0, gave_up = 0;
    int quit = 0;
    if (lane == 0) {
      unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      unsigned seen = te_ld_relaxed(&q[TE_QDONE]);
      for (;;) {
        bool all = true, got = false;
        for (int v = 0; v < TE_QLEVELS && !got; v++) {
          unsigned hv = te_ld_relaxed(&q[TE_QHEAD(v)]);
          if (hv >= QL.cap[v]) continue;
          all = false;
          if (hv >= te_ld_relaxed(&q[TE_QTAIL(v)])) continue;
          hv = __hip_atomic_fetch_add(&q[TE_QHEAD(v)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (hv >= QL.cap[v]) continue;
          const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
          while ((item = te_ld_relaxed(&items[QL.off[v] + hv])) == TE_Q_EMPTY) {
            __builtin_amdgcn_s_sleep(4);
            if (__builtin_amdgcn_s_memrealtime() - t1 > spin_limit) {
              atomicOr(err, 1u);
              gave_up = 1;
              break;
            }
          }
          got = true;
        }
        if (got || all) {
          quit = !got;
          break;
        }
        const unsigned d = te_ld_relaxed(&q[TE_QDONE]);
        const unsigned long long now = __builtin_amdgcn_s_memrealtime();
        if (d != seen) seen = d, t0 = now;
        if (now - t0 > spin_limit || te_ld_relaxed(err)) {
          atomicOr(err, 1u);
          gave_up = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(8);
      }
    }
    if (__builtin_amdgcn_readfirstlane(quit)) break;
    {
#elif TE_CONT
    unsigned item = 0, gave_up = 0;
    int quit = 0;
    if (lane == 0) {
      if (keep != TE_Q_EMPTY) {
        item = keep;
        keep = TE_Q_EMPTY;
      } else {
        h = __hip_atomic_fetch_add(&q[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (h >= te_ld_relaxed(&q[TE_QTOTAL])) {
          quit = 1;
        } else {
          const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
          while ((item = te_ld_relaxed(&items[h])) == TE_Q_EMPTY) {
            __builtin_amdgcn_s_sleep(4);
            if (h >= te_ld_relaxed(&q[TE_QTOTAL])) {  // kept SBs left this slot unfilled for good
              quit = 1;
              break;
            }
            if (__builtin_amdgcn_s_memrealtime() - t0 > spin_limit) {
              atomicOr(err, 1u);
              gave_up = 1;
              break;
            }
          }
        }
      }
    }
    if (__builtin_amdgcn_readfirstlane(quit)) break;
    {
#else
    if (lane == 0) h = __hip_atomic_fetch_add(&q[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    h = __builtin_amdgcn_readfirstlane(h);
    if (h >= total) break;
    unsigned item = 0, gave_up = 0;
    {
#endif
      TE_P(TP_WAIT);
      if (TE_QLEVELS == 1 && !TE_CONT && lane == 0) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
        while ((item = te_ld_relaxed(&items[h])) == TE_Q_EMPTY) {
          __builtin_amdgcn_s_sleep(4);
          // a wedged dependency (spin_limit, 5 minutes by default): give up, reported; never hang the GPU
          if (__builtin_amdgcn_s_memrealtime() - t0 > spin_limit) {
            atomicOr(err, 1u);
            gave_up = 1;
            break;
          }
        }
      }
    }
    if (__builtin_amdgcn_readfirstlane(gave_up)) break;  // this wave waits no more, so the grid drains
    item = __builtin_amdgcn_readfirstlane(item);
    const unsigned long long tb0 = __builtin_amdgcn_s_memrealtime();
    t_wait += tb0 - tw0;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const int s = (int)(item >> 22), k = (int)((item >> 11) & 2047), l = (int)(item & 2047);
    const TeJob &J = jobs[s];
    if (s != cur) {  // the job's frame parameters into LDS
      const uint32_t *src = (const uint32_t *)&J.F;
      uint32_t *dst = (uint32_t *)&s_F;
      te_sync();
      for (int e = lane; e < (int)(sizeof(TeFrame) / 4); e += 64) dst[e] = src[e];
      te_sync();
      cur = s;
    }
    const int sbi = k * J.nsbh + l;
    sb.bits.w = J.sb_words + (size_t)sbi * THOR_ENC_SB_WORDS;
    sb.bits.cap = THOR_ENC_SB_WORDS * 32;
    te_encode_sb(s_F, sb, k, l, J.sb_costs ? J.sb_costs + (size_t)sbi * J.cost_stride : nullptr);
    if (lane == 0) {
      J.sb_nbits[sbi] = sb.bits.pos;
      if (sb.bits.pos > sb.bits.cap) atomicOr(err, 2u);
    }
    te_sync();  // the SB's cells (written by every lane) -> the loop filters' 16-bit words
    te_sb_cellinfo(J, k, l);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
      // dependants: (k, l + 1) by its left neighbour; (k + 1, l - 1) by its up-right one, and
      // (k + 1, l) too at the row end (its up-right is clipped to this SB).  stall_row: a
      // diagnostics hook (thor_enc_debug_stall) -- that row never releases the row below
#if TE_CONT && TE_QLEVELS == 1
      if (l + 1 < J.nsbh) {  // the right neighbour: kept when this completes it
        const unsigned need = 1u + (k > 0);
        const unsigned old = __hip_atomic_fetch_add(&J.deps[sbi + 1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old + 1 == need) {
          keep = te_q_item(s, k, l + 1);
          __hip_atomic_fetch_sub(&q[TE_QTOTAL], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
#else
      if (l + 1 < J.nsbh) te_dep_done(J, s, k, l + 1, q, items, QL);
#endif
      if (k + 1 < J.nsbv && k != stall_row) {
        if (l >= 1) te_dep_done(J, s, k + 1, l - 1, q, items, QL);
        if (l == J.nsbh - 1) te_dep_done(J, s, k + 1, l, q, items, QL);
      }
      if (TE_QLEVELS > 1) __hip_atomic_fetch_add(&q[TE_QDONE], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      t_work += __builtin_amdgcn_s_memrealtime() - tb0;
      n_sb++;
    }
  }
  if (lane == 0) {
    atomicAdd(&g_te_rows_prof[0], t_work);
    atomicAdd(&g_te_rows_prof[1], t_wait);
    atomicAdd(&g_te_rows_prof[2], n_sb);
  }
}

// Every context's cell state (deblock_data, cleared per frame: enc/encode_frame.c:74)
// and SB dependency counters to zero, one launch for the batch (grid y =
// context), 16-byte stores; the scheduler queue: each job's SB (0, 0) in slot
// s, the job's other SBs' slots empty, head 0, tail n.
__global__ __launch_bounds__(256) void k_enc_clear(const TeJob *__restrict__ jobs, long long cell_bytes, unsigned *q,
                                                   unsigned *items, unsigned long long *arena_ctr) {
  const int s = blockIdx.y;
  const TeJob &J = jobs[s];
  uint4 *c = (uint4 *)J.F.cells;
  const long long n16 = cell_bytes >> 4;
  const int nsb = J.nsbv * J.nsbh;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n16; i += (long long)gridDim.x * 256)
    c[i] = make_uint4(0u, 0u, 0u, 0u);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < nsb; i += gridDim.x * 256) {
    J.deps[i] = 0u;
    J.sb_nbits[i] = 0;  // an SB a failed launch never codes packs as nothing
  }
  for (int i = blockIdx.x * 256 + threadIdx.x; i < nsb - 1; i += gridDim.x * 256) items[J.qbase + i] = TE_Q_EMPTY;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    items[s] = te_q_item(s, 0, 0);
    if (s == 0) {
#if TE_QLEVELS > 1
      for (int v = 0; v < TE_QLEVELS; v++) q[TE_QHEAD(v)] = q[TE_QTAIL(v)] = 0u;
      q[TE_QTAIL(0)] = gridDim.y;  // every job's SB (0, 0): level 0's slots [0, n)
      q[TE_QDONE] = 0u;
#else
      q[0] = 0u;
      q[1] = gridDim.y;
      q[TE_QTOTAL] = (unsigned)gridDim.y * (unsigned)nsb;  // (TE_CONT) slots that will fill
#endif
      *arena_ctr = 0ull;  // this batch's packed frames start at the host arena's first word
    }
  }
}

// CLPF of a full SB with one 8x8 block per lane (block b = lane: row b >> 3,
// column b & 7), the side info from the 16-bit cell words -- te_clpf_decide's
// and clpf_block's arithmetic (enc/encode_frame.c:50-63, common/common_block.c:
// 180-197: the 4-neighbour majority vote, neighbours clamped at the SB border),
// each lane holding its block and a one-pixel ring in registers.
struct TeClpfBlk {
  uint32_t cy[10][3];  // luma rows y0-1 .. y0+8: bytes x0-1 (word 0 byte 3), x0 .. x0+7 (words 1, 2), x0+8 (word 0 byte 0)
};
// luma pixel (r, c) of the block's ring, r, c in -1 .. 8, clamped to the SB (at the SB's edge the
// neighbour is the pixel itself)
__device__ __forceinline__ int te_clpf_ring(const uint32_t (&v)[10][3], int r, int c) {
  const uint32_t *w = v[r + 1];
  if (c < 0) return (int)(w[0] >> 24);
  if (c > 7) return (int)(w[0] & 255);
  return (int)((w[1 + (c >> 2)] >> (8 * (c & 3))) & 255);
}
// loads the ring of the lane's luma block (rows / columns outside the SB: clamped)
__device__ __forceinline__ void te_clpf_load(uint32_t (&v)[10][3], const uint8_t *ry, int rsy, int k, int l) {
  const int lane = threadIdx.x, br = lane >> 3, bc = lane & 7;
  const int y0 = k * 64 + br * 8, x0 = l * 64 + bc * 8;
#pragma unroll
  for (int r = -1; r <= 8; r++) {
    int y = y0 + r;
    if (br == 0 && r < 0) y = y0;  // SB top: the row itself
    if (br == 7 && r > 7) y = y0 + 7;
    const uint8_t *row = ry + (long long)y * rsy + x0;
    const uint2 m = *(const uint2 *)row;
    const uint32_t lft = bc == 0 ? (m.x & 255) : row[-1], rgt = bc == 7 ? (m.y >> 24) : row[8];
    v[r + 1][0] = (lft << 24) | rgt;
    v[r + 1][1] = m.x;
    v[r + 1][2] = m.y;
  }
}
__device__ __forceinline__ int te_clpf_delta(const uint32_t (&v)[10][3], int r, int c, int X) {
  const int A = te_clpf_ring(v, r - 1, c), B = te_clpf_ring(v, r, c - 1), C = te_clpf_ring(v, r, c + 1),
            D = te_clpf_ring(v, r + 1, c);
  return ((A > X) + (B > X) + (C > X) + (D > X) > 2) - ((A < X) + (B < X) + (C < X) + (D < X) > 2);
}
// te_clpf_decide from the cell words: -1 no candidate block, else the flag
__device__ int te_clpf_decide_blk(const uint16_t *cellinfo, int W, const uint8_t *ry, int rsy, const uint8_t *oy,
                                  int osy, int k, int l) {
  const int lane = threadIdx.x, br = lane >> 3, bc = lane & 7;
  const int y0 = k * 64 + br * 8, x0 = l * 64 + bc * 8;
  const uint16_t ci = cellinfo[(y0 >> 2) * (W >> 2) + (x0 >> 2)];
  const int cand = CI_MODE(ci) != 3 && (CI_CBPY(ci) | CI_CBPU(ci) | CI_CBPV(ci));
  uint32_t s0 = 0, s1 = 0;
  if (CI_MODE(ci) != 3 && CI_CBPY(ci)) {
    uint32_t v[10][3];
    te_clpf_load(v, ry, rsy, k, l);
#pragma unroll
    for (int r = 0; r < 8; r++) {
      const uint2 o = *(const uint2 *)(oy + (long long)(y0 + r) * osy + x0);
#pragma unroll
      for (int c = 0; c < 8; c++) {
        const int X = te_clpf_ring(v, r, c), O = (int)(((c < 4 ? o.x : o.y) >> (8 * (c & 3))) & 255);
        const int delta = te_clpf_delta(v, r, c, X);
        s0 += (uint32_t)((O - X) * (O - X));
        s1 += (uint32_t)((O - X - delta) * (O - X - delta));
      }
    }
  }
  const int any = te_any(cand);
  s0 = te_sum(s0);
  s1 = te_sum(s1);
  if (!any) return -1;
  return (int)s1 < (int)s0;
}
// CLPF of a flagged SB in place: every lane loads its ring (all loads before any store), then
// writes its filtered luma block and its 4x4 chroma blocks where the plane has coded residual
__device__ void te_clpf_apply_blk(const uint16_t *cellinfo, int W, uint8_t *ry, int rsy, uint8_t *ru, uint8_t *rv,
                                  int rsc, int k, int l) {
  const int lane = threadIdx.x, br = lane >> 3, bc = lane & 7;
  const int y0 = k * 64 + br * 8, x0 = l * 64 + bc * 8;
  const uint16_t ci = cellinfo[(y0 >> 2) * (W >> 2) + (x0 >> 2)];
  const bool ny = CI_MODE(ci) != 3 && CI_CBPY(ci), nu = CI_MODE(ci) != 3 && CI_CBPU(ci),
             nv = CI_MODE(ci) != 3 && CI_CBPV(ci);
  uint32_t v[10][3];
  te_clpf_load(v, ry, rsy, k, l);
  // chroma 4x4 blocks with their rings (6 x 6), clamped to the SB's 32 x 32
  uint32_t cu[6][2], cv[6][2];  // word 0: bytes c = -1 .. 2, word 1: c = 3, 4 (bytes 0, 1)
  const int cy0 = k * 32 + br * 4, cx0 = l * 32 + bc * 4;
#pragma unroll
  for (int pl = 0; pl < 2; pl++) {
    const uint8_t *P = pl ? rv : ru;
    uint32_t (&w)[6][2] = pl ? cv : cu;
#pragma unroll
    for (int r = -1; r <= 4; r++) {
      int y = cy0 + r;
      if (br == 0 && r < 0) y = cy0;
      if (br == 7 && r > 3) y = cy0 + 3;
      const uint8_t *row = P + (long long)y * rsc + cx0;
      const uint32_t m = *(const uint32_t *)row;
      const uint32_t lft = bc == 0 ? (m & 255) : row[-1], rgt = bc == 7 ? (m >> 24) : row[4];
      w[r + 1][0] = lft | (m << 8);
      w[r + 1][1] = (m >> 24) | (rgt << 8);
    }
  }
  __builtin_amdgcn_wave_barrier();  // (every lane's loads are in registers before the first store)
  if (ny) {
#pragma unroll
    for (int r = 0; r < 8; r++) {
      uint32_t o[2] = {0u, 0u};
#pragma unroll
      for (int c = 0; c < 8; c++) {
        const int X = te_clpf_ring(v, r, c);
        o[c >> 2] |= (uint32_t)((X + te_clpf_delta(v, r, c, X)) & 255) << (8 * (c & 3));
      }
      *(uint2 *)(ry + (long long)(y0 + r) * rsy + x0) = make_uint2(o[0], o[1]);
    }
  }
#pragma unroll
  for (int pl = 0; pl < 2; pl++) {
    if (!(pl ? nv : nu)) continue;
    const uint32_t (&w)[6][2] = pl ? cv : cu;
    auto px = [&](int r, int c) -> int {  // r, c in -1 .. 4
      const int b = c + 1;
      return (int)((b < 4 ? w[r + 1][0] >> (8 * b) : w[r + 1][1] >> (8 * (b - 4))) & 255);
    };
    uint8_t *P = pl ? rv : ru;
#pragma unroll
    for (int r = 0; r < 4; r++) {
      uint32_t o = 0;
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const int X = px(r, c), A = px(r - 1, c), B = px(r, c - 1), C = px(r, c + 1), D = px(r + 1, c);
        const int delta = ((A > X) + (B > X) + (C > X) + (D > X) > 2) - ((A < X) + (B < X) + (C < X) + (D < X) > 2);
        o |= (uint32_t)((X + delta) & 255) << (8 * c);
      }
      *(uint32_t *)(P + (long long)(cy0 + r) * rsc + cx0) = o;
    }
  }
}

// The frame's loop filters, every job of the batch in one launch per pass
// (grid y = job; the decoder's deblocking bodies, loopfilter.hip):
// vertical edges, then horizontal edges, then CLPF decision + CLPF of each
// full SB (one wave per SB: decide, then filter it in place when flagged --
// an SB reads nothing outside itself), then padding.
__global__ __launch_bounds__(256) void k_enc_db_v(const TeJob *__restrict__ jobs, int nbl) {
  const TeJob &J = jobs[blockIdx.y];
  if (!J.deblock) return;
  const TeFrame &F = J.F;
  const int b = blockIdx.x;
  if (b < nbl) {
    luma_v_items<DB_ITEMS>(b * 256 + (int)threadIdx.x, nbl * 256, F.ry, F.rsy, F.W, F.H, J.cellinfo, F.qp);
    return;
  }
  const int c = (b - nbl) >= nbl, bb = b - nbl - c * nbl;  // every chroma edge segment, per plane
  for (int r = 0; r < DB_ITEMS; r++)
    k_deblock_chroma_v_body(bb * 256 + (int)threadIdx.x + r * nbl * 256, c, F.ru, F.rv, F.rsc, F.W, F.H, J.cellinfo,
                            te_chroma_qp(F.qp));
}
__global__ __launch_bounds__(256) void k_enc_db_h(const TeJob *__restrict__ jobs, int nbl) {
  const TeJob &J = jobs[blockIdx.y];
  if (!J.deblock) return;
  const TeFrame &F = J.F;
  const int b = blockIdx.x;
  if (b < nbl) {
    luma_h_items<DB_ITEMS>(b * 256 + (int)threadIdx.x, nbl * 256, F.ry, F.rsy, F.W, F.H, J.cellinfo, F.qp);
    return;
  }
  const int c = (b - nbl) >= nbl, bb = b - nbl - c * nbl;
  for (int r = 0; r < DB_ITEMS; r++)
    k_deblock_chroma_h_body(bb * 256 + (int)threadIdx.x + r * nbl * 256, c, F.ru, F.rv, F.rsc, F.W, F.H, J.cellinfo,
                            te_chroma_qp(F.qp));
}
__global__ __launch_bounds__(64) void k_enc_clpf(const TeJob *__restrict__ jobs) {
  const TeJob &J = jobs[blockIdx.y];
  const int nh = J.F.W >> 6, nv = J.F.H >> 6;
  const int sb = blockIdx.x;
  if (sb >= nh * nv || !J.clpf) return;
  const TeFrame &F = J.F;
  const int k = sb / nh, l = sb % nh;
  const int d = te_clpf_decide_blk(J.cellinfo, F.W, F.ry, F.rsy, F.oy, F.osy, k, l);
  if (threadIdx.x == 0) {
    J.clpf_bits[sb] = (int8_t)d;
    J.clpf_flags[sb] = (uint8_t)(d == 1);
  }
  if (d == 1) te_clpf_apply_blk(J.cellinfo, F.W, F.ry, F.rsy, F.ru, F.rv, F.rsc, k, l);
}
__global__ __launch_bounds__(256) void k_enc_pad(const TeJob *__restrict__ jobs) {
  const TeJob &J = jobs[blockIdx.y];
  const TeFrame &F = J.F;
  k_pad_body(blockIdx.x * 256 + threadIdx.x, F.ry, F.ru, F.rv, F.rsy, F.rsc, F.W, F.H, 0, F.H);
}

// Frame bit string: header | SB strings (raster) | [CLPF: 1, 0, one bit per
// candidate SB] -> MSB-first words, zero padded.  One workgroup per stream.
__device__ __forceinline__ void te_or_bits(uint32_t *dst, long long pos, const uint32_t *src, int n) {
  for (int j = 0; j * 32 < n; j++) {
    uint32_t w = src[j];
    const int nb = n - j * 32 < 32 ? n - j * 32 : 32;
    if (nb < 32) w &= ~(0xffffffffu >> nb);  // drop stale bits past the string's end
    const long long p = pos + 32LL * j;
    const int sh = (int)(p & 31);
    atomicOr(&dst[p >> 5], w >> sh);
    if (sh && (w << (32 - sh))) atomicOr(&dst[(p >> 5) + 1], w << (32 - sh));
  }
}
// An SB's bit count as packed: within its word buffer (a count past it is an
// error the launch already flagged; packing stays inside the buffers).
__device__ __forceinline__ int te_sb_bits(const TeJob &J, int i) {
  const int b = J.sb_nbits[i];
  return b < 0 ? 0 : (b > THOR_ENC_SB_WORDS * 32 ? THOR_ENC_SB_WORDS * 32 : b);
}
// ... then the packed words, byte-swapped (the stream's byte order), into the
// batch's page-locked host arena at a word offset the block takes from
// `arena_ctr`, and (offset, bit count) into `meta` behind a system-scope
// release: the host reads the frame with no copy kernel (small D2H copies run
// as blit kernels, which wait for CU slots the next batch's workers hold).
// Offset -1: the arena was full (the host copies J.out_words instead);
// bit count -1: the frame is over the output buffer.
__global__ __launch_bounds__(256) void k_enc_pack(const TeJob *__restrict__ jobs, long long *scan_tmp, int out_cap_words,
                                                  uint32_t *arena, unsigned long long arena_words,
                                                  unsigned long long *arena_ctr, int *meta, const unsigned *err) {
  const TeJob &J = jobs[blockIdx.x];
  const int nsb = J.nsbh * J.nsbv;
  (void)scan_tmp;
  __shared__ long long total, sbend;
  __shared__ long long aoff;
  __shared__ long long part[256];  // per thread: its SBs' bit count, then their first bit position
  __shared__ int cpart[256];       // per thread: its CLPF candidates, then the first one's bit index
  // thread t packs SBs [s0, s1) and CLPF candidates [c0, c1): the offsets from two block scans
  const int t = threadIdx.x;
  const int per = (nsb + 255) >> 8, s0 = min(t * per, nsb), s1 = min(s0 + per, nsb);
  const int nf = J.clpf ? (J.F.W >> 6) * (J.F.H >> 6) : 0;
  const int perc = (nf + 255) >> 8, c0 = min(t * perc, nf), c1 = min(c0 + perc, nf);
  {
    long long mine = 0;
    for (int i = s0; i < s1; i++) mine += te_sb_bits(J, i);
    int cm = 0;
    for (int i = c0; i < c1; i++) cm += J.clpf_bits[i] >= 0;
    part[t] = mine;
    cpart[t] = cm;
  }
  __syncthreads();
  if (t == 0) {  // exclusive scans over the 256 partial sums (LDS)
    long long o = J.hdr_bits;
    int co = 0;
    for (int i = 0; i < 256; i++) {
      const long long v = part[i];
      part[i] = o;
      o += v;
      const int c = cpart[i];
      cpart[i] = co;
      co += c;
    }
    sbend = o;
    total = o + (J.clpf ? 2 + co : 0);
  }
  __syncthreads();
  const long long nw = (total + 31) >> 5;
  if (nw > out_cap_words) {
    if (threadIdx.x == 0) {
      *J.out_bits = -1;
      meta[2 * blockIdx.x] = -1;
      if (blockIdx.x == 0) meta[2 * THOR_ENC_MAX_BATCH] = (int)*err;
      __hip_atomic_store(&meta[2 * blockIdx.x + 1], -1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    return;
  }
  for (long long i = threadIdx.x; i < nw + 1 && i < out_cap_words; i += 256) J.out_words[i] = 0;
  __syncthreads();
  if (t == 0) te_or_bits(J.out_words, 0, J.hdr_words, J.hdr_bits);
  {
    long long pos = part[t];
    for (int i = s0; i < s1; i++) {
      const int b = te_sb_bits(J, i);
      te_or_bits(J.out_words, pos, J.sb_words + (size_t)i * THOR_ENC_SB_WORDS, b);
      pos += b;
    }
  }
  if (J.clpf) {
    if (t == 0) {
      const uint32_t two = 0x80000000u;  // bits 1, 0
      te_or_bits(J.out_words, sbend, &two, 2);
    }
    long long p = sbend + 2 + cpart[t];
    for (int i = c0; i < c1; i++) {
      const int d = J.clpf_bits[i];
      if (d < 0) continue;
      if (d) atomicOr(&J.out_words[p >> 5], 0x80000000u >> (p & 31));
      p++;
    }
  }
  if (threadIdx.x == 0) {
    *J.out_bits = (int)total;
    const unsigned long long need = (unsigned long long)((nw + 3) & ~3LL);
    const unsigned long long o = arena ? atomicAdd(arena_ctr, need) : ~0ull;
    aoff = arena && o + need <= arena_words ? (long long)o : -1;
  }
  __threadfence();  // every thread's ORs are in before any thread reads the words back
  __syncthreads();
  if (aoff >= 0) {
    const uint4 *src = (const uint4 *)J.out_words;
    uint4 *dst = (uint4 *)(arena + aoff);
    for (long long i = threadIdx.x; i < (nw + 3) >> 2; i += 256) {
      const uint4 v = src[i];
      dst[i] = make_uint4(__builtin_bswap32(v.x), __builtin_bswap32(v.y), __builtin_bswap32(v.z), __builtin_bswap32(v.w));
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // (system scope: the host reads them)
  __syncthreads();
  if (threadIdx.x == 0) {
    meta[2 * blockIdx.x] = (int)aoff;
    if (blockIdx.x == 0) meta[2 * THOR_ENC_MAX_BATCH] = (int)*err;  // k_enc_rows' error flags (it ran before)
    __hip_atomic_store(&meta[2 * blockIdx.x + 1], (int)total, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ============================================================================
// Host side
// ============================================================================
#define EHIP(x)                                                                                        \
  do {                                                                                                  \
    hipError_t e_ = (x);                                                                                \
    if (e_ != hipSuccess) {                                                                             \
      fprintf(stderr, "thor_amd enc: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
      (void)hipGetLastError();                                                                          \
      return e_ == hipErrorOutOfMemory ? THOR_ERR_NOMEM : THOR_ERR_HIP;                                 \
    }                                                                                                   \
  } while (0)

struct thor_enc {
  thor_enc_params_t p;
  TeGop *gop;
  size_t pos;  // next plan
  int device;
  hipStream_t stream;
  int W, H, nsbh, nsbv, nsb, nsb_full;
  int sy, sc;
  long long offy, offu, offv, slot_bytes;
  int nslots;  // the window's 33 + the frame being coded (+ the interpolation slot `islot`)
  int islot;   // interp_ref: the frame's interpolated reference (interp_frames[0]), -1 without
  thor_ti_t *ti;
  uint8_t *slots;
  std::vector<int> slot_of_window;  // window index -> slot (-1: empty)
  std::vector<int> slot_busy;
  TeCell *cells;
  uint16_t *cellinfo;
  uint32_t *sb_words;
  int *sb_nbits;
  unsigned *deps;
  int8_t *clpf_bits;
  uint8_t *clpf_flags;
  int *es_thr;
  uint32_t *hdr_words;   // device, 64 words
  uint32_t *out_words;   // device
  uint32_t *out_words2;  // device: the other frame of a begin / end pipeline (thor_enc_frames_begin)
  int opar;              // which of the two the next frame packs into
  int out_cap_words;
  int *out_bits;         // device
  uint32_t *sb_words2;   // device: the SB buffers of odd frames of a sequence launch (enc_seq.hip), on first use
  int *sb_nbits2;
  int8_t *clpf_bits2;
  int32_t *sb_costs;     // device, thor_enc_record_sb_costs: per SB its top-level process_block costs
  int cost_stride;       // per SB: the delta-QP trials + the final encode
  // last coded frame
  int last_slot, last_frame_num;
  std::vector<uint8_t> chunk;  // 4-byte length + bytes of the last frame
  bool first;
};

static int enc_alloc(thor_enc *e) {
  const int W = e->W, H = e->H;
  e->sy = (W + 2 * THOR_PAD_Y + 15) & ~15;
  e->sc = (W / 2 + 2 * THOR_PAD_C + 15) & ~15;
  long long yb = ((long long)(H + 2 * THOR_PAD_Y) * e->sy + 255) & ~255LL;
  long long cb = ((long long)(H / 2 + 2 * THOR_PAD_C) * e->sc + 255) & ~255LL;
  e->offy = (long long)THOR_PAD_Y * e->sy + THOR_PAD_Y;
  e->offu = yb + (long long)THOR_PAD_C * e->sc + THOR_PAD_C;
  e->offv = yb + cb + (long long)THOR_PAD_C * e->sc + THOR_PAD_C;
  e->slot_bytes = yb + 2 * cb + 256;
  e->nslots = 34;  // the 33-frame window + the frame being coded
  e->islot = -1;
  if (e->p.interp_ref) e->islot = e->nslots++;
  if (!dev_alloc(&e->slots, e->slot_bytes * e->nslots, "thor_enc_create: reconstruction ring")) return g_create_err.code;
  EHIP(hipMemset(e->slots, 0, e->slot_bytes * e->nslots));
  const size_t ncell = (size_t)(W / 4) * (H / 4);
  if (!dev_alloc(&e->cells, ncell * sizeof(TeCell) + 16, "thor_enc_create: cell state")) return g_create_err.code;  // + k_enc_clear's 16-byte rounding
  if (!dev_alloc(&e->cellinfo, ncell * sizeof(uint16_t), "thor_enc_create: cell side info")) return g_create_err.code;
  if (!dev_alloc(&e->sb_words, (size_t)e->nsb * THOR_ENC_SB_WORDS * 4, "thor_enc_create: SB bit strings")) return g_create_err.code;
  if (!dev_alloc(&e->sb_nbits, (size_t)e->nsb * sizeof(int), "thor_enc_create: SB bit counts")) return g_create_err.code;
  if (!dev_alloc(&e->deps, (size_t)e->nsb * sizeof(unsigned), "thor_enc_create: SB dependency counters")) return g_create_err.code;
  if (!dev_alloc(&e->clpf_bits, (size_t)e->nsb_full + 1, "thor_enc_create: CLPF bits")) return g_create_err.code;
  if (!dev_alloc(&e->clpf_flags, (size_t)e->nsb_full + 1, "thor_enc_create: CLPF flags")) return g_create_err.code;
  if (!dev_alloc(&e->es_thr, 2 * 52 * 4 * sizeof(int), "thor_enc_create: early-skip thresholds")) return g_create_err.code;
  if (!dev_alloc(&e->hdr_words, 64 * 4, "thor_enc_create: header words")) return g_create_err.code;
  e->out_cap_words = (int)(((size_t)W * H * 2) / 4 + 1024);  // 16 bits per pixel: far above any real frame
  if (!dev_alloc(&e->out_words, (size_t)e->out_cap_words * 4 + 64, "thor_enc_create: output words")) return g_create_err.code;
  if (!dev_alloc(&e->out_words2, (size_t)e->out_cap_words * 4 + 64, "thor_enc_create: output words (2)")) return g_create_err.code;
  if (!dev_alloc(&e->out_bits, sizeof(int), "thor_enc_create: output bit count")) return g_create_err.code;
  std::vector<int> es(2 * 52 * 4);
  te_es_thresholds(e->p.early_skip_thr, es.data());
  EHIP(hipMemcpy(e->es_thr, es.data(), es.size() * sizeof(int), hipMemcpyHostToDevice));
  return THOR_OK;
}

// Work pools shared by the streams of one launch: one per device, held (its
// mutex) for the whole of a thor_enc_frames call, so concurrent callers on one
// device take turns and callers on different devices never share buffers.
// A pool lives as long as the process (a few MB of scratch per device).
struct EncPool {
  std::mutex mu;
  size_t nwork = 0;
  TeScratchMem *scratch = nullptr;
  unsigned *ticket = nullptr, *err = nullptr;  // ticket: the SB scheduler queue's head and tail
  unsigned *qitems = nullptr;                  // the queue's slots, one per SB of the batch
  size_t qcap = 0;
  TeJob *jobs = nullptr;
  long long *scan = nullptr;
  size_t scan_n = 0;
  // per batch: every context's frame-header words (one upload) and coded-bit
  // counts (one readback), and pinned staging for the coded words (async
  // readbacks, one synchronisation)
  uint32_t *hdr_all = nullptr;
  // per in-flight batch buffer (two): page-locked staging of the jobs and headers (truly
  // asynchronous uploads), the host arena k_enc_pack writes the packed frames into and the
  // (offset, bit count) meta words, and the arena's device allocation counter
  TeJob *jobs_host[2] = {nullptr, nullptr};
  uint32_t *hdr_host[2] = {nullptr, nullptr};
  uint32_t *arena[2] = {nullptr, nullptr};
  size_t arena_words[2] = {0, 0};
  size_t arena_want[2] = {0, 0};
  int *meta[2] = {nullptr, nullptr};
  unsigned long long *arena_ctr = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
  // batches begun and not yet ended (thor_enc_frames_begin / _end), oldest first
  struct Pending {
    std::vector<thor_enc *> es;
    std::vector<int> cur;        // the slot each context coded into
    std::vector<uint32_t *> words;  // the output buffer each context packed into
    std::vector<int> frame_num;
    int buf;                     // jobs_host / hdr_host / arena / meta / ev index
    hipStream_t st;
    // each context's state before the batch (restored when the batch fails)
    struct Snap {
      size_t pos;
      bool first;
      int last_slot, last_frame_num, opar;
      std::vector<int> window;
    };
    std::vector<Snap> snap;
  };
  std::deque<Pending> pending;
};
static std::mutex g_pools_mu;
static std::map<int, EncPool *> g_pools;
static EncPool &pool_for(int device) {
  std::lock_guard<std::mutex> lk(g_pools_mu);
  EncPool *&p = g_pools[device];
  if (!p) p = new EncPool();
  return *p;
}

// A pending batch's contexts back to their state before it (except `skip`,
// a context being destroyed).
static void pending_restore(const EncPool::Pending &q, const thor_enc *skip) {
  for (size_t i = 0; i < q.es.size(); i++) {
    thor_enc *e = q.es[i];
    if (e == skip) continue;
    const EncPool::Pending::Snap &sn = q.snap[i];
    e->pos = sn.pos;
    e->first = sn.first;
    e->last_slot = sn.last_slot;
    e->last_frame_num = sn.last_frame_num;
    e->opar = sn.opar;
    e->slot_of_window = sn.window;
  }
}

// (the caller holds P.mu and has made P's device current)
static int pool_reserve(EncPool &P, size_t nwork, size_t scan_n, size_t nsb_total) {
  if (!P.ticket) {
    EHIP(hipMalloc(&P.ticket, 4096));  // queue heads / tails (TE_QLEVELS: one 128-byte line each)
    EHIP(hipMalloc(&P.err, 64));
    EHIP(hipMemset(P.err, 0, 64));
    EHIP(hipMalloc(&P.jobs, THOR_ENC_MAX_BATCH * sizeof(TeJob)));
    EHIP(hipMalloc(&P.hdr_all, THOR_ENC_MAX_BATCH * 64 * sizeof(uint32_t)));
    EHIP(hipMalloc(&P.arena_ctr, 2 * sizeof(unsigned long long)));
    for (int b = 0; b < 2; b++) {
      EHIP(hipHostMalloc((void **)&P.jobs_host[b], THOR_ENC_MAX_BATCH * sizeof(TeJob), hipHostMallocDefault));
      EHIP(hipHostMalloc((void **)&P.hdr_host[b], THOR_ENC_MAX_BATCH * 64 * sizeof(uint32_t), hipHostMallocDefault));
      EHIP(hipHostMalloc((void **)&P.meta[b], (THOR_ENC_MAX_BATCH * 2 + 2) * sizeof(int), hipHostMallocCoherent | hipHostMallocMapped));
    }
    for (int i = 0; i < 2; i++) EHIP(hipEventCreateWithFlags(&P.ev[i], hipEventDisableTiming));
  }
  if (nwork > P.nwork) {
    if (P.scratch) (void)hipFree(P.scratch);
    P.scratch = nullptr;
    P.nwork = 0;
    EHIP(hipMalloc(&P.scratch, nwork * sizeof(TeScratchMem)));
    P.nwork = nwork;
  }
  if (nsb_total > P.qcap) {
    if (P.qitems) (void)hipFree(P.qitems);
    P.qitems = nullptr;
    P.qcap = 0;
    EHIP(hipMalloc(&P.qitems, nsb_total * sizeof(unsigned)));
    P.qcap = nsb_total;
  }
  if (scan_n > P.scan_n) {
    if (P.scan) (void)hipFree(P.scan);
    P.scan = nullptr;
    P.scan_n = 0;
    EHIP(hipMalloc(&P.scan, scan_n * sizeof(long long)));
    P.scan_n = scan_n;
  }
  return THOR_OK;
}

// diagnostics (thor_enc_debug_stall): the scheduler's wait bound and a row that never releases the next
// thor_enc_debug_stall's settings, read by every thor_enc_frames call: atomics,
// so a call on another thread sees either the old or the new value, never a torn one
static std::atomic<unsigned long long> g_spin_limit{30000000000ULL};  // s_memrealtime ticks (100 MHz): 5 minutes
static std::atomic<int> g_stall_row{-1};
// sequence launches (enc_seq.hip): one in flight on the device? / a context leaving one
static bool ts_active(int device);
static bool ts_member(const thor_enc *e);
static void ts_forget(thor_enc *e);

extern "C" {

void thor_enc_default_params(thor_enc_params_t *p) {
  if (p) te_default_params(p);
}
int thor_enc_check_params(const thor_enc_params_t *p) { return p ? te_check_params(p) : THOR_ERR_ARG; }

thor_enc_t *thor_enc_create(const thor_enc_params_t *p, int device) {
  create_begin();
  if (!p || te_check_params(p) != THOR_OK) {
    create_fail(THOR_ERR_ARG, 0, "thor_enc_create: parameters the device encoder does not support (thor_enc_check_params)");
    return nullptr;
  }
  if (hipSetDevice(device) != hipSuccess) {
    (void)hipGetLastError();
    create_fail(THOR_ERR_ARG, 0, "thor_enc_create: no HIP device %d", device);
    return nullptr;
  }
  thor_enc *e = new thor_enc();
  e->p = *p;
  e->gop = new TeGop(*p);
  e->pos = 0;
  e->device = device;
  e->W = p->width;
  e->H = p->height;
  e->nsbh = (e->W + 63) / 64;
  e->nsbv = (e->H + 63) / 64;
  e->nsb = e->nsbh * e->nsbv;
  e->nsb_full = (e->W / 64) * (e->H / 64);
  e->first = true;
  e->last_slot = -1;
  e->last_frame_num = -1;
  e->slot_of_window.assign(33, -1);
  if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess || enc_alloc(e) != THOR_OK ||
      (p->interp_ref && !(e->ti = thor_ti_create(e->W, e->H, device)))) {
    create_fail(THOR_ERR_HIP, 0, "thor_enc_create: HIP call failed");  // no-op when an allocation said why
    (void)hipGetLastError();
    thor_enc_destroy(e);
    return nullptr;
  }
  e->slot_busy.assign(e->nslots, 0);
  return e;
}

void thor_enc_destroy(thor_enc_t *e) {
  if (!e) return;
  (void)hipSetDevice(e->device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  ts_forget(e);  // a sequence launch in flight with this context: waited for, the context dropped from it
  void *bufs[] = {e->slots,   e->cells,     e->cellinfo, e->sb_words,  e->sb_nbits, e->deps,   e->clpf_bits,
                  e->clpf_flags, e->es_thr, e->hdr_words, e->out_words, e->out_words2, e->out_bits, e->sb_costs,
                  e->sb_words2, e->sb_nbits2, e->clpf_bits2};
  {  // a batch still pending with this context (begun, never ended) is dropped; the
     // batch's other contexts return to their state before it (newest batch first,
     // so a context in two dropped batches ends at the older one's snapshot)
    EncPool &P = pool_for(e->device);
    std::lock_guard<std::mutex> lk(P.mu);
    for (size_t b = P.pending.size(); b-- > 0;) {
      bool has = false;
      for (thor_enc *x : P.pending[b].es) has |= x == e;
      if (has) {
        (void)hipStreamSynchronize(P.pending[b].st);
        pending_restore(P.pending[b], e);
        P.pending.erase(P.pending.begin() + b);
      }
    }
  }
  for (void *b : bufs)
    if (b) (void)hipFree(b);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  if (e->ti) thor_ti_destroy(e->ti);
  delete e->gop;
  delete e;
}

int thor_enc_num_frames(const thor_enc_t *e) { return e ? (int)e->gop->plans.size() : THOR_ERR_ARG; }
// input frame index (display order, after -skip) the next call codes; -1 when done
int thor_enc_next_input(const thor_enc_t *e) {
  if (!e) return THOR_ERR_ARG;
  return e->pos < e->gop->plans.size() ? e->gop->plans[e->pos].input_index : -1;
}
// input frame index of the frame `ahead` frames after the next one in coding order; -1 past the end
int thor_enc_plan_input(const thor_enc_t *e, int ahead) {
  if (!e || ahead < 0) return THOR_ERR_ARG;
  const size_t q = e->pos + (size_t)ahead;
  return q < e->gop->plans.size() ? e->gop->plans[q].input_index : -1;
}
void *thor_enc_stream(thor_enc_t *e) { return e ? (void *)e->stream : nullptr; }
// Re-create the context's stream restricted to a set of CUs
// (hipExtStreamCreateWithCUMask: bit c % 32 of word c / 32 = CU c may run the
// context's kernels).  A scheduling experiment (bench.py --enc-cu-exclude):
// CUs the encoder's persistent row workers cannot hold stay free for
// concurrent decode launches.  The masked stream is a blocking stream (the HIP
// call takes no flags): null-stream copies (thor_h2d / thor_d2h) wait for it.
int thor_enc_set_cu_mask(thor_enc_t *e, const uint32_t *mask, int nwords) {
  if (!e || !mask || nwords <= 0) return THOR_ERR_ARG;
  (void)hipSetDevice(e->device);
  hipStream_t s = nullptr;
  if (hipExtStreamCreateWithCUMask(&s, (uint32_t)nwords, mask) != hipSuccess) {
    (void)hipGetLastError();
    return THOR_ERR_HIP;
  }
  // the old stream drains and goes; on a failure the new one is destroyed and the old one kept
  if (hipStreamSynchronize(e->stream) != hipSuccess || hipStreamDestroy(e->stream) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipStreamDestroy(s);
    return THOR_ERR_HIP;
  }
  e->stream = s;
  return THOR_OK;
}

// One context's frame job.  Its device setup (cells, SB dependency counters,
// scheduler queue: k_enc_clear) runs on the batch stream `st`; its header words go to `hw` (host), which
// the caller uploads with every context's in one copy to `hdr_dev`.
static int enc_prepare(thor_enc *e, const uint8_t *orig, int orig_stride, TeJob &J, TeFramePlan &pl, int &cur_slot,
                       hipStream_t st, uint32_t *hw, uint32_t *hdr_dev) {
  pl = e->gop->plans[e->pos];
  // the frame being coded takes a slot no window entry holds
  std::vector<int> held(e->nslots, 0);
  for (int w = 0; w < 33; w++)
    if (e->slot_of_window[w] >= 0) held[e->slot_of_window[w]] = 1;
  if (e->islot >= 0) held[e->islot] = 1;
  cur_slot = -1;
  for (int s = 0; s < e->nslots && cur_slot < 0; s++)
    if (!held[s]) cur_slot = s;
  if (cur_slot < 0) return THOR_ERR_REF;
  memset(&J, 0, sizeof(J));
  TeFrame &F = J.F;
  const int W = e->W, H = e->H;
  F.oy = orig;
  F.ou = orig + (size_t)orig_stride * H;
  F.ov = F.ou + (size_t)(orig_stride / 2) * (H / 2);
  F.osy = orig_stride;
  F.osc = orig_stride / 2;
  uint8_t *cur = e->slots + (long long)cur_slot * e->slot_bytes;
  F.ry = cur + e->offy;
  F.ru = cur + e->offu;
  F.rv = cur + e->offv;
  F.rsy = e->sy;
  F.rsc = e->sc;
  for (int r = 0; r < pl.num_ref; r++) {
    const int w = pl.ref_array[r];
    int slot;
    if (w < 0) {  // the interpolated reference (encode_block.c: `r >= 0 ? ref[r] : interp_frames[0]`)
      if (!pl.interp_ref || e->islot < 0) return THOR_ERR_REF;
      slot = e->islot;
    } else {
      if (w >= 33 || e->slot_of_window[w] < 0) return THOR_ERR_REF;
      slot = e->slot_of_window[w];
    }
    const uint8_t *rs = e->slots + (long long)slot * e->slot_bytes;
    F.refy[r] = rs + e->offy;
    F.refu[r] = rs + e->offu;
    F.refv[r] = rs + e->offv;
    F.ref_fnum[r] = pl.ref_fnum[r];
  }
  F.cells = e->cells;
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
  const thor_enc_params_t &P = e->p;
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
  F.es_thr = e->es_thr;
  J.sb_words = e->sb_words;
  J.sb_nbits = e->sb_nbits;
  J.deps = e->deps;
  J.clpf_bits = e->clpf_bits;
  J.clpf_flags = e->clpf_flags;
  J.cellinfo = e->cellinfo;
  J.out_words = e->opar ? e->out_words2 : e->out_words;
  J.out_bits = e->out_bits;
  J.nsbh = e->nsbh;
  J.nsbv = e->nsbv;
  J.clpf = P.clpf;
  J.deblock = P.deblocking;
  J.sb_costs = e->sb_costs;
  J.cost_stride = e->cost_stride;
  // header bits (sequence header before the first frame)
  TeHostBits hb;
  if (e->first) te_seq_header(hb, P);
  te_frame_header(hb, pl);
  for (int i = 0; i < 64; i++) hw[i] = 0;
  if (hb.nbits > 64 * 32) return THOR_ERR_ARG;
  for (uint64_t i = 0; i < hb.nbits; i++)
    if (hb.bytes[i >> 3] & (0x80 >> (i & 7))) hw[i >> 5] |= 0x80000000u >> (i & 31);
  J.hdr_bits = (int)hb.nbits;
  J.hdr_words = hdr_dev;
  return THOR_OK;  // the cells, SB dependency counters and queue are set up by k_enc_clear (one launch for the batch)
}

static thor_yuv_planes_t enc_slot_planes(const thor_enc *e, int slot) {
  uint8_t *b = e->slots + (long long)slot * e->slot_bytes;
  return thor_yuv_planes_t{b + e->offy, b + e->offu, b + e->offv, e->sy, e->sc};
}

// The frame's interpolated reference into the interpolation slot, on the
// context's stream: interpolate_frames + pad_yuv_frame (enc/mainenc.c:328-330,
// :385-387), the decoder's kernels (tme.hip, k_pad).
static int enc_interp(thor_enc *e, const TeFramePlan &pl) {
  const int a = pl.interp_a, b = pl.interp_b;
  if (!e->ti || e->islot < 0 || a < 0 || a >= 33 || b < 0 || b >= 33 || e->slot_of_window[a] < 0 ||
      e->slot_of_window[b] < 0)
    return THOR_ERR_REF;
  const thor_yuv_planes_t ra = enc_slot_planes(e, e->slot_of_window[a]), rb = enc_slot_planes(e, e->slot_of_window[b]);
  const thor_yuv_planes_t o = enc_slot_planes(e, e->islot);
  const int rc = thor_interpolate_frames(e->ti, &ra, &rb, THOR_PAD_Y, &o, pl.interp_ratio, pl.interp_pos, e->stream);
  if (rc != THOR_OK) return rc;
  FrameBatch fb;
  memset(&fb, 0, sizeof(fb));
  fb.f[0].cy = o.y;
  fb.f[0].cu = o.u;
  fb.f[0].cv = o.v;
  fb.f[0].sy = e->sy;
  fb.f[0].sc = e->sc;
  fb.f[0].W = e->W;
  fb.f[0].H = e->H;
  k_pad<<<dim3((pad_chunks(e->W, e->H) + 255) / 256, 1), 256, 0, e->stream>>>(fb, 0, 0);
  EHIP(hipGetLastError());
  return THOR_OK;
}

// Encode the next frame (coding order) of each of `n` contexts with one
// launch per stage, in two halves: thor_enc_frames_begin enqueues every stage
// of the batch (RD loop, loop filters, CLPF decision, bit packing, the bit
// counts' readback) and advances the contexts' host state (GOP position,
// reference window) without waiting; thor_enc_frames_end waits for the oldest
// batch begun, reads its coded words back and makes them the contexts' chunks
// (thor_enc_frame_bytes).  Up to two batches may be in flight, so a caller can
// begin frame i + 1 before ending frame i: the device codes the next frame
// while the host collects the last one.  orig[i]: DEVICE pointer to context i's
// input frame thor_enc_next_input(es[i]) as planar I420 (luma stride
// orig_stride[i], chroma stride / 2).  All contexts must share device and frame
// size.  thor_enc_frames = begin + end.
static int frames_args_ok(thor_enc_t *const *es, int n, const uint8_t *const *orig) {
  if (!es || !orig || n <= 0 || n > THOR_ENC_MAX_BATCH) return THOR_ERR_ARG;
  thor_enc *lead = es[0];
  for (int i = 0; i < n; i++) {
    if (!es[i] || !orig[i] || es[i]->device != lead->device || es[i]->W != lead->W || es[i]->H != lead->H)
      return THOR_ERR_ARG;
    for (int j = 0; j < i; j++)
      if (es[j] == es[i]) return THOR_ERR_ARG;
  }
  return THOR_OK;
}

// thor_enc_frames_begin with P.mu held and the device current.
static int frames_begin_locked(EncPool &P, thor_enc_t *const *es, int n, const uint8_t *const *orig,
                               const int *orig_stride) {
  thor_enc *lead = es[0];
  for (int i = 0; i < n; i++)
    if (es[i]->pos >= es[i]->gop->plans.size()) return THOR_ERR_ARG;
  const int W = lead->W, H = lead->H;
  const int nrows = lead->nsbv;
  const int nwork = n * nrows;
  if (P.pending.size() >= 2) return THOR_ERR_ARG;  // end the oldest batch first
  if (ts_active(lead->device)) return THOR_ERR_ARG;  // a sequence launch holds the pool's workers
  for (const EncPool::Pending &q : P.pending)
    for (thor_enc *x : q.es)
      for (int i = 0; i < n; i++)
        if (x == es[i] && q.st != lead->stream) return THOR_ERR_ARG;  // a context's frames stay on one batch stream
  int rc = pool_reserve(P, (size_t)(nwork < TE_MAX_WORKERS ? nwork : TE_MAX_WORKERS), (size_t)n * (lead->nsb + 1),
                        (size_t)n * lead->nsb);
  if (rc != THOR_OK) return rc;
  hipStream_t st = lead->stream;
  // the pool's workers and scratch are shared: a batch on another stream first waits for the pending ones
  for (const EncPool::Pending &q : P.pending)
    if (q.st != st) EHIP(hipStreamSynchronize(q.st));
  std::vector<TeJob> jobs(n);
  std::vector<TeFramePlan> plans(n);
  std::vector<int> cur(n);
  // the buffer set no pending batch holds (at most one is pending here)
  int buf = 0;
  for (const EncPool::Pending &q : P.pending)
    if (q.buf == 0) buf = 1;
  uint32_t *hdr = P.hdr_host[buf];
  for (int i = 0; i < n; i++) {
    thor_enc *e = es[i];
    if (e->stream != st) {  // the members' earlier work on their own streams comes first
      EHIP(hipStreamSynchronize(e->stream));
    }
    const int s = orig_stride ? orig_stride[i] : W;
    if ((rc = enc_prepare(e, orig[i], s, jobs[i], plans[i], cur[i], st, hdr + (size_t)i * 64, P.hdr_all + i * 64)) !=
        THOR_OK)
      return rc;
  }
  EHIP(hipMemcpyAsync(P.hdr_all, hdr, (size_t)n * 64 * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  // interpolated references: each context's on its own stream (they overlap), all done before the RD loop;
  // each after every pending batch (their loop filters still write the slots the interpolation reads,
  // their RD loops may still read the interpolation slot it overwrites)
  bool any_interp = false;
  for (int i = 0; i < n; i++)
    if (plans[i].interp_ref) {
      for (const EncPool::Pending &q : P.pending)
        if (q.st != es[i]->stream) EHIP(hipStreamWaitEvent(es[i]->stream, P.ev[q.buf], 0));
      if ((rc = enc_interp(es[i], plans[i])) != THOR_OK) return rc;
      any_interp = true;
    }
  if (any_interp)
    for (int i = 0; i < n; i++)
      if (plans[i].interp_ref) {
        EHIP(hipStreamSynchronize(es[i]->stream));
        if ((rc = thor_ti_status(es[i]->ti)) != THOR_OK) return rc;
      }
  for (int i = 0; i < n; i++) jobs[i].qbase = n + i * (lead->nsb - 1);  // slots [n, n * nsb): empty
  memcpy(P.jobs_host[buf], jobs.data(), n * sizeof(TeJob));
  EHIP(hipMemcpyAsync(P.jobs, P.jobs_host[buf], n * sizeof(TeJob), hipMemcpyHostToDevice, st));
  {  // the host arena: room for every frame of the batch at W*H/16 bytes (grown after an overflow)
    size_t want = (size_t)n * (((size_t)W * H / 16) / 4 + 1024);
    if (P.arena_want[buf] > want) want = P.arena_want[buf];
    if (want > P.arena_words[buf]) {
      if (P.arena[buf]) (void)hipHostFree(P.arena[buf]);
      P.arena[buf] = nullptr;
      P.arena_words[buf] = 0;
      EHIP(hipHostMalloc((void **)&P.arena[buf], want * 4 + 64, hipHostMallocCoherent | hipHostMallocMapped));
      P.arena_words[buf] = want;
    }
  }
  {
    const long long cb = (long long)(W / 4) * (H / 4) * (long long)sizeof(TeCell);
    static_assert(sizeof(TeCell) % 4 == 0, "cells clear as words");
    const long long n16 = (cb + 15) / 16;
    const int gx = (int)((n16 + 255) / 256 < 1024 ? (n16 + 255) / 256 : 1024);
    k_enc_clear<<<dim3(gx > 0 ? gx : 1, n), 256, 0, st>>>(P.jobs, ((cb + 15) / 16) * 16, P.ticket, P.qitems,
                                                        P.arena_ctr + buf);
    EHIP(hipGetLastError());
  }
  // the queue's priority levels (TE_QLEVELS > 1): level v holds the SBs of rows k with k * L / nsbv == v,
  // its slots after the lower levels'; level 0 starts with every job's SB (0, 0)
  TeQLevels QL;
  memset(&QL, 0, sizeof(QL));
  {
    unsigned o = 0;
    for (int v = 0; v < TE_QLEVELS; v++) {
      int rows = 0;
      for (int k = 0; k < lead->nsbv; k++) rows += k * TE_QLEVELS / lead->nsbv == v;
      QL.off[v] = o;
      QL.cap[v] = (unsigned)(n * rows * lead->nsbh);
      o += QL.cap[v];
    }
  }
  // persistent workers take SBs from the queue until every slot is taken:
  // more workgroups than the chip holds at once (two per SIMD at this kernel's
  // register and LDS use) would only start as the first ones run out of work
  k_enc_rows<<<nwork < TE_MAX_WORKERS ? nwork : TE_MAX_WORKERS, 64, 0, st>>>(
      P.jobs, (unsigned)(n * lead->nsb), P.ticket, P.qitems, P.scratch, P.err, g_spin_limit.load(), g_stall_row.load(), QL);
  EHIP(hipGetLastError());
  // loop filters of every job, one launch per pass (the cell words came from k_enc_rows itself)
  {
    const int nv = ((W >> 3) - 1) * (H >> 3), nh = (W >> 3) * ((H >> 3) - 1);
    const int bv = (nv + 256 * DB_ITEMS - 1) / (256 * DB_ITEMS), bh = (nh + 256 * DB_ITEMS - 1) / (256 * DB_ITEMS);
    k_enc_db_v<<<dim3(3 * bv, n), 256, 0, st>>>(P.jobs, bv);
    k_enc_db_h<<<dim3(3 * bh, n), 256, 0, st>>>(P.jobs, bh);
    EHIP(hipGetLastError());
  }
  if (lead->nsb_full > 0) {
    k_enc_clpf<<<dim3(lead->nsb_full, n), 64, 0, st>>>(P.jobs);
    EHIP(hipGetLastError());
  }
  k_enc_pad<<<dim3((pad_chunks(W, H) + 255) / 256, n), 256, 0, st>>>(P.jobs);
  EHIP(hipGetLastError());
  // the packed frames straight into the host arena, their sizes into the meta words; an event behind
  k_enc_pack<<<n, 256, 0, st>>>(P.jobs, P.scan, lead->out_cap_words, P.arena[buf], P.arena_words[buf],
                                P.arena_ctr + buf, P.meta[buf], P.err);
  EHIP(hipGetLastError());
  EHIP(hipEventRecord(P.ev[buf], st));
  // the batch is in flight: advance every context (the next plan, the reference window)
  EncPool::Pending q;
  q.buf = buf;
  q.st = st;
  for (int i = 0; i < n; i++) {
    thor_enc *e = es[i];
    q.snap.push_back({e->pos, e->first, e->last_slot, e->last_frame_num, e->opar, e->slot_of_window});
    q.es.push_back(e);
    q.cur.push_back(cur[i]);
    q.words.push_back(e->opar ? e->out_words2 : e->out_words);
    q.frame_num.push_back(plans[i].frame_num);
    // slide the window: the frame shifted out of ref[32] frees its slot
    for (int r = 32; r > 0; r--) e->slot_of_window[r] = e->slot_of_window[r - 1];
    e->slot_of_window[0] = cur[i];
    e->last_slot = cur[i];
    e->last_frame_num = plans[i].frame_num;
    e->first = false;
    e->pos++;
    e->opar ^= 1;
  }
  P.pending.push_back(std::move(q));
  return THOR_OK;
}

int thor_enc_frames_begin(thor_enc_t *const *es, int n, const uint8_t *const *orig, const int *orig_stride) {
  int rc = frames_args_ok(es, n, orig);
  if (rc != THOR_OK) return rc;
  EHIP(hipSetDevice(es[0]->device));
  EncPool &P = pool_for(es[0]->device);
  std::lock_guard<std::mutex> pool_lock(P.mu);
  return frames_begin_locked(P, es, n, orig, orig_stride);
}

// thor_enc_frames_end with P.mu held and the device current: the oldest pending
// batch of exactly these contexts (es / n as passed to its begin).  On a device
// error (e.g. a WPP wait that gave up) every pending batch is dropped and the
// contexts return to their state before the failed one: that frame can be
// coded again.
static int frames_end_locked(EncPool &P, thor_enc_t *const *es, int n) {
  size_t qi = 0;
  for (; qi < P.pending.size(); qi++) {
    const EncPool::Pending &c = P.pending[qi];
    bool same = (int)c.es.size() == n;
    for (int i = 0; same && i < n; i++) same = c.es[i] == es[i];
    if (same) break;
  }
  if (qi == P.pending.size()) return THOR_ERR_ARG;
  EncPool::Pending q = std::move(P.pending[qi]);
  P.pending.erase(P.pending.begin() + qi);
  hipStream_t st = q.st;
  EHIP(hipEventSynchronize(P.ev[q.buf]));
  // k_enc_pack left (arena offset, bit count) per context and the error flags in page-locked memory
  const volatile int *meta = P.meta[q.buf];
  const unsigned err = (unsigned)meta[2 * THOR_ENC_MAX_BATCH];
  bool bad = err != 0;
  for (int i = 0; i < n && !bad; i++) bad = meta[2 * i + 1] < 0;
  if (bad) {  // drop what is in flight, restore the contexts to before this batch (and the other pending ones)
    EHIP(hipStreamSynchronize(st));
    for (const EncPool::Pending &r : P.pending) EHIP(hipStreamSynchronize(r.st));
    std::deque<EncPool::Pending> later;
    later.swap(P.pending);
    // newest first, so a context in several batches ends at its oldest snapshot (q was at index qi)
    for (size_t b = later.size(); b-- > qi;) pending_restore(later[b], nullptr);
    pending_restore(q, nullptr);
    for (size_t b = qi; b-- > 0;) pending_restore(later[b], nullptr);
    if (err) {
      fprintf(stderr, "thor_amd enc: device error flags 0x%x\n", err);
      EHIP(hipMemset(P.err, 0, 4));
      return THOR_ERR_HIP;
    }
    return THOR_ERR_NOMEM;  // a frame over the output buffer
  }
  const uint8_t *arena = (const uint8_t *)P.arena[q.buf];
  std::vector<uint32_t> tmp;
  for (int i = 0; i < n; i++) {
    thor_enc *e = q.es[i];
    const int off = meta[2 * i];
    const size_t nb = ((size_t)meta[2 * i + 1] + 7) / 8;
    e->chunk.resize(4 + nb);
    e->chunk[0] = (uint8_t)(nb >> 24);
    e->chunk[1] = (uint8_t)(nb >> 16);
    e->chunk[2] = (uint8_t)(nb >> 8);
    e->chunk[3] = (uint8_t)nb;
    if (off >= 0) {  // the stream's bytes, already in order
      memcpy(e->chunk.data() + 4, arena + (size_t)off * 4, nb);
    } else {  // the arena was full: this frame's words from device memory; a larger arena next time
      tmp.resize((nb + 3) / 4);
      EHIP(hipMemcpy(tmp.data(), q.words[i], tmp.size() * 4, hipMemcpyDeviceToHost));
      for (size_t b = 0; b < nb; b++) e->chunk[4 + b] = (uint8_t)(tmp[b >> 2] >> (24 - 8 * (b & 3)));
      P.arena_want[q.buf] = 2 * P.arena_words[q.buf];
    }
  }
  return THOR_OK;
}

int thor_enc_frames_end(thor_enc_t *const *es, int n) {
  if (!es || n <= 0 || !es[0]) return THOR_ERR_ARG;
  EHIP(hipSetDevice(es[0]->device));
  EncPool &P = pool_for(es[0]->device);
  std::lock_guard<std::mutex> pool_lock(P.mu);
  return frames_end_locked(P, es, n);
}

// begin + end under one hold of the pool lock: a concurrent call on another
// thread cannot interleave its batch between this call's two halves.
int thor_enc_frames(thor_enc_t *const *es, int n, const uint8_t *const *orig, const int *orig_stride) {
  int rc = frames_args_ok(es, n, orig);
  if (rc != THOR_OK) return rc;
  EHIP(hipSetDevice(es[0]->device));
  EncPool &P = pool_for(es[0]->device);
  std::lock_guard<std::mutex> pool_lock(P.mu);
  if ((rc = frames_begin_locked(P, es, n, orig, orig_stride)) != THOR_OK) return rc;
  return frames_end_locked(P, es, n);
}

int thor_enc_reset(thor_enc_t *e) {
  if (!e || ts_member(e)) return THOR_ERR_ARG;
  {  // not with a batch begun and not ended
    EncPool &P = pool_for(e->device);
    std::lock_guard<std::mutex> lk(P.mu);
    for (const EncPool::Pending &q : P.pending)
      for (thor_enc *x : q.es)
        if (x == e) return THOR_ERR_ARG;
  }
  EHIP(hipSetDevice(e->device));
  EHIP(hipStreamSynchronize(e->stream));
  e->pos = 0;
  e->first = true;
  e->last_slot = -1;
  e->last_frame_num = -1;
  e->slot_of_window.assign(33, -1);
  e->chunk.clear();
  return THOR_OK;
}

// Diagnostics: superblock row `row` of every stream never releases the row
// below (-1: off) and a worker's wait for its next SB gives up after `spin_ms`
// (<= 0: the 5-minute default), so the bounded-time failure path can be exercised.
int thor_enc_debug_stall(int row, int spin_ms) {
  g_stall_row.store(row);
  g_spin_limit.store(spin_ms > 0 ? (unsigned long long)spin_ms * 100000ULL : 30000000000ULL);
  return THOR_OK;
}

// k_enc_rows' profile since the last call, summed over its workers (100 MHz ticks): time coding
// SBs, time waiting for a queue slot, SBs coded; cleared.  Returns 3.
int thor_enc_rows_profile(int device, long long *out) {
  unsigned long long v[4] = {0, 0, 0, 0};
  EHIP(hipSetDevice(device));
  EHIP(hipDeviceSynchronize());
  EHIP(hipMemcpyFromSymbol(v, HIP_SYMBOL(g_te_rows_prof), sizeof(v)));
  const unsigned long long z[4] = {0, 0, 0, 0};
  EHIP(hipMemcpyToSymbol(HIP_SYMBOL(g_te_rows_prof), z, sizeof(z)));
  for (int i = 0; out && i < 3; i++) out[i] = (long long)v[i];
  return 3;
}

int thor_enc_frame(thor_enc_t *e, const uint8_t *orig, int orig_stride) {
  return thor_enc_frames(&e, 1, &orig, &orig_stride);
}

// Bytes of the frame the last thor_enc_frame(s) call coded: the .bit chunk
// (4-byte big-endian length + payload, enc/putbits.c:57-95).  Returns the
// chunk size; copies min(size, cap) bytes when dst is non-NULL.
long long thor_enc_frame_bytes(const thor_enc_t *e, uint8_t *dst, size_t cap) {
  if (!e) return THOR_ERR_ARG;
  if (dst) memcpy(dst, e->chunk.data(), e->chunk.size() < cap ? e->chunk.size() : cap);
  return (long long)e->chunk.size();
}

// Per-superblock RD costs (parity instrumentation): from the next frame on,
// every SB's top-level process_block costs go to a device buffer (on = 1).
int thor_enc_record_sb_costs(thor_enc_t *e, int on) {
  if (!e) return THOR_ERR_ARG;
  EHIP(hipSetDevice(e->device));
  EHIP(hipStreamSynchronize(e->stream));
  if (!on) {
    if (e->sb_costs) EHIP(hipFree(e->sb_costs));
    e->sb_costs = nullptr;
    return THOR_OK;
  }
  if (e->sb_costs) return THOR_OK;
  // encode_frame's trial loop (enc/encode_frame.c:133): qp - d .. qp + d in steps of delta_qp_step
  const int d = e->p.max_delta_qp, step = e->p.delta_qp_step > 0 ? e->p.delta_qp_step : 1;
  e->cost_stride = (d ? (2 * d) / step + 1 : 0) + 1;
  EHIP(hipMalloc(&e->sb_costs, (size_t)e->nsb * e->cost_stride * sizeof(int32_t)));
  EHIP(hipMemset(e->sb_costs, 0, (size_t)e->nsb * e->cost_stride * sizeof(int32_t)));
  return THOR_OK;
}

// The last ended frame's per-SB costs (raster SB order, cost_stride int32 per
// SB: the delta-QP trials in order, then the final encode).  Returns the count
// (nsb x per_sb), copies min(count, cap); *per_sb = cost_stride.
long long thor_enc_sb_costs(thor_enc_t *e, int32_t *dst, size_t cap, int *per_sb) {
  if (!e || !e->sb_costs) return THOR_ERR_ARG;
  const size_t n = (size_t)e->nsb * e->cost_stride;
  if (per_sb) *per_sb = e->cost_stride;
  if (dst && cap) {
    EHIP(hipSetDevice(e->device));
    EHIP(hipDeviceSynchronize());
    EHIP(hipMemcpy(dst, e->sb_costs, (n < cap ? n : cap) * sizeof(int32_t), hipMemcpyDeviceToHost));
  }
  return (long long)n;
}

// The reconstruction of the last coded frame (deblocked, CLPF'd), host planes.
int thor_enc_read_recon(thor_enc_t *e, uint8_t *y, uint8_t *u, uint8_t *v) {
  if (!e || e->last_slot < 0) return THOR_ERR_ARG;
  EHIP(hipSetDevice(e->device));
  EHIP(hipStreamSynchronize(e->stream));
  const uint8_t *b = e->slots + (long long)e->last_slot * e->slot_bytes;
  if (y) EHIP(hipMemcpy2D(y, e->W, b + e->offy, e->sy, e->W, e->H, hipMemcpyDeviceToHost));
  if (u) EHIP(hipMemcpy2D(u, e->W / 2, b + e->offu, e->sc, e->W / 2, e->H / 2, hipMemcpyDeviceToHost));
  if (v) EHIP(hipMemcpy2D(v, e->W / 2, b + e->offv, e->sc, e->W / 2, e->H / 2, hipMemcpyDeviceToHost));
  return THOR_OK;
}

}  // extern "C"

#if defined(THOR_ENC_TRACE)
// debug builds only (tools/enc_trace.py): record the RD decision trace of frame
// `frame` into dev_buf (int [8 + 8 * cap], dev_buf[0] = record count)
extern "C" int thor_enc_trace_buffer(void *dev_buf, unsigned cap, int frame) {
  if (hipMemcpyToSymbol(HIP_SYMBOL(te_trace_buf), &dev_buf, sizeof(void *)) != hipSuccess) return THOR_ERR_HIP;
  if (hipMemcpyToSymbol(HIP_SYMBOL(te_trace_cap), &cap, sizeof(cap)) != hipSuccess) return THOR_ERR_HIP;
  if (hipMemcpyToSymbol(HIP_SYMBOL(te_trace_frame), &frame, sizeof(frame)) != hipSuccess) return THOR_ERR_HIP;
  return THOR_OK;
}
#endif

#if defined(THOR_ENC_PROFILE)
extern "C" int thor_enc_profile_buffer(void *dev_buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(te_prof_buf), &dev_buf, sizeof(void *)) == hipSuccess ? THOR_OK : THOR_ERR_HIP;
}
#endif
