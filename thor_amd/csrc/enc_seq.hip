// Sequence launch of the device-resident encoder (include/thor_amd.h,
// thor_enc_seq_*): every frame of a batch of streams in ONE persistent launch.
//
// The per-frame batch (thor_enc_frames, enc.hip) codes frame f of every stream,
// then filters and packs it, then starts frame f + 1: each P frame costs one
// stream's whole SB dependency chain (126 wavefront steps at 4K) with most of
// the machine idle, and the I-frame batch cannot overlap them.
// Here the frame boundary is a dependency like any other: the work of a frame
// is split into tasks on the SB scheduler's queues, and frame f + 1 of a stream
// starts as soon as ITS frame f is a finished reference, whatever the other
// streams are doing -- stream A's P chain runs while stream B's I frame fills
// the workers.  Tasks of frame f of stream s (one wave each):
//   FETCH(k)  the input rows of SB row k, host (page-locked) -> HBM: the raw
//             frame upload inside the launch, one frame ahead of the RD loop
//             (the blit copies of a separate H2D would need CU slots the
//             persistent workers hold)
//   RD(k, l)  te_encode_sb of SB (k, l) (enc/encode_frame.c:112-147) + its
//             cells' loop-filter words; ready when (k, l - 1) and
//             (k - 1, l + 1) are done (enc.hip's scheduler rule) and, for
//             (0, 0), when the inputs are in, frame f - 1 is a finished
//             reference and frame f - 2's bits are packed (its SB buffers free)
//   DBV(k)    vertical luma + chroma edges of the 8-row groups of SB row k
//             (deblock_frame_y / _uv, common/common_frame.c:46-321): after RD
//             of rows k and k + 1 (row k + 1's intra prediction reads row k's
//             last pixel row unfiltered)
//   DBH(k)    horizontal edges at luma rows [64k, 64k + 56]: after DBV(k - 1),
//             DBV(k) (the reference filters every vertical edge first)
//   FIN(k)    CLPF decision + CLPF of the full SBs of row k
//             (enc/encode_frame.c:50-63, common/common_frame.c:485-557), the
//             row's padding (pad_yuv_frame, :405-462), its cell state cleared
//             for the next frame (enc/encode_frame.c:74): after DBH(k), DBH(k+1)
//   PACK      the frame's bit string (header | SBs | CLPF bits; putbits /
//             flush_all_bits, enc/putbits.c:57-129) -> page-locked host memory,
//             then its size, so the host can parse it while the launch runs
// A frame is a finished reference when its FIN tasks are done.  Queues: one
// FIFO per priority class (stream s -> class s * 16 / n); a worker takes the
// oldest ready task of the highest class, so the first streams run their whole
// chains ahead and the last ones fill the idle capacity.
// (unity build: follows enc.hip in libthor_amd.hip)

#define TS_NCLS 16
#define TS_MAX_JOBS 4096          // 12 bits of a queue item
#define TS_MAX_SB (1 << 17)       // 17 bits: SB index within a frame
#define TS_CTL_WORDS (TS_NCLS * 64 + 512)
enum { TS_RD = 0, TS_FETCH = 1, TS_DBV = 2, TS_DBH = 3, TS_FIN = 4, TS_PACK = 5 };
// control words (device): class c's head at [c * 64], tail at [c * 64 + 32]
// (separate 128-byte lines), then the launch's counters
#define TS_HEAD(c) ((c)*64)
#define TS_TAIL(c) ((c)*64 + 32)
#define TS_NDONE (TS_NCLS * 64)
#define TS_ALIVE (TS_NCLS * 64 + 32)
#define TS_ARENA (TS_NCLS * 64 + 64)
#define TS_IDONE (TS_NCLS * 64 + 96)
#define TS_RETIRED (TS_NCLS * 64 + 128)
// per-launch profile (64-bit sums over the workers, added once per worker at its exit):
// [t] ticks and [t + 6] count per task type, then idle ticks, claim waits, failed claims
#define TS_PROF (TS_NCLS * 64 + 192)
#define TS_NPROF 15

struct TsJob {
  TeJob J;                   // J.deps: the frame's SB counters; J.sb_words / sb_nbits / clpf_bits: the frame parity's
  unsigned *dbh, *fin, *done;  // DBH(k) / FIN(k) counters [nsbv], frame-done counter
  const uint8_t *src;        // FETCH source (host), nullptr: the input is resident at dst
  uint8_t *dst;              // the input frame in HBM (I420, stride W)
  int next, next2;           // this stream's jobs for frames f + 1, f + 2 (-1: none)
  int cls, aux, need0, is_i;  // queue class of the job's RD tasks / of its other tasks
  uint8_t *cy, *cu, *cv;     // the reconstruction (loop filters, padding)
  int sy, sc, qp, qpc, deblock;
};
struct TsArgs {
  const TsJob *jobs;
  TeScratchMem *scratch;
  unsigned *ctl, *items, *err;
  unsigned qoff[TS_NCLS];
  unsigned qtot[TS_NCLS];    // tasks of each class (ticket claims past it find nothing)
  int ncls;                  // classes in use (stream i -> class i * ncls / n)
  int claim;                 // 0: compare-and-swap claims (never block), 1: tickets (a claim may wait for its slot)
  unsigned total;            // tasks of the launch
  unsigned n_ijobs;          // I-frame jobs (idle workers may retire once they are all done)
  int min_alive;
  unsigned long long spin_limit, retire_ticks;
  uint32_t *arena;           // host, page-locked: the packed frames
  unsigned long long arena_words;
  int *meta;                 // host: [job][2] = word offset in the arena, bit count (-1 until final)
  int out_cap_words;
};

__host__ __device__ inline unsigned ts_item(int job, int type, int idx) {
  return (unsigned)job << 20 | (unsigned)type << 17 | (unsigned)idx;
}
// (lane 0) queue a ready task in its job's class
__device__ __forceinline__ void ts_push(const TsArgs &A, int cls, unsigned item) {
  const unsigned slot = __hip_atomic_fetch_add(&A.ctl[TS_TAIL(cls)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&A.items[A.qoff[cls] + slot], item, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// (lane 0) one more finished dependency of a task; queue it when that was its last
__device__ __forceinline__ void ts_dep(const TsArgs &A, unsigned *cnt, unsigned need, int cls, unsigned item) {
  const unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (old + 1 == need) ts_push(A, cls, item);
}
// (lane 0) the oldest ready task of the highest class with one, TE_Q_EMPTY if none.
// claim 0: a slot below the tail is taken by compare-and-swap on the head
// (never waits; contended when many idle workers race for one item);
// claim 1: a ticket (one fetch-and-add) as soon as the class looks non-empty --
// a ticket past the items pushed so far waits for its slot (every slot below
// the class's task count fills: its tasks depend only on its own), one past
// the class's task count is dropped.
__device__ __forceinline__ unsigned ts_pop(const TsArgs &A, unsigned long long &fails, unsigned long long &waits) {
  for (int c = 0; c < A.ncls; c++) {
    unsigned h = te_ld_relaxed(&A.ctl[TS_HEAD(c)]);
    if (A.claim) {
      if (h >= A.qtot[c] || h >= te_ld_relaxed(&A.ctl[TS_TAIL(c)])) continue;
      h = __hip_atomic_fetch_add(&A.ctl[TS_HEAD(c)], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (h >= A.qtot[c]) continue;
    } else {
      bool got = false;
      for (;;) {
        const unsigned t = te_ld_relaxed(&A.ctl[TS_TAIL(c)]);
        if (h >= t) break;
        if (__hip_atomic_compare_exchange_strong(&A.ctl[TS_HEAD(c)], &h, h + 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)) {
          got = true;
          break;
        }
        fails++;  // h now holds the head another worker moved it to
      }
      if (!got) continue;
    }
    unsigned item;
    const unsigned long long w0 = __builtin_amdgcn_s_memrealtime();
    while ((item = te_ld_relaxed(&A.items[A.qoff[c] + h])) == TE_Q_EMPTY) __builtin_amdgcn_s_sleep(4);
    waits += __builtin_amdgcn_s_memrealtime() - w0;
    return item;
  }
  return TE_Q_EMPTY;
}

// FETCH: bytes [a, b) of the I420 frame, host -> HBM, 16 bytes per lane access,
// eight in flight (the host reads cross PCIe: latency bound per wave).
__device__ void ts_copy_range(uint8_t *dst, const uint8_t *src, long long a, long long b) {
  const int lane = threadIdx.x;
  if (((a | b | (long long)(uintptr_t)dst | (long long)(uintptr_t)src) & 15) == 0) {
    const uint4 *s = (const uint4 *)(src + a);
    uint4 *d = (uint4 *)(dst + a);
    const long long n = (b - a) >> 4;
    long long i = lane;
    for (; i + 7 * 64 < n; i += 8 * 64) {
      uint4 v[8];
#pragma unroll
      for (int q = 0; q < 8; q++) v[q] = s[i + q * 64];
#pragma unroll
      for (int q = 0; q < 8; q++) d[i + q * 64] = v[q];
    }
    for (; i < n; i += 64) d[i] = s[i];
  } else {
    for (long long i = a + lane; i < b; i += 64) dst[i] = src[i];
  }
}

// The tasks other than RD (FETCH, DBV, DBH, FIN, PACK), out of line: k_enc_seq's
// RD path keeps the register allocation k_enc_rows has (the task bodies inlined
// beside te_encode_sb cost the P-frame SBs a third more time).
__device__ __noinline__ void ts_aux(const TsArgs &A, int j, int type, int idx) {
  const int lane = threadIdx.x;
  const TsJob &T = A.jobs[j];
  const TeJob &J = T.J;
  const int W = J.F.W, H = J.F.H, nsbh = J.nsbh, nsbv = J.nsbv;
  (void)nsbh;
  if (type == TS_FETCH) {
    const int k = idx;
    const long long ys = (long long)W * H, cw = W >> 1;
    const long long y0 = (long long)(k * 64) * W, y1 = (long long)min(k * 64 + 64, H) * W;
    const long long c0 = (long long)(k * 32) * cw, c1 = (long long)min(k * 32 + 32, H >> 1) * cw;
    ts_copy_range(T.dst, T.src, y0, y1);
    ts_copy_range(T.dst, T.src, ys + c0, ys + c1);
    ts_copy_range(T.dst, T.src, ys + ys / 4 + c0, ys + ys / 4 + c1);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) ts_dep(A, &J.deps[0], (unsigned)T.need0, T.cls, ts_item(j, TS_RD, 0));
  } else if (type == TS_DBV) {
    const int k = idx;
    if (T.deblock) {
      const int ne = (W >> 3) - 1, g0 = k * 8, g1 = min(k * 8 + 8, H >> 3);
      for (int b = g0 * ne; b < g1 * ne; b += 64 * DB_ITEMS)
        luma_v_items<DB_ITEMS>(b + lane, 64, T.cy, T.sy, W, H, J.cellinfo, T.qp, g0, g1);
      for (int t = g0 * ne + lane; t < g1 * ne; t += 64)
        for (int pl = 0; pl < 2; pl++)
          k_deblock_chroma_v_body(t, pl, T.cu, T.cv, T.sc, W, H, J.cellinfo, T.qpc, g0, g1);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
      ts_dep(A, &T.dbh[k], 1u + (k > 0), T.aux, ts_item(j, TS_DBH, k));
      if (k + 1 < nsbv) ts_dep(A, &T.dbh[k + 1], 2u, T.aux, ts_item(j, TS_DBH, k + 1));
    }
  } else if (type == TS_DBH) {
    const int k = idx;
    if (T.deblock) {
      // edges at luma rows i = (kk + 1) * 8 in [64k, 64k + 56]
      const int ng = W >> 3, kk0 = k * 8 - 1 < 0 ? 0 : k * 8 - 1, kk1 = min(k * 8 + 7, (H >> 3) - 1);
      const int i0 = k * 64, i1 = k * 64 + 56;
      for (int b = kk0 * ng; b < kk1 * ng; b += 64 * DB_ITEMS)
        luma_h_items<DB_ITEMS>(b + lane, 64, T.cy, T.sy, W, H, J.cellinfo, T.qp, i0, i1);
      for (int t = kk0 * ng + lane; t < kk1 * ng; t += 64)
        for (int pl = 0; pl < 2; pl++)
          k_deblock_chroma_h_body(t, pl, T.cu, T.cv, T.sc, W, H, J.cellinfo, T.qpc, i0, i1);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
      if (k > 0) ts_dep(A, &T.fin[k - 1], 2u, T.aux, ts_item(j, TS_FIN, k - 1));
      ts_dep(A, &T.fin[k], 1u + (k + 1 < nsbv), T.aux, ts_item(j, TS_FIN, k));
    }
  } else if (type == TS_FIN) {
    const int k = idx;
    if (J.clpf && k < (H >> 6)) {
      for (int l = 0; l < (W >> 6); l++) {
        const int d = te_clpf_decide_blk(J.cellinfo, W, J.F.ry, J.F.rsy, J.F.oy, J.F.osy, k, l);
        if (lane == 0) J.clpf_bits[k * (W >> 6) + l] = (int8_t)d;
        if (d == 1) te_clpf_apply_blk(J.cellinfo, W, T.cy, T.sy, T.cu, T.cv, T.sc, k, l);
      }
    }
    te_sync();
    {  // padding of the row's pixels (and the top / bottom pad rows at the frame's ends)
      const int r0 = k * 64, r1 = min(k * 64 + 64, H);
      const PadPlane py(T.cy, T.sy, W, H, THOR_PAD_Y, r0, r1);
      for (int e = lane; e < py.total; e += 64) py.chunk(e);
      const PadPlane pu(T.cu, T.sc, W >> 1, H >> 1, THOR_PAD_C, r0 >> 1, r1 >> 1);
      for (int e = lane; e < pu.total; e += 64) pu.chunk(e);
      const PadPlane pv(T.cv, T.sc, W >> 1, H >> 1, THOR_PAD_C, r0 >> 1, r1 >> 1);
      for (int e = lane; e < pv.total; e += 64) pv.chunk(e);
    }
    {  // the row's cell state to zero (deblock_data, cleared per frame): the next frame's RD loop
      const int cs = W >> 2, q0 = k * 16, q1 = min(k * 16 + 16, H >> 2);
      uint4 *c = (uint4 *)(J.F.cells + (long long)q0 * cs);
      const long long n16 = (long long)(q1 - q0) * cs * (long long)sizeof(TeCell) / 16;
      for (long long i = lane; i < n16; i += 64) c[i] = make_uint4(0u, 0u, 0u, 0u);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
      const unsigned old = __hip_atomic_fetch_add(T.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old + 1 == (unsigned)nsbv) {  // the frame is a finished reference
        ts_push(A, T.aux, ts_item(j, TS_PACK, 0));
        if (T.next >= 0) {
          const TsJob &N = A.jobs[T.next];
          ts_dep(A, &N.J.deps[0], (unsigned)N.need0, N.cls, ts_item(T.next, TS_RD, 0));
        }
        if (T.is_i) atomicAdd(&A.ctl[TS_IDONE], 1u);
      }
    }
  } else {  // TS_PACK
    const int nsb = nsbh * nsbv;
    const int per = (nsb + 63) >> 6, s0 = min(lane * per, nsb), s1 = min(s0 + per, nsb);
    int mine = 0;
    for (int i = s0; i < s1; i++) mine += te_sb_bits(J, i);
    int incl = mine;
    for (int d = 1; d < 64; d <<= 1) {
      const int v = __shfl_up(incl, d);
      if (lane >= d) incl += v;
    }
    const int sbits = __builtin_amdgcn_readlane(incl, 63);
    int nclpf = 0;
    const int nf = (W >> 6) * (H >> 6);
    if (J.clpf)
      for (int i = lane; i < nf; i += 64) nclpf += J.clpf_bits[i] >= 0;
    const long long total = (long long)J.hdr_bits + sbits + (J.clpf ? 2 + (long long)te_sum((uint32_t)nclpf) : 0);
    const long long nw = (total + 31) >> 5;
    unsigned long long off = 0;
    int ok = nw <= A.out_cap_words;
    if (ok && lane == 0) {
      off = __hip_atomic_fetch_add((unsigned long long *)&A.ctl[TS_ARENA], (unsigned long long)((nw + 3) & ~3LL),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (off + nw > A.arena_words) ok = 0;
    }
    ok = __builtin_amdgcn_readfirstlane(ok);
    off = ((unsigned long long)__builtin_amdgcn_readfirstlane((int)(off >> 32)) << 32) |
          (unsigned)__builtin_amdgcn_readfirstlane((int)(off & 0xffffffffu));
    if (!ok) {
      if (lane == 0) atomicOr(A.err, 4u);  // the frame exceeds the output buffer or the host arena
    } else {
      uint32_t *out = J.out_words;
      for (long long i = lane; i < ((nw + 3) & ~3LL) + 4; i += 64) out[i] = 0u;
      __threadfence();
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) te_or_bits(out, 0, J.hdr_words, J.hdr_bits);
      long long pos = (long long)J.hdr_bits + (incl - mine);
      for (int i = s0; i < s1; i++) {
        const int b = te_sb_bits(J, i);
        te_or_bits(out, pos, J.sb_words + (size_t)i * THOR_ENC_SB_WORDS, b);
        pos += b;
      }
      if (lane == 0 && J.clpf) {
        long long p = (long long)J.hdr_bits + sbits;
        const uint32_t two = 0x80000000u;  // bits 1, 0
        te_or_bits(out, p, &two, 2);
        p += 2;
        for (int i = 0; i < nf; i++) {
          const int d = J.clpf_bits[i];
          if (d < 0) continue;
          if (d) atomicOr(&out[p >> 5], 0x80000000u >> (p & 31));
          p++;
        }
      }
      __threadfence();
      __builtin_amdgcn_wave_barrier();
      uint4 *dst = (uint4 *)(A.arena + off);
      const uint4 *src = (const uint4 *)out;
      for (long long i = lane; i < (nw + 3) >> 2; i += 64) dst[i] = src[i];
      // a system-scope RELEASE (the words reach host memory before the size): __threadfence_system
      // would also invalidate this XCD's L2 under every other worker there
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) {
        A.meta[2 * j] = (int)off;
        __hip_atomic_store(&A.meta[2 * j + 1], (int)total, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __builtin_amdgcn_wave_barrier();
    if (lane == 0 && T.next2 >= 0) {  // frame f + 2 may write this frame's SB buffers
      const TsJob &N = A.jobs[T.next2];
      ts_dep(A, &N.J.deps[0], (unsigned)N.need0, N.cls, ts_item(T.next2, TS_RD, 0));
    }
  }
}

__global__ __launch_bounds__(64) TE_WPE void k_enc_seq(const TsArgs A) {
  __shared__ TeFrame s_F;
  __shared__ TeSB s_sb;
  __shared__ unsigned long long s_prof[TS_NPROF];  // (lane 0) this worker's profile, added to the launch's at exit
  if (threadIdx.x < TS_NPROF) s_prof[threadIdx.x] = 0;
  g_te_mem = &A.scratch[blockIdx.x];
  te_load_basis(g_te_tx);
  te_load_zig();
  TeSB &sb = s_sb;
  const int lane = threadIdx.x;
  int cur = -1;  // the job whose frame parameters s_F holds
  unsigned long long idle0 = 0, prog0 = __builtin_amdgcn_s_memrealtime();
  unsigned nd = 0, nd_seen = 0;
  bool idle = false;
  unsigned long long t_prev = __builtin_amdgcn_s_memrealtime(), t_task = 0;
  for (;;) {
    unsigned item = TE_Q_EMPTY, state = 0;  // 0: nothing ready, 1: a task, 2: leave
    if (lane == 0) {
      const unsigned long long t_now = __builtin_amdgcn_s_memrealtime();
      if (idle) s_prof[12] += t_now - t_prev;
      t_prev = t_now;
      unsigned long long fails = 0, waits = 0;
      item = ts_pop(A, fails, waits);
      s_prof[13] += waits;
      s_prof[14] += fails;
      t_task = __builtin_amdgcn_s_memrealtime();
      if (item != TE_Q_EMPTY) {
        state = 1;
      } else if ((nd = te_ld_relaxed(&A.ctl[TS_NDONE])) >= A.total || te_ld_relaxed(A.err)) {
        state = 2;  // every task done (or the launch failed): the grid drains
      } else {
        const unsigned long long now = __builtin_amdgcn_s_memrealtime();  // 100 MHz
        if (!idle) idle = true, idle0 = now;
        if (nd != nd_seen) nd_seen = nd, prog0 = now;  // the launch is moving (a long SB elsewhere is not a wedge)
        if (now - prog0 > A.spin_limit) {  // no task finished anywhere for that long: give up, reported; never hang the GPU
          atomicOr(A.err, 1u);
          state = 2;
        } else if (now - idle0 > A.retire_ticks && te_ld_relaxed(&A.ctl[TS_IDONE]) >= A.n_ijobs) {
          // the I frames are done and this worker found nothing for a while: leave (down to
          // min_alive workers), so concurrent decode launches get the CU slots
          unsigned a = te_ld_relaxed(&A.ctl[TS_ALIVE]);
          while ((int)a > A.min_alive) {
            if (__hip_atomic_compare_exchange_strong(&A.ctl[TS_ALIVE], &a, a - 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT)) {
              atomicAdd(&A.ctl[TS_RETIRED], 1u);
              state = 2;
              break;
            }
          }
        }
      }
    }
    state = __builtin_amdgcn_readfirstlane(state);
    if (state == 2) break;
    if (state == 0) {
      __builtin_amdgcn_s_sleep(32);
      continue;
    }
    idle = false;
    item = __builtin_amdgcn_readfirstlane(item);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const int j = (int)(item >> 20), type = (int)((item >> 17) & 7), idx = (int)(item & (TS_MAX_SB - 1));
    const TsJob &T = A.jobs[j];
    const TeJob &J = T.J;
    const int nsbh = J.nsbh, nsbv = J.nsbv;
    if (type == TS_RD && j != cur) {  // the job's frame parameters into LDS
      const uint32_t *src = (const uint32_t *)&J.F;
      uint32_t *dst = (uint32_t *)&s_F;
      te_sync();
      for (int e = lane; e < (int)(sizeof(TeFrame) / 4); e += 64) dst[e] = src[e];
      te_sync();
      cur = j;
    }
    if (type == TS_RD) {
      const int k = idx / nsbh, l = idx - k * nsbh;
      if (idx == 0 && T.next >= 0 && A.jobs[T.next].src && lane == 0) {  // the next frame's input starts moving
        const TsJob &N = A.jobs[T.next];
        for (int r = 0; r < nsbv; r++) ts_push(A, N.aux, ts_item(T.next, TS_FETCH, r));
      }
      sb.bits.w = J.sb_words + (size_t)idx * THOR_ENC_SB_WORDS;
      sb.bits.cap = THOR_ENC_SB_WORDS * 32;
      TE_NB_FORGET();  // (another job's block may have left the key)
      te_encode_sb(s_F, sb, k, l, nullptr);
      if (lane == 0) {
        J.sb_nbits[idx] = sb.bits.pos;
        if (sb.bits.pos > sb.bits.cap) atomicOr(A.err, 2u);
      }
      te_sync();  // the SB's cells (written by every lane) before their loop-filter words
      te_sb_cellinfo(J, k, l);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) {  // dependants (enc.hip's rule), and the row's vertical deblocking
        if (l + 1 < nsbh) ts_dep(A, &J.deps[idx + 1], 1u + (k > 0), T.cls, ts_item(j, TS_RD, idx + 1));
        if (k + 1 < nsbv) {
          if (l >= 1) ts_dep(A, &J.deps[idx + nsbh - 1], 1u + (l - 1 > 0), T.cls, ts_item(j, TS_RD, idx + nsbh - 1));
          if (l == nsbh - 1) ts_dep(A, &J.deps[idx + nsbh], 1u + (l > 0), T.cls, ts_item(j, TS_RD, idx + nsbh));
        }
        if (l == nsbh - 1) {  // row k complete (and with it every row above)
          if (k >= 1) ts_push(A, T.aux, ts_item(j, TS_DBV, k - 1));
          if (k == nsbv - 1) ts_push(A, T.aux, ts_item(j, TS_DBV, k));
        }
      }
    } else {
      ts_aux(A, j, type, idx);
    }
    if (lane == 0) {
      __hip_atomic_fetch_add(&A.ctl[TS_NDONE], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
      s_prof[type] += t1 - t_task;
      s_prof[6 + type] += 1;
      t_prev = t1;
    }
  }
  if (lane == 0)
    for (int i = 0; i < TS_NPROF; i++)
      if (s_prof[i]) atomicAdd((unsigned long long *)&A.ctl[TS_PROF + 2 * i], s_prof[i]);
}

// ============================================================================
// Host side
// ============================================================================
struct TsRun {  // one sequence launch in flight on a device
  bool active = false;
  std::vector<thor_enc *> es;
  int n = 0, nframes = 0;
  hipStream_t st = nullptr;
  hipEvent_t ev = nullptr;
  std::vector<EncPool::Pending::Snap> snap;
  std::vector<std::vector<int>> frame_num;  // [i][f]
};
struct TsPool {  // per device: the sequence launch's buffers (grown, never shrunk)
  TsJob *jobs = nullptr;
  size_t njobs = 0;
  unsigned *cnt = nullptr;
  size_t ncnt = 0;
  unsigned *items = nullptr;
  size_t nitems = 0;
  unsigned *ctl = nullptr;
  uint32_t *hdr = nullptr;
  size_t nhdr = 0;
  uint32_t *arena = nullptr;  // host, page-locked
  size_t arena_words = 0;
  int *meta = nullptr;        // host, page-locked
  size_t nmeta = 0;
  int max_workers = 0;
  long long prof[TS_NPROF] = {};
  TsRun run;
};
static std::map<int, TsPool *> g_ts_pools;
static TsPool &ts_pool_for(int device) {
  std::lock_guard<std::mutex> lk(g_pools_mu);
  TsPool *&p = g_ts_pools[device];
  if (!p) p = new TsPool();
  return *p;
}

static bool ts_active(int device) {
  std::lock_guard<std::mutex> lk(g_pools_mu);
  auto it = g_ts_pools.find(device);
  return it != g_ts_pools.end() && it->second->run.active;
}
static bool ts_member(const thor_enc *e) {
  std::lock_guard<std::mutex> lk(g_pools_mu);
  auto it = g_ts_pools.find(e->device);
  if (it == g_ts_pools.end() || !it->second->run.active) return false;
  for (const thor_enc *x : it->second->run.es)
    if (x == e) return true;
  return false;
}
static void ts_forget(thor_enc *e) {
  TsPool *S = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_pools_mu);
    auto it = g_ts_pools.find(e->device);
    if (it != g_ts_pools.end()) S = it->second;
  }
  if (!S) return;
  EncPool &P = pool_for(e->device);
  std::lock_guard<std::mutex> pl(P.mu);
  for (thor_enc *&x : S->run.es)
    if (x == e) {
      if (S->run.active) (void)hipEventSynchronize(S->run.ev);
      x = nullptr;
    }
}

// a context's second set of SB buffers (frame parity 1 of a sequence launch)
static int ts_context_buffers(thor_enc *e) {
  if (e->sb_words2) return THOR_OK;
  if (!dev_alloc(&e->sb_words2, (size_t)e->nsb * THOR_ENC_SB_WORDS * 4, "thor_enc_seq_begin: SB bit strings (2)"))
    return g_create_err.code;
  if (!dev_alloc(&e->sb_nbits2, (size_t)e->nsb * sizeof(int), "thor_enc_seq_begin: SB bit counts (2)")) return g_create_err.code;
  if (!dev_alloc(&e->clpf_bits2, (size_t)e->nsb_full + 1, "thor_enc_seq_begin: CLPF bits (2)")) return g_create_err.code;
  return THOR_OK;
}

template <typename T>
static int ts_grow_dev(T **p, size_t &have, size_t want) {
  if (want <= have) return THOR_OK;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  have = 0;
  EHIP(hipMalloc(p, want * sizeof(T)));
  have = want;
  return THOR_OK;
}

extern "C" {

int thor_enc_seq_begin(thor_enc_t *const *es, int n, int nframes, const uint8_t *const *in, uint8_t *const *dev,
                       int fetch, long long arena_bytes) {
  if (!es || !in || n <= 0 || nframes <= 0 || (long long)n * nframes > TS_MAX_JOBS || (fetch && !dev)) return THOR_ERR_ARG;
  thor_enc *lead = es[0];
  for (int i = 0; i < n; i++) {
    thor_enc *e = es[i];
    if (!e || e->device != lead->device || e->W != lead->W || e->H != lead->H) return THOR_ERR_ARG;
    if (e->p.interp_ref || e->sb_costs) return THOR_ERR_ARG;  // (thor_enc_frames codes those)
    if (e->pos + nframes > e->gop->plans.size()) return THOR_ERR_ARG;
    for (int j = 0; j < i; j++)
      if (es[j] == e) return THOR_ERR_ARG;
    for (int f = 0; f < nframes; f++)
      if (!in[i * nframes + f] || (fetch && !dev[i * nframes + f])) return THOR_ERR_ARG;
  }
  if (lead->nsb >= TS_MAX_SB) return THOR_ERR_ARG;
  EHIP(hipSetDevice(lead->device));
  EncPool &P = pool_for(lead->device);
  std::lock_guard<std::mutex> pool_lock(P.mu);
  TsPool &S = ts_pool_for(lead->device);
  if (S.run.active || !P.pending.empty()) return THOR_ERR_ARG;  // one launch at a time per device
  const int W = lead->W, H = lead->H, nsbv = lead->nsbv, nsb = lead->nsb;
  const int njobs = n * nframes;
  int rc;
  for (int i = 0; i < n; i++) {
    if (es[i]->stream != lead->stream) EHIP(hipStreamSynchronize(es[i]->stream));
    if ((rc = ts_context_buffers(es[i])) != THOR_OK) return rc;
  }
  if (!S.max_workers) {
    int dev_id = lead->device, ncu = 0, per = 0;
    EHIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev_id));
    EHIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_enc_seq, 64, 0));
    S.max_workers = ncu * (per > 0 ? per : 1);
  }
  const int nwork = S.max_workers < TE_MAX_WORKERS ? S.max_workers : TE_MAX_WORKERS;
  if ((rc = pool_reserve(P, (size_t)nwork, 1, 1)) != THOR_OK) return rc;
  const size_t per_cnt = (size_t)nsb + 2 * nsbv + 1;
  if ((rc = ts_grow_dev(&S.jobs, S.njobs, (size_t)njobs)) != THOR_OK) return rc;
  if ((rc = ts_grow_dev(&S.cnt, S.ncnt, (size_t)njobs * per_cnt)) != THOR_OK) return rc;
  if ((rc = ts_grow_dev(&S.hdr, S.nhdr, (size_t)njobs * 64)) != THOR_OK) return rc;
  if (!S.ctl) EHIP(hipMalloc(&S.ctl, TS_CTL_WORDS * sizeof(unsigned)));
  if ((size_t)njobs * 2 > S.nmeta) {
    if (S.meta) (void)hipHostFree(S.meta);
    S.meta = nullptr;
    S.nmeta = 0;
    EHIP(hipHostMalloc((void **)&S.meta, (size_t)njobs * 2 * sizeof(int), hipHostMallocCoherent | hipHostMallocMapped));
    S.nmeta = (size_t)njobs * 2;
  }
  size_t aw = arena_bytes > 0 ? (size_t)(arena_bytes / 4) : (size_t)njobs * ((size_t)W * H / 128 + 4096);
  if (aw > S.arena_words) {
    if (S.arena) (void)hipHostFree(S.arena);
    S.arena = nullptr;
    S.arena_words = 0;
    EHIP(hipHostMalloc((void **)&S.arena, aw * 4 + 64, hipHostMallocCoherent | hipHostMallocMapped));
    S.arena_words = aw;
  }
  // scheduling knobs (experiments): THOR_SEQ_CLASSES (1..16, default 16), THOR_SEQ_CLAIM
  // (0 compare-and-swap, 1 tickets), THOR_SEQ_RETIRE (0: workers never leave early)
  auto knob = [](const char *name, int dflt) {
    const char *v = getenv(name);
    return v && *v ? atoi(v) : dflt;
  };
  int ncls = knob("THOR_SEQ_CLASSES", TS_NCLS);
  ncls = ncls < 1 ? 1 : (ncls > TS_NCLS ? TS_NCLS : ncls);
  const int prio = knob("THOR_SEQ_PRIO", 0) && ncls >= 3;
  // the jobs: each context's frames in coding order, its host state advanced frame by frame
  hipStream_t st = lead->stream;
  std::vector<TsJob> jobs(njobs);
  std::vector<uint32_t> hdr((size_t)njobs * 64);
  std::vector<unsigned> qn(TS_NCLS, 0);
  TsRun run;
  run.n = n;
  run.nframes = nframes;
  run.st = st;
  run.frame_num.assign(n, std::vector<int>(nframes));
  for (int i = 0; i < n; i++) {
    thor_enc *e = es[i];
    run.snap.push_back({e->pos, e->first, e->last_slot, e->last_frame_num, e->opar, e->slot_of_window});
    run.es.push_back(e);
  }
  auto restore = [&]() {
    for (int i = 0; i < n; i++) {
      thor_enc *e = es[i];
      const EncPool::Pending::Snap &sn = run.snap[i];
      e->pos = sn.pos;
      e->first = sn.first;
      e->last_slot = sn.last_slot;
      e->last_frame_num = sn.last_frame_num;
      e->opar = sn.opar;
      e->slot_of_window = sn.window;
    }
  };
  for (int i = 0; i < n; i++) {
    thor_enc *e = es[i];
    const int cls = (int)((long long)i * ncls / n);
    for (int f = 0; f < nframes; f++) {
      const int jx = i * nframes + f;
      TsJob &T = jobs[jx];
      memset(&T, 0, sizeof(T));
      TeFramePlan pl;
      int cur = -1;
      uint8_t *orig = fetch ? dev[jx] : (uint8_t *)in[jx];
      if ((rc = enc_prepare(e, orig, W, T.J, pl, cur, st, &hdr[(size_t)jx * 64], S.hdr + (size_t)jx * 64)) != THOR_OK) {
        restore();
        return rc;
      }
      const int par = f & 1;
      TeJob &J = T.J;
      J.sb_words = par ? e->sb_words2 : e->sb_words;
      J.sb_nbits = par ? e->sb_nbits2 : e->sb_nbits;
      J.clpf_bits = par ? e->clpf_bits2 : e->clpf_bits;
      J.out_words = par ? e->out_words2 : e->out_words;
      unsigned *c = S.cnt + (size_t)jx * per_cnt;
      J.deps = c;
      T.dbh = c + nsb;
      T.fin = c + nsb + nsbv;
      T.done = c + nsb + 2 * nsbv;
      T.src = fetch ? in[jx] : nullptr;
      T.dst = orig;
      T.next = f + 1 < nframes ? jx + 1 : -1;
      T.next2 = f + 2 < nframes ? jx + 2 : -1;
      // classes: stream groups (THOR_SEQ_PRIO 0), or by task kind (1): the loop filters, packing and
      // input copies first (a frame's hand-off to the next), then P-frame SBs, then I-frame SBs by stream group
      T.cls = cls;
      T.aux = cls;
      if (prio) {
        T.aux = 0;
        T.cls = pl.frame_type != TE_I ? 1 : 2 + (int)((long long)i * (ncls - 2) / n);
      }
      T.need0 = (fetch ? nsbv : 0) + (f > 0) + (f > 1);
      T.is_i = pl.frame_type == TE_I;
      uint8_t *cs = e->slots + (long long)cur * e->slot_bytes;
      T.cy = cs + e->offy;
      T.cu = cs + e->offu;
      T.cv = cs + e->offv;
      T.sy = e->sy;
      T.sc = e->sc;
      T.qp = pl.qp;
      T.qpc = chroma_qp_host(pl.qp);
      T.deblock = e->p.deblocking;
      run.frame_num[i][f] = pl.frame_num;
      // tasks of the job: RD nsb, DBV / DBH / FIN nsbv each, PACK 1 (+ FETCH nsbv)
      qn[T.cls] += nsb;
      qn[T.aux] += 3 * nsbv + 1 + (fetch ? nsbv : 0);
      // advance the context as thor_enc_frames_begin does
      for (int r = 32; r > 0; r--) e->slot_of_window[r] = e->slot_of_window[r - 1];
      e->slot_of_window[0] = cur;
      e->last_slot = cur;
      e->last_frame_num = pl.frame_num;
      e->first = false;
      e->pos++;
    }
  }
  // queues: class regions, the initial items (each stream's first frame: its input rows, or its SB (0, 0))
  std::vector<unsigned> qoff(TS_NCLS, 0);
  size_t tot_items = 0;
  unsigned total = 0;
  for (int c = 0; c < TS_NCLS; c++) {
    qoff[c] = (unsigned)tot_items;
    tot_items += qn[c];
    total += qn[c];
  }
  if ((rc = ts_grow_dev(&S.items, S.nitems, tot_items)) != THOR_OK) {
    restore();
    return rc;
  }
  std::vector<unsigned> ctl(TS_CTL_WORDS, 0);
  std::vector<std::vector<unsigned>> init(TS_NCLS);
  unsigned n_i = 0;
  for (int i = 0; i < n; i++) {
    const int jx = i * nframes;
    const TsJob &T = jobs[jx];
    if (fetch)
      for (int r = 0; r < nsbv; r++) init[T.aux].push_back(ts_item(jx, TS_FETCH, r));
    else
      init[T.cls].push_back(ts_item(jx, TS_RD, 0));
    for (int f = 0; f < nframes; f++) n_i += jobs[jx + f].is_i;
  }
  ctl[TS_ALIVE] = (unsigned)nwork;
  EHIP(hipMemsetAsync(S.items, 0xff, tot_items * sizeof(unsigned), st));
  for (int c = 0; c < TS_NCLS; c++) {
    ctl[TS_TAIL(c)] = (unsigned)init[c].size();
    if (!init[c].empty())
      EHIP(hipMemcpyAsync(S.items + qoff[c], init[c].data(), init[c].size() * sizeof(unsigned), hipMemcpyHostToDevice, st));
  }
  EHIP(hipMemcpyAsync(S.ctl, ctl.data(), ctl.size() * sizeof(unsigned), hipMemcpyHostToDevice, st));
  EHIP(hipMemsetAsync(S.cnt, 0, (size_t)njobs * per_cnt * sizeof(unsigned), st));
  EHIP(hipMemcpyAsync(S.hdr, hdr.data(), hdr.size() * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  EHIP(hipMemcpyAsync(S.jobs, jobs.data(), njobs * sizeof(TsJob), hipMemcpyHostToDevice, st));
  for (int i = 0; i < n; i++) {  // every context's cell state to zero before its first frame
    const long long cb = (long long)(W / 4) * (H / 4) * (long long)sizeof(TeCell);
    EHIP(hipMemsetAsync(es[i]->cells, 0, cb, st));
  }
  for (size_t m = 0; m < (size_t)njobs; m++) {
    S.meta[2 * m] = 0;
    S.meta[2 * m + 1] = -1;
  }
  EHIP(hipMemsetAsync(P.err, 0, sizeof(unsigned), st));
  TsArgs A;
  memset(&A, 0, sizeof(A));
  A.jobs = S.jobs;
  A.scratch = P.scratch;
  A.ctl = S.ctl;
  A.items = S.items;
  A.err = P.err;
  for (int c = 0; c < TS_NCLS; c++) {
    A.qoff[c] = qoff[c];
    A.qtot[c] = qn[c];
  }
  A.ncls = ncls;
  A.claim = knob("THOR_SEQ_CLAIM", 0);
  A.total = total;
  A.n_ijobs = n_i;
  A.min_alive = nwork / 2;
  A.spin_limit = g_spin_limit.load();
  A.retire_ticks = knob("THOR_SEQ_RETIRE", 1) ? 50000 : ~0ULL >> 1;  // 0.5 ms without a ready task
  A.arena = S.arena;
  A.arena_words = S.arena_words;
  A.meta = S.meta;
  A.out_cap_words = lead->out_cap_words;
  k_enc_seq<<<nwork, 64, 0, st>>>(A);
  {
    hipError_t le = hipGetLastError();
    if (le != hipSuccess) {
      restore();
      fprintf(stderr, "thor_amd enc: k_enc_seq launch failed: %s\n", hipGetErrorString(le));
      return THOR_ERR_HIP;
    }
  }
  if (!S.run.ev) EHIP(hipEventCreateWithFlags(&S.run.ev, hipEventDisableTiming));
  run.ev = S.run.ev;
  EHIP(hipEventRecord(run.ev, st));
  run.active = true;
  S.run = std::move(run);
  return THOR_OK;
}

// Which frames of the launch in flight (or the last one ended) are final: out[i * nframes + f] = the
// chunk size in bytes (4-byte length + payload), -1 not yet.  Non-blocking.
// Returns the number of final frames.
int thor_enc_seq_ready(thor_enc_t *e0, long long *out, int count) {
  if (!e0) return THOR_ERR_ARG;
  TsPool &S = ts_pool_for(e0->device);
  if (!S.meta || S.run.n <= 0) return THOR_ERR_ARG;  // (the launch in flight, or the last one ended)
  const int nj = S.run.n * S.run.nframes;
  int done = 0;
  for (int m = 0; m < nj; m++) {
    const int nb = __atomic_load_n(&S.meta[2 * m + 1], __ATOMIC_ACQUIRE);
    const long long sz = nb >= 0 ? 4 + ((long long)nb + 7) / 8 : -1;
    if (out && m < count) out[m] = sz;
    done += nb >= 0;
  }
  return done;
}

// The chunk of frame f of context i of the launch in flight (or just ended):
// 4-byte big-endian length + payload, min(size, cap) bytes copied; returns the size.
long long thor_enc_seq_chunk(thor_enc_t *e0, int i, int f, uint8_t *dst, size_t cap) {
  if (!e0) return THOR_ERR_ARG;
  TsPool &S = ts_pool_for(e0->device);
  if (i < 0 || i >= S.run.n || f < 0 || f >= S.run.nframes) return THOR_ERR_ARG;
  const int m = i * S.run.nframes + f;
  const int nb = __atomic_load_n(&S.meta[2 * m + 1], __ATOMIC_ACQUIRE);
  if (nb < 0) return THOR_ERR_ARG;
  const size_t nbytes = ((size_t)nb + 7) / 8;
  if (dst && cap) {
    const uint32_t *w = S.arena + (unsigned)S.meta[2 * m];
    uint8_t hdr4[4] = {(uint8_t)(nbytes >> 24), (uint8_t)(nbytes >> 16), (uint8_t)(nbytes >> 8), (uint8_t)nbytes};
    for (size_t b = 0; b < 4 && b < cap; b++) dst[b] = hdr4[b];
    for (size_t b = 0; b < nbytes && 4 + b < cap; b++) dst[4 + b] = (uint8_t)(w[b >> 2] >> (24 - 8 * (b & 3)));
  }
  return (long long)(4 + nbytes);
}

// Wait for the launch in flight.  On a device error the contexts return to
// their state before the launch (THOR_ERR_HIP; THOR_ERR_NOMEM when a frame
// outgrew the output buffer or the host arena).  Stats (optional, 4 values):
// workers launched, workers retired, tasks, arena words used.
int thor_enc_seq_end(thor_enc_t *e0, long long *stats) {
  if (!e0) return THOR_ERR_ARG;
  EHIP(hipSetDevice(e0->device));
  EncPool &P = pool_for(e0->device);
  std::lock_guard<std::mutex> pool_lock(P.mu);
  TsPool &S = ts_pool_for(e0->device);
  if (!S.run.active) return THOR_ERR_ARG;
  TsRun &R = S.run;
  const hipError_t se = hipEventSynchronize(R.ev);
  R.active = false;
  unsigned err = 0;
  std::vector<unsigned> ctl(TS_CTL_WORDS);
  if (se == hipSuccess) {
    EHIP(hipMemcpy(&err, P.err, sizeof(unsigned), hipMemcpyDeviceToHost));
    EHIP(hipMemcpy(ctl.data(), S.ctl, ctl.size() * sizeof(unsigned), hipMemcpyDeviceToHost));
  }
  for (int i = 0; i < TS_NPROF; i++)
    S.prof[i] = (long long)ctl[TS_PROF + 2 * i] | ((long long)ctl[TS_PROF + 2 * i + 1] << 32);
  if (stats) {
    stats[0] = S.max_workers < TE_MAX_WORKERS ? S.max_workers : TE_MAX_WORKERS;
    stats[1] = ctl[TS_RETIRED];
    stats[2] = ctl[TS_NDONE];
    stats[3] = (long long)ctl[TS_ARENA] | ((long long)ctl[TS_ARENA + 1] << 32);
  }
  int bad = se != hipSuccess || err != 0;
  for (int m = 0; m < R.n * R.nframes && !bad; m++) bad = S.meta[2 * m + 1] < 0;
  if (bad) {
    for (int i = 0; i < R.n; i++) {
      thor_enc *e = R.es[i];
      if (!e) continue;  // destroyed meanwhile
      const EncPool::Pending::Snap &sn = R.snap[i];
      e->pos = sn.pos;
      e->first = sn.first;
      e->last_slot = sn.last_slot;
      e->last_frame_num = sn.last_frame_num;
      e->opar = sn.opar;
      e->slot_of_window = sn.window;
    }
    if (se != hipSuccess) {
      fprintf(stderr, "thor_amd enc: sequence launch failed: %s\n", hipGetErrorString(se));
      (void)hipGetLastError();
      return THOR_ERR_HIP;
    }
    EHIP(hipMemset(P.err, 0, 4));
    fprintf(stderr, "thor_amd enc: sequence launch: device error flags 0x%x\n", err);
    return (err & 4) && !(err & 3) ? THOR_ERR_NOMEM : THOR_ERR_HIP;
  }
  // each context's last frame is its chunk for thor_enc_frame_bytes
  for (int i = 0; i < R.n; i++) {
    thor_enc *e = R.es[i];
    if (!e) continue;
    const long long sz = thor_enc_seq_chunk(e0, i, R.nframes - 1, nullptr, 0);
    e->chunk.resize((size_t)sz);
    thor_enc_seq_chunk(e0, i, R.nframes - 1, e->chunk.data(), e->chunk.size());
  }
  return THOR_OK;
}

// The last ended launch's profile (sums over its workers, 100 MHz ticks):
// per task type (RD, FETCH, DBV, DBH, FIN, PACK) the time in tasks, then the
// task counts, then idle time, time waiting for a claimed slot, failed claims.
// Returns the count (15), copies min(15, n).
int thor_enc_seq_profile(thor_enc_t *e0, long long *out, int n) {
  if (!e0) return THOR_ERR_ARG;
  TsPool &S = ts_pool_for(e0->device);
  for (int i = 0; i < TS_NPROF && i < n && out; i++) out[i] = S.prof[i];
  return TS_NPROF;
}

}  // extern "C"
