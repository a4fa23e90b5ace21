"""Row-band sharding of one stream (thor_amd/shard.py):
the band partition and the all-gather exchange protocol, on CPU with the
gloo backend at world size 2 and 3.  A numpy stand-in for the decoder context
(same begin / get_rows / put_rows / end surface as GpuDecoder) reconstructs
only its band; after the exchange every rank must hold the whole frame.  The
same RowShard drives the GPU contexts in tests/test_gpu_shard.py."""
import os

import numpy as np
import pytest


def test_band_partition():
    from thor_amd.shard import band_of, band_rows

    for H in (64, 288, 1080, 2160):
        nsb = (H + 63) // 64
        for world in (1, 2, 3, 4, 8):
            rows = band_rows(H, world)
            assert rows % 64 == 0 and rows * world >= nsb * 64
            covered, sizes = [], []
            for r in range(world):
                b0, b1 = band_of(H, world, r)
                covered += list(range(b0, b1))
                sizes.append(b1 - b0)
                assert 64 * (b1 - b0) <= rows
            assert covered == list(range(nsb)), (H, world)
            assert max(sizes) - min(sizes) <= 1, (H, world, sizes)  # balanced
            if nsb >= world:
                assert min(sizes) >= 1, (H, world, sizes)  # no empty band
    # the north star's 8-way split: 4K = 34 SB rows -> 5, 5, 4 x 6; 1080p = 17 -> 3, 2 x 7
    assert [band_of(2160, 8, r)[1] - band_of(2160, 8, r)[0] for r in range(8)] == [5, 5, 4, 4, 4, 4, 4, 4]
    assert [band_of(1080, 8, r)[1] - band_of(1080, 8, r)[0] for r in range(8)] == [3, 2, 2, 2, 2, 2, 2, 2]


class NumpyContext:
    """Decoder-context stand-in: frames are dicts of numpy planes."""

    def __init__(self, W, H, truth):
        self.W, self.H, self.truth = W, H, truth
        self.band = None
        self.local = False
        self.halo = False
        self.cur = None
        self.bufs = {}
        self.refs = {}
        self.frames = {}  # halo mode: parse-output stand-ins, to check the fetched rows
        self.band_intra = False  # boundary mode: intra of the band only, rows above via the edge exchange
        self.intra_done = False

    def set_band_intra(self, on):
        self.band_intra = on

    def intra(self):
        """The band's intra chains: the first one reads the two rows above the
        band, which must be final by now when the band holds intra CUs."""
        fnum, planes = self.cur
        r0 = 64 * self.band[0]
        fr = self.frames.get(fnum)
        if fr is not None and r0 > 0 and len(fr.blocks):
            rows = fr.blocks["ypos"][fr.blocks["mode"] == 1].astype(np.int64) >> 6
            if np.any((rows >= self.band[0]) & (rows < self.band[1])):
                assert np.array_equal(planes[0][r0 - 2:r0], self.truth[fnum][0][r0 - 2:r0]), (fnum, "edge rows")
                for k in (1, 2):
                    assert np.array_equal(planes[k][r0 // 2 - 1], self.truth[fnum][k][r0 // 2 - 1]), (fnum, k)
        self.intra_done = True

    def set_band(self, b0, b1):
        self.band = (b0, b1)

    def set_band_local(self, on):
        self.local = on

    def set_band_pad(self, on):  # halo modes: finish() pads only the band (nothing to model here)
        self.band_pad = on

    def begin(self, fnum):  # the "device frame" is the frame number here
        if self.halo and fnum in self.frames:  # every reference row the band's vectors reach is final
            from thor_amd.shard import halo_requests

            r0, r1 = 64 * self.band[0], min(64 * self.band[1], self.H)
            for f, (lo, hi) in halo_requests(self.frames[fnum], self.H, r0, r1).items():
                for k, (got, want) in enumerate(zip(self.refs[f], self.truth[f])):
                    a, b = (lo, hi) if k == 0 else (lo // 2, hi // 2)
                    assert np.array_equal(got[a:b], want[a:b]), (fnum, f, k, lo, hi)
        y, u, v = (np.zeros_like(p) for p in self.truth[fnum])
        r0, r1 = 64 * self.band[0], min(64 * self.band[1], self.H)
        y[r0:r1] = self.truth[fnum][0][r0:r1]
        u[r0 // 2:r1 // 2] = self.truth[fnum][1][r0 // 2:r1 // 2]
        v[r0 // 2:r1 // 2] = self.truth[fnum][2][r0 // 2:r1 // 2]
        self.cur = (fnum, [y, u, v])

    def scratch(self, nbytes):
        k = len(self.bufs) + 1
        self.bufs[k] = np.zeros(nbytes, np.uint8)
        return k

    def get_rows(self, fnum, y0, n, key):
        planes = self.cur[1] if self.cur is not None and fnum == self.cur[0] else self.refs[fnum]
        buf, (y, u, v) = self.bufs[key], planes
        m = max(0, min(n, self.H - y0))
        W = self.W
        buf[:m * W] = y[y0:y0 + m].reshape(-1)
        o = n * W
        for p in (u, v):
            buf[o:o + (m // 2) * (W // 2)] = p[y0 // 2:y0 // 2 + m // 2].reshape(-1)
            o += (n // 2) * (W // 2)

    def put_rows(self, fnum, y0, n, key):
        assert fnum == self.cur[0] and y0 % 2 == 0
        buf, (y, u, v) = self.bufs[key], self.cur[1]
        m = max(0, min(n, self.H - y0))
        W = self.W
        y[y0:y0 + m] = buf[:m * W].reshape(m, W)
        o = n * W
        for p in (u, v):
            p[y0 // 2:y0 // 2 + m // 2] = buf[o:o + (m // 2) * (W // 2)].reshape(m // 2, W // 2)
            o += (n // 2) * (W // 2)

    def d2h(self, out, key):  # the first out.nbytes bytes, as GpuDecoder.d2h
        out[:] = self.bufs[key][:out.size]

    def h2d(self, key, arr):
        self.bufs[key][:arr.size] = arr

    def end(self):
        fnum, planes = self.cur
        if self.band_intra:  # boundary mode: the band, its intra done, and 8 halo rows either side are final
            assert self.intra_done
            self.intra_done = False
            r0, r1 = max(0, 64 * self.band[0] - 8), min(self.H, 64 * self.band[1] + 8)
            for k, (got, want) in enumerate(zip(planes, self.truth[fnum])):
                a, b = (r0, r1) if k == 0 else (r0 // 2, r1 // 2)
                assert np.array_equal(got[a:b], want[a:b]), (fnum, k, a, b)
        else:
            for got, want in zip(planes, self.truth[fnum]):
                assert np.array_equal(got, want), fnum
        if self.local:  # band-local phase B: only the band's rows are final, model the rest as stale
            r0, r1 = 64 * self.band[0], min(64 * self.band[1], self.H)
            for k, p in enumerate(planes):
                a, b = (r0, r1) if k == 0 else (r0 // 2, r1 // 2)
                p[:a] ^= 0x5A
                p[b:] ^= 0x5A

    def finish(self):
        assert self.local
        fnum, planes = self.cur
        if not self.halo:
            for got, want in zip(planes, self.truth[fnum]):
                assert np.array_equal(got, want), fnum
        self.refs[fnum] = planes  # a reference from now on (halo mode: final in the band only)
        self.cur = None

    # --- halo mode (MV-reach exchange of reference rows) ---
    def put_ref_rows(self, fnum, y0, n, key):
        buf, (y, u, v) = self.bufs[key], self.refs[fnum]
        m = max(0, min(n, self.H - y0))
        W = self.W
        y[y0:y0 + m] = buf[:m * W].reshape(m, W)
        o = n * W
        for p in (u, v):
            p[y0 // 2:y0 // 2 + m // 2] = buf[o:o + (m // 2) * (W // 2)].reshape(m // 2, W // 2)
            o += (n // 2) * (W // 2)

    def pad_frame(self, fnum):
        assert fnum in self.refs

    def sync(self):
        pass


def _worker(rank, world, port, W, H, q, local=False):
    import torch.distributed as dist

    from thor_amd.shard import RowShard

    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        rng = np.random.default_rng(7)  # same frames on every rank
        truth = {f: (rng.integers(0, 256, (H, W), dtype=np.uint8), rng.integers(0, 256, (H // 2, W // 2), dtype=np.uint8),
                     rng.integers(0, 256, (H // 2, W // 2), dtype=np.uint8)) for f in range(3)}
        ctx = NumpyContext(W, H, truth)
        sh = RowShard(ctx, dist, W, H, device_exchange=False, band_local=local)
        for f in range(3):
            sh.decode(f, f)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))


@pytest.mark.parametrize("world,W,H,local", [(2, 352, 288, False), (3, 256, 200, False), (2, 128, 64, False),
                                             (2, 352, 288, True), (3, 256, 200, True), (8, 128, 2160, False),
                                             (8, 128, 2160, True)])
def test_row_shard_exchange_gloo(world, W, H, local):
    import random

    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = random.randint(20000, 40000)
    procs = [ctx.Process(target=_worker, args=(r, world, port, W, H, q, local)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(res) == [(r, "ok") for r in range(world)], res


class FakeFrame:
    """Parse-output stand-in for halo_requests: 64x64 inter CUs with random
    vectors (display-order reference = the previous frame)."""

    def __init__(self, fnum, W, H, rng, reach):
        from thor_amd.trace import BLOCK_DTYPE

        self.frame_num = fnum
        self.interp_refs = (-1, -1)
        self.interp_ratio = 0
        n = ((W + 63) // 64) * ((H + 63) // 64) if fnum > 0 else 0
        b = np.zeros(n, BLOCK_DTYPE)
        k = 0
        for sy in range(0, H, 64):
            for sx in range(0, W, 64):
                if k >= n:
                    break
                b[k]["ypos"], b[k]["xpos"], b[k]["size"] = sy, sx, 64
                b[k]["bwidth"], b[k]["bheight"] = min(64, W - sx), min(64, H - sy)
                b[k]["mode"] = 2
                b[k]["ref0"], b[k]["ref1"] = fnum - 1, -1
                b[k]["mv0"][:] = rng.integers(-4 * reach, 4 * reach + 1, 8)
                k += 1
        self.blocks = b


def test_halo_requests_cover_every_footprint():
    """Every 6-tap luma / 4-tap chroma footprint of every inter CU of a band,
    for either sign of its vectors, lies inside the requested rows."""
    from thor_amd.shard import halo_requests

    rng = np.random.default_rng(3)
    W, H = 192, 320
    for fnum in range(1, 6):
        fr = FakeFrame(fnum, W, H, rng, reach=50)
        for r0, r1 in ((0, 128), (128, 256), (256, 320)):
            req = halo_requests(fr, H, r0, r1)
            for blk in fr.blocks:
                if not (r0 <= blk["ypos"] < r1):
                    continue
                lo, hi = req[int(blk["ref0"])]
                for q in range(4):
                    mvy = int(blk["mv0"][2 * q + 1])
                    for s_ in (1, -1):
                        dy = (s_ * mvy) >> 2
                        a = max(0, int(blk["ypos"]) + dy - 2)
                        b_ = min(H, int(blk["ypos"]) + int(blk["bheight"]) + dy + 3)
                        assert lo <= a and b_ <= hi, (fnum, r0, lo, hi, a, b_)
                        cdy = (s_ * mvy) >> 3  # chroma rows, in luma units
                        assert lo <= max(0, 2 * ((int(blk["ypos"]) >> 1) + cdy - 1))
                        assert min(H, 2 * ((int(blk["ypos"]) + int(blk["bheight"])) // 2 + cdy + 2)) <= hi


def _halo_worker(rank, world, port, W, H, q):
    import torch.distributed as dist

    from thor_amd.shard import RowShard

    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        rng = np.random.default_rng(7)  # same frames on every rank
        nf = 5
        truth = {f: (rng.integers(0, 256, (H, W), dtype=np.uint8), rng.integers(0, 256, (H // 2, W // 2), dtype=np.uint8),
                     rng.integers(0, 256, (H // 2, W // 2), dtype=np.uint8)) for f in range(nf)}
        frames = {f: FakeFrame(f, W, H, rng, reach=40) for f in range(nf)}
        ctx = NumpyContext(W, H, truth)
        ctx.halo = True
        ctx.frames = frames
        sh = RowShard(ctx, dist, W, H, device_exchange=False, band_local=True, halo=True)
        for f in range(nf):
            sh.decode(f, f, frames[f])
        assert sh.halo_bytes[0] == 0 and sum(sh.halo_bytes) > 0, sh.halo_bytes
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, repr(e) + traceback.format_exc()[-600:]))


@pytest.mark.parametrize("world,W,H", [(2, 192, 320), (3, 128, 448), (8, 128, 2160)])
def test_row_shard_halo_exchange_gloo(world, W, H):
    """Halo mode: no second all-gather; before each frame every rank fetches the
    reference rows its band's vectors reach from their owners, and those rows
    must be final (NumpyContext.begin checks them against the truth)."""
    import random

    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = random.randint(20000, 40000)
    procs = [ctx.Process(target=_halo_worker, args=(r, world, port, W, H, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(res) == [(r, "ok") for r in range(world)], res


def test_missing_rows_tracking():
    """RowShard.missing: only the requested rows a rank does not already hold
    final are fetched (its own band, every halo fetched before)."""
    from thor_amd.shard import RowShard

    sh = object.__new__(RowShard)
    sh.final = {}
    sh._hold(5, 128, 256)
    assert sh.missing({5: (100, 300)}) == [(5, 100, 128), (5, 256, 300)]
    sh._hold(5, 256, 300)
    sh._hold(5, 90, 130)
    assert sh.final[5] == [(90, 300)]
    assert sh.missing({5: (100, 300)}) == []
    assert sh.missing({5: (0, 320), 6: (10, 20)}) == [(5, 0, 90), (5, 300, 320), (6, 10, 20)]
    # frames that leave the reference window are forgotten (bounded over a long stream)
    sh.decoded, sh.window = [], 3
    for f in (5, 6, 7, 8):
        sh._retire(f)
    assert 5 not in sh.final and sh.decoded == [6, 7, 8]


def _halo_interp_worker(rank, world, port, W, H, q):
    import torch.distributed as dist

    from thor_amd.shard import RowShard, rows_bytes

    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        rng = np.random.default_rng(11)
        nf = 6
        truth = {f: (rng.integers(0, 256, (H, W), dtype=np.uint8), rng.integers(0, 256, (H // 2, W // 2), dtype=np.uint8),
                     rng.integers(0, 256, (H // 2, W // 2), dtype=np.uint8)) for f in range(nf)}
        frames = {f: FakeFrame(f, W, H, rng, reach=8) for f in range(nf)}
        for f in range(2, nf):  # temporal-interpolated reference built from frames 0 and 1 (both read whole)
            frames[f].interp_refs, frames[f].interp_ratio = (0, 1), 2
        ctx = NumpyContext(W, H, truth)
        ctx.halo = True
        ctx.frames = frames
        sh = RowShard(ctx, dist, W, H, device_exchange=False, band_local=True, halo=True)
        for f in range(nf):
            sh.decode(f, f, frames[f])
        full = rows_bytes(W, H)
        # frame 2 fetches both interpolation sources whole (less this rank's own bands of them);
        # frames 3.. hold them already: only their small MV halos of the previous frame move
        assert sh.halo_bytes[2] > full // 2, sh.halo_bytes
        assert all(b < full // 4 for b in sh.halo_bytes[3:]), sh.halo_bytes
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, repr(e) + traceback.format_exc()[-600:]))


def _halo_overflow_worker(rank, world, port, W, H, q):
    import torch.distributed as dist

    from thor_amd.shard import MAX_REQ, RowShard

    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        rng = np.random.default_rng(5)
        nf = MAX_REQ + 3
        truth = {f: (rng.integers(0, 256, (H, W), dtype=np.uint8), rng.integers(0, 256, (H // 2, W // 2), dtype=np.uint8),
                     rng.integers(0, 256, (H // 2, W // 2), dtype=np.uint8)) for f in range(nf)}
        frames = {f: FakeFrame(f, W, H, rng, reach=2) for f in range(nf)}
        last = frames[nf - 1]
        last.blocks = np.repeat(last.blocks[:1], nf - 1)  # rank 0's first SB, once per older frame
        last.blocks["ref0"] = np.arange(nf - 1)
        last.blocks["mv0"][:] = 4 * 200  # reaching far below the band: rows it does not hold
        ctx = NumpyContext(W, H, truth)
        ctx.halo = True
        sh = RowShard(ctx, dist, W, H, device_exchange=False, band_local=True, halo=True)
        for f in range(nf - 1):
            sh.decode(f, f, frames[f])
        try:
            sh.decode(nf - 1, nf - 1, last)
            res = "no error"
        except ValueError as e:
            res = "raised" if "reference ranges" in str(e) else repr(e)
        dist.barrier()  # every rank got here: nobody is stuck in a collective
        dist.destroy_process_group()
        q.put((rank, res))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, repr(e) + traceback.format_exc()[-600:]))


def _run_world(target, world, W, H, want):
    import random

    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = random.randint(20000, 40000)
    procs = [ctx.Process(target=target, args=(r, world, port, W, H, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(res) == [(r, want) for r in range(world)], res


def test_row_shard_halo_interp_sources_fetched_once_gloo():
    """Frames whose interpolated reference reads both sources whole fetch them
    once; later frames over the same sources move only their MV halos."""
    _run_world(_halo_interp_worker, 2, 192, 320, "ok")


def test_row_shard_halo_request_overflow_raises_everywhere_gloo():
    """A rank with more than MAX_REQ reference ranges flags the request table:
    every rank raises after the all-gather instead of one rank raising before it
    and the others blocking in the collective."""
    _run_world(_halo_overflow_worker, 2, 192, 320, "raised")


def _boundary_worker(rank, world, port, W, H, q):
    import torch.distributed as dist

    from thor_amd.shard import RowShard, rows_bytes

    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        rng = np.random.default_rng(13)
        nf = 6
        truth = {f: (rng.integers(0, 256, (H, W), dtype=np.uint8), rng.integers(0, 256, (H // 2, W // 2), dtype=np.uint8),
                     rng.integers(0, 256, (H // 2, W // 2), dtype=np.uint8)) for f in range(nf)}
        frames = {f: FakeFrame(f, W, H, rng, reach=6) for f in range(nf)}
        # intra CUs: every SB row of frame 0 (an I frame's serial chain across the bands), then
        # frame-dependent rows -- some bands' last rows ("late" edge), some first rows only ("early")
        for f in range(nf):
            b = frames[f].blocks
            if len(b) == 0:
                continue
            rows = b["ypos"].astype(np.int64) >> 6
            pick = np.isin(rows, [(f + k) % ((H + 63) // 64) for k in (0, 2)])
            b["mode"][pick & (np.arange(len(b)) % 2 == 0)] = 1
        ctx = NumpyContext(W, H, truth)
        ctx.halo = True
        ctx.frames = frames
        sh = RowShard(ctx, dist, W, H, device_exchange=False, band_local=True, halo=True, boundary=True)
        for f in range(nf):
            sh.decode(f, f, frames[f])
        full = rows_bytes(W, H)
        assert max(sh.boundary_bytes) < full // 4, (sh.boundary_bytes, full)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback

        q.put((rank, repr(e) + traceback.format_exc()[-800:]))


@pytest.mark.parametrize("world,W,H", [(2, 192, 320), (3, 128, 448), (8, 128, 2160), (8, 96, 1080)])
def test_row_shard_boundary_exchange_gloo(world, W, H):
    """Boundary mode: no pre-deblock all-gather -- the band below gets the two
    edge rows of the band above (after that band's intra chains when its last
    SB row holds intra CUs) before its own intra, then 8 deblocking halo rows
    either side; NumpyContext checks the edge rows at intra time and the band
    plus halos at deblocking time."""
    _run_world(_boundary_worker, world, W, H, "ok")


def test_boundary_plan():
    from thor_amd.shard import RowShard

    class D:
        def get_rank(self):
            return 1

        def get_world_size(self):
            return 3

    sh = object.__new__(RowShard)
    sh.H, sh.world, sh.rank = 448, 3, 1  # 7 SB rows, balanced bands: [0,3) [3,5) [5,7)
    fr = FakeFrame(1, 128, 448, np.random.default_rng(0), reach=2)
    fr.blocks["mode"][:] = 2
    assert sh.boundary_plan(fr) == {}
    rows = fr.blocks["ypos"] >> 6
    fr.blocks["mode"][np.flatnonzero(rows == 3)[:1]] = 1  # band 1's first row: band 0 hands over early
    assert sh.boundary_plan(fr) == {0: "early"}
    fr.blocks["mode"][np.flatnonzero(rows == 2)[:1]] = 1  # band 0's last row has intra: late
    fr.blocks["mode"][np.flatnonzero(rows == 6)[:1]] = 1  # band 2 has intra; band 1's last row (4) none
    assert sh.boundary_plan(fr) == {0: "late", 1: "early"}


@pytest.mark.parametrize("mode,world,W,H", [("gather", 3, 256, 200), ("local", 8, 128, 2160), ("halo", 3, 128, 448),
                                            ("boundary", 3, 128, 448), ("boundary", 8, 96, 1080)])
def test_fake_dist_carries_row_shard_protocols(mode, world, W, H):
    """tests/fake_dist.py (the thread-per-rank stand-in the device-exchange GPU
    test drives RowShard through) matches and orders every op of the gather,
    band-local, halo and boundary protocols as gloo does: the same NumpyContext
    checks pass with CPU tensors and no rank blocks."""
    import sys

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from fake_dist import run_ranks

    from thor_amd.shard import RowShard

    local, halo, boundary = mode != "gather", mode in ("halo", "boundary"), mode == "boundary"

    def body(rank, dist):
        rng = np.random.default_rng(13)  # same frames on every rank
        nf = 5
        truth = {f: (rng.integers(0, 256, (H, W), dtype=np.uint8), rng.integers(0, 256, (H // 2, W // 2), dtype=np.uint8),
                     rng.integers(0, 256, (H // 2, W // 2), dtype=np.uint8)) for f in range(nf)}
        frames = {f: FakeFrame(f, W, H, rng, reach=6) for f in range(nf)}
        for f in range(nf):
            b = frames[f].blocks
            if len(b):
                rows = b["ypos"].astype(np.int64) >> 6
                pick = np.isin(rows, [(f + k) % ((H + 63) // 64) for k in (0, 2)])
                b["mode"][pick & (np.arange(len(b)) % 2 == 0)] = 1
        ctx = NumpyContext(W, H, truth)
        if halo:
            ctx.halo = True
            ctx.frames = frames
        sh = RowShard(ctx, dist, W, H, device_exchange=False, band_local=local, halo=halo, boundary=boundary)
        for f in range(nf):
            sh.decode(f, f, frames[f])
        dist.barrier()
        return dist.bytes_moved

    moved = run_ranks(world, body)
    assert all(m > 0 for m in moved), moved
