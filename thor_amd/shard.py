"""Row-band sharding of ONE stream across ranks.

Every rank holds a full decoder context for the stream.  Per frame:

  1. thor_dec_frame_begin: side info, residuals, intra setup for the whole
     frame, inter reconstruction (k_recon) of the rank's band of SB rows only;
  2. all-gather of the bands' pre-deblock rows (thor_dec_get_rows /
     thor_dec_put_rows; put_rows also refreshes the SB-row edge rows the intra
     chains read) -- RCCL over xGMI with the nccl backend, host-staged with gloo;
  3. thor_dec_frame_end: intra (it reads neighbours across bands), deblock,
     CLPF and padding of the whole frame, replicated on every rank, so every
     rank ends the frame with the identical full reference.

With band_local=True, step 3 deblocks and CLPFs only the rank's band (the
deblocking's 2-row halo is already there from step 2), then:

  4. a second all-gather, of the bands' final rows;
  5. thor_dec_frame_finish: padding, the frame becomes a reference.

Each rank's loop filters then cover 1/N of the frame, for a second exchange of
the same size.  Every rank still ends the frame with the identical full
reference, so the next frame's motion vectors may reach anywhere.

With halo=True (band-local only), step 4 is replaced by an MV-reach halo
exchange at the start of the NEXT frames (variant 2): before
a frame's step 1 every rank works out, from the frame's parse output, which
rows of which reference frames the vectors of its band can reach (the 6-tap
luma / 4-tap chroma footprints, both signs of each vector component), drops the
rows it already holds final (its own band, and every halo it fetched before:
RowShard.final), the remaining requests are all-gathered, every owner sends the
parts of them that lie in its band (point to point, one grouped batch), and the
receivers write them into their copies of the references
(thor_dec_put_ref_rows) and re-pad those (thor_dec_pad_frame).  A rank then
holds final pixels only for its band plus the halos its vectors need; per
frame it moves one full-frame exchange (step 2: the whole-frame intra chains
read across bands) plus the halo rows it does not hold yet.  Frames with a
temporal-interpolated reference need both sources whole (the interpolation's
motion search spans the frame) -- fetched once per source, not per frame.

Bands are balanced: with S SB rows over N ranks, the first S mod N bands hold
floor(S / N) + 1 SB rows and the others floor(S / N) (4K, 34 rows over 8: 5, 5,
4, 4, 4, 4, 4, 4), so no band is empty while S >= N.  The all-gather slots are
sized for the largest band; each rank copies only its own rows.
"""
from __future__ import annotations

import numpy as np

MAX_REQ = 16  # reference ranges one rank may request per frame (MAX_REF_FRAMES-bounded lists: 4 references
# x 2 legs + 2 interpolation sources fit with room); a rank over it flags the table and every rank raises



def band_rows(height: int, world: int) -> int:
    """Luma rows of the largest band (whole SB rows): the all-gather slot size."""
    nsb = (height + 63) // 64
    return ((nsb + world - 1) // world) * 64


def band_of(height: int, world: int, rank: int):
    """(first SB row, end SB row) of `rank`'s band: balanced, the first
    nsb mod world bands one SB row taller (empty only when nsb < world)."""
    nsb = (height + 63) // 64
    q, r = divmod(nsb, world)

    def start(b):
        return b * q + min(b, r)

    return start(rank), start(rank + 1)


def band_bytes(width: int, height: int, world: int) -> int:
    rows = band_rows(height, world)
    return rows * width + 2 * (rows // 2) * (width // 2)


def rows_bytes(width: int, nrows: int) -> int:
    """Bytes of nrows luma rows + their chroma rows, packed as get_rows packs them."""
    return nrows * width + 2 * (nrows // 2) * (width // 2)


def halo_requests(frame, height: int, r0: int, r1: int):
    """{reference frame_num: (lo, hi)} -- the luma rows (even-aligned, inside
    the frame) of each reference that the inter CUs of luma rows [r0, r1) of
    `frame` (a parse-output Frame) can read: per CU and prediction leg, the CU's
    rows widened by its largest vertical vector component (either sign, the
    decoder negates vectors toward later references) in whole pixels plus the
    6-tap footprint (-2 .. +3) and a margin; the chroma 4-tap footprint (-1 ..
    +2 chroma rows) lies inside that.  A frame with a temporal-interpolated
    reference (-2) needs both its sources whole (interpolate_frames reads them
    all)."""
    b = frame.blocks
    req = {}

    def add(f, lo, hi):
        lo, hi = max(0, int(lo) & ~1), min(height, (int(hi) + 1) & ~1)
        if hi <= lo:
            return
        if f in req:
            a, c = req[f]
            req[f] = (min(a, lo), max(c, hi))
        else:
            req[f] = (lo, hi)

    if getattr(frame, "interp_ratio", 0) > 0:  # the interpolated reference is built from both sources whole
        for src in frame.interp_refs:
            if src >= 0:
                add(int(src), 0, height)
    if len(b) == 0:
        return req
    mode = b["mode"].astype(np.int64)
    y = b["ypos"].astype(np.int64)
    hgt = b["bheight"].astype(np.int64)
    sel = (mode != 1) & (y >= r0) & (y < r1)
    bi = (mode == 3) | (((mode == 0) | (mode == 4)) & (b["dir"] == 2))
    for leg, refk, mvk in ((0, "ref0", "mv0"), (1, "ref1", "mv1")):
        m = sel & (bi if leg else True)
        if not np.any(m):
            continue
        mvy = np.abs(b[mvk][:, 1::2].astype(np.int64)).max(axis=1)
        reach = (mvy + 3) // 4 + 6
        for f, lo, hi in zip(b[refk][m], (y - reach)[m], (y + hgt + reach)[m]):
            f = int(f)
            if f >= 0:  # (-2, the interpolated reference, is covered above)
                add(f, lo, hi)
    return req



class RowShard:
    """Drives one rank's decoder context through band-sharded frames.

    `dec` is a thor_amd.decoder.GpuDecoder (or any object with the same
    begin/get_rows/put_rows/end methods, as the CPU tests use); `dist` is
    torch.distributed, initialised; `device_exchange` selects device buffers
    (nccl/RCCL) or host staging (gloo)."""

    def __init__(self, dec, dist, width: int, height: int, device_exchange: bool, band_local: bool = False,
                 halo: bool = False, boundary: bool = False):
        if halo and not band_local:
            raise ValueError("the halo exchange replaces band-local phase B's second all-gather")
        if boundary and not halo:
            raise ValueError("the boundary exchange replaces the first all-gather of the halo mode")
        self.boundary = boundary
        self.boundary_bytes = []  # per frame: bytes this rank received in the boundary exchange
        self.halo = halo
        self.halo_bytes = []  # per frame: bytes this rank received in halo exchanges
        self.final = {}  # halo mode: frame_num -> sorted disjoint luma row ranges this rank holds final
        self.decoded = []  # halo mode: frame numbers in decode order (the last `window` keep their `final` entry)
        self.window = 34  # MAX_SLOTS (thor_amd/decoder.py): a frame further back is no longer a reference
        self.dec, self.dist = dec, dist
        self.W, self.H = width, height
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.rows = band_rows(height, self.world)
        self.nbytes = band_bytes(width, height, self.world)
        self.device_exchange = device_exchange
        b0, b1 = band_of(height, self.world, self.rank)
        dec.set_band(b0, b1)
        self.band_local = band_local
        if band_local:
            dec.set_band_local(True)
        if halo and hasattr(dec, "set_band_pad"):  # only the band's rows are final here: pad just those
            dec.set_band_pad(True)
        if boundary:
            if any(self.owned(q)[1] - self.owned(q)[0] < 8 for q in range(self.world)):
                raise ValueError("the boundary exchange needs every band at least 8 rows high")
            dec.set_band_intra(True)
        import torch

        self.dstream = None
        if device_exchange:
            dev = torch.device("cuda", torch.cuda.current_device())
            # the band copies run on the decoder's stream, the collective on
            # torch's current stream: events order them both ways (decode())
            if hasattr(dec, "stream"):
                self.dstream = torch.cuda.ExternalStream(dec.stream(), device=dev)
            self.send = torch.empty(self.nbytes, dtype=torch.uint8, device=dev)
            self.recv = torch.empty(self.world * self.nbytes, dtype=torch.uint8, device=dev)
        else:
            self.send = torch.empty(self.nbytes, dtype=torch.uint8)
            self.recv = [torch.empty(self.nbytes, dtype=torch.uint8) for _ in range(self.world)]
            self.scratch = [dec.scratch(self.nbytes) for _ in range(self.world)]
        if halo:  # one full-frame staging buffer per peer (a halo may be a whole reference)
            self.fbytes = rows_bytes(width, height + (height & 1))
            self.hbuf = [dec.scratch(self.fbytes) for _ in range(self.world)]
        if boundary and not device_exchange:  # host staging of the boundary pieces (edge, 4 halo pieces)
            self.bscratch = [dec.scratch(rows_bytes(width, self.HALO_ROWS)) for _ in range(6)]

    def owned(self, rank: int):
        """Luma rows [lo, hi) of the frame `rank` holds final."""
        b0, b1 = band_of(self.H, self.world, rank)
        return min(64 * b0, self.H), min(64 * b1, self.H)

    def decode(self, devframe, frame_num: int, frame=None):
        """One frame: `devframe` is the decoder's uploaded parse output;
        halo mode also needs `frame`, the parse output (its blocks name the
        references and vectors)."""
        d = self.dec
        if self.halo:
            self._fetch_halo(frame)
            self.final[int(frame_num)] = []  # (re)decoded: only this rank's band is final
            self._retire(int(frame_num))
            lo, hi = self.owned(self.rank)
            if hi > lo:
                self._hold(frame_num, lo, hi)
        d.begin(devframe)
        if self.boundary:
            self._boundary(frame_num, frame)  # edge rows for the intra chains, deblocking halos
        else:
            self._exchange(frame_num)  # the bands' pre-deblock rows (inter reconstruction)
        d.end()
        if self.band_local:
            if not self.halo:
                self._exchange(frame_num)  # the bands' final rows (intra, deblocked, CLPF'd)
            d.finish()

    def _fetch_halo(self, frame):
        """Before `frame`'s band reconstruction: every rank's reference rows
        within its vectors' reach that it does not already hold final, from
        their owners (point to point)."""
        import torch

        d, dist = self.dec, self.dist
        r0, r1 = self.owned(self.rank)
        req = self.missing(halo_requests(frame, self.H, r0, r1))
        mine = np.full((MAX_REQ, 3), -1, np.int32)
        if len(req) > MAX_REQ:  # flagged in the table: every rank raises after the all-gather, none blocks
            mine[0] = (-2, len(req), 0)
        else:
            for k, (f, lo, hi) in enumerate(req):
                mine[k] = (f, lo, hi)
        dev = torch.device("cuda", torch.cuda.current_device()) if self.device_exchange else None
        table = [torch.empty((MAX_REQ, 3), dtype=torch.int32, device=dev) for _ in range(self.world)]
        dist.all_gather(table, torch.from_numpy(mine).to(dev) if dev is not None else torch.from_numpy(mine))
        table = [t.cpu().numpy() for t in table]
        over = [q for q in range(self.world) if table[q][0][0] == -2]
        if over:
            raise ValueError("rank(s) %s need more than %d reference ranges in one frame" % (over, MAX_REQ))

        def parts(q, p):  # the (frame, lo, hi) pieces rank q asked for that rank p owns
            plo, phi = self.owned(p)
            out = []
            for f, lo, hi in table[q]:
                if f < 0:
                    continue
                a, c = max(lo, plo), min(hi, phi)
                if c > a:
                    out.append((int(f), int(a), int(c)))
            return out

        for p in range(self.world):  # what this rank receives is final from now on
            if p != self.rank:
                for f, a, c in parts(self.rank, p):
                    self._hold(f, a, c)
        if self.device_exchange:
            self.halo_bytes.append(self._fetch_halo_device(parts, dev))
            return
        # host-staged point to point (gloo): sends from this rank's final rows, receives into
        # numpy, one grouped batch, then into the references in order (one staging buffer per
        # peer, synchronised)
        ops, recvs, keep, got = [], [], [], 0
        for q in range(self.world):
            if q == self.rank:
                continue
            for f, a, c in parts(q, self.rank):
                buf = np.empty(rows_bytes(self.W, c - a), np.uint8)
                d.get_rows(f, a, c - a, self.hbuf[q])
                d.d2h(buf, self.hbuf[q])
                ops.append(dist.P2POp(dist.isend, torch.from_numpy(buf), q))
                keep.append(buf)
        for p in range(self.world):
            if p == self.rank:
                continue
            for f, a, c in parts(self.rank, p):
                t = torch.empty(rows_bytes(self.W, c - a), dtype=torch.uint8)
                ops.append(dist.P2POp(dist.irecv, t, p))
                recvs.append((t, p, f, a, c))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        padded = set()
        for t, p, f, a, c in recvs:
            d.h2d(self.hbuf[p], t.numpy())
            d.put_ref_rows(f, a, c - a, self.hbuf[p])
            d.sync()  # the staging buffer is reused by the next piece from p
            padded.add(f)
            got += t.numel()
        for f in sorted(padded):
            d.pad_frame(f)
        self.halo_bytes.append(got)

    # ---- boundary exchange (replaces the pre-deblock all-gather) ----
    HALO_ROWS = 8  # pre-deblock rows either side of a band its deblocking reads (3 needed, 8-row groups)

    def boundary_plan(self, frame):
        """Which ranks hand their band's bottom edge rows to the rank below this
        frame, and when: {rank: "early" | "late"} -- "early" (right after the
        band's inter reconstruction) when the band's last SB row holds no intra
        CU, "late" (after its intra chains) otherwise; only toward a band that
        has intra CUs (its first chain reads the row above).  Every rank derives
        the same plan from the frame's parse output."""
        b = frame.blocks
        intra_rows = set((b["ypos"][b["mode"] == 1].astype(np.int64) >> 6).tolist()) if len(b) else set()
        plan = {}
        for r in range(self.world - 1):
            a0, a1 = band_of(self.H, self.world, r)
            c0, c1 = band_of(self.H, self.world, r + 1)
            if a1 <= a0 or c1 <= c0 or not any(c0 <= y < c1 for y in intra_rows):
                continue
            plan[r] = "late" if (a1 - 1) in intra_rows else "early"
        return plan

    def _boundary(self, frame_num: int, frame):
        """Between the band's inter reconstruction and its deblocking: (1) the
        edge rows -- the two luma rows ending the band above (and their chroma
        row) -- from the rank above, whose intra chains may write them, before
        this band's intra chains (thor_dec_frame_intra, the band's rows only);
        (2) after intra, HALO_ROWS pre-deblock rows either side of the band,
        grouped both ways, for the band-local deblocking.  Bytes per rank and
        frame: 3W per edge + 2 x 1.5 x HALO_ROWS x W, against a whole frame in
        the all-gather."""
        d, r = self.dec, self.rank
        plan = self.boundary_plan(frame)
        got = 0
        lo, hi = self.owned(r)
        if r in plan and plan[r] == "early":
            self._send_rows(frame_num, hi - 2, 2, r + 1)
        if (r - 1) in plan:
            got += self._recv_rows(frame_num, lo - 2, 2, r - 1)
        d.intra()
        if r in plan and plan[r] == "late":
            self._send_rows(frame_num, hi - 2, 2, r + 1)
        h = self.HALO_ROWS
        pieces = []  # (peer, y0, n, send?)
        if r > 0 and hi > lo:
            pieces += [(r - 1, lo, min(h, self.H - lo), True), (r - 1, lo - h, h, False)]
        if r + 1 < self.world and hi > lo and hi < self.H:
            pieces += [(r + 1, hi - h, h, True), (r + 1, hi, min(h, self.H - hi), False)]
        got += self._swap_rows(frame_num, pieces)
        self.boundary_bytes.append(got)

    def _stage(self, nbytes):
        import torch

        if self.device_exchange:
            return torch.empty(nbytes, dtype=torch.uint8, device=torch.device("cuda", torch.cuda.current_device()))
        return torch.empty(nbytes, dtype=torch.uint8)

    def _rows_out(self, frame_num, y0, n, t, k):
        """Rows [y0, y0 + n) of the frame into staging tensor t (host path: via scratch k)."""
        d = self.dec
        if self.device_exchange:
            d.get_rows(frame_num, y0, n, t.data_ptr())
        else:
            d.get_rows(frame_num, y0, n, self.bscratch[k])
            d.d2h(t.numpy(), self.bscratch[k])

    def _rows_in(self, frame_num, y0, n, t, k):
        d = self.dec
        if self.device_exchange:
            d.put_rows(frame_num, y0, n, t.data_ptr())
        else:
            d.h2d(self.bscratch[k], t.numpy())
            d.put_rows(frame_num, y0, n, self.bscratch[k])
            d.sync()  # the scratch buffer is reused

    def _order(self, to_torch: bool):
        """Order the decoder stream's copies before (to_torch) or after torch's stream (device path)."""
        if self.device_exchange and self.dstream is not None:
            import torch

            cur = torch.cuda.current_stream()
            ev = torch.cuda.Event()
            if to_torch:
                ev.record(self.dstream)
                cur.wait_event(ev)
            else:
                ev.record(cur)
                self.dstream.wait_event(ev)

    def _keep(self, ts):
        if self.device_exchange and self.dstream is not None:
            for t in ts:
                t.record_stream(self.dstream)

    def _send_rows(self, frame_num, y0, n, peer):
        t = self._stage(rows_bytes(self.W, n))
        self._rows_out(frame_num, y0, n, t, 0)
        self._order(True)
        self.dist.send(t, peer)
        self._keep([t])

    def _recv_rows(self, frame_num, y0, n, peer):
        t = self._stage(rows_bytes(self.W, n))
        self.dist.recv(t, peer)
        self._order(False)
        self._rows_in(frame_num, y0, n, t, 1)
        self._keep([t])
        return t.numel()

    def _swap_rows(self, frame_num, pieces):
        """One grouped batch of sends and receives of row ranges: [(peer, y0, n, is_send)]."""
        if not pieces:
            return 0
        ops, recvs, keep = [], [], []
        for k, (peer, y0, n, snd) in enumerate(pieces):
            t = self._stage(rows_bytes(self.W, n))
            if snd:
                self._rows_out(frame_num, y0, n, t, 2 + k)
                ops.append(self.dist.P2POp(self.dist.isend, t, peer))
            else:
                ops.append(self.dist.P2POp(self.dist.irecv, t, peer))
                recvs.append((y0, n, t, 2 + k))
            keep.append(t)
        self._order(True)
        for w in self.dist.batch_isend_irecv(ops):
            w.wait()
        self._order(False)
        got = 0
        for y0, n, t, k in recvs:
            self._rows_in(frame_num, y0, n, t, k)
            got += t.numel()
        self._keep(keep)
        return got

    def _exchange(self, frame_num: int):
        """All-gather of the bands' rows: rank r's slot holds its owned rows
        [lo, hi), packed as get_rows packs hi - lo rows (slots sized for the
        largest band)."""
        d = self.dec
        y0, y1 = self.owned(self.rank)
        if self.device_exchange:
            import torch

            if y1 > y0:
                d.get_rows(frame_num, y0, y1 - y0, self.send.data_ptr())
            cur = torch.cuda.current_stream()
            if self.dstream is not None:  # the band rows are in `send` before the all-gather reads them
                ev = torch.cuda.Event()
                ev.record(self.dstream)
                cur.wait_event(ev)
            self.dist.all_gather_into_tensor(self.recv, self.send)
            if self.dstream is not None:  # put_rows (and the next frame's get_rows) after the all-gather
                ev = torch.cuda.Event()
                ev.record(cur)
                self.dstream.wait_event(ev)
            for r in range(self.world):
                a, b = self.owned(r)
                if r != self.rank and b > a:
                    d.put_rows(frame_num, a, b - a, self.recv.data_ptr() + r * self.nbytes)
        else:
            if y1 > y0:
                d.get_rows(frame_num, y0, y1 - y0, self.scratch[self.rank])
                d.d2h(self.send.numpy(), self.scratch[self.rank])  # waits for the decoder's stream
            self.dist.all_gather(self.recv, self.send)
            for r in range(self.world):
                a, b = self.owned(r)
                if r != self.rank and b > a:
                    d.h2d(self.scratch[r], self.recv[r].numpy())
                    d.put_rows(frame_num, a, b - a, self.scratch[r])

    def _fetch_halo_device(self, parts, dev):
        """_fetch_halo's data movement with device buffers (nccl = RCCL point
        to point): get_rows on the decoder's stream -> event -> one grouped
        batch of every isend and irecv on torch's stream (dist.batch_isend_irecv,
        i.e. one RCCL group: no send waits on a peer's unposted receive) ->
        event -> put_ref_rows on the decoder's stream.  The staging tensors are
        recorded on the decoder's stream, so the caching allocator keeps them
        until its copies are done -- no host synchronisation.  Returns the
        bytes received."""
        import torch

        d, dist = self.dec, self.dist
        cur = torch.cuda.current_stream()
        ops, recvs, keep, got = [], [], [], 0
        for q in range(self.world):
            if q == self.rank:
                continue
            for f, a, c in parts(q, self.rank):
                t = torch.empty(rows_bytes(self.W, c - a), dtype=torch.uint8, device=dev)
                d.get_rows(f, a, c - a, t.data_ptr())
                ops.append(dist.P2POp(dist.isend, t, q))
                keep.append(t)
        for p in range(self.world):
            if p == self.rank:
                continue
            for f, a, c in parts(self.rank, p):
                t = torch.empty(rows_bytes(self.W, c - a), dtype=torch.uint8, device=dev)
                ops.append(dist.P2POp(dist.irecv, t, p))
                recvs.append((t, f, a, c))
                keep.append(t)
        if not ops:
            return 0
        if self.dstream is not None:  # the sent rows are staged before the group reads them
            ev = torch.cuda.Event()
            ev.record(self.dstream)
            cur.wait_event(ev)
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        if self.dstream is not None:  # the received rows land before the decoder stream reads them
            ev = torch.cuda.Event()
            ev.record(cur)
            self.dstream.wait_event(ev)
        padded = set()
        for t, f, a, c in recvs:
            d.put_ref_rows(f, a, c - a, t.data_ptr())
            padded.add(f)
            got += t.numel()
        for f in sorted(padded):
            d.pad_frame(f)
        if self.dstream is not None:
            for t in keep:  # freed only after the decoder stream's copies
                t.record_stream(self.dstream)
        else:
            d.sync()  # no stream to record on: the staging tensors may be freed after this
        return got

    # ---- which rows of which frames this rank holds final (halo mode) ----
    def _retire(self, f: int):
        """Frame f was just decoded: forget what this rank holds of frames that
        left the reference window (so `final` stays bounded over a long stream)."""
        if f in self.decoded:
            self.decoded.remove(f)
        self.decoded.append(f)
        while len(self.decoded) > self.window:
            self.final.pop(self.decoded.pop(0), None)

    def _hold(self, f: int, a: int, c: int):
        iv = self.final.setdefault(int(f), [])
        iv.append((int(a), int(c)))
        iv.sort()
        merged = []
        for lo, hi in iv:
            if merged and lo <= merged[-1][1]:
                merged[-1] = (merged[-1][0], max(merged[-1][1], hi))
            else:
                merged.append((lo, hi))
        self.final[int(f)] = merged

    def missing(self, req):
        """[(frame, lo, hi)]: the parts of the requested row ranges {frame: (lo,
        hi)} this rank does not hold final yet (even-aligned, sorted)."""
        out = []
        for f, (lo, hi) in sorted(req.items()):
            cur = lo
            for a, c in self.final.get(int(f), []):
                if c <= cur or a >= hi:
                    continue
                if a > cur:
                    out.append((int(f), cur, min(a, hi)))
                cur = max(cur, c)
                if cur >= hi:
                    break
            if cur < hi:
                out.append((int(f), cur, hi))
        return [(f, a & ~1, (c + 1) & ~1) for f, a, c in out]

    def assemble(self, frame_num: int) -> bytes:
        """The whole frame (I420 bytes) from its bands' owners (one all-gather;
        a check outside any timed region -- in halo mode no rank holds every
        row final)."""
        import torch

        d, W, H, world = self.dec, self.W, self.H, self.world
        mine = np.zeros(self.nbytes, np.uint8)
        lo, hi = self.owned(self.rank)
        if hi > lo:
            buf = d.scratch(self.nbytes)
            d.get_rows(frame_num, lo, hi - lo, buf)
            d.d2h(mine, buf)
        dev = torch.device("cuda", torch.cuda.current_device()) if self.device_exchange else None
        src = torch.from_numpy(mine).to(dev) if dev is not None else torch.from_numpy(mine)
        parts = [torch.empty(self.nbytes, dtype=torch.uint8, device=dev) for _ in range(world)]
        self.dist.all_gather(parts, src)
        y = np.zeros((H, W), np.uint8)
        u = np.zeros((H // 2, W // 2), np.uint8)
        v = np.zeros((H // 2, W // 2), np.uint8)
        for r in range(world):
            a, b = self.owned(r)
            n = b - a
            if n <= 0:
                continue
            p = parts[r].cpu().numpy()
            y[a:b] = p[:n * W].reshape(n, W)
            o = n * W
            for pl in (u, v):
                pl[a // 2:b // 2] = p[o:o + (n // 2) * (W // 2)].reshape(n // 2, W // 2)
                o += (n // 2) * (W // 2)
        return y.tobytes() + u.tobytes() + v.tobytes()
