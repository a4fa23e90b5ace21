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
luma / 4-tap chroma footprints, both signs of each vector component), the
requests are all-gathered, every owner sends the parts of them that lie in its
band (point to point), and the receivers write them into their copies of the
references (thor_dec_put_ref_rows) and re-pad those (thor_dec_pad_frame).  A
rank then holds final pixels only for its band plus the halos its vectors
need; per frame it moves one full-frame exchange (step 2: the whole-frame
intra chains read across bands) plus its halos, instead of two full ones.
Frames with a temporal-interpolated reference fetch both sources whole (the
interpolation's motion search spans the frame).

Band b covers SB rows [b*R, (b+1)*R), R = ceil(SB rows / world); the last band
may run past the frame (those rows are not copied).
"""
from __future__ import annotations

import numpy as np

MAX_REQ = 8  # reference ranges one rank may request per frame (4 references x 2 legs)



def band_rows(height: int, world: int) -> int:
    """Luma rows per band: whole SB rows, equal for every rank (all-gather)."""
    nsb = (height + 63) // 64
    return ((nsb + world - 1) // world) * 64


def band_of(height: int, world: int, rank: int):
    """(first SB row, end SB row) of `rank`'s band (end clamped to the frame)."""
    nsb = (height + 63) // 64
    r = band_rows(height, world) // 64
    return min(rank * r, nsb), min((rank + 1) * r, nsb)


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
                 halo: bool = False):
        if halo and not band_local:
            raise ValueError("the halo exchange replaces band-local phase B's second all-gather")
        self.halo = halo
        self.halo_bytes = []  # per frame: bytes this rank received in halo exchanges
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
        d.begin(devframe)
        self._exchange(frame_num)  # the bands' pre-deblock rows (inter reconstruction)
        d.end()
        if self.band_local:
            if not self.halo:
                self._exchange(frame_num)  # the bands' final rows (intra, deblocked, CLPF'd)
            d.finish()

    def _fetch_halo(self, frame):
        """Before `frame`'s band reconstruction: every rank's reference rows
        within its vectors' reach, from their owners (point to point)."""
        import torch

        d, dist = self.dec, self.dist
        r0, r1 = self.owned(self.rank)
        req = halo_requests(frame, self.H, r0, r1)
        if len(req) > MAX_REQ:
            raise ValueError("more than %d reference ranges in one frame" % MAX_REQ)
        mine = np.full((MAX_REQ, 3), -1, np.int32)
        for k, (f, (lo, hi)) in enumerate(sorted(req.items())):
            mine[k] = (f, lo, hi)
        dev = torch.device("cuda", torch.cuda.current_device()) if self.device_exchange else None
        table = [torch.empty((MAX_REQ, 3), dtype=torch.int32, device=dev) for _ in range(self.world)]
        dist.all_gather(table, torch.from_numpy(mine).to(dev) if dev is not None else torch.from_numpy(mine))
        table = [t.cpu().numpy() for t in table]

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

        if self.device_exchange:
            self.halo_bytes.append(self._fetch_halo_device(parts, dev))
            return
        # host-staged point to point (gloo): sends from this rank's final rows, receives into
        # numpy, then into the references in order (one staging buffer per peer, synchronised)
        sends, recvs, got = [], [], 0
        for q in range(self.world):
            if q == self.rank:
                continue
            for f, a, c in parts(q, self.rank):
                buf = np.empty(rows_bytes(self.W, c - a), np.uint8)
                d.get_rows(f, a, c - a, self.hbuf[q])
                d.d2h(buf, self.hbuf[q])
                sends.append((dist.isend(torch.from_numpy(buf), q), buf))
        for p in range(self.world):
            if p == self.rank:
                continue
            for f, a, c in parts(self.rank, p):
                t = torch.empty(rows_bytes(self.W, c - a), dtype=torch.uint8)
                recvs.append((dist.irecv(t, p), t, p, f, a, c))
        padded = set()
        for w, t, p, f, a, c in recvs:
            w.wait()
            d.h2d(self.hbuf[p], t.numpy())
            d.put_ref_rows(f, a, c - a, self.hbuf[p])
            d.sync()  # the staging buffer is reused by the next piece from p
            padded.add(f)
            got += t.numel()
        for w, _ in sends:
            w.wait()
        for f in sorted(padded):
            d.pad_frame(f)
        self.halo_bytes.append(got)

    def _exchange(self, frame_num: int):
        d = self.dec
        y0 = self.rank * self.rows
        if self.device_exchange:
            import torch

            d.get_rows(frame_num, y0, self.rows, self.send.data_ptr())
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
                if r != self.rank:
                    d.put_rows(frame_num, r * self.rows, self.rows, self.recv.data_ptr() + r * self.nbytes)
        else:
            d.get_rows(frame_num, y0, self.rows, self.scratch[self.rank])
            d.d2h(self.send.numpy(), self.scratch[self.rank])  # waits for the decoder's stream
            self.dist.all_gather(self.recv, self.send)
            for r in range(self.world):
                if r != self.rank:
                    d.h2d(self.scratch[r], self.recv[r].numpy())
                    d.put_rows(frame_num, r * self.rows, self.rows, self.scratch[r])

    def _fetch_halo_device(self, parts, dev):
        """_fetch_halo's data movement with device buffers (nccl = RCCL point
        to point): get_rows on the decoder's stream -> event -> isend on
        torch's stream; irecv -> event -> put_ref_rows on the decoder's
        stream.  Returns the bytes received."""
        import torch

        d, dist = self.dec, self.dist
        cur = torch.cuda.current_stream()
        sends, keep, got = [], [], 0
        for q in range(self.world):
            if q == self.rank:
                continue
            for f, a, c in parts(q, self.rank):
                t = torch.empty(rows_bytes(self.W, c - a), dtype=torch.uint8, device=dev)
                d.get_rows(f, a, c - a, t.data_ptr())
                if self.dstream is not None:
                    ev = torch.cuda.Event()
                    ev.record(self.dstream)
                    cur.wait_event(ev)
                sends.append(dist.isend(t, q))
                keep.append(t)
        recvs = []
        for p in range(self.world):
            if p == self.rank:
                continue
            for f, a, c in parts(self.rank, p):
                t = torch.empty(rows_bytes(self.W, c - a), dtype=torch.uint8, device=dev)
                recvs.append((dist.irecv(t, p), t, f, a, c))
        padded = set()
        for w, t, f, a, c in recvs:
            w.wait()
            if self.dstream is not None:
                ev = torch.cuda.Event()
                ev.record(cur)
                self.dstream.wait_event(ev)
            d.put_ref_rows(f, a, c - a, t.data_ptr())
            keep.append(t)
            padded.add(f)
            got += t.numel()
        for w in sends:
            w.wait()
        for f in sorted(padded):
            d.pad_frame(f)
        d.sync()  # the staging tensors may be freed
        return got
