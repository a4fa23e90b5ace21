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

Band b covers SB rows [b*R, (b+1)*R), R = ceil(SB rows / world); the last band
may run past the frame (those rows are not copied).
"""
from __future__ import annotations



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


class RowShard:
    """Drives one rank's decoder context through band-sharded frames.

    `dec` is a thor_amd.decoder.GpuDecoder (or any object with the same
    begin/get_rows/put_rows/end methods, as the CPU tests use); `dist` is
    torch.distributed, initialised; `device_exchange` selects device buffers
    (nccl/RCCL) or host staging (gloo)."""

    def __init__(self, dec, dist, width: int, height: int, device_exchange: bool, band_local: bool = False):
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

    def decode(self, devframe, frame_num: int):
        d = self.dec
        d.begin(devframe)
        self._exchange(frame_num)  # the bands' pre-deblock rows (inter reconstruction)
        d.end()
        if self.band_local:
            self._exchange(frame_num)  # the bands' final rows (intra, deblocked, CLPF'd)
            d.finish()

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
