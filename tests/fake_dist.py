"""An in-process stand-in for torch.distributed with the nccl (RCCL) backend's
stream semantics, one thread per rank, every rank's tensors on the same GPU --
test infrastructure only.

The GPU box has one card, so RCCL cannot run two ranks there; this lets the
device-exchange branches of thor_amd/shard.py (device staging tensors, the
decoder stream, the events between it and the collective's stream) run with
several ranks and partial bands on one GPU.  The ordering model is nccl's:

  * a collective or point-to-point op is enqueued on the calling thread's
    current torch stream; it reads its inputs after everything already on that
    stream (an event recorded at the call), and later work on that stream runs
    after the op has finished on every rank it involves (the peers' copies'
    events are waited on before the call returns);
  * point-to-point ops match in posting order per (src, dst) pair; a blocking
    send returns once the receiver has enqueued its copy (host-side), a
    grouped batch posts all its sends before it takes any receive, so the
    batch needs no peer's receive to be posted first;
  * work.wait() is stream-side, as nccl's: it returns at once.

The data moves with copies on the receiving rank's stream.  Every rank should
give its thread its own current stream (torch.cuda.stream(...)); with the
shared default stream the ordering would be trivially serial.  A rank that
raises breaks every other rank's wait (FakeWorld.abort), so a failing test
ends instead of hanging."""
import collections
import threading

import torch

TIMEOUT = 60.0


class FakeWorld:
    def __init__(self, n: int):
        self.n = n
        self.cond = threading.Condition()
        self.box = collections.defaultdict(collections.deque)  # (src, dst) -> posted sends
        self.bar = threading.Barrier(n, timeout=TIMEOUT)
        self.slots = {}  # collective sequence number -> {rank: (tensor, ready event)}
        self.done = {}  # collective sequence number -> {rank: done event}
        self.broken = False

    def abort(self):
        with self.cond:
            self.broken = True
            self.cond.notify_all()
        self.bar.abort()

    def dist(self, rank: int) -> "FakeDist":
        return FakeDist(self, rank)


class _Post:
    __slots__ = ("tensor", "ready", "done", "taken")

    def __init__(self, tensor, ready):
        self.tensor, self.ready, self.done, self.taken = tensor, ready, None, False


class _Work:
    def wait(self):
        return True


class P2POp:
    def __init__(self, op, tensor, peer):
        self.op, self.tensor, self.peer = op, tensor, peer


class _NoStream:
    """CPU tensors (the no-GPU self-test): copies are synchronous, no events."""

    def wait_event(self, ev):
        pass


def _cur():
    return torch.cuda.current_stream() if torch.cuda.is_available() else _NoStream()


def _event(stream):
    if isinstance(stream, _NoStream):
        return None
    ev = torch.cuda.Event()
    ev.record(stream)
    return ev


class FakeDist:
    """The subset of torch.distributed RowShard uses."""

    P2POp = P2POp

    def __init__(self, world: FakeWorld, rank: int):
        self.w, self.rank, self.seq = world, rank, 0
        self.bytes_moved = 0

    def get_rank(self):
        return self.rank

    def get_world_size(self):
        return self.w.n

    # markers for P2POp (torch.distributed.isend / irecv)
    def isend(self, tensor, dst):  # pragma: no cover - only its identity is used
        raise NotImplementedError

    def irecv(self, tensor, src):  # pragma: no cover
        raise NotImplementedError

    # ---- point to point ----
    def _wait_for(self, pred):
        w = self.w
        with w.cond:
            if not w.cond.wait_for(lambda: w.broken or pred(), timeout=TIMEOUT):
                raise TimeoutError("fake_dist: rank %d timed out" % self.rank)
            if w.broken:
                raise RuntimeError("fake_dist: another rank failed")

    def _post(self, tensor, dst):
        assert tensor.is_contiguous()
        p = _Post(tensor, _event(_cur()))
        with self.w.cond:
            self.w.box[(self.rank, dst)].append(p)
            self.w.cond.notify_all()
        return p

    def _take(self, tensor, src):
        key = (src, self.rank)
        self._wait_for(lambda: len(self.w.box[key]) > 0)
        with self.w.cond:
            p = self.w.box[key].popleft()
        if p.tensor.numel() != tensor.numel() or p.tensor.dtype != tensor.dtype:
            raise ValueError("fake_dist: rank %d receives %d x %s from rank %d, which sent %d x %s" % (
                self.rank, tensor.numel(), tensor.dtype, src, p.tensor.numel(), p.tensor.dtype))
        cur = _cur()
        cur.wait_event(p.ready)  # the sender's stream has staged the data
        tensor.copy_(p.tensor)
        self.bytes_moved += tensor.numel() * tensor.element_size()
        with self.w.cond:
            p.done, p.taken = _event(cur), True
            self.w.cond.notify_all()

    def _settle(self, posts):
        """Later work on this rank's stream waits for its sends' copies (the
        sender may reuse a send buffer once the op is done)."""
        self._wait_for(lambda: all(p.taken for p in posts))
        cur = _cur()
        for p in posts:
            cur.wait_event(p.done)

    def send(self, tensor, dst):
        self._settle([self._post(tensor, dst)])

    def recv(self, tensor, src):
        self._take(tensor, src)

    def batch_isend_irecv(self, ops):
        posts = [self._post(o.tensor, o.peer) for o in ops if o.op == self.isend]
        for o in ops:
            if o.op == self.irecv:
                self._take(o.tensor, o.peer)
            elif o.op != self.isend:
                raise ValueError("fake_dist: P2POp needs isend or irecv")
        self._settle(posts)
        return [_Work() for _ in ops]

    # ---- collectives ----
    def _gather(self, tensor):
        """Every rank's (tensor, ready event) for this collective, in rank order."""
        seq, self.seq = self.seq, self.seq + 1
        w = self.w
        with w.cond:
            w.slots.setdefault(seq, {})[self.rank] = (tensor, _event(_cur()))
        self._barrier()
        with w.cond:
            got = [w.slots[seq][r] for r in range(w.n)]
        return seq, got

    def _finish(self, seq):
        w = self.w
        with w.cond:
            w.done.setdefault(seq, {})[self.rank] = _event(_cur())
        self._barrier()
        cur = _cur()
        with w.cond:
            evs = [w.done[seq][r] for r in range(w.n)]
        for ev in evs:  # a peer's copy out of this rank's input is done before the input changes
            cur.wait_event(ev)
        self._barrier()
        if self.rank == 0:
            with w.cond:
                w.slots.pop(seq, None)
                w.done.pop(seq, None)

    def all_gather_into_tensor(self, out, tensor):
        seq, got = self._gather(tensor)
        n = tensor.numel()
        if out.numel() != n * self.w.n:
            raise ValueError("fake_dist: all_gather_into_tensor output is not world x input")
        cur = _cur()
        for r, (t, ev) in enumerate(got):
            cur.wait_event(ev)
            out[r * n:(r + 1) * n].copy_(t.reshape(-1))
            if r != self.rank:
                self.bytes_moved += n * t.element_size()
        self._finish(seq)
        return _Work()

    def all_gather(self, out_list, tensor):
        seq, got = self._gather(tensor)
        cur = _cur()
        for r, (t, ev) in enumerate(got):
            cur.wait_event(ev)
            out_list[r].copy_(t)
            if r != self.rank:
                self.bytes_moved += t.numel() * t.element_size()
        self._finish(seq)
        return _Work()

    def _barrier(self):
        try:
            self.w.bar.wait()
        except threading.BrokenBarrierError:
            raise RuntimeError("fake_dist: another rank failed or timed out") from None

    def barrier(self):
        self._barrier()


def run_ranks(n: int, body):
    """Run body(rank, dist) on n threads, each on its own current stream;
    returns the per-rank results (re-raises the first rank's exception)."""
    world = FakeWorld(n)
    out, err = [None] * n, [None] * n
    gpu = torch.cuda.is_available()
    dev = torch.cuda.current_device() if gpu else None

    def thread(r):
        try:
            if not gpu:
                out[r] = body(r, world.dist(r))
                return
            torch.cuda.set_device(dev)
            with torch.cuda.stream(torch.cuda.Stream()):
                out[r] = body(r, world.dist(r))
                torch.cuda.current_stream().synchronize()
        except BaseException as e:  # noqa: BLE001 - reported to the caller
            err[r] = e
            world.abort()

    ts = [threading.Thread(target=thread, args=(r,), daemon=True) for r in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=10 * TIMEOUT)
    if any(t.is_alive() for t in ts):
        raise TimeoutError("fake_dist: a rank thread did not finish")
    first = next((e for e in err if e is not None and not isinstance(e, RuntimeError)), None) or next(
        (e for e in err if e is not None), None)
    if first is not None:
        raise first
    return out
