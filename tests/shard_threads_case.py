"""Child process of tests/test_gpu_shard.py::test_row_shard_device_exchange_threads:
RowShard's device-exchange path at world 2-4 on one GPU, one thread per rank
over tests/fake_dist.py.  Arguments: name,nframes,world,mode ...; prints one
JSON line: per case, [per-rank bad decode orders, per-rank bytes received]."""
import hashlib
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))


def run_case(name, nframes, world, mode):
    from fake_dist import run_ranks
    from test_gpu_shard import _load

    from thor_amd.decoder import GpuDecoder
    from thor_amd.shard import RowShard

    meta, seq, frames = _load(name, nframes)
    local, halo, boundary = mode != "gather", mode in ("halo", "boundary"), mode == "boundary"

    def body(rank, dist):
        dec = GpuDecoder(seq)
        try:
            sh = RowShard(dec, dist, seq.width, seq.height, device_exchange=True, band_local=local, halo=halo,
                          boundary=boundary)
            assert sh.dstream is not None
            bad = []
            for fr in frames:
                sh.decode(dec.upload(fr), fr.frame_num, fr)
                got = hashlib.md5(sh.assemble(fr.frame_num) if halo else dec.read_i420(fr.frame_num)).hexdigest()
                if got != meta["stage_md5"][fr.decode_order]["final"]:
                    bad.append(fr.decode_order)
            return bad, dist.bytes_moved
        finally:
            dec.close()

    res = run_ranks(world, body)
    return [r[0] for r in res], [r[1] for r in res]


def main():
    if not torch.cuda.is_available():
        raise SystemExit("no GPU")
    torch.cuda.init()  # torch's HIP runtime first, then the decoder library's
    from thor_amd.lib import load

    load()
    out = []
    for a in sys.argv[1:]:
        name, nframes, world, mode = a.split(",")
        out.append(run_case(name, int(nframes), int(world), mode))
        print("case %s done" % a, file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
