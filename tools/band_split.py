#!/usr/bin/env python3
"""One rank's share of an N-way row split, its kernels alone on this GPU
(bench.band_kernel_ms: boundary-mode decoder context, no exchange), for the
isolated per-rank rocprof evidence of the row split.

  band_split.py [stream] [world] [rank|all] [reps]

Prints the per-frame stage times (hipEvents) and the kernel sum; run under
`rocprofv3 --kernel-trace --stats` for the per-kernel launch durations."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from thor_amd import lib as L  # noqa: E402
from thor_amd.bitstream import parse_stream  # noqa: E402

args = sys.argv[1:]
name = args[0] if args else "k4_med"
world = int(args[1]) if len(args) > 1 else 8
which = args[2] if len(args) > 2 else "all"
reps = int(args[3]) if len(args) > 3 else 3
seq, frames = parse_stream(open(os.path.join(ROOT, "tests", "golden", name + ".bit"), "rb").read())
lib = L.load()
ranks = range(world) if which == "all" else [int(which)]
for r in ranks:
    ms, wall = bench.band_kernel_ms(lib, seq, frames, world, r, reps)
    print(json.dumps({"stream": name, "world": world, "rank": r,
                      "stage_ms_per_frame": dict(zip(bench.STAGES + ["interp"], [round(x, 4) for x in ms])),
                      "kernel_ms_per_frame": round(sum(ms), 4), "wall_ms_per_frame": round(wall, 4)}), flush=True)
