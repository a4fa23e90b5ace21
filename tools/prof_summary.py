#!/usr/bin/env python3
"""Summarise the rocprofv3 databases written by tools/profile_round.sh into
committed text/JSON under profiles/:

  <tag>_rocprof_stats.txt   per-kernel calls / average / total duration
                            (the --kernel-trace --stats pass)
  <tag>_traffic.json        per-kernel HBM bytes per launch from the separate
                            FETCH_SIZE and WRITE_SIZE --pmc passes

HBM correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE
reports half the bytes of a wide coalesced read, so fetched bytes are
FETCH_SIZE(KiB) x 1024 x 2; WRITE_SIZE is taken as reported.

usage: prof_summary.py <prof_dir> <tag> [<profiled command>]
"""
import json
import os
import sqlite3
import sys
from collections import defaultdict


def short(name: str) -> str:
    return name.split("(")[0]


def kernel_stats(db):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    return rows


def pmc(db, counter):
    c = sqlite3.connect(db)
    acc = defaultdict(list)
    for name, val in c.execute("select kernel_name, value from counters_collection where counter_name=?", (counter,)):
        acc[short(name)].append(float(val))
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


def per_dispatch(db, counter, kernel):
    """Values of `counter` for every dispatch of `kernel`, in dispatch order
    (the PMC driver launches one per frame; k_recon's grid now varies with the
    frame's slow list, so the grid size no longer identifies them)."""
    c = sqlite3.connect(db)
    return [float(v) for n, v in c.execute(
        "select kernel_name, value from counters_collection where counter_name=? order by dispatch_id",
        (counter,)) if short(n) == kernel]


def main():
    d, tag = sys.argv[1], sys.argv[2]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = os.path.join(root, "profiles")
    os.makedirs(out, exist_ok=True)
    rows = kernel_stats(os.path.join(d, "trace", "run_results.db"))
    lines = ["# rocprofv3 --kernel-trace --stats  (%s)" % tag,
             "# command: rocprofv3 --kernel-trace --stats -- " + (sys.argv[3] if len(sys.argv) > 3 else
                                                                   "python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline"),
             "# (averages below mix the concurrent multi-stream timed region and the single-stream passes)",
             "%-24s %8s %14s %12s %8s" % ("kernel", "calls", "total_us", "avg_us", "pct")]
    for name, calls, tot, avg, pct in rows:
        lines.append("%-24s %8d %14.1f %12.3f %8.2f" % (short(name), calls, tot, avg, pct))
    # per-dispatch durations of the last step (one launch per frame, 8 frames)
    c = sqlite3.connect(os.path.join(d, "trace", "run_results.db"))
    seq = [(short(n), dur / 1e3) for n, dur in c.execute("select name, duration from kernels order by start")]
    # the bench's last phase is the single-context instrumented pass (5 steps x 8
    # frames, frame order 0..7): its k_recon P-frame dispatches are the ones the
    # bench's hipEvent roofline times
    rec = [v for n, v in seq if n == "k_recon"][-40:]
    prec = [v for i, v in enumerate(rec) if i % 8 != 0]
    if prec:
        lines.append("# k_recon, instrumented single-stream pass, P frames: %d dispatches, avg %.2f us"
                     % (len(prec), sum(prec) / len(prec)))
    lines.append("# last step, per frame (us): I P P P P P P P")
    for k in sorted({n for n, _ in seq if n.startswith("k_")}):
        ds = [v for n, v in seq if n == k][-8:]
        lines.append("%-24s %s" % (k, " ".join("%8.1f" % v for v in ds)))
    open(os.path.join(out, "%s_rocprof_stats.txt" % tag), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))
    if not os.path.exists(os.path.join(d, "fetch", "run_results.db")):
        print("no PMC passes under", d)
        return
    import subprocess

    commit = subprocess.run(["git", "-C", os.path.dirname(os.path.abspath(__file__)), "rev-parse", "--short=12", "HEAD"],
                            capture_output=True, text=True).stdout.strip() or None
    traffic = {"tag": tag, "commit": commit, "profile": "profiles/%s_traffic.json" % tag, "correction": "fetch_bytes = FETCH_SIZE_KiB*1024*2 (gfx950 half-count); "
                                         "write_bytes = WRITE_SIZE_KiB*1024", "kernels": {}}
    f, nf = pmc(os.path.join(d, "fetch", "run_results.db"), "FETCH_SIZE")
    w, nw = pmc(os.path.join(d, "write", "run_results.db"), "WRITE_SIZE")
    for k in sorted(set(f) | set(w)):
        fb = f.get(k, 0.0) * 1024 * 2
        wb = w.get(k, 0.0) * 1024
        traffic["kernels"][k] = {"fetch_kib_raw": round(f.get(k, 0.0), 1), "write_kib_raw": round(w.get(k, 0.0), 1),
                                 "hbm_bytes_per_launch": round(fb + wb), "launches": nf.get(k, 0)}
    # k_recon on P frames only: the batched launches (one group, frame order
    # 0..7: frame 0 is the I frame, no inter pixels), so drop every 8th
    fr = per_dispatch(os.path.join(d, "fetch", "run_results.db"), "FETCH_SIZE", "k_recon")
    wr = per_dispatch(os.path.join(d, "write", "run_results.db"), "WRITE_SIZE", "k_recon")
    if fr and wr and len(fr) == len(wr):
        pf = [v for i, v in enumerate(fr) if i % 8 != 0]
        pw = [v for i, v in enumerate(wr) if i % 8 != 0]
        # the PMC driver (profile_round.sh: tools/decode_frames.py) launches one frame per k_recon; the
        # bench's roofline launch carries 8 frames (THOR_MAX_BATCH), so its per-launch traffic is 8 x that
        per_frame = (sum(pf) * 2 + sum(pw)) * 1024 / len(pf)
        traffic["recon_hbm_bytes_per_p_frame"] = round(per_frame)
        traffic["recon_hbm_bytes_per_p_launch"] = round(8 * per_frame)
        traffic["recon_p_launches"] = len(pf)
        traffic["recon_note"] = ("tools/decode_frames.py k4_low 8: one k_recon launch per frame; per_p_launch = 8 "
                                 "frames, the bench's batched launch (THOR_MAX_BATCH)")
    json.dump(traffic, open(os.path.join(out, "%s_traffic.json" % tag), "w"), indent=1)
    # the GPU box does not receive profiles/ (.gpurunignore): bench.py reads tools/traffic_latest.json,
    # replaced only on request (PROF_LATEST=1), so a summary run cannot swap the bench's figure silently
    if os.environ.get("PROF_LATEST") == "1":
        json.dump(traffic, open(os.path.join(root, "tools", "traffic_latest.json"), "w"), indent=1)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
