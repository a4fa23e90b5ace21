#!/usr/bin/env python3
"""Kernel concurrency histogram of a rocprofv3 kernel trace (diagnostic):
time spent with 0, 1, 2, ... kernels in flight, over the window between the
first and last dispatch of the densest stretch (or the whole run)."""
import collections
import sqlite3
import sys

db = sys.argv[1]
c = sqlite3.connect(db)
rows = [(n.split("(")[0], s, e, q) for n, s, e, q in c.execute("select name, start, end, queue_id from kernels order by start")]
ev = sorted([(s, 1) for _, s, _, _ in rows] + [(e, -1) for _, _, e, _ in rows])
cur, last, hist = 0, ev[0][0], collections.Counter()
for t, d in ev:
    hist[cur] += t - last
    last, cur = t, cur + d
busy = sum(v for k, v in hist.items() if k > 0)
print("time by kernels in flight (ms):", {k: round(v / 1e6, 2) for k, v in sorted(hist.items())})
print("busy ms %.2f, mean concurrency while busy %.2f" % (busy / 1e6, sum(k * v for k, v in hist.items()) / busy))
print("dispatches per queue:", dict(collections.Counter(q for *_, q in rows)))
