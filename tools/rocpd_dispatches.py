#!/usr/bin/env python3
"""Per-dispatch kernel durations (us) from a rocprofv3 run_results.db, in
dispatch order, for kernels whose name contains any of the given substrings.
  rocpd_dispatches.py <db> substr [substr ...]"""
import collections
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
q = ("select k.kernel_name, d.start, d.end from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol k "
     "on d.kernel_id = k.id order by d.start")
by = collections.defaultdict(list)
for n, a, b in c.execute(q):
    s = n.split("(")[0]
    if any(x in s for x in sys.argv[2:]):
        by[s].append((b - a) / 1e3)
for s, v in by.items():
    print("%-16s n %3d  %s" % (s, len(v), " ".join("%.1f" % x for x in v[:24])))
