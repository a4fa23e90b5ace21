#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc databases of one kernel into JSON (run on the GPU
box, so that only the summary comes back): usage sq_summary.py KERNEL OUT.json DIR [DIR ...]"""
import json
import sqlite3
import sys
from collections import defaultdict

kern, out, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
res = {}
for d in dirs:
    c = sqlite3.connect(d + "/run_results.db")
    by = defaultdict(dict)
    for n, cn, v, disp in c.execute("select kernel_name, counter_name, value, dispatch_id from counters_collection"):
        if n.split("(")[0] == kern:
            by[disp][cn] = float(v)
    for disp, cs in by.items():
        for cn, v in cs.items():
            res.setdefault(cn, []).append(v)
per = {}  # counter -> values in dispatch order (e.g. an I-frame batch, then a P-frame batch)
for d in dirs:
    c = sqlite3.connect(d + "/run_results.db")
    rows = sorted(c.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection"))
    acc = defaultdict(lambda: defaultdict(float))
    for disp, n, cn, v in rows:
        if n.split("(")[0] == kern:
            acc[cn][disp] += float(v)
    for cn, byd in acc.items():
        per[cn] = [byd[k] for k in sorted(byd)]
json.dump({"kernel": kern, "counters": {k: sum(v) for k, v in res.items()}, "dispatches": {k: len(v) for k, v in res.items()},
           "per_dispatch": per}, open(out, "w"), indent=1)
print(json.dumps({k: "%.4g" % sum(v) for k, v in sorted(res.items())}))
