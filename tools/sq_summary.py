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
json.dump({"kernel": kern, "counters": {k: sum(v) for k, v in res.items()}, "dispatches": {k: len(v) for k, v in res.items()}},
          open(out, "w"), indent=1)
print(json.dumps({k: "%.4g" % sum(v) for k, v in sorted(res.items())}))
