#!/usr/bin/env python3
"""Per-dispatch PMC values of one kernel from rocprofv3 databases (tools/prof_recon.sh
passes sq1 / sq2 / fetch / write): averages over the widest-grid dispatches whose
first counter is above the kernel's median (the 8-frame P launches, not the I ones).
usage: pmc_kernel.py <prof_dir> [kernel]"""
import os
import sqlite3
import sys
from collections import defaultdict

d = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "k_recon"
res = {}
for p in ("sq1", "sq2", "fetch", "write", "ta"):
    db = os.path.join(d, p, "run_results.db")
    if not os.path.exists(db):
        continue
    c = sqlite3.connect(db)
    by = defaultdict(dict)
    for n, cn, v, disp in c.execute("select kernel_name, counter_name, value, dispatch_id from counters_collection"):
        if n.split("(")[0] == kern:
            by[disp][cn] = float(v)
    disps = sorted(by)
    if not disps:
        continue
    first = sorted(by[disps[0]])[0]
    vals = sorted(by[x][first] for x in disps)
    med = vals[len(vals) // 2]
    keep = [x for x in disps if by[x][first] >= 0.5 * med]
    for cn in by[disps[0]]:
        res[cn] = sum(by[x][cn] for x in keep) / len(keep)
w = res.get("SQ_WAVES", 1)
for k in sorted(res):
    print("%-24s %14.0f  per wave %10.1f" % (k, res[k], res[k] / w))
if "SQ_WAVE_CYCLES" in res:
    wc = res["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
        if k in res:
            print("%-24s %5.1f %% of wave cycles" % (k, 100 * res[k] / wc))
if "FETCH_SIZE" in res and "WRITE_SIZE" in res:
    print("HBM bytes per launch (FETCH x2 + WRITE): %.1f MB" % ((2 * res["FETCH_SIZE"] + res["WRITE_SIZE"]) * 1024 / 1e6))
