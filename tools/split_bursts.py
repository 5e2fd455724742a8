#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace into bursts separated by idle gaps (> gap_ms) and print the
timeline of the last N bursts (start/end relative to each burst, ms, queue, kernel).
usage: split_bursts.py run_kernel_trace.csv [N=2] [gap_ms=50] [--min-us X]"""
import csv
import re
import sys

path = sys.argv[1]
N = int(sys.argv[2]) if len(sys.argv) > 2 else 2
gap = float(sys.argv[3]) if len(sys.argv) > 3 else 50.0
min_us = float(sys.argv[sys.argv.index("--min-us") + 1]) if "--min-us" in sys.argv else 0.0
rows = []
for r in csv.DictReader(open(path)):
    n = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("bh::", "")
    n = n.replace("CurveOps<FpOpsT<FpCfg> >", "G1").replace("CurveOps<Fp2Ops>", "G2")[:44]
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "?"), n))
rows.sort()
bursts, cur, last_end = [], [], None
for row in rows:
    if last_end is not None and row[0] - last_end > gap * 1e6:
        bursts.append(cur)
        cur = []
    cur.append(row)
    last_end = row[1] if last_end is None else max(last_end, row[1])
bursts.append(cur)
for b in bursts[-N:]:
    t0, t1 = b[0][0], max(r[1] for r in b)
    print(f"=== burst: {(t1 - t0) / 1e6:.3f} ms, {len(b)} dispatches")
    for s, e, q, n in b:
        if (e - s) / 1e3 >= min_us:
            print(f"{(s - t0) / 1e6:8.3f} {(e - t0) / 1e6:8.3f} {(e - s) / 1e6:7.3f} q{q} {n}")
