#!/usr/bin/env python3
"""Summarise one proof of a rocprofv3 kernel trace: per-queue busy time, critical-path gaps
between accumulate launches.  usage: trace_timeline.py run_kernel_trace.csv [--full]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    r["s"] = int(r["Start_Timestamp"])
    r["e"] = int(r["End_Timestamp"])
    r["n"] = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("bh::", "")[:44]
rows.sort(key=lambda r: r["s"])
# last proof = from the last first-NTT pass that follows a gap
starts = [i for i, r in enumerate(rows) if "density_popc" in r["n"]]
first = starts[-3]
j = first
while j > 0 and rows[first]["s"] - rows[j - 1]["s"] < 3e6 and "cont_tree" not in rows[j - 1]["n"] and "sum_groups" not in rows[j-1]["n"]:
    j -= 1
sel = rows[j:]
t0 = min(r["s"] for r in sel)
t1 = max(r["e"] for r in sel)
print(f"proof span {(t1 - t0) / 1e6:.3f} ms, {len(sel)} dispatches")
agg = {}
for r in sel:
    agg.setdefault(r["n"], [0, 0.0])
    agg[r["n"]][0] += 1
    agg[r["n"]][1] += (r["e"] - r["s"]) / 1e6
for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:20]:
    print(f"  {t:8.3f} ms {c:4d}x {k}")
acc = [r for r in sel if "accumulate" in r["n"]]
print("accumulate launches (start, dur, gap before):")
prev = t0
for r in acc:
    print(f"  {(r['s'] - t0) / 1e6:8.3f} {(r['e'] - r['s']) / 1e6:8.3f} gap {(r['s'] - prev) / 1e6:7.3f} {r['n']} grid={r['Grid_Size_X']}")
    prev = r["e"]
print(f"  after last accumulate: {(t1 - prev) / 1e6:.3f} ms")
if "--full" in sys.argv:
    for r in sel:
        print(f"{(r['s'] - t0) / 1e6:8.3f} {(r['e'] - r['s']) / 1e6:7.3f} q{r['Queue_Id']} {r['n']} grid={r['Grid_Size_X']}")
