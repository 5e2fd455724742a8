#!/usr/bin/env python3
"""Kernel timeline of the last proof of a rocprofv3 run (kernel_trace.csv or rocpd .db):
one line per dispatch with start/end relative to the window, duration and stream.
usage: proof_timeline.py TRACE [window_ms] [--min-us N]"""
import csv
import re
import sqlite3
import sys


def load(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        return [(n, s, e, st) for n, s, e, st in c.execute("select name,start,end,stream_id from kernels")]
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                     r.get("Stream_Id", r.get("Queue_Id", "?"))))
    return rows


def short(n):
    n = re.sub(r"\(.*", "", n).replace("void ", "").replace("bh::", "")
    return n.replace("CurveOps<FpOps> ", "G1").replace("CurveOps<Fp2Ops> ", "G2")[:40]


def main():
    path = sys.argv[1]
    win = float(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else 70.0
    min_us = float(sys.argv[sys.argv.index("--min-us") + 1]) if "--min-us" in sys.argv else 0.0
    rows = sorted(load(path), key=lambda r: r[1])
    tend = max(r[2] for r in rows)
    sel = [r for r in rows if r[1] > tend - win * 1e6]
    t0 = sel[0][1]
    for n, s, e, st in sel:
        if (e - s) / 1e3 >= min_us:
            print(f"{(s - t0) / 1e6:8.3f} {(e - t0) / 1e6:8.3f} {(e - s) / 1e6:7.3f} s{st} {short(n)}")


if __name__ == "__main__":
    main()
