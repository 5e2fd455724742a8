#!/usr/bin/env python3
"""HBM traffic of the dominant kernel from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE
collected separately: MI355X_MICROARCH.md 'rocprofv3 PMC slots').  FETCH_SIZE/WRITE_SIZE are
in KiB; on gfx950 FETCH_SIZE reports half the bytes of 16-B-per-lane reads (our LDS-DMA base
gathers are exactly that), so it is doubled (MI355X_MICROARCH.md 'HBM').

usage: pmc_traffic.py FETCH.csv WRITE.csv KERNEL_SUBSTRING OUT.json
Averages over every dispatch of the kernel (all proofs of the run) -> bytes per launch."""
import csv
import json
import sys


def per_dispatch(path, counter, sub):
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and sub in r["Kernel_Name"]:
            vals[int(r["Dispatch_Id"])] = (float(r["Counter_Value"]) * 1024.0,
                                           int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                           int(r["Grid_Size"]))
    return vals


def main():
    fpath, wpath, sub, out = sys.argv[1:5]
    f = per_dispatch(fpath, "FETCH_SIZE", sub)
    w = per_dispatch(wpath, "WRITE_SIZE", sub)
    fetch = [2.0 * v[0] for v in f.values()]
    write = [v[0] for v in w.values()]
    res = {
        "kernel": sub,
        "launches_fetch": len(fetch), "launches_write": len(write),
        "fetch_bytes_per_launch": sum(fetch) / len(fetch),
        "write_bytes_per_launch": sum(write) / len(write),
        "correction": "FETCH_SIZE x2 (gfx950, 16-B lanes), KiB -> bytes",
    }
    res["traffic_bytes_per_launch"] = res["fetch_bytes_per_launch"] + res["write_bytes_per_launch"]
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
