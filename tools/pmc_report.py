#!/usr/bin/env python3
"""Per-kernel summary of the tools/gpu_pmc.sh passes: for each kernel substring, the per-dispatch
average of every counter (FETCH_SIZE doubled for gfx950's 16-B-lane reads, KiB -> bytes;
MI355X_MICROARCH.md 'HBM'), plus derived VALU utilisation and L2 hit rate.
usage: pmc_report.py PMC_DIR KERNEL_SUBSTRING [...] > out.json"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    vals = defaultdict(lambda: defaultdict(dict))  # kernel -> counter -> dispatch -> value
    for path in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(path)):
            vals[r["Kernel_Name"]][r["Counter_Name"]][(path, int(r["Dispatch_Id"]))] = float(r["Counter_Value"])
    return vals


def main():
    d, subs = sys.argv[1], sys.argv[2:]
    vals = load(d)
    out = {}
    for sub in subs:
        agg = defaultdict(list)
        for k, cs in vals.items():
            if sub not in k:
                continue
            for c, per in cs.items():
                agg[c].extend(per.values())
        res = {c: sum(v) / len(v) for c, v in agg.items() if v}
        res["dispatches"] = {c: len(v) for c, v in agg.items()}
        if "FETCH_SIZE" in res:
            res["fetch_bytes"] = 2.0 * 1024.0 * res["FETCH_SIZE"]
        if "WRITE_SIZE" in res:
            res["write_bytes"] = 1024.0 * res["WRITE_SIZE"]
        if "fetch_bytes" in res and "write_bytes" in res:
            res["traffic_bytes"] = res["fetch_bytes"] + res["write_bytes"]
        if res.get("SQ_BUSY_CYCLES") and "SQ_ACTIVE_INST_VALU" in res:
            res["valu_active_per_busy_cycle"] = res["SQ_ACTIVE_INST_VALU"] / res["SQ_BUSY_CYCLES"]
        if "TCC_HIT_sum" in res and "TCC_MISS_sum" in res:
            res["l2_hit_rate"] = res["TCC_HIT_sum"] / max(1.0, res["TCC_HIT_sum"] + res["TCC_MISS_sum"])
        out[sub] = res
    out["notes"] = ("per-dispatch averages over every dispatch of the kernel in the run (2^22 bench: 1 warm-up + "
                    "2 timed proofs, plus setup); FETCH_SIZE x2 (gfx950 16-B lanes), KiB -> bytes")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
