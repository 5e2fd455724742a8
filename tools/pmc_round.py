#!/usr/bin/env python3
"""One round's PMC summary of the 2^22 bench from the tools/gpu_pmc.sh passes (fetch, write, sq,
tcc, grbm; one counter group per rocprofv3 run), plus the kernel trace of the same bench command:

  * per-kernel per-dispatch averages of every counter (tools/pmc_report.py: FETCH_SIZE x2 for
    gfx950's 16-B lanes, KiB -> bytes; MI355X_MICROARCH.md 'HBM');
  * held_clock_ghz = GRBM_GUI_ACTIVE / 8 XCDs / dispatch wall time (counter passes serialise
    kernels, so these are solo clocks; 'DVFS give-back');
  * VALU lane-instructions per mixed addition (SQ_INSTS_VALU x 64 / madds per dispatch), the madds
    taken from the bench line each pass printed (breakdown_ms.g1_adds / g2_adds per proof);
  * the kernel trace's average duration of k_accumulate_pf<G1> (co-running, as shipped), which the
    bench line's roofline.avg_launch_ms must match.

usage: pmc_round.py PMC_DIR TRACE_KERNEL_STATS_CSV OUT_PREFIX NOTE
  writes OUT_PREFIX_pmc_2p22.json and OUT_PREFIX_pmc_traffic_accumulate_g1.json"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_report import load  # noqa: E402

KERNELS = ["k_accumulate_pf<CurveOps<FpOps", "k_accumulate_pf<CurveOps<Fp2Ops", "k_ntt_pass<true>",
           "k_ntt_pass<false>", "k_reduce_blocks", "k_reduce_window", "k_part_", "k_cont_seq", "k_dist"]
G1 = KERNELS[0]


def bench_line(log):
    for line in open(log):
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    return None


def main():
    d, stats_csv, prefix, note = sys.argv[1:5]
    vals = load(d)
    out = {}
    for sub in KERNELS:
        agg = {}
        for k, cs in vals.items():
            if sub not in k:
                continue
            for c, per in cs.items():
                agg.setdefault(c, []).extend(per.values())
        if not agg:
            continue
        res = {c: sum(v) / len(v) for c, v in agg.items()}
        res["dispatches"] = {c: len(v) for c, v in agg.items()}
        if "FETCH_SIZE" in res:
            res["fetch_bytes"] = 2.0 * 1024.0 * res["FETCH_SIZE"]
        if "WRITE_SIZE" in res:
            res["write_bytes"] = 1024.0 * res["WRITE_SIZE"]
        if "fetch_bytes" in res and "write_bytes" in res:
            res["traffic_bytes"] = res["fetch_bytes"] + res["write_bytes"]
        if "TCC_HIT_sum" in res and "TCC_MISS_sum" in res:
            res["l2_hit_rate"] = res["TCC_HIT_sum"] / max(1.0, res["TCC_HIT_sum"] + res["TCC_MISS_sum"])
        out[sub] = res
    # held clocks and solo dispatch times from the GRBM pass (dispatches >= 0.3 ms)
    for path in glob.glob(os.path.join(d, "grbm", "*counter_collection.csv")):
        per = {}
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
                continue
            ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            for sub in out:
                if sub in r["Kernel_Name"] and ns >= 300000:
                    per.setdefault(sub, []).append((float(r["Counter_Value"]), ns))
        for sub, v in per.items():
            out[sub]["held_clock_ghz"] = round(sum(a / 8.0 / ns for a, ns in v) / len(v), 3)
            out[sub]["avg_dispatch_ms_grbm_pass"] = round(sum(ns for _, ns in v) / len(v) / 1e6, 3)
    line = bench_line(os.path.join(d, "sq.log"))
    proofs = line["steps"] + line["warmup"]
    bd = line["breakdown_ms"]
    out["proofs"] = proofs
    g1_launches = out[G1]["dispatches"]["SQ_INSTS_VALU"] / proofs
    out["g1_accumulations_per_proof"] = g1_launches
    if "g1_adds" in bd:
        g1_adds, g2_adds = bd["g1_adds"], bd["g2_adds"]
        src = "breakdown_ms.g1_adds / g2_adds of the pass's own bench line"
    else:  # earlier bench lines: madd rate x accumulation time
        g1_adds = line["valu_roofline"]["achieved"] * 1e9 * bd["g1_accumulate"] / 1e3
        g2_adds = None
        src = "valu_roofline.achieved x breakdown_ms.g1_accumulate of the pass's bench line"
    out["g1_madds_per_proof"] = round(g1_adds)
    out["valu_lane_instructions_per_g1_madd"] = round(out[G1]["SQ_INSTS_VALU"] * 64 * g1_launches / g1_adds, 1)
    g2k = KERNELS[1]
    if g2_adds and g2k in out:
        g2_launches = out[g2k]["dispatches"]["SQ_INSTS_VALU"] / proofs
        out["g2_madds_per_proof"] = round(g2_adds)
        out["valu_lane_instructions_per_g2_madd"] = round(out[g2k]["SQ_INSTS_VALU"] * 64 * g2_launches / g2_adds, 1)
    out["madds_source"] = src
    # the kernel trace of the same bench command (no counters: kernels co-run as shipped)
    for r in csv.DictReader(open(stats_csv)):
        if "k_accumulate_pf<CurveOps<FpOps" in r["Name"]:
            out["trace_g1_accumulate"] = {"calls": int(r["Calls"]), "avg_ms": round(float(r["AverageNs"]) / 1e6, 4),
                                          "source": stats_csv}
    # the kernel's own time per proof: the union of its dispatch intervals in the kernel trace
    # (run_kernel_trace.csv beside the stats), per proof of `launches` G1 launches; the first proof
    # (warmup) is skipped, the median taken -- what bench.py's roofline.avg_launch_ms measures
    trace_csv = stats_csv.replace("kernel_stats", "kernel_trace")
    if os.path.exists(trace_csv):
        iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(trace_csv))
                    if "k_accumulate_pf<CurveOps<FpOps" in r["Kernel_Name"])
        per = int(os.environ.get("G1_LAUNCHES_PER_PROOF", "4"))
        unions = []
        for i in range(per, len(iv) - per + 1, per):
            tot, cs, ce = 0, None, None
            for a, b in iv[i:i + per]:
                if cs is None:
                    cs, ce = a, b
                elif a <= ce:
                    ce = max(ce, b)
                else:
                    tot += ce - cs
                    cs, ce = a, b
            unions.append((tot + ce - cs) / 1e6)
        if unions:
            med = sorted(unions)[len(unions) // 2]
            out["trace_g1_accumulate_union"] = {"per_proof_ms": round(med, 4), "launches_per_proof": per,
                                                "per_launch_ms": round(med / per, 4), "proofs": len(unions),
                                                "per_proof_all": [round(u, 3) for u in unions], "source": trace_csv}
    out["notes"] = note
    json.dump(out, open(prefix + "_pmc_2p22.json", "w"), indent=1)
    g = out[G1]
    traffic = {"kernel": G1, "launches_fetch": g["dispatches"].get("FETCH_SIZE"),
               "launches_write": g["dispatches"].get("WRITE_SIZE"),
               "fetch_bytes_per_launch": g.get("fetch_bytes"), "write_bytes_per_launch": g.get("write_bytes"),
               "correction": "FETCH_SIZE x2 (gfx950, 16-B lanes), KiB -> bytes",
               "traffic_bytes_per_launch": g.get("traffic_bytes")}
    json.dump(traffic, open(prefix + "_pmc_traffic_accumulate_g1.json", "w"), indent=1)
    print(json.dumps({k: out[k] for k in out if not isinstance(out[k], dict)}, indent=1))


if __name__ == "__main__":
    main()
