#!/usr/bin/env python3
"""Per-rank cost of the sharded prover on ONE GPU (strong-scaling rehearsal).

For N in --shards, prepares the SRS window tables for N shards and times shard k's
bh_prove_witness_partial (each rank's whole device work: replicated H pipeline + its
1/N of every multiexp).  The exchange (960 B per rank over RCCL) and the host combine
are not included.  Predicted speed-up = t(1) / max_k t_k(N).
usage: shard_rehearsal.py [--log-constraints 22] [--shards 1,2,4,8] [--reps 3]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bellman-mpc_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-constraints", type=int, default=22)
    ap.add_argument("--shards", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--all-ranks", type=int, default=0, help="time every shard, not only shard 0 and N-1")
    ap.add_argument("--local", type=int, default=0,
                    help="also time bh_prove_witness_partials_local (all N ranks, distributed H emulated)")
    args = ap.parse_args()
    import bellman_hip as bh
    rounds = (1 << (args.log_constraints - 1)) - 1
    ctx = bh.Context(0)
    params = bh.Parameters.chain(ctx, rounds)
    w = bh.Witness.chain(ctx, rounds)
    out = {"log_constraints": args.log_constraints, "per_rank_ms": {}}
    for n in [int(x) for x in args.shards.split(",")]:
        params.prepare(w, n)
        ks = range(n) if args.all_ranks else sorted({0, n - 1})
        worst = 0.0
        per = {}
        for k in ks:
            bh.prove_witness_partial(ctx, params, w, k, n)  # warm-up
            ts = []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                bh.prove_witness_partial(ctx, params, w, k, n)
                ts.append((time.perf_counter() - t0) * 1e3)
            per[k] = round(min(ts), 3)
            worst = max(worst, min(ts))
        out["per_rank_ms"][n] = {"shards": per, "max": round(worst, 3)}
        if args.local and n > 1:
            bh.prove_witness_partials_local(ctx, params, w, n)  # warm-up
            t0 = time.perf_counter()
            bh.prove_witness_partials_local(ctx, params, w, n)
            out.setdefault("local_all_ranks_ms", {})[n] = round((time.perf_counter() - t0) * 1e3, 3)
        print(json.dumps({"N": n, "per_rank_ms": per}), flush=True)
    base = out["per_rank_ms"].get(1, {}).get("max")
    if base:
        out["predicted_speedup"] = {n: round(base / v["max"], 2) for n, v in out["per_rank_ms"].items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
