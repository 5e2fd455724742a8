#!/usr/bin/env python3
"""Per-rank cost of the N-GPU prover on ONE GPU (strong-scaling rehearsal).

For each N and rank k (default: 0 and N-1): the rank's Parameters are prepared exactly as a
rank process of an N-GPU run holds them (bh_params_prepare_shard: its window-table slices
and, for N >= 2, its gathered share of the h vector), then bh_rehearse_rank runs that rank's
whole device work -- its 1/N of every multiexp and, for N >= 2, its part of the distributed
H block, each all-to-all moving only the rank's own chunks (the xGMI transfer itself, ~2 MB
per link per all-to-all at 2^22 and N = 8, is not included; neither are the 960-byte
all-gather and rank 0's host combine, ~0.5 ms).  Predicted speed-up = t(1) / max_k t_k(N).
usage: shard_rehearsal.py [--log-constraints 22] [--shards 1,2,4,8] [--reps 5] [--all-ranks 1]
       [--rank-only N:k]  (one rank, for a kernel trace)"""
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
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--all-ranks", type=int, default=0, help="time every rank, not only 0 and N-1")
    ap.add_argument("--rank-only", default=None, help="N:k -- only rank k of N (profiling)")
    args = ap.parse_args()
    import bellman_hip as bh
    rounds = (1 << (args.log_constraints - 1)) - 1
    ctx = bh.Context(0)
    params = bh.Parameters.chain(ctx, rounds)
    w = bh.Witness.chain(ctx, rounds)
    out = {"log_constraints": args.log_constraints, "per_rank_ms": {}, "setup_s": {}, "tables": {}}
    plan = ([(int(args.rank_only.split(":")[0]), [int(args.rank_only.split(":")[1])])] if args.rank_only else
            [(n, list(range(n)) if args.all_ranks else sorted({0, n - 1}))
             for n in (int(x) for x in args.shards.split(","))])
    for n, ks in plan:
        worst = 0.0
        per, setup, tabs = {}, {}, {}
        for k in ks:
            t0 = time.perf_counter()
            params.prepare_shard(w, k, n)  # this rank's slices only (and its h share for N >= 2)
            setup[k] = round(time.perf_counter() - t0, 3)
            bh.rehearse_rank(ctx, params, w, k, n)  # warm-up
            ts = [bh.rehearse_rank(ctx, params, w, k, n) for _ in range(args.reps)]
            st = ctx.last_stats()
            tabs[k] = {"used": int(st[10]), "large": int(st[11]), "table_GB": round(st[12] / 1e9, 2)}
            per[k] = round(min(ts), 3)
            worst = max(worst, min(ts))
        out["per_rank_ms"][n] = {"ranks": per, "max": round(worst, 3)}
        out["setup_s"][n] = setup
        out["tables"][n] = tabs
        print(json.dumps({"N": n, "per_rank_ms": per, "setup_s": setup, "tables": tabs}), flush=True)
    base = out["per_rank_ms"].get(1, {}).get("max")
    if base:
        out["predicted_speedup"] = {n: round(base / v["max"], 2) for n, v in out["per_rank_ms"].items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
