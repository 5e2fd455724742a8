#!/usr/bin/env python3
"""prove_seam per-call times at 2^22 in the bench's order (resident Witness proofs, then bh_prove
from host buffers, then the seam), with the resident Witness kept alive or released before the
seam calls (argv[1]: keep | drop).  Why does the bench's seam leg read ~69.5 ms where
tools/seam_gc.py reads ~63 ms?"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bellman-mpc_amd"))
import bellman_hip as bh  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "keep"
rounds = (1 << 21) - 1
r, s = 27134, 17146
ctx = bh.Context(0)
params = bh.Parameters.chain(ctx, rounds)
witness = bh.Witness.chain(ctx, rounds)
params.prepare(witness)
for _ in range(7):
    bh.prove_witness(ctx, params, witness, r, s)
ctx.synchronize()
asg = bh.chain_assignment(rounds)
for _ in range(6):
    bh.prove(ctx, params, asg, r, s)
ctx.synchronize()
if mode == "drop":
    del witness
ts = []
for _ in range(10):
    t0 = time.perf_counter()
    bh.prove_seam(ctx, params, asg, r, s)
    ts.append(round((time.perf_counter() - t0) * 1e3, 2))
    if os.environ.get("BH_HOST_TIMING"):
        print(f"call {len(ts)}: {ts[-1]} ms", file=sys.stderr, flush=True)
print(mode, ts, "mean of the last 8", round(sum(ts[2:]) / 8, 2), flush=True)
