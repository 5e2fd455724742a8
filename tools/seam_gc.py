#!/usr/bin/env python3
"""prove_seam back to back at 2^22 with Python's cyclic GC on and off (is a collection inside a timed
call what stalls the h producer?); h producer stamps with BH_HOST_TIMING=1."""
import gc
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bellman-mpc_amd"))
import bellman_hip as bh  # noqa: E402

rounds = (1 << 21) - 1
ctx = bh.Context(0)
params = bh.Parameters.chain(ctx, rounds)
params.prepare(bh.Witness.chain(ctx, rounds))
asg = bh.chain_assignment(rounds)
for _ in range(2):
    bh.prove_seam(ctx, params, asg, 27134, 17146)
for mode in ("gc on", "gc off", "gc on", "gc off"):
    if mode == "gc off":
        gc.collect()
        gc.disable()
    else:
        gc.enable()
    ts = []
    for _ in range(8):
        t0 = time.perf_counter()
        bh.prove_seam(ctx, params, asg, 27134, 17146)
        ts.append(round((time.perf_counter() - t0) * 1e3, 2))
    print(mode, ts, "mean", round(sum(ts) / len(ts), 2), flush=True)
gc.enable()
