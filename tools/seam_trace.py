#!/usr/bin/env python3
"""The same 2^k-constraint proof three ways, 200 ms apart: resident witness (prove_witness, the
bench's value), bh_prove from host buffers (the drop-in), and the multiexp seam
(bellman_hip.prove_seam).  Run under rocprofv3 --kernel-trace: the three device windows are the
last three bursts of the trace (tools/split_bursts.py)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bellman-mpc_amd"))
import bellman_hip as bh  # noqa: E402

logc = int(sys.argv[1]) if len(sys.argv) > 1 else 22
rounds = (1 << (logc - 1)) - 1
ctx = bh.Context(0)
params = bh.Parameters.chain(ctx, rounds)
params.prepare(bh.Witness.chain(ctx, rounds))
asg = bh.chain_assignment(rounds)
r, s = 27134, 17146
w = bh.Witness.chain(ctx, rounds)
for _ in range(2):
    want = bh.prove(ctx, params, asg, r, s)
    assert bh.prove_seam(ctx, params, asg, r, s) == want
    assert bh.prove_witness(ctx, params, w, r, s) == want
time.sleep(0.2)
tr = time.perf_counter()
bh.prove_witness(ctx, params, w, r, s)
tr1 = time.perf_counter()
time.sleep(0.2)
t0 = time.perf_counter()
bh.prove(ctx, params, asg, r, s)
t1 = time.perf_counter()
time.sleep(0.2)
t2 = time.perf_counter()
assert bh.prove_seam(ctx, params, asg, r, s) == want
t3 = time.perf_counter()
print(f"resident {1e3 * (tr1 - tr):.2f} ms, bh_prove {1e3 * (t1 - t0):.2f} ms, seam {1e3 * (t3 - t2):.2f} ms",
      flush=True)
