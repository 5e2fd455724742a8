#!/usr/bin/env python3
"""Phase timings of bellman_hip.prove_seam at 2^22 (host side) next to bh_prove from the same
host buffers; run under rocprofv3 --kernel-trace for the device timeline."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bellman-mpc_amd"))
import bellman_hip as bh  # noqa: E402


def main():
    logc = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    rounds = (1 << (logc - 1)) - 1
    ctx = bh.Context(0)
    params = bh.Parameters.chain(ctx, rounds)
    params.prepare(bh.Witness.chain(ctx, rounds))
    asg = bh.chain_assignment(rounds)
    r, s = 27134, 17146
    want = bh.prove(ctx, params, asg, r, s)
    t0 = time.perf_counter()
    for _ in range(reps):
        bh.prove(ctx, params, asg, r, s)
    print(f"bh_prove from host buffers: {round((time.perf_counter() - t0) * 1e3 / reps, 2)} ms", flush=True)
    for rep in range(reps):
        t = [time.perf_counter()]
        ni, na = asg["inputs"].shape[0], asg["aux"].shape[0]
        h = bh.compute_h_scalars(ctx, asg["a"], asg["b"], asg["c"])
        t.append(time.perf_counter())
        inp = bh.Scalars(ctx, asg["inputs"], montgomery=True)
        aux = bh.Scalars(ctx, asg["aux"], montgomery=True)
        t.append(time.perf_counter())
        a_aux = bh.DensityWords(asg["a_aux_density"], na)
        b_in = bh.DensityWords(asg["b_input_density"], ni)
        b_aux = bh.DensityWords(asg["b_aux_density"], na)
        bt = b_in.total()
        H, L, A, B1, B2 = (params.vector(k) for k in range(5))
        ws = [bh.multiexp_async(ctx, H, 0, None, h), bh.multiexp_async(ctx, L, 0, None, aux),
              bh.multiexp_async(ctx, A, 0, None, inp), bh.multiexp_async(ctx, A, ni, a_aux, aux),
              bh.multiexp_async(ctx, B1, 0, b_in, inp), bh.multiexp_async(ctx, B1, bt, b_aux, aux),
              bh.multiexp_async(ctx, B2, 0, b_in, inp), bh.multiexp_async(ctx, B2, bt, b_aux, aux)]
        t.append(time.perf_counter())
        outs = []
        for w in ws:
            outs.append(w.wait())
            t.append(time.perf_counter())
        proof = bh.proof_from_partials(params.vk_bytes(), b"".join(outs), 1, r, s)
        t.append(time.perf_counter())
        ms = [round((b - a) * 1e3, 2) for a, b in zip(t, t[1:])]
        print(f"rep {rep}: total {round((t[-1] - t[0]) * 1e3, 2)} ms; h_call {ms[0]} uploads {ms[1]} "
              f"submits {ms[2]} waits {ms[3:11]} assemble {ms[11]} ok {proof == want}", flush=True)
    # prove_seam back to back (as bench.py times it) and 200 ms apart
    for gap in (0.0, 0.2, 0.0):
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            bh.prove_seam(ctx, params, asg, r, s)
            ts.append(round((time.perf_counter() - t0) * 1e3, 2))
            if gap:
                time.sleep(gap)
        print(f"prove_seam gap {gap}s: {ts}", flush=True)


if __name__ == "__main__":
    main()
