#!/usr/bin/env python3
"""CPU baseline at the headline size: the oracle's C++ restatement of bellman's
multicore prover core (oracle/cpu) timed once on the 2^22-constraint MiMC chain (C3) with every
hardware thread of this host, next to the bench's bounded 2^16 sample.  The proof must equal the
device proof.  Reports hardware threads, online CPUs, physical cores and sockets (from
/proc/cpuinfo), so that threads are not mistaken for cores.  A reported baseline, not a target.
With --fixture PATH the port's proof (and the device proof, and the SHA-256 of the Parameters
bytes both proved with) is written into that JSON file under the key "2^k": the full-size
parity fixture tests/golden/port_proofs.json that -m gpu compares the benchmark proof with.
usage: cpu_baseline_full.py [--log-constraints 22] [--reps 1] [--threads 0] [--fixture PATH]"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bellman-mpc_amd"))
sys.path.insert(0, ROOT)


def cpu_topology():
    model, sockets, cores = None, set(), set()
    phys = core = None
    with open("/proc/cpuinfo") as f:
        for line in f:
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "model name":
                model = v
            elif k == "physical id":
                phys = v
                sockets.add(v)
            elif k == "core id":
                core = v
            elif not k and phys is not None and core is not None:
                cores.add((phys, core))
                phys = core = None
    if phys is not None and core is not None:
        cores.add((phys, core))
    return {"cpu_model": model, "sockets": len(sockets) or None, "physical_cores": len(cores) or None,
            "online_cpus": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-constraints", type=int, default=22)
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--threads", type=int, default=0,
                    help="0: the box's CPU share (OMP_NUM_THREADS, 16 per GPU on the GPU pool) when set, else "
                         "every hardware thread")
    ap.add_argument("--fixture", default=None, help="JSON file to record the port's proof in")
    args = ap.parse_args()
    import bellman_hip as bh
    from oracle import cpu_port
    rounds = (1 << (args.log_constraints - 1)) - 1
    n_c = 2 * rounds + 2
    ctx = bh.Context(0)
    params = bh.Parameters.chain(ctx, rounds)
    gpu_proof = bh.prove_witness(ctx, params, bh.Witness.chain(ctx, rounds), 27134, 17146)
    pbytes = params.write()
    psha = hashlib.sha256(pbytes).hexdigest()
    del params
    share = os.environ.get("OMP_NUM_THREADS", "")
    threads = args.threads or (int(share) if share.isdigit() and int(share) > 0 else cpu_port.hardware_threads())
    t0 = time.time()
    proof, ms, ms_syn = cpu_port.chain_prove(pbytes, rounds, threads=threads, reps=args.reps)
    wall = time.time() - t0
    out = {"log_constraints": args.log_constraints, "constraints": n_c, "threads": threads,
           "value": round(n_c / (ms / 1e3), 1), "unit": "constraints/s", "kind": "port",
           "ms_per_proof": round(ms, 1), "synthesis_ms": round(ms_syn, 1), "reps": args.reps,
           "wall_s": round(wall, 1), "proof_matches_gpu": proof == gpu_proof}
    out.update(cpu_topology())
    out["params_sha256"] = psha
    print(json.dumps(out), flush=True)
    if args.fixture:
        fx = {}
        if os.path.exists(args.fixture):
            with open(args.fixture) as f:
                fx = json.load(f)
        fx[f"2^{args.log_constraints}"] = {
            "rounds": rounds, "constraints": n_c, "seed": 7, "preimage_seed": 8, "r": 27134, "s": 17146,
            "params_sha256": psha, "proof_port": proof.hex(), "proof_gpu": gpu_proof.hex(),
            "port_ms": round(ms, 1), "threads": threads,
            "generator": "tools/cpu_baseline_full.py --fixture (oracle/cpu port of bellman's multicore prover)"}
        with open(args.fixture, "w") as f:
            json.dump(fx, f, indent=1, sort_keys=True)
            f.write("\n")


if __name__ == "__main__":
    main()
