#!/usr/bin/env python3
"""Benchmark: Groth16 constraints/sec on BLS12-381 (BASELINE.json `metric`).

Workload (BASELINE.json configs[2], "C3"): the synthetic MiMC-chain R1CS with
R = 2^(k-1) - 1 rounds -> exactly 2^k constraints (k = 22 by default), its CRS
generated on the device with the fork's fixed toxic waste (generator.rs:32-38),
and the fork's fixed r, s (prover.rs:169-170).  One "step" = one create_proof
after synthesis (prover.rs:206-349: H pipeline + 8 multiexps + assembly) with
the complete assignment already resident in HBM; the output is the 192-byte
proof.  Synthesis and CRS generation are outside the timed region.

Multi-GPU (`--gpus N`, launched by torch.distributed.run): every MSM is
sharded by scalar/point range over the N ranks; for N >= 2 (power of two) the H
block is distributed too (three RCCL all-to-alls per proof, dist_h.h) and each
rank's h multiexp covers the coefficients it ends with.  Each rank returns its 8
partial sums, RCCL all-gathers them and rank 0 adds them and assembles the
proof.  Total work is fixed, so scaling is "strong".

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "bellman-mpc_amd"))

HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: 8.0 TB/s spec
G1_PAIR_BYTES = 128       # 96 B affine base + 32 B scalar per (point, scalar)
G2_PAIR_BYTES = 224
TRAFFIC_FILE = "r06_final_pmc_traffic_accumulate_g1.json"  # tools/pmc_round.py output for the 2^22 workload
G1_MADD_PEAK = 7.04            # G mixed-add/s, tools/microbench/curvebench.hip on MI355X (profiles/r01_curvebench.txt)
G1_MADD_PEAK_CLOCK_GHZ = 2.27  # the clock curvebench's G1 (2 waves) kernel held (profiles/r03_curvebench_clock.txt)
MADS_PER_G1_MADD = 6 * 391 + 587 + 2 * 300  # 6 Fp-mul, Y3 as one two-product fe_mul2, 2 Fp-sqr
MAD_U64_PEAK_TPS = 27.22       # T v_mad_u64_u32/s, tools/microbench/madbench.hip on MI355X
PMC_FILE = "r06_final_pmc_2p22.json"  # tools/gpu_pmc.sh -> tools/pmc_round.py over the 2^22 bench (+ held clocks, trace)
SOLO_WAVE_INSTR_RATE = 510.0   # G wave-instr/s: the G1 accumulation alone (6.38 G madd/s x 5116 lane-instr / 64;
                               # profiles/r03_ab_accumulate_variants.txt serial run, r03_pmc_2p22.json)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--log-constraints", type=int, default=22)
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU port on a bounded sample (rank 0)")
    ap.add_argument("--cpu-log-constraints", type=int, default=16)
    ap.add_argument("--cpu-1t-log-constraints", type=int, default=12, help="1-thread CPU sample (0: skip)")
    ap.add_argument("--cpu-full", type=int, default=1,
                    help="also time the CPU port once on the bench's own workload (2^22: ~25 s on the GPU box's "
                         "16-thread share; 0: report the committed run profiles/r03_cpu_baseline_2p22.json)")
    ap.add_argument("--check", type=int, default=1, help="verify the proof bytes are identical every step")
    ap.add_argument("--tables", type=int, default=1, help="prover SRS window tables (bh_ctx_set_tables)")
    ap.add_argument("--c5", type=int, default=64,
                    help="throughput mode (BASELINE configs[4]): this many 2^20-constraint proofs split over the GPUs "
                         "(0: skip)")
    ap.add_argument("--c5-log-constraints", type=int, default=20)
    ap.add_argument("--c5-lanes", type=int, default=0, help="bh_prove_batch lanes per GPU (0: library default)")
    ap.add_argument("--seam", type=int, default=1,
                    help="with --dropin: also time the multiexp-level seam (bellman_hip.prove_seam)")
    ap.add_argument("--domain", type=int, default=1,
                    help="with --dropin: also time the EvaluationDomain seam (ifft, coset_fft, the H block) from "
                         "host buffers")
    ap.add_argument("--dropin", type=int, default=1,
                    help="also time bh_prove from host buffers (the drop-in path; 1-GPU runs)")
    return ap.parse_args()


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_topology():
    """physical cores and sockets from /proc/cpuinfo (hardware threads are not cores)"""
    cores, sockets, phys, core = set(), set(), None, None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                if k == "physical id":
                    phys = v
                    sockets.add(v)
                elif k == "core id":
                    core = v
                elif not k and phys is not None and core is not None:
                    cores.add((phys, core))
                    phys = core = None
    except OSError:
        pass
    if phys is not None and core is not None:
        cores.add((phys, core))
    return len(cores) or None, len(sockets) or None


def cpu_threads(cpu_port):
    """The host threads the CPU baseline may use: the box's CPU share when the environment
    states it (OMP_NUM_THREADS: 16 per GPU on the GPU pool), else every hardware thread."""
    share = os.environ.get("OMP_NUM_THREADS", "")
    return int(share) if share.isdigit() and int(share) > 0 else cpu_port.hardware_threads()


def cpu_baseline(bh, ctx, log_c, log_c_1t, full=None):
    """bench leg only: the oracle's C++ port of bellman's multicore prover core
    (oracle/cpu/bellman_port.cpp), timed on this host's cores on a bounded sample
    (a 2^log_c-constraint MiMC chain, median of 3 after the port's own warm-up), plus a
    1-thread figure on a smaller sample, and (full = (params, rounds, proof)) one run at the
    headline size.  Its proofs must equal the GPU's."""
    from oracle import cpu_port
    rounds = (1 << (log_c - 1)) - 1
    params = bh.Parameters.chain(ctx, rounds)
    gpu_proof = bh.prove_witness(ctx, params, bh.Witness.chain(ctx, rounds), 27134, 17146)
    threads = cpu_threads(cpu_port)
    reps = 3
    t0 = time.time()
    proof, ms, ms_syn = cpu_port.chain_prove(params.write(), rounds, threads=threads, reps=reps)
    wall = time.time() - t0
    n_c = 2 * rounds + 2
    phys, sockets = cpu_topology()
    out = {"value": round(n_c / (ms / 1e3), 1), "unit": "constraints/s", "cores": threads, "kind": "port",
           "threads_are": "host threads used: the box's CPU share (OMP_NUM_THREADS) when set, else every "
                          "hardware thread", "machine_physical_cores": phys,
           "sockets": sockets, "cpu_model": cpu_model(),
           "sample": f"median of {reps} prover-core runs (assignment -> proof) of a 2^{log_c}-constraint "
                     f"MiMC chain; bellman's multicore algorithm restated in C++ (oracle/cpu); "
                     f"{wall:.1f} s CPU wall incl. synthesis",
           "ms_per_proof": round(ms, 1), "synthesis_ms": round(ms_syn, 1),
           "end_to_end_value": round(n_c / ((ms + ms_syn) / 1e3), 1),
           "proof_matches_gpu": proof == gpu_proof}
    if full is not None:
        # the same port once at the headline size, in this run: the bench's own 2^22 Parameters
        # and chain, the same threads; its proof must equal the bench's proof
        fparams, frounds, fproof = full
        t0 = time.time()
        pbytes = fparams.write()
        proof_f, ms_f, syn_f = cpu_port.chain_prove(pbytes, frounds, threads=threads, reps=1)
        del pbytes
        nf = 2 * frounds + 2
        out["headline_size_run"] = {"log_constraints": nf.bit_length() - 1, "value": round(nf / (ms_f / 1e3), 1),
                                    "unit": "constraints/s", "ms_per_proof": round(ms_f, 1),
                                    "synthesis_ms": round(syn_f, 1), "threads": threads,
                                    "sockets": sockets, "proof_matches_gpu": proof_f == fproof,
                                    "wall_s": round(time.time() - t0, 1),
                                    "source": "timed in this run (one prover-core run, after synthesis)"}
    else:
        for name in ("r03_cpu_baseline_2p22.json", "r02_cpu_baseline_2p22.json"):
            path = os.path.join(ROOT, "profiles", name)
            if os.path.exists(path):  # the same port once at the headline size (tools/cpu_baseline_full.py)
                with open(path) as f:
                    fr = json.loads(f.read().strip().splitlines()[-1])
                out["headline_size_run"] = {k: fr.get(k) for k in ("log_constraints", "value", "ms_per_proof",
                                                                    "threads", "physical_cores", "sockets",
                                                                    "proof_matches_gpu")}
                out["headline_size_run"]["source"] = f"profiles/{name} (a committed run; --cpu-full 1 times it here)"
                break
    if log_c_1t:
        r1 = (1 << (log_c_1t - 1)) - 1
        p1 = bh.Parameters.chain(ctx, r1)
        g1 = bh.prove_witness(ctx, p1, bh.Witness.chain(ctx, r1), 27134, 17146)
        proof1, ms1, _ = cpu_port.chain_prove(p1.write(), r1, threads=1, reps=3)
        out["one_thread"] = {"value": round((2 * r1 + 2) / (ms1 / 1e3), 1), "unit": "constraints/s",
                             "sample": f"median of 3, 2^{log_c_1t}-constraint chain, 1 thread",
                             "proof_matches_gpu": proof1 == g1}
    return out


def c5_leg(bh, args, ctx, world, rank, comm, r, s, barrier):
    """BASELINE.json configs[4]: a batch of independent proofs of one circuit (distinct
    witnesses: preimage seed 8 + i, shared Parameters), split over the ranks with no
    collective (replicas), each rank pipelining its share with bh_prove_batch.  Returns the
    whole-job constraints/s (max over ranks of the batch time)."""
    from concurrent.futures import ThreadPoolExecutor
    rounds = (1 << (args.c5_log_constraints - 1)) - 1
    n_c = 2 * rounds + 2
    params = bh.Parameters.chain(ctx, rounds)
    mine = list(range(rank, args.c5, world))
    t0 = time.time()
    with ThreadPoolExecutor(8) as ex:  # host synthesis in parallel (ctypes releases the GIL)
        ws = list(ex.map(lambda i: bh.Witness.chain(ctx, rounds, seed=7, preimage_seed=8 + i), mine))
    t_syn = time.time() - t0
    params.prepare(ws[0])
    bh.prove_batch(ctx, params, ws[:4], r, s, args.c5_lanes)  # warm-up
    barrier()
    t0 = time.perf_counter()
    proofs = bh.prove_batch(ctx, params, ws, r, s, args.c5_lanes)
    barrier()
    el = time.perf_counter() - t0
    # every batched proof is the single-proof path's proof (spot-check first and last)
    ok = (proofs[0] == bh.prove_witness(ctx, params, ws[0], r, s)
          and proofs[-1] == bh.prove_witness(ctx, params, ws[-1], r, s) and len(set(proofs)) == len(proofs))
    if comm is not None:
        el = comm.allreduce_max(el)
        ok = comm.allreduce_max(0.0 if ok else 1.0) == 0.0
    del ws, params
    return {"workload": f"C5: {args.c5} independent proofs of a 2^{args.c5_log_constraints}-constraint MiMC chain "
                        f"(distinct preimages), {len(mine)} per GPU, bh_prove_batch",
            "value": round(args.c5 * n_c / el, 1), "unit": "constraints/s", "proofs": args.c5,
            "ms_per_proof": round(el * 1e3 / max(1, len(mine)), 3), "batch_s": round(el, 3),
            "lanes": args.c5_lanes or 2, "proofs_match_single": ok, "synthesis_s": round(t_syn, 2)}


def domain_leg(bh, ctx, asg, n_constraints, reps=2):
    """The EvaluationDomain seam (domain.rs:81-189) at the bench's size from host buffers: one
    ifft and one coset_fft (each: upload, device transform, download; the split from device
    events), and the H block of create_proof as prover.rs:210-231 drives it through that seam
    (3 x (ifft, coset_fft), mul_assign, sub_assign, divide_by_z_on_coset, icoset_fft: ten host
    calls), against bh_compute_h (one call) on the same a, b, c; the two h vectors must agree."""
    import numpy as np
    a0, b0, c0 = (np.ascontiguousarray(asg[k]) for k in ("a", "b", "c"))
    d = bh.EvaluationDomain(ctx, a0)
    out = {"log_m": d.exp, "m": d.m}
    for name in ("ifft", "coset_fft"):
        best, split = None, None
        for _ in range(reps + 1):
            d.coeffs[: a0.shape[0]] = a0
            t0 = time.perf_counter()
            getattr(d, name)()
            ms = (time.perf_counter() - t0) * 1e3
            if best is None or ms < best:
                best, split = ms, ctx.last_stats()[18:21]
        out[name] = {"ms": round(best, 3), "upload_ms": round(split[0], 3), "transform_ms": round(split[1], 3),
                     "download_ms": round(split[2], 3),
                     "host_share": round((split[0] + split[2]) / best, 3) if best else None}
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        A, B, C = (bh.EvaluationDomain(ctx, x) for x in (a0, b0, c0))
        for D_ in (A, B, C):
            D_.ifft()
            D_.coset_fft()
        A.mul_assign(B)
        A.sub_assign(C)
        A.divide_by_z_on_coset()
        A.icoset_fft()
        ms = (time.perf_counter() - t0) * 1e3
        best = ms if best is None else min(best, ms)
    h_host_seam = A.coeffs[: A.m - 1].copy()
    del A, B, C
    # the same ten calls on the resident EvaluationDomain (bh_evdom_*): the coefficients stay in
    # HBM, each from_coeffs streams in while the previous domain transforms; h read back at the
    # end (into_coeffs) -- and, for a caller swapping multiexp too, handed over on the device
    rbest, sbest = None, None
    h_seam = np.zeros((d.m - 1, 4), dtype=np.uint64)  # the caller's h buffer, reused (as h below)
    h_seam[:] = 1
    for _ in range(reps):
        t0 = time.perf_counter()
        A, B, C = (bh.ResidentEvaluationDomain(ctx, x) for x in (a0, b0, c0))
        for D_ in (A, B, C):
            D_.ifft()
            D_.coset_fft()
        A.mul_assign(B)
        B.close()  # drop(b), prover.rs:222
        A.sub_assign(C)
        C.close()
        A.divide_by_z_on_coset()
        A.icoset_fft()
        A.as_mont(A.m - 1, out=h_seam)
        ms = (time.perf_counter() - t0) * 1e3
        A.close()
        rbest = ms if rbest is None else min(rbest, ms)
        t0 = time.perf_counter()
        hs = bh.compute_h_resident(ctx, a0, b0, c0, scalars=True)
        ctx.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        sbest = ms if sbest is None else min(sbest, ms)
        hs.close()
    import ctypes
    h = np.zeros((d.m - 1, 4), dtype=np.uint64)
    hl = ctypes.c_size_t()
    hbest = None
    for _ in range(reps):
        t0 = time.perf_counter()
        bh._check(bh._lib.bh_compute_h(ctx.h, bh._ptr(a0), bh._ptr(b0), bh._ptr(c0), a0.shape[0], bh._ptr(h),
                                       ctypes.byref(hl)), "bh_compute_h")
        ms = (time.perf_counter() - t0) * 1e3
        hbest = ms if hbest is None else min(hbest, ms)
    out["h_via_domain_seam"] = {"ms": round(rbest, 3), "calls": 10, "domain": "resident (bh_evdom)",
                                "value": round(n_constraints / (rbest / 1e3), 1), "unit": "constraints/s",
                                "vs_bh_compute_h": round(rbest / hbest, 3)}
    out["h_via_domain_seam_to_scalars"] = {"ms": round(sbest, 3), "note": "h left on the device (into_scalars) "
                                           "for the multiexp seam; timed to device completion"}
    out["h_via_host_domain"] = {"ms": round(best, 3), "calls": 10, "domain": "host buffers (bh_fft & co.)"}
    out["h_via_bh_compute_h"] = {"ms": round(hbest, 3), "calls": 1}
    out["h_equal"] = bool(np.array_equal(h_seam, h[: hl.value]) and np.array_equal(h_host_seam, h[: hl.value]))
    out["note"] = ("ifft / coset_fft: host (Montgomery) buffers in and out of every call (bh_fft & co.), most of "
                   "it PCIe (host_share); h_via_domain_seam: the resident domain, uploads of a, b, c and the "
                   "download of h only")
    return out


def main():
    args = parse()
    import bh_launch  # pure Python: loads no HIP library
    try:
        world, rank, local, spawn = bh_launch.rank_env(args.gpus)
    except bh_launch.LaunchError as e:
        print(f"bench.py: {e}", file=sys.stderr)
        sys.exit(2)
    # the hardware-queue setting the library will raise (include/bellman_hip.h), recorded as found
    hwq_env = os.environ.get("GPU_MAX_HW_QUEUES")
    hwq_keep = os.environ.get("BH_KEEP_HW_QUEUES") == "1"
    # (the library reads it with atoi: an unparseable value counts as 0 and is raised too)
    hwq_ok = bool(hwq_env) and hwq_env.strip().isdigit() and int(hwq_env) >= 16
    hw_queues = {"env": hwq_env, "effective": hwq_env if hwq_keep or hwq_ok else "16",
                 "raised_by_library": not hwq_keep and not hwq_ok}
    if spawn:
        # plain `python bench.py --gpus N`: start the N rank processes (one per GPU, LOCAL_RANK =
        # device) before this parent touches HIP, and exit with the first failing rank's code
        rc = bh_launch.spawn_ranks(world, [os.path.abspath(__file__)] + sys.argv[1:])
        sys.exit(rc if rc >= 0 else 128 - rc)
    import bellman_hip as bh

    device = local
    if world > 1:
        ndev = bh.device_count()
        if ndev < world:
            print(f"bench.py rank {rank}: --gpus {world} needs {world} devices, HIP sees {ndev}", file=sys.stderr)
            sys.exit(3)
    k = args.log_constraints
    rounds = (1 << (k - 1)) - 1
    n_constraints = 2 * rounds + 2
    ctx = bh.Context(device)
    t0 = time.time()
    params = bh.Parameters.chain(ctx, rounds)
    t_params = time.time() - t0
    t0 = time.time()
    witness = bh.Witness.chain(ctx, rounds)
    t_wit = time.time() - t0
    t0 = time.time()
    prepared = None
    if args.tables:
        # SRS window tables: a function of the CRS only.  A rank of an N-GPU run builds exactly
        # the slices its shard reads (and, with the H block distributed, the table over its own
        # share of h) -- the per-rank tables tools/shard_rehearsal.py times, 1/N of the memory
        # and setup of the full tables
        if world > 1:
            params.prepare_shard(witness, rank, world, distributed_h=True)
            prepared = "shard"
        else:
            params.prepare(witness)
            prepared = "full"
    else:
        ctx.set_tables(False)
    t_tables = time.time() - t0
    r, s = 27134, 17146
    vk = params.vk_bytes()
    comm, rccl = None, None
    if world > 1:
        # RCCL communicator over xGMI: the unique id travels through a rendezvous file, every
        # other byte through RCCL.  Any failure ends this rank (and the launcher the run).
        rdzv = bh_launch.rendezvous_dir()
        if rank == 0:
            uid = bh.Comm.unique_id()
            bh_launch.publish(rdzv, "uid", uid)
        else:
            uid = bh_launch.wait_for(rdzv, "uid", timeout=600)
        comm = bh.Comm(ctx, uid, world, rank)
        if rank == 0:
            bh_launch.cleanup(rdzv)
        n_seen, r_seen, d_seen = comm.info()
        if (n_seen, r_seen, d_seen) != (world, rank, device):
            print(f"bench.py rank {rank}: RCCL reports ranks={n_seen} rank={r_seen} device={d_seen}, "
                  f"expected {world}/{rank}/{device}", file=sys.stderr)
            sys.exit(4)
        recs = comm.allgather_bytes(json.dumps([rank, device, os.getpid()]).encode().ljust(64))
        rccl = {"ranks": n_seen, "devices": [json.loads(x.decode().strip())[1] for x in recs]}
        if len(set(rccl["devices"])) != world:
            print(f"bench.py: ranks share devices {rccl['devices']}", file=sys.stderr)
            sys.exit(4)

    def step():
        if world == 1:
            return bh.prove_witness(ctx, params, witness, r, s)
        # this rank's share of every multiexp (H block distributed over RCCL for N >= 2),
        # the 960-byte partial records all-gathered over RCCL, rank 0 sums and assembles
        parts = comm.allgather(comm.prove_partial(ctx, params, witness))
        if rank == 0:
            return bh.proof_from_partials(vk, parts, world, r, s)
        return None

    def barrier():
        ctx.synchronize()
        if comm is not None:
            comm.allreduce_max(0.0)

    ref = None
    for _ in range(args.warmup):
        ref = step()
    barrier()
    timings, unions = [], []
    t_start = time.perf_counter()
    for _ in range(args.steps):
        p = step()
        if rank == 0:
            if args.check and ref is not None:
                assert p == ref, "proof bytes changed between steps"
            ref = p
            timings.append(ctx.last_timings())
            unions.append(list(ctx.last_stats()[21:23]))
    barrier()
    elapsed = time.perf_counter() - t_start
    # window tables the timed proofs read (rank 0 of N, or every rank's own slices for N > 1)
    st = ctx.last_stats()
    tables = {"used": int(st[10]), "large_multiexps": int(st[11]), "GB": round(st[12] / 1e9, 2),
              "prepare": prepared, "setup_s": round(t_tables, 2)}
    per_rank_ms = None
    if comm is not None:
        mine = [elapsed * 1000.0 / args.steps, tables["used"], tables["large_multiexps"], tables["GB"], prepared,
                round(t_tables, 2)]
        recs = [json.loads(x.decode().strip()) for x in comm.allgather_bytes(json.dumps(mine).encode().ljust(128))]
        per_rank_ms = [round(x[0], 3) for x in recs]
        tables = {"used": [x[1] for x in recs], "large_multiexps": [x[2] for x in recs], "GB": [x[3] for x in recs],
                  "prepare": [x[4] for x in recs], "setup_s": [x[5] for x in recs]}
        elapsed = comm.allreduce_max(elapsed)
    ms = elapsed * 1000.0 / args.steps
    value = n_constraints * args.steps / elapsed
    # dominant kernel: G1 bucket accumulation (k_accumulate_pf<G1>), device events around every
    # launch of the timed steps; algorithmic bytes = 128 B per (base, scalar) pair
    acc_ms = sum(t[2] for t in timings)
    launches = sum(t[3] for t in timings)
    pairs = sum(t[4] for t in timings)
    # The kernel's own time: the union of its launches' event intervals per proof (bh_last_stats
    # [21]).  Two accumulation lanes run G1 launches side by side, so the summed launch time counts
    # shared time twice (4 launches x the co-run average exceeded ms_per_step in round 5); the
    # union never exceeds the step and is what the G1 multiexps cost the proof.
    g1_union = sum(u[0] for u in unions if len(u) == 2)
    kern_ms = g1_union if g1_union > 0 else acc_ms
    achieved = (pairs * G1_PAIR_BYTES / 1e9) / (kern_ms / 1e3) if kern_ms > 0 else None
    corun = (pairs * G1_PAIR_BYTES / 1e9) / (acc_ms / 1e3) if acc_ms > 0 else None
    traffic, traffic_src = None, None
    tpath = os.path.join(ROOT, "profiles", TRAFFIC_FILE)
    if os.path.exists(tpath) and k == 22:
        with open(tpath) as f:
            traffic = round(json.load(f)["traffic_bytes_per_launch"])
        traffic_src = f"profiles/{TRAFFIC_FILE} (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, separate passes)"
    alg_per_launch = pairs * G1_PAIR_BYTES / launches if launches else None
    roof = {"bound": "hbm", "kernel": "k_accumulate_pf<G1>",
            "achieved": round(achieved, 2) if achieved else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5) if achieved else None, "traffic": traffic,
            "traffic_source": traffic_src,
            "avg_launch_ms": round(kern_ms / launches, 4) if launches else None,
            "launches_per_proof": round(launches / max(1, len(timings)), 2),
            "kernel_ms_per_proof": round(kern_ms / max(1, len(timings)), 3),
            "avg_launch_source": ("union of the launches' HIP-event intervals per proof (bh_last_stats [21], events "
                                  "recorded on the stream each launch runs on) / launches per proof"
                                  if g1_union > 0 else "HIP events around every launch (summed)"),
            "corun_avg_launch_ms": round(acc_ms / launches, 4) if launches else None,
            "corun_frac": round(corun / HBM_PEAK_GBS, 5) if corun else None,
            "corun_source": "summed per-launch event durations: two G1 launches often co-run (two lanes), so "
                            "this average counts shared time twice",
            "algorithmic_bytes_per_launch": round(alg_per_launch) if launches else None,
            "note": "VALU-bound (XYZZ mixed additions on 29-bit limbs): see DESIGN.md section 4"}
    # the same kernel in the committed profiles of this workload: its rocprofv3 kernel-trace average
    # (same co-running schedule; must agree with avg_launch_ms) and its solo duration in the counter
    # passes (rocprofv3 --pmc serialises dispatches)
    ppath = os.path.join(ROOT, "profiles", PMC_FILE)
    if os.path.exists(ppath) and k == 22 and launches:
        with open(ppath) as f:
            pmc = json.load(f)
        tu = pmc.get("trace_g1_accumulate_union")
        if tu:
            # the same union from the rocprofv3 kernel trace of the same workload
            roof["rocprof_avg_launch_ms"] = tu["per_launch_ms"]
            roof["rocprof_frac"] = round(alg_per_launch / (tu["per_launch_ms"] / 1e3) / 1e9 / HBM_PEAK_GBS, 5)
            roof["rocprof_source"] = f"profiles/{PMC_FILE} trace_g1_accumulate_union ({tu['source']})"
            roof["events_vs_rocprof"] = round((kern_ms / launches) / tu["per_launch_ms"], 4)
        tr = pmc.get("trace_g1_accumulate")
        if tr:
            roof["rocprof_corun_avg_launch_ms"] = tr["avg_ms"]
            roof["rocprof_corun_source"] = f"profiles/{PMC_FILE} trace_g1_accumulate ({tr['source']})"
        solo = pmc.get("k_accumulate_pf<CurveOps<FpOps", {}).get("avg_dispatch_ms_grbm_pass")
        if solo:
            roof["solo_avg_launch_ms"] = solo
            roof["solo_frac"] = round(alg_per_launch / (solo / 1e3) / 1e9 / HBM_PEAK_GBS, 5)
    # integer-ALU roofline: G1 mixed additions/s against the microbenchmarked peak, and the
    # v_mad_u64_u32 issue rate they imply (see MADS_PER_G1_MADD)
    g1_adds = sum(t[8] for t in timings)
    # the rate while G1 accumulations run: over the union of their launches (two accumulation
    # lanes overlap launches, so the summed launch time would count shared time twice)
    g1_wall = g1_union
    busy_ms = g1_wall if g1_wall > 0 else acc_ms
    madd_rate = g1_adds / (busy_ms / 1e3) / 1e9 if busy_ms > 0 else None
    valu = {"kernel": "k_accumulate_pf<G1>", "unit": "G mixed-add/s",
            "achieved": round(madd_rate, 3) if madd_rate else None, "peak": G1_MADD_PEAK,
            "g1_accumulation_wall_ms_per_proof": round(busy_ms / max(1, len(timings)), 3),
            "achieved_source": ("G1 mixed additions / the wall time during which at least one G1 accumulation "
                                "ran (bh_last_stats [21], union of the launches' events)" if g1_wall > 0 else
                                "G1 mixed additions / summed G1 launch time"),
            "frac": round(madd_rate / G1_MADD_PEAK, 4) if madd_rate else None,
            "peak_source": "tools/microbench/curvebench.hip (L2-resident bases, 2 waves/SIMD)",
            "mad_u64_tps": round(madd_rate * MADS_PER_G1_MADD / 1e3, 2) if madd_rate else None,
            "mad_u64_frac": round(madd_rate * MADS_PER_G1_MADD / 1e3 / MAD_U64_PEAK_TPS, 4) if madd_rate else None,
            "mad_u64_peak_tps": MAD_U64_PEAK_TPS, "mad_u64_peak_source": "tools/microbench/madbench.hip"}
    # the clock the chip holds under this kernel (GRBM_GUI_ACTIVE / 8 XCDs / wall time, from the
    # committed PMC passes; 2.4 GHz peak): the VALU peaks above are per-clock rates at whatever
    # clock the microbenchmark ran ('DVFS')
    cpath = os.path.join(ROOT, "profiles", PMC_FILE)
    if os.path.exists(cpath):
        with open(cpath) as f:
            g1pmc = json.load(f).get("k_accumulate_pf<CurveOps<FpOps", {})
        if "held_clock_ghz" in g1pmc:
            valu["held_clock_ghz"] = g1pmc["held_clock_ghz"]
            valu["held_clock_source"] = f"profiles/{PMC_FILE} (GRBM_GUI_ACTIVE, counter passes)"
            # the microbenchmark peak was taken at its own held clock: scaled to this kernel's
            scaled = G1_MADD_PEAK * g1pmc["held_clock_ghz"] / G1_MADD_PEAK_CLOCK_GHZ
            valu["peak_clock_scaled"] = round(scaled, 3)
            valu["frac_clock_scaled"] = round(madd_rate / scaled, 4) if madd_rate else None
            valu["peak_clock_source"] = ("curvebench at %.2f GHz (profiles/r03_curvebench_clock.txt)"
                                         % G1_MADD_PEAK_CLOCK_GHZ)
    # whole-proof VALU issue: the PMC pass's VALU wave-instructions per proof (every kernel)
    # against the rate the G1 accumulation issues at alone
    proof_valu = None
    ppath = os.path.join(ROOT, "profiles", PMC_FILE)
    if os.path.exists(ppath) and k == 22 and world == 1:
        with open(ppath) as f:
            pmc = json.load(f)
        per = [v for v in pmc.values() if isinstance(v, dict) and "SQ_INSTS_VALU" in v]
        if per and pmc.get("proofs"):
            n_proofs = pmc["proofs"]
            wi = sum(v["SQ_INSTS_VALU"] * v["dispatches"]["SQ_INSTS_VALU"] for v in per) / n_proofs
            rate = wi / (ms / 1e3) / 1e9
            proof_valu = {"wave_instructions_per_proof": round(wi), "achieved": round(rate, 1),
                          "peak": SOLO_WAVE_INSTR_RATE, "unit": "G VALU wave-instructions/s",
                          "frac": round(rate / SOLO_WAVE_INSTR_RATE, 4),
                          "source": f"profiles/{PMC_FILE} (SQ_INSTS_VALU, every dispatch) / this run's ms_per_step",
                          "peak_source": "k_accumulate_pf<G1> alone (BH_PROVER_SERIAL=1): 6.38 G madd/s x 5116 / 64"}
    c5 = c5_leg(bh, args, ctx, world, rank, comm, r, s, barrier) if args.c5 else None
    if rank != 0:
        comm.close()
        return
    # the drop-in path: bh_prove from the ProvingAssignment's host
    # buffers, i.e. the resident-witness step plus streaming ~0.5 GB of witness over PCIe
    # (pinned ring, overlapped with the first sorts and accumulation)
    dropin = None
    if args.dropin and world == 1:
        asg = bh.chain_assignment(rounds)
        p0 = bh.prove(ctx, params, asg, r, s)
        ctx.synchronize()
        t0 = time.perf_counter()
        landed = []
        for _ in range(args.steps):
            pd = bh.prove(ctx, params, asg, r, s)
            landed.append([round(x, 2) for x in ctx.last_stats()[13:18]])
        ctx.synchronize()
        dms = (time.perf_counter() - t0) * 1000.0 / args.steps
        wbytes = sum(int(v.nbytes) for v in asg.values())
        dropin = {"value": round(n_constraints / (dms / 1e3), 1), "unit": "constraints/s", "ms_per_step": round(dms, 3),
                  "witness_bytes": wbytes, "proof_matches": pd == p0 == ref,
                  "landed_ms": {"fields": ["inputs+aux", "a", "b", "c", "H done"], "per_call": landed,
                                "source": "device events on the copy and H streams, ms from the call's start"},
                  "note": "bh_prove from host (pageable) buffers: witness upload overlapped with the proof"}
        # the proof is valid: the native verifier (verify_proof, verifier.rs:23-62) on the public
        # input (the chain's image; input 0 is ONE)
        public = bh.fr_from_mont(asg["inputs"])[1:]
        t0 = time.perf_counter()
        dropin["proof_verifies"] = bh.verify_proof(vk, ref, public)
        dropin["verify_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
        # the multiexp-level seam: the same host buffers through
        # bh_compute_h_scalars + bh_scalars_upload + eight bh_multiexp_submit_scalars on the
        # Parameters' vectors + the host assembly, i.e. what a caller swapping only multiexp()
        # and the H block gets
        if args.seam:
            # two untimed calls: the first sizes one job slot per multiexp kind, the second settles
            # the derived-sort scratch of the slots that copy or compact another job's sort
            s0 = bh.prove_seam(ctx, params, asg, r, s)
            bh.prove_seam(ctx, params, asg, r, s)
            ctx.synchronize()
            t0 = time.perf_counter()
            stamps, call_ms = [], []
            for _ in range(args.steps):
                tc = time.perf_counter()
                ps = bh.prove_seam(ctx, params, asg, r, s, profile=stamps)
                call_ms.append(round((time.perf_counter() - tc) * 1e3, 2))
            ctx.synchronize()
            sms = (time.perf_counter() - t0) * 1000.0 / args.steps
            dropin["seam"] = {"value": round(n_constraints / (sms / 1e3), 1), "unit": "constraints/s",
                              "ms_per_step": round(sms, 3), "vs_dropin": round(dms / sms, 4),
                              "proof_matches": ps == s0 == ref,
                              "per_call": {"ms": call_ms, "h_producer_ms": stamps,
                                           "fields": "bh_scalars_stamps: a, b, c copies enqueued, H enqueued, "
                                                     "deferred multiexps enqueued (ms since the call), "
                                                     "multiexps deferred"},
                              "note": "prove_seam: h on the device, assignments uploaded once, 8 multiexp "
                                      "jobs on the Parameters' vectors (window tables), host assembly"}
        if args.domain:
            dropin["domain_seam"] = domain_leg(bh, ctx, asg, n_constraints)
        del asg
    # CPU baseline: rank 0 of a 1-GPU run only (a bounded sample; see cpu_baseline)
    base = (cpu_baseline(bh, ctx, args.cpu_log_constraints, args.cpu_1t_log_constraints,
                         (params, rounds, ref) if args.cpu_full else None)
            if args.cpu_baseline and world == 1 else None)
    out = {
        "metric": "Groth16 constraints/sec, BLS12-381, 2^22-constraint R1CS",
        "value": round(value, 1),
        "unit": "constraints/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u32 limbs (BLS12-381 Fp/Fr modular integer)",
        "data": "synthetic MiMC-chain witness (splitmix64 seed 7), device-generated CRS (alpha=6,beta=24,gamma=6,delta=24,tau=2)",
        "config": {"workload": f"C3: full create_proof after synthesis, MiMC chain R={rounds}",
                   "constraints": n_constraints, "log_domain": k, "parallelism": f"msm-shard{world}",
                   "exchange": "rccl" if world > 1 else None},
        "rccl": rccl,
        "gpu_max_hw_queues": hw_queues,
        # scratch (private segment) budget of the library's spilling kernels against the device's
        # shared scratch limit, checked before every proof ('Scratch budget')
        "scratch": ctx.scratch_report(),
        "per_rank_ms_per_step": per_rank_ms,
        "srs_window_tables": tables,
        "dropin": dropin,
        "c5": c5,
        "roofline": roof,
        "valu_roofline": valu,
        "proof_valu_issue": proof_valu,
        "end_to_end": {"value": round(n_constraints / (t_wit + ms / 1e3), 1), "unit": "constraints/s",
                       "note": "host witness synthesis (native; serial MiMC recurrence, rows/densities/constants on several threads) + upload + prover core"},
        "cpu_baseline": base,
        "breakdown_ms": {"h_pipeline": round(sum(t[1] for t in timings) / len(timings), 3),
                         "g1_accumulate": round(acc_ms / len(timings), 3),
                         "g2_accumulate": round(sum(t[5] for t in timings) / len(timings), 3),
                         "g1_pairs": int(timings[-1][4]), "g2_pairs": int(timings[-1][7]),
                         "g1_adds": int(timings[-1][8]), "g2_adds": int(timings[-1][9]),
                         "host_wall_prove": round(sum(t[0] for t in timings) / len(timings), 3)},
        "setup_s": {"crs_generation": round(t_params, 2), "witness_synthesis_and_upload": round(t_wit, 2),
                    "srs_window_tables": round(t_tables, 2) if args.tables else None},
        "proof_sha_prefix": ref.hex()[:32] if ref else None,
    }
    print(json.dumps(out), flush=True)
    if comm is not None:
        comm.close()


if __name__ == "__main__":
    main()
