"""World-size-2 `gloo` test of the multi-GPU path on CPU.

Each rank computes the partial sums of the 8 multiexps over its scalar shard
(bh.shard_range, the product's sharding rule).  Without a GPU the per-shard MSM
is computed by the oracle (standing in for bh_prove_witness_partial); the
partial records are all-gathered over gloo and rank 0 combines them with the
product's host-only bh_proof_from_partials.  The result must equal the golden
single-device proof byte for byte."""
import json
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _partials(fx, shard, nshards):
    import bellman_hip as bh
    from oracle import bellman as bm
    from oracle import bls12_381 as bls
    E = bm.BLS12_381
    data = bytes.fromhex(fx["params"])
    # Parameters::read layout (groth16/mod.rs:292-400)
    off = 96 * 3 + 192 * 3
    n_ic = int.from_bytes(data[off:off + 4], "big")
    off += 4 + 96 * n_ic
    vecs = []
    for width in (96, 96, 96, 96, 192):
        n = int.from_bytes(data[off:off + 4], "big")
        off += 4
        dec = bls.g1_from_uncompressed if width == 96 else bls.g2_from_uncompressed
        vecs.append([dec(data[off + i * width: off + (i + 1) * width])[1] for i in range(n)])
        off += n * width
    h_b, l_b, a_b, b1_b, b2_b = vecs
    a, b, c = ([int(x, 16) for x in fx[k]] for k in "abc")
    inputs = [int(x, 16) for x in fx["inputs"]]
    aux = [int(x, 16) for x in fx["aux"]]
    dens = {k: [ch == "1" for ch in fx[k]] for k in ("a_aux_density", "b_input_density", "b_aux_density")}
    h = bm.compute_h(E, a, b, c)
    b_in_total = sum(dens["b_input_density"])

    def part(G, bases, base_off, exps, density):
        lo, hi = bh.shard_range(len(exps), shard, nshards)
        acc = G.identity
        j = base_off + (sum(density[:lo]) if density is not None else lo)
        for i in range(lo, hi):
            if density is not None and not density[i]:
                continue
            acc = G.add(acc, G.mul(G.from_affine(bases[j]), exps[i]))
            j += 1
        return G.to_affine(acc)

    g1 = [part(E.G1, h_b, 0, h, None), part(E.G1, l_b, 0, aux, None), part(E.G1, a_b, 0, inputs, None),
          part(E.G1, a_b, len(inputs), aux, dens["a_aux_density"]),
          part(E.G1, b1_b, 0, inputs, dens["b_input_density"]),
          part(E.G1, b1_b, b_in_total, aux, dens["b_aux_density"])]
    g2 = [part(E.G2, b2_b, 0, inputs, dens["b_input_density"]),
          part(E.G2, b2_b, b_in_total, aux, dens["b_aux_density"])]
    rec = b"".join(bls.g1_to_uncompressed(p) for p in g1) + b"".join(bls.g2_to_uncompressed(p) for p in g2)
    assert len(rec) == bh.PARTIAL_BYTES
    vk = data[:96 * 3 + 192 * 3 + 4 + 96 * n_ic]
    return rec, vk


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "bellman-mpc_amd"))
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        fx = [p for p in json.load(f)["proofs"] if p["name"] == "mimc_chain_r7"][0]
    rec, vk = _partials(fx, rank, world)
    t = torch.frombuffer(bytearray(rec), dtype=torch.uint8)
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    if rank == 0:
        import bellman_hip as bh
        parts = b"".join(bytes(x.numpy().tobytes()) for x in out)
        proof = bh.proof_from_partials(vk, parts, world, fx["r"], fx["s"])
        q.put(proof.hex() == fx["proof"])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_msm_gather_combine_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    assert ok
    assert all(p.exitcode == 0 for p in procs)


def test_shard_ranges_partition():
    import bellman_hip as bh
    for n in (0, 1, 2, 7, 1000, (1 << 22) - 1):
        for N in (1, 2, 3, 8):
            spans = [bh.shard_range(n, k, N) for k in range(N)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[k][1] == spans[k + 1][0] for k in range(N - 1))


# ---------------------------------------------------------------- distributed H (dist_h.hip)
def _dist_h_share(a, b, c, N, rank, exchange):
    """This rank's share {k: h[k]} of the H block computed as dist_h.hip does (three
    all-to-alls, local M-point transforms, N-point DFTs); `exchange(blocks)` sends
    blocks[p] to rank p and returns the blocks received, indexed by source rank."""
    from oracle import bls12_381 as bls
    q = bls.R
    m = len(a)
    L = m.bit_length() - 1
    M, C = m // N, m // N // N
    w = pow(bls.FR_ROOT_OF_UNITY, 1 << (32 - L), q)
    wi = pow(w, q - 2, q)
    wN, wNi = pow(w, M, q), pow(wi, M, q)
    g, gi = 7, pow(7, q - 2, q)
    minv = pow(m, q - 2, q)
    zinv = pow((pow(g, m, q) - 1) % q, q - 2, q)

    def dft(x, root):
        n = len(x)
        return [sum(x[j] * pow(root, j * k, q) for j in range(n)) % q for k in range(n)]

    # phase 1: residue class r, local inverse M-point NTT (root w^-N)
    Y = [dft([v[N * j + rank] for j in range(M)], pow(wi, N, q)) for v in (a, b, c)]
    got = exchange([[y[p * C:(p + 1) * C] for y in Y] for p in range(N)])
    # phase 2: inverse N-DFT over sources (twiddle w^-qr), coset scale, forward N-DFT (w^qr)
    rows = [[[0] * C for _ in range(3)] for _ in range(N)]
    for vi in range(3):
        for u in range(C):
            qq = rank * C + u
            R = [got[r][vi][u] * pow(wi, qq * r, q) % q for r in range(N)]
            X = dft(R, wNi)
            X = [X[t] * pow(g, t * M + qq, q) * minv % q for t in range(N)]
            Wv = dft(X, wN)
            for r2 in range(N):
                rows[r2][vi][u] = Wv[r2] * pow(w, qq * r2, q) % q
    got = exchange(rows)
    V = [sum((got[src][vi] for src in range(N)), []) for vi in range(3)]  # natural q
    # phase 3: forward M-point NTTs (root w^N), a*b - c, / Z(g), inverse M-point NTT
    Fa, Fb, Fc = (dft(v, pow(w, N, q)) for v in V)
    hc = [(Fa[j] * Fb[j] - Fc[j]) * zinv % q for j in range(M)]
    Yh = dft(hc, pow(wi, N, q))
    got = exchange([[Yh[p * C:(p + 1) * C]] for p in range(N)])
    # final: inverse N-DFT over sources, icoset scale
    share = {}
    for u in range(C):
        qq = rank * C + u
        R = [got[r][0][u] * pow(wi, qq * r, q) % q for r in range(N)]
        X = dft(R, wNi)
        for t in range(N):
            k = t * M + qq
            share[k] = X[t] * pow(gi, k, q) * minv % q
    return share


def _dist_h_worker(rank, world, port, q):
    import random
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import bls12_381 as bls
    rng = random.Random(1234)
    m = 64
    a, b, c = ([rng.randrange(bls.R) for _ in range(m)] for _ in range(3))

    def exchange(blocks):
        allb = [None] * world
        dist.all_gather_object(allb, blocks)
        return [allb[src][rank] for src in range(world)]

    share = _dist_h_share(a, b, c, world, rank, exchange)
    shares = [None] * world
    dist.all_gather_object(shares, share)
    if rank == 0:
        from oracle import bellman as bm
        want = bm.compute_h(bm.BLS12_381, a, b, c)
        merged = {}
        for s in shares:
            assert not set(s) & set(merged)
            merged.update(s)
        q.put(sorted(merged) == list(range(m)) and [merged[k] for k in range(m - 1)] == want)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_distributed_h_gloo(world):
    """The distributed H block (dist_h.hip's index algebra and exchange pattern) with `world`
    gloo ranks: the union of the ranks' shares is the oracle's H (prover.rs:210-231)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dist_h_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    assert ok
    assert all(p.exitcode == 0 for p in procs)
