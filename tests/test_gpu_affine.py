"""Batch-affine bucket accumulation (csrc/msm_g1_aff.hip) on the GPU, through the C ABI.

The levels are opt-in (BH_AFFINE / BH_AFFINE_G1 / BH_AFFINE_G2 = 1; off by default: slower than the
XYZZ accumulation at 2^22), so the default full-size proof tests do NOT cover
them; these forced small-size tests are their coverage.  The plan's knobs (read from the environment
on every multiexp) force levels at small sizes, so that the exceptional pairs -- P + P (doubling) and P + (-P) (the point at
infinity, carried as a marked record) -- occur inside table buckets, at level 0 and deeper, and
results are compared with the oracle and with the XYZZ-only accumulation (BH_AFFINE=0).
Reference: multiexp.rs:191-223 (the bucket loop the levels replace)."""
import contextlib
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def _bh():
    import bellman_hip as bh
    return bh


@contextlib.contextmanager
def env(**kv):
    old = {k: os.environ.get(k) for k in kv}
    os.environ.update({k: str(v) for k, v in kv.items()})
    try:
        yield
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


FORCE = dict(BH_AFFINE=1, BH_AFF_KMIN=1, BH_AFF_ROUNDS=1, BH_AFF_MIN_E=1)


def _exps_array(vals):
    a = np.zeros((len(vals), 4), dtype=np.uint64)
    for i, v in enumerate(vals):
        for k in range(4):
            a[i, k] = (v >> (64 * k)) & 0xFFFFFFFFFFFFFFFF
    return a


def test_affine_exceptional_pairs_in_table_buckets(ctx):
    """l replaced by multiples of the generator from a small set {11, -11, 29, 22} (so equal and
    opposite points sit under equal digits in the same bucket, at every level), scalars from a
    small set: the table multiexp with forced affine levels equals sum(e_i k_i) * G (oracle) and
    the XYZZ-only result."""
    bh = _bh()
    from oracle import bellman as bm
    from oracle import bls12_381 as bls
    from params_bytes import split_params
    E = bm.BLS12_381
    G = E.G1
    gen = bls.G1.generator()
    rounds = (1 << 16) - 1
    base = bh.Parameters.chain(ctx, rounds)
    raw = base.write()
    sp = split_params(raw)
    n = sp["l_len"]
    ks = [11, R - 11, 29, 22]
    enc = {k: bls.g1_to_uncompressed(G.to_affine(G.mul(gen, k))) for k in ks}
    rng = random.Random(3)
    pick = [ks[(i * 7 + (i >> 5)) % 4] for i in range(n)]
    l_bytes = b"".join(enc[k] for k in pick)
    start = raw.index(sp["l"])
    crafted = raw[:start] + l_bytes + raw[start + len(sp["l"]):]
    params = bh.Parameters.read(ctx, crafted, checked=False)
    params.prepare(bh.Witness.chain(ctx, rounds))
    L = params.vector(bh.BH_VEC_L)
    e1, e2 = rng.randrange(R), rng.randrange(R)
    for exps in ([e1 if i % 3 else e2 for i in range(n)],
                 [1 if i % 2 else R - 1 for i in range(n)],
                 [e1] * n):
        want_k = sum(e * k for e, k in zip(exps, pick)) % R
        want = bls.g1_to_uncompressed(G.to_affine(G.mul(gen, want_k)))
        ex = _exps_array(exps)
        with env(**FORCE):
            got = bh.multiexp_async(ctx, L, 0, None, ex).wait()
        with env(BH_AFFINE=0):
            xyzz = bh.multiexp_async(ctx, L, 0, None, ex).wait()
        assert xyzz == want
        assert got == want


def test_affine_exceptional_pairs_g2(ctx):
    """The same for G2: b_g2 replaced by multiples of the G2 generator from {11, -11, 29, 22}, a
    table multiexp over it (level 0 from the packed G2 table records, Fp2 affine levels, one Fp
    inversion of the norm per thread) == sum(e_i k_i) * G2 (oracle) and the XYZZ-only result."""
    bh = _bh()
    from oracle import bellman as bm
    from oracle import bls12_381 as bls
    from params_bytes import split_params
    E = bm.BLS12_381
    G = E.G2
    gen = bls.G2.generator()
    rounds = (1 << 17) - 1
    raw = bh.Parameters.chain(ctx, rounds).write()
    sp = split_params(raw)
    n = sp["b_g2_len"]
    ks = [11, R - 11, 29, 22]
    enc = {k: bls.g2_to_uncompressed(G.to_affine(G.mul(gen, k))) for k in ks}
    pick = [ks[(i * 5 + (i >> 6)) % 4] for i in range(n)]
    start = raw.index(sp["b_g2"])
    crafted = raw[:start] + b"".join(enc[k] for k in pick) + raw[start + len(sp["b_g2"]):]
    params = bh.Parameters.read(ctx, crafted, checked=False)
    w = bh.Witness.chain(ctx, rounds)
    params.prepare(w)
    B2 = params.vector(bh.BH_VEC_B_G2)
    asg = bh.chain_assignment(rounds)
    off = bh.DensityWords(asg["b_input_density"], asg["inputs"].shape[0]).total()
    m = n - off
    rng = random.Random(8)
    e1, e2 = rng.randrange(R), rng.randrange(R)
    for exps in ([e1 if i % 3 else e2 for i in range(m)], [e2] * m):
        want_k = sum(e * k for e, k in zip(exps, pick[off:])) % R
        want = bls.g2_to_uncompressed(G.to_affine(G.mul(gen, want_k)))
        ex = _exps_array(exps)
        with env(**FORCE):
            got = bh.multiexp_async(ctx, B2, off, None, ex).wait()
        with env(BH_AFFINE=0):
            xyzz = bh.multiexp_async(ctx, B2, off, None, ex).wait()
        assert xyzz == want
        assert got == want


@pytest.mark.parametrize("rounds", [(1 << 15) - 1, (1 << 16) - 1])
def test_affine_forced_levels_proof_equals_xyzz(ctx, rounds):
    """Whole proofs with window tables: forced affine levels (several per multiexp at these
    sizes) == the XYZZ-only accumulation, byte for byte."""
    bh = _bh()
    params = bh.Parameters.chain(ctx, rounds)
    w = bh.Witness.chain(ctx, rounds)
    params.prepare(w)
    with env(BH_AFFINE=0):
        want = bh.prove_witness(ctx, params, w, 27134, 17146)
    with env(**FORCE):
        got = bh.prove_witness(ctx, params, w, 27134, 17146)
    assert got == want


@pytest.mark.parametrize("value", [1, 5, R - 1])
def test_affine_forced_levels_degenerate_scalars(ctx, value):
    """Every aux scalar equal (one bucket per window takes every entry: the deepest level tree and
    the longest final-level spans): forced affine levels == plain windows without tables."""
    bh = _bh()
    rounds = (1 << 16) - 1
    params = bh.Parameters.chain(ctx, rounds)
    asg = bh.chain_assignment(rounds)
    asg["aux"][:] = bh.fr_to_mont([value])[0]
    h = bh.ctypes.c_void_p()
    bh._check(bh._lib.bh_witness_upload(ctx.h, bh._ptr(asg["a"]), bh._ptr(asg["b"]), bh._ptr(asg["c"]),
                                        asg["a"].shape[0], bh._ptr(asg["inputs"]), asg["inputs"].shape[0],
                                        bh._ptr(asg["aux"]), asg["aux"].shape[0], bh._ptr(asg["a_aux_density"]),
                                        bh._ptr(asg["b_input_density"]), bh._ptr(asg["b_aux_density"]),
                                        bh.ctypes.byref(h)), "bh_witness_upload")
    w = bh.Witness(ctx, h, asg["a"].shape[0])
    ctx.set_tables(False)
    try:
        plain = bh.prove_witness(ctx, params, w, 27134, 17146)
    finally:
        ctx.set_tables(True)
    params.prepare(w)
    with env(**FORCE):
        assert bh.prove_witness(ctx, params, w, 27134, 17146) == plain


def test_witness_of_ones_tail_latency(ctx):
    """with device-decided tails a bucket holding most entries (a witness full of ones:
    multiexp.rs:193-201's exp == 1 case) used to be folded by one serial chain.  At 2^20 scalars,
    90 % of them 1, the table multiexp (affine levels, then the long-span fold k_cont_long) equals
    plain windows and the host-decided tree fold, and finishes in bounded time."""
    import time
    bh = _bh()
    rounds = (1 << 19) - 1
    params = bh.Parameters.chain(ctx, rounds)
    params.prepare(bh.Witness.chain(ctx, rounds))
    L = params.vector(bh.BH_VEC_L)
    n = params.sizes()["l"]
    rng = np.random.default_rng(4)
    ex = np.zeros((n, 4), dtype=np.uint64)
    ex[:, 0] = 1
    rnd = rng.random(n) < 0.1
    ex[rnd] = rng.integers(0, 2**63, size=(int(rnd.sum()), 4), dtype=np.uint64)
    ex[rnd, 3] &= np.uint64(0x0FFFFFFFFFFFFFFF)
    want = bh.multiexp(ctx, L, 0, None, ex)  # plain per-window buckets
    with env(BH_AFFINE=1):
        got = bh.multiexp_async(ctx, L, 0, None, ex).wait()
        t0 = time.perf_counter()
        got2 = bh.multiexp_async(ctx, L, 0, None, ex).wait()
        dt = time.perf_counter() - t0
    with env(BH_AFFINE=0):
        xyzz = bh.multiexp_async(ctx, L, 0, None, ex).wait()
    assert got == got2 == xyzz == want
    assert dt < 0.5, f"{dt * 1e3:.1f} ms"


def test_scratch_budget_report(ctx):
    """the scratch the spilling kernels need (private segment x 64 lanes x resident waves
    per queue, times the context's queues) is checked against the device limit before proofs and
    multiexps (BH_ERR_SCRATCH_LIMIT instead of an HSA abort); the report names the worst kernel."""
    r = ctx.scratch_report()
    assert r["kernels_checked"] >= 20
    assert r["worst_bytes_per_lane"] > 0 and r["worst_kernel"] != "-"
    assert r["total_need"] == r["worst_per_queue"] * r["queues"]
    assert r["fits"]
    print("scratch report:", r)
