"""GPU parity of the device-resident EvaluationDomain (bh_evdom_*, csrc/evaldomain.hip): the
coefficients stay in HBM from from_coeffs to into_coeffs (domain.rs:21-190), every method is an
enqueue, and the pending transform / constant / coset-power bookkeeping must give exactly the
reference's values -- checked against the oracle's golden vectors, the host-buffer
EvaluationDomain (itself golden-checked), the oracle's serial_fft and the H block."""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
GEN = 7  # Fr::multiplicative_generator()


def _bh():
    import bellman_hip as bh
    return bh


def test_resident_domain_ops_golden(ctx, golden):
    """Every EvaluationDomain method at m = 1 .. 512 (tests/golden/golden.json, oracle-made)."""
    bh = _bh()
    for case in golden["domain"]:
        coeffs = [int(x, 16) for x in case["coeffs"]]
        other = [int(x, 16) for x in case["other"]]
        for op, want in case["results"].items():
            d = bh.ResidentEvaluationDomain(ctx, coeffs)
            if op == "distribute_powers_12345":
                d.distribute_powers(12345)
            elif op in ("mul_assign", "sub_assign"):
                o = bh.ResidentEvaluationDomain(ctx, other)
                getattr(d, op)(o)
                o.close()
            else:
                getattr(d, op)()
            assert [format(v, "x") for v in d.into_coeffs()] == want, (case["log_m"], op)
            d.close()


def _host_apply(bh, ctx, seq, a, b):
    """The same op sequence on the host-buffer EvaluationDomain (bh_fft & co., golden-checked)."""
    d = bh.EvaluationDomain(ctx, a)
    o = bh.EvaluationDomain(ctx, b)
    for op in seq:
        if op[0] == "dist":
            d.distribute_powers(op[1])
        elif op[0] in ("mul_assign", "sub_assign"):
            getattr(d, op[0])(o)
        elif op[0] == "other":
            getattr(o, op[1])()
        else:
            getattr(d, op[0])()
    return d.into_coeffs()


def _dev_apply(bh, ctx, seq, a, b, reads=False):
    d = bh.ResidentEvaluationDomain(ctx, a)
    o = bh.ResidentEvaluationDomain(ctx, b)
    mid = []
    for op in seq:
        if op[0] == "dist":
            d.distribute_powers(op[1])
        elif op[0] in ("mul_assign", "sub_assign"):
            getattr(d, op[0])(o)
        elif op[0] == "other":
            getattr(o, op[1])()
        else:
            getattr(d, op[0])()
        if reads:  # as_ref in the middle leaves the pending state as it was
            mid.append(d.as_ref())
    out = d.into_coeffs()
    d.close()
    o.close()
    return out, mid


TRANSFORMS = ["fft", "ifft", "coset_fft", "icoset_fft", "divide_by_z_on_coset"]


@pytest.mark.parametrize("logm", [0, 1, 3, 9, 11])
def test_resident_random_op_chains_equal_host_domain(ctx, logm):
    """Random chains of methods (transforms in any order, so DIF / DIT alternate from either stored
    order; coset powers that accumulate to +-2 before a transform; an arbitrary distribute_powers
    base; mul / sub against a domain with other pending constants and the other stored order)
    equal the host-buffer EvaluationDomain step for step."""
    bh = _bh()
    rng = random.Random(7000 + logm)
    m = 1 << logm
    for trial in range(6):
        a = [rng.randrange(R) for _ in range(m)]
        b = [rng.randrange(R) for _ in range(m)]
        seq = []
        for _ in range(rng.randrange(3, 9)):
            x = rng.random()
            if x < 0.5:
                seq.append((rng.choice(TRANSFORMS),))
            elif x < 0.62:
                seq.append(("dist", rng.choice([GEN, pow(GEN, R - 2, R), GEN * GEN % R, 12345])))
            elif x < 0.8:
                seq.append(("other", rng.choice(TRANSFORMS)))
            else:
                seq.append((rng.choice(["mul_assign", "sub_assign"]),))
        want = _host_apply(bh, ctx, seq, a, b)
        got, mid = _dev_apply(bh, ctx, seq, a, b, reads=(trial % 2 == 1))
        assert got == want, (logm, seq)
        if mid:
            assert mid[-1] == want


def test_resident_full_range_and_extremes_equal_oracle(ctx):
    """fft / ifft / coset_fft / icoset_fft from natural order, and the same transforms applied
    after an ifft (bit-reversed stored order, DIT), on full-range values and the limb-maximising
    extremes, against the oracle's serial_fft (domain.rs:261-303) at 2^11."""
    bh = _bh()
    from oracle import bellman as bm
    E = bm.BLS12_381
    m = 1 << 11
    rng = np.random.default_rng(211)
    cases = {
        "random": [int.from_bytes(rng.bytes(32), "little") % R for _ in range(m)],
        "r-1": [R - 1] * m,
        "alternating": [(R - 1) if i % 2 == 0 else 0 for i in range(m)],
    }
    for name, vals in cases.items():
        for pre in (None, "ifft"):
            for op in ("fft", "ifft", "coset_fft", "icoset_fft"):
                d = bh.ResidentEvaluationDomain(ctx, vals)
                o = bm.EvaluationDomain(E, list(vals))
                if pre:
                    d.ifft()
                    o.ifft()
                getattr(d, op)()
                getattr(o, op)()
                assert d.into_coeffs() == [int(x) for x in o.coeffs], (name, pre, op)
                d.close()


def test_resident_h_block_golden_and_equal_compute_h(ctx, golden):
    """The H block as create_proof drives EvaluationDomain (prover.rs:210-231, ten calls) on the
    resident domain: the golden h (ragged length, zero padding) and, at 2^16, bh_compute_h's h;
    into_scalars hands the same h to the multiexp without leaving the device."""
    bh = _bh()
    g = golden["h_random"]
    a, b, c = ([int(x, 16) for x in g[k]] for k in "abc")
    assert [format(v, "x") for v in bh.compute_h_resident(ctx, a, b, c)] == g["h"]
    rng = np.random.default_rng(16)
    n = (1 << 16) - 3
    A, B, C = (bh.fr_to_mont([int.from_bytes(rng.bytes(32), "little") % R for _ in range(n)]) for _ in range(3))
    want = bh.compute_h(ctx, A, B, C)
    assert bh.compute_h_resident(ctx, A, B, C) == want
    # h as device scalars: a multiexp over them equals the one over the host h
    params = bh.Parameters.chain(ctx, (1 << 15) - 1)
    H = params.vector(bh.BH_VEC_H)
    hs = bh.compute_h_resident(ctx, A, B, C, scalars=True)
    assert len(hs) == len(want)
    got = bh.multiexp_async(ctx, H, 0, None, hs).wait()
    assert got == bh.multiexp_async(ctx, H, 0, None, want).wait()


@pytest.mark.parametrize("rounds", [15, (1 << 15) - 1])
def test_seam_proof_with_resident_domain_equals_prove(ctx, golden, rounds):
    """A caller that swaps EvaluationDomain AND multiexp: the H block
    through the resident domain, h into the multiexp as a device vector, the eight multiexps on
    the Parameters' vectors -> the bh_prove proof, byte for byte."""
    bh = _bh()
    params = bh.Parameters.chain(ctx, rounds)
    asg = bh.chain_assignment(rounds)
    want = bh.prove(ctx, params, asg, 27134, 17146)
    assert bh.prove_seam(ctx, params, asg, 27134, 17146, h_via_domain=True) == want
    if rounds == 15:
        fx = [f for f in golden["proofs"] if f["name"] == "mimc_chain_r15"][0]
        assert want.hex() == fx["proof"]


def test_resident_domain_write_back_errors_and_pool(ctx):
    """as_mut written back replaces the coefficients behind the queued work; a consumed domain
    and mismatched lengths are errors (the reference asserts); freed buffers are reused across
    sizes without changing results."""
    bh = _bh()
    rng = random.Random(5)
    for logm in (4, 10, 4, 12, 10, 0, 12):
        m = 1 << logm
        a = [rng.randrange(R) for _ in range(m)]
        b = [rng.randrange(R) for _ in range(m)]
        d = bh.ResidentEvaluationDomain(ctx, a)
        d.fft()
        d.write(b)  # behind the fft still pending/queued: b replaces the values
        d.ifft()
        h = bh.EvaluationDomain(ctx, b)
        h.ifft()
        assert d.into_coeffs() == h.into_coeffs()
        d.close()
    d = bh.ResidentEvaluationDomain(ctx, [1, 2, 3])
    o = bh.ResidentEvaluationDomain(ctx, [1, 2, 3, 4, 5])
    with pytest.raises(bh.SynthesisError):
        d.mul_assign(o)
    s = d.into_scalars(3)
    assert len(s) == 3
    with pytest.raises(bh.SynthesisError):
        d.fft()
    d.close()
    o.close()
    assert bh.lib().bh_evdom_fft(None) == bh.BH_ERR_INVALID_ARGUMENT
