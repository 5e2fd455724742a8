"""Pins the CPU oracle (oracle/) to the reference's own known-answer constants
and self-consistency properties.  CPU only."""
import random

import pytest

from oracle import bellman as bm
from oracle import bls12_381 as bls
from oracle import circuits as cc

D = bm.DUMMY
BLS = bm.BLS12_381


def test_dummy_root_of_unity_kat():
    # groth16/tests/mod.rs:334-342
    q = D.Fr.q
    w = D.Fr.root_of_unity
    assert pow(w, 1 << 10, q) == 1
    w8 = pow(w, 1 << 7, q)
    assert pow(w8, 8, q) == 1
    assert w8 == 20201


def _xor_params():
    # groth16/tests/mod.rs:302-319 toxic waste
    return bm.generate_parameters(D, cc.XorDemo(None, None), alpha=48577, beta=22580, gamma=53332,
                                  delta=5481, tau=3673)


def test_dummy_xordemo_qap_kat():
    # groth16/tests/mod.rs:330-470: h query, u_i / v_i / w_i at tau, IC and L queries
    q = D.Fr.q
    alpha, beta, gamma, delta, tau = 48577, 22580, 53332, 5481, 3673
    p = _xor_params()
    assert len(p.h) == 7
    t_at_tau = (pow(tau, 8, q) - 1) % q
    coeff = pow(delta, -1, q) * t_at_tau % q
    assert p.h == [pow(tau, i, q) * coeff % q for i in range(7)]
    u = [59158, 48317, 21767, 10402]
    v = [0, 0, 60619, 30791]
    w = [0, 23320, 41193, 41193]
    assert p.a == u
    assert p.b_g1 == [x for x in v if x] and p.b_g2 == [x for x in v if x]
    gi, di = pow(gamma, -1, q), pow(delta, -1, q)
    for i in range(4):
        t = (beta * u[i] + alpha * v[i] + w[i]) % q
        if i < 2:
            assert p.vk["ic"][i] == t * gi % q
        else:
            assert p.l[i - 2] == t * di % q
    assert (p.vk["alpha_g1"], p.vk["beta_g1"], p.vk["beta_g2"]) == (alpha, beta, beta)
    assert (p.vk["gamma_g2"], p.vk["delta_g1"], p.vk["delta_g2"]) == (gamma, delta, delta)


def test_dummy_xordemo_h_query_kat():
    # groth16/tests/mod.rs:574 H-query scalars for witness (a=true, b=false) (upstream witness)
    pr = bm.synthesize_for_proving(D, cc.XorDemo(True, False))
    assert bm.compute_h(D, pr.a, pr.b, pr.c) == [5040, 11763, 10755, 63633, 128, 9747, 8739]


def test_dummy_xordemo_proof_kat():
    # groth16/tests/mod.rs:490-585: proof A/B/C formulas with r=27134, s=17146, then verify
    q = D.Fr.q
    p = _xor_params()
    alpha, beta, delta = 48577, 22580, 5481
    r, s = 27134, 17146
    pr = bm.synthesize_for_proving(D, cc.XorDemo(True, False))
    proof = bm.prove_from_assignment(D, pr, p, r, s)
    u = [59158, 48317, 21767, 10402]
    v = [0, 0, 60619, 30791]
    # witness a_0=1 (one), a_1=c=1, a_2=a=1, a_3=b=0
    assert proof.a == (delta * r + alpha + u[0] + u[1] + u[2]) % q
    assert proof.b == (delta * s + beta + v[0] + v[1] + v[2]) % q
    h = [5040, 11763, 10755, 63633, 128, 9747, 8739]
    expected_c = (proof.a * s + proof.b * r - delta * r * s + p.l[0]
                  + sum(hh * hq for hh, hq in zip(h, p.h))) % q
    assert proof.c == expected_c
    assert bm.verify_dummy(D, p, proof, [1])
    # the fork's witness (false, false) also verifies
    pr2 = bm.synthesize_for_proving(D, cc.XorDemo(False, False))
    assert bm.verify_dummy(D, p, bm.prove_from_assignment(D, pr2, p, r, s), [0])


@pytest.mark.parametrize("circuit,inputs", [(cc.AndDemo(True, False), [0]), (cc.AndDemo(True, True), [1])])
def test_dummy_anddemo_verifies(circuit, inputs):
    # groth16/tests/mod.rs:262-295
    p = bm.generate_parameters(D, cc.AndDemo(None, None), 48577, 22580, 53332, 5481, 3673)
    pr = bm.synthesize_for_proving(D, circuit)
    assert bm.verify_dummy(D, p, bm.prove_from_assignment(D, pr, p, 27134, 17146), inputs)


def test_dummy_mimc_chain_verifies():
    q = D.Fr.q
    p = bm.generate_parameters(D, cc.chain_circuit(q, 5, witness=False), 48577, 22580, 53332, 5481, 3673)
    circ = cc.chain_circuit(q, 5)
    pr = bm.synthesize_for_proving(D, circ)
    image = cc.mimc(circ.xl, circ.xr, circ.constants, q)
    assert len(pr.a) == 2 * 5 + 2
    assert bm.verify_dummy(D, p, bm.prove_from_assignment(D, pr, p, 27134, 17146), [image])


# ---------------------------------------------------------------- BLS12-381 constants (first principles)
def test_bls_constants():
    P, R = bls.P, bls.R
    assert P.bit_length() == 381 and R.bit_length() == 255
    assert bls.FP_INV == 0x89F3FFFCFFFCFFFD  # gt_bytes.rs:30
    # gt_bytes.rs:20-27 limbs
    limbs = [0xB9FEFFFFFFFFAAAB, 0x1EABFFFEB153FFFF, 0x6730D2A0F6B0F624, 0x64774B84F38512BF,
             0x4B1BA7B6434BACD7, 0x1A0111EA397FE69A]
    assert sum(l << (64 * i) for i, l in enumerate(limbs)) == P
    w = bls.FR_ROOT_OF_UNITY
    assert pow(w, 1 << 32, R) == 1 and pow(w, 1 << 31, R) != 1
    assert pow(7, (R - 1) // 2, R) == R - 1  # 7 is a non-residue
    assert w == 0x16A2A19EDFE81F20D09B681922C813B4B63683508C2280B93829971F439F0D2B


def test_bls_generators():
    G1, G2 = bls.G1, bls.G2
    assert G1.on_curve_affine(bls.G1_GEN) and G2.on_curve_affine(bls.G2_GEN)
    assert G1.is_identity(G1.mul(G1.generator(), bls.R))
    assert G2.is_identity(G2.mul(G2.generator(), bls.R))
    # published zcash serialization of the G1 generator
    assert bls.g1_to_compressed(bls.G1_GEN).hex().startswith("97f1d3a73197d794")


def test_encoding_roundtrip():
    G1, G2 = bls.G1, bls.G2
    p = G1.to_affine(G1.mul(G1.generator(), 12345))
    ok, q = bls.g1_from_uncompressed(bls.g1_to_uncompressed(p))
    assert ok and q == p
    p2 = G2.to_affine(G2.mul(G2.generator(), 777))
    ok, q2 = bls.g2_from_uncompressed(bls.g2_to_uncompressed(p2))
    assert ok and q2 == p2
    assert bls.g1_from_uncompressed(bls.g1_to_uncompressed(None)) == (True, None)


# ---------------------------------------------------------------- self-consistency (domain.rs:374-498)
@pytest.mark.parametrize("eng", [D, BLS], ids=["dummy", "bls"])
def test_fft_composition(eng):
    rng = random.Random(1)
    q = eng.Fr.q
    for logd in range(0, 8):
        v = [rng.randrange(q) for _ in range(1 << logd)]
        for fwd, inv in (("fft", "ifft"), ("ifft", "fft"), ("coset_fft", "icoset_fft"), ("icoset_fft", "coset_fft")):
            d = bm.EvaluationDomain(eng, v)
            getattr(d, fwd)()
            getattr(d, inv)()
            assert d.coeffs == v


@pytest.mark.parametrize("eng", [D, BLS], ids=["dummy", "bls"])
def test_parallel_fft_consistency(eng):
    rng = random.Random(2)
    q = eng.Fr.q
    for log_d in range(0, 8):
        for log_cpus in range(log_d, min(log_d + 1, 3)):
            v = [rng.randrange(q) for _ in range(1 << log_d)]
            a, b = list(v), list(v)
            w = pow(eng.Fr.root_of_unity, 1 << (eng.Fr.S - log_d), q)
            bm.serial_fft(eng.Fr, a, w, log_d)
            bm.parallel_fft(eng.Fr, b, w, log_d, log_cpus)
            assert a == b


def test_polynomial_arith():
    # domain.rs:374-425 with BLS Fr, smaller ranges
    rng = random.Random(3)
    q = bls.R
    for la in range(0, 12, 3):
        for lb in range(0, 12, 4):
            a = [rng.randrange(q) for _ in range(la)]
            b = [rng.randrange(q) for _ in range(lb)]
            naive = [0] * (la + lb)
            for i, x in enumerate(a):
                for j, y in enumerate(b):
                    naive[i + j] = (naive[i + j] + x * y) % q
            da = bm.EvaluationDomain(BLS, a + [0] * lb)
            db = bm.EvaluationDomain(BLS, b + [0] * la)
            da.fft(); db.fft(); da.mul_assign(db); da.ifft()
            assert da.coeffs[: la + lb] == naive


def test_multiexp_matches_naive_and_errors():
    rng = random.Random(4)
    G = BLS.G1
    pts = [G.to_affine(G.mul(G.from_affine(bls.G1_GEN), rng.randrange(1, bls.R))) for _ in range(40)]
    ex = [rng.randrange(bls.R) for _ in range(40)]
    ex[3], ex[7] = 0, 1
    assert G.eq(bm.multiexp(BLS, G, pts, 0, None, ex), bm.multiexp_naive(G, pts, 0, None, ex))
    dens = [rng.random() < 0.5 for _ in range(40)]
    assert G.eq(bm.multiexp(BLS, G, pts, 2, dens, ex), bm.multiexp_naive(G, pts, 2, dens, ex))
    with pytest.raises(bm.UnexpectedEof):
        bm.multiexp(BLS, G, pts[:10], 0, None, ex)
    with pytest.raises(bm.DensitySizeMismatch):
        bm.multiexp(BLS, G, pts, 0, dens[:5], ex)
    bad = list(pts)
    bad[0] = None
    with pytest.raises(bm.UnexpectedIdentity):
        bm.multiexp(BLS, G, bad, 0, None, ex)
    ex0 = list(ex)
    ex0[0] = 0  # an identity base paired with a zero scalar is skipped, never an error
    # ... so the result is the naive sum over the remaining pairs
    assert G.eq(bm.multiexp(BLS, G, bad, 0, None, ex0), bm.multiexp_naive(G, bad[1:], 0, None, ex0[1:]))


def test_domain_degree_too_large():
    with pytest.raises(bm.PolynomialDegreeTooLarge):
        bm.EvaluationDomain(D, [0] * ((1 << 10) + 1))  # DummyEngine S = 10


def test_chain_circuit_shape():
    # R rounds -> 2R+2 constraints, 2 inputs, 2R+1 aux, densities
    q = bls.R
    for R in (3, 7):
        pr = bm.synthesize_for_proving(BLS, cc.chain_circuit(q, R))
        assert len(pr.a) == 2 * R + 2
        assert len(pr.input_assignment) == 2 and len(pr.aux_assignment) == 2 * R + 1
        assert pr.a_aux_density.get_total_density() == 2 * R
        assert pr.b_aux_density.get_total_density() == R
        assert pr.b_input_density.get_total_density() == 1
        for x, y, z in zip(pr.a, pr.b, pr.c):
            assert x * y % q == z


def test_subgroup_fixture_is_on_curve_but_not_torsion_free():
    """tests/golden/subgroup.json: the oracle's checked decoders reject it, unchecked accept."""
    import json
    import os
    from oracle import bls12_381 as bls
    fx = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "subgroup.json")))
    for key, dec, C in (("g1_off_subgroup", bls.g1_from_uncompressed, bls.G1),
                        ("g2_off_subgroup", bls.g2_from_uncompressed, bls.G2)):
        raw = bytes.fromhex(fx[key])
        ok, pt = dec(raw, checked=False)
        assert ok and C.on_curve_affine(pt)
        assert not dec(raw, checked=True)[0]
