"""The oracle's pairing and Groth16 verifier (oracle/pairing.py, restating verifier.rs:11-62):
pinned by bilinearity / non-degeneracy / order r, then used to show that every committed
golden proof is a VALID Groth16 proof for its verifying key and public input -- an
acceptance check that does not depend on how the proof was computed -- and that tampered
proofs and inputs are rejected."""
import json
import os

import pytest

from oracle import bls12_381 as bls
from oracle import pairing as pr

G1, G2 = bls.G1, bls.G2


@pytest.fixture(scope="module")
def gens():
    return G1.to_affine(G1.generator()), G2.to_affine(G2.generator())


def test_pairing_bilinear_nondegenerate_order_r(gens):
    p, q = gens
    e = pr.pairing(p, q)
    assert not pr.f12_is_one(e)
    assert pr.f12_is_one(pr.f12_pow(e, bls.R))
    a, b = 5, 11
    pa = G1.to_affine(G1.mul(G1.generator(), a))
    qb = G2.to_affine(G2.mul(G2.generator(), b))
    assert pr.pairing(pa, qb) == pr.f12_pow(e, a * b)
    # e(P, Q) e(-P, Q) == 1 through the multi-Miller loop + one final exponentiation
    assert pr.pairing_product_is_one([(p, q), ((p[0], (-p[1]) % bls.P), q)])


def test_compressed_decoding_roundtrip(gens):
    p, q = gens
    for k in (1, 2, 12345):
        pk = G1.to_affine(G1.mul(G1.generator(), k))
        qk = G2.to_affine(G2.mul(G2.generator(), k))
        assert pr.g1_from_compressed(bls.g1_to_compressed(pk)) == pk
        assert pr.g2_from_compressed(bls.g2_to_compressed(qk)) == qk


def _golden():
    with open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")) as f:
        return json.load(f)["proofs"]


@pytest.mark.parametrize("fx", _golden(), ids=lambda f: f["name"])
def test_golden_proofs_verify(fx):
    vk = pr.vk_from_params_bytes(bytes.fromhex(fx["params"]))
    proof = pr.proof_from_bytes(bytes.fromhex(fx["proof"]))
    public = [int(x, 16) for x in fx["inputs"]][1:]  # input 0 is ONE (prover.rs:202-204)
    assert pr.verify_proof(vk, proof, public)
    # wrong public input, and A/C exchanged, are rejected
    assert not pr.verify_proof(vk, proof, [(public[0] + 1) % bls.R] + public[1:])
    a, b, c = proof
    assert not pr.verify_proof(vk, (c, b, a), public)
    with pytest.raises(ValueError):
        pr.verify_proof(vk, proof, public + [1])
