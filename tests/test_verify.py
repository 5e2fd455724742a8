"""Native verifier (csrc/verify.cpp: bh_verify_proof, bh_verify_batch) on the committed golden
proofs (BLS12-381, tests/golden/golden.json): valid proofs accepted, tampered proofs and wrong
inputs rejected, the same verdicts as the oracle's pairing (oracle/pairing.py), the reference's
InvalidVerifyingKey on an input-count mismatch, and Proof::read's rejections.  Host code only:
runs on the CPU."""
import json
import os
import random
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bellman-mpc_amd"))


def _golden():
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        return json.load(f)["proofs"]


@pytest.fixture(scope="module")
def bh():
    import bellman_hip
    return bellman_hip


def _case(fx):
    params = bytes.fromhex(fx["params"])
    proof = bytes.fromhex(fx["proof"])
    public = [int(x, 16) for x in fx["inputs"]][1:]  # input 0 is ONE (prover.rs:202-204)
    return params, proof, public


@pytest.mark.parametrize("fx", _golden(), ids=lambda f: f["name"])
def test_native_verify_matches_oracle(bh, fx):
    from oracle import bls12_381 as bls, pairing as pr
    params, proof, public = _case(fx)
    assert bh.verify_proof(params, proof, public)
    wrong = [(public[0] + 1) % bls.R] + public[1:]
    assert not bh.verify_proof(params, proof, wrong)
    # A and C exchanged: well-formed but invalid (the oracle agrees)
    swapped = proof[144:] + proof[48:144] + proof[:48]
    assert not bh.verify_proof(params, swapped, public)
    vk = pr.vk_from_params_bytes(params)
    assert not pr.verify_proof(vk, pr.proof_from_bytes(swapped), public)
    with pytest.raises(bh.SynthesisError):
        bh.verify_proof(params, proof, public + [1])  # VerificationError::InvalidVerifyingKey


def test_native_verify_rejects_bad_encodings(bh):
    params, proof, public = _case(_golden()[0])
    bad = bytearray(proof)
    bad[0] &= 0x7F  # compression flag cleared: not a compressed encoding
    with pytest.raises(bh.SynthesisError):
        bh.verify_proof(params, bytes(bad), public)
    inf = bytearray(proof)
    inf[0:48] = bytes([0xC0]) + bytes(47)  # A = identity: "point at infinity"
    with pytest.raises(bh.SynthesisError):
        bh.verify_proof(params, bytes(inf), public)


def test_native_batch_verify(bh):
    from oracle import bls12_381 as bls
    rng = random.Random(11)
    by_vk = {}
    for fx in _golden():
        params, proof, public = _case(fx)
        by_vk.setdefault(params, []).append((proof, public))
    checked = 0
    for params, items in by_vk.items():
        proofs = [p for p, _ in items] * 3  # the same proof three times: a batch of equal statements
        inputs = [i for _, i in items] * 3
        zs = [rng.randrange(1, bls.R) for _ in proofs]
        assert bh.verify_batch(params, proofs, inputs, zs)
        swapped = [proofs[0][144:] + proofs[0][48:144] + proofs[0][:48]] + proofs[1:]
        assert not bh.verify_batch(params, swapped, inputs, zs)
        bad_inputs = [[(inputs[0][0] + 1) % bls.R] + inputs[0][1:]] + inputs[1:]
        assert not bh.verify_batch(params, proofs, bad_inputs, zs)
        with pytest.raises(bh.SynthesisError):
            bh.verify_batch(params, proofs, inputs, [0] + zs[1:])  # z must be nonzero
        checked += 1
    assert checked >= 1
