"""The public-input multiexps (a_inputs, b_g1_inputs, b_g2_inputs: prover.rs:259-307 over the input
assignment) on the device.  Up to HOST_INPUT_MSM_MAX (64) terms they run on a host thread
(prover.hip); above it, and with BH_HOST_INPUTS=0 for any count, on the device like the others.
VERDICT r3: that device branch had no proof test.  Here a circuit with 70 public inputs, all of
them in B terms (so b_g1_inputs / b_g2_inputs have 71 terms with the input "one"), is proved on the
device and compared with the oracle's proof over the oracle's Parameters; and the golden proofs
(<= 3 inputs) are re-proved with the inputs forced onto the device."""
import os

import pytest

pytestmark = pytest.mark.gpu

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


class ManyInputs:
    """70 public inputs x_i, each constrained by (3 * one) * x_i = y_i with an aux y_i."""

    def __init__(self, vals):
        self.vals = vals

    def synthesize(self, cs):
        for i, v in enumerate(self.vals):
            x = cs.alloc_input(f"x{i}", lambda v=v: v)
            y = cs.alloc(f"y{i}", lambda v=v: None if v is None else 3 * v % R)
            cs.enforce(f"c{i}", lambda lc: lc + (3, cs.one()), lambda lc, x=x: lc + x, lambda lc, y=y: lc + y)


def test_seventy_public_inputs_device_branch_equals_oracle(ctx):
    import bellman_hip as bh
    from oracle import bellman as bm
    E = bm.BLS12_381
    vals = [(7919 * i * i + 13) % R for i in range(70)]
    params = bm.generate_parameters(E, ManyInputs([None] * 70), 6, 24, 6, 24, 2)
    raw = bm.params_to_bytes(params)
    want = bm.proof_to_bytes(bm.create_proof(E, ManyInputs(vals), params, 27134, 17146))
    dev = bh.Parameters.read(ctx, raw)
    assert bh.create_proof(ctx, ManyInputs(vals), dev, 27134, 17146) == want
    os.environ["BH_HOST_INPUTS"] = "1"  # (the count is above 64: device either way)
    try:
        assert bh.create_proof(ctx, ManyInputs(vals), dev, 27134, 17146) == want
    finally:
        os.environ.pop("BH_HOST_INPUTS", None)


def test_golden_proofs_with_inputs_on_the_device(ctx, golden):
    import bellman_hip as bh
    from test_gpu_parity import _proof_from_fixture
    os.environ["BH_HOST_INPUTS"] = "0"
    try:
        for fx in golden["proofs"]:
            params, w = _proof_from_fixture(ctx, fx)
            assert bh.prove_witness(ctx, params, w, fx["r"], fx["s"]).hex() == fx["proof"], fx["name"]
    finally:
        os.environ.pop("BH_HOST_INPUTS", None)
