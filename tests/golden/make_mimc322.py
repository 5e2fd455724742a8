"""C1 fixture (BASELINE.json configs[0]): the reference's MiMCDemo with MIMC_ROUNDS = 322
(mimc_mod.rs:6, 646 constraints incl. the 2 input constraints, domain m = 1024), its
constants and preimage from the seeded stream the native synthesizer uses (splitmix64, seed
7 / 8: oracle/circuits.py:chain_circuit), Parameters by the oracle's classic generator
(toxic waste alpha=6, beta=24, gamma=6, delta=24, tau=2 as bh_chain_params) and the proof
with the fork's fixed r, s (prover.rs:158-173).  Writes mimc322.json (proof, image, params
SHA-256) and mimc322_params.bin (Parameters::write bytes).  Oracle output, generated here
(the Rust reference cannot be built).

    python tests/golden/make_mimc322.py      (a few minutes: pure-Python group arithmetic)
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))

from oracle import bls12_381 as bls  # noqa: E402
from oracle import bellman as bm  # noqa: E402
from oracle import circuits as cc  # noqa: E402

ROUNDS = 322


def main():
    E = bm.BLS12_381
    R = bls.R
    params = bm.generate_random_parameters(E, cc.chain_circuit(R, ROUNDS, witness=False))
    pbytes = bm.params_to_bytes(params)
    print("params", len(pbytes), "bytes", file=sys.stderr)
    prover = bm.synthesize_for_proving(E, cc.chain_circuit(R, ROUNDS))
    proof = bm.prove_from_assignment(E, prover, params, 27134, 17146)
    xl, xr = cc.fr_stream(8, 2, R)
    image = cc.mimc(xl, xr, cc.fr_stream(7, ROUNDS, R), R)
    with open(os.path.join(HERE, "mimc322_params.bin"), "wb") as f:
        f.write(pbytes)
    out = {"rounds": ROUNDS, "constraints": len(prover.a), "image": format(image, "x"),
           "params_sha256": hashlib.sha256(pbytes).hexdigest(), "r": 27134, "s": 17146,
           "proof": bm.proof_to_bytes(proof).hex()}
    with open(os.path.join(HERE, "mimc322.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
