"""The CPU port of bellman's multicore prover (oracle/cpu, the bench baseline and the
at-size checker of the GPU tests) reproduces the oracle's golden proofs and multiexps byte
for byte.  CPU only."""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import cpu_port

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("name,rounds", [("mimc_chain_r7", 7), ("mimc_chain_r15", 15)])
def test_port_matches_golden(golden, name, rounds):
    fx = [f for f in golden["proofs"] if f["name"] == name][0]
    for threads in (1, 4):
        proof, ms, _ = cpu_port.chain_prove(bytes.fromhex(fx["params"]), rounds, threads=threads)
        assert proof.hex() == fx["proof"]


@pytest.mark.parametrize("group", [1, 2])
def test_port_multiexp_matches_golden(golden, group):
    """bp_multiexp (G1 and G2, base offsets, density maps, EOF) == the golden cases."""
    data = golden["msm_g1" if group == 1 else "msm_g2"]
    bases = b"".join(bytes.fromhex(h) for h in data["bases"])
    for case in data["cases"]:
        exps = np.array([[(int(x, 16) >> (64 * k)) & (2**64 - 1) for k in range(4)] for x in case["exps"]],
                        dtype=np.uint64).reshape(-1, 4)
        dens = None
        if case["density"] is not None:
            bits = [c == "1" for c in case["density"]]
            dens = np.zeros(max(1, (len(bits) + 63) // 64), dtype=np.uint64)
            for i, b in enumerate(bits):
                if b:
                    dens[i >> 6] |= np.uint64(1) << np.uint64(i & 63)
        if exps.shape[0] == 0:
            continue
        if "error" in case:
            with pytest.raises(RuntimeError):
                cpu_port.multiexp(group, bases, exps, case["offset"], dens, threads=4)
        else:
            got, _ = cpu_port.multiexp(group, bases, exps, case["offset"], dens, threads=4)
            assert got.hex() == case["point"], case["note"]


def test_port_c1_mimc322_matches_fixture():
    """C1 (BASELINE.json configs[0]): MiMCDemo with MIMC_ROUNDS = 322 (mimc_mod.rs:6) on the
    CPU path -- the port's proof from the oracle's Parameters equals the oracle's proof."""
    with open(os.path.join(HERE, "golden", "mimc322.json")) as f:
        fx = json.load(f)
    with open(os.path.join(HERE, "golden", "mimc322_params.bin"), "rb") as f:
        params = f.read()
    assert hashlib.sha256(params).hexdigest() == fx["params_sha256"]
    proof, _, _ = cpu_port.chain_prove(params, fx["rounds"], threads=4)
    assert proof.hex() == fx["proof"]
    assert fx["constraints"] == 646
