"""The CPU port of bellman's multicore prover (bench baseline) reproduces the
oracle's golden proofs byte for byte.  CPU only."""
import pytest

from oracle import cpu_port


@pytest.mark.parametrize("name,rounds", [("mimc_chain_r7", 7), ("mimc_chain_r15", 15)])
def test_port_matches_golden(golden, name, rounds):
    fx = [f for f in golden["proofs"] if f["name"] == name][0]
    for threads in (1, 4):
        proof, ms, _ = cpu_port.chain_prove(bytes.fromhex(fx["params"]), rounds, threads=threads)
        assert proof.hex() == fx["proof"]
