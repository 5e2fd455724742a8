"""The fused, multithreaded MiMC-chain synthesizer (chain.hip: chain_fused) against the generic
ProvingAssignment mirror (BH_CHAIN_GENERIC=1) -- every assignment, row and density word
byte-identical -- and against the oracle's ProvingAssignment at a small size.  CPU only: the
chain assignment never touches the device."""
import json
import os
import subprocess
import sys


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import sys, json, hashlib
sys.path.insert(0, %r)
import bellman_hip as bh
out = {}
for rounds in (1, 2, 7, 63, 64, 65, 1000, 70000):
    asg = bh.chain_assignment(rounds, seed=7, preimage_seed=9)
    out[rounds] = {k: hashlib.sha256(v.tobytes()).hexdigest() for k, v in asg.items()}
print(json.dumps(out))
"""


def _run(generic):
    env = dict(os.environ)
    if generic:
        env["BH_CHAIN_GENERIC"] = "1"
    else:
        env.pop("BH_CHAIN_GENERIC", None)
    r = subprocess.run([sys.executable, "-c", SCRIPT % os.path.join(ROOT, "bellman-mpc_amd")], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_fused_chain_synthesis_equals_generic_mirror():
    fused, generic = _run(False), _run(True)
    assert fused == generic


def test_fused_chain_synthesis_matches_oracle_small():
    sys.path.insert(0, os.path.join(ROOT, "bellman-mpc_amd"))
    import bellman_hip as bh
    from oracle import bellman as ob, circuits as cc
    rounds = 7
    asg = bh.chain_assignment(rounds, seed=7, preimage_seed=8)
    q = ob.BLS12_381.Fr.q
    pa = ob.synthesize_for_proving(ob.BLS12_381, cc.chain_circuit(q, rounds, seed=7, preimage_seed=8))
    assert bh.fr_from_mont(asg["aux"]) == list(pa.aux_assignment)
    assert bh.fr_from_mont(asg["inputs"]) == list(pa.input_assignment)
    assert bh.fr_from_mont(asg["a"]) == list(pa.a)
    assert bh.fr_from_mont(asg["b"]) == list(pa.b)
    assert bh.fr_from_mont(asg["c"]) == list(pa.c)
