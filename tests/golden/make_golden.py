"""Generates the committed golden fixtures under tests/golden/ with the CPU
oracle (oracle/, a restatement of the reference: see its headers).  The
reference is Rust and cannot be built here, so these vectors are
oracle outputs; the oracle itself is pinned by the reference's own DummyEngine
known-answer constants (tests/test_oracle_kat.py).

    python tests/golden/make_golden.py      (about a minute)
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))

from oracle import bls12_381 as bls  # noqa: E402
from oracle import bellman as bm  # noqa: E402
from oracle import circuits as cc  # noqa: E402

E = bm.BLS12_381
G1, G2 = E.G1, E.G2
R = bls.R


def hx(b):
    return b.hex()


def rand_points(G, enc, n, rng):
    pts = [G.to_affine(G.mul(G.from_affine(G.c.gen_affine), rng.randrange(1, R))) for _ in range(n)]
    return pts


def msm_cases(G, enc, bases, rng, label):
    n_b = len(bases)
    cases = []

    def add(exps, offset=0, density=None, note=""):
        try:
            res = bm.multiexp(E, G, bases, offset, density, exps)
            expect = {"point": hx(enc(G.to_affine(res)))}
        except bm.SynthesisError as e:
            expect = {"error": e.code}
        cases.append({"note": note, "offset": offset,
                      "density": None if density is None else "".join("1" if d else "0" for d in density),
                      "exps": [format(x, "x") for x in exps], **expect})

    for n in (1, 2, 3, 31, 32, 33, 100):
        add([rng.randrange(R) for _ in range(n)], note=f"random n={n}")
    add([0, 1, R - 1, 2, 0, 1, 1, R - 1] * 4, note="edge scalars 0/1/r-1")
    add([0] * 20, note="all zero")
    add([1] * 40, note="all one")
    add([R - 1] * 40, note="all r-1")
    add([rng.randrange(1 << 16) for _ in range(64)], note="small scalars")
    add([rng.randrange(R) for _ in range(n_b)], note=f"random n={n_b} (all bases)")
    dens = [rng.random() < 0.6 for _ in range(90)]
    add([rng.randrange(R) for _ in range(90)], offset=3, density=dens, note="density + offset")
    add([rng.randrange(R) for _ in range(10)], offset=n_b - 5, note="EOF (offset too large)")
    add([rng.randrange(R) for _ in range(n_b + 1)], note="EOF (more exps than bases)")
    return cases


def main():
    rng = random.Random(20251015)
    out = {}
    # ---------------- G1 / G2 MSM
    g1_bases = rand_points(G1, bls.g1_to_uncompressed, 160, rng)
    # duplicate and negated bases exercise doubling / cancellation in buckets
    g1_bases[10] = g1_bases[11]
    x, y = g1_bases[12]
    g1_bases[13] = (x, bls.P - y)
    out["msm_g1"] = {"bases": [hx(bls.g1_to_uncompressed(p)) for p in g1_bases],
                     "cases": msm_cases(G1, bls.g1_to_uncompressed, g1_bases, rng, "g1")}
    g2_bases = rand_points(G2, bls.g2_to_uncompressed, 48, rng)
    g2_bases[5] = g2_bases[6]
    out["msm_g2"] = {"bases": [hx(bls.g2_to_uncompressed(p)) for p in g2_bases],
                     "cases": msm_cases(G2, bls.g2_to_uncompressed, g2_bases, rng, "g2")}
    # ---------------- EvaluationDomain ops (domain.rs)
    dom_cases = []
    for logm in (0, 1, 2, 3, 6, 9):
        m = 1 << logm
        coeffs = [rng.randrange(R) for _ in range(m)]
        other = [rng.randrange(R) for _ in range(m)]
        res = {}
        for op in ("fft", "ifft", "coset_fft", "icoset_fft", "divide_by_z_on_coset"):
            d = bm.EvaluationDomain(E, coeffs)
            getattr(d, op)()
            res[op] = [format(v, "x") for v in d.coeffs]
        d = bm.EvaluationDomain(E, coeffs)
        d.distribute_powers(12345)
        res["distribute_powers_12345"] = [format(v, "x") for v in d.coeffs]
        d = bm.EvaluationDomain(E, coeffs); d.mul_assign(bm.EvaluationDomain(E, other))
        res["mul_assign"] = [format(v, "x") for v in d.coeffs]
        d = bm.EvaluationDomain(E, coeffs); d.sub_assign(bm.EvaluationDomain(E, other))
        res["sub_assign"] = [format(v, "x") for v in d.coeffs]
        dom_cases.append({"log_m": logm, "coeffs": [format(v, "x") for v in coeffs],
                          "other": [format(v, "x") for v in other], "results": res})
    out["domain"] = dom_cases
    # ---------------- H block (prover.rs:210-231) on random a, b, c (ragged length 37 -> m = 64)
    a = [rng.randrange(R) for _ in range(37)]
    b = [rng.randrange(R) for _ in range(37)]
    c = [rng.randrange(R) for _ in range(37)]
    out["h_random"] = {"a": [format(v, "x") for v in a], "b": [format(v, "x") for v in b],
                       "c": [format(v, "x") for v in c],
                       "h": [format(v, "x") for v in bm.compute_h(E, a, b, c)]}
    # ---------------- full proofs (create_proof with the fork's fixed r, s)
    proofs = []
    for name, circuit_nw, circuit_w in (
        ("xor_true_false", cc.XorDemo(None, None), cc.XorDemo(True, False)),
        ("and_true_true", cc.AndDemo(None, None), cc.AndDemo(True, True)),
        ("mimc_chain_r7", cc.chain_circuit(R, 7, witness=False), cc.chain_circuit(R, 7)),
        ("mimc_chain_r15", cc.chain_circuit(R, 15, witness=False), cc.chain_circuit(R, 15)),
    ):
        params = bm.generate_random_parameters(E, circuit_nw)
        prover = bm.synthesize_for_proving(E, circuit_w)
        proof = bm.prove_from_assignment(E, prover, params, 27134, 17146)
        proofs.append({
            "name": name,
            "params": hx(bm.params_to_bytes(params)),
            "a": [format(v, "x") for v in prover.a], "b": [format(v, "x") for v in prover.b],
            "c": [format(v, "x") for v in prover.c],
            "inputs": [format(v, "x") for v in prover.input_assignment],
            "aux": [format(v, "x") for v in prover.aux_assignment],
            "a_aux_density": "".join("1" if d else "0" for d in prover.a_aux_density.bv),
            "b_input_density": "".join("1" if d else "0" for d in prover.b_input_density.bv),
            "b_aux_density": "".join("1" if d else "0" for d in prover.b_aux_density.bv),
            "r": 27134, "s": 17146,
            "proof": hx(bm.proof_to_bytes(proof)),
        })
        print("proof", name, "done", file=sys.stderr)
    out["proofs"] = proofs
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=0)
    print("wrote", os.path.join(HERE, "golden.json"))


if __name__ == "__main__":
    main()
