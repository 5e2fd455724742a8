"""Fixture: points ON the BLS12-381 curves but OUTSIDE the prime-order subgroups, which
Parameters::read(checked = true) must reject (G1Affine/G2Affine::from_uncompressed check
torsion-freeness; groth16/mod.rs:292-400 maps that to an InvalidData error).  Found by
scanning x = 1, 2, ... for x^3 + b square and keeping the first point with [r]P != O
(the oracle's checked decoder confirms each).

    python tests/golden/make_subgroup.py   (seconds)
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))

from oracle import bls12_381 as bls  # noqa: E402

P = bls.P


def fp_sqrt(a):
    y = pow(a, (P + 1) // 4, P)  # p = 3 mod 4
    return y if y * y % P == a % P else None


def fp2_sqrt(a):
    a0, a1 = a
    if a1 == 0:
        r = fp_sqrt(a0)
        if r is not None:
            return (r, 0)
        r = fp_sqrt((-a0) % P)
        return (0, r) if r is not None else None
    alpha = fp_sqrt((a0 * a0 + a1 * a1) % P)  # norm
    if alpha is None:
        return None
    inv2 = pow(2, P - 2, P)
    for s in (alpha, (-alpha) % P):
        x0 = fp_sqrt((a0 + s) * inv2 % P)
        if x0 is not None and x0 != 0:
            x1 = a1 * pow(2 * x0, P - 2, P) % P
            if bls.Fp2Ops.sqr((x0, x1)) == (a0 % P, a1 % P):
                return (x0, x1)
    return None


def first_g1():
    x = 1
    while True:
        y = fp_sqrt((x ** 3 + 4) % P)
        if y is not None:
            pt = (x, y)
            assert bls.G1.on_curve_affine(pt)
            if not bls.G1.is_identity(bls.G1.mul(bls.G1.from_affine(pt), bls.R)):
                return pt
        x += 1


def first_g2():
    x0 = 1
    b = (4, 4)
    while True:
        x = (x0, 1)
        rhs = bls.Fp2Ops.add(bls.Fp2Ops.mul(bls.Fp2Ops.sqr(x), x), b)
        y = fp2_sqrt(rhs)
        if y is not None:
            pt = (x, y)
            assert bls.G2.on_curve_affine(pt)
            if not bls.G2.is_identity(bls.G2.mul(bls.G2.from_affine(pt), bls.R)):
                return pt
        x0 += 1


def main():
    g1 = bls.g1_to_uncompressed(first_g1())
    g2 = bls.g2_to_uncompressed(first_g2())
    for enc, dec in ((g1, bls.g1_from_uncompressed), (g2, bls.g2_from_uncompressed)):
        assert dec(enc, checked=False)[0] and not dec(enc, checked=True)[0]
    out = {"g1_off_subgroup": g1.hex(), "g2_off_subgroup": g2.hex()}
    with open(os.path.join(HERE, "subgroup.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(out)


if __name__ == "__main__":
    main()
