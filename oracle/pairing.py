"""ORACLE (test infrastructure only) -- BLS12-381 optimal-ate pairing and the Groth16
verifier, used to check that proofs are VALID, independently of how they were computed.

Only tests/ may import this module, and only as the CHECKER.

Restates `verifier.rs:11-62` (prepare_verifying_key / verify_proof) over the pairing of the
external crate `bls12_381` 0.6.0 (pinned in /root/reference/bellman/Cargo.lock, not vendored).
The pairing is restated from its published definition, not from that crate's code:

  * tower: Fp12 = Fp2[w]/(w^6 - xi), xi = u + 1  (Fp6 = Fp2[v]/(v^3 - xi), v = w^2);
  * G2 lives on the M-type sextic twist y^2 = x^3 + 4*xi, untwisted by
    (x', y') -> (x'/w^2, y'/w^3);
  * Miller loop over |x|, x = -0xd201000000010000 (the BLS12-381 seed), lines evaluated at
    P and scaled by w^3 (an Fp4 element, killed by the final exponentiation), vertical lines
    dropped (Fp6 elements, likewise);
  * final exponentiation f^((p^12 - 1) / r) computed directly.

The sign of x only inverts every pairing value, so equality tests of the form
prod_i e(P_i, Q_i) == 1 -- which is how verify_proof uses the pairing -- are unaffected.
The implementation is pinned by its own bilinearity / non-degeneracy / order-r tests
(tests/test_pairing.py), and the verifier by the reference's DummyEngine proofs being
accepted and tampered proofs rejected.
"""
from . import bls12_381 as bls

P = bls.P
R = bls.R
F2 = bls.Fp2Ops
X_ABS = 0xD201000000010000
XI = (1, 1)

_FINAL_EXP = (P ** 12 - 1) // R


# ---------------------------------------------------------------- Fp12 = Fp2[w]/(w^6 - xi)
def f12_one():
    return [(1, 0)] + [(0, 0)] * 5


def f12_mul(a, b):
    t = [(0, 0)] * 11
    for i in range(6):
        ai = a[i]
        if ai == (0, 0):
            continue
        for j in range(6):
            bj = b[j]
            if bj == (0, 0):
                continue
            t[i + j] = F2.add(t[i + j], F2.mul(ai, bj))
    # w^6 = xi
    return [F2.add(t[k], F2.mul(XI, t[k + 6])) if k + 6 < 11 else t[k] for k in range(6)]


def f12_sqr(a):
    return f12_mul(a, a)


def f12_pow(a, e):
    r = f12_one()
    for bit in bin(e)[2:]:
        r = f12_sqr(r)
        if bit == "1":
            r = f12_mul(r, a)
    return r


def f12_is_one(a):
    return a == f12_one()


# ---------------------------------------------------------------- Miller loop
def _line(lam, xt, yt, p):
    """line through T with slope lam (twist coordinates), evaluated at P = (xp, yp) and
    scaled by w^3:  (lam*xt - yt) - lam*xp * w^2 + yp * w^3."""
    xp, yp = p
    c0 = F2.sub(F2.mul(lam, xt), yt)
    c2 = F2.neg(F2.mul(lam, (xp, 0)))
    return [c0, (0, 0), c2, (yp, 0), (0, 0), (0, 0)]


def multi_miller_loop(pairs):
    """prod_i f_{|x|, Q_i}(P_i) for affine P_i in G1 (None = identity) and affine Q_i on the twist."""
    terms = [(p, q) for p, q in pairs if p is not None and q is not None]
    f = f12_one()
    ts = [q for _, q in terms]
    for bit in bin(X_ABS)[3:]:
        f = f12_sqr(f)
        for i, (p, q) in enumerate(terms):
            xt, yt = ts[i]
            lam = F2.mul(F2.mul((3, 0), F2.sqr(xt)), F2.inv(F2.add(yt, yt)))
            f = f12_mul(f, _line(lam, xt, yt, p))
            x3 = F2.sub(F2.sqr(lam), F2.add(xt, xt))
            ts[i] = (x3, F2.sub(F2.mul(lam, F2.sub(xt, x3)), yt))
        if bit == "1":
            for i, (p, q) in enumerate(terms):
                xt, yt = ts[i]
                xq, yq = q
                lam = F2.mul(F2.sub(yq, yt), F2.inv(F2.sub(xq, xt)))
                f = f12_mul(f, _line(lam, xt, yt, p))
                x3 = F2.sub(F2.sub(F2.sqr(lam), xt), xq)
                ts[i] = (x3, F2.sub(F2.mul(lam, F2.sub(xt, x3)), yt))
    return f


def final_exponentiation(f):
    return f12_pow(f, _FINAL_EXP)


def pairing(p, q):
    """e(P, Q) up to the sign convention of the seed (see module header)."""
    return final_exponentiation(multi_miller_loop([(p, q)]))


def pairing_product_is_one(pairs):
    return f12_is_one(final_exponentiation(multi_miller_loop(pairs)))


# ---------------------------------------------------------------- point decompression
def _fp_sqrt(a):
    y = pow(a, (P + 1) // 4, P)  # p = 3 mod 4
    return y if y * y % P == a % P else None


def _fp2_sqrt(a):
    # p = 3 mod 4 algorithm for Fp2 = Fp[u]/(u^2+1)
    if a == (0, 0):
        return (0, 0)
    a1 = F2.mul(_fp2_pow(a, (P - 3) // 4), (1, 0))
    alpha = F2.mul(F2.sqr(a1), a)
    x0 = F2.mul(a1, a)
    if alpha == (P - 1, 0):
        x = F2.mul((0, 1), x0)
    else:
        b = _fp2_pow(F2.add((1, 0), alpha), (P - 1) // 2)
        x = F2.mul(b, x0)
    return x if F2.sqr(x) == a else None


def _fp2_pow(a, e):
    r = (1, 0)
    for bit in bin(e)[2:]:
        r = F2.sqr(r)
        if bit == "1":
            r = F2.mul(r, a)
    return r


def g1_from_compressed(b):
    assert len(b) == 48 and b[0] & 0x80, "not a compressed G1 encoding"
    if b[0] & 0x40:
        return None
    x = int.from_bytes(bytes([b[0] & 0x1F]) + b[1:], "big")
    y = _fp_sqrt((x * x * x + 4) % P)
    assert y is not None, "G1 point not on curve"
    if bls.fp_lex_largest(y) != bool(b[0] & 0x20):
        y = (P - y) % P
    return (x, y)


def g2_from_compressed(b):
    assert len(b) == 96 and b[0] & 0x80, "not a compressed G2 encoding"
    if b[0] & 0x40:
        return None
    c1 = int.from_bytes(bytes([b[0] & 0x1F]) + b[1:48], "big")
    c0 = int.from_bytes(b[48:96], "big")
    x = (c0, c1)
    y = _fp2_sqrt(F2.add(F2.mul(F2.sqr(x), x), (4, 4)))
    assert y is not None, "G2 point not on curve"
    if bls.fp2_lex_largest(y) != bool(b[0] & 0x20):
        y = F2.neg(y)
    return (x, y)


def proof_from_bytes(b):
    """Proof::read (groth16/mod.rs:50-103): compressed A (48) || B (96) || C (48)."""
    assert len(b) == 192
    return g1_from_compressed(b[:48]), g2_from_compressed(b[48:144]), g1_from_compressed(b[144:])


def vk_from_params_bytes(b):
    """VerifyingKey::read (groth16/mod.rs:145-205) at the head of Parameters::write bytes."""
    o = 0

    def g1():
        nonlocal o
        ok, pt = bls.g1_from_uncompressed(b[o:o + 96], checked=True)
        assert ok, "invalid G1 point in the verifying key"
        o += 96
        return pt

    def g2():
        nonlocal o
        ok, pt = bls.g2_from_uncompressed(b[o:o + 192], checked=True)
        assert ok, "invalid G2 point in the verifying key"
        o += 192
        return pt

    vk = {"alpha_g1": g1(), "beta_g1": g1(), "beta_g2": g2(), "gamma_g2": g2(), "delta_g1": g1(),
          "delta_g2": g2()}
    n = int.from_bytes(b[o:o + 4], "big")
    o += 4
    vk["ic"] = [g1() for _ in range(n)]
    return vk


# ---------------------------------------------------------------- verifier.rs
def _neg2(q):
    return None if q is None else (q[0], F2.neg(q[1]))


def verify_proof(vk, proof, public_inputs):
    """verify_proof (verifier.rs:23-62): e(A,B) == e(alpha,beta) e(acc,gamma) e(C,delta),
    acc = ic[0] + sum_i public_inputs[i] * ic[i+1]; checked as a single product == 1."""
    if len(public_inputs) + 1 != len(vk["ic"]):
        raise ValueError("InvalidVerifyingKey")
    G1 = bls.G1
    acc = G1.from_affine(vk["ic"][0])
    for x, b in zip(public_inputs, vk["ic"][1:]):
        acc = G1.add(acc, G1.mul(G1.from_affine(b), x % R))
    a, b, c = proof
    neg_alpha = None if vk["alpha_g1"] is None else (vk["alpha_g1"][0], (-vk["alpha_g1"][1]) % P)
    return pairing_product_is_one([
        (a, b),
        (G1.to_affine(acc), _neg2(vk["gamma_g2"])),
        (c, _neg2(vk["delta_g2"])),
        (neg_alpha, vk["beta_g2"]),
    ])
