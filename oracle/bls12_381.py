"""ORACLE (test infrastructure only) -- exact big-integer BLS12-381 arithmetic.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the CHECKER.  The product path (bellman-mpc_amd/) never
imports it.

This restates the arithmetic of the external crate `bls12_381` 0.6.0 (pinned in
/root/reference/bellman/Cargo.lock; not vendored) that the reference hot path
calls (multiexp.rs:39,217,231-232,248; domain.rs:250-257; prover.rs:315-349):

  * Fp   : p = 0x1a0111ea...aaab (matches gt_bytes.rs:20-27), Montgomery R = 2^384
  * Fr   : r = 0x73eda753...00000001, S = 32, multiplicative generator 7,
           root of unity 7^((r-1)/2^32), Montgomery R = 2^256
  * Fp2  : Fp[u]/(u^2+1)
  * G1   : y^2 = x^3 + 4 over Fp;  G2 : y^2 = x^3 + 4(u+1) over Fp2
  * encodings: zcash/bls12_381 compressed (48/96 B) and uncompressed (96/192 B)
    big-endian with the 3 flag bits (compression, infinity, sort) in byte 0,
    G2 writes c1 before c0 -- used by Proof::write (groth16/mod.rs:42-48) and
    Parameters::write (groth16/mod.rs:260-290).

Parity status: BLS12-381 constants are pinned by first-principles checks
(tests/test_oracle_bls.py: on-curve generators, r*G = O, root-of-unity order
exactly 2^32, p/INV vs gt_bytes.rs:20-30); the reference holds no BLS12-381
golden vector, so group-level results are pinned by exact math.

Points are represented in Jacobian coordinates (X, Y, Z) with Z == 0 meaning
the identity; any correct formula gives the same affine result as bls12_381's
homogeneous projective formulas, which is all that is ever compared.
"""

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001

FR_S = 32
FR_GENERATOR = 7
FR_NUM_BITS = 255
FR_ROOT_OF_UNITY = pow(FR_GENERATOR, (R - 1) >> FR_S, R)

FP_MONT_R = pow(2, 384, P)
FR_MONT_R = pow(2, 256, R)
FP_INV = (-pow(P, -1, 2 ** 64)) % 2 ** 64   # gt_bytes.rs:30

G1_B = 4
G1_GEN = (
    0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB,
    0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1,
)
G2_GEN = (
    (0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
     0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E),
    (0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
     0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE),
)


# ---------------------------------------------------------------- field ops
class FpOps:
    """Prime field Fp; elements are ints in [0, p)."""
    zero = 0
    one = 1

    @staticmethod
    def add(a, b):
        s = a + b
        return s - P if s >= P else s

    @staticmethod
    def sub(a, b):
        s = a - b
        return s + P if s < 0 else s

    @staticmethod
    def neg(a):
        return P - a if a else 0

    @staticmethod
    def mul(a, b):
        return a * b % P

    @staticmethod
    def sqr(a):
        return a * a % P

    @staticmethod
    def inv(a):
        return pow(a, P - 2, P)

    @staticmethod
    def is_zero(a):
        return a == 0

    @staticmethod
    def small(k):
        return k % P


class Fp2Ops:
    """Fp2 = Fp[u]/(u^2+1); elements are tuples (c0, c1)."""
    zero = (0, 0)
    one = (1, 0)

    @staticmethod
    def add(a, b):
        return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)

    @staticmethod
    def sub(a, b):
        return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)

    @staticmethod
    def neg(a):
        return ((-a[0]) % P, (-a[1]) % P)

    @staticmethod
    def mul(a, b):
        a0, a1 = a
        b0, b1 = b
        return ((a0 * b0 - a1 * b1) % P, (a0 * b1 + a1 * b0) % P)

    @staticmethod
    def sqr(a):
        a0, a1 = a
        return ((a0 + a1) * (a0 - a1) % P, 2 * a0 * a1 % P)

    @staticmethod
    def inv(a):
        a0, a1 = a
        t = pow((a0 * a0 + a1 * a1) % P, P - 2, P)
        return (a0 * t % P, (-a1) * t % P)

    @staticmethod
    def is_zero(a):
        return a[0] == 0 and a[1] == 0

    @staticmethod
    def small(k):
        return (k % P, 0)


# ---------------------------------------------------------------- curves
class Curve:
    """Short Weierstrass y^2 = x^3 + b (a = 0) in Jacobian coordinates."""

    def __init__(self, F, b, gen, name):
        self.F = F
        self.b = b
        self.gen_affine = gen
        self.name = name
        self.identity = (F.one, F.one, F.zero)

    # -- predicates / conversions
    def is_identity(self, p):
        return self.F.is_zero(p[2])

    def from_affine(self, a):
        if a is None:
            return self.identity
        return (a[0], a[1], self.F.one)

    def to_affine(self, p):
        """None for the identity, else (x, y)."""
        F = self.F
        if F.is_zero(p[2]):
            return None
        zi = F.inv(p[2])
        zi2 = F.sqr(zi)
        return (F.mul(p[0], zi2), F.mul(p[1], F.mul(zi2, zi)))

    def on_curve_affine(self, a):
        if a is None:
            return True
        F = self.F
        x, y = a
        return F.sqr(y) == F.add(F.mul(F.sqr(x), x), self.b)

    def eq(self, p, q):
        return self.to_affine(p) == self.to_affine(q)

    def generator(self):
        return self.from_affine(self.gen_affine)

    # -- group law
    def neg(self, p):
        return (p[0], self.F.neg(p[1]), p[2])

    def double(self, p):
        F = self.F
        X, Y, Z = p
        if F.is_zero(Z) or F.is_zero(Y):
            return self.identity
        A = F.sqr(X)
        B = F.sqr(Y)
        C = F.sqr(B)
        t = F.add(X, B)
        D = F.sub(F.sqr(t), F.add(A, C))
        D = F.add(D, D)
        E = F.add(F.add(A, A), A)
        Fv = F.sqr(E)
        X3 = F.sub(Fv, F.add(D, D))
        C8 = F.add(C, C)
        C8 = F.add(C8, C8)
        C8 = F.add(C8, C8)
        Y3 = F.sub(F.mul(E, F.sub(D, X3)), C8)
        Z3 = F.mul(Y, Z)
        Z3 = F.add(Z3, Z3)
        return (X3, Y3, Z3)

    def add(self, p, q):
        F = self.F
        if F.is_zero(p[2]):
            return q
        if F.is_zero(q[2]):
            return p
        X1, Y1, Z1 = p
        X2, Y2, Z2 = q
        Z1Z1 = F.sqr(Z1)
        Z2Z2 = F.sqr(Z2)
        U1 = F.mul(X1, Z2Z2)
        U2 = F.mul(X2, Z1Z1)
        S1 = F.mul(F.mul(Y1, Z2), Z2Z2)
        S2 = F.mul(F.mul(Y2, Z1), Z1Z1)
        if U1 == U2:
            if S1 == S2:
                return self.double(p)
            return self.identity
        H = F.sub(U2, U1)
        I = F.sqr(F.add(H, H))
        J = F.mul(H, I)
        r = F.sub(S2, S1)
        r = F.add(r, r)
        V = F.mul(U1, I)
        X3 = F.sub(F.sub(F.sqr(r), J), F.add(V, V))
        S1J = F.mul(S1, J)
        Y3 = F.sub(F.mul(r, F.sub(V, X3)), F.add(S1J, S1J))
        Z3 = F.mul(F.sub(F.sqr(F.add(Z1, Z2)), F.add(Z1Z1, Z2Z2)), H)
        return (X3, Y3, Z3)

    def add_affine(self, p, a):
        """p + a where a is an affine point (not None)."""
        return self.add(p, (a[0], a[1], self.F.one))

    def mul(self, p, k):
        """Scalar multiplication by a non-negative integer k (double-and-add)."""
        acc = self.identity
        for bit in bin(k)[2:] if k > 0 else "":
            acc = self.double(acc)
            if bit == "1":
                acc = self.add(acc, p)
        return acc

    def sum(self, pts):
        acc = self.identity
        for q in pts:
            acc = self.add(acc, q)
        return acc


G1 = Curve(FpOps, G1_B, G1_GEN, "G1")
G2 = Curve(Fp2Ops, (4, 4), G2_GEN, "G2")


# ---------------------------------------------------------------- encodings
def _fp_be(x):
    return x.to_bytes(48, "big")


def fp_lex_largest(y):
    return y > (P - 1) // 2


def fp2_lex_largest(y):
    return fp_lex_largest(y[1]) or (y[1] == 0 and fp_lex_largest(y[0]))


def g1_to_uncompressed(a):
    """bls12_381 G1Affine::to_uncompressed (96 B)."""
    if a is None:
        out = bytearray(96)
        out[0] |= 0x40
        return bytes(out)
    return _fp_be(a[0]) + _fp_be(a[1])


def g1_to_compressed(a):
    """bls12_381 G1Affine::to_compressed (48 B) -- used by Proof::write."""
    if a is None:
        out = bytearray(48)
        out[0] |= 0xC0
        return bytes(out)
    out = bytearray(_fp_be(a[0]))
    out[0] |= 0x80
    if fp_lex_largest(a[1]):
        out[0] |= 0x20
    return bytes(out)


def g2_to_uncompressed(a):
    if a is None:
        out = bytearray(192)
        out[0] |= 0x40
        return bytes(out)
    (x0, x1), (y0, y1) = a
    return _fp_be(x1) + _fp_be(x0) + _fp_be(y1) + _fp_be(y0)


def g2_to_compressed(a):
    if a is None:
        out = bytearray(96)
        out[0] |= 0xC0
        return bytes(out)
    (x0, x1), y = a
    out = bytearray(_fp_be(x1) + _fp_be(x0))
    out[0] |= 0x80
    if fp2_lex_largest(y):
        out[0] |= 0x20
    return bytes(out)


def g1_from_uncompressed(b, checked=True):
    """G1Affine::from_uncompressed[_unchecked]; returns (ok, point_or_None)."""
    b = bytes(b)
    flags = b[0] >> 5
    comp, inf, srt = (flags >> 2) & 1, (flags >> 1) & 1, flags & 1
    x = int.from_bytes(bytes([b[0] & 0x1F]) + b[1:48], "big")
    y = int.from_bytes(b[48:96], "big")
    if comp or srt:
        return False, None
    if inf:
        return (x == 0 and y == 0), None
    if x >= P or y >= P:
        return False, None
    pt = (x, y)
    if checked:
        if not G1.on_curve_affine(pt):
            return False, None
        if not G1.is_identity(G1.mul(G1.from_affine(pt), R)):
            return False, None
    return True, pt


def g2_from_uncompressed(b, checked=True):
    b = bytes(b)
    flags = b[0] >> 5
    comp, inf, srt = (flags >> 2) & 1, (flags >> 1) & 1, flags & 1
    x1 = int.from_bytes(bytes([b[0] & 0x1F]) + b[1:48], "big")
    x0 = int.from_bytes(b[48:96], "big")
    y1 = int.from_bytes(b[96:144], "big")
    y0 = int.from_bytes(b[144:192], "big")
    if comp or srt:
        return False, None
    if inf:
        return (x0 == x1 == y0 == y1 == 0), None
    if max(x0, x1, y0, y1) >= P:
        return False, None
    pt = ((x0, x1), (y0, y1))
    if checked:
        if not G2.on_curve_affine(pt):
            return False, None
        if not G2.is_identity(G2.mul(G2.from_affine(pt), R)):
            return False, None
    return True, pt


# ---------------------------------------------------------------- Montgomery limbs
def fr_to_mont_limbs(x):
    """Fr element -> 4 little-endian u64 limbs of its Montgomery form (bls12_381 layout)."""
    v = x * FR_MONT_R % R
    return [(v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)]


def fr_from_mont_limbs(limbs):
    v = sum(int(l) << (64 * i) for i, l in enumerate(limbs))
    return v * pow(FR_MONT_R, -1, R) % R


def fr_to_le_limbs(x):
    """Scalar::to_le_bits() storage: canonical value as 4 LE u64 limbs."""
    return [(x >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)]
