"""The arithmetic behind the NTT's one-step reduction (ntt.hip fr_qreduce) and its pass split,
restated on the host: the device kernels themselves are checked against the oracle by the GPU
parity tests (golden domains, extreme values, every proof); these pin the bounds they rely on.

fr_qreduce: x < 2^261 held as 9 x 29-bit limbs (the low 8 normalised), q = floor(x8 / (r8 + 1))
from the top limb via one FP64 fma of (x8 + 1/2) * (r8 + 1)^-1, then x - q r < 2r."""
import math
import random

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
BITS = 29
R8 = R >> (8 * BITS)  # the modulus' top limb
INV = 1.0 / float(R8 + 1)  # (r8 + 1) is exact in a double, its inverse rounded once


def fma(a, b, c):
    """a * b + c with one rounding (math.fma where Python has it; exact rationals otherwise)."""
    if hasattr(math, "fma"):
        return math.fma(a, b, c)
    from fractions import Fraction
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def qreduce(x):
    x8 = x >> (8 * BITS)
    q = int(fma(float(x8), INV, 0.5 * INV))
    return q, x - q * R


def test_quotient_is_exact_at_every_multiple_boundary():
    d = R8 + 1
    for k in range(0, (1 << 29) // d + 1):
        for x8 in (k * d - 1, k * d, k * d + 1):
            if 0 <= x8 < (1 << 29):
                assert int(fma(float(x8), INV, 0.5 * INV)) == x8 // d


def test_remainder_below_two_r_for_any_value_below_2_261():
    rng = random.Random(2606)
    lows = [0, (1 << (8 * BITS)) - 1]
    for _ in range(20000):
        x = rng.randrange(1 << 261)
        for low in lows + [x & ((1 << (8 * BITS)) - 1)]:
            v = ((x >> (8 * BITS)) << (8 * BITS)) | low
            q, y = qreduce(v)
            assert 0 <= y < 2 * R
            assert q * R <= v


def test_lazy_dit_bound_fits_the_product():
    # a DIT pass adds at most 2r per stage to inputs < 2r (<= 10 stages per pass: < 22r), and a
    # Montgomery product of an operand < A r with a twiddle < r ends < 2r while A < 2^261 / r
    assert 2 * 11 * R < (1 << 261)
    assert (1 << 261) // R >= 70


def pass_depths(L):
    """launch_ntt's split of L stages into passes of <= 10 (ntt.hip): even depths where possible."""
    passes = (L + 9) // 10
    pairs = L // 2
    ds = [2 * (pairs // passes + (1 if p < pairs % passes else 0)) for p in range(passes)]
    if L & 1:
        q = passes - 1
        for p in range(passes - 1, -1, -1):
            if ds[p] < ds[q]:
                q = p
        ds[q] += 1
    return ds


def test_pass_depths_cover_every_size_with_at_most_one_odd_pass():
    for L in range(1, 33):
        ds = pass_depths(L)
        assert sum(ds) == L and all(1 <= d <= 10 for d in ds)
        assert len(ds) == (L + 9) // 10
        assert sum(d & 1 for d in ds) == (L & 1)
    assert pass_depths(22) == [8, 8, 6]
