"""Device self-tests of hand-bounded field arithmetic (csrc/selftest.hip).

fe2_mul_sub_kara (field.cuh, the G2 mixed addition's Y3 = R (Q - X3) - Y1 PPP under one
Montgomery reduction per half) keeps signed Karatsuba column sums in a biased unsigned 64-bit
accumulator and adds p when the top limb comes out negative; its bounds are argued for operands
< 2^386 with normalised 29-bit limbs.  Checked here at those maxima (every limb 2^29 - 1 below a
top limb of 2^9 - 1), at the madd's stated operand bounds (R < 6p, Q - X3 + 16p < 18p, Y < 4p,
PPP < 2p), where the result is negative before the fix-up (c*d > a*b), and on random values,
against host big integers and against two full Fp2 products and a subtraction."""
import ctypes
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R_MONT = 1 << 406
N, BITS = 14, 29


def _limbs(x):
    assert 0 <= x < 1 << 386
    return [(x >> (BITS * i)) & ((1 << BITS) - 1) if i < N - 1 else x >> (BITS * (N - 1)) for i in range(N)]


def _value(ls):
    return sum(int(v) << (BITS * i) for i, v in enumerate(ls))


def _run(cases):
    import bellman_hip as bh
    lib = bh.lib()
    f = lib.bh_selftest_fp2_mul_sub
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    inp = np.array([_limbs(x) for case in cases for x in case], dtype=np.uint32)
    out = np.zeros((len(cases) * 4, N), dtype=np.uint32)
    assert f(0, inp.ctypes.data, len(cases), out.ctypes.data) == 0
    return out.reshape(len(cases), 4, N)


def test_fp2_mul_sub_lazy_at_operand_maxima_and_negative_results():
    rinv = pow(R_MONT, -1, P)
    top = (1 << 386) - 1  # every limb 2^29 - 1, top limb 2^9 - 1
    rng = random.Random(386)
    pool = [0, 1, P - 1, P, 2 * P - 1, 4 * P - 1, 6 * P - 1, 18 * P - 1, top, top - 1]
    cases = [
        [6 * P - 1] * 2 + [18 * P - 1] * 2 + [4 * P - 1] * 2 + [2 * P - 1] * 2,  # the madd's stated bounds
        [top] * 8,                                                           # limb maxima everywhere
        [0, 0, 0, 0, top, top, top, top],                                    # -c*d: negative halves
        [1, 0, 1, 0, top, 0, top, 0],                                        # c0 negative only
        [0, 1, 0, 1, top, top, 0, top],
        [top, 0, 0, top, 0, top, top, 0],
    ]
    for _ in range(3000):
        cases.append([rng.choice(pool) if rng.random() < 0.7 else rng.randrange(1 << 386) for _ in range(8)])
    out = _run(cases)
    neg_seen = 0
    for case, res in zip(cases, out):
        a0, a1, b0, b1, c0, c1, d0, d1 = case
        want0 = ((a0 * b0 - a1 * b1) - (c0 * d0 - c1 * d1)) * rinv % P
        want1 = ((a0 * b1 + a1 * b0) - (c0 * d1 + c1 * d0)) * rinv % P
        lz0, lz1, tw0, tw1 = (_value(r) for r in res)
        for v in res:  # normalised limbs below the top one
            assert all(int(x) < 1 << BITS for x in v[:-1]), case
        assert lz0 < 2 * P and lz1 < 2 * P, case
        assert lz0 % P == want0 and lz1 % P == want1, case
        assert tw0 % P == want0 and tw1 % P == want1, case
        neg_seen += (a0 * b0 - a1 * b1) < (c0 * d0 - c1 * d1)
    assert neg_seen > 100
