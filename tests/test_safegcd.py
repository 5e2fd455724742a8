"""The device Fp inversion (csrc/safegcd.h, Bernstein-Yang divsteps) built for the host with g++:
x * x^-1 = 1 mod p on random and edge values, within the 32-batch bound the device loop uses.
The batch-affine bucket accumulation (csrc/msm_affine.cuh) inverts one product per thread per
level with it; the proof parity tests cover it on the device."""
import os
import random
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB


@pytest.fixture(scope="module")
def exe():
    d = tempfile.mkdtemp()
    out = os.path.join(d, "safegcd_test")
    subprocess.check_call(["g++", "-O2", "-std=c++17", os.path.join(ROOT, "tests", "cpp", "safegcd_test.cpp"),
                           "-o", out])
    return out


def run(exe, xs):
    inp = "".join(" ".join("%x" % ((x >> (32 * k)) & 0xffffffff) for k in range(12)) + "\n" for x in xs)
    res = subprocess.run([exe], input=inp, capture_output=True, text=True, check=True).stdout.split("\n")
    out = []
    for line in res[:len(xs)]:
        parts = line.split()
        v = sum(int(parts[k], 16) << (32 * k) for k in range(12))
        out.append((v, int(parts[12])))
    return out


def test_inverse_random_and_edges(exe):
    rng = random.Random(7)
    xs = [1, 2, 3, P - 1, P - 2, (P + 1) // 2, 1 << 380, (1 << 381) % P, 0x1fffffff, 1 << 29, 1 << 30]
    xs += [rng.randrange(1, P) for _ in range(2000)]
    xs += [rng.randrange(1, 1 << rng.randrange(1, 381)) % P or 1 for _ in range(500)]
    got = run(exe, xs)
    worst = 0
    for x, (inv, nb) in zip(xs, got):
        assert inv < P
        assert x * inv % P == 1, hex(x)
        assert 0 < nb <= 32
        worst = max(worst, nb)
    assert worst <= 32


def test_inverse_of_zero_is_zero(exe):
    assert run(exe, [0])[0][0] == 0
