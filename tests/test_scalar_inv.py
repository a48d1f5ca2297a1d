"""CPU: the safegcd (divsteps) scalar inversion of bdls_amd/csrc/fe.h
(mod_inv_sg / mont_inv_sg, used by k_inv for s^-1 mod n), compiled for the host
by the test-only harness, against Python's pow(a, -1, n) for both group orders.
Inputs at the edges (1, 2, n-1, n-2, powers of two, all-ones limbs below n) and
seeded random values."""
import ctypes
import os
import random

import pytest

from tests.conftest import ROOT

N = {0: 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551,
     1: 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141}
LIB = os.path.join(ROOT, "tests", "native", "build", "libhostsim.so")


@pytest.fixture(scope="module")
def L():
    if not os.path.exists(LIB):
        pytest.skip("hostsim not built")
    return ctypes.CDLL(LIB)


def to8(v):
    return (ctypes.c_uint32 * 8)(*[(v >> (32 * i)) & 0xFFFFFFFF for i in range(8)])


def from8(a):
    return sum(int(a[i]) << (32 * i) for i in range(8))


def cases(n):
    rng = random.Random(n & 0xFFFF)
    edge = [1, 2, 3, n - 1, n - 2, (n - 1) // 2, (n + 1) // 2, 2**255 % n, 2**128, 2**30,
            2**30 - 1, (2**256 - 1) % n, int("3fffffff" * 8, 16) % n]
    return edge + [rng.randrange(1, n) for _ in range(400)]


@pytest.mark.parametrize("curve", [0, 1])
def test_mod_inv_sg(L, curve):
    n = N[curve]
    out = (ctypes.c_uint32 * 8)()
    for a in cases(n):
        L.hs_n_inv(curve, to8(a), out)
        assert from8(out) == pow(a, -1, n), hex(a)


@pytest.mark.parametrize("curve", [0, 1])
def test_mont_inv_sg(L, curve):
    n = N[curve]
    R = 2**256
    out = (ctypes.c_uint32 * 8)()
    for a in cases(n)[:100]:
        L.hs_n_mont_inv(curve, to8(a * R % n), out)
        assert from8(out) == pow(a, -1, n) * R % n, hex(a)


@pytest.mark.parametrize("curve", [0, 1])
def test_mod_inv_sg_variable_time(L, curve):
    """The latency kernel's variable-time divsteps (divsteps30_var: runs of
    zeros shifted at once, up to 6 low bits cancelled per step, early exit at
    g = 0) give the same inverse as the constant-time schedule."""
    n = N[curve]
    rng = random.Random(curve + 99)
    out = (ctypes.c_uint32 * 8)()
    for a in cases(n) + [rng.randrange(1, n) for _ in range(3000)] + \
            [rng.randrange(1, 2**k) for k in range(1, 257, 5)]:
        L.hs_n_inv_var(curve, to8(a), out)
        assert from8(out) == pow(a, -1, n), hex(a)
