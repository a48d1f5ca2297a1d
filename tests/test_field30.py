"""CPU: the radix-2^30 lazy field (bdls_amd/csrc/fp30.h, compiled for the host by
the test-only harness) at the edges of its value contract:
  f_mul needs beta_a * beta_b <= 16000 (tested to 16000; the formulas stay <= 9604) and returns t < 2p, t == a b 2^-270 (mod p);
  f_sub<K> needs beta_b <= K - 1 and returns a - b + K p with normalised limbs;
  round 6's fused one-pass forms (f_add2x a + 2b, f_addsub a + b - c + K p,
  f_sub2 a - b - c + K p, f_csub +-s - y + K p) on both curves, with values and
  limb patterns (every limb 0 or 2^30 - 1) at their contracts' edges: a limb
  sum leaving u32 would show as a wrong value.
Values are drawn at the bounds (beta p - 1, all-ones limbs, 0, p) to catch
64-bit column overflow."""
import ctypes
import os
import random

import pytest

from tests.conftest import ROOT

P = 2**256 - 2**224 + 2**192 + 2**96 - 1
R = 2**270
M = 2**30 - 1
LIB = os.path.join(ROOT, "tests", "native", "build", "libhostsim.so")


@pytest.fixture(scope="module")
def L():
    if not os.path.exists(LIB):
        pytest.skip("hostsim not built")
    return ctypes.CDLL(LIB)


def to9(v):
    l = [(v >> (30 * i)) & M for i in range(8)] + [v >> 240]
    assert l[8] < 2**32
    return (ctypes.c_uint32 * 9)(*l)


def from9(a):
    return sum(int(a[i]) << (30 * i) for i in range(9))


def normalised(a):
    return all(int(a[i]) <= M for i in range(8))


def edge_values(beta, rng, k=40):
    hi = beta * P - 1
    vals = [0, 1, P - 1, P, P + 1, hi, hi - P, 2**256 - 1 if 2**256 - 1 <= hi else hi]
    # all limbs 0..7 at 2^30 - 1 with the largest admissible top limb
    top = hi >> 240
    v = sum(M << (30 * i) for i in range(8)) + (top << 240)
    while v > hi:
        top -= 1
        v = sum(M << (30 * i) for i in range(8)) + (top << 240)
    vals.append(v)
    vals += [rng.randrange(hi + 1) for _ in range(k)]
    return [v for v in vals if v <= hi]


@pytest.mark.parametrize("ba,bb", [(2, 2), (34, 34), (66, 66), (66, 36), (126, 126), (6, 56),
                                   (98, 98), (236, 6), (8000, 2), (2, 8000), (90, 90)])
def test_f_mul_bounds(L, ba, bb):
    rng = random.Random(ba * 1000 + bb)
    out = (ctypes.c_uint32 * 9)()
    Rinv = pow(R, -1, P)
    for a in edge_values(ba, rng, 25):
        for b in edge_values(bb, rng, 5):
            L.hs_f_mul(to9(a), to9(b), out)
            t = from9(out)
            assert normalised(out)
            assert t < 2 * P, (ba, bb)
            assert t % P == a * b * Rinv % P


@pytest.mark.parametrize("K", [32, 64])
def test_f_sub_bounds(L, K):
    rng = random.Random(K)
    out = (ctypes.c_uint32 * 9)()
    fn = L.hs_f_sub32 if K == 32 else L.hs_f_sub64
    for a in edge_values(66, rng, 30):
        for b in edge_values(K - 1, rng, 30):
            fn(to9(a), to9(b), out)
            assert normalised(out)
            assert from9(out) == a - b + K * P


def test_f_add_reduce(L):
    rng = random.Random(3)
    out = (ctypes.c_uint32 * 9)()
    for a in edge_values(64, rng, 20):
        for b in edge_values(64, rng, 5):
            L.hs_f_add(to9(a), to9(b), out)
            assert normalised(out) and from9(out) == a + b
            L.hs_f_reduce(to9(a + b), out)
            assert from9(out) == (a + b) % P


@pytest.mark.parametrize("ba", [2, 34, 66, 98, 126])
def test_f_sqr_bounds(L, ba):
    rng = random.Random(ba)
    out = (ctypes.c_uint32 * 9)()
    Rinv = pow(R, -1, P)
    for a in edge_values(ba, rng, 200):
        L.hs_f_sqr(to9(a), out)
        t = from9(out)
        assert normalised(out) and t < 2 * P
        assert t % P == a * a * Rinv % P


P_K1 = 2**256 - 2**32 - 977


def limb_patterns(beta, p, rng, k=30):
    """Values <= beta p - 1 whose low limbs are each 0 or 2^30 - 1 (the per-limb
    extremes of the fused passes' u32 sums), top limb as large as allowed."""
    hi = beta * p - 1
    out = []
    for _ in range(k):
        low = sum((M if rng.random() < 0.5 else 0) << (30 * i) for i in range(8))
        top = (hi - low) >> 240
        if top >= 0:
            out.append(low + (top << 240))
    return out


def edge_all(beta, p, rng, k=12):
    return [v for v in edge_values(beta, rng, k) if v <= beta * p - 1] + limb_patterns(beta, p, rng)


@pytest.mark.parametrize("curve", [0, 1])
@pytest.mark.parametrize("K", [32, 64])
def test_fused_passes(L, curve, K):
    p = P if curve == 0 else P_K1
    rng = random.Random(curve * 100 + K)
    out = (ctypes.c_uint32 * 9)()
    call = L.hs_f_fused
    z = to9(0)
    # f_add2x: a + 2 b (the formulas: H^3 + 2V, beta 2 + 2 * 2)
    for a in edge_all(34, p, rng):
        for b in edge_all(34, p, rng, 4):
            call(curve, K, 0, to9(a), to9(b), z, out)
            assert normalised(out) and from9(out) == a + 2 * b
    # f_addsub: a + b - c + K p, value(c) <= K p (V - X3 = w + V - r^2, beta 6 + 2 + 32)
    for a in edge_all(34, p, rng):
        for b in edge_all(34, p, rng, 3):
            for c in edge_all(K, p, rng, 3):
                call(curve, K, 1, to9(a), to9(b), to9(c), out)
                assert normalised(out) and from9(out) == a + b - c + K * p
    # f_sub2: a - b - c + K p, value(b) + value(c) <= K p (X3 = D - W1 - W2)
    for a in edge_all(66, p, rng):
        for bb, bc in ((K // 2, K // 2), (2, K - 2), (K - 2, 2)):
            for b in edge_all(bb, p, rng, 3):
                for c in edge_all(bc, p, rng, 3):
                    call(curve, K, 2, to9(a), to9(b), to9(c), out)
                    assert normalised(out) and from9(out) == a - b - c + K * p
    # f_csub: (+-s) - y + K p (the additions' r with the table point's sign)
    for s_ in edge_all(2, p, rng):
        for y in edge_all(K, p, rng, 6):
            call(curve, K, 3, to9(s_), to9(y), z, out)
            assert normalised(out) and from9(out) == s_ - y + K * p
        for y in edge_all(K - 2, p, rng, 6):
            call(curve, K, 4, to9(s_), to9(y), z, out)
            assert normalised(out) and from9(out) == K * p - s_ - y


@pytest.mark.parametrize("curve", [0, 1])
def test_csub_96(L, curve):
    """f_csub<96>: the mixed addition's r = +-S2 - Y1 + 96 p with Y1 up to a
    negated table y (64 p) -- the case a GPU edge batch caught at K = 64."""
    p = P if curve == 0 else P_K1
    rng = random.Random(96 + curve)
    out = (ctypes.c_uint32 * 9)()
    z = to9(0)
    for s_ in edge_all(2, p, rng):
        for y in edge_all(94, p, rng, 8):
            L.hs_f_fused(curve, 96, 4, to9(s_), to9(y), z, out)
            assert normalised(out) and from9(out) == 96 * p - s_ - y
        for y in edge_all(96, p, rng, 8):
            L.hs_f_fused(curve, 96, 3, to9(s_), to9(y), z, out)
            assert normalised(out) and from9(out) == s_ - y + 96 * p
