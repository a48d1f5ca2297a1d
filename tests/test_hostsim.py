"""CPU: the device arithmetic (bdls_amd/csrc/verify.h -- the exact stage
functions the HIP kernels run) compiled for the host by the TEST-ONLY harness
tests/native/hostsim.cpp, checked against the golden vectors and a generated
batch. This is logic validation without a GPU; it is never the product path."""
import ctypes
import os

import numpy as np
import pytest

from tests.conftest import ROOT, pack

LIB = os.path.join(ROOT, "tests", "native", "build", "libhostsim.so")


@pytest.fixture(scope="module")
def hs():
    if not os.path.exists(LIB):
        pytest.skip("hostsim not built (make)")
    L = ctypes.CDLL(LIB)
    vp = ctypes.c_void_p
    L.hs_verify.argtypes = [vp] * 7 + [ctypes.c_uint32] * 3 + [vp]
    L.hs_verify2.argtypes = [vp] * 7 + [ctypes.c_uint32] * 4 + [vp, vp]
    return L


def run(L, arrs, fused, chunk=4):
    pub, sig, so, sl, msg, mo, ml = arrs
    n = len(sl)
    out = np.zeros(n, np.uint8)
    L.hs_verify(pub.ctypes.data, sig.ctypes.data, so.ctypes.data, sl.ctypes.data, msg.ctypes.data,
                mo.ctypes.data, ml.ctypes.data, n, 1 if fused else 0, chunk, out.ctypes.data)
    return out


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("chunk", [1, 7])
def test_hostsim_golden(hs, golden, fused, chunk):
    recs = [r for r in golden if (not fused) or "msg" in r]
    out = run(hs, pack(recs, fused), fused, chunk)
    bad = [(r["tag"], int(o), r["reason"]) for r, o in zip(recs, out) if o != r["reason"]]
    assert not bad


def test_hostsim_workload(hs):
    from bdls_amd import workload
    w = workload.generate(700, 50, 256, 4, seed=11, nthreads=4)
    out = run(hs, w.arrays(), True, 16)
    assert (out == w.reason).all()


def run2(L, arrs, fused, min_uses):
    pub, sig, so, sl, msg, mo, ml = arrs
    n = len(sl)
    out = np.zeros(n, np.uint8)
    ncomb = ctypes.c_uint32()
    L.hs_verify2(pub.ctypes.data, sig.ctypes.data, so.ctypes.data, sl.ctypes.data, msg.ctypes.data,
                 mo.ctypes.data, ml.ctypes.data, n, 1 if fused else 0, 4, min_uses,
                 out.ctypes.data, ctypes.byref(ncomb))
    return out, ncomb.value


@pytest.mark.parametrize("fused", [False, True])
def test_hostsim_golden_keycomb_path(hs, golden, fused):
    """min_uses = 1 forces every record through the per-key table path."""
    recs = [r for r in golden if (not fused) or "msg" in r]
    out, ncomb = run2(hs, pack(recs, fused), fused, 1)
    assert ncomb > 0
    bad = [(r["tag"], int(o), r["reason"]) for r, o in zip(recs, out) if o != r["reason"]]
    assert not bad


@pytest.mark.parametrize("wide", [4, 16])
@pytest.mark.parametrize("fused", [False, True])
def test_hostsim_golden_wide_keycomb(hs, golden, fused, wide):
    """The L-lanes-per-record key-table path (k_keycomb_wide): interleaved
    windows, offset recoding, butterfly combine -- bit-exact on every golden
    record, including the crafted infinity / u1 G == u2 Q / x-wrap cases."""
    recs = [r for r in golden if (not fused) or "msg" in r]
    hs.hs_set_wide(wide)
    try:
        out, ncomb = run2(hs, pack(recs, fused), fused, 1)
    finally:
        hs.hs_set_wide(1)
    assert ncomb > 0
    bad = [(r["tag"], int(o), r["reason"]) for r, o in zip(recs, out) if o != r["reason"]]
    assert not bad


def test_hostsim_workload_mixed_paths(hs):
    from bdls_amd import workload
    w = workload.generate(900, 60, 256, 4, seed=13, nthreads=4)
    out, ncomb = run2(hs, w.arrays(), True, 4)
    assert 0 < ncomb < w.n
    assert (out == w.reason).all()


def test_hostsim_workload_sha3(hs):
    """SHA3 hash family (msp/identities.go:219-227): records signed over
    SHA3-256(msg); the SHA-256 flag must reject the valid ones."""
    from bdls_amd import workload
    from bdls_amd._lib import BH_F_HASH_SHA3_256
    w = workload.generate(300, 40, 300, 4, seed=13, nthreads=4, family="SHA3")
    pub, sig, so, sl, msg, mo, ml = w.arrays()
    out = np.zeros(w.n, np.uint8)
    hs.hs_verify(pub.ctypes.data, sig.ctypes.data, so.ctypes.data, sl.ctypes.data,
                 msg.ctypes.data, mo.ctypes.data, ml.ctypes.data, w.n, BH_F_HASH_SHA3_256, 8,
                 out.ctypes.data)
    assert (out == w.reason).all()
    out2 = run(hs, w.arrays(), True, 8)
    assert (out2[w.reason == 0] != 0).all()
