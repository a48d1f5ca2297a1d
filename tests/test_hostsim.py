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


def split_layout(msgs, seed):
    """Each message m as two spans (m[:k], m[k:]) at seam k (0, 1, block
    edges, len, random), laid out second span first with random gaps, as
    bh_verify_2seg sees a block's prp / endorser fields."""
    rng = np.random.default_rng(seed)
    buf, off1, len1, off2, len2 = bytearray(), [], [], [], []
    for i, m in enumerate(msgs):
        choices = [0, 1, 55, 56, 63, 64, 65, 128, len(m) - 1, len(m), int(rng.integers(0, len(m) + 1))]
        k = min(len(m), max(0, choices[i % len(choices)]))
        a, b = m[:k], m[k:]
        buf += bytes(int(rng.integers(0, 7)))
        off2.append(len(buf)); len2.append(len(b)); buf += b
        buf += bytes(int(rng.integers(0, 7)))
        off1.append(len(buf)); len1.append(len(a)); buf += a
    buf += b"\0"
    return (np.frombuffer(bytes(buf), np.uint8), np.array(off1, np.uint64), np.array(len1, np.uint32),
            np.array(off2, np.uint64), np.array(len2, np.uint32))


@pytest.mark.parametrize("family", ["SHA2", "SHA3"])
def test_hostsim_two_span_messages(hs, family):
    """bh_verify_2seg's device hashing (sha256_msg2 / sha3_256_msg2): every
    seam position gives the verdicts of the one-span message."""
    from bdls_amd import workload
    from bdls_amd._lib import BH_F_HASH_SHA256, BH_F_HASH_SHA3_256
    w = workload.generate(330, 30, 300, 4, seed=17, nthreads=4, family=family)
    pub, sig, so, sl, msg, mo, ml = w.arrays()
    msgs = [bytes(msg[int(o):int(o) + int(l)]) for o, l in zip(mo, ml)]
    mbuf, o1, l1, o2, l2 = split_layout(msgs, 5)
    flags = BH_F_HASH_SHA3_256 if family == "SHA3" else BH_F_HASH_SHA256
    vp = ctypes.c_void_p
    hs.hs_verify_2seg.argtypes = [vp] * 9 + [ctypes.c_uint32] * 2 + [vp]
    out = np.full(w.n, 255, np.uint8)
    hs.hs_verify_2seg(pub.ctypes.data, sig.ctypes.data, so.ctypes.data, sl.ctypes.data,
                      mbuf.ctypes.data, o1.ctypes.data, l1.ctypes.data, o2.ctypes.data,
                      l2.ctypes.data, w.n, flags, out.ctypes.data)
    assert (out == w.reason).all()
    assert (l1 == 0).any() and (l2 == 0).any() and ((l1 > 64) & (l2 > 64)).any()
