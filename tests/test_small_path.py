"""The latency path (k_small: one launch per batch of <= 256 records, used by
bh_verify / the coalesced single Verify for small host batches) against the
oracle and against the batch path (BH_NO_SMALL) on the golden records: every
reject class, digest and fused (SHA-256 / SHA3-256) modes, registered and
unregistered keys, batch sizes 1 .. 256 (ragged), and no-low-S (x509 mode)."""
import hashlib
import os

import numpy as np
import pytest

from bdls_amd import _lib
from bdls_amd.bccsp import verify_packed
from oracle import ecdsa_ref as O
from tests.conftest import pack


def _chunks(recs, sizes):
    i, k = 0, 0
    while i < len(recs):
        m = sizes[k % len(sizes)]
        yield recs[i:i + m]
        i += m
        k += 1


def _want(recs, fused, sha3=False):
    out = []
    for r in recs:
        qx, qy = int(r["qx"], 16), int(r["qy"], 16)
        sig = bytes.fromhex(r["sig"])
        if fused:
            m = bytes.fromhex(r["msg"])
            dg = hashlib.sha3_256(m).digest() if sha3 else hashlib.sha256(m).digest()
        else:
            dg = bytes.fromhex(r["digest"])
        out.append(O.csp_verify(O.P256, qx, qy, sig, dg))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("registered", [False, True])
def test_small_batches_match_oracle(golden, fused, registered):
    recs = [r for r in golden if (not fused or "msg" in r)]
    L = _lib.lib()
    _lib.ensure_init()
    _lib.check(L.bh_keys_clear(-1, 0))
    if registered:
        keys = sorted({(int(r["qx"], 16), int(r["qy"], 16)) for r in recs
                       if int(r["qx"], 16) < 2**256 and int(r["qy"], 16) < 2**256})
        pub = np.frombuffer(b"".join(x.to_bytes(32, "big") + y.to_bytes(32, "big")
                                     for x, y in keys), np.uint8)
        st = np.zeros(len(keys), np.uint8)
        _lib.check(L.bh_keys_register(-1, 0, pub.ctypes.data, len(keys), st.ctypes.data))
    want = _want(recs, fused)
    got = []
    for ch in _chunks(recs, [1, 7, 64, 256, 3, 200]):
        v, rs = verify_packed(*pack(ch, fused), flags=_lib.BH_F_HASH_SHA256 if fused else 0)
        got += list(zip(v.tolist(), rs.tolist()))
    _lib.check(L.bh_keys_clear(-1, 0))
    bad = [(r["tag"], g, w) for r, g, w in zip(recs, got, want) if g != (w[0], w[1])]
    assert not bad, bad[:5]


@pytest.mark.gpu
def test_small_matches_batch_path(golden):
    """Same records, small path vs batch path (BH_NO_SMALL), SHA3 fused and
    no-low-S modes included."""
    recs = [r for r in golden if "msg" in r][:256]
    for flags in (_lib.BH_F_HASH_SHA256, _lib.BH_F_HASH_SHA3_256,
                  _lib.BH_F_HASH_SHA256 | _lib.BH_F_NO_LOW_S):
        small = verify_packed(*pack(recs, True), flags=flags)
        os.environ["BH_NO_SMALL"] = "1"
        try:
            batch = verify_packed(*pack(recs, True), flags=flags)
        finally:
            del os.environ["BH_NO_SMALL"]
        assert (small[0] == batch[0]).all() and (small[1] == batch[1]).all(), flags
