"""bh_verify_x509 (Go crypto/x509 CheckSignatureFrom for ECDSA issuers) on the
reference's own MSP test certificates (msp/testdata, sampleconfig/msp:
tests/golden/x509_vectors.json, made by tests/golden/gen_x509.py) and
mutations of them. CPU: the oracle (oracle/x509_ref.py) against OpenSSL's
ECDSA core (oracle/orc.c) on every vector whose signature parses. GPU: the
engine, bit-exact in bitmap and reason."""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import ecdsa_ref as O
from oracle import x509_ref as X
from tests.conftest import ROOT

VEC = os.path.join(ROOT, "tests", "golden", "x509_vectors.json")


@pytest.fixture(scope="module")
def vectors():
    with open(VEC) as f:
        return json.load(f)


def test_fixture_covers_reference_chains(vectors):
    ref = [v for v in vectors if v["tag"].startswith("ref:")]
    assert sum(v["reason"] == 0 for v in ref) >= 40       # real CA -> cert links verify
    assert {v["reason"] for v in vectors} >= {0, 3, 4, 5, 7, 8, 9, 10, 11}


def test_oracle_matches_openssl(vectors):
    from oracle import orc
    n = O.P256.n
    checked = 0
    for v in vectors:
        der = bytes.fromhex(v["cert"])
        parts = X.split_cert(der)
        if parts is None or v["reason"] in (X.R_UNSUPPORTED, O.R_DER):
            continue
        tbs, _, _, sig = parts
        r, s = X.parse_signature(sig)
        if not (0 < r < n and 0 < s < n):
            continue
        low = O.marshal_ecdsa_signature(r, min(s, n - s))
        pub = bytes.fromhex(v["qx"] + v["qy"])
        got = orc.csp_verify(pub, low, hashlib.sha256(tbs).digest())
        assert (got == 0) == (v["reason"] == 0), v["tag"]
        checked += 1
    assert checked > 200


def _pack(vecs):
    certs = [bytes.fromhex(v["cert"]) for v in vecs]
    ln = np.array([len(c) for c in certs], np.uint32)
    off = np.zeros(len(certs), np.uint64)
    off[1:] = np.cumsum(ln[:-1])
    buf = np.frombuffer(b"".join(certs) + b"\0", np.uint8)
    pub = np.frombuffer(b"".join(bytes.fromhex(v["qx"] + v["qy"]) for v in vecs), np.uint8)
    return buf, off, ln, pub


@pytest.mark.gpu
def test_gpu_x509_vectors(vectors):
    from bdls_amd import _lib
    _lib.ensure_init()
    buf, off, ln, pub = _pack(vectors)
    n = len(vectors)
    bm = np.zeros((n + 7) // 8, np.uint8)
    rs = np.zeros(n, np.uint8)
    _lib.check(_lib.lib().bh_verify_x509(buf.ctypes.data, off.ctypes.data, ln.ctypes.data,
                                         pub.ctypes.data, n, bm.ctypes.data, rs.ctypes.data))
    bad = [(v["tag"], int(g), v["reason"]) for v, g in zip(vectors, rs) if g != v["reason"]]
    assert not bad, bad[:5]
    bits = np.unpackbits(bm, bitorder="little")[:n].astype(bool)
    assert (bits == np.array([v["reason"] == 0 for v in vectors])).all()
