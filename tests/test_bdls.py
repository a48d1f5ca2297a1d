"""BDLS consensus-message verification:
SignedProto.Hash (BLAKE2b-256 framing, message.go:97-138) + SignedProto.Verify
(message.go:170-184) on secp256k1 (as wired, chain.go:60-61 -> Go verifyLegacy)
and P-256 (curve-generic library -> verifyNISTEC).

CPU: the oracle re-derives every golden record and agrees with OpenSSL; the
device arithmetic (host build) matches on both curves and both verify paths,
plus secp256k1 curve-level edge cases at the digest level.
GPU (-m gpu): the same golden set through bh_verify_bdls, bit-exact."""
import ctypes
import hashlib
import json
import os
import random

import numpy as np
import pytest

from oracle import ecdsa_ref as O
from tests.bdls_util import pack_bdls
from tests.conftest import ROOT

GOLD = os.path.join(ROOT, "tests", "golden", "bdls_vectors.jsonl")
LIB = os.path.join(ROOT, "tests", "native", "build", "libhostsim.so")
CURVE_ID = {"P-256": 0, "secp256k1": 1}


@pytest.fixture(scope="module")
def bdls_golden():
    with open(GOLD) as f:
        return [json.loads(l) for l in f]


def test_bdls_golden_rederive(bdls_golden):
    for r in bdls_golden:
        c = O.SECP256K1 if r["curve"] == "secp256k1" else O.P256
        x, y, m = bytes.fromhex(r["x"]), bytes.fromhex(r["y"]), bytes.fromhex(r["msg"])
        assert O.bdls_signed_proto_hash(r["version"], x, y, m).hex() == r["digest"]
        ok = O.bdls_signed_proto_verify(c, r["version"], x, y, m, bytes.fromhex(r["r"]),
                                        bytes.fromhex(r["s"]))
        assert ok == r["valid"], r["tag"]


def test_bdls_golden_vs_openssl(bdls_golden):
    from oracle import orc
    for r in bdls_golden:
        rv, sv = int(r["r"] or "0", 16), int(r["s"] or "0", 16)
        if not (0 < rv < 2**256 and 0 < sv < 2**256):
            continue
        rc = orc.go_verify(bytes.fromhex(r["x"] + r["y"]), bytes.fromhex(r["digest"]), rv, sv,
                           curve=CURVE_ID[r["curve"]])
        assert rc == r["reason"], r["tag"]


@pytest.fixture(scope="module")
def hs():
    if not os.path.exists(LIB):
        pytest.skip("hostsim not built")
    L = ctypes.CDLL(LIB)
    vp = ctypes.c_void_p
    L.hs_verify_bdls.argtypes = [ctypes.c_int] + [vp] * 11 + [ctypes.c_uint32] * 2 + [vp]
    L.hs_verify_k1_digest.argtypes = [vp] * 7 + [ctypes.c_uint32] * 2 + [vp]
    return L


@pytest.mark.parametrize("curve", ["secp256k1", "P-256"])
@pytest.mark.parametrize("min_uses", [1, 1000])
def test_bdls_hostsim(hs, bdls_golden, curve, min_uses):
    recs = [r for r in bdls_golden if r["curve"] == curve]
    arrs = pack_bdls(recs)
    out = np.zeros(len(recs), np.uint8)
    hs.hs_verify_bdls(CURVE_ID[curve], *[a.ctypes.data for a in arrs], len(recs), min_uses,
                      out.ctypes.data)
    bad = [(r["tag"], int(o), r["reason"]) for r, o in zip(recs, out) if o != r["reason"]]
    assert not bad


def _k1_edge_records():
    """secp256k1 digest-level edge cases (x wrap, infinity, internal doubling)."""
    c = O.SECP256K1
    rng = random.Random(99)
    recs = []

    def add(tag, qx, qy, r, s, digest):
        reason = O.go_ecdsa_verify(c, qx, qy, digest, r, s)
        recs.append((tag, qx, qy, O.marshal_ecdsa_signature(r, s), digest, reason))

    d = rng.randrange(1, c.n)
    qx, qy = O.pubkey(c, d)
    for _ in range(2):  # x(R) in [n, p): accepted through x mod n == r
        while True:
            x = c.n + rng.randrange(c.p - c.n)
            rhs = (x ** 3 + 7) % c.p
            y = pow(rhs, (c.p + 1) // 4, c.p)
            if y * y % c.p == rhs:
                break
        add("k1_xwrap_accept", x, y, x - c.n, x - c.n, b"\x00" * 32)
        add("k1_xwrap_wrong_r", x, y, x - c.n + 1, x - c.n, b"\x00" * 32)
    for _ in range(2):  # u1 G + u2 Q = infinity
        r = rng.randrange(1, c.n)
        add("k1_sum_inf", qx, qy, r, rng.randrange(1, c.n), ((-r * d) % c.n).to_bytes(32, "big"))
    for _ in range(3):  # u1 G == u2 Q (doubling inside the final addition)
        k = rng.randrange(1, c.n)
        r = O.scalar_mult(c, k, (c.gx, c.gy))[0] % c.n
        e = r * d % c.n
        s = 2 * r * d * pow(k, -1, c.n) % c.n
        add("k1_u1G_eq_u2Q", qx, qy, r, s, e.to_bytes(32, "big"))
        add("k1_u1G_eq_u2Q_high_s", qx, qy, r, c.n - s, e.to_bytes(32, "big"))
    for _ in range(6):  # plain valid / invalid, high-S accepted (no low-S rule)
        msgd = bytes(rng.getrandbits(8) for _ in range(32))
        r, s = O.sign_digest(c, d, msgd, rng.randrange(1, c.n), low_s=False)
        add("k1_valid", qx, qy, r, s, msgd)
        add("k1_flip", qx, qy, r, s, bytes([msgd[0] ^ 1]) + msgd[1:])
    return recs


@pytest.mark.parametrize("min_uses", [1, 1000])
def test_k1_curve_edges_hostsim(hs, min_uses):
    recs = _k1_edge_records()
    pub = np.frombuffer(b"".join(qx.to_bytes(32, "big") + qy.to_bytes(32, "big")
                                 for _, qx, qy, _, _, _ in recs), np.uint8)
    sigs = [t[3] for t in recs]
    dgs = [t[4] for t in recs]
    sl = np.array([len(x) for x in sigs], np.uint32)
    dl = np.array([len(x) for x in dgs], np.uint32)
    so = np.concatenate([[0], np.cumsum(sl[:-1])]).astype(np.uint64)
    do = np.concatenate([[0], np.cumsum(dl[:-1])]).astype(np.uint64)
    sig = np.frombuffer(b"".join(sigs), np.uint8)
    dg = np.frombuffer(b"".join(dgs), np.uint8)
    out = np.zeros(len(recs), np.uint8)
    hs.hs_verify_k1_digest(pub.ctypes.data, sig.ctypes.data, so.ctypes.data, sl.ctypes.data,
                           dg.ctypes.data, do.ctypes.data, dl.ctypes.data, len(recs), min_uses,
                           out.ctypes.data)
    bad = [(t[0], int(o), t[5]) for t, o in zip(recs, out) if o != t[5]]
    assert not bad
    assert any(t[0] == "k1_xwrap_accept" and t[5] == 0 for t in recs)


@pytest.mark.gpu
@pytest.mark.parametrize("curve", ["secp256k1", "P-256"])
def test_bdls_gpu_golden(bdls_golden, curve):
    from bdls_amd import _lib
    _lib.ensure_init()
    recs = [r for r in bdls_golden if r["curve"] == curve]
    arrs = pack_bdls(recs)
    n = len(recs)
    bitmap = np.zeros((n + 7) // 8, np.uint8)
    reason = np.zeros(n, np.uint8)
    b = _lib.BhBdlsBatch(*[a.ctypes.data for a in arrs])
    _lib.check(_lib.lib().bh_verify_bdls(CURVE_ID[curve], ctypes.byref(b), n, bitmap.ctypes.data,
                                         reason.ctypes.data))
    bad = [(r["tag"], int(g), r["reason"]) for r, g in zip(recs, reason) if g != r["reason"]]
    assert not bad
    valid = np.unpackbits(bitmap, bitorder="little")[:n].astype(bool)
    assert [bool(v) for v in valid] == [r["valid"] for r in recs]
