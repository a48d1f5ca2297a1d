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
@pytest.mark.parametrize("min_uses,ll", [(1, 0), (1000, 0), (1, 1)])
def test_bdls_hostsim(hs, bdls_golden, curve, min_uses, ll):
    """ll = 1: per-batch key tables as the signed Lim-Lee comb (what the device
    builds for BDLS batches above 32,768 records), secp256k1 included."""
    recs = [r for r in bdls_golden if r["curve"] == curve]
    arrs = pack_bdls(recs)
    out = np.zeros(len(recs), np.uint8)
    hs.hs_set_ll(ll)
    try:
        hs.hs_verify_bdls(CURVE_ID[curve], *[a.ctypes.data for a in arrs], len(recs), min_uses,
                          out.ctypes.data)
    finally:
        hs.hs_set_ll(0)
    bad = [(r["tag"], int(o), r["reason"]) for r, o in zip(recs, out) if o != r["reason"]]
    assert not bad


def _k1_edge_records(comb_shape=(7, 37)):
    """secp256k1 digest-level edge cases (x wrap, infinity, internal doubling,
    GLV split edges, signed-comb edges)."""
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
    # GLV split edges (verify.h q_ladder_glv): valid signatures built for a
    # chosen u2 -- R = u1 G + u2 Q, r = x(R) mod n, s = r / u2, e = u1 s
    lam = 0x5363AD4CC05C30E0A5261C028812645A122E22EA20816678DF02967C1B23BD72
    n = c.n
    u2s = [1, 2, 3, 15, 16, 17, 31, 32, 33, lam, n - lam, lam * lam % n, 2**127, 2**128 - 1,
           2**128, 2**128 + 1, n - 1, n - 2, n // 2, n // 2 + 1, (2**128 * lam) % n,
           (12345 * lam) % n, (n - 12345 * lam % n) % n, (2**64 + 5 * lam) % n]
    u2s += [rng.randrange(1, n) for _ in range(8)] + [rng.randrange(1, 2**128) for _ in range(4)]
    # the signed comb's edges for the shape the harness was built with
    from tests.comb_cases import signed_comb_u2
    u2s += signed_comb_u2(n, *comb_shape)
    for u2 in u2s:
        u1 = rng.randrange(1, n)
        R = O.point_add(c, O.scalar_mult(c, u1, (c.gx, c.gy)), O.scalar_mult(c, u2, (qx, qy)))
        if R is None or R[0] % n == 0:
            continue
        r = R[0] % n
        s = r * pow(u2, -1, n) % n
        e = u1 * s % n
        add("k1_glv_u2", qx, qy, r, s, e.to_bytes(32, "big"))
        add("k1_glv_u2_flip", qx, qy, r, s, (e ^ 1).to_bytes(32, "big"))
    for _ in range(6):  # plain valid / invalid, high-S accepted (no low-S rule)
        msgd = bytes(rng.getrandbits(8) for _ in range(32))
        r, s = O.sign_digest(c, d, msgd, rng.randrange(1, c.n), low_s=False)
        add("k1_valid", qx, qy, r, s, msgd)
        add("k1_flip", qx, qy, r, s, bytes([msgd[0] ^ 1]) + msgd[1:])
    return recs


@pytest.mark.parametrize("min_uses,wide,ll", [(1, 1, 0), (1000, 1, 0), (1, 16, 0), (1, 4, 0),
                                              (1000, 4, 0), (1, 1, 1)])
def test_k1_curve_edges_hostsim(hs, min_uses, wide, ll):
    """ll = 1: the signed Lim-Lee comb tables over secp256k1."""
    sh = hs.hs_ll_shape()
    recs = _k1_edge_records((sh >> 8, sh & 0xFF))
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
    hs.hs_set_wide(wide)
    hs.hs_set_ll(ll)
    try:
        hs.hs_verify_k1_digest(pub.ctypes.data, sig.ctypes.data, so.ctypes.data, sl.ctypes.data,
                               dg.ctypes.data, do.ctypes.data, dl.ctypes.data, len(recs),
                               min_uses, out.ctypes.data)
    finally:
        hs.hs_set_wide(1)
        hs.hs_set_ll(0)
    bad = [(t[0], int(o), t[5]) for t, o in zip(recs, out) if o != t[5]]
    assert not bad
    assert any(t[0] == "k1_xwrap_accept" and t[5] == 0 for t in recs)
    assert sum(t[0] == "k1_glv_u2" and t[5] == 0 for t in recs) >= 30


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


def _round_records(b, idx):
    out = []
    for i in idx:
        xy = bytes(b.xy[64 * i:64 * i + 64])
        out.append(dict(x=xy[:32], y=xy[32:],
                        r=bytes(b.r[b.r_off[i]:b.r_off[i] + b.r_len[i]]),
                        s=bytes(b.s[b.s_off[i]:b.s_off[i] + b.s_len[i]]),
                        msg=bytes(b.msg[b.msg_off[i]:b.msg_off[i] + b.msg_len[i]]),
                        version=int(b.version[i])))
    return out


@pytest.mark.parametrize("curve", [1, 0])
def test_bdls_round_generator_vs_oracle(curve):
    """gen.c's round (BASELINE config 4): structure and signatures, checked on
    the lock/decide records, first/last votes and a proof copy."""
    from bdls_amd.workload import generate_bdls_round
    b = generate_bdls_round(nval=10, curve=curve, small_len=50, seed=7)
    t2p1 = 2 * 3 + 1
    assert b.n == 2 * 10 + 2 * (1 + t2p1)
    c = O.SECP256K1 if curve == 1 else O.P256
    lock, decide = 10, 10 + 1 + t2p1 + 10
    recs = _round_records(b, [0, 9, lock, lock + 1, decide, b.n - 1])
    for rec in recs:
        dg = O.bdls_signed_proto_hash(rec["version"], rec["x"], rec["y"], rec["msg"])
        rc = O.go_ecdsa_verify(c, int.from_bytes(rec["x"], "big"), int.from_bytes(rec["y"], "big"),
                               dg, int.from_bytes(rec["r"], "big"), int.from_bytes(rec["s"], "big"))
        assert rc == O.R_OK
    assert recs[3] == _round_records(b, [0])[0]  # proof re-verifies roundchange 0
    assert recs[2]["x"] == recs[0]["x"]          # leader signs <lock>
    assert len(recs[2]["msg"]) > t2p1 * 50


@pytest.mark.parametrize("curve", [1, 0])
def test_bdls_round_hostsim(hs, curve):
    from bdls_amd.workload import generate_bdls_round
    b = generate_bdls_round(nval=16, curve=curve, small_len=120, seed=3)
    out = np.full(b.n, 255, np.uint8)
    hs.hs_verify_bdls(curve, *[a.ctypes.data for a in b.arrays()], b.n, 1000, out.ctypes.data)
    assert not out.any()


@pytest.mark.gpu
@pytest.mark.parametrize("curve", [1, 0])
def test_bdls_round_gpu(curve):
    from bdls_amd import _lib
    from bdls_amd.workload import generate_bdls_round
    _lib.ensure_init()
    b = generate_bdls_round(nval=100, curve=curve, seed=11)
    bitmap = np.zeros((b.n + 7) // 8, np.uint8)
    reason = np.full(b.n, 255, np.uint8)
    bb = _lib.BhBdlsBatch(*[a.ctypes.data for a in b.arrays()])
    _lib.check(_lib.lib().bh_verify_bdls(curve, ctypes.byref(bb), b.n, bitmap.ctypes.data,
                                         reason.ctypes.data))
    assert not reason.any()
    assert np.unpackbits(bitmap, bitorder="little")[:b.n].all()
    # a flipped message byte in the <decide> record is rejected, nothing else changes
    t2p1 = 2 * 33 + 1
    dec = 100 + 1 + t2p1 + 100
    b.msg[b.msg_off[dec] + 5] ^= 0x40
    _lib.check(_lib.lib().bh_verify_bdls(curve, ctypes.byref(bb), b.n, bitmap.ctypes.data,
                                         reason.ctypes.data))
    assert reason[dec] == 9 and np.count_nonzero(reason) == 1


def test_c_oracle_bdls_golden(bdls_golden):
    """oracle/orc.c's BDLS hash + verify against the golden set."""
    from oracle import orc
    for curve in ("secp256k1", "P-256"):
        recs = [r for r in bdls_golden if r["curve"] == curve]
        for r in recs[:20]:
            assert orc.bdls_hash(r["version"], bytes.fromhex(r["x"] + r["y"]),
                                 bytes.fromhex(r["msg"])).hex() == r["digest"]
        got = orc.bdls_verify(CURVE_ID[curve], *pack_bdls(recs))
        bad = [(r["tag"], int(g), r["reason"]) for r, g in zip(recs, got)
               if g != r["reason"] and not (r["reason"] == 7 and g == 9)]
        assert not bad


@pytest.mark.gpu
@pytest.mark.parametrize("curve", ["secp256k1", "P-256"])
@pytest.mark.parametrize("reps", [60, 80])
def test_bdls_gpu_mixed_wide(bdls_golden, curve, reps):
    """Batches below chip size (16 lanes per record at <= 8,192 records, 4 at
    <= 32,768): the golden set repeated (its 4 keys get per-batch key tables)
    plus a generated 100-validator round (keys used 2-4 times: ladder and key
    table records mixed). Runs the split kernels -- u2 Q halves while the
    BLAKE2b digests are hashed on the second stream, u1 G halves after -- and,
    at 4 lanes, the 2-slots-per-record Q tables of the 2-lane ladder."""
    from bdls_amd import _lib
    from bdls_amd.workload import generate_bdls_round
    _lib.ensure_init()
    gold = [r for r in bdls_golden if r["curve"] == curve]
    rb = generate_bdls_round(nval=100, curve=CURVE_ID[curve], seed=23)
    rnd = [dict(x=d["x"].hex(), y=d["y"].hex(), r=d["r"].hex(), s=d["s"].hex(),
                msg=d["msg"].hex(), version=d["version"])
           for d in _round_records(rb, range(rb.n))]
    recs = gold * reps + rnd
    n = len(recs)
    assert (n <= 8192) == (reps == 60) and n <= 32768
    arrs = pack_bdls(recs)
    bitmap = np.zeros((n + 7) // 8, np.uint8)
    reason = np.full(n, 255, np.uint8)
    b = _lib.BhBdlsBatch(*[a.ctypes.data for a in arrs])
    _lib.check(_lib.lib().bh_verify_bdls(CURVE_ID[curve], ctypes.byref(b), n,
                                         bitmap.ctypes.data, reason.ctypes.data))
    want = [r["reason"] for r in gold] * reps + [0] * rb.n
    bad = [(k, int(g), w) for k, (g, w) in enumerate(zip(reason, want)) if g != w]
    assert not bad[:10]
    valid = np.unpackbits(bitmap, bitorder="little")[:n].astype(bool)
    assert (valid == (np.array(want) == 0)).all()
