"""GPU: the one-lane-per-record key-table route -- the signed Lim-Lee comb
tables (verify.h lltab_build / q_llcomb, k_ktab_ladder + k_keycomb) that every
batch above 32,768 records takes -- on the crafted edge cases, not only on
generator signatures (VERDICT r3 missing #4 / weak #1), and config 5's
per-rank pass shape (VERDICT r3 missing #1).

  * P-256: the golden records (x-wrap, u1 G + u2 Q = infinity, u1 G == u2 Q,
    r / s boundaries, DER rejects, the real mspid CA signatures, ...) and
    signatures built for the comb's own edge scalars (tests/comb_cases.py:
    odd / even u2, empty and full columns, negated top tooth, the Horner
    doubling branch) plus the key-table window edges, every key used >= 4
    times, in a 40k+ batch with generator filler: bitmap and reasons equal the
    golden / constructed ones, and every record that reaches the group
    equation went through the comb (n_keycomb), with BH_LL=1 and BH_LL=0.
  * secp256k1: a BDLS batch above 32,768 records (golden x 280 +
    a generated round) through the comb tables and through BH_LL=0's windowed
    tables, record by record.
  * 4,194,304 unique keys in one pass: the ladder's Q-table scratch at the
    pass size a config-5 rank runs.
Reference predicate: bccsp/sw/ecdsa.go:41-57 -> Go 1.21 crypto/ecdsa verifyNISTEC.
"""
import ctypes
import hashlib
import os

import numpy as np
import pytest

from bdls_amd import _lib, workload
from oracle import ecdsa_ref as O
from oracle import orc
from tests.comb_cases import (fold_crafted, g_comb_u1, records_for_fold, records_for_u2,
                              signed_comb_u2, unsigned_comb_u2)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    _lib.ensure_init()
    return _lib.lib()


def _window_edge_u2(n):
    return [1, 7, 8, 9, 15, 16, 17, 0x88, 0x8888, 0x7777, 2**252, 2**256 - n, n - 1, n - 2,
            n // 2, n // 2 + 1, (16**64 - 1) % n, sum(8 * 16**k for k in range(64)) % n]


def _pack(recs):
    """[(pub64, sig, digest)] -> bh_batch arrays (digest mode)."""
    pub = np.frombuffer(b"".join(r[0] for r in recs), np.uint8)
    sl = np.array([len(r[1]) for r in recs], np.uint32)
    dl = np.array([len(r[2]) for r in recs], np.uint32)
    so = np.zeros(len(recs), np.uint64)
    do = np.zeros(len(recs), np.uint64)
    so[1:] = np.cumsum(sl[:-1])
    do[1:] = np.cumsum(dl[:-1])
    sig = np.frombuffer(b"".join(r[1] for r in recs) + b"\0", np.uint8)
    dg = np.frombuffer(b"".join(r[2] for r in recs) + b"\0", np.uint8)
    return pub, sig, so, sl, dg, do, dl


def _dev_verify(L, arrs, n, flags=0, curve=0):
    DA = _lib.DeviceArray
    d = [DA.from_numpy(0, x) for x in arrs]
    words = DA(0, ((n + 63) // 64) * 8)
    reason = DA(0, n)
    tm = _lib.BhTiming()
    b = _lib.BhBatch(*[x.ptr for x in d])
    _lib.check(L.bh_verify_dev(0, curve, ctypes.byref(b), n, flags, words.ptr, reason.ptr, None,
                               1, ctypes.byref(tm)))
    bits = np.unpackbits(words.to_numpy(np.uint64, (n + 63) // 64).view(np.uint8),
                         bitorder="little")[:n].astype(bool)
    out = bits, reason.to_numpy(np.uint8, n), tm
    for x in d + [words, reason]:
        x.free()
    return out


@pytest.fixture(scope="module")
def p256_edge_batch(golden):
    """(arrays, expected reasons): golden x 4 + crafted comb / window records x 4
    + digest-mode generator filler, >= 40,000 records."""
    recs, want = [], []
    for r in golden:  # every golden key used 4 times
        for _ in range(4):
            recs.append((bytes.fromhex(r["qx"] + r["qy"]), bytes.fromhex(r["sig"]),
                         bytes.fromhex(r["digest"])))
            want.append(r["reason"])
    c = O.P256
    u2s = signed_comb_u2(c.n, 7, 37) + signed_comb_u2(c.n, 6, 43) + unsigned_comb_u2(6, 43) \
        + _window_edge_u2(c.n)
    crafted = records_for_u2(c, u2s, seed=91, low_s=True)
    assert len(crafted) >= 2 * 60
    # the u1 G comb's edges (zero digits, most negative digit, carries) at
    # every window width the library may be built with
    import random
    u1s = [u for gw in (10, 11, 12, 13, 14) for u in g_comb_u1(c.n, gw)]
    rng = random.Random(5)
    crafted += records_for_u2(c, [rng.randrange(1, c.n) for _ in u1s], seed=92, low_s=True,
                              u1s=u1s)
    for qx, qy, sig, dg in crafted:
        for _ in range(4):
            recs.append((qx.to_bytes(32, "big") + qy.to_bytes(32, "big"), sig, dg))
    for k in range(len(crafted)):  # valid signature, then its flipped-digest twin
        want += [0 if k % 2 == 0 else 9] * 4
    # round 5: the folded u1 G (k_keycomb's q_llcomb_g) on records whose joint
    # Horner takes each degenerate branch (tests/comb_cases.py fold_crafted)
    kgf = int(os.environ.get("BH_GFOLD", 3))  # the library's G group size (verify.h kGF)
    fold = records_for_fold(c, fold_crafted(c, 7, 37, seed=33, low_s=True, kgf=kgf), low_s=True)
    assert len(fold) >= 13
    for qx, qy, sig, dg, exp in fold:
        for _ in range(4):
            recs.append((qx.to_bytes(32, "big") + qy.to_bytes(32, "big"), sig, dg))
            want.append(exp)
    fill = 40_960 - len(recs)
    w = workload.generate(fill, fill // 64, 64, 16, seed=47)  # ~64 uses per key
    for i in range(w.n):
        m = bytes(w.msg[w.msg_off[i]:w.msg_off[i] + w.msg_len[i]])
        recs.append((bytes(w.pub[64 * i:64 * i + 64]),
                     bytes(w.sig[w.sig_off[i]:w.sig_off[i] + w.sig_len[i]]),
                     hashlib.sha256(m).digest()))
    want += [int(x) for x in w.reason]
    # the filler's reasons in digest mode, on a sample, against the C oracle
    rng = np.random.default_rng(3)
    base = len(recs) - w.n
    for i in rng.choice(w.n, 100, replace=False):
        q, s, dg = recs[base + i]
        assert orc.csp_verify(q, s, dg) == want[base + i]
    return _pack(recs), np.array(want, np.uint8)


@pytest.mark.parametrize("ll", ["1", "0"])
def test_comb_route_edge_cases_p256(L, p256_edge_batch, ll):
    (arrs, want) = p256_edge_batch
    n = len(want)
    assert n >= 40_000
    os.environ["BH_LL"] = ll
    try:
        bits, reason, tm = _dev_verify(L, arrs, n)
    finally:
        del os.environ["BH_LL"]
    bad = np.nonzero(reason != want)[0]
    assert not len(bad), [(int(i), int(reason[i]), int(want[i])) for i in bad[:10]]
    assert (bits == (want == 0)).all()
    # one lane per record, and every record that reaches the group equation
    # (verdict 0 or R_MATH) went through the key tables
    assert tm.wide == 1
    assert tm.n_keycomb == int(((want == 0) | (want == 9)).sum()) and tm.n_ladder == 0
    assert tm.n_keytables >= 20 + 0.9 * ((n - 4 * 359 - 480) // 64)


def test_comb_and_windows_agree_k1_bdls(L):
    """secp256k1 BDLS batch above 32,768 records: the signed comb tables
    (default) and the windowed tables (BH_LL=0) give the expected verdict on
    every record (lltab_build<F30_k1> / q_llcomb<F30_k1> on device)."""
    import json
    from tests.bdls_util import pack_bdls
    from tests.conftest import ROOT
    from tests.test_bdls import _round_records
    with open(os.path.join(ROOT, "tests", "golden", "bdls_vectors.jsonl")) as f:
        gold = [r for r in map(json.loads, f) if r["curve"] == "secp256k1"]
    rb = workload.generate_bdls_round(nval=100, curve=1, seed=29)
    rnd = [dict(x=d["x"].hex(), y=d["y"].hex(), r=d["r"].hex(), s=d["s"].hex(),
                msg=d["msg"].hex(), version=d["version"]) for d in _round_records(rb, range(rb.n))]
    reps = 280
    recs = gold * reps + rnd
    n = len(recs)
    assert n > 32_768
    arrs = pack_bdls(recs)
    want = np.array([r["reason"] for r in gold] * reps + [0] * rb.n, np.uint8)
    DA = _lib.DeviceArray
    got = {}
    for ll in ("1", "0"):
        d = [DA.from_numpy(0, x) for x in arrs]
        words = DA(0, ((n + 63) // 64) * 8)
        reason = DA(0, n)
        tm = _lib.BhTiming()
        b = _lib.BhBdlsBatch(*[x.ptr for x in d])
        os.environ["BH_LL"] = ll
        try:
            _lib.check(L.bh_verify_bdls_dev(0, 1, ctypes.byref(b), n, words.ptr, reason.ptr, None,
                                            1, ctypes.byref(tm)))
        finally:
            del os.environ["BH_LL"]
        got[ll] = (reason.to_numpy(np.uint8, n), tm.n_keycomb, tm.n_keytables, tm.wide)
        for x in d + [words, reason]:
            x.free()
    for ll, (reason, ncomb, ntab, wide) in got.items():
        bad = np.nonzero(reason != want)[0]
        assert not len(bad), (ll, [(int(i), int(reason[i]), int(want[i])) for i in bad[:10]])
        assert wide == 1 and ntab > 0 and ncomb > 0.9 * int(((want == 0) | (want == 9)).sum())


def test_unique_keys_one_pass_of_4m(L):
    """Config 5's per-rank pass: 4,194,304 records with a distinct key each in
    ONE pass of the pass loop (the variable-base ladder's Q-table scratch at
    1,792 B x 4M = 7.5 GB), checked against construction and a 200-record
    sample of the C oracle."""
    n = 1 << 22
    w = workload.generate(n, n, 64, 16, seed=48)
    arrs = w.arrays()
    bits, reason, tm = _dev_verify(L, arrs, n, flags=_lib.BH_F_HASH_SHA256)
    assert (reason == w.reason).all() and (bits == w.expected_valid).all()
    assert tm.n_keycomb == 0 and tm.n_keytables == 0
    assert tm.n_ladder == int(((w.reason == 0) | (w.reason == 9)).sum())
    idx = np.random.default_rng(4).choice(n, 200, replace=False)
    for i in idx:
        q = bytes(w.pub[64 * i:64 * i + 64])
        s = bytes(w.sig[w.sig_off[i]:w.sig_off[i] + w.sig_len[i]])
        dg = hashlib.sha256(bytes(w.msg[w.msg_off[i]:w.msg_off[i] + w.msg_len[i]])).digest()
        assert orc.csp_verify(q, s, dg) == w.reason[i], i


@pytest.mark.parametrize("route", ["default", "noreg", "ladder"])
def test_ladder_route_crafted_events_p256(L, golden, route):
    """The one-lane P-256 ladder (verify.h q_ladder_odd_g: odd signed windows,
    the composite 2 A + T, u1 G folded into the last doublings) on records
    crafted so that its last window takes every degenerate branch reachable
    by construction (tests/comb_cases.py ladder_crafted, one key per event),
    plus the golden file's x-wrap / infinity / u1 G == u2 Q classes rebuilt on
    a fresh key each (comb_cases.distinct_key_classes), in a > 32,768-record
    batch of distinct keys: bitmap and reasons equal the construction (and
    the C oracle), and EVERY record that reaches the group equation ran on
    the ladder. route: "default" routing, "noreg"
    (BH_ROUTE: no registry lookup), "ladder" (no registry, no per-batch
    tables), the last also carrying every golden record on its shared keys."""
    from tests.comb_cases import distinct_key_classes, ladder_crafted
    c = O.P256
    kgf = int(os.environ.get("BH_GFOLD", 3))
    recs, want = [], []
    for seed in (43, 44, 45):
        trip = ladder_crafted(c, seed=seed, low_s=True, kgf=kgf)
        assert len(trip) == 9 and len({t[2] for t in trip}) == 9
        for qx, qy, sig, dg, exp in records_for_fold(c, trip, low_s=True):
            recs.append((qx.to_bytes(32, "big") + qy.to_bytes(32, "big"), sig, dg))
            want.append(exp)
    assert len(recs) >= 3 * 9
    for qx, qy, sig, dg, exp, _tag in distinct_key_classes(c, seed=61, reps=4):
        recs.append((qx.to_bytes(32, "big") + qy.to_bytes(32, "big"), sig, dg))
        want.append(exp)
    # the crafted records against the C oracle as well
    assert all(orc.csp_verify(*r) == w for r, w in zip(recs, want))
    if route == "ladder":  # the golden records keep their shared keys
        for r in golden:
            recs.append((bytes.fromhex(r["qx"] + r["qy"]), bytes.fromhex(r["sig"]),
                         bytes.fromhex(r["digest"])))
            want.append(r["reason"])
    keys = [r[0] for r in recs]
    if route != "ladder":
        assert len(set(keys)) * 2 >= len(keys)  # <= 2 records per crafted key
    fill = 40_960 - len(recs)
    w = workload.generate(fill, fill, 64, 16, seed=49)  # distinct keys
    for i in range(w.n):
        m = bytes(w.msg[w.msg_off[i]:w.msg_off[i] + w.msg_len[i]])
        recs.append((bytes(w.pub[64 * i:64 * i + 64]),
                     bytes(w.sig[w.sig_off[i]:w.sig_off[i] + w.sig_len[i]]),
                     hashlib.sha256(m).digest()))
    want += [int(x) for x in w.reason]
    want = np.array(want, np.uint8)
    n = len(recs)
    assert n > 32_768
    if route != "default":
        os.environ["BH_ROUTE"] = route
    try:
        bits, reason, tm = _dev_verify(L, _pack(recs), n)
    finally:
        os.environ.pop("BH_ROUTE", None)
    bad = np.nonzero(reason != want)[0]
    assert not len(bad), [(int(i), int(reason[i]), int(want[i])) for i in bad[:10]]
    assert (bits == (want == 0)).all()
    math = int(((want == 0) | (want == 9)).sum())
    assert tm.wide == 1 and tm.n_keycomb == 0 and tm.n_keytables == 0
    assert tm.n_ladder == math
    base = n - w.n
    for i in np.random.default_rng(5).choice(w.n, 100, replace=False):
        q, s, dg = recs[base + i]
        assert orc.csp_verify(q, s, dg) == want[base + i]
