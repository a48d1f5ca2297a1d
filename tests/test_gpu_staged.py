"""GPU: the staged BatchVerify (bh_batch_verify*, bdls_amd/csrc/pack.h; VERDICT
r5 next #2) -- BatchVerify straight from the caller's pageable, per-record
buffers, packed by the library into its own page-locked staging (key
de-duplication, lengths, chunked signature / message bytes whose H2D starts
while the next chunk packs). Bit-exact bar: bitmap AND reason equal the
construction (the generator's expected reasons, confirmed on samples against
oracle/orc.c) and the golden records' Go-derived reasons, for both input forms
(SoA bh_batch and per-record pointers bh_pbatch), shared / unique keys, NULL
fields, the latency path, several shards, and submit/wait pipelines whose
caller buffers are overwritten as soon as submit returns (everything is copied
by then). Reference batch points: common/policies/policy.go:363-395,
core/committer/txvalidator/v20/validator.go:193-208."""
import ctypes
import hashlib
import os

import numpy as np
import pytest

from bdls_amd import _lib, workload
from oracle import orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L():
    _lib.ensure_init()
    return _lib.lib()


def _bits(bm, n):
    return np.unpackbits(bm, bitorder="little")[:n].astype(bool)


def staged(L, arrs, n, flags=_lib.BH_F_HASH_SHA256):
    bm = np.zeros((n + 7) // 8 or 1, np.uint8)
    rs = np.zeros(n or 1, np.uint8)
    b = _lib.BhBatch(*[x.ctypes.data for x in arrs])
    _lib.check(L.bh_batch_verify(0, ctypes.byref(b), n, flags, bm.ctypes.data, rs.ctypes.data))
    return _bits(bm, n), rs[:n]


def ptr_form(arrs, n, null_sig=(), null_msg=(), null_key=()):
    """bh_pbatch arrays over a SoA batch: per-record addresses (NULL where asked)."""
    pub, sig, so, sl, msg, mo, ml = arrs
    kp = (pub.ctypes.data + 64 * np.arange(n, dtype=np.uint64)).astype(np.uint64)
    sp = (sig.ctypes.data + so[:n]).astype(np.uint64)
    mp = (msg.ctypes.data + mo[:n]).astype(np.uint64)
    sp[list(null_sig)] = 0
    mp[list(null_msg)] = 0
    kp[list(null_key)] = 0
    return kp, sp, np.ascontiguousarray(sl[:n]), mp, np.ascontiguousarray(ml[:n])


def staged_ptrs(L, parr, n, flags=_lib.BH_F_HASH_SHA256):
    bm = np.zeros((n + 7) // 8 or 1, np.uint8)
    rs = np.zeros(n or 1, np.uint8)
    b = _lib.BhPBatch(*[x.ctypes.data for x in parr])
    _lib.check(L.bh_batch_verify_ptrs(0, ctypes.byref(b), n, flags, bm.ctypes.data,
                                      rs.ctypes.data))
    return _bits(bm, n), rs[:n]


@pytest.fixture(scope="module")
def shared():
    return workload.generate(150_000, 3_000, 256, 16, seed=71)


def test_staged_shared_keys_soa(L, shared):
    w = shared
    bits, rs = staged(L, w.arrays(), w.n)
    assert (rs == w.reason).all() and (bits == w.expected_valid).all()
    st = _lib.pack_stats()
    assert st["dedup"] == 1 and st["records"] == w.n and st["nkeys"] < 2 * 3_000
    assert st["threads"] >= 1 and st["chunks"] >= 1


def test_staged_pointer_form_with_nulls(L, shared):
    w = shared
    n = w.n
    nul_s, nul_m, nul_k = [5, 77, 1000], [6, 78], [7, 79]
    parr = ptr_form(w.arrays(), n, nul_s, nul_m, nul_k)
    bits, rs = staged_ptrs(L, parr, n)
    want = w.reason.copy()
    want[nul_s] = 1  # BH_R_EMPTY_SIG (a nil signature)
    want[nul_k] = 7  # BH_R_BAD_KEY (the all-zero point)
    # a nil message is hashed as the empty message: the signature over the
    # real message fails the group equation (unless prep rejected it first)
    for i in nul_m:
        want[i] = 9 if w.reason[i] in (0, 9) else w.reason[i]
    assert (rs == want).all(), [(int(i), int(rs[i]), int(want[i]))
                                for i in np.nonzero(rs != want)[0][:10]]
    assert (bits == (want == 0)).all()


def test_staged_golden_digest_mode(L, golden):
    """Every golden record (Go-derived reasons: DER rejects, x-wrap, infinity,
    boundaries, the mspid CA signatures) through both staged forms."""
    from tests.conftest import pack
    arrs = pack(golden, False)
    n = len(golden)
    want = np.array([r["reason"] for r in golden], np.uint8)
    for form in ("soa", "ptrs"):
        if form == "soa":
            bits, rs = staged(L, arrs, n, 0)
        else:
            bits, rs = staged_ptrs(L, ptr_form(arrs, n), n, 0)
        assert (rs == want).all(), (form, np.nonzero(rs != want)[0][:10])
        assert (bits == (want == 0)).all()
    # a nil digest in digest mode: BH_R_EMPTY_DIGEST
    bits, rs = staged_ptrs(L, ptr_form(arrs, n, null_msg=[0, 1]), n, 0)
    assert rs[0] == 2 and rs[1] == 2 and (rs[2:] == want[2:]).all()


def test_staged_unique_keys_and_sample(L):
    w = workload.generate(70_000, 70_000, 256, 16, seed=72)
    bits, rs = staged(L, w.arrays(), w.n)
    assert (rs == w.reason).all() and (bits == w.expected_valid).all()
    assert _lib.pack_stats()["dedup"] == 0
    for i in np.random.default_rng(1).choice(w.n, 50, replace=False):
        q = bytes(w.pub[64 * i:64 * i + 64])
        s = bytes(w.sig[w.sig_off[i]:w.sig_off[i] + w.sig_len[i]])
        dg = hashlib.sha256(bytes(w.msg[w.msg_off[i]:w.msg_off[i] + w.msg_len[i]])).digest()
        assert orc.csp_verify(q, s, dg) == w.reason[i]


@pytest.mark.parametrize("n", [1, 17, 256, 257])
def test_staged_small_batches(L, shared, n):
    """<= 256 records take the latency path (packed on the host by the same
    accessors); 257 the smallest staged pass."""
    w = shared
    lo = 999
    sub = [np.ascontiguousarray(x) for x in
           (w.pub[64 * lo:64 * (lo + n)], w.sig, w.sig_off[lo:lo + n], w.sig_len[lo:lo + n],
            w.msg, w.msg_off[lo:lo + n], w.msg_len[lo:lo + n])]
    for form in ("soa", "ptrs"):
        if form == "soa":
            bits, rs = staged(L, sub, n)
        else:
            bits, rs = staged_ptrs(L, ptr_form(sub, n), n)
        assert (rs == w.reason[lo:lo + n]).all(), form
        assert (bits == w.expected_valid[lo:lo + n]).all()


@pytest.mark.parametrize("shards", ["1", "2", "4"])
def test_staged_pipeline_buffers_reused(L, shards, monkeypatch):
    """Six batches through bh_batch_verify_submit, up to four in flight, the
    caller's buffers overwritten right after each submit returns (the staged
    path copies everything before returning); BH_HOST_SHARDS splits each
    batch into shards with their own slots, packs and bitmaps."""
    monkeypatch.setenv("BH_HOST_SHARDS", shards)
    ws = [workload.generate(40_000 + 1_000 * k, 400 + 300 * k, 256, 16, seed=80 + k)
          for k in range(3)]
    want = [(w.reason.copy(), w.expected_valid.copy()) for w in ws]
    scratch = [tuple(x.copy() for x in w.arrays()) for w in ws]
    jobs, outs = [], []
    for k in range(6):
        w = ws[k % 3]
        arrs = scratch[k % 3]
        for x, src in zip(arrs, w.arrays()):
            x[:] = src
        n = w.n
        bm = np.zeros((n + 7) // 8, np.uint8)
        rs = np.zeros(n, np.uint8)
        b = _lib.BhBatch(*[x.ctypes.data for x in arrs])
        job = ctypes.c_void_p()
        _lib.check(L.bh_batch_verify_submit(0, ctypes.byref(b), n, _lib.BH_F_HASH_SHA256,
                                            bm.ctypes.data, rs.ctypes.data, ctypes.byref(job)))
        for x in arrs:  # the caller reuses its buffers at once
            x[:] = 0xA5 if x.dtype == np.uint8 else 0
        jobs.append(job)
        outs.append((k % 3, bm, rs, n))
        if len(jobs) == 4:
            _lib.check(L.bh_verify_wait(jobs.pop(0)))
    while jobs:
        _lib.check(L.bh_verify_wait(jobs.pop(0)))
    for k, bm, rs, n in outs:
        assert (rs == want[k][0]).all() and (_bits(bm, n) == want[k][1]).all(), k


def test_staged_invalid_args(L):
    n = 10
    bm = np.zeros(2, np.uint8)
    rs = np.zeros(n, np.uint8)
    b = _lib.BhPBatch(0, 0, 0, 0, 0)
    assert L.bh_batch_verify_ptrs(0, ctypes.byref(b), n, 0, bm.ctypes.data, rs.ctypes.data) == -1
    assert L.bh_batch_verify(1, None, 0, 0, bm.ctypes.data, rs.ctypes.data) == -1  # curve
    b2 = _lib.BhBatch(0, 0, 0, 0, 0, 0, 0)
    assert L.bh_batch_verify(0, ctypes.byref(b2), 0, 0, bm.ctypes.data, rs.ctypes.data) == 0
