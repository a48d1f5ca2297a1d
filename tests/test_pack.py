"""Staged BatchVerify packing (bdls_amd/csrc/pack.h) on
the CPU through the host harness (tests/native/hostsim.cpp hs_pack): the
compact layout the library uploads -- distinct keys + u32 indices (or one key
per record), lengths, contiguous signature and message bytes in chunks whose
callbacks fire only when complete -- reconstructs every caller record exactly,
for shared, unique, skewed (table rebuild) and ragged batches, any thread
count, with and without de-duplication."""
import ctypes
import os

import numpy as np
import pytest

from bdls_amd import workload

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tests", "native", "build", "libhostsim.so")


@pytest.fixture(scope="module")
def hs():
    if not os.path.exists(LIB):
        pytest.skip("hostsim not built (make)")
    L = ctypes.CDLL(LIB)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    L.hs_pack.argtypes = [vp] * 7 + [sz, sz, ctypes.c_int, ctypes.c_int] + [vp] * 8
    L.hs_pack.restype = ctypes.c_int
    L.hs_estimate_distinct.argtypes = [sz, sz]
    L.hs_estimate_distinct.restype = ctypes.c_double
    return L


def _soa(pub, sigs, msgs):
    sl = np.array([len(x) for x in sigs], np.uint32)
    ml = np.array([len(x) for x in msgs], np.uint32)
    so = np.zeros(len(sigs), np.uint64)
    mo = np.zeros(len(msgs), np.uint64)
    so[1:] = np.cumsum(sl[:-1])
    mo[1:] = np.cumsum(ml[:-1])
    sig = np.frombuffer(b"".join(sigs) + b"\0", np.uint8)
    msg = np.frombuffer(b"".join(msgs) + b"\0", np.uint8)
    return np.ascontiguousarray(pub, np.uint8), sig, so, sl, msg, mo, ml


def pack(hs, arrs, lo, m, threads, force=-1):
    pub, sig, so, sl, msg, mo, ml = arrs
    keys = np.zeros(max(1, m) * 64, np.uint8)
    kidx = np.full(max(1, m), 0xFFFFFFFF, np.uint32)
    slen = np.zeros(max(1, m), np.uint32)
    mlen = np.zeros(max(1, m), np.uint32)
    sbytes = int(sl[lo:lo + m].sum())
    mbytes = int(ml[lo:lo + m].sum())
    sout = np.zeros(sbytes + 1, np.uint8)
    mout = np.zeros(mbytes + 1, np.uint8)
    info = np.zeros(10, np.uint64)
    bounds = np.zeros(2 * 65 + 2, np.uint64)
    rc = hs.hs_pack(*[x.ctypes.data for x in (pub, sig, so, sl, msg, mo, ml)], lo, m, threads,
                    force, keys.ctypes.data, kidx.ctypes.data, slen.ctypes.data, mlen.ctypes.data,
                    sout.ctypes.data, mout.ctypes.data, info.ctypes.data, bounds.ctypes.data)
    assert rc == 0, "a chunk callback fired early or out of order"
    nkeys, dedup, fixed, stride, sb, mb, K, rebuilds = (int(x) for x in info[:8])
    assert (sb, mb) == (sbytes, mbytes)
    # reconstruct every record
    for i in range(m):
        k = keys[64 * kidx[i]:64 * kidx[i] + 64] if dedup else keys[64 * i:64 * i + 64]
        assert (k == pub[64 * (lo + i):64 * (lo + i) + 64]).all(), i
    assert (slen[:m] == sl[lo:lo + m]).all() and (mlen[:m] == ml[lo:lo + m]).all()
    want_s = b"".join(bytes(sig[int(so[i]):int(so[i]) + int(sl[i])]) for i in range(lo, lo + m))
    want_m = b"".join(bytes(msg[int(mo[i]):int(mo[i]) + int(ml[i])]) for i in range(lo, lo + m))
    assert bytes(sout[:sbytes]) == want_s and bytes(mout[:mbytes]) == want_m
    if dedup:
        # ids come in per-thread blocks: the key array may hold a few zero holes
        distinct = len({bytes(pub[64 * i:64 * i + 64]) for i in range(lo, lo + m)})
        assert distinct <= nkeys <= distinct + threads * 64
        assert (kidx[:m] < nkeys).all()
        used = np.zeros(nkeys, bool)
        used[kidx[:m]] = True
        assert not keys[:64 * nkeys].reshape(-1, 64)[~used].any()  # holes are zero
    else:
        assert nkeys == m
    assert fixed == int(m > 0 and ml[lo:lo + m].min() == ml[lo:lo + m].max())
    sbnd, mbnd = bounds[:K + 1], bounds[K + 1:2 * K + 2]
    assert sbnd[0] == 0 and sbnd[-1] == sbytes and (np.diff(sbnd.astype(np.int64)) >= 0).all()
    assert mbnd[0] == 0 and mbnd[-1] == mbytes
    return dict(nkeys=nkeys, dedup=dedup, fixed=fixed, stride=stride, chunks=K, rebuilds=rebuilds)


@pytest.fixture(scope="module")
def cfg2_like():
    w = workload.generate(20_000, 500, 256, 16, seed=7, nthreads=4)
    return w.arrays()


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_pack_shared_keys(hs, cfg2_like, threads):
    pub, sig, so, sl, msg, mo, ml = cfg2_like
    arrs = (pub, sig, so, sl, msg, mo, ml)
    r = pack(hs, arrs, 0, 20_000, threads)
    assert r["dedup"] and 500 <= r["nkeys"] < 1_500 and r["fixed"] and r["stride"] == 256
    assert r["rebuilds"] == 0
    r = pack(hs, arrs, 1_000, 7_000, threads)  # a shard in the middle
    assert r["dedup"]
    r = pack(hs, arrs, 0, 20_000, threads, force=0)  # no dedup: one key per record
    assert not r["dedup"]


def test_pack_unique_keys_skip_dedup(hs):
    w = workload.generate(12_000, 12_000, 64, 16, seed=8, nthreads=4)
    r = pack(hs, w.arrays(), 0, w.n, 4)
    assert not r["dedup"] and r["nkeys"] == w.n  # config 5's shape: nothing to dedup
    r = pack(hs, w.arrays(), 0, w.n, 4, force=1)
    assert r["dedup"] and r["nkeys"] <= w.n


def test_pack_skewed_keys_rebuild(hs):
    """Half the records on one hot key, the rest unique: the sample sees a
    small key population, the table fills, and is rebuilt at full size --
    the packed batch is still exact."""
    rng = np.random.default_rng(9)
    m = 60_000
    pub = rng.integers(0, 256, (m, 64), dtype=np.uint8)
    pub[::2] = pub[0]
    sigs = [bytes(rng.integers(0, 256, int(rng.integers(0, 80)), dtype=np.uint8)) for _ in range(m)]
    msgs = [bytes(rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8))
            for _ in range(m)]
    arrs = _soa(pub.reshape(-1), sigs, msgs)
    r = pack(hs, arrs, 0, m, 6)
    assert r["dedup"] and r["rebuilds"] == 1 and m // 2 + 1 <= r["nkeys"] <= m // 2 + 1 + 6 * 64
    assert not r["fixed"]


@pytest.mark.parametrize("m", [0, 1, 2, 63, 64, 65, 1000])
def test_pack_ragged_small(hs, m):
    rng = np.random.default_rng(m)
    pub = rng.integers(0, 256, (max(m, 1), 64), dtype=np.uint8)
    if m > 4:
        pub[3] = pub[1]
    sigs = [b"" if i % 7 == 0 else bytes(rng.integers(0, 256, 71, dtype=np.uint8))
            for i in range(max(m, 1))]
    msgs = [bytes(rng.integers(0, 256, 32, dtype=np.uint8)) for _ in range(max(m, 1))]
    arrs = _soa(pub.reshape(-1), sigs, msgs)
    for t in (1, 5):
        for force in (-1, 0, 1):
            pack(hs, arrs, 0, m, t, force)


def test_pack_many_chunks(hs, cfg2_like, monkeypatch):
    """BH_PACK_CHUNKS forces the chunked copy (the H2D stream of pass B) at a
    small size: every chunk callback sees its own records complete."""
    monkeypatch.setenv("BH_PACK_CHUNKS", "7")
    r = pack(hs, cfg2_like, 0, 20_000, 5)
    assert r["chunks"] == 7


def test_estimate_distinct(hs):
    # D (1 - e^(-s/D)) inverted: a uniform draw of s from D keys
    for D in (10, 1_000, 65_536, 1_000_000):
        s = 8192
        ds = D * (1 - np.exp(-s / D))
        est = hs.hs_estimate_distinct(s, int(round(ds)))
        assert abs(est - D) / D < 0.05 or (D > 200_000 and est > 200_000), (D, est)
    assert hs.hs_estimate_distinct(8192, 8192) == 0.0  # no repeat seen
