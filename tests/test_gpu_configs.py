"""GPU parity on the shapes BASELINE configs 3 and 5 actually hit, plus the
host-API pipeline (bh_verify_submit / bh_verify_wait, page-locked inputs).

Bit-exact bar as everywhere: bitmap AND per-record reason equal the expected
results (by construction, confirmed on samples against oracle/orc.c).
  * config 3: one block (generate_block: 500 creators over 4 KB + 1,500
    endorsements over 1.5 KB), cold (ladder) and warm (registered keys);
  * the multi-pass loop for batches above the 4M-record pass size
    (bdls_hip.cpp run_dev) at its real size, and forced on small batches with
    BH_MAX_CHUNK, with kept keys (registry ids mixed with per-batch ids in the
    key-sorted comb list);
  * the key-table overflow route: more than 65,536 keys used >= 4 times, so
    k_key_plan drops builds past max_tables and those records take the ladder.
"""
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


def host_verify(L, w, flags=_lib.BH_F_HASH_SHA256):
    n = w.n
    bm = np.zeros((n + 7) // 8 or 1, np.uint8)
    rs = np.zeros(n or 1, np.uint8)
    b = _lib.BhBatch(*[x.ctypes.data for x in w.arrays()])
    _lib.check(L.bh_verify(0, ctypes.byref(b), n, flags, bm.ctypes.data, rs.ctypes.data))
    return np.unpackbits(bm, bitorder="little")[:n].astype(bool), rs[:n]


def dev_verify(L, w, flags=_lib.BH_F_HASH_SHA256):
    DA = _lib.DeviceArray
    d = [DA.from_numpy(0, x) for x in w.arrays()]
    words = DA(0, ((w.n + 63) // 64) * 8)
    reason = DA(0, w.n)
    b = _lib.BhBatch(*[x.ptr for x in d])
    tm = _lib.BhTiming()
    _lib.check(L.bh_verify_dev(0, 0, ctypes.byref(b), w.n, flags, words.ptr, reason.ptr, None, 1,
                               ctypes.byref(tm)))
    bits = np.unpackbits(words.to_numpy(np.uint64, (w.n + 63) // 64).view(np.uint8),
                         bitorder="little")[:w.n].astype(bool)
    out = bits, reason.to_numpy(np.uint8, w.n), tm
    for x in d + [words, reason]:
        x.free()
    return out


def orc_sample(w, k, seed=0):
    idx = np.random.default_rng(seed).choice(w.n, k, replace=False)
    for i in idx:
        q = bytes(w.pub[64 * i:64 * i + 64])
        s = bytes(w.sig[w.sig_off[i]:w.sig_off[i] + w.sig_len[i]])
        dg = hashlib.sha256(bytes(w.msg[w.msg_off[i]:w.msg_off[i] + w.msg_len[i]])).digest()
        assert orc.csp_verify(q, s, dg) == w.reason[i], i


def test_config3_block_cold_and_warm(L):
    """BASELINE config 3 through the host ABI: cold (no key known: ladder) and
    warm (the block's 54 keys registered: key-table path)."""
    w = workload.generate_block(seed=3)
    assert w.n == 2000
    orc_sample(w, 300)
    _lib.check(L.bh_keys_clear(-1, 0))
    valid, reason = host_verify(L, w)
    assert (reason == w.reason).all() and (valid == w.expected_valid).all()
    _, dreason, tm = dev_verify(L, w)
    assert (dreason == w.reason).all() and tm.n_keycomb == 0
    pubs = np.unique(w.pub.reshape(-1, 64), axis=0)
    st = np.zeros(len(pubs), np.uint8)
    _lib.check(L.bh_keys_register(-1, 0, np.ascontiguousarray(pubs).ctypes.data, len(pubs),
                                  st.ctypes.data))
    # the off-curve / >= p corruptions are not valid keys; every real key registers
    good = st == 0
    assert good.sum() >= 54
    valid, reason = host_verify(L, w)
    assert (reason == w.reason).all() and (valid == w.expected_valid).all()
    _, dreason, tm = dev_verify(L, w)
    assert (dreason == w.reason).all()
    assert tm.n_keycomb >= 0.97 * (tm.n_keycomb + tm.n_ladder)
    _lib.check(L.bh_keys_clear(-1, 0))


def test_pass_loop_real_size(L):
    """4M + 65 records: the library's multi-pass loop (4,194,304-record passes),
    one full pass and a ragged 65-record one, on the host and device APIs."""
    n = (1 << 22) + 65
    w = workload.generate(n, 4096, 64, 16, seed=41)
    valid, reason = host_verify(L, w)
    assert (reason == w.reason).all()
    assert (valid == w.expected_valid).all()
    bits, dreason, _ = dev_verify(L, w)
    assert (dreason == w.reason).all() and (bits == w.expected_valid).all()
    # the records straddling the pass boundary, against the oracle
    for i in range((1 << 22) - 3, n):
        q = bytes(w.pub[64 * i:64 * i + 64])
        s = bytes(w.sig[w.sig_off[i]:w.sig_off[i] + w.sig_len[i]])
        dg = hashlib.sha256(bytes(w.msg[w.msg_off[i]:w.msg_off[i] + w.msg_len[i]])).digest()
        assert orc.csp_verify(q, s, dg) == reason[i]


@pytest.fixture
def small_chunks():
    os.environ["BH_MAX_CHUNK"] = "131072"
    yield 131072
    del os.environ["BH_MAX_CHUNK"]


def test_pass_loop_forced_with_kept_keys(L, small_chunks):
    """200k records in 131,072-record passes with BH_F_KEEP_KEYS and a small
    registry: pass 1 fills the registry and overflows to per-batch tables, so
    the key-sorted comb list mixes registry ids and per-batch ids; pass 2 hits
    the registry. Host and device APIs, twice (second call: all keys kept)."""
    w = workload.generate(200_000, 3000, 100, 16, seed=42)
    _lib.check(L.bh_keys_reserve(0, 0, 1024))
    try:
        for _ in range(2):
            valid, reason = host_verify(L, w, _lib.BH_F_HASH_SHA256 | _lib.BH_F_KEEP_KEYS)
            assert (reason == w.reason).all() and (valid == w.expected_valid).all()
        cnt = ctypes.c_size_t()
        _lib.check(L.bh_keys_count(0, 0, ctypes.byref(cnt)))
        assert cnt.value == 1024
        bits, dreason, tm = dev_verify(L, w, _lib.BH_F_HASH_SHA256 | _lib.BH_F_KEEP_KEYS)
        assert (dreason == w.reason).all() and (bits == w.expected_valid).all()
        assert tm.n_keycomb > 0.9 * (tm.n_keycomb + tm.n_ladder)
    finally:
        _lib.check(L.bh_keys_reserve(0, 0, 65536))
        _lib.check(L.bh_keys_clear(0, 0))


def test_key_table_overflow_to_ladder(L):
    """600k records over 100k keys (~85k keys used >= 4 times): k_key_plan
    builds the first 65,536 tables and the rest of the repeated keys' records
    are routed to the variable-base ladder."""
    w = workload.generate(600_000, 100_000, 64, 16, seed=43)
    bits, reason, tm = dev_verify(L, w)
    assert (reason == w.reason).all() and (bits == w.expected_valid).all()
    assert tm.n_keytables == 65536
    assert tm.n_ladder > 50_000 and tm.n_keycomb > 300_000
    orc_sample(w, 200, seed=1)


def test_submit_wait_pipeline(L):
    """Several batches in flight from page-locked buffers: slot reuse collects
    an uncollected batch early, waits may come in any order."""
    ws = [workload.generate(30_000 + 777 * k, 500, 128, 8, seed=50 + k) for k in range(4)]
    keep, jobs = [], []
    for w in ws:
        arrs = []
        for x in w.arrays():
            h, v = _lib.HostArray.from_numpy(x)
            keep.append(h)
            arrs.append(v)
        b = _lib.BhBatch(*[x.ctypes.data for x in arrs])
        keep.append(b)
        bm = np.zeros((w.n + 7) // 8, np.uint8)
        rs = np.zeros(w.n, np.uint8)
        job = ctypes.c_void_p()
        _lib.check(L.bh_verify_submit(0, ctypes.byref(b), w.n, _lib.BH_F_HASH_SHA256,
                                      bm.ctypes.data, rs.ctypes.data, ctypes.byref(job)))
        jobs.append((job, bm, rs, w))
    for job, bm, rs, w in [jobs[2], jobs[0], jobs[3], jobs[1]]:
        _lib.check(L.bh_verify_wait(job))
        assert (rs == w.reason).all()
        assert (np.unpackbits(bm, bitorder="little")[:w.n].astype(bool) == w.expected_valid).all()
    # an empty batch is a valid job
    job = ctypes.c_void_p()
    b = _lib.BhBatch(*([0] * 7))
    _lib.check(L.bh_verify_submit(0, ctypes.byref(b), 0, 0, None, None, ctypes.byref(job)))
    _lib.check(L.bh_verify_wait(job))


def test_concurrent_host_callers(L):
    """Goroutine-style callers: six threads (ctypes drops the GIL in the call)
    run whole batches through bh_verify at once -- the one-launch small path,
    windowed and comb key tables, the ladder, and a BH_F_KEEP_KEYS caller whose
    registry writes are serialised behind every lane -- so passes of different
    callers share the compute lanes and pipeline slots. Every result is exact."""
    import threading
    shapes = [(200, 20, 0), (9_000, 300, 0), (50_000, 2_000, 0), (40_000, 40_000, 0),
              (60_000, 3_000, _lib.BH_F_KEEP_KEYS), (700, 700, 0)]
    ws = [workload.generate(n, k, 96, 8, seed=90 + j) for j, (n, k, _) in enumerate(shapes)]
    errors = []

    def caller(j):
        try:
            w, flags = ws[j], _lib.BH_F_HASH_SHA256 | shapes[j][2]
            for rep in range(3):
                valid, reason = host_verify(L, w, flags)
                if not ((reason == w.reason).all() and (valid == w.expected_valid).all()):
                    errors.append((j, rep))
        except Exception as e:  # noqa: BLE001 -- reported below with its caller
            errors.append((j, repr(e)))

    _lib.check(L.bh_keys_clear(0, 0))
    threads = [threading.Thread(target=caller, args=(j,)) for j in range(len(ws))]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in threads)
    assert not errors, errors
    _lib.check(L.bh_keys_clear(0, 0))


def test_unique_keys_forced_passes(L, small_chunks):
    """Config 5's shape (every key used once: the variable-base ladder, no key
    tables) through the pass loop: 300,000 unique keys in 131,072-record passes
    (two full passes and a ragged one), host and device APIs."""
    n = 300_000
    w = workload.generate(n, n, 64, 16, seed=44)
    valid, reason = host_verify(L, w)
    assert (reason == w.reason).all() and (valid == w.expected_valid).all()
    bits, dreason, tm = dev_verify(L, w)
    assert (dreason == w.reason).all() and (bits == w.expected_valid).all()
    assert tm.n_keytables == 0 and tm.n_keycomb == 0
    orc_sample(w, 200, seed=2)


def test_unique_keys_one_pass_of_1m(L):
    """One 1,048,576-record pass of unique keys: the ladder's per-lane Q-table
    scratch at pass size (1,792 B per record), as each config-5 rank runs it."""
    n = 1 << 20
    w = workload.generate(n, n, 64, 16, seed=45)
    bits, reason, tm = dev_verify(L, w)
    assert (reason == w.reason).all() and (bits == w.expected_valid).all()
    assert tm.n_ladder == int((w.reason == 0).sum()) + int((w.reason == 9).sum())
    orc_sample(w, 200, seed=3)


def test_two_lanes_with_registry_writes(L):
    """Host batches alternate between the device's two compute lanes; a
    BH_F_KEEP_KEYS batch writes the key registry and is serialised behind both
    lanes, and the lane-1 batches after it wait for that write. Six batches in
    flight in submission order [plain, keep, plain, plain, keep, plain] over
    overlapping key sets (large enough for key tables), collected out of order:
    every bitmap and reason equal the expected ones, and the registry holds
    the kept keys afterwards."""
    _lib.check(L.bh_keys_clear(0, 0))
    ws = [workload.generate(40_000 + 1111 * k, 800 + 50 * k, 96, 8, seed=60 + k % 3)
          for k in range(6)]
    flags = [0, _lib.BH_F_KEEP_KEYS, 0, 0, _lib.BH_F_KEEP_KEYS, 0]
    keep, jobs = [], []
    for w, f in zip(ws, flags):
        arrs = []
        for x in w.arrays():
            h, v = _lib.HostArray.from_numpy(x)
            keep.append(h)
            arrs.append(v)
        b = _lib.BhBatch(*[x.ctypes.data for x in arrs])
        keep.append(b)
        bm = np.zeros((w.n + 7) // 8, np.uint8)
        rs = np.zeros(w.n, np.uint8)
        job = ctypes.c_void_p()
        _lib.check(L.bh_verify_submit(0, ctypes.byref(b), w.n, _lib.BH_F_HASH_SHA256 | f,
                                      bm.ctypes.data, rs.ctypes.data, ctypes.byref(job)))
        jobs.append((job, bm, rs, w))
    for k in [3, 0, 5, 1, 4, 2]:
        job, bm, rs, w = jobs[k]
        _lib.check(L.bh_verify_wait(job))
        assert (rs == w.reason).all(), k
        assert (np.unpackbits(bm, bitorder="little")[:w.n].astype(bool) == w.expected_valid).all(), k
    cnt = ctypes.c_size_t()
    _lib.check(L.bh_keys_count(0, 0, ctypes.byref(cnt)))
    assert cnt.value > 0
    _lib.check(L.bh_keys_clear(0, 0))


def test_comb_and_window_tables_agree(L):
    """A large batch (one lane per record) uses per-batch Lim-Lee comb tables
    (verify.h lltab_build / q_llcomb); BH_LL=0 forces the 4-bit windowed
    tables. Both give the expected bitmap and reasons, record for record."""
    w = workload.generate(200_000, 8_000, 64, 16, seed=46)
    bits1, r1, tm1 = dev_verify(L, w)
    os.environ["BH_LL"] = "0"
    try:
        bits0, r0, tm0 = dev_verify(L, w)
    finally:
        del os.environ["BH_LL"]
    assert tm1.n_keytables > 0 and tm1.n_keycomb > 0.9 * w.n * 15 / 16
    for bits, r in ((bits1, r1), (bits0, r0)):
        assert (r == w.reason).all() and (bits == w.expected_valid).all()


def test_comb_tables_beyond_the_lds_slots(L):
    """k_keycomb copies the comb tables of each 256-record workgroup's runs of
    equal table ids into 17 LDS slots; runs past the slots read their table in
    global memory. At ~6 records per key a workgroup spans ~40 tables, so most
    workgroups (and waves) mix LDS-staged and global runs, and keys used < 4
    times take the ladder in between: bitmap and reasons still exact."""
    w = workload.generate(120_000, 20_000, 64, 16, seed=47)
    bits, r, tm = dev_verify(L, w)
    assert tm.n_keytables > 10_000 and tm.n_keycomb > 0.8 * w.n and tm.n_ladder > 1_000
    assert (r == w.reason).all() and (bits == w.expected_valid).all()
    orc_sample(w, 100, seed=47)


# ---------------------------------------------------------------- compact host layout
def _compact_verify(L, cb, n, flags=_lib.BH_F_HASH_SHA256, submit=False):
    bm = np.zeros((n + 7) // 8 or 1, np.uint8)
    rs = np.zeros(n or 1, np.uint8)
    if submit:
        job = ctypes.c_void_p()
        _lib.check(L.bh_verify_compact_submit(0, ctypes.byref(cb), n, flags, bm.ctypes.data,
                                              rs.ctypes.data, ctypes.byref(job)))
        _lib.check(L.bh_verify_wait(job))
    else:
        _lib.check(L.bh_verify_compact(0, ctypes.byref(cb), n, flags, bm.ctypes.data,
                                       rs.ctypes.data))
    return np.unpackbits(bm, bitorder="little")[:n].astype(bool), rs[:n]


@pytest.mark.parametrize("dedup,stride", [(True, True), (True, False), (False, True),
                                          (False, False)])
def test_compact_layout_matches(L, dedup, stride):
    """bh_verify_compact (distinct keys + u32 indices, lengths only, fixed
    message stride) gives the bitmap and reasons of the same records in the
    bh_batch layout: every corruption class, keys shared (key tables) and
    unique, one-lane (> 32,768 records) and split path."""
    for n, nkeys in ((70_000, 3000), (5000, 5000)):
        w = workload.generate(n, nkeys, 96, 8, seed=61)
        arrs, cb = _lib.compact_layout(*w.arrays(), dedup=dedup, stride=stride)
        if dedup:
            assert cb.nkeys < n or nkeys == n
        for submit in (False, True):
            bits, reason = _compact_verify(L, cb, n, submit=submit)
            assert (reason == w.reason).all() and (bits == w.expected_valid).all(), (n, submit)


def test_compact_layout_ragged_messages_and_passes(L, small_chunks):
    """Variable message lengths (msg_len given) through the pass loop
    (131,072-record passes): the device prefix sums restart per shard and the
    passes slice the expanded batch; digest mode (flags 0) with empty digests."""
    n = 300_000
    w = workload.generate(n, 20_000, 64, 16, seed=62)
    dg = [hashlib.sha256(bytes(w.msg[o:o + l])).digest()[:(i % 33)] for i, (o, l) in
          enumerate(zip(w.msg_off, w.msg_len))]
    dl = np.array([len(x) for x in dg], np.uint32)
    do = np.zeros(n, np.uint64)
    do[1:] = np.cumsum(dl[:-1], dtype=np.uint64)
    dgb = np.frombuffer(b"".join(dg) + b"\0", np.uint8)
    plain = (w.pub, w.sig, w.sig_off, w.sig_len, dgb, do, dl)
    arrs, cb = _lib.compact_layout(*plain)
    assert cb.msg_len  # lengths kept: not a fixed stride
    want_bits, want = host_verify(L, type("W", (), {"n": n, "arrays": lambda self: plain})(), 0)
    bits, reason = _compact_verify(L, cb, n, flags=0)
    assert (reason == want).all() and (bits == want_bits).all()
    assert (want == 2).sum() > 0  # empty digests -> BH_R_EMPTY_DIGEST


@pytest.fixture
def host_shards():
    os.environ["BH_HOST_SHARDS"] = "3"
    yield 3
    del os.environ["BH_HOST_SHARDS"]


@pytest.mark.parametrize("nkeys", [40_000, 3000])
def test_compact_layout_shards_gather_keys(L, host_shards, nkeys):
    """A host batch dealt as 3 shards (the multi-device shard path on one
    device, BH_HOST_SHARDS): with more distinct keys than a shard has records
    each shard uploads its keys gathered per record (no whole key table per
    shard); with few keys the table + indices. Same bits and reasons as the
    one-shard bh_batch layout, both entry points."""
    n = 70_001  # shards of 23,360 / 23,360 / 23,281 records (64-record groups)
    w = workload.generate(n, nkeys, 96, 8, seed=64)
    arrs, cb = _lib.compact_layout(*w.arrays())
    assert (cb.nkeys > n // 3) == (nkeys > n // 3)
    for submit in (False, True):
        bits, reason = _compact_verify(L, cb, n, submit=submit)
        assert (reason == w.reason).all() and (bits == w.expected_valid).all(), submit
    valid, r2 = host_verify(L, w)  # the plain layout, sharded the same way
    assert (r2 == w.reason).all() and (valid == w.expected_valid).all()


def test_compact_layout_rejects_bad_input(L):
    w = workload.generate(1000, 10, 32, 0, seed=63)
    arrs, cb = _lib.compact_layout(*w.arrays())
    arrs["key_idx"][500] = cb.nkeys  # out of range
    bm = np.zeros(125, np.uint8)
    rs = np.zeros(1000, np.uint8)
    assert L.bh_verify_compact(0, ctypes.byref(cb), 1000, 1, bm.ctypes.data, rs.ctypes.data) != 0
    assert b"key index" in L.bh_last_error()
    cb0 = _lib.BhCBatch()
    assert L.bh_verify_compact(0, ctypes.byref(cb0), 1000, 1, bm.ctypes.data, rs.ctypes.data) != 0
    # an empty batch is fine
    _lib.check(L.bh_verify_compact(0, ctypes.byref(cb0), 0, 1, None, None))


def test_resident_passes_on_two_lanes(L):
    """BH_F_ANY_LANE: consecutive bh_verify_dev calls rotate over the device's
    compute lanes (each with its own workspace) and overlap; with
    distinct outputs every pass's bitmap and reasons are exact after bh_sync,
    for batches of different shapes (key tables and ladder) in flight
    together."""
    DA = _lib.DeviceArray
    ws = [workload.generate(40_000 + 5000 * k, [2000, 45_000, 500, 3000][k], 128, 8,
                            seed=70 + k) for k in range(4)]
    bufs = []
    for w in ws:
        d = [DA.from_numpy(0, x) for x in w.arrays()]
        bufs.append((w, d, DA(0, ((w.n + 63) // 64) * 8), DA(0, w.n),
                     _lib.BhBatch(*[x.ptr for x in d])))
    for rep in range(2):
        for w, d, words, reason, b in bufs:
            _lib.check(L.bh_verify_dev(0, 0, ctypes.byref(b), w.n,
                                       _lib.BH_F_HASH_SHA256 | _lib.BH_F_ANY_LANE, words.ptr,
                                       reason.ptr, None, 0, None))
        _lib.check(L.bh_sync(0))
        for w, d, words, reason, b in bufs:
            bits = np.unpackbits(words.to_numpy(np.uint64, (w.n + 63) // 64).view(np.uint8),
                                 bitorder="little")[:w.n].astype(bool)
            assert (reason.to_numpy(np.uint8, w.n) == w.reason).all(), rep
            assert (bits == w.expected_valid).all(), rep
    for w, d, words, reason, b in bufs:
        for x in d + [words, reason]:
            x.free()


def test_any_lane_four_rotating_output_sets(L):
    """the BH_F_ANY_LANE contract -- 4 rotating output
    sets are safe -- now holds by construction (pass k + 4 waits for pass k,
    bdls_hip.cpp any_ring), at every lane count and with host batches taking
    lanes in between. 12 passes over 3 DIFFERENT batches into 4 output sets:
    after bh_sync set s holds exactly pass 8 + s's result (batch (8 + s) % 3)."""
    DA = _lib.DeviceArray
    n = 60_000
    ws = [workload.generate(n, [3000, 60_000, 700][k], 96, 8, seed=90 + k) for k in range(3)]
    ins = []
    for w in ws:
        d = [DA.from_numpy(0, x) for x in w.arrays()]
        ins.append((d, _lib.BhBatch(*[x.ptr for x in d])))
    outs = [(DA(0, ((n + 63) // 64) * 8), DA(0, n)) for _ in range(4)]
    small = workload.generate(3000, 40, 64, 8, seed=99)
    for k in range(12):
        words, reason = outs[k % 4]
        _lib.check(L.bh_verify_dev(0, 0, ctypes.byref(ins[k % 3][1]), n,
                                   _lib.BH_F_HASH_SHA256 | _lib.BH_F_ANY_LANE, words.ptr,
                                   reason.ptr, None, 0, None))
        if k % 5 == 2:  # a host batch takes a lane in between
            _, rs = host_verify(L, small)
            assert (rs == small.reason).all()
    _lib.check(L.bh_sync(0))
    for s, (words, reason) in enumerate(outs):
        w = ws[(8 + s) % 3]
        bits = np.unpackbits(words.to_numpy(np.uint64, (n + 63) // 64).view(np.uint8),
                             bitorder="little")[:n].astype(bool)
        assert (reason.to_numpy(np.uint8, n) == w.reason).all(), s
        assert (bits == w.expected_valid).all(), s
    for d, _ in ins:
        for x in d:
            x.free()
    for pair in outs:
        for x in pair:
            x.free()


def test_config2_exact_shape(L):
    """BASELINE config 2's exact batch -- 1,048,576 records,
    65,536 keys, 256-B messages, 1/16 corrupted, seed 2 (bench.py's default
    line) -- through the compact host ABI (the bench's host path) and the
    device-resident ABI (its `value`): bitmap and reasons against construction,
    the routes the roofline prices (every key-table record on the comb, every
    key used >= 4 times gets a table), and a 300-record orc.csp_verify sample."""
    n, nkeys = 1 << 20, 1 << 16
    w = workload.generate(n, nkeys, 256, 16, seed=2)
    orc_sample(w, 300, seed=2)
    carrs, cb = _lib.compact_layout(*w.arrays())
    # the off-curve / >= p corruptions each add a distinct (invalid) key row
    bad_keys = int(np.isin(w.cls, [6, 7]).sum())
    assert nkeys <= len(carrs["keys"]) // 64 <= nkeys + bad_keys
    bm = np.zeros(n // 8, np.uint8)
    rs = np.zeros(n, np.uint8)
    _lib.check(L.bh_verify_compact(0, ctypes.byref(cb), n, _lib.BH_F_HASH_SHA256,
                                   bm.ctypes.data, rs.ctypes.data))
    assert (rs == w.reason).all()
    assert (np.unpackbits(bm, bitorder="little").astype(bool) == w.expected_valid).all()
    bits, dreason, tm = dev_verify(L, w)
    assert (dreason == w.reason).all() and (bits == w.expected_valid).all()
    ok_prep = int((w.reason == 0).sum() + (w.reason == 9).sum())  # math-checked records
    assert tm.n_keycomb + tm.n_ladder == ok_prep
    assert tm.n_keytables >= 65_000 and tm.n_keycomb >= 0.99 * ok_prep


@pytest.mark.parametrize("shards", ["2", "8"])
def test_config2_exact_shape_host_shards(L, shards, monkeypatch):
    """config 2's exact batch split the way a 2- and an
    8-device node splits it (bdls_amd/csrc/shard.h: contiguous 64-aligned
    shards, each with its own pipeline slot, staging, key tables and bitmap
    words, merged into the caller's bitmap) -- here as BH_HOST_SHARDS shards on
    the one device -- through the plain host ABI and the staged BatchVerify:
    bitmap and reasons equal the construction, so the in-process multi-device
    path is exercised on hardware."""
    n, nkeys = 1 << 20, 1 << 16
    w = workload.generate(n, nkeys, 256, 16, seed=2)
    monkeypatch.setenv("BH_HOST_SHARDS", shards)
    bits, rs = host_verify(L, w)
    assert (rs == w.reason).all() and (bits == w.expected_valid).all()
    bm = np.zeros(n // 8, np.uint8)
    rs2 = np.zeros(n, np.uint8)
    b = _lib.BhBatch(*[x.ctypes.data for x in w.arrays()])
    _lib.check(L.bh_batch_verify(0, ctypes.byref(b), n, _lib.BH_F_HASH_SHA256, bm.ctypes.data,
                                 rs2.ctypes.data))
    assert (rs2 == w.reason).all()
    assert (np.unpackbits(bm, bitorder="little").astype(bool) == w.expected_valid).all()
    assert _lib.pack_stats()["records"] == n // int(shards)
