"""CPU: the synthetic workload generator's expected results (by construction)
agree with the independent C oracle, for every corruption class."""
import numpy as np

from bdls_amd import workload
from oracle import orc


def test_workload_expected_matches_oracle():
    w = workload.generate(6000, 300, 256, 4, seed=2, nthreads=4)
    assert set(np.unique(w.cls)) == set(range(len(workload.CLASS_NAMES)))
    got = orc.batch_verify(w.pub.reshape(-1, 64), w.msg, w.msg_off, w.msg_len, w.sig, w.sig_off,
                           w.sig_len, fused=True, nthreads=4)
    assert (got == w.reason).all()


def test_workload_deterministic():
    a = workload.generate(300, 7, 100, 8, seed=5, nthreads=1)
    b = workload.generate(300, 7, 100, 8, seed=5, nthreads=3)
    assert (a.sig == b.sig).all() and (a.msg == b.msg).all() and (a.pub == b.pub).all()


def test_workload_sha3_family_matches_oracle():
    """SHA3 family records (msp/identities.go:219-227): the C oracle hashes with
    SHA3-256 (bccsp/sw/new.go:72) and agrees with the construction."""
    w = workload.generate(2000, 100, 200, 4, seed=12, nthreads=4, family="SHA3")
    args = (w.pub.reshape(-1, 64), w.msg, w.msg_off, w.msg_len, w.sig, w.sig_off, w.sig_len)
    assert (orc.batch_verify(*args, fused="SHA3", nthreads=4) == w.reason).all()
    sha2 = orc.batch_verify(*args, fused="SHA2", nthreads=4)
    assert (sha2[w.reason == 0] != 0).all()


def test_config5_shard_chunks_and_cache(tmp_path):
    """Config 5's shard generator (VERDICT r4 missing #1): chunked generation of
    a unique-key shard equals the one-call shard byte for byte; the on-disk copy
    written after generation is read back identically (and reported as such);
    a different shard never takes another shard's copy."""
    n_total, lo, count = 1 << 20, 4096, 1000
    ref = workload.generate_shard(n_total, lo, count, n_total, 256, 64, seed=5, nthreads=2)
    logs = []
    w, info = workload.generate_shard_cached(n_total, lo, count, n_total, 256, 64, seed=5,
                                             nthreads=2, cache_dir=str(tmp_path), chunk=300,
                                             log=logs.append)
    assert info["source"] == "generator" and info.get("saved")
    assert any("generated 1000/1000" in m for m in logs)
    for name in ("pub", "msg", "msg_off", "msg_len", "sig", "sig_off", "sig_len", "reason", "cls"):
        assert (getattr(w, name) == getattr(ref, name)).all(), name
    w2, info2 = workload.generate_shard_cached(n_total, lo, count, n_total, 256, 64, seed=5,
                                               nthreads=2, cache_dir=str(tmp_path))
    assert info2["source"] == "cache"
    for name in ("pub", "msg", "msg_off", "sig", "sig_off", "sig_len", "reason"):
        assert (getattr(w2, name) == getattr(ref, name)).all(), name
    w3, info3 = workload.generate_shard_cached(n_total, lo + 64, count, n_total, 256, 64, seed=5,
                                               nthreads=2, cache_dir=str(tmp_path), save=False)
    assert info3["source"] == "generator" and not (w3.pub == ref.pub).all()
    got = orc.batch_verify(w2.pub.reshape(-1, 64), w2.msg, w2.msg_off, w2.msg_len, w2.sig,
                           w2.sig_off, w2.sig_len, fused=True, nthreads=4)
    assert (got == w2.reason).all()


def test_config5_cache_rejects_tampered_copy(tmp_path):
    """the cache key carries the generator library's fingerprint and
    meta.json every array's byte count; a copy whose file sizes disagree (a
    longer file, a foreign write) is regenerated, never loaded."""
    n_total, lo, count = 1 << 20, 0, 200
    key = workload.cache_key(n_total, lo, count, n_total, 256, 64, 5)
    assert "_g" in key and not key.endswith("_gnolib_v2")
    w, info = workload.generate_shard_cached(n_total, lo, count, n_total, 256, 64, seed=5,
                                             nthreads=2, cache_dir=str(tmp_path))
    assert info.get("saved")
    with open(tmp_path / key / "pub.bin", "ab") as f:  # one byte too many
        f.write(b"\0")
    logs = []
    w2, info2 = workload.generate_shard_cached(n_total, lo, count, n_total, 256, 64, seed=5,
                                               nthreads=2, cache_dir=str(tmp_path),
                                               save=False, log=logs.append)
    assert info2["source"] == "generator" and any("does not match" in m for m in logs)
    assert (w2.pub == w.pub).all()
