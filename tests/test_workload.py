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
