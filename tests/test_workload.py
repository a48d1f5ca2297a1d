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
