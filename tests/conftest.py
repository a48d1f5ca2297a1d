import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden", "p256_vectors.jsonl")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) device")


@pytest.fixture(scope="session")
def golden():
    with open(GOLDEN) as f:
        return [json.loads(l) for l in f]


def pack(recs, fused):
    """SoA numpy packing of golden records (digest mode or fused-message mode)."""
    import numpy as np
    pub = np.frombuffer(b"".join(bytes.fromhex(r["qx"] + r["qy"]) for r in recs), np.uint8)
    sigs = [bytes.fromhex(r["sig"]) for r in recs]
    msgs = [bytes.fromhex(r["msg"] if fused else r["digest"]) for r in recs]
    sl = np.array([len(s) for s in sigs], np.uint32)
    ml = np.array([len(m) for m in msgs], np.uint32)
    so = np.zeros(len(recs), np.uint64)
    mo = np.zeros(len(recs), np.uint64)
    if recs:
        so[1:] = np.cumsum(sl[:-1])
        mo[1:] = np.cumsum(ml[:-1])
    sig = np.frombuffer(b"".join(sigs) + b"\0", np.uint8)
    msg = np.frombuffer(b"".join(msgs) + b"\0", np.uint8)
    return pub, sig, so, sl, msg, mo, ml
