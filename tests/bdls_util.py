"""Shared packing helpers for BDLS SignedProto batches (tests and bench)."""
import numpy as np


def pack_bdls(recs):
    """SoA arrays in bh_bdls_batch order from golden-style dict records."""
    n = len(recs)
    xy = np.frombuffer(b"".join(bytes.fromhex(r["x"] + r["y"]) for r in recs) or b"\0", np.uint8)

    def cat(field):
        parts = [bytes.fromhex(r[field]) for r in recs]
        ln = np.array([len(p) for p in parts], np.uint32)
        off = np.zeros(n, np.uint64)
        if n:
            off[1:] = np.cumsum(ln[:-1])
        return np.frombuffer(b"".join(parts) + b"\0", np.uint8), off, ln

    r, ro, rl = cat("r")
    s, so, sl = cat("s")
    m, mo, ml = cat("msg")
    ver = np.array([r_["version"] for r_ in recs], np.uint32)
    return xy, r, ro, rl, s, so, sl, ver, m, mo, ml
