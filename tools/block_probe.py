"""Workgroup-size probe for the latency-bound kernels: small host batches
(k_small, BH_SMALL_BLOCK) and the multi-lane kernels of the batch path
(BH_WIDE_BLOCK), cold and registered keys, plus configs 3 / 4 latencies."""
import ctypes
import hashlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bdls_amd import _lib, workload  # noqa: E402


def batch(n, seed=5):
    w = workload.generate(n, max(1, n // 4), 256, 0, seed=seed)
    dg = np.frombuffer(b"".join(hashlib.sha256(bytes(w.msg[o:o + l])).digest()
                                for o, l in zip(w.msg_off, w.msg_len)), np.uint8)
    doff = np.arange(n, dtype=np.uint64) * 32
    dlen = np.full(n, 32, np.uint32)
    return w, (w.pub, w.sig, w.sig_off, w.sig_len, dg, doff, dlen)


def main():
    L = _lib.lib()
    _lib.check(L.bh_init(1, 0))
    res = {}
    for n in (1, 4, 16, 64, 256, 2048):
        w, arrs = batch(n)
        hb = _lib.BhBatch(*[x.ctypes.data for x in arrs])
        bm = np.zeros((n + 7) // 8, np.uint8)
        rs = np.zeros(n, np.uint8)
        for mode in ("cold", "registered"):
            _lib.check(L.bh_keys_clear(-1, 0))
            if mode == "registered":
                uk = np.unique(w.pub.reshape(-1, 64), axis=0)
                st = np.zeros(len(uk), np.uint8)
                _lib.check(L.bh_keys_register(-1, 0, np.ascontiguousarray(uk).ctypes.data,
                                              len(uk), st.ctypes.data))
            for env in ("BH_SMALL_BLOCK", "BH_WIDE_BLOCK"):
                if env == "BH_SMALL_BLOCK" and n > 256:
                    continue
                for bs in ("64", "256"):
                    os.environ[env] = bs
                    if env == "BH_WIDE_BLOCK":
                        os.environ["BH_NO_SMALL"] = "1"
                    t = []
                    for k in range(12):
                        t0 = time.perf_counter()
                        _lib.check(L.bh_verify(0, ctypes.byref(hb), n, 0, bm.ctypes.data,
                                               rs.ctypes.data))
                        t.append((time.perf_counter() - t0) * 1e6)
                    os.environ.pop(env)
                    os.environ.pop("BH_NO_SMALL", None)
                    key = f"{mode}_n{n}_{env[3:]}{bs}"
                    res[key] = round(float(np.median(t[2:])), 1)
                    assert (rs == 0).all()
            print(json.dumps({k: v for k, v in res.items() if f"_n{n}_" in k and k.startswith(mode)}),
                  flush=True)
    _lib.check(L.bh_keys_clear(-1, 0))


if __name__ == "__main__":
    main()
