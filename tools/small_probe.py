"""Small-batch latency probe: where a lone / small BatchVerify spends its time.
Per batch size n (digest mode, keys registered or cold): host bh_verify p50,
device-resident bh_verify_dev p50 and the per-stage HIP-event times."""
import ctypes
import hashlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bdls_amd import _lib, workload  # noqa: E402


def main():
    L = _lib.lib()
    _lib.check(L.bh_init(1, 0))
    out = {}
    for n in [int(x) for x in (sys.argv[1:] or ["1", "8", "64", "512"])]:
        w = workload.generate(n, max(1, n // 4), 256, 0, seed=5)
        dg = np.frombuffer(b"".join(hashlib.sha256(bytes(w.msg[o:o + l])).digest()
                                    for o, l in zip(w.msg_off, w.msg_len)), np.uint8)
        doff = np.arange(n, dtype=np.uint64) * 32
        dlen = np.full(n, 32, np.uint32)
        arrs = (w.pub, w.sig, w.sig_off, w.sig_len, dg, doff, dlen)
        hb = _lib.BhBatch(*[x.ctypes.data for x in arrs])
        dev = [_lib.DeviceArray.from_numpy(0, x) for x in arrs]
        db = _lib.BhBatch(*[x.ptr for x in dev])
        bm = np.zeros((n + 7) // 8, np.uint8)
        rs = np.zeros(n, np.uint8)
        dw = _lib.DeviceArray(0, ((n + 63) // 64) * 8)
        dr = _lib.DeviceArray(0, n)
        for mode in ("cold", "registered"):
            _lib.check(L.bh_keys_clear(-1, 0))
            if mode == "registered":
                uk = np.unique(w.pub.reshape(-1, 64), axis=0)
                st = np.zeros(len(uk), np.uint8)
                _lib.check(L.bh_keys_register(-1, 0, np.ascontiguousarray(uk).ctypes.data, len(uk),
                                              st.ctypes.data))
            host, devt = [], []
            for k in range(30):
                t = time.perf_counter()
                _lib.check(L.bh_verify(0, ctypes.byref(hb), n, 0, bm.ctypes.data, rs.ctypes.data))
                host.append((time.perf_counter() - t) * 1e6)
                t = time.perf_counter()
                _lib.check(L.bh_verify_dev(0, 0, ctypes.byref(db), n, 0, dw.ptr, dr.ptr, None, 1,
                                           None))
                devt.append((time.perf_counter() - t) * 1e6)
            tm = _lib.BhTiming()
            _lib.check(L.bh_verify_dev(0, 0, ctypes.byref(db), n, 0, dw.ptr, dr.ptr, None, 1,
                                       ctypes.byref(tm)))
            out[f"{mode}_n{n}"] = {
                "host_p50_us": round(float(np.median(host[5:])), 1),
                "dev_p50_us": round(float(np.median(devt[5:])), 1),
                "stages_us": {k: round(getattr(tm, k) * 1e3, 1) for k in _lib.BhTiming.STAGES},
                "routes": [tm.n_keycomb, tm.n_ladder, tm.n_keytables, tm.wide],
                "parity": bool((rs == 0).all())}
            print(json.dumps({f"{mode}_n{n}": out[f"{mode}_n{n}"]}), flush=True)
    _lib.check(L.bh_keys_clear(-1, 0))


if __name__ == "__main__":
    main()
