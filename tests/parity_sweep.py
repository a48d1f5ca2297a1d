#!/usr/bin/env python3
"""Randomised parity sweep on the GPU (evidence beyond the fixed -m gpu cases).

usage: python tests/parity_sweep.py [cases] [seed] > out.jsonl

(Test infrastructure, not collected by pytest: it imports the oracle as the
checker, so it lives under tests/.)

Each case draws a batch shape -- records (1 .. 300,000, biased to the edges
of the routing rules: the small-batch kernels, the 32,768-record wide/comb
boundary, key-table thresholds), distinct keys, message length, corruption
rate, SHA-256 or SHA3-256 family -- generates it with workload/gen.c (which
knows every record's expected reason) and runs it through the host ABI
(bh_verify, bh_verify_compact), the staged BatchVerify (bh_batch_verify and
bh_batch_verify_ptrs, round 6) and the device ABI (bh_verify_dev). Every
bitmap bit and reason byte must equal the construction's; a 50-record sample
per case is re-checked against oracle/orc.c (OpenSSL's ECDSA core).
"""
import ctypes
import hashlib
import json
import os
import random
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bdls_amd import _lib, workload  # noqa: E402
from oracle import orc  # noqa: E402  (the checker only)


def bits_of(bm, n):
    return np.unpackbits(bm, bitorder="little")[:n].astype(bool)


def main():
    cases = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    rng = random.Random(int(sys.argv[2]) if len(sys.argv) > 2 else 7)
    _lib.ensure_init()
    L = _lib.lib()
    bad = 0
    for c in range(cases):
        n = rng.choice([1, 7, 63, 64, 65, 255, 256, 257, 1000, 4095, 32767, 32768, 32769,
                        rng.randrange(2, 300_000)])
        nkeys = max(1, min(n, rng.choice([1, 3, n // 4 or 1, n // 16 or 1, n, rng.randrange(1, n + 1)])))
        mlen = rng.choice([0, 1, 32, 55, 56, 64, 100, 256, 1500])
        mlen = max(mlen, 1)
        corrupt = rng.choice([2, 8, 16, 64])
        family = rng.choice(["SHA2", "SHA2", "SHA3"])
        flag = _lib.BH_F_HASH_SHA256 if family == "SHA2" else _lib.BH_F_HASH_SHA3_256
        t0 = time.time()
        w = workload.generate(n, nkeys, mlen, corrupt, seed=1000 + c, family=family)
        res = {"case": c, "n": n, "nkeys": nkeys, "msg_len": mlen, "corrupt_den": corrupt,
               "family": family}
        # host ABI, plain layout
        bm = np.zeros((n + 7) // 8, np.uint8)
        rs = np.zeros(n, np.uint8)
        b = _lib.BhBatch(*[x.ctypes.data for x in w.arrays()])
        _lib.check(L.bh_verify(0, ctypes.byref(b), n, flag, bm.ctypes.data, rs.ctypes.data))
        res["host"] = bool((rs == w.reason).all() and (bits_of(bm, n) == w.expected_valid).all())
        # host ABI, compact layout
        keep, cb = _lib.compact_layout(w.pub, w.sig, w.sig_off, w.sig_len, w.msg, w.msg_off,
                                       w.msg_len, dedup=True, stride=False)
        bm2 = np.zeros((n + 7) // 8, np.uint8)
        rs2 = np.zeros(n, np.uint8)
        _lib.check(L.bh_verify_compact(0, ctypes.byref(cb), n, flag, bm2.ctypes.data,
                                       rs2.ctypes.data))
        res["compact"] = bool((rs2 == w.reason).all() and (bits_of(bm2, n) == w.expected_valid).all())
        # staged BatchVerify from the same pageable arrays (pack.h: the library
        # dedups and packs into its own page-locked staging)
        bm3 = np.zeros((n + 7) // 8, np.uint8)
        rs3 = np.zeros(n, np.uint8)
        _lib.check(L.bh_batch_verify(0, ctypes.byref(b), n, flag, bm3.ctypes.data, rs3.ctypes.data))
        res["staged"] = bool((rs3 == w.reason).all() and (bits_of(bm3, n) == w.expected_valid).all())
        # ... and its per-record pointer form (the Go binding's bh_pbatch)
        kp = (w.pub.ctypes.data + 64 * np.arange(n, dtype=np.uint64)).astype(np.uint64)
        sp = (w.sig.ctypes.data + w.sig_off[:n]).astype(np.uint64)
        mp = (w.msg.ctypes.data + w.msg_off[:n]).astype(np.uint64)
        sl = np.ascontiguousarray(w.sig_len[:n])
        ml = np.ascontiguousarray(w.msg_len[:n])
        pb = _lib.BhPBatch(*[x.ctypes.data for x in (kp, sp, sl, mp, ml)])
        bm4 = np.zeros((n + 7) // 8, np.uint8)
        rs4 = np.zeros(n, np.uint8)
        _lib.check(L.bh_batch_verify_ptrs(0, ctypes.byref(pb), n, flag, bm4.ctypes.data,
                                          rs4.ctypes.data))
        res["staged_ptrs"] = bool((rs4 == w.reason).all()
                                  and (bits_of(bm4, n) == w.expected_valid).all())
        # device ABI
        DA = _lib.DeviceArray
        d = [DA.from_numpy(0, x) for x in w.arrays()]
        words, reason = DA(0, ((n + 63) // 64) * 8), DA(0, n)
        db = _lib.BhBatch(*[x.ptr for x in d])
        _lib.check(L.bh_verify_dev(0, 0, ctypes.byref(db), n, flag, words.ptr, reason.ptr, None, 1,
                                   None))
        dbits = bits_of(words.to_numpy(np.uint64, (n + 63) // 64).view(np.uint8), n)
        res["device"] = bool((reason.to_numpy(np.uint8, n) == w.reason).all()
                             and (dbits == w.expected_valid).all())
        for x in d + [words, reason]:
            x.free()
        # the OpenSSL-backed oracle on a sample
        idx = np.random.default_rng(c).choice(n, min(n, 50), replace=False)
        hf = hashlib.sha256 if family == "SHA2" else hashlib.sha3_256
        ok = True
        for i in idx:
            q = bytes(w.pub[64 * i:64 * i + 64])
            s = bytes(w.sig[w.sig_off[i]:w.sig_off[i] + w.sig_len[i]])
            dg = hf(bytes(w.msg[w.msg_off[i]:w.msg_off[i] + w.msg_len[i]])).digest()
            ok = ok and orc.csp_verify(q, s, dg) == w.reason[i]
        res["oracle_sample"] = bool(ok)
        res["valid"] = int(w.expected_valid.sum())
        res["s"] = round(time.time() - t0, 2)
        good = (res["host"] and res["compact"] and res["staged"] and res["staged_ptrs"]
                and res["device"]
                and res["oracle_sample"])
        bad += 0 if good else 1
        print(json.dumps(res), flush=True)
    print(json.dumps({"cases": cases, "failed": bad}), flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
