"""ctypes binding for oracle/build/liborc.so (CPU ORACLE -- test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

P256, SECP256K1 = 0, 1


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "build", "liborc.so")
        if not os.path.exists(path):
            raise RuntimeError(f"oracle library not built: {path} (run `make -C oracle`)")
        L = ctypes.CDLL(path)
        u8p = ctypes.c_void_p
        L.orc_csp_verify.argtypes = [ctypes.c_int, u8p, u8p, ctypes.c_size_t, u8p, ctypes.c_size_t]
        L.orc_csp_verify.restype = ctypes.c_int
        L.orc_go_verify.argtypes = [ctypes.c_int, u8p, u8p, ctypes.c_size_t, u8p, u8p]
        L.orc_go_verify.restype = ctypes.c_int
        L.orc_unmarshal.argtypes = [u8p, ctypes.c_size_t, u8p, u8p,
                                    ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        L.orc_unmarshal.restype = ctypes.c_int
        L.orc_batch_verify.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_size_t] + [u8p] * 7 + \
            [u8p, ctypes.c_int]
        L.orc_batch_verify.restype = ctypes.c_int
        L.orc_bdls_verify.argtypes = [ctypes.c_int, ctypes.c_size_t] + [u8p] * 12
        L.orc_bdls_verify.restype = ctypes.c_int
        L.orc_bdls_hash.argtypes = [ctypes.c_uint32, u8p, u8p, ctypes.c_uint32, u8p]
        _LIB = L
    return _LIB


def _buf(b: bytes):
    return ctypes.create_string_buffer(bytes(b), max(1, len(b)))


def csp_verify(q64: bytes, sig: bytes, digest: bytes, curve: int = P256) -> int:
    return lib().orc_csp_verify(curve, _buf(q64), _buf(sig), len(sig), _buf(digest), len(digest))


def go_verify(q64: bytes, digest: bytes, r: int, s: int, curve: int = P256) -> int:
    return lib().orc_go_verify(curve, _buf(q64), _buf(digest), len(digest),
                               _buf(r.to_bytes(32, "big")), _buf(s.to_bytes(32, "big")))


def unmarshal(sig: bytes):
    r = ctypes.create_string_buffer(32)
    s = ctypes.create_string_buffer(32)
    rb, sb = ctypes.c_int(), ctypes.c_int()
    rc = lib().orc_unmarshal(_buf(sig), len(sig), r, s, ctypes.byref(rb), ctypes.byref(sb))
    return rc, r.raw, s.raw, rb.value, sb.value


def batch_verify(q: np.ndarray, msg: np.ndarray, moff: np.ndarray, mlen: np.ndarray,
                 sig: np.ndarray, soff: np.ndarray, slen: np.ndarray, fused=True,
                 nthreads: int = 1, curve: int = P256) -> np.ndarray:
    """Returns the reason code per record (0 = valid). fused: False (msg is the
    digest), True / "SHA2" (SHA-256 of msg), "SHA3" (SHA3-256 of msg)."""
    n = len(mlen)
    reason = np.zeros(n, dtype=np.uint8)
    q = np.ascontiguousarray(q, dtype=np.uint8)
    msg = np.ascontiguousarray(msg, dtype=np.uint8)
    moff = np.ascontiguousarray(moff, dtype=np.uint64)
    mlen = np.ascontiguousarray(mlen, dtype=np.uint32)
    sig = np.ascontiguousarray(sig, dtype=np.uint8)
    soff = np.ascontiguousarray(soff, dtype=np.uint64)
    slen = np.ascontiguousarray(slen, dtype=np.uint32)
    mode = {False: 0, True: 1, "SHA2": 1, "SHA3": 2}[fused]
    lib().orc_batch_verify(curve, mode, n, q.ctypes.data, msg.ctypes.data,
                           moff.ctypes.data, mlen.ctypes.data, sig.ctypes.data,
                           soff.ctypes.data, slen.ctypes.data, reason.ctypes.data, nthreads)
    return reason


def bdls_hash(version: int, xy: bytes, msg: bytes) -> bytes:
    """SignedProto.Hash (message.go:97-138)."""
    out = ctypes.create_string_buffer(32)
    lib().orc_bdls_hash(version, _buf(xy), _buf(msg), len(msg), out)
    return out.raw


def bdls_verify(curve: int, xy, r, r_off, r_len, s, s_off, s_len, version, msg, msg_off,
                msg_len) -> np.ndarray:
    """Serial SignedProto.Verify over a bh_bdls_batch-shaped SoA; reason per record."""
    arrs = [np.ascontiguousarray(a) for a in (xy, r, r_off, r_len, s, s_off, s_len, version, msg,
                                              msg_off, msg_len)]
    n = len(arrs[7])
    reason = np.zeros(n, dtype=np.uint8)
    lib().orc_bdls_verify(curve, n, *[a.ctypes.data for a in arrs], reason.ctypes.data)
    return reason
