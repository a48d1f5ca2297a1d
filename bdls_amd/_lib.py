"""ctypes binding of libbdlship.so (include/bdls_hip.h).

The product path is the HIP library: if it is missing, or no gfx950 device is
visible, every entry point raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# BDLS_HIP_LIB overrides the library path (A/B runs of build variants).
LIB_PATH = os.environ.get("BDLS_HIP_LIB") or os.path.join(_HERE, "lib", "libbdlship.so")

BH_OK = 0
BH_F_HASH_SHA256 = 1
BH_F_NO_LOW_S = 2
BH_F_KEEP_KEYS = 4
BH_F_HASH_SHA3_256 = 8
BH_F_ANY_LANE = 16
BH_CURVE_P256 = 0
BH_CURVE_SECP256K1 = 1

# Every symbol include/bdls_hip.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "bh_init", "bh_shutdown", "bh_device_count", "bh_last_error", "bh_version",
    "bh_workspace_bytes", "bh_verify", "bh_verify_2seg", "bh_verify_dev", "bh_csp_verify_p256",
    "bh_parse_der_sig", "bh_dev_alloc", "bh_dev_free", "bh_memcpy_h2d", "bh_memcpy_d2h",
    "bh_sync", "bh_verify_bdls", "bh_verify_bdls_dev", "bh_keys_reserve", "bh_keys_register",
    "bh_keys_clear", "bh_keys_count", "bh_timing_begin", "bh_timing_end", "bh_bdls_preverify",
    "bh_verify_submit", "bh_verify_wait", "bh_host_alloc", "bh_host_free", "bh_csp_stats",
    "bh_fabric_block_preverify", "bh_verify_x509", "bh_signature_sets_verify",
    "bh_envelopes_preverify", "bh_block_signatures_preverify",
    "bh_block_signatures_preverify_bft", "bh_fabric_block_preverify_refs", "bh_device_stats",
    "bh_verify_compact", "bh_verify_compact_submit",
    "bh_batch_verify", "bh_batch_verify_submit", "bh_batch_verify_ptrs",
    "bh_batch_verify_ptrs_submit", "bh_pack_stats",
)
KEY_FULL = 255  # bh_keys_register status: registry full


class BhBatch(ctypes.Structure):
    _fields_ = [
        ("pub", ctypes.c_void_p),
        ("sig", ctypes.c_void_p),
        ("sig_off", ctypes.c_void_p),
        ("sig_len", ctypes.c_void_p),
        ("msg", ctypes.c_void_p),
        ("msg_off", ctypes.c_void_p),
        ("msg_len", ctypes.c_void_p),
    ]


class BhCBatch(ctypes.Structure):
    """include/bdls_hip.h bh_cbatch: the compact host layout (distinct keys +
    u32 indices, lengths only, optional fixed message stride)."""
    _fields_ = [("keys", ctypes.c_void_p), ("key_idx", ctypes.c_void_p),
                ("nkeys", ctypes.c_size_t), ("sig", ctypes.c_void_p),
                ("sig_len", ctypes.c_void_p), ("msg", ctypes.c_void_p),
                ("msg_len", ctypes.c_void_p), ("msg_stride", ctypes.c_uint32)]


class BhPBatch(ctypes.Structure):
    """include/bdls_hip.h bh_pbatch: per-record pointers (the staged
    BatchVerify's Go-side form)."""
    _fields_ = [("pub", ctypes.c_void_p), ("sig", ctypes.c_void_p),
                ("sig_len", ctypes.c_void_p), ("msg", ctypes.c_void_p),
                ("msg_len", ctypes.c_void_p)]


PACK_STATS = ("pass_a_ms", "pass_b_ms", "threads", "chunks", "dedup", "nkeys", "records",
              "est_distinct", "rebuilds", "shards")


class BhBdlsBatch(ctypes.Structure):
    _fields_ = [(name, ctypes.c_void_p) for name in
                ("xy", "r", "r_off", "r_len", "s", "s_off", "s_len", "version", "msg",
                 "msg_off", "msg_len")]


class BhTiming(ctypes.Structure):
    _fields_ = [("prep_ms", ctypes.c_float), ("inv_ms", ctypes.c_float),
                ("plan_ms", ctypes.c_float), ("build_ladder_ms", ctypes.c_float),
                ("publish_ms", ctypes.c_float), ("keycomb_ms", ctypes.c_float),
                ("n_keycomb", ctypes.c_uint32), ("n_ladder", ctypes.c_uint32),
                ("n_keytables", ctypes.c_uint32), ("wide", ctypes.c_uint32)]

    STAGES = ("prep_ms", "inv_ms", "plan_ms", "build_ladder_ms", "publish_ms", "keycomb_ms")


class BhBdlsMsgResult(ctypes.Structure):
    """include/bdls_hip.h bh_bdls_msg_result."""
    _fields_ = [("status", ctypes.c_int32), ("bad_sp", ctypes.c_int32),
                ("type", ctypes.c_uint32), ("distinct_signers", ctypes.c_uint32),
                ("height", ctypes.c_uint64), ("round", ctypes.c_uint64),
                ("sp_first", ctypes.c_uint32), ("sp_count", ctypes.c_uint32)]


class BhFabTx(ctypes.Structure):
    """include/bdls_hip.h bh_fab_tx."""
    _fields_ = [("status", ctypes.c_int32), ("type", ctypes.c_int32),
                ("creator", ctypes.c_uint32), ("endorse_first", ctypes.c_uint32),
                ("endorse_count", ctypes.c_uint32), ("valid_endorsers", ctypes.c_uint32)]


class BhFabSigref(ctypes.Structure):
    """include/bdls_hip.h bh_fab_sigref."""
    _fields_ = [("ident_off", ctypes.c_uint64), ("sig_off", ctypes.c_uint64),
                ("msg_off", ctypes.c_uint64), ("msg2_off", ctypes.c_uint64),
                ("ident_len", ctypes.c_uint32), ("sig_len", ctypes.c_uint32),
                ("msg_len", ctypes.c_uint32), ("msg2_len", ctypes.c_uint32),
                ("reason", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


class BhSdBatch(ctypes.Structure):
    _fields_ = [(name, ctypes.c_void_p) for name in
                ("identity", "identity_off", "identity_len", "data", "data_off", "data_len",
                 "sig", "sig_off", "sig_len")]


class BhBlocksigResult(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int32), ("sig_first", ctypes.c_uint32),
                ("sig_count", ctypes.c_uint32), ("valid_identities", ctypes.c_uint32)]


BH_FAB_F_SHA3 = 1
BH_FAB_F_KEEP_KEYS = 2
BH_FAB_F_DECODE_ONLY = 4
BH_BLK_F_BFT = 8


class BhConsenterSet(ctypes.Structure):
    """include/bdls_hip.h bh_consenter_set."""
    _fields_ = [(name, ctypes.c_void_p) for name in
                ("id", "msp_id", "msp_id_off", "msp_id_len", "identity", "identity_off",
                 "identity_len")] + [("n", ctypes.c_size_t)]


class EngineError(RuntimeError):
    """The HIP engine itself failed (no device, HIP error, bad arguments)."""


_lib = None
_init_lock = threading.Lock()
_initialised = False


def lib() -> ctypes.CDLL:
    """Load libbdlship.so (no device access)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise EngineError(f"{LIB_PATH} is not built (run `make` or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        vp, sz, u32, i32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_int
        L.bh_init.argtypes = [u32, u32]
        L.bh_init.restype = i32
        L.bh_shutdown.restype = i32
        L.bh_device_count.restype = i32
        L.bh_last_error.restype = ctypes.c_char_p
        L.bh_version.restype = ctypes.c_char_p
        L.bh_workspace_bytes.argtypes = [sz]
        L.bh_workspace_bytes.restype = sz
        L.bh_verify.argtypes = [i32, ctypes.POINTER(BhBatch), sz, u32, vp, vp]
        L.bh_verify.restype = i32
        L.bh_verify_2seg.argtypes = [i32, ctypes.POINTER(BhBatch), vp, vp, sz, u32, vp, vp]
        L.bh_verify_2seg.restype = i32
        L.bh_verify_submit.argtypes = [i32, ctypes.POINTER(BhBatch), sz, u32, vp, vp,
                                       ctypes.POINTER(vp)]
        L.bh_verify_submit.restype = i32
        L.bh_verify_wait.argtypes = [vp]
        L.bh_verify_wait.restype = i32
        try:  # (an A/B run may load a library built before these entry points)
            L.bh_verify_compact.argtypes = [i32, ctypes.POINTER(BhCBatch), sz, u32, vp, vp]
            L.bh_verify_compact.restype = i32
            L.bh_verify_compact_submit.argtypes = [i32, ctypes.POINTER(BhCBatch), sz, u32, vp, vp,
                                                   ctypes.POINTER(vp)]
            L.bh_verify_compact_submit.restype = i32
        except AttributeError:
            pass
        try:  # round 6: the staged BatchVerify
            L.bh_batch_verify.argtypes = [i32, ctypes.POINTER(BhBatch), sz, u32, vp, vp]
            L.bh_batch_verify.restype = i32
            L.bh_batch_verify_submit.argtypes = [i32, ctypes.POINTER(BhBatch), sz, u32, vp, vp,
                                                 ctypes.POINTER(vp)]
            L.bh_batch_verify_submit.restype = i32
            L.bh_batch_verify_ptrs.argtypes = [i32, ctypes.POINTER(BhPBatch), sz, u32, vp, vp]
            L.bh_batch_verify_ptrs.restype = i32
            L.bh_batch_verify_ptrs_submit.argtypes = [i32, ctypes.POINTER(BhPBatch), sz, u32,
                                                      vp, vp, ctypes.POINTER(vp)]
            L.bh_batch_verify_ptrs_submit.restype = i32
            L.bh_pack_stats.argtypes = [vp]
            L.bh_pack_stats.restype = i32
        except AttributeError:
            pass
        L.bh_host_alloc.argtypes = [sz, ctypes.POINTER(vp)]
        L.bh_host_alloc.restype = i32
        L.bh_host_free.argtypes = [vp]
        L.bh_host_free.restype = i32
        L.bh_verify_dev.argtypes = [i32, i32, ctypes.POINTER(BhBatch), sz, u32, vp, vp, vp, i32,
                                    ctypes.POINTER(BhTiming)]
        L.bh_verify_dev.restype = i32
        L.bh_csp_verify_p256.argtypes = [vp, vp, sz, vp, sz, ctypes.POINTER(i32),
                                         ctypes.POINTER(i32)]
        L.bh_csp_verify_p256.restype = i32
        L.bh_fabric_block_preverify.argtypes = [vp, sz, u32, vp, sz, ctypes.POINTER(sz), vp, sz,
                                                ctypes.POINTER(sz)]
        L.bh_fabric_block_preverify.restype = i32
        L.bh_fabric_block_preverify_refs.argtypes = [vp, sz, u32, vp, sz, ctypes.POINTER(sz), vp,
                                                     sz, ctypes.POINTER(sz), vp, sz,
                                                     ctypes.POINTER(sz)]
        L.bh_fabric_block_preverify_refs.restype = i32
        L.bh_signature_sets_verify.argtypes = [ctypes.POINTER(BhSdBatch), sz, vp, sz, u32, vp, vp]
        L.bh_signature_sets_verify.restype = i32
        L.bh_envelopes_preverify.argtypes = [vp, vp, vp, sz, u32, vp, vp]
        L.bh_envelopes_preverify.restype = i32
        L.bh_block_signatures_preverify.argtypes = [vp, vp, vp, sz, u32, vp, vp, sz,
                                                    ctypes.POINTER(sz)]
        L.bh_block_signatures_preverify.restype = i32
        L.bh_block_signatures_preverify_bft.argtypes = [vp, vp, vp, sz, u32,
                                                        ctypes.POINTER(BhConsenterSet), vp, vp,
                                                        sz, ctypes.POINTER(sz)]
        L.bh_block_signatures_preverify_bft.restype = i32
        L.bh_verify_x509.argtypes = [vp, vp, vp, vp, sz, vp, vp]
        L.bh_verify_x509.restype = i32
        L.bh_csp_stats.argtypes = [vp]
        L.bh_csp_stats.restype = i32
        try:  # (an A/B run may load a library built before this entry point)
            L.bh_device_stats.argtypes = [vp]
            L.bh_device_stats.restype = i32
        except AttributeError:
            pass
        L.bh_parse_der_sig.argtypes = [vp, sz, vp, vp, ctypes.POINTER(i32), ctypes.POINTER(i32)]
        L.bh_parse_der_sig.restype = i32
        L.bh_verify_bdls.argtypes = [i32, ctypes.POINTER(BhBdlsBatch), sz, vp, vp]
        L.bh_verify_bdls.restype = i32
        L.bh_verify_bdls_dev.argtypes = [i32, i32, ctypes.POINTER(BhBdlsBatch), sz, vp, vp, vp,
                                         i32, ctypes.POINTER(BhTiming)]
        L.bh_verify_bdls_dev.restype = i32
        L.bh_dev_alloc.argtypes = [i32, sz, ctypes.POINTER(vp)]
        L.bh_dev_alloc.restype = i32
        L.bh_dev_free.argtypes = [i32, vp]
        L.bh_dev_free.restype = i32
        L.bh_memcpy_h2d.argtypes = [i32, vp, vp, sz]
        L.bh_memcpy_h2d.restype = i32
        L.bh_memcpy_d2h.argtypes = [i32, vp, vp, sz]
        L.bh_memcpy_d2h.restype = i32
        L.bh_sync.argtypes = [i32]
        L.bh_sync.restype = i32
        L.bh_timing_begin.argtypes = [i32]
        L.bh_timing_begin.restype = i32
        L.bh_timing_end.argtypes = [i32, vp]
        L.bh_timing_end.restype = i32
        L.bh_keys_reserve.argtypes = [i32, i32, sz]
        L.bh_keys_reserve.restype = i32
        L.bh_keys_register.argtypes = [i32, i32, vp, sz, vp]
        L.bh_keys_register.restype = i32
        L.bh_keys_clear.argtypes = [i32, i32]
        L.bh_keys_clear.restype = i32
        L.bh_keys_count.argtypes = [i32, i32, ctypes.POINTER(sz)]
        L.bh_keys_count.restype = i32
        L.bh_bdls_preverify.argtypes = [i32, vp, vp, vp, sz, vp, sz, u32, vp, vp, sz,
                                        ctypes.POINTER(sz)]
        L.bh_bdls_preverify.restype = i32
        _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != BH_OK:
        raise EngineError(f"libbdlship error {rc}: {lib().bh_last_error().decode(errors='replace')}")


def ensure_init(device_mask: int = 0) -> None:
    """bh_init on first use; raises EngineError without a gfx950 device."""
    global _initialised
    with _init_lock:
        if not _initialised:
            check(lib().bh_init(device_mask, 0))
            _initialised = True


def last_error() -> str:
    return lib().bh_last_error().decode(errors="replace")


class HostArray:
    """Page-locked host memory from libbdlship.so (bh_host_alloc) viewed as a
    numpy array: the host-API batch layout that lets uploads overlap kernels."""

    def __init__(self, nbytes: int):
        import numpy as np
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        check(lib().bh_host_alloc(max(1, self.nbytes), ctypes.byref(p)))
        self.ptr = p.value
        buf = (ctypes.c_uint8 * max(1, self.nbytes)).from_address(self.ptr)
        self.u8 = np.frombuffer(buf, np.uint8)[:self.nbytes]

    @classmethod
    def from_numpy(cls, a):
        import numpy as np
        a = np.ascontiguousarray(a)
        h = cls(a.nbytes)
        h.u8[:] = a.view(np.uint8).reshape(-1)
        return h, h.u8.view(a.dtype)

    def free(self):
        if self.ptr:
            self.u8 = None
            lib().bh_host_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:  # noqa: BLE001 (interpreter shutdown)
            pass


class DeviceArray:
    """A device buffer owned by libbdlship.so (HBM-resident batch data)."""

    def __init__(self, device: int, nbytes: int):
        self.device = device
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        check(lib().bh_dev_alloc(device, self.nbytes, ctypes.byref(p)))
        self.ptr = p.value

    @classmethod
    def from_numpy(cls, device: int, a):
        import numpy as np
        a = np.ascontiguousarray(a)
        d = cls(device, max(1, a.nbytes))
        if a.nbytes:
            check(lib().bh_memcpy_h2d(device, d.ptr, a.ctypes.data, a.nbytes))
        return d

    def to_numpy(self, dtype, count: int):
        import numpy as np
        out = np.empty(count, dtype=dtype)
        if out.nbytes:
            check(lib().bh_memcpy_d2h(self.device, out.ctypes.data, self.ptr, out.nbytes))
        return out

    def free(self):
        if self.ptr:
            lib().bh_dev_free(self.device, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:  # noqa: BLE001 (interpreter shutdown)
            pass


def device_stats() -> tuple[int, int]:
    """(device batches launched, records they carried) since bh_init, over
    every entry point (bh_device_stats)."""
    import numpy as _np
    out = _np.zeros(2, _np.uint64)
    check(lib().bh_device_stats(out.ctypes.data))
    return int(out[0]), int(out[1])


def compact_layout(pub, sig, sig_off, sig_len, msg, msg_off, msg_len, dedup: bool = True,
                   stride: bool = True, alloc=None):
    """The bh_cbatch arrays of a bh_batch (numpy): distinct keys + u32 indices
    (dedup), signatures and messages re-packed in record order with lengths
    only, msg_len dropped when every message has one length (stride).
    Returns (dict of arrays, BhCBatch)."""
    import numpy as np
    n = len(sig_len)
    mk = alloc or (lambda nb: np.empty(nb, np.uint8))

    def arr(a, dtype):
        out = mk(a.nbytes).view(dtype)
        out[:] = a
        return out
    keys64 = np.ascontiguousarray(pub[:64 * n]).reshape(n, 64)
    if dedup:
        uk, idx = np.unique(keys64, axis=0, return_inverse=True)
        keys = arr(np.ascontiguousarray(uk).reshape(-1), np.uint8)
        key_idx = arr(idx.astype(np.uint32).reshape(-1), np.uint32)
    else:
        keys, key_idx = arr(keys64.reshape(-1), np.uint8), None

    def repack(buf, off, ln):
        total = int(ln.sum(dtype=np.uint64))
        if n and (np.diff(off.astype(np.int64)) == ln[:-1].astype(np.int64)).all():
            return buf[int(off[0]):int(off[0]) + total]
        ex = np.zeros(n, np.int64)
        ex[1:] = np.cumsum(ln[:-1], dtype=np.int64)
        idx = np.repeat(off.astype(np.int64) - ex, ln.astype(np.int64)) + np.arange(total)
        return buf[idx]
    s_b = arr(repack(sig, sig_off, sig_len), np.uint8)
    m_b = arr(repack(msg, msg_off, msg_len), np.uint8)
    fixed = stride and n > 0 and (msg_len == msg_len[0]).all()
    out = {"keys": keys, "key_idx": key_idx, "sig": s_b, "sig_len": arr(sig_len, np.uint32),
           "msg": m_b, "msg_len": None if fixed else arr(msg_len, np.uint32)}
    cb = BhCBatch(keys.ctypes.data, key_idx.ctypes.data if key_idx is not None else None,
                  len(keys) // 64, s_b.ctypes.data if s_b.nbytes else None,
                  out["sig_len"].ctypes.data, m_b.ctypes.data if m_b.nbytes else None,
                  out["msg_len"].ctypes.data if out["msg_len"] is not None else None,
                  int(msg_len[0]) if fixed else 0)
    return out, cb


def pack_stats() -> dict:
    """bh_pack_stats: the last staged shard's packing (include/bdls_hip.h)."""
    import numpy as np
    out = np.zeros(10, np.float64)
    check(lib().bh_pack_stats(out.ctypes.data))
    return {k: float(v) for k, v in zip(PACK_STATS, out)}
