"""Synthetic verify workloads (BASELINE.json configs 2 and 5) from
bdls_amd/workload/gen.c (libbdlsgen.so). Data preparation only."""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

_LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib",
                    "libbdlsgen.so")
SIG_STRIDE = 80
CLASS_NAMES = ["none", "msg_flip", "high_s", "r_zero", "r_ge_n", "s_ge_n", "q_offcurve",
               "q_ge_p", "der_trailing_ok", "der_extra_ok", "der_nonminimal", "der_longlen"]


@dataclass
class Workload:
    pub: np.ndarray      # n*64 u8
    msg: np.ndarray      # n*msg_len u8
    msg_off: np.ndarray  # u64
    msg_len: np.ndarray  # u32
    sig: np.ndarray      # n*80 u8
    sig_off: np.ndarray  # u64
    sig_len: np.ndarray  # u32
    reason: np.ndarray   # expected reason u8 (by construction)
    cls: np.ndarray      # corruption class u8

    @property
    def n(self) -> int:
        return len(self.msg_len)

    @property
    def expected_valid(self) -> np.ndarray:
        return self.reason == 0

    def arrays(self):
        return (self.pub, self.sig, self.sig_off, self.sig_len, self.msg, self.msg_off,
                self.msg_len)


def generate(n: int, nkeys: int, msg_len: int = 256, corrupt_den: int = 16, seed: int = 2,
             nthreads: int | None = None) -> Workload:
    if not os.path.exists(_LIB):
        raise RuntimeError(f"{_LIB} not built (run `make`)")
    L = ctypes.CDLL(_LIB)
    vp = ctypes.c_void_p
    L.gen_p256.argtypes = [ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                           ctypes.c_uint64, ctypes.c_int] + [vp] * 9
    L.gen_p256.restype = ctypes.c_int
    if nthreads is None:
        nthreads = min(16, os.cpu_count() or 1)
    w = Workload(
        pub=np.empty(n * 64, np.uint8), msg=np.empty(n * msg_len, np.uint8),
        msg_off=np.empty(n, np.uint64), msg_len=np.empty(n, np.uint32),
        sig=np.zeros(n * SIG_STRIDE, np.uint8), sig_off=np.empty(n, np.uint64),
        sig_len=np.empty(n, np.uint32), reason=np.empty(n, np.uint8), cls=np.empty(n, np.uint8))
    rc = L.gen_p256(n, nkeys, msg_len, corrupt_den, seed, nthreads, w.pub.ctypes.data,
                    w.msg.ctypes.data, w.msg_off.ctypes.data, w.msg_len.ctypes.data,
                    w.sig.ctypes.data, w.sig_off.ctypes.data, w.sig_len.ctypes.data,
                    w.reason.ctypes.data, w.cls.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"gen_p256 failed: {rc}")
    return w
