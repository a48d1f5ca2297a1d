"""BDLS agent-side batch pre-verification.

Mirror of what a patched `agent-tcp/tcp_peer.go:176-192` inputConsensusMessage
does with libbdlship.so: take the drained `[][]byte` of raw consensus
messages, run ONE bh_bdls_preverify (decode, participant gate, every
reachable SignedProto verified in one device batch, Go-ordered structural
checks), fill a verified-signature cache from the per-SignedProto results,
then hand the messages to the unchanged Consensus.ReceiveMessage, whose
SignedProto.Verify becomes a cache lookup. Status codes: include/bdls_hip.h
BH_BDLS_*.
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import numpy as np

from . import _lib

STATUS_NAMES = [
    "OK", "DECODE", "VERSION", "UNKNOWN_PARTICIPANT", "BAD_SIGNATURE", "MSG_DECODE",
    "UNKNOWN_TYPE", "EMPTY_STATE", "NOT_LEADER", "PROOF_UNKNOWN_PARTICIPANT",
    "PROOF_BAD_SIGNATURE", "PROOF_DECODE", "PROOF_TYPE_MISMATCH", "PROOF_HEIGHT_MISMATCH",
    "PROOF_ROUND_MISMATCH", "PROOF_INSUFFICIENT", "SELECT_STATE_MISMATCH",
    "SELECT_PROOF_EXCEEDED", "LOCKRELEASE_EMPTY"]
BH_BDLS_F_GIVEN_REASONS = 1
BH_BDLS_F_NO_QUORUM = 2
SP_NOT_VERIFIED = 255
CURVES = {"P-256": _lib.BH_CURVE_P256, "secp256k1": _lib.BH_CURVE_SECP256K1}


def preverify(curve: str, raw_msgs: Sequence[bytes], participants: Sequence[bytes],
              quorum: bool = True, given_reasons: np.ndarray | None = None):
    """-> (list of bh_bdls_msg_result as dicts, sp_reason u8[total]).

    given_reasons: per-SignedProto results supplied by the caller (cache hits;
    BH_BDLS_F_GIVEN_REASONS) -- then no device work is done."""
    L = _lib.lib()
    if given_reasons is None:
        _lib.ensure_init()
    n = len(raw_msgs)
    lens = np.fromiter((len(m) for m in raw_msgs), np.uint32, count=n)
    offs = np.zeros(n, np.uint64)
    if n:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    buf = np.frombuffer(b"".join(raw_msgs) + b"\0", np.uint8)
    parts = np.frombuffer(b"".join(participants) + b"\0", np.uint8)
    res = (_lib.BhBdlsMsgResult * max(n, 1))()
    flags = (0 if quorum else BH_BDLS_F_NO_QUORUM)
    total = ctypes.c_size_t()
    args = (CURVES[curve], buf.ctypes.data, offs.ctypes.data, lens.ctypes.data, n,
            parts.ctypes.data, len(participants))
    if given_reasons is not None:
        rs = np.ascontiguousarray(given_reasons, np.uint8).copy()
        _lib.check(L.bh_bdls_preverify(*args, flags | BH_BDLS_F_GIVEN_REASONS, res,
                                       rs.ctypes.data if rs.size else None, rs.size,
                                       ctypes.byref(total)))
        rs = rs[:total.value].copy()
        # the library returns the gated view: not-verified entries are not written back
    else:
        # every nested SignedProto occupies >= 2 bytes (tag + length) of its
        # parent, so n + bytes/2 bounds the flattened count: one call.
        rs = np.zeros(n + len(buf) // 2 + 1, np.uint8)
        _lib.check(L.bh_bdls_preverify(*args, flags, res, rs.ctypes.data, rs.size,
                                       ctypes.byref(total)))
        rs = rs[:total.value].copy()
    out = [{f: getattr(res[i], f) for f, _ in _lib.BhBdlsMsgResult._fields_} for i in range(n)]
    return out, rs
