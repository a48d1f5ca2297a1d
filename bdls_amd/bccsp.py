"""Host-side mirror of the reference's BCCSP provider interface for the verify
hot path, backed by the HIP engine (libbdlship.so).

Mirrors (names, argument meaning, error behaviour):
  bccsp/bccsp.go:90-134        BCCSP.Verify / Hash / KeyImport
  bccsp/sw/impl.go:247-270     CSP.Verify argument checks and error wrapping
  bccsp/sw/ecdsa.go:41-57      verifyECDSA
  bccsp/utils/ecdsa.go:41-89   UnmarshalECDSASignature / IsLowS
  msp/identities.go:170-199    identity.Verify (SHA-256 then Verify)
and adds the batch entry points a `bccsp/hip` provider exposes:
  BatchVerify(keys, signatures, digests)          -> valid[], errors[]
  BatchIdentityVerify(keys, messages, signatures) -> fused SHA-256 + verify

A Go `(false, err)` is raised here as BCCSPError; `(false, nil)` returns False,
exactly as the reference distinguishes them. Batch calls return per-record
reason codes instead of raising.
"""
from __future__ import annotations

import ctypes
import hashlib
from dataclasses import dataclass
from typing import Sequence

import numpy as np

from . import _lib
from ._lib import BH_F_HASH_SHA256, BH_F_HASH_SHA3_256, BH_F_NO_LOW_S, BhBatch

# reason codes (include/bdls_hip.h)
R_OK, R_EMPTY_SIG, R_EMPTY_DIGEST, R_DER, R_R_NONPOS, R_S_NONPOS, R_HIGH_S = range(7)
R_BAD_KEY, R_R_RANGE, R_MATH, R_S_RANGE = 7, 8, 9, 10
ERROR_REASONS = frozenset({R_EMPTY_SIG, R_EMPTY_DIGEST, R_DER, R_R_NONPOS, R_S_NONPOS, R_HIGH_S})

P256_N = 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551
P256_HALF_N = P256_N >> 1

# Go error strings (bccsp/sw/impl.go, bccsp/sw/ecdsa.go, bccsp/utils/ecdsa.go)
_ERR_TEXT = {
    R_EMPTY_SIG: "Invalid signature. Cannot be empty.",
    R_EMPTY_DIGEST: "Invalid digest. Cannot be empty.",
    R_DER: "Failed verifing with opts [%s]: Failed unmashalling signature [failed unmashalling signature]",
    R_R_NONPOS: "Failed verifing with opts [%s]: Failed unmashalling signature [invalid signature, R must be larger than zero]",
    R_S_NONPOS: "Failed verifing with opts [%s]: Failed unmashalling signature [invalid signature, S must be larger than zero]",
    R_HIGH_S: "Failed verifing with opts [%s]: Invalid S. Must be smaller than half the order [%s][" + str(P256_HALF_N) + "].",
}


class BCCSPError(Exception):
    """A Go `(false, err)` result of BCCSP.Verify."""

    def __init__(self, reason: int, msg: str):
        super().__init__(msg)
        self.reason = reason


@dataclass(frozen=True)
class ECDSAPublicKey:
    """bccsp/sw/ecdsakey.go:72 ecdsaPublicKey (P-256 only on this provider)."""
    x: int
    y: int
    curve: str = "P-256"

    def raw64(self) -> bytes:
        if self.x < 0 or self.y < 0 or self.x.bit_length() > 256 or self.y.bit_length() > 256:
            # pointFromAffine rejects these; encode an off-curve marker the engine rejects
            return b"\x00" * 64
        return self.x.to_bytes(32, "big") + self.y.to_bytes(32, "big")

    def symmetric(self) -> bool:
        return False

    def private(self) -> bool:
        return False


class ECDSAGoPublicKeyImportOpts:
    """bccsp/opts.go ECDSAGoPublicKeyImportOpts (raw = (x, y))."""


class SHA256Opts:
    """bccsp/hashopts.go SHA256Opts."""


class SHA3_256Opts:
    """bccsp/hashopts.go SHA3_256Opts."""


# msp/identities.go:219-227 getHashOpt: MSP SignatureHashFamily -> device hash flag
_FAMILY_FLAG = {"SHA2": BH_F_HASH_SHA256, "SHA3": BH_F_HASH_SHA3_256}


def family_flag(family: str) -> int:
    if family not in _FAMILY_FLAG:
        raise BCCSPError(-1, f"hash family not recognized [{family}]")
    return _FAMILY_FLAG[family]


def _arr(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


def pack_records(keys: Sequence[ECDSAPublicKey], sigs: Sequence[bytes], msgs: Sequence[bytes]):
    """SoA packing of a batch (host numpy buffers)."""
    n = len(keys)
    pub = np.frombuffer(b"".join(k.raw64() for k in keys) or b"\0", dtype=np.uint8)
    sig_len = np.fromiter((len(s) for s in sigs), dtype=np.uint32, count=n)
    msg_len = np.fromiter((len(m) for m in msgs), dtype=np.uint32, count=n)
    sig_off = np.zeros(n, dtype=np.uint64)
    msg_off = np.zeros(n, dtype=np.uint64)
    if n:
        sig_off[1:] = np.cumsum(sig_len[:-1], dtype=np.uint64)
        msg_off[1:] = np.cumsum(msg_len[:-1], dtype=np.uint64)
    sig = np.frombuffer(b"".join(sigs) + b"\0", dtype=np.uint8)
    msg = np.frombuffer(b"".join(msgs) + b"\0", dtype=np.uint8)
    return pub, sig, sig_off, sig_len, msg, msg_off, msg_len


def verify_packed(pub, sig, sig_off, sig_len, msg, msg_off, msg_len, flags: int = 0):
    """Host-buffer batch through bh_verify. Returns (valid bool[n], reason u8[n])."""
    _lib.ensure_init()
    n = len(sig_len)
    bitmap = np.zeros((n + 7) // 8 or 1, dtype=np.uint8)
    reason = np.zeros(n or 1, dtype=np.uint8)
    b = BhBatch(_arr(pub), _arr(sig), _arr(sig_off), _arr(sig_len), _arr(msg), _arr(msg_off),
                _arr(msg_len))
    _lib.check(_lib.lib().bh_verify(_lib.BH_CURVE_P256, ctypes.byref(b), n, flags,
                                    bitmap.ctypes.data, reason.ctypes.data))
    valid = np.unpackbits(bitmap, bitorder="little")[:n].astype(bool)
    return valid, reason[:n]


class HipCSP:
    """The `bccsp/hip` provider's verify/hash surface (embeds sw semantics)."""

    def __init__(self, device_mask: int = 0, low_s: bool = True):
        self._flags = 0 if low_s else BH_F_NO_LOW_S
        _lib.ensure_init(device_mask)

    # -- BCCSP.Hash (bccsp/sw/hash.go:29-33). Single-message hashing stays on the
    # host like sw; batched hashing is fused into BatchIdentityVerify on device.
    def hash(self, msg: bytes, opts=None) -> bytes:
        if isinstance(opts, SHA3_256Opts):
            return hashlib.sha3_256(msg).digest()
        return hashlib.sha256(msg).digest()

    def key_import(self, raw, opts) -> ECDSAPublicKey:
        if isinstance(opts, ECDSAGoPublicKeyImportOpts):
            x, y = raw
            return ECDSAPublicKey(int(x), int(y))
        raise BCCSPError(-1, f"Unsupported 'KeyImportOpts' provided [{opts}]")

    # -- BCCSP.Verify (bccsp/sw/impl.go:247-270 -> sw/ecdsa.go:41-57)
    def verify(self, k, signature: bytes, digest: bytes, opts=None) -> bool:
        if k is None:
            raise BCCSPError(-1, "Invalid Key. It must not be nil.")
        if not isinstance(k, ECDSAPublicKey) or k.curve != "P-256":
            raise BCCSPError(-1, f"Unsupported 'VerifyKey' provided [{k}]")
        sig, dg = bytes(signature or b""), bytes(digest or b"")
        if self._flags:  # a no-low-S provider: plain one-record batch
            valid, reason = verify_packed(*pack_records([k], [sig], [dg]), flags=self._flags)
            return self._result(int(reason[0]), bool(valid[0]), opts)
        # bh_csp_verify_p256: concurrent callers share device passes (coalescer);
        # ctypes releases the GIL for the call
        v, r = ctypes.c_int(), ctypes.c_int()
        _lib.check(_lib.lib().bh_csp_verify_p256(k.raw64(), sig, len(sig), dg, len(dg),
                                                 ctypes.byref(v), ctypes.byref(r)))
        return self._result(r.value, bool(v.value), opts)

    def _result(self, reason: int, valid: bool, opts) -> bool:
        if reason in ERROR_REASONS:
            txt = _ERR_TEXT[reason]
            if "%s" in txt:
                txt = txt.replace("%s", str(opts), 1).replace("%s", "", 1)
            raise BCCSPError(reason, txt)
        return valid

    # -- batch extensions
    def batch_verify(self, keys: Sequence[ECDSAPublicKey], signatures: Sequence[bytes],
                     digests: Sequence[bytes]):
        """Returns (valid bool[n], reason u8[n]); reason in ERROR_REASONS <=> Go error."""
        return verify_packed(*pack_records(keys, signatures, digests), flags=self._flags)

    def batch_identity_verify(self, keys: Sequence[ECDSAPublicKey], messages: Sequence[bytes],
                              signatures: Sequence[bytes], family: str = "SHA2"):
        """msp/identities.go:170-199 for a whole batch with the MSP's hash family
        (SHA2 -> SHA-256, SHA3 -> SHA3-256) fused on device."""
        return verify_packed(*pack_records(keys, signatures, messages),
                             flags=self._flags | family_flag(family))

    def identity_verify(self, k, msg: bytes, sig: bytes, family: str = "SHA2") -> None:
        """identity.Verify: raises on error or invalid signature (returns None if valid)."""
        valid, reason = self.batch_identity_verify([k], [msg], [sig], family)
        r = int(reason[0])
        if r in ERROR_REASONS:
            raise BCCSPError(r, "could not determine the validity of the signature: " +
                             _ERR_TEXT[r].replace("%s", "<nil>", 1).replace("%s", "", 1))
        if not valid[0]:
            raise BCCSPError(r, "The signature is invalid")


def parse_der_sig(der: bytes):
    """bh_parse_der_sig (host, Go-asn1 exact). Returns (reason, r|None, s|None)."""
    L = _lib.lib()
    r = ctypes.create_string_buffer(32)
    s = ctypes.create_string_buffer(32)
    rb, sb = ctypes.c_int(), ctypes.c_int()
    buf = ctypes.create_string_buffer(bytes(der), max(1, len(der)))
    rc = L.bh_parse_der_sig(ctypes.cast(buf, ctypes.c_void_p), len(der), ctypes.cast(r, ctypes.c_void_p),
                            ctypes.cast(s, ctypes.c_void_p), ctypes.byref(rb), ctypes.byref(sb))
    if rc < 0:
        raise _lib.EngineError(_lib.last_error())
    if rc != R_OK:
        return rc, None, None
    rv = None if rb.value else int.from_bytes(r.raw, "big")
    sv = None if sb.value else int.from_bytes(s.raw, "big")
    return rc, rv, sv
