"""CPU oracle for bh_verify_x509 (TEST INFRASTRUCTURE ONLY: tests/ and the
fixture generator import it; the product never does).

Restates Go 1.21 crypto/x509 Certificate.CheckSignatureFrom for an ECDSA
issuer -- checkSignature(algo, RawTBSCertificate, Signature, parent key):
hash the TBS with the algorithm's hash, then crypto/ecdsa VerifyASN1:
  parseSignature (golang.org/x/crypto/cryptobyte: ReadASN1 SEQUENCE with DER
  length rules, nothing after it; ReadASN1Integer into []byte =
  readASN1Bytes: minimal encoding, non-negative, leading zeros stripped;
  nothing after s), then verifyNISTEC: pointFromAffine, bigmod SetBytes of
  r and s (< n, non-zero), hashToNat, u1 G + u2 Q, x mod n == r. No low-S
  rule (Fabric's sanitizeCert, msp/cert.go:76-116, only rewrites s to n - s,
  which verifies identically).
The per-record reason follows the engine's order of checks (every reject is
`false` in Go): structure / algorithm -> BH_R_UNSUPPORTED, strict DER ->
BH_R_DER, zero r / s -> NONPOS, key -> BAD_KEY, r / s >= n -> RANGE, math.
"""
from __future__ import annotations

import hashlib

from . import ecdsa_ref as O

R_UNSUPPORTED = 11
OID_ECDSA_SHA256 = bytes.fromhex("2a8648ce3d040302")


def _cb_read(b: bytes, i: int, want: int):
    """cryptobyte readASN1 + tag compare -> (content, new index) or None."""
    if len(b) - i < 2:
        return None
    tag, lb = b[i], b[i + 1]
    if tag & 0x1F == 0x1F:
        return None
    if not lb & 0x80:
        hl, ln = 2, lb
    else:
        ll = lb & 0x7F
        if ll == 0 or ll > 4 or len(b) - i < 2 + ll:
            return None
        ln = int.from_bytes(b[i + 2:i + 2 + ll], "big")
        if ln < 128 or (ln >> ((ll - 1) * 8)) == 0:
            return None
        hl = 2 + ll
    if ln > len(b) - i - hl or tag != want:
        return None
    return b[i + hl:i + hl + ln], i + hl + ln


def _cb_uint(b: bytes, i: int):
    got = _cb_read(b, i, 0x02)
    if got is None:
        return None
    v, j = got
    if not v:
        return None
    if len(v) > 1 and ((v[0] == 0 and not v[1] & 0x80) or (v[0] == 0xFF and v[1] & 0x80)):
        return None
    if v[0] & 0x80:
        return None
    return int.from_bytes(v, "big"), j


def parse_signature(sig: bytes):
    """crypto/ecdsa parseSignature -> (r, s) or None."""
    got = _cb_read(sig, 0, 0x30)
    if got is None or got[1] != len(sig):
        return None
    inner = got[0]
    a = _cb_uint(inner, 0)
    if a is None:
        return None
    b = _cb_uint(inner, a[1])
    if b is None or b[1] != len(inner):
        return None
    return a[0], b[0]


def _tlv(b: bytes, i: int):
    """DER TLV -> (tag, content, raw, next) (the engine's structural walk)."""
    if i >= len(b) or b[i] & 0x1F == 0x1F or i + 1 >= len(b):
        return None
    ln = b[i + 1]
    j = i + 2
    if ln & 0x80:
        k = ln & 0x7F
        if k == 0 or k > 4 or j + k > len(b):
            return None
        ln = int.from_bytes(b[j:j + k], "big")
        if ln < 0x80 or (k > 1 and b[j] == 0):
            return None
        j += k
    if ln > len(b) - j:
        return None
    return b[i], b[j:j + ln], b[i:j + ln], j + ln


def split_cert(der: bytes):
    """(tbs_raw, inner_alg_oid, outer_alg_oid, signature) or None."""
    c = _tlv(der, 0)
    if c is None or c[0] != 0x30 or c[3] != len(der):
        return None
    body = c[1]
    tbs = _tlv(body, 0)
    if tbs is None or tbs[0] != 0x30:
        return None
    alg = _tlv(body, tbs[3])
    if alg is None or alg[0] != 0x30:
        return None
    sv = _tlv(body, alg[3])
    if sv is None or sv[0] != 0x03 or not sv[1] or sv[1][0] != 0:
        return None
    outer = _tlv(alg[1], 0)
    if outer is None or outer[0] != 0x06:
        return None
    t = _tlv(tbs[1], 0)
    if t is None:
        return None
    if t[0] == 0xA0:
        t = _tlv(tbs[1], t[3])
        if t is None:
            return None
    if t[0] != 0x02:
        return None
    inner_seq = _tlv(tbs[1], t[3])
    if inner_seq is None or inner_seq[0] != 0x30:
        return None
    inner = _tlv(inner_seq[1], 0)
    if inner is None:
        return None
    return tbs[2], inner[2], outer[2], sv[1][1:]


def check_signature_from(der: bytes, qx: int, qy: int) -> int:
    """BH_R_* of Certificate.CheckSignatureFrom(issuer with key (qx, qy))."""
    parts = split_cert(der)
    if parts is None:
        return R_UNSUPPORTED
    tbs, inner, outer, sig = parts
    if inner != outer or outer[2:] != OID_ECDSA_SHA256 or outer[1] != len(OID_ECDSA_SHA256):
        return R_UNSUPPORTED
    rs = parse_signature(sig)
    if rs is None:
        return O.R_DER
    r, s = rs
    c = O.P256
    if r == 0:
        return O.R_R_NONPOS
    if s == 0:
        return O.R_S_NONPOS
    return O.go_ecdsa_verify(c, qx, qy, hashlib.sha256(tbs).digest(), r, s)
