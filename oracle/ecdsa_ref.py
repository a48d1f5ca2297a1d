"""CPU ORACLE (test infrastructure only) -- pure-Python restatement of the ECDSA
acceptance predicate on the reference's signature-verification hot path.

*** This module is a CHECKER. Only tests/, __graft_entry__.smoke() and bench.py's
*** cpu_baseline leg may import it. The product path (bdls_amd/, libbdlship.so)
*** never imports, links or calls anything under oracle/.

What it restates (reference = /root/reference, hyperledger-labs/bdls @ 2025-07-18):

* bccsp/sw/impl.go:247-270      CSP.Verify argument checks (nil key / empty sig /
                                 empty digest -> (false, error)).
* bccsp/sw/ecdsa.go:41-57       verifyECDSA: UnmarshalECDSASignature -> IsLowS ->
                                 ecdsa.Verify.
* bccsp/utils/ecdsa.go:41-65    UnmarshalECDSASignature = encoding/asn1.Unmarshal
                                 into struct{R,S *big.Int} (rest discarded), then
                                 R > 0, S > 0.
* bccsp/utils/ecdsa.go:26-31,82-89  curveHalfOrders / IsLowS: S <= floor(n/2).
* Go 1.21.4 stdlib (pinned by reference Makefile:81 GO_VER, NOT vendored under
  /root/reference): encoding/asn1 parseTagAndLength/parseField/parseBigInt/
  checkInteger; crypto/ecdsa Verify -> VerifyASN1 -> verifyNISTEC (P-256),
  hashToNat, pointFromAffine; verifyLegacy + hashToInt for non-NIST curves
  (secp256k1 as used by vendor/github.com/BDLS-bft/bdls/message.go:170-184).
* vendor/github.com/BDLS-bft/bdls/message.go:97-138  SignedProto.Hash
  (BLAKE2b-256 over prefix|version|X|Y|len|msg).

Parity pinning: the DER rules are pinned by the reference's own fixed vectors
(bccsp/sw/impl_test.go:924-961, bccsp/utils/ecdsa_test.go:19-110) and the curve
arithmetic by the fixed certificate fixture msp/testdata/mspid (a real P-256
ECDSA-SHA256 signature chain produced outside this repo); the full fixture set is
additionally cross-checked against OpenSSL libcrypto (oracle/orc.c).
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass

# ----------------------------------------------------------------------------
# Reason codes -- MUST match include/bdls_hip.h (BH_R_*).
# Codes 1..6 are Go `(false, error)`; 7..9 are Go `(false, nil)`.
# ----------------------------------------------------------------------------
R_OK = 0
R_EMPTY_SIG = 1        # impl.go:252-254
R_EMPTY_DIGEST = 2     # impl.go:255-257
R_DER = 3              # utils/ecdsa.go:44-47 (asn1.Unmarshal error)
R_R_NONPOS = 4         # utils/ecdsa.go:57-59
R_S_NONPOS = 5         # utils/ecdsa.go:60-62
R_HIGH_S = 6           # sw/ecdsa.go:52-54
R_BAD_KEY = 7          # Go pointFromAffine error inside ecdsa.Verify -> false
R_R_RANGE = 8          # bigmod SetBytes(r, N) error (r >= n) -> false
R_MATH = 9             # u1*G + u2*Q == inf, or x mod n != r -> false
R_S_RANGE = 10         # s >= n inside ecdsa.Verify (only reachable w/o low-S rule)

ERROR_REASONS = {R_EMPTY_SIG, R_EMPTY_DIGEST, R_DER, R_R_NONPOS, R_S_NONPOS, R_HIGH_S}

REASON_NAMES = {
    R_OK: "ok", R_EMPTY_SIG: "empty_sig", R_EMPTY_DIGEST: "empty_digest",
    R_DER: "der", R_R_NONPOS: "r_nonpos", R_S_NONPOS: "s_nonpos",
    R_HIGH_S: "high_s", R_BAD_KEY: "bad_key", R_R_RANGE: "r_range",
    R_MATH: "math", R_S_RANGE: "s_range",
}


@dataclass(frozen=True)
class Curve:
    name: str
    p: int
    a: int
    b: int
    n: int
    gx: int
    gy: int
    nist: bool  # True -> Go verifyNISTEC path; False -> verifyLegacy path


P256 = Curve(
    name="P-256",
    p=2**256 - 2**224 + 2**192 + 2**96 - 1,
    a=-3,
    b=0x5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B,
    n=0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551,
    gx=0x6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296,
    gy=0x4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5,
    nist=True,
)

# vendor/github.com/BDLS-bft/bdls/crypto/btcec/btcec.go:924-931 (initS256)
SECP256K1 = Curve(
    name="secp256k1",
    p=2**256 - 2**32 - 977,
    a=0,
    b=7,
    n=0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141,
    gx=0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798,
    gy=0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8,
    nist=False,
)


def half_order(c: Curve) -> int:
    """bccsp/utils/ecdsa.go:26-31  new(big.Int).Rsh(N, 1)."""
    return c.n >> 1


# ----------------------------------------------------------------------------
# Curve arithmetic (Jacobian, plain Python ints). Textbook formulas; speed is
# irrelevant -- this is the checker.
# ----------------------------------------------------------------------------
INF = None


def on_curve(c: Curve, x: int, y: int) -> bool:
    return (y * y - (x * x * x + c.a * x + c.b)) % c.p == 0


def _to_jac(pt):
    return None if pt is None else (pt[0], pt[1], 1)


def _from_jac(c: Curve, J):
    if J is None or J[2] % c.p == 0:
        return None
    X, Y, Z = J
    zi = pow(Z, -1, c.p)
    return (X * zi * zi % c.p, Y * zi * zi * zi % c.p)


def _jdbl(c: Curve, J):
    if J is None:
        return None
    X, Y, Z = J
    p = c.p
    if Y % p == 0:
        return None
    S = 4 * X * Y * Y % p
    M = (3 * X * X + c.a * pow(Z, 4, p)) % p
    X3 = (M * M - 2 * S) % p
    Y3 = (M * (S - X3) - 8 * pow(Y, 4, p)) % p
    Z3 = 2 * Y * Z % p
    return (X3, Y3, Z3)


def _jadd(c: Curve, J1, J2):
    if J1 is None:
        return J2
    if J2 is None:
        return J1
    p = c.p
    X1, Y1, Z1 = J1
    X2, Y2, Z2 = J2
    Z1Z1 = Z1 * Z1 % p
    Z2Z2 = Z2 * Z2 % p
    U1 = X1 * Z2Z2 % p
    U2 = X2 * Z1Z1 % p
    S1 = Y1 * Z2 * Z2Z2 % p
    S2 = Y2 * Z1 * Z1Z1 % p
    if U1 == U2:
        if S1 != S2:
            return None
        return _jdbl(c, J1)
    H = (U2 - U1) % p
    R = (S2 - S1) % p
    H2 = H * H % p
    H3 = H * H2 % p
    U1H2 = U1 * H2 % p
    X3 = (R * R - H3 - 2 * U1H2) % p
    Y3 = (R * (U1H2 - X3) - S1 * H3) % p
    Z3 = H * Z1 * Z2 % p
    return (X3, Y3, Z3)


def _jmul(c: Curve, k: int, J):
    R = None
    for bit in bin(k)[2:] if k > 0 else "":
        R = _jdbl(c, R)
        if bit == "1":
            R = _jadd(c, R, J)
    return R


def point_add(c: Curve, P1, P2):
    return _from_jac(c, _jadd(c, _to_jac(P1), _to_jac(P2)))


def scalar_mult(c: Curve, k: int, pt):
    """k*pt in affine (None = point at infinity)."""
    return _from_jac(c, _jmul(c, k % c.n, _to_jac(pt)))


def double_scalar(c: Curve, u1: int, u2: int, Q):
    """u1*G + u2*Q, the verify equation (affine result or None)."""
    A = _jmul(c, u1 % c.n, (c.gx, c.gy, 1))
    Bq = _jmul(c, u2 % c.n, _to_jac(Q))
    return _from_jac(c, _jadd(c, A, Bq))


# ----------------------------------------------------------------------------
# encoding/asn1 (Go 1.21.4) restatement, only as far as Unmarshal(raw,
# &struct{R, S *big.Int}) exercises it (bccsp/utils/ecdsa.go:44).
# ----------------------------------------------------------------------------
class Asn1Error(Exception):
    pass


def _parse_tag_and_length(b: bytes, off: int):
    """Go asn1.parseTagAndLength. Returns (cls, compound, tag, length, off)."""
    if off >= len(b):
        raise Asn1Error("internal error in parseTagAndLength")
    t = b[off]
    off += 1
    cls = t >> 6
    compound = (t & 0x20) == 0x20
    tag = t & 0x1F
    if tag == 0x1F:
        # parseBase128Int (Go 1.21): at most 4 bytes / 31 bits, no leading 0x80
        ret = 0
        shifted = 0
        while True:
            if off >= len(b):
                raise Asn1Error("truncated base 128 integer")
            if shifted == 5:  # 5*7 bits > 31
                raise Asn1Error("base 128 integer too large")
            ret <<= 7
            x = b[off]
            if shifted == 0 and x == 0x80:
                raise Asn1Error("integer is not minimally encoded")
            ret |= x & 0x7F
            off += 1
            shifted += 1
            if x & 0x80 == 0:
                if ret > 0x7FFFFFFF:
                    raise Asn1Error("base 128 integer too large")
                break
        tag = ret
        if tag < 0x1F:
            raise Asn1Error("non-minimal tag")
    if off >= len(b):
        raise Asn1Error("truncated tag or length")
    lb = b[off]
    off += 1
    if lb & 0x80 == 0:
        length = lb & 0x7F
    else:
        nbytes = lb & 0x7F
        if nbytes == 0:
            raise Asn1Error("indefinite length found (not DER)")
        length = 0
        for _ in range(nbytes):
            if off >= len(b):
                raise Asn1Error("truncated tag or length")
            x = b[off]
            off += 1
            if length >= 1 << 23:
                raise Asn1Error("length too large")
            length = (length << 8) | x
            if length == 0:
                raise Asn1Error("superfluous leading zeros in length")
        if length < 0x80:
            raise Asn1Error("non-minimal length")
    return cls, compound, tag, length, off


def _parse_big_int(body: bytes) -> int:
    """Go asn1.parseBigInt + checkInteger."""
    if len(body) == 0:
        raise Asn1Error("empty integer")
    if len(body) > 1 and (
        (body[0] == 0 and body[1] & 0x80 == 0) or (body[0] == 0xFF and body[1] & 0x80 == 0x80)
    ):
        raise Asn1Error("integer not minimally-encoded")
    return int.from_bytes(body, "big", signed=True)


def _parse_int_field(b: bytes, off: int):
    """parseField for a *big.Int field (universal INTEGER, primitive)."""
    if off == len(b):
        raise Asn1Error("sequence truncated")
    cls, compound, tag, length, off = _parse_tag_and_length(b, off)
    if cls != 0 or tag != 2 or compound:
        raise Asn1Error("tags don't match")
    if off + length > len(b):
        raise Asn1Error("data truncated")
    return _parse_big_int(b[off:off + length]), off + length


def asn1_unmarshal_ecdsa_sig(raw: bytes):
    """asn1.Unmarshal(raw, &ECDSASignature{}) -> (R, S, rest). Raises Asn1Error."""
    raw = bytes(raw)
    if len(raw) == 0:
        # parseField: offset == len(bytes) -> setDefaultValue fails -> "sequence truncated"
        raise Asn1Error("sequence truncated")
    cls, compound, tag, length, off = _parse_tag_and_length(raw, 0)
    if cls != 0 or tag != 16 or not compound:
        raise Asn1Error("tags don't match")
    if off + length > len(raw):
        raise Asn1Error("data truncated")
    inner = raw[off:off + length]
    rest = raw[off + length:]
    r, ioff = _parse_int_field(inner, 0)
    s, ioff = _parse_int_field(inner, ioff)
    # Extra elements after S inside the SEQUENCE are accepted (Go parseField
    # "We allow extra bytes at the end of the SEQUENCE").
    return r, s, rest


def unmarshal_ecdsa_signature(raw: bytes):
    """bccsp/utils/ecdsa.go:41-65. Returns (reason, R, S)."""
    try:
        r, s, _rest = asn1_unmarshal_ecdsa_sig(raw)
    except Asn1Error:
        return R_DER, None, None
    if r <= 0:
        return R_R_NONPOS, r, s
    if s <= 0:
        return R_S_NONPOS, r, s
    return R_OK, r, s


def asn1_marshal_int(v: int) -> bytes:
    """Go asn1 INTEGER body (two's complement, minimal)."""
    if v == 0:
        return b"\x00"
    if v > 0:
        nb = (v.bit_length() + 8) // 8  # room for a sign bit
        out = v.to_bytes(nb, "big")
        while len(out) > 1 and out[0] == 0 and out[1] & 0x80 == 0:
            out = out[1:]
        return out
    nb = ((-v - 1).bit_length() + 8) // 8
    out = v.to_bytes(max(nb, 1), "big", signed=True)
    while len(out) > 1 and out[0] == 0xFF and out[1] & 0x80 == 0x80:
        out = out[1:]
    return out


def der_len(n: int) -> bytes:
    if n < 0x80:
        return bytes([n])
    body = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(body)]) + body


def marshal_ecdsa_signature(r: int, s: int) -> bytes:
    """bccsp/utils/ecdsa.go:37-39 MarshalECDSASignature (asn1.Marshal)."""
    rb, sb = asn1_marshal_int(r), asn1_marshal_int(s)
    body = b"\x02" + der_len(len(rb)) + rb + b"\x02" + der_len(len(sb)) + sb
    return b"\x30" + der_len(len(body)) + body


# ----------------------------------------------------------------------------
# crypto/ecdsa (Go 1.21.4)
# ----------------------------------------------------------------------------
def hash_to_nat(c: Curve, digest: bytes) -> int:
    """Go hashToNat (NIST path): left-most 32 bytes, then SetOverflowingBytes (mod n)."""
    size = (c.n.bit_length() + 7) // 8
    h = digest[:size] if len(digest) >= size else digest
    excess = len(h) * 8 - c.n.bit_length()
    v = int.from_bytes(h, "big")
    if excess > 0:
        v >>= excess
    return v % c.n


def hash_to_int(c: Curve, digest: bytes) -> int:
    """Go hashToInt (legacy path): left-most orderBytes, shift excess; NO reduction."""
    order_bits = c.n.bit_length()
    order_bytes = (order_bits + 7) // 8
    h = digest[:order_bytes]
    v = int.from_bytes(h, "big")
    excess = len(h) * 8 - order_bits
    if excess > 0:
        v >>= excess
    return v


def go_ecdsa_verify(c: Curve, qx: int, qy: int, digest: bytes, r: int, s: int) -> int:
    """crypto/ecdsa.Verify(pub, hash, r, s) -> reason (R_OK iff true).

    NIST path (verifyNISTEC): pointFromAffine rejects negative / >bitSize /
    >= p / off-curve coordinates *before* the r, s range checks; r, s must be in
    [1, n-1]; e = hashToNat; (x, y) = u1 G + u2 Q; infinity -> false; x mod n == r.
    Legacy path (verifyLegacy, secp256k1 as wired in BDLS): r, s in [1, n-1],
    e = hashToInt, no on-curve check, infinity (0,0) -> false, x mod n == r.
    """
    if r <= 0 or s <= 0:
        return R_R_NONPOS if r <= 0 else R_S_NONPOS
    if c.nist:
        if qx < 0 or qy < 0 or qx >= c.p or qy >= c.p or not on_curve(c, qx, qy):
            return R_BAD_KEY
        if r >= c.n:
            return R_R_RANGE
        if s >= c.n:
            return R_S_RANGE
        e = hash_to_nat(c, digest)
    else:
        if r >= c.n:
            return R_R_RANGE
        if s >= c.n:
            return R_S_RANGE
        e = hash_to_int(c, digest)
    w = pow(s, -1, c.n)
    u1 = e * w % c.n
    u2 = r * w % c.n
    if c.nist:
        pt = double_scalar(c, u1, u2, (qx, qy))
    else:
        # verifyLegacy: x1,y1 = ScalarBaseMult(u1); x2,y2 = ScalarMult(Q,u2);
        # x,y = Add(...). btcec's affine formulas on an off-curve Q are not
        # modelled: BDLS gates participants before verify (consensus.go:456-466).
        pt = double_scalar(c, u1, u2, (qx, qy))
    if pt is None:
        return R_MATH
    return R_OK if pt[0] % c.n == r else R_MATH


def csp_verify(c: Curve, qx: int, qy: int, sig: bytes, digest: bytes):
    """bccsp/sw/impl.go:247-270 + bccsp/sw/ecdsa.go:41-57 -> (valid, reason).

    valid is True iff reason == R_OK; reason in ERROR_REASONS means Go returned
    a non-nil error.
    """
    if len(sig) == 0:
        return False, R_EMPTY_SIG
    if len(digest) == 0:
        return False, R_EMPTY_DIGEST
    reason, r, s = unmarshal_ecdsa_signature(sig)
    if reason != R_OK:
        return False, reason
    if s > half_order(c):  # IsLowS: s.Cmp(halfOrder) != 1
        return False, R_HIGH_S
    reason = go_ecdsa_verify(c, qx, qy, digest, r, s)
    return reason == R_OK, reason


def identity_verify(c: Curve, qx: int, qy: int, msg: bytes, sig: bytes, family: str = "SHA2"):
    """msp/identities.go:170-199: digest = Hash(msg) with the MSP's hash family
    (getHashOpt :219-227: SHA2 -> SHA-256, SHA3 -> SHA3-256, the sha3.New256 of
    bccsp/sw/new.go:72), then Verify."""
    return csp_verify(c, qx, qy, sig, family_digest(family, msg))


def family_digest(family: str, msg: bytes) -> bytes:
    """bccsp/sw/new.go:70-72 hashers for identity.getHashOpt (identities.go:219-227)."""
    if family == "SHA2":
        return hashlib.sha256(msg).digest()
    if family == "SHA3":
        return hashlib.sha3_256(msg).digest()
    raise ValueError(f"hash family not recognized [{family}]")


# ----------------------------------------------------------------------------
# Signing helpers (fixture generation only; mirrors bccsp/sw/ecdsa.go:27-39
# signECDSA = ecdsa.Sign + ToLowS + Marshal, with a caller-supplied nonce so
# the fixtures are reproducible).
# ----------------------------------------------------------------------------
def pubkey(c: Curve, d: int):
    return scalar_mult(c, d, (c.gx, c.gy))


def sign_digest(c: Curve, d: int, digest: bytes, k: int, low_s: bool = True):
    e = hash_to_nat(c, digest) if c.nist else hash_to_int(c, digest) % c.n
    R = scalar_mult(c, k, (c.gx, c.gy))
    r = R[0] % c.n
    s = pow(k, -1, c.n) * (e + r * d) % c.n
    if low_s and s > half_order(c):
        s = c.n - s
    return r, s


# ----------------------------------------------------------------------------
# BDLS SignedProto hash (vendor/github.com/BDLS-bft/bdls/message.go:97-138)
# ----------------------------------------------------------------------------
BDLS_SIGNATURE_PREFIX = b"BDLS_CONSENSUS_SIGNATURE"  # message.go SignaturePrefix
BDLS_PROTOCOL_VERSION = 1                            # consensus.go:22


def bdls_signed_proto_hash(version: int, x32: bytes, y32: bytes, message: bytes) -> bytes:
    h = hashlib.blake2b(digest_size=32)
    h.update(BDLS_SIGNATURE_PREFIX)
    h.update(int(version).to_bytes(4, "little"))
    h.update(x32)
    h.update(y32)
    h.update(len(message).to_bytes(4, "little"))
    h.update(message)
    return h.digest()


def bdls_signed_proto_verify(c: Curve, version: int, x32: bytes, y32: bytes,
                             message: bytes, rbytes: bytes, sbytes: bytes) -> bool:
    """message.go:170-184: R, S are raw big-endian bytes (SetBytes, any length)."""
    digest = bdls_signed_proto_hash(version, x32, y32, message)
    r = int.from_bytes(rbytes, "big")
    s = int.from_bytes(sbytes, "big")
    return go_ecdsa_verify(c, int.from_bytes(x32, "big"), int.from_bytes(y32, "big"),
                           digest, r, s) == R_OK
