#!/usr/bin/env python3
"""Generate the committed golden fixtures for the P-256 verify path.

Run from the repo root:  python tests/golden/gen_golden.py
Outputs (committed):
  tests/golden/p256_vectors.jsonl   one record per line (hex fields)
  tests/golden/mspid_fixture.json   values extracted from the reference's
                                    msp/testdata/mspid certificates

Every expected (valid, reason) comes from oracle/ecdsa_ref.py (the CPU
restatement); tests/test_oracle_golden.py re-derives them and
oracle/orc.c cross-checks the curve math against OpenSSL libcrypto.

Sources of fixed data from the reference (read as data, never executed):
  * bccsp/sw/impl_test.go:924-961      five DER vectors that must be rejected
  * bccsp/utils/ecdsa_test.go:19-110   R/S in {-1,0} rejects, S = n/2 boundary
  * bccsp/sw/ecdsa_test.go:47-74       11-byte "digest" ("hello world")
  * msp/testdata/mspid/{cacerts,signcerts}/*.pem  real CA-issued P-256
    signatures (high-S: ECDSA-valid but Fabric-reject) -- only used when
    /root/reference is present; the extracted values are committed in
    mspid_fixture.json so the GPU box never needs the reference.
"""
from __future__ import annotations

import base64
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import ecdsa_ref as O  # noqa: E402

C = O.P256
N, P = C.n, C.p
HALF = N >> 1
REF = "/root/reference"


def h32(v: int) -> str:
    return v.to_bytes(32, "big").hex()


def rec(tag, qx, qy, sig: bytes, digest: bytes | None = None, msg: bytes | None = None):
    if msg is not None:
        digest = hashlib.sha256(msg).digest()
    valid, reason = O.csp_verify(C, qx, qy, sig, digest)
    out = {"tag": tag, "qx": h32(qx), "qy": h32(qy), "sig": sig.hex(),
           "digest": digest.hex(), "valid": valid, "reason": reason}
    if msg is not None:
        out["msg"] = msg.hex()
    return out


def der_raw(*elems: bytes, outer_tag=0x30, trailing=b"") -> bytes:
    body = b"".join(elems)
    return bytes([outer_tag]) + O.der_len(len(body)) + body + trailing


def der_int(v: int) -> bytes:
    b = O.asn1_marshal_int(v)
    return b"\x02" + O.der_len(len(b)) + b


def der_int_body(body: bytes, lenbytes: bytes | None = None) -> bytes:
    return b"\x02" + (lenbytes if lenbytes is not None else O.der_len(len(body))) + body


def find_wrap_point(rng):
    """A curve point with x in [n, p) (x mod n wraps). p - n ~ 2^128, so build it
    directly: pick x in [n, p) until x^3 - 3x + b is a square mod p."""
    while True:
        x = N + rng.randrange(P - N)
        rhs = (x * x * x - 3 * x + C.b) % P
        y = pow(rhs, (P + 1) // 4, P)  # p = 3 mod 4
        if y * y % P == rhs:
            return x, y


def pem_body(path):
    lines = open(path).read().strip().splitlines()
    return base64.b64decode("".join(l for l in lines if not l.startswith("-----")))


def der_tlv(b, off):
    """Minimal DER walker (lengths are DER-minimal in real certs)."""
    tag = b[off]
    lb = b[off + 1]
    if lb < 0x80:
        ln, hdr = lb, 2
    else:
        nb = lb & 0x7F
        ln = int.from_bytes(b[off + 2:off + 2 + nb], "big")
        hdr = 2 + nb
    return tag, off + hdr, ln, off + hdr + ln  # tag, content start, length, end


def cert_parts(der: bytes):
    """Certificate ::= SEQUENCE { tbs, sigAlg, BIT STRING sig }."""
    _, c0, _, _ = der_tlv(der, 0)
    _, _, _, tbs_end = der_tlv(der, c0)
    tbs = der[c0:tbs_end]
    _, _, _, alg_end = der_tlv(der, tbs_end)
    tag, bs, ln, _ = der_tlv(der, alg_end)
    assert tag == 0x03
    sig = der[bs + 1:bs + ln]  # skip unused-bits octet
    return tbs, sig


def cert_pubkey(der: bytes):
    """Find the 65-byte uncompressed point inside the SubjectPublicKeyInfo."""
    i = der.find(bytes.fromhex("034200"))
    pt = der[i + 3:i + 3 + 65]
    assert pt[0] == 4
    return int.from_bytes(pt[1:33], "big"), int.from_bytes(pt[33:65], "big")


def mspid_fixture():
    path = os.path.join(HERE, "mspid_fixture.json")
    ca = os.path.join(REF, "msp/testdata/mspid/cacerts/ca.example.com-cert.pem")
    peer = os.path.join(REF, "msp/testdata/mspid/signcerts/peer0-cert.pem")
    if os.path.exists(ca):
        ca_der, peer_der = pem_body(ca), pem_body(peer)
        qx, qy = cert_pubkey(ca_der)
        fx = {"source": "msp/testdata/mspid (reference fixture, extracted by gen_golden.py)",
              "ca_qx": h32(qx), "ca_qy": h32(qy), "certs": []}
        for name, d in (("ca.example.com-cert.pem", ca_der), ("peer0-cert.pem", peer_der)):
            tbs, sig = cert_parts(d)
            fx["certs"].append({"name": name, "tbs": tbs.hex(), "sig": sig.hex()})
        with open(path, "w") as f:
            json.dump(fx, f, indent=1)
    with open(path) as f:
        return json.load(f)


def main():
    rng = random.Random(20250718)
    out = []

    keys = []
    for i in range(8):
        d = rng.randrange(1, N)
        keys.append((d,) + O.pubkey(C, d))
    keys.append((1, C.gx, C.gy))                        # Q = G
    keys.append((N - 1,) + O.pubkey(C, N - 1))          # Q = -G

    def signed(d, digest, low=True):
        k = rng.randrange(1, N)
        return O.sign_digest(C, d, digest, k, low_s=low)

    # --- valid signatures, fused-SHA messages over SHA-256 padding edges -----
    for i, L in enumerate([0, 1, 3, 55, 56, 57, 63, 64, 65, 111, 119, 120, 128, 255, 256, 257,
                           1000, 1500, 4096]):
        d, qx, qy = keys[i % len(keys)]
        msg = bytes(rng.getrandbits(8) for _ in range(L))
        r, s = signed(d, hashlib.sha256(msg).digest())
        out.append(rec(f"valid_msg_len{L}", qx, qy, O.marshal_ecdsa_signature(r, s), msg=msg))

    # --- more valid + single-bit corruptions ---------------------------------
    for i in range(40):
        d, qx, qy = keys[i % len(keys)]
        msg = bytes(rng.getrandbits(8) for _ in range(256))
        dg = hashlib.sha256(msg).digest()
        r, s = signed(d, dg)
        sig = O.marshal_ecdsa_signature(r, s)
        out.append(rec("valid_256", qx, qy, sig, msg=msg))
        bad = bytearray(msg)
        bad[rng.randrange(256)] ^= 1 << rng.randrange(8)
        out.append(rec("msg_bitflip", qx, qy, sig, msg=bytes(bad)))
        out.append(rec("high_s", qx, qy, O.marshal_ecdsa_signature(r, N - s), msg=msg))
        out.append(rec("r_plus1", qx, qy, O.marshal_ecdsa_signature(r + 1, s), msg=msg))
        out.append(rec("s_plus1", qx, qy, O.marshal_ecdsa_signature(r, s + 1), msg=msg))
        out.append(rec("wrong_key", *keys[(i + 1) % len(keys)][1:], sig, msg=msg))

    d, qx, qy = keys[0]
    dg = hashlib.sha256(b"fabric").digest()
    r, s = signed(d, dg)

    # --- range / sign edges (bccsp/utils/ecdsa_test.go:19-62) ---------------
    for tag, rr, ss in [("r_zero", 0, s), ("s_zero", r, 0), ("r_neg1", -1, s), ("s_neg1", r, -1),
                        ("r_neg_big", -r, s), ("s_neg_big", r, -s),
                        ("r_eq_n", N, s), ("r_n_plus1", N + 1, s), ("r_2p256m1", 2**256 - 1, s),
                        ("r_33byte", 2**256 + 5, s), ("r_huge", 2**600 + 1, s),
                        ("s_huge", r, 2**600 + 1), ("r1_s1", 1, 1), ("r_nm1", N - 1, s),
                        ("s_eq_n", r, N), ("s_half", r, HALF), ("s_half_plus1", r, HALF + 1)]:
        out.append(rec(tag, qx, qy, O.marshal_ecdsa_signature(rr, ss), digest=dg))

    # --- s exactly n/2, valid (boundary accept) and n/2+1 ---------------------
    k = rng.randrange(1, N)
    Rpt = O.scalar_mult(C, k, (C.gx, C.gy))
    rr = Rpt[0] % N
    e = (HALF * k - rr * d) % N
    out.append(rec("s_eq_half_valid", qx, qy, O.marshal_ecdsa_signature(rr, HALF), digest=h32b(e)))
    out.append(rec("s_eq_half_plus1", qx, qy, O.marshal_ecdsa_signature(rr, HALF + 1), digest=h32b(e)))

    # --- bad public keys ------------------------------------------------------
    sig = O.marshal_ecdsa_signature(r, s)
    out.append(rec("q_offcurve", qx, (qy + 1) % P, sig, digest=dg))
    out.append(rec("q_x_ge_p", qx + P if qx + P < 2**256 else P, qy, sig, digest=dg))
    out.append(rec("q_y_ge_p", qx, P + 1, sig, digest=dg))
    out.append(rec("q_zero", 0, 0, sig, digest=dg))
    out.append(rec("q_eq_p", P, P, sig, digest=dg))
    out.append(rec("q_neg_y", qx, P - qy, sig, digest=dg))   # on curve (= -Q), math reject
    out.append(rec("q_offcurve_r_range", qx, (qy + 1) % P,
                   O.marshal_ecdsa_signature(N + 5, s), digest=dg))  # Go order: key first

    # --- DER quirks (encoding/asn1 semantics) ---------------------------------
    ri, si = der_int(r), der_int(s)
    out.append(rec("der_trailing_garbage_ok", qx, qy, der_raw(ri, si, trailing=b"\xde\xad\xbe\xef"), digest=dg))
    out.append(rec("der_trailing_zero_ok", qx, qy, der_raw(ri, si, trailing=b"\x00"), digest=dg))
    out.append(rec("der_extra_elem_ok", qx, qy, der_raw(ri, si, der_int(7)), digest=dg))
    out.append(rec("der_extra_junk_in_seq_ok", qx, qy, der_raw(ri, si, b"\xff\xff\xff"), digest=dg))
    out.append(rec("der_nonminimal_int", qx, qy,
                   der_raw(der_int_body(b"\x00" + O.asn1_marshal_int(r)) if O.asn1_marshal_int(r)[0] < 0x80
                           else der_int_body(b"\x00\x00" + O.asn1_marshal_int(r)[1:]), si), digest=dg))
    out.append(rec("der_nonminimal_ff", qx, qy, der_raw(der_int_body(b"\xff\x80"), si), digest=dg))
    out.append(rec("der_longform_short_len", qx, qy,
                   der_raw(der_int_body(O.asn1_marshal_int(r), b"\x81" + bytes([len(O.asn1_marshal_int(r))])), si),
                   digest=dg))
    body = ri + si
    out.append(rec("der_seq_longform_short", qx, qy, b"\x30\x81" + bytes([len(body)]) + body, digest=dg))
    out.append(rec("der_seq_len_leading_zero", qx, qy, b"\x30\x82\x00" + bytes([len(body)]) + body, digest=dg))
    out.append(rec("der_indefinite", qx, qy, b"\x30\x80" + body + b"\x00\x00", digest=dg))
    out.append(rec("der_seq_truncated_len", qx, qy, b"\x30" + bytes([len(body) + 1]) + body, digest=dg))
    out.append(rec("der_seq_shorter_len", qx, qy, b"\x30" + bytes([len(body) - 1]) + body, digest=dg))
    out.append(rec("der_missing_s", qx, qy, der_raw(ri), digest=dg))
    out.append(rec("der_set_tag", qx, qy, der_raw(ri, si, outer_tag=0x31), digest=dg))
    out.append(rec("der_seq_primitive", qx, qy, der_raw(ri, si, outer_tag=0x10), digest=dg))
    out.append(rec("der_ctx_tag", qx, qy, der_raw(ri, si, outer_tag=0xA0), digest=dg))
    out.append(rec("der_int_tag_wrong", qx, qy, der_raw(b"\x03" + ri[1:], si), digest=dg))
    out.append(rec("der_int_constructed", qx, qy, der_raw(b"\x22" + ri[1:], si), digest=dg))
    out.append(rec("der_int_empty", qx, qy, der_raw(b"\x02\x00", si), digest=dg))
    out.append(rec("der_high_tag", qx, qy, b"\x3f\x81\x00" + O.der_len(len(body)) + body, digest=dg))
    out.append(rec("der_high_tag_int", qx, qy, der_raw(b"\x1f\x02" + ri[1:], si), digest=dg))
    out.append(rec("der_only_tag", qx, qy, b"\x30", digest=dg))
    out.append(rec("der_zero_byte", qx, qy, b"\x00", digest=dg))
    out.append(rec("der_empty_seq", qx, qy, b"\x30\x00", digest=dg))
    out.append(rec("der_int_len_past_seq", qx, qy, b"\x30\x06\x02\x10" + ri[2:6], digest=dg))
    big_r = der_int(2**1100 + 3)  # 138-byte INTEGER -> long-form length 0x81 0x8a, valid DER, R >= n
    out.append(rec("der_longform_valid_big_r", qx, qy, der_raw(big_r, si), digest=dg))
    out.append(rec("der_seq_len_0x84", qx, qy, b"\x30\x84\x7f\xff\xff\xff" + body, digest=dg))
    out.append(rec("der_seq_len_too_large", qx, qy, b"\x30\x85\x01\x00\x00\x00\x00" + body, digest=dg))
    # bccsp/sw/impl_test.go:924-961 -- fixed reject vectors (verbatim data)
    for j, v in enumerate(["30070201 8f0202ff f1", "30070201 8f020200 01", "30070201 8f028101 01",
                           "30070201 8f028101 8f", "300a0201 8f020500 0000008f"]):
        out.append(rec(f"ref_impl_test_der_{j}", qx, qy, bytes.fromhex(v.replace(" ", "")), digest=dg))
    # empty inputs (impl.go:249-257; sw_test.go:130-149)
    out.append(rec("empty_sig", qx, qy, b"", digest=dg))
    out.append(rec("empty_digest", qx, qy, sig, digest=b""))
    out.append(rec("empty_both", qx, qy, b"", digest=b""))

    # --- digest lengths (hashToNat) ------------------------------------------
    for L in (1, 11, 20, 31, 32, 33, 48, 64):
        dgx = bytes(rng.getrandbits(8) for _ in range(L))
        rr, ss = signed(d, dgx)
        out.append(rec(f"digest_len{L}", qx, qy, O.marshal_ecdsa_signature(rr, ss), digest=dgx))
    hw = b"hello world"  # bccsp/sw/ecdsa_test.go:47-55 verifies msg as "digest"
    rr, ss = signed(d, hw)
    out.append(rec("digest_hello_world_11B", qx, qy, O.marshal_ecdsa_signature(rr, ss), digest=hw))
    # digest value >= n (reduced mod n)
    for dv in (N, N + 1, 2**256 - 1):
        dgx = dv.to_bytes(32, "big")
        rr, ss = signed(d, dgx)
        out.append(rec("digest_ge_n", qx, qy, O.marshal_ecdsa_signature(rr, ss), digest=dgx))
    # 48-byte digest where the first 32 bytes are >= n
    dgx = (2**256 - 1).to_bytes(32, "big") + b"\x01" * 16
    rr, ss = signed(d, dgx)
    out.append(rec("digest_48_ge_n", qx, qy, O.marshal_ecdsa_signature(rr, ss), digest=dgx))

    # --- x-wrap: R.x in [n, p) accepted via x mod n == r ----------------------
    for _ in range(2):
        xw, yw = find_wrap_point(rng)
        rw = xw - N
        out.append(rec("xwrap_accept", xw, yw, O.marshal_ecdsa_signature(rw, rw), digest=b"\x00" * 32))
        out.append(rec("xwrap_accept_1B", xw, yw, O.marshal_ecdsa_signature(rw, rw), digest=b"\x00"))
        out.append(rec("xwrap_wrong_r", xw, yw, O.marshal_ecdsa_signature(rw + 1, rw), digest=b"\x00" * 32))
        # e = 0 with r = x: x >= n so r >= n -> range reject
        out.append(rec("xwrap_r_eq_x", xw, yw, O.marshal_ecdsa_signature(xw, rw), digest=b"\x00" * 32))

    # --- u1 G + u2 Q = infinity ----------------------------------------------
    for _ in range(2):
        rr = rng.randrange(1, N)
        ss = rng.randrange(1, HALF)
        e = (-rr * d) % N
        out.append(rec("sum_infinity", qx, qy, O.marshal_ecdsa_signature(rr, ss), digest=h32b(e)))

    # --- u1 G == u2 Q (doubling inside the final addition) --------------------
    for j in range(3):
        dd, qxx, qyy = keys[j]
        k = rng.randrange(1, N)
        Rpt = O.scalar_mult(C, k, (C.gx, C.gy))
        rr = Rpt[0] % N
        e = rr * dd % N
        ss = 2 * rr * dd * pow(k, -1, N) % N
        if ss > HALF:
            ss = N - ss
        out.append(rec("u1G_eq_u2Q_accept", qxx, qyy, O.marshal_ecdsa_signature(rr, ss), digest=h32b(e)))
        out.append(rec("u1G_eq_u2Q_wrong_r", qxx, qyy, O.marshal_ecdsa_signature((rr + 1) % N or 1, ss),
                       digest=h32b(e)))
    # u1 = 0 (e = 0) ordinary signature
    rr, ss = signed(d, b"\x00" * 32)
    out.append(rec("e_zero_valid", qx, qy, O.marshal_ecdsa_signature(rr, ss), digest=b"\x00" * 32))
    # small scalars: u2 = 1 (s = r), u1 = e/r
    for dd, qxx, qyy in keys[:2]:
        # want s = r: s = k^-1 (e + r d) = r  ->  e = r k - r d
        k = rng.randrange(1, N)
        rr = O.scalar_mult(C, k, (C.gx, C.gy))[0] % N
        e = (rr * k - rr * dd) % N
        sig2 = O.marshal_ecdsa_signature(rr, rr if rr <= HALF else N - rr)
        out.append(rec("s_eq_r", qxx, qyy, sig2, digest=h32b(e)))

    # --- msp/testdata/mspid: real CA-issued P-256 signatures -----------------
    fx = mspid_fixture()
    cqx, cqy = int(fx["ca_qx"], 16), int(fx["ca_qy"], 16)
    for cert in fx["certs"]:
        tbs = bytes.fromhex(cert["tbs"])
        csig = bytes.fromhex(cert["sig"])
        out.append(rec("mspid_" + cert["name"] + "_highS", cqx, cqy, csig, msg=tbs))
        r0, s0, _ = O.asn1_unmarshal_ecdsa_sig(csig)
        out.append(rec("mspid_" + cert["name"] + "_lowS_twin", cqx, cqy,
                       O.marshal_ecdsa_signature(r0, N - s0), msg=tbs))
        bad = bytearray(tbs)
        bad[10] ^= 0x40
        out.append(rec("mspid_" + cert["name"] + "_lowS_twin_badmsg", cqx, cqy,
                       O.marshal_ecdsa_signature(r0, N - s0), msg=bytes(bad)))

    with open(os.path.join(HERE, "p256_vectors.jsonl"), "w") as f:
        for o in out:
            f.write(json.dumps(o, sort_keys=True) + "\n")
    # sanity: the mspid twins must accept and the originals must be high-S
    names = {o["tag"]: o for o in out}
    assert names["mspid_ca.example.com-cert.pem_lowS_twin"]["valid"]
    assert names["mspid_ca.example.com-cert.pem_highS"]["reason"] == O.R_HIGH_S
    from collections import Counter
    print(len(out), "records;", dict(Counter(O.REASON_NAMES[o["reason"]] for o in out)))


def h32b(v: int) -> bytes:
    return v.to_bytes(32, "big")


if __name__ == "__main__":
    main()
