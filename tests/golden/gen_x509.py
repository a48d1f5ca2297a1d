"""Generate tests/golden/x509_vectors.json: (certificate DER, issuer public key,
expected BH_R_* of CheckSignatureFrom) for bh_verify_x509.

Sources (data files the reference's own tests hold, read as data):
  * every X.509 certificate in /root/reference/msp/testdata/**/*.pem and
    /root/reference/sampleconfig/msp/**/*.pem, paired with every certificate
    in that set whose subject equals its issuer (CA -> intermediate -> leaf
    links of the MSP test chains, self-signed roots, and deliberately wrong
    same-name issuers such as the revoked / external fixtures);
  * mutations of a few real links: TBS bit flip, high-S twin (still valid: no
    low-S rule for certificates), non-strict DER signatures (trailing bytes,
    non-minimal INTEGER, long-form short length: encoding/asn1 would accept
    some of these, cryptobyte does not), zero / out-of-range r and s, a
    wrong / off-curve issuer key, SHA-384 and mismatched algorithm
    identifiers.
Expected results come from oracle/x509_ref.py (Go 1.21 x509 + VerifyASN1
restated). Run from the repo root: python tests/golden/gen_x509.py
"""
from __future__ import annotations

import base64
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import ecdsa_ref as O  # noqa: E402
from oracle import x509_ref as X  # noqa: E402

REF = "/root/reference"
OUT = os.path.join(ROOT, "tests", "golden", "x509_vectors.json")


def pem_certs(path):
    txt = open(path, "rb").read()
    for m in re.finditer(rb"-----BEGIN CERTIFICATE-----(.*?)-----END CERTIFICATE-----", txt, re.S):
        try:
            yield base64.b64decode(b"".join(m.group(1).split()))
        except Exception:  # noqa: BLE001
            continue


def tlv(b, i):
    return X._tlv(b, i)


def names_and_key(der):
    """(issuer raw, subject raw, (x, y) or None) of a certificate."""
    c = tlv(der, 0)
    tbs = tlv(c[1], 0)
    t = tlv(tbs[1], 0)
    if t[0] == 0xA0:
        t = tlv(tbs[1], t[3])
    sig = tlv(tbs[1], t[3])
    issuer = tlv(tbs[1], sig[3])
    validity = tlv(tbs[1], issuer[3])
    subject = tlv(tbs[1], validity[3])
    spki = tlv(tbs[1], subject[3])
    algid = tlv(spki[1], 0)
    bits = tlv(spki[1], algid[3])
    key = None
    if bits[1][:2] == b"\x00\x04" and len(bits[1]) == 66 and b"\x2a\x86\x48\xce\x3d\x03\x01\x07" in algid[1]:
        key = (int.from_bytes(bits[1][2:34], "big"), int.from_bytes(bits[1][34:], "big"))
    return issuer[2], subject[2], key


def rebuild(der, sig_der=None, tbs_mut=None, alg_oid=None, inner_oid=None):
    """Re-encode a certificate with a new signature / TBS / algorithm OIDs."""
    from bdls_amd.workload.fabric import der as enc
    c = tlv(der, 0)
    tbs = tlv(c[1], 0)
    alg = tlv(c[1], tbs[3])
    sv = tlv(c[1], alg[3])
    tbs_raw = tbs[2]
    if inner_oid is not None:
        t = tlv(tbs[1], 0)
        head = b""
        if t[0] == 0xA0:
            head = t[2]
            t = tlv(tbs[1], t[3])
        serial = t[2]
        inner = tlv(tbs[1], t[3])
        rest = tbs[1][inner[3]:]
        tbs_raw = enc(0x30, head + serial + enc(0x30, enc(0x06, inner_oid)) + rest)
    if tbs_mut is not None:
        tbs_raw = tbs_mut(tbs_raw)
    alg_raw = alg[2] if alg_oid is None else enc(0x30, enc(0x06, alg_oid))
    sig = sv[1][1:] if sig_der is None else sig_der
    return enc(0x30, tbs_raw + alg_raw + enc(0x03, b"\x00" + sig))


def main():
    certs = {}
    for pat in ("msp/testdata/**/*.pem", "sampleconfig/msp/**/*.pem"):
        for path in sorted(glob.glob(os.path.join(REF, pat), recursive=True)):
            for der in pem_certs(path):
                try:
                    iss, sub, key = names_and_key(der)
                except (TypeError, IndexError):
                    continue
                certs.setdefault(der, (iss, sub, key, os.path.relpath(path, REF)))
    by_subject = {}
    for der, (iss, sub, key, path) in certs.items():
        if key is not None:
            by_subject.setdefault(sub, []).append((der, key, path))
    vecs = []
    for der, (iss, sub, key, path) in sorted(certs.items(), key=lambda kv: kv[1][3]):
        for cadir, ckey, cpath in by_subject.get(iss, []):
            want = X.check_signature_from(der, *ckey)
            vecs.append({"tag": f"ref:{path}<-{cpath}", "cert": der.hex(), "qx": f"{ckey[0]:064x}",
                         "qy": f"{ckey[1]:064x}", "reason": want})
    # mutations of real, verifying links
    good = [v for v in vecs if v["reason"] == 0][:6]
    n = O.P256.n
    for g in good:
        der = bytes.fromhex(g["cert"])
        qx, qy = int(g["qx"], 16), int(g["qy"], 16)
        tbs, _, _, sig = X.split_cert(der)
        r, s = X.parse_signature(sig)

        def m_int(v, nonmin=False, longlen=False):
            b = v.to_bytes(max(1, (v.bit_length() + 8) // 8), "big")
            if nonmin:
                b = b"\x00" + b
            return b"\x02" + (b"\x81" if longlen else b"") + bytes([len(b)]) + b

        def m_sig(rr, ss, tail=b"", extra=b"", rnm=False, rll=False):
            body = m_int(rr, rnm, rll) + m_int(ss) + extra
            return b"\x30" + bytes([len(body)]) + body + tail

        flip = lambda t: t[:-3] + bytes([t[-3] ^ 1]) + t[-2:]  # noqa: E731
        cases = {
            "tbs_flip": rebuild(der, tbs_mut=flip),
            "high_s_twin": rebuild(der, m_sig(r, n - s)),
            "der_trailing": rebuild(der, m_sig(r, s, tail=b"\x00")),
            "der_extra_elem": rebuild(der, m_sig(r, s, extra=b"\x02\x01\x07")),
            "der_nonminimal_r": rebuild(der, m_sig(r, s, rnm=True)),
            "der_longform_short": rebuild(der, m_sig(r, s, rll=True)),
            "r_zero": rebuild(der, m_sig(0, s)),
            "s_zero": rebuild(der, m_sig(r, 0)),
            "r_plus_n": rebuild(der, m_sig(r + n, s)),
            "s_plus_n": rebuild(der, m_sig(r, s + n)),
            "negative_r": rebuild(der, b"\x30\x06\x02\x01\xff\x02\x01\x01"),
            "sha384_alg": rebuild(der, alg_oid=bytes.fromhex("2a8648ce3d040303"),
                                  inner_oid=bytes.fromhex("2a8648ce3d040303")),
            "alg_mismatch": rebuild(der, alg_oid=bytes.fromhex("2a8648ce3d040303")),
            "not_a_cert": der[:40],
        }
        for tag, c in cases.items():
            vecs.append({"tag": f"mut:{tag}:{g['tag']}", "cert": c.hex(), "qx": g["qx"],
                         "qy": g["qy"], "reason": X.check_signature_from(c, qx, qy)})
        for tag, (kx, ky) in {"wrong_key": O.pubkey(O.P256, 12345),
                              "offcurve_key": (qx, qy ^ 1)}.items():
            vecs.append({"tag": f"mut:{tag}:{g['tag']}", "cert": g["cert"], "qx": f"{kx:064x}",
                         "qy": f"{ky:064x}", "reason": X.check_signature_from(der, kx, ky)})
    with open(OUT, "w") as f:
        json.dump(vecs, f, indent=0)
    from collections import Counter
    print(len(vecs), "vectors", Counter(v["reason"] for v in vecs))


if __name__ == "__main__":
    main()
