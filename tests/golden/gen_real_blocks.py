"""Generate tests/golden/real_blocks.json: blocks that Go (protobuf-go + the
reference's own orderers) marshalled and signed, with the results the
reference's validation flow gives on them.

Sources (data files the reference's own tests hold, read as data):
  orderer/common/cluster/testdata/block3.pb          block 3 of a system channel,
      one ORDERER_TRANSACTION envelope, an orderer block signature (non-BFT)
  orderer/common/cluster/testdata/mychannel.block    genesis block (CONFIG)
  orderer/consensus/etcdraft/testdata/mychannel.block
  orderer/consensus/etcdraft/testdata/etcdraftgenesis.block
  orderer/consensus/smartbft/testdata/mychannel.block (CONFIG, empty creator)

Expected results come from oracle/fabric_ref.py (validateTx /
SignatureSetToValidIdentities / SigFilter / BlockSignatureVerifier restated)
with the group equation checked twice: by oracle/ecdsa_ref.py and by OpenSSL
(oracle/orc.c); the generator fails if the two disagree. Besides the blocks
as they are, a few deterministic mutations of the real bytes (signature bit
flips, a changed header number, a high-S twin of the real block signature,
the BFT form of the same block) pin the reject paths on Go-produced bytes.
X.509 links: every certificate embedded in these blocks (MSP root / admin /
signer certificates of the channel configs, the creators) paired with every
embedded certificate whose subject equals its issuer, for bh_verify_x509.

Run from the repo root (needs /root/reference; the fixture travels, the
reference does not): python tests/golden/gen_real_blocks.py
"""
from __future__ import annotations

import base64
import hashlib
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import ecdsa_ref as O  # noqa: E402
from oracle import fabric_ref as R  # noqa: E402
from oracle import orc  # noqa: E402
from oracle import x509_ref as X  # noqa: E402

REF = "/root/reference"
OUT = os.path.join(ROOT, "tests", "golden", "real_blocks.json")
SOURCES = {
    "cluster_block3": "orderer/common/cluster/testdata/block3.pb",
    "cluster_mychannel": "orderer/common/cluster/testdata/mychannel.block",
    "etcdraft_mychannel": "orderer/consensus/etcdraft/testdata/mychannel.block",
    "etcdraft_genesis": "orderer/consensus/etcdraft/testdata/etcdraftgenesis.block",
    "smartbft_mychannel": "orderer/consensus/smartbft/testdata/mychannel.block",
}


def py_verify(x, y, msg, sig):
    return O.identity_verify(O.P256, x, y, msg, sig)[1]


def orc_verify(x, y, msg, sig):
    return orc.csp_verify(x.to_bytes(32, "big") + y.to_bytes(32, "big"), sig,
                          hashlib.sha256(msg).digest())


def both(fn):
    """fn(verify) under both group-equation checkers; they must agree."""
    a, b = fn(py_verify), fn(orc_verify)
    assert a == b, (a, b)
    return a


def tx_tuple(t):
    return [t.status, t.type, t.creator, t.endorse, t.valid_endorsers]


def envelopes(block):
    blk = R.unmarshal(block, R.BLOCK_SPEC)
    return (blk["data"] or {"data": []})["data"]


# ---------------------------------------------------------------- protobuf re-encoding
def varint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def fld(num, b):
    return varint(num << 3 | 2) + varint(len(b)) + b


def replace_metadata0(block, md0):
    """The block with Metadata.metadata[0] replaced (other fields as they were)."""
    out = b""
    i = 0
    while i < len(block):  # walk raw fields to keep the header and data bytes verbatim
        tag, j = R.consume_varint(block, i)
        num, typ = tag >> 3, tag & 7
        ln, k = R.consume_varint(block, j)
        raw, body = block[i:k + ln], block[k:k + ln]
        if num == 3 and typ == 2:
            mds = [v for n2, t2, v in R.fields(body) if n2 == 1 and t2 == 2]
            mds[0] = md0
            raw = fld(3, b"".join(fld(1, m) for m in mds))
        out += raw
        i = k + ln
    return out


def replace_header_number(block, number):
    out, i = b"", 0
    while i < len(block):
        tag, j = R.consume_varint(block, i)
        num, typ = tag >> 3, tag & 7
        ln, k = R.consume_varint(block, j)
        raw, body = block[i:k + ln], block[k:k + ln]
        if num == 1 and typ == 2:
            h = R.unmarshal(body, R.BLOCK_HEADER_SPEC)
            nb = varint(1 << 3) + varint(number) + fld(2, h["previous_hash"] or b"") \
                + fld(3, h["data_hash"] or b"")
            raw = fld(1, nb)
        out += raw
        i = k + ln
    return out


def metadata0(block):
    blk = R.unmarshal(block, R.BLOCK_SPEC)
    return blk["metadata"]["metadata"][0]


def sig_fields(md):
    m = R.unmarshal(md, R.METADATA_SPEC)
    return m["value"] or b"", m["signatures"]


def encode_md(value, sigs):
    body = (fld(1, value) if value else b"")
    for s in sigs:
        e = b""
        if s.get("signature_header"):
            e += fld(1, s["signature_header"])
        if s.get("signature"):
            e += fld(2, s["signature"])
        if s.get("identifier_header"):
            e += fld(3, s["identifier_header"])
        body += fld(2, e)
    return body


def high_s_twin(sig_der):
    rc, r, s = O.unmarshal_ecdsa_signature(sig_der)
    assert rc == O.R_OK
    s2 = O.P256.n - s

    def di(v):
        b = v.to_bytes((v.bit_length() + 8) // 8, "big")
        return b"\x02" + bytes([len(b)]) + b

    body = di(r) + di(s2)
    return b"\x30" + bytes([len(body)]) + body


# ---------------------------------------------------------------- x509 links
def pem_certs(b):
    for m in re.finditer(rb"-----BEGIN CERTIFICATE-----(.*?)-----END CERTIFICATE-----", b, re.S):
        try:
            yield base64.b64decode(b"".join(m.group(1).replace(b"\\n", b"\n").split()))
        except Exception:  # noqa: BLE001
            continue


def names_and_key(der):
    c = X._tlv(der, 0)
    tbs = X._tlv(c[1], 0)
    t = X._tlv(tbs[1], 0)
    if t[0] == 0xA0:
        t = X._tlv(tbs[1], t[3])
    sig = X._tlv(tbs[1], t[3])
    issuer = X._tlv(tbs[1], sig[3])
    validity = X._tlv(tbs[1], issuer[3])
    subject = X._tlv(tbs[1], validity[3])
    spki = X._tlv(tbs[1], subject[3])
    key = None
    try:
        alg = X._tlv(spki[1], 0)
        bits = X._tlv(spki[1], alg[3])
        if bits[1][:2] == b"\x00\x04" and len(bits[1]) == 66 and R.OID_P256 in alg[1]:
            key = (int.from_bytes(bits[1][2:34], "big"), int.from_bytes(bits[1][34:66], "big"))
    except Exception:  # noqa: BLE001
        pass
    return issuer[2], subject[2], key


def x509_links(raw_blocks):
    certs = []
    for b in raw_blocks:
        for der in pem_certs(b):
            if der not in certs:
                certs.append(der)
    info = []
    for der in certs:
        try:
            info.append(names_and_key(der))
        except Exception:  # noqa: BLE001
            info.append(None)
    links, wrong = [], []
    for i, der in enumerate(certs):
        if info[i] is None:
            continue
        for j, _ in enumerate(certs):
            if info[j] is None or info[j][2] is None or info[j][1] != info[i][0]:
                continue
            x, y = info[j][2]
            want = X.check_signature_from(der, x, y)
            (links if want == O.R_OK else wrong).append([i, j, want])
    # every verifying link, and every 4th same-name wrong issuer (the configs
    # of several test networks reuse CA names)
    return {"certs": [c.hex() for c in certs], "links": links + wrong[::4]}


def main():
    raw = {k: open(os.path.join(REF, p), "rb").read() for k, p in SOURCES.items()}
    out = {"sources": SOURCES, "blocks": {}, "mutations": [], "x509": []}
    for name, b in raw.items():
        envs = envelopes(b)
        out["blocks"][name] = {
            "hex": b.hex(),
            "sha256": hashlib.sha256(b).hexdigest(),
            "block_signatures": list(both(lambda v: R.block_signatures(b, v))),
            "block_signatures_bft": list(both(lambda v: R.block_signatures(b, v, bft=True))),
            "txs": both(lambda v: [tx_tuple(t) for t in R.validate_block(b, v)]),
            "sigfilter": both(lambda v: [list(R.sigfilter(e, v)) for e in envs]),
        }
    # mutations of block3's real orderer signature (non-BFT form)
    b3 = raw["cluster_block3"]
    value, sigs = sig_fields(metadata0(b3))
    real = sigs[0]
    flipped = dict(real)
    flipped["signature"] = real["signature"][:-1] + bytes([real["signature"][-1] ^ 1])
    twin = dict(real)
    twin["signature"] = high_s_twin(real["signature"])
    sh = R.unmarshal(real["signature_header"], R.SIGNATURE_HEADER_SPEC)
    cons = [(7, b"OrdererMSP", R.unmarshal(sh["creator"], R.SERIALIZED_IDENTITY_SPEC)["id_bytes"])]
    cases = {
        "sig_flip": (replace_metadata0(b3, encode_md(value, [flipped])), False, None),
        "high_s_twin": (replace_metadata0(b3, encode_md(value, [twin])), False, None),
        "header_number": (replace_header_number(b3, 4), False, None),
        "value_changed": (replace_metadata0(b3, encode_md(value + b"\x00", [real])), False, None),
        "duplicate": (replace_metadata0(b3, encode_md(value, [real, real])), False, None),
        "failed_then_valid": (replace_metadata0(b3, encode_md(value, [flipped, real])), False, None),
        # the BFT form with the real signer as consenter 7: the signed bytes
        # now hold the IdentifierHeader, so the real signature no longer
        # verifies (reject), and an identifier outside the set is skipped
        "bft_form": (replace_metadata0(b3, encode_md(value, [
            {"signature": real["signature"], "identifier_header": varint(8) + varint(7)},
            {"signature": real["signature"], "identifier_header": varint(8) + varint(8)}])),
            True, cons),
        "bft_flag_creator_form": (b3, True, cons),
    }
    for name, (blk, bft, c) in cases.items():
        out["mutations"].append({
            "name": name, "hex": blk.hex(), "bft": bft,
            "consenters": [[i, m.hex(), d.hex()] for i, m, d in (c or [])],
            "block_signatures": list(both(lambda v: R.block_signatures(blk, v, bft=bft,
                                                                         consenters=c))),
        })
    # envelope mutations: the real creator signatures, flipped / high-S twin
    for name in ("cluster_block3", "cluster_mychannel", "etcdraft_genesis"):
        env = envelopes(raw[name])[0]
        e = R.unmarshal(env, R.ENVELOPE_SPEC)
        for kind, sg in (("flip", e["signature"][:-1] + bytes([e["signature"][-1] ^ 1])),
                         ("high_s", high_s_twin(e["signature"]))):
            env2 = fld(1, e["payload"]) + fld(2, sg)
            out["mutations"].append({"name": f"{name}_envelope_{kind}", "envelope": env2.hex(),
                                     "sigfilter": list(both(lambda v: R.sigfilter(env2, v)))})
    out["x509"] = x509_links(raw.values())
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {OUT}: {len(out['blocks'])} blocks, {len(out['mutations'])} mutations, "
          f"{len(out['x509']['links'])} x509 links")


if __name__ == "__main__":
    main()
