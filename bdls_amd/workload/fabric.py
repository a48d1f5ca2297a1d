"""Synthetic Fabric blocks (BASELINE config 3) as the peer receives them: a
serialized common.Block whose envelopes are endorser transactions assembled the
way protoutil.CreateSignedTx assembles them, with real X.509 certificates in
the SerializedIdentities and P-256 signatures made as bccsp/sw signs
(ecdsa.Sign + ToLowS, via OpenSSL in libbdlsgen.so). Data preparation only.

Wire layout (fabric-protos-go v0.3.1 field numbers):
  Block{1 header: BlockHeader{1 number, 2 previous_hash, 3 data_hash},
        2 data: BlockData{1 repeated data: Envelope bytes}, 3 metadata}
  Envelope{1 payload, 2 signature}
  Payload{1 header: Header{1 channel_header, 2 signature_header}, 2 data}
  ChannelHeader{1 type=3, 2 version, 3 timestamp, 4 channel_id, 5 tx_id, 6 epoch}
  SignatureHeader{1 creator: SerializedIdentity{1 mspid, 2 id_bytes (PEM)}, 2 nonce}
  Transaction{1 actions: TransactionAction{1 header (SignatureHeader), 2 payload}}
  ChaincodeActionPayload{1 chaincode_proposal_payload, 2 action:
      ChaincodeEndorsedAction{1 proposal_response_payload,
                              2 endorsements: Endorsement{1 endorser, 2 signature}}}
  ProposalResponsePayload{1 proposal_hash, 2 extension}

Signed data (what the reference verifies):
  creator     : Envelope.payload, by SignatureHeader.creator
                (core/common/validation/msgvalidation.go:26-64, :274)
  endorsement : proposal_response_payload || endorser, by endorser
                (core/common/validation/statebased/validator_keylevel.go:246-260)
"""
from __future__ import annotations

import base64
import ctypes
import hashlib
import os
import struct
from dataclasses import dataclass, field

import numpy as np

_LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib",
                    "libbdlsgen.so")
SIG_STRIDE = 80

# ---------------------------------------------------------------- protobuf
def varint(v: int) -> bytes:
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def pb_bytes(num: int, b: bytes) -> bytes:
    return varint(num << 3 | 2) + varint(len(b)) + b


def pb_varint(num: int, v: int) -> bytes:
    return varint(num << 3) + varint(v & 0xFFFFFFFFFFFFFFFF)


# ---------------------------------------------------------------- DER / X.509
def der(tag: int, content: bytes) -> bytes:
    n = len(content)
    if n < 0x80:
        ln = bytes([n])
    else:
        b = n.to_bytes((n.bit_length() + 7) // 8, "big")
        ln = bytes([0x80 | len(b)]) + b
    return bytes([tag]) + ln + content


def der_int(v: int) -> bytes:
    b = v.to_bytes(max(1, (v.bit_length() + 8) // 8), "big")
    return der(0x02, b)


def der_oid(dotted: str) -> bytes:
    parts = [int(x) for x in dotted.split(".")]
    body = bytearray([40 * parts[0] + parts[1]])
    for p in parts[2:]:
        enc = [p & 0x7F]
        p >>= 7
        while p:
            enc.append(0x80 | (p & 0x7F))
            p >>= 7
        body += bytes(reversed(enc))
    return der(0x06, bytes(body))


SEQ = lambda *xs: der(0x30, b"".join(xs))  # noqa: E731
OID_ECDSA_SHA256 = "1.2.840.10045.4.3.2"
OID_EC_PUBKEY = "1.2.840.10045.2.1"
OID_P256 = "1.2.840.10045.3.1.7"


def x509_name(org: str, cn: str) -> bytes:
    return SEQ(der(0x31, SEQ(der_oid("2.5.4.10"), der(0x0C, org.encode()))),
               der(0x31, SEQ(der_oid("2.5.4.3"), der(0x0C, cn.encode()))))


def x509_tbs(serial: int, issuer: bytes, subject: bytes, pub64: bytes) -> bytes:
    alg = SEQ(der_oid(OID_ECDSA_SHA256))
    validity = SEQ(der(0x17, b"250101000000Z"), der(0x17, b"350101000000Z"))
    spki = SEQ(SEQ(der_oid(OID_EC_PUBKEY), der_oid(OID_P256)), der(0x03, b"\x00\x04" + pub64))
    return SEQ(der(0xA0, der_int(2)), der_int(serial), alg, issuer, validity, subject, spki)


def x509_cert(tbs: bytes, sig_der: bytes) -> bytes:
    return SEQ(tbs, SEQ(der_oid(OID_ECDSA_SHA256)), der(0x03, b"\x00" + sig_der))


def pem(cert: bytes) -> bytes:
    b = base64.b64encode(cert)
    lines = [b[i:i + 64] for i in range(0, len(b), 64)]
    return b"-----BEGIN CERTIFICATE-----\n" + b"\n".join(lines) + b"\n-----END CERTIFICATE-----\n"


def serialized_identity(mspid: str, cert_pem: bytes) -> bytes:
    return pb_bytes(1, mspid.encode()) + pb_bytes(2, cert_pem)


# ---------------------------------------------------------------- signing
def _gen():
    if not os.path.exists(_LIB):
        raise RuntimeError(f"{_LIB} not built (run `make`)")
    L = ctypes.CDLL(_LIB)
    vp = ctypes.c_void_p
    L.gen_p256_keypair.argtypes = [ctypes.c_uint64, ctypes.c_uint64, vp, vp]
    L.gen_p256_sign_batch.argtypes = [ctypes.c_size_t, vp, vp, ctypes.c_uint64, ctypes.c_int,
                                      vp, vp]
    return L


def keypair(L, seed: int, idx: int):
    priv = ctypes.create_string_buffer(32)
    pub = ctypes.create_string_buffer(64)
    L.gen_p256_keypair(seed, idx, priv, pub)
    return priv.raw, pub.raw


def sign_batch(L, privs: list[bytes], digests: list[bytes], seed: int,
               high_s: bool = False) -> list[bytes]:
    n = len(privs)
    if n == 0:
        return []
    pv = np.frombuffer(b"".join(privs), np.uint8)
    dg = np.frombuffer(b"".join(digests), np.uint8)
    out = np.zeros(n * SIG_STRIDE, np.uint8)
    ln = np.zeros(n, np.uint32)
    L.gen_p256_sign_batch(n, pv.ctypes.data, dg.ctypes.data, seed, 1 if high_s else 0,
                          out.ctypes.data, ln.ctypes.data)
    return [out[i * SIG_STRIDE:i * SIG_STRIDE + int(ln[i])].tobytes() for i in range(n)]


def sign(L, priv: bytes, msg: bytes, seed: int, high_s: bool = False) -> bytes:
    return sign_batch(L, [priv], [hashlib.sha256(msg).digest()], seed, high_s)[0]


# ---------------------------------------------------------------- identities
@dataclass
class Identity:
    mspid: str
    priv: bytes
    pub: bytes
    serialized: bytes
    cert_pem: bytes = b""


def make_identities(L, seed: int, norgs: int, nclients: int):
    """One CA per org; one peer (endorser) per org; nclients client identities
    spread over the orgs. Certificates signed by their org's CA."""
    cas, peers, clients = [], [], []
    for o in range(norgs):
        cas.append(keypair(L, seed, 1000 + o))
    tbs_list, signer, meta = [], [], []
    for o in range(norgs):
        priv, pub = keypair(L, seed, 2000 + o)
        org = f"Org{o + 1}MSP"
        tbs_list.append(x509_tbs(2000 + o, x509_name(org, f"ca.org{o + 1}"),
                                 x509_name(org, f"peer0.org{o + 1}"), pub))
        signer.append(cas[o][0])
        meta.append(("peer", org, priv, pub))
    for c in range(nclients):
        o = c % norgs
        priv, pub = keypair(L, seed, 3000 + c)
        org = f"Org{o + 1}MSP"
        tbs_list.append(x509_tbs(3000 + c, x509_name(org, f"ca.org{o + 1}"),
                                 x509_name(org, f"User{c}@org{o + 1}"), pub))
        signer.append(cas[o][0])
        meta.append(("client", org, priv, pub))
    sigs = sign_batch(L, signer, [hashlib.sha256(t).digest() for t in tbs_list], seed + 77)
    for tbs, sg, (kind, org, priv, pub) in zip(tbs_list, sigs, meta):
        cp = pem(x509_cert(tbs, sg))
        ident = Identity(org, priv, pub, serialized_identity(org, cp), cp)
        (peers if kind == "peer" else clients).append(ident)
    return cas, peers, clients


# ---------------------------------------------------------------- block
CORRUPTIONS = ["none", "creator_sig_flip", "creator_high_s", "endorse_sig_flip", "endorse_dup",
               "endorse_bad_identity", "payload_garbage", "epoch", "endorse_high_s",
               "creator_bad_identity", "two_actions", "endorse_dup_after_invalid",
               "envelope_garbage"]

# expected results (bdls_hip.h BH_FAB_* statuses, BH_R_* reasons)
FAB_OK, FAB_ENVELOPE, FAB_PAYLOAD, FAB_HEADER, FAB_CREATOR_IDENTITY = 0, 1, 2, 3, 4
FAB_CREATOR_SIGNATURE, FAB_TX = 5, 6
E_DUP, E_BAD_IDENTITY, E_NOT_VERIFIED = 253, 254, 255


@dataclass
class FabricBlock:
    block: bytes
    tx_status: list[int] = field(default_factory=list)
    tx_creator: list[int] = field(default_factory=list)   # BH_R_* or 255
    tx_endorse: list[list[int]] = field(default_factory=list)
    tx_valid_identities: list[int] = field(default_factory=list)
    tx_class: list[str] = field(default_factory=list)
    n_signatures: int = 0

    @property
    def ntx(self) -> int:
        return len(self.tx_status)


def _rng_u64(st: list[int]) -> int:
    st[0] = (st[0] + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    z = st[0]
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 31)


def _rand_bytes(st, n: int) -> bytes:
    out = bytearray()
    while len(out) < n:
        out += _rng_u64(st).to_bytes(8, "little")
    return bytes(out[:n])


def generate_fabric_block(ntx: int = 500, endorsements: int = 3, norgs: int = 4,
                          nclients: int = 50, corrupt_den: int = 100, seed: int = 3,
                          ext_len: int = 600, ccpp_len: int = 300,
                          classes: list[str] | None = None) -> FabricBlock:
    """BASELINE config 3: one block of ntx endorser transactions, each with a
    creator signature and `endorsements` endorsements by distinct org peers.
    1/corrupt_den of the transactions carry one corruption from CORRUPTIONS
    (or `classes`, cycled, when given: then every tx is corrupted in turn)."""
    L = _gen()
    st = [seed * 0x2545F4914F6CDD1D + 11]
    cas, peers, clients = make_identities(L, seed, norgs, nclients)
    bad_ident = serialized_identity("Org1MSP", b"-----BEGIN CERTIFICATE-----\nnot base64!\n"
                                               b"-----END CERTIFICATE-----\n")
    fb = FabricBlock(block=b"")
    # phase 1: per tx, everything up to the endorsement signatures
    txs = []
    for t in range(ntx):
        if classes is not None:
            cls = classes[t % len(classes)]
        elif corrupt_den and _rng_u64(st) % corrupt_den == 0:
            cls = CORRUPTIONS[1 + _rng_u64(st) % (len(CORRUPTIONS) - 1)]
        else:
            cls = "none"
        creator = clients[_rng_u64(st) % len(clients)]
        nonce = _rand_bytes(st, 24)
        creator_ser = bad_ident if cls == "creator_bad_identity" else creator.serialized
        txid = hashlib.sha256(nonce + creator_ser).hexdigest()
        chdr = (pb_varint(1, 3) + pb_bytes(3, pb_varint(1, 1_750_000_000 + t) + pb_varint(2, t))
                + pb_bytes(4, b"mychannel") + pb_bytes(5, txid.encode())
                + (pb_varint(6, 7) if cls == "epoch" else b""))
        shdr = pb_bytes(1, creator_ser) + pb_bytes(2, nonce)
        ccpp = _rand_bytes(st, ccpp_len)
        phash = hashlib.sha256(chdr + shdr + ccpp).digest()
        prp = pb_bytes(1, phash) + pb_bytes(2, _rand_bytes(st, ext_len))
        eps = [peers[(t + k) % len(peers)] for k in range(min(endorsements, len(peers)))]
        txs.append(dict(cls=cls, creator=creator, chdr=chdr, shdr=shdr, ccpp=ccpp, prp=prp,
                        eps=eps))
    # endorsement signatures over prp || endorser (one OpenSSL batch)
    e_priv, e_dig, e_where = [], [], []
    for ti, tx in enumerate(txs):
        for k, ep in enumerate(tx["eps"]):
            e_priv.append(ep.priv)
            e_dig.append(hashlib.sha256(tx["prp"] + ep.serialized).digest())
            e_where.append((ti, k))
    e_sigs = sign_batch(L, e_priv, e_dig, seed + 1)
    for (ti, k), sg in zip(e_where, e_sigs):
        txs[ti].setdefault("esig", {})[k] = sg
    # assemble payloads; creator signatures (second batch)
    payloads = []
    for ti, tx in enumerate(txs):
        cls = tx["cls"]
        ends, expect_e = [], []
        for k, ep in enumerate(tx["eps"]):
            ends.append([ep.serialized, tx["esig"][k]])
            expect_e.append(0)
        if cls == "endorse_sig_flip":
            s = bytearray(ends[0][1])
            s[-1] ^= 1
            ends[0][1] = bytes(s)
            expect_e[0] = 9
        elif cls == "endorse_high_s":
            ends[0][1] = sign(L, tx["eps"][0].priv, tx["prp"] + tx["eps"][0].serialized,
                              seed + 5 + ti, high_s=True)
            expect_e[0] = 6
        elif cls == "endorse_dup":
            ends[1] = list(ends[0])
            expect_e[1] = E_DUP
        elif cls == "endorse_bad_identity":
            ends[0][0] = bad_ident
            expect_e[0] = E_BAD_IDENTITY
        elif cls == "endorse_dup_after_invalid":
            # [A bad sig, A good sig, C]: Go verifies the second A (the first
            # did not enter the validated set) and accepts it
            good = list(ends[0])
            s = bytearray(good[1])
            s[-1] ^= 1
            ends.insert(0, [good[0], bytes(s)])
            expect_e = [9] + expect_e
            ends = ends[:len(tx["eps"])]
            expect_e = expect_e[:len(tx["eps"])]
        endorsements_pb = b"".join(pb_bytes(2, pb_bytes(1, e) + pb_bytes(2, s)) for e, s in ends)
        cea = pb_bytes(1, tx["prp"]) + endorsements_pb
        ccap = pb_bytes(1, tx["ccpp"]) + pb_bytes(2, cea)
        action = pb_bytes(1, tx["shdr"]) + pb_bytes(2, ccap)
        txn = pb_bytes(1, action) + (pb_bytes(1, action) if cls == "two_actions" else b"")
        payload = pb_bytes(1, pb_bytes(1, tx["chdr"]) + pb_bytes(2, tx["shdr"])) + pb_bytes(2, txn)
        if cls == "payload_garbage":
            payload = b"\x0a\xff\xff\x03" + payload
        tx["payload"], tx["ends"], tx["expect_e"] = payload, ends, expect_e
        payloads.append(payload)
    c_sigs = sign_batch(L, [tx["creator"].priv for tx in txs],
                        [hashlib.sha256(p).digest() for p in payloads], seed + 2)
    envs = []
    for ti, (tx, csig) in enumerate(zip(txs, c_sigs)):
        cls = tx["cls"]
        if cls == "creator_sig_flip":
            s = bytearray(csig)
            s[-1] ^= 1
            csig = bytes(s)
        elif cls == "creator_high_s":
            csig = sign(L, tx["creator"].priv, tx["payload"], seed + 9 + ti, high_s=True)
        env = pb_bytes(1, tx["payload"]) + pb_bytes(2, csig)
        if cls == "envelope_garbage":
            env = env[:-5]  # truncated signature field
        envs.append(env)
        # expected outcome in Go's order
        status, creator_r = FAB_OK, 0
        endorse = list(tx["expect_e"])
        if cls == "envelope_garbage":
            status, creator_r = FAB_ENVELOPE, E_NOT_VERIFIED
        elif cls == "payload_garbage":
            status, creator_r = FAB_PAYLOAD, E_NOT_VERIFIED
        elif cls == "epoch":
            status, creator_r = FAB_HEADER, E_NOT_VERIFIED
        elif cls == "creator_bad_identity":
            status, creator_r = FAB_CREATOR_IDENTITY, E_NOT_VERIFIED
        elif cls == "creator_sig_flip":
            status, creator_r = FAB_CREATOR_SIGNATURE, 9
        elif cls == "creator_high_s":
            status, creator_r = FAB_CREATOR_SIGNATURE, 6
        elif cls == "two_actions":
            status = FAB_TX
        if status in (FAB_ENVELOPE, FAB_PAYLOAD, FAB_HEADER, FAB_TX):
            endorse = []
        valid_ids = len({tx["ends"][k][0] for k, r in enumerate(endorse) if r == 0})
        fb.tx_status.append(status)
        fb.tx_creator.append(creator_r)
        fb.tx_endorse.append(endorse)
        fb.tx_valid_identities.append(valid_ids)
        fb.tx_class.append(cls)
        fb.n_signatures += (creator_r != E_NOT_VERIFIED) + sum(r <= 10 for r in endorse)
    data = b"".join(pb_bytes(1, e) for e in envs)
    data_hash = hashlib.sha256(b"".join(envs)).digest()
    header = pb_varint(1, 42) + pb_bytes(2, b"\x11" * 32) + pb_bytes(3, data_hash)
    metadata = b"".join(pb_bytes(1, b"") for _ in range(5))
    fb.block = pb_bytes(1, header) + pb_bytes(2, data) + pb_bytes(3, metadata)
    return fb


# ---------------------------------------------------------------- block signatures
def block_header_der(number: int, prev: bytes, data_hash: bytes) -> bytes:
    """protoutil.BlockHeaderBytes: ASN.1 DER of (number, previous_hash, data_hash)."""
    num = number.to_bytes(max(1, (number.bit_length() + 8) // 8), "big")
    return der(0x30, der(0x02, num) + der(0x04, prev) + der(0x04, data_hash))


BLOCKSIG_CORRUPTIONS = ["none", "sig_flip", "dup_signer", "bad_identity", "high_s",
                        "bad_sig_header", "no_metadata", "header_number"]


def generate_signed_blocks(nblocks: int = 16, norderers: int = 4, seed: int = 21,
                           classes: list[str] | None = None):
    """Blocks as an orderer cluster delivers them: the SIGNATURES metadata
    entry carries one MetadataSignature per orderer over Metadata.value ||
    signature_header || BlockHeaderBytes(header) (protoutil/blockutils.go
    :245-300). Returns (blocks, expected) with expected[i] = (status,
    per-signature BH_R_* / 253 dup / 254 bad identity, valid identities)."""
    L = _gen()
    st = [seed * 0x2545F4914F6CDD1D + 5]
    _, orderers, _ = make_identities(L, seed, norderers, 0)
    bad_ident = serialized_identity("OrdererMSP", b"-----BEGIN CERTIFICATE-----\n!!\n"
                                                  b"-----END CERTIFICATE-----\n")
    blocks, expected = [], []
    prev = b"\x00" * 32
    for bi in range(nblocks):
        cls = classes[bi % len(classes)] if classes else "none"
        data = b"".join(pb_bytes(1, _rand_bytes(st, 100)) for _ in range(3))
        dhash = hashlib.sha256(data).digest()
        number = 1000 + bi
        hdr_pb = pb_varint(1, number) + pb_bytes(2, prev) + pb_bytes(3, dhash)
        hder = block_header_der(number, prev, dhash)
        value = pb_bytes(1, pb_varint(1, number - 1))  # OrdererBlockMetadata-like value
        sigs, want = [], []
        for k, o in enumerate(orderers):
            shdr = pb_bytes(1, bad_ident if (cls == "bad_identity" and k == 0) else o.serialized) \
                + pb_bytes(2, _rand_bytes(st, 24))
            sg = sign(L, o.priv, value + shdr + hder, seed + 100 * bi + k,
                      high_s=(cls == "high_s" and k == 1))
            if cls == "sig_flip" and k == 2:
                sg = sg[:-1] + bytes([sg[-1] ^ 1])
            sigs.append(pb_bytes(1, shdr) + pb_bytes(2, sg))
            want.append(254 if (cls == "bad_identity" and k == 0) else
                        6 if (cls == "high_s" and k == 1) else
                        9 if (cls == "sig_flip" and k == 2) else 0)
        if cls == "dup_signer":
            sigs.append(sigs[0])
            want.append(253)
        if cls == "bad_sig_header":
            sigs.append(pb_bytes(1, b"\x0a\xff") + pb_bytes(2, b"\x30\x00"))
        md = pb_bytes(1, value) + b"".join(pb_bytes(2, x) for x in sigs)
        meta = b"" if cls == "no_metadata" else pb_bytes(1, md) + pb_bytes(1, b"") + pb_bytes(1, b"")
        hdr_used = hdr_pb if cls != "header_number" else (pb_varint(1, number + 1) + pb_bytes(2, prev)
                                                          + pb_bytes(3, dhash))
        blocks.append(pb_bytes(1, hdr_used) + pb_bytes(2, data) + pb_bytes(3, meta))
        if cls == "bad_sig_header":
            expected.append((4, [], 0))
        elif cls == "no_metadata":
            expected.append((2, [], 0))
        elif cls == "header_number":
            expected.append((0, [9] * len(orderers), 0))
        else:
            expected.append((0, want, sum(1 for w in want if w == 0)))
        prev = hashlib.sha256(hder).digest()
    return blocks, expected


BFT_BLOCKSIG_CORRUPTIONS = ["none", "sig_flip", "unknown_id", "dup_consenter", "bad_idh",
                            "creator_form", "both_headers", "consenter_bad_identity", "high_s",
                            "id_wrap"]


def generate_bft_signed_blocks(nblocks: int = 20, norderers: int = 4, seed: int = 31,
                               classes: list[str] | None = None):
    """Blocks as a BFT orderer cluster (consensus type "BFT", which this fork
    gives BDLS) signs them: each MetadataSignature has an empty
    signature_header and an IdentifierHeader{identifier: consenter Id, nonce};
    the signed bytes are Metadata.value || identifier_header ||
    BlockHeaderBytes(header) (protoutil/blockutils.go:261-272). Returns
    (blocks, consenters, expected): consenters = [(id, msp_id, identity PEM)]
    with Ids 1..norderers, expected[i] = (status, per-signature result, valid
    identities) with 252 for identifiers outside the set."""
    L = _gen()
    st = [seed * 0x2545F4914F6CDD1D + 9]
    _, orderers, _ = make_identities(L, seed, norderers, 0)
    garbage = b"-----BEGIN CERTIFICATE-----\n!!\n-----END CERTIFICATE-----\n"
    consenters = [(k + 1, o.mspid.encode(), o.cert_pem) for k, o in enumerate(orderers)]
    # first match wins (a later consenter with Id 2 is never consulted); Id 90
    # has an identity that does not deserialize; Id 91 marshals to nothing
    consenters += [(2, b"OtherMSP", garbage), (90, b"OrdererMSP", garbage), (91, b"", b"")]
    blocks, expected = [], []
    prev = b"\x00" * 32
    for bi in range(nblocks):
        cls = classes[bi % len(classes)] if classes else "none"
        data = b"".join(pb_bytes(1, _rand_bytes(st, 80)) for _ in range(2))
        dhash = hashlib.sha256(data).digest()
        number = 500 + bi
        hdr_pb = pb_varint(1, number) + pb_bytes(2, prev) + pb_bytes(3, dhash)
        hder = block_header_der(number, prev, dhash)
        value = pb_bytes(1, pb_varint(1, number - 1))
        sigs, want = [], []
        for k, o in enumerate(orderers):
            ident = k + 1
            if cls == "unknown_id" and k == 3:
                ident = 77
            if cls == "unknown_id" and k == 2:
                ident = 91  # in the set, but its SerializedIdentity marshals to nothing
            if cls == "consenter_bad_identity" and k == 0:
                ident = 90
            if cls == "id_wrap" and k == 0:
                ident_field = pb_varint(1, (1 << 32) + 1)  # uint32 field: low 32 bits -> Id 1
            else:
                ident_field = pb_varint(1, ident)
            idh = ident_field + pb_bytes(2, _rand_bytes(st, 24))
            if cls == "creator_form" and k == 1:  # this signer uses the SignatureHeader form
                shdr = pb_bytes(1, o.serialized) + pb_bytes(2, _rand_bytes(st, 24))
                sg = sign(L, o.priv, value + shdr + hder, seed + 100 * bi + k)
                sigs.append(pb_bytes(1, shdr) + pb_bytes(2, sg))
                want.append(0)
                continue
            sg = sign(L, o.priv, value + idh + hder, seed + 100 * bi + k,
                      high_s=(cls == "high_s" and k == 2))
            if cls == "sig_flip" and k == 1:
                sg = sg[:-1] + bytes([sg[-1] ^ 1])
            if cls == "both_headers" and k == 0:
                # a signature header present: the SignatureHeader form is taken,
                # over value || signature_header || header; signed with the
                # idh form, so it fails
                shdr = pb_bytes(1, o.serialized) + pb_bytes(2, b"n" * 24)
                sigs.append(pb_bytes(1, shdr) + pb_bytes(2, sg) + pb_bytes(3, idh))
                want.append(9)
                continue
            sigs.append(pb_bytes(2, sg) + pb_bytes(3, idh))
            want.append(252 if (cls == "unknown_id" and k in (2, 3)) else
                        254 if (cls == "consenter_bad_identity" and k == 0) else
                        6 if (cls == "high_s" and k == 2) else
                        9 if (cls == "sig_flip" and k == 1) else 0)
        if cls == "dup_consenter":
            sigs.append(sigs[2])
            want.append(253)
        if cls == "bad_idh":
            sigs.insert(1, pb_bytes(2, b"\x30\x00") + pb_bytes(3, b"\x08"))  # truncated varint
        md = pb_bytes(1, value) + b"".join(pb_bytes(2, x) for x in sigs)
        meta = pb_bytes(1, md) + pb_bytes(1, b"") + pb_bytes(1, b"")
        blocks.append(pb_bytes(1, hdr_pb) + pb_bytes(2, data) + pb_bytes(3, meta))
        if cls == "bad_idh":
            expected.append((5, [], 0))
        else:
            expected.append((0, want, sum(1 for w in want if w == 0)))
        prev = hashlib.sha256(hder).digest()
    return blocks, consenters, expected
