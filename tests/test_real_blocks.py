"""The Fabric decoders and callers on blocks Go itself marshalled and signed:
the reference's orderer test blocks (tests/golden/real_blocks.json, made by
tests/golden/gen_real_blocks.py from orderer/common/cluster/testdata and
orderer/consensus/{etcdraft,smartbft}/testdata). This pins the C++ protobuf /
PEM / X.509 decoding and the signed-bytes construction to bytes the
generator of this repo did not produce.

CPU: the oracle reproduces the fixture (its expectations were checked against
OpenSSL when generated); the C++ decode (BH_FAB_F_DECODE_ONLY) agrees with the
oracle on the real blocks, their envelopes and thousands of mutations of them.
GPU: bh_block_signatures_preverify (plain and BFT), bh_fabric_block_preverify,
bh_envelopes_preverify and bh_verify_x509 give the fixture's results.
"""
import json
import os
import random

import numpy as np
import pytest

from bdls_amd import fabric
from oracle import ecdsa_ref as O
from oracle import fabric_ref as R
from tests.conftest import ROOT

FIX = os.path.join(ROOT, "tests", "golden", "real_blocks.json")


def _py_verify(x, y, msg, sig):
    return O.identity_verify(O.P256, x, y, msg, sig)[1]


@pytest.fixture(scope="module")
def fx():
    with open(FIX) as f:
        return json.load(f)


def _blocks(fx):
    return {k: bytes.fromhex(v["hex"]) for k, v in fx["blocks"].items()}


def _envs(block):
    return R.unmarshal(block, R.BLOCK_SPEC)["data"]["data"]


def _cons(m):
    return [(c[0], bytes.fromhex(c[1]), bytes.fromhex(c[2])) for c in m["consenters"]]


def _tx(t):
    return [t.status, t.type, t.creator, t.endorse, t.valid_endorsers]


def test_fixture_content(fx):
    """What the real blocks hold: block 3's orderer signature verifies (1
    valid identity), the genesis blocks' CONFIG envelopes carry a creator
    signature that verifies."""
    b = fx["blocks"]
    assert b["cluster_block3"]["block_signatures"] == [0, [0], 1]
    for k in ("cluster_mychannel", "etcdraft_mychannel", "etcdraft_genesis"):
        assert b[k]["txs"] == [[0, 1, 0, [], 0]]
        assert b[k]["sigfilter"] == [[0, 0]]
    assert b["cluster_block3"]["sigfilter"] == [[0, 0]]  # the ORDERER_TRANSACTION's creator
    assert sum(1 for l in fx["x509"]["links"] if l[2] == 0) >= 40


def test_oracle_reproduces_fixture(fx):
    for name, blk in _blocks(fx).items():
        v = fx["blocks"][name]
        assert list(R.block_signatures(blk, _py_verify)) == v["block_signatures"], name
        assert [_tx(t) for t in R.validate_block(blk, _py_verify)] == v["txs"], name
        assert [list(R.sigfilter(e, _py_verify)) for e in _envs(blk)] == v["sigfilter"], name
    for m in fx["mutations"]:
        if "hex" in m:
            got = R.block_signatures(bytes.fromhex(m["hex"]), _py_verify, bft=m["bft"],
                                     consenters=_cons(m))
            assert list(got) == m["block_signatures"], m["name"]
        else:
            assert list(R.sigfilter(bytes.fromhex(m["envelope"]), _py_verify)) == m["sigfilter"]


def test_decode_matches_oracle(fx):
    blocks = _blocks(fx)
    for name, blk in blocks.items():
        py = [_tx(t) for t in R.validate_block(blk, None, decode_only=True)]
        cc = [_tx(t) for t in fabric.block_preverify(blk, decode_only=True)]
        assert py == cc, name
    lst = list(blocks.values()) + [bytes.fromhex(m["hex"]) for m in fx["mutations"] if "hex" in m]
    py = [R.block_signatures(b, None, decode_only=True) for b in lst]
    assert py == [tuple(c) for c in fabric.block_signatures_preverify(lst, decode_only=True)]
    envs = [e for b in blocks.values() for e in _envs(b)]
    assert [R.sigfilter(e, None, decode_only=True) for e in envs] == \
        fabric.envelopes_preverify(envs, decode_only=True)


def _mutate(rng, b: bytes) -> bytes:
    b = bytearray(b)
    for _ in range(rng.randrange(1, 4)):
        op = rng.randrange(5)
        if op == 0 and b:
            b[rng.randrange(len(b))] = rng.randrange(256)
        elif op == 1 and b:
            i = rng.randrange(len(b))
            del b[i:i + rng.randrange(1, 6)]
        elif op == 2:
            b.insert(rng.randrange(len(b) + 1), rng.randrange(256))
        elif op == 3 and b:
            b[rng.randrange(len(b))] ^= 0x80
        else:
            tag = rng.choice([0x0b, 0x0c, 0x0e, 0x0f, 0x14, 0x1a, 0x08, 0xf8, 0x80])
            b[rng.randrange(len(b) + 1):0] = bytes([tag, rng.randrange(256)])
    return bytes(b)


def _fld(num, b):
    from bdls_amd.workload import fabric as F
    return F.pb_bytes(num, b)


def _nested(rng, env: bytes) -> bytes:
    """Mutate one nested message of a real envelope (payload, header, channel
    header, signature header, serialized creator, PEM body) and re-encode."""
    e = R.unmarshal(env, R.ENVELOPE_SPEC)
    pl = R.unmarshal(e["payload"], R.PAYLOAD_SPEC)
    ch, sh = pl["header"]["channel_header"] or b"", pl["header"]["signature_header"] or b""
    data = pl["data"] or b""
    sig = e["signature"] or b""
    which = rng.randrange(6)
    if which == 2 and not R.unmarshal(sh, R.SIGNATURE_HEADER_SPEC)["creator"]:
        which = 1
    if which == 0:
        ch = _mutate(rng, ch)
    elif which == 1:
        sh = _mutate(rng, sh)
    elif which == 2:
        s = R.unmarshal(sh, R.SIGNATURE_HEADER_SPEC)
        si = R.unmarshal(s["creator"], R.SERIALIZED_IDENTITY_SPEC)
        idb = si["id_bytes"]
        if rng.random() < 0.5:  # PEM framing / base64 body
            k = rng.randrange(len(idb))
            idb = idb[:k] + bytes([rng.choice(b"\n\r =-A/+!")]) + idb[k + 1:]
        else:
            idb = _mutate(rng, idb)
        sh = _fld(1, _fld(1, si["mspid"] or b"") + _fld(2, idb)) + _fld(2, s["nonce"] or b"")
    elif which == 3:
        data = _mutate(rng, data)
    elif which == 4:
        return _fld(1, _mutate(rng, e["payload"])) + _fld(2, sig)
    else:
        return _mutate(rng, env)
    payload = _fld(1, _fld(1, ch) + _fld(2, sh)) + _fld(2, data)
    return _fld(1, payload) + _fld(2, sig)


def test_decode_fuzz_real_envelopes(fx):
    """C++ decode vs the oracle on mutations of Go-marshalled envelopes, both
    as block transactions (validateTx order) and through SigFilter."""
    rng = random.Random(13)
    base = [e for b in _blocks(fx).values() for e in _envs(b)]
    cases = [_nested(rng, rng.choice(base)) for _ in range(1500)]
    assert [R.sigfilter(e, None, decode_only=True) for e in cases] == \
        fabric.envelopes_preverify(cases, decode_only=True)
    for it, env in enumerate(cases[:600]):
        block = _fld(2, _fld(1, env))
        py = [_tx(t) for t in R.validate_block(block, None, decode_only=True)]
        cc = [_tx(t) for t in fabric.block_preverify(block, decode_only=True)]
        assert py == cc, (it, env.hex())


def test_decode_fuzz_real_block_signatures(fx):
    rng = random.Random(14)
    b3 = bytes.fromhex(fx["blocks"]["cluster_block3"]["hex"])
    md0 = R.unmarshal(b3, R.BLOCK_SPEC)["metadata"]["metadata"][0]
    cases = []
    for _ in range(600):  # mutate the SIGNATURES metadata (value, signature headers, signatures)
        m = _mutate(rng, md0)
        rest = R.unmarshal(b3, R.BLOCK_SPEC)["metadata"]["metadata"][1:]
        hdr = R.unmarshal(b3, {1: ("h", "bytes")})["h"]
        data = R.unmarshal(b3, {2: ("d", "bytes")})["d"]
        cases.append(_fld(1, hdr) + _fld(2, data) + _fld(3, b"".join(_fld(1, x) for x in [m] + rest)))
    cases += [_mutate(rng, b3) for _ in range(200)]
    cons = [(7, b"OrdererMSP", b"x")]
    for bft in (False, True):
        py = [R.block_signatures(b, None, decode_only=True, bft=bft, consenters=cons) for b in cases]
        cc = fabric.block_signatures_preverify(cases, decode_only=True, bft=bft, consenters=cons)
        assert py == [tuple(c) for c in cc]


# ---------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_gpu_real_block_signatures(fx):
    blocks = _blocks(fx)
    names = list(blocks)
    got = fabric.block_signatures_preverify([blocks[k] for k in names])
    assert [list(g) for g in got] == [fx["blocks"][k]["block_signatures"] for k in names]
    got = fabric.block_signatures_preverify([blocks[k] for k in names], bft=True)
    assert [list(g) for g in got] == [fx["blocks"][k]["block_signatures_bft"] for k in names]
    for m in fx["mutations"]:
        if "hex" in m:
            g = fabric.block_signatures_preverify([bytes.fromhex(m["hex"])], bft=m["bft"],
                                                  consenters=_cons(m))
            assert list(g[0]) == m["block_signatures"], m["name"]


@pytest.mark.gpu
def test_gpu_real_blocks_validate(fx):
    for name, blk in _blocks(fx).items():
        for keep in (False, True):
            got = [_tx(t) for t in fabric.block_preverify(blk, keep_keys=keep)]
            assert got == fx["blocks"][name]["txs"], (name, keep)


@pytest.mark.gpu
def test_gpu_real_sigfilter(fx):
    envs, want = [], []
    for name, blk in _blocks(fx).items():
        envs += _envs(blk)
        want += [tuple(x) for x in fx["blocks"][name]["sigfilter"]]
    for m in fx["mutations"]:
        if "envelope" in m:
            envs.append(bytes.fromhex(m["envelope"]))
            want.append(tuple(m["sigfilter"]))
    assert fabric.envelopes_preverify(envs) == want


@pytest.mark.gpu
def test_gpu_real_x509_links(fx):
    from bdls_amd import _lib
    _lib.ensure_init()
    certs = [bytes.fromhex(c) for c in fx["x509"]["certs"]]
    links = fx["x509"]["links"]
    ders = [certs[i] for i, _, _ in links]
    ln = np.array([len(c) for c in ders], np.uint32)
    off = np.zeros(len(ders), np.uint64)
    off[1:] = np.cumsum(ln[:-1])
    buf = np.frombuffer(b"".join(ders) + b"\0", np.uint8)

    def pub_of(der):
        from tests.golden.gen_real_blocks import names_and_key
        x, y = names_and_key(der)[2]
        return x.to_bytes(32, "big") + y.to_bytes(32, "big")

    pub = np.frombuffer(b"".join(pub_of(certs[j]) for _, j, _ in links), np.uint8)
    n = len(links)
    bm = np.zeros((n + 7) // 8, np.uint8)
    rs = np.zeros(n, np.uint8)
    _lib.check(_lib.lib().bh_verify_x509(buf.ctypes.data, off.ctypes.data, ln.ctypes.data,
                                         pub.ctypes.data, n, bm.ctypes.data, rs.ctypes.data))
    assert [int(x) for x in rs] == [l[2] for l in links]
