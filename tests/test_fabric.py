"""Fabric block pre-verification (bh_fabric_block_preverify) against the CPU
oracle (oracle/fabric_ref.py: the reference's sequential validateTx /
ValidateTransaction / SignatureSetToValidIdentities flow and protobuf-go wire
rules, restated) and the generator's by-construction expectations.

CPU (no device work): the oracle against the generator on every corruption
class; the C++ decode / identity resolution (BH_FAB_F_DECODE_ONLY) against the
oracle's, on the generated blocks and on thousands of mutated envelopes.
GPU: the full pre-verification, bit-exact per transaction and per
endorsement, on config 3's block and on every corruption class.
"""
import hashlib
import random

import pytest

from bdls_amd import fabric
from bdls_amd.workload import fabric as F
from oracle import ecdsa_ref as O
from oracle import fabric_ref as R


def _py_verify(x, y, msg, sig):
    return O.identity_verify(O.P256, x, y, msg, sig)[1]


def _orc_verify(x, y, msg, sig):
    from oracle import orc
    return orc.csp_verify(x.to_bytes(32, "big") + y.to_bytes(32, "big"), sig,
                          hashlib.sha256(msg).digest())


def _want(fb, i):
    return (fb.tx_status[i], fb.tx_creator[i], fb.tx_endorse[i], fb.tx_valid_identities[i])


def _got(t):
    return (t.status, t.creator, t.endorse, t.valid_endorsers)


@pytest.fixture(scope="module")
def classes_block():
    return F.generate_fabric_block(ntx=2 * len(F.CORRUPTIONS), corrupt_den=0,
                                   classes=F.CORRUPTIONS, seed=7)


def test_oracle_matches_construction(classes_block):
    fb = classes_block
    out = R.validate_block(fb.block, _py_verify)
    assert [_got(o) for o in out] == [_want(fb, i) for i in range(fb.ntx)]


def _decode_pair(block):
    py = R.validate_block(block, None, decode_only=True)
    cc = fabric.block_preverify(block, decode_only=True)
    return [_got(o) for o in py], [_got(o) for o in cc]


def test_decode_only_matches_oracle(classes_block):
    py, cc = _decode_pair(classes_block.block)
    assert py == cc


def _block_of(envs):
    data = b"".join(F.pb_bytes(1, e) for e in envs)
    return F.pb_bytes(2, data)


def _envelopes(block):
    blk = R.unmarshal(block, R.BLOCK_SPEC)
    return blk["data"]["data"]


def _mutate(rng, b: bytes) -> bytes:
    b = bytearray(b)
    for _ in range(rng.randrange(1, 4)):
        op = rng.randrange(6)
        if op == 0 and b:
            b[rng.randrange(len(b))] = rng.randrange(256)
        elif op == 1 and b:
            i = rng.randrange(len(b))
            del b[i:i + rng.randrange(1, 6)]
        elif op == 2:
            b.insert(rng.randrange(len(b) + 1), rng.randrange(256))
        elif op == 3 and b:  # truncate
            b = b[:rng.randrange(len(b))]
        elif op == 4 and b:  # flip a varint continuation bit
            b[rng.randrange(len(b))] ^= 0x80
        else:  # a field with a rare wire type / number
            tag = rng.choice([0x0b, 0x0c, 0x0e, 0x0f, 0x14, 0x1a, 0x08, 0xf8, 0x80])
            b[rng.randrange(len(b) + 1):0] = bytes([tag, rng.randrange(256)])
    return bytes(b)


def _nested_mutation(rng, env: bytes) -> bytes:
    """Mutate one nested message (payload / header / channel header /
    signature header / transaction / endorsement) and re-encode outward."""
    e = R.unmarshal(env, R.ENVELOPE_SPEC)
    pl = R.unmarshal(e["payload"], R.PAYLOAD_SPEC)
    which = rng.randrange(6)
    hdr = pl["header"]
    ch, sh = hdr["channel_header"], hdr["signature_header"]
    data = pl["data"]
    if which == 0:
        ch = _mutate(rng, ch)
    elif which == 1:
        sh = _mutate(rng, sh)
    elif which == 2:
        data = _mutate(rng, data)
    elif which == 3:
        tx = R.unmarshal(data, R.TRANSACTION_SPEC)
        act = tx["actions"][0]
        cap = R.unmarshal(act["payload"], R.CC_ACTION_PAYLOAD_SPEC)
        ea = cap["action"]
        ends = ea["endorsements"]
        k = rng.randrange(len(ends))
        enc = [F.pb_bytes(1, x["endorser"]) + F.pb_bytes(2, x["signature"]) for x in ends]
        enc[k] = _mutate(rng, enc[k]) if rng.random() < 0.5 else \
            F.pb_bytes(1, _mutate(rng, ends[k]["endorser"])) + F.pb_bytes(2, ends[k]["signature"])
        cea = F.pb_bytes(1, ea["proposal_response_payload"]) + b"".join(F.pb_bytes(2, x) for x in enc)
        capb = F.pb_bytes(1, cap["chaincode_proposal_payload"]) + F.pb_bytes(2, cea)
        data = F.pb_bytes(1, F.pb_bytes(1, act["header"]) + F.pb_bytes(2, capb))
    elif which == 4:
        hdr_b = _mutate(rng, F.pb_bytes(1, ch) + F.pb_bytes(2, sh))
        return F.pb_bytes(1, F.pb_bytes(1, hdr_b) + F.pb_bytes(2, data)) + F.pb_bytes(2, e["signature"])
    else:
        return _mutate(rng, env)
    payload = F.pb_bytes(1, F.pb_bytes(1, ch) + F.pb_bytes(2, sh)) + F.pb_bytes(2, data)
    return F.pb_bytes(1, payload) + F.pb_bytes(2, e["signature"])


def test_decode_fuzz_matches_oracle(classes_block):
    rng = random.Random(11)
    envs = _envelopes(classes_block.block)
    base = [envs[0], envs[3], envs[4]]  # a valid tx and two endorsement variants
    for it in range(3000):
        env = _nested_mutation(rng, rng.choice(base))
        block = _block_of([env])
        py, cc = _decode_pair(block)
        assert py == cc, (it, env.hex())


def test_identity_pem_variants():
    """PEM framing cases of Go encoding/pem Decode as the MSP meets them."""
    fb = F.generate_fabric_block(ntx=1, corrupt_den=0, seed=9)
    env = _envelopes(fb.block)[0]
    e = R.unmarshal(env, R.ENVELOPE_SPEC)
    pl = R.unmarshal(e["payload"], R.PAYLOAD_SPEC)
    sh = R.unmarshal(pl["header"]["signature_header"], R.SIGNATURE_HEADER_SPEC)
    si = R.unmarshal(sh["creator"], R.SERIALIZED_IDENTITY_SPEC)
    p = si["id_bytes"]
    body = p.split(b"\n", 1)[1].rsplit(b"-----END", 1)[0]
    variants = [p, b"junk\n" + p, p.replace(b"\n", b"\r\n"), p + b"trailing",
                b"-----BEGIN CERTIFICATE-----\nX: y\n\n" + body + b"-----END CERTIFICATE-----\n",
                p.replace(b"-----END CERTIFICATE-----", b"-----END CERT-----"),
                p.replace(b"\n-----END", b"  \t\n-----END"), p[:-1], p.replace(b"=", b""),
                b"-----BEGIN CERTIFICATE-----\n" + body.replace(b"\n", b" \n") +
                b"-----END CERTIFICATE-----   \n"]
    for v in variants:
        ser = F.pb_bytes(1, si["mspid"]) + F.pb_bytes(2, v)
        sh2 = F.pb_bytes(1, ser) + F.pb_bytes(2, sh["nonce"])
        payload = F.pb_bytes(1, F.pb_bytes(1, pl["header"]["channel_header"]) + F.pb_bytes(2, sh2)) \
            + F.pb_bytes(2, pl["data"])
        block = _block_of([F.pb_bytes(1, payload) + F.pb_bytes(2, e["signature"])])
        py, cc = _decode_pair(block)
        assert py == cc, v


@pytest.mark.gpu
def test_gpu_every_class(classes_block):
    fb = classes_block
    got = fabric.block_preverify(fb.block)
    assert [_got(t) for t in got] == [_want(fb, i) for i in range(fb.ntx)]


@pytest.mark.gpu
def test_gpu_config3_block():
    """BASELINE config 3's block: 500 txs x (creator + 3 endorsements), 1/100
    corrupted; bit-exact against the construction and the oracle (OpenSSL
    verify), then again with the endorser keys kept in the device registry."""
    fb = F.generate_fabric_block(seed=3)
    assert fb.ntx == 500
    want = [_want(fb, i) for i in range(fb.ntx)]
    oracle = [_got(o) for o in R.validate_block(fb.block, _orc_verify)]
    assert oracle == want
    for keep in (False, True, True):
        got = fabric.block_preverify(fb.block, keep_keys=keep)
        assert [_got(t) for t in got] == want


# ---------------------------------------------------------------- orderer callers
@pytest.fixture(scope="module")
def signed_blocks():
    return F.generate_signed_blocks(nblocks=2 * len(F.BLOCKSIG_CORRUPTIONS),
                                    classes=F.BLOCKSIG_CORRUPTIONS)


def test_blocksig_oracle_matches_construction(signed_blocks):
    blocks, exp = signed_blocks
    assert [R.block_signatures(b, _py_verify) for b in blocks] == exp


def test_blocksig_decode_matches_oracle(signed_blocks):
    blocks, _ = signed_blocks
    rng = random.Random(5)
    cases = list(blocks) + [_mutate(rng, rng.choice(blocks)) for _ in range(1500)]
    py = [R.block_signatures(b, None, decode_only=True) for b in cases]
    cc = fabric.block_signatures_preverify(cases, decode_only=True)
    assert py == [tuple(c) for c in cc]


def test_sigfilter_decode_matches_oracle(classes_block):
    rng = random.Random(6)
    envs = _envelopes(classes_block.block)
    cases = list(envs) + [_nested_mutation(rng, rng.choice(envs[:5])) for _ in range(1500)]
    py = [R.sigfilter(e, None, decode_only=True) for e in cases]
    cc = fabric.envelopes_preverify(cases, decode_only=True)
    assert py == cc


def _sets_case(seed=8):
    """Signature sets drawn from a block's endorsements: duplicates, bad
    identities, failed-then-valid identities, empty sets."""
    fb = F.generate_fabric_block(ntx=12, corrupt_den=0, classes=F.CORRUPTIONS, seed=seed)
    sds = []
    for env in _envelopes(fb.block):
        try:
            e = R.unmarshal(env, R.ENVELOPE_SPEC)
            pl = R.unmarshal(e["payload"], R.PAYLOAD_SPEC)
            tx = R.unmarshal(pl["data"], R.TRANSACTION_SPEC)
            cap = R.unmarshal(tx["actions"][0]["payload"], R.CC_ACTION_PAYLOAD_SPEC)
        except (R.DecodeError, IndexError, TypeError):
            continue
        prp = cap["action"]["proposal_response_payload"]
        for x in cap["action"]["endorsements"]:
            sds.append((x["endorser"], prp + x["endorser"], x["signature"]))
    rng = random.Random(seed)
    sets = [[]]
    for _ in range(40):
        sets.append([rng.choice(sds) for _ in range(rng.randrange(1, 7))])
    return sets


def test_sets_decode_matches_oracle():
    sets = _sets_case()
    py = [R.signature_set_to_valid_identities(s, None, decode_only=True) for s in sets]
    cc = fabric.signature_sets_verify(sets, decode_only=True)
    assert py == cc


@pytest.mark.gpu
def test_gpu_signature_sets():
    sets = _sets_case()
    want = [R.signature_set_to_valid_identities(s, _orc_verify) for s in sets]
    assert fabric.signature_sets_verify(sets) == want


@pytest.mark.gpu
def test_gpu_sigfilter(classes_block):
    envs = _envelopes(classes_block.block)
    want = [R.sigfilter(e, _orc_verify) for e in envs]
    assert fabric.envelopes_preverify(envs) == want


@pytest.mark.gpu
def test_gpu_block_signatures(signed_blocks):
    blocks, exp = signed_blocks
    got = fabric.block_signatures_preverify(blocks)
    assert [tuple(g) for g in got] == exp


# ---------------------------------------------------------------- BFT block signatures
@pytest.fixture(scope="module")
def bft_blocks():
    return F.generate_bft_signed_blocks(nblocks=len(F.BFT_BLOCKSIG_CORRUPTIONS),
                                        classes=F.BFT_BLOCKSIG_CORRUPTIONS)


def test_bft_oracle_matches_construction(bft_blocks):
    blocks, cons, exp = bft_blocks
    assert [R.block_signatures(b, _py_verify, bft=True, consenters=cons) for b in blocks] == exp


def test_bft_reference_cases():
    """protoutil/blockutils_test.go:382-493 restated on the oracle and the C++
    decode: empty metadata; signatures by identifier 1 and 3 resolve to
    MarshalOrPanic(SerializedIdentity{msp1, identity1}) / {msp3, identity3};
    a SignatureHeader signature keeps the creator form with bftEnabled."""
    cons = [(1, b"msp1", b"identity1"), (2, b"msp2", b"identity2"), (3, b"msp3", b"identity3")]
    assert R.search_consenter_identity_by_id(cons, 1) == b"\n\x04msp1\x12\tidentity1"
    assert R.search_consenter_identity_by_id(cons, 3) == b"\n\x04msp3\x12\tidentity3"
    assert R.search_consenter_identity_by_id(cons, 4) == b""
    empty = F.pb_bytes(1, b"")  # header {}, metadata {}
    by_id = F.pb_bytes(1, b"") + F.pb_bytes(3, F.pb_bytes(1, F.pb_bytes(2, F.pb_bytes(
        3, F.pb_varint(1, 1))) + F.pb_bytes(2, F.pb_bytes(3, F.pb_varint(1, 3)))))
    by_creator = F.pb_bytes(1, b"") + F.pb_bytes(3, F.pb_bytes(1, F.pb_bytes(2, F.pb_bytes(
        1, F.pb_bytes(1, b"creator1")))))
    # the identities are not certificates: DeserializeIdentity fails -> 254
    want = [(R.BLK_NO_SIGNATURES, [], 0), (R.BLK_OK, [254, 254], 0), (R.BLK_OK, [254], 0)]
    cases = [empty, by_id, by_creator]
    assert [R.block_signatures(b, None, decode_only=True, bft=True, consenters=cons)
            for b in cases] == want
    got = fabric.block_signatures_preverify(cases, decode_only=True, bft=True, consenters=cons)
    assert [tuple(g) for g in got] == want
    # without bftEnabled the identifier form is a SignatureHeader form with an
    # empty header: empty creator -> 254 for both
    assert R.block_signatures(by_id, None, decode_only=True, bft=False)[1] == [254, 254]


def test_bft_decode_matches_oracle(bft_blocks):
    blocks, cons, _ = bft_blocks
    rng = random.Random(15)
    cases = list(blocks) + [_mutate(rng, rng.choice(blocks)) for _ in range(1000)]
    for bft in (True, False):
        py = [R.block_signatures(b, None, decode_only=True, bft=bft, consenters=cons) for b in cases]
        cc = fabric.block_signatures_preverify(cases, decode_only=True, bft=bft, consenters=cons)
        assert py == [tuple(c) for c in cc]


@pytest.mark.gpu
def test_gpu_bft_block_signatures(bft_blocks):
    blocks, cons, exp = bft_blocks
    want = [R.block_signatures(b, _orc_verify, bft=True, consenters=cons) for b in blocks]
    assert want == exp
    got = fabric.block_signatures_preverify(blocks, bft=True, consenters=cons)
    assert [tuple(g) for g in got] == exp
    # the same blocks without bftEnabled: identifier-form signatures have no creator
    got = fabric.block_signatures_preverify(blocks, consenters=cons)
    assert [tuple(g) for g in got] == [R.block_signatures(b, _orc_verify) for b in blocks]


@pytest.mark.gpu
def test_gpu_sets_many_failed_duplicates():
    """An identity that repeats itself after bad signatures (Go verifies each
    until one verifies): 300 failing entries then a valid one then more --
    two device passes, bit-exact with the sequential loop."""
    sets = _sets_case()
    sds = [sd for s in sets for sd in s]
    good = next(sd for sd in sds if R.signature_set_to_valid_identities([sd], _orc_verify)[1] == 1)
    bad = (good[0], good[1] + b"x", good[2])
    other = next(sd for sd in sds if sd[0] != good[0])
    big = [bad] * 300 + [good, bad, other, good]
    cases = [big, [bad, bad], [good, bad, good]]
    want = [R.signature_set_to_valid_identities(s, _orc_verify) for s in cases]
    assert want[0][0][300] == 0 and want[0][0][301] == 253
    assert fabric.signature_sets_verify(cases) == want


P384_N = int("ffffffffffffffffffffffffffffffffffffffffffffffffc7634d81f4372ddf"
             "581a0db248b0a77aecec196accc52973", 16)


def _twin_identity(ser: bytes, order: int) -> bytes:
    """The same certificate with its signature's S replaced by order - S (the
    high-S / low-S twin that sanitizeECDSASignedCert maps back, msp/cert.go:
    76-116, when `order` is the issuer's curve order)."""
    si = R.unmarshal(ser, R.SERIALIZED_IDENTITY_SPEC)
    der = R.pem_decode(si["id_bytes"])
    _x, _y, tbs, sig = R.cert_p256_key(der)
    rc, r, s = O.unmarshal_ecdsa_signature(sig)
    assert rc == O.R_OK
    twin_sig = F.der(0x30, F.der_int(r) + F.der_int(order - s))
    return F.serialized_identity(si["mspid"].decode(), F.pem(F.x509_cert(tbs, twin_sig)))


def test_twin_certificates_share_the_identity_key():
    """Go's identity Id hashes the certificate sanitized to low-S with
    the ISSUER's order, so a certificate and its S-twin are one identity even
    for a P-384 CA; the de-duplication key must not depend on P-256's order."""
    sets = _sets_case()
    ser = sets[1][0][0]
    base = R.deserialize(ser)
    for order in (O.P256.n, P384_N):
        twin = R.deserialize(_twin_identity(ser, order))
        assert twin is not None and twin.key == base.key
        assert (twin.x, twin.y) == (base.x, base.y)


@pytest.mark.gpu
def test_gpu_twin_certificates_deduplicated():
    sets = _sets_case()
    sds = [sd for s in sets for sd in s]
    good = next(sd for sd in sds if R.signature_set_to_valid_identities([sd], _orc_verify)[1] == 1)
    cases = []
    for order in (O.P256.n, P384_N):
        twin = (_twin_identity(good[0], order), good[1], good[2])
        cases += [[good, twin], [twin, good], [(good[0], good[1] + b"x", good[2]), twin]]
    want = [R.signature_set_to_valid_identities(s, _orc_verify) for s in cases]
    assert [w[1] for w in want] == [1, 1, 1] * 2
    assert want[0][0] == [0, 253]
    assert fabric.signature_sets_verify(cases) == want


def _recorded_calls(block):
    """Every (x, y, msg, sig) the sequential validator flow verifies."""
    calls = []

    def rec(x, y, msg, sig):
        calls.append((x, y, bytes(msg), bytes(sig)))
        return _orc_verify(x, y, msg, sig)
    out = R.validate_block(block, rec)
    return out, calls


def _ref_key(ref):
    ident = R.deserialize(ref.identity)
    return None if ident is None else (ident.x, ident.y, ref.data, ref.signature)


def test_block_refs_cover_every_go_verify(classes_block):
    """bh_fabric_block_preverify_refs (decode only): every signature check the
    sequential flow makes (checkSignatureFromCreator, SignatureSetToValid-
    Identities) has a reference with the same identity key, signed bytes and
    signature -- the keys of the verified-signature cache."""
    block = classes_block.block
    txs, creators, ends = fabric.block_preverify_refs(block, decode_only=True)
    assert [_got(t) for t in txs] == [_got(t) for t in fabric.block_preverify(block, decode_only=True)]
    assert len(ends) == sum(len(t.endorse) for t in txs)
    keys = {_ref_key(r) for r in creators + ends if r is not None}
    _, calls = _recorded_calls(block)
    assert calls and set(calls) <= keys
    assert all(r is None or r.reason in (fabric.NOT_VERIFIED, fabric.E_BAD_IDENTITY, fabric.E_DUPLICATE)
               for r in creators + ends)


@pytest.mark.gpu
def test_gpu_block_refs_two_phase(classes_block):
    """Phase 1: the device batch with references; phase 2: the sequential flow
    consulting a cache of the cacheable outcomes (BH_R_OK -> valid, BH_R_BAD_KEY
    / R_RANGE / MATH -> invalid), falling back to a CPU verify on a miss. The
    results equal the plain flow, and only non-cacheable records miss."""
    block = classes_block.block
    txs, creators, ends = fabric.block_preverify_refs(block)
    plain = fabric.block_preverify(block)
    assert [_got(t) for t in txs] == [_got(t) for t in plain]
    assert [r.reason if r else None for r in ends] == [e for t in plain for e in t.endorse]
    for t, c in zip(plain, creators):
        if c is not None:
            assert c.reason == t.creator
    cache = {}
    for r in creators + ends:
        if r is not None and r.reason in (0, 7, 8, 9):
            cache[_ref_key(r)] = r.reason
    misses = []

    def phase2(x, y, msg, sig):
        k = (x, y, bytes(msg), bytes(sig))
        if k in cache:
            return cache[k]
        misses.append(k)
        return _orc_verify(x, y, msg, sig)
    want, calls = _recorded_calls(block)
    got = R.validate_block(block, phase2)
    assert [_got(o) for o in got] == [_got(o) for o in want]
    assert len(cache) > 0 and len(misses) < len(calls)
    for k in misses:  # a miss is a record whose Go error text depends on the parse
        assert _orc_verify(*k) in (1, 2, 3, 4, 5, 6)


# ---------------------------------------------------------------- implicit-meta policies, cache first
ORGS = [b"Org1MSP", b"Org2MSP", b"Org3MSP", b"Org4MSP"]


def _identity_verify(ident_bytes, data, sig):
    ident = R.deserialize(ident_bytes)
    return _orc_verify(ident.x, ident.y, data, sig)


def _policy_results(block, identity_verify, before=None, statuses=None):
    """The validation plugin's endorsement-policy evaluation per transaction
    that passed validateTx (status OK, endorser tx): the channel default
    "MAJORITY Endorsement" (sampleconfig/configtx.yaml:241-243) over the four
    orgs' "OR('OrgN.member')" policies (:69-71)."""
    subs = [R.signed_by_member(o) for o in ORGS]
    sets = R.endorsement_sets(block)
    out = []
    for st, sd in zip(statuses, sets):
        if st != R.OK or sd is None:
            out.append(None)
            continue
        out.append(R.implicit_meta_evaluate(sd, subs, "MAJORITY", identity_verify, before))
    return out


def test_implicit_meta_majority_oracle(classes_block):
    """The oracle's implicit-meta flow on the classes block: a transaction's
    endorsement policy holds iff at least 3 of its 4 orgs have a valid,
    de-duplicated endorser -- the generator's own count."""
    fb = classes_block
    statuses = [o.status for o in R.validate_block(fb.block, _orc_verify)]
    pol = _policy_results(fb.block, _identity_verify, statuses=statuses)
    for i, p in enumerate(pol):
        if p is not None:
            assert p == (fb.tx_valid_identities[i] >= 3), (i, fb.tx_class[i])
    assert any(p is True for p in pol) and any(p is False for p in pol)


def test_sigcache_key_unambiguous():
    """identity || 0x00 || sig collided for (b"a\\0", b"b") and
    (b"a", b"\\0b"); the length-prefixed key does not."""
    c = fabric.SigCache()
    g = c.begin()
    c.put(g, b"a\0", b"b", b"data", fabric.VALID)
    assert c.lookup(b"a", b"data", b"\0b") is None
    assert c.lookup(b"a\0", b"data", b"b") == fabric.VALID
    assert c.lookup(b"a\0", b"other", b"b") is None  # the signed bytes must match
    c.release(g)
    assert c.lookup(b"a\0", b"data", b"b") is None


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["config3", "classes"])
def test_gpu_two_phase_implicit_meta_one_device_batch(classes_block, which):
    """VERDICT r3 missing #2: phase 1 verifies the block's signatures in ONE
    device batch and fills the verified-signature cache; phase 2 is the
    unchanged sequential validation -- creator checks consulting the cache,
    then per transaction the implicit-meta MAJORITY endorsement policy whose
    EvaluateSignedData first runs the cache-first PreverifySets
    (INTEGRATION.md 6). Phase 2 issues NO device work (bh_device_stats), its
    results equal the plain sequential flow's, and the old consumer (no cache
    lookup, min batch 1) would have issued one device batch per evaluation."""
    from bdls_amd import _lib
    _lib.ensure_init()
    fb = classes_block if which == "classes" else F.generate_fabric_block(seed=3)
    block = fb.block
    # the plain flow (no engine): statuses and policy outcomes
    plain = R.validate_block(block, _orc_verify)
    statuses = [o.status for o in plain]
    want_pol = _policy_results(block, _identity_verify, statuses=statuses)
    # phase 1: one device batch
    b0 = _lib.device_stats()[0]
    txs, creators, ends = fabric.block_preverify_refs(block)
    b1 = _lib.device_stats()[0]
    # one device batch; the classes block holds the endorse_dup_after_invalid
    # class, whose later signature of an identity that failed earlier in the
    # set is checked in the documented follow-up round
    assert b1 - b0 == (2 if which == "classes" else 1)
    cache = fabric.SigCache()
    gen = cache.begin()
    for r in creators + ends:
        if r is not None and r.reason in fabric.CACHEABLE:
            cache.put(gen, r.identity, r.signature, r.data, fabric.CACHEABLE[r.reason])
    xy_cache = {_ref_key(r): r.reason for r in creators + ends
                if r is not None and r.reason in fabric.CACHEABLE}
    go_verifies = []

    def creator_verify(x, y, msg, sig):  # checkSignatureFromCreator's consult site
        k = (x, y, bytes(msg), bytes(sig))
        if k in xy_cache:
            return xy_cache[k]
        go_verifies.append(k)
        return _orc_verify(x, y, msg, sig)

    def identity_verify(ident_bytes, data, sig):  # SignatureSetToValidIdentities' consult site
        out = cache.lookup(ident_bytes, data, sig)
        if out is not None:
            return 0 if out == fabric.VALID else 9
        go_verifies.append((ident_bytes, data, sig))
        return _identity_verify(ident_bytes, data, sig)

    stats = {}

    def before(sd):
        return fabric.preverify_sets(cache, [sd], stats=stats)

    got = R.validate_block(block, creator_verify)
    got_pol = _policy_results(block, identity_verify, before, [o.status for o in got])
    b2 = _lib.device_stats()[0]
    assert [_got(o) for o in got] == [_got(o) for o in plain]
    assert got_pol == want_pol
    assert b2 == b1 and stats.get("device_calls", 0) == 0  # phase 2: no device work
    # every lookup that missed is a record whose outcome is not cacheable
    # (parse-dependent Go error); the loop may not even reach it (the policy
    # threshold is met first)
    uncacheable = {(r.identity, r.data, r.signature) for r in ends
                   if r is not None and r.reason not in fabric.CACHEABLE}
    assert stats["lookups"] > 0 and stats["lookups"] - stats["hits"] <= len(uncacheable)
    # the misses are exactly the non-cacheable records (parse-dependent Go errors)
    for k in go_verifies:
        r = _orc_verify(*k) if len(k) == 4 and isinstance(k[0], int) else _identity_verify(*k)
        assert r in (1, 2, 3, 4, 5, 6)
    if which == "classes":
        # the round-3 consumer (device call whenever the set is non-empty, no
        # cache lookup) issues one device batch per policy evaluation
        empty = fabric.SigCache()
        n_eval = sum(p is not None for p in want_pol)
        b3 = _lib.device_stats()[0]
        _policy_results(block, identity_verify,
                        lambda sd: fabric.preverify_sets(empty, [sd], min_batch=1),
                        [o.status for o in got])
        assert _lib.device_stats()[0] - b3 == n_eval


_DECODE_SCRIPT = r"""
import json, sys
sys.path.insert(0, sys.argv[1])
from bdls_amd import fabric
from bdls_amd.workload import fabric as F
from tests.test_fabric import _got
out = []
for seed, kw in ((7, dict(ntx=2 * len(F.CORRUPTIONS), corrupt_den=0, classes=F.CORRUPTIONS)),
                 (3, {})):
    fb = F.generate_fabric_block(seed=seed, **kw)
    for _ in range(3):  # the pool reused call after call
        out.append([list(map(str, _got(o))) for o in fabric.block_preverify(fb.block,
                                                                            decode_only=True)])
print(json.dumps(out))
"""


def test_parallel_decode_matches_serial():
    """The block decode's worker pool (fabric.cpp Pool: generation-tagged
    chunk claims, per-chunk identity memos; one thread by default since round
    6) gives the same per-transaction outcome at 1, 2, 4 and 8 threads, on the
    every-class block and on a config-3 block, three calls each in one
    process. Subprocesses: the pool size is read once per process."""
    import json
    import os
    import subprocess
    import sys
    from tests.conftest import ROOT
    outs = {}
    for t in (1, 2, 4, 8):
        env = dict(os.environ, BH_DECODE_THREADS=str(t))
        r = subprocess.run([sys.executable, "-c", _DECODE_SCRIPT, ROOT], env=env, cwd=ROOT,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        outs[t] = json.loads(r.stdout.strip().splitlines()[-1])
    for t in (2, 4, 8):
        assert outs[t] == outs[1]
