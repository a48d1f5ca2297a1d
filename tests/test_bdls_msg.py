"""BDLS drained-batch pre-verification (bh_bdls_preverify; SURVEY.md 8(a)
rows A15-A16): gogo/protobuf decoding of SignedProto / Message
(message.pb.go), participant gate and verifyMessage (consensus.go:449-493),
the proof loops of <lock>/<select>/<decide>/<lock-release>, <resync>
loopback flattening.

CPU: the committed fixture (tests/golden/bdls_messages.json, made by
tests/golden/gen_golden_bdls_msgs.py from oracle/bdls_msg_ref.py) is
re-derived by the oracle, and the C++ message logic in libbdlship.so agrees
with it when the per-SignedProto results are supplied
(BH_BDLS_F_GIVEN_REASONS -- no device work).
GPU (-m gpu): the same fixture and a 100-validator round verified on device,
statuses and per-SignedProto reasons bit-exact with the oracle."""
import json
import os
import random

import numpy as np
import pytest

from oracle import bdls_msg_ref as M
from oracle import ecdsa_ref as O
from tests.conftest import ROOT

FIX = os.path.join(ROOT, "tests", "golden", "bdls_messages.json")
CURVES = {"secp256k1": O.SECP256K1, "P-256": O.P256}
FIELDS = ("status", "bad_sp", "type", "distinct_signers", "height", "round", "sp_first",
          "sp_count")


@pytest.fixture(scope="module")
def fixture():
    with open(FIX) as f:
        return json.load(f)


def _lib_or_skip():
    from bdls_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libbdlship.so not built")


def test_fixture_covers_every_status(fixture):
    for case in fixture:
        seen = {m["status"] for m in case["messages"]}
        assert seen == set(range(19)), sorted(set(range(19)) - seen)


def test_oracle_rederives_fixture(fixture):
    for case in fixture:
        ids = [bytes.fromhex(h) for h in case["participants"]]
        res, rs = M.Preverifier(ids, CURVES[case["curve"]]).run(
            [bytes.fromhex(m["raw"]) for m in case["messages"]])
        assert rs == case["sp_reason"]
        for r, m in zip(res, case["messages"]):
            assert {f: getattr(r, f) for f in FIELDS} == {f: m[f] for f in FIELDS}, m["tag"]


def test_encode_decode_roundtrip():
    rng = random.Random(3)
    for _ in range(200):
        sp = M.SignedProto(rng.randrange(1, 2**32), rng.randbytes(rng.randrange(0, 300)),
                           rng.randbytes(32), rng.randbytes(32), rng.randbytes(rng.randrange(1, 33)),
                           rng.randbytes(rng.randrange(1, 33)))
        m = M.Message(rng.randrange(8), rng.randrange(2**64), rng.randrange(2**64),
                      rng.randbytes(rng.randrange(1, 50)), [sp] * rng.randrange(3),
                      sp if rng.random() < 0.5 else None)
        assert M.decode_message(M.encode_message(m)) == m
        assert M.decode_signed(M.encode_signed(sp)) == sp


def test_native_logic_matches_fixture(fixture):
    """C++ decode + gate + Go-ordered checks, signature results given."""
    _lib_or_skip()
    from bdls_amd import consensus
    for case in fixture:
        ids = [bytes.fromhex(h) for h in case["participants"]]
        raws = [bytes.fromhex(m["raw"]) for m in case["messages"]]
        res, rs = consensus.preverify(case["curve"], raws, ids,
                                      given_reasons=np.array(case["sp_reason"], np.uint8))
        assert len(rs) == len(case["sp_reason"])
        for r, m in zip(res, case["messages"]):
            assert {f: r[f] for f in FIELDS} == {f: m[f] for f in FIELDS}, m["tag"]


def test_native_no_quorum_flag(fixture):
    _lib_or_skip()
    from bdls_amd import consensus
    case = fixture[0]
    ids = [bytes.fromhex(h) for h in case["participants"]]
    raws = [bytes.fromhex(m["raw"]) for m in case["messages"]]
    res, _ = consensus.preverify(case["curve"], raws, ids, quorum=False,
                                 given_reasons=np.array(case["sp_reason"], np.uint8))
    ores, _ = M.Preverifier(ids, CURVES[case["curve"]], quorum=False).run(raws)
    for r, o, m in zip(res, ores, case["messages"]):
        assert r["status"] == o.status, m["tag"]
        assert r["status"] not in (15, 16, 17)


def test_native_wire_fuzz():
    """Random mutations of real messages: C++ and Python decoders agree on
    every status (signature results taken from the oracle)."""
    _lib_or_skip()
    from bdls_amd import consensus
    from tests.golden.gen_golden_bdls_msgs import build_round
    ids, msgs = build_round(O.SECP256K1, 4, 77, corrupt=False)
    rng = random.Random(5)
    raws = []
    for _ in range(400):
        b = bytearray(rng.choice(msgs)[1])
        for _ in range(rng.randrange(1, 4)):
            op = rng.randrange(3)
            if op == 0 and b:
                b[rng.randrange(len(b))] = rng.randrange(256)
            elif op == 1 and b:
                del b[rng.randrange(len(b)):]
            else:
                b.insert(rng.randrange(len(b) + 1), rng.randrange(256))
        raws.append(bytes(b))
    ores, ors = M.Preverifier(ids, O.SECP256K1).run(raws)
    res, rs = consensus.preverify("secp256k1", raws, ids, given_reasons=np.array(ors, np.uint8))
    assert len(rs) == len(ors)
    for r, o in zip(res, ores):
        assert {f: r[f] for f in FIELDS} == {f: getattr(o, f) for f in FIELDS}


def test_native_inner_fuzz():
    """Mutations INSIDE the signed Message of leader messages, re-signed by
    the leader: exercises proof decoding, proof checks and quorum logic."""
    _lib_or_skip()
    from bdls_amd import consensus
    from tests.golden.gen_golden_bdls_msgs import build_round
    ids, msgs, R = build_round(O.SECP256K1, 4, 78, corrupt=False, with_round=True)
    leaders = [m for t, m in msgs if t in ("lock", "decide", "select_nil", "resync")]
    rng = random.Random(6)
    raws = []
    for _ in range(300):
        sp = M.decode_signed(rng.choice(leaders))
        b = bytearray(sp.message)
        for _ in range(rng.randrange(1, 3)):
            op = rng.randrange(3)
            if op == 0 and b:
                b[rng.randrange(len(b))] ^= 1 << rng.randrange(8)
            elif op == 1 and b:
                del b[rng.randrange(len(b))]
            else:
                b.insert(rng.randrange(len(b) + 1), rng.randrange(256))
        raws.append(M.encode_signed(M.sign(O.SECP256K1, R.keys[R.leader], bytes(b),
                                           rng.randrange(1, O.SECP256K1.n))))
    ores, ors = M.Preverifier(ids, O.SECP256K1).run(raws)
    assert len({o.status for o in ores}) >= 6
    res, rs = consensus.preverify("secp256k1", raws, ids, given_reasons=np.array(ors, np.uint8))
    for r, o in zip(res, ores):
        assert {f: r[f] for f in FIELDS} == {f: getattr(o, f) for f in FIELDS}


def test_native_rejects_bad_args():
    _lib_or_skip()
    from bdls_amd import _lib, consensus
    with pytest.raises(_lib.EngineError):
        consensus.preverify("secp256k1", [b"\x08\x01"], [bytes(64)],
                            given_reasons=np.zeros(0, np.uint8))  # sp_cap too small


@pytest.mark.gpu
@pytest.mark.parametrize("ci", [0, 1])
def test_gpu_fixture(fixture, ci):
    from bdls_amd import consensus
    case = fixture[ci]
    ids = [bytes.fromhex(h) for h in case["participants"]]
    res, rs = consensus.preverify(case["curve"], [bytes.fromhex(m["raw"]) for m in case["messages"]],
                                  ids)
    assert [int(x) for x in rs] == case["sp_reason"]
    for r, m in zip(res, case["messages"]):
        assert {f: r[f] for f in FIELDS} == {f: m[f] for f in FIELDS}, m["tag"]


@pytest.mark.gpu
@pytest.mark.parametrize("curve", ["secp256k1", "P-256"])
def test_gpu_round_100_validators(curve):
    """BASELINE config 4 shape with real wire messages: 100 validators."""
    from bdls_amd import consensus
    from tests.golden.gen_golden_bdls_msgs import build_round
    ids, msgs = build_round(CURVES[curve], 100, 4, corrupt=False)
    raws = [m for _, m in msgs]
    res, rs = consensus.preverify(curve, raws, ids)
    ores, ors = M.Preverifier(ids, CURVES[curve]).run(raws)
    assert [int(x) for x in rs] == ors
    assert all(r["status"] == 0 for r in res)
    for r, o in zip(res, ores):
        assert {f: r[f] for f in FIELDS} == {f: getattr(o, f) for f in FIELDS}


@pytest.mark.parametrize("curve,cname", [(1, "secp256k1"), (0, "P-256")])
def test_wire_round_generator(curve, cname):
    """workload/gen.c wire rounds (bench config 4) decode and verify as
    all-valid under the oracle, and the native logic agrees."""
    _lib_or_skip()
    from bdls_amd import consensus, workload
    ids, raws = workload.generate_bdls_wire_round(10, curve, seed=9)
    res, rs = M.Preverifier(ids, CURVES[cname]).run(raws)
    assert all(r.status == 0 for r in res) and set(rs) == {0}
    t2p1 = 2 * 3 + 1
    assert len(rs) == 2 * 10 + 2 * (1 + t2p1)
    assert [r.distinct_signers for r in res if r.type in (2, 6)] == [t2p1, t2p1]
    nres, nrs = consensus.preverify(cname, raws, ids, given_reasons=np.array(rs, np.uint8))
    assert all(r["status"] == 0 for r in nres)
