#!/usr/bin/env python3
"""Golden fixtures for the BDLS drained-batch pre-verifier (bh_bdls_preverify).

Run from the repo root:  python tests/golden/gen_golden_bdls_msgs.py
Output (committed): tests/golden/bdls_messages.json

Raw consensus messages as vendor/github.com/BDLS-bft/bdls would put on the
wire (SignedProto.Marshal of a signed Message, message.pb.go :300-356), for
one height/round driven the way consensus.go does it: <roundchange> from every
participant, the leader's <lock> with 2t+1 <roundchange> proofs, <select>,
<commit> from every participant, the leader's <decide> with 2t+1 <commit>
proofs, a <lock-release> embedding the lock, a <resync> carrying messages
for the loopback, plus one corrupted variant per check of the pre-verifier
contract (include/bdls_hip.h) and wire-format edge cases. Expected statuses
and per-SignedProto reasons come from oracle/bdls_msg_ref.py (which uses
oracle/ecdsa_ref.py for SignedProto.Verify). Keys and nonces are seeded.
"""
from __future__ import annotations

import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import bdls_msg_ref as M  # noqa: E402
from oracle import ecdsa_ref as O  # noqa: E402


class Round:
    """Participants + signing helpers for one (height, round)."""

    def __init__(self, curve: O.Curve, nval: int, seed: int, height: int = 7, rnd: int = 3):
        self.c = curve
        self.rng = random.Random(seed)
        self.keys = [self.rng.randrange(1, curve.n) for _ in range(nval)]
        self.ids = []
        for d in self.keys:
            x, y = O.pubkey(curve, d)
            self.ids.append(x.to_bytes(32, "big") + y.to_bytes(32, "big"))
        self.h, self.r = height, rnd
        self.t = (nval - 1) // 3
        self.leader = rnd % nval
        self.state = b"block-" + bytes(self.rng.randrange(256) for _ in range(40))

    def signed(self, who: int | None, m: M.Message, d: int | None = None,
               version: int = 1) -> M.SignedProto:
        key = self.keys[who] if who is not None else d
        return M.sign(self.c, key, M.encode_message(m), self.rng.randrange(1, self.c.n), version)

    def msg(self, typ, state=None, proofs=(), lr=None, h=None, r=None):
        return M.Message(type=typ, height=self.h if h is None else h,
                         round=self.r if r is None else r, state=state, proofs=list(proofs),
                         lock_release=lr)


def build_round(curve: O.Curve, nval: int, seed: int, corrupt: bool = True,
                with_round: bool = False):
    """-> (participants list, list of (tag, raw bytes)[, Round])"""
    R = Round(curve, nval, seed)
    q = 2 * R.t + 1
    L = R.leader
    out = []
    rc = [R.signed(v, R.msg(M.ROUNDCHANGE, R.state)) for v in range(nval)]
    cm = [R.signed(v, R.msg(M.COMMIT, R.state)) for v in range(nval)]
    for v in range(nval):
        out.append(("roundchange", M.encode_signed(rc[v])))
    lock = R.signed(L, R.msg(M.LOCK, R.state, rc[:q]))
    out.append(("lock", M.encode_signed(lock)))
    rc_nil = [R.signed(v, R.msg(M.ROUNDCHANGE, None)) for v in range(q)]
    out.append(("select_nil", M.encode_signed(R.signed(L, R.msg(M.SELECT, None, rc_nil)))))
    for v in range(nval):
        out.append(("commit", M.encode_signed(cm[v])))
    out.append(("decide", M.encode_signed(R.signed(L, R.msg(M.DECIDE, R.state, cm[:q])))))
    out.append(("lockrelease", M.encode_signed(
        R.signed((L + 1) % nval, R.msg(M.LOCKRELEASE, None, lr=lock, r=R.r + 1)))))
    out.append(("resync", M.encode_signed(R.signed(L, R.msg(M.RESYNC, None, [rc[1], lock, cm[2]])))))
    out.append(("nop", M.encode_signed(R.signed(2, R.msg(M.NOP)))))
    if not corrupt:
        return (R.ids, out, R) if with_round else (R.ids, out)

    def bad_sig(sp):
        s = int.from_bytes(sp.s, "big")
        return M.SignedProto(sp.version, sp.message, sp.x, sp.y, sp.r, M.minimal(s ^ 1))

    stranger = R.rng.randrange(1, curve.n)
    E = M.encode_signed
    out += [
        ("x_outer_bad_sig", E(bad_sig(rc[3]))),
        ("x_outer_version0", E(R.signed(3, R.msg(M.ROUNDCHANGE, R.state), version=0))),
        ("x_outer_version2", E(R.signed(3, R.msg(M.ROUNDCHANGE, R.state), version=2))),
        ("x_outer_stranger", E(R.signed(None, R.msg(M.ROUNDCHANGE, R.state), d=stranger))),
        ("x_truncated", E(rc[4])[:-3]),
        ("x_garbage", bytes([0xFF] * 9)),
        ("x_empty", b""),
        ("x_msg_undecodable", E(M.sign(curve, R.keys[5], b"\x0a\xff", 12345))),
        ("x_unknown_type", E(R.signed(1, R.msg(9, R.state)))),
        ("x_lock_not_leader", E(R.signed((L + 1) % nval, R.msg(M.LOCK, R.state, rc[:q])))),
        ("x_lock_empty_state", E(R.signed(L, R.msg(M.LOCK, None, rc[:q])))),
        ("x_lock_proof_bad_sig", E(R.signed(L, R.msg(M.LOCK, R.state,
                                                      rc[:2] + [bad_sig(rc[2])] + rc[3:q])))),
        ("x_lock_proof_stranger", E(R.signed(L, R.msg(M.LOCK, R.state, rc[:q - 1] + [
            R.signed(None, R.msg(M.ROUNDCHANGE, R.state), d=stranger)])))),
        ("x_lock_proof_type", E(R.signed(L, R.msg(M.LOCK, R.state, rc[:q - 1] + [cm[q]])))),
        ("x_lock_proof_height", E(R.signed(L, R.msg(M.LOCK, R.state, rc[:q - 1] + [
            R.signed(q, R.msg(M.ROUNDCHANGE, R.state, h=R.h + 1))])))),
        ("x_lock_proof_round", E(R.signed(L, R.msg(M.LOCK, R.state, rc[:q - 1] + [
            R.signed(q, R.msg(M.ROUNDCHANGE, R.state, r=R.r + 1))])))),
        ("x_lock_proof_undecodable", E(R.signed(L, R.msg(M.LOCK, R.state, rc[:q - 1] + [
            M.sign(curve, R.keys[q], b"\x12\x05ab", 999)])))),
        ("x_lock_insufficient", E(R.signed(L, R.msg(M.LOCK, R.state, rc[:q - 1])))),
        ("x_lock_duplicate_signer", E(R.signed(L, R.msg(M.LOCK, R.state, rc[:q - 1] + [
            R.signed(0, R.msg(M.ROUNDCHANGE, R.state))])))),
        ("x_lock_other_state", E(R.signed(L, R.msg(M.LOCK, R.state, rc[:q - 1] + [
            R.signed(q, R.msg(M.ROUNDCHANGE, b"other"))])))),
        ("lock_extra_proofs", E(R.signed(L, R.msg(M.LOCK, R.state, rc)))),
        ("x_decide_proof_type", E(R.signed(L, R.msg(M.DECIDE, R.state, cm[:q - 1] + [rc[q]])))),
        ("x_decide_empty_state", E(R.signed(L, R.msg(M.DECIDE, None, cm[:q])))),
        ("x_decide_insufficient", E(R.signed(L, R.msg(M.DECIDE, R.state, cm[:q - 1])))),
        ("x_select_insufficient", E(R.signed(L, R.msg(M.SELECT, None, rc_nil[:q - 1])))),
        ("x_select_state_mismatch", E(R.signed(L, R.msg(M.SELECT, None, rc_nil[:q - 1] + [rc[q]])))),
        ("x_select_exceeded", E(R.signed(L, R.msg(M.SELECT, R.state, rc[:q])))),
        ("select_mixed", E(R.signed(L, R.msg(M.SELECT, R.state, rc_nil[:q - 1] + [rc[q]])))),
        ("x_lockrelease_empty", E(R.signed(1, R.msg(M.LOCKRELEASE, None)))),
        ("x_lockrelease_bad_lock", E(R.signed(1, R.msg(M.LOCKRELEASE, None, lr=bad_sig(lock))))),
        ("x_lockrelease_lock_insufficient", E(R.signed(1, R.msg(M.LOCKRELEASE, None, lr=R.signed(
            L, R.msg(M.LOCK, R.state, rc[:q - 1])))))),
        ("resync_with_bad_inner", E(R.signed(L, R.msg(M.RESYNC, None, [bad_sig(rc[1]), lock])))),
    ]
    # wire-format edge cases on a valid roundchange
    base = E(rc[6 % nval])
    out += [
        ("unknown_field_varint", base + b"\x38\x05"),            # field 7, varint: skipped
        ("unknown_field_bytes", base + b"\x42\x03abc"),          # field 8, bytes: skipped
        ("unknown_field_fixed64", base + b"\x49" + bytes(8)),    # field 9, fixed64
        ("unknown_group", base + b"\x53\x08\x01\x54"),           # field 10 group {1: 1}
        ("x_unknown_group_open", base + b"\x53\x08\x01"),        # unterminated group
        ("x_end_group", base + b"\x54"),                         # wiretype 4
        ("x_tag_zero", base + b"\x00\x00"),                      # illegal tag 0
        ("x_wrong_wiretype_version", b"\x0a\x00" + base),        # field 1 as bytes
        ("x_axis_33", base + b"\x1a\x21" + bytes(33)),           # X longer than 32 bytes
        ("axis_short_tail_copy", base + b"\x22\x01\x07"),        # Y: 1-byte tail copy
        ("x_varint_overflow", base + b"\x38" + b"\xff" * 10 + b"\x01"),
        ("version_wide_varint", b"\x08\x81\x80\x80\x80\x10" + base[2:]),  # 2^32 + 1 -> uint32 1
        ("x_len_negative", base + b"\x42" + b"\xff" * 9 + b"\x01"),
        ("repeated_r_last_wins", E(M.SignedProto(rc[0].version, rc[0].message, rc[0].x, rc[0].y,
                                                  b"\x01", rc[0].s)) + b"\x2a" +
         bytes([len(rc[0].r)]) + rc[0].r),
    ]
    return R.ids, out


def expected(curve, ids, msgs):
    res, rs = M.Preverifier(ids, curve).run([m for _, m in msgs])
    return res, rs


def main():
    cases = []
    for cname, curve, nval, seed in (("secp256k1", O.SECP256K1, 7, 41), ("P-256", O.P256, 7, 42)):
        ids, msgs = build_round(curve, nval, seed)
        res, rs = expected(curve, ids, msgs)
        cases.append({
            "curve": cname, "participants": [i.hex() for i in ids],
            "messages": [{"tag": t, "raw": m.hex(), "status": r.status, "bad_sp": r.bad_sp,
                          "type": r.type, "distinct_signers": r.distinct_signers,
                          "height": r.height, "round": r.round, "sp_first": r.sp_first,
                          "sp_count": r.sp_count} for (t, m), r in zip(msgs, res)],
            "sp_reason": rs,
        })
    with open(os.path.join(HERE, "bdls_messages.json"), "w") as f:
        json.dump(cases, f, indent=0)
    for c in cases:
        from collections import Counter
        print(c["curve"], len(c["messages"]), "messages", len(c["sp_reason"]), "SignedProtos",
              Counter(m["status"] for m in c["messages"]))


if __name__ == "__main__":
    main()
