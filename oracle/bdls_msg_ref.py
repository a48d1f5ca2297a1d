"""TEST INFRASTRUCTURE (oracle) -- pure-Python restatement of the BDLS
consensus-message checks that bh_bdls_preverify batches (SURVEY.md 8(a) rows
A15-A16). Only tests/ may import this; it is the checker, never the product.

Follows, in /root/reference/vendor/github.com/BDLS-bft/bdls/:
  message.pb.go  SignedProto.Unmarshal :516-755, Message.Unmarshal :757-970,
                 skipMessage :972-1049, MarshalToSizedBuffer :300-356 (encoder)
  message.go     PubKeyAxis.Unmarshal :45-55, SignedProto.Verify :170-184
  consensus.go   receiveMessage :1209-1226, verifyMessage :449-493,
                 verifyLockMessage :520-600, verifyLockReleaseMessage :604-623,
                 verifySelectMessage :628-728, verifyDecideMessage :829-902,
                 roundLeader :1148-1154, t() :1173, numIdentities :362-367,
                 Resync loopback :1483-1492 (errors ignored, :1197-1204)
Checks needing consensus state or callbacks (height/round vs the current
round, StateValidate, StateCompare, MessageValidator, lock-release stage) are
not evaluated -- the same contract as include/bdls_hip.h. Quorums use the
default StateHash (blake2b-256, consensus.go:41): equal hash <=> equal bytes,
nil == empty.

Parity: the Go code cannot run here (no Go toolchain); this restatement and
the C++ one (bdls_amd/csrc/bdls_msg.cpp) are independent implementations of
the same reference lines, checked against each other on generated rounds and
on wire-format edge cases (tests/test_bdls_msg.py).
"""
from __future__ import annotations

from dataclasses import dataclass, field

from oracle import ecdsa_ref as O

OK, DECODE, VERSION, UNKNOWN_PARTICIPANT, BAD_SIGNATURE, MSG_DECODE, UNKNOWN_TYPE, \
    EMPTY_STATE, NOT_LEADER, PROOF_UNKNOWN_PARTICIPANT, PROOF_BAD_SIGNATURE, PROOF_DECODE, \
    PROOF_TYPE_MISMATCH, PROOF_HEIGHT_MISMATCH, PROOF_ROUND_MISMATCH, PROOF_INSUFFICIENT, \
    SELECT_STATE_MISMATCH, SELECT_PROOF_EXCEEDED, LOCKRELEASE_EMPTY = range(19)
NOT_VERIFIED = 255

NOP, ROUNDCHANGE, LOCK, SELECT, COMMIT, LOCKRELEASE, DECIDE, RESYNC = range(8)
MAX_RESYNC_DEPTH = 8


class DecodeError(Exception):
    pass


@dataclass
class SignedProto:
    version: int = 0
    message: bytes = b""
    x: bytes = bytes(32)
    y: bytes = bytes(32)
    r: bytes = b""
    s: bytes = b""


@dataclass
class Message:
    type: int = 0
    height: int = 0
    round: int = 0
    state: bytes | None = None
    proofs: list = field(default_factory=list)
    lock_release: SignedProto | None = None


# ---------------------------------------------------------------- encoding
def _uvarint(v: int) -> bytes:
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _lenf(tag: int, b: bytes) -> bytes:
    return bytes([tag]) + _uvarint(len(b)) + b


def encode_signed(sp: SignedProto) -> bytes:
    """SignedProto.MarshalToSizedBuffer (:300-356): fields 1..6 in order."""
    out = b""
    if sp.version:
        out += b"\x08" + _uvarint(sp.version)
    if sp.message:
        out += _lenf(0x12, sp.message)
    out += _lenf(0x1A, sp.x) + _lenf(0x22, sp.y)
    if sp.r:
        out += _lenf(0x2A, sp.r)
    if sp.s:
        out += _lenf(0x32, sp.s)
    return out


def encode_message(m: Message) -> bytes:
    out = b""
    if m.type:
        out += b"\x08" + _uvarint(m.type & 0xFFFFFFFFFFFFFFFF)
    if m.height:
        out += b"\x10" + _uvarint(m.height)
    if m.round:
        out += b"\x18" + _uvarint(m.round)
    if m.state:
        out += _lenf(0x22, m.state)
    for p in m.proofs:
        out += _lenf(0x2A, encode_signed(p))
    if m.lock_release is not None:
        out += _lenf(0x32, encode_signed(m.lock_release))
    return out


def minimal(v: int) -> bytes:
    return v.to_bytes((v.bit_length() + 7) // 8, "big")


def sign(c: O.Curve, d: int, msg: bytes, k: int, version: int = 1) -> SignedProto:
    """SignedProto.Sign (message.go:140-168) with a caller-chosen nonce."""
    qx, qy = O.pubkey(c, d)
    sp = SignedProto(version=version, message=msg, x=qx.to_bytes(32, "big"),
                     y=qy.to_bytes(32, "big"))
    h = O.bdls_signed_proto_hash(version, sp.x, sp.y, msg)
    e = int.from_bytes(h, "big") % c.n
    r = O.scalar_mult(c, k, (c.gx, c.gy))[0] % c.n
    s = pow(k, -1, c.n) * (e + r * d) % c.n
    sp.r, sp.s = minimal(r), minimal(s)
    return sp


# ---------------------------------------------------------------- decoding
def _varint(d: bytes, i: int):
    v = 0
    shift = 0
    while True:
        if shift >= 64:
            raise DecodeError("proto: integer overflow")
        if i >= len(d):
            raise DecodeError("unexpected EOF")
        b = d[i]
        i += 1
        v |= (b & 0x7F) << shift
        if b < 0x80:
            return v & 0xFFFFFFFFFFFFFFFF, i
        shift += 7


def _bytes(d: bytes, i: int):
    v, i = _varint(d, i)
    if v >= 1 << 63:  # Go int negative
        raise DecodeError("negative length")
    if i + v > len(d):
        raise DecodeError("unexpected EOF")
    return d[i:i + v], i + v


def _skip(d: bytes) -> int:
    """skipMessage (:972-1049)."""
    i, depth = 0, 0
    while i < len(d):
        wire, i = _varint(d, i)
        wt = wire & 7
        if wt == 0:
            _, i = _varint(d, i)
        elif wt == 1:
            i += 8
        elif wt == 2:
            ln, i = _varint(d, i)
            if ln >= 1 << 63:
                raise DecodeError("negative length")
            i += ln
        elif wt == 3:
            depth += 1
        elif wt == 4:
            if depth == 0:
                raise DecodeError("unexpected end of group")
            depth -= 1
        elif wt == 5:
            i += 4
        else:
            raise DecodeError("illegal wireType")
        if depth == 0:
            return i
    raise DecodeError("unexpected EOF")


def _tag(d: bytes, i: int):
    wire, i = _varint(d, i)
    fn = wire >> 3 & 0xFFFFFFFF
    if fn >= 1 << 31:
        fn -= 1 << 32  # int32(wire >> 3)
    wt = wire & 7
    if wt == 4:
        raise DecodeError("wiretype end group for non-group")
    if fn <= 0:
        raise DecodeError("illegal tag")
    return fn, wt, i


def _default(d: bytes, pre: int) -> int:
    sk = _skip(d[pre:])
    if pre + sk > len(d):
        raise DecodeError("unexpected EOF")
    return pre + sk


def decode_signed(d: bytes, into: SignedProto | None = None) -> SignedProto:
    m = into if into is not None else SignedProto()
    i = 0
    while i < len(d):
        pre = i
        fn, wt, i = _tag(d, i)
        want = 0 if fn == 1 else 2
        if 1 <= fn <= 6 and wt != want:
            raise DecodeError(f"wrong wireType = {wt}")
        if fn == 1:
            v, i = _varint(d, i)
            m.version = v & 0xFFFFFFFF
        elif fn == 2:
            m.message, i = _bytes(d, i)
        elif fn in (3, 4):
            b, i = _bytes(d, i)
            if len(b) > 32:
                raise DecodeError("incorrect pubkey format")
            cur = bytearray(m.x if fn == 3 else m.y)
            cur[32 - len(b):] = b  # tail copy, head kept (PubKeyAxis.Unmarshal)
            if fn == 3:
                m.x = bytes(cur)
            else:
                m.y = bytes(cur)
        elif fn == 5:
            m.r, i = _bytes(d, i)
        elif fn == 6:
            m.s, i = _bytes(d, i)
        else:
            i = _default(d, pre)
    return m


def decode_message(d: bytes) -> Message:
    m = Message()
    i = 0
    while i < len(d):
        pre = i
        fn, wt, i = _tag(d, i)
        want = 0 if fn in (1, 2, 3) else 2
        if 1 <= fn <= 6 and wt != want:
            raise DecodeError(f"wrong wireType = {wt}")
        if fn == 1:
            v, i = _varint(d, i)
            v &= 0xFFFFFFFF
            m.type = v - (1 << 32) if v >= 1 << 31 else v
        elif fn == 2:
            m.height, i = _varint(d, i)
        elif fn == 3:
            m.round, i = _varint(d, i)
        elif fn == 4:
            m.state, i = _bytes(d, i)
        elif fn == 5:
            b, i = _bytes(d, i)
            m.proofs.append(decode_signed(b))
        elif fn == 6:
            b, i = _bytes(d, i)
            if m.lock_release is None:
                m.lock_release = SignedProto()
            decode_signed(b, m.lock_release)
        else:
            i = _default(d, pre)
    return m


# ---------------------------------------------------------------- checks
def ident(sp: SignedProto) -> bytes:
    return bytes(sp.x) + bytes(sp.y)


@dataclass
class _Node:
    sp: SignedProto
    idx: int
    gate: bool
    msg: Message | None


@dataclass
class Result:
    status: int
    bad_sp: int
    type: int
    distinct_signers: int
    height: int
    round: int
    sp_first: int
    sp_count: int


class Preverifier:
    """Flatten + evaluate; `reasons` for the flattened SignedProtos either
    given or computed with oracle/ecdsa_ref.py's SignedProto.Verify."""

    def __init__(self, participants: list[bytes], curve: O.Curve, quorum: bool = True):
        self.plist = list(participants)
        self.parts = set(self.plist)
        self.n_ident = len(self.parts)
        self.curve = curve
        self.quorum = quorum
        self.flat: list[SignedProto] = []
        self.verify: list[bool] = []

    def _node(self, sp: SignedProto, verify_it: bool) -> _Node:
        nd = _Node(sp, len(self.flat), ident(sp) in self.parts, None)
        self.flat.append(sp)
        self.verify.append(verify_it and nd.gate)
        try:
            nd.msg = decode_message(sp.message)
        except DecodeError:
            nd.msg = None
        return nd

    def _plan(self, sp: SignedProto, depth: int) -> dict:
        vok = sp.version == O.BDLS_PROTOCOL_VERSION
        p = {"outer": self._node(sp, vok), "proofs": [], "lr": None, "lr_proofs": []}
        o = p["outer"]
        if not vok or not o.gate or o.msg is None:
            return p
        m = o.msg
        if m.type in (LOCK, SELECT, DECIDE):
            p["proofs"] = [self._node(q, True) for q in m.proofs]
        elif m.type == LOCKRELEASE and m.lock_release is not None:
            p["lr"] = lr = self._node(m.lock_release, True)
            if lr.gate and lr.msg is not None:
                p["lr_proofs"] = [self._node(q, True) for q in lr.msg.proofs]
        elif m.type == RESYNC and depth < MAX_RESYNC_DEPTH:
            for q in m.proofs:
                self._plan(q, depth + 1)
        return p

    def _leader(self, rnd: int, sp: SignedProto) -> bool:
        if not self.plist or rnd >= 1 << 63:
            return False
        return self.plist[rnd % len(self.plist)] == ident(sp)

    def _proof_sig(self, nd, rs, base):
        if not nd.gate:
            return PROOF_UNKNOWN_PARTICIPANT, nd.idx - base
        if rs[nd.idx] != O.R_OK:
            return PROOF_BAD_SIGNATURE, nd.idx - base
        if nd.msg is None:
            return PROOF_DECODE, nd.idx - base
        return None

    def _check_proofs(self, m: Message, signer: _Node, proofs, kind, rs, base):
        """-> (status, bad, distinct)"""
        if kind in (LOCK, DECIDE) and m.state is None:
            return EMPTY_STATE, -1, 0
        if not self._leader(m.round, signer.sp):
            return NOT_LEADER, -1, 0
        want = COMMIT if kind == DECIDE else ROUNDCHANGE
        signers: dict[bytes, bytes | None] = {}
        for pf in proofs:
            e = self._proof_sig(pf, rs, base)
            if e:
                return e[0], e[1], 0
            rel = pf.idx - base
            if pf.msg.type != want:
                return PROOF_TYPE_MISMATCH, rel, 0
            if pf.msg.height != m.height:
                return PROOF_HEIGHT_MISMATCH, rel, 0
            if pf.msg.round != m.round:
                return PROOF_ROUND_MISMATCH, rel, 0
            signers[ident(pf.sp)] = pf.msg.state
        distinct = len(signers)
        if not self.quorum:
            return OK, -1, distinct
        need = 2 * ((self.n_ident - 1) // 3) + 1
        if kind == SELECT:
            if len(signers) < need:
                return PROOF_INSUFFICIENT, -1, distinct
            props: dict[bytes, int] = {}
            for st in signers.values():
                if st is not None:
                    props[st] = props.get(st, 0) + 1
            if m.state is None and props:
                return SELECT_STATE_MISMATCH, -1, distinct
            if props and max(props.values()) >= need:
                return SELECT_PROOF_EXCEEDED, -1, distinct
            return OK, -1, distinct
        cnt = sum(1 for st in signers.values() if (st or b"") == (m.state or b""))
        return (PROOF_INSUFFICIENT if cnt < need else OK), -1, distinct

    def _evaluate(self, p, rs, base):
        o = p["outer"]
        if o.sp.version != O.BDLS_PROTOCOL_VERSION:
            return VERSION, 0, 0
        if not o.gate:
            return UNKNOWN_PARTICIPANT, 0, 0
        if rs[o.idx] != O.R_OK:
            return BAD_SIGNATURE, 0, 0
        if o.msg is None:
            return MSG_DECODE, 0, 0
        m = o.msg
        if m.type in (NOP, ROUNDCHANGE, COMMIT, RESYNC):
            return OK, -1, 0
        if m.type in (LOCK, SELECT, DECIDE):
            return self._check_proofs(m, o, p["proofs"], m.type, rs, base)
        if m.type == LOCKRELEASE:
            if p["lr"] is None:
                return LOCKRELEASE_EMPTY, -1, 0
            e = self._proof_sig(p["lr"], rs, base)
            if e:
                return e[0], e[1], 0
            return self._check_proofs(p["lr"].msg, p["lr"], p["lr_proofs"], LOCK, rs, base)
        return UNKNOWN_TYPE, -1, 0

    def run(self, raw_msgs: list[bytes], reasons: list[int] | None = None):
        plans, spans = [], []
        for raw in raw_msgs:
            first = len(self.flat)
            try:
                sp = decode_signed(raw)
            except DecodeError:
                sp = None
            plans.append(self._plan(sp, 0) if sp is not None else None)
            spans.append((first, len(self.flat) - first))
        if reasons is None:
            rs = []
            for sp, v in zip(self.flat, self.verify):
                if v:
                    # SignedProto.Verify (message.go:170-184), reason-coded
                    dg = O.bdls_signed_proto_hash(sp.version, sp.x, sp.y, sp.message)
                    rs.append(O.go_ecdsa_verify(
                        self.curve, int.from_bytes(sp.x, "big"), int.from_bytes(sp.y, "big"),
                        dg, int.from_bytes(sp.r, "big"), int.from_bytes(sp.s, "big")))
                else:
                    rs.append(NOT_VERIFIED)
        else:
            rs = [r if v else NOT_VERIFIED for r, v in zip(reasons, self.verify)]
        out = []
        for p, (first, cnt) in zip(plans, spans):
            if p is None:
                out.append(Result(DECODE, -1, 0, 0, 0, 0, first, cnt))
                continue
            st, bad, dist = self._evaluate(p, rs, first)
            m = p["outer"].msg
            out.append(Result(st, bad, m.type if m else 0, dist, m.height if m else 0,
                              m.round if m else 0, first, cnt))
        return out, rs
