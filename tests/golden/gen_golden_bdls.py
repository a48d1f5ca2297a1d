#!/usr/bin/env python3
"""Golden fixtures for BDLS consensus-message verification.

Run from the repo root:  python tests/golden/gen_golden_bdls.py
Output (committed): tests/golden/bdls_vectors.jsonl

One record = one vendor/github.com/BDLS-bft/bdls/message.go SignedProto
(Version, X, Y, Message, R, S) and the expected SignedProto.Verify(curve)
(message.go:170-184) from oracle/ecdsa_ref.py:
  hash = BLAKE2b-256(prefix || version LE || X || Y || len LE || msg)   (:97-138)
  Verify = crypto/ecdsa.Verify(pub, hash, SetBytes(R), SetBytes(S))
secp256k1 (as wired, orderer/consensus/bdls/chain.go:60-61 -> Go verifyLegacy)
and P-256 (the curve-generic library with NIST keys -> verifyNISTEC). No low-S
rule on this path. Keys are valid curve points (BDLS admits only registered
participants, consensus.go:456-466). Signing follows SignedProto.Sign (:140-168)
with a seeded nonce.
"""
from __future__ import annotations

import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import ecdsa_ref as O  # noqa: E402

CURVES = {"secp256k1": O.SECP256K1, "P-256": O.P256}


def minimal(v: int) -> bytes:
    """big.Int.Bytes(): minimal big-endian, empty for 0."""
    return v.to_bytes((v.bit_length() + 7) // 8, "big")


def rec(tag, cname, version, x32, y32, msg, rb, sb):
    c = CURVES[cname]
    digest = O.bdls_signed_proto_hash(version, x32, y32, msg)
    r, s = int.from_bytes(rb, "big"), int.from_bytes(sb, "big")
    reason = O.go_ecdsa_verify(c, int.from_bytes(x32, "big"), int.from_bytes(y32, "big"),
                               digest, r, s)
    return {"tag": tag, "curve": cname, "version": version, "x": x32.hex(), "y": y32.hex(),
            "msg": msg.hex(), "r": rb.hex(), "s": sb.hex(), "digest": digest.hex(),
            "valid": reason == O.R_OK, "reason": reason}


def sign(c, d, version, x32, y32, msg, k):
    """SignedProto.Sign: ecdsa.Sign over Hash() (legacy/NIST e = left-most 32 B)."""
    digest = O.bdls_signed_proto_hash(version, x32, y32, msg)
    e = int.from_bytes(digest, "big") % c.n
    R = O.scalar_mult(c, k, (c.gx, c.gy))
    r = R[0] % c.n
    s = pow(k, -1, c.n) * (e + r * d) % c.n
    return r, s


def main():
    rng = random.Random(20230426)
    out = []
    for cname, c in CURVES.items():
        keys = []
        for _ in range(4):
            d = rng.randrange(1, c.n)
            x, y = O.pubkey(c, d)
            keys.append((d, x.to_bytes(32, "big"), y.to_bytes(32, "big")))
        # message lengths around BLAKE2b block edges (header is 96 bytes)
        for j, L in enumerate([0, 1, 31, 32, 33, 100, 159, 160, 161, 287, 288, 289, 1000, 13000]):
            d, x, y = keys[j % len(keys)]
            msg = bytes(rng.getrandbits(8) for _ in range(L))
            r, s = sign(c, d, 1, x, y, msg, rng.randrange(1, c.n))
            out.append(rec(f"valid_len{L}", cname, 1, x, y, msg, minimal(r), minimal(s)))
        for j in range(12):
            d, x, y = keys[j % len(keys)]
            msg = bytes(rng.getrandbits(8) for _ in range(80 + 7 * j))
            r, s = sign(c, d, 1, x, y, msg, rng.randrange(1, c.n))
            R, S = minimal(r), minimal(s)
            out.append(rec("valid", cname, 1, x, y, msg, R, S))
            bad = bytearray(msg)
            bad[j % len(bad)] ^= 0x10
            out.append(rec("msg_flip", cname, 1, x, y, bytes(bad), R, S))
            out.append(rec("high_s_accepted", cname, 1, x, y, msg, R, minimal(c.n - s)))
            out.append(rec("r_leading_zeros", cname, 1, x, y, msg, b"\x00\x00" + R, S))
            out.append(rec("s_leading_zeros", cname, 1, x, y, msg, R, b"\x00" * 5 + S))
            out.append(rec("r_plus1", cname, 1, x, y, msg, minimal(r + 1), S))
            out.append(rec("version2_mismatch", cname, 2, x, y, msg, R, S))
            d2, x2, y2 = keys[(j + 1) % len(keys)]
            out.append(rec("other_participant_key", cname, 1, x2, y2, msg, R, S))
        d, x, y = keys[0]
        msg = b"commit:" + bytes(range(40))
        r, s = sign(c, d, 2, x, y, msg, rng.randrange(1, c.n))
        out.append(rec("version2_signed", cname, 2, x, y, msg, minimal(r), minimal(s)))
        r, s = sign(c, d, 1, x, y, msg, rng.randrange(1, c.n))
        R, S = minimal(r), minimal(s)
        for tag, rb, sb in [("r_empty", b"", S), ("s_empty", R, b""), ("r_zero_bytes", b"\x00" * 32, S),
                            ("r_eq_n", minimal(c.n), S), ("s_eq_n", R, minimal(c.n)),
                            ("r_33B_big", b"\x01" + R.rjust(32, b"\x00"), S),
                            ("s_40B_big", R, b"\x07" * 40), ("r_n_plus_r", minimal(c.n + r), S),
                            ("r1_s1", b"\x01", b"\x01")]:
            out.append(rec(tag, cname, 1, x, y, msg, rb, sb))
    with open(os.path.join(HERE, "bdls_vectors.jsonl"), "w") as f:
        for o in out:
            f.write(json.dumps(o, sort_keys=True) + "\n")
    from collections import Counter
    print(len(out), "records;", dict(Counter((o["curve"], O.REASON_NAMES[o["reason"]]) for o in out)))


if __name__ == "__main__":
    main()
