"""Host-side mirror of the block-validation batch point
over bh_fabric_block_preverify (include/bdls_hip.h).

The reference validates a block transaction by transaction
(core/committer/txvalidator/v20/validator.go:180-265): per transaction one
creator identity.Verify (core/common/validation/msgvalidation.go:26-64) and,
inside the endorsement policy, one identity.Verify per de-duplicated endorser
(common/policies/policy.go:363-395). `block_preverify` runs all of those
signature checks for a whole serialized block as one device batch and returns
them per transaction: the verified-signature set the unchanged validator
consults.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib

FAB_STATUS = {0: "OK", 1: "ENVELOPE", 2: "PAYLOAD", 3: "HEADER", 4: "CREATOR_IDENTITY",
              5: "CREATOR_SIGNATURE", 6: "TX", 7: "UNSUPPORTED"}
E_DUPLICATE, E_BAD_IDENTITY, NOT_VERIFIED = 253, 254, 255


@dataclass
class TxResult:
    status: int
    type: int
    creator: int              # BH_R_* or NOT_VERIFIED
    endorse: list[int]        # per endorsement: BH_R_*, E_DUPLICATE, E_BAD_IDENTITY, NOT_VERIFIED
    valid_endorsers: int


def block_preverify(block: bytes, sha3: bool = False, keep_keys: bool = False,
                    decode_only: bool = False) -> list[TxResult]:
    """All signature checks of one serialized common.Block in one device batch.
    decode_only: host decode / identity resolution only (no device work)."""
    L = _lib.lib()
    if not decode_only:
        _lib.ensure_init()
    flags = ((_lib.BH_FAB_F_SHA3 if sha3 else 0) | (_lib.BH_FAB_F_KEEP_KEYS if keep_keys else 0)
             | (_lib.BH_FAB_F_DECODE_ONLY if decode_only else 0))
    buf = np.frombuffer(bytes(block) + b"\0", np.uint8)
    ntx, nend = ctypes.c_size_t(), ctypes.c_size_t()
    # sizing pass (decode only, no device work), then the real call
    rc = L.bh_fabric_block_preverify(buf.ctypes.data, len(block), flags | _lib.BH_FAB_F_DECODE_ONLY,
                                     None, 0, ctypes.byref(ntx), None, 0, ctypes.byref(nend))
    if rc != 0 and (ntx.value == 0 and nend.value == 0):
        _lib.check(rc)
    txs = (_lib.BhFabTx * max(1, ntx.value))()
    end = np.zeros(max(1, nend.value), np.uint8)
    _lib.check(L.bh_fabric_block_preverify(buf.ctypes.data, len(block), flags, txs, ntx.value,
                                           ctypes.byref(ntx), end.ctypes.data, nend.value,
                                           ctypes.byref(nend)))
    out = []
    for i in range(ntx.value):
        t = txs[i]
        out.append(TxResult(t.status, t.type, t.creator,
                            [int(x) for x in end[t.endorse_first:t.endorse_first + t.endorse_count]],
                            t.valid_endorsers))
    return out


@dataclass
class SigRef:
    """One signature of a block and its verified outcome: the key of the
    caller's verified-signature cache."""
    identity: bytes
    data: bytes       # the signed bytes (msg || msg2)
    signature: bytes
    reason: int       # BH_R_*, E_DUPLICATE, E_BAD_IDENTITY, NOT_VERIFIED


def block_preverify_refs(block: bytes, sha3: bool = False, keep_keys: bool = False,
                         decode_only: bool = False):
    """block_preverify plus, per signature, its (identity, signed bytes,
    signature) inside the block (bh_fabric_block_preverify_refs): the creator
    signatures (one per transaction, None when the transaction has no creator
    to check) and the endorsements, in endorse[] order."""
    L = _lib.lib()
    if not decode_only:
        _lib.ensure_init()
    flags = _flags(sha3, keep_keys, decode_only)
    buf = np.frombuffer(bytes(block) + b"\0", np.uint8)
    ntx, nend, nref = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
    rc = L.bh_fabric_block_preverify_refs(buf.ctypes.data, len(block),
                                          flags | _lib.BH_FAB_F_DECODE_ONLY, None, 0,
                                          ctypes.byref(ntx), None, 0, ctypes.byref(nend), None, 0,
                                          ctypes.byref(nref))
    if rc != 0 and nref.value == 0:
        _lib.check(rc)
    txs = (_lib.BhFabTx * max(1, ntx.value))()
    end = np.zeros(max(1, nend.value), np.uint8)
    refs = (_lib.BhFabSigref * max(1, nref.value))()
    _lib.check(L.bh_fabric_block_preverify_refs(
        buf.ctypes.data, len(block), flags, txs, ntx.value, ctypes.byref(ntx), end.ctypes.data,
        nend.value, ctypes.byref(nend), refs, nref.value, ctypes.byref(nref)))
    assert nref.value == ntx.value + nend.value
    out = []
    for i in range(ntx.value):
        t = txs[i]
        out.append(TxResult(t.status, t.type, t.creator,
                            [int(x) for x in end[t.endorse_first:t.endorse_first + t.endorse_count]],
                            t.valid_endorsers))

    def ref(r):
        if r.ident_len == 0:
            return None
        sp = lambda off, n: bytes(block[off:off + n])  # noqa: E731
        return SigRef(sp(r.ident_off, r.ident_len),
                      sp(r.msg_off, r.msg_len) + sp(r.msg2_off, r.msg2_len),
                      sp(r.sig_off, r.sig_len), int(r.reason))
    creators = [ref(refs[i]) for i in range(ntx.value)]
    endorsements = [ref(refs[ntx.value + j]) for j in range(nend.value)]
    return out, creators, endorsements


def _concat(items):
    ln = np.array([len(x) for x in items], np.uint32)
    off = np.zeros(len(items), np.uint64)
    if len(items):
        off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    buf = np.frombuffer(b"".join(items) + b"\0", np.uint8)
    return buf, off, ln


def _flags(sha3, keep_keys, decode_only):
    return ((_lib.BH_FAB_F_SHA3 if sha3 else 0) | (_lib.BH_FAB_F_KEEP_KEYS if keep_keys else 0)
            | (_lib.BH_FAB_F_DECODE_ONLY if decode_only else 0))


def signature_sets_verify(sets, sha3: bool = False, keep_keys: bool = False,
                          decode_only: bool = False):
    """common/policies/policy.go:363-395 SignatureSetToValidIdentities for many
    sets of (identity, data, signature) in one device batch. Returns
    [(per-entry results, valid identities)] per set."""
    L = _lib.lib()
    if not decode_only:
        _lib.ensure_init()
    flat = [sd for s in sets for sd in s]
    first = np.zeros(max(1, len(sets)), np.uint32)
    k = 0
    for i, s in enumerate(sets):
        first[i] = k
        k += len(s)
    ib, io, il = _concat([x[0] for x in flat])
    db, do, dl = _concat([x[1] for x in flat])
    sb, so, sl = _concat([x[2] for x in flat])
    b = _lib.BhSdBatch(ib.ctypes.data, io.ctypes.data, il.ctypes.data, db.ctypes.data,
                       do.ctypes.data, dl.ctypes.data, sb.ctypes.data, so.ctypes.data,
                       sl.ctypes.data)
    res = np.zeros(max(1, len(flat)), np.uint8)
    valid = np.zeros(max(1, len(sets)), np.uint32)
    _lib.check(L.bh_signature_sets_verify(ctypes.byref(b), len(flat), first.ctypes.data, len(sets),
                                          _flags(sha3, keep_keys, decode_only), res.ctypes.data,
                                          valid.ctypes.data))
    out, k = [], 0
    for i, s in enumerate(sets):
        out.append(([int(x) for x in res[k:k + len(s)]], int(valid[i])))
        k += len(s)
    return out


def envelopes_preverify(envs, sha3: bool = False, keep_keys: bool = False,
                        decode_only: bool = False):
    """SigFilter over n serialized envelopes: [(status, reason)]."""
    L = _lib.lib()
    if not decode_only:
        _lib.ensure_init()
    buf, off, ln = _concat(envs)
    n = len(envs)
    st = np.zeros(max(1, n), np.int32)
    rs = np.zeros(max(1, n), np.uint8)
    _lib.check(L.bh_envelopes_preverify(buf.ctypes.data, off.ctypes.data, ln.ctypes.data, n,
                                        _flags(sha3, keep_keys, decode_only), st.ctypes.data,
                                        rs.ctypes.data))
    return [(int(st[i]), int(rs[i])) for i in range(n)]


def block_signatures_preverify(blocks, sha3: bool = False, keep_keys: bool = False,
                               decode_only: bool = False, bft: bool = False, consenters=None):
    """Block signature sets of n serialized blocks: [(status, per-signature,
    valid identities)] (protoutil/blockutils.go:245-308 BlockSignatureVerifier).
    bft: bftEnabled; consenters: [(id, msp_id bytes, identity bytes)], the
    channel's cb.Consenter set searched by IdentifierHeader.identifier."""
    L = _lib.lib()
    if not decode_only:
        _lib.ensure_init()
    buf, off, ln = _concat(blocks)
    n = len(blocks)
    res = (_lib.BhBlocksigResult * max(1, n))()
    total = ctypes.c_size_t()
    cap = sum(len(b) for b in blocks) // 8 + 64
    sr = np.zeros(cap, np.uint8)
    flags = _flags(sha3, keep_keys, decode_only)
    if bft or consenters is not None:
        cons = list(consenters or [])
        ids = np.array([c[0] for c in cons] or [0], np.uint32)
        mb, mo, ml = _concat([c[1] for c in cons])
        ib, io, il = _concat([c[2] for c in cons])
        cs = _lib.BhConsenterSet(ids.ctypes.data, mb.ctypes.data, mo.ctypes.data, ml.ctypes.data,
                                 ib.ctypes.data, io.ctypes.data, il.ctypes.data, len(cons))
        _lib.check(L.bh_block_signatures_preverify_bft(
            buf.ctypes.data, off.ctypes.data, ln.ctypes.data, n,
            flags | (_lib.BH_BLK_F_BFT if bft else 0), ctypes.byref(cs), res, sr.ctypes.data,
            cap, ctypes.byref(total)))
    else:
        _lib.check(L.bh_block_signatures_preverify(buf.ctypes.data, off.ctypes.data,
                                                   ln.ctypes.data, n, flags, res, sr.ctypes.data,
                                                   cap, ctypes.byref(total)))
    return [(res[i].status, [int(x) for x in sr[res[i].sig_first:res[i].sig_first + res[i].sig_count]],
             res[i].valid_identities) for i in range(n)]


# ---------------------------------------------------------------- the Go consumer, mirrored
# The verified-signature cache and the cache-first PreverifySets of
# INTEGRATION.md sections 4 and 6 (common/sigcache, common/policies/
# preverify.go), restated so the tests can drive the exact consumer flow.
VALID, INVALID = 1, 2
# engine reasons whose identity.Verify outcome is parse-independent (cacheable)
CACHEABLE = {0: VALID, 7: INVALID, 8: INVALID, 9: INVALID}
# Below this many cache misses a policy evaluation does not call the device:
# the misses go to identity.Verify (the sw provider, or the coalescing single
# Verify). INTEGRATION.md 6 / HIPOpts.MinBatch.
PREVERIFY_MIN_BATCH = 16


class SigCache:
    """common/sigcache: (identity, signature) -> (signed bytes, outcome,
    generation). The key is length-prefixed, so no two (identity, signature)
    pairs collide; a lookup also compares the signed bytes exactly."""

    def __init__(self):
        self.m, self.gen = {}, 0

    @staticmethod
    def key(identity: bytes, sig: bytes) -> bytes:
        return len(identity).to_bytes(8, "big") + identity + sig

    def begin(self) -> int:
        self.gen += 1
        return self.gen

    def put(self, gen: int, identity: bytes, sig: bytes, data: bytes, out: int) -> None:
        self.m[self.key(identity, sig)] = (bytes(data), out, gen)

    def release(self, gen: int) -> None:
        self.m = {k: v for k, v in self.m.items() if v[2] != gen}

    def lookup(self, identity: bytes, data: bytes, sig: bytes):
        e = self.m.get(self.key(identity, sig))
        return e[1] if e is not None and e[0] == bytes(data) else None


def preverify_sets(cache: SigCache, sets, min_batch: int = PREVERIFY_MIN_BATCH,
                   sha3: bool = False, stats=None):
    """INTEGRATION.md 6 PreverifySets, cache first: every (identity, data,
    signature) of the sets is looked up; only the misses go to the device,
    each as its own one-signature set (no de-duplication: every miss gets its
    own outcome), and only when there are at least min_batch of them -- fewer
    stay with identity.Verify. Returns the release function of the entries
    it added. stats (dict) counts lookups / hits / device calls."""
    seen, misses = set(), []
    for s in sets:
        for ident, data, sig in s:
            k = (cache.key(ident, sig), bytes(data))
            if k in seen:
                continue
            seen.add(k)
            if stats is not None:
                stats["lookups"] = stats.get("lookups", 0) + 1
            if cache.lookup(ident, data, sig) is not None:
                if stats is not None:
                    stats["hits"] = stats.get("hits", 0) + 1
                continue
            misses.append((ident, data, sig))
    if len(misses) < max(1, min_batch):
        return lambda: None
    if stats is not None:
        stats["device_calls"] = stats.get("device_calls", 0) + 1
    res = signature_sets_verify([[sd] for sd in misses], sha3=sha3, keep_keys=True)
    gen = cache.begin()
    for (ident, data, sig), (r, _) in zip(misses, res):
        if r[0] in CACHEABLE:
            cache.put(gen, ident, sig, data, CACHEABLE[r[0]])
    return lambda: cache.release(gen)
