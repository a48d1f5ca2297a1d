"""Synthetic verify workloads (BASELINE.json configs 2 and 5) from
bdls_amd/workload/gen.c (libbdlsgen.so). Data preparation only."""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

_LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib",
                    "libbdlsgen.so")
SIG_STRIDE = 80
CLASS_NAMES = ["none", "msg_flip", "high_s", "r_zero", "r_ge_n", "s_ge_n", "q_offcurve",
               "q_ge_p", "der_trailing_ok", "der_extra_ok", "der_nonminimal", "der_longlen"]


@dataclass
class Workload:
    pub: np.ndarray      # n*64 u8
    msg: np.ndarray      # n*msg_len u8
    msg_off: np.ndarray  # u64
    msg_len: np.ndarray  # u32
    sig: np.ndarray      # n*80 u8
    sig_off: np.ndarray  # u64
    sig_len: np.ndarray  # u32
    reason: np.ndarray   # expected reason u8 (by construction)
    cls: np.ndarray      # corruption class u8

    @property
    def n(self) -> int:
        return len(self.msg_len)

    @property
    def expected_valid(self) -> np.ndarray:
        return self.reason == 0

    def arrays(self):
        return (self.pub, self.sig, self.sig_off, self.sig_len, self.msg, self.msg_off,
                self.msg_len)


def _empty(alloc, count: int, dtype):
    """numpy array of `count` items, from alloc(nbytes) -> uint8 array if given
    (e.g. page-locked memory for the pipelined host path)."""
    if alloc is None:
        return np.empty(count, dtype)
    return alloc(count * np.dtype(dtype).itemsize).view(dtype)


def generate_shard(n_total: int, lo: int, count: int, nkeys: int, msg_len: int = 256,
                   corrupt_den: int = 16, seed: int = 2, nthreads: int | None = None,
                   family: str = "SHA2", alloc=None) -> Workload:
    """Records [lo, lo + count) of ONE seeded batch of n_total records: every
    record is a function of (seed, global index), so the shards of any split
    concatenate to the same batch (config 5: one 64M batch over N ranks).
    nkeys >= n_total: one distinct key per record. Records are signed over
    Hash(msg) with the MSP hash family (SHA2: SHA-256, SHA3: SHA3-256;
    msp/identities.go:219-227)."""
    if not os.path.exists(_LIB):
        raise RuntimeError(f"{_LIB} not built (run `make`)")
    L = ctypes.CDLL(_LIB)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    L.gen_p256_shard.argtypes = [sz, sz, sz, sz, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                 ctypes.c_int, ctypes.c_int] + [vp] * 9
    L.gen_p256_shard.restype = ctypes.c_int
    fam = {"SHA2": 0, "SHA3": 1}[family]
    if nthreads is None:
        nthreads = min(16, os.cpu_count() or 1)
    n = count
    w = Workload(
        pub=_empty(alloc, n * 64, np.uint8), msg=_empty(alloc, n * msg_len, np.uint8),
        msg_off=_empty(alloc, n, np.uint64), msg_len=_empty(alloc, n, np.uint32),
        sig=_empty(alloc, n * SIG_STRIDE, np.uint8), sig_off=_empty(alloc, n, np.uint64),
        sig_len=_empty(alloc, n, np.uint32), reason=np.empty(n, np.uint8), cls=np.empty(n, np.uint8))
    w.sig[:] = 0
    rc = L.gen_p256_shard(n_total, lo, count, nkeys, msg_len, corrupt_den, seed, nthreads, fam,
                          w.pub.ctypes.data, w.msg.ctypes.data, w.msg_off.ctypes.data,
                          w.msg_len.ctypes.data, w.sig.ctypes.data, w.sig_off.ctypes.data,
                          w.sig_len.ctypes.data, w.reason.ctypes.data, w.cls.ctypes.data)
    if rc != 0:
        raise RuntimeError(f"gen_p256_shard failed: {rc}")
    return w


_FIELDS = (("pub", np.uint8, 64), ("msg", np.uint8, None), ("msg_off", np.uint64, 1),
           ("msg_len", np.uint32, 1), ("sig", np.uint8, SIG_STRIDE), ("sig_off", np.uint64, 1),
           ("sig_len", np.uint32, 1), ("reason", np.uint8, 1), ("cls", np.uint8, 1))


def _alloc_workload(n: int, msg_len: int, alloc) -> Workload:
    return Workload(
        pub=_empty(alloc, n * 64, np.uint8), msg=_empty(alloc, n * msg_len, np.uint8),
        msg_off=_empty(alloc, n, np.uint64), msg_len=_empty(alloc, n, np.uint32),
        sig=_empty(alloc, n * SIG_STRIDE, np.uint8), sig_off=_empty(alloc, n, np.uint64),
        sig_len=_empty(alloc, n, np.uint32), reason=np.empty(n, np.uint8),
        cls=np.empty(n, np.uint8))


def _gen_fingerprint() -> str:
    """First 12 hex digits of the generator library's sha256 (a
    rebuilt generator never reads a cache another build wrote)."""
    import hashlib
    if not os.path.exists(_LIB):
        return "nolib"
    h = hashlib.sha256()
    with open(_LIB, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()[:12]


def cache_key(n_total, lo, count, nkeys, msg_len, corrupt_den, seed, family="SHA2") -> str:
    return (f"p256_{family}_t{n_total}_lo{lo}_c{count}_k{nkeys}_m{msg_len}_d{corrupt_den}"
            f"_s{seed}_g{_gen_fingerprint()}_v2")


def generate_shard_cached(n_total: int, lo: int, count: int, nkeys: int, msg_len: int = 256,
                          corrupt_den: int = 16, seed: int = 2, nthreads: int | None = None,
                          alloc=None, cache_dir: str | None = None, save: bool = True,
                          chunk: int = 1 << 20, log=None) -> tuple[Workload, dict]:
    """generate_shard for big unique-key shards (config 5: SURVEY 8(d) row 5,
    "generated once ... and cached on local disk"):
      * the arrays are allocated ONCE (e.g. page-locked through `alloc`) and
        filled in place -- from the cache directory when a complete copy of
        this exact shard is there, else by the generator in chunks of `chunk`
        records (record i is a function of (seed, i), so chunks concatenate to
        the same shard), calling log(msg) after each chunk so a long run
        reports progress;
      * a freshly generated shard is written to cache_dir/<key>/ (one raw file
        per array + meta.json last, so a partial write is never taken for a
        copy) when `save` and the file system has room for it.
    Returns (workload, info) -- info says where the records came from."""
    log = log or (lambda m: None)
    w = _alloc_workload(count, msg_len, alloc)
    info = {"source": "generator", "cache_dir": cache_dir}
    key = cache_key(n_total, lo, count, nkeys, msg_len, corrupt_den, seed)
    path = os.path.join(cache_dir, key) if cache_dir else None
    meta_path = os.path.join(path, "meta.json") if path else None
    t0 = __import__("time").time()
    if meta_path and os.path.exists(meta_path):
        import json
        with open(meta_path) as f:
            meta = json.load(f)
        sizes = meta.get("sizes") or {}
        ok = meta.get("key") == key and all(
            sizes.get(name) == getattr(w, name).nbytes
            and os.path.getsize(os.path.join(path, name + ".bin")) == getattr(w, name).nbytes
            for name, _, _ in _FIELDS if os.path.exists(os.path.join(path, name + ".bin")))
        ok = ok and all(os.path.exists(os.path.join(path, name + ".bin")) for name, _, _ in _FIELDS)
        if not ok:
            log(f"cache: {path} does not match this shard / generator, regenerating")
        if ok:
            for name, _, _ in _FIELDS:
                a = getattr(w, name)
                mv = memoryview(a.view(np.uint8).reshape(-1))
                with open(os.path.join(path, name + ".bin"), "rb", buffering=0) as f:
                    got, step = 0, 1 << 28
                    while got < len(mv):
                        k = f.readinto(mv[got:got + step])
                        if not k:
                            raise RuntimeError(f"cache file {name}.bin is short")
                        got += k
                log(f"cache: loaded {name} ({len(mv) / 1e9:.2f} GB)")
            info.update(source="cache", path=path, load_s=round(__import__("time").time() - t0, 2))
            return w, info
    if not os.path.exists(_LIB):
        raise RuntimeError(f"{_LIB} not built (run `make`)")
    L = ctypes.CDLL(_LIB)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    L.gen_p256_shard.argtypes = [sz, sz, sz, sz, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                 ctypes.c_int, ctypes.c_int] + [vp] * 9
    L.gen_p256_shard.restype = ctypes.c_int
    if nthreads is None:
        nthreads = min(16, os.cpu_count() or 1)
    # shared keys are derived once per call: chunk only unique-key shards
    step = chunk if nkeys >= n_total else count
    w.sig[:] = 0
    for b in range(0, count, step):
        m = min(step, count - b)
        rc = L.gen_p256_shard(n_total, lo + b, m, nkeys, msg_len, corrupt_den, seed, nthreads, 0,
                              w.pub[64 * b:].ctypes.data, w.msg[msg_len * b:].ctypes.data,
                              w.msg_off[b:].ctypes.data, w.msg_len[b:].ctypes.data,
                              w.sig[SIG_STRIDE * b:].ctypes.data, w.sig_off[b:].ctypes.data,
                              w.sig_len[b:].ctypes.data, w.reason[b:].ctypes.data,
                              w.cls[b:].ctypes.data)
        if rc != 0:
            raise RuntimeError(f"gen_p256_shard failed: {rc}")
        if b:  # the generator's offsets are local to its call
            w.msg_off[b:b + m] += np.uint64(msg_len * b)
            w.sig_off[b:b + m] += np.uint64(SIG_STRIDE * b)
        if step < count:
            log(f"generated {b + m}/{count} records ({nthreads} threads)")
    info["gen_s"] = round(__import__("time").time() - t0, 2)
    if path and save:
        import json
        import shutil
        need = sum(getattr(w, name).nbytes for name, _, _ in _FIELDS)
        os.makedirs(cache_dir, exist_ok=True)
        free = shutil.disk_usage(cache_dir).free
        if free < need * 1.1 + (1 << 30):
            info["cache_skipped"] = f"{free / 1e9:.1f} GB free < {need / 1e9:.1f} GB needed"
            log(f"cache: not written ({info['cache_skipped']})")
            return w, info
        t1 = __import__("time").time()
        os.makedirs(path, exist_ok=True)
        if os.path.exists(meta_path):
            os.unlink(meta_path)
        for name, _, _ in _FIELDS:
            getattr(w, name).tofile(os.path.join(path, name + ".bin"))
            log(f"cache: wrote {name}")
        with open(meta_path + ".tmp", "w") as f:
            json.dump({"key": key, "bytes": need,
                       "sizes": {name: getattr(w, name).nbytes for name, _, _ in _FIELDS}}, f)
        os.replace(meta_path + ".tmp", meta_path)
        info.update(saved=path, save_s=round(__import__("time").time() - t1, 2))
    return w, info


def generate(n: int, nkeys: int, msg_len: int = 256, corrupt_den: int = 16, seed: int = 2,
             nthreads: int | None = None, family: str = "SHA2", alloc=None) -> Workload:
    """A whole batch of n records (see generate_shard)."""
    return generate_shard(n, 0, n, nkeys, msg_len, corrupt_den, seed, nthreads, family, alloc)


@dataclass
class BdlsRound:
    """One BDLS height/round of SignedProto records (BASELINE config 4)."""
    curve: int           # 0 P-256, 1 secp256k1 (bh_curve)
    xy: np.ndarray       # n*64 u8
    r: np.ndarray
    r_off: np.ndarray
    r_len: np.ndarray
    s: np.ndarray
    s_off: np.ndarray
    s_len: np.ndarray
    version: np.ndarray  # u32
    msg: np.ndarray
    msg_off: np.ndarray
    msg_len: np.ndarray

    @property
    def n(self) -> int:
        return len(self.version)

    def arrays(self):
        return (self.xy, self.r, self.r_off, self.r_len, self.s, self.s_off, self.s_len,
                self.version, self.msg, self.msg_off, self.msg_len)


def generate_bdls_round(nval: int = 100, curve: int = 1, small_len: int = 200,
                        seed: int = 4) -> BdlsRound:
    """nval roundchange + lock (+2t+1 proofs) + nval commit + decide (+2t+1
    proofs), t = (nval-1)//3, all valid, signed by the validators' keys."""
    if not os.path.exists(_LIB):
        raise RuntimeError(f"{_LIB} not built (run `make`)")
    L = ctypes.CDLL(_LIB)
    vp = ctypes.c_void_p
    L.gen_bdls_round.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_uint64, ctypes.c_int] + [vp] * 9 + [
                                     ctypes.c_uint64, vp, vp]
    L.gen_bdls_round.restype = ctypes.c_int
    t = (nval - 1) // 3
    t2p1 = 2 * t + 1
    cap = 2 * nval + 2 * (1 + t2p1)
    msg_cap = 2 * nval * small_len + 2 * t2p1 * (small_len + 200) * 2 + 64
    b = BdlsRound(curve=curve, xy=np.zeros(cap * 64, np.uint8), r=np.zeros(cap * 33, np.uint8),
                  r_off=np.zeros(cap, np.uint64), r_len=np.zeros(cap, np.uint32),
                  s=np.zeros(cap * 33, np.uint8), s_off=np.zeros(cap, np.uint64),
                  s_len=np.zeros(cap, np.uint32), version=np.zeros(cap, np.uint32),
                  msg=np.zeros(msg_cap, np.uint8), msg_off=np.zeros(cap, np.uint64),
                  msg_len=np.zeros(cap, np.uint32))
    rc = L.gen_bdls_round(curve, nval, t2p1, small_len, seed, cap, b.xy.ctypes.data,
                          b.r.ctypes.data, b.r_off.ctypes.data, b.r_len.ctypes.data,
                          b.s.ctypes.data, b.s_off.ctypes.data, b.s_len.ctypes.data,
                          b.version.ctypes.data, b.msg.ctypes.data, msg_cap,
                          b.msg_off.ctypes.data, b.msg_len.ctypes.data)
    if rc != cap:
        raise RuntimeError(f"gen_bdls_round failed: {rc}")
    return b


def concat(parts: list[Workload]) -> Workload:
    """One batch from several (offsets rebased)."""
    msg_base = np.cumsum([0] + [len(p.msg) for p in parts[:-1]]).astype(np.uint64)
    sig_base = np.cumsum([0] + [len(p.sig) for p in parts[:-1]]).astype(np.uint64)
    return Workload(
        pub=np.concatenate([p.pub for p in parts]), msg=np.concatenate([p.msg for p in parts]),
        msg_off=np.concatenate([p.msg_off + b for p, b in zip(parts, msg_base)]),
        msg_len=np.concatenate([p.msg_len for p in parts]),
        sig=np.concatenate([p.sig for p in parts]),
        sig_off=np.concatenate([p.sig_off + b for p, b in zip(parts, sig_base)]),
        sig_len=np.concatenate([p.sig_len for p in parts]),
        reason=np.concatenate([p.reason for p in parts]),
        cls=np.concatenate([p.cls for p in parts]))


def generate_block(ntx: int = 500, endorsements: int = 3, norgs: int = 4, nclients: int = 50,
                   creator_len: int = 4096, endorse_len: int = 1536, corrupt_den: int = 100,
                   seed: int = 3) -> Workload:
    """BASELINE config 3: one block's signatures as txvalidator checks them --
    per tx a creator signature over the ~4 KB envelope payload
    (core/common/validation/msgvalidation.go:245-256 checkSignatureFromCreator)
    and `endorsements` endorser signatures over proposal-response-payload ||
    endorser (core/common/validation/... via policy evaluation,
    common/policies/policy.go:363-395). Endorsers are the norgs peers, creators
    nclients client identities; 1/corrupt_den of the records corrupted."""
    creators = generate(ntx, nclients, creator_len, corrupt_den, seed=seed * 7 + 1)
    endorse = generate(ntx * endorsements, norgs, endorse_len, corrupt_den, seed=seed * 7 + 2)
    return concat([creators, endorse])


def generate_bdls_wire_round(nval: int = 100, curve: int = 1, seed: int = 4):
    """One BDLS round as raw wire messages (SignedProto encodings) for
    bh_bdls_preverify: nval <roundchange>, the leader's <lock> with 2t+1
    proofs, nval <commit>, the leader's <decide> with 2t+1 proofs, all valid.
    Returns (participants: list of 64-byte X||Y, messages: list of bytes)."""
    if not os.path.exists(_LIB):
        raise RuntimeError(f"{_LIB} not built (run `make`)")
    L = ctypes.CDLL(_LIB)
    vp = ctypes.c_void_p
    L.gen_bdls_wire_round.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                      vp, vp, ctypes.c_uint64, vp, vp]
    L.gen_bdls_wire_round.restype = ctypes.c_int
    t2p1 = 2 * ((nval - 1) // 3) + 1
    cnt = 2 * nval + 2
    parts = np.zeros(nval * 64, np.uint8)
    cap = cnt * 512 + 2 * t2p1 * 512
    out = np.zeros(cap, np.uint8)
    off = np.zeros(cnt, np.uint64)
    ln = np.zeros(cnt, np.uint32)
    rc = L.gen_bdls_wire_round(curve, nval, t2p1, seed, parts.ctypes.data, out.ctypes.data, cap,
                               off.ctypes.data, ln.ctypes.data)
    if rc != cnt:
        raise RuntimeError(f"gen_bdls_wire_round failed: {rc}")
    pb = parts.tobytes()
    return ([pb[64 * i:64 * i + 64] for i in range(nval)],
            [out[int(o):int(o) + int(l)].tobytes() for o, l in zip(off, ln)])
