#!/usr/bin/env python3
"""bench.py -- P-256 ECDSA batch-verify throughput on MI355X (BASELINE.json).

Workload (BASELINE.json configs[1] = SURVEY.md 8(d) config 2): per GPU, a batch
of 1,048,576 P-256 records -- 256-byte messages hashed on device (fused
SHA-256, identity.Verify semantics), 65,536 distinct keys, 1/16 of the records
corrupted over eleven reject/accept classes, seed 2 (+ rank).

One "step" = one verify pass over the whole batch with its inputs already
resident in HBM (bh_verify_dev: DER parse, checks, SHA-256, batched inversion,
u1 G + u2 Q, bitmap): `value` is that rate, barrier + device sync around the
K timed steps. The PCIe-inclusive rate SURVEY 8(d) also names for config 2
(H2D + verify + results to page-locked memory per step through
bh_verify_submit from page-locked host buffers, four batches in flight, so
batch k+1's upload runs under batch k's kernels) is measured first and reported beside it as `host_path`.

`--config 5`: ONE seeded batch of 67,108,864 records with a distinct key per
record, split over the ranks by dist.shard_range (8,388,608 per rank at 8 GPUs,
run through the library's 4M-record pass loop); strong scaling.
`--config 3` / `--config 4`: latency of one block (2,000 records) / one BDLS
round (336 SignedProtos), warm and cold.

Multi-GPU: one process per GPU. Under torch.distributed.run the ranks come from
the environment; `--gpus N` without a launcher spawns the N ranks itself (before
anything touches a GPU). Records shard with no data-path collective; a barrier
over bdls_amd.dist's stdlib control channel (127.0.0.1 sockets, rank 0 the hub)
brackets the timed region and the max time over ranks is reported. No rank
process imports torch: libbdlship.so must bind /opt/rocm's HIP runtime, not
the copy torch bundles.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
_T0 = time.time()


def phase(msg: str) -> None:
    """A flushed, timestamped progress line on stderr (stdout carries only the
    JSON line): every long phase of a run -- generation, page-locked
    allocations, uploads, each pass of a multi-pass batch -- says when it
    starts and ends, so a run that stalls shows where (the
    config-5 run was killed after 180 s of silence)."""
    sys.stderr.write(f"[bench +{time.time() - _T0:8.1f}s rank {os.environ.get('RANK', '0')}] "
                     f"{msg}\n")
    sys.stderr.flush()

# Algorithmic work per verify in SURVEY.md 8(d) units: F_p mul/sqr x 128 u32
# MACs (64 product + 64 reduction). SURVEY's fixed schedule S0 prices any
# verify at 3.2e3 F_p ops (4.1e5 MACs). The per-key comb path is split over two
# kernels: k_ktab_ladder builds the key tables (and runs the ladder records),
# k_keycomb walks each record's comb with u1 G folded into the same doublings
# and checks x. Per-batch tables of large batches are signed Lim-Lee combs
# (verify.h lltab_build; BH_LL=0: 4-bit windows) with LL_T teeth spaced LL_S
# bits (BH_LL_T, 7 x 37), 2^(LL_T-1) entries:
#   build (round 5, verify.h lltab_build): (LL_T-1) LL_S doublings (8 ops);
#     the 2 (LL_T-1) chain points made affine (prefix products + 6 per point +
#     an inversion); L over a = (LL_T-1)//2 low digits and H over the rest by
#     two Gray walks (start: a - 1 and LL_T-1-a mixed additions; 2^a - 1 and
#     2^(LL_T-1-a) - 1 steps of a mixed addition (11) + a Z product (1)), made
#     affine (6 per point + an inversion); each entry E = H + L one affine
#     addition whose denominators share an inversion (6 per entry); three
#     safegcd inversions (~14k VALU instructions each, ~85 F_p-op equivalents)
#   comb: LL_S - 1 composite steps 2A + T per record (the top column is
#     loaded, every column is nonzero) + the folded G groups (below)
# windows: build 65 x 58 = 3,770 per table (co-Z chain), comb 65 additions
# (16 ops: the tables are Jacobian) = 1,040 per record + the 13-bit G comb
# (G_WINDOWS mixed additions, computed beside the builds: FP_GPART).
MAC_PER_FP = 128
G_COMB_BITS = 13
G_WINDOWS = (257 + G_COMB_BITS - 1) // G_COMB_BITS
LL_TABLES = os.environ.get("BH_LL", "1") != "0"
# The P-256 ladder (round 5, verify.h q_ladder_odd_g): odd multiples Q..31 Q by
# a co-Z chain (a DBLU ~9 + 15 ZADDU x 7), 51 windows of 4 doublings (8) + the
# composite 2 A + T (16 + 7), 13 folded G additions (11), the x check (~7).
# SURVEY 8(d)'s fixed schedule S0 prices any verify at 3,200 (s0_schedule_frac).
FP_S0 = 3200
FP_LADDER = 9 + 15 * 7 + 51 * (4 * 8 + 16 + 7) + ((-(-257 // 7) - 1) // int(
    os.environ.get("BH_GFOLD", 3)) + 1) * 11 + 7
FP_GPART = G_WINDOWS * 11
LL_T = int(os.environ.get("BH_LL_T", 7))  # the comb shape the library was built with (verify.h)
LL_S = -(-257 // LL_T)
FP_INV_SG = 85
_LL_ENT = 2**(LL_T - 1)
_LL_CHAIN = 2 * (LL_T - 1)
_LL_A = (LL_T - 1) // 2
_LL_NL, _LL_NH = 2**_LL_A, 2**(LL_T - 1 - _LL_A)
FP_KTAB = ((LL_T - 1) * LL_S * 8                                     # the doubling chain
           + (_LL_CHAIN - 1) + 6 * _LL_CHAIN + FP_INV_SG             # chain points affine
           + ((_LL_A - 1) + (LL_T - 1 - _LL_A)) * 11                 # walk starts
           + (_LL_NL - 1 + _LL_NH - 1) * 12                          # walk steps + Z products
           + 6 * (_LL_NL + _LL_NH) + FP_INV_SG                       # L, H affine
           + 6 * _LL_ENT - 1 + FP_INV_SG) if LL_TABLES else 65 * 58  # entries H + L
# round 5: with comb tables u1 G is folded into k_keycomb's Horner (verify.h
# q_llcomb_g): (LL_S - 1) / G_FOLD + 1 mixed additions (13 at 3 columns per
# entry: 12 column groups + column 0) and the x check (~7 ops), no stored u1 G
# half and no final A + B
G_FOLD = int(os.environ.get("BH_GFOLD", 3))  # u1 columns per folded G entry (verify.h kGF)
FOLD_G_ADDS = (LL_S - 1) // G_FOLD + 1
# Each Horner step A = 2 A + V_j Q is (A + T) + A: a mixed addition that also
# rescales A (8M + 3S) + a co-Z addition (5M + 2S) = 18 ops (verify.h ll_dbladd)
FP_KEYCOMB = ((LL_S - 1) * 18 + FOLD_G_ADDS * 11 + 7) if LL_TABLES else 65 * 16 + 23
MACS_PER_VERIFY = FP_S0 * MAC_PER_FP
KERNELS = {"build_ladder_ms": "k_ktab_ladder", "keycomb_ms": "k_keycomb"}
MAX_LANES = 4  # bdls_hip.cpp kMaxLanes


def lane_count() -> int:
    """The library's compute lanes (bdls_hip.cpp lanes(): BH_LANES, default 3)."""
    try:
        v = int(os.environ.get("BH_LANES", "3"))
    except ValueError:
        v = 3
    return min(MAX_LANES, max(1, v))
CONFIG5_TOTAL = 1 << 26


NOMINAL_MAC_PEAK = 256 * 4 * 16 * 2.4e9  # u32 MAC/s at the nominal VOP3 issue rate


def kernel_fp_ops(stage: str, routes: dict) -> float:
    """Algorithmic F_p ops of one launch of the stage's kernel."""
    if stage == "build_ladder_ms":
        return (routes["ladder"] * FP_LADDER + routes["key_tables"] * FP_KTAB
                + (0 if LL_TABLES else routes["keycomb"] * FP_GPART))
    return routes["keycomb"] * FP_KEYCOMB


# Algorithmic HBM bytes per verify record (config 2): pub 64 + sig ~71 + msg 256
# + offsets/lengths 24 + reason 1 + bitmap 1/8.
def alg_bytes_per_record(msg_len: int) -> float:
    return 64 + 72 + msg_len + 24 + 1 + 0.125


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=1 << 20, help="config 2: records per GPU")
    ap.add_argument("--n-total", type=int, default=CONFIG5_TOTAL,
                    help="config 5: records of the one batch split over all GPUs")
    ap.add_argument("--config", type=int, default=2, choices=[1, 2, 3, 4, 5],
                    help="1: host-CPU reference proxy; 2/5: throughput; 3 (block) / 4 (BDLS "
                         "round): latency")
    ap.add_argument("--curve", type=int, default=1, help="config 4: 1 secp256k1 (as wired), 0 P-256")
    ap.add_argument("--validators", type=int, default=100, help="config 4")
    ap.add_argument("--nkeys", type=int, default=65536)
    ap.add_argument("--msg-len", type=int, default=256)
    ap.add_argument("--corrupt-den", type=int, default=16)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--host-layout", choices=["compact", "plain"], default="compact",
                    help="host path input layout: bh_cbatch (distinct keys + u32 indices, "
                         "lengths only) or bh_batch (per-record keys, u64 offsets)")
    ap.add_argument("--e2e", type=int, default=1,
                    help="time host_path_e2e: the staged BatchVerify (bh_batch_verify_submit) "
                         "from pageable generator arrays, packing inside the timed region")
    ap.add_argument("--resident-lanes", type=int, default=1,
                    help="timed resident passes rotate over the compute lanes (BH_F_ANY_LANE)")
    ap.add_argument("--hbm-resident", type=int, default=1,
                    help="also time the same passes on inputs already in HBM")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the CPU oracle on rank 0")
    ap.add_argument("--cpu-sample", type=int, default=1 << 20)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = os.cpu_count()")
    ap.add_argument("--mac-peak", type=float, default=float(os.environ.get("BH_MAC_PEAK", 0) or 0),
                    help="measured v_mad_u64_u32 peak (MAC/s); default: profiles/ubench.json")
    ap.add_argument("--side-configs", type=int, default=1,
                    help="default run: also measure configs 1, 3, 4 and the single Verify")
    ap.add_argument("--side-steps", type=int, default=20)
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: exercise the launcher and the rank plumbing only")
    ap.add_argument("--c5-cache", default=os.environ.get("BDLS_C5_CACHE", ""),
                    help="config 5: directory of the on-disk copy of the seeded shard "
                         "(default: <tmp>/bdls_c5_cache; 'off' disables)")
    ap.add_argument("--c5-cache-save", type=int, default=1,
                    help="config 5: write a freshly generated shard to the cache")
    return ap.parse_args(argv)


def mac_peak_default() -> tuple[float, str]:
    path = os.path.join(ROOT, "profiles", "ubench.json")
    if os.path.exists(path):
        with open(path) as f:
            u = json.load(f)
        return (float(u.get("mad_u64_u32_per_s_32ch", u["mad_u64_u32_per_s"])),
                "profiles/ubench.json: measured chip-wide v_mad_u64_u32 throughput (32 chains/lane)")
    # 256 CU x 4 SIMD x 32 lanes x 2.4 GHz / 4 (quarter-rate assumption)
    return 256 * 4 * 32 * 2.4e9 / 4, "assumed quarter-rate v_mad_u64_u32"


def percentile(v, q):
    return float(np.percentile(np.asarray(v), q))


def host_cpus() -> dict:
    """The host's CPU count (os.cpu_count, = nproc without affinity limits) and
    what this process may actually run on (affinity mask, cgroup quota)."""
    info = {"nproc": os.cpu_count() or 1}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            info["cgroup_quota_cpus"] = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return info


# ---------------------------------------------------------------- launcher
def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` without a launcher: start N rank processes (this
    script again, one GPU each) -- the parent never touches a GPU -- and exit
    with the worst child status. Rank 0 prints the JSON line."""
    import shutil
    import tempfile
    port = free_port()
    ctrl = tempfile.mkdtemp(prefix="bdls_ctrl_")  # the ranks' rendezvous (bdls_amd/dist.py)
    procs = []
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                       LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                       BDLS_CTRL_DIR=ctrl)
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)]
                                          + sys.argv[1:], env=env))
        rcs = [p.wait() for p in procs]
    finally:
        shutil.rmtree(ctrl, ignore_errors=True)
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


# ---------------------------------------------------------------- latency
def bench_latency(a, rank, world, local):
    """Configs 3 and 4: latency of one batch through the host C ABI (H2D +
    verify + D2H, what a Go caller sees) and device-resident, p50/p99 over
    --steps calls. N GPUs run N independent replicas (the path does not shard
    at this size)."""
    from bdls_amd import _lib, dist, workload
    local, _ = dist.device_for_rank(local)
    L = _lib.lib()
    _lib.check(L.bh_init(1 << local, 0))
    assert "torch" not in sys.modules, "torch must not share a process with libbdlship.so"
    DA = _lib.DeviceArray
    if a.config == 3:
        w = workload.generate_block(seed=a.seed + 1000 * rank)
        n, curve = w.n, _lib.BH_CURVE_P256
        hb = _lib.BhBatch(*[x.ctypes.data for x in (w.pub, w.sig, w.sig_off, w.sig_len, w.msg,
                                                    w.msg_off, w.msg_len)])
        dev = [DA.from_numpy(local, x) for x in (w.pub, w.sig, w.sig_off, w.sig_len, w.msg,
                                                 w.msg_off, w.msg_len)]
        db = _lib.BhBatch(*[x.ptr for x in dev])
        expect = w.reason
        workload_desc = (f"BASELINE config 3: one block, 500 tx x (creator over 4096 B + 3 "
                         f"endorsements over 1536 B) = {n} P-256 records, 50 client + 4 peer "
                         f"keys, 1/100 corrupted, fused SHA-256")
        flags = _lib.BH_F_HASH_SHA256

        def host_call(bitmap, reason):
            return L.bh_verify(curve, ctypes.byref(hb), n, flags, bitmap.ctypes.data,
                               reason.ctypes.data)

        def dev_call(words, reason, tm):
            return L.bh_verify_dev(local, curve, ctypes.byref(db), n, flags, words.ptr,
                                   reason.ptr, None, 1, tm)
    else:
        r = workload.generate_bdls_round(a.validators, a.curve, seed=a.seed + 1000 * rank)
        n, curve = r.n, a.curve
        arrs = r.arrays()
        hb = _lib.BhBdlsBatch(*[x.ctypes.data for x in arrs])
        dev = [DA.from_numpy(local, x) for x in arrs]
        db = _lib.BhBdlsBatch(*[x.ptr for x in dev])
        expect = np.zeros(n, np.uint8)
        t2p1 = 2 * ((a.validators - 1) // 3) + 1
        workload_desc = (f"BASELINE config 4: one BDLS round at {a.validators} validators -- "
                         f"{a.validators} roundchange + lock + {t2p1} proofs + "
                         f"{a.validators} commit + decide + {t2p1} proofs = {n} SignedProto "
                         f"records, {'secp256k1' if curve == 1 else 'P-256'}, BLAKE2b-256")

        def host_call(bitmap, reason):
            return L.bh_verify_bdls(curve, ctypes.byref(hb), n, bitmap.ctypes.data,
                                    reason.ctypes.data)

        def dev_call(words, reason, tm):
            return L.bh_verify_bdls_dev(local, curve, ctypes.byref(db), n, words.ptr,
                                        reason.ptr, None, 1, tm)

    bitmap = np.zeros((n + 7) // 8, np.uint8)
    reason = np.zeros(n, np.uint8)
    dwords = DA(local, ((n + 63) // 64) * 8)
    dreason = DA(local, n)
    pubs = np.unique((w.pub if a.config == 3 else r.xy).reshape(-1, 64)[:n], axis=0)

    def measure(tag):
        for _ in range(max(1, a.warmup)):
            _lib.check(host_call(bitmap, reason))
            _lib.check(dev_call(dwords, dreason, None))
        dist.barrier(world)
        host_ms, dev_ms = [], []
        for _ in range(a.steps):
            t = time.perf_counter()
            _lib.check(host_call(bitmap, reason))
            host_ms.append((time.perf_counter() - t) * 1e3)
        for _ in range(a.steps):
            t = time.perf_counter()
            _lib.check(dev_call(dwords, dreason, None))
            dev_ms.append((time.perf_counter() - t) * 1e3)
        tm = _lib.BhTiming()
        _lib.check(dev_call(dwords, dreason, ctypes.byref(tm)))
        ok = bool((reason == expect).all() and (dreason.to_numpy(np.uint8, n) == expect).all()
                  and (np.unpackbits(bitmap, bitorder="little")[:n].astype(bool)
                       == (expect == 0)).all())
        return {
            "host_p50": round(percentile(host_ms, 50), 4),
            "host_p99": round(percentile(host_ms, 99), 4),
            "device_resident_p50": round(percentile(dev_ms, 50), 4),
            "device_resident_p99": round(percentile(dev_ms, 99), 4),
            "kernel_ms": {k: round(getattr(tm, k), 4) for k in _lib.BhTiming.STAGES},
            "routes": {"keycomb": tm.n_keycomb, "ladder": tm.n_ladder,
                       "key_tables": tm.n_keytables, "wide": tm.wide},
            "parity": ok,
        }

    # cold: no key known to the device (per-batch tables are off at this size,
    # every record takes the ladder)
    _lib.check(L.bh_keys_clear(-1, curve))
    cold = measure("cold")
    # warm: the batch's public keys registered once beforehand (the Fabric
    # MSP identity cache / the BDLS participant set); registration timed alone
    t = time.perf_counter()
    st = np.zeros(len(pubs), np.uint8)
    _lib.check(L.bh_keys_register(-1, curve, np.ascontiguousarray(pubs).ctypes.data, len(pubs),
                                  st.ctypes.data))
    reg_ms = (time.perf_counter() - t) * 1e3
    warm = measure("warm")
    _lib.check(L.bh_keys_clear(-1, curve))
    wire = measure_wire(a, L, curve, rank) if a.config == 4 else None
    block = measure_block(a, L, rank) if a.config == 3 else None
    _lib.check(L.bh_keys_clear(-1, curve))
    if block is not None:
        # config 3's value: the whole block through bh_fabric_block_preverify
        # (decode + identities + every creator / endorsement signature in one
        # device batch), endorser / creator keys kept in the registry
        p50 = dist.max_over_ranks(block["warm"]["p50"], world)
        value_is = ("bh_fabric_block_preverify on the serialized common.Block (500 endorser "
                    "txs, creator + 3 endorsements each): decode + identity resolution + one "
                    "device batch, keys kept in the registry (warm) p50, host-to-host")
    elif wire is not None:
        # config 4's value: the A16 entry (bh_bdls_preverify) that
        # inputConsensusMessage calls, participants' keys registered
        p50 = dist.max_over_ranks(wire["warm"]["p50"], world)
        value_is = ("bh_bdls_preverify (agent-tcp/tcp_peer.go:176-192 inputConsensusMessage: "
                    "decode + participant gate + proof checks + one device batch) on the raw "
                    "wire round, participants' keys registered (warm) p50")
    else:
        p50 = dist.max_over_ranks(warm["host_p50"], world)
        value_is = ("warm host_p50: keys registered before timing (bh_keys_register); "
                    "cold = no key known")
    parity_ok = dist.all_true(cold["parity"] and warm["parity"], world)
    out = {
        "metric": ("block-validate latency (ms, one block's signatures, host C ABI)"
                   if a.config == 3 else "BDLS round verify latency (ms, host C ABI)"),
        "value": round(p50, 4), "unit": "ms", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(p50, 4), "higher_is_better": False,
        "scaling": "replicas", "vs_baseline": None,
        "dtype": "u32", "data": "synthetic (seeded keys/signatures, workload/gen.c)",
        "config": {"workload": workload_desc, "records": n, "distinct_keys": len(pubs),
                   "value_is": value_is},
        "parity": parity_ok,
        "latency_ms": {"warm": warm, "cold": cold,
                       "register_keys_ms": round(reg_ms, 3)},
    }
    if block is not None:
        out["latency_ms"]["block_preverify"] = block
        out["parity"] = parity_ok = dist.all_true(parity_ok and block["parity"], world)
        out["config"]["block_bytes"] = block["block_bytes"]
    if wire is not None:
        out["latency_ms"]["wire_preverify"] = wire
        out["parity"] = parity_ok = dist.all_true(parity_ok and wire["parity"], world)
    if rank == 0 and a.cpu_baseline:
        from oracle import orc
        cpu = []
        cpus = host_cpus()
        threads = a.cpu_threads or int(min(cpus.get("affinity", cpus["nproc"]),
                                           cpus.get("cgroup_quota_cpus", cpus["nproc"]))) or 1
        deadline = time.perf_counter() + 10.0
        while time.perf_counter() < deadline and len(cpu) < a.steps:
            t = time.perf_counter()
            if a.config == 3:
                got = orc.batch_verify(w.pub.reshape(-1, 64), w.msg, w.msg_off, w.msg_len, w.sig,
                                       w.sig_off, w.sig_len, fused=True, nthreads=threads)
            else:
                got = orc.bdls_verify(curve, *arrs)
            cpu.append((time.perf_counter() - t) * 1e3)
        cores = threads if a.config == 3 else 1
        out["cpu_baseline"] = {
            "value": round(percentile(cpu, 50), 4), "unit": "ms", "cores": cores, "kind": "port",
            "host_cpus": cpus,
            "sample": f"the same {n} records, {len(cpu)} repetitions, p50; "
                      + ("identity.Verify semantics, OpenSSL ECDSA_do_verify, "
                         f"{cores} threads (the CPUs this process may use)" if a.config == 3 else
                         "serial SignedProto.Verify as the consensus loop runs it "
                         "(BLAKE2b-256 + OpenSSL ECDSA_do_verify), 1 thread"),
            "parity": bool((got == expect).all()),
        }
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.finalize(world)
    return 0 if parity_ok else 3


def measure_block(a, L, rank):
    """Config 3 through bh_fabric_block_preverify: one serialized block
    (bdls_amd/workload/fabric.py: 500 endorser txs, X.509 identities of 4 peers
    and 50 clients, 1/100 corrupted). Cold = no key known to the device (every
    signature on the ladder); warm = BH_FAB_F_KEEP_KEYS after a first block
    (the peer's long-lived identities keep device tables)."""
    from bdls_amd import _lib
    from bdls_amd.workload import fabric as F
    fb = F.generate_fabric_block(seed=a.seed + 1000 * rank)
    buf = np.frombuffer(fb.block + b"\0", np.uint8)
    ntx, nend = ctypes.c_size_t(), ctypes.c_size_t()
    txs = (_lib.BhFabTx * fb.ntx)()
    cap = sum(len(e) for e in fb.tx_endorse) + 64 * fb.ntx
    end = np.zeros(cap, np.uint8)
    want = [(fb.tx_status[i], fb.tx_creator[i], fb.tx_endorse[i], fb.tx_valid_identities[i])
            for i in range(fb.ntx)]

    def call(flags):
        return L.bh_fabric_block_preverify(buf.ctypes.data, len(fb.block), flags, txs, fb.ntx,
                                           ctypes.byref(ntx), end.ctypes.data, cap,
                                           ctypes.byref(nend))

    def check():
        got = [(t.status, t.creator,
                [int(x) for x in end[t.endorse_first:t.endorse_first + t.endorse_count]],
                t.valid_endorsers) for t in txs[:ntx.value]]
        return got == want

    def run(flags, clear):
        for _ in range(max(1, a.warmup)):
            if clear:
                _lib.check(L.bh_keys_clear(-1, 0))
            _lib.check(call(flags))
        ms = []
        for _ in range(a.steps):
            if clear:
                _lib.check(L.bh_keys_clear(-1, 0))
            t = time.perf_counter()
            _lib.check(call(flags))
            ms.append((time.perf_counter() - t) * 1e3)
        return {"p50": round(percentile(ms, 50), 4), "p99": round(percentile(ms, 99), 4),
                "parity": check()}

    cold = run(0, True)
    dec = []
    for _ in range(max(5, a.steps)):  # host half alone: decode + identities, p50
        t = time.perf_counter()
        _lib.check(call(_lib.BH_FAB_F_DECODE_ONLY))
        dec.append((time.perf_counter() - t) * 1e3)
    decode_ms = percentile(dec, 50)
    warm = run(_lib.BH_FAB_F_KEEP_KEYS, False)
    return {"warm": warm, "cold": cold, "decode_only_ms": round(decode_ms, 4),
            "transactions": fb.ntx, "signatures": fb.n_signatures,
            "block_bytes": len(fb.block), "parity": bool(warm["parity"] and cold["parity"])}


def measure_wire(a, L, curve, rank):
    """Config 4 through bh_bdls_preverify: the round as raw wire messages
    (what agent-tcp's inputConsensusMessage drains), decoded, gated and
    structurally checked on the host, every SignedProto verified in one device
    batch. Cold = no key known to the device; warm = the wire round's own
    participants registered first (the BDLS participant set,
    consensus.go:456-466)."""
    from bdls_amd import _lib, workload
    ids, raws = workload.generate_bdls_wire_round(a.validators, curve, seed=a.seed + 1000 * rank)
    n = len(raws)
    ln = np.array([len(m) for m in raws], np.uint32)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    buf = np.frombuffer(b"".join(raws), np.uint8)
    parts = np.frombuffer(b"".join(ids), np.uint8)
    res = (_lib.BhBdlsMsgResult * n)()
    cap = n + len(buf) // 2 + 1
    rs = np.zeros(cap, np.uint8)
    total = ctypes.c_size_t()

    def call():
        return L.bh_bdls_preverify(curve, buf.ctypes.data, off.ctypes.data, ln.ctypes.data, n,
                                   parts.ctypes.data, len(ids), 0, res, rs.ctypes.data, cap,
                                   ctypes.byref(total))
    t2p1 = 2 * ((a.validators - 1) // 3) + 1

    def run():
        for _ in range(max(1, a.warmup)):
            _lib.check(call())
        ms = []
        for _ in range(a.steps):
            t = time.perf_counter()
            _lib.check(call())
            ms.append((time.perf_counter() - t) * 1e3)
        ok = (total.value == 2 * a.validators + 2 * (1 + t2p1)
              and all(res[i].status == 0 for i in range(n)) and not rs[:total.value].any())
        return {"p50": round(percentile(ms, 50), 4), "p99": round(percentile(ms, 99), 4),
                "parity": bool(ok)}

    _lib.check(L.bh_keys_clear(-1, curve))
    cold = run()
    st = np.zeros(len(ids), np.uint8)
    _lib.check(L.bh_keys_register(-1, curve, parts.ctypes.data, len(ids), st.ctypes.data))
    assert not st.any(), "participant key registration failed"
    warm = run()
    return {"warm": warm, "cold": cold, "messages": n, "wire_bytes": int(len(buf)),
            "signed_protos": int(total.value), "parity": bool(warm["parity"] and cold["parity"])}


# ---------------------------------------------------------------- throughput
def load_counters(config: int, n_rank: int):
    """Per-launch HBM traffic and counter-based VALU utilisation of the
    kernels, from the rocprofv3 --pmc passes summarised in
    profiles/traffic.json (tools/pmc_summary.py), when they were taken on
    this same workload AND on this kernel build: the file's kernel_src_sha must
    equal the hash of the kernel sources beside the library (bdls_amd/
    provenance.py); otherwise the counters are stale and not printed.
    Returns (source, kernels, stale_reason)."""
    from bdls_amd import _lib
    from bdls_amd.provenance import lib_kernel_sha
    prof = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(prof):
        return None, {}, "no profiles/traffic.json"
    with open(prof) as f:
        tr = json.load(f)
    want = f"config{config}:n{n_rank}"
    if tr.get("workload") != want:
        return None, {}, f"counters taken on {tr.get('workload')}, not {want}"
    cur = lib_kernel_sha(_lib.LIB_PATH)
    if cur is None:
        return None, {}, "the loaded library has no build record (bdls_amd/lib/BUILD_INFO.json)"
    if tr.get("kernel_src_sha") != cur:
        return None, {}, (f"stale: counters describe kernel sources {tr.get('kernel_src_sha')} "
                          f"(rev {tr.get('git_rev')}), this library was built from {cur}")
    return (f"{tr.get('source')} @ rev {tr.get('git_rev')}, kernel_src_sha {cur}",
            tr.get("kernels", {}), None)


def cpu_baseline(a, w, n):
    """oracle/orc.c (Fabric DER + low-S rules restated in C, the ECDSA core in
    OpenSSL's P-256 assembly) on this host's CPUs, on the first records of the
    same batch. Timed twice: with the CPUs this process may actually use
    (affinity mask and cgroup quota -- on the GPU box a 16-CPU quota of a
    256-thread host) and with os.cpu_count() threads (nproc); `value` is the
    faster of the two (the conservative baseline for the GPU's claim)."""
    from oracle import orc
    cpus = host_cpus()
    usable = int(min(cpus.get("affinity", cpus["nproc"]),
                     cpus.get("cgroup_quota_cpus", cpus["nproc"]))) or 1
    m = min(a.cpu_sample, n)
    runs = {}
    for threads in sorted({a.cpu_threads or usable, cpus["nproc"]}):
        t = time.perf_counter()
        orc.batch_verify(w.pub[:64 * m].reshape(-1, 64), w.msg, w.msg_off[:m], w.msg_len[:m],
                         w.sig, w.sig_off[:m], w.sig_len[:m], fused=True, nthreads=threads)
        dt = time.perf_counter() - t
        runs[threads] = {"value": round(m / dt, 1), "seconds": round(dt, 3)}
    best = max(runs, key=lambda k: runs[k]["value"])
    return {
        "value": runs[best]["value"], "unit": "verifies/s", "cores": best, "kind": "port",
        "host_cpus": cpus,
        "by_threads": {str(k): v for k, v in runs.items()},
        "per_thread": round(runs[best]["value"] / min(best, usable), 1),
        "sample": f"first {m} records of the same batch, identity.Verify semantics (SHA-256 + "
                  f"DER + low-S + ECDSA via OpenSSL ECDSA_do_verify), timed at {sorted(runs)} "
                  f"threads (usable CPUs, os.cpu_count()); value = the faster",
    }


def cgroup_throttle():
    """(nr_throttled, throttled_usec) of this process's cgroup (v2), or zeros."""
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            d = dict(l.split() for l in f)
        return int(d.get("nr_throttled", 0)), int(d.get("throttled_usec", 0))
    except (OSError, ValueError):
        return 0, 0


def measure_e2e(a, L, w, n, flags, local, world, depth, h2d_gbps):
    """host_path_e2e: K BatchVerify calls through bh_batch_verify_submit /
    bh_verify_wait from PAGEABLE arrays (the generator's, copied into ordinary
    numpy memory), up to `depth` in flight. Timed: everything per batch --
    the library's key dedup + packing into its page-locked ring (pack.h),
    the H2D, the pass, the results. Its PCIe bound counts the bytes the staged
    path uploads (the compact layout it builds: distinct keys + u32 indices,
    lengths, signature and message bytes)."""
    from collections import deque

    from bdls_amd import _lib, dist
    phase("host_path_e2e: pageable copies of the batch")
    arrs = [np.array(x, copy=True) for x in w.arrays()]  # ordinary (pageable) memory
    b = _lib.BhBatch(*[x.ctypes.data for x in arrs])
    outs = [(np.zeros((n + 7) // 8, np.uint8), np.zeros(n, np.uint8)) for _ in range(depth)]

    acc = {"submit_s": 0.0, "wait_s": 0.0}

    def run(steps):
        q = deque()
        pc = time.perf_counter
        for k in range(steps):
            if len(q) == depth:
                t = pc()
                _lib.check(L.bh_verify_wait(q.popleft()))
                acc["wait_s"] += pc() - t
            bm, rs = outs[k % depth]
            job = ctypes.c_void_p()
            t = pc()
            _lib.check(L.bh_batch_verify_submit(0, ctypes.byref(b), n, flags, bm.ctypes.data,
                                                rs.ctypes.data, ctypes.byref(job)))
            acc["submit_s"] += pc() - t
            q.append(job)
        t = pc()
        while q:
            _lib.check(L.bh_verify_wait(q.popleft()))
        acc["wait_s"] += pc() - t

    run(max(1, a.warmup))
    _lib.check(L.bh_sync(local))
    # one call alone: a BatchVerify's latency (pack + upload + pass + results)
    t = time.perf_counter()
    run(1)
    single_ms = (time.perf_counter() - t) * 1e3
    st1 = _lib.pack_stats()
    dist.barrier(world)
    shards0 = st1["shards"]
    phase(f"host_path_e2e: {a.steps} timed batches")
    acc.update(submit_s=0.0, wait_s=0.0)
    thr0 = cgroup_throttle()
    t0 = time.perf_counter()
    run(a.steps)
    t1 = time.perf_counter()
    thr1 = cgroup_throttle()
    st = _lib.pack_stats()
    dist.barrier(world)
    elapsed = dist.max_over_ranks(t1 - t0, world)
    bm, rs = outs[(a.steps - 1) % depth]
    bits = np.unpackbits(bm, bitorder="little")[:n].astype(bool)
    ok = bool((rs == w.reason).all() and (bits == w.expected_valid).all())
    # bytes the staged path uploads per batch (its compact layout)
    nk = int(st["nkeys"])
    fixed = bool((w.msg_len == w.msg_len[0]).all()) if n else True
    up_bytes = (nk * 64 + (4 * n if st["dedup"] else 0) + 4 * n + (0 if fixed else 4 * n)
                + int(w.sig_len.sum()) + int(w.msg_len.sum()))
    value = dist.sum_over_ranks(n, world) * a.steps / elapsed
    pcie_bound = world * n * h2d_gbps * 1e9 / up_bytes
    ms = elapsed * 1e3 / a.steps
    pack_ms = st["pass_a_ms"] + st["pass_b_ms"]
    phase(f"host_path_e2e: {ms:.2f} ms per batch ({value / 1e6:.1f} M/s), pack "
          f"{pack_ms:.2f} ms on {int(st['threads'])} threads, parity {ok}")
    return {"value": round(value, 1), "ms_per_step": round(ms, 3), "parity": ok,
            "what": ("bh_batch_verify_submit / bh_verify_wait over the generator's batch copied "
                     "into pageable memory, up to %d in flight; timed per batch: key dedup + "
                     "packing into the library's reused page-locked staging (pack.h worker "
                     "pool), chunked H2D, the pass, results -- no untimed per-batch step" % depth),
            "single_batch_ms": round(single_ms, 3),
            "cgroup_throttled_ms": round((thr1[1] - thr0[1]) / 1e3, 1),
            "cgroup_nr_throttled": thr1[0] - thr0[0],
            "submit_ms_per_batch": round(acc["submit_s"] * 1e3 / a.steps, 3),
            "wait_ms_per_batch": round(acc["wait_s"] * 1e3 / a.steps, 3),
            "upload_bytes_per_batch": up_bytes,
            "pcie_bound_verifies_per_s": round(pcie_bound, 1),
            "pcie_frac": round(value / pcie_bound, 3),
            "pack": {"pass_a_ms": round(st["pass_a_ms"], 3), "pass_b_ms": round(st["pass_b_ms"], 3),
                     "threads": int(st["threads"]), "chunks": int(st["chunks"]),
                     "dedup": bool(st["dedup"]), "keys_uploaded": nk,
                     "est_distinct": round(st["est_distinct"], 1),
                     "batches": int(st["shards"] - shards0),
                     "note": "the last timed batch's passes (wall time on the submitting "
                             "thread; pass B's H2D copies run under it)"},
            "per_batch_ms": {"pack_cpu": round(pack_ms, 3),
                             "pcie": round(up_bytes / (h2d_gbps * 1e9) * 1e3, 3)},
            }


def bench_throughput(a, rank, world, local):
    from bdls_amd import _lib, dist, workload
    if a.config == 5:
        n_total = a.n_total
        lo, hi = dist.shard_range(n_total, rank, world)
        seed, nkeys, corrupt = 5, n_total, 64
        scaling = "strong"
        desc = (f"BASELINE config 5: one seeded batch of {n_total} records, one distinct key "
                f"per record, 256B messages, 1/64 corrupted, fused SHA-256; rank {rank} "
                f"verifies records [{lo}, {hi}) (dist.shard_range)")
    else:
        lo, hi = 0, a.n
        n_total = a.n * world
        seed, nkeys, corrupt = a.seed + 1000 * rank, a.nkeys, a.corrupt_den
        scaling = "weak"
        desc = (f"BASELINE config 2: {a.n} records/GPU, {a.msg_len}B messages, {nkeys} distinct "
                f"keys, 1/{corrupt} corrupted, fused SHA-256")
    n = hi - lo
    dev, dev_why = dist.device_for_rank(local)
    phase(f"config {a.config}: {n} records [{lo}, {hi}) of {n_total}; device {dev} ({dev_why})")
    local = dev  # the device index every call below addresses

    # Page-locked host memory comes from libbdlship.so (bh_host_alloc); torch
    # ships its own HIP runtime and is never imported into a rank process.
    L = _lib.lib()
    _lib.check(L.bh_init(1 << local, 0))
    assert "torch" not in sys.modules, "torch must not share a process with libbdlship.so"
    phase("bh_init done")

    pinned = []

    def alloc(nbytes):
        t = time.time()
        h = _lib.HostArray(nbytes)
        pinned.append(h)
        if nbytes >= (256 << 20):
            phase(f"page-locked {nbytes / 1e9:.2f} GB in {time.time() - t:.2f} s")
        return h.u8

    t_gen = time.time()
    # generator threads: the CPUs this node's ranks may actually use (affinity
    # and cgroup quota, not os.cpu_count()) shared by the local ranks -- 8
    # ranks on a 16-CPU quota get 2 each, not 4
    cpus = host_cpus()
    usable = int(min(cpus.get("affinity", cpus["nproc"]),
                     cpus.get("cgroup_quota_cpus", cpus["nproc"]))) or 1
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", min(world, 8)))
    gen_threads = max(1, min(32, usable // max(1, local_world)))
    gen_info = {"threads": gen_threads}
    if a.config == 5:
        # one seeded unique-key batch: generated in 1M-record chunks with a
        # progress line each, into page-locked arrays allocated once, and
        # kept on local disk for the next run
        import tempfile
        cache = a.c5_cache or os.path.join(tempfile.gettempdir(), "bdls_c5_cache")
        phase(f"shard: cache {cache if cache != 'off' else 'off'}, {gen_threads} generator "
              f"threads")
        w, info = workload.generate_shard_cached(
            n_total, lo, n, nkeys, a.msg_len, corrupt, seed=seed, nthreads=gen_threads,
            alloc=alloc, cache_dir=None if cache == "off" else cache, save=bool(a.c5_cache_save),
            log=phase)
        gen_info.update(info)
    else:
        w = workload.generate_shard(a.n, lo, n, nkeys, a.msg_len, corrupt, seed=seed,
                                    nthreads=gen_threads, alloc=alloc)
    t_gen = time.time() - t_gen
    phase(f"workload ready in {t_gen:.1f} s ({gen_info.get('source', 'generator')})")
    flags = _lib.BH_F_HASH_SHA256
    hb = _lib.BhBatch(*[x.ctypes.data for x in (w.pub, w.sig, w.sig_off, w.sig_len, w.msg,
                                                w.msg_off, w.msg_len)])
    # config 5's keys are all distinct: the compact layout would hold the whole
    # batch a second time in page-locked memory (and its key dedup / signature
    # repack are minutes of numpy at 64M records) to save nothing -- plain
    layout = "plain" if a.config == 5 else a.host_layout
    compact = layout == "compact"
    if compact:
        # what a Go BatchVerify hands over: each distinct key once + a u32
        # index per record, lengths only (fixed 256-byte messages: none)
        t = time.time()
        carrs, cb = _lib.compact_layout(w.pub, w.sig, w.sig_off, w.sig_len, w.msg, w.msg_off,
                                        w.msg_len, alloc=alloc)
        layout_s = time.time() - t
        phase(f"compact layout built in {layout_s:.2f} s")
    # batches in flight (the library keeps 4 pipeline slots per device)
    depth = int(os.environ.get("BENCH_HOST_DEPTH", "4"))
    outs = [(np.zeros((n + 7) // 8, np.uint8), np.zeros(n, np.uint8)) for _ in range(depth)]
    multipass = n > (1 << 22)

    def submit(k):
        job = ctypes.c_void_p()
        bm, rs = outs[k % depth]
        if compact:
            _lib.check(L.bh_verify_compact_submit(0, ctypes.byref(cb), n, flags, bm.ctypes.data,
                                                  rs.ctypes.data, ctypes.byref(job)))
        else:
            _lib.check(L.bh_verify_submit(0, ctypes.byref(hb), n, flags, bm.ctypes.data,
                                          rs.ctypes.data, ctypes.byref(job)))
        return job

    def run_host(steps):
        """steps BatchVerify calls, up to `depth` in flight: batch k+2's upload
        is enqueued while batch k still computes, so no upload waits on the
        host's collection of an earlier batch."""
        from collections import deque
        q = deque()
        for k in range(steps):
            if len(q) == depth:
                _lib.check(L.bh_verify_wait(q.popleft()))
                if multipass:
                    phase(f"host path: batch {k - depth} done")
            q.append(submit(k))
        while q:
            _lib.check(L.bh_verify_wait(q.popleft()))
            if multipass:
                phase("host path: batch done")

    phase(f"host path: {a.warmup} warmup batches")
    run_host(a.warmup)
    _lib.check(L.bh_sync(local))
    # one batch alone (nothing in flight): H2D + verify + results latency, and the
    # page-locked H2D bandwidth of the batch's largest array
    phase("host path: one batch alone")
    t = time.perf_counter()
    run_host(1)
    single_ms = (time.perf_counter() - t) * 1e3
    probe = _lib.DeviceArray(local, w.msg.nbytes)
    t = time.perf_counter()
    _lib.check(L.bh_memcpy_h2d(local, probe.ptr, w.msg.ctypes.data, w.msg.nbytes))
    h2d_gbps = w.msg.nbytes / (time.perf_counter() - t) / 1e9
    probe.free()
    if compact:
        batch_bytes = sum(int(x.nbytes) for x in carrs.values() if x is not None)
    else:
        batch_bytes = sum(int(x.nbytes) for x in (w.pub, w.sig, w.sig_off, w.sig_len, w.msg,
                                                  w.msg_off, w.msg_len))
    dist.barrier(world)
    # Timed region: K host-buffer batches. The library rotates them over its
    # compute lanes (bdls_hip.cpp Lane1), so batch k+1's kernels run beside
    # batch k's; per-kernel durations are therefore taken from the serialised
    # HBM-resident passes below (HIP events around every stage of every pass,
    # bh_timing_begin/_end), where each kernel has the device to itself --
    # unless those are skipped, then from these passes.
    tm = _lib.BhTiming()
    if not a.hbm_resident:
        _lib.check(L.bh_timing_begin(local))
    phase(f"host path: {a.steps} timed batches")
    t0 = time.perf_counter()
    run_host(a.steps)
    t1 = time.perf_counter()
    phase(f"host path: {(t1 - t0) * 1e3 / a.steps:.2f} ms per batch")
    if not a.hbm_resident:
        _lib.check(L.bh_timing_end(local, ctypes.byref(tm)))
    dist.barrier(world)
    elapsed = dist.max_over_ranks(t1 - t0, world)
    bm, rs = outs[(a.steps - 1) % depth]
    bits = np.unpackbits(bm, bitorder="little")[:n].astype(bool)
    parity_ok = bool((rs == w.reason).all() and (bits == w.expected_valid).all())

    # host_path_e2e: what a Go BatchVerify caller gets --
    # the records in ordinary pageable memory (copies of the generator's
    # arrays), and every per-batch host step inside the timed region: the
    # library's key de-duplication and packing into its own reused page-locked
    # staging (pack.h worker pool), the chunked H2D, the pass, the results
    e2e = None
    if a.e2e and a.config != 5:
        e2e = measure_e2e(a, L, w, n, flags, local, world, depth, h2d_gbps)
        parity_ok = parity_ok and e2e["parity"]

    # the same passes on inputs already resident in HBM (no PCIe in the loop).
    # Timed: K passes rotating over the compute lanes (BH_F_ANY_LANE; one
    # output set per possible lane, so no in-flight pass shares its outputs),
    # so pass k+1's early kernels fill pass k's tail as host batches do. Per-kernel durations (roofline) come from K more passes run
    # serialised, each kernel alone on the device.
    resident = None
    if a.hbm_resident:
        DA = _lib.DeviceArray
        phase("resident: uploading the batch to HBM")
        d = [DA.from_numpy(local, x) for x in (w.pub, w.sig, w.sig_off, w.sig_len, w.msg,
                                               w.msg_off, w.msg_len)]
        # one output set per in-flight pass: BH_F_ANY_LANE orders pass k + 4
        # after pass k (bdls_hip.cpp any_lane ring), so 4 rotating sets are safe
        outs_dev = [(DA(local, ((n + 63) // 64) * 8), DA(local, n)) for _ in range(MAX_LANES)]
        db = _lib.BhBatch(*[x.ptr for x in d])
        lane_flag = _lib.BH_F_ANY_LANE if a.resident_lanes else 0

        def step(k, f=flags | lane_flag):
            words, dreason = outs_dev[k % MAX_LANES]
            _lib.check(L.bh_verify_dev(local, 0, ctypes.byref(db), n, f, words.ptr,
                                       dreason.ptr, None, 0, None))
        phase("resident: warmup passes")
        for k in range(max(1, a.warmup)):
            step(k)
        _lib.check(L.bh_sync(local))
        dist.barrier(world)
        phase(f"resident: {a.steps} timed passes")
        r0 = time.perf_counter()
        for k in range(a.steps):
            step(k)
        _lib.check(L.bh_sync(local))
        r1 = time.perf_counter()
        phase(f"resident: {(r1 - r0) * 1e3 / a.steps:.2f} ms per pass")
        r_el = dist.max_over_ranks(r1 - r0, world)
        r_ok = True
        for words, dreason in outs_dev[:min(MAX_LANES, a.steps)]:
            rbits = np.unpackbits(words.to_numpy(np.uint64, (n + 63) // 64).view(np.uint8),
                                  bitorder="little")[:n].astype(bool)
            r_ok = r_ok and bool((dreason.to_numpy(np.uint8, n) == w.reason).all()
                                 and (rbits == w.expected_valid).all())
        # the per-kernel timing passes (serialised, not part of `value`)
        phase(f"resident: {a.steps} serialised passes (per-kernel HIP-event times)")
        _lib.check(L.bh_timing_begin(local))
        t_t0 = time.perf_counter()
        for k in range(a.steps):
            step(k, flags)
        _lib.check(L.bh_sync(local))
        t_el = time.perf_counter() - t_t0
        _lib.check(L.bh_timing_end(local, ctypes.byref(tm)))
        phase("resident: done")
        parity_ok = parity_ok and r_ok
        resident = {"value": round(dist.sum_over_ranks(n, world) * a.steps / r_el, 1),
                    "ms_per_step": round(r_el * 1e3 / a.steps, 3), "parity": r_ok,
                    "lanes": lane_count() if a.resident_lanes else 1,
                    "serialised_ms_per_step": round(t_el * 1e3 / a.steps, 3)}
        for x in d + [y for pair in outs_dev for y in pair]:
            x.free()
    parity_ok = dist.all_true(parity_ok, world)
    if e2e:
        # what bounds it: the longest per-batch stage of the three that overlap
        pb = e2e["per_batch_ms"]
        if resident:
            pb["gpu_resident"] = resident["ms_per_step"]
        e2e["bound"] = max(pb, key=pb.get)
    kern = {k: getattr(tm, k) for k in _lib.BhTiming.STAGES}
    routes = {"keycomb": tm.n_keycomb, "ladder": tm.n_ladder, "key_tables": tm.n_keytables}

    total = dist.sum_over_ranks(n, world) * a.steps
    host_value = total / elapsed
    host_ms_per_step = elapsed * 1e3 / a.steps
    # `value` is the whole-job rate with the inputs already resident in HBM
    # when the timed region starts (the bench contract); the PCIe-inclusive
    # host-API rate SURVEY 8(d) also names is reported beside it (host_path)
    if resident:
        value, ms_per_step = resident["value"], resident["ms_per_step"]
    else:
        value, ms_per_step = host_value, host_ms_per_step
    peak, peak_src = (a.mac_peak, "--mac-peak") if a.mac_peak else mac_peak_default()
    # dominant kernel of the step and its algorithmic work per launch
    dom = max(KERNELS, key=lambda k: kern[k])
    # the library verifies a shard in passes of <= 4M records (equal-sized
    # here); kern sums every launch, routes count the last pass
    passes = max(1, -(-n // (1 << 22)))
    dom_avg_s = kern[dom] * 1e-3 / (a.steps * passes)
    fp_ops = kernel_fp_ops(dom, routes)
    achieved = fp_ops * MAC_PER_FP / dom_avg_s if dom_avg_s > 0 else 0.0
    kname = KERNELS[dom]
    out = {
        "metric": "P-256 ECDSA verifies/sec (fused SHA-256, bit-exact vs Go crypto/ecdsa + Fabric low-S)",
        "value": round(value, 1),
        "unit": "verifies/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (seeded P-256 keys/signatures, workload/gen.c)",
        "config": {
            "workload": desc,
            "records_per_gpu": n, "records_total": dist.sum_over_ranks(n, world),
            "msg_len": a.msg_len, "nkeys": nkeys, "corrupt_den": corrupt,
            "parallelism": f"shard{world} (no collective)",
            "value_is": ("HBM-resident: bh_verify_dev passes over inputs already in device "
                         "memory (one pass = one step; consecutive passes rotate over the "
                         "compute lanes, BH_F_ANY_LANE), barrier + device sync around the "
                         "timed steps" if resident else
                         "host C ABI BatchVerify (bh_verify_submit/wait) from page-locked host "
                         "buffers: H2D + verify + results to page-locked memory per step (--hbm-resident 0)"),
        },
        "parity": parity_ok,
        "hbm_resident": resident,
        "host_path": {"value": round(host_value, 1), "ms_per_step": round(host_ms_per_step, 3),
                      "what": (("host C ABI BatchVerify (bh_verify_compact_submit / "
                                "bh_verify_wait, the compact bh_cbatch layout: distinct keys "
                                "+ u32 indices, lengths only) " if compact else
                                "host C ABI BatchVerify (bh_verify_submit/wait, bh_batch) ")
                               + "from page-locked host buffers: H2D + verify + results to page-locked memory per step, "
                               "batches in flight over the compute lanes (SURVEY 8(d)'s "
                               "config-2 timed quantity, PCIe-inclusive)"),
                      "layout": layout,
                      "layout_build_s": round(layout_s, 3) if compact else None,
                      "layout_note": ("the bh_cbatch arrays (np.unique key dedup + signature "
                                      "repack) are built once before the timed region; a Go "
                                      "caller pays that per BatchVerify (layout_build_s)"
                                      if compact else "the generator's arrays as they are"),
                      "single_batch_ms": round(single_ms, 3), "batch_bytes": batch_bytes,
                      "h2d_gbps_pinned": round(h2d_gbps, 2),
                      # the host path's own roofline: every batch crosses PCIe once
                      "pcie_bound_verifies_per_s": round(world * n * h2d_gbps * 1e9 / batch_bytes, 1),
                      "pcie_frac": round(host_value / (world * n * h2d_gbps * 1e9 / batch_bytes), 3),
                      "note": "value amortises the first batch's upload (pipeline fill) "
                              "over --steps batches"},
        "host_path_e2e": e2e,
        "kernel_ms_per_step": {k: round(v / a.steps, 3) for k, v in kern.items()},
        "kernel_ms_source": ("K serialised HBM-resident passes (bh_verify_dev, HIP events) run "
                             "after the timed ones" if a.hbm_resident
                             else "the timed host-path passes (compute lanes overlap)"),
        "routes": routes,
        "roofline": {
            "bound": "valu",
            "kernel": kname,
            "achieved": achieved / 1e12,
            "peak": peak / 1e12,
            "unit": "TMAC/s (u32 x u32 -> u64)",
            "frac": achieved / peak if peak else None,
            # the same work against the nominal VOP3 issue rate: 256 CUs x 4 SIMDs
            # x 16 lane-ops/cycle (a wave64 v_mad_u64_u32 every 4 cycles) x 2.4 GHz
            "peak_nominal": NOMINAL_MAC_PEAK / 1e12,
            "frac_nominal": achieved / NOMINAL_MAC_PEAK,
            "peak_nominal_source": "256 CU x 4 SIMD x 16 lane-ops/cycle (4-cycle VOP3) x 2.4 GHz "
                                   "(MI355X_MICROARCH.md peak clock)",
            "work_per_launch": (f"{routes['ladder']} ladder verifies x {FP_LADDER} + "
                                f"{routes['key_tables']} key tables x {FP_KTAB}"
                                + ("" if LL_TABLES else
                                   f" + {routes['keycomb']} u1 G halves x {FP_GPART}")
                                if dom == "build_ladder_ms" else
                                f"{routes['keycomb']} key-table verifies x {FP_KEYCOMB}"
                                + (" (u2 Q comb + folded u1 G)" if LL_TABLES else ""))
                               + f" F_p mul/sqr x {MAC_PER_FP} u32 MACs (SURVEY 8(d) units)",
            "fp_ops_per_launch": fp_ops,
            "launch_ms": round(dom_avg_s * 1e3, 4),
            "peak_source": peak_src,
            "traffic": None,
            "alg_bytes_per_record": alg_bytes_per_record(a.msg_len),
        },
        "gen_s": round(t_gen, 2),
        "workload_source": gen_info,
        "device": {"index": local, "why": dev_why},
    }
    # the whole step priced two ways: the F_p ops this engine actually runs
    # (key tables skip the S0 doublings), and SURVEY 8(d)'s fixed schedule S0
    # (3,200 F_p ops per verify whatever the route) -- the latter can exceed 1
    # because the algorithm does less work than S0, not because of a faster chip
    step_ops = (kernel_fp_ops("build_ladder_ms", routes) + kernel_fp_ops("keycomb_ms", routes)) \
        * passes
    rate = resident["value"] / world if resident else value / world
    step_s = n / rate
    out["roofline"]["whole_step"] = {
        "fp_ops_per_step": step_ops,
        "frac_of_peak": round(step_ops * MAC_PER_FP / step_s / peak, 4) if peak else None,
        "s0_schedule_frac": round(rate * FP_S0 * MAC_PER_FP / peak, 4) if peak else None,
        "note": "per GPU, HBM-resident step; s0_schedule_frac prices every verify at SURVEY "
                "8(d)'s 3,200 F_p ops (schedule S0)"}
    src, counters, stale = load_counters(a.config, n)
    hit = [v for k, v in counters.items() if k.startswith(kname + "<")]
    if stale:
        out["roofline"]["counters_refused"] = stale
    if hit:
        c = hit[0]
        if "bytes_per_launch" in c:
            out["roofline"]["traffic"] = c["bytes_per_launch"]
        if "sq_insts_valu" in c:
            out["roofline"]["valu_counters"] = {
                "sq_insts_valu_per_launch": c["sq_insts_valu"],
                "grbm_gui_active_per_launch": c["grbm_gui_active"],
                "formula": "SQ_INSTS_VALU x cyc / (GRBM_GUI_ACTIVE/8 XCDs x 256 CUs x 4 SIMDs)",
                "util_2cyc": c["valu_util_2cyc"],
                "util_4cyc": c["valu_util_4cyc"],
                "sq_active_inst_valu_per_launch": c.get("sq_active_inst_valu"),
                "valu_busy": c.get("valu_busy"),
                "valu_busy_formula": "rocprof VALUBusy: SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x "
                                     "GRBM_GUI_ACTIVE/8 XCDs)",
                "cost_model": ("2cyc: a wave64 VALU instruction occupies a SIMD-32 for 2 cycles "
                               "(MI355X_MICROARCH.md:54); 4cyc: one wave's issue rate and the "
                               "measured v_mad_u64_u32 / u32-add rate (profiles/ubench.json: "
                               "13-16 lane-ops/cycle/SIMD)"),
                "source": src,
            }

    if rank == 0 and world == 1 and a.cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(a, w, n)
        out["cpu_baseline"]["full_host_extrapolation"] = round(
            out["cpu_baseline"]["per_thread"] * out["cpu_baseline"]["host_cpus"]["nproc"], 1)
        out["cpu_baseline"]["gpu_vs_full_host"] = round(
            value / out["cpu_baseline"]["full_host_extrapolation"], 2)
    if world == 1 and a.config == 2 and a.side_configs:
        # configs 1, 3, 4 and the single Verify, driver-observed in the same line
        out["side_configs"] = side_configs(a, L, rank)
        side_ok = all(v.get("parity", True) for v in out["side_configs"].values()
                      if isinstance(v, dict))
        out["parity"] = parity_ok = bool(parity_ok and side_ok)
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.finalize(world)
    return 0 if parity_ok else 3


def config1_measure(steps: int, gpu: bool = True) -> dict:
    """BASELINE config 1: 10k synthetic P-256 verifies through bccsp/sw on the
    host CPU (go test -bench, plumbing, no GPU). No Go toolchain exists here or
    on the GPU box, so the measured figure is the labelled proxy SURVEY 8(d)
    prescribes: oracle/orc.c (Fabric's DER + low-S rules in C, the ECDSA core in
    OpenSSL's P-256 assembly -- the class of Go's crypto/internal/nistec asm)
    at 1 thread, every usable CPU and os.cpu_count() threads. 10,000 records,
    1,000 keys, SHA-256 digests of 256-byte messages, all valid, seed 1. The
    same batch through the engine is reported beside it (one bh_verify call,
    host buffers, digests given as in bccsp.Verify)."""
    import hashlib
    from bdls_amd import _lib, workload
    from oracle import orc
    w = workload.generate(10_000, 1_000, 256, 0, seed=1)
    dg = np.frombuffer(b"".join(hashlib.sha256(bytes(w.msg[o:o + l])).digest()
                                for o, l in zip(w.msg_off, w.msg_len)), np.uint8)
    doff = np.arange(w.n, dtype=np.uint64) * 32
    dlen = np.full(w.n, 32, np.uint32)
    cpus = host_cpus()
    usable = int(min(cpus.get("affinity", cpus["nproc"]),
                     cpus.get("cgroup_quota_cpus", cpus["nproc"]))) or 1
    runs, ok = {}, True
    for threads in sorted({1, usable, cpus["nproc"]}):
        best = 0.0
        for _ in range(max(1, steps)):
            t = time.perf_counter()
            got = orc.batch_verify(w.pub.reshape(-1, 64), dg, doff, dlen, w.sig, w.sig_off,
                                   w.sig_len, fused=False, nthreads=threads)
            best = max(best, w.n / (time.perf_counter() - t))
        ok = ok and bool((got == 0).all())
        runs[str(threads)] = round(best, 1)
    top = max(runs, key=lambda k: runs[k])
    out = {"value": runs[top], "unit": "verifies/s", "threads": int(top), "by_threads": runs,
           "per_thread": runs["1"], "full_host_extrapolation": round(runs["1"] * cpus["nproc"], 1),
           "host_cpus": cpus, "kind": "port (no Go toolchain: OpenSSL-backed restatement of "
                                      "bccsp/sw Verify, labelled proxy per SURVEY 8(d))",
           "parity": ok}
    if gpu:  # the same 10k records through the engine (digest mode)
        try:
            _lib.check(_lib.lib().bh_init(1, 0))
            b = _lib.BhBatch(w.pub.ctypes.data, w.sig.ctypes.data, w.sig_off.ctypes.data,
                             w.sig_len.ctypes.data, dg.ctypes.data, doff.ctypes.data,
                             dlen.ctypes.data)
            bm = np.zeros((w.n + 7) // 8, np.uint8)
            rs = np.zeros(w.n, np.uint8)
            ms = []
            for _ in range(max(3, steps)):
                t = time.perf_counter()
                _lib.check(_lib.lib().bh_verify(0, ctypes.byref(b), w.n, 0, bm.ctypes.data,
                                                rs.ctypes.data))
                ms.append((time.perf_counter() - t) * 1e3)
            out["gpu_same_batch"] = {"p50_ms": round(percentile(ms, 50), 4),
                                     "verifies_per_s": round(w.n / percentile(ms, 50) * 1e3, 1),
                                     "parity": bool((rs == 0).all())}
            out["parity"] = ok and out["gpu_same_batch"]["parity"]
        except _lib.EngineError as e:
            out["gpu_same_batch"] = {"skipped": str(e)}
    return out


def bench_config1(a):
    c = config1_measure(a.steps)
    out = {
        "metric": "P-256 ECDSA verifies/sec, host CPU (bccsp/sw proxy)",
        "value": c["value"], "unit": "verifies/s", "n_gpus": 0, "steps": a.steps,
        "warmup": 0, "ms_per_step": round(10_000 / c["value"] * 1e3, 3), "higher_is_better": True,
        "scaling": "none", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic (seeded P-256 keys/signatures, workload/gen.c)",
        "config": {"workload": "BASELINE config 1: 10,000 P-256 records, 1,000 keys, SHA-256 "
                               "digests of 256 B messages, all valid, seed 1", "kind": c["kind"]},
        "cpu": {k: c[k] for k in ("threads", "by_threads", "per_thread",
                                  "full_host_extrapolation", "host_cpus")},
        "gpu_same_batch": c.get("gpu_same_batch"),
        "parity": c["parity"],
    }
    print(json.dumps(out), flush=True)
    return 0


def single_verify_measure(L, threads_list=(1, 8, 64, 256)) -> dict:
    """The drop-in single BCCSP.Verify (bh_csp_verify_p256, the coalescer;
    bccsp/sw/impl.go:247-270 as msp/identities.go:190 calls it): per-call
    latency p50 / p99 and throughput at 1 .. 256 concurrent callers, driven by
    the native load generator (bdls_amd/lib/csp_load: pthreads, as Go's
    validator goroutines call Verify) in a child process. cold = the device
    has never seen the keys (the coalescer registers each key on its first
    sighting, the MSP-identity-cache analog); registered = registered before
    timing. The CPU proxy of one call beside it."""
    import hashlib
    import subprocess
    import tempfile
    from bdls_amd import workload
    from oracle import orc
    w = workload.generate(4096, 64, 256, 0, seed=11)
    recs = []
    for i in range(w.n):
        sig = bytes(w.sig[int(w.sig_off[i]):int(w.sig_off[i]) + int(w.sig_len[i])])
        dg = hashlib.sha256(bytes(w.msg[int(w.msg_off[i]):int(w.msg_off[i]) + int(w.msg_len[i])]))
        recs.append(bytes(w.pub[64 * i:64 * i + 64]) + dg.digest() + bytes([len(sig)]) + sig)
    tool = os.path.join(ROOT, "bdls_amd", "lib", "csp_load")
    out, ok = {}, True
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(b"".join(recs))
        path = f.name
    try:
        for mode in ("cold", "registered"):
            for nth in threads_list:
                per = max(16, min(400, 8192 // nth))
                r = subprocess.run([tool, path, str(nth), str(per), "1" if mode == "registered" else "0"],
                                   capture_output=True, text=True, timeout=120)
                if r.returncode not in (0, 1) or not r.stdout.strip():
                    out[f"{mode}_{nth}thr"] = {"error": r.stderr[-300:]}
                    ok = False
                    continue
                res = json.loads(r.stdout.strip().splitlines()[-1])
                ok = ok and res["bad"] == 0
                out[f"{mode}_{nth}thr"] = res
        # the same 256 registered callers confined to the CPUs the cgroup
        # quota grants (csp_load's cpus argument: the cpuset of a peer pinned
        # to its CPU limit). Unconfined, their wake-ups cost ~48 us of system
        # time each on a 256-CPU box and can trip the quota.
        cpus = host_cpus()
        usable = int(min(cpus.get("affinity", cpus["nproc"]),
                         cpus.get("cgroup_quota_cpus", cpus["nproc"]))) or 1
        if 256 in threads_list and usable < cpus.get("affinity", cpus["nproc"]):
            r = subprocess.run([tool, path, "256", str(max(16, min(400, 8192 // 256))), "1",
                                str(usable)], capture_output=True, text=True, timeout=120)
            if r.returncode in (0, 1) and r.stdout.strip():
                res = json.loads(r.stdout.strip().splitlines()[-1])
                ok = ok and res["bad"] == 0
                out["registered_256thr_cpuset"] = res
    finally:
        os.unlink(path)
    m = 512
    rates = {}
    for nth in (1, 16):
        t = time.perf_counter()
        orc.batch_verify(w.pub[:64 * m].reshape(-1, 64), w.msg, w.msg_off[:m], w.msg_len[:m],
                         w.sig, w.sig_off[:m], w.sig_len[:m], fused=True, nthreads=nth)
        rates[nth] = m / (time.perf_counter() - t)
    out["cpu_proxy"] = {"one_call_us_1thr": round(1e6 / rates[1], 1),
                        "verifies_per_s_1thr": round(rates[1], 1),
                        "verifies_per_s_16thr": round(rates[16], 1)}
    # The crossover the Go provider routes on (HIPOpts.
    # MinInflight): at c concurrent callers the embedded sw provider does
    # min(c, usable CPUs) x its one-core rate; the device path is the
    # registered-key coalescer rate. Below the first c where the device wins,
    # lone calls stay on sw.
    cpus = host_cpus()
    usable = int(min(cpus.get("affinity", cpus["nproc"]),
                     cpus.get("cgroup_quota_cpus", cpus["nproc"]))) or 1
    cmp_ = {}
    for nth in threads_list:
        g = out.get(f"registered_{nth}thr", {}).get("verifies_per_s")
        if g:
            cmp_[str(nth)] = {"device": g, "sw_proxy": round(min(nth, usable) * rates[1], 1)}
    wins = [int(k) for k, v in cmp_.items() if v["device"] > v["sw_proxy"]]
    out["crossover"] = {"by_callers": cmp_, "usable_cpus": usable,
                        "min_inflight": min(wins) if wins else None,
                        "note": "sw_proxy = min(callers, usable CPUs) x the one-core OpenSSL "
                                "rate; the Go provider sends calls to the device only at or "
                                "above min_inflight concurrent callers"}
    out["parity"] = ok
    return out


def config5_rank_measure(L, local: int, n: int = 1 << 20, steps: int = 3, gen_threads: int = 16):
    """VERDICT r3 missing #1 on the driver's line: config 5's per-rank work on
    one GPU -- the first 1,048,576 records of rank 0's shard of the seeded
    67,108,864-record unique-key batch (workload.generate_shard: record i is a
    function of (seed 5, i), the same records an 8-GPU run gives rank 0) --
    every key distinct, so every verify is a variable-base ladder (no key
    tables). Host path (bh_verify_submit/wait from page-locked buffers, two in
    flight) and HBM-resident (bh_verify_dev) rates over `steps` passes each,
    route counts and parity. Generation is timed separately."""
    from bdls_amd import _lib, workload
    pinned = []

    def alloc(nbytes):
        h = _lib.HostArray(nbytes)
        pinned.append(h)
        return h.u8
    t = time.perf_counter()
    w = workload.generate_shard(CONFIG5_TOTAL, 0, n, CONFIG5_TOTAL, 256, 64, seed=5,
                                nthreads=gen_threads, alloc=alloc)
    gen_s = time.perf_counter() - t
    flags = _lib.BH_F_HASH_SHA256
    hb = _lib.BhBatch(*[x.ctypes.data for x in w.arrays()])
    outs = [(np.zeros((n + 7) // 8, np.uint8), np.zeros(n, np.uint8)) for _ in range(2)]

    def submit(k):
        job = ctypes.c_void_p()
        bm, rs = outs[k % 2]
        _lib.check(L.bh_verify_submit(0, ctypes.byref(hb), n, flags, bm.ctypes.data,
                                      rs.ctypes.data, ctypes.byref(job)))
        return job
    _lib.check(L.bh_verify_wait(submit(0)))  # warmup
    t = time.perf_counter()
    jobs = [submit(0)]
    for k in range(1, steps):
        jobs.append(submit(k))
        _lib.check(L.bh_verify_wait(jobs.pop(0)))
    _lib.check(L.bh_verify_wait(jobs.pop(0)))
    host_s = time.perf_counter() - t
    bm, rs = outs[(steps - 1) % 2]
    ok = bool((rs == w.reason).all() and (np.unpackbits(bm, bitorder="little")[:n].astype(bool)
                                            == w.expected_valid).all())
    DA = _lib.DeviceArray
    d = [DA.from_numpy(local, x) for x in w.arrays()]
    words, dreason = DA(local, ((n + 63) // 64) * 8), DA(local, n)
    db = _lib.BhBatch(*[x.ptr for x in d])
    tm = _lib.BhTiming()
    _lib.check(L.bh_verify_dev(local, 0, ctypes.byref(db), n, flags, words.ptr, dreason.ptr, None,
                               1, ctypes.byref(tm)))
    t = time.perf_counter()
    for _ in range(steps):
        _lib.check(L.bh_verify_dev(local, 0, ctypes.byref(db), n, flags, words.ptr, dreason.ptr,
                                   None, 0, None))
    _lib.check(L.bh_sync(local))
    dev_s = time.perf_counter() - t
    ok = ok and bool((dreason.to_numpy(np.uint8, n) == w.reason).all())
    for x in d + [words, dreason]:
        x.free()
    return {"records": n, "distinct_keys": n, "gen_s": round(gen_s, 2),
            "host_path_verifies_per_s": round(n * steps / host_s, 1),
            "hbm_resident_verifies_per_s": round(n * steps / dev_s, 1),
            "steps": steps,
            "routes": {"ladder": tm.n_ladder, "keycomb": tm.n_keycomb,
                       "key_tables": tm.n_keytables},
            "kernel_ms": {k: round(getattr(tm, k), 3) for k in _lib.BhTiming.STAGES},
            "workload": f"records [0, {n}) of rank 0's shard of config 5's seeded "
                        f"{CONFIG5_TOTAL}-record unique-key batch (seed 5, 256 B messages, "
                        f"1/64 corrupted, fused SHA-256)",
            "parity": ok}


def side_configs(a, L, rank) -> dict:
    """Configs 1, 3 and 4 and the single-Verify drop-in on the same box, in
    the default run (each a bounded measurement: ~10 s together)."""
    import types
    from bdls_amd import workload
    from oracle import orc
    sub = types.SimpleNamespace(**vars(a))
    sub.steps, sub.warmup, sub.seed = a.side_steps, 2, 3
    out = {}
    t0 = time.perf_counter()
    # config 3: the whole block through bh_fabric_block_preverify + the CPU proxy
    blk = measure_block(sub, L, rank)
    wb = workload.generate_block(seed=3)
    cpus = host_cpus()
    usable = int(min(cpus.get("affinity", cpus["nproc"]),
                     cpus.get("cgroup_quota_cpus", cpus["nproc"]))) or 1
    cpu = []
    for _ in range(5):
        t = time.perf_counter()
        got = orc.batch_verify(wb.pub.reshape(-1, 64), wb.msg, wb.msg_off, wb.msg_len, wb.sig,
                               wb.sig_off, wb.sig_len, fused=True, nthreads=usable)
        cpu.append((time.perf_counter() - t) * 1e3)
    blk["cpu_proxy_ms"] = {"p50": round(percentile(cpu, 50), 4), "threads": usable,
                           "sample": f"{wb.n} records of a config-3-shaped block, identity.Verify "
                                     "semantics (OpenSSL), signature checks only",
                           "parity": bool((got == wb.reason).all())}
    blk["parity"] = blk["parity"] and blk["cpu_proxy_ms"]["parity"]
    out["config3"] = blk
    # config 4: the wire round through bh_bdls_preverify + the serial CPU loop
    wire = measure_wire(sub, L, 1, rank)
    r = workload.generate_bdls_round(100, 1, seed=3)
    arrs = r.arrays()
    cpu = []
    for _ in range(3):
        t = time.perf_counter()
        got = orc.bdls_verify(1, *arrs)
        cpu.append((time.perf_counter() - t) * 1e3)
    wire["cpu_serial_ms"] = {"p50": round(percentile(cpu, 50), 4), "threads": 1,
                             "sample": f"{r.n} SignedProtos of a 100-validator round, "
                                       "BLAKE2b-256 + OpenSSL, serial as the agent loop runs",
                             "parity": bool((got == 0).all())}
    wire["parity"] = wire["parity"] and wire["cpu_serial_ms"]["parity"]
    out["config4"] = wire
    _lib_keys_clear(L)
    # config 1: the bccsp/sw proxy and the engine on the same 10k batch
    out["config1"] = config1_measure(max(1, a.side_steps // 10))
    # the coalesced single Verify
    out["single_verify"] = single_verify_measure(L)
    # config 5's per-rank shape (unique keys: the ladder)
    cpus = host_cpus()
    usable = int(min(cpus.get("affinity", cpus["nproc"]),
                     cpus.get("cgroup_quota_cpus", cpus["nproc"]))) or 1
    out["config5_rank"] = config5_rank_measure(L, 0, gen_threads=max(4, min(32, usable)))
    out["seconds"] = round(time.perf_counter() - t0, 2)
    return out


def _lib_keys_clear(L):
    from bdls_amd import _lib
    _lib.check(L.bh_keys_clear(-1, 0))
    _lib.check(L.bh_keys_clear(-1, 1))


def dry_run(a, rank, world):
    """Launcher + rank plumbing without a GPU (tests/test_bench_launch.py)."""
    from bdls_amd import dist
    dist.barrier(world)
    t = dist.max_over_ranks(0.001 * (rank + 1), world)
    ok = dist.all_true(True, world)
    lo, hi = dist.shard_range(a.n_total if a.config == 5 else a.n * world, rank, world)
    recs = dist.sum_over_ranks(hi - lo, world)
    torch_free = dist.all_true("torch" not in sys.modules, world)
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "config": a.config,
                          "records_total": recs, "max_t": t, "parity": ok,
                          "torch_free_ranks": torch_free}), flush=True)
    dist.finalize(world)
    return 0


def main(argv=None):
    a = parse(argv)
    from bdls_amd import dist
    if a.config == 1:
        return bench_config1(a)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(a.gpus)
    rank, world, local = dist.env_rank()
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}: launch with "
                         f"--nproc-per-node {a.gpus}, or drop the launcher")
    dist.init(world)
    if a.dry_run:
        return dry_run(a, rank, world)
    if a.config in (3, 4):
        return bench_latency(a, rank, world, local)
    return bench_throughput(a, rank, world, local)


if __name__ == "__main__":
    sys.exit(main())
