"""Multi-GPU orchestration for batch verification.

Records are independent, so the batch shards into contiguous per-rank ranges
with no data-path collective. The control the bench needs -- the barrier
around the timed region, the max-over-ranks time, the AND of per-rank parity,
the sum of records -- goes over a stdlib TCP channel on 127.0.0.1 with rank 0
as the hub (one node: the bench contract). torch is never imported: it bundles
its own HIP runtime (libamdhip64.so.7 of ROCm 7.0) under the same soname as the
/opt/rocm runtime libbdlship.so links, and a rank process that loaded it first
would bind the library to torch's copy.

Rendezvous: rank 0 listens on an ephemeral port and publishes "port nonce" in
a file; the other ranks read it, connect and present (nonce, rank, world).
The file lives in $BDLS_CTRL_DIR when the launcher set one (bench.py's own
spawner makes a fresh directory per run), else in the temp directory keyed by
the launcher's pid and MASTER_PORT (torch.distributed.run: every rank of one
job has the agent as parent). A rank that dies closes its socket, so the
others fail loudly instead of hanging.
"""
from __future__ import annotations

import json
import os
import secrets
import socket
import tempfile
import time

_CONNECT_TIMEOUT_S = float(os.environ.get("BDLS_CTRL_TIMEOUT", 600))
_st = None  # {"rank", "world", "conns" (rank 0: [None, sock1, ...]) / "hub" (rank > 0)}


def env_rank():
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


_VISIBLE_VARS = ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES",
                 "GPU_DEVICE_ORDINAL")


def visible_device_count(environ=None):
    """Devices a rank process may see when a launcher or scheduler narrowed
    them with a visibility variable (the smallest list among those set), or
    None when none is set (every device of the node is visible). Read from
    the environment only: counting through HIP would initialise the runtime
    before the rank has chosen its device."""
    env = os.environ if environ is None else environ
    counts = []
    for k in _VISIBLE_VARS:
        v = env.get(k)
        if v is None:
            continue
        items = [x for x in v.split(",") if x.strip() != ""]
        counts.append(len(items))
    return min(counts) if counts else None


def device_for_rank(local: int, environ=None):
    """(device index, why) for local rank `local`: the rank's own index when
    more than `local` devices are visible (the launcher left every GPU of the
    node visible: rank r drives GPU r), else device 0 (the launcher gave each
    rank exactly its own GPU, e.g. HIP_VISIBLE_DEVICES=<r>)."""
    vis = visible_device_count(environ)
    if vis is None:
        return local, "all devices visible: device = LOCAL_RANK"
    if vis > local:
        return local, f"{vis} devices visible: device = LOCAL_RANK"
    if vis <= 0:
        return 0, "visibility variable lists no device: device 0 (bh_init will fail loudly)"
    return 0, f"{vis} device(s) visible to this rank (LOCAL_RANK {local}): device 0"


def shard_range(n_total: int, rank: int, world: int, align: int = 64):
    """Contiguous [lo, hi) of rank in a batch of n_total records; boundaries are
    multiples of `align` so per-rank bitmap words concatenate without shifts."""
    per = -(-n_total // world)
    per = -(-per // align) * align
    lo = min(n_total, rank * per)
    hi = min(n_total, lo + per)
    return lo, hi


def _rdv_file() -> str:
    d = os.environ.get("BDLS_CTRL_DIR")
    if d:
        return os.path.join(d, "hub")
    return os.path.join(tempfile.gettempdir(),
                        f"bdls_ctrl_{os.getppid()}_{os.environ.get('MASTER_PORT', '0')}")


def _send(sock, obj):
    sock.sendall((json.dumps(obj) + "\n").encode())


def _recv(sock):
    buf = bytearray()
    while not buf.endswith(b"\n"):
        chunk = sock.recv(4096)
        if not chunk:
            raise RuntimeError("dist: a rank closed its control channel (did it fail?)")
        buf += chunk
    return json.loads(buf)


def init(world: int):
    global _st
    if world == 1 or _st is not None:
        return
    rank = env_rank()[0]
    path = _rdv_file()
    deadline = time.monotonic() + _CONNECT_TIMEOUT_S
    if rank == 0:
        srv = socket.create_server(("127.0.0.1", 0))
        nonce = secrets.token_hex(8)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "w") as f:
            f.write(f"{srv.getsockname()[1]} {nonce}\n")
        os.replace(tmp, path)
        conns = [None] * world
        try:
            while any(c is None for c in conns[1:]):
                srv.settimeout(max(0.1, deadline - time.monotonic()))
                try:
                    c, _ = srv.accept()
                except socket.timeout:
                    raise RuntimeError(f"dist: ranks {[r for r in range(1, world) if conns[r] is None]}"
                                       f" did not connect within {_CONNECT_TIMEOUT_S:.0f} s")
                c.settimeout(30)
                try:
                    hello = _recv(c)
                except (OSError, ValueError, RuntimeError):
                    c.close()
                    continue
                r = hello.get("rank", -1)
                if hello.get("nonce") != nonce or hello.get("world") != world or not 0 < r < world \
                        or conns[r] is not None:
                    c.close()
                    continue
                c.settimeout(None)
                conns[r] = c
        finally:
            srv.close()
            try:
                os.unlink(path)
            except OSError:
                pass
        for c in conns[1:]:
            _send(c, {"ok": True})
        _st = {"rank": 0, "world": world, "conns": conns}
        return
    while True:
        if time.monotonic() > deadline:
            raise RuntimeError(f"dist: rank {rank} found no hub at {path} within "
                               f"{_CONNECT_TIMEOUT_S:.0f} s")
        try:
            with open(path) as f:
                port, nonce = f.read().split()
            s = socket.create_connection(("127.0.0.1", int(port)), timeout=30)
        except (OSError, ValueError):
            time.sleep(0.05)
            continue
        try:
            _send(s, {"nonce": nonce, "rank": rank, "world": world})
            if _recv(s).get("ok"):
                s.settimeout(None)
                _st = {"rank": rank, "world": world, "hub": s}
                return
        except (OSError, ValueError, RuntimeError):
            pass
        s.close()
        time.sleep(0.05)


def _allreduce(x, op):
    """Every rank's x reduced by op (a function of a list) at rank 0 and
    returned to all ranks."""
    if _st is None:
        raise RuntimeError("dist.init(world) was not called")
    if _st["rank"] == 0:
        vals = [x] + [_recv(c)["v"] for c in _st["conns"][1:]]
        out = op(vals)
        for c in _st["conns"][1:]:
            _send(c, {"v": out})
        return out
    _send(_st["hub"], {"v": x})
    return _recv(_st["hub"])["v"]


def barrier(world: int):
    if world > 1:
        _allreduce(0, lambda v: 0)


def max_over_ranks(x: float, world: int) -> float:
    return x if world == 1 else float(_allreduce(float(x), max))


def all_true(ok: bool, world: int) -> bool:
    return ok if world == 1 else bool(_allreduce(bool(ok), all))


def sum_over_ranks(x: int, world: int) -> int:
    return x if world == 1 else int(_allreduce(int(x), sum))


def finalize(world: int):
    global _st
    if world == 1 or _st is None:
        return
    barrier(world)
    for s in ([_st.get("hub")] + (_st.get("conns") or [])):
        if s is not None:
            s.close()
    _st = None
