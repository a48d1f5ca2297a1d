"""CPU: bench.py's multi-GPU launcher. `--gpus N` without torch.distributed.run
spawns N ranks itself (no GPU is touched in --dry-run) and reports n_gpus: N;
a rank count that disagrees with --gpus fails loudly."""
import json
import os
import subprocess
import sys

from tests.conftest import ROOT


def _run(args, env=None):
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=e,
                          capture_output=True, text=True, timeout=300)


def test_gpus2_spawns_two_ranks():
    r = _run(["--gpus", "2", "--dry-run"])
    assert r.returncode == 0, r.stderr
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    assert lines[0]["n_gpus"] == 2 and lines[0]["dry_run"] and lines[0]["parity"]
    assert lines[0]["records_total"] == 2 * (1 << 20)
    assert lines[0]["torch_free_ranks"]  # no rank process imported torch


def test_torch_distributed_run_launcher():
    """The driver's N>1 launch: python -m torch.distributed.run ... bench.py
    --gpus 2 (the ranks come from the environment; the control channel keys its
    rendezvous on the agent's pid and MASTER_PORT)."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "BDLS_CTRL_DIR"):
        e.pop(k, None)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                        str(port), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run",
                        "--config", "5"], env=e, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["n_gpus"] == 2 and out["records_total"] == 1 << 26 and out["torch_free_ranks"]


def test_config5_is_one_batch_split_over_ranks():
    r = _run(["--gpus", "2", "--dry-run", "--config", "5"])
    assert r.returncode == 0, r.stderr
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["records_total"] == 1 << 26


def test_world_mismatch_fails():
    r = _run(["--gpus", "2", "--dry-run"], env={"WORLD_SIZE": "1", "RANK": "0",
                                                "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr
