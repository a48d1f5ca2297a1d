"""CPU: the multi-GPU control path (bdls_amd/dist.py: a stdlib socket channel on
127.0.0.1, rank 0 the hub, no torch) at world sizes 2 and 4, and the shard
arithmetic bench.py / bh_verify rely on."""
import os
import socket

import pytest

from bdls_amd import dist


def test_shard_ranges_cover_and_align():
    for n in (1, 63, 64, 65, 1000, 1 << 20, (1 << 20) + 7):
        for world in (1, 2, 3, 4, 8):
            spans = [dist.shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (lo, hi), (lo2, _) in zip(spans, spans[1:]):
                assert hi == lo2
            for lo, _ in spans:
                assert lo % 64 == 0 or lo == n


@pytest.mark.parametrize("env,local,want", [
    ({}, 0, 0), ({}, 5, 5),                                        # nothing narrowed
    ({"HIP_VISIBLE_DEVICES": "3"}, 3, 0),                          # one GPU per rank
    ({"HIP_VISIBLE_DEVICES": "3"}, 0, 0),
    ({"HIP_VISIBLE_DEVICES": "0,1,2,3,4,5,6,7"}, 7, 7),            # all eight listed
    ({"ROCR_VISIBLE_DEVICES": "GPU-ab12"}, 6, 0),                  # UUID form, one device
    ({"HIP_VISIBLE_DEVICES": "0,1,2,3,4,5,6,7", "ROCR_VISIBLE_DEVICES": "4"}, 4, 0),
    ({"CUDA_VISIBLE_DEVICES": "0,1"}, 1, 1), ({"CUDA_VISIBLE_DEVICES": "0,1"}, 2, 0),
])
def test_device_for_rank(env, local, want):
    """a rank drives device LOCAL_RANK only when more than
    LOCAL_RANK devices are visible; a launcher that gives each rank its own GPU
    (a visibility list of length 1) maps every rank to device 0."""
    dev, why = dist.device_for_rank(local, env)
    assert dev == want, why
    assert dist.visible_device_count(env) == (None if not env else min(
        len(v.split(",")) for v in env.values()))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, ctrl, q):
    import sys
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if ctrl:
        os.environ["BDLS_CTRL_DIR"] = ctrl
    dist.init(world)
    dist.barrier(world)
    t = dist.max_over_ranks(0.5 + rank, world)
    ok = dist.all_true(rank == 0, world)
    tot = dist.sum_over_ranks(10 * (rank + 1), world)
    lo, hi = dist.shard_range(1000, rank, world)
    for _ in range(20):  # many collectives in a row keep their order
        dist.barrier(world)
    dist.finalize(world)
    q.put((rank, t, ok, tot, lo, hi, "torch" in sys.modules))


@pytest.mark.parametrize("world,ctrl_dir", [(2, True), (2, False), (4, True)])
def test_ctrl_channel(world, ctrl_dir, tmp_path):
    """world ranks in separate processes: barrier, max, AND, sum; with the
    launcher's rendezvous directory (bench.py's spawner) and without it (the
    temp-dir key a torch.distributed.run job uses); no rank imports torch."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ctrl = str(tmp_path) if ctrl_dir else ""
    ps = [ctx.Process(target=_worker, args=(r, world, port, ctrl, q)) for r in range(world)]
    [p.start() for p in ps]
    res = sorted(q.get(timeout=120) for _ in ps)
    [p.join(timeout=60) for p in ps]
    assert [r[1] for r in res] == [world - 0.5] * world       # max over ranks
    assert [r[2] for r in res] == [False] * world             # parity AND
    assert [r[3] for r in res] == [10 * world * (world + 1) // 2] * world
    spans = [r[4:6] for r in res]
    assert spans[0][0] == 0 and spans[-1][1] == 1000
    assert not any(r[6] for r in res)
    assert not os.listdir(tmp_path)  # the rendezvous file is gone


def test_ctrl_channel_dead_rank_fails_loudly(tmp_path):
    """A rank that never arrives makes the hub fail within the timeout."""
    import subprocess
    import sys
    code = ("import os; from bdls_amd import dist; dist.init(2)")
    env = dict(os.environ, RANK="0", WORLD_SIZE="2", LOCAL_RANK="0", BDLS_CTRL_DIR=str(tmp_path),
               BDLS_CTRL_TIMEOUT="2", PYTHONPATH=os.path.dirname(os.path.dirname(
                   os.path.abspath(__file__))))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=60)
    assert r.returncode != 0 and "did not connect" in r.stderr
