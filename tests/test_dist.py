"""CPU: the multi-GPU control path (bdls_amd/dist.py) with world_size 2 over
gloo on 127.0.0.1, and the shard arithmetic bench.py / bh_verify rely on."""
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


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init(world)
    dist.barrier(world)
    t = dist.max_over_ranks(0.5 + rank, world)
    ok = dist.all_true(rank == 0, world)
    tot = dist.sum_over_ranks(10 * (rank + 1), world)
    lo, hi = dist.shard_range(1000, rank, world)
    dist.finalize(world)
    q.put((rank, t, ok, tot, lo, hi))


def test_gloo_world2():
    pytest.importorskip("torch.distributed")
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    [p.start() for p in ps]
    res = sorted(q.get(timeout=120) for _ in ps)
    [p.join(timeout=60) for p in ps]
    assert [r[1] for r in res] == [1.5, 1.5]        # max over ranks
    assert [r[2] for r in res] == [False, False]    # parity AND
    assert [r[3] for r in res] == [30, 30]
    assert res[0][4:] == (0, 512) and res[1][4:] == (512, 1000)
