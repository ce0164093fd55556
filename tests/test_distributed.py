"""The multi-GPU driver logic (bench.py --gpus N, Monte Carlo sharding) with
world_size 2 over gloo on the CPU: every rank gets a disjoint share of the
independent hashgraphs, and the whole-job line combines max step time and the
sum of ordered events.  (The data path has no collective: SURVEY.md §8e.)"""
import os
import socket

import pytest
import torch.multiprocessing as mp

from babble_amd.dist import reduce_step, shard_range


@pytest.mark.parametrize("total,world", [(1024, 8), (1024, 3), (5, 8), (7, 2), (0, 2)])
def test_shard_range_partitions(total, world):
    seen = []
    for r in range(world):
        first, count = shard_range(total, world, r)
        seen.extend(range(first, first + count))
        assert count in (total // world, total // world + 1)
    assert seen == list(range(total))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, count = shard_range(1024, world, rank)
    step = 0.010 + 0.005 * rank          # rank 1 is the slow one
    ordered = 1000 * count + rank
    q.put((rank, first, count) + reduce_step(dist, step, ordered))
    dist.destroy_process_group()


def test_world2_gloo_reduction():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [o[1:3] for o in out] == [(0, 512), (512, 512)]
    for _, _, _, max_step, tot in out:
        assert abs(max_step - 0.015) < 1e-12       # max over ranks
        assert tot == 1000 * 1024 + 1               # sum over ranks
