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


# ---- one hashgraph split across ranks: the join of the walkers' rows ----------

def true_frontier(n, dag, k):
    """The rounds frontier C_r[c] (first chain-c position with round >= r; INT32_MAX
    = none) for every round, from the oracle's per-event rounds, plus the empty row."""
    import numpy as np
    from babble_amd.gossip import schedule
    from oracle.oracle import replay
    o, st, _, _ = replay(dag, schedule(len(dag["creator"]), k))
    E = int((st >= 0).sum())
    rounds = np.array([o.round(x) for x in range(E)])
    R = int(rounds.max()) + 1
    INF = np.iinfo(np.int32).max
    C = np.full((R + 1, n), INF, np.int32)
    for x in range(E - 1, -1, -1):  # ids are insertion order: the last write is the first event
        c, p = int(dag["creator"][x]), int(dag["index"][x])
        for r in range(rounds[x] + 1):
            if C[r, c] == INF or p < C[r, c]:
                C[r, c] = p
    return C


def _marks(rows, tag):
    import numpy as np
    n, N = rows.shape
    return (np.arange(n, dtype=np.uint64)[:, None, None] * 1000 + tag).repeat(N, 1).repeat(1, 2)


def test_join_histories_follows_merges():
    import numpy as np
    from babble_amd.dist import join_histories
    from babble_amd.gossip import random_gossip
    n = 6
    C = true_frontier(n, random_gossip(n, 3000, seed=31), n)
    R = len(C) - 1
    assert R > 40
    rng = np.random.default_rng(1)
    junk = C[20:24] + rng.integers(1, 3, (4, n)).astype(np.int32)  # a guessed start converging
    h0 = (C[:30].copy(), None, False)                  # rank 0: true rows 0..29, then stopped
    r1 = np.concatenate([junk, C[25:]])                # rank 1: 4 wrong rows, then true 25..R
    h1 = (r1, None, True)
    hists = [(h0[0], _marks(h0[0], 0), False), (h1[0], _marks(h1[0], 1), True)]
    rows, ssc, natural = join_histories(hists)
    assert natural and len(rows) == R
    np.testing.assert_array_equal(rows, C[:R])
    # rows 0..25 come from rank 0 (row 25 is where the walk hands over), 26.. from rank 1
    assert (ssc[:26, 0, 0] % 1000 == 0).all() and (ssc[26:, 0, 0] % 1000 == 1).all()
    assert ssc[26, 0, 0] // 1000 == 4 + 1               # rank 1's row of round 26
    # no overlap: the join stops at rank 0's last row (the sequential walk resumes there)
    rows, _, natural = join_histories([(C[:20].copy(), _marks(C[:20], 0), False),
                                       (r1, _marks(r1, 1), True)])
    assert not natural and len(rows) == 20
    # a single rank that walked to the end
    rows, _, natural = join_histories([(C.copy(), _marks(C, 0), True)])
    assert natural and len(rows) == R


def test_join_histories_three_walkers_overlapping():
    """Walker p runs past walker p + 1's start, so rows of the true trajectory are
    in both: the join must move on to the furthest walker holding a row (1 -> 2
    here), not stop at the end of walker 1's history."""
    import numpy as np
    from babble_amd.dist import join_histories
    from babble_amd.gossip import random_gossip
    n = 6
    C = true_frontier(n, random_gossip(n, 4000, seed=32), n)
    R = len(C) - 1
    assert R > 70
    rng = np.random.default_rng(2)
    j1 = C[20:23] + rng.integers(1, 3, (3, n)).astype(np.int32)
    j2 = C[40:43] + rng.integers(1, 3, (3, n)).astype(np.int32)
    h = [C[:30].copy(),                      # rank 0: true rows 0..29
         np.concatenate([j1, C[25:60]]),     # rank 1: converges at 25, walks past rank 2's merge
         np.concatenate([j2, C[45:]])]       # rank 2: converges at 45, walks to the end
    hists = [(r, _marks(r, g), g == 2) for g, r in enumerate(h)]
    rows, ssc, natural = join_histories(hists)
    assert natural and len(rows) == R
    np.testing.assert_array_equal(rows, C[:R])
    # rank 0 up to its hand-over row 25, rank 1 up to 45, rank 2 after
    tags = ssc[:, 0, 0] % 1000
    assert (tags[:26] == 0).all() and (tags[26:46] == 1).all() and (tags[46:] == 2).all()


def _gather_worker(rank, world, port, q):
    import numpy as np
    import torch.distributed as dist
    from babble_amd.dist import torch_gather
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 5 + 3 * rank
    rows = np.full((n, 8), rank, np.int32)
    ssc = np.full((n, 8, 1), 10 + rank, np.uint64)
    out = torch_gather(dist)((rows, ssc, rank == 1))
    q.put((rank, [(r.shape, int(r[0, 0]), s.shape, int(s[0, 0, 0]), nat) for r, s, nat in out]))
    dist.destroy_process_group()


def test_world2_gloo_history_gather():
    """The split's one collective (babble_amd.dist.torch_gather) with world_size 2."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp = [((5, 8), 0, (5, 8, 1), 10, False), ((8, 8), 1, (8, 8, 1), 11, True)]
    assert out[0][1] == exp and out[1][1] == exp


# ---- one hashgraph sharded by time (split_plan) -----------------
@pytest.mark.parametrize("world,ncalls,K,tail", [(2, 10, 64, 0), (3, 100, 256, 17), (8, 39063, 256, 128),
                                                  (4, 4, 16, 0)])
def test_split_plan_covers_the_stream(world, ncalls, K, tail):
    """Parts own disjoint call ranges and event ranges that tile the stream; the
    candidate halo stays inside it; the last part ends at E."""
    import numpy as np
    from babble_amd.dist import split_plan
    calls = K * np.arange(1, ncalls + 1, dtype=np.int64)
    E = int(calls[-1]) + tail
    plan = split_plan(calls, E, world, 3 * K)
    ev, cb, clo = plan["ev_bounds"], plan["call_bounds"], plan["cand_lo"]
    assert ev[0] == 0 and ev[-1] == E and cb[0] == 0 and cb[-1] == ncalls
    for g in range(world):
        assert cb[g + 1] > cb[g] and ev[g + 1] > ev[g]
        # a part's events are those inserted during its calls
        if g > 0:
            assert ev[g] == calls[cb[g] - 1]
        if g < world - 1:
            assert ev[g + 1] == calls[cb[g + 1] - 1]
        assert clo[g] == max(0, ev[g] - 3 * K) and clo[g] <= ev[g]
    # call shares differ by at most one
    sizes = np.diff(cb)
    assert sizes.max() - sizes.min() <= 1
    with pytest.raises(ValueError):
        split_plan(calls[:1], E, 2, 0)


def _exchange_worker(rank, world, port, q):
    import ctypes

    import numpy as np
    import torch.distributed as dist
    from babble_amd.dist import TorchExchange
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ex = TorchExchange(dist, "cpu")
    out = []
    for nbytes in (16, 1000, 64):  # the engine's op 0 / op 1 sequence, sizes varying
        ptr = ex(0, nbytes)
        slot = np.ctypeslib.as_array((ctypes.c_uint8 * (nbytes * world)).from_address(ptr))
        slot[rank * nbytes:(rank + 1) * nbytes] = (rank + 1) * 7 % 256
        ex(1, nbytes)
        out.append([int(slot[g * nbytes]) for g in range(world)] + [int(slot[(g + 1) * nbytes - 1]) for g in range(world)])
    q.put((rank, out))
    dist.destroy_process_group()


def test_world2_gloo_engine_exchange():
    """The engine's all-gather (hge_split_exchange) over torch.distributed: op 0
    hands out the slots' memory, op 1 leaves every rank's slot in every buffer."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp = [[7, 14, 7, 14]] * 3
    assert out[0][1] == exp and out[1][1] == exp
