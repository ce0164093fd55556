"""One hashgraph split across GPUs (babble_amd/dist.py): the
rounds walk by several walkers from different starts, joined by row equality,
must give exactly the single-GPU replay -- order, batches, rounds, witnesses.

* single process: the walkers of G "ranks" run one after the other on one
  engine (the real kernels and join, no collective);
* two processes on the one GPU of the box, over gloo (the real collective
  path, world_size 2), each with its own engine and the whole stream.
"""
import os
import socket

import numpy as np
import pytest

from babble_amd.gossip import random_gossip, schedule
from parity import compare_golden, load_golden

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def walk_all(eng, G, extra):
    from babble_amd.dist import join_histories
    eng.split_begin()
    hists = []
    for p in range(G):
        start = eng.frontier_guess(p, G)
        stop = eng.frontier_guess(p + 1, G) if p + 1 < G else None
        hists.append(eng.frontier_walk(start, stop, extra if stop is not None else 0))
    rows, ssc, natural = join_histories(hists)
    return eng.split_finish(rows, ssc, natural), hists, natural


@pytest.mark.parametrize("n,E,G,extra", [(64, 40_000, 2, 256), (64, 40_000, 4, 256), (128, 60_000, 3, 200),
                                         (64, 40_000, 4, 0)])
def test_split_equals_replay(n, E, G, extra):
    from babble_amd.engine import Engine, events_array
    dag = random_gossip(n, E, seed=70 + n + G)
    ev = events_array(dag)
    calls = schedule(E, n)
    ref = Engine(n, E + 64)
    eng = Engine(n, E + 64)
    try:
        st, order, counts = ref.replay(ev, calls)
        eng.prepare(ev, calls)
        nord, hists, natural = walk_all(eng, G, extra)
        _, o2, c2 = eng.fetch()
        assert nord == len(order)
        np.testing.assert_array_equal(o2, order)
        np.testing.assert_array_equal(c2, counts)
        assert eng.rounds() == ref.rounds()
        r1, w1 = ref.event_rounds()
        r2, w2 = eng.event_rounds()
        np.testing.assert_array_equal(r2, r1)
        np.testing.assert_array_equal(w2, w1)
        # the later walkers started mid-way (rank 0 may walk to the end when the
        # overlap `extra` reaches past the last round)
        assert all(len(h[0]) < ref.rounds() for h in hists[1:])
    finally:
        ref.close()
        eng.close()


def test_split_on_golden():
    from babble_amd.engine import Engine, events_array
    dag, g = load_golden(os.path.join(ROOT, "tests", "golden", "wide_n64_e100000_k64.npz"))
    eng = Engine(int(g["n"]), len(dag["creator"]) + 64)
    try:
        eng.prepare(events_array(dag), g["calls"])
        walk_all(eng, 4, 256)
        _, order, counts = eng.fetch()
        np.testing.assert_array_equal(order, g["order"])
        np.testing.assert_array_equal(counts, g["counts"])
        rounds, wit = eng.event_rounds()
        np.testing.assert_array_equal(rounds, g["rounds"])
    finally:
        eng.close()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, q):
    import torch.distributed as dist
    from babble_amd.dist import split_run, torch_gather
    from babble_amd.engine import Engine, events_array
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, E = 64, 30_000
    dag = random_gossip(n, E, seed=91)
    ev = events_array(dag)
    calls = schedule(E, n)
    eng = Engine(n, E + 64, device=0)
    eng.prepare(ev, calls)
    split_run(eng, rank, world, torch_gather(dist))
    _, order, counts = eng.fetch()
    ref = Engine(n, E + 64, device=0)
    _, rorder, rcounts = ref.replay(ev, calls)
    q.put((rank, bool(np.array_equal(order, rorder) and np.array_equal(counts, rcounts)), len(order)))
    eng.close()
    ref.close()
    dist.destroy_process_group()


def test_split_two_ranks_gloo_one_gpu():
    import torch.multiprocessing as mp
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=200) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[0][1] and out[1][1], out
    assert out[0][2] == out[1][2] > 0
