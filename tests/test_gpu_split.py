"""One hashgraph split across GPUs (babble_amd/dist.py) must give
exactly the single-GPU replay -- order, batches, rounds, witnesses, fame, round
received, timestamps, LastConsensusRound, the undetermined list.

* walk-only split, single process: the walkers of G "ranks" run one after the
  other on one engine (the real kernels and join, no collective);
* sharded split (hge_split_plan / hge_split_run): G parts, one engine and host
  thread each on the one GPU of the box, exchanging through device memory
  (ThreadExchange): each part decides its rounds' fame and its calls' order;
* two processes on the one GPU, over gloo (the real torch.distributed path,
  world_size 2), each with its own engine and the whole stream.
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
    """The walk-only split (dist.walk_split_run) with G walkers on one engine."""
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


def compare_state(ref, eng, order, counts, o2, c2):
    np.testing.assert_array_equal(o2, order)
    np.testing.assert_array_equal(c2, counts)
    assert eng.rounds() == ref.rounds()
    r1, w1 = ref.event_rounds()
    r2, w2 = eng.event_rounds()
    np.testing.assert_array_equal(r2, r1)
    np.testing.assert_array_equal(w2, w1)
    np.testing.assert_array_equal(eng.fame_table(), ref.fame_table())
    rr1, ct1 = ref.event_received()
    rr2, ct2 = eng.event_received()
    np.testing.assert_array_equal(rr2[order], rr1[order])
    np.testing.assert_array_equal(ct2[order], ct1[order])
    assert eng.last_consensus_round() == ref.last_consensus_round()
    assert eng.consensus_transactions() == ref.consensus_transactions()
    np.testing.assert_array_equal(eng.undetermined(), ref.undetermined())


def run_parts(engs, G, halo_rounds):
    """The G parts of a sharded split replay, one host thread per engine."""
    import threading
    from babble_amd.dist import ThreadExchange, split_run
    xg = ThreadExchange(G)
    res, stats = [None] * G, [{} for _ in range(G)]

    def run(p):
        try:
            res[p] = split_run(engs[p], p, G, xg.make(p), halo_rounds, stats[p])
        except BaseException as e:  # noqa: BLE001 -- release the other parts
            res[p] = e
            xg.bar.abort()

    ths = [threading.Thread(target=run, args=(p,)) for p in range(G)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=300)
    for r in res:
        if isinstance(r, BaseException):
            raise r
    return res, stats


@pytest.mark.parametrize("n,E,G,halo,fallback", [
    (64, 60_000, 3, 8, False),
    (128, 80_000, 2, 4, False),
    (64, 40_000, 4, 8, False),
    (256, 60_000, 3, 8, False),
    (64, 30_000, 2, 0, True),   # no candidate halo: events received late are nobody's -> unsplit replay
])
def test_sharded_split_equals_replay(n, E, G, halo, fallback):
    from babble_amd.engine import Engine, events_array
    dag = random_gossip(n, E, seed=170 + n + G)
    ev = events_array(dag)
    calls = schedule(E, n)
    ref = Engine(n, E + 64)
    engs = [Engine(n, E + 64) for _ in range(G)]
    try:
        _, order, counts = ref.replay(ev, calls)
        for e in engs:
            e.prepare(ev, calls)
        res, stats = run_parts(engs, G, halo)
        assert all(r == len(order) for r in res)
        assert any(s.get("fallback", 0) for s in stats) == fallback, stats
        for e in engs:
            _, o2, c2 = e.fetch()
            compare_state(ref, e, order, counts, o2, c2)
        # a second replay of the same engines (buffers reused) gives the same again
        res, _ = run_parts(engs, G, halo)
        for e in engs:
            _, o2, c2 = e.fetch()
            np.testing.assert_array_equal(o2, order)
    finally:
        ref.close()
        for e in engs:
            e.close()


def test_sharded_split_on_golden():
    """The sharded split against the oracle's golden (64 participants, 100k events)."""
    from babble_amd.engine import Engine, events_array
    dag, g = load_golden(os.path.join(ROOT, "tests", "golden", "wide_n64_e100000_k64.npz"))
    n, G = int(g["n"]), 3
    engs = [Engine(n, len(dag["creator"]) + 64) for _ in range(G)]
    try:
        for e in engs:
            e.prepare(events_array(dag), g["calls"])
        _, stats = run_parts(engs, G, 8)
        assert not any(s.get("fallback", 0) for s in stats)
        for e in engs:
            _, order, counts = e.fetch()
            np.testing.assert_array_equal(order, g["order"])
            np.testing.assert_array_equal(counts, g["counts"])
            rounds, wit = e.event_rounds()
            np.testing.assert_array_equal(rounds, g["rounds"])
    finally:
        for e in engs:
            e.close()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, q):
    import torch.distributed as dist
    from babble_amd.dist import TorchExchange, split_run
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
    stats = {}
    split_run(eng, rank, world, TorchExchange(dist, "cuda:0"), 8, stats)
    _, order, counts = eng.fetch()
    ref = Engine(n, E + 64, device=0)
    _, rorder, rcounts = ref.replay(ev, calls)
    q.put((rank, bool(np.array_equal(order, rorder) and np.array_equal(counts, rcounts)) and not stats,
           len(order), len(rorder), stats))
    eng.close()
    ref.close()
    dist.destroy_process_group()


def test_sharded_split_two_ranks_gloo_one_gpu():
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


@pytest.mark.parametrize("n,E,G", [(64, 40_000, 3), (256, 40_000, 2)])
def test_sharded_split_emulated_parts(n, E, G):
    """hge_split_emulate: one engine records an unsplit replay, then runs every part
    of a G-way split alone (the other parts' exchange slots from the record); every
    part ends with the replay's state (the measurement path of
    scripts/analysis/split_emulate.py)."""
    from babble_amd.dist import ROUND_EVENTS_PER_PARTICIPANT, split_plan
    from babble_amd.engine import Engine, events_array
    dag = random_gossip(n, E, seed=270 + n)
    ev = events_array(dag)
    calls = schedule(E, n)
    ref = Engine(n, E + 64)
    eng = Engine(n, E + 64)
    try:
        _, order, counts = ref.replay(ev, calls)
        eng.prepare(ev, calls)
        eng.split_emulate(True)
        eng.run()
        plan = split_plan(eng.call_events(), eng.event_count(), G, 8 * ROUND_EVENTS_PER_PARTICIPANT * n)
        for p in range(G):
            eng.split_plan(p, G, plan)
            eng.clear_exchange()
            assert eng.split_run() == len(order)
            _, o2, c2 = eng.fetch()
            compare_state(ref, eng, order, counts, o2, c2)
    finally:
        ref.close()
        eng.close()


def _nccl_world1(port, q):
    import torch
    import torch.distributed as dist
    from babble_amd.dist import TorchExchange, split_run
    from babble_amd.engine import Engine, events_array
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda:0"))
    out = {"slots": []}
    try:
        x = TorchExchange(dist, "cuda:0")
        out["nccl"] = x.nccl
        # op 0 / op 1 as the engine calls them (hge_split_exchange): the slot comes back
        # unchanged through all_gather_into_tensor; a larger exchange regrows the buffer
        for nbytes, seed in ((4096, 1), (1 << 20, 2), (4096, 3)):
            p = x(0, nbytes)
            g = torch.Generator(device="cuda:0").manual_seed(seed)
            want = torch.randint(0, 256, (nbytes,), generator=g, device="cuda:0").to(torch.uint8)
            torch.cuda.synchronize()
            x.buf[:nbytes].copy_(want)
            torch.cuda.synchronize()
            assert x(1, nbytes) is None
            out["slots"].append(p == x.buf.data_ptr() and bool(torch.equal(x.buf[:nbytes], want)))
        # a world of one: split_run replays unsplit with the exchange installed
        n, E = 64, 12_000
        dag = random_gossip(n, E, seed=93)
        ev = events_array(dag)
        calls = schedule(E, n)
        eng = Engine(n, E + 64, device=0)
        ref = Engine(n, E + 64, device=0)
        try:
            eng.prepare(ev, calls)
            stats = {}
            split_run(eng, 0, 1, x, 8, stats)
            _, order, counts = eng.fetch()
            _, rorder, rcounts = ref.replay(ev, calls)
            out["equal"] = bool(np.array_equal(order, rorder) and np.array_equal(counts, rcounts))
            out["stats"] = stats
        finally:
            eng.close()
            ref.close()
    except Exception as e:  # reported to the parent
        out["error"] = repr(e)
    finally:
        dist.destroy_process_group()
    q.put(out)


def test_torch_exchange_nccl_world_one():
    """TorchExchange on a world-size-1 "nccl" (RCCL) group: op 0 hands out the slot
    buffer and op 1 runs all_gather_into_tensor -- the branch the multi-GPU bench's
    split replay takes -- at two sizes (the buffer regrows), then split_run with the
    exchange installed equals the one-GPU replay."""
    import torch.multiprocessing as mp
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_world1, args=(port, q))
    p.start()
    out = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert "error" not in out, out
    assert out["nccl"] and out["slots"] == [True, True, True], out
    assert out["equal"] and not out["stats"], out
