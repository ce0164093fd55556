"""Sweep coordinates at small N against the live oracle, and the wide online
path against the bulk replay (the wide goldens are in test_gpu_golden.py)."""
import numpy as np
import pytest

from babble_amd.gossip import random_gossip
from parity import run_case

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,events,k", [(4, 1000, 4), (16, 3000, 16), (16, 3000, 1), (32, 4000, 32),
                                        (7, 2000, 50)])
def test_sweep_coordinates_small_n(n, events, k):
    """Sweeps + transposes at small N (several sweep groups, K from 1 to 50) vs the live oracle."""
    from babble_amd.engine import Engine
    eng = Engine(n, 1 << 14)
    try:
        run_case(eng, random_gossip(n, events, seed=400 + n + k), k)
    finally:
        eng.close()


def test_wide_online_matches_replay():
    """N=64 through the online API (one batch per RunConsensus) equals the bulk replay."""
    from babble_amd.engine import Engine, events_array
    from babble_amd.gossip import schedule
    n, E, k = 64, 3000, 64
    dag = random_gossip(n, E, seed=21)
    calls = schedule(E, k)
    a = Engine(n, 1 << 13)
    b = Engine(n, 1 << 13)
    try:
        _, order, _ = a.replay(dag, calls)
        ev = events_array(dag)
        nxt = 0
        for c in calls:
            b.insert_events(ev[nxt:c].copy())
            b.run_consensus()
            nxt = c
        np.testing.assert_array_equal(b.consensus_events(), order)
        assert b.rounds() == a.rounds()
    finally:
        a.close()
        b.close()


def _np_coords(dag, n):
    """lastAncestors rows (insertion order) and a firstDescendants lookup, numpy."""
    cr = np.asarray(dag["creator"], np.int64)
    ix = np.asarray(dag["index"], np.int64)
    sp = np.asarray(dag["sp"], np.int64)
    op = np.asarray(dag["op"], np.int64)
    E = len(cr)
    LA = np.full((E, n), -1, np.int32)
    for x in range(E):
        row = LA[sp[x]].copy() if sp[x] >= 0 else np.full(n, -1, np.int32)
        if op[x] >= 0:
            np.maximum(row, LA[op[x]], out=row)
        row[cr[x]] = ix[x]
        LA[x] = row
    chains = [np.flatnonzero(cr == j) for j in range(n)]  # positions in insertion order

    def fd(x):
        c, i = cr[x], ix[x]
        out = np.full(n, np.iinfo(np.int32).max, np.int64)
        for j in range(n):
            col = LA[chains[j], c]  # non-decreasing along chain j
            k = int(np.searchsorted(col, i, "left"))
            if k < len(col):
                out[j] = k
        return out
    return LA, fd


def test_wide256_fd_rows_online_and_growth():
    """N=256 (FD rows built straight from LAT, k_fd_rows): the online path with a
    small starting capacity (the chain tables grow, LAT keeps its old positions)
    equals the bulk replay, and sampled coordinates equal a numpy restatement of
    InitEventCoordinates / UpdateAncestorFirstDescendant (hashgraph.go:399-494)."""
    from babble_amd.engine import Engine, events_array
    from babble_amd.gossip import schedule
    n, E, k = 256, 12_000, 256
    dag = random_gossip(n, E, seed=77)
    calls = schedule(E, k)
    a = Engine(n, E + 64)
    b = Engine(n, 1024)
    try:
        _, order, _ = a.replay(dag, calls)
        ev = events_array(dag)
        nxt = 0
        for c in calls:
            b.insert_events(ev[nxt:c].copy())
            b.run_consensus()
            nxt = c
        np.testing.assert_array_equal(b.consensus_events(), order)
        assert b.rounds() == a.rounds()
        LA, fd = _np_coords(dag, n)
        rng = np.random.default_rng(3)
        for x in rng.choice(E, 40, replace=False).tolist() + [0, E - 1]:
            for eng in (a, b):
                gla, gfd = eng.coordinates(int(x))
                np.testing.assert_array_equal(gla, LA[x])
                np.testing.assert_array_equal(np.asarray(gfd, np.int64), fd(x))
    finally:
        a.close()
        b.close()


@pytest.mark.parametrize("n,events,G", [(64, 6000, 8), (256, 5000, 5), (128, 6000, 3)])
def test_stale_other_parents_in_windows(n, events, G, monkeypatch):
    """Other-parents that are not their chain's head when the event is inserted (a
    node inserting events it learned late; `op_lag`) are the windowed lastAncestors
    kernels' "risky" path: read from HBM, chunk-level store drains, no early exit
    past them.  Forced into several windows (HGE_LW_G), compared with the oracle."""
    from babble_amd.engine import Engine
    monkeypatch.setenv("HGE_LW_G", str(G))
    dag = random_gossip(n, events, seed=77 + n, op_lag=4)
    eng = Engine(n, 1 << 14)
    try:
        run_case(eng, dag, n)
        LA, fd = _np_coords(dag, n)
        rng = np.random.default_rng(5)
        for x in rng.choice(events, 30, replace=False).tolist() + [events - 1]:
            gla, gfd = eng.coordinates(int(x))
            np.testing.assert_array_equal(gla, LA[x])
            np.testing.assert_array_equal(np.asarray(gfd, np.int64), fd(x))
    finally:
        eng.close()


@pytest.mark.parametrize("n,events", [(32, 4000), (64, 6000)])
def test_timestamp_offsets_outside_int32(n, events):
    """The wide median reads the FD timestamps as int32 offsets from each event's own
    timestamp; rows whose offsets do not fit (clocks 3 s apart every 500 events here)
    are flagged per 64-column tile and gathered exactly.  Consensus timestamps and
    order vs the oracle (MedianTimestamp, hashgraph.go:762-770)."""
    from babble_amd.engine import Engine
    dag = random_gossip(n, events, seed=90 + n)
    dag["ts"] = dag["ts"] + (np.arange(events, dtype=np.int64) // 500) * 3_000_000_000
    eng = Engine(n, 1 << 14)
    try:
        run_case(eng, dag, n)
    finally:
        eng.close()


@pytest.mark.parametrize("n,events,kind", [(64, 5000, "spread"), (256, 3000, "spread"),
                                           (64, 5000, "ties"), (128, 4000, "ties")])
def test_median_select_extremes(n, events, kind):
    """The 32-bit select on timestamp offsets at its edges: timestamps out of order
    and spread over +-2^30 ns (offsets up to +-(2^31 - 2): spans close to 2^32, the
    order-preserving images near 1 and 2^32 - 1), and long runs of equal timestamps
    (ties: the select runs every bit without isolating a single value).  Consensus
    timestamps and order vs the oracle (MedianTimestamp, hashgraph.go:762-770)."""
    from babble_amd.engine import Engine
    dag = random_gossip(n, events, seed=300 + n)
    if kind == "spread":
        rng = np.random.default_rng(n)
        dag["ts"] = 1_700_000_000_000_000_000 + rng.integers(-(1 << 30) + 1, 1 << 30, events, dtype=np.int64)
    else:
        dag["ts"] = 1_700_000_000_000_000_000 + (np.arange(events, dtype=np.int64) // 97) * 1000
    eng = Engine(n, 1 << 14)
    try:
        run_case(eng, dag, n)
    finally:
        eng.close()


@pytest.mark.parametrize("n,events", [(128, 16000), (256, 12000), (64, 20000), (4, 20000)])
def test_oversized_call_buckets(n, events):
    """One RunConsensus over the whole stream: a single FindOrder call bucket of more
    than 8,192 keys, sorted by k_bucket_sort_all (one call: both sort paths in one
    launch).  128/16k and 256/12k (8,193 .. 16,384 keys): two halves sorted in LDS
    and merged; 64/20k and 4/20k (more than 16,384 keys): the chunk sort + merges,
    here by a 1024-thread block.  Order and consensus state vs the oracle
    (FindOrder, hashgraph.go:744-745)."""
    from babble_amd.engine import Engine
    eng = Engine(n, 1 << 15)
    try:
        run_case(eng, random_gossip(n, events, seed=500 + n), events)
    finally:
        eng.close()


def test_two_wide_engines_concurrently():
    """Two N > 32 engines replaying at the same time from two host threads on one
    device: their frontier grids (one co-resident 1024-thread workgroup per
    chain) are serialised inside the process, so neither waits on workgroups
    the other holds; both results equal the sequential replays."""
    from concurrent.futures import ThreadPoolExecutor
    from babble_amd.engine import Engine
    from babble_amd.gossip import schedule
    cases = [(128, 12_000, 128, 61), (256, 20_000, 256, 62)]
    dags = [random_gossip(n, E, seed=s) for n, E, _, s in cases]
    engines = [Engine(n, E) for n, E, _, _ in cases]
    try:
        want = [e.replay(d, schedule(len(d["creator"]), k))[1] for e, d, (_, _, k, _) in zip(engines, dags, cases)]

        def run(i):
            out = None
            for _ in range(3):
                out = engines[i].replay(dags[i], schedule(len(dags[i]["creator"]), cases[i][2]))[1]
            return out

        with ThreadPoolExecutor(2) as pool:
            got = list(pool.map(run, range(2)))
        for g, w in zip(got, want):
            np.testing.assert_array_equal(g, w)
    finally:
        for e in engines:
            e.close()


@pytest.mark.parametrize("n,events,k", [(64, 4000, 16), (128, 6000, 1)])
def test_handoff_timeout_falls_back_per_round(n, events, k, monkeypatch):
    """A wide walk whose frontier hand-off times out (forced: HGE_TEST_HANDOFF_FAIL
    makes the walk report the timeout after it ran) walks again one launch per round
    (k_round_step32) and keeps that walk; the results equal the oracle's."""
    from babble_amd.engine import Engine
    monkeypatch.setenv("HGE_TEST_HANDOFF_FAIL", "1")
    eng = Engine(n, 1 << 14)
    try:
        run_case(eng, random_gossip(n, events, seed=900 + n), k)
        assert eng.frontier_fallbacks() == 1
    finally:
        eng.close()


def test_handoff_timeout_online_path(monkeypatch):
    """The fallback in the middle of an online run (one RunConsensus per batch): the
    rows of the batch are recomputed from the rounds it started with."""
    from babble_amd.engine import Engine, events_array
    from babble_amd.gossip import schedule
    n, E, k = 64, 3000, 12
    dag = random_gossip(n, E, seed=31)
    calls = schedule(E, k)
    a = Engine(n, 1 << 13)
    b = Engine(n, 1 << 13)
    try:
        _, order, _ = a.replay(dag, calls)
        ev = events_array(dag)
        nxt = 0
        for q, c in enumerate(calls):
            if q == 5:
                monkeypatch.setenv("HGE_TEST_HANDOFF_FAIL", "1")
            b.insert_events(ev[nxt:c].copy())
            b.run_consensus()
            nxt = c
        assert b.frontier_fallbacks() == 1
        np.testing.assert_array_equal(b.consensus_events(), order)
        assert b.rounds() == a.rounds()
        assert a.frontier_fallbacks() == 0
    finally:
        a.close()
        b.close()


@pytest.mark.parametrize("n,events,k,epoch", [(64, 4000, 16, 3), (128, 6000, 1, 2)])
def test_handoff_stall_mid_walk(n, events, k, epoch, monkeypatch):
    """A walk that gives up part-way (HGE_TEST_HANDOFF_STALL: at hand-off `epoch`
    chain 0 never publishes and every workgroup stops as on a timed-out poll), so
    that round's row is written for every chain but chain 0: the launch-per-round
    walk takes over from the rows as left (kept rows stand, missing ones are
    computed) and the results equal the oracle's."""
    from babble_amd.engine import Engine
    monkeypatch.setenv("HGE_TEST_HANDOFF_STALL", str(epoch))
    eng = Engine(n, 1 << 14)
    try:
        run_case(eng, random_gossip(n, events, seed=950 + n), k)
        assert eng.frontier_fallbacks() == 1
    finally:
        eng.close()


@pytest.mark.parametrize("n,events", [(16, 3000), (32, 11000)])
def test_coin_rounds_wide_one_shot(n, events):
    """One RunConsensus over a whole stream long enough that DecideFame's j loop
    reaches diff = N (hashgraph.go:645-649, the coin branch) at N = 16 and N = 32:
    the engine equals the live oracle field by field, and the oracle's statistics
    show the coin branch taken."""
    from babble_amd.engine import Engine
    eng = Engine(n, events + 64)
    try:
        o, _ = run_case(eng, random_gossip(n, events, seed=78 if n == 32 else 77), events)
        assert o.stats()["coin_evals"] > 0
    finally:
        eng.close()
