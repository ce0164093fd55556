"""Config 5 on the GPU: many independent 32-participant hashgraphs with
Byzantine forkers (and fork cascades).  The batch engine (hge_batch_*, what
bench.py --workload mc times) replays all 1,024 graphs of the bench's batch and
every graph's full state must equal the oracle's committed digest; the
single-graph engines, driven by host threads, are checked on a smaller batch."""
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from babble_amd.gossip import random_gossip, schedule
from oracle.oracle import replay as oracle_replay

pytestmark = pytest.mark.gpu


def test_monte_carlo_batch_threads():
    from babble_amd.engine import Engine, events_array
    graphs, threads, n, events, k = 64, 8, 32, 1500, 32
    dags = [random_gossip(n, events, seed=5000 + g, forkers=10, fork_p=0.05, cascade_p=0.5)
            for g in range(graphs)]
    engines = [Engine(n, len(d["creator"]) + 64) for d in dags]
    try:
        for e, d in zip(engines, dags):
            e.prepare(events_array(d), schedule(len(d["creator"]), k))

        def run(i):
            engines[i].run()
            engines[i].run()  # a second replay on the same staged events: same result
            return engines[i].fetch()

        with ThreadPoolExecutor(threads) as pool:
            got = list(pool.map(run, range(graphs)))
            want = list(pool.map(lambda d: oracle_replay(d, schedule(len(d["creator"]), k)), dags))
        rejected, codes = 0, set()
        for g, ((st, order, counts), (_, ost, oorder, ocounts)) in enumerate(zip(got, want)):
            np.testing.assert_array_equal(st, ost, err_msg=f"graph {g}: admission")
            np.testing.assert_array_equal(order, oorder, err_msg=f"graph {g}: order")
            np.testing.assert_array_equal(counts, ocounts, err_msg=f"graph {g}: batches")
            rejected += int((st < 0).sum())
            codes |= set(np.unique(st[st < 0]).tolist())
        assert rejected > graphs  # forks and cascades were generated and refused
        assert {-5, -4, -2} <= codes  # fork, op on a rejected event, child of a rejected event
    finally:
        for e in engines:
            e.close()


def test_monte_carlo_config5_batch_all_digests():
    """Config 5 at its stated size on the batch engine: all 1,024 graphs x 10k
    submissions of bench.py --workload mc in one batch, each graph's FULL state
    (status, order, batches, rounds, witnesses, fame, round received, timestamps,
    undetermined list, scalars) against the oracle digests committed in
    tests/golden/mc_n32_e10000_k32_digests.json, and 8 graphs against the oracle
    run live, field by field."""
    from babble_amd.engine import Batch
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    sys.path.insert(0, here)
    from digest import digest, first_difference
    from make_mc_digests import OUT, graph_stream, oracle_state
    ref = json.load(open(OUT))
    graphs = ref["graphs"]
    assert graphs == 1024
    streams = [graph_stream(g) for g in range(graphs)]
    b = Batch(32)
    try:
        for d, calls in streams:
            b.add(d, calls)
        tot = b.run()
        got = [b.state(g) for g in range(graphs)]
        bad = [g for g in range(graphs) if digest(got[g]) != ref["digests"][g]]
        assert not bad, f"graphs differing from the oracle digests: {bad[:16]}"
        assert tot == sum(ref["ordered"])
        assert sum(int((s["status"] < 0).sum()) for s in got) == sum(ref["rejected"])
        with ThreadPoolExecutor(8) as pool:
            live = list(pool.map(lambda g: oracle_state(*streams[g]), range(0, graphs, graphs // 8)))
        for j, g in enumerate(range(0, graphs, graphs // 8)):
            assert first_difference(got[g], live[j]) is None, f"graph {g}: {first_difference(got[g], live[j])}"
    finally:
        b.close()


def test_monte_carlo_config5_size():
    """Config 5's graphs on the single-graph engines: 256 of the batch's 1024 graphs
    x 10k submissions (graphs 0-255 of bench.py --workload mc), 8 host threads, each
    graph's FULL state (order, batches, rounds, witnesses, fame, round received,
    timestamps, undetermined list, scalars) against the oracle digests committed
    in tests/golden/mc_n32_e10000_k32_digests.json, and 8 graphs also against the
    oracle run live, field by field."""
    from babble_amd.engine import Engine, events_array
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    sys.path.insert(0, here)
    from digest import digest, engine_state, first_difference
    from make_mc_digests import OUT, graph_stream, oracle_state
    ref = json.load(open(OUT))
    graphs, threads = 256, 8
    streams = [graph_stream(g) for g in range(graphs)]
    engines = [Engine(32, len(d["creator"]) + 64) for d, _ in streams]
    try:
        for e, (d, calls) in zip(engines, streams):
            e.prepare(events_array(d), calls)

        def run(i):
            engines[i].run()
            st, order, counts = engines[i].fetch()
            return engine_state(engines[i], st, order, counts)

        with ThreadPoolExecutor(threads) as pool:
            got = list(pool.map(run, range(graphs)))
            live = list(pool.map(lambda g: oracle_state(*streams[g]), range(0, graphs, graphs // 8)))
        bad = [g for g in range(graphs) if digest(got[g]) != ref["digests"][g]]
        assert not bad, f"graphs differing from the oracle digests: {bad[:16]}"
        for j, g in enumerate(range(0, graphs, graphs // 8)):
            assert first_difference(got[g], live[j]) is None, f"graph {g}: {first_difference(got[g], live[j])}"
        assert sum(int((s["status"] < 0).sum()) for s in got) == sum(ref["rejected"][:graphs])
        assert sum(len(s["order"]) for s in got) == sum(ref["ordered"][:graphs])
    finally:
        for e in engines:
            e.close()
