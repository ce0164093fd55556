"""Config 5 on the GPU: many independent 32-participant hashgraphs with
Byzantine forkers (and fork cascades), one engine (HIP stream) each, driven
concurrently by host threads on one device -- the shape bench.py --workload mc
times.  Every graph is compared bit-exact with the oracle."""
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
