"""The batch engine (hge_batch_*, hge_batch.hip: many independent hashgraphs, one
launch per stage) against the oracle, field by field: admission status, order,
per-call batches, every event's round and witness flag, the fame of every
(round, creator) slot, round received, consensus timestamps, the undetermined
list and the scalars (tests/golden/digest.py's state).

The graphs cover N from 1 to 64, forkers and fork cascades (every admission
error), call schedules from K = 1 to one call for the whole stream (a batch
past the LDS sort, the global-scratch path), other-parents that are not their
chain's head (op_lag), coin rounds (N = 4 one-shot), and a second run of the
same batch.  The call schedule runs in bulk (hge_batch_bulk.hip); a graph past
the bulk fold's 256 rounds is replayed call by call by kb_consensus in the same
run, and HGB_SERIAL=1 puts every graph through kb_consensus."""
import os
import sys

import numpy as np
import pytest

from babble_amd.gossip import random_gossip, schedule

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

CASES = [
    # n, events, k, seed, forkers, fork_p, cascade_p, op_lag
    (4, 1000, 4, 1, 0, 0.0, 0.0, 0),
    (4, 1000, 1, 2, 0, 0.0, 0.0, 0),
    (4, 1500, 1500, 12, 0, 0.0, 0.0, 0),     # one call: coin rounds, a 1.4k-key batch (global sort)
    (1, 50, 5, 3, 0, 0.0, 0.0, 0),
    (1, 700, 5, 5, 0, 0.0, 0.0, 0),          # ~700 rounds: past the bulk fold, replayed by kb_consensus
    (2, 300, 2, 3, 0, 0.0, 0.0, 0),
    (5, 2000, 3, 13, 0, 0.0, 0.0, 0),
    (7, 3000, 7, 14, 2, 0.1, 0.5, 0),
    (16, 3000, 16, 2, 0, 0.0, 0.0, 0),
    (16, 4000, 50, 21, 0, 0.0, 0.0, 6),      # other-parents behind their chain's head
    (32, 3000, 32, 4, 10, 0.05, 0.5, 0),     # config 5's graph shape with cascades
    (32, 4000, 32, 16, 10, 0.05, 0.0, 0),
    (32, 2500, 2500, 22, 0, 0.0, 0.0, 0),    # one call at N = 32
    (32, 5000, 700, 25, 0, 0.0, 0.0, 0),     # 513-1,024-key batches: the LDS sort pads to 1,024
    (16, 4000, 900, 26, 2, 0.05, 0.5, 0),
    (33, 3000, 50, 17, 0, 0.0, 0.0, 3),
    (48, 5000, 48, 23, 5, 0.05, 0.5, 0),
    (64, 6000, 64, 18, 0, 0.0, 0.0, 0),
    (64, 3000, 7, 24, 0, 0.0, 0.0, 2),
]


def _stream(n, E, k, seed, fk, fp, cp, lag):
    dag = random_gossip(n, E, seed=seed, forkers=fk, fork_p=fp, cascade_p=cp, op_lag=lag)
    return dag, schedule(len(dag["creator"]), k)


@pytest.mark.parametrize("n", sorted({c[0] for c in CASES}))
def test_batch_matches_oracle(n):
    from babble_amd.engine import Batch
    from digest import first_difference
    from make_mc_digests import oracle_state
    cases = [c for c in CASES if c[0] == n]
    streams = [_stream(*c) for c in cases]
    b = Batch(n)
    try:
        for dag, calls in streams:
            b.add(dag, calls)
        tot = b.run()
        want = [oracle_state(dag, calls) for dag, calls in streams]
        assert tot == sum(len(w["order"]) for w in want)
        for rep in range(2):  # a second replay of the staged batch gives the same state
            for g, (case, w) in enumerate(zip(cases, want)):
                got = b.state(g)
                diff = first_difference(got, w)
                assert diff is None, f"case {case}: first differing field {diff}"
            if rep == 0:
                b.run()
    finally:
        b.close()


def test_batch_many_graphs_one_launch_per_stage():
    """256 graphs of config 5's shape in one batch, each equal to the oracle."""
    from babble_amd.engine import Batch
    from digest import first_difference
    from make_mc_digests import oracle_state
    streams = [_stream(32, 1200, 32, 7000 + g, 10, 0.05, 0.5, 0) for g in range(256)]
    b = Batch(32)
    try:
        for dag, calls in streams:
            b.add(dag, calls)
        b.run()
        ms = b.kernel_ms()
        assert set(ms) == {"kb_coords", "kb_fd", "kb_fdrows", "kb_front", "kb_fame", "kb_fold", "kb_receive",
                           "kb_order"}
        assert b.fallbacks() == 0  # every graph in bulk
        for g in range(0, 256, 5):
            w = oracle_state(*streams[g])
            assert first_difference(b.state(g), w) is None, f"graph {g}"
    finally:
        b.close()


def test_batch_refuses_bad_arguments():
    from babble_amd.engine import Batch, HgeError
    with pytest.raises(HgeError):
        Batch(65)
    b = Batch(4)
    try:
        dag, _ = _stream(4, 100, 4, 1, 0, 0.0, 0.0, 0)
        with pytest.raises(HgeError):
            b.add(dag, np.array([5, 3], np.int64))  # not ascending
        with pytest.raises(HgeError):
            b.info(0)  # no graph yet
    finally:
        b.close()


@pytest.mark.parametrize("n", [4, 32, 64])
def test_batch_serial_path_matches_oracle(n, monkeypatch):
    """HGB_SERIAL=1: every graph through the call-by-call kb_consensus (the bulk
    path's fallback), against the oracle."""
    from babble_amd.engine import Batch
    from digest import first_difference
    from make_mc_digests import oracle_state
    monkeypatch.setenv("HGB_SERIAL", "1")
    cases = [c for c in CASES if c[0] == n]
    streams = [_stream(*c) for c in cases]
    b = Batch(n)
    try:
        for dag, calls in streams:
            b.add(dag, calls)
        b.run()
        assert b.fallbacks() == len(cases)
        for g, (case, (dag, calls)) in enumerate(zip(cases, streams)):
            diff = first_difference(b.state(g), oracle_state(dag, calls))
            assert diff is None, f"case {case}: first differing field {diff}"
    finally:
        b.close()


def test_batch_fallback_mixed_with_bulk():
    """One batch holding a graph past the bulk fold (N = 1, ~700 rounds) and bulk
    graphs: only that graph is replayed by kb_consensus, all equal the oracle."""
    from babble_amd.engine import Batch
    from digest import first_difference
    from make_mc_digests import oracle_state
    cases = [c for c in CASES if c[0] == 1]
    streams = [_stream(*c) for c in cases]
    b = Batch(1)
    try:
        for dag, calls in streams:
            b.add(dag, calls)
        b.run()
        assert b.fallbacks() == 1
        for g, (case, (dag, calls)) in enumerate(zip(cases, streams)):
            assert first_difference(b.state(g), oracle_state(dag, calls)) is None, f"case {case}"
    finally:
        b.close()
