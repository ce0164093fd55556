"""Full-size configurations on the GPU (BASELINE.json configs[1] to configs[3] on
one MI355X, and the 32/1M and 128/1M lines of DESIGN.md §5): 16 participants /
100k events, 32 / 1M, 64 / 1M, 128 / 1M and 256 / 10M, K = N.

Parity is checked by
  * the oracle's digests of the WHOLE stream (tests/golden/*_full.json, made by
    tests/golden/make_bench_full.py with the oracle's scale mode): every field
    of the parity contract -- status, order, per-call batches, every event's
    round, witness flag, round received and consensus timestamp, the fame of
    every (round, creator) slot, the undetermined list and the scalars -- must
    hash identically; a mismatch names the first differing chunk;
  * the committed oracle golden of the first calls of the SAME stream
    (tests/golden/bench_*_prefix.npz, every field of the parity contract): the
    engine reproduces per-call semantics, so the first calls' batches and
    order, the prefix events' rounds and witness flags, the round received and
    timestamp of every event the prefix ordered and the fame of every round up
    to the prefix's LastConsensusRound must be identical (parity.check_prefix);
  * size-independent properties of the reference's algorithm on the whole run:
    the order is a set of distinct accepted events and the per-call batches
    add up to it; inside every call's batch the ConsensusSorter keys
    (roundReceived, consensus timestamp, S; consensus_sorter.go:36-59) strictly
    increase; every ordered event was received after its round
    (hashgraph.go:680-684) and every unordered one has no roundReceived;
    Round(x) is ParentRound(x) or ParentRound(x) + 1 (hashgraph.go:287-305);
    witnesses are exactly the first events of their round on their chain
    (hashgraph.go:253-266).
"""
import json
import os
import sys

import numpy as np
import pytest

from babble_amd.gossip import random_gossip, schedule
from parity import check_prefix, check_run

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


@pytest.mark.parametrize("n,E", [(16, 100_000), (32, 1_000_000), (64, 1_000_000), (128, 1_000_000),
                                 (256, 10_000_000)])
def test_full_size(n, E):
    from babble_amd.engine import Engine, events_array
    K, seed = n, 1
    dag = random_gossip(n, E, seed=seed)
    calls = schedule(E, K)
    eng = Engine(n, E)
    try:
        st, order, counts = eng.replay(events_array(dag), calls)
        assert (st >= 0).all()
        assert len(order) > 0.99 * E  # all but the last rounds' events are ordered
        rounds, wit = eng.event_rounds()
        rr, cts = eng.event_received()
        pp = os.path.join(ROOT, "tests", "golden", f"bench_n{n}_e{E}_k{K}_s{seed}_prefix.npz")
        if os.path.exists(pp):
            bad = check_prefix(np.load(pp), order, counts, rounds, wit, rr, cts, eng.fame_table())
            assert not bad, f"fields differing from the oracle prefix golden: {bad}"
        check_run(dag, st, order, counts, rounds, wit, rr, cts)
        gf = json.load(open(os.path.join(ROOT, "tests", "golden", f"bench_n{n}_e{E}_k{K}_s{seed}_full.json")))
        from digest import compare_full, engine_state
        bad = compare_full(engine_state(eng, st, order, counts), gf)
        assert not bad, f"fields differing from the oracle's whole-stream digests: {bad}"
    finally:
        eng.close()

