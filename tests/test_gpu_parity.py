"""HIP engine vs the Go-faithful oracle (bit-exact), through the C ABI.

Every case compares: admission status, the full consensus order, the batch
size of every RunConsensus call, Rounds(), LastConsensusRound,
LastCommitedRoundEvents, ConsensusTransactions, the undetermined list, every
event's round and witness flag, every witness's fame, and every ordered
event's roundReceived and consensus timestamp.
"""
import numpy as np
import pytest

from babble_amd.gossip import random_gossip, schedule
from parity import run_case, with_creators, compare_state, oracle_run
from refdags import CONSENSUS_DAG, ROUND_DAG, to_stream

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engines():
    from babble_amd.engine import Engine
    cache = {}

    def get(n):
        if n not in cache:
            cache[n] = Engine(n, 1 << 14)
        return cache[n]

    yield get
    for e in cache.values():
        e.close()


def test_reference_consensus_dag_one_shot(engines):
    s, ix = to_stream(CONSENSUS_DAG)
    eng = engines(3)
    o, order = run_case(eng, s, len(CONSENSUS_DAG))
    names = {v: k for k, v in ix.items()}
    assert [names[i] for i in order] == ["e0", "e1", "e10", "e2", "e21", "e02"]
    for nm in ("e0", "e1", "e2"):
        assert eng.fame(0, int(s["creator"][ix[nm]])) == 1


@pytest.mark.parametrize("k", [1, 2, 3, 21])
def test_reference_consensus_dag_schedules(engines, k):
    s, _ = to_stream(CONSENSUS_DAG)
    run_case(engines(3), s, k)


@pytest.mark.parametrize("n,events,k", [
    (4, 1000, 1), (4, 1000, 4), (4, 1000, 13), (4, 1000, 1000),
    (3, 600, 3), (5, 1500, 5), (7, 2000, 7), (7, 2000, 50),
    (16, 3000, 16), (16, 3000, 1), (16, 3000, 200), (16, 3000, 3000),
])
def test_random_gossip(engines, n, events, k):
    dag = random_gossip(n, events, seed=1000 + n * 7 + k)
    run_case(engines(n), dag, k)


@pytest.mark.parametrize("n,events,k", [(32, 4000, 32), (64, 4000, 64),
                                         # N = 192: DecideFame's per-round widening (N % 64 == 0, N >= 192)
                                         # and uint16 FD rows; N = 200 / 224: the median's 4-witness
                                         # lanes past N / 4 (N < 256) and uint16 FD rows
                                         (192, 24000, 192), (200, 16000, 200), (224, 16000, 224)])
def test_random_gossip_wide(engines, n, events, k):
    dag = random_gossip(n, events, seed=5 + n)
    run_case(engines(n), dag, k, check_events=False)


def test_forkers(engines):
    dag = random_gossip(16, 3000, seed=77, forkers=5, fork_p=0.05)
    assert (~dag["honest"]).sum() > 0
    o, _ = run_case(engines(16), dag, 16)


def test_online_matches_replay(engines):
    """The online API (one batch per call) equals the bulk replay."""
    from babble_amd.engine import Engine, events_array
    n, E, k = 5, 800, 7
    dag = random_gossip(n, E, seed=9)
    calls = schedule(E, k)
    o, ost, oorder, _ = oracle_run(dag, calls)
    eng = Engine(n, 1 << 12)
    ev = events_array(dag)
    nxt = 0
    for c in calls:
        chunk = ev[nxt:c].copy()
        eng.insert_events(chunk)  # submission index == id (no rejections)
        eng.run_consensus()
        nxt = c
    np.testing.assert_array_equal(eng.consensus_events(), oorder)
    with_creators(eng, dag, ost)
    compare_state(eng, o)
    eng.close()


@pytest.mark.parametrize("n,E,k", [(16, 6000, 16), (16, 3000, 3), (32, 6000, 32), (12, 2000, 1), (48, 5000, 48),
                                   (64, 6000, 64), (128, 6000, 128), (192, 16000, 192), (224, 12000, 224)])
def test_online_matches_oracle_single_block_paths(engines, n, E, k):
    """Online calls take the single-block stages (k_fame_call; k_order_call at
    N <= 16; the frontier start in k_la_seq, the rounds assignment in the walk): the
    order, every call's batch and the whole state equal the oracle's."""
    from babble_amd.engine import Engine, events_array
    dag = random_gossip(n, E, seed=41 + n + k)
    calls = schedule(E, k)
    o, ost, oorder, ocounts = oracle_run(dag, calls)
    eng = Engine(n, 1 << 14)
    ev = events_array(dag)
    nxt, counts = 0, []
    for c in calls:
        eng.insert_events(ev[nxt:c].copy())  # submission index == id (no rejections)
        counts.append(len(eng.run_consensus()))
        nxt = c
    np.testing.assert_array_equal(eng.consensus_events(), oorder)
    np.testing.assert_array_equal(np.asarray(counts), np.asarray(ocounts))
    with_creators(eng, dag, ost)
    compare_state(eng, o)
    eng.close()


@pytest.mark.parametrize("n,E,k", [(16, 4000, 16), (8, 2000, 2), (64, 4000, 64)])
def test_online_single_block_paths_match_stage_kernels(engines, n, E, k, monkeypatch):
    """The online call's fused paths (one round trip at N <= 16, the single-block order
    and the batch's FD written by k_la_seq) against the per-stage kernels they replace
    (HGE_NO_ONLINE_FAST / HGE_NO_ORDER_CALL / HGE_NO_FD_DIRECT): the same order, batches
    and state."""
    from babble_amd.engine import Engine, events_array
    dag = random_gossip(n, E, seed=77 + n + k)
    ev = events_array(dag)
    calls = schedule(E, k)

    def run():
        eng = Engine(n, 1 << 13)
        nxt, batches = 0, []
        for c in calls:
            eng.insert_events(ev[nxt:c].copy())
            batches.append(eng.run_consensus())
            nxt = c
        state = (eng.consensus_events(), eng.undetermined(), eng.rounds(), eng.last_consensus_round(),
                 eng.last_committed_round_events(), eng.consensus_transactions())
        eng.close()
        return batches, state

    fused = run()
    for v in ("HGE_NO_ONLINE_FAST", "HGE_NO_ORDER_CALL", "HGE_NO_FD_DIRECT"):
        monkeypatch.setenv(v, "1")
    staged = run()
    assert len(fused[0]) == len(staged[0])
    for a, b in zip(fused[0], staged[0]):
        np.testing.assert_array_equal(a, b)
    for a, b in zip(fused[1], staged[1]):
        np.testing.assert_array_equal(np.asarray(a), np.asarray(b))


def test_split_calls_match_run_consensus(engines):
    """DivideRounds / DecideFame / FindOrder as separate calls (node/core.go:179-202)."""
    from babble_amd.engine import Engine, events_array
    n, E, k = 4, 600, 9
    dag = random_gossip(n, E, seed=11)
    calls = schedule(E, k)
    o, ost, oorder, _ = oracle_run(dag, calls)
    eng = Engine(n, 1 << 12)
    ev = events_array(dag)
    nxt = 0
    for c in calls:
        eng.insert_events(ev[nxt:c].copy())
        eng.divide_rounds()
        eng.decide_fame()
        eng.find_order()
        nxt = c
    np.testing.assert_array_equal(eng.consensus_events(), oorder)
    eng.close()
