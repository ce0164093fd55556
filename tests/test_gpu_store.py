"""Coordinates, predicates, Store semantics and sync-path reads of the HIP engine
against the oracle and the reference's container semantics.

* every event's lastAncestors / firstDescendants row (hge_coordinates) equals
  the oracle's (InitEventCoordinates / UpdateAncestorFirstDescendant,
  hashgraph.go:399-494), on the small-N path and on the wide (N > 32) path;
* the predicates the reference's tests call (hashgraph.go:83-326) agree with
  the oracle on random pairs;
* Store.ParticipantEvents / ParticipantEvent / LastFrom / ConsensusEvents follow
  the RollingList window and ErrTooLate (caches.go:45-97,
  common/rolling_list.go:42-67), Core.Diff's selection (node/core.go:108-132)
  and ReadWireInfo's parent resolution (hashgraph.go:526-571);
* admission refuses chains beyond the wide kernels' capacity and the engine
  stays usable; replay call points are validated.
"""
import numpy as np
import pytest

from babble_amd.gossip import random_gossip, schedule
from oracle.oracle import replay as oracle_replay
from parity import run_case

pytestmark = pytest.mark.gpu
INT64_MAX = np.iinfo(np.int64).max
INT32_MAX = np.iinfo(np.int32).max


def engine_replay(n, dag, k, cap=None):
    from babble_amd.engine import Engine
    eng = Engine(n, cap or len(dag["creator"]) + 64)
    st, order, counts = eng.replay(dag, schedule(len(dag["creator"]), k))
    return eng, st, order, counts


@pytest.mark.parametrize("n,events,k", [(4, 600, 4), (16, 2500, 16), (40, 5000, 40), (64, 6000, 64)])
def test_coordinates_match_oracle(n, events, k):
    dag = random_gossip(n, events, seed=300 + n)
    o, ost, oorder, _ = oracle_replay(dag, schedule(events, k))
    eng, st, order, _ = engine_replay(n, dag, k)
    try:
        np.testing.assert_array_equal(st, ost)
        for x in range(events):
            la, fd = eng.coordinates(x)
            ola, _, ofd, _ = o.coords(x)
            np.testing.assert_array_equal(la, ola, err_msg=f"lastAncestors of {x}")
            fd64 = np.where(fd == INT32_MAX, INT64_MAX, fd.astype(np.int64))
            np.testing.assert_array_equal(fd64, ofd, err_msg=f"firstDescendants of {x}")
    finally:
        eng.close()


@pytest.mark.parametrize("n,events,k", [(5, 1200, 5), (16, 3000, 16), (48, 6000, 48)])
def test_predicates_match_oracle(n, events, k):
    dag = random_gossip(n, events, seed=900 + n)
    o, _, _, _ = oracle_replay(dag, schedule(events, k))
    eng, _, _, _ = engine_replay(n, dag, k)
    rng = np.random.default_rng(n)
    try:
        # pairs near each other in time (where the answers are mixed) and anywhere
        xs = rng.integers(0, events, 1500)
        ys = np.clip(xs - rng.integers(0, 6 * n, 1500), 0, events - 1)
        ys[::3] = rng.integers(0, events, len(ys[::3]))
        for x, y in zip(xs.tolist(), ys.tolist()):
            assert eng.ancestor(x, y) == o.ancestor(x, y), ("ancestor", x, y)
            assert eng.self_ancestor(x, y) == o.self_ancestor(x, y), ("self_ancestor", x, y)
            assert eng.see(x, y) == o.see(x, y), ("see", x, y)
            assert eng.strongly_see(x, y) == o.strongly_see(x, y), ("strongly_see", x, y)
            assert eng.oldest_self_ancestor_to_see(x, y) == o.oldest_self_ancestor_to_see(x, y), ("osa", x, y)
        for x in rng.integers(0, events, 300).tolist():
            assert eng.parent_round(x) == o.parent_round(x), ("parent_round", x)
            assert eng.round_inc(x) == o.round_inc(x), ("round_inc", x)
            assert eng.round(x) == o.round(x), ("round", x)
            assert eng.witness(x) == o.witness(x), ("witness", x)
        # the bulk reads equal the per-event ones
        r, w = eng.event_rounds()
        np.testing.assert_array_equal(r, [o.round(x) for x in range(events)])
        np.testing.assert_array_equal(w, [o.witness(x) for x in range(events)])
        rr, cts = eng.event_received()
        for x in o.consensus_events().tolist():
            assert rr[x] == o.round_received(x) and cts[x] == o.consensus_timestamp(x)
    finally:
        eng.close()


def rolling_model(items, size):
    """common/rolling_list.go:55-67: (window, tot)."""
    win, tot = [], 0
    for it in items:
        if size > 0 and len(win) >= 2 * size:
            win = win[size:]
        win.append(it)
        tot += 1
    return win, tot


@pytest.mark.parametrize("size", [0, 7, 50])
def test_store_windows_and_sync_reads(size):
    from babble_amd.engine import HgeError
    n, events, k = 6, 1500, 6
    dag = random_gossip(n, events, seed=17)
    o, _, oorder, _ = oracle_replay(dag, schedule(events, k))
    eng, st, order, _ = engine_replay(n, dag, k)
    try:
        eng.set_cache_size(size)
        chains = [np.nonzero(dag["creator"] == c)[0] for c in range(n)]
        for c in range(n):
            win, tot = rolling_model(chains[c].tolist(), size)
            oldest = tot - len(win)
            for skip in (0, oldest - 1, oldest, tot - 3, tot - 1, tot, tot + 5):
                if skip < 0:
                    continue
                if skip < oldest and skip < tot:
                    with pytest.raises(HgeError) as ei:
                        eng.participant_events(c, skip)
                    assert ei.value.code == -11  # ErrTooLate
                else:
                    assert eng.participant_events(c, skip).tolist() == chains[c][skip:].tolist()
            assert eng.last_from(c) == chains[c][-1]
            assert eng.participant_event(c, tot - 1) == chains[c][-1]
            with pytest.raises(HgeError) as ei:
                eng.participant_event(c, tot)  # not found
            assert ei.value.code == -12
            with pytest.raises(HgeError) as ei:
                eng.participant_event(c, -1)  # below oldestCached (>= 0): ErrTooLate
            assert ei.value.code == -11
        # ConsensusEvents: the rolling window of the consensus list
        win, tot = rolling_model(oorder.tolist(), size)
        assert eng.consensus_events().tolist() == win
        assert eng.consensus_log().tolist() == oorder.tolist()
        # Core.Diff: what we know beyond `known`, in topological (insertion) order
        known = np.array([len(ch) - 3 for ch in chains], np.int32)
        exp = sorted(x for c in range(n) for x in chains[c][known[c]:].tolist())
        assert eng.diff(known).tolist() == exp
        # wire info and its inverse (ReadWireInfo)
        oldest = []
        for c in range(n):
            win, tot = rolling_model(chains[c].tolist(), size)
            oldest.append(tot - len(win))
        for x in range(0, events, 37):
            wi = eng.wire_info(x)
            assert wi == o.wire_info(x)
            if (wi[0] >= 0 and wi[0] < oldest[wi[3]]) or (wi[2] >= 0 and wi[2] < oldest[wi[1]]):
                with pytest.raises(HgeError) as ei:  # ParticipantEvent below the window
                    eng.read_wire_parents(wi[3], wi[0], wi[1], wi[2])
                assert ei.value.code == -11
                continue
            sp, op = eng.read_wire_parents(wi[3], wi[0], wi[1], wi[2])
            assert (sp, op) == (int(dag["sp"][x]), int(dag["op"][x]))
    finally:
        eng.close()


@pytest.mark.parametrize("n,events,limit", [(36, 2000, 40), (64, 6000, 60), (128, 12000, 70), (256, 20000, 60)])
def test_chain_past_uint16_switches_to_int32_replay(monkeypatch, n, events, limit):
    """Wide graphs keep chain positions as uint16 until a chain reaches the limit,
    then switch to int32 positions for good (hge_wide32.hip; the reference has no
    cap, hashgraph.go:328-363).  HGE_CHAIN_LIMIT lowers the switch point so a small
    stream crosses it: the replay (switched at admission) equals the live oracle."""
    from babble_amd.engine import Engine
    monkeypatch.setenv("HGE_CHAIN_LIMIT", str(limit))
    dag = random_gossip(n, events, seed=5 + n)
    assert np.bincount(np.asarray(dag["creator"]), minlength=n).max() > limit
    eng = Engine(n, events + 64)
    try:
        run_case(eng, dag, n)
    finally:
        eng.close()


@pytest.mark.parametrize("n,events,limit", [(40, 4000, 50), (256, 24000, 50)])
def test_chain_past_uint16_switches_mid_stream_online(monkeypatch, n, events, limit):
    """The online path crosses the limit mid-stream (the packed table is unpacked
    into int32 rows at the next coordinate step): the order, batches, rounds and
    round received equal an engine that never switched (the bulk replay of the
    packed path, no limit) and the fork-free stream stays fully accepted."""
    from babble_amd.engine import Engine, events_array
    from babble_amd.gossip import schedule
    dag = random_gossip(n, events, seed=90 + n)
    ev = events_array(dag)
    calls = schedule(events, n)
    ref = Engine(n, events + 64)  # created before the limit is set: packed all the way
    monkeypatch.setenv("HGE_CHAIN_LIMIT", str(limit))
    eng = Engine(n, events + 64)
    try:
        _, order, counts = ref.replay(ev, calls)
        nxt, per = 0, []
        for c in calls:
            eng.insert_events(ev[nxt:c].copy())
            per.append(len(eng.run_consensus()))
            nxt = c
        np.testing.assert_array_equal(eng.consensus_events(), order)
        np.testing.assert_array_equal(np.asarray(per), counts)
        assert eng.rounds() == ref.rounds()
        assert eng.last_consensus_round() == ref.last_consensus_round()
        for x, y in zip(eng.event_rounds(), ref.event_rounds()):
            np.testing.assert_array_equal(x, y)
        for x, y in zip(eng.event_received(), ref.event_received()):
            np.testing.assert_array_equal(x, y)
        # the coordinates read back from the int32 rows equal the packed ones
        for i in (0, events // 2, events - 1):
            for x, y in zip(eng.coordinates(i), ref.coordinates(i)):
                np.testing.assert_array_equal(x, y)
    finally:
        eng.close()
        ref.close()


@pytest.mark.parametrize("stage", [1, 2, 3])
def test_chain_switch_resumes_after_a_failed_widening(monkeypatch, stage):
    """The switch to int32 positions at N = 256 widens the uint16 runs and FD rows one
    table at a time.  A failure part-way (HGE_TEST_W32_FAIL: once, after the int32 LA
    table is allocated, after the runs are widened, or after the FD rows are) fails
    that RunConsensus; the retry resumes from the tables not yet widened (never reading
    a widened one as uint16) and the stream ends equal to an engine that never
    switched."""
    from babble_amd.engine import Engine, HgeError, events_array
    from babble_amd.gossip import schedule
    n, events = 256, 16000
    dag = random_gossip(n, events, seed=91)
    ev = events_array(dag)
    calls = schedule(events, n)
    ref = Engine(n, events + 64)
    monkeypatch.setenv("HGE_CHAIN_LIMIT", "50")
    monkeypatch.setenv("HGE_TEST_W32_FAIL", str(stage))
    eng = Engine(n, events + 64)
    try:
        _, order, counts = ref.replay(ev, calls)
        nxt, per, failed = 0, [], 0
        for c in calls:
            eng.insert_events(ev[nxt:c].copy())
            try:
                got = eng.run_consensus()
            except HgeError as e:
                assert "to_wide32 stopped" in str(e)
                failed += 1
                got = eng.run_consensus()
            per.append(len(got))
            nxt = c
        assert failed == 1
        np.testing.assert_array_equal(eng.consensus_events(), order)
        np.testing.assert_array_equal(np.asarray(per), counts)
        for x, y in zip(eng.event_received(), ref.event_received()):
            np.testing.assert_array_equal(x, y)
        for i in (0, events // 2, events - 1):
            for x, y in zip(eng.coordinates(i), ref.coordinates(i)):
                np.testing.assert_array_equal(x, y)
    finally:
        eng.close()
        ref.close()


def test_replay_rejects_bad_call_points():
    from babble_amd.engine import Engine, HgeError, events_array
    dag = random_gossip(4, 200, seed=2)
    eng = Engine(4, 512)
    try:
        for cp in ([0, 10], [10, 10], [20, 10], [10, 201]):
            with pytest.raises(HgeError) as ei:
                eng.prepare(events_array(dag), cp)
            assert ei.value.code == -8
        st, order, counts = eng.replay(dag, [50, 100, 200])
        assert len(counts) == 3
    finally:
        eng.close()


def test_round_event_ids_match_event_rounds():
    """hge_round_event_ids (Store.GetRound's RoundInfo.Events): every event of the
    round with its witness flag, in insertion order."""
    from babble_amd.engine import Engine, events_array
    from babble_amd.gossip import random_gossip, schedule
    n, E = 64, 20_000
    dag = random_gossip(n, E, seed=41)
    eng = Engine(n, E + 64)
    try:
        eng.replay(events_array(dag), schedule(E, n))
        rounds, wit = eng.event_rounds()
        R = eng.rounds()
        for r in [0, 1, R // 2, R - 2, R - 1]:
            ids, w = eng.round_event_ids(r)
            exp = np.flatnonzero(rounds == r)
            np.testing.assert_array_equal(ids, exp)
            np.testing.assert_array_equal(w, wit[exp].astype(bool))
            assert w.sum() == (eng.fame_table()[r] >= 0).sum()
        assert len(eng.round_event_ids(R)[0]) == 0
    finally:
        eng.close()
