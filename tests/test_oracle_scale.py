"""The oracle's scale mode against its faithful mode (hg_oracle.cpp header).

The scale mode computes the faithful restatement's results without the pure
memo caches, with bitset votes in DecideFame, a per-round undecided counter
and per-(round, creator) thresholds in DecideRoundReceived, and optionally
releases the coordinates of events ordered long ago.  It makes the whole-stream
goldens possible (tests/golden/make_bench_full.py); here it must agree with the
faithful mode on every field of the parity contract, including DecideFame's
coin / re-decision statistics, over streams that reach coin rounds, flipped
re-decisions, forks and cascades.
"""
import numpy as np
import pytest

from babble_amd.gossip import random_gossip, schedule
from oracle.oracle import Oracle, replay

FIELDS = ("status", "order", "counts", "rounds", "witness", "fame", "rr", "cts", "undetermined", "scalars",
          "fame_stats")


def state(dag, calls, **kw):
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    from make_golden import describe
    o, status, order, counts = replay(dag, calls, **kw)
    d = describe(o, dag, status, order, counts, calls)
    return o, d


CASES = [
    # n, events, k, seed, forkers, fork_p, cascade_p
    (4, 1500, 1, 11, 0, 0.0, 0.0),
    (4, 1500, 1500, 12, 0, 0.0, 0.0),     # one shot: long fame chains, coin rounds at diff % 4 == 0
    (5, 2000, 3, 13, 0, 0.0, 0.0),
    (7, 3000, 7, 14, 2, 0.1, 0.5),
    (16, 4000, 16, 15, 0, 0.0, 0.0),
    (32, 4000, 32, 16, 10, 0.05, 0.5),
    (33, 3000, 50, 17, 0, 0.0, 0.0),
    (64, 6000, 64, 18, 0, 0.0, 0.0),
]


@pytest.mark.parametrize("n,E,k,seed,fk,fp,cp", CASES)
def test_scale_equals_faithful(n, E, k, seed, fk, fp, cp):
    dag = random_gossip(n, E, seed=seed, forkers=fk, fork_p=fp, cascade_p=cp)
    calls = schedule(len(dag["creator"]), k)
    of, f = state(dag, calls)
    os_, s = state(dag, calls, scale=True)
    assert not of.is_scale() and os_.is_scale()
    for key in FIELDS:
        np.testing.assert_array_equal(np.asarray(s[key]), np.asarray(f[key]), err_msg=key)


def test_scale_reaches_coin_rounds_and_flips():
    """The one-shot N=4 stream exercises the coin branch and flipped re-decisions
    in both modes (the statistics are part of the comparison above)."""
    dag = random_gossip(4, 1500, seed=12)
    _, s = state(dag, schedule(1500, 1500), scale=True)
    coin_evals, coin_votes, redecided, flipped = s["fame_stats"].tolist()
    assert coin_evals > 0 and redecided > 0


def test_release_changes_nothing():
    dag = random_gossip(64, 30_000, seed=19)
    calls = schedule(30_000, 64)
    _, a = state(dag, calls, scale=True)
    o, b = state(dag, calls, scale=True, release_lag=4)
    for key in FIELDS:
        np.testing.assert_array_equal(np.asarray(b[key]), np.asarray(a[key]), err_msg=key)


def test_scale_off_for_random_order_and_seeded_rounds():
    assert not Oracle(4, order_seed=3, scale=True).is_scale()
    o = Oracle(3, scale=True)
    assert o.is_scale()
    o.insert(0, 0, -1, -1, 0)
    o.set_round(0, [(0, True, 0)])
    assert not o.is_scale()


def test_index_outside_int32_refused():
    o = Oracle(2)
    with pytest.raises(ValueError, match="int32"):
        o.insert(0, 2**31, -1, -1, 0)
