"""The batch engine's bulk call schedule (hge_batch_bulk.hip), restated in plain
Python (tests/bulk_model.py), against the oracle on small streams: the
formulation itself -- DecideFame per (call, round) pair, one fold over the calls
into (decided, famous set) intervals per round, each event received at the first
call an interval above it sees it -- reproduces RunConsensus after every call
point (order, batches, round received, timestamps, fame, undetermined list,
scalars).  CPU only; the GPU tests check the kernels against the oracle."""
import os
import sys

import numpy as np
import pytest

from babble_amd.gossip import random_gossip, schedule

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "golden"))

CASES = [
    # n, events, k, seed, forkers, fork_p, cascade_p, op_lag, NS
    (4, 800, 4, 1, 0, 0.0, 0.0, 0, 3),
    (4, 600, 1, 2, 0, 0.0, 0.0, 0, 1),       # K = 1, a one-pair window: misses decided inline
    (4, 500, 500, 12, 0, 0.0, 0.0, 0, 3),    # one call
    (1, 50, 5, 3, 0, 0.0, 0.0, 0, 3),        # coin rounds only
    (2, 300, 2, 3, 0, 0.0, 0.0, 0, 3),
    (7, 1200, 7, 14, 2, 0.1, 0.5, 0, 2),     # forks and cascades
    (16, 1200, 50, 21, 0, 0.0, 0.0, 6, 3),   # other-parents behind their chain's head
    (32, 1500, 32, 4, 10, 0.05, 0.5, 0, 3),  # config 5's shape
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"n{c[0]}_e{c[1]}_k{c[2]}_ns{c[8]}")
def test_bulk_model_matches_oracle(case):
    from bulk_model import bulk_replay
    from make_mc_digests import oracle_state
    n, E, k, seed, fk, fp, cp, lag, ns = case
    dag = random_gossip(n, E, seed=seed, forkers=fk, fork_p=fp, cascade_p=cp, op_lag=lag)
    calls = schedule(len(dag["creator"]), k)
    want = oracle_state(dag, calls)
    got = bulk_replay(dag, calls, want["status"], want["rounds"], want["witness"], NS=ns)
    for f in ("order", "counts", "fame", "undetermined", "scalars", "rr"):
        np.testing.assert_array_equal(np.asarray(got[f]), np.asarray(want[f]), err_msg=f)
    o = np.asarray(want["order"])
    np.testing.assert_array_equal(got["cts"][o], np.asarray(want["cts"])[o], err_msg="cts")
    # one receive interval per round at most (kb_fold writes it when the round is decided)
    assert got["stats"]["max_intervals"] <= 1
