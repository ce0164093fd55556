"""Speculative walkers of the wide (N > 32) rounds walk (k_rounds_coop_spec /
k_coop_join in babble_amd/csrc/hge_rounds_coop.hip).

From a fresh state, up to 8 walkers of N co-resident workgroups walk the
frontier recurrence from guessed frontiers and merge on equal rows; a walker
whose history fills without a merge ends the chain and the sequential
cooperative kernel resumes from the last true row.  Every case is bit-exact:
against the committed wide goldens (oracle outputs), against the live oracle,
and against the sequential kernel (HGE_COOP_WALKERS=0) on the same graph,
for several walker counts and forced capacity breaks (HGE_WALK_HCAP).
"""
import glob
import os

import numpy as np
import pytest

from babble_amd.gossip import random_gossip, schedule
from parity import compare_golden, load_golden, run_case

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WIDE = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "wide_*.npz")))


def _state(n, dag, calls, cap):
    from babble_amd.engine import Engine
    eng = Engine(n, cap)
    try:
        st, order, counts = eng.replay(dag, calls)
        ids = [int(s) for s in st if s >= 0]
        return (np.array([eng.round(x) for x in ids]), np.array([eng.witness(x) for x in ids]),
                order, counts, eng.rounds(), eng.last_consensus_round())
    finally:
        eng.close()


@pytest.mark.parametrize("walkers", [2, 4])
@pytest.mark.parametrize("path", WIDE, ids=lambda p: os.path.basename(p))
def test_coop_spec_golden(monkeypatch, path, walkers):
    from babble_amd.engine import Engine
    monkeypatch.setenv("HGE_COOP_WALKERS", str(walkers))
    dag, g = load_golden(path)
    eng = Engine(int(g["n"]), len(dag["creator"]) + 16)
    try:
        compare_golden(eng, dag, g)
    finally:
        eng.close()


def test_coop_spec_vs_oracle(monkeypatch):
    """N = 40 (odd word split of the member rows), long enough chains for 3 walkers."""
    from babble_amd.engine import Engine
    monkeypatch.setenv("HGE_COOP_WALKERS", "3")
    eng = Engine(40, 1 << 13)
    try:
        run_case(eng, random_gossip(40, 8000, seed=640), 40)
    finally:
        eng.close()


@pytest.mark.parametrize("n,events,walkers,hcap", [
    (64, 40_000, 4, None),
    (64, 40_000, 2, None),
    (64, 40_000, 4, 7),      # histories too short to merge: chain breaks, sequential resume
    (64, 40_000, 4, 60),
    (96, 40_000, 2, None),
    (128, 60_000, 2, 90),
])
def test_coop_spec_equals_sequential(monkeypatch, n, events, walkers, hcap):
    """Per-event rounds, witnesses, fame-derived order and round count equal the
    sequential cooperative kernel's on the same graph."""
    dag = random_gossip(n, events, seed=700 + n + walkers)
    calls = schedule(events, n)
    monkeypatch.delenv("HGE_WALK_HCAP", raising=False)
    monkeypatch.setenv("HGE_COOP_WALKERS", "0")
    ref = _state(n, dag, calls, events + 64)
    monkeypatch.setenv("HGE_COOP_WALKERS", str(walkers))
    if hcap is not None:
        monkeypatch.setenv("HGE_WALK_HCAP", str(hcap))
    got = _state(n, dag, calls, events + 64)
    for a, b in zip(ref, got):
        np.testing.assert_array_equal(a, b)
    assert ref[4] > 20
