"""CPU-side checks: the C ABI library loads and exports every symbol include/hge.h
declares; the oracle reproduces the committed golden vectors; the synthetic
generator honours the gossip rules."""
import glob
import json
import os
import re

import numpy as np
import pytest

from babble_amd.gossip import random_gossip, schedule
from oracle.oracle import replay

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def header_symbols():
    src = open(os.path.join(ROOT, "include", "hge.h")).read()
    return sorted(set(re.findall(r"\b(hge_[a-z_]+)\s*\(", src)))


def test_header_symbols_exported():
    from babble_amd import engine
    L = engine.lib()
    syms = header_symbols()
    assert len(syms) >= 30
    for s in syms:
        assert hasattr(L, s), s
    assert sorted(engine.EXPORTS) == syms


def test_engine_fails_loudly_without_library(monkeypatch, tmp_path):
    import importlib
    import babble_amd.engine as eng
    monkeypatch.setattr(eng, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(eng, "_lib", None)
    with pytest.raises(ImportError):
        eng.lib()
    importlib.reload(eng)


def test_event_record_layout():
    import ctypes
    from babble_amd.engine import EVENT_DTYPE, HgeEvent
    assert ctypes.sizeof(HgeEvent) == EVENT_DTYPE.itemsize == 96


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "gossip_*.npz"))),
                         ids=lambda p: os.path.basename(p))
def test_oracle_reproduces_golden(path):
    g = np.load(path, allow_pickle=False)
    dag = {k: g[k] for k in ("creator", "index", "sp", "op", "ts", "S", "hash", "ntx")}
    dag["n"] = int(g["n"])
    o, status, order, counts = replay(dag, g["calls"])
    np.testing.assert_array_equal(status, g["status"])
    np.testing.assert_array_equal(order, g["order"])
    np.testing.assert_array_equal(counts, g["counts"])
    R, lcr, lcre, ctx = g["scalars"].tolist()
    assert o.rounds() == R
    assert (o.last_consensus_round() if o.last_consensus_round() is not None else -1) == lcr
    assert o.last_committed_round_events() == lcre
    assert o.consensus_transactions() == ctx
    np.testing.assert_array_equal(o.undetermined(), g["undetermined"])
    rounds = np.array([o.round(x) for x in range(len(g["rounds"]))])
    np.testing.assert_array_equal(rounds, g["rounds"])


def test_reference_dag_golden_json():
    ref = json.load(open(os.path.join(GOLD, "reference_dags.json")))
    assert ref["consensus"]["order_one_shot"] == ["e0", "e1", "e10", "e2", "e21", "e02"]
    assert ref["round"]["rounds"]["f1"] == 1 and ref["round"]["rounds"]["e02"] == 0
    assert ref["consensus"]["rounds"]["g0"] == 2


def test_gossip_rules():
    n = 8
    d = random_gossip(n, 2000, seed=4)
    E = len(d["creator"])
    assert (d["sp"][:n] == -1).all() and (d["op"][:n] == -1).all()
    for i in range(n, E):
        c = d["creator"][i]
        sp, op = d["sp"][i], d["op"][i]
        assert 0 <= sp < i and d["creator"][sp] == c
        assert 0 <= op < i and d["creator"][op] != c  # never self (peer_selector.go:53-61)
        assert d["index"][i] == d["index"][sp] + 1
        # op is the latest event of its creator before i
        later = np.nonzero((d["creator"][op + 1:i] == d["creator"][op]))[0]
        assert later.size == 0
    assert (np.diff(d["ts"]) > 0).all()


def test_forks_are_rejected_like_from_parents_latest():
    d = random_gossip(12, 1500, seed=8, forkers=4, fork_p=0.1)
    o, status, order, _ = replay(d, schedule(len(d["creator"]), 12))
    twins = ~d["honest"]
    assert twins.sum() > 0
    assert (status[twins] == -5).all()          # "Self-parent not last known event by creator"
    assert (status[~twins] >= 0).all()


def test_schedule():
    assert schedule(10, 4).tolist() == [4, 8, 10]
    assert schedule(8, 4).tolist() == [4, 8]
    assert schedule(5, 100).tolist() == [5]
