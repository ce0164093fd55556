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
    return sorted(set(re.findall(r"\b(hge_[a-z0-9_]+)\s*\(", src)))


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


def test_golden_fame_statistics():
    """The goldens the GPU replays reach DecideFame's rare branches: coin rounds with
    coin votes (hashgraph.go:645-649) and witnesses re-decided with a different
    value inside one call (missing votes read as nays, SURVEY.md TL;DR 4)."""
    stats = {os.path.basename(p): np.load(p)["fame_stats"]
             for p in glob.glob(os.path.join(GOLD, "*.npz")) if "fame_stats" in np.load(p).files}
    assert len(stats) >= 10
    assert stats["gossip_n4_e1000_oneshot.npz"][0] > 0   # coin-branch evaluations
    assert stats["gossip_n4_e1000_oneshot.npz"][1] > 0   # votes taken from the coin
    assert sum(1 for v in stats.values() if v[3] > 0) >= 8  # fame flipped by a re-decision


@pytest.mark.parametrize("name", ["gossip_n4_e1000_k1", "gossip_n4_e1000_oneshot"])
def test_witness_order_invariance_flags(name):
    """Re-run the recorded invariance check (roundInfo.go:88-96: Go iterates round
    witnesses in random map order) and compare with the flags in the golden."""
    g = np.load(os.path.join(GOLD, name + ".npz"))
    dag = {k: g[k] for k in ("creator", "index", "sp", "op", "ts", "S", "hash", "ntx")}
    dag["n"] = int(g["n"])
    same = True
    for sd in g["order_seeds"].tolist():
        _, _, order, _ = replay(dag, g["calls"], order_seed=sd)
        same &= bool(np.array_equal(order, g["order"]))
    assert same == bool(g["order_invariant"])


def test_cascade_generator_and_oracle():
    d = random_gossip(16, 3000, seed=21, forkers=5, fork_p=0.08, cascade_p=0.6)
    o, status, order, _ = replay(d, schedule(len(d["creator"]), 16))
    assert (status[d["honest"]] >= 0).all()
    codes = set(np.unique(status[status < 0]).tolist())
    assert {-5, -4, -2} <= codes
    i = np.arange(len(d["creator"]))
    assert (d["sp"] < i).all() and (d["op"] < i).all() and (np.diff(d["ts"]) > 0).all()


def test_property_checker_on_an_oracle_run():
    """tests/parity.check_run (the full-size GPU checks) holds on an oracle run."""
    from parity import check_run
    n, E = 8, 3000
    dag = random_gossip(n, E, seed=12, forkers=2, fork_p=0.05, cascade_p=0.5)
    calls = schedule(len(dag["creator"]), n)
    o, st, order, counts = replay(dag, calls)
    m = int((st >= 0).sum())
    rounds = np.array([o.round(x) for x in range(m)])
    wit = np.array([o.witness(x) for x in range(m)])
    rr = np.array([o.round_received(x) if o.round_received(x) is not None else -1 for x in range(m)])
    cts = np.array([o.consensus_timestamp(x) if rr[x] >= 0 else 0 for x in range(m)], np.int64)
    check_run(dag, st, order, counts, rounds, wit, rr, cts)


def test_cpp_abi_binary_cpu_checks():
    """tests/abi/hge_abi_test.cpp: the C ABI from C++ (argument errors, null handle)."""
    import subprocess
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "abi")])
    out = subprocess.run([os.path.join(ROOT, "build", "hge_abi_test")], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
