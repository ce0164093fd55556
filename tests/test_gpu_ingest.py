"""hge_ingest on the device: InsertEvent with its signature check (host threads,
overlapped with the device) in batches of K, RunConsensus after each batch
(node/core.go:179-202), against the oracle replaying the same stream with the
same call points.  A bad signature ends the stream there ("Invalid signature",
hashgraph.go:330-336): the events before it are ordered exactly as the
oracle orders that prefix."""
import numpy as np
import pytest

from babble_amd import signing
from babble_amd.engine import Engine, events_array
from babble_amd.gossip import random_gossip
from oracle.oracle import replay as oracle_replay

pytestmark = pytest.mark.gpu


def _calls(n, k):
    pts = list(range(k, n + 1, k))
    if not pts or pts[-1] != n:
        pts.append(n)
    return np.array(pts, np.int64)


@pytest.mark.parametrize("n,E,k", [(16, 3000, 16), (64, 6000, 64)])
def test_ingest_matches_oracle(n, E, k):
    dag = random_gossip(n, E, seed=4)
    pubs, bodies, sigs = signing.signed_stream(dag, seed=2, threads=8)
    ev = events_array(dag)
    eng = Engine(n, E)
    rc, status, acc, tm = eng.ingest(ev, bodies, pubs, sigs, k, threads=4)
    assert rc == 0 and acc == E
    assert np.array_equal(status, np.arange(E))
    order = eng.consensus_log()
    _, ostatus, oorder, _ = oracle_replay(dag, _calls(E, k))
    assert np.array_equal(order, oorder)
    assert tm["wall_ms"] > 0
    eng.close()


def test_ingest_stops_at_bad_signature():
    n, E, k, bad = 16, 2400, 16, 1203
    dag = random_gossip(n, E, seed=6)
    pubs, bodies, sigs = signing.signed_stream(dag, seed=3, threads=8)
    sigs = sigs.copy()
    sigs[bad, 40] ^= 0x10
    eng = Engine(n, E)
    rc, status, acc, _ = eng.ingest(events_array(dag), bodies, pubs, sigs, k, threads=3)
    assert rc == -13 and acc == bad and status[bad] == -13
    assert eng.event_count() == bad
    pre = {key: (v[:bad] if isinstance(v, np.ndarray) else v) for key, v in dag.items()}
    _, _, oorder, _ = oracle_replay(pre, _calls(bad, k))
    assert np.array_equal(eng.consensus_log(), oorder)
    eng.close()


def test_ingest_refuses_body_signed_by_another_creator():
    """A validly signed body whose key is not its creator id's key is refused
    (in the reference the creator id is looked up from Body.Creator, so the
    signature binds the event to its creator: hashgraph.go:330-336, 366-370)."""
    n, E, k, bad = 16, 1600, 16, 777
    dag = random_gossip(n, E, seed=7)
    pubs, bodies, sigs = signing.signed_stream(dag, seed=4, threads=8)
    c = int(dag["creator"][bad])
    # the body and signature of event `bad` replaced by another creator's signed event
    other = int(np.nonzero(dag["creator"] != c)[0][-1])
    flat, off = bodies
    flat = flat.copy()
    flat[off[bad]:off[bad + 1]] = flat[off[other]:off[other + 1]]
    bodies = (flat, off)
    sigs = sigs.copy()
    sigs[bad] = sigs[other]
    eng = Engine(n, E)
    rc, status, acc, _ = eng.ingest(events_array(dag), bodies, pubs, sigs, k, threads=3)
    assert rc == -13 and acc == bad and status[bad] == -13
    eng.close()
