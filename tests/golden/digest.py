"""Full-state digests of a replay (test infrastructure).

One SHA-256 over everything the parity contract calls bit-exact:
admission status, the order, per-call batch sizes, every event's round and
witness flag, the fame of every (round, creator) slot, every event's round
received, the consensus timestamp of every ordered event, the undetermined list
and the scalars (Rounds(), LastConsensusRound, LastCommitedRoundEvents,
ConsensusTransactions).  The same canonical byte layout is built from the CPU
oracle (make_mc_digests.py, make_golden.py's `describe`) and from the engine
(`engine_state`), so equal digests mean equal state, field by field.
"""
import hashlib

import numpy as np

FIELDS = (("status", "<i4"), ("order", "<i4"), ("counts", "<i8"), ("rounds", "<i4"),
          ("witness", "u1"), ("fame", "i1"), ("rr", "<i4"), ("cts", "<i8"),
          ("undetermined", "<i4"), ("scalars", "<i8"))


def canonical(state):
    """The state dict with canonical dtypes; cts kept for ordered events only."""
    out = {k: np.ascontiguousarray(np.asarray(state[k]).astype(dt)) for k, dt in FIELDS}
    cts = np.zeros_like(out["cts"])
    cts[out["order"]] = out["cts"][out["order"]]
    out["cts"] = cts
    return out


def digest(state):
    s = canonical(state)
    h = hashlib.sha256()
    for k, _ in FIELDS:
        a = s[k]
        h.update(k.encode())
        h.update(np.array(a.shape, "<i8").tobytes())
        h.update(a.tobytes())
    return h.hexdigest()


EVENT_CHUNK = 1 << 20   # events per chunk digest of rounds / witness / rr / cts
ORDER_CHUNK = 1 << 20   # order positions per chunk digest
CALL_CHUNK = 1 << 12    # calls per chunk digest of counts


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:32]


def _chunks(a, step):
    return [_sha(a[i:i + step]) for i in range(0, max(len(a), 1), step)]


def field_digests(state):
    """Per-field and per-chunk digests of a state (the `canonical` layout), and
    the whole-state digest: what tests/golden/*_full.json hold."""
    s = canonical(state)
    out = {"fields": {k: _sha(s[k]) for k, _ in FIELDS},
           "chunks": {"order": _chunks(s["order"], ORDER_CHUNK), "counts": _chunks(s["counts"], CALL_CHUNK)}}
    for k in ("rounds", "witness", "rr", "cts"):
        out["chunks"][k] = _chunks(s[k], EVENT_CHUNK)
    out["digest"] = digest(state)
    return out


def compare_full(state, golden, fields=None):
    """Fields of `state` whose digest differs from a *_full.json golden, each with
    the first differing chunk where the field is chunked: [] when identical.
    `fields`: only these (e.g. order and counts for a sharded run)."""
    got = field_digests(state)
    bad = []
    for k, _ in FIELDS:
        if fields is not None and k not in fields:
            continue
        if got["fields"][k] != golden["fields"][k]:
            ch = golden["chunks"].get(k)
            if ch is not None:
                gc = got["chunks"][k]
                first = next((i for i in range(max(len(ch), len(gc)))
                              if i >= len(ch) or i >= len(gc) or ch[i] != gc[i]), None)
                bad.append(f"{k}[chunk {first}]")
            else:
                bad.append(k)
    return bad


def engine_state(eng, status, order, counts):
    """The engine's side of `canonical` after a replay (status/order/counts from
    Engine.fetch)."""
    rounds, wit = eng.event_rounds()
    rr, cts = eng.event_received()
    lcr = eng.last_consensus_round()
    return dict(status=status, order=order, counts=counts, rounds=rounds, witness=wit, fame=eng.fame_table(),
                rr=rr, cts=cts, undetermined=eng.undetermined(),
                scalars=np.array([eng.rounds(), -1 if lcr is None else lcr, eng.last_committed_round_events(),
                                  eng.consensus_transactions()], np.int64))


def first_difference(a, b):
    """Name of the first field where two states differ (None if equal)."""
    ca, cb = canonical(a), canonical(b)
    for k, _ in FIELDS:
        if ca[k].shape != cb[k].shape or not np.array_equal(ca[k], cb[k]):
            return k
    return None
