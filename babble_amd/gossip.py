"""Seeded synthetic event streams.

Random gossip, mirroring babble's RandomPeerSelector
(/root/reference/node/peer_selector.go:53-61: a node never picks itself):
  * the first N submissions are the initial events (index 0, no parents);
  * every later submission picks creator a ~ U[0,N) and peer b ~ U[0,N)\\{a}
    and emits (creator a, index seq[a]++, self-parent head[a], other-parent head[b]).

Fields: ts = base + 1000 * submission (strictly increasing ns), S = 256-bit
uniform (SplitMix64 stream keyed by (seed, submission)), hash = 32 bytes from
the same family (only hash[16], the coin bit of hashgraph.go:781-790, and
identity matter to the ordering path).

Byzantine forkers (config 5): a subset of creators, with probability p per
event, also submit a second event with the same (creator, index, parents) and
a different hash/S right after the honest one.  The first-inserted branch wins;
the fork is rejected by FromParentsLatest (hashgraph.go:366-396).

Cascades (cascade_p > 0): a peer that saw the losing branch first builds on
it.  With probability cascade_p per fork twin, a random other creator submits,
right after the twin, an event whose other-parent IS the twin ("Other-parent
not known", hashgraph.go:381-384); with probability 1/2 that creator then
submits a child of the rejected event ("Self-parent not known",
hashgraph.go:373-376), and with probability 1/2 a third creator submits an
event whose other-parent is the rejected one (rejected again).  Rejected
submissions are never referenced by honest ones, so the honest stream goes on
(the node keeps syncing with everyone else).
"""
import numpy as np

TS_BASE = 1_500_000_000_000_000_000  # 2017-07-14 in ns; any fixed epoch works


def _splitmix64(x):
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & np.uint64(0xFFFFFFFFFFFFFFFF)
    z = x
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & np.uint64(0xFFFFFFFFFFFFFFFF)
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & np.uint64(0xFFFFFFFFFFFFFFFF)
    return z ^ (z >> np.uint64(31))


def _bytes32(seed, salt, n):
    """n x 32 pseudo-random bytes keyed by (seed, salt, row)."""
    rows = np.arange(n, dtype=np.uint64)
    out = np.empty((n, 4), np.uint64)
    base = np.uint64((seed * 0x100000001B3 + salt * 0x9E3779B1) & 0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        for k in range(4):
            out[:, k] = _splitmix64(rows * np.uint64(4) + np.uint64(k) + base * np.uint64(7919))
    return out.astype(">u8").view(np.uint8).reshape(n, 32)


def random_gossip(n, events, seed=1, forkers=0, fork_p=0.0, cascade_p=0.0, op_lag=0):
    """Return a dict describing a submission stream of `events` honest events.

    op_lag > 0: the other-parent is the peer's event `lag` positions before its
    latest, lag ~ U{0..op_lag} (a stale view of the peer, as when a node inserts
    events it learned late): other-parents that are not their chain's head.

    Keys: n, creator, index, sp, op (submission indices, -1 = none), ts, S
    (uint8[E,32] big-endian), hash (uint8[E,32]), ntx, honest (bool mask).
    """
    assert n >= 1 and events >= n
    rng = np.random.default_rng(seed)
    m = events - n
    a = rng.integers(0, n, m)
    if n > 1:
        b = rng.integers(0, n - 1, m)
        b = b + (b >= a)  # U[0,N) \ {a}
    else:
        b = np.zeros(m, np.int64)
    creator = np.concatenate([np.arange(n), a]).astype(np.int32)
    E = events
    # sp = previous submission of the same creator
    order = np.argsort(creator, kind="stable")
    cs = creator[order]
    prev = np.full(E, -1, np.int64)
    same = cs[1:] == cs[:-1]
    prev[order[1:][same]] = order[:-1][same]
    index = np.zeros(E, np.int64)
    # index = rank within creator
    starts = np.searchsorted(cs, np.arange(n))
    rank = np.arange(E) - starts[cs]
    index[order] = rank
    # op = latest submission of creator b strictly before this one
    op = np.full(E, -1, np.int64)
    if m:
        subs = np.arange(n, E)
        ends = np.searchsorted(cs, np.arange(n), side="right")
        # position of the last event of creator b before `sub`: events of b sorted by submission
        bb = b.astype(np.int64)
        lo = starts[bb]
        # per creator, submissions in order -> searchsorted within the creator's slice
        pos = np.empty(m, np.int64)
        for c in range(n):
            sel = np.nonzero(bb == c)[0]
            if sel.size == 0:
                continue
            slice_ = order[starts[c]:ends[c]]
            k = np.searchsorted(slice_, subs[sel], side="left") - 1
            if op_lag > 0:
                k = np.maximum(0, k - rng.integers(0, op_lag + 1, len(k)))
            pos[sel] = slice_[k]
        del lo
        op[n:] = pos
    dag = {
        "n": n,
        "creator": creator,
        "index": index.astype(np.int32),
        "sp": prev.astype(np.int32),
        "op": op.astype(np.int32),
        "ts": (TS_BASE + 1000 * np.arange(E, dtype=np.int64)),
        "S": _bytes32(seed, 1, E),
        "hash": _bytes32(seed, 2, E),
        "ntx": np.ones(E, np.int32),
        "honest": np.ones(E, bool),
    }
    if forkers and fork_p > 0:
        dag = _inject_forks(dag, rng, forkers, fork_p, seed)
        if cascade_p > 0:
            dag = _inject_cascades(dag, rng, cascade_p, seed)
    return dag


def _inject_forks(dag, rng, forkers, p, seed):
    E = len(dag["creator"])
    n = dag["n"]
    fset = np.zeros(n, bool)
    fset[rng.choice(n, size=min(forkers, n), replace=False)] = True
    fork = fset[dag["creator"]] & (rng.random(E) < p) & (dag["sp"] >= 0)
    nf = int(fork.sum())
    if nf == 0:
        return dag
    # new submission order: each forked event is followed by its fork twin
    reps = 1 + fork.astype(np.int64)
    new_pos = np.cumsum(reps) - reps  # position of the honest copy
    tot = E + nf
    src = np.repeat(np.arange(E), reps)
    is_twin = np.zeros(tot, bool)
    is_twin[new_pos[fork] + 1] = True

    def remap(p_):
        return np.where(p_ >= 0, new_pos[np.maximum(p_, 0)], -1).astype(np.int32)

    out = {"n": n}
    for k in ("creator", "index", "ntx"):
        out[k] = dag[k][src]
    out["sp"] = remap(dag["sp"])[src]
    out["op"] = remap(dag["op"])[src]
    out["ts"] = dag["ts"][src].copy()
    out["S"] = dag["S"][src].copy()
    out["hash"] = dag["hash"][src].copy()
    twin_S = _bytes32(seed, 3, nf)
    twin_H = _bytes32(seed, 4, nf)
    out["S"][is_twin] = twin_S
    out["hash"][is_twin] = twin_H
    out["ts"][is_twin] += 1
    out["honest"] = ~is_twin
    return out


def _inject_cascades(dag, rng, p, seed):
    """Submissions that build on fork twins (see the module docstring).  Each
    doomed record is inserted right after the twin it descends from."""
    n = dag["n"]
    E = len(dag["creator"])
    twins = np.nonzero(~dag["honest"])[0]
    chosen = twins[rng.random(len(twins)) < p]
    if chosen.size == 0:
        return dag
    creator = dag["creator"]
    honest = dag["honest"]
    # honest positions of every creator, for "the head of creator c before position t"
    pos_by_c = [np.nonzero((creator == c) & honest)[0] for c in range(n)]

    def head(c, t):
        k = np.searchsorted(pos_by_c[c], t) - 1
        return int(pos_by_c[c][k]) if k >= 0 else -1

    recs = []  # (insert after stream position, creator, index, sp, op) with sp/op = ("s", pos) or ("d", j)
    for t in chosen.tolist():
        tc = int(creator[t])
        others = [c for c in range(n) if c != tc]
        c2 = int(others[rng.integers(len(others))])
        h2 = head(c2, t)
        if h2 < 0:
            continue
        j0 = len(recs)
        recs.append((t, c2, int(dag["index"][h2]) + 1, ("s", h2), ("s", t)))     # op = twin
        if rng.random() < 0.5:                                                  # child of the doomed one
            h_any = head(int(others[rng.integers(len(others))]), t)
            recs.append((t, c2, int(dag["index"][h2]) + 2, ("d", j0), ("s", max(h_any, 0))))
        if rng.random() < 0.5 and n > 2:                                        # op = the doomed one
            c3 = int([c for c in others if c != c2][rng.integers(n - 2)])
            h3 = head(c3, t)
            if h3 >= 0:
                recs.append((t, c3, int(dag["index"][h3]) + 1, ("s", h3), ("d", j0)))
    if not recs:
        return dag
    after = np.array([r[0] for r in recs], np.int64)
    m = len(recs)
    # new position of old stream position q: q + #records inserted after positions < q
    shift = np.searchsorted(np.sort(after), np.arange(E), side="left")
    newpos_old = np.arange(E) + shift
    # records after the same twin keep their relative order: position = twin's new pos + 1 + k
    k_same = np.zeros(m, np.int64)
    seen = {}
    for j in range(m):
        k_same[j] = seen.get(after[j], 0)
        seen[after[j]] = k_same[j] + 1
    newpos_rec = newpos_old[after] + 1 + k_same
    tot = E + m
    out = {"n": n}
    sel_old = newpos_old
    for key in ("creator", "index", "ntx", "ts", "honest"):
        arr = np.empty(tot, dag[key].dtype)
        arr[sel_old] = dag[key]
        out[key] = arr

    def remap_old(v):
        return np.where(v >= 0, newpos_old[np.maximum(v, 0)], -1)

    sp = np.empty(tot, np.int64)
    op = np.empty(tot, np.int64)
    sp[sel_old] = remap_old(dag["sp"])
    op[sel_old] = remap_old(dag["op"])
    S = np.empty((tot, 32), np.uint8)
    H = np.empty((tot, 32), np.uint8)
    S[sel_old] = dag["S"]
    H[sel_old] = dag["hash"]
    rS = _bytes32(seed, 5, m)
    rH = _bytes32(seed, 6, m)

    def ref(r):
        return newpos_old[r[1]] if r[0] == "s" else newpos_rec[r[1]]

    for j, (t, c, idx, rsp, rop) in enumerate(recs):
        q = newpos_rec[j]
        out["creator"][q] = c
        out["index"][q] = idx
        out["ntx"][q] = 1
        out["ts"][q] = dag["ts"][t] + 2 + j % 997  # between the twin and the next honest event
        out["honest"][q] = False
        sp[q] = ref(rsp)
        op[q] = ref(rop)
        S[q] = rS[j]
        H[q] = rH[j]
    out["sp"] = sp.astype(np.int32)
    out["op"] = op.astype(np.int32)
    out["S"] = S
    out["hash"] = H
    return out


def schedule(n_submissions, k):
    """RunConsensus after every k submissions and after the last one."""
    k = max(1, int(k))
    pts = list(range(k, n_submissions + 1, k))
    if not pts or pts[-1] != n_submissions:
        pts.append(n_submissions)
    return np.array(pts, np.int64)
