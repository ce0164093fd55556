"""ctypes front-end of the CPU oracle (TEST INFRASTRUCTURE ONLY).

The oracle is a line-faithful C++ restatement of the reference Go hashgraph
(`/root/reference/hashgraph/hashgraph.go`, `roundInfo.go`,
`consensus_sorter.go`, `inmem_store.go`) — see hg_oracle.cpp.  Only tests/,
`__graft_entry__.smoke()` and bench.py's cpu_baseline leg may import this
module; the product engine never does.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libhg_oracle.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, i32, i64, u64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64
        P = ctypes.POINTER
        L.hgo_create.restype = vp
        L.hgo_create.argtypes = [ctypes.c_int, u64]
        L.hgo_create2.restype = vp
        L.hgo_create2.argtypes = [ctypes.c_int, u64, ctypes.c_int]
        L.hgo_set_release.argtypes = [vp, ctypes.c_int]
        L.hgo_is_scale.argtypes = [vp]
        L.hgo_is_scale.restype = ctypes.c_int
        L.hgo_event_rounds.argtypes = [vp, P(i32), P(ctypes.c_uint8)]
        L.hgo_event_received.argtypes = [vp, P(i32), P(i64)]
        L.hgo_fame_table.argtypes = [vp, P(ctypes.c_int8), ctypes.c_int]
        L.hgo_destroy.argtypes = [vp]
        L.hgo_last_error.restype = ctypes.c_char_p
        L.hgo_last_error.argtypes = [vp]
        L.hgo_insert.restype = ctypes.c_int
        L.hgo_insert.argtypes = [vp, ctypes.c_int, i64, ctypes.c_int, ctypes.c_int, i64,
                                 ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]
        for name in ("hgo_divide_rounds", "hgo_decide_fame", "hgo_decide_round_received",
                     "hgo_run_consensus"):
            getattr(L, name).argtypes = [vp]
            getattr(L, name).restype = None
        L.hgo_find_order.argtypes = [vp]
        for name in ("hgo_event_count", "hgo_rounds", "hgo_last_consensus_round",
                     "hgo_last_committed_round_events"):
            getattr(L, name).argtypes = [vp]
            getattr(L, name).restype = ctypes.c_int
        for name in ("hgo_consensus_transactions", "hgo_consensus_count"):
            getattr(L, name).argtypes = [vp]
            getattr(L, name).restype = i64
        L.hgo_consensus_events.argtypes = [vp, P(i32), i64]
        L.hgo_consensus_events.restype = i64
        L.hgo_undetermined.argtypes = [vp, P(i32), i64]
        L.hgo_undetermined.restype = i64
        L.hgo_known.argtypes = [vp, P(i32)]
        for name in ("hgo_round", "hgo_parent_round", "hgo_witness", "hgo_round_inc",
                     "hgo_round_received", "hgo_round_event_count"):
            getattr(L, name).argtypes = [vp, ctypes.c_int]
            getattr(L, name).restype = ctypes.c_int
        for name in ("hgo_ancestor", "hgo_self_ancestor", "hgo_see", "hgo_strongly_see",
                     "hgo_oldest_self_ancestor_to_see", "hgo_round_fame", "hgo_round_is_witness"):
            getattr(L, name).argtypes = [vp, ctypes.c_int, ctypes.c_int]
            getattr(L, name).restype = ctypes.c_int
        L.hgo_round_witnesses.argtypes = [vp, ctypes.c_int, P(i32), ctypes.c_int]
        L.hgo_round_witnesses.restype = ctypes.c_int
        L.hgo_consensus_timestamp.argtypes = [vp, ctypes.c_int]
        L.hgo_consensus_timestamp.restype = i64
        L.hgo_coords.argtypes = [vp, ctypes.c_int, P(i64), P(i32), P(i64), P(i32)]
        L.hgo_wire_info.argtypes = [vp, ctypes.c_int, P(i32)]
        L.hgo_set_round.argtypes = [vp, ctypes.c_int, P(i32), P(i32), P(i32), ctypes.c_int]
        L.hgo_stats.argtypes = [vp, P(i64), ctypes.c_int]
        L.hgo_replay.restype = i64
        L.hgo_replay.argtypes = [vp, i64, P(i32), P(i32), P(i32), P(i32), P(i64),
                                 ctypes.c_char_p, ctypes.c_char_p, P(i32), P(i64), i64,
                                 P(i32), P(i32), i64, P(i64)]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


class Oracle:
    """Go-shaped hashgraph (one `Hashgraph` + `InmemStore` with infinite caches).

    order_seed=0 iterates round witnesses in ascending creator id (the parity
    contract); any other seed emulates Go's randomised map iteration.

    scale=True selects the scale mode of hg_oracle.cpp (same results, computed
    without the memo caches and with bitset votes; canonical order only), and
    release_lag >= 0 lets it drop the coordinates of events ordered that many
    rounds behind LastConsensusRound (a later read of them aborts).
    """

    def __init__(self, n, order_seed=0, scale=False, release_lag=-1):
        self.L = lib()
        self.n = n
        self.h = self.L.hgo_create2(n, order_seed, 1 if scale else 0)
        if release_lag >= 0:
            self.L.hgo_set_release(self.h, release_lag)

    def close(self):
        if self.h:
            self.L.hgo_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- hashgraph.go API -------------------------------------------------
    def insert(self, creator, index, sp, op, ts, S=b"\0" * 32, hash32=b"\1" * 32, ntx=0):
        r = self.L.hgo_insert(self.h, creator, index, sp, op, ts, S, hash32, ntx)
        if r < 0:
            raise ValueError(self.L.hgo_last_error(self.h).decode())
        return r

    def divide_rounds(self):
        self.L.hgo_divide_rounds(self.h)

    def decide_fame(self):
        self.L.hgo_decide_fame(self.h)

    def decide_round_received(self):
        self.L.hgo_decide_round_received(self.h)

    def find_order(self):
        return self.L.hgo_find_order(self.h)

    def run_consensus(self):
        self.L.hgo_run_consensus(self.h)

    def rounds(self):
        return self.L.hgo_rounds(self.h)

    def last_consensus_round(self):
        r = self.L.hgo_last_consensus_round(self.h)
        return None if r < 0 else r

    def last_committed_round_events(self):
        return self.L.hgo_last_committed_round_events(self.h)

    def consensus_transactions(self):
        return self.L.hgo_consensus_transactions(self.h)

    def consensus_events(self):
        m = self.L.hgo_consensus_count(self.h)
        out = np.zeros(max(m, 1), np.int32)
        self.L.hgo_consensus_events(self.h, _p(out, ctypes.c_int32), m)
        return out[:m]

    def undetermined(self):
        m = self.L.hgo_undetermined(self.h, None, 0)
        out = np.zeros(max(m, 1), np.int32)
        self.L.hgo_undetermined(self.h, _p(out, ctypes.c_int32), m)
        return out[:m]

    def known(self):
        out = np.zeros(self.n, np.int32)
        self.L.hgo_known(self.h, _p(out, ctypes.c_int32))
        return out

    def round(self, x):
        return self.L.hgo_round(self.h, x)

    def parent_round(self, x):
        return self.L.hgo_parent_round(self.h, x)

    def witness(self, x):
        return bool(self.L.hgo_witness(self.h, x))

    def round_inc(self, x):
        return bool(self.L.hgo_round_inc(self.h, x))

    def round_diff(self, x, y):
        return self.round(x) - self.round(y)

    def ancestor(self, x, y):
        return bool(self.L.hgo_ancestor(self.h, x, y))

    def self_ancestor(self, x, y):
        return bool(self.L.hgo_self_ancestor(self.h, x, y))

    def see(self, x, y):
        return bool(self.L.hgo_see(self.h, x, y))

    def strongly_see(self, x, y):
        return bool(self.L.hgo_strongly_see(self.h, x, y))

    def oldest_self_ancestor_to_see(self, x, y):
        r = self.L.hgo_oldest_self_ancestor_to_see(self.h, x, y)
        return None if r < 0 else r

    def round_fame(self, r, x):
        return self.L.hgo_round_fame(self.h, r, x)

    def round_witnesses(self, r):
        out = np.zeros(max(self.n, 1) * 4, np.int32)
        m = self.L.hgo_round_witnesses(self.h, r, _p(out, ctypes.c_int32), len(out))
        return sorted(out[:m].tolist())

    def round_event_count(self, r):
        return self.L.hgo_round_event_count(self.h, r)

    def round_received(self, x):
        r = self.L.hgo_round_received(self.h, x)
        return None if r < 0 else r

    def consensus_timestamp(self, x):
        return self.L.hgo_consensus_timestamp(self.h, x)

    def coords(self, x):
        la = np.zeros(self.n, np.int64)
        lah = np.zeros(self.n, np.int32)
        fd = np.zeros(self.n, np.int64)
        fdh = np.zeros(self.n, np.int32)
        self.L.hgo_coords(self.h, x, _p(la, ctypes.c_int64), _p(lah, ctypes.c_int32),
                          _p(fd, ctypes.c_int64), _p(fdh, ctypes.c_int32))
        return la, lah, fd, fdh

    def wire_info(self, x):
        out = np.zeros(4, np.int32)
        self.L.hgo_wire_info(self.h, x, _p(out, ctypes.c_int32))
        return tuple(int(v) for v in out)

    def stats(self):
        """DecideFame instrumentation: coin-branch evaluations, coin votes,
        re-decided witnesses, re-decisions that changed the value."""
        out = np.zeros(4, np.int64)
        self.L.hgo_stats(self.h, _p(out, ctypes.c_int64), 4)
        return dict(zip(("coin_evals", "coin_votes", "redecided", "flipped"), out.tolist()))

    def is_scale(self):
        return bool(self.L.hgo_is_scale(self.h))

    def event_rounds(self):
        """Round and witness flag of every event (bulk Round / Witness)."""
        E = self.L.hgo_event_count(self.h)
        r = np.zeros(max(E, 1), np.int32)
        w = np.zeros(max(E, 1), np.uint8)
        self.L.hgo_event_rounds(self.h, _p(r, ctypes.c_int32), _p(w, ctypes.c_uint8))
        return r[:E], w[:E]

    def event_received(self):
        """Round received (-1 = none) and consensus timestamp (0 = none) of every event."""
        E = self.L.hgo_event_count(self.h)
        rr = np.zeros(max(E, 1), np.int32)
        cts = np.zeros(max(E, 1), np.int64)
        self.L.hgo_event_received(self.h, _p(rr, ctypes.c_int32), _p(cts, ctypes.c_int64))
        return rr[:E], cts[:E]

    def fame_table(self):
        """fame[r, creator] of every witness slot: -1 none, 0 undefined, 1 true, 2 false."""
        R = self.rounds()
        out = np.zeros((max(R, 1), self.n), np.int8)
        self.L.hgo_fame_table(self.h, _p(out, ctypes.c_int8), R)
        return out[:R]

    def set_round(self, r, entries):
        """entries: list of (id, witness: bool, fame: 0/1/2) (Store.SetRound)."""
        ids = np.array([e[0] for e in entries], np.int32)
        w = np.array([int(e[1]) for e in entries], np.int32)
        f = np.array([e[2] for e in entries], np.int32)
        self.L.hgo_set_round(self.h, r, _p(ids, ctypes.c_int32), _p(w, ctypes.c_int32),
                             _p(f, ctypes.c_int32), len(ids))


def replay(dag, call_points, order_seed=0, scale=False, release_lag=-1):
    """Run the Go-shaped path over a whole submission stream.

    dag: dict of numpy arrays (creator, index, sp, op, ts, S[n,32] u8, hash[n,32] u8, ntx)
    call_points: ascending 1-based submission counts after which RunConsensus runs.
    scale / release_lag: see Oracle.
    Returns (oracle, status, order, call_counts).
    """
    o = Oracle(int(dag["n"]), order_seed, scale=scale, release_lag=release_lag)
    n_sub = len(dag["creator"])
    cp = np.ascontiguousarray(call_points, np.int64)
    status = np.zeros(n_sub, np.int32)
    order = np.zeros(max(n_sub, 1), np.int32)
    counts = np.zeros(max(len(cp), 1), np.int64)
    c = {k: np.ascontiguousarray(dag[k], np.int32) for k in ("creator", "index", "sp", "op", "ntx")}
    ts = np.ascontiguousarray(dag["ts"], np.int64)
    S = np.ascontiguousarray(dag["S"], np.uint8)
    H = np.ascontiguousarray(dag["hash"], np.uint8)
    m = o.L.hgo_replay(o.h, n_sub, _p(c["creator"], ctypes.c_int32), _p(c["index"], ctypes.c_int32),
                       _p(c["sp"], ctypes.c_int32), _p(c["op"], ctypes.c_int32),
                       _p(ts, ctypes.c_int64), S.ctypes.data_as(ctypes.c_char_p),
                       H.ctypes.data_as(ctypes.c_char_p), _p(c["ntx"], ctypes.c_int32),
                       _p(cp, ctypes.c_int64), len(cp), _p(status, ctypes.c_int32),
                       _p(order, ctypes.c_int32), len(order), _p(counts, ctypes.c_int64))
    return o, status, order[:m], counts[:len(cp)]
