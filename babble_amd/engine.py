"""ctypes front-end of the MI355X engine's C ABI (include/hge.h).

`Engine` mirrors the methods of babble's Go `hashgraph.Hashgraph` that the
caller (node/core.go) uses — InsertEvent, DivideRounds, DecideFame,
DecideRoundReceived, FindOrder, ConsensusEvents, Known — plus the predicates
the reference's tests call.  Events are addressed by the dense ids the engine
assigns in insertion order.  The library is the product path: if it is
missing or cannot load, this module raises — there is no CPU fallback.
"""
import ctypes
import os

import numpy as np

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("HGE_LIB", os.path.join(_ROOT, "build", "libhge.so"))

HGE_NONE = -1
HGE_UNKNOWN = -2

ERRORS = {
    -1: "Could not find fake creator id",
    -2: "Self-parent not known",
    -3: "Self-parent has different creator",
    -4: "Other-parent not known",
    -5: "Self-parent not last known event by creator",
    -6: "Event index does not match the creator's chain position",
    -7: "Chain capacity exceeded",
    -11: "too late",
    -12: "not found",
}
HGE_ERR_CAPACITY = -7
HGE_ERR_TOO_LATE = -11
HGE_ERR_NOT_FOUND = -12
HGE_ERR_SIGNATURE = -13
HGE_ERR_SPLIT = -14

# hge_exchange_fn (include/hge.h): op 0 -> *buf = device memory for nparts slots of
# bytes_per_part bytes; op 1 -> all-gather the slots in place
EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64,
                               ctypes.POINTER(ctypes.c_void_p))


class HgeEvent(ctypes.Structure):
    _fields_ = [
        ("creator", ctypes.c_int32),
        ("index", ctypes.c_int32),
        ("self_parent", ctypes.c_int32),
        ("other_parent", ctypes.c_int32),
        ("timestamp_ns", ctypes.c_int64),
        ("s", ctypes.c_uint8 * 32),
        ("hash", ctypes.c_uint8 * 32),
        ("n_tx", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


EVENT_DTYPE = np.dtype([
    ("creator", "<i4"), ("index", "<i4"), ("self_parent", "<i4"), ("other_parent", "<i4"),
    ("timestamp_ns", "<i8"), ("s", "u1", (32,)), ("hash", "u1", (32,)), ("n_tx", "<i4"),
    ("reserved", "<i4"),
])
assert EVENT_DTYPE.itemsize == ctypes.sizeof(HgeEvent)

EXPORTS = [
    "hge_create", "hge_destroy", "hge_last_error", "hge_reset", "hge_insert_events",
    "hge_divide_rounds", "hge_decide_fame", "hge_decide_round_received", "hge_find_order",
    "hge_run_consensus", "hge_replay", "hge_replay_prepare", "hge_replay_run",
    "hge_replay_fetch", "hge_replay_order", "hge_event_count", "hge_participants", "hge_rounds",
    "hge_last_consensus_round", "hge_last_committed_round_events",
    "hge_consensus_transactions", "hge_consensus_count", "hge_consensus_events",
    "hge_undetermined", "hge_known", "hge_round_of", "hge_is_witness", "hge_round_witness",
    "hge_fame", "hge_round_events", "hge_round_received", "hge_consensus_timestamp",
    "hge_consensus_timestamp_sources",
    "hge_ancestor", "hge_self_ancestor", "hge_see", "hge_strongly_see",
    "hge_oldest_self_ancestor_to_see", "hge_coordinates", "hge_coordinate_sweeps", "hge_host_syncs", "hge_frontier_fallbacks",
    "hge_stage_times",
    "hge_set_profiling", "hge_reset_kernel_stats", "hge_kernel_stats",
    "hge_consensus_log", "hge_event_rounds", "hge_event_received", "hge_set_cache_size",
    "hge_cache_size", "hge_participant_events", "hge_participant_event", "hge_last_from",
    "hge_diff", "hge_wire_info", "hge_read_wire_parents", "hge_parent_round", "hge_round_inc",
    "hge_round_diff", "hge_set_round", "hge_round_event_ids", "hge_split_begin", "hge_frontier_guess",
    "hge_frontier_walk", "hge_split_finish", "hge_frontier_rows", "hge_split_plan", "hge_split_exchange", "hge_split_run", "hge_split_emulate",
    "hge_verify_events", "hge_sha256_batch", "hge_ingest", "hge_fame_table",
    # the standalone Store (host only; the Go shim's NewInmemStore, tests/abi/hge_store_test.cpp)
    "hge_store_create", "hge_store_destroy", "hge_store_set_event", "hge_store_has_event",
    "hge_store_participant_events", "hge_store_participant_event", "hge_store_last_from",
    "hge_store_known", "hge_store_add_consensus_event", "hge_store_consensus_events",
    "hge_store_consensus_count", "hge_store_set_round", "hge_store_get_round", "hge_store_rounds",
    "hge_store_round_witnesses", "hge_store_round_events",
    # a batch of independent hashgraphs (config 5, hge_batch.hip)
    "hge_batch_create", "hge_batch_destroy", "hge_batch_last_error", "hge_batch_add", "hge_batch_stage",
    "hge_batch_run", "hge_batch_graphs", "hge_batch_info", "hge_batch_results", "hge_batch_kernel_ms",
    "hge_batch_fallbacks",
    # the wire / hashing format (host only, hge_gob.cpp)
    "hge_gob_encode_wire_events", "hge_gob_decode_wire_events", "hge_gob_encode_event_body",
]

_lib = None


class HgeError(RuntimeError):
    """A negative hge_status.  `accepted` holds the ids the engine assigned
    before the failing event of an insert batch (they stay inserted)."""

    def __init__(self, code, msg, accepted=None):
        super().__init__(f"{msg} (hge status {code})")
        self.code = code
        self.accepted = accepted


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"HIP engine library not built: {LIB_PATH} (run __graft_entry__.build())")
    # torch (the collectives' plumbing, babble_amd.dist) ships its own HIP runtime; it
    # must be mapped before this library maps /opt/rocm's, or torch's runtime finds no
    # GPU in this process (measured on the MI355X box)
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    P = ctypes.POINTER
    L.hge_create.argtypes = [i32, i64, i32, ctypes.c_uint32, P(vp)]
    L.hge_destroy.argtypes = [vp]
    L.hge_destroy.restype = None
    L.hge_last_error.argtypes = [vp]
    L.hge_last_error.restype = ctypes.c_char_p
    L.hge_reset.argtypes = [vp]
    L.hge_insert_events.argtypes = [vp, ctypes.c_void_p, i64, P(i32), P(i64)]
    for f in ("hge_divide_rounds", "hge_decide_fame", "hge_decide_round_received"):
        getattr(L, f).argtypes = [vp]
    for f in ("hge_find_order", "hge_run_consensus"):
        getattr(L, f).argtypes = [vp, P(i32), i64, P(i64)]
    L.hge_replay.argtypes = [vp, ctypes.c_void_p, i64, P(i64), i64, P(i32), P(i32), i64, P(i64),
                             P(i64)]
    L.hge_replay_prepare.argtypes = [vp, ctypes.c_void_p, i64, P(i64), i64, P(i32)]
    L.hge_replay_run.argtypes = [vp, P(i64)]
    L.hge_replay_fetch.argtypes = [vp, P(i32), i64, P(i64)]
    L.hge_replay_order.argtypes = [vp, P(P(i32)), P(i64)]
    for f in ("hge_event_count", "hge_consensus_transactions", "hge_consensus_count"):
        getattr(L, f).argtypes = [vp]
        getattr(L, f).restype = i64
    for f in ("hge_participants", "hge_rounds", "hge_last_consensus_round",
              "hge_last_committed_round_events"):
        getattr(L, f).argtypes = [vp]
        getattr(L, f).restype = i32
    for f in ("hge_consensus_events", "hge_undetermined"):
        getattr(L, f).argtypes = [vp, P(i32), i64]
        getattr(L, f).restype = i64
    L.hge_known.argtypes = [vp, P(i32)]
    for f in ("hge_round_of", "hge_is_witness", "hge_round_events", "hge_round_received"):
        getattr(L, f).argtypes = [vp, i32]
        getattr(L, f).restype = i32
    L.hge_consensus_timestamp.argtypes = [vp, i32]
    L.hge_consensus_timestamp.restype = i64
    for f in ("hge_round_witness", "hge_fame", "hge_ancestor", "hge_self_ancestor", "hge_see",
              "hge_strongly_see", "hge_oldest_self_ancestor_to_see"):
        getattr(L, f).argtypes = [vp, i32, i32]
        getattr(L, f).restype = i32
    L.hge_coordinates.argtypes = [vp, i32, P(i32), P(i32)]
    L.hge_stage_times.argtypes = [vp, P(ctypes.c_float), ctypes.c_int]
    L.hge_coordinate_sweeps.restype = ctypes.c_int32
    L.hge_coordinate_sweeps.argtypes = [vp]
    if hasattr(L, "hge_gob_encode_wire_events"):
        L.hge_gob_encode_wire_events.argtypes = [vp, i64, P(ctypes.c_uint8), P(i64), i32, P(ctypes.c_uint8), i64,
                                                 P(i64)]
        L.hge_gob_decode_wire_events.argtypes = [P(ctypes.c_uint8), i64, vp, i64, P(ctypes.c_uint8), i64, P(i64),
                                                 i64, P(i64), P(i64), P(i64)]
        L.hge_gob_encode_event_body.argtypes = [vp, P(ctypes.c_uint8), P(i64), P(ctypes.c_uint8), P(i64), i32,
                                                P(ctypes.c_uint8), i64, P(i64)]
    if hasattr(L, "hge_host_syncs"):
        L.hge_host_syncs.restype = i64
        L.hge_host_syncs.argtypes = [vp]
    L.hge_frontier_fallbacks.restype = i64
    L.hge_frontier_fallbacks.argtypes = [vp]
    L.hge_consensus_log.argtypes = [vp, i64, P(i32), i64]
    L.hge_consensus_log.restype = i64
    L.hge_event_rounds.argtypes = [vp, P(i32), P(ctypes.c_uint8), i64]
    L.hge_event_received.argtypes = [vp, P(i32), P(i64), i64]
    L.hge_consensus_timestamp_sources.argtypes = [vp, P(i32), i64, P(i32)]
    L.hge_fame_table.argtypes = [vp, i32, P(ctypes.c_int8)]
    L.hge_fame_table.restype = i32
    L.hge_set_cache_size.argtypes = [vp, i64]
    L.hge_cache_size.argtypes = [vp]
    L.hge_cache_size.restype = i64
    L.hge_participant_events.argtypes = [vp, i32, i64, P(i32), i64, P(i64)]
    L.hge_participant_event.argtypes = [vp, i32, i64]
    L.hge_participant_event.restype = i32
    L.hge_last_from.argtypes = [vp, i32]
    L.hge_last_from.restype = i32
    L.hge_diff.argtypes = [vp, P(i32), P(i32), i64, P(i64)]
    L.hge_wire_info.argtypes = [vp, i32, P(i32)]
    L.hge_read_wire_parents.argtypes = [vp, i32, i32, i32, i32, P(i32), P(i32)]
    L.hge_parent_round.argtypes = [vp, i32]
    L.hge_parent_round.restype = i32
    L.hge_round_inc.argtypes = [vp, i32]
    L.hge_round_inc.restype = i32
    L.hge_round_diff.argtypes = [vp, i32, i32, P(i32)]
    L.hge_set_round.argtypes = [vp, i32, P(i32), P(ctypes.c_uint8), P(ctypes.c_uint8), i32]
    if hasattr(L, "hge_round_event_ids"):
        L.hge_round_event_ids.argtypes = [vp, i32, P(i32), P(ctypes.c_uint8), i64, P(i64)]
    L.hge_split_begin.argtypes = [vp]
    L.hge_frontier_guess.argtypes = [vp, i32, i32, P(i32)]
    L.hge_frontier_walk.argtypes = [vp, P(i32), P(i32), i32, i32, P(i32), P(ctypes.c_uint64), P(i32), P(i32)]
    L.hge_split_finish.argtypes = [vp, P(i32), P(ctypes.c_uint64), i32, i32, P(i64)]
    L.hge_frontier_rows.argtypes = [vp, i32, i32, P(i32), P(ctypes.c_uint64)]
    if hasattr(L, "hge_split_run"):  # (a diagnostic build of an older tree, HGE_LIB, may lack them)
        L.hge_split_plan.argtypes = [vp, i32, i32, P(i64), P(i32), P(i64)]
        L.hge_split_run.argtypes = [vp, P(i64)]
        L.hge_split_exchange.argtypes = [vp, EXCHANGE_FN, vp]
    if hasattr(L, "hge_split_emulate"):
        L.hge_split_emulate.argtypes = [vp, i32]
    u8p = P(ctypes.c_uint8)
    L.hge_verify_events.argtypes = [i64, u8p, P(i64), u8p, u8p, i32, u8p, P(i32)]
    L.hge_sha256_batch.argtypes = [i64, u8p, P(i64), i32, u8p]
    L.hge_ingest.argtypes = [vp, ctypes.c_void_p, i64, u8p, P(i64), u8p, u8p, i64, i32, P(i32), P(i64),
                             P(ctypes.c_double)]
    L.hge_set_profiling.argtypes = [vp, ctypes.c_int]
    L.hge_reset_kernel_stats.argtypes = [vp]
    L.hge_kernel_stats.argtypes = [vp, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                   P(ctypes.c_double), P(i64)]
    L.hge_batch_create.argtypes = [i32, i32, P(vp)]
    L.hge_batch_destroy.argtypes = [vp]
    L.hge_batch_destroy.restype = None
    L.hge_batch_last_error.argtypes = [vp]
    L.hge_batch_last_error.restype = ctypes.c_char_p
    L.hge_batch_add.argtypes = [vp, ctypes.c_void_p, i64, P(i64), i64, P(i32), P(i32)]
    L.hge_batch_stage.argtypes = [vp]
    L.hge_batch_run.argtypes = [vp, P(i64)]
    L.hge_batch_graphs.argtypes = [vp]
    L.hge_batch_graphs.restype = i32
    L.hge_batch_info.argtypes = [vp, i32, P(i64)]
    L.hge_batch_results.argtypes = [vp, i32, P(i32), P(i64), P(i32), P(ctypes.c_uint8), P(i32), P(i64),
                                    P(ctypes.c_int8), P(i32)]
    L.hge_batch_kernel_ms.argtypes = [vp, P(ctypes.c_float), i32]
    L.hge_batch_fallbacks.argtypes = [vp]
    L.hge_batch_fallbacks.restype = ctypes.c_int64
    _lib = L
    return L


def _p32(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


def _p64(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))


def _pu8(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def _flat(bodies):
    """(flat uint8 bytes, int64 offsets[n+1]) from a list of bytes or a (flat, off) pair."""
    if isinstance(bodies, tuple):
        flat, off = bodies
        return np.ascontiguousarray(flat, np.uint8), np.ascontiguousarray(off, np.int64)
    off = np.zeros(len(bodies) + 1, np.int64)
    off[1:] = np.cumsum([len(b) for b in bodies])
    flat = np.frombuffer(b"".join(bodies), np.uint8) if off[-1] else np.zeros(1, np.uint8)
    return np.ascontiguousarray(flat), off


def verify_events(bodies, pubs, sigs, threads=0):
    """Event.Verify for a batch on host threads (hge_verify_events): returns
    (ok bool[n], body hashes uint8[n, 32]).  bodies: list of bytes or (flat, off);
    pubs uint8[n, 65]; sigs uint8[n, 64] (r || s)."""
    flat, off = _flat(bodies)
    n = len(off) - 1
    pubs = np.ascontiguousarray(pubs, np.uint8).reshape(n, 65)
    sigs = np.ascontiguousarray(sigs, np.uint8).reshape(n, 64)
    ok = np.zeros(max(n, 1), np.int32)
    hashes = np.zeros((max(n, 1), 32), np.uint8)
    rc = lib().hge_verify_events(n, _pu8(flat), _p64(off), _pu8(pubs), _pu8(sigs), threads, _pu8(hashes), _p32(ok))
    if rc != 0:
        raise HgeError(rc, "hge_verify_events failed")
    return ok[:n].astype(bool), hashes[:n]


class GobTime(ctypes.Structure):
    _fields_ = [("unix_sec", ctypes.c_int64), ("nsec", ctypes.c_int32), ("offset_min", ctypes.c_int16),
                ("set", ctypes.c_int16)]


class WireEvent(ctypes.Structure):
    """hge_wire_event (include/hge.h): a babble WireEvent (hashgraph/event.go:244-259)."""
    _fields_ = [("self_parent_index", ctypes.c_int64), ("other_parent_creator_id", ctypes.c_int64),
                ("other_parent_index", ctypes.c_int64), ("creator_id", ctypes.c_int64), ("index", ctypes.c_int64),
                ("timestamp", GobTime), ("r", ctypes.c_uint8 * 32), ("s", ctypes.c_uint8 * 32),
                ("r_set", ctypes.c_int32), ("s_set", ctypes.c_int32), ("tx_first", ctypes.c_int64),
                ("tx_count", ctypes.c_int32), ("pad", ctypes.c_int32)]


class GobBody(ctypes.Structure):
    _fields_ = [("tx_count", ctypes.c_int32), ("n_parents", ctypes.c_int32),
                ("creator", ctypes.POINTER(ctypes.c_uint8)), ("creator_len", ctypes.c_int64),
                ("timestamp", GobTime), ("index", ctypes.c_int64)]


WIRE_INT_FIELDS = ("self_parent_index", "other_parent_creator_id", "other_parent_index", "creator_id", "index")


def _gob_time(ts):
    """(unix_sec, nsec, offset_min) or None (the zero time.Time)."""
    if ts is None:
        return GobTime(0, 0, 0, 0)
    return GobTime(int(ts[0]), int(ts[1]), int(ts[2]), 1)


def gob_encode_wire_events(events, first_type_id=65):
    """One gob encoder's stream of WireEvents (hge_gob_encode_wire_events).  events:
    dicts with the WIRE_INT_FIELDS, "timestamp" (unix_sec, nsec, offset_min | None),
    "r" / "s" (non-negative ints < 2**256 | None), "transactions" (list of bytes)."""
    n = len(events)
    arr = (WireEvent * max(n, 1))()
    txs = []
    for k, e in enumerate(events):
        w = arr[k]
        for f in WIRE_INT_FIELDS:
            setattr(w, f, int(e.get(f, 0)))
        w.timestamp = _gob_time(e.get("timestamp"))
        for name in ("r", "s"):
            v = e.get(name)
            if v is not None:
                getattr(w, name)[:] = list(int(v).to_bytes(32, "big"))
                setattr(w, name + "_set", 1)
        w.tx_first = len(txs)
        w.tx_count = len(e.get("transactions", []))
        txs.extend(e.get("transactions", []))
    flat, off = _flat(txs)
    L = lib()
    nout = ctypes.c_int64()
    rc = L.hge_gob_encode_wire_events(arr, n, _pu8(flat), _p64(off), first_type_id, None, 0, ctypes.byref(nout))
    if rc != 0:
        raise HgeError(rc, "hge_gob_encode_wire_events failed")
    out = np.zeros(max(1, nout.value), np.uint8)
    rc = L.hge_gob_encode_wire_events(arr, n, _pu8(flat), _p64(off), first_type_id, _pu8(out), nout.value,
                                      ctypes.byref(nout))
    if rc != 0:
        raise HgeError(rc, "hge_gob_encode_wire_events failed")
    return out[:nout.value].tobytes()


def gob_decode_wire_events(buf):
    """Every WireEvent in a gob stream (hge_gob_decode_wire_events), as the dicts
    gob_encode_wire_events takes."""
    b = np.frombuffer(bytes(buf), np.uint8) if len(buf) else np.zeros(1, np.uint8)
    L = lib()
    ne, nt, nb = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    rc = L.hge_gob_decode_wire_events(_pu8(b), len(buf), None, 0, None, 0, None, 0, ctypes.byref(ne),
                                      ctypes.byref(nt), ctypes.byref(nb))
    if rc not in (0, -12):
        raise HgeError(rc, "not a gob stream of WireEvents")
    arr = (WireEvent * max(1, ne.value))()
    tx = np.zeros(max(1, nb.value), np.uint8)
    off = np.zeros(nt.value + 1, np.int64)
    rc = L.hge_gob_decode_wire_events(_pu8(b), len(buf), arr, ne.value, _pu8(tx), nb.value, _p64(off), len(off),
                                      ctypes.byref(ne), ctypes.byref(nt), ctypes.byref(nb))
    if rc != 0:
        raise HgeError(rc, "not a gob stream of WireEvents")
    out = []
    for k in range(ne.value):
        w = arr[k]
        e = {f: int(getattr(w, f)) for f in WIRE_INT_FIELDS}
        t = w.timestamp
        e["timestamp"] = (int(t.unix_sec), int(t.nsec), int(t.offset_min)) if t.set else None
        e["r"] = int.from_bytes(bytes(w.r), "big") if w.r_set else None
        e["s"] = int.from_bytes(bytes(w.s), "big") if w.s_set else None
        e["transactions"] = [tx[off[w.tx_first + j]:off[w.tx_first + j + 1]].tobytes() for j in range(w.tx_count)]
        out.append(e)
    return out


def gob_encode_event_body(transactions, parents, creator, timestamp, index, first_type_id=65):
    """EventBody.Marshal (hge_gob_encode_event_body): the bytes Sign/Verify hash."""
    tflat, toff = _flat(list(transactions))
    pflat, poff = _flat([p.encode() for p in parents])
    cr = np.frombuffer(bytes(creator), np.uint8) if len(creator) else np.zeros(1, np.uint8)
    body = GobBody(len(transactions), len(parents), _pu8(cr), len(creator), _gob_time(timestamp), int(index))
    L = lib()
    nout = ctypes.c_int64()
    rc = L.hge_gob_encode_event_body(ctypes.byref(body), _pu8(tflat), _p64(toff), _pu8(pflat), _p64(poff),
                                     first_type_id, None, 0, ctypes.byref(nout))
    if rc != 0:
        raise HgeError(rc, "hge_gob_encode_event_body failed")
    out = np.zeros(max(1, nout.value), np.uint8)
    rc = L.hge_gob_encode_event_body(ctypes.byref(body), _pu8(tflat), _p64(toff), _pu8(pflat), _p64(poff),
                                     first_type_id, _pu8(out), nout.value, ctypes.byref(nout))
    if rc != 0:
        raise HgeError(rc, "hge_gob_encode_event_body failed")
    return out[:nout.value].tobytes()


def sha256_batch(data, threads=0):
    """SHA-256 of each byte string (hge_sha256_batch): uint8[n, 32]."""
    flat, off = _flat(data)
    n = len(off) - 1
    out = np.zeros((max(n, 1), 32), np.uint8)
    rc = lib().hge_sha256_batch(n, _pu8(flat), _p64(off), threads, _pu8(out))
    if rc != 0:
        raise HgeError(rc, "hge_sha256_batch failed")
    return out[:n]


def events_array(dag):
    """Pack a submission-stream dict (babble_amd.gossip layout) into hge_event records.
    Parents stay submission indices (hge_replay's convention)."""
    E = len(dag["creator"])
    ev = np.zeros(E, EVENT_DTYPE)
    ev["creator"] = dag["creator"]
    ev["index"] = dag["index"]
    ev["self_parent"] = dag["sp"]
    ev["other_parent"] = dag["op"]
    ev["timestamp_ns"] = dag["ts"]
    ev["s"] = dag["S"]
    ev["hash"] = dag["hash"]
    ev["n_tx"] = dag.get("ntx", np.zeros(E, np.int32))
    return ev


class Engine:
    """One hashgraph (Hashgraph + Store) resident on one GPU."""

    def __init__(self, n_participants, capacity_events=1 << 16, device=0):
        self.L = lib()
        h = ctypes.c_void_p()
        rc = self.L.hge_create(n_participants, capacity_events, device, 0, ctypes.byref(h))
        if rc != 0:
            raise HgeError(rc, "hge_create failed")
        self.h = h
        self.n = n_participants
        self._obuf = None

    def close(self):
        if getattr(self, "h", None):
            self.L.hge_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != 0:
            xe, self._xerr = getattr(self, "_xerr", None), None
            if xe is not None:
                raise HgeError(rc, self.L.hge_last_error(self.h).decode()) from xe
            raise HgeError(rc, self.L.hge_last_error(self.h).decode())
        return rc

    # --- ingest ----------------------------------------------------------
    def insert_events(self, ev):
        """InsertEvent for each record (stops at the first rejection, like Core.Sync).
        Returns the assigned ids; on the first rejected event raises HgeError
        whose `accepted` holds the ids of the events inserted before it."""
        ev = np.ascontiguousarray(ev, EVENT_DTYPE)
        status = np.zeros(len(ev), np.int32)
        acc = ctypes.c_int64()
        rc = self.L.hge_insert_events(self.h, ev.ctypes.data, len(ev), _p32(status), ctypes.byref(acc))
        if rc != 0:
            raise HgeError(rc, self.L.hge_last_error(self.h).decode(), accepted=status[:acc.value].copy())
        return status[:acc.value]

    def ingest(self, ev, bodies, keys, sigs, k, threads=0):
        """hge_ingest: InsertEvent with signature checks in batches of k, RunConsensus
        after each batch, the next batch verified on host threads meanwhile.
        keys: uint8[N, 65], participant c's key; event i is checked under
        keys[ev[i].creator] (a body signed by another participant is refused).
        Returns (rc, status int32[n], n_accepted, times {verify_ms, device_ms, wall_ms});
        rc is 0 or the negative status that ended the stream (HGE_ERR_SIGNATURE = -13)."""
        ev = np.ascontiguousarray(ev, EVENT_DTYPE)
        flat, off = _flat(bodies)
        n = len(ev)
        assert len(off) == n + 1
        keys = np.ascontiguousarray(keys, np.uint8).reshape(self.n, 65)
        sigs = np.ascontiguousarray(sigs, np.uint8).reshape(n, 64)
        status = np.zeros(max(n, 1), np.int32)
        acc = ctypes.c_int64()
        tm = (ctypes.c_double * 3)()
        rc = self.L.hge_ingest(self.h, ev.ctypes.data, n, _pu8(flat), _p64(off), _pu8(keys), _pu8(sigs), int(k),
                               threads, _p32(status), ctypes.byref(acc), tm)
        if rc in (-8, -9, -10):  # argument, device or internal error (admission errors end the stream)
            raise HgeError(rc, self.L.hge_last_error(self.h).decode())
        return rc, status[:n], acc.value, {"verify_ms": tm[0], "device_ms": tm[1], "wall_ms": tm[2]}

    def insert(self, creator, index, sp, op, ts, S=b"\0" * 32, hash32=b"\1" * 32, ntx=0):
        ev = np.zeros(1, EVENT_DTYPE)
        ev["creator"], ev["index"], ev["self_parent"], ev["other_parent"] = creator, index, sp, op
        ev["timestamp_ns"] = ts
        ev["s"][0] = np.frombuffer(S, np.uint8)
        ev["hash"][0] = np.frombuffer(hash32, np.uint8)
        ev["n_tx"] = ntx
        return int(self.insert_events(ev)[0])

    # --- consensus -------------------------------------------------------
    def divide_rounds(self):
        self._check(self.L.hge_divide_rounds(self.h))

    def decide_fame(self):
        self._check(self.L.hge_decide_fame(self.h))

    def decide_round_received(self):
        self._check(self.L.hge_decide_round_received(self.h))

    def _order_call(self, fn):
        # one output buffer for the engine's life, grown geometrically: a fresh
        # zeroed array of every event's size per call cost more than the call at
        # 1M events (~200 us)
        cap = max(1, int(self.L.hge_event_count(self.h)))
        if self._obuf is None or len(self._obuf) < cap:
            self._obuf = np.empty(max(cap, 2 * (0 if self._obuf is None else len(self._obuf))), np.int32)
        out = self._obuf
        n = ctypes.c_int64()
        self._check(fn(self.h, _p32(out), len(out), ctypes.byref(n)))
        return out[:n.value].copy()

    def find_order(self):
        return self._order_call(self.L.hge_find_order)

    def run_consensus(self):
        return self._order_call(self.L.hge_run_consensus)

    def replay(self, dag_or_events, call_points):
        ev = dag_or_events if isinstance(dag_or_events, np.ndarray) else events_array(dag_or_events)
        self.prepare(ev, call_points)
        self.run()
        return self.fetch()

    def prepare(self, ev, call_points):
        ev = np.ascontiguousarray(ev, EVENT_DTYPE)
        cp = np.ascontiguousarray(call_points, np.int64)
        self._status = np.zeros(len(ev), np.int32)
        self._ncalls = len(cp)
        self._calls = cp.copy()
        self._check(self.L.hge_replay_prepare(self.h, ev.ctypes.data, len(ev), _p64(cp), len(cp),
                                              _p32(self._status)))
        return self._status

    def run(self):
        n = ctypes.c_int64()
        self._check(self.L.hge_replay_run(self.h, ctypes.byref(n)))
        self._nordered = n.value
        return n.value

    def order_view(self):
        """The replay's order where hge_replay_run delivered it (pinned host memory), as a
        numpy view without a copy: valid until the next replay or consensus call."""
        p = ctypes.POINTER(ctypes.c_int32)()
        n = ctypes.c_int64()
        self._check(self.L.hge_replay_order(self.h, ctypes.byref(p), ctypes.byref(n)))
        if n.value == 0:
            return np.zeros(0, np.int32)
        return np.ctypeslib.as_array(p, shape=(n.value,))

    def fetch(self):
        order = np.zeros(max(1, self._nordered), np.int32)
        counts = np.zeros(max(1, self._ncalls), np.int64)
        self._check(self.L.hge_replay_fetch(self.h, _p32(order), len(order), _p64(counts)))
        return self._status, order[:self._nordered], counts[:self._ncalls]

    # --- one hashgraph split across GPUs (babble_amd.dist.split_run) ----
    def call_events(self):
        """Events accepted at each call point of the staged replay (hge_replay_prepare)."""
        acc = np.cumsum(self._status >= 0)
        return acc[self._calls - 1].astype(np.int64)

    def split_plan(self, part, nparts, plan=None):
        """hge_split_plan: shard the staged replay by time (babble_amd.dist.split_plan);
        nparts <= 1 clears the plan."""
        if nparts <= 1 or plan is None:
            self._check(self.L.hge_split_plan(self.h, 0, 0, None, None, None))
            return
        evb = np.ascontiguousarray(plan["ev_bounds"], np.int64)
        cb = np.ascontiguousarray(plan["call_bounds"], np.int32)
        clo = np.ascontiguousarray(plan["cand_lo"], np.int64)
        self._check(self.L.hge_split_plan(self.h, part, nparts, _p64(evb), _p32(cb), _p64(clo)))

    def clear_exchange(self):
        self._xcb = None
        self._check(self.L.hge_split_exchange(self.h, ctypes.cast(None, EXCHANGE_FN), None))

    def split_emulate(self, on=True):
        """hge_split_emulate: the next run() records every part's exchange slots; a
        split_run() without an exchange then takes the other parts' from the record."""
        self._check(self.L.hge_split_emulate(self.h, 1 if on else 0))

    def split_run(self):
        """hge_split_run: this part of the sharded replay (plan + exchange set);
        returns the number of events ordered by the whole replay."""
        n = ctypes.c_int64()
        self._check(self.L.hge_split_run(self.h, ctypes.byref(n)))
        self._nordered = n.value
        return n.value

    def set_exchange(self, fn):
        """fn(op, bytes_per_part) -> device pointer (op 0) / None (op 1): the
        all-gather of a split replay (hge_split_exchange)."""
        def cb(_ctx, op, nbytes, bufp):
            try:
                r = fn(int(op), int(nbytes))
                if op == 0:
                    bufp[0] = r
                return 0
            except Exception as e:  # the engine fails the replay with HGE_ERR_DEVICE
                self._xerr = e
                return 1
        self._xcb = EXCHANGE_FN(cb)  # kept alive with the engine
        self._check(self.L.hge_split_exchange(self.h, self._xcb, None))

    def split_begin(self):
        self._check(self.L.hge_split_begin(self.h))

    def frontier_guess(self, part, nparts):
        out = np.zeros(self.n, np.int32)
        self._check(self.L.hge_frontier_guess(self.h, part, nparts, _p32(out)))
        return out

    def frontier_walk(self, start, stopcut=None, extra=0, hmax=None):
        """Rounds-frontier walk from `start`: (rows [n, N] int32, ssc [n, N, NW] uint64, natural).
        hmax bounds the rows (default: every chain advances at least one position per
        round, so the longest chain + 2 always suffices)."""
        nw = (self.n + 63) // 64
        if hmax is None:
            hmax = int(self.known().max()) + 2
        nr = ctypes.c_int32()
        nat = ctypes.c_int32()
        start = np.ascontiguousarray(start, np.int32)
        cut = None if stopcut is None else np.ascontiguousarray(stopcut, np.int32)
        self._check(self.L.hge_frontier_walk(self.h, _p32(start), None if cut is None else _p32(cut),
                                             extra, hmax, None, None, ctypes.byref(nr), ctypes.byref(nat)))
        n = nr.value
        rows = np.zeros((n, self.n), np.int32)
        ssc = np.zeros((n, self.n, nw), np.uint64)
        self._check(self.L.hge_frontier_rows(self.h, 0, n, _p32(rows),
                                             ssc.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))))
        return rows, ssc, bool(nat.value)

    def split_finish(self, rows, ssc, natural):
        rows = np.ascontiguousarray(rows, np.int32)
        ssc = np.ascontiguousarray(ssc, np.uint64)
        n = ctypes.c_int64()
        self._check(self.L.hge_split_finish(self.h, _p32(rows),
                                            ssc.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                            len(rows), 1 if natural else 0, ctypes.byref(n)))
        self._nordered = n.value
        return n.value

    def set_profiling(self, on=True):
        self.L.hge_set_profiling(self.h, 1 if on else 0)
        self.L.hge_reset_kernel_stats(self.h)

    def kernel_stats(self):
        """{kernel name: (total device ms, launches)} from HIP events on the engine stream."""
        out = {}
        n = self.L.hge_kernel_stats(self.h, -1, None, 0, None, None)
        buf = ctypes.create_string_buffer(128)
        for k in range(n):
            ms = ctypes.c_double()
            cnt = ctypes.c_int64()
            self.L.hge_kernel_stats(self.h, k, buf, 128, ctypes.byref(ms), ctypes.byref(cnt))
            out[buf.value.decode()] = (ms.value, cnt.value)
        return out

    def coordinate_sweeps(self):
        """lastAncestors sweeps of the last coordinate pass (hge_coords.hip)."""
        return self.L.hge_coordinate_sweeps(self.h)

    def host_syncs(self):
        """Host round trips so far (waits on the engine stream)."""
        return int(self.L.hge_host_syncs(self.h))

    def frontier_fallbacks(self):
        """Times the wide rounds walk timed out on its frontier hand-off and walked
        again launch per round (hge_frontier_fallbacks)."""
        return int(self.L.hge_frontier_fallbacks(self.h))

    def stage_times(self):
        out = (ctypes.c_float * 7)()
        n = self.L.hge_stage_times(self.h, out, 7)
        return list(out)[:n]

    # --- state -----------------------------------------------------------
    def event_count(self):
        return self.L.hge_event_count(self.h)

    def rounds(self):
        return self.L.hge_rounds(self.h)

    def last_consensus_round(self):
        r = self.L.hge_last_consensus_round(self.h)
        return None if r < 0 else r

    def last_committed_round_events(self):
        return self.L.hge_last_committed_round_events(self.h)

    def consensus_transactions(self):
        return self.L.hge_consensus_transactions(self.h)

    def consensus_events(self):
        """Store.ConsensusEvents: the rolling window (the whole list when the
        cache size is 0, the default)."""
        m = self.L.hge_consensus_events(self.h, None, 0)
        out = np.zeros(max(1, m), np.int32)
        self.L.hge_consensus_events(self.h, _p32(out), m)
        return out[:m]

    def undetermined(self):
        m = self.L.hge_undetermined(self.h, None, 0)
        out = np.zeros(max(1, m), np.int32)
        self.L.hge_undetermined(self.h, _p32(out), m)
        return out[:m]

    def known(self):
        out = np.zeros(self.n, np.int32)
        self.L.hge_known(self.h, _p32(out))
        return out

    def round(self, x):
        return self.L.hge_round_of(self.h, x)

    def witness(self, x):
        return bool(self.L.hge_is_witness(self.h, x))

    def round_witness(self, r, creator):
        w = self.L.hge_round_witness(self.h, r, creator)
        return None if w < 0 else w

    def round_witnesses(self, r):
        return sorted(w for w in (self.round_witness(r, c) for c in range(self.n)) if w is not None)

    def fame(self, r, creator):
        return self.L.hge_fame(self.h, r, creator)

    def round_events(self, r):
        return self.L.hge_round_events(self.h, r)

    def round_received(self, x):
        r = self.L.hge_round_received(self.h, x)
        return None if r < 0 else r

    def consensus_timestamp(self, x):
        return self.L.hge_consensus_timestamp(self.h, x)

    def ancestor(self, x, y):
        return bool(self.L.hge_ancestor(self.h, x, y))

    def self_ancestor(self, x, y):
        return bool(self.L.hge_self_ancestor(self.h, x, y))

    def see(self, x, y):
        return bool(self.L.hge_see(self.h, x, y))

    def strongly_see(self, x, y):
        return bool(self.L.hge_strongly_see(self.h, x, y))

    def oldest_self_ancestor_to_see(self, x, y):
        r = self.L.hge_oldest_self_ancestor_to_see(self.h, x, y)
        return None if r < 0 else r

    # --- bulk reads ------------------------------------------------------
    def event_rounds(self):
        """(round, witness) of every event (DivideRounds state)."""
        m = self.event_count()
        r = np.zeros(max(m, 1), np.int32)
        w = np.zeros(max(m, 1), np.uint8)
        self._check(self.L.hge_event_rounds(self.h, _p32(r), w.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), m))
        return r[:m], w[:m].astype(bool)

    def event_received(self):
        """(roundReceived (-1 nil), consensus timestamp) of every event."""
        m = self.event_count()
        rr = np.zeros(max(m, 1), np.int32)
        cts = np.zeros(max(m, 1), np.int64)
        self._check(self.L.hge_event_received(self.h, _p32(rr), _p64(cts), m))
        return rr[:m], cts[:m]

    def consensus_timestamp_sources(self, ids):
        """For each id, the event whose timestamp is its consensus timestamp
        (MedianTimestamp's source, hge_consensus_timestamp_sources; -1: not received)."""
        ids = np.ascontiguousarray(ids, np.int32)
        out = np.zeros(max(len(ids), 1), np.int32)
        if len(ids):
            self._check(self.L.hge_consensus_timestamp_sources(self.h, _p32(ids), len(ids), _p32(out)))
        return out[:len(ids)]

    def round_event_ids(self, r):
        """Every event of round r (insertion order) and its witness flag (hge_round_event_ids)."""
        n = ctypes.c_int64()
        self._check(self.L.hge_round_event_ids(self.h, r, None, None, 0, ctypes.byref(n)))
        ids = np.zeros(max(1, n.value), np.int32)
        wit = np.zeros(max(1, n.value), np.uint8)
        self._check(self.L.hge_round_event_ids(self.h, r, _p32(ids), _pu8(wit), n.value, ctypes.byref(n)))
        return ids[:n.value], wit[:n.value].astype(bool)

    def fame_table(self):
        """Fame of every (round, creator) slot: int8 [Rounds(), N], -1 = no witness
        (hge_fame's encoding: 0 undefined, 1 true, 2 false)."""
        R = self.rounds()
        out = np.full((max(R, 1), self.n), -1, np.int8)
        got = self.L.hge_fame_table(self.h, R, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int8)))
        if got < 0:
            raise HgeError(got, self.L.hge_last_error(self.h).decode())
        return out[:R]

    def consensus_log(self, start=0):
        m = self.L.hge_consensus_log(self.h, start, None, 0)
        out = np.zeros(max(m, 1), np.int32)
        self.L.hge_consensus_log(self.h, start, _p32(out), m)
        return out[:m]

    # --- Store semantics / sync path ---------------------------------------
    def set_cache_size(self, size):
        self._check(self.L.hge_set_cache_size(self.h, size))

    def participant_events(self, creator, skip):
        """Store.ParticipantEvents: ids from position `skip` (HgeError -11 = ErrTooLate)."""
        n = ctypes.c_int64()
        rc = self.L.hge_participant_events(self.h, creator, skip, None, 0, ctypes.byref(n))
        if rc != 0:
            raise HgeError(rc, self.L.hge_last_error(self.h).decode())
        out = np.zeros(max(n.value, 1), np.int32)
        self._check(self.L.hge_participant_events(self.h, creator, skip, _p32(out), n.value, ctypes.byref(n)))
        return out[:n.value]

    def participant_event(self, creator, index):
        r = self.L.hge_participant_event(self.h, creator, index)
        if r < 0:
            raise HgeError(r, ERRORS.get(r, "error"))
        return r

    def last_from(self, creator):
        r = self.L.hge_last_from(self.h, creator)
        if r < -1:
            raise HgeError(r, ERRORS.get(r, "error"))
        return None if r == -1 else r

    def diff(self, known):
        known = np.ascontiguousarray(known, np.int32)
        n = ctypes.c_int64()
        rc = self.L.hge_diff(self.h, _p32(known), None, 0, ctypes.byref(n))
        if rc != 0:
            raise HgeError(rc, self.L.hge_last_error(self.h).decode())
        out = np.zeros(max(n.value, 1), np.int32)
        self._check(self.L.hge_diff(self.h, _p32(known), _p32(out), n.value, ctypes.byref(n)))
        return out[:n.value]

    def wire_info(self, x):
        out = np.zeros(4, np.int32)
        self._check(self.L.hge_wire_info(self.h, x, _p32(out)))
        return tuple(int(v) for v in out)

    def read_wire_parents(self, creator_id, sp_index, op_creator_id, op_index):
        sp = ctypes.c_int32()
        op = ctypes.c_int32()
        rc = self.L.hge_read_wire_parents(self.h, creator_id, sp_index, op_creator_id, op_index,
                                          ctypes.byref(sp), ctypes.byref(op))
        if rc != 0:
            raise HgeError(rc, ERRORS.get(rc, "error"))
        return sp.value, op.value

    # --- round predicates ----------------------------------------------------
    def parent_round(self, x):
        return self.L.hge_parent_round(self.h, x)

    def round_inc(self, x):
        return bool(self.L.hge_round_inc(self.h, x))

    def round_diff(self, x, y):
        out = ctypes.c_int32()
        self._check(self.L.hge_round_diff(self.h, x, y, ctypes.byref(out)))
        return out.value

    def set_round(self, r, entries):
        """Store.SetRound: entries = [(id, witness: bool, fame 0/1/2)]."""
        ids = np.array([e[0] for e in entries], np.int32)
        w = np.array([int(e[1]) for e in entries], np.uint8)
        f = np.array([e[2] for e in entries], np.uint8)
        u8 = ctypes.POINTER(ctypes.c_uint8)
        self._check(self.L.hge_set_round(self.h, r, _p32(ids), w.ctypes.data_as(u8),
                                         f.ctypes.data_as(u8), len(ids)))

    def coordinates(self, x):
        la = np.zeros(self.n, np.int32)
        fd = np.zeros(self.n, np.int32)
        self._check(self.L.hge_coordinates(self.h, x, _p32(la), _p32(fd)))
        return la, fd


class Batch:
    """Many independent hashgraphs of N <= 64 participants replayed together on one
    GPU (hge_batch_*: one launch per stage for the whole batch).  add() admits a
    graph's stream (hge_replay's conventions), run() replays every graph, state(g)
    gives graph g's full state in tests/golden/digest.py's layout."""

    def __init__(self, n_participants, device=0):
        self.L = lib()
        h = ctypes.c_void_p()
        rc = self.L.hge_batch_create(n_participants, device, ctypes.byref(h))
        if rc != 0:
            raise HgeError(rc, "hge_batch_create failed")
        self.h = h
        self.n = n_participants
        self.status = []

    def close(self):
        if getattr(self, "h", None):
            self.L.hge_batch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != 0:
            raise HgeError(rc, self.L.hge_batch_last_error(self.h).decode())

    def add(self, dag_or_events, call_points):
        ev = dag_or_events if isinstance(dag_or_events, np.ndarray) else events_array(dag_or_events)
        ev = np.ascontiguousarray(ev, EVENT_DTYPE)
        cp = np.ascontiguousarray(call_points, np.int64)
        st = np.zeros(max(len(ev), 1), np.int32)
        g = ctypes.c_int32()
        self._check(self.L.hge_batch_add(self.h, ev.ctypes.data, len(ev), _p64(cp), len(cp), _p32(st),
                                         ctypes.byref(g)))
        self.status.append(st[:len(ev)])
        return g.value

    def stage(self):
        self._check(self.L.hge_batch_stage(self.h))

    def run(self):
        m = ctypes.c_int64()
        self._check(self.L.hge_batch_run(self.h, ctypes.byref(m)))
        return m.value

    def graphs(self):
        return self.L.hge_batch_graphs(self.h)

    def info(self, g):
        a = np.zeros(8, np.int64)
        self._check(self.L.hge_batch_info(self.h, g, _p64(a)))
        keys = ("events", "calls", "rounds", "lcr", "lcre", "transactions", "ordered", "undetermined")
        return dict(zip(keys, a.tolist()))

    KERNELS = ("kb_coords", "kb_fd", "kb_fdrows", "kb_front", "kb_fame", "kb_fold", "kb_receive", "kb_order")

    def fallbacks(self):
        """Graphs the last run replayed call by call (kb_consensus) instead of in bulk."""
        return int(self.L.hge_batch_fallbacks(self.h))

    def kernel_ms(self):
        """Device ms of the last run's stages (HIP events between the launches)."""
        a = (ctypes.c_float * 8)()
        n = self.L.hge_batch_kernel_ms(self.h, a, 8)
        if n < 0:
            self._check(n)
        return dict(zip(self.KERNELS, [float(a[k]) for k in range(n)]))

    def state(self, g):
        """Graph g's state: the fields of tests/golden/digest.py (status, order, counts,
        rounds, witness, fame, rr, cts, undetermined, scalars)."""
        inf = self.info(g)
        E, K, R = inf["events"], inf["calls"], inf["rounds"]
        order = np.zeros(max(inf["ordered"], 1), np.int32)
        counts = np.zeros(max(K, 1), np.int64)
        rounds = np.zeros(max(E, 1), np.int32)
        wit = np.zeros(max(E, 1), np.uint8)
        rr = np.zeros(max(E, 1), np.int32)
        cts = np.zeros(max(E, 1), np.int64)
        fame = np.zeros((max(R, 1), self.n), np.int8)
        und = np.zeros(max(inf["undetermined"], 1), np.int32)
        self._check(self.L.hge_batch_results(self.h, g, _p32(order), _p64(counts), _p32(rounds),
                                             wit.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), _p32(rr),
                                             _p64(cts), fame.ctypes.data_as(ctypes.POINTER(ctypes.c_int8)),
                                             _p32(und)))
        return dict(status=self.status[g], order=order[:inf["ordered"]], counts=counts[:K], rounds=rounds[:E],
                    witness=wit[:E].astype(bool), fame=fame[:R], rr=rr[:E], cts=cts[:E],
                    undetermined=und[:inf["undetermined"]],
                    scalars=np.array([R, inf["lcr"], inf["lcre"], inf["transactions"]], np.int64))
