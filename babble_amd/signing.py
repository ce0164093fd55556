"""Synthetic signed streams: what a babble node does before InsertEvent.

Every participant holds an ECDSA P-256 key (crypto.GenerateECDSAKey,
/root/reference/crypto/utils.go:36-38) and signs SHA-256 of each event body
(Event.Sign, /root/reference/hashgraph/event.go:131-138).  Keys derive from a
seed (build/libhge_tools.so, hge_tools.cpp); signatures use random nonces like
Go's ecdsa.Sign.  Bodies are fixed-layout byte strings carrying the body's
fields (creator key, parents' hashes, timestamp, index, one transaction) at the
size of a gob-encoded EventBody; the engine never parses them, it only hashes
and verifies them (the ingest pipeline, hge_ingest).
"""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOLS_PATH = os.path.join(ROOT, "build", "libhge_tools.so")
BODY_BYTES = 65 + 2 * 32 + 8 + 8 + 16  # creator key, parent hashes, timestamp, index, transaction
_tools = None


def tools():
    global _tools
    if _tools is None:
        if not os.path.exists(TOOLS_PATH):
            raise ImportError(f"tools library not built: {TOOLS_PATH} (run __graft_entry__.build())")
        L = ctypes.CDLL(TOOLS_PATH)
        P = ctypes.POINTER
        L.hgt_keys.argtypes = [ctypes.c_int32, ctypes.c_uint64, P(ctypes.c_uint8)]
        L.hgt_sign.argtypes = [ctypes.c_int64, P(ctypes.c_uint8), P(ctypes.c_int64), P(ctypes.c_int32),
                               ctypes.c_int32, ctypes.c_uint64, ctypes.c_int32, P(ctypes.c_uint8)]
        _tools = L
    return _tools


def keys(n, seed=1):
    """uint8[n, 65]: the participants' uncompressed public keys."""
    out = np.zeros((n, 65), np.uint8)
    tools().hgt_keys(n, seed, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
    return out


def bodies(dag, pubs):
    """(flat uint8, offsets int64[E+1]) of the stream's event bodies."""
    E = len(dag["creator"])
    b = np.zeros((E, BODY_BYTES), np.uint8)
    b[:, :65] = pubs[dag["creator"]]
    h = dag["hash"]
    sp, op = dag["sp"], dag["op"]
    b[:, 65:97] = np.where((sp >= 0)[:, None], h[np.maximum(sp, 0)], 0)
    b[:, 97:129] = np.where((op >= 0)[:, None], h[np.maximum(op, 0)], 0)
    b[:, 129:137] = dag["ts"].astype(">i8").view(np.uint8).reshape(E, 8)
    b[:, 137:145] = dag["index"].astype(">i8").view(np.uint8).reshape(E, 8)
    b[:, 145:161] = h[:, :16]  # the transaction payload
    return b.reshape(-1), np.arange(E + 1, dtype=np.int64) * BODY_BYTES


def sign(flat, off, creator, n, seed=1, threads=8):
    """uint8[E, 64] signatures r || s of every body by its creator's key."""
    E = len(off) - 1
    out = np.zeros((max(E, 1), 64), np.uint8)
    P8 = ctypes.POINTER(ctypes.c_uint8)
    flat = np.ascontiguousarray(flat, np.uint8)
    off = np.ascontiguousarray(off, np.int64)
    cr = np.ascontiguousarray(creator, np.int32)
    rc = tools().hgt_sign(E, flat.ctypes.data_as(P8), off.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                          cr.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), n, seed, threads,
                          out.ctypes.data_as(P8))
    if rc != 0:
        raise ValueError("hgt_sign: creator out of range")
    return out[:E]


def signed_stream(dag, seed=1, threads=8):
    """(pubs, (flat, off), sigs) for a gossip stream."""
    pubs = keys(dag["n"], seed)
    flat, off = bodies(dag, pubs)
    sigs = sign(flat, off, dag["creator"], dag["n"], seed, threads)
    return pubs, (flat, off), sigs
