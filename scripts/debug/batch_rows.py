"""Compare the batch engine's LA / FD rows with the oracle's coordinates."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from babble_amd.engine import Batch, lib  # noqa: E402
from babble_amd.gossip import random_gossip, schedule  # noqa: E402
from oracle.oracle import replay  # noqa: E402

L = lib()
L.hgb_debug_rows.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)]
for n, E, k, seed in [(1, 50, 5, 3), (4, 1000, 4, 1), (2, 300, 2, 3)]:
    dag = random_gossip(n, E, seed=seed)
    calls = schedule(len(dag["creator"]), k)
    b = Batch(n)
    b.add(dag, calls)
    b.run()
    o, st, order, counts = replay(dag, calls)
    rows = {}
    for which in (0, 1):
        a = np.zeros((E, n), np.int32)
        assert L.hgb_debug_rows(b.h, 0, which, a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))) == 0
        rows[which] = a
    la = np.array([o.coords(x)[0] for x in range(E)])
    fd = np.array([o.coords(x)[2] for x in range(E)])
    fd = np.where(fd == np.iinfo(np.int64).max, 2**31 - 1, fd)
    bad_la = np.nonzero((rows[0] != la).any(1))[0]
    bad_fd = np.nonzero((rows[1] != fd).any(1))[0]
    print(n, E, "LA bad rows", len(bad_la), bad_la[:8].tolist(), "FD bad rows", len(bad_fd), bad_fd[:8].tolist())
    # the run layout
    cc = int(L.hgb_debug_ccap(b.h)) if hasattr(L, "hgb_debug_ccap") else None
    for x in bad_fd[:3]:
        print("  x", x, "creator", dag["creator"][x], "got", rows[1][x].tolist(), "want", fd[x].tolist())
    import math
    tot = np.zeros(1 << 22, np.int32)
    assert L.hgb_debug_rows(b.h, 0, 2, tot.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))) == 0
    lens = np.bincount(dag["creator"], minlength=n)
    ccap = int(lens.max())
    fdt = tot[:n * n * ccap].reshape(n, n, ccap)
    pos = np.zeros(E, np.int64)
    for c in range(n):
        pos[dag["creator"] == c] = np.arange(lens[c])
    bad = 0
    for x in range(E):
        c, p = dag["creator"][x], pos[x]
        if not np.array_equal(fdt[:, c, p], fd[x]):
            bad += 1
            if bad <= 3:
                print("  FDT x", x, "got", fdt[:, c, p].tolist(), "want", fd[x].tolist())
    print("  FDT bad", bad)
    b.close()
