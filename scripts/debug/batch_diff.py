"""Print where the batch engine first differs from the oracle for a few small cases."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
from babble_amd.engine import Batch  # noqa: E402
from babble_amd.gossip import random_gossip, schedule  # noqa: E402
from digest import canonical, FIELDS  # noqa: E402
from make_mc_digests import oracle_state  # noqa: E402

cases = [(1, 50, 5, 3), (2, 300, 2, 3), (4, 1000, 4, 1)]
for n, E, k, seed in cases:
    dag = random_gossip(n, E, seed=seed)
    calls = schedule(len(dag["creator"]), k)
    b = Batch(n)
    b.add(dag, calls)
    b.run()
    got, want = canonical(b.state(0)), canonical(oracle_state(dag, calls))
    for f, _ in FIELDS:
        a, w = got[f], want[f]
        if a.shape != w.shape or not np.array_equal(a, w):
            if a.shape == w.shape:
                idx = np.nonzero((a != w).reshape(len(a), -1).any(1))[0][:10]
                print(n, E, k, f, "first diffs at", idx.tolist(), "got", a[idx].tolist(), "want", w[idx].tolist())
            else:
                print(n, E, k, f, "shape", a.shape, w.shape, a[:20].tolist(), w[:20].tolist())
    print(n, E, k, "done", b.kernel_ms())
    b.close()
