"""Golden prefix for bench.py's in-run parity check (test infrastructure).

The bench replays the full seeded stream on the GPU; the engine reproduces the
reference's per-call semantics, so the batches of the first calls depend only
on the submissions before them.  This script runs the CPU oracle
(oracle/hg_oracle.cpp, the Go-faithful restatement, in its scale mode: same
results, pinned to the faithful mode by tests/test_oracle_scale.py and by
tests/golden/regen_check.py over every committed golden) on the first PREFIX
submissions of the same stream with the same schedule and stores every field
of the parity contract (make_golden.describe: status, order, per-call batch
sizes, rounds, witness flags, fame of every round slot, round received,
consensus timestamps, undetermined list, scalars):

    python tests/golden/make_bench_prefix.py [n] [events] [k] [seed] [prefix]

Committed: 256/10M with prefix 2,560,000 (10,000 calls) and 64/1M with the whole
stream (prefix 1,000,000).  Round 3's faithful-mode oracle took 1,850 s and
~26 GB for an 819,200 prefix; the scale mode takes ~35 s for that.  The whole
streams are pinned by digests as well (make_bench_full.py).
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

from babble_amd.gossip import random_gossip, schedule  # noqa: E402
from make_golden import describe  # noqa: E402
from oracle.oracle import replay  # noqa: E402


def main():
    a = [int(x) for x in sys.argv[1:]]
    n, E, K, seed, prefix = (a + [256, 10_000_000, 256, 1, 20480][len(a):])[:5]
    prefix = prefix // K * K
    dag = random_gossip(n, E, seed=seed)
    sub = {k: (v[:prefix] if isinstance(v, np.ndarray) else v) for k, v in dag.items()}
    calls = schedule(prefix, K)
    t = time.time()
    o, status, order, counts = replay(sub, calls, scale=True, release_lag=12)
    assert (status >= 0).all()
    d = describe(o, sub, status, order, counts, calls)
    d.pop("status")  # every submission of a gossip stream is accepted: status = iota
    d.pop("calls")
    d["order"] = d["order"].astype(np.int32)
    d["counts"] = d["counts"].astype(np.int64)
    out = os.path.join(HERE, f"bench_n{n}_e{E}_k{K}_s{seed}_prefix.npz")
    np.savez_compressed(out, n_calls=len(calls), prefix=prefix, n=n, events=E, k=K, seed=seed, **d)
    print(f"{out}: {len(order)} ordered over {len(calls)} calls ({time.time() - t:.1f} s)")


if __name__ == "__main__":
    main()
