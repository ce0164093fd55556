"""Whole-stream digests of the bench streams (test infrastructure).

The oracle (oracle/hg_oracle.cpp, scale mode: the faithful restatement's
results computed without re-deriving what cannot change within a call; pinned
to the faithful mode by tests/test_oracle_scale.py and by regenerating every
committed golden byte-identically) replays the WHOLE seeded stream that
bench.py replays, with the same RunConsensus schedule, and this script stores:
  * the SHA-256 of every field of the parity contract over the whole stream
    (tests/golden/digest.py's canonical layout: status, order, per-call batch
    sizes, rounds, witness flags, fame of every (round, creator) slot, round
    received, consensus timestamps of ordered events, undetermined list,
    scalars) and the digest of the whole state;
  * digests of consecutive chunks of every per-event and per-call field, so a
    mismatch names the first chunk that differs;
  * the scalars, DecideFame's statistics and the ordered count in clear.

    python tests/golden/make_bench_full.py [n] [events] [k] [seed] [release_lag]

256/10M: about 10 minutes and 4 GB of host memory (release lag 12 rounds).
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

from babble_amd.gossip import random_gossip, schedule  # noqa: E402
from digest import CALL_CHUNK, EVENT_CHUNK, FIELDS, ORDER_CHUNK, field_digests  # noqa: E402
from make_golden import describe  # noqa: E402
from oracle.oracle import replay  # noqa: E402


def path_for(n, E, K, seed):
    return os.path.join(HERE, f"bench_n{n}_e{E}_k{K}_s{seed}_full.json")


def main():
    a = [int(x) for x in sys.argv[1:]]
    n, E, K, seed, lag = (a + [256, 10_000_000, 256, 1, 12][len(a):])[:5]
    dag = random_gossip(n, E, seed=seed)
    calls = schedule(E, K)
    t = time.time()
    o, status, order, counts = replay(dag, calls, scale=True, release_lag=lag)
    dt = time.time() - t
    d = describe(o, dag, status, order, counts, calls)
    state = {k: d[k] for k, _ in FIELDS}
    out = {"params": {"n": n, "events": E, "k": K, "seed": seed, "generator": "random_gossip"},
           "n_calls": int(len(calls)), "ordered": int(len(order)), "rejected": int((status < 0).sum()),
           "scalars": [int(v) for v in d["scalars"]], "fame_stats": [int(v) for v in d["fame_stats"]],
           "chunk_sizes": {"events": EVENT_CHUNK, "order": ORDER_CHUNK, "calls": CALL_CHUNK},
           "oracle": {"mode": "scale", "release_lag": lag, "seconds": round(dt, 1)},
           **field_digests(state)}
    with open(path_for(n, E, K, seed), "w") as f:
        json.dump(out, f, indent=1)
    print(f"{path_for(n, E, K, seed)}: {len(order)} ordered over {len(calls)} calls, "
          f"scalars {out['scalars']} ({dt:.1f} s)")


if __name__ == "__main__":
    main()
