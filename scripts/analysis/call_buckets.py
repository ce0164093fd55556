"""Histogram of per-call FindOrder batch sizes (the sort's call buckets) of one replay.
usage: python scripts/analysis/call_buckets.py N E K"""
import sys
import os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from babble_amd.engine import Engine, events_array
from babble_amd.gossip import random_gossip, schedule

n, E, K = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
dag = random_gossip(n, E, seed=1)
eng = Engine(n, E)
_, _, counts = eng.replay(events_array(dag), schedule(E, K))
c = np.asarray(counts)
edges = [0, 1, 2, 65, 257, 513, 1025, 2049, 4097, 8193, 16385, 1 << 30]
h = np.histogram(c, bins=edges)[0]
keys = [int(c[(c >= lo) & (c < hi)].sum()) for lo, hi in zip(edges[:-1], edges[1:])]
for lo, hi, m, k in zip(edges[:-1], edges[1:], h, keys):
    print(f"[{lo:6d}, {hi:10d}): {m:7d} calls, {k:9d} keys")
