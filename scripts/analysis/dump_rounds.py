"""Dump every event's round / witness flag and chain coordinates of one replay
(for offline analysis of the frontier recurrence, e.g. how predictable each
chain's per-round advance is).  usage: python scripts/analysis/dump_rounds.py N E K out.npz"""
import sys
import os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from babble_amd.engine import Engine, events_array
from babble_amd.gossip import random_gossip, schedule

n, E, K, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
dag = random_gossip(n, E, seed=1)
eng = Engine(n, E)
eng.replay(events_array(dag), schedule(E, K))
r, w = eng.event_rounds()
np.savez_compressed(out, round=r, wit=w, creator=dag["creator"], index=dag["index"])
print("rounds", int(r.max()) + 1, "witnesses", int(w.sum()))
