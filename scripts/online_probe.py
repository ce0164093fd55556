"""Times the online per-call path (bench.online_path) at 16/100k, 64/1M and a
256-participant prefix; prints one JSON object per line."""
import json
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from babble_amd.gossip import random_gossip  # noqa: E402

which = sys.argv[1:] or ["16", "64", "256"]
if "16" in which:
    print(json.dumps({"online_16_100k": bench.online_path(16, 100_000, 16, 1, 0)}), flush=True)
if "64" in which:
    print(json.dumps({"online_64_1m": bench.online_path(64, 1_000_000, 64, 1, 0)}), flush=True)
if "256" in which:
    dag = random_gossip(256, bench.ONLINE_PREFIX, seed=1)
    print(json.dumps({"online_256_prefix": bench.online_path(256, bench.ONLINE_PREFIX, 256, 1, 0, dag=dag)}),
          flush=True)
