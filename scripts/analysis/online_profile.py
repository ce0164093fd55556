"""Where an online call's time goes (the per-call path of bench.online_path):
per-kernel device ms and launches per call (hge_set_profiling: HIP events around
every launch), host round trips per call, and the call latency with profiling
off.  Usage: python scripts/analysis/online_profile.py N E K [calls]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def run(n, E, K, ncalls, profile):
    from babble_amd.engine import Engine, events_array
    from babble_amd.gossip import random_gossip, schedule
    dag = random_gossip(n, E, seed=1)
    ev = events_array(dag)
    calls = schedule(E, K)[:ncalls]
    eng = Engine(n, E, device=0)
    if profile:
        eng.set_profiling(True)
    lat = []
    cpu = []
    prev = 0
    s0 = eng.host_syncs()
    warm = min(200, len(calls) // 4)
    for i, c in enumerate(calls):
        if profile and i == warm:
            eng.set_profiling(True)  # (resets the stats)
        t = time.perf_counter()
        tc = time.thread_time()
        eng.insert_events(ev[prev:c])
        eng.run_consensus()
        lat.append(time.perf_counter() - t)
        cpu.append(time.thread_time() - tc)
        prev = c
    syncs = (eng.host_syncs() - s0) / len(calls)
    stats = eng.kernel_stats() if profile else {}
    eng.close()
    lat = np.array(lat[warm:])
    cpu = np.array(cpu[warm:])
    per = len(calls) - warm
    ks = sorted(((k, v[0] * 1e3 / per, v[1] / per) for k, v in stats.items()), key=lambda x: -x[1])
    return {"p50_us": round(float(np.percentile(lat, 50)) * 1e6, 1),
            "mean_us": round(float(lat.mean()) * 1e6, 1),
            "host_cpu_us_mean": round(float(cpu.mean()) * 1e6, 1),
            "round_trips_per_call": round(syncs, 2),
            "device_us_per_call": round(sum(k[1] for k in ks), 1),
            "launches_per_call": round(sum(k[2] for k in ks), 1),
            "kernels": [(k, round(us, 2), round(l, 2)) for k, us, l in ks]}


if __name__ == "__main__":
    n, E, K = (int(a) for a in sys.argv[1:4])
    ncalls = int(sys.argv[4]) if len(sys.argv) > 4 else 2000
    out = {"config": [n, E, K, ncalls], "plain": run(n, E, K, ncalls, False)}
    out["profiled"] = run(n, E, K, ncalls, True)
    print(json.dumps(out, indent=1))
