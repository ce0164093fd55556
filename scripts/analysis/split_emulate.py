"""The sharded split emulated on ONE GPU: every part of a G-way split
of one replay runs alone, the other parts' exchange slots taken from a recorded
unsplit replay (hge_split_emulate), so each part's device work is timed without
the others competing for the GPU.  Per part: the sum of its kernels' device
times (HIP events on the engine stream; the emulation's host copies of the
other slots are not kernels) and whether its final state equals the replay's.
The collectives themselves (RCCL all-gathers over xGMI) are not in these numbers:
their payload per part is printed instead.

usage: python scripts/analysis/split_emulate.py [N] [E] [G ...]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def kernel_ms(eng):
    return sum(ms for ms, _ in eng.kernel_stats().values())


def main():
    from babble_amd.dist import ROUND_EVENTS_PER_PARTICIPANT, split_plan
    from babble_amd.engine import Engine, events_array
    from babble_amd.gossip import random_gossip, schedule
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    E = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000_000
    Gs = [int(g) for g in sys.argv[3:]] or [2, 4, 8]
    dag = random_gossip(n, E, seed=1)
    eng = Engine(n, E)
    eng.prepare(events_array(dag), schedule(E, n))
    for _ in range(2):
        eng.run()  # warm
    eng.set_profiling(True)
    eng.run()
    base = kernel_ms(eng)
    eng.set_profiling(False)
    top = sorted(eng.kernel_stats().items(), key=lambda kv: -kv[1][0])[:12]
    eng.split_emulate(True)
    eng.run()  # the record
    _, ref_order, ref_counts = eng.fetch()
    ref_rr, ref_cts = eng.event_received()
    out = {"n": n, "E": E, "unsplit_kernel_ms": round(base, 3),
           "unsplit_top": {k: round(v[0], 3) for k, v in top}, "splits": {}}
    print("unsplit", round(base, 3), flush=True)
    for G in Gs:
        plan = split_plan(eng.call_events(), eng.event_count(), G, 8 * ROUND_EVENTS_PER_PARTICIPANT * n)
        parts = []
        for p in range(G):
            eng.split_plan(p, G, plan)
            eng.clear_exchange()
            eng.split_run()  # warm
            eng.set_profiling(True)
            t0 = time.perf_counter()
            eng.split_run()
            wall = (time.perf_counter() - t0) * 1e3
            ks = eng.kernel_stats()
            eng.set_profiling(False)
            _, order, counts = eng.fetch()
            rr, cts = eng.event_received()
            same = bool(np.array_equal(order, ref_order) and np.array_equal(counts, ref_counts)
                        and np.array_equal(rr, ref_rr) and np.array_equal(cts, ref_cts))
            tops = sorted(ks.items(), key=lambda kv: -kv[1][0])[:10]
            parts.append({"part": p, "kernel_ms": round(sum(v[0] for v in ks.values()), 3),
                          "wall_ms_with_emulated_copies": round(wall, 3), "identical_to_replay": same,
                          "events": plan["ev_bounds"][p + 1] - plan["ev_bounds"][p],
                          "candidates": plan["ev_bounds"][p + 1] - plan["cand_lo"][p],
                          "top": {k: round(v[0], 3) for k, v in tops}})
            print(G, p, parts[-1]["kernel_ms"], same, flush=True)
        eng.split_plan(0, 0)
        mx = max(q["kernel_ms"] for q in parts)
        out["splits"][G] = {"parts": parts, "max_part_kernel_ms": round(mx, 3),
                            "speedup_vs_unsplit_kernels": round(base / mx, 3)}
        print(G, "max part", round(mx, 3), "speedup", round(base / mx, 3), flush=True)
    eng.close()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"split_emulate_n{n}_e{E}.json"), "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
