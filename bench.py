"""Benchmark: consensus-ordered events/sec of the hashgraph ordering hot path.

Workload (BASELINE.json configs[1]): synthetic random-gossip DAG, 16
participants, 100k events, RunConsensus every K=16 inserted events (the
caller's schedule is part of the semantics: SURVEY.md TL;DR 5).  One step =
one full replay of the stream on the device: coordinates (InsertEvent),
DivideRounds, DecideFame and FindOrder at all 6,250 call points, from event
tables already resident in HBM to the complete consensus order.

Multi-GPU (torch.distributed, one process per GPU): every rank replays its own
independent hashgraph (seed base + rank) — the Monte Carlo / independent-replay
sharding of north_star; no data-path collective.  value = events ordered by
all ranks per step / max-over-ranks step time ("scaling": "weak").

Also reported: roofline of the dominant kernel (HIP events on the engine
stream), and the single-core CPU baseline (the Go-faithful oracle, timed on
the same host in the same run, rank 0 only).
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def algorithmic_bytes(kernel, n, events, ordered, calls):
    """Algorithmic HBM bytes one launch of `kernel` must move.

    k_coord_final: per event LA[sp]+D rows read, LA row written, FD row
    written once in total (16N bytes/event, SURVEY.md §8d 'coordinate kernel').
    k_rounds_frontier: per event its LA row read once for the strongly-see
    round test (4N bytes/event).  k_round_received: FD row of every ordered
    event (4N) + its key.  Others: the 48-byte sort key per ordered event.
    """
    if kernel.startswith("k_coord_final"):
        return 16 * n * events
    if kernel.startswith("k_coord_local"):
        return 8 * n * events
    if kernel.startswith("k_rounds_frontier"):
        return 4 * n * events
    if kernel.startswith("k_round_received"):
        return (4 * n + 48) * ordered
    return 48 * ordered


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--participants", type=int, default=16)
    ap.add_argument("--events", type=int, default=100_000)
    ap.add_argument("--k", type=int, default=16, help="RunConsensus every k inserted events")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-events", type=int, default=100_000)
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist_
        torch.cuda.set_device(local_rank)
        dist_.init_process_group("nccl")
        dist = dist_

    from babble_amd.engine import Engine, events_array
    from babble_amd.gossip import random_gossip, schedule

    n, E, K = args.participants, args.events, args.k
    dag = random_gossip(n, E, seed=args.seed + rank)
    calls = schedule(E, K)
    ev = events_array(dag)
    eng = Engine(n, E, device=local_rank)
    t0 = time.perf_counter()
    eng.prepare(ev, calls)  # FromParentsLatest admission on the host + staging into HBM
    ingest_s = time.perf_counter() - t0

    for _ in range(args.warmup):
        eng.run()

    def sync_all():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    sync_all()
    eng.set_profiling(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.run()  # returns after the device finished (stream synchronised)
    t1 = time.perf_counter()
    ordered = eng._nordered
    sync_all()
    step_s = (t1 - t0) / args.steps
    kstats = eng.kernel_stats()
    eng.set_profiling(False)

    tot_ordered = ordered
    max_step = step_s
    if dist is not None:
        import torch
        tt = torch.tensor([step_s], dtype=torch.float64, device=f"cuda:{local_rank}")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        max_step = float(tt.item())
        oo = torch.tensor([ordered], dtype=torch.float64, device=f"cuda:{local_rank}")
        dist.all_reduce(oo, op=dist.ReduceOp.SUM)
        tot_ordered = int(oo.item())

    # dominant kernel (largest total device time over the timed steps)
    dom, (dom_ms, dom_n) = max(kstats.items(), key=lambda kv: kv[1][0])
    per_launch_ms = dom_ms / max(dom_n, 1)
    launches_per_step = max(dom_n // args.steps, 1)
    alg = algorithmic_bytes(dom, n, E, ordered, len(calls)) / launches_per_step
    achieved = alg / (per_launch_ms * 1e-3) / 1e9
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_path):
        try:
            pm = json.load(open(pmc_path))
            if dom.split("<")[0] in pm:
                traffic = pm[dom.split("<")[0]]
        except Exception:
            traffic = None

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        from oracle.oracle import replay as oracle_replay
        ns = min(args.cpu_sample_events, E)
        sub = {k: (v[:ns] if isinstance(v, np.ndarray) else v) for k, v in dag.items()}
        t0 = time.perf_counter()
        _, _, corder, _ = oracle_replay(sub, schedule(ns, K))
        cs = time.perf_counter() - t0
        cpu = {"value": len(corder) / cs, "unit": "events/s", "cores": 1, "kind": "port",
               "sample": f"Go-faithful C++ oracle, first {ns} events of the same stream, K={K}, "
                         f"{cs:.2f} s on {platform.processor() or platform.machine()} "
                         f"(nproc {os.cpu_count()})"}

    if rank == 0:
        value = tot_ordered / max_step
        line = {
            "metric": "consensus-ordered events/sec at N participants",
            "value": round(value, 1),
            "unit": "events/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(max_step * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic",
            "config": {"workload": f"random-gossip DAG, {n} participants, {E} events per GPU, "
                                   f"RunConsensus every K={K} events ({len(calls)} calls)",
                       "participants": n, "events_per_gpu": E, "k": K, "calls": len(calls),
                       "ordered_per_step": tot_ordered, "parallelism": f"replicas{world}"},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "launch_ms": round(per_launch_ms, 4)},
            "cpu_baseline": cpu,
            "ingest_host_ms": round(ingest_s * 1e3, 2),
            "kernels_ms_per_step": {k: round(v[0] / args.steps, 4) for k, v in
                                    sorted(kstats.items(), key=lambda kv: -kv[1][0])},
        }
        print(json.dumps(line))
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
