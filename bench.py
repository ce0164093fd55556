"""Benchmark: consensus-ordered events/sec of the hashgraph ordering hot path.

Workloads (BASELINE.json configs):
  gossip (default, configs[1]): synthetic random-gossip DAG, 16 participants,
      100k events, RunConsensus every K=16 inserted events (the caller's
      schedule is part of the semantics: SURVEY.md TL;DR 5).  One step = one
      full replay of the stream on the device: coordinates (InsertEvent),
      DivideRounds, DecideFame and FindOrder at all 6,250 call points, from
      event tables already resident in HBM to the complete consensus order.
      --participants/--events/--k select configs[2] (64/1M) and configs[3]
      (256/10M).
  mc (configs[4]): Monte Carlo batch of independent 32-participant
      hashgraphs with simulated Byzantine forkers (10 of 32 creators fork with
      p=0.05), 10k submissions each, K=32; the batch is split across ranks.
      Every graph has its own engine (HIP stream); host threads drive them
      concurrently.

Multi-GPU (torch.distributed over RCCL, one process per GPU): gossip = every
rank replays its own independent hashgraph (seed + rank), mc = every rank
replays its share of the batch; no data-path collective.  value = events
ordered by all ranks per step / max-over-ranks step time ("scaling": "weak").

The timed steps run without per-kernel instrumentation; a separate profiled
pass (HIP events around every launch on the engine stream) gives the
dominant kernel's average launch time for the roofline.  The CPU baseline is
the Go-faithful oracle on one host core over a bounded sample of the same
workload (rank 0 only), and its order is compared with the device's.
"""
import argparse
import json
import os
import platform
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)


def algorithmic_bytes(kernel, n, events, ordered, sweeps=1):
    """Algorithmic HBM bytes of ONE launch of `kernel` over a whole replay
    (B(N) = 24N + 48 per ordered event).

    coordinates: k_coord_final 16N/event (read LA[sp] and D, write LA and FD),
    k_coord_local 8N/event, k_la_sweep 8N/event per sweep (op row + own row
    read) plus the own row written once over all `sweeps` (a sweep stores only
    the values that changed, so a converged row is not re-written), k_transpose and k_fdt_runs 8N/event; rounds: k_fss 8N/event (FD row read,
    fss row written), k_rounds_walk / k_rounds_coop 4N/event (the strongly-see
    round test reads each event's LA row once); order: k_round_received /
    k_median_wave (4N + 48)/ordered event; anything else the 48-byte sort key.
    """
    name = kernel.strip("()").split("<")[0]
    if name == "k_la_sweep":
        return 8 * n * events + 4 * n * events / max(sweeps, 1)
    per_event = {"k_coord_final": 16 * n, "k_coord_local": 8 * n,
                 "k_transpose": 8 * n, "k_fdt_runs": 8 * n, "k_fss": 8 * n, "k_rounds_walk": 4 * n,
                 "k_rounds_coop": 4 * n, "k_rounds_fss": 4 * n, "k_rounds_frontier": 4 * n}
    if name in per_event:
        return per_event[name] * events
    if name in ("k_round_received", "k_median_wave"):
        return (4 * n + 48) * ordered
    return 48 * ordered


def pmc_traffic(config_key, kernel):
    """HBM bytes per launch of `kernel` in this configuration from the committed
    rocprofv3 PMC passes (profiles/pmc_traffic.json, made by
    scripts/pmc_traffic.py on the GPU box), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        pm = json.load(open(path))
    except (OSError, ValueError):
        return None
    name = kernel.strip("()").split("<")[0]
    v = pm.get("configs", {}).get(config_key, {}).get(name)
    return v.get("bytes_per_launch") if isinstance(v, dict) else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--ramp-s", type=float, default=0.3,
                    help="untimed clock ramp before the warmup steps (seconds)")
    ap.add_argument("--workload", choices=("gossip", "mc"), default="gossip")
    ap.add_argument("--participants", type=int, default=None)
    ap.add_argument("--events", type=int, default=None)
    ap.add_argument("--k", type=int, default=None, help="RunConsensus every k submissions")
    ap.add_argument("--graphs", type=int, default=1024, help="mc: hashgraphs in the whole batch")
    ap.add_argument("--threads", type=int, default=8, help="mc: host threads driving engines")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-events", type=int, default=100_000)
    ap.add_argument("--profile-steps", type=int, default=2)
    args = ap.parse_args()
    mc = args.workload == "mc"
    n = args.participants or (32 if mc else 16)
    E = args.events or (10_000 if mc else 100_000)
    K = args.k or n

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

    from babble_amd.dist import reduce_step, shard_range
    from babble_amd.engine import Engine, events_array
    from babble_amd.gossip import random_gossip, schedule

    # ---- stage the workload in HBM (host admission + upload; not timed) ----
    t0 = time.perf_counter()
    if mc:
        first, per = shard_range(args.graphs, world, rank)
        dags = [random_gossip(n, E, seed=args.seed + first + g, forkers=10, fork_p=0.05)
                for g in range(per)]
        engines = [Engine(n, len(d["creator"]) + 64, device=local_rank) for d in dags]
        for eng, d in zip(engines, dags):
            eng.prepare(events_array(d), schedule(len(d["creator"]), K))
    else:
        dags = [random_gossip(n, E, seed=args.seed + rank)]
        engines = [Engine(n, E, device=local_rank)]
        engines[0].prepare(events_array(dags[0]), schedule(E, K))
    ingest_s = time.perf_counter() - t0
    pool = ThreadPoolExecutor(max_workers=max(1, min(args.threads, len(engines))))

    def step():
        if len(engines) == 1:
            return engines[0].run()
        return sum(pool.map(lambda e: e.run(), engines))

    def sync_all():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    # the GPU and the host thread leave their idle clocks only under sustained load:
    # run the path for ~0.3 s before the W warmup steps (none of it is timed)
    t_ramp = time.perf_counter()
    while time.perf_counter() - t_ramp < args.ramp_s:
        step()
    for _ in range(args.warmup):
        step()
    sync_all()
    t0 = time.perf_counter()
    ordered = 0
    for _ in range(args.steps):
        ordered = step()  # every engine returns after its stream drained
    t1 = time.perf_counter()
    sync_all()
    step_s = (t1 - t0) / args.steps

    # ---- one more unprofiled replay: GPU-busy vs wall split of a step ----
    eng0 = engines[0]
    eng0.run()
    st_ms = eng0.stage_times()
    replay_ms = {"coords_gpu": st_ms[0], "coords_wall": st_ms[1], "consensus_gpu": st_ms[3],
                 "consensus_wall": st_ms[2], "gpu": st_ms[6], "wall": st_ms[4]}
    replay_ms = {k: round(v, 4) for k, v in replay_ms.items()}

    # ---- profiled pass: per-kernel device time (HIP events on the engine stream) ----
    eng0.set_profiling(True)
    for _ in range(max(1, args.profile_steps)):
        eng0.run()
    kstats = eng0.kernel_stats()
    eng0.set_profiling(False)
    ev0 = len(dags[0]["creator"])
    ord0 = eng0._nordered

    tot_ordered, max_step = ordered, step_s
    if dist is not None:
        max_step, tot_ordered = reduce_step(dist, step_s, ordered, f"cuda:{local_rank}")

    nprof = max(1, args.profile_steps)

    sweeps = eng0.coordinate_sweeps()

    def kernel_gbs(name):
        """(algorithmic bytes per launch, avg launch ms, achieved GB/s) of one kernel.
        k_la_sweep: every sweep that does work reads the own and op rows once (8N
        bytes per event) and the row writes are spread over the sweeps; the
        queued launches after the converged one return at once and are left out
        of the launch count."""
        ms, cnt = kstats[name]
        if name.startswith("k_la_sweep"):
            cnt = sweeps * nprof
            b = algorithmic_bytes(name, n, ev0, ord0, sweeps)
        else:
            b = algorithmic_bytes(name, n, ev0, ord0) / max(cnt // nprof, 1)
        per_launch = ms / max(cnt, 1)
        return b, per_launch, b / (per_launch * 1e-3) / 1e9

    dom = max(kstats.items(), key=lambda kv: kv[1][0])[0]
    alg, per_launch_ms, achieved = kernel_gbs(dom)
    # the bandwidth-bound kernels (streaming passes over the N-wide tables)
    hbm_kernels = {}
    for name in kstats:
        base = name.strip("()").split("<")[0]
        if base in ("k_la_sweep", "k_transpose", "k_fss", "k_fdt_runs"):
            b, pl, gbs = kernel_gbs(name)
            hbm_kernels[name] = {"achieved_gbs": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
                                 "launch_ms": round(pl, 4),
                                 "launches_per_replay": (sweeps if base == "k_la_sweep"
                                                         else kstats[name][1] // nprof)}

    cpu, parity = None, None
    if rank == 0 and not args.no_cpu_baseline:
        from oracle.oracle import replay as oracle_replay
        d = dags[0]
        ns = min(args.cpu_sample_events, len(d["creator"]))
        sub = {k: (v[:ns] if isinstance(v, np.ndarray) else v) for k, v in d.items()}
        t0 = time.perf_counter()
        _, _, corder, _ = oracle_replay(sub, schedule(ns, K))
        cs = time.perf_counter() - t0
        what = (f"graph 0 of the batch ({ns} submissions)" if mc else
                f"first {ns} of {len(d['creator'])} submissions of the same stream")
        cpu = {"value": round(len(corder) / cs, 1), "unit": "events/s", "cores": 1, "kind": "port",
               "sample": f"Go-faithful C++ oracle (oracle/hg_oracle.cpp), {what}, K={K}, "
                         f"{cs:.2f} s on {platform.processor() or platform.machine()} "
                         f"(host nproc {os.cpu_count()})"}
        if ns == len(d["creator"]):
            _, gorder, _ = eng0.fetch()
            parity = ("bit-exact vs CPU oracle (full stream of graph 0)"
                      if np.array_equal(gorder, corder) else "MISMATCH vs CPU oracle")

    if rank == 0:
        value = tot_ordered / max_step
        if mc:
            workload = (f"Monte Carlo batch: {args.graphs} independent random-gossip hashgraphs, "
                        f"{n} participants, {E} submissions each, 10 forkers p=0.05, "
                        f"RunConsensus every K={K}")
        else:
            workload = (f"random-gossip DAG, {n} participants, {E} events per GPU, "
                        f"RunConsensus every K={K} events ({len(schedule(E, K))} calls)")
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
            "config": {"workload": workload, "participants": n, "events_per_graph": E, "k": K,
                       "graphs_per_gpu": len(engines), "ordered_per_step": tot_ordered,
                       "parallelism": f"replicas{world}"},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": pmc_traffic(f"{args.workload}_n{n}_e{E}_k{K}", dom),
                         "algorithmic_bytes_per_launch": int(alg),
                         "launch_ms": round(per_launch_ms, 4),
                         "hbm_kernels": hbm_kernels,
                         # the whole path against HBM, B(N) = 24N + 48 bytes/event
                         "path": {"bytes_per_event": 24 * n + 48,
                                  "achieved_gbs": round(value / world * (24 * n + 48) / 1e9, 2),
                                  "frac": round(value / world * (24 * n + 48) / 1e9 / HBM_PEAK_GBS, 5)}},
            "cpu_baseline": cpu,
            "parity": parity,
            "ingest_host_ms": round(ingest_s * 1e3, 2),
            "replay_ms": replay_ms,
            "kernels_ms_per_replay": {k: round(v[0] / nprof, 4) for k, v in
                                      sorted(kstats.items(), key=lambda kv: -kv[1][0])},
            "kernel_launches_per_replay": {k: v[1] // nprof for k, v in kstats.items()},
        }
        print(json.dumps(line), flush=True)
    pool.shutdown()
    for e in engines:
        e.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
