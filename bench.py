"""Benchmark: consensus-ordered events/sec of the hashgraph ordering hot path.

Workloads (BASELINE.json configs):
  gossip (default): synthetic random-gossip DAG, 256 participants, 10M events,
      RunConsensus every K=256 inserted events (configs[3] on one MI355X, the
      largest single-GPU configuration; the caller's schedule is part of the
      semantics: SURVEY.md TL;DR 5).  One step = one full replay of the stream
      on the device: coordinates (InsertEvent), DivideRounds, DecideFame and
      FindOrder at all 39,063 call points, from event tables already resident in
      HBM to the complete consensus order.  --participants/--events/--k select
      the other gossip configs (16/100k = configs[1], 64/1M = configs[2]).
  mc (configs[4]): Monte Carlo batch of independent 32-participant
      hashgraphs with simulated Byzantine forkers (10 of 32 creators fork with
      p=0.05; half of the fork twins get events built on them, which are
      rejected in cascade), 10k submissions each, K=32; the batch is split
      across ranks.  One step = one replay of every graph of the rank's share
      on the batch engine (hge_batch_*: four launches for the whole batch, the
      graphs' call schedules inside the consensus kernel).

Multi-GPU (torch.distributed over RCCL, one process per GPU):
  gossip (default): ONE hashgraph sharded by time across the ranks
      (babble_amd.dist.split_run, DESIGN.md §6: every rank computes the
      coordinates and the sequential rounds walk, then decides the fame of its
      rounds and orders its calls' events; fame decisions and ordered slices are
      all-gathered over RCCL), "scaling": "strong": value = the one hashgraph's
      ordered events / max-over-ranks step time.  --replicas: every rank replays its own independent hashgraph
      (seed + rank), no data-path collective, "scaling": "weak".
  mc: every rank replays its share of the batch; no data-path collective
      ("scaling": "weak").

The timed steps run without per-kernel instrumentation; a separate profiled
pass (HIP events around every launch on the engine stream) gives every
kernel's device time for the roofline.  Rank 0 also
  * checks its order against a committed golden prefix (tests/golden/bench_*,
    the oracle's output for the first calls of the same seeded stream): the
    engine reproduces per-call semantics, so the first calls' batches of the
    full replay must equal the prefix replay's;
  * times the CPU baseline: the Go-faithful oracle on one host core over a
    bounded prefix of the same stream, and compares its order too;
  * with the default configuration, adds a `secondary` object: the 16/100k
    replay (bit-exact against the oracle over the whole stream), the online
    per-call path (hge_insert_events of K events + hge_run_consensus per call,
    what node/core.go:179-202 does) at 16/100k, 64/1M and on the bench's own
    256-wide stream, the ingest pipeline, and config 5 (`mc_1024x32x10k`: the
    1,024-graph Monte Carlo batch on the batch engine, every graph against the
    oracle's digest, with its own CPU baseline).
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

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
DEFAULT = (256, 10_000_000)
ONLINE_PREFIX = 512_000  # online per-call line at the default width


def algorithmic_bytes(kernel, n, events, ordered, rounds=0):
    """Algorithmic HBM bytes of `kernel` over ONE whole replay (all its launches),
    int32 coordinates (B(N) = 24N + 48 per ordered event).

    Each byte is counted once per replay, however many launches touch it:
      k_la_sweep    12N/event: read LA[sp] and LA[op], write LA[x] -- once, not
                    once per fixed-point sweep (the sweeps' re-reads are waste);
      k_la_clear     4N/event (the new rows' -1 fill);
      k_la_sweep16 / k_la_clear16  6N / 2N per event (N > 32: the same on packed u16);
      k_transpose    8N/event at N <= 16 (FDT -> FD: reads and writes 4N);
      k_fd_transpose_ts 12N/event (N > 16: FDT read, FD and the 4-byte FD
                    timestamp offsets written); 8N with uint16 runs and FD rows
                    (N > 128: 2N FDT read, 2N FD and 4N offsets written).  These
                    figures include the FDT intermediate and the offsets; SURVEY
                    8(d)'s FD write alone (4N, 2N as uint16) is reported beside
                    them as `fd_write_frac`;
      k_witness_la   8N^2 per round (frontier rows read, transposed rows written);
      k_la16_rows_runs 6N/event (N > 32: LA16 read, the FDT runs written); 8N/event
                    over int32 LA tiles (<int32_t, true>: N <= 32 and wide hashgraphs);
                    4N with uint16 runs (<uint16_t>, N > 128);
      k_la_win      (2N + 20)/event (32 < N <= 256, windowed exact propagation: the
                    head rows live in LDS, so per event only the packed row is
                    written, the 16-byte plan entry read and the 4-byte row sum
                    written -- once per replay, however many passes);
      k_lw_plan     40/event (creator, index, other-parent and two chain gathers
                    read, the plan entry written);
      k_fdt_clear    4N/event;
      k_fss          8N/event (FD row read, fss row written, N <= 32);
      rounds        4N/event (the strongly-see round test reads each row once);
      k_round_received / k_median_wave (4N + 48) per ordered event (FD row for
                    the median, sort key); everything else the 48-byte key.
                    (k_median_wave reads 4N + 8N: the thresholds row and the FD
                    timestamps row; 4N + 48 stays the SURVEY 8(d) figure.)
    """
    name = kernel.strip("()").split("<")[0]
    if name == "k_witness_la":
        return 8 * n * n * rounds
    if name == "k_la16_rows_runs" and "true" in kernel:
        return 8 * n * events
    if name == "k_la16_rows_runs" and "uint16_t" in kernel:
        return 4 * n * events
    if name == "k_fd_transpose_ts" and "uint16_t" in kernel:
        return 8 * n * events
    per_event = {"k_la_sweep": 12 * n, "k_la_clear": 4 * n, "k_transpose": 8 * n,
                 "k_fd_transpose_ts": 12 * n,
                 "k_fdt_clear": 4 * n, "k_fss": 8 * n,
                 "k_rounds_walk": 4 * n, "k_rounds_coop": 4 * n, "k_rounds_coop_spec": 4 * n,
                 "k_walk_spec": 4 * n, "k_rounds_fss": 4 * n, "k_rounds_direct": 4 * n,
                 "k_la_clear16": 2 * n, "k_la_sweep16": 6 * n, "k_la16_rows_runs": 6 * n,
                 "k_la_win": 2 * n + 20, "k_lw_plan": 40, "k_lw_pos": 0}
    if name in per_event:
        return per_event[name] * events
    if name in ("k_round_received", "k_median_wave"):
        return (4 * n + 48) * ordered
    return 48 * ordered


def pmc_traffic(config_key, kernel, launches_per_replay):
    """HBM bytes per launch of `kernel` in this configuration from the committed
    rocprofv3 PMC passes (profiles/r06/pmc_traffic.json, else an earlier round's, made by
    scripts/pmc_traffic.py on the GPU box): the kernel's bytes per replay over
    the launches that did work (k_la_sweep: the sweeps up to the quiet one), or None."""
    name = kernel.strip("()").split("<")[0]
    for rnd in ("r06", "r05", "r04", "r03", "r02"):  # the latest round's passes of this kernel
        try:
            pm = json.load(open(os.path.join(ROOT, "profiles", rnd, "pmc_traffic.json")))
        except (OSError, ValueError):
            continue
        v = pm.get("configs", {}).get(config_key, {}).get(name)
        if isinstance(v, dict) and "bytes_per_replay" in v:
            return int(v["bytes_per_replay"] / max(launches_per_replay, 1))
    return None


def golden_prefix(n, E, K, seed):
    """The committed oracle prefix of this exact stream, or None
    (tests/golden/make_bench_prefix.py)."""
    path = os.path.join(ROOT, "tests", "golden", f"bench_n{n}_e{E}_k{K}_s{seed}_prefix.npz")
    if not os.path.exists(path):
        return None
    return np.load(path)


def golden_full(n, E, K, seed):
    """The committed whole-stream oracle digests of this exact stream, or None
    (tests/golden/make_bench_full.py)."""
    path = os.path.join(ROOT, "tests", "golden", f"bench_n{n}_e{E}_k{K}_s{seed}_full.json")
    if not os.path.exists(path):
        return None
    return json.load(open(path))


def mc_digests(n, E, K, seed):
    """The committed oracle digests of config 5's batch (tests/golden/make_mc_digests.py)
    when this run replays exactly that batch, else None."""
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    path = os.path.join(ROOT, "tests", "golden", f"mc_n{n}_e{E}_k{K}_digests.json")
    if not os.path.exists(path):
        return None
    d = json.load(open(path))
    p = d["params"]
    if (p["seed0"], p["forkers"], p["fork_p"], p["cascade_p"]) != (seed, 10, 0.05, 0.5):
        return None
    return d["digests"]


def sub_stream(dag, ns):
    return {k: (v[:ns] if isinstance(v, np.ndarray) else v) for k, v in dag.items()}


def online_path(n, E, K, seed, device, dag=None, what=None):
    """The per-call production path: for every call, hge_insert_events of the
    next K submissions, then hge_run_consensus (node/core.go:179-202).  Returns
    per-call latency (p50/p99), the host admission share, host round trips per
    call, events/s, and whether the order equals the replay's.  `dag`: a stream
    to take (else a fresh random_gossip(n, E, seed))."""
    from babble_amd.engine import Engine, events_array
    from babble_amd.gossip import random_gossip, schedule
    if dag is None:
        dag = random_gossip(n, E, seed=seed)
    ev = events_array(dag)[:E]
    calls = schedule(E, K)
    rep = Engine(n, E, device=device)
    _, rorder, _ = rep.replay(ev, calls)
    rep.close()
    eng = Engine(n, E, device=device)
    lat = np.zeros(len(calls))
    adm = np.zeros(len(calls))
    parts = []
    prev = 0
    s0 = eng.host_syncs()
    t0 = time.perf_counter()
    for i, c in enumerate(calls):
        t = time.perf_counter()
        # every submission of a gossip stream is accepted: engine id == submission index
        eng.insert_events(ev[prev:c])
        ta = time.perf_counter()
        parts.append(eng.run_consensus())
        lat[i] = time.perf_counter() - t
        adm[i] = ta - t
        prev = c
    wall = time.perf_counter() - t0
    syncs = eng.host_syncs() - s0
    order = np.concatenate(parts) if parts else np.zeros(0, np.int32)
    eng.close()
    us = lambda a, q: round(float(np.percentile(a, q)) * 1e6, 1)
    return {"workload": what or (f"online per-call path, {n} participants, {E} events, "
                                 f"hge_insert_events(K={K}) + hge_run_consensus per call ({len(calls)} calls)"),
            "value": round(len(order) / wall, 1), "unit": "events/s",
            "call_latency_us": {"mean": round(float(lat.mean()) * 1e6, 1), "p50": us(lat, 50), "p99": us(lat, 99)},
            "admission_us": {"p50": us(adm, 50), "p99": us(adm, 99)},
            "host_round_trips_per_call": round(syncs / max(1, len(calls)), 2),
            "parity": ("identical to the bulk replay" if np.array_equal(order, rorder)
                       else "MISMATCH vs the bulk replay")}


def ingest_path(n, E, K, seed, device, threads=16):
    """The online path with InsertEvent's front half: hge_ingest
    verifies each batch's ECDSA P-256 signatures over SHA-256 of the bodies on
    `threads` host threads while the device runs the previous batch's consensus.
    Reports the pipeline's events/s, the host verification rate alone, and how
    much verification time the device did not hide."""
    from babble_amd import signing
    from babble_amd.engine import Engine, events_array, verify_events
    from babble_amd.gossip import random_gossip, schedule
    dag = random_gossip(n, E, seed=seed)
    pubs, bodies, sigs = signing.signed_stream(dag, seed=seed, threads=threads)
    ev = events_array(dag)
    t0 = time.perf_counter()
    ok, _ = verify_events(bodies, pubs[dag["creator"]], sigs, threads=threads)
    vdt = time.perf_counter() - t0
    rep = Engine(n, E, device=device)
    _, rorder, _ = rep.replay(ev, schedule(E, K))
    rep.close()
    eng = Engine(n, E, device=device)
    rc, _, acc, tm = eng.ingest(ev, bodies, pubs, sigs, K, threads=threads)
    order = eng.consensus_log()
    eng.close()
    return {"workload": f"online path with signature checks, {n} participants, {E} events, hge_ingest "
                        f"(K={K}; ECDSA P-256 + SHA-256 of each body on {threads} host threads, overlapped "
                        f"with the device's consensus calls)",
            "value": round(len(order) / (tm["wall_ms"] / 1e3), 1), "unit": "events/s",
            "verify_only_events_per_s": round(E / vdt, 1),
            "verify_unhidden_ms": round(tm["verify_ms"], 1), "device_ms": round(tm["device_ms"], 1),
            "wall_ms": round(tm["wall_ms"], 1), "accepted": int(acc), "all_signatures_valid": bool(ok.all()),
            "parity": ("identical to the bulk replay" if rc == 0 and np.array_equal(order, rorder)
                       else "MISMATCH vs the bulk replay")}


def small_replay(n, E, K, seed, device, steps=20):
    """A second, small gossip line (configs[1]) checked bit-exact against the
    oracle over the whole stream."""
    from babble_amd.engine import Engine, events_array
    from babble_amd.gossip import random_gossip, schedule
    from oracle.oracle import replay as oracle_replay
    dag = random_gossip(n, E, seed=seed)
    calls = schedule(E, K)
    eng = Engine(n, E, device=device)
    eng.prepare(events_array(dag), calls)
    for _ in range(5):
        eng.run()
    t0 = time.perf_counter()
    for _ in range(steps):
        nord = eng.run()
    dt = (time.perf_counter() - t0) / steps
    _, gorder, _ = eng.fetch()
    eng.close()
    _, _, corder, _ = oracle_replay(dag, calls)
    return {"workload": f"random-gossip DAG, {n} participants, {E} events, RunConsensus every K={K}",
            "value": round(nord / dt, 1), "unit": "events/s", "ms_per_step": round(dt * 1e3, 4),
            "parity": ("bit-exact vs CPU oracle (full stream)" if np.array_equal(gorder, corder)
                       else "MISMATCH vs CPU oracle")}


def mc_kernel_bytes(kernel, n, events, ordered, rounds, calls=0):
    """Algorithmic bytes of one batch-engine stage over the whole batch:
    `events` accepted events, `ordered` ordered ones, `rounds` and `calls` summed over
    the graphs."""
    per_event = {
        "kb_coords": 4 * n + 16,  # the LA row written, the parents' creator / index / ids read
        "kb_fd": 8 * n,           # the LA row read, its firstDescendant runs written
        "kb_fdrows": 8 * n,       # the runs read, the firstDescendant row written
    }
    if kernel in per_event:
        return per_event[kernel] * events
    if kernel == "kb_front":
        # per round: N member rows and, per member, the N rows FD[(i, FD[w][i])]
        # (4N bytes each); per event its chain slot read and round / witness written
        return rounds * (4 * n * n + 4 * n * n * n) + 9 * events
    if kernel == "kb_fame":  # per (call, s) pair: two rounds' witness ids, vote bits and coins read, 16 B out
        return calls * 3 * (2 * 13 * n + 16)
    if kernel == "kb_fold":  # the pairs' decisions read, the arrivals; per round its thresholds
        return calls * 3 * 16 + rounds * 8 * n
    if kernel == "kb_receive":  # per event its round / creator / index / call read; per ordered one the FD row
        return 16 * events + (4 * n + 16) * ordered
    return (4 * n + 48) * ordered  # kb_order (kb_consensus): the median's rows and the sort key


def mc_main(args, n, E, K, rank, world, local_rank, dist):
    line = mc_line(args, n, E, K, rank, world, local_rank, dist)
    if line is not None:
        print(json.dumps(line), flush=True)


def mc_line(args, n, E, K, rank, world, local_rank, dist, cpu_s=10.0):
    """Config 5 on the batch engine: this rank's share of the Monte Carlo batch,
    one replay of all of it per step (five launches), every graph checked
    against the oracle's committed full-state digest.  Returns rank 0's line
    (None elsewhere); the CPU baseline takes about `cpu_s` seconds."""
    from babble_amd.dist import reduce_step, shard_range
    from babble_amd.engine import Batch
    from babble_amd.gossip import random_gossip, schedule
    first, per = shard_range(args.graphs, world, rank)
    t0 = time.perf_counter()
    dags = [random_gossip(n, E, seed=args.seed + first + g, forkers=10, fork_p=0.05, cascade_p=0.5)
            for g in range(per)]
    batch = Batch(n, device=local_rank)
    t_adm = time.perf_counter()
    for d in dags:
        batch.add(d, schedule(len(d["creator"]), K))
    batch.stage()
    admission_s = time.perf_counter() - t_adm
    ingest_s = time.perf_counter() - t0
    events = sum(len(d["creator"]) for d in dags)

    def sync_all():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    t_ramp = time.perf_counter()
    while time.perf_counter() - t_ramp < args.ramp_s:
        batch.run()
    for _ in range(args.warmup):
        batch.run()
    sync_all()
    kacc = {}
    t0 = time.perf_counter()
    ordered = 0
    for _ in range(args.steps):
        ordered = batch.run()
        for k_, v_ in batch.kernel_ms().items():  # HIP events between the launches, on the batch stream
            kacc[k_] = kacc.get(k_, 0.0) + v_
    t1 = time.perf_counter()
    sync_all()
    step_s = (t1 - t0) / args.steps
    kms = {k_: v_ / args.steps for k_, v_ in kacc.items()}
    tot_ordered, max_step = ordered, step_s
    if dist is not None:
        max_step, tot_ordered = reduce_step(dist, step_s, ordered, f"cuda:{local_rank}")

    rounds_tot = sum(batch.info(g)["rounds"] for g in range(per))
    calls_tot = sum(batch.info(g)["calls"] for g in range(per))
    # every graph of this rank against the oracle's full-state digest
    checks = []
    dg = mc_digests(n, E, K, args.seed)
    bad, nchk = 0, 0
    if dg is not None:
        sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
        from digest import digest
        for g in range(per):
            gi = first + g
            if gi >= len(dg):
                continue
            nchk += 1
            bad += digest(batch.state(g)) != dg[gi]
    if dist is not None:
        import torch
        t_ = torch.tensor([nchk, bad], dtype=torch.int64, device=f"cuda:{local_rank}")
        dist.all_reduce(t_)
        nchk, bad = int(t_[0].item()), int(t_[1].item())
    if nchk:
        checks.append(f"{'bit-exact' if bad == 0 else f'MISMATCH on {bad} graphs'} vs the oracle's "
                      f"full-state digests on {nchk} of {args.graphs} graphs (status, order, batches, rounds, "
                      f"witnesses, fame, round received, timestamps, undetermined, scalars; "
                      f"tests/golden/mc_*_digests.json)")
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        # the Go-faithful oracle on whole graphs of the batch, one core, ~10 s of work
        from oracle.oracle import replay as oracle_replay
        tc = time.perf_counter()
        tot, ng = 0, 0
        for d in dags:
            _, _, corder, _ = oracle_replay(d, schedule(len(d["creator"]), K))
            tot += len(corder)
            ng += 1
            if time.perf_counter() - tc > cpu_s:
                break
        cs = time.perf_counter() - tc
        cpu = {"value": round(tot / cs, 1), "unit": "events/s", "cores": 1, "kind": "port",
               "sample": f"Go-faithful C++ oracle (oracle/hg_oracle.cpp, faithful mode), the first {ng} graphs "
                         f"of the batch (whole graphs, K={K}), {tot} ordered in {cs:.2f} s on "
                         f"{platform.processor() or platform.machine()} (host nproc {os.cpu_count()})"}
    if rank != 0:
        batch.close()
        return None
    value = tot_ordered / max_step
    dom = max(kms, key=kms.get)
    kb = {k_: mc_kernel_bytes(k_, n, events, ordered, rounds_tot, calls_tot) for k_ in kms}
    alg = kb[dom]
    achieved = alg / (kms[dom] * 1e-3) / 1e9
    hbm = {k_: {"ms": round(v_, 4), "alg_bytes": kb[k_], "achieved_gbs": round(kb[k_] / (v_ * 1e-3) / 1e9, 2)}
           for k_, v_ in kms.items()}
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
        "config": {"workload": (f"Monte Carlo batch: {args.graphs} independent random-gossip hashgraphs, "
                                f"{n} participants, {E} submissions each, 10 forkers p=0.05 with cascades, "
                                f"RunConsensus every K={K}"),
                   "participants": n, "events_per_graph": E, "k": K, "graphs_per_gpu": per,
                   "ordered_per_step": tot_ordered,
                   "parallelism": f"replicas{world}: the batch split across {world} GPUs, no collective"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                     "traffic": pmc_traffic(f"mc_n{n}_e{E}_k{K}_g{args.graphs}" if world == 1 else None, dom, 1),
                     "algorithmic_bytes_per_launch": int(alg), "launch_ms": round(kms[dom], 4),
                     "hbm_kernels": hbm,
                     "path": {"bytes_per_event": 24 * n + 48,
                              "achieved_gbs": round(value / world * (24 * n + 48) / 1e9, 2),
                              "frac": round(value / world * (24 * n + 48) / 1e9 / HBM_PEAK_GBS, 5)}},
        "cpu_baseline": cpu,
        "parity": "; ".join(checks) if checks else None,
        "ingest_host_ms": round(ingest_s * 1e3, 2),
        "admission_ms": round(admission_s * 1e3, 2),
        "kernels_ms_per_replay": {k_: round(v_, 4) for k_, v_ in sorted(kms.items(), key=lambda kv: -kv[1])},
        "kernel_launches_per_replay": {"kb_coords": 1 if per > 512 else 2, "kb_fd": 1, "kb_fdrows": 1, "kb_front": 1, "kb_fame": 2,
                                       "kb_fold": 2, "kb_receive": 1, "kb_order": 2},
        "graphs_replayed_call_by_call": batch.fallbacks(),
    }
    batch.close()
    return line


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
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--cpu-sample-events", type=int, default=None,
                    help="CPU baseline prefix (default: 20480 at N >= 128, 100k below)")
    ap.add_argument("--profile-steps", type=int, default=1)
    ap.add_argument("--replicas", action="store_true",
                    help="gossip, N > 1: one independent hashgraph per rank (weak scaling) instead of "
                         "ONE hashgraph sharded across the ranks (babble_amd.dist.split_run)")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="torch.distributed backend (nccl = RCCL; gloo: rehearsing N ranks on one GPU)")
    args = ap.parse_args()
    mc = args.workload == "mc"
    n = args.participants or (32 if mc else DEFAULT[0])
    E = args.events or (10_000 if mc else DEFAULT[1])
    K = args.k or n

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist_
        # one GPU per rank; ranks past the box's GPU count share them (--dist-backend gloo)
        local_rank = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local_rank)
        dist_.init_process_group(args.dist_backend)
        dist = dist_

    if mc:
        mc_main(args, n, E, K, rank, world, local_rank, dist)
        if dist is not None:
            dist.destroy_process_group()
        return

    from babble_amd.dist import reduce_step
    from babble_amd.engine import Engine, events_array
    from babble_amd.gossip import random_gossip, schedule

    # ---- stage the workload in HBM (host admission + upload; not timed) ----
    t0 = time.perf_counter()
    split = not args.replicas and world > 1
    # split: every rank stages the same stream (seed, not seed + rank)
    dags = [random_gossip(n, E, seed=args.seed + (0 if split else rank))]
    engines = [Engine(n, E, device=local_rank)]
    ev0 = events_array(dags[0])
    t_adm = time.perf_counter()
    engines[0].prepare(ev0, schedule(E, K))
    admission_s = time.perf_counter() - t_adm
    del ev0
    ingest_s = time.perf_counter() - t0

    exchange, split_stats = None, {}
    if split:
        from babble_amd.dist import TorchExchange, split_run
        exchange = TorchExchange(dist, f"cuda:{local_rank}")

    def step():
        if split:
            return split_run(engines[0], rank, world, exchange, stats=split_stats)
        return engines[0].run()

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
    f0 = split_stats.get("fallback", 0)
    t0 = time.perf_counter()
    ordered = 0
    for _ in range(args.steps):
        ordered = step()  # every engine returns after its stream drained
    t1 = time.perf_counter()
    sync_all()
    step_s = (t1 - t0) / args.steps

    # ---- one more unprofiled replay: GPU-busy vs wall split of a step ----
    eng0 = engines[0]
    nfall = split_stats.get("fallback", 0) - f0
    if split:
        sync_all()
        step()
    else:
        eng0.run()
    st_ms = eng0.stage_times()
    replay_ms = {"coords_gpu": st_ms[0], "coords_wall": st_ms[1], "consensus_gpu": st_ms[3],
                 "consensus_wall": st_ms[2], "gpu": st_ms[6], "wall": st_ms[4],
                 "order_delivery_wall": st_ms[5]}
    replay_ms = {k: round(v, 4) for k, v in replay_ms.items()}
    # the step ends with the order in host memory (one DMA copy into the pinned buffer
    # sized at hge_replay_prepare, replay_ms.order_delivery_wall); copying it out into a
    # caller's array is timed apart
    t_f = time.perf_counter()
    gstatus, gorder, gcounts = eng0.fetch()
    order_fetch_ms = (time.perf_counter() - t_f) * 1e3

    # ---- profiled pass: per-kernel device time (HIP events on the engine stream) ----
    nprof = max(1, args.profile_steps)
    eng0.set_profiling(True)
    for _ in range(nprof):
        step() if split else eng0.run()
    kstats = eng0.kernel_stats()
    eng0.set_profiling(False)
    ev0 = len(dags[0]["creator"])
    ord0 = eng0._nordered
    sweeps = eng0.coordinate_sweeps()

    tot_ordered, max_step = ordered, step_s
    if dist is not None:
        max_step, tot_ordered = reduce_step(dist, step_s, ordered, f"cuda:{local_rank}")
        if split:
            tot_ordered = ordered  # one hashgraph for the whole job

    def kernel_roofline(name):
        """(algorithmic bytes per launch, average launch ms, achieved GB/s).
        The algorithmic bytes of a replay are spread over the launches that did
        work: for k_la_sweep the sweeps up to the first quiet one (the queued
        launches after it return at once and are left out)."""
        ms, cnt = kstats[name]
        base = name.strip("()").split("<")[0]
        launches = sweeps * nprof if base in ("k_la_sweep", "k_la_sweep16") else cnt
        per_replay = launches / nprof
        b = algorithmic_bytes(name, n, ev0, ord0, eng0.rounds()) / max(per_replay, 1)
        per_launch = ms / max(launches, 1)
        return b, per_launch, b / (per_launch * 1e-3) / 1e9, per_replay

    dom = max(kstats.items(), key=lambda kv: kv[1][0])[0]
    alg, per_launch_ms, achieved, dom_lpr = kernel_roofline(dom)
    # every kernel that streams the N-wide tables, with its roofline
    hbm_kernels = {}
    for name in kstats:
        base = name.strip("()").split("<")[0]
        if base in ("k_la_sweep", "k_la_clear", "k_transpose", "k_fss",
                    "k_fdt_clear", "k_rounds_coop", "k_rounds_coop_spec", "k_median_wave",
                    "k_la_clear16", "k_la_sweep16", "k_la16_rows_runs", "k_rounds_direct",
                    "k_fd_transpose_ts", "k_witness_la", "k_la_win", "k_lw_plan"):
            b, pl, gbs, lpr = kernel_roofline(name)
            hbm_kernels[name] = {"achieved_gbs": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
                                 "alg_bytes_per_launch": int(b), "launch_ms": round(pl, 4),
                                 "launches_per_replay": lpr}
            if base == "k_fd_transpose_ts":
                # SURVEY 8(d)'s FD write alone (the FDT read and the offsets excluded)
                fdw = (2 if "uint16_t" in name else 4) * n * ev0 / max(lpr, 1)
                hbm_kernels[name]["fd_write_frac"] = round(fdw / (pl * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)

    cpu, parity, checks = None, None, []
    if rank == 0:
        gp = golden_prefix(n, E, K, args.seed)
        if gp is not None:
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            from parity import check_prefix
            nc = int(gp["n_calls"])
            rounds_, wit_ = eng0.event_rounds()
            rr_, cts_ = eng0.event_received()
            bad = check_prefix(gp, gorder, gcounts, rounds_, wit_, rr_, cts_, eng0.fame_table())
            full = "rounds" in gp.files
            what = ("order, batches, rounds, witnesses, round received, timestamps, fame to LCR "
                    f"{int(gp['scalars'][1])}" if full else "order and batches")
            checks.append(f"{'bit-exact' if not bad else 'MISMATCH in ' + ','.join(bad)} vs committed oracle "
                          f"golden ({what}; first {int(gp['prefix'])} submissions, {nc} calls, "
                          f"{len(gp['order'])} ordered)")
        gf = golden_full(n, E, K, args.seed)
        if gf is not None:
            # the whole stream: every field of the parity contract against the
            # oracle's digests (tests/golden/make_bench_full.py); a sharded run
            # holds the whole order and batches on every rank, the per-event
            # fields only for its own slice
            sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
            from digest import compare_full, engine_state
            only = ("order", "counts") if split else None
            bad = compare_full(engine_state(eng0, gstatus, gorder, gcounts), gf, only)
            what = "order, batches" if split else ("status, order, batches, rounds, witnesses, fame, round "
                                                   "received, timestamps, undetermined, scalars")
            checks.append(f"{'bit-exact' if not bad else 'MISMATCH in ' + ','.join(bad)} vs the oracle's "
                          f"whole-stream digests ({what}; all {gf['n_calls']} calls, {gf['ordered']} ordered, "
                          f"{gf['scalars'][0]} rounds, LCR {gf['scalars'][1]})")
    if rank == 0 and not args.no_cpu_baseline:
        from oracle.oracle import replay as oracle_replay
        d = dags[0]
        ns = args.cpu_sample_events or (20480 if n >= 128 else 100_000)
        ns = min(ns, len(d["creator"]))
        ns = max(K, ns // K * K)  # whole calls only: the prefix's calls are the full run's
        sub = sub_stream(d, ns)
        calls = schedule(ns, K)
        t0 = time.perf_counter()
        _, _, corder, ccounts = oracle_replay(sub, calls)
        cs = time.perf_counter() - t0
        what = f"first {ns} of {len(d['creator'])} submissions of the same stream"
        cpu = {"value": round(len(corder) / cs, 1), "unit": "events/s", "cores": 1, "kind": "port",
               "sample": f"Go-faithful C++ oracle (oracle/hg_oracle.cpp), {what}, K={K}, "
                         f"{len(corder)} ordered in {cs:.2f} s on "
                         f"{platform.processor() or platform.machine()} (host nproc {os.cpu_count()})"}
        ok = (np.array_equal(gcounts[:len(calls)], ccounts) and
              np.array_equal(gorder[:len(corder)], corder))
        checks.append(f"{'bit-exact' if ok else 'MISMATCH'} vs CPU oracle run live "
                      f"(first {ns} submissions, {len(calls)} calls, {len(corder)} ordered)")
    if rank == 0:
        parity = "; ".join(checks) if checks else None

    secondary = None
    if split:
        # the same job as independent replicas (every rank replays the whole stream on
        # its own GPU, no collective): the weak-scaling line next to the strong one
        sync_all()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            rep_ordered = eng0.run()
        t1 = time.perf_counter()
        sync_all()
        rep_step, rep_tot = reduce_step(dist, (t1 - t0) / args.steps, rep_ordered, f"cuda:{local_rank}")
        secondary = {"replicas": {
            "workload": f"{world} independent replays of the same stream, one per GPU (no collective)",
            "value": round(rep_tot / rep_step, 1), "unit": "events/s", "ms_per_step": round(rep_step * 1e3, 4),
            "scaling": "weak"}}
    if rank == 0 and not args.no_secondary and (n, E) == DEFAULT and world == 1:
        secondary = {"replay_16_100k": small_replay(16, 100_000, 16, args.seed, local_rank),
                     "online_16_100k": online_path(16, 100_000, 16, args.seed, local_rank),
                     "online_64_1m": online_path(64, 1_000_000, 64, args.seed, local_rank),
                     "online_256_prefix": online_path(
                         n, ONLINE_PREFIX, K, args.seed, local_rank, dag=dags[0],
                         what=f"online per-call path on the first {ONLINE_PREFIX} submissions of the bench's own "
                              f"{n}-participant stream, hge_insert_events(K={K}) + hge_run_consensus per call "
                              f"({len(schedule(ONLINE_PREFIX, K))} calls)"),
                     "ingest_16_100k": ingest_path(16, 100_000, 16, args.seed, local_rank)}
        # config 5 (BASELINE configs[4]) on the batch engine, the same steps as this line
        import copy
        mca = copy.copy(args)
        mca.graphs = 1024
        secondary["mc_1024x32x10k"] = mc_line(mca, 32, 10_000, 32, 0, 1, local_rank, None, cpu_s=5.0)

    if rank == 0:
        value = tot_ordered / max_step
        workload = (f"random-gossip DAG, {n} participants, {E} events "
                    f"{'in one hashgraph' if split else 'per GPU'}, "
                    f"RunConsensus every K={K} events ({len(schedule(E, K))} calls)")
        cfg_key = f"{args.workload}_n{n}_e{E}_k{K}"
        line = {
            "metric": "consensus-ordered events/sec at N participants",
            "value": round(value, 1),
            "unit": "events/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(max_step * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if split else "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic",
            "config": {"workload": workload, "participants": n, "events_per_graph": E, "k": K,
                       "graphs_per_gpu": 1, "ordered_per_step": tot_ordered,
                       "parallelism": ((f"shard{world}: one hashgraph sharded by time across {world} GPUs "
                                        f"(fame by round, round received / median / order by call; RCCL "
                                        f"all-gathers; coordinates and the sequential rounds walk on every "
                                        f"rank)") if split else f"replicas{world}")},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": pmc_traffic(cfg_key, dom, dom_lpr),
                         "traffic_unit": "HBM bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)",
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
            "admission_ms": None if admission_s is None else round(admission_s * 1e3, 2),
            "replay_ms": replay_ms,
            "order_fetch_copy_ms": round(order_fetch_ms, 3),
            "coordinate_sweeps": sweeps,
            "rounds": eng0.rounds(),
            "kernels_ms_per_replay": {k: round(v[0] / nprof, 4) for k, v in
                                      sorted(kstats.items(), key=lambda kv: -kv[1][0])},
            "kernel_launches_per_replay": {k: v[1] // nprof for k, v in kstats.items()},
        }
        if split:
            # timed steps that fell back to the unsplit replay (HGE_ERR_SPLIT): 0 means
            # every timed step ran sharded
            line["split_fallbacks"] = nfall
        if secondary is not None:
            line["secondary"] = secondary
        print(json.dumps(line), flush=True)
    for e in engines:
        e.close()
    if os.environ.get("HGE_DUMP_MAPS"):
        # diagnostics for crashes after main (rocprofv3 exit SIGSEGV): the library map
        with open("/proc/self/maps") as f, open(os.environ["HGE_DUMP_MAPS"], "w") as g:
            g.write(f.read())
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
