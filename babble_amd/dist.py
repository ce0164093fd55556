"""Multi-GPU layer of the engine (one process per GPU, torch.distributed).

Two ways to use N GPUs:
  * independent hashgraphs (gossip replicas, the Monte Carlo batch of config 5)
    shard with no data-path collective: ranks only agree on who replays what
    (shard_range) and combine their step times and event counts (reduce_step);
  * ONE hashgraph sharded by time across GPUs (split_run, north_star's config 4
    at 2/4/8 GPUs).  Part p owns the events inserted during its share of the
    RunConsensus calls (split_plan).  Every rank computes the coordinates and
    walks the rounds recurrence: it is sequential over rounds, and walkers
    started mid-stream rarely meet the true trajectory (profiles/r03/split), so it
    is not split.  DecideFame is sharded by round (each rank decides the (round,
    call) pairs of the rounds whose first witness it owns) and the decisions are
    all-gathered over RCCL; DecideRoundReceived, MedianTimestamp and FindOrder's
    call buckets are sharded by call, and the ordered slices are all-gathered.
    Every rank ends with the whole replay's state, identical to the one-GPU
    replay; a stream the candidate halo does not cover (HGE_ERR_SPLIT, every rank
    at the same point) is replayed unsplit.
  * walk_split_run is DIAGNOSTIC only: round 2's walk-only split (walkers + one
    all-gather of their rows), kept for the convergence measurements of
    scripts/analysis/split_converge.py; bench.py no longer offers it (its walkers
    do not meet at N = 256, profiles/r03/split).
torch.distributed is plumbing here: "nccl" (RCCL over xGMI) on the GPU box,
"gloo" in the CPU tests.
"""
import threading

import numpy as np

INF32 = np.iinfo(np.int32).max


def shard_range(total, world, rank):
    """Contiguous share of `total` independent items for `rank`: (first, count).
    Shares differ by at most one and cover [0, total) exactly once."""
    base, extra = divmod(total, world)
    count = base + (1 if rank < extra else 0)
    first = rank * base + min(rank, extra)
    return first, count


def reduce_step(dist, step_s, ordered, device="cpu"):
    """Whole-job step time (max over ranks) and events ordered (sum over ranks)."""
    import torch
    t = torch.tensor([float(step_s)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    o = torch.tensor([float(ordered)], dtype=torch.float64, device=device)
    dist.all_reduce(o, op=dist.ReduceOp.SUM)
    return float(t.item()), int(o.item())


# One round of random gossip spans about 14 positions of every chain (DESIGN.md
# §4.2), i.e. ~14 N events: the candidate halo is set in rounds.
ROUND_EVENTS_PER_PARTICIPANT = 16


def split_plan(call_events, n_events, world, halo_lo):
    """Time shards of one replay (hge_split_plan, include/hge.h).

    call_events: events accepted at each RunConsensus call (ascending).  Part g
    owns the calls [cb[g], cb[g+1]) (equal shares) and the events inserted during
    them, [ev[g], ev[g+1]) with ev[g] = the count at call cb[g] - 1 (the last part
    also takes any events after the last call).  Its candidates for the order start
    halo_lo events earlier (events its calls receive late).
    Returns {"ev_bounds", "call_bounds", "cand_lo"} (lists)."""
    ncalls = len(call_events)
    if world < 1 or ncalls < world:
        raise ValueError(f"split_plan: {ncalls} calls cannot be shared by {world} parts")
    cb = [ncalls * g // world for g in range(world + 1)]
    ev = [0] + [int(call_events[cb[g] - 1]) for g in range(1, world)] + [int(n_events)]
    for g in range(world):
        if ev[g + 1] <= ev[g]:
            raise ValueError(f"split_plan: part {g} holds no events")
    cand_lo = [max(0, ev[g] - halo_lo) for g in range(world)]
    return {"ev_bounds": ev, "call_bounds": cb, "cand_lo": cand_lo}


def join_histories(hists):
    """Join the walkers' rows into the true frontier trajectory.

    hists: per rank (rows [n, N] int32, ssc [n, N, NW] uint64, natural): rank 0's
    walk starts at the true first frontier.  Following rank g from row i, a row
    that also appears in a later rank g' (at row j) hands the walk over to g'
    from row j on.  Returns (rows [K, N], ssc [K, N, NW], natural): natural = the
    trajectory reached the empty frontier (Rounds() = K); otherwise it stops at
    the end of a walker's history and the sequential walk resumes from row K-1.
    """
    G = len(hists)
    # each row -> the FURTHEST walker that holds it: walker p runs past walker
    # p + 1's start, so a row on the true trajectory is often in both, and the
    # join must move on to p + 1 (a later rank overwrites an earlier one)
    index = {}
    for g in range(1, G):
        rows = hists[g][0]
        for i in range(len(rows)):
            index[rows[i].tobytes()] = (g, i)
    out_r, out_s = [], []
    g, i = 0, 0
    while True:
        rows, ssc, _ = hists[g]
        row = rows[i]
        if (row == INF32).all():  # the empty frontier: the walk ended
            return np.stack(out_r), np.stack(out_s), True
        out_r.append(row)
        out_s.append(ssc[i])
        hit = index.get(row.tobytes())
        if hit is not None and hit[0] > g:
            g, i = hit
            rows = hists[g][0]
        if i + 1 < len(rows):
            i += 1
            continue
        return np.stack(out_r), np.stack(out_s), False


def split_run(eng, rank, world, exchange, halo_rounds=8, stats=None):
    """This rank's part of one replay of the staged stream (eng.prepare) sharded
    across `world` ranks (hge_split_run).  exchange: the engine's all-gather
    (TorchExchange / ThreadExchange).  Returns the number of events ordered
    (identical to eng.run()); stats["fallback"] counts unsplit replays."""
    from .engine import HGE_ERR_SPLIT, HgeError
    if world <= 1:  # nothing to shard: the one-GPU replay
        return eng.run()
    plan = split_plan(eng.call_events(), eng.event_count(), world,
                      halo_rounds * ROUND_EVENTS_PER_PARTICIPANT * eng.n)
    eng.split_plan(rank, world, plan)
    eng.set_exchange(exchange)
    try:
        return eng.split_run()
    except HgeError as e:
        # every rank meets the same condition at the same point (the coverage flags
        # are exchanged): all replay unsplit
        if e.code != HGE_ERR_SPLIT:
            raise
        if stats is not None:
            stats["fallback"] = stats.get("fallback", 0) + 1
            stats["fallback_reason"] = str(e)
        eng.split_plan(rank, 0)
        return eng.run()


def walk_rows(eng, rank, world, extra):
    """This rank's walker (hge_frontier_walk) from its time cut, until `extra` rows
    past the next rank's cut."""
    start = eng.frontier_guess(rank, world)
    stop = eng.frontier_guess(rank + 1, world) if rank + 1 < world else None
    return eng.frontier_walk(start, stop, extra if stop is not None else 0)


def walk_split_run(eng, rank, world, gather, extra=256):
    """DIAGNOSTIC (not a production path).  Round 2's walk-only split: every rank computes everything but the rounds
    walk, which is walked by one walker per rank from its time cut; the rows are
    all-gathered (gather(obj) -> [obj of every rank]) and joined.  Exact; the
    sequential walk resumes where the walkers did not meet, which at N = 256 is
    most of the time (profiles/r03/split)."""
    eng.split_begin()
    hist = walk_rows(eng, rank, world, extra)
    rows, ssc, natural = join_histories(gather(hist))
    return eng.split_finish(rows, ssc, natural)


def torch_gather(dist, device="cpu"):
    """gather(obj) for split_run over torch.distributed: the histories travel as
    int32 / uint64 tensors (sizes first), one all-gather each."""
    import torch

    def gather(h):
        rows, ssc, natural = h
        world = dist.get_world_size()
        n, N = rows.shape
        NW = ssc.shape[2] if ssc.ndim == 3 else 1
        meta = torch.tensor([n, int(natural)], dtype=torch.int64, device=device)
        metas = [torch.zeros_like(meta) for _ in range(world)]
        dist.all_gather(metas, meta)
        counts = [int(m[0].item()) for m in metas]
        nmax = max(max(counts), 1)
        r = torch.full((nmax, N), INF32, dtype=torch.int32, device=device)
        r[:n] = torch.from_numpy(rows).to(device)
        s = torch.zeros((nmax, N, NW), dtype=torch.int64, device=device)
        s[:n] = torch.from_numpy(np.ascontiguousarray(ssc).reshape(n, N, NW).view(np.int64)).to(device)
        rs = [torch.empty_like(r) for _ in range(world)]
        ss = [torch.empty_like(s) for _ in range(world)]
        dist.all_gather(rs, r)
        dist.all_gather(ss, s)
        return [(rs[g][:counts[g]].cpu().numpy(), ss[g][:counts[g]].cpu().numpy().view(np.uint64),
                 bool(metas[g][1].item())) for g in range(world)]
    return gather


class TorchExchange:
    """The engine's all-gather (hge_split_exchange) over torch.distributed.

    The slots live in a torch tensor on this rank's GPU: op 0 hands out
    world * bytes of it, op 1 all-gathers the slots in place -- one
    all_gather_into_tensor (RCCL over xGMI) with the "nccl" backend; through host
    memory with "gloo" (the CPU-backend tests)."""

    def __init__(self, dist, device):
        import torch
        self.torch, self.dist, self.device = torch, dist, torch.device(device)
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.nccl = dist.get_backend() == "nccl"
        self.buf = None
        self.inp = None

    def __call__(self, op, nbytes):
        torch = self.torch
        if op == 0:
            need = nbytes * self.world
            if self.buf is None or self.buf.numel() < need:
                self.buf = torch.empty(need, dtype=torch.uint8, device=self.device)
            return self.buf.data_ptr()
        out = self.buf[:nbytes * self.world]
        mine = out[self.rank * nbytes:(self.rank + 1) * nbytes]
        if self.nccl:
            if self.inp is None or self.inp.numel() < nbytes:
                self.inp = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
            inp = self.inp[:nbytes]
            inp.copy_(mine)
            self.dist.all_gather_into_tensor(out, inp)
        else:
            parts = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(self.world)]
            self.dist.all_gather(parts, mine.cpu())
            out.copy_(torch.cat(parts).to(self.device))
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()
        return None


class ThreadExchange:
    """The all-gather between the parts of a split replay driven by threads of one
    process on one GPU (tests: every part on its own engine).  make(part) gives
    part's exchange function."""

    def __init__(self, world, device=0):
        import torch
        self.torch, self.world = torch, world
        self.device = torch.device(f"cuda:{device}")
        self.bufs = [None] * world
        self.nbytes = 0
        self.bar = threading.Barrier(world)

    def make(self, part):
        torch = self.torch

        def fn(op, nbytes):
            if op == 0:
                need = nbytes * self.world
                if self.bufs[part] is None or self.bufs[part].numel() < need:
                    self.bufs[part] = torch.empty(need, dtype=torch.uint8, device=self.device)
                return self.bufs[part].data_ptr()
            self.bar.wait()
            mine = self.bufs[part]
            for g in range(self.world):
                if g != part:
                    mine[g * nbytes:(g + 1) * nbytes].copy_(self.bufs[g][g * nbytes:(g + 1) * nbytes])
            torch.cuda.synchronize(self.device)
            self.bar.wait()  # nobody reuses its slot before every part has read it
            return None
        return fn


class ThreadGather:
    """gather(obj) between threads of one process (the walkers' rows)."""

    def __init__(self, world):
        self.world = world
        self.items = [None] * world
        self.bar = threading.Barrier(world)

    def make(self, part):
        def gather(obj):
            self.items[part] = obj
            self.bar.wait()
            out = list(self.items)
            self.bar.wait()
            return out
        return gather
