"""Multi-GPU layer of the engine (one process per GPU, torch.distributed).

Two ways to use N GPUs:
  * independent hashgraphs (gossip replicas, the Monte Carlo batch of config 5)
    shard with no data-path collective: ranks only agree on who replays what
    (shard_range) and combine their step times and event counts (reduce_step);
  * ONE hashgraph split across GPUs (split_run): every rank holds the whole
    stream and its coordinates; the rounds frontier recurrence, the longest
    sequential stage, is walked by one walker per rank from a
    different start (rank 0 from the true first frontier, rank p from the time
    cut at p * E / nranks); the ranks all-gather their rows (one collective) and
    every rank joins them (join_histories) and finishes the replay.  The join is
    exact: the recurrence C_{r+1} = F(C_r) is a function of the row alone, so a
    walker whose row equals a row of the true trajectory continues it.
torch.distributed is plumbing here: "nccl" (RCCL over xGMI) on the GPU box,
"gloo" in the CPU tests.
"""
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


def split_run(eng, rank, world, gather, extra=256):
    """One replay of the staged stream (eng.prepare) with the rounds walk split
    across `world` ranks.  gather(obj) -> [obj of every rank] (all-gather).
    Returns the number of events ordered (identical to eng.run())."""
    eng.split_begin()
    start = eng.frontier_guess(rank, world)
    stop = eng.frontier_guess(rank + 1, world) if rank + 1 < world else None
    hist = eng.frontier_walk(start, stop, extra if stop is not None else 0)
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
        nmax = max(counts)
        r = torch.full((nmax, N), INF32, dtype=torch.int32, device=device)
        r[:n] = torch.from_numpy(rows).to(device)
        s = torch.zeros((nmax, N, NW), dtype=torch.int64, device=device)
        s[:n] = torch.from_numpy(ssc.view(np.int64)).to(device)
        rs = [torch.empty_like(r) for _ in range(world)]
        ss = [torch.empty_like(s) for _ in range(world)]
        dist.all_gather(rs, r)
        dist.all_gather(ss, s)
        return [(rs[g][:counts[g]].cpu().numpy(), ss[g][:counts[g]].cpu().numpy().view(np.uint64),
                 bool(metas[g][1].item())) for g in range(world)]
    return gather
