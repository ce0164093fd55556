"""Multi-GPU plumbing of the benchmark / Monte Carlo driver (one process per GPU).

The ordering path itself has no data-path collective: independent hashgraphs
(replays of config 2, the Monte Carlo batch of config 5) shard perfectly, so
ranks only agree on who replays what and combine their step times and event
counts at the end.  torch.distributed is plumbing here: "nccl" (RCCL over
xGMI) on the GPU box, "gloo" in the CPU tests.
"""


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
