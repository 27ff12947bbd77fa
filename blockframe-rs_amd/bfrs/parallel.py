"""Multi-GPU partitioning for the RS path.

The code acts independently on every 64-byte chunk (32 symbols) of a shard,
so work shards across GPUs with no exchange step:

  * weak scaling (bench default): every rank owns an independent batch of
    RS blocks (BlockFrame's blocks are independent, src/chunker/commit.rs:391);
  * strong scaling (config C4, 10 GiB over 1/2/4/8 GPUs): rank g owns the
    byte range stripe_ranges(S, G)[g] of EVERY shard of every block, 64-byte
    aligned, so 11 blocks balance perfectly on 8 GPUs.

No collective touches the data path; the only collectives are the timing
barrier and the max-over-ranks reduction of the elapsed time.
"""
from __future__ import annotations

CHUNK = 64  # reed-solomon-simd symbol chunk


def stripe_ranges(shard_bytes: int, world: int):
    """[(start, end)) per rank, 64-byte aligned, covering [0, shard_bytes).
    A shard's tail chunk (shard_bytes % 64) goes to the last rank, so every
    rank except the last holds whole chunks."""
    if world < 1:
        raise ValueError("world must be >= 1")
    chunks = shard_bytes // CHUNK
    out = []
    for g in range(world):
        a = chunks * g // world
        b = chunks * (g + 1) // world
        start, end = a * CHUNK, b * CHUNK
        if g == world - 1:
            end = shard_bytes
        out.append((start, end))
    return out


def max_over_ranks(value: float, dist=None, device=None) -> float:
    """Max of a per-rank float over all ranks (identity without a process group)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    import torch
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_over_ranks(value: float, dist=None, device=None) -> list:
    """Every rank's float, in rank order (a one-element list without a process group)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return [value]
    import torch
    t = torch.tensor([value], dtype=torch.float64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(x.item()) for x in out]


def throughput(bytes_per_rank_per_step: float, world: int, steps: int, elapsed_max: float,
               scaling: str) -> float:
    """Whole-job GiB/s: weak = every rank processed its own bytes; strong = the
    ranks together processed one job's bytes (bytes_per_rank_per_step is then
    the whole job's bytes)."""
    total = bytes_per_rank_per_step * (world if scaling == "weak" else 1) * steps
    return total / 2**30 / elapsed_max
