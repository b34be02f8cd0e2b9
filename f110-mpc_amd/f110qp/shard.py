"""Batch sharding over the GPUs of one node.

QPs are independent, so a global batch is split into contiguous per-rank ranges with no
collective on the data path. Ranges are aligned to the candidate-group size (e.g. 120
candidates of one scenario share x0 and the linearisation point) so that a scenario never
straddles two GPUs. The collectives are the optional result gather to every rank (all_gather
over RCCL/xGMI on GPUs, gloo in the CPU tests: a few KB per QP batch) and the per-scenario
min-loc of the downstream selection (select_sharded: two all_reduce MIN over [scenarios] words),
needed when a scenario's candidates straddle ranks (any split not aligned to the scenarios).
"""
from __future__ import annotations

from typing import Callable, Dict


def shard_range(total: int, world: int, rank: int, align: int = 1):
    """Contiguous [lo, hi) of `total` items for `rank`, boundaries multiples of `align`
    (except the end). Every item is owned by exactly one rank."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    if align < 1:
        raise ValueError("align must be >= 1")
    groups = -(-total // align)
    per = groups // world
    extra = groups % world
    g_lo = rank * per + min(rank, extra)
    g_hi = g_lo + per + (1 if rank < extra else 0)
    return min(total, g_lo * align), min(total, g_hi * align)


def solve_sharded(solve_fn: Callable[[Dict], Dict], inputs: Dict, group_align: int = 1, gather: bool = True,
                  pg=None) -> Dict:
    """Run `solve_fn` on this rank's shard of `inputs` (dict of tensors with the batch in dim 0)
    and, if `gather`, all-gather the per-rank outputs into the global batch on every rank."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(pg) if dist.is_initialized() else 1
    rank = dist.get_rank(pg) if dist.is_initialized() else 0
    total = next(iter(inputs.values())).shape[0]
    lo, hi = shard_range(total, world, rank, group_align)
    out = solve_fn({k: (v[lo:hi] if v is not None else None) for k, v in inputs.items()})
    if not gather or world == 1:
        return out
    sizes = [shard_range(total, world, r, group_align) for r in range(world)]
    maxn = max(h - l for l, h in sizes)
    res = {}
    for k, v in out.items():
        pad = torch.zeros((maxn,) + tuple(v.shape[1:]), dtype=v.dtype, device=v.device)
        pad[: v.shape[0]] = v
        bufs = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(bufs, pad, group=pg)
        res[k] = torch.cat([b[: h - l] for b, (l, h) in zip(bufs, sizes)], 0)
    return res


INDEX_NONE = (1 << 62)  # "no solved candidate on this rank" in the index all-reduce


def select_sharded(best, winner, pg=None):
    """Min-loc over the ranks of the per-scenario selection: every rank
    holds, for ALL scenarios g (global ids), its local best cost best[g] (float64, +inf when it
    has no solved candidate of g) and the GLOBAL index winner[g] of that candidate (int, -1 none),
    e.g. from f110qp_select_dev on its shard plus the shard offset. Returns the global (best,
    winner) on every rank: the minimal cost over all ranks, ties to the smallest global index.
    The min-loc is exact over the costs the ranks hold. Those equal the costs one process would
    compute over the whole batch only when every rank's launch is the same kernel: the launch
    policy depends on the per-rank batch size (lane_seg_kernel's S, lane vs wave back end), so
    costs can differ in the last bits and a near-tie (candidates within rounding of each other)
    may resolve to the other one; up to that it is what one process selecting over the whole
    batch returns (tests/test_gpu_shard.py checks both cases). Two all_reduce(MIN) of G words
    each (RCCL over xGMI with the nccl backend: device tensors; gloo: host tensors)."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized():
        return best, winner
    # (a world of one still runs the two all_reduces: an identity, and the RCCL path exercised)
    on_dev = dist.get_backend(pg) == "nccl"
    dev = best.device if on_dev else torch.device("cpu")
    b = best.to(dev, torch.float64).clone()
    w = winner.to(dev, torch.int64)
    dist.all_reduce(b, op=dist.ReduceOp.MIN, group=pg)
    mine = (w >= 0) & (best.to(dev, torch.float64) == b)
    idx = torch.where(mine, w, torch.full_like(w, INDEX_NONE))
    dist.all_reduce(idx, op=dist.ReduceOp.MIN, group=pg)
    idx = torch.where(idx == INDEX_NONE, torch.full_like(idx, -1), idx)
    return b.to(best.device), idx.to(winner.device)
