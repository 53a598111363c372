"""Group-per-GPU sharding: the host-side rule that assigns
Raft groups to GPUs and the once-per-report reduction of statistics.

Groups are independent, so the data path has no collective: rank r owns the
clusters with cid % world == r % world — dragonboat's FixedPartitioner rule
(internal/server/partition.go:28-40, used by execEngine at
execengine.go:89-101 to pick a step worker).  The engine numbers its groups
g = 0..G-1 and names group g's cluster cid_base + g * cid_stride, so the
rank's share is cid_base = 1 + r, cid_stride = world (cluster ids start at 1).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple


def shard_params(rank: int, world: int) -> Tuple[int, int]:
    """(cid_base, cid_stride) of the engine on `rank` of `world` GPUs."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    return 1 + rank, world


def cluster_ids(rank: int, world: int, groups_per_rank: int) -> List[int]:
    base, stride = shard_params(rank, world)
    return [base + g * stride for g in range(groups_per_rank)]


def owner_of(cluster_id: int, world: int) -> int:
    """FixedPartitioner.GetPartitionID (partition.go:38-40) with the 1-based
    cluster ids used here: the rank that steps `cluster_id`."""
    return (cluster_id - 1) % world


def reduce_results(dist, wall: float, sums: Sequence[float], device=None):
    """Max-over-ranks wall time and sum-over-ranks counters (one all_reduce
    each; the only collective — statistics, not protocol data)."""
    import torch
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return wall, [float(x) for x in sums]
    w = torch.tensor([wall], dtype=torch.float64, device=device)
    s = torch.tensor([float(x) for x in sums], dtype=torch.float64, device=device)
    dist.all_reduce(w, op=dist.ReduceOp.MAX)
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    return float(w.item()), [float(x) for x in s.cpu().tolist()]
