"""Sharding of Raft groups over the GPUs of one node.

The rule is the reference's own partitioner: a cluster lands on partition ``clusterID % capacity``
(``FixedPartitioner.GetPartitionID``, internal/server/partition.go:38), the same rule that picks a
step worker (``workReady.clusterReady``, execengine.go:115-123). With 16 step workers and 8 GPUs,
16 % 8 == 0 keeps every step worker's clusters on one GPU (``DoubleFixedPartitioner``,
partition.go:59-61). Groups are independent, so sharding needs no data-path collective.
"""
from __future__ import annotations

from dataclasses import dataclass

MIXED_VOTERS = (3, 5, 7)  # n = MIXED_VOTERS[clusterID % 3] in the mixed-membership configs


def partition_of(cluster_id: int, n_partitions: int) -> int:
    """FixedPartitioner.GetPartitionID (partition.go:38)."""
    return cluster_id % n_partitions


@dataclass(frozen=True)
class ShardRange:
    """Arithmetic progression of clusterIDs: cid(j) = cid_base + j * cid_stride, j < count."""

    cid_base: int
    cid_stride: int
    count: int

    def cids(self):
        return range(self.cid_base, self.cid_base + self.count * self.cid_stride, self.cid_stride)


def rank_shard(rank: int, world: int, groups_per_rank: int) -> ShardRange:
    """The clusterIDs GPU ``rank`` owns: every cid >= 1 with cid % world == rank, in order.

    cid 0 is NoNode (raft.go:48); the first owned cid of rank r is ``world + r`` when r == 0
    would otherwise hit 0, so we start every rank at ``world + r``. For world == 1 this is
    cid = j + 1, the single-GPU numbering.
    """
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    base = world + rank if world > 1 else 1
    return ShardRange(base, world, groups_per_rank)


def rank_bucket(rank: int, world: int, bucket: int, groups: int) -> ShardRange:
    """Groups of GPU ``rank`` whose voter count is MIXED_VOTERS[bucket] (cid % 3 == bucket).

    For world in {1, 2, 4, 8}, gcd(3, world) == 1, so the cids with cid % world == rank and
    cid % 3 == bucket form one progression of stride 3 * world (CRT).
    """
    if not 0 <= bucket < 3:
        raise ValueError("bucket out of range")
    if world % 3 == 0:
        raise ValueError("world size must be coprime to 3 for voter-count buckets")
    stride = 3 * world
    for c in range(1, stride + 1):
        if c % world == rank and c % 3 == bucket:
            return ShardRange(c, stride, groups)
    raise AssertionError("unreachable")


def interleave_bitmaps(rank_bitmaps, groups_per_rank: int):
    """The node's bitmap in clusterID order from the per-GPU bitmaps of ``rank_shard``.

    Rank r's bit j is clusterID ``world + r + j * world`` (rank_shard, world > 1), i.e. node
    position ``j * world + r`` of the clusterIDs world .. world * (G + 1) - 1; for world == 1 the
    rank's bitmap is the node's. Used after the optional result gather: changed /
    confirmed bits of every GPU collected over xGMI for the host that applies them.
    """
    import numpy as np

    world = len(rank_bitmaps)
    G = groups_per_rank
    bits = np.stack([np.unpackbits(np.ascontiguousarray(b, np.uint64).view(np.uint8),
                                   bitorder="little")[:G] for b in rank_bitmaps])
    node = bits.T.reshape(-1)                       # position j * world + r
    pad = (-node.size) % 64
    node = np.concatenate([node, np.zeros(pad, np.uint8)])
    return np.packbits(node, bitorder="little").view(np.uint64)
