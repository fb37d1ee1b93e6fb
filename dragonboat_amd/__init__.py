"""dragonboat_amd — MI355X-native batched quorum engine for dragonboat's multi-group Raft leader.

The product is the C-ABI library ``dragonboat_amd/lib/libhipquorum.so`` (include/hipquorum.h):
hand-written gfx950 HIP kernels that decide commit index, ReadIndex confirmation, vote outcome and
CheckQuorum for millions of independent Raft groups per launch. ``hipquorum`` is its ctypes
binding; ``shard`` holds the clusterID -> GPU partition rule.
"""
__all__ = ["hipquorum", "shard"]
