#!/usr/bin/env python3
"""Quorum-decision throughput of the MI355X batched quorum engine (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2tl|c2t|c3mt|c4t|...] [--no-cpu]

A step is one pass of the hot path over one batch of synthetic groups resident in HBM: for the
headline workload (BASELINE configs[1], "c2tl") one hq_commit_dev launch over 1,048,576 groups x 3
voters in the term-start form, read from 128-group tiles that carry the leader's match as its
lastIndex (HQ_LAYOUT_TILES_LEADER, raft.go:918; 48 B per decision). Inputs are generated on the device from splitmix64 seeds and rotate
over >= 1.1 GiB of distinct batches so that the 256 MiB Infinity Cache cannot serve them.

N > 1: one process per GPU (torch.distributed.run), groups sharded clusterID % N
(internal/server/partition.go:38), weak scaling (fixed groups per GPU), no data-path collective;
the barrier and the max-over-ranks time use torch.distributed.

Rank 0 prints ONE JSON line. `roofline.achieved` = algorithmic bytes per launch / average kernel
duration measured with HIP events on the launching stream over the timed region;
`cpu_baseline` = the C restatement (oracle/qref.c, test infrastructure) timed on this host.
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# The HIP runtime copies a large pageable host buffer by pinning its pages in place (a userptr
# mapping of the caller's memory). When those pages' mappings later change — the allocator
# handing them back after the oracle's replay churned GBs of host memory — the driver evicts and
# restores the process's queues, and a device step queued meanwhile starts 5-24 ms late: in the
# step legs 2 of 2 runs with the runtime's default, 0 of 2 with large copies staged through its
# own pinned buffers (no slower), 0 of 6 without the replay (profiles/r06l/). Staged here, before
# the runtime starts (a host app: pass pinned memory for large transfers, or set the same
# variable).
os.environ.setdefault("GPU_PINNED_MIN_XFER_SIZE", "1000000")

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md "Chip-level parameters")
HBM_MEASURED_COPY_GBS = 6290.0  # measured float4 copy ceiling (same table)
ROTATE_BYTES = int(1.1 * (1 << 30))
SEED_BASE = 0x5EED0000

WORKLOADS = {
    "c2": dict(cfg=1, kind="commit", G=1 << 20, n=3, form=0, mixed=False,
               desc="1M groups x 3 voters, batched commit-index kernel (term-start form)"),
    "c2t": dict(cfg=1, kind="commit", G=1 << 20, n=3, form=0, mixed=False, tiled=True,
                desc="1M groups x 3 voters, batched commit-index kernel (term-start form) over "
                     "128-group tiles (HQ_LAYOUT_TILES: one contiguous stream per wave)"),
    "c2tl": dict(cfg=1, kind="commit", G=1 << 20, n=3, form=0, mixed=False, tiled=True, lead=True,
                 desc="1M groups x 3 voters, batched commit-index kernel (term-start form) over "
                      "128-group tiles without the leader's match row (HQ_LAYOUT_TILES_LEADER: "
                      "slot 0 = lastIndex, raft.go:918; 48 B per decision)"),
    "c3mtl": dict(cfg=2, kind="commit", G=1 << 20, n=5, form=2, mixed=False, tiled=True,
                  lead=True,
                  desc="BASELINE config 3: 1M groups x 5 voting members (4 full incl. the leader "
                       "+ 1 witness; the 2 observers are never packed, raft.go:894-901), commit "
                       "+ current-term check (16-bit term mask over the last 16 indexes, exact "
                       "twin of the term-ring gather), 128-group tiles without the leader's match "
                       "row (slot 0 = lastIndex, raft.go:918; 58 B per decision)"),
    "c5v5tl": dict(cfg=2, kind="commit", G=8 << 20, n=5, form=2, mixed=False, tiled=True,
                   lead=True, desc="as c5v5t without the leader's match row "
                                   "(HQ_LAYOUT_TILES_LEADER)"),
    "c5tl": dict(cfg=4, kind="commit", G=8 << 20, n=5, form=2, mixed=True, tiled=True, lead=True,
                 desc="as c5t without the leader's match row (HQ_LAYOUT_TILES_LEADER)"),
    "c3mt": dict(cfg=2, kind="commit", G=1 << 20, n=5, form=2, mixed=False, tiled=True,
                 desc="1M groups x 5 voters (4 full + 1 witness), current-term mask, "
                      "128-group tiles"),
    "c3r32t": dict(cfg=2, kind="commit", G=1 << 20, n=5, form=3, mixed=False, tiled=True,
                   desc="1M groups x 5 voters (4 full + 1 witness), u32 term-ring gather, "
                        "128-group tiles"),
    "c5t": dict(cfg=4, kind="commit", G=8 << 20, n=5, form=2, mixed=True, tiled=True,
                desc="as c5 over 128-group tiles (the three buckets in one fused launch)"),
    "c5v5t": dict(cfg=2, kind="commit", G=8 << 20, n=5, form=2, mixed=False, tiled=True,
                  desc="8M groups x 5 voters (4 full + 1 witness) per GPU, the per-GPU share of "
                       "64M 5-voter groups on 8 GPUs: current-term mask, 128-group tiles"),
    "c5v5r32t": dict(cfg=2, kind="commit", G=8 << 20, n=5, form=3, mixed=False, tiled=True,
                     desc="8M groups x 5 voters (4 full + 1 witness) per GPU, u32 term-ring "
                          "gather, 128-group tiles"),
    "c3": dict(cfg=2, kind="commit", G=1 << 20, n=5, form=1, mixed=False,
               desc="1M groups x 5 voters (4 full + 1 witness; observers never packed), "
                    "commit + term-ring gather R=16"),
    "c3r32": dict(cfg=2, kind="commit", G=1 << 20, n=5, form=3, mixed=False,
                  desc="1M groups x 5 voters (4 full + 1 witness), commit + term-ring gather "
                       "from a u32 ring (R = 16; two groups per gathered 128-B line)"),
    "c3m": dict(cfg=2, kind="commit", G=1 << 20, n=5, form=2, mixed=False,
                desc="1M groups x 5 voters (4 full + 1 witness), commit + 16-bit current-term "
                     "mask (exact replacement of the ring gather)"),
    "c2l": dict(cfg=1, kind="lag", G=1 << 20, n=3, form=0, mixed=False,
                desc="1M groups x 3 voters, commit over int32 lags below lastIndex (term-start "
                     "form; 24 B per decision against 56 B)"),
    "c3l": dict(cfg=2, kind="lag", G=1 << 20, n=5, form=2, mixed=False,
                desc="1M groups x 5 voters (4 full + 1 witness), commit over int32 lags with the "
                     "lag-indexed current-term mask (30 B per decision)"),
    "c2ll": dict(cfg=1, kind="lag", G=1 << 20, n=3, form=0, mixed=False, lead=True,
                 desc="as c2l without the leader's lag row (HQ_LAG_LEADER_IMPLICIT: slot 0 = "
                      "lastIndex, raft.go:918; 20 B per decision)"),
    "c5ll": dict(cfg=4, kind="lag", G=8 << 20, n=5, form=2, mixed=True, lead=True,
                 desc="as c5l without the leader's lag row (HQ_LAG_LEADER_IMPLICIT)"),
    "c5l": dict(cfg=4, kind="lag", G=8 << 20, n=5, form=2, mixed=True,
                desc="as c5 in the int32 lag layout (lag-indexed mask), the three buckets in one "
                     "fused launch"),
    "c4": dict(cfg=3, kind="bits", G=16 << 20, n=7,
               desc="16M groups x 7 voters, fused ReadIndex ack quorum + vote tally"),
    "c4u": dict(cfg=3, kind="bits", G=16 << 20, n=7, uniform=True,
                desc="as c4 with the voter count uniform over the batch (a step worker's "
                     "7-voter bucket): no per-group n column"),
    "c4t": dict(cfg=3, kind="bits", G=16 << 20, n=7, tiled=True,
                desc="as c4 over 1024-group bitmap tiles (rows n, ack, granted, rejected: one "
                     "contiguous stream per wave)"),
    "c4ut": dict(cfg=3, kind="bits", G=16 << 20, n=7, uniform=True, tiled=True,
                 desc="as c4u over 1024-group bitmap tiles (rows ack, granted, rejected)"),
    "c4t3": dict(cfg=3, kind="bits", G=16 << 20, n=7, tiled3=True,
                 desc="as c4t over 3-byte tiles: the leader's own slot implicit (never acks its "
                      "ctx, always grants its vote), 7 bits per bitmap + 3 bits of n - 1 "
                      "(3.375 B per group instead of 4.375)"),
    "c4p": dict(cfg=3, kind="bits", G=16 << 20, n=7, planes=True,
                desc="as c4t3 over bit-plane tiles (the 3-byte tiles' bits transposed, 2048 "
                     "groups per tile): 32 groups per lane decided with bitwise adders "
                     "(3.375 B per group)"),
    "c5": dict(cfg=4, kind="commit", G=8 << 20, n=5, form=2, mixed=True,
               desc="64M groups mixed 3/5/7 voters (n = {3,5,7}[clusterID % 3]) sharded "
                    "clusterID % 8: 8M groups per GPU, the three voter-count buckets in one "
                    "fused launch, current-term mask"),
    "c5r": dict(cfg=4, kind="commit", G=8 << 20, n=5, form=1, mixed=True,
                desc="as c5 with the u64 term-ring gather (R = 16)"),
    "c5r32": dict(cfg=4, kind="commit", G=8 << 20, n=5, form=3, mixed=True,
                  desc="as c5 with the u32 term-ring gather (R = 16)"),
    "c5s": dict(cfg=4, kind="commit", G=8 << 20, n=5, form=2, mixed=True, separate=True,
                desc="as c5 with one launch per voter-count bucket (3 launches per step)"),
}


# BASELINE.json configs[2] (1M x 5 voters + witness/observers, commit + term check): the largest
# single-GPU commit config and the north star's 5-voter bar
HEADLINE = "c3mtl"
DEFAULT_EXTRAS = ("c2tl,c2t,c2,c2l,c3,c3r32,c3r32t,c3m,c3mt,c3l,c5v5t,c5v5tl,c5v5r32t,"
                  "c4,c4t,c4t3,c4p,c4u,c4ut,c5,c5t,c5tl,c5s,c5l,c2ll,c5ll,c5r,c5r32,rim,"
                  "rimt,rimtc,cq,cqp,c4pq,ing,ingo,ingu,inga,w2,sweep,e2e,step,step5,wire,wire_step")
# the same generated groups decided with the other exact term-check forms (same cfg, n, G)
SAME_DATA_FORMS = {"c3mtl": ("c3", "c3r32", "c3r32t", "c3m", "c3mt"),
                   "c3mt": ("c3", "c3r32", "c3r32t", "c3m", "c3mtl")}


def algo_bytes_per_group(w):
    """bytes the decision must move per group."""
    if w["kind"] == "lag":
        # lag rows + cin_lag + cout_lag + (ts_lag | lag_mask)
        # (HQ_LAG_LEADER_IMPLICIT: no row for the leader's lag, always 0)
        return 4 * (w["n"] - 1 if w.get("lead") else w["n"]) + 8 + {0: 4, 2: 2}[w["form"]]
    if w["kind"] == "commit":
        n, extra_n = w["n"], (1 if w["mixed"] else 0)
        # match + committed in/out + last + (term_start | term + gathered ring term | u16 mask
        # | term + gathered u32 ring term)
        # (the leader-row tile layout carries slot 0 as last_index: 8 bytes less)
        return (8 * (n - 1 if w.get("lead") else n) + 24 + {0: 8, 1: 16, 2: 2, 3: 12}[w["form"]]
                + extra_n)
    # ack, granted, rejected (+ n unless uniform or packed into the 3-byte tiles) u8 each in;
    # confirmed bit + 2-bit outcome out
    return (3 if w.get("uniform") or w.get("tiled3") or w.get("planes") else 4) + 3 / 8


def decisions_per_group(w):
    return 2 if w["kind"] == "bits" else 1


def log(msg):
    print(msg, file=sys.stderr, flush=True)


class Dist:
    """Rank bookkeeping; torch.distributed only when launched with WORLD_SIZE > 1."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.torch = None
        self.device = self.local_rank
        self.backend = None
        if self.world > 1:
            import torch
            import torch.distributed as dist

            self.torch, self.dist = torch, dist
            ngpu = torch.cuda.device_count() if torch.cuda.is_available() else 0
            if ngpu >= self.world:
                self.device = self.local_rank
                torch.cuda.set_device(self.device)
                backend = "nccl"   # RCCL on ROCm: barrier + MAX/SUM all-reduce only
            else:
                # more ranks than GPUs (rehearsal on a small box): ranks share GPUs and the
                # timing collectives run on the host
                self.device = self.local_rank % max(1, ngpu)
                backend = "gloo"
            dist.init_process_group(backend=backend)
            self.backend = backend

    def barrier(self):
        if self.torch is not None:
            self.dist.barrier()

    def sync_device(self):
        if self.torch is not None and self.torch.cuda.is_available():
            self.torch.cuda.synchronize()

    def max(self, x: float) -> float:
        if self.torch is None:
            return x
        dev = "cuda" if self.backend == "nccl" else "cpu"
        t = self.torch.tensor([x], dtype=self.torch.float64, device=dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def gather(self, xs) -> list:
        """Every rank's list of floats, in rank order (all_gather; RCCL when each rank has its
        own GPU)."""
        if self.torch is None:
            return [list(xs)]
        dev = "cuda" if self.backend == "nccl" else "cpu"
        t = self.torch.tensor(list(xs), dtype=self.torch.float64, device=dev)
        out = [self.torch.zeros_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [o.cpu().tolist() for o in out]

    def gather_words(self, ctx, dev_words, nwords: int):
        """All ranks' device uint64 words (an hq DeviceArray) on every rank, rank-major: one
        all_gather over RCCL (xGMI) when each rank has its own GPU, over gloo from host copies
        otherwise. Returns (numpy [world, nwords], seconds spent in the collective)."""
        torch = self.torch
        if self.backend == "nccl":
            t = torch.empty(nwords, dtype=torch.int64, device=f"cuda:{self.device}")
            ctx.copy_to_ptr(t.data_ptr(), dev_words, nwords * 8)   # device to device
            ctx.sync()
            out = torch.empty(self.world * nwords, dtype=torch.int64, device=t.device)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            self.dist.all_gather_into_tensor(out, t)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            return out.view(self.world, nwords).cpu().numpy().view(np.uint64), dt
        t = torch.from_numpy(ctx.download(dev_words).view(np.int64).copy())
        outs = [torch.zeros_like(t) for _ in range(self.world)]
        t0 = time.perf_counter()
        self.dist.all_gather(outs, t)
        dt = time.perf_counter() - t0
        return np.stack([o.numpy() for o in outs]).view(np.uint64), dt

    def sum(self, x: float) -> float:
        if self.torch is None:
            return x
        dev = "cuda" if self.backend == "nccl" else "cpu"
        t = self.torch.tensor([x], dtype=self.torch.float64, device=dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def gather_obj(self, o) -> list:
        """Every rank's picklable object, in rank order (off the timed region)."""
        if self.torch is None:
            return [o]
        out = [None] * self.world
        self.dist.all_gather_object(out, o)
        return out

    def close(self):
        if self.torch is not None:
            self.dist.destroy_process_group()


class ThreadGroup:
    """State shared by the host threads of one launcher-free multi-GPU run."""

    def __init__(self, n: int):
        self.n = n
        self.bar = threading.Barrier(n, timeout=1800)
        self.slots = [None] * n


class ThreadDist:
    """`python bench.py --gpus N` without a launcher: one process, one host thread and one hq_ctx
    (one HIP stream) per GPU, the way SURVEY.md §8e and the reference's step workers run
    (execengine.go:675-690: one goroutine per worker, groups on worker clusterID % N,
    partition.go:38). Same interface as Dist; the barrier and the max / sum over ranks are host
    thread barriers, taken only at the start and end of a timed region. A GPU index beyond the
    visible devices wraps (rehearsal of N ranks on fewer GPUs)."""

    def __init__(self, group: ThreadGroup, rank: int, ngpu: int):
        self.g = group
        self.world, self.rank, self.local_rank = group.n, rank, rank
        self.device = rank % max(1, ngpu)
        self.backend = "threads"
        self.torch = None

    def barrier(self):
        self.g.bar.wait()

    def sync_device(self):
        pass          # every leg syncs its own contexts before the barrier

    def _all(self, x) -> list:
        self.g.slots[self.rank] = x
        self.g.bar.wait()
        vals = list(self.g.slots)
        self.g.bar.wait()             # nobody overwrites a slot before all have read it
        return vals

    def max(self, x: float) -> float:
        return max(self._all(x))

    def sum(self, x: float) -> float:
        return float(sum(self._all(x)))

    def gather(self, xs) -> list:
        return [list(v) for v in self._all(list(xs))]

    def gather_obj(self, o) -> list:
        return self._all(o)

    def gather_words(self, ctx, dev_words, nwords: int):
        t0 = time.perf_counter()
        words = self._all(ctx.download(dev_words)[:nwords].copy())
        return np.stack(words).view(np.uint64), time.perf_counter() - t0

    def close(self):
        pass


# ----------------------------------------------------------------------------- GPU legs -------
def build_sets(ctx, hq, shard, w, d: "Dist"):
    """Device-generated input batches for this rank, enough to rotate over ROTATE_BYTES.
    Commit workloads: each set is a list of CommitBuffers launched back to back in one step
    (one per voter-count bucket for the mixed-membership workload)."""
    G = w["G"]
    per_set = algo_bytes_per_step(w)
    nsets = max(4, int(np.ceil(ROTATE_BYTES / per_set)))
    seed = SEED_BASE + w["cfg"]
    sets = []
    for s in range(nsets):
        if w["kind"] == "commit":
            buckets = []
            for n, rng in commit_buckets(shard, w, d):
                spec = hq.synth_spec(seed + (s << 40), rng.count, n, cid_base=rng.cid_base,
                                     cid_stride=rng.cid_stride)
                lay = hq.HQ_LAYOUT_TILES_LEADER if w.get("lead") else hq.HQ_LAYOUT_TILES
                b = hq.alloc_commit(ctx, rng.count, n, w["form"], 16,
                                    tiled=w.get("tiled", False), tile_layout=lay)
                ctx.synth_commit_dev(spec, b.args())
                if b.tiles is not None:
                    ctx.tile_commit_dev(b.args(), b.tiles, lay)
                buckets.append(b)
            sets.append(buckets)
        elif w["kind"] == "lag":
            buckets = []
            for n, rng in commit_buckets(shard, w, d):
                spec = hq.synth_spec(seed + (s << 40), rng.count, n, cid_base=rng.cid_base,
                                     cid_stride=rng.cid_stride)
                b = hq.alloc_commit_lag(ctx, rng.count, n, w["form"], 16)
                ctx.synth_commit_lag_dev(spec, b.args())
                buckets.append(b)
            sets.append(buckets)
        else:
            rng = shard.rank_shard(d.rank, d.world, G)
            spec = hq.synth_spec(seed + (s << 40), G, w["n"], cid_base=rng.cid_base,
                                 cid_stride=rng.cid_stride)
            arrs = [ctx.empty(G, np.uint8) for _ in range(4)]
            ctx.synth_bitmaps_dev(spec, *arrs)
            conf = ctx.empty(hq.words64(G), np.uint64)
            outc = ctx.empty(hq.words32(G), np.uint64)
            tiles = None
            if w.get("planes"):
                tiles = ctx.empty(hq.plane_tiles(G) * 3 * hq.HQ_PLANE_TILE_GROUPS, np.uint8)
                ctx.tile_planes_dev(G, *arrs, 0, tiles)
                ctx.sync()
                for a in arrs:
                    ctx.free(a)
                arrs = None
            elif w.get("tiled3"):
                tiles = ctx.empty(hq.bits_tiles(G) * 3 * hq.HQ_BITS_TILE_GROUPS, np.uint8)
                ctx.tile_bits3_dev(G, *arrs, 0, tiles)
                ctx.sync()
                for a in arrs:
                    ctx.free(a)
                arrs = None
            elif w.get("tiled"):
                pern = not w.get("uniform")
                tiles = ctx.empty(hq.bits_tile_bytes(G, pern), np.uint8)
                ctx.tile_bits_dev(G, *arrs[:3], arrs[3] if pern else None, tiles)
                ctx.sync()
                for a in arrs:
                    ctx.free(a)
                arrs = None
            sets.append((arrs, conf, outc, tiles))
    ctx.sync()
    return sets, per_set


def batch_args(b):
    """The launch arguments of one commit batch: its tiles when it has them."""
    return b.tile_args() if b.tiles is not None else b.args()


def commit_buckets(shard, w, d):
    """(voters, clusterID progression) per launch of one step on this rank."""
    if not w["mixed"]:
        return [(w["n"], shard.rank_shard(d.rank, d.world, w["G"]))]
    per = w["G"] // 3
    return [(shard.MIXED_VOTERS[b], shard.rank_bucket(d.rank, d.world, b, per)) for b in range(3)]


def algo_bytes_per_step(w):
    if w["kind"] in ("commit", "lag") and w["mixed"]:
        per = w["G"] // 3
        return sum(per * algo_bytes_per_group(dict(w, n=n, mixed=False)) for n in (3, 5, 7))
    return algo_bytes_per_group(w) * w["G"]


def groups_per_step(w):
    return (w["G"] // 3) * 3 if w["kind"] in ("commit", "lag") and w["mixed"] else w["G"]


def run_gpu(w, steps, warmup, d: Dist):
    from dragonboat_amd import hipquorum as hq
    from dragonboat_amd import shard

    ctx = hq.Context(d.device)
    sets, per_set = build_sets(ctx, hq, shard, w, d)
    G = w["G"]
    nsets = len(sets)
    # Warm-up decides sets 0 .. W-1; the timed steps continue the rotation at set W, so no timed
    # launch re-reads a batch touched less than (nsets - 1) batches (>= 1.1 GiB) earlier: the
    # 256 MiB Infinity Cache cannot hold it (MI355X_MICROARCH.md "Infinity Cache").
    first = max(1, warmup) % nsets
    launches_per_step = 1
    if w["kind"] == "commit" and w["mixed"] and not w.get("separate"):
        # a step = the rank's voter-count buckets decided by one fused launch
        per_step = [hq.commit_batch_array([batch_args(b) for b in bs]) for bs in sets]

        def run(idx):
            for i in idx:
                ctx.commit_fused_dev(per_step[i % nsets])
    elif w["kind"] == "lag":
        # one launch per step: the bucket set's batches fused (a single batch: plain launch)
        per_step = [hq.lag_batch_array([b.args(bool(w.get("lead"))) for b in bs]) for bs in sets]

        def run(idx):
            for i in idx:
                arr = per_step[i % nsets]
                if len(arr) == 1:
                    ctx.commit_lag_dev(arr[0])
                else:
                    ctx.commit_lag_fused_dev(arr)
    elif w["kind"] == "commit":
        # every launch of the sequence enqueued by one C call (hq_commit_many_dev)
        launches_per_step = len(sets[0])
        cache = {}

        def prepare(idx):   # the argument array of a sequence, built outside the timed region
            cache[(idx.start, idx.stop)] = hq.commit_batch_array(
                [batch_args(b) for i in idx for b in sets[i % nsets]])

        def run(idx):
            ctx.commit_many_dev(cache[(idx.start, idx.stop)])
    else:
        def run(idx):
            for i in idx:
                arrs, conf, outc, tiles = sets[i % nsets]
                if w.get("planes"):
                    ctx.readindex_vote_planes_dev(G, tiles, conf, outc)
                    continue
                if w.get("tiled3"):
                    ctx.readindex_vote_tiles3_dev(G, tiles, conf, outc)
                    continue
                if tiles is not None:
                    uni = w.get("uniform", False)
                    ctx.readindex_vote_tiles_dev(G, tiles, not uni, w["n"] if uni else 0, conf,
                                                 outc)
                    continue
                da, dg, dr, dn = arrs
                if w.get("uniform"):
                    ctx.readindex_vote_dev(G, da, dg, dr, None, w["n"], conf, outc)
                else:
                    ctx.readindex_vote_dev(G, da, dg, dr, dn, 0, conf, outc)

    wseq, seq = range(0, max(1, warmup)), range(first, first + steps)
    if w["kind"] == "commit" and not (w["mixed"] and not w.get("separate")):
        prepare(wseq)
        prepare(seq)
        prepare(range(0, 1))
    if warmup > 0:
        run(wseq)
    ctx.sync()
    d.sync_device()
    d.barrier()
    ctx.timing_reset()
    # The HIP-event region opens behind the first timed launch (in stream order: when it ends,
    # with the second one already queued) and closes right behind the last one, so it holds
    # back-to-back kernels only: no host launch latency at its start, no host sync at its end.
    ctx.timing_begin_after(1 if steps * launches_per_step > 1 else 0)
    t0 = time.perf_counter()
    run(seq)
    ctx.timing(False)
    ctx.sync()
    d.sync_device()
    d.barrier()
    t1 = time.perf_counter()
    kernel_ms, launches = ctx.timing_read()
    local = t1 - t0
    elapsed = d.max(local)
    avg_kernel_s = kernel_ms / 1e3 / max(1, launches)
    bytes_per_launch = per_set / launches_per_step
    achieved_local = bytes_per_launch / avg_kernel_s / 1e9 if launches else 0.0
    # per-GPU numbers (SURVEY.md §8e reporting), gathered off the timed region
    try:
        per_gpu = d.gather([groups_per_step(w) * steps * decisions_per_group(w) / local,
                            avg_kernel_s * 1e6, achieved_local])
    except Exception as e:  # a diagnostic must never cost the benchmark line
        log(f"per-GPU gather failed: {e!r}")
        per_gpu = [[groups_per_step(w) * steps * decisions_per_group(w) / local,
                    avg_kernel_s * 1e6, achieved_local]]
    # node-level roofline: every GPU's achieved bytes/s over N x the peak
    achieved_node = d.sum(achieved_local)
    # The decisions of set 0, taken once more after the timed region, for the full-size parity
    # check of the cpu_baseline leg (every bucket of the step; outputs only, no timing).
    set0 = None
    if w["kind"] in ("commit", "lag"):
        if w["kind"] == "commit" and w["mixed"] and not w.get("separate"):
            ctx.commit_fused_dev(per_step[0])
        else:
            run(range(0, 1))
        ctx.sync()
        set0 = []
        for (n, rng), b in zip(commit_buckets(shard, w, d), sets[0]):
            outs = (b.cout_lag if w["kind"] == "lag" else b.committed_out, b.changed,
                    b.fallback)
            set0.append(dict(n=n, cid_base=rng.cid_base, cid_stride=rng.cid_stride,
                             count=rng.count, out=[ctx.download(a) for a in outs]))
    gather = None
    if d.world > 1 and w["kind"] == "commit" and not w["mixed"]:
        # optional result gather: every GPU's changed bits of batch 0 to every
        # rank, in clusterID order; off the timed region
        try:
            nw = hq.words64(G)
            words, dt = d.gather_words(ctx, sets[0][0].changed, nw)
            node = shard.interleave_bitmaps(list(words), G)
            gather = {"bytes": int(words.nbytes), "ms": dt * 1e3, "backend": d.backend,
                      "node_changed": int(np.unpackbits(node.view(np.uint8)).sum())}
        except Exception as e:   # optional: report, never abort the bench
            log(f"result gather failed: {e!r}")
            gather = {"error": repr(e)}
    total_groups = d.sum(float(groups_per_step(w) * steps))
    res = dict(
        elapsed=elapsed, launches=launches, avg_kernel_s=avg_kernel_s,
        decisions=total_groups * decisions_per_group(w), nsets=nsets, first_timed_set=first,
        bytes_per_launch=bytes_per_launch, launches_per_step=launches_per_step, steps=steps,
        achieved_gbs=achieved_local, achieved_node_gbs=achieved_node,
        per_gpu=per_gpu, set0=set0, gather=gather,
    )
    ctx.close()
    return res


def engine_ok(w):
    """The persistent commit engine serves uniform-n tiled batches in the term-start / mask form."""
    return (w["kind"] == "commit" and not w["mixed"] and w.get("tiled")
            and w["form"] in (0, 2))


def fused_chunks(steps):
    """The window's batches split into hq_commit_fused_dev launches of at most 32 (the kernel's
    batch limit), as even as possible: (first, count) per launch."""
    n = max(1, -(-steps // 32))
    bounds = [steps * i // n for i in range(n + 1)]
    return [(bounds[i], bounds[i + 1] - bounds[i]) for i in range(n)]


def run_engine(w, steps, warmup, d: Dist, windows=3, headline="fused", share=1):
    """A commit workload stepped through the persistent commit engine (hq_engine_*,
    dragonboat_amd/csrc/hq_engine.hip): per timed window the K steps are posted one hq_engine_post call each
    (post-as-ready, the reference's step-worker shape) and decided by ONE resident launch (no
    dependent-launch boundary between steps) that the drain's STOP ends. Beside each engine window, the same K batches as K back-to-back
    launches (hq_commit_many_dev), so the line carries both on the same data. `windows` windows
    of K = `steps` steps each continue the rotation (>= 1.1 GiB of distinct batches: no step
    re-reads a batch the 256 MiB Infinity Cache could still hold); the median window is reported
    (the median over repeated timings).

    headline "fused": the line's value and roofline are the window's batches decided by fused
    launches (hq_commit_fused_dev, up to 32 batches each). Each batch is one step worker's step of
    1 M groups (the groups are disjoint between batches), so one launch decides the co-resident
    workers' batches of a step (16 step workers in the reference, internal/settings/hard.go:35,
    execengine.go:675-690). headline "engine": the resident engine's windows. share: the ranks
    on this GPU; above 1 each engine is capped at its share of the full grid (max_workgroups), so
    that the co-located engines are all resident."""
    from dragonboat_amd import hipquorum as hq
    from dragonboat_amd import shard

    ctx = hq.Context(d.device)
    sets, per_set = build_sets(ctx, hq, shard, w, d)
    nsets = len(sets)
    lay = hq.HQ_LAYOUT_TILES_LEADER if w.get("lead") else hq.HQ_LAYOUT_TILES
    mw = 0
    if share > 1:
        e0 = hq.Engine(ctx, w["n"], w["form"], lay, ring_len=16)
        mw = max(1, e0.info().grid // share)
        e0.close()
    eng = hq.Engine(ctx, w["n"], w["form"], lay, ring_len=16, max_workgroups=mw)
    # the same engine with per-step completion flags (what a step worker that applies each step's
    # commits as soon as they are decided runs): its windows are reported beside the others
    eng_sig = hq.Engine(ctx, w["n"], w["form"], lay, ring_len=16, signal=True, max_workgroups=mw)

    def arr(i0, k):
        return hq.commit_batch_array([batch_args(sets[(i0 + i) % nsets][0]) for i in range(k)])

    W = max(1, warmup)
    eng.run(arr(0, W))
    eng_sig.post(arr(0, W))
    eng_sig.drain()
    eng_sig.timing(reset=True)
    ctx.commit_many_dev(arr(0, min(W, nsets)))
    ctx.sync()
    eng.timing(reset=True)
    first = W % nsets
    wins = []
    for k in range(windows):
        a = arr(first + k * steps, steps)
        a1 = [arr(first + k * steps + i, 1) for i in range(steps)]
        fa = [arr(first + k * steps + c0, cn) for c0, cn in fused_chunks(steps)]
        rec = {}
        for mode in ("engine", "launches", "signal", "fused"):
            ctx.sync()
            d.sync_device()
            d.barrier()
            if mode == "launches":
                ctx.timing_reset()
                ctx.timing_begin_after(1 if steps > 1 else 0)
            elif mode == "fused":
                ctx.timing_reset()
                ctx.timing(True)
            t0 = time.perf_counter()
            if mode == "engine":
                # post-as-ready: one hq_engine_post per step, as each step worker posts its own
                # step when it is ready (execengine.go:860-882); the first post launches the
                # grid, the later ones reach it through the ring; the drain's STOP ends it
                for one in a1:
                    eng.post(one)
                eng.drain()
            elif mode == "signal":
                q0 = eng_sig.post(a)
                eng_sig.wait(q0 + steps - 1)       # the last step's flag: every step decided
                sig_local = time.perf_counter() - t0
                # (each step's flag is written by its own last arriving workgroup: an earlier
                # step's may land just after a later one's, so every flag is awaited before its
                # clock is read; the engine keeps the clocks of its last `depth` steps)
                for i in range(steps):
                    eng_sig.wait(q0 + i)
                nclk = min(steps, eng_sig.info().depth)
                clocks = [eng_sig.done_clock(q0 + i) for i in range(steps - nclk, steps)]
                eng_sig.drain()
            elif mode == "fused":
                for x in fa:
                    ctx.commit_fused_dev(x)
                ctx.timing(False)
                ctx.sync()
            else:
                ctx.commit_many_dev(a)
                ctx.timing(False)
                ctx.sync()
            local = time.perf_counter() - t0
            d.barrier()
            if mode == "engine":
                nl, ms = eng.timing(reset=True)
                kernel_s = ms / 1e3 / max(1, steps)        # resident launch time per step
            elif mode == "signal":
                nl, ms = eng_sig.timing(reset=True)
                local = sig_local
                # device clock (100 MHz) between the first and the last step's completion
                kernel_s = (clocks[-1] - clocks[0]) / 1e8 / max(1, len(clocks) - 1)
            elif mode == "fused":
                ms, nl = ctx.timing_read()
                kernel_s = ms / 1e3 / max(1, steps)        # one launch for the window's steps
            else:
                ms, nl = ctx.timing_read()
                kernel_s = ms / 1e3 / max(1, nl)           # back-to-back launch time
            rec[mode] = {"elapsed": d.max(local), "local": local, "kernel_s": kernel_s,
                         "launches": nl}
        wins.append(rec)

    def med(mode, key):
        return float(np.median([x[mode][key] for x in wins]))

    # set 0 once more through the engine, its outputs poisoned first: the full-size parity check
    # of the cpu_baseline leg reads what the engine wrote; the launch path's decisions of the
    # same batch must be identical
    b0 = sets[0][0]
    for x in (b0.committed_out, b0.changed, b0.fallback):
        ctx.memset(x, 0xA5)
    ctx.sync()
    eng.post(arr(0, 1))
    eng.drain()
    outs = [ctx.download(x) for x in (b0.committed_out, b0.changed, b0.fallback)]
    info = eng.info()
    ctx.commit_dev(batch_args(b0))
    ctx.sync()
    launch_outs = [ctx.download(x) for x in (b0.committed_out, b0.changed, b0.fallback)]
    rng = commit_buckets(shard, w, d)[0][1]
    set0 = [dict(n=w["n"], cid_base=rng.cid_base, cid_stride=rng.cid_stride, count=rng.count,
                 out=outs)]
    engine_eq_launch = all(np.array_equal(x, y) for x, y in zip(outs, launch_outs))
    # set 0 through a fused launch beside set 1, its outputs poisoned first
    for x in (b0.committed_out, b0.changed, b0.fallback):
        ctx.memset(x, 0xA5)
    ctx.commit_fused_dev(arr(0, 2))
    ctx.sync()
    fused_outs = [ctx.download(x) for x in (b0.committed_out, b0.changed, b0.fallback)]
    fused_eq_launch = all(np.array_equal(x, y) for x, y in zip(fused_outs, launch_outs))
    if headline == "fused":
        set0[0]["out"] = fused_outs
    eng.close()
    eng_sig.close()
    hm = "fused" if headline == "fused" else "engine"
    elapsed = med(hm, "elapsed")
    kernel_s = med(hm, "kernel_s")
    local = med(hm, "local")
    achieved_local = per_set / kernel_s / 1e9
    per_gpu = d.gather([groups_per_step(w) * steps / local, kernel_s * 1e6, achieved_local])
    achieved_node = d.sum(achieved_local)
    total_groups = d.sum(float(groups_per_step(w) * steps))
    lk = med("launches", "kernel_s")
    le = med("launches", "elapsed")
    res = dict(
        elapsed=elapsed, launches=steps, avg_kernel_s=kernel_s,
        decisions=total_groups * decisions_per_group(w), nsets=nsets, first_timed_set=first,
        bytes_per_launch=per_set, launches_per_step=1, steps=steps,
        achieved_gbs=achieved_local, achieved_node_gbs=achieved_node, per_gpu=per_gpu,
        set0=set0, gather=None, windows=len(wins), headline_mode=hm,
        engine={
            "mode": "persistent commit engine (hq_engine), post-as-ready: the window's "
                    f"{steps} steps ({groups_per_step(w)} groups each) posted one hq_engine_post "
                    "call per step as the step workers would; the first post launches the grid, "
                    "the others reach it through the pinned ring, and the drain's STOP ends it",
            "groups_per_step": groups_per_step(w), "steps_per_window": steps,
            "grid": info.grid, "block": info.block,
            "window_ms": [round(x["engine"]["elapsed"] * 1e3, 4) for x in wins],
            "window_kernel_us_per_step": [round(x["engine"]["kernel_s"] * 1e6, 3) for x in wins],
            "median_kernel_us_per_step": med("engine", "kernel_s") * 1e6,
            "median_ms_per_step": med("engine", "elapsed") / steps * 1e3,
            "value": total_groups * decisions_per_group(w) / med("engine", "elapsed"),
            "frac": d.sum(per_set / med("engine", "kernel_s") / 1e9) / (HBM_PEAK_GBS * d.world),
            "engine_equals_launch_set0": engine_eq_launch,
        },
        engine_signal={
            "mode": "the same engine with per-step completion flags (HQ_ENGINE_SIGNAL): the host "
                    "waits for the last step's flag",
            "window_ms": [round(x["signal"]["elapsed"] * 1e3, 4) for x in wins],
            "median_ms_per_step": med("signal", "elapsed") / steps * 1e3,
            "median_us_between_step_completions": med("signal", "kernel_s") * 1e6,
            "value": total_groups * decisions_per_group(w) / med("signal", "elapsed"),
        },
        fused_window={
            "mode": f"the window's {steps} batches in {len(fused_chunks(steps))} fused launch(es) "
                    "(hq_commit_fused_dev, one workgroup range per batch, <= 32 batches each)",
            "batches_per_launch": [cn for _, cn in fused_chunks(steps)],
            "groups_per_launch": [cn * groups_per_step(w) for _, cn in fused_chunks(steps)],
            "fused_equals_launch_set0": fused_eq_launch,
            "window_ms": [round(x["fused"]["elapsed"] * 1e3, 4) for x in wins],
            "median_ms_per_step": med("fused", "elapsed") / steps * 1e3,
            "median_kernel_us_per_step": med("fused", "kernel_s") * 1e6,
            "value": total_groups * decisions_per_group(w) / med("fused", "elapsed"),
            "frac": d.sum(per_set / med("fused", "kernel_s") / 1e9) / (HBM_PEAK_GBS * d.world),
        },
        launch_per_step={
            "mode": "the same batches as back-to-back launches (hq_commit_many_dev)",
            "groups_per_launch": groups_per_step(w),
            "window_ms": [round(x["launches"]["elapsed"] * 1e3, 4) for x in wins],
            "median_ms_per_step": le / steps * 1e3,
            "median_kernel_us": lk * 1e6,
            "value": total_groups * decisions_per_group(w) / le,
            "frac": d.sum(per_set / lk / 1e9) / (HBM_PEAK_GBS * d.world),
        },
    )
    ctx.close()
    return res


def run_size_sweep(name, steps, warmup, d: Dist, sizes=(1 << 18, 1 << 19, 1 << 20, 1 << 21,
                                                        1 << 22, 1 << 23)):
    """The headline kernel at batch sizes 256K..8M groups per GPU (same generator, same
    rotation past the Infinity Cache), and the least-squares line t(launch) = t0 + bytes / BW
    over them: BW is the kernel's streaming rate, t0 what one launch costs whatever its size (the
    dependent-launch boundary, fill and drain; MI355X_MICROARCH.md "boundary")."""
    w = WORKLOADS[name]
    pts = []
    for g in sizes:
        re_ = run_gpu(dict(w, G=g), steps, warmup, d)
        pts.append({"groups": g, "bytes_per_launch": re_["bytes_per_launch"],
                    "kernel_us": re_["avg_kernel_s"] * 1e6,
                    "frac": re_["achieved_node_gbs"] / (HBM_PEAK_GBS * d.world)})
    x = np.array([p["bytes_per_launch"] for p in pts], np.float64)
    y = np.array([p["kernel_us"] for p in pts], np.float64)
    slope, t0 = np.polyfit(x, y, 1)
    resid = y - (t0 + slope * x)
    return {"workload": f"sweep: {name} kernel vs batch size (t = t0 + bytes / BW)",
            "points": pts, "fit_t0_us": float(t0),
            "fit_stream_gbs": float(1e-3 / slope) if slope > 0 else None,
            "fit_stream_frac_of_peak": float(1e-3 / slope / HBM_PEAK_GBS) if slope > 0 else None,
            "fit_max_resid_us": float(np.abs(resid).max())}


def _timed(ctx, d, run, steps, warmup):
    """Warm up, then time `steps` calls of run(i) with a barrier + sync on both sides; returns
    (max-over-ranks seconds, average launch seconds from the HIP-event region)."""
    w0 = max(1, warmup)
    for i in range(w0):
        run(i)
    ctx.sync()
    d.sync_device()
    d.barrier()
    ctx.timing_reset()
    ctx.timing_begin_after(1 if steps > 1 else 0)   # as in run_gpu: back-to-back kernels only
    t0 = time.perf_counter()
    for i in range(w0, w0 + steps):    # the rotation continues past the warm-up's batches
        run(i)
    ctx.timing(False)
    ctx.sync()
    d.sync_device()
    d.barrier()
    t1 = time.perf_counter()
    ms, launches = ctx.timing_read()
    return d.max(t1 - t0), ms / 1e3 / max(1, launches), launches


def rim_inputs(rank: int, G: int = 2 << 20, K: int = 4, n: int = 7):
    """The multi-ctx ReadIndex legs' inputs (rim / rimt) of one rank: first-ack ordinals
    uint16 [K][n][G] (~70 % of (ctx, voter) pairs acked, arrival order 1..K*n, 0xFFFF = no ack)
    and the pending ctxs' indexes uint64 [K][G] (non-decreasing per group)."""
    r = np.random.default_rng(SEED_BASE + rank)
    ordn = r.integers(1, K * n + 1, (K, n, G)).astype(np.uint16)
    ordn[r.random((K, n, G)) < 0.3] = 0xFFFF
    idx = (np.uint64(1 << 30) + np.arange(K, dtype=np.uint64)[:, None] * np.uint64(3)
           + r.integers(0, 1 << 20, G, dtype=np.uint64)[None, :])
    return G, K, n, ordn, idx


def rim_parity(inputs, got, nthreads):
    """A multi-ctx ReadIndex batch's released indexes, counts and batch ends against the oracle
    (oracle/qref.c's message replay, readindex.go:77-116) on the same inputs, at full size."""
    from oracle import qref

    G, K, n, ordn, idx = inputs
    t0 = time.perf_counter()
    rel, cnt, fb, bend = qref.readindex_multi_batch(ordn.reshape(-1), idx.reshape(-1), None, None,
                                                    n, K, n, nthreads=nthreads)
    want = {"released_index": rel, "released_count": cnt, "batch_end": bend}
    eq = {k: bool(np.array_equal(got[k], want[k])) for k in want}
    return dict(groups=G, equal=all(eq.values()) and not fb.any(), oracle_fallback=int(fb.any()),
                check_s=time.perf_counter() - t0, **eq)


def c4pq_oracle(seed_votes, seed_active, G, n, nthreads):
    """The fused ReadIndex + vote + CheckQuorum pass's expected outputs: the oracle's readindex /
    vote / leaderHasQuorum batches (readindex.go:77-116, raft.go:1968-1985, raft.go:380-390) on the
    generator's bitmaps (the active flags: the ack bitmaps of another seed, as the leg packs
    them), the voter count of the vote bitmaps for all three."""
    from oracle import qref

    inp = qref.BitmapInputs(qref.spec(seed_votes, G, n))
    act = qref.BitmapInputs(qref.spec(seed_active, G, n)).ack
    conf = qref.readindex_batch(inp.ack, inp.n_voting, 0, nthreads=nthreads)[0]
    outc = qref.vote_batch(inp.granted, inp.rejected, inp.n_voting, 0, nthreads=nthreads)[0]
    hqb = qref.check_quorum_batch(act, inp.n_voting, 0, 0, nthreads=nthreads)[0]
    return {"confirmed": conf, "outcome": outc, "has_quorum": hqb}


def run_kernel_leg(name, steps, warmup, d: Dist, parity_threads=0):
    """The remaining decision kernels, each on its own BASELINE-shaped batch, device-resident and
    rotated past the Infinity Cache like the commit legs:
      rim: general multi-ctx ReadIndex (k_ri_multi), 2M groups x 4 pending ctxs x 7 voters
      cq:  CheckQuorum (k_bits CHECKQ), 16M groups x 7 voters, active flags reset in place
      cqp: the same over active-flag planes (k_cq_planes)
      c4pq: c4p's ReadIndex + vote planes and CheckQuorum's active planes in one launch
      ing: match-delta ingest, 4M ReplicateResp deltas in random order into a 4M x 3 table
           (binned: k_bin + k_apply)
      ingo: the same deltas in group order, the order a step worker emits them
      ingu: distinct (group, slot) keys in random order (HQ_INGEST_UNIQUE)
      inga: as ing with the per-record atomic path forced (HQ_INGEST_ATOMIC)"""
    from dragonboat_amd import hipquorum as hq

    ctx = hq.Context(d.device)
    r = np.random.default_rng(SEED_BASE + d.rank)
    parity = None
    if name in ("rim", "rimt", "rimtc"):
        rim_in = rim_inputs(d.rank)
        G, K, n, ordn, idx = rim_in
        # ordinals + ctx index in; released index (not for rimtc), count and batch end out
        per = G * (2 * K * n + 8 * K + (0 if name == "rimtc" else 8 * K) + 2)
        nsets = max(4, int(np.ceil(ROTATE_BYTES / per)))
        sets = [(ctx.upload(ordn.reshape(-1)), ctx.upload(idx.reshape(-1)),
                 ctx.empty(K * G, np.uint64), ctx.empty(G, np.uint8), ctx.empty(G, np.uint8))
                for _ in range(nsets)]
        if name in ("rimt", "rimtc"):     # the same inputs as 128-group tiles (one per wave)
            tb = hq.ri_tile_bytes(K, n, 0)
            tiled = []
            for o, x, rel, cnt, bend in sets:
                t = ctx.empty((G // 128) * tb, np.uint8)
                ctx.tile_ri_multi_dev(G, K, n, o, x, None, None, t)
                ctx.sync()
                ctx.free(o)
                ctx.free(x)
                tiled.append((t, rel, cnt, bend))

            def run(i):
                t, rel, cnt, bend = tiled[i % nsets]
                ctx.readindex_multi_tiles_dev(G, K, n, t, 0, n, None if name == "rimtc" else rel,
                                              cnt, batch_end=bend)
        else:
            def run(i):
                o, x, rel, cnt, bend = sets[i % nsets]
                ctx.readindex_multi_dev(G, K, n, o, x, None, None, n, rel, cnt, batch_end=bend)
        desc = (f"{name}: general multi-ctx ReadIndex release (suffix-min), {G} groups x {K} "
                f"pending ctxs x {n} voters" + (", 128-group tiles" if name != "rim" else "")
                + (", compact outputs (released count + batch ends; the released index derived "
                   "from ctx_index by the caller, hq_ri_released_host, outside the timed region)"
                   if name == "rimtc" else ""))
        units, unit = G, "releases/s"
    elif name == "cq":
        G, n = 16 << 20, 7
        per = G * 2 + G // 8
        nsets = max(4, int(np.ceil(ROTATE_BYTES / per)))
        sets = []
        for k in range(nsets):
            act = ctx.empty(G, np.uint8)
            ctx.synth_bitmaps_dev(hq.synth_spec(SEED_BASE + 3 + (k << 40), G, n), act)
            sets.append((act, ctx.empty(hq.words64(G), np.uint64)))
        ctx.sync()

        def run(i):
            act, hqb = sets[i % nsets]
            ctx.check_quorum_dev(G, act, None, n, 0, hqb)
        desc = f"cq: CheckQuorum (leaderHasQuorum + setNotActive), {G} groups x {n} voters"
        units, unit = G, "decisions/s"
    elif name == "cqp":
        G, n = 16 << 20, 7
        pb = hq.cq_plane_bytes(G, n)
        per = 2 * pb + G // 8          # active planes read + zeroed, has_quorum bits
        nsets = max(4, int(np.ceil(ROTATE_BYTES / per)))
        sets = []
        for k in range(nsets):
            act = ctx.empty(G, np.uint8)
            ctx.synth_bitmaps_dev(hq.synth_spec(SEED_BASE + 3 + (k << 40), G, n), act)
            pl = ctx.empty(pb, np.uint8)
            ctx.tile_cq_planes_dev(G, act, None, n, 0, pl)
            ctx.sync()
            ctx.free(act)
            sets.append((pl, ctx.empty(hq.words64(G), np.uint64)))

        def run(i):
            pl, hqb = sets[i % nsets]
            ctx.check_quorum_planes_dev(G, pl, n, hqb)
        desc = (f"cqp: CheckQuorum over active-flag planes (the leader's slot implicit, "
                f"{n - 1} planes of 2048 groups; bit-sliced count, planes zeroed in place), "
                f"{G} groups x {n} voters")
        units, unit = G, "decisions/s"
    elif name == "c4pq":
        G, n = 16 << 20, 7
        T = hq.HQ_PLANE_TILE_GROUPS
        pb, ab = hq.plane_tiles(G) * 3 * T, hq.cq_plane_bytes(G, 8)
        # 24 vote / ack planes + 7 active planes read, the active planes zeroed, confirmed +
        # has-quorum bits and the 2-bit outcome codes written
        per = pb + 2 * ab + hq.words64(G) * 8 * 2 + hq.words32(G) * 8
        nsets = max(4, int(np.ceil(ROTATE_BYTES / per)))
        sets = []
        for k in range(nsets):
            arrs = [ctx.empty(G, np.uint8) for _ in range(4)]
            ctx.synth_bitmaps_dev(hq.synth_spec(SEED_BASE + 3 + (k << 40), G, n), *arrs)
            pl, apl = ctx.empty(pb, np.uint8), ctx.empty(ab, np.uint8)
            ctx.tile_planes_dev(G, *arrs, 0, pl)
            # the active flags: the same generator's ack bitmaps of another seed
            ctx.synth_bitmaps_dev(hq.synth_spec(SEED_BASE + 5 + (k << 40), G, n), arrs[0])
            ctx.tile_cq_planes_dev(G, arrs[0], None, 8, 0, apl)
            ctx.sync()
            for a in arrs:
                ctx.free(a)
            sets.append((pl, apl, ctx.empty(hq.words64(G), np.uint64),
                         ctx.empty(hq.words32(G), np.uint64), ctx.empty(hq.words64(G), np.uint64)))

        def run(i):
            ctx.readindex_vote_cq_planes_dev(G, *sets[i % nsets])
        desc = (f"c4pq: ReadIndex confirm + vote tally + CheckQuorum (setNotActive) in one pass "
                f"over bit planes (24 vote / ack planes + 7 active planes per 2048 groups), {G} "
                f"groups x {n} voters, 3 decisions per group")
        units, unit = 3 * G, "decisions/s"
    else:   # ing / ingo / ingu / inga: the device table in the headline layout (leader-row tiles)
        G, n, U = 4 << 20, 3, 4 << 20
        form = hq.HQ_FORM_TERM_MASK
        per = U * 16 + U * 16          # the update + the 8-byte read-modify-write of its match
        nsets = max(4, int(np.ceil(ROTATE_BYTES / (U * 16))))
        table = ctx.empty(hq.commit_tiles(G) * hq.commit_tile_words(n, form,
                                                                    hq.HQ_LAYOUT_TILES_LEADER),
                          np.uint64)
        ctx.memset(table, 0)
        ups = []
        for k in range(nsets):
            if name == "ingu":     # distinct (group, slot) keys: a step's final ack per member
                keys = r.permutation(G * (n - 1))[:U].astype(np.uint64)
                g, s = keys // np.uint64(n - 1), keys % np.uint64(n - 1) + np.uint64(1)
            else:
                g = r.integers(0, G, U, dtype=np.uint64)
                s = r.integers(1, n, U, dtype=np.uint64)
            u = np.stack([(g << np.uint64(8)) | s,
                          np.uint64(1 << 30) + np.uint64(k) + r.integers(0, 64, U, dtype=np.uint64)],
                         axis=1)
            if name == "ingo":
                # the order a step worker emits them: node by node (execengine.go:923-1000)
                u = u[np.argsort(u[:, 0], kind="stable")]
            ups.append(ctx.upload(u.reshape(-1)))
        flags = {"ingo": hq.HQ_INGEST_GROUPED, "ingu": hq.HQ_INGEST_UNIQUE,
                 "inga": hq.HQ_INGEST_ATOMIC}.get(name, 0)

        def run(i):
            ctx.table_ingest_match_dev(ups[i % nsets], U, table, G, n, form, flags)
        desc = (f"{name}: ReplicateResp match-delta ingest (remote.tryUpdate) into a {G} x {n} "
                f"device table in the headline layout (leader-row tiles), {U} deltas "
                + {"ingo": "in group order (as a step worker emits them): runs reduced in "
                           "registers, plain read-modify-write, atomics only at wave edges "
                           "(HQ_INGEST_GROUPED)",
                   "ingu": "with distinct (group, slot) keys in random order (HQ_INGEST_UNIQUE; "
                           "a dense batch goes binned, as ing)",
                   "inga": "in random order, one 64-bit atomic max each (HQ_INGEST_ATOMIC: the "
                           "per-record path, forced)"}.get(
                       name, "in random order: binned in two streaming passes without global "
                             "atomics (k_bin + k_apply, the default for a dense batch)"))
        units, unit = U, "updates/s"
    elapsed, avg, launches = _timed(ctx, d, run, steps, warmup)
    if parity_threads and name in ("rim", "rimt", "rimtc"):
        # every set holds the same inputs: set 0's outputs as the timed runs left them
        rel, cnt, bend = (tiled[0][1:] if name != "rim" else sets[0][2:])
        ctx.sync()
        got = {"released_count": ctx.download(cnt), "batch_end": ctx.download(bend)}
        got["released_index"] = (hq.ri_released_host(K, idx, got["released_count"],
                                                     got["batch_end"])
                                 if name == "rimtc" else ctx.download(rel))
        parity = rim_parity(rim_in, got, parity_threads)
    elif parity_threads and name == "c4pq":
        # set 0 once more with its active planes packed afresh (the timed runs zeroed them, as
        # setNotActive does), its outputs poisoned first
        pl, apl, conf, outc, hqb = sets[0]
        act = ctx.empty(G, np.uint8)
        ctx.synth_bitmaps_dev(hq.synth_spec(SEED_BASE + 5, G, n), act)
        ctx.tile_cq_planes_dev(G, act, None, 8, 0, apl)
        for x in (conf, outc, hqb):
            ctx.memset(x, 0xA5)
        ctx.readindex_vote_cq_planes_dev(G, pl, apl, conf, outc, hqb)
        ctx.sync()
        got = {"confirmed": ctx.download(conf), "outcome": ctx.download(outc),
               "has_quorum": ctx.download(hqb)}
        t0 = time.perf_counter()
        want = c4pq_oracle(SEED_BASE + 3, SEED_BASE + 5, G, n, parity_threads)
        eq = {k: bool(np.array_equal(got[k], want[k])) for k in want}
        parity = dict(groups=G, equal=all(eq.values()), check_s=time.perf_counter() - t0, **eq)
    ctx.close()
    # the timed region opens behind the first launch: a step of L launches counts L * steps - 1
    L = max(1, round((launches + 1) / max(1, steps)))
    step_s = avg * L                     # the kernels of one step, back to back
    return {
        "workload": desc, "value": d.sum(float(units * steps)) / elapsed, "unit": unit,
        "kernel_avg_us": avg * 1e6, "launches_per_step": L,
        "kernel_us_per_step": step_s * 1e6,
        "roofline_achieved_gbs": per / step_s / 1e9,
        "roofline_frac": per / step_s / 1e9 / HBM_PEAK_GBS,
        "algorithmic_bytes_per_step": per,
        **({"parity_full_size": parity} if parity is not None else {}),
    }


def run_concurrent(w, steps, warmup, d: Dist, W=2):
    """W step workers stepping the same workload concurrently, each with its own hq_ctx (= its
    own HIP stream; dragonboat runs one goroutine per step worker, execengine.go:675-690, and
    the boundary gives each its own context): step i runs on worker i % W, so one worker's
    grid fill / drain overlaps another's stream. Kernels of different workers overlap, so only
    the aggregate rate (bytes / wall time) is meaningful here, not a per-kernel duration."""
    from dragonboat_amd import hipquorum as hq
    from dragonboat_amd import shard

    ctxs = [hq.Context(d.device) for _ in range(W)]
    sets, per_set = build_sets(ctxs[0], hq, shard, w, d)

    def seqs(k):
        return [hq.commit_batch_array([batch_args(b) for i in range(c, k, W)
                                       for b in sets[i % len(sets)]]) for c in range(W)]

    def run(arrs):
        for c, a in zip(ctxs, arrs):
            c.commit_many_dev(a)
        for c in ctxs:
            c.sync()

    run(seqs(max(W, warmup)))
    d.sync_device()
    d.barrier()
    timed = seqs(steps)
    t0 = time.perf_counter()
    run(timed)
    d.sync_device()
    d.barrier()
    elapsed = d.max(time.perf_counter() - t0)
    for c in ctxs:
        c.close()
    gbs = d.sum(float(per_set * steps)) / elapsed / 1e9
    return {
        "workload": f"w{W}: the headline workload ({w['G']} groups x {w['n']} voters per step, "
                    f"{w['desc'].split(',')[0]}) stepped by {W} concurrent step workers, one HIP stream "
                    f"each, step i on worker i % {W}",
        "value": d.sum(float(groups_per_step(w) * steps)) / elapsed, "unit": "decisions/s",
        "ms_per_step": elapsed / steps * 1e3,
        "aggregate_gbs": gbs, "aggregate_frac_of_peak": gbs / d.world / HBM_PEAK_GBS,
        "note": "kernels of different workers overlap; rate = algorithmic bytes / wall time",
    }


def run_e2e(steps, warmup, d: Dist, G=1 << 20, n=5, variants=None):
    """Host-fed end to end, PCIe included — never the headline `value`.
    Per step: pinned H2D of G/4 leader appends + G follower match deltas, append + ingest kernels
    into the device-resident table held in the headline layout (leader-row tiles, term mask), the
    headline kernel deciding it in place, then D2H of the changed and fallback bitmaps and the
    committed column (dragonboat_amd/pipeline.py). Reported: 8-byte records in group order
    (grouped ingest, no atomics) with no copies at all (the kernels read the records and write
    the results over PCIe, one stream: steady at the link's read + write time); beside it the
    copy-engine pipelines over 2 contexts (8- and 16-byte records, atomic ingest of unsorted
    records) and one stream. Timed over >= 100 steps: the copy pipelines run faster for their
    first ~20 steps and then alternate with multi-ms stalls (profiles/r02k/)."""
    from dragonboat_amd import hipquorum as hq
    from dragonboat_amd import shard
    from dragonboat_amd.pipeline import HostFedPipeline

    rng = shard.rank_shard(d.rank, d.world, G)
    spec = hq.synth_spec(SEED_BASE + 9, G, n, cid_base=rng.cid_base, cid_stride=rng.cid_stride)
    nb = 4   # distinct host batches cycled through
    out = {}
    # the first pipeline of a process pays one-time costs (first touch of pinned staging, the
    # copy engines' first mappings): a throwaway run of the headline variant goes first
    variants = variants or ((2, True, True, True), (2, True, True, True), (2, True, True),
                            (2, False, True), (2, True, False), (2, False, False),
                            (1, False, False))
    for v in variants:
        depth, compact, grouped = v[:3]
        zero_copy = len(v) > 3 and bool(v[3])
        r = np.random.default_rng(d.rank)
        p = HostFedPipeline(d.device, G, n, G // 4, G, depth=depth, compact=compact,
                            grouped=grouped, zero_copy=zero_copy)
        p.synth(spec)
        last = hq.tile_view(p.ctxs[0].download(p.tiles), G, n, p.form,
                            p.layout).row("last_index")
        apps, upds = [], []
        for k in range(nb):
            g = np.sort(r.choice(G, G // 4, replace=False)).astype(np.uint64)
            gu = r.integers(0, G, G, dtype=np.uint64)
            su = r.integers(1, n, G, dtype=np.uint64)
            if grouped:   # node by node, as a step worker emits them
                o = np.lexsort((su, gu))
                gu, su = gu[o], su[o]
            if compact:
                app = p.ctxs[0].pinned(len(g), np.uint64)
                app[:] = hq.pack_append_counts(g, np.full(len(g), k + 1, np.uint64))
                upd = p.ctxs[0].pinned(G, np.uint64)
                upd[:] = hq.pack_lag_updates(gu, su, r.integers(0, 4, G, dtype=np.uint64))
            else:
                app = p.ctxs[0].pinned(2 * len(g), np.uint64)
                app[0::2], app[1::2] = g, last[g] + np.uint64(k + 1)
                upd = p.ctxs[0].pinned(2 * G, np.uint64)
                upd[0::2] = (gu << np.uint64(8)) | su
                upd[1::2] = last[gu] + np.uint64(k)
            apps.append(app)
            upds.append(upd)
        for i in range(warmup):
            p.step(i, apps[i % nb], G // 4, upds[i % nb], G)
        p.sync()
        d.barrier()
        t0 = time.perf_counter()
        for i in range(steps):
            p.step(i, apps[i % nb], G // 4, upds[i % nb], G)
        p.sync()
        d.barrier()
        out[tuple(v)] = d.max(time.perf_counter() - t0)
        p.close()

    def pcie(w):   # H2D records + D2H changed / fallback bitmaps and committed column per step
        return (G // 4) * w + G * w + 2 * hq.words64(G) * 8 + G * 8

    def rec(key):
        w = 8 if key[1] else 16
        return {"value": d.sum(float(G * steps)) / out[key], "ms_per_step": out[key] / steps * 1e3,
                "pcie_bytes_per_step": pcie(w), "pcie_gbs": pcie(w) * steps / out[key] / 1e9}

    res = {
        "workload": f"e2e: host-fed {G} groups x {n} voters per GPU per step into the device "
                    f"table in the headline layout (leader-row tiles, term mask): {G // 4} "
                    f"appends + {G} match deltas (8-byte records in pinned host memory, group "
                    f"order) read over PCIe by the append + grouped ingest kernels, the headline "
                    f"kernel deciding in place, the changed / fallback bitmaps and the committed "
                    f"column written straight into pinned host memory (zero-copy, one stream); "
                    f"beside it the same with copy-engine copies pipelined over 2 contexts",
        "unit": "decisions/s",
    }
    if (2, True, True, True) in out:
        res.update(rec((2, True, True, True)))
    for key, name in (((2, True, True), "records_8B_grouped_copies_pipelined"),
                      ((2, False, True), "records_16B_grouped_pipelined"),
                      ((2, True, False), "records_8B_atomic_pipelined"),
                      ((2, False, False), "records_16B_atomic_pipelined"),
                      ((1, False, False), "records_16B_atomic_one_stream"),
                      ((1, True, True), "records_8B_grouped_one_stream")):
        if key in out:
            res[name] = rec(key)
    return res


STEP_ROLES = {
    # node 1 leads; the rest follow in member order
    "step": ("remote",) * 3,
    # BASELINE config 3's membership: 4 full members (leader included), 1 witness, 2 observers
    "step5": ("remote",) * 4 + ("witness",) + ("observer",) * 2,
}


def step_groups(hq, G, cid_base, cid_stride, roles=STEP_ROLES["step"], last0=1000):
    """Leader groups of the step workload (node 1 leads, term 5, all caught up); member k has
    node id k + 1 and role roles[k]."""
    role_code = {"remote": hq.ROLE_REMOTE, "witness": hq.ROLE_WITNESS,
                 "observer": hq.ROLE_OBSERVER}
    nm = len(roles)
    cids = np.uint64(cid_base) + np.arange(G, dtype=np.uint64) * np.uint64(cid_stride)
    g = np.zeros(G, hq.WORKER_GROUP_DTYPE)
    g["cluster_id"], g["node_id"], g["term"], g["state"] = cids, 1, 5, hq.STATE_LEADER
    g["committed"], g["last_index"], g["term_start"], g["n_members"] = last0, last0, last0 - 10, nm
    m = np.zeros(nm * G, hq.MEMBER_DTYPE)
    m["node_id"] = np.tile(np.arange(1, nm + 1, dtype=np.uint64), G)
    m["role"] = np.tile(np.array([role_code[r] for r in roles], np.uint32), G)
    m["match"] = last0
    return g, m, cids


def step_events(hq, G, s, roles=STEP_ROLES["step"], last0=1000):
    """Step s of the steady-state leader workload, as hq_step_input rows (every group, in
    handle order): every 4th group serves a local ReadIndex; every other member acks the
    leader's previous append (ReplicateResp, witnesses and observers included) and answers a
    heartbeat (the ReadIndex groups' heartbeats to voting members carry the ctx, observers get
    ctx-less ones, raft.go:836-848); every group proposes one entry. Per group: 2 (m - 1)
    messages, 1 proposal, 1/4 read -> 1 commit decision and 1/4 ReadIndex decision."""
    others = [(k + 1, r) for k, r in enumerate(roles)][1:]
    nmsg = 2 * len(others)
    last_s = np.uint64(last0 + s)
    has_read = (np.arange(G) % 4) == 0
    per = nmsg + 1 + has_read.astype(np.int64)
    offsets = np.zeros(G + 1, np.uint64)
    offsets[1:] = np.cumsum(per)
    ev = np.zeros(int(offsets[-1]), hq.EVENT_DTYPE)
    base = offsets[:-1].astype(np.int64)
    ctx_low = (np.uint64(s + 1) << np.uint64(32)) | np.arange(G, dtype=np.uint64)
    rd = np.nonzero(has_read)[0]
    r = ev[base[rd]]                                   # node.handleReadIndex
    r["kind"], r["hint"], r["hint_high"] = hq.EV_READ, ctx_low[rd], s + 1
    ev[base[rd]] = r
    first_msg = base + has_read
    msgs = [(frm, 13, role) for frm, role in others] + [(frm, 18, role) for frm, role in others]
    for k, (frm, typ, role) in enumerate(msgs):
        idx = first_msg + k
        blk = ev[idx]
        blk["kind"], blk["type"], blk["from"], blk["term"] = hq.EV_MESSAGE, typ, frm, 5
        if typ == 13:
            blk["log_index"] = last_s
        elif role != "observer":
            blk["hint"] = np.where(has_read, ctx_low, 0)
            blk["hint_high"] = np.where(has_read, s + 1, 0)
        ev[idx] = blk
    p = ev[first_msg + nmsg]
    p["kind"], p["log_index"] = hq.EV_PROPOSE, 1
    ev[first_msg + nmsg] = p
    return np.arange(G, dtype=np.uint32), offsets, ev


def _partition(ev_full, b0, b1):
    """The step input of groups [b0, b1) of a full step_events() input, as its own worker's
    (handles 0 .. b1 - b0 - 1)."""
    _, off, ev = ev_full
    o = off[b0:b1 + 1]
    return (np.arange(b1 - b0, dtype=np.uint32), o - o[0], ev[int(o[0]):int(o[-1])])


STEP_WARM = 2
STEP_WAIT_DEFAULT = "block"      # the step legs' wait policy (run_step_leg, BENCH_STEP_WAIT)


class StepRows:
    """The steady-state step inputs of step_events(), kept in ONE row array and advanced in
    place. Rows of step s + 1 differ from step s only in the ReplicateResp log index and the
    ReadIndex ctx words, and the rows repeat with a period of 4 groups (group 4p serves the read),
    so set(s) is a few strided column writes instead of a regeneration (equality with
    step_events() is tested in tests/test_bench_host.py)."""

    WORDS = 7     # hq_event = 56 bytes = 7 u64 words: kind|type, from, term, log_index, hint,
    #               hint_high, reject|reserved

    def __init__(self, hq, G, roles, last0=1000):
        assert G % 4 == 0 and hq.EVENT_DTYPE.itemsize == 8 * self.WORDS
        self.G, self.last0, self.s = G, last0, 0
        self.groups, self.offsets, self.ev = step_events(hq, G, 0, roles, last0)
        others = list(enumerate(roles))[1:]
        k = len(others)
        per = 2 * k + 1                      # ReplicateResps, HeartbeatResps, the proposal
        self.period = 4 * per + 1
        assert len(self.ev) == (G // 4) * self.period
        self.u = self.ev.view(np.uint64).reshape(G // 4, self.period, self.WORDS)
        starts = [1] + [per + 1 + j * per for j in range(3)]
        self.repl = [st + j for st in starts for j in range(k)]
        self.hb_ctx = [1 + k + j for j, (_, r) in enumerate(others) if r != "observer"]
        self.read = 0
        self.g0 = np.arange(0, G, 4, dtype=np.uint64)

    def set(self, s):
        """Make the rows those of step s."""
        u, s1 = self.u, np.uint64(s + 1)
        u[:, self.repl, 3] = np.uint64(self.last0 + s)
        ctx = (s1 << np.uint64(32)) | self.g0
        u[:, self.read, 4] = ctx
        u[:, self.read, 5] = s1
        for p in self.hb_ctx:
            u[:, p, 4] = ctx
            u[:, p, 5] = s1
        self.s = s
        return self.groups, self.offsets, self.ev


class StepRows16:
    """The producer's form of the same steps (step_events / StepRows): one 16-byte compact record
    per message (hq_event16) instead of the 56-byte row, what a step worker's queue must hold of a
    received pb.Message for this path (raft.proto:154-168); hq_events16_encode_sized turns them
    into the same stream bytes. The steady-state step needs no escape, so record i is row i and
    set(s) writes the same few strided columns as StepRows.set (equality with hq_events_to16 of
    step_events() is tested in tests/test_bench_host.py)."""

    def __init__(self, hq, G, roles, last0=1000):
        assert G % 4 == 0
        self.G, self.last0, self.s = G, last0, 0
        _, off, ev = step_events(hq, G, 0, roles, last0)
        self.recs, self.offsets = hq.events_to16(off, ev)
        assert np.array_equal(self.offsets, off)
        k = len(roles) - 1
        per = 2 * k + 1
        self.period = 4 * per + 1
        self.r = self.recs.reshape(G // 4, self.period)
        starts = [1] + [per + 1 + j * per for j in range(3)]
        self.repl = [st + j for st in starts for j in range(k)]
        self.g0 = np.arange(0, G, 4, dtype=np.uint64)

    def set(self, s):
        """Make the records those of step s (the heartbeat acks refer to the READ's ctx)."""
        s1 = np.uint64(s + 1)
        v = self.r["value"]
        v[:, self.repl] = np.uint64(self.last0 + s)
        v[:, 0] = (s1 << np.uint64(32)) | self.g0
        self.r["term"][:, 0] = s + 1
        self.s = s
        return self.offsets, self.recs


def _shard_of(d, G):
    from dragonboat_amd import shard

    return shard.rank_shard(d.rank, d.world, G)


def _median(xs):
    return float(np.median(xs)) if xs else None


_MIX_C1, _MIX_C2 = np.uint64(0xbf58476d1ce4e5b9), np.uint64(0x94d049bb133111eb)
_READY_K = (np.uint64(0x9e3779b97f4a7c15), np.uint64(0xc2b2ae3d27d4eb4f),
            np.uint64(0x165667b19e3779f9))


def mix64(z):
    """splitmix64's finalizer over a u64 array (qref_mix64, oracle/qref.h)."""
    z = (z ^ (z >> np.uint64(30))) * _MIX_C1
    z = (z ^ (z >> np.uint64(27))) * _MIX_C2
    return z ^ (z >> np.uint64(31))


def ready_terms(ready):
    """qref_digest_ready of each ReadyToRead record (READY_DTYPE), as uint64."""
    k1, k2, k3 = _READY_K
    return mix64(mix64(ready["cluster_id"]) ^ (ready["index"] * k1 + ready["ctx_low"] * k2 +
                                                ready["ctx_high"] * k3))


def ready_digest(ready):
    """Sum over ReadyToRead records (READY_DTYPE) of qref_digest_ready, mod 2^64."""
    if len(ready) == 0:
        return 0
    return int(ready_terms(ready).sum(dtype=np.uint64))


def ready_order_digest(ready, pos0=0):
    """qref_step_totals.ready_order_digest's terms for records at positions pos0, pos0 + 1, ...:
    the sum of (position + 1) * qref_digest_ready, mod 2^64 (a reordered list changes it)."""
    if len(ready) == 0:
        return 0
    w = np.arange(pos0 + 1, pos0 + 1 + len(ready), dtype=np.uint64)
    return int((ready_terms(ready) * w).sum(dtype=np.uint64))


class CommitMirror:
    """The committed index of every group of one step-leg mode, advanced from that mode's
    results, so each step's commits reduce to (cluster, advance) pairs whatever form the worker
    returned them in ('committed_advance', 'committed_column' or the 'commits' list); their
    digest is qref_digest_commit's sum (oracle/qref.h)."""

    def __init__(self, cids, committed, bounds):
        assert np.all(cids[1:] > cids[:-1])         # sorted: the commits list maps by search
        self.cids, self.bounds = cids, bounds
        self.coef = mix64(cids) | np.uint64(1)
        self.c = committed.astype(np.uint64).copy()

    def step(self, res):
        """(commits, ReadyToReads, sum of advances, ready digest, commit digest, ordered ready
        digest) of one step; the workers' lists in worker order make the step's list."""
        from dragonboat_amd import hipquorum as hq
        n_c = n_r = adv_sum = rd = cd = od = 0
        for i, r in enumerate(res):
            lo, hi = self.bounds[i], self.bounds[i + 1]
            # ReadyToReads as 24-byte records (HQ_WORKER_READY_COMPACT) in the list and the
            # per-tile slots (HQ_WORKER_READY_SLOTS): the cluster id and the index rebuilt from
            # the group's position and its committed index before the step, the two merged in
            # group order (the reference's)
            ready = hq.merge_ready(r, self.cids[lo:hi], self.c[lo:hi])
            if "committed_advance" in r:
                ix = np.arange(lo, hi)
                adv = r["committed_advance"][:hi - lo].astype(np.uint64)
            elif "committed_column" in r:
                ix = np.arange(lo, hi)
                adv = r["committed_column"][:hi - lo] - self.c[lo:hi]
            else:
                cm = r["commits"]
                ix = np.searchsorted(self.cids, cm["cluster_id"])
                assert np.array_equal(self.cids[ix], cm["cluster_id"])
                adv = cm["committed"] - self.c[ix]
            self.c[ix] += adv
            n_c += int(r.get("n_commits", len(r["commits"])))
            adv_sum += int(adv.sum(dtype=np.uint64))
            cd += int((self.coef[ix] * adv).sum(dtype=np.uint64))
            od += ready_order_digest(ready, n_r)
            n_r += len(ready)
            rd += ready_digest(ready)
        m = (1 << 64) - 1
        return (n_c, n_r, adv_sum & m, rd & m, cd & m, od & m)


def _latency(ts):
    """p50 / p99 / max (ms) of per-step wall times (s)."""
    if not ts:
        return None
    a = np.asarray(ts) * 1e3
    return {"p50": round(float(np.percentile(a, 50)), 4), "p99": round(float(np.percentile(a, 99)), 4),
            "max": round(float(a.max()), 4), "n": len(a)}


def _device_split(rs):
    """One jobs step's device time split (ms) from its workers' outputs (hq_step_output): the
    host's submit, the GPU's time between the step's timing events, the outputs' mapping, and the
    rest of the wait (the waiting thread's wake-up and queueing ahead of the step's work); the
    wait itself (its poll and sleep), and the raw clocks of its end for _wake_lag: the host's
    steady clock at the wait's return and the device's 100-MHz stamp after the step
    (HQ_WAIT_CLOCK)."""
    r = max(rs, key=lambda x: x["pass_ns"])
    rest = r["pass_ns"] - r["pack_ns"] - r["gpu_ns"] - r["apply_ns"]
    return {"submit_ms": r["pack_ns"] / 1e6, "gpu_ms": r["gpu_ns"] / 1e6,
            "outputs_ms": r["apply_ns"] / 1e6, "wait_rest_ms": rest / 1e6,
            "wait_ms": r["device_ns"] / 1e6, "wait_poll_ms": r["wait_poll_ns"] / 1e6,
            "wait_sleep_ms": r["wait_sleep_ns"] / 1e6, "wait_sleeps": r["wait_sleeps"],
            "_end_ns": r["wait_end_ns"], "_end_ticks": r["device_end_ticks"],
            # the device's own span of the step, first stamp to last (HQ_WAIT_CLOCK): far above
            # gpu_ms, the step waited in the device's queue or behind its last kernel
            "span_ms": ((r["device_end_ticks"] - r["device_start_ticks"]) / 1e5
                        if r["device_start_ticks"] and r["device_end_ticks"] else None)}


_LINK = {}


def _link_probe(d):
    """The host link's measured rates for kernels that read / write pinned host memory in place
    (tools/link_probe --json, 64 MiB per direction, best of its grids; built by `make all`):
    one direction at a time and both at once. Run once per process, on rank 0 (None elsewhere
    or when the probe is missing or fails)."""
    if "v" in _LINK:
        return _LINK["v"]
    v = None
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools", "link_probe")
    if d.rank == 0 and os.path.exists(exe):
        import subprocess
        try:
            r = subprocess.run([exe, "64", str(d.device), "--json"], capture_output=True,
                               text=True, timeout=90)
            if r.returncode == 0:
                v = json.loads(r.stdout.strip().splitlines()[-1])
        except (subprocess.SubprocessError, ValueError, IndexError):
            v = None
    _LINK["v"] = v
    return v


def _out_bytes(rs):
    """The bytes one jobs step's kernels wrote into the workers' pinned output (the host link's
    write direction): every list and column the results view, the ReadyToRead slots by their
    records and count words (the rest of each tile's slot is not written)."""
    n = 0
    for r in rs:
        for k, v in r.items():
            if k == "ready_slots":
                continue
            if isinstance(v, np.ndarray):
                n += v.nbytes
        if "ready_slots" in r:
            n += len(r["ready_slots"]) * 24 + 4 * ((len(r.get("committed_advance", ())) + 255) // 256)
    return n


def _link_block(d, bytes_in, bytes_out, gpu_ms):
    """The step's host-link roofline: bytes read from pinned memory (the stream and its size
    words) and written to it (the outputs) per step, over the GPU time of the step (median of
    the W = 1 device-only steps), against the probe's rates. frac = both directions' bytes per
    second over the probe's both-at-once total; frac_serial = the time the two directions
    would take one after the other at the probe's one-direction rates, over the GPU time."""
    lk = _link_probe(d)
    t = gpu_ms / 1e3
    out = {"bytes_in": int(bytes_in), "bytes_out": int(bytes_out), "gpu_ms": round(gpu_ms, 4),
           "in_GBps": round(bytes_in / t / 1e9, 2), "out_GBps": round(bytes_out / t / 1e9, 2),
           "both_GBps": round((bytes_in + bytes_out) / t / 1e9, 2), "probe": lk}
    if lk:
        out["frac"] = round((bytes_in + bytes_out) / t / 1e9 / lk["both_GBps"], 3)
        out["frac_serial"] = round((bytes_in / lk["read_GBps"] + bytes_out / lk["write_GBps"])
                                   / 1e9 / t, 3)
    else:
        out["frac"] = None
    return out


def _wake_lag(phases, prefix):
    """Each step's wake-up lateness (ms) from the clocks of its wait's end: the host's return
    time less the device's end stamp (10 ns per tick), each against the run's smallest such
    difference (the two clocks' offset: the best wake-up of the run counts as 0; the clocks
    drift by far less than a microsecond over a run). Written into the phases as
    <prefix>wake_lag_ms; the raw clocks are dropped."""
    d = [p[prefix + "_end_ns"] - 10 * p[prefix + "_end_ticks"] for p in phases
         if p.get(prefix + "_end_ticks")]
    base = min(d) if d else None
    for p in phases:
        t, k = p.pop(prefix + "_end_ns", 0), p.pop(prefix + "_end_ticks", 0)
        p[prefix + "wake_lag_ms"] = (t - 10 * k - base) / 1e6 if (k and base is not None) else None


def _phase_summary(ph):
    """The end-to-end steps' phases: medians, and the three slowest steps in full."""
    if not ph:
        return None
    keys = ("e2e_ms", "encode_max_ms", "execute_ms", "dev_ms", "enc_wall_ms", "enc_task_lag_max_ms",
            "cgroup_throttled_ms", "exe_gpu_ms", "exe_wait_rest_ms", "dev_gpu_ms",
            "dev_wait_rest_ms", "exe_wake_lag_ms", "dev_wake_lag_ms", "exe_wait_sleep_ms",
            "dev_wait_sleep_ms", "exe_span_ms", "dev_span_ms")
    med = {k: round(float(np.median([p[k] for p in ph])), 4) for k in keys
           if all(p.get(k) is not None for p in ph)}
    th = [p["cgroup_throttled_ms"] for p in ph if p.get("cgroup_throttled_ms") is not None]
    if th:
        med["steps_throttled"] = int(sum(1 for x in th if x > 0))
        med["throttled_ms_total"] = round(float(sum(th)), 3)
    slow = sorted(ph, key=lambda p: -p["e2e_ms"])[:3]
    slow_dev = sorted(ph, key=lambda p: -p["dev_ms"])[:2]
    rnd = lambda p: {k: (round(v, 4) if isinstance(v, float) else v) for k, v in p.items()}
    return {"median": med, "slowest": [rnd(p) for p in slow],
            "slowest_device_only": [rnd(p) for p in slow_dev]}


def run_step_leg(d, G=1 << 20, steps=50, with_cpu=True, name="step"):
    """The device step engine (hq_worker_step_stream, HQ_WORKER_ON_DEVICE: every event of the
    step taken on the GPU) over G leader groups per GPU, W = 1, 2 and 16 workers (dragonboat runs
    16 step workers, internal/settings/hard.go:35; each worker one native thread and one HIP
    stream, stepped at once by hq_worker_step_jobs), in two timings over the same `steps` steps:

      device_only  the step's event stream already encoded in pinned memory (the producer's
                   encode outside the timed region);
      end_to_end   the producer's encode inside: while the device takes step s, the producer
                   encodes step s + 1's messages for all W workers into their other pinned
                   stream buffers (one hq_events16_encode_sized_multi call on the encode
                   threads), and a step costs the longer of the two. The rows
                   stand for the pb.Message values the reference's step worker holds
                   (execengine.go:923-1000 -> node.go:1257-1287); making them (the messages
                   arriving) is outside both timings.

    Beside it the CPU event-by-event replay of the reference path (oracle/qref_step.c) over the
    same rows of the same steps, on all usable host cores, 16 threads and 1 thread. Every step's
    commit count, ReadyToRead count, sum of the committed advances and the content digests of
    (cluster, advance) over the groups that committed and of the ReadyToRead records (cluster,
    index, ctx) (CommitMirror; qref_step_totals, oracle/qref.h) must agree between every mode
    and the replay."""
    from concurrent.futures import ThreadPoolExecutor

    from dragonboat_amd import hipquorum as hq

    roles = STEP_ROLES[name]
    n_voting = sum(r != "observer" for r in roles)
    nm = len(roles)
    rng = _shard_of(d, G)
    g, m, cids = step_groups(hq, G, rng.cid_base, rng.cid_stride, roles)
    rows = StepRows(hq, G, roles)
    recs = StepRows16(hq, G, roles)      # the producer's compact form of the same messages
    offsets = rows.offsets
    # the producer's native encode threads per step, shared by the W workers' encodes
    enc_threads = encode_threads()
    # the step thread's wait (hq_worker_set_wait; BENCH_STEP_WAIT=block|sleep|spin[:poll:sleep])
    wait_name, *wv = os.environ.get("BENCH_STEP_WAIT", STEP_WAIT_DEFAULT).split(":")
    wait = ({"block": hq.HQ_WAIT_BLOCK, "sleep": hq.HQ_WAIT_SLEEP, "spin": hq.HQ_WAIT_SPIN,
             "adapt": hq.HQ_WAIT_ADAPT}[wait_name],
            int(wv[0]) if wv else 50, int(wv[1]) if len(wv) > 1 else 20)
    pin = hq.Context(d.device)
    Ws = (1, 2, 16)
    modes = {}
    for W in Ws:
        bounds = [G * i // W for i in range(W + 1)]
        parts = []
        for i in range(W):
            o = offsets[bounds[i]:bounds[i + 1] + 1]
            parts.append((o - o[0], int(o[0]), int(o[-1])))

        def workers():
            ws = []
            for i in range(W):
                wk = hq.Worker(d.device, n_voting, on_device=True, commit_column=True,
                               commit_advance=True, ready_compact=True, ready_slots=True)
                wk.set_wait(wait[0], wait[1], wait[2], clock=True)
                wk.add_groups(g[bounds[i]:bounds[i + 1]], m[nm * bounds[i]:nm * bounds[i + 1]])
                ws.append(wk)
            return ws
        # the receive buffers: the stream bytes and the 2-byte size words (hq_step_stream.sizes16)
        bufs = [[(pin.pinned((e1 - e0) * 5 + 64, np.uint8), pin.pinned(len(o) - 1, np.uint16))
                 for o, e0, e1 in parts] for _ in range(2)]
        modes[W] = dict(parts=parts, bufs=bufs, nbytes=[[0] * W, [0] * W], dev=workers(),
                        e2e=workers(), t={"dev": [], "e2e": []}, bytes=0, phases=[],
                        check={"dev": [], "e2e": []}, link=[],
                        mirror={k: CommitMirror(cids, g["committed"], bounds)
                                for k in ("dev", "e2e")})
    pool = ThreadPoolExecutor(max(Ws) + 1)

    # the producer's encode calls, one per (W, buffer slot): the records and the receive buffers
    # stay in place from step to step (StepRows16.set rewrites the records in place), so each
    # call's job table is built once (hq.Encode16Batch)
    batches = {(W, slot): hq.Encode16Batch([
        (off, recs.recs[e0:e1], modes[W]["bufs"][slot][i][0], modes[W]["bufs"][slot][i][1])
        for i, (off, e0, e1) in enumerate(modes[W]["parts"])]) for W in Ws for slot in (0, 1)}

    def encode(W, slot):
        """The W workers' streams of the current step from the producer's compact records, in
        one call on the encode threads (hq_events16_encode_sized_multi: the threads split the
        records of all workers evenly), each straight into its worker's pinned receive buffer.
        Returns its wall time (s)."""
        t0 = time.perf_counter()
        mo = modes[W]
        for i, (ne, nb) in enumerate(batches[(W, slot)].run(enc_threads)):
            assert ne == mo["parts"][i][2] - mo["parts"][i][1]
            mo["nbytes"][slot][i] = nb
        return time.perf_counter() - t0

    def timed_execute(j):
        t0 = time.perf_counter()
        j.execute()
        return time.perf_counter() - t0

    def jobs(W, slot, which):
        mo = modes[W]
        return hq.StepJobs([
            (wk, hq.SizedStream(None, mo["bufs"][slot][i][1], mo["parts"][i][2] - mo["parts"][i][1],
                                mo["bufs"][slot][i][0][:mo["nbytes"][slot][i]]))
            for i, wk in enumerate(mo[which])])

    cpus = {}
    # (BENCH_STEP_REPLAY=0: the legs without their CPU replay, the rest of the run's oracle
    # checks kept — a probe of the late-starting steps, profiles/r06l/)
    if with_cpu and d.rank == 0 and d.world == 1 and os.environ.get("BENCH_STEP_REPLAY", "1") != "0":
        from oracle import qref

        _, counts = cpu_thread_counts()
        cpus = {nt: [qref.StepBatch(g, m), [], []] for nt in counts}
    prev_sum = int(g["committed"].sum(dtype=np.uint64))
    rows.set(0)
    recs.set(0)
    for W in Ws:                       # step 0's streams (untimed)
        encode(W, 0)
    # the compact producer writes the bytes the rows encode to (step 0, one worker)
    want_data, want_sizes = hq.encode_events_sized(offsets, rows.ev)
    producer_equal = bool(np.array_equal(modes[1]["bufs"][0][0][0][:modes[1]["nbytes"][0][0]],
                                         want_data) and
                          np.array_equal(modes[1]["bufs"][0][0][1], hq.sizes16_of(want_sizes)))
    del want_data, want_sizes
    n_events = len(rows.ev)
    timed = 0
    # The CPU replay of every step's rows first, then the device steps: the replay (GBs of host
    # memory touched per step on up to all host cores) run between the device steps was followed,
    # about once per full run, by a device step whose first kernel started 5-18 ms after it was
    # queued (profiles/r06q/, r06l2/: never without the replay); a step worker has no replay
    # beside it. The replay's own timing and digests are the same work in the same order.
    for s in range(steps + STEP_WARM if cpus else 0):
        for nt, (b, ts, dg) in cpus.items():    # the CPU replay of the same rows
            t0 = time.perf_counter()
            tot = b.step(rows.groups, offsets, rows.ev, nthreads=nt)
            dt = time.perf_counter() - t0
            if s >= STEP_WARM:
                ts.append(dt)
            dg.append((tot["commits"], tot["ready"],
                       (tot["committed_sum"] - prev_sum) & ((1 << 64) - 1),
                       tot["ready_digest"], tot["commit_digest"], tot["ready_order_digest"]))
        prev_sum = tot["committed_sum"]
        rows.set(s + 1)
    for s in range(steps + STEP_WARM):
        slot = s % 2
        recs.set(s + 1)                # untimed: step s + 1's messages arrive
        for W in Ws:
            mo = modes[W]
            if s >= STEP_WARM:
                mo["bytes"] += sum(mo["nbytes"][slot])
            # (timed: the native step of the W workers; their result views are built after)
            j = jobs(W, slot, "dev")
            d.barrier()
            tq0 = cgroup_throttled_us()
            t0 = time.perf_counter()
            j.execute()
            dt = time.perf_counter() - t0
            tq1 = cgroup_throttled_us()
            rs = j.results(copy=False)
            dev_split = _device_split(rs)
            if W == 1 and s >= STEP_WARM:
                mo["link"].append((sum(mo["nbytes"][slot]) + 2 * G, _out_bytes(rs),
                                   dev_split["gpu_ms"]))
            mo["check"]["dev"].append(mo["mirror"]["dev"].step(rs))
            j = jobs(W, slot, "e2e")
            d.barrier()
            hq.encode_stats(reset=True)
            th0 = cgroup_throttled_us()
            t1 = time.perf_counter()
            fut = pool.submit(timed_execute, j)
            enc_s = [encode(W, 1 - slot)]      # (the producer's thread: this one)
            exe_s = fut.result()
            dt2 = time.perf_counter() - t1
            th1 = cgroup_throttled_us()
            es = hq.encode_stats(reset=True)
            rs = j.results(copy=False)
            e2e_split = _device_split(rs)
            mo["check"]["e2e"].append(mo["mirror"]["e2e"].step(rs))
            if s >= STEP_WARM:
                mo["t"]["dev"].append(dt)
                mo["t"]["e2e"].append(dt2)
                # where the end-to-end step went: the encodes (the slowest call), the device
                # step beside them, the encoder's task-start lag (hq_encode_stats)
                mo["phases"].append({"step": s - STEP_WARM, "e2e_ms": dt2 * 1e3,
                                     "encode_max_ms": max(enc_s) * 1e3,
                                     "execute_ms": exe_s * 1e3, "dev_ms": dt * 1e3,
                                     **{f"exe_{k}": v for k, v in e2e_split.items()},
                                     **{f"dev_{k}": v for k, v in dev_split.items()},
                                     "dev_throttled_ms": (None if tq0 is None or tq1 is None
                                                          else (tq1 - tq0) / 1e3),
                                     "enc_wall_ms": es["wall_ns"] / 1e6 / max(1, es["calls"]),
                                     "enc_task_lag_max_ms": es["max_lag_ns"] / 1e6,
                                     "cgroup_throttled_ms": (None if th0 is None or th1 is None
                                                             else (th1 - th0) / 1e3)})
        if s >= STEP_WARM:
            timed += 1
    pool.shutdown()
    committed = {}
    for W in Ws:
        for which in ("dev", "e2e"):
            committed[(W, which)] = [int(modes[W][which][0].get_group(int(c))[0]["committed"])
                                     for c in cids[:min(1024, G // max(Ws))]]
            for wk in modes[W][which]:
                wk.close()
    pin.close()
    ref = modes[1]["check"]["dev"]
    same_modes = all(modes[W]["check"][k] == ref for W in Ws for k in ("dev", "e2e")) and \
        len(set(map(tuple, committed.values()))) == 1
    mismatch = []
    if not same_modes:        # the first differing step of each mode, for the log
        for W in Ws:
            for k in ("dev", "e2e"):
                got = modes[W]["check"][k]
                bad = [i for i, (a, b) in enumerate(zip(got, ref)) if a != b]
                if bad or len(got) != len(ref):
                    i = bad[0] if bad else min(len(got), len(ref))
                    mismatch.append({"mode": f"{k}_w{W}", "step": i,
                                     "got": list(got[i]) if i < len(got) else None,
                                     "want": list(ref[i]) if i < len(ref) else None})
        c1 = committed[(1, "dev")]
        mismatch += [{"mode": f"{k}_w{W}", "committed_differs_at": next(
            (i for i, (a, b) in enumerate(zip(v, c1)) if a != b), len(v))}
            for (W, k), v in committed.items() if v != c1]
    for W in Ws:
        _wake_lag(modes[W]["phases"], "exe_")
        _wake_lag(modes[W]["phases"], "dev_")
    members = ", ".join(f"{roles.count(r)} {r}" for r in ("remote", "witness", "observer")
                        if roles.count(r))
    ev_total = n_events * timed

    def rate(ts):
        return d.sum(float(n_events * len(ts))) / d.max(sum(ts)) if ts else None

    dev = {f"w{W}": rate(modes[W]["t"]["dev"]) for W in Ws}
    e2e = {f"w{W}": rate(modes[W]["t"]["e2e"]) for W in Ws}
    out = {
        "workload": f"{name}: device step engine over {G} leader groups per GPU ({members}); per "
                    f"group and step {nm - 1} ReplicateResp + {nm - 1} HeartbeatResp, 1 proposal, "
                    f"1/4 local ReadIndex; {timed} timed steps",
        "unit": "events/s",
        "events_per_step": n_events,
        "value": e2e["w16"], "ms_per_step": n_events / e2e["w16"] * 1e3 * d.world,
        "median_ms_per_step": _median(modes[16]["t"]["e2e"]) * 1e3,
        "end_to_end": e2e, "device_only": dev,
        "ms_per_step_detail": {f"{k}_w{W}": {"mean": float(np.mean(modes[W]["t"][k]) * 1e3),
                                             "median": _median(modes[W]["t"][k]) * 1e3,
                                             "max": float(np.max(modes[W]["t"][k]) * 1e3)}
                               for W in Ws for k in ("dev", "e2e")},
        # step latency as the reference reports it (README.md:55-62: P99 / P99.9): per mode the
        # p50 / p99 / max of the timed steps, and the slowest end-to-end steps with their phases
        "latency_ms": {f"{k}_w{W}": _latency(modes[W]["t"][k]) for W in Ws for k in ("dev", "e2e")},
        "e2e_phases": {f"w{W}": _phase_summary(modes[W]["phases"]) for W in Ws},
        "wait_policy": {"mode": wait_name, "poll_us": wait[1], "sleep_us": wait[2],
                        "clock": "HQ_WAIT_CLOCK: the device's end stamp beside the host's return"},
        "stream_bytes_per_event": modes[1]["bytes"] / max(1, ev_total),
        # the host-link roofline of the W = 1 device-only steps (medians over the timed steps)
        "link": (_link_block(d, *(float(np.median([x[i] for x in modes[1]["link"]]))
                                  for i in range(3))) if modes[1]["link"] else None),
        "modes_agree": same_modes,
        **({"modes_mismatch": mismatch} if mismatch else {}),
        "producer": f"compact 16-byte message records (hq_event16), the W workers' streams "
                    f"encoded by one hq_events16_encode_sized_multi call per step on "
                    f"{enc_threads} native threads (the usable CPUs less two, capped by the "
                    f"cgroup quota) splitting the records of all workers evenly",
        "producer_equal_rows": producer_equal,
        "note": "end_to_end: the producer's encode of step s + 1 overlapped with the device step "
                "s; device_only: the encoded stream given",
    }
    if cpus:
        cpu = {str(nt): n_events * len(ts) / sum(ts) for nt, (_, ts, _) in cpus.items()}
        best = max(cpu.values())
        digs = [dg for _, _, dg in cpus.values()]
        out["cpu_replay"] = dict(cpu, sample=f"the same rows of the same {timed} timed steps "
                                             "replayed event by event (oracle/qref_step.c)")
        # every step: commit and ReadyToRead counts, the sum of the committed advances and the
        # content digests of (cluster, advance) and of the ReadyToRead records (cluster, index,
        # ctx), equal between the replay at every thread count, and every device mode
        out["parity_committed"] = bool(all(x == digs[0] for x in digs) and digs[0] == ref and
                                       same_modes)
        out["parity_checks"] = ("per step: commits, ReadyToReads, committed advance sum, "
                                "digest of (cluster, advance) and of ReadyToRead (cluster, "
                                "index, ctx), and a position-weighted ReadyToRead digest "
                                "(the list's order)")
        out["vs_cpu_replay_end_to_end"] = {k: v / best for k, v in e2e.items()}
        out["vs_cpu_replay_device_only"] = {k: v / best for k, v in dev.items()}
        for b, _, _ in cpus.values():
            b.close()
    return out


HQ_MSG_REPLICATE_RESP, HQ_MSG_HEARTBEAT_RESP = 13, 18


def _wire_arrivals(hq, ev, off, cids, roles, bounds, dep):
    """The step's received messages (a step_events() input) for the workers owning groups
    [bounds[i], bounds[i + 1]) as MessageBatch bytes, per worker, in the arrival order that keeps
    every group's messages in the rows' order (step_events: the ReplicateResps of the other
    members, then their HeartbeatResps): one batch per (message type, sender), the
    ReplicateResps' batches first — the senders' batches of one tick, marshalled by
    hq_wire_encode_batch (MessageBatch.MarshalTo) — and the worker's local events (ReadIndex,
    proposals) as (cluster ids, offsets, rows) for hq_wire_add_locals."""
    per = np.diff(off).astype(np.int64)
    grp = np.repeat(np.arange(len(off) - 1), per)
    is_msg = ev["kind"] == hq.EV_MESSAGE
    out = [([], None) for _ in range(len(bounds) - 1)]
    for typ in (HQ_MSG_REPLICATE_RESP, HQ_MSG_HEARTBEAT_RESP):
        for k in range(2, len(roles) + 1):
            sel = np.nonzero(is_msg & (ev["type"] == typ) & (ev["from"] == k))[0]
            gs = grp[sel]                                # (in group order)
            m = np.zeros(len(sel), hq.WIRE_MESSAGE_DTYPE)
            m["ev"] = ev[sel]
            m["cluster_id"] = cids[gs]
            m["to"] = 1
            cut = np.searchsorted(gs, bounds)
            for i in range(len(bounds) - 1):
                out[i][0].append(hq.encode_wire_batch(m[cut[i]:cut[i + 1]], deployment_id=dep,
                                                      source_address=b"n%d:63000" % k).copy())
    loc = np.nonzero(~is_msg)[0]
    gl = grp[loc]
    cnt = np.bincount(gl, minlength=len(off) - 1)
    res = []
    for i in range(len(bounds) - 1):
        lo, hi = bounds[i], bounds[i + 1]
        o = np.zeros(hi - lo + 1, np.uint64)
        o[1:] = np.cumsum(cnt[lo:hi])
        a, b = np.searchsorted(gl, [lo, hi])
        res.append((out[i][0], (cids[lo:hi].copy(), o, ev[loc[a:b]].copy())))
    return res


def run_wire_leg(d: Dist, G=1 << 14, reps=20):
    """The step worker's input from the wire (hq_wire.cpp), host side: the received messages of
    a steady-state step of G leader groups (3 voters: a ReplicateResp and a HeartbeatResp from
    each follower) marshalled as raftpb.MessageBatch bytes (one batch per message type and sending
    node), then per step, on one host thread: the production feed — hq_wire_reset +
    hq_wire_add_batch of every batch (protobuf decode with the Message.MarshalTo fast path,
    deployment / version check, each message's cluster resolved to the attached worker's handle)
    + hq_wire_add_locals + hq_wire_step_sized (the step's sized stream with 2-byte words, in
    handle order, straight into pinned buffers) — and, beside it, the first-appearance form
    (hq_wire_step_stream: clusters in order of first appearance, prefix arrays). The bytes are
    built outside the timed region. Both streams are stepped on the device engine and decide
    like the same step fed as rows."""
    from dragonboat_amd import hipquorum as hq

    roles = STEP_ROLES["step"]
    rng = _shard_of(d, G)
    g, m, cids = step_groups(hq, G, rng.cid_base, rng.cid_stride, roles)
    g["committed"] -= np.uint64(10)          # the step's acks (of lastIndex) commit
    m["match"][m["node_id"] != 1] -= np.uint64(10)
    dep = 0x5EED
    _, off, ev = step_events(hq, G, 0, roles)
    [(bufs, (lc, lo_, lev))] = _wire_arrivals(hq, ev, off, cids, roles, [0, G], dep)
    n_msg = int((ev["kind"] == hq.EV_MESSAGE).sum())
    n_bytes = sum(len(b) for b in bufs)
    nv = sum(r != "observer" for r in roles)
    w = hq.Worker(d.device, nv, on_device=True, commit_advance=True)
    w.add_groups(g, m)
    wa = hq.Worker(d.device, nv, on_device=True, commit_advance=True, ready_compact=True,
                   ready_slots=True)
    wa.add_groups(g, m)
    pin = hq.Context(d.device)
    pdata = pin.pinned(len(ev) * hq.HQ_EVENT_STREAM_MAX + 64, np.uint8)
    psizes = pin.pinned(G, np.uint16)
    wire, wire_a = hq.Wire(dep), hq.Wire(dep)
    wire_a.attach(wa)
    times, times_a = [], []
    for r in range(reps + 2):
        t0 = time.perf_counter()
        wire_a.reset()
        for b in bufs:
            wire_a.add_batch_at(b.ctypes.data, len(b))
        wire_a.add_locals(lc, lo_, lev)
        ss, st_a = wire_a.step_sized(pdata, psizes)
        t1 = time.perf_counter()
        wire.reset()
        for b in bufs:
            wire.add_batch_at(b.ctypes.data, len(b))
        wire.add_locals(lc, lo_, lev)
        grp, o, bo, data, st = wire.step_stream(w)
        t2 = time.perf_counter()
        if r >= 2:
            times_a.append(t1 - t0)
            times.append(t2 - t1)
    assert st.messages == n_msg and st.dropped_messages == 0 and st_a.messages == n_msg
    # both streams from the wire decide like the same step fed as rows
    res_a = wa.step_sized(*ss)
    res = w.step_stream(grp, o, bo, data)
    w2 = hq.Worker(d.device, nv, on_device=True, commit_advance=True)
    w2.add_groups(g, m)
    ref = w2.step(np.arange(G, dtype=np.uint32), off, ev)
    same = all(np.array_equal(x.get("committed_advance"), ref.get("committed_advance"))
               for x in (res, res_a))
    same = same and np.array_equal(res["ready"], ref["ready"]) and np.array_equal(
        hq.merge_ready(res_a, cids, g["committed"]), ref["ready"])
    for x in (w, w2, wa, wire, wire_a, pin):
        x.close()
    t, ta = float(np.median(times)), float(np.median(times_a))
    return {
        "workload": f"wire: the received messages of one steady-state step of {G} leader groups "
                    f"(3 voters), {n_msg} raftpb.Message in {len(bufs)} MessageBatch "
                    f"({n_bytes} bytes) + the local ReadIndex / proposals, decoded and assembled "
                    f"into the worker's sized stream (hq_wire_attach: handles resolved as the "
                    f"batches decode; hq_wire_step_sized), one host thread",
        "unit": "messages/s", "value": n_msg / ta, "ms_per_step": ta * 1e3,
        "ns_per_message": ta / n_msg * 1e9, "wire_mb_per_s": n_bytes / ta / 1e6,
        "stream_bytes_per_message": int(ss[3].nbytes) / n_msg,
        "first_appearance_form": {"ns_per_message": t / n_msg * 1e9,
                                  "api": "hq_wire_step_stream (clusters in order of first "
                                         "appearance, prefix arrays)"},
        "decisions_equal_rows_path": bool(same),
        "commits": int((res_a["committed_advance"] != 0).sum()),
    }


def run_wire_step_leg(d: Dist, G=1 << 20, steps=6, name="step5", with_cpu=True):
    """The device step fed from the wire at step size: every step's received messages of G
    leader groups (BENCH step5's membership: 4 full members, a witness, 2 observers: 12 messages
    per group) arrive as MessageBatch bytes (one batch per message type and sending node, per
    step worker; marshalled outside the timed region, hq_wire_encode_batch), W = 1 and 16 step
    workers each with its own hq_wire attached to its worker. A step: on each worker's own thread
    hq_wire_reset + hq_wire_add_batch of its batches + hq_wire_add_locals (its nodes' ReadIndex
    and proposals) + hq_wire_step_sized straight into its pinned receive buffers (2-byte size
    words); then the W workers' device step (hq_worker_step_jobs: ReadyToRead slots, advance
    column). Pipelined as a host would run it: while the device takes step s the workers decode
    step s + 1 into their other buffers. Every step's commits and ReadyToReads (order included)
    match the CPU replay of the same rows (oracle/qref_step.c)."""
    from concurrent.futures import ThreadPoolExecutor

    from dragonboat_amd import hipquorum as hq

    roles = STEP_ROLES[name]
    nv, nm = sum(r != "observer" for r in roles), len(roles)
    rng = _shard_of(d, G)
    g, m, cids = step_groups(hq, G, rng.cid_base, rng.cid_stride, roles)
    dep = 0x5EED
    Ws = (1, 16)
    pin = hq.Context(d.device)
    nsteps = steps + STEP_WARM

    # every step's arrivals per W (the rows advanced in place, StepRows; outside the timed
    # region), and the CPU replay of the same rows (its digests are the parity reference)
    rows = StepRows(hq, G, roles)
    n_events, n_msg = len(rows.ev), int((rows.ev["kind"] == hq.EV_MESSAGE).sum())
    arrivals = {W: [] for W in Ws}
    cpu = None
    if with_cpu and d.rank == 0 and d.world == 1:
        from oracle import qref

        _, counts = cpu_thread_counts()
        nt = 16 if 16 in counts else max(counts)
        rb = qref.StepBatch(g, m)
        cpu = {"threads": nt, "digests": [], "t": []}
        prev = int(g["committed"].sum(dtype=np.uint64))
    for s in range(nsteps + 1):
        rows.set(s)
        if cpu is not None and s < nsteps:
            t0 = time.perf_counter()
            tot = rb.step(rows.groups, rows.offsets, rows.ev, nthreads=cpu["threads"])
            cpu["t"].append(time.perf_counter() - t0)
            cpu["digests"].append((tot["commits"], tot["ready"],
                                   (tot["committed_sum"] - prev) & ((1 << 64) - 1),
                                   tot["ready_digest"], tot["commit_digest"],
                                   tot["ready_order_digest"]))
            prev = tot["committed_sum"]
        for W in Ws:
            bounds = [G * i // W for i in range(W + 1)]
            arrivals[W].append(_wire_arrivals(hq, rows.ev, rows.offsets, cids, roles, bounds, dep))
    if cpu is not None:
        rb.close()
        cpu["events_per_s"] = n_events * steps / sum(cpu["t"][STEP_WARM:])
    ev0 = int(rows.offsets[-1])
    out = {}
    for W in Ws:
        bounds = [G * i // W for i in range(W + 1)]
        workers, wires, bufs = [], [], []
        for i in range(W):
            wk = hq.Worker(d.device, nv, on_device=True, commit_column=True, commit_advance=True,
                           ready_compact=True, ready_slots=True)
            wk.add_groups(g[bounds[i]:bounds[i + 1]], m[nm * bounds[i]:nm * bounds[i + 1]])
            wr = hq.Wire(dep)
            wr.attach(wk)
            n_i = bounds[i + 1] - bounds[i]
            ev_i = int(rows.offsets[bounds[i + 1]] - rows.offsets[bounds[i]])
            bufs.append([(pin.pinned(ev_i * 5 + 4096, np.uint8), pin.pinned(n_i, np.uint16))
                         for _ in range(2)])
            workers.append(wk)
            wires.append(wr)
        pool = ThreadPoolExecutor(W + 1)
        mirror = CommitMirror(cids, g["committed"], bounds)

        def decode(i, s, slot):
            """Worker i's thread: step s's arrivals into its pinned buffers; (stream, seconds)."""
            t0 = time.perf_counter()
            wr = wires[i]
            wr.reset()
            batches, (lc, lo_, lev) = arrivals[W][s][i]
            for b in batches:
                wr.add_batch_at(b.ctypes.data, len(b))
            wr.add_locals(lc, lo_, lev)
            ss, _ = wr.step_sized(*bufs[i][slot])
            return ss, time.perf_counter() - t0

        def decode_all(s, slot):
            t0 = time.perf_counter()
            rs = list(pool.map(lambda i: decode(i, s, slot), range(W)))
            return [x for x, _ in rs], max(t for _, t in rs), time.perf_counter() - t0

        def device(streams):
            j = hq.StepJobs(list(zip(workers, streams)))
            t0 = time.perf_counter()
            j.execute()
            return j, time.perf_counter() - t0

        checks, t_e2e, t_dec, t_dev = [], [], [], []
        streams, _, _ = decode_all(0, 0)
        for s in range(nsteps):
            slot = s % 2
            t0 = time.perf_counter()
            fut = pool.submit(device, streams)           # step s on the device
            nxt, dec_max, dec_wall = decode_all(s + 1, 1 - slot)   # step s + 1 from the wire
            j, dt_dev = fut.result()
            dt = time.perf_counter() - t0
            checks.append(mirror.step(j.results(copy=False)))
            streams = nxt
            if s >= STEP_WARM:
                t_e2e.append(dt)
                t_dec.append(dec_wall)
                t_dev.append(dt_dev)
        pool.shutdown()
        for x in workers + wires:
            x.close()
        arrivals[W] = None
        parity = cpu is not None and checks == cpu["digests"]
        out[f"w{W}"] = {
            "events_per_s": n_events / float(np.median(t_e2e)),
            "latency_ms": _latency(t_e2e),
            "decode_ms_p50": float(np.median(t_dec)) * 1e3,
            "device_ms_p50": float(np.median(t_dev)) * 1e3,
            "decode_ns_per_message_per_thread": float(np.median(t_dec)) * W / n_msg * 1e9,
            "parity_committed": bool(parity) if cpu is not None else None,
        }
    pin.close()
    rec = {
        "workload": f"wire_step: {name}'s step of {G} leader groups from MessageBatch bytes "
                    f"({n_msg} messages + {n_events - n_msg} local events per step), decoded on "
                    f"each step worker's thread straight into its sized stream, then the device "
                    f"step; decode of step s + 1 overlapped with the device's step s; {steps} "
                    f"timed steps",
        "unit": "events/s", "value": out["w16"]["events_per_s"],
        "events_per_step": n_events, "messages_per_step": n_msg,
        "end_to_end": {k: v["events_per_s"] for k, v in out.items()}, "modes": out,
    }
    if cpu is not None:
        rec["cpu_replay"] = {"threads": cpu["threads"], "events_per_s": cpu["events_per_s"],
                             "sample": "the same rows of the same steps replayed event by event "
                                       "(oracle/qref_step.c)"}
        rec["vs_cpu_replay_end_to_end"] = {k: v["events_per_s"] / cpu["events_per_s"]
                                           for k, v in out.items()}
        rec["parity_committed"] = all(v["parity_committed"] for v in out.values())
    return rec


def run_share_leg(d: Dist, steps=20, step_steps=8, variants=None):
    """One GPU shared by three of the path's kernels, in one process: the persistent commit engine
    (hq_engine, post-as-ready windows of `steps` c3mtl steps, BASELINE config 3), the fused
    ReadIndex + vote + CheckQuorum plane pass (c4pq, 16 M x 7, back-to-back launches on its own
    context) and a device step worker (step5, 1 M groups, sized stream with ReadyToRead slots) —
    what a node's 16 step workers run at once (execengine.go:675-690, 860-882). Each is timed
    alone and then all three together (each on its own thread and stream, the engine and the
    plane pass looping until the step worker's steps are done), for each engine policy in
    `variants`: (max_workgroups, idle_us) — the full grid or a capped one, the 20 ms idle exit or
    a short one. Every output of the shared run equals the solo run's: the engine's batches
    (against a launch of the same batch), the plane pass's outputs on a freshly packed set, the
    step worker's per-step digests."""
    import threading

    from dragonboat_amd import hipquorum as hq
    from dragonboat_amd import shard

    w = WORKLOADS["c3mtl"]
    variants = variants or [(0, 20000), (0, 500), (-2, 500)]
    ctx_e, ctx_q = hq.Context(d.device), hq.Context(d.device)
    sets, per_set = build_sets(ctx_e, hq, shard, w, d)
    nsets = len(sets)
    lay = hq.HQ_LAYOUT_TILES_LEADER
    arr1 = [hq.commit_batch_array([batch_args(sets[i % nsets][0])]) for i in range(nsets)]
    # c4pq: rotating plane sets (as run_kernel_leg), one more kept for the equality check
    G4, n4, T = 16 << 20, 7, hq.HQ_PLANE_TILE_GROUPS
    pb, ab = hq.plane_tiles(G4) * 3 * T, hq.cq_plane_bytes(G4, 8)

    def plane_set(k):
        arrs = [ctx_q.empty(G4, np.uint8) for _ in range(4)]
        ctx_q.synth_bitmaps_dev(hq.synth_spec(SEED_BASE + 3 + (k << 40), G4, n4), *arrs)
        pl, apl = ctx_q.empty(pb, np.uint8), ctx_q.empty(ab, np.uint8)
        ctx_q.tile_planes_dev(G4, *arrs, 0, pl)
        ctx_q.synth_bitmaps_dev(hq.synth_spec(SEED_BASE + 5 + (k << 40), G4, n4), arrs[0])
        ctx_q.tile_cq_planes_dev(G4, arrs[0], None, 8, 0, apl)
        ctx_q.sync()
        act = arrs[0]
        for a in arrs[1:]:
            ctx_q.free(a)
        return [pl, apl, ctx_q.empty(hq.words64(G4), np.uint64), ctx_q.empty(hq.words32(G4), np.uint64),
                ctx_q.empty(hq.words64(G4), np.uint64), act]
    qsets = [plane_set(k) for k in range(4)]

    def q_repack(x):
        ctx_q.tile_cq_planes_dev(G4, x[5], None, 8, 0, x[1])

    def q_outputs(x):
        ctx_q.sync()
        return [ctx_q.download(y) for y in x[2:5]]
    # the step worker: step5's groups, every step's sized stream pre-encoded into pinned memory
    roles = STEP_ROLES["step5"]
    Gs = 1 << 20
    rng = _shard_of(d, Gs)
    g, m, cids = step_groups(hq, Gs, rng.cid_base, rng.cid_stride, roles)
    nv = sum(r != "observer" for r in roles)
    pin = hq.Context(d.device)
    rows = StepRows(hq, Gs, roles)
    streams = []
    for s_ in range(step_steps):
        rows.set(s_)
        data, sz = hq.encode_events_sized(rows.offsets, rows.ev)
        pd, ps = pin.pinned(len(data), np.uint8), pin.pinned(Gs, np.uint16)
        pd[:], ps[:] = data, hq.sizes16_of(sz)
        streams.append(hq.SizedStream(None, ps, len(rows.ev), pd))

    def step_run(stop=None):
        """step_steps steps of a fresh worker: (ms per step, digests)."""
        wk = hq.Worker(d.device, nv, on_device=True, commit_column=True, commit_advance=True,
                       ready_compact=True, ready_slots=True)
        wk.add_groups(g, m)
        mir = CommitMirror(cids, g["committed"], [0, Gs])
        ts, dg = [], []
        for ss in streams:
            j = hq.StepJobs([(wk, ss)])
            t0 = time.perf_counter()
            j.execute()
            ts.append(time.perf_counter() - t0)
            dg.append(mir.step(j.results(copy=False)))
        wk.close()
        if stop is not None:
            stop.set()
        return float(np.median(ts)) * 1e3, dg

    def engine_run(eng, stop=None, windows=3):
        """post-as-ready windows (one post per step, the drain's STOP): us per step (median)."""
        out, k = [], 0
        while True:
            t0 = time.perf_counter()
            for i in range(steps):
                eng.post(arr1[(k * steps + i) % nsets])
            eng.drain()
            out.append((time.perf_counter() - t0) / steps * 1e6)
            k += 1
            if (stop is None and k >= windows) or (stop is not None and stop.is_set()):
                return float(np.median(out)), k

    def q_run(stop=None, launches=100):
        """back-to-back plane passes: us per launch, launches."""
        k, t0 = 0, time.perf_counter()
        while True:
            for _ in range(10):
                ctx_q.readindex_vote_cq_planes_dev(G4, *qsets[k % 3][:5])
                k += 1
            ctx_q.sync()
            if (stop is None and k >= launches) or (stop is not None and stop.is_set()):
                return (time.perf_counter() - t0) / k * 1e6, k

    # solo: the plane pass and the step worker; the engine per policy
    q_run(launches=20)
    q_solo, _ = q_run()
    q_repack(qsets[3])
    ctx_q.readindex_vote_cq_planes_dev(G4, *qsets[3][:5])
    q_ref = q_outputs(qsets[3])
    st_solo, st_dg = step_run()
    # the engine's decisions of set 0 against a launch of the same batch
    b0 = sets[0][0]
    ctx_e.commit_dev(batch_args(b0))
    ctx_e.sync()
    e_ref = [ctx_e.download(x) for x in (b0.committed_out, b0.changed, b0.fallback)]
    out = {"solo": {"c4pq_us_per_launch": q_solo, "step5_ms_per_step": st_solo}, "policies": []}
    info = None
    for cap, idle in variants:
        eng0 = hq.Engine(ctx_e, w["n"], w["form"], lay, ring_len=16)
        grid = eng0.info().grid
        eng0.close()
        mw = grid // -cap if cap < 0 else cap
        eng = hq.Engine(ctx_e, w["n"], w["form"], lay, ring_len=16, idle_us=idle, max_workgroups=mw)
        engine_run(eng, windows=1)                       # (warm)
        e_solo, _ = engine_run(eng)
        stop = threading.Event()
        res = {}
        th = [threading.Thread(target=lambda: res.__setitem__("e", engine_run(eng, stop))),
              threading.Thread(target=lambda: res.__setitem__("q", q_run(stop)))]
        for t in th:
            t.start()
        st_shared, dg = step_run(stop)
        for t in th:
            t.join()
        # outputs of the shared run: the engine's set 0 (poisoned, decided by the engine after
        # the shared phase ran through it), a freshly packed plane set, the step digests
        for x in (b0.committed_out, b0.changed, b0.fallback):
            ctx_e.memset(x, 0xA5)
        ctx_e.sync()
        eng.post(arr1[0])
        eng.drain()
        e_out = [ctx_e.download(x) for x in (b0.committed_out, b0.changed, b0.fallback)]
        q_repack(qsets[3])
        ctx_q.readindex_vote_cq_planes_dev(G4, *qsets[3][:5])
        q_out = q_outputs(qsets[3])
        info = eng.info()
        eng.close()
        out["policies"].append({
            "engine_max_workgroups": mw or grid, "engine_grid": grid, "engine_idle_us": idle,
            "alone": {"engine_us_per_step": e_solo},
            "together": {"engine_us_per_step": res["e"][0], "engine_windows": res["e"][1],
                         "c4pq_us_per_launch": res["q"][0], "c4pq_launches": res["q"][1],
                         "step5_ms_per_step": st_shared},
            "outputs_equal": {"engine": all(np.array_equal(a, b) for a, b in zip(e_out, e_ref)),
                              "c4pq": all(np.array_equal(a, b) for a, b in zip(q_out, q_ref)),
                              "step5": dg == st_dg},
        })
    for c in (ctx_e, ctx_q, pin):
        c.close()
    return {
        "workload": f"share: the commit engine (c3mtl, {steps}-step post-as-ready windows), the "
                    f"c4pq plane pass (16 M x 7, back to back) and a step5 device step worker "
                    f"(1 M groups, {step_steps} steps) on one GPU, alone and together, per engine "
                    f"policy (max_workgroups, idle_us)",
        "unit": "us", "value": None, **out,
    }


# ----------------------------------------------------------------------------- CPU leg --------
def full_size_parity(w, set0, nthreads):
    """The GPU's decisions of batch set 0 (every voter-count bucket of the step, at the
    workload's full size) against the oracle (oracle/qref.c, test infrastructure) on the same
    generated inputs: committed', changed and fallback bit for bit. Lag workloads are unpacked
    with the oracle-side lastIndex (committed' = lastIndex - cout_lag for decided groups,
    hq_unpack_lags) and compared with the oracle's u64 decision."""
    from oracle import qref

    t0 = time.perf_counter()
    res = {"groups": 0, "buckets": [], "equal": True}
    for b in set0:
        s = qref.spec(SEED_BASE + w["cfg"], b["count"], b["n"], cid_base=b["cid_base"],
                      cid_stride=b["cid_stride"])
        inp = qref.CommitInputs(s)
        want_out, want_chg, want_fb, rc = inp.run(w["form"], False, nthreads=nthreads)
        out, chg, fb = b["out"]
        if w["kind"] == "lag":
            fbit = np.unpackbits(fb.view(np.uint8), bitorder="little")[:b["count"]].astype(bool)
            out = np.where(fbit, inp.committed_in,
                           inp.last_index - out.astype(np.int64).astype(np.uint64))
        eq = dict(committed=bool(np.array_equal(out, want_out)),
                  changed=bool(np.array_equal(chg, want_chg)),
                  fallback=bool(np.array_equal(fb, want_fb)), oracle_rc=int(rc))
        ok = eq["committed"] and eq["changed"] and eq["fallback"] and rc == 0
        res["buckets"].append(dict(voters=b["n"], groups=b["count"], **eq))
        res["groups"] += b["count"]
        res["equal"] &= ok
    res["check_s"] = time.perf_counter() - t0
    return res


def host_cores():
    """(CPUs the host shows, CPUs this process may run on, the cgroup CPU quota or None). On the
    GPU box the first two show the whole machine while the quota is the box's share."""
    visible = os.cpu_count() or 1
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = visible
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    return visible, usable, quota


def cgroup_throttled_us():
    """CPU time (us) this process's cgroup has been throttled by its CPU quota so far (cgroup v2
    cpu.stat throttled_usec, v1 throttled_time), or None where it cannot be read. A box whose
    share of a large host is a quota of 16 CPUs stops every thread of the cgroup for the rest of
    a quota period once its threads have used the period's CPU time."""
    for path, key, scale in (("/sys/fs/cgroup/cpu.stat", "throttled_usec", 1.0),
                             ("/sys/fs/cgroup/cpu/cpu.stat", "throttled_time", 1e-3),
                             ("/sys/fs/cgroup/cpu,cpuacct/cpu.stat", "throttled_time", 1e-3)):
        try:
            for ln in open(path):
                k, v = ln.split()
                if k == key:
                    return int(v) * scale
        except (OSError, ValueError):
            continue
    return None


def encode_threads():
    """The producer's native encode threads: the usable CPUs (capped by the cgroup quota) less
    two (the step's own thread and the GPU runtime's), at most 16 — so that the encodes, the step
    and the runtime never ask for more CPU than the quota gives (BENCH_HQ_ENCODE_THREADS
    overrides)."""
    v = os.environ.get("BENCH_HQ_ENCODE_THREADS")
    if v:
        return max(1, int(v))
    return max(1, min(16, cpu_thread_counts()[0] - 2))


def cpu_thread_counts():
    """(all usable cores, the thread counts the CPU legs run at: all cores, 16 = the reference's
    StepEngineWorkerCount (internal/settings/hard.go:35), 1)."""
    _, usable, quota = host_cores()
    allc = min(usable, quota) if quota else usable
    return allc, sorted({allc, min(16, allc), 1}, reverse=True)


def cpu_baseline(w, budget_s=9.0, gpu_set0=None):
    """The oracle (C restatement of the reference path) on a bounded sample of the workload, on
    all usable host cores, on 16 threads and on 1. gpu_set0: the GPU's decisions of batch set 0
    (run_gpu), compared bit for bit with the oracle's on the same inputs at full size
    (full_size_parity)."""
    from oracle import qref

    host_threads, counts = cpu_thread_counts()
    G = min(w["G"], 1 << 20)
    s = qref.spec(SEED_BASE + w["cfg"], G, w["n"])
    out = {}
    if w["kind"] in ("commit", "lag"):   # the oracle decides the u64 layout
        inp = qref.CommitInputs(s)

        def one(nt):
            inp.run(w["form"], False, nthreads=nt)
    else:
        inp = qref.BitmapInputs(s)

        def one(nt):
            qref.readindex_batch(inp.ack, inp.n_voting, 0, nthreads=nt)
            qref.vote_batch(inp.granted, inp.rejected, inp.n_voting, 0, nthreads=nt)
    for nt in counts:
        passes, t0 = 0, time.perf_counter()
        while True:
            one(nt)
            passes += 1
            dt = time.perf_counter() - t0
            if dt >= budget_s / len(counts):
                break
        out[nt] = (passes * G * decisions_per_group(w) / dt, passes, dt)
    best = max(counts, key=lambda nt: out[nt][0])
    rate, passes, dt = out[best]
    parity = full_size_parity(w, gpu_set0, host_threads) if gpu_set0 else None
    # BASELINE config C1: the reference's own CPU case, one group x 3 voters, tryCommit per step
    T = 4 << 20
    match, last = qref.c1_stream(SEED_BASE, T, 1000, 1005)
    t0 = time.perf_counter()
    qref.c1_run(match, last, 1003, 1000)
    c1_s = time.perf_counter() - t0
    visible, usable, quota = host_cores()
    return {
        "value": rate, "unit": "decisions/s", "cores": best, "kind": "port",
        "sample": (f"{G} groups of the same workload and generator, {passes} passes in {dt:.1f} s "
                   f"on {best} host threads (oracle/qref.c -O3, C restatement of the reference "
                   f"Go path; Go toolchain unavailable)"),
        "by_threads": {str(nt): out[nt][0] for nt in counts},
        "host_cpus": {"visible": visible, "usable": usable, "cgroup_quota": quota},
        "c1_single_group_ns_per_trycommit": c1_s / T * 1e9,
        "parity_full_size": parity,
    }


def pmc_traffic(workload):
    """HBM bytes per launch from the committed rocprofv3 PMC summary of this workload (the
    (2 x FETCH_SIZE + WRITE_SIZE) x 1 KiB gfx950 reading, MI355X_MICROARCH.md "HBM"), with the
    profile it comes from; None if no PMC pass of this workload is committed."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        e = json.load(open(p))[workload]
        return e["hbm_bytes_per_launch"], e.get("source")
    except (OSError, KeyError, ValueError):
        return None, None


def extra_record(name, we, re_, parity=None):
    rec = {
        "workload": f"{name}: {we['desc']}",
        "value": re_["decisions"] / re_["elapsed"], "unit": "decisions/s",
        "kernel_avg_us": re_["avg_kernel_s"] * 1e6,
        "launches_per_step": re_["launches_per_step"],
        "roofline_achieved_gbs": re_["achieved_node_gbs"],
        "roofline_frac": re_["achieved_node_gbs"] / (HBM_PEAK_GBS * re_["world"]),
        "algorithmic_bytes_per_launch": re_["bytes_per_launch"],
    }
    if parity is not None:
        rec["parity_full_size"] = parity
    return rec


def same_decisions(a, b):
    """Two runs' set-0 decisions (committed', changed, fallback of every bucket) are equal."""
    if not a or not b or len(a) != len(b):
        return None
    return all(all(np.array_equal(x, y) for x, y in zip(p["out"], q["out"]))
               for p, q in zip(a, b))


EXTRAS_MULTI = "c5tl,c5v5tl,c4p,cqp,c4pq,rimt,rimtc,ingo"


def rank_parity(w, r, d, no_cpu):
    """Every rank checks its own shard's set 0 at full size against the oracle (the C
    restatement, test infrastructure) on its share of the host cores, at any N: r["parity"] is
    this rank's full record, r["parity_by_rank"] every rank's verdict in rank order (it travels
    with per_gpu in the final line)."""
    host_threads, _ = cpu_thread_counts()
    r["parity"] = None
    if not no_cpu and r.get("set0"):
        r["parity"] = full_size_parity(w, r["set0"], max(1, host_threads // d.world))
    mine = None if r["parity"] is None else {"equal": r["parity"]["equal"],
                                             "groups": r["parity"]["groups"]}
    r["parity_by_rank"] = d.gather_obj(mine)
    return r


def run_rank(args, d, progress):
    """Everything one rank measures: the headline, the extra legs, and (rank 0 at N = 1) the CPU
    baseline. Every rank runs the same legs in the same order (their collectives pair up)."""
    w = WORKLOADS[args.workload]
    use_engine = args.mode in ("engine", "fused") and engine_ok(w)
    progress(f"headline {args.workload}: {args.windows if use_engine else 1} x {args.steps} steps"
             f" ({args.mode if use_engine else 'launch per step'}), {args.warmup} warmup")
    from dragonboat_amd import hipquorum as hq

    devices = d.gather_obj({"rank": d.rank, "device": d.device,
                            "pci_bus_id": hq.device_pci_bus_id(d.device)})
    # ranks sharing one GPU (a rehearsal of N ranks on fewer devices) split its CUs between their
    # engines, so that every engine's grid is resident at once
    per_device = max(1, d.world // max(1, len({x["pci_bus_id"] or x["device"] for x in devices})))
    r = (run_engine(w, args.steps, args.warmup, d, windows=args.windows, headline=args.mode,
                    share=per_device)
         if use_engine else run_gpu(w, args.steps, args.warmup, d))
    r["world"] = d.world
    host_threads, _ = cpu_thread_counts()
    progress("full-size parity of every rank's set 0")
    rank_parity(w, r, d, args.no_cpu)
    oracle_here = d.rank == 0 and d.world == 1 and not args.no_cpu
    extra_names = args.extra if args.extra is not None else (
        DEFAULT_EXTRAS if d.world == 1 else EXTRAS_MULTI)
    records, extra_runs = [], {}
    for name in [x for x in extra_names.split(",") if x and x != args.workload]:
        we = WORKLOADS.get(name)
        if we is not None and we.get("mixed") and d.world % 3 == 0:
            # voter-count buckets need gcd(3, world) == 1 (shard.rank_bucket); same on every rank
            records.append({"name": name, "skipped": "world size divisible by 3"})
            continue
        progress(f"extra {name}")
        try:
            if name == "e2e":
                rec = run_e2e(max(100, args.steps // 4), 5, d)   # >= 30 ms timed per variant
            elif name == "wire":
                rec = run_wire_leg(d)
            elif name == "share":
                rec = run_share_leg(d)
            elif name == "wire_step":
                rec = run_wire_step_leg(d, G=args.step_groups, steps=min(args.step_steps, 8),
                                        with_cpu=not args.no_cpu)
            elif name in STEP_ROLES:
                rec = run_step_leg(d, G=args.step_groups, steps=args.step_steps,
                                   with_cpu=not args.no_cpu, name=name)
            elif name in ("rim", "rimt", "rimtc", "cq", "cqp", "c4pq", "ing", "ingo", "ingu",
                          "inga"):
                pt = 0 if args.no_cpu or args.no_extra_parity else max(1, host_threads // d.world)
                rec = run_kernel_leg(name, max(50, args.steps // 4), max(5, args.warmup // 4), d,
                                     parity_threads=pt)
            elif name == "sweep":
                rec = run_size_sweep(args.workload, max(50, args.steps // 4),
                                     max(5, args.warmup // 4), d)
            elif name.startswith("w") and name[1:].isdigit():
                rec = run_concurrent(w, args.steps, args.warmup, d, W=int(name[1:]))
            else:
                re_ = run_gpu(we, max(50, args.steps // 4), max(5, args.warmup // 4), d)
                re_["world"] = d.world
                par = None
                if oracle_here and re_.get("set0") and not args.no_extra_parity:
                    par = full_size_parity(we, re_["set0"], host_threads)
                rec = extra_record(name, we, re_, par)
                extra_runs[name] = re_
        except Exception as e:   # an extra leg never costs the headline line
            log(f"extra leg {name} failed: {e!r}")
            rec = {"error": repr(e)}
        rec = dict(name=name, **rec)
        records.append(rec)
        if d.rank == 0:     # each leg's record as it lands (the final line only summarises it)
            log("extra " + json.dumps(rec)[:4000])
    cpu = None
    if d.rank == 0 and not args.no_cpu:    # once per run, on all usable host cores (any N)
        progress("cpu baseline")
        cpu = cpu_baseline(w)
        cpu["parity_full_size"] = r["parity"]
    # the term check of the same groups in its other exact forms (the ring gathers the north
    # star names, the mask the headline streams): rate and whether every decision is identical
    forms = []
    for name in SAME_DATA_FORMS.get(args.workload, ()):
        if name in extra_runs:
            re_ = extra_runs[name]
            forms.append({
                "workload": name, "form": {0: "term_start", 1: "ring_u64", 2: "term_mask",
                                           3: "ring_u32"}[WORKLOADS[name]["form"]]
                + (" tiles" if WORKLOADS[name].get("tiled") else ""),
                "value": re_["decisions"] / re_["elapsed"],
                "frac": re_["achieved_node_gbs"] / (HBM_PEAK_GBS * d.world),
                "equal": same_decisions(r.get("set0"), re_.get("set0")),
            })
    r.pop("set0", None)
    return dict(r=r, devices=devices, records=records, cpu=cpu, forms=forms)


def _short(rec):
    """The few numbers of one extra record that the final line carries."""
    if "error" in rec or "skipped" in rec:
        return {k: str(rec.get(k))[:120] for k in ("error", "skipped") if k in rec}
    out = {}
    # (kernel times, units and the rest stay in the detail file: the line must stay < 8 KB)
    for k in ("value", "roofline_frac", "aggregate_frac_of_peak", "fit_t0_us",
              "fit_stream_frac_of_peak"):
        v = rec.get(k)
        if v is not None:
            out[k] = round(v, 4) if isinstance(v, float) and abs(v) < 1e4 else (
                float(f"{v:.4g}") if isinstance(v, float) else v)
    par = rec.get("parity_full_size")
    if isinstance(par, dict):
        out["parity_equal"] = par.get("equal")
    lk = rec.get("link")
    if isinstance(lk, dict):
        out["link"] = {k: lk.get(k) for k in ("frac", "frac_serial", "both_GBps", "gpu_ms")}
        if lk.get("probe"):
            out["link"]["peak_both_GBps"] = lk["probe"].get("both_GBps")
    lat = rec.get("latency_ms")
    if isinstance(lat, dict):          # per mode [p50, p99] (ms)
        out["lat_ms"] = {k: [round(v["p50"], 3), round(v["p99"], 3)] for k, v in lat.items() if v}
    for k in (("end_to_end", "vs_cpu_replay_end_to_end", "parity_committed") if lat else
              ("end_to_end", "device_only", "vs_cpu_replay_end_to_end", "parity_committed")):
        if k in rec:
            v = rec[k]
            if isinstance(v, dict):
                v = {a: (float(f"{b:.4g}") if isinstance(b, float) else b)
                     for a, b in v.items() if not isinstance(b, (dict, list))}
            out[k] = v
    return out


def report(args, d, res, launcher):
    """Rank 0: the full record to a side file, ONE compact JSON line (<= 8 KB) to stdout."""
    w = WORKLOADS[args.workload]
    r = res["r"]
    traffic, traffic_src = pmc_traffic(args.workload)
    peak = HBM_PEAK_GBS * d.world
    achieved = r["achieved_node_gbs"]
    devs = res["devices"]
    line = {
        "metric": "quorum-commit decisions/sec (whole node) + % HBM roofline at 1/2/4/8 GPUs",
        "value": r["decisions"] / r["elapsed"],
        "unit": "decisions/s",
        "n_gpus": d.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": r["elapsed"] / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": f"synthetic: device-generated splitmix64 batches, {r['nsets']} distinct per GPU "
                f"rotated (>= 1.1 GiB); timed steps start at batch {r['first_timed_set']}"
                + (f"; {r['windows']} timed windows of {args.steps} steps, the median window "
                   f"reported (every window in "
                   f"{'fused_window' if r.get('headline_mode') == 'fused' else 'engine'}"
                   f".window_ms)" if r.get("windows") else ""),
        "config": {
            "workload": args.workload,
            "desc": w["desc"],
            "groups_per_gpu": w["G"], "voters": w["n"],
            "form": ({0: "term_start", 1: "ring", 2: "term_mask", 3: "ring32"}[w["form"]]
                     + ("_lag" if w["kind"] == "lag" else ""))
            if w["kind"] in ("commit", "lag") else "bitmaps",
            "layout": ("tiles_leader" if w.get("lead") else "tiles") if w.get("tiled")
            else "columns",
            "global_groups_per_step": groups_per_step(w) * d.world,
            **({"headline_mode": r["headline_mode"], "steps_per_window": args.steps,
                "groups_per_launch": (r["fused_window"]["groups_per_launch"]
                                      if r["headline_mode"] == "fused" else
                                      "one resident launch per window")}
               if r.get("headline_mode") else {}),
            "parallelism": f"shard{d.world} (clusterID % {d.world}, partition.go:38)",
            "launcher": launcher,
            "devices_seen": len({x["pci_bus_id"] or x["device"] for x in devs}),
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": peak, "unit": "GB/s",
            "frac": achieved / peak, "traffic": traffic,
            "traffic_source": traffic_src,
            "kernel_avg_us": r["avg_kernel_s"] * 1e6,
            "algorithmic_bytes_per_launch": r["bytes_per_launch"],
            "kernel_time": ("HIP events around the fused launch(es) of the median window, / "
                            "steps" if r.get("headline_mode") == "fused" else
                            "HIP events around the resident engine launch of the median "
                            "window (steps posted one by one, then STOP), / steps" if r.get("engine") else
                            "HIP events on the launch stream around the timed launches "
                            "(back to back), / launches"),
            "achieved_scope": f"sum over {d.world} GPU(s) of bytes per launch / kernel time",
        },
        "per_gpu": [{"rank": i, "device": devs[i]["device"], "pci": devs[i]["pci_bus_id"],
                     "value": float(f"{v:.5g}"), "kernel_us": round(k, 3),
                     "frac": round(a / HBM_PEAK_GBS, 4),
                     "parity_equal": ((r.get("parity_by_rank") or [None] * d.world)[i]
                                      or {}).get("equal")}
                    for i, (v, k, a) in enumerate(r["per_gpu"])],
        "cpu_baseline": res["cpu"],
        "term_check_forms_same_data": res["forms"],
    }
    if r.get("engine"):
        line["engine"] = r["engine"]
        line["launch_per_step"] = r["launch_per_step"]
        line["engine_signal"] = r["engine_signal"]
        line["fused_window"] = r["fused_window"]
    summary = {rec["name"]: _short(rec) for rec in res["records"]}
    detail = dict(line, result_gather=r.get("gather"), extra=res["records"])
    # (the modes' descriptions stay in the detail file; the line keeps their figures)
    for k in ("engine", "launch_per_step", "engine_signal", "fused_window"):
        if k in line:
            line[k] = {kk: v for kk, v in line[k].items() if kk != "mode"}
    path = args.detail_out
    try:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump(detail, f, indent=1)
        line["detail_file"] = os.path.relpath(os.path.abspath(path), ROOT)
    except OSError as e:
        log(f"detail file not written: {e!r}")
    line["extra"] = summary
    text = json.dumps(line, separators=(",", ":"))
    if len(text) > 8000:       # the driver parses this line: never let the summary break it
        # the step legs keep their p99 per mode and their replay ratios; the others their value
        # and roofline fraction
        line["extra"] = {k: ({kk: v[kk] for kk in ("value", "lat_ms", "vs_cpu_replay_end_to_end",
                                                     "parity_committed", "link") if kk in v}
                             if k in ("step", "step5") else
                             {kk: v.get(kk) for kk in ("value", "roofline_frac") if kk in v})
                         for k, v in summary.items()}
        text = json.dumps(line, separators=(",", ":"))
    if len(text) > 8000:
        line["extra"] = {k: {kk: v.get(kk) for kk in ("value", "roofline_frac") if kk in v}
                         for k, v in summary.items()}
        text = json.dumps(line, separators=(",", ":"))
    if len(text) > 8000:
        line.pop("extra")
        text = json.dumps(line, separators=(",", ":"))
    print(text, flush=True)


def main_threads(args, t_start):
    """--gpus N with no launcher: N host threads in this process, thread i opens its contexts on
    GPU i (i % visible GPUs when fewer are visible: a rehearsal), groups sharded clusterID % N."""
    from dragonboat_amd import hipquorum as hq

    ngpu = hq.device_count()
    if ngpu < 1:
        log("no GPU visible")
        sys.exit(1)
    if ngpu < args.gpus:
        log(f"--gpus {args.gpus} with {ngpu} GPU(s) visible: ranks share GPUs (rehearsal)")
    grp = ThreadGroup(args.gpus)
    ds = [ThreadDist(grp, i, ngpu) for i in range(args.gpus)]
    results, errors = [None] * args.gpus, []

    def progress(msg):
        log(f"[bench {time.perf_counter() - t_start:7.1f} s] {msg}")

    def body(i):
        try:
            results[i] = run_rank(args, ds[i], progress if i == 0 else (lambda m: None))
        except BaseException as e:    # one failed rank releases the others' barriers
            errors.append((i, e))
            grp.bar.abort()

    threads = [threading.Thread(target=body, args=(i,), name=f"rank{i}")
               for i in range(args.gpus)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errors:
        i, e = errors[0]
        raise RuntimeError(f"rank {i} failed") from e
    report(args, ds[0], results[0], f"threads: 1 process, {args.gpus} host threads, one hq_ctx "
                                    f"per GPU ({ngpu} visible)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--workload", default=HEADLINE, choices=sorted(WORKLOADS))
    ap.add_argument("--mode", default="fused", choices=("fused", "engine", "launch"),
                    help="headline commit steps: the co-resident step workers' batches fused "
                         "into launches of up to 32 (fused), the persistent engine (one resident "
                         "launch per window), or one launch per step; fused and engine apply to "
                         "uniform tiled term-start / mask workloads, others take launches. All "
                         "three are timed on the same windows and reported")
    ap.add_argument("--windows", type=int, default=3,
                    help="timed windows of --steps steps (engine mode); the median is reported")
    ap.add_argument("--step-groups", type=int, default=1 << 20,
                    help="groups per GPU of the step-worker legs (extras 'step', 'step5')")
    ap.add_argument("--step-steps", type=int, default=50,
                    help="timed steps of the step-worker legs")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extra-parity", action="store_true",
                    help="skip the full-size oracle check of the commit / lag extras")
    ap.add_argument("--extra", default=None,
                    help="comma list of extra legs ('' for none; default: all at N = 1, "
                         f"{EXTRAS_MULTI} at N > 1)")
    ap.add_argument("--detail-out", default=os.path.join(ROOT, "gpurun_out", "bench_detail.json"),
                    help="where the full record (every extra leg) is written")
    args = ap.parse_args()
    t_start = time.perf_counter()
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and world_env == 1:
        main_threads(args, t_start)
        return
    d = Dist()
    if args.gpus != d.world:
        log(f"--gpus {args.gpus} but WORLD_SIZE={d.world}: measuring WORLD_SIZE ranks")

    def progress(msg):          # one line per phase (a long run must keep writing)
        if d.rank == 0:
            log(f"[bench {time.perf_counter() - t_start:7.1f} s] {msg}")

    res = run_rank(args, d, progress)
    if d.rank == 0:
        report(args, d, res, "one process" if d.world == 1 else
               f"torch.distributed.run: {d.world} processes, {d.backend}")
    d.close()


if __name__ == "__main__":
    main()
