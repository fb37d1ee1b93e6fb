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
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

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
                  "rimt,cq,cqp,ing,ingo,ingu,w2,sweep,e2e,step,step5,wire")
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

    def close(self):
        if self.torch is not None:
            self.dist.destroy_process_group()


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


def run_kernel_leg(name, steps, warmup, d: Dist):
    """The remaining decision kernels, each on its own BASELINE-shaped batch, device-resident and
    rotated past the Infinity Cache like the commit legs:
      rim: general multi-ctx ReadIndex (k_ri_multi), 2M groups x 4 pending ctxs x 7 voters
      cq:  CheckQuorum (k_bits CHECKQ), 16M groups x 7 voters, active flags reset in place
      cqp: the same over active-flag planes (k_cq_planes)
      ing: match-delta ingest (k_ingest_match), 4M ReplicateResp deltas into a 4M x 3 table
      ingo: the same deltas in group order, the order a step worker emits them
      ingu: distinct (group, slot) keys in random order (HQ_INGEST_UNIQUE)"""
    from dragonboat_amd import hipquorum as hq

    ctx = hq.Context(d.device)
    r = np.random.default_rng(SEED_BASE + d.rank)
    if name in ("rim", "rimt"):
        G, K, n = 2 << 20, 4, 7
        # first-ack ordinals: ~70 % of (ctx, voter) pairs acked, in arrival order 1..K*n
        ordn = r.integers(1, K * n + 1, (K, n, G)).astype(np.uint16)
        ordn[r.random((K, n, G)) < 0.3] = 0xFFFF
        idx = (np.uint64(1 << 30) + np.arange(K, dtype=np.uint64)[:, None] * np.uint64(3)
               + r.integers(0, 1 << 20, G, dtype=np.uint64)[None, :])
        per = G * (2 * K * n + 8 * K + 8 * K + 2)      # ordinals + ctx index in; released out
        nsets = max(4, int(np.ceil(ROTATE_BYTES / per)))
        sets = [(ctx.upload(ordn.reshape(-1)), ctx.upload(idx.reshape(-1)),
                 ctx.empty(K * G, np.uint64), ctx.empty(G, np.uint8), ctx.empty(G, np.uint8))
                for _ in range(nsets)]
        if name == "rimt":     # the same inputs as 128-group tiles (one block per wave)
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
                ctx.readindex_multi_tiles_dev(G, K, n, t, 0, n, rel, cnt, batch_end=bend)
        else:
            def run(i):
                o, x, rel, cnt, bend = sets[i % nsets]
                ctx.readindex_multi_dev(G, K, n, o, x, None, None, n, rel, cnt, batch_end=bend)
        desc = (f"{name}: general multi-ctx ReadIndex release (suffix-min), {G} groups x {K} "
                f"pending ctxs x {n} voters" + (", 128-group tiles" if name == "rimt" else ""))
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
    else:   # ing / ingo: the device table in the headline layout (leader-row tiles)
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
        flags = {"ingo": hq.HQ_INGEST_GROUPED, "ingu": hq.HQ_INGEST_UNIQUE}.get(name, 0)

        def run(i):
            ctx.table_ingest_match_dev(ups[i % nsets], U, table, G, n, form, flags)
        desc = (f"{name}: ReplicateResp match-delta ingest (remote.tryUpdate) into a {G} x {n} "
                f"device table in the headline layout (leader-row tiles), {U} deltas "
                + {"ingo": "in group order (as a step worker emits them): runs reduced in "
                           "registers, plain read-modify-write, atomics only at wave edges "
                           "(HQ_INGEST_GROUPED)",
                   "ingu": "with distinct (group, slot) keys in random order: one plain "
                           "read-modify-write each (HQ_INGEST_UNIQUE)"}.get(
                       name, "in random order: one 64-bit atomic max each"))
        units, unit = U, "updates/s"
    elapsed, avg, launches = _timed(ctx, d, run, steps, warmup)
    ctx.close()
    return {
        "workload": desc, "value": d.sum(float(units * steps)) / elapsed, "unit": unit,
        "kernel_avg_us": avg * 1e6, "launches_per_step": launches / max(1, steps),
        "roofline_achieved_gbs": per / avg / 1e9, "roofline_frac": per / avg / 1e9 / HBM_PEAK_GBS,
        "algorithmic_bytes_per_launch": per,
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


def _run_workers(hq, d: Dist, G, W, steps, cpu_steps, roles, on_device=False, stream=False,
                 events=None):
    """W workers (one native thread each, own HIP stream) over G groups split into W contiguous
    partitions, stepping concurrently; returns (timed seconds, events, counter sums, committed
    of the first 4096 groups after the last step, ..., encode seconds). on_device:
    HQ_WORKER_ON_DEVICE workers, the step's input in pinned host memory (a step worker's receive
    buffers) so that it crosses PCIe at the link's rate. stream: the input is the event stream
    (hq_worker_step_stream), written by the producer — here hq_events_encode over the rows,
    outside the timed region and timed on its own (encode seconds). events(s): the full step s
    input (cached by the caller across modes)."""
    rng = _shard_of(d, G)
    g, m, cids = step_groups(hq, G, rng.cid_base, rng.cid_stride, roles)
    nm = len(roles)
    n_voting = sum(r != "observer" for r in roles)
    bounds = [G * i // W for i in range(W + 1)]
    workers = []
    for i in range(W):
        w = hq.Worker(d.device, n_voting, on_device=on_device, commit_column=stream == "sized",
                      commit_advance=stream == "sized")
        w.add_groups(g[bounds[i]:bounds[i + 1]], m[nm * bounds[i]:nm * bounds[i + 1]])
        workers.append(w)
    pin_ctx = hq.Context(d.device) if on_device else None
    pinned = [None] * W
    acc = dict(handle_ns=0, pass_ns=0, pack_ns=0, device_ns=0, apply_ns=0, gpu_passes=0,
               decisions=0)
    t_total, n_events, committed, t_enc, nb_total = 0.0, 0, None, 0.0, 0
    step_ms = []
    warm = STEP_WARM   # untimed: allocations, first touch, and the first step with commits
    for s in range(steps + warm):   # (its output lists size the pinned result buffers)
        full = events(s) if events else step_events(hq, G, s, roles)
        evs = [_partition(full, bounds[i], bounds[i + 1]) for i in range(W)]
        n_step = sum(len(e[2]) for e in evs)
        n_ev = [len(e[2]) for e in evs]
        if stream:
            t0 = time.perf_counter()
            enc = [hq.encode_events_sized(e[1], e[2]) if stream == "sized" else
                   hq.encode_events(e[1], e[2]) for e in evs]
            if s >= warm:
                t_enc += time.perf_counter() - t0
                nb_total += sum(len(data) for data, _ in enc)
            # sized: (groups, size words, bytes); else (groups, offsets, boffsets, bytes)
            evs = [(e[0], z, data) if stream == "sized" else (e[0], e[1], z, data)
                   for e, (data, z) in zip(evs, enc)]
        if pin_ctx is not None:      # copied into pinned buffers outside the timed region
            for i, e in enumerate(evs):
                if pinned[i] is None or any(p.size < x.size for p, x in zip(pinned[i], e)):
                    pinned[i] = tuple(pin_ctx.pinned(x.size + x.size // 4 + 1, x.dtype)
                                      for x in e)
                for dst, src in zip(pinned[i], e):
                    dst[:src.size] = src
            evs = [tuple(p[k][:e[k].size] for k in range(len(e))) for p, e in zip(pinned, evs)]
        if stream == "sized":   # every group in handle order: the handles stay implicit
            evs = [hq.SizedStream(None, e[1], ne, e[2]) for e, ne in zip(evs, n_ev)]
        # the W workers stepped at once on native threads (hq_worker_step_jobs), as W step-
        # worker goroutines each calling its own worker
        jobs = hq.StepJobs(list(zip(workers, evs)))
        t0 = time.perf_counter()
        res = jobs.run(copy=False)
        dt = time.perf_counter() - t0
        if s < warm:
            continue
        step_ms.append(round(dt * 1e3, 3))
        t_total += dt
        n_events += n_step
        for r in res:
            for k in acc:
                acc[k] += r[k]
    # the state after the last step, checked against the CPU replay of the same steps (read
    # after the timed steps: reading a device worker's state downloads all of it)
    committed = [int(workers[0].get_group(int(c))[0]["committed"])
                 for c in cids[:min(4096, bounds[1])]]
    for w in workers:
        w.close()
    if pin_ctx is not None:
        pin_ctx.close()
    acc["stream_bytes"] = nb_total
    acc["step_ms"] = step_ms
    return t_total, n_events, acc, committed, (g, m), t_enc


def _shard_of(d, G):
    from dragonboat_amd import shard

    return shard.rank_shard(d.rank, d.world, G)


def run_step_leg(d: Dist, G=1 << 20, steps=6, cpu_steps=3, with_cpu=True, name="step"):
    """The step worker end to end (hq_worker_step): host bookkeeping of every event plus the
    GPU passes, against the event-by-event C restatement of the reference (oracle, CPU) on the
    same events; the committed indexes of both must agree. Run with one worker (one step-worker
    thread), two (dragonboat's 16 step workers on an 8-GPU node: two per GPU) and T workers
    stepping concurrently (dragonboat runs 16 step workers, internal/settings/hard.go:36), next
    to the CPU replay on 1 and T threads."""
    from dragonboat_amd import hipquorum as hq

    assert cpu_steps <= steps
    T = min(16, os.cpu_count() or 1)
    roles = STEP_ROLES[name]
    nmsg = 2 * (len(roles) - 1)
    members = ", ".join(f"{roles.count(r)} {r}" for r in ("remote", "witness", "observer")
                        if roles.count(r))
    out = {
        "workload": f"{name}: hq_worker_step (device engine; host worker beside it) over {G} "
                    f"leader groups per GPU ({members}); per group "
                    f"and step {nmsg} messages ({nmsg // 2} ReplicateResp, {nmsg // 2} "
                    f"HeartbeatResp), 1 proposal, 1/4 local ReadIndex",
        "unit": "events/s",
    }
    committed = {}
    cache = {}

    def events(s):            # one generation per step index, shared by every mode
        if s not in cache:
            cache[s] = step_events(hq, G, s, roles)
        return cache[s]

    modes = {"device_sized": "device worker (HQ_WORKER_ON_DEVICE: every event on the GPU), "
                             "events as the event stream in the sized form (hq_worker_step_stream:"
                             " 4-byte per-group size words, scanned on the device), commits as a "
                             "column of 4-byte advances when > 1/4 of the groups commit "
                             "(HQ_WORKER_COMMIT_ADVANCE | _COLUMN)",
             "device_stream": "device worker, events as the event stream with the two 8-byte "
                              "prefix arrays (hq_worker_step_stream)",
             "device_rows": "device worker, events as 56-byte hq_event rows (hq_worker_step)",
             "host": "host worker (events on the host, decisions in GPU passes), rows"}
    all_modes = (("device_sized", 1), ("device_sized", 2), ("device_sized", T),
                 ("device_stream", 1), ("device_stream", T), ("device_rows", 1),
                 ("device_rows", T), ("host", 1), ("host", T))
    # with several ranks (a node's GPUs, each with its own share) only the device engine's modes
    # run: the comparison modes are host-bound and would share the node's cores
    for mode, W in all_modes if d.world == 1 else all_modes[:3]:
        if d.rank == 0:
            log(f"  step leg {name}: {mode}, {W} worker(s)")
        t, ne, acc, committed[mode], gm, t_enc = _run_workers(
            hq, d, G, W, steps, cpu_steps, roles, mode != "host",
            {"device_sized": "sized", "device_stream": True}.get(mode, False), events)
        elapsed = d.max(t)
        rec = {
            "workers": W,
            "mode": modes[mode],
            "value": d.sum(float(ne)) / elapsed,
            "decisions_per_s": d.sum(float(acc["decisions"])) / elapsed,
            "ms_per_step": elapsed / steps * 1e3,
            "step_ms": acc["step_ms"],
            # the copy-engine paths see occasional multi-ms idle gaps on these boxes:
            # the median step beside the mean
            "median_ms_per_step": float(np.median(acc["step_ms"])) if acc["step_ms"] else None,
            "gpu_passes_per_step": acc["gpu_passes"] / steps / W,
            "host_ms_per_step_per_worker": acc["handle_ns"] / steps / W / 1e6,
            "pass_split_ms_per_worker": {k: acc[k + "_ns"] / steps / W / 1e6
                                         for k in ("pack", "device", "apply")},
        }
        if mode in ("device_sized", "device_stream"):
            rec["stream_bytes_per_event"] = acc.get("stream_bytes", 0) / max(1, ne)
            rec["producer_encode_ns_per_event"] = t_enc / max(1, ne) * 1e9
        key = {("device_sized", 1): None, ("device_sized", T): "concurrent_workers",
               ("device_sized", 2): "two_workers",
               ("device_stream", 1): "device_stream", ("device_stream", T): "device_stream_concurrent",
               ("device_rows", 1): "device_rows", ("device_rows", T): "device_rows_concurrent",
               ("host", 1): "host_worker", ("host", T): "host_worker_concurrent"}[(mode, W)]
        if key is None:
            out.update(rec)
        else:
            out[key] = rec
    if with_cpu and d.rank == 0 and d.world == 1:
        from oracle import qref

        g, m = gm
        cpu = {}
        for nt in (1, T):
            b = qref.StepBatch(g, m)
            tc, ne = 0.0, 0
            for s in range(steps + STEP_WARM):   # timed: steps 1 .. cpu_steps; the rest
                ev = events(s)                       # replayed for the final state
                t0 = time.perf_counter()
                b.step(*ev, nthreads=nt)
                if 0 < s <= cpu_steps:
                    tc += time.perf_counter() - t0
                    ne += len(ev[2])
            committed_cpu = [b.committed(i) for i in range(len(committed["host"]))]
            b.close()
            cpu[nt] = ne / tc
        out["cpu_reference"] = {
            "value": cpu[T], "unit": "events/s", "threads": T, "single_thread_value": cpu[1],
            "sample": f"the same events of the first {cpu_steps} steps, replayed event by "
                      f"event (oracle/qref_step.c, C restatement of the reference path)",
        }
        # the same events left the same committed indexes
        out["parity_committed"] = all(c == committed_cpu for c in committed.values())
        for k in ("value", "two_workers", "concurrent_workers", "device_stream",
                  "device_stream_concurrent",
                  "device_rows", "device_rows_concurrent", "host_worker",
                  "host_worker_concurrent"):
            v = out.get(k)
            v = v["value"] if isinstance(v, dict) else v
            if v:
                out.setdefault("vs_cpu_replay", {})[k] = v / cpu[T]
    return out


def run_wire_leg(d: Dist, G=1 << 14, reps=20):
    """The step worker's input from the wire (hq_wire.cpp), host side: the received messages of
    a steady-state step of G leader groups (3 voters: a ReplicateResp and a HeartbeatResp from
    each follower) marshalled as raftpb.MessageBatch bytes, one batch per sending node
    (tests/wire_encode.py, the gogo layout), then per step: hq_wire_reset + hq_wire_add_batch of
    every batch (protobuf decode, deployment / version check, per-cluster queues) +
    hq_wire_step_stream (the step's event stream for the worker). One host thread; the bytes are
    built outside the timed region. The stream it produces is then stepped on the device engine,
    and its commits are checked against the same step fed as rows."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests"))
    import wire_encode as we
    from dragonboat_amd import hipquorum as hq

    roles = STEP_ROLES["step"]
    rng = _shard_of(d, G)
    g, m, cids = step_groups(hq, G, rng.cid_base, rng.cid_stride, roles)
    g["committed"] -= np.uint64(10)          # the step's acks (of lastIndex) commit
    m["match"][m["node_id"] != 1] -= np.uint64(10)
    dep = 0x5EED
    _, off, ev = step_events(hq, G, 0, roles)
    msgs = {}
    cols = {k: ev[k].tolist() for k in ("kind", "type", "from", "term", "log_index", "hint",
                                        "hint_high")}
    offl, cidl = off.tolist(), cids.tolist()
    for i in range(G):
        for j in range(offl[i], offl[i + 1]):
            if cols["kind"][j] == hq.EV_MESSAGE:
                msgs.setdefault(cols["from"][j], []).append(
                    we.message(type=cols["type"][j], to=1, frm=cols["from"][j],
                               cluster_id=cidl[i], term=cols["term"][j],
                               log_index=cols["log_index"][j], hint=cols["hint"][j],
                               hint_high=cols["hint_high"][j]))
    batches = [we.batch(v, deployment_id=dep, source_address=b"n%d:63000" % k)
               for k, v in sorted(msgs.items())]
    n_msg = sum(len(v) for v in msgs.values())
    n_bytes = sum(len(b) for b in batches)
    w = hq.Worker(d.device, sum(r != "observer" for r in roles), on_device=True)
    w.add_groups(g, m)
    wire = hq.Wire(dep)
    bufs = [np.frombuffer(b, np.uint8) for b in batches]
    times = []
    for r in range(reps + 2):
        t0 = time.perf_counter()
        wire.reset()
        for b in bufs:
            wire.add_batch(b)
        grp, o, bo, data, st = wire.step_stream(w)
        dt = time.perf_counter() - t0
        if r >= 2:
            times.append(dt)
    assert st.messages == n_msg and st.dropped_messages == 0
    # the stream from the wire decides like the same messages fed as rows
    res = w.step_stream(grp, o, bo, data)
    w2 = hq.Worker(d.device, sum(r != "observer" for r in roles), on_device=True)
    w2.add_groups(g, m)
    msg_only = ev[ev["kind"] == hq.EV_MESSAGE]
    per = np.array([int(((ev["kind"][int(off[i]):int(off[i + 1])]) == hq.EV_MESSAGE).sum())
                    for i in range(G)], np.int64)
    moff = np.concatenate([[0], np.cumsum(per)]).astype(np.uint64)
    ref = w2.step(np.arange(G, dtype=np.uint32), moff, msg_only)
    same = bool(np.array_equal(np.sort(res["commits"]["cluster_id"]),
                               np.sort(ref["commits"]["cluster_id"])) and
                np.array_equal(res["commits"]["committed"][np.argsort(res["commits"]["cluster_id"])],
                               ref["commits"]["committed"][np.argsort(ref["commits"]["cluster_id"])]))
    w.close()
    w2.close()
    wire.close()
    t = float(np.median(times))
    return {
        "workload": f"wire: the received messages of one steady-state step of {G} leader groups "
                    f"(3 voters), {n_msg} raftpb.Message in {len(batches)} MessageBatch "
                    f"({n_bytes} bytes), decoded and assembled into the step's event stream "
                    f"(hq_wire_add_batch + hq_wire_step_stream), one host thread",
        "unit": "messages/s", "value": n_msg / t, "ms_per_step": t * 1e3,
        "ns_per_message": t / n_msg * 1e9, "wire_mb_per_s": n_bytes / t / 1e6,
        "stream_bytes_per_message": len(data) / n_msg,
        "commits_equal_rows_path": same and len(res["commits"]) == G,
        "commits": int(len(res["commits"])),
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


def cpu_baseline(w, budget_s=8.0, gpu_set0=None):
    """The oracle (C restatement of the reference path) on a bounded sample of the workload.
    gpu_set0: the GPU's decisions of batch set 0 (run_gpu), compared bit for bit with the
    oracle's on the same inputs at full size (full_size_parity)."""
    from oracle import qref

    host_threads = min(16, os.cpu_count() or 1)
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
    for nt in (1, host_threads):
        passes, t0 = 0, time.perf_counter()
        while True:
            one(nt)
            passes += 1
            dt = time.perf_counter() - t0
            if dt >= budget_s / 2:
                break
        out[nt] = (passes * G * decisions_per_group(w) / dt, passes, dt)
    rate, passes, dt = out[host_threads]
    parity = full_size_parity(w, gpu_set0, host_threads) if gpu_set0 else None
    # BASELINE config C1: the reference's own CPU case, one group x 3 voters, tryCommit per step
    T = 4 << 20
    match, last = qref.c1_stream(SEED_BASE, T, 1000, 1005)
    t0 = time.perf_counter()
    qref.c1_run(match, last, 1003, 1000)
    c1_s = time.perf_counter() - t0
    return {
        "value": rate, "unit": "decisions/s", "cores": host_threads, "kind": "port",
        "sample": (f"{G} groups of the same workload and generator, {passes} passes in {dt:.1f} s "
                   f"on {host_threads} host threads (oracle/qref.c -O3, C restatement of the "
                   f"reference Go path; Go toolchain unavailable)"),
        "single_thread_value": out[1][0],
        "c1_single_group_ns_per_trycommit": c1_s / T * 1e9,
        "c1_sample": f"BASELINE config C1: 1 group x 3 voters, {T} sequential tryCommit steps",
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--workload", default=HEADLINE, choices=sorted(WORKLOADS))
    ap.add_argument("--step-groups", type=int, default=1 << 20,
                    help="groups per GPU of the step-worker leg (extra 'step')")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extra-parity", action="store_true",
                    help="skip the full-size oracle check of the commit / lag extras")
    ap.add_argument("--extra", default=DEFAULT_EXTRAS,
                    help="comma list of extra workloads reported under 'extra' ('' for none)")
    args = ap.parse_args()

    d = Dist()
    if args.gpus != d.world:
        log(f"--gpus {args.gpus} but WORLD_SIZE={d.world}: launch N>1 with torch.distributed.run")
        if d.world == 1 and args.gpus > 1:
            sys.exit(2)
    w = WORKLOADS[args.workload]
    t_start = time.perf_counter()

    def progress(msg):          # one line per phase (a long run must keep writing)
        if d.rank == 0:
            log(f"[bench {time.perf_counter() - t_start:7.1f} s] {msg}")

    progress(f"headline {args.workload}: {args.steps} steps, {args.warmup} warmup")
    r = run_gpu(w, args.steps, args.warmup, d)
    r["world"] = d.world
    host_threads = min(16, os.cpu_count() or 1)
    oracle_here = d.rank == 0 and d.world == 1 and not args.no_cpu
    extras, extra_runs = [], {}
    e2e = None
    steps_legs = []
    conc, kern = [], []
    failed = []
    for name in [x for x in args.extra.split(",") if x and x != args.workload]:
        we = WORKLOADS.get(name)
        if we is not None and we.get("mixed") and d.world % 3 == 0:
            # voter-count buckets need gcd(3, world) == 1 (shard.rank_bucket); same on every rank
            failed.append({"workload": name, "skipped": "world size divisible by 3"})
            continue
        progress(f"extra {name}")
        try:
            if name == "e2e":
                e2e = run_e2e(max(100, args.steps // 4), 5, d)   # >= 30 ms timed per variant
            elif name == "wire":
                steps_legs.append(run_wire_leg(d))
            elif name in STEP_ROLES:
                steps_legs.append(run_step_leg(d, G=args.step_groups, with_cpu=not args.no_cpu,
                                               name=name))
            elif name in ("rim", "rimt", "cq", "cqp", "ing", "ingo", "ingu"):
                kern.append(run_kernel_leg(name, max(50, args.steps // 4),
                                           max(5, args.warmup // 4), d))
            elif name == "sweep":
                conc.append(run_size_sweep(args.workload, max(50, args.steps // 4),
                                           max(5, args.warmup // 4), d))
            elif name.startswith("w") and name[1:].isdigit():
                conc.append(run_concurrent(w, args.steps, args.warmup, d, W=int(name[1:])))
            else:
                re_ = run_gpu(we, max(50, args.steps // 4), max(5, args.warmup // 4), d)
                re_["world"] = d.world
                par = None
                if oracle_here and re_.get("set0") and not args.no_extra_parity:
                    par = full_size_parity(we, re_["set0"], host_threads)
                extras.append(extra_record(name, we, re_, par))
                extra_runs[name] = re_
        except Exception as e:   # an extra leg never costs the headline line
            log(f"extra leg {name} failed: {e!r}")
            failed.append({"workload": name, "error": repr(e)})
    cpu = None
    if oracle_here:
        progress("cpu baseline")
        cpu = cpu_baseline(w, gpu_set0=r.get("set0"))
    # the term check of the same groups in its other exact forms (the ring gathers the north
    # star names, the mask the headline streams): rate and whether every decision is identical
    forms_same_data = []
    for name in SAME_DATA_FORMS.get(args.workload, ()):
        if name in extra_runs:
            re_ = extra_runs[name]
            forms_same_data.append({
                "workload": name, "form": WORKLOADS[name]["desc"],
                "value": re_["decisions"] / re_["elapsed"],
                "roofline_frac": re_["achieved_node_gbs"] / (HBM_PEAK_GBS * d.world),
                "decisions_equal_to_headline": same_decisions(r.get("set0"), re_.get("set0")),
            })
    if d.rank == 0:
        traffic, traffic_src = pmc_traffic(args.workload)
        peak = HBM_PEAK_GBS * d.world
        achieved = r["achieved_node_gbs"]
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
            "data": "synthetic: device-generated splitmix64 batches (DESIGN.md), "
                    f"{r['nsets']} distinct batches per GPU rotated (>= 1.1 GiB); the timed "
                    f"steps start at batch {r['first_timed_set']}, after the warm-up's",
            "config": {
                "workload": f"{args.workload}: {w['desc']}",
                "groups_per_gpu": w["G"], "voters": w["n"],
                "form": ({0: "term_start", 1: "ring", 2: "term_mask", 3: "ring32"}[w["form"]]
                         + ("_lag" if w["kind"] == "lag" else ""))
                if w["kind"] in ("commit", "lag") else "bitmaps",
                "layout": ("tiles_leader" if w.get("lead") else "tiles") if w.get("tiled")
                else "columns",
                "global_groups_per_step": w["G"] * d.world,
                "parallelism": f"shard{d.world} (clusterID % {d.world})",
                "world_size": d.world,
                "backend": d.backend or "none (one process)",
            },
            "roofline": {
                "bound": "hbm", "achieved": achieved, "peak": peak, "unit": "GB/s",
                "frac": achieved / peak, "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel_avg_us": r["avg_kernel_s"] * 1e6,
                "kernel_time": "HIP events on the launch stream: a region opened behind the first "
                               "timed launch and closed behind the last one, / the launches in "
                               "it (back-to-back kernels: duration + dependent-launch boundary)",
                "algorithmic_bytes_per_launch": r["bytes_per_launch"],
                "achieved_scope": f"node: sum over {d.world} GPU(s) of bytes per launch / "
                                  "kernel time; peak = 8 TB/s x GPUs",
                "measured_copy_ceiling_gbs": HBM_MEASURED_COPY_GBS * d.world,
            },
            "per_gpu": [{"rank": i, "decisions_per_s": v, "kernel_avg_us": k,
                         "achieved_gbs": a, "frac": a / HBM_PEAK_GBS}
                        for i, (v, k, a) in enumerate(r["per_gpu"])],
            "result_gather": r["gather"],
            "cpu_baseline": cpu,
            "term_check_forms_same_data": forms_same_data,
            "extra": extras + kern + conc + ([e2e] if e2e else []) + steps_legs + failed,
        }
        print(json.dumps(line), flush=True)
    d.close()


if __name__ == "__main__":
    main()
