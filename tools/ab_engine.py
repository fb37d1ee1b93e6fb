#!/usr/bin/env python3
"""A/B of ways to run K commit steps of the headline workload (c3mtl: 1M groups x 5 voters,
leader-row tiles, mask form) on one GPU, same data, alternated rounds:
  launches      K back-to-back launches (hq_commit_many_dev)
  fused         the K batches in fused launches of <= 32 (hq_commit_fused_dev, the bench headline)
  engine        the persistent engine (hq_engine): K descriptors posted in one call, one resident
                launch, drained
  engine_each   the same, one hq_engine_post per step (a step worker posting as it is ready)
  signal        the engine with per-step completion flags, waited on the last step
  flat, claim512, loop512, gclaim512, pool   experiment kernels of tools/engine_exp.hip (one
                launch each; tools/lib_engexp/libengexp.so, `make tools/lib_engexp/libengexp.so`)
Kernel time: HIP events around the window (the engine's: around its resident launch).
AB_STEPS (K, default 20), AB_ROUNDS (5), AB_ONLY (comma list), AB_WORKLOAD (c3mtl)."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from dragonboat_amd import hipquorum as hq  # noqa: E402
from dragonboat_amd import shard  # noqa: E402

K = int(os.environ.get("AB_STEPS", "20"))
ROUNDS = int(os.environ.get("AB_ROUNDS", "5"))
EXP_LIB = os.path.join(ROOT, "tools", "lib_engexp", "libengexp.so")


def main():
    w = bench.WORKLOADS[os.environ.get("AB_WORKLOAD", "c3mtl")]
    d = bench.Dist()
    ctx = hq.Context(0)
    sets, per_set = bench.build_sets(ctx, hq, shard, w, d)
    nsets = len(sets)
    lay = hq.HQ_LAYOUT_TILES_LEADER

    def arr(i0, k=K):
        return hq.commit_batch_array([bench.batch_args(sets[(i0 + i) % nsets][0]) for i in range(k)])

    exp = None
    if os.path.exists(EXP_LIB):
        exp = ctypes.CDLL(EXP_LIB)
        exp.hq_exp_multi.restype = ctypes.c_int
        exp.hq_exp_multi.argtypes = [ctypes.c_void_p, ctypes.POINTER(hq.CommitArgs),
                                     ctypes.c_uint32, ctypes.c_int, ctypes.c_uint32]
    engines = {"engine": hq.Engine(ctx, w["n"], w["form"], lay, ring_len=16),
               "signal": hq.Engine(ctx, w["n"], w["form"], lay, ring_len=16, signal=True)}
    engines["engine_each"] = engines["engine"]

    def fused(a0):
        for c0, cn in bench.fused_chunks(K):
            ctx.commit_fused_dev(arr(a0 + c0, cn))

    variants = {
        "launches": lambda a0: ctx.commit_many_dev(arr(a0)),
        "fused": fused,
        "engine": None,
        "engine_each": None,
        "signal": None,
    }
    if exp is not None:
        for name, v, g in (("flat", 2, 0), ("claim512", 4, 512), ("loop512", 1, 512),
                           ("gclaim512", 6, 512), ("pool", 7, 512)):
            variants[name] = (lambda v, g: lambda a0: ctx._check(
                exp.hq_exp_multi(ctx.h, arr(a0), K, v, g)))(v, g)
    only = os.environ.get("AB_ONLY")
    if only:
        variants = {k: v for k, v in variants.items() if k in only.split(",")}
    res = {k: [] for k in variants}
    i0 = 0
    for r in range(ROUNDS + 1):
        for name, fn in variants.items():
            a0 = i0
            i0 += K
            ctx.sync()
            t0 = time.perf_counter()
            if name in engines:
                eng = engines[name]
                if name == "engine_each":
                    a = arr(a0)
                    for i in range(K):
                        eng.post(a[i])
                    eng.drain()
                elif name == "signal":
                    q0 = eng.post(arr(a0))
                    eng.wait(q0 + K - 1)
                    wall_sig = time.perf_counter() - t0
                    eng.drain()
                else:
                    eng.post(arr(a0))
                    eng.drain()
                n, ms = eng.timing(reset=True)
            else:
                ctx.timing_reset()
                ctx.timing(True)
                fn(a0)
                ctx.timing(False)
                ctx.sync()
                ms, n = ctx.timing_read()
            wall = time.perf_counter() - t0
            if name == "signal":
                wall = wall_sig
            if r > 0:
                res[name].append((ms * 1e3 / K, wall * 1e6 / K))
    # every variant's decisions of set 0 equal the launch path's
    b = sets[0][0]
    ctx.memset(b.committed_out, 0xA5)
    ctx.commit_dev(bench.batch_args(b))
    ctx.sync()
    ref = ctx.download(b.committed_out)
    for name in variants:
        ctx.memset(b.committed_out, 0xA5)
        ctx.sync()
        if name in engines:
            engines[name].post(arr(0))
            engines[name].drain()
        else:
            variants[name](0)
            ctx.sync()
        print(f"{name}: set0 equal to launches: {np.array_equal(ctx.download(b.committed_out), ref)}")
    for name, v in res.items():
        k = np.array([x[0] for x in v])
        wl = np.array([x[1] for x in v])
        print(f"{name:12s} kernel us/step median {np.median(k):7.3f} (min {k.min():7.3f} max "
              f"{k.max():7.3f})  frac {per_set / np.median(k) / 1e3 / 8000:.3f}   wall us/step "
              f"{np.median(wl):7.3f}", flush=True)
    for eng in {id(e): e for e in engines.values()}.values():
        eng.close()
    ctx.close()


if __name__ == "__main__":
    main()
