#!/usr/bin/env python3
"""A/B of ways to run K commit steps of the headline workload (c3mtl: 1M groups x 5 voters,
leader-row tiles, mask form) on one GPU, same data, alternated rounds:
  launches   K back-to-back launches (hq_commit_many_dev)
  loop       ONE launch, every wave loops over the K batches (the engine's ownership, no doorbell)
  flat       ONE launch, one wave per (batch, tile), batch-major
  engine     the persistent engine (hq_engine): K posted descriptors, one resident launch
             (engine512: HQ_ENGINE_BLOCK=512, 512-thread workgroups; experiment build only)
Needs the experiment build: HQ_LIB_PATH=tools/lib_engexp/libhipquorum.so (make that target)."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("HQ_LIB_PATH", os.path.join(ROOT, "tools", "lib_engexp", "libhipquorum.so"))

import bench  # noqa: E402
from dragonboat_amd import hipquorum as hq  # noqa: E402
from dragonboat_amd import shard  # noqa: E402

K = int(os.environ.get("AB_STEPS", "20"))
ROUNDS = int(os.environ.get("AB_ROUNDS", "5"))
hq.lib.hq_exp_engine_probe.restype = ctypes.c_int
hq.lib.hq_exp_engine_probe.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]
PROBES = ["start min", "start max", "relay first", "relay last", "wg desc first", "wg desc last",
          "step done first", "step done last", "-", "-", "at STOP (last)", "host flag (last)"]
hq.lib.hq_exp_multi.restype = ctypes.c_int
hq.lib.hq_exp_multi.argtypes = [ctypes.c_void_p, ctypes.POINTER(hq.CommitArgs), ctypes.c_uint32,
                                ctypes.c_int, ctypes.c_uint32]


def main():
    w = bench.WORKLOADS[os.environ.get("AB_WORKLOAD", "c3mtl")]
    d = bench.Dist()
    ctx = hq.Context(0)
    sets, per_set = bench.build_sets(ctx, hq, shard, w, d)
    nsets = len(sets)

    def arr(i0):
        return hq.commit_batch_array([bench.batch_args(sets[(i0 + i) % nsets][0]) for i in range(K)])

    engines = {}
    hq.lib.hq_exp_engine_set.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    for name, blk in (("engine", ""), ("engine512", "512")):
        os.environ["HQ_ENGINE_BLOCK"] = blk
        engines[name] = hq.Engine(ctx, w["n"], w["form"], hq.HQ_LAYOUT_TILES_LEADER, ring_len=16)
        hq.lib.hq_exp_engine_set(engines[name].h, int(os.environ.get("AB_ENGINE_EXP", "0")))
    os.environ.pop("HQ_ENGINE_BLOCK")
    variants = {
        "launches": lambda a: ctx.commit_many_dev(a),
        "loop512": lambda a: ctx._check(hq.lib.hq_exp_multi(ctx.h, a, K, 1, 512)),
        "loop1024": lambda a: ctx._check(hq.lib.hq_exp_multi(ctx.h, a, K, 1, 1024)),
        "loop256": lambda a: ctx._check(hq.lib.hq_exp_multi(ctx.h, a, K, 1, 256)),
        "flat": lambda a: ctx._check(hq.lib.hq_exp_multi(ctx.h, a, K, 2, 0)),
        "claim256": lambda a: ctx._check(hq.lib.hq_exp_multi(ctx.h, a, K, 3, 256)),
        "claim512": lambda a: ctx._check(hq.lib.hq_exp_multi(ctx.h, a, K, 4, 512)),
        "claim512x2": lambda a: ctx._check(hq.lib.hq_exp_multi(ctx.h, a, K, 5, 1024)),
        "gclaim512": lambda a: ctx._check(hq.lib.hq_exp_multi(ctx.h, a, K, 6, 512)),
        # claim512 + a shared pool of the last AB_POOL permille tiles per batch (device claims)
        "pool": lambda a: ctx._check(hq.lib.hq_exp_multi(ctx.h, a, K, 7, 512)),
        "engine": None,
        "engine512": None,
    }
    only = os.environ.get("AB_ONLY")
    if only:
        variants = {k: v for k, v in variants.items() if k in only.split(",")}
    res = {k: [] for k in variants}
    i0 = 0
    for r in range(ROUNDS + 1):
        for name, fn in variants.items():
            a = arr(i0)
            i0 += K
            ctx.sync()
            t0 = time.perf_counter()
            if name in engines:
                eng = engines[name]
                pr = (ctypes.c_uint64 * (64 + 16384))()
                hq.lib.hq_exp_engine_probe(eng.h, pr)
                eng.post(a)
                eng.drain()
                n, ms = eng.timing(reset=True)
                hq.lib.hq_exp_engine_probe(eng.h, pr)
                if r == ROUNDS and name == "engine":
                    t0p = pr[0]
                    print("engine phases (us after the first sampled wave started): " + ", ".join(
                        f"{PROBES[i]} {(pr[i] - t0p) / 100:.2f}" for i in range(12)
                        if PROBES[i] != "-" and pr[i] not in (0, 2**64 - 1)))
                    wt = (np.array(pr[64:64 + 8192], np.float64) - t0p) / 100
                    np.save(os.path.join(ROOT, "gpurun_out", "wave_done.npy"), wt)
                    print("wave finish (us): min %.1f median %.1f max %.1f" % (
                        wt.min(), np.median(wt), wt.max()))
            else:
                ctx.timing_reset()
                ctx.timing(True)
                fn(a)
                ctx.timing(False)
                ctx.sync()
                ms, n = ctx.timing_read()
            wall = time.perf_counter() - t0
            if r > 0:
                res[name].append((ms * 1e3 / K, wall * 1e6 / K))
    # correctness of the experiment kernels: set 0 decided by each equals the launch path
    ref = None
    for name in [x for x in ("launches", "loop512", "flat", "claim256", "claim512", "claim512x2",
                             "gclaim512", "pool")
                 if x in variants]:
        b = sets[0][0]
        ctx.memset(b.committed_out, 0xA5)
        a = arr(0)
        variants[name](a)
        ctx.sync()
        out = ctx.download(b.committed_out)
        ref = out if ref is None else ref
        print(f"{name}: set0 equal to launches: {np.array_equal(out, ref)}")
    for name, v in res.items():
        k = np.array([x[0] for x in v])
        wl = np.array([x[1] for x in v])
        print(f"{name:9s} kernel us/step median {np.median(k):7.3f} (min {k.min():7.3f})  "
              f"frac {per_set / np.median(k) / 1e3 / 8000:.3f}   wall us/step {np.median(wl):7.3f}")
    for name, eng in engines.items():
        b = sets[0][0]
        ctx.memset(b.committed_out, 0xA5)
        eng.post(arr(0))
        eng.drain()
        out = ctx.download(b.committed_out)
        print(f"{name}: set0 equal to launches: {ref is None or np.array_equal(out, ref)}")
        eng.close()
    ctx.close()


if __name__ == "__main__":
    main()
