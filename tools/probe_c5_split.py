#!/usr/bin/env python3
"""The north star's per-GPU share (c5v5tl: 8 M groups x 5 voters, leader-row tiles, term mask)
decided as ONE hq_commit_dev launch (k_commit_big) against the same arrays cut into 8 views of
1 M groups in ONE hq_commit_fused_dev launch (k_commit_fused), alternated on one box, sets rotated
past the Infinity Cache as in bench.py; the two forms' outputs are checked equal on set 0.
Prints the kernel time per launch (HIP events) and the fraction of 8 TB/s."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import bench  # noqa: E402
from dragonboat_amd import hipquorum as hq  # noqa: E402
from dragonboat_amd import shard  # noqa: E402


def views(a, parts, n, form, layout):
    G = a.G
    per = G // parts
    assert G % parts == 0 and per % 128 == 0
    tw = hq.commit_tile_words(n, form, layout)
    out = []
    for k in range(parts):
        v = hq.CommitArgs()
        ctypes.memmove(ctypes.addressof(v), ctypes.addressof(a), ctypes.sizeof(a))
        g0 = k * per
        v.G = per
        v.match = a.match + (g0 // 128) * tw * 8
        if a.committed_out:
            v.committed_out = a.committed_out + g0 * 8
        v.changed = a.changed + (g0 // 64) * 8
        if a.fallback:
            v.fallback = a.fallback + (g0 // 64) * 8
        out.append(v)
    return out


def main():
    d = bench.Dist()
    w = bench.WORKLOADS["c5v5tl"]
    ctx = hq.Context(d.device)
    sets, per_set = bench.build_sets(ctx, hq, shard, w, d)
    nsets = len(sets)
    full = [bench.batch_args(s[0]) for s in sets]
    lay = full[0].layout
    split = [hq.commit_batch_array(views(a, 8, w["n"], w["form"], lay)) for a in full]

    def d2h(ptr, words):
        out = np.empty(words, np.uint64)
        rc = hq.lib.hq_memcpy_async(ctx.h, out.ctypes.data_as(ctypes.c_void_p),
                                    ctypes.c_void_p(ptr), words * 8, 1)
        assert rc == 0, rc
        ctx.sync()
        return out

    def outputs(a):
        ctx.sync()
        cout = d2h(a.committed_out, a.G) if a.committed_out else None
        return cout, d2h(a.changed, hq.words64(a.G))

    a0 = full[0]
    ctx.commit_dev(a0)
    want = outputs(a0)
    ctx.commit_fused_dev(split[0])
    got = outputs(a0)
    same = all((x is None and y is None) or np.array_equal(x, y) for x, y in zip(want, got))
    print("outputs equal:", same, flush=True)
    algo = per_set
    for r in range(3):
        for name, run in (("one 8M launch", lambda i: ctx.commit_dev(full[i % nsets])),
                          ("8 x 1M fused", lambda i: ctx.commit_fused_dev(split[i % nsets]))):
            _, avg, _ = bench._timed(ctx, d, run, 40, 5)
            print(f"round {r} {name}: {avg * 1e6:.2f} us per launch, "
                  f"{algo / avg / 1e9 / bench.HBM_PEAK_GBS:.4f} of 8 TB/s", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
