#!/usr/bin/env python3
"""The persistent engine's cost per launch for K steps of G groups: posted in one call then
drained (the STOP reaches the running grid through the ring), posted one call per step then
drained (post-as-ready), handed over with the STOP (hq_engine_run), beside the same K batches
in one fused launch. NB batches rotate (NB = 24 x 1 M groups: 1.4 GB, past the Infinity Cache).
Prints us per launch (HIP events around the launch)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dragonboat_amd import hipquorum as hq  # noqa: E402


def main():
    ctx = hq.Context(0)
    n, form, lay = 5, hq.HQ_FORM_TERM_MASK, hq.HQ_LAYOUT_TILES_LEADER
    sig = os.environ.get("SIG", "0") == "1"
    for G, NB in ((128, 4), (1 << 20, 24)):
        bs = []
        for s in range(NB):
            b = hq.alloc_commit(ctx, G, n, form, 16, tiled=True, tile_layout=lay)
            ctx.synth_commit_dev(hq.synth_spec(7 + s, G, n), b.args())
            ctx.tile_commit_dev(b.args(), b.tiles, lay)
            bs.append(b)
        ctx.sync()
        eng = hq.Engine(ctx, n, form, lay, ring_len=16, signal=sig)
        rot = [0]

        def arr(k):
            r0 = rot[0]
            rot[0] += k
            return hq.commit_batch_array([bs[(r0 + i) % NB].tile_args() for i in range(k)])
        eng.run(arr(2))
        eng.timing(reset=True)
        for K in (1, 2, 5, 20):
            res = {"post": [], "posts": [], "run": [], "fused": []}
            for _ in range(7):
                eng.post(arr(K))
                eng.drain()
                nl, ms = eng.timing(reset=True)
                res["post"].append(ms * 1e3 / max(1, nl))
                for one in [arr(1) for _ in range(K)]:
                    eng.post(one)
                eng.drain()
                nl, ms = eng.timing(reset=True)
                res["posts"].append(ms * 1e3 / max(1, nl))
                eng.run(arr(K))
                nl, ms = eng.timing(reset=True)
                res["run"].append(ms * 1e3 / max(1, nl))
                ctx.timing_reset()
                ctx.timing(True)
                ctx.commit_fused_dev(arr(K))
                ctx.timing(False)
                ctx.sync()
                fms, fnl = ctx.timing_read()
                res["fused"].append(fms * 1e3 / max(1, fnl))
            print(f"G={G:8d} K={K:2d} " + "  ".join(
                f"{k} {np.median(v):7.2f} us ({np.median(v) / K:6.2f}/step)" for k, v in res.items()),
                flush=True)
        eng.close()
    ctx.close()


if __name__ == "__main__":
    main()
