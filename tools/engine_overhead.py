#!/usr/bin/env python3
"""The persistent engine's cost per launch: K steps posted then drained (one resident launch; the
STOP reaches it through the ring), or handed over with the STOP (hq_engine_run),
for K = 1, 2, 5, 20 and batches of 1 tile and of 1 M groups (c3mtl shape), beside the same K
batches in one fused launch. Prints us per launch (HIP events around the launch) and the
fixed part (the K = 1 launch less one step)."""
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
    for G in (128, 1 << 20):
        bs = []
        for s in range(4):
            b = hq.alloc_commit(ctx, G, n, form, 16, tiled=True, tile_layout=lay)
            ctx.synth_commit_dev(hq.synth_spec(7 + s, G, n), b.args())
            ctx.tile_commit_dev(b.args(), b.tiles, lay)
            bs.append(b)
        ctx.sync()
        eng = hq.Engine(ctx, n, form, lay, ring_len=16, signal=sig)

        def arr(k):
            return hq.commit_batch_array([bs[i % 4].tile_args() for i in range(k)])
        eng.post(arr(2))
        eng.drain()
        eng.timing(reset=True)
        for K in (1, 2, 5, 20):
            ts, rs, fs = [], [], []
            for _ in range(7):
                eng.post(arr(K))
                eng.drain()
                nl, ms = eng.timing(reset=True)
                ts.append(ms * 1e3 / max(1, nl))
                eng.run(arr(K))
                nl, ms = eng.timing(reset=True)
                rs.append(ms * 1e3 / max(1, nl))
                ctx.timing_reset()
                ctx.timing(True)
                ctx.commit_fused_dev(arr(K))
                ctx.timing(False)
                ctx.sync()
                fms, fnl = ctx.timing_read()
                fs.append(fms * 1e3 / max(1, fnl))
            print(f"G={G:8d} K={K:2d} engine {np.median(ts):8.2f} us/launch "
                  f"({np.median(ts) / K:7.2f} per step)  run {np.median(rs):8.2f} "
                  f"({np.median(rs) / K:7.2f} per step)  fused {np.median(fs):8.2f} us/launch "
                  f"({np.median(fs) / K:7.2f} per step)", flush=True)
        eng.close()
        for b in bs:
            b.free() if hasattr(b, "free") else None
    ctx.close()


if __name__ == "__main__":
    main()
