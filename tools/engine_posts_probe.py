#!/usr/bin/env python3
"""Where a post-as-ready window of the signalled engine spends its extra time: 20 steps of 1 M
groups (24 rotating batches, past the Infinity Cache) posted in one call or one call per step;
per window the launch time (HIP events), the device clock's interval between the first and the
last step's completion ((K - 1) intervals: the steady state), and the rest (start + tail)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dragonboat_amd import hipquorum as hq  # noqa: E402


def main():
    ctx = hq.Context(0)
    n, form, lay = 5, hq.HQ_FORM_TERM_MASK, hq.HQ_LAYOUT_TILES_LEADER
    G, NB, K = 1 << 20, 24, 20
    bs = []
    for s in range(NB):
        b = hq.alloc_commit(ctx, G, n, form, 16, tiled=True, tile_layout=lay)
        ctx.synth_commit_dev(hq.synth_spec(7 + s, G, n), b.args())
        ctx.tile_commit_dev(b.args(), b.tiles, lay)
        bs.append(b)
    ctx.sync()
    eng = hq.Engine(ctx, n, form, lay, ring_len=16, signal=True)
    rot = [0]

    def arr(k):
        r0 = rot[0]
        rot[0] += k
        return hq.commit_batch_array([bs[(r0 + i) % NB].tile_args() for i in range(k)])
    eng.run(arr(2))
    eng.timing(reset=True)
    for mode in ("one post", "posts", "one post", "posts"):
        wins, steady = [], []
        for _ in range(7):
            if mode == "posts":
                batches = [arr(1) for _ in range(K)]
                q0 = None
                for one in batches:
                    q = eng.post(one)
                    q0 = q if q0 is None else q0
            else:
                q0 = eng.post(arr(K))
            for i in range(K):
                eng.wait(q0 + i)
            clk = [eng.done_clock(q0 + i) for i in range(K)]
            eng.drain()
            nl, ms = eng.timing(reset=True)
            wins.append(ms * 1e3)
            steady.append((clk[-1] - clk[0]) / 1e2 / (K - 1))     # 100 MHz ticks -> us
        w, st = np.median(wins), np.median(steady)
        print(f"{mode:9s}: window {w:7.1f} us, step interval {st:6.2f} us (steady {st * K:6.1f} us "
              f"for {K}), start + tail {w - st * (K - 1):6.1f} us", flush=True)
    eng.close()
    ctx.close()


if __name__ == "__main__":
    main()
