#!/usr/bin/env python3
"""Reproduce an engine scenario step by step with the device state printed (hq_engine_dump):
post-one-at-a-time into a small ring (PROBE_DEPTH, default 4), PROBE_STEPS steps, no signal
unless PROBE_SIGNAL=1. HQ_ENGINE_WAIT_MS bounds every wait."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("HQ_ENGINE_WAIT_MS", "3000")
from dragonboat_amd import hipquorum as hq  # noqa: E402


def show(eng, tag):
    st = eng.dump()
    cur = st.pop("cursor")
    vals, counts = np.unique(cur, return_counts=True)
    print(f"{tag}: {st} cursors {dict(zip(vals.tolist(), counts.tolist()))}", flush=True)


def main():
    depth = int(os.environ.get("PROBE_DEPTH", "4"))
    steps = int(os.environ.get("PROBE_STEPS", "10"))
    signal = os.environ.get("PROBE_SIGNAL", "0") == "1"
    n, form, lay = 5, hq.HQ_FORM_TERM_MASK, hq.HQ_LAYOUT_TILES_LEADER
    ctx = hq.Context(0)
    G = int(os.environ.get("PROBE_G", "5000"))
    b = hq.alloc_commit(ctx, G, n, form, 16, tiled=True, tile_layout=lay)
    ctx.synth_commit_dev(hq.synth_spec(7, G, n, parity_extras=True), b.args())
    ctx.tile_commit_dev(b.args(), b.tiles, lay)
    ctx.sync()
    eng = hq.Engine(ctx, n, form, lay, depth=depth, signal=signal)
    try:
        for s in range(steps):
            q = eng.post(b.tile_args())
            time.sleep(0.002)
            show(eng, f"posted {q}")
        eng.drain()
        show(eng, "drained")
    except hq.HQError as e:
        print("ERROR", e, flush=True)
        show(eng, "after error")
        sys.exit(1)
    finally:
        pass
    print("ok")


if __name__ == "__main__":
    main()
