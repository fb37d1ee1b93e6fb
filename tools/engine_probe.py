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
    arrive, top = st.pop("arrive"), st.pop("top")
    print(f"  arrive counters per slot: {arrive.tolist()} top {top.tolist()}")
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
    if os.environ.get("PROBE_MODE") == "idle":
        # how long a resident grid stays after its last step, per idle limit
        for idle_us in (2000, 20000, 100000):
            eng = hq.Engine(ctx, n, form, lay, depth=depth, signal=signal, idle_us=idle_us)
            for rep in range(2):
                q = eng.post(b.tile_args())
                t0 = time.perf_counter()
                while True:
                    st = eng.dump()
                    if int(st["cursor"].min()) > q:
                        break
                    if time.perf_counter() - t0 > 2:
                        break
                dt = time.perf_counter() - t0
                print(f"idle_us {idle_us}: grid ended {dt * 1e3:.2f} ms after the post "
                      f"(cursor min {int(st['cursor'].min())}, exit epoch {st['exit_epoch']}, "
                      f"launches {st['launches']})", flush=True)
            eng.drain()
            eng.close()
        return
    eng = hq.Engine(ctx, n, form, lay, depth=depth, signal=signal)
    try:
        quiet = os.environ.get("PROBE_QUIET") == "1"
        for s in range(steps):
            q = eng.post(b.tile_args())
            if not quiet:
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
