"""Probe: where the persistent engine's windows lose against the fused launch — per workgroup.
Runs the headline's engine windows (c3mtl, 20 steps of 1 M groups posted one hq_engine_post each,
as bench.run_engine's `engine` mode) on the probe build (HQ_LIB_PATH=tools/lib_engprof/...,
-DHQ_ENGINE_WGPROF) and reads each workgroup's clocks: its start, the ticks its waves spent in
their tile loops, the tiles it decided, the moment its last wave left. Prints, per window: the
window's span on the device clock, the spread of the workgroups' end times, the busy time per
tile by XCC, and whether the slow workgroups of one window are the slow ones of the next (the
rank correlation of their busy times per tile)."""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from dragonboat_amd import hipquorum as hq  # noqa: E402
from dragonboat_amd import shard  # noqa: E402

lib = hq.lib
lib.hq_engine_wgprof.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int]
WG = 2048
buf = np.zeros(WG * 8, np.uint64)
STEPS = int(os.environ.get("STEPS", 20))
WINDOWS = int(os.environ.get("WINDOWS", 4))   # MW: max_workgroups (0: the full grid)


def wgprof(reset=True):
    rc = lib.hq_engine_wgprof(buf.ctypes.data, WG * 8, int(reset))
    assert rc == 0, rc
    return buf.reshape(WG, 8).copy()


d = bench.Dist()
w = bench.WORKLOADS[bench.HEADLINE]
ctx = hq.Context(0)
sets, per_set = bench.build_sets(ctx, hq, shard, w, d)
lay = hq.HQ_LAYOUT_TILES_LEADER if w.get("lead") else hq.HQ_LAYOUT_TILES
eng = hq.Engine(ctx, w["n"], w["form"], lay, ring_len=16,
                max_workgroups=int(os.environ.get("MW", 0)))
grid = eng.info().grid


def arr(i0, k):
    return hq.commit_batch_array([bench.batch_args(sets[(i0 + i) % len(sets)][0]) for i in range(k)])


eng.run(arr(0, 5))
ctx.sync()
wgprof(True)
eng.timing(reset=True)
prev = None
for k in range(WINDOWS):
    a1 = [arr(5 + k * STEPS + i, 1) for i in range(STEPS)]
    tp0 = time.perf_counter()
    if os.environ.get("ONEPOST"):          # the window's steps in one hq_engine_post call
        eng.post(arr(5 + k * STEPS, STEPS))
    else:
        for one in a1:
            eng.post(one)
    post_us = (time.perf_counter() - tp0) * 1e6
    eng.drain()
    nl, ms = eng.timing(reset=True)
    p = wgprof(True)[:grid]
    start, xcc, hwid, busy, tiles, end = (p[:, i].astype(np.int64) for i in range(6))
    front = (p[:, 6] & np.uint64((1 << 40) - 1)).astype(np.int64)
    nfront = (p[:, 6] >> np.uint64(40)).astype(np.int64)
    refr = p[:, 7].astype(np.int64)
    t0 = start.min()
    per_tile = busy / np.maximum(tiles, 1)      # wave-ticks per tile (10 ns)
    by_xcc = {int(x): {"wgs": int((xcc == x).sum()),
                       "busy_per_tile_us": round(float(per_tile[xcc == x].mean()) / 100, 3),
                       "end_mean_us": round(float((end[xcc == x] - t0).mean()) / 100, 2),
                       "end_max_us": round(float((end[xcc == x] - t0).max()) / 100, 2)}
              for x in sorted(set(xcc.tolist()))}
    rank = np.argsort(np.argsort(per_tile))
    corr = None if prev is None else float(np.corrcoef(rank, prev)[0, 1])
    prev = rank
    busy_frac = busy / np.maximum(end - start, 1) / (eng.info().block // 64)
    half = grid // 2
    wps = eng.info().block // 64
    life = np.maximum(end - start, 1) * wps             # wave-ticks of each workgroup's life
    out = {"window": k, "launches": nl, "event_ms": round(ms, 4), "post_us": round(post_us, 1),
           "frontier_frac_halves": [round(float((front / life)[:grid // 2].mean()), 4),
                                    round(float((front / life)[grid // 2:].mean()), 4)],
           "frontier_entries_per_wg_halves": [round(float(nfront[:grid // 2].mean()), 1),
                                              round(float(nfront[grid // 2:].mean()), 1)],
           "lookahead_us_per_wg_halves": [round(float(refr[:grid // 2].mean()) / 100, 2),
                                          round(float(refr[grid // 2:].mean()) / 100, 2)],
           "busy_frac_first_half_second_half": [round(float(busy_frac[:half].mean()), 3),
                                                round(float(busy_frac[half:].mean()), 3)],
           "event_us_per_step": round(ms * 1e3 / STEPS, 3),
           "device_span_us": round(float(end.max() - t0) / 100, 2),
           "start_spread_us": round(float(start.max() - t0) / 100, 2),
           "end_p0_p50_p100_us": [round(float(np.percentile(end - t0, q)) / 100, 2) for q in (0, 50, 100)],
           "tiles_per_wg": [int(tiles.min()), int(tiles.max())],
           "busy_per_tile_us_p0_p50_p100": [round(float(np.percentile(per_tile, q)) / 100, 3)
                                            for q in (0, 50, 100)],
           "slowest_wgs": [int(i) for i in np.argsort(end)[-8:]],
           "rank_corr_with_prev_window": corr, "by_xcc": by_xcc}
    print(json.dumps(out), flush=True)
    if os.environ.get("RAW") and k == WINDOWS - 1:       # every workgroup's words, last window
        np.save(os.environ["RAW"], p)
eng.close()
ctx.close()
