#!/usr/bin/env python3
"""Encode concurrency probe: the step5 producer (hq_events16_encode_sized) of 1 M groups split
over W concurrent calls of T native threads each; min / median ms of 5 runs."""
import time, threading, numpy as np, sys
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
import bench
from dragonboat_amd import hipquorum as hq
G = 1 << 20
roles = bench.STEP_ROLES["step5"]
recs = bench.StepRows16(hq, G, roles)
off16, r = recs.set(1)
ctx_bufs = None
def split(W):
    b = [G * i // W for i in range(W + 1)]
    parts = []
    for i in range(W):
        o = off16[b[i]:b[i + 1] + 1]
        parts.append((o - o[0], int(o[0]), int(o[-1])))
    return parts
def run(W, T, reps=5):
    parts = split(W)
    outs = [(np.zeros((e1 - e0) * 5 + 64, np.uint8), np.zeros(len(o) - 1, np.uint32)) for o, e0, e1 in parts]
    def one(i):
        o, e0, e1 = parts[i]
        hq.encode_events16_sized_into(o, r[e0:e1], outs[i][0], outs[i][1], T)
    ts = []
    hq.encode_stats(reset=True)
    for _ in range(reps):
        th = [threading.Thread(target=one, args=(i,)) for i in range(W)]
        t0 = time.perf_counter()
        for t in th: t.start()
        for t in th: t.join()
        ts.append(time.perf_counter() - t0)
    st = hq.encode_stats(reset=True)
    c = max(1, st["calls"])
    ph = (f"per call: encode {st['encode_ns'] / c / 1e6:.2f} copy {st['copy_ns'] / c / 1e6:.2f} ms, "
          f"task run sum {st['run_ns'] / c / 1e6:.2f} ms, helped {st['helped'] / c:.1f}, "
          f"lag max {st['max_lag_ns'] / 1e6:.3f} ms") if st["calls"] else ""
    return min(ts) * 1e3, np.median(ts) * 1e3, ph
import os
for W, T in ((1, 16), (1, 14), (2, 8), (2, 7), (16, 1), (14, 1), (1, 8), (1, 1)):
    mn, md, ph = run(W, T)
    print(W, T, "%.2f %.2f" % (mn, md), ph, flush=True)
os.environ["HQ_ENCODE_DIRECT"] = "1"
for W, T in ((16, 1), (1, 1)):
    mn, md, ph = run(W, T)
    print("direct", W, T, "%.2f %.2f" % (mn, md), ph, flush=True)
