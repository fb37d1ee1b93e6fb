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
    for _ in range(reps):
        th = [threading.Thread(target=one, args=(i,)) for i in range(W)]
        t0 = time.perf_counter()
        for t in th: t.start()
        for t in th: t.join()
        ts.append(time.perf_counter() - t0)
    return min(ts) * 1e3, np.median(ts) * 1e3
for W, T in ((1, 16), (2, 8), (16, 1), (1, 8), (2, 4)):
    print(W, T, ["%.2f" % x for x in run(W, T)])
