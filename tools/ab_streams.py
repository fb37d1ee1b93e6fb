"""Experiment: does overlapping commit launches on several HIP streams (several step-worker
contexts) raise whole-node throughput on the c2 workload? One process, interleaved rounds.
  A: 1 context, every step one 1M-group launch (the bench's headline mode)
  B: 2 contexts, alternate steps (launch i+1 may start while launch i drains)
  C: 2 contexts, every step split in two 512K-group halves (two step workers, one node-step)
  D: 4 contexts, every step split in four 256K-group quarters
Prints median ms per step and the implied decisions/s."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dragonboat_amd import hipquorum as hq  # noqa: E402

G, N = 1 << 20, 3
STEPS = 400
ctxs = [hq.Context(0) for _ in range(4)]
base = ctxs[0]
sets = []
for s in range(21):
    b = hq.alloc_commit(base, G, N, hq.HQ_FORM_TERM_START, 16)
    base.synth_commit_dev(hq.synth_spec(0x5EED0001 + (s << 40), G, N), b.args())
    sets.append(b)
base.sync()


def part(b, k, parts):
    """args for the k-th of `parts` contiguous slices of batch b"""
    a = b.args()
    n = G // parts
    off = k * n
    a.G = n
    a.match = b.match.ptr + off * 8           # stride stays G (slot-major rows)
    a.committed_in = b.committed_in.ptr + off * 8
    a.committed_out = b.committed_out.ptr + off * 8
    a.last_index = b.last_index.ptr + off * 8
    a.term_start = b.term_start.ptr + off * 8
    a.changed = b.changed.ptr + off // 8
    a.fallback = b.fallback.ptr + off // 8
    return a


def plan(mode):
    """list of (ctx index, ctypes array of args)"""
    if mode == "A":
        return [(0, hq.commit_batch_array([sets[i % 21].args() for i in range(STEPS)]))]
    if mode == "B":
        return [(c, hq.commit_batch_array([sets[i % 21].args() for i in range(c, STEPS, 2)]))
                for c in range(2)]
    parts = 2 if mode == "C" else 4
    return [(c, hq.commit_batch_array([part(sets[i % 21], c, parts) for i in range(STEPS)]))
            for c in range(parts)]


plans = {m: plan(m) for m in "ABCD"}
res = {m: [] for m in plans}
for rnd in range(5):
    for m, p in plans.items():
        for c in ctxs:
            c.sync()
        t0 = time.perf_counter()
        for ci, arr in p:
            ctxs[ci].commit_many_dev(arr)
        for c in ctxs:
            c.sync()
        res[m].append((time.perf_counter() - t0) / STEPS * 1e3)
for m, v in res.items():
    ms = float(np.median(v))
    print(f"mode {m}: {ms * 1e3:.2f} us/step  {G / (ms * 1e-3):.3e} decisions/s  "
          f"({G * 56 / (ms * 1e-3) / 1e9:.0f} GB/s aggregate)")
