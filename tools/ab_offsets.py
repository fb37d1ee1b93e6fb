"""Experiment: do the c2 commit launch's seven column streams (3 match rows, committed in/out,
last, term_start) slow each other down when they start at the same large-alignment offsets?
Variants place the columns of each batch inside one allocation at a stagger of `delta` bytes
between consecutive columns. One process, interleaved rounds, hq_commit_dev unchanged."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dragonboat_amd import hipquorum as hq  # noqa: E402

G, N, STEPS, NSETS = 1 << 20, 3, 400, 21
ctx = hq.Context(0)
COL = G * 8


def build(delta):
    """NSETS batches; columns at offsets k * (COL + delta) inside one allocation per batch."""
    out = []
    for s in range(NSETS):
        ncol = N + 4
        buf = ctx.empty((ncol * (COL + delta) + 4096) // 8, np.uint64)
        base = (buf.ptr + 255) // 256 * 256
        off = [base + k * (COL + delta) for k in range(ncol)]
        a = hq.CommitArgs()
        a.G, a.n_max, a.form, a.ring_len = G, N, hq.HQ_FORM_TERM_START, 16
        # match rows are contiguous with stride G + delta/8 so every row gets its own stagger
        a.match_stride = G + delta // 8
        a.match = off[0]
        a.committed_in, a.committed_out, a.last_index, a.term_start = off[3], off[4], off[5], off[6]
        chg = ctx.empty(hq.words64(G), np.uint64)
        fb = ctx.empty(hq.words64(G), np.uint64)
        a.changed, a.fallback = chg.ptr, fb.ptr
        ctx.synth_commit_dev(hq.synth_spec(0x5EED0001 + (s << 40), G, N), a)
        out.append(a)
    ctx.sync()
    return hq.commit_batch_array([out[i % NSETS] for i in range(STEPS)])


variants = {d: build(d) for d in (0, 256, 4096, 65536 + 512, 1 << 20)}
res = {d: [] for d in variants}
for rnd in range(5):
    for d, arr in variants.items():
        ctx.sync()
        ctx.timing_reset()
        ctx.timing(True)
        ctx.commit_many_dev(arr)
        ms, n = ctx.timing_read()
        ctx.timing(False)
        res[d].append(ms * 1e3 / n)
for d, v in res.items():
    print(f"stagger {d:>8} B: median {np.median(v):.2f} us  min {min(v):.2f} us")
