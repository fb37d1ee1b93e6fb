"""A/B of the bitmap kernel launch geometry in ONE process (interleaved rounds): contexts opened
with HQ_BITS_BLOCK = 256 / 512 / 1024 run the c4 fused ReadIndex+vote workload on the same
rotating inputs. Prints the median per-launch time per variant."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dragonboat_amd import hipquorum as hq

G = 16 << 20
variants = {}
for b in (256, 512, 1024):
    os.environ["HQ_BITS_BLOCK"] = str(b)
    variants[b] = hq.Context(0)
base = variants[256]
sets = []
for s in range(17):
    arrs = [base.empty(G, np.uint8) for _ in range(4)]
    base.synth_bitmaps_dev(hq.synth_spec(0x5EED0003 + (s << 40), G, 7), *arrs)
    sets.append((arrs, base.empty(hq.words64(G), np.uint64), base.empty(hq.words32(G), np.uint64)))
base.sync()
res = {b: [] for b in variants}
for rnd in range(6):
    for b, ctx in variants.items():
        for i in range(20):
            (da, dg, dr, dn), c, o = sets[i % len(sets)]
            ctx.readindex_vote_dev(G, da, dg, dr, dn, 0, c, o)
        ctx.sync()
        ctx.timing_reset(); ctx.timing(True)
        for i in range(100):
            (da, dg, dr, dn), c, o = sets[i % len(sets)]
            ctx.readindex_vote_dev(G, da, dg, dr, dn, 0, c, o)
        ms, n = ctx.timing_read(); ctx.timing(False)
        res[b].append(ms * 1e3 / n)
for b, v in res.items():
    print(f"bits block {b}: median {np.median(v):.2f} us  min {min(v):.2f}  ({G*4.375/np.median(v)/1e3:.0f} GB/s)")
