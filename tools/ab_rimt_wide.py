#!/usr/bin/env python3
"""A/B of the multi-ctx ReadIndex tile kernels on the rimt leg (2 M groups x 4 ctxs x 7 voters,
128-group tiles), alternated over rounds on the same box:

  HQ_RI_WIDE     0: ordinal rows of 128 entries per (ctx, voter); 1: voter-major (each lane's
                 K_max ctx ordinals contiguous: one 16-byte load per voter at K_max = 4)
  HQ_RI_BLOCK    256, 512 or 1024 threads per workgroup (k_ri_multi2)
  HQ_RI_UNIFORM  1: uniform wide tiles on k_ri_tiles_u (constant K and n); 0: on k_ri_multi2

Usage: ab_rimt_wide.py ROUNDS [WIDE:BLOCK[:UNIFORM],...]; LEG=rimtc times the compact outputs
(released_index not written). The first round checks the leg's full-size parity."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
variants = [v.split(":") for v in (sys.argv[2] if len(sys.argv) > 2 else "0:256,1:256").split(",")]
leg = os.environ.get("LEG", "rimt")
d = bench.Dist()
for r in range(rounds):
    for v in variants:
        wide, blk, uni = (v + ["1"])[:3]
        os.environ["HQ_RI_WIDE"] = wide
        os.environ["HQ_RI_BLOCK"] = blk
        os.environ["HQ_RI_UNIFORM"] = uni
        rec = bench.run_kernel_leg(leg, 20, 4, d, parity_threads=16 if r == 0 else 0)
        par = rec.get("parity_full_size")
        print(f"round {r} {leg} wide={wide} block={blk} uniform={uni} "
              f"kernel_avg_us={rec.get('kernel_avg_us'):.2f} frac={rec.get('roofline_frac'):.4f} "
              f"parity={par and par.get('equal')}", flush=True)
