#!/usr/bin/env python3
"""The rimt leg (multi-ctx ReadIndex over 128-group tiles, k_ri_multi2<..., true>: 2 M groups x
4 ctxs x 7 voters, bench.run_kernel_leg) beside a device-to-device copy of the same bytes
(hq_memcpy_async, the runtime's copy kernel), for SQ counter passes:

  rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
      --output-format csv -d DIR -o run -- python3 tools/sq_rimt.py

then `python3 tools/sq_rimt.py --summary DIR` prints the per-kernel medians (VERDICT r03 item 6:
where rimt's time goes against the copy floor)."""
import csv
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run():
    import numpy as np

    import bench
    from dragonboat_amd import hipquorum as hq

    d = bench.Dist()
    rec = bench.run_kernel_leg("rimt", 20, 4, d, parity_threads=0)
    print("rimt", rec.get("kernel_avg_us"), rec.get("roofline_frac"), flush=True)
    G, K, n = 1 << 21, 4, 7
    nbytes = G * (2 * K * n + 8 * K + 8 * K + 2)       # the leg's bytes per launch (in + out)
    ctx = hq.Context(0)
    # read half, write half: the same total; 5 buffer pairs (1.28 GB) rotated, so no copy finds
    # its bytes in the 256 MB Infinity Cache (as the leg's own rotation)
    pairs = [(ctx.empty(nbytes // 2 // 8, np.uint64), ctx.empty(nbytes // 2 // 8, np.uint64))
             for _ in range(5)]
    for i in range(24):
        src, dst = pairs[i % 5]
        ctx.copy_to_ptr(dst.ptr, src, nbytes // 2)
    ctx.sync()
    print("copy", nbytes // 2, "bytes each way", flush=True)
    ctx.close()


def summary(d):
    rows = []
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv"):
                rows += list(csv.DictReader(open(os.path.join(root, f))))
    by = {}
    for r in rows:
        k = r["Kernel_Name"]
        k = "rimt k_ri_multi2" if "k_ri_multi2" in k else "copy" if "copyBuffer" in k else None
        if k:
            by.setdefault((k, r["Counter_Name"]), []).append(float(r["Counter_Value"]))
    for (k, c), v in sorted(by.items()):
        print(f"{k:18s} {c:22s} median {statistics.median(v):16.1f}  ({len(v)} dispatches)")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summary":
        summary(sys.argv[2])
    else:
        run()
