"""Probe: the device step engine on the bench's step workload (1M leader groups), one worker,
events in pinned memory (FEED=stream: as the event stream, FEED=rows: as hq_event rows); prints
per-step wall time. Run under rocprofv3 --kernel-trace --stats for the kernels' share."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402
from dragonboat_amd import hipquorum as hq  # noqa: E402

G = int(os.environ.get("G", 1 << 20))
roles = bench.STEP_ROLES[os.environ.get("LEG", "step")]
g, m, cids = bench.step_groups(hq, G, 1, 1, roles)
w = hq.Worker(0, sum(r != "observer" for r in roles), on_device=True)
w.add_groups(g, m)
pc = hq.Context(0)
stream = os.environ.get("FEED", "stream") == "stream"
for s in range(6):
    e = bench.step_events(hq, G, s, roles)
    ne = len(e[2])
    if stream:
        data, boff = hq.encode_events(e[1], e[2])
        e = (e[0], e[1], boff, data)
    p = tuple(pc.pinned(x.size, x.dtype) for x in e)
    for dst, src in zip(p, e):
        dst[:] = src
    t0 = time.perf_counter()
    r = w.step_stream(*p, copy=False) if stream else w.step(*p, copy=False)
    dt = time.perf_counter() - t0
    print(f"step {s}: {dt * 1e3:.2f} ms, {ne} events, {ne / dt:.3e} events/s, "
          f"device {r['device_ns'] / 1e6:.2f} ms, input {sum(x.nbytes for x in p) / 1e6:.1f} MB",
          flush=True)
w.close()
pc.close()
