"""Host probe: the producer's encode of one step5 step (1 M groups, 13.9 M compact records, the
bench's hq_events16_encode_sized_multi over 16 workers' streams) on this process's CPUs: the
topology it sees, then the min / median of 12 encodes. Run under taskset to compare placements."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from dragonboat_amd import hipquorum as hq  # noqa: E402

G, W = 1 << 20, 16
roles = bench.STEP_ROLES["step5"]
recs = bench.StepRows16(hq, G, roles)
recs.set(1)
off = bench.StepRows(hq, G, roles).offsets
bounds = [G * i // W for i in range(W + 1)]
jobs = []
for i in range(W):
    o = off[bounds[i]:bounds[i + 1] + 1]
    e0, e1 = int(o[0]), int(o[-1])
    jobs.append((o - o[0], recs.recs[e0:e1], np.zeros((e1 - e0) * 5 + 64, np.uint8),
                 np.zeros(len(o) - 1, np.uint16)))
batch = hq.Encode16Batch(jobs)
T = bench.encode_threads()
ts = []
for _ in range(12):
    t0 = time.perf_counter()
    batch.run(T)
    ts.append((time.perf_counter() - t0) * 1e3)
cpus = sorted(os.sched_getaffinity(0))
print(f"cpus {len(cpus)} [{cpus[0]}..{cpus[-1]}] threads {T}: encode ms min {min(ts):.2f} "
      f"median {float(np.median(ts)):.2f} max {max(ts):.2f}", flush=True)
