"""Probe: the device step engine on the bench's step workload (G = 1M leader groups), W workers
(one native thread each via hq_worker_step_jobs, G / W groups each), events in pinned memory (FEED=sized: the event
stream with per-group size words, FEED=stream: with the two prefix arrays, FEED=rows: hq_event rows); prints per-step wall time. Run under rocprofv3
--kernel-trace --stats for the kernels' share."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from dragonboat_amd import hipquorum as hq  # noqa: E402

G = int(os.environ.get("G", 1 << 20))
W = int(os.environ.get("W", 1))
STEPS = int(os.environ.get("STEPS", 6))
roles = bench.STEP_ROLES[os.environ.get("LEG", "step")]
feed = os.environ.get("FEED", "sized")      # sized | stream | rows
stream = feed in ("stream", "sized")
bounds = [G * i // W for i in range(W + 1)]
g, m, cids = bench.step_groups(hq, G, 1, 1, roles)
nm = len(roles)
workers = []
for i in range(W):
    w = hq.Worker(0, sum(r != "observer" for r in roles), on_device=True,
                  commit_column=os.environ.get("COLUMN", "1") == "1",
                  commit_advance=os.environ.get("ADVANCE", "1") == "1",
                  ready_compact=os.environ.get("COMPACT", "0") == "1" or
                  os.environ.get("SLOTS", "0") == "1",
                  ready_slots=os.environ.get("SLOTS", "0") == "1")
    if os.environ.get("WAIT"):             # WAIT=block|sleep|spin (hq_worker_set_wait)
        w.set_wait({"block": 0, "sleep": 1, "spin": 2}[os.environ["WAIT"]],
                   int(os.environ.get("POLL_US", 50)), int(os.environ.get("SLEEP_US", 20)))
    w.add_groups(g[bounds[i]:bounds[i + 1]], m[nm * bounds[i]:nm * bounds[i + 1]])
    workers.append(w)
pc = hq.Context(0)
for s in range(STEPS):
    inputs, ne = [], 0
    for i in range(W):
        e = bench.step_events(hq, bounds[i + 1] - bounds[i], s, roles)
        ne += len(e[2])
        nev = len(e[2])
        if feed == "sized":
            data, sizes = hq.encode_events_sized(e[1], e[2])
            if os.environ.get("S16", "0") == "1":     # 2-byte size words
                sizes = hq.sizes16_of(sizes)
            e = (e[0], sizes, data)
        elif stream:
            data, boff = hq.encode_events(e[1], e[2])
            e = (e[0], e[1], boff, data)
        p = tuple(pc.pinned(x.size, x.dtype) for x in e)
        for dst, src in zip(p, e):
            dst[:] = src
        if feed == "sized":       # IMPLICIT=1 (default): groups = NULL, as the bench's legs
            implicit = os.environ.get("IMPLICIT", "1") == "1"
            p = hq.SizedStream(None if implicit else p[0], p[1], nev, p[2])
        inputs.append(p)
    jobs = hq.StepJobs(list(zip(workers, inputs)))
    t0 = time.perf_counter()
    res = jobs.run(copy=False)
    dt = time.perf_counter() - t0
    dev = max(r["gpu_ns"] for r in res) / 1e6
    slotted = sum(len(r.get("ready_slots", ())) for r in res)
    if os.environ.get("PER_WORKER") and W > 1:
        print("  device ms per worker:", " ".join(f"{r['device_ns'] / 1e6:.2f}" for r in res),
              "| host ms:", " ".join(f"{r['handle_ns'] / 1e6:.2f}" for r in res), flush=True)
    if os.environ.get("LISTS"):
        print("  lists:", {k: sum(len(r[k]) for r in res if r.get(k) is not None)
                           for k in ("ready", "read_resps", "state_changes", "dropped_reads",
                                     "deferred", "fallback_groups")}, flush=True)
    print(f"step {s}: {dt * 1e3:.2f} ms, {ne} events, {ne / dt:.3e} events/s, W={W}, "
          f"gpu {dev:.3f} ms, slotted {slotted}, input {sum(getattr(x, 'nbytes', 0) for p in inputs for x in p) / 1e6:.1f} MB",
          flush=True)
for w in workers:
    w.close()
pc.close()
