"""Debug: the consecutive-run differential (tests/test_gpu_worker.py) for one seed and feed; at the
first step whose fallbacks differ between the host worker and the device, print a differing
group's events, both outputs and states."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from dragonboat_amd import hipquorum as hq  # noqa: E402
import test_gpu_worker as t  # noqa: E402
from step_harness import WorkerBackend  # noqa: E402

seed = int(os.environ.get("SEED", 31))
stream = {"rows": False, "stream": True}.get(os.environ.get("FEED", "stream"), os.environ.get("FEED"))
rng = np.random.default_rng(seed)
host = WorkerBackend(hq, n_max=8, seed=seed, on_device=False, stream=False)
dev = WorkerBackend(hq, n_max=8, seed=seed, on_device=True, stream=stream)
groups = t._consecutive_groups(rng, 2000)
for g in groups:
    host.add_group(*g)
    dev.add_group(*g)
ctx_seq = [0]
for s in range(5):
    per = {g[0]: t._run_events(rng, host.state(g[0]), ctx_seq) for g in groups if rng.random() < 0.9}
    before = {cid: host.state(cid) for cid in per}
    want, got = host.step(per), dev.step(per)
    a, b = set(want["_fallback"]), set(got["_fallback"])
    bad = sorted(a ^ b)
    diff_out = [cid for cid in per if any(want[cid][k] != got[cid][k] for k in
                ("committed", "commit_changed", "ready", "resps", "states", "dropped", "deferred"))]
    print(f"step {s}: fallback host {len(a)} device {len(b)}, differ {len(bad)}, outputs differ {len(diff_out)}")
    for cid in (bad + diff_out)[:3]:
        print("cid", cid, "host fb", cid in a, "dev fb", cid in b)
        print("  state before", before[cid])
        print("  events", per[cid])
        for k in ("committed", "ready", "resps", "states", "dropped", "deferred"):
            if want[cid][k] != got[cid][k]:
                print("  ", k, "host", want[cid][k], "dev", got[cid][k])
        print("  host after", host.state(cid))
        print("  dev after ", dev.state(cid))
    if bad or diff_out:
        break
host.close()
dev.close()
