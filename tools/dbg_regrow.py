"""Debug: the slot form across an output-region regrow (tests/test_gpu_slots.py
test_slots_survive_region_regrow), printing where the step's lists and slots differ."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from dragonboat_amd import hipquorum as hq  # noqa: E402

G = int(os.environ.get("G", 40000))
roles = bench.STEP_ROLES["step"]
g, m, cids = bench.step_groups(hq, G, 1, 1, roles)
nv = sum(r != "observer" for r in roles)
grp, off, ev = bench.step_events(hq, G, 0, roles)
X = 4
per = np.diff(off).astype(np.int64)
odd = ((np.arange(G) % 2) == 1).astype(np.int64)
new_off = np.zeros(G + 1, np.uint64)
new_off[1:] = np.cumsum(per + X * odd)
new_ev = np.zeros(int(new_off[-1]), hq.EVENT_DTYPE)
new_ev[np.arange(len(ev)) + np.repeat(X * np.cumsum(odd), per)] = ev
first = new_off[:-1][odd == 1].astype(np.int64)
new_ev["kind"][first] = hq.EV_CHECK_QUORUM
for k in range(1, X):
    new_ev["kind"][first + k] = hq.EV_PROPOSE
    new_ev["log_index"][first + k] = 1
data, sz = hq.encode_events_sized(new_off, new_ev)
pin = hq.Context(0)
for variant in ("slots+small-first", "slots", "compact+small-first"):
    slots = variant.startswith("slots")
    a = hq.Worker(0, nv, on_device=True, commit_advance=True, ready_compact=True, ready_slots=slots)
    b = hq.Worker(0, nv, on_device=True, commit_advance=True)
    a.add_groups(g, m)
    b.add_groups(g, m)
    if variant.endswith("small-first"):
        a.step_sized(np.array([0], np.uint32), np.zeros(1, np.uint16), 0, np.zeros(0, np.uint8))
    s16 = pin.pinned(G, np.uint16)
    s16[:] = hq.sizes16_of(sz)
    pd = pin.pinned(len(data), np.uint8)
    pd[:] = data
    got = a.step_sized(np.arange(G, dtype=np.uint32), s16, len(new_ev), pd)
    want = b.step_sized(None, sz, len(new_ev), data)
    for k in ("read_resps", "state_changes", "dropped_reads", "deferred", "fallback_groups"):
        bad = np.nonzero(got[k] != want[k])[0] if len(got[k]) == len(want[k]) else "len"
        print(variant, k, len(got[k]), len(want[k]), "bad at", bad[:5] if not isinstance(bad, str) else bad,
              got[k][bad[:2]] if not isinstance(bad, str) and len(bad) else "", flush=True)
    r = hq.merge_ready(got, cids, g["committed"])
    print(variant, "ready equal", np.array_equal(r, want["ready"]), "slotted",
          len(got.get("ready_slots", ())), "list", len(got.get("ready_compact", ())), flush=True)
    a.close()
    b.close()
pin.close()
