"""Probe: the host-fed pipeline (bench.py e2e leg) at several step counts, or one variant
(VARIANT=depth,compact,grouped) for a rocprofv3 timeline; prints ms per step."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

d = bench.Dist()
var = os.environ.get("VARIANT")
variants = (tuple(bool(int(x)) if i else int(x) for i, x in enumerate(var.split(","))),) \
    if var else None
for steps in [int(x) for x in os.environ.get("STEPS", "20,100,20,50").split(",")]:
    r = bench.run_e2e(steps, 3, d, variants=variants)
    print(steps, round(r.get("ms_per_step", 0), 3),
          {k: round(v["ms_per_step"], 3) for k, v in r.items() if isinstance(v, dict)}, flush=True)
