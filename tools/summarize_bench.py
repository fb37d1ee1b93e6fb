"""Print a compact table of a bench.py JSON line (headline + extras)."""
import json
import sys

line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
r = json.loads(line)
rf = r["roofline"]
print(f"headline {r['config']['workload'][:60]}: {r['value']:.3e} {r['unit']}  "
      f"{rf['kernel_avg_us']:.2f} us  {rf['achieved']:.0f} GB/s  frac {rf['frac']:.3f}")
if r.get("cpu_baseline"):
    c = r["cpu_baseline"]
    print(f"cpu_baseline {c['value']:.3e} ({c['cores']} cores), 1 thread {c['single_thread_value']:.3e}")
for e in r["extra"]:
    keys = [k for k in ("value", "kernel_avg_us", "launches_per_step", "roofline_achieved_gbs",
                        "roofline_frac", "aggregate_gbs", "aggregate_frac_of_peak", "ms_per_step")
            if k in e]
    print(e["workload"][:40], " ".join(f"{k}={e[k]:.4g}" for k in keys))
