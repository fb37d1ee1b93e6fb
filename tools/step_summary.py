"""Print the step legs (step, step5) of a bench.py JSON line: events/s per feed and worker count,
the CPU replay beside them, and parity."""
import json
import sys


def walk(o):
    if isinstance(o, dict):
        if "cpu_reference" in o and "concurrent_workers" in o:
            yield o
            return
        for v in o.values():
            yield from walk(v)
    elif isinstance(o, list):
        for v in o:
            yield from walk(v)


line = [x for x in open(sys.argv[1]).read().splitlines() if x.startswith("{")][-1]
for x in walk(json.loads(line)):
    print(x["workload"][:70])
    print(f"  {'device_stream 1':26s} {x['value']:.3e} ev/s  {x['ms_per_step']:.2f} ms/step  "
          f"{x.get('stream_bytes_per_event', 0):.2f} B/event")
    for k in ("concurrent_workers", "device_rows", "device_rows_concurrent", "host_worker",
              "host_worker_concurrent"):
        y = x[k]
        print(f"  {k:26s} {y['value']:.3e} ev/s  {y['ms_per_step']:.2f} ms/step")
    c = x["cpu_reference"]
    print(f"  cpu replay {c['value']:.3e} (16 thr) {c['single_thread_value']:.3e} (1 thr); "
          f"parity {x.get('parity_committed')}")
    print("  vs replay:", {k: round(v, 2) for k, v in x["vs_cpu_replay"].items()})
