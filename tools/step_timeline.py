"""Device timeline of the last step of tools/step_probe.py under
`rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d DIR -o run`: the step's
window (first copy / kernel of the last step to the last end), the host-to-device copies (bytes,
their busy union, the link rate over it), the kernels (busy union, per kind), and how the window
splits into copy-only, kernel-only, both and idle time — where W concurrent workers lose against
one. Usage: step_timeline.py DIR STEPS [W]"""
import csv
import os
import sys


def load(d, name):
    p = os.path.join(d, f"run_{name}.csv")
    return list(csv.DictReader(open(p))) if os.path.exists(p) else []


def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def length(iv):
    return sum(b - a for a, b in iv)


def intersect(x, y):
    i = j = 0
    out = []
    while i < len(x) and j < len(y):
        a, b = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
        if a < b:
            out.append([a, b])
        if x[i][1] < y[j][1]:
            i += 1
        else:
            j += 1
    return out


def main(d, steps, W=1):
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
          for r in load(d, "kernel_trace")]
    cs = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", ""),
           int(r.get("Size", 0) or 0)) for r in load(d, "memory_copy_trace")]
    in_mb = float(os.environ.get("INPUT_MB", 0))    # the trace has no copy sizes: the step's input
    # pass B launches (k_step<true, ...>) end each worker's step: the last step's window opens
    # after the previous step's last pass B of every worker
    pb = sorted(e for a, e, n in ks if "k_step<true" in n or "k_step_jobs<true" in n)
    if len(pb) < steps:
        print(f"expected >= {steps} pass-B launches, found {len(pb)}")
    # the host builds the next step's events between steps (milliseconds with no device
    # activity): the window opens at the first copy or kernel after the last such gap
    t_close = pb[-1]
    acts = sorted([(a, b) for a, b, _ in ks] + [(a, b) for a, b, _, _ in cs])
    t_open, reach = acts[0][0], acts[0][1]
    for a, b in acts:
        if a > t_close:
            break
        if a - reach > 1_000_000:
            t_open = a
        reach = max(reach, b)
    kl = [(max(a, t_open), min(b, t_close), n) for a, b, n in ks if b > t_open and a < t_close]
    cl = [(max(a, t_open), min(b, t_close), dr, sz) for a, b, dr, sz in cs
          if b > t_open and a < t_close]
    win = (t_close - t_open) / 1e3
    ku = union([[a, b] for a, b, _ in kl])
    h2d = [c for c in cl if "HOST_TO_DEVICE" in c[2]]
    cu = union([[a, b] for a, b, _, _ in h2d])
    both = length(intersect(ku, cu))
    print(f"last step window {win:.1f} us (W={W})")
    nb = sum(sz for _, _, _, sz in h2d) or in_mb * 1e6
    print(f"  H2D copies: {len(h2d)}, {nb / 1e6:.2f} MB, busy {length(cu) / 1e3:.1f} us "
          f"({nb / max(length(cu), 1):.1f} GB/s while busy, {nb / max(t_close - t_open, 1):.1f} "
          f"GB/s over the window)")
    per = {}
    for a, b, n in kl:
        k = n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:48]
        per.setdefault(k, []).append(b - a)
    print(f"  kernels busy {length(ku) / 1e3:.1f} us")
    for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"    {k:48s} {len(v):4d} launches, {sum(v) / 1e3:8.1f} us summed, "
              f"{sum(v) / len(v) / 1e3:7.1f} us avg")
    t = t_close - t_open
    print(f"  copy only {(length(cu) - both) / 1e3:.1f} us, kernel only {(length(ku) - both) / 1e3:.1f} "
          f"us, both {both / 1e3:.1f} us, neither {(t - length(cu) - length(ku) + both) / 1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 1)
