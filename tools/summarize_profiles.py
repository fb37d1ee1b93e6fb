#!/usr/bin/env python3
"""Condense the rocprofv3 outputs of tools/profile_bench.sh into profiles/<round>/ and update
profiles/pmc_traffic.json (read by bench.py for roofline.traffic).

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024, the gfx950 correction of
MI355X_MICROARCH.md §HBM: FETCH_SIZE reports half of a wide (16 B/lane) coalesced streaming read;
WRITE_SIZE is exact for 16 B/lane stores. Both counters are per-dispatch kilobytes.

usage: python tools/summarize_profiles.py r01 c2 c3m ...
"""
import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = {"c2": "k_commit_big<3, 0, 2, false, 0>", "c2t": "k_commit_big<3, 0, 2, false, 1>",
          "c3": "k_commit_big<5, 1, 2, false, 0>", "c3m": "k_commit_big<5, 2, 2, false, 0>",
          "c3mt": "k_commit_big<5, 2, 2, false, 1>",
          "c2tl": "k_commit_big<3, 0, 2, false, 2>", "c3mtl": "k_commit_big<5, 2, 2, false, 2>",
          "c5v5tl": "k_commit_big<5, 2, 2, false, 2>", "c5tl": "k_commit_fused<2, 512, 2>",
          "c3r32": "k_commit_big<5, 3, 2, false, 0>",
          "c3r32t": "k_commit_big<5, 3, 2, false, 1>",
          "c5v5t": "k_commit_big<5, 2, 2, false, 1>",
          "c5v5r32t": "k_commit_big<5, 3, 2, false, 1>",
          "c4": "k_bits<3, true, 256, false, true>", "c4u": "k_bits<3, false, 256, false, true>",
          "c4t": "k_bits<3, true, 256, true, false>", "c4ut": "k_bits<3, false, 256, true, false>", "c5": "k_commit_fused<2, 512, 0>",
          "c5t": "k_commit_fused<2, 512, 1>", "c5s": "k_commit<7, 2, 2, false, 0>",
          "c2l": "k_commit_lag_big<3, 0, 4, false, 0>", "c3l": "k_commit_lag<5, 2, 4, false, 0>",
          "c2ll": "k_commit_lag_big<3, 0, 4, false, 1>", "c5ll": "k_commit_lag_fused<2, 512, 1>",
          "c5l": "k_commit_lag_fused<2, 512, 0>", "rim": "k_ri_multi2<false, false, 4, false>",
          # uniform tiles (K = 4, n = 7): k_ri_tiles_u since r04d; rimtc without released_index
          "rimt": "k_ri_tiles_u<4, 7>", "rimtc": "k_ri_tiles_u<4, 7>",
          "cq": "k_bits<4, false, 256, false, true>", "cqp": "k_cq_planes<6, false, 256>",
          "ing": ("k_bin<false>", "k_apply<false>"), "c4pq": "k_planes_cq<256>",
          "ingo": "k_table_ingest<1, false>", "rim2": "k_ri_multi2",
          "c4t3": "k_bits3<256>", "c4p": "k_planes<256>"}


# headline workloads decided by fused launches (bench.py --mode fused): a dispatch holds several
# batches, grid threads per batch below; the kernel time and the counters are per batch (a step)
FUSED_THREADS_PER_BATCH = {"c3mtl": 524288}
KERNEL_FUSED = {"c3mtl": "k_commit_fused<2, 1024, 2>"}


# the default line's headline mode "engine" (bench.py run_engine): the persistent engine's launch
# per timed window of --steps steps; its dispatches are the warm-up (warmup steps), the timed
# windows (steps each, in order) and the parity launch (1 step). Per step: a window dispatch's
# duration or counter over its steps.
KERNEL_ENGINE = {"c3mtl-engine": ("c3mtl", "k_commit_engine<5, 2, 1, false, 1024, false, false>")}
ENGINE_STEPS, ENGINE_WARMUP, ENGINE_WINDOWS = 20, 5, 3


def engine_windows(path, kernel, value_key):
    """per-step values of the timed-window dispatches (2nd .. windows + 1st of the kernel's)."""
    rows = [r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0))
    wins = rows[1:1 + ENGINE_WINDOWS]
    return [value_key(r) / ENGINE_STEPS for r in wins], len(rows)


def per_batch(path, kernel, tpb, value_key, grid_key):
    """sum over the kernel's dispatches of value / sum of their batches (grid / tpb)."""
    rows = [r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]
    batches = sum(int(r[grid_key]) // tpb for r in rows)
    return sum(value_key(r) for r in rows) / batches, len(rows), batches


def counter(path, kernel):
    rows = list(csv.DictReader(open(path)))
    vals = [float(r["Counter_Value"]) for r in rows if kernel in r["Kernel_Name"]]
    return statistics.median(vals), len(vals)


def main():
    rnd, workloads = sys.argv[1], sys.argv[2:]
    dst = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dst, exist_ok=True)
    tj = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    traffic = json.load(open(tj)) if os.path.exists(tj) else {}
    for w in workloads:
        src = os.path.join(ROOT, "gpurun_out", f"prof_{w}")
        if w in KERNEL_ENGINE:
            base, k = KERNEL_ENGINE[w]
            for f, name in (("trace/run_kernel_stats.csv", f"{w}_kernel_stats.csv"),
                            ("trace/run_kernel_trace.csv", f"{w}_kernel_trace.csv"),
                            ("pmc_FETCH_SIZE/run_counter_collection.csv", f"{w}_pmc_FETCH_SIZE.csv"),
                            ("pmc_WRITE_SIZE/run_counter_collection.csv", f"{w}_pmc_WRITE_SIZE.csv"),
                            ("trace_stdout.log", f"{w}_bench_line.log")):
                shutil.copy(os.path.join(src, f), os.path.join(dst, name))
            ns, nd = engine_windows(os.path.join(dst, f"{w}_kernel_trace.csv"), k,
                                    lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            fetch, nf = engine_windows(os.path.join(dst, f"{w}_pmc_FETCH_SIZE.csv"), k,
                                       lambda r: float(r["Counter_Value"]))
            write, nw = engine_windows(os.path.join(dst, f"{w}_pmc_WRITE_SIZE.csv"), k,
                                       lambda r: float(r["Counter_Value"]))
            f_med, w_med = statistics.median(fetch), statistics.median(write)
            traffic[w] = {
                "kernel": k, "mode": "engine",
                "rocprof_window_ns_per_step": ns, "rocprof_avg_ns": statistics.median(ns),
                "rocprof_calls": nd, "steps_per_window": ENGINE_STEPS,
                "fetch_size_kb_median": f_med, "write_size_kb_median": w_med,
                "dispatches": min(nf, nw),
                "hbm_bytes_per_launch": (2 * f_med + w_med) * 1024,
                "per": f"step (one step of 1 M groups; a window launch decides {ENGINE_STEPS})",
                "correction": "(2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950 FETCH_SIZE halves 16B/lane "
                              "streams)",
                "round": rnd,
                "source": f"profiles/{rnd}/{w}_pmc_FETCH_SIZE.csv + {w}_pmc_WRITE_SIZE.csv "
                          f"(kernel time: {w}_kernel_trace.csv, the timed windows' launches / "
                          f"{ENGINE_STEPS} steps)",
            }
            print(w, json.dumps(traffic[w]))
            continue
        if w in FUSED_THREADS_PER_BATCH:
            tpb, k = FUSED_THREADS_PER_BATCH[w], KERNEL_FUSED[w]
            for f, name in (("trace/run_kernel_stats.csv", f"{w}_kernel_stats.csv"),
                            ("trace/run_kernel_trace.csv", f"{w}_kernel_trace.csv"),
                            ("pmc_FETCH_SIZE/run_counter_collection.csv", f"{w}_pmc_FETCH_SIZE.csv"),
                            ("pmc_WRITE_SIZE/run_counter_collection.csv", f"{w}_pmc_WRITE_SIZE.csv")):
                shutil.copy(os.path.join(src, f), os.path.join(dst, name))
            ns, nd, nb = per_batch(os.path.join(dst, f"{w}_kernel_trace.csv"), k, tpb,
                                   lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                   "Grid_Size_X")
            fetch, nf, _ = per_batch(os.path.join(dst, f"{w}_pmc_FETCH_SIZE.csv"), k, tpb,
                                     lambda r: float(r["Counter_Value"]), "Grid_Size")
            write, nw, _ = per_batch(os.path.join(dst, f"{w}_pmc_WRITE_SIZE.csv"), k, tpb,
                                     lambda r: float(r["Counter_Value"]), "Grid_Size")
            traffic[w] = {
                "kernel": k, "rocprof_avg_ns": ns, "rocprof_calls": nd, "rocprof_batches": nb,
                "fetch_size_kb_median": fetch, "write_size_kb_median": write,
                "dispatches": min(nf, nw),
                "hbm_bytes_per_launch": (2 * fetch + write) * 1024,
                "per": "batch (one step of 1 M groups; a fused dispatch decides several)",
                "correction": "(2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950 FETCH_SIZE halves 16B/lane "
                              "streams)",
                "round": rnd,
                "source": f"profiles/{rnd}/{w}_pmc_FETCH_SIZE.csv + {w}_pmc_WRITE_SIZE.csv "
                          f"(kernel time: {w}_kernel_trace.csv, per batch)",
            }
            print(w, json.dumps(traffic[w]))
            continue
        ks = KERNEL[w] if isinstance(KERNEL[w], tuple) else (KERNEL[w],)   # a step's kernels
        k = " + ".join(ks)
        shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                    os.path.join(dst, f"{w}_kernel_stats.csv"))
        stats = {r["Name"]: r for r in csv.DictReader(open(os.path.join(dst, f"{w}_kernel_stats.csv")))}
        rows = [next(v for n, v in stats.items() if kk in n) for kk in ks]
        row = {"AverageNs": sum(float(r["AverageNs"]) for r in rows),
               "Calls": min(int(r["Calls"]) for r in rows)}
        fc = [counter(os.path.join(src, "pmc_FETCH_SIZE", "run_counter_collection.csv"), kk)
              for kk in ks]
        wc = [counter(os.path.join(src, "pmc_WRITE_SIZE", "run_counter_collection.csv"), kk)
              for kk in ks]
        fetch, nf = sum(v for v, _ in fc), min(n for _, n in fc)
        write, nw = sum(v for v, _ in wc), min(n for _, n in wc)
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            shutil.copy(os.path.join(src, f"pmc_{c}", "run_counter_collection.csv"),
                        os.path.join(dst, f"{w}_pmc_{c}.csv"))
        hbm = (2 * fetch + write) * 1024
        traffic[w] = {
            "kernel": k,
            "rocprof_avg_ns": float(row["AverageNs"]),
            "rocprof_calls": int(row["Calls"]),
            "fetch_size_kb_median": fetch,
            "write_size_kb_median": write,
            "dispatches": min(nf, nw),
            "hbm_bytes_per_launch": hbm,
            "correction": "(2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950 FETCH_SIZE halves 16B/lane streams)",
            "round": rnd,
            "source": f"profiles/{rnd}/{w}_pmc_FETCH_SIZE.csv + {w}_pmc_WRITE_SIZE.csv "
                      f"(kernel time: {w}_kernel_stats.csv)",
        }
        print(w, json.dumps(traffic[w]))
    json.dump(traffic, open(tj, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
