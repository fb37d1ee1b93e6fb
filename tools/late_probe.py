"""Probe: the late-starting device steps of the step legs' end-to-end timing (BENCH_r05 / r06e:
a step whose GPU time and device span are normal but whose first kernel ran milliseconds after the
host had queued it). One step5-shaped worker (W = 1, 1 M leader groups), STEPS steps per mode:

  dev    the step alone (its stream encoded beforehand)
  seq    the producer's encode, then the step, on one thread
  conc   the step on a pool thread while the producer encodes the next step (bench's e2e)
  plain  as conc, but the encode writes ordinary (pageable) memory, not the pinned buffers
  sleep  as conc, with the wait policy `sleep` instead of `block`
  gap    as the bench's step legs: before each step GAP s without GPU work (the CPU replays'
         time), then the step alone (dev) and then the step beside the encode (conc) — the row
         is the conc step's
  busy   as gap, the GPU idle for GAP s while the encode threads run (the replays' CPU load)
  churn  as the bench's second step leg: CHURN workers opened, stepped once together and closed
         (the first leg's teardown), then fresh workers stepped alone and beside the encode as in
         `gap` without the gap; CHURN_ROUNDS times

Per mode: the start lag of every step (the wait beyond the device's own span: poll + sleep -
span), how many steps started > 0.5 ms late, the worst, and the e2e p50 / p99. Prints one JSON
line per mode."""
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from dragonboat_amd import hipquorum as hq  # noqa: E402

G = int(os.environ.get("G", 1 << 20))
STEPS = int(os.environ.get("STEPS", 100))
GAP = float(os.environ.get("GAP", 1.0))
GAP_STEPS = int(os.environ.get("GAP_STEPS", 30))
# AB=8,1: the conc modes alternate HQ_ENC_CHUNKS over these values step by step (the encode
# profiling build reads it at every call); each row records the value its encode ran with
AB = [x for x in os.environ.get("AB", "").split(",") if x]
MODES = os.environ.get("MODES", "dev,seq,conc,plain,sleep").split(",")
roles = bench.STEP_ROLES["step5"]
nv = sum(r != "observer" for r in roles)
nm = len(roles)
g, m, cids = bench.step_groups(hq, G, 1, 1, roles)
recs = bench.StepRows16(hq, G, roles)
enc_threads = bench.encode_threads()
pin = hq.Context(0)
ne = len(recs.recs)
bufs = [(pin.pinned(ne * 5 + 64, np.uint8), pin.pinned(G, np.uint16)) for _ in range(2)]
plain = (np.zeros(ne * 5 + 64, np.uint8), np.zeros(G, np.uint16))
off = recs.offsets
batch = {k: hq.Encode16Batch([(off, recs.recs, b[0], b[1])]) for k, b in
         (("p0", bufs[0]), ("p1", bufs[1]), ("plain", plain))}
pool = ThreadPoolExecutor(2)
print(json.dumps({"G": G, "steps": STEPS, "encode_threads": enc_threads,
                  "cpus": bench.host_cores()}), flush=True)


def churn():
    """CHURN workers of the same groups opened, stepped once as one jobs call (each its own
    pinned stream copy) and closed."""
    recs.set(0)                            # (slot 0 holds a fresh step-0 stream)
    NB0[0] = batch["p0"].run(enc_threads)[0][1]
    ws = []
    for _ in range(int(os.environ.get("CHURN", 18))):
        x = hq.Worker(0, nv, on_device=True, commit_column=True, commit_advance=True,
                      ready_compact=True, ready_slots=True)
        x.add_groups(g, m)
        ws.append(x)
    hq.StepJobs([(x, hq.SizedStream(None, bufs[0][1], ne, bufs[0][0][:NB0[0]])) for x in ws]).execute()
    for x in ws:
        x.close()


NB0 = [0]


def run_mode(mode):
    wk = hq.Worker(0, nv, on_device=True, commit_column=True, commit_advance=True,
                   ready_compact=True, ready_slots=True)
    pol = hq.HQ_WAIT_SLEEP if mode == "sleep" else hq.HQ_WAIT_BLOCK
    wk.set_wait(pol, 50, 20, clock=True)
    wk.add_groups(g, m)
    wk2 = None
    if mode in ("gap", "busy", "churn"):
        wk2 = hq.Worker(0, nv, on_device=True, commit_column=True, commit_advance=True,
                        ready_compact=True, ready_slots=True)
        wk2.set_wait(pol, 50, 20, clock=True)
        wk2.add_groups(g, m)
    nbytes = [0, 0]

    def encode(slot, dst=None):
        t0 = time.perf_counter()
        (n_e, nb), = batch[dst or f"p{slot}"].run(enc_threads)
        if dst is None:
            nbytes[slot] = nb
        return time.perf_counter() - t0

    def job(slot):
        return hq.StepJobs([(wk, hq.SizedStream(None, bufs[slot][1], ne, bufs[slot][0][:nbytes[slot]]))])

    recs.set(0)
    encode(0)
    NB0[0] = nbytes[0]
    rows = []
    for s in range((GAP_STEPS if mode in ("gap", "busy", "churn") else STEPS) + 3):
        slot = s % 2
        recs.set(s + 1)
        j = job(slot)
        if mode in ("gap", "busy", "churn"):
            tg = time.perf_counter()
            if mode == "churn":
                pass
            elif mode == "gap":
                time.sleep(GAP)
            else:
                while time.perf_counter() - tg < GAP:
                    encode(1 - slot, "plain")
            # the step alone first on the bench's other worker (its device-only timing)
            hq.StepJobs([(wk2, hq.SizedStream(None, bufs[slot][1], ne,
                                              bufs[slot][0][:nbytes[slot]]))]).execute()
        t0 = time.perf_counter()
        enc = 0.0
        if mode == "dev":
            j.execute()
            dt = time.perf_counter() - t0
            encode(1 - slot)               # (outside the step's time)
        elif mode == "seq":
            j.execute()
            enc = encode(1 - slot)
            dt = time.perf_counter() - t0
        else:
            fut = pool.submit(j.execute)
            if mode in ("plain",):
                enc = encode(1 - slot, "plain")
                encode(1 - slot)           # (the next step's real stream, after the timed part)
            else:
                if AB:                     # alternate the encoder's chunking step by step
                    os.environ["HQ_ENC_CHUNKS"] = AB[s % len(AB)]
                enc = encode(1 - slot)
            fut.result()
            dt = time.perf_counter() - t0
        r = max(j.results(copy=False), key=lambda x: x["pass_ns"])
        span = (r["device_end_ticks"] - r["device_start_ticks"]) / 1e5 \
            if r["device_start_ticks"] and r["device_end_ticks"] else None
        wait = (r["wait_poll_ns"] + r["wait_sleep_ns"]) / 1e6
        if s >= 3 or mode == "churn":      # (churn: the first steps after the teardown too)
            rows.append({"s": s - 3, "k": AB[s % len(AB)] if AB else None,
                         "e2e": dt * 1e3, "enc": enc * 1e3, "gpu": r["gpu_ns"] / 1e6,
                         "span": span, "wait": wait, "submit": r["pack_ns"] / 1e6,
                         "lag": (wait - span) if span is not None else None})
    wk.close()
    if wk2 is not None:
        wk2.close()
    lags = np.array([x["lag"] for x in rows if x["lag"] is not None])
    e2e = np.array([x["e2e"] for x in rows])
    late = [x for x in rows if x["lag"] is not None and x["lag"] > 0.5]
    out = {"mode": mode, "n": len(rows), "late_gt_0p5ms": len(late),
           "lag_p50": round(float(np.median(lags)), 4), "lag_max": round(float(lags.max()), 3),
           "e2e_p50": round(float(np.percentile(e2e, 50)), 3),
           "e2e_p99": round(float(np.percentile(e2e, 99)), 3),
           "gpu_p50": round(float(np.median([x["gpu"] for x in rows])), 4),
           "late": [{k: (round(v, 3) if isinstance(v, float) else v) for k, v in x.items()}
                    for x in late[:8]]}
    if os.environ.get("ROWS"):
        out["rows"] = [{k: (round(v, 3) if isinstance(v, float) else v) for k, v in x.items()}
                       for x in rows]
    print(json.dumps(out), flush=True)


for md in MODES:
    if md == "churn":
        for _ in range(int(os.environ.get("CHURN_ROUNDS", 3))):
            churn()
            run_mode(md)
    else:
        run_mode(md)
pool.shutdown()
pin.close()
