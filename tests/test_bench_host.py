"""bench.py host logic that needs no GPU: the step leg's in-place row advance equals a fresh
generation, the launcher-free multi-GPU plumbing (one host thread per GPU, ThreadDist
collectives) and the final JSON line's shape and size (the driver parses it: <= 8 KB)."""
import argparse
import io
import json
import threading
from contextlib import redirect_stdout

import numpy as np
import pytest

import bench


@pytest.mark.parametrize("name", ["step", "step5"])
def test_step_rows_advance_equals_generation(hq, name):
    roles = bench.STEP_ROLES[name]
    G = 1 << 10
    rows = bench.StepRows(hq, G, roles)
    for s in (0, 5, 1, 2, 40):
        rows.set(s)
        want = bench.step_events(hq, G, s, roles)
        assert np.array_equal(rows.offsets, want[1])
        assert rows.ev.tobytes() == want[2].tobytes(), (name, s)


@pytest.mark.parametrize("name", ["step", "step5"])
def test_step_rows16_follow_step_events(hq, name):
    """The producer's compact records advanced in place (StepRows16.set) are hq_events_to16 of
    step_events() of the same step, and encode (16 threads) to the rows' bytes."""
    G = 1 << 10
    roles = bench.STEP_ROLES[name]
    recs = bench.StepRows16(hq, G, roles)
    for s in (0, 5, 1, 2, 40):
        off16, r = recs.set(s)
        _, off, ev = bench.step_events(hq, G, s, roles)
        want, woff = hq.events_to16(off, ev)
        assert np.array_equal(off16, woff) and r.tobytes() == want.tobytes(), (name, s)
        data, sizes, ne = hq.encode_events16_sized(off16, r, threads=16)
        wdata, wsizes = hq.encode_events_sized(off, ev)
        assert ne == len(ev) and data.tobytes() == wdata.tobytes()
        assert np.array_equal(sizes, wsizes)


def test_encode_into_matches_encode(hq):
    G = 1 << 9
    rows = bench.StepRows(hq, G, bench.STEP_ROLES["step5"])
    rows.set(3)
    data, sizes = hq.encode_events_sized(rows.offsets, rows.ev)
    out = np.zeros(len(rows.ev) * 5 + 64, np.uint8)
    sz = np.zeros(G, np.uint32)
    nb = hq.encode_events_sized_into(rows.offsets, rows.ev, out, sz)
    assert nb == len(data) and out[:nb].tobytes() == data.tobytes()
    assert np.array_equal(sz, sizes)
    with pytest.raises(hq.HQError):      # too small: HQ_E_STATE, never a write past the end
        hq.encode_events_sized_into(rows.offsets, rows.ev, np.zeros(100, np.uint8), sz)


def _in_threads(n, fn):
    grp = bench.ThreadGroup(n)
    ds = [bench.ThreadDist(grp, i, ngpu=1) for i in range(n)]
    out, errs = [None] * n, []

    def body(i):
        try:
            out[i] = fn(ds[i])
        except BaseException as e:
            errs.append(e)
            grp.bar.abort()
    ts = [threading.Thread(target=body, args=(i,)) for i in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
    return ds, out


@pytest.mark.parametrize("n", [2, 3])
def test_thread_dist_collectives(n):
    def fn(d):
        d.barrier()
        return (d.max(float(d.rank)), d.sum(float(d.rank + 1)), d.gather([d.rank, 2 * d.rank]),
                d.gather_obj({"r": d.rank}), d.device)
    ds, out = _in_threads(n, fn)
    for r, (mx, sm, ga, go, dev) in enumerate(out):
        assert mx == n - 1 and sm == n * (n + 1) / 2
        assert ga == [[i, 2 * i] for i in range(n)]
        assert go == [{"r": i} for i in range(n)]
        assert dev == 0              # one visible GPU: every rank wraps onto it (rehearsal)
    assert [d.world for d in ds] == [n] * n


def _args(**kw):
    a = dict(gpus=2, steps=5, warmup=1, workload=bench.HEADLINE, step_groups=1 << 10,
             step_steps=2, no_cpu=True, no_extra_parity=True, extra="", detail_out=None,
             mode="fused", windows=3)
    a.update(kw)
    return argparse.Namespace(**a)


def _fake_rank(args, d, progress):
    """run_rank's result shape, with the ranks' collectives exercised the way run_gpu uses
    them (the per-GPU gather, the node sums, the max over ranks)."""
    G = bench.WORKLOADS[args.workload]["G"]
    elapsed = d.max(1e-3 * (1 + d.rank))
    per_gpu = d.gather([1e9, 11.5, 5000.0])
    r = dict(elapsed=elapsed, launches=args.steps, avg_kernel_s=11.5e-6,
             decisions=d.sum(float(G * args.steps)), nsets=20, first_timed_set=1,
             bytes_per_launch=58 * G, launches_per_step=1, steps=args.steps,
             achieved_gbs=5000.0, achieved_node_gbs=d.sum(5000.0), per_gpu=per_gpu,
             gather=None, world=d.world)
    devices = d.gather_obj({"rank": d.rank, "device": d.device, "pci_bus_id": ""})
    records = [dict(name=f"x{i}", workload="w" * 300, value=1.0e10 + i, unit="decisions/s",
                    roofline_frac=0.7, kernel_avg_us=10.0, step_ms=list(range(200)))
               for i in range(60)]
    return dict(r=r, devices=devices, records=records, cpu=None, forms=[])


def test_main_threads_prints_one_parseable_line(monkeypatch, tmp_path, hq):
    monkeypatch.setattr(bench, "run_rank", _fake_rank)
    monkeypatch.setattr(hq, "device_count", lambda: 1)
    args = _args(detail_out=str(tmp_path / "detail.json"))
    buf = io.StringIO()
    with redirect_stdout(buf):
        bench.main_threads(args, 0.0)
    lines = buf.getvalue().strip().splitlines()
    assert len(lines) == 1
    assert len(lines[0]) <= 8000
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["launcher"].startswith("threads")
    assert len(line["per_gpu"]) == 2
    G = bench.WORKLOADS[bench.HEADLINE]["G"]
    # value = every rank's decisions / the slowest rank's time
    assert line["value"] == pytest.approx(2 * G * 5 / 2e-3)
    assert line["roofline"]["frac"] == pytest.approx(10000.0 / 16000.0)
    detail = json.load(open(tmp_path / "detail.json"))
    assert len(detail["extra"]) == 60 and detail["extra"][0]["step_ms"][-1] == 199


def test_main_threads_rank_failure_releases_the_others(monkeypatch, tmp_path, hq):
    def bad(args, d, progress):
        if d.rank == 1:
            raise ValueError("boom")
        d.barrier()           # would wait forever without the abort
        return None
    monkeypatch.setattr(bench, "run_rank", bad)
    monkeypatch.setattr(hq, "device_count", lambda: 1)
    with pytest.raises(RuntimeError, match="rank 1 failed"):
        bench.main_threads(_args(detail_out=str(tmp_path / "d.json")), 0.0)


def _oracle_set0(w, d, corrupt=False):
    """What run_engine / run_gpu hand to the parity check, made by the oracle itself on the CPU
    (a small shard of the headline workload per rank)."""
    from dragonboat_amd import shard
    from oracle import qref

    rng = shard.rank_shard(d.rank, d.world, w["G"])
    s = qref.spec(bench.SEED_BASE + w["cfg"], rng.count, w["n"], cid_base=rng.cid_base,
                  cid_stride=rng.cid_stride)
    out, chg, fb, rc = qref.CommitInputs(s).run(w["form"], False, nthreads=2)
    assert rc == 0
    if corrupt:
        out = out.copy()
        out[7] += np.uint64(1)
    return [dict(n=w["n"], cid_base=rng.cid_base, cid_stride=rng.cid_stride, count=rng.count,
                 out=[out, chg, fb])]


@pytest.mark.parametrize("n", [2, 3])
def test_rank_parity_checks_every_rank(n):
    """at N > 1 every rank's set 0 is checked against the oracle (no
    world == 1 gate) and every rank's verdict reaches rank 0; a wrong decision on one rank
    shows on that rank only."""
    w = dict(bench.WORKLOADS[bench.HEADLINE], G=3 * 4096 + 5)

    def fn(d):
        r = {"set0": _oracle_set0(w, d, corrupt=(d.rank == 1))}
        return bench.rank_parity(w, r, d, no_cpu=False)
    ds, out = _in_threads(n, fn)
    for rank, r in enumerate(out):
        assert r["parity"]["equal"] == (rank != 1)
        assert [p["equal"] for p in r["parity_by_rank"]] == [i != 1 for i in range(n)]
        assert sum(p["groups"] for p in r["parity_by_rank"]) == n * w["G"]   # weak scaling
    # --no-cpu: no check, and the line says so (None), never a silent "equal"
    _, out = _in_threads(n, lambda d: bench.rank_parity(w, {"set0": None}, d, no_cpu=True))
    assert all(r["parity_by_rank"] == [None] * n for r in out)


def test_host_cores_reports_counts():
    visible, usable, quota = bench.host_cores()
    assert visible >= 1 and 1 <= usable <= visible
    allc, counts = bench.cpu_thread_counts()
    assert counts[0] == allc and counts[-1] == 1 and 1 <= allc <= usable


def test_fused_chunks_cover_the_window():
    """The fused headline's launches: at most 32 batches each (hq_commit_fused_dev's limit), as
    even as possible, covering the window once in order."""
    for steps in (1, 2, 20, 32, 33, 64, 400):
        ch = bench.fused_chunks(steps)
        assert ch[0][0] == 0 and all(n <= 32 for _, n in ch)
        assert all(a + n == b for (a, n), (b, _) in zip(ch, ch[1:]))
        assert ch[-1][0] + ch[-1][1] == steps and len(ch) == -(-steps // 32)
        assert max(n for _, n in ch) - min(n for _, n in ch) <= 1
