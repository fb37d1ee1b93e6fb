"""Round 6 forms of the device step (hq_dstep.hip) against the forms they replace, bit for bit:

* HQ_WORKER_READY_SLOTS — the single ReadyToReads written by pass A into per-tile slots (the
  reference's consumer is node.processReadyToRead, node.go:1026-1031): merged with the list by
  group position they must be the 32-byte records of a worker without the flag, in order;
* 2-byte size words (hq_step_stream.sizes16: bytes only, the engine counts the events): every
  output, deferred event indexes included, equal to the 4-byte words' step;
* the wait policies (hq_worker_set_wait) and the look-back give-up path (kErrScan re-run).

The oracle-level equality of these paths over the reference's scenarios and random streams is in
tests/test_gpu_worker.py (feeds "device-sized16", "host-sized16", "device-sized16-slots")."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LISTS = ("read_resps", "state_changes", "dropped_reads", "deferred", "fallback_groups")


def _pinned(ctx, a):
    p = ctx.pinned(len(a), a.dtype)
    p[:] = a
    return p


def _same_outputs(hq, got, want, cids, committed, what):
    """got (any ReadyToRead form) against want (32-byte records), every list and the commits."""
    np.testing.assert_array_equal(hq.merge_ready(got, cids, committed), want["ready"],
                                  err_msg=f"{what}: ready")
    for k in LISTS:
        np.testing.assert_array_equal(got[k], want[k], err_msg=f"{what}: {k}")
    for k in ("committed_advance", "commits"):
        if k in want:
            np.testing.assert_array_equal(got[k], want[k], err_msg=f"{what}: {k}")


def _same_lists(got, want):
    """Every list and the commits (in whichever form both steps returned them) equal."""
    for k in LISTS + ("commits",):
        np.testing.assert_array_equal(got[k], want[k], err_msg=k)
    for k in ("committed_advance", "committed_column"):
        assert (k in got) == (k in want), k
        if k in want:
            np.testing.assert_array_equal(got[k], want[k], err_msg=k)


def _advance(committed, want):
    if "committed_advance" in want:
        committed += want["committed_advance"].astype(np.uint64)
    else:
        ix = want["commits"]["cluster_id"].astype(np.int64) - 1
        committed[ix] = want["commits"]["committed"]


@pytest.mark.parametrize("G", [5000, 4 * 65536 + 5])
def test_slots_equal_records(hq, G):
    """A slots worker (2-byte words, pinned: the jobs path) against a plain worker (4-byte words,
    32-byte records), three steps of the step5 workload; step 2 gives group 8 a ReadIndexResp
    beside its ReadyToRead (replayed by pass B: its record stays in the list)."""
    import bench

    roles = bench.STEP_ROLES["step5"]
    g, m, cids = bench.step_groups(hq, G, 1, 1, roles)
    nv = sum(r != "observer" for r in roles)
    a = hq.Worker(0, nv, on_device=True, commit_advance=True, ready_compact=True, ready_slots=True)
    b = hq.Worker(0, nv, on_device=True, commit_advance=True)
    pin = hq.Context(0)
    committed = g["committed"].astype(np.uint64).copy()
    try:
        a.add_groups(g, m)
        b.add_groups(g, m)
        for s in range(3):
            grp, off, ev = bench.step_events(hq, G, s, roles)
            if s == 2:
                lo = int(off[8])
                fwd = ev[lo + 1].copy()
                fwd["type"], fwd["hint"], fwd["hint_high"], fwd["log_index"] = 19, 99, 0, 0
                ev[lo + 1] = ev[lo]
                ev[lo] = fwd
            data, sz = hq.encode_events_sized(off, ev)
            got = a.step_sized(None, _pinned(pin, hq.sizes16_of(sz)), len(ev), _pinned(pin, data))
            want = b.step_sized(None, sz, len(ev), data)
            assert "ready_slots" in got and len(got["ready_slots"]) > G // 5
            if s == 2:
                assert len(want["read_resps"]) == 1 and len(got["ready_compact"]) == 1
            _same_outputs(hq, got, want, cids, committed, f"step {s}")
            _advance(committed, want)
    finally:
        a.close()
        b.close()
        pin.close()


def test_slots_step_jobs(hq):
    """Three slot workers stepped as one launch sequence (hq_worker_step_jobs) equal three plain
    workers stepped one by one: each worker's slots are its own tiles."""
    import bench

    G, W = 3 * 20000, 3
    roles = bench.STEP_ROLES["step5"]
    g, m, cids = bench.step_groups(hq, G, 1, 1, roles)
    nv, nm = sum(r != "observer" for r in roles), len(roles)
    bounds = [G * i // W for i in range(W + 1)]
    pin = hq.Context(0)
    A = [hq.Worker(0, nv, on_device=True, commit_advance=True, ready_compact=True, ready_slots=True)
         for _ in range(W)]
    B = [hq.Worker(0, nv, on_device=True, commit_advance=True) for _ in range(W)]
    committed = g["committed"].astype(np.uint64).copy()
    try:
        for i in range(W):
            for w in (A[i], B[i]):
                w.add_groups(g[bounds[i]:bounds[i + 1]], m[nm * bounds[i]:nm * bounds[i + 1]])
        for s in range(2):
            grp, off, ev = bench.step_events(hq, G, s, roles)
            jobs, wants = [], []
            for i in range(W):
                o = off[bounds[i]:bounds[i + 1] + 1]
                e = ev[int(o[0]):int(o[-1])]
                data, sz = hq.encode_events_sized(o - o[0], e)
                jobs.append((A[i], hq.SizedStream(None, _pinned(pin, hq.sizes16_of(sz)), len(e),
                                                  _pinned(pin, data))))
                wants.append(B[i].step_sized(None, sz, len(e), data))
            gots = hq.step_jobs(jobs)
            for i in range(W):
                lo, hi = bounds[i], bounds[i + 1]
                assert gots[i]["gpu_jobs"] == W
                _same_outputs(hq, gots[i], wants[i], cids[lo:hi], committed[lo:hi],
                              f"step {s} worker {i}")
                c = committed[lo:hi]
                _advance(c, wants[i])
                committed[lo:hi] = c
    finally:
        for w in A + B:
            w.close()
        pin.close()


def test_slots_wide_delta_stays_in_list(hq):
    """A ReadyToRead whose index lies 2^33 above its group's committed index before the step does
    not fit a slot: it stays in the list (which then holds 32-byte records) while the other
    groups' go to their slots; merged they equal a plain worker's records."""
    import bench

    G, big, special = 8192, 1 << 33, 4
    roles = bench.STEP_ROLES["step"]
    g, m, cids = bench.step_groups(hq, G, 1, 1, roles)
    g["committed"] -= np.uint64(10)
    g["term_start"] = g["committed"]
    m["match"][m["node_id"] != 1] -= np.uint64(10)
    g["last_index"][special] = big
    m["match"][len(roles) * special] = big
    grp, off, ev = bench.step_events(hq, G, 0, roles)
    lo, hi = int(off[special]), int(off[special + 1])
    rows = ev[lo:hi].copy()
    rows["log_index"][(rows["kind"] == hq.EV_MESSAGE) & (rows["type"] == 13)] = big
    k = len(roles) - 1
    ev[lo:hi] = np.concatenate([rows[1:1 + k], rows[:1], rows[1 + k:]])
    data, sz = hq.encode_events_sized(off, ev)
    nv = sum(r != "observer" for r in roles)
    a = hq.Worker(0, nv, on_device=True, commit_advance=True, ready_compact=True, ready_slots=True)
    b = hq.Worker(0, nv, on_device=True, commit_advance=True)
    pin = hq.Context(0)
    try:
        a.add_groups(g, m)
        b.add_groups(g, m)
        committed = g["committed"].astype(np.uint64).copy()
        got = a.step_sized(None, _pinned(pin, hq.sizes16_of(sz)), len(ev), _pinned(pin, data))
        want = b.step_sized(grp, sz, len(ev), data)
        assert "ready_compact" not in got and len(got["ready"]) == 1
        assert int(got["ready"]["cluster_id"][0]) == cids[special]
        assert len(got["ready_slots"]) == G // 4 - 1
        _same_outputs(hq, got, want, cids, committed, "wide")
    finally:
        a.close()
        b.close()
        pin.close()


def test_slots_survive_region_regrow(hq):
    """A step whose lists overflow the host region after pass A wrote the slots into it: the
    region grows and k_step_lite writes the slots again into the new one. Half the groups step
    down on a CheckQuorum (every member inactive) ahead of their events, so their proposals and
    reads are deferred and their state changes listed (> 16 bytes per group: past the margin
    the slot form sizes the region with)."""
    import bench

    G = 40000
    roles = bench.STEP_ROLES["step"]
    g, m, cids = bench.step_groups(hq, G, 1, 1, roles)
    nv = sum(r != "observer" for r in roles)
    grp, off, ev = bench.step_events(hq, G, 0, roles)
    # groups with an odd index: a CHECK_QUORUM (no member active yet: the leader steps down)
    # and three proposals (deferred: a follower forwards them) ahead of their events
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
    a = hq.Worker(0, nv, on_device=True, commit_advance=True, ready_compact=True, ready_slots=True)
    b = hq.Worker(0, nv, on_device=True, commit_advance=True)
    pin = hq.Context(0)
    try:
        a.add_groups(g, m)
        b.add_groups(g, m)
        committed = g["committed"].astype(np.uint64).copy()
        # a first step listing one group (no bytes) sizes the region for one group's lists; the
        # slot step then grows it to the slots + 16 bytes per group, which these lists overflow
        a.step_sized(np.array([0], np.uint32), np.zeros(1, np.uint16), 0, np.zeros(0, np.uint8))
        got = a.step_sized(np.arange(G, dtype=np.uint32), _pinned(pin, hq.sizes16_of(sz)),
                           len(new_ev), _pinned(pin, data))
        want = b.step_sized(None, sz, len(new_ev), data)
        assert len(want["state_changes"]) == G // 2 and len(want["deferred"]) >= 3 * G // 2
        assert "ready_slots" in got and len(got["ready_slots"]) > 0
        _same_outputs(hq, got, want, cids, committed, "regrow")
    finally:
        a.close()
        b.close()
        pin.close()


@pytest.mark.parametrize("where", ["pinned", "pageable", "host"])
def test_sizes16_rejects_bad_input(hq, where):
    """2-byte words: a group's bytes that do not decode (a truncated varint), byte totals that
    do not match, or an event total that is not the events decoded make the step HQ_E_INVAL with
    no group state written; the same step with the right input then runs."""
    import bench

    G = 3000
    roles = bench.STEP_ROLES["step"]
    g, m, cids = bench.step_groups(hq, G, 1, 1, roles)
    nv = sum(r != "observer" for r in roles)
    grp, off, ev = bench.step_events(hq, G, 0, roles)
    data, sz = hq.encode_events_sized(off, ev)
    s16 = hq.sizes16_of(sz)
    w = hq.Worker(0, nv, on_device=where != "host", commit_advance=where != "host")
    fresh = hq.Worker(0, nv, on_device=where != "host", commit_advance=where != "host")
    pin = hq.Context(0)
    try:
        w.add_groups(g, m)
        fresh.add_groups(g, m)
        before = [w.get_group(int(c))[0]["committed"] for c in cids[::101]]

        def run(s, d, ne):
            if where == "pinned":
                s, d = _pinned(pin, s), _pinned(pin, d)
            return w.step_sized(None, s, ne, d)

        bad = data.copy()
        b0 = int(s16[:7].astype(np.int64).sum())
        bad[b0 + int(s16[7]) - 1] |= 0x80            # group 7's last varint runs past its bytes
        with pytest.raises(hq.HQError):
            run(s16, bad, len(ev))
        moved = s16.copy()
        moved[3] += 1                                 # totals off by one byte
        with pytest.raises(hq.HQError):
            run(moved, data, len(ev))
        with pytest.raises(hq.HQError):
            run(s16, data, len(ev) + 1)               # an event total that was not decoded
        assert [w.get_group(int(c))[0]["committed"] for c in cids[::101]] == before
        # the rejected steps left nothing behind: the step then gives what a fresh worker's does
        _same_lists(run(s16, data, len(ev)), fresh.step_sized(None, s16, len(ev), data))
    finally:
        w.close()
        fresh.close()
        pin.close()


@pytest.mark.parametrize("mode", ["block", "sleep", "spin", "adapt"])
def test_wait_policies_same_results(hq, mode):
    """Every wait policy steps the same: outputs equal, the wait's clock filled in (a blocking
    wait is one sleep), the device's end stamp taken with HQ_WAIT_CLOCK."""
    import bench

    G = 20000
    roles = bench.STEP_ROLES["step"]
    g, m, cids = bench.step_groups(hq, G, 1, 1, roles)
    nv = sum(r != "observer" for r in roles)
    code = {"block": hq.HQ_WAIT_BLOCK, "sleep": hq.HQ_WAIT_SLEEP, "spin": hq.HQ_WAIT_SPIN,
            "adapt": hq.HQ_WAIT_ADAPT}[mode]
    a = hq.Worker(0, nv, on_device=True, commit_advance=True)
    b = hq.Worker(0, nv, on_device=True, commit_advance=True)
    pin = hq.Context(0)
    try:
        a.set_wait(code, poll_us=0 if mode == "sleep" else 50, sleep_us=10, clock=True)
        with pytest.raises(hq.HQError):
            a.set_wait(7)
        a.add_groups(g, m)
        b.add_groups(g, m)
        ticks = []
        for s in range(3):
            grp, off, ev = bench.step_events(hq, G, s, roles)
            data, sz = hq.encode_events_sized(off, ev)
            got = a.step_sized(None, _pinned(pin, sz), len(ev), _pinned(pin, data))
            want = b.step_sized(None, sz, len(ev), data)
            _same_lists(got, want)
            np.testing.assert_array_equal(got["ready"], want["ready"])
            assert got["device_end_ticks"] > 0 and got["wait_end_ns"] > 0 and got["gpu_ns"] > 0
            # the device's span of the step covers the GPU's time between its timing events
            assert 0 < got["device_start_ticks"] < got["device_end_ticks"]
            assert (got["device_end_ticks"] - got["device_start_ticks"]) * 10 >= got["gpu_ns"] * 0.9
            assert want["device_end_ticks"] == 0
            if mode == "spin":
                assert got["wait_sleeps"] == 0 and got["wait_sleep_ns"] == 0
            elif mode in ("block", "adapt"):
                assert got["wait_sleeps"] in (0, 1, 2)
            ticks.append(got["device_end_ticks"])
        assert ticks == sorted(ticks) and len(set(ticks)) == 3   # the device's clock advances
    finally:
        a.close()
        b.close()
        pin.close()


def test_scan_giveup_reruns_copy_out(hq, monkeypatch):
    """when pass A's chained scan of the ReadyToRead places gives up on a
    stalled predecessor (forced here: HQ_TEST_SCAN_FAIL at open makes every look-back give up),
    the step is not failed: the copy-out runs again through k_step_lite and the outputs equal a
    worker's whose look-backs succeed (the copy path with the speculated advance column)."""
    import bench

    G = 30000
    roles = bench.STEP_ROLES["step"]
    g, m, cids = bench.step_groups(hq, G, 1, 1, roles)
    nv = sum(r != "observer" for r in roles)
    monkeypatch.setenv("HQ_TEST_SCAN_FAIL", "1")
    a = hq.Worker(0, nv, on_device=True, commit_advance=True)
    monkeypatch.delenv("HQ_TEST_SCAN_FAIL")
    b = hq.Worker(0, nv, on_device=True, commit_advance=True)
    try:
        a.add_groups(g, m)
        b.add_groups(g, m)
        for s in range(2):
            grp, off, ev = bench.step_events(hq, G, s, roles)
            data, sz = hq.encode_events_sized(off, ev)       # pageable: the copy path
            got = a.step_sized(grp, sz, len(ev), data)
            want = b.step_sized(grp, sz, len(ev), data)
            np.testing.assert_array_equal(got["ready"], want["ready"])
            _same_lists(got, want)
            assert len(got["ready"]) == (G + 3) // 4
    finally:
        a.close()
        b.close()


def test_large_job_scans_tile_totals(hq):
    """A job of more than 2048 size tiles (> 2 M groups) scans its tiles' totals in a launch of
    their own (k_bsum_scan_jobs) instead of each tile summing those before it: its step (pinned,
    the jobs path) equals the copy path's (pageable: hipcub's scan), 2-byte words."""
    import bench

    G = 2048 * 1024 + 4099
    roles = bench.STEP_ROLES["step"]
    g, m, cids = bench.step_groups(hq, G, 1, 1, roles)
    nv = sum(r != "observer" for r in roles)
    grp, off, ev = bench.step_events(hq, G, 0, roles)
    data, sz = hq.encode_events_sized(off, ev)
    s16 = hq.sizes16_of(sz)
    a = hq.Worker(0, nv, on_device=True, commit_advance=True)
    b = hq.Worker(0, nv, on_device=True, commit_advance=True)
    pin = hq.Context(0)
    try:
        a.add_groups(g, m)
        b.add_groups(g, m)
        got = a.step_sized(None, _pinned(pin, s16), len(ev), _pinned(pin, data))
        want = b.step_sized(None, s16, len(ev), data)
        np.testing.assert_array_equal(got["ready"], want["ready"])
        _same_lists(got, want)
    finally:
        a.close()
        b.close()
        pin.close()
