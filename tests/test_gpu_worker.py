"""The GPU step worker (hq_worker_*, dragonboat_amd/csrc/hq_worker.cpp) against the sequential
step oracle (oracle/qref_step.c): the reference's raft-level tests restated as step scenarios,
then random multi-step differential runs over thousands of groups. Every quorum decision of the
worker is a kernel launch; results must be identical to the reference processing the same events
one at a time."""
import numpy as np
import pytest

import step_random as sr
import step_scenarios as sc
from step_harness import OracleBackend, WorkerBackend, same_step

pytestmark = pytest.mark.gpu
CASES = list(sc.all_cases())


MODES = [False, True]
MODE_IDS = ["host", "device"]      # the host worker / HQ_WORKER_ON_DEVICE (hq_dstep.hip)
# (on_device, stream): events as rows or as an event stream (hq_worker_step_stream)
FEEDS = [(False, False), (True, False), (True, True), (False, True), (True, "sized"),
         (False, "sized"), (True, "sized-column"), (True, "sized-advance"), (True, "sized16"),
         (False, "sized16"), (True, "sized16-slots")]
FEED_IDS = ["host", "device", "device-stream", "host-stream", "device-sized", "host-sized",
            "device-sized-column", "device-sized-advance", "device-sized16", "host-sized16",
            "device-sized16-slots"]


@pytest.fixture(scope="module", params=FEEDS, ids=FEED_IDS)
def worker_backend(hq, request):
    b = WorkerBackend(hq, n_max=8, seed=1, on_device=request.param[0], stream=request.param[1])
    yield b
    b.close()


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_reference_scenario_on_gpu(worker_backend, case):
    outs, state = sc.run_case(worker_backend, case)
    sc.check_case(case, outs, state)
    want_outs, want_state = sc.run_case(OracleBackend(), case)
    assert state == want_state, case["name"]
    for w, o in zip(outs, want_outs):
        for k in ("committed", "commit_changed", "ready", "resps", "states", "dropped",
                  "deferred"):
            assert w[k] == o[k], (case["name"], k, w[k], o[k])


@pytest.mark.parametrize("on_device", MODES, ids=MODE_IDS)
def test_one_gpu_pass_per_plain_step(hq, on_device):
    """Commit + ReadIndex acks + CheckQuorum of many groups: one GPU batch per step."""
    b = WorkerBackend(hq, n_max=5, on_device=on_device)
    try:
        for cid in range(1, 101):
            b.add_group(cid, 1, 3, sc.LEADER, 10, 12, 10,
                        [(i, 12 if i == 1 else 10, sc.REMOTE, 0) for i in range(1, 6)])
        out = b.step({cid: [sc.msg(sc.RREP, 2, 3, 12), sc.msg(sc.RREP, 3, 3, 11),
                            ("check_quorum",)] for cid in range(1, 101)})
        # host: one commit + one CheckQuorum decision per group in one pass; device: every
        # ReplicateResp's tryCommit and the CheckQuorum, in one launch pair
        assert b.last_passes == 1 and b.last_decisions == (300 if on_device else 200)
        assert all(out[cid]["committed"] == 11 for cid in range(1, 101))
        assert all(out[cid]["states"] == [] for cid in range(1, 101))
    finally:
        b.close()


@pytest.mark.parametrize("feed", FEEDS, ids=FEED_IDS)
@pytest.mark.parametrize("seed,G,steps", [(1, 3000, 6), (2, 1500, 10), (3, 400, 25)])
def test_random_differential(hq, seed, G, steps, feed):
    on_device, stream = feed
    rng = np.random.default_rng(seed)
    groups = sr.random_groups(rng, G)
    o, w = OracleBackend(), WorkerBackend(hq, n_max=8, seed=seed, on_device=on_device,
                                          stream=stream)
    try:
        for g in groups:
            o.add_group(*g)
            w.add_group(*g)
        ctx_seq = [0]
        seen = dict(ready=0, resps=0, states=0, dropped=0, deferred=0, commit=0)
        passes = []
        for s in range(steps):
            per = {}
            for g in groups:
                if rng.random() < 0.85:
                    per[g[0]] = sr.random_events(rng, o.state(g[0]), s + 1, ctx_seq)
            want = o.step(per)
            got = w.step(per)
            passes.append(w.last_passes)
            assert got["_fallback"] == []
            for cid in per:
                same_step(want, got, cid)
                seen["commit"] += want[cid]["commit_changed"]
                for k in ("ready", "resps", "states", "dropped", "deferred"):
                    seen[k] += len(want[cid][k])
            for g in groups:
                assert w.state(g[0]) == o.state(g[0]), (s, g[0])
        # the streams exercised every output kind, and runs cut by barriers (several passes)
        assert all(v > 0 for v in seen.values()), seen
        # host: runs cut by barriers take several passes; device: every step is one launch pair
        assert max(passes) == 1 if on_device else max(passes) >= 2, passes
    finally:
        w.close()


@pytest.mark.parametrize("on_device", MODES, ids=MODE_IDS)
def test_fallback_suspends_and_resync_resumes(hq, on_device):
    """An observer acknowledging a pending ctx cannot be taken by the slot model: the group is
    suspended from that event on (its tail deferred) and resumes after hq_worker_set_group."""
    w = hq.Worker(0, 8, on_device=on_device)
    try:
        mem = [(i, 9, sc.REMOTE, 0) for i in range(1, 6)] + [(6, 0, sc.OBSERVER, 0)]
        w.add_group(7, 1, 2, sc.LEADER, 9, 9, 9, mem)
        b = WorkerBackend(hq, worker=w)
        out = b.step({7: [("read", 5, 6), sc.msg(sc.HBRESP, 2, 2, hint=5, high=6),
                          sc.msg(sc.HBRESP, 6, 2, hint=5, high=6), sc.msg(sc.RREP, 2, 2, 9),
                          ("propose", 1)]})
        assert out["_fallback"] == [7]
        assert out[7]["deferred"] == [2, 3, 4]
        g, m, r = w.get_group(7)
        assert g["suspended"] == 1 and len(r) == 1 and r[0]["n_confirmed"] == 1
        out = b.step({7: [("propose", 1)]})
        assert out[7]["deferred"] == [0]       # still suspended
        w.set_group(7, 1, 2, sc.LEADER, 9, 10, 9, [(1, 10, 0, 0), (2, 10, 0, 0), (3, 9, 0, 0),
                                                   (4, 9, 0, 0), (5, 9, 0, 0), (6, 0, 1, 0)])
        out = b.step({7: [sc.msg(sc.RREP, 3, 2, 10)]})
        assert out["_fallback"] == [] and out[7]["committed"] == 10
    finally:
        w.close()


@pytest.mark.parametrize("on_device", MODES, ids=MODE_IDS)
def test_ack_above_last_index_is_fallback(hq, on_device):
    w = hq.Worker(0, 4, on_device=on_device)
    try:
        w.add_group(1, 1, 2, sc.LEADER, 5, 6, 5, [(1, 6, 0, 0), (2, 5, 0, 0), (3, 5, 0, 0)])
        b = WorkerBackend(hq, worker=w)
        out = b.step({1: [sc.msg(sc.RREP, 2, 2, 6), sc.msg(sc.RREP, 3, 2, 7)]})
        assert out["_fallback"] == [1] and out[1]["deferred"] == [1]
        assert out[1]["committed"] == 6        # decided up to the offending message
    finally:
        w.close()


@pytest.mark.parametrize("on_device", MODES, ids=MODE_IDS)
def test_add_group_validation(hq, on_device):
    w = hq.Worker(0, 3, on_device=on_device)
    try:
        with pytest.raises(hq.HQError, match="n_max"):
            w.add_group(1, 1, 1, 0, 0, 0, 0, [(i, 0, 0, 0) for i in range(1, 5)])
        with pytest.raises(hq.HQError, match="remotes"):
            w.add_group(2, 9, 1, 0, 0, 0, 0, [(1, 0, 0, 0)])
        w.add_group(3, 1, 1, 0, 0, 0, 0, [(1, 0, 0, 0)])
        with pytest.raises(hq.HQError, match="exists"):
            w.add_group(3, 1, 1, 0, 0, 0, 0, [(1, 0, 0, 0)])
    finally:
        w.close()


# ---- the same worker driven from wire bytes (raftpb.MessageBatch, hq_wire) --------------------
@pytest.fixture(scope="module", params=FEEDS, ids=FEED_IDS)
def wire_backend(hq, request):
    from step_harness import WireBackend

    b = WireBackend(hq, n_max=8, seed=5, on_device=request.param[0], stream=request.param[1])
    yield b
    b.close()


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_reference_scenario_from_wire_bytes(wire_backend, case):
    outs, state = sc.run_case(wire_backend, case)
    sc.check_case(case, outs, state)
    want_outs, want_state = sc.run_case(OracleBackend(), case)
    assert state == want_state, case["name"]
    for w, o in zip(outs, want_outs):
        for k in ("committed", "commit_changed", "ready", "resps", "states", "dropped",
                  "deferred"):
            assert w[k] == o[k], (case["name"], k, w[k], o[k])


@pytest.mark.parametrize("feed", FEEDS, ids=FEED_IDS)
@pytest.mark.parametrize("seed,G,steps", [(11, 1500, 6), (12, 300, 15)])
def test_random_differential_from_wire_bytes(hq, seed, G, steps, feed):
    from step_harness import WireBackend

    rng = np.random.default_rng(seed)
    groups = sr.random_groups(rng, G)
    o, w = OracleBackend(), WireBackend(hq, n_max=8, seed=seed, on_device=feed[0],
                                        stream=feed[1])
    try:
        for g in groups:
            o.add_group(*g)
            w.add_group(*g)
        ctx_seq = [0]
        dropped = 0
        for s in range(steps):
            per = {}
            for g in groups:
                if rng.random() < 0.85:
                    per[g[0]] = sr.random_events(rng, o.state(g[0]), s + 1, ctx_seq)
            want = o.step(per)
            got = w.step(per)
            st = w.last_stats
            assert st.dropped_batches == 1 and st.batches >= 2
            dropped += st.dropped_no_cluster + st.snapshot_received
            assert got["_fallback"] == []
            for cid in per:
                same_step(want, got, cid)
            for g in groups:
                assert w.state(g[0]) == o.state(g[0]), (s, g[0])
        assert dropped > 0
    finally:
        w.close()


def test_device_worker_member_cap(hq):
    """The device path holds at most 16 members per group (8 voting + observers)."""
    w = hq.Worker(0, 8, on_device=True)
    try:
        mem = [(i, 0, sc.REMOTE, 0) for i in range(1, 4)] + \
              [(i, 0, sc.OBSERVER, 0) for i in range(4, 18)]
        with pytest.raises(hq.HQError, match="16 members"):
            w.add_group(1, 1, 1, 0, 0, 0, 0, mem)
        w.add_group(2, 1, 1, 0, 0, 0, 0, mem[:16])
    finally:
        w.close()


@pytest.mark.parametrize("on_device", MODES, ids=MODE_IDS)
def test_malformed_stream(hq, on_device):
    """A device worker falls the group back at the event that does not decode (the events
    before it taken); a host worker rejects the step."""
    w = hq.Worker(0, 4, on_device=on_device)
    try:
        w.add_group(1, 1, 2, sc.LEADER, 5, 6, 5, [(1, 6, 0, 0), (2, 5, 0, 0), (3, 5, 0, 0)])
        w.add_group(2, 1, 2, sc.LEADER, 5, 6, 5, [(1, 6, 0, 0), (2, 5, 0, 0), (3, 5, 0, 0)])
        ev = np.array([(hq.EV_MESSAGE, sc.RREP, 2, 2, 6, 0, 0, 0, 0),
                       (hq.EV_MESSAGE, sc.RREP, 3, 2, 6, 0, 0, 0, 0),
                       (hq.EV_MESSAGE, sc.RREP, 2, 2, 6, 0, 0, 0, 0)], hq.EVENT_DTYPE)
        off = np.array([0, 2, 3], np.uint64)
        data, boff = hq.encode_events(off, ev)
        # group 0's second event cut short: its last varint loses its final byte
        cut = np.concatenate([data[:int(boff[1]) - 1], data[int(boff[1]):]])
        boff2 = boff.copy()
        boff2[1:] -= 1
        grp = np.array([w.find(1), w.find(2)], np.uint32)
        if not on_device:
            with pytest.raises(hq.HQError, match="malformed"):
                w.step_stream(grp, off, boff2, cut)
            return
        res = w.step_stream(grp, off, boff2, cut)
        assert list(res["fallback_groups"]) == [1] and list(res["deferred"]) == [1]
        assert w.get_group(2)[0]["committed"] == 6       # the other group is unaffected
        g1 = w.get_group(1)[0]                            # its first ack was taken
        assert g1["committed"] == 6 and g1["suspended"] == 1
    finally:
        w.close()


@pytest.mark.parametrize("feed", FEEDS[:4], ids=FEED_IDS[:4])
def test_step_input_errors_leave_state(hq, feed):
    """Bad step inputs are rejected whole (HQ_E_INVAL) with no group state changed: an unknown
    handle, a group listed twice, decreasing offsets."""
    on_device, stream = feed
    w = hq.Worker(0, 4, on_device=on_device)
    try:
        for cid in (1, 2):
            w.add_group(cid, 1, 2, sc.LEADER, 5, 6, 5, [(1, 6, 0, 0), (2, 5, 0, 0), (3, 5, 0, 0)])
        ev = np.array([(hq.EV_MESSAGE, sc.RREP, 2, 2, 6, 0, 0, 0, 0)] * 2, hq.EVENT_DTYPE)

        def step(grp, off):
            grp, off = np.array(grp, np.uint32), np.array(off, np.uint64)
            if stream:                   # each group's one event: 4 bytes
                data, boff = hq.encode_events(np.array([0, 1, 2], np.uint64), ev)
                return w.step_stream(grp, off, boff, data)
            return w.step(grp, off, ev)

        for grp, off, msg in (([0, 7], [0, 1, 2], "unknown group handle"),
                              ([1, 1], [0, 1, 2], "listed twice"),
                              ([0, 1], [0, 2, 1], "offsets decrease")):
            with pytest.raises(hq.HQError, match=msg):
                step(grp, off)
            assert w.get_group(1)[0]["committed"] == 5 and w.get_group(2)[0]["committed"] == 5
        res = step([1, 0], [0, 1, 2])                        # and the worker still steps
        assert sorted(int(c["cluster_id"]) for c in res["commits"]) == [1, 2]
    finally:
        w.close()


@pytest.mark.parametrize("on_device", MODES, ids=MODE_IDS)
def test_sized_input_errors_leave_state(hq, on_device):
    """The sized stream form: sizes that do not sum to the totals, an unknown handle or a group
    listed twice reject the step whole, no group state changed."""
    w = hq.Worker(0, 4, on_device=on_device)
    try:
        for cid in (1, 2):
            w.add_group(cid, 1, 2, sc.LEADER, 5, 6, 5, [(1, 6, 0, 0), (2, 5, 0, 0), (3, 5, 0, 0)])
        ev = np.array([(hq.EV_MESSAGE, sc.RREP, 2, 2, 6, 0, 0, 0, 0)] * 2, hq.EVENT_DTYPE)
        data, sizes = hq.encode_events_sized(np.array([0, 1, 2], np.uint64), ev)
        assert list(sizes) == [1 | 4 << 16, 1 | 4 << 16] and len(data) == 8
        for grp, z, ne, d, msg in (
                ([0, 7], sizes, 2, data, "unknown group handle"),
                ([1, 1], sizes, 2, data, "listed twice"),
                ([0, 1], sizes, 3, data, "sizes"),                        # events total
                ([0, 1], sizes, 2, np.concatenate([data, data[:1]]), "sizes"),   # bytes total
                ([0, 1], [1 | 4 << 16, 1 | 5 << 16], 2, data, "sizes"),
                # totals right, split wrong: group 0 keeps a byte of group 1's event (the host
                # decoder's p != end; the device engine's left-over-bytes check, pass A)
                ([0, 1], [1 | 5 << 16, 1 | 3 << 16], 2, data, "malformed")):
            with pytest.raises(hq.HQError, match=msg):
                w.step_sized(np.array(grp, np.uint32), np.array(z, np.uint32), ne, d)
            assert w.get_group(1)[0]["committed"] == 5 and w.get_group(2)[0]["committed"] == 5
        res = w.step_sized(np.array([1, 0], np.uint32), sizes, 2, data)
        assert sorted(int(c["cluster_id"]) for c in res["commits"]) == [1, 2]
    finally:
        w.close()


@pytest.mark.parametrize("on_device", MODES, ids=MODE_IDS)
def test_sized_stream_implicit_handles(hq, on_device):
    """The sized form with groups NULL lists handles 0 .. n - 1: the same results and state as
    the explicit list (step workload, 3 steps, every group committing from step 1 on)."""
    import bench

    G = 5000
    roles = bench.STEP_ROLES["step5"]
    g, m, _ = bench.step_groups(hq, G, 1, 1, roles)
    nv = sum(r != "observer" for r in roles)
    a, b = hq.Worker(0, nv, on_device=on_device), hq.Worker(0, nv, on_device=on_device)
    try:
        a.add_groups(g, m)
        b.add_groups(g, m)
        for s in range(3):
            grp, off, ev = bench.step_events(hq, G, s, roles)
            data, sizes = hq.encode_events_sized(off, ev)
            got = a.step_sized(None, sizes, len(ev), data)
            want = b.step_sized(grp, sizes, len(ev), data)
            for k in ("commits", "ready", "read_resps", "state_changes", "dropped_reads",
                      "deferred", "fallback_groups"):
                np.testing.assert_array_equal(got[k], want[k], err_msg=f"step {s} {k}")
            assert len(got["commits"]) == (G if s else 0)
        assert a.get_group(G)[0]["committed"] == b.get_group(G)[0]["committed"]
        with pytest.raises(hq.HQError):                  # more sizes than groups on the worker
            a.step_sized(None, np.zeros(G + 1, np.uint32), 0, np.zeros(0, np.uint8))
    finally:
        a.close()
        b.close()


def test_wide_advance_survives_output_regrow(hq):
    """HQ_WORKER_COMMIT_ADVANCE with a committed index that moves by 2^33 in a step whose lists
    overflow the pinned output region: the region is grown and the layout run again, and the
    re-run must keep pass A's "wide" flag (the 4-byte advance column would truncate 2^33 to 0).
    Worker a's region is sized by a first step listing one group; b's by a first step listing
    all of them (no overflow). Both must return the same 8-byte commit column."""
    import bench

    G, big, special = 8192, 1 << 33, 5
    roles = bench.STEP_ROLES["step"]
    g, m, cids = bench.step_groups(hq, G, 1, 1, roles)
    g["committed"] -= np.uint64(10)                  # the step's acks of lastIndex commit
    g["term_start"] = g["committed"]
    m["match"][m["node_id"] != 1] -= np.uint64(10)
    g["last_index"][special] = big                   # this group commits 2^33 - 990 at once
    m["match"][len(roles) * special] = big           # the leader's own match = lastIndex
    grp, off, ev = bench.step_events(hq, G, 0, roles)
    rows = ev[int(off[special]):int(off[special + 1])]
    rows["log_index"][(rows["kind"] == hq.EV_MESSAGE) & (rows["type"] == 13)] = big
    ev[int(off[special]):int(off[special + 1])] = rows
    data, sizes = hq.encode_events_sized(off, ev)
    nv = sum(r != "observer" for r in roles)
    a = hq.Worker(0, nv, on_device=True, commit_column=True, commit_advance=True)
    b = hq.Worker(0, nv, on_device=True, commit_column=True, commit_advance=True)
    try:
        a.add_groups(g, m)
        b.add_groups(g, m)
        empty = np.zeros(0, np.uint8)
        a.step_sized(np.array([0], np.uint32), np.zeros(1, np.uint32), 0, empty)
        b.step_sized(grp, np.zeros(G, np.uint32), 0, empty)
        got = a.step_sized(grp, sizes, len(ev), data)
        want = b.step_sized(grp, sizes, len(ev), data)
        assert len(got["ready"]) == G // 4 and 32 * (G // 4) + 8 * G > 1 << 16   # a overflows
        assert "committed_advance" not in got and "committed_advance" not in want
        np.testing.assert_array_equal(got["committed_column"], want["committed_column"])
        assert int(got["committed_column"][special]) == big
        assert a.get_group(int(cids[special]))[0]["committed"] == big
    finally:
        a.close()
        b.close()


def test_step_jobs_equal_sequential_steps(hq):
    """hq_worker_step_jobs: several workers (device and host, rows and streams) stepped at once
    on native threads end in the same results and state as stepping them one by one."""
    import bench

    G = 3000
    roles = bench.STEP_ROLES["step5"]
    g, m, _ = bench.step_groups(hq, G, 1, 1, roles)
    nm, nv = len(roles), sum(r != "observer" for r in roles)
    kinds = [(True, True), (True, False), (False, False), (True, True), (True, "sized")]
    bounds = [G * i // len(kinds) for i in range(len(kinds) + 1)]

    def make():
        ws = []
        for i, (dev, _) in enumerate(kinds):
            w = hq.Worker(0, nv, on_device=dev)
            w.add_groups(g[bounds[i]:bounds[i + 1]], m[nm * bounds[i]:nm * bounds[i + 1]])
            ws.append(w)
        return ws

    a, b = make(), make()
    try:
        for s in range(3):
            jobs = []
            for i, (_, stream) in enumerate(kinds):
                e = bench.step_events(hq, bounds[i + 1] - bounds[i], s, roles)
                if stream == "sized":
                    data, sizes = hq.encode_events_sized(e[1], e[2])
                    e = hq.SizedStream(e[0], sizes, len(e[2]), data)
                elif stream:
                    data, boff = hq.encode_events(e[1], e[2])
                    e = (e[0], e[1], boff, data)
                jobs.append(e)
            got = hq.step_jobs(list(zip(a, jobs)))
            for i, (w, e) in enumerate(zip(b, jobs)):
                want = w.step_sized(*e) if isinstance(e, hq.SizedStream) else \
                    w.step(*e) if len(e) == 3 else w.step_stream(*e)
                for k in ("commits", "ready", "read_resps", "state_changes", "dropped_reads",
                          "deferred", "fallback_groups"):
                    np.testing.assert_array_equal(got[i][k], want[k], err_msg=k)
                assert len(want["commits"]) == (bounds[i + 1] - bounds[i] if s else 0)
        with pytest.raises(hq.HQError):
            hq.step_jobs([(a[0], jobs[0]), (a[0], jobs[0])])      # a worker twice
    finally:
        for w in a + b:
            w.close()


@pytest.mark.parametrize("wide", [False, True], ids=["8-member-slots", "16-member-slots"])
def test_fused_step_jobs_equal_single_steps(hq, wide):
    """hq_worker_step_jobs over device workers that all take sized streams on one GPU steps them
    through shared launches (hq_dstep_run_jobs: one pass A per input chunk, one layout, one
    k_step_lite, one pass B). Every job's lists and its workers' state equal the same worker
    stepped alone (its own launch sequence): ragged sizes (1, 63, 64, 4097 groups ...), implicit
    handles, the list / column / advance forms of the commits, a job whose output region
    overflows and is regrown, and a job with an input error (failed alone, state untouched)."""
    import bench

    sizes_g = [3000, 1, 64, 4097, 20000, 63, 700]
    wide_roles = ("remote",) * 3 + ("observer",) * 7          # 10 members: 16 slots
    specs = []
    for i, G in enumerate(sizes_g):
        roles = wide_roles if wide and i == 3 else bench.STEP_ROLES["step5" if i % 2 else "step"]
        specs.append((G, roles, dict(commit_column=i % 3 == 1, commit_advance=i % 3 == 2),
                      i in (1, 4)))                            # implicit handles
    def make():
        ws = []
        for G, roles, flags, _ in specs:
            g, m, _ = bench.step_groups(hq, G, 1, 1, roles)
            w = hq.Worker(0, sum(r != "observer" for r in roles), on_device=True, **flags)
            w.add_groups(g, m)
            ws.append(w)
        return ws

    def compare(got, want, what):
        assert set(k for k in want if isinstance(want[k], np.ndarray)) == \
            set(k for k in got if isinstance(got[k], np.ndarray)), what
        for k, v in want.items():
            if isinstance(v, np.ndarray):
                np.testing.assert_array_equal(got[k], v, err_msg=f"{what} {k}")
        assert got.get("n_commits") == want.get("n_commits"), what

    a, b = make(), make()
    empty = np.zeros(0, np.uint8)
    pin = hq.Context(0)       # sizes in pinned memory are read over the link (k_size_sums)
    try:
        # step 0 lists one group with no events: every output region starts at its 64 KB minimum
        jobs = [hq.SizedStream(np.zeros(1, np.uint32), np.zeros(1, np.uint32), 0, empty)
                for _ in specs]
        for i, (res, w) in enumerate(zip(hq.step_jobs(list(zip(a, jobs))), b)):
            compare(res, w.step_sized(*jobs[i]), f"step 0 job {i}")
        for s in range(3):
            jobs = []
            for G, roles, _, implicit in specs:
                grp, off, ev = bench.step_events(hq, G, s, roles)
                data, sz = hq.encode_events_sized(off, ev)
                if s != 1:                                  # pinned sizes (s 1: pageable)
                    p = pin.pinned(len(sz), np.uint32)
                    p[:] = sz
                    sz = p
                if s == 2:                                  # pinned bytes: read in place
                    p = pin.pinned(len(data), np.uint8)
                    p[:] = data
                    data = p
                jobs.append(hq.SizedStream(None if implicit else grp, sz, len(ev), data))
            got = hq.step_jobs(list(zip(a, jobs)))          # (the 20000-group job overflows at s 0)
            for i, (res, w) in enumerate(zip(got, b)):
                compare(res, w.step_sized(*jobs[i]), f"step {s + 1} job {i}")
        # a job listing a group twice fails alone; the others step
        G, roles, _, _ = specs[2]
        grp, off, ev = bench.step_events(hq, G, 3, roles)
        data, sz = hq.encode_events_sized(off, ev)
        bad = grp.copy()
        bad[1] = bad[0]
        jobs[2] = hq.SizedStream(bad, sz, len(ev), data)
        with pytest.raises(hq.HQError, match="listed twice"):
            hq.step_jobs(list(zip(a, jobs)))
        for i, w in enumerate(b):
            if i != 2:
                w.step_sized(*jobs[i])
        for i, (G, _, _, _) in enumerate(specs):
            for c in sorted({1, G // 2 + 1, G}):
                ga, ma = a[i].get_group(c)[:2]
                gb, mb = b[i].get_group(c)[:2]
                assert ga.tobytes() == gb.tobytes() and ma.tobytes() == mb.tobytes(), (i, c)
    finally:
        for w in a + b:
            w.close()
        pin.close()


@pytest.mark.parametrize("flags", [{}, {"commit_column": True}, {"commit_advance": True}],
                         ids=["list", "column", "advance"])
def test_pinned_sized_stream_equals_pageable(hq, flags):
    """A sized stream in pinned host memory (copied in chunks by the copy engine, or read in
    place by the jobs path) decides as the same steps fed from pageable memory — at a size the
    copy path chunks, with ragged groups from step_events."""
    import bench

    G = 4 * 65536 + 5
    roles = bench.STEP_ROLES["step5"]
    g, m, cids = bench.step_groups(hq, G, 1, 1, roles)
    nv = sum(r != "observer" for r in roles)
    a = hq.Worker(0, nv, on_device=True, **flags)
    b = hq.Worker(0, nv, on_device=True, **flags)
    pin = hq.Context(0)
    try:
        a.add_groups(g, m)
        b.add_groups(g, m)
        for s in range(3):
            grp, off, ev = bench.step_events(hq, G, s, roles)
            data, sz = hq.encode_events_sized(off, ev)
            pd, ps = pin.pinned(len(data), np.uint8), pin.pinned(len(sz), np.uint32)
            pd[:], ps[:] = data, sz
            got = a.step_sized(None, ps, len(ev), pd)
            want = b.step_sized(None, sz, len(ev), data)
            for k, v in want.items():
                if isinstance(v, np.ndarray):
                    np.testing.assert_array_equal(got[k], v, err_msg=f"step {s} {k}")
            assert got.get("n_commits") == want.get("n_commits")
        for c in (1, G // 2, G):
            ga, ma = a.get_group(int(cids[c - 1]))[:2]
            gb, mb = b.get_group(int(cids[c - 1]))[:2]
            assert ga.tobytes() == gb.tobytes() and ma.tobytes() == mb.tobytes()
    finally:
        a.close()
        b.close()
        pin.close()


@pytest.mark.parametrize("stream", [True, False, "sized", "sized-column", "sized-advance",
                                    "stream-advance"],
                         ids=["stream", "rows", "sized", "sized-column", "sized-advance",
                              "stream-advance"])
def test_chunked_device_step_equals_host_worker(hq, stream):
    """A step of >= 256 Ki groups runs in 4 chunks whose copies overlap the neighbouring chunks'
    passes (hq_dstep.hip); its lists equal the host worker's on the same events (the host
    worker is checked against the oracle above), in the same order. With the advance column a
    stream's pass A also writes the single ReadyToReads at their places (ready_tail's chained
    scan across the chunks' launches: byte chunks for a sized stream, group chunks for one with
    offsets)."""
    import bench

    G = 4 * 65536 + 5
    roles = bench.STEP_ROLES["step5"]
    g, m, _ = bench.step_groups(hq, G, 1, 1, roles)
    nv = sum(r != "observer" for r in roles)
    dev = hq.Worker(0, nv, on_device=True, commit_column=stream == "sized-column",
                    commit_advance=str(stream).endswith("advance"))
    host = hq.Worker(0, nv)
    try:
        dev.add_groups(g, m)
        host.add_groups(g, m)
        for s in range(3):
            e = bench.step_events(hq, G, s, roles)
            prev_col = np.array([host.get_group(c)[0]["committed"] for c in range(1, G + 1)],
                                np.uint64) if str(stream).endswith("advance") and s else None
            want = host.step(*e)
            if str(stream).startswith("sized"):   # byte chunks, each group's pass A in the
                data, sizes = hq.encode_events_sized(e[1], e[2])   # chunk its bytes end in
                got = dev.step_sized(e[0], sizes, len(e[2]), data)
                if "committed_column" in got:     # every group commits from step 1 on
                    assert s and stream == "sized-column" and got["n_commits"] == G
                    want_col = np.zeros(G, np.uint64)
                    want_col[want["commits"]["cluster_id"].astype(np.int64) - 1] = \
                        want["commits"]["committed"]
                    np.testing.assert_array_equal(got["committed_column"], want_col)
                    got["commits"] = want["commits"]
                elif "committed_advance" in got:  # the advance over the previous step's
                    assert s and stream == "sized-advance" and got["n_commits"] == G
                    want_col = np.zeros(G, np.uint64)
                    want_col[want["commits"]["cluster_id"].astype(np.int64) - 1] = \
                        want["commits"]["committed"]
                    np.testing.assert_array_equal(prev_col + got["committed_advance"], want_col)
                    got["commits"] = want["commits"]
                else:
                    assert not s or stream == "sized"
            elif stream:
                data, boff = hq.encode_events(e[1], e[2])
                got = dev.step_stream(e[0], e[1], boff, data)
                if "committed_advance" in got:
                    assert s and stream == "stream-advance" and got["n_commits"] == G
                    want_col = np.zeros(G, np.uint64)
                    want_col[want["commits"]["cluster_id"].astype(np.int64) - 1] = \
                        want["commits"]["committed"]
                    np.testing.assert_array_equal(prev_col + got["committed_advance"], want_col)
                    got["commits"] = want["commits"]
            else:
                got = dev.step(*e)
            for k in ("commits", "ready", "read_resps", "state_changes", "dropped_reads",
                      "deferred", "fallback_groups"):
                np.testing.assert_array_equal(got[k], want[k], err_msg=f"step {s} {k}")
            assert len(want["commits"]) == (G if s else 0) and len(want["ready"]) > G // 5
        for cid in (1, 65537, 131073, 4 * 65536 + 5):
            assert dev.get_group(cid)[0]["committed"] == host.get_group(cid)[0]["committed"]
    finally:
        dev.close()
        host.close()


def test_chunked_step_outgrows_the_pinned_region(hq):
    """The pinned region a device worker writes its lists into is sized by its first step: after
    a 20 000-group step, a chunked step with the advance column (pass A's speculative advance
    words in the region, the single ReadyToReads copied out by k_step_lite) needs 3 MB, the layout
    overflows, and the step's lists are written again into a larger region; the next steps fit.
    Every step's lists equal the host worker's."""
    import bench

    G = 4 * 65536 + 5
    roles = bench.STEP_ROLES["step5"]
    g, m, _ = bench.step_groups(hq, G, 1, 1, roles)
    nv = sum(r != "observer" for r in roles)
    dev = hq.Worker(0, nv, on_device=True, commit_advance=True)
    host = hq.Worker(0, nv)
    try:
        dev.add_groups(g, m)
        host.add_groups(g, m)
        # (the full steps restart at step 0: a group's first step must be step 0's events)
        for n, s in ((20000, 0), (G, 0), (G, 1), (G, 2)):
            e = bench.step_events(hq, n, s, roles)
            prev = np.array([host.get_group(c)[0]["committed"] for c in range(1, n + 1)], np.uint64)
            want = host.step(*e)
            data, sizes = hq.encode_events_sized(e[1], e[2])
            got = dev.step_sized(e[0], sizes, len(e[2]), data)
            if "committed_advance" in got:
                col = prev.copy()
                col[want["commits"]["cluster_id"].astype(np.int64) - 1] = want["commits"]["committed"]
                np.testing.assert_array_equal(prev + got["committed_advance"], col)
                got["commits"] = want["commits"]
            for k in ("commits", "ready", "read_resps", "state_changes", "dropped_reads",
                      "deferred", "fallback_groups"):
                np.testing.assert_array_equal(got[k], want[k], err_msg=f"step {s} {k}")
            assert len(want["ready"]) > n // 5    # (2 MB of records after the column's 1 MB)
        for cid in (1, 20001, 131073, G):
            assert dev.get_group(cid)[0]["committed"] == host.get_group(cid)[0]["committed"]
    finally:
        dev.close()
        host.close()


@pytest.mark.parametrize("feed", ["sized", "sized-advance"])
@pytest.mark.parametrize("seed", [11, 12])
def test_rejected_steps_restore_state_on_device(hq, seed, feed):
    """The device engine writes each group's new state in pass A and puts the saved state back
    when the step turns out to have an input error (k_step_restore): before every good step of a
    random multi-step run, the same step is offered with a group listed twice or with one byte
    moved between two groups' sizes (the left-over-bytes check) and must be rejected whole —
    every group's full state (members' match and active flags, pending reads, votes) equal to
    the oracle's, which never saw the bad step — and the good step then matches the oracle."""
    rng = np.random.default_rng(seed)
    G, steps = 600, 8
    groups = sr.random_groups(rng, G)
    o = OracleBackend()
    w = WorkerBackend(hq, n_max=8, seed=seed, on_device=True, stream=feed)
    try:
        for g in groups:
            o.add_group(*g)
            w.add_group(*g)
        ctx_seq = [0]
        rejected = 0
        for s in range(steps):
            per = {g[0]: sr.random_events(rng, o.state(g[0]), s + 1, ctx_seq)
                   for g in groups if rng.random() < 0.9}
            (grp, sizes, ne, data), _ = w.build_inputs(per)
            bad = [(np.concatenate([grp[:1], grp[:1], grp[2:]]), sizes, "listed twice")]
            nb = sizes >> 16                   # per-group bytes
            k = int(np.nonzero(nb[1:] > 0)[0][0])
            moved = sizes.copy()
            moved[k] += np.uint32(1 << 16)     # group k keeps the first byte of group k + 1:
            moved[k + 1] -= np.uint32(1 << 16)  # its events leave that byte over
            bad.append((grp, moved, "malformed"))
            for bg, bz, msg in bad:
                with pytest.raises(hq.HQError, match=msg):
                    w.w.step_sized(bg, bz, ne, data)
                rejected += 1
                for g in groups:
                    assert w.state(g[0]) == o.state(g[0]), (s, msg, g[0])
            want = o.step(per)
            got = w.step(per)
            assert got["_fallback"] == []
            for cid in per:
                same_step(want, got, cid)
            for g in groups:
                assert w.state(g[0]) == o.state(g[0]), (s, g[0])
        assert rejected == 2 * steps
    finally:
        w.close()


def test_failed_regrow_leaves_state(hq, monkeypatch):
    """a device step whose output region cannot be grown fails with every
    group's state as it was before the step (pass A's in-place state taken back by
    k_step_restore). The allocation failure is injected (HQ_TEST_FAIL_REGROW at open); the same
    step on a worker whose region grows does change the state compared."""
    import bench

    G = 16384                      # step 0's G/4 ReadyToReads (128 KB) overflow the 64 KB region
    roles = bench.STEP_ROLES["step"]
    g, m, cids = bench.step_groups(hq, G, 1, 1, roles)
    grp, off, ev = bench.step_events(hq, G, 0, roles)
    data, sizes = hq.encode_events_sized(off, ev)
    nv = sum(r != "observer" for r in roles)
    empty = np.zeros(0, np.uint8)
    b = hq.Worker(0, nv, on_device=True)
    monkeypatch.setenv("HQ_TEST_FAIL_REGROW", "1")
    a = hq.Worker(0, nv, on_device=True)
    monkeypatch.delenv("HQ_TEST_FAIL_REGROW")
    sample = [int(c) for c in cids[::97]]

    def state(w):
        return [w.get_group(c) for c in sample]

    def same(x, y):
        return all(np.array_equal(u, v) for p, q in zip(x, y) for u, v in zip(p, q))
    try:
        for w in (a, b):
            w.add_groups(g, m)
            # a first step listing one group sizes the output region for one group's lists
            w.step_sized(np.array([0], np.uint32), np.zeros(1, np.uint32), 0, empty)
        before = state(a)
        assert same(before, state(b))
        with pytest.raises(hq.HQError, match="injected"):
            a.step_sized(grp, sizes, len(ev), data)
        assert same(before, state(a))
        res = b.step_sized(grp, sizes, len(ev), data)
        assert len(res["ready"]) == G // 4
        assert not same(before, state(b))
    finally:
        a.close()
        b.close()


def _expand(hq, got, cids, committed_before):
    """A compact step's ReadyToReads as full records (hq.expand_ready over the listed groups)."""
    if "ready_compact" not in got:
        return got["ready"]
    assert len(got["ready"]) == 0
    return hq.expand_ready(got["ready_compact"], cids, committed_before)


@pytest.mark.parametrize("G,pinned", [(5000, False), (4 * 65536 + 5, False),
                                      (4 * 65536 + 5, True)],
                         ids=["small", "chunked-copy", "pinned-job"])
def test_ready_compact_equals_records(hq, G, pinned):
    """HQ_WORKER_READY_COMPACT: the 24-byte ReadyToReads (the group's position, index - its
    committed index before the step, the ctx) rebuild exactly the 32-byte records of a worker
    without the flag, step after step (the single-ReadyToRead groups copied out by k_step_lite,
    pass B's replayed groups, the copy path and the pinned one-job path); every other list and
    the commits are unchanged."""
    import bench

    roles = bench.STEP_ROLES["step5"]
    g, m, cids = bench.step_groups(hq, G, 1, 1, roles)
    nv = sum(r != "observer" for r in roles)
    a = hq.Worker(0, nv, on_device=True, commit_advance=True, ready_compact=True)
    b = hq.Worker(0, nv, on_device=True, commit_advance=True)
    pin = hq.Context(0) if pinned else None
    committed = g["committed"].astype(np.uint64).copy()
    try:
        a.add_groups(g, m)
        b.add_groups(g, m)
        for s in range(3):
            grp, off, ev = bench.step_events(hq, G, s, roles)
            if s == 2:
                # group 8 gets a follower's ReadIndex ahead of its local read: the heartbeat
                # acks release both, so the group has a ReadIndexResp besides its ReadyToRead
                # and pass B replays it (its compact record written by pass B itself)
                lo = int(off[8])
                assert ev["kind"][lo] == hq.EV_READ and ev["type"][lo + 1] == 13
                fwd = ev[lo + 1].copy()
                fwd["type"], fwd["hint"], fwd["hint_high"], fwd["log_index"] = 19, 99, 0, 0
                ev[lo + 1] = ev[lo]
                ev[lo] = fwd
            data, sz = hq.encode_events_sized(off, ev)
            if pinned:
                pd, ps = pin.pinned(len(data), np.uint8), pin.pinned(len(sz), np.uint32)
                pd[:], ps[:] = data, sz
                data, sz = pd, ps
            got = a.step_sized(None, sz, len(ev), data)
            want = b.step_sized(None, sz, len(ev), data)
            assert "ready_compact" in got and len(want["ready"]) > G // 5
            if s == 2:
                assert len(want["read_resps"]) == 1
            np.testing.assert_array_equal(_expand(hq, got, cids, committed), want["ready"],
                                          err_msg=f"step {s}")
            for k in ("read_resps", "state_changes", "dropped_reads", "deferred", "fallback_groups"):
                np.testing.assert_array_equal(got[k], want[k], err_msg=f"step {s} {k}")
            for k in ("committed_advance", "commits"):
                if k in want:
                    np.testing.assert_array_equal(got[k], want[k], err_msg=f"step {s} {k}")
            if "committed_advance" in want:
                committed += want["committed_advance"].astype(np.uint64)
            else:
                ix = want["commits"]["cluster_id"].astype(np.int64) - 1
                committed[ix] = want["commits"]["committed"]
    finally:
        a.close()
        b.close()
        if pin:
            pin.close()


def test_ready_compact_wide_delta_keeps_records(hq):
    """A ReadyToRead whose index lies 2^33 above its group's committed index before the step (the
    group commits 2^33 entries in the step and then receives a ReadIndex): the delta does not fit
    the compact record, so the step returns the 32-byte records — equal to a worker's without the
    flag — and the next steps are compact again."""
    import bench

    G, big, special = 8192, 1 << 33, 4               # group 4 serves a read (every 4th)
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
    assert rows["kind"][0] == hq.EV_READ
    rows["log_index"][(rows["kind"] == hq.EV_MESSAGE) & (rows["type"] == 13)] = big
    k = len(roles) - 1                                # the ReplicateResps, then the READ
    ev[lo:hi] = np.concatenate([rows[1:1 + k], rows[:1], rows[1 + k:]])
    data, sizes = hq.encode_events_sized(off, ev)
    nv = sum(r != "observer" for r in roles)
    a = hq.Worker(0, nv, on_device=True, commit_column=True, commit_advance=True, ready_compact=True)
    b = hq.Worker(0, nv, on_device=True, commit_column=True, commit_advance=True)
    try:
        a.add_groups(g, m)
        b.add_groups(g, m)
        got = a.step_sized(grp, sizes, len(ev), data)
        want = b.step_sized(grp, sizes, len(ev), data)
        assert "ready_compact" not in got
        np.testing.assert_array_equal(got["ready"], want["ready"])
        r4 = got["ready"][got["ready"]["cluster_id"] == cids[special]]
        assert len(r4) == 1 and int(r4["index"][0]) == big
        before = np.array([a.get_group(int(c))[0]["committed"] for c in cids], np.uint64)
        grp, off, ev = bench.step_events(hq, G, 1, roles)
        ev["log_index"][(ev["kind"] == hq.EV_MESSAGE) & (ev["type"] == 13)] = 0   # no commits
        data, sizes = hq.encode_events_sized(off, ev)
        got = a.step_sized(grp, sizes, len(ev), data)
        want = b.step_sized(grp, sizes, len(ev), data)
        assert "ready_compact" in got
        np.testing.assert_array_equal(_expand(hq, got, cids, before), want["ready"])
    finally:
        a.close()
        b.close()


def test_ready_compact_needs_the_device_worker(hq):
    with pytest.raises(hq.HQError):
        hq.Worker(0, 3, on_device=False, ready_compact=True)


def _consecutive_groups(rng, G):
    """Groups whose members are node ids 1..n (the leader node 1), in a random member order: the
    followers' acks then arrive as runs of consecutive senders (the stream's consecutive form)."""
    groups = []
    for j in range(G):
        n = int(rng.integers(3, 9))
        n_wit = int(rng.integers(0, 2)) if n >= 4 else 0
        n_obs = int(rng.integers(0, 3)) if n - n_wit >= 3 else 0
        roles = [sc.REMOTE] * (n - n_wit - n_obs) + [sc.WITNESS] * n_wit + [sc.OBSERVER] * n_obs
        state = int(rng.choice([sc.LEADER] * 7 + [sc.CANDIDATE, sc.FOLLOWER]))
        term = int(rng.integers(2, 9))
        last = 100 + int(rng.integers(0, 50))
        term_start = last - int(rng.integers(0, 6))
        committed = last - int(rng.integers(0, 9))
        mem = []
        for i, r in zip(range(1, n + 1), roles):
            m = last if i == 1 else (int(rng.integers(max(0, committed - 3), last + 1))
                                     if state == sc.LEADER else 0)
            mem.append((i, m, r, int(rng.random() < 0.5)))
        order = rng.permutation(n)
        groups.append((1 + j, 1, term, state, committed, last, term_start,
                       [mem[k] for k in order]))
    return groups


def _run_events(rng, state, ctx_seq):
    """One step of a group inside the worker's contract: maybe a ReadIndex, then runs of
    ReplicateResps and HeartbeatResps from consecutive node ids (some past the members, some from
    the node itself) at the group's term or another, rejecting now and then, at or below
    lastIndex, HeartbeatResps without a ctx from anyone and with a pending ctx from voting members
    only (an observer acking a ctx is the worker's fallback); maybe CheckQuorum and a proposal."""
    term, st, committed, last, ts, mem, reads = state
    ev = []
    ctxs = [r[2] for r in reads]
    if rng.random() < 0.3 and len(ctxs) < 8:
        ctx_seq[0] += 1
        c = (ctx_seq[0], 7)
        ctxs.append(c)
        ev.append(("read", c[0], c[1]))
    n = len(mem)
    n_vote = sum(1 for m in mem if m[2] != sc.OBSERVER)     # (observers hold the top ids)
    for _ in range(int(rng.integers(1, 4))):
        t = int(rng.choice([term] * 17 + [0, term - 1, term + 1]))
        if rng.random() < 0.5:
            s0, k = int(rng.integers(1, 4)), int(rng.integers(3, n + 3))
            idx = int(rng.choice([last, last, last - 1, committed]))
            rej = int(rng.random() < 0.1)
            ev += [sc.msg(sc.RREP, s0 + i, t, idx, reject=rej) for i in range(k)]
        elif ctxs and rng.random() < 0.4 and n_vote >= 3:
            c = ctxs[int(rng.integers(len(ctxs)))]
            s0 = int(rng.integers(1, n_vote - 1))
            k = int(rng.integers(3, n_vote - s0 + 2))
            ev += [sc.msg(sc.HBRESP, s0 + i, t, hint=c[0], high=c[1]) for i in range(k)]
        else:
            s0, k = int(rng.integers(1, 4)), int(rng.integers(3, n + 3))
            ev += [sc.msg(sc.HBRESP, s0 + i, t) for i in range(k)]
    if rng.random() < 0.2:
        ev.append(("check_quorum",))
    if rng.random() < 0.5:
        ev.append(("propose", 1))
    return ev


@pytest.mark.parametrize("stream", [True, "sized16", "sized16-slots"])
@pytest.mark.parametrize("seed", [31, 32])
def test_consecutive_runs_device_equals_reference(hq, seed, stream):
    """Runs of acks from consecutive node ids, which the device takes a run at a time where each
    member can only raise its match and mark itself active (hq_dstep.hip take_run), against the
    reference replay (oracle/qref_step.c) taking the same events one at a time: every output list
    and every group's state equal, no fallback."""
    rng = np.random.default_rng(seed)
    o = OracleBackend()
    dev = WorkerBackend(hq, n_max=8, seed=seed, on_device=True, stream=stream)
    try:
        groups = _consecutive_groups(rng, 2000)
        for g in groups:
            o.add_group(*g)
            dev.add_group(*g)
        ctx_seq = [0]
        events = 0
        for s in range(5):
            per = {g[0]: _run_events(rng, o.state(g[0]), ctx_seq) for g in groups
                   if rng.random() < 0.9}
            events += sum(len(e) for e in per.values())
            want, got = o.step(per), dev.step(per)
            assert got["_fallback"] == []
            for cid in per:
                same_step(want, got, cid)
            for g in groups:
                assert dev.state(g[0]) == o.state(g[0]), (s, g[0])
        assert events > 20000
    finally:
        dev.close()
