"""The event stream (include/hipquorum.h "event streams", dragonboat_amd/csrc/hq_stream.cpp):
rows -> bytes -> rows keeps every field a handler reads (the others come back 0), steady-state
events take a few bytes, and malformed streams are rejected. CPU only (host encoder/decoder);
the device decoder is checked against these bytes through the step worker in
tests/test_gpu_worker.py (device-stream feeds)."""
import numpy as np
import pytest

RREP, VRESP, HBRESP, READIDX = 13, 15, 18, 19


def carried(hq, ev):
    """The fields the stream carries for each row (the rest zeroed), as the decoder returns."""
    out = np.zeros_like(ev)
    kind = ev["kind"].copy()
    kind[(kind < 1) | (kind > 5)] = 0
    out["kind"] = kind
    rd = kind == hq.EV_READ
    pr = kind == hq.EV_PROPOSE
    ms = kind == hq.EV_MESSAGE
    out["hint"][rd], out["hint_high"][rd] = ev["hint"][rd], ev["hint_high"][rd]
    out["log_index"][pr] = ev["log_index"][pr]
    t = ev["type"]
    known = np.isin(t, [RREP, VRESP, HBRESP, READIDX])
    out["type"][ms] = t[ms]
    out["reject"][ms] = ev["reject"][ms] != 0
    out["from"][ms], out["term"][ms] = ev["from"][ms], ev["term"][ms]
    li = ms & ((t == RREP) | ~known)
    out["log_index"][li] = ev["log_index"][li]
    hh = ms & (((t == HBRESP) | (t == READIDX)) | ~known)
    out["hint"][hh], out["hint_high"][hh] = ev["hint"][hh], ev["hint_high"][hh]
    return out


def random_rows(rng, ne, small=False):
    """Random rows; small: indexes and ctxs from {0, 1, 2}, so that the codes repeating a
    group's previous index (4) or ctx (5) fire often."""
    ev = np.zeros(ne, dtype=[("kind", "<u4"), ("type", "<u4"), ("from", "<u8"),
                             ("term", "<u8"), ("log_index", "<u8"), ("hint", "<u8"),
                             ("hint_high", "<u8"), ("reject", "<u4"), ("reserved", "<u4")])
    ev["kind"] = rng.choice([0, 1, 2, 2, 2, 2, 3, 4, 5, 6, 9], ne)
    ev["type"] = rng.choice([RREP, VRESP, HBRESP, READIDX, 1, 22, 1 << 31], ne)
    big = lambda: np.where(rng.random(ne) < 0.2, rng.integers(0, 2**63, ne, dtype=np.uint64) * 2
                           + 1, rng.integers(0, 300, ne).astype(np.uint64))
    for k in ("from", "log_index", "hint", "hint_high"):
        ev[k] = rng.integers(0, 3, ne).astype(np.uint64) if small and k != "from" else big()
    ev["term"] = np.where(rng.random(ne) < 0.7, 7, big())        # mostly repeating
    ev["reject"] = rng.choice([0, 0, 1, 5], ne)
    ev["reserved"] = rng.integers(0, 9, ne)
    return ev


@pytest.mark.parametrize("seed,small", [(1, False), (2, False), (3, False), (4, True),
                                        (5, True)])
def test_round_trip(hq, seed, small):
    rng = np.random.default_rng(seed)
    n = 500
    counts = rng.integers(0, 12, n)
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
    ev = random_rows(rng, int(off[-1]), small).view(hq.EVENT_DTYPE)
    data, boff = hq.encode_events(off, ev)
    assert boff[0] == 0 and np.all(np.diff(boff.astype(np.int64)) >= 0)
    assert len(data) <= len(ev) * hq.HQ_EVENT_STREAM_MAX
    back = hq.decode_events(off, boff, data)
    want = carried(hq, ev)
    for k in ("kind", "type", "from", "term", "log_index", "hint", "hint_high", "reject"):
        np.testing.assert_array_equal(back[k], want[k], err_msg=k)
    assert (back["reserved"] == 0).all()


def test_steady_state_sizes(hq):
    """A leader's steady step: ReplicateResp / HeartbeatResp at the group's term, a proposal."""
    ev = np.zeros(6, hq.EVENT_DTYPE)
    ev[0] = (hq.EV_MESSAGE, RREP, 2, 41, 1_000_000, 0, 0, 0, 0)     # first message: the term
    ev[1] = (hq.EV_MESSAGE, RREP, 3, 41, 1_000_001, 0, 0, 0, 0)     # same term: 1 + 1 + 3
    ev[2] = (hq.EV_MESSAGE, HBRESP, 4, 41, 0, 0, 0, 0, 0)           # ctx-less ack: code 5
    ev[3] = (hq.EV_CHECK_QUORUM, 0, 0, 0, 0, 0, 0, 0, 0)
    ev[4] = (hq.EV_PROPOSE, 0, 0, 0, 3, 0, 0, 0, 0)
    ev[5] = (hq.EV_READ, 0, 0, 0, 0, 77, 0, 0, 0)
    off = np.array([0, 6], np.uint64)
    data, boff = hq.encode_events(off, ev)
    sizes = []
    for i in range(6):                     # per-event sizes from prefixes
        d, _ = hq.encode_events(np.array([0, i + 1], np.uint64), ev[:i + 1])
        sizes.append(len(d))
    sizes = np.diff([0] + sizes)
    assert list(sizes) == [1 + 1 + 1 + 3, 1 + 1 + 3, 1 + 1, 1, 2, 3]
    assert len(data) == sum(sizes) and int(boff[1]) == len(data)


def test_empty_and_groups_without_events(hq):
    off = np.array([0, 0, 0], np.uint64)
    data, boff = hq.encode_events(off, np.zeros(0, hq.EVENT_DTYPE))
    assert len(data) == 0 and list(boff) == [0, 0, 0]
    assert len(hq.decode_events(off, boff, data)) == 0


def test_malformed_rejected(hq):
    ev = np.zeros(2, hq.EVENT_DTYPE)
    ev[0] = (hq.EV_MESSAGE, RREP, 2, 41, 1_000_000, 0, 0, 0, 0)
    ev[1] = (hq.EV_READ, 0, 0, 0, 0, 5, 6, 0, 0)
    off = np.array([0, 2], np.uint64)
    data, boff = hq.encode_events(off, ev)
    with pytest.raises(hq.HQError):                          # truncated
        hq.decode_events(off, np.array([0, len(data) - 1], np.uint64), data[:-1])
    with pytest.raises(hq.HQError):                          # trailing bytes
        hq.decode_events(off, np.array([0, len(data) + 1], np.uint64),
                         np.concatenate([data, [0]]).astype(np.uint8))
    over = np.concatenate([data[:1], [0xFF] * 11, data[1:]]).astype(np.uint8)
    with pytest.raises(hq.HQError):                          # a varint over 64 bits
        hq.decode_events(off, np.array([0, len(over)], np.uint64), over)


def test_encode_capacity(hq):
    ev = np.zeros(3, hq.EVENT_DTYPE)
    ev["kind"] = hq.EV_CHECK_QUORUM
    off = np.array([0, 3], np.uint64)
    out = np.zeros(hq.HQ_EVENT_STREAM_MAX + 1, np.uint8)     # room checked per event
    boff = np.zeros(2, np.uint64)
    rc = hq.lib.hq_events_encode(1, off.ctypes.data, ev.ctypes.data, out.ctypes.data,
                                 len(out), boff.ctypes.data)
    assert rc == hq.HQ_E_STATE


@pytest.mark.parametrize("seed", [4, 5])
def test_sized_encoding_equals_prefix_encoding(hq, seed):
    """hq_events_encode_sized: the same bytes as hq_events_encode, and size words = (events,
    bytes) of each group = the differences of the two prefix arrays."""
    rng = np.random.default_rng(seed)
    n = 700
    counts = rng.integers(0, 12, n)
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
    ev = random_rows(rng, int(off[-1])).view(hq.EVENT_DTYPE)
    data, boff = hq.encode_events(off, ev)
    sdata, sizes = hq.encode_events_sized(off, ev)
    np.testing.assert_array_equal(sdata, data)
    np.testing.assert_array_equal(sizes & 0xFFFF, np.diff(off))
    np.testing.assert_array_equal(sizes >> 16, np.diff(boff))


def test_sized_encoding_limits(hq):
    """A group of 2^16 events (or bytes) does not fit a size word: HQ_E_INVAL."""
    ev = np.zeros(1 << 16, hq.EVENT_DTYPE)
    ev["kind"] = hq.EV_CHECK_QUORUM                           # 1 byte each
    with pytest.raises(hq.HQError):
        hq.encode_events_sized(np.array([0, 1 << 16], np.uint64), ev)
    data, sizes = hq.encode_events_sized(np.array([0, (1 << 16) - 1], np.uint64), ev[:-1])
    assert int(sizes[0]) == 0xFFFF | 0xFFFF << 16 and len(data) == 0xFFFF
    big = np.zeros(9000, hq.EVENT_DTYPE)                     # ~10 bytes each: > 2^16 bytes
    big["kind"], big["hint"], big["hint_high"] = hq.EV_READ, 1 << 40, 1 << 30
    with pytest.raises(hq.HQError):
        hq.encode_events_sized(np.array([0, 9000], np.uint64), big)


def test_repeated_replicate_index(hq):
    """Type code 4: a ReplicateResp whose log_index repeats the group's previous ReplicateResp
    (the followers of a steady leader ack the same index) leaves its index varint out; the
    decoder restores it, per group; a code 4 before any ReplicateResp of the group is malformed."""
    ev = np.zeros(5, hq.EVENT_DTYPE)
    ev[0] = (hq.EV_MESSAGE, RREP, 2, 41, 1_000_000, 0, 0, 0, 0)   # 1 + 1 + 1 + 3
    ev[1] = (hq.EV_MESSAGE, RREP, 3, 41, 1_000_000, 0, 0, 0, 0)   # 1 + 1: code 4
    ev[2] = (hq.EV_MESSAGE, HBRESP, 4, 41, 0, 0, 0, 0, 0)         # ctx-less: 1 + 1, code 5
    ev[3] = (hq.EV_MESSAGE, RREP, 4, 41, 1_000_000, 0, 0, 1, 0)   # rejected, same index: code 4
    ev[4] = (hq.EV_MESSAGE, RREP, 5, 41, 999, 0, 0, 0, 0)         # another index: code 0
    off = np.array([0, 5], np.uint64)
    data, boff = hq.encode_events(off, ev)
    assert len(data) == 6 + 2 + 2 + 2 + (1 + 1 + 2)
    assert (data[6] >> 3) & 7 == 4 and (data[10] >> 3) & 7 == 4
    back = hq.decode_events(off, boff, data)
    want = carried(hq, ev)
    for k in ("kind", "type", "from", "term", "log_index", "hint", "hint_high", "reject"):
        np.testing.assert_array_equal(back[k], want[k], err_msg=k)
    # per group: the second group's first ReplicateResp is written in full
    off2 = np.array([0, 1, 2], np.uint64)
    d2, b2 = hq.encode_events(off2, ev[:2])
    assert int(b2[1]) == 6 and int(b2[2]) == 12
    bad = np.array([hq.EV_MESSAGE | 4 << 3 | 0x80, 2], np.uint8)
    with pytest.raises(hq.HQError):
        hq.decode_events(np.array([0, 1], np.uint64), np.array([0, 2], np.uint64), bad)


def test_repeated_heartbeat_ctx(hq):
    """Type code 5: a HeartbeatResp whose hint / hint_high repeat the group's previous
    HeartbeatResp (0 / 0 before the first: a ctx-less ack, or every follower acking the same
    ReadIndex ctx) leaves both varints out; a ReadIndex between them does not reset it."""
    ev = np.zeros(6, hq.EVENT_DTYPE)
    ev[0] = (hq.EV_MESSAGE, HBRESP, 2, 41, 0, 0, 0, 0, 0)         # 1 + 1 + 1: code 5 (0 / 0)
    ev[1] = (hq.EV_MESSAGE, HBRESP, 3, 41, 0, 900, 7, 0, 0)       # a ctx: 1 + 1 + 2 + 1, code 2
    ev[2] = (hq.EV_MESSAGE, 19, 9, 41, 0, 5, 6, 0, 0)             # ReadIndex (code 3)
    ev[3] = (hq.EV_MESSAGE, HBRESP, 4, 41, 0, 900, 7, 0, 0)       # same ctx: 1 + 1, code 5
    ev[4] = (hq.EV_MESSAGE, HBRESP, 5, 41, 0, 900, 8, 1, 0)       # another high: code 2
    ev[5] = (hq.EV_MESSAGE, HBRESP, 6, 41, 0, 0, 0, 0, 0)         # back to 0 / 0: code 2
    off = np.array([0, 6], np.uint64)
    data, boff = hq.encode_events(off, ev)
    back = hq.decode_events(off, boff, data)
    want = carried(hq, ev)
    for k in ("kind", "type", "from", "term", "log_index", "hint", "hint_high", "reject"):
        np.testing.assert_array_equal(back[k], want[k], err_msg=k)
    codes = []
    d, prev = None, 0
    for i in range(6):
        d, _ = hq.encode_events(np.array([0, i + 1], np.uint64), ev[:i + 1])
        codes.append((int(d[prev]) >> 3) & 7)
        prev = len(d)
    assert codes == [5, 2, 3, 5, 2, 2]
    assert len(data) == 3 + 5 + 4 + 2 + 5 + 4
    # per group: a group's first ctx-ful ack is written in full even if the last group's matched
    off2 = np.array([0, 2, 3], np.uint64)
    d2, b2 = hq.encode_events(off2, ev[[0, 1, 3]])
    assert (int(d2[int(b2[1])]) >> 3) & 7 == 2


# --- compact 16-byte records (hq_event16, hq_events16_encode_sized) ----------------------------

def _random_groups(hq, seed, n=700, small=False):
    rng = np.random.default_rng(seed)
    counts = rng.integers(0, 12, n)
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
    ev = random_rows(rng, int(off[-1]), small).view(hq.EVENT_DTYPE)
    # ReadIndex acks: some groups read, then their heartbeats carry that ctx (READ_CTX records)
    for i in range(0, n, 3):
        a, b = int(off[i]), int(off[i + 1])
        if b - a >= 2:
            ev[a]["kind"], ev[a]["hint"], ev[a]["hint_high"] = hq.EV_READ, 1000 + i, 7
            for j in range(a + 1, b, 2):
                ev[j]["kind"], ev[j]["type"] = hq.EV_MESSAGE, HBRESP
                ev[j]["hint"], ev[j]["hint_high"] = 1000 + i, 7
    return off, ev


@pytest.mark.parametrize("seed,small", [(11, False), (12, False), (13, True)])
@pytest.mark.parametrize("threads", [1, 3, 8])
def test_compact_records_encode_like_rows(hq, seed, small, threads):
    """Rows -> hq_events_to16 -> hq_events16_encode_sized writes the bytes and size words of
    hq_events_encode_sized on the rows themselves, on any thread count: random rows with big
    node ids / terms / ctxs (escapes), invalid kinds, other message types, ReadIndex acks."""
    off, ev = _random_groups(hq, seed, small=small)
    want_data, want_sizes = hq.encode_events_sized(off, ev)
    recs, off16 = hq.events_to16(off, ev)
    full = (recs["kind"] & hq.EV16_FULL) != 0
    assert full.any() and (recs["kind"] & hq.EV16_READ_CTX).any() and (~full).sum() > len(ev) // 3
    data, sizes, ne = hq.encode_events16_sized(off16, recs, threads=threads)
    np.testing.assert_array_equal(data, want_data)
    np.testing.assert_array_equal(sizes, want_sizes)
    assert ne == len(ev)


@pytest.mark.parametrize("name", ["step", "step5"])
def test_compact_step_workload_has_no_escapes(hq, name):
    """The bench's steady-state step (tests on bench.step_events): every event fits one 16-byte
    record (no escape), the heartbeat acks of a ReadIndex refer to its READ, and the encoding
    equals the rows' on 16 threads."""
    import bench

    roles = bench.STEP_ROLES[name]
    grp, off, ev = bench.step_events(hq, 4096, 3, roles)
    recs, off16 = hq.events_to16(off, ev)
    np.testing.assert_array_equal(off16, off)
    assert not (recs["kind"] & hq.EV16_FULL).any()
    assert np.count_nonzero(recs["kind"] & hq.EV16_READ_CTX) == 1024 * sum(
        r != "observer" for r in roles[1:])
    want_data, want_sizes = hq.encode_events_sized(off, ev)
    data, sizes, ne = hq.encode_events16_sized(off16, recs, threads=16)
    np.testing.assert_array_equal(data, want_data)
    np.testing.assert_array_equal(sizes, want_sizes)


def test_compact_records_malformed(hq):
    """An escape without its 4 records is HQ_E_INVAL; an output region too small is HQ_E_STATE."""
    recs = np.zeros(3, hq.EVENT16_DTYPE)
    recs["kind"] = hq.EV16_FULL
    with pytest.raises(hq.HQError):
        hq.encode_events16_sized(np.array([0, 3], np.uint64), recs)
    off, ev = _random_groups(hq, 21)
    recs, off16 = hq.events_to16(off, ev)
    _, want_sizes = hq.encode_events_sized(off, ev)
    nb = int((want_sizes >> 16).sum())
    for threads in (1, 4):
        out = np.zeros(nb - 1, np.uint8)
        sizes = np.zeros(len(off) - 1, np.uint32)
        with pytest.raises(hq.HQError):
            hq.encode_events16_sized_into(off16, recs, out, sizes, threads)


def test_compact_capacity_rule_same_on_every_thread_count(hq):
    """The capacity rule does not depend on the thread count: HQ_EVENT_STREAM_MAX
    bytes free before every event, as hq_events_encode_sized. Every cap from just below the
    stream's length to HQ_EVENT_STREAM_MAX past it succeeds or fails alike on 1, 4 and 8 threads,
    with the same bytes when it succeeds."""
    off, ev = _random_groups(hq, 22)
    recs, off16 = hq.events_to16(off, ev)
    want_data, want_sizes = hq.encode_events_sized(off, ev)
    nb = len(want_data)
    outcomes = set()
    for cap in range(nb - 2, nb + hq.HQ_EVENT_STREAM_MAX + 2):
        got = []
        for threads in (1, 4, 8):
            out = np.zeros(cap, np.uint8)
            sizes = np.zeros(len(off) - 1, np.uint32)
            try:
                ne, n = hq.encode_events16_sized_into(off16, recs, out, sizes, threads)
                assert (ne, n) == (len(ev), nb)
                np.testing.assert_array_equal(out[:n], want_data)
                np.testing.assert_array_equal(sizes, want_sizes)
                got.append("ok")
            except hq.HQError as e:
                assert e.code == hq.HQ_E_STATE
                got.append("state")
        assert len(set(got)) == 1, (cap, got)
        outcomes.add(got[0])
    assert outcomes == {"ok", "state"}   # the boundary lies inside the swept caps


def test_encode_stats_count_threaded_calls(hq):
    """hq_encode_stats_read: a threaded call is counted with its tasks and phase clocks."""
    off, ev = _random_groups(hq, 23, n=4000)
    recs, off16 = hq.events_to16(off, ev)
    hq.encode_stats(reset=True)
    hq.encode_events16_sized(off16, recs, threads=4)
    st = hq.encode_stats(reset=True)
    assert st["calls"] == 1 and st["tasks"] == 4          # 4 ranges, encoded and copied by one task each
    assert st["wall_ns"] >= st["encode_ns"] > 0 and st["run_ns"] > 0
    assert st["helped"] <= st["tasks"] and st["max_lag_ns"] <= st["lag_ns"]
    assert hq.encode_stats()["calls"] == 0


def test_threaded_encodes_side_by_side(hq):
    """Threaded encodes called from several threads at once share the encoder's task pool: each
    call's bytes and size words equal its single-thread encode."""
    import threading

    import bench
    G, W = 1 << 14, 4
    recs = bench.StepRows16(hq, G, bench.STEP_ROLES["step5"])
    off16, r = recs.set(3)
    b = [G * i // W for i in range(W + 1)]
    parts = [(off16[b[i]:b[i + 1] + 1] - off16[b[i]], int(off16[b[i]]), int(off16[b[i + 1]]))
             for i in range(W)]
    want = [hq.encode_events16_sized(o, r[e0:e1], 1) for o, e0, e1 in parts]
    bad = []

    def one(i, T):
        o, e0, e1 = parts[i]
        out = np.zeros((e1 - e0) * 5 + 64, np.uint8)
        sz = np.zeros(len(o) - 1, np.uint32)
        ne, nb = hq.encode_events16_sized_into(o, r[e0:e1], out, sz, T)
        if out[:nb].tobytes() != want[i][0].tobytes() or not np.array_equal(sz, want[i][1]):
            bad.append((i, T))
    for _ in range(5):
        th = [threading.Thread(target=one, args=(i, (2, 3, 4, 8)[i])) for i in range(W)]
        for t in th:
            t.start()
        for t in th:
            t.join()
    assert not bad


@pytest.mark.parametrize("threads,G", [(1, 1 << 13), (3, 1 << 13), (14, 1 << 13), (14, 1 << 16)])
def test_multi_encode_equals_one_call_per_job(hq, threads, G):
    """hq_events16_encode_sized_multi: 16 workers' streams (ragged: a worker with no groups, one
    with groups but no records, others of unequal size) encoded in one call whose chunks (taken
    by the threads from a shared counter: 26 and 112 chunks here) cross job boundaries; every
    job's bytes, size words and totals equal its own single call's."""
    import bench
    recs = bench.StepRows16(hq, G, bench.STEP_ROLES["step5"])
    off16, r = recs.set(2)
    b = sorted({0, G} | {int(x) for x in np.random.default_rng(5).integers(0, G, 14)})
    b = [0, 0] + b[1:]                       # worker 0: no groups
    parts = [(off16[b[i]:b[i + 1] + 1] - off16[b[i]], int(off16[b[i]]), int(off16[b[i + 1]]))
             for i in range(len(b) - 1)]
    empty = (np.zeros(4, np.uint64), 0, 0)   # 3 groups without records
    parts.insert(3, empty)
    want = [hq.encode_events16_sized(o, r[e0:e1], 1) for o, e0, e1 in parts]
    jobs = [(o, r[e0:e1], np.zeros((e1 - e0) * 5 + 64, np.uint8), np.zeros(len(o) - 1, np.uint32))
            for o, e0, e1 in parts]
    hq.encode_stats(reset=True)
    got = hq.encode_events16_sized_multi(jobs, threads)
    assert hq.encode_stats(reset=True)["calls"] == 1
    for (o, rr, out, sz), (ne, nb), (wd, ws, wne) in zip(jobs, got, want):
        assert ne == wne and nb == len(wd)
        np.testing.assert_array_equal(out[:nb], wd)
        np.testing.assert_array_equal(sz, ws)


def test_multi_encode_errors_per_job(hq):
    """A job whose region is too small fails with HQ_E_STATE and one with a malformed escape with
    HQ_E_INVAL, each in its own rc; the other jobs are encoded as alone."""
    off, ev = _random_groups(hq, 24, n=3000)
    recs, off16 = hq.events_to16(off, ev)
    wd, ws, wne = hq.encode_events16_sized(off16, recs, 1)
    bad = np.zeros(3, hq.EVENT16_DTYPE)
    bad["kind"] = hq.EV16_FULL
    for T in (1, 4):
        jobs = [(off16, recs, np.zeros(len(wd) + 64 * 8, np.uint8), np.zeros(len(off) - 1, np.uint32)),
                (off16, recs, np.zeros(len(wd) - 1, np.uint8), np.zeros(len(off) - 1, np.uint32)),
                (np.array([0, 3], np.uint64), bad, np.zeros(256, np.uint8), np.zeros(1, np.uint32))]
        arr = (hq.Encode16Job * 3)()
        for a, (o, rr, out, sz) in zip(arr, jobs):
            a.n_groups, a.offsets16, a.recs = len(o) - 1, o.ctypes.data, rr.ctypes.data
            a.out, a.cap, a.sizes = out.ctypes.data, len(out), sz.ctypes.data
        rc = hq.lib.hq_events16_encode_sized_multi(hq.ctypes.addressof(arr), 3, T)
        assert rc == hq.HQ_E_STATE            # the first failing job's
        assert [a.rc for a in arr] == [hq.HQ_OK, hq.HQ_E_STATE, hq.HQ_E_INVAL]
        assert arr[0].n_events == wne and arr[0].n_bytes == len(wd)
        np.testing.assert_array_equal(jobs[0][2][:len(wd)], wd)
        np.testing.assert_array_equal(jobs[0][3], ws)
        assert arr[1].n_bytes == 0 and arr[2].n_bytes == 0


# --- runs (code 6): acks repeating the group's previous message but for the sender --------------

def runny_rows(hq, rng, groups=300):
    """Groups whose steps a steady leader sees: runs of ReplicateResp / HeartbeatResp acks with one
    index / ctx, term and reject, senders random (some >= 2^16: escapes in the compact form),
    broken now and then by another index, a reject, another type, a READ or a proposal."""
    rows, off = [], [0]
    for _ in range(groups):
        term = int(rng.choice([7, 7, 7, 9, 1 << 40]))
        for _ in range(int(rng.integers(0, 5))):
            typ = int(rng.choice([RREP, RREP, HBRESP, HBRESP, VRESP]))
            idx, ctx = int(rng.choice([10, 11, 1 << 50])), int(rng.choice([0, 0, 5, 1 << 33]))
            rej = int(rng.random() < 0.15)
            for _ in range(int(rng.integers(1, 10))):
                frm = int(rng.choice([2, 3, 4, 5, 6, 7, 100, 300, 1 << 20]))
                r = (hq.EV_MESSAGE, typ, frm, term, idx if typ == RREP else 0,
                     ctx if typ == HBRESP else 0, 0, rej, 0)
                if rng.random() < 0.08:
                    r = (hq.EV_MESSAGE, typ, frm, term, idx + 1 if typ == RREP else 0,
                         ctx + 1 if typ == HBRESP else 0, 0, rej, 0)
                rows.append(r)
            if rng.random() < 0.3:
                rows.append((hq.EV_READ, 0, 0, 0, 0, int(rng.integers(1, 99)), 0, 0, 0))
            if rng.random() < 0.3:
                rows.append((hq.EV_PROPOSE, 0, 0, 0, 3, 0, 0, 0, 0))
        off.append(len(rows))
    return np.array(rows, dtype=hq.EVENT_DTYPE), np.array(off, np.uint64)


@pytest.mark.parametrize("seed", [31, 32, 33])
@pytest.mark.parametrize("threads", [1, 4])
def test_runs_round_trip(hq, seed, threads):
    """Runs are written by the row encoder and the compact-record encoder alike (escaped senders
    included), never longer than 6 events, and decode back to the rows."""
    ev, off = runny_rows(hq, np.random.default_rng(seed))
    data, boff = hq.encode_events(off, ev)
    hdr_run = 2 | 6 << 3
    assert (data == hdr_run).sum() > 50
    np.testing.assert_array_equal(hq.decode_events(off, boff, data), carried(hq, ev))
    want, want_sizes = hq.encode_events_sized(off, ev)
    np.testing.assert_array_equal(want, data)
    recs, off16 = hq.events_to16(off, ev)
    assert (recs["kind"] & hq.EV16_FULL).any()
    got, sizes, ne = hq.encode_events16_sized(off16, recs, threads=threads)
    np.testing.assert_array_equal(got, data)
    np.testing.assert_array_equal(sizes, want_sizes)
    assert ne == len(ev)


def _one_group(hq, rows):
    ev = np.array(rows, dtype=hq.EVENT_DTYPE)
    return ev, np.array([0, len(ev)], np.uint64)


def test_run_length_and_split(hq):
    """A ReplicateResp and 8 repeats: the first in full, a run of 6, then two code-4 events (a run
    needs 3); the same message with another term, index or reject breaks a run. Senders in node
    order make the run's consecutive form (header bit 7, the count, the first sender)."""
    senders = [2, 5, 3, 9, 4, 7, 6, 8, 10]
    rows = [(hq.EV_MESSAGE, RREP, senders[i], 41, 1000, 0, 0, 0, 0) for i in range(9)]
    ev, off = _one_group(hq, rows)
    data, _ = hq.encode_events(off, ev)
    # code 0: header, from, term (41), index (1000: 2 bytes) = 5; run: header, 6, six senders = 8;
    # two code-4 events of 2 bytes
    assert len(data) == 5 + 8 + 4
    assert data[5] == (2 | 6 << 3) and data[6] == 6 and list(data[7:13]) == senders[1:7]
    seq = ev.copy()
    seq["from"] = np.arange(2, 11)
    d_seq, _ = hq.encode_events(off, seq)
    assert len(d_seq) == 5 + 3 + 4
    assert d_seq[5] == (2 | 6 << 3 | 0x80) and d_seq[6] == 6 and d_seq[7] == 3
    np.testing.assert_array_equal(
        hq.decode_events(off, np.array([0, len(d_seq)], np.uint64), d_seq), carried(hq, seq))
    recs, off16 = hq.events_to16(off, seq)
    got, _, _ = hq.encode_events16_sized(off16, recs)
    np.testing.assert_array_equal(got, d_seq)
    np.testing.assert_array_equal(hq.decode_events(off, np.array([0, len(data)], np.uint64), data),
                                  carried(hq, ev))
    for k, v in (("term", 42), ("log_index", 1001), ("reject", 1)):
        ev2 = ev.copy()
        ev2[3][k] = v
        d2, _ = hq.encode_events(off, ev2)
        assert (d2 == (2 | 6 << 3)).sum() <= 1 and len(d2) > len(data)
        np.testing.assert_array_equal(
            hq.decode_events(off, np.array([0, len(d2)], np.uint64), d2), carried(hq, ev2))


def test_run_malformed(hq):
    """A run with nothing to repeat (first in the group, or after a RequestVoteResp), a count of
    0, or a count past the group's events is HQ_E_INVAL."""
    run = 2 | 6 << 3
    bad = [
        (np.array([run, 1, 5], np.uint8), 1),                       # nothing before it
        (np.array([2 | 1 << 3, 5, 7, run, 1, 6], np.uint8), 2),     # after a RequestVoteResp
        (np.array([2 | 0 << 3, 5, 7, 9, run, 0], np.uint8), 2),     # count 0
        (np.array([2 | 0 << 3, 5, 7, 9, run, 3, 6, 7, 8], np.uint8), 3),   # 3 announced, 2 left
        (np.array([2 | 0 << 3, 5, 7, 9, run | 0x80, 3], np.uint8), 4),      # consecutive, no s0
        # consecutive senders past 2^32 - 1
        (np.array([2 | 0 << 3, 5, 7, 9, run | 0x80, 3, 0xFE, 0xFF, 0xFF, 0xFF, 0x0F], np.uint8), 4),
    ]
    for data, n in bad:
        with pytest.raises(hq.HQError):
            hq.decode_events(np.array([0, n], np.uint64), np.array([0, len(data)], np.uint64),
                             data)


@pytest.mark.parametrize("threads", [1, 2, 5])
def test_multi_encode_bad_job_before_good_ones(hq, threads):
    """A malformed job ahead of good ones in the same thread's pieces: the good jobs' bytes land
    where their own calls put them (a thread's pieces follow each other in its scratch, and a
    failed piece takes no room)."""
    off, ev = _random_groups(hq, 25, n=2000)
    recs, off16 = hq.events_to16(off, ev)
    wd, ws, wne = hq.encode_events16_sized(off16, recs, 1)
    bad = np.zeros(3, hq.EVENT16_DTYPE)
    bad["kind"] = hq.EV16_FULL
    jobs = [(np.array([0, 3], np.uint64), bad, np.zeros(256, np.uint8), np.zeros(1, np.uint32))]
    jobs += [(off16, recs, np.zeros(len(wd) + 64 * 8, np.uint8), np.zeros(len(off) - 1, np.uint32))
             for _ in range(2)]
    arr = (hq.Encode16Job * 3)()
    for a, (o, rr, out, sz) in zip(arr, jobs):
        a.n_groups, a.offsets16, a.recs = len(o) - 1, o.ctypes.data, rr.ctypes.data
        a.out, a.cap, a.sizes = out.ctypes.data, len(out), sz.ctypes.data
    rc = hq.lib.hq_events16_encode_sized_multi(hq.ctypes.addressof(arr), 3, threads)
    assert rc == hq.HQ_E_INVAL
    assert [a.rc for a in arr] == [hq.HQ_E_INVAL, hq.HQ_OK, hq.HQ_OK]
    for a, (o, rr, out, sz) in zip(arr[1:], jobs[1:]):
        assert a.n_events == wne and a.n_bytes == len(wd)
        np.testing.assert_array_equal(out[:len(wd)], wd)
        np.testing.assert_array_equal(sz, ws)


def test_encode_batch_reuses_its_buffers(hq):
    """hq.Encode16Batch: one job table, called step after step while the records change in place
    (StepRows16.set): every call's bytes and sizes equal a fresh call's."""
    import bench
    G = 1 << 12
    recs = bench.StepRows16(hq, G, bench.STEP_ROLES["step5"])
    off16, r = recs.set(0)
    bounds = [0, G // 3, G // 2, G]
    parts = [(off16[b0:b1 + 1] - off16[b0], int(off16[b0]), int(off16[b1]))
             for b0, b1 in zip(bounds, bounds[1:])]
    bufs = [(np.zeros((e1 - e0) * 5 + 64, np.uint8), np.zeros(len(o) - 1, np.uint32))
            for o, e0, e1 in parts]
    batch = hq.Encode16Batch([(o, r[e0:e1], out, sz) for (o, e0, e1), (out, sz) in zip(parts, bufs)])
    for s in range(3):
        recs.set(s)
        got = batch.run(4)
        for (o, e0, e1), (out, sz), (ne, nb) in zip(parts, bufs, got):
            wd, ws, wne = hq.encode_events16_sized(o, r[e0:e1], 1)
            assert ne == wne and nb == len(wd)
            np.testing.assert_array_equal(out[:nb], wd)
            np.testing.assert_array_equal(sz, ws)
