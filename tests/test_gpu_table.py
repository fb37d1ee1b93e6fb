"""The device-resident progress table in the headline layout (HQ_LAYOUT_TILES_LEADER tiles,
SURVEY.md §8f-1): the hq_table_* delta kernels against the oracle's sequential restatements
(remote.tryUpdate, appendEntries) with atomics and with the grouped (segmented-scan) path, the
in-place decision against the oracle's tryCommit, and the host-fed pipeline built on them."""
import numpy as np
import pytest

from oracle import qref

SEED = 0x5EED7000
pytestmark = pytest.mark.gpu


def _table(ctx, hq, inp, form):
    """Leader-row tiles of a generated batch, packed by the host packer, uploaded."""
    G, n = inp.G, inp.n_max
    a = hq.CommitArgs()
    a.G, a.n_max, a.form, a.ring_len, a.match_stride = G, n, form, inp.R, G
    a.match, a.committed_in = inp.match.ctypes.data, inp.committed_in.ctypes.data
    a.last_index = inp.last_index.ctypes.data
    a.term_mask, a.term_start = inp.term_mask.ctypes.data, inp.term_start.ctypes.data
    tiles = hq.tile_commit_host(a, hq.HQ_LAYOUT_TILES_LEADER)
    return ctx.upload(tiles)


def _view(ctx, hq, dt, G, n, form):
    return hq.tile_view(ctx.download(dt), G, n, form, hq.HQ_LAYOUT_TILES_LEADER)


def _match_updates(rng, G, n, count, last, grouped, dup=True):
    g = rng.integers(0, G, count, dtype=np.uint64)
    s = rng.integers(0, n + 2, count, dtype=np.uint64)        # slot 0 and >= n are skipped
    g[rng.random(count) < 0.01] += np.uint64(G)               # group out of range
    idx = last[g % np.uint64(G)] - rng.integers(0, 24, count, dtype=np.uint64)
    key = (g << np.uint64(8)) | s
    if grouped:
        o = np.argsort(key, kind="stable")
        key, idx = key[o], idx[o]
    return np.stack([key, idx], axis=1).astype(np.uint64)


# ingest modes: the per-record atomic kernel, the default (binned for these dense batches), the
# binned two-pass kernels forced, the grouped segmented scan
MODES = ["atomic", "default", "binned", "grouped"]


def _flags(hq, mode):
    return {"atomic": hq.HQ_INGEST_ATOMIC, "default": 0, "binned": hq.HQ_INGEST_BINNED,
            "grouped": hq.HQ_INGEST_GROUPED}[mode]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("form", [2, 0])
def test_table_ingest_match(gpu_ctx, hq, mode, form):
    grouped = mode == "grouped"
    rng = np.random.default_rng(SEED + MODES.index(mode) + 7 * form)
    G, n = 70_001, 5
    inp = qref.CommitInputs(qref.spec(SEED + 1, G, n))
    dt = _table(gpu_ctx, hq, inp, form)
    upd = _match_updates(rng, G, n, 400_000, inp.last_index, grouped)
    # indexes of 2^48 and more (the binned entries cannot hold them: applied with an atomic)
    upd[[10, 20, 30], 1] = np.uint64(1 << 50) + np.arange(3, dtype=np.uint64)
    if grouped:   # long runs of one key across wave edges too
        upd = np.concatenate([upd[:1000], np.repeat(upd[1000:1003], 150, axis=0), upd[1003:]])
        o = np.argsort(upd[:, 0], kind="stable")
        upd = upd[o]
    s = upd[:, 0] & np.uint64(0xFF)
    g = upd[:, 0] >> np.uint64(8)
    valid = (g < G) & (s >= 1) & (s < n)
    want = inp.match.copy()
    qref.ingest_match(upd[valid].copy(), want, G, G, n)
    du = gpu_ctx.upload(upd.reshape(-1))
    skip = gpu_ctx.upload(np.zeros(1, np.uint64))
    gpu_ctx.table_ingest_match_dev(du, len(upd), dt, G, n, form, _flags(hq, mode), skip)
    v = _view(gpu_ctx, hq, dt, G, n, form)
    np.testing.assert_array_equal(v.match().reshape(-1), want)
    np.testing.assert_array_equal(v.row("committed"), inp.committed_in)
    assert int(gpu_ctx.download(skip)[0]) == int((~valid).sum())
    for x in (dt, du, skip):
        gpu_ctx.free(x)


@pytest.mark.parametrize("mode", MODES)
def test_table_ingest_lag(gpu_ctx, hq, mode):
    grouped = mode == "grouped"
    rng = np.random.default_rng(SEED + 10 + MODES.index(mode))
    G, n = 50_003, 4
    form = hq.HQ_FORM_TERM_MASK
    inp = qref.CommitInputs(qref.spec(SEED + 2, G, n))
    # five groups near the start of the log, so that acks above their lastIndex fit a lag
    inp.last_index[:5] = inp.match[:5] = inp.committed_in[:5] = 10
    dt = _table(gpu_ctx, hq, inp, form)
    cnt = 300_000
    g = rng.integers(0, G, cnt, dtype=np.uint64)
    s = rng.integers(0, n + 1, cnt, dtype=np.uint64)
    lag = rng.integers(0, 40, cnt, dtype=np.uint64)
    g[:5], s[:5], lag[:5] = np.arange(5), 1, 11                # above lastIndex: skipped
    g[5:9] = np.uint64(G + 3)                                  # out of range: skipped
    wire = hq.pack_lag_updates(g, s, lag)
    if grouped:
        wire = wire[np.argsort(wire >> np.uint64(28), kind="stable")]
    wg, ws, wl = wire >> np.uint64(32), (wire >> np.uint64(28)) & np.uint64(15), \
        wire & np.uint64((1 << 28) - 1)
    valid = (wg < G) & (ws >= 1) & (ws < n)
    valid &= wl <= inp.last_index[np.minimum(wg, G - 1)]
    want = inp.match.copy()
    upd = np.stack([(wg[valid] << np.uint64(8)) | ws[valid],
                    inp.last_index[wg[valid]] - wl[valid]], axis=1).astype(np.uint64)
    qref.ingest_match(upd, want, G, G, n)
    du = gpu_ctx.upload(wire)
    skip = gpu_ctx.upload(np.zeros(1, np.uint64))
    gpu_ctx.table_ingest_lag_dev(du, len(wire), dt, G, n, form, _flags(hq, mode), skip)
    v = _view(gpu_ctx, hq, dt, G, n, form)
    np.testing.assert_array_equal(v.match().reshape(-1), want)
    assert int(gpu_ctx.download(skip)[0]) == int((~valid).sum())
    for x in (dt, du, skip):
        gpu_ctx.free(x)


@pytest.mark.parametrize("lag", [False, True])
@pytest.mark.parametrize("n", [2, 3, 8])
def test_binned_ingest_many_launches_and_shapes(hq, monkeypatch, lag, n):
    """The binned ingest split over several launch pairs (HQ_BIN_LAUNCH_CHUNKS = 3 chunks of
    8192 records per pair), a ragged last tile, a batch that is not a multiple of the chunk, and
    voter counts whose match rows shrink the regions (n = 8: 7 rows, 16 tiles per region):
    equal to the oracle's sequential tryUpdate."""
    monkeypatch.setenv("HQ_BIN_LAUNCH_CHUNKS", "3")
    rng = np.random.default_rng(SEED + 50 + n + 10 * lag)
    G, form = 30_011, hq.HQ_FORM_TERM_MASK
    inp = qref.CommitInputs(qref.spec(SEED + 7, G, n))
    with hq.Context(0) as ctx:
        dt = _table(ctx, hq, inp, form)
        cnt = 8192 * 7 + 4321
        g = rng.integers(0, G, cnt, dtype=np.uint64)
        s = rng.integers(1, n, cnt, dtype=np.uint64)
        lagv = rng.integers(0, 30, cnt, dtype=np.uint64)
        want = inp.match.copy()
        if lag:
            wire = hq.pack_lag_updates(g, s, lagv)
            ok = lagv <= inp.last_index[g]
            upd = np.stack([(g[ok] << np.uint64(8)) | s[ok], inp.last_index[g[ok]] - lagv[ok]],
                           axis=1).astype(np.uint64)
        else:
            upd = np.stack([(g << np.uint64(8)) | s, inp.last_index[g] - lagv],
                           axis=1).astype(np.uint64)
            wire = upd.reshape(-1)
            ok = np.ones(cnt, bool)
        qref.ingest_match(upd.copy(), want, G, G, n)
        du = ctx.upload(wire)
        skip = ctx.upload(np.zeros(1, np.uint64))
        if lag:
            ctx.table_ingest_lag_dev(du, cnt, dt, G, n, form, hq.HQ_INGEST_BINNED, skip)
        else:
            ctx.table_ingest_match_dev(du, cnt, dt, G, n, form, hq.HQ_INGEST_BINNED, skip)
        v = _view(ctx, hq, dt, G, n, form)
        np.testing.assert_array_equal(v.match().reshape(-1), want)
        np.testing.assert_array_equal(v.row("committed"), inp.committed_in)
        np.testing.assert_array_equal(v.row("last_index"), inp.last_index)
        assert int(ctx.download(skip)[0]) == int((~ok).sum())
        with pytest.raises(hq.HQError):          # modes that exclude each other
            ctx.table_ingest_match_dev(du, 4, dt, G, n, form,
                                       hq.HQ_INGEST_BINNED | hq.HQ_INGEST_GROUPED)
        with pytest.raises(hq.HQError):
            ctx.table_ingest_match_dev(du, 4, dt, G, n, form,
                                       hq.HQ_INGEST_ATOMIC | hq.HQ_INGEST_UNIQUE)


@pytest.mark.parametrize("grouped", [False, True])
@pytest.mark.parametrize("counts", [False, True])
def test_table_append(gpu_ctx, hq, grouped, counts):
    rng = np.random.default_rng(SEED + 20 + grouped + 2 * counts)
    G, n, R = 40_009, 3, 16
    form = hq.HQ_FORM_TERM_MASK
    inp = qref.CommitInputs(qref.spec(SEED + 3, G, n))
    dt = _table(gpu_ctx, hq, inp, form)
    cnt = 120_000
    g = rng.integers(0, 20_000, cnt, dtype=np.uint64)          # duplicates: runs per group
    g[:7] = np.uint64(G + 1)                                   # out of range
    if grouped:
        g = np.sort(g, kind="stable")
    k = rng.choice(np.array([0, 1, 2, 3, 5, 15, 16, 17, 40], np.uint64), cnt)
    last, match0, mask = inp.last_index.copy(), inp.match[:G].copy(), inp.term_mask.copy()
    if counts:
        seq, cur = [], last.copy()
        for gg, kk in zip(g, k):                               # the sequential meaning: += n
            if gg < G and kk:
                cur[gg] += kk
                seq.append((gg, cur[gg]))
        qref.append(np.array(seq, np.uint64).reshape(-1, 2), last, match0, mask, R, G)
        wire = hq.pack_append_counts(g, k)
        n_bad = int(((g >= G) | (k == 0)).sum())
    else:
        newl = last[np.minimum(g, G - 1)] + k
        newl[rng.random(cnt) < 0.05] -= np.uint64(3)           # stale appends: no-op
        app = np.stack([g, newl], axis=1).astype(np.uint64)
        qref.append(app, last, match0, mask, R, G)
        wire = app.reshape(-1)
        n_bad = int((g >= G).sum())
    du = gpu_ctx.upload(wire)
    skip = gpu_ctx.upload(np.zeros(1, np.uint64))
    f = gpu_ctx.table_append_count_dev if counts else gpu_ctx.table_append_dev
    f(du, cnt, dt, G, n, form, R, hq.HQ_INGEST_GROUPED if grouped else 0, skip)
    v = _view(gpu_ctx, hq, dt, G, n, form)
    np.testing.assert_array_equal(v.row("last_index"), last)
    np.testing.assert_array_equal(v.row("aux"), mask)
    np.testing.assert_array_equal(v.match()[1:], inp.match.reshape(n, G)[1:])
    assert int(gpu_ctx.download(skip)[0]) == n_bad
    for x in (dt, du, skip):
        gpu_ctx.free(x)


@pytest.mark.parametrize("form", [2, 0])
def test_table_decided_in_place(gpu_ctx, hq, form):
    """The headline kernel over the table with HQ_LAYOUT_IN_PLACE: committed' lands in the
    tiles' committed row, identical to the oracle; hq_table_committed_dev reads it back."""
    G, n = 100_000 + 77, 5
    inp = qref.CommitInputs(qref.spec(SEED + 4, G, n, parity_extras=True))
    want_out, want_chg, want_fb, rc = inp.run(form, False, nthreads=8)
    assert rc == 0
    dt = _table(gpu_ctx, hq, inp, form)
    chg = gpu_ctx.empty(hq.words64(G), np.uint64)
    fb = gpu_ctx.empty(hq.words64(G), np.uint64)
    com = gpu_ctx.empty(G, np.uint64)
    a = hq.CommitArgs()
    a.G, a.n_max, a.form, a.ring_len = G, n, form, 16
    a.layout = hq.HQ_LAYOUT_TILES_LEADER | hq.HQ_LAYOUT_IN_PLACE
    a.match, a.changed, a.fallback = dt.ptr, chg.ptr, fb.ptr
    gpu_ctx.commit_dev(a)
    gpu_ctx.table_committed_dev(dt, G, n, form, com)
    np.testing.assert_array_equal(gpu_ctx.download(com), want_out)
    np.testing.assert_array_equal(gpu_ctx.download(chg), want_chg)
    np.testing.assert_array_equal(gpu_ctx.download(fb), want_fb)
    v = _view(gpu_ctx, hq, dt, G, n, form)
    np.testing.assert_array_equal(v.row("committed"), want_out)
    np.testing.assert_array_equal(v.row("last_index"), inp.last_index)
    # idempotent: deciding the decided table again changes nothing
    gpu_ctx.commit_dev(a)
    gpu_ctx.table_committed_dev(dt, G, n, form, com)
    np.testing.assert_array_equal(gpu_ctx.download(com), want_out)
    for x in (dt, chg, fb, com):
        gpu_ctx.free(x)


def test_table_validation(gpu_ctx, hq):
    t = gpu_ctx.empty(4096, np.uint64)
    u = gpu_ctx.empty(64, np.uint64)
    with pytest.raises(hq.HQError):   # ring forms are not a table form
        gpu_ctx.table_ingest_match_dev(u, 4, t, 100, 3, hq.HQ_FORM_TERM_RING)
    with pytest.raises(hq.HQError):   # unknown flag
        gpu_ctx.table_ingest_match_dev(u, 4, t, 100, 3, hq.HQ_FORM_TERM_MASK, 0x80)
    with pytest.raises(hq.HQError):   # misaligned tiles
        hq._chk(hq.lib.hq_table_append_count_dev(gpu_ctx.h, hq._p(u), 4, t.ptr + 8, 100, 3, 2,
                                                 16, 0, None), "x")
    a = hq.CommitArgs()
    a.G, a.n_max, a.form, a.ring_len = 100, 3, hq.HQ_FORM_TERM_RING, 16
    a.layout = hq.HQ_LAYOUT_TILES_LEADER | hq.HQ_LAYOUT_IN_PLACE
    a.match = t.ptr
    with pytest.raises(hq.HQError):   # in place: term-start / mask only
        gpu_ctx.commit_dev(a)
    a.form = hq.HQ_FORM_TERM_MASK
    with pytest.raises(hq.HQError):   # the host-pointer entry point has no in-place form
        gpu_ctx.commit_host(a)
    gpu_ctx.free(t)
    gpu_ctx.free(u)


@pytest.mark.parametrize("depth,compact,grouped,zero_copy",
                         [(1, False, False, False), (2, False, True, False),
                          (3, False, False, False), (1, True, True, False),
                          (2, True, False, False), (2, True, True, False),
                          (2, True, True, True), (1, False, False, True),
                          (3, True, False, True)])
def test_host_fed_pipeline_matches_oracle(hq, depth, compact, grouped, zero_copy):
    """dragonboat_amd.pipeline over the leader-row tile table: host-fed steps (pinned appends +
    match deltas -> append, ingest, commit in place -> readback) over `depth` contexts, or with
    no copies at all (zero_copy: the kernels read the pinned records and write the pinned results
    over PCIe). Every
    step's read-back changed / fallback bitmaps and committed column equal the oracle's
    sequential run, whatever the pipelining and the ingest path."""
    from dragonboat_amd.pipeline import HostFedPipeline

    rng = np.random.default_rng(SEED + 30 + depth)
    G, n, R, T = 40_009, 3, 16, 7
    inp = qref.CommitInputs(qref.spec(SEED + 5, G, n))
    host = dict(match=inp.match.copy(), last=inp.last_index.copy(), mask=inp.term_mask.copy(),
                committed=inp.committed_in.copy())
    p = HostFedPipeline(0, G, n, G // 2, G, depth=depth, ring_len=R, compact=compact,
                        grouped=grouped, zero_copy=zero_copy)
    p.upload(host["match"], host["committed"], host["last"], host["mask"])
    want, slots = [], []
    for step in range(T):
        gsel = np.sort(rng.choice(G, G // 3, replace=False)).astype(np.uint64)
        app = np.stack([gsel, host["last"][gsel] + rng.integers(1, 4, len(gsel), dtype=np.uint64)],
                       axis=1).astype(np.uint64)
        counts = app[:, 1] - host["last"][gsel]           # entries appended (gsel distinct)
        qref.append(app, host["last"], host["match"][:G], host["mask"], R, G)
        g = rng.integers(0, G, G, dtype=np.uint64)
        s = rng.integers(1, n, G, dtype=np.uint64)
        if grouped:
            o = np.lexsort((s, g))
            g, s = g[o], s[o]
        lag = rng.integers(0, 6, G, dtype=np.uint64)
        idx = host["last"][g] - lag                       # lastIndex after the step's appends
        upd = np.stack([(g << np.uint64(8)) | s, idx], axis=1).astype(np.uint64)
        qref.ingest_match(upd, host["match"], G, G, n)
        out = np.zeros(G, np.uint64)
        wchg = np.zeros(hq.words64(G), np.uint64)
        wfb = np.zeros(hq.words64(G), np.uint64)
        qa = qref.commit_args(G, n, 2, R, host["match"], host["committed"], out, host["last"],
                              changed=wchg, fallback=wfb, term_mask=host["mask"])
        assert qref.commit_batch(qa, 8) == 0
        host["committed"] = out
        want.append((wchg, out, wfb))
        wire_app = hq.pack_append_counts(gsel, counts) if compact else app.reshape(-1)
        wire_upd = hq.pack_lag_updates(g, s, lag) if compact else upd.reshape(-1)
        pa = p.ctxs[step % len(p.ctxs)].pinned(wire_app.size, np.uint64)
        pa[:] = wire_app
        pu = p.ctxs[step % len(p.ctxs)].pinned(wire_upd.size, np.uint64)
        pu[:] = wire_upd
        slots.append(p.step(step, pa, len(app), pu, G))
        if step % depth == depth - 1 or step == T - 1:
            # read back the steps whose result buffers are about to be reused
            for j in range(step - step % depth, step + 1):
                chg, com, fb = p.results(slots[j])
                np.testing.assert_array_equal(chg, want[j][0])
                np.testing.assert_array_equal(com, want[j][1])
                np.testing.assert_array_equal(fb, want[j][2])
    v = hq.tile_view(p.ctxs[0].download(p.tiles), G, n, 2, hq.HQ_LAYOUT_TILES_LEADER)
    np.testing.assert_array_equal(v.match().reshape(-1), host["match"])
    np.testing.assert_array_equal(v.row("aux"), host["mask"])
    assert sum(int(np.unpackbits(w[0].view(np.uint8)).sum()) for w in want) > G
    p.close()


def test_zero_copy_pipeline_refuses_pageable_records(hq):
    """zero_copy kernels read the records over PCIe: ordinary numpy (pageable) arrays are
    refused with ValueError before any launch, pinned ones are accepted (hq_pointer_kind)."""
    from dragonboat_amd.pipeline import HostFedPipeline

    G, n = 4096, 3
    p = HostFedPipeline(0, G, n, 16, 16, depth=1, compact=True, zero_copy=True)
    try:
        c = p.ctxs[0]
        z = np.zeros(16, np.uint64)
        assert hq.pointer_kind(z) == hq.HQ_PTR_UNREGISTERED
        pz = c.pinned(16, np.uint64)
        pz[:] = 0
        assert hq.pointer_kind(pz) == hq.HQ_PTR_PINNED_HOST
        assert hq.pointer_kind(p.tiles) == hq.HQ_PTR_DEVICE
        with pytest.raises(ValueError, match="pinned"):
            p.step(0, z, 1, pz, 0)
        with pytest.raises(ValueError, match="pinned"):
            p.step(0, pz, 0, z, 1)
        p.step(0, pz, 0, pz, 0)     # no records: nothing to check, the decision still runs
        p.results(0)
    finally:
        p.close()


def test_pipeline_surfaces_fallback_groups(hq):
    """Appends that push lastIndex - committed past the mask's 16 indexes leave those groups
    undecided: the pipeline returns their fallback bits (equal to the oracle's), the caller
    decides them on the CPU (tryCommit) and writes them back, and the next step continues."""
    from dragonboat_amd.pipeline import HostFedPipeline

    rng = np.random.default_rng(SEED + 40)
    G, n, R = 20_011, 3, 16
    inp = qref.CommitInputs(qref.spec(SEED + 6, G, n))
    host = dict(match=inp.match.copy(), last=inp.last_index.copy(), mask=inp.term_mask.copy(),
                committed=inp.committed_in.copy())
    p = HostFedPipeline(0, G, n, G, G, depth=1, ring_len=R)
    p.upload(host["match"], host["committed"], host["last"], host["mask"])
    far = rng.choice(G, 500, replace=False)
    for step in range(2):
        k = np.ones(G, np.uint64)
        if step == 0:
            k[far] = 20                                    # 20 entries: beyond the 16-bit mask
        app = np.stack([np.arange(G, dtype=np.uint64), host["last"] + k], axis=1)
        qref.append(app, host["last"], host["match"][:G], host["mask"], R, G)
        g = np.arange(G, dtype=np.uint64)
        upd = np.stack([(g << np.uint64(8)) | np.uint64(1), host["last"] - np.uint64(1)], axis=1)
        qref.ingest_match(upd, host["match"], G, G, n)
        out = np.zeros(G, np.uint64)
        wchg = np.zeros(hq.words64(G), np.uint64)
        wfb = np.zeros(hq.words64(G), np.uint64)
        qa = qref.commit_args(G, n, 2, R, host["match"], host["committed"], out, host["last"],
                              changed=wchg, fallback=wfb, term_mask=host["mask"])
        assert qref.commit_batch(qa, 8) == 0
        pa = p.ctxs[0].pinned(app.size, np.uint64)
        pa[:] = app.reshape(-1)
        pu = p.ctxs[0].pinned(upd.size, np.uint64)
        pu[:] = upd.reshape(-1)
        chg, com, fb = p.results(p.step(step, pa, G, pu, G))
        np.testing.assert_array_equal(fb, wfb)
        np.testing.assert_array_equal(chg, wchg)
        np.testing.assert_array_equal(com, out)
        fbg = np.nonzero(np.unpackbits(fb.view(np.uint8), bitorder="little")[:G])[0]
        if step == 0:
            assert set(fbg) >= set(far.tolist())            # every far-behind group surfaced
        # the CPU path decides the fallback groups (the reference tryCommit with the full term
        # information: every entry appended this term is at the leader's term) and re-syncs them
        cpu = np.maximum(host["committed"][fbg], np.sort(host["match"].reshape(n, G)[:, fbg],
                                                         axis=0)[n - (n // 2 + 1)])
        out[fbg] = cpu
        p.set_committed(fbg, cpu)
        host["committed"] = out
    p.close()


@pytest.mark.parametrize("lag", [False, True])
def test_table_ingest_unique(gpu_ctx, hq, lag):
    """HQ_INGEST_UNIQUE: every (group, slot) at most once, random order, plain read-modify-writes;
    invalid records (slot 0, slot >= n, group out of range, ack above lastIndex) skipped."""
    rng = np.random.default_rng(SEED + 40 + lag)
    G, n = 60_007, 5
    form = hq.HQ_FORM_TERM_MASK
    inp = qref.CommitInputs(qref.spec(SEED + 4, G, n))
    inp.last_index[:5] = inp.match[:5] = inp.committed_in[:5] = 10
    dt = _table(gpu_ctx, hq, inp, form)
    keys = rng.permutation(G * (n + 1))[:200_000].astype(np.uint64)   # distinct (g, s), s <= n
    g, s = keys // np.uint64(n + 1), keys % np.uint64(n + 1)
    g[:7] = np.uint64(G) + np.arange(7, dtype=np.uint64)              # out of range (distinct)
    lg = rng.integers(0, 40, len(g), dtype=np.uint64)
    gi = np.minimum(g, G - 1)
    valid = (g < G) & (s >= 1) & (s < n)
    if lag:
        valid &= lg <= inp.last_index[gi]
        wire = hq.pack_lag_updates(g, s, lg)
        val = inp.last_index[gi] - np.minimum(lg, inp.last_index[gi])
    else:
        val = inp.last_index[gi] - lg
        wire = np.stack([(g << np.uint64(8)) | s, val], axis=1).astype(np.uint64).reshape(-1)
    want = inp.match.copy()
    upd = np.stack([(g[valid] << np.uint64(8)) | s[valid], val[valid]], axis=1).astype(np.uint64)
    qref.ingest_match(upd, want, G, G, n)
    du = gpu_ctx.upload(wire)
    skip = gpu_ctx.upload(np.zeros(1, np.uint64))
    f = gpu_ctx.table_ingest_lag_dev if lag else gpu_ctx.table_ingest_match_dev
    f(du, len(g), dt, G, n, form, hq.HQ_INGEST_UNIQUE, skip)
    v = _view(gpu_ctx, hq, dt, G, n, form)
    np.testing.assert_array_equal(v.match().reshape(-1), want)
    assert int(gpu_ctx.download(skip)[0]) == int((~valid).sum())
    for x in (dt, du, skip):
        gpu_ctx.free(x)


@pytest.mark.parametrize("counts", [False, True])
def test_table_append_unique(gpu_ctx, hq, counts):
    rng = np.random.default_rng(SEED + 50 + counts)
    G, n, R = 40_009, 3, 16
    form = hq.HQ_FORM_TERM_MASK
    inp = qref.CommitInputs(qref.spec(SEED + 5, G, n))
    dt = _table(gpu_ctx, hq, inp, form)
    g = rng.permutation(G).astype(np.uint64)[:30_000]             # each group at most once
    k = rng.choice(np.array([0, 1, 2, 3, 5, 15, 16, 17, 40], np.uint64), len(g))
    last, match0, mask = inp.last_index.copy(), inp.match[:G].copy(), inp.term_mask.copy()
    if counts:
        app = np.stack([g[k > 0], last[g[k > 0]] + k[k > 0]], axis=1).astype(np.uint64)
        wire = hq.pack_append_counts(g, k)
        n_bad = int((k == 0).sum())
    else:
        newl = last[g] + k
        app = np.stack([g, newl], axis=1).astype(np.uint64)
        wire = app.reshape(-1)
        n_bad = 0
    qref.append(app, last, match0, mask, R, G)
    du = gpu_ctx.upload(wire)
    skip = gpu_ctx.upload(np.zeros(1, np.uint64))
    f = gpu_ctx.table_append_count_dev if counts else gpu_ctx.table_append_dev
    f(du, len(g), dt, G, n, form, R, hq.HQ_INGEST_UNIQUE, skip)
    v = _view(gpu_ctx, hq, dt, G, n, form)
    np.testing.assert_array_equal(v.row("last_index"), last)
    np.testing.assert_array_equal(v.row("aux"), mask)
    assert int(gpu_ctx.download(skip)[0]) == n_bad
    for x in (dt, du, skip):
        gpu_ctx.free(x)
