"""Device-resident progress table against the oracle's sequential restatements:
match ingest (remote.tryUpdate), ack ingest (confirmed-set insert), leader append, and a
multi-step pipeline (append -> acks -> commit in place) that must track the oracle step by step.
The same kernels over the headline tile layout, and the host-fed pipeline: tests/test_gpu_table.py."""
import numpy as np
import pytest

from oracle import qref

SEED = 0x5EED1000


def _updates(rng, G, n_max, count, base, spread, bad_frac=0.01):
    g = rng.integers(0, G, count, dtype=np.uint64)
    s = rng.integers(0, n_max, count, dtype=np.uint64)
    bad = rng.random(count) < bad_frac
    g[bad[: count // 2].nonzero()[0]] += np.uint64(G)          # group out of range
    s[bad[count // 2:].nonzero()[0] + count // 2] = np.uint64(n_max + 3)   # slot out of range
    idx = base[g % np.uint64(G)] + rng.integers(0, spread, count, dtype=np.uint64)
    return np.stack([(g << np.uint64(8)) | s, idx], axis=1).astype(np.uint64)


@pytest.mark.gpu
def test_ingest_match_matches_sequential_try_update(gpu_ctx, hq):
    rng = np.random.default_rng(SEED)
    G, n = 100_003, 5
    base = rng.integers(1 << 20, 1 << 40, G, dtype=np.uint64)
    match = np.repeat(base[None, :], n, axis=0).reshape(-1) + rng.integers(0, 8, G * n, dtype=np.uint64)
    upd = _updates(rng, G, n, 600_000, base, 32)
    want = match.copy()
    want_skip = qref.ingest_match(upd, want, G, G, n)
    dm, du = gpu_ctx.upload(match), gpu_ctx.upload(upd.reshape(-1))
    skip = gpu_ctx.upload(np.zeros(1, np.uint64))
    gpu_ctx.ingest_match_dev(du, len(upd), dm, G, G, n, skip)
    np.testing.assert_array_equal(gpu_ctx.download(dm), want)
    assert int(gpu_ctx.download(skip)[0]) == want_skip > 0
    for x in (dm, du, skip):
        gpu_ctx.free(x)


@pytest.mark.gpu
def test_ingest_ack_is_a_set_insert(gpu_ctx, hq):
    rng = np.random.default_rng(SEED + 1)
    G, n = 50_001, 7
    ack = rng.integers(0, 2, G, dtype=np.uint8)
    gs = _updates(rng, G, n, 300_000, np.zeros(G, np.uint64), 1)[:, 0].copy()
    want = ack.copy()
    want_skip = qref.ingest_ack(gs, want, G, n)
    da, dg = gpu_ctx.upload(ack), gpu_ctx.upload(gs)
    skip = gpu_ctx.upload(np.zeros(1, np.uint64))
    gpu_ctx.ingest_ack_dev(dg, len(gs), da, G, n, skip)
    np.testing.assert_array_equal(gpu_ctx.download(da), want)
    assert int(gpu_ctx.download(skip)[0]) == want_skip
    for x in (da, dg, skip):
        gpu_ctx.free(x)


@pytest.mark.gpu
def test_append_maintains_last_self_match_and_term_mask(gpu_ctx, hq):
    rng = np.random.default_rng(SEED + 2)
    G = 40_000
    last = rng.integers(1 << 20, 1 << 30, G, dtype=np.uint64)
    m0 = last.copy()
    mask = rng.integers(0, 1 << 16, G, dtype=np.uint16)
    g = rng.integers(0, G + 10, 120_000, dtype=np.uint64)            # some out of range
    step = rng.choice(np.array([0, 1, 2, 3, 5, 15, 16, 17, 40], np.uint64), len(g))
    newl = last[np.minimum(g, G - 1)] + step
    newl[rng.random(len(g)) < 0.05] -= np.uint64(2)                    # stale appends: no-op
    upd = np.stack([g, newl], axis=1).astype(np.uint64)
    wl, wm, wk = last.copy(), m0.copy(), mask.copy()
    want_skip = qref.append(upd, wl, wm, wk, 16, G)
    dl, dm, dk, du = (gpu_ctx.upload(x) for x in (last, m0, mask, upd.reshape(-1)))
    skip = gpu_ctx.upload(np.zeros(1, np.uint64))
    gpu_ctx.append_dev(du, len(upd), dl, dm, dk, 16, G, skip)
    np.testing.assert_array_equal(gpu_ctx.download(dl), wl)
    np.testing.assert_array_equal(gpu_ctx.download(dm), wm)
    np.testing.assert_array_equal(gpu_ctx.download(dk), wk)
    assert int(gpu_ctx.download(skip)[0]) == want_skip > 0
    for x in (dl, dm, dk, du, skip):
        gpu_ctx.free(x)


@pytest.mark.gpu
def test_device_resident_leader_pipeline(gpu_ctx, hq):
    """T steps of a fleet of leaders kept on the GPU: each step appends entries, ingests the
    followers' ReplicateResp match deltas, then decides commits in place (mask form). After every
    step committed / changed / fallback equal the oracle's run of the same step on host state."""
    rng = np.random.default_rng(SEED + 3)
    G, n, R = 65_537, 5, 16
    inp = qref.CommitInputs(qref.spec(SEED + 3, G, n))
    host = dict(match=inp.match.copy(), last=inp.last_index.copy(), mask=inp.term_mask.copy(),
                committed=inp.committed_in.copy())
    d = {k: gpu_ctx.upload(v) for k, v in host.items()}
    chg = gpu_ctx.empty(hq.words64(G), np.uint64)
    fb = gpu_ctx.empty(hq.words64(G), np.uint64)
    a = hq.CommitArgs()
    a.G, a.n_max, a.form, a.ring_len, a.match_stride = G, n, hq.HQ_FORM_TERM_MASK, R, G
    a.match, a.committed_in, a.committed_out = d["match"].ptr, d["committed"].ptr, d["committed"].ptr
    a.last_index, a.term_mask = d["last"].ptr, d["mask"].ptr
    a.changed, a.fallback = chg.ptr, fb.ptr
    total_changed = 0
    for step in range(6):
        gsel = rng.integers(0, G, G // 3, dtype=np.uint64)
        app = np.stack([gsel, host["last"][gsel] + rng.integers(1, 4, len(gsel), dtype=np.uint64)],
                       axis=1).astype(np.uint64)
        qref.append(app, host["last"], host["match"][:G], host["mask"], R, G)
        da = gpu_ctx.upload(app.reshape(-1))
        gpu_ctx.append_dev(da, len(app), d["last"], d["match"], d["mask"], R, G)
        cnt = G
        g = rng.integers(0, G, cnt, dtype=np.uint64)
        s = rng.integers(1, n, cnt, dtype=np.uint64)
        idx = host["last"][g] - rng.integers(0, 6, cnt, dtype=np.uint64)
        upd = np.stack([(g << np.uint64(8)) | s, idx], axis=1).astype(np.uint64)
        qref.ingest_match(upd, host["match"], G, G, n)
        du = gpu_ctx.upload(upd.reshape(-1))
        gpu_ctx.ingest_match_dev(du, cnt, d["match"], G, G, n)
        gpu_ctx.commit_dev(a)
        gpu_ctx.sync()
        out = np.zeros(G, np.uint64)
        wchg = np.zeros(hq.words64(G), np.uint64)
        wfb = np.zeros(hq.words64(G), np.uint64)
        qa = qref.commit_args(G, n, 2, R, host["match"], host["committed"], out, host["last"],
                              changed=wchg, fallback=wfb, term_mask=host["mask"])
        assert qref.commit_batch(qa, 8) == 0
        host["committed"] = out
        np.testing.assert_array_equal(gpu_ctx.download(d["committed"]), out)
        np.testing.assert_array_equal(gpu_ctx.download(chg), wchg)
        np.testing.assert_array_equal(gpu_ctx.download(fb), wfb)
        np.testing.assert_array_equal(gpu_ctx.download(d["match"]), host["match"])
        total_changed += int(np.unpackbits(wchg.view(np.uint8)).sum())
        gpu_ctx.free(da)
        gpu_ctx.free(du)
    assert total_changed > G  # commits advanced on many groups across the steps
    for x in list(d.values()) + [chg, fb]:
        gpu_ctx.free(x)


@pytest.mark.gpu
def test_compact_deltas_equal_the_16_byte_forms(gpu_ctx, hq):
    """hq_append_count_dev / hq_ingest_lag_dev against the sequential restatements of the
    16-byte forms: repeated appends of one group in a batch add up, acks are relative to the
    post-append lastIndex, out-of-range records are skipped and counted."""
    rng = np.random.default_rng(SEED + 5)
    G, n, R = 30_011, 5, 16
    inp = qref.CommitInputs(qref.spec(SEED + 5, G, n))
    last, match, mask = inp.last_index.copy(), inp.match.copy(), inp.term_mask.copy()
    dl, dm, dk = gpu_ctx.upload(last), gpu_ctx.upload(match), gpu_ctx.upload(mask)
    skip = gpu_ctx.upload(np.zeros(1, np.uint64))
    # appends: 20 000 records over 8 000 groups (duplicates), 1..20 entries, + 2 bad records
    ga = rng.integers(0, 8000, 20_000, dtype=np.uint64)
    na = rng.integers(1, 21, 20_000, dtype=np.uint64)
    seq = []
    cur = last.copy()
    for gg, nn in zip(ga, na):                           # the sequential meaning: += n
        cur[gg] += nn
        seq.append((gg, cur[gg]))
    want_last, want_match, want_mask = last.copy(), match.copy(), mask.copy()
    qref.append(np.array(seq, np.uint64), want_last, want_match[:G], want_mask, R, G)
    wire = np.concatenate([hq.pack_append_counts(ga, na),
                           hq.pack_append_counts([G + 5, 3], [1, 0])])
    du = gpu_ctx.upload(wire)
    gpu_ctx.append_count_dev(du, len(wire), dl, dm, dk, R, G, skip)
    np.testing.assert_array_equal(gpu_ctx.download(dl), want_last)
    np.testing.assert_array_equal(gpu_ctx.download(dk), want_mask)
    np.testing.assert_array_equal(gpu_ctx.download(dm)[:G], want_match[:G])
    assert int(gpu_ctx.download(skip)[0]) == 2
    # acks: lags relative to the new lastIndex, + records beyond G / n_max / lastIndex
    g = rng.integers(0, G, 100_000, dtype=np.uint64)
    s = rng.integers(1, n, 100_000, dtype=np.uint64)
    lag = rng.integers(0, 40, 100_000, dtype=np.uint64)
    upd = np.stack([(g << np.uint64(8)) | s, want_last[g] - lag], axis=1).astype(np.uint64)
    # the two valid records among the edge cases below, in the 16-byte form
    extra = [((1 << 8) | 1, int(want_last[1]))]
    if (1 << 28) - 1 <= int(want_last[2]):
        extra.append(((2 << 8) | 1, int(want_last[2]) - ((1 << 28) - 1)))
    upd = np.concatenate([upd, np.array(extra, np.uint64)])
    qref.ingest_match(upd, want_match, G, G, n)
    wire = np.concatenate([hq.pack_lag_updates(g, s, lag),
                           hq.pack_lag_updates([G, 0, 1], [1, 7, 1], [0, 0, 0]),
                           hq.pack_lag_updates([2], [1], [(1 << 28) - 1])])
    du2 = gpu_ctx.upload(wire)
    gpu_ctx.ingest_lag_dev(du2, len(wire), dm, G, dl, G, n, skip)
    np.testing.assert_array_equal(gpu_ctx.download(dm), want_match)
    skipped = int(gpu_ctx.download(skip)[0]) - 2
    assert skipped == 2 + int((1 << 28) - 1 > int(want_last[2]))
    with pytest.raises(ValueError):
        hq.pack_lag_updates([1], [1], [1 << 28])
    for x in (dl, dm, dk, skip, du, du2):
        gpu_ctx.free(x)
