"""Full-size parity of the per-GPU shares the bench reports, and the term
check's exact forms against each other on the reference's own term tables (item 6).

* BASELINE config 5 per GPU: 8M groups, voter count n = {3, 5, 7}[clusterID % 3] bucketed by n
  (three progressions of clusterIDs, shard.rank_bucket), decided by ONE fused launch over
  leader-row tiles (c5tl) and in the leader-implicit lag layout (c5ll), every bucket compared
  bit for bit with the oracle (oracle/qref.c) on the same generated inputs.
* Ring gather vs mask vs term-start: groups built from the logs of TestTerm,
  TestTermWithUnstableSnapshot, TestInMemGetTerm(ReturnSnapshotTerm) and the commit tables
  (logentry_etcd_test.go:566-629, inmemory_test.go:164-224, raft_etcd_test.go:1111-1160, ...),
  every (leader term, committed, quorum index) the 16-index window can hold; the u64 ring, u32
  ring, mask and (where it applies) term-start forms decide identically, and equal the oracle's
  tryCommit over the table's term() (logentry.go:143-160, 378-393)."""
import json
import os

import numpy as np
import pytest

from dragonboat_amd import shard
from oracle import qref

pytestmark = pytest.mark.gpu
SEED = 0x5EED0000 + 4          # bench.py SEED_BASE + BASELINE config index of C5
G5 = 8 << 20


def _buckets():
    per = G5 // 3
    return [(shard.MIXED_VOTERS[b], shard.rank_bucket(0, 1, b, per)) for b in range(3)]


def test_c5_share_fused_leader_tiles_full_size(gpu_ctx, hq):
    form = hq.HQ_FORM_TERM_MASK
    bufs = []
    for n, rng in _buckets():
        b = hq.alloc_commit(gpu_ctx, rng.count, n, form, 16, tiled=True,
                            tile_layout=hq.HQ_LAYOUT_TILES_LEADER)
        gpu_ctx.synth_commit_dev(hq.synth_spec(SEED, rng.count, n, cid_base=rng.cid_base,
                                               cid_stride=rng.cid_stride), b.args())
        gpu_ctx.tile_commit_dev(b.args(), b.tiles, hq.HQ_LAYOUT_TILES_LEADER)
        bufs.append((n, rng, b))
    gpu_ctx.sync()
    gpu_ctx.timing_reset()
    gpu_ctx.timing(True)
    gpu_ctx.commit_fused_dev(hq.commit_batch_array([b.tile_args() for _, _, b in bufs]))
    gpu_ctx.timing(False)
    gpu_ctx.sync()
    assert gpu_ctx.timing_read()[1] == 1                 # one launch for the three buckets
    for n, rng, b in bufs:
        inp = qref.CommitInputs(qref.spec(SEED, rng.count, n, cid_base=rng.cid_base,
                                          cid_stride=rng.cid_stride))
        want_out, want_chg, want_fb, rc = inp.run(form, False, nthreads=16)
        assert rc == 0
        np.testing.assert_array_equal(gpu_ctx.download(b.committed_out), want_out)
        np.testing.assert_array_equal(gpu_ctx.download(b.changed), want_chg)
        np.testing.assert_array_equal(gpu_ctx.download(b.fallback), want_fb)
        assert int(np.unpackbits(want_chg.view(np.uint8)).sum()) > rng.count // 2
        hq.free_commit(gpu_ctx, b)


def test_c5_share_fused_leader_implicit_lags_full_size(gpu_ctx, hq):
    form = hq.HQ_FORM_TERM_MASK
    bufs = []
    for n, rng in _buckets():
        b = hq.alloc_commit_lag(gpu_ctx, rng.count, n, form, 16)
        gpu_ctx.synth_commit_lag_dev(hq.synth_spec(SEED, rng.count, n, cid_base=rng.cid_base,
                                                   cid_stride=rng.cid_stride), b.args())
        bufs.append((n, rng, b))
    gpu_ctx.sync()
    gpu_ctx.timing_reset()
    gpu_ctx.timing(True)
    gpu_ctx.commit_lag_fused_dev(hq.lag_batch_array([b.args(True) for _, _, b in bufs]))
    gpu_ctx.timing(False)
    gpu_ctx.sync()
    assert gpu_ctx.timing_read()[1] == 1
    for n, rng, b in bufs:
        inp = qref.CommitInputs(qref.spec(SEED, rng.count, n, cid_base=rng.cid_base,
                                          cid_stride=rng.cid_stride))
        want_out, want_chg, want_fb, rc = inp.run(form, False, nthreads=16)
        fb = gpu_ctx.download(b.fallback)
        com = inp.committed_in.copy()
        hq.unpack_lags(inp.last_index, gpu_ctx.download(b.cout_lag), com, fb)
        np.testing.assert_array_equal(com, want_out)
        np.testing.assert_array_equal(gpu_ctx.download(b.changed), want_chg)
        np.testing.assert_array_equal(fb, want_fb)
        hq.free_commit(gpu_ctx, b)


# ---- ring gather == mask == term-start on the reference's term tables -------------------------
KATS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kats.json")))
TERM_TABLES = ("TestTerm", "TestTermWithUnstableSnapshot", "TestInMemGetTerm",
               "TestInMemGetTermReturnSnapshotTerm", "TestCommit",
               "TestLeaderOnlyCommitsLogFromCurrentTerm", "TestCannotCommitWithoutNewTermEntry",
               "TestCommitWithoutNewTermEntry", "TestLeaderCommitPrecedingEntries")
R = 16


def _logs():
    """The distinct logs (first_minus_1, last, index -> term) of the tables."""
    seen = {}
    for name in TERM_TABLES:
        for case in KATS.get(name, []):
            log = {int(k): int(v) for k, v in case["log"].items()}
            key = (case["first_minus_1"], case["last"], tuple(sorted(log.items())))
            seen[key] = (name, case["first_minus_1"], case["last"], log)
    return list(seen.values())


def _groups():
    """One n = 1 group per (log, leader term, committed, quorum index): match[0] = q."""
    rows = []
    for name, f1, last, log in _logs():
        terms = sorted(set(log.values()) | {max(log.values()) + 1}) if log else [1]
        for T in terms:
            if T == 0:
                continue                                   # a leader's term is >= 1
            for c in range(max(f1, last - R), last + 1):   # committed >= first - 1
                for q in range(max(0, c - 2), last + 3):
                    rows.append((name, f1, last, log, T, c, q))
    return rows


def test_term_check_forms_agree_on_reference_term_tables(gpu_ctx, hq):
    rows = _groups()
    G = len(rows)
    assert G > 5000
    match = np.zeros(G, np.uint64)
    cin, last, term = (np.zeros(G, np.uint64) for _ in range(3))
    ring = np.zeros(G * R, np.uint64)
    mask = np.zeros(G, np.uint16)
    ts = np.zeros(G, np.uint64)
    ts_ok = np.zeros(G, bool)
    want_out, want_chg = np.zeros(G, np.uint64), np.zeros(G, bool)
    for g, (name, f1, l, log, T, c, q) in enumerate(rows):
        match[g], cin[g], last[g], term[g] = q, c, l, T
        el = qref.EntryLog(f1, l, c, log)
        for i in range(l - R + 1, l + 1):
            t = el.term(i) if i >= 0 else 0
            ring[g * R + (i % R)] = t
            if t == T:
                mask[g] |= 1 << (i % R)
        # term-start applies when the last entry is at the leader's term (its no-op, raft.go:987)
        cur = [i for i in range(f1, l + 1) if log.get(i) == T]
        if log.get(l) == T and cur:
            ts[g], ts_ok[g] = min(cur), True
        rc, qq = qref.try_commit([q], [], el, T)
        assert rc >= 0 and qq == q
        want_out[g] = el.committed
        want_chg[g] = el.committed != c
    inp_args = dict(match=match, committed_in=cin, last_index=last, term=term, ring=ring,
                    term_mask=mask, term_start=ts)
    dev = {k: gpu_ctx.upload(v) for k, v in inp_args.items()}
    dev["ring32"] = gpu_ctx.upload(hq.pack_ring32(ring))
    out = gpu_ctx.empty(G, np.uint64)
    chg = gpu_ctx.empty(hq.words64(G), np.uint64)
    fb = gpu_ctx.empty(hq.words64(G), np.uint64)
    results = {}
    for form in (hq.HQ_FORM_TERM_RING, hq.HQ_FORM_TERM_RING32, hq.HQ_FORM_TERM_MASK,
                 hq.HQ_FORM_TERM_START):
        a = hq.CommitArgs()
        a.G, a.n_max, a.form, a.ring_len, a.match_stride = G, 1, form, R, G
        for k in ("match", "committed_in", "last_index", "term", "ring", "term_mask",
                  "term_start", "ring32"):
            setattr(a, k, dev[k].ptr)
        a.committed_out, a.changed, a.fallback = out.ptr, chg.ptr, fb.ptr
        gpu_ctx.commit_dev(a)
        gpu_ctx.sync()
        bits = lambda w: np.unpackbits(gpu_ctx.download(w).view(np.uint8),
                                       bitorder="little")[:G].astype(bool)
        results[form] = (gpu_ctx.download(out), bits(chg), bits(fb))
    ring_out, ring_chg, ring_fb = results[hq.HQ_FORM_TERM_RING]
    assert not ring_fb.any()          # every group is inside the 16-index window
    np.testing.assert_array_equal(ring_out, want_out)
    np.testing.assert_array_equal(ring_chg, want_chg)
    for form in (hq.HQ_FORM_TERM_RING32, hq.HQ_FORM_TERM_MASK):
        o, c, f = results[form]
        np.testing.assert_array_equal(o, ring_out)
        np.testing.assert_array_equal(c, ring_chg)
        np.testing.assert_array_equal(f, ring_fb)
    o, c, _ = results[hq.HQ_FORM_TERM_START]
    np.testing.assert_array_equal(o[ts_ok], ring_out[ts_ok])
    np.testing.assert_array_equal(c[ts_ok], ring_chg[ts_ok])
    assert ts_ok.sum() > 100 and want_chg.sum() > 100 and (~want_chg).sum() > 100
    for x in list(dev.values()) + [out, chg, fb]:
        gpu_ctx.free(x)
