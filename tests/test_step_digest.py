"""The step legs' content digests (bench.CommitMirror / bench.ready_digest against the replay's
qref_step_totals.ready_digest / commit_digest, oracle/qref.h): the numpy restatement equals the
C terms, the replay's totals do not depend on how the list is split over threads, the three
forms a worker returns its commits in reduce to the same digest, and one changed advance or
ReadyToRead record changes it. The device side of the comparison is tests/test_gpu_step_leg.py."""
import numpy as np
import pytest

import bench
from oracle import qref

U64 = (1 << 64) - 1


def _rng_u64(rng, n):
    return rng.integers(0, 1 << 63, n, dtype=np.uint64) * np.uint64(2) + \
        rng.integers(0, 2, n, dtype=np.uint64)


def test_numpy_terms_equal_c_terms():
    rng = np.random.default_rng(7)
    n = 257
    r = np.zeros(n, bench_ready_dtype())
    for f in ("cluster_id", "index", "ctx_low", "ctx_high"):
        r[f] = _rng_u64(rng, n)
    r[0] = (0, 0, 0, 0)
    r[1] = (U64, U64, U64, U64)
    want = sum(qref.lib.qref_digest_ready_term(int(x["cluster_id"]), int(x["index"]),
                                               int(x["ctx_low"]), int(x["ctx_high"]))
               for x in r) & U64
    assert bench.ready_digest(r) == want
    cids = np.sort(_rng_u64(rng, n))
    adv = rng.integers(0, 1 << 32, n, dtype=np.uint64)
    coef = bench.mix64(cids) | np.uint64(1)
    got = int((coef * adv).sum(dtype=np.uint64))
    assert got == sum(qref.lib.qref_digest_commit_term(int(c), int(a))
                      for c, a in zip(cids, adv)) & U64


def bench_ready_dtype():
    from dragonboat_amd import hipquorum as hq
    return hq.READY_DTYPE


@pytest.mark.parametrize("name", ["step", "step5"])
def test_replay_digests_do_not_depend_on_threads(hq, name):
    G = 1 << 10
    roles = bench.STEP_ROLES[name]
    g, m, _ = bench.step_groups(hq, G, 1, 1, roles)
    rows = bench.StepRows(hq, G, roles)
    batches = {nt: qref.StepBatch(g, m) for nt in (1, 3, 8)}
    try:
        for s in range(4):
            rows.set(s)
            tots = {nt: b.step(rows.groups, rows.offsets, rows.ev, nthreads=nt)
                    for nt, b in batches.items()}
            assert all(t == tots[1] for t in tots.values()), (s, tots)
            t = tots[1]
            # step 0 acks the initial last index (nothing to commit); later steps commit
            assert (t["commits"] > 0) == (s > 0) == (t["commit_digest"] != 0)
            assert (t["ready"] > 0) == (t["ready_digest"] != 0)
    finally:
        for b in batches.values():
            b.close()


def _ready(rng, cids, k):
    r = np.zeros(k, bench_ready_dtype())
    r["cluster_id"] = rng.choice(cids, k, replace=False)
    r["index"] = rng.integers(1, 1 << 40, k, dtype=np.uint64)
    r["ctx_low"] = _rng_u64(rng, k)
    r["ctx_high"] = rng.integers(0, 1000, k, dtype=np.uint64)
    return r


def test_commit_forms_reduce_to_one_digest():
    """'committed_advance', 'committed_column' and the 'commits' list of the same step give the
    same (commits, ReadyToReads, advance sum, digests); a changed advance or record differs."""
    from dragonboat_amd import hipquorum as hq
    rng = np.random.default_rng(3)
    G, W = 96, 3
    cids = np.uint64(5) + np.arange(G, dtype=np.uint64) * np.uint64(8)
    committed = rng.integers(100, 1 << 40, G, dtype=np.uint64)
    bounds = [0, 40, 41, G]
    adv = rng.integers(0, 4, G).astype(np.uint32)
    adv[:8] = 0
    ready = _ready(rng, cids, 20)

    def results(form, adv=adv, ready=ready, committed=committed):
        out = []
        for i in range(W):
            lo, hi = bounds[i], bounds[i + 1]
            a = adv[lo:hi]
            rr = ready[(ready["cluster_id"] >= cids[lo]) &
                       (ready["cluster_id"] <= cids[hi - 1])]
            r = {"ready": rr, "n_commits": int(np.count_nonzero(a))}
            if form == "advance":
                r["committed_advance"] = a
                r["commits"] = np.zeros(0, hq.COMMIT_EVENT_DTYPE)
            elif form == "column":
                r["committed_column"] = committed[lo:hi] + a.astype(np.uint64)
                r["commits"] = np.zeros(0, hq.COMMIT_EVENT_DTYPE)
            else:
                nz = np.nonzero(a)[0]
                c = np.zeros(len(nz), hq.COMMIT_EVENT_DTYPE)
                c["cluster_id"] = cids[lo + nz]
                c["committed"] = committed[lo + nz] + a[nz].astype(np.uint64)
                r = {"ready": rr, "commits": c[::-1]}      # any order
            out.append(r)
        return out

    got = {f: bench.CommitMirror(cids, committed, bounds).step(results(f))
           for f in ("advance", "column", "list")}
    assert len(set(got.values())) == 1, got
    n_c, n_r, s, rd, cd, od = got["advance"]
    assert n_c == np.count_nonzero(adv) and n_r == len(ready) and s == int(adv.sum())
    # the replay's terms, summed in any order
    want_cd = sum(qref.lib.qref_digest_commit_term(int(c), int(a))
                  for c, a in zip(cids, adv) if a) & U64
    assert cd == want_cd
    # a second step continues from the advanced mirror
    mir = bench.CommitMirror(cids, committed, bounds)
    mir.step(results("column"))
    after = committed + adv.astype(np.uint64)
    assert mir.step(results("column", adv=np.zeros(G, np.uint32), committed=after))[:3] == \
        (0, len(ready), 0)
    # sensitivity: one advance moved between two groups, one record's ctx changed
    a2 = adv.copy()
    a2[10] += 1
    a2[11] -= 1 if a2[11] else -1
    assert bench.CommitMirror(cids, committed, bounds).step(results("advance", adv=a2))[4] != cd
    r2 = ready.copy()
    r2["ctx_high"][0] ^= 1
    assert bench.CommitMirror(cids, committed, bounds).step(results("advance", ready=r2))[3] != rd
    # order: two records swapped leave the order-free digest and change the ordered one
    wk = np.searchsorted(np.array([cids[b] for b in bounds[1:-1]]), ready["cluster_id"], "right")
    i, j = next((i, j) for i in range(len(ready)) for j in range(i + 1, len(ready))
                if wk[i] == wk[j])           # two records of one worker's list
    r3 = ready.copy()
    r3[[i, j]] = r3[[j, i]]
    got3 = bench.CommitMirror(cids, committed, bounds).step(results("advance", ready=r3))
    assert got3[3] == rd and got3[5] != od


def test_ordered_digest_terms():
    """bench.ready_order_digest is the sum of (position + 1) * qref_digest_ready, positions
    continuing across workers' lists (pos0)."""
    rng = np.random.default_rng(11)
    r = np.zeros(40, bench_ready_dtype())
    for f in ("cluster_id", "index", "ctx_low", "ctx_high"):
        r[f] = _rng_u64(rng, 40)
    terms = [qref.lib.qref_digest_ready_term(int(x["cluster_id"]), int(x["index"]),
                                             int(x["ctx_low"]), int(x["ctx_high"])) for x in r]
    want = sum((k + 1) * t for k, t in enumerate(terms)) & U64
    assert bench.ready_order_digest(r) == want
    assert (bench.ready_order_digest(r[:17]) + bench.ready_order_digest(r[17:], 17)) & U64 == want
