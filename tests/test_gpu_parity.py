"""Parity of the HIP kernels (through the C-ABI) with the CPU oracle. Needs an MI355X.

Bar: bit-exact — committed', changed and fallback bitmaps, confirmed bits, 2-bit vote outcomes,
has-quorum bits and the rewritten active flags must equal the oracle's for every group.
"""

import numpy as np
import pytest

from kats import KATS, commit_cases
from oracle import qref

pytestmark = pytest.mark.gpu

SEED = 0x5EED0000


# ----------------------------------------------------------------------------- helpers -------
def upload_commit(ctx, hq, inp, form, per_group_n, stride_pad=0, offset_elems=0):
    """Device SoA copies of oracle-generated inputs. stride_pad / offset_elems force the 8-byte
    (VEC=1) kernel path by making rows odd-strided or 8-byte-misaligned."""
    G, n = inp.G, inp.n_max
    stride = G + stride_pad
    dev = {}
    m = np.zeros((n, stride), np.uint64)
    m[:, :G] = inp.match.reshape(n, G)
    bufs = []

    def up(a):
        full = np.concatenate([np.zeros(offset_elems, a.dtype), a]) if offset_elems else a
        d = ctx.upload(full)
        bufs.append(d)
        return d.ptr + offset_elems * a.dtype.itemsize

    a = hq.CommitArgs()
    a.G, a.n_max, a.form, a.ring_len = G, n, form, inp.R
    a.match_stride = stride
    a.match = up(m.reshape(-1))
    a.committed_in = up(inp.committed_in)
    out = ctx.empty(G + offset_elems + 1, np.uint64)
    bufs.append(out)
    a.committed_out = out.ptr + offset_elems * 8
    a.last_index = up(inp.last_index)
    a.term_start = up(inp.term_start)
    a.term = up(inp.term)
    a.ring = up(inp.ring)
    a.ring32 = up(hq.pack_ring32(inp.ring))
    if inp.term_mask is not None:
        a.term_mask = up(inp.term_mask)
    if per_group_n:
        a.n_voting = up(inp.n_voting)
    chg = ctx.empty(hq.words64(G), np.uint64)
    fb = ctx.empty(hq.words64(G), np.uint64)
    ctx.memset(chg, 0xFF)
    ctx.memset(fb, 0xFF)
    bufs += [chg, fb]
    a.changed, a.fallback = chg.ptr, fb.ptr
    dev.update(args=a, out=out, chg=chg, fb=fb, bufs=bufs, off=offset_elems)
    return dev


def run_commit(ctx, hq, inp, form, per_group_n, **kw):
    d = upload_commit(ctx, hq, inp, form, per_group_n, **kw)
    ctx.commit_dev(d["args"])
    ctx.sync()
    out = ctx.download(d["out"])[d["off"]:d["off"] + inp.G]
    chg = ctx.download(d["chg"])
    fb = ctx.download(d["fb"])
    for b in d["bufs"]:
        ctx.free(b)
    return out, chg, fb


def check_commit(ctx, hq, inp, form, per_group_n, **kw):
    out, chg, fb = run_commit(ctx, hq, inp, form, per_group_n, **kw)
    want_out, want_chg, want_fb, rc = inp.run(form, per_group_n, nthreads=8)
    assert rc == 0
    bad = np.nonzero(out != want_out)[0]
    assert bad.size == 0, f"{bad.size} groups differ, first {bad[:5]}"
    np.testing.assert_array_equal(chg, want_chg)
    np.testing.assert_array_equal(fb, want_fb)
    return want_out, want_chg, want_fb


def popcount(words):
    return int(sum(bin(int(w)).count("1") for w in words))


# ----------------------------------------------------------------------- generators ----------
GEN_SPECS = [
    dict(n_max=3), dict(n_max=5), dict(n_max=7), dict(n_max=8, mixed_n=True),
    dict(n_max=5, parity_extras=True), dict(n_max=7, mixed_n=True, parity_extras=True),
    dict(n_max=3, cid_base=10, cid_stride=8),
]


@pytest.mark.parametrize("kw", GEN_SPECS)
def test_synth_commit_matches_cpu_generator(gpu_ctx, hq, kw):
    G = 100_003
    host = qref.CommitInputs(qref.spec(SEED + 2, G, **kw))
    spec = hq.synth_spec(SEED + 2, G, **kw)
    b = hq.alloc_commit(gpu_ctx, G, kw["n_max"], hq.HQ_FORM_TERM_RING, 16, per_group_n=True,
                        with_both_aux=True)
    gpu_ctx.synth_commit_dev(spec, b.args())
    gpu_ctx.sync()
    np.testing.assert_array_equal(gpu_ctx.download(b.match), host.match)
    np.testing.assert_array_equal(gpu_ctx.download(b.n_voting), host.n_voting)
    np.testing.assert_array_equal(gpu_ctx.download(b.committed_in), host.committed_in)
    np.testing.assert_array_equal(gpu_ctx.download(b.last_index), host.last_index)
    np.testing.assert_array_equal(gpu_ctx.download(b.term_start), host.term_start)
    np.testing.assert_array_equal(gpu_ctx.download(b.term), host.term)
    np.testing.assert_array_equal(gpu_ctx.download(b.ring), host.ring)
    np.testing.assert_array_equal(gpu_ctx.download(b.term_mask), host.term_mask)
    np.testing.assert_array_equal(gpu_ctx.download(b.ring32), hq.pack_ring32(host.ring))
    hq.free_commit(gpu_ctx, b)


@pytest.mark.parametrize("kw", [dict(n_max=7), dict(n_max=8, mixed_n=True, parity_extras=True),
                                dict(n_max=3, cid_base=3, cid_stride=4)])
def test_synth_bitmaps_matches_cpu_generator(gpu_ctx, hq, kw):
    G = 77_777
    host = qref.BitmapInputs(qref.spec(SEED + 3, G, **kw))
    arrs = [gpu_ctx.empty(G, np.uint8) for _ in range(4)]
    gpu_ctx.synth_bitmaps_dev(hq.synth_spec(SEED + 3, G, **kw), *arrs)
    gpu_ctx.sync()
    for d, h in zip(arrs, (host.ack, host.granted, host.rejected, host.n_voting)):
        np.testing.assert_array_equal(gpu_ctx.download(d), h)
        gpu_ctx.free(d)


# ----------------------------------------------------------------------- commit parity -------
FORMS = [0, 1, 2, 3]   # term-start, u64 ring gather, current-term mask, u32 ring gather


@pytest.mark.parametrize("form", FORMS)
@pytest.mark.parametrize("n_max", [1, 2, 3, 4, 5, 6, 7, 8])
def test_commit_uniform_n(gpu_ctx, hq, form, n_max):
    inp = qref.CommitInputs(qref.spec(SEED + 1, 65_537, n_max, parity_extras=True))
    _, chg, _ = check_commit(gpu_ctx, hq, inp, form, per_group_n=False)
    if n_max > 1:
        assert 0 < popcount(chg) < inp.G  # both outcomes exercised


@pytest.mark.parametrize("form", FORMS)
@pytest.mark.parametrize("n_max", [7, 8])
def test_commit_per_group_n(gpu_ctx, hq, form, n_max):
    inp = qref.CommitInputs(qref.spec(SEED + 4, 99_999, n_max, mixed_n=True, parity_extras=True))
    check_commit(gpu_ctx, hq, inp, form, per_group_n=True)


@pytest.mark.parametrize("form", FORMS)
def test_commit_vec1_paths(gpu_ctx, hq, form):
    inp = qref.CommitInputs(qref.spec(SEED + 5, 10_001, 5, parity_extras=True))
    check_commit(gpu_ctx, hq, inp, form, per_group_n=False, stride_pad=1)     # odd stride
    check_commit(gpu_ctx, hq, inp, form, per_group_n=False, offset_elems=1)   # 8B-aligned only
    inp7 = qref.CommitInputs(qref.spec(SEED + 5, 10_001, 7, mixed_n=True))
    check_commit(gpu_ctx, hq, inp7, form, per_group_n=True, offset_elems=1)


@pytest.mark.parametrize("G", [1, 2, 3, 63, 64, 65, 127, 128, 129, 130, 1000, 4097])
def test_commit_ragged_sizes(gpu_ctx, hq, G):
    for form in FORMS:
        inp = qref.CommitInputs(qref.spec(SEED + G, G, 3, parity_extras=True))
        check_commit(gpu_ctx, hq, inp, form, per_group_n=False)
        inp8 = qref.CommitInputs(qref.spec(SEED + G, G, 8, mixed_n=True))
        check_commit(gpu_ctx, hq, inp8, form, per_group_n=True)


def _kat_inputs(cases, R=16):
    """Known-answer commit cases as one ring-form batch (one group per case)."""
    G = len(cases)
    n_max = max(len(c["remotes"]) + len(c["witnesses"]) for c in cases)
    inp = qref.CommitInputs(qref.spec(1, G, n_max))   # allocate, then overwrite
    m = np.zeros((n_max, G), np.uint64)
    for g, c in enumerate(cases):
        vals = c["remotes"] + c["witnesses"]
        m[:len(vals), g] = vals
        inp.n_voting[g] = len(vals)
        inp.committed_in[g] = c["committed"]
        inp.last_index[g] = c["last"]
        inp.term[g] = c["term"]
        log = {int(k): v for k, v in c["log"].items()}
        mask = 0
        for i in range(max(0, c["last"] - R + 1), c["last"] + 1):
            inp.ring[g * R + (i % R)] = log.get(i, 0)
            mask |= int(log.get(i, 0) == c["term"]) << (i % R)
        inp.term_mask[g] = mask
        # term-start form: first index carrying the current term (entryutils.go:44-47)
        cur = [i for i, t in log.items() if t == c["term"]]
        inp.term_start[g] = min(cur) if cur else c["last"] + 1
    inp.match[:] = m.reshape(-1)
    return inp


def _term_start_representable(c):
    """term(i) == term <=> term_start <= i <= last holds for this log (the invariant the
    term-start form relies on); some unit-test logs carry entries above the node's term."""
    log = {int(k): v for k, v in c["log"].items()}
    cur = sorted(i for i, t in log.items() if t == c["term"])
    return not cur or cur == list(range(cur[0], c["last"] + 1))


def test_commit_reference_kats_on_gpu(gpu_ctx, hq):
    cases = commit_cases()
    inp = _kat_inputs(cases)
    want = np.array([c["want_committed"] for c in cases], np.uint64)
    for form in (1, 2, 3):   # ring gathers and current-term mask: every case representable
        out, chg, fb = run_commit(gpu_ctx, hq, inp, form, per_group_n=True)
        assert popcount(fb) == 0
        np.testing.assert_array_equal(out, want)
    ok = np.array([_term_start_representable(c) for c in cases])
    assert ok.sum() >= len(cases) - 3
    out, chg, fb = run_commit(gpu_ctx, hq, inp, 0, per_group_n=True)
    np.testing.assert_array_equal(out[ok], want[ok])


def test_commit_contract_fallbacks(gpu_ctx, hq):
    G, R = 8, 16
    inp = qref.CommitInputs(qref.spec(SEED, G, 3))
    last = int(inp.last_index[0])
    inp.last_index[:] = last
    inp.term[:] = 7
    inp.committed_in[:] = last - 2
    inp.term_start[:] = last - 3
    inp.ring[:] = 7
    inp.match[:] = last
    inp.n_voting[:] = 3
    inp.term[1] = 0                        # term 0: the reference would panic in commitTo
    inp.committed_in[2] = last + 5         # committed beyond last
    inp.committed_in[3] = last - R - 1     # ring window too short
    inp.n_voting[4] = 0                    # no voting member
    inp.n_voting[5] = 9                    # more than n_max
    inp.committed_in[6] = last - R         # exactly R behind: still exact
    inp.term_mask[:] = 0xFFFF
    out, chg, fb = run_commit(gpu_ctx, hq, inp, 1, per_group_n=True)
    assert int(fb[0]) == 0b111110
    assert int(chg[0]) == 0b11000001
    np.testing.assert_array_equal(out[1:6], inp.committed_in[1:6])
    want_out, want_chg, want_fb, rc = inp.run(1, True)
    np.testing.assert_array_equal(out, want_out)
    np.testing.assert_array_equal(fb, want_fb)
    # mask form: no term column, so group 1 (term 0) is decided normally
    out, chg, fb = run_commit(gpu_ctx, hq, inp, 2, per_group_n=True)
    assert int(fb[0]) == 0b111100
    assert int(chg[0]) == 0b11000011
    want_out, want_chg, want_fb, rc = inp.run(2, True)
    np.testing.assert_array_equal(out, want_out)
    np.testing.assert_array_equal(chg, want_chg)
    np.testing.assert_array_equal(fb, want_fb)
    # u32 ring: the ring form's fallbacks, plus a term that does not fit below 0xFFFFFFFF
    inp.term[7] = 1 << 32
    out, chg, fb = run_commit(gpu_ctx, hq, inp, 3, per_group_n=True)
    assert int(fb[0]) == 0b10111110
    want_out, want_chg, want_fb, rc = inp.run(3, True)
    np.testing.assert_array_equal(out, want_out)
    np.testing.assert_array_equal(chg, want_chg)
    np.testing.assert_array_equal(fb, want_fb)


def test_commit_ring32_wide_terms(gpu_ctx, hq):
    """Terms around 2^32: the u32 ring decides exactly what the u64 ring decides (entries at or
    above 0xFFFFFFFF saturate and never equal a decidable term; larger terms fall back)."""
    G, R = 4096, 16
    inp = qref.CommitInputs(qref.spec(SEED + 11, G, 5))
    rng = np.random.default_rng(5)
    base = np.array([0xFFFFFFFE, 0xFFFFFFFF, 0x100000000, 0x1FFFFFFFE, 0xFFFFFFF0, 3],
                    np.uint64)
    inp.term[:] = base[rng.integers(0, len(base), G)]
    # ring entries: the term itself, its low 32 bits with a high bit set (equal after
    # truncation, not after saturation), or an older term
    pick = rng.integers(0, 3, G * R)
    t = np.repeat(inp.term, R)
    inp.ring[:] = np.where(pick == 0, t, np.where(pick == 1, (t & np.uint64(0xFFFFFFFF)) |
                                                   np.uint64(1 << 33), t // np.uint64(2)))
    out, chg, fb = run_commit(gpu_ctx, hq, inp, 3, per_group_n=False)
    want_out, want_chg, want_fb, rc = inp.run(3, False)
    assert rc == 0
    np.testing.assert_array_equal(out, want_out)
    np.testing.assert_array_equal(chg, want_chg)
    np.testing.assert_array_equal(fb, want_fb)
    assert 0 < popcount(chg) and 0 < popcount(fb) < G
    # groups the u32 form decides are decided as the u64 ring form decides them
    out1, chg1, _ = run_commit(gpu_ctx, hq, inp, 1, per_group_n=False)
    dec = inp.term < np.uint64(0xFFFFFFFF)
    np.testing.assert_array_equal(out[dec], out1[dec])


def _fused_buckets(ctx, hq, form, sizes):
    """Device batches of several voter counts (a step worker's buckets) with their oracle
    answers."""
    bs, want = [], []
    for k, (n, G) in enumerate(sizes):
        inp = qref.CommitInputs(qref.spec(SEED + 40 + k, G, n, parity_extras=True))
        # even row stride: 16-byte loads of every row (what a fused launch needs)
        d = upload_commit(ctx, hq, inp, form, per_group_n=False, stride_pad=G % 2)
        bs.append(d)
        want.append(inp.run(form, False, nthreads=8)[:3])
    return bs, want


@pytest.mark.parametrize("form", FORMS)
@pytest.mark.parametrize("sizes", [[(3, 100_001), (5, 99_999), (7, 100_003)],
                                   [(3, 1), (5, 64), (7, 65), (1, 129), (8, 3000)],
                                   [(5, 1 << 20), (3, 2049)]])
def test_commit_fused_buckets(gpu_ctx, hq, form, sizes):
    """One launch over several voter-count buckets equals the oracle on each bucket."""
    bs, want = _fused_buckets(gpu_ctx, hq, form, sizes)
    gpu_ctx.timing_reset()
    gpu_ctx.timing(True)
    gpu_ctx.commit_fused_dev(hq.commit_batch_array([d["args"] for d in bs]))
    gpu_ctx.sync()
    gpu_ctx.timing(False)
    assert gpu_ctx.timing_read()[1] == 1          # one launch
    for d, (wo, wc, wf) in zip(bs, want):
        np.testing.assert_array_equal(gpu_ctx.download(d["out"])[:len(wo)], wo)
        np.testing.assert_array_equal(gpu_ctx.download(d["chg"]), wc)
        np.testing.assert_array_equal(gpu_ctx.download(d["fb"]), wf)
        for b in d["bufs"]:
            gpu_ctx.free(b)


def test_commit_fused_unfusable_batches(gpu_ctx, hq):
    """Batches that cannot share a launch (per-group n, more than 32, one batch) are launched
    separately with the same results; 32 still share one launch."""
    sizes = [(3, 5000), (5, 4000), (7, 3000)] * 11           # 33 batches: one too many
    bs, want = _fused_buckets(gpu_ctx, hq, 2, sizes)
    gpu_ctx.timing_reset()
    gpu_ctx.timing(True)
    gpu_ctx.commit_fused_dev(hq.commit_batch_array([d["args"] for d in bs]))
    gpu_ctx.sync()
    gpu_ctx.timing(False)
    assert gpu_ctx.timing_read()[1] == 33                     # a launch per batch
    for d, (wo, wc, wf) in zip(bs, want):
        np.testing.assert_array_equal(gpu_ctx.download(d["out"])[:len(wo)], wo)
        np.testing.assert_array_equal(gpu_ctx.download(d["chg"]), wc)
    for d in bs:                                              # 32 of them: one launch
        for x in (d["out"], d["chg"]):
            gpu_ctx.memset(x, 0xA5)
    gpu_ctx.timing_reset()
    gpu_ctx.timing(True)
    gpu_ctx.commit_fused_dev(hq.commit_batch_array([d["args"] for d in bs[:32]]))
    gpu_ctx.sync()
    gpu_ctx.timing(False)
    assert gpu_ctx.timing_read()[1] == 1
    for d, (wo, wc, wf) in zip(bs[:32], want):
        np.testing.assert_array_equal(gpu_ctx.download(d["out"])[:len(wo)], wo)
        np.testing.assert_array_equal(gpu_ctx.download(d["chg"]), wc)
    for d in bs:
        for b in d["bufs"]:
            gpu_ctx.free(b)
    inp = qref.CommitInputs(qref.spec(SEED + 50, 7777, 7, mixed_n=True, parity_extras=True))
    d0 = upload_commit(gpu_ctx, hq, inp, 1, per_group_n=True)
    d1 = upload_commit(gpu_ctx, hq, inp, 1, per_group_n=False)
    gpu_ctx.commit_fused_dev(hq.commit_batch_array([d0["args"], d1["args"]]))
    gpu_ctx.sync()
    for d, pern in ((d0, True), (d1, False)):
        wo, wc, wf, _ = inp.run(1, pern)
        np.testing.assert_array_equal(gpu_ctx.download(d["out"])[:len(wo)], wo)
        np.testing.assert_array_equal(gpu_ctx.download(d["fb"]), wf)
        for b in d["bufs"]:
            gpu_ctx.free(b)


def test_commit_host_entry_point(gpu_ctx, hq):
    inp = qref.CommitInputs(qref.spec(SEED + 9, 30_001, 5, parity_extras=True))
    ring32 = hq.pack_ring32(inp.ring)
    for form in FORMS:
        out = np.zeros(inp.G, np.uint64)
        chg = np.zeros(hq.words64(inp.G), np.uint64)
        fb = np.zeros(hq.words64(inp.G), np.uint64)
        a = hq.CommitArgs()
        a.G, a.n_max, a.form, a.ring_len, a.match_stride = inp.G, 5, form, 16, inp.G
        a.match, a.committed_in, a.committed_out = (inp.match.ctypes.data,
                                                    inp.committed_in.ctypes.data, out.ctypes.data)
        a.last_index, a.term_start = inp.last_index.ctypes.data, inp.term_start.ctypes.data
        a.term, a.ring = inp.term.ctypes.data, inp.ring.ctypes.data
        a.term_mask = inp.term_mask.ctypes.data
        a.ring32 = ring32.ctypes.data
        a.changed, a.fallback = chg.ctypes.data, fb.ctypes.data
        gpu_ctx.commit_host(a)
        want_out, want_chg, want_fb, _ = inp.run(form, False)
        np.testing.assert_array_equal(out, want_out)
        np.testing.assert_array_equal(chg, want_chg)
        np.testing.assert_array_equal(fb, want_fb)


def test_commit_inplace_idempotent(gpu_ctx, hq):
    """Running the decision again on its own output changes nothing (q <= committed')."""
    G = 200_000
    b = hq.alloc_commit(gpu_ctx, G, 5, hq.HQ_FORM_TERM_RING, 16)
    gpu_ctx.synth_commit_dev(hq.synth_spec(SEED + 7, G, 5), b.args())
    a = b.args()
    a.committed_out = a.committed_in          # in place
    gpu_ctx.commit_dev(a)
    first = popcount(gpu_ctx.download(b.changed))
    gpu_ctx.commit_dev(a)
    assert first > G // 4
    assert popcount(gpu_ctx.download(b.changed)) == 0
    assert popcount(gpu_ctx.download(b.fallback)) == 0
    hq.free_commit(gpu_ctx, b)


@pytest.mark.parametrize("n_max,form", [(3, 0), (5, 1), (5, 2), (5, 3)])
def test_commit_full_size_configs(gpu_ctx, hq, n_max, form):
    """BASELINE configs 2 and 3 at full size (1M groups): device-generated inputs, oracle on the
    CPU generator's copy; the three term forms agree on the same data."""
    G = 1 << 20
    b = hq.alloc_commit(gpu_ctx, G, n_max, form, 16, with_both_aux=True)
    gpu_ctx.synth_commit_dev(hq.synth_spec(SEED + n_max, G, n_max), b.args())
    gpu_ctx.commit_dev(b.args())
    gpu_ctx.sync()
    out, chg = gpu_ctx.download(b.committed_out), gpu_ctx.download(b.changed)
    inp = qref.CommitInputs(qref.spec(SEED + n_max, G, n_max))
    want_out, want_chg, want_fb, rc = inp.run(form, False, nthreads=16)
    np.testing.assert_array_equal(out, want_out)
    np.testing.assert_array_equal(chg, want_chg)
    assert popcount(gpu_ctx.download(b.fallback)) == 0
    extra_out = gpu_ctx.empty(G, np.uint64)
    for other_form in set(FORMS) - {form}:
        other = b.args()
        other.form = other_form
        other.committed_out = extra_out.ptr
        gpu_ctx.commit_dev(other)
        gpu_ctx.sync()
        np.testing.assert_array_equal(gpu_ctx.download(b.changed), want_chg)
        np.testing.assert_array_equal(gpu_ctx.download(extra_out), want_out)
    gpu_ctx.free(extra_out)
    hq.free_commit(gpu_ctx, b)


# ----------------------------------------------------------------------- bitmaps --------------
def _dev_bits(ctx, hq, G, *arrays):
    return [ctx.upload(a) if a is not None else None for a in arrays]


def test_vote_readindex_exhaustive(gpu_ctx, hq):
    """Every (granted, rejected) byte pair and every ack byte for n = 0..9 (0 and 9 invalid)."""
    g, r = np.meshgrid(np.arange(256, dtype=np.uint8), np.arange(256, dtype=np.uint8))
    g, r = g.reshape(-1), r.reshape(-1)
    nv = np.repeat(np.arange(10, dtype=np.uint8), g.size)
    g, r = np.tile(g, 10), np.tile(r, 10)
    ack = r.copy()
    G = g.size
    dg, dr, da, dn = _dev_bits(gpu_ctx, hq, G, g, r, ack, nv)
    conf = gpu_ctx.empty(hq.words64(G), np.uint64)
    outc = gpu_ctx.empty(hq.words32(G), np.uint64)
    fb = gpu_ctx.empty(hq.words64(G), np.uint64)
    want_out, want_fb = qref.vote_batch(g, r, nv, 0, nthreads=8)
    want_conf, want_fb2 = qref.readindex_batch(ack, nv, 0, nthreads=8)
    gpu_ctx.vote_dev(G, dg, dr, dn, 0, outc, fb)
    np.testing.assert_array_equal(gpu_ctx.download(outc), want_out)
    np.testing.assert_array_equal(gpu_ctx.download(fb), want_fb)
    gpu_ctx.readindex_dev(G, da, dn, 0, conf, fb)
    np.testing.assert_array_equal(gpu_ctx.download(conf), want_conf)
    np.testing.assert_array_equal(gpu_ctx.download(fb), want_fb2)
    gpu_ctx.memset(conf, 0xAB)
    gpu_ctx.memset(outc, 0xCD)
    gpu_ctx.readindex_vote_dev(G, da, dg, dr, dn, 0, conf, outc, fb)
    np.testing.assert_array_equal(gpu_ctx.download(conf), want_conf)
    np.testing.assert_array_equal(gpu_ctx.download(outc), want_out)
    for x in (dg, dr, da, dn, conf, outc, fb):
        gpu_ctx.free(x)


def test_check_quorum_exhaustive(gpu_ctx, hq):
    act = np.tile(np.arange(256, dtype=np.uint8), 10 * 8)
    nv = np.repeat(np.arange(10, dtype=np.uint8), 256 * 8)
    G = act.size
    for self_slot in (0, 3, 7):
        da, dn = _dev_bits(gpu_ctx, hq, G, act, nv)
        hqb = gpu_ctx.empty(hq.words64(G), np.uint64)
        fb = gpu_ctx.empty(hq.words64(G), np.uint64)
        gpu_ctx.check_quorum_dev(G, da, dn, 0, self_slot, hqb, fb)
        want_hq, want_fb, want_act = qref.check_quorum_batch(act, nv, 0, self_slot)
        np.testing.assert_array_equal(gpu_ctx.download(hqb), want_hq)
        np.testing.assert_array_equal(gpu_ctx.download(fb), want_fb)
        np.testing.assert_array_equal(gpu_ctx.download(da), want_act)
        for x in (da, dn, hqb, fb):
            gpu_ctx.free(x)


@pytest.mark.parametrize("G", [1, 15, 16, 17, 31, 33, 63, 64, 65, 1023, 1025, 5000])
def test_bitmaps_ragged_sizes(gpu_ctx, hq, G):
    inp = qref.BitmapInputs(qref.spec(SEED + G, G, 8, mixed_n=True, parity_extras=True))
    da, dg, dr, dn = _dev_bits(gpu_ctx, hq, G, inp.ack, inp.granted, inp.rejected, inp.n_voting)
    conf = gpu_ctx.empty(hq.words64(G), np.uint64)
    outc = gpu_ctx.empty(hq.words32(G), np.uint64)
    gpu_ctx.memset(conf, 0xFF)
    gpu_ctx.memset(outc, 0xFF)
    gpu_ctx.readindex_vote_dev(G, da, dg, dr, dn, 0, conf, outc)
    want_conf, _ = qref.readindex_batch(inp.ack, inp.n_voting, 0)
    want_out, _ = qref.vote_batch(inp.granted, inp.rejected, inp.n_voting, 0)
    np.testing.assert_array_equal(gpu_ctx.download(conf), want_conf)
    np.testing.assert_array_equal(gpu_ctx.download(outc), want_out)
    for x in (da, dg, dr, dn, conf, outc):
        gpu_ctx.free(x)


def test_bitmaps_host_entry_points(gpu_ctx, hq):
    G = 12_345
    inp = qref.BitmapInputs(qref.spec(SEED + 11, G, 7, parity_extras=True))
    conf = np.zeros(hq.words64(G), np.uint64)
    outc = np.zeros(hq.words32(G), np.uint64)
    gpu_ctx.readindex_host(G, inp.ack, None, 7, conf)
    gpu_ctx.vote_host(G, inp.granted, inp.rejected, None, 7, outc)
    np.testing.assert_array_equal(conf, qref.readindex_batch(inp.ack, None, 7)[0])
    np.testing.assert_array_equal(outc, qref.vote_batch(inp.granted, inp.rejected, None, 7)[0])


def test_bitmaps_full_size_config4(gpu_ctx, hq):
    """BASELINE config 4 at full size: 16M groups x 7 voters, fused ReadIndex + vote."""
    G = 16 << 20
    arrs = [gpu_ctx.empty(G, np.uint8) for _ in range(4)]
    da, dg, dr, dn = arrs
    gpu_ctx.synth_bitmaps_dev(hq.synth_spec(SEED + 3, G, 7), da, dg, dr, dn)
    conf = gpu_ctx.empty(hq.words64(G), np.uint64)
    outc = gpu_ctx.empty(hq.words32(G), np.uint64)
    gpu_ctx.readindex_vote_dev(G, da, dg, dr, dn, 0, conf, outc)
    inp = qref.BitmapInputs(qref.spec(SEED + 3, G, 7))
    want_conf, _ = qref.readindex_batch(inp.ack, inp.n_voting, 0, nthreads=16)
    want_out, _ = qref.vote_batch(inp.granted, inp.rejected, inp.n_voting, 0, nthreads=16)
    np.testing.assert_array_equal(gpu_ctx.download(conf), want_conf)
    np.testing.assert_array_equal(gpu_ctx.download(outc), want_out)
    for x in arrs + [conf, outc]:
        gpu_ctx.free(x)


def test_timing_counts_launches(gpu_ctx, hq):
    G = 1 << 16
    b = hq.alloc_commit(gpu_ctx, G, 3, hq.HQ_FORM_TERM_START, 16)
    gpu_ctx.synth_commit_dev(hq.synth_spec(SEED, G, 3), b.args())
    gpu_ctx.timing_reset()
    gpu_ctx.timing(True)
    for _ in range(5):
        gpu_ctx.commit_dev(b.args())
    ms, n = gpu_ctx.timing_read()
    gpu_ctx.timing(False)
    assert n == 5 and ms > 0
    hq.free_commit(gpu_ctx, b)


# ----------------------------------------------------------------------- lag layout ----------
I32_MIN, I32_MAX = -(1 << 31), (1 << 31) - 1


def run_commit_lag(ctx, hq, inp, form, per_group_n, stride_pad=0, offset_elems=0,
                   lags=None, lead=False):
    """The oracle-generated u64 batch packed into lags on the host (hq_pack_lags), decided by
    hq_commit_lag_dev; returns (committed' unpacked, changed, fallback)."""
    G, n = inp.G, inp.n_max
    flags = hq.HQ_LAG_LEADER_IMPLICIT if lead else 0
    lag, cin, aux = lags if lags is not None else hq.pack_lags(
        G, n, form, inp.R, inp.match, inp.committed_in, inp.last_index, inp.term_start,
        inp.term_mask, flags=flags)
    nr = n - 1 if lead else n   # lag rows (lead: slots 1..n-1)
    stride = G + stride_pad
    rows = np.zeros((max(nr, 1), stride), np.int32)
    rows[:nr, :G] = lag.reshape(nr, G)
    bufs = []

    def up(a):
        full = np.concatenate([np.zeros(offset_elems, a.dtype), a]) if offset_elems else a
        d = ctx.upload(full)
        bufs.append(d)
        return d.ptr + offset_elems * a.dtype.itemsize

    out = ctx.empty(G + offset_elems + 4, np.int32)
    chg = ctx.empty(hq.words64(G), np.uint64)
    fb = ctx.empty(hq.words64(G), np.uint64)
    ctx.memset(chg, 0xFF)
    ctx.memset(fb, 0xFF)
    bufs += [out, chg, fb]
    a = hq.lag_args(G, n, form, inp.R, up(rows.reshape(-1)), up(cin),
                    out.ptr + offset_elems * 4,
                    up(aux) if form == 0 else None, up(aux) if form == 2 else None,
                    up(inp.n_voting) if per_group_n else None, chg, fb, lag_stride=stride)
    a.flags = flags
    ctx.commit_lag_dev(a)
    ctx.sync()
    cout = ctx.download(out)[offset_elems:offset_elems + G]
    c, f = ctx.download(chg), ctx.download(fb)
    for b in bufs:
        ctx.free(b)
    com = inp.committed_in.copy()
    hq.unpack_lags(inp.last_index, cout, com, f)
    return com, c, f


def check_commit_lag(ctx, hq, inp, form, per_group_n, **kw):
    com, chg, fb = run_commit_lag(ctx, hq, inp, form, per_group_n, **kw)
    want_out, want_chg, want_fb, rc = inp.run(form, per_group_n, nthreads=8)
    assert rc == 0
    bad = np.nonzero(com != want_out)[0]
    assert bad.size == 0, f"{bad.size} groups differ, first {bad[:5]}"
    np.testing.assert_array_equal(chg, want_chg)
    np.testing.assert_array_equal(fb, want_fb)
    return chg


@pytest.mark.parametrize("form", [0, 2])
@pytest.mark.parametrize("n_max", [1, 2, 3, 4, 5, 6, 7, 8])
def test_commit_lag_uniform_n(gpu_ctx, hq, form, n_max):
    inp = qref.CommitInputs(qref.spec(SEED + 21, 65_537, n_max, parity_extras=True))
    chg = check_commit_lag(gpu_ctx, hq, inp, form, per_group_n=False)
    if n_max > 1:
        assert 0 < popcount(chg) < inp.G


@pytest.mark.parametrize("form", [0, 2])
@pytest.mark.parametrize("n_max", [7, 8])
def test_commit_lag_per_group_n(gpu_ctx, hq, form, n_max):
    inp = qref.CommitInputs(qref.spec(SEED + 22, 99_999, n_max, mixed_n=True, parity_extras=True))
    check_commit_lag(gpu_ctx, hq, inp, form, per_group_n=True)


@pytest.mark.parametrize("form", [0, 2])
@pytest.mark.parametrize("n_max", [1, 2, 3, 4, 5, 6, 7, 8])
def test_commit_lag_leader_implicit(gpu_ctx, hq, form, n_max):
    """HQ_LAG_LEADER_IMPLICIT: rows from slot 1, slot 0's lag 0 (the leader's own match is its
    lastIndex, raft.go:918): the same decisions, vector and scalar paths, per-group n."""
    inp = qref.CommitInputs(qref.spec(SEED + 26 + n_max, 65_537, n_max, parity_extras=True))
    check_commit_lag(gpu_ctx, hq, inp, form, per_group_n=False, lead=True)
    check_commit_lag(gpu_ctx, hq, inp, form, per_group_n=False, lead=True, offset_elems=1)
    for G in (1, 5, 65, 257):
        inp = qref.CommitInputs(qref.spec(SEED + G + n_max, G, n_max, parity_extras=True))
        check_commit_lag(gpu_ctx, hq, inp, form, per_group_n=False, lead=True)
    if n_max >= 7:
        inp = qref.CommitInputs(qref.spec(SEED + 27, 30_001, n_max, mixed_n=True,
                                          parity_extras=True))
        check_commit_lag(gpu_ctx, hq, inp, form, per_group_n=True, lead=True)


@pytest.mark.parametrize("form", [0, 2])
def test_commit_lag_vec1_and_ragged(gpu_ctx, hq, form):
    inp = qref.CommitInputs(qref.spec(SEED + 23, 10_001, 5, parity_extras=True))
    check_commit_lag(gpu_ctx, hq, inp, form, per_group_n=False, stride_pad=1)
    check_commit_lag(gpu_ctx, hq, inp, form, per_group_n=False, offset_elems=1)
    for G in (1, 2, 3, 4, 5, 63, 64, 65, 255, 256, 257, 1001):
        inp = qref.CommitInputs(qref.spec(SEED + G, G, 3, parity_extras=True))
        check_commit_lag(gpu_ctx, hq, inp, form, per_group_n=False)
        inp8 = qref.CommitInputs(qref.spec(SEED + G, G, 8, mixed_n=True))
        check_commit_lag(gpu_ctx, hq, inp8, form, per_group_n=True)


def test_commit_lag_reference_kats(gpu_ctx, hq):
    cases = commit_cases()
    inp = _kat_inputs(cases)
    want = np.array([c["want_committed"] for c in cases], np.uint64)
    com, chg, fb = run_commit_lag(gpu_ctx, hq, inp, 2, per_group_n=True)
    assert popcount(fb) == 0
    np.testing.assert_array_equal(com, want)
    ok = np.array([_term_start_representable(c) for c in cases])
    com, chg, fb = run_commit_lag(gpu_ctx, hq, inp, 0, per_group_n=True)
    np.testing.assert_array_equal(com[ok], want[ok])


def test_commit_lag_saturation_is_exact(gpu_ctx, hq):
    """Indexes 2^31 and more away from lastIndex: saturated lags never change a decision; only
    an unrepresentable committed falls back (term-start form)."""
    G, n = 4096, 5
    rng = np.random.default_rng(9)
    inp = qref.CommitInputs(qref.spec(SEED + 24, G, n))
    last = inp.last_index
    m = inp.match.reshape(n, G).copy()
    lastb = np.broadcast_to(last, (n, G))
    far = rng.random((n, G)) < 0.25
    m[far] = lastb[far] - np.uint64(1 << 35)                            # far behind
    ahead = rng.random((n, G)) < 0.05
    m[ahead] = lastb[ahead] + np.uint64((1 << 33) + 5)                  # far above last
    inp.match[:] = m.reshape(-1)
    cfar = rng.random(G) < 0.05
    inp.committed_in[cfar] = last[cfar] - np.uint64((1 << 31) + 7)       # not representable
    tsfar = rng.random(G) < 0.1
    inp.term_start[tsfar] = last[tsfar] - np.uint64(1 << 34)            # far below: any q >= ts
    com, chg, fb = run_commit_lag(gpu_ctx, hq, inp, 0, per_group_n=False)
    want_out, want_chg, _, rc = inp.run(0, False)
    fbits = np.unpackbits(fb.view(np.uint8), bitorder="little")[:G].astype(bool)
    np.testing.assert_array_equal(fbits, cfar)
    np.testing.assert_array_equal(com[~cfar], want_out[~cfar])
    cbits = np.unpackbits(chg.view(np.uint8), bitorder="little")[:G].astype(bool)
    wbits = np.unpackbits(want_chg.view(np.uint8), bitorder="little")[:G].astype(bool)
    np.testing.assert_array_equal(cbits[~cfar], wbits[~cfar])
    assert cbits.sum() > G // 10


@pytest.mark.parametrize("kw", [dict(n_max=3), dict(n_max=5, parity_extras=True),
                                dict(n_max=8, mixed_n=True, parity_extras=True)])
def test_synth_commit_lag_matches_host_packer(gpu_ctx, hq, kw):
    G = 50_003
    host = qref.CommitInputs(qref.spec(SEED + 25, G, **kw))
    spec = hq.synth_spec(SEED + 25, G, **kw)
    for form in (0, 2):
        lag, cin, aux = hq.pack_lags(G, kw["n_max"], form, 16, host.match, host.committed_in,
                                     host.last_index, host.term_start, host.term_mask)
        if kw.get("mixed_n"):   # the device generator writes 0 into slots >= n
            rows = lag.reshape(kw["n_max"], G)
            for s in range(kw["n_max"]):
                rows[s][host.n_voting <= s] = 0
        b = hq.alloc_commit_lag(gpu_ctx, G, kw["n_max"], form, 16, with_last=True)
        gpu_ctx.synth_commit_lag_dev(spec, b.args(), b.last_index)
        gpu_ctx.sync()
        dl = gpu_ctx.download(b.lag).reshape(kw["n_max"], b.stride)[:, :G].reshape(-1)
        np.testing.assert_array_equal(dl, lag)
        np.testing.assert_array_equal(gpu_ctx.download(b.cin_lag), cin)
        np.testing.assert_array_equal(gpu_ctx.download(b.aux), aux)
        np.testing.assert_array_equal(gpu_ctx.download(b.last_index), host.last_index)
        hq.free_commit(gpu_ctx, b)


@pytest.mark.parametrize("n_max,form", [(3, 0), (5, 2)])
def test_commit_lag_full_size(gpu_ctx, hq, n_max, form):
    """BASELINE configs 2 and 3 at full size in the lag layout: device-generated, decided,
    unpacked, equal to the oracle's u64 decision on the CPU generator's copy."""
    G = 1 << 20
    b = hq.alloc_commit_lag(gpu_ctx, G, n_max, form, 16, with_last=True)
    gpu_ctx.synth_commit_lag_dev(hq.synth_spec(SEED + n_max, G, n_max), b.args(), b.last_index)
    gpu_ctx.commit_lag_dev(b.args())
    gpu_ctx.sync()
    inp = qref.CommitInputs(qref.spec(SEED + n_max, G, n_max))
    want_out, want_chg, want_fb, rc = inp.run(form, False, nthreads=16)
    com = inp.committed_in.copy()
    hq.unpack_lags(inp.last_index, gpu_ctx.download(b.cout_lag), com,
                   gpu_ctx.download(b.fallback))
    np.testing.assert_array_equal(com, want_out)
    np.testing.assert_array_equal(gpu_ctx.download(b.changed), want_chg)
    assert popcount(gpu_ctx.download(b.fallback)) == 0
    hq.free_commit(gpu_ctx, b)


@pytest.mark.parametrize("lead", [False, True])
@pytest.mark.parametrize("form", [0, 2])
@pytest.mark.parametrize("sizes", [[(3, 100_001), (5, 99_999), (7, 100_003)],
                                   [(3, 1), (5, 64), (7, 65), (1, 129), (8, 3000)]])
def test_commit_lag_fused_buckets(gpu_ctx, hq, form, sizes, lead):
    """One launch over several voter-count buckets in the lag layout (device generator) equals
    the oracle's u64 decision on each bucket."""
    bufs, want = [], []
    for k, (n, G) in enumerate(sizes):
        spec = qref.spec(SEED + 60 + k, G, n, parity_extras=True)
        b = hq.alloc_commit_lag(gpu_ctx, G, n, form, 16, with_last=True)
        gpu_ctx.synth_commit_lag_dev(hq.synth_spec(SEED + 60 + k, G, n, parity_extras=True),
                                     b.args(), b.last_index)
        inp = qref.CommitInputs(spec)
        bufs.append((b, inp))
        want.append(inp.run(form, False, nthreads=8)[:3])
    gpu_ctx.sync()
    gpu_ctx.timing_reset()
    gpu_ctx.timing(True)
    gpu_ctx.commit_lag_fused_dev(hq.lag_batch_array([b.args(lead) for b, _ in bufs]))
    gpu_ctx.sync()
    gpu_ctx.timing(False)
    assert gpu_ctx.timing_read()[1] == 1
    for (b, inp), (wo, wc, wf) in zip(bufs, want):
        fb = gpu_ctx.download(b.fallback)
        com = inp.committed_in.copy()
        hq.unpack_lags(inp.last_index, gpu_ctx.download(b.cout_lag), com, fb)
        np.testing.assert_array_equal(com, wo)
        np.testing.assert_array_equal(gpu_ctx.download(b.changed), wc)
        np.testing.assert_array_equal(fb, wf)
        hq.free_commit(gpu_ctx, b)
