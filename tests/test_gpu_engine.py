"""The persistent commit engine (hq_engine_*) on the GPU: every posted step decides exactly what
hq_commit_dev decides for the same batch, and the launch-per-step kernels are themselves pinned
to the oracle (the first test re-checks that anchor through the engine). Covers voter counts 1-8,
both served term forms, the three served layouts (leader-row tiles, tiles, the in-place table),
ragged and empty batches, the ring wrapping many times, per-step completion signals with device
clocks, an idle exit followed by a relaunch, and several threads posting into one engine."""
import threading
import time

import numpy as np
import pytest

from oracle import qref

pytestmark = pytest.mark.gpu

SEED = 0x5EED0000 + 0xE0


def make_batch(ctx, hq, G, n, form, layout, seed):
    b = hq.alloc_commit(ctx, G, n, form, 16, tiled=True, tile_layout=layout)
    ctx.synth_commit_dev(hq.synth_spec(seed, G, n, parity_extras=True), b.args())
    ctx.tile_commit_dev(b.args(), b.tiles, layout)
    return b


def outputs(ctx, b):
    return [ctx.download(a) for a in (b.committed_out, b.changed, b.fallback)]


def poison(ctx, b):
    for a in (b.committed_out, b.changed, b.fallback):
        ctx.memset(a, 0xA5)


def launch_reference(ctx, b):
    """The same batch through the launch-per-step kernel (pinned to the oracle elsewhere)."""
    ctx.commit_dev(b.tile_args())
    ctx.sync()
    return outputs(ctx, b)


@pytest.mark.parametrize("form", [0, 2])
def test_engine_matches_oracle_c3_shape(gpu_ctx, hq, form):
    """BASELINE config 3's shape (5 voters, leader-row tiles) at 100 003 groups: the engine's
    decisions equal the CPU restatement's (oracle/qref.c) directly."""
    G, n = 100_003, 5
    b = make_batch(gpu_ctx, hq, G, n, form, hq.HQ_LAYOUT_TILES_LEADER, SEED + 1)
    poison(gpu_ctx, b)
    with hq.Engine(gpu_ctx, n, form, hq.HQ_LAYOUT_TILES_LEADER) as eng:
        seq = eng.post(b.tile_args())
        eng.wait(seq)
        got = outputs(gpu_ctx, b)
    inp = qref.CommitInputs(qref.spec(SEED + 1, G, n, parity_extras=True))
    want_out, want_chg, want_fb, rc = inp.run(form, False, nthreads=8)
    assert rc == 0
    np.testing.assert_array_equal(got[0], want_out)
    np.testing.assert_array_equal(got[1], want_chg)
    np.testing.assert_array_equal(got[2], want_fb)
    hq.free_commit(gpu_ctx, b)


@pytest.mark.parametrize("layout", [1, 2])
@pytest.mark.parametrize("form", [0, 2])
@pytest.mark.parametrize("n", range(1, 9))
def test_engine_equals_launches(gpu_ctx, hq, n, form, layout):
    """Several steps of different sizes (ragged, one group, empty) posted in one call."""
    sizes = [20_011, 1, 128, 0, 70_001, 129]
    bufs = [make_batch(gpu_ctx, hq, max(G, 1), n, form, layout, SEED + 31 * n + k)
            for k, G in enumerate(sizes)]
    want = [launch_reference(gpu_ctx, b) for b in bufs]
    for b in bufs:
        poison(gpu_ctx, b)
    gpu_ctx.sync()
    args = []
    for b, G in zip(bufs, sizes):
        a = b.tile_args()
        a.G = G
        args.append(a)
    with hq.Engine(gpu_ctx, n, form, layout) as eng:
        eng.post(hq.commit_batch_array(args))
        eng.drain()
    for b, G, w in zip(bufs, sizes, want):
        got = outputs(gpu_ctx, b)
        if G == 0:   # an empty step writes nothing
            assert (got[0] == np.uint64(0xA5A5A5A5A5A5A5A5)).all()
            continue
        for x, y in zip(got, w):
            np.testing.assert_array_equal(x, y)
        hq.free_commit(gpu_ctx, b)


@pytest.mark.parametrize("signal", [False, True])
def test_engine_ring_wraps(gpu_ctx, hq, signal):
    """37 steps through a 4-slot ring: the host waits for room (signal) or drains (no signal)
    every few posts; every step's outputs are the launch path's."""
    n, form, lay = 5, hq.HQ_FORM_TERM_MASK, hq.HQ_LAYOUT_TILES_LEADER
    bufs = [make_batch(gpu_ctx, hq, 5_000 + 77 * k, n, form, lay, SEED + 400 + k)
            for k in range(6)]
    want = [launch_reference(gpu_ctx, b) for b in bufs]
    with hq.Engine(gpu_ctx, n, form, lay, depth=4, signal=signal) as eng:
        seqs = []
        for s in range(37):
            b = bufs[s % len(bufs)]
            seqs.append(eng.post(b.tile_args()))
        eng.wait(seqs[-1])
        st = eng.info()
        assert st.completed >= seqs[-1] or not signal
        if signal:
            clocks = [eng.done_clock(q) for q in seqs[-4:]]
            assert clocks == sorted(clocks)
        eng.drain()
    for b, w in zip(bufs, want):
        for x, y in zip(outputs(gpu_ctx, b), w):
            np.testing.assert_array_equal(x, y)
        hq.free_commit(gpu_ctx, b)


def test_engine_idle_exit_and_relaunch(gpu_ctx, hq):
    """A resident launch with a 2 ms idle limit exits between posts; later posts relaunch it and
    every workgroup resumes at its own cursor."""
    n, form, lay = 3, hq.HQ_FORM_TERM_START, hq.HQ_LAYOUT_TILES_LEADER
    bufs = [make_batch(gpu_ctx, hq, 33_333, n, form, lay, SEED + 500 + k) for k in range(3)]
    want = [launch_reference(gpu_ctx, b) for b in bufs]
    for b in bufs:
        poison(gpu_ctx, b)
    gpu_ctx.sync()
    with hq.Engine(gpu_ctx, n, form, lay, signal=True, idle_us=2000) as eng:
        for b in bufs:
            seq = eng.post(b.tile_args())
            eng.wait(seq)
            time.sleep(0.05)           # well past the idle limit: the grid has exited
            assert eng.info().running in (0, 1)
        launches, ms = eng.timing()
        assert launches >= 2 and ms > 0
    for b, w in zip(bufs, want):
        for x, y in zip(outputs(gpu_ctx, b), w):
            np.testing.assert_array_equal(x, y)
        hq.free_commit(gpu_ctx, b)


def test_engine_in_place_table_steps(gpu_ctx, hq):
    """HQ_LAYOUT_IN_PLACE: a device-resident table posted as consecutive steps is decided in
    order per group; after two steps the table equals two in-place launches on a copy."""
    G, n, form = 50_000, 5, hq.HQ_FORM_TERM_MASK
    lay = hq.HQ_LAYOUT_TILES_LEADER
    b = make_batch(gpu_ctx, hq, G, n, form, lay, SEED + 600)
    words = b.tiles.count
    ref = gpu_ctx.empty(words, np.uint64)
    gpu_ctx.copy_to_ptr(ref.ptr, b.tiles, words * 8)
    chg_ref, chg = gpu_ctx.empty(hq.words64(G), np.uint64), gpu_ctx.empty(hq.words64(G), np.uint64)

    def table_args(tiles, changed):
        a = b.tile_args()
        a.layout = lay | hq.HQ_LAYOUT_IN_PLACE
        a.match = tiles.ptr
        a.committed_out = None
        a.changed = changed.ptr
        a.fallback = None
        return a

    for _ in range(2):
        gpu_ctx.commit_dev(table_args(ref, chg_ref))
    gpu_ctx.sync()
    with hq.Engine(gpu_ctx, n, form, lay | hq.HQ_LAYOUT_IN_PLACE) as eng:
        eng.post(hq.commit_batch_array([table_args(b.tiles, chg)] * 2))
        eng.drain()
    np.testing.assert_array_equal(gpu_ctx.download(b.tiles), gpu_ctx.download(ref))
    # the second step re-decides a decided table: nothing changes any more
    assert not gpu_ctx.download(chg).any() and not gpu_ctx.download(chg_ref).any()
    hq.free_commit(gpu_ctx, b)


def test_engine_threads_post_together(gpu_ctx, hq):
    """Four step workers (host threads) share one engine: 4 x 8 steps, all decided exactly."""
    n, form, lay = 5, hq.HQ_FORM_TERM_MASK, hq.HQ_LAYOUT_TILES_LEADER
    bufs = [make_batch(gpu_ctx, hq, 40_000 + 1_000 * k, n, form, lay, SEED + 700 + k)
            for k in range(4)]
    want = [launch_reference(gpu_ctx, b) for b in bufs]
    for b in bufs:
        poison(gpu_ctx, b)
    gpu_ctx.sync()
    errors = []
    with hq.Engine(gpu_ctx, n, form, lay, depth=8, signal=True) as eng:
        def worker(k):
            try:
                for _ in range(8):
                    eng.wait(eng.post(bufs[k].tile_args()))
            except Exception as e:  # surfaced below
                errors.append(e)

        ts = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=120)
        assert not errors, errors
        assert eng.info().posted >= 32
    for b, w in zip(bufs, want):
        for x, y in zip(outputs(gpu_ctx, b), w):
            np.testing.assert_array_equal(x, y)
        hq.free_commit(gpu_ctx, b)


def test_engine_rejects_mismatched_batches(gpu_ctx, hq):
    n, form, lay = 5, hq.HQ_FORM_TERM_MASK, hq.HQ_LAYOUT_TILES_LEADER
    b = make_batch(gpu_ctx, hq, 1_000, 3, form, lay, SEED + 800)
    with hq.Engine(gpu_ctx, n, form, lay) as eng:
        with pytest.raises(hq.HQError) as e:
            eng.post(b.tile_args())          # 3 voters into a 5-voter engine
        assert e.value.code == hq.HQ_E_INVAL
        with pytest.raises(hq.HQError):
            hq.Engine(gpu_ctx, n, hq.HQ_FORM_TERM_RING, lay)
    hq.free_commit(gpu_ctx, b)
