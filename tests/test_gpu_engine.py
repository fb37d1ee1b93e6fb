"""The persistent commit engine (hq_engine_*) on the GPU: every posted step decides exactly what
hq_commit_dev decides for the same batch, and the launch-per-step kernels are themselves pinned
to the oracle (the first test re-checks that anchor through the engine). Covers voter counts 1-8,
both served term forms, the three served layouts (leader-row tiles, tiles, the in-place table),
ragged and empty batches, the ring wrapping many times, per-step completion signals with device
clocks, an idle exit followed by a relaunch, and several threads posting into one engine."""
import os
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
            # (a step's flag is written by its own last workgroup: an earlier step's may land
            # just after a later one's, so each is awaited before its clock is read)
            for q in seqs[-4:]:
                eng.wait(q)
            clocks = [eng.done_clock(q) for q in seqs[-4:]]
            # (static ownership completes steps in post order; the balanced mode's pools can
            # finish an older step after a newer one, each step's flag still its own)
            if os.environ.get("HQ_ENGINE_BALANCE", "0") == "0":
                assert clocks == sorted(clocks)
        eng.drain()
    for b, w in zip(bufs, want):
        for x, y in zip(outputs(gpu_ctx, b), w):
            np.testing.assert_array_equal(x, y)
        hq.free_commit(gpu_ctx, b)


@pytest.mark.parametrize("signal", [False, True])
@pytest.mark.parametrize("steps", [6, 45])
def test_engine_run_bounded(gpu_ctx, hq, signal, steps):
    """hq_engine_run: the steps and the STOP in one launch (45 > the 32 descriptors a launch's
    arguments carry: the rest arrive through the ring); then, with a grid left resident by a
    signalled post, a run whose STOP reaches the running grid. Every step's outputs are the
    launch path's and no launch is left running."""
    n, form, lay = 5, hq.HQ_FORM_TERM_MASK, hq.HQ_LAYOUT_TILES_LEADER
    bufs = [make_batch(gpu_ctx, hq, 3_000 + 131 * k, n, form, lay, SEED + 700 + k) for k in range(5)]
    want = [launch_reference(gpu_ctx, b) for b in bufs]
    with hq.Engine(gpu_ctx, n, form, lay, signal=signal) as eng:
        for rnd in range(2):
            for b in bufs:
                poison(gpu_ctx, b)
            gpu_ctx.sync()
            if rnd == 1 and signal:          # a grid resident when the run posts
                eng.wait(eng.post(bufs[0].tile_args()))
                assert eng.info().running
            first = eng.run(hq.commit_batch_array([bufs[s % 5].tile_args() for s in range(steps)]))
            st = eng.info()
            assert not st.running and st.completed == st.posted and first + steps < st.posted + 1
            for b, w in zip(bufs, want):
                for x, y in zip(outputs(gpu_ctx, b), w):
                    np.testing.assert_array_equal(x, y)
    for b in bufs:
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


@pytest.mark.parametrize("signal", [False, True])
def test_engine_in_place_dependent_steps(gpu_ctx, hq, signal):
    """HQ_LAYOUT_IN_PLACE with an ordering the result depends on: two steps over one
    undecided 1 M-group table (every workgroup of the grid owns tiles), each with its own
    `changed` bitmap. Step 1 must see the table as posted (its bitmap = the launch path's), step 2
    the table step 1 left (nothing changes any more: an all-zero bitmap). A step 2 tile decided
    before step 1's would re-set its changed bits."""
    G, n, form = 1 << 20, 5, hq.HQ_FORM_TERM_MASK
    lay = hq.HQ_LAYOUT_TILES_LEADER
    b = make_batch(gpu_ctx, hq, G, n, form, lay, SEED + 650)
    words = b.tiles.count
    ref = gpu_ctx.empty(words, np.uint64)
    gpu_ctx.copy_to_ptr(ref.ptr, b.tiles, words * 8)
    chg = [gpu_ctx.empty(hq.words64(G), np.uint64) for _ in range(3)]

    def table_args(tiles, changed):
        a = b.tile_args()
        a.layout = lay | hq.HQ_LAYOUT_IN_PLACE
        a.match = tiles.ptr
        a.committed_out = None
        a.changed = changed.ptr
        a.fallback = None
        return a

    gpu_ctx.commit_dev(table_args(ref, chg[0]))          # the launch path, one step
    gpu_ctx.sync()
    want1 = gpu_ctx.download(chg[0])
    assert want1.any()                                    # the table was undecided
    for c in chg[1:]:
        gpu_ctx.memset(c, 0xA5)
    gpu_ctx.sync()
    with hq.Engine(gpu_ctx, n, form, lay | hq.HQ_LAYOUT_IN_PLACE, signal=signal) as eng:
        eng.post(hq.commit_batch_array([table_args(b.tiles, chg[1]), table_args(b.tiles, chg[2])]))
        eng.drain()
    np.testing.assert_array_equal(gpu_ctx.download(chg[1]), want1)
    assert not gpu_ctx.download(chg[2]).any()
    np.testing.assert_array_equal(gpu_ctx.download(b.tiles), gpu_ctx.download(ref))
    hq.free_commit(gpu_ctx, b)


def test_engine_in_place_keeps_one_G(gpu_ctx, hq):
    """An in-place table's steps keep the G of the engine's first in-place post: a tile then stays
    with its workgroup, which is what orders a group's steps; another G is HQ_E_INVAL."""
    G, n, form = 20_000, 3, hq.HQ_FORM_TERM_START
    lay = hq.HQ_LAYOUT_TILES_LEADER
    b = make_batch(gpu_ctx, hq, G, n, form, lay, SEED + 660)
    a = b.tile_args()
    a.layout = lay | hq.HQ_LAYOUT_IN_PLACE
    a.committed_out = None
    with hq.Engine(gpu_ctx, n, form, lay | hq.HQ_LAYOUT_IN_PLACE) as eng:
        eng.post(a)
        a2 = b.tile_args()
        a2.layout, a2.committed_out, a2.G = a.layout, None, G - 128
        with pytest.raises(hq.HQError) as e:
            eng.post(a2)
        assert e.value.code == hq.HQ_E_INVAL and "one G" in str(e.value)
        with pytest.raises(hq.HQError):            # also inside one post call
            eng.post(hq.commit_batch_array([a, a2]))
        eng.post(a)                                 # the same G still posts
        eng.drain()
    hq.free_commit(gpu_ctx, b)


def test_engine_wait_near_the_idle_limit(gpu_ctx, hq):
    """Posts that land around the idle limit: the grid ends as a whole (workgroup 0
    publishes the exit, the others follow once they hold every relayed step), so a post that
    arrives as it ends waits for a relaunch, never for another idle limit. idle_us = 20 ms; every
    wait must be well below it."""
    n, form, lay = 3, hq.HQ_FORM_TERM_START, hq.HQ_LAYOUT_TILES_LEADER
    b = make_batch(gpu_ctx, hq, 65_536, n, form, lay, SEED + 520)
    want = launch_reference(gpu_ctx, b)
    worst = 0.0
    with hq.Engine(gpu_ctx, n, form, lay, signal=True, idle_us=20_000) as eng:
        eng.wait(eng.post(b.tile_args()))
        for gap_ms in (19.0, 19.5, 19.8, 20.0, 20.2, 20.5, 21.0, 22.0, 25.0):
            time.sleep(gap_ms / 1e3)
            t0 = time.perf_counter()
            eng.wait(eng.post(b.tile_args()))
            worst = max(worst, time.perf_counter() - t0)
        launches, _ = eng.timing()
    assert worst < 0.010, worst
    for x, y in zip(outputs(gpu_ctx, b), want):
        np.testing.assert_array_equal(x, y)
    hq.free_commit(gpu_ctx, b)


def test_engine_many_steps_one_post_each(gpu_ctx, hq):
    """200 steps posted one call each into a 64-slot engine without signals (drains keep a slot
    for the STOP): the workgroups' tickets run across many ring wraps and relaunches; the last
    batch's outputs are the launch path's."""
    n, form, lay = 5, hq.HQ_FORM_TERM_MASK, hq.HQ_LAYOUT_TILES_LEADER
    bufs = [make_batch(gpu_ctx, hq, 30_000 + 4_000 * k, n, form, lay, SEED + 900 + k)
            for k in range(3)]
    want = [launch_reference(gpu_ctx, b) for b in bufs]
    for b in bufs:
        poison(gpu_ctx, b)
    gpu_ctx.sync()
    with hq.Engine(gpu_ctx, n, form, lay) as eng:
        for s in range(200):
            eng.post(bufs[s % 3].tile_args())
        eng.drain()
        st = eng.info()
        assert st.completed == st.posted >= 200
    for b, w in zip(bufs, want):
        for x, y in zip(outputs(gpu_ctx, b), w):
            np.testing.assert_array_equal(x, y)
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
