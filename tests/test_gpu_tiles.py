"""HQ_LAYOUT_TILES commit decisions on the GPU, bit-exact with the CPU oracle: every term form,
voter counts 1-8, uniform and per-group n, ragged last tiles, the fused multi-bucket launch, the
host-staged entry point, and the full BASELINE size. The device tile packer is checked word for
word against the host one first."""
import ctypes

import numpy as np
import pytest

from oracle import qref
from test_gpu_parity import popcount, upload_commit

pytestmark = pytest.mark.gpu

SEED = 0x5EED0000


def tiled_args(hq, cols, tiles, layout=None):
    a = hq.CommitArgs.from_buffer_copy(cols)
    a.layout = hq.HQ_LAYOUT_TILES if layout is None else layout
    a.match = tiles.ptr
    a.match_stride = 0
    a.committed_in = a.last_index = a.term_start = a.term = a.term_mask = None
    return a


def host_tiles(hq, inp, form, layout=None):
    a = hq.CommitArgs()
    a.G, a.n_max, a.form, a.ring_len = inp.G, inp.n_max, form, inp.R
    a.match_stride = inp.G
    a.match = inp.match.ctypes.data
    a.committed_in = inp.committed_in.ctypes.data
    a.last_index = inp.last_index.ctypes.data
    a.term_start = inp.term_start.ctypes.data
    a.term = inp.term.ctypes.data
    if inp.term_mask is not None:
        a.term_mask = inp.term_mask.ctypes.data
    return hq.tile_commit_host(a, hq.HQ_LAYOUT_TILES if layout is None else layout)


def run_tiled(ctx, hq, inp, form, per_group_n, layout=None):
    """Columns uploaded, tiled on the device (checked against the host packer), decided from
    the tiles. Returns (committed_out, changed, fallback)."""
    layout = hq.HQ_LAYOUT_TILES if layout is None else layout
    d = upload_commit(ctx, hq, inp, form, per_group_n)
    words = hq.commit_tiles(inp.G) * hq.commit_tile_words(inp.n_max, form, layout)
    tiles = ctx.empty(words, np.uint64)
    ctx.tile_commit_dev(d["args"], tiles, layout)
    ctx.sync()
    np.testing.assert_array_equal(ctx.download(tiles), host_tiles(hq, inp, form, layout))
    ctx.commit_dev(tiled_args(hq, d["args"], tiles, layout))
    ctx.sync()
    out = ctx.download(d["out"])[:inp.G]
    chg, fb = ctx.download(d["chg"]), ctx.download(d["fb"])
    for b in d["bufs"] + [tiles]:
        ctx.free(b)
    return out, chg, fb


@pytest.mark.parametrize("form", [0, 1, 2, 3])
@pytest.mark.parametrize("n", range(1, 9))
def test_tiled_commit_every_form_and_n(gpu_ctx, hq, form, n):
    for G, pern in ((1, False), (129, True), (20_011, False), (20_011, True)):
        inp = qref.CommitInputs(qref.spec(SEED + 7 * n + G, G, n, mixed_n=pern and n >= 7,
                                          parity_extras=True))
        out, chg, fb = run_tiled(gpu_ctx, hq, inp, form, pern)
        want_out, want_chg, want_fb, rc = inp.run(form, pern, nthreads=8)
        assert rc == 0
        np.testing.assert_array_equal(out, want_out)
        np.testing.assert_array_equal(chg, want_chg)
        np.testing.assert_array_equal(fb, want_fb)


@pytest.mark.parametrize("form", [0, 1, 2, 3])
@pytest.mark.parametrize("n", range(1, 9))
def test_leader_tiles_every_form_and_n(gpu_ctx, hq, form, n):
    """HQ_LAYOUT_TILES_LEADER (slot 0 taken from last_index): the same decisions."""
    for G, pern in ((1, False), (129, True), (20_011, False), (20_011, True)):
        inp = qref.CommitInputs(qref.spec(SEED + 11 * n + G, G, n, mixed_n=pern and n >= 7,
                                          parity_extras=True))
        out, chg, fb = run_tiled(gpu_ctx, hq, inp, form, pern, hq.HQ_LAYOUT_TILES_LEADER)
        want_out, want_chg, want_fb, rc = inp.run(form, pern, nthreads=8)
        assert rc == 0
        np.testing.assert_array_equal(out, want_out)
        np.testing.assert_array_equal(chg, want_chg)
        np.testing.assert_array_equal(fb, want_fb)


@pytest.mark.parametrize("layout", [1, 2])
def test_tiled_full_size_c2(gpu_ctx, hq, layout):
    """BASELINE config 2 (1M groups x 3 voters, term-start) in tiles, device-generated."""
    G, n = 1 << 20, 3
    b = hq.alloc_commit(gpu_ctx, G, n, hq.HQ_FORM_TERM_START, 16, tiled=True, tile_layout=layout)
    gpu_ctx.synth_commit_dev(hq.synth_spec(SEED + 1, G, n), b.args())
    gpu_ctx.tile_commit_dev(b.args(), b.tiles, layout)
    gpu_ctx.commit_dev(b.tile_args())
    gpu_ctx.sync()
    inp = qref.CommitInputs(qref.spec(SEED + 1, G, n))
    want_out, want_chg, want_fb, rc = inp.run(hq.HQ_FORM_TERM_START, False, nthreads=8)
    assert rc == 0
    np.testing.assert_array_equal(gpu_ctx.download(b.committed_out), want_out)
    np.testing.assert_array_equal(gpu_ctx.download(b.changed), want_chg)
    assert popcount(gpu_ctx.download(b.fallback)) == 0
    hq.free_commit(gpu_ctx, b)


@pytest.mark.parametrize("layout", [1, 2])
@pytest.mark.parametrize("form", [0, 2, 1, 3])
def test_tiled_fused_buckets_equal_separate(gpu_ctx, hq, form, layout):
    """Voter-count buckets of one step in one tiled launch = each bucket decided alone."""
    sizes = [(3, 70_001), (5, 40_000), (7, 33_333), (1, 5), (8, 1_000)]
    bufs = []
    for k, (n, G) in enumerate(sizes):
        b = hq.alloc_commit(gpu_ctx, G, n, form, 16, tiled=True, tile_layout=layout)
        gpu_ctx.synth_commit_dev(hq.synth_spec(SEED + 40 + k, G, n, parity_extras=True),
                                 b.args())
        gpu_ctx.tile_commit_dev(b.args(), b.tiles, layout)
        bufs.append(b)
    gpu_ctx.commit_fused_dev(hq.commit_batch_array([b.tile_args() for b in bufs]))
    gpu_ctx.sync()
    for k, (b, (n, G)) in enumerate(zip(bufs, sizes)):
        inp = qref.CommitInputs(qref.spec(SEED + 40 + k, G, n, parity_extras=True))
        want_out, want_chg, want_fb, rc = inp.run(form, False, nthreads=8)
        assert rc == 0
        np.testing.assert_array_equal(gpu_ctx.download(b.committed_out), want_out)
        np.testing.assert_array_equal(gpu_ctx.download(b.changed), want_chg)
        np.testing.assert_array_equal(gpu_ctx.download(b.fallback), want_fb)
        hq.free_commit(gpu_ctx, b)


def test_headline_window_in_one_fused_launch(gpu_ctx, hq):
    """The bench headline's shape (bench.py --mode fused): 20 batches of 5-voter groups in the
    mask form over leader-row tiles, disjoint groups per batch, decided by ONE launch; each batch
    equals the oracle (at 1/16 of the bench's 1 M groups per batch)."""
    n, form, lay, G = 5, hq.HQ_FORM_TERM_MASK, hq.HQ_LAYOUT_TILES_LEADER, 65_536
    bufs = []
    for k in range(20):
        b = hq.alloc_commit(gpu_ctx, G, n, form, 16, tiled=True, tile_layout=lay)
        gpu_ctx.synth_commit_dev(hq.synth_spec(SEED + 300 + k, G, n, parity_extras=True),
                                 b.args())
        gpu_ctx.tile_commit_dev(b.args(), b.tiles, lay)
        bufs.append(b)
    gpu_ctx.timing_reset()
    gpu_ctx.timing(True)
    gpu_ctx.commit_fused_dev(hq.commit_batch_array([b.tile_args() for b in bufs]))
    gpu_ctx.sync()
    gpu_ctx.timing(False)
    assert gpu_ctx.timing_read()[1] == 1
    for k, b in enumerate(bufs):
        inp = qref.CommitInputs(qref.spec(SEED + 300 + k, G, n, parity_extras=True))
        want_out, want_chg, want_fb, rc = inp.run(form, False, nthreads=8)
        assert rc == 0
        np.testing.assert_array_equal(gpu_ctx.download(b.committed_out), want_out)
        np.testing.assert_array_equal(gpu_ctx.download(b.changed), want_chg)
        np.testing.assert_array_equal(gpu_ctx.download(b.fallback), want_fb)
        hq.free_commit(gpu_ctx, b)


@pytest.mark.parametrize("layout", [1, 2])
def test_tiled_host_entry_point(gpu_ctx, hq, layout):
    """hq_commit with host tiles: one H2D block, same decisions."""
    G, n, form = 10_007, 5, hq.HQ_FORM_TERM_RING32
    inp = qref.CommitInputs(qref.spec(SEED + 99, G, n, parity_extras=True))
    tiles = host_tiles(hq, inp, form, layout)
    ring32 = hq.pack_ring32(inp.ring)
    out = np.zeros(G, np.uint64)
    chg = np.zeros(hq.words64(G), np.uint64)
    fb = np.zeros(hq.words64(G), np.uint64)
    a = hq.CommitArgs()
    a.G, a.n_max, a.form, a.ring_len, a.layout = G, n, form, 16, layout
    a.match = tiles.ctypes.data
    a.ring32 = ring32.ctypes.data
    a.committed_out = out.ctypes.data
    a.changed, a.fallback = chg.ctypes.data, fb.ctypes.data
    gpu_ctx.commit_host(a)
    want_out, want_chg, want_fb, rc = inp.run(form, False, nthreads=8)
    np.testing.assert_array_equal(out, want_out)
    np.testing.assert_array_equal(chg, want_chg)
    np.testing.assert_array_equal(fb, want_fb)


def test_tiled_validation(gpu_ctx, hq):
    a = hq.CommitArgs()
    a.G, a.n_max, a.form, a.layout = 1000, 3, 0, hq.HQ_LAYOUT_TILES
    with pytest.raises(hq.HQError):
        gpu_ctx.commit_dev(a)                       # no tiles
    t = gpu_ctx.empty(4096, np.uint64)
    o = gpu_ctx.empty(1001, np.uint64)
    a.match, a.committed_out = t.ptr + 8, o.ptr      # misaligned tiles
    with pytest.raises(hq.HQError):
        gpu_ctx.commit_dev(a)
    a.layout = 7
    with pytest.raises(hq.HQError):
        gpu_ctx.commit_dev(a)
    assert hq.lib.hq_commit_dev(gpu_ctx.h, ctypes.byref(a)) == hq.HQ_E_INVAL
    gpu_ctx.free(t)
    gpu_ctx.free(o)


@pytest.mark.parametrize("tiled", [False, True])
def test_commit_grid_stride_beyond_cap(gpu_ctx, hq, tiled):
    """More groups than one capped grid covers (HQ_MAX_BLOCKS x 256 threads, two groups per
    lane = 8M groups): the grid-stride loop's second iteration, columns and tiles, bit-exact."""
    G, n = (8 << 20) + 4099, 5
    form = hq.HQ_FORM_TERM_MASK
    b = hq.alloc_commit(gpu_ctx, G, n, form, 16, tiled=tiled)
    gpu_ctx.synth_commit_dev(hq.synth_spec(SEED + 11, G, n), b.args())
    if tiled:
        gpu_ctx.tile_commit_dev(b.args(), b.tiles)
        gpu_ctx.commit_dev(b.tile_args())
    else:
        gpu_ctx.commit_dev(b.args())
    gpu_ctx.sync()
    inp = qref.CommitInputs(qref.spec(SEED + 11, G, n))
    want_out, want_chg, want_fb, rc = inp.run(form, False, nthreads=16)
    assert rc == 0
    np.testing.assert_array_equal(gpu_ctx.download(b.committed_out), want_out)
    np.testing.assert_array_equal(gpu_ctx.download(b.changed), want_chg)
    assert popcount(gpu_ctx.download(b.fallback)) == 0
    hq.free_commit(gpu_ctx, b)


# ---- bitmap tiles: fused ReadIndex + vote over 1024-group tiles ------------------------------
def _bits_tiled(ctx, hq, inp, G, pern, n_uniform):
    """Columns uploaded, tiled on the device (checked against the host packer), decided from
    the tiles. Returns (confirmed, outcome, fallback) words."""
    nv = inp.n_voting if pern else None
    cols = [ctx.upload(np.ascontiguousarray(a)) if a is not None else None
            for a in (inp.ack, inp.granted, inp.rejected, nv)]
    tiles = ctx.empty(hq.bits_tile_bytes(G, pern), np.uint8)
    ctx.memset(tiles, 0xAB)
    ctx.tile_bits_dev(G, *cols, tiles)
    ctx.sync()
    np.testing.assert_array_equal(ctx.download(tiles),
                                  hq.tile_bits_host(inp.ack, inp.granted, inp.rejected, nv))
    conf = ctx.empty(hq.words64(G), np.uint64)
    outc = ctx.empty(hq.words32(G), np.uint64)
    fb = ctx.empty(hq.words64(G), np.uint64)
    for x in (conf, outc, fb):
        ctx.memset(x, 0xFF)
    ctx.readindex_vote_tiles_dev(G, tiles, pern, n_uniform, conf, outc, fb)
    ctx.sync()
    res = [ctx.download(x) for x in (conf, outc, fb)]
    for x in [c for c in cols if c is not None] + [tiles, conf, outc, fb]:
        ctx.free(x)
    return res


@pytest.mark.parametrize("G", [1, 16, 17, 63, 65, 1023, 1024, 1025, 5000, 20_011])
@pytest.mark.parametrize("pern", [True, False])
def test_tiled_bits_equal_oracle(gpu_ctx, hq, G, pern):
    n = 8 if pern else 7
    inp = qref.BitmapInputs(qref.spec(SEED + G + pern, G, n, mixed_n=pern, parity_extras=True))
    nu = 0 if pern else n
    conf, outc, fb = _bits_tiled(gpu_ctx, hq, inp, G, pern, nu)
    nv = inp.n_voting if pern else None
    want_conf, want_fb = qref.readindex_batch(inp.ack, nv, nu)
    want_out, want_fb2 = qref.vote_batch(inp.granted, inp.rejected, nv, nu)
    np.testing.assert_array_equal(conf, want_conf)
    np.testing.assert_array_equal(outc, want_out)
    np.testing.assert_array_equal(fb, want_fb)
    np.testing.assert_array_equal(fb, want_fb2)


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 6, 8])
def test_tiled_bits_uniform_n(gpu_ctx, hq, n):
    G = 3000
    inp = qref.BitmapInputs(qref.spec(SEED + 100 + n, G, n, parity_extras=True))
    conf, outc, fb = _bits_tiled(gpu_ctx, hq, inp, G, False, n)
    np.testing.assert_array_equal(conf, qref.readindex_batch(inp.ack, None, n)[0])
    np.testing.assert_array_equal(outc, qref.vote_batch(inp.granted, inp.rejected, None, n)[0])
    assert popcount(fb) == 0


def test_tiled_bits_validation(gpu_ctx, hq):
    G = 100
    tiles = gpu_ctx.empty(hq.bits_tile_bytes(G, False), np.uint8)
    conf = gpu_ctx.empty(hq.words64(G), np.uint64)
    outc = gpu_ctx.empty(hq.words32(G), np.uint64)
    with pytest.raises(hq.HQError):
        gpu_ctx.readindex_vote_tiles_dev(G, tiles, False, 0, conf, outc)   # n_uniform 0
    with pytest.raises(hq.HQError):
        gpu_ctx.readindex_vote_tiles_dev(G, tiles.ptr + 1, False, 7, conf, outc)   # misaligned
    with pytest.raises(hq.HQError):
        gpu_ctx.readindex_vote_tiles_dev(G, None, False, 7, conf, outc)
    for x in (tiles, conf, outc):
        gpu_ctx.free(x)


@pytest.mark.parametrize("pern", [True, False])
def test_tiled_bits_full_size_config4(gpu_ctx, hq, pern):
    """BASELINE config 4 at full size (16M groups x 7 voters) over tiles, device-generated."""
    G = 16 << 20
    arrs = [gpu_ctx.empty(G, np.uint8) for _ in range(4)]
    da, dg, dr, dn = arrs
    gpu_ctx.synth_bitmaps_dev(hq.synth_spec(SEED + 3, G, 7), da, dg, dr, dn)
    tiles = gpu_ctx.empty(hq.bits_tile_bytes(G, pern), np.uint8)
    gpu_ctx.tile_bits_dev(G, da, dg, dr, dn if pern else None, tiles)
    conf = gpu_ctx.empty(hq.words64(G), np.uint64)
    outc = gpu_ctx.empty(hq.words32(G), np.uint64)
    gpu_ctx.readindex_vote_tiles_dev(G, tiles, pern, 0 if pern else 7, conf, outc)
    inp = qref.BitmapInputs(qref.spec(SEED + 3, G, 7))
    nv = inp.n_voting if pern else None
    nu = 0 if pern else 7
    want_conf, _ = qref.readindex_batch(inp.ack, nv, nu, nthreads=16)
    want_out, _ = qref.vote_batch(inp.granted, inp.rejected, nv, nu, nthreads=16)
    np.testing.assert_array_equal(gpu_ctx.download(conf), want_conf)
    np.testing.assert_array_equal(gpu_ctx.download(outc), want_out)
    for x in arrs + [tiles, conf, outc]:
        gpu_ctx.free(x)
