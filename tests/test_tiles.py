"""HQ_LAYOUT_TILES on the host (no GPU): hq_tile_commit_host cuts the input columns of a commit
batch into 128-group tiles exactly as include/hipquorum.h lays them out."""
import ctypes

import numpy as np
import pytest

from oracle import qref

T = 128


def column_args(hq, inp, form, n):
    """CommitArgs over the host columns of a qref.CommitInputs (kept alive by the caller)."""
    a = hq.CommitArgs()
    a.G, a.n_max, a.form, a.ring_len, a.layout = inp.G, n, form, 16, hq.HQ_LAYOUT_COLUMNS
    a.match_stride = inp.G
    a.match = inp.match.ctypes.data
    a.committed_in = inp.committed_in.ctypes.data
    a.last_index = inp.last_index.ctypes.data
    a.term_start = inp.term_start.ctypes.data
    a.term = inp.term.ctypes.data
    a.term_mask = inp.term_mask.ctypes.data
    return a


def expected_tiles(hq, inp, form, n, lead=0):
    """lead = 1: HQ_LAYOUT_TILES_LEADER, the same tiles without match slot 0's row."""
    G = inp.G
    nt = hq.commit_tiles(G)
    rows = []
    pad = nt * T - G
    for s in range(lead, n):
        rows.append(inp.match[s * G:(s + 1) * G])
    rows += [inp.committed_in, inp.last_index]
    rows = [np.concatenate([r, np.zeros(pad, np.uint64)]).reshape(nt, T) for r in rows]
    if form == hq.HQ_FORM_TERM_MASK:
        m = np.concatenate([inp.term_mask, np.zeros(pad, np.uint16)]).reshape(nt, T)
        rows.append(m.view(np.uint64).reshape(nt, T // 4))
    else:
        aux = inp.term_start if form == hq.HQ_FORM_TERM_START else inp.term
        rows.append(np.concatenate([aux, np.zeros(pad, np.uint64)]).reshape(nt, T))
    tiles = np.concatenate(rows, axis=1)
    # row position 2i = group i of the tile, 2i + 1 = group 64 + i (include/hipquorum.h)
    perm = np.empty(T, np.int64)
    perm[0::2] = np.arange(T // 2)
    perm[1::2] = np.arange(T // 2) + T // 2
    out = np.empty_like(tiles)
    nrow = n - lead + 2
    for r in range(nrow):
        out[:, r * T:(r + 1) * T] = tiles[:, r * T:(r + 1) * T][:, perm]
    if form == hq.HQ_FORM_TERM_MASK:
        m = tiles[:, nrow * T:].copy().view(np.uint16)
        out[:, nrow * T:] = np.ascontiguousarray(m[:, perm]).view(np.uint64)
    else:
        out[:, nrow * T:] = tiles[:, nrow * T:][:, perm]
    return out.reshape(-1)


@pytest.mark.parametrize("G", [1, 127, 128, 129, 1000])
@pytest.mark.parametrize("n", [1, 3, 5, 8])
@pytest.mark.parametrize("form", [0, 1, 2, 3])
def test_tile_commit_host(hq, G, n, form):
    inp = qref.CommitInputs(qref.spec(0x5EED0100 + G, G, n, parity_extras=True))
    a = column_args(hq, inp, form, n)
    tiles = hq.tile_commit_host(a)
    assert tiles.size == hq.commit_tiles(G) * hq.commit_tile_words(n, form)
    np.testing.assert_array_equal(tiles, expected_tiles(hq, inp, form, n))


@pytest.mark.parametrize("G", [1, 129, 1000])
@pytest.mark.parametrize("n", [1, 3, 5, 8])
@pytest.mark.parametrize("form", [0, 1, 2, 3])
def test_tile_commit_host_leader(hq, G, n, form):
    """HQ_LAYOUT_TILES_LEADER: rows of match slots 1..n-1, then committed_in, last_index, term."""
    inp = qref.CommitInputs(qref.spec(0x5EED0200 + G, G, n, parity_extras=True))
    assert (inp.match[:G] == inp.last_index).all()   # the generator's leader slot (raft.go:918)
    a = column_args(hq, inp, form, n)
    tiles = hq.tile_commit_host(a, hq.HQ_LAYOUT_TILES_LEADER)
    assert tiles.size == hq.commit_tiles(G) * hq.commit_tile_words(n - 1, form)
    np.testing.assert_array_equal(tiles, expected_tiles(hq, inp, form, n, lead=1))


def test_tile_commit_host_leader_refuses_other_slot0(hq):
    """A group whose slot 0 is not its lastIndex cannot be carried by the leader layout."""
    G, n = 300, 3
    inp = qref.CommitInputs(qref.spec(0x5EED0300, G, n))
    inp.match[17] -= 1
    a = column_args(hq, inp, 0, n)
    out = np.zeros(hq.commit_tiles(G) * hq.commit_tile_words(n - 1, 0), np.uint64)
    assert hq.lib.hq_tile_commit_as_host(ctypes.byref(a), out.ctypes.data,
                                         hq.HQ_LAYOUT_TILES_LEADER) == hq.HQ_E_INVAL
    assert hq.lib.hq_tile_commit_as_host(ctypes.byref(a), out.ctypes.data, 7) == hq.HQ_E_INVAL
    # per-group n = 0 groups carry no slot 0 and are not checked
    nv = np.full(G, n, np.uint8)
    nv[17] = 0
    a.n_voting = nv.ctypes.data
    assert hq.lib.hq_tile_commit_as_host(ctypes.byref(a), out.ctypes.data,
                                         hq.HQ_LAYOUT_TILES_LEADER) == 0


def test_tile_commit_host_rejects_bad_input(hq):
    a = hq.CommitArgs()
    assert hq.lib.hq_tile_commit_host(ctypes.byref(a), None) == hq.HQ_E_INVAL
    a.G, a.n_max, a.layout = 4, 3, hq.HQ_LAYOUT_TILES
    out = np.zeros(1024, np.uint64)
    assert hq.lib.hq_tile_commit_host(ctypes.byref(a), out.ctypes.data) == hq.HQ_E_INVAL


# ---- bitmap tiles (hq_tile_bits_host) ------------------------------------------------------
@pytest.mark.parametrize("G,pern", [(1, False), (1023, True), (1024, False), (2049, True)])
def test_tile_bits_host_layout(hq, G, pern):
    """Tile t holds rows [n] ack granted rejected of groups [1024 t, 1024 t + 1024), 1024 bytes
    each, byte (g & 1023) = group g; the last tile's padding is zero."""
    rng = np.random.default_rng(G)
    cols = [rng.integers(0, 256, G, dtype=np.uint8) for _ in range(4)]
    ack, gr, rj, nv = cols
    t = hq.tile_bits_host(ack, gr, rj, nv if pern else None)
    rows = 4 if pern else 3
    T = hq.HQ_BITS_TILE_GROUPS
    assert t.size == hq.bits_tiles(G) * rows * T
    tiles = t.reshape(hq.bits_tiles(G), rows, T)
    want = ([nv] if pern else []) + [ack, gr, rj]
    for r, col in enumerate(want):
        flat = tiles[:, r, :].reshape(-1)
        np.testing.assert_array_equal(flat[:G], col)
        assert not flat[G:].any()


def test_bench_byte_accounting():
    """bench.py's algorithmic bytes per decision for the headline layouts:
    56 B (tiles), 48 B (leader-row tiles), 24 B (lags), 20 B (lags without the leader row)."""
    import bench

    w = bench.WORKLOADS
    assert bench.algo_bytes_per_group(w["c2t"]) == 56
    assert bench.algo_bytes_per_group(w["c2tl"]) == 48
    assert bench.algo_bytes_per_group(w["c2l"]) == 24
    assert bench.algo_bytes_per_group(w["c2ll"]) == 20
    assert bench.algo_bytes_per_group(w["c5v5tl"]) == 58
    # the headline: BASELINE config 3, 1M x 5 voters, mask form, leader rows
    assert bench.HEADLINE == "c3mtl"
    assert bench.algo_bytes_per_group(w["c3mtl"]) == 58
    assert w["c3mtl"]["G"] == 1 << 20 and w["c3mtl"]["n"] == 5 and w["c3mtl"]["cfg"] == 2


@pytest.mark.parametrize("form,lead", [(2, 1), (0, 1), (2, 0), (0, 0)])
def test_tile_view_reads_back_the_columns(hq, form, lead):
    """hipquorum.TileView (the host-side view of a device table's tiles) recovers every column
    the host packer put into the tiles, and set_row writes one group's field in place."""
    G, n = 1000 + 37, 5
    inp = qref.CommitInputs(qref.spec(0x5EED3000, G, n))
    lay = hq.HQ_LAYOUT_TILES_LEADER if lead else hq.HQ_LAYOUT_TILES
    tiles = hq.tile_commit_host(column_args(hq, inp, form, n), lay)
    v = hq.tile_view(tiles, G, n, form, lay)
    np.testing.assert_array_equal(v.match().reshape(-1), inp.match)
    np.testing.assert_array_equal(v.row("committed"), inp.committed_in)
    np.testing.assert_array_equal(v.row("last_index"), inp.last_index)
    np.testing.assert_array_equal(v.row("aux"), inp.term_mask if form == 2 else inp.term_start)
    g = np.array([0, 63, 64, 127, 128, G - 1])
    v.set_row("committed", g, np.arange(6, dtype=np.uint64) + 7)
    got = hq.tile_view(tiles, G, n, form, lay).row("committed")
    np.testing.assert_array_equal(got[g], np.arange(6, dtype=np.uint64) + 7)
    keep = np.setdiff1d(np.arange(G), g)
    np.testing.assert_array_equal(got[keep], inp.committed_in[keep])
