"""General multi-ctx ReadIndex (readindex.go:43-116).

CPU: the oracle's message replay against the reference's own table
(TestReadIndexLeaderCanBeConfirmed) and against the closed form the kernel uses (reach time =
max(q-1, 1)-th smallest first-ack ordinal, suffix-min release). GPU: the kernel against the
oracle, bit-exact, on random queues."""
import numpy as np
import pytest

from oracle import qref

NONE = 0xFFFF
U64MAX = np.uint64(0xFFFFFFFFFFFFFFFF)


def random_batch(rng, G, K_max, n_max, carried=True):
    K = rng.integers(1, K_max + 1, G).astype(np.uint8)
    n = rng.integers(1, n_max + 1, G).astype(np.uint8)
    idx = np.cumsum(rng.integers(0, 3, (K_max, G)), axis=0).astype(np.uint64) + np.uint64(100)
    ord_ = np.full((K_max, n_max, G), NONE, np.uint16)
    for g in range(G):
        cells = [(k, s) for k in range(K[g]) for s in range(n[g]) if rng.random() < 0.45]
        perm = rng.permutation(len(cells)) + 1
        for (k, s), o in zip(cells, perm):
            ord_[k, s, g] = 0 if (carried and rng.random() < 0.1) else o
    return ord_.reshape(-1), idx.reshape(-1), K, n


def closed_form(ord_, idx, K, n, K_max, n_max, G):
    ord_ = ord_.reshape(K_max, n_max, G)
    idx = idx.reshape(K_max, G)
    rel = np.full((K_max, G), U64MAX)
    cnt = np.zeros(G, np.uint8)
    bend = np.zeros(G, np.uint8)
    for g in range(G):
        q = int(n[g]) // 2 + 1
        r = max(q - 1, 1)
        t = []
        for k in range(K[g]):
            v = sorted(int(x) for x in ord_[k, :n[g], g] if x != NONE)
            t.append(v[r - 1] if len(v) >= r else None)
        best = None
        for k in reversed(range(K[g])):
            if t[k] is not None and (best is None or t[k] <= best[0]):
                best = (t[k], k)
            if best is not None:
                rel[k, g] = idx[best[1], g]
                cnt[g] += 1
                if best[1] == k:
                    bend[g] |= 1 << k
    return rel.reshape(-1), cnt, bend


def test_reference_table_as_batch():
    # readindex_test.go:125-162: queue ctx2(3), ctx(4), ctx3(5); ctx confirmed by 1 and 3, q = 3
    K_max, n_max, G = 3, 5, 1
    ord_ = np.full((K_max, n_max, G), NONE, np.uint16)
    ord_[1, 0, 0], ord_[1, 2, 0] = 1, 2          # from 1 -> slot 0, from 3 -> slot 2
    idx = np.array([[3], [4], [5]], np.uint64)
    rel, cnt, fb, bend = qref.readindex_multi_batch(ord_.reshape(-1), idx.reshape(-1), None, None,
                                                    5, K_max, n_max)
    assert list(rel) == [4, 4, int(U64MAX)] and cnt[0] == 2 and fb[0] == 0
    assert bend[0] == 0b010    # one confirm() released ctx2 and ctx: ctx closes the batch


def test_oracle_replay_equals_closed_form():
    rng = np.random.default_rng(5)
    G, K_max, n_max = 3000, 6, 7
    ord_, idx, K, n = random_batch(rng, G, K_max, n_max)
    rel, cnt, fb, bend = qref.readindex_multi_batch(ord_, idx, K, n, 0, K_max, n_max)
    want_rel, want_cnt, want_bend = closed_form(ord_, idx, K, n, K_max, n_max, G)
    assert not fb.any()
    np.testing.assert_array_equal(rel, want_rel)
    np.testing.assert_array_equal(cnt, want_cnt)
    np.testing.assert_array_equal(bend, want_bend)
    assert 0 < cnt.astype(int).sum() < K.astype(int).sum()


def test_decreasing_index_is_fallback():
    ord_ = np.full(2 * 3, NONE, np.uint16)
    rel, cnt, fb, bend = qref.readindex_multi_batch(ord_, np.array([5, 4], np.uint64), None, None,
                                                    3, 2, 3)
    assert fb[0] == 1 and cnt[0] == 0 and bend[0] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("K_max,n_max,G", [(8, 8, 20_011), (3, 5, 4097), (1, 3, 65)])
@pytest.mark.parametrize("compact", [False, True])
def test_kernel_matches_oracle(gpu_ctx, hq, K_max, n_max, G, compact):
    rng = np.random.default_rng(K_max * 100 + n_max)
    ord_, idx, K, n = random_batch(rng, G, K_max, n_max)
    n[::97] = 0                                   # invalid n -> fallback
    idx.reshape(K_max, G)[:, 5] = np.arange(K_max, 0, -1)   # decreasing -> fallback
    want_rel, want_cnt, want_fb, want_bend = qref.readindex_multi_batch(ord_, idx, K, n, 0, K_max,
                                                                        n_max)
    d = [gpu_ctx.upload(x) for x in (ord_, idx, K, n)]
    rel = gpu_ctx.empty(K_max * G, np.uint64)
    cnt = gpu_ctx.empty(G, np.uint8)
    bend = gpu_ctx.empty(G, np.uint8)
    fb = gpu_ctx.empty(hq.words64(G), np.uint64)
    gpu_ctx.memset(rel, 0x5A)
    gpu_ctx.readindex_multi_dev(G, K_max, n_max, d[0], d[1], d[2], d[3], 0,
                                None if compact else rel, cnt, fb, bend)
    _check_outputs(gpu_ctx, hq, K_max, idx, rel, cnt, fb, bend, compact,
                   (want_rel, want_cnt, want_fb, want_bend))
    for x in d + [rel, cnt, bend, fb]:
        gpu_ctx.free(x)


@pytest.mark.gpu
@pytest.mark.parametrize("K_max,n_max,G,perk,pern", [(8, 8, 20_010, True, True),
                                                     (4, 7, 4096, False, False),
                                                     (4, 7, 4098, True, False),
                                                     (3, 5, 130, False, True),
                                                     (2, 3, 2, True, True),
                                                     (1, 1, 64, False, False)])
@pytest.mark.parametrize("compact", [False, True])
def test_kernel_pairs_match_oracle(gpu_ctx, hq, K_max, n_max, G, perk, pern, compact):
    """Even G with aligned columns takes the two-groups-per-lane kernel (packed u16 sorting):
    every combination of per-group / uniform pending count and voter count, bit-exact."""
    rng = np.random.default_rng(K_max * 1000 + n_max + G)
    ord_, idx, K, n = random_batch(rng, G, K_max, n_max)
    if pern:
        n[::97] = 0
    if G > 5:
        idx.reshape(K_max, G)[:, 5] = np.arange(K_max, 0, -1)
    Kp = K if perk else None
    nv = n if pern else None
    nu = 0 if pern else n_max
    want_rel, want_cnt, want_fb, want_bend = qref.readindex_multi_batch(ord_, idx, Kp, nv, nu,
                                                                        K_max, n_max)
    d = [gpu_ctx.upload(x) if x is not None else None for x in (ord_, idx, Kp, nv)]
    rel = gpu_ctx.empty(K_max * G, np.uint64)
    cnt = gpu_ctx.empty(G, np.uint8)
    bend = gpu_ctx.empty(G, np.uint8)
    fb = gpu_ctx.empty(hq.words64(G), np.uint64)
    gpu_ctx.memset(fb, 0xFF)
    gpu_ctx.memset(rel, 0x5A)
    gpu_ctx.readindex_multi_dev(G, K_max, n_max, d[0], d[1], d[2], d[3], nu,
                                None if compact else rel, cnt, fb, bend)
    _check_outputs(gpu_ctx, hq, K_max, idx, rel, cnt, fb, bend, compact,
                   (want_rel, want_cnt, want_fb, want_bend))
    for x in [x for x in d if x is not None] + [rel, cnt, bend, fb]:
        gpu_ctx.free(x)


def tiles_reference(ord_, idx, Kp, nv, K_max, n_max, G):
    """numpy restatement of the 128-group tile layout (include/hipquorum.h)."""
    T = 128
    nt = (G + T - 1) // T
    o = np.full((K_max, n_max, nt * T), NONE, np.uint16)
    o[:, :, :G] = ord_.reshape(K_max, n_max, G)
    x = np.zeros((K_max, nt * T), np.uint64)
    x[:, :G] = idx.reshape(K_max, G)
    # ordinals voter-major: [tile][voter][pair of groups][ctx][2 groups]
    o = o.reshape(K_max, n_max, nt, T // 2, 2).transpose(2, 1, 3, 0, 4)
    parts = [np.ascontiguousarray(o).reshape(nt, -1).view(np.uint8),
             x.reshape(K_max, nt, T).transpose(1, 0, 2).reshape(nt, -1).view(np.uint8)]
    for c in (Kp, nv):
        if c is not None:
            u = np.zeros(nt * T, np.uint8)
            u[:G] = c
            parts.append(u.reshape(nt, T))
    return np.concatenate(parts, axis=1).reshape(-1)


@pytest.mark.parametrize("K_max,n_max,G,perk,pern", [(4, 7, 300, False, False),
                                                     (3, 5, 129, True, True),
                                                     (8, 8, 128, True, False)])
def test_tile_packer_layout(hq, K_max, n_max, G, perk, pern):
    rng = np.random.default_rng(G)
    ord_, idx, K, n = random_batch(rng, G, K_max, n_max)
    Kp, nv = (K if perk else None), (n if pern else None)
    tiles, flags = hq.tile_ri_multi_host(G, K_max, n_max, ord_, idx, Kp, nv)
    assert flags == (hq.HQ_RI_TILE_PER_K if perk else 0) | (hq.HQ_RI_TILE_PER_N if pern else 0)
    assert len(tiles) == (G + 127) // 128 * hq.ri_tile_bytes(K_max, n_max, flags)
    np.testing.assert_array_equal(tiles, tiles_reference(ord_, idx, Kp, nv, K_max, n_max, G))


TILE_CASES = [(8, 8, 20_010, True, True), (4, 7, 4096, False, False), (4, 7, 4098, True, False),
              (3, 5, 130, False, True), (2, 3, 2, True, True), (1, 1, 64, False, False),
              # uniform K_max in {2, 4, 8} and n = n_max: k_ri_tiles_u; K_max = 3: dword loads
              (8, 5, 2050, False, False), (2, 3, 258, False, False), (4, 1, 128, False, False),
              (3, 4, 514, False, False)]


@pytest.mark.gpu
@pytest.mark.parametrize("compact", [False, True])
@pytest.mark.parametrize("K_max,n_max,G,perk,pern", TILE_CASES)
def test_kernel_tiles_match_oracle(gpu_ctx, hq, K_max, n_max, G, perk, pern, compact):
    """The 128-group tile layout: the device packer equals the host packer, and the kernel over
    tiles is bit-exact with the oracle (every per-group / uniform combination). compact: no
    released_index written; hq_ri_released_host rebuilds it from the counts and batch ends."""
    rng = np.random.default_rng(K_max * 1000 + n_max + G + 7)
    ord_, idx, K, n = random_batch(rng, G, K_max, n_max)
    if pern:
        n[::97] = 0
    if G > 5:
        idx.reshape(K_max, G)[:, 5] = np.arange(K_max, 0, -1)
    Kp = K if perk else None
    nv = n if pern else None
    nu = 0 if pern else n_max
    want_rel, want_cnt, want_fb, want_bend = qref.readindex_multi_batch(ord_, idx, Kp, nv, nu,
                                                                        K_max, n_max)
    tiles_h, flags = hq.tile_ri_multi_host(G, K_max, n_max, ord_, idx, Kp, nv)
    d = [gpu_ctx.upload(x) if x is not None else None for x in (ord_, idx, Kp, nv)]
    dt = gpu_ctx.empty(len(tiles_h), np.uint8)
    gpu_ctx.memset(dt, 0xAB)
    gpu_ctx.tile_ri_multi_dev(G, K_max, n_max, d[0], d[1], d[2], d[3], dt)
    np.testing.assert_array_equal(gpu_ctx.download(dt), tiles_h)
    rel = gpu_ctx.empty(K_max * G, np.uint64)
    cnt = gpu_ctx.empty(G, np.uint8)
    bend = gpu_ctx.empty(G, np.uint8)
    fb = gpu_ctx.empty(hq.words64(G), np.uint64)
    gpu_ctx.memset(fb, 0xFF)
    gpu_ctx.memset(rel, 0x5A)
    gpu_ctx.readindex_multi_tiles_dev(G, K_max, n_max, dt, flags, nu, None if compact else rel,
                                      cnt, fb, bend)
    _check_outputs(gpu_ctx, hq, K_max, idx, rel, cnt, fb, bend, compact,
                   (want_rel, want_cnt, want_fb, want_bend))
    for x in [x for x in d if x is not None] + [dt, rel, cnt, bend, fb]:
        gpu_ctx.free(x)


def _check_outputs(gpu_ctx, hq, K_max, idx, rel, cnt, fb, bend, compact, want):
    want_rel, want_cnt, want_fb, want_bend = want
    c, b = gpu_ctx.download(cnt), gpu_ctx.download(bend)
    np.testing.assert_array_equal(c, want_cnt)
    np.testing.assert_array_equal(gpu_ctx.download(fb), want_fb)
    np.testing.assert_array_equal(b, want_bend)
    if compact:     # not written: still the poison; the host rebuild equals the kernels' output
        assert (gpu_ctx.download(rel).view(np.uint8) == 0x5A).all()
        np.testing.assert_array_equal(hq.ri_released_host(K_max, idx, c, b), want_rel)
    else:
        np.testing.assert_array_equal(gpu_ctx.download(rel), want_rel)


@pytest.mark.gpu
def test_uniform_tiles_on_the_general_kernel(hq):
    """HQ_RI_UNIFORM=0 (read at hq_open) sends uniform tiles through k_ri_multi2: same outputs."""
    import os
    K_max, n_max, G = 4, 7, 4098
    rng = np.random.default_rng(77)
    ord_, idx, K, n = random_batch(rng, G, K_max, n_max)
    want = qref.readindex_multi_batch(ord_, idx, None, None, n_max, K_max, n_max)
    tiles_h, flags = hq.tile_ri_multi_host(G, K_max, n_max, ord_, idx, None, None)
    os.environ["HQ_RI_UNIFORM"] = "0"
    try:
        ctx = hq.Context(0)
    finally:
        del os.environ["HQ_RI_UNIFORM"]
    try:
        dt = ctx.upload(tiles_h)
        rel, cnt = ctx.empty(K_max * G, np.uint64), ctx.empty(G, np.uint8)
        bend, fb = ctx.empty(G, np.uint8), ctx.empty(hq.words64(G), np.uint64)
        ctx.readindex_multi_tiles_dev(G, K_max, n_max, dt, flags, n_max, rel, cnt, fb, bend)
        _check_outputs(ctx, hq, K_max, idx, rel, cnt, fb, bend, False, want)
    finally:
        ctx.close()


@pytest.mark.parametrize("K_max,n", [(1, 3), (4, 7), (8, 5)])
def test_released_index_from_compact_outputs(K_max, n):
    """hq_ri_released_host rebuilds the released index the kernels write from the compact outputs
    (released count, batch ends) and the caller's ctx indexes: on the oracle's own outputs it
    gives the oracle's released index; a released entry without a closing ctx is refused."""
    from dragonboat_amd import hipquorum as hq

    rng = np.random.default_rng(11 + K_max)
    G = 5003
    ordn = rng.integers(1, K_max * n + 1, (K_max, n, G)).astype(np.uint16)
    ordn[rng.random((K_max, n, G)) < 0.3] = 0xFFFF
    idx = np.uint64(1000) + np.cumsum(rng.integers(0, 3, (K_max, G)), axis=0).astype(np.uint64)
    rel, cnt, fb, bend = qref.readindex_multi_batch(ordn.reshape(-1), idx.reshape(-1), None, None,
                                                    n, K_max, n, nthreads=2)
    assert not fb.any() and cnt.any()
    got = hq.ri_released_host(K_max, idx, cnt, bend)
    assert np.array_equal(got, rel)
    bad = bend.copy()
    g = int(np.flatnonzero(cnt)[0])
    bad[g] = 0                               # released entries, no closing ctx
    with pytest.raises(hq.HQError):
        hq.ri_released_host(K_max, idx, cnt, bad)


def test_released_index_host_edges():
    """hq_ri_released_host on the edges: an empty batch, K_max outside 1..8, a released count
    above K_max and mismatched column lengths are refused or empty, never a write past the end."""
    from dragonboat_amd import hipquorum as hq

    assert hq.ri_released_host(4, np.zeros(0, np.uint64), np.zeros(0, np.uint8),
                               np.zeros(0, np.uint8)).size == 0
    idx = np.arange(8, dtype=np.uint64)
    for K in (0, 9):
        with pytest.raises((hq.HQError, ValueError)):
            hq.ri_released_host(K, np.zeros(K * 2, np.uint64), np.zeros(2, np.uint8),
                                np.zeros(2, np.uint8))
    with pytest.raises(hq.HQError):                       # count 5 > K_max 4
        hq.ri_released_host(4, idx, np.array([5, 0], np.uint8), np.array([0x10, 0], np.uint8))
    with pytest.raises(ValueError):                       # ctx_index is not [K_max][G]
        hq.ri_released_host(4, idx[:6], np.zeros(2, np.uint8), np.zeros(2, np.uint8))
    # nothing released: every entry ~0, whatever the batch ends say
    out = hq.ri_released_host(4, idx, np.zeros(2, np.uint8), np.array([0xF, 0x1], np.uint8))
    assert (out == np.uint64(2**64 - 1)).all()
