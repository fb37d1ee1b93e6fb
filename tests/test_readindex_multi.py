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
def test_kernel_matches_oracle(gpu_ctx, hq, K_max, n_max, G):
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
    gpu_ctx.readindex_multi_dev(G, K_max, n_max, d[0], d[1], d[2], d[3], 0, rel, cnt, fb, bend)
    np.testing.assert_array_equal(gpu_ctx.download(rel), want_rel)
    np.testing.assert_array_equal(gpu_ctx.download(cnt), want_cnt)
    np.testing.assert_array_equal(gpu_ctx.download(fb), want_fb)
    np.testing.assert_array_equal(gpu_ctx.download(bend), want_bend)
    for x in d + [rel, cnt, bend, fb]:
        gpu_ctx.free(x)


@pytest.mark.gpu
@pytest.mark.parametrize("K_max,n_max,G,perk,pern", [(8, 8, 20_010, True, True),
                                                     (4, 7, 4096, False, False),
                                                     (4, 7, 4098, True, False),
                                                     (3, 5, 130, False, True),
                                                     (2, 3, 2, True, True),
                                                     (1, 1, 64, False, False)])
def test_kernel_pairs_match_oracle(gpu_ctx, hq, K_max, n_max, G, perk, pern):
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
    gpu_ctx.readindex_multi_dev(G, K_max, n_max, d[0], d[1], d[2], d[3], nu, rel, cnt, fb, bend)
    np.testing.assert_array_equal(gpu_ctx.download(rel), want_rel)
    np.testing.assert_array_equal(gpu_ctx.download(cnt), want_cnt)
    np.testing.assert_array_equal(gpu_ctx.download(fb), want_fb)
    np.testing.assert_array_equal(gpu_ctx.download(bend), want_bend)
    for x in [x for x in d if x is not None] + [rel, cnt, bend, fb]:
        gpu_ctx.free(x)


def tiles_reference(ord_, idx, Kp, nv, K_max, n_max, G):
    """numpy restatement of the 128-group tile layout (include/hipquorum.h)."""
    T = 128
    nt = (G + T - 1) // T
    o = np.full((K_max * n_max, nt * T), NONE, np.uint16)
    o[:, :G] = ord_.reshape(K_max * n_max, G)
    x = np.zeros((K_max, nt * T), np.uint64)
    x[:, :G] = idx.reshape(K_max, G)
    parts = [o.reshape(K_max * n_max, nt, T).transpose(1, 0, 2).reshape(nt, -1).view(np.uint8),
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


@pytest.mark.gpu
@pytest.mark.parametrize("K_max,n_max,G,perk,pern", [(8, 8, 20_010, True, True),
                                                     (4, 7, 4096, False, False),
                                                     (4, 7, 4098, True, False),
                                                     (3, 5, 130, False, True),
                                                     (2, 3, 2, True, True),
                                                     (1, 1, 64, False, False)])
def test_kernel_tiles_match_oracle(gpu_ctx, hq, K_max, n_max, G, perk, pern):
    """The 128-group tile layout: the device packer equals the host packer, and the kernel over
    tiles is bit-exact with the oracle (every per-group / uniform combination)."""
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
    gpu_ctx.readindex_multi_tiles_dev(G, K_max, n_max, dt, flags, nu, rel, cnt, fb, bend)
    np.testing.assert_array_equal(gpu_ctx.download(rel), want_rel)
    np.testing.assert_array_equal(gpu_ctx.download(cnt), want_cnt)
    np.testing.assert_array_equal(gpu_ctx.download(fb), want_fb)
    np.testing.assert_array_equal(gpu_ctx.download(bend), want_bend)
    for x in [x for x in d if x is not None] + [dt, rel, cnt, bend, fb]:
        gpu_ctx.free(x)
