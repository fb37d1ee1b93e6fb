"""3-byte bitmap tiles (hq_readindex_vote_tiles3_dev) and their bit-plane
transpose (hq_readindex_vote_planes_dev): the leader's own slot
is implicit (never acks its ctx — readindex.go:84 counts it as the +1 —, always grants its own
vote, raft.go:1093, never rejects it), so ack / granted / rejected / n fit 3 bytes per group.

CPU: the host packer against a numpy restatement of the layout and its contract checks.
GPU: every (ack, granted, rejected) combination of the 7 other slots for every n in [1, 8]
(2^21 x 8 groups, tiles built directly) decided and compared with the oracle (oracle/qref.c
readIndex.confirm / handleVoteResp restatements) on the same groups in the 4-byte form; the
device packer equals the host packer. The bit-plane tiles are checked the same way, and their host
packer against the transpose of the 3-byte tiles."""
import numpy as np
import pytest

from oracle import qref


def pack3_reference(ack, gr, rj, nv):
    """numpy restatement of the 3-byte layout (include/hipquorum.h)."""
    G = len(ack)
    n = nv.astype(np.uint32)
    bad = (n < 1) | (n > 8) | (ack & 1).astype(bool) | ~(gr & 1).astype(bool) | \
        (rj & 1).astype(bool)
    keep = ((1 << np.clip(n, 1, 8)) - 2).astype(np.uint32)
    m = (np.clip(n, 1, 8) - 1).astype(np.uint32)
    rows = []
    for k, col in enumerate((ack, gr, rj)):
        r = ((col.astype(np.uint32) & keep) >> 1) | (((m >> k) & 1) << 7)
        rows.append(np.where(bad, 0, r).astype(np.uint8))
    nt = (G + 1023) // 1024
    out = np.zeros((nt, 3, 1024), np.uint8)
    for k in range(3):
        flat = np.zeros(nt * 1024, np.uint8)
        flat[:G] = rows[k]
        out[:, k, :] = flat.reshape(nt, 1024)
    fb = np.zeros(((G + 63) // 64) * 64, np.uint8)
    fb[:G] = bad
    return out.reshape(-1), np.packbits(fb, bitorder="little").view(np.uint64)


@pytest.mark.parametrize("G", [1, 1000, 1024, 3001])
def test_host_packer_layout(hq, G):
    rng = np.random.default_rng(G)
    ack = rng.integers(0, 256, G, dtype=np.uint8)
    gr = rng.integers(0, 256, G, dtype=np.uint8)
    rj = rng.integers(0, 256, G, dtype=np.uint8)
    ack[rng.random(G) < 0.7] &= 0xFE        # mostly inside the contract
    gr[rng.random(G) < 0.7] |= 1
    rj[rng.random(G) < 0.7] &= 0xFE
    nv = rng.integers(0, 10, G, dtype=np.uint8)
    tiles, fb = hq.tile_bits3_host(ack, gr, rj, nv)
    want_t, want_fb = pack3_reference(ack, gr, rj, nv)
    np.testing.assert_array_equal(tiles, want_t)
    np.testing.assert_array_equal(fb, want_fb)
    # uniform n
    tiles, fb = hq.tile_bits3_host(ack, gr, rj, None, 5)
    want_t, want_fb = pack3_reference(ack, gr, rj, np.full(G, 5, np.uint8))
    np.testing.assert_array_equal(tiles, want_t)
    np.testing.assert_array_equal(fb, want_fb)


@pytest.mark.gpu
def test_tiles3_exhaustive(gpu_ctx, hq):
    x = np.arange(1 << 21, dtype=np.uint32)
    a7, g7, r7 = x & 0x7F, (x >> 7) & 0x7F, (x >> 14) & 0x7F
    G = (1 << 21) * 8
    ack = np.tile((a7 << 1).astype(np.uint8), 8)
    gr = np.tile(((g7 << 1) | 1).astype(np.uint8), 8)
    rj = np.tile((r7 << 1).astype(np.uint8), 8)
    nv = np.repeat(np.arange(1, 9, dtype=np.uint8), 1 << 21)
    # tiles built directly from the definition (bits >= n - 1 of the others kept: the kernel
    # must ignore them, as the 4-byte kernels ignore bits >= n)
    m = (nv.astype(np.uint32) - 1)
    rows = [((np.tile(v, 8) | (((m >> k) & 1) << 7))).astype(np.uint8)
            for k, v in enumerate((a7, g7, r7))]
    tiles = np.stack([r.reshape(-1, 1024) for r in rows], axis=1).reshape(-1)
    dt = gpu_ctx.upload(tiles)
    conf = gpu_ctx.empty(hq.words64(G), np.uint64)
    outc = gpu_ctx.empty(hq.words32(G), np.uint64)
    gpu_ctx.readindex_vote_tiles3_dev(G, dt, conf, outc)
    want_conf = qref.readindex_batch(ack, nv, 0, nthreads=16)[0]
    want_outc = qref.vote_batch(gr, rj, nv, 0, nthreads=16)[0]
    np.testing.assert_array_equal(gpu_ctx.download(conf), want_conf)
    np.testing.assert_array_equal(gpu_ctx.download(outc), want_outc)
    for d in (dt, conf, outc):
        gpu_ctx.free(d)


@pytest.mark.gpu
@pytest.mark.parametrize("G", [1, 1000, 70_001])
def test_device_packer_equals_host_and_decides(gpu_ctx, hq, G):
    rng = np.random.default_rng(G + 1)
    inp = qref.BitmapInputs(qref.spec(0x5EED3300 + G, G, 7, mixed_n=True, parity_extras=True))
    ack, gr, rj, nv = inp.ack.copy(), inp.granted.copy(), inp.rejected.copy(), inp.n_voting
    # the generator's parity extras include self acks and missing self grants: contract
    # violations the packer must flag
    tiles_h, fb_h = hq.tile_bits3_host(ack, gr, rj, nv)
    cols = [gpu_ctx.upload(c) for c in (ack, gr, rj, nv)]
    dt = gpu_ctx.empty(hq.bits_tiles(G) * 3072, np.uint8)
    gpu_ctx.memset(dt, 0xAB)
    dfb = gpu_ctx.empty(hq.words64(G), np.uint64)
    gpu_ctx.tile_bits3_dev(G, *cols, 0, dt, dfb)
    np.testing.assert_array_equal(gpu_ctx.download(dt), tiles_h)
    np.testing.assert_array_equal(gpu_ctx.download(dfb), fb_h)
    conf = gpu_ctx.empty(hq.words64(G), np.uint64)
    outc = gpu_ctx.empty(hq.words32(G), np.uint64)
    gpu_ctx.readindex_vote_tiles3_dev(G, dt, conf, outc)
    want_conf = qref.readindex_batch(ack, nv, 0, nthreads=8)[0]
    want_outc = qref.vote_batch(gr, rj, nv, 0, nthreads=8)[0]
    ok = ~np.unpackbits(fb_h.view(np.uint8), bitorder="little")[:G].astype(bool)
    got_c = np.unpackbits(gpu_ctx.download(conf).view(np.uint8), bitorder="little")[:G]
    want_c = np.unpackbits(want_conf.view(np.uint8), bitorder="little")[:G]
    np.testing.assert_array_equal(got_c[ok], want_c[ok])
    o = gpu_ctx.download(outc)
    got_o = (o[np.arange(G) // 32] >> (2 * (np.arange(G) % 32)).astype(np.uint64)) & 3
    want_o = (want_outc[np.arange(G) // 32] >> (2 * (np.arange(G) % 32)).astype(np.uint64)) & 3
    np.testing.assert_array_equal(got_o[ok], want_o[ok])
    assert ok.sum() > G * 0.9 or G < 100
    for d in cols + [dt, dfb, conf, outc]:
        gpu_ctx.free(d)


def planes_from_tiles3(tiles3, G):
    """The bit-plane layout as a transpose of the 3-byte tiles (include/hipquorum.h)."""
    T = 2048
    nt = (G + T - 1) // T
    rows = tiles3.reshape(-1, 3, 1024)                 # 1024-group tiles: rows ack, gr, rj
    flat = np.zeros((3, nt * T), np.uint8)
    k = min(rows.shape[0] * 1024, nt * T)
    for r in range(3):
        flat[r, :k] = rows[:, r, :].reshape(-1)[:k]
    bits = np.unpackbits(flat[:, :, None], axis=2, bitorder="little")   # [3, g, 8]
    out = np.zeros((nt, 24, T // 8), np.uint8)
    for r in range(3):
        for b in range(8):
            plane = bits[r, :, b].reshape(nt, T)
            out[:, 8 * r + b, :] = np.packbits(plane, axis=1, bitorder="little")
    return out.reshape(-1)


@pytest.mark.parametrize("G", [1, 1000, 2048, 5001])
def test_plane_packer_is_the_transpose(hq, G):
    rng = np.random.default_rng(G + 7)
    ack = rng.integers(0, 256, G, dtype=np.uint8)
    gr = rng.integers(0, 256, G, dtype=np.uint8)
    rj = rng.integers(0, 256, G, dtype=np.uint8)
    ack[rng.random(G) < 0.7] &= 0xFE
    gr[rng.random(G) < 0.7] |= 1
    rj[rng.random(G) < 0.7] &= 0xFE
    nv = rng.integers(0, 10, G, dtype=np.uint8)
    t3, fb3 = hq.tile_bits3_host(ack, gr, rj, nv)
    pl, fbp = hq.tile_planes_host(ack, gr, rj, nv)
    np.testing.assert_array_equal(pl, planes_from_tiles3(t3, G))
    np.testing.assert_array_equal(fbp, fb3)


@pytest.mark.gpu
def test_planes_exhaustive(gpu_ctx, hq):
    """Every (ack, granted, rejected) combination of the 7 other slots for every n in [1, 8]."""
    x = np.arange(1 << 21, dtype=np.uint32)
    a7, g7, r7 = x & 0x7F, (x >> 7) & 0x7F, (x >> 14) & 0x7F
    G = (1 << 21) * 8
    ack = np.tile((a7 << 1).astype(np.uint8), 8)
    gr = np.tile(((g7 << 1) | 1).astype(np.uint8), 8)
    rj = np.tile((r7 << 1).astype(np.uint8), 8)
    nv = np.repeat(np.arange(1, 9, dtype=np.uint8), 1 << 21)
    # the planes of groups whose bits >= n - 1 are kept (the kernel must ignore them)
    m = (nv.astype(np.uint32) - 1)
    rows = [((np.tile(v, 8) | (((m >> k) & 1) << 7))).astype(np.uint8)
            for k, v in enumerate((a7, g7, r7))]
    tiles3 = np.stack([r.reshape(-1, 1024) for r in rows], axis=1).reshape(-1)
    dp = gpu_ctx.upload(planes_from_tiles3(tiles3, G))
    conf = gpu_ctx.empty(hq.words64(G), np.uint64)
    outc = gpu_ctx.empty(hq.words32(G), np.uint64)
    gpu_ctx.readindex_vote_planes_dev(G, dp, conf, outc)
    want_conf = qref.readindex_batch(ack, nv, 0, nthreads=16)[0]
    want_outc = qref.vote_batch(gr, rj, nv, 0, nthreads=16)[0]
    np.testing.assert_array_equal(gpu_ctx.download(conf), want_conf)
    np.testing.assert_array_equal(gpu_ctx.download(outc), want_outc)
    for d in (dp, conf, outc):
        gpu_ctx.free(d)


@pytest.mark.gpu
@pytest.mark.parametrize("G", [1, 20, 1000, 2048, 70_001])
def test_plane_device_packer_equals_host_and_decides(gpu_ctx, hq, G):
    inp = qref.BitmapInputs(qref.spec(0x5EED3400 + G, G, 7, mixed_n=True, parity_extras=True))
    ack, gr, rj, nv = inp.ack.copy(), inp.granted.copy(), inp.rejected.copy(), inp.n_voting
    pl_h, fb_h = hq.tile_planes_host(ack, gr, rj, nv)
    cols = [gpu_ctx.upload(c) for c in (ack, gr, rj, nv)]
    dp = gpu_ctx.empty(hq.plane_tiles(G) * 3 * hq.HQ_PLANE_TILE_GROUPS, np.uint8)
    gpu_ctx.memset(dp, 0xAB)
    dfb = gpu_ctx.empty(hq.words64(G), np.uint64)
    gpu_ctx.tile_planes_dev(G, *cols, 0, dp, dfb)
    np.testing.assert_array_equal(gpu_ctx.download(dp), pl_h)
    np.testing.assert_array_equal(gpu_ctx.download(dfb), fb_h)
    conf = gpu_ctx.empty(hq.words64(G), np.uint64)
    outc = gpu_ctx.empty(hq.words32(G), np.uint64)
    gpu_ctx.memset(conf, 0xCD)
    gpu_ctx.memset(outc, 0xCD)
    gpu_ctx.readindex_vote_planes_dev(G, dp, conf, outc)
    want_conf = qref.readindex_batch(ack, nv, 0, nthreads=8)[0]
    want_outc = qref.vote_batch(gr, rj, nv, 0, nthreads=8)[0]
    ok = ~np.unpackbits(fb_h.view(np.uint8), bitorder="little")[:G].astype(bool)
    got_c = np.unpackbits(gpu_ctx.download(conf).view(np.uint8), bitorder="little")
    want_c = np.unpackbits(want_conf.view(np.uint8), bitorder="little")
    np.testing.assert_array_equal(got_c[:G][ok], want_c[:G][ok])
    assert not got_c[G:].any()                  # the last bitmap word is zero beyond G
    o = gpu_ctx.download(outc)
    idx = np.arange(G)
    got_o = (o[idx // 32] >> (2 * (idx % 32)).astype(np.uint64)) & 3
    want_o = (want_outc[idx // 32] >> (2 * (idx % 32)).astype(np.uint64)) & 3
    np.testing.assert_array_equal(got_o[ok], want_o[ok])
    tail = G % 32
    if tail:                                    # codes beyond G in the last word are 0
        assert int(o[-1]) >> (2 * tail) == 0
    for d in cols + [dp, dfb, conf, outc]:
        gpu_ctx.free(d)
