"""CheckQuorum over active-flag planes (hq_check_quorum_planes_dev; raft.go:380-390 with the
setNotActive reset of remote.go:196-198).

The leader's own slot always counts (raft.go:384), so a group keeps the active flags of its other
voting slots as bit planes (plus 3 planes of n - 1 when n is per group), 32 groups per lane
decided with bitwise adders as the vote / ReadIndex planes.

CPU: the host packer against a numpy restatement of the layout and its contract checks.
GPU: every active byte for every n in [1, 8] and every valid self slot, packed on the device
(== the host packer), decided and compared with the oracle (oracle/qref.c leaderHasQuorum); the
kernel ignores plane bits beyond a group's n - 1 voters; uniform-n batches for n = 1..8; ragged
sizes; the active planes are zero afterwards and the n planes untouched."""
import numpy as np
import pytest

from oracle import qref

T = 2048


def cq_planes_reference(active, nv, n_uniform, self_slot):
    """numpy restatement of the CheckQuorum plane layout (include/hipquorum.h)."""
    G = len(active)
    per = nv is not None
    n = nv.astype(np.int64) if per else np.full(G, n_uniform, np.int64)
    bad = (n < 1) | (n > 8) | (self_slot >= n)
    nc = np.clip(n, 1, 8)
    a = active.astype(np.int64) & ((1 << nc) - 1)
    bits = (a & ((1 << self_slot) - 1)) | ((a >> (self_slot + 1)) << self_slot)
    if per:
        bits |= (nc - 1) << 7
    bits = np.where(bad, 0, bits)
    NP = 10 if per else n_uniform - 1
    nt = (G + T - 1) // T
    flat = np.zeros(nt * T, np.int64)
    flat[:G] = bits
    out = np.zeros((nt, NP, T // 8), np.uint8)
    for q in range(NP):
        out[:, q, :] = np.packbits(((flat >> q) & 1).astype(np.uint8).reshape(nt, T), axis=1,
                                   bitorder="little")
    fb = np.zeros(((G + 63) // 64) * 64, np.uint8)
    fb[:G] = bad
    return out.reshape(-1), np.packbits(fb, bitorder="little").view(np.uint64)


@pytest.mark.parametrize("G", [1, 1000, 2048, 5001])
@pytest.mark.parametrize("self_slot", [0, 2, 7])
def test_host_packer_layout(hq, G, self_slot):
    rng = np.random.default_rng(G + 31 * self_slot)
    act = rng.integers(0, 256, G, dtype=np.uint8)
    nv = rng.integers(0, 10, G, dtype=np.uint8)
    pl, fb = hq.tile_cq_planes_host(act, nv, 0, self_slot)
    want_p, want_fb = cq_planes_reference(act, nv, 0, self_slot)
    np.testing.assert_array_equal(pl, want_p)
    np.testing.assert_array_equal(fb, want_fb)
    for nu in range(max(1, self_slot + 1), 9):
        pl, fb = hq.tile_cq_planes_host(act, None, nu, self_slot)
        want_p, want_fb = cq_planes_reference(act, None, nu, self_slot)
        np.testing.assert_array_equal(pl, want_p)
        np.testing.assert_array_equal(fb, want_fb)
        assert len(pl) == hq.cq_plane_bytes(G, nu)


def test_host_packer_contract(hq):
    act = np.zeros(10, np.uint8)
    with pytest.raises(Exception):
        hq.tile_cq_planes_host(act, None, 0, 0)        # neither n_voting nor n_uniform
    with pytest.raises(Exception):
        hq.tile_cq_planes_host(act, None, 9, 0)        # n_uniform > 8
    with pytest.raises(Exception):
        hq.tile_cq_planes_host(act, None, 3, 3)        # self_slot >= n_uniform
    with pytest.raises(Exception):
        hq.tile_cq_planes_host(act, np.full(10, 3, np.uint8), 3, 0)   # both


def _bits(words, G):
    return np.unpackbits(np.asarray(words).view(np.uint8), bitorder="little")[:G]


@pytest.mark.gpu
@pytest.mark.parametrize("self_slot", [0, 3, 7])
def test_cq_planes_exhaustive(gpu_ctx, hq, self_slot):
    """Every active byte x n in 0..9 (0 and 9 break the contract) x 8 copies, per-group n."""
    act = np.tile(np.arange(256, dtype=np.uint8), 10 * 8)
    nv = np.repeat(np.arange(10, dtype=np.uint8), 256 * 8)
    G = act.size
    pl_h, fb_h = hq.tile_cq_planes_host(act, nv, 0, self_slot)
    da, dn = gpu_ctx.upload(act), gpu_ctx.upload(nv)
    dp = gpu_ctx.empty(hq.cq_plane_bytes(G, 0), np.uint8)
    gpu_ctx.memset(dp, 0xAB)
    dfb = gpu_ctx.empty(hq.words64(G), np.uint64)
    gpu_ctx.tile_cq_planes_dev(G, da, dn, 0, self_slot, dp, dfb)
    np.testing.assert_array_equal(gpu_ctx.download(dp), pl_h)
    np.testing.assert_array_equal(gpu_ctx.download(dfb), fb_h)
    hqb = gpu_ctx.empty(hq.words64(G), np.uint64)
    gpu_ctx.memset(hqb, 0xCD)
    gpu_ctx.check_quorum_planes_dev(G, dp, 0, hqb)
    want_hq, want_fb, _ = qref.check_quorum_batch(act, nv, 0, self_slot)
    np.testing.assert_array_equal(gpu_ctx.download(dfb), want_fb)
    ok = ~_bits(want_fb, G).astype(bool)
    np.testing.assert_array_equal(_bits(gpu_ctx.download(hqb), G)[ok], _bits(want_hq, G)[ok])
    after = gpu_ctx.download(dp).reshape(-1, 10, T // 8)
    assert not after[:, :7].any()                                  # setNotActive
    np.testing.assert_array_equal(after[:, 7:], pl_h.reshape(-1, 10, T // 8)[:, 7:])
    for x in (da, dn, dp, dfb, hqb):
        gpu_ctx.free(x)


@pytest.mark.gpu
def test_cq_planes_ignore_bits_beyond_n(gpu_ctx, hq):
    """Random planes: active bits of slots >= n - 1 are set too, and the kernel must not count
    them (the byte kernel ignores bits >= n likewise)."""
    rng = np.random.default_rng(7)
    G = 40 * T + 777
    nt = (G + T - 1) // T
    planes = rng.integers(0, 256, nt * 10 * (T // 8), dtype=np.uint8)
    bits = np.unpackbits(planes.reshape(nt, 10, T // 8), axis=2, bitorder="little")  # [t, q, j]
    bits = bits.transpose(0, 2, 1).reshape(nt * T, 10)[:G].astype(np.int64)
    n = 1 + bits[:, 7] + 2 * bits[:, 8] + 4 * bits[:, 9]
    cnt = sum(bits[:, k] * (k < n - 1) for k in range(7))
    want = (1 + cnt >= n // 2 + 1).astype(np.uint8)
    dp = gpu_ctx.upload(planes)
    hqb = gpu_ctx.empty(hq.words64(G), np.uint64)
    gpu_ctx.memset(hqb, 0xCD)
    gpu_ctx.check_quorum_planes_dev(G, dp, 0, hqb)
    got = np.unpackbits(gpu_ctx.download(hqb).view(np.uint8), bitorder="little")
    np.testing.assert_array_equal(got[:G], want)
    assert not got[G:].any()                                       # zero beyond G
    gpu_ctx.free(dp)
    gpu_ctx.free(hqb)


@pytest.mark.gpu
@pytest.mark.parametrize("n", range(1, 9))
@pytest.mark.parametrize("G", [1, 33, 2049, 70_001])
def test_cq_planes_uniform_n(gpu_ctx, hq, n, G):
    rng = np.random.default_rng(1000 * n + G)
    act = rng.integers(0, 256, G, dtype=np.uint8)
    self_slot = int(rng.integers(0, n))
    pl_h, fb_h = hq.tile_cq_planes_host(act, None, n, self_slot)
    assert not fb_h.any()
    da = gpu_ctx.upload(act)
    dp = gpu_ctx.empty(max(16, hq.cq_plane_bytes(G, n)), np.uint8)
    gpu_ctx.tile_cq_planes_dev(G, da, None, n, self_slot, dp)
    np.testing.assert_array_equal(gpu_ctx.download(dp)[:len(pl_h)], pl_h)
    hqb = gpu_ctx.empty(hq.words64(G), np.uint64)
    gpu_ctx.memset(hqb, 0xCD)
    gpu_ctx.check_quorum_planes_dev(G, dp, n, hqb)
    want_hq, _, _ = qref.check_quorum_batch(act, None, n, self_slot)
    np.testing.assert_array_equal(gpu_ctx.download(hqb), want_hq)
    assert not gpu_ctx.download(dp)[:len(pl_h)].any()              # setNotActive
    for x in (da, dp, hqb):
        gpu_ctx.free(x)


@pytest.mark.gpu
@pytest.mark.parametrize("G", [1, 31, 32, 33, 63, 64, 65, 2047, 2048, 2049, 5000])
def test_cq_planes_ragged(gpu_ctx, hq, G):
    inp = qref.BitmapInputs(qref.spec(0x5EED3500 + G, G, 7, mixed_n=True, parity_extras=True))
    act, nv = inp.ack.copy(), inp.n_voting
    pl_h, fb_h = hq.tile_cq_planes_host(act, nv, 0, 0)
    dp = gpu_ctx.upload(pl_h)
    hqb = gpu_ctx.empty(hq.words64(G), np.uint64)
    gpu_ctx.memset(hqb, 0xCD)
    gpu_ctx.check_quorum_planes_dev(G, dp, 0, hqb)
    want_hq, want_fb, _ = qref.check_quorum_batch(act, nv, 0, 0)
    np.testing.assert_array_equal(fb_h, want_fb)
    ok = ~_bits(want_fb, G).astype(bool)
    got = np.unpackbits(gpu_ctx.download(hqb).view(np.uint8), bitorder="little")
    np.testing.assert_array_equal(got[:G][ok], _bits(want_hq, G)[ok])
    assert not got[G:].any()
    gpu_ctx.free(dp)
    gpu_ctx.free(hqb)
