"""ReadIndex + vote + CheckQuorum in one pass over bit planes (hq_readindex_vote_cq_planes_dev).

A step worker decides the ReadIndex confirmation (readindex.go:77-116), the vote tally
(raft.go:1968-1985) and CheckQuorum (raft.go:380-390, with the setNotActive reset of
remote.go:196-198) for the same leader groups, so the fused kernel reads a tile's 24 ack / vote
planes and its 7 active-flag planes in one launch.

GPU: against the oracle (oracle/qref.c readindex / vote / leaderHasQuorum batches) on
generator batches with contract-breaking groups (masked by the packers' fallback bits), on
every active byte x n in 1..8, and on ragged sizes; the fused outputs equal the two separate
kernels' bit for bit, the active planes are zero afterwards and the vote planes untouched.
CPU: the ABI export (test_abi.py covers every declared symbol)."""
import numpy as np
import pytest

from oracle import qref

T = 2048


def _bits(words, G):
    return np.unpackbits(np.asarray(words).view(np.uint8), bitorder="little")[:G]


def _codes(words, G):
    idx = np.arange(G)
    return (np.asarray(words)[idx // 32] >> (2 * (idx % 32)).astype(np.uint64)) & 3


def _run_fused(ctx, hq, ack, gr, rj, act, nv):
    G = len(ack)
    cols = [ctx.upload(c) for c in (ack, gr, rj, nv)]
    dp = ctx.empty(hq.plane_tiles(G) * 3 * T, np.uint8)
    dfb = ctx.empty(hq.words64(G), np.uint64)
    ctx.tile_planes_dev(G, *cols, 0, dp, dfb)
    da = ctx.upload(act)
    dap = ctx.empty(hq.cq_plane_bytes(G, 8), np.uint8)
    ctx.tile_cq_planes_dev(G, da, None, 8, 0, dap)
    ctx.sync()
    planes_before = ctx.download(dp)
    conf = ctx.empty(hq.words64(G), np.uint64)
    outc = ctx.empty(hq.words32(G), np.uint64)
    hqb = ctx.empty(hq.words64(G), np.uint64)
    for x in (conf, outc, hqb):
        ctx.memset(x, 0xCD)
    ctx.readindex_vote_cq_planes_dev(G, dp, dap, conf, outc, hqb)
    out = {"conf": ctx.download(conf), "outc": ctx.download(outc), "hq": ctx.download(hqb),
           "fb": ctx.download(dfb), "active_after": ctx.download(dap),
           "planes_after": ctx.download(dp), "planes_before": planes_before}
    # the ReadIndex + vote kernel alone on the same planes
    c2, o2 = ctx.empty(hq.words64(G), np.uint64), ctx.empty(hq.words32(G), np.uint64)
    ctx.readindex_vote_planes_dev(G, dp, c2, o2)
    out["sep_conf"], out["sep_outc"] = ctx.download(c2), ctx.download(o2)
    for x in cols + [dp, dfb, da, dap, conf, outc, hqb, c2, o2]:
        ctx.free(x)
    return out


def _check(hq, out, ack, gr, rj, act, nv):
    G = len(ack)
    want_conf = qref.readindex_batch(ack, nv, 0, nthreads=8)[0]
    want_outc = qref.vote_batch(gr, rj, nv, 0, nthreads=8)[0]
    want_hq = qref.check_quorum_batch(act, nv, 0, 0, nthreads=8)[0]
    ok = ~_bits(out["fb"], G).astype(bool)
    np.testing.assert_array_equal(_bits(out["conf"], G)[ok], _bits(want_conf, G)[ok])
    np.testing.assert_array_equal(_codes(out["outc"], G)[ok], _codes(want_outc, G)[ok])
    np.testing.assert_array_equal(_bits(out["hq"], G)[ok], _bits(want_hq, G)[ok])
    # fused == separate, bit for bit (fallback groups included), zero beyond G
    np.testing.assert_array_equal(out["conf"], out["sep_conf"])
    np.testing.assert_array_equal(out["outc"], out["sep_outc"])
    got_hq = np.unpackbits(out["hq"].view(np.uint8), bitorder="little")
    assert not got_hq[G:].any()
    assert not out["active_after"].any()                         # setNotActive
    np.testing.assert_array_equal(out["planes_after"], out["planes_before"])


@pytest.mark.gpu
@pytest.mark.parametrize("G", [1, 31, 33, 2047, 2048, 2049, 70_001, 1 << 20])
def test_fused_planes_cq_generator(gpu_ctx, hq, G):
    inp = qref.BitmapInputs(qref.spec(0x5EED3600 + G, G, 7, mixed_n=True, parity_extras=True))
    ack, gr, rj, nv = inp.ack.copy(), inp.granted.copy(), inp.rejected.copy(), inp.n_voting
    rng = np.random.default_rng(G)
    act = rng.integers(0, 256, G, dtype=np.uint8)     # bits >= n set too: must be ignored
    out = _run_fused(gpu_ctx, hq, ack, gr, rj, act, nv)
    _check(hq, out, ack, gr, rj, act, nv)


@pytest.mark.gpu
def test_fused_planes_cq_every_active_byte(gpu_ctx, hq):
    """Every active byte for every n in [1, 8] (x 4 copies), random valid ack / vote bytes."""
    act = np.tile(np.arange(256, dtype=np.uint8), 8 * 4)
    nv = np.repeat(np.arange(1, 9, dtype=np.uint8), 256 * 4)
    G = act.size
    rng = np.random.default_rng(11)
    ack = (rng.integers(0, 128, G, dtype=np.uint8) << 1).astype(np.uint8)
    gr = ((rng.integers(0, 128, G, dtype=np.uint8) << 1) | 1).astype(np.uint8)
    rj = ((rng.integers(0, 128, G, dtype=np.uint8) << 1) & ~gr).astype(np.uint8)
    out = _run_fused(gpu_ctx, hq, ack, gr, rj, act, nv)
    assert not out["fb"].any()
    _check(hq, out, ack, gr, rj, act, nv)


@pytest.mark.gpu
def test_fused_planes_cq_rejects_bad_args(gpu_ctx, hq):
    d = gpu_ctx.empty(4096, np.uint8)
    with pytest.raises(Exception):
        gpu_ctx.readindex_vote_cq_planes_dev(100, d, None, d, d, d)
    gpu_ctx.readindex_vote_cq_planes_dev(0, None, None, None, None, None)   # G = 0: no-op
    gpu_ctx.free(d)
