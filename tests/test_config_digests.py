"""Golden digests of the BASELINE configs at full size (tests/golden/config_digests.json, made
by tests/golden/make_config_digests.py from the oracle's decisions on the generator's inputs).

CPU: the oracle and the CPU generator still reproduce them (1 M-group configs; the ring and mask
forms of C3 have one digest). GPU: the kernels, fed by the device generator, produce the same
bytes in the headline layouts — leader-row tiles (term-start, mask), the ring gather in
columns, the bit-plane and 4-byte bitmap paths, and C5's fused three-bucket launch."""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import qref

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "config_digests.json")))


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_ring_and_mask_forms_share_one_digest():
    for k in ("committed", "changed", "fallback"):
        assert GOLD["C3_ring"][k] == GOLD["C3_mask"][k]


@pytest.mark.parametrize("name", ["C2", "C3_mask"])
def test_oracle_reproduces_digest(name):
    c = GOLD[name]
    inp = qref.CommitInputs(qref.spec(c["seed"], c["G"], c["n"], cid_base=c["cid_base"],
                                      cid_stride=c["cid_stride"]))
    out, chg, fb, rc = inp.run(c["form"], False, nthreads=os.cpu_count() or 1)
    assert rc == 0
    assert (digest(out), digest(chg), digest(fb)) == (c["committed"], c["changed"], c["fallback"])


def _commit_on_gpu(ctx, hq, cases, layout):
    """Generate every case on the device, decide them (one fused launch when several), return
    each case's (committed, changed, fallback) digests."""
    bufs = []
    for c in cases:
        tiled = layout is not None
        b = hq.alloc_commit(ctx, c["G"], c["n"], c["form"], 16, tiled=tiled,
                            tile_layout=layout if tiled else hq.HQ_LAYOUT_TILES)
        ctx.synth_commit_dev(hq.synth_spec(c["seed"], c["G"], c["n"], cid_base=c["cid_base"],
                                           cid_stride=c["cid_stride"]), b.args())
        if tiled:
            ctx.tile_commit_dev(b.args(), b.tiles, layout)
        bufs.append(b)
    ctx.sync()
    if len(bufs) > 1:
        ctx.commit_fused_dev(hq.commit_batch_array([b.tile_args() for b in bufs]))
    else:
        ctx.commit_dev(bufs[0].tile_args() if layout is not None else bufs[0].args())
    ctx.sync()
    res = []
    for c, b in zip(cases, bufs):
        res.append((digest(ctx.download(b.committed_out)[:c["G"]]), digest(ctx.download(b.changed)),
                    digest(ctx.download(b.fallback))))
        hq.free_commit(ctx, b)
    return res


@pytest.mark.gpu
@pytest.mark.parametrize("name,layout", [("C2", "leader"), ("C3_mask", "leader"),
                                         ("C3_mask", "tiles"), ("C3_ring", None)])
def test_gpu_commit_digest(gpu_ctx, hq, name, layout):
    c = GOLD[name]
    lay = {"leader": hq.HQ_LAYOUT_TILES_LEADER, "tiles": hq.HQ_LAYOUT_TILES, None: None}[layout]
    got = _commit_on_gpu(gpu_ctx, hq, [c], lay)[0]
    assert got == (c["committed"], c["changed"], c["fallback"])


@pytest.mark.gpu
def test_gpu_c5_fused_digest(gpu_ctx, hq):
    cases = [GOLD[f"C5_bucket{b}"] for b in range(3)]
    got = _commit_on_gpu(gpu_ctx, hq, cases, hq.HQ_LAYOUT_TILES_LEADER)
    for c, g in zip(cases, got):
        assert g == (c["committed"], c["changed"], c["fallback"])


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["planes", "columns"])
def test_gpu_c4_digest(gpu_ctx, hq, path):
    c = GOLD["C4"]
    G, n = c["G"], c["n"]
    cols = [gpu_ctx.empty(G, np.uint8) for _ in range(4)]      # ack, granted, rejected, n
    gpu_ctx.synth_bitmaps_dev(hq.synth_spec(c["seed"], G, n), *cols)
    conf = gpu_ctx.empty(hq.words64(G), np.uint64)
    outc = gpu_ctx.empty(hq.words32(G), np.uint64)
    extra = []
    if path == "planes":
        planes = gpu_ctx.empty(hq.plane_tiles(G) * 3 * hq.HQ_PLANE_TILE_GROUPS, np.uint8)
        fb = gpu_ctx.empty(hq.words64(G), np.uint64)
        gpu_ctx.tile_planes_dev(G, *cols, 0, planes, fb)
        gpu_ctx.readindex_vote_planes_dev(G, planes, conf, outc)
        gpu_ctx.sync()
        assert not gpu_ctx.download(fb).any()      # every generated group is in the contract
        extra = [planes, fb]
    else:
        gpu_ctx.readindex_vote_dev(G, cols[0], cols[1], cols[2], cols[3], 0, conf, outc)
        gpu_ctx.sync()
    assert digest(gpu_ctx.download(conf)) == c["confirmed"]
    assert digest(gpu_ctx.download(outc)) == c["outcome"]
    for x in cols + [conf, outc] + extra:
        gpu_ctx.free(x)


@pytest.mark.gpu
@pytest.mark.parametrize("rank", range(8))
def test_gpu_c5_node_shard_digest(gpu_ctx, hq, rank):
    """BASELINE config 5 — 64 Mi groups with 3 / 5 / 7 voters (clusterID % 3), sharded
    clusterID % 8 over 8 GPUs (partition.go:38) — one GPU's share per case: its three buckets
    generated on the device, decided in one fused launch over leader-row tiles, equal to the
    oracle's digests of that shard (tests/golden/make_config_digests.py --c5-node). Together the
    eight cases check 24 x ((8 Mi) // 3) = 67,108,848 groups on one GPU: the configuration's
    64 Mi groups less the 16 that 8 Mi per rank leaves over after three equal buckets (the
    bench's per-rank shape, bench.py commit_buckets)."""
    cases = [GOLD[f"C5x8_rank{rank}_bucket{b}"] for b in range(3)]
    got = _commit_on_gpu(gpu_ctx, hq, cases, hq.HQ_LAYOUT_TILES_LEADER)
    for c, g in zip(cases, got):
        assert g == (c["committed"], c["changed"], c["fallback"])


def test_c5_node_digests_cover_the_config():
    """The 24 shard-bucket cases are the 64 Mi-group config: 8 ranks x 3 buckets, disjoint
    clusterID progressions covering cid % 24 == every residue."""
    from dragonboat_amd import shard

    keys = [f"C5x8_rank{r}_bucket{b}" for r in range(8) for b in range(3)]
    assert all(k in GOLD for k in keys)
    assert sum(GOLD[k]["G"] for k in keys) == 24 * ((8 << 20) // 3)
    assert len({GOLD[k]["cid_base"] % 24 for k in keys}) == 24
    for r in range(8):
        for b in range(3):
            c = GOLD[f"C5x8_rank{r}_bucket{b}"]
            assert c["cid_base"] % 8 == r and c["cid_base"] % 3 == b and c["cid_stride"] == 24
            assert c["n"] == shard.MIXED_VOTERS[b]


def test_oracle_reproduces_rim_and_c4pq_digests():
    """The multi-ctx ReadIndex batch the rim / rimt legs time (2 Mi x 4 ctxs x 7 voters) and the
    fused ReadIndex + vote + CheckQuorum batch c4pq times (16 Mi x 7): the oracle still makes the
    committed digests from bench.py's own input helpers."""
    import bench

    nt = os.cpu_count() or 1
    c = GOLD["RIM"]
    G, K, n, ordn, idx = bench.rim_inputs(c["rank"])
    assert (G, K, n) == (c["G"], c["K"], c["n"])
    rel, cnt, fb, bend = qref.readindex_multi_batch(ordn.reshape(-1), idx.reshape(-1), None, None,
                                                    n, K, n, nthreads=nt)
    assert not fb.any()
    assert (digest(rel), digest(cnt), digest(bend)) == (
        c["released_index"], c["released_count"], c["batch_end"])
    c = GOLD["C4PQ"]
    want = bench.c4pq_oracle(c["seed_votes"], c["seed_active"], c["G"], c["n"], nt)
    for k in ("confirmed", "outcome", "has_quorum"):
        assert digest(want[k]) == c[k], k


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["tiles", "columns", "tiles_compact"])
def test_gpu_rim_digest(gpu_ctx, hq, path):
    """rim / rimt / rimtc at the bench's full size: the multi-ctx release (the uniform tile
    kernel over 128-group tiles, k_ri_multi2 over columns, and the tiles with released_index
    NULL, rebuilt by hq_ri_released_host) equals the oracle's replay digests."""
    import bench

    c = GOLD["RIM"]
    G, K, n, ordn, idx = bench.rim_inputs(c["rank"])
    o, x = gpu_ctx.upload(ordn.reshape(-1)), gpu_ctx.upload(idx.reshape(-1))
    rel, cnt, bend = (gpu_ctx.empty(K * G, np.uint64), gpu_ctx.empty(G, np.uint8),
                      gpu_ctx.empty(G, np.uint8))
    extra = []
    if path.startswith("tiles"):
        t = gpu_ctx.empty((G // 128) * hq.ri_tile_bytes(K, n, 0), np.uint8)
        gpu_ctx.tile_ri_multi_dev(G, K, n, o, x, None, None, t)
        gpu_ctx.readindex_multi_tiles_dev(G, K, n, t, 0, n,
                                          None if path == "tiles_compact" else rel, cnt,
                                          batch_end=bend)
        extra = [t]
    else:
        gpu_ctx.readindex_multi_dev(G, K, n, o, x, None, None, n, rel, cnt, batch_end=bend)
    gpu_ctx.sync()
    got_cnt, got_bend = gpu_ctx.download(cnt), gpu_ctx.download(bend)
    got_rel = (hq.ri_released_host(K, idx, got_cnt, got_bend) if path == "tiles_compact"
               else gpu_ctx.download(rel))
    assert (digest(got_rel), digest(got_cnt), digest(got_bend)) == (
        c["released_index"], c["released_count"], c["batch_end"])
    for a in [o, x, rel, cnt, bend] + extra:
        gpu_ctx.free(a)


@pytest.mark.gpu
def test_gpu_c4pq_digest(gpu_ctx, hq):
    """c4pq at the bench's full size (16 Mi x 7): ReadIndex + vote + CheckQuorum in one pass over
    the bit planes equals the oracle's three batches; the active planes are zeroed."""
    c = GOLD["C4PQ"]
    G, n = c["G"], c["n"]
    T = hq.HQ_PLANE_TILE_GROUPS
    arrs = [gpu_ctx.empty(G, np.uint8) for _ in range(4)]
    gpu_ctx.synth_bitmaps_dev(hq.synth_spec(c["seed_votes"], G, n), *arrs)
    pl, apl = gpu_ctx.empty(hq.plane_tiles(G) * 3 * T, np.uint8), gpu_ctx.empty(
        hq.cq_plane_bytes(G, 8), np.uint8)
    gpu_ctx.tile_planes_dev(G, *arrs, 0, pl)
    gpu_ctx.synth_bitmaps_dev(hq.synth_spec(c["seed_active"], G, n), arrs[0])
    gpu_ctx.tile_cq_planes_dev(G, arrs[0], None, 8, 0, apl)
    conf, outc, hqb = (gpu_ctx.empty(hq.words64(G), np.uint64), gpu_ctx.empty(hq.words32(G), np.uint64),
                       gpu_ctx.empty(hq.words64(G), np.uint64))
    gpu_ctx.readindex_vote_cq_planes_dev(G, pl, apl, conf, outc, hqb)
    gpu_ctx.sync()
    assert digest(gpu_ctx.download(conf)) == c["confirmed"]
    assert digest(gpu_ctx.download(outc)) == c["outcome"]
    assert digest(gpu_ctx.download(hqb)) == c["has_quorum"]
    assert not gpu_ctx.download(apl).any()
    for a in arrs + [pl, apl, conf, outc, hqb]:
        gpu_ctx.free(a)
