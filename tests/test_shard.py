"""The N > 1 path on CPU: the clusterID partition rule and a world_size-2 gloo run of the
bench's rank plumbing, with per-rank decisions (oracle as the stand-in compute on this GPU-less
host) stitched back together and compared with a single-process run over the same clusterIDs."""
import os
import socket

import numpy as np
import pytest

from dragonboat_amd import shard


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_rank_shards_partition_cluster_ids(world):
    G = 1000
    seen = set()
    for r in range(world):
        rng = shard.rank_shard(r, world, G)
        cids = list(rng.cids())
        assert len(cids) == G
        assert all(c >= 1 and shard.partition_of(c, world) == r for c in cids)
        seen.update(cids)
    assert len(seen) == G * world
    if world == 1:
        assert list(shard.rank_shard(0, 1, 5).cids()) == [1, 2, 3, 4, 5]


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_rank_buckets_by_voter_count(world):
    for r in range(world):
        for b in range(3):
            rng = shard.rank_bucket(r, world, b, 50)
            for c in rng.cids():
                assert c % world == r and c % 3 == b
                assert shard.MIXED_VOTERS[c % 3] == shard.MIXED_VOTERS[b]
    with pytest.raises(ValueError):
        shard.rank_bucket(0, 3, 0, 1)


def test_step_workers_map_to_one_gpu():
    # 16 step workers over 8 GPUs: clusterID % 16 -> worker, % 8 -> GPU (partition.go:59-61)
    for cid in range(1, 4096):
        assert shard.partition_of(shard.partition_of(cid, 16), 8) == shard.partition_of(cid, 8)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, G, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import bench
    from oracle import qref

    d = bench.Dist()
    assert d.backend == "gloo"
    rng = shard.rank_shard(rank, world, G)
    inp = qref.CommitInputs(qref.spec(0x5EED0001, G, 5, cid_base=rng.cid_base,
                                      cid_stride=rng.cid_stride, parity_extras=True))
    out, chg, fb, rc = inp.run(1, False)
    d.barrier()
    total = d.sum(float(np.unpackbits(chg.view(np.uint8)).sum()))
    slowest = d.max(float(rank + 1))
    gathered = d.gather([float(rank), float(len(out))])   # per-GPU numbers, rank order
    assert gathered == [[float(r), float(G)] for r in range(world)]

    class _Host:   # the gloo path of Dist.gather_words reads the rank's words via download()
        def download(self, a):
            return a
    words, _ = d.gather_words(_Host(), chg, len(chg))
    node = shard.interleave_bitmaps(list(words), G)
    q.put((rank, list(rng.cids()), out.tolist(), total, slowest, node.tolist()))
    d.close()


def test_gloo_world2_sharded_equals_single_process():
    import torch.multiprocessing as mp

    world, G = 2, 4096
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, G, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from oracle import qref

    by_cid = {}
    totals = set()
    nodes = []
    for rank, cids, out, total, slowest, node in res:
        assert slowest == world  # max over ranks
        totals.add(total)
        by_cid.update(zip(cids, out))
        nodes.append(node)
    assert len(totals) == 1      # every rank sees the same all-reduced sum
    # single process over the union of clusterIDs: world + r, 2*world + r, ... == 2 .. 2G+1
    single = qref.CommitInputs(qref.spec(0x5EED0001, G * world, 5, cid_base=world, cid_stride=1,
                                         parity_extras=True))
    s_out, s_chg, _, _ = single.run(1, False)
    cids = range(world, world + G * world)
    assert [by_cid[c] for c in cids] == s_out.tolist()
    assert totals.pop() == float(np.unpackbits(s_chg.view(np.uint8)).sum())
    # the gathered per-GPU changed bits, interleaved by clusterID, are the single-process bitmap
    for node in nodes:
        assert node == s_chg.tolist()


@pytest.mark.parametrize("world,G", [(1, 100), (2, 64), (4, 1000), (8, 77)])
def test_interleave_bitmaps_orders_by_cluster_id(world, G):
    rng = np.random.default_rng(world * G)
    node_bits = rng.integers(0, 2, world * G).astype(np.uint8)   # bit k <-> cid k + base
    ranks = []
    for r in range(world):
        mine = node_bits[r::world] if world > 1 else node_bits
        ranks.append(np.packbits(np.concatenate([mine, np.zeros((-len(mine)) % 64, np.uint8)]),
                                 bitorder="little").view(np.uint64))
    node = shard.interleave_bitmaps(ranks, G)
    got = np.unpackbits(node.view(np.uint8), bitorder="little")[:world * G]
    np.testing.assert_array_equal(got, node_bits)
    if world > 1:   # rank r's group j is cid world + r + j * world
        cids = [list(shard.rank_shard(r, world, G).cids()) for r in range(world)]
        assert cids[1][2] - world == 2 * world + 1
