"""Golden output digests of the BASELINE configs at full size (SURVEY.md §8c "golden vectors for
large configs"): the inputs are the deterministic generator's (oracle/qgen.c, its device twin in
hq_kernels.hip) at the seeds below, the outputs the oracle's (oracle/qref.c) decisions, and only
their SHA-256 digests (plus counts) are committed, in config_digests.json. The CPU tests check the
oracle still reproduces them; the GPU tests check the kernels produce the same bytes from the
device generator's inputs, in the headline layouts.

usage: python tests/golden/make_config_digests.py   (from the repo root; ~1 minute on 8 cores)
       python tests/golden/make_config_digests.py --c5-node   (adds only the 8-GPU C5 shards)
       python tests/golden/make_config_digests.py --planes    (adds only RIM and C4PQ)
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import qref  # noqa: E402

SEED = 0x5EED0000        # + BASELINE config index, as bench.py
THREADS = os.cpu_count() or 1


def digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def bits(w: np.ndarray, G: int) -> int:
    return int(np.unpackbits(w.view(np.uint8), bitorder="little")[:G].sum())


def commit_case(name, seed, G, n, form, cid_base=1, cid_stride=1):
    inp = qref.CommitInputs(qref.spec(seed, G, n, cid_base=cid_base, cid_stride=cid_stride))
    out, chg, fb, rc = inp.run(form, False, nthreads=THREADS)
    assert rc == 0
    return {"kind": "commit", "seed": seed, "G": G, "n": n, "form": form, "cid_base": cid_base,
            "cid_stride": cid_stride, "committed": digest(out), "changed": digest(chg),
            "fallback": digest(fb), "n_changed": bits(chg, G), "n_fallback": bits(fb, G)}


def bitmap_case(name, seed, G, n):
    inp = qref.BitmapInputs(qref.spec(seed, G, n))
    conf = qref.readindex_batch(inp.ack, inp.n_voting, 0, nthreads=THREADS)[0]
    outc = qref.vote_batch(inp.granted, inp.rejected, inp.n_voting, 0, nthreads=THREADS)[0]
    return {"kind": "bitmaps", "seed": seed, "G": G, "n": n, "confirmed": digest(conf),
            "outcome": digest(outc), "n_confirmed": bits(conf, G)}


def rim_case():
    """The multi-ctx ReadIndex legs' batch (bench.py rim / rimt, rank 0: 2 Mi groups x 4 pending
    ctxs x 7 voters) decided by the oracle's message replay."""
    import bench

    G, K, n, ordn, idx = bench.rim_inputs(0)
    rel, cnt, fb, bend = qref.readindex_multi_batch(ordn.reshape(-1), idx.reshape(-1), None, None,
                                                    n, K, n, nthreads=THREADS)
    assert not fb.any()
    return {"kind": "readindex_multi", "G": G, "K": K, "n": n, "rank": 0,
            "released_index": digest(rel), "released_count": digest(cnt),
            "batch_end": digest(bend), "n_released": int(cnt.astype(np.int64).sum())}


def c4pq_case():
    """BASELINE config 4 with CheckQuorum (bench.py c4pq, set 0: 16 Mi groups x 7 voters, the
    active flags the ack bitmaps of seed + 2) decided by the oracle's batches."""
    import bench

    G, n = 16 << 20, 7
    want = bench.c4pq_oracle(SEED + 3, SEED + 5, G, n, THREADS)
    return {"kind": "readindex_vote_checkquorum", "G": G, "n": n, "seed_votes": SEED + 3,
            "seed_active": SEED + 5, **{k: digest(v) for k, v in want.items()},
            "n_has_quorum": bits(want["has_quorum"], G)}


def main():
    from dragonboat_amd import shard

    cases = {
        "C2": commit_case("C2", SEED + 1, 1 << 20, 3, 0),                 # term-start
        "C3_ring": commit_case("C3_ring", SEED + 2, 1 << 20, 5, 1),       # u64 term-ring gather
        "C3_mask": commit_case("C3_mask", SEED + 2, 1 << 20, 5, 2),       # 16-bit term mask
        "C4": bitmap_case("C4", SEED + 3, 16 << 20, 7),
    }
    per = (8 << 20) // 3              # C5: rank 0 of 8 GPUs, buckets n = 3 / 5 / 7
    for b in range(3):
        rng = shard.rank_bucket(0, 1, b, per)
        cases[f"C5_bucket{b}"] = commit_case(f"C5_bucket{b}", SEED + 4, rng.count,
                                             shard.MIXED_VOTERS[b], 2, rng.cid_base,
                                             rng.cid_stride)
    cases.update(c5_node_cases())
    cases["RIM"] = rim_case()
    cases["C4PQ"] = c4pq_case()
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "config_digests.json")
    json.dump(cases, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(cases, indent=1))


def c5_node_cases():
    """BASELINE config 5 whole: 64 Mi groups, n = 3 / 5 / 7 by clusterID % 3, sharded
    clusterID % 8 over 8 GPUs (partition.go:38): 8 ranks x 3 buckets of (8 Mi / 3) groups, each
    rank's buckets as bench.py builds them (shard.rank_bucket)."""
    from dragonboat_amd import shard

    per = (8 << 20) // 3
    out = {}
    for r in range(8):
        for b in range(3):
            rng = shard.rank_bucket(r, 8, b, per)
            out[f"C5x8_rank{r}_bucket{b}"] = commit_case(
                f"C5x8_rank{r}_bucket{b}", SEED + 4, rng.count, shard.MIXED_VOTERS[b], 2,
                rng.cid_base, rng.cid_stride)
    return out


if __name__ == "__main__":
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "config_digests.json")
    if "--c5-node" in sys.argv:
        cases = json.load(open(path))
        cases.update(c5_node_cases())
        json.dump(cases, open(path, "w"), indent=1, sort_keys=True)
    elif "--planes" in sys.argv:       # adds only the multi-ctx ReadIndex and fused-planes cases
        cases = json.load(open(path))
        cases["RIM"] = rim_case()
        cases["C4PQ"] = c4pq_case()
        json.dump(cases, open(path, "w"), indent=1, sort_keys=True)
    else:
        main()
