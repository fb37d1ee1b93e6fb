"""Host side of the ReadyToRead slot form (HQ_WORKER_READY_SLOTS) and of the step's wait clocks,
on CPU: the slots gathered from hq_step_output (Worker._results), the merge of slots and list
into the reference's order (merge_ready, as the Go EachReady walks them), and the wake-up
lateness bench.py reads from the wait's clocks."""
import numpy as np
import pytest

import bench
from dragonboat_amd import hipquorum as hq


def _records(rng, pos, committed):
    r = np.zeros(len(pos), hq.READY_COMPACT_DTYPE)
    r["pos"] = pos
    r["delta"] = rng.integers(-3, 40, len(pos))
    r["ctx_low"] = rng.integers(1, 1 << 62, len(pos), dtype=np.uint64)
    r["ctx_high"] = rng.integers(0, 4, len(pos), dtype=np.uint64)
    return r


def _split(rng, n=3000, frac_list=0.1):
    """Groups 0..n-1 of which a quarter have one read: some in the list, the rest in slots."""
    cids = np.uint64(7) + np.arange(n, dtype=np.uint64) * np.uint64(3)
    committed = rng.integers(100, 1 << 40, n, dtype=np.uint64)
    readers = np.sort(rng.choice(n, n // 4, replace=False))
    in_list = rng.random(len(readers)) < frac_list
    return cids, committed, readers, in_list


def test_merge_is_group_order():
    rng = np.random.default_rng(1)
    cids, committed, readers, in_list = _split(rng)
    allr = _records(rng, readers, committed)
    want = hq.expand_ready(allr, cids, committed)          # group order: the reference's
    res = {"ready_compact": allr[in_list], "ready_slots": allr[~in_list]}
    np.testing.assert_array_equal(hq.merge_ready(res, cids, committed), want)
    # the list as 32-byte records (a step whose deltas do not all fit 32 bits)
    res32 = {"ready": want[in_list], "ready_slots": allr[~in_list]}
    np.testing.assert_array_equal(hq.merge_ready(res32, cids, committed), want)
    # either part alone, and nothing
    np.testing.assert_array_equal(hq.merge_ready({"ready_slots": allr}, cids, committed), want)
    np.testing.assert_array_equal(hq.merge_ready({"ready_compact": allr}, cids, committed), want)
    assert len(hq.merge_ready({"ready": np.zeros(0, hq.READY_DTYPE)}, cids, committed)) == 0


def test_merge_keeps_a_misordered_list_misordered():
    """The merge does not sort: two list records swapped stay swapped (so bench's position-
    weighted digest still sees a misordered list)."""
    rng = np.random.default_rng(2)
    cids, committed, readers, in_list = _split(rng, frac_list=0.3)
    allr = _records(rng, readers, committed)
    lst = allr[in_list].copy()
    lst[[3, 4]] = lst[[4, 3]]
    got = hq.merge_ready({"ready_compact": lst, "ready_slots": allr[~in_list]}, cids, committed)
    ok = hq.expand_ready(allr, cids, committed)
    assert len(got) == len(ok) and not np.array_equal(got, ok)
    assert bench.ready_digest(got) == bench.ready_digest(ok)
    assert bench.ready_order_digest(got) != bench.ready_order_digest(ok)


def test_results_gather_slots():
    """Worker._results reads tile t's count and its records at ready_slots[256 t ..] in tile
    order (the rest of each tile's slot is never read)."""
    rng = np.random.default_rng(3)
    tiles = 5
    counts = np.array([3, 0, 256, 1, 17], np.uint32)
    slots = np.zeros(tiles * hq.SLOT_TILE, hq.READY_COMPACT_DTYPE)
    slots["pos"] = 0xDEADBEEF                                 # (garbage past each count)
    want = []
    for t, c in enumerate(counts):
        pos = np.sort(rng.choice(hq.SLOT_TILE, int(c), replace=False)) + t * hq.SLOT_TILE
        r = _records(rng, pos, None)
        slots[t * hq.SLOT_TILE:t * hq.SLOT_TILE + c] = r
        want.append(r)
    out = hq.StepOutput()
    out.ready_slots = slots.ctypes.data
    out.ready_slot_counts = counts.ctypes.data
    out.n_ready_tiles = tiles
    out.n_ready_slotted = int(counts.sum())
    res = hq.Worker._results(out, True, tiles * hq.SLOT_TILE)
    np.testing.assert_array_equal(res["ready_slots"], np.concatenate(want))


def test_wake_lag_from_clocks():
    """The wake-up lateness of each step: host return - 10 ns x device tick, against the run's
    smallest difference; steps without a device stamp get None."""
    off = 5_000_000_000
    ph = []
    for k, late in enumerate([30_000, 10_000, 2_000_000, 10_000]):
        ticks = 1_000_000 + 100_000 * k
        ph.append({"dev__end_ns": off + 10 * ticks + late, "dev__end_ticks": ticks})
    ph.append({"dev__end_ns": 123, "dev__end_ticks": 0})
    bench._wake_lag(ph, "dev_")
    lags = [p["dev_wake_lag_ms"] for p in ph]
    assert lags[:4] == pytest.approx([0.02, 0.0, 1.99, 0.0]) and lags[4] is None
    assert all("dev__end_ns" not in p for p in ph)


def test_link_block_bytes():
    """The step legs' link roofline: output bytes counted from the results (slots by records and
    count words), rates over the GPU time, frac against the probe's both-ways total."""
    rs = [{"committed_advance": np.zeros(600, np.uint32),
           "ready_compact": np.zeros(5, hq.READY_COMPACT_DTYPE),
           "ready_slots": np.zeros(40, hq.READY_COMPACT_DTYPE), "gpu_ns": 7}]
    assert bench._out_bytes(rs) == 600 * 4 + 5 * 24 + 40 * 24 + 4 * 3

    class D:
        rank, device = 1, 0
    bench._LINK["v"] = {"read_GBps": 50.0, "write_GBps": 40.0, "both_GBps": 80.0}
    try:
        b = bench._link_block(D(), 40e6, 10e6, 1.0)
    finally:
        bench._LINK.clear()
    assert b["both_GBps"] == 50.0 and b["frac"] == 0.625
    assert b["frac_serial"] == pytest.approx((40e6 / 50e9 + 10e6 / 40e9) / 1e-3, abs=1e-3)
