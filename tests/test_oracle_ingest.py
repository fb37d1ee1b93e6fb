"""The oracle's delta-ingest restatements against direct numpy statements of the reference rules
(remote.tryUpdate raises match only; the confirmed set is a set; appendEntries stamps the
leader's term on every new index)."""
import numpy as np

from oracle import qref


def test_ingest_match_is_running_max():
    rng = np.random.default_rng(1)
    G, n = 1000, 3
    match = rng.integers(0, 100, G * n, dtype=np.uint64)
    g = rng.integers(0, G + 5, 5000, dtype=np.uint64)
    s = rng.integers(0, n + 1, 5000, dtype=np.uint64)
    idx = rng.integers(0, 200, 5000, dtype=np.uint64)
    want = match.copy()
    skipped = 0
    for gi, si, ii in zip(g, s, idx):
        if gi >= G or si >= n:
            skipped += 1
            continue
        k = int(si) * G + int(gi)
        want[k] = max(want[k], ii)
    got = match.copy()
    upd = np.stack([(g << np.uint64(8)) | s, idx], axis=1)
    assert qref.ingest_match(upd, got, G, G, n) == skipped
    np.testing.assert_array_equal(got, want)


def test_ingest_ack_sets_bits_once():
    ack = np.zeros(10, np.uint8)
    gs = np.array([(3 << 8) | 2, (3 << 8) | 2, (3 << 8) | 5, (11 << 8) | 1, (4 << 8) | 9], np.uint64)
    assert qref.ingest_ack(gs, ack, 10, 8) == 2
    assert ack[3] == 0b100100 and ack.sum() == ack[3]


def test_append_sets_term_bits_and_self_match():
    last = np.array([100, 100, 100], np.uint64)
    m0 = last.copy()
    mask = np.zeros(3, np.uint16)
    upd = np.array([[0, 103], [1, 140], [2, 99], [7, 200], [0, 101]], np.uint64)
    assert qref.append(upd, last, m0, mask, 16, 3) == 1
    assert list(last) == [103, 140, 100] and list(m0) == [103, 140, 100]
    assert mask[0] == sum(1 << (i % 16) for i in (101, 102, 103))
    assert mask[1] == 0xFFFF and mask[2] == 0
