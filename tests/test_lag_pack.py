"""Host packer of the lag layout (hq_pack_lags / hq_unpack_lags, include/hipquorum.h "commit over
lags"): every index becomes its int32 distance below lastIndex, saturated; unpacking a
representable cout_lag gives back the index. CPU only (the C-ABI host packers)."""
import numpy as np
import pytest

from oracle import qref

SEED = 0x5EED2000
I32_MIN, I32_MAX = -(1 << 31), (1 << 31) - 1


def _clamp_lag(last, x):
    d = last.astype(object) - x.astype(object)
    return np.array([min(max(v, I32_MIN), I32_MAX) for v in d], np.int64).astype(np.int32)


@pytest.fixture(scope="module")
def hq():
    from dragonboat_amd import hipquorum
    return hipquorum


@pytest.mark.parametrize("form", [0, 2])
def test_pack_lags_generator_data(hq, form):
    G, n = 5003, 5
    inp = qref.CommitInputs(qref.spec(SEED, G, n, parity_extras=True))
    lag, cin, aux = hq.pack_lags(G, n, form, 16, inp.match, inp.committed_in, inp.last_index,
                                 inp.term_start, inp.term_mask)
    m = inp.match.reshape(n, G)
    for s in range(n):
        np.testing.assert_array_equal(lag.reshape(n, G)[s], _clamp_lag(inp.last_index, m[s]))
    np.testing.assert_array_equal(cin, _clamp_lag(inp.last_index, inp.committed_in))
    if form == 0:
        np.testing.assert_array_equal(aux, _clamp_lag(inp.last_index, inp.term_start))
    else:
        # bit k of the lag mask = bit (last - k) % 16 of the index mask
        for g in range(0, G, 97):
            last = int(inp.last_index[g])
            want = sum(((int(inp.term_mask[g]) >> ((last - k) % 16)) & 1) << k for k in range(16))
            assert int(aux[g]) == want
    # committed round-trips through its own lag
    out = np.zeros(G, np.uint64)
    hq.unpack_lags(inp.last_index, cin, out)
    np.testing.assert_array_equal(out, inp.committed_in)


@pytest.mark.parametrize("form", [0, 2])
def test_pack_lags_leader_implicit(hq, form):
    """HQ_LAG_LEADER_IMPLICIT: rows of slots 1..n-1 only; a slot 0 other than lastIndex refused."""
    G, n = 3001, 5
    inp = qref.CommitInputs(qref.spec(SEED + 1, G, n, parity_extras=True))
    full = hq.pack_lags(G, n, form, 16, inp.match, inp.committed_in, inp.last_index,
                        inp.term_start, inp.term_mask)
    lead = hq.pack_lags(G, n, form, 16, inp.match, inp.committed_in, inp.last_index,
                        inp.term_start, inp.term_mask, flags=hq.HQ_LAG_LEADER_IMPLICIT)
    assert not full[0].reshape(n, G)[0].any()        # the leader's lag is 0
    np.testing.assert_array_equal(lead[0], full[0].reshape(n, G)[1:].reshape(-1))
    np.testing.assert_array_equal(lead[1], full[1])
    np.testing.assert_array_equal(lead[2], full[2])
    bad = inp.match.copy()
    bad[7] += 1
    with pytest.raises(hq.HQError):
        hq.pack_lags(G, n, form, 16, bad, inp.committed_in, inp.last_index, inp.term_start,
                     inp.term_mask, flags=hq.HQ_LAG_LEADER_IMPLICIT)
    with pytest.raises(hq.HQError):
        hq.pack_lags(G, n, form, 16, inp.match, inp.committed_in, inp.last_index,
                     inp.term_start, inp.term_mask, flags=2)


def test_pack_lags_saturates(hq):
    last = np.array([1 << 40, 1 << 40, 5, 1 << 40, 100], np.uint64)
    match = np.array([0, (1 << 40) + (1 << 33), 9, (1 << 40) - I32_MAX, 100], np.uint64)
    lag, cin, ts = hq.pack_lags(5, 1, 0, 16, match, last, last, last)
    assert list(lag) == [I32_MAX, I32_MIN, -4, I32_MAX, 0]
    assert list(cin) == [0] * 5 and list(ts) == [0] * 5


def test_unpack_lags_keeps_fallback_groups(hq):
    last = np.array([1000, 2000, 3000], np.uint64)
    com = np.array([7, 8, 9], np.uint64)
    fb = np.array([0b010], np.uint64)
    hq.unpack_lags(last, np.array([1, 2, 3], np.int32), com, fb)
    assert list(com) == [999, 8, 2997]
