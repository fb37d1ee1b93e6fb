"""Commit decisions at the edges of the u64 range, bit-exact with the oracle: indexes and terms
next to 0 and 2^64 - 1, matches above lastIndex (the term() = 0 branch), committed above
lastIndex, terms at 0 and around 2^32 (the u32 ring's saturation), random masks and rings, voter
counts 0..n_max + 1 — in every term form, columns, tiles and leader-row tiles, uniform and
per-group n."""
import numpy as np
import pytest

from oracle import qref
from test_gpu_parity import upload_commit
from test_gpu_tiles import run_tiled

pytestmark = pytest.mark.gpu

SEED = 0x5EED0000
U64 = np.uint64
TOP = (1 << 64) - 1


def below(last, d):
    """last - d for signed d, clamped to [0, 2^64 - 1] (exact, through Python integers)."""
    v = [min(max(int(x) - int(y), 0), TOP) for x, y in zip(last, d)]
    return np.array(v, dtype=np.uint64)


def adversarial(G, n, seed):
    """Oracle-generated inputs with every column overwritten by edge values."""
    inp = qref.CommitInputs(qref.spec(SEED + seed, G, n, parity_extras=True))
    rng = np.random.default_rng(seed)
    R = inp.R
    # lastIndex: near 0, near 2^64 - 1, or mid-range
    kind = rng.integers(0, 3, G)
    base = np.where(kind == 0, rng.integers(0, 40, G).astype(np.uint64),
                    np.where(kind == 1, U64(TOP) - rng.integers(0, 40, G).astype(np.uint64),
                             rng.integers(1 << 40, 1 << 62, G, dtype=np.uint64)))
    last = base
    # committed: usually within R below last, sometimes above it or far below it
    committed = below(last, rng.integers(0, R + 3, G))
    over = rng.random(G) < 0.05
    committed = np.where(over & (last < U64(TOP)), last + U64(1), committed)
    far = rng.random(G) < 0.05
    committed = np.where(far, last // U64(2), committed)
    # matches: around committed / last, some above last, some at the extremes
    m = inp.match.reshape(n, G)
    for s in range(n):
        v = below(last, rng.integers(-3, R + 3, G))
        pick = rng.random(G)
        v = np.where(pick < 0.03, U64(TOP), np.where(pick < 0.06, U64(0), v))
        m[s] = v
    inp.last_index[:] = last
    inp.committed_in[:] = committed
    # term-start anywhere around the window
    inp.term_start[:] = below(last, rng.integers(-2, R + 3, G))
    # leader term: 0 (ring fallback), around 2^32 (u32 ring saturation), top, random
    tk = rng.integers(0, 8, G)
    term = np.select([tk == 0, tk == 1, tk == 2, tk == 3, tk == 4],
                     [U64(0), U64(0xFFFFFFFE), U64(0xFFFFFFFF), U64(TOP),
                      rng.integers(1 << 40, 1 << 63, G, dtype=np.uint64)],
                     rng.integers(1, 1 << 31, G, dtype=np.uint64))
    inp.term[:] = term
    # ring: entries equal to the term or not, at random
    ring = inp.ring.reshape(G, R)
    eq = rng.random((G, R)) < 0.6
    other = np.where(rng.random((G, R)) < 0.5, rng.integers(0, 1 << 63, (G, R), dtype=np.uint64),
                     term[:, None] + U64(1 << 32))   # equal to the term in its low 32 bits
    ring[:] = np.where(eq, term[:, None], other)
    if inp.term_mask is not None:
        inp.term_mask[:] = rng.integers(0, 1 << 16, G).astype(np.uint16)
    inp.n_voting[:] = rng.integers(0, n + 2, G).astype(np.uint8)
    return inp


@pytest.mark.parametrize("form", [0, 1, 2, 3])
@pytest.mark.parametrize("n", [1, 3, 5, 8])
@pytest.mark.parametrize("pern", [False, True])
def test_commit_extremes_columns(gpu_ctx, hq, form, n, pern):
    G = 5003
    inp = adversarial(G, n, 17 * n + form + 100 * pern)
    d = upload_commit(gpu_ctx, hq, inp, form, pern)
    gpu_ctx.commit_dev(d["args"])
    gpu_ctx.sync()
    want_out, want_chg, want_fb, rc = inp.run(form, pern)
    np.testing.assert_array_equal(gpu_ctx.download(d["out"])[:G], want_out)
    np.testing.assert_array_equal(gpu_ctx.download(d["chg"]), want_chg)
    np.testing.assert_array_equal(gpu_ctx.download(d["fb"]), want_fb)
    for b in d["bufs"]:
        gpu_ctx.free(b)


@pytest.mark.parametrize("form", [0, 1, 2, 3])
@pytest.mark.parametrize("n", [2, 3, 5, 7])
@pytest.mark.parametrize("pern", [False, True])
def test_commit_extremes_tiles(gpu_ctx, hq, form, n, pern):
    G = 4099
    inp = adversarial(G, n, 31 * n + form + 100 * pern)
    out, chg, fb = run_tiled(gpu_ctx, hq, inp, form, pern)
    want_out, want_chg, want_fb, rc = inp.run(form, pern)
    np.testing.assert_array_equal(out, want_out)
    np.testing.assert_array_equal(chg, want_chg)
    np.testing.assert_array_equal(fb, want_fb)


@pytest.mark.parametrize("form", [0, 1, 2, 3])
@pytest.mark.parametrize("n", [1, 3, 5, 8])
@pytest.mark.parametrize("pern", [False, True])
def test_commit_extremes_leader_tiles(gpu_ctx, hq, form, n, pern):
    """HQ_LAYOUT_TILES_LEADER at the edges: slot 0 = lastIndex (the layout's precondition, the
    leader's own match, raft.go:918), everything else adversarial."""
    G = 4099
    inp = adversarial(G, n, 43 * n + form + 100 * pern)
    inp.match[:G] = inp.last_index
    out, chg, fb = run_tiled(gpu_ctx, hq, inp, form, pern, hq.HQ_LAYOUT_TILES_LEADER)
    want_out, want_chg, want_fb, rc = inp.run(form, pern)
    np.testing.assert_array_equal(out, want_out)
    np.testing.assert_array_equal(chg, want_chg)
    np.testing.assert_array_equal(fb, want_fb)
