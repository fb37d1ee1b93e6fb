"""bench.py's step legs at a small size on the GPU (the step legs checked only
commit counts): every step of every mode (W = 1, 2, 16 workers; device-only and end-to-end)
must equal the CPU event replay (oracle/qref_step.c) in commit and ReadyToRead counts, the sum
of the committed advances and the content digests of (cluster, advance) and of the
ReadyToRead records (cluster, index, ctx)."""
import pytest

import bench

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["step", "step5"])
def test_step_leg_matches_replay(name):
    out = bench.run_step_leg(bench.Dist(), G=1 << 12, steps=3, name=name)
    assert out["producer_equal_rows"]
    assert out["modes_agree"], out.get("modes_mismatch")
    assert out["parity_committed"], out
